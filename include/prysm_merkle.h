/*
 * prysm_merkle.h — C ABI of the MI355X Merkleization engine (libprysm_merkle.so).
 *
 * Drop-in boundary for the Keccak-era Prysm SSZ tree-hash path.  The reference
 * is pure Go with no FFI; these entry points are what a new
 * cgo package `gpu/merkle` binds (INTEGRATION.md shows the binding), called
 * from the unchanged exported Go signatures:
 *
 *   hashutil.Hash(data []byte) [32]byte      shared/hashutil/hash.go:11
 *   ssz.merkleHash(list [][]byte)            shared/ssz/hash.go:194
 *   ssz.TreeHash(val interface{})            shared/ssz/hash.go:23 (via
 *                                            makeSliceHasher hash.go:118-139)
 *   (*trieutil.DepositTrie).UpdateDepositTrie / GenerateMerkleBranch / Root
 *                                            shared/trieutil/deposit_trie.go:29-63
 *   trieutil.VerifyMerkleBranch              shared/trieutil/deposit_trie.go:68-81
 *   hashutil.MerkleRoot                      shared/hashutil/merkleRoot.go:12
 *
 * Conventions
 *   - Every compute entry point takes a per-call context `mk_call*` first
 *     (NULL = defaults).  cgo may run two consecutive C calls of one goroutine
 *     on different OS threads, so the device and the error detail travel with
 *     the call, never with the thread:
 *       call->device  in:  device index; -1 = for dev entry points the device
 *                          of `stream` (the thread's current HIP device when
 *                          stream is NULL), for host-buffer entry points the
 *                          thread's current HIP device (0 unless set).
 *       call->code    out: the status returned.
 *       call->err     out: NUL-terminated detail of a failure ("" on success).
 *     The calling thread's current HIP device is the same after the call as
 *     before it.  mk_last_error() keeps the thread's last detail for C callers.
 *   - Every function returns 0 (MK_OK) or a negative MK_E* code; mk_strerror()
 *     names it.  Nothing panics across the boundary; there is NO CPU
 *     fallback: without a usable gfx950 device every compute entry point
 *     returns MK_ENODEV.
 *   - Host-buffer entry points (no `dev` in the name) borrow caller memory for
 *     the duration of the call only (cgo rule: Go memory is never retained);
 *     `[][]byte` inputs are passed flattened as (data, offs[n+1]).
 *   - `dev` entry points take device pointers (HBM-resident inputs) and a
 *     hipStream_t passed as void* (NULL = the device's default stream); they
 *     enqueue work and return without synchronising.  Their scratch space is
 *     caller-provided (size from the *_workspace_bytes query), so they never
 *     allocate and can be captured into a hipGraph -- except
 *     mk_dev_ssz_merkle_many (host-planned descriptors, uploaded per call)
 *     and mk_dev_ssz_merkle_hash_multi (RCCL, library workspaces), which
 *     refuse / are not meant for capture.
 *   - Thread safety: every entry point may be called concurrently from any OS
 *     thread; host-buffer entry points take a per-device lock, deposit-trie
 *     handles a per-handle lock.
 *   - Digests are 32 bytes; node arrays are n x 32 contiguous bytes.
 */
#ifndef PRYSM_MERKLE_H
#define PRYSM_MERKLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MK_OK 0
#define MK_EINVAL (-22)  /* bad argument (also: reference panics, e.g. len(list[0]) == 0) */
#define MK_ENODEV (-19)  /* no usable gfx950 device / device index out of range */
#define MK_ENOMEM (-12)  /* device or host allocation failed / workspace too small */
#define MK_EHIP (-5)     /* a HIP runtime call failed (see call->err) */
#define MK_ECOMM (-71)   /* RCCL failure in the multi-device path */

#define MK_ERR_LEN 256
typedef struct mk_call {
    int32_t device;         /* in: device index, -1 = default (see Conventions) */
    int32_t code;           /* out: status of the call */
    char err[MK_ERR_LEN];   /* out: detail of a failure, "" on success */
} mk_call;

/* ---- lifecycle --------------------------------------------------------- */
int mk_init(int device);          /* idempotent: creates `device`'s streams; 0 ok */
int mk_device_count(void);        /* number of visible gfx950 devices (0 if none) */
const char* mk_strerror(int code);
const char* mk_last_error(void);  /* the calling thread's last failure detail */
const char* mk_version(void);

/* ---- hashutil.Hash (hash.go:11-25): legacy Keccak-256 ------------------- */
/* Single message.  Provided for completeness; Go keeps single Hash calls on
 * the CPU (launch latency, and Hash cannot return an error). */
int mk_hash(mk_call* call, const uint8_t* data, uint64_t len, uint8_t out[32]);
/* Batched form ("HashBatch"): n messages of msg_len bytes, contiguous -> n*32. */
int mk_hash_batch(mk_call* call, const uint8_t* in, uint64_t n, uint32_t msg_len, uint8_t* out);
/* Variable-length batch: message i = in[offs[i], offs[i+1]) -> n*32. */
int mk_hash_batch_var(mk_call* call, const uint8_t* in, const uint64_t* offs, uint64_t n, uint8_t* out);
int mk_dev_hash_batch(mk_call* call, const void* d_in, uint64_t n, uint32_t msg_len, void* d_out, void* stream);
int mk_dev_hash_batch_var(mk_call* call, const void* d_in, const uint64_t* d_offs, uint64_t n, void* d_out,
                          void* stream);

/* ---- ssz.merkleHash (hash.go:194-239) ---------------------------------- */
/* n items of item_len bytes each, contiguous (the flattened [][]byte; every
 * list TreeHash builds has uniform element length).  out = 32-B result.
 * item_len == 0 with n > 0 is the reference's divide-by-zero panic: MK_EINVAL. */
int mk_ssz_merkle_hash(mk_call* call, const uint8_t* items, uint64_t n, uint32_t item_len, uint8_t out[32]);
uint64_t mk_ssz_merkle_workspace_bytes(uint64_t n, uint32_t item_len);
int mk_dev_ssz_merkle_hash(mk_call* call, const void* d_items, uint64_t n, uint32_t item_len, void* d_out32,
                           void* d_ws, uint64_t ws_bytes, void* stream);

/* Many lists in one call (makeSliceHasher over a list of lists, a struct's
 * list fields, a state's lists): list i = n[i] items of item_len[i] bytes at
 * byte offset offs[i] of d_items (16-B aligned offsets take the streaming
 * path); d_roots[i] (32 B each) = merkleHash(list i).  offs, n and item_len
 * are HOST arrays (the library plans on the host and uploads the per-list
 * descriptors into the workspace).  Lists of up to 2^15 chunks share one leaf
 * launch and one launch per level; longer lists run their own fused passes.
 * Workspace from mk_ssz_merkle_many_workspace_bytes (same n, item_len).
 * The descriptors go through a small pinned host ring on every call, so the
 * call cannot be captured into a hipGraph: on a capturing stream it returns
 * MK_EINVAL. */
uint64_t mk_ssz_merkle_many_workspace_bytes(const uint64_t* n, const uint32_t* item_len, uint32_t nlists);
int mk_dev_ssz_merkle_many(mk_call* call, const void* d_items, const uint64_t* offs, const uint64_t* n,
                           const uint32_t* item_len, uint32_t nlists, void* d_roots, void* d_ws, uint64_t ws_bytes,
                           void* stream);
/* Host-buffer form: list i = items[offs[i], offs[i] + n[i]*item_len[i]). */
int mk_ssz_merkle_many(mk_call* call, const uint8_t* items, const uint64_t* offs, const uint64_t* n,
                       const uint32_t* item_len, uint32_t nlists, uint8_t* roots);

/* ---- ssz.TreeHash of a list of byte strings (hash.go:100-107, 118-139) -- */
/* TreeHash([][N]byte) / TreeHash([][]byte) with n elements of elem_len bytes
 * each, contiguous: makeSliceHasher hashes every element with hashedEncoding
 * (Keccak(le32(elem_len) || element)) and runs merkleHash over those 32-B
 * digests.  One call, no host round trip: with 32-B elements (16-B aligned)
 * the digests are computed inside the tree's leaf pass and never reach HBM.
 * Workspace from mk_ssz_tree_hash_bytes_list_workspace_bytes (for a 16-B
 * aligned d_elems; other alignments need the two-phase size, n*32 + the
 * plan's, and report MK_ENOMEM when the workspace is short). */
uint64_t mk_ssz_tree_hash_bytes_list_workspace_bytes(uint64_t n, uint32_t elem_len);
int mk_dev_ssz_tree_hash_bytes_list(mk_call* call, const void* d_elems, uint64_t n, uint32_t elem_len,
                                    void* d_out32, void* d_ws, uint64_t ws_bytes, void* stream);
int mk_ssz_tree_hash_bytes_list(mk_call* call, const uint8_t* elems, uint64_t n, uint32_t elem_len,
                                uint8_t out[32]);

/* ---- subtree sharding across GPUs ----------------------- */
/* Split a merkleHash of n items over `nshards` devices: every shard is a
 * power-of-two-aligned run of 2^height chunks.  item_begin[nshards+1] gets
 * each shard's item range (empty shards have begin == end); *nonempty the
 * number of non-empty shards.  When the tree is too small to shard
 * (*nonempty == 1) shard 0 holds everything and is hashed with
 * mk_dev_ssz_merkle_hash instead. */
int mk_ssz_merkle_shard_plan(mk_call* call, uint64_t n, uint32_t item_len, uint32_t nshards, uint32_t* height,
                             uint32_t* nonempty, uint64_t* item_begin);
/* Root (32 B, height `height` above the chunks) of one shard.  pad_at_one=1
 * for every shard of a tree with >1 non-empty shard: a ragged last shard keeps
 * applying the reference's odd rule (node || 0^128) up to `height`. */
int mk_dev_ssz_merkle_subtree(mk_call* call, const void* d_shard_items, uint64_t shard_n, uint32_t item_len,
                              uint32_t height, int pad_at_one, void* d_out32, void* d_ws, uint64_t ws_bytes,
                              void* stream);
/* Frontier variant: stop `frontier_log2` levels below the shard root and
 * write the shard's nodes at height (height - frontier_log2) to d_out (32 B
 * each, 2^frontier_log2 of them, fewer for a ragged last shard; *nodes_out
 * gets the count).  The shards' frontiers, concatenated in shard order, are
 * that level of the whole tree, so ranks gather a few KB each and the top
 * levels move to the finisher (mk_dev_ssz_merkle_finish_nodes), which can
 * overlap the ranks' next Merkleization.  0 < frontier_log2 < height. */
int mk_dev_ssz_merkle_subtree_frontier(mk_call* call, const void* d_shard_items, uint64_t shard_n,
                                       uint32_t item_len, uint32_t height, uint32_t frontier_log2, int pad_at_one,
                                       void* d_out, uint64_t* nodes_out, void* d_ws, uint64_t ws_bytes,
                                       void* stream);
/* The same subtree continued from one of its node levels: `count` 32-B nodes
 * (a shard's level, e.g. the output of the leaf pass) reduced for `height`
 * levels with the reference's odd rule (hash.go:225-235; pad_at_one as
 * above), stopping `frontier_log2` levels below the top (0 = to the top
 * node).  Lets a rank split its shard into the leaf pass and the narrower
 * node passes and run the latter on another stream (prysm_amd/parallel.py
 * ShardedMerklePipeline).  Workspace from
 * mk_ssz_merkle_node_frontier_workspace_bytes. */
uint64_t mk_ssz_merkle_node_frontier_workspace_bytes(uint64_t count, uint32_t height, uint32_t frontier_log2);
int mk_dev_ssz_merkle_node_frontier(mk_call* call, const void* d_nodes, uint64_t count, uint32_t height,
                                    uint32_t frontier_log2, int pad_at_one, void* d_out, uint64_t* nodes_out,
                                    void* d_ws, uint64_t ws_bytes, void* stream);
/* Finisher over `count` nodes forming one complete tree level in order (the
 * gathered frontiers): the reference level loop (odd -> 0^128 pad) and
 * Keccak(root || le64(n_total) || 0^24).  Workspace from
 * mk_ssz_merkle_finish_workspace_bytes(count). */
uint64_t mk_ssz_merkle_finish_workspace_bytes(uint64_t count);
int mk_dev_ssz_merkle_finish_nodes(mk_call* call, const void* d_nodes, uint64_t count, uint64_t n_total,
                                   void* d_out32, void* d_ws, uint64_t ws_bytes, void* stream);
/* The same finisher for one field of a two-field struct whose fields are
 * both lists (hash.go:141-159; the State{registry, balances} of BASELINE
 * config 3): the list root goes to d_pair_block[32 slot, 32 slot + 32), and
 * whichever of the two finishers of one pair (slot 0 and slot 1, the same
 * `epoch`, launched in any order on any streams; neither waits for the other)
 * completes second writes the struct root Keccak(d_pair_block[0, 64)) to
 * d_pair_block[64, 96).  d_pair_block[96, 100) is the arrival word: zero
 * before the block's first use, then owned by the finishers.  Each pair takes
 * the next epoch of a counter over 1 .. 2^30 - 1 (wrapping; "newer" = ahead by
 * less than 2^29), so a pair left half-done by a failed call never completes
 * with the next one, and a finisher whose epoch is already behind the word's
 * when it starts is ignored.  That check is best-effort (it precedes the
 * finisher's slot store): two epochs' finishers of one slot must not run
 * concurrently -- order them on one stream or by events.  The
 * first finisher of an epoch zeroes d_pair_block[64, 96), so a pair that
 * never completes reads back as zeros, not as the previous pair's root.  The
 * block is MK_PAIR_BLOCK_BYTES, 16-B aligned; the caller waits for both
 * finishers before reading the struct root. */
#define MK_PAIR_BLOCK_BYTES 128
int mk_dev_ssz_merkle_finish_nodes_pair(mk_call* call, const void* d_nodes, uint64_t count, uint64_t n_total,
                                        void* d_pair_block, uint32_t slot, uint32_t epoch, void* d_ws,
                                        uint64_t ws_bytes, void* stream);
/* One or two lists' trees above a complete node level, to the roots, in ONE
 * launch (round 6): `count0` 32-B nodes at d_nodes0 (8-B
 * aligned) forming one complete level of a list of `n0` items, reduced with
 * the reference level loop (hash.go:225-236, odd -> 0^128) and mixed in
 * (Keccak(root || le64(n0) || 0^24), :237-238); count1 == 0: d_out gets the
 * 32-B list root.  count1 > 0: a second list (d_nodes1, count1, n1) side by
 * side, and d_out is a pair block laid out as for
 * mk_dev_ssz_merkle_finish_nodes_pair (list 0's root at [0, 32), list 1's at
 * [32, 64), the struct root Keccak(d_out[0, 64)) at [64, 96) written by
 * whichever list finishes second; both finishers are in this launch, so the
 * arrival word at [96, 100) is not used; `epoch` 1 .. 2^30 - 1 is checked
 * and otherwise unused): the State root of BASELINE config 3 from the two
 * trees' level-1 nodes in one call on one stream.  Each count is 1 .. 2^20; at most
 * 4096 such launches in flight per device (arrival counters).  Workspace from
 * mk_ssz_merkle_top_fused_workspace_bytes(count0, count1), 16-B aligned.
 * Replaces: ssz.merkleHash's level loop (shared/ssz/hash.go:223-239) for a
 * list whose lower levels are already built. */
uint64_t mk_ssz_merkle_top_fused_workspace_bytes(uint64_t count0, uint64_t count1);
int mk_dev_ssz_merkle_top_fused(mk_call* call, const void* d_nodes0, uint64_t count0, uint64_t n0,
                                const void* d_nodes1, uint64_t count1, uint64_t n1, void* d_out, uint32_t epoch,
                                void* d_ws, uint64_t ws_bytes, void* stream);
/* Finisher on one device: the reference level loop over the `nroots`
 * gathered shard roots (odd -> 0^128 pad), then Keccak(root || le64(n) || 0^24). */
int mk_dev_ssz_merkle_finish(mk_call* call, const void* d_roots, uint64_t nroots, uint64_t n_total, void* d_out32,
                             void* stream);
/* Single-process multi-device merkleHash for the cgo caller.  The items are
 * split by mk_ssz_merkle_shard_plan into `nshards` shards; shard s runs on
 * device devs[s] (devs == NULL: device s).  Every device uploads its shards
 * from its own host thread (chunked async copies from the caller's buffer),
 * so the PCIe links copy in parallel and a shard's passes overlap the upload
 * of the device's next shard; every shard is reduced to its frontier level (up to 1024
 * nodes).  When each device holds exactly one shard the frontiers are
 * all-gathered over RCCL (xGMI); otherwise they are copied to devs[0].  The
 * top levels and the length mix-in finish on devs[0]. */
int mk_ssz_merkle_hash_multi(mk_call* call, const uint8_t* items, uint64_t n, uint32_t item_len, int nshards,
                             const int* devs, uint8_t out[32]);
/* Device-resident form on devices 0..ndev-1 (one shard per device, shard d =
 * items [item_begin[d], item_begin[d+1]) of mk_ssz_merkle_shard_plan(n,
 * item_len, ndev), at d_shards[d] on device d).  Each device reduces its
 * shard to its frontier on streams[d] (NULL entries: the library's stream of
 * that device), the frontiers are all-gathered over RCCL and device 0
 * finishes into d_out32 (device 0 memory).  Enqueues only; the library's
 * per-device workspaces are reused by the next call, so successive calls
 * must be on the same streams (or synchronised). */
int mk_dev_ssz_merkle_hash_multi(mk_call* call, const void* const* d_shards, uint64_t n, uint32_t item_len,
                                 int ndev, void* d_out32, void* const* streams);

/* ---- struct hashing (hash.go:141-159) for flat fixed-layout records ------ */
/* The typed-registry path behind ssz.Hashable (hash.go:18-20, 57-58): a Go
 * wrapper flattens []*ValidatorRecord into n records of record_len bytes once
 * and describes the fields in declaration order ("XXX" fields omitted, as
 * structFields does, ssz_utils_cache.go:100).  Field hash = MK_FIELD_BYTES:
 * Keccak(le32(len) || bytes) (offset must be 4-byte aligned, record_len too);
 * MK_FIELD_RAW: raw little-endian scalar of len 1/2/4/8 (not hashed).
 * The struct root is Keccak(concat of field outputs). */
#define MK_FIELD_BYTES 1
#define MK_FIELD_RAW 2
typedef struct mk_field {
    uint32_t kind;
    uint32_t offset;
    uint32_t len;
} mk_field;
uint64_t mk_ssz_struct_msg_len(const mk_field* fields, uint32_t nfields);
/* roots of n records -> n x 32 bytes (one struct hash per record). */
int mk_ssz_struct_roots(mk_call* call, const uint8_t* records, uint64_t n, uint32_t record_len,
                        const mk_field* fields, uint32_t nfields, uint8_t* roots);
/* Device-resident struct roots (makeStructHasher per element,
 * hash.go:141-159): n records -> d_roots (n x 32) on `stream`; d_ws of at
 * least n * mk_ssz_struct_msg_len bytes. */
int mk_dev_ssz_struct_roots(mk_call* call, const void* d_records, uint64_t n, uint32_t record_len,
                            const mk_field* fields, uint32_t nfields, void* d_roots, void* d_ws, uint64_t ws_bytes,
                            void* stream);
/* TreeHash of a list of such structs: merkleHash over the n struct roots. */
uint64_t mk_ssz_struct_list_workspace_bytes(uint64_t n, const mk_field* fields, uint32_t nfields);
int mk_dev_ssz_struct_list_root(mk_call* call, const void* d_records, uint64_t n, uint32_t record_len,
                                const mk_field* fields, uint32_t nfields, void* d_out32, void* d_ws,
                                uint64_t ws_bytes, void* stream);
int mk_ssz_struct_list_root(mk_call* call, const uint8_t* records, uint64_t n, uint32_t record_len,
                            const mk_field* fields, uint32_t nfields, uint8_t out[32]);
/* The list root's first tree level in the struct-roots launch: d_roots (n x
 * 32) and the level-1 nodes of merkleHash over them, d_nodes (ceil(n/8) x 32:
 * node j = Keccak of roots 8j..8j+7, the ragged last window as merkleHash
 * hashes it, hash.go:205-228).  Optionally (nvalues > 0) the same launch
 * also writes the level-1 nodes of merkleHash over a second list -- nvalues
 * items of value_len bytes (8, 16, 32, 64 or 128) at a 16-B aligned
 * d_values, more than one chunk: ceil(nvalues * value_len / 256) nodes to
 * d_value_nodes (the State's balances, BASELINE config 3).  Finish each with
 * mk_dev_ssz_merkle_finish_nodes(nodes, count, n) -- the split lets the two
 * trees' latency-bound levels run side by side.
 * mk_ssz_struct_list_level1_ok says whether the records qualify (the
 * ValidatorRecord layout at a 16-B aligned address, n >= 2^18); otherwise
 * mk_dev_ssz_struct_list_level1 returns MK_EINVAL. */
int mk_ssz_struct_list_level1_ok(const void* d_records, uint64_t n, uint32_t record_len, const mk_field* fields,
                                 uint32_t nfields);
int mk_dev_ssz_struct_list_level1(mk_call* call, const void* d_records, uint64_t n, uint32_t record_len,
                                  const mk_field* fields, uint32_t nfields, void* d_roots, void* d_nodes,
                                  const void* d_values, uint64_t nvalues, uint32_t value_len, void* d_value_nodes,
                                  void* stream);
/* A stream of states (the State{registry, balances} of BASELINE config 3,
 * hash.go:118-159, one TreeHash per state) with each state's trees folded
 * into the NEXT state's struct launch: mk_dev_ssz_struct_list_level1 plus,
 * in the same launch, levels 2..10 of the PREVIOUS state's registry tree from
 * its level-1 nodes d_prev_nodes (NULL for the first state) over every
 * complete 512-node subtree, into d_prev_levels, and levels 2..4 of its
 * second list's tree from d_prev_value_nodes over every complete 128-node
 * subtree, into d_prev_value_levels (NULL: none).  Buffer sizes from
 * mk_ssz_struct_pipe_levels_bytes(n, nvalues, value_len, which): which = 0
 * the registry's, 1 the second list's.  Then mk_dev_ssz_struct_pipe_top
 * finishes each of the previous state's trees (the ragged last subtree, the
 * levels above the slots and the length mix-in) as one field of a pair
 * block, on another stream, beside the next launch.  Takes what
 * mk_ssz_struct_pipe_ok accepts on the same stream (as
 * mk_ssz_struct_list_level1_ok, with exactly 4 groups of 1024 records per
 * workgroup: 3 x 2^18 < n <= 2^20 on 256 CUs; a second list of at most 128
 * windows per workgroup, e.g. n 8-B balances); MK_EINVAL otherwise.  The
 * previous state must have the same n and second-list shape. */
int mk_ssz_struct_pipe_ok(const void* d_records, uint64_t n, uint32_t record_len, const mk_field* fields,
                          uint32_t nfields, void* stream);
uint64_t mk_ssz_struct_pipe_levels_bytes(uint64_t n, uint64_t nvalues, uint32_t value_len, uint32_t which);
uint64_t mk_ssz_struct_pipe_top_workspace_bytes(uint64_t n, uint64_t nvalues, uint32_t value_len, uint32_t which);
int mk_dev_ssz_struct_list_level1_pipe(mk_call* call, const void* d_records, uint64_t n, uint32_t record_len,
                                       const mk_field* fields, uint32_t nfields, void* d_roots, void* d_nodes,
                                       const void* d_values, uint64_t nvalues, uint32_t value_len,
                                       void* d_value_nodes, const void* d_prev_nodes, void* d_prev_levels,
                                       const void* d_prev_value_nodes, void* d_prev_value_levels, void* stream);
/* One tree's root of a state whose slot levels a later pipelined launch
 * built (d_nodes: its level-1 nodes, d_levels: those levels; which = 0 the
 * registry of n records, 1 the second list of nvalues items of value_len
 * bytes), as one field of a pair block (mk_dev_ssz_merkle_finish_nodes_pair
 * semantics: slot, epoch, the second finisher hashes the struct root). */
int mk_dev_ssz_struct_pipe_top(mk_call* call, const void* d_nodes, uint64_t n, uint64_t nvalues,
                               uint32_t value_len, uint32_t which, void* d_levels, void* d_pair_block, uint32_t slot,
                               uint32_t epoch, void* d_ws, uint64_t ws_bytes, void* stream);

/* ---- hashutil.MerkleRoot (merkleRoot.go:12-30) -------------------------- */
/* Root of the heap o[i] = Hash(o[2i] || o[2i+1]) over leaves
 * o[n+i] = Hash(values[i]); values i = data[offs[i], offs[i+1]).  leaves_out
 * (optional, n x 32) receives Hash(values[i]): the reference overwrites its
 * input slice with them (merkleRoot.go:16-19) and a drop-in keeps that side
 * effect.  n == 0 is MK_EINVAL (the reference panics: index out of range). */
int mk_merkle_root(mk_call* call, const uint8_t* data, const uint64_t* offs, uint64_t n, uint8_t* leaves_out,
                   uint8_t out[32]);
uint64_t mk_merkle_root_workspace_bytes(uint64_t n);
/* Device-resident: d_offs (n+1, device) or fixed_len; d_heap of
 * mk_merkle_root_workspace_bytes(n); d_leaves32 optional (n x 32). */
int mk_dev_merkle_root(mk_call* call, const void* d_data, const uint64_t* d_offs, uint64_t n, uint32_t fixed_len,
                       void* d_heap, uint64_t heap_bytes, void* d_leaves32, void* d_out32, void* stream);

/* ---- trieutil deposit trie (deposit_trie.go:29-81) ---------------------- */
/* Level array of a depth-`depth` trie with room for `capacity` leaves: level
 * d (d = 0: leaf hashes Hash(deposit)) starts at node
 * sum_{i<d} ceil(capacity / 2^i) and holds ceil(count / 2^d) nodes.  Empty
 * nodes are 0^32 (Go map miss), root = level `depth` node 0 (0^32 when
 * count == 0). */
uint64_t mk_deposit_trie_levels_bytes(uint64_t capacity, uint32_t depth);
/* Batch build of n deposits (message i = data[offs[i], offs[i+1])) = n calls
 * of UpdateDepositTrie.  levels_out (nullable) receives the level array with
 * capacity n (the data GenerateMerkleBranch reads). */
int mk_deposit_trie_build(mk_call* call, const uint8_t* data, const uint64_t* offs, uint64_t n, uint32_t depth,
                          uint8_t* levels_out, uint8_t root[32]);
/* Device-resident append: the trie in d_levels (capacity `capacity`) holds
 * `count` deposits; deposits count .. count+k-1 are d_data[d_offs[i],
 * d_offs[i+1]) (i < k) or, with d_offs == NULL, fixed_len-byte records (the
 * 280-B deposit-data layout of core/blocks/block.go:103-130).  Hashes the k
 * leaves and recomputes only the right edge of every level above them
 * (<= k/2^d + 2 nodes at level d): UpdateDepositTrie's O(depth) path per
 * deposit (deposit_trie.go:29-40), batched.  count == 0 is the batch build.
 * The new root goes to d_root32.  count + k <= capacity. */
int mk_dev_deposit_trie_append(mk_call* call, void* d_levels, uint64_t capacity, uint64_t count, const void* d_data,
                               const uint64_t* d_offs, uint64_t k, uint32_t fixed_len, uint32_t depth,
                               void* d_root32, void* stream);
/* Batch build front: the leaf hashes Hash(deposit) of n deposits into level 0
 * of an empty trie plus levels 1 .. d_to (the root to d_root32 when d_to ==
 * depth; d_root32 may be NULL otherwise).  Deposits as in
 * mk_dev_deposit_trie_append.  With mk_dev_deposit_trie_levels(d_to, depth)
 * this splits one batch build (deposit_trie.go:29-40) across two streams. */
int mk_dev_deposit_trie_build(mk_call* call, void* d_levels, uint64_t capacity, const void* d_data,
                              const uint64_t* d_offs, uint64_t n, uint32_t fixed_len, uint32_t d_to, uint32_t depth,
                              void* d_root32, void* stream);
/* A stream of equal-size tries with each trie's wide top folded into the
 * NEXT trie's front: levels 0..2 of the trie in d_levels (its leaves and the
 * nodes over 2 and 4 of them) and, in the same launch, levels 3..7 of the
 * previous trie in d_prev_levels (NULL for the first trie; the same n and
 * capacity; its levels 0..2 from the previous call).  Then
 * mk_dev_deposit_trie_pipe_top(d_prev_levels, ..) finishes the previous trie
 * (on another stream, beside the next front), and
 * mk_dev_deposit_trie_levels(d_levels, .., 2, depth) the last one.  Takes what
 * mk_deposit_trie_pipe_ok accepts on the same stream (280-B deposits, 16-B
 * aligned, n a multiple of 4096 and at most 4096 x the CUs the stream may
 * use, depth >= 7); MK_EINVAL otherwise.  pipe_ok returns 1 or 0 (0 also
 * when the stream cannot be bound). */
int mk_deposit_trie_pipe_ok(const void* d_data, uint64_t n, uint32_t deposit_len, uint32_t depth, void* stream);
/* Levels 8 .. depth and the root of a trie whose levels 0..7 are complete
 * (a pipelined front's previous trie), in launches of at most one wave per
 * SIMD, which run beside the next pipelined front instead of after it. */
int mk_dev_deposit_trie_pipe_top(mk_call* call, void* d_levels, uint64_t capacity, uint64_t count, uint32_t depth,
                                 void* d_root32, void* stream);
int mk_dev_deposit_trie_build_pipe(mk_call* call, void* d_levels, void* d_prev_levels, uint64_t capacity,
                                   const void* d_data, uint64_t n, uint32_t deposit_len, uint32_t depth,
                                   void* stream);
/* Levels d_from+1 .. d_to of the batch build of a `count`-deposit trie whose
 * level d_from is complete (the root to d_root32 when d_to == depth): lets a
 * caller hash the leaves and the wide levels of trie i+1 on one stream while
 * the narrow, latency-bound top of trie i runs on another. */
int mk_dev_deposit_trie_levels(mk_call* call, void* d_levels, uint64_t capacity, uint64_t count, uint32_t d_from,
                               uint32_t d_to, uint32_t depth, void* d_root32, void* stream);
/* GenerateMerkleBranch (deposit_trie.go:43-58) from a device level array:
 * d_branch[d] = sibling of `index`'s ancestor at level d (0^32 if absent). */
int mk_dev_deposit_trie_branch(mk_call* call, const void* d_levels, uint64_t capacity, uint64_t count,
                               uint32_t depth, uint64_t index, void* d_branch, void* stream);

/* Device-resident trie handle: the Go DepositTrie (deposit_trie.go:13-16)
 * holds one.  Levels stay in HBM (capacity doubles on demand); appends
 * recompute only the right edge, so powchain's read-Root-then-Update loop
 * (powchain/service.go:379-386) costs O(depth) hashes per deposit. */
typedef struct mk_trie mk_trie;
int mk_deposit_trie_new(mk_call* call, uint32_t depth, uint64_t capacity, mk_trie** out);
void mk_deposit_trie_free(mk_trie* t);
uint64_t mk_deposit_trie_count(const mk_trie* t);
/* Appends k deposits (host data, message i = data[offs[i], offs[i+1])). */
int mk_deposit_trie_append(mk_call* call, mk_trie* t, const uint8_t* data, const uint64_t* offs, uint64_t k);
/* powchain's deposit-log loop in one call (ProcessDepositLog -> saveInTrie,
 * powchain/service.go:248-258, 379-386): for each of the k logs in order,
 * deposit j (data[offs[j], offs[j+1])) is appended iff the trie's Root()
 * before it equals log_roots[32 j .. 32 j + 32) (the merkle root the log
 * carries); a mismatching log is skipped, as the reference skips a log
 * whose saveInTrie fails, and processing continues with the next log.
 * accepted[j] = 1 if deposit j was appended, else 0.  All roots are
 * computed on the device in parallel (one chain of `depth` permutations
 * per log), so a batch costs about one append. */
int mk_deposit_trie_save_logs(mk_call* call, mk_trie* t, const uint8_t* data, const uint64_t* offs, uint64_t k,
                              const uint8_t* log_roots, uint8_t* accepted);
int mk_deposit_trie_root(mk_call* call, mk_trie* t, uint8_t root[32]);
/* depth x 32 bytes: GenerateMerkleBranch(index). */
int mk_deposit_trie_branch(mk_call* call, mk_trie* t, uint64_t index, uint8_t* branch);
/* Leaf hashes [first, first + cnt) (Hash(deposit)), cnt x 32 bytes. */
int mk_deposit_trie_leaves(mk_call* call, mk_trie* t, uint64_t first, uint64_t cnt, uint8_t* out);

/* Batched VerifyMerkleBranch: ok[i] = fold(leaves[i], branches[i*depth..],
 * indices[i] + 2^tree_depth) == roots[i]. */
int mk_verify_merkle_branches(mk_call* call, const uint8_t* leaves, const uint8_t* branches,
                              const uint64_t* indices, uint64_t n, uint32_t depth, uint32_t tree_depth,
                              const uint8_t* roots, uint8_t* ok);

/* ---- synthetic inputs (bench / tests) ----------------------------------- */
/* Bytes [8*word0, 8*word0 + nbytes) of the SplitMix64 stream;
 * nbytes must be a multiple of 8. */
int mk_dev_synth_fill(mk_call* call, void* d_dst, uint64_t nbytes, uint64_t seed, uint64_t word0, void* stream);

/* ---- measurement -------------------------------------------------------- */
/* When enabled, every dev merkle call records hipEvents around its dominant
 * (leaf) kernel launches on the call's stream; mk_prof_read synchronises those
 * events and returns the summed milliseconds, launch count, algorithmic
 * Keccak-f permutations and digests (hashes) of those launches, then resets.
 * Any out-pointer may be NULL. */
int mk_prof_enable(int on);
int mk_prof_read(mk_call* call, double* leaf_ms, uint64_t* leaf_launches, double* leaf_perms, double* leaf_hashes);

#ifdef __cplusplus
}
#endif
#endif /* PRYSM_MERKLE_H */
