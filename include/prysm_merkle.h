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
 *   - Every function returns 0 (MK_OK) or a negative MK_E* code; mk_strerror()
 *     names it and mk_last_error() returns the thread's last detailed message.
 *     Nothing panics across the boundary; there is NO CPU fallback: without a
 *     usable gfx950 device every compute entry point returns MK_ENODEV.
 *   - Host-buffer entry points (no `dev` in the name) borrow caller memory for
 *     the duration of the call only (cgo rule: Go memory is never retained);
 *     `[][]byte` inputs are passed flattened as (data, offs[n+1]).
 *   - `dev` entry points take device pointers (HBM-resident inputs) and a
 *     hipStream_t passed as void* (NULL = the device's default stream); they
 *     enqueue work and return without synchronising.  Their scratch space is
 *     caller-provided (size from the *_workspace_bytes query), so they never
 *     allocate and can be captured into a hipGraph.
 *   - Thread safety: host-buffer entry points may be called concurrently from
 *     any OS thread; each takes the current device's lock.  mk_init selects the
 *     device for the calling thread.
 *   - Digests are 32 bytes; node arrays are n x 32 contiguous bytes.
 */
#ifndef PRYSM_MERKLE_H
#define PRYSM_MERKLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MK_OK 0
#define MK_EINVAL (-22)  /* bad argument (also: reference panics, e.g. len(list[0]) == 0) */
#define MK_ENODEV (-19)  /* no usable gfx950 device / device index out of range */
#define MK_ENOMEM (-12)  /* device or host allocation failed / workspace too small */
#define MK_EHIP (-5)     /* a HIP runtime call failed (see mk_last_error) */
#define MK_ECOMM (-71)   /* RCCL failure in the multi-device path */

/* ---- lifecycle --------------------------------------------------------- */
int mk_init(int device);          /* idempotent; binds the calling thread to `device` */
int mk_device_count(void);        /* number of visible gfx950 devices (0 if none) */
const char* mk_strerror(int code);
const char* mk_last_error(void);  /* thread-local detail of the last failure */
const char* mk_version(void);

/* ---- hashutil.Hash (hash.go:11-25): legacy Keccak-256 ------------------- */
/* Single message.  Provided for completeness; Go keeps single Hash calls on
 * the CPU (launch latency, and Hash cannot return an error). */
int mk_hash(const uint8_t* data, uint64_t len, uint8_t out[32]);
/* Batched form ("HashBatch"): n messages of msg_len bytes, contiguous -> n*32. */
int mk_hash_batch(const uint8_t* in, uint64_t n, uint32_t msg_len, uint8_t* out);
/* Variable-length batch: message i = in[offs[i], offs[i+1]) -> n*32. */
int mk_hash_batch_var(const uint8_t* in, const uint64_t* offs, uint64_t n, uint8_t* out);
int mk_dev_hash_batch(const void* d_in, uint64_t n, uint32_t msg_len, void* d_out, void* stream);
int mk_dev_hash_batch_var(const void* d_in, const uint64_t* d_offs, uint64_t n, void* d_out, void* stream);

/* ---- ssz.merkleHash (hash.go:194-239) ---------------------------------- */
/* n items of item_len bytes each, contiguous (the flattened [][]byte; every
 * list TreeHash builds has uniform element length).  out = 32-B result.
 * item_len == 0 with n > 0 is the reference's divide-by-zero panic: MK_EINVAL. */
int mk_ssz_merkle_hash(const uint8_t* items, uint64_t n, uint32_t item_len, uint8_t out[32]);
uint64_t mk_ssz_merkle_workspace_bytes(uint64_t n, uint32_t item_len);
int mk_dev_ssz_merkle_hash(const void* d_items, uint64_t n, uint32_t item_len, void* d_out32,
                           void* d_ws, uint64_t ws_bytes, void* stream);

/* ---- subtree sharding across GPUs ----------------------- */
/* Split a merkleHash of n items over `nshards` devices: every shard is a
 * power-of-two-aligned run of 2^height chunks.  item_begin[nshards+1] gets
 * each shard's item range (empty shards have begin == end); *nonempty the
 * number of non-empty shards.  When the tree is too small to shard
 * (*nonempty == 1) shard 0 holds everything and is hashed with
 * mk_dev_ssz_merkle_hash instead. */
int mk_ssz_merkle_shard_plan(uint64_t n, uint32_t item_len, uint32_t nshards, uint32_t* height,
                             uint32_t* nonempty, uint64_t* item_begin);
/* Root (32 B, height `height` above the chunks) of one shard.  pad_at_one=1
 * for every shard of a tree with >1 non-empty shard: a ragged last shard keeps
 * applying the reference's odd rule (node || 0^128) up to `height`. */
int mk_dev_ssz_merkle_subtree(const void* d_shard_items, uint64_t shard_n, uint32_t item_len,
                              uint32_t height, int pad_at_one, void* d_out32, void* d_ws,
                              uint64_t ws_bytes, void* stream);
/* Frontier variant: stop `frontier_log2` levels below the shard root and
 * write the shard's nodes at height (height - frontier_log2) to d_out (32 B
 * each, 2^frontier_log2 of them, fewer for a ragged last shard; *nodes_out
 * gets the count).  The shards' frontiers, concatenated in shard order, are
 * that level of the whole tree, so ranks gather a few KB each and the top
 * levels move to the finisher (mk_dev_ssz_merkle_finish_nodes), which can
 * overlap the ranks' next Merkleization.  0 < frontier_log2 < height. */
int mk_dev_ssz_merkle_subtree_frontier(const void* d_shard_items, uint64_t shard_n, uint32_t item_len,
                                       uint32_t height, uint32_t frontier_log2, int pad_at_one, void* d_out,
                                       uint64_t* nodes_out, void* d_ws, uint64_t ws_bytes, void* stream);
/* The same subtree continued from one of its node levels: `count` 32-B nodes
 * (a shard's level, e.g. the output of the leaf pass) reduced for `height`
 * levels with the reference's odd rule (hash.go:225-235; pad_at_one as
 * above), stopping `frontier_log2` levels below the top (0 = to the top
 * node).  Lets a rank split its shard into the leaf pass and the narrower
 * node passes and run the latter on another stream (prysm_amd/parallel.py
 * ShardedMerklePipeline).  Workspace from
 * mk_ssz_merkle_node_frontier_workspace_bytes. */
uint64_t mk_ssz_merkle_node_frontier_workspace_bytes(uint64_t count, uint32_t height, uint32_t frontier_log2);
int mk_dev_ssz_merkle_node_frontier(const void* d_nodes, uint64_t count, uint32_t height, uint32_t frontier_log2,
                                    int pad_at_one, void* d_out, uint64_t* nodes_out, void* d_ws,
                                    uint64_t ws_bytes, void* stream);
/* Finisher over `count` nodes forming one complete tree level in order (the
 * gathered frontiers): the reference level loop (odd -> 0^128 pad) and
 * Keccak(root || le64(n_total) || 0^24).  Workspace from
 * mk_ssz_merkle_finish_workspace_bytes(count). */
uint64_t mk_ssz_merkle_finish_workspace_bytes(uint64_t count);
int mk_dev_ssz_merkle_finish_nodes(const void* d_nodes, uint64_t count, uint64_t n_total, void* d_out32,
                                   void* d_ws, uint64_t ws_bytes, void* stream);
/* Finisher on one device: the reference level loop over the `nroots`
 * gathered shard roots (odd -> 0^128 pad), then Keccak(root || le64(n) || 0^24). */
int mk_dev_ssz_merkle_finish(const void* d_roots, uint64_t nroots, uint64_t n_total, void* d_out32,
                             void* stream);
/* Single-process multi-device merkleHash for the cgo caller: shards the host
 * items over devices 0..ndev-1, reduces every shard to its frontier level
 * (up to 1024 nodes), all-gathers the frontiers over RCCL (xGMI) and finishes
 * on device 0. */
int mk_ssz_merkle_hash_multi(const uint8_t* items, uint64_t n, uint32_t item_len, int ndev,
                             uint8_t out[32]);

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
int mk_ssz_struct_roots(const uint8_t* records, uint64_t n, uint32_t record_len, const mk_field* fields,
                        uint32_t nfields, uint8_t* roots);
/* Device-resident struct roots (makeStructHasher per element,
 * hash.go:141-159): n records -> d_roots (n x 32) on `stream`; d_ws of at
 * least n * mk_ssz_struct_msg_len bytes.  Lets a caller run the list's
 * merkleHash on another stream (a stream of states: struct roots of state
 * i+1 overlap the merkle top of state i). */
int mk_dev_ssz_struct_roots(const void* d_records, uint64_t n, uint32_t record_len, const mk_field* fields,
                            uint32_t nfields, void* d_roots, void* d_ws, uint64_t ws_bytes, void* stream);
/* TreeHash of a list of such structs: merkleHash over the n struct roots. */
uint64_t mk_ssz_struct_list_workspace_bytes(uint64_t n, const mk_field* fields, uint32_t nfields);
int mk_dev_ssz_struct_list_root(const void* d_records, uint64_t n, uint32_t record_len, const mk_field* fields,
                                uint32_t nfields, void* d_out32, void* d_ws, uint64_t ws_bytes, void* stream);
int mk_ssz_struct_list_root(const uint8_t* records, uint64_t n, uint32_t record_len, const mk_field* fields,
                            uint32_t nfields, uint8_t out[32]);

/* ---- hashutil.MerkleRoot (merkleRoot.go:12-30) -------------------------- */
/* Root of the heap o[i] = Hash(o[2i] || o[2i+1]) over leaves
 * o[n+i] = Hash(values[i]); values i = data[offs[i], offs[i+1]).  leaves_out
 * (optional, n x 32) receives Hash(values[i]): the reference overwrites its
 * input slice with them (merkleRoot.go:16-19) and a drop-in keeps that side
 * effect.  n == 0 is MK_EINVAL (the reference panics: index out of range). */
int mk_merkle_root(const uint8_t* data, const uint64_t* offs, uint64_t n, uint8_t* leaves_out, uint8_t out[32]);
uint64_t mk_merkle_root_workspace_bytes(uint64_t n);
/* Device-resident: d_offs (n+1, device) or fixed_len; d_heap of
 * mk_merkle_root_workspace_bytes(n); d_leaves32 optional (n x 32). */
int mk_dev_merkle_root(const void* d_data, const uint64_t* d_offs, uint64_t n, uint32_t fixed_len, void* d_heap,
                       uint64_t heap_bytes, void* d_leaves32, void* d_out32, void* stream);

/* ---- trieutil deposit trie (deposit_trie.go:29-81) ---------------------- */
/* Batch build of the depth-`depth` sparse trie over n deposits (message i =
 * data[offs[i], offs[i+1])).  Equals n calls of UpdateDepositTrie: empty nodes
 * are 0^32 (map miss), root = node 1 (0^32 when n == 0).  levels_out
 * (nullable) receives, for d = 0..depth, ceil(n / 2^d) nodes of level d
 * (d = 0: leaf hashes), concatenated — the data GenerateMerkleBranch reads. */
uint64_t mk_deposit_trie_levels_bytes(uint64_t n, uint32_t depth);
int mk_deposit_trie_build(const uint8_t* data, const uint64_t* offs, uint64_t n, uint32_t depth,
                          uint8_t* levels_out, uint8_t root[32]);
/* Device-resident build: d_levels (mk_deposit_trie_levels_bytes) and the
 * deposits in device memory; root to d_root32.  Deposit i is
 * d_data[d_offs[i], d_offs[i+1]) or, with d_offs == NULL, the fixed-length
 * record d_data[i*fixed_len, (i+1)*fixed_len) (the 280-B deposit-data layout
 * of core/blocks/block.go:103-130). */
int mk_dev_deposit_trie_build(const void* d_data, const uint64_t* d_offs, uint64_t n, uint32_t fixed_len,
                              uint32_t depth, void* d_levels, void* d_root32, void* stream);
/* Batched VerifyMerkleBranch: ok[i] = fold(leaves[i], branches[i*depth..],
 * indices[i] + 2^tree_depth) == roots[i]. */
int mk_verify_merkle_branches(const uint8_t* leaves, const uint8_t* branches, const uint64_t* indices,
                              uint64_t n, uint32_t depth, uint32_t tree_depth, const uint8_t* roots,
                              uint8_t* ok);

/* ---- synthetic inputs (bench / tests) ----------------------------------- */
/* Bytes [8*word0, 8*word0 + nbytes) of the SplitMix64 stream;
 * nbytes must be a multiple of 8. */
int mk_dev_synth_fill(void* d_dst, uint64_t nbytes, uint64_t seed, uint64_t word0, void* stream);

/* ---- measurement -------------------------------------------------------- */
/* When enabled, every dev merkle call records hipEvents around its dominant
 * (leaf) kernel launches on the call's stream; mk_prof_read synchronises those
 * events and returns the summed milliseconds, launch count, algorithmic
 * Keccak-f permutations and digests (hashes) of those launches, then resets.
 * Any out-pointer may be NULL. */
int mk_prof_enable(int on);
int mk_prof_read(double* leaf_ms, uint64_t* leaf_launches, double* leaf_perms, double* leaf_hashes);

#ifdef __cplusplus
}
#endif
#endif /* PRYSM_MERKLE_H */
