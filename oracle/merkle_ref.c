/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see keccak_ref.c header).
 *
 * CPU restatement of the reference's Merkleization algorithms:
 *   - ssz.merkleHash            shared/ssz/hash.go:194-239
 *       lenc = le64(len(list)) || 0^24              (hash.go:196-197)
 *       emptyChunk = 0^128 (sszChunkSize)            (hash.go:15,200)
 *       len==0 -> chunks=[emptyChunk]                (hash.go:202-204)
 *       len(list[0])<128 -> pack 128/len(list[0]) items per chunk, last chunk
 *                           may be short            (hash.go:205-220)
 *       else chunks = list                           (hash.go:221-223)
 *       while len>1: odd -> append emptyChunk (128 B at EVERY level);
 *                    next[i] = Hash(c[2i] || c[2i+1]) (hash.go:225-235)
 *       return Hash(chunks[0] || lenc)               (hash.go:237)
 *   - trieutil.DepositTrie       shared/trieutil/deposit_trie.go:29-63
 *       depth 32 (shared/params/config.go:109), leaves Hash(depositData),
 *       missing map keys read as 0^32, root = node 1 (0^32 when empty).
 *       The batch build below equals the incremental UpdateDepositTrie
 *       (tests/test_oracle.py checks it against a literal dict restatement).
 *   - trieutil.VerifyMerkleBranch deposit_trie.go:68-81
 *   - hashutil.MerkleRoot        shared/hashutil/merkleRoot.go:12-30
 *
 * Synthetic inputs: counter-based SplitMix64 — byte b of a
 * synthetic stream is byte (b % 8) (little-endian) of word b/8, word k =
 * mix(seed + k * 0x9E3779B97F4A7C15).  The HIP product generates the same
 * stream on the device (k_synth in prysm_amd/csrc/merkle_kernels.hip).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define CHUNK 128
#define HASHLEN 32

uint64_t or_splitmix64_word(uint64_t seed, uint64_t k) {
    uint64_t z = seed + k * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* bytes [8*word0, 8*word0 + nbytes) of the synthetic stream */
void or_fill_splitmix(uint8_t* out, uint64_t nbytes, uint64_t seed, uint64_t word0) {
    uint64_t nw = nbytes / 8;
    for (uint64_t k = 0; k < nw; ++k) {
        uint64_t w = or_splitmix64_word(seed, word0 + k);
        for (int b = 0; b < 8; ++b) out[8 * k + b] = (uint8_t)(w >> (8 * b));
    }
    if (nbytes % 8) {
        uint64_t w = or_splitmix64_word(seed, word0 + nw);
        for (uint64_t b = 0; b < nbytes % 8; ++b) out[8 * nw + b] = (uint8_t)(w >> (8 * b));
    }
}

/* ---- generic level loop over "chunks" supplied by a callback ---------- */
typedef uint64_t (*chunk_fn)(void* ctx, uint64_t i, uint8_t* buf); /* returns length */

/* Hashes chunk pairs (level 0) then 32-B node pairs until one node remains
 * or `max_levels` hashing levels were done.  `global_count_fn` semantics:
 * the subtree variant must keep applying the odd rule when the global tree
 * still has >1 node (see or_merkle_subtree_gen).  Returns root length. */
static uint64_t reduce_levels(uint64_t nchunks, uint32_t max_chunk_len, chunk_fn get, void* ctx,
                              uint32_t max_levels, int keep_padding_at_one, uint8_t* root,
                              int nthreads) {
    if (nchunks == 0) return 0;
    uint8_t zero[CHUNK];
    memset(zero, 0, sizeof zero);
    if (max_levels == 0 || (nchunks == 1 && !keep_padding_at_one)) {
        return get(ctx, 0, root);
    }
    uint64_t count = (nchunks + 1) / 2;
    uint8_t* cur = (uint8_t*)malloc(count * HASHLEN);
    /* level 0: chunk pairs */
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
    {
        uint8_t* msg = (uint8_t*)malloc(2 * (size_t)max_chunk_len + CHUNK);
#pragma omp for schedule(static)
        for (int64_t j = 0; j < (int64_t)count; ++j) {
            uint64_t l = get(ctx, 2 * (uint64_t)j, msg);
            uint64_t r;
            if (2 * (uint64_t)j + 1 < nchunks) {
                r = get(ctx, 2 * (uint64_t)j + 1, msg + l);
            } else {
                memset(msg + l, 0, CHUNK);
                r = CHUNK;
            }
            or_keccak256(msg, l + r, cur + HASHLEN * j);
        }
        free(msg);
    }
    uint32_t levels = 1;
    while ((count > 1 || keep_padding_at_one) && levels < max_levels) {
        uint64_t next = (count + 1) / 2;
        uint8_t* nxt = (uint8_t*)malloc(next * HASHLEN);
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
        for (int64_t j = 0; j < (int64_t)next; ++j) {
            uint8_t msg[HASHLEN + CHUNK];
            memcpy(msg, cur + 2 * HASHLEN * j, HASHLEN);
            uint64_t len;
            if (2 * (uint64_t)j + 1 < count) {
                memcpy(msg + HASHLEN, cur + (2 * j + 1) * HASHLEN, HASHLEN);
                len = 2 * HASHLEN;
            } else {
                memset(msg + HASHLEN, 0, CHUNK);
                len = HASHLEN + CHUNK;
            }
            or_keccak256(msg, len, nxt + HASHLEN * j);
        }
        free(cur);
        cur = nxt;
        count = next;
        ++levels;
    }
    memcpy(root, cur, HASHLEN);
    free(cur);
    return HASHLEN;
}

static void final_hash(const uint8_t* root, uint64_t root_len, uint64_t n, uint8_t out[32]) {
    uint8_t* msg = (uint8_t*)malloc(root_len + HASHLEN);
    memcpy(msg, root, root_len);
    memset(msg + root_len, 0, HASHLEN);
    for (int b = 0; b < 8; ++b) msg[root_len + b] = (uint8_t)(n >> (8 * b));
    or_keccak256(msg, root_len + HASHLEN, out);
    free(msg);
}

/* ---- fixed-size items in one flat buffer ------------------------------ */
struct flat_ctx {
    const uint8_t* items;
    uint64_t total;
    uint64_t cb;
};
static uint64_t flat_chunk(void* c, uint64_t i, uint8_t* buf) {
    struct flat_ctx* f = (struct flat_ctx*)c;
    uint64_t lo = i * f->cb, hi = lo + f->cb;
    if (hi > f->total) hi = f->total;
    memcpy(buf, f->items + lo, hi - lo);
    return hi - lo;
}

static uint64_t chunk_bytes(uint32_t item_len) {
    return item_len < CHUNK ? (uint64_t)(CHUNK / item_len) * item_len : item_len;
}

int or_merkle_hash(const uint8_t* items, uint64_t n, uint32_t item_len, uint8_t out[32], int nthreads) {
    uint8_t root[CHUNK > HASHLEN ? 4096 : 4096];
    if (n == 0) {
        uint8_t z[CHUNK];
        memset(z, 0, CHUNK);
        final_hash(z, CHUNK, 0, out);
        return 0;
    }
    if (item_len == 0) return -1; /* reference: integer divide by zero panic (hash.go:207) */
    struct flat_ctx f = {items, n * (uint64_t)item_len, chunk_bytes(item_len)};
    if (f.cb > sizeof root) return -2;
    uint64_t nchunks = (f.total + f.cb - 1) / f.cb;
    uint64_t rl = reduce_levels(nchunks, (uint32_t)f.cb, flat_chunk, &f, 0xFFFFFFFFu, 0, root, nthreads);
    final_hash(root, rl, n, out);
    return 0;
}

/* ---- variable-length items: exact reference list semantics ------------ */
struct var_ctx {
    const uint8_t* data;
    const uint64_t* offs;
    uint64_t n;
    uint64_t per; /* items per chunk (1 when len(list[0]) >= 128) */
};
static uint64_t var_chunk(void* c, uint64_t i, uint8_t* buf) {
    struct var_ctx* v = (struct var_ctx*)c;
    uint64_t a = i * v->per, b = a + v->per;
    if (b > v->n) b = v->n;
    uint64_t len = v->offs[b] - v->offs[a];
    memcpy(buf, v->data + v->offs[a], len);
    return len;
}

int or_merkle_hash_var(const uint8_t* data, const uint64_t* offs, uint64_t n, uint8_t out[32]) {
    if (n == 0) {
        uint8_t z[CHUNK];
        memset(z, 0, CHUNK);
        final_hash(z, CHUNK, 0, out);
        return 0;
    }
    uint64_t l0 = offs[1] - offs[0];
    if (l0 == 0) return -1; /* reference panics: integer divide by zero */
    struct var_ctx v = {data, offs, n, l0 < CHUNK ? CHUNK / l0 : 1};
    uint64_t maxc = 0;
    uint64_t nchunks = (n + v.per - 1) / v.per;
    for (uint64_t i = 0; i < nchunks; ++i) {
        uint64_t a = i * v.per, b = a + v.per;
        if (b > n) b = n;
        if (offs[b] - offs[a] > maxc) maxc = offs[b] - offs[a];
    }
    uint8_t* root = (uint8_t*)malloc(maxc > HASHLEN ? maxc : HASHLEN);
    uint64_t rl = reduce_levels(nchunks, (uint32_t)maxc, var_chunk, &v, 0xFFFFFFFFu, 0, root, 1);
    final_hash(root, rl, n, out);
    free(root);
    return 0;
}

/* ---- synthetic SplitMix64 items (no materialised buffer) -------------- */
struct gen_ctx {
    uint64_t seed, total, cb, chunk0;
};
static uint64_t gen_chunk(void* c, uint64_t i, uint8_t* buf) {
    struct gen_ctx* g = (struct gen_ctx*)c;
    uint64_t lo = (g->chunk0 + i) * g->cb, hi = lo + g->cb;
    if (hi > g->total) hi = g->total;
    /* generic byte-addressed fill */
    uint64_t w0 = lo / 8, skip = lo % 8, len = hi - lo;
    uint8_t tmp[4096 + 16];
    or_fill_splitmix(tmp, skip + len, g->seed, w0);
    memcpy(buf, tmp + skip, len);
    return len;
}

int or_merkle_hash_gen(uint64_t n, uint32_t item_len, uint64_t seed, uint8_t out[32], int nthreads) {
    if (n == 0) return or_merkle_hash(NULL, 0, item_len, out, 1);
    if (item_len == 0) return -1;
    struct gen_ctx g = {seed, n * (uint64_t)item_len, chunk_bytes(item_len), 0};
    if (g.cb > 4096) return -2;
    uint64_t nchunks = (g.total + g.cb - 1) / g.cb;
    uint8_t root[4096];
    uint64_t rl = reduce_levels(nchunks, (uint32_t)g.cb, gen_chunk, &g, 0xFFFFFFFFu, 0, root, nthreads);
    final_hash(root, rl, n, out);
    return 0;
}

/* ---- a level of 32-B nodes to the root (the finisher's semantics) ----------
 * hash.go:225-237 continued from `count` nodes of a level above the chunks:
 * the same loop (odd level -> append 0^128, Hash(c[2i] || c[2i+1])) and the
 * length mix-in of the whole list's n_total items.  The device's node-input
 * passes (mk_dev_ssz_merkle_finish_nodes) compute this. */
struct node_ctx {
    const uint8_t* nodes;
};
static uint64_t node_chunk(void* c, uint64_t i, uint8_t* buf) {
    memcpy(buf, ((struct node_ctx*)c)->nodes + HASHLEN * i, HASHLEN);
    return HASHLEN;
}

int or_merkle_nodes(const uint8_t* nodes, uint64_t count, uint64_t n_total, uint8_t out[32], int nthreads) {
    if (count == 0 || !nodes) return -1;
    struct node_ctx c = {nodes};
    uint8_t root[HASHLEN];
    uint64_t rl = reduce_levels(count, HASHLEN, node_chunk, &c, 0xFFFFFFFFu, 0, root, nthreads);
    final_hash(root, rl, n_total, out);
    return 0;
}

/* Root of shard `shard` (chunks [shard<<H, (shard+1)<<H)) at height H of the
 * synthetic tree: the per-GPU subtree root of the sharded path.
 * A ragged last shard keeps applying the odd rule (hash(node || 0^128))
 * until height H whenever it is not the only shard. */
int or_merkle_subtree_gen(uint64_t n, uint32_t item_len, uint64_t seed, uint64_t shard,
                          uint32_t shard_height, uint8_t out[32], int nthreads) {
    if (item_len == 0 || n == 0) return -1;
    uint64_t cb = chunk_bytes(item_len);
    uint64_t total = n * (uint64_t)item_len;
    uint64_t nchunks = (total + cb - 1) / cb;
    uint64_t per = 1ULL << shard_height;
    uint64_t c0 = shard * per;
    if (c0 >= nchunks) return -3;
    uint64_t mine = nchunks - c0 < per ? nchunks - c0 : per;
    int only = (nchunks <= per);
    struct gen_ctx g = {seed, total, cb, c0};
    uint8_t root[4096];
    uint64_t rl = reduce_levels(mine, (uint32_t)cb, gen_chunk, &g, shard_height, !only, root, nthreads);
    if (rl != HASHLEN) return -4; /* H=0 or single chunk: not a 32-B node */
    memcpy(out, root, HASHLEN);
    return 0;
}

/* ---- deposit trie -------------------------------------------------------
 * levels_out (optional): concatenation over d = 0..depth of ceil(n/2^d)
 * 32-byte nodes (d = 0 leaves).  Nodes with no leaf below them are absent
 * (map miss -> 0^32 in the reference). */
int or_deposit_trie_build(const uint8_t* data, const uint64_t* offs, uint64_t n, uint32_t depth,
                          uint8_t* levels_out, uint8_t root[32]) {
    if (n == 0) {
        memset(root, 0, HASHLEN);
        return 0;
    }
    uint8_t* cur = (uint8_t*)malloc(n * HASHLEN);
    or_keccak256_var(data, offs, n, cur);
    uint64_t count = n;
    uint8_t* lv = levels_out;
    if (lv) {
        memcpy(lv, cur, count * HASHLEN);
        lv += count * HASHLEN;
    }
    for (uint32_t d = 0; d < depth; ++d) {
        uint64_t next = (count + 1) / 2;
        uint8_t* nxt = (uint8_t*)malloc(next * HASHLEN);
        for (uint64_t j = 0; j < next; ++j) {
            uint8_t msg[2 * HASHLEN];
            memcpy(msg, cur + 2 * j * HASHLEN, HASHLEN);
            if (2 * j + 1 < count)
                memcpy(msg + HASHLEN, cur + (2 * j + 1) * HASHLEN, HASHLEN);
            else
                memset(msg + HASHLEN, 0, HASHLEN);
            or_keccak256(msg, 2 * HASHLEN, nxt + j * HASHLEN);
        }
        free(cur);
        cur = nxt;
        count = next;
        if (lv) {
            memcpy(lv, cur, count * HASHLEN);
            lv += count * HASHLEN;
        }
    }
    memcpy(root, cur, HASHLEN);
    free(cur);
    return 0;
}

/* The reference's own incremental algorithm, one deposit at a time
 * (UpdateDepositTrie, deposit_trie.go:29-40): leaf = Hash(deposit), then all
 * `depth` ancestors recomputed from their two children, where a node not
 * written yet reads as 0^32 (Go map miss).  The map is replaced by one
 * zero-initialised array per level.  1 + depth hashes per deposit (35
 * permutations for a 280-B deposit at depth 32) -- the CPU baseline of the
 * reference's cost; or_deposit_trie_build is the batch form (same root). */
int or_deposit_trie_incremental(const uint8_t* data, const uint64_t* offs, uint64_t n, uint32_t depth,
                                uint8_t root[32]) {
    memset(root, 0, HASHLEN);
    if (n == 0) return 0;
    uint8_t** lv = (uint8_t**)calloc(depth + 1, sizeof(uint8_t*));
    uint64_t cap = n;
    for (uint32_t d = 0; d <= depth; ++d) {
        lv[d] = (uint8_t*)calloc(cap + 1, HASHLEN);  /* + 1: the right sibling slot of the last node */
        cap = (cap + 1) / 2;
    }
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t idx = i;
        or_keccak256(data + offs[i], offs[i + 1] - offs[i], lv[0] + idx * HASHLEN);
        for (uint32_t d = 0; d < depth; ++d) {
            const uint64_t p = idx / 2;
            or_keccak256(lv[d] + 2 * p * HASHLEN, 2 * HASHLEN, lv[d + 1] + p * HASHLEN);
            idx = p;
        }
    }
    memcpy(root, lv[depth], HASHLEN);
    for (uint32_t d = 0; d <= depth; ++d) free(lv[d]);
    free(lv);
    return 0;
}

/* deposit_trie.go:68-81; tree_depth = params DepositContractTreeDepth */
int or_verify_merkle_branch(const uint8_t leaf[32], const uint8_t* branch, uint32_t depth,
                            uint64_t index, uint32_t tree_depth, const uint8_t root[32]) {
    uint64_t idx = index + (tree_depth >= 64 ? 0 : (1ULL << tree_depth));
    uint8_t value[HASHLEN], msg[2 * HASHLEN];
    memcpy(value, leaf, HASHLEN);
    for (uint32_t i = 0; i < depth; ++i) {
        if (idx % 2 == 1) {
            memcpy(msg, branch + HASHLEN * i, HASHLEN);
            memcpy(msg + HASHLEN, value, HASHLEN);
        } else {
            memcpy(msg, value, HASHLEN);
            memcpy(msg + HASHLEN, branch + HASHLEN * i, HASHLEN);
        }
        or_keccak256(msg, 2 * HASHLEN, value);
        idx /= 2;
    }
    return memcmp(value, root, HASHLEN) == 0;
}

/* hashutil.MerkleRoot, merkleRoot.go:12-30: o = [nil]*n + [Hash(v)...];
 * for i = n-1 .. 0: o[i] = Hash(o[2i] || o[2i+1]); return o[1].
 * (i = 0 hashes nil || o[1]; it is computed by the reference, unused.) */
int or_merkle_root(const uint8_t* data, const uint64_t* offs, uint64_t n, uint8_t out[32]) {
    if (n == 0) return -1; /* reference: index out of range panic */
    uint8_t* o = (uint8_t*)calloc(2 * n, HASHLEN);
    for (uint64_t i = 0; i < n; ++i) or_keccak256(data + offs[i], offs[i + 1] - offs[i], o + (n + i) * HASHLEN);
    for (uint64_t i = n - 1; i >= 1; --i) or_keccak256(o + 2 * i * HASHLEN, 2 * HASHLEN, o + i * HASHLEN);
    memcpy(out, o + HASHLEN, HASHLEN);
    free(o);
    return 0;
}

/* ---- flat fixed-layout structs (ssz/hash.go:141-159) -------------------
 * kind 1: bytes field -> Keccak(le32(len) || bytes)  (hash.go:100-107,
 *         encode.go:148-159); kind 2: raw little-endian scalar (hash.go:84-98).
 * roots (n x 32) = Keccak(concat of field outputs) per record. */
int or_struct_roots(const uint8_t* rec, uint64_t n, uint32_t rec_len, const uint32_t* kind,
                    const uint32_t* off, const uint32_t* len, uint32_t nf, uint8_t* roots, int nthreads) {
    uint32_t msg_len = 0, maxb = 0;
    for (uint32_t f = 0; f < nf; ++f) {
        msg_len += kind[f] == 1 ? 32 : len[f];
        if (kind[f] == 1 && len[f] > maxb) maxb = len[f];
    }
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
    {
        uint8_t* msg = (uint8_t*)malloc(msg_len + 1);
        uint8_t* fb = (uint8_t*)malloc(maxb + 4);
#pragma omp for schedule(static)
        for (int64_t i = 0; i < (int64_t)n; ++i) {
            const uint8_t* r = rec + (uint64_t)i * rec_len;
            uint32_t o = 0;
            for (uint32_t f = 0; f < nf; ++f) {
                if (kind[f] == 1) {
                    for (int b = 0; b < 4; ++b) fb[b] = (uint8_t)(len[f] >> (8 * b));
                    memcpy(fb + 4, r + off[f], len[f]);
                    or_keccak256(fb, len[f] + 4, msg + o);
                    o += 32;
                } else {
                    memcpy(msg + o, r + off[f], len[f]);
                    o += len[f];
                }
            }
            or_keccak256(msg, msg_len, roots + 32 * (uint64_t)i);
        }
        free(msg);
        free(fb);
    }
    return 0;
}
