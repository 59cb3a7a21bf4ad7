// Shared declarations between the HIP kernels and the host planner / C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mk {

constexpr uint32_t kReduceThreads = 256;             // 4 waves
constexpr uint64_t kReduceSpan1 = 4 * kReduceThreads;  // first-level nodes per workgroup
constexpr uint64_t kReduceSpan2 = kReduceSpan1 / 2;    // level-2 nodes per workgroup (LDS)
constexpr uint32_t kMaxPassLevels = 5;               // levels per non-final pass (1024 -> 64)
constexpr uint32_t kWaveThreads = 64;                // latency pass: one wave per workgroup
constexpr uint32_t kWaveLevels = 7;                  // first level + 6 in-wave levels (64 -> 1)
constexpr uint64_t kWaveMaxC1 = 1ull << 16;          // use the latency pass at or below this width (A/B: 2^19 is slower)
constexpr uint32_t kWave2Span = kWaveThreads / 2;    // two lanes per state: 32 nodes per wave
constexpr uint32_t kWave2Levels = 6;                 // first level + 5 in-wave levels (32 -> 1)
constexpr uint32_t kMidThreads = 1024;               // largest k_wave3: 16 waves, 512 lane pairs, 10 levels

struct ReduceArgs {
    const uint8_t* items;  // LEAF: item bytes; NODE: 32-B input nodes
    uint64_t total;        // LEAF: item bytes in the tree (shard)
    uint64_t cb;           // LEAF: chunk bytes
    uint64_t nchunks;      // LEAF: chunks in the tree (shard)
    uint64_t cin;          // NODE: input node count
    uint64_t c1;           // first-level node count (windows / input pairs)
    uint64_t c1_full;      // first-level nodes eligible for the fast path
    uint8_t* out;          // output nodes (or the 32-B digest when finalize)
    uint64_t n_items;      // length mix-in value (finalize)
    uint32_t levels;       // hashing levels this pass performs
    uint32_t finalize;     // reduce to the root and mix in the length
    uint32_t pad_at_one;   // subtree mode: keep hashing (x || 0^128) at count 1
    uint64_t wg_base;      // workgroup index offset of this launch
    uint32_t in_ilv;       // k_wave3: input nodes are bit-interleaved lane pairs
    uint32_t out_ilv;      // k_wave3: write bit-interleaved output nodes
};

constexpr uint32_t kMaxStructFields = 32;
#ifndef MK_STRUCT_THREADS
#define MK_STRUCT_THREADS 256
#endif
constexpr uint32_t kStructThreads = MK_STRUCT_THREADS;  // k_struct_fused: one record per thread
constexpr uint32_t kStructFusedMaxMsg = 160;          // LDS: kStructThreads * msg_len bytes
constexpr uint32_t kStructFusedMaxField = 64;         // bytes fields held in 16 registers
struct StructSpec {                 // flat fixed-layout record (hash.go:141-159)
    uint32_t kind[kMaxStructFields];   // 1 = bytes (hashed with le32 prefix), 2 = raw scalar
    uint32_t off[kMaxStructFields];    // byte offset inside the record
    uint32_t len[kMaxStructFields];    // field length in bytes
    uint32_t out_off[kMaxStructFields];  // byte offset inside the struct message
    uint32_t nfields, rec_len, msg_len;
};

template <bool LEAF, bool FAST, int NI>
__global__ void k_reduce(ReduceArgs a);
template <bool FAST>
__global__ void k_struct_fields(const uint8_t* rec, uint64_t n, StructSpec sp, uint8_t* msg);
__global__ void k_struct_fused(const uint8_t* rec, uint64_t n, StructSpec sp, uint32_t vec16, uint4* roots);
template <bool LEAF>
__global__ void k_wave(ReduceArgs a);
template <bool LEAF>
__global__ void k_wave2(ReduceArgs a);
template <uint32_t NT, bool LEAF>
__global__ void k_wave3(ReduceArgs a);
__global__ void k_final_small(const uint8_t* items, uint64_t total, uint64_t n, uint8_t* out);
__global__ void k_finish_roots(const uint4* roots, uint64_t nroots, uint64_t n_items, uint4* out);
__global__ void k_keccak64(const uint4* in, uint64_t n, uint4* out);
__global__ void k_keccak_fixed(const uint8_t* in, uint64_t n, uint32_t msg_len, uint4* out);
__global__ void k_keccak_var(const uint8_t* in, const uint64_t* offs, uint64_t n, uint4* out);
__global__ void k_trie_level(const uint4* in, uint64_t cin, uint4* out);
__global__ void k_keccak_words(const uint2* in, uint64_t n, uint32_t nwords, uint4* out);
template <int NW>
__global__ void k_keccak_rec(const uint2* in, uint64_t n, uint4* out);
#ifndef MK_REC_THREADS
#define MK_REC_THREADS 256
#endif
constexpr uint32_t kRecThreads = MK_REC_THREADS;  // k_keccak_rec workgroup size
#ifndef MK_REC_GRID
#define MK_REC_GRID 4096
#endif
constexpr uint32_t kRecGridMax = MK_REC_GRID;  // k_keccak_rec grid cap (A/B at 2^20: 512..4096 WGs, 4096 best)
__global__ void k_trie_reduce(const uint4* in, uint64_t cin, uint4* lv_out, uint32_t levels);
__global__ void k_trie_top2(const uint32_t* in, uint64_t cin, uint32_t* lv_out, uint32_t levels);
template <uint32_t NT>
__global__ void k_trie_top3(const uint32_t* in, uint64_t cin, uint32_t* lv_out, uint32_t levels);
__global__ void k_trie_tail(uint4* node, uint32_t count, uint4* levels);
__global__ void k_verify_branches(const uint4* leaves, const uint4* branches, const uint64_t* indices,
                                  uint32_t depth, uint32_t tree_depth, const uint4* roots, uint64_t n,
                                  uint8_t* ok);
__global__ void k_synth(uint64_t* dst, uint64_t nwords, uint64_t seed, uint64_t word0);

}  // namespace mk
