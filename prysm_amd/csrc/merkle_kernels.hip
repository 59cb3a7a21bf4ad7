// HIP kernels of the MI355X Merkleization engine (gfx950 only).
//
// Hot path: ssz.merkleHash (reference shared/ssz/hash.go:194-239) over a flat
// array of n items of `item_len` bytes, plus the digest it is built on
// (hashutil.Hash, shared/hashutil/hash.go:11-25) and the deposit trie
// (shared/trieutil/deposit_trie.go:29-81).
//
// Tree shape of merkleHash, restated for a flat buffer:
//   cb      = item_len < 128 ? (128 / item_len) * item_len : item_len
//   chunk i = bytes [i*cb, min(total, (i+1)*cb))          (last may be short)
//   level 1 = "windows": node j = K(chunk 2j || chunk 2j+1), or
//             K(chunk 2j || 0^128) when 2j+1 == nchunks (odd count)
//   level l>1: node j = K(n[2j] || n[2j+1]) or K(n[2j] || 0^128) when odd;
//             a level with a single node is the root (no more hashing)
//   final   = K(root || le64(n) || 0^24)
// For item_len | 128 every window is 256 contiguous bytes of the input, so
// level 1 is a pure streaming pass (2 Keccak blocks per window).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "keccak_dev.hpp"
#include "merkle_kernels.hpp"

namespace mk {

// ----------------------------------------------------------------------------
// Generic byte-addressed sponge (edge windows, odd sizes, var-len messages).
// Message = A (global bytes [p, p+la)) || 0^lz || (lenc ? le64(nval)||0^24 : -)
__device__ __noinline__ void sponge_generic(const uint8_t* __restrict__ p, uint64_t la, uint32_t lz,
                                            bool lenc, uint64_t nval, uint4& d0, uint4& d1) {
    const uint64_t len = la + lz + (lenc ? 32u : 0u);
    const uint64_t nb = len / 136 + 1;
    const bool aligned = (((uintptr_t)p) & 7u) == 0;
    State s;
    zero(s);
    for (uint64_t b = 0; b < nb; ++b) {
        const uint64_t base = b * 136;
#pragma unroll
        for (int w = 0; w < 17; ++w) {
            const uint64_t m0 = base + 8u * w;
            uint32_t lo = 0, hi = 0;
            if (aligned && m0 + 8 <= la) {
                const uint2 v = *reinterpret_cast<const uint2*>(p + m0);
                lo = v.x;
                hi = v.y;
            } else if (m0 < len) {
#pragma unroll 1
                for (int k = 0; k < 8; ++k) {
                    const uint64_t m = m0 + k;
                    uint32_t byte = 0;
                    if (m < la) {
                        byte = p[m];
                    } else if (m >= la + lz && m < len) {
                        const uint64_t e = m - la - lz;  // lenc byte
                        byte = e < 8 ? (uint32_t)((nval >> (8 * e)) & 0xFF) : 0u;
                    }
                    if (k < 4)
                        lo |= byte << (8 * k);
                    else
                        hi |= byte << (8 * (k - 4));
                }
            }
            if (m0 <= len && len < m0 + 8) {  // domain pad byte 0x01
                const uint32_t k = (uint32_t)(len - m0);
                if (k < 4)
                    lo ^= 1u << (8 * k);
                else
                    hi ^= 1u << (8 * (k - 4));
            }
            if (b == nb - 1 && w == 16) hi ^= 0x80000000u;
            s.lo[w] ^= lo;
            s.hi[w] ^= hi;
        }
        keccak_f(s);
    }
    digest(s, d0, d1);
}

// K(L || R) (64 B, 1 permutation) or K(L || 0^128) (160 B, 2 permutations);
// `padded` may differ between lanes (the block-1 permutation then diverges).
// The final permutation computes only the digest lanes (keccak_f_digest).
__device__ __forceinline__ void hash_pair(uint4 l0, uint4 l1, uint4 r0, uint4 r1, bool padded,
                                          uint4& d0, uint4& d1) {
    State s;
    zero(s);
    xor_lane(s, 0, make_uint2(l0.x, l0.y));
    xor_lane(s, 1, make_uint2(l0.z, l0.w));
    xor_lane(s, 2, make_uint2(l1.x, l1.y));
    xor_lane(s, 3, make_uint2(l1.z, l1.w));
    if (!padded) {
        xor_lane(s, 4, make_uint2(r0.x, r0.y));
        xor_lane(s, 5, make_uint2(r0.z, r0.w));
        xor_lane(s, 6, make_uint2(r1.x, r1.y));
        xor_lane(s, 7, make_uint2(r1.z, r1.w));
    }
    if (padded) keccak_f(s);  // block 1 = L || 0^104; block 2 = 0^24 || padding
    if (padded)
        s.lo[3] ^= 1u;  // byte 160 = byte 24 of block 1
    else
        s.lo[8] ^= 1u;  // byte 64
    s.hi[16] ^= 0x80000000u;
    keccak_f_digest(s);
    digest(s, d0, d1);
}

// K(root || le64(n) || 0^24)
__device__ __forceinline__ void hash_final(uint4 r0, uint4 r1, uint64_t n, uint4& d0, uint4& d1) {
    State s;
    zero(s);
    xor_lane(s, 0, make_uint2(r0.x, r0.y));
    xor_lane(s, 1, make_uint2(r0.z, r0.w));
    xor_lane(s, 2, make_uint2(r1.x, r1.y));
    xor_lane(s, 3, make_uint2(r1.z, r1.w));
    xor_lane(s, 4, make_uint2((uint32_t)n, (uint32_t)(n >> 32)));
    s.lo[8] ^= 1u;
    s.hi[16] ^= 0x80000000u;
    keccak_f_digest(s);
    digest(s, d0, d1);
}

// ----------------------------------------------------------------------------
// Full 256-B window (two Keccak blocks) for the general leaf paths
// (first_level_generic, k_spread_leaf neighbours): the whole window is in
// registers before the first permutation, so each 128-B line is fetched once.
// The throughput leaf pass uses hash_window256_split below instead.
#define MK_MIN_WAVES 1

__device__ __forceinline__ void hash_window256(const uint4* __restrict__ w, uint4& d0, uint4& d1) {
    State s;
    zero(s);
    uint4 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = ld_stream(w + k);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        s.lo[2 * k] ^= v[k].x;
        s.hi[2 * k] ^= v[k].y;
        s.lo[2 * k + 1] ^= v[k].z;
        s.hi[2 * k + 1] ^= v[k].w;
    }
    s.lo[16] ^= v[8].x;
    s.hi[16] ^= v[8].y;
    keccak_f(s);
    s.lo[0] ^= v[8].z;
    s.hi[0] ^= v[8].w;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        s.lo[1 + 2 * k] ^= v[9 + k].x;
        s.hi[1 + 2 * k] ^= v[9 + k].y;
        s.lo[2 + 2 * k] ^= v[9 + k].z;
        s.hi[2 + 2 * k] ^= v[9 + k].w;
    }
    s.lo[15] ^= 1u;
    s.hi[16] ^= 0x80000000u;
    keccak_f_digest(s);
    digest(s, d0, d1);
}

// The throughput leaf pass's window (k_reduce<LEAF, FAST>; the only form
// since round 3).  Block 1 (bytes 0..135) is loaded straight into
// the state registers, block 2 only after the first permutation, in two
// halves, so at most 16 data VGPRs are live beside the state; the thread's
// held digests live in its own LDS level slots (k_reduce), so the kernel
// fits MK_LEAF_SPLIT_WAVES waves per SIMD with 16 KB of LDS per workgroup.
// The 128-B line shared by both blocks is fetched twice when it leaves L2 in
// between (infinity-cache hit).  Against round 2's LDS-staged form (block 2
// parked in LDS through the first permutation: 1.04x fetch, 32 KB LDS): at
// 6 waves 0.4 % faster at 2^28, 1-2 % at 2^25 (profiles/r02zg/README.md), at
// 5 waves about 1 % more (below); the staged form was removed in round 3.
// 5 waves: 94 VGPRs and no spill, 0.8-1.7 % faster than 6 waves (80 VGPRs,
// 15 dwords in scratch) and 7 waves (54 spilled) slower still
// (profiles/r02zi, r02zj).
#define MK_LEAF_SPLIT_WAVES 5
__device__ __forceinline__ void hash_window256_split(const uint4* __restrict__ w, uint4& d0, uint4& d1) {
    State s;
    uint4 v[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) v[k] = ld_stream(w + k);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        s.lo[2 * k] = v[k].x;
        s.hi[2 * k] = v[k].y;
        s.lo[2 * k + 1] = v[k].z;
        s.hi[2 * k + 1] = v[k].w;
    }
    s.lo[16] = v[8].x;
    s.hi[16] = v[8].y;
    const uint32_t t0 = v[8].z, t1 = v[8].w;
#pragma unroll
    for (int k = 17; k < 25; ++k) s.lo[k] = s.hi[k] = 0;
    keccak_f(s);
    asm volatile("" ::: "memory");  // block 2 loads stay after the permutation
    s.lo[0] ^= t0;
    s.hi[0] ^= t1;
    {
        uint4 u[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) u[k] = ld_stream(w + 9 + k);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            s.lo[1 + 2 * k] ^= u[k].x;
            s.hi[1 + 2 * k] ^= u[k].y;
            s.lo[2 + 2 * k] ^= u[k].z;
            s.hi[2 + 2 * k] ^= u[k].w;
        }
    }
    {
        uint4 u[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) u[k] = ld_stream(w + 13 + k);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            s.lo[9 + 2 * k] ^= u[k].x;
            s.hi[9 + 2 * k] ^= u[k].y;
            s.lo[10 + 2 * k] ^= u[k].z;
            s.hi[10 + 2 * k] ^= u[k].w;
        }
    }
    s.lo[15] ^= 1u;  // byte 256 = byte 120 of block 1
    s.hi[16] ^= 0x80000000u;
    keccak_f_digest(s);
    digest(s, d0, d1);
}

// K(L || R) of two 32-B nodes with phase-locked rounds (the locked kernels).
__device__ __forceinline__ void hash_node_lock(uint4 l0, uint4 l1, uint4 r0, uint4 r1, uint4& d0, uint4& d1) {
    State s;
    s.lo[0] = l0.x; s.hi[0] = l0.y; s.lo[1] = l0.z; s.hi[1] = l0.w;
    s.lo[2] = l1.x; s.hi[2] = l1.y; s.lo[3] = l1.z; s.hi[3] = l1.w;
    s.lo[4] = r0.x; s.hi[4] = r0.y; s.lo[5] = r0.z; s.hi[5] = r0.w;
    s.lo[6] = r1.x; s.hi[6] = r1.y; s.lo[7] = r1.z; s.hi[7] = r1.w;
#pragma unroll
    for (int k = 8; k < 25; ++k) s.lo[k] = s.hi[k] = 0;
    s.lo[8] = 1u;  // byte 64
    s.hi[16] = 0x80000000u;
    keccak_f_digest_lock(s);
    digest(s, d0, d1);
}

// Node-pass inputs (read once; MK_NODE_NT=1: non-temporal)
#define MK_NODE_NT 0
__device__ __forceinline__ uint4 ld_node(const uint4* p) {
    if constexpr (MK_NODE_NT) {
        const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return ld_stream(p);
    }
}

// ----------------------------------------------------------------------------
// First-level node j of a reduce pass.
//   LEAF: window j of the item buffer.
//   NODE: pair j of the 32-B input nodes (count cin).
template <bool LEAF>
__device__ __forceinline__ void first_level_generic(const ReduceArgs& a, uint64_t j, uint4& d0, uint4& d1) {
    if constexpr (LEAF) {
        if (j < a.c1_full) {  // full 256-B window (item_len | 128, 16-B aligned)
            hash_window256(reinterpret_cast<const uint4*>(a.items) + j * 16, d0, d1);
            return;
        }
        const uint64_t lo = j * 2 * a.cb;
        uint64_t la;
        uint32_t lz;
        if (2 * j + 1 < a.nchunks) {
            la = (lo + 2 * a.cb < a.total ? lo + 2 * a.cb : a.total) - lo;
            lz = 0;
        } else {
            la = a.total - lo;
            lz = 128;
        }
        sponge_generic(a.items + lo, la, lz, false, 0, d0, d1);
    } else {
        const uint4* in = reinterpret_cast<const uint4*>(a.items);
        const uint4 l0 = in[4 * j], l1 = in[4 * j + 1];
        if (a.cin == 1 && !a.pad_at_one) {  // single node: it is the root
            d0 = l0;
            d1 = l1;
            return;
        }
        const bool padded = !(2 * j + 1 < a.cin);
        uint4 r0 = make_uint4(0, 0, 0, 0), r1 = r0;
        if (!padded) {
            r0 = in[4 * j + 2];
            r1 = in[4 * j + 3];
        }
        hash_pair(l0, l1, r0, r1, padded, d0, d1);
    }
}

// Phase B of a fused pass (k_reduce, k_reduce_elem) after the workgroup's
// first two levels sit in LDS (m2 level-2 nodes, lds[2k], lds[2k+1]): the
// remaining levels in LDS, one node per thread per level (read -> barrier ->
// permute -> write -> barrier), then the workgroup's nodes (or, in the final
// pass, the root with the length mix-in) to HBM.
template <int NI>
__device__ __forceinline__ void reduce_levels_out(const ReduceArgs& a, uint4* lds, uint32_t tid, uint64_t lo1,
                                                  uint64_t c2, uint64_t m2, bool pair) {
    uint64_t c = c2, m = m2;
    int left = a.finalize ? 64 : (int)a.levels - (pair ? 2 : 1);
    int done = 0;
    while (left > 0 && (c > 1 || a.pad_at_one)) {
        const uint64_t mn = (m + 1) / 2;
        const bool act = tid < mn;
        uint4 l0, l1, r0 = make_uint4(0, 0, 0, 0), r1 = r0;
        bool padded = false;
        if (act) {
            l0 = lds[4 * tid];
            l1 = lds[4 * tid + 1];
            padded = !(2 * (uint64_t)tid + 1 < m);
            if (!padded) {
                r0 = lds[4 * tid + 2];
                r1 = lds[4 * tid + 3];
            }
        }
        __syncthreads();
        if (act) {
            uint4 d0, d1;
            hash_pair(l0, l1, r0, r1, padded, d0, d1);
            lds[2 * tid] = d0;
            lds[2 * tid + 1] = d1;
        }
        __syncthreads();
        c = (c + 1) / 2;
        m = mn;
        --left;
        ++done;
    }

    // ---- output ------------------------------------------------------------
    uint4* out = reinterpret_cast<uint4*>(a.out);
    if (a.finalize) {
        if (tid == 0) {
            uint4 d0, d1;
            hash_final(lds[0], lds[1], a.n_items, d0, d1);
            out[0] = d0;
            out[1] = d1;
        }
    } else {
        const uint64_t lo_out = (pair ? lo1 / 2 : lo1) >> done;  // the workgroup's first node of this level
        for (uint32_t k = tid; k < m; k += kReduceThreads) {
            out[2 * (lo_out + k)] = lds[2 * k];
            out[2 * (lo_out + k) + 1] = lds[2 * k + 1];
        }
    }
}

// One fused reduce pass.  256 threads; the workgroup owns first-level nodes
// [S*wg, S*wg+S) with S = 512*NI (NI = 2 for wide passes; NI = 1 halves the
// serial work per thread so mid-size trees still spread over all CUs),
// folds them pairwise in registers into S/2 level-2 nodes in LDS, then reduces further levels in LDS (one node per
// thread per level, read -> barrier -> permute -> write -> barrier).
// Non-final passes write 512 >> (levels-2) nodes per workgroup; the final
// pass (one workgroup) reduces to the root and applies the length mix-in.
template <bool LEAF, bool FAST, int NI>
__global__ __launch_bounds__(kReduceThreads, (LEAF && FAST) ? MK_LEAF_SPLIT_WAVES : MK_MIN_WAVES) void
k_reduce(ReduceArgs a) {
    constexpr uint64_t kSpan1 = 2 * NI * kReduceThreads;  // first-level nodes per workgroup
    constexpr uint64_t kSpan2 = kSpan1 / 2;
    constexpr bool kSplit = LEAF && FAST;  // the split window form (hash_window256_split)
    __shared__ uint4 lds[2 * kSpan2];
    const uint32_t tid = threadIdx.x;
    const uint64_t wg = a.wg_base + blockIdx.x;
    const uint64_t lo1 = wg * kSpan1;
    const uint64_t span1 = kSpan1;
    const uint64_t c1 = a.c1;
    const uint64_t m1 = (c1 - lo1) < span1 ? (c1 - lo1) : span1;
    const bool pair = a.levels >= 2 && (c1 > 1 || a.pad_at_one);
    const uint64_t c2 = pair ? (c1 + 1) / 2 : c1;
    const uint64_t m2 = pair ? (m1 + 1) / 2 : m1;

    // ---- phase A: first level (+ pair level) from global memory ----------
    if constexpr (kSplit) {
        // the left window's digest waits in the thread's own level slot (the
        // pair node overwrites it), so no digest is held across a window
#pragma unroll 1
        for (int i = 0; i < NI; ++i) {
            const uint32_t q = i * kReduceThreads + tid;
            const uint4* w = reinterpret_cast<const uint4*>(a.items) + (lo1 + 2 * (uint64_t)q) * 16;
            uint4 l0, l1, r0, r1, d0, d1;
            hash_window256_split(w, d0, d1);
            lds[2 * q] = d0;
            lds[2 * q + 1] = d1;
            hash_window256_split(w + 16, r0, r1);
            l0 = lds[2 * q];
            l1 = lds[2 * q + 1];
            hash_pair(l0, l1, r0, r1, false, d0, d1);
            lds[2 * q] = d0;
            lds[2 * q + 1] = d1;
        }
    } else if constexpr (FAST) {
        // Full workgroup of complete node pairs (host-checked): no bounds
        // checks, no odd padding, one keccak_f copy per call site.
#pragma unroll 1
        for (int i = 0; i < NI; ++i) {
            const uint32_t q = i * kReduceThreads + tid;
            const uint64_t j0 = lo1 + 2 * (uint64_t)q;
            uint4 l0, l1, r0, r1, d0, d1;
            const uint4* in = reinterpret_cast<const uint4*>(a.items) + j0 * 4;
            hash_pair(ld_node(in), ld_node(in + 1), ld_node(in + 2), ld_node(in + 3), false, l0, l1);
            hash_pair(ld_node(in + 4), ld_node(in + 5), ld_node(in + 6), ld_node(in + 7), false, r0, r1);
            hash_pair(l0, l1, r0, r1, false, d0, d1);
            lds[2 * q] = d0;
            lds[2 * q + 1] = d1;
        }
    } else if (pair) {
#pragma unroll 1
        for (int i = 0; i < NI; ++i) {
            const uint32_t q = i * kReduceThreads + tid;
            if (q < m2) {
                const uint64_t j0 = lo1 + 2 * (uint64_t)q;
                uint4 l0, l1, r0 = make_uint4(0, 0, 0, 0), r1 = r0, d0, d1;
                first_level_generic<LEAF>(a, j0, l0, l1);
                const bool padded = !(2 * (uint64_t)q + 1 < m1);
                if (!padded) first_level_generic<LEAF>(a, j0 + 1, r0, r1);
                hash_pair(l0, l1, r0, r1, padded, d0, d1);
                lds[2 * q] = d0;
                lds[2 * q + 1] = d1;
            }
        }
    } else {
        // no pair level (levels == 1, or a single first-level node); the host
        // guarantees m1 <= kSpan2 here.
#pragma unroll 1
        for (int i = 0; i < NI; ++i) {
            const uint32_t q = i * kReduceThreads + tid;
            if (q < m1) {
                uint4 d0, d1;
                first_level_generic<LEAF>(a, lo1 + q, d0, d1);
                lds[2 * q] = d0;
                lds[2 * q + 1] = d1;
            }
        }
    }
    __syncthreads();

    reduce_levels_out<NI>(a, lds, tid, lo1, c2, m2, pair);
}

// ----------------------------------------------------------------------------
// Phase-locked leaf pass (MK_LEAF_LOCK): 1024 threads, one workgroup per CU,
// so the 4 waves of each SIMD belong to one workgroup and the s_barrier in
// every Keccak round (round_asm<true>, keccak_dev.hpp) keeps them on the same
// instruction: the round issues at ~2.8 cycles per wave instruction instead of
// the ~3.5 of free-running waves.  Every thread hashes 4
// consecutive full windows, folds them in registers into one node three
// levels above the chunks (4 x 2 + 2 + 1 = 11 permutations, all locked) and
// writes it: workgroup g covers windows [4096 g, 4096 g + 4096) of the pass,
// i.e. the spans of k_reduce workgroups 4g..4g+3 run with a.levels == 3, and
// writes their output nodes [1024 g, 1024 g + 1024).  No divergence: every
// wave runs the same number of barriers (the host launches only full
// workgroups of full windows).  The windows are staged in LDS by COALESCED
// DMA (global_load_lds_dwordx4: no VGPRs held while a load is in flight) on a
// persistent grid.  With direct per-lane loads (round 3's k_leaf_lock, 2^28
// leaf pass 8.54 vs 8.25 ms, profiles/r03i/ab_lock4_28.jsonl; removed in
// round 4) every wave waits for its window loads, and a locked workgroup has
// no other workgroup on its CU to cover the wait;
// its per-lane 16-B loads of lanes 1 KB apart also touch 64 lines per
// instruction and every line 8 times.  Here phase A of window j (units
// 0..8 = block 1) lands in the wave's LDS (10 KB per wave) during the
// previous window's second permutation and phase B (units 9..15) during this
// window's first.  The 16-B units of a step are flattened window-major
// (phase A: U = 9 m + u; phase B: U = 7 m + u - 9), so consecutive lanes of a
// DMA instruction read consecutive units of one window (~15 lines per
// instruction, each line once), and the LDS image is that flat order: lane m
// reads its unit u at row 9 m + u (or 7 m + u - 9) -- an odd stride, so the
// 16-B reads of any 16 consecutive lanes hit distinct bank quads.
// MK_LOCK_NT=1 (default): the window's line 0 (units 0..7) and block 2
// (units 9..15, their last use) are fetched non-temporally, so they do not
// push line 1 out of L2 between block 1's unit 8 and block 2.  Phase A is
// then 9 instructions of line-0 units in a stride-9 image (the 9th position
// repeats unit 7) plus one of unit 8 into rows 576..639 (160 KB of LDS).
// One process, 2^28 (profiles/r03q): fetch 12.14 -> 8.89 GB per leaf pass
// (1.41x -> 1.03x the algorithmic 8.59 GB), leaf pass 8.138 -> 8.071 ms.
#define MK_LOCK_NT 1
// The DMA of each phase in three parts spread over a permutation instead of
// one burst (the C5 front's finding): phase B (the window's
// second block) 3 + 2 + 2 instructions before round 0 and after rounds B1,
// B2 of the first permutation; phase A (the next window's first block) 3 +
// 3 + 3 (+1) after rounds A1, A2 and MK_LOCK_DMA_ROUND of the second.  One
// process A/B (profiles/r05/leaf_dma_split/, 7-9 interleaved rounds, two
// boxes): 2^28 tree -0.6..-0.8 % (leaf pass 7.943 -> 7.885 ms at 2/8/14),
// 2^25 -2.6 %.  0: one burst each (round 4's form).
#define MK_LOCK_DMA_SPLIT 1
#define MK_LOCK_SPLIT_B1 4
#define MK_LOCK_SPLIT_B2 8
#define MK_LOCK_SPLIT_A1 2
#define MK_LOCK_SPLIT_A2 8
constexpr int kLockAux = MK_LOCK_NT ? 2 : 0;  // global_load_lds aux: nt
// the side configs' locked kernels (C2 messages, C3 records): inputs read once
#define MK_SIDE_NT 0
constexpr int kSideAux = MK_SIDE_NT ? 2 : 0;
template <int NU, int U0, int AUX = 0, int I0 = 0, int I1 = NU>
__device__ __forceinline__ void lock_dma_c(uint4* Bw, const uint4* __restrict__ Rj, uint32_t lane) {
    // launder the lane index so the per-lane offsets are recomputed here (a
    // few VALU per DMA) instead of being hoisted and held in 16+ VGPRs;
    // instructions [I0, I1) of the NU (a part of a split issue)
    asm volatile("" : "+v"(lane));
#pragma unroll
    for (int i = I0; i < I1; ++i) {
        const uint32_t U = 64u * i + lane;
        const uint32_t m = U / NU, u = U - m * NU;
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(Rj + m * 64 + U0 + u),
                                         (__attribute__((address_space(3))) void*)(Bw + 64 * i), 16, 0, AUX);
    }
}
// phase A of a window step (block 1 = units 0..8); instructions [I0, I1) of
// the 9 (+ the unit-8 copy with the last part)
template <int I0 = 0, int I1 = 9>
__device__ __forceinline__ void lock_dma_a(uint4* Bw, const uint4* __restrict__ Rj, uint32_t lane) {
    if constexpr (!MK_LOCK_NT) {
        lock_dma_c<9, 0, 0, I0, I1>(Bw, Rj, lane);
    } else {
        asm volatile("" : "+v"(lane));
#pragma unroll
        for (int i = I0; i < I1; ++i) {
            const uint32_t U = 64u * i + lane;
            const uint32_t m = U / 9, u = U - m * 9;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(Rj + m * 64 + (u < 8 ? u : 7)),
                                             (__attribute__((address_space(3))) void*)(Bw + 64 * i), 16, 0, kLockAux);
        }
        if constexpr (I1 == 9)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(Rj + lane * 64 + 8),
                                             (__attribute__((address_space(3))) void*)(Bw + 576), 16, 0, 0);
    }
}

// `after_wait` runs right after phase A's wait: the previous group's output
// store goes there, so no wait ever covers a store issued just before it
// (stores count in vmcnt; a store's wait is the write's round trip).
template <typename F>
__device__ __forceinline__ void hash_window_sc(uint4* Bw, uint32_t lane, const uint4* __restrict__ Rj,
                                               const uint4* __restrict__ Rnext, uint4& d0, uint4& d1,
                                               F&& after_wait) {
    State s;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // phase A has landed
    after_wait();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint4 v = Bw[9 * lane + k];
        s.lo[2 * k] = v.x;
        s.hi[2 * k] = v.y;
        s.lo[2 * k + 1] = v.z;
        s.hi[2 * k + 1] = v.w;
    }
    const uint4 v8 = Bw[MK_LOCK_NT ? 576 + lane : 9 * lane + 8];
    s.lo[16] = v8.x;
    s.hi[16] = v8.y;
#pragma unroll
    for (int k = 17; k < 25; ++k) s.lo[k] = s.hi[k] = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // rows read: phase B may overwrite them
    if constexpr (MK_LOCK_DMA_SPLIT) {  // phase B in three parts over the first permutation
        lock_dma_c<7, 9, kLockAux, 0, 3>(Bw, Rj, lane);
        keccak_f_lock_mid2<MK_LOCK_SPLIT_B1, MK_LOCK_SPLIT_B2>(
            s, [&] { lock_dma_c<7, 9, kLockAux, 3, 5>(Bw, Rj, lane); },
            [&] { lock_dma_c<7, 9, kLockAux, 5, 7>(Bw, Rj, lane); });
    } else {
        lock_dma_c<7, 9, kLockAux>(Bw, Rj, lane);
        keccak_f_lock(s);
    }
    s.lo[0] ^= v8.z;
    s.hi[0] ^= v8.w;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // phase B has landed
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const uint4 u = Bw[7 * lane + k];
        s.lo[1 + 2 * k] ^= u.x;
        s.hi[1 + 2 * k] ^= u.y;
        s.lo[2 + 2 * k] ^= u.z;
        s.hi[2 + 2 * k] ^= u.w;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    s.lo[15] ^= 1u;
    s.hi[16] ^= 0x80000000u;
    // the next window's block 1 goes out MK_LOCK_DMA_ROUND rounds into this
    // permutation: late enough that little of the data streamed in between
    // evicts the line block 2 shares with it, early enough to land in time
    if constexpr (MK_LOCK_DMA_SPLIT) {  // phase A of the next window in three parts
        keccak_f_digest_lock_mid3<MK_LOCK_SPLIT_A1, MK_LOCK_SPLIT_A2, MK_LOCK_DMA_ROUND>(
            s, [&] { if (Rnext) lock_dma_a<0, 3>(Bw, Rnext, lane); },
            [&] { if (Rnext) lock_dma_a<3, 6>(Bw, Rnext, lane); },
            [&] { if (Rnext) lock_dma_a<6, 9>(Bw, Rnext, lane); });
    } else {
        keccak_f_digest_lock<MK_LOCK_DMA_ROUND>(s, [&] {
            if (Rnext) lock_dma_a(Bw, Rnext, lane);
        });
    }
    digest(s, d0, d1);
}

#if MK_TOP_STAMPS
// diagnostic build only (tools/top_probe.hip): s_memrealtime at the start and
// the end of each workgroup of the leaf pass
__device__ uint64_t g_leaf_stamps[2 * 1024];
#endif
__global__ __launch_bounds__(kLockThreads, 1) void k_leaf_lock_sc(ReduceArgs a, uint64_t ngroups) {
#if MK_TOP_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_leaf_stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif
    __shared__ uint4 buf[kLockThreads / 64][(MK_LOCK_NT ? 10 : 9) * 64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint4* Bw = buf[wave];
    const uint4* items = reinterpret_cast<const uint4*>(a.items);
    uint4* out = reinterpret_cast<uint4*>(a.out);
    // the wave's 64 nodes = 256 consecutive windows (64 KB); lane m's windows at m * 64 uint4
    auto region = [&](uint64_t g) { return items + (g * kLockThreads + 64 * wave) * 64; };
    uint64_t g = blockIdx.x;
    if (g < ngroups) lock_dma_a(Bw, region(g), lane);
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;  // the previous group's node, stored one group late
    uint64_t qnode = 0;
    bool pend = false;
    auto flush = [&] {
        if (pend) {
            out[2 * qnode] = q0;
            out[2 * qnode + 1] = q1;
        }
    };
    auto none = [] {};
#pragma unroll 1
    for (; g < ngroups; g += gridDim.x) {
        const uint4* R = region(g);
        const uint64_t gn = g + gridDim.x;
        const uint4* Rn = gn < ngroups ? region(gn) : nullptr;
        uint4 l0, l1, r0, r1, p0, p1;
        hash_window_sc(Bw, lane, R, R + 16, l0, l1, flush);
        hash_window_sc(Bw, lane, R + 16, R + 32, r0, r1, none);
        hash_node_lock(l0, l1, r0, r1, p0, p1);
        hash_window_sc(Bw, lane, R + 32, R + 48, l0, l1, none);
        hash_window_sc(Bw, lane, R + 48, Rn, r0, r1, none);
        hash_node_lock(l0, l1, r0, r1, l0, l1);
        hash_node_lock(p0, p1, l0, l1, q0, q1);
        qnode = g * kLockThreads + threadIdx.x;
        pend = true;
    }
    flush();
#if MK_TOP_STAMPS
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_leaf_stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
#endif
}

template __global__ void k_reduce<true, true, 2>(ReduceArgs);
template __global__ void k_reduce<true, false, 2>(ReduceArgs);
template __global__ void k_reduce<false, true, 2>(ReduceArgs);
template __global__ void k_reduce<false, false, 2>(ReduceArgs);
template __global__ void k_reduce<true, true, 1>(ReduceArgs);
template __global__ void k_reduce<true, false, 1>(ReduceArgs);

// ----------------------------------------------------------------------------
// ssz.TreeHash of a list of byte strings in one pass (makeSliceHasher over
// []byte / [N]byte elements, hash.go:118-139 with hashedEncoding,
// hash.go:100-107): the tree's items are the element digests
// K(le32(elem_len) || element), 32 B each, 4 per chunk, so a level-1 window is
// the 8 digests of 8 consecutive elements.  k_reduce_elem computes those
// digests in registers and goes straight on into the window, the pair level
// and the LDS levels -- no n x 32-B digest array in HBM.

// K(le32(32) || e), e = 32 B at a 16-B aligned address: one block.
__device__ __forceinline__ void elem32_digest(const uint4* __restrict__ e, uint32_t (&d)[8]) {
    asm volatile("" ::: "memory");  // the loads stay here (not hoisted over earlier permutations)
    const uint4 v0 = ld_stream(e), v1 = ld_stream(e + 1);
    State s;
    s.lo[0] = 32u;  // le32(len)
    s.hi[0] = v0.x;
    s.lo[1] = v0.y;
    s.hi[1] = v0.z;
    s.lo[2] = v0.w;
    s.hi[2] = v1.x;
    s.lo[3] = v1.y;
    s.hi[3] = v1.z;
    s.lo[4] = v1.w;
    s.hi[4] = 1u;  // domain pad at byte 36
#pragma unroll
    for (int k = 5; k < 25; ++k) s.lo[k] = s.hi[k] = 0;
    s.hi[16] = 0x80000000u;
    keccak_f_digest(s);
    d[0] = s.lo[0];
    d[1] = s.hi[0];
    d[2] = s.lo[1];
    d[3] = s.hi[1];
    d[4] = s.lo[2];
    d[5] = s.hi[2];
    d[6] = s.lo[3];
    d[7] = s.hi[3];
}

__device__ __noinline__ void sponge_prefix4(const uint8_t* __restrict__ A, uint32_t L, uint4& d0, uint4& d1);

// K(le32(L) || p[0, L)) for any length and alignment (byte loads).
__device__ __noinline__ void elem_digest_any(const uint8_t* __restrict__ p, uint32_t L, uint32_t (&d)[8]) {
    uint4 d0, d1;
    if ((((uintptr_t)p) & 3u) == 0) {
        sponge_prefix4(p, L, d0, d1);
    } else {
        const uint64_t len = (uint64_t)L + 4;
        const uint64_t nb = len / 136 + 1;
        State s;
        zero(s);
        for (uint64_t b = 0; b < nb; ++b) {
#pragma unroll 1
            for (int w = 0; w < 17; ++w) {
                uint32_t h[2] = {0u, 0u};
#pragma unroll 1
                for (int k = 0; k < 8; ++k) {
                    const uint64_t m = b * 136 + 8u * w + k;
                    uint32_t byte = 0;
                    if (m < 4)
                        byte = (L >> (8 * m)) & 0xFFu;
                    else if (m < len)
                        byte = p[m - 4];
                    else if (m == len)
                        byte = 1u;  // domain pad
                    h[k >> 2] |= byte << (8 * (k & 3));
                }
                if (b == nb - 1 && w == 16) h[1] ^= 0x80000000u;
                s.lo[w] ^= h[0];
                s.hi[w] ^= h[1];
            }
            keccak_f(s);
        }
        digest(s, d0, d1);
    }
    d[0] = d0.x, d[1] = d0.y, d[2] = d0.z, d[3] = d0.w;
    d[4] = d1.x, d[5] = d1.y, d[6] = d1.z, d[7] = d1.w;
}

// Full window of 8 elements of 32 B (256 contiguous bytes, 16-B aligned).
// Two Keccak states cannot be live at once within 128 VGPRs (a permutation
// alone takes ~80), so digests 4..7 -- the last 8 bytes of block 1 and all of
// block 2 of the window message -- are parked in this thread's LDS column
// (stg[k * kReduceThreads], dword-major across the workgroup: conflict-free),
// digests 0..3 stay in registers as block 1, and the window absorbs block 2
// from LDS after its first permutation.
__device__ __forceinline__ void elem_window32(const uint4* __restrict__ w, uint32_t* stg, uint4& o0, uint4& o1) {
#pragma unroll
    for (int e = 4; e < 8; ++e) {
        uint32_t d[8];
        elem32_digest(w + 2 * e, d);
#pragma unroll
        for (int k = 0; k < 8; ++k) stg[(8 * (e - 4) + k) * kReduceThreads] = d[k];
    }
    uint32_t m[32];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        uint32_t d[8];
        elem32_digest(w + 2 * e, d);
#pragma unroll
        for (int k = 0; k < 8; ++k) m[8 * e + k] = d[k];
    }
    State s;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        s.lo[k] = m[2 * k];
        s.hi[k] = m[2 * k + 1];
    }
    s.lo[16] = stg[0];
    s.hi[16] = stg[kReduceThreads];
#pragma unroll
    for (int k = 17; k < 25; ++k) s.lo[k] = s.hi[k] = 0;
    keccak_f(s);
#pragma unroll
    for (int q = 0; q < 30; ++q) {  // block 2 = staged dwords 2..31
        const uint32_t v = stg[(2 + q) * kReduceThreads];
        if (q & 1)
            s.hi[q >> 1] ^= v;
        else
            s.lo[q >> 1] ^= v;
    }
    s.lo[15] ^= 1u;  // byte 256 = byte 120 of block 2
    s.hi[16] ^= 0x80000000u;
    keccak_f_digest(s);
    digest(s, o0, o1);
}

// Window j of the digest tree in general form: digests [8j, min(8j+8, n)),
// odd chunk count -> the 128-B zero chunk appended (hash.go:225-228).
__device__ __noinline__ void elem_window_generic(const ReduceArgs& a, uint64_t j, uint4& o0, uint4& o1) {
    const uint64_t n = a.n_items;
    const uint32_t cnt = (uint32_t)((n - 8 * j) < 8 ? (n - 8 * j) : 8);
    const bool padded = !(2 * j + 1 < a.nchunks);
    const uint32_t L = a.elem_len;
    uint32_t m[64];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if ((uint32_t)e < cnt) elem_digest_any(a.items + (8 * j + e) * (uint64_t)L, L, d);
#pragma unroll
        for (int k = 0; k < 8; ++k) m[8 * e + k] = d[k];
    }
    const uint32_t lm = 32 * cnt + (padded ? 128u : 0u);  // message bytes (<= 256, a multiple of 4)
    const uint32_t nb = lm / 136 + 1;
    State s;
    zero(s);
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        if ((uint32_t)b >= nb) break;
#pragma unroll
        for (int w = 0; w < 34; ++w) {
            const int q = 34 * b + w;
            uint32_t v = q < 64 ? m[q] : 0u;
            if ((uint32_t)q * 4 == lm) v ^= 1u;
            if ((uint32_t)b == nb - 1 && w == 33) v ^= 0x80000000u;
            if (w & 1)
                s.hi[w >> 1] ^= v;
            else
                s.lo[w >> 1] ^= v;
        }
        if ((uint32_t)b + 1 < nb)
            keccak_f(s);
        else
            keccak_f_digest(s);
    }
    digest(s, o0, o1);
}

#define MK_ELEM_WAVES 4
// The leaf pass of the element-digest tree (a.n_items elements, a.nchunks =
// ceil(n / 4) chunks, a.c1 windows), one window pair per thread (NI = 1:
// 512 windows = 4096 elements per workgroup; LDS 8 KB of levels + 32 KB of
// staged digests, so 4 workgroups of 4 waves fill a CU's 160 KB at 4
// waves/SIMD).  FAST: every window of the workgroup has 8 elements of 32 B,
// 16-B aligned (host-checked).  Otherwise the general window (any elem_len
// and alignment, ragged last window, odd pad).
template <bool FAST>
__global__ __launch_bounds__(kReduceThreads, FAST ? MK_ELEM_WAVES : 1) void k_reduce_elem(ReduceArgs a) {
    constexpr int NI = 1;
    constexpr uint64_t kSpan1 = 2 * NI * kReduceThreads;
    constexpr uint64_t kSpan2 = kSpan1 / 2;
    __shared__ uint4 lds[2 * kSpan2];
    __shared__ uint32_t stg[FAST ? 32 * kReduceThreads : 1];
    const uint32_t tid = threadIdx.x;
    const uint64_t wg = a.wg_base + blockIdx.x;
    const uint64_t lo1 = wg * kSpan1;
    const uint64_t c1 = a.c1;
    const uint64_t m1 = (c1 - lo1) < kSpan1 ? (c1 - lo1) : kSpan1;
    const bool pair = a.levels >= 2 && c1 > 1;  // the host plans k_reduce_elem for trees of > 2^17 windows
    const uint64_t c2 = pair ? (c1 + 1) / 2 : c1;
    const uint64_t m2 = pair ? (m1 + 1) / 2 : m1;
    const uint32_t q = tid;
    if (FAST || q < m2) {
        const uint64_t j0 = lo1 + 2 * (uint64_t)q;
        uint4 l0, l1, r0 = make_uint4(0, 0, 0, 0), r1 = r0, d0, d1;
        bool padded = false;
        if constexpr (FAST) {
            const uint4* w = reinterpret_cast<const uint4*>(a.items) + j0 * 16;
            elem_window32(w, stg + tid, d0, d1);
            lds[2 * q] = d0;  // the left digest waits in this thread's own level slot
            lds[2 * q + 1] = d1;
            elem_window32(w + 16, stg + tid, r0, r1);
            l0 = lds[2 * q];
            l1 = lds[2 * q + 1];
        } else {
            elem_window_generic(a, j0, l0, l1);
            padded = !(2 * (uint64_t)q + 1 < m1);
            if (!padded) elem_window_generic(a, j0 + 1, r0, r1);
        }
        hash_pair(l0, l1, r0, r1, padded, d0, d1);
        lds[2 * q] = d0;
        lds[2 * q + 1] = d1;
    }
    __syncthreads();
    reduce_levels_out<NI>(a, lds, tid, lo1, c2, m2, pair);
}

template __global__ void k_reduce_elem<true>(ReduceArgs);

// Phase-locked element windows (MK_ELEM_LOCK; C4 secondary, TreeHash of
// [][32]byte): lane m of wave w hashes window g * 1024 + 64 w + m of group g
// -- its 8 element digests K(le32(32) || e) (1 permutation each) and the
// window K(d0 || .. || d7) (2) -- with phase-locked permutations and writes
// the window digest (a level-1 node of the tree; the host finishes the tree
// from those nodes).  n windows in all; a partial last group's lanes past n
// hash copies of window n - 1 and store nothing.  The window's two halves
// (elements 0..3, 4..7: 128 B = 8 units each) are staged in the wave's 9 KB
// of LDS by coalesced non-temporal DMA in a stride-9 image (the 9th
// position repeats unit 7); digests 0..3 wait in VGPRs, digests 4..7 replace
// their elements in LDS, and the next window's first half goes out once
// block 2 of this window's message has been read.
__device__ __forceinline__ void elem_dma_half(uint4* Bw, const uint4* __restrict__ W0, uint64_t m0, uint64_t nwin,
                                              int half, uint32_t lane) {
    asm volatile("" : "+v"(lane));
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const uint32_t U = 64u * i + lane;
        const uint32_t m = U / 9, u = U - m * 9;
        const uint64_t win = m0 + m < nwin ? m0 + m : nwin - 1;
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(W0 + win * 16 + 8 * half + (u < 8 ? u : 7)),
                                         (__attribute__((address_space(3))) void*)(Bw + 64 * i), 16, 0, kLockAux);
    }
}
__device__ __forceinline__ void elem_digest_lock(uint4 a, uint4 b, uint32_t (&d)[8]) {
    State s;
    s.lo[0] = 32u;  // le32(len)
    s.hi[0] = a.x;
    s.lo[1] = a.y;
    s.hi[1] = a.z;
    s.lo[2] = a.w;
    s.hi[2] = b.x;
    s.lo[3] = b.y;
    s.hi[3] = b.z;
    s.lo[4] = b.w;
    s.hi[4] = 1u;  // domain pad at byte 36
#pragma unroll
    for (int k = 5; k < 25; ++k) s.lo[k] = s.hi[k] = 0;
    s.hi[16] = 0x80000000u;
    keccak_f_digest_lock(s);
    d[0] = s.lo[0]; d[1] = s.hi[0]; d[2] = s.lo[1]; d[3] = s.hi[1];
    d[4] = s.lo[2]; d[5] = s.hi[2]; d[6] = s.lo[3]; d[7] = s.hi[3];
}
__global__ __launch_bounds__(kLockThreads, 1) void k_elem_lock(const uint4* __restrict__ elems, uint64_t nwin,
                                                               uint4* __restrict__ out) {
    __shared__ uint4 buf[kLockThreads / 64][9 * 64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint4* Bw = buf[wave];
    const uint4* Rl = Bw + 9 * lane;  // this lane's 8 staged units (+1 repeat)
    const uint64_t ngroups = (nwin + kLockThreads - 1) / kLockThreads;
    uint64_t g = blockIdx.x;
    if (g < ngroups) elem_dma_half(Bw, elems, g * kLockThreads + 64 * wave, nwin, 0, lane);
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
    uint64_t qi = 0;
    bool pend = false;
#pragma unroll 1
    for (; g < ngroups; g += gridDim.x) {
        const uint64_t m0 = g * kLockThreads + 64 * wave;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // first half landed
        if (pend && qi < nwin) {
            out[2 * qi] = q0;
            out[2 * qi + 1] = q1;
        }
        uint32_t dlo[4][8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 a = Rl[2 * k], b = Rl[2 * k + 1];
            if (k == 3) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // first half read: the second may land
                elem_dma_half(Bw, elems, m0, nwin, 1, lane);
            }
            elem_digest_lock(a, b, dlo[k]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // second half landed
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 a = Rl[2 * k], b = Rl[2 * k + 1];
            uint32_t d[8];
            elem_digest_lock(a, b, d);
            // digest 4 + k replaces element 4 + k (same 32 B, already absorbed)
            uint4* R = Bw + 9 * lane;
            R[2 * k] = make_uint4(d[0], d[1], d[2], d[3]);
            R[2 * k + 1] = make_uint4(d[4], d[5], d[6], d[7]);
        }
        // the window message d0..d7 (256 B): block 1 = d0..d3 + the first 8 B of d4
        State s;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                s.lo[4 * k + w] = dlo[k][2 * w];
                s.hi[4 * k + w] = dlo[k][2 * w + 1];
            }
        const uint4 t4a = Rl[0];
        s.lo[16] = t4a.x;
        s.hi[16] = t4a.y;
#pragma unroll
        for (int k = 17; k < 25; ++k) s.lo[k] = s.hi[k] = 0;
        keccak_f_lock(s);
        // block 2 = d4[8..32) + d5 + d6 + d7 + padding at byte 256 = byte 120
        s.lo[0] ^= t4a.z;
        s.hi[0] ^= t4a.w;
        {
            const uint4 t = Rl[1];
            s.lo[1] ^= t.x; s.hi[1] ^= t.y; s.lo[2] ^= t.z; s.hi[2] ^= t.w;
        }
#pragma unroll
        for (int k = 1; k < 4; ++k) {
            const uint4 a = Rl[2 * k], b = Rl[2 * k + 1];
            s.lo[4 * k - 1] ^= a.x; s.hi[4 * k - 1] ^= a.y; s.lo[4 * k] ^= a.z; s.hi[4 * k] ^= a.w;
            s.lo[4 * k + 1] ^= b.x; s.hi[4 * k + 1] ^= b.y; s.lo[4 * k + 2] ^= b.z; s.hi[4 * k + 2] ^= b.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // digests read: the next window's first half may land
        if (g + gridDim.x < ngroups)
            elem_dma_half(Bw, elems, (g + gridDim.x) * kLockThreads + 64 * wave, nwin, 0, lane);
        s.lo[15] ^= 1u;  // byte 256 = byte 120 of block 2
        s.hi[16] ^= 0x80000000u;
        keccak_f_digest_lock(s);
        digest(s, q0, q1);
        qi = g * kLockThreads + threadIdx.x;
        pend = true;
    }
    if (pend && qi < nwin) {
        out[2 * qi] = q0;
        out[2 * qi + 1] = q1;
    }
}


template __global__ void k_reduce_elem<false>(ReduceArgs);

// Element digests K(le32(elem_len) || element i) -> out[i] (32 B): the first
// half of the two-phase form, for trees too small for k_reduce_elem's
// throughput pass and for element lengths other than 32.
// FAST32: 32-B elements at a 16-B aligned base (one block, 16-B loads);
// otherwise any length and alignment (the general sponge, its own kernel so
// the fast form keeps its few VGPRs).
template <bool FAST32>
__global__ __launch_bounds__(256) void k_elem_digests(const uint8_t* __restrict__ elems, uint64_t n, uint32_t elem_len,
                                                      uint4* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t d[8];
    if constexpr (FAST32)
        elem32_digest(reinterpret_cast<const uint4*>(elems) + 2 * i, d);
    else
        elem_digest_any(elems + i * (uint64_t)elem_len, elem_len, d);
    out[2 * i] = make_uint4(d[0], d[1], d[2], d[3]);
    out[2 * i + 1] = make_uint4(d[4], d[5], d[6], d[7]);
}
template __global__ void k_elem_digests<true>(const uint8_t*, uint64_t, uint32_t, uint4*);
template __global__ void k_elem_digests<false>(const uint8_t*, uint64_t, uint32_t, uint4*);


// ----------------------------------------------------------------------------
// Node pass of the latency form with BIT-INTERLEAVED lane pairs
// (keccak_dev.hpp, mk::ilv): lane p of pair k owns the parity-p words of node
// k.  Nodes in LDS and, between consecutive wave3 passes, in HBM stay in
// that form ("ilv nodes": dword 2w + p = parity-p word of digest lane w);
// a.in_ilv / a.out_ilv select conversion from / to plain 32-B digests at the
// pass boundary, so a chain of passes converts once at each end.
// NT = 64..1024 threads own NT/2 lane pairs and reduce them through
// log2(NT/2) more levels in LDS.  The host picks NT so the first level's
// workgroups spread over all 256 CUs (NT = 1024 for 2^17 pairs): the first,
// throughput-bound level fills the chip, and each later level halves the
// number of waves that still issue (waves with no active lane skip the
// permutation and wait at the barrier), so one launch covers up to 10 levels
// at close to one permutation latency each.
namespace {

__device__ __forceinline__ void hash_pair3(const uint32_t (&l)[4], const uint32_t (&r)[4], bool padded, uint32_t p,
                                           uint32_t (&d)[4]) {
    ilv::Half s;
    ilv::zero(s);
#pragma unroll
    for (int w = 0; w < 4; ++w) s.v[w] = l[w];
    if (!padded) {
#pragma unroll
        for (int w = 0; w < 4; ++w) s.v[4 + w] = r[w];
    }
    const int nperm = padded ? 2 : 1;
#pragma unroll 1
    for (int k = 0; k < nperm; ++k) {
        if (k == nperm - 1) {  // bit 0 of a lane is even (p = 0), bit 63 odd (p = 1)
            if (p == 1)
                s.v[16] ^= 0x80000000u;
            else if (padded)  // (two static indices: a runtime one sent the state to scratch)
                s.v[3] ^= 1u;
            else
                s.v[8] ^= 1u;
        }
        ilv::keccak_f(s, p);
    }
#pragma unroll
    for (int w = 0; w < 4; ++w) d[w] = s.v[w];
}

// full 256-B window (two blocks) on this lane's parity words; each 64-bit
// message lane is split into its even / odd bits on the way in
__device__ __forceinline__ void hash_window3(const uint4* __restrict__ w, uint32_t p, uint32_t (&d)[4]) {
    uint4 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = ld_stream(w + k);
    uint32_t m[32];  // message lanes 0..31 as parity-p words
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        m[2 * k] = ilv::to_ilv(v[k].x, v[k].y, p);
        m[2 * k + 1] = ilv::to_ilv(v[k].z, v[k].w, p);
    }
    ilv::Half s;
    ilv::zero(s);
#pragma unroll 1
    for (int b = 0; b < 2; ++b) {
        if (b == 0) {
#pragma unroll
            for (int i = 0; i < 17; ++i) s.v[i] ^= m[i];
        } else {
#pragma unroll
            for (int i = 0; i < 15; ++i) s.v[i] ^= m[17 + i];
            if (p == 0)
                s.v[15] ^= 1u;  // byte 256 = byte 120 of block 1: bit 0 of lane 15
            else
                s.v[16] ^= 0x80000000u;
        }
        ilv::keccak_f(s, p);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = s.v[k];
}

// node j of a plain or ilv node array -> this lane's parity words
__device__ __forceinline__ void load_node3(const uint32_t* __restrict__ in, uint64_t j, bool is_ilv, uint32_t p,
                                           uint32_t (&w4)[4]) {
    if (is_ilv) {
#pragma unroll
        for (int w = 0; w < 4; ++w) w4[w] = in[8 * j + 2 * w + p];
    } else {
        const uint4 a = reinterpret_cast<const uint4*>(in)[2 * j];
        const uint4 b = reinterpret_cast<const uint4*>(in)[2 * j + 1];
        w4[0] = ilv::to_ilv(a.x, a.y, p);
        w4[1] = ilv::to_ilv(a.z, a.w, p);
        w4[2] = ilv::to_ilv(b.x, b.y, p);
        w4[3] = ilv::to_ilv(b.z, b.w, p);
    }
}

// this lane's dwords (2w + p) of a node, plain or ilv
__device__ __forceinline__ void store_node3(uint32_t* __restrict__ out, uint64_t j, bool is_ilv, uint32_t p,
                                            const uint32_t (&w4)[4]) {
#pragma unroll
    for (int w = 0; w < 4; ++w) out[8 * j + 2 * w + p] = is_ilv ? w4[w] : ilv::from_ilv(w4[w], p);
}

}  // namespace

// Levels of k_wave3 once a level has at most one parent per wave: ONE
// STATE PER WAVE (mk::spread, ilv words, ~6.4 k cycles per lone-wave
// permutation against ~12.8 k for a lane pair).  Wave w hashes parent w; the
// nodes stay in k_wave3's LDS layout (lds[8 node + 2 word + parity]).  GPU
// lane L holds Keccak lane i = lane_consts(L).i: i < 4 the left node's word
// i, 4..7 the right node's, 8 / 16 (3 / 16 in the second block of a padded
// node) the padding bits.
template <uint32_t NT>
__device__ __forceinline__ void wave3_spread_levels(uint32_t* lds, uint64_t& c, uint64_t& m, int& left, int& done,
                                                    uint32_t pad_at_one) {
    const uint32_t w = threadIdx.x >> 6, L = threadIdx.x & 63u;
    const spread::Lane cst = spread::lane_consts(L);
    const uint32_t i = cst.i;
    while (left > 0 && (c > 1 || pad_at_one)) {
        const uint64_t mn = (m + 1) / 2;
        uint32_t e = 0u, o = 0u;
        if (w < mn) {  // wave-uniform
            const bool padded = !(2 * (uint64_t)w + 1 < m);
            if (i < 4u) {
                e = lds[16 * w + 2 * i];
                o = lds[16 * w + 2 * i + 1];
            } else if (i < 8u && !padded) {
                e = lds[16 * w + 8 + 2 * (i - 4u)];
                o = lds[16 * w + 8 + 2 * (i - 4u) + 1];
            }
            if (padded) {  // K(l || 0^128): 160 bytes, two blocks
                spread::keccak_f(e, o, cst);
                if (i == 3u) e ^= 1u;
            } else if (i == 8u) {
                e ^= 1u;
            }
            if (i == 16u) o ^= 0x80000000u;
            spread::keccak_f(e, o, cst);
        }
        __syncthreads();
        if (w < mn && L < 4u) {
            lds[8 * w + 2 * L] = e;
            lds[8 * w + 2 * L + 1] = o;
        }
        __syncthreads();
        c = (c + 1) / 2;
        m = mn;
        --left;
        ++done;
    }
}

// K(root || le64(n) || 0^24) by wave 0 in spread form; plain digest to out.
// With `pair` (a two-field struct root, hash.go:141-159: the State{registry,
// balances} of BASELINE config 3): out is this field's slot of the pair
// block, and the second of the two finishers to arrive -- they run as
// separate launches on two streams, neither waits for the other -- hashes
// K(slot 0 || slot 1) into pair[64..96).  Arrival word pair[24] = epoch << 2 |
// arrived-slot bits (epochs are 30-bit and wrap; "newer" = ahead by less than
// 2^29): a finisher of a newer epoch than the word's starts the mask afresh,
// so a pair left half-done (a failed launch) cannot pair with the next one; a
// finisher of an OLDER epoch (a late one) is ignored -- it writes neither its
// slot nor the arrival word -- so it cannot clear the current pair's bits.
// Best-effort: the epoch is read before the slot store, so a finisher that
// falls behind while it runs may still overwrite its slot; callers never run
// two epochs' finishers of one slot concurrently (include/prysm_merkle.h).  The first finisher of an epoch zeroes pair[64..96)
// before it sets its bit, so a pair that never completes reads back as
// zeros, never as the previous epoch's root.
// How far `epoch` is ahead of an arrival word's epoch (mod 2^30; >= 2^29:
// behind).  A word whose epoch is 0 was never used (valid epochs are >= 1):
// every epoch is ahead of it.
__device__ __forceinline__ uint32_t epoch_ahead(uint32_t epoch, uint32_t word) {
    return (word >> 2) == 0u ? 1u : (epoch - (word >> 2)) & 0x3FFFFFFFu;
}
__device__ __forceinline__ void spread_store_digest(uint32_t e, uint32_t o, uint32_t L, uint32_t* out) {
    if (L < 4u) {
        out[2 * L] = ilv::spread16(e) | (ilv::spread16(o) << 1);
        out[2 * L + 1] = ilv::spread16(e >> 16) | (ilv::spread16(o >> 16) << 1);
    }
}
__device__ __forceinline__ void wave3_spread_final(const uint32_t* lds, uint64_t n_items, uint32_t* out,
                                                   uint32_t* pair = nullptr, uint32_t slot = 0, uint32_t epoch = 0) {
    const uint32_t L = threadIdx.x & 63u;
    const spread::Lane cst = spread::lane_consts(L);
    const uint32_t i = cst.i;
    uint32_t e = 0u, o = 0u;
    if (i < 4u) {
        e = lds[2 * i];
        o = lds[2 * i + 1];
    } else if (i == 4u) {
        e = ilv::to_ilv((uint32_t)n_items, (uint32_t)(n_items >> 32), 0);
        o = ilv::to_ilv((uint32_t)n_items, (uint32_t)(n_items >> 32), 1);
    } else if (i == 8u) {
        e = 1u;
    }
    if (i == 16u) o ^= 0x80000000u;
    spread::keccak_f(e, o, cst);
    if (pair) {  // a late finisher of an older epoch than the word's leaves the block alone
        uint32_t stale = 0;
        if (L == 0) stale = epoch_ahead(epoch, atomicAdd(pair + 24, 0u)) >= (1u << 29);
        if (__shfl(stale, 0)) return;
    }
    spread_store_digest(e, o, L, out);
    if (!pair) return;
    __threadfence();  // this field's root is visible before its arrival bit
    uint32_t second = 0;
    if (L == 0) {
        uint32_t* word = pair + 24;
        uint32_t old = atomicAdd(word, 0u);  // an atomic read of the arrival word
        for (;;) {
            const uint32_t ahead = epoch_ahead(epoch, old);
            if (ahead >= (1u << 29)) break;  // an older epoch than the word's: a late finisher, ignored
            if (ahead != 0u || (old & 3u) == 0u) {  // first of this epoch (so far): clear the pair root
                for (uint32_t w = 16; w < 24; ++w) pair[w] = 0u;
                __threadfence();
            }
            const uint32_t nw = (ahead == 0u ? old : epoch << 2) | (1u << slot);
            const uint32_t seen = atomicCAS(word, old, nw);
            if (seen == old) {
                second = (nw & 3u) == 3u;
                break;
            }
            old = seen;
        }
    }
    if (!__shfl(second, 0)) return;  // the other field's finisher is still running: it completes the pair
    __threadfence();
    const volatile uint32_t* both = pair;
    uint32_t e2 = 0u, o2 = 0u;
    if (i < 8u) {  // lanes 0..3: field 0's root, 4..7: field 1's
        const uint32_t lo = both[2 * i], hi = both[2 * i + 1];
        e2 = ilv::to_ilv(lo, hi, 0);
        o2 = ilv::to_ilv(lo, hi, 1);
    } else if (i == 8u) {
        e2 = 1u;  // byte 64
    }
    if (i == 16u) o2 ^= 0x80000000u;
    spread::keccak_f(e2, o2, cst);
    spread_store_digest(e2, o2, L, pair + 16);
}

template <uint32_t NT, bool LEAF>
__global__ __launch_bounds__(NT) void k_wave3(ReduceArgs a) {
    constexpr uint32_t kSpan = NT / 2;  // first-level nodes (lane pairs) per workgroup
    __shared__ uint32_t lds[8 * kSpan];
    const uint32_t tid = threadIdx.x;
    const uint32_t k = tid >> 1;
    const uint32_t p = tid & 1u;
    const uint64_t wg = a.wg_base + blockIdx.x;
    const uint64_t lo1 = wg * kSpan;
    const uint64_t c1 = a.c1;
    const uint64_t m1 = (c1 - lo1) < kSpan ? (c1 - lo1) : kSpan;
    const uint32_t* in = reinterpret_cast<const uint32_t*>(a.items);
    if (LEAF && k < m1) {  // window j of the item bytes
        const uint64_t j = lo1 + k;
        uint32_t d[4];
        if (j < a.c1_full) {
            hash_window3(reinterpret_cast<const uint4*>(a.items) + j * 16, p, d);
        } else {  // ragged window: both lanes run the full-state sponge
            uint4 d0, d1;
            first_level_generic<true>(a, j, d0, d1);
            d[0] = ilv::to_ilv(d0.x, d0.y, p);
            d[1] = ilv::to_ilv(d0.z, d0.w, p);
            d[2] = ilv::to_ilv(d1.x, d1.y, p);
            d[3] = ilv::to_ilv(d1.z, d1.w, p);
        }
#pragma unroll
        for (int w = 0; w < 4; ++w) lds[8 * k + 2 * w + p] = d[w];
    } else if (!LEAF && k < m1) {
        const uint64_t j = lo1 + k;
        uint32_t l[4], r[4] = {0, 0, 0, 0}, d[4];
        load_node3(in, 2 * j, a.in_ilv, p, l);
        if (a.cin == 1 && !a.pad_at_one) {  // single node: it is the root
#pragma unroll
            for (int w = 0; w < 4; ++w) d[w] = l[w];
        } else {
            const bool padded = !(2 * j + 1 < a.cin);
            if (!padded) load_node3(in, 2 * j + 1, a.in_ilv, p, r);
            hash_pair3(l, r, padded, p, d);
        }
#pragma unroll
        for (int w = 0; w < 4; ++w) lds[8 * k + 2 * w + p] = d[w];
    }
    __syncthreads();
    uint64_t c = c1, m = m1;
    int left = a.finalize ? 64 : (int)a.levels - 1;
    int done = 0;
    while (left > 0 && (c > 1 || a.pad_at_one)) {
        const uint64_t mn = (m + 1) / 2;
        if (MK_WAVE3_SPREAD && mn <= NT / 64) break;  // one parent per wave from here
        const bool act = k < mn;
        uint32_t l[4], r[4] = {0, 0, 0, 0};
        bool padded = false;
        if (act) {
            padded = !(2 * (uint64_t)k + 1 < m);
#pragma unroll
            for (int w = 0; w < 4; ++w) l[w] = lds[16 * k + 2 * w + p];
            if (!padded) {
#pragma unroll
                for (int w = 0; w < 4; ++w) r[w] = lds[16 * k + 8 + 2 * w + p];
            }
        }
        __syncthreads();
        if (act) {
            uint32_t d[4];
            hash_pair3(l, r, padded, p, d);
#pragma unroll
            for (int w = 0; w < 4; ++w) lds[8 * k + 2 * w + p] = d[w];
        }
        __syncthreads();
        c = (c + 1) / 2;
        m = mn;
        --left;
        ++done;
    }
    if (MK_WAVE3_SPREAD) wave3_spread_levels<NT>(lds, c, m, left, done, a.pad_at_one);
    uint32_t* out = reinterpret_cast<uint32_t*>(a.out);
    if (MK_WAVE3_SPREAD && a.finalize) {
        if (tid < 64)
            wave3_spread_final(lds, a.n_items, out, reinterpret_cast<uint32_t*>(a.pair_block), a.pair_slot,
                               a.pair_epoch);
    } else if (a.finalize) {
        if (k == 0) {  // K(root || le64(n) || 0^24) on lanes 0/1
            ilv::Half s;
            ilv::zero(s);
#pragma unroll
            for (int w = 0; w < 4; ++w) s.v[w] = lds[2 * w + p];
            s.v[4] = ilv::to_ilv((uint32_t)a.n_items, (uint32_t)(a.n_items >> 32), p);
            if (p == 0)
                s.v[8] ^= 1u;
            else
                s.v[16] ^= 0x80000000u;
            ilv::keccak_f(s, p);
            uint32_t d[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) d[w] = s.v[w];
            store_node3(out, 0, false, p, d);
        }
    } else if (k < m) {
        const uint64_t lo_out = lo1 >> done;
        uint32_t d[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) d[w] = lds[8 * k + 2 * w + p];
        store_node3(out, lo_out + k, a.out_ilv, p, d);
    }
}

template __global__ void k_wave3<64, false>(ReduceArgs);
template __global__ void k_wave3<128, false>(ReduceArgs);
template __global__ void k_wave3<256, false>(ReduceArgs);
template __global__ void k_wave3<512, false>(ReduceArgs);
template __global__ void k_wave3<1024, false>(ReduceArgs);
template __global__ void k_wave3<64, true>(ReduceArgs);
template __global__ void k_wave3<128, true>(ReduceArgs);
template __global__ void k_wave3<256, true>(ReduceArgs);
template __global__ void k_wave3<512, true>(ReduceArgs);
template __global__ void k_wave3<1024, true>(ReduceArgs);

// Wave priority of the trie's latency-bound top kernels (s_setprio): they run
// beside a phase-locked front at one wave per SIMD (the pipelined C5 stream),
// where the locked waves otherwise take most of the issue slots and the top's
// dependent chain, not the front, sets the step.  One
// process A/B (profiles/r05/c5_front_ab/ab_knobs.txt): the pipelined stream
// 0.4386 -> 0.4231 ms/step at priority 1 (0.4239 at 3); 0 = the default
// wave priority.
#define MK_TRIE_TOP_PRIO 1
// Narrow top of the deposit trie, bit-interleaved lane pairs (mk::ilv): the
// workgroup owns NT input nodes of level d (NT/2 lane pairs) and writes
// `levels` levels to the (plain) level array; once the count is 1 it goes on
// with node = K(node || 0^32), the zero-sibling levels of
// deposit_trie.go:33-38.  The host picks NT so a launch has <= ~256
// workgroups; the last launch (one workgroup) runs to the top of the trie.
template <uint32_t NT>
__global__ __launch_bounds__(NT) void k_trie_top3(const uint32_t* __restrict__ in, uint64_t cin,
                                                  uint32_t* __restrict__ lv_out, uint32_t levels, uint64_t capn) {
    if constexpr (MK_TRIE_TOP_PRIO > 0) __builtin_amdgcn_s_setprio(MK_TRIE_TOP_PRIO);
    constexpr uint32_t kPairs = NT / 2;
    __shared__ uint32_t lds[8 * kPairs];
    const uint32_t tid = threadIdx.x, k = tid >> 1, p = tid & 1u;
    uint64_t c = cin;
    uint64_t lo = (uint64_t)blockIdx.x * NT;  // first input node of this workgroup
    uint64_t m = (c - lo) < NT ? (c - lo) : NT;
    uint32_t* dst = lv_out;
    for (uint32_t l = 0; l < levels; ++l) {
        const uint64_t cn = (c + 1) / 2, mn = (m + 1) / 2;
        const bool act = k < mn;
        uint32_t a[4], b[4] = {0, 0, 0, 0};
        if (act) {
            const bool right = 2 * (uint64_t)k + 1 < m;
            if (l == 0) {
                load_node3(in, lo + 2 * (uint64_t)k, false, p, a);
                if (right) load_node3(in, lo + 2 * (uint64_t)k + 1, false, p, b);
            } else {
#pragma unroll
                for (int w = 0; w < 4; ++w) a[w] = lds[16 * k + 2 * w + p];
                if (right) {
#pragma unroll
                    for (int w = 0; w < 4; ++w) b[w] = lds[16 * k + 8 + 2 * w + p];
                }
            }
        }
        __syncthreads();
        if (act) {
            uint32_t d[4];
            hash_pair3(a, b, false, p, d);
#pragma unroll
            for (int w = 0; w < 4; ++w) lds[8 * k + 2 * w + p] = d[w];
            store_node3(dst, lo / 2 + k, false, p, d);
        }
        __syncthreads();
        dst += 8 * capn;  // next level's slot of the level array (capacity layout)
        capn = (capn + 1) / 2;
        c = cn;
        m = mn;
        lo /= 2;
    }
}

template __global__ void k_trie_top3<64>(const uint32_t*, uint64_t, uint32_t*, uint32_t, uint64_t);
template __global__ void k_trie_top3<128>(const uint32_t*, uint64_t, uint32_t*, uint32_t, uint64_t);
template __global__ void k_trie_top3<256>(const uint32_t*, uint64_t, uint32_t*, uint32_t, uint64_t);
template __global__ void k_trie_top3<512>(const uint32_t*, uint64_t, uint32_t*, uint32_t, uint64_t);
template __global__ void k_trie_top3<1024>(const uint32_t*, uint64_t, uint32_t*, uint32_t, uint64_t);

// ----------------------------------------------------------------------------
// Final hash for trees with <= 1 chunk: K(bytes[0,total) || [0^128 if n==0] || lenc)
__global__ void k_final_small(const uint8_t* __restrict__ items, uint64_t total, uint64_t n, uint8_t* out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint4 d0, d1;
    sponge_generic(items, total, n == 0 ? 128u : 0u, true, n, d0, d1);
    reinterpret_cast<uint4*>(out)[0] = d0;
    reinterpret_cast<uint4*>(out)[1] = d1;
}

// ----------------------------------------------------------------------------
// Batched hashutil.Hash: n messages of 64 B (one permutation each).
// 6 waves/SIMD (73 VGPRs, no spill): 2^24 messages 1.804 -> 1.749 ms against
// the unconstrained 82 VGPRs / 5 waves (8 waves spills and halves the rate)
#define MK_K64_WAVES 6
__global__ __launch_bounds__(256, MK_K64_WAVES) void k_keccak64(const uint4* __restrict__ in, uint64_t n,
                                                               uint4* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4* p = in + 4 * i;
    const uint4 v0 = ld_stream(p), v1 = ld_stream(p + 1);
    const uint4 v2 = ld_stream(p + 2), v3 = ld_stream(p + 3);
    uint4 d0, d1;
    hash_pair(v0, v1, v2, v3, false, d0, d1);
    out[2 * i] = d0;
    out[2 * i + 1] = d1;
}

// digest outputs nobody in this kernel reads again: non-temporal with MK_SIDE_NT
__device__ __forceinline__ void st_out(uint4* p, uint4 v) {
    if constexpr (MK_SIDE_NT) {
        __builtin_nontemporal_store(*reinterpret_cast<const u32x4_t*>(&v), reinterpret_cast<u32x4_t*>(p));
    } else {
        *p = v;
    }
}

// Phase-locked 64-B messages (MK_K64_LOCK; C2 and 64-B node pairs) for n =
// 1024 * ngroups messages, the rest by k_keccak64.  1024-thread workgroups,
// one per CU, persistent; lane m of wave w hashes message g * 1024 + 64 w + m
// (one phase-locked permutation).  The wave's 64 messages (4 KB, contiguous)
// land in its 5 KB of LDS by coalesced DMA in a stride-5 image: position
// 5 m + u holds unit u of message m (u = 4 repeats unit 3), so consecutive
// lanes of an instruction read consecutive 16-B units and lane m reads its
// 4 units back at an odd stride, conflict-free.  The next group's copy goes
// out as soon as the message is read (one permutation ahead).
__global__ __launch_bounds__(kLockThreads, 1) void k_keccak64_lock(const uint4* __restrict__ in, uint64_t n,
                                                                   uint4* __restrict__ out) {
    __shared__ uint4 buf[kLockThreads / 64][5 * 64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint4* Bw = buf[wave];
    // a partial last group: lanes past n hash a copy of message n - 1 and store nothing
    const uint64_t ngroups = (n + kLockThreads - 1) / kLockThreads;
    // instructions [i0, i1) of the 5 (issued in parts over the permutation)
    auto dma = [&](uint64_t g, uint32_t i0, uint32_t i1) {
        const uint64_t m0 = g * kLockThreads + 64 * wave;
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (uint32_t i = i0; i < i1; ++i) {
            const uint32_t p = 64 * i + ln, m = p / 5, u = p - 5 * m;
            const uint64_t msg = m0 + m < n ? m0 + m : n - 1;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(in + 4 * msg + (u < 4 ? u : 3)),
                                             (__attribute__((address_space(3))) void*)(Bw + 64 * i), 16, 0,
                                             kSideAux);
        }
    };
    uint64_t g = blockIdx.x;
    if (g < ngroups) dma(g, 0, 5);
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;  // the previous group's digest, stored after the next wait
    uint64_t qi = 0;
    bool pend = false;
#pragma unroll 1
    for (; g < ngroups; g += gridDim.x) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the wave's messages have landed
        if (pend && qi < n) {
            st_out(out + 2 * qi, q0);
            st_out(out + 2 * qi + 1, q1);
        }
        State s;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint4 v = Bw[5 * lane + u];
            s.lo[2 * u] = v.x;
            s.hi[2 * u] = v.y;
            s.lo[2 * u + 1] = v.z;
            s.hi[2 * u + 1] = v.w;
        }
#pragma unroll
        for (int k = 8; k < 25; ++k) s.lo[k] = s.hi[k] = 0;
        s.lo[8] = 1u;  // byte 64
        s.hi[16] = 0x80000000u;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read: the next group's copy may land
        // one burst (5 instructions; in three parts over the permutation:
        // 1.476 -> 1.483 ms at 2^24, within noise, profiles/r05/side_dma_split/)
        if (g + gridDim.x < ngroups) dma(g + gridDim.x, 0, 5);
        keccak_f_digest_lock(s);
        digest(s, q0, q1);
        qi = g * kLockThreads + threadIdx.x;
        pend = true;
    }
    if (pend && qi < n) {
        st_out(out + 2 * qi, q0);
        st_out(out + 2 * qi + 1, q1);
    }
}

// Phase-locked node pass (the wide node pass of a whole tree, planner.cpp):
// 1024-thread workgroups, one per CU, persistent.  Thread t of group g folds
// the 16 node pairs [16 (1024 g + t), +16) -- 32 consecutive nodes, a subtree
// -- through 5 levels in registers (16 + 8 + 4 + 2 + 1 = 31 locked
// permutations) into output node 1024 g + t: the spans of k_reduce<NODE>
// workgroups 16 g .. 16 g + 15 with a.levels == 5, same output order.  Pair j
// of every lane of a wave (64 B, lanes 1 KB apart) lands in the wave's 5 KB
// of LDS by coalesced DMA in k_keccak64_lock's stride-5 image, issued as soon
// as pair j - 1 has been read (one permutation or more ahead); pairs j and
// j + 1 share a 128-B line, the second read an L2 hit.  All pairs are
// complete (no odd padding): the host launches whole groups of full pairs.
// Stores go right after a wait, as in k_leaf_lock_sc.
__global__ __launch_bounds__(kLockThreads, 1) void k_node_lock(ReduceArgs a, uint64_t ngroups) {
    __shared__ uint4 buf[kLockThreads / 64][5 * 64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint4* Bw = buf[wave];
    const uint4* in = reinterpret_cast<const uint4*>(a.items);
    uint4* out = reinterpret_cast<uint4*>(a.out);
    auto dma = [&](uint64_t g, uint32_t j) {
        const uint64_t p0 = (g * kLockThreads + 64 * wave) * kNodeLockPairs + j;  // lane 0's pair j
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (uint32_t i = 0; i < 5; ++i) {
            const uint32_t p = 64 * i + ln, m = p / 5, u = p - 5 * m;
            __builtin_amdgcn_global_load_lds(
                reinterpret_cast<const void*>(in + 4 * (p0 + (uint64_t)kNodeLockPairs * m) + (u < 4 ? u : 3)),
                (__attribute__((address_space(3))) void*)(Bw + 64 * i), 16, 0, 0);
        }
    };
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;  // the previous group's node, stored one group late
    uint64_t qi = 0;
    bool pend = false;
    uint64_t g = blockIdx.x;
    if (g < ngroups) dma(g, 0);
    // pair j of group g: wait for its DMA, read it, send the next pair's
    // DMA (pair j + 1, or pair 0 of the workgroup's next group), hash it
    auto pair = [&](uint64_t gg, uint32_t j, uint4& d0, uint4& d1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (j == 0 && pend) {
            out[2 * qi] = q0;
            out[2 * qi + 1] = q1;
            pend = false;
        }
        const uint4 l0 = Bw[5 * lane], l1 = Bw[5 * lane + 1], r0 = Bw[5 * lane + 2], r1 = Bw[5 * lane + 3];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read: the next pair may land
        if (j + 1 < kNodeLockPairs)
            dma(gg, j + 1);
        else if (gg + gridDim.x < ngroups)
            dma(gg + gridDim.x, 0);
        hash_node_lock(l0, l1, r0, r1, d0, d1);
    };
#pragma unroll 1
    for (; g < ngroups; g += gridDim.x) {
        uint4 a0 = q0, a1 = q1;  // level-3 node of the even quarter (the value is never read before it is set)
        uint4 b0 = q0, b1 = q1;  // level-4 node of the first half
#pragma unroll 1
        for (uint32_t k = 0; k < kNodeLockPairs / 4; ++k) {
            uint4 l0, l1, r0, r1, e0, e1;
            pair(g, 4 * k, l0, l1);
            pair(g, 4 * k + 1, r0, r1);
            hash_node_lock(l0, l1, r0, r1, e0, e1);
            pair(g, 4 * k + 2, l0, l1);
            pair(g, 4 * k + 3, r0, r1);
            hash_node_lock(l0, l1, r0, r1, l0, l1);
            hash_node_lock(e0, e1, l0, l1, e0, e1);  // level 3
            if ((k & 1) == 0) {
                a0 = e0;
                a1 = e1;
            } else {
                hash_node_lock(a0, a1, e0, e1, e0, e1);  // level 4
                if (k == 1) {
                    b0 = e0;
                    b1 = e1;
                } else {
                    hash_node_lock(b0, b1, e0, e1, q0, q1);  // level 5: the thread's output node
                }
            }
        }
        qi = g * kLockThreads + threadIdx.x;
        pend = true;
    }
    if (pend) {
        out[2 * qi] = q0;
        out[2 * qi + 1] = q1;
    }
}

// n messages of fixed msg_len bytes (any length / alignment).
__global__ __launch_bounds__(256) void k_keccak_fixed(const uint8_t* __restrict__ in, uint64_t n, uint32_t msg_len,
                                                      uint4* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint4 d0, d1;
    sponge_generic(in + i * msg_len, msg_len, 0, false, 0, d0, d1);
    out[2 * i] = d0;
    out[2 * i + 1] = d1;
}

// n variable-length messages: message i = in[offs[i], offs[i+1]).
__global__ __launch_bounds__(256) void k_keccak_var(const uint8_t* __restrict__ in, const uint64_t* __restrict__ offs,
                                                    uint64_t n, uint4* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = offs[i], b = offs[i + 1];
    uint4 d0, d1;
    sponge_generic(in + a, b - a, 0, false, 0, d0, d1);
    out[2 * i] = d0;
    out[2 * i + 1] = d1;
}

// ----------------------------------------------------------------------------
// Struct hashing (hash.go:141-159) for flat fixed-layout records: every
// record's message is the concatenation, in declaration order, of
//   MK_FIELD_BYTES: Keccak(le32(len) || bytes)   (hashedEncoding, hash.go:100-107)
//   MK_FIELD_RAW:   the raw little-endian bytes  (getEncoding of bool/uintN)
// k_struct_fields writes those messages; k_keccak_fixed hashes them.

// Keccak(le32(L) || A[0, L)) with 32-bit loads (A 4-byte aligned).
__device__ __noinline__ void sponge_prefix4(const uint8_t* __restrict__ A, uint32_t L, uint4& d0, uint4& d1) {
    const uint32_t* A32 = reinterpret_cast<const uint32_t*>(A);
    const uint32_t len = L + 4;
    const uint32_t nb = len / 136 + 1;
    State s;
    zero(s);
    for (uint32_t b = 0; b < nb; ++b) {
#pragma unroll
        for (int w = 0; w < 17; ++w) {
            const uint32_t m0 = b * 136 + 8u * w;  // message byte of this word
            uint32_t half[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t m = m0 + 4u * h;  // 4-byte group [m, m+4) of the message
                uint32_t v = 0;
                if (m == 0) {
                    v = L;
                } else if (m + 4 <= len) {
                    v = A32[(m - 4) / 4];
                } else if (m < len) {
                    for (uint32_t k = 0; k < len - m; ++k) v |= (uint32_t)A[m - 4 + k] << (8 * k);
                }
                if (m <= len && len < m + 4) v ^= 1u << (8 * (len - m));  // pad 0x01
                half[h] = v;
            }
            if (b == nb - 1 && w == 16) half[1] ^= 0x80000000u;
            s.lo[w] ^= half[0];
            s.hi[w] ^= half[1];
        }
        keccak_f(s);
    }
    digest(s, d0, d1);
}

template <bool FAST>
__global__ __launch_bounds__(256) void k_struct_fields(const uint8_t* __restrict__ rec, uint64_t n, StructSpec sp,
                                                       uint8_t* __restrict__ msg) {
    // one thread per (record, field): field-major so neighbouring lanes hash
    // the same field of neighbouring records
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * sp.nfields) return;
    const uint32_t f = (uint32_t)(t / n);
    const uint64_t i = t - (uint64_t)f * n;
    const uint8_t* r = rec + i * sp.rec_len;
    uint8_t* m = msg + i * sp.msg_len;
    const uint32_t off = sp.off[f], len = sp.len[f], out = sp.out_off[f];
    if (sp.kind[f] == 1) {  // MK_FIELD_BYTES
        uint4 d0, d1;
        if constexpr (FAST) {  // host-checked: every bytes field has len % 4 == 0, len + 4 < 136
            // one block, dword-granular: dword 0 = le32(len), dwords 1.. = bytes
            const uint32_t* A32 = reinterpret_cast<const uint32_t*>(r + off);
            const uint32_t nd = len / 4 + 1;  // message dwords
            State s;
            zero(s);
#pragma unroll
            for (int q = 0; q < 34; ++q) {
                uint32_t v = q == 0 ? len : ((uint32_t)q < nd ? A32[q - 1] : 0u);
                if ((uint32_t)q == nd) v ^= 1u;  // domain pad byte
                if (q & 1)
                    s.hi[q / 2] ^= v;
                else
                    s.lo[q / 2] ^= v;
            }
            s.hi[16] ^= 0x80000000u;
            keccak_f_digest(s);
            digest(s, d0, d1);
        } else {
            sponge_prefix4(r + off, len, d0, d1);
        }
        const uint32_t dw[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
        if ((out & 3u) == 0 && (((uintptr_t)m) & 3u) == 0) {
            uint32_t* o = reinterpret_cast<uint32_t*>(m + out);
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] = dw[k];
        } else {
#pragma unroll
            for (int k = 0; k < 32; ++k) m[out + k] = (uint8_t)(dw[k / 4] >> (8 * (k % 4)));
        }
    } else if (len == 8 && ((off | out) & 7u) == 0 && ((((uintptr_t)r) | ((uintptr_t)m)) & 7u) == 0) {
        *reinterpret_cast<uint2*>(m + out) = *reinterpret_cast<const uint2*>(r + off);
    } else {  // MK_FIELD_RAW
        for (uint32_t k = 0; k < len; ++k) m[out + k] = r[off + k];
    }
}

template __global__ void k_struct_fields<true>(const uint8_t*, uint64_t, StructSpec, uint8_t*);
template __global__ void k_struct_fields<false>(const uint8_t*, uint64_t, StructSpec, uint8_t*);

// Fused struct roots: one thread per record hashes every bytes field
// (Keccak(le32(len) || bytes), one block), assembles the struct message in
// LDS (dword-major: dword q of thread t at msg[q * 256 + t], conflict-free)
// and absorbs it -- no message round trip through HBM and one launch instead
// of two.  The next bytes field's loads are issued before the current
// field's permutation, so their latency hides behind it.  Host-checked
// layout: every bytes field dword-granular and at most 64 B, every output
// offset and raw length a multiple of 4, records 4-byte aligned (16-B
// aligned records and field offsets use 16-B loads).
// Dynamic LDS: kStructThreads * msg_len bytes.
namespace {
__device__ __forceinline__ void load_field16(const uint8_t* __restrict__ p, uint32_t len, uint32_t vec16,
                                             uint32_t (&a)[16]) {
    if (vec16) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 v = (4u * k < len / 4) ? *reinterpret_cast<const uint4*>(p + 16 * k) : make_uint4(0, 0, 0, 0);
            a[4 * k] = v.x;
            a[4 * k + 1] = v.y;
            a[4 * k + 2] = v.z;
            a[4 * k + 3] = v.w;
        }
    } else {
        const uint32_t* A32 = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
        for (int k = 0; k < 16; ++k) a[k] = (uint32_t)k < len / 4 ? A32[k] : 0u;
    }
}
}  // namespace

__global__ __launch_bounds__(kStructThreads) void k_struct_fused(const uint8_t* __restrict__ rec, uint64_t n,
                                                                 StructSpec sp, uint32_t vec16,
                                                                 uint4* __restrict__ roots) {
    extern __shared__ uint32_t msg[];
    const uint32_t tid = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * kStructThreads + tid;
    const bool live = i < n;
    const uint8_t* r = rec + (live ? i : 0) * sp.rec_len;
    // first bytes field: loads in flight while the raw scalars are copied
    uint32_t f = 0;
    while (f < sp.nfields && sp.kind[f] != 1) ++f;
    uint32_t nxt[16];
    if (f < sp.nfields) load_field16(r + sp.off[f], sp.len[f], vec16, nxt);
#pragma unroll 1
    for (uint32_t g = 0; g < sp.nfields; ++g) {  // MK_FIELD_RAW, len 4 or 8
        if (sp.kind[g] == 1) continue;
        const uint32_t* A32 = reinterpret_cast<const uint32_t*>(r + sp.off[g]);
        const uint32_t q0 = sp.out_off[g] / 4;
        msg[q0 * kStructThreads + tid] = A32[0];
        if (sp.len[g] == 8) msg[(q0 + 1) * kStructThreads + tid] = A32[1];
    }
#pragma unroll 1
    while (f < sp.nfields) {  // MK_FIELD_BYTES: Keccak(le32(len) || bytes), one block
        const uint32_t len = sp.len[f], q0 = sp.out_off[f] / 4;
        uint32_t a[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) a[k] = nxt[k];
        ++f;
        while (f < sp.nfields && sp.kind[f] != 1) ++f;
        if (f < sp.nfields) load_field16(r + sp.off[f], sp.len[f], vec16, nxt);
        const uint32_t nd = len / 4 + 1;  // message dwords (<= 17)
        State s;
        zero(s);
#pragma unroll
        for (int q = 0; q < 18; ++q) {
            uint32_t v = q == 0 ? len : ((uint32_t)q < nd ? a[q - 1] : 0u);
            if ((uint32_t)q == nd) v ^= 1u;  // domain pad byte
            if (q & 1)
                s.hi[q / 2] ^= v;
            else
                s.lo[q / 2] ^= v;
        }
        s.hi[16] ^= 0x80000000u;
        keccak_f_digest(s);
        uint4 d0, d1;
        digest(s, d0, d1);
        const uint32_t dw[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
        for (int w = 0; w < 8; ++w) msg[(q0 + w) * kStructThreads + tid] = dw[w];
    }
    // struct hash over the msg_len-byte message (msg_len % 4 == 0)
    const uint32_t mw = sp.msg_len / 4, nb = sp.msg_len / 136 + 1;
    State s;
    zero(s);
#pragma unroll 1
    for (uint32_t b = 0; b < nb; ++b) {
#pragma unroll
        for (int w = 0; w < 34; ++w) {
            const uint32_t q = 34 * b + w;
            uint32_t v = q < mw ? msg[q * kStructThreads + tid] : 0u;
            if (q == mw) v ^= 1u;
            if (b == nb - 1 && w == 33) v ^= 0x80000000u;
            if (w & 1)
                s.hi[w / 2] ^= v;
            else
                s.lo[w / 2] ^= v;
        }
        if (b + 1 < nb)  // nb is uniform (one struct layout)
            keccak_f(s);
        else
            keccak_f_digest(s);
    }
    if (live) {
        uint4 d0, d1;
        digest(s, d0, d1);
        roots[2 * i] = d0;
        roots[2 * i + 1] = d1;
    }
}

// Struct roots for the "bytes fields first, then 8-byte scalars" layout
// (pb.Validator: 3 bytes fields + 6 uint64) with the message
// layout known at compile time: the NB field digests go to this thread's
// LDS column (24 KB per workgroup for NB = 3, against 36 KB for the whole
// message in k_struct_fused), the NRAW scalars are re-read from the record
// at absorb time, and the absorb loop is unrolled over compile-time message
// dwords.  No barrier: a thread only touches its own LDS column.
#define MK_STRUCT_REG_WAVES 6
template <int NB, int NRAW>
__global__ __launch_bounds__(kStructThreads, MK_STRUCT_REG_WAVES) void k_struct_reg(const uint8_t* __restrict__ rec,
                                                                                  uint64_t n, StructSpec sp,
                                                                                  uint32_t vec16,
                                                                                  uint4* __restrict__ roots) {
    __shared__ uint32_t dg[NB * 8 * kStructThreads];
    const uint32_t tid = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * kStructThreads + tid;
    if (i >= n) return;
    const uint8_t* r = rec + i * sp.rec_len;
    uint32_t nxt[16];
    load_field16(r + sp.off[0], sp.len[0], vec16, nxt);
#pragma unroll 1
    for (uint32_t f = 0; f < (uint32_t)NB; ++f) {  // Keccak(le32(len) || bytes), one block
        const uint32_t len = sp.len[f];
        uint32_t a[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) a[k] = nxt[k];
        if (f + 1 < (uint32_t)NB) load_field16(r + sp.off[f + 1], sp.len[f + 1], vec16, nxt);
        const uint32_t nd = len / 4 + 1;
        State s;
        zero(s);
#pragma unroll
        for (int q = 0; q < 18; ++q) {
            uint32_t v = q == 0 ? len : ((uint32_t)q < nd ? a[q - 1] : 0u);
            if ((uint32_t)q == nd) v ^= 1u;
            if (q & 1)
                s.hi[q / 2] ^= v;
            else
                s.lo[q / 2] ^= v;
        }
        s.hi[16] ^= 0x80000000u;
        keccak_f_digest(s);
        uint4 d0, d1;
        digest(s, d0, d1);
        const uint32_t dw[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
        for (int w = 0; w < 8; ++w) dg[(8 * f + w) * kStructThreads + tid] = dw[w];
    }
    uint32_t raw[2 * NRAW > 0 ? 2 * NRAW : 1];
#pragma unroll
    for (int k = 0; k < NRAW; ++k) {
        const uint32_t* A32 = reinterpret_cast<const uint32_t*>(r + sp.off[NB + k]);
        raw[2 * k] = A32[0];
        raw[2 * k + 1] = A32[1];
    }
    constexpr int MW = 8 * NB + 2 * NRAW;  // message dwords
    constexpr int NBLK = 4 * MW / 136 + 1;
    State s;
    zero(s);
#pragma unroll
    for (int b = 0; b < NBLK; ++b) {
#pragma unroll
        for (int w = 0; w < 34; ++w) {
            const int q = 34 * b + w;
            uint32_t v = q < 8 * NB ? dg[q * kStructThreads + tid] : (q < MW ? raw[q - 8 * NB] : 0u);
            if (q == MW) v ^= 1u;
            if (b == NBLK - 1 && w == 33) v ^= 0x80000000u;
            if (w & 1)
                s.hi[w / 2] ^= v;
            else
                s.lo[w / 2] ^= v;
        }
        if (b + 1 < NBLK)
            keccak_f(s);
        else
            keccak_f_digest(s);
    }
    uint4 d0, d1;
    digest(s, d0, d1);
    roots[2 * i] = d0;
    roots[2 * i + 1] = d1;
}
template __global__ void k_struct_reg<3, 6>(const uint8_t*, uint64_t, StructSpec, uint32_t, uint4*);

// Phase-locked struct roots (MK_STRUCT_LOCK) for the validator layout of
// SURVEY §8d (ValidatorRecord: Pubkey 48 B @0, WithdrawalCredentialsHash32
// 32 B @48, RandaoCommitmentHash32 32 B @80, six uint64 @112..152; 160-B
// records, 16-B aligned; the host checks the StructSpec against
// kValOff/kValLen) for n = 1024 * ngroups records, the rest by k_struct_reg.
// 1024-thread workgroups, one per CU, persistent; lane m of wave w hashes
// record g * 1024 + 64 w + m with 3 + 2 phase-locked permutations
// (hash.go:141-159 over the field hashes of :100-107).  The wave's 64
// records (10 KB, contiguous) are copied into its LDS by coalesced DMA (64 x
// 16 B per instruction, consecutive lanes on consecutive units; 160 KB for
// the workgroup), each field digest overwrites that field's own bytes once
// they are absorbed, and the struct message is read back from the record's
// slot; the next group's copy goes out once it is (before the two
// struct-message permutations).
// Level-1 window w of merkleHash over `total` bytes of items whose length
// divides 128 (chunks of 128 B, windows of 256 B) at a 16-B aligned `base`
// (total % 8 == 0): a full window streams its 256 B; the ragged last one
// hashes its r bytes, plus 0^128 when they fill one chunk only (hash.go:225-228).
__device__ __forceinline__ void window256_or_ragged(const uint8_t* __restrict__ base, uint64_t total, uint64_t w,
                                                    uint4& d0, uint4& d1) {
    if (256 * w + 256 <= total) {
        hash_window256(reinterpret_cast<const uint4*>(base) + 16 * w, d0, d1);
        return;
    }
    const uint32_t r = (uint32_t)(total - 256 * w);                // 8..248 bytes
    const uint32_t nwd = r / 8, len = r + (r <= 128 ? 128u : 0u);  // 136..256 B: two blocks
    const uint2* p = reinterpret_cast<const uint2*>(base + 256 * w);
    State s;
    zero(s);
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int k = 0; k < 17; ++k) {
            const uint32_t q = 17 * b + k;
            uint2 v = q < nwd ? p[q] : make_uint2(0, 0);
            if (q == len / 8) v.x ^= 1u;  // domain pad (len % 8 == 0)
            s.lo[k] ^= v.x;
            s.hi[k] ^= v.y;
        }
        if (b == 0) {
            keccak_f(s);
        } else {
            s.hi[16] ^= 0x80000000u;
            keccak_f_digest(s);
        }
    }
    digest(s, d0, d1);
}

__device__ constexpr uint32_t kValOff[9] = {0, 48, 80, 112, 120, 128, 136, 144, 152};
__device__ constexpr uint32_t kValLen[9] = {48, 32, 32, 8, 8, 8, 8, 8, 8};
//
// gpw > 0 (the list root, mk_dev_ssz_struct_list_root): workgroup b takes the
// CONTIGUOUS groups [gpw b, gpw b + gpw) instead of striding over the grid,
// and after its last group hashes the level-1 windows of the registry's
// merkleHash (hash.go:194-239 over the 32-B roots: 8 roots = 2 chunks per
// window) from the roots it has just written -- one window per lane on waves
// 0..(gpw*2 - 1), free-running (the other waves have left), into `wins`.  That
// replaces the merkleHash leaf pass, a latency-bound pass over the whole
// roots array.
//
// PREV (gpw == 4, a stream of states, registry.StatePipeline): the launch
// also builds levels 2..10 of the PREVIOUS state's registry tree from that
// state's level-1 windows (its own launch wrote them): workgroup b < nfull
// takes the subtree over windows [512 b, 512 b + 512) -- 256 + 128 + ... + 1
// node permutations -- and writes its level-10 node, so what is left of that
// tree is a 245-node top.  Each wave does ONE of them as an extra lock-step
// permutation (level 2 on waves 0-3, 3 on 4-5, then levels 4..10 on waves
// 6..12, one node per lane), so every wave runs 21 permutations and the
// same barriers; waves 13-15 take levels 2, 3, 4 of the previous state's
// second list (the balances: 128 windows per workgroup, 64 + 32 + 16 node
// permutations), leaving 16 nodes per workgroup.  Level k sits before the field
// permutation at position 2 (k - 2) of the 16 (4 groups x f0, f1, f2, s1);
// level 10 after the group loop: the writer waits for its store at round 12
// of the field permutation that follows its slot, and counted in barriers
// (waves line up by barrier count, not by position) every reader loads at
// least half a permutation after that wait (through L2: this CU never read
// those lines, and its L1 was invalidated at dispatch).
template <bool PREV>
__global__ __launch_bounds__(kLockThreads, 1) void k_struct_lock(const uint8_t* __restrict__ rec, uint64_t n,
                                                                 uint4* __restrict__ roots, uint32_t gpw,
                                                                 uint4* __restrict__ wins,
                                                                 const uint8_t* __restrict__ vals, uint64_t vbytes,
                                                                 uint4* __restrict__ vwins, StructPrev prev) {
    constexpr uint32_t kRecLen = 160, kRw = kRecLen / 4, kNinstr = kRecLen / 16;
    __shared__ uint32_t buf[kLockThreads / 64][64 * kRw];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t* Bw = buf[wave];
    const uint32_t wv = __builtin_amdgcn_readfirstlane(wave);
    // this wave's slot: the registry's level my_k (waves 0-12: 2 on 0-3, 3 on
    // 4-5, 4..10 on 6..12) or the second list's (waves 13-15: levels 2, 3,
    // 4), at position my_pos (2 (k - 2); the registry's level 10 at 16, after
    // the group loop)
    const bool my_val = wv >= 13;
    const uint32_t my_k = my_val ? wv - 11u : wv < 4 ? 2u : wv < 6 ? 3u : wv - 2u;
    const uint32_t my_pos = my_k == 10 ? 16u : 2u * (my_k - 2u);
    auto prev_slot = [&] {
        const uint32_t k = my_k;
        const uint32_t sub = my_val ? 128u : 512u;                           // level-1 nodes per subtree
        const uint32_t w0 = my_val ? wv : k == 2 ? 0u : k == 3 ? 4u : k + 2u;  // first wave of level k
        const uint32_t per = sub >> (k - 1);                                 // level-k nodes per subtree
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));  // computed here, not hoisted and kept live across the loop
        const uint32_t j = 64u * (wv - w0) + ln;
        const bool act = prev.live && blockIdx.x < (my_val ? prev.nvfull : prev.nfull) && j < per;
        const uint4* src = k == 2 ? (my_val ? prev.v1 : prev.l1) + 2 * (sub * blockIdx.x)
                                  : (my_val ? prev.vlv[k - 3] : prev.lv[k - 3]) + 4 * (per * blockIdx.x);
        asm volatile("" ::: "memory");
        State s;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 v = act ? src[4 * j + q] : make_uint4(0, 0, 0, 0);
            s.lo[2 * q] = v.x;
            s.hi[2 * q] = v.y;
            s.lo[2 * q + 1] = v.z;
            s.hi[2 * q + 1] = v.w;
        }
#pragma unroll
        for (int w = 8; w < 25; ++w) s.lo[w] = s.hi[w] = 0;
        s.lo[8] = 1u;  // byte 64
        s.hi[16] = 0x80000000u;
        keccak_f_digest_lock(s);
        if (act) {
            uint4 d0, d1;
            digest(s, d0, d1);
            uint4* dst = (my_val ? prev.vlv[k - 2] : prev.lv[k - 2]) + 2 * (per * blockIdx.x + j);
            dst[0] = d0;
            dst[1] = d1;
        }
        asm volatile("" ::: "memory");
    };
    // the last group may be partial: its lanes past n copy the last record
    // (every wave still runs the same permutations and barriers) and store nothing
    const uint64_t ngroups = (n + kLockThreads - 1) / kLockThreads;
    const uint64_t last_unit = n * (kRecLen / 16) - 1;
    // instructions [i0, i1) of the kNinstr (issued in parts).  Record m of
    // the wave sits in 16-B slots [10 m, 10 m + 10) rotated by one unit when
    // bits 2 and 3 of m differ (unit u in slot 10 m + (u + rot) mod 10).  On
    // gfx950 a ds_read_b128 is conflict-free when the slots of each 16
    // consecutive lanes differ mod 16, a ds_write_b128 when those of each 8
    // differ mod 8 (tools/lds_bank_probe.hip, profiles/r06/lds_bank_probe.txt);
    // the plain 160-B stride fails both (lanes l, l + 8 and l, l + 4 collide:
    // 1.63 M SQ_LDS_BANK_CONFLICT per launch, profiles/r05/pmc/), this
    // rotation passes both.  The copy stays one contiguous 1-KB LDS write per
    // instruction, each lane fetching the unit its slot holds
    auto dma = [&](uint64_t g, uint32_t i0 = 0, uint32_t i1 = kNinstr) {
        const uint64_t u0 = (g * kLockThreads + 64 * wave) * (kRecLen / 16);
        const uint4* src = reinterpret_cast<const uint4*>(rec);
#pragma unroll
        for (uint32_t i = i0; i < i1; ++i) {
            const uint32_t sl = 64 * i + lane, m = sl / 10u, v = sl - 10u * m;
            const uint32_t rot = ((m >> 2) ^ (m >> 3)) & 1u;
            const uint64_t u = u0 + 10u * m + (v >= rot ? v - rot : v + 10u - rot);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (u < last_unit ? u : last_unit)),
                                             (__attribute__((address_space(3))) void*)(Bw + 256 * i), 16, 0,
                                             kSideAux);
        }
    };
    const uint64_t g_begin = gpw ? (uint64_t)blockIdx.x * gpw : blockIdx.x;
    const uint64_t g_end = gpw ? (g_begin + gpw < ngroups ? g_begin + gpw : ngroups) : ngroups;
    const uint64_t g_step = gpw ? 1 : gridDim.x;
    uint64_t g = g_begin;
    if (g < g_end) dma(g);
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;  // the previous group's root, stored after the next wait
    uint64_t qi = 0;
    bool pend = false;
    // the previous state's slots run in workgroups of exactly gpw == 4 groups
    // (uniform over the workgroup: all its waves run the same permutations)
    const bool slots = PREV && gpw == 4 && g_end - g_begin == 4;
    // this lane's record: units 0..8 at R (rotated), unit 9 at R9
    const uint32_t rot = ((lane >> 2) ^ (lane >> 3)) & 1u;
    uint32_t* const R = Bw + lane * kRw + 4u * rot;
    const uint32_t* const R9 = Bw + lane * kRw + (rot ? 0u : 36u);
#pragma unroll 1
    for (; g < g_end; g += g_step) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the wave's records have landed
        if (pend && qi < n) {
            roots[2 * qi] = q0;
            roots[2 * qi + 1] = q1;
        }
        const uint32_t pos0 = 4u * (uint32_t)(g - g_begin);  // slot position of field 0 of this group
#pragma unroll
        for (int f = 0; f < 3; ++f) {  // Keccak(le32(len) || bytes), one block
            // this wave's slot of the previous state's tree (f = 0, 2 only: positions 2 (k - 2))
            const bool slot_here = slots && (f == 0 || f == 2) && my_pos == pos0 + f;
            if (slot_here) prev_slot();
            const uint32_t len = kValLen[f], off = kValOff[f] / 4, nd = len / 4 + 1;
            State s;
#pragma unroll
            for (uint32_t q = 0; q < 18; ++q) {
                uint32_t v = q == 0 ? len : (q < nd ? R[off + q - 1] : 0u);
                if (q == nd) v ^= 1u;
                if (q & 1)
                    s.hi[q / 2] = v;
                else
                    s.lo[q / 2] = v;
            }
#pragma unroll
            for (int k = 9; k < 25; ++k) s.lo[k] = s.hi[k] = 0;
            s.hi[16] = 0x80000000u;
            if constexpr (PREV) {
                // the slot's node store completes mid-permutation, before the
                // next level's reader (two positions on) can pass a barrier
                keccak_f_digest_lock<12>(s, [&] {
                    if (slot_here) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                });
            } else {
                keccak_f_digest_lock(s);
            }
            // the digest replaces the field's own bytes (absorbed above)
            R[off + 0] = s.lo[0]; R[off + 1] = s.hi[0]; R[off + 2] = s.lo[1]; R[off + 3] = s.hi[1];
            R[off + 4] = s.lo[2]; R[off + 5] = s.hi[2]; R[off + 6] = s.lo[3]; R[off + 7] = s.hi[3];
        }
        // struct message (hash.go:141-159): the digests of fields 0..2, then
        // the six uint64 raw: 36 dwords = block 1 (34) + 2 dwords of block 2
        State s;
#pragma unroll
        for (int q = 0; q < 34; ++q) {
            // the six uint64 are dwords 28..39: units 7, 8 and (dwords 36..39) 9
            const uint32_t v = q < 24 ? R[kValOff[q / 8] / 4 + q % 8]
                                      : (q < 32 ? R[kValOff[3] / 4 + (q - 24)] : R9[q - 32]);
            if (q & 1)
                s.hi[q / 2] = v;
            else
                s.lo[q / 2] = v;
        }
#pragma unroll
        for (int k = 17; k < 25; ++k) s.lo[k] = s.hi[k] = 0;
        const uint32_t t0 = R9[2], t1 = R9[3];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // record read: the next group's copy may land
        // the next group's copy in three parts over the first struct
        // permutation, not one burst of 16 waves' DMA (the
        // 10^6 list root 0.600 -> 0.593 ms, profiles/r05/side_dma_split/)
        const bool more = g + g_step < g_end;
        keccak_f_lock_mid3<2, 8, 14>(s, [&] { if (more) dma(g + g_step, 0, 4); },
                                     [&] { if (more) dma(g + g_step, 4, 7); },
                                     [&] { if (more) dma(g + g_step, 7, 10); });
        s.lo[0] ^= t0;
        s.hi[0] ^= t1;
        s.lo[1] ^= 1u;  // domain pad at message byte 144 = block 2 byte 8
        s.hi[16] ^= 0x80000000u;
        keccak_f_digest_lock(s);
        digest(s, q0, q1);
        qi = g * kLockThreads + threadIdx.x;
        pend = true;
    }
    // the registry's level 10 (wave 12) after the loop.  Waves line up by
    // barrier count: the level-9 writer (wave 11) stores at the end of its
    // slot permutation (its 18th of 21) and waits for the store at round 12 of
    // the next (group 3's f2); wave 12 runs f2 as its 18th, the two struct
    // permutations as its 19th-20th and loads level 9 at the start of its
    // 21st, 1.5 permutations after that wait (before the loop's end it would
    // load at the writer's store).  Nothing in this launch reads it.
    if (slots && my_pos == 16u) prev_slot();
    if (pend && qi < n) {
        roots[2 * qi] = q0;
        roots[2 * qi + 1] = q1;
    }
    if (!wins || g_begin >= g_end) return;
    // the workgroup's roots are in L2 (written above; this CU never read those
    // lines, and its L1 was invalidated at dispatch): every wave's stores
    // complete, then one window per lane -- the registry's windows over the
    // roots just written, then this workgroup's share of the optional second
    // list's windows (`vals`, vbytes bytes of items dividing 128; the State's
    // balances) on the lanes left over
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint64_t r0 = g_begin * kLockThreads, r1 = g_end * kLockThreads < n ? g_end * kLockThreads : n;
    const uint64_t w0 = r0 / 8, nw = (r1 - r0 + 7) / 8;
    // PREV: 128 windows per workgroup (the subtrees the next launch's slots
    // take; 128 >= ceil(vw_total / grid) for the State's 8-B balances)
    const uint64_t vw_total = (vbytes + 255) / 256;
    const uint64_t vpw = PREV && gpw == 4 ? 128u : (vw_total + gridDim.x - 1) / gridDim.x;
    const uint64_t v0 = (uint64_t)blockIdx.x * vpw;
    const uint64_t nv = vals && v0 < vw_total ? (vw_total - v0 < vpw ? vw_total - v0 : vpw) : 0;
#pragma unroll 1
    for (uint64_t t = threadIdx.x; t < nw + nv; t += kLockThreads) {
        const bool reg = t < nw;
        const uint64_t w = reg ? w0 + t : v0 + (t - nw);
        const uint8_t* base = reg ? reinterpret_cast<const uint8_t*>(roots) : vals;
        const uint64_t total = reg ? 32 * n : vbytes;
        uint4 d0, d1;
        window256_or_ragged(base, total, w, d0, d1);
        uint4* o = reg ? wins : vwins;
        o[2 * w] = d0;
        o[2 * w + 1] = d1;
    }
}

template __global__ void k_struct_lock<false>(const uint8_t*, uint64_t, uint4*, uint32_t, uint4*, const uint8_t*,
                                              uint64_t, uint4*, StructPrev);
template __global__ void k_struct_lock<true>(const uint8_t*, uint64_t, uint4*, uint32_t, uint4*, const uint8_t*,
                                             uint64_t, uint4*, StructPrev);
template __global__ void k_struct_reg<2, 0>(const uint8_t*, uint64_t, StructSpec, uint32_t, uint4*);

// The same layouts for SMALL registries (the 16,384-validator C1 shape),
// where every wave runs alone on its SIMD and the cost is the chain of
// permutation latencies, not throughput: four lanes per record.  Lanes
// 0..NB-1 of a record hash its NB bytes fields side by side (one
// permutation of latency instead of NB), the digests meet in LDS, and lanes
// 0 and 1 hash the struct message (2 blocks) as a lo/hi lane pair (round 6:
// C1's struct roots 29.6 -> see DESIGN §4.5): 3 serial permutations per
// record instead of 5, the last two at lane-pair latency.  The host takes this form while 4 lanes per record still fit
// the chip once (n <= kStructSplitMaxN).
// The body, for the first 256 threads of the calling workgroup (every
// thread of it must call: the digests meet in LDS behind a barrier):
// records [64 blk, 64 blk + 64), roots to roots[].
template <int NB, int NRAW>
__device__ __forceinline__ void struct_split_body(const uint8_t* __restrict__ rec, uint64_t n, const StructSpec& sp,
                                                  uint32_t vec16, uint4* __restrict__ roots, uint64_t blk,
                                                  uint32_t (&dg)[NB * 8][64]) {
    static_assert(NB <= 4, "one lane per bytes field");
    constexpr uint32_t kV = 256 / 4;  // records per workgroup
    const uint32_t tid = threadIdx.x, v = (tid >> 2) & (kV - 1), role = tid & 3u;
    const uint64_t i = blk * kV + v;
    const bool live = tid < 256u && i < n;
    const uint8_t* r = rec + (live ? i : 0) * sp.rec_len;
    if (live && role < (uint32_t)NB) {  // Keccak(le32(len) || bytes), one block
        const uint32_t off = role == 0 ? sp.off[0] : role == 1 ? sp.off[1 % NB] : sp.off[2 % NB];
        const uint32_t len = role == 0 ? sp.len[0] : role == 1 ? sp.len[1 % NB] : sp.len[2 % NB];
        uint32_t a[16];
        load_field16(r + off, len, vec16, a);
        const uint32_t nd = len / 4 + 1;
        State s;
        zero(s);
#pragma unroll
        for (int q = 0; q < 18; ++q) {
            uint32_t x = q == 0 ? len : ((uint32_t)q < nd ? a[q - 1] : 0u);
            if ((uint32_t)q == nd) x ^= 1u;
            if (q & 1)
                s.hi[q / 2] ^= x;
            else
                s.lo[q / 2] ^= x;
        }
        s.hi[16] ^= 0x80000000u;
        keccak_f_digest(s);
        uint4 d0, d1;
        digest(s, d0, d1);
        const uint32_t dw[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
        for (int w = 0; w < 8; ++w) dg[8 * role + w][v] = dw[w];
    }
    __syncthreads();
    // the struct message (the digests, then the raw scalars) on lanes 0 and 1
    // of the record as a lo/hi lane pair (mk::pair: lane p holds half p of
    // every Keccak lane, so message dword 2k + p is its word k and no
    // conversion is needed): 2 x ~12.8 k cycles of latency for the two
    // blocks against 2 x ~21 k on one lane
    if (!live || role > 1u) return;
    const uint32_t p = role;
    uint32_t raw[NRAW > 0 ? NRAW : 1];
#pragma unroll
    for (int k = 0; k < NRAW; ++k) raw[k] = reinterpret_cast<const uint32_t*>(r + sp.off[NB + k])[p];
    constexpr int MW = 8 * NB + 2 * NRAW;  // message dwords
    constexpr int NBLK = 4 * MW / 136 + 1;
    pair::Half s;
    pair::zero(s);
#pragma unroll
    for (int b = 0; b < NBLK; ++b) {
#pragma unroll
        for (int k = 0; k < 17; ++k) {
            const int q0 = 34 * b + 2 * k;  // this Keccak lane's lo dword (MW and 8 NB are even)
            uint32_t x = q0 < 8 * NB ? dg[q0 + p][v] : (q0 < MW ? raw[(q0 - 8 * NB) / 2] : 0u);
            if (q0 == MW && p == 0u) x ^= 1u;
            if (b == NBLK - 1 && k == 16 && p == 1u) x ^= 0x80000000u;
            s.v[k] ^= x;
        }
        pair::keccak_f(s, p != 0u);
    }
    uint32_t* out = reinterpret_cast<uint32_t*>(roots) + 8 * i;
#pragma unroll
    for (int k = 0; k < 4; ++k) out[2 * k + p] = s.v[k];
}

template <int NB, int NRAW>
__global__ __launch_bounds__(256) void k_struct_split(const uint8_t* __restrict__ rec, uint64_t n, StructSpec sp,
                                                      uint32_t vec16, uint4* __restrict__ roots) {
    __shared__ uint32_t dg[NB * 8][64];
    struct_split_body<NB, NRAW>(rec, n, sp, vec16, roots, blockIdx.x, dg);
}
template __global__ void k_struct_split<3, 6>(const uint8_t*, uint64_t, StructSpec, uint32_t, uint4*);
template __global__ void k_struct_split<2, 0>(const uint8_t*, uint64_t, StructSpec, uint32_t, uint4*);

// ----------------------------------------------------------------------------
// n messages of msg_len bytes, msg_len % 8 == 0, 8-byte aligned: whole-word
// loads only (deposit leaves: 280 B = 35 words = 3 blocks).
__global__ __launch_bounds__(256) void k_keccak_words(const uint2* __restrict__ in, uint64_t n, uint32_t nwords,
                                                      uint4* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint2* p = in + i * nwords;
    const uint32_t nb = nwords / 17 + 1;
    State s;
    zero(s);
    if ((((uintptr_t)p) & 7u) == 0) {
        // 16-B loads: a message starts 16-B aligned or 8 bytes past it; each
        // block reads the 9 aligned 16-B units that cover its 17 words and
        // selects per lane (deposit leaves: 35 words, 3 blocks)
        const uint32_t so = (((uintptr_t)p) & 15u) ? 1u : 0u;
        const uint4* q = reinterpret_cast<const uint4*>(p - so);
        const uint32_t nq = (nwords + so + 1) / 2;
#pragma unroll 1
        for (uint32_t b = 0; b < nb; ++b) {
            const uint32_t first = 17 * b + so;  // aligned word index of block word 0
            const uint32_t pb = first >> 1, odd = first & 1u;
            uint2 e[18];
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const uint4 t = (pb + k) < nq ? ld_stream(q + pb + k) : make_uint4(0, 0, 0, 0);
                e[2 * k] = make_uint2(t.x, t.y);
                e[2 * k + 1] = make_uint2(t.z, t.w);
            }
#pragma unroll
            for (int w = 0; w < 17; ++w) {
                const uint32_t idx = 17 * b + w;
                // static-index select (a conditional index would spill e[] to scratch)
                const uint32_t msk = 0u - odd;
                uint2 v = make_uint2(__builtin_amdgcn_bitop3_b32(e[w].x, e[w + 1].x, msk, 0xD8),
                                     __builtin_amdgcn_bitop3_b32(e[w].y, e[w + 1].y, msk, 0xD8));
                if (idx >= nwords) v = make_uint2(idx == nwords ? 1u : 0u, 0u);  // zero / domain pad
                s.lo[w] ^= v.x;
                s.hi[w] ^= v.y;
            }
            if (b == nb - 1) s.hi[16] ^= 0x80000000u;
            if (b + 1 < nb)  // nb is uniform (fixed message length)
                keccak_f(s);
            else
                keccak_f_digest(s);
        }
    } else {
#pragma unroll 1
        for (uint32_t b = 0; b < nb; ++b) {
            const uint32_t base = b * 17;
#pragma unroll
            for (int w = 0; w < 17; ++w) {
                const uint32_t idx = base + w;
                if (idx < nwords) {
                    const uint2 v = ld_stream(p + idx);
                    s.lo[w] ^= v.x;
                    s.hi[w] ^= v.y;
                } else if (idx == nwords) {
                    s.lo[w] ^= 1u;  // domain pad byte right after the message
                }
            }
            if (b == nb - 1) s.hi[16] ^= 0x80000000u;
            if (b + 1 < nb)  // nb is uniform (fixed message length)
                keccak_f(s);
            else
                keccak_f_digest(s);
        }
    }
    uint4 d0, d1;
    digest(s, d0, d1);
    out[2 * i] = d0;
    out[2 * i + 1] = d1;
}

// Fixed-size records of NW 8-byte words (8-B aligned; deposit leaves: 280 B
// = 35 words = 3 blocks), grid-stride; each block is loaded right before it
// is absorbed.  8-B loads need no per-lane alignment select (k_keccak_words
// spends 2 VALU per word on it).  Prefetching block b+1 into 34 VGPRs while
// block b permutes was 1-2 % slower on the 2^20-deposit trie (0.588 vs
// 0.582 ms, profiles/r02d/ab_rec_prefetch.log): the other resident waves
// hide the load as well.  At 5 waves/SIMD (96 VGPRs, 4 dwords spilled) the
// stream of 2^20-deposit tries got 3 % slower (profiles/r02m/rejected/).
#define MK_REC_WAVES 1
template <int NW>
__global__ __launch_bounds__(kRecThreads, MK_REC_WAVES) void k_keccak_rec(const uint2* __restrict__ in, uint64_t n,
                                                                          uint4* __restrict__ out) {
    constexpr int NB = NW / 17 + 1;
    const uint64_t stride = (uint64_t)gridDim.x * kRecThreads;
#pragma unroll 1
    for (uint64_t i = (uint64_t)blockIdx.x * kRecThreads + threadIdx.x; i < n; i += stride) {
        const uint2* p = in + i * NW;
        State s;
        zero(s);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
#pragma unroll
            for (int w = 0; w < 17; ++w) {
                const int idx = 17 * b + w;
                if (idx < NW) {
                    const uint2 v = p[idx];
                    s.lo[w] ^= v.x;
                    s.hi[w] ^= v.y;
                } else if (idx == NW) {
                    s.lo[w] ^= 1u;  // domain pad byte right after the message
                }
            }
            if (b == NB - 1) s.hi[16] ^= 0x80000000u;
            if (b + 1 < NB)
                keccak_f(s);
            else
                keccak_f_digest(s);
        }
        uint4 d0, d1;
        digest(s, d0, d1);
        out[2 * i] = d0;
        out[2 * i + 1] = d1;
    }
}
template __global__ void k_keccak_rec<35>(const uint2*, uint64_t, uint4*);

// Phase-locked deposit-trie front (MK_TRIE_LOCK): the leaf hashes of 280-B
// deposits (deposit_trie.go:32, Hash(depositData)) AND the trie levels above
// them up to the node over DPT leaves (deposit_trie.go:33-38), in one launch.
// Every thread owns DPT consecutive deposits: 3 permutations each (2 full
// rate blocks + the 8-B tail), then DPT - 1 node permutations, all phase-
// locked (two s_barriers per round) -- DPT = 4: 15 permutations,
// levels 1-2.  Thread t of group g holds deposits DPT (g NT + t) + i; it
// writes its leaves and nodes to levels 0..log2(DPT) of the trie (all kept:
// GenerateMerkleBranch reads them), so the 2^20-leaf round trip through HBM
// and the level launches of the free-running form go away.
// Staging (the k_leaf_lock_sc scheme): block b of slot i of the wave's 64
// lanes is DMA'd into the wave's 9 KB of LDS, the 9 16-B units covering each
// lane's 136-B block flattened U = 9 m + u (consecutive lanes on consecutive
// units of one deposit).  Deposit DPT m + i starts 8 (i & 1) bytes into a
// 16-B unit (280 = 17.5 x 16, DPT even), so lane m's 17 words sit at byte
// 144 m + 8 ((i + b) & 1) of the image.  Block 1 of slot i is in flight
// during block 0's permutation, block 0 of slot i + 1 (or of the next group)
// during block 1's; the 8-B tail words are loaded per lane one slot ahead.
// Whole groups only (the host runs the rest with k_keccak_rec + k_trie_level).
// global_load_lds policy of the deposit DMA: 0 (nt = 2: +0.7 % on the
// pipelined stream, profiles/r05/c5_front_ab/)
#define MK_TRIE_LOCK_AUX 0
// The next block's 9-unit DMA goes out in parts spread over the current
// block's permutation: units 0-2, 3-5, 6-8 after rounds MK_TRIE_DMA_SPLIT,
// MK_TRIE_DMA_SPLIT3 and MK_TRIE_DMA_ROUND (SPLIT3 = 0: units 0-4 / 5-8
// after SPLIT / ROUND; SPLIT = 0: all after ROUND).  Issued all at once, 16
// waves' DMA instructions burst together and the locked waves wait on the
// slowest issue.  One process A/B (profiles/r05/c5_front_ab/ab_dma_split*.txt,
// 9 interleaved rounds each, two boxes): pipelined stream 0.4086 -> 0.4017
// and 0.4163 -> 0.4092 ms/step (4/10/16 against all after 12), one trie
// 0.543 -> 0.515 and 0.561 -> 0.534 ms; two parts -1.1 %, one unit per round
// or two -0.4 to -1.1 %.
#define MK_TRIE_DMA_SPLIT 4
#define MK_TRIE_DMA_SPLIT3 10
// round of a block's permutation after which the next block's DMA (its last
// part) goes out; as one part: 12 (mid-permutation) over 0, one trie 1.2-2.3
// % faster on two boxes (profiles/r04/trie_dma_ab/); in three parts: 16
#define MK_TRIE_DMA_ROUND 16

// PIPE (a stream of tries, pipeline.TriePipeline): workgroup b also takes the
// previous trie's subtree over its level-2 nodes [1024 b, 1024 b + 1024) up
// to level 7: 512 + 256 + 128 + 64 + 32 node permutations.  Each wave does
// ONE of them (level 3 on waves 0-7, 4 on 8-11, 5 on 12-13, 6 on 14, 7 on
// 15, one node per lane) as an extra lock-step permutation inserted into its
// own sequence, so every wave runs 16 permutations and the same barriers; a
// level is inserted at least one whole permutation after the level it reads
// was stored (slots 0, 3, 7, 10, 15: between deposits, where no state is
// live), through L2 (same CU, lines it never read).  The 15 per-thread permutations of the front cost 15 slots alone;
// the previous trie's wide top levels cost one more instead of a separate
// latency-bound pass beside the front.
template <uint32_t NT, int DPT, bool PIPE>
__global__ __launch_bounds__(NT, 1) void k_trie_rec_lock(const uint2* __restrict__ in, uint64_t ngroups,
                                                         uint4* __restrict__ L0, uint4* __restrict__ L1,
                                                         uint4* __restrict__ L2, uint4* __restrict__ L3,
                                                         TriePrev prev) {
    static_assert(!PIPE || (NT == 1024 && DPT == 4), "the previous-trie slots assume 16 waves x 4 deposits");
    constexpr uint32_t NW = 35;  // 8-B words per deposit
    constexpr int NLV = DPT == 8 ? 3 : DPT == 4 ? 2 : 1;
    static_assert(DPT == 2 || DPT == 4 || DPT == 8, "deposits per thread");
    __shared__ uint4 buf[NT / 64][9 * 64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint4* Bw = buf[wave];
    uint4* const lv[4] = {L0, L1, L2, L3};
    auto first = [&](uint64_t g) { return (g * NT + 64 * wave) * DPT; };  // lane 0's first deposit
    // units [k0, k1) of the 9 (MK_TRIE_DMA_SPLIT: issued in two parts)
    auto dma = [&](uint64_t g, int i, int b, int k0 = 0, int k1 = 9) {
        const uint8_t* region = reinterpret_cast<const uint8_t*>(in + first(g) * NW);
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));  // recompute the offsets here (see lock_dma_c)
#pragma unroll
        for (int k = k0; k < k1; ++k) {
            const uint32_t U = 64u * k + ln;
            const uint32_t m = U / 9, u = U - m * 9;
            const uint32_t start = (DPT * m + i) * (8 * NW) + 136 * b;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(region + (start & ~15u) + 16 * u),
                                             (__attribute__((address_space(3))) void*)(Bw + 64 * k), 16, 0,
                                             MK_TRIE_LOCK_AUX);
        }
    };
    // a node is stored after the next slot's first wait, so no wait covers a
    // store issued just before it (stores count in vmcnt)
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
    uint4* qp = nullptr;
    auto flush = [&] {
        if (qp) {
            qp[0] = q0;
            qp[1] = q1;
        }
    };
    // the previous trie's level k node of this lane (waves of level k only)
    const uint32_t wv = __builtin_amdgcn_readfirstlane(wave);
    auto prev_slot = [&](int k) {
        const uint32_t w0 = 16u - (16u >> (k - 3)), per = 512u >> (k - 3);  // first wave, nodes per workgroup
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));  // computed here, not hoisted and kept live across the loop
        const uint32_t j = 64u * (wv - w0) + ln;
        const bool act = prev.live && j < per;
        const uint32_t jg = blockIdx.x * per + j;  // < 2^19: 32-bit offsets from the uniform bases
        const uint4* src = k == 3 ? prev.l2 : prev.l[k - 4];
        asm volatile("" ::: "memory");
        State s;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 v = act ? src[4 * jg + q] : make_uint4(0, 0, 0, 0);
            s.lo[2 * q] = v.x;
            s.hi[2 * q] = v.y;
            s.lo[2 * q + 1] = v.z;
            s.hi[2 * q + 1] = v.w;
        }
#pragma unroll
        for (int w = 8; w < 25; ++w) s.lo[w] = s.hi[w] = 0;
        s.lo[8] = 1u;  // byte 64
        s.hi[16] = 0x80000000u;
        keccak_f_digest_lock(s);
        if (act) {
            uint4 d0, d1;
            digest(s, d0, d1);
            prev.l[k - 3][2 * jg] = d0;
            prev.l[k - 3][2 * jg + 1] = d1;
        }
        asm volatile("" ::: "memory");
    };
    // Absorb lane m's staged block (17 8-B words) into s (XOR; SET: assign)
    // from its 9 16-B units, read as rows at the odd stride 9 (conflict-free
    // ds_read_b128: a b64 read of 8 B from each lane's own 16-B unit needs two
    // LDS cycles per 32 lanes whatever the layout).  The block starts `o8`
    // words (0 or 1, wave-uniform) into unit 0, so word w is half (w + o8) & 1
    // of unit (w + o8) / 2: one select per dword, every state index static
    // (the slot loop stays rolled).  Units are consumed one at a time (a
    // compiler fence between) so few data VGPRs are live beside the state.
    // Returns word 17 (the word after the block when o8 = 0).
    auto absorb = [&](State& st, uint32_t o8, auto setc) {
        constexpr bool SET = decltype(setc)::value;
        const bool sh = o8 != 0;
        uint4 prev = Bw[9 * lane];
        uint2 w17 = make_uint2(0, 0);
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            // words 2k and 2k + 1: unshifted (x, y) (z, w) of unit k; shifted
            // (z, w) of unit k and (x, y) of unit k + 1
            const uint4 cur = k + 1 < 9 ? Bw[9 * lane + k + 1] : make_uint4(0, 0, 0, 0);
            const uint32_t a0 = sh ? prev.z : prev.x, a1 = sh ? prev.w : prev.y;
            const uint32_t b0 = sh ? cur.x : prev.z, b1 = sh ? cur.y : prev.w;
            const int wa = 2 * k, wb = 2 * k + 1;
            st.lo[wa] = SET ? a0 : st.lo[wa] ^ a0;
            st.hi[wa] = SET ? a1 : st.hi[wa] ^ a1;
            if (wb < 17) {
                st.lo[wb] = SET ? b0 : st.lo[wb] ^ b0;
                st.hi[wb] = SET ? b1 : st.hi[wb] ^ b1;
            } else {
                w17 = make_uint2(prev.z, prev.w);
            }
            prev = cur;
            asm volatile("" ::: "memory");
        }
        return w17;
    };
    using Set = std::true_type;
    using Xor = std::false_type;
    uint64_t g = blockIdx.x;
    if (g < ngroups) dma(g, 0, 0);
#pragma unroll 1
    for (; g < ngroups; g += gridDim.x) {
        const uint64_t gn = g + gridDim.x;
        const uint64_t r0 = first(g) + DPT * lane;  // this lane's first deposit (leaf index)
        uint4 kl0[NLV], kl1[NLV];                   // the pending left node of each level
#pragma unroll
        for (int i = 0; i < DPT; ++i) {
            // the previous trie's slots sit between deposits (no state live)
            if (PIPE && i == 0 && wv < 8) prev_slot(3);                // slot 0
            if (PIPE && i == 1 && (wv >> 2) == 2) prev_slot(4);        // slot 3
            if (PIPE && i == 2 && (wv == 12 || wv == 13)) prev_slot(5);  // slot 7
            if (PIPE && i == 3 && wv == 14) prev_slot(6);              // slot 10
            State s;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // block 0 landed
            flush();
            qp = nullptr;
            absorb(s, i & 1, Set{});
#pragma unroll
            for (int w = 17; w < 25; ++w) s.lo[w] = s.hi[w] = 0;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // rows read: block 1 may land
            if constexpr (MK_TRIE_DMA_SPLIT3 > 0)
                keccak_f_lock_mid3<MK_TRIE_DMA_SPLIT, MK_TRIE_DMA_SPLIT3, MK_TRIE_DMA_ROUND>(
                    s, [&] { dma(g, i, 1, 0, 3); }, [&] { dma(g, i, 1, 3, 6); }, [&] { dma(g, i, 1, 6, 9); });
            else if constexpr (MK_TRIE_DMA_SPLIT > 0)
                keccak_f_lock_mid2<MK_TRIE_DMA_SPLIT, MK_TRIE_DMA_ROUND>(s, [&] { dma(g, i, 1, 0, 5); },
                                                                         [&] { dma(g, i, 1, 5, 9); });
            else
                keccak_f_lock_mid<MK_TRIE_DMA_ROUND>(s, [&] { dma(g, i, 1); });
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // block 1 landed
            // the 8-B tail word (deposit bytes 272..279): an odd slot's block 1
            // image ends with it (the block starts 16-B aligned, 9 units = 144
            // B); an even slot's is the first word of the NEXT slot's block 0
            // image (that deposit starts 8 B into the unit holding it), read
            // after its DMA lands below -- no per-lane load of its own
            // an odd slot's block 1 starts 16-B aligned and ends with the tail word
            uint2 tl = absorb(s, (i + 1) & 1, Xor{});
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            auto next_dma = [&](int k0, int k1) {
                if (i + 1 < DPT)
                    dma(g, i + 1, 0, k0, k1);
                else if (gn < ngroups)
                    dma(gn, 0, 0, k0, k1);
            };
            if constexpr (MK_TRIE_DMA_SPLIT3 > 0)
                keccak_f_lock_mid3<MK_TRIE_DMA_SPLIT, MK_TRIE_DMA_SPLIT3, MK_TRIE_DMA_ROUND>(
                    s, [&] { next_dma(0, 3); }, [&] { next_dma(3, 6); }, [&] { next_dma(6, 9); });
            else if constexpr (MK_TRIE_DMA_SPLIT > 0)
                keccak_f_lock_mid2<MK_TRIE_DMA_SPLIT, MK_TRIE_DMA_ROUND>(s, [&] { next_dma(0, 5); },
                                                                         [&] { next_dma(5, 9); });
            else
                keccak_f_lock_mid<MK_TRIE_DMA_ROUND>(s, [&] { next_dma(0, 9); });
            if (!(i & 1)) {  // slot i + 1 < DPT of this group: its block 0 holds the tail
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const uint4 v = Bw[9 * lane];
                tl = make_uint2(v.x, v.y);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
            s.lo[0] ^= tl.x;  // word 34, then the domain pad byte (word 35 = lane 1)
            s.hi[0] ^= tl.y;
            s.lo[1] ^= 1u;
            s.hi[16] ^= 0x80000000u;
            keccak_f_digest_lock(s);
            uint4 d0, d1;
            digest(s, d0, d1);
            // fold: level l + 1 gets a node once slot i closes a pair at level l
            uint4* dst = lv[0] + 2 * (r0 + i);
#pragma unroll
            for (int l = 0; l <= NLV; ++l) {
                if (l == NLV || ((i >> l) & 1) == 0) {
                    if (l < NLV) {
                        kl0[l] = d0;
                        kl1[l] = d1;
                    }
                    q0 = d0;  // stored after the next wait
                    q1 = d1;
                    qp = dst;
                    break;
                }
                dst[0] = d0;  // covered by the node permutation below
                dst[1] = d1;
                hash_node_lock(kl0[l], kl1[l], d0, d1, d0, d1);
                dst = lv[l + 1] + 2 * ((r0 + i) >> (l + 1));
            }
        }
        if (PIPE && wv == 15) prev_slot(7);  // slot 15
    }
    flush();
}
template __global__ void k_trie_rec_lock<1024, 4, true>(const uint2*, uint64_t, uint4*, uint4*, uint4*, uint4*,
                                                        TriePrev);

// Slot-major form of the whole-trie front (round 6, the verdict's A/B; the
// one-trie front since, profiles/r06/c5_slot_major/): lane m of wave w hashes deposits base + 64 i + m
// (slot i = 0..3, base = the wave's first of 256), so a DMA phase reads 64
// consecutive deposits and the lines two consecutive deposits share are
// fetched by adjacent parts, where the row form fetches every fourth such
// line seven phases apart.  The blocks are staged and read exactly as in
// k_trie_rec_lock (9 units per lane, rows at stride 9), with the 8-B offset
// now per lane (deposit parity = lane parity).  An even lane's tail word is
// the first word of the NEXT lane's block-0 image (read before block 1's
// copy lands); an odd lane's block-1 image ends with it.  Leaves sit in
// consecutive lanes, so the folds move them with ds_bpermute: after slots 1
// and 3 one locked permutation hashes the 64 level-1 nodes of the two slots
// (lane m: slot pair half m >> 5, pair m & 31), after slot 3 one more the 64
// level-2 nodes (lane m: level-1 nodes 2m, 2m + 1) -- 15 locked permutations
// per thread, as in the row form; levels 0-2 are stored as consecutive
// nodes per wave.
#if MK_TOP_STAMPS
// diagnostic build only (tools/top_probe.hip): s_memrealtime at the start and
// the end of each workgroup of the slot-major front
__device__ uint64_t g_front_stamps[2 * 1024];
#endif
template <uint32_t NT>
__global__ __launch_bounds__(NT, 1) void k_trie_rec_lock_sm(const uint2* __restrict__ in, uint64_t ngroups,
                                                            uint4* __restrict__ L0, uint4* __restrict__ L1,
                                                            uint4* __restrict__ L2) {
#if MK_TOP_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_front_stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif
    constexpr uint32_t NW = 35;  // 8-B words per deposit
    __shared__ uint4 buf[NT / 64][9 * 64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint4* Bw = buf[wave];
    auto first = [&](uint64_t g) { return (g * NT + 64 * wave) * 4; };  // the wave's first deposit
    // units [k0, k1) of slot i's block b (the slot's 64 deposits start 16-B aligned)
    auto dma = [&](uint64_t g, int i, int b, int k0, int k1) {
        const uint8_t* region = reinterpret_cast<const uint8_t*>(in + (first(g) + 64u * i) * NW);
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int k = k0; k < k1; ++k) {
            const uint32_t U = 64u * k + ln;
            const uint32_t m = U / 9, u = U - m * 9;
            const uint32_t start = m * (8 * NW) + 136 * b;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(region + (start & ~15u) + 16 * u),
                                             (__attribute__((address_space(3))) void*)(Bw + 64 * k), 16, 0,
                                             MK_TRIE_LOCK_AUX);
        }
    };
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;  // a node stored after the next wait
    uint4* qp = nullptr;
    auto flush = [&] {
        if (qp) {
            qp[0] = q0;
            qp[1] = q1;
        }
        qp = nullptr;
    };
    // 17 words of this lane's staged block into st (rows at stride 9; the
    // block starts o8 words into unit 0); returns word 17
    auto absorb = [&](State& st, uint32_t o8, auto setc) {
        constexpr bool SET = decltype(setc)::value;
        const bool sh = o8 != 0;
        uint4 prev = Bw[9 * lane];
        uint2 w17 = make_uint2(0, 0);
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const uint4 cur = k + 1 < 9 ? Bw[9 * lane + k + 1] : make_uint4(0, 0, 0, 0);
            const uint32_t a0 = sh ? prev.z : prev.x, a1 = sh ? prev.w : prev.y;
            const uint32_t b0 = sh ? cur.x : prev.z, b1 = sh ? cur.y : prev.w;
            const int wa = 2 * k, wb = 2 * k + 1;
            st.lo[wa] = SET ? a0 : st.lo[wa] ^ a0;
            st.hi[wa] = SET ? a1 : st.hi[wa] ^ a1;
            if (wb < 17) {
                st.lo[wb] = SET ? b0 : st.lo[wb] ^ b0;
                st.hi[wb] = SET ? b1 : st.hi[wb] ^ b1;
            } else {
                w17 = make_uint2(prev.z, prev.w);
            }
            prev = cur;
            asm volatile("" ::: "memory");
        }
        return w17;
    };
    // node (x, y of two uint4) of lane `src` (8 bpermutes)
    auto bperm8 = [](uint32_t src, const uint4& a, const uint4& b, uint4& ra, uint4& rb) {
        const int ad = (int)(4u * src);
        ra.x = (uint32_t)__builtin_amdgcn_ds_bpermute(ad, (int)a.x);
        ra.y = (uint32_t)__builtin_amdgcn_ds_bpermute(ad, (int)a.y);
        ra.z = (uint32_t)__builtin_amdgcn_ds_bpermute(ad, (int)a.z);
        ra.w = (uint32_t)__builtin_amdgcn_ds_bpermute(ad, (int)a.w);
        rb.x = (uint32_t)__builtin_amdgcn_ds_bpermute(ad, (int)b.x);
        rb.y = (uint32_t)__builtin_amdgcn_ds_bpermute(ad, (int)b.y);
        rb.z = (uint32_t)__builtin_amdgcn_ds_bpermute(ad, (int)b.z);
        rb.w = (uint32_t)__builtin_amdgcn_ds_bpermute(ad, (int)b.w);
    };
    auto sel4 = [](bool c, const uint4& a, const uint4& b) {
        return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
    };
    // level-1 nodes of slots (i0, i0 + 1) from their leaves in (xa, ya) / (xb, yb):
    // lane m hashes pair m & 31 of slot i0 + (m >> 5)
    auto level1 = [&](const uint4& xa, const uint4& ya, const uint4& xb, const uint4& yb, uint4& n0, uint4& n1) {
        const uint32_t p = lane & 31u;
        const bool hi_half = lane >= 32u;
        uint4 la0, la1, lb0, lb1, ra0, ra1, rb0, rb1;
        bperm8(2 * p, xa, ya, la0, la1);
        bperm8(2 * p, xb, yb, lb0, lb1);
        bperm8(2 * p + 1, xa, ya, ra0, ra1);
        bperm8(2 * p + 1, xb, yb, rb0, rb1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        hash_node_lock(sel4(hi_half, lb0, la0), sel4(hi_half, lb1, la1), sel4(hi_half, rb0, ra0),
                       sel4(hi_half, rb1, ra1), n0, n1);
    };
    using Set = std::true_type;
    using Xor = std::false_type;
    uint64_t g = blockIdx.x;
    if (g < ngroups) {
        dma(g, 0, 0, 0, 9);
    }
#pragma unroll 1
    for (; g < ngroups; g += gridDim.x) {
        const uint64_t gn = g + gridDim.x;
        const uint64_t base = first(g);
        uint4 xa = make_uint4(0, 0, 0, 0), ya = xa;  // leaf of the even slot of a pair
        uint4 n10 = xa, n11 = xa;                    // level-1 node of slots 0, 1
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            State s;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // block 0 landed
            flush();
            // an even lane's tail word: the first word of the next lane's block-0 image
            uint2 te = make_uint2(0, 0);
            if (!(lane & 1u)) {
                const uint4 v = Bw[9 * (lane + 1)];
                te = make_uint2(v.x, v.y);
            }
            absorb(s, lane & 1u, Set{});
#pragma unroll
            for (int w = 17; w < 25; ++w) s.lo[w] = s.hi[w] = 0;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // rows read: block 1 may land
            keccak_f_lock_mid3<MK_TRIE_DMA_SPLIT, MK_TRIE_DMA_SPLIT3, MK_TRIE_DMA_ROUND>(
                s, [&] { dma(g, i, 1, 0, 3); }, [&] { dma(g, i, 1, 3, 6); }, [&] { dma(g, i, 1, 6, 9); });
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // block 1 landed
            const uint2 to = absorb(s, (lane + 1) & 1u, Xor{});
            const uint2 tl = (lane & 1u) ? to : te;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            auto next_dma = [&](int k0, int k1) {
                if (i + 1 < 4)
                    dma(g, i + 1, 0, k0, k1);
                else if (gn < ngroups)
                    dma(gn, 0, 0, k0, k1);
            };
            keccak_f_lock_mid3<MK_TRIE_DMA_SPLIT, MK_TRIE_DMA_SPLIT3, MK_TRIE_DMA_ROUND>(
                s, [&] { next_dma(0, 3); }, [&] { next_dma(3, 6); }, [&] { next_dma(6, 9); });
            s.lo[0] ^= tl.x;  // word 34, then the domain pad byte
            s.hi[0] ^= tl.y;
            s.lo[1] ^= 1u;
            s.hi[16] ^= 0x80000000u;
            keccak_f_digest_lock(s);
            uint4 d0, d1;
            digest(s, d0, d1);
            uint4* leaf = L0 + 2 * (base + 64u * i + lane);
            if (!(i & 1)) {
                xa = d0;
                ya = d1;
                q0 = d0;  // stored after the next wait
                q1 = d1;
                qp = leaf;
            } else {
                leaf[0] = d0;  // covered by the node permutation below
                leaf[1] = d1;
                uint4 n0, n1;
                level1(xa, ya, d0, d1, n0, n1);
                uint4* nd = L1 + 2 * (base / 2 + 64u * (i >> 1) + lane);
                if (i == 1) {
                    n10 = n0;
                    n11 = n1;
                    q0 = n0;
                    q1 = n1;
                    qp = nd;
                } else {
                    nd[0] = n0;
                    nd[1] = n1;
                    // level 2: lane m hashes level-1 nodes 2m, 2m + 1 (of slots 0-1
                    // for m < 32, of slots 2-3 after)
                    const bool hi_half = lane >= 32u;
                    const uint32_t src = (2u * lane) & 63u;
                    uint4 la0, la1, lb0, lb1, ra0, ra1, rb0, rb1;
                    bperm8(src, n10, n11, la0, la1);
                    bperm8(src, n0, n1, lb0, lb1);
                    bperm8(src + 1, n10, n11, ra0, ra1);
                    bperm8(src + 1, n0, n1, rb0, rb1);
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    uint4 m0, m1;
                    hash_node_lock(sel4(hi_half, lb0, la0), sel4(hi_half, lb1, la1), sel4(hi_half, rb0, ra0),
                                   sel4(hi_half, rb1, ra1), m0, m1);
                    q0 = m0;
                    q1 = m1;
                    qp = L2 + 2 * (base / 4 + lane);
                }
            }
        }
    }
    flush();
#if MK_TOP_STAMPS
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_front_stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
#endif
}
template __global__ void k_trie_rec_lock_sm<1024>(const uint2*, uint64_t, uint4*, uint4*, uint4*);

// ----------------------------------------------------------------------------
// Deposit trie level: node j = K(in[2j] || (2j+1 < cin ? in[2j+1] : 0^32)),
// the map-miss-reads-zero rule of deposit_trie.go:35-37.
#define MK_TRIE_LEVEL_WAVES 1
__global__ __launch_bounds__(256, MK_TRIE_LEVEL_WAVES) void k_trie_level(const uint4* __restrict__ in, uint64_t cin,
                                                                        uint4* __restrict__ out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t cout = (cin + 1) / 2;
    if (j >= cout) return;
    const uint4 l0 = in[4 * j], l1 = in[4 * j + 1];
    uint4 r0 = make_uint4(0, 0, 0, 0), r1 = r0;
    if (2 * j + 1 < cin) {
        r0 = in[4 * j + 2];
        r1 = in[4 * j + 3];
    }
    uint4 d0, d1;
    hash_pair(l0, l1, r0, r1, false, d0, d1);
    out[2 * j] = d0;
    out[2 * j + 1] = d1;
}

// Batched VerifyMerkleBranch (deposit_trie.go:68-81): thread i folds its
// `depth` siblings into leaf i and compares with root i.
__global__ __launch_bounds__(256) void k_verify_branches(const uint4* __restrict__ leaves, const uint4* __restrict__ branches,
                                                         const uint64_t* __restrict__ indices, uint32_t depth,
                                                         uint32_t tree_depth, const uint4* __restrict__ roots,
                                                         uint64_t n, uint8_t* __restrict__ ok) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t idx = indices[i] + (tree_depth >= 64 ? 0ull : (1ull << tree_depth));
    uint4 v0 = leaves[2 * i], v1 = leaves[2 * i + 1];
    const uint4* br = branches + 2 * (uint64_t)depth * i;
    for (uint32_t d = 0; d < depth; ++d) {
        const uint4 b0 = br[2 * d], b1 = br[2 * d + 1];
        if (idx & 1)
            hash_pair(b0, b1, v0, v1, false, v0, v1);
        else
            hash_pair(v0, v1, b0, b1, false, v0, v1);
        idx >>= 1;
    }
    const uint4 r0 = roots[2 * i], r1 = roots[2 * i + 1];
    ok[i] = (v0.x == r0.x && v0.y == r0.y && v0.z == r0.z && v0.w == r0.w && v1.x == r1.x && v1.y == r1.y &&
             v1.z == r1.z && v1.w == r1.w);
}

// ----------------------------------------------------------------------------
// Synthetic SplitMix64 stream: word k = mix(seed + k*gamma),
// byte b of the stream = byte b%8 (LE) of word b/8.  Writes words
// [word0, word0 + nwords) to dst.  Identical to oracle/merkle_ref.c.
__device__ __forceinline__ uint64_t splitmix(uint64_t seed, uint64_t k) {
    uint64_t z = seed + k * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_synth(uint64_t* __restrict__ dst, uint64_t nwords, uint64_t seed, uint64_t word0) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nwords; k += stride)
        dst[k] = splitmix(seed, word0 + k);
}


// ----------------------------------------------------------------------------
// Incremental deposit trie (UpdateDepositTrie, deposit_trie.go:29-40, for a
// batch of appended leaves): level d0 of the level array already holds the
// new nodes [lo, c) (c = count at d0 after the append).  For every level d0+1
// .. depth the workgroup recomputes the right edge [lo/2, ceil(c/2)) with
// node = K(left || right), a missing right child read as 0^32 (map miss).
// The only child left of the changed range (index lo-1 when lo is odd) is
// old and read from the level array; the changed children are carried from
// level to level in LDS (bit-interleaved lane pairs, mk::ilv).  One
// workgroup, one parent per lane pair: the host keeps c - lo <= NT - 4.
// Level d starts at node trie_level_off(cap, d) = sum_{i<d} ceil(cap/2^i).
template <uint32_t NT>
__global__ __launch_bounds__(NT) void k_trie_append(uint32_t* __restrict__ levels, uint64_t cap, uint32_t d0,
                                                    uint64_t lo, uint64_t c, uint32_t d_end, uint32_t depth,
                                                    uint32_t* __restrict__ root_out) {
    constexpr uint32_t kPairs = NT / 2;
    __shared__ uint32_t lds[2][8 * kPairs];
    const uint32_t tid = threadIdx.x, k = tid >> 1, p = tid & 1u;
    uint64_t off = 0, capd = cap;  // node offset and capacity of level d0
    for (uint32_t i = 0; i < d0; ++i) {
        off += capd;
        capd = (capd + 1) / 2;
    }
    int buf = 0;
    for (uint32_t d = d0; d < d_end; ++d) {
        const uint32_t* cur = levels + 8 * off;
        uint32_t* nxt = levels + 8 * (off + capd);
        const uint64_t plo = lo >> 1, cp = (c + 1) >> 1, np = cp - plo;
        const uint64_t j = plo + k;
        if (k < np) {
            uint32_t a[4], b[4] = {0, 0, 0, 0};
            const uint64_t il = 2 * j, ir = 2 * j + 1;
            if (d == d0 || il < lo)
                load_node3(cur, il, false, p, a);
            else
#pragma unroll
                for (int w = 0; w < 4; ++w) a[w] = lds[buf][8 * (il - lo) + 2 * w + p];
            if (ir < c) {
                if (d == d0)
                    load_node3(cur, ir, false, p, b);
                else
#pragma unroll
                    for (int w = 0; w < 4; ++w) b[w] = lds[buf][8 * (ir - lo) + 2 * w + p];
            }
            uint32_t h[4];
            hash_pair3(a, b, false, p, h);
#pragma unroll
            for (int w = 0; w < 4; ++w) lds[buf ^ 1][8 * k + 2 * w + p] = h[w];
            store_node3(nxt, j, false, p, h);
            if (d + 1 == depth && k == 0) store_node3(root_out, 0, false, p, h);
        }
        __syncthreads();
        buf ^= 1;
        off += capd;
        capd = (capd + 1) / 2;
        lo = plo;
        c = cp;
    }
}
template __global__ void k_trie_append<64>(uint32_t*, uint64_t, uint32_t, uint64_t, uint64_t, uint32_t, uint32_t,
                                           uint32_t*);
template __global__ void k_trie_append<256>(uint32_t*, uint64_t, uint32_t, uint64_t, uint64_t, uint32_t, uint32_t,
                                            uint32_t*);
template __global__ void k_trie_append<1024>(uint32_t*, uint64_t, uint32_t, uint64_t, uint64_t, uint32_t, uint32_t,
                                             uint32_t*);

// The narrow right edge / top of the deposit trie with ONE STATE PER WAVE
// (mk::spread, lo/hi form: ~6.3 k cycles per permutation on a lone wave
// against ~12.8 k for a lane pair, profiles/r02d/lat_probe_spread.json).
// Wave w hashes parent plo + w of every level d0 .. d_end-1 (the host
// guarantees at most NW parents per level); level d0 and the untouched left
// neighbours come from the level array, later children from LDS.  A missing
// right child is 0^32 (deposit_trie.go:33-38), so once the count is 1 the
// levels above are the zero-sibling tail.  GPU lane L holds Keccak lane i
// (mk::spread::lane_consts): lanes i < 8 load the message words (left node
// words 0-3, right node 4-7), i = 8 / 16 carry the 0x01 / 0x80 padding, and
// lanes 0..3 hold the digest.
// Keccak-256 of p[0, la) || 0^lz (a deposit, deposit_trie.go:32; a merkleHash
// window, hash.go:205-222) in spread form: per 136-B block, lane i < 17
// absorbs message word i (0x01 at byte la + lz, 0x80 at byte 135 of the
// last block).
// Result (lo, hi) on the lanes of Keccak lanes 0..3.  W8: p and len are
// 8-byte aligned, so whole words load at once.
template <bool W8>
__device__ __forceinline__ void spread_sponge(const uint8_t* __restrict__ p, uint64_t la, const spread::LaneLH& c,
                                              uint32_t& lo, uint32_t& hi, uint64_t lz = 0) {
    const uint64_t len = la + lz;  // the message is p[0, la) || 0^lz
    const uint64_t nb = len / 136 + 1;
    lo = hi = 0u;
    for (uint64_t b = 0; b < nb; ++b) {  // nb is wave-uniform
        if (c.i < 17u) {
            const uint64_t base = 136 * b + 8 * c.i;
            uint64_t v = 0;
            if (W8 && base + 8 <= la) {
                v = *reinterpret_cast<const uint64_t*>(p + base);
            } else {
                for (uint32_t k = 0; k < 8; ++k) {
                    const uint64_t o = base + k;
                    const uint64_t byte = o < la ? p[o] : 0u;
                    v |= byte << (8 * k);
                }
            }
            if (len >= base && len < base + 8) v |= 1ull << (8 * (len - base));
            if (b + 1 == nb && c.i == 16u) v |= 0x8000000000000000ull;
            lo ^= (uint32_t)v;
            hi ^= (uint32_t)(v >> 32);
        }
        spread::keccak_f_lh(lo, hi, c);
    }
}

template <uint32_t NW>
__global__ __launch_bounds__(64 * NW) void k_trie_spread(uint32_t* __restrict__ levels, uint64_t cap, uint32_t d0,
                                                         uint64_t lo, uint64_t c, uint32_t d_end, uint32_t depth,
                                                         uint32_t* __restrict__ root_out, SpreadLeaves lv) {
    if constexpr (MK_TRIE_TOP_PRIO > 0) __builtin_amdgcn_s_setprio(MK_TRIE_TOP_PRIO);
    __shared__ uint2 lds[2][4 * NW];
    const uint32_t w = threadIdx.x >> 6, L = threadIdx.x & 63u;
    const spread::LaneLH cst = spread::lane_consts_lh(L);
    const uint32_t i = cst.i;
    if (w < lv.k) {  // wave w hashes new deposit w into level-0 node lo + w (d0 == 0)
        const uint64_t a = lv.offs ? lv.offs[w] : (uint64_t)w * lv.fixed_len;
        const uint64_t len = lv.offs ? lv.offs[w + 1] - a : lv.fixed_len;
        uint32_t hlo, hhi;
        if (lv.aligned8)
            spread_sponge<true>(lv.data + a, len, cst, hlo, hhi);
        else
            spread_sponge<false>(lv.data + a, len, cst, hlo, hhi);
        if (L < 4u) reinterpret_cast<uint2*>(levels)[4 * (lo + w) + L] = make_uint2(hlo, hhi);
    }
    __syncthreads();
    uint64_t off = 0, capd = cap;  // node offset and capacity of level d0
    for (uint32_t k = 0; k < d0; ++k) {
        off += capd;
        capd = (capd + 1) / 2;
    }
    int buf = 0;
    for (uint32_t d = d0; d < d_end; ++d) {
        const uint2* cur = reinterpret_cast<const uint2*>(levels) + 4 * off;
        uint2* nxt = reinterpret_cast<uint2*>(levels) + 4 * (off + capd);
        const uint64_t plo = lo >> 1, cp = (c + 1) >> 1;
        if (w < cp - plo) {  // wave-uniform: the permutation needs every lane
            const uint64_t j = plo + w;
            uint32_t slo = 0u, shi = 0u;
            if (i < 8u) {
                const uint64_t ch = 2 * j + (i >> 2);
                if (ch < c) {
                    const uint2 v = (d == d0 || ch < lo) ? cur[4 * ch + (i & 3u)] : lds[buf][4 * (ch - lo) + (i & 3u)];
                    slo = v.x;
                    shi = v.y;
                }
            }
            if (i == 8u) slo = 1u;
            if (i == 16u) shi = 0x80000000u;
            spread::keccak_f_lh(slo, shi, cst);
            if (L < 4u) {
                const uint2 h = make_uint2(slo, shi);
                lds[buf ^ 1][4 * w + L] = h;
                nxt[4 * j + L] = h;
                if (d + 1 == depth && root_out) reinterpret_cast<uint2*>(root_out)[L] = h;
            }
        }
        __syncthreads();
        buf ^= 1;
        off += capd;
        capd = (capd + 1) / 2;
        lo = plo;
        c = cp;
    }
}
template __global__ void k_trie_spread<1>(uint32_t*, uint64_t, uint32_t, uint64_t, uint64_t, uint32_t, uint32_t,
                                          uint32_t*, SpreadLeaves);
template __global__ void k_trie_spread<2>(uint32_t*, uint64_t, uint32_t, uint64_t, uint64_t, uint32_t, uint32_t,
                                          uint32_t*, SpreadLeaves);
template __global__ void k_trie_spread<4>(uint32_t*, uint64_t, uint32_t, uint64_t, uint64_t, uint32_t, uint32_t,
                                          uint32_t*, SpreadLeaves);
template __global__ void k_trie_spread<16>(uint32_t*, uint64_t, uint32_t, uint64_t, uint64_t, uint32_t, uint32_t,
                                           uint32_t*, SpreadLeaves);

// ONE deposit appended to a trie of `count` (powchain's one log at a time,
// powchain/service.go:379-386 -> UpdateDepositTrie, deposit_trie.go:29-40): the
// leaf hash and its whole path to the root on one wave as a register chain
// (lo/hi spread form).  The path's left siblings (node (count >> d) - 1 of
// level d wherever count >> d is odd; a missing right sibling is 0^32) are all
// loaded into LDS up front, so no level waits on a global load; the new node
// moves to the right half of the next message (Keccak lanes 4..7) with one
// ds_bpermute pair when it is a right child.  Every node of the path is
// stored (GenerateMerkleBranch reads them).  Replaces k_trie_spread<1> for
// k = 1 (one LDS exchange, one dependent load of a sibling and a barrier per
// level there).
__global__ __launch_bounds__(64) void k_trie_append1(uint32_t* __restrict__ levels, uint64_t cap, uint64_t count,
                                                     uint32_t depth, uint32_t* __restrict__ root_out,
                                                     SpreadLeaves lv) {
    if constexpr (MK_TRIE_TOP_PRIO > 0) __builtin_amdgcn_s_setprio(MK_TRIE_TOP_PRIO);
    __shared__ uint2 sib[64][4];
    const uint32_t L = threadIdx.x;
    const spread::LaneLH cst = spread::lane_consts_lh(L);
    const uint32_t i = cst.i;
    const uint2* lv2 = reinterpret_cast<const uint2*>(levels);
    // the path's left siblings, 4 words per level, one word per thread a pass
    for (uint32_t q = L; q < 4 * depth; q += 64) {
        const uint32_t d = q >> 2, w = q & 3u;
        uint64_t off = 0, capd = cap;
        for (uint32_t k = 0; k < d; ++k) {
            off += capd;
            capd = (capd + 1) / 2;
        }
        const uint64_t j = count >> d;
        sib[d][w] = (j & 1u) ? lv2[4 * (off + j - 1) + w] : make_uint2(0, 0);
    }
    uint32_t lo = 0u, hi = 0u;
    const uint64_t len = lv.offs ? lv.offs[1] - lv.offs[0] : lv.fixed_len;
    const uint8_t* dep = lv.data + (lv.offs ? lv.offs[0] : 0);
    if (lv.aligned8)
        spread_sponge<true>(dep, len, cst, lo, hi);
    else
        spread_sponge<false>(dep, len, cst, lo, hi);
    uint2* lvw = reinterpret_cast<uint2*>(levels);
    if (L < 4u) lvw[4 * count + L] = make_uint2(lo, hi);
    __syncthreads();  // the siblings are in LDS
    uint64_t off = 0, capd = cap;
    for (uint32_t d = 0; d < depth; ++d) {
        const uint64_t j = count >> d;
        const bool right = (j & 1u) != 0;  // wave-uniform
        // the node, from the digest lanes (Keccak lanes 0..3 = GPU lanes 0..3)
        // to Keccak lanes 4..7 when it is the right child
        uint32_t rlo = 0u, rhi = 0u;
        if (right) {
            const uint32_t src = 4u * (i >= 4u && i < 8u ? i - 4u : 0u);
            rlo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)lo);
            rhi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)hi);
        }
        uint32_t mlo = 0u, mhi = 0u;
        if (i < 4u) {
            const uint2 sv = sib[d][i];
            mlo = right ? sv.x : lo;
            mhi = right ? sv.y : hi;
        } else if (i < 8u && right) {
            mlo = rlo;
            mhi = rhi;
        }
        if (i == 8u) mlo ^= 1u;  // byte 64
        if (i == 16u) mhi ^= 0x80000000u;
        lo = mlo;
        hi = mhi;
        spread::keccak_f_lh(lo, hi, cst);
        off += capd;
        capd = (capd + 1) / 2;
        if (L < 4u) lvw[4 * (off + (j >> 1)) + L] = make_uint2(lo, hi);
    }
    if (L < 4u) reinterpret_cast<uint2*>(root_out)[L] = make_uint2(lo, hi);
}

// ----------------------------------------------------------------------------
// Fused tree tops (round 6): every level above a complete level of a tree in
// ONE launch, for the callers that build one tree at a time (one trie from
// its deposits, powchain/service.go:366-386; one state root,
// core/state/state.go:168-174), where the latency-bound levels, not the
// throughput passes, set the call's time.  Workgroup b reduces its NT nodes
// of the start level to one node log2(NT) levels up inside the workgroup --
// per level, bit-interleaved lane pairs (mk::ilv) while the parents outnumber
// the waves, one state per wave (mk::spread) after (a level of <= 16 parents
// costs one spread permutation, ~6.3 k cycles, instead of one lane-pair
// permutation, ~12.8 k) -- then publishes that node (write-through store,
// drained) and bumps an arrival counter; the LAST workgroup to arrive loads
// the published nodes and reduces them to the root.  No launch boundary, no
// narrow one-workgroup launch waiting for the wide one.

// Arrival counters of the fused tops, one per launch in flight (the host
// hands out slots round-robin, capi.cpp next_arrive_slot); zero at module
// load, and the last arriver of a launch resets its slot, so at most
// kArriveSlots fused launches may be in flight on one device.
__device__ uint32_t g_arrive[kArriveSlots];
// Diagnostic build only (tools/top_probe.hip: -DMK_TOP_STAMPS=1): s_memtime
// at each level of a fused top, per workgroup; never in the shipped library.
#ifndef MK_TOP_STAMPS
#define MK_TOP_STAMPS 0
#endif
#if MK_TOP_STAMPS
__device__ uint64_t g_top_stamps[1024 * 64];
#define TOP_STAMP(k) \
    do { if (threadIdx.x == 0) g_top_stamps[blockIdx.x * 64 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define TOP_STAMP(k) \
    do { (void)(k); } while (0)
#endif

namespace {

// ilv words (e, o) of a 64-bit lane -> its plain (lo, hi) dwords
__device__ __forceinline__ void ilv_to_plain(uint32_t e, uint32_t o, uint32_t& lo, uint32_t& hi) {
    lo = ilv::spread16(e) | (ilv::spread16(o) << 1);
    hi = ilv::spread16(e >> 16) | (ilv::spread16(o >> 16) << 1);
}

// One level of a fused top inside the workgroup (every thread calls it): the
// m <= NT nodes in lds (ilv words: node k at lds[8 k + 2 w + p]) -> ceil(m/2)
// parents at lds[8 j ..].  TRIE: K(l || r) with a missing r = 0^32, 64 B
// (deposit_trie.go:33-38); otherwise merkleHash's rule: the unpaired last
// node is K(l || 0^128), 160 B (hash.go:229-236).  The form follows the
// parent count (cycles per level measured in-kernel, tools/top_probe.hip):
//   > 256 parents: one state per lane (two waves per SIMD; 512 parents
//       ~39 k cycles, against ~44 k as lane pairs at four waves per SIMD;
//       256 parents as lane pairs at two waves per SIMD: one trie -0.6 us,
//       one state -0.9 us against one state per lane at one wave per SIMD,
//       3 interleaved rounds, profiles/r06/lane257/);
//   > NT/128: bit-interleaved lane pairs (mk::ilv: ~13 k cycles a level for
//       up to one wave per SIMD; 16 parents in one wave 12.8 k, against
//       17.8 k as 16 spread waves, four per SIMD);
//   <= NT/128 (<= two waves per SIMD): one state per wave (mk::spread).
// Each parent also goes to lane_out(j, d0, d1) (plain digest), pair_out(j,
// words, p) (ilv words of a lane pair) or wave_out(j, e, o, L) (lanes 0..3
// of the wave hold the digest's ilv words).
// parents from which a level runs one state per lane (below: lane pairs)
constexpr uint32_t kTopLaneMin = 257;
template <uint32_t NT, bool TRIE, typename LaneOut, typename PairOut, typename WaveOut>
__device__ __forceinline__ void wg_level(uint32_t* lds, uint32_t m, const spread::Lane& cst, LaneOut&& lane_out,
                                         PairOut&& pair_out, WaveOut&& wave_out) {
    const uint32_t tid = threadIdx.x, mn = (m + 1) / 2;
    const uint32_t w = tid >> 6, L = tid & 63u, i = cst.i;
    // spread form (one parent per wave): wave `sw` hashes parent `j`
    auto spread_load = [&](uint32_t j, uint32_t& e, uint32_t& o) {
        const bool right = 2 * j + 1 < m;
        e = o = 0u;
        if (i < 4u) {
            e = lds[16 * j + 2 * i];
            o = lds[16 * j + 2 * i + 1];
        } else if (i < 8u && right) {
            e = lds[16 * j + 8 + 2 * (i - 4u)];
            o = lds[16 * j + 8 + 2 * (i - 4u) + 1];
        }
    };
    auto spread_hash = [&](uint32_t j, uint32_t& e, uint32_t& o) {
        if (!TRIE && !(2 * j + 1 < m)) {  // K(l || 0^128): 160 bytes, two blocks
            spread::keccak_f(e, o, cst);
            if (i == 3u) e ^= 1u;
        } else if (i == 8u) {
            e ^= 1u;
        }
        if (i == 16u) o ^= 0x80000000u;
        spread::keccak_f(e, o, cst);
    };
    auto spread_store = [&](uint32_t j, uint32_t e, uint32_t o) {
        if (L < 4u) {
            lds[8 * j + 2 * L] = e;
            lds[8 * j + 2 * L + 1] = o;
            wave_out(j, e, o, L);
        }
    };
    if (mn > NT / 128) {
        // The unpaired last node of an odd merkleHash level is K(l || 0^128),
        // two permutations: the last wave hashes it in spread form (2 x ~7 k
        // cycles) beside the lane / pair forms' one permutation (13-20 k),
        // where as one of theirs it doubled the level (C3's registry top: the
        // 123 -> 62 and 31 -> 16 levels 29.6 k and 32.5 k cycles,
        // tools/top_probe.hip)
        const bool side = !TRIE && (m & 1u) && 2 * (mn - 1) <= NT - 64;
        const uint32_t mh = side ? mn - 1 : mn;  // parents of the lane / pair forms
        const bool sw = side && w == NT / 64 - 1;
        uint32_t e = 0u, o = 0u;
        if (sw) spread_load(mn - 1, e, o);
        if (mh >= kTopLaneMin) {  // one state per lane
            const bool act = tid < mh;
            const bool right = 2 * tid + 1 < m;
            State s;
            if (act) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    ilv_to_plain(lds[16 * tid + 2 * q], lds[16 * tid + 2 * q + 1], s.lo[q], s.hi[q]);
                    if (right)
                        ilv_to_plain(lds[16 * tid + 8 + 2 * q], lds[16 * tid + 8 + 2 * q + 1], s.lo[4 + q],
                                     s.hi[4 + q]);
                    else
                        s.lo[4 + q] = s.hi[4 + q] = 0u;
                }
            }
            __syncthreads();
            if (act) {
#pragma unroll
                for (int q = 8; q < 25; ++q) s.lo[q] = s.hi[q] = 0u;
                if (!TRIE && !right) {  // K(l || 0^128): block 1 = l || 0, block 2 = 0^24 || pad
                    keccak_f(s);
                    s.lo[3] ^= 1u;
                } else {
                    s.lo[8] ^= 1u;  // byte 64
                }
                s.hi[16] ^= 0x80000000u;
                keccak_f_digest(s);
                uint4 d0, d1;
                digest(s, d0, d1);
                const uint32_t lo4[4] = {d0.x, d0.z, d1.x, d1.z}, hi4[4] = {d0.y, d0.w, d1.y, d1.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    lds[8 * tid + 2 * q] = ilv::to_ilv(lo4[q], hi4[q], 0);
                    lds[8 * tid + 2 * q + 1] = ilv::to_ilv(lo4[q], hi4[q], 1);
                }
                lane_out(tid, d0, d1);
            }
        } else {  // lane pairs
            const uint32_t k = tid >> 1, p = tid & 1u;
            const bool act = k < mh;
            uint32_t a[4], b[4] = {0, 0, 0, 0};
            bool padded = false;
            if (act) {
                const bool right = 2 * k + 1 < m;
                padded = !TRIE && !right;
#pragma unroll
                for (int q = 0; q < 4; ++q) a[q] = lds[16 * k + 2 * q + p];
                if (right) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) b[q] = lds[16 * k + 8 + 2 * q + p];
                }
            }
            __syncthreads();
            if (act) {
                uint32_t h[4];
                hash_pair3(a, b, padded, p, h);
#pragma unroll
                for (int q = 0; q < 4; ++q) lds[8 * k + 2 * q + p] = h[q];
                pair_out(k, h, p);
            }
        }
        if (sw) {
            spread_hash(mn - 1, e, o);
            spread_store(mn - 1, e, o);
        }
    } else {  // one parent per wave
        // parent j on wave j: a workgroup's waves go to its SIMDs round-robin
        // (wave w on SIMD w mod 4), so the first 4 parents get a SIMD each
        // (parents 0..3 on waves 0, 4, 8, 12 -- one SIMD -- took 15.9 k
        // cycles a level against 7.8 k, tools/top_probe.hip, profiles/r06/single/)
        const uint32_t j = w;
        uint32_t e = 0u, o = 0u;
        if (j < mn) spread_load(j, e, o);  // wave-uniform
        __syncthreads();
        if (j < mn) {
            spread_hash(j, e, o);
            spread_store(j, e, o);
        }
    }
    __syncthreads();
}

// plain node j of `in` (32 B, `stride` nodes apart) -> lds as ilv words,
// thread t loading node t; SC1: agent-scope loads (nodes another CU
// published in this launch)
template <bool SC1>
__device__ __forceinline__ void wg_load_nodes(uint32_t* lds, const uint32_t* in, uint32_t m, uint32_t stride = 1) {
    const uint32_t t = threadIdx.x;
    if (t < m) {
        const uint64_t* q = reinterpret_cast<const uint64_t*>(in) + 4 * (uint64_t)t * stride;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint64_t v = SC1 ? __hip_atomic_load(q + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : q[w];
            lds[8 * t + 2 * w] = ilv::to_ilv((uint32_t)v, (uint32_t)(v >> 32), 0);
            lds[8 * t + 2 * w + 1] = ilv::to_ilv((uint32_t)v, (uint32_t)(v >> 32), 1);
        }
    }
    __syncthreads();
}

// node 0 of lds (ilv words) -> plain 32 B at out, by wave 0's lanes 0..3;
// SC1: a write-through store, drained, so another CU may read it after the
// arrival counter says so
template <bool SC1>
__device__ __forceinline__ void wg_store_node0(const uint32_t* lds, uint32_t* out) {
    const uint32_t tid = threadIdx.x;
    if (tid < 4u) {
        const uint32_t e = lds[2 * tid], o = lds[2 * tid + 1];
        const uint64_t v = (uint64_t)(ilv::spread16(e) | (ilv::spread16(o) << 1)) |
                           ((uint64_t)(ilv::spread16(e >> 16) | (ilv::spread16(o >> 16) << 1)) << 32);
        uint64_t* q = reinterpret_cast<uint64_t*>(out) + tid;
        if (SC1)
            __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            *q = v;
    }
    if (SC1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Arrival of this workgroup (after its published node's store drained); true
// in every thread of the last of `total` workgroups, which also resets the slot.
__device__ __forceinline__ bool wg_arrive_last(uint32_t slot, uint32_t total, uint32_t* flag) {
    if (threadIdx.x == 0) {
        const uint32_t old = __hip_atomic_fetch_add(&g_arrive[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = old + 1 == total;
        if (last) __hip_atomic_store(&g_arrive[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last ? 1u : 0u;
    }
    __syncthreads();
    return *flag != 0u;
}

}  // namespace

// The deposit trie above its complete level d0 (c0 nodes) up to the root, in
// one launch: workgroup b takes level-d0 nodes [NT b, NT b +
// NT) up to level d0 + log2(NT) (every node stored: GenerateMerkleBranch reads
// them), the last workgroup to arrive the rest, including the zero-sibling
// levels (deposit_trie.go:33-38) and the root.  grid = ceil(c0 / NT) <= NT;
// a grid of more than kTopGroup workgroups also uses the arrival slots after
// `slot`, one per group of each stage (kTopGroupSlots in all at most).
template <uint32_t NT>
__global__ __launch_bounds__(NT) void k_trie_top_fused(uint32_t* __restrict__ levels, uint64_t cap, uint64_t c0,
                                                       uint32_t d0, uint32_t depth, uint32_t* __restrict__ root_out,
                                                       uint32_t slot) {
    constexpr uint32_t kLog = NT == 1024 ? 10 : NT == 512 ? 9 : NT == 256 ? 8 : NT == 128 ? 7 : 6;
    __shared__ uint32_t lds[8 * NT];
    __shared__ uint32_t flag;
    uint64_t off = 0, capd = cap;  // node offset and capacity of level d
    for (uint32_t k = 0; k < d0; ++k) {
        off += capd;
        capd = (capd + 1) / 2;
    }
    const uint32_t dtop = depth - d0 < kLog ? depth : d0 + kLog;  // this workgroup's part ends at level dtop
    uint64_t lo = (uint64_t)blockIdx.x * NT;                      // level-d node of lds[0]
    uint32_t m = (uint32_t)(c0 - lo < NT ? c0 - lo : NT);
    wg_load_nodes<false>(lds, levels + 8 * (off + lo), m);
    uint32_t d = d0;
    const uint32_t L = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const spread::Lane cst = spread::lane_consts(L);
    uint32_t nst = 0;
    TOP_STAMP(nst++);
    auto run = [&](uint32_t d_end) {
        for (; d < d_end && m > 1; ++d) {
            TOP_STAMP(nst++);
            uint32_t* out = levels + 8 * (off + capd + (lo >> 1));  // level d + 1, this part's first parent
            wg_level<NT, true>(
                lds, m, cst,
                [&](uint32_t j, const uint4& d0, const uint4& d1) {
                    reinterpret_cast<uint4*>(out)[2 * j] = d0;
                    reinterpret_cast<uint4*>(out)[2 * j + 1] = d1;
                },
                [&](uint32_t j, const uint32_t(&h)[4], uint32_t p) { store_node3(out, j, false, p, h); },
                [&](uint32_t j, uint32_t e, uint32_t o, uint32_t L) { spread_store_digest(e, o, L, out + 8 * j); });
            m = (m + 1) / 2;
            lo >>= 1;
            off += capd;
            capd = (capd + 1) / 2;
        }
        if (d < d_end) {
            // one node left: the zero-sibling levels K(node || 0^32) as a
            // chain on wave 0, the node kept in registers as plain (lo, hi)
            // words (no LDS round trip, no barrier, no bit (de)interleave per
            // level; the lo/hi round, 6.29 k cycles a permutation against
            // 6.44 k, profiles/r02d/lat_probe_spread.json)
            const spread::LaneLH ch = spread::lane_consts_lh(L);
            const uint32_t i = ch.i;
            uint32_t lo32 = 0u, hi32 = 0u;
            if (w == 0 && i < 4u) ilv_to_plain(lds[2 * i], lds[2 * i + 1], lo32, hi32);
            for (; d < d_end; ++d) {
                TOP_STAMP(nst++);
                if (w == 0) {
                    if (i >= 4u) lo32 = hi32 = 0u;
                    if (i == 8u) lo32 ^= 1u;
                    if (i == 16u) hi32 ^= 0x80000000u;
                    spread::keccak_f_lh(lo32, hi32, ch);
                    if (L < 4u)
                        reinterpret_cast<uint2*>(levels + 8 * (off + capd + (lo >> 1)))[L] = make_uint2(lo32, hi32);
                }
                lo >>= 1;
                off += capd;
                capd = (capd + 1) / 2;
            }
            if (w == 0 && L < 4u) {
                lds[2 * L] = ilv::to_ilv(lo32, hi32, 0);
                lds[2 * L + 1] = ilv::to_ilv(lo32, hi32, 1);
            }
            __syncthreads();
        }
    };
    run(dtop);
    if (gridDim.x > 1) {
        // publish this part's node (level dtop, node blockIdx.x: already
        // stored above, again write-through) and arrive
        wg_store_node0<true>(lds, levels + 8 * (off + lo));
        TOP_STAMP(nst++);
        uint32_t parts = gridDim.x;  // nodes of level d, one published per workgroup
        uint32_t gslot = slot + 1;   // arrival slots of this stage's groups
        while (kTopGroupLog2 > 0 && parts > kTopGroup) {
            // the last of each kTopGroup workgroups of a stage takes its
            // group's nodes log2(kTopGroup) levels up, so those levels run on
            // many CUs at once, not one after another on a lone workgroup (a
            // missing right sibling is 0^32 here too)
            const uint32_t b = (uint32_t)lo;  // this workgroup's node of level d
            const uint32_t grp = b / kTopGroup, g0 = grp * kTopGroup;
            const uint32_t members = parts - g0 < kTopGroup ? parts - g0 : kTopGroup;
            const uint32_t groups = (parts + kTopGroup - 1) / kTopGroup;
            if (!wg_arrive_last(gslot + grp, members, &flag)) return;
            TOP_STAMP(nst++);
            lo = g0;
            m = members;
            wg_load_nodes<true>(lds, levels + 8 * (off + lo), m);
            run(d + kTopGroupLog2);
            wg_store_node0<true>(lds, levels + 8 * (off + lo));
            TOP_STAMP(nst++);
            gslot += groups;
            parts = groups;
        }
        if (!wg_arrive_last(slot, parts, &flag)) return;
        TOP_STAMP(nst++);
        lo = 0;
        m = parts;
        wg_load_nodes<true>(lds, levels + 8 * off, m);
    }
    run(depth);
    wg_store_node0<false>(lds, root_out);
    TOP_STAMP(nst++);
}
template __global__ void k_trie_top_fused<1024>(uint32_t*, uint64_t, uint64_t, uint32_t, uint32_t, uint32_t*,
                                                uint32_t);

// merkleHash above a complete level of one or two lists' trees, to the list
// roots with the length mix-in (hash.go:194-239), in one launch: list l's
// workgroups [wg0, wg0 + nwg) reduce 2^span_log2 nodes each by span_log2
// levels (a ragged last part keeps the odd rule at count 1: the other parts
// are even at every level below, so its count's parity is the level's),
// publish their node to `sub`, and the last to arrive reduces the nwg nodes
// to the root and mixes in the length.  Two lists (the State's registry and
// balances, hash.go:141-159): each list's last workgroup is one finisher of
// the pair block (wave3_spread_final), the second to complete hashes the
// struct root -- the two trees' latency-bound tops run side by side in one
// launch on one stream, where the "level1" schedule ran four launches on two
// streams with an event between them.
template <uint32_t NT>
__global__ __launch_bounds__(NT) void k_merkle_top_fused(MerkleTopArgs a) {
    __shared__ uint32_t lds[8 * NT];
    __shared__ uint32_t flag;
    const uint32_t li = a.nlists > 1 && blockIdx.x >= a.l[1].wg0 ? 1u : 0u;
    const MerkleTopList t = li ? a.l[1] : a.l[0];  // no dynamic index into the kernarg (scratch)
    const uint32_t b = blockIdx.x - t.wg0;
    const spread::Lane cst = spread::lane_consts(threadIdx.x & 63u);
    const uint64_t lo = (uint64_t)b << t.span_log2;
    const uint64_t span = 1ull << t.span_log2;
    uint32_t m = (uint32_t)(t.c - lo < span ? t.c - lo : span);
    wg_load_nodes<false>(lds, reinterpret_cast<const uint32_t*>(t.nodes) + 8 * lo, m);
    auto none3 = [](uint32_t, const uint4&, const uint4&) {};
    auto none_p = [](uint32_t, const uint32_t(&)[4], uint32_t) {};
    auto none_w = [](uint32_t, uint32_t, uint32_t, uint32_t) {};
    uint32_t nst = 0;
    TOP_STAMP(nst++);
    if (t.nwg > 1) {
        for (uint32_t k = 0; k < t.span_log2; ++k) {
            wg_level<NT, false>(lds, m, cst, none3, none_p, none_w);
            m = (m + 1) / 2;
            TOP_STAMP(nst++);
        }
        wg_store_node0<true>(lds, t.sub + 8 * b);
        // groups of kTopGroup parts first, as in k_trie_top_fused: the last of
        // each group takes the group's nodes log2(kTopGroup) levels up and
        // stores its node over the group's first (node idx of a stage at
        // sub[8 stride idx]).  Every group but a ragged last one is even at
        // each of those levels, so the ragged group's count has the level's
        // parity and a lone node there is the level's unpaired last node,
        // K(l || 0^128), as wg_level hashes it.
        uint32_t parts = t.nwg, stride = 1, idx = b, gslot = t.slot + 1;
        while (kTopGroupLog2 > 0 && parts > kTopGroup) {
            const uint32_t grp = idx / kTopGroup, g0 = grp * kTopGroup;
            const uint32_t members = parts - g0 < kTopGroup ? parts - g0 : kTopGroup;
            const uint32_t groups = (parts + kTopGroup - 1) / kTopGroup;
            if (!wg_arrive_last(gslot + grp, members, &flag)) return;
            m = members;
            wg_load_nodes<true>(lds, t.sub + 8 * stride * g0, m, stride);
            for (uint32_t k = 0; k < kTopGroupLog2; ++k) {
                wg_level<NT, false>(lds, m, cst, none3, none_p, none_w);
                m = (m + 1) / 2;
            }
            stride *= kTopGroup;
            idx = grp;
            wg_store_node0<true>(lds, t.sub + 8 * stride * idx);
            TOP_STAMP(nst++);
            gslot += groups;
            parts = groups;
        }
        if (!wg_arrive_last(t.slot, parts, &flag)) return;
        m = parts;
        wg_load_nodes<true>(lds, t.sub, m, stride);
        TOP_STAMP(nst++);
    }
    while (m > 1) {
        wg_level<NT, false>(lds, m, cst, none3, none_p, none_w);
        m = (m + 1) / 2;
        TOP_STAMP(nst++);
    }
    // the length mix-in K(root || le64(n) || 0^24) on wave 0 (spread form)
    const uint32_t L = threadIdx.x & 63u, i = cst.i;
    uint32_t e = 0u, o = 0u;
    if (threadIdx.x < 64) {
        if (i < 4u) {
            e = lds[2 * i];
            o = lds[2 * i + 1];
        } else if (i == 4u) {
            e = ilv::to_ilv((uint32_t)t.n_items, (uint32_t)(t.n_items >> 32), 0);
            o = ilv::to_ilv((uint32_t)t.n_items, (uint32_t)(t.n_items >> 32), 1);
        } else if (i == 8u) {
            e = 1u;
        }
        if (i == 16u) o ^= 0x80000000u;
        spread::keccak_f(e, o, cst);
    }
    if (a.nlists == 1) {
        if (threadIdx.x < 64) spread_store_digest(e, o, L, t.out);
        TOP_STAMP(nst++);
        return;
    }
    // Two lists: publish this list's root to its slot of the pair block
    // (write-through, drained) and arrive on the pair's counter; the second
    // list to arrive hashes the struct root K(root 0 || root 1) (hash.go:141-
    // 159) into pair[64..96).  Both finishers are in this launch, so an
    // arrival counter does what the epoch-tagged arrival word does between
    // two launches (wave3_spread_final), without its fences.
    __syncthreads();
    if (threadIdx.x < 64 && L < 4u) {
        lds[2 * L] = e;
        lds[2 * L + 1] = o;
    }
    __syncthreads();
    wg_store_node0<true>(lds, t.out);
    if (!wg_arrive_last(a.pair_slot, 2, &flag)) return;
    if (threadIdx.x < 64) {
        e = o = 0u;
        if (i < 8u) {  // lanes of Keccak lanes 0..3: list 0's root, 4..7: list 1's
            const uint64_t v = __hip_atomic_load(reinterpret_cast<const uint64_t*>(a.pair) + i, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            e = ilv::to_ilv((uint32_t)v, (uint32_t)(v >> 32), 0);
            o = ilv::to_ilv((uint32_t)v, (uint32_t)(v >> 32), 1);
        } else if (i == 8u) {
            e = 1u;  // byte 64
        }
        if (i == 16u) o ^= 0x80000000u;
        spread::keccak_f(e, o, cst);
        spread_store_digest(e, o, L, a.pair + 16);
    }
    TOP_STAMP(nst++);
}
template __global__ void k_merkle_top_fused<1024>(MerkleTopArgs);

// Small merkleHash leaf passes in spread form (one state per wave): a
// workgroup of 16 waves owns 16 windows; wave w hashes window w (256 B, the
// ragged last one, or one padded with 0^128: hash.go:205-222), then the
// workgroup folds them through up to 4 levels in LDS (parent w on wave w,
// K(l || r) or K(l || 0^128)), like k_wave3.  The final pass (<= 16
// windows) continues to the root and the length mix-in.  Where a tree's
// first level has few windows every wave runs nearly alone, and a window
// costs 2 x 6.3 k cycles here against 2 x 12.8 k in a lane pair.
// The body (every thread of the workgroup calls it): windows [SPAN blk,
// SPAN blk + SPAN); with STORE the pass's nodes go to a.out, else the
// workgroup's node (a.levels = 1 + log2 SPAN) is left in nodes[0..3].
template <uint32_t SPAN, bool STORE>
__device__ __forceinline__ void spread_leaf_body(const ReduceArgs& a, uint32_t w8, uint64_t blk, uint2 (&nodes)[64]) {
    static_assert(SPAN == 8 || SPAN == 16, "windows per workgroup");
    const uint32_t w = threadIdx.x >> 6, L = threadIdx.x & 63u;
    const spread::LaneLH cst = spread::lane_consts_lh(L);
    const uint32_t i = cst.i;
    const uint64_t lo1 = (a.wg_base + blk) * (uint64_t)SPAN;
    const uint64_t m1 = a.c1 - lo1 < SPAN ? a.c1 - lo1 : SPAN;
    if (w < m1) {  // wave-uniform
        const uint64_t j = lo1 + w;
        const uint64_t lo = j * 2 * a.cb;
        uint64_t la;
        uint32_t lz;
        if (2 * j + 1 < a.nchunks) {
            la = (lo + 2 * a.cb < a.total ? lo + 2 * a.cb : a.total) - lo;
            lz = 0;
        } else {
            la = a.total - lo;
            lz = 128;
        }
        uint32_t hlo, hhi;
        if (w8)
            spread_sponge<true>(a.items + lo, la, cst, hlo, hhi, lz);
        else
            spread_sponge<false>(a.items + lo, la, cst, hlo, hhi, lz);
        if (L < 4u) nodes[4 * w + L] = make_uint2(hlo, hhi);
    }
    __syncthreads();
    uint64_t c = a.c1, m = m1;
    int left = a.finalize ? 64 : (int)a.levels - 1;
    int done = 0;
    while (left > 0 && (c > 1 || a.pad_at_one)) {
        const uint64_t mn = (m + 1) / 2;
        uint32_t slo = 0u, shi = 0u;
        if (w < mn) {
            const bool padded = !(2 * (uint64_t)w + 1 < m);
            if (i < 4u) {
                const uint2 v = nodes[8 * w + i];
                slo = v.x;
                shi = v.y;
            } else if (i < 8u && !padded) {
                const uint2 v = nodes[8 * w + i];  // node 2w+1, word i-4
                slo = v.x;
                shi = v.y;
            }
            if (padded) {  // 160 bytes: two blocks
                spread::keccak_f_lh(slo, shi, cst);
                if (i == 3u) slo ^= 1u;
            } else if (i == 8u) {
                slo ^= 1u;
            }
            if (i == 16u) shi ^= 0x80000000u;
            spread::keccak_f_lh(slo, shi, cst);
        }
        __syncthreads();
        if (w < mn && L < 4u) nodes[4 * w + L] = make_uint2(slo, shi);
        __syncthreads();
        c = (c + 1) / 2;
        m = mn;
        --left;
        ++done;
    }
    uint2* out = reinterpret_cast<uint2*>(a.out);
    if (a.finalize) {
        if (w == 0) {  // K(root || le64(n) || 0^24)
            uint32_t slo = 0u, shi = 0u;
            if (i < 4u) {
                const uint2 v = nodes[i];
                slo = v.x;
                shi = v.y;
            } else if (i == 4u) {
                slo = (uint32_t)a.n_items;
                shi = (uint32_t)(a.n_items >> 32);
            } else if (i == 8u) {
                slo = 1u;
            }
            if (i == 16u) shi ^= 0x80000000u;
            spread::keccak_f_lh(slo, shi, cst);
            if (L < 4u) out[L] = make_uint2(slo, shi);
        }
    } else if (STORE && w < m && L < 4u) {
        out[4 * ((lo1 >> done) + w) + L] = nodes[4 * w + L];
    }
}
template <uint32_t SPAN>
__global__ __launch_bounds__(1024) void k_spread_leaf(ReduceArgs a, uint32_t w8) {
    __shared__ uint2 nodes[16 * 4];
    spread_leaf_body<SPAN, true>(a, w8, blockIdx.x, nodes);
}
template __global__ void k_spread_leaf<16>(ReduceArgs, uint32_t);
template __global__ void k_spread_leaf<8>(ReduceArgs, uint32_t);

// TreeHash of a small list of structs in ONE launch (round 6: C1, 16,384
// ValidatorRecords, hash.go:118-159 -> 194-239): workgroup b hashes records
// [64 b, 64 b + 64) as k_struct_split does (the fields side by side, the
// struct message on a lane pair; roots to `roots`), then their 8 windows
// and 3 levels as k_spread_leaf<8> does (one window per wave), publishes
// its node (write-through, drained) and arrives; groups of kTopGroup
// workgroups and the last one take the nodes to the list root and the
// length mix-in as k_merkle_top_fused does.  Three launches' boundaries
// and the roots' trip through a second kernel go away.  `a` is the window
// pass over `roots` (a.levels = 4); sub: one published node per workgroup.
template <int NB, int NRAW>
__global__ __launch_bounds__(1024) void k_struct_list_fused(const uint8_t* __restrict__ rec, uint64_t n, StructSpec sp,
                                                            uint32_t vec16, uint4* __restrict__ roots, ReduceArgs a,
                                                            uint32_t* __restrict__ sub, uint32_t* __restrict__ out,
                                                            uint32_t slot) {
    __shared__ uint32_t dg[NB * 8][64];
    __shared__ uint2 nodes[16 * 4];
    __shared__ uint32_t lds[8 * 1024];
    __shared__ uint32_t flag;
    constexpr uint32_t NT = 1024;
    const uint32_t b = blockIdx.x, nwg = gridDim.x;
    struct_split_body<NB, NRAW>(rec, n, sp, vec16, roots, b, dg);
    __threadfence_block();  // this workgroup's roots, read back by its own waves below
    __syncthreads();
    spread_leaf_body<8, false>(a, 1u, b, nodes);
    // publish node b: plain (lo, hi) words of lanes 0..3, write-through, drained
    if (threadIdx.x < 4u) {
        const uint2 v = nodes[threadIdx.x];
        __hip_atomic_store(reinterpret_cast<uint64_t*>(sub) + 4 * b + threadIdx.x,
                           (uint64_t)v.x | ((uint64_t)v.y << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const spread::Lane cst = spread::lane_consts(threadIdx.x & 63u);
    auto none3 = [](uint32_t, const uint4&, const uint4&) {};
    auto none_p = [](uint32_t, const uint32_t(&)[4], uint32_t) {};
    auto none_w = [](uint32_t, uint32_t, uint32_t, uint32_t) {};
    uint32_t m = 1;
    // as k_merkle_top_fused: groups of kTopGroup parts first, each group's
    // last arriver takes its nodes log2(kTopGroup) levels up (a ragged last
    // group's count has the level's parity: a lone node is the level's
    // unpaired last node, K(l || 0^128))
    uint32_t parts = nwg, stride = 1, idx = b, gslot = slot + 1;
    while (kTopGroupLog2 > 0 && parts > kTopGroup) {
        const uint32_t grp = idx / kTopGroup, g0 = grp * kTopGroup;
        const uint32_t members = parts - g0 < kTopGroup ? parts - g0 : kTopGroup;
        const uint32_t groups = (parts + kTopGroup - 1) / kTopGroup;
        if (!wg_arrive_last(gslot + grp, members, &flag)) return;
        m = members;
        wg_load_nodes<true>(lds, sub + 8 * stride * g0, m, stride);
        for (uint32_t k = 0; k < kTopGroupLog2; ++k) {
            wg_level<NT, false>(lds, m, cst, none3, none_p, none_w);
            m = (m + 1) / 2;
        }
        stride *= kTopGroup;
        idx = grp;
        wg_store_node0<true>(lds, sub + 8 * stride * idx);
        gslot += groups;
        parts = groups;
    }
    if (!wg_arrive_last(slot, parts, &flag)) return;
    m = parts;
    wg_load_nodes<true>(lds, sub, m, stride);
    while (m > 1) {
        wg_level<NT, false>(lds, m, cst, none3, none_p, none_w);
        m = (m + 1) / 2;
    }
    // the length mix-in K(root || le64(n) || 0^24) on wave 0 (spread form)
    if (threadIdx.x < 64) {
        const uint32_t L = threadIdx.x, i = cst.i;
        uint32_t e = 0u, o = 0u;
        if (i < 4u) {
            e = lds[2 * i];
            o = lds[2 * i + 1];
        } else if (i == 4u) {
            e = ilv::to_ilv((uint32_t)n, (uint32_t)(n >> 32), 0);
            o = ilv::to_ilv((uint32_t)n, (uint32_t)(n >> 32), 1);
        } else if (i == 8u) {
            e = 1u;
        }
        if (i == 16u) o ^= 0x80000000u;
        spread::keccak_f(e, o, cst);
        spread_store_digest(e, o, L, out);
    }
}
template __global__ void k_struct_list_fused<3, 6>(const uint8_t*, uint64_t, StructSpec, uint32_t, uint4*, ReduceArgs,
                                                   uint32_t*, uint32_t*, uint32_t);

// Root() after each of m deposits appended at count0 (powchain's saveInTrie
// reads Root() before every UpdateDepositTrie, service.go:379-386): wave g
// walks leaf i = count0 + g to the top in spread form.  At level d the path
// node p = i >> d is a right child (p odd: its left sibling p - 1 covers only
// leaves < i, a complete subtree, so the level array holds its final value)
// or a left child (the right sibling lies past the prefix: 0^32), so the m
// prefix roots are m independent 32-permutation chains over the level array
// the batched append left behind.  The left siblings of a chain go to LDS
// first (lane d loads level d's), then the chain runs with no global loads.
template <uint32_t NW>
__global__ __launch_bounds__(64 * NW) void k_trie_prefix_roots(const uint4* __restrict__ levels, uint64_t cap,
                                                               uint64_t count0, uint64_t m, uint32_t depth,
                                                               uint4* __restrict__ roots) {
    __shared__ uint4 sib[NW][64][2];
    const uint32_t w = threadIdx.x >> 6, L = threadIdx.x & 63u;
    const uint64_t g = (uint64_t)blockIdx.x * NW + w;
    const bool live = g < m;  // wave-uniform
    const uint64_t i = count0 + (live ? g : 0);
    if (live && L < depth && ((i >> L) & 1u)) {
        uint64_t off = 0, capd = cap;
        for (uint32_t d = 0; d < L; ++d) {
            off += capd;
            capd = (capd + 1) / 2;
        }
        const uint64_t node = off + (i >> L) - 1;
        sib[w][L][0] = levels[2 * node];
        sib[w][L][1] = levels[2 * node + 1];
    }
    __syncthreads();
    if (!live) return;
    const spread::LaneLH cst = spread::lane_consts_lh(L);
    const uint32_t ci = cst.i;
    uint32_t plo = 0u, phi = 0u;  // the path node's word ci on lanes ci < 4
    if (ci < 4u) {
        const uint2 v = reinterpret_cast<const uint2*>(levels)[4 * i + ci];
        plo = v.x;
        phi = v.y;
    }
    for (uint32_t d = 0; d < depth; ++d) {
        const bool right = ((i >> d) & 1u) != 0;  // wave-uniform
        // path words moved to Keccak lanes 4..7 (GPU lanes 0..3 hold 0..3)
        const uint32_t src = 4u * ((ci - 4u) & 3u);
        const uint32_t mlo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)plo);
        const uint32_t mhi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)phi);
        uint32_t lo = 0u, hi = 0u;
        if (ci < 4u) {
            if (right) {
                const uint4 h = sib[w][d][ci >> 1];
                lo = (ci & 1u) ? h.z : h.x;
                hi = (ci & 1u) ? h.w : h.y;
            } else {
                lo = plo;
                hi = phi;
            }
        } else if (ci < 8u && right) {
            lo = mlo;
            hi = mhi;
        } else if (ci == 8u) {
            lo = 1u;
        }
        if (ci == 16u) hi = 0x80000000u;
        spread::keccak_f_lh(lo, hi, cst);
        plo = lo;
        phi = hi;
    }
    if (L < 4u) reinterpret_cast<uint2*>(roots)[4 * g + L] = make_uint2(plo, phi);
}
template __global__ void k_trie_prefix_roots<4>(const uint4*, uint64_t, uint64_t, uint64_t, uint32_t, uint4*);

// GenerateMerkleBranch (deposit_trie.go:43-58): branch[d] = the sibling of
// index's ancestor at level d, 0^32 when that node does not exist.
__global__ void k_trie_branch(const uint4* __restrict__ levels, uint64_t cap, uint64_t count, uint32_t depth,
                              uint64_t index, uint4* __restrict__ branch) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= depth) return;
    uint64_t off = 0, capd = cap, cd = count;
    for (uint32_t i = 0; i < d; ++i) {
        off += capd;
        capd = (capd + 1) / 2;
        cd = (cd + 1) / 2;
    }
    const uint64_t sib = (index >> d) ^ 1ull;
    uint4 v0 = make_uint4(0, 0, 0, 0), v1 = v0;
    if (sib < cd) {
        v0 = levels[2 * (off + sib)];
        v1 = levels[2 * (off + sib) + 1];
    }
    branch[2 * d] = v0;
    branch[2 * d + 1] = v1;
}

// ----------------------------------------------------------------------------
// Many lists (segmented merkleHash, hash.go:194-239 per list): one launch per
// level for all lists with nodes at that level.  Thread t of the launch maps
// to (list, node j) by binary search over the level's act table (exclusive
// prefix sums of the per-list node counts).  LEAF: node j = K(window j of the
// list's chunks) (256-B contiguous windows on the streaming path, the generic
// sponge for odd item sizes and ragged / padded windows); NODE: K(n[2j] ||
// n[2j+1]) or K(n[2j] || 0^128) on an odd count.
__device__ __forceinline__ uint32_t many_find(const ManyAct* __restrict__ act, uint32_t cnt, uint64_t t) {
    uint32_t lo = 0, hi = cnt;  // act[lo].out_first <= t < act[hi].out_first
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (act[mid].out_first <= t)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

template <bool LEAF>
__global__ __launch_bounds__(256) void k_many_level(const uint8_t* __restrict__ items,
                                                    const ManyList* __restrict__ lists,
                                                    const ManyAct* __restrict__ act, uint32_t nact, uint64_t nodes,
                                                    const uint4* __restrict__ in, uint4* __restrict__ out,
                                                    uint4* __restrict__ tops) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nodes) return;
    const ManyAct A = act[many_find(act, nact, t)];
    const ManyList L = lists[A.list];
    const uint64_t j = t - A.out_first;
    uint4 d0, d1;
    if constexpr (LEAF) {
        const uint8_t* base = items + L.items_off;
        if (L.fast && j < L.total / 256) {
            hash_window256(reinterpret_cast<const uint4*>(base) + j * 16, d0, d1);
        } else {
            const uint64_t lo = j * 2 * L.cb;
            uint64_t la;
            uint32_t lz;
            if (2 * j + 1 < L.nchunks) {
                la = (lo + 2 * L.cb < L.total ? lo + 2 * L.cb : L.total) - lo;
                lz = 0;
            } else {
                la = L.total - lo;
                lz = 128;
            }
            sponge_generic(base + lo, la, lz, false, 0, d0, d1);
        }
    } else {
        const uint64_t cprev = (L.c1 + (1ull << (A.level - 2)) - 1) >> (A.level - 2);  // nodes at level - 1
        const uint4* src = in + 2 * (A.in_first + 2 * j);
        const bool padded = !(2 * j + 1 < cprev);
        uint4 r0 = make_uint4(0, 0, 0, 0), r1 = r0;
        if (!padded) {
            r0 = src[2];
            r1 = src[3];
        }
        hash_pair(src[0], src[1], r0, r1, padded, d0, d1);
    }
    if (A.level == L.levels) {  // the list's top node (its only node at this level)
        tops[2 * A.list] = d0;
        tops[2 * A.list + 1] = d1;
    } else {
        out[2 * (A.out_first + j)] = d0;
        out[2 * (A.out_first + j) + 1] = d1;
    }
}
template __global__ void k_many_level<true>(const uint8_t*, const ManyList*, const ManyAct*, uint32_t, uint64_t,
                                            const uint4*, uint4*, uint4*);
template __global__ void k_many_level<false>(const uint8_t*, const ManyList*, const ManyAct*, uint32_t, uint64_t,
                                             const uint4*, uint4*, uint4*);

// Root of every list that is not a big list: K(top || le64(n) || 0^24), or
// for <= 1 chunk K(bytes || [0^128 if n == 0] || le64(n) || 0^24).
__global__ __launch_bounds__(256) void k_many_final(const uint8_t* __restrict__ items,
                                                    const ManyList* __restrict__ lists, uint32_t nlists,
                                                    const uint4* __restrict__ tops, uint4* __restrict__ roots) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlists) return;
    const ManyList L = lists[i];
    if (L.levels == 0xFFFFFFFFu) return;  // big list: its own plan wrote the root
    uint4 d0, d1;
    if (L.levels == 0) {
        sponge_generic(items + L.items_off, L.total, L.n == 0 ? 128u : 0u, true, L.n, d0, d1);
    } else {
        hash_final(tops[2 * i], tops[2 * i + 1], L.n, d0, d1);
    }
    roots[2 * i] = d0;
    roots[2 * i + 1] = d1;
}

}  // namespace mk
