// Keccak-f[1600] for gfx950 (CDNA4), one permutation state per lane.
//
// Replaces the digest under shared/hashutil/hash.go:11-25 (legacy
// Keccak-256 from golang.org/x/crypto/sha3 @ b8fe1690c613: rate 136 B,
// pad 0x01 .. 0x80, 24 rounds).
//
// Layout: the 25 64-bit lanes live in 50 VGPRs as (lo, hi) 32-bit halves.
// Every instruction is an integer VALU op chosen for the gfx950 ISA:
//   theta column parity  2 x v_bitop3_b32 (xor3, LUT 0x96) per half
//   theta D rotation     2 x v_alignbit_b32 per column
//   theta apply          1 x v_bitop3_b32 (a ^ c[x-1] ^ rot(c[x+1])) per half
//   rho                  2 x v_alignbit_b32 per lane (no offset is 0 mod 32
//                        except lane 0, which is free)
//   pi                   register renaming (no instructions)
//   chi                  1 x v_bitop3_b32 (a ^ (~b & c), LUT 0xD2) per half
//   iota                 <= 2 x v_xor_b32 with a scalar round constant
// = 180 VALU per round, 4320 per permutation (BASELINE.md §2 op model).
// hipcc does not select bitop3/alignbit from plain C++, so
// the builtins are used explicitly.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mk {

__constant__ uint32_t kRcLo[24] = {
    0x00000001u, 0x00008082u, 0x0000808Au, 0x80008000u, 0x0000808Bu, 0x80000001u,
    0x80008081u, 0x00008009u, 0x0000008Au, 0x00000088u, 0x80008009u, 0x8000000Au,
    0x8000808Bu, 0x0000008Bu, 0x00008089u, 0x00008003u, 0x00008002u, 0x00000080u,
    0x0000800Au, 0x8000000Au, 0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
__constant__ uint32_t kRcHi[24] = {
    0x00000000u, 0x00000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x00000000u,
    0x80000000u, 0x80000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u,
    0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u,
    0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u};

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// a ^ (~b & c): LUT index = (a << 2) | (b << 1) | c  ->  0b11010010
__device__ __forceinline__ uint32_t chi3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xD2);
}
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbit(hi, lo, s);  // (hi:lo >> s)[31:0]
}

// 64-bit rotate-left by a compile-time N of the pair (lo, hi).
template <int N>
__device__ __forceinline__ void rotl64(uint32_t lo, uint32_t hi, uint32_t& olo, uint32_t& ohi) {
    if constexpr (N == 0) {
        olo = lo;
        ohi = hi;
    } else if constexpr (N == 32) {
        olo = hi;
        ohi = lo;
    } else if constexpr (N < 32) {
        ohi = funnel(hi, lo, 32 - N);
        olo = funnel(lo, hi, 32 - N);
    } else {
        ohi = funnel(lo, hi, 64 - N);
        olo = funnel(hi, lo, 64 - N);
    }
}

struct State {
    uint32_t lo[25];
    uint32_t hi[25];
};

__device__ __forceinline__ void zero(State& s) {
#pragma unroll
    for (int i = 0; i < 25; ++i) {
        s.lo[i] = 0u;
        s.hi[i] = 0u;
    }
}

// rho offsets r[x][y], lane index x + 5y
#define MK_RHO(i)                                                                          \
    ((i) == 0 ? 0 : (i) == 1 ? 1 : (i) == 2 ? 62 : (i) == 3 ? 28 : (i) == 4 ? 27          \
   : (i) == 5 ? 36 : (i) == 6 ? 44 : (i) == 7 ? 6 : (i) == 8 ? 55 : (i) == 9 ? 20          \
   : (i) == 10 ? 3 : (i) == 11 ? 10 : (i) == 12 ? 43 : (i) == 13 ? 25 : (i) == 14 ? 39    \
   : (i) == 15 ? 41 : (i) == 16 ? 45 : (i) == 17 ? 15 : (i) == 18 ? 21 : (i) == 19 ? 8    \
   : (i) == 20 ? 18 : (i) == 21 ? 2 : (i) == 22 ? 61 : (i) == 23 ? 56 : 14)

template <int I>
__device__ __forceinline__ void rho_pi_one(const State& a, uint32_t (&blo)[25], uint32_t (&bhi)[25]) {
    constexpr int x = I % 5, y = I / 5;
    constexpr int dst = y + 5 * ((2 * x + 3 * y) % 5);
    rotl64<MK_RHO(I)>(a.lo[I], a.hi[I], blo[dst], bhi[dst]);
}

template <int... Is>
__device__ __forceinline__ void rho_pi_all(const State& a, uint32_t (&blo)[25], uint32_t (&bhi)[25],
                                           std::integer_sequence<int, Is...>) {
    (rho_pi_one<Is>(a, blo, bhi), ...);
}

// The round with its instruction order fixed: one asm volatile statement per
// VALU op, phases in sequence (20 bitop3 | 10 alignbit | 50 bitop3 | 48
// alignbit | 52 bitop3/xor): four full-/half-rate class switches per round.
// The compiler's own schedule of the same C++ round interleaves the classes
// and issued ~2 % slower (tools/asm_round_probe.hip, register-resident 43.4 vs
// 42.7 T ops/s; leaf kernel 2^28: 10.35 -> 10.13 ms in one-process A/B);
// interleaving rho and chi row by row is slower still (41.7-42.1 T); fencing
// the C++ round's phases with sched_barrier did not change it.  Register
// allocation stays with the compiler.
__device__ __forceinline__ uint32_t ax3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t achi(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xd2" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
template <int S>
__device__ __forceinline__ uint32_t aalign(uint32_t hi, uint32_t lo) {
    uint32_t r;
    asm volatile("v_alignbit_b32 %0, %1, %2, %3" : "=v"(r) : "v"(hi), "v"(lo), "i"(S));
    return r;
}
__device__ __forceinline__ uint32_t axs(uint32_t a, uint32_t s) {
    uint32_t r;
    asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "s"(s), "v"(a));
    return r;
}
template <int N>
__device__ __forceinline__ void arot(uint32_t lo, uint32_t hi, uint32_t& olo, uint32_t& ohi) {
    if constexpr (N == 0) {
        olo = lo;
        ohi = hi;
    } else if constexpr (N < 32) {
        ohi = aalign<32 - N>(hi, lo);
        olo = aalign<32 - N>(lo, hi);
    } else {
        ohi = aalign<64 - N>(lo, hi);
        olo = aalign<64 - N>(hi, lo);
    }
}
template <int I>
__device__ __forceinline__ void arho(const State& a, uint32_t (&blo)[25], uint32_t (&bhi)[25]) {
    constexpr int x = I % 5, y = I / 5;
    constexpr int dst = y + 5 * ((2 * x + 3 * y) % 5);
    arot<MK_RHO(I)>(a.lo[I], a.hi[I], blo[dst], bhi[dst]);
}
template <int... Is>
__device__ __forceinline__ void arho_all(const State& a, uint32_t (&blo)[25], uint32_t (&bhi)[25],
                                         std::integer_sequence<int, Is...>) {
    (arho<Is>(a, blo, bhi), ...);
}

// BAR (phase-locked rounds, the locked kernels): an s_barrier between rho and chi.
// In a 1024-thread workgroup (4 waves per SIMD, all of one workgroup) it
// starts every round's chi with the 4 waves of each SIMD on the same
// instruction.  The round's two long full-rate runs (chi + the next
// round's parity, 72; theta apply, 50) then issue in pairs across waves at
// ~2.2 cycles per wave instruction, and the whole round at ~2.8 against 3.5-3.7
// free running (tools/replay_probe.py, profiles/r03i: the compiled round's
// exact text 56.2 vs 42.7 T ops/s).  The barrier's position is what matters:
// after iota (the round's end) the same stream runs at 3.5, before rho at 4.45.
#ifndef MK_LOCK_BARS
#define MK_LOCK_BARS 2  // 1: before chi; 2: also before theta apply (57.2 vs 51.9 T register-resident)
#endif
template <bool BAR = false>
__device__ __forceinline__ void round_asm(State& s, uint32_t rclo, uint32_t rchi) {
    uint32_t clo[5], chi_[5];
#pragma unroll
    for (int x = 0; x < 5; ++x) {
        clo[x] = ax3(s.lo[x], s.lo[x + 5], s.lo[x + 10]);
        chi_[x] = ax3(s.hi[x], s.hi[x + 5], s.hi[x + 10]);
    }
#pragma unroll
    for (int x = 0; x < 5; ++x) {
        clo[x] = ax3(clo[x], s.lo[x + 15], s.lo[x + 20]);
        chi_[x] = ax3(chi_[x], s.hi[x + 15], s.hi[x + 20]);
    }
    uint32_t rlo[5], rhi[5];
#pragma unroll
    for (int x = 0; x < 5; ++x) arot<1>(clo[x], chi_[x], rlo[x], rhi[x]);
    if constexpr (BAR && MK_LOCK_BARS >= 2) __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int i = 0; i < 25; ++i) {
        const int x = i % 5;
        s.lo[i] = ax3(s.lo[i], clo[(x + 4) % 5], rlo[(x + 1) % 5]);
        s.hi[i] = ax3(s.hi[i], chi_[(x + 4) % 5], rhi[(x + 1) % 5]);
    }
    uint32_t blo[25], bhi[25];
    arho_all(s, blo, bhi, std::make_integer_sequence<int, 25>{});
    if constexpr (BAR) __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int y = 0; y < 5; ++y) {
#pragma unroll
        for (int x = 0; x < 5; ++x) {
            const int i = x + 5 * y;
            const int i1 = (x + 1) % 5 + 5 * y, i2 = (x + 2) % 5 + 5 * y;
            s.lo[i] = achi(blo[i], blo[i1], blo[i2]);
            s.hi[i] = achi(bhi[i], bhi[i1], bhi[i2]);
        }
    }
    s.lo[0] = axs(s.lo[0], rclo);
    s.hi[0] = axs(s.hi[0], rchi);
}

__device__ __forceinline__ void round_fn(State& s, uint32_t rclo, uint32_t rchi) { round_asm(s, rclo, rchi); }

#ifndef MK_ROUND_UNROLL
#define MK_ROUND_UNROLL 2
#endif
constexpr int kRoundUnroll = MK_ROUND_UNROLL;

// The round loop is only partially unrolled: pi is a pure renaming and chi
// writes the canonical lane positions, so a rolled loop needs no moves, and
// one permutation stays ~6 KB of code instead of ~35 KB (several copies of
// it live in one kernel).  Round constants come from the scalar cache.
__device__ __forceinline__ void keccak_f(State& s) {
#pragma unroll kRoundUnroll
    for (int r = 0; r < 24; ++r) round_fn(s, kRcLo[r], kRcHi[r]);
}

// Last round when only the 32-byte digest (lanes 0..3) is read afterwards:
// chi of row 0 needs b[X,0] = rho(theta(A))[X,X] (pi maps the diagonal to
// row 0), so theta is applied to the 5 diagonal lanes only and chi computed
// for 4 lanes: 58 VALU instead of 180 (20 parity + 10 D + 10 apply + 8 rho +
// 8 chi + 2 iota).  Lanes 4..24 are left stale.
template <int X>
__device__ __forceinline__ void diag_rho(const State& s, const uint32_t (&clo)[5], const uint32_t (&chi_)[5],
                                         const uint32_t (&rlo)[5], const uint32_t (&rhi)[5], uint32_t (&blo)[5],
                                         uint32_t (&bhi)[5]) {
    constexpr int i = 6 * X;  // lane (X, X)
    const uint32_t alo = xor3(s.lo[i], clo[(X + 4) % 5], rlo[(X + 1) % 5]);
    const uint32_t ahi = xor3(s.hi[i], chi_[(X + 4) % 5], rhi[(X + 1) % 5]);
    rotl64<MK_RHO(i)>(alo, ahi, blo[X], bhi[X]);
}

__device__ __forceinline__ void last_round_digest(State& s, uint32_t rclo, uint32_t rchi) {
    uint32_t clo[5], chi_[5];
#pragma unroll
    for (int x = 0; x < 5; ++x) {
        clo[x] = xor3(xor3(s.lo[x], s.lo[x + 5], s.lo[x + 10]), s.lo[x + 15], s.lo[x + 20]);
        chi_[x] = xor3(xor3(s.hi[x], s.hi[x + 5], s.hi[x + 10]), s.hi[x + 15], s.hi[x + 20]);
    }
    uint32_t rlo[5], rhi[5];
#pragma unroll
    for (int x = 0; x < 5; ++x) rotl64<1>(clo[x], chi_[x], rlo[x], rhi[x]);
    uint32_t blo[5], bhi[5];
    diag_rho<0>(s, clo, chi_, rlo, rhi, blo, bhi);
    diag_rho<1>(s, clo, chi_, rlo, rhi, blo, bhi);
    diag_rho<2>(s, clo, chi_, rlo, rhi, blo, bhi);
    diag_rho<3>(s, clo, chi_, rlo, rhi, blo, bhi);
    diag_rho<4>(s, clo, chi_, rlo, rhi, blo, bhi);
#pragma unroll
    for (int x = 0; x < 4; ++x) {
        s.lo[x] = chi3(blo[x], blo[(x + 1) % 5], blo[(x + 2) % 5]);
        s.hi[x] = chi3(bhi[x], bhi[(x + 1) % 5], bhi[(x + 2) % 5]);
    }
    s.lo[0] ^= rclo;
    s.hi[0] ^= rchi;
}

// Final permutation of a hash: only digest(s) may read the state afterwards.
__device__ __forceinline__ void keccak_f_digest(State& s) {
#pragma unroll kRoundUnroll
    for (int r = 0; r < 22; ++r) round_fn(s, kRcLo[r], kRcHi[r]);
    round_fn(s, kRcLo[22], kRcHi[22]);
    last_round_digest(s, kRcLo[23], kRcHi[23]);
    // Pin the digest here: without a use in this block LLVM sinks the two
    // straight-line rounds towards the digest's consumer (past the next
    // window's permutations in k_reduce), keeping this state alive across
    // them (117 -> 159 VGPRs, 4 -> 3 waves/SIMD).
    asm volatile("" : "+v"(s.lo[0]), "+v"(s.hi[0]), "+v"(s.lo[1]), "+v"(s.hi[1]), "+v"(s.lo[2]), "+v"(s.hi[2]),
                 "+v"(s.lo[3]), "+v"(s.hi[3]));
}

// Phase-locked permutations (round_asm<true>): every wave of the workgroup
// must run the same number of them -- each round holds an s_barrier.
__device__ __forceinline__ void keccak_f_lock(State& s) {
#pragma unroll kRoundUnroll
    for (int r = 0; r < 24; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
}
// Locked permutation with `mid` run after round K (K = 0: before it).
template <int K, typename F>
__device__ __forceinline__ void keccak_f_lock_mid(State& s, F&& mid) {
    static_assert(K >= 0 && K <= 24, "mid point");
    if constexpr (K == 0) mid();
#pragma unroll kRoundUnroll
    for (int r = 0; r < K; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
    if constexpr (K > 0) mid();
#pragma unroll kRoundUnroll
    for (int r = K; r < 24; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
}
// Locked permutation with `m1` run after round K1 and `m2` after round K2
// (0 < K1 < K2 < 24).
template <int K1, int K2, typename F1, typename F2>
__device__ __forceinline__ void keccak_f_lock_mid2(State& s, F1&& m1, F2&& m2) {
    static_assert(K1 > 0 && K1 < K2 && K2 < 24, "mid points");
#pragma unroll kRoundUnroll
    for (int r = 0; r < K1; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
    m1();
#pragma unroll kRoundUnroll
    for (int r = K1; r < K2; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
    m2();
#pragma unroll kRoundUnroll
    for (int r = K2; r < 24; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
}
// ... with m1, m2, m3 after rounds K1 < K2 < K3.
template <int K1, int K2, int K3, typename F1, typename F2, typename F3>
__device__ __forceinline__ void keccak_f_lock_mid3(State& s, F1&& m1, F2&& m2, F3&& m3) {
    static_assert(K1 > 0 && K1 < K2 && K2 < K3 && K3 < 24, "mid points");
#pragma unroll kRoundUnroll
    for (int r = 0; r < K1; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
    m1();
#pragma unroll kRoundUnroll
    for (int r = K1; r < K2; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
    m2();
#pragma unroll kRoundUnroll
    for (int r = K2; r < K3; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
    m3();
#pragma unroll kRoundUnroll
    for (int r = K3; r < 24; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
}
// `mid` runs after round K (K = 0: before the permutation), e.g. the issue of
// the next window's DMA in k_leaf_lock_sc.
template <int K = 0, typename F>
__device__ __forceinline__ void keccak_f_digest_lock(State& s, F&& mid) {
    static_assert(K >= 0 && K <= 22, "mid point");
    if constexpr (K == 0) mid();
#pragma unroll kRoundUnroll
    for (int r = 0; r < K; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
    if constexpr (K > 0) mid();
#pragma unroll kRoundUnroll
    for (int r = K; r < 22; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
    round_asm<true>(s, kRcLo[22], kRcHi[22]);
    last_round_digest(s, kRcLo[23], kRcHi[23]);
    asm volatile("" : "+v"(s.lo[0]), "+v"(s.hi[0]), "+v"(s.lo[1]), "+v"(s.hi[1]), "+v"(s.lo[2]), "+v"(s.hi[2]),
                 "+v"(s.lo[3]), "+v"(s.hi[3]));
}
// The digest-only form with m1, m2, m3 after rounds K1 < K2 < K3 <= 22.
template <int K1, int K2, int K3, typename F1, typename F2, typename F3>
__device__ __forceinline__ void keccak_f_digest_lock_mid3(State& s, F1&& m1, F2&& m2, F3&& m3) {
    static_assert(K1 > 0 && K1 < K2 && K2 < K3 && K3 <= 22, "mid points");
#pragma unroll kRoundUnroll
    for (int r = 0; r < K1; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
    m1();
#pragma unroll kRoundUnroll
    for (int r = K1; r < K2; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
    m2();
#pragma unroll kRoundUnroll
    for (int r = K2; r < K3; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
    m3();
#pragma unroll kRoundUnroll
    for (int r = K3; r < 22; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
    round_asm<true>(s, kRcLo[22], kRcHi[22]);
    last_round_digest(s, kRcLo[23], kRcHi[23]);
    asm volatile("" : "+v"(s.lo[0]), "+v"(s.hi[0]), "+v"(s.lo[1]), "+v"(s.hi[1]), "+v"(s.lo[2]), "+v"(s.hi[2]),
                 "+v"(s.lo[3]), "+v"(s.hi[3]));
}
__device__ __forceinline__ void keccak_f_digest_lock(State& s) {
#pragma unroll kRoundUnroll
    for (int r = 0; r < 22; ++r) round_asm<true>(s, kRcLo[r], kRcHi[r]);
    round_asm<true>(s, kRcLo[22], kRcHi[22]);
    last_round_digest(s, kRcLo[23], kRcHi[23]);
    asm volatile("" : "+v"(s.lo[0]), "+v"(s.hi[0]), "+v"(s.lo[1]), "+v"(s.hi[1]), "+v"(s.lo[2]), "+v"(s.hi[2]),
                 "+v"(s.lo[3]), "+v"(s.hi[3]));
}

// ---- absorb helpers --------------------------------------------------------
__device__ __forceinline__ void xor_lane(State& s, int i, uint2 w) {
    s.lo[i] ^= w.x;
    s.hi[i] ^= w.y;
}

// Final-block padding for legacy Keccak: byte `pos` (< 136) of the block gets
// 0x01, byte 135 gets 0x80.  pos is a compile-time constant here.
template <int POS>
__device__ __forceinline__ void pad_const(State& s) {
    constexpr int lane = POS / 8, sh = (POS % 8) * 8;
    if constexpr (sh < 32)
        s.lo[lane] ^= 1u << sh;
    else
        s.hi[lane] ^= 1u << (sh - 32);
    s.hi[16] ^= 0x80000000u;
}

// Streaming (non-temporal) loads of input that is read exactly once.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
// Loads of the streamed inputs (items, node levels, deposit records): plain,
// L2-allocating loads.  Non-temporal loads (rounds 1-2) let the leaf kernel's
// lines leave L2 before all of a window's 16-B loads had hit them: 10.09 GB
// fetched per 2^28 launch against 8.90 GB with plain loads (8.59 GB
// algorithmic), and the leaf pass ran 1.3-2.5 % slower (profiles/r02zc/ab.txt,
// three boxes).
__device__ __forceinline__ uint4 ld_stream(const uint4* p) { return *p; }
__device__ __forceinline__ uint2 ld_stream(const uint2* p) { return *p; }

// Squeeze the 32-byte digest (lanes 0..3, little-endian).
__device__ __forceinline__ void digest(const State& s, uint4& d0, uint4& d1) {
    d0 = make_uint4(s.lo[0], s.hi[0], s.lo[1], s.hi[1]);
    d1 = make_uint4(s.lo[2], s.hi[2], s.lo[3], s.hi[3]);
}

}  // namespace mk

// ============================================================================
// Two lanes per state (latency form).  Lane pair (2k, 2k+1) holds one state:
// the even lane the low 32-bit halves of all 25 lanes, the odd lane the high
// halves.  Every 64-bit rotation needs the partner's half (one DPP
// quad_perm [1,0,3,2] move) and ONE v_alignbit_b32 per lane instead of two,
// so a lane issues 120 instructions per round instead of 180: for the
// narrow top of a tree, where one permutation's latency on a lone wave is
// the cost of a whole level, that is ~1.6x less time per level.
namespace mk {
namespace pair {

__device__ __forceinline__ uint32_t partner(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1 /* quad_perm [1,0,3,2] */, 0xF, 0xF, false);
}

// own half of rotl64 by N, given own and partner halves (same formula for
// the low and the high lane).
template <int N>
__device__ __forceinline__ uint32_t rot(uint32_t own, uint32_t par) {
    if constexpr (N == 0)
        return own;
    else if constexpr (N == 32)
        return par;
    else if constexpr (N < 32)
        return funnel(own, par, 32 - N);
    else
        return funnel(par, own, 64 - N);
}

struct Half {
    uint32_t v[25];
};

template <int I>
__device__ __forceinline__ void rho_pi_one(const Half& a, uint32_t (&b)[25]) {
    constexpr int x = I % 5, y = I / 5;
    constexpr int dst = y + 5 * ((2 * x + 3 * y) % 5);
    constexpr int r = MK_RHO(I);
    if constexpr (r == 0)
        b[dst] = a.v[I];
    else
        b[dst] = rot<r>(a.v[I], partner(a.v[I]));
}

template <int... Is>
__device__ __forceinline__ void rho_pi_all(const Half& a, uint32_t (&b)[25], std::integer_sequence<int, Is...>) {
    (rho_pi_one<Is>(a, b), ...);
}

__device__ __forceinline__ void round_fn(Half& s, uint32_t rc_own) {
    uint32_t c[5], r[5];
#pragma unroll
    for (int x = 0; x < 5; ++x) c[x] = xor3(xor3(s.v[x], s.v[x + 5], s.v[x + 10]), s.v[x + 15], s.v[x + 20]);
#pragma unroll
    for (int x = 0; x < 5; ++x) r[x] = rot<1>(c[x], partner(c[x]));
#pragma unroll
    for (int i = 0; i < 25; ++i) s.v[i] = xor3(s.v[i], c[(i % 5 + 4) % 5], r[(i % 5 + 1) % 5]);
    uint32_t b[25];
    rho_pi_all(s, b, std::make_integer_sequence<int, 25>{});
#pragma unroll
    for (int y = 0; y < 5; ++y)
#pragma unroll
        for (int x = 0; x < 5; ++x)
            s.v[x + 5 * y] = chi3(b[x + 5 * y], b[(x + 1) % 5 + 5 * y], b[(x + 2) % 5 + 5 * y]);
    s.v[0] ^= rc_own;
}

// odd = this lane holds the high halves
__device__ __forceinline__ void keccak_f(Half& s, bool odd) {
#pragma unroll kRoundUnroll
    for (int r = 0; r < 24; ++r) round_fn(s, odd ? kRcHi[r] : kRcLo[r]);
}

__device__ __forceinline__ void zero(Half& s) {
#pragma unroll
    for (int i = 0; i < 25; ++i) s.v[i] = 0u;
}

}  // namespace pair
}  // namespace mk

// ============================================================================
// Two lanes per state, BIT-INTERLEAVED (latency form, v2).  Lane pair
// (2k, 2k+1) holds one state; lane p (= lane & 1) holds, for each of the 25
// Keccak lanes, the 32 bits of parity p: bit j of word v[i] = bit 2j+p of
// Keccak lane i.  A 64-bit rotation by an even r is then a 32-bit rotation of
// the lane's OWN word by r/2 (one v_alignbit, no exchange); an odd r swaps the
// parities: the lane rotates its own word by the amount its partner needs
// (m + p for r = 2m+1) and takes the partner's result (one DPP move).  Per
// round and lane: 60 bitop3 + 25 xor + 29 alignbit + 17 DPP (vs 120 bitop3 +
// 58 alignbit for a whole state in one lane, 119 in the lo/hi pair form).
namespace mk {
namespace ilv {

// round constants split into even / odd bits (computed from kRcLo/kRcHi)
__constant__ uint32_t kRcE[24] = {
    0x00000001u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000001u, 0x00000001u,
    0x00000001u, 0x00000001u, 0x00000000u, 0x00000000u, 0x00000001u, 0x00000000u,
    0x00000001u, 0x00000001u, 0x00000001u, 0x00000001u, 0x00000000u, 0x00000000u,
    0x00000000u, 0x00000000u, 0x00000001u, 0x00000000u, 0x00000001u, 0x00000000u};
__constant__ uint32_t kRcO[24] = {
    0x00000000u, 0x00000089u, 0x8000008bu, 0x80008080u, 0x0000008bu, 0x00008000u,
    0x80008088u, 0x80000082u, 0x0000000bu, 0x0000000au, 0x00008082u, 0x00008003u,
    0x0000808bu, 0x8000000bu, 0x8000008au, 0x80000081u, 0x80000081u, 0x80000008u,
    0x00000083u, 0x80008003u, 0x80008088u, 0x80000088u, 0x00008000u, 0x80008082u};

__device__ __forceinline__ uint32_t partner(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1 /* quad_perm [1,0,3,2] */, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t rot32(uint32_t x, uint32_t sh /* = 32 - amount, mod 32 */) {
    return __builtin_amdgcn_alignbit(x, x, sh);
}

struct Half {
    uint32_t v[25];
};

// own word of rotl64 by R; p = lane parity (0/1)
template <int R>
__device__ __forceinline__ uint32_t rot(uint32_t own, uint32_t p) {
    if constexpr (R == 0) {
        return own;
    } else if constexpr (R % 2 == 0) {
        return rot32(own, 32 - R / 2);
    } else {
        constexpr uint32_t m = (R - 1) / 2;
        return partner(rot32(own, (32 - m - p) & 31u));  // partner needs own rotated by m + p
    }
}

template <int I>
__device__ __forceinline__ void rho_pi_one(const Half& a, uint32_t (&b)[25], uint32_t p) {
    constexpr int x = I % 5, y = I / 5;
    constexpr int dst = y + 5 * ((2 * x + 3 * y) % 5);
    b[dst] = rot<MK_RHO(I)>(a.v[I], p);
}

template <int... Is>
__device__ __forceinline__ void rho_pi_all(const Half& a, uint32_t (&b)[25], uint32_t p,
                                           std::integer_sequence<int, Is...>) {
    (rho_pi_one<Is>(a, b, p), ...);
}

__device__ __forceinline__ void round_fn(Half& s, uint32_t rc_own, uint32_t p) {
    uint32_t c[5], d[5];
#pragma unroll
    for (int x = 0; x < 5; ++x) c[x] = xor3(xor3(s.v[x], s.v[x + 5], s.v[x + 10]), s.v[x + 15], s.v[x + 20]);
#pragma unroll
    for (int x = 0; x < 5; ++x) d[x] = c[(x + 4) % 5] ^ rot<1>(c[(x + 1) % 5], p);
#pragma unroll
    for (int i = 0; i < 25; ++i) s.v[i] ^= d[i % 5];
    uint32_t b[25];
    rho_pi_all(s, b, p, std::make_integer_sequence<int, 25>{});
#pragma unroll
    for (int y = 0; y < 5; ++y)
#pragma unroll
        for (int x = 0; x < 5; ++x)
            s.v[x + 5 * y] = chi3(b[x + 5 * y], b[(x + 1) % 5 + 5 * y], b[(x + 2) % 5 + 5 * y]);
    s.v[0] ^= rc_own;
}

__device__ __forceinline__ void keccak_f(Half& s, uint32_t p) {
#pragma unroll kRoundUnroll
    for (int r = 0; r < 24; ++r) round_fn(s, p ? kRcO[r] : kRcE[r], p);
}

__device__ __forceinline__ void zero(Half& s) {
#pragma unroll
    for (int i = 0; i < 25; ++i) s.v[i] = 0u;
}

// ---- conversion between (lo, hi) 32-bit halves and the parity-p word -------
// even bits of x gathered into the low 16 bits
__device__ __forceinline__ uint32_t pack_even16(uint32_t x) {
    x &= 0x55555555u;
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0F0F0F0Fu;
    x = (x | (x >> 4)) & 0x00FF00FFu;
    x = (x | (x >> 8)) & 0x0000FFFFu;
    return x;
}
// low 16 bits of x spread to the even bit positions
__device__ __forceinline__ uint32_t spread16(uint32_t x) {
    x &= 0x0000FFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}
// parity-p word of the 64-bit lane (hi:lo)
__device__ __forceinline__ uint32_t to_ilv(uint32_t lo, uint32_t hi, uint32_t p) {
    return pack_even16(lo >> p) | (pack_even16(hi >> p) << 16);
}
// this lane's half (p = 0: lo, p = 1: hi) of the 64-bit lane whose parity
// words are `own` (this lane's) and the partner lane's
__device__ __forceinline__ uint32_t from_ilv(uint32_t own, uint32_t p) {
    const uint32_t par = partner(own);
    const uint32_t e = p ? par : own, o = p ? own : par;
    const uint32_t sh = p ? 16u : 0u;
    return spread16(e >> sh) | (spread16(o >> sh) << 1);
}

}  // namespace ilv
}  // namespace mk

// ============================================================================
// One state spread over a whole wave (latency form, v3).  GPU lane L = 8g + q
// holds, bit-interleaved (ilv words: e = even bits, o = odd bits), the Keccak
// lane (x, y) = (q mod 5, min(g, 4)): group g < 5 is row y = g, positions
// 0..4 are the canonical x = 0..4 and positions 5..7 repeat x = 0..2, and
// groups 5..7 mirror row 4.  Per round and lane: theta's column parity is an
// all-reduce over the groups (row_ror:8 DPP with rows {0,1,3} enabled, then
// v_permlane16_swap and v_permlane32_swap: the mirrors make rows 2/3 hold
// row 4 twice and 0 after the first two steps), its x-1 / x+1 neighbours are
// row_shr:1 / row_shl:1 DPP moves (row_shl:4 for x-1 at position 0), rho is
// a per-lane rotation with shift amounts in VGPRs, pi is one ds_bpermute per
// word from the canonical source lane (which also refreshes the repeats and
// mirrors), and chi reads x+1 / x+2 with row_shl:1 / row_shl:2.  ~36 VALU
// instructions and 2 bpermutes per round instead of 107 per lane for the
// lane pair: the narrow top of a tree, where one permutation's latency on a
// lone wave is the cost of a whole level.  Canonical positions are correct
// after every round; positions 6/7 are scratch between pi and the next pi.
namespace mk {
namespace spread {

struct Lane {
    uint32_t i;      // Keccak lane index x + 5y of this GPU lane
    uint32_t sh1;    // rho: alignbit shift rotating the even word
    uint32_t sh2;    // rho: alignbit shift rotating the odd word
    uint32_t swap;   // rho: all-ones when the offset is odd (the parities trade places)
    uint32_t src;    // pi: ds_bpermute byte address of the source lane
    uint32_t wrap;   // theta: all-ones at position 0 (x - 1 = 4 sits at position 4)
    uint32_t iota;   // all-ones on the two GPU lanes holding Keccak lane 0
};

__device__ __forceinline__ Lane lane_consts(uint32_t L) {
    const uint32_t g = (L >> 3) & 7u, q = L & 7u;
    const uint32_t x = q % 5u, y = g < 4u ? g : 4u;
    Lane c;
    c.i = x + 5u * y;
    const uint32_t r = MK_RHO(c.i);
    const uint32_t m = r >> 1;
    // rotl by k == alignbit(v, v, (32 - k) & 31)
    c.swap = (r & 1u) ? 0xFFFFFFFFu : 0u;
    c.sh1 = (32u - m) & 31u;                   // even word rotated by m
    c.sh2 = (32u - (m + (r & 1u))) & 31u;      // odd word by m (+1 if r odd)
    // pi: destination (X, Y) = (y', 2x' + 3y') of source (x', y'):
    // y' = X, x' = 3 (Y - 3X) mod 5
    const uint32_t xs = (3u * ((y + 15u - 3u * x) % 5u)) % 5u, ys = x;
    c.src = 4u * (8u * ys + xs);
    c.wrap = q == 0u ? 0xFFFFFFFFu : 0u;
    c.iota = c.i == 0u ? 0xFFFFFFFFu : 0u;
    return c;
}

// lanes whose source is outside the 16-lane row read 0 (never used).  Every
// lane must be written (bound_ctrl): with an undefined old value the DPP
// combiner may fold the move into its user (e.g. a v_cndmask) and leave
// such lanes unwritten, which corrupted the x-1 select at positions 0/1.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
constexpr int kShl1 = 0x101, kShl2 = 0x102, kShl4 = 0x104, kShr1 = 0x111, kRor8 = 0x128;

// column parity of this lane's x (valid at positions 0..5 of every group)
__device__ __forceinline__ uint32_t colsum(uint32_t v) {
    // rows 0, 1: g0^g1, g2^g3; row 2 kept (g4 | g5 = g4); row 3: g6^g7 = 0
    const uint32_t t = v ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRor8, 0xB, 0xF, false);
    const auto a = __builtin_amdgcn_permlane16_swap(t, t, false, false);
    const uint32_t s = a[0] ^ a[1];  // rows 0, 1: g0^..^g3; rows 2, 3: g4
    const auto b = __builtin_amdgcn_permlane32_swap(s, s, false, false);
    return b[0] ^ b[1];
}

// m ? a : b per bit (LUT 0xCA).  Lane selects must not be written as ?: on a
// DPP result: the compiler turns that into exec-masked DPP moves, and a DPP
// read of a lane that is off in EXEC returns 0.
__device__ __forceinline__ uint32_t sel(uint32_t m, uint32_t a, uint32_t b) {
    return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
}

// column parities of both words at once: the first swap pairs the even
// word's rows with the odd word's, so rows 0/2 carry even sums and rows 1/3
// odd sums until the last swap spreads each over the wave
__device__ __forceinline__ void colsum2(uint32_t e, uint32_t o, uint32_t& ce, uint32_t& co) {
    const uint32_t te = e ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e, kRor8, 0xB, 0xF, false);
    const uint32_t to = o ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)o, kRor8, 0xB, 0xF, false);
    const auto a = __builtin_amdgcn_permlane16_swap(te, to, false, false);
    const uint32_t r = a[0] ^ a[1];  // rows: e(0^1), o(0^1), e(2^3), o(2^3)
    const auto b = __builtin_amdgcn_permlane32_swap(r, r, false, false);
    const uint32_t s = b[0] ^ b[1];  // rows: Ce, Co, Ce, Co
    const auto d = __builtin_amdgcn_permlane16_swap(s, s, false, false);
    ce = d[0];
    co = d[1];
}

__device__ __forceinline__ void round_fn(uint32_t& e, uint32_t& o, const Lane& c, uint32_t rce, uint32_t rco) {
    uint32_t ce, co;
    colsum2(e, o, ce, co);
    const uint32_t me = sel(c.wrap, dpp<kShl4>(ce), dpp<kShr1>(ce));
    const uint32_t mo = sel(c.wrap, dpp<kShl4>(co), dpp<kShr1>(co));
    // D = C[x-1] ^ rotl64(C[x+1], 1): even word rotl32(odd, 1), odd word = even
    e = xor3(e, me, __builtin_amdgcn_alignbit(dpp<kShl1>(co), dpp<kShl1>(co), 31u));
    o = xor3(o, mo, dpp<kShl1>(ce));
    const uint32_t t1 = __builtin_amdgcn_alignbit(e, e, c.sh1);
    const uint32_t t2 = __builtin_amdgcn_alignbit(o, o, c.sh2);
    const uint32_t re = sel(c.swap, t2, t1), ro = sel(c.swap, t1, t2);
    const uint32_t be = (uint32_t)__builtin_amdgcn_ds_bpermute((int)c.src, (int)re);
    const uint32_t bo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)c.src, (int)ro);
    // iota: v ^ (iota & rc), LUT 0x78
    e = __builtin_amdgcn_bitop3_b32(chi3(be, dpp<kShl1>(be), dpp<kShl2>(be)), c.iota, rce, 0x78);
    o = __builtin_amdgcn_bitop3_b32(chi3(bo, dpp<kShl1>(bo), dpp<kShl2>(bo)), c.iota, rco, 0x78);
}

// ---- the same permutation on (lo, hi) halves instead of parity words ----------
// One more alignbit per round (theta's rotl 1 needs both halves), but nodes
// go in and out as plain 64-bit words: for one permutation per tree level
// that is cheaper than the bit (de)interleave.  rho: rotl64 by r = 32s + t
// takes (a, b) = (hi, lo) or, for r >= 32, (lo, hi) and shifts by 32 - t;
// r = 0 is run as r = 64 (shift 0 returns the second operand).
struct LaneLH {
    uint32_t swap;   // all-ones when r >= 32 or r == 0
    uint32_t sh;     // (32 - r mod 32) mod 32
    uint32_t src;    // pi: ds_bpermute byte address of the source lane
    uint32_t wrap;   // theta: all-ones at position 0
    uint32_t iota;   // all-ones on the lanes holding Keccak lane 0
    uint32_t i;      // Keccak lane index of this GPU lane
};

__device__ __forceinline__ LaneLH lane_consts_lh(uint32_t L) {
    const Lane c = lane_consts(L);
    const uint32_t r = MK_RHO(c.i);
    LaneLH h;
    h.swap = (r >= 32u || r == 0u) ? 0xFFFFFFFFu : 0u;
    h.sh = (32u - (r & 31u)) & 31u;
    h.src = c.src;
    h.wrap = c.wrap;
    h.iota = c.iota;
    h.i = c.i;
    return h;
}

__device__ __forceinline__ void round_lh(uint32_t& lo, uint32_t& hi, const LaneLH& c, uint32_t rcl, uint32_t rch) {
    uint32_t cl, ch;
    colsum2(lo, hi, cl, ch);
    const uint32_t ml = sel(c.wrap, dpp<kShl4>(cl), dpp<kShr1>(cl));
    const uint32_t mh = sel(c.wrap, dpp<kShl4>(ch), dpp<kShr1>(ch));
    const uint32_t pl = dpp<kShl1>(cl), ph = dpp<kShl1>(ch);
    lo = xor3(lo, ml, __builtin_amdgcn_alignbit(pl, ph, 31u));
    hi = xor3(hi, mh, __builtin_amdgcn_alignbit(ph, pl, 31u));
    const uint32_t a = sel(c.swap, lo, hi), b = sel(c.swap, hi, lo);
    const uint32_t th = __builtin_amdgcn_alignbit(a, b, c.sh);
    const uint32_t tl = __builtin_amdgcn_alignbit(b, a, c.sh);
    const uint32_t bl = (uint32_t)__builtin_amdgcn_ds_bpermute((int)c.src, (int)tl);
    const uint32_t bh = (uint32_t)__builtin_amdgcn_ds_bpermute((int)c.src, (int)th);
    lo = __builtin_amdgcn_bitop3_b32(chi3(bl, dpp<kShl1>(bl), dpp<kShl2>(bl)), c.iota, rcl, 0x78);
    hi = __builtin_amdgcn_bitop3_b32(chi3(bh, dpp<kShl1>(bh), dpp<kShl2>(bh)), c.iota, rch, 0x78);
}

#define MK_SPREAD_UNROLL 24
__device__ __forceinline__ void keccak_f(uint32_t& e, uint32_t& o, const Lane& c) {
#pragma unroll MK_SPREAD_UNROLL
    for (int r = 0; r < 24; ++r) round_fn(e, o, c, ilv::kRcE[r], ilv::kRcO[r]);
}

__device__ __forceinline__ void keccak_f_lh(uint32_t& lo, uint32_t& hi, const LaneLH& c) {
#pragma unroll MK_SPREAD_UNROLL
    for (int r = 0; r < 24; ++r) round_lh(lo, hi, c, kRcLo[r], kRcHi[r]);
}

}  // namespace spread
}  // namespace mk
