// Probe: a Keccak-f round whose instruction ORDER is fixed (one asm volatile
// statement per VALU instruction, class-grouped: 20 bitop3 | 10 alignbit |
// 50 bitop3 | 48 alignbit | 50 bitop3 + iota), against the compiled round
// (mk::keccak_f), register resident, with and without an s_barrier per
// round in a 1024-thread workgroup (4 waves per SIMD, all in phase).
// tools/isa_rates.py --only-sync measured a round-shaped stream of
// independent chains at 2.7-2.8 cycles/instruction phase-locked vs 3.4-3.6
// free running; this checks whether the real dependency structure keeps it.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../prysm_amd/csrc asm_round_probe.hip -o asm_round_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include "keccak_dev.hpp"

#define CHECK(x)                                                   \
    do {                                                           \
        hipError_t e = (x);                                        \
        if (e != hipSuccess) {                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
            exit(1);                                               \
        }                                                          \
    } while (0)

// mk::round_asm lives in keccak_dev.hpp.

// Alternative fixed orders.  Lane b[X + 5Y] (after pi) comes from a[x + 5X]
// with x = 3 (Y - 3X) mod 5.
template <int X, int Y>
__device__ __forceinline__ void rot_into(const mk::State& a, uint32_t (&blo)[25], uint32_t (&bhi)[25]) {
    constexpr int x = ((3 * (Y - 3 * X)) % 5 + 5) % 5;
    constexpr int src = x + 5 * X;
    mk::arot<MK_RHO(src)>(a.lo[src], a.hi[src], blo[X + 5 * Y], bhi[X + 5 * Y]);
}
template <int Y>
__device__ __forceinline__ void rot_row(const mk::State& a, uint32_t (&blo)[25], uint32_t (&bhi)[25]) {
    rot_into<0, Y>(a, blo, bhi);
    rot_into<1, Y>(a, blo, bhi);
    rot_into<2, Y>(a, blo, bhi);
    rot_into<3, Y>(a, blo, bhi);
    rot_into<4, Y>(a, blo, bhi);
}
template <int Y>
__device__ __forceinline__ void chi_row(mk::State& s, const uint32_t (&blo)[25], const uint32_t (&bhi)[25]) {
#pragma unroll
    for (int x = 0; x < 5; ++x) {
        const int i = x + 5 * Y, i1 = (x + 1) % 5 + 5 * Y, i2 = (x + 2) % 5 + 5 * Y;
        s.lo[i] = mk::achi(blo[i], blo[i1], blo[i2]);
        s.hi[i] = mk::achi(bhi[i], bhi[i1], bhi[i2]);
    }
}
template <int Y>
__device__ __forceinline__ void apply_rot_row(mk::State& s, const uint32_t (&clo)[5], const uint32_t (&chi_)[5],
                                              const uint32_t (&rlo)[5], const uint32_t (&rhi)[5],
                                              uint32_t (&blo)[25], uint32_t (&bhi)[25]) {
    // theta-apply the 5 source lanes of b-row Y, then rotate them
#pragma unroll
    for (int X = 0; X < 5; ++X) {
        const int x = ((3 * (Y - 3 * X)) % 5 + 5) % 5;
        const int src = x + 5 * X;
        s.lo[src] = mk::ax3(s.lo[src], clo[(x + 4) % 5], rlo[(x + 1) % 5]);
        s.hi[src] = mk::ax3(s.hi[src], chi_[(x + 4) % 5], rhi[(x + 1) % 5]);
    }
    rot_row<Y>(s, blo, bhi);
}

// ORDER 1: parity | D | per b-row: apply 10, rot 10, chi 10.   ORDER 2: parity | D | apply 50 | per row: rot 10, chi 10.
template <int ORDER>
__device__ __forceinline__ void round_ord(mk::State& s, uint32_t rclo, uint32_t rchi) {
    uint32_t clo[5], chi_[5];
#pragma unroll
    for (int x = 0; x < 5; ++x) {
        clo[x] = mk::ax3(s.lo[x], s.lo[x + 5], s.lo[x + 10]);
        chi_[x] = mk::ax3(s.hi[x], s.hi[x + 5], s.hi[x + 10]);
    }
#pragma unroll
    for (int x = 0; x < 5; ++x) {
        clo[x] = mk::ax3(clo[x], s.lo[x + 15], s.lo[x + 20]);
        chi_[x] = mk::ax3(chi_[x], s.hi[x + 15], s.hi[x + 20]);
    }
    uint32_t rlo[5], rhi[5];
#pragma unroll
    for (int x = 0; x < 5; ++x) mk::arot<1>(clo[x], chi_[x], rlo[x], rhi[x]);
    uint32_t blo[25], bhi[25];
    if constexpr (ORDER == 1) {
        mk::State o;  // chi output: a row's lanes may still be sources of later rows
        apply_rot_row<0>(s, clo, chi_, rlo, rhi, blo, bhi);
        chi_row<0>(o, blo, bhi);
        apply_rot_row<1>(s, clo, chi_, rlo, rhi, blo, bhi);
        chi_row<1>(o, blo, bhi);
        apply_rot_row<2>(s, clo, chi_, rlo, rhi, blo, bhi);
        chi_row<2>(o, blo, bhi);
        apply_rot_row<3>(s, clo, chi_, rlo, rhi, blo, bhi);
        chi_row<3>(o, blo, bhi);
        apply_rot_row<4>(s, clo, chi_, rlo, rhi, blo, bhi);
        chi_row<4>(o, blo, bhi);
        s = o;
    } else {
#pragma unroll
        for (int i = 0; i < 25; ++i) {
            const int x = i % 5;
            s.lo[i] = mk::ax3(s.lo[i], clo[(x + 4) % 5], rlo[(x + 1) % 5]);
            s.hi[i] = mk::ax3(s.hi[i], chi_[(x + 4) % 5], rhi[(x + 1) % 5]);
        }
        mk::State a = s;
        rot_row<0>(a, blo, bhi);
        chi_row<0>(s, blo, bhi);
        rot_row<1>(a, blo, bhi);
        chi_row<1>(s, blo, bhi);
        rot_row<2>(a, blo, bhi);
        chi_row<2>(s, blo, bhi);
        rot_row<3>(a, blo, bhi);
        chi_row<3>(s, blo, bhi);
        rot_row<4>(a, blo, bhi);
        chi_row<4>(s, blo, bhi);
    }
    s.lo[0] = mk::axs(s.lo[0], rclo);
    s.hi[0] = mk::axs(s.hi[0], rchi);
}

// ASM: 0 compiled round, 1 fixed-order asm round.  SYNC: s_barrier every SYNC rounds (0 = none).
template <int NT, int ASM, int SYNC>
__global__ __launch_bounds__(NT) void k_perm(uint32_t* out, int iters) {
    const uint32_t g = blockIdx.x * NT + threadIdx.x;
    mk::State s;
#pragma unroll
    for (int i = 0; i < 25; ++i) {
        s.lo[i] = g * 2654435761u + i;
        s.hi[i] = g ^ (0x9E3779B9u * (i + 1));
    }
#pragma unroll 1
    for (int k = 0; k < iters; ++k) {
        if constexpr (ASM == 9) {  // the phase-locked permutation of k_leaf_lock (round_asm<true>)
            mk::keccak_f_lock(s);
            continue;
        }
#pragma unroll 2
        for (int r = 0; r < 24; ++r) {
            if constexpr (ASM == 1)
                mk::round_asm(s, mk::kRcLo[r], mk::kRcHi[r]);
            else if constexpr (ASM >= 2)
                round_ord<ASM - 1>(s, mk::kRcLo[r], mk::kRcHi[r]);
            else
                mk::round_fn(s, mk::kRcLo[r], mk::kRcHi[r]);
            if constexpr (SYNC > 0)
                if ((r + 1) % SYNC == 0) __builtin_amdgcn_s_barrier();
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 25; ++i) x ^= s.lo[i] ^ s.hi[i];
    out[g] = x;
}

template <int NT, int ASM, int SYNC>
static void run(const char* name, int blocks, int iters, uint32_t* out, uint32_t* ref) {
    hipLaunchKernelGGL((k_perm<NT, ASM, SYNC>), dim3(blocks), dim3(NT), 0, 0, out, iters);
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL((k_perm<NT, ASM, SYNC>), dim3(blocks), dim3(NT), 0, 0, out, iters);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    // every variant must compute the same permutations
    const size_t n = (size_t)blocks * NT;
    uint32_t* h = (uint32_t*)malloc(n * 4);
    CHECK(hipMemcpy(h, out, n * 4, hipMemcpyDeviceToHost));
    bool same = true;
    if (ref[0] == 0xFFFFFFFFu && ref[1] == 0xFFFFFFFFu)
        for (size_t i = 0; i < n; ++i) ref[i] = h[i];
    else
        for (size_t i = 0; i < n; ++i) same &= ref[i] == h[i];
    free(h);
    const double perms = (double)n * iters;
    printf("{\"test\": \"%s\", \"threads\": %d, \"blocks\": %d, \"ms\": %.3f, \"Tops\": %.2f, \"same\": %s}\n", name,
           NT, blocks, best, perms * 4320 / (best / 1e3) / 1e12, same ? "true" : "false");
    fflush(stdout);
}

int main() {
    uint32_t* out;
    const size_t n = 4096 * 256;
    CHECK(hipMalloc(&out, n * 4));
    uint32_t* ref = (uint32_t*)malloc(n * 4);
    const int it = 400;
    // 256 CUs, 4 waves per SIMD (16 per CU) in every configuration: same
    // total threads (262,144) and permutations.
    ref[0] = ref[1] = 0xFFFFFFFFu;
    run<256, 0, 0>("compiled_free", 1024, it, out, ref);
    run<256, 1, 0>("asm_free", 1024, it, out, ref);
    run<256, 2, 0>("asm_rowwise_free", 1024, it, out, ref);
    run<256, 3, 0>("asm_rotchi_rows_free", 1024, it, out, ref);
    run<256, 0, 0>("compiled_free_again", 1024, it, out, ref);
    run<256, 1, 0>("asm_free_again", 1024, it, out, ref);
    run<256, 2, 0>("asm_rowwise_free_again", 1024, it, out, ref);
    run<256, 3, 0>("asm_rotchi_rows_free_again", 1024, it, out, ref);
    if (getenv("PROBE_KLOCK")) {  // keccak_f_lock as compiled (MK_LOCK_BARS, MK_ROUND_UNROLL)
        run<1024, 9, 0>("keccak_f_lock_wg1024", 256, it, out, ref);
        run<256, 0, 0>("compiled_free", 1024, it, out, ref);
        run<1024, 9, 0>("keccak_f_lock_wg1024_again", 256, it, out, ref);
    }
    if (getenv("PROBE_LOCK")) {
        run<1024, 0, 1>("compiled_lock1", 256, it, out, ref);
        run<1024, 1, 1>("asm_lock1", 256, it, out, ref);
        run<1024, 1, 24>("asm_lock24", 256, it, out, ref);
        run<1024, 1, 0>("asm_wg1024_nobar", 256, it, out, ref);
    }
    free(ref);
    return 0;
}
