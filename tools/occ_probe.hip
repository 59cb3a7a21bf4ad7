// Probe: how fast one SIMD runs one-state-per-lane permutations when only a
// few waves of a 1024-thread workgroup have work -- the regime of a fused
// top's widest in-workgroup levels (512 / 256 parents per workgroup: 8 / 4
// active waves).  One workgroup of 1024 threads; waves 0..A-1 each run
// `iters` dependent permutations (waves go to SIMD w mod 4), the others
// idle.  Variants:
//   free   A waves, one state per lane, free running (mk::keccak_f)
//   lock   the same with the locked round (mk::keccak_f_lock: s_barrier
//          twice a round), the idle waves running the matching barriers
//   two    A waves, TWO states per lane, rounds alternated (twice the work
//          per wave: cycles reported per pair of permutations)
// Cycles from s_memtime (wave 0's loop, and the max over the active waves).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../prysm_amd/csrc occ_probe.hip -o occ_probe
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

// the same permutation on two states with their rounds alternated
__device__ __forceinline__ void keccak_f2(mk::State& a, mk::State& b) {
#pragma unroll 1
    for (int r = 0; r < 24; ++r) {
        mk::round_fn(a, mk::kRcLo[r], mk::kRcHi[r]);
        mk::round_fn(b, mk::kRcLo[r], mk::kRcHi[r]);
    }
}

template <int V>
__global__ __launch_bounds__(1024) void k_occ(uint32_t* io, int active, int iters, unsigned long long* clk) {
    const uint32_t t = threadIdx.x, w = t >> 6;
    const bool act = (int)w < active;
    mk::State s, s2;
    for (int i = 0; i < 25; ++i) {
        s.lo[i] = io[(50 * t + 2 * i) % 65536];
        s.hi[i] = io[(50 * t + 2 * i + 1) % 65536];
        s2.lo[i] = s.lo[i] ^ 0x9E3779B9u;
        s2.hi[i] = s.hi[i] ^ 0x7F4A7C15u;
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (V == 0) {
        if (act)
            for (int k = 0; k < iters; ++k) mk::keccak_f(s);
    } else if constexpr (V == 1) {
        if (act) {
            for (int k = 0; k < iters; ++k) mk::keccak_f_lock(s);
        } else {
            for (int k = 0; k < iters * 24 * MK_LOCK_BARS; ++k) __builtin_amdgcn_s_barrier();
        }
    } else {
        if (act)
            for (int k = 0; k < iters; ++k) keccak_f2(s, s2);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
    for (int i = 0; i < 25; ++i) acc ^= s.lo[i] ^ s.hi[i] ^ s2.lo[i] ^ s2.hi[i];
    io[65536 + t] = acc;
    if ((t & 63u) == 0) clk[w] = act ? t1 - t0 : 0;
}

template <int V>
void run(uint32_t* d, unsigned long long* c, int active, int iters, const char* name) {
    hipLaunchKernelGGL(k_occ<V>, 1, 1024, 0, 0, d, active, iters, c);  // warm
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_occ<V>, 1, 1024, 0, 0, d, active, iters, c);
    CHECK(hipDeviceSynchronize());
    unsigned long long cyc[16];
    CHECK(hipMemcpy(cyc, c, sizeof(cyc), hipMemcpyDeviceToHost));
    unsigned long long mx = 0;
    for (int w = 0; w < active; ++w) mx = cyc[w] > mx ? cyc[w] : mx;
    printf("{\"variant\": \"%s\", \"active_waves\": %d, \"waves_per_simd\": %.2f, \"cycles_per_perm_wave0\": %.0f, "
           "\"cycles_per_perm_max\": %.0f}\n",
           name, active, active / 4.0, (double)cyc[0] / iters, (double)mx / iters);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 50;
    uint32_t* d;
    unsigned long long* c;
    CHECK(hipMalloc(&d, (65536 + 1024) * 4));
    CHECK(hipMalloc(&c, 16 * 8));
    CHECK(hipMemset(d, 0x5A, (65536 + 1024) * 4));
    for (int a : {1, 4, 8, 12, 16}) run<0>(d, c, a, iters, "free");
    for (int a : {4, 8, 16}) run<1>(d, c, a, iters, "lock");
    for (int a : {1, 4, 8}) run<2>(d, c, a, iters, "two");
    CHECK(hipFree(d));
    CHECK(hipFree(c));
    return 0;
}
