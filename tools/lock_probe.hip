// Probe: does phase-locking the waves of a SIMD speed up the compiled
// Keccak-f round?  tools/isa_rates.py --only-sync shows a Keccak-round-shaped
// stream (122 full-rate + 58 half-rate instructions) issuing at 2.7-2.8
// cycles per instruction when every wave of the SIMD is on the same
// instruction (1024-thread workgroup + s_barrier) against 3.4-3.6 free
// running.  Here the same register-resident permutation loop (mk::keccak_f,
// the leaf kernel's round) runs
//   free:  256-thread workgroups, 4 per CU (4 waves per SIMD, from 4 WGs)
//   lockS: 1024-thread workgroups, 1 per CU, s_barrier every S rounds
// with no memory traffic.  Output: T int32 ops/s at 4320 ops per permutation.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../prysm_amd/csrc lock_probe.hip -o lock_probe
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

template <int NT, int SYNC>
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
        if constexpr (SYNC != 0)
            mk::keccak_f_lock(s);  // the phase-locked round (an s_barrier per round)
        else
            mk::keccak_f(s);
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 25; ++i) x ^= s.lo[i] ^ s.hi[i];
    out[g] = x;
}

template <int NT, int SYNC>
static void run(const char* name, int blocks, int iters, uint32_t* out) {
    hipLaunchKernelGGL((k_perm<NT, SYNC>), dim3(blocks), dim3(NT), 0, 0, out, iters);
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL((k_perm<NT, SYNC>), dim3(blocks), dim3(NT), 0, 0, out, iters);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    const double perms = (double)blocks * NT * iters;
    printf("{\"test\": \"%s\", \"threads\": %d, \"blocks\": %d, \"ms\": %.3f, \"Tops\": %.2f}\n", name, NT,
           blocks, best, perms * 4320 / (best / 1e3) / 1e12);
}

int main() {
    uint32_t* out;
    CHECK(hipMalloc(&out, 4096 * 1024 * 4));
    const int it = 400;
    // 256 CUs; 4 waves per SIMD in every configuration (16 per CU)
    run<256, 0>("free", 1024, it, out);
    run<256, 0>("free_x4", 4096, it / 4, out);
    run<1024, 0>("wg1024_nobar", 256, it, out);
    run<1024, 24>("lock24", 256, it, out);
    run<1024, 12>("lock12", 256, it, out);
    run<1024, 4>("lock4", 256, it, out);
    run<1024, 2>("lock2", 256, it, out);
    run<1024, 1>("lock1", 256, it, out);
    run<512, 0>("wg512_nobar", 512, it, out);
    run<512, 2>("wg512_lock2", 512, it, out);
    CHECK(hipFree(out));
    return 0;
}
