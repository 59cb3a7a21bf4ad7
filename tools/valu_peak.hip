// Microbenchmarks that pin the integer-VALU roofline used by bench.py:
//   - bitop3 / alignbit / xor issue rate with 8 independent chains per lane
//   - register-resident Keccak-f[1600] throughput (no memory), round loop
//     rolled x4 (scalar round constants) vs fully unrolled (immediates)
//   - the shader clock under that load: s_memtime / s_memrealtime (100 MHz)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../prysm_amd/csrc valu_peak.hip -o valu_peak
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define MK_ROUND_UNROLL 4
#include "keccak_dev.hpp"

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

template <int OP>
__global__ __launch_bounds__(256) void k_ops(uint32_t* out, int iters, unsigned long long* clk) {
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * (i + 1) + blockIdx.x;
    const uint32_t b = threadIdx.x ^ 0x5555, c = blockIdx.x ^ 0x3333;
    uint32_t vs = (threadIdx.x & 7) | 8;  // per-lane value: lives in a VGPR
    const uint32_t tq = threadIdx.x & 3u;
    uint32_t vsh[4] = {tq | 4u, tq | 8u, tq | 12u, tq | 16u};
    const uint32_t ss = __builtin_amdgcn_readfirstlane(threadIdx.x + 5) & 31;
    const uint32_t ss2[2] = {(uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x * 3 + 1), (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x + 77)};
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if constexpr (OP == 0)
                    a[i] = __builtin_amdgcn_bitop3_b32(a[i], b, c, 0x96);
                else if constexpr (OP == 1)
                    a[i] = __builtin_amdgcn_alignbit(a[i], a[(i + 1) & 7], 7);
                else if constexpr (OP == 2)
                    a[i] = a[i] ^ a[(i + 3) & 7];
                else if constexpr (OP == 3)  // three chain operands, distinct
                    a[i] = __builtin_amdgcn_bitop3_b32(a[i], a[(i + 1) & 7], a[(i + 2) & 7], 0x96);
                else if constexpr (OP == 4)  // operands 4 registers apart
                    a[i] = __builtin_amdgcn_bitop3_b32(a[i], a[(i + 4) & 7], b, 0x96);
                else if constexpr (OP == 5)  // two VGPR + one SGPR-uniform
                    a[i] = __builtin_amdgcn_bitop3_b32(a[i], a[(i + 1) & 7], (uint32_t)blockIdx.x, 0xD2);
                else if constexpr (OP == 6)  // alignbit two chains, 3 apart
                    a[i] = __builtin_amdgcn_alignbit(a[i], a[(i + 3) & 7], 13);
                else if constexpr (OP == 7)  // alignbit same register (rotate)
                    a[i] = __builtin_amdgcn_alignbit(a[i], a[i], 13);
                else if constexpr (OP == 8)
                    a[i] = (a[i] & a[(i + 1) & 7]) | b;
                else if constexpr (OP == 9)  // alignbit, shift in a VGPR
                    a[i] = __builtin_amdgcn_alignbit(a[i], a[(i + 1) & 7], vs);
                else if constexpr (OP == 10)  // alignbit, shift in an SGPR
                    a[i] = __builtin_amdgcn_alignbit(a[i], a[(i + 1) & 7], ss);
                else if constexpr (OP == 11)  // bitop3 with an inline-constant operand
                    a[i] = __builtin_amdgcn_bitop3_b32(a[i], a[(i + 1) & 7], 0x3Fu, 0x96);
                else if constexpr (OP == 12)  // VOP2 xor with an SGPR operand
                    a[i] = a[i] ^ ss2[i & 1];
                else if constexpr (OP == 13)  // alignbit, VGPR shift, 3 distinct VGPRs per instruction
                    a[i] = __builtin_amdgcn_alignbit(a[i], a[(i + 1) & 7], vsh[i & 3]);
                else  // v_lshl_or_b32 (VOP3, all VGPR)
                    a[i] = (a[i] << 3) | a[(i + 1) & 7];
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int NB, int NA>
__global__ __launch_bounds__(256) void k_mix(uint32_t* out, int iters, unsigned long long* clk) {
    uint32_t a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * (i + 3) + blockIdx.x * 7 + i;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
#pragma unroll
            for (int i = 0; i < NB; ++i)
                a[i & 15] = (k & 1) ? __builtin_amdgcn_bitop3_b32(a[i & 15], a[(i + 5) & 15], a[(i + 11) & 15], 0xD2) : __builtin_amdgcn_bitop3_b32(a[i & 15], a[(i + 5) & 15], a[(i + 11) & 15], 0x96);
#pragma unroll
            for (int i = 0; i < NA; ++i)
                a[(i + 8) & 15] = __builtin_amdgcn_alignbit(a[(i + 8) & 15], a[(i + 3) & 15], 5 + (i & 7) * 3);
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) x ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <bool FULL>
__global__ __launch_bounds__(256) void k_perm(uint32_t* out, int iters, unsigned long long* clk) {
    mk::State s;
#pragma unroll
    for (int i = 0; i < 25; ++i) {
        s.lo[i] = threadIdx.x * 2654435761u + i;
        s.hi[i] = blockIdx.x * 40503u + i;
    }
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (FULL) {
#pragma unroll
            for (int r = 0; r < 24; ++r) mk::round_fn(s, mk::kRcLo[r], mk::kRcHi[r]);
        } else {
            mk::keccak_f(s);
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 25; ++i) x ^= s.lo[i] ^ s.hi[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <typename F>
void run(const char* name, F launch, double ops_per_thread, int blocks, int threads) {
    uint32_t* out;
    unsigned long long* clk;
    CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
    CHECK(hipMalloc(&clk, 16));
    launch(out, clk);  // warm
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int reps = 5;
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) launch(out, clk);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    unsigned long long h[2];
    CHECK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
    const double sec = ms / 1e3 / reps;
    const double ops = ops_per_thread * blocks * threads;
    const double ghz = h[1] ? (double)h[0] / (double)h[1] * 0.1 : 0;
    printf("{\"bench\": \"%s\", \"blocks\": %d, \"ms\": %.3f, \"Tops\": %.2f, \"clock_GHz\": %.3f, "
           "\"Tops_per_GHz\": %.2f}\n",
           name, blocks, sec * 1e3, ops / sec / 1e12, ghz, ghz > 0 ? ops / sec / 1e12 / ghz : 0);
    CHECK(hipFree(out));
    CHECK(hipFree(clk));
}

int main(int argc, char** argv) {
    const int threads = 256;
    for (int wpb : {4}) {  // blocks per CU x 256 CUs (waves/SIMD = wpb)
        const int blocks = 256 * wpb;
        const int iters = 2000;
#define OPRUN(NAME, K) run(NAME, [&](uint32_t* o, unsigned long long* c) { hipLaunchKernelGGL(k_ops<K>, blocks, threads, 0, 0, o, iters, c); }, iters * 128.0, blocks, threads)
        OPRUN("bitop3_a_b_c", 0);
        OPRUN("alignbit_a_a1", 1);
        OPRUN("xor_a_a3", 2);
        OPRUN("bitop3_a_a1_a2", 3);
        OPRUN("bitop3_a_a4_b", 4);
        OPRUN("bitop3_a_a1_s", 5);
        OPRUN("alignbit_a_a3", 6);
        OPRUN("alignbit_a_a", 7);
        OPRUN("and_or", 8);
        OPRUN("alignbit_vgpr_shift", 9);
        OPRUN("alignbit_sgpr_shift", 10);
        OPRUN("bitop3_inline_const", 11);
        OPRUN("xor_sgpr", 12);
        OPRUN("alignbit_vgpr_shift4", 13);
        OPRUN("lshl_or", 14);
#define MIXRUN(NAME, B, A) run(NAME, [&](uint32_t* o, unsigned long long* c) { hipLaunchKernelGGL((k_mix<B, A>), blocks, threads, 0, 0, o, iters, c); }, iters * 8.0 * (B + A), blocks, threads)
        MIXRUN("mix_b16_a0", 16, 0);
        MIXRUN("mix_b0_a16", 0, 16);
        MIXRUN("mix_b16_a16", 16, 16);
        MIXRUN("mix_b32_a16", 32, 16);
        MIXRUN("mix_b16_a8", 16, 8);
        const int piters = 200;
        run("keccak_f_rolled4", [&](uint32_t* o, unsigned long long* c) { hipLaunchKernelGGL(k_perm<false>, blocks, threads, 0, 0, o, piters, c); },
            piters * 4320.0, blocks, threads);
        run("keccak_f_full", [&](uint32_t* o, unsigned long long* c) { hipLaunchKernelGGL(k_perm<true>, blocks, threads, 0, 0, o, piters, c); },
            piters * 4320.0, blocks, threads);
    }
    return 0;
}
