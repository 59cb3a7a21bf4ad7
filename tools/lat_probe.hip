// Probe: latency of ONE Keccak-f[1600] on a lone wave (the cost of a level
// at the narrow top of a Merkle tree), for the three state layouts in
// keccak_dev.hpp:
//   V0  one state per lane (mk::keccak_f)            64 states / wave
//   V1  two lanes per state, lo/hi halves (mk::pair)  32 states / wave
//   V2  two lanes per state, bit-interleaved (mk::ilv) 32 states / wave
//   V3  one state per wave, bit-interleaved (mk::spread) 1 state / wave
//   V4  one state per wave, lo/hi halves (mk::spread, _lh)  1 state / wave
// One workgroup of 64 threads runs `iters` dependent permutations; cycles
// from s_memtime.  Checks V1 and V2 against V0 on the same 32 states, V3
// on state 0.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../prysm_amd/csrc lat_probe.hip -o lat_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "keccak_dev.hpp"

#define CHECK(x)                                                         \
    do {                                                                 \
        hipError_t e = (x);                                              \
        if (e != hipSuccess) {                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));       \
            exit(1);                                                     \
        }                                                                \
    } while (0)

// io: 64 states x 50 dwords (lane i: lo at 2i, hi at 2i+1)
template <int V>
__global__ __launch_bounds__(64) void k_lat(uint32_t* io, int iters, unsigned long long* clk) {
    const uint32_t t = threadIdx.x;
    unsigned long long t0 = 0, t1 = 0;
    if constexpr (V == 0) {
        mk::State s;
        for (int i = 0; i < 25; ++i) {
            s.lo[i] = io[50 * t + 2 * i];
            s.hi[i] = io[50 * t + 2 * i + 1];
        }
        t0 = __builtin_amdgcn_s_memtime();
        for (int k = 0; k < iters; ++k) mk::keccak_f(s);
        t1 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < 25; ++i) {
            io[50 * t + 2 * i] = s.lo[i];
            io[50 * t + 2 * i + 1] = s.hi[i];
        }
    } else if constexpr (V == 1) {
        const uint32_t k2 = t >> 1, p = t & 1u;
        mk::pair::Half s;
        for (int i = 0; i < 25; ++i) s.v[i] = io[50 * k2 + 2 * i + p];
        t0 = __builtin_amdgcn_s_memtime();
        for (int k = 0; k < iters; ++k) mk::pair::keccak_f(s, p != 0);
        t1 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < 25; ++i) io[50 * k2 + 2 * i + p] = s.v[i];
    } else if constexpr (V == 3) {
        const mk::spread::Lane c = mk::spread::lane_consts(t);
        uint32_t e = mk::ilv::to_ilv(io[2 * c.i], io[2 * c.i + 1], 0);
        uint32_t o = mk::ilv::to_ilv(io[2 * c.i], io[2 * c.i + 1], 1);
        t0 = __builtin_amdgcn_s_memtime();
        for (int k = 0; k < iters; ++k) mk::spread::keccak_f(e, o, c);
        t1 = __builtin_amdgcn_s_memtime();
        // back to (lo, hi): spread16 of the even / odd words
        const uint32_t lo = mk::ilv::spread16(e) | (mk::ilv::spread16(o) << 1);
        const uint32_t hi = mk::ilv::spread16(e >> 16) | (mk::ilv::spread16(o >> 16) << 1);
        __syncthreads();
        if ((t & 7u) < 5u && (t >> 3) < 5u) {
            io[2 * c.i] = lo;
            io[2 * c.i + 1] = hi;
        }
    } else if constexpr (V == 4) {
        const mk::spread::LaneLH c = mk::spread::lane_consts_lh(t);
        uint32_t lo = io[2 * c.i], hi = io[2 * c.i + 1];
        t0 = __builtin_amdgcn_s_memtime();
        for (int k = 0; k < iters; ++k) mk::spread::keccak_f_lh(lo, hi, c);
        t1 = __builtin_amdgcn_s_memtime();
        __syncthreads();
        if ((t & 7u) < 5u && (t >> 3) < 5u) {
            io[2 * c.i] = lo;
            io[2 * c.i + 1] = hi;
        }
    } else {
        const uint32_t k2 = t >> 1, p = t & 1u;
        mk::ilv::Half s;
        for (int i = 0; i < 25; ++i) s.v[i] = mk::ilv::to_ilv(io[50 * k2 + 2 * i], io[50 * k2 + 2 * i + 1], p);
        t0 = __builtin_amdgcn_s_memtime();
        for (int k = 0; k < iters; ++k) mk::ilv::keccak_f(s, p);
        t1 = __builtin_amdgcn_s_memtime();
        uint32_t w[25];
        for (int i = 0; i < 25; ++i) w[i] = mk::ilv::from_ilv(s.v[i], p);
        for (int i = 0; i < 25; ++i) io[50 * k2 + 2 * i + p] = w[i];
    }
    if (t == 0) clk[0] = t1 - t0;
}

template <int V>
double run(const uint32_t* init, uint32_t* result, int iters) {
    uint32_t* d;
    unsigned long long* c;
    CHECK(hipMalloc(&d, 64 * 50 * 4));
    CHECK(hipMalloc(&c, 8));
    CHECK(hipMemcpy(d, init, 64 * 50 * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_lat<V>, 1, 64, 0, 0, d, iters, c);  // warm (changes d; reload)
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(d, init, 64 * 50 * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_lat<V>, 1, 64, 0, 0, d, iters, c);
    CHECK(hipDeviceSynchronize());
    unsigned long long cyc;
    CHECK(hipMemcpy(&cyc, c, 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(result, d, 64 * 50 * 4, hipMemcpyDeviceToHost));
    CHECK(hipFree(d));
    CHECK(hipFree(c));
    return (double)cyc / iters;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    static uint32_t init[64 * 50], r0[64 * 50], r1[64 * 50], r2[64 * 50], r3[64 * 50], r4[64 * 50];
    uint64_t x = 0x1234567887654321ull;
    for (int i = 0; i < 64 * 50; ++i) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        init[i] = (uint32_t)x;
    }
    const double c0 = run<0>(init, r0, iters);
    const double c1 = run<1>(init, r1, iters);
    const double c2 = run<2>(init, r2, iters);
    const double c3 = run<3>(init, r3, iters);
    const bool ok1 = memcmp(r0, r1, 32 * 50 * 4) == 0, ok2 = memcmp(r0, r2, 32 * 50 * 4) == 0;
    const double c4 = run<4>(init, r4, iters);
    const bool ok3 = memcmp(r0, r3, 50 * 4) == 0, ok4 = memcmp(r0, r4, 50 * 4) == 0;
    if (!ok3)
        for (int i = 0; i < 25; ++i)
            if (r0[2 * i] != r3[2 * i] || r0[2 * i + 1] != r3[2 * i + 1])
                fprintf(stderr, "spread lane %d: %08x%08x vs %08x%08x\n", i, r3[2 * i + 1], r3[2 * i], r0[2 * i + 1], r0[2 * i]);
    printf("{\"probe\": \"lone-wave keccak_f latency\", \"unroll\": %d, \"iters\": %d, "
           "\"cycles_per_perm\": {\"single_lane\": %.0f, \"pair_lohi\": %.0f, \"pair_interleaved\": %.0f, "
           "\"wave_spread\": %.0f, \"wave_spread_lohi\": %.0f}, \"match_pair\": %s, \"match_interleaved\": %s, "
           "\"match_spread\": %s, \"match_spread_lohi\": %s}\n",
           mk::kRoundUnroll, iters, c0, c1, c2, c3, c4, ok1 ? "true" : "false", ok2 ? "true" : "false",
           ok3 ? "true" : "false", ok4 ? "true" : "false");
    return (ok1 && ok2 && ok3 && ok4) ? 0 : 1;
}
