// Probe: bit-sliced Keccak-f[1600] throughput on gfx950 (research, not product).
//
// Layout: one wave = 32 independent states; lane z (0..63) holds slice z of
// every state: VGPR A[x][y] bit s = bit z of lane (x,y) of state s.
//   theta: column parity per lane (bitop3), rot-by-1 along z = take C from
//          lane z-1 (DPP wave_ror / ds_bpermute), apply with v_xor.
//   rho:   rotation along z = cross-lane rotate of a whole register
//          (ds_bpermute with a per-rotation address), pi = renaming.
//   chi:   bitop3 per lane.   iota: per-lane mask from the round constant.
// The lane-sliced kernel spends 58 half-rate v_alignbit per round per state;
// here those become 24 LDS-crossbar bpermutes + 5 lane shifts per 32 states.
// Checks: the result equals the lane-sliced keccak_f on the same 32 states.
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

__constant__ uint64_t kRC64[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

template <int I>
struct Rho {
    static constexpr int v = MK_RHO(I);
};

__device__ __forceinline__ uint32_t from_lane_minus(uint32_t v, uint32_t addr) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)addr, (int)v);
}

#ifndef USE_DPP
#define USE_DPP 1
#endif

// value of lane z-1 (lane 0 gets lane 63)
__device__ __forceinline__ uint32_t lane_prev(uint32_t v, uint32_t addr_prev) {
#if USE_DPP
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x13C /* wave_ror:1 */, 0xF, 0xF, false);
#else
    return from_lane_minus(v, addr_prev);
#endif
}

template <int I>
__device__ __forceinline__ void rho_pi_bs(const uint32_t (&A)[25], uint32_t (&B)[25], const uint32_t (&addr)[64]) {
    constexpr int x = I % 5, y = I / 5;
    constexpr int dst = y + 5 * ((2 * x + 3 * y) % 5);
    constexpr int r = Rho<I>::v;
    if constexpr (r == 0)
        B[dst] = A[I];
    else
        B[dst] = from_lane_minus(A[I], addr[r]);
}

template <int... Is>
__device__ __forceinline__ void rho_pi_bs_all(const uint32_t (&A)[25], uint32_t (&B)[25], const uint32_t (&addr)[64],
                                              std::integer_sequence<int, Is...>) {
    (rho_pi_bs<Is>(A, B, addr), ...);
}

__device__ __forceinline__ void round_bs(uint32_t (&A)[25], const uint32_t (&addr)[64], uint32_t rcmask) {
    uint32_t C[5], E[5];
#pragma unroll
    for (int x = 0; x < 5; ++x) C[x] = mk::xor3(mk::xor3(A[x], A[x + 5], A[x + 10]), A[x + 15], A[x + 20]);
#pragma unroll
    for (int x = 0; x < 5; ++x) E[x] = C[(x + 4) % 5] ^ lane_prev(C[(x + 1) % 5], addr[1]);
#pragma unroll
    for (int i = 0; i < 25; ++i) A[i] ^= E[i % 5];
    uint32_t B[25];
    rho_pi_bs_all(A, B, addr, std::make_integer_sequence<int, 25>{});
#pragma unroll
    for (int y = 0; y < 5; ++y)
#pragma unroll
        for (int x = 0; x < 5; ++x)
            A[x + 5 * y] = mk::chi3(B[x + 5 * y], B[(x + 1) % 5 + 5 * y], B[(x + 2) % 5 + 5 * y]);
    A[0] ^= rcmask;
}

// addr[r] = byte address of lane (z - r) mod 64
__device__ __forceinline__ void make_addr(uint32_t (&addr)[64]) {
    const uint32_t z = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < 64; ++r) addr[r] = ((z - r) & 63u) * 4u;
}

__device__ __forceinline__ uint32_t rc_mask(int round) {
    const uint32_t z = threadIdx.x & 63;
    return ((kRC64[round] >> z) & 1ull) ? 0xFFFFFFFFu : 0u;
}

__global__ __launch_bounds__(256) void k_bs_perm(uint32_t* out, int iters) {
    uint32_t addr[64];
    make_addr(addr);
    uint32_t A[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) A[i] = (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u + i * 977u);
    for (int it = 0; it < iters; ++it) {
#pragma unroll 2
        for (int r = 0; r < 24; ++r) round_bs(A, addr, rc_mask(r));
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 25; ++i) x ^= A[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// Correctness: 32 random states per wave, transposed in and out on the host.
__global__ void k_bs_once(const uint32_t* in_slices, uint32_t* out_slices) {
    uint32_t addr[64];
    make_addr(addr);
    uint32_t A[25];
    const uint32_t z = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 25; ++i) A[i] = in_slices[i * 64 + z];
#pragma unroll 1
    for (int r = 0; r < 24; ++r) round_bs(A, addr, rc_mask(r));
#pragma unroll
    for (int i = 0; i < 25; ++i) out_slices[i * 64 + z] = A[i];
}

__global__ __launch_bounds__(256) void k_lane_perm(uint32_t* out, int iters) {
    mk::State s;
#pragma unroll
    for (int i = 0; i < 25; ++i) {
        s.lo[i] = threadIdx.x * 2654435761u + i;
        s.hi[i] = blockIdx.x * 40503u + i;
    }
    for (int it = 0; it < iters; ++it) mk::keccak_f(s);
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 25; ++i) x ^= s.lo[i] ^ s.hi[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

static void keccak_f_host(uint64_t A[25]) {
    static const int R[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
    static const uint64_t RC[24] = {
        0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
        0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
        0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
        0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
        0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
        0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
    auto rot = [](uint64_t v, int n) { return n ? (v << n) | (v >> (64 - n)) : v; };
    for (int r = 0; r < 24; ++r) {
        uint64_t C[5], D[5], B[25];
        for (int x = 0; x < 5; ++x) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
        for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rot(C[(x + 1) % 5], 1);
        for (int i = 0; i < 25; ++i) A[i] ^= D[i % 5];
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y) B[y + 5 * ((2 * x + 3 * y) % 5)] = rot(A[x + 5 * y], R[x + 5 * y]);
        for (int y = 0; y < 5; ++y)
            for (int x = 0; x < 5; ++x) A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
        A[0] ^= RC[r];
    }
}

int main() {
    // ---- correctness
    uint64_t st[32][25];
    srand(7);
    for (int s = 0; s < 32; ++s)
        for (int i = 0; i < 25; ++i) st[s][i] = ((uint64_t)rand() << 33) ^ ((uint64_t)rand() << 11) ^ rand();
    uint32_t slices[25 * 64];
    memset(slices, 0, sizeof slices);
    for (int i = 0; i < 25; ++i)
        for (int z = 0; z < 64; ++z)
            for (int s = 0; s < 32; ++s) slices[i * 64 + z] |= (uint32_t)((st[s][i] >> z) & 1) << s;
    uint32_t *din, *dout;
    CHECK(hipMalloc(&din, sizeof slices));
    CHECK(hipMalloc(&dout, sizeof slices));
    CHECK(hipMemcpy(din, slices, sizeof slices, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_bs_once, 1, 64, 0, 0, din, dout);
    CHECK(hipDeviceSynchronize());
    uint32_t res[25 * 64];
    CHECK(hipMemcpy(res, dout, sizeof res, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int s = 0; s < 32; ++s) {
        keccak_f_host(st[s]);
        for (int i = 0; i < 25; ++i) {
            uint64_t v = 0;
            for (int z = 0; z < 64; ++z) v |= (uint64_t)((res[i * 64 + z] >> s) & 1) << z;
            bad += v != st[s][i];
        }
    }
    printf("{\"bitslice_correct\": %s, \"bad_lanes\": %d}\n", bad ? "false" : "true", bad);

    // ---- throughput
    for (int blocks : {1024, 2048, 4096}) {
        uint32_t* o;
        CHECK(hipMalloc(&o, (size_t)blocks * 256 * 4));
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        const int iters = 100;
        float ms_bs = 0, ms_lane = 0;
        hipLaunchKernelGGL(k_bs_perm, blocks, 256, 0, 0, o, iters);
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_bs_perm, blocks, 256, 0, 0, o, iters);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms_bs, a, b));
        hipLaunchKernelGGL(k_lane_perm, blocks, 256, 0, 0, o, iters);
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_lane_perm, blocks, 256, 0, 0, o, iters);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms_lane, a, b));
        // states: bitsliced = 32 per wave, lane-sliced = 64 per wave
        const double waves = blocks * 4.0;
        const double perms_bs = waves * 32 * iters, perms_lane = waves * 64 * iters;
        printf("{\"blocks\": %d, \"bitslice_perms_per_s\": %.4g, \"lane_perms_per_s\": %.4g, \"ratio\": %.3f}\n", blocks,
               perms_bs / (ms_bs / 1e3), perms_lane / (ms_lane / 1e3),
               (perms_bs / ms_bs) / (perms_lane / ms_lane));
        CHECK(hipFree(o));
    }
    return 0;
}
