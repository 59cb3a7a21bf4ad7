#include <hip/hip_runtime.h>
#include <cstdio>
#include "keccak_dev.hpp"
using namespace mk::spread;
using mk::xor3;
using mk::chi3;
__global__ __launch_bounds__(64) void k(const uint32_t* in, uint32_t* out) {
    const uint32_t L = threadIdx.x;
    const Lane c = lane_consts(L);
    uint32_t v = in[L], w = in[64 + L];
    const uint32_t t = v ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kRor8, 0xB, 0xF, false);
    out[0 * 64 + L] = t;
    const auto a = __builtin_amdgcn_permlane16_swap(t, t, false, false);
    out[1 * 64 + L] = a[0];
    out[2 * 64 + L] = a[1];
    const uint32_t s = a[0] ^ a[1];
    const auto b = __builtin_amdgcn_permlane32_swap(s, s, false, false);
    out[3 * 64 + L] = b[0];
    out[4 * 64 + L] = b[1];
    out[5 * 64 + L] = colsum(v);
    out[6 * 64 + L] = dpp<kShl1>(v);
    out[7 * 64 + L] = dpp<kShr1>(v);
    out[8 * 64 + L] = dpp<kShl4>(v);
    out[9 * 64 + L] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)c.src, (int)v);
    uint32_t e = v, o = w;
    {
        const uint32_t ce = colsum(e), co = colsum(o);
        const uint32_t me = sel(c.wrap, dpp<kShl4>(ce), dpp<kShr1>(ce));
        const uint32_t mo = sel(c.wrap, dpp<kShl4>(co), dpp<kShr1>(co));
        out[14 * 64 + L] = me;
        out[15 * 64 + L] = mo;
        e = xor3(e, me, __builtin_amdgcn_alignbit(dpp<kShl1>(co), dpp<kShl1>(co), 31u));
        o = xor3(o, mo, dpp<kShl1>(ce));
        out[16 * 64 + L] = e;
        out[17 * 64 + L] = o;
        const uint32_t t1 = __builtin_amdgcn_alignbit(e, e, c.sh1);
        const uint32_t t2 = __builtin_amdgcn_alignbit(o, o, c.sh2);
        const uint32_t re = sel(c.swap, t2, t1), ro = sel(c.swap, t1, t2);
        out[18 * 64 + L] = re;
        out[19 * 64 + L] = ro;
        const uint32_t be = (uint32_t)__builtin_amdgcn_ds_bpermute((int)c.src, (int)re);
        const uint32_t bo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)c.src, (int)ro);
        out[20 * 64 + L] = be;
        out[21 * 64 + L] = bo;
        e = __builtin_amdgcn_bitop3_b32(chi3(be, dpp<kShl1>(be), dpp<kShl2>(be)), c.iota, 0x12345678u, 0x78);
        o = __builtin_amdgcn_bitop3_b32(chi3(bo, dpp<kShl1>(bo), dpp<kShl2>(bo)), c.iota, 0x9abcdef0u, 0x78);
    }
    out[10 * 64 + L] = e;
    out[11 * 64 + L] = o;
    out[12 * 64 + L] = c.src;
    out[13 * 64 + L] = c.sh1 | (c.sh2 << 8) | ((c.swap & 1u) << 16) | ((c.wrap & 1u) << 17) | (c.i << 24);
}
int main() {
    uint32_t h[128], r[22 * 64];
    uint64_t x = 88172645463325252ull;
    for (int i = 0; i < 128; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = (uint32_t)x; }
    uint32_t *di, *dout;
    hipMalloc(&di, sizeof h); hipMalloc(&dout, sizeof r);
    hipMemcpy(di, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, 1, 64, 0, 0, di, dout);
    hipMemcpy(r, dout, sizeof r, hipMemcpyDeviceToHost);
    printf("{\"in\": [");
    for (int i = 0; i < 128; ++i) printf("%u%s", h[i], i < 127 ? "," : "");
    printf("], \"out\": [");
    for (int i = 0; i < 22 * 64; ++i) printf("%u%s", r[i], i < 22 * 64 - 1 ? "," : "");
    printf("]}\n");
    return 0;
}
