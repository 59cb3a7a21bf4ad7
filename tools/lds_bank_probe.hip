// Probe: LDS bank conflicts of ds_read_b128 / ds_write_b128 by lane address
// pattern (16-B slot of lane l), to pick a conflict-free record layout for a
// 160-B lane stride (k_struct_lock).  One kernel per pattern, 1 workgroup of
// 64 threads, 4096 reads each; run under
//   rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -- ./lds_bank_probe
// and divide the conflict cycles by the LDS instructions per pattern.
// Build: hipcc --offload-arch=gfx950 -O3 lds_bank_probe.hip -o lds_bank_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ uint32_t slot_of(int P, uint32_t l) {
    switch (P) {
        case 0: return 10u * l;                          // plain 160-B stride
        case 1: return 10u * l + ((l >> 3) & 1u);        // +1 unit when bit 3 set
        case 2: return 9u * l;                           // odd stride
        case 3: return l;                                // contiguous
        case 4: return 10u * l + ((l >> 2) & 1u);        // +1 when bit 2 set
        case 5: return 10u * l + ((l >> 4) & 1u);        // +1 when bit 4 set
        case 6: return 10u * l + ((l >> 3) & 7u);        // +0..7 by bits 3-5
        case 7: return 10u * l + ((l >> 2) & 1u) + 2u * ((l >> 3) & 1u);
        case 8: return 10u * l + (l >> 3);               // +0..7 by bits 3-5
        default: return 10u * l + (((l >> 2) ^ (l >> 3)) & 1u);  // 9: bit 2 xor bit 3 (k_struct_lock)
    }
}

template <int P, bool WRITE>
__global__ __launch_bounds__(64) void k_probe(uint4* out, int iters) {
    __shared__ uint4 buf[64 * 12];
    const uint32_t l = threadIdx.x;
    for (uint32_t i = l; i < 64 * 12; i += 64) buf[i] = make_uint4(i, i, i, i);
    __syncthreads();
    const uint32_t s = slot_of(P, l) % (64 * 12);
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int k = 0; k < iters; ++k) {
        if (WRITE) {
            buf[s] = make_uint4(k, k, k, k);
        } else {
            const uint4 v = buf[s];
            acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    out[l] = acc;
}

template <int P>
void run(uint4* d) {
    hipLaunchKernelGGL((k_probe<P, false>), dim3(1), dim3(64), 0, 0, d, 4096);
    hipLaunchKernelGGL((k_probe<P, true>), dim3(1), dim3(64), 0, 0, d, 4096);
}

int main() {
    uint4* d;
    if (hipMalloc(&d, 64 * 16) != hipSuccess) return 1;
    run<0>(d); run<1>(d); run<2>(d); run<3>(d); run<4>(d); run<5>(d); run<6>(d); run<7>(d); run<8>(d); run<9>(d);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("ok\n");
    return 0;
}
