// HBM ceiling for the mapping kernel's traffic mix (dccrgx_map_ids_to_indices:
// read 8 B of id, write 24 B of indices and 4 B of level per id): the same
// three streams with no arithmetic, 4 ids per lane per pass (2 dwordx4 in,
// 6 + 1 dwordx4 out, non-temporal), grid-stride; and a plain copy.
//   hipcc --offload-arch=gfx950 -O3 map_mix.hip -o map_mix && ./map_mix
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_mix(const u32x4* __restrict__ ids, u32x4* __restrict__ idx,
                                             u32x4* __restrict__ lvl, size_t n4)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const size_t w0 = 2 * (i & ~(size_t)63) + (i & 63);  // lane-contiguous loads too
        const u32x4 a = __builtin_nontemporal_load(ids + w0), b = __builtin_nontemporal_load(ids + w0 + 64);
#pragma unroll
        for (int k = 0; k < 6; k++)  // the wave's 6 x 64 outputs one contiguous run, lane-contiguous per store
            __builtin_nontemporal_store(k & 1 ? b + (unsigned)k : a + (unsigned)k, idx + 6 * (i & ~(size_t)63) + 64 * k + (i & 63));
        __builtin_nontemporal_store(a ^ b, lvl + i);
    }
}

__global__ void __launch_bounds__(256) k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        __builtin_nontemporal_store(a[i], b + i);
}

int main()
{
    const size_t nid = 1ull << 26, n4 = nid / 4;
    u32x4 *ids, *idx, *lvl;
    hipMalloc(&ids, nid * 8);
    hipMalloc(&idx, nid * 24);
    hipMalloc(&lvl, nid * 4);
    hipMemset(ids, 1, nid * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int grid : {2048, 4096, 8192, 16384, 65536}) {
        hipLaunchKernelGGL(k_mix, dim3(grid), dim3(256), 0, 0, ids, idx, lvl, n4);
        hipEventRecord(e0);
        for (int r = 0; r < 10; r++) hipLaunchKernelGGL(k_mix, dim3(grid), dim3(256), 0, 0, ids, idx, lvl, n4);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 10;
        printf("mix r8 w28 grid %6d: %.4f ms  %.0f GB/s  frac %.3f\n", grid, ms, 36.0 * nid / ms / 1e6,
               36.0 * nid / ms / 1e6 / 8000);
    }
    for (int grid : {4096, 16384}) {
        const size_t n = nid * 24 / 16;
        hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, idx, (u32x4*)ids, nid * 8 / 16);
        hipEventRecord(e0);
        for (int r = 0; r < 10; r++) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, (const u32x4*)idx, idx + n / 2, n / 2);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 10;
        printf("copy r1 w1 grid %6d: %.4f ms  %.0f GB/s\n", grid, ms, 2.0 * (n / 2) * 16 / ms / 1e6);
    }
    return 0;
}
