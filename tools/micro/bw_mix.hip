// HBM ceiling for the stencil's traffic mix: read 1 stream, write 2 streams
// (the 3-D GoL step reads is_alive, writes is_alive' and the count), against
// a plain copy (read 1, write 1).  dwordx4 per lane, grid-stride, NT stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int NT>
__global__ void __launch_bounds__(256) k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        u32x4 v = a[i];
        if (NT) __builtin_nontemporal_store(v, b + i);
        else b[i] = v;
    }
}

template <int NT>
__global__ void __launch_bounds__(256) k_r1w2(const u32x4* __restrict__ a, u32x4* __restrict__ b,
                                              u32x4* __restrict__ c, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        u32x4 v = a[i];
        u32x4 w = v ^ 0x01010101u;
        if (NT) {
            __builtin_nontemporal_store(v + 1u, b + i);
            __builtin_nontemporal_store(w, c + i);
        } else {
            b[i] = v + 1u;
            c[i] = w;
        }
    }
}

// U independent dwordx4 loads in flight per lane, block-contiguous chunks;
// NTL: non-temporal loads
template <int U, bool NTL>
__global__ void __launch_bounds__(256) k_r1w2_u(const u32x4* __restrict__ a, u32x4* __restrict__ b,
                                                u32x4* __restrict__ c, size_t n)
{
    const size_t chunk = 256 * U;  // per block per iteration
    for (size_t base = blockIdx.x * chunk; base < n; base += (size_t)gridDim.x * chunk) {
        u32x4 v[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t i = base + k * 256 + threadIdx.x;
            v[k] = i < n ? (NTL ? __builtin_nontemporal_load(a + i) : a[i]) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t i = base + k * 256 + threadIdx.x;
            if (i < n) {
                __builtin_nontemporal_store(v[k] + 1u, b + i);
                __builtin_nontemporal_store(v[k] ^ 0x01010101u, c + i);
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_write(u32x4* __restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        u32x4 v = {(unsigned)i, 1u, 2u, 3u};
        __builtin_nontemporal_store(v, b + i);
    }
}

int main(int argc, char** argv)
{
    const size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 8ull) << 30;  // per array
    const size_t n = bytes / 16;
    u32x4 *a, *b, *c;
    if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&c, bytes)) return 1;
    hipMemset(a, 1, bytes);
    hipMemset(b, 0, bytes);
    hipMemset(c, 0, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int blocks : {8192, 32768, 131072}) {
        float ms;
        auto run = [&](auto launch, double moved, const char* name) {
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            for (int r = 0; r < 5; r++) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            printf("%-12s blocks %6d  %.1f GB/s\n", name, blocks, moved * 5 / (ms * 1e-3) / 1e9);
        };
        run([&] { hipLaunchKernelGGL(k_r1w2<1>, dim3(blocks), dim3(256), 0, 0, a, b, c, n); }, 3.0 * bytes, "r1w2_nt");
        run([&] { hipLaunchKernelGGL((k_r1w2_u<1, false>), dim3(blocks), dim3(256), 0, 0, a, b, c, n); }, 3.0 * bytes, "u1");
        run([&] { hipLaunchKernelGGL((k_r1w2_u<1, true>), dim3(blocks), dim3(256), 0, 0, a, b, c, n); }, 3.0 * bytes, "u1_ntl");
        run([&] { hipLaunchKernelGGL((k_r1w2_u<4, false>), dim3(blocks), dim3(256), 0, 0, a, b, c, n); }, 3.0 * bytes, "u4");
        run([&] { hipLaunchKernelGGL((k_r1w2_u<4, true>), dim3(blocks), dim3(256), 0, 0, a, b, c, n); }, 3.0 * bytes, "u4_ntl");
        run([&] { hipLaunchKernelGGL((k_r1w2_u<8, false>), dim3(blocks), dim3(256), 0, 0, a, b, c, n); }, 3.0 * bytes, "u8");
        run([&] { hipLaunchKernelGGL((k_r1w2_u<8, true>), dim3(blocks), dim3(256), 0, 0, a, b, c, n); }, 3.0 * bytes, "u8_ntl");
    }
    return 0;
}
