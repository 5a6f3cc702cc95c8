// us_sweep.hip -- time the staged user-stencil kernel (include/dccrgx_stencil.hpp
// k_staged) in several tilings / prefetch depths on a raw 2048^3 u32 slab,
// without the library: the game-of-life functor of examples/user_stencil.hip.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include us_sweep.hip -o us_sweep
//   ./us_sweep [n]
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "dccrgx_stencil.hpp"

using namespace dccrgx_user;

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

struct Gol {
    uint32_t *out, *cnt;
    unsigned long long* checked;  // cells the staged kernel ran with per-item tests
    template <class C>
    __device__ void operator()(const C& cell) const
    {
        uint32_t n = 0;
        cell.for_each_neighbor([&](const auto& nb) { n += nb.value(0) != 0u ? 1u : 0u; });
        cnt[cell.slot] = n;
        out[cell.slot] = n == 3u ? 1u : (n == 2u ? cell.value(0) : 0u);
    }
};

__global__ void k_init(uint32_t* f, uint64_t n)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        uint64_t z = i + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        f[i] = ((z ^ (z >> 31)) % 1000u) < 200u ? 1u : 0u;
    }
}

__global__ void k_sum(const uint32_t* f, uint64_t n, unsigned long long* out)
{
    unsigned long long s = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) s += f[i] * (i % 977 + 1);
    atomicAdd(out, s);
}

// the same bytes, no stencil: read in, write out and cnt
__global__ void k_copy3(const uint4* in, uint4* out, uint4* cnt, uint64_t n4)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256) {
        uint4 v = in[i];
        out[i] = v;
        cnt[i] = v;
    }
}

template <int NW, int NB, int PF>
float run(const detail::StagedGeo& g0, Fields<uint32_t, 1> fld, Gol f, int64_t want, int reps)
{
    detail::StagedGeo g = g0;
    g.tiles_a = (uint32_t)((g.la + 63) / 64);
    g.tiles_b = (uint32_t)((g.lb + NW * NB - 1) / (NW * NB));
    const int64_t tiles = (int64_t)g.tiles_a * g.tiles_b, nsl = g.s1 - g.s0;
    int64_t chunks = (want + tiles - 1) / tiles;
    chunks = chunks < 1 ? 1 : (chunks > nsl ? nsl : chunks);
    g.chunk = (nsl + chunks - 1) / chunks;
    g.nwg = (uint32_t)(tiles * ((nsl + g.chunk - 1) / g.chunk));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((detail::k_staged<uint32_t, 1, DCCRGX_SHAPE_CUBE1, NW, NB, 4, PF, Gol>), dim3(g.nwg),
                       dim3(64 * NW), 0, 0, g, fld, f);
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++)
        hipLaunchKernelGGL((detail::k_staged<uint32_t, 1, DCCRGX_SHAPE_CUBE1, NW, NB, 4, PF, Gol>), dim3(g.nwg),
                           dim3(64 * NW), 0, 0, g, fld, f);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char** argv)
{
    const uint64_t n = argc > 1 ? atoll(argv[1]) : 2048;
    const uint64_t S = n * n, ns = n + 2, tot = S * ns;
    uint32_t *in, *out, *cnt;
    CK(hipMalloc(&in, tot * 4));
    CK(hipMalloc(&out, tot * 4));
    CK(hipMalloc(&cnt, tot * 4));
    hipLaunchKernelGGL(k_init, dim3(8192), dim3(256), 0, 0, in, tot);
    CK(hipMemset(out, 0, tot * 4));
    CK(hipMemset(cnt, 0, tot * 4));
    unsigned long long* dsum;
    CK(hipMalloc(&dsum, 8));
    detail::StagedGeo g{};
    g.la = g.lb = g.lc = n;
    g.S = S;
    g.lo = 0;
    g.hi = S * n;
    g.cbase = -1;
    g.s0 = 2;  // canonical 1 .. n-2: the MID planes of a periodic C
    g.s1 = (int64_t)n;
    g.pa = g.pb = 0;
    g.pc = 1;
    g.inv[0] = 0;
    g.inv[1] = 1;
    g.inv[2] = 2;
    g.scale = 1;
    Fields<uint32_t, 1> fld{{in}};
    unsigned long long* checked;
    CK(hipMalloc(&checked, 8));
    CK(hipMemset(checked, 0, 8));
    Gol f{out, cnt, checked};
    const double cells = (double)S * (double)(n - 2);
    auto report = [&](const char* name, float ms) {
        CK(hipMemset(dsum, 0, 8));
        hipLaunchKernelGGL(k_sum, dim3(8192), dim3(256), 0, 0, cnt, tot, dsum);
        unsigned long long h;
        CK(hipMemcpy(&h, dsum, 8, hipMemcpyDeviceToHost));
        unsigned long long nc;
        CK(hipMemcpy(&nc, checked, 8, hipMemcpyDeviceToHost));
        CK(hipMemset(checked, 0, 8));
        printf("%-28s %8.3f ms  %7.1f GB/s  frac %.3f  sum %llu  checked %llu\n", name, ms, 12.0 * cells / ms / 1e6,
               12.0 * cells / ms / 1e6 / 8000.0, h, nc);
        fflush(stdout);
        CK(hipMemset(cnt, 0, tot * 4));
    };
    const int reps = 5;
    {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        hipLaunchKernelGGL(k_copy3, dim3(16384), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, (uint4*)cnt, tot / 4);
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; r++)
            hipLaunchKernelGGL(k_copy3, dim3(16384), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, (uint4*)cnt,
                               tot / 4);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s %8.3f ms  %7.1f GB/s (read 1 write 2 stream)\n", "copy3", ms / reps, 12.0 * tot / (ms / reps) / 1e6);
        CK(hipMemset(cnt, 0, tot * 4));
    }
    for (int64_t want : {131072, 262144, 524288, 1048576}) {
        char nm[64];
#define V(NW, NB, PF)                                                      \
    snprintf(nm, sizeof nm, "NW%d NB%d PF%d want%lld", NW, NB, PF, (long long)want); \
    report(nm, run<NW, NB, PF>(g, fld, f, want, reps));
        V(4, 4, 1)
        V(4, 6, 1)
        V(4, 5, 1)
        V(8, 4, 1)
    }
    return 0;
}
