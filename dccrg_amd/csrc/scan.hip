// scan.hip -- device prefix sums for CSR row pointers (count -> scan -> fill).
//
// Three launches: per-tile inclusive scans (wave prefix by cross-lane adds,
// wave totals through LDS) with a per-tile total; one workgroup scans the
// tile totals; every tile adds its exclusive offset.  Integer, so the result
// is exact and independent of the tiling.
#include "grid.hpp"

namespace dccrgx {

namespace {

constexpr int ST = 256;        // threads per tile
constexpr int SE = 4;          // elements per thread
constexpr int STILE = ST * SE;

__device__ __forceinline__ uint64_t wave_inclusive(uint64_t v, int lane)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t u = __shfl_up(v, d);
        if (lane >= d) v += u;
    }
    return v;
}

// block-wide inclusive scan of one value per thread; returns the block total
__device__ __forceinline__ uint64_t block_inclusive(uint64_t& v, uint64_t* wtot)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    v = wave_inclusive(v, lane);
    if (lane == 63) wtot[w] = v;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int k = 0; k < ST / 64; k++) {
        before += k < w ? wtot[k] : 0;
        all += wtot[k];
    }
    __syncthreads();
    v += before;
    return all;
}

__global__ void __launch_bounds__(ST) k_scan_tiles(uint64_t* __restrict__ x, uint64_t m,
                                                   uint64_t* __restrict__ tile_sum, uint64_t* __restrict__ zero)
{
    __shared__ uint64_t wtot[ST / 64];
    if (zero && blockIdx.x == 0 && threadIdx.x == 0) *zero = 0;  // a CSR's row[0] (no separate memset launch)
    const uint64_t base = (uint64_t)blockIdx.x * STILE + (uint64_t)threadIdx.x * SE;
    uint64_t e[SE];
    uint64_t t = 0;
#pragma unroll
    for (int k = 0; k < SE; k++) {
        e[k] = base + k < m ? x[base + k] : 0;
        t += e[k];
        e[k] = t;  // thread-local inclusive
    }
    uint64_t v = t;
    const uint64_t all = block_inclusive(v, wtot);
    const uint64_t before = v - t;
#pragma unroll
    for (int k = 0; k < SE; k++)
        if (base + k < m) x[base + k] = e[k] + before;
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = all;
}

// one workgroup: exclusive scan of the tile totals in place
__global__ void __launch_bounds__(ST) k_scan_sums(uint64_t* __restrict__ s, uint64_t nt)
{
    __shared__ uint64_t wtot[ST / 64];
    uint64_t carry = 0;
    for (uint64_t b = 0; b < nt; b += ST) {
        const uint64_t i = b + threadIdx.x;
        const uint64_t own = i < nt ? s[i] : 0;
        uint64_t v = own;
        const uint64_t all = block_inclusive(v, wtot);
        if (i < nt) s[i] = carry + v - own;
        carry += all;
    }
}

__global__ void __launch_bounds__(ST) k_scan_add(uint64_t* __restrict__ x, uint64_t m,
                                                 const uint64_t* __restrict__ off)
{
    const uint64_t o = off[blockIdx.x];
    if (!o) return;
    const uint64_t base = (uint64_t)blockIdx.x * STILE + (uint64_t)threadIdx.x * SE;
#pragma unroll
    for (int k = 0; k < SE; k++)
        if (base + k < m) x[base + k] += o;
}

}  // namespace

static int inclusive_scan(uint64_t* x, uint64_t m, hipStream_t st, uint64_t* zero)
{
    if (!m) {
        if (zero) DX_HIP(hipMemsetAsync(zero, 0, 8, st));
        return DCCRGX_OK;
    }
    const uint64_t nt = (m + STILE - 1) / STILE;
    DX_CHECK(nt < (1ull << 31), DCCRGX_EINVAL, "scan of %llu elements", (unsigned long long)m);
    uint64_t* sums = nullptr;
    DX_HIP(ds_malloc(&sums, nt * 8, st));
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)nt), dim3(ST), 0, st, x, m, sums, zero);
    if (nt > 1) {
        hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(ST), 0, st, sums, nt);
        hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nt), dim3(ST), 0, st, x, m, (const uint64_t*)sums);
    }
    DX_HIP(hipGetLastError());
    DX_HIP(ds_free(sums, st));
    return DCCRGX_OK;
}

int device_inclusive_scan(uint64_t* x, uint64_t m, hipStream_t st) { return inclusive_scan(x, m, st, nullptr); }

int device_scan_rows(uint64_t* row, uint64_t n, hipStream_t st, uint64_t* total)
{
    DX_TRY(inclusive_scan(row + 1, n, st, row));  // row[0] = 0 written by the first tile
    if (total) {  // through a pinned word: a pageable read-back costs a staging copy
        static thread_local uint64_t* word = nullptr;
        if (!word) DX_HIP(hipHostMalloc((void**)&word, 64, hipHostMallocDefault));
        DX_HIP(hipMemcpyAsync(word, row + n, 8, hipMemcpyDeviceToHost, st));
        DX_HIP(hipStreamSynchronize(st));
        *total = *word;
    }
    return DCCRGX_OK;
}

}  // namespace dccrgx
