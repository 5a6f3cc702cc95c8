// scan.hip -- device prefix sums for CSR row pointers (count -> scan -> fill).
//
// Up to 2048 tiles of 4096 elements (8.4 M rows): two launches -- the tile
// totals, then every tile sums the totals before it (at most 16 KB from L2)
// and scans itself.  Larger: three launches -- per-tile inclusive scans
// (wave prefix by cross-lane adds, wave totals through LDS) with a per-tile
// total; one workgroup scans the tile totals; every tile adds its exclusive
// offset.  Each launch of an adaptive step's chain costs a few microseconds
// whatever its size, so the short form matters there.  Integer, so the result
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

constexpr int T2 = 256;  // the two-launch form: threads per tile
constexpr int E2 = 16;   // elements per thread
constexpr int TILE2 = T2 * E2;
constexpr uint64_t MAX_TILES2 = 2048;

__device__ __forceinline__ uint64_t block_sum(uint64_t v, uint64_t* wtot)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) wtot[w] = v;
    __syncthreads();
    uint64_t all = 0;
#pragma unroll
    for (int k = 0; k < T2 / 64; k++) all += wtot[k];
    __syncthreads();
    return all;
}

template <class In>
__global__ void __launch_bounds__(T2) k_tile_totals(const In* __restrict__ x, uint64_t m, uint64_t* __restrict__ tot)
{
    __shared__ uint64_t wtot[T2 / 64];
    const uint64_t base = (uint64_t)blockIdx.x * TILE2;
    uint64_t t = 0;
#pragma unroll
    for (int k = 0; k < E2; k++) {
        const uint64_t i = base + (uint64_t)k * T2 + threadIdx.x;  // coalesced
        t += i < m ? (uint64_t)x[i] : 0;
    }
    const uint64_t all = block_sum(t, wtot);
    if (threadIdx.x == 0) tot[blockIdx.x] = all;
}

// out[i] = x[0] + ... + x[i] (out may be x); *zero = 0 when given
template <class In>
__global__ void __launch_bounds__(T2) k_tile_scan(const In* x, uint64_t m, const uint64_t* __restrict__ tot,
                                                  uint64_t* out, uint64_t* __restrict__ zero)
{
    __shared__ uint64_t wtot[T2 / 64];
    if (zero && blockIdx.x == 0 && threadIdx.x == 0) *zero = 0;  // a CSR's row[0]
    uint64_t o = 0;
    for (uint64_t j = threadIdx.x; j < blockIdx.x; j += T2) o += tot[j];
    o = block_sum(o, wtot);
    const uint64_t base = (uint64_t)blockIdx.x * TILE2 + (uint64_t)threadIdx.x * E2;
    uint64_t e[E2];
    uint64_t t = 0;
#pragma unroll
    for (int k = 0; k < E2; k++) {
        t += base + k < m ? (uint64_t)x[base + k] : 0;
        e[k] = t;  // thread-local inclusive
    }
    uint64_t v = t;
    block_inclusive(v, wtot);
    const uint64_t before = o + v - t;
#pragma unroll
    for (int k = 0; k < E2; k++)
        if (base + k < m) out[base + k] = e[k] + before;
}

__global__ void __launch_bounds__(256) k_copy_counts(const uint32_t* __restrict__ cnt, uint64_t n,
                                                     uint64_t* __restrict__ row)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) row[i + 1] = cnt[i];
}

}  // namespace

// out[i] = in[0] + ... + in[i] over m elements in two launches (m within
// MAX_TILES2 tiles); *zero = 0 when given
template <class In>
static int scan_two(const In* in, uint64_t m, uint64_t* out, uint64_t* zero, hipStream_t st)
{
    const uint64_t nt = (m + TILE2 - 1) / TILE2;
    uint64_t* tot = nullptr;
    DX_HIP(ds_malloc(&tot, nt * 8, st));
    hipLaunchKernelGGL((k_tile_totals<In>), dim3((unsigned)nt), dim3(T2), 0, st, in, m, tot);
    hipLaunchKernelGGL((k_tile_scan<In>), dim3((unsigned)nt), dim3(T2), 0, st, in, m, (const uint64_t*)tot, out, zero);
    DX_HIP(hipGetLastError());
    DX_HIP(ds_free(tot, st));
    return DCCRGX_OK;
}

static int inclusive_scan(uint64_t* x, uint64_t m, hipStream_t st, uint64_t* zero)
{
    if (!m) {
        if (zero) DX_HIP(hipMemsetAsync(zero, 0, 8, st));
        return DCCRGX_OK;
    }
    if ((m + TILE2 - 1) / TILE2 <= MAX_TILES2) return scan_two<uint64_t>(x, m, x, zero, st);
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

// row[0] = 0, row[i + 1] = cnt[0] + ... + cnt[i]
int device_scan_counts(const uint32_t* cnt, uint64_t n, uint64_t* row, hipStream_t st)
{
    if (n && (n + TILE2 - 1) / TILE2 <= MAX_TILES2) return scan_two<uint32_t>(cnt, n, row + 1, row, st);
    if (n) hipLaunchKernelGGL(k_copy_counts, dim3((unsigned)std::min<uint64_t>((n + 255) / 256, 65536)), dim3(256), 0,
                              st, cnt, n, row);
    DX_HIP(hipGetLastError());
    return inclusive_scan(row + 1, n, st, row);
}

int device_scan_rows(uint64_t* row, uint64_t n, hipStream_t st, uint64_t* total)
{
    DX_TRY(inclusive_scan(row + 1, n, st, row));  // row[0] = 0 written by the first tile
    return total ? device_scan_rows_total(row, n, st, total) : DCCRGX_OK;
}

// *total = row[n] (waits for the stream)
int device_scan_rows_total(const uint64_t* row, uint64_t n, hipStream_t st, uint64_t* total)
{
    {  // through a pinned word: a pageable read-back costs a staging copy
        static thread_local uint64_t* word = nullptr;
        if (!word) DX_HIP(hipHostMalloc((void**)&word, 64, hipHostMallocDefault));
        DX_HIP(hipMemcpyAsync(word, row + n, 8, hipMemcpyDeviceToHost, st));
        DX_HIP(hipStreamSynchronize(st));
        *total = *word;
    }
    return DCCRGX_OK;
}

}  // namespace dccrgx
