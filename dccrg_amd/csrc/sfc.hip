// sfc.hip -- space-filling-curve placement of the level-0 cells on the device
// (the reference's USE_SFC branch of create_level_0_cells,
// dccrg.hpp:8147-8220).
//
// The reference walks the level-0 cells in the order of sfc++'s curve and
// gives each process the same number of consecutive cells as its block
// partition (cells_per_process, procs_with_fewer: :8098-8114).  sfc++ is not
// part of the reference tree, so its curve cannot be reproduced; here the
// curve is the 3-D Hilbert curve (Skilling, "Programming the Hilbert curve",
// AIP Conf. Proc. 707, 2004: axes -> transpose -> interleave) over the
// smallest power-of-two cube holding the grid, cells outside the grid
// skipped.  One key per level-0 cell, a device radix sort of (key, cell),
// then the sorted positions are cut exactly as the block partition cuts ids.
// The result is a replicated owner table of the level-0 cells (the
// reference's cell_process holds the same information for every cell).
#include <hipcub/hipcub.hpp>

#include "grid.hpp"

namespace dccrgx {

namespace {

// Hilbert index of (x, y, z) with `b` bits per axis (x = X[0])
__host__ __device__ inline uint64_t hilbert3(uint32_t x, uint32_t y, uint32_t z, int b)
{
    uint32_t X[3] = {x, y, z};
    const uint32_t M = 1u << (b - 1);
    for (uint32_t Q = M; Q > 1; Q >>= 1) {  // inverse undo
        const uint32_t P = Q - 1;
        for (int i = 0; i < 3; i++) {
            if (X[i] & Q) {
                X[0] ^= P;
            } else {
                const uint32_t t = (X[0] ^ X[i]) & P;
                X[0] ^= t;
                X[i] ^= t;
            }
        }
    }
    X[1] ^= X[0];  // Gray encode
    X[2] ^= X[1];
    uint32_t t = 0;
    for (uint32_t Q = M; Q > 1; Q >>= 1)
        if (X[2] & Q) t ^= Q - 1;
    for (int i = 0; i < 3; i++) X[i] ^= t;
    uint64_t key = 0;
    for (int bit = b - 1; bit >= 0; bit--)
        for (int i = 0; i < 3; i++) key = (key << 1) | ((X[i] >> bit) & 1u);
    return key;
}

__global__ void __launch_bounds__(256) k_hilbert_keys(uint64_t lx, uint64_t ly, uint64_t n, int b,
                                                      uint64_t* __restrict__ keys, uint32_t* __restrict__ cells)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t x = i % lx, y = (i / lx) % ly, z = i / (lx * ly);
        keys[i] = hilbert3((uint32_t)x, (uint32_t)y, (uint32_t)z, b);
        cells[i] = (uint32_t)i;
    }
}

// position p on the curve -> the process the block partition gives id p + 1
__global__ void __launch_bounds__(256) k_assign(const uint32_t* __restrict__ sorted, uint64_t n, Partition P,
                                                int32_t* __restrict__ owner)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += stride)
        owner[sorted[p]] = part_owner(P, p + 1);
}

unsigned blocks(uint64_t n)
{
    uint64_t b = (n + 255) / 256;
    if (b > 256 * 16) b = 256 * 16;
    return (unsigned)(b ? b : 1);
}

// device buffers freed on every path
struct Bufs {
    std::vector<void*> p;
    ~Bufs()
    {
        for (void* q : p) (void)dx_free(q);
    }
    template <class T> int get(T** out, size_t bytes)
    {
        void* q = nullptr;
        DX_HIP(dx_malloc(&q, bytes ? bytes : 1));
        p.push_back(q);
        *out = (T*)q;
        return DCCRGX_OK;
    }
};

}  // namespace

int sfc_owners(const uint64_t length[3], int comm_size, hipStream_t st, std::vector<int32_t>& owner)
{
    const uint64_t n = length[0] * length[1] * length[2];
    DX_CHECK(n > 0 && n < (1ull << 32), DCCRGX_EINVAL, "SFC placement of %llu level-0 cells",
             (unsigned long long)n);
    DX_CHECK(comm_size > 0, DCCRGX_EINVAL, "comm size %d", comm_size);
    const uint64_t side = std::max(length[0], std::max(length[1], length[2]));
    int b = 1;
    while ((1ull << b) < side) b++;
    DX_CHECK(b <= 21, DCCRGX_EINVAL, "grid side %llu too long for 64-bit Hilbert keys", (unsigned long long)side);
    Bufs B;
    uint64_t *keys = nullptr, *keys2 = nullptr;
    uint32_t *cells = nullptr, *cells2 = nullptr;
    int32_t* d_owner = nullptr;
    DX_TRY(B.get(&keys, n * 8));
    DX_TRY(B.get(&keys2, n * 8));
    DX_TRY(B.get(&cells, n * 4));
    DX_TRY(B.get(&cells2, n * 4));
    DX_TRY(B.get(&d_owner, n * 4));
    hipLaunchKernelGGL(k_hilbert_keys, dim3(blocks(n)), dim3(256), 0, st, length[0], length[1], n, b, keys, cells);
    DX_HIP(hipGetLastError());
    size_t tmp_bytes = 0;
    DX_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys, keys2, cells, cells2, (int)n, 0, 3 * b, st));
    void* tmp = nullptr;
    DX_TRY(B.get(&tmp, tmp_bytes));
    DX_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, keys2, cells, cells2, (int)n, 0, 3 * b, st));
    hipLaunchKernelGGL(k_assign, dim3(blocks(n)), dim3(256), 0, st, (const uint32_t*)cells2, n,
                       make_partition(n, comm_size), d_owner);
    DX_HIP(hipGetLastError());
    owner.resize(n);
    DX_HIP(hipMemcpyAsync(owner.data(), d_owner, n * 4, hipMemcpyDeviceToHost, st));
    DX_HIP(hipStreamSynchronize(st));
    return DCCRGX_OK;
}

}  // namespace dccrgx

using namespace dccrgx;

extern "C" {

int dccrgx_hilbert_keys_host(const uint64_t length[3], uint64_t* keys_out)
{
    DX_CHECK(length && keys_out, DCCRGX_EINVAL, "null argument");
    const uint64_t n = length[0] * length[1] * length[2];
    const uint64_t side = std::max(length[0], std::max(length[1], length[2]));
    int b = 1;
    while ((1ull << b) < side) b++;
    DX_CHECK(b <= 21, DCCRGX_EINVAL, "grid side too long");
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t x = i % length[0], y = (i / length[0]) % length[1], z = i / (length[0] * length[1]);
        keys_out[i] = hilbert3((uint32_t)x, (uint32_t)y, (uint32_t)z, b);
    }
    return DCCRGX_OK;
}

int dccrgx_sfc_owners(dccrgx_ctx* ctx, const uint64_t length[3], int32_t comm_size, int32_t* owner_host)
{
    DX_CHECK(ctx && length && owner_host, DCCRGX_EINVAL, "null argument");
    DX_HIP(hipSetDevice(ctx->device));
    std::vector<int32_t> o;
    DX_TRY(sfc_owners(length, comm_size, ctx->compute, o));
    std::copy(o.begin(), o.end(), owner_host);
    return DCCRGX_OK;
}

}  // extern "C"
