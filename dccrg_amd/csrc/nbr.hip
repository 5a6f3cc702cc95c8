// nbr.hip -- neighbor lists of arbitrary cells as device CSR (uniform grids).
//
// get_neighbors_of (dccrg.hpp:836-883, built by find_neighbors_of :4375-4716):
// for a single-level grid the face-graph walk of the reference always ends on
// the cell at the item's window, so the list is closed form: one entry per
// item in neighborhood order, dropped outside non-periodic boundaries,
// offset = item * 2^max_ref_lvl (geometric, not wrapped: dccrg.hpp:7408-7430).
// get_neighbors_to (find_neighbors_to :4744-4897): unique cells found with
// hood_to = -hood_of, ascending here (the reference: unordered_map order).
#include <algorithm>
#include <cstring>

#include "face.hpp"
#include "grid.hpp"

namespace dccrgx {

int explicit_face_neighbors(const dccrgx_grid* grid, const uint64_t* cells, size_t n, uint64_t* row,
                            uint64_t* ids, int32_t* dirs, size_t cap, hipStream_t st);

namespace {
// a single-level grid: exactly the level-0 ids exist
struct UniformExists {
    MapParams mp;
    __host__ __device__ bool operator()(uint64_t c) const { return map_level(mp, c) == 0; }
};
}  // namespace

static unsigned grid_for(uint64_t n)
{
    uint64_t g = (n + 255) / 256;
    if (g > 256 * 16) g = 256 * 16;
    if (g == 0) g = 1;
    return (unsigned)g;
}

// pass 1 (ids == nullptr): per-cell counts into row[i + 1]; pass 2: fill
__global__ void __launch_bounds__(256) k_uniform_nbrs(UGeom g, const int32_t* __restrict__ items, int K,
                                                      const uint64_t* __restrict__ cells, size_t n,
                                                      uint64_t* __restrict__ row, uint64_t* __restrict__ ids,
                                                      int32_t* __restrict__ off3, int32_t* __restrict__ err,
                                                      int32_t sx, int32_t sy, int32_t sz)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t id = cells[i];
        if (id < 1 || id > g.N) {
            atomicOr(err, 1);
            if (!ids) row[i + 1] = 0;
            continue;
        }
        int64_t a, b, c;
        ug_decompose(g, id - 1, a, b, c);
        uint64_t w = ids ? row[i] : 0;
        for (int k = 0; k < K; k++) {
            uint64_t nlin;
            int64_t cu;
            if (!ug_neighbor(g, a, b, c, items + 3 * k, nlin, cu)) continue;
            if (ids) {
                ids[w] = nlin + 1;
                if (off3) {
                    // canonical item back to x, y, z (perm maps canonical -> original)
                    int32_t o[3];
                    for (int d = 0; d < 3; d++) o[g.perm[d]] = items[3 * k + d];
                    off3[3 * w + 0] = o[0] * sx;
                    off3[3 * w + 1] = o[1] * sy;
                    off3[3 * w + 2] = o[2] * sz;
                }
            }
            w++;
        }
        if (!ids) row[i + 1] = w;
    }
}

// ---------------------------------------------------------------------------
// Row pointers of a batch of query cells without a count array: each cell's count in
// closed form where the neighborhood allows (the full cube of length L: the
// product over axes of the in-grid offsets in [-L, L], minus the cell itself;
// the six face items: the in-grid ones), else by testing every item; then
// reduce-then-scan over tiles of 1024 cells (tile totals, their scan, and the
// rows written with the counts recomputed -- no count array in memory).
// ---------------------------------------------------------------------------
constexpr int RT = 256, RE = 4, RTILE = RT * RE;  // threads, cells per thread, cells per tile

__device__ __forceinline__ uint32_t uniform_count(const UGeom& g, const int32_t* items, int K, int cube, bool faces,
                                                  int64_t a, int64_t b, int64_t c)
{
    const int64_t pos[3] = {a, b, c};
    const uint64_t len[3] = {g.LA, g.LB, g.LC};
    const int32_t per[3] = {g.perA, g.perB, g.perC};
    if (cube >= 0) {
        uint32_t prod = 1;
        for (int d = 0; d < 3; d++) {
            const int64_t L = cube;
            const int64_t lo = per[d] ? L : (pos[d] < L ? pos[d] : L);
            const int64_t hi = per[d] ? L : ((int64_t)len[d] - 1 - pos[d] < L ? (int64_t)len[d] - 1 - pos[d] : L);
            prod *= (uint32_t)(lo + hi + 1);
        }
        return prod - 1;
    }
    if (faces) {
        uint32_t n = 0;
        for (int d = 0; d < 3; d++)
            n += per[d] ? 2u : (uint32_t)(pos[d] > 0) + (uint32_t)(pos[d] + 1 < (int64_t)len[d]);
        return n;
    }
    uint32_t n = 0;
    for (int k = 0; k < K; k++) {
        uint64_t nlin;
        int64_t cu;
        n += ug_neighbor(g, a, b, c, items + 3 * k, nlin, cu) ? 1u : 0u;
    }
    return n;
}

// pass 1 (tile_sum != null): the total of each tile; pass 2: row[i + 1] =
// (the inclusive scan of the tile totals before this tile) + the prefix
// inside the tile.  The counts are recomputed in pass 2 (a few ALU ops).
__global__ void __launch_bounds__(RT) k_uniform_rows(UGeom g, const int32_t* __restrict__ items, int K, int cube,
                                                     int faces, const uint64_t* __restrict__ cells, size_t n,
                                                     int check_local, uint64_t* __restrict__ tile_sum,
                                                     const uint64_t* __restrict__ tile_incl, uint64_t* __restrict__ row,
                                                     int32_t* __restrict__ err)
{
    __shared__ uint64_t s_wave[RT / 64];
    const uint64_t tile = blockIdx.x;
    const uint64_t i0 = tile * RTILE + (uint64_t)threadIdx.x * RE;
    uint64_t inc[RE];
    uint64_t t = 0;
    bool bad = false;
#pragma unroll
    for (int k = 0; k < RE; k++) {
        const uint64_t i = i0 + k;
        uint32_t cnt = 0;
        if (i < n) {
            const uint64_t id = cells[i];
            if (id < 1 || id > g.N || (check_local && (id - 1 < g.lo || id - 1 >= g.hi))) {
                bad = true;
            } else {
                int64_t a, b, c;
                ug_decompose(g, id - 1, a, b, c);
                cnt = uniform_count(g, items, K, cube, faces != 0, a, b, c);
            }
        }
        t += cnt;
        inc[k] = t;
    }
    if (bad && tile_sum) atomicOr(err, 1);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t v = t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t u = __shfl_up(v, d, 64);
        if (lane >= d) v += u;
    }
    if (lane == 63) s_wave[w] = v;
    __syncthreads();
    uint64_t before = 0, total = 0;
#pragma unroll
    for (int k = 0; k < RT / 64; k++) {
        before += k < w ? s_wave[k] : 0;
        total += s_wave[k];
    }
    if (tile_sum) {
        if (threadIdx.x == 0) tile_sum[tile] = total;
        return;
    }
    const uint64_t base = (tile ? tile_incl[tile - 1] : 0) + before + v - t;
    if (tile == 0 && threadIdx.x == 0) row[0] = 0;
#pragma unroll
    for (int k = 0; k < RE; k++)
        if (i0 + k < n) row[i0 + k + 1] = base + inc[k];
}

// row pointers of `cells` into row[0..n] (device); *total on the host.
// check_local: every query cell must be local to this rank
static int uniform_rows(const dccrgx_grid* grid, const Hood& h, const int32_t* d_items, const uint64_t* cells,
                        size_t n, int check_local, uint64_t* row, uint64_t* total, hipStream_t st)
{
    const UGeom& g = grid->g;
    const uint64_t tiles = std::max<uint64_t>((n + RTILE - 1) / RTILE, 1);
    DX_CHECK(tiles < (1ull << 31), DCCRGX_EINVAL, "%zu query cells", n);
    // one scratch block: the tile sums (scanned in place), the error word, the total
    uint64_t* scratch = nullptr;
    const size_t words = tiles + 2;
    DX_HIP(ds_malloc(&scratch, words * 8, st));
    auto done = [&](int code) {
        (void)ds_free(scratch, st);
        return code;
    };
    if (hipMemsetAsync(scratch, 0, words * 8, st) != hipSuccess) return done(set_error(DCCRGX_EHIP, "memset"));
    int32_t* err = reinterpret_cast<int32_t*>(scratch + tiles);
    hipLaunchKernelGGL(k_uniform_rows, dim3((unsigned)tiles), dim3(RT), 0, st, g, d_items, h.K, (int)h.count_cube,
                       h.count_faces ? 1 : 0, cells, n, check_local, scratch, (const uint64_t*)nullptr, row, err);
    int s = device_inclusive_scan(scratch, tiles, st);
    if (s != DCCRGX_OK) return done(s);
    hipLaunchKernelGGL(k_uniform_rows, dim3((unsigned)tiles), dim3(RT), 0, st, g, d_items, h.K, (int)h.count_cube,
                       h.count_faces ? 1 : 0, cells, n, check_local, (uint64_t*)nullptr, (const uint64_t*)scratch, row,
                       err);
    if (hipGetLastError() != hipSuccess) return done(set_error(DCCRGX_EHIP, "row kernel launch failed"));
    // the error word and the total in one copy
    if (hipMemcpyAsync(scratch + tiles + 1, scratch + tiles - 1, 8, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return done(set_error(DCCRGX_EHIP, "copy"));
    uint64_t tail[2] = {0, 0};
    if ((s = dx_d2h(grid->ctx, tail, scratch + tiles, 16, st)) != DCCRGX_OK) return done(s);
    *total = tail[1];
    if (tail[0])
        return done(set_error(DCCRGX_ENOTFOUND, check_local ? "a query cell is not a local cell of this rank"
                                                            : "cell outside the grid"));
    return done(DCCRGX_OK);
}

// fill pass with coalesced stores: one wave per 64 query cells.  Each lane
// lists its cell's valid neighbors (id and item) in LDS at the cell's
// position in the wave's output run (row[] is already scanned), then the wave
// writes the run entry by entry, consecutive lanes on consecutive entries;
// the offsets of an item come from a per-item table in LDS.  LDS: 10 B per
// (cell, item) record + 12 B per item.
__global__ void __launch_bounds__(64) k_uniform_fill(UGeom g, const int32_t* __restrict__ items, int K,
                                                     const uint64_t* __restrict__ cells, size_t n,
                                                     const uint64_t* __restrict__ row, uint64_t* __restrict__ ids,
                                                     int32_t* __restrict__ off3, int32_t sx, int32_t sy, int32_t sz)
{
    extern __shared__ uint64_t nid[];                       // 64 * K neighbor ids
    uint16_t* kit = reinterpret_cast<uint16_t*>(nid + 64 * K);  // 64 * K item numbers
    int32_t* otab = reinterpret_cast<int32_t*>(kit + 64 * K);   // K * 3 offsets (original axes, scaled)
    const int lane = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * 64;
    const uint64_t i = t0 + lane;
    const uint64_t base = row[t0];
    const uint64_t end = row[t0 + 64 < n ? t0 + 64 : n];
    if (off3)
        for (int k = lane; k < K; k += 64) {
            int32_t o[3];
            for (int d = 0; d < 3; d++) o[g.perm[d]] = items[3 * k + d];
            otab[3 * k + 0] = o[0] * sx;
            otab[3 * k + 1] = o[1] * sy;
            otab[3 * k + 2] = o[2] * sz;
        }
    if (i < n) {
        const uint64_t id = cells[i];
        if (id >= 1 && id <= g.N) {
            int64_t a, b, c;
            ug_decompose(g, id - 1, a, b, c);
            uint32_t w = (uint32_t)(row[i] - base);
            for (int k = 0; k < K; k++) {
                uint64_t nlin;
                int64_t cu;
                if (ug_neighbor(g, a, b, c, items + 3 * k, nlin, cu)) {
                    nid[w] = nlin + 1;
                    kit[w] = (uint16_t)k;
                    w++;
                }
            }
        }
    }
    __syncthreads();
    const uint64_t tot = end - base;
    for (uint64_t e = lane; e < tot; e += 64) {
        ids[base + e] = nid[e];
        if (off3) {
            const int k = kit[e];
            off3[3 * (base + e) + 0] = otab[3 * k + 0];
            off3[3 * (base + e) + 1] = otab[3 * k + 1];
            off3[3 * (base + e) + 2] = otab[3 * k + 2];
        }
    }
}

// the same for large neighborhoods (4-B records, ids recomputed at the store)
__global__ void __launch_bounds__(64) k_uniform_fill_rec(UGeom g, const int32_t* __restrict__ items, int K,
                                                     const uint64_t* __restrict__ cells, size_t n,
                                                     const uint64_t* __restrict__ row, uint64_t* __restrict__ ids,
                                                     int32_t* __restrict__ off3, int32_t sx, int32_t sy, int32_t sz)
{
    extern __shared__ uint32_t rec[];  // 64 * K records (lane << 16 | item)
    __shared__ int64_t abc[3][64];
    const int lane = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * 64;
    const uint64_t i = t0 + lane;
    const uint64_t base = row[t0];
    const uint64_t end = row[t0 + 64 < n ? t0 + 64 : n];
    if (i < n) {
        const uint64_t id = cells[i];
        if (id >= 1 && id <= g.N) {
            int64_t a, b, c;
            ug_decompose(g, id - 1, a, b, c);
            abc[0][lane] = a;
            abc[1][lane] = b;
            abc[2][lane] = c;
            uint32_t w = (uint32_t)(row[i] - base);
            for (int k = 0; k < K; k++) {
                uint64_t nlin;
                int64_t cu;
                if (ug_neighbor(g, a, b, c, items + 3 * k, nlin, cu)) rec[w++] = ((uint32_t)lane << 16) | (uint32_t)k;
            }
        }
    }
    __syncthreads();
    const uint64_t tot = end - base;
    for (uint64_t e = lane; e < tot; e += 64) {
        const uint32_t r = rec[e];
        const int l = (int)(r >> 16), k = (int)(r & 0xffffu);
        uint64_t nlin;
        int64_t cu;
        ug_neighbor(g, abc[0][l], abc[1][l], abc[2][l], items + 3 * k, nlin, cu);
        ids[base + e] = nlin + 1;
        if (off3) {
            int32_t o[3];
            for (int d = 0; d < 3; d++) o[g.perm[d]] = items[3 * k + d];
            off3[3 * (base + e) + 0] = o[0] * sx;
            off3[3 * (base + e) + 1] = o[1] * sy;
            off3[3 * (base + e) + 2] = o[2] * sz;
        }
    }
}

// neighbor gather on uniform grids: the field element of every neighbors_of
// entry of the query cells, laid out like dccrgx_neighbors_of's ids (one wave
// per 64 cells, LDS records, consecutive lanes on consecutive entries).
__global__ void __launch_bounds__(64) k_uniform_gather(UGeom g, const int32_t* __restrict__ items, int K,
                                                       const uint64_t* __restrict__ cells, size_t n,
                                                       const uint64_t* __restrict__ row,
                                                       const uint8_t* __restrict__ field, uint32_t elem,
                                                       uint8_t* __restrict__ out)
{
    extern __shared__ uint32_t rec[];
    __shared__ int64_t abc[3][64];
    const int lane = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * 64;
    const uint64_t i = t0 + lane;
    const uint64_t base = row[t0];
    const uint64_t end = row[t0 + 64 < n ? t0 + 64 : n];
    if (i < n) {
        const uint64_t id = cells[i];
        if (id >= 1 && id <= g.N) {
            int64_t a, b, c;
            ug_decompose(g, id - 1, a, b, c);
            abc[0][lane] = a;
            abc[1][lane] = b;
            abc[2][lane] = c;
            uint32_t w = (uint32_t)(row[i] - base);
            for (int k = 0; k < K; k++) {
                uint64_t nlin;
                int64_t cu;
                if (ug_neighbor(g, a, b, c, items + 3 * k, nlin, cu)) rec[w++] = ((uint32_t)lane << 16) | (uint32_t)k;
            }
        }
    }
    __syncthreads();
    const uint64_t tot = end - base;
    for (uint64_t e = lane; e < tot; e += 64) {
        const uint32_t r = rec[e];
        const int l = (int)(r >> 16), k = (int)(r & 0xffffu);
        uint64_t nlin;
        int64_t cu;
        ug_neighbor(g, abc[0][l], abc[1][l], abc[2][l], items + 3 * k, nlin, cu);
        // a local neighbor (also one reached through a periodic wrap) is read
        // from its own slot, as the reference reads the cell itself; a remote
        // one from its ghost slot (unwrapped c)
        const int64_t cw = ug_wrap(cu, (int64_t)g.LC);
        const int64_t cs = ug_local(g, nlin) ? cw : cu;
        const uint64_t slot = nlin - (uint64_t)cw * g.S + (uint64_t)(cs - g.cbase) * g.S;
        const uint8_t* src = field + slot * elem;
        uint8_t* dst = out + (base + e) * elem;
        if (elem == 4) {
            *reinterpret_cast<uint32_t*>(dst) = *reinterpret_cast<const uint32_t*>(src);
        } else if (elem == 8) {
            *reinterpret_cast<uint64_t*>(dst) = *reinterpret_cast<const uint64_t*>(src);
        } else if (elem % 4 == 0) {
            for (uint32_t q = 0; q < elem; q += 4)
                *reinterpret_cast<uint32_t*>(dst + q) = *reinterpret_cast<const uint32_t*>(src + q);
        } else {
            for (uint32_t q = 0; q < elem; q++) dst[q] = src[q];
        }
    }
}

// the same for neighborhoods too large for the LDS records (> 192 items):
// one thread per query cell writes its own run
__global__ void __launch_bounds__(256) k_uniform_gather_direct(UGeom g, const int32_t* __restrict__ items, int K,
                                                               const uint64_t* __restrict__ cells, size_t n,
                                                               const uint64_t* __restrict__ row,
                                                               const uint8_t* __restrict__ field, uint32_t elem,
                                                               uint8_t* __restrict__ out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t id = cells[i];
        if (id < 1 || id > g.N) continue;
        int64_t a, b, c;
        ug_decompose(g, id - 1, a, b, c);
        uint64_t w = row[i];
        for (int k = 0; k < K; k++) {
            uint64_t nlin;
            int64_t cu;
            if (!ug_neighbor(g, a, b, c, items + 3 * k, nlin, cu)) continue;
            const int64_t cw = ug_wrap(cu, (int64_t)g.LC);
            const int64_t cs = ug_local(g, nlin) ? cw : cu;
            const uint64_t slot = nlin - (uint64_t)cw * g.S + (uint64_t)(cs - g.cbase) * g.S;
            const uint8_t* src = field + slot * elem;
            uint8_t* dst = out + (w++) * elem;
            for (uint32_t q = 0; q < elem; q++) dst[q] = src[q];
        }
    }
}

int explicit_gather_neighbors(const dccrgx_grid* grid, const Hood& h, const Field& F, const uint64_t* cells, size_t n,
                              uint64_t* row, void* out, size_t cap_bytes, hipStream_t st);

// query cells must be local (lin in [lo, hi))
__global__ void __launch_bounds__(256) k_check_local(UGeom g, const uint64_t* __restrict__ cells, size_t n,
                                                     int32_t* __restrict__ err)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t id = cells[i];
        if (id < 1 || id - 1 < g.lo || id - 1 >= g.hi) atomicOr(err, 1);
    }
}

int explicit_neighbors_of(const dccrgx_grid* grid, const Hood& h, const uint64_t* cells, size_t n,
                          uint64_t* row, uint64_t* ids, int32_t* off3, size_t cap, hipStream_t st);
int explicit_neighbors_to(const dccrgx_grid* grid, const Hood& h, const uint64_t* cells, size_t n,
                          uint64_t* row, uint64_t* ids, size_t cap, hipStream_t st);

// row[1..n] counts -> row pointers, on the device (scan.hip)
static int scan_rows(uint64_t* row, size_t n, hipStream_t st, uint64_t* total)
{
    return device_scan_rows(row, n, st, total);
}

}  // namespace dccrgx

using namespace dccrgx;

extern "C" {

int dccrgx_neighbors_of(const dccrgx_grid* grid, int32_t hood_id, const uint64_t* cells, size_t n,
                        uint64_t* row, uint64_t* ids, int32_t* off3, size_t cap, void* stream)
{
    DX_CHECK(grid && row && (cells || n == 0), DCCRGX_EINVAL, "null argument");
    const Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    hipStream_t st = stream ? (hipStream_t)stream : grid->ctx->compute;
    const CallerStream fence(grid->ctx, st);
    if (grid->hy) return hybrid_neighbors(grid, hood_id, false, cells, n, row, ids, off3, cap, st);
    if (!grid->uniform) return explicit_neighbors_of(grid, *h, cells, n, row, ids, off3, cap, st);
    const UGeom& g = grid->g;
    const int32_t sc = 1 << grid->map.max_lvl;  // offsets in indices of the finest level
    uint64_t total = 0;
    DX_TRY(uniform_rows(grid, *h, h->d_of_c, cells, n, 0, row, &total, st));
    if (!ids) return DCCRGX_OK;
    DX_CHECK(cap >= total, DCCRGX_ERANGE, "capacity %zu < %llu", cap, (unsigned long long)total);
    if (n && h->K <= 76) {  // LDS records: 652 B per item (48 KiB at 76)
        hipLaunchKernelGGL(k_uniform_fill, dim3((unsigned)((n + 63) / 64)), dim3(64), 64 * 10 * h->K + 12 * h->K, st,
                           g, h->d_of_c, h->K, cells, n, row, ids, off3, sc, sc, sc);
    } else if (n && h->K <= 192) {  // 256 B per item (48 KiB at 192)
        hipLaunchKernelGGL(k_uniform_fill_rec, dim3((unsigned)((n + 63) / 64)), dim3(64), 64 * 4 * h->K, st, g,
                           h->d_of_c, h->K, cells, n, row, ids, off3, sc, sc, sc);
    } else if (n) {  // per-thread rows (the cells were checked by uniform_rows)
        int32_t* d_err = nullptr;
        DX_HIP(ds_malloc(&d_err, 4, st));
        hipLaunchKernelGGL(k_uniform_nbrs, dim3(grid_for(n)), dim3(256), 0, st, g, h->d_of_c, h->K, cells,
                           n, row, ids, off3, d_err, sc, sc, sc);
        DX_HIP(ds_free(d_err, st));
    }
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

int dccrgx_gather_neighbors(const dccrgx_grid* grid, int32_t hood_id, int32_t field_id, const uint64_t* cells,
                            size_t n, uint64_t* row, void* out, size_t cap_bytes, void* stream)
{
    DX_CHECK(grid && row && (cells || n == 0), DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    const Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    DX_CHECK(field_id >= 0 && (size_t)field_id < grid->fields.size(), DCCRGX_EINVAL, "bad field %d", field_id);
    const Field& F = grid->fields[field_id];
    DX_CHECK(!F.variable, DCCRGX_EINVAL, "variable-size field: use dccrgx_field_read_cells");
    hipStream_t st = stream ? (hipStream_t)stream : grid->ctx->compute;
    const CallerStream fence(grid->ctx, st);
    if (!grid->uniform) return explicit_gather_neighbors(grid, *h, F, cells, n, row, out, cap_bytes, st);
    const UGeom& g = grid->g;
    uint64_t total = 0;
    DX_TRY(uniform_rows(grid, *h, h->d_of_c, cells, n, 1, row, &total, st));
    if (!out) return DCCRGX_OK;
    DX_CHECK(cap_bytes >= total * F.elem, DCCRGX_ERANGE, "capacity %zu < %llu bytes", cap_bytes,
             (unsigned long long)(total * F.elem));
    if (n && h->K <= 192)  // LDS records: 256 B per item (48 KiB at 192)
        hipLaunchKernelGGL(k_uniform_gather, dim3((unsigned)((n + 63) / 64)), dim3(64), 64 * 4 * h->K, st, g,
                           h->d_of_c, h->K, cells, n, (const uint64_t*)row, (const uint8_t*)F.ptr, F.elem,
                           (uint8_t*)out);
    else if (n)
        hipLaunchKernelGGL(k_uniform_gather_direct, dim3(grid_for(n)), dim3(256), 0, st, g, h->d_of_c, h->K, cells, n,
                           (const uint64_t*)row, (const uint8_t*)F.ptr, F.elem, (uint8_t*)out);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

int dccrgx_face_neighbors_of(const dccrgx_grid* grid, const uint64_t* cells, size_t n, uint64_t* row,
                             uint64_t* ids, int32_t* dirs, size_t cap, void* stream)
{
    DX_CHECK(grid && row && (cells || n == 0), DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    hipStream_t st = stream ? (hipStream_t)stream : grid->ctx->compute;
    const CallerStream fence(grid->ctx, st);
    if (!grid->uniform) return explicit_face_neighbors(grid, cells, n, row, ids, dirs, cap, st);
    return face_neighbors_launch(grid->map, grid->params.periodic, UniformExists{grid->map}, cells, n, row, ids,
                                 dirs, cap, st);
}

int dccrgx_face_neighbors_of_host(const dccrgx_grid* grid, const uint64_t* cells, size_t n, uint64_t* row,
                                  uint64_t* ids, int32_t* dirs, size_t cap)
{
    DX_CHECK(grid && row && (cells || n == 0), DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    DX_TRY(explicit_host_leaves(grid));
    hipStream_t st = grid->ctx->compute;
    uint64_t *d_cells = nullptr, *d_row = nullptr, *d_ids = nullptr;
    int32_t* d_dirs = nullptr;
    DX_HIP(dx_malloc(&d_cells, std::max<size_t>(n, 1) * 8));
    DX_HIP(dx_malloc(&d_row, (n + 1) * 8));
    DX_HIP(dx_malloc(&d_ids, std::max<size_t>(cap, 1) * 8));
    DX_HIP(dx_malloc(&d_dirs, std::max<size_t>(cap, 1) * 4));
    if (n) DX_HIP(hipMemcpyAsync(d_cells, cells, n * 8, hipMemcpyHostToDevice, st));
    int s = dccrgx_face_neighbors_of(grid, d_cells, n, d_row, ids ? d_ids : nullptr, d_dirs, cap, st);
    if (s == DCCRGX_OK || s == DCCRGX_ERANGE) {
        DX_HIP(hipMemcpyAsync(row, d_row, (n + 1) * 8, hipMemcpyDeviceToHost, st));
        DX_HIP(hipStreamSynchronize(st));
        if (s == DCCRGX_OK && ids && row[n]) {
            DX_HIP(hipMemcpyAsync(ids, d_ids, row[n] * 8, hipMemcpyDeviceToHost, st));
            if (dirs) DX_HIP(hipMemcpyAsync(dirs, d_dirs, row[n] * 4, hipMemcpyDeviceToHost, st));
        }
    }
    DX_HIP(hipStreamSynchronize(st));
    dx_free(d_cells);
    dx_free(d_row);
    dx_free(d_ids);
    dx_free(d_dirs);
    return s;
}

int dccrgx_neighbors_to(const dccrgx_grid* grid, int32_t hood_id, const uint64_t* cells, size_t n,
                        uint64_t* row, uint64_t* ids, size_t cap, void* stream)
{
    DX_CHECK(grid && row && (cells || n == 0), DCCRGX_EINVAL, "null argument");
    const Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    hipStream_t st = stream ? (hipStream_t)stream : grid->ctx->compute;
    const CallerStream fence(grid->ctx, st);
    if (grid->hy) return hybrid_neighbors(grid, hood_id, true, cells, n, row, ids, nullptr, cap, st);
    if (!grid->uniform) return explicit_neighbors_to(grid, *h, cells, n, row, ids, cap, st);
    // candidates with hood_to on the device, unique + sort per cell on the host
    const UGeom& g = grid->g;
    int32_t* d_err = nullptr;
    uint64_t *d_row = nullptr, *d_ids = nullptr;
    DX_HIP(dx_malloc(&d_err, 4));
    DX_HIP(hipMemsetAsync(d_err, 0, 4, st));
    DX_HIP(dx_malloc(&d_row, (n + 1) * 8));
    DX_HIP(hipMemsetAsync(d_row, 0, 8, st));
    if (n)
        hipLaunchKernelGGL(k_uniform_nbrs, dim3(grid_for(n)), dim3(256), 0, st, g, h->d_to_c, h->K, cells, n,
                           d_row, (uint64_t*)nullptr, (int32_t*)nullptr, d_err, 1, 1, 1);
    uint64_t total = 0;
    DX_TRY(scan_rows(d_row, n, st, &total));
    DX_HIP(dx_malloc(&d_ids, std::max<uint64_t>(total, 1) * 8));
    if (n)
        hipLaunchKernelGGL(k_uniform_nbrs, dim3(grid_for(n)), dim3(256), 0, st, g, h->d_to_c, h->K, cells, n,
                           d_row, d_ids, (int32_t*)nullptr, d_err, 1, 1, 1);
    DX_HIP(hipGetLastError());
    std::vector<uint64_t> hr(n + 1), hi(total);
    int32_t err = 0;
    DX_HIP(hipMemcpyAsync(hr.data(), d_row, (n + 1) * 8, hipMemcpyDeviceToHost, st));
    if (total) DX_HIP(hipMemcpyAsync(hi.data(), d_ids, total * 8, hipMemcpyDeviceToHost, st));
    DX_HIP(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, st));
    DX_HIP(hipStreamSynchronize(st));
    dx_free(d_err);
    dx_free(d_row);
    dx_free(d_ids);
    DX_CHECK(!err, DCCRGX_ENOTFOUND, "cell outside the grid");
    std::vector<uint64_t> orow(n + 1, 0), oids;
    oids.reserve(total);
    for (size_t i = 0; i < n; i++) {
        std::vector<uint64_t> v(hi.begin() + hr[i], hi.begin() + hr[i + 1]);
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        oids.insert(oids.end(), v.begin(), v.end());
        orow[i + 1] = oids.size();
    }
    DX_HIP(hipMemcpyAsync(row, orow.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
    if (ids) {
        DX_CHECK(cap >= oids.size(), DCCRGX_ERANGE, "capacity %zu < %zu", cap, oids.size());
        if (!oids.empty())
            DX_HIP(hipMemcpyAsync(ids, oids.data(), oids.size() * 8, hipMemcpyHostToDevice, st));
    }
    DX_HIP(hipStreamSynchronize(st));
    return DCCRGX_OK;
}

int dccrgx_neighbors_of_host(const dccrgx_grid* grid, int32_t hood_id, const uint64_t* cells, size_t n,
                             uint64_t* row, uint64_t* ids, int32_t* off3, size_t cap)
{
    DX_CHECK(grid && row && (cells || n == 0), DCCRGX_EINVAL, "null argument");
    DX_TRY(explicit_host_leaves(grid));
    hipStream_t st = grid->ctx->compute;
    uint64_t *d_cells = nullptr, *d_row = nullptr, *d_ids = nullptr;
    int32_t* d_off = nullptr;
    DX_HIP(dx_malloc(&d_cells, std::max<size_t>(n, 1) * 8));
    DX_HIP(dx_malloc(&d_row, (n + 1) * 8));
    if (n) DX_HIP(hipMemcpyAsync(d_cells, cells, n * 8, hipMemcpyHostToDevice, st));
    int s = dccrgx_neighbors_of(grid, hood_id, d_cells, n, d_row, nullptr, nullptr, 0, st);
    if (s == DCCRGX_OK) {
        DX_HIP(hipMemcpyAsync(row, d_row, (n + 1) * 8, hipMemcpyDeviceToHost, st));
        DX_HIP(hipStreamSynchronize(st));
        const uint64_t total = row[n];
        if (ids) {
            if (cap < total) {
                s = set_error(DCCRGX_ERANGE, "capacity %zu < %llu", cap, (unsigned long long)total);
            } else {
                DX_HIP(dx_malloc(&d_ids, std::max<uint64_t>(total, 1) * 8));
                DX_HIP(dx_malloc(&d_off, std::max<uint64_t>(total, 1) * 12));
                s = dccrgx_neighbors_of(grid, hood_id, d_cells, n, d_row, d_ids, d_off, total, st);
                if (s == DCCRGX_OK && total) {
                    DX_HIP(hipMemcpyAsync(ids, d_ids, total * 8, hipMemcpyDeviceToHost, st));
                    if (off3) DX_HIP(hipMemcpyAsync(off3, d_off, total * 12, hipMemcpyDeviceToHost, st));
                }
            }
        }
    }
    DX_HIP(hipStreamSynchronize(st));
    dx_free(d_cells);
    dx_free(d_row);
    dx_free(d_ids);
    dx_free(d_off);
    return s;
}

int dccrgx_neighbors_to_host(const dccrgx_grid* grid, int32_t hood_id, const uint64_t* cells, size_t n,
                             uint64_t* row, uint64_t* ids, size_t cap)
{
    DX_CHECK(grid && row && (cells || n == 0), DCCRGX_EINVAL, "null argument");
    DX_TRY(explicit_host_leaves(grid));
    hipStream_t st = grid->ctx->compute;
    uint64_t *d_cells = nullptr, *d_row = nullptr, *d_ids = nullptr;
    DX_HIP(dx_malloc(&d_cells, std::max<size_t>(n, 1) * 8));
    DX_HIP(dx_malloc(&d_row, (n + 1) * 8));
    if (n) DX_HIP(hipMemcpyAsync(d_cells, cells, n * 8, hipMemcpyHostToDevice, st));
    int s = dccrgx_neighbors_to(grid, hood_id, d_cells, n, d_row, nullptr, 0, st);
    if (s == DCCRGX_OK) {
        DX_HIP(hipMemcpyAsync(row, d_row, (n + 1) * 8, hipMemcpyDeviceToHost, st));
        DX_HIP(hipStreamSynchronize(st));
        const uint64_t total = row[n];
        if (ids) {
            if (cap < total) {
                s = set_error(DCCRGX_ERANGE, "capacity %zu < %llu", cap, (unsigned long long)total);
            } else {
                DX_HIP(dx_malloc(&d_ids, std::max<uint64_t>(total, 1) * 8));
                s = dccrgx_neighbors_to(grid, hood_id, d_cells, n, d_row, d_ids, total, st);
                if (s == DCCRGX_OK && total) DX_HIP(hipMemcpyAsync(ids, d_ids, total * 8, hipMemcpyDeviceToHost, st));
            }
        }
    }
    DX_HIP(hipStreamSynchronize(st));
    dx_free(d_cells);
    dx_free(d_row);
    dx_free(d_ids);
    return s;
}

}  // extern "C"
