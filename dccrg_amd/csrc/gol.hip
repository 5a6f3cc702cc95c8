// gol.hip -- game-of-life stencil over a rank's slab (the user hot loop of
// examples/game_of_life.cpp:54-79 and tests/game_of_life/scalability3d.cpp:
// 136-165, executed on the device with the neighbor gather staged in LDS).
//
// Fast path (the default 26-item cube, i.e. neighborhood length 1): each
// workgroup owns a TA x TB tile of the (A, B) plane and marches along the
// slab axis C.  Every plane is read from HBM once into a double-buffered LDS
// tile (+1 apron in A and B, periodic wrap in index space), the 3x3 box sum
// of the plane is formed from LDS row sums and kept in registers, and the
// 27-point sum of plane c is S(c-1) + S(c) + S(c+1) - centre.  HBM traffic per
// cell: 4 B read (is_alive) + 4 B write (next is_alive) + 4 B write
// (live_neighbor_count) = 12 B -- the algorithmic minimum.
//
// Any other neighborhood (face neighbors, length >= 2, user neighborhoods)
// uses the generic item loop (one lane per cell, neighbor slots computed in
// closed form) -- same results, not bandwidth-optimised.
#include <algorithm>
#include <cstdlib>

#include "gol_kernels.hpp"

namespace dccrgx {

// generic neighborhood: one lane per local cell, closed-form neighbor slots
__global__ void __launch_bounds__(256) k_gol_items(UGeom g, const uint32_t* __restrict__ in,
                                                   uint32_t* __restrict__ out, uint32_t* __restrict__ cnt,
                                                   const int32_t* __restrict__ items, int K,
                                                   uint64_t lin0, uint64_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const uint64_t soff = (uint64_t)(-g.cbase * (int64_t)g.S);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t lin = lin0 + i;
        int64_t a, b, c;
        ug_decompose(g, lin, a, b, c);
        uint32_t count = 0;
        for (int k = 0; k < K; k++) {
            const int32_t* d = items + 3 * k;
            int64_t a2 = a + d[0], b2 = b + d[1], c2 = c + d[2];
            if (a2 < 0 || a2 >= (int64_t)g.LA) {
                if (!g.perA) continue;
                a2 = ug_wrap(a2, (int64_t)g.LA);
            }
            if (b2 < 0 || b2 >= (int64_t)g.LB) {
                if (!g.perB) continue;
                b2 = ug_wrap(b2, (int64_t)g.LB);
            }
            if ((c2 < 0 || c2 >= (int64_t)g.LC) && !g.perC) continue;
            count += alive_bit(in[ug_slot(g, a2, b2, c2)]);
        }
        const uint64_t s = lin + soff;
        cnt[s] = count;
        out[s] = gol_rule(count, in[s]);
    }
}

// deterministic synthetic initial state: alive = splitmix64(id) % 1000 < permille
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) k_init_hash(uint32_t* __restrict__ f, uint64_t lin0, uint64_t n,
                                                   uint64_t soff, uint32_t permille)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t id = lin0 + i + 1;
        f[lin0 + i + soff] = (splitmix64(id) % 1000u) < permille ? 1u : 0u;
    }
}

static unsigned grid_for(uint64_t n)
{
    uint64_t g = (n + 255) / 256;
    if (g > 256 * 16) g = 256 * 16;
    if (g == 0) g = 1;
    return (unsigned)g;
}

// checksum of a 4-byte field over the local cells: (sum v, sum v * splitmix64(id))
// mod 2^64.  Local position i holds cell ids[i] (explicit grids) or lin0 + i + 1
// (uniform grids, slot lin0 + i + soff).  Per-block partials, then one block
// sums them in a fixed order (no atomics, bit-reproducible).
__global__ void __launch_bounds__(256) k_checksum(const uint32_t* __restrict__ f, uint64_t n, uint64_t lin0,
                                                  uint64_t soff, const uint64_t* __restrict__ ids,
                                                  uint64_t* __restrict__ partial)
{
    uint64_t s0 = 0, s1 = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t v = ids ? f[i] : f[lin0 + i + soff];
        const uint64_t id = ids ? ids[i] : lin0 + i + 1;
        s0 += v;
        s1 += v * splitmix64(id);
    }
    for (int o = 32; o > 0; o >>= 1) {
        s0 += __shfl_down(s0, o, 64);
        s1 += __shfl_down(s1, o, 64);
    }
    __shared__ uint64_t w0[4], w1[4];
    if (threadIdx.x % 64 == 0) {
        w0[threadIdx.x / 64] = s0;
        w1[threadIdx.x / 64] = s1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[2 * blockIdx.x] = w0[0] + w0[1] + w0[2] + w0[3];
        partial[2 * blockIdx.x + 1] = w1[0] + w1[1] + w1[2] + w1[3];
    }
}

__global__ void __launch_bounds__(64) k_checksum_final(const uint64_t* __restrict__ partial, uint32_t nb,
                                                       uint64_t* __restrict__ out)
{
    uint64_t s0 = 0, s1 = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += 64) {
        s0 += partial[2 * b];
        s1 += partial[2 * b + 1];
    }
    for (int o = 32; o > 0; o >>= 1) {
        s0 += __shfl_down(s0, o, 64);
        s1 += __shfl_down(s1, o, 64);
    }
    if (threadIdx.x == 0) {
        out[0] = s0;
        out[1] = s1;
    }
}

// the local cells' ids in slot order, explicit grids (explicit.hip)
int explicit_local_ids(const dccrgx_grid* grid, uint64_t* d_ids, hipStream_t st);

int gol_launch(dccrgx_grid* grid, const Hood& h, const Field& in, const Field& out, const Field& cnt,
               int64_t s0, int64_t s1, hipStream_t st)
{
    const UGeom& u = grid->g;
    if (s1 <= s0 || grid->n_local == 0) return DCCRGX_OK;
    if (!h.cube1) {
        // local lin range of the slices
        const int64_t S = (int64_t)u.S;
        const uint64_t l0 = std::max<int64_t>((s0 + u.cbase) * S, (int64_t)u.lo);
        const uint64_t l1 = std::min<int64_t>((s1 + u.cbase) * S, (int64_t)u.hi);
        if (l1 <= l0) return DCCRGX_OK;
        hipLaunchKernelGGL(k_gol_items, dim3(grid_for(l1 - l0)), dim3(256), 0, st, u,
                           (const uint32_t*)in.ptr, (uint32_t*)out.ptr, (uint32_t*)cnt.ptr, h.d_of_c, h.K,
                           l0, l1 - l0);
        DX_HIP(hipGetLastError());
        return DCCRGX_OK;
    }
    GolArgs a{};
    a.in = (const uint32_t*)in.ptr;
    a.out = (uint32_t*)out.ptr;
    a.cnt = (uint32_t*)cnt.ptr;
    a.LA = u.LA;
    a.LB = u.LB;
    a.S = u.S;
    a.lo = u.lo;
    a.hi = u.hi;
    a.cbase = u.cbase;
    a.s0 = s0;
    a.s1 = s1;
    a.perA = u.perA;
    a.perB = u.perB;
    const int64_t nsl = s1 - s0;
    // test options: slices per workgroup (chunk seams in small grids); the
    // LDS-tiled scalar kernels on grids the vector kernels take
    const int64_t chunk = test_opt(OPT_GOL_CHUNK, 0);
    const bool vec = u.LA % 4 == 0 && u.S < (1ull << 31) && !test_opt(OPT_GOL_SCALAR, 0);
    const uint32_t mult = u.perB ? 3u : 1u;
    if (u.LB == 1 && vec) {
        // 2-D / 1-D grids: k_gol26_rowv, 4 waves x 256 cells of a row per
        // workgroup, non-temporal stores (1-2 % faster than plain stores in
        // every A/B pairing, profiles/r7c_gol2d_nts_ab.log); 65536 workgroups
        // (4 rows each at 16384^2): 5.20 -> 5.46-5.56 TB/s against 8192, in
        // both of two A/B rounds on one box (2048 / 4096 / 16384 / 32768 /
        // 131072 in between or slower, profiles/s13_gol2d_want_ab.log)
        Gol4Args v = gol4_plan(a, 1024, 1, nsl, chunk, 65536);
        DX_CHECK(v.nwg, DCCRGX_EINVAL, "grid too large for one launch");
        hipLaunchKernelGGL((k_gol26_rowv<4, true>), dim3(v.nwg), dim3(256), 0, st, v, mult);
    } else if (u.LB == 1) {
        constexpr int TA = 1024, NA = 4;
        a.tiles_a = (uint32_t)((u.LA + TA - 1) / TA);
        a.tiles_b = 1;
        a.chunk = gol_chunk(nsl, a.tiles_a, 2048, chunk);
        const int64_t chunks = (nsl + a.chunk - 1) / a.chunk;
        hipLaunchKernelGGL((k_gol26_row<TA, NA>), dim3((unsigned)(a.tiles_a * chunks)), dim3(256), 0, st, a,
                           mult);
    } else if (vec) {
        // 3-D grids: k_gol26v, 8 waves x 4 rows (256 x 32 cells) per workgroup,
        // non-temporal stores -- the fastest tiling of the sweep
        // (tools/gol_sweep.hip; profiles/r1_summary.md)
        Gol4Args v = gol4_plan(a, 256, 32, nsl, chunk);
        DX_CHECK(v.nwg, DCCRGX_EINVAL, "grid too large for one launch");
        hipLaunchKernelGGL((k_gol26v<8, 4, true>), dim3(v.nwg), dim3(512), 0, st, v);
    } else {
        constexpr int TA = 64, TB = 16, NA = 1, NB = 4;
        a.tiles_a = (uint32_t)((u.LA + TA - 1) / TA);
        a.tiles_b = (uint32_t)((u.LB + TB - 1) / TB);
        const int64_t tiles = (int64_t)a.tiles_a * a.tiles_b;
        a.chunk = gol_chunk(nsl, tiles, 2048, chunk);
        const int64_t chunks = (nsl + a.chunk - 1) / a.chunk;
        DX_CHECK(tiles * chunks < (int64_t)UINT32_MAX, DCCRGX_EINVAL, "grid too large for one launch");
        hipLaunchKernelGGL((k_gol26<TA, TB, NA, NB>), dim3((unsigned)(tiles * chunks)), dim3(256), 0, st, a);
    }
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

// explicit grids: CSR gather (explicit.hip)
int explicit_gol(dccrgx_grid* grid, const Hood& h, const Field& in, const Field& out, const Field& cnt,
                 int32_t region, hipStream_t st);

struct TimerPool {
    std::vector<hipEvent_t> ev;
    size_t used = 0;
    bool on = false;
};
static std::map<const dccrgx_grid*, TimerPool> g_timers;

static int timed(dccrgx_grid* grid, bool begin, hipStream_t st)
{
    auto it = g_timers.find(grid);
    if (it == g_timers.end() || !it->second.on) return DCCRGX_OK;
    TimerPool& T = it->second;
    if (T.used == T.ev.size()) {
        hipEvent_t e;
        DX_HIP(hipEventCreate(&e));
        T.ev.push_back(e);
    }
    (void)begin;
    DX_HIP(hipEventRecord(T.ev[T.used++], st));
    return DCCRGX_OK;
}

void region_slices(const dccrgx_grid* grid, const Hood& h, int32_t region, int64_t r[2][2])
{
    const UGeom& u = grid->g;
    const int64_t all0 = u.pad, all1 = (int64_t)u.nslices - u.pad;
    r[0][0] = r[0][1] = r[1][0] = r[1][1] = 0;
    if (region == DCCRGX_REGION_ALL) {
        r[0][0] = all0;
        r[0][1] = all1;
    } else if (region == DCCRGX_REGION_INNER) {
        r[0][0] = h.inner_s0;
        r[0][1] = h.inner_s1;
    } else {
        r[0][0] = all0;
        r[0][1] = std::min(h.inner_s0, all1);
        r[1][0] = std::max(h.inner_s1, all0);
        r[1][1] = all1;
        if (h.inner_s1 <= h.inner_s0) {  // no inner slices: everything is outer
            r[0][1] = all1;
            r[1][0] = r[1][1] = 0;
        }
    }
}

static int compute_region(dccrgx_grid* grid, const Hood& h, const Field& in, const Field& out,
                          const Field& cnt, int32_t region, hipStream_t st)
{
    if (!grid->uniform) return explicit_gol(grid, h, in, out, cnt, region, st);
    int64_t r[2][2];
    region_slices(grid, h, region, r);
    for (auto& x : r) {
        if (x[1] <= x[0]) continue;
        DX_TRY(timed(grid, true, st));
        DX_TRY(gol_launch(grid, h, in, out, cnt, x[0], x[1], st));
        DX_TRY(timed(grid, false, st));
    }
    // refined cells inside the uniform grid: the overlay's cells again, from
    // their stored rows (every region call: the overlay is small, and the
    // rewrite is idempotent)
    if (grid->hy) DX_TRY(hybrid_gol(grid, in.ptr, out.ptr, cnt.ptr, st));
    return DCCRGX_OK;
}

}  // namespace dccrgx

using namespace dccrgx;

extern "C" {

static int gol_fields(dccrgx_grid* grid, int32_t a, int32_t b, int32_t c)
{
    const int32_t f[3] = {a, b, c};
    for (int i = 0; i < 3; i++) {
        DX_CHECK(f[i] >= 0 && (size_t)f[i] < grid->fields.size(), DCCRGX_EINVAL, "bad field %d", f[i]);
        DX_CHECK(grid->fields[f[i]].elem == 4 && !grid->fields[f[i]].variable, DCCRGX_EINVAL,
                 "game of life fields are 4-byte");
    }
    DX_CHECK(a != b && a != c && b != c, DCCRGX_EINVAL, "fields must be distinct (double buffered)");
    return DCCRGX_OK;
}

int dccrgx_gol_compute(dccrgx_grid* grid, int32_t hood_id, int32_t fin, int32_t fout, int32_t fcnt,
                       int32_t region)
{
    DX_NOT_PENDING(grid);
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    const Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    DX_TRY(gol_fields(grid, fin, fout, fcnt));
    DX_CHECK(region >= DCCRGX_REGION_ALL && region <= DCCRGX_REGION_OUTER, DCCRGX_EINVAL, "bad region");
    return compute_region(grid, *h, grid->fields[fin], grid->fields[fout], grid->fields[fcnt], region,
                          grid->ctx->compute);
}

int dccrgx_gol_step(dccrgx_grid* grid, int32_t hood_id, int32_t fin, int32_t fout, int32_t fcnt)
{
    DX_NOT_PENDING(grid);
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    const Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    DX_TRY(gol_fields(grid, fin, fout, fcnt));
    // scalability3d.cpp:122-166: start halo, inner cells, wait, outer cells
    DX_TRY(dccrgx_halo_start(grid, hood_id, &fin, 1));
    DX_TRY(dccrgx_gol_compute(grid, hood_id, fin, fout, fcnt, DCCRGX_REGION_INNER));
    DX_TRY(dccrgx_halo_wait(grid, hood_id, DCCRGX_WAIT_ALL));
    // test option corrupt_ghost: after every exchange, mark the ghost cell
    // just below the rank's first local cell alive, as a lost or misplaced
    // halo message would; bench.py's self-check must then fail
    if (test_opt(OPT_CORRUPT_GHOST, 0) && grid->uniform && grid->n_local) {
        const uint64_t slot0 = grid->g.lo + (uint64_t)(-grid->g.cbase * (int64_t)grid->g.S);
        if (slot0 > 0)
            DX_HIP(hipMemsetD32Async((hipDeviceptr_t)((uint32_t*)grid->fields[fin].ptr + slot0 - 1), 1, 1,
                                     grid->ctx->compute));
    }
    DX_TRY(dccrgx_gol_compute(grid, hood_id, fin, fout, fcnt, DCCRGX_REGION_OUTER));
    return DCCRGX_OK;
}

int dccrgx_field_init_hash(dccrgx_grid* grid, int32_t fid, uint32_t permille)
{
    DX_NOT_PENDING(grid);
    DX_CHECK(grid && fid >= 0 && (size_t)fid < grid->fields.size(), DCCRGX_EINVAL, "bad field");
    DX_CHECK(grid->fields[fid].elem == 4, DCCRGX_EINVAL, "4-byte field expected");
    DX_CHECK(grid->uniform, DCCRGX_EINVAL, "uniform grids only");
    DX_NO_HYBRID(grid);
    if (!grid->n_local) return DCCRGX_OK;
    const uint64_t soff = (uint64_t)(-grid->g.cbase * (int64_t)grid->g.S);
    hipLaunchKernelGGL(k_init_hash, dim3(grid_for(grid->n_local)), dim3(256), 0, grid->ctx->compute,
                       (uint32_t*)grid->fields[fid].ptr, grid->g.lo, grid->n_local, soff, permille);
    DX_HIP(hipGetLastError());
    DX_HIP(hipStreamSynchronize(grid->ctx->compute));
    return DCCRGX_OK;
}

int dccrgx_field_checksum(const dccrgx_grid* grid, int32_t fid, uint64_t out[2])
{
    DX_CHECK(grid && out && fid >= 0 && (size_t)fid < grid->fields.size(), DCCRGX_EINVAL, "bad argument");
    const Field& F = grid->fields[fid];
    DX_CHECK(F.elem == 4 && !F.variable, DCCRGX_EINVAL, "4-byte field expected");
    out[0] = out[1] = 0;
    const uint64_t n = grid->n_local;
    if (!n) return DCCRGX_OK;
    hipStream_t st = grid->ctx->compute;
    const unsigned nb = grid_for(n);
    uint64_t* d = nullptr;
    uint64_t* ids = nullptr;
    DX_HIP(dx_malloc(&d, (2 * (size_t)nb + 2) * 8));
    int s = DCCRGX_OK;
    uint64_t lin0 = 0, soff = 0;
    if (grid->uniform) {
        lin0 = grid->g.lo;
        soff = (uint64_t)(-grid->g.cbase * (int64_t)grid->g.S);
    } else {
        if (dx_malloc(&ids, n * 8) != hipSuccess) s = set_error(DCCRGX_ENOMEM, "checksum: no device memory");
        if (s == DCCRGX_OK) s = explicit_local_ids(grid, ids, st);
    }
    if (s == DCCRGX_OK) {
        hipLaunchKernelGGL(k_checksum, dim3(nb), dim3(256), 0, st, (const uint32_t*)F.ptr, n, lin0, soff,
                           (const uint64_t*)ids, d);
        hipLaunchKernelGGL(k_checksum_final, dim3(1), dim3(64), 0, st, (const uint64_t*)d, nb, d + 2 * nb);
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(out, d + 2 * nb, 16, hipMemcpyDeviceToHost, st) ||
            hipStreamSynchronize(st) != hipSuccess)
            s = set_error(DCCRGX_EHIP, "checksum kernel failed");
    }
    dx_free(ids);
    dx_free(d);
    if (s == DCCRGX_OK && grid->hy) {
        // the slab's sum holds the refined cells' slots and not their children:
        // correct it cell by cell (refined cells are few)
        const Hybrid& H = *grid->hy;
        const uint64_t soff = (uint64_t)(-grid->g.cbase * (int64_t)grid->g.S);
        auto value = [&](uint64_t slot, uint32_t* v) -> int {
            DX_HIP(hipMemcpy(v, (const uint32_t*)F.ptr + slot, 4, hipMemcpyDeviceToHost));
            return DCCRGX_OK;
        };
        for (uint64_t r : H.refined) {
            uint32_t v = 0;
            DX_TRY(value(r - 1 + soff, &v));
            out[0] -= v;
            out[1] -= (uint64_t)v * splitmix64(r);
        }
        for (size_t k = 0; k < H.children.size(); k++) {
            uint32_t v = 0;
            DX_TRY(value(H.child_slot[k], &v));
            out[0] += v;
            out[1] += (uint64_t)v * splitmix64(H.children[k]);
        }
    }
    return s;
}

int dccrgx_kernel_timer(dccrgx_grid* grid, int32_t reset, double* ms, uint64_t* launches)
{
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    TimerPool& T = g_timers[grid];
    if (reset) {
        DX_HIP(hipStreamSynchronize(grid->ctx->compute));
        T.used = 0;
        T.on = reset > 0;
        if (ms) *ms = 0;
        if (launches) *launches = 0;
        return DCCRGX_OK;
    }
    DX_HIP(hipStreamSynchronize(grid->ctx->compute));
    double tot = 0;
    for (size_t i = 0; i + 1 < T.used; i += 2) {
        float x = 0;
        DX_HIP(hipEventElapsedTime(&x, T.ev[i], T.ev[i + 1]));
        tot += x;
    }
    if (ms) *ms = tot;
    if (launches) *launches = T.used / 2;
    return DCCRGX_OK;
}

}  // extern "C"
