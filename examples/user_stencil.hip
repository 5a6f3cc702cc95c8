// user_stencil.hip -- user programs written against include/dccrgx_stencil.hpp:
// the reference's game of life (examples/game_of_life.cpp:54-79: count the
// live neighbors over cell.neighbors_of, then apply B3/S23) and a neighbor
// walk that digests each cell's (neighbor id, x, y, z) sequence, as device
// functors over a region's cells.  Built into examples/libuser_stencil.so
// (extern "C", called by tests/test_gpu_user_stencil.py and bench.py).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I../include
//         user_stencil.hip -o libuser_stencil.so -L../dccrg_amd -ldccrgx
#include "dccrgx_stencil.hpp"

namespace {

template <class T>
int field_ptr(const dccrgx_grid* grid, int32_t fid, T** p)
{
    void* v = nullptr;
    uint64_t n = 0;
    const int e = dccrgx_field_device_ptr(grid, fid, &v, &n);
    *p = (T*)v;
    return e;
}

__device__ inline uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace

extern "C" {

// one game-of-life half step over the region: live-neighbor counts of the
// cells into fcnt, the next state into fout (fin's ghosts must be current)
int us_gol(const dccrgx_grid* grid, int32_t hood_id, int32_t fin, int32_t fout, int32_t fcnt, int32_t region)
{
    const uint32_t* in;
    uint32_t *out, *cnt;
    int e = field_ptr(grid, fin, &in);
    if (!e) e = field_ptr(grid, fout, &out);
    if (!e) e = field_ptr(grid, fcnt, &cnt);
    if (e) return e;
    return dccrgx_user::for_each_cell(grid, hood_id, region, [=] __device__(const auto& cell) {
        uint32_t n = 0;
        cell.for_each_neighbor([&](const dccrgx_user::Neighbor& nb) { n += in[nb.slot] != 0u ? 1u : 0u; });
        cnt[cell.slot] = n;
        out[cell.slot] = n == 3u ? 1u : (n == 2u ? in[cell.slot] : 0u);
    });
}

// the same step with the neighbors' alive values staged
// (dccrgx_user::for_each_cell_staged: LDS tiles and a register window on
// uniform grids whose neighborhood is the cube or the faces); staged == 0
// sends every cell through the walk with the values loaded at the slots
int us_gol_staged(const dccrgx_grid* grid, int32_t hood_id, int32_t fin, int32_t fout, int32_t fcnt, int32_t region,
                  int32_t staged)
{
    const uint32_t* in;
    uint32_t *out, *cnt;
    int e = field_ptr(grid, fin, &in);
    if (!e) e = field_ptr(grid, fout, &out);
    if (!e) e = field_ptr(grid, fcnt, &cnt);
    if (e) return e;
    dccrgx_user::StagedOptions opt;
    opt.staged = staged != 0;
    opt.side_stream = staged != 2;  // 2: the edge launches on the caller's stream too
    if (staged == 3) opt.workgroups = 1;  // 3: one workgroup per tile, marching through every slice
    return dccrgx_user::for_each_cell_staged(
        grid, hood_id, region, dccrgx_user::Fields<uint32_t, 1>{{in}},
        [=] __device__(const auto& cell) {
            uint32_t n = 0;
            cell.for_each_neighbor([&](const auto& nb) { n += nb.value(0) != 0u ? 1u : 0u; });
            cnt[cell.slot] = n;
            // n == 3 ? 1 : (n == 2 ? value : 0), written without branches
            // (the nested conditional compiled to exec-mask branches: ~20
            // scalar and vector instructions per cell more)
            out[cell.slot] = (cell.value(0) & (0u - (uint32_t)(n == 2u))) | (uint32_t)(n == 3u);
        },
        nullptr, opt);
}

// us_digest with the neighbor ids as staged values (8-byte elements)
int us_digest_staged(const dccrgx_grid* grid, int32_t hood_id, int32_t region, int32_t fids, int32_t fcid,
                     int32_t fdig, int32_t fcnt)
{
    const uint64_t* ids;
    uint64_t *cid, *dig;
    uint32_t* cnt;
    int e = field_ptr(grid, fids, &ids);
    if (!e) e = field_ptr(grid, fcid, &cid);
    if (!e) e = field_ptr(grid, fdig, &dig);
    if (!e) e = field_ptr(grid, fcnt, &cnt);
    if (e) return e;
    return dccrgx_user::for_each_cell_staged(
        grid, hood_id, region, dccrgx_user::Fields<uint64_t, 1>{{ids}}, [=] __device__(const auto& cell) {
            uint64_t h = 0xCBF29CE484222325ull;
            uint32_t n = 0;
            cell.for_each_neighbor([&](const auto& nb) {
                const uint64_t v = mix64(nb.value(0)) + (uint64_t)(int64_t)nb.x * 0x100000001B3ull +
                                   (uint64_t)(int64_t)nb.y * 0x5851F42D4C957F2Dull +
                                   (uint64_t)(int64_t)nb.z * 0x14057B7EF767814Full;
                h = (h ^ v) * 0x00000100000001B3ull;
                n++;
            });
            cid[cell.slot] = cell.value(0) == cell.id ? cell.id : 0;
            dig[cell.slot] = h;
            cnt[cell.slot] = n;
        });
}

// an order-sensitive floating-point stencil over two staged f64 fields:
// out = u + sum over the neighbors in order of (w_nb * u_nb - 0.25 * u)
// (summed in the iteration order, so the rounding follows it); staged == 0:
// the walk
int us_fsum_staged(const dccrgx_grid* grid, int32_t hood_id, int32_t fu, int32_t fw, int32_t fout, int32_t region,
                   int32_t staged)
{
    const double *u, *wt;
    double* out;
    int e = field_ptr(grid, fu, &u);
    if (!e) e = field_ptr(grid, fw, &wt);
    if (!e) e = field_ptr(grid, fout, &out);
    if (e) return e;
    dccrgx_user::StagedOptions opt;
    opt.staged = staged != 0;
    return dccrgx_user::for_each_cell_staged(
        grid, hood_id, region, dccrgx_user::Fields<double, 2>{{u, wt}},
        [=] __device__(const auto& cell) {
            const double me = cell.value(0);
            double s = me;
            cell.for_each_neighbor([&](const auto& nb) { s += nb.value(1) * nb.value(0) - 0.25 * me; });
            out[cell.slot] = s;
        },
        nullptr, opt);
}

// the same over two staged f32 fields (4-byte elements: the LDS-DMA staged
// kernel with two fields)
int us_fsum32_staged(const dccrgx_grid* grid, int32_t hood_id, int32_t fu, int32_t fw, int32_t fout, int32_t region,
                     int32_t staged)
{
    const float *u, *wt;
    float* out;
    int e = field_ptr(grid, fu, &u);
    if (!e) e = field_ptr(grid, fw, &wt);
    if (!e) e = field_ptr(grid, fout, &out);
    if (e) return e;
    dccrgx_user::StagedOptions opt;
    opt.staged = staged != 0;
    if (staged == 3) opt.workgroups = 1;
    return dccrgx_user::for_each_cell_staged(
        grid, hood_id, region, dccrgx_user::Fields<float, 2>{{u, wt}},
        [=] __device__(const auto& cell) {
            // no contraction: the staged and walked instantiations of this
            // body round alike (with contraction the compiler fused them
            // differently, 1-2 ulp apart)
#pragma clang fp contract(off)
            const float me = cell.value(0);
            float s = me;
            cell.for_each_neighbor([&](const auto& nb) { s += nb.value(1) * nb.value(0) - 0.25f * me; });
            out[cell.slot] = s;
        },
        nullptr, opt);
}

// per cell: cid = the cell's id as for_each_cell reports it, dig = a digest of
// its neighbor sequence h = (h ^ (mix64(id) + x * K1 + y * K2 + z * K3)) * P
// over the neighbors in order (ids read from field fids, whose ghosts must be
// current), cnt = the number of neighbors
int us_digest(const dccrgx_grid* grid, int32_t hood_id, int32_t region, int32_t fids, int32_t fcid, int32_t fdig,
              int32_t fcnt)
{
    const uint64_t* ids;
    uint64_t *cid, *dig;
    uint32_t* cnt;
    int e = field_ptr(grid, fids, &ids);
    if (!e) e = field_ptr(grid, fcid, &cid);
    if (!e) e = field_ptr(grid, fdig, &dig);
    if (!e) e = field_ptr(grid, fcnt, &cnt);
    if (e) return e;
    return dccrgx_user::for_each_cell(grid, hood_id, region, [=] __device__(const auto& cell) {
        uint64_t h = 0xCBF29CE484222325ull;
        uint32_t n = 0;
        cell.for_each_neighbor([&](const dccrgx_user::Neighbor& nb) {
            const uint64_t v = mix64(ids[nb.slot]) + (uint64_t)(int64_t)nb.x * 0x100000001B3ull +
                               (uint64_t)(int64_t)nb.y * 0x5851F42D4C957F2Dull +
                               (uint64_t)(int64_t)nb.z * 0x14057B7EF767814Full;
            h = (h ^ v) * 0x00000100000001B3ull;
            n++;
        });
        cid[cell.slot] = cell.id;
        dig[cell.slot] = h;
        cnt[cell.slot] = n;
    });
}

// cells a region holds (dccrgx_stencil_view_get's n_cells), -1 on error
long long us_region_cells(const dccrgx_grid* grid, int32_t hood_id, int32_t region)
{
    dccrgx_stencil_view v;
    if (dccrgx_stencil_view_get(grid, hood_id, region, &v) != DCCRGX_OK) return -1;
    return (long long)v.n_cells;
}

}  // extern "C"

extern "C" {
// the neighbors of the cell at `slot` as the functor sees them: (id read from
// fids, x, y, z) into out (4 x int64 per neighbor, at most cap), count returned
// through *n (device); for debugging a walk
int us_list(const dccrgx_grid* grid, int32_t hood_id, int32_t fids, uint64_t slot, int64_t* out, uint32_t cap,
            uint32_t* n)
{
    const uint64_t* ids;
    int e = field_ptr(grid, fids, &ids);
    if (e) return e;
    return dccrgx_user::for_each_cell(grid, hood_id, DCCRGX_REGION_ALL, [=] __device__(const auto& cell) {
        if (cell.slot != slot) return;
        uint32_t k = 0;
        cell.for_each_neighbor([&](const dccrgx_user::Neighbor& nb) {
            if (k < cap) {
                out[4 * k] = (int64_t)ids[nb.slot];
                out[4 * k + 1] = nb.x;
                out[4 * k + 2] = nb.y;
                out[4 * k + 3] = nb.z;
            }
            k++;
        });
        *n = k;
    });
}
}  // extern "C"
