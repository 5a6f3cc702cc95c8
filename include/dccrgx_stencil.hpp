/* dccrgx_stencil.hpp -- device user stencils over a dccrgx grid (HIP, gfx950;
 * compile the including file with hipcc --offload-arch=gfx950 -std=c++17).
 *
 * The reference's users write their solver as a loop over a region's cells
 * and each cell's neighbors_of (examples/game_of_life.cpp:54-79,
 * tests/advection/solve.hpp:44-279):
 *
 *     for (const auto& cell: grid.inner_cells())
 *         for (const auto& nb: cell.neighbors_of)
 *             if (nb.data->is_alive) cell.data->live_neighbor_count++;
 *
 * over the iteration cache (Cells_Item {id, data, neighbors_of}, Neighbors_Item
 * {id, data, x, y, z}, dccrg.hpp:7395-7456, :11570-11712).  Here the same loop
 * is a device functor that for_each_cell() runs once per cell of the region,
 * one thread per cell:
 *
 *     uint32_t* alive = ...; uint32_t* count = ...;   // dccrgx_field_device_ptr
 *     dccrgx_user::for_each_cell(grid, DCCRGX_DEFAULT_NEIGHBORHOOD_ID, DCCRGX_REGION_INNER,
 *         [=] __device__ (const auto& cell) {
 *             uint32_t n = 0;
 *             cell.for_each_neighbor([&](const dccrgx_user::Neighbor& nb) { n += alive[nb.slot] != 0; });
 *             count[cell.slot] = n;
 *         });
 *
 * A cell's or neighbor's data is the element at its `slot` in every field
 * array (dccrgx_field_device_ptr); a remote neighbor's slot holds its ghost
 * copy (dccrgx_halo_update / _start + _wait first).  Neighbor offsets are the
 * reference's x, y, z: indices of the finest level.  Launches go to the
 * grid's compute stream unless a stream is passed; work on a stream of the
 * caller's must be finished (or the stream synchronised) before the grid's
 * next structural call (refine, load, new neighborhood, destroy), which frees
 * what the view points to.  Neighbors come in the
 * iteration cache's order (dccrg.hpp:11590-11640): unique (id, offset) pairs,
 * those whose id is not also a neighbor_to first, each group ascending by
 * (id, x, y, z) -- so floating-point sums over them round as the reference's
 * do.  Uniform grids compute them in closed form (nothing stored per cell),
 * grids with refined cells read their stencil rows.
 */
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <type_traits>

#include "dccrgx.h"

namespace dccrgx_user {

struct Neighbor {
    uint64_t slot;    /* index of the neighbor's data in every field array */
    int32_t x, y, z;  /* offset from the cell, indices of the finest level */
};

namespace detail {

/* the uniform geometry a kernel needs, by value (SGPRs) */
struct UniformGeo {
    uint64_t la, lb, lc, S, lo, hi;
    int64_t cbase;
    const int32_t* items; /* 8 per item: canonical a, b, c, mirror flag, x, y, z (iteration order) */
    const int64_t* delta; /* slot distance per item */
    int32_t K;
    int32_t pa, pb, pc;
    int32_t ra, rb, rc; /* reach per canonical axis */
    int32_t sym;        /* every item's mirror is an item (DCCRGX_SHAPE_SYMMETRIC) */
};

/* the iteration cache's order of two entries: (group, id, x, y, z) */
struct Key {
    int32_t grp;
    uint64_t id;
    int32_t x, y, z;
};

__host__ __device__ inline bool key_less(const Key& p, const Key& q)
{
    if (p.grp != q.grp) return p.grp < q.grp;
    if (p.id != q.id) return p.id < q.id;
    if (p.x != q.x) return p.x < q.x;
    if (p.y != q.y) return p.y < q.y;
    return p.z < q.z;
}

__host__ __device__ inline int64_t wrap(int64_t v, int64_t L)
{
    const int64_t r = v % L;
    return r < 0 ? r + L : r;
}

}  // namespace detail

/* a cell of a uniform grid: canonical indices (a fastest, c the partitioned
 * axis); neighbors in closed form, as the library's own kernels find them */
struct UniformCell {
    uint64_t slot; /* index of the cell's data in every field array */
    uint64_t id;   /* cell id */
    detail::UniformGeo g;
    int64_t a, b, c;

    /* neighbor of canonical (a0, b0, c0) at item (da, db, dc): false if it
     * falls outside a non-periodic grid (dccrg.hpp:4670-4672); else a + la * b
     * (wrapped), the wrapped and the unwrapped c */
    __host__ __device__ inline bool step(int64_t a0, int64_t b0, int64_t c0, int32_t da, int32_t db, int32_t dc, uint64_t& ab,
                                int64_t& cw, int64_t& cu) const
    {
        int64_t a2 = a0 + da, b2 = b0 + db;
        cu = c0 + dc;
        cw = cu;
        if (a2 < 0 || a2 >= (int64_t)g.la) {
            if (!g.pa) return false;
            a2 = detail::wrap(a2, (int64_t)g.la);
        }
        if (b2 < 0 || b2 >= (int64_t)g.lb) {
            if (!g.pb) return false;
            b2 = detail::wrap(b2, (int64_t)g.lb);
        }
        if (cu < 0 || cu >= (int64_t)g.lc) {
            if (!g.pc) return false;
            cw = detail::wrap(cu, (int64_t)g.lc);
        }
        ab = (uint64_t)a2 + g.la * (uint64_t)b2;
        return true;
    }

    __host__ __device__ inline Neighbor make(uint64_t nslot, int32_t k) const
    {
        Neighbor nb;
        nb.slot = nslot;
        nb.x = g.items[8 * k + 4];
        nb.y = g.items[8 * k + 5];
        nb.z = g.items[8 * k + 6];
        return nb;
    }

    template <class G>
    __host__ __device__ inline void for_each_neighbor(G&& fn) const
    {
        // no grid boundary within the reach: every item's neighbor exists at
        // a fixed slot distance, in the items' order
        const bool inside = a >= g.ra && a + g.ra < (int64_t)g.la && b >= g.rb && b + g.rb < (int64_t)g.lb &&
                            c >= g.rc && c + g.rc < (int64_t)g.lc;
        if (inside) {
            // unrolled, so that the neighbors' loads of many items are in
            // flight at once: fully for the default neighborhoods of length 1
            // (26 items) and 0 (6 items)
            if (g.K == 26) {
#pragma unroll
                for (int32_t k = 0; k < 26; k++) fn(make(slot + (uint64_t)g.delta[k], k));
            } else if (g.K == 6) {
#pragma unroll
                for (int32_t k = 0; k < 6; k++) fn(make(slot + (uint64_t)g.delta[k], k));
            } else {
#pragma unroll 8
                for (int32_t k = 0; k < g.K; k++) fn(make(slot + (uint64_t)g.delta[k], k));
            }
            return;
        }
        // no periodic wrap within the reach: the items' order is still the
        // iteration order (ids grow with (c, b, a)), items past a non-periodic
        // boundary are dropped.  An entry is a neighbor_to exactly when the
        // mirrored item exists -- always, for a symmetric neighborhood; else
        // only if no wrap is within twice the reach (a neighbor's items could
        // reach back through it)
        const int64_t m = g.sym ? 1 : 2;
        const bool nowrap = (!g.pa || (a >= m * g.ra && a + m * g.ra < (int64_t)g.la)) &&
                            (!g.pb || (b >= m * g.rb && b + m * g.rb < (int64_t)g.lb)) &&
                            (!g.pc || (c >= m * g.rc && c + m * g.rc < (int64_t)g.lc));
        if (nowrap) {
            for (int32_t k = 0; k < g.K; k++) {
                uint64_t ab;
                int64_t cw, cu;
                if (!step(a, b, c, g.items[8 * k], g.items[8 * k + 1], g.items[8 * k + 2], ab, cw, cu)) continue;
                fn(make(ab + g.S * (uint64_t)(cu - g.cbase), k));  // the slot of c + dc, local or ghost
            }
            return;
        }
        // near a wrap: pick the entries in key order, one per pass
        const uint64_t self = (uint64_t)a + g.la * (uint64_t)b + g.S * (uint64_t)c;
        detail::Key prev{-1, 0, 0, 0, 0};
        for (int32_t pass = 0; pass < g.K; pass++) {
            int32_t bk = -1;
            uint64_t bslot = 0;
            detail::Key best{0, 0, 0, 0, 0};
            for (int32_t k = 0; k < g.K; k++) {
                uint64_t ab;
                int64_t cw, cu;
                if (!step(a, b, c, g.items[8 * k], g.items[8 * k + 1], g.items[8 * k + 2], ab, cw, cu)) continue;
                const uint64_t nlin = ab + g.S * (uint64_t)cw;
                // a local neighbor (also one reached through a periodic wrap)
                // is read from its own slot, a remote one from its ghost slot
                const int64_t cs = (nlin >= g.lo && nlin < g.hi) ? cw : cu;
                int32_t grp = g.items[8 * k + 3];
                if (!grp) {  // another item of the neighbor may reach this cell through a wrap
                    const int64_t na = (int64_t)(ab % g.la), nbb = (int64_t)(ab / g.la);
                    for (int32_t j = 0; j < g.K && !grp; j++) {
                        uint64_t ab2;
                        int64_t cw2, cu2;
                        if (step(na, nbb, cw, g.items[8 * j], g.items[8 * j + 1], g.items[8 * j + 2], ab2, cw2, cu2))
                            grp = ab2 + g.S * (uint64_t)cw2 == self ? 1 : 0;
                    }
                }
                const detail::Key key{grp, nlin, g.items[8 * k + 4], g.items[8 * k + 5], g.items[8 * k + 6]};
                if (!detail::key_less(prev, key)) continue;
                if (bk < 0 || detail::key_less(key, best)) {
                    best = key;
                    bk = k;
                    bslot = ab + g.S * (uint64_t)(cs - g.cbase);
                }
            }
            if (bk < 0) break;
            fn(make(bslot, bk));
            prev = best;
        }
    }
};

/* a cell of a grid with refined cells: its stored stencil row */
struct ExplicitCell {
    uint64_t slot;
    uint64_t id;
    const uint64_t* row;
    const uint32_t* nbr_slot;
    const int32_t* nbr_off;
    uint32_t q; /* local position */

    template <class G>
    __host__ __device__ inline void for_each_neighbor(G&& fn) const
    {
        const uint64_t e1 = row[q + 1];
        uint64_t e = row[q];
        auto one = [&](uint64_t k) {
            Neighbor nb;
            nb.slot = nbr_slot[k];
            nb.x = nbr_off[3 * k];
            nb.y = nbr_off[3 * k + 1];
            nb.z = nbr_off[3 * k + 2];
            fn(nb);
        };
        // each lane walks its own row: four entries per 16-byte load (slots)
        // and three (offsets) once the row is at a multiple of four -- a
        // quarter of the load instructions, each line used for more entries
        for (; e < e1 && (e & 3); e++) one(e);
        for (; e + 4 <= e1; e += 4) {
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            typedef int32_t i4 __attribute__((ext_vector_type(4)));
            const u4 s = *reinterpret_cast<const u4*>(nbr_slot + e);
            const i4* po = reinterpret_cast<const i4*>(nbr_off + 3 * e);
            const i4 o0 = po[0], o1 = po[1], o2 = po[2];
            const int32_t o[12] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w, o2.x, o2.y, o2.z, o2.w};
            const uint32_t sl[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                Neighbor nb;
                nb.slot = sl[k];
                nb.x = o[3 * k];
                nb.y = o[3 * k + 1];
                nb.z = o[3 * k + 2];
                fn(nb);
            }
        }
        for (; e < e1; e++) one(e);
    }
};

namespace detail {

/* uniform: 256 consecutive cells of a slice per workgroup, `chunk` slices of
 * them per thread (consecutive lanes on consecutive cells: coalesced) */
template <class F>
__global__ void __launch_bounds__(256) k_user_uniform(UniformGeo g, int64_t s0, int64_t s1, uint32_t tiles,
                                                      uint32_t chunk, F f)
{
    const uint32_t t = blockIdx.x % tiles, k = blockIdx.x / tiles;
    const uint64_t i = (uint64_t)t * 256 + threadIdx.x;
    if (i >= g.S) return;
    const uint64_t b = i / g.la, a = i - b * g.la;
    const int64_t sb = s0 + (int64_t)k * chunk, se = sb + (int64_t)chunk < s1 ? sb + (int64_t)chunk : s1;
    for (int64_t s = sb; s < se; s++) {
        const int64_t c = s + g.cbase;
        const uint64_t lin = i + g.S * (uint64_t)c;
        if (lin < g.lo || lin >= g.hi) continue;
        UniformCell cell;
        cell.slot = i + g.S * (uint64_t)s;
        cell.id = lin + 1;
        cell.g = g;
        cell.a = (int64_t)a;
        cell.b = (int64_t)b;
        cell.c = c;
        f(cell);
    }
}

template <class F>
__global__ void __launch_bounds__(256) k_user_explicit(const uint32_t* __restrict__ pos,
                                                       const uint32_t* __restrict__ local_slot,
                                                       const uint32_t* __restrict__ local_g,
                                                       const uint64_t* __restrict__ leaves,
                                                       const uint64_t* __restrict__ row,
                                                       const uint32_t* __restrict__ nbr_slot,
                                                       const int32_t* __restrict__ nbr_off, uint64_t n, F f)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        ExplicitCell cell;
        cell.q = pos[i];
        cell.slot = local_slot[cell.q];
        cell.id = leaves[local_g[cell.q]];
        cell.row = row;
        cell.nbr_slot = nbr_slot;
        cell.nbr_off = nbr_off;
        f(cell);
    }
}

/* the uniform geometry of a view */
inline UniformGeo uniform_geo(const dccrgx_stencil_view& v)
{
    UniformGeo g;
    g.la = v.la;
    g.lb = v.lb;
    g.lc = v.lc;
    g.S = v.la * v.lb;
    g.lo = v.lo;
    g.hi = v.hi;
    g.cbase = v.cbase;
    g.items = v.items;
    g.delta = v.item_delta;
    g.K = v.n_items;
    g.pa = v.per[0];
    g.pb = v.per[1];
    g.pc = v.per[2];
    g.ra = v.reach[0];
    g.rb = v.reach[1];
    g.rc = v.reach[2];
    g.sym = (v.shape & DCCRGX_SHAPE_SYMMETRIC) != 0;
    return g;
}

/* the walk over whole storage slices [s0, s1) of a uniform grid */
template <class F>
int launch_slices(const UniformGeo& g, int64_t s0, int64_t s1, F f, hipStream_t st)
{
    const int64_t nsl = s1 - s0;
    if (nsl <= 0) return DCCRGX_OK;
    const uint64_t tiles = (g.S + 255) / 256;
    if (tiles >= (1ull << 31)) return DCCRGX_EINVAL;
    // about 2^20 workgroups (4096 per CU) and never more than 2^31
    uint64_t chunk = (tiles * (uint64_t)nsl + (1u << 20) - 1) >> 20;
    if (chunk < 1) chunk = 1;
    const uint64_t nch = ((uint64_t)nsl + chunk - 1) / chunk;
    if (tiles * nch >= (1ull << 31)) return DCCRGX_EINVAL;
    hipLaunchKernelGGL(k_user_uniform<F>, dim3((unsigned)(tiles * nch)), dim3(256), 0, st, g, s0, s1,
                       (uint32_t)tiles, (uint32_t)chunk, f);
    return DCCRGX_OK;
}

}  // namespace detail

/* Launch f(cell) for every cell of the region described by v on stream st
 * (asynchronous).  f is a device functor taking `const auto&` (UniformCell on
 * uniform grids, ExplicitCell otherwise).  Returns a DCCRGX_* code. */
template <class F>
int for_each_cell(const dccrgx_stencil_view& v, F f, hipStream_t st)
{
    if (v.n_cells == 0) return DCCRGX_OK;
    if (v.kind == 0) {
        const detail::UniformGeo g = detail::uniform_geo(v);
        for (int r = 0; r < 2; r++) {
            const int e = detail::launch_slices(g, (int64_t)v.s0[r], (int64_t)v.s1[r], f, st);
            if (e != DCCRGX_OK) return e;
        }
    } else {
        uint64_t blocks = (v.n_cells + 255) / 256;
        if (blocks > 65536) blocks = 65536;
        hipLaunchKernelGGL(detail::k_user_explicit<F>, dim3((unsigned)blocks), dim3(256), 0, st, v.pos,
                           v.local_slot, v.local_g, v.leaves, v.row, v.nbr_slot, v.nbr_off, v.n_cells, f);
    }
    return hipGetLastError() == hipSuccess ? DCCRGX_OK : DCCRGX_EHIP;
}

/* the same for neighborhood hood_id and region (DCCRGX_REGION_*) of a grid,
 * on the grid's compute stream unless st is given */
template <class F>
int for_each_cell(const dccrgx_grid* grid, int32_t hood_id, int32_t region, F f, hipStream_t st = nullptr)
{
    dccrgx_stencil_view v;
    const int e = dccrgx_stencil_view_get(grid, hood_id, region, &v);
    if (e != DCCRGX_OK) return e;
    return for_each_cell(v, f, st ? st : (hipStream_t)v.stream);
}

/* ------------------------------------------------------------------------
 * Staged launches: the caller names the fields its functor reads at the
 * neighbors (one element type T, NF fields), and the functor reads them as
 * values -- cell.value(j), nb.value(j) -- instead of through slots:
 *
 *     dccrgx_user::for_each_cell_staged(grid, hood, region, dccrgx_user::Fields<uint32_t, 1>{{alive}},
 *         [=] __device__ (const auto& cell) {
 *             uint32_t n = 0;
 *             cell.for_each_neighbor([&](const auto& nb) { n += nb.value(0) != 0; });
 *             count[cell.slot] = n;
 *         });
 *
 * Same cells, same neighbors in the same order as for_each_cell (nb.slot,
 * x, y, z are there too).  On uniform grids whose neighborhood is the 26-cell
 * cube or the 6 faces (DCCRGX_SHAPE_CUBE1 / _FACES: the default
 * neighborhoods of length 1 and 0), the cells no grid boundary reaches run
 * k_staged: a workgroup owns a 64 x (NW * NB) tile of the (A, B) plane and
 * marches along C; each plane of the declared fields is read from HBM once
 * (16-byte loads, +1 apron) into LDS, every lane reads the 3 x (NB + 2)
 * values around its column of NB cells into a register window of three
 * planes, and the functor's neighbor loop is unrolled over compile-time
 * offsets into that window.  4-byte fields on rows of a multiple of 4 cells
 * run k_staged_g instead: the planes come into LDS by LDS-DMA buffer loads,
 * two in flight, and with A not periodic the edge columns are its own cells.
 * The other cells within reach of a grid boundary (the rest of the ring of
 * each slice, the slices next to a C boundary) run in separate launches (the
 * edge rows' march k_staged_rows, the exact-order walk); so do other
 * neighborhoods and refined grids.  Build knobs (defaults measured fastest on
 * 2048^3): DCCRGX_STAGED_GLDS, _COLS, _ROWS, _G_MINWG, _NB1, _PF.
 * ---------------------------------------------------------------------- */

template <class T, int NF>
struct Fields {
    const T* p[NF];
};

/* a neighbor with the values of the declared fields */
template <class T, int NF>
struct ValueNeighbor : Neighbor {
    T v[NF];
    __host__ __device__ inline T value(int j) const { return v[j]; }
};

/* a walk cell (UniformCell / ExplicitCell) whose values are loaded from the
 * fields at the slots */
template <class Cell, class T, int NF>
struct LoadedCell {
    Cell cell;
    Fields<T, NF> fld;
    uint64_t slot, id;

    __host__ __device__ inline T value(int j) const { return fld.p[j][slot]; }

    template <class G>
    __host__ __device__ inline void for_each_neighbor(G&& fn) const
    {
        cell.for_each_neighbor([&](const Neighbor& nb) {
            ValueNeighbor<T, NF> v;
            v.slot = nb.slot;
            v.x = nb.x;
            v.y = nb.y;
            v.z = nb.z;
#pragma unroll
            for (int j = 0; j < NF; j++) v.v[j] = fld.p[j][nb.slot];
            fn(v);
        });
    }
};

namespace detail {

/* the items of the staged shapes, canonical (a, b, c) of item k in the
 * iteration order of a cell no periodic wrap reaches (ascending (c, b, a);
 * every entry is also a neighbor_to) */
template <int SHAPE>
struct StagedItems;
template <>
struct StagedItems<DCCRGX_SHAPE_CUBE1> {
    static constexpr int K = 26;
    __host__ __device__ static constexpr int d(int k, int axis)
    {
        return ((k < 13 ? k : k + 1) / (axis == 0 ? 1 : (axis == 1 ? 3 : 9))) % 3 - 1;
    }
};
template <>
struct StagedItems<DCCRGX_SHAPE_FACES> {
    static constexpr int K = 6;  // (0,0,-1) (0,-1,0) (-1,0,0) (1,0,0) (0,1,0) (0,0,1)
    __host__ __device__ static constexpr int d(int k, int axis)
    {
        return axis == 2 ? (k == 0 ? -1 : (k == 5 ? 1 : 0))
                         : (axis == 1 ? (k == 1 ? -1 : (k == 4 ? 1 : 0)) : (k == 2 ? -1 : (k == 3 ? 1 : 0)));
    }
};

/* where a cell's plane sits on a periodic C axis: inside, or the first / last
 * slice, whose neighbors across the wrap have the largest / smallest ids (so
 * their c-groups come last / first in the iteration order) */
enum { CLS_MID = 0, CLS_LOW = 1, CLS_HIGH = 2 };

__host__ __device__ constexpr int class_dc(int cls, int grp)
{
    return cls == CLS_MID ? grp - 1 : (cls == CLS_LOW ? (grp == 2 ? -1 : grp) : (grp == 0 ? 1 : grp - 2));
}

struct StagedGeo {
    uint64_t la, lb, lc, S, lo, hi;
    int64_t cbase;
    int64_t s0, s1;    // storage slices computed by the launch
    int64_t chunk;     // slices per workgroup
    int64_t wrap_lo;   // storage slice to read for the plane below canonical 0 (wrap launches)
    int64_t wrap_hi;   // ... above canonical LC - 1
    uint32_t tiles_a, tiles_b, nwg;
    int32_t pa, pb, pc;
    int32_t inv[3];    // x, y, z -> canonical axis
    int32_t scale;
    int64_t nslices;   // storage slices
    int32_t cols_in;   // k_staged_g also takes the columns a = 0, LA - 1 (rows 1 .. LB - 2; A not periodic)
};

/* a cell of the staged kernels: values from the register window
 * W[field][plane][row][col] (planes c - 1, c, c + 1, read from storage slices
 * ps0..ps2); every neighbor exists (cells next to a grid boundary or a
 * periodic wrap in A / B run the edge walk) */
template <class T, int NF, int SHAPE, int NB, int CLS>
struct StagedCell {
    uint64_t slot, id;
    const T (*w)[3][NB + 2][3];
    int64_t la, S;
    int64_t ps0, ps1, ps2;
    int32_t inv[3], scale;
    int r;  // the cell's row in the window is r + 1

    __host__ __device__ inline T value(int j) const { return w[j][1][r + 1][1]; }

    template <class G>
    __host__ __device__ inline void for_each_neighbor(G&& fn) const
    {
        typedef StagedItems<SHAPE> It;
#pragma unroll
        for (int grp = 0; grp < 3; grp++) {
            const int dcg = class_dc(CLS, grp);
#pragma unroll
            for (int k = 0; k < It::K; k++) {
                const int da = It::d(k, 0), db = It::d(k, 1), dc = It::d(k, 2);
                if (dc != dcg) continue;
                ValueNeighbor<T, NF> nb;
                const int64_t dps = dc < 0 ? ps0 - ps1 : (dc > 0 ? ps2 - ps1 : 0);
                nb.slot = slot + (uint64_t)((int64_t)da + la * db + S * dps);
                nb.x = (inv[0] == 0 ? da : (inv[0] == 1 ? db : dc)) * scale;
                nb.y = (inv[1] == 0 ? da : (inv[1] == 1 ? db : dc)) * scale;
                nb.z = (inv[2] == 0 ? da : (inv[2] == 1 ? db : dc)) * scale;
#pragma unroll
                for (int j = 0; j < NF; j++) nb.v[j] = w[j][dc + 1][r + 1 + db][da + 1];
                fn(nb);
            }
        }
    }
};

/* a cell of the edge walk (a cell of a staged shape next to a grid boundary
 * or a periodic wrap): its neighbors in closed form, values read at their
 * slots.  Per axis the neighbors' coordinates sort as -1, 0, +1, or -- at
 * the first / last cell of a periodic axis of >= 3 cells -- as 0, +1, -1 /
 * +1, -1, 0 (the wrapped one has the largest / smallest index), so nested
 * loops over those orders give the iteration order (ids ascending by (c, b,
 * a)); neighbors past a non-periodic boundary are dropped. */
template <class T, int NF, int SHAPE>
struct EdgeCell {
    uint64_t slot, id;
    Fields<T, NF> fld;
    uint64_t la, lb, lc, S, lo, hi;
    int64_t a, b, c, cbase;  // c canonical
    int32_t pa, pb, pc;
    int32_t inv[3], scale;

    __host__ __device__ inline T value(int j) const { return fld.p[j][slot]; }

    __host__ __device__ static inline int axis_class(int64_t x, uint64_t L, int32_t p)
    {
        return !p ? CLS_MID : (x == 0 ? CLS_LOW : (x == (int64_t)L - 1 ? CLS_HIGH : CLS_MID));
    }

    template <class G>
    __host__ __device__ inline void for_each_neighbor(G&& fn) const
    {
        walk(fn, [&](int j, uint64_t nslot, int, int, int) { return fld.p[j][nslot]; });
    }

    // the neighbors in the iteration cache's order, each value from
    // load(field, slot, da, db, dc)
    template <class G, class L>
    __host__ __device__ inline void walk(G&& fn, L&& load) const
    {
        const int ka = axis_class(a, la, pa), kb = axis_class(b, lb, pb), kc = axis_class(c, lc, pc);
#pragma unroll
        for (int rc = 0; rc < 3; rc++) {
#pragma unroll
            for (int rb = 0; rb < 3; rb++) {
#pragma unroll
                for (int ra = 0; ra < 3; ra++) {
                    const int da = class_dc(ka, ra), db = class_dc(kb, rb), dc = class_dc(kc, rc);
                    const int nz = (da != 0) + (db != 0) + (dc != 0);
                    if (nz == 0 || (SHAPE == DCCRGX_SHAPE_FACES && nz != 1)) continue;
                    int64_t a2 = a + da, b2 = b + db, cu = c + dc, cw = cu;
                    if (a2 < 0 || a2 >= (int64_t)la) {
                        if (!pa) continue;
                        a2 = a2 < 0 ? a2 + (int64_t)la : a2 - (int64_t)la;
                    }
                    if (b2 < 0 || b2 >= (int64_t)lb) {
                        if (!pb) continue;
                        b2 = b2 < 0 ? b2 + (int64_t)lb : b2 - (int64_t)lb;
                    }
                    if (cu < 0 || cu >= (int64_t)lc) {
                        if (!pc) continue;
                        cw = cu < 0 ? cu + (int64_t)lc : cu - (int64_t)lc;
                    }
                    const uint64_t ab = (uint64_t)a2 + la * (uint64_t)b2, nlin = ab + S * (uint64_t)cw;
                    // a local neighbor (also one across a wrap) is read from its
                    // own slot, a remote one from its ghost slot
                    const int64_t cs = (nlin >= lo && nlin < hi) ? cw : cu;
                    ValueNeighbor<T, NF> nb;
                    nb.slot = ab + S * (uint64_t)(cs - cbase);
                    nb.x = (inv[0] == 0 ? da : (inv[0] == 1 ? db : dc)) * scale;
                    nb.y = (inv[1] == 0 ? da : (inv[1] == 1 ? db : dc)) * scale;
                    nb.z = (inv[2] == 0 ? da : (inv[2] == 1 ? db : dc)) * scale;
#pragma unroll
                    for (int j = 0; j < NF; j++) nb.v[j] = load(j, nb.slot, da, db, dc);
                    fn(nb);
                }
            }
        }
    }
};

template <int VEC, class T>
struct StagedChunk {
    typedef uint32_t type __attribute__((ext_vector_type(4)));  // VEC elements, 16 bytes
};
template <class T>
struct StagedChunk<1, T> {
    typedef T type;
};

template <class V>
__device__ inline V buffer_load(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    if constexpr (sizeof(V) == 16) {
        return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
    } else if constexpr (sizeof(V) == 8) {
        return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
    } else if constexpr (sizeof(V) == 4) {
        return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
    } else if constexpr (sizeof(V) == 2) {
        return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b16(r, (int)off, 0, 0));
    } else {
        return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b8(r, (int)off, 0, 0));
    }
}

/* One workgroup's tile: 64 columns (lane l: column a0 + l) x NW * NB rows
 * (wave w: rows w * NB ..) of the (A, B) plane, + 1 apron.  Planes go HBM ->
 * registers (16-byte loads, VEC elements; VEC = 1: element loads) -> LDS ->
 * each lane's 3 x (NB + 2) window of one plane. */
template <class T, int NF, int NW, int NB, int VEC>
struct StagedTile {
    typedef typename StagedChunk<VEC, T>::type Chunk;
    static constexpr int NT = 64 * NW, TB = NW * NB, WB = TB + 2;
    static constexpr int X0 = VEC > 1 ? VEC : 1;  // LDS row: apron at X0 - 1, cells at X0.., apron at X0 + 64
    static constexpr int RS = 64 + 2 * X0;
    static constexpr int CR = 64 / VEC;           // chunks per tile row
    static constexpr int NCH = (WB * CR + NT - 1) / NT;

    uint32_t moff[NCH], mdst[NCH], mmask;
    uint32_t eoff, edst;
    bool eok;

    __device__ inline void init(const StagedGeo& g, int64_t a0, int64_t b0, int t)
    {
        const int64_t LA = (int64_t)g.la, LB = (int64_t)g.lb;
        mmask = 0;
#pragma unroll
        for (int i = 0; i < NCH; i++) {
            const int e = t + NT * i;
            const int row = e / CR, q = e - row * CR;
            const int64_t a = a0 + VEC * q, b = b0 - 1 + row;
            const bool ok = e < WB * CR && a < LA && b >= 0 && b < LB;
            moff[i] = ok ? (uint32_t)((a + LA * b) * (int64_t)sizeof(T)) : 0u;  // bytes
            mdst[i] = ok ? (uint32_t)(row * RS + X0 + VEC * q) : 0u;
            mmask |= ok ? (1u << i) : 0u;
        }
        eoff = edst = 0;
        eok = false;
        if (t < 2 * WB) {
            const int row = t >> 1;
            const int64_t a = (t & 1) ? a0 + 64 : a0 - 1, b = b0 - 1 + row;
            eok = a >= 0 && a < LA && b >= 0 && b < LB;
            eoff = eok ? (uint32_t)((a + LA * b) * (int64_t)sizeof(T)) : 0u;
            edst = (uint32_t)(row * RS + ((t & 1) ? X0 + 64 : X0 - 1));
        }
    }
    __device__ inline void fetch(const Fields<T, NF>& fld, uint64_t S, int64_t sc, Chunk (&FM)[NF][NCH],
                                 T (&FE)[NF]) const
    {
#pragma unroll
        for (int j = 0; j < NF; j++) {
            // buffer loads: a scalar resource per plane + a 32-bit byte
            // offset per load; unconditional (a chunk outside the grid reads
            // the plane's first bytes and is not stashed)
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<T*>(fld.p[j] + (uint64_t)sc * S), 0, (int)(S * sizeof(T)), 0x00020000);
#pragma unroll
            for (int i = 0; i < NCH; i++) FM[j][i] = buffer_load<Chunk>(rs, moff[i]);
            FE[j] = buffer_load<T>(rs, eoff);
        }
    }
    __device__ inline void stash(T* lds, const Chunk (&FM)[NF][NCH], const T (&FE)[NF]) const
    {
#pragma unroll
        for (int j = 0; j < NF; j++) {
            T* l = lds + j * WB * RS;
#pragma unroll
            for (int i = 0; i < NCH; i++)
                if ((mmask >> i) & 1u) *reinterpret_cast<Chunk*>(l + mdst[i]) = FM[j][i];
            if (eok) l[edst] = FE[j];
        }
    }
    // the lane's 3 x (NB + 2) values of the plane in lds into W[.][pl]
    __device__ static inline void window(const T* lds, int w, int lane, T (&W)[NF][3][NB + 2][3], int pl)
    {
#pragma unroll
        for (int j = 0; j < NF; j++)
#pragma unroll
            for (int rr = 0; rr < NB + 2; rr++)
#pragma unroll
                for (int q = 0; q < 3; q++) W[j][pl][rr][q] = lds[(j * WB + w * NB + rr) * RS + X0 + lane + q - 1];
    }
};

/* f(std::integral_constant<int, J>()) for J = 0 .. N - 1, unrolled at compile
 * time (register arrays indexed by J stay registers) */
template <int J, int N>
struct StaticFor {
    template <class G>
    __device__ static inline void run(G& g)
    {
        g(std::integral_constant<int, J>());
        StaticFor<J + 1, N>::run(g);
    }
};
template <int N>
struct StaticFor<N, N> {
    template <class G>
    __device__ static inline void run(G&)
    {
    }
};

/* XCD-aware workgroup order: each XCD takes a contiguous run of tiles
 * (vertically adjacent tiles share apron rows through its L2) */
__device__ inline uint32_t xcd_wgid(uint32_t nwg)
{
    const uint32_t bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

/* f on the NB cells of plane c of the lane's column (window planes read from
 * storage slices ps); only cells with a in [1, LA - 1), b in [1, LB - 1).  A
 * wave whose rows all qualify on a plane this rank holds (nearly every wave)
 * calls f with no per-cell test, the slots and ids stepped from the column's
 * first (20.7 against 21.2-21.5 ms per 2048^3 step, profiles/s31_staged_ab.log). */
template <class T, int NF, int SHAPE, int NB, int CLS, class F>
__device__ inline void staged_cells(const StagedGeo& g, F& f, const T (&W)[NF][3][NB + 2][3], const int64_t (&ps)[3],
                                    int64_t c, int64_t a, int64_t bw)
{
    const int64_t LA = (int64_t)g.la, LB = (int64_t)g.lb, cg = c + g.cbase;
    if (a < 1 || a + 1 >= LA) return;
    const uint64_t plin = g.S * (uint64_t)cg;
    const bool plane_local = plin >= g.lo && plin + g.S <= g.hi;  // uniform
    StagedCell<T, NF, SHAPE, NB, CLS> cell;
    cell.w = W;
    cell.la = LA;
    cell.S = (int64_t)g.S;
    cell.ps0 = ps[0];
    cell.ps1 = ps[1];
    cell.ps2 = ps[2];
    cell.inv[0] = g.inv[0];
    cell.inv[1] = g.inv[1];
    cell.inv[2] = g.inv[2];
    cell.scale = g.scale;
    const uint64_t col = (uint64_t)a + g.la * (uint64_t)bw;
    const uint64_t slot0 = (uint64_t)c * g.S + col, id0 = plin + col + 1;
    if (plane_local && bw >= 1 && bw + NB < LB) {  // wave-uniform
#pragma unroll
        for (int k = 0; k < NB; k++) {
            cell.slot = slot0 + g.la * (uint64_t)k;
            cell.id = id0 + g.la * (uint64_t)k;
            cell.r = k;
            f(cell);
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < NB; k++) {
        const int64_t b = bw + k;
        if (b < 1 || b + 1 >= LB) continue;
        const uint64_t lin = plin + (uint64_t)a + g.la * (uint64_t)b;
        if (!plane_local && (lin < g.lo || lin >= g.hi)) continue;
        cell.slot = slot0 + g.la * (uint64_t)k;
        cell.id = lin + 1;
        cell.r = k;
        f(cell);
    }
}

/* The staged kernel over storage slices [s0, s1), none of them the first or
 * last slice of a periodic C: a workgroup marches its tile through `chunk`
 * slices; plane q of the march is fetched PF planes ahead into its own
 * registers (the loop is unrolled by PF so loads land where they are used),
 * stashed to one of two LDS buffers, and read into the register window. */
template <class T, int NF, int SHAPE, int NW, int NB, int VEC, int PF, class F>
__global__ void __launch_bounds__(64 * NW) k_staged(StagedGeo g, Fields<T, NF> fld, F f)
{
    typedef StagedTile<T, NF, NW, NB, VEC> Tile;
    typedef typename Tile::Chunk Chunk;
    __shared__ __attribute__((aligned(16))) T P[2][NF][Tile::WB][Tile::RS];

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t wgid = xcd_wgid(g.nwg);
    const uint32_t tiles = g.tiles_a * g.tiles_b;
    const uint32_t tile_id = wgid % tiles;
    const int64_t chunk_id = wgid / tiles;
    const int64_t a0 = (int64_t)(tile_id % g.tiles_a) * 64;
    const int64_t b0 = (int64_t)(tile_id / g.tiles_a) * Tile::TB;
    const int64_t c0 = g.s0 + chunk_id * g.chunk;
    const int64_t c1 = min(g.s1, c0 + g.chunk);
    if (c0 >= c1) return;

    Tile tile;
    tile.init(g, a0, b0, t);
    Chunk FM[PF][NF][Tile::NCH];
    T FE[PF][NF];
    T W[NF][3][NB + 2][3];
    // plane q = storage slice c0 - 1 + q, q in [0, Q); computed: q in [2, Q) -> slice c0 + q - 2
    const int64_t Q = c1 - c0 + 2;
    auto pre = [&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if (j < Q) tile.fetch(fld, g.S, c0 - 1 + j, FM[j], FE[j]);
    };
    StaticFor<0, PF>::run(pre);
    const int64_t a = a0 + lane, bw = b0 + w * NB;
    for (int64_t qb = 0; qb < Q; qb += PF) {
        auto step = [&](auto jc) {
            constexpr int j = decltype(jc)::value;
            const int64_t q = qb + j;
            if (q < Q) {
                T* lds = &P[q & 1][0][0][0];
                tile.stash(lds, FM[j], FE[j]);
                if (q + PF < Q) tile.fetch(fld, g.S, c0 - 1 + q + PF, FM[j], FE[j]);
                __syncthreads();
                Tile::window(lds, w, lane, W, 2);
                if (q >= 2) {
                    const int64_t c = c0 + q - 2;
                    const int64_t pls[3] = {c - 1, c, c + 1};
                    staged_cells<T, NF, SHAPE, NB, CLS_MID>(g, f, W, pls, c, a, bw);
                }
                // the window moves down a plane (a march unrolled by three
                // with the planes' roles rotated instead measured 10 % slower:
                // three times the code, profiles/s31_staged_ab.log)
#pragma unroll
                for (int jj = 0; jj < NF; jj++)
#pragma unroll
                    for (int rr = 0; rr < NB + 2; rr++)
#pragma unroll
                        for (int qq = 0; qq < 3; qq++) {
                            W[jj][0][rr][qq] = W[jj][1][rr][qq];
                            W[jj][1][rr][qq] = W[jj][2][rr][qq];
                        }
            }
        };
        StaticFor<0, PF>::run(step);
    }
}

/* k_staged for 4-byte elements on rows of a multiple of 4 cells, its planes
 * fetched by buffer loads that write LDS directly (no register staging): two
 * planes in flight in three LDS buffers at no register cost (the register
 * path's second plane in flight costs ~40 VGPRs and a wave per SIMD).  A
 * field's plane image is the tile's WB rows of 64 cells, dense (a 64-lane
 * 16-byte load writes 1 KiB contiguously: four rows), then its two apron
 * columns as [WB][2].  Wave w issues the loads i = w, w + NW, ... of each
 * field; the wave with one fewer also loads the aprons (4 bytes per lane).
 * The next plane's loads are issued after the cells' stores, so a wave's own
 * loads of plane q are the oldest of its memory operations but those of plane
 * q + 1: `s_waitcnt vmcnt(G_w)` (G_w its loads per plane) leaves exactly
 * plane q + 1 in flight; a raw s_barrier then publishes every wave's share
 * (__syncthreads would wait for every load in flight). */
template <class T, int NF, int NW, int NB>
struct StagedTileG {
    static_assert(sizeof(T) == 4, "LDS-DMA staging: 4-byte elements");
    static constexpr int TB = NW * NB, WB = TB + 2;
    static_assert(2 * WB <= 64, "the apron columns are one 64-lane load");
    static constexpr int MAIN = WB * 64;         // elements of the dense rows
    static constexpr int PLANE = MAIN + 2 * WB;  // + the apron columns
    static constexpr int NCHUNK = MAIN / 4;      // 16-byte loads
    static constexpr int NI = (NCHUNK + 63) / 64;
    static constexpr int KI = (NI + NW - 1) / NW;
    static constexpr int AW = NI % NW;  // the apron wave (0 when every wave issues KI)
    __host__ __device__ static constexpr int loads(int w)
    {
        return NF * ((NI - w + NW - 1) / NW + (w == AW ? 1 : 0));
    }

    // byte offsets in the plane; a position outside the grid reads past the
    // plane (the buffer returns zeros).  Every load a wave counts in loads(w)
    // is issued whatever the grid holds: a skipped one would let the wait
    // count a younger plane's load as this plane's
    static constexpr uint32_t OUT = 0x80000000u;
    uint32_t off[KI], aoff;
    int w, lane;

    __device__ inline void init(const StagedGeo& g, int64_t a0, int64_t b0, int t)
    {
        const int64_t LA = (int64_t)g.la, LB = (int64_t)g.lb;
        w = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform: scalar branches on it
        lane = t & 63;
#pragma unroll
        for (int k = 0; k < KI; k++) {
            const int i = w + NW * k, e = 64 * i + lane;
            const int row = e >> 4, q = e & 15;
            const int64_t a = a0 + 4 * q, b = b0 - 1 + row;
            const bool ok = i < NI && e < NCHUNK && a < LA && b >= 0 && b < LB;
            off[k] = ok ? (uint32_t)((a + LA * b) * 4) : OUT;
        }
        aoff = OUT;
        if (w == AW && lane < 2 * WB) {
            const int row = lane >> 1;
            const int64_t a = (lane & 1) ? a0 + 64 : a0 - 1, b = b0 - 1 + row;
            if (a >= 0 && a < LA && b >= 0 && b < LB) aoff = (uint32_t)((a + LA * b) * 4);
        }
    }
    // plane image of storage slice sc into LDS buffer img (NF planes of PLANE)
    __device__ inline void issue(const Fields<T, NF>& fld, uint64_t S, int64_t sc, T* img) const
    {
#if defined(__HIP_DEVICE_COMPILE__)  // the LDS-DMA builtins exist for the device only
#pragma unroll
        for (int j = 0; j < NF; j++) {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<T*>(fld.p[j] + (uint64_t)sc * S), 0, (int)(S * sizeof(T)), 0x00020000);
            T* l = img + j * PLANE;
#pragma unroll
            for (int k = 0; k < KI; k++)
                if (w + NW * k < NI && 64 * (w + NW * k) + lane < NCHUNK)  // lane 0 always: the load is issued
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        rs, (__attribute__((address_space(3))) void*)(l + 256 * (w + NW * k)), 16, off[k], 0, 0, 0);
            if (w == AW && lane < 2 * WB)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(l + MAIN), 4,
                                                         aoff, 0, 0, 0);
        }
#endif
    }
    // the lane's 3 x (NB + 2) values of image img into W[.][pl]
    __device__ inline void window(const T* img, T (&W)[NF][3][NB + 2][3], int pl) const
    {
        const int il = lane == 0 ? MAIN : lane - 1, sl = lane == 0 ? 2 : 64;
        const int ir = lane == 63 ? MAIN + 1 : lane + 1, sr = lane == 63 ? 2 : 64;
#pragma unroll
        for (int j = 0; j < NF; j++) {
            const T* l = img + j * PLANE;
#pragma unroll
            for (int rr = 0; rr < NB + 2; rr++) {
                const int row = w * NB + rr;
                W[j][pl][rr][0] = l[il + sl * row];
                W[j][pl][rr][1] = l[64 * row + lane];
                W[j][pl][rr][2] = l[ir + sr * row];
            }
        }
    }
};

template <int N>
__device__ inline void vm_wait()
{
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

/* s_waitcnt vmcnt(loads(w)) for this wave (the immediate is per wave) */
template <class Tile, int W, int NW>
struct WaitOwn {
    __device__ static inline void run(int w)
    {
        if (w == W) {
            vm_wait<Tile::loads(W)>();
            return;
        }
        WaitOwn<Tile, W + 1, NW>::run(w);
    }
};
template <class Tile, int NW>
struct WaitOwn<Tile, NW, NW> {
    __device__ static inline void run(int)
    {
        vm_wait<0>();
    }
};

/* a column cell a = 0 / LA - 1 (A not periodic, B and C inside) of a
 * k_staged_g tile: the inner order with the neighbors past A's end dropped
 * (the edge walk's order there), the values from the three plane images in
 * LDS at the cell's row and column.  (The rows b = 0, LB - 1 taken the same
 * way, 64 lanes a row, measured 0.5 ms per 2048^3 step slower than leaving
 * them to the edge walk: the extra functor body cost the march its register
 * schedule, profiles/s53_staged_rows_ab.log.) */
template <class T, int NF, int SHAPE, int PLANE>
struct ImgEdgeCell {
    uint64_t slot, id;
    const T* img[3];  // planes c - 1, c, c + 1
    int64_t la, S;
    int32_t inv[3], scale;
    int row, col;
    bool lo_end, hi_end;  // a = 0 / a = LA - 1

    __host__ __device__ inline T value(int j) const { return img[1][j * PLANE + row * 64 + col]; }

    template <class G>
    __host__ __device__ inline void for_each_neighbor(G&& fn) const
    {
        typedef StagedItems<SHAPE> It;
#pragma unroll
        for (int k = 0; k < It::K; k++) {
            const int da = It::d(k, 0), db = It::d(k, 1), dc = It::d(k, 2);
            if ((da < 0 && lo_end) || (da > 0 && hi_end)) continue;
            ValueNeighbor<T, NF> nb;
            nb.slot = slot + (uint64_t)((int64_t)da + la * db + S * dc);
            nb.x = (inv[0] == 0 ? da : (inv[0] == 1 ? db : dc)) * scale;
            nb.y = (inv[1] == 0 ? da : (inv[1] == 1 ? db : dc)) * scale;
            nb.z = (inv[2] == 0 ? da : (inv[2] == 1 ? db : dc)) * scale;
#pragma unroll
            for (int j = 0; j < NF; j++) nb.v[j] = img[dc + 1][j * PLANE + (row + db) * 64 + col + da];
            fn(nb);
        }
    }
};

// MINWG: the waves per SIMD the build must allow (HIP's second launch bound).
// With 4 (at most 128 VGPRs) the game-of-life functor with the column cells
// fits with no spill (130 VGPRs unbounded, 3 waves); a functor that would
// spill under the bound runs the unbounded build (launch_staged asks the
// runtime for the bounded build's scratch once)
#ifndef DCCRGX_STAGED_G_MINWG
#define DCCRGX_STAGED_G_MINWG 4
#endif
template <class T, int NF, int SHAPE, int NW, int NB, int MINWG, class F>
__global__ void __launch_bounds__(64 * NW, MINWG) k_staged_g(StagedGeo g, Fields<T, NF> fld, F f)
{
    typedef StagedTileG<T, NF, NW, NB> Tile;
    // planes q - 2 .. q read at step q (the column cells read all three),
    // q + 1 and q + 2 in flight
    constexpr int NBUF = 5;
    __shared__ __attribute__((aligned(16))) T P[NBUF * NF * Tile::PLANE];

    const int t = threadIdx.x;
    const uint32_t wgid = xcd_wgid(g.nwg);
    const uint32_t tiles = g.tiles_a * g.tiles_b;
    const uint32_t tile_id = wgid % tiles;
    const int64_t chunk_id = wgid / tiles;
    const int64_t a0 = (int64_t)(tile_id % g.tiles_a) * 64;
    const int64_t b0 = (int64_t)(tile_id / g.tiles_a) * Tile::TB;
    const int64_t c0 = g.s0 + chunk_id * g.chunk;
    const int64_t c1 = min(g.s1, c0 + g.chunk);
    if (c0 >= c1) return;

    Tile tile;
    tile.init(g, a0, b0, t);
    T W[NF][3][NB + 2][3];
    // plane q = storage slice c0 - 1 + q, q in [0, Q), in buffer q % NBUF;
    // computed: q in [2, Q) -> slice c0 + q - 2
    const int64_t Q = c1 - c0 + 2;
    tile.issue(fld, g.S, c0 - 1, P);
    tile.issue(fld, g.S, c0, P + NF * Tile::PLANE);
    const int64_t a = a0 + tile.lane, bw = b0 + tile.w * NB;
    // the column cells: lanes [0, NB) take a = 0 in the first tile, lanes
    // [NB, 2 NB) a = LA - 1 in the last (rows bw ..; wave-uniform test first)
    const int64_t LA = (int64_t)g.la, LB = (int64_t)g.lb;
    const bool col_tile = g.cols_in && (a0 == 0 || a0 + 64 >= LA);  // uniform
    for (int64_t q = 0; q < Q; q++) {
        // this wave's loads of plane q are done (those of q + 1 may fly)
        if (q + 1 < Q) WaitOwn<Tile, 0, NW>::run(tile.w);
        else vm_wait<0>();
        asm volatile("s_barrier" ::: "memory");
        if (q >= 2) {
            // the column cells first, from the images: plane q's window
            // registers are not live yet
            const int64_t c = c0 + q - 2;
            // (the lane's column cell recomputed here: fewer registers live
            // across the march)
            const int cside = tile.lane < NB ? 0 : (tile.lane < 2 * NB ? 1 : -1);
            const int64_t ca = cside == 0 ? 0 : LA - 1, cb = bw + tile.lane - (cside == 1 ? NB : 0);
            if (col_tile && cside >= 0 && (cside == 0 ? a0 == 0 : a0 + 64 >= LA) && cb >= 1 && cb + 1 < LB) {
                const int64_t cg = c + g.cbase;
                const uint64_t lin = (uint64_t)ca + g.la * (uint64_t)cb + g.S * (uint64_t)cg;
                if (lin >= g.lo && lin < g.hi) {
                    ImgEdgeCell<T, NF, SHAPE, Tile::PLANE> cell;
                    cell.slot = (uint64_t)ca + g.la * (uint64_t)cb + g.S * (uint64_t)c;
                    cell.id = lin + 1;
                    cell.la = (int64_t)g.la;
                    cell.S = (int64_t)g.S;
                    cell.lo_end = ca == 0;
                    cell.hi_end = ca == LA - 1;
                    cell.inv[0] = g.inv[0];
                    cell.inv[1] = g.inv[1];
                    cell.inv[2] = g.inv[2];
                    cell.scale = g.scale;
#pragma unroll
                    for (int d = 0; d < 3; d++) cell.img[d] = P + (int)((q - 2 + d) % NBUF) * NF * Tile::PLANE;
                    cell.row = (int)(cb - b0) + 1;
                    cell.col = (int)(ca - a0);
                    f(cell);
                }
            }
        }
        const T* img = P + (int)(q % NBUF) * NF * Tile::PLANE;
        tile.window(img, W, 2);
        if (q >= 2) {
            const int64_t c = c0 + q - 2;
            const int64_t pls[3] = {c - 1, c, c + 1};
            staged_cells<T, NF, SHAPE, NB, CLS_MID>(g, f, W, pls, c, a, bw);
        }
#pragma unroll
        for (int jj = 0; jj < NF; jj++)
#pragma unroll
            for (int rr = 0; rr < NB + 2; rr++)
#pragma unroll
                for (int qq = 0; qq < 3; qq++) {
                    W[jj][0][rr][qq] = W[jj][1][rr][qq];
                    W[jj][1][rr][qq] = W[jj][2][rr][qq];
                }
        // plane q + 2 into the buffer no wave reads after step q
        if (q + 2 < Q) tile.issue(fld, g.S, c0 + 1 + q, P + (int)((q + 2) % NBUF) * NF * Tile::PLANE);
    }
}

/* The first (CLS_LOW) or last (CLS_HIGH) slice of a periodic C axis, storage
 * slice g.s0: the plane across the wrap is read from storage slice
 * g.wrap_lo / g.wrap_hi (the local slice itself when this rank holds it, as
 * the walk reads it; else the ghost copy), one tile per workgroup. */
template <class T, int NF, int SHAPE, int NW, int NB, int VEC, int CLS, class F>
__global__ void __launch_bounds__(64 * NW) k_staged_wrap(StagedGeo g, Fields<T, NF> fld, F f)
{
    typedef StagedTile<T, NF, NW, NB, VEC> Tile;
    typedef typename Tile::Chunk Chunk;
    __shared__ __attribute__((aligned(16))) T P[3][NF][Tile::WB][Tile::RS];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t tile_id = blockIdx.x;
    const int64_t a0 = (int64_t)(tile_id % g.tiles_a) * 64;
    const int64_t b0 = (int64_t)(tile_id / g.tiles_a) * Tile::TB;
    const int64_t c = g.s0;
    const int64_t ps[3] = {CLS == CLS_LOW ? g.wrap_lo : c - 1, c, CLS == CLS_HIGH ? g.wrap_hi : c + 1};
    Tile tile;
    tile.init(g, a0, b0, t);
    Chunk FM[NF][Tile::NCH];
    T FE[NF];
#pragma unroll
    for (int pl = 0; pl < 3; pl++) {
        tile.fetch(fld, g.S, ps[pl], FM, FE);
        tile.stash(&P[pl][0][0][0], FM, FE);
    }
    __syncthreads();
    T W[NF][3][NB + 2][3];
#pragma unroll
    for (int pl = 0; pl < 3; pl++) Tile::window(&P[pl][0][0][0], w, lane, W, pl);
    staged_cells<T, NF, SHAPE, NB, CLS>(g, f, W, ps, c, a0 + lane, b0 + w * NB);
}

/* The edge walk over storage slices [s0, s1): with whole == 0 the ring of
 * each slice (rows b = 0 and LB - 1 whole, the other rows' cells a = 0 and
 * LA - 1), 1 every cell of the slices, 2 the rows b = 0 and LB - 1 only (the
 * columns go to k_staged_cols); one thread per cell. */
template <class T, int NF, int SHAPE, class F>
__global__ void __launch_bounds__(256) k_staged_edge(StagedGeo g, Fields<T, NF> fld, int64_t s0, int64_t s1,
                                                      int32_t whole, F f)
{
    const uint64_t per = whole == 1 ? g.S : whole == 2 ? 2 * g.la : 2 * g.la + 2 * (g.lb - 2);
    const uint64_t n = per * (uint64_t)(s1 - s0);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t si = i / per, j = i - si * per;
        uint64_t a, b;
        if (whole == 1) {
            b = j / g.la;
            a = j - b * g.la;
        } else if (j < 2 * g.la) {
            b = j < g.la ? 0 : g.lb - 1;
            a = j < g.la ? j : j - g.la;
        } else {
            // column a = 0, then a = LA - 1: consecutive lanes on consecutive
            // rows share their neighbors' lines
            const uint64_t k = j - 2 * g.la, h = g.lb - 2;
            b = 1 + (k < h ? k : k - h);
            a = k < h ? 0 : g.la - 1;
        }
        const int64_t s = s0 + (int64_t)si, c = s + g.cbase;
        const uint64_t lin = a + g.la * b + g.S * (uint64_t)c;
        if (lin < g.lo || lin >= g.hi) continue;
        EdgeCell<T, NF, SHAPE> cell;
        cell.slot = a + g.la * b + g.S * (uint64_t)s;
        cell.id = lin + 1;
        cell.fld = fld;
        cell.la = g.la;
        cell.lb = g.lb;
        cell.lc = g.lc;
        cell.S = g.S;
        cell.lo = g.lo;
        cell.hi = g.hi;
        cell.a = (int64_t)a;
        cell.b = (int64_t)b;
        cell.c = c;
        cell.cbase = g.cbase;
        cell.pa = g.pa;
        cell.pb = g.pb;
        cell.pc = g.pc;
        cell.inv[0] = g.inv[0];
        cell.inv[1] = g.inv[1];
        cell.inv[2] = g.inv[2];
        cell.scale = g.scale;
        f(cell);
    }
}

/* The edge columns a = 0 and a = LA - 1 (rows 1 .. LB - 2) of slices [s0,
 * s1): a workgroup stages a column's 64 rows x 4 slices with their apron (the
 * three columns a - 1 .. a + 1, periodic wrap included) in LDS with one load
 * per value, then each thread walks one cell as the edge walk does, its
 * neighbors' values from LDS.  (One thread per cell straight from memory put
 * 64 rows' lines behind every load of a wave: ~50x the cells' bytes fetched.)
 * Positions no processed cell reads, or outside the grid or the storage,
 * stage 0. */
constexpr int COL_B = 64, COL_C = 4;

template <class T, int NF, int SHAPE>
struct ColCell : EdgeCell<T, NF, SHAPE> {
    const T* lds;  // [NF][COL_C + 2][COL_B + 2][3]
    int tb, tc;
    template <class G>
    __device__ inline void for_each_neighbor(G&& fn) const
    {
        this->walk(fn, [&](int j, uint64_t, int da, int db, int dc) {
            return lds[((j * (COL_C + 2) + (tc + 1 + dc)) * (COL_B + 2) + (tb + 1 + db)) * 3 + (da + 1)];
        });
    }
};

template <class T, int NF, int SHAPE, class F>
__global__ void __launch_bounds__(COL_B* COL_C) k_staged_cols(StagedGeo g, Fields<T, NF> fld, int64_t s0, int64_t s1,
                                                              F f)
{
    __shared__ T V[NF][COL_C + 2][COL_B + 2][3];
    const uint64_t nbch = (g.lb - 2 + COL_B - 1) / COL_B;
    const uint64_t ncch = (uint64_t)(s1 - s0 + COL_C - 1) / COL_C;
    const uint64_t nblk = 2 * nbch * ncch;
    const int tb = threadIdx.x % COL_B, tc = threadIdx.x / COL_B;
    for (uint64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {  // uniform per workgroup
        const int side = (int)(blk & 1);
        const uint64_t rest = blk >> 1, bch = rest % nbch, cch = rest / nbch;
        const int64_t a = side ? (int64_t)g.la - 1 : 0, b0 = 1 + (int64_t)(bch * COL_B);
        const int64_t sc0 = s0 + (int64_t)(cch * COL_C);
        for (int idx = threadIdx.x; idx < (COL_C + 2) * (COL_B + 2) * 3; idx += COL_B * COL_C) {
            const int ja = idx % 3, t = idx / 3, jb = t % (COL_B + 2), jc = t / (COL_B + 2);
            int64_t a2 = a + ja - 1, b2 = b0 - 1 + jb;
            const int64_t cu = sc0 - 1 + jc + g.cbase;
            bool ok = b2 < (int64_t)g.lb;  // b2 >= 0 always
            if (a2 < 0 || a2 >= (int64_t)g.la) {
                ok = ok && g.pa;
                a2 = a2 < 0 ? a2 + (int64_t)g.la : a2 - (int64_t)g.la;
            }
            int64_t cw = cu;
            if (cu < 0 || cu >= (int64_t)g.lc) {
                ok = ok && g.pc;
                cw = cu < 0 ? cu + (int64_t)g.lc : cu - (int64_t)g.lc;
            }
            // the slot the edge walk reads: a local neighbor from its own slot,
            // a remote one from its ghost slot
            const uint64_t ab = (uint64_t)a2 + g.la * (uint64_t)b2, nlin = ab + g.S * (uint64_t)cw;
            const int64_t ss = ((nlin >= g.lo && nlin < g.hi) ? cw : cu) - g.cbase;
            ok = ok && ss >= 0 && ss < g.nslices;
            const uint64_t slot = ab + g.S * (uint64_t)(ok ? ss : 0);
#pragma unroll
            for (int j = 0; j < NF; j++) V[j][jc][jb][ja] = ok ? fld.p[j][slot] : T(0);
        }
        __syncthreads();
        const int64_t b = b0 + tb, sl = sc0 + tc, c = sl + g.cbase;
        const uint64_t lin = (uint64_t)a + g.la * (uint64_t)b + g.S * (uint64_t)c;
        if (b <= (int64_t)g.lb - 2 && sl < s1 && lin >= g.lo && lin < g.hi) {
            ColCell<T, NF, SHAPE> cell;
            cell.slot = (uint64_t)a + g.la * (uint64_t)b + g.S * (uint64_t)sl;
            cell.id = lin + 1;
            cell.fld = fld;
            cell.la = g.la;
            cell.lb = g.lb;
            cell.lc = g.lc;
            cell.S = g.S;
            cell.lo = g.lo;
            cell.hi = g.hi;
            cell.a = a;
            cell.b = b;
            cell.c = c;
            cell.cbase = g.cbase;
            cell.pa = g.pa;
            cell.pb = g.pb;
            cell.pc = g.pc;
            cell.inv[0] = g.inv[0];
            cell.inv[1] = g.inv[1];
            cell.inv[2] = g.inv[2];
            cell.scale = g.scale;
            cell.lds = &V[0][0][0][0];
            cell.tb = tb;
            cell.tc = tc;
            f(cell);
        }
        __syncthreads();
    }
}

/* The edge rows b = 0 and LB - 1 of storage slices [s0, s1) whose canonical c
 * is inside (A and B not periodic): a wave owns 64 cells of one row and
 * marches along C through `chunk` slices; each plane's edge row and the
 * inner row next to it are read once (a - 1, a, a + 1: three coalesced
 * loads each) into a register window of three planes.  A cell's neighbors
 * come in the inner order with those past the grid's ends dropped, as the
 * edge walk gives them (ROW 0: b = 0, ROW 1: b = LB - 1).  (The edge walk,
 * one thread per cell and every neighbor loaded at its slot: 0.52 ms per
 * 2048^3 step.) */
template <class T, int NF, int SHAPE, int ROW>
struct RowCell {
    uint64_t slot, id;
    const T (*w)[3][2][3];  // [field][plane c - 1 .. c + 1][row: inner-order][a - 1 .. a + 1]
    int64_t la, S;
    int32_t inv[3], scale;
    bool a_lo, a_hi;

    __host__ __device__ inline T value(int j) const { return w[j][1][ROW == 0 ? 0 : 1][1]; }

    template <class G>
    __host__ __device__ inline void for_each_neighbor(G&& fn) const
    {
        typedef StagedItems<SHAPE> It;
#pragma unroll
        for (int k = 0; k < It::K; k++) {
            const int da = It::d(k, 0), db = It::d(k, 1), dc = It::d(k, 2);
            if ((ROW == 0 && db < 0) || (ROW == 1 && db > 0)) continue;
            if ((da < 0 && a_lo) || (da > 0 && a_hi)) continue;
            ValueNeighbor<T, NF> nb;
            nb.slot = slot + (uint64_t)((int64_t)da + la * db + S * dc);
            nb.x = (inv[0] == 0 ? da : (inv[0] == 1 ? db : dc)) * scale;
            nb.y = (inv[1] == 0 ? da : (inv[1] == 1 ? db : dc)) * scale;
            nb.z = (inv[2] == 0 ? da : (inv[2] == 1 ? db : dc)) * scale;
#pragma unroll
            for (int j = 0; j < NF; j++) nb.v[j] = w[j][dc + 1][ROW == 0 ? db : db + 1][da + 1];
            fn(nb);
        }
    }
};

template <class T, int NF, int SHAPE, int ROW, class F>
__device__ inline void staged_row_march(const StagedGeo& g, const Fields<T, NF>& fld, int64_t cs, int64_t ce,
                                        int64_t a, F& f)
{
    const int64_t LA = (int64_t)g.la, LB = (int64_t)g.lb;
    const int64_t r0 = ROW == 0 ? 0 : LB - 2;  // window rows r0, r0 + 1
    const int64_t b = ROW == 0 ? 0 : LB - 1;
    T W[NF][3][2][3];
    auto load = [&](int64_t sl, int pl) {
#pragma unroll
        for (int j = 0; j < NF; j++) {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<T*>(fld.p[j] + (uint64_t)sl * g.S), 0, (int)(g.S * sizeof(T)), 0x00020000);
#pragma unroll
            for (int r = 0; r < 2; r++)
#pragma unroll
                for (int q = 0; q < 3; q++) {
                    // a - 1 < 0 / a + 1 = LA read past the row (a neighbor
                    // dropped anyway): the plane's bounds give 0 outside it
                    const int64_t e = a + q - 1 + LA * (r0 + r);
                    W[j][pl][r][q] = buffer_load<T>(rs, e < 0 ? 0x80000000u : (uint32_t)(e * (int64_t)sizeof(T)));
                }
        }
    };
    load(cs - 1, 0);
    load(cs, 1);
    RowCell<T, NF, SHAPE, ROW> cell;
    cell.w = W;
    cell.la = LA;
    cell.S = (int64_t)g.S;
    cell.inv[0] = g.inv[0];
    cell.inv[1] = g.inv[1];
    cell.inv[2] = g.inv[2];
    cell.scale = g.scale;
    cell.a_lo = a == 0;
    cell.a_hi = a == LA - 1;
    for (int64_t sl = cs; sl < ce; sl++) {
        load(sl + 1, 2);
        const uint64_t lin = (uint64_t)a + g.la * (uint64_t)b + g.S * (uint64_t)(sl + g.cbase);
        if (a < LA && lin >= g.lo && lin < g.hi) {
            cell.slot = (uint64_t)a + g.la * (uint64_t)b + g.S * (uint64_t)sl;
            cell.id = lin + 1;
            f(cell);
        }
#pragma unroll
        for (int j = 0; j < NF; j++)
#pragma unroll
            for (int r = 0; r < 2; r++)
#pragma unroll
                for (int q = 0; q < 3; q++) {
                    W[j][0][r][q] = W[j][1][r][q];
                    W[j][1][r][q] = W[j][2][r][q];
                }
    }
}

template <class T, int NF, int SHAPE, class F>
__global__ void __launch_bounds__(256) k_staged_rows(StagedGeo g, Fields<T, NF> fld, int64_t s0, int64_t s1,
                                                      int64_t chunk, F f)
{
    const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const uint64_t ta = (g.la + 63) / 64, per = 2 * ta;
    const uint64_t cid = wave / per, rem = wave - cid * per, side = rem / ta, at = rem - side * ta;
    const int64_t cs = s0 + (int64_t)cid * chunk, ce = min(s1, cs + chunk);
    if (cs >= ce) return;  // wave-uniform
    const int64_t a = (int64_t)(at * 64) + (threadIdx.x & 63);
    if (side == 0) staged_row_march<T, NF, SHAPE, 0>(g, fld, cs, ce, a, f);
    else staged_row_march<T, NF, SHAPE, 1>(g, fld, cs, ce, a, f);
}

template <class T, int NF>
struct StagedShape {
    // the register window holds 9 (NB + 2) elements per field: NB rows per
    // lane for 4-byte data, fewer (and more waves) for more bytes
    static constexpr int units = (int)((NF * sizeof(T) + 3) / 4);
#ifndef DCCRGX_STAGED_NB1
#define DCCRGX_STAGED_NB1 4
#endif
    static constexpr int NB = units <= 1 ? DCCRGX_STAGED_NB1 : (units == 2 ? 2 : 1);
    static constexpr int NW = units <= 1 ? 4 : 8;
    static constexpr int TB = NW * NB;
    static constexpr int VEC = (int)(16 / sizeof(T));
    static constexpr int PF = 1;  // planes in flight (deeper costs occupancy: tools/us_sweep.hip; k_staged_g keeps two)
};

inline StagedGeo staged_geo(const dccrgx_stencil_view& v, int TB)
{
    StagedGeo g;
    g.la = v.la;
    g.lb = v.lb;
    g.lc = v.lc;
    g.S = v.la * v.lb;
    g.lo = v.lo;
    g.hi = v.hi;
    g.cbase = v.cbase;
    g.s0 = g.s1 = g.chunk = g.wrap_lo = g.wrap_hi = 0;
    g.pa = v.per[0];
    g.pb = v.per[1];
    g.pc = v.per[2];
    for (int d = 0; d < 3; d++) g.inv[v.perm[d]] = d;
    g.scale = v.scale;
    g.nslices = v.nslices;
    g.tiles_a = (uint32_t)((v.la + 63) / 64);
    g.tiles_b = (uint32_t)((v.lb + TB - 1) / TB);
    g.nwg = 0;
    g.cols_in = 0;
    return g;
}

#ifndef DCCRGX_STAGED_GLDS
#define DCCRGX_STAGED_GLDS 1  // 0: the register-staged k_staged for every element size
#endif
#ifndef DCCRGX_STAGED_COLS
#define DCCRGX_STAGED_COLS 1  // 0: k_staged_g leaves the edge columns to k_staged_cols
#endif
/* *cols_done: the launch took the edge columns a = 0, LA - 1 too */
template <class T, int NF, int SHAPE, class F>
int launch_staged(const dccrgx_stencil_view& v, Fields<T, NF> fld, int64_t s0, int64_t s1, F f, hipStream_t st,
                  int64_t want, bool* cols_done)
{
    *cols_done = false;
    typedef StagedShape<T, NF> Sh;
    StagedGeo g = staged_geo(v, Sh::TB);
    g.s0 = s0;
    g.s1 = s1;
    const int64_t tiles = (int64_t)g.tiles_a * g.tiles_b, nsl = s1 - s0;
    int64_t chunks = (want + tiles - 1) / tiles;
    chunks = chunks < 1 ? 1 : (chunks > nsl ? nsl : chunks);
    g.chunk = (nsl + chunks - 1) / chunks;
    const int64_t nwg = tiles * ((nsl + g.chunk - 1) / g.chunk);
    if (nwg >= (1ll << 31)) return DCCRGX_EINVAL;
    g.nwg = (uint32_t)nwg;
    if constexpr (sizeof(T) == 4 && DCCRGX_STAGED_GLDS) {
        if (v.la % 4 == 0 && g.S * 4 < (1ull << 31)) {
            g.cols_in = DCCRGX_STAGED_COLS && !v.per[0];
            *cols_done = g.cols_in != 0;
            // the bounded build unless it spills (scratch), asked once per
            // instantiation
            static const bool bounded = [] {
                hipFuncAttributes at{};
                return hipFuncGetAttributes(
                           &at, reinterpret_cast<const void*>(
                                    &k_staged_g<T, NF, SHAPE, Sh::NW, Sh::NB, DCCRGX_STAGED_G_MINWG, F>)) ==
                           hipSuccess &&
                       at.localSizeBytes == 0;
            }();
            if (bounded)
                hipLaunchKernelGGL((k_staged_g<T, NF, SHAPE, Sh::NW, Sh::NB, DCCRGX_STAGED_G_MINWG, F>), dim3(g.nwg),
                                   dim3(64 * Sh::NW), 0, st, g, fld, f);
            else
                hipLaunchKernelGGL((k_staged_g<T, NF, SHAPE, Sh::NW, Sh::NB, 1, F>), dim3(g.nwg), dim3(64 * Sh::NW), 0,
                                   st, g, fld, f);
            return DCCRGX_OK;
        }
    }
    if (v.la % Sh::VEC == 0)
        hipLaunchKernelGGL((k_staged<T, NF, SHAPE, Sh::NW, Sh::NB, Sh::VEC, Sh::PF, F>), dim3(g.nwg),
                           dim3(64 * Sh::NW), 0, st, g, fld, f);
    else
        hipLaunchKernelGGL((k_staged<T, NF, SHAPE, Sh::NW, Sh::NB, 1, Sh::PF, F>), dim3(g.nwg), dim3(64 * Sh::NW),
                           0, st, g, fld, f);
    return DCCRGX_OK;
}

/* the wrap slice s (canonical 0: CLS_LOW, LC - 1: CLS_HIGH), the plane across
 * the wrap read from storage slice `across` */
template <class T, int NF, int SHAPE, int CLS, class F>
int launch_staged_wrap(const dccrgx_stencil_view& v, Fields<T, NF> fld, int64_t s, int64_t across, F f,
                       hipStream_t st)
{
    typedef StagedShape<T, NF> Sh;
    StagedGeo g = staged_geo(v, Sh::TB);
    g.s0 = s;
    g.s1 = s + 1;
    g.wrap_lo = g.wrap_hi = across;
    const int64_t tiles = (int64_t)g.tiles_a * g.tiles_b;
    if (tiles >= (1ll << 31)) return DCCRGX_EINVAL;
    if (v.la % Sh::VEC == 0)
        hipLaunchKernelGGL((k_staged_wrap<T, NF, SHAPE, Sh::NW, Sh::NB, Sh::VEC, CLS, F>), dim3((unsigned)tiles),
                           dim3(64 * Sh::NW), 0, st, g, fld, f);
    else
        hipLaunchKernelGGL((k_staged_wrap<T, NF, SHAPE, Sh::NW, Sh::NB, 1, CLS, F>), dim3((unsigned)tiles),
                           dim3(64 * Sh::NW), 0, st, g, fld, f);
    return DCCRGX_OK;
}

#ifndef DCCRGX_STAGED_ROWS
#define DCCRGX_STAGED_ROWS 1  // 0: the edge rows of inner slices by the edge walk too
#endif
/* inner: [s0, s1) are slices whose canonical c is inside (planes c - 1 .. c +
 * 1 are storage slices s - 1 .. s + 1) */
template <class T, int NF, int SHAPE, class F>
int launch_edge(const dccrgx_stencil_view& v, Fields<T, NF> fld, int64_t s0, int64_t s1, bool whole, F f,
                hipStream_t st, bool cols_done = false, bool inner = false)
{
    if (s1 <= s0) return DCCRGX_OK;
    const StagedGeo g = staged_geo(v, 1);
    // the ring: rows b = 0 and LB - 1 by the row march (inner slices, A and B
    // not periodic) or the edge walk, the columns staged (k_staged_cols) when
    // their values fit LDS, or none when the staged kernel took them
    const bool fits = v.lb >= 3 && sizeof(T) * NF * (COL_C + 2) * (COL_B + 2) * 3 <= 48 * 1024;
    // (columns that fit no LDS go with the rows in the ring walk)
    const bool rows_march = DCCRGX_STAGED_ROWS && !whole && inner && !v.per[0] && !v.per[1] && (cols_done || fits);
    if (rows_march) {
        const uint64_t ta = (v.la + 63) / 64, nsl = (uint64_t)(s1 - s0);
        uint64_t chunks = 16384 / (2 * ta);
        chunks = chunks < 1 ? 1 : (chunks > nsl ? nsl : chunks);
        const int64_t chunk = (int64_t)((nsl + chunks - 1) / chunks);
        const uint64_t waves = 2 * ta * ((nsl + chunk - 1) / chunk);
        hipLaunchKernelGGL((k_staged_rows<T, NF, SHAPE, F>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, g, fld,
                           s0, s1, chunk, f);
    }
    const bool cols = !whole && !cols_done && fits;
    const int32_t mode = whole ? 1 : (rows_march ? -1 : (cols || cols_done) ? 2 : 0);  // -1: no walk
    const uint64_t per = mode == 1 ? v.la * v.lb : mode == 2 ? 2 * v.la : 2 * v.la + 2 * (v.lb - 2);
    const uint64_t n = per * (uint64_t)(s1 - s0);
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks && mode >= 0)
        hipLaunchKernelGGL((k_staged_edge<T, NF, SHAPE, F>), dim3((unsigned)blocks), dim3(256), 0, st, g, fld, s0, s1,
                           mode, f);
    if (cols) {
        const uint64_t nblk = 2 * ((v.lb - 2 + COL_B - 1) / COL_B) * (((uint64_t)(s1 - s0) + COL_C - 1) / COL_C);
        const uint64_t wg = nblk < 65536 ? nblk : 65536;
        if (wg)
            hipLaunchKernelGGL((k_staged_cols<T, NF, SHAPE, F>), dim3((unsigned)wg), dim3(COL_B * COL_C), 0, st, g,
                               fld, s0, s1, f);
    }
    return DCCRGX_OK;
}

/* the staged launches of one slice range [s0, s1) of a region: the staged
 * kernel for the slices whose canonical c is in [1, LC - 1); the first and
 * last slice of a periodic C by the wrap kernel when the slice across the
 * wrap is held whole or not at all by this rank, else (and for a
 * non-periodic C) by the edge walk; the ring of every other slice by the
 * edge walk */
template <class T, int NF, int SHAPE, class F>
int staged_range(const dccrgx_stencil_view& v, Fields<T, NF> fld, int64_t s0, int64_t s1, F f, hipStream_t st,
                 int64_t want, hipStream_t se)
{
    // st: the staged kernel; se: the edge walks and wrap slices (cells
    // disjoint from the staged kernel's, run beside it when se != st)
    const int64_t lc = (int64_t)v.lc, cb = v.cbase;
    const int64_t m0 = s0 > 1 - cb ? s0 : 1 - cb;
    const int64_t m1 = s1 < lc - 1 - cb ? s1 : lc - 1 - cb;
    int e = DCCRGX_OK;
    if (m1 > m0) {
        bool cols_done = false;
        e = launch_staged<T, NF, SHAPE>(v, fld, m0, m1, f, st, want, &cols_done);
        if (e == DCCRGX_OK) e = launch_edge<T, NF, SHAPE>(v, fld, m0, m1, false, f, se, cols_done, true);
        if (e != DCCRGX_OK) return e;
    }
    for (int side = 0; side < 2; side++) {
        const int64_t s = side == 0 ? -cb : lc - 1 - cb;
        if (s < s0 || s >= s1 || (side == 1 && lc == 1)) continue;
        const uint64_t oc = side == 0 ? (uint64_t)(lc - 1) : 0;  // canonical slice across the wrap
        const uint64_t o0 = oc * v.la * v.lb, o1 = o0 + v.la * v.lb;
        const bool whole = o0 >= v.lo && o1 <= v.hi, none = o1 <= v.lo || o0 >= v.hi;
        if (v.per[2] && lc >= 3 && (whole || none)) {
            const int64_t across = whole ? (int64_t)oc - cb : (side == 0 ? s - 1 : s + 1);
            e = side == 0 ? launch_staged_wrap<T, NF, SHAPE, CLS_LOW>(v, fld, s, across, f, se)
                          : launch_staged_wrap<T, NF, SHAPE, CLS_HIGH>(v, fld, s, across, f, se);
            if (e == DCCRGX_OK) e = launch_edge<T, NF, SHAPE>(v, fld, s, s + 1, false, f, se);
        } else {
            e = launch_edge<T, NF, SHAPE>(v, fld, s, s + 1, true, f, se);
        }
        if (e != DCCRGX_OK) return e;
    }
    return DCCRGX_OK;
}

/* a second stream per device for the edge launches of a staged launch (they
 * run beside the staged kernel: edge walks are latency-bound on few waves),
 * with the events that fork it from and join it to the caller's stream;
 * made on first use, kept for the process */
struct SideStream {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    bool ok = false;
};

inline SideStream* side_stream()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    static SideStream ss[64];
    static std::mutex m;
    std::lock_guard<std::mutex> lk(m);
    SideStream& x = ss[dev];
    if (!x.ok) {
        if (hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
        if (hipEventCreateWithFlags(&x.fork, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&x.join, hipEventDisableTiming) != hipSuccess)
            return nullptr;
        x.ok = true;
    }
    return &x;
}

}  // namespace detail

/* options of the staged launches */
struct StagedOptions {
    // target workgroups of the staged kernel (tiles x slice chunks): 2^18 was
    // 0.4-1.0 ms faster than 2^17 and 2^19 on 2048^3 in two sweeps
    // (profiles/s32_us_sweep.log, s34_us_sweep.log)
    int64_t workgroups = 262144;
    bool staged = true;          // false: every cell through the walk (for comparisons)
    bool side_stream = true;     // edge launches on a second stream beside the staged kernel
};

/* Launch f(cell) for every cell of the region described by v, the declared
 * fields' values staged (see above).  Returns a DCCRGX_* code. */
template <class T, int NF, class F>
int for_each_cell_staged(const dccrgx_stencil_view& v, Fields<T, NF> fld, F f, hipStream_t st,
                         const StagedOptions& opt = StagedOptions())
{
    static_assert(sizeof(T) == 1 || sizeof(T) == 2 || sizeof(T) == 4 || sizeof(T) == 8, "element of 1-8 bytes");
    static_assert(NF >= 1 && NF <= 8, "1 to 8 staged fields");
    if (v.n_cells == 0) return DCCRGX_OK;
    auto walk = [=] __device__(const auto& cell) {
        LoadedCell<typename std::decay<decltype(cell)>::type, T, NF> lc{cell, fld, cell.slot, cell.id};
        f(lc);
    };
    if (v.kind != 0) return for_each_cell(v, walk, st);
    const detail::UniformGeo g = detail::uniform_geo(v);
    const int shape = v.shape & (DCCRGX_SHAPE_CUBE1 | DCCRGX_SHAPE_FACES);
    // staged: the cube / the faces on axes of >= 3 cells (periodic axes of 1
    // or 2 cells repeat neighbors across the wrap; shorter non-periodic ones
    // leave no inner cells), planes of < 2^31 bytes
    const bool fast = opt.staged && shape != 0 && v.la >= 3 && v.lb >= 3 && v.lc >= 3 &&
                      v.la * v.lb * sizeof(T) < (1ull << 31);
    // the edge launches fork onto a second stream and join back, so the
    // caller's stream orders everything as one launch would
    detail::SideStream* side = fast && opt.side_stream ? detail::side_stream() : nullptr;
    std::unique_lock<std::mutex> side_lock;
    if (side) {
        static std::mutex side_m;  // one staged launch at a time uses the side stream's events
        side_lock = std::unique_lock<std::mutex>(side_m);
        if (hipEventRecord(side->fork, st) != hipSuccess || hipStreamWaitEvent(side->s, side->fork, 0) != hipSuccess)
            return DCCRGX_EHIP;
    }
    hipStream_t se = side ? side->s : st;
    int err = DCCRGX_OK;
    for (int r = 0; r < 2 && err == DCCRGX_OK; r++) {
        const int64_t s0 = v.s0[r], s1 = v.s1[r];
        if (s1 <= s0) continue;
        if (!fast)
            err = detail::launch_slices(g, s0, s1, walk, st);
        else if (shape == DCCRGX_SHAPE_CUBE1)
            err = detail::staged_range<T, NF, DCCRGX_SHAPE_CUBE1>(v, fld, s0, s1, f, st, opt.workgroups, se);
        else
            err = detail::staged_range<T, NF, DCCRGX_SHAPE_FACES>(v, fld, s0, s1, f, st, opt.workgroups, se);
    }
    if (side) {  // joined also after a failed launch: the caller's stream never runs ahead of the side stream
        if (hipEventRecord(side->join, side->s) != hipSuccess || hipStreamWaitEvent(st, side->join, 0) != hipSuccess)
            return DCCRGX_EHIP;
    }
    if (err != DCCRGX_OK) return err;
    return hipGetLastError() == hipSuccess ? DCCRGX_OK : DCCRGX_EHIP;
}

/* the same for neighborhood hood_id and region of a grid */
template <class T, int NF, class F>
int for_each_cell_staged(const dccrgx_grid* grid, int32_t hood_id, int32_t region, Fields<T, NF> fld, F f,
                         hipStream_t st = nullptr, const StagedOptions& opt = StagedOptions())
{
    dccrgx_stencil_view v;
    const int e = dccrgx_stencil_view_get(grid, hood_id, region, &v);
    if (e != DCCRGX_OK) return e;
    return for_each_cell_staged(v, fld, f, st ? st : (hipStream_t)v.stream, opt);
}

}  // namespace dccrgx_user
