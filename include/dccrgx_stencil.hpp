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
        // no periodic wrap within twice the reach: the items' order is still
        // the iteration order (ids grow with (c, b, a); an entry is a
        // neighbor_to exactly when the mirrored item exists), items past a
        // non-periodic boundary are dropped
        const bool nowrap = (!g.pa || (a >= 2 * g.ra && a + 2 * g.ra < (int64_t)g.la)) &&
                            (!g.pb || (b >= 2 * g.rb && b + 2 * g.rb < (int64_t)g.lb)) &&
                            (!g.pc || (c >= 2 * g.rc && c + 2 * g.rc < (int64_t)g.lc));
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
        for (uint64_t e = row[q]; e < e1; e++) {
            Neighbor nb;
            nb.slot = nbr_slot[e];
            nb.x = nbr_off[3 * e];
            nb.y = nbr_off[3 * e + 1];
            nb.z = nbr_off[3 * e + 2];
            fn(nb);
        }
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

}  // namespace detail

/* Launch f(cell) for every cell of the region described by v on stream st
 * (asynchronous).  f is a device functor taking `const auto&` (UniformCell on
 * uniform grids, ExplicitCell otherwise).  Returns a DCCRGX_* code. */
template <class F>
int for_each_cell(const dccrgx_stencil_view& v, F f, hipStream_t st)
{
    if (v.n_cells == 0) return DCCRGX_OK;
    if (v.kind == 0) {
        detail::UniformGeo g;
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
        const uint64_t tiles = (g.S + 255) / 256;
        if (tiles >= (1ull << 31)) return DCCRGX_EINVAL;
        for (int r = 0; r < 2; r++) {
            const int64_t nsl = v.s1[r] - v.s0[r];
            if (nsl <= 0) continue;
            // about 2^20 workgroups (4096 per CU) and never more than 2^31
            uint64_t chunk = (tiles * (uint64_t)nsl + (1u << 20) - 1) >> 20;
            if (chunk < 1) chunk = 1;
            const uint64_t nch = ((uint64_t)nsl + chunk - 1) / chunk;
            if (tiles * nch >= (1ull << 31)) return DCCRGX_EINVAL;
            hipLaunchKernelGGL(detail::k_user_uniform<F>, dim3((unsigned)(tiles * nch)), dim3(256), 0, st, g,
                               (int64_t)v.s0[r], (int64_t)v.s1[r], (uint32_t)tiles, (uint32_t)chunk, f);
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

}  // namespace dccrgx_user
