// stencil.hip -- the device user-stencil view (include/dccrgx_stencil.hpp):
// what a caller's device functor needs to walk a region's cells and each
// cell's neighbors_of in the reference's iteration-cache order
// (dccrg.hpp:11590-11640: unique (id, offset) pairs, the ones whose id is not
// also a neighbor_to first, each group ascending by (id, x, y, z)).
//
// Uniform grids: nothing per cell is stored.  The neighborhood's items are
// sorted once into that order for a cell no periodic wrap reaches (ids then
// grow with the canonical (c, b, a) offsets, and an entry is a neighbor_to
// exactly when the mirrored item is in the neighborhood); cells near a
// periodic wrap select their entries by key in the header.
// Explicit grids: the stencil rows (sorted by (id, offset)) regrouped per cell
// by membership in its neighbors_to row.
#include <algorithm>
#include <array>
#include <cstring>
#include <vector>

#include "grid.hpp"

namespace dccrgx {

IterCache::~IterCache()
{
    FreeBatch fb;
    for (void* q : {(void*)items, (void*)delta, (void*)slot, (void*)off}) fb.add(q);
}

namespace {

unsigned blocks_for(uint64_t n)
{
    const uint64_t b = (n + 255) / 256;
    return (unsigned)(b < 8192 ? (b ? b : 1) : 8192);
}

// the leaf index held by each slot of a leaf (local and ghost slots)
__global__ void __launch_bounds__(256) k_slot_leaf(const uint32_t* __restrict__ slot_of_g, uint64_t n,
                                                   uint32_t* __restrict__ slot_g)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += stride) {
        const uint32_t s = slot_of_g[g];
        if (s != NO_SLOT) slot_g[s] = (uint32_t)g;
    }
}

// one wave per local cell: its stencil row, entries that are not in the
// cell's neighbors_to row first, both groups in row order (ascending (id,
// offset)).  Both rows ascend by leaf index (ids ascend with it); the
// neighbors_to row goes to LDS (up to NTO_LDS entries, else it is searched in
// place), each lane takes one entry of a 64-entry chunk and finds its leaf
// there by binary search, and the wave's ballots place the entries: a count
// pass, then a write pass.  Reads and writes of a chunk are coalesced.
// (Per-entry group flags instead of the copy made this 2.4x faster and the
// walks over the view 2x slower: profiles/r5g_iter_view_time_groupflags.log.)
constexpr int ITER_WAVES = 4, NTO_LDS = 1024, ITER_MASKS = 16, ITER_CH = 3;

__device__ inline bool in_sorted(const uint32_t* a, uint32_t n, uint32_t x)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (a[m] < x) lo = m + 1;
        else hi = m;
    }
    return lo < n && a[lo] == x;
}

__global__ void __launch_bounds__(64 * ITER_WAVES) k_iter_rows(const uint64_t* __restrict__ st_row,
                                                               const uint32_t* __restrict__ st_slot,
                                                               const int32_t* __restrict__ st_off,
                                                               const uint64_t* __restrict__ nto_row,
                                                               const uint32_t* __restrict__ nto_g,
                                                               const uint32_t* __restrict__ slot_g, uint64_t nl,
                                                               int identity,  // slot_g[s] == s (one rank)
                                                               uint32_t* __restrict__ it_slot,
                                                               int32_t* __restrict__ it_off)
{
    __shared__ uint32_t lds[ITER_WAVES][NTO_LDS];
    __shared__ uint64_t msk[ITER_WAVES][ITER_MASKS];  // membership ballots of the first chunks
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    uint32_t* L = lds[w];
    uint64_t* M = msk[w];
    const uint64_t step = (uint64_t)gridDim.x * ITER_WAVES;
    uint64_t i = (uint64_t)blockIdx.x * ITER_WAVES + w;
    // the next row's bounds are loaded while this row is processed
    uint64_t n_e0 = 0, n_e1 = 0, n_t0 = 0, n_t1 = 0;
    if (i < nl) {
        n_e0 = st_row[i];
        n_e1 = st_row[i + 1];
        n_t0 = nto_row[i];
        n_t1 = nto_row[i + 1];
    }
    for (; i < nl; i += step) {
        const uint64_t e0 = n_e0, e1 = n_e1, t0 = n_t0, t1 = n_t1;
        if (i + step < nl) {
            n_e0 = st_row[i + step];
            n_e1 = st_row[i + step + 1];
            n_t0 = nto_row[i + step];
            n_t1 = nto_row[i + step + 1];
        }
        const uint32_t nt = (uint32_t)(t1 - t0);
        if (e1 - e0 <= 64 * ITER_CH && nt <= NTO_LDS) {
            // short row (most): every load of the row issued at once and held
            // in registers -- the row costs three dependent memory round trips
            uint32_t sl[ITER_CH], lg[ITER_CH];
            int32_t o[ITER_CH][3];
            bool valid[ITER_CH];
#pragma unroll
            for (int j = 0; j < ITER_CH; j++) {
                const uint64_t e = e0 + 64 * j + lane;
                valid[j] = e < e1;
                sl[j] = valid[j] ? st_slot[e] : 0;
                for (int a = 0; a < 3; a++) o[j][a] = valid[j] ? st_off[3 * e + a] : 0;
            }
            for (uint32_t k = lane; k < nt; k += 64) L[k] = nto_g[t0 + k];
#pragma unroll
            for (int j = 0; j < ITER_CH; j++) lg[j] = identity ? sl[j] : valid[j] ? slot_g[sl[j]] : 0;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            uint64_t m[ITER_CH];
            uint32_t n_in = 0;
#pragma unroll
            for (int j = 0; j < ITER_CH; j++) {
                m[j] = __ballot(valid[j] && in_sorted(L, nt, lg[j]));
                n_in += (uint32_t)__popcll(m[j]);
            }
            uint64_t w0 = e0, w1 = e1 - n_in;
            const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
            for (int j = 0; j < ITER_CH; j++) {
                const uint64_t m_in = m[j], m_out = __ballot(valid[j]) & ~m_in;
                if (valid[j]) {
                    const bool in = (m_in >> lane) & 1;
                    const uint64_t d = in ? w1 + __popcll(m_in & below) : w0 + __popcll(m_out & below);
                    it_slot[d] = sl[j];
                    for (int a = 0; a < 3; a++) it_off[3 * d + a] = o[j][a];
                }
                w0 += __popcll(m_out);
                w1 += __popcll(m_in);
            }
            __builtin_amdgcn_wave_barrier();  // L is rewritten for the next row
            continue;
        }
        const bool local = nt <= NTO_LDS;
        if (local)
            for (uint32_t k = lane; k < nt; k += 64) L[k] = nto_g[t0 + k];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const uint32_t* T = local ? L : nto_g + t0;
        auto member = [&](uint64_t e) {
            const uint32_t s = st_slot[e];
            return in_sorted(T, nt, identity ? s : slot_g[s]);
        };
        // count pass: entries in the neighbors_to row (the first chunks'
        // ballots are kept for the write pass)
        uint32_t n_in = 0;
        for (uint64_t c = e0, j = 0; c < e1; c += 64, j++) {
            const uint64_t e = c + lane;
            const uint64_t m = __ballot(e < e1 && member(e));
            if (j < ITER_MASKS && lane == 0) M[j] = m;
            n_in += (uint32_t)__popcll(m);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // write pass
        uint64_t w0 = e0, w1 = e1 - n_in;
        for (uint64_t c = e0, j = 0; c < e1; c += 64, j++) {
            const uint64_t e = c + lane;
            const bool valid = e < e1;
            const bool in = valid && (j < ITER_MASKS ? (M[j] >> lane) & 1 : member(e));
            const uint64_t m_out = __ballot(valid && !in), m_in = __ballot(in);
            const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
            if (valid) {
                const uint64_t d = in ? w1 + __popcll(m_in & below) : w0 + __popcll(m_out & below);
                it_slot[d] = st_slot[e];
                it_off[3 * d] = st_off[3 * e];
                it_off[3 * d + 1] = st_off[3 * e + 1];
                it_off[3 * d + 2] = st_off[3 * e + 2];
            }
            w0 += __popcll(m_out);
            w1 += __popcll(m_in);
        }
        __builtin_amdgcn_wave_barrier();  // L is rewritten for the next row
    }
}

int build_iter(const dccrgx_grid* grid, Hood& h, hipStream_t st)
{
    auto ic = std::make_shared<IterCache>();
    if (grid->uniform) {
        const int K = h.K;
        std::vector<std::array<int32_t, 4>> it(K);
        for (int k = 0; k < K; k++) {
            const int32_t* d = &h.of_c[3 * k];
            bool mirror = false;
            for (int j = 0; j < K && !mirror; j++)
                mirror = h.of_c[3 * j] == -d[0] && h.of_c[3 * j + 1] == -d[1] && h.of_c[3 * j + 2] == -d[2];
            it[k] = {d[0], d[1], d[2], mirror ? 1 : 0};
            for (int a = 0; a < 3; a++) ic->reach[a] = std::max(ic->reach[a], std::abs(d[a]));
        }
        // only-neighbors_of entries first, then by id: canonical (c, b, a)
        std::sort(it.begin(), it.end(), [](const std::array<int32_t, 4>& x, const std::array<int32_t, 4>& y) {
            if (x[3] != y[3]) return x[3] < y[3];
            if (x[2] != y[2]) return x[2] < y[2];
            if (x[1] != y[1]) return x[1] < y[1];
            return x[0] < y[0];
        });
        // shape flags: all mirrored; the 26-cube / 6 faces in ascending (c, b, a)
        // order, which is the order the sort gives them when all are mirrored
        bool sym = true;
        for (int k = 0; k < K; k++) sym = sym && it[k][3] == 1;
        ic->shape = sym ? DCCRGX_SHAPE_SYMMETRIC : 0;
        if (sym && K == 26) {
            bool cube = true;
            for (int k = 0, dc = -1; dc <= 1; dc++)
                for (int db = -1; db <= 1; db++)
                    for (int da = -1; da <= 1; da++) {
                        if (!da && !db && !dc) continue;
                        cube = cube && it[k][0] == da && it[k][1] == db && it[k][2] == dc;
                        k++;
                    }
            if (cube) ic->shape |= DCCRGX_SHAPE_CUBE1;
        }
        if (sym && K == 6) {
            static const int32_t fc[6][3] = {{0, 0, -1}, {0, -1, 0}, {-1, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
            bool faces = true;
            for (int k = 0; k < 6; k++)
                faces = faces && it[k][0] == fc[k][0] && it[k][1] == fc[k][1] && it[k][2] == fc[k][2];
            if (faces) ic->shape |= DCCRGX_SHAPE_FACES;
        }
        const UGeom& g = grid->g;
        const int32_t sc = 1 << grid->map.max_lvl;
        std::vector<int32_t> rec(std::max(K, 1) * 8, 0);
        std::vector<int64_t> delta(std::max(K, 1), 0);
        for (int k = 0; k < K; k++) {
            int32_t o[3];
            for (int d = 0; d < 3; d++) o[g.perm[d]] = it[k][d] * sc;  // canonical axis d is axis perm[d]
            const int32_t r[8] = {it[k][0], it[k][1], it[k][2], it[k][3], o[0], o[1], o[2], 0};
            std::memcpy(&rec[8 * k], r, sizeof r);
            delta[k] = it[k][0] + (int64_t)g.LA * it[k][1] + (int64_t)g.S * it[k][2];
        }
        DX_HIP(dx_malloc(&ic->items, rec.size() * 4));
        DX_HIP(dx_malloc(&ic->delta, delta.size() * 8));
        if (K) {
            DX_TRY(dx_h2d(grid->ctx, ic->items, rec.data(), (size_t)K * 32, st));
            DX_TRY(dx_h2d(grid->ctx, ic->delta, delta.data(), (size_t)K * 8, st));
        }
    } else {
        const Explicit* E = grid->ex;
        const uint64_t nl = E->n_local();
        DX_CHECK(!nl || (h.d_st_row && h.d_nto_row && E->d_slot_of_g), DCCRGX_EINTERNAL,
                 "neighborhood %d has no stencil rows", h.id);
        const uint64_t cap = std::max<uint64_t>(h.st_cap, 1);
        PhaseTimer T("build_iter");
        DX_HIP(dx_malloc(&ic->slot, cap * 4));
        DX_HIP(dx_malloc(&ic->off, cap * 12));
        T.lap("allocations");
        if (nl) {
            // the leaf of each slot (one rank: slot s holds leaf s)
            uint32_t* slot_g = nullptr;
            const int identity = E->slot_identity ? 1 : 0;
            if (!identity) {
                DX_HIP(ds_malloc(&slot_g, std::max<uint64_t>(grid->n_slots, 1) * 4, st));
                hipLaunchKernelGGL(k_slot_leaf, dim3(blocks_for(E->n)), dim3(256), 0, st,
                                   (const uint32_t*)E->d_slot_of_g, (uint64_t)E->n, slot_g);
            }
            const unsigned nb = (unsigned)std::min<uint64_t>((nl + ITER_WAVES - 1) / ITER_WAVES, 16384);
            hipLaunchKernelGGL(k_iter_rows, dim3(nb), dim3(64 * ITER_WAVES), 0, st, (const uint64_t*)h.d_st_row,
                               (const uint32_t*)h.d_st_slot, (const int32_t*)h.d_st_off, (const uint64_t*)h.d_nto_row,
                               (const uint32_t*)h.d_nto_g, (const uint32_t*)slot_g, nl, identity, ic->slot, ic->off);
            DX_HIP(hipGetLastError());
            if (slot_g) ds_free(slot_g, st);
            T.lap("rows");
        }
    }
    h.iter = ic;
    return DCCRGX_OK;
}

}  // namespace
}  // namespace dccrgx

using namespace dccrgx;

extern "C" {

int dccrgx_stencil_view_get(const dccrgx_grid* grid, int32_t hood_id, int32_t region, dccrgx_stencil_view* out)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid && out, DCCRGX_EINVAL, "null argument");
    Hood* h = const_cast<Hood*>(find_hood(grid, hood_id));  // the view's data is made on first use
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    DX_CHECK(region >= DCCRGX_REGION_ALL && region <= DCCRGX_REGION_OUTER, DCCRGX_EINVAL, "bad region %d", region);
    DX_CHECK(!grid->load, DCCRGX_ESTATE, "grid data is being loaded");
    hipStream_t st = grid->ctx->compute;
    if (!h->iter) {
        DX_TRY(build_iter(grid, *h, st));
        // the caller may launch on a stream of its own: the rows are complete
        // before the view is handed out (once per structural change)
        DX_HIP(hipStreamSynchronize(st));
    }
    const IterCache& ic = *h->iter;
    dccrgx_stencil_view v;
    std::memset(&v, 0, sizeof v);
    v.stream = (void*)st;
    v.scale = 1 << grid->map.max_lvl;
    if (grid->uniform) {
        const UGeom& g = grid->g;
        v.kind = 0;
        v.n_items = h->K;
        v.items = ic.items;
        v.item_delta = ic.delta;
        for (int d = 0; d < 3; d++) v.reach[d] = ic.reach[d];
        v.shape = ic.shape;
        v.la = g.LA;
        v.lb = g.LB;
        v.lc = g.LC;
        v.lo = g.lo;
        v.hi = g.hi;
        v.cbase = g.cbase;
        v.nslices = (int32_t)g.nslices;
        v.per[0] = g.perA;
        v.per[1] = g.perB;
        v.per[2] = g.perC;
        for (int d = 0; d < 3; d++) v.perm[d] = g.perm[d];
        int64_t r[2][2];
        region_slices(grid, *h, region, r);
        for (int k = 0; k < 2; k++) {
            v.s0[k] = r[k][0];
            v.s1[k] = std::max(r[k][0], r[k][1]);
            // the range's local cells: its slices' lin range within [lo, hi)
            if (v.s1[k] <= v.s0[k]) continue;
            const uint64_t a = (uint64_t)(v.s0[k] + g.cbase) * g.S, b = (uint64_t)(v.s1[k] + g.cbase) * g.S;
            const uint64_t lo = std::max(a, g.lo), hi = std::min(b, g.hi);
            if (hi > lo) v.n_cells += hi - lo;
        }
    } else {
        ExRegion R;
        DX_TRY(explicit_region(grid, *h, region, &R));
        const Explicit* E = grid->ex;
        v.kind = 1;
        v.n_cells = R.n;
        v.pos = R.pos;
        v.local_slot = R.local_slot;
        v.local_g = E->d_local_g;
        v.leaves = E->d_leaves;
        v.row = h->d_st_row;
        v.nbr_slot = ic.slot;
        v.nbr_off = ic.off;
    }
    *out = v;
    return DCCRGX_OK;
}

}  // extern "C"
