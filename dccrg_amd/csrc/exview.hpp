// exview.hpp -- device lookups into an explicit grid's replicated leaf set
// (explicit.hip builds it; explicit.hip and amr_dev.hip read it).
#pragma once

#include "internal.hpp"

struct dccrgx_grid;

namespace dccrgx {

// lookups of existing leaves: id -> global leaf index (position in the
// ascending leaf list).  Grids whose id space is small enough keep a rank
// bitmap: one bit per possible id (dccrg_mapping.hpp's ids are dense per
// level) plus, per 64-bit word, the number of leaves before it -- a lookup is
// one word load, a popcount and one rank load, and neighbors' ids are close
// together (same level: the same z-plane +-1), so the words stay in L2.
// Other grids use an open-addressing hash (2x capacity, linear probing).
struct ExView {
    MapParams mp;
    const uint64_t* keys;
    const uint32_t* vals;
    uint64_t mask;
    const uint64_t* bits;   // rank bitmap (null: use the hash)
    const uint32_t* rank;
    int32_t per[3];
};

__host__ __device__ inline uint64_t hmix(uint64_t x)
{
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

__device__ inline int64_t ex_find(const ExView& v, uint64_t id)
{
    if (id == 0) return -1;
    if (v.bits) {
        if (id > v.mp.last_cell) return -1;
        const uint64_t w = v.bits[id >> 6];
        const uint32_t b = (uint32_t)(id & 63);
        if (!((w >> b) & 1ull)) return -1;
        return (int64_t)v.rank[id >> 6] + __popcll(w & ((1ull << b) - 1ull));
    }
    uint64_t h = hmix(id) & v.mask;
    for (;;) {
        const uint64_t k = v.keys[h];
        if (k == id) return (int64_t)v.vals[h];
        if (k == 0) return -1;
        h = (h + 1) & v.mask;
    }
}

// the window of neighborhood item h around a cell at indices idx of length
// L (in indices), wrapped where the grid is periodic; false outside a
// non-periodic grid (dccrg.hpp:4670-4672, indices_from_neighborhood)
__device__ inline bool nof_window(const MapParams& p, const int32_t* per, const uint64_t idx[3],
                                           const int32_t* h, int64_t L, uint64_t wi[3])
{
    const int M = p.max_lvl;
    for (int d = 0; d < 3; d++) {
        const int64_t G = (int64_t)(p.length[d] << M);
        int64_t x = (int64_t)idx[d] + (int64_t)h[d] * L;
        if (x < 0 || x >= G) {
            if (!per[d]) return false;
            x %= G;
            if (x < 0) x += G;
        }
        wi[d] = (uint64_t)x;
    }
    return true;
}

// neighbors_of of leaf c (find_neighbors_of, dccrg.hpp:4375-4716) as f(leaf
// index) per entry, in the reference's list order: per item, the window's
// cell, else its parent, else its existing children
template <class F>
__device__ inline void nof_search(const ExView& v, const int32_t* items, int K, uint64_t c, F f)
{
    const MapParams& p = v.mp;
    const int M = p.max_lvl;
    uint64_t idx[3];
    int l;
    if (!map_indices(p, c, idx, &l)) return;
    const int64_t L = (int64_t)1 << (M - l);
    for (int k = 0; k < K; k++) {
        uint64_t wi[3];
        if (!nof_window(p, v.per, idx, items + 3 * k, L, wi)) continue;
        int64_t g = ex_find(v, map_cell(p, wi, l));
        if (g >= 0) {
            f((uint32_t)g);
            continue;
        }
        if (l > 0 && (g = ex_find(v, map_cell(p, wi, l - 1))) >= 0) {
            f((uint32_t)g);
            continue;
        }
        if (l >= M) continue;
        const uint64_t hl = (uint64_t)(L / 2);
        for (int ch = 0; ch < 8; ch++) {
            const uint64_t ci[3] = {wi[0] + (ch & 1) * hl, wi[1] + ((ch >> 1) & 1) * hl, wi[2] + ((ch >> 2) & 1) * hl};
            const int64_t gc = ex_find(v, map_cell(p, ci, l + 1));
            if (gc >= 0) f((uint32_t)gc);
        }
    }
}

// neighbors_to by the reference's own search (find_neighbors_to,
// dccrg.hpp:4744-4897): the windows of the neighborhood_to items around the
// cell's parent (one level coarser), around each of its children (one level
// finer) and around the cell itself; a window whose cell at that level is an
// existing leaf is a cell that has this one among its neighbors_of.  Rows of
// any leaf from the replicated leaf lookup alone, so a rank builds them for
// its own cells only (the transpose of neighbors_of needs every leaf's row).
// Entries may repeat (sorted and made unique afterwards).
template <class F>
__device__ inline void nto_search(const ExView& v, const int32_t* items_to, int K, uint64_t c, F f)
{
    const MapParams& p = v.mp;
    const int M = p.max_lvl;
    uint64_t idx[3];
    int l;
    if (!map_indices(p, c, idx, &l)) return;
    const int64_t L = (int64_t)1 << (M - l);
    auto probe = [&](const uint64_t base[3], int lv, int64_t len) {
        for (int k = 0; k < K; k++) {
            uint64_t wi[3];
            if (!nof_window(p, v.per, base, items_to + 3 * k, len, wi)) continue;
            const int64_t g = ex_find(v, map_cell(p, wi, lv));
            if (g >= 0) f((uint32_t)g);
        }
    };
    if (l > 0) {  // larger cells: windows around the parent
        const uint64_t pi[3] = {idx[0] - idx[0] % (uint64_t)(2 * L), idx[1] - idx[1] % (uint64_t)(2 * L),
                                idx[2] - idx[2] % (uint64_t)(2 * L)};
        probe(pi, l - 1, 2 * L);
    }
    if (l < M) {  // smaller cells: windows around each child
        const uint64_t hl = (uint64_t)(L / 2);
        for (int ch = 0; ch < 8; ch++) {
            const uint64_t ci[3] = {idx[0] + (ch & 1) * hl, idx[1] + ((ch >> 1) & 1) * hl, idx[2] + ((ch >> 2) & 1) * hl};
            probe(ci, l + 1, (int64_t)hl);
        }
    }
    probe(idx, l, L);
}

// places for `cnt` entries per lane in a list whose length is *ctr: one
// atomic per wave (a wave prefix sum over the active lanes, which are a
// prefix of the wave in a grid-stride loop) instead of one per lane -- with
// tens of thousands of refined leaves the per-lane atomics on four counters
// serialised at the L2 (k_exec took ~300 us on 3.5 M leaves)
__device__ inline uint32_t wave_reserve(uint32_t* ctr, uint32_t cnt)
{
    const int lane = threadIdx.x & 63;
    const uint64_t act = __ballot(1);
    const int last = 63 - __clzll((long long)act);
    uint32_t x = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    const uint32_t total = __shfl(x, last, 64);
    uint32_t base = 0;
    if (lane == last && total) base = atomicAdd(ctr, total);
    base = __shfl(base, last, 64);
    return base + x - cnt;
}

// the lookups of an explicit grid (explicit.hip)
ExView explicit_view(const dccrgx_grid* grid);

}  // namespace dccrgx
