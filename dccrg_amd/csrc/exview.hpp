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

// the lookups of an explicit grid (explicit.hip)
ExView explicit_view(const dccrgx_grid* grid);

}  // namespace dccrgx
