// amr_dev.hip -- the refinement requests and the decisions of stop_refining on
// the device, for grids with the explicit (mixed-level) layout.
//
// The reference keeps four per-rank id sets (cells_to_refine,
// cells_not_to_refine, cells_to_unrefine, cells_not_to_unrefine,
// dccrg.hpp:7355-7360) and walks neighbor lists on the host for every request
// (:2456-2806) and every decision pass (:9730-10240).  Here the sets of an
// explicit grid are bit flags over the replicated leaf list (one u32 per
// leaf), and each phase is a batch of independent per-cell kernels over the
// device neighbor CSRs:
//   - requests (refine_completely, dont_unrefine, unrefine_completely,
//     dont_refine) of a whole id array at once.  Their outcome within a batch
//     does not depend on the order of the calls except through "a sibling is
//     already recorded" (dont_unrefine, unrefine_completely): the first
//     request of each sibling group in call order wins (atomicMin of the call
//     index), as the sequential calls would have it;
//   - override_refines / induce_refines as frontier expansions, at most
//     max_refinement_level rounds each (a dont_refine spreads only to finer
//     cells, an induced refine only to coarser ones), with no host round trip;
//   - override_unrefines as one wave per sibling group walking the face graph
//     in LDS (the walk's outcome is an existence test over a closure, so a
//     level-synchronous walk gives the sequential walk's answer, amr.hip);
//   - execute_refines' new leaf list: surviving leaves compacted in order,
//     new cells radix-sorted, one merge.
// The host keeps the same four sets for single request calls (amr.hip); each
// side is brought up to date from the other only when it is next used.
#include <hipcub/hipcub.hpp>

#include "exview.hpp"
#include "face.hpp"
#include "grid.hpp"

namespace dccrgx {

enum : uint32_t {
    RF_REFINE = 1u,
    RF_UNREFINE = 2u,
    RF_NOT_UNREFINE = 4u,
    RF_NOT_REFINE = 8u,
    RF_GONE = 16u,   // execute: the leaf disappears
    RF_KEEP = 32u,   // override_unrefines: the walk of this group / cell passed
};
constexpr uint32_t RF_SETS = RF_REFINE | RF_UNREFINE | RF_NOT_UNREFINE | RF_NOT_REFINE;
static_assert(RF_GONE == AMR_FLAG_GONE, "the rebuild reads the gone flag (grid.hpp)");
constexpr uint32_t NONE32 = 0xffffffffu;

// one explicit grid, its default neighborhood and the request flags
struct AView {
    ExView v;
    const uint64_t* leaves;
    uint64_t n;
    const uint64_t* nof_row;  // the local cells' rows (row = local position = slot)
    const uint32_t* nof_g;
    const uint64_t* nto_row;
    const uint32_t* nto_g;
    const uint32_t* slot_of_g;  // leaf index -> slot (the row of a local cell)
    int rows_all;               // one process: the rows are every leaf's (row = leaf index)
    const int32_t* items;     // default neighborhood items (original axes)
    const int32_t* items_to;  // and their negation (neighborhood_to)
    int32_t K;
    uint32_t hood_len;
    Partition part;
    SfcCuts sfc;  // SFC placement (device cut keys), or sfc.cut null (block partition)
    int32_t rank;
    uint32_t* flags;
};

struct AExists {
    ExView v;
    __device__ bool operator()(uint64_t c) const { return ex_find(v, c) >= 0; }
};

__device__ inline int a_level(const AView& a, uint64_t c) { return map_level(a.v.mp, c); }

// Mapping::get_parent (dccrg_mapping.hpp:298-330): a level-0 cell is its own
__device__ inline uint64_t a_parent(const AView& a, uint64_t c)
{
    uint64_t idx[3];
    int l;
    if (!map_indices(a.v.mp, c, idx, &l)) return 0;
    return l == 0 ? c : map_cell(a.v.mp, idx, l - 1);
}

// Mapping::get_all_children (:392-442), x fastest; zeros at the maximum level
__device__ inline void a_children(const AView& a, uint64_t c, uint64_t out[8])
{
    uint64_t idx[3];
    int l;
    for (int i = 0; i < 8; i++) out[i] = 0;
    if (!map_indices(a.v.mp, c, idx, &l) || l >= a.v.mp.max_lvl) return;
    const uint64_t h = (uint64_t)1 << (a.v.mp.max_lvl - l - 1);
    for (int i = 0; i < 8; i++) {
        const uint64_t ci[3] = {idx[0] + (i & 1) * h, idx[1] + ((i >> 1) & 1) * h, idx[2] + ((i >> 2) & 1) * h};
        out[i] = map_cell(a.v.mp, ci, l + 1);
    }
}

// Mapping::get_siblings (:450-471)
__device__ inline void a_siblings(const AView& a, uint64_t c, uint64_t out[8])
{
    if (a_level(a, c) == 0) {
        out[0] = c;
        for (int i = 1; i < 8; i++) out[i] = 0;
        return;
    }
    a_children(a, a_parent(a, c), out);
}

// process of a cell: its level-0 ancestor's (dccrg.hpp:10368, :10437)
__device__ inline int a_owner(const AView& a, uint64_t c)
{
    uint64_t idx[3];
    int l;
    map_indices(a.v.mp, c, idx, &l);
    const uint64_t l0 = map_cell(a.v.mp, idx, 0);
    return a.sfc.cut ? sfc_owner(a.sfc, l0) : part_owner(a.part, l0);
}

// c != get_child(c), dccrg.hpp:9694-9718
__device__ inline bool a_has_children(const AView& a, uint64_t c)
{
    const int l = a_level(a, c);
    const bool ex = ex_find(a.v, c) >= 0;
    if (l == a.v.mp.max_lvl) return !ex;
    uint64_t idx[3];
    int ll;
    map_indices(a.v.mp, c, idx, &ll);
    if (ex_find(a.v, map_cell(a.v.mp, idx, l + 1)) >= 0) return true;
    return !ex;
}

// is_neighbor, dccrg.hpp:9603-9683
__device__ inline bool a_is_neighbor(const AView& a, uint64_t c1, uint64_t c2)
{
    const MapParams& mp = a.v.mp;
    const int M = mp.max_lvl;
    uint64_t i1[3], i2[3];
    int l1, l2;
    map_indices(mp, c1, i1, &l1);
    map_indices(mp, c2, i2, &l2);
    const uint64_t len1 = (uint64_t)1 << (M - l1), len2 = (uint64_t)1 << (M - l2);
    uint64_t maxd = 0;
    int overlap = 0;
    for (int d = 0; d < 3; d++) {
        const uint64_t G = mp.length[d] << M;
        uint64_t dist;
        if (i1[d] <= i2[d]) {
            dist = i2[d] <= i1[d] + len1 ? 0 : i2[d] - (i1[d] + len1);
            if (a.v.per[d]) dist = min(dist, i1[d] + (G - (i2[d] + len2)));
        } else {
            dist = i1[d] <= i2[d] + len2 ? 0 : i1[d] - (i2[d] + len2);
            if (a.v.per[d]) dist = min(dist, i2[d] + (G - (i1[d] + len1)));
        }
        maxd = max(maxd, dist);
        overlap += (i1[d] + len1 > i2[d] && i1[d] < i2[d] + len2) ? 1 : 0;  // dccrg.hpp:11364-11405
    }
    if (a.hood_len == 0) return maxd < len1 && overlap >= 2;
    return maxd < (uint64_t)a.hood_len * len1;
}

// cells_to_unrefine.erase(every sibling of c)
__device__ inline void a_erase_sibling_unrefines(const AView& a, uint64_t c)
{
    uint64_t s[8];
    a_siblings(a, c, s);
    for (int k = 0; k < 8; k++) {
        if (!s[k]) continue;
        const int64_t g = ex_find(a.v, s[k]);
        if (g >= 0 && (a.flags[g] & RF_UNREFINE)) atomicAnd(&a.flags[g], ~RF_UNREFINE);
    }
}

// ---------------------------------------------------------------------------
// requests
// ---------------------------------------------------------------------------

// refine_completely, dccrg.hpp:2476-2546.  Requests at the maximum level are
// dont_unrefine calls (:2486-2488): they are queued for the dont_unrefine
// kernels with their call index.  One wave per request, its lanes over the
// cell's rows (the blocking test, then the sibling unrefines erased around it).
__global__ void __launch_bounds__(256) k_req_refine(AView a, const uint64_t* __restrict__ ids, uint64_t n,
                                                    int32_t* __restrict__ res, uint64_t* __restrict__ du_ids,
                                                    uint32_t* __restrict__ du_ord, uint32_t* __restrict__ du_n, int erase)
{
    const int M = a.v.mp.max_lvl;
    const int lane = threadIdx.x & 63;
    const uint64_t nwave = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n; i += nwave) {
        const uint64_t c = ids[i];  // wave-uniform from here on
        int32_t r = 0;
        const int64_t g = ex_find(a.v, c);
        if (g >= 0 && a_owner(a, c) == a.rank) {
            const int lvl = a_level(a, c);
            if (lvl == M) {
                if (lane == 0) {
                    const uint32_t p = atomicAdd(du_n, 1u);
                    du_ids[p] = c;
                    du_ord[p] = (uint32_t)i;
                }
                r = 1;  // dont_unrefine of an existing cell
            } else if (!(a.flags[g] & RF_NOT_REFINE)) {
                const uint32_t rw = a.slot_of_g[g];  // a local cell: its row
                bool blk = false;
                for (uint64_t e = a.nof_row[rw] + lane; e < a.nof_row[rw + 1]; e += 64) {
                    const uint32_t t = a.nof_g[e];
                    blk |= a_level(a, a.leaves[t]) < lvl && (a.flags[t] & RF_NOT_REFINE);
                }
                if (!__ballot(blk)) {
                    r = 1;
                    if (lane == 0) atomicOr(&a.flags[g], RF_REFINE);
                    if (erase) {  // (no cells_to_unrefine to erase when the adapter refines first)
                        if (lane == 0) a_erase_sibling_unrefines(a, c);
                        for (int pass = 0; pass < 2; pass++) {
                            const uint64_t* row = pass ? a.nto_row : a.nof_row;
                            const uint32_t* val = pass ? a.nto_g : a.nof_g;
                            for (uint64_t e = row[rw] + lane; e < row[rw + 1]; e += 64) {
                                const uint64_t nb = a.leaves[val[e]];
                                if (a_level(a, nb) <= lvl) a_erase_sibling_unrefines(a, nb);
                            }
                        }
                    }
                }
            }
        }
        if (lane == 0 && res) res[i] = r;
    }
}

// dont_unrefine, dccrg.hpp:2715-2759, phase 1 (reads the flags only): the
// sibling group's key (its smallest existing leaf index) unless a sibling is
// already in cells_not_to_unrefine; the first call of each group wins
__global__ void __launch_bounds__(256) k_req_du_a(AView a, const uint64_t* __restrict__ ids,
                                                  const uint32_t* __restrict__ ord, const uint32_t* __restrict__ n_dev,
                                                  uint64_t n_host, int32_t* __restrict__ res, uint32_t* __restrict__ grp,
                                                  uint32_t* __restrict__ key)
{
    const uint64_t n = n_dev ? *n_dev : n_host;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t c = ids[i];
        const uint32_t o = ord ? ord[i] : (uint32_t)i;
        key[i] = NONE32;
        const int64_t g = ex_find(a.v, c);
        if (res) res[o] = g >= 0 ? 1 : 0;
        if (g < 0 || a_level(a, c) == 0) continue;
        uint64_t s[8];
        a_siblings(a, c, s);
        uint32_t kmin = NONE32;
        bool recorded = false;
        for (int k = 0; k < 8; k++) {
            const int64_t gs = s[k] ? ex_find(a.v, s[k]) : -1;
            if (gs < 0) continue;
            kmin = min(kmin, (uint32_t)gs);
            recorded |= (a.flags[gs] & RF_NOT_UNREFINE) != 0;
        }
        if (recorded) continue;
        key[i] = kmin;
        atomicMin(&grp[kmin], o);
    }
}

// phase 2: the winner erases its siblings from cells_to_unrefine and is recorded
__global__ void __launch_bounds__(256) k_req_du_b(AView a, const uint64_t* __restrict__ ids,
                                                  const uint32_t* __restrict__ ord, const uint32_t* __restrict__ n_dev,
                                                  uint64_t n_host, const uint32_t* __restrict__ grp,
                                                  const uint32_t* __restrict__ key, int erase)
{
    const uint64_t n = n_dev ? *n_dev : n_host;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t k = key[i];
        if (k == NONE32 || grp[k] != (ord ? ord[i] : (uint32_t)i)) continue;
        const uint64_t c = ids[i];
        if (erase) a_erase_sibling_unrefines(a, c);
        atomicOr(&a.flags[ex_find(a.v, c)], RF_NOT_UNREFINE);
    }
}

// the leaves overlapping the neighborhood windows of a parent that does not
// exist (its children are leaves): does any of them block unrefining it?
// (amr.hip View::parent_window_leaves and unrefine_completely's tests, :2638-2670.)
// A window W at the parent's level is covered by W itself, by W's parent, by
// a coarser ancestor (no leaf inside W) or by W's children; a child that is
// not a leaf is refined, so its leaves are finer than plvl + 1.
// does the window of item k of a parent at indices pi, level pl block it?
__device__ inline bool a_item_blocks(const AView& a, const uint64_t pi[3], int pl, int k)
{
    const MapParams& mp = a.v.mp;
    const int M = mp.max_lvl;
    const int64_t L = (int64_t)1 << (M - pl);
    uint64_t wi[3];
    for (int d = 0; d < 3; d++) {
        const int64_t G = (int64_t)(mp.length[d] << M);
        int64_t x = (int64_t)pi[d] + (int64_t)a.items[3 * k + d] * L;
        if (x < 0 || x >= G) {
            if (!a.v.per[d]) return false;
            x %= G;
            if (x < 0) x += G;
        }
        wi[d] = (uint64_t)x;
    }
    const uint64_t W = map_cell(mp, wi, pl);
    // W and its parent looked up together, then W's eight children together
    // and their flags together: three dependent lookups, not up to eighteen
    const int64_t gw = ex_find(a.v, W);
    const int64_t gp = pl > 0 ? ex_find(a.v, map_cell(mp, wi, pl - 1)) : -1;
    if (gw >= 0) return false;  // a leaf of the parent's level
    if (gp >= 0) return false;  // coarser
    for (int l = pl - 2; l >= 0; l--)  // covered by a coarser ancestor: no leaf inside W
        if (ex_find(a.v, map_cell(mp, wi, l)) >= 0) return false;
    if (pl >= M) return false;
    uint64_t ch[8];
    a_children(a, W, ch);
    int64_t gc[8];
#pragma unroll
    for (int j = 0; j < 8; j++) gc[j] = ex_find(a.v, ch[j]);
    bool refined = false;  // a child that is not a leaf: leaves at plvl + 2 or finer
#pragma unroll
    for (int j = 0; j < 8; j++) refined |= gc[j] < 0;
    if (refined) return true;
    uint32_t f = 0;  // plvl + 1 and about to be refined
#pragma unroll
    for (int j = 0; j < 8; j++) f |= a.flags[gc[j]];
    return (f & RF_REFINE) != 0;
}

// unrefine_completely, dccrg.hpp:2596-2675, phase 1 (reads the flags only).
// L lanes per request (L = 8 .. 64, the window items' count rounded up, at
// least the 8 siblings): lanes 0-7 of the group test the siblings (their
// outcome in the reference's order, :2617-2633, is the first sibling that
// stops the loop, found by ballot), then the group's lanes share the
// parent's window items (a serial walk of them was a chain of ~100 dependent
// lookups per request).  A group's control flow is uniform (one request), so
// its ballots are its own bits of the wave's.
template <int L>
__global__ void __launch_bounds__(256) k_req_unref_a(AView a, const uint64_t* __restrict__ ids, uint64_t n,
                                                     int32_t* __restrict__ res, uint32_t* __restrict__ grp,
                                                     uint32_t* __restrict__ key)
{
    const int lane = threadIdx.x & 63, sl = lane % L, gb = lane - sl;
    const uint64_t gmask = L == 64 ? ~0ull : ((1ull << L) - 1);
    auto gballot = [&](bool x) { return (uint64_t)(__ballot(x) >> gb) & gmask; };
    const uint64_t ngroup = (uint64_t)gridDim.x * (blockDim.x / L);
    for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x / L) + threadIdx.x / L; i < n; i += ngroup) {
        const uint64_t c = ids[i];  // group-uniform from here on
        int32_t r = 0;
        uint32_t kk = NONE32;
        const int64_t g = ex_find(a.v, c);
        if (g >= 0 && a_owner(a, c) == a.rank) {
            r = 1;
            uint64_t pi[3];
            int pl;
            const uint64_t parent = a_parent(a, c);
            if (a_level(a, c) > 0 && map_indices(a.v.mp, parent, pi, &pl)) {
                const uint64_t h = (uint64_t)1 << (a.v.mp.max_lvl - pl - 1);
                bool hc = false, fl = false, un = false;
                int64_t gk = -1;
                if (sl < 8) {  // sibling `sl` (x fastest, Mapping::get_all_children)
                    const uint64_t ci[3] = {pi[0] + (sl & 1) * h, pi[1] + ((sl >> 1) & 1) * h,
                                            pi[2] + ((sl >> 2) & 1) * h};
                    const uint64_t sk = map_cell(a.v.mp, ci, pl + 1);
                    hc = a_has_children(a, sk);
                    if (!hc) {  // no children: a leaf
                        gk = ex_find(a.v, sk);
                        const uint32_t f = a.flags[gk];
                        fl = (f & (RF_REFINE | RF_NOT_UNREFINE)) != 0;
                        un = (f & RF_UNREFINE) != 0;
                    }
                }
                const uint64_t stop1 = gballot(hc || fl);
                bool stop = stop1 != 0;
                if (stop) {
                    if ((gballot(hc) >> (__ffsll((unsigned long long)stop1) - 1)) & 1) r = 0;  // first stop: children
                } else {
                    stop = gballot(un) != 0;  // a sibling already recorded (amr.hip)
                }
                if (!stop) {
                    bool blk = false;
                    for (int k = sl; k < a.K; k += L) blk |= a_item_blocks(a, pi, pl, k);
                    if (!gballot(blk)) {
                        const uint32_t k0 = (uint32_t)__shfl(gk, gb, 64);  // sibling 0, a leaf
                        kk = k0;
                        if (sl == 0) atomicMin(&grp[k0], (uint32_t)i);
                    }
                }
            }
        }
        if (sl == 0) {
            key[i] = kk;
            if (res) res[i] = r;
        }
    }
}

__global__ void __launch_bounds__(256) k_req_unref_b(AView a, const uint64_t* __restrict__ ids, uint64_t n,
                                                     const uint32_t* __restrict__ grp, const uint32_t* __restrict__ key)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t k = key[i];
        if (k != NONE32 && grp[k] == (uint32_t)i) atomicOr(&a.flags[ex_find(a.v, ids[i])], RF_UNREFINE);
    }
}

// dont_refine, dccrg.hpp:2782-2805
__global__ void __launch_bounds__(256) k_req_dont_refine(AView a, const uint64_t* __restrict__ ids, uint64_t n,
                                                         int32_t* __restrict__ res)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t c = ids[i];
        const int64_t g = ex_find(a.v, c);
        if (res) res[i] = g >= 0 ? 1 : 0;
        if (g < 0 || a_level(a, c) == a.v.mp.max_lvl) continue;
        atomicAnd(&a.flags[g], ~RF_REFINE);
        atomicOr(&a.flags[g], RF_NOT_REFINE);
    }
}

// host sets -> flags: ids[i] gets bits[i]; dont_refine ids that are not
// leaves are kept aside (the set persists, :10178)
__global__ void __launch_bounds__(256) k_flags_scatter(AView a, const uint64_t* __restrict__ ids,
                                                       const uint32_t* __restrict__ bits, uint64_t n,
                                                       uint64_t* __restrict__ other, uint32_t* __restrict__ other_n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t g = ex_find(a.v, ids[i]);
        if (g >= 0) atomicOr(&a.flags[g], bits[i]);
        else if (bits[i] & RF_NOT_REFINE) other[atomicAdd(other_n, 1u)] = ids[i];
    }
}

// flags -> (id, bits) of every leaf in any set
__global__ void __launch_bounds__(256) k_flags_gather(AView a, uint64_t* __restrict__ ids, uint32_t* __restrict__ bits,
                                                      uint32_t* __restrict__ cnt)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < a.n; g += stride) {
        const uint32_t f = a.flags[g] & RF_SETS;
        const uint32_t p = wave_reserve(cnt, f ? 1u : 0u);
        if (!f) continue;
        ids[p] = a.leaves[g];
        bits[p] = f;
    }
}

// ---------------------------------------------------------------------------
// stop_refining
// ---------------------------------------------------------------------------

// frontier: leaves with `bit`; refines of dont_refine leaves are dropped
// first (override_refines' last step, :10181-10183)
__global__ void __launch_bounds__(256) k_collect(AView a, uint32_t bit, uint32_t* __restrict__ out,
                                                 uint32_t* __restrict__ cnt)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < a.n; g += stride) {
        uint32_t f = a.flags[g];
        if (bit == RF_REFINE && (f & RF_NOT_REFINE) && (f & RF_REFINE)) a.flags[g] = f &= ~RF_REFINE;
        const uint32_t p = wave_reserve(cnt, (f & bit) ? 1u : 0u);
        if (f & bit) out[p] = (uint32_t)g;
    }
}

// one round of override_refines (finer = 1: every finer neighbor of a
// dont_refine leaf joins, :10130-10177) or induce_refines (finer = 0: every
// coarser neighbor of a refined leaf, :9730-9907); neighbors of / to.  The
// frontier holds cells of every process: with several processes their
// neighbors are searched from the replicated leaf lookup (nof_search /
// nto_search), since a process keeps lists for its own cells only; one
// process reads its lists.
__global__ void __launch_bounds__(256) k_spread(AView a, uint32_t bit, int finer, const uint32_t* __restrict__ front,
                                                const uint32_t* __restrict__ front_n, uint32_t* __restrict__ next,
                                                uint32_t* __restrict__ next_n)
{
    const uint32_t n = *front_n;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t g = front[i];
        const uint64_t c = a.leaves[g];
        const int l = a_level(a, c);
        auto visit = [&](uint32_t t) {
            const int lt = a_level(a, a.leaves[t]);
            if (finer ? lt <= l : lt >= l) return;
            if (a.flags[t] & bit) return;
            if (!(atomicOr(&a.flags[t], bit) & bit)) next[atomicAdd(next_n, 1u)] = t;
        };
        if (a.rows_all) {  // one process holds every leaf's rows: read them
            for (uint64_t e = a.nof_row[g]; e < a.nof_row[g + 1]; e++) visit(a.nof_g[e]);
            for (uint64_t e = a.nto_row[g]; e < a.nto_row[g + 1]; e++) visit(a.nto_g[e]);
        } else {
            nof_search(a.v, a.items, a.K, c, visit);
            nto_search(a.v, a.items_to, a.K, c, visit);
        }
    }
}

// k_spread on one process (every leaf's rows held): one wave per frontier
// cell, its lanes over the cell's rows (the per-cell loop over ~50 entries
// was a latency chain with a few hundred cells in flight)
__global__ void __launch_bounds__(256) k_spread_rows(AView a, uint32_t bit, int finer, const uint32_t* __restrict__ front,
                                                     const uint32_t* __restrict__ front_n, uint32_t* __restrict__ next,
                                                     uint32_t* __restrict__ next_n)
{
    const uint32_t n = *front_n;
    const int lane = threadIdx.x & 63;
    const uint64_t nwave = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n; i += nwave) {
        const uint32_t g = front[i];
        const int l = a_level(a, a.leaves[g]);
        const uint64_t b0 = a.nof_row[g], n0 = a.nof_row[g + 1] - b0;
        const uint64_t b1 = a.nto_row[g], n1 = a.nto_row[g + 1] - b1;
        for (uint64_t e = lane; e < n0 + n1; e += 64) {
            const uint32_t t = e < n0 ? a.nof_g[b0 + e] : a.nto_g[b1 + (e - n0)];
            const int lt = a_level(a, a.leaves[t]);
            if (finer ? lt <= l : lt >= l) continue;
            if (a.flags[t] & bit) continue;
            if (!(atomicOr(&a.flags[t], bit) & bit)) next[atomicAdd(next_n, 1u)] = t;
        }
    }
}

// override_unrefines, dccrg.hpp:9935-10124 (amr.hip explains the
// restatement): sibling groups whose children are all leaves walk once, from
// their smallest requested leaf; other requests walk alone.  key[i] (and
// lkey[leaf], for execute_refines) = the group's first child's leaf index, or
// NONE32 for a lone request.  The eight children are looked up together.
__global__ void __launch_bounds__(256) k_ou_group(AView a, const uint32_t* __restrict__ us, const uint32_t* __restrict__ nu,
                                                  uint32_t* __restrict__ grp, uint32_t* __restrict__ key,
                                                  uint32_t* __restrict__ lkey)
{
    const uint32_t n = *nu;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t g = us[i];
        uint64_t ch[8];
        a_children(a, a_parent(a, a.leaves[g]), ch);
        int64_t gc[8];
        bool all = true;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            gc[k] = ch[k] ? ex_find(a.v, ch[k]) : -1;
            all &= gc[k] >= 0;
        }
        const uint32_t k0 = all ? (uint32_t)gc[0] : NONE32;
        key[i] = k0;
        lkey[g] = k0;
        if (all) atomicMin(&grp[k0], g);
    }
}

// LDS-or-global workspace of one walk
struct Walk {
    uint64_t* queue;  // Q entries
    uint64_t* seen;   // S entries (open addressing, 0 = empty), S a power of two
    uint32_t Q, S;
};

// insert x into the seen set; true if it was not there.  *over on a full table.
__device__ inline bool walk_insert(const Walk& w, uint64_t x, int* over)
{
    uint32_t h = (uint32_t)hmix(x) & (w.S - 1);
    for (uint32_t probe = 0; probe < w.S; probe++) {
        const unsigned long long prev =
            atomicCAS(reinterpret_cast<unsigned long long*>(&w.seen[h]), 0ull, (unsigned long long)x);
        if (prev == 0ull) return true;
        if (prev == (unsigned long long)x) return false;
        h = (h + 1) & (w.S - 1);
    }
    *over = 1;
    return false;
}

// one wave (workgroup of 64) per walk; `use_lds`: the workspace is in LDS,
// else `scratch` holds one workspace per workgroup.  The walks are the
// entries of `us` (or the entries idx[0 .. *n_idx) of it).  With `retry`
// non-null a walk whose workspace overflows is appended there (its `us`
// index) for a pass with a larger workspace, instead of failing.
__global__ void __launch_bounds__(64) k_ou_walk(AView a, const uint32_t* __restrict__ us, const uint32_t* __restrict__ nu,
                                                const uint32_t* __restrict__ idx, const uint32_t* __restrict__ n_idx,
                                                const uint32_t* __restrict__ grp, const uint32_t* __restrict__ key,
                                                uint32_t Q, uint32_t S, int use_lds, uint64_t* __restrict__ scratch,
                                                uint32_t* __restrict__ retry, uint32_t* __restrict__ n_retry,
                                                int32_t* __restrict__ err)
{
    extern __shared__ uint64_t lds[];
    __shared__ uint32_t head, tail, fail;
    __shared__ int over;
    const int lane = threadIdx.x;
    Walk w;
    w.Q = Q;
    w.S = S;
    w.queue = use_lds ? lds : scratch + (size_t)blockIdx.x * (Q + S);
    w.seen = w.queue + Q;
    const uint32_t n = idx ? *n_idx : *nu;
    AExists exists{a.v};
    int32_t per[3] = {a.v.per[0], a.v.per[1], a.v.per[2]};
    for (uint32_t j0 = blockIdx.x; j0 < n; j0 += gridDim.x) {
        const uint32_t i = idx ? idx[j0] : j0;
        const uint32_t g = us[i];
        const uint32_t k = key[i];
        if (k != NONE32 && grp[k] != g) continue;  // not the group's walker (uniform across the wave)
        const uint64_t u = a.leaves[g];
        const uint64_t parent = a_parent(a, u);
        const int ul = a_level(a, u);
        for (uint32_t s = lane; s < S; s += 64) w.seen[s] = 0;
        if (lane == 0) {
            head = 0;
            tail = 0;
            over = 0;
            fail = 0;
        }
        __syncthreads();
        if (lane < 8) {  // a sibling to be refined or kept (:9960-9975), one lookup per lane
            uint64_t sib[8];
            a_children(a, parent, sib);
            const int64_t gs = sib[lane] ? ex_find(a.v, sib[lane]) : -1;
            if (gs >= 0 && (a.flags[gs] & (RF_REFINE | RF_NOT_UNREFINE))) atomicOr(&fail, 1u);
        }
        __syncthreads();
        if (lane == 0 && !fail) {
            uint64_t f6[6];
            face_graph(a.v.mp, per, u, f6, exists);
            int ov = 0;
            for (int j = 0; j < 6; j++)
                if (f6[j] && walk_insert(w, f6[j], &ov)) w.queue[tail++] = f6[j];
            over |= ov;
        }
        __syncthreads();
        while (!fail && !over && head < tail) {
            const uint32_t h0 = head, t0 = tail;
            const uint32_t batch = min(t0 - h0, 64u);
            if ((uint32_t)lane < batch) {
                const uint64_t x = w.queue[h0 + lane];
                const int rl = a_level(a, x);
                const int64_t gx = ex_find(a.v, x);
                if (rl > ul || (rl == ul && gx >= 0 && (a.flags[gx] & RF_REFINE))) {
                    atomicOr(&fail, 1u);
                } else {
                    uint64_t f6[6];
                    face_graph(a.v.mp, per, x, f6, exists);
                    int ov = 0;
                    for (int j = 0; j < 6; j++) {
                        if (!f6[j] || !walk_insert(w, f6[j], &ov)) continue;
                        if (!a_is_neighbor(a, parent, f6[j])) continue;
                        const uint32_t p = atomicAdd(&tail, 1u);
                        if (p < Q) w.queue[p] = f6[j];
                        else ov = 1;
                    }
                    if (ov) atomicOr(&over, 1);
                }
            }
            __syncthreads();
            if (lane == 0) head = h0 + batch;
            __syncthreads();
        }
        if (lane == 0) {
            if (over && retry) retry[atomicAdd(n_retry, 1u)] = i;
            else if (over) atomicOr(err, 1);
            else if (!fail) atomicOr(&a.flags[k != NONE32 ? k : g], RF_KEEP);
        }
        __syncthreads();
    }
}

// override_unrefines as a window test (the default; k_ou_walk, the
// reference's walk, under the test option "ou_walk").  The walk of
// dccrg.hpp:9975-10040 starts at the unrefined cell's face neighbors and
// spreads through face neighbors that are is_neighbor(parent, .) (:9603-9683),
// failing at a leaf finer than the unrefined cell or at one of its level to
// be refined.  Those leaves are the ones overlapping the parent's
// neighborhood box (the parent-sized windows at the neighborhood's offsets,
// and the parent itself); leaves tiling a box are face-connected inside it
// and the start cells lie in it, so the walk reaches every one of them and
// no other: it fails exactly when a sibling is not a leaf (finer leaves
// inside the parent) or is to be refined, or a window holds such leaves
// (a_item_blocks, the request-time test of unrefine_completely, :2638-2670).
// One wave per group walker / lone request: lanes 0-7 the siblings, then the
// lanes over the window items.
__global__ void __launch_bounds__(256) k_ou_check(AView a, const uint32_t* __restrict__ us,
                                                  const uint32_t* __restrict__ nu, const uint32_t* __restrict__ grp,
                                                  const uint32_t* __restrict__ key)
{
    const uint32_t n = *nu;
    const int lane = threadIdx.x & 63;
    const uint64_t nwave = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n; i += nwave) {
        const uint32_t g = us[i];
        const uint32_t k = key[i];
        if (k != NONE32 && grp[k] != g) continue;  // not the group's walker (wave-uniform)
        uint64_t pi[3];
        int pl;
        if (!map_indices(a.v.mp, a_parent(a, a.leaves[g]), pi, &pl)) continue;
        bool bad = false;
        if (lane < 8) {  // a sibling that is not a leaf, or is to be refined or kept (:9960-9975)
            const uint64_t h = (uint64_t)1 << (a.v.mp.max_lvl - pl - 1);
            const uint64_t ci[3] = {pi[0] + (lane & 1) * h, pi[1] + ((lane >> 1) & 1) * h,
                                    pi[2] + ((lane >> 2) & 1) * h};
            const int64_t gs = ex_find(a.v, map_cell(a.v.mp, ci, pl + 1));
            bad = gs < 0 || (a.flags[gs] & (RF_REFINE | RF_NOT_UNREFINE)) != 0;
        }
        if (__ballot(bad)) continue;
        for (int q = lane; q < a.K; q += 64) bad |= a_item_blocks(a, pi, pl, q);
        if (!__ballot(bad) && lane == 0) atomicOr(&a.flags[k != NONE32 ? k : g], RF_KEEP);
    }
}

// execute_refines, dccrg.hpp:10243-10693: children of refined leaves and
// parents of unrefined groups are added; refined leaves and every child of an
// unrefined parent go.  Local ones are reported (new / removed / retired).
// A group with all children leaves is handled by its walker only; lone
// requests may repeat a parent (sorted and made unique afterwards).
struct ExecOut {
    uint64_t* added;
    uint64_t* newc;
    uint64_t* removed;
    uint64_t* retired;
    uint64_t* nr;
    uint32_t* cnt;  // added, new, removed, retired, nr
};

__global__ void __launch_bounds__(256) k_exec(AView a, const uint32_t* __restrict__ grp,
                                              const uint32_t* __restrict__ lkey, ExecOut o)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < a.n; g += stride) {
        const uint32_t f = a.flags[g];
        const bool unref = (f & RF_UNREFINE) != 0, nr = (f & RF_NOT_REFINE) != 0;
        // most waves hold no request at all (active lanes agree: the
        // reservations below need every active lane)
        if (!__ballot((f & RF_REFINE) || unref || nr)) continue;
        const uint64_t c = a.leaves[g];
        // what this leaf adds: children of a refined leaf; the parent of an
        // unrefined group (by its walker, or by a lone request)
        const bool ref = (f & RF_REFINE) != 0;
        const bool ref_local = ref && a_owner(a, c) == a.rank;
        bool fin = false, fin_local = false;
        uint64_t par = 0, ch[8];
        int64_t gc[8];
        if (unref) {
            // override_unrefines' outcome: k_ou_check / k_ou_walk kept the
            // group (on its first child's flags when every child is a leaf,
            // k_ou_group's key) or the lone request (on its own)
            const uint32_t k0 = lkey[g];
            if (a.flags[k0 != NONE32 ? k0 : (uint32_t)g] & RF_KEEP) {
                fin = !(k0 != NONE32 && grp[k0] != (uint32_t)g);  // the group's walker does it
                if (fin) {
                    par = a_parent(a, c);
                    a_children(a, par, ch);
#pragma unroll
                    for (int k = 0; k < 8; k++) gc[k] = ch[k] ? ex_find(a.v, ch[k]) : -1;
                    fin_local = a_owner(a, par) == a.rank;  // the children's process too
                }
            }
        }
        uint32_t nch = 0;
        if (fin_local)
            for (int k = 0; k < 8; k++) nch += ch[k] ? 1u : 0u;
        const uint32_t p_add = wave_reserve(&o.cnt[0], (ref ? 8u : 0u) + (fin ? 1u : 0u));
        const uint32_t p_new = wave_reserve(&o.cnt[1], ref_local ? 8u : 0u);
        const uint32_t p_rem = wave_reserve(&o.cnt[2], nch);
        uint32_t p_ret = wave_reserve(&o.cnt[3], (ref_local ? 1u : 0u) + nch);
        // dont_refine ids that persist (:10178): leaves with the flag
        const uint32_t p_nr = wave_reserve(&o.cnt[4], nr ? 1u : 0u);
        if (nr) o.nr[p_nr] = c;
        if (ref) {
            atomicOr(&a.flags[g], RF_GONE);
            uint64_t cc[8];
            a_children(a, c, cc);
            for (int k = 0; k < 8; k++) o.added[p_add + k] = cc[k];
            if (ref_local) {
                for (int k = 0; k < 8; k++) o.newc[p_new + k] = cc[k];
                o.retired[p_ret++] = c;
            }
        }
        if (!fin) continue;
        o.added[p_add + (ref ? 8u : 0u)] = par;
        uint32_t w = 0;
        for (int k = 0; k < 8; k++) {
            if (!ch[k]) continue;
            if (gc[k] >= 0) atomicOr(&a.flags[gc[k]], RF_GONE);
            if (fin_local) {
                o.removed[p_rem + w] = ch[k];
                o.retired[p_ret + w] = ch[k];
                w++;
            }
        }
    }
}

__device__ inline uint64_t lower_bound_u64(const uint64_t* v, uint64_t n, uint64_t x)
{
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (v[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// merge of two ascending, disjoint lists (counts on the device)
__global__ void __launch_bounds__(256) k_merge(const uint64_t* __restrict__ a, const uint64_t* __restrict__ na_p,
                                               const uint64_t* __restrict__ b, const uint64_t* __restrict__ nb_p,
                                               uint64_t* __restrict__ out)
{
    const uint64_t na = *na_p, nb = *nb_p;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < na + nb; i += stride) {
        if (i < na) out[i + lower_bound_u64(b, nb, a[i])] = a[i];
        else out[(i - na) + lower_bound_u64(a, na, b[i - na])] = b[i - na];
    }
}

// a leaf goes: its keep flag is clear (the ordered selection of their indices)
// the leaves that stay / go, read straight from the decision flags
struct Kept {
    __host__ __device__ bool operator()(uint32_t f) const { return (f & RF_GONE) == 0; }
};
struct Gone {
    __host__ __device__ bool operator()(uint32_t f) const { return (f & RF_GONE) != 0; }
};

// new = (old without the leaves at `gone`, ascending) merged with `added`
// (ascending, disjoint from the kept leaves), on the host threads: each takes a run of
// the old list, the new ids in its id range, and writes at its place
static void merge_leaves_host(const std::vector<uint64_t>& old, const std::vector<uint32_t>& gone,
                              const std::vector<uint64_t>& added, std::vector<uint64_t>& out)
{
    const size_t N = old.size(), na = added.size();
    out.resize(N - gone.size() + na);
    if (!N) {
        std::copy(added.begin(), added.end(), out.begin());
        return;
    }
    const size_t nt = std::max<size_t>(1, std::min<size_t>(host_threads(), (N + (1u << 16) - 1) >> 16));
    const size_t per = (N + nt - 1) / nt;
    auto job = [&](size_t t) {
        const size_t b = std::min(N, t * per), e = std::min(N, b + per);
        if (b >= e) return;  // the run ending at N takes the new ids above the last old one
        // new ids below this run's first old id belong to it (all of them to run 0)
        const size_t a0 = t == 0 ? 0 : (size_t)(std::lower_bound(added.begin(), added.end(), old[b]) - added.begin());
        const size_t a1 = e >= N ? na : (size_t)(std::lower_bound(added.begin(), added.end(), old[e]) - added.begin());
        const size_t g0 = (size_t)(std::lower_bound(gone.begin(), gone.end(), (uint32_t)b) - gone.begin());
        size_t w = (b - g0) + a0, gi = g0, ai = a0;
        for (size_t i = b; i < e; i++) {
            if (gi < gone.size() && gone[gi] == i) {
                gi++;
                continue;
            }
            while (ai < a1 && added[ai] < old[i]) out[w++] = added[ai++];
            out[w++] = old[i];
        }
        while (ai < a1) out[w++] = added[ai++];
    };
    if (nt == 1) job(0);
    else pool_run(nt, job);
}

// four id lists into one array of sort keys, list k tagged k above the ids' bits
struct TagLists {
    const uint64_t* in[4];
    uint32_t n[4];
    int bits;
};

__global__ void __launch_bounds__(256) k_tag_lists(TagLists t, uint64_t* __restrict__ keys)
{
    const uint64_t tot = (uint64_t)t.n[0] + t.n[1] + t.n[2] + t.n[3];
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += stride) {
        uint64_t j = i;
        int k = 0;
        while (k < 3 && j >= t.n[k]) j -= t.n[k++];
        keys[i] = (t.bits < 64 ? (uint64_t)k << t.bits : 0) | t.in[k][j];
    }
}

static unsigned blocks(uint64_t n, unsigned cap = 4096)
{
    uint64_t g = (n + 255) / 256;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, cap));
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

// stream-ordered scratch of one call, freed in one go
struct Scratch {
    hipStream_t st;
    std::vector<void*> v;
    explicit Scratch(hipStream_t s) : st(s) {}
    template <class T>
    int get(T** p, size_t count)
    {
        *p = nullptr;
        DX_HIP(ds_malloc(p, std::max<size_t>(count, 1) * sizeof(T), st));
        v.push_back(*p);
        return DCCRGX_OK;
    }
    ~Scratch()
    {
        for (void* p : v) ds_free(p, st);
    }
};

static AView aview(const dccrgx_grid* grid, uint32_t* flags)
{
    const Explicit* E = grid->ex;
    const Hood& h = grid->hoods.at(DCCRGX_DEFAULT_NEIGHBORHOOD_ID);
    AView a{};
    a.v = explicit_view(grid);
    a.leaves = E->d_leaves;
    a.n = E->n;
    a.nof_row = h.d_nof_row;
    a.nof_g = h.d_nof_g;
    a.nto_row = h.d_nto_row;
    a.nto_g = h.d_nto_g;
    a.slot_of_g = E->d_slot_of_g;
    a.rows_all = h.n_rows == E->n && E->slot_identity ? 1 : 0;
    a.items = h.d_of_c;
    a.items_to = h.d_to_c;
    a.K = h.K;
    a.hood_len = grid->params.neighborhood_length;
    a.part = E->part;
    a.sfc = SfcCuts{};
    if (grid->sfc.on()) a.sfc = grid->sfc.view(grid->d_sfc_cut);
    a.rank = grid->ctx->rank;
    a.flags = flags;
    return a;
}

// the flags over the current leaves from the host sets (when the host has
// the newer state)
int amr_dev_sync(dccrgx_grid* grid)
{
    Amr& A = *grid->amr;
    Explicit* E = grid->ex;
    hipStream_t st = grid->ctx->compute;
    if (grid->sfc.on() && !grid->d_sfc_cut) {  // P - 1 cut keys
        const size_t bytes = std::max<size_t>(8, grid->sfc.cut.size() * 8);
        DX_HIP(dx_malloc(&grid->d_sfc_cut, bytes));
        if (!grid->sfc.cut.empty())
            DX_TRY(dx_h2d(grid->ctx, grid->d_sfc_cut, grid->sfc.cut.data(), grid->sfc.cut.size() * 8, st));
    }
    if (A.dev_current && A.flags_n == E->n && A.d_flags) return DCCRGX_OK;
    if (A.flags_cap < E->n) {
        ds_free(A.d_flags, st);
        A.flags_cap = E->n + E->n / 8 + 64;
        DX_HIP(ds_malloc(&A.d_flags, A.flags_cap * 4, st));
    }
    A.flags_n = E->n;
    DX_HIP(hipMemsetAsync(A.d_flags, 0, E->n * 4, st));
    std::vector<uint64_t> ids;
    std::vector<uint32_t> bits;
    const std::pair<const FlatSet*, uint32_t> sets[4] = {
        {&A.to_refine, RF_REFINE}, {&A.not_to_refine, RF_NOT_REFINE}, {&A.to_unrefine, RF_UNREFINE},
        {&A.not_to_unrefine, RF_NOT_UNREFINE}};
    for (const auto& s : sets)
        for (uint64_t c : *s.first) {
            ids.push_back(c);
            bits.push_back(s.second);
        }
    A.nr_other.clear();
    if (!ids.empty()) {
        Scratch S(st);
        uint64_t *d_ids, *d_other;
        uint32_t *d_bits, *d_cnt;
        DX_TRY(S.get(&d_ids, ids.size()));
        DX_TRY(S.get(&d_bits, bits.size()));
        DX_TRY(S.get(&d_other, ids.size()));
        DX_TRY(S.get(&d_cnt, 1));
        DX_HIP(hipMemsetAsync(d_cnt, 0, 4, st));
        DX_TRY(dx_h2d_async(grid->ctx, d_ids, ids.data(), ids.size() * 8, st));
        DX_TRY(dx_h2d_async(grid->ctx, d_bits, bits.data(), bits.size() * 4, st));
        hipLaunchKernelGGL(k_flags_scatter, dim3(blocks(ids.size())), dim3(256), 0, st, aview(grid, A.d_flags), d_ids,
                           d_bits, (uint64_t)ids.size(), d_other, d_cnt);
        DX_HIP(hipGetLastError());
        uint32_t no = 0;
        DX_TRY(dx_d2h(grid->ctx, &no, d_cnt, 4, st));
        A.nr_other.resize(no);
        if (no) DX_TRY(dx_d2h(grid->ctx, A.nr_other.data(), d_other, no * 8ull, st));
    }
    A.dev_current = true;
    A.dev_unrefines = !A.to_unrefine.empty();
    return DCCRGX_OK;
}

// the host sets from the flags (when the device has the newer state)
int amr_host_sync(dccrgx_grid* grid)
{
    Amr& A = *grid->amr;
    if (A.host_current) return DCCRGX_OK;
    hipStream_t st = grid->ctx->compute;
    Scratch S(st);
    uint64_t* d_ids;
    uint32_t *d_bits, *d_cnt;
    DX_TRY(S.get(&d_ids, A.flags_n));
    DX_TRY(S.get(&d_bits, A.flags_n));
    DX_TRY(S.get(&d_cnt, 1));
    DX_HIP(hipMemsetAsync(d_cnt, 0, 4, st));
    hipLaunchKernelGGL(k_flags_gather, dim3(blocks(A.flags_n)), dim3(256), 0, st, aview(grid, A.d_flags), d_ids,
                       d_bits, d_cnt);
    DX_HIP(hipGetLastError());
    uint32_t n = 0;
    DX_TRY(dx_d2h(grid->ctx, &n, d_cnt, 4, st));
    std::vector<uint64_t> ids(n);
    std::vector<uint32_t> bits(n);
    if (n) {
        DX_TRY(dx_d2h(grid->ctx, ids.data(), d_ids, n * 8ull, st));
        DX_TRY(dx_d2h(grid->ctx, bits.data(), d_bits, n * 4ull, st));
    }
    A.to_refine.clear();
    A.not_to_refine.clear();
    A.to_unrefine.clear();
    A.not_to_unrefine.clear();
    for (uint32_t i = 0; i < n; i++) {
        if (bits[i] & RF_REFINE) A.to_refine.insert(ids[i]);
        if (bits[i] & RF_NOT_REFINE) A.not_to_refine.insert(ids[i]);
        if (bits[i] & RF_UNREFINE) A.to_unrefine.insert(ids[i]);
        if (bits[i] & RF_NOT_UNREFINE) A.not_to_unrefine.insert(ids[i]);
    }
    for (uint64_t c : A.nr_other) A.not_to_refine.insert(c);
    A.host_current = true;
    return DCCRGX_OK;
}

// a batch of request calls of one kind in call order (explicit grids)
int amr_dev_requests(dccrgx_grid* grid, int32_t kind, const uint64_t* ids, size_t n, int32_t* results)
{
    return amr_dev_requests_ex(grid, kind, ids, nullptr, n, results);
}

// ids on the host, or dev_ids already on the device (stream-ordered on the
// compute stream: the adaptation lists of dccrgx_advect_adapt_requests)
int amr_dev_requests_ex(dccrgx_grid* grid, int32_t kind, const uint64_t* ids, const uint64_t* dev_ids, size_t n,
                        int32_t* results)
{
    return amr_dev_requests_many(grid, 1, &kind, &ids, &dev_ids, &n, &results);
}

// several request batches in call order: their scratch cleared by one fill
// and their results read back behind one synchronisation (each batch's
// kernels follow the previous batch's on the stream, as separate calls do)
int amr_dev_requests_many(dccrgx_grid* grid, int nk, const int32_t* kinds, const uint64_t* const* ids,
                          const uint64_t* const* dev_ids, const size_t* counts, int32_t* const* results)
{
    Amr& A = *grid->amr;
    DX_TRY(amr_dev_sync(grid));
    DX_CHECK(nk >= 0 && nk <= 3, DCCRGX_EINTERNAL, "%d request batches", nk);
    hipStream_t st = grid->ctx->compute;
    const AView a = aview(grid, A.d_flags);
    Scratch S(st);
    struct Batch {
        uint64_t *ids = nullptr, *du = nullptr;
        int32_t* res = nullptr;
        uint32_t *grp = nullptr, *key = nullptr, *ord = nullptr, *dun = nullptr;
    } B[3];
    Fill z[8];
    int nz = 0;
    for (int k = 0; k < nk; k++) {
        const size_t n = counts[k];
        if (!n) continue;
        Batch& b = B[k];
        if (dev_ids && dev_ids[k]) {
            b.ids = const_cast<uint64_t*>(dev_ids[k]);
        } else {
            DX_TRY(S.get(&b.ids, n));
            DX_TRY(dx_h2d_async(grid->ctx, b.ids, ids[k], n * 8, st));
        }
        if (results && results[k]) DX_TRY(S.get(&b.res, n));
        DX_TRY(S.get(&b.grp, a.n));
        DX_TRY(S.get(&b.key, n));
        z[nz++] = Fill{b.grp, a.n * 4, 0xff};
        if (kinds[k] == DCCRGX_AMR_REFINE) {
            DX_TRY(S.get(&b.du, n));
            DX_TRY(S.get(&b.ord, n));
            DX_TRY(S.get(&b.dun, 1));
            z[nz++] = Fill{b.dun, 4, 0};
        }
    }
    DX_TRY(dx_fill_many(z, nz, st));
    std::vector<D2H> back;
    for (int k = 0; k < nk; k++) {
        const size_t n = counts[k];
        if (!n) continue;
        const Batch& b = B[k];
        const unsigned bl = blocks(n), bw = blocks(64 * (uint64_t)n);  // a thread / a wave per request
        if (kinds[k] == DCCRGX_AMR_UNREFINE) A.dev_unrefines = true;
        const int erase = A.dev_unrefines ? 1 : 0;
        switch (kinds[k]) {
        case DCCRGX_AMR_REFINE:
            hipLaunchKernelGGL(k_req_refine, dim3(bw), dim3(256), 0, st, a, (const uint64_t*)b.ids, (uint64_t)n,
                               b.res, b.du, b.ord, b.dun, erase);
            hipLaunchKernelGGL(k_req_du_a, dim3(bl), dim3(256), 0, st, a, (const uint64_t*)b.du,
                               (const uint32_t*)b.ord, (const uint32_t*)b.dun, (uint64_t)0, (int32_t*)nullptr, b.grp,
                               b.key);
            hipLaunchKernelGGL(k_req_du_b, dim3(bl), dim3(256), 0, st, a, (const uint64_t*)b.du,
                               (const uint32_t*)b.ord, (const uint32_t*)b.dun, (uint64_t)0, (const uint32_t*)b.grp,
                               (const uint32_t*)b.key, erase);
            break;
        case DCCRGX_AMR_DONT_UNREFINE:
            hipLaunchKernelGGL(k_req_du_a, dim3(bl), dim3(256), 0, st, a, (const uint64_t*)b.ids,
                               (const uint32_t*)nullptr, (const uint32_t*)nullptr, (uint64_t)n, b.res, b.grp, b.key);
            hipLaunchKernelGGL(k_req_du_b, dim3(bl), dim3(256), 0, st, a, (const uint64_t*)b.ids,
                               (const uint32_t*)nullptr, (const uint32_t*)nullptr, (uint64_t)n,
                               (const uint32_t*)b.grp, (const uint32_t*)b.key, erase);
            break;
        case DCCRGX_AMR_UNREFINE:
        {
            const unsigned bu = blocks((uint64_t)n * (a.K <= 8 ? 8 : a.K <= 16 ? 16 : a.K <= 32 ? 32 : 64));
            if (a.K <= 8)
                hipLaunchKernelGGL(k_req_unref_a<8>, dim3(bu), dim3(256), 0, st, a, (const uint64_t*)b.ids,
                                   (uint64_t)n, b.res, b.grp, b.key);
            else if (a.K <= 16)
                hipLaunchKernelGGL(k_req_unref_a<16>, dim3(bu), dim3(256), 0, st, a, (const uint64_t*)b.ids,
                                   (uint64_t)n, b.res, b.grp, b.key);
            else if (a.K <= 32)
                hipLaunchKernelGGL(k_req_unref_a<32>, dim3(bu), dim3(256), 0, st, a, (const uint64_t*)b.ids,
                                   (uint64_t)n, b.res, b.grp, b.key);
            else
                hipLaunchKernelGGL(k_req_unref_a<64>, dim3(bu), dim3(256), 0, st, a, (const uint64_t*)b.ids,
                                   (uint64_t)n, b.res, b.grp, b.key);
        }
            hipLaunchKernelGGL(k_req_unref_b, dim3(bl), dim3(256), 0, st, a, (const uint64_t*)b.ids, (uint64_t)n,
                               (const uint32_t*)b.grp, (const uint32_t*)b.key);
            break;
        default:
            hipLaunchKernelGGL(k_req_dont_refine, dim3(bl), dim3(256), 0, st, a, (const uint64_t*)b.ids, (uint64_t)n,
                               b.res);
            break;
        }
        DX_HIP(hipGetLastError());
        if (b.res) back.push_back(D2H{results[k], b.res, n * 4});
    }
    if (!back.empty()) DX_TRY(dx_d2h_many(grid->ctx, back.data(), back.size(), st));
    A.host_current = false;
    return DCCRGX_OK;
}

// override_refines, induce_refines and override_unrefines on the flags, then
// the new leaf list (device, ascending, its first leaf, and with several
// ranks its host copy -- left empty on one rank), this rank's new /
// removed cells (A.new_cells / A.removed) and retired cells (ascending), and
// the dont_refine ids that persist (`nr`).  The grid is not changed; the
// flags hold the decisions afterwards (the caller restores them if the
// rebuild fails).
int amr_dev_decide(dccrgx_grid* grid, uint64_t** d_leaves_out, uint64_t* n_out, uint64_t* first_out,
                   std::vector<uint64_t>& leaves_host,
                   std::vector<uint64_t>& retired, std::vector<uint64_t>& nr, bool* changed)
{
    Amr& A = *grid->amr;
    DX_TRY(amr_dev_sync(grid));
    Ctx* ctx = grid->ctx;
    hipStream_t st = ctx->compute;
    const AView a = aview(grid, A.d_flags);
    const uint64_t N = a.n;
    const int M = grid->map.max_lvl;
    Scratch S(st);
    PhaseTimer T("amr_dev_decide");
    // counters: [0..M+1] frontier sizes of a spread, then the same again
    uint32_t *d_cnt, *d_fa, *d_fb, *d_grp, *d_key;
    const int NC = 2 * (M + 2) + 10;  // ..., gone count (NC - 3), error (NC - 2), retries (NC - 1)
    DX_TRY(S.get(&d_cnt, NC));
    DX_TRY(S.get(&d_fa, N));
    DX_TRY(S.get(&d_fb, N));
    DX_TRY(S.get(&d_grp, N));
    DX_TRY(S.get(&d_key, N));
    {
        const Fill z[2] = {{d_cnt, (size_t)NC * 4, 0}, {d_grp, N * 4, 0xff}};
        DX_TRY(dx_fill_many(z, 2, st));
    }
    const unsigned bN = blocks(N);
    // override_refines then induce_refines: at most M rounds each
    for (int phase = 0; phase < 2; phase++) {
        const uint32_t bit = phase == 0 ? RF_NOT_REFINE : RF_REFINE;
        uint32_t* c = d_cnt + phase * (M + 2);
        hipLaunchKernelGGL(k_collect, dim3(bN), dim3(256), 0, st, a, bit, d_fa, c);
        uint32_t *f = d_fa, *nx = d_fb;
        for (int r = 0; r < M; r++) {
            if (a.rows_all)
                hipLaunchKernelGGL(k_spread_rows, dim3(blocks(64 * N, 1024)), dim3(256), 0, st, a, bit, phase == 0 ? 1 : 0,
                                   (const uint32_t*)f, (const uint32_t*)(c + r), nx, c + r + 1);
            else
                hipLaunchKernelGGL(k_spread, dim3(bN), dim3(256), 0, st, a, bit, phase == 0 ? 1 : 0, (const uint32_t*)f,
                                   (const uint32_t*)(c + r), nx, c + r + 1);
            std::swap(f, nx);
        }
    }
    // refines of dont_refine cells were dropped by the second k_collect
    // override_unrefines
    uint32_t* cu = d_cnt + 2 * (M + 2);
    hipLaunchKernelGGL(k_collect, dim3(bN), dim3(256), 0, st, a, RF_UNREFINE, d_fa, cu);
    uint32_t* d_lkey;  // per leaf, read only at the unrefine requests
    DX_TRY(S.get(&d_lkey, N));
    hipLaunchKernelGGL(k_ou_group, dim3(bN), dim3(256), 0, st, a, (const uint32_t*)d_fa, (const uint32_t*)cu, d_grp,
                       d_key, d_lkey);
    int32_t* d_err = (int32_t*)(d_cnt + NC - 2);  // zeroed with the counters (walk overflow)
    if (!test_opt(OPT_OU_WALK, 0)) {
        hipLaunchKernelGGL(k_ou_check, dim3(blocks(64 * N, 2048)), dim3(256), 0, st, a, (const uint32_t*)d_fa,
                           (const uint32_t*)cu, (const uint32_t*)d_grp, (const uint32_t*)d_key);
    } else {
        // the walks: first with a small LDS workspace (a walk visits tens of
        // cells; many waves per CU), the few that overflow it again with one
        // sized for the largest possible closure
        const uint32_t hl = grid->params.neighborhood_length;
        const uint64_t P = 8ull * (2 * hl + 3) * (2 * hl + 3) * (2 * hl + 3);
        const uint32_t Q = (uint32_t)(6 * P + 8);
        uint32_t Sz = 16;
        while (Sz < 2 * Q) Sz <<= 1;
        const size_t ws = (size_t)(Q + Sz) * 8;
        const bool lds = ws <= 48 * 1024;
        const unsigned waves = lds ? 4096 : 1024;
        uint64_t* d_scr = nullptr;
        if (!lds) DX_TRY(S.get(&d_scr, (size_t)waves * (Q + Sz)));
        uint32_t *d_retry, *d_nretry = d_cnt + NC - 1;
        DX_TRY(S.get(&d_retry, N));
        // DCCRGX_OU_SMALL (tests): the first pass's queue length, to send walks to the second pass
        const uint32_t Q1 = (uint32_t)std::max<int64_t>(2, test_opt(OPT_OU_SMALL, 256));
        uint32_t S1 = 16;
        while (S1 < 2 * Q1) S1 <<= 1;  // 256 -> 512: 6 KiB per wave
        if (Q1 < Q && (size_t)(Q1 + S1) * 8 <= 48 * 1024) {
            hipLaunchKernelGGL(k_ou_walk, dim3(8192), dim3(64), (Q1 + S1) * 8, st, a, (const uint32_t*)d_fa,
                               (const uint32_t*)cu, (const uint32_t*)nullptr, (const uint32_t*)nullptr,
                               (const uint32_t*)d_grp, (const uint32_t*)d_key, Q1, S1, 1, (uint64_t*)nullptr, d_retry,
                               d_nretry, d_err);
            hipLaunchKernelGGL(k_ou_walk, dim3(waves), dim3(64), lds ? ws : 0, st, a, (const uint32_t*)d_fa,
                               (const uint32_t*)cu, (const uint32_t*)d_retry, (const uint32_t*)d_nretry,
                               (const uint32_t*)d_grp, (const uint32_t*)d_key, Q, Sz, lds ? 1 : 0, d_scr,
                               (uint32_t*)nullptr, (uint32_t*)nullptr, d_err);
        } else {
            hipLaunchKernelGGL(k_ou_walk, dim3(waves), dim3(64), lds ? ws : 0, st, a, (const uint32_t*)d_fa,
                               (const uint32_t*)cu, (const uint32_t*)nullptr, (const uint32_t*)nullptr,
                               (const uint32_t*)d_grp, (const uint32_t*)d_key, Q, Sz, lds ? 1 : 0, d_scr,
                               (uint32_t*)nullptr, (uint32_t*)nullptr, d_err);
        }
    }
    // execute_refines (with override_unrefines' outcome and the persisting
    // dont_refine ids)
    ExecOut o;
    DX_TRY(S.get(&o.added, 8 * N + 8));
    DX_TRY(S.get(&o.newc, 8 * N + 8));
    DX_TRY(S.get(&o.removed, 8 * N + 8));
    DX_TRY(S.get(&o.retired, 9 * N + 8));
    DX_TRY(S.get(&o.nr, N));
    uint64_t* d_nr = o.nr;
    o.cnt = d_cnt + 2 * (M + 2) + 1;  // 5 counters
    hipLaunchKernelGGL(k_exec, dim3(bN), dim3(256), 0, st, a, (const uint32_t*)d_grp, (const uint32_t*)d_lkey, o);
    DX_HIP(hipGetLastError());
    uint32_t cnt[6] = {0, 0, 0, 0, 0, 0};
    int32_t err = 0;
    const D2H first[2] = {{&err, d_err, 4}, {cnt, o.cnt, 5 * 4}};
    DX_TRY(dx_d2h_many(ctx, first, 2, st));
    T.lap("decisions");
    DX_CHECK(!err, DCCRGX_EINTERNAL, "override_unrefines walk exceeded its workspace");
    // the persisting dont_refine set (flagged leaves, and the ids that are not
    // leaves) and this rank's new / removed / retired cells
    nr.resize(cnt[4]);
    A.new_cells.resize(cnt[1]);
    A.removed.resize(cnt[2]);
    retired.resize(cnt[3]);
    *changed = cnt[0] > 0;
    T.lap("lists");
    if (!*changed) {  // one read-back, sorted on the host threads
        const D2H lists[4] = {{nr.data(), d_nr, cnt[4] * 8ull},
                              {A.new_cells.data(), o.newc, cnt[1] * 8ull},
                              {A.removed.data(), o.removed, cnt[2] * 8ull},
                              {retired.data(), o.retired, cnt[3] * 8ull}};
        DX_TRY(dx_d2h_many(ctx, lists, 4, st));
        nr.insert(nr.end(), A.nr_other.begin(), A.nr_other.end());
        std::vector<uint64_t>* lv[3] = {&A.new_cells, &A.removed, &retired};
        const size_t nt = std::min<size_t>(3, host_threads());
        pool_run(nt, [&](size_t t) {
            for (size_t k = t; k < 3; k += nt) {
                std::vector<uint64_t>& v = *lv[k];
                radix_sort_u64(v);
                v.erase(std::unique(v.begin(), v.end()), v.end());
            }
        });
        return DCCRGX_OK;
    }
    // the new leaf list: surviving leaves in order, merged with the sorted new ones
    uint64_t *d_kept, *d_cnt64;
    DX_TRY(S.get(&d_kept, N));
    DX_TRY(S.get(&d_cnt64, 2));
    // the new ids and the new / removed / retired lists sorted on the device
    // (the host would sort them while the device waits) in one radix sort:
    // each list tagged in the two bits above the ids' bits, so the sorted
    // keys are the four lists one after the other; the three lists are
    // untagged and unique-d on the host after the read-back
    int bits = 1;  // ids are at most last_cell: sort only their bits
    while (bits < 64 && (grid->map.last_cell >> bits)) bits++;
    // (ids of more than 62 bits leave no room for the tags: the four lists
    // are then sorted one by one into the same places)
    const bool tagged = bits <= 62;
    const int sort_bits = tagged ? bits + 2 : bits;
    const uint64_t n_all = (uint64_t)cnt[0] + cnt[1] + cnt[2] + cnt[3];
    uint64_t *d_keys, *d_all;
    DX_TRY(S.get(&d_keys, std::max<uint64_t>(n_all, 1)));
    DX_TRY(S.get(&d_all, std::max<uint64_t>(n_all, 1)));
    TagLists tl{{o.added, o.newc, o.removed, o.retired}, {cnt[0], cnt[1], cnt[2], cnt[3]}, tagged ? bits : 64};
    if (n_all) hipLaunchKernelGGL(k_tag_lists, dim3(blocks(n_all)), dim3(256), 0, st, tl, d_keys);
    const uint64_t off_ls[3] = {cnt[0], (uint64_t)cnt[0] + cnt[1], (uint64_t)cnt[0] + cnt[1] + cnt[2]};
    const uint64_t off4[5] = {0, off_ls[0], off_ls[1], off_ls[2], n_all};
    // the indices of the leaves that go, ascending: a selection over the
    // leaf indices (the host merge needs them in order)
    uint32_t* d_gone;
    DX_TRY(S.get(&d_gone, N));
    uint32_t* d_ngone = d_cnt + NC - 3;
    const hipcub::TransformInputIterator<bool, Kept, const uint32_t*> d_keep(a.flags, Kept{});
    const hipcub::CountingInputIterator<uint32_t> leaf_idx(0);
    const hipcub::TransformInputIterator<bool, Gone, const uint32_t*> gone_flags(a.flags, Gone{});
    size_t tb[4] = {0, 0, 0, 0};
    DX_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb[0], a.leaves, d_keep, d_kept, d_cnt64, (int)N, st));
    DX_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tb[1], d_keys, d_all, (int)n_all, 0, sort_bits, st));
    DX_HIP(hipcub::DeviceSelect::Unique(nullptr, tb[2], d_all, o.added, d_cnt64 + 1, (int)cnt[0], st));
    DX_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb[3], leaf_idx, gone_flags, d_gone, d_ngone, (int)N, st));
    const size_t tmax = *std::max_element(tb, tb + 4);
    uint8_t* d_tmp;
    DX_TRY(S.get(&d_tmp, std::max<size_t>(tmax, 1)));
    size_t t = tmax;
    DX_HIP(hipcub::DeviceSelect::Flagged(d_tmp, t, a.leaves, d_keep, d_kept, d_cnt64, (int)N, st));
    t = tmax;
    if (tagged && n_all) {
        DX_HIP(hipcub::DeviceRadixSort::SortKeys(d_tmp, t, d_keys, d_all, (int)n_all, 0, sort_bits, st));
    } else {
        for (int k = 0; k < 4; k++) {
            const uint64_t nk = off4[k + 1] - off4[k];
            if (!nk) continue;
            t = tmax;
            DX_HIP(hipcub::DeviceRadixSort::SortKeys(d_tmp, t, d_keys + off4[k], d_all + off4[k], (int)nk, 0,
                                                     sort_bits, st));
        }
    }
    t = tmax;
    DX_HIP(hipcub::DeviceSelect::Unique(d_tmp, t, d_all, o.added, d_cnt64 + 1, (int)cnt[0], st));
    t = tmax;
    if (grid->ctx->comm_size > 1)  // for the host merge
        DX_HIP(hipcub::DeviceSelect::Flagged(d_tmp, t, leaf_idx, gone_flags, d_gone, d_ngone, (int)N, st));
    // the merge reads both counts on the device, into a list sized for the
    // most leaves there can be
    const uint64_t n_max = N + cnt[0];
    uint64_t* d_new = nullptr;
    DX_HIP(ds_malloc(&d_new, std::max<uint64_t>(n_max, 1) * 8, st));
    hipLaunchKernelGGL(k_merge, dim3(blocks(n_max)), dim3(256), 0, st, (const uint64_t*)d_kept,
                       (const uint64_t*)d_cnt64, (const uint64_t*)o.added, (const uint64_t*)(d_cnt64 + 1), d_new);
    DX_HIP(hipGetLastError());
    T.lap("kept + sorted new");
    // several ranks: the host's copy of the new list is merged on the host
    // from its copy of the old one, the gone leaves and the new ids -- small
    // lists instead of the whole list over PCIe (28 MB at 3.5 M leaves, 0.5 ms
    // of copy plus the staging copy).  One rank keeps the list on the device
    // only (Explicit::leaves() fetches it if host code asks).
    const bool host_list = grid->ctx->comm_size > 1;
    uint64_t nk[2] = {0, 0}, first_leaf = 0;
    uint32_t ngone = 0;
    int e = DCCRGX_OK;
    const D2H c2[3] = {{nk, d_cnt64, 16}, {&ngone, d_ngone, 4}, {&first_leaf, d_new, 8}};
    const D2H l1[4] = {{nr.data(), d_nr, cnt[4] * 8ull},
                       {A.new_cells.data(), d_all + off_ls[0], cnt[1] * 8ull},
                       {A.removed.data(), d_all + off_ls[1], cnt[2] * 8ull},
                       {retired.data(), d_all + off_ls[2], cnt[3] * 8ull}};
    if (!host_list) {  // one rank: the counts and the lists (sized by the first read-back) in one read-back
        D2H all[7];
        std::copy(c2, c2 + 3, all);
        std::copy(l1, l1 + 4, all + 3);
        e = dx_d2h_many(ctx, all, 7, st);
    } else {
        e = dx_d2h_many(ctx, c2, 3, st);
    }
    std::vector<uint64_t> added(host_list ? nk[1] : 0);
    std::vector<uint32_t> gone(host_list ? ngone : 0);
    if (e == DCCRGX_OK && host_list) {
        const D2H l2[6] = {{nr.data(), d_nr, cnt[4] * 8ull},
                           {A.new_cells.data(), d_all + off_ls[0], cnt[1] * 8ull},
                           {A.removed.data(), d_all + off_ls[1], cnt[2] * 8ull},
                           {retired.data(), d_all + off_ls[2], cnt[3] * 8ull},
                           {added.data(), o.added, added.size() * 8},
                           {gone.data(), d_gone, gone.size() * 4}};
        e = dx_d2h_many(ctx, l2, 6, st);
    }
    if (e != DCCRGX_OK) {
        ds_free(d_new, st);
        return e;
    }
    T.lap("lists read back");
    nr.insert(nr.end(), A.nr_other.begin(), A.nr_other.end());
    const uint64_t id_mask = tagged ? (1ull << bits) - 1 : ~0ull;
    for (std::vector<uint64_t>* v : {&A.new_cells, &A.removed, &retired}) {
        for (uint64_t& x : *v) x &= id_mask;  // the sort's list tags
        v->erase(std::unique(v->begin(), v->end()), v->end());
    }
    const uint64_t n_new = nk[0] + nk[1];
    leaves_host.clear();
    if (host_list) {
        merge_leaves_host(grid->ex->leaves(), gone, added, leaves_host);
        DX_CHECK(leaves_host.size() == n_new, DCCRGX_EINTERNAL, "host leaf list %zu, device %llu",
                 leaves_host.size(), (unsigned long long)n_new);
    }
    T.lap("new leaf list");
    *d_leaves_out = d_new;
    *n_out = n_new;
    *first_out = first_leaf;
    return DCCRGX_OK;
}

// ---------------------------------------------------------------------------
// data of new / removed cells, adaptation sets
// ---------------------------------------------------------------------------

// storage slot of a leaf, or of a cell retired by the last rebuild (its
// table: ids ascending, then their slots), -1 if none
struct SlotView {
    ExView v;
    const uint32_t* slot_of_g;
    const uint64_t* ret;   // retired ids ascending, then their slots (RET_REMOVED set for removed cells)
    uint64_t n_ret;
    const uint64_t* hkey;  // id -> slot table of the retired cells (hcap keys, then hcap slots)
    uint64_t hmask;        // hcap - 1
};

__host__ __device__ inline uint64_t ret_hash(uint64_t id)  // splitmix64 finaliser
{
    id ^= id >> 31;
    id *= 0x7fb5d329728ea185ull;
    id ^= id >> 27;
    id *= 0x81dadef4bc2dd44dull;
    return id ^ (id >> 33);
}

// the table's value of a retired cell: its slot, with RET_REMOVED set if the
// cell is one of the removed cells (a child of an unrefined parent, not a
// refined leaf); ~0 if the id is not retired
constexpr uint64_t RET_REMOVED = 1ull << 63;
__device__ inline uint64_t ret_entry(const SlotView& s, uint64_t id)
{
    if (!s.n_ret) return ~0ull;
    for (uint64_t h = ret_hash(id) & s.hmask;; h = (h + 1) & s.hmask) {
        const uint64_t k = s.hkey[h];
        if (k == id) return s.hkey[s.hmask + 1 + h];
        if (k == 0) return ~0ull;
    }
}

// slot of a retired cell, -1 if it is not one
__device__ inline int64_t ret_slot(const SlotView& s, uint64_t id)
{
    const uint64_t e = ret_entry(s, id);
    return e == ~0ull ? -1 : (int64_t)(e & ~RET_REMOVED);
}

__device__ inline int64_t slot_lookup(const SlotView& s, uint64_t id)
{
    const int64_t g = ex_find(s.v, id);
    if (g >= 0) {
        const uint32_t x = s.slot_of_g[g];
        return x == NO_SLOT ? -1 : (int64_t)x;
    }
    return ret_slot(s, id);
}

static SlotView slot_view(const dccrgx_grid* grid)
{
    const Explicit* E = grid->ex;
    const uint64_t* hk = E->d_ret ? E->d_ret + 2 * E->n_ret : nullptr;
    return SlotView{explicit_view(grid), E->d_slot_of_g, E->d_ret, E->n_ret, hk, E->ret_hcap ? E->ret_hcap - 1 : 0};
}

// the retired cells' table on the device: ids ascending, then their slots
// (the removed cells marked), then the hash (hcap keys, hcap values) filled
// by one insertion kernel -- the host only lists the ids and slots (the
// table itself was 16 B per hash entry zeroed, filled and uploaded by the
// host: ~0.5 ms at 77k retired cells)
__global__ void __launch_bounds__(256) k_ret_insert(const uint64_t* __restrict__ ids, const uint64_t* __restrict__ val,
                                                    uint64_t n, unsigned long long* __restrict__ hk,
                                                    uint64_t* __restrict__ hv, uint64_t mask)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t id = ids[i];
        for (uint64_t h = ret_hash(id) & mask;; h = (h + 1) & mask) {
            const unsigned long long prev = atomicCAS(&hk[h], 0ull, (unsigned long long)id);
            if (prev == 0ull || prev == id) {
                hv[h] = val[i];
                break;
            }
        }
    }
}

int amr_dev_retired_table(dccrgx_grid* grid)
{
    Explicit* E = grid->ex;
    const uint64_t n = E->retired.size();
    E->n_ret = 0;
    E->ret_hcap = 0;
    if (!n) return DCCRGX_OK;
    uint64_t cap = 64;
    while (cap < 2 * n) cap <<= 1;  // load factor <= 1/2
    std::vector<uint64_t> t(2 * n);
    // the removed cells among them (both lists ascending): marked in the table
    static const std::vector<uint64_t> none;
    const std::vector<uint64_t>& rem = grid->amr ? grid->amr->removed : none;
    size_t r = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t id = E->retired[i], slot = E->ret_slot0 + i;
        while (r < rem.size() && rem[r] < id) r++;
        const bool removed = r < rem.size() && rem[r] == id;
        t[i] = id;
        t[n + i] = slot | (removed ? RET_REMOVED : 0);
    }
    hipStream_t st = grid->ctx->compute;
    ds_free(E->d_ret, st);
    E->d_ret = nullptr;
    DX_HIP(ds_malloc(&E->d_ret, (2 * n + 2 * cap) * 8, st));
    uint64_t* hk = E->d_ret + 2 * n;
    const Fill z[1] = {{hk, cap * 8, 0}};
    DX_TRY(dx_fill_many(z, 1, st));
    DX_TRY(dx_h2d_async(grid->ctx, E->d_ret, t.data(), t.size() * 8, st));
    hipLaunchKernelGGL(k_ret_insert, dim3(blocks(n)), dim3(256), 0, st, (const uint64_t*)E->d_ret,
                       (const uint64_t*)(E->d_ret + n), n, (unsigned long long*)hk, hk + cap, cap - 1);
    DX_HIP(hipGetLastError());
    E->n_ret = n;
    E->ret_hcap = cap;
    return DCCRGX_OK;
}

struct FieldSet {
    uint8_t* p[8];
    uint32_t elem[8];
    int n;
};

// adapter.hpp:229-251: a new cell takes its parent's data
__global__ void __launch_bounds__(256) k_copy_from_parents(SlotView sv, MapParams mp, const uint64_t* __restrict__ cells,
                                                           uint64_t n, FieldSet fs, int32_t* __restrict__ err)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t c = cells[i];
        uint64_t idx[3];
        int l;
        map_indices(mp, c, idx, &l);
        const uint64_t par = l > 0 ? map_cell(mp, idx, l - 1) : c;
        const int64_t dst = slot_lookup(sv, c), src = slot_lookup(sv, par);
        if (dst < 0 || src < 0) {
            atomicOr(err, 1);
            continue;
        }
        for (int k = 0; k < fs.n; k++) {
            const uint32_t e = fs.elem[k];
            const uint8_t* a = fs.p[k] + (uint64_t)src * e;
            uint8_t* b = fs.p[k] + (uint64_t)dst * e;
            if (e == 8) *reinterpret_cast<uint64_t*>(b) = *reinterpret_cast<const uint64_t*>(a);
            else if (e == 4) *reinterpret_cast<uint32_t*>(b) = *reinterpret_cast<const uint32_t*>(a);
            else
                for (uint32_t q = 0; q < e; q++) b[q] = a[q];
        }
    }
}

// adapter.hpp:253-300: the parent of removed cells is 0, then += child / 8
// over its removed children in ascending order (the first removed child of
// each parent does the sum; `removed` ascending).  Eight lanes per removed
// cell, lane k on the parent's child k (x fastest: ascending ids): the
// children's entries in the retired cells' table (removed cells are retired
// and marked there) are probed together, the values gathered together and
// summed by lane 0 of the group in child order, as the reference adds them.
__global__ void __launch_bounds__(256) k_average_children(SlotView sv, MapParams mp, const uint64_t* __restrict__ removed,
                                                          uint64_t n, FieldSet fs, int32_t* __restrict__ err)
{
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63, k = lane & 7, g0 = lane & ~7;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // wave-uniform trip count (the shuffles need every lane)
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x - lane); base < 8 * n; base += stride) {
        const uint64_t i = (base + lane) >> 3;
        const bool valid = i < n;
        uint64_t c = 0, par = 0, ch = 0, ent = ~0ull;
        if (valid) {
            c = removed[i];
            uint64_t idx[3];
            int l;
            map_indices(mp, c, idx, &l);
            par = map_cell(mp, idx, l - 1);
            uint64_t pi[3];
            int pl;
            map_indices(mp, par, pi, &pl);
            const uint64_t h = (uint64_t)1 << (mp.max_lvl - l);
            const uint64_t ci[3] = {pi[0] + (k & 1) * h, pi[1] + ((k >> 1) & 1) * h, pi[2] + ((k >> 2) & 1) * h};
            ch = map_cell(mp, ci, l);
            ent = ret_entry(sv, ch);
        }
        const bool rem = ent != ~0ull && (ent & RET_REMOVED);
        // the first removed child of the parent does the sum
        const bool first = ((__ballot(valid && rem && ch < c) >> g0) & 0xffull) == 0 && valid;
        const int64_t ps = first ? slot_lookup(sv, par) : -1;
        if (first && ps < 0 && k == 0) atomicOr(err, 1);
        const bool in = first && ps >= 0 && rem && ch >= c;
        const int64_t cs = in ? (int64_t)(ent & ~RET_REMOVED) : -1;
        const uint64_t inmask = (__ballot(in) >> g0) & 0xffull;
        for (int f = 0; f < fs.n; f++) {
            double* d = reinterpret_cast<double*>(fs.p[f]);
            const double q = in ? d[cs] / 8 : 0.0;
            double acc = 0;
            for (int j = 0; j < 8; j++) {
                const double v = __shfl(q, g0 + j, 64);
                if (inmask >> j & 1) acc += v;
            }
            if (k == 0 && first && ps >= 0) d[ps] = acc;
        }
    }
}

static int field_sets(const dccrgx_grid* grid, const int32_t* fields, size_t nf, bool f64, std::vector<FieldSet>& out)
{
    out.clear();
    for (size_t k = 0; k < nf; k++) {
        DX_CHECK(fields[k] >= 0 && (size_t)fields[k] < grid->fields.size() && !grid->fields[fields[k]].variable,
                 DCCRGX_EINVAL, "bad field %d", fields[k]);
        const Field& F = grid->fields[fields[k]];
        DX_CHECK(!f64 || F.elem == 8, DCCRGX_EINVAL, "field %d is not an f64 field", fields[k]);
        if (out.empty() || out.back().n == 8) out.push_back(FieldSet{});
        FieldSet& fs = out.back();
        fs.p[fs.n] = static_cast<uint8_t*>(F.ptr);
        fs.elem[fs.n++] = F.elem;
    }
    return DCCRGX_OK;
}

// the rules over `new_cells` (copy from parents) and then `removed`
// (average of children; f64 fields), either list may be empty: one upload,
// one error word read back
static int run_rules(dccrgx_grid* grid, const std::vector<uint64_t>* new_cells, const std::vector<uint64_t>* removed,
                     const int32_t* fields, size_t nf)
{
    DX_CHECK(!grid->uniform, DCCRGX_ESTATE, "no refinement happened");
    const size_t nn = new_cells ? new_cells->size() : 0, nr = removed ? removed->size() : 0;
    if (!nn && !nr) return DCCRGX_OK;
    std::vector<FieldSet> copy_sets, avg_sets;
    if (nn) DX_TRY(field_sets(grid, fields, nf, false, copy_sets));
    if (nr) DX_TRY(field_sets(grid, fields, nf, true, avg_sets));
    hipStream_t st = grid->ctx->compute;
    Scratch S(st);
    uint64_t* d_cells;
    int32_t* d_err;
    DX_TRY(S.get(&d_cells, nn + nr + 1));
    d_err = reinterpret_cast<int32_t*>(d_cells + nn + nr);
    std::vector<uint64_t> up(nn + nr + 1, 0);  // the lists and a zeroed error word in one upload
    if (nn) std::copy(new_cells->begin(), new_cells->end(), up.begin());
    if (nr) std::copy(removed->begin(), removed->end(), up.begin() + nn);
    DX_TRY(dx_h2d_async(grid->ctx, d_cells, up.data(), up.size() * 8, st));
    const SlotView sv = slot_view(grid);
    for (const FieldSet& fs : copy_sets)
        hipLaunchKernelGGL(k_copy_from_parents, dim3(blocks(nn)), dim3(256), 0, st, sv, grid->map,
                           (const uint64_t*)d_cells, (uint64_t)nn, fs, d_err);
    for (const FieldSet& fs : avg_sets)  // after the copies (the reference's order, adapter.hpp:229-300)
        hipLaunchKernelGGL(k_average_children, dim3(blocks(8 * (uint64_t)nr)), dim3(256), 0, st, sv, grid->map,
                           (const uint64_t*)d_cells + nn, (uint64_t)nr, fs, d_err);
    DX_HIP(hipGetLastError());
    int32_t err = 0;
    DX_TRY(dx_d2h(grid->ctx, &err, d_err, 4, st));
    DX_CHECK(!err, DCCRGX_ENOTFOUND, "no data for a new or removed cell or its parent");
    return DCCRGX_OK;
}

int amr_dev_copy_from_parents(dccrgx_grid* grid, const int32_t* fields, size_t nf)
{
    return run_rules(grid, &grid->amr->new_cells, nullptr, fields, nf);
}

int amr_dev_average_children(dccrgx_grid* grid, const int32_t* fields, size_t nf)
{
    return run_rules(grid, nullptr, &grid->amr->removed, fields, nf);
}

int amr_dev_data_rules(dccrgx_grid* grid, const int32_t* fields, size_t nf)
{
    return run_rules(grid, &grid->amr->new_cells, &grid->amr->removed, fields, nf);
}

// codes 1..3 of the local cells (k_adapt_codes) into three id lists, each in
// local (ascending id) order, back to back in one buffer: per block of CODE_R
// * 256 cells the count of each code, one scan over the [code][block] counts,
// then each block writes its cells at the scanned offsets (wave ballots keep
// the order inside a block)
constexpr int CODE_R = 4;

__global__ void __launch_bounds__(256) k_code_count(const uint8_t* __restrict__ code, uint64_t n, uint32_t nb,
                                                    uint32_t* __restrict__ cnt)
{
    __shared__ uint32_t c3[3];
    if (threadIdx.x < 3) c3[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t q0 = (uint64_t)blockIdx.x * 256 * CODE_R;
    uint32_t m[3] = {0, 0, 0};
    for (int r = 0; r < CODE_R; r++) {
        const uint64_t q = q0 + r * 256 + threadIdx.x;
        const uint8_t c = q < n ? code[q] : 0;
        for (int k = 0; k < 3; k++) m[k] += __popcll(__ballot(c == k + 1));
    }
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 3; k++) atomicAdd(&c3[k], m[k]);
    __syncthreads();
    if (threadIdx.x < 3) cnt[threadIdx.x * nb + blockIdx.x] = c3[threadIdx.x];
}

__global__ void __launch_bounds__(256) k_code_scatter(const uint8_t* __restrict__ code, const uint64_t* __restrict__ leaves,
                                                      const uint32_t* __restrict__ local_g, uint64_t n, uint32_t nb,
                                                      const uint32_t* __restrict__ off, uint64_t* __restrict__ out)
{
    __shared__ uint32_t wsum[3][4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t below = (1ull << lane) - 1;
    uint32_t base[3];
    for (int k = 0; k < 3; k++) base[k] = off[k * nb + blockIdx.x];
    const uint64_t q0 = (uint64_t)blockIdx.x * 256 * CODE_R;
    for (int r = 0; r < CODE_R; r++) {
        const uint64_t q = q0 + r * 256 + threadIdx.x;
        const uint8_t c = q < n ? code[q] : 0;
        uint64_t m[3];
        for (int k = 0; k < 3; k++) m[k] = __ballot(c == k + 1);
        if (lane == 0)
            for (int k = 0; k < 3; k++) wsum[k][w] = (uint32_t)__popcll(m[k]);
        __syncthreads();
        uint32_t pre[3] = {0, 0, 0}, tot[3] = {0, 0, 0};
        for (int k = 0; k < 3; k++)
            for (int j = 0; j < 4; j++) {
                pre[k] += j < w ? wsum[k][j] : 0;
                tot[k] += wsum[k][j];
            }
        if (c >= 1 && c <= 3) {
            const int k = c - 1;
            out[base[k] + pre[k] + (uint32_t)__popcll(m[k] & below)] = leaves[local_g[q]];
        }
        for (int k = 0; k < 3; k++) base[k] += tot[k];
        __syncthreads();
    }
}

int amr_dev_codes_to_lists(dccrgx_grid* grid, const uint8_t* d_code, uint64_t n, uint64_t* out[3], size_t counts[3])
{
    Scratch S(grid->ctx->compute);
    uint64_t* d_out;
    DX_TRY(S.get(&d_out, std::max<uint64_t>(n, 1)));
    uint64_t* dev[3];
    DX_TRY(amr_dev_codes_to_device_lists(grid, d_code, n, d_out, dev, counts));
    D2H v[3];
    for (int k = 0; k < 3; k++) v[k] = D2H{out[k], dev[k], counts[k] * 8};
    return dx_d2h_many(grid->ctx, v, 3, grid->ctx->compute);  // the three lists behind one synchronisation
}

// the same lists left on the device in d_out (n entries): dev[k] = list k,
// counts[k] its length (one small read-back of the offsets)
int amr_dev_codes_to_device_lists(dccrgx_grid* grid, const uint8_t* d_code, uint64_t n, uint64_t* d_out,
                                  uint64_t* dev[3], size_t counts[3])
{
    hipStream_t st = grid->ctx->compute;
    const Explicit* E = grid->ex;
    DX_CHECK(n < (1ull << 32), DCCRGX_EINVAL, "%llu local cells", (unsigned long long)n);
    Scratch S(st);
    const uint32_t nb = (uint32_t)std::max<uint64_t>(1, (n + 256 * CODE_R - 1) / (256 * CODE_R));
    uint32_t *d_cnt, *d_off;
    DX_TRY(S.get(&d_cnt, 3ull * nb + 1));
    DX_TRY(S.get(&d_off, 3ull * nb + 1));
    DX_HIP(hipMemsetAsync(d_cnt + 3ull * nb, 0, 4, st));  // the scan's last entry: the total
    hipLaunchKernelGGL(k_code_count, dim3(nb), dim3(256), 0, st, d_code, n, nb, d_cnt);
    size_t tb = 0;
    DX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, d_cnt, d_off, (int)(3 * nb + 1), st));
    uint8_t* d_tmp;
    DX_TRY(S.get(&d_tmp, std::max<size_t>(tb, 1)));
    DX_HIP(hipcub::DeviceScan::ExclusiveSum(d_tmp, tb, d_cnt, d_off, (int)(3 * nb + 1), st));
    hipLaunchKernelGGL(k_code_scatter, dim3(nb), dim3(256), 0, st, d_code, (const uint64_t*)E->d_leaves,
                       (const uint32_t*)E->d_local_g, n, nb, (const uint32_t*)d_off, d_out);
    DX_HIP(hipGetLastError());
    // the lists start at the scanned offsets of their first blocks
    uint32_t start[4] = {0, 0, 0, 0};
    {
        const D2H c[4] = {{&start[0], d_off, 4}, {&start[1], d_off + nb, 4}, {&start[2], d_off + 2ull * nb, 4},
                          {&start[3], d_off + 3ull * nb, 4}};
        DX_TRY(dx_d2h_many(grid->ctx, c, 4, st));
    }
    for (int k = 0; k < 3; k++) {
        counts[k] = (size_t)(start[k + 1] - start[k]);
        dev[k] = d_out + start[k];
    }
    return DCCRGX_OK;
}

}  // namespace dccrgx
