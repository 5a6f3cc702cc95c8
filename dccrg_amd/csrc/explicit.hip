// explicit.hip -- grids with mixed refinement levels.
//
// The set of existing leaf cells is replicated on every rank (as the
// reference's cell_process, dccrg.hpp:7311) in a device open-addressing hash
// (64-bit id -> global leaf index).  Neighbor lists are built on the device
// for every leaf, in closed form instead of the reference's face-graph walk
// (dccrg.hpp:4375-4716): for item h of a cell at level l (length L in
// indices) the window is the level-l cell at idx + h*L (periodic wrap in
// index space, dropped outside a non-periodic grid); it is covered by
//   - that cell itself                  -> one entry, offset h*L
//   - its parent at level l-1           -> one entry, offset h*L - (window mod 2L)
//   - its 8 children at level l+1       -> 8 entries x-fastest, offset h*L + d*L/2
// which is exactly where the walk ends on a 2:1-balanced grid (the
// reference's own assumption, dccrg.hpp:4736-4737).  neighbors_to
// (dccrg.hpp:4744-4897) is the transpose of neighbors_of on such grids; it
// is built by transposing the device CSR.  Only the leaf ids and the lists
// are replicated; field storage is per rank: local cells, then ghosts, then
// retired cells (grid.hpp, Explicit).
#include <algorithm>
#include <mutex>
#include <cstring>
#include <set>

#include "exview.hpp"
#include "face.hpp"
#include "grid.hpp"

namespace dccrgx {

__global__ void __launch_bounds__(256) k_hash_insert(const uint64_t* __restrict__ ids, size_t n,
                                                     unsigned long long* keys, uint32_t* vals, uint64_t mask)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const unsigned long long id = ids[i];
        uint64_t h = hmix(id) & mask;
        for (;;) {
            const unsigned long long prev = atomicCAS(&keys[h], 0ull, id);
            if (prev == 0ull || prev == id) {
                vals[h] = (uint32_t)i;
                break;
            }
            h = (h + 1) & mask;
        }
    }
}

// the bitmap of the ascending leaf list: lanes holding ids of the same 64-bit
// word OR their bits together across the wave (a segmented doubling
// reduction) and the first lane of each run stores them with one atomic --
// one atomic per leaf on the same few words serialised (230 us on 3.5 M leaves)
__global__ void __launch_bounds__(256) k_bits_set(const uint64_t* __restrict__ leaves, size_t n,
                                                  unsigned long long* bits)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const int lane = threadIdx.x & 63;
    const size_t n64 = (n + 63) & ~(size_t)63;  // every lane of a wave runs every iteration
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n64; i += stride) {
        const bool valid = i < n;
        const uint64_t id = valid ? leaves[i] : 0;
        const uint64_t w = valid ? id >> 6 : ~0ull;
        unsigned long long b = valid ? 1ull << (id & 63) : 0ull;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long y = __shfl_down(b, d, 64);
            const uint64_t yw = __shfl_down(w, d, 64);
            if (lane + d < 64 && yw == w) b |= y;
        }
        const uint64_t pw = __shfl_up(w, 1, 64);
        if (valid && (lane == 0 || pw != w)) atomicOr(&bits[w], b);
    }
}

// rank[w] = number of leaves with id < 64 w (binary search in the ascending
// list), and bits[w] cleared for k_bits_set (no memset launch)
__global__ void __launch_bounds__(256) k_bits_rank(const uint64_t* __restrict__ leaves, uint64_t n, uint64_t nw,
                                                   uint32_t* __restrict__ rank, uint64_t* __restrict__ bits)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
        const uint64_t key = (uint64_t)w << 6;
        uint64_t lo = 0, hi = n;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (leaves[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        rank[w] = (uint32_t)lo;
        bits[w] = 0;
    }
}

// neighbors_of of `cells` (pass 1: counts in row[i+1]; pass 2: fill from row[i])
__global__ void __launch_bounds__(256) k_ex_nof(ExView v, const int32_t* __restrict__ items, int K,
                                                const uint64_t* __restrict__ cells, size_t n,
                                                uint64_t* __restrict__ row, uint64_t* __restrict__ ids,
                                                int32_t* __restrict__ off, uint32_t* __restrict__ gidx,
                                                int32_t* __restrict__ err, uint64_t* __restrict__ codes = nullptr)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const MapParams& p = v.mp;
    const int M = p.max_lvl;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t c = cells[i];
        uint64_t w = ids ? row[i] : 0;
        uint64_t code = 0;  // count pass, K <= 32: each item's case in 2 bits (k_ex_nof_fill_codes)
        uint64_t idx[3];
        int l;
        if (ex_find(v, c) < 0 || !map_indices(p, c, idx, &l)) {
            atomicOr(err, 1);
            if (!ids) row[i + 1] = 0;
            continue;
        }
        const int64_t L = (int64_t)1 << (M - l);
        auto emit = [&](uint64_t id, int64_t g, int64_t ox, int64_t oy, int64_t oz) {
            if (ids) {
                ids[w] = id;
                if (gidx) gidx[w] = (uint32_t)g;
                if (off) {
                    off[3 * w + 0] = (int32_t)ox;
                    off[3 * w + 1] = (int32_t)oy;
                    off[3 * w + 2] = (int32_t)oz;
                }
            }
            w++;
        };
        for (int k = 0; k < K; k++) {
            const int32_t* h = items + 3 * k;
            uint64_t wi[3];
            bool ok = true;
            for (int d = 0; d < 3; d++) {
                const int64_t G = (int64_t)(p.length[d] << M);
                int64_t x = (int64_t)idx[d] + (int64_t)h[d] * L;
                if (x < 0 || x >= G) {
                    if (!v.per[d]) {
                        ok = false;
                        break;
                    }
                    x %= G;
                    if (x < 0) x += G;
                }
                wi[d] = (uint64_t)x;
            }
            if (!ok) continue;  // outside a non-periodic grid: dropped (dccrg.hpp:4670-4672)
            const uint64_t W = map_cell(p, wi, l);
            int64_t g = ex_find(v, W);
            if (g >= 0) {
                emit(W, g, h[0] * L, h[1] * L, h[2] * L);
                code |= 1ull << (2 * k);
                continue;
            }
            if (l > 0) {
                const uint64_t P = map_cell(p, wi, l - 1);
                g = ex_find(v, P);
                if (g >= 0) {
                    code |= 2ull << (2 * k);
                    const int64_t L2 = 2 * L;
                    emit(P, g, h[0] * L - (int64_t)(wi[0] % L2), h[1] * L - (int64_t)(wi[1] % L2),
                         h[2] * L - (int64_t)(wi[2] % L2));
                    continue;
                }
            }
            if (l < M) {  // the 8 children, listed only when all exist
                const int64_t hl = L / 2;
                int64_t gc[8];
                bool all = true;
                for (int j = 0; j < 8; j++) {
                    const uint64_t ci[3] = {wi[0] + (j & 1) * hl, wi[1] + ((j >> 1) & 1) * hl, wi[2] + ((j >> 2) & 1) * hl};
                    gc[j] = ex_find(v, map_cell(p, ci, l + 1));
                    all &= gc[j] >= 0;
                }
                if (all) {
                    code |= 3ull << (2 * k);
                    for (int j = 0; j < 8; j++) {
                        const int64_t dx = j & 1, dy = (j >> 1) & 1, dz = (j >> 2) & 1;
                        const uint64_t ci[3] = {wi[0] + dx * hl, wi[1] + dy * hl, wi[2] + dz * hl};
                        emit(map_cell(p, ci, l + 1), gc[j], h[0] * L + dx * hl, h[1] * L + dy * hl, h[2] * L + dz * hl);
                    }
                    continue;
                }
            }
            // no leaf covers the window: a level difference > 1 (outside the
            // reference's assumptions, an error) or, on a grid holding part of
            // the leaves (hybrid.hip's box), a window beyond them: dropped
            atomicOr(err, 2);
        }
        if (!ids) row[i + 1] = w;
        if (codes) codes[i] = code;
    }
}

// Fill pass of k_ex_nof with coalesced stores: one wave per 64 cells whose
// rows (already counted and scanned) form one output run.  Each lane lists
// its cell's entries as 8-byte records (leaf index; lane, case, item) in LDS
// at the entry's place in the run; the wave then writes the run entry by
// entry, consecutive lanes on consecutive entries, recomputing the id and
// offset from the record and the cell's indices (no hash probe at store
// time).  case 0: the window's cell, 1: its parent, 2 + d: child d (x fastest).
// Entries beyond the LDS capacity are written by their lane directly.
constexpr int NOF_REC_CAP = 1024;  // records per wave (8 KiB; four independent waves per workgroup)


__device__ __forceinline__ void nof_entry(const MapParams& p, const uint64_t wi[3], int l, const int32_t* h, int64_t L,
                                          int cs, uint64_t& id, int32_t o[3])
{
    if (cs == 0) {
        id = map_cell(p, wi, l);
        for (int d = 0; d < 3; d++) o[d] = (int32_t)(h[d] * L);
    } else if (cs == 1) {
        id = map_cell(p, wi, l - 1);
        for (int d = 0; d < 3; d++) o[d] = (int32_t)(h[d] * L - (int64_t)(wi[d] % (uint64_t)(2 * L)));
    } else {
        const int c = cs - 2;
        const int64_t hl = L / 2;
        const int64_t dd[3] = {c & 1, (c >> 1) & 1, (c >> 2) & 1};
        uint64_t ci[3];
        for (int d = 0; d < 3; d++) {
            ci[d] = wi[d] + (uint64_t)(dd[d] * hl);
            o[d] = (int32_t)(h[d] * L + dd[d] * hl);
        }
        id = map_cell(p, ci, l + 1);
    }
}

__global__ void __launch_bounds__(256) k_ex_nof_fill(ExView v, const int32_t* __restrict__ items, int K,
                                                     const uint64_t* __restrict__ cells, size_t n,
                                                     const uint64_t* __restrict__ row, uint64_t* __restrict__ ids,
                                                     int32_t* __restrict__ off, uint32_t* __restrict__ gidx)
{
    __shared__ uint2 rec_all[4][NOF_REC_CAP];
    __shared__ uint64_t s_idx_all[4][3][64];
    __shared__ int32_t s_lvl_all[4][64];
    const int wv = threadIdx.x >> 6;
    uint2* rec = rec_all[wv];
    uint64_t(*s_idx)[64] = s_idx_all[wv];
    int32_t* s_lvl = s_lvl_all[wv];
    const MapParams& p = v.mp;
    const int M = p.max_lvl;
    const int lane = threadIdx.x & 63;
    const uint64_t r0 = ((uint64_t)blockIdx.x * 4 + wv) * 64;
    const bool live = r0 < n;  // a wave past the end still meets the block barrier
    const uint64_t last = r0 + 64 < n ? r0 + 64 : n;
    const uint64_t base = live ? row[r0] : 0, end = live ? row[last] : 0;
    const uint64_t i = r0 + lane;
    if (i < n) {
        uint64_t idx[3];
        int l;
        const uint64_t c = cells[i];
        if (map_indices(p, c, idx, &l) && ex_find(v, c) >= 0) {
            for (int d = 0; d < 3; d++) s_idx[d][lane] = idx[d];
            s_lvl[lane] = l;
            const int64_t L = (int64_t)1 << (M - l);
            uint64_t w = row[i] - base;
            auto put = [&](uint32_t g, int cs, int k, const uint64_t* wi) {
                if (w < NOF_REC_CAP) {
                    rec[w] = make_uint2(g, ((uint32_t)lane << 24) | ((uint32_t)cs << 16) | (uint32_t)k);
                } else {  // beyond the staging capacity: this lane stores the entry
                    uint64_t id;
                    int32_t o[3];
                    nof_entry(p, wi, l, items + 3 * k, L, cs, id, o);
                    const uint64_t e = base + w;
                    ids[e] = id;
                    if (gidx) gidx[e] = g;
                    if (off) {
                        off[3 * e + 0] = o[0];
                        off[3 * e + 1] = o[1];
                        off[3 * e + 2] = o[2];
                    }
                }
                w++;
            };
            for (int k = 0; k < K; k++) {
                const int32_t* h = items + 3 * k;
                uint64_t wi[3];
                if (!nof_window(p, v.per, idx, h, L, wi)) continue;  // outside: dropped (dccrg.hpp:4670-4672)
                int64_t g = ex_find(v, map_cell(p, wi, l));
                if (g >= 0) {
                    put((uint32_t)g, 0, k, wi);
                    continue;
                }
                if (l > 0) {
                    g = ex_find(v, map_cell(p, wi, l - 1));
                    if (g >= 0) {
                        put((uint32_t)g, 1, k, wi);
                        continue;
                    }
                }
                if (l < M) {  // the 8 children, listed (as in the count pass) only when all exist
                    const uint64_t hl = (uint64_t)(L / 2);
                    int64_t gc[8];
                    bool all = true;
                    for (int cix = 0; cix < 8; cix++) {
                        const uint64_t ci[3] = {wi[0] + (cix & 1) * hl, wi[1] + ((cix >> 1) & 1) * hl,
                                                wi[2] + ((cix >> 2) & 1) * hl};
                        gc[cix] = ex_find(v, map_cell(p, ci, l + 1));
                        all &= gc[cix] >= 0;
                    }
                    if (all)
                        for (int cix = 0; cix < 8; cix++) put((uint32_t)gc[cix], 2 + cix, k, wi);
                }
            }
        }
    }
    __syncthreads();
    const uint64_t tot = end - base < (uint64_t)NOF_REC_CAP ? end - base : (uint64_t)NOF_REC_CAP;
    for (uint64_t e = lane; e < tot; e += 64) {
        const uint2 r = rec[e];
        const int ln = (int)(r.y >> 24), cs = (int)((r.y >> 16) & 0xffu), k = (int)(r.y & 0xffffu);
        const uint64_t idx[3] = {s_idx[0][ln], s_idx[1][ln], s_idx[2][ln]};
        const int l = s_lvl[ln];
        const int64_t L = (int64_t)1 << (M - l);
        uint64_t wi[3];
        nof_window(p, v.per, idx, items + 3 * k, L, wi);
        uint64_t id;
        int32_t o[3];
        nof_entry(p, wi, l, items + 3 * k, L, cs, id, o);
        ids[base + e] = id;
        if (gidx) gidx[base + e] = r.x;
        if (off) {
            off[3 * (base + e) + 0] = o[0];
            off[3 * (base + e) + 1] = o[1];
            off[3 * (base + e) + 2] = o[2];
        }
    }
}

// Fill pass from the count pass's per-item cases (K <= 32), entry-parallel:
// one wave per 64 cells whose rows form one output run.  The wave walks its
// run 64 entries at a time; each lane finds its entry's cell (binary search
// over the 65 row offsets in LDS) and item (the cell's 2-bit cases: 0
// dropped, 1 the window's cell, 2 its parent, 3 its 8 children), rebuilds id
// and offset from the cell's indices and looks up the leaf index.  Every
// store is coalesced whatever the row lengths (k_ex_nof_fill stages 1024
// records per wave and stores the rest per lane: 2.5x the output's bytes
// written for 26-item neighborhoods), and an entry costs one lookup.
__global__ void __launch_bounds__(256) k_ex_nof_fill_codes(ExView v, const int32_t* __restrict__ items, int K,
                                                           const uint64_t* __restrict__ cells, size_t n,
                                                           const uint64_t* __restrict__ row,
                                                           const uint64_t* __restrict__ codes, uint64_t* __restrict__ ids,
                                                           int32_t* __restrict__ off, uint32_t* __restrict__ gidx)
{
    __shared__ uint64_t s_row_all[4][65];
    __shared__ uint64_t s_code_all[4][64];
    __shared__ uint64_t s_idx_all[4][3][64];
    __shared__ int32_t s_lvl_all[4][64];
    const int wv = threadIdx.x >> 6;
    uint64_t* s_row = s_row_all[wv];
    uint64_t* s_code = s_code_all[wv];
    uint64_t(*s_idx)[64] = s_idx_all[wv];
    int32_t* s_lvl = s_lvl_all[wv];
    const MapParams& p = v.mp;
    const int M = p.max_lvl;
    const int lane = threadIdx.x & 63;
    const uint64_t r0 = ((uint64_t)blockIdx.x * 4 + wv) * 64;
    const bool live = r0 < n;  // a wave past the end still meets the block barrier
    const uint64_t last = r0 + 64 < n ? r0 + 64 : n;
    const uint64_t i = r0 + lane;
    if (live) {
        const uint64_t end_row = row[last];
        s_row[lane] = i < n ? row[i] : end_row;
        if (lane == 0) s_row[64] = end_row;
        uint64_t idx[3] = {0, 0, 0};
        int l = 0;
        if (i < n) map_indices(p, cells[i], idx, &l);  // cells the count pass refused have empty rows
        for (int d = 0; d < 3; d++) s_idx[d][lane] = idx[d];
        s_lvl[lane] = l;
        s_code[lane] = i < n ? codes[i] : 0;
    }
    __syncthreads();
    if (!live) return;
    const uint64_t base = s_row[0], end = s_row[64];
    for (uint64_t e = base + lane; e < end; e += 64) {
        int lo = 0, hi = 64;  // the last cell whose row starts at or before e
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s_row[mid] <= e) lo = mid;
            else hi = mid;
        }
        uint64_t t = e - s_row[lo];
        const uint64_t code = s_code[lo];
        int k = 0, cs = 0;
        for (; k < K; k++) {
            const uint32_t c2 = (uint32_t)(code >> (2 * k)) & 3u;
            const uint64_t cnt = c2 == 3u ? 8 : (c2 ? 1 : 0);
            if (t < cnt) {
                cs = c2 == 1u ? 0 : c2 == 2u ? 1 : 2 + (int)t;
                break;
            }
            t -= cnt;
        }
        const uint64_t idx[3] = {s_idx[0][lo], s_idx[1][lo], s_idx[2][lo]};
        const int l = s_lvl[lo];
        const int64_t L = (int64_t)1 << (M - l);
        uint64_t wi[3];
        nof_window(p, v.per, idx, items + 3 * k, L, wi);
        uint64_t id;
        int32_t o[3];
        nof_entry(p, wi, l, items + 3 * k, L, cs, id, o);
        ids[e] = id;
        gidx[e] = (uint32_t)ex_find(v, id);
        off[3 * e + 0] = o[0];
        off[3 * e + 1] = o[1];
        off[3 * e + 2] = o[2];
    }
}

// row classes of the sort-unique passes (in the count array until sorted)
constexpr uint32_t ROW_MEDIUM = 0xfffffffeu;  // row for the LDS kernel (65..WAVE_SORT_MAX entries)
constexpr uint32_t ROW_LONG = 0xffffffffu;    // row for the per-thread kernel (> WAVE_SORT_MAX)

// transpose helpers: rows = global leaves
__global__ void __launch_bounds__(256) k_tr_count(const uint64_t* __restrict__ row, const uint32_t* __restrict__ tgt,
                                                  uint64_t n, uint32_t* __restrict__ cnt)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += stride)
        row_walk4(row[s], row[s + 1], tgt, [&](uint64_t, uint32_t t) { atomicAdd(&cnt[t], 1u); });
}

__global__ void __launch_bounds__(256) k_tr_scatter(const uint64_t* __restrict__ row, const uint32_t* __restrict__ tgt,
                                                    uint64_t n, const uint64_t* __restrict__ trow,
                                                    uint32_t* __restrict__ cursor, uint32_t* __restrict__ out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += stride)
        row_walk4(row[s], row[s + 1], tgt,
                  [&](uint64_t, uint32_t t) { out[trow[t] + atomicAdd(&cursor[t], 1u)] = (uint32_t)s; });
}

// per row: insertion sort + unique in place; unique count -> ucnt
// (rows longer than the wave kernel takes: those flagged ~0 in ucnt)
__global__ void __launch_bounds__(256) k_sort_unique_rows(const uint64_t* __restrict__ row, uint64_t n,
                                                          uint32_t* __restrict__ v, uint32_t* __restrict__ ucnt)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += stride) {
        if (ucnt[r] != ROW_LONG) continue;
        uint32_t* a = v + row[r];
        const uint64_t m = row[r + 1] - row[r];
        for (uint64_t i = 1; i < m; i++) {
            const uint32_t x = a[i];
            uint64_t j = i;
            while (j > 0 && a[j - 1] > x) {
                a[j] = a[j - 1];
                j--;
            }
            a[j] = x;
        }
        uint64_t u = 0;
        for (uint64_t i = 0; i < m; i++)
            if (u == 0 || a[i] != a[u - 1]) a[u++] = a[i];
        ucnt[r] = (uint32_t)u;
    }
}

__global__ void __launch_bounds__(256) k_copy_rows(const uint64_t* __restrict__ srow, const uint32_t* __restrict__ sv,
                                                   const uint64_t* __restrict__ drow, uint64_t n,
                                                   uint32_t* __restrict__ dv)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += stride)
        for (uint64_t i = 0; i < drow[r + 1] - drow[r]; i++) dv[drow[r] + i] = sv[srow[r] + i];
}

// stencil rows for local cells: unique (leaf, offset) pairs of neighbors_of
struct Pair {
    uint32_t g;
    int32_t x, y, z;
};
__device__ inline bool pair_less(const Pair& a, const Pair& b)
{
    if (a.g != b.g) return a.g < b.g;
    if (a.x != b.x) return a.x < b.x;
    if (a.y != b.y) return a.y < b.y;
    return a.z < b.z;
}
__device__ inline bool pair_eq(const Pair& a, const Pair& b)
{
    return a.g == b.g && a.x == b.x && a.y == b.y && a.z == b.z;
}
__device__ __forceinline__ bool pair_less_(const Pair& a, const Pair& b) { return pair_less(a, b); }

__global__ void __launch_bounds__(256) k_stencil_rows(const uint64_t* __restrict__ nof_row,
                                                      const uint32_t* __restrict__ nof_g,
                                                      const int32_t* __restrict__ nof_off,
                                                      const uint32_t* __restrict__ local_g, uint64_t nl,
                                                      const uint64_t* __restrict__ tmp_row, Pair* __restrict__ tmp,
                                                      uint32_t* __restrict__ ucnt)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += stride) {
        if (ucnt[i] != ROW_LONG) continue;  // done by k_stencil_rows_seg / k_stencil_rows_wave
        const uint32_t r = local_g[i];
        Pair* a = tmp + tmp_row[i];
        const uint64_t m = nof_row[r + 1] - nof_row[r];
        for (uint64_t e = 0; e < m; e++) {
            const uint64_t s = nof_row[r] + e;
            Pair x{nof_g[s], nof_off[3 * s], nof_off[3 * s + 1], nof_off[3 * s + 2]};
            uint64_t j = e;
            while (j > 0 && pair_less(x, a[j - 1])) {
                a[j] = a[j - 1];
                j--;
            }
            a[j] = x;
        }
        uint64_t u = 0;
        for (uint64_t e = 0; e < m; e++)
            if (u == 0 || !pair_eq(a[e], a[u - 1])) a[u++] = a[e];
        ucnt[i] = (uint32_t)u;
    }
}

__global__ void __launch_bounds__(256) k_stencil_slots(const uint64_t* __restrict__ tmp_row, const Pair* __restrict__ tmp,
                                                       const uint64_t* __restrict__ st_row, uint64_t nl,
                                                       const uint32_t* __restrict__ slot_of_g,
                                                       uint32_t* __restrict__ st_slot, int32_t* __restrict__ st_off)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += stride)
        for (uint64_t e = 0; e < st_row[i + 1] - st_row[i]; e++) {
            const Pair& p = tmp[tmp_row[i] + e];
            const uint64_t o = st_row[i] + e;
            st_slot[o] = slot_of_g[p.g];
            st_off[3 * o + 0] = p.x;
            st_off[3 * o + 1] = p.y;
            st_off[3 * o + 2] = p.z;
        }
}

// the same per wavefront in LDS (rows up to WAVE_SORT_MAX; longer ones flagged
// ~0 in ucnt for k_stencil_rows); defined after the wave helpers
// count pass (out == null: row[i + 1] = entries) / fill pass (from row[i])
__global__ void __launch_bounds__(256) k_ex_nto(ExView v, const int32_t* __restrict__ items_to, int K,
                                                const uint64_t* __restrict__ cells, size_t n, uint64_t* __restrict__ row,
                                                uint32_t* __restrict__ out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t w = out ? row[i] : 0;
        nto_search(v, items_to, K, cells[i], [&](uint32_t g) {
            if (out) out[w] = g;
            w++;
        });
        if (!out) row[i + 1] = w;
    }
}

__global__ void __launch_bounds__(256) k_ex_gol(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                uint32_t* __restrict__ cnt, const uint64_t* __restrict__ st_row,
                                                const uint32_t* __restrict__ st_slot,
                                                const uint32_t* __restrict__ local_slot,
                                                const uint32_t* __restrict__ pos, uint64_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t q = pos[i];
        uint32_t c = 0;
        row_walk4(st_row[q], st_row[q + 1], st_slot, [&](uint64_t, uint32_t sl) { c += in[sl] != 0u ? 1u : 0u; });
        const uint32_t s = local_slot[q];
        cnt[s] = c;
        out[s] = c == 3u ? 1u : (c == 2u ? in[s] : 0u);
    }
}

__global__ void __launch_bounds__(256) k_ex_slots(ExView v, const uint32_t* __restrict__ slot_of_g,
                                                  const uint64_t* __restrict__ ids, size_t n,
                                                  int64_t* __restrict__ slots)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t g = ex_find(v, ids[i]);
        const uint32_t s = g < 0 ? NO_SLOT : slot_of_g[g];
        slots[i] = s == NO_SLOT ? -1 : (int64_t)s;
    }
}

// ---------------------------------------------------------------------------
// wave-cooperative CSR kernels.  A row of a neighbor list is short (tens of
// entries), so one thread per row writes scattered 4-24 B pieces; instead a
// wavefront takes 64 consecutive rows, whose output is one contiguous run,
// and its lanes write consecutive entries of that run (each lane finds the
// row of its entry by a binary search over the 65 row starts kept in LDS).
// ---------------------------------------------------------------------------
// index j in [0, 64) with s[j] <= e < s[j + 1] (s ascending, s[64] > e)
__device__ __forceinline__ int wave_row_of(const uint64_t* s, uint64_t e)
{
    int lo = 0, hi = 64;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (s[mid] <= e) lo = mid;
        else hi = mid;
    }
    return lo;
}

// rows of the query cells copied from the stored CSR of every leaf:
// out entry k of query i = CSR entry nof_row[gq[i]] + k (ids, offsets)
__global__ void __launch_bounds__(64) k_rows_gather(const uint32_t* __restrict__ gq, uint64_t n,
                                                    const uint64_t* __restrict__ src_row,
                                                    const uint64_t* __restrict__ row,
                                                    const uint64_t* __restrict__ src_id,
                                                    const int32_t* __restrict__ src_off, uint64_t* __restrict__ ids,
                                                    int32_t* __restrict__ off3)
{
    __shared__ uint64_t s_dst[65], s_src[64];
    const int lane = threadIdx.x;
    const uint64_t r0 = (uint64_t)blockIdx.x * 64;
    const uint64_t last = r0 + 64 < n ? r0 + 64 : n;  // rows [r0, last); rows past the end are empty
    s_dst[lane] = row[r0 + lane < last ? r0 + lane : last];
    if (lane == 0) s_dst[64] = row[last];
    if (r0 + lane < n) s_src[lane] = src_row[gq[r0 + lane]];
    __syncthreads();
    const uint64_t end = s_dst[64];
    // the 64 rows one run of the source (queries of consecutive cells: every
    // leaf, a slab): a straight copy, no row search per entry
    const bool run = r0 + lane + 1 >= last || s_src[lane + 1] == s_src[lane] + (s_dst[lane + 1] - s_dst[lane]);
    if (__all(run)) {
        const uint64_t d0 = s_dst[0], s0 = s_src[0];
        for (uint64_t e = d0 + lane; e < end; e += 64) ids[e] = src_id[s0 + (e - d0)];
        if (off3)
            for (uint64_t w = lane; w < 3 * (end - d0); w += 64) off3[3 * d0 + w] = src_off[3 * s0 + w];
        return;
    }
    for (uint64_t e = s_dst[0] + lane; e < end; e += 64) {
        const int j = wave_row_of(s_dst, e);
        const uint64_t src = s_src[j] + (e - s_dst[j]);
        ids[e] = src_id[src];
        if (off3)  // one 12-byte load and store per entry (dwordx3)
            reinterpret_cast<int3*>(off3)[e] = reinterpret_cast<const int3*>(src_off)[src];
    }
}

// the same for neighbors_to rows, whose entries are leaf indices: out entry
// k of query i = leaves[src_g[src_row[gq[i]] + k]]
__global__ void __launch_bounds__(64) k_rows_gather_g(const uint32_t* __restrict__ gq, uint64_t n,
                                                      const uint64_t* __restrict__ src_row,
                                                      const uint64_t* __restrict__ row,
                                                      const uint32_t* __restrict__ src_g,
                                                      const uint64_t* __restrict__ leaves, uint64_t* __restrict__ ids)
{
    __shared__ uint64_t s_dst[65], s_src[64];
    const int lane = threadIdx.x;
    const uint64_t r0 = (uint64_t)blockIdx.x * 64;
    const uint64_t last = r0 + 64 < n ? r0 + 64 : n;
    s_dst[lane] = row[r0 + lane < last ? r0 + lane : last];
    if (lane == 0) s_dst[64] = row[last];
    if (r0 + lane < n) s_src[lane] = src_row[gq[r0 + lane]];
    __syncthreads();
    const uint64_t end = s_dst[64];
    const bool run = r0 + lane + 1 >= last || s_src[lane + 1] == s_src[lane] + (s_dst[lane + 1] - s_dst[lane]);
    if (__all(run)) {  // one run of the source (see k_rows_gather)
        const uint64_t d0 = s_dst[0], s0 = s_src[0];
        for (uint64_t e = d0 + lane; e < end; e += 64) ids[e] = leaves[src_g[s0 + (e - d0)]];
        return;
    }
    for (uint64_t e = s_dst[0] + lane; e < end; e += 64) {
        const int j = wave_row_of(s_dst, e);
        ids[e] = leaves[src_g[s_src[j] + (e - s_dst[j])]];
    }
}

// query cells -> their row (local position) and its length in the stored
// CSR; err bit 1: not a leaf, bit 4: a leaf of another process (no row here)
__global__ void __launch_bounds__(256) k_ex_query_rows(ExView v, const uint64_t* __restrict__ cells, size_t n,
                                                       const uint64_t* __restrict__ nof_row,
                                                       const uint32_t* __restrict__ slot_of_g, uint64_t n_local,
                                                       uint32_t* __restrict__ gq, uint64_t* __restrict__ row,
                                                       int32_t* __restrict__ err)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t g = ex_find(v, cells[i]);
        const uint32_t r = g < 0 ? NO_SLOT : slot_of_g[g];
        if (g < 0 || r >= n_local) {
            atomicOr(err, g < 0 ? 1 : 4);
            row[i + 1] = 0;
            gq[i] = 0;
            continue;
        }
        gq[i] = r;
        row[i + 1] = nof_row[r + 1] - nof_row[r];
    }
}

// sort + unique of one row per wavefront, in LDS (bitonic over the next power
// of two >= the row length, at most WAVE_SORT_MAX); the unique prefix is
// written back in place and its length to ucnt.  Longer rows are left to the
// per-thread kernels (flagged in ucnt as ~0).
constexpr int WAVE_SORT_MAX = 1024;


// bitonic sort of one element per lane across the wavefront (ascending by
// lane), exchanges by cross-lane shuffles: no LDS
__device__ __forceinline__ uint32_t shfl_xor_any(uint32_t x, int j) { return __shfl_xor(x, j, 64); }
__device__ __forceinline__ Pair shfl_xor_any(const Pair& x, int j)
{
    return Pair{(uint32_t)__shfl_xor(x.g, j, 64), __shfl_xor(x.x, j, 64), __shfl_xor(x.y, j, 64),
                __shfl_xor(x.z, j, 64)};
}

template <class T, class Less>
__device__ void wave_bitonic(T* a, int m2, Less less)
{
    for (int k = 2; k <= m2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < m2; i += 64) {
                const int p = i ^ j;
                if (p > i) {
                    const bool up = (i & k) == 0;
                    const T x = a[i], y = a[p];
                    if (up ? less(y, x) : less(x, y)) {
                        a[i] = y;
                        a[p] = x;
                    }
                }
            }
            __syncthreads();
        }
}

// unique of a sorted LDS array of m entries by one wave: out[0..u) = the
// first of every run of equal entries; returns u
template <class T, class Eq, class Out>
__device__ uint32_t wave_unique(const T* a, int m, Eq eq, Out out)
{
    uint32_t base = 0;
    for (int c = 0; c < m; c += 64) {
        const int i = c + (int)threadIdx.x;
        const bool keep = i < m && (i == 0 || !eq(a[i], a[i - 1]));
        const uint64_t mask = __ballot(keep);
        const uint32_t before = (uint32_t)__popcll(mask & ((1ull << threadIdx.x) - 1ull));
        if (keep) out(base + before, a[i]);
        base += (uint32_t)__popcll(mask);
    }
    return base;
}

// bitonic sort across segments of W lanes (W | 64), ascending in every segment
template <int W, class T, class Less>
__device__ __forceinline__ T seg_sort(T x, Less less)
{
    const int lane = threadIdx.x & 63;
    for (int k = 2; k <= W; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            const T y = shfl_xor_any(x, j);
            const bool up = k == W || (lane & k) == 0;
            const bool keep_min = ((lane & j) == 0) == up;
            if (keep_min == less(y, x)) x = y;
        }
    return x;
}

constexpr uint32_t ROW_PEND = 0xfffffffdu;  // row of 17..64 entries, for the 64-lane pass

// rows sorted and made unique in registers, W lanes per row (64 / W rows per
// wave): the short rows of face neighborhoods fill a wave 4 at a time.  A
// row longer than W is flagged -- for the 64-lane pass (PEND_ONLY: the
// flagged rows only), then for the LDS / per-thread kernels.
// rows handed from one pass to the next as compacted lists: the 16-lane pass
// appends the rows it leaves for the 64-lane pass, which appends the rows it
// leaves for the LDS pass (a pass that walked every row to find its few cost
// ~250 us per pass on 3.5 M rows)
struct RowLists {
    uint32_t* pend;  // rows longer than 16 entries
    uint32_t* med;   // rows of 65..WAVE_SORT_MAX entries
    uint32_t* cnt;   // [0] pend, [1] med
};

template <int W, bool PEND_ONLY>
__global__ void __launch_bounds__(256) k_sort_unique_rows_seg(const uint64_t* __restrict__ row, uint64_t n,
                                                              uint32_t* __restrict__ v, uint32_t* __restrict__ ucnt,
                                                              RowLists L)
{
    constexpr int R = 64 / W;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const int lane = threadIdx.x & 63, sl = lane & (W - 1), seg = lane / W;
    const uint64_t segmask = (W >= 64 ? ~0ull : ((1ull << (W & 63)) - 1ull)) << (seg * W);
    if constexpr (PEND_ONLY) {  // W == 64: a wave per row the 16-lane pass left
        const uint32_t np = L.cnt[0];
        for (uint64_t k = wave; k < np; k += waves) {
            const uint64_t r = L.pend[k];
            const uint64_t b = row[r];
            const int m = (int)(row[r + 1] - b);
            if (m > 64) {
                if (lane == 0) {
                    ucnt[r] = m > WAVE_SORT_MAX ? ROW_LONG : ROW_MEDIUM;
                    if (m <= WAVE_SORT_MAX) L.med[atomicAdd(&L.cnt[1], 1u)] = (uint32_t)r;
                }
                continue;
            }
            uint32_t x = lane < m ? v[b + lane] : 0xffffffffu;
            x = seg_sort<64>(x, [](uint32_t a, uint32_t c) { return a < c; });
            const uint32_t prev = __shfl_up(x, 1, 64);
            const bool keep = lane < m && (lane == 0 || x != prev);
            const uint64_t mask = __ballot(keep);
            if (keep) v[b + __popcll(mask & ((1ull << lane) - 1ull))] = x;
            if (lane == 0) ucnt[r] = (uint32_t)__popcll(mask);
        }
        return;
    }
    for (uint64_t r0 = wave * R; r0 < n; r0 += waves * R) {
        const uint64_t r = r0 + seg;
        bool active = r < n;
        uint64_t b = 0;
        int m = 0;
        bool pend = false;
        if (active) {
            b = row[r];
            m = (int)(row[r + 1] - b);
            if (m > W) {
                pend = true;
                if (sl == 0) ucnt[r] = ROW_PEND;
                active = false;
            }
        }
        if (__ballot(pend && sl == 0)) {  // rare: most rows fit the pass
            const uint32_t pk = wave_reserve(&L.cnt[0], pend && sl == 0 ? 1u : 0u);
            if (pend && sl == 0) L.pend[pk] = (uint32_t)r;
        }
        if (!__ballot(active)) continue;
        uint32_t x = active && sl < m ? v[b + sl] : 0xffffffffu;
        x = seg_sort<W>(x, [](uint32_t a, uint32_t c) { return a < c; });
        const uint32_t prev = __shfl_up(x, 1, W);
        const bool keep = active && sl < m && (sl == 0 || x != prev);
        const uint64_t mask = __ballot(keep);
        if (keep) v[b + __popcll(mask & segmask & ((1ull << lane) - 1ull))] = x;
        if (active && sl == 0) ucnt[r] = (uint32_t)__popcll(mask & segmask);
    }
}

__global__ void __launch_bounds__(64) k_sort_unique_rows_wave(const uint64_t* __restrict__ row, uint64_t n,
                                                              uint32_t* __restrict__ v, uint32_t* __restrict__ ucnt,
                                                              RowLists L)
{
    __shared__ uint32_t a[WAVE_SORT_MAX];
    const uint32_t nm = L.cnt[1];
    for (uint32_t k = blockIdx.x; k < nm; k += gridDim.x) {
        const uint64_t r = L.med[k];
        const uint64_t b = row[r];
        const int m = (int)(row[r + 1] - b);
        int m2 = 1;
        while (m2 < m) m2 <<= 1;
        for (int i = threadIdx.x; i < m2; i += 64) a[i] = i < m ? v[b + i] : 0xffffffffu;
        __syncthreads();
        wave_bitonic(a, m2, [](uint32_t x, uint32_t y) { return x < y; });
        const uint32_t u = wave_unique(a, m, [](uint32_t x, uint32_t y) { return x == y; },
                                       [&](uint32_t kk, uint32_t x) { v[b + kk] = x; });
        if (threadIdx.x == 0) ucnt[r] = u;
        __syncthreads();
    }
}

// rows copied to their final place (drow), one wave per 64 rows
__global__ void __launch_bounds__(64) k_copy_rows_wave(const uint64_t* __restrict__ srow, const uint32_t* __restrict__ sv,
                                                       const uint64_t* __restrict__ drow, uint64_t n,
                                                       uint32_t* __restrict__ dv)
{
    __shared__ uint64_t s_dst[65], s_src[64];
    const int lane = threadIdx.x;
    const uint64_t r0 = (uint64_t)blockIdx.x * 64;
    const uint64_t last = r0 + 64 < n ? r0 + 64 : n;
    s_dst[lane] = drow[r0 + lane < last ? r0 + lane : last];
    if (lane == 0) s_dst[64] = drow[last];
    if (r0 + lane < n) s_src[lane] = srow[r0 + lane];
    __syncthreads();
    const uint64_t end = s_dst[64];
    for (uint64_t e = s_dst[0] + lane; e < end; e += 64) {
        const int j = wave_row_of(s_dst, e);
        dv[e] = sv[s_src[j] + (e - s_dst[j])];
    }
}

__global__ void __launch_bounds__(64) k_stencil_rows_wave(const uint64_t* __restrict__ nof_row,
                                                          const uint32_t* __restrict__ nof_g,
                                                          const int32_t* __restrict__ nof_off,
                                                          const uint32_t* __restrict__ local_g, uint64_t nl,
                                                          const uint64_t* __restrict__ tmp_row, Pair* __restrict__ tmp,
                                                          uint32_t* __restrict__ ucnt, RowLists L)
{
    __shared__ Pair a[WAVE_SORT_MAX];
    const uint32_t nm = L.cnt[1];
    for (uint32_t k0 = blockIdx.x; k0 < nm; k0 += gridDim.x) {
        const uint64_t i = L.med[k0];
        const uint32_t r = local_g[i];
        const uint64_t b = nof_row[r];
        const int m = (int)(nof_row[r + 1] - b);
        int m2 = 1;
        while (m2 < m) m2 <<= 1;
        for (int k = threadIdx.x; k < m2; k += 64) {
            if (k < m) {
                const uint64_t e = b + k;
                a[k] = Pair{nof_g[e], nof_off[3 * e], nof_off[3 * e + 1], nof_off[3 * e + 2]};
            } else {
                a[k] = Pair{0xffffffffu, 0x7fffffff, 0x7fffffff, 0x7fffffff};  // sorts last
            }
        }
        __syncthreads();
        wave_bitonic(a, m2, [](const Pair& x, const Pair& y) { return pair_less(x, y); });
        Pair* out = tmp + tmp_row[i];
        const uint32_t u = wave_unique(a, m, [](const Pair& x, const Pair& y) { return pair_eq(x, y); },
                                       [&](uint32_t k, const Pair& x) { out[k] = x; });
        if (threadIdx.x == 0) ucnt[i] = u;
        __syncthreads();
    }
}

// the same for the stencil rows' (leaf, offset) pairs (see k_sort_unique_rows_seg)
template <int W, bool PEND_ONLY>
__global__ void __launch_bounds__(256) k_stencil_rows_seg(const uint64_t* __restrict__ nof_row,
                                                          const uint32_t* __restrict__ nof_g,
                                                          const int32_t* __restrict__ nof_off,
                                                          const uint32_t* __restrict__ local_g, uint64_t nl,
                                                          const uint64_t* __restrict__ tmp_row, Pair* __restrict__ tmp,
                                                          uint32_t* __restrict__ ucnt, RowLists L)
{
    constexpr int R = 64 / W;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const int lane = threadIdx.x & 63, sl = lane & (W - 1), seg = lane / W;
    const uint64_t segmask = (W >= 64 ? ~0ull : ((1ull << (W & 63)) - 1ull)) << (seg * W);
    if constexpr (PEND_ONLY) {  // W == 64: a wave per row the 16-lane pass left
        const uint32_t np = L.cnt[0];
        for (uint64_t k = wave; k < np; k += waves) {
            const uint64_t i = L.pend[k];
            const uint32_t r = local_g[i];
            const uint64_t b = nof_row[r];
            const int m = (int)(nof_row[r + 1] - b);
            if (m > 64) {
                if (lane == 0) {
                    ucnt[i] = m > WAVE_SORT_MAX ? ROW_LONG : ROW_MEDIUM;
                    if (m <= WAVE_SORT_MAX) L.med[atomicAdd(&L.cnt[1], 1u)] = (uint32_t)i;
                }
                continue;
            }
            Pair x{0xffffffffu, 0x7fffffff, 0x7fffffff, 0x7fffffff};
            if (lane < m) {
                const uint64_t e = b + lane;
                x = Pair{nof_g[e], nof_off[3 * e], nof_off[3 * e + 1], nof_off[3 * e + 2]};
            }
            x = seg_sort<64>(x, [](const Pair& a, const Pair& c) { return pair_less_(a, c); });
            Pair prev;
            prev.g = __shfl_up(x.g, 1, 64);
            prev.x = __shfl_up(x.x, 1, 64);
            prev.y = __shfl_up(x.y, 1, 64);
            prev.z = __shfl_up(x.z, 1, 64);
            const bool keep = lane < m && (lane == 0 || !pair_eq(x, prev));
            const uint64_t mask = __ballot(keep);
            if (keep) tmp[tmp_row[i] + __popcll(mask & ((1ull << lane) - 1ull))] = x;
            if (lane == 0) ucnt[i] = (uint32_t)__popcll(mask);
        }
        return;
    }
    for (uint64_t i0 = wave * R; i0 < nl; i0 += waves * R) {
        const uint64_t i = i0 + seg;
        bool active = i < nl;
        uint64_t b = 0;
        int m = 0;
        bool pend = false;
        if (active) {
            const uint32_t r = local_g[i];
            b = nof_row[r];
            m = (int)(nof_row[r + 1] - b);
            if (m > W) {
                pend = true;
                if (sl == 0) ucnt[i] = ROW_PEND;
                active = false;
            }
        }
        if (__ballot(pend && sl == 0)) {
            const uint32_t pk = wave_reserve(&L.cnt[0], pend && sl == 0 ? 1u : 0u);
            if (pend && sl == 0) L.pend[pk] = (uint32_t)i;
        }
        if (!__ballot(active)) continue;
        Pair x{0xffffffffu, 0x7fffffff, 0x7fffffff, 0x7fffffff};
        if (active && sl < m) {
            const uint64_t e = b + sl;
            x = Pair{nof_g[e], nof_off[3 * e], nof_off[3 * e + 1], nof_off[3 * e + 2]};
        }
        x = seg_sort<W>(x, [](const Pair& a, const Pair& c) { return pair_less_(a, c); });
        Pair prev;
        prev.g = __shfl_up(x.g, 1, W);
        prev.x = __shfl_up(x.x, 1, W);
        prev.y = __shfl_up(x.y, 1, W);
        prev.z = __shfl_up(x.z, 1, W);
        const bool keep = active && sl < m && (sl == 0 || !pair_eq(x, prev));
        const uint64_t mask = __ballot(keep);
        if (keep) tmp[tmp_row[i] + __popcll(mask & segmask & ((1ull << lane) - 1ull))] = x;
        if (active && sl == 0) ucnt[i] = (uint32_t)__popcll(mask & segmask);
    }
}

// stencil rows' final form: storage slot + offset of each unique entry
__global__ void __launch_bounds__(64) k_stencil_slots_wave(const uint64_t* __restrict__ tmp_row,
                                                           const Pair* __restrict__ tmp,
                                                           const uint64_t* __restrict__ st_row, uint64_t nl,
                                                           const uint32_t* __restrict__ slot_of_g,
                                                           uint32_t* __restrict__ st_slot, int32_t* __restrict__ st_off)
{
    __shared__ uint64_t s_dst[65], s_src[64];
    const int lane = threadIdx.x;
    const uint64_t r0 = (uint64_t)blockIdx.x * 64;
    const uint64_t last = r0 + 64 < nl ? r0 + 64 : nl;
    s_dst[lane] = st_row[r0 + lane < last ? r0 + lane : last];
    if (lane == 0) s_dst[64] = st_row[last];
    if (r0 + lane < nl) s_src[lane] = tmp_row[r0 + lane];
    __syncthreads();
    const uint64_t end = s_dst[64];
    for (uint64_t o = s_dst[0] + lane; o < end; o += 64) {
        const int j = wave_row_of(s_dst, o);
        const Pair p = tmp[s_src[j] + (o - s_dst[j])];
        st_slot[o] = slot_of_g[p.g];
        st_off[3 * o + 0] = p.x;
        st_off[3 * o + 1] = p.y;
        st_off[3 * o + 2] = p.z;
    }
}

static unsigned grid_for(uint64_t n)
{
    uint64_t g = (n + 255) / 256;
    if (g > 256 * 16) g = 256 * 16;
    if (g == 0) g = 1;
    return (unsigned)g;
}

__global__ void k_check_lookup(ExView v, const uint64_t* __restrict__ leaves, uint64_t n, int32_t* err)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (ex_find(v, leaves[i]) != (int64_t)i) {
            atomicAdd(err, 1);
            atomicCAS(err + 1, 0, (int32_t)i + 1);
        }
}

static ExView view(const dccrgx_grid* grid)
{
    ExView v{};
    v.mp = grid->map;
    v.keys = grid->ex->d_keys;
    v.vals = grid->ex->d_vals;
    v.mask = grid->ex->mask;
    v.bits = grid->ex->d_bits;
    v.rank = grid->ex->d_rank;
    for (int d = 0; d < 3; d++) v.per[d] = grid->params.periodic[d] ? 1 : 0;
    return v;
}

ExView explicit_view(const dccrgx_grid* grid) { return view(grid); }

// CSR row offsets (n + 1, device, allocated here) of per-row counts on the
// device; *total (host) = row[n]
static int scan_counts_device(const uint32_t* d_cnt, uint64_t n, uint64_t** d_row, uint64_t* total, hipStream_t st)
{
    DX_HIP(ds_malloc(d_row, (n + 1) * 8, st));
    DX_TRY(device_scan_counts(d_cnt, n, *d_row, st));
    return total ? device_scan_rows_total(*d_row, n, st, total) : DCCRGX_OK;
}

__global__ void __launch_bounds__(256) k_iota(uint32_t* __restrict__ out, uint64_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = (uint32_t)i;
}

// 0, 1, ..., n-1 on the device (identity maps need no upload)
static int device_iota(uint32_t** d, uint64_t n, hipStream_t st)
{
    DX_HIP(ds_malloc(d, std::max<uint64_t>(n, 1) * 4, st));
    if (n) hipLaunchKernelGGL(k_iota, dim3(grid_for(n)), dim3(256), 0, st, *d, n);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

template <class T>
static int upload(Ctx* c, const std::vector<T>& v, T** d, hipStream_t st)
{
    *d = nullptr;
    DX_HIP(ds_malloc(d, std::max<size_t>(v.size(), 1) * sizeof(T), st));
    return dx_h2d_async(c, *d, v.data(), v.size() * sizeof(T), st);
}

// neighbors_of for a device array of cells: row (n+1, device) + optional outputs
static int nof_device(dccrgx_grid* grid, const Hood& h, const uint64_t* cells, size_t n, uint64_t* row,
                      uint64_t** ids, int32_t** off, uint32_t** gidx, uint64_t* total, hipStream_t st)
{
    const ExView v = view(grid);
    int32_t* d_err = nullptr;  // error word, then (at +8) the total
    DX_HIP(ds_malloc(&d_err, 16, st));
    DX_HIP(hipMemsetAsync(d_err, 0, 16, st));  // row[0] is written by the scan
    uint64_t* d_codes = nullptr;  // per-item cases for the entry-parallel fill
    if (ids && h.K <= 32 && n) DX_HIP(ds_malloc(&d_codes, n * 8, st));
    if (n)
        hipLaunchKernelGGL(k_ex_nof, dim3(grid_for(n)), dim3(256), 0, st, v, h.d_of_c, h.K, cells, n, row,
                           (uint64_t*)nullptr, (int32_t*)nullptr, (uint32_t*)nullptr, d_err, d_codes);
    DX_HIP(hipGetLastError());
    DX_TRY(device_scan_rows(row, n, st, nullptr));
    uint64_t back[2] = {0, 0};  // total, error word: one read-back
    {
        const D2H rb[2] = {{&back[0], d_err, 8}, {&back[1], row + n, 8}};
        DX_TRY(dx_d2h_many(grid->ctx, rb, 2, st));
    }
    *total = back[1];
    // a box of leaves cut from a larger grid (hybrid.hip): a window outside
    // the box finds no cell -- an entry of a cell at the box's edge, skipped
    const int32_t err = (int32_t)(back[0] & 0xffffffffu) & (grid->partial_leaves ? ~2 : ~0);
    if (err) {
        ds_free(d_err, st);
        ds_free(d_codes, st);
        return set_error(err & 1 ? DCCRGX_ENOTFOUND : DCCRGX_EINTERNAL,
                         err & 1 ? "cell does not exist" : "neighbor more than one level apart");
    }
    if (ids) {
        uint64_t t = std::max<uint64_t>(*total, 1);
        DX_HIP(ds_malloc(ids, t * 8, st));
        DX_HIP(ds_malloc(off, t * 12, st));
        DX_HIP(ds_malloc(gidx, t * 4, st));
        if (n && d_codes)
            hipLaunchKernelGGL(k_ex_nof_fill_codes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, v, h.d_of_c,
                               h.K, cells, n, (const uint64_t*)row, (const uint64_t*)d_codes, *ids, *off, *gidx);
        else if (n)
            hipLaunchKernelGGL(k_ex_nof_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, v, h.d_of_c, h.K,
                               cells, n, (const uint64_t*)row, *ids, *off, *gidx);
        DX_HIP(hipGetLastError());
    }
    ds_free(d_codes, st);
    ds_free(d_err, st);
    return DCCRGX_OK;
}

static int sync_slots(dccrgx_grid* grid, bool slot_map_changed);
int explicit_local_ids(const dccrgx_grid* grid, uint64_t* d_ids, hipStream_t st);

// ids of the local cells, from the device leaf list
__global__ void __launch_bounds__(256) k_local_ids(const uint64_t* __restrict__ leaves,
                                                   const uint32_t* __restrict__ local_g, uint64_t n,
                                                   uint64_t* __restrict__ out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = leaves[local_g[i]];
}

// the row lists of one sort (RowLists), freed with it
struct RowListBufs {
    RowLists L{};
    hipStream_t st = nullptr;
    int make(uint64_t n, hipStream_t s)
    {
        st = s;
        DX_HIP(ds_malloc(&L.pend, std::max<uint64_t>(n, 1) * 4, st));
        DX_HIP(ds_malloc(&L.med, std::max<uint64_t>(n, 1) * 4, st));
        DX_HIP(ds_malloc(&L.cnt, 8, st));
        DX_HIP(hipMemsetAsync(L.cnt, 0, 8, st));
        return DCCRGX_OK;
    }
    ~RowListBufs()
    {
        for (void* q : {(void*)L.pend, (void*)L.med, (void*)L.cnt}) ds_free(q, st);
    }
};

// rows (row[n + 1], `tot` entries in v) sorted and made unique in place,
// then copied compacted into a new CSR (*out_row, *out_v)
static int sort_unique_compact(const uint64_t* row, uint32_t* v, uint64_t n, uint64_t tot, uint64_t** out_row,
                               uint32_t** out_v, hipStream_t st)
{
    uint32_t* d_ucnt = nullptr;
    DX_HIP(ds_malloc(&d_ucnt, std::max<uint64_t>(n, 1) * 4, st));
    RowListBufs RL;
    DX_TRY(RL.make(n, st));
    if (n) {
        hipLaunchKernelGGL((k_sort_unique_rows_seg<16, false>), dim3((unsigned)std::min<uint64_t>((n + 15) / 16, 16384)),
                           dim3(256), 0, st, row, n, v, d_ucnt, RL.L);
        hipLaunchKernelGGL((k_sort_unique_rows_seg<64, true>), dim3((unsigned)std::min<uint64_t>((n + 3) / 4, 4096)),
                           dim3(256), 0, st, row, n, v, d_ucnt, RL.L);
        hipLaunchKernelGGL(k_sort_unique_rows_wave, dim3((unsigned)std::min<uint64_t>(n, 4096)), dim3(64), 0, st, row, n,
                           v, d_ucnt, RL.L);
        hipLaunchKernelGGL(k_sort_unique_rows, dim3(grid_for(n)), dim3(256), 0, st, row, n, v, d_ucnt);
    }
    DX_HIP(hipGetLastError());
    const int e = scan_counts_device(d_ucnt, n, out_row, nullptr, st);
    if (e != DCCRGX_OK) {
        ds_free(d_ucnt, st);
        return e;
    }
    DX_HIP(ds_malloc(out_v, std::max<uint64_t>(tot, 1) * 4, st));  // unique entries: at most tot
    if (n)
        hipLaunchKernelGGL(k_copy_rows_wave, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, row, (const uint32_t*)v,
                           (const uint64_t*)*out_row, n, *out_v);
    DX_HIP(hipGetLastError());
    ds_free(d_ucnt, st);
    return DCCRGX_OK;
}

// neighbors_to rows (ascending leaf indices) of `cells` by the reference's
// search (k_ex_nto): count, scan, fill, sort + unique
static int nto_direct(const dccrgx_grid* grid, const Hood& h, const uint64_t* cells, uint64_t n, uint64_t** out_row,
                      uint32_t** out_g, hipStream_t st)
{
    const ExView v = view(grid);
    uint64_t* d_row = nullptr;
    uint32_t* d_tmp = nullptr;
    DX_HIP(ds_malloc(&d_row, (n + 1) * 8, st));
    auto done = [&](int code) {
        ds_free(d_row, st);
        ds_free(d_tmp, st);
        return code;
    };
    if (n)  // row[0] is written by the scan
        hipLaunchKernelGGL(k_ex_nto, dim3(grid_for(n)), dim3(256), 0, st, v, (const int32_t*)h.d_to_c, h.K, cells,
                           (size_t)n, d_row, (uint32_t*)nullptr);
    uint64_t tot = 0;
    int e = device_scan_rows(d_row, n, st, &tot);
    if (e != DCCRGX_OK) return done(e);
    if (ds_malloc(&d_tmp, std::max<uint64_t>(tot, 1) * 4, st) != hipSuccess)
        return done(set_error(DCCRGX_ENOMEM, "neighbors_to of %llu cells", (unsigned long long)n));
    if (n)
        hipLaunchKernelGGL(k_ex_nto, dim3(grid_for(n)), dim3(256), 0, st, v, (const int32_t*)h.d_to_c, h.K, cells,
                           (size_t)n, d_row, d_tmp);
    return done(sort_unique_compact(d_row, d_tmp, n, tot, out_row, out_g, st));
}


int explicit_init(dccrgx_grid* grid, const uint64_t* leaves, size_t n, uint64_t* d_leaves,
                  std::vector<uint64_t>* take, uint64_t first_leaf)
{
    Ctx* ctx = grid->ctx;
    hipStream_t st = ctx->compute;
    auto* E = new Explicit();
    E->d_leaves = d_leaves;  // adopted (ascending, unique, = leaves): freed with E from here on
    E->ctx = ctx;
    E->one_rank = ctx->comm_size == 1;
    if (n == 0 || n >= (1ull << 32) || (!leaves && (!d_leaves || !E->one_rank))) {
        explicit_free(E);
        return set_error(DCCRGX_EINVAL, "leaf count %zu", n);
    }
    PhaseTimer T("explicit_init");
    if (grid->spare_host) {  // the previous state's host arrays: their capacity is reused
        Explicit* S = grid->spare_host;
        E->leaves_.swap(S->leaves_);
        E->local_.swap(S->local_);
        E->local_g.swap(S->local_g);
        E->owner.swap(S->owner);
        E->slot_ids_.swap(S->slot_ids_);
        E->slot_of_g.swap(S->slot_of_g);
        E->dir.swap(S->dir);
        E->local_.clear();
        E->slot_ids_.clear();
        delete S;
        grid->spare_host = nullptr;
    }
    grid->ex = E;
    if (!leaves) {  // one rank, the device's list (amr_dev_decide): fetched if host code asks
        E->host_leaves = false;
        E->n = n;
    } else {
        if (take && take->data() == leaves && take->size() == n) E->leaves_.swap(*take);  // the caller's list, moved
        else E->leaves_.assign(leaves, leaves + n);
        if (!d_leaves) {
            if (!std::is_sorted(E->leaves_.begin(), E->leaves_.end())) std::sort(E->leaves_.begin(), E->leaves_.end());
            E->leaves_.erase(std::unique(E->leaves_.begin(), E->leaves_.end()), E->leaves_.end());
        }
        DX_CHECK(E->leaves_[0] > 0 && E->leaves_.back() <= grid->map.last_cell, DCCRGX_EINVAL, "invalid cell %llu",
                 (unsigned long long)(E->leaves_[0] == 0 ? 0 : E->leaves_.back()));
        E->n = E->leaves_.size();
        first_leaf = E->leaves_[0];
    }
    E->dir_valid = false;  // built on the first host lookup
    uint64_t cap = 16;
    while (cap < 2 * E->n) cap <<= 1;
    if (!E->d_leaves) DX_TRY(upload(grid->ctx, E->leaves_, &E->d_leaves, st));
    // the rank bitmap when it is small (at most 1 GiB, and at most 16x the hash)
    const uint64_t nw = (grid->map.last_cell >> 6) + 1;
    if (nw <= (1ull << 26) && nw * 12 <= 16 * cap * 12) {
        E->nwords = nw;
        DX_HIP(ds_malloc(&E->d_bits, nw * 8, st));
        DX_HIP(ds_malloc(&E->d_rank, nw * 4, st));
        hipLaunchKernelGGL(k_bits_rank, dim3(grid_for(nw)), dim3(256), 0, st, E->d_leaves, E->n, nw, E->d_rank,
                           E->d_bits);
        hipLaunchKernelGGL(k_bits_set, dim3(grid_for(E->n)), dim3(256), 0, st, E->d_leaves, E->n,
                           (unsigned long long*)E->d_bits);
    } else {
        E->mask = cap - 1;
        DX_HIP(ds_malloc(&E->d_keys, cap * 8, st));
        DX_HIP(ds_malloc(&E->d_vals, cap * 4, st));
        DX_HIP(hipMemsetAsync(E->d_keys, 0, cap * 8, st));
        hipLaunchKernelGGL(k_hash_insert, dim3(grid_for(E->n)), dim3(256), 0, st, E->d_leaves, E->n,
                           (unsigned long long*)E->d_keys, E->d_vals, E->mask);
    }
    DX_HIP(hipGetLastError());
    T.lap("leaves+lookup");
    if (test_opt(OPT_CHECK_INIT, 0)) {  // device leaves and lookups against the host list
        const std::vector<uint64_t>& L = E->leaves();
        std::vector<uint64_t> back(E->n);
        DX_TRY(dx_d2h(ctx, back.data(), E->d_leaves, E->n * 8, st));
        uint64_t bad = 0;
        for (uint64_t i = 0; i < E->n; i++) bad += back[i] != L[i];
        int32_t* d_e = nullptr;
        DX_HIP(dx_malloc(&d_e, 8));
        DX_HIP(hipMemsetAsync(d_e, 0, 8, st));
        hipLaunchKernelGGL(k_check_lookup, dim3(grid_for(E->n)), dim3(256), 0, st, view(grid), E->d_leaves, E->n, d_e);
        int32_t e[2] = {0, 0};
        DX_TRY(dx_d2h(ctx, e, d_e, 8, st));
        dx_free(d_e);
        std::fprintf(stderr, "[dccrgx] check_init n %llu leaves differing %llu lookups failing %d first %d bitmap %d\n",
                     (unsigned long long)E->n, (unsigned long long)bad, e[0], e[1] - 1, E->d_bits != nullptr);
        DX_CHECK(!bad && !e[0], DCCRGX_EINTERNAL, "check_init: %llu leaves of the host list differ from the "
                 "device list, %d lookups fail", (unsigned long long)bad, e[0]);
    }
    // ownership: the process of the level-0 ancestor (no load balancing),
    // block partition or the grid's SFC table
    E->part = make_partition(grid->map.nlevel0, ctx->comm_size);
    if (E->one_rank) {  // one process owns every leaf: owner 0 and identity maps, so no host arrays
        E->owner.clear();
        E->local_g.clear();
        E->slot_of_g.clear();
        E->slot_identity = true;
        DX_TRY(ctx_identity(ctx, E->n, &E->d_local_g, st));
    } else {
        const std::vector<uint64_t>& L = E->leaves_;
        E->local_g.clear();
        E->owner.resize(E->n);
        for (uint64_t i = 0; i < E->n; i++) {
            uint64_t idx[3];
            int l;
            map_indices(grid->map, L[i], idx, &l);
            const uint64_t l0 = l == 0 ? L[i] : map_cell(grid->map, idx, 0);
            E->owner[i] = level0_owner(grid, E->part, l0);
            if (E->owner[i] == ctx->rank) {
                E->local_.push_back(L[i]);
                E->local_g.push_back((uint32_t)i);
            }
        }
        DX_TRY(upload(grid->ctx, E->local_g, &E->d_local_g, st));
        // storage: the local cells first (ghosts are added by the neighborhoods)
        E->slot_ids_ = E->local_;
        E->slot_of_g.assign(E->n, NO_SLOT);
        for (uint64_t i = 0; i < E->local_.size(); i++) E->slot_of_g[E->local_g[i]] = (uint32_t)i;
    }
    grid->n_local = E->n_local();
    grid->first_local = !grid->n_local ? 0 : E->one_rank ? first_leaf : E->local_[0];
    DX_TRY(ctx_identity(ctx, grid->n_local, &E->d_local_slot, st));  // local position -> slot: identity
    T.lap("owners+local");
    DX_TRY(sync_slots(grid, true));
    T.lap("sync_slots");
    return DCCRGX_OK;
}

// device copies of the slot map and per-slot levels; n_slots
__global__ void __launch_bounds__(256) k_slot_levels(MapParams mp, const uint64_t* __restrict__ leaves,
                                                     const uint32_t* __restrict__ local_g, uint64_t n,
                                                     uint8_t* __restrict__ level)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += stride)
        level[q] = (uint8_t)map_level(mp, leaves[local_g[q]]);
}

// device copies of the slot map (when it changed) and of the per-slot levels
// (slots only ever append, or roll back: the local cells' levels come from
// the device leaf list, appended slots' from the host); n_slots
static int sync_slots(dccrgx_grid* grid, bool slot_map_changed)
{
    Explicit* E = grid->ex;
    hipStream_t st = grid->ctx->compute;
    const uint64_t ns = E->n_slot_ids(), nl = E->n_local();
    if (slot_map_changed || !E->d_slot_of_g) {
        if (!ctx_is_identity(grid->ctx, E->d_slot_of_g)) dx_free(E->d_slot_of_g);
        E->d_slot_of_g = nullptr;
        if (E->slot_identity) DX_TRY(ctx_identity(grid->ctx, E->n, &E->d_slot_of_g, st));  // one rank: leaf g in slot g
        else DX_TRY(upload(grid->ctx, E->slot_of_g, &E->d_slot_of_g, st));
    }
    if (ns > E->d_level_cap || !E->d_level) {
        const uint64_t cap = std::max<uint64_t>(ns + ns / 4, 16);
        uint8_t* d = nullptr;
        DX_HIP(dx_malloc(&d, cap));
        if (E->d_level && E->d_level_n) DX_HIP(hipMemcpyAsync(d, E->d_level, E->d_level_n, hipMemcpyDeviceToDevice, st));
        dx_free(E->d_level);  // waits for the copy
        E->d_level = d;
        E->d_level_cap = cap;
    }
    if (E->d_level_n == 0 && nl) {
        hipLaunchKernelGGL(k_slot_levels, dim3(grid_for(nl)), dim3(256), 0, st, grid->map, E->d_leaves, E->d_local_g,
                           nl, E->d_level);
        DX_HIP(hipGetLastError());
        E->d_level_n = nl;
    }
    E->d_level_n = std::min(E->d_level_n, ns);
    if (ns > E->d_level_n) {
        std::vector<uint8_t> tail(ns - E->d_level_n);
        const uint64_t k0 = E->d_level_n;
        parallel_ranges(ns - k0, 1u << 15, [&](size_t b, size_t e) {
            for (size_t k = b; k < e; k++) tail[k] = (uint8_t)map_level(grid->map, E->slot_id(k0 + k));
        });
        DX_TRY(dx_h2d_async(grid->ctx, E->d_level + E->d_level_n, tail.data(), tail.size(), st));
        E->d_level_n = ns;
    }
    if (!grid->rebuilding) DX_HIP(hipStreamSynchronize(st));  // a rebuild synchronises once, at its end
    grid->n_slots = ns;
    return DCCRGX_OK;
}

// every field grows to `ns` slots (new slots zero, value-initialised ghosts
// as allocate_copies_of_remote_neighbors, dccrg.hpp:7153-7184); all new
// arrays are allocated before any pointer is swapped
static int grow_fields(dccrgx_grid* grid, uint64_t old_ns, uint64_t ns)
{
    hipStream_t st = grid->ctx->compute;
    std::vector<void*> np(grid->fields.size(), nullptr);
    int s = DCCRGX_OK;
    for (size_t i = 0; i < grid->fields.size() && s == DCCRGX_OK; i++) {
        const Field& F = grid->fields[i];
        if (F.variable) continue;
        if (dx_malloc(&np[i], std::max<uint64_t>(ns, 1) * F.elem) != hipSuccess) {
            np[i] = nullptr;
            s = set_error(DCCRGX_ENOMEM, "out of device memory for %llu ghost slots", (unsigned long long)ns);
            break;
        }
        if (hipMemsetAsync(np[i], 0, std::max<uint64_t>(ns, 1) * F.elem, st) != hipSuccess ||
            (old_ns && hipMemcpyAsync(np[i], F.ptr, old_ns * F.elem, hipMemcpyDeviceToDevice, st) != hipSuccess))
            s = set_error(DCCRGX_EHIP, "growing field %zu failed", i);
    }
    if (s == DCCRGX_OK && hipStreamSynchronize(st) != hipSuccess) s = set_error(DCCRGX_EHIP, "growing fields failed");
    if (s != DCCRGX_OK) {
        for (void* q : np) dx_free(q);
        return s;
    }
    for (size_t i = 0; i < grid->fields.size(); i++) {
        Field& F = grid->fields[i];
        if (F.variable) {  // new slots hold zero elements
            F.count.resize(ns, 0);
            F.off.resize(ns, F.pool_bytes);
            F.epoch = next_var_epoch();
            continue;
        }
        dx_free(F.ptr);
        F.ptr = np[i];
        F.cap_bytes = 0;  // exact size
    }
    return DCCRGX_OK;
}

int explicit_add_slots(dccrgx_grid* grid, const std::vector<uint64_t>& ids)
{
    Explicit* E = grid->ex;
    const uint64_t old_ns = E->n_slot_ids();
    bool leaf_slot = false;  // a leaf got a (ghost) slot: the slot map changes
    E->extra.reserve(E->extra.size() + ids.size());
    uint64_t ns = old_ns;
    for (uint64_t c : ids) {
        const int64_t g = E->find(c);
        if ((g >= 0 && (E->slot_identity || E->slot_of_g[g] != NO_SLOT)) || E->extra.count(c)) continue;  // has a slot
        DX_CHECK(g < 0 || g < (int64_t)E->slot_of_g.size(), DCCRGX_EINTERNAL, "no slot map for leaf %llu",
                 (unsigned long long)c);
        const uint32_t s = (uint32_t)ns++;
        E->push_slot(c);
        E->extra.set(c, s);
        if (g >= 0) {
            E->slot_of_g[g] = s;
            leaf_slot = true;
            E->slot_identity = false;
        }
    }
    DX_CHECK(ns < NO_SLOT, DCCRGX_EINVAL, "%llu storage slots on one rank", (unsigned long long)ns);
    if (ns == old_ns) return DCCRGX_OK;
    if (!E->defer_fields) {
        const int s = grow_fields(grid, old_ns, ns);
        if (s != DCCRGX_OK) {  // undo the new slots
            for (uint64_t k = old_ns; k < ns; k++) {
                const uint64_t c = E->slot_id(k);
                E->extra.erase(c);
                const int64_t g = E->find(c);
                if (g >= 0) E->slot_of_g[g] = NO_SLOT;
            }
            E->truncate_slots(old_ns);
            return s;
        }
    }
    return sync_slots(grid, leaf_slot);
}

int explicit_add_retired(dccrgx_grid* grid, const std::vector<uint64_t>& ids)
{
    Explicit* E = grid->ex;
    E->retired.clear();
    if (ids.empty()) return DCCRGX_OK;
    const uint64_t ns = E->n_slot_ids() + ids.size();
    DX_CHECK(ns < NO_SLOT, DCCRGX_EINVAL, "%llu storage slots on one rank", (unsigned long long)ns);
    DX_CHECK(E->defer_fields, DCCRGX_EINTERNAL, "retired slots outside a rebuild");
    E->retired = ids;
    E->ret_slot0 = E->n_slot_ids();
    for (uint64_t c : ids) E->push_slot(c);
    return sync_slots(grid, false);
}

int explicit_create(dccrgx_grid* grid, const uint64_t* leaves, size_t n)
{
    DX_TRY(explicit_init(grid, leaves, n));
    Hood h;
    h.id = DCCRGX_DEFAULT_NEIGHBORHOOD_ID;
    // default items, dccrg.hpp:8017-8076
    const uint32_t hl = grid->params.neighborhood_length;
    if (hl == 0) {
        const int32_t f[6][3] = {{0, 0, -1}, {0, -1, 0}, {-1, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
        for (auto& it : f) h.items.insert(h.items.end(), it, it + 3);
    } else {
        const int hh = (int)hl;
        for (int z = -hh; z <= hh; z++)
            for (int y = -hh; y <= hh; y++)
                for (int x = -hh; x <= hh; x++)
                    if (x || y || z) h.items.insert(h.items.end(), {x, y, z});
    }
    grid->hoods[h.id] = h;
    return explicit_build_hood(grid, grid->hoods[h.id]);
}

// Explicit::leaves() of a list held on the device only: one copy, made once
// (a lookup may ask from several host threads)
static int fetch_leaves(const Explicit* E)
{
    static std::mutex m;
    std::lock_guard<std::mutex> g(m);
    if (E->host_leaves) return DCCRGX_OK;
    E->leaves_.resize(E->n);
    DX_TRY(dx_d2h(E->ctx, E->leaves_.data(), E->d_leaves, E->n * 8, E->ctx->compute));
    E->host_leaves = true;
    return DCCRGX_OK;
}

int explicit_host_leaves(const dccrgx_grid* grid)
{
    if (!grid || grid->uniform || !grid->ex || grid->ex->host_leaves) return DCCRGX_OK;
    return fetch_leaves(grid->ex);
}

// the backstop of Explicit::leaves(): every public entry point that reaches
// host lookups fetches first through explicit_host_leaves, which returns
// the error instead (DCCRGX_EHIP); reaching this with a failing copy is a bug
void explicit_fetch_leaves(const Explicit* E)
{
    if (fetch_leaves(E) != DCCRGX_OK) {
        std::fprintf(stderr, "dccrgx: reading the leaf list from the device failed: %s\n", dccrgx_last_error());
        std::abort();
    }
}

void explicit_recycle(dccrgx_grid* grid, Explicit* E)
{
    if (!E) return;
    auto* S = new Explicit();
    S->leaves_.swap(E->leaves_);  // (empty while the leaves are on the device only)
    S->local_.swap(E->local_);
    S->local_g.swap(E->local_g);
    S->owner.swap(E->owner);
    S->slot_ids_.swap(E->slot_ids_);
    S->slot_of_g.swap(E->slot_of_g);
    S->dir.swap(E->dir);
    explicit_free(E);
    delete grid->spare_host;
    grid->spare_host = S;
}

void explicit_free(Explicit* E)
{
    if (!E) return;
    FreeBatch fb;
    for (void* q : {(void*)E->d_leaves, (void*)E->d_keys, (void*)E->d_vals, (void*)E->d_bits, (void*)E->d_rank,
                    (void*)E->d_local_g, (void*)E->d_level, (void*)E->d_slot_of_g, (void*)E->d_local_slot,
                    (void*)E->d_ret})
        if (!ctx_is_identity(E->ctx, q)) fb.add(q);
    for (auto& kv : E->hl)
        for (void* q : {(void*)kv.second.d_inner_pos, (void*)kv.second.d_outer_pos, (void*)kv.second.d_all_pos})
            if (!ctx_is_identity(E->ctx, q)) fb.add(q);
    delete E;
}

// retired cells' data is no longer addressable (their slots are reused by
// the next rebuild)
void explicit_clear_retired(Explicit* E)
{
    E->retired.clear();
    E->n_ret = 0;  // the table stays allocated until E is freed
}

void explicit_destroy(dccrgx_grid* grid)
{
    explicit_free(grid->ex);
    grid->ex = nullptr;
    delete grid->spare_host;
    grid->spare_host = nullptr;
}

// host copies of a neighborhood's device CSRs (neighbors_of / neighbors_to
// as global leaf indices), made once per build when host code needs them
int explicit_host_lists(const dccrgx_grid* grid, const Hood& h)
{
    Explicit* E = grid->ex;
    Explicit::HoodLists& L = E->hl[h.id];
    if (L.host_valid) return DCCRGX_OK;
    Ctx* ctx = grid->ctx;
    hipStream_t st = ctx->compute;
    const uint64_t N = h.n_rows;  // the local cells' rows (row = local position)
    L.h_nof_row.resize(N + 1);
    L.h_nto_row.resize(N + 1);
    DX_TRY(dx_d2h(ctx, L.h_nof_row.data(), h.d_nof_row, (N + 1) * 8, st));
    DX_TRY(dx_d2h(ctx, L.h_nto_row.data(), h.d_nto_row, (N + 1) * 8, st));
    L.h_nof_g.resize(L.h_nof_row[N]);
    L.h_nto_g.resize(L.h_nto_row[N]);
    DX_TRY(dx_d2h(ctx, L.h_nof_g.data(), h.d_nof_g, L.h_nof_g.size() * 4, st));
    DX_TRY(dx_d2h(ctx, L.h_nto_g.data(), h.d_nto_g, L.h_nto_g.size() * 4, st));
    L.host_valid = true;
    return DCCRGX_OK;
}

// the rows of leaves gs[]: row[i + 1] = neighbors_of + neighbors_to length,
// alen[i] = neighbors_of length; then the rows concatenated (of, then to)
__global__ void __launch_bounds__(256) k_rows_len(const uint32_t* __restrict__ gs, uint64_t n,
                                                  const uint64_t* __restrict__ arow, const uint64_t* __restrict__ brow,
                                                  uint64_t* __restrict__ row, uint64_t* __restrict__ alen)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t g = gs[i];
        alen[i] = arow[g + 1] - arow[g];
        row[i + 1] = alen[i] + (brow[g + 1] - brow[g]);
    }
}

__global__ void __launch_bounds__(256) k_rows_cat(const uint32_t* __restrict__ gs, uint64_t n,
                                                  const uint64_t* __restrict__ arow, const uint32_t* __restrict__ aval,
                                                  const uint64_t* __restrict__ brow, const uint32_t* __restrict__ bval,
                                                  const uint64_t* __restrict__ row, uint32_t* __restrict__ out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t g = gs[i];
        uint64_t w = row[i];
        for (uint64_t e = arow[g]; e < arow[g + 1]; e++) out[w++] = aval[e];
        for (uint64_t e = brow[g]; e < brow[g + 1]; e++) out[w++] = bval[e];
    }
}

int explicit_fetch_rows(const dccrgx_grid* grid, const Hood& h, const std::vector<uint32_t>& leaves)
{
    Explicit* E = grid->ex;
    Explicit::HoodLists& L = E->hl[h.id];
    if (L.host_valid) return DCCRGX_OK;  // the whole lists are on the host already
    std::vector<uint32_t> want;  // leaves of this rank (the rows held here) not fetched yet
    for (uint32_t g : leaves)
        if (g < E->n && E->row_of(g) >= 0 && !L.row_at.count(g)) want.push_back(g);
    std::sort(want.begin(), want.end());
    want.erase(std::unique(want.begin(), want.end()), want.end());
    if (want.empty()) return DCCRGX_OK;
    std::vector<uint32_t> rows(want.size());
    for (size_t i = 0; i < want.size(); i++) rows[i] = (uint32_t)E->row_of(want[i]);
    Ctx* ctx = grid->ctx;
    hipStream_t st = ctx->compute;
    const uint64_t n = want.size();
    uint32_t* d_g = nullptr;
    uint64_t* d_row = nullptr;  // n + 1 row pointers, then n neighbors_of lengths
    uint32_t* d_out = nullptr;
    DX_HIP(ds_malloc(&d_g, n * 4, st));
    DX_HIP(ds_malloc(&d_row, (2 * n + 1) * 8, st));
    auto done = [&](int code) {
        (void)ds_free(d_g, st);
        (void)ds_free(d_row, st);
        if (d_out) (void)ds_free(d_out, st);
        return code;
    };
    int s = dx_h2d_async(ctx, d_g, rows.data(), n * 4, st);
    if (s != DCCRGX_OK) return done(s);
    hipLaunchKernelGGL(k_rows_len, dim3(grid_for(n)), dim3(256), 0, st, (const uint32_t*)d_g, n, h.d_nof_row,
                       h.d_nto_row, d_row, d_row + n + 1);
    uint64_t total = 0;
    if ((s = device_scan_rows(d_row, n, st, &total)) != DCCRGX_OK) return done(s);
    if (ds_malloc(&d_out, std::max<uint64_t>(total, 1) * 4, st) != hipSuccess)
        return done(set_error(DCCRGX_ENOMEM, "row cache"));
    hipLaunchKernelGGL(k_rows_cat, dim3(grid_for(n)), dim3(256), 0, st, (const uint32_t*)d_g, n, h.d_nof_row,
                       h.d_nof_g, h.d_nto_row, h.d_nto_g, (const uint64_t*)d_row, d_out);
    std::vector<uint64_t> row(2 * n + 1);
    if ((s = dx_d2h(ctx, row.data(), d_row, (2 * n + 1) * 8, st)) != DCCRGX_OK) return done(s);
    const uint64_t base = L.row_vals.size();
    L.row_vals.resize(base + total);
    if ((s = dx_d2h(ctx, L.row_vals.data() + base, d_out, total * 4, st)) != DCCRGX_OK) return done(s);
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t a = row[n + 1 + i];
        L.row_at[want[i]] = {base + row[i], a, base + row[i] + a, row[i + 1] - row[i] - a};
    }
    return done(DCCRGX_OK);
}

int explicit_host_lists(const dccrgx_grid* grid, int32_t hood_id)
{
    const Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    return explicit_host_lists(grid, *h);
}

// Incremental neighbors_of after a refinement round (rebuild
// around the changed cells).  A kept leaf whose old row references no gone
// leaf has the same row as before -- its windows are still covered by the
// same leaves, since new leaves only cover regions that gone leaves covered
// -- so its ids and offsets are copied and only the leaf indices remapped;
// rows of new leaves and of kept leaves next to a change are recomputed.
__global__ void __launch_bounds__(256) k_inc_new2old(ExView oldv, const uint64_t* __restrict__ leaves, uint64_t n,
                                                     uint32_t* __restrict__ new2old, uint32_t* __restrict__ old2new)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
        const int64_t o = ex_find(oldv, leaves[j]);
        new2old[j] = o < 0 ? NO_SLOT : (uint32_t)o;
        if (o >= 0) old2new[o] = (uint32_t)j;
    }
}

// Rows are the local cells' by local position; with one process position
// == leaf index (the maps below are null: identity), with several a local
// position maps to its leaf through local_g and a leaf to its position
// through slot_of_g (local slots are [0, n_local)).  A kept leaf local
// before is local after (owners follow the level-0 ancestor).
__device__ inline uint32_t pos_map(const uint32_t* m, uint64_t i) { return m ? m[i] : (uint32_t)i; }

// old rows that reference a gone leaf (or whose cell is gone)
__global__ void __launch_bounds__(256) k_inc_touched(const uint64_t* __restrict__ row, const uint32_t* __restrict__ g,
                                                     uint64_t n, const uint32_t* __restrict__ old_pos_leaf,
                                                     const uint32_t* __restrict__ flags, uint32_t gone,
                                                     uint8_t* __restrict__ touched)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x; o < n; o += stride) {
        bool t = (flags[pos_map(old_pos_leaf, o)] & gone) != 0;
        for (uint64_t e = row[o]; e < row[o + 1] && !t; e++) t = (flags[g[e]] & gone) != 0;
        touched[o] = t ? 1 : 0;
    }
}

// the old row of new row j, or NO_SLOT: recomputed
__device__ inline uint32_t inc_src_row(uint64_t j, const uint32_t* new_pos_leaf, const uint32_t* new2old,
                                       const uint32_t* old_leaf_pos, uint64_t old_rows, const uint8_t* touched)
{
    const uint32_t o = new2old[pos_map(new_pos_leaf, j)];
    if (o == NO_SLOT) return NO_SLOT;
    const uint32_t p = pos_map(old_leaf_pos, o);
    return p < old_rows && !touched[p] ? p : NO_SLOT;
}

// counts of copied rows; the other leaves listed for recomputation
__global__ void __launch_bounds__(256) k_inc_count(const uint32_t* __restrict__ new2old,
                                                   const uint8_t* __restrict__ touched, const uint64_t* __restrict__ orow,
                                                   const uint64_t* __restrict__ leaves, uint64_t n,
                                                   const uint32_t* __restrict__ new_pos_leaf,
                                                   const uint32_t* __restrict__ old_leaf_pos, uint64_t old_rows,
                                                   uint64_t* __restrict__ row, uint32_t* __restrict__ aff,
                                                   uint64_t* __restrict__ aff_ids, uint32_t* __restrict__ naff)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
        const uint32_t o = inc_src_row(j, new_pos_leaf, new2old, old_leaf_pos, old_rows, touched);
        const bool copied = o != NO_SLOT;
        const uint32_t k = wave_reserve(naff, copied ? 0u : 1u);
        if (copied) {
            row[j + 1] = orow[o + 1] - orow[o];
            continue;
        }
        aff[k] = (uint32_t)j;
        aff_ids[k] = leaves[pos_map(new_pos_leaf, j)];
    }
}

__global__ void __launch_bounds__(256) k_inc_aff_rows(const uint32_t* __restrict__ aff, uint64_t naff,
                                                      const uint64_t* __restrict__ cnt_row, uint64_t* __restrict__ row,
                                                      uint64_t* __restrict__ start, int fill)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < naff; k += stride) {
        if (!fill) row[aff[k] + 1] = cnt_row[k + 1];  // the count pass' counts into the full row array
        else start[k] = row[aff[k]];                  // the recomputed rows' places
    }
}

// copied rows: one wave per 64 new leaves, consecutive lanes on consecutive entries
__global__ void __launch_bounds__(64) k_inc_copy(const uint32_t* __restrict__ new2old, const uint8_t* __restrict__ touched,
                                                 uint64_t n, const uint32_t* __restrict__ new_pos_leaf,
                                                 const uint32_t* __restrict__ old_leaf_pos, uint64_t old_rows,
                                                 const uint64_t* __restrict__ orow,
                                                 const uint64_t* __restrict__ oid, const int32_t* __restrict__ ooff,
                                                 const uint32_t* __restrict__ og, const uint32_t* __restrict__ old2new,
                                                 const uint64_t* __restrict__ row, uint64_t* __restrict__ ids,
                                                 int32_t* __restrict__ off, uint32_t* __restrict__ g)
{
    __shared__ uint64_t s_dst[65], s_src[64];
    const int lane = threadIdx.x;
    const uint64_t r0 = (uint64_t)blockIdx.x * 64;
    const uint64_t j = r0 + lane;
    // rows of recomputed leaves take no entries here (empty source runs)
    uint64_t len = 0, src = 0;
    if (j < n) {
        const uint32_t o = inc_src_row(j, new_pos_leaf, new2old, old_leaf_pos, old_rows, touched);
        if (o != NO_SLOT) {
            src = orow[o];
            len = orow[o + 1] - src;
        }
    }
    s_src[lane] = src;
    // a run per lane: the copied rows are not contiguous in the output when
    // recomputed rows sit between them, so each entry finds its lane
    __shared__ uint64_t s_len[64], s_out[64];
    s_len[lane] = len;
    s_out[lane] = j < n ? row[j] : 0;
    __syncthreads();
    if (lane == 0) {
        uint64_t acc = 0;
        for (int k = 0; k < 64; k++) {
            s_dst[k] = acc;
            acc += s_len[k];
        }
        s_dst[64] = acc;
    }
    __syncthreads();
    const uint64_t tot = s_dst[64];
    for (uint64_t e = lane; e < tot; e += 64) {
        int lo = 0, hi = 64;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s_dst[mid] <= e) lo = mid;
            else hi = mid;
        }
        const uint64_t k = e - s_dst[lo];
        const uint64_t se = s_src[lo] + k, de = s_out[lo] + k;
        ids[de] = oid[se];
        g[de] = old2new[og[se]];
        off[3 * de + 0] = ooff[3 * se + 0];
        off[3 * de + 1] = ooff[3 * se + 1];
        off[3 * de + 2] = ooff[3 * se + 2];
    }
}

static bool incremental_rebuild(uint64_t n)
{
    const int64_t force = test_opt(OPT_INCREMENTAL, -1);  // 1 / 0: always / never (tests)
    if (force >= 0) return force != 0;
    return n >= (1ull << 20);  // below, one full pass costs less than the extra launches
}

// the maps of an incremental neighbors_of, kept for the stencil rows
struct IncMaps {
    uint32_t* n2o = nullptr;     // new leaf -> old leaf (NO_SLOT: new)
    uint32_t* o2n = nullptr;     // old leaf -> new leaf (NO_SLOT: gone)
    uint8_t* touched = nullptr;  // old leaf: its row was recomputed
    uint32_t* aff = nullptr;     // new leaves whose rows were recomputed
    uint64_t naff = 0;
    hipStream_t st = nullptr;
    ~IncMaps()
    {
        for (void* q : {(void*)n2o, (void*)o2n, (void*)touched, (void*)aff}) ds_free(q, st);
    }
};

// neighbors_of of every leaf from the previous lists (see above); `keep`
// takes over the maps
static int nof_incremental(dccrgx_grid* grid, Hood& h, const NofHint& H, uint64_t* total, hipStream_t st,
                           IncMaps* keep)
{
    Explicit* E = grid->ex;
    Ctx* ctx = grid->ctx;
    const uint64_t N = E->n, oN = H.old_ex->n;
    const Hood& oh = *H.old_h;
    // rows: local positions (several processes: through the position maps)
    const bool per_rank = ctx->comm_size > 1;
    const uint64_t R = per_rank ? E->n_local() : N, oR = per_rank ? oh.n_rows : oN;
    const uint32_t* new_pos_leaf = per_rank ? E->d_local_g : nullptr;
    const uint32_t* old_pos_leaf = per_rank ? H.old_ex->d_local_g : nullptr;
    const uint32_t* old_leaf_pos = per_rank ? H.old_ex->d_slot_of_g : nullptr;
    const ExView v = view(grid);
    ExView ov = v;
    ov.keys = H.old_ex->d_keys;
    ov.vals = H.old_ex->d_vals;
    ov.mask = H.old_ex->mask;
    ov.bits = H.old_ex->d_bits;
    ov.rank = H.old_ex->d_rank;
    uint32_t *d_n2o = nullptr, *d_o2n = nullptr, *d_aff = nullptr, *d_naff = nullptr;
    uint8_t* d_touched = nullptr;
    uint64_t *d_aff_ids = nullptr, *d_crow = nullptr, *d_start = nullptr;
    int32_t* d_err = nullptr;
    auto done = [&](int code) {
        for (void* q : {(void*)d_n2o, (void*)d_o2n, (void*)d_aff, (void*)d_naff, (void*)d_touched, (void*)d_aff_ids,
                        (void*)d_crow, (void*)d_start, (void*)d_err})
            ds_free(q, st);
        return code;
    };
    if (ds_malloc(&d_n2o, N * 4, st) != hipSuccess || ds_malloc(&d_o2n, oN * 4, st) != hipSuccess ||
        ds_malloc(&d_aff, std::max<uint64_t>(R, 1) * 4, st) != hipSuccess || ds_malloc(&d_naff, 16, st) != hipSuccess ||
        ds_malloc(&d_touched, std::max<uint64_t>(oR, 1), st) != hipSuccess ||
        ds_malloc(&d_aff_ids, std::max<uint64_t>(R, 1) * 8, st) != hipSuccess ||
        ds_malloc(&d_err, 16, st) != hipSuccess)
        return done(set_error(DCCRGX_ENOMEM, "incremental neighbor lists"));
    {
        const Fill z[4] = {{d_o2n, oN * 4, 0xff}, {d_naff, 16, 0}, {d_err, 16, 0}, {h.d_nof_row, 8, 0}};
        if (dx_fill_many(z, 4, st) != DCCRGX_OK) return done(DCCRGX_EHIP);
    }
    hipLaunchKernelGGL(k_inc_new2old, dim3(grid_for(N)), dim3(256), 0, st, ov, (const uint64_t*)E->d_leaves, N, d_n2o,
                       d_o2n);
    if (oR)
        hipLaunchKernelGGL(k_inc_touched, dim3(grid_for(oR)), dim3(256), 0, st, (const uint64_t*)oh.d_nof_row,
                           (const uint32_t*)oh.d_nof_g, oR, old_pos_leaf, H.old_flags, H.gone_bit, d_touched);
    if (R)
        hipLaunchKernelGGL(k_inc_count, dim3(grid_for(R)), dim3(256), 0, st, (const uint32_t*)d_n2o,
                           (const uint8_t*)d_touched, (const uint64_t*)oh.d_nof_row, (const uint64_t*)E->d_leaves, R,
                           new_pos_leaf, old_leaf_pos, oR, h.d_nof_row, d_aff, d_aff_ids, d_naff);
    if (hipGetLastError() != hipSuccess) return done(set_error(DCCRGX_EHIP, "incremental neighbor lists"));
    uint32_t naff = 0;
    int s = dx_d2h(ctx, &naff, d_naff, 4, st);
    if (s != DCCRGX_OK) return done(s);
    if (ds_malloc(&d_crow, (uint64_t)(naff + 1) * 8, st) != hipSuccess ||
        ds_malloc(&d_start, std::max<uint64_t>(naff, 1) * 8, st) != hipSuccess)
        return done(set_error(DCCRGX_ENOMEM, "incremental neighbor lists"));
    if (naff) {  // counts of the recomputed rows
        hipLaunchKernelGGL(k_ex_nof, dim3(grid_for(naff)), dim3(256), 0, st, v, h.d_of_c, h.K,
                           (const uint64_t*)d_aff_ids, (size_t)naff, d_crow, (uint64_t*)nullptr, (int32_t*)nullptr,
                           (uint32_t*)nullptr, d_err);
        hipLaunchKernelGGL(k_inc_aff_rows, dim3(grid_for(naff)), dim3(256), 0, st, (const uint32_t*)d_aff,
                           (uint64_t)naff, (const uint64_t*)d_crow, h.d_nof_row, d_start, 0);
    }
    if ((s = device_scan_rows(h.d_nof_row, R, st, nullptr)) != DCCRGX_OK) return done(s);
    uint64_t back[2] = {0, 0};  // error word, total
    {
        const D2H rb[2] = {{&back[0], d_err, 8}, {&back[1], h.d_nof_row + R, 8}};
        if ((s = dx_d2h_many(ctx, rb, 2, st)) != DCCRGX_OK) return done(s);
    }
    if ((back[0] & 0xffffffffu) & (grid->partial_leaves ? ~2u : ~0u))
        return done(set_error(back[0] & 1 ? DCCRGX_ENOTFOUND : DCCRGX_EINTERNAL,
                              back[0] & 1 ? "cell does not exist" : "neighbor more than one level apart"));
    *total = back[1];
    const uint64_t t = std::max<uint64_t>(*total, 1);
    if (ds_malloc(&h.d_nof_id, t * 8, st) != hipSuccess || ds_malloc(&h.d_nof_off, t * 12, st) != hipSuccess ||
        ds_malloc(&h.d_nof_g, t * 4, st) != hipSuccess)
        return done(set_error(DCCRGX_ENOMEM, "neighbor lists of %llu entries", (unsigned long long)*total));
    if (R)
        hipLaunchKernelGGL(k_inc_copy, dim3((unsigned)((R + 63) / 64)), dim3(64), 0, st, (const uint32_t*)d_n2o,
                       (const uint8_t*)d_touched, R, new_pos_leaf, old_leaf_pos, oR, (const uint64_t*)oh.d_nof_row,
                       (const uint64_t*)oh.d_nof_id,
                       (const int32_t*)oh.d_nof_off, (const uint32_t*)oh.d_nof_g, (const uint32_t*)d_o2n,
                       (const uint64_t*)h.d_nof_row, h.d_nof_id, h.d_nof_off, h.d_nof_g);
    if (naff) {  // the recomputed rows, each thread at its row's place
        hipLaunchKernelGGL(k_inc_aff_rows, dim3(grid_for(naff)), dim3(256), 0, st, (const uint32_t*)d_aff,
                           (uint64_t)naff, (const uint64_t*)d_crow, h.d_nof_row, d_start, 1);
        hipLaunchKernelGGL(k_ex_nof, dim3(grid_for(naff)), dim3(256), 0, st, v, h.d_of_c, h.K,
                           (const uint64_t*)d_aff_ids, (size_t)naff, d_start, h.d_nof_id, h.d_nof_off, h.d_nof_g,
                           d_err);
    }
    if (hipGetLastError() != hipSuccess) return done(set_error(DCCRGX_EHIP, "incremental neighbor lists"));
    if (keep) {
        keep->st = st;
        keep->n2o = d_n2o;
        keep->o2n = d_o2n;
        keep->touched = d_touched;
        keep->aff = d_aff;
        keep->naff = naff;
        d_n2o = d_o2n = d_aff = nullptr;
        d_touched = nullptr;
    }
    return done(DCCRGX_OK);
}

// incremental stencil rows (one rank, slot == leaf index before and after):
// the row of a leaf whose neighbors_of was copied is its old row with the
// slots remapped (the pairs sort by leaf index, which the remap keeps in
// order); the others were sorted anew into a compact CSR (arow / apairs)
__global__ void __launch_bounds__(256) k_st_inc_counts(const uint32_t* __restrict__ n2o,
                                                       const uint8_t* __restrict__ touched,
                                                       const uint64_t* __restrict__ ost_row,
                                                       const uint32_t* __restrict__ aidx,
                                                       const uint32_t* __restrict__ apc, uint64_t n,
                                                       uint32_t* __restrict__ cnt)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
        const uint32_t k = aidx[j];
        if (k != NO_SLOT) {
            cnt[j] = apc[k];
        } else {
            const uint32_t o = n2o[j];
            cnt[j] = (uint32_t)(ost_row[o + 1] - ost_row[o]);
        }
    }
}

__global__ void __launch_bounds__(256) k_st_aff_rows(const uint32_t* __restrict__ aff, uint64_t naff,
                                                     const uint64_t* __restrict__ nof_row, uint64_t* __restrict__ arow,
                                                     uint32_t* __restrict__ aidx)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < naff; k += stride) {
        const uint32_t j = aff[k];
        arow[k + 1] = nof_row[j + 1] - nof_row[j];
        aidx[j] = (uint32_t)k;
    }
}

// one wave per 64 rows, consecutive lanes on consecutive entries (k_inc_copy)
__global__ void __launch_bounds__(64) k_st_inc_fill(const uint32_t* __restrict__ n2o, const uint32_t* __restrict__ o2n,
                                                    const uint32_t* __restrict__ aidx, uint64_t n,
                                                    const uint64_t* __restrict__ ost_row,
                                                    const uint32_t* __restrict__ ost_slot,
                                                    const int32_t* __restrict__ ost_off,
                                                    const uint64_t* __restrict__ arow, const Pair* __restrict__ apairs,
                                                    const uint64_t* __restrict__ st_row, uint32_t* __restrict__ st_slot,
                                                    int32_t* __restrict__ st_off)
{
    __shared__ uint64_t s_dst[65], s_src[64];
    __shared__ uint32_t s_aff[64];
    const int lane = threadIdx.x;
    const uint64_t r0 = (uint64_t)blockIdx.x * 64;
    const uint64_t last = r0 + 64 < n ? r0 + 64 : n;
    s_dst[lane] = st_row[r0 + lane < last ? r0 + lane : last];
    if (lane == 0) s_dst[64] = st_row[last];
    uint32_t k = NO_SLOT;
    uint64_t src = 0;
    if (r0 + lane < n) {
        k = aidx[r0 + lane];
        src = k != NO_SLOT ? arow[k] : ost_row[n2o[r0 + lane]];
    }
    s_aff[lane] = k;
    s_src[lane] = src;
    __syncthreads();
    const uint64_t end = s_dst[64];
    for (uint64_t o = s_dst[0] + lane; o < end; o += 64) {
        const int j = wave_row_of(s_dst, o);
        const uint64_t e = s_src[j] + (o - s_dst[j]);
        if (s_aff[j] != NO_SLOT) {
            const Pair p = apairs[e];
            st_slot[o] = p.g;  // slot == leaf index
            st_off[3 * o + 0] = p.x;
            st_off[3 * o + 1] = p.y;
            st_off[3 * o + 2] = p.z;
        } else {
            st_slot[o] = o2n[ost_slot[e]];
            st_off[3 * o + 0] = ost_off[3 * e + 0];
            st_off[3 * o + 1] = ost_off[3 * e + 1];
            st_off[3 * o + 2] = ost_off[3 * e + 2];
        }
    }
}

// Incremental neighbors_to (one rank, after nof_incremental).  A kept leaf's
// row -- the leaves whose neighbors_of holds it -- can change only through a
// row that changed: it is marked if it appears in the new row of a recomputed
// neighbors_of row or in the old row of a recomputed or removed leaf (new
// leaves are recomputed rows themselves).  Every unmarked row is its old row
// with the indices remapped (each leaf in it is kept with a copied row, so it
// still holds the leaf; the remap keeps the order).  Marked rows are searched
// anew by the reference's three-level search (nto_direct).  No symmetry of
// the neighborhood is assumed.
__global__ void __launch_bounds__(256) k_nto_mark_new(const uint32_t* __restrict__ aff, uint64_t naff,
                                                      const uint64_t* __restrict__ row, const uint32_t* __restrict__ g,
                                                      uint32_t* __restrict__ mark)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < naff; k += stride) {
        const uint32_t j = aff[k];
        mark[j] = 1;
        for (uint64_t e = row[j]; e < row[j + 1]; e++) mark[g[e]] = 1;
    }
}

__global__ void __launch_bounds__(256) k_nto_mark_old(const uint8_t* __restrict__ touched, uint64_t on,
                                                      const uint64_t* __restrict__ orow, const uint32_t* __restrict__ og,
                                                      const uint32_t* __restrict__ o2n, uint32_t* __restrict__ mark)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x; o < on; o += stride) {
        if (!touched[o]) continue;
        for (uint64_t e = orow[o]; e < orow[o + 1]; e++) {
            const uint32_t t = o2n[og[e]];
            if (t != NO_SLOT) mark[t] = 1;
        }
    }
}

// ids of the marked rows, in order (pos: exclusive scan of the marks)
__global__ void __launch_bounds__(256) k_nto_marked_ids(const uint32_t* __restrict__ mark, const uint64_t* __restrict__ pos,
                                                        uint64_t n, const uint64_t* __restrict__ leaves,
                                                        uint64_t* __restrict__ ids)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride)
        if (mark[j]) ids[pos[j]] = leaves[j];
}

// (rows: local positions; new_pos_leaf / old_leaf_pos: the position maps of
// several processes, null with one -- see k_inc_touched)
__global__ void __launch_bounds__(256) k_nto_inc_counts(const uint32_t* __restrict__ mark,
                                                        const uint64_t* __restrict__ pos,
                                                        const uint64_t* __restrict__ mrow,
                                                        const uint32_t* __restrict__ n2o,
                                                        const uint64_t* __restrict__ orow, uint64_t n,
                                                        const uint32_t* __restrict__ new_pos_leaf,
                                                        const uint32_t* __restrict__ old_leaf_pos,
                                                        uint32_t* __restrict__ cnt)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
        if (mark[j]) {
            const uint64_t k = pos[j];
            cnt[j] = (uint32_t)(mrow[k + 1] - mrow[k]);
        } else {
            const uint32_t o = pos_map(old_leaf_pos, n2o[pos_map(new_pos_leaf, j)]);
            cnt[j] = (uint32_t)(orow[o + 1] - orow[o]);
        }
    }
}

// one wave per 64 rows, consecutive lanes on consecutive entries (k_st_inc_fill)
__global__ void __launch_bounds__(64) k_nto_inc_fill(const uint32_t* __restrict__ mark, const uint64_t* __restrict__ pos,
                                                     const uint64_t* __restrict__ mrow, const uint32_t* __restrict__ mval,
                                                     const uint32_t* __restrict__ n2o, const uint32_t* __restrict__ o2n,
                                                     const uint64_t* __restrict__ orow, const uint32_t* __restrict__ og,
                                                     uint64_t n, const uint32_t* __restrict__ new_pos_leaf,
                                                     const uint32_t* __restrict__ old_leaf_pos,
                                                     const uint64_t* __restrict__ row, uint32_t* __restrict__ out)
{
    __shared__ uint64_t s_dst[65], s_src[64];
    __shared__ uint32_t s_new[64];
    const int lane = threadIdx.x;
    const uint64_t r0 = (uint64_t)blockIdx.x * 64;
    const uint64_t last = r0 + 64 < n ? r0 + 64 : n;
    s_dst[lane] = row[r0 + lane < last ? r0 + lane : last];
    if (lane == 0) s_dst[64] = row[last];
    uint32_t fresh = 0;
    uint64_t src = 0;
    if (r0 + lane < n) {
        const uint64_t j = r0 + lane;
        fresh = mark[j];
        src = fresh ? mrow[pos[j]] : orow[pos_map(old_leaf_pos, n2o[pos_map(new_pos_leaf, j)])];
    }
    s_new[lane] = fresh;
    s_src[lane] = src;
    __syncthreads();
    const uint64_t end = s_dst[64];
    for (uint64_t o = s_dst[0] + lane; o < end; o += 64) {
        const int j = wave_row_of(s_dst, o);
        const uint64_t e = s_src[j] + (o - s_dst[j]);
        out[o] = s_new[j] ? mval[e] : o2n[og[e]];
    }
}

static int nto_direct(const dccrgx_grid* grid, const Hood& h, const uint64_t* cells, uint64_t n, uint64_t** out_row,
                      uint32_t** out_g, hipStream_t st);

// the new neighbors_to CSR of every leaf (rows: leaves) from the old one; tot:
// the new neighbors_of's entries (a bound on the transpose's)
static int nto_incremental(dccrgx_grid* grid, Hood& h, const Hood& oh, const IncMaps& inc, uint64_t old_n,
                           uint64_t tot, hipStream_t st)
{
    Explicit* E = grid->ex;
    const uint64_t N = E->n;
    uint32_t *d_mark = nullptr, *d_mval = nullptr, *d_cnt = nullptr;
    uint64_t *d_pos = nullptr, *d_ids = nullptr, *d_mrow = nullptr;
    auto done = [&](int code) {
        for (void* q : {(void*)d_mark, (void*)d_mval, (void*)d_cnt, (void*)d_pos, (void*)d_ids, (void*)d_mrow})
            ds_free(q, st);
        return code;
    };
    if (ds_malloc(&d_mark, std::max<uint64_t>(N, 1) * 4, st) != hipSuccess ||
        ds_malloc(&d_cnt, std::max<uint64_t>(N, 1) * 4, st) != hipSuccess)
        return done(set_error(DCCRGX_ENOMEM, "incremental neighbors_to"));
    {
        const Fill z[1] = {{d_mark, N * 4, 0}};
        if (dx_fill_many(z, 1, st) != DCCRGX_OK) return done(DCCRGX_EHIP);
    }
    if (inc.naff)
        hipLaunchKernelGGL(k_nto_mark_new, dim3(grid_for(inc.naff)), dim3(256), 0, st, (const uint32_t*)inc.aff,
                           inc.naff, (const uint64_t*)h.d_nof_row, (const uint32_t*)h.d_nof_g, d_mark);
    hipLaunchKernelGGL(k_nto_mark_old, dim3(grid_for(old_n)), dim3(256), 0, st, (const uint8_t*)inc.touched, old_n,
                       (const uint64_t*)oh.d_nof_row, (const uint32_t*)oh.d_nof_g, (const uint32_t*)inc.o2n, d_mark);
    uint64_t nm = 0;
    int e = scan_counts_device(d_mark, N, &d_pos, &nm, st);  // the marked rows' places (one read-back)
    if (e != DCCRGX_OK) return done(e);
    if (ds_malloc(&d_ids, std::max<uint64_t>(nm, 1) * 8, st) != hipSuccess)
        return done(set_error(DCCRGX_ENOMEM, "incremental neighbors_to"));
    hipLaunchKernelGGL(k_nto_marked_ids, dim3(grid_for(N)), dim3(256), 0, st, (const uint32_t*)d_mark,
                       (const uint64_t*)d_pos, N, (const uint64_t*)E->d_leaves, d_ids);
    if (hipGetLastError() != hipSuccess) return done(set_error(DCCRGX_EHIP, "incremental neighbors_to"));
    if ((e = nto_direct(grid, h, d_ids, nm, &d_mrow, &d_mval, st)) != DCCRGX_OK) return done(e);
    hipLaunchKernelGGL(k_nto_inc_counts, dim3(grid_for(N)), dim3(256), 0, st, (const uint32_t*)d_mark,
                       (const uint64_t*)d_pos, (const uint64_t*)d_mrow, (const uint32_t*)inc.n2o,
                       (const uint64_t*)oh.d_nto_row, N, (const uint32_t*)nullptr, (const uint32_t*)nullptr, d_cnt);
    if ((e = scan_counts_device(d_cnt, N, &h.d_nto_row, nullptr, st)) != DCCRGX_OK) return done(e);
    if (ds_malloc(&h.d_nto_g, std::max<uint64_t>(tot, 1) * 4, st) != hipSuccess)
        return done(set_error(DCCRGX_ENOMEM, "neighbors_to lists"));
    if (N)
        hipLaunchKernelGGL(k_nto_inc_fill, dim3((unsigned)((N + 63) / 64)), dim3(64), 0, st, (const uint32_t*)d_mark,
                           (const uint64_t*)d_pos, (const uint64_t*)d_mrow, (const uint32_t*)d_mval,
                           (const uint32_t*)inc.n2o, (const uint32_t*)inc.o2n, (const uint64_t*)oh.d_nto_row,
                           (const uint32_t*)oh.d_nto_g, N, (const uint32_t*)nullptr, (const uint32_t*)nullptr,
                           (const uint64_t*)h.d_nto_row, h.d_nto_g);
    if (hipGetLastError() != hipSuccess) return done(set_error(DCCRGX_EHIP, "incremental neighbors_to"));
    return done(DCCRGX_OK);
}

// Several processes: a local cell's neighbors_to row holds cells of any
// process, whose neighbors_of rows this rank does not keep, so the marks
// come from the leaves instead.  Whether a kept leaf c is in the neighbors_of
// of a kept leaf d depends on those two cells alone (d's windows and c's
// extent), so a kept cell's row changes only by leaves that are gone (they
// drop out of it) or new (they may name it).  Marked: new cells, kept cells
// whose old row holds a gone leaf, and cells some new leaf (of any process:
// the leaf set is replicated) names in its neighbors_of; they are searched
// anew (nto_direct), every other row is its old row remapped.
__global__ void __launch_bounds__(256) k_nto_is_new(const uint32_t* __restrict__ n2o, uint64_t n,
                                                    uint32_t* __restrict__ flag)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) flag[j] = n2o[j] == NO_SLOT;
}

__global__ void __launch_bounds__(256) k_nto_mark_ranks(const uint32_t* __restrict__ local_g, uint64_t nl,
                                                        const uint32_t* __restrict__ n2o,
                                                        const uint32_t* __restrict__ slot_of_g,
                                                        const uint32_t* __restrict__ tgt, uint64_t nt,
                                                        const uint64_t* __restrict__ orow,
                                                        const uint32_t* __restrict__ og,
                                                        const uint32_t* __restrict__ old_local_g, uint64_t onl,
                                                        const uint32_t* __restrict__ flags, uint32_t gone,
                                                        const uint32_t* __restrict__ o2n, uint32_t* __restrict__ mark)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (size_t q = t0; q < nl; q += stride)  // new cells
        if (n2o[local_g[q]] == NO_SLOT) mark[q] = 1;
    for (size_t e = t0; e < nt; e += stride) {  // named by a new leaf
        const uint32_t sl = slot_of_g[tgt[e]];
        if (sl < nl) mark[sl] = 1;
    }
    for (size_t p = t0; p < onl; p += stride) {  // old rows holding a gone leaf
        bool g = false;
        for (uint64_t e = orow[p]; e < orow[p + 1] && !g; e++) g = (flags[og[e]] & gone) != 0;
        if (!g) continue;
        const uint32_t j = o2n[old_local_g[p]];
        const uint32_t sl = j == NO_SLOT ? NO_SLOT : slot_of_g[j];
        if (sl < nl) mark[sl] = 1;
    }
}

// marked positions' ids, in order (pos: exclusive scan of the marks)
__global__ void __launch_bounds__(256) k_nto_marked_pos_ids(const uint32_t* __restrict__ mark,
                                                            const uint64_t* __restrict__ pos, uint64_t n,
                                                            const uint32_t* __restrict__ local_g,
                                                            const uint64_t* __restrict__ leaves,
                                                            uint64_t* __restrict__ ids)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += stride)
        if (mark[q]) ids[pos[q]] = leaves[local_g[q]];
}

static int nto_incremental_ranks(dccrgx_grid* grid, Hood& h, const NofHint& H, const IncMaps& inc, hipStream_t st)
{
    Explicit* E = grid->ex;
    const Explicit* O = H.old_ex;
    const Hood& oh = *H.old_h;
    const uint64_t N = E->n, nl = E->n_local(), onl = oh.n_rows;
    uint32_t *d_isnew = nullptr, *d_mark = nullptr, *d_cnt = nullptr, *d_mval = nullptr, *d_ng = nullptr;
    uint64_t *d_npos = nullptr, *d_nids = nullptr, *d_nrow = nullptr, *d_nid = nullptr, *d_mpos = nullptr,
             *d_mids = nullptr, *d_mrow = nullptr;
    int32_t* d_noff = nullptr;
    auto done = [&](int code) {
        for (void* q : {(void*)d_isnew, (void*)d_mark, (void*)d_cnt, (void*)d_mval, (void*)d_ng, (void*)d_npos,
                        (void*)d_nids, (void*)d_nrow, (void*)d_nid, (void*)d_mpos, (void*)d_mids, (void*)d_mrow,
                        (void*)d_noff})
            ds_free(q, st);
        return code;
    };
    // the new leaves of every process and their neighbors_of
    if (ds_malloc(&d_isnew, std::max<uint64_t>(N, 1) * 4, st) != hipSuccess ||
        ds_malloc(&d_mark, std::max<uint64_t>(nl, 1) * 4, st) != hipSuccess ||
        ds_malloc(&d_cnt, std::max<uint64_t>(nl, 1) * 4, st) != hipSuccess)
        return done(set_error(DCCRGX_ENOMEM, "incremental neighbors_to"));
    hipLaunchKernelGGL(k_nto_is_new, dim3(grid_for(N)), dim3(256), 0, st, (const uint32_t*)inc.n2o, N, d_isnew);
    uint64_t n_new = 0;
    int e = scan_counts_device(d_isnew, N, &d_npos, &n_new, st);
    if (e != DCCRGX_OK) return done(e);
    if (ds_malloc(&d_nids, std::max<uint64_t>(n_new, 1) * 8, st) != hipSuccess ||
        ds_malloc(&d_nrow, (n_new + 1) * 8, st) != hipSuccess)
        return done(set_error(DCCRGX_ENOMEM, "incremental neighbors_to"));
    hipLaunchKernelGGL(k_nto_marked_ids, dim3(grid_for(N)), dim3(256), 0, st, (const uint32_t*)d_isnew,
                       (const uint64_t*)d_npos, N, (const uint64_t*)E->d_leaves, d_nids);
    uint64_t nt = 0;
    if ((e = nof_device(grid, h, d_nids, n_new, d_nrow, &d_nid, &d_noff, &d_ng, &nt, st)) != DCCRGX_OK)
        return done(e);
    {
        const Fill z[1] = {{d_mark, nl * 4, 0}};
        if (nl && dx_fill_many(z, 1, st) != DCCRGX_OK) return done(DCCRGX_EHIP);
    }
    const uint64_t most = std::max<uint64_t>({nl, nt, onl, 1});
    hipLaunchKernelGGL(k_nto_mark_ranks, dim3(grid_for(most)), dim3(256), 0, st, (const uint32_t*)E->d_local_g, nl,
                       (const uint32_t*)inc.n2o, (const uint32_t*)E->d_slot_of_g, (const uint32_t*)d_ng, nt,
                       (const uint64_t*)oh.d_nto_row, (const uint32_t*)oh.d_nto_g, (const uint32_t*)O->d_local_g, onl,
                       H.old_flags, H.gone_bit, (const uint32_t*)inc.o2n, d_mark);
    // the marked cells searched anew
    uint64_t nm = 0;
    if ((e = scan_counts_device(d_mark, nl, &d_mpos, &nm, st)) != DCCRGX_OK) return done(e);
    if (ds_malloc(&d_mids, std::max<uint64_t>(nm, 1) * 8, st) != hipSuccess)
        return done(set_error(DCCRGX_ENOMEM, "incremental neighbors_to"));
    if (nl)
        hipLaunchKernelGGL(k_nto_marked_pos_ids, dim3(grid_for(nl)), dim3(256), 0, st, (const uint32_t*)d_mark,
                           (const uint64_t*)d_mpos, nl, (const uint32_t*)E->d_local_g, (const uint64_t*)E->d_leaves,
                           d_mids);
    if ((e = nto_direct(grid, h, d_mids, nm, &d_mrow, &d_mval, st)) != DCCRGX_OK) return done(e);
    // every row: marked ones from the search, the others from the old rows
    if (nl)
        hipLaunchKernelGGL(k_nto_inc_counts, dim3(grid_for(nl)), dim3(256), 0, st, (const uint32_t*)d_mark,
                           (const uint64_t*)d_mpos, (const uint64_t*)d_mrow, (const uint32_t*)inc.n2o,
                           (const uint64_t*)oh.d_nto_row, nl, (const uint32_t*)E->d_local_g,
                           (const uint32_t*)O->d_slot_of_g, d_cnt);
    uint64_t total = 0;
    if ((e = scan_counts_device(d_cnt, nl, &h.d_nto_row, &total, st)) != DCCRGX_OK) return done(e);
    if (ds_malloc(&h.d_nto_g, std::max<uint64_t>(total, 1) * 4, st) != hipSuccess)
        return done(set_error(DCCRGX_ENOMEM, "neighbors_to lists"));
    if (nl)
        hipLaunchKernelGGL(k_nto_inc_fill, dim3((unsigned)((nl + 63) / 64)), dim3(64), 0, st, (const uint32_t*)d_mark,
                           (const uint64_t*)d_mpos, (const uint64_t*)d_mrow, (const uint32_t*)d_mval,
                           (const uint32_t*)inc.n2o, (const uint32_t*)inc.o2n, (const uint64_t*)oh.d_nto_row,
                           (const uint32_t*)oh.d_nto_g, nl, (const uint32_t*)E->d_local_g,
                           (const uint32_t*)O->d_slot_of_g, (const uint64_t*)h.d_nto_row, h.d_nto_g);
    if (hipGetLastError() != hipSuccess) return done(set_error(DCCRGX_EHIP, "incremental neighbors_to"));
    return done(DCCRGX_OK);
}

int explicit_build_hood_async(dccrgx_grid* grid, Hood& h, const NofHint* hint)
{
    Explicit* E = grid->ex;
    Ctx* ctx = grid->ctx;
    hipStream_t st = ctx->compute;
    free_hood(h);
    PhaseTimer T("build_hood");
    h.K = (int32_t)(h.items.size() / 3);
    h.of_c = h.items;  // explicit grids use the original axes
    h.to_c.resize(h.items.size());
    for (size_t i = 0; i < h.items.size(); i++) h.to_c[i] = -h.items[i];
    DX_TRY(upload(grid->ctx, h.of_c, &h.d_of_c, st));
    DX_TRY(upload(grid->ctx, h.to_c, &h.d_to_c, st));
    h.outer.clear();
    h.remote.clear();
    const uint64_t N = E->n;
    const uint64_t nl = E->n_local();
    // The CSRs hold the rows of this rank's local cells, indexed by local
    // position (= storage slot).  One process: every leaf, in leaf order.
    // Several: only the local cells' rows -- the reference builds lists for
    // every cell (dccrg.hpp:8371-8397); here a rank's list memory scales with
    // its own cells, and rows of other cells are searched on demand from the
    // replicated leaf lookup (queries, the refinement decisions).
    const bool per_rank = ctx->comm_size > 1;
    h.n_rows = nl;
    DX_HIP(ds_malloc(&h.d_nof_row, (nl + 1) * 8, st));
    uint64_t tot = 0;
    IncMaps inc;
    const bool inc_nof = hint && hint->old_h && hint->old_h->d_nof_row && hint->old_h->items == h.items &&
                         hint->old_ex && incremental_rebuild(hint->old_ex->n);
    // the stencil rows follow incrementally where slots are leaf indices before and after
    const bool inc_st = inc_nof && E->slot_identity && hint->old_ex->slot_identity && hint->old_h->d_st_row &&
                        hint->old_ex->n_local() == hint->old_ex->n;
    uint64_t* d_local_ids = nullptr;  // several processes: the local cells' ids
    if (per_rank) {
        DX_HIP(ds_malloc(&d_local_ids, std::max<uint64_t>(nl, 1) * 8, st));
        DX_TRY(explicit_local_ids(grid, d_local_ids, st));
    }
    struct FreeIds {
        uint64_t*& p;
        hipStream_t st;
        ~FreeIds() { ds_free(p, st); }
    } free_ids{d_local_ids, st};
    if (inc_nof)
        DX_TRY(nof_incremental(grid, h, *hint, &tot, st, &inc));
    else
        DX_TRY(nof_device(grid, h, per_rank ? d_local_ids : E->d_leaves, per_rank ? nl : N, h.d_nof_row, &h.d_nof_id,
                          &h.d_nof_off, &h.d_nof_g, &tot, st));
    T.lap("neighbors_of");
    if (per_rank && inc.n2o && hint->old_h->d_nto_row && hint->old_h->d_nto_g && !test_opt(OPT_FULL_NTO, 0)) {
        // several processes after an incremental neighbors_of: the old rows around the changes
        DX_TRY(nto_incremental_ranks(grid, h, *hint, inc, st));
    } else if (per_rank) {  // neighbors_to of the local cells by the reference's search
        DX_TRY(nto_direct(grid, h, d_local_ids, nl, &h.d_nto_row, &h.d_nto_g, st));
    } else if (inc.n2o && hint->old_h->d_nto_row && hint->old_h->d_nto_g && !test_opt(OPT_FULL_NTO, 0)) {
        // one process after an incremental neighbors_of: the old transpose, remapped, around the changes
        DX_TRY(nto_incremental(grid, h, *hint->old_h, inc, hint->old_ex->n, tot, st));
    } else {  // one process: the transpose of every leaf's neighbors_of (rows: leaves)
        uint32_t *d_cnt = nullptr, *d_cur = nullptr, *d_tmp = nullptr;
        DX_HIP(ds_malloc(&d_cnt, N * 4, st));
        DX_HIP(ds_malloc(&d_cur, N * 4, st));
        {
            const Fill z[2] = {{d_cnt, N * 4, 0}, {d_cur, N * 4, 0}};
            DX_TRY(dx_fill_many(z, 2, st));
        }
        hipLaunchKernelGGL(k_tr_count, dim3(grid_for(N)), dim3(256), 0, st, h.d_nof_row, h.d_nof_g, N, d_cnt);
        uint64_t* d_trow = nullptr;
        const uint64_t ttot = tot;  // the transpose has as many entries as neighbors_of: no read-back
        DX_TRY(scan_counts_device(d_cnt, N, &d_trow, nullptr, st));
        DX_HIP(ds_malloc(&d_tmp, std::max<uint64_t>(ttot, 1) * 4, st));
        hipLaunchKernelGGL(k_tr_scatter, dim3(grid_for(N)), dim3(256), 0, st, h.d_nof_row, h.d_nof_g, N, d_trow,
                           d_cur, d_tmp);
        DX_HIP(hipGetLastError());
        const int e = sort_unique_compact(d_trow, d_tmp, N, ttot, &h.d_nto_row, &h.d_nto_g, st);
        ds_free(d_cnt, st);
        ds_free(d_cur, st);
        ds_free(d_tmp, st);
        ds_free(d_trow, st);
        DX_TRY(e);
    }

    T.lap("neighbors_to");
    // per-rank bookkeeping from the device lists (dccrg.hpp:9131-9234, 8729-8891)
    Explicit::HoodLists& L = E->hl[h.id];
    for (uint32_t* p : {L.d_inner_pos, L.d_outer_pos, L.d_all_pos})
        if (!ctx_is_identity(ctx, p)) dx_free(p);
    L = Explicit::HoodLists{};
    // host copies of the lists only where host code reads them: the
    // classification of several ranks here; refinement requests and
    // neighbors_to queries fetch them on first use (explicit_host_lists)
    if (ctx->comm_size > 1) {
        DX_TRY(explicit_host_lists(grid, h));
        T.lap("lists to host");
    }
    const std::vector<uint64_t>& nof_row = L.h_nof_row;
    const std::vector<uint64_t>& nto_row = L.h_nto_row;
    const std::vector<int32_t>& owner = E->owner;
    const int me = ctx->rank;
    std::set<uint64_t> remote;
    std::map<int, std::set<uint64_t>> send, recv;
    L.inner_all = ctx->comm_size == 1;  // one process: every cell is inner, nothing remote
    for (uint64_t i = 0; ctx->comm_size > 1 && i < nl; i++) {
        const uint64_t r = i;  // rows by local position
        bool outer = false;
        for (uint64_t e = nof_row[r]; e < nof_row[r + 1]; e++) {
            const uint32_t t = L.h_nof_g[e];
            if (owner[t] != me) {
                outer = true;
                remote.insert(E->leaves_[t]);
                recv[owner[t]].insert(E->leaves_[t]);
            }
        }
        for (uint64_t e = nto_row[r]; e < nto_row[r + 1]; e++) {
            const uint32_t t = L.h_nto_g[e];
            if (owner[t] != me) {
                outer = true;
                remote.insert(E->leaves_[t]);
                send[owner[t]].insert(E->local_[i]);
            }
        }
        (outer ? L.outer_pos : L.inner_pos).push_back((uint32_t)i);
        if (outer) h.outer.push_back(E->local_[i]);
    }
    h.remote.assign(remote.begin(), remote.end());
    T.lap("classification");
    // ghost slots for this neighborhood's remote neighbors
    DX_TRY(explicit_add_slots(grid, h.remote));
    T.lap("ghost slots");

    // stencil rows of local cells (iteration-cache neighbors_of: unique pairs)
    if (inc_st && inc.n2o) {  // one rank after an incremental neighbors_of: old rows remapped, the rest sorted
        const Hood& oh = *hint->old_h;
        const uint64_t na = inc.naff;
        uint64_t* d_arow = nullptr;
        uint32_t *d_aidx = nullptr, *d_apc = nullptr, *d_cnt2 = nullptr;
        Pair* d_apairs = nullptr;
        auto st_done = [&](int code) {
            for (void* q : {(void*)d_arow, (void*)d_aidx, (void*)d_apc, (void*)d_cnt2, (void*)d_apairs}) ds_free(q, st);
            return code;
        };
        if (ds_malloc(&d_arow, (na + 1) * 8, st) != hipSuccess || ds_malloc(&d_aidx, N * 4, st) != hipSuccess ||
            ds_malloc(&d_apc, std::max<uint64_t>(na, 1) * 4, st) != hipSuccess ||
            ds_malloc(&d_cnt2, std::max<uint64_t>(N, 1) * 4, st) != hipSuccess)
            return st_done(set_error(DCCRGX_ENOMEM, "incremental stencil rows"));
        {
            const Fill z[2] = {{d_aidx, N * 4, 0xff}, {d_arow, 8, 0}};
            if (dx_fill_many(z, 2, st) != DCCRGX_OK) return st_done(DCCRGX_EHIP);
        }
        if (na)
            hipLaunchKernelGGL(k_st_aff_rows, dim3(grid_for(na)), dim3(256), 0, st, (const uint32_t*)inc.aff, na,
                               (const uint64_t*)h.d_nof_row, d_arow, d_aidx);
        uint64_t atot = 0;
        int e = device_scan_rows(d_arow, na, st, &atot);
        if (e != DCCRGX_OK) return st_done(e);
        if (ds_malloc(&d_apairs, std::max<uint64_t>(atot, 1) * sizeof(Pair), st) != hipSuccess)
            return st_done(set_error(DCCRGX_ENOMEM, "incremental stencil rows"));
        RowListBufs RL;
        if (na && (e = RL.make(na, st)) != DCCRGX_OK) return st_done(e);
        if (na) {
            hipLaunchKernelGGL((k_stencil_rows_seg<16, false>), dim3((unsigned)std::min<uint64_t>((na + 15) / 16, 16384)),
                               dim3(256), 0, st, h.d_nof_row, h.d_nof_g, h.d_nof_off, (const uint32_t*)inc.aff, na,
                               (const uint64_t*)d_arow, d_apairs, d_apc, RL.L);
            hipLaunchKernelGGL((k_stencil_rows_seg<64, true>), dim3((unsigned)std::min<uint64_t>((na + 3) / 4, 4096)),
                               dim3(256), 0, st, h.d_nof_row, h.d_nof_g, h.d_nof_off, (const uint32_t*)inc.aff, na,
                               (const uint64_t*)d_arow, d_apairs, d_apc, RL.L);
            hipLaunchKernelGGL(k_stencil_rows_wave, dim3((unsigned)std::min<uint64_t>(na, 4096)), dim3(64), 0, st,
                               h.d_nof_row, h.d_nof_g, h.d_nof_off, (const uint32_t*)inc.aff, na,
                               (const uint64_t*)d_arow, d_apairs, d_apc, RL.L);
            hipLaunchKernelGGL(k_stencil_rows, dim3(grid_for(na)), dim3(256), 0, st, h.d_nof_row, h.d_nof_g,
                               h.d_nof_off, (const uint32_t*)inc.aff, na, (const uint64_t*)d_arow, d_apairs, d_apc);
        }
        hipLaunchKernelGGL(k_st_inc_counts, dim3(grid_for(N)), dim3(256), 0, st, (const uint32_t*)inc.n2o,
                           (const uint8_t*)inc.touched, (const uint64_t*)oh.d_st_row, (const uint32_t*)d_aidx,
                           (const uint32_t*)d_apc, N, d_cnt2);
        if ((e = scan_counts_device(d_cnt2, N, &h.d_st_row, nullptr, st)) != DCCRGX_OK) return st_done(e);
        const uint64_t stot = tot;  // unique pairs: at most the rows' entries
        h.st_cap = std::max<uint64_t>(stot, 1);
        if (ds_malloc(&h.d_st_slot, std::max<uint64_t>(stot, 1) * 4, st) != hipSuccess ||
            ds_malloc(&h.d_st_off, std::max<uint64_t>(stot, 1) * 12, st) != hipSuccess)
            return st_done(set_error(DCCRGX_ENOMEM, "stencil rows"));
        if (N)
            hipLaunchKernelGGL(k_st_inc_fill, dim3((unsigned)((N + 63) / 64)), dim3(64), 0, st,
                               (const uint32_t*)inc.n2o, (const uint32_t*)inc.o2n, (const uint32_t*)d_aidx, N,
                               (const uint64_t*)oh.d_st_row, (const uint32_t*)oh.d_st_slot, (const int32_t*)oh.d_st_off,
                               (const uint64_t*)d_arow, (const Pair*)d_apairs, (const uint64_t*)h.d_st_row, h.d_st_slot,
                               h.d_st_off);
        if (hipGetLastError() != hipSuccess) return st_done(set_error(DCCRGX_EHIP, "incremental stencil rows"));
        st_done(DCCRGX_OK);
    } else {
        uint64_t* d_tmp_row = nullptr;
        Pair* d_pairs = nullptr;
        uint32_t* d_pc = nullptr;
        uint64_t tmp_tot = 0;
        // the rows are the local cells' neighbors_of rows, in local order
        DX_HIP(ds_malloc(&d_tmp_row, (nl + 1) * 8, st));
        DX_HIP(hipMemcpyAsync(d_tmp_row, h.d_nof_row, (nl + 1) * 8, hipMemcpyDeviceToDevice, st));
        tmp_tot = tot;
        if (!L.d_all_pos) DX_TRY(ctx_identity(ctx, nl, &L.d_all_pos, st));  // row of local position i: i
        DX_HIP(ds_malloc(&d_pairs, std::max<uint64_t>(tmp_tot, 1) * sizeof(Pair), st));
        DX_HIP(ds_malloc(&d_pc, std::max<uint64_t>(nl, 1) * 4, st));
        RowListBufs RL;
        if (nl) DX_TRY(RL.make(nl, st));
        if (nl) {
            hipLaunchKernelGGL((k_stencil_rows_seg<16, false>), dim3((unsigned)std::min<uint64_t>((nl + 15) / 16, 16384)),
                               dim3(256), 0, st, h.d_nof_row, h.d_nof_g, h.d_nof_off, L.d_all_pos, nl, d_tmp_row, d_pairs,
                               d_pc, RL.L);
            hipLaunchKernelGGL((k_stencil_rows_seg<64, true>), dim3((unsigned)std::min<uint64_t>((nl + 3) / 4, 4096)),
                               dim3(256), 0, st, h.d_nof_row, h.d_nof_g, h.d_nof_off, L.d_all_pos, nl, d_tmp_row, d_pairs,
                               d_pc, RL.L);
            hipLaunchKernelGGL(k_stencil_rows_wave, dim3((unsigned)std::min<uint64_t>(nl, 4096)), dim3(64), 0, st,
                               h.d_nof_row, h.d_nof_g, h.d_nof_off, L.d_all_pos, nl, d_tmp_row, d_pairs, d_pc, RL.L);
            hipLaunchKernelGGL(k_stencil_rows, dim3(grid_for(nl)), dim3(256), 0, st, h.d_nof_row, h.d_nof_g,
                               h.d_nof_off, L.d_all_pos, nl, d_tmp_row, d_pairs, d_pc);
        }
        const uint64_t stot = tmp_tot;  // unique pairs: at most the rows' entries (no read-back)
        DX_TRY(scan_counts_device(d_pc, nl, &h.d_st_row, nullptr, st));
        h.st_cap = std::max<uint64_t>(stot, 1);
        DX_HIP(ds_malloc(&h.d_st_slot, std::max<uint64_t>(stot, 1) * 4, st));
        DX_HIP(ds_malloc(&h.d_st_off, std::max<uint64_t>(stot, 1) * 12, st));
        if (nl)
            hipLaunchKernelGGL(k_stencil_slots_wave, dim3((unsigned)((nl + 63) / 64)), dim3(64), 0, st, d_tmp_row,
                               d_pairs, h.d_st_row, nl, E->d_slot_of_g, h.d_st_slot, h.d_st_off);
        DX_HIP(hipGetLastError());
        ds_free(d_tmp_row, st);
        ds_free(d_pairs, st);
        ds_free(d_pc, st);
    }

    T.lap("stencil rows");
    struct Lap {
        PhaseTimer& t;
        ~Lap() { t.lap("peer plans"); }
    } lap_end{T};
    // per-peer plans: send from local slots, receive into ghost slots
    std::set<int> peers;
    for (auto& kv : send) peers.insert(kv.first);
    for (auto& kv : recv) peers.insert(kv.first);
    auto local_pos = [&](uint64_t id) {
        const std::vector<uint64_t>& loc = E->local();
        return (uint64_t)(std::lower_bound(loc.begin(), loc.end(), id) - loc.begin());
    };
    for (int p : peers) {
        PeerPlan pp;
        pp.peer = p;
        pp.send_ids.assign(send[p].begin(), send[p].end());
        pp.recv_ids.assign(recv[p].begin(), recv[p].end());
        std::vector<uint64_t> ss, rd;
        for (uint64_t c : pp.send_ids) ss.push_back(local_pos(c));
        for (uint64_t c : pp.recv_ids) {
            const uint32_t* x = E->extra.find(c);
            DX_CHECK(x, DCCRGX_EINTERNAL, "remote cell %llu has no ghost slot", (unsigned long long)c);
            rd.push_back(*x);
        }
        if (!ss.empty()) DX_TRY(upload(grid->ctx, ss, &pp.d_send_slots, st));
        if (!rd.empty()) DX_TRY(upload(grid->ctx, rd, &pp.d_unpack_dst, st));
        pp.n_unpack = rd.size();
        pp.h_send_slots = ss;
        pp.h_unpack_dst = rd;
        pp.h_unpack_src.resize(rd.size());
        for (size_t i = 0; i < rd.size(); i++) pp.h_unpack_src[i] = i;
        h.peers.push_back(std::move(pp));
    }

    if (ctx->comm_size == 1) DX_TRY(ctx_identity(ctx, nl, &L.d_inner_pos, st));  // every cell inner
    else DX_TRY(upload(grid->ctx, L.inner_pos, &L.d_inner_pos, st));
    DX_TRY(upload(grid->ctx, L.outer_pos, &L.d_outer_pos, st));
    if (!L.d_all_pos) DX_TRY(ctx_identity(ctx, nl, &L.d_all_pos, st));
    return DCCRGX_OK;
}

int explicit_build_hood(dccrgx_grid* grid, Hood& h, const NofHint* hint)
{
    DX_TRY(explicit_build_hood_async(grid, h, hint));
    DX_HIP(hipStreamSynchronize(grid->ctx->compute));
    return DCCRGX_OK;
}

int explicit_get_cells(const dccrgx_grid* grid, const Hood& h, int32_t which, uint64_t* ids, size_t cap,
                       size_t* n)
{
    const Explicit* E = grid->ex;
    const std::vector<uint64_t>* v = nullptr;
    std::vector<uint64_t> inner;
    switch (which) {
    case DCCRGX_CELLS_LOCAL: v = &E->local(); break;
    case DCCRGX_CELLS_OUTER: v = &h.outer; break;
    case DCCRGX_CELLS_REMOTE: v = &h.remote; break;
    case DCCRGX_CELLS_INNER: {
        const auto& L = E->hl.at(h.id);
        if (L.inner_all) inner = E->local();
        for (uint32_t p : L.inner_pos) inner.push_back(E->local()[p]);
        v = &inner;
        break;
    }
    default: return set_error(DCCRGX_EINVAL, "unknown cell class %d", which);
    }
    *n = v->size();
    DX_CHECK(cap >= *n && (ids || !*n), DCCRGX_ERANGE, "capacity");
    std::copy(v->begin(), v->end(), ids);
    return DCCRGX_OK;
}

int64_t explicit_host_slot(const dccrgx_grid* grid, uint64_t id)
{
    const Explicit* E = grid->ex;
    const int64_t g = E->find(id);  // a leaf: local or ghost slot, if any
    if (g >= 0 && E->slot_identity) return g;  // one rank
    if (g >= 0 && E->slot_of_g[g] != NO_SLOT) return (int64_t)E->slot_of_g[g];
    // ghosts, and data of refined / unrefined cells kept until
    // clear_refined_unrefined_data
    const uint32_t* x = E->extra.find(id);
    return x ? (int64_t)*x : E->retired_slot(id);
}

// rebuild(): new slot k takes old slot src[k] (-1: value-initialised), looked
// up in the old leaf hash and slot map on the device
// (ids of slots [0, na) from `ids`, of the rest from `tail`)
__global__ void __launch_bounds__(256) k_old_slots(ExView old, const uint32_t* __restrict__ old_slot_of_g,
                                                   const uint64_t* __restrict__ ids, uint64_t na,
                                                   const uint64_t* __restrict__ tail, uint64_t n,
                                                   int64_t* __restrict__ src)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        const int64_t g = ex_find(old, k < na ? ids[k] : tail[k - na]);
        const uint32_t s = g < 0 ? NO_SLOT : old_slot_of_g[g];
        src[k] = s == NO_SLOT ? -1 : (int64_t)s;
    }
}

template <class T>
__global__ void __launch_bounds__(256) k_move(const T* __restrict__ src, const int64_t* __restrict__ from, uint64_t n,
                                              uint32_t words, T* __restrict__ dst)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const uint64_t tot = n * words;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += stride) {
        const uint64_t k = i / words, w = i - k * words;
        const int64_t f = from[k];
        dst[i] = f >= 0 ? src[(uint64_t)f * words + w] : T(0);
    }
}

int explicit_old_slots(const dccrgx_grid* grid, const Explicit* old, int64_t* d_src, hipStream_t st)
{
    const Explicit* E = grid->ex;
    const uint64_t n = E->n_slot_ids();
    if (!n) return DCCRGX_OK;
    uint64_t* d_ids = nullptr;
    const uint64_t *ids = nullptr, *tail = nullptr;
    uint64_t na = n;
    // one rank: the slot ids are the device leaf list, then the retired cells
    // in the order of the device retired table -- no upload of the host copy
    const uint64_t nr = n > E->n ? n - E->n : 0;
    if (E->one_rank && E->slot_identity && E->d_leaves && nr == E->n_ret && (!nr || E->d_ret) &&
        E->retired.size() == nr && std::equal(E->slot_ids_.begin(), E->slot_ids_.end(), E->retired.begin())) {
        ids = E->d_leaves;
        na = E->n;
        tail = E->d_ret;
    } else {
        DX_HIP(ds_malloc(&d_ids, n * 8, st));
        std::vector<uint64_t> h_ids(n);
        for (uint64_t k = 0; k < n; k++) h_ids[k] = E->slot_id(k);
        const int e = dx_h2d(grid->ctx, d_ids, h_ids.data(), n * 8, st);
        if (e != DCCRGX_OK) {
            ds_free(d_ids, st);
            return e;
        }
        ids = d_ids;
    }
    ExView v{};
    v.mp = grid->map;
    v.keys = old->d_keys;
    v.vals = old->d_vals;
    v.mask = old->mask;
    v.bits = old->d_bits;
    v.rank = old->d_rank;
    hipLaunchKernelGGL(k_old_slots, dim3(grid_for(n)), dim3(256), 0, st, v, old->d_slot_of_g, ids, na, tail, n,
                       d_src);
    const hipError_t e = hipGetLastError();
    if (d_ids) ds_free(d_ids, st);  // after the kernel, in stream order
    DX_HIP(e);
    return DCCRGX_OK;
}

// dst[k] = src[from[k]] (or zero), elements of `elem` bytes
// up to 8 fields of 8-byte elements moved behind one read of `from`
struct MoveSet {
    const uint64_t* src[8];
    uint64_t* dst[8];
    int n;
};

__global__ void __launch_bounds__(256) k_move_many(MoveSet m, const int64_t* __restrict__ from, uint64_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        const int64_t f = from[k];
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (j < m.n) m.dst[j][k] = f >= 0 ? m.src[j][f] : 0;
    }
}

int launch_move_many(const void* const* src, void* const* dst, const uint32_t* elem, size_t nf, const int64_t* from,
                     uint64_t n, hipStream_t st)
{
    MoveSet m{};
    auto flush = [&]() {
        if (m.n) hipLaunchKernelGGL(k_move_many, dim3(grid_for(n)), dim3(256), 0, st, m, from, n);
        m.n = 0;
    };
    for (size_t i = 0; i < nf && n; i++) {
        if (elem[i] != 8) {
            DX_TRY(launch_move(src[i], from, n, elem[i], dst[i], st));
            continue;
        }
        m.src[m.n] = (const uint64_t*)src[i];
        m.dst[m.n++] = (uint64_t*)dst[i];
        if (m.n == 8) flush();
    }
    flush();
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

int launch_move(const void* src, const int64_t* from, uint64_t n, uint32_t elem, void* dst, hipStream_t st)
{
    if (!n) return DCCRGX_OK;
    if (elem % 4 == 0)
        hipLaunchKernelGGL(k_move<uint32_t>, dim3(grid_for(n * (elem / 4))), dim3(256), 0, st, (const uint32_t*)src,
                           from, n, elem / 4, (uint32_t*)dst);
    else
        hipLaunchKernelGGL(k_move<uint8_t>, dim3(grid_for(n * elem)), dim3(256), 0, st, (const uint8_t*)src, from, n,
                           elem, (uint8_t*)dst);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

int explicit_slots_of(const dccrgx_grid* grid, const uint64_t* ids, size_t n, int64_t* slots, hipStream_t st)
{
    hipLaunchKernelGGL(k_ex_slots, dim3(grid_for(n)), dim3(256), 0, st, view(grid), grid->ex->d_slot_of_g, ids, n,
                       slots);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

// neighbor gather (dccrgx_gather_neighbors) on explicit grids: the query
// cells' rows of the neighborhood's device CSR (reference list order), each
// entry's field element copied from its storage slot
__global__ void __launch_bounds__(256) k_ex_gather_count(ExView v, const uint64_t* __restrict__ cells, size_t n,
                                                         const uint64_t* __restrict__ nof_row,
                                                         const uint32_t* __restrict__ slot_of_g, uint64_t n_local,
                                                         uint32_t* __restrict__ gidx, uint64_t* __restrict__ row,
                                                         int32_t* __restrict__ err)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t g = ex_find(v, cells[i]);
        if (g < 0 || slot_of_g[g] >= n_local) {  // not a local cell of this rank
            atomicOr(err, 1);
            row[i + 1] = 0;
            gidx[i] = 0;
            continue;
        }
        const uint32_t r = slot_of_g[g];  // its row: local position
        gidx[i] = r;
        row[i + 1] = nof_row[r + 1] - nof_row[r];
    }
}

__global__ void __launch_bounds__(256) k_ex_gather_fill(const uint32_t* __restrict__ gidx, size_t n,
                                                        const uint64_t* __restrict__ nof_row,
                                                        const uint32_t* __restrict__ nof_g,
                                                        const uint32_t* __restrict__ slot_of_g,
                                                        const uint64_t* __restrict__ row, const uint8_t* __restrict__ field,
                                                        uint32_t elem, uint8_t* __restrict__ out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t g = gidx[i];  // row of the query cell
        uint64_t w = row[i];
        for (uint64_t e = nof_row[g]; e < nof_row[g + 1]; e++, w++) {
            const uint8_t* src = field + (uint64_t)slot_of_g[nof_g[e]] * elem;
            uint8_t* dst = out + w * elem;
            if (elem % 4 == 0)
                for (uint32_t k = 0; k < elem; k += 4)
                    *reinterpret_cast<uint32_t*>(dst + k) = *reinterpret_cast<const uint32_t*>(src + k);
            else
                for (uint32_t k = 0; k < elem; k++) dst[k] = src[k];
        }
    }
}

int explicit_gather_neighbors(const dccrgx_grid* grid, const Hood& h, const Field& F, const uint64_t* cells, size_t n,
                              uint64_t* row, void* out, size_t cap_bytes, hipStream_t st)
{
    const Explicit* E = grid->ex;
    DX_CHECK(h.d_nof_row, DCCRGX_EINTERNAL, "no device lists for neighborhood %d", h.id);
    uint32_t* gidx = nullptr;
    int32_t* d_err = nullptr;
    DX_HIP(dx_malloc(&gidx, std::max<size_t>(n, 1) * 4));
    DX_HIP(dx_malloc(&d_err, 4));
    auto done = [&](int code) {
        (void)dx_free(gidx);
        (void)dx_free(d_err);
        return code;
    };
    if (hipMemsetAsync(d_err, 0, 4, st) != hipSuccess) return done(set_error(DCCRGX_EHIP, "memset"));
    if (n)
        hipLaunchKernelGGL(k_ex_gather_count, dim3(grid_for(n)), dim3(256), 0, st, view(grid), cells, n, h.d_nof_row,
                           E->d_slot_of_g, E->n_local(), gidx, row, d_err);
    uint64_t total = 0;
    int s = device_scan_rows(row, n, st, &total);
    if (s != DCCRGX_OK) return done(s);
    int32_t err = 0;
    if (hipMemcpy(&err, d_err, 4, hipMemcpyDeviceToHost) != hipSuccess) return done(set_error(DCCRGX_EHIP, "copy"));
    if (err) return done(set_error(DCCRGX_ENOTFOUND, "a query cell is not a local cell of this rank"));
    if (!out) return done(DCCRGX_OK);
    if (cap_bytes < total * F.elem)
        return done(set_error(DCCRGX_ERANGE, "capacity %zu < %llu bytes", cap_bytes,
                              (unsigned long long)(total * F.elem)));
    if (n)
        hipLaunchKernelGGL(k_ex_gather_fill, dim3(grid_for(n)), dim3(256), 0, st, (const uint32_t*)gidx, n,
                           h.d_nof_row, h.d_nof_g, E->d_slot_of_g, (const uint64_t*)row, (const uint8_t*)F.ptr, F.elem,
                           (uint8_t*)out);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
        return done(set_error(DCCRGX_EHIP, "gather kernel failed"));
    return done(DCCRGX_OK);
}

// get_neighbors_of (dccrg.hpp:836-883) is a lookup of lists built with the
// grid (initialize_neighbors, :8371-8420): the query cells' rows are copied
// out of the neighborhood's device CSR of every leaf -- row lengths, a scan,
// then one coalesced copy of the ids and offsets
int explicit_neighbors_of(const dccrgx_grid* grid, const Hood& h, const uint64_t* cells, size_t n, uint64_t* row,
                          uint64_t* ids, int32_t* off3, size_t cap, hipStream_t st)
{
    DX_CHECK(h.d_nof_row, DCCRGX_EINTERNAL, "no device lists for neighborhood %d", h.id);
    uint32_t* gq = nullptr;
    int32_t* d_err = nullptr;
    DX_HIP(ds_malloc(&gq, std::max<size_t>(n, 1) * 4, st));
    DX_HIP(ds_malloc(&d_err, 4, st));
    auto done = [&](int code) {
        (void)ds_free(gq, st);
        (void)ds_free(d_err, st);
        return code;
    };
    if (hipMemsetAsync(d_err, 0, 4, st) != hipSuccess) return done(set_error(DCCRGX_EHIP, "memset"));
    const Explicit* E = grid->ex;
    if (n)
        hipLaunchKernelGGL(k_ex_query_rows, dim3(grid_for(n)), dim3(256), 0, st, view(grid), cells, n, h.d_nof_row,
                           (const uint32_t*)E->d_slot_of_g, E->n_local(), gq, row, d_err);
    uint64_t total = 0;
    int s = device_scan_rows(row, n, st, nullptr);
    if (s != DCCRGX_OK) return done(s);
    int32_t err = 0;
    {  // the total and the error word behind one synchronisation
        const D2H rb[2] = {{&total, row + n, 8}, {&err, d_err, 4}};
        if ((s = dx_d2h_many(grid->ctx, rb, 2, st)) != DCCRGX_OK) return done(s);
    }
    if (err & 1) return done(set_error(DCCRGX_ENOTFOUND, "cell does not exist"));
    if (err & 4) {  // rows of other processes' cells: searched now (the reference's lists of every cell)
        if (hipMemsetAsync(d_err, 0, 4, st) != hipSuccess) return done(set_error(DCCRGX_EHIP, "memset"));
        hipLaunchKernelGGL(k_ex_nof, dim3(grid_for(n)), dim3(256), 0, st, view(grid), (const int32_t*)h.d_of_c, h.K,
                           cells, n, row, (uint64_t*)nullptr, (int32_t*)nullptr, (uint32_t*)nullptr, d_err,
                           (uint64_t*)nullptr);
        if ((s = device_scan_rows(row, n, st, &total)) != DCCRGX_OK) return done(s);
        if ((s = dx_d2h(grid->ctx, &err, d_err, 4, st)) != DCCRGX_OK) return done(s);
        if (err) return done(set_error(err & 1 ? DCCRGX_ENOTFOUND : DCCRGX_EINTERNAL,
                                       err & 1 ? "cell does not exist" : "neighbor more than one level apart"));
        if (!ids) return done(DCCRGX_OK);
        if (cap < total) return done(set_error(DCCRGX_ERANGE, "capacity %zu < %llu", cap, (unsigned long long)total));
        hipLaunchKernelGGL(k_ex_nof, dim3(grid_for(n)), dim3(256), 0, st, view(grid), (const int32_t*)h.d_of_c, h.K,
                           cells, n, row, ids, off3, (uint32_t*)nullptr, d_err, (uint64_t*)nullptr);
        if (hipGetLastError() != hipSuccess) return done(set_error(DCCRGX_EHIP, "neighbor list search failed"));
        return done(DCCRGX_OK);
    }
    if (!ids) return done(DCCRGX_OK);
    if (cap < total) return done(set_error(DCCRGX_ERANGE, "capacity %zu < %llu", cap, (unsigned long long)total));
    if (n)
        hipLaunchKernelGGL(k_rows_gather, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, (const uint32_t*)gq,
                           (uint64_t)n, h.d_nof_row, (const uint64_t*)row, h.d_nof_id, h.d_nof_off, ids, off3);
    if (hipGetLastError() != hipSuccess) return done(set_error(DCCRGX_EHIP, "neighbor list copy failed"));
    return done(DCCRGX_OK);
}

int explicit_neighbors_to(const dccrgx_grid* grid, const Hood& h, const uint64_t* cells, size_t n, uint64_t* row,
                          uint64_t* ids, size_t cap, hipStream_t st)
{
    // rows of the neighborhood's device neighbors_to CSR (ascending leaf
    // indices = ascending ids), looked up and copied as neighbors_of's are
    DX_CHECK(h.d_nto_row, DCCRGX_EINTERNAL, "no device lists for neighborhood %d", h.id);
    uint32_t* gq = nullptr;
    int32_t* d_err = nullptr;
    DX_HIP(ds_malloc(&gq, std::max<size_t>(n, 1) * 4, st));
    DX_HIP(ds_malloc(&d_err, 4, st));
    auto done = [&](int code) {
        (void)ds_free(gq, st);
        (void)ds_free(d_err, st);
        return code;
    };
    if (hipMemsetAsync(d_err, 0, 4, st) != hipSuccess) return done(set_error(DCCRGX_EHIP, "memset"));
    const Explicit* E = grid->ex;
    if (n)
        hipLaunchKernelGGL(k_ex_query_rows, dim3(grid_for(n)), dim3(256), 0, st, view(grid), cells, n, h.d_nto_row,
                           (const uint32_t*)E->d_slot_of_g, E->n_local(), gq, row, d_err);
    uint64_t total = 0;
    int s = device_scan_rows(row, n, st, &total);  // synchronises (total)
    if (s != DCCRGX_OK) return done(s);
    int32_t err = 0;
    if ((s = dx_d2h(grid->ctx, &err, d_err, 4, st)) != DCCRGX_OK) return done(s);
    if (err & 1) return done(set_error(DCCRGX_ENOTFOUND, "cell does not exist"));
    if (err & 4) {  // rows of other processes' cells: the reference's search, now
        uint64_t* trow = nullptr;
        uint32_t* tg = nullptr;
        uint32_t* iota = nullptr;
        auto done2 = [&](int code) {
            ds_free(trow, st);
            ds_free(tg, st);
            ds_free(iota, st);
            return done(code);
        };
        if ((s = nto_direct(grid, h, cells, n, &trow, &tg, st)) != DCCRGX_OK) return done2(s);
        if (hipMemcpyAsync(row, trow, (n + 1) * 8, hipMemcpyDeviceToDevice, st) != hipSuccess)
            return done2(set_error(DCCRGX_EHIP, "copy"));
        if ((s = dx_d2h(grid->ctx, &total, trow + n, 8, st)) != DCCRGX_OK) return done2(s);
        if (!ids) return done2(DCCRGX_OK);
        if (cap < total) return done2(set_error(DCCRGX_ERANGE, "capacity %zu < %llu", cap, (unsigned long long)total));
        if ((s = device_iota(&iota, n, st)) != DCCRGX_OK) return done2(s);
        hipLaunchKernelGGL(k_rows_gather_g, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, (const uint32_t*)iota,
                           (uint64_t)n, (const uint64_t*)trow, (const uint64_t*)row, (const uint32_t*)tg,
                           (const uint64_t*)E->d_leaves, ids);
        if (hipGetLastError() != hipSuccess) return done2(set_error(DCCRGX_EHIP, "neighbor list copy failed"));
        return done2(DCCRGX_OK);
    }
    if (!ids) return done(DCCRGX_OK);
    if (cap < total) return done(set_error(DCCRGX_ERANGE, "capacity %zu < %llu", cap, (unsigned long long)total));
    if (n)
        hipLaunchKernelGGL(k_rows_gather_g, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, (const uint32_t*)gq,
                           (uint64_t)n, h.d_nto_row, (const uint64_t*)row, h.d_nto_g,
                           (const uint64_t*)grid->ex->d_leaves, ids);
    if (hipGetLastError() != hipSuccess) return done(set_error(DCCRGX_EHIP, "neighbor list copy failed"));
    return done(DCCRGX_OK);
}

namespace {
struct ExExists {
    ExView v;
    __device__ bool operator()(uint64_t c) const { return ex_find(v, c) >= 0; }
};
}  // namespace

int explicit_face_neighbors(const dccrgx_grid* grid, const uint64_t* cells, size_t n, uint64_t* row,
                            uint64_t* ids, int32_t* dirs, size_t cap, hipStream_t st)
{
    return face_neighbors_launch(grid->map, grid->params.periodic, ExExists{view(grid)}, cells, n, row, ids, dirs,
                                 cap, st);
}

int explicit_region(const dccrgx_grid* grid, const Hood& h, int32_t region, ExRegion* out)
{
    const Explicit* E = grid->ex;
    const auto it = E->hl.find(h.id);
    DX_CHECK(it != E->hl.end(), DCCRGX_EINTERNAL, "no lists for neighborhood %d", h.id);
    const auto& L = it->second;
    out->pos = region == DCCRGX_REGION_INNER ? L.d_inner_pos
               : region == DCCRGX_REGION_OUTER ? L.d_outer_pos : L.d_all_pos;
    out->n = region == DCCRGX_REGION_INNER ? (L.inner_all ? E->n_local() : L.inner_pos.size())
             : region == DCCRGX_REGION_OUTER ? L.outer_pos.size() : E->n_local();
    out->local_slot = E->d_local_slot;
    out->level = E->d_level;
    return DCCRGX_OK;
}

int explicit_gol(dccrgx_grid* grid, const Hood& h, const Field& in, const Field& out, const Field& cnt,
                 int32_t region, hipStream_t st)
{
    ExRegion R;
    DX_TRY(explicit_region(grid, h, region, &R));
    if (!R.n) return DCCRGX_OK;
    hipLaunchKernelGGL(k_ex_gol, dim3(grid_for(R.n)), dim3(256), 0, st, (const uint32_t*)in.ptr,
                       (uint32_t*)out.ptr, (uint32_t*)cnt.ptr, h.d_st_row, h.d_st_slot, R.local_slot, R.pos, R.n);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

// local values in ascending id order <-> slots [0, nl)
int explicit_local_copy(const dccrgx_grid* grid, const Field& F, void* host, bool to_device)
{
    const uint64_t n = grid->ex->n_local();
    if (!n) return DCCRGX_OK;
    hipStream_t st = grid->ctx->compute;
    if (to_device) DX_TRY(dx_h2d(grid->ctx, F.ptr, host, n * F.elem, st));
    else DX_TRY(dx_d2h(grid->ctx, host, F.ptr, n * F.elem, st));
    DX_HIP(hipStreamSynchronize(st));
    return DCCRGX_OK;
}

// id of each local slot [0, nl): the ascending local ids
int explicit_local_ids(const dccrgx_grid* grid, uint64_t* d_ids, hipStream_t st)
{
    const Explicit* E = grid->ex;
    const uint64_t n = E->n_local();
    if (!n) return DCCRGX_OK;
    hipLaunchKernelGGL(k_local_ids, dim3(grid_for(n)), dim3(256), 0, st, (const uint64_t*)E->d_leaves,
                       (const uint32_t*)E->d_local_g, n, d_ids);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

}  // namespace dccrgx
