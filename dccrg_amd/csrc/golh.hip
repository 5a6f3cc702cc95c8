// golh.hip -- the AMR-aware game of life of tests/game_of_life/solve.hpp:40-170
// (= solve_optimized.hpp:40-133), "emulating unrefined behaviour" on refined
// grids (tests/game_of_life/refined*.cpp).
//
// The cell is the test's Cell::data, 9 x u64 in one 72-byte field
// (tests/game_of_life/cell.hpp:32-47): data[0] the state, data[1..8] the
// level-0 parents of live neighbors.  One call of get_live_neighbors is
//   (1) record: every local cell lists the distinct level-0 parents of its
//       live neighbors_of entries (own parent skipped, in list order),
//   (2) update_copies_of_remote_neighbors of the field,
//   (3) spread: a cell takes the union with the lists of neighbors that share
//       its level-0 parent (its siblings, always on the same rank),
//   (4) apply: B3/S23 on the number of recorded parents, lists reset to
//       error_cell.
// (1) and (4) are independent per cell.  The reference runs (3) as a
// sequential loop in unordered_map order, where a cell may see merges done
// earlier in the loop; here every cell takes the union of its own and its
// siblings' (1)-lists at once.  Both give the union of the whole sibling
// group whenever siblings are mutual neighbors (cells refined at most once
// and neighborhood length >= 1, the setting solve_optimized.hpp states it is
// for); there the reference's result does not depend on its iteration order
// and the two are equal (tests/test_oracle_gol_amr.py checks both orders).
// The reference's aborts (list overflow, dead neighbor already recorded) come
// back as DCCRGX_ERANGE / DCCRGX_ESTATE.
//
// Uniform grids: level-0 parent = the cell, so (3) finds no siblings; the
// count is taken from the cell's own list in (4).
#include "grid.hpp"

namespace dccrgx {

namespace {

constexpr int W = 9;  // u64 words per cell
enum { ERR_OVERFLOW = 1, ERR_DEAD_RECORDED = 2 };

__device__ __forceinline__ uint64_t l0_parent(const MapParams& p, uint64_t cell)
{
    uint64_t idx[3];
    int l = 0;
    if (!map_indices(p, cell, idx, &l)) return 0;
    return l == 0 ? cell : map_cell(p, idx, 0);
}

// insert v into an error_cell-terminated list of 8 (no duplicates); false on overflow
__device__ __forceinline__ bool list_insert(uint64_t (&L)[8], uint64_t v)
{
    for (int i = 0; i < 8; i++) {
        if (L[i] == v) return true;
        if (L[i] == 0) {
            L[i] = v;
            return true;
        }
    }
    return false;
}

__device__ __forceinline__ bool list_has(const uint64_t (&L)[8], uint64_t v)
{
    bool f = false;
    for (int i = 0; i < 8; i++) f |= L[i] == v;
    return f;
}

__device__ __forceinline__ void record(uint64_t (&L)[8], uint64_t nparent, uint64_t nalive, int& err)
{
    if (nalive == 0) {
        if (list_has(L, nparent)) err |= ERR_DEAD_RECORDED;  // solve.hpp:73-84
        return;
    }
    if (!list_insert(L, nparent)) err |= ERR_OVERFLOW;       // solve.hpp:86-96
}

__device__ __forceinline__ void apply(uint64_t* d, uint32_t live)
{
    for (int i = 1; i < W; i++) d[i] = 0;
    if (live == 3) d[0] = 1;                                  // solve.hpp:158-166
    else if (live != 2) d[0] = 0;
}

// (1) on a uniform grid: neighbors_of = the neighborhood items in order
__global__ void __launch_bounds__(256) k_golh_record_u(UGeom g, uint64_t* __restrict__ data,
                                                      const int32_t* __restrict__ items, int K, uint64_t lin0,
                                                      uint64_t n, int* __restrict__ err_out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const uint64_t soff = (uint64_t)(-g.cbase * (int64_t)g.S);
    int err = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t lin = lin0 + i;
        int64_t a, b, c;
        ug_decompose(g, lin, a, b, c);
        uint64_t L[8] = {0, 0, 0, 0, 0, 0, 0, 0};
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
            int64_t cw = c2;
            if (c2 < 0 || c2 >= (int64_t)g.LC) {
                if (!g.perC) continue;
                cw = ug_wrap(c2, (int64_t)g.LC);
            }
            const uint64_t nid = (uint64_t)a2 + g.LA * ((uint64_t)b2 + g.LB * (uint64_t)cw) + 1;
            if (nid == lin + 1) continue;  // same level-0 parent
            record(L, nid, data[ug_slot(g, a2, b2, c2) * W], err);
        }
        uint64_t* own = data + (lin + soff) * W;
        for (int j = 0; j < 8; j++) own[1 + j] = L[j];
    }
    if (err) atomicOr(err_out, err);
}

struct XArgs {
    MapParams map;
    const uint64_t* leaves;      // global leaves (ascending)
    const uint32_t* local_g;     // local position -> global leaf index
    const uint32_t* local_slot;  // local position -> storage slot
    const uint64_t* nof_row;     // neighbors_of CSR of the local cells (row = local position), reference order
    const uint64_t* nof_id;
    const uint32_t* nof_g;
    const uint32_t* slot_of_g;   // global leaf index -> storage slot
    uint64_t n;                  // local cells
};

// (1) on an explicit grid
__global__ void __launch_bounds__(256) k_golh_record_x(XArgs x, uint64_t* __restrict__ data,
                                                      int* __restrict__ err_out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    int err = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < x.n; i += stride) {
        const uint32_t gi = x.local_g[i];
        const uint64_t own_parent = l0_parent(x.map, x.leaves[gi]);
        uint64_t L[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (uint64_t e = x.nof_row[i]; e < x.nof_row[i + 1]; e++) {  // rows by local position
            const uint64_t nid = x.nof_id[e];
            if (nid == 0) continue;
            const uint64_t np = l0_parent(x.map, nid);
            if (np == own_parent) continue;
            record(L, np, data[(uint64_t)x.slot_of_g[x.nof_g[e]] * W], err);
        }
        uint64_t* own = data + (uint64_t)x.local_slot[i] * W;
        for (int j = 0; j < 8; j++) own[1 + j] = L[j];
    }
    if (err) atomicOr(err_out, err);
}

// (3) on an explicit grid: union with the siblings' lists -> live count
__global__ void __launch_bounds__(256) k_golh_spread_x(XArgs x, const uint64_t* __restrict__ data,
                                                      uint32_t* __restrict__ live, int* __restrict__ err_out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    int err = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < x.n; i += stride) {
        const uint32_t gi = x.local_g[i];
        const uint64_t own_parent = l0_parent(x.map, x.leaves[gi]);
        uint64_t L[8];
        const uint64_t* own = data + (uint64_t)x.local_slot[i] * W;
        for (int j = 0; j < 8; j++) L[j] = own[1 + j];
        for (uint64_t e = x.nof_row[i]; e < x.nof_row[i + 1]; e++) {  // rows by local position
            const uint64_t nid = x.nof_id[e];
            if (nid == 0 || l0_parent(x.map, nid) != own_parent) continue;
            const uint64_t* nd = data + (uint64_t)x.slot_of_g[x.nof_g[e]] * W;
            for (int j = 0; j < 8; j++) {
                const uint64_t v = nd[1 + j];
                if (v == 0) break;
                if (!list_insert(L, v)) err |= ERR_OVERFLOW;  // solve.hpp:136-143
            }
        }
        uint32_t c = 0;
        for (int j = 0; j < 8; j++) c += L[j] != 0 ? 1u : 0u;
        live[i] = c;
    }
    if (err) atomicOr(err_out, err);
}

// (4) on an explicit grid
__global__ void __launch_bounds__(256) k_golh_apply_x(XArgs x, uint64_t* __restrict__ data,
                                                     const uint32_t* __restrict__ live)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < x.n; i += stride)
        apply(data + (uint64_t)x.local_slot[i] * W, live[i]);
}

// (4) on a uniform grid: the count is the cell's own list
__global__ void __launch_bounds__(256) k_golh_apply_u(UGeom g, uint64_t* __restrict__ data, uint64_t lin0,
                                                     uint64_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const uint64_t soff = (uint64_t)(-g.cbase * (int64_t)g.S);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t* d = data + (lin0 + i + soff) * W;
        uint32_t c = 0;
        for (int j = 1; j < W; j++) c += d[j] != 0 ? 1u : 0u;
        apply(d, c);
    }
}

unsigned blocks_for(uint64_t n)
{
    uint64_t b = (n + 255) / 256;
    if (b > 256 * 16) b = 256 * 16;
    return (unsigned)(b ? b : 1);
}

int xargs(const dccrgx_grid* grid, const Hood& h, XArgs* x)
{
    const Explicit* E = grid->ex;
    DX_CHECK(E && h.d_nof_row, DCCRGX_EINTERNAL, "no device lists for neighborhood %d", h.id);
    x->map = grid->map;
    x->leaves = E->d_leaves;
    x->local_g = E->d_local_g;
    x->local_slot = E->d_local_slot;
    x->nof_row = h.d_nof_row;
    x->nof_id = h.d_nof_id;
    x->nof_g = h.d_nof_g;
    x->slot_of_g = E->d_slot_of_g;
    x->n = E->n_local();
    return DCCRGX_OK;
}

// device scratch: error word + live counts, freed on every exit path
struct Scratch {
    int* err = nullptr;
    uint32_t* live = nullptr;
    ~Scratch()
    {
        if (err) (void)dx_free(err);
        if (live) (void)dx_free(live);
    }
};

int finish(int* d_err, hipStream_t st)
{
    int err = 0;
    DX_HIP(hipMemcpyAsync(&err, d_err, sizeof err, hipMemcpyDeviceToHost, st));
    DX_HIP(hipStreamSynchronize(st));
    DX_CHECK(!(err & ERR_OVERFLOW), DCCRGX_ERANGE,
             "No more room in live neighbor list (more than 8 live level-0 parents, solve.hpp:93-96)");
    DX_CHECK(!(err & ERR_DEAD_RECORDED), DCCRGX_ESTATE,
             "a dead neighbor's level-0 parent is already recorded as alive (solve.hpp:73-84)");
    return DCCRGX_OK;
}

int golh_phase(dccrgx_grid* grid, const Hood& h, const Field& F, int32_t phase)
{
    hipStream_t st = grid->ctx->compute;
    Scratch s;
    DX_HIP(dx_malloc(&s.err, sizeof(int)));
    DX_HIP(hipMemsetAsync(s.err, 0, sizeof(int), st));
    uint64_t* data = (uint64_t*)F.ptr;
    if (grid->uniform) {
        const uint64_t n = grid->n_local;
        if (n) {
            if (phase == DCCRGX_GOLH_RECORD)
                hipLaunchKernelGGL(k_golh_record_u, dim3(blocks_for(n)), dim3(256), 0, st, grid->g, data,
                                   (const int32_t*)h.d_of_c, h.K, grid->g.lo, n, s.err);
            else
                hipLaunchKernelGGL(k_golh_apply_u, dim3(blocks_for(n)), dim3(256), 0, st, grid->g, data,
                                   grid->g.lo, n);
            DX_HIP(hipGetLastError());
        }
        return finish(s.err, st);
    }
    XArgs x;
    DX_TRY(xargs(grid, h, &x));
    if (x.n) {
        if (phase == DCCRGX_GOLH_RECORD) {
            hipLaunchKernelGGL(k_golh_record_x, dim3(blocks_for(x.n)), dim3(256), 0, st, x, data, s.err);
        } else {
            DX_HIP(dx_malloc(&s.live, x.n * sizeof(uint32_t)));
            hipLaunchKernelGGL(k_golh_spread_x, dim3(blocks_for(x.n)), dim3(256), 0, st, x,
                               (const uint64_t*)data, s.live, s.err);
            hipLaunchKernelGGL(k_golh_apply_x, dim3(blocks_for(x.n)), dim3(256), 0, st, x, data,
                               (const uint32_t*)s.live);
        }
        DX_HIP(hipGetLastError());
    }
    return finish(s.err, st);
}

}  // namespace
}  // namespace dccrgx

using namespace dccrgx;

extern "C" {

int dccrgx_gol_amr_phase(dccrgx_grid* grid, int32_t hood_id, int32_t f_data, int32_t phase)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    const Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    DX_CHECK(f_data >= 0 && (size_t)f_data < grid->fields.size(), DCCRGX_EINVAL, "bad field %d", f_data);
    const Field& F = grid->fields[f_data];
    DX_CHECK(F.elem == 8 * W && !F.variable, DCCRGX_EINVAL, "the cell is 9 x u64 (tests/game_of_life/cell.hpp:47)");
    DX_CHECK(phase == DCCRGX_GOLH_RECORD || phase == DCCRGX_GOLH_SPREAD_APPLY, DCCRGX_EINVAL, "bad phase %d",
             phase);
    return golh_phase(grid, *h, F, phase);
}

int dccrgx_gol_amr_step(dccrgx_grid* grid, int32_t hood_id, int32_t f_data)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_TRY(dccrgx_gol_amr_phase(grid, hood_id, f_data, DCCRGX_GOLH_RECORD));
    DX_TRY(dccrgx_halo_update(grid, hood_id, &f_data, 1));  // solve.hpp:105
    return dccrgx_gol_amr_phase(grid, hood_id, f_data, DCCRGX_GOLH_SPREAD_APPLY);
}

}  // extern "C"
