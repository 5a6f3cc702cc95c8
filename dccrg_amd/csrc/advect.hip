// advect.hip -- the advection solver of tests/advection/solve.hpp on the device.
//
// The reference loops over inner (or outer) cells and, for every face
// neighbor in the iteration cache, computes one upwind flux and adds it to
// BOTH cells (solve.hpp:224-230), skipping the negative direction of
// local-local pairs so each face is solved once (:125-128).  On the GPU that
// scatter would need atomics on doubles; instead every local cell gathers
// the fluxes of all of its own faces (both directions).  Per face the flux is
// the same expression evaluated in the same order (contraction off), so each
// face value is bit-identical to the reference's; only the order in which a
// cell's face fluxes are summed differs (fp64, checked at 1e-12 relative).
//
// Fields are SoA f64 (one field per Cell::data member, cell.hpp:34-44), so
// the per-step halo moves only density -- the reference's
// transfer_all_data = false datatype (cell.hpp:47-57).
#include <cfloat>
#include <cstring>

#include "exview.hpp"
#include "grid.hpp"

namespace dccrgx {

namespace {

struct AdvPtrs {
    const double* rho;
    double* flux;
    const double* v[3];
    const double* l[3];
};

unsigned grid_for(uint64_t n)
{
    uint64_t g = (n + 255) / 256;
    if (g > 256 * 64) g = 256 * 64;
    if (g == 0) g = 1;
    return (unsigned)g;
}

// flux of one face, solve.hpp:134-221; dir = +-1, +-2, +-3 (x, y, z).
// Returns the contribution to the cell's flux: -flux / V for dir > 0,
// +flux / V for dir < 0 (:224-230).
__device__ inline double face_term(const AdvPtrs& p, uint64_t c, uint64_t n, int dir, double dt, double vol_c)
{
#pragma clang fp contract(off)
    const int ax = (dir > 0 ? dir : -dir) - 1;
    const int a1 = ax == 0 ? 1 : 0, a2 = ax == 2 ? 1 : 2;  // the other two axes, ascending
    const double area_c = p.l[a1][c] * p.l[a2][c], area_n = p.l[a1][n] * p.l[a2][n];
    const double min_area = area_c < area_n ? area_c : area_n;
    const double lc = p.l[ax][c], ln = p.l[ax][n];
    const double v = (lc * p.v[ax][n] + ln * p.v[ax][c]) / (lc + ln);
    const double rho_c = p.rho[c], rho_n = p.rho[n];
    double f;
    if (dir > 0) f = (v >= 0 ? rho_c : rho_n) * dt * v * min_area;
    else f = (v >= 0 ? rho_n : rho_c) * dt * v * min_area;
    return dir > 0 ? -(f / vol_c) : f / vol_c;
}

// face classification of one cache entry, solve.hpp:73-99
__device__ inline int face_dir(int64_t cl, int64_t nl, const int32_t* off)
{
    int overlaps = 0, direction = 0;
    for (int d = 0; d < 3; d++) {
        const int64_t o = off[d];
        if (o < cl && o > -nl) overlaps++;
        else if (o == cl) direction = d + 1;
        else if (o == -nl) direction = -(d + 1);
    }
    // overlaps > 2 would be a neighbor overlapping the cell itself, which a
    // valid leaf set cannot produce (the reference aborts, :101-116)
    return overlaps == 2 ? direction : 0;
}

// face lists of local cells from the stencil rows, in one pass.  Column k of
// the first six holds the cell's face neighbor in direction k = -x, +x, -y,
// +y, -z, +z (the first one met in stencil order; 0xffffffff: none), so the
// kernels know each column's axis and sign at compile time; further
// neighbors in a direction (finer cells: 2 per face in 2-D, 4 in 3-D) go to
// the overflow with their direction, o_cnt[q] of them from the cell's
// stencil row offset (a row's overflow is a subset of the row): no count
// pass, scan or read-back.  *over = 1 when some cell has overflow.
__global__ void __launch_bounds__(256) k_face_build(const uint64_t* __restrict__ st_row,
                                                    const uint32_t* __restrict__ st_slot,
                                                    const int32_t* __restrict__ st_off,
                                                    const uint32_t* __restrict__ local_g,
                                                    const uint8_t* __restrict__ level, int M, uint64_t n,
                                                    uint32_t* __restrict__ ell_slot, uint32_t* __restrict__ o_cnt,
                                                    uint32_t* __restrict__ o_slot, int8_t* __restrict__ o_dir,
                                                    uint32_t* __restrict__ over)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += stride) {
        const int64_t cl = 1ll << (M - level[local_g[q]]);
        uint32_t used = 0, k = 0;
        const uint64_t base = st_row[q];
        row_walk4(base, st_row[q + 1], st_slot, st_off, [&](uint64_t, uint32_t nb, int32_t x, int32_t y, int32_t z) {
            const int32_t o[3] = {x, y, z};
            const int dir = face_dir(cl, 1ll << (M - level[nb]), o);
            if (!dir) return;
            const int col = 2 * ((dir > 0 ? dir : -dir) - 1) + (dir > 0 ? 1 : 0);
            if (!(used >> col & 1u)) {
                used |= 1u << col;
                ell_slot[col * n + q] = nb;
                return;
            }
            o_slot[base + k] = nb;
            o_dir[base + k] = (int8_t)dir;
            k++;
        });
        for (int col = 0; col < 6; col++)
            if (!(used >> col & 1u)) ell_slot[col * n + q] = 0xffffffffu;
        o_cnt[q] = k;
        if (__ballot(k > 0) && (threadIdx.x & 63) == 0) atomicOr(over, 1u);
    }
}

// explicit grids over the face lists: the 6 column-major faces are
// independent loads (issued together), the overflow is rare
struct FaceView {  // trivially copyable kernel argument
    uint64_t n;
    const uint32_t* ell_slot;
    const uint64_t* o_base;
    const uint32_t* o_cnt;
    const uint32_t* o_slot;
    const int8_t* o_dir;
    const uint32_t* over;  // device flag (a scalar load per wave)
};

__device__ inline double sel3(int k, double x0, double x1, double x2) { return k == 0 ? x0 : (k == 1 ? x1 : x2); }

// face_term over values already in registers (same expression, same order)
__device__ inline double face_term_v(int dir, double dt, double vol_c, const double lc3[3], const double vc3[3],
                                     double rho_c, double ln0, double ln1, double ln2, double vn, double rho_n)
{
#pragma clang fp contract(off)
    const int ax = (dir > 0 ? dir : -dir) - 1;
    const int a1 = ax == 0 ? 1 : 0, a2 = ax == 2 ? 1 : 2;
    const double area_c = lc3[a1] * lc3[a2];
    const double area_n = sel3(a1, ln0, ln1, ln2) * sel3(a2, ln0, ln1, ln2);
    const double min_area = area_c < area_n ? area_c : area_n;
    const double lc = lc3[ax], ln = sel3(ax, ln0, ln1, ln2);
    const double v = (lc * vn + ln * vc3[ax]) / (lc + ln);
    double f;
    if (dir > 0) f = (v >= 0 ? rho_c : rho_n) * dt * v * min_area;
    else f = (v >= 0 ? rho_n : rho_c) * dt * v * min_area;
    return dir > 0 ? -(f / vol_c) : f / vol_c;
}

// explicit grids over the face lists: the 6 column-major faces are
// independent loads, and every neighbour value of all 6 faces is gathered
// unconditionally (an absent face reads the cell itself and is masked out)
// so the ~30 gathers of a cell are in flight together instead of one face's
// loads waiting behind the previous face's branch.  Column k's direction is
// k itself (k_face_build), so the axis of the velocity gathered and the
// face expression are resolved at compile time.  The overflow (faces next
// to finer cells beyond the first per direction) is rare.
//
// rho_out == null: calculate_fluxes (flux[c] += the cell's face terms).
// rho_out != null: one fused solver step (calculate_fluxes then
// apply_fluxes, solve.hpp:283-293): rho_out[c] = rho[c] + (flux[c] + terms),
// the same additions in the same order as the two passes, and flux[c] left
// 0; rho_out is the other buffer of a double-buffered density, so no flux
// array is written and read back.  Slots [t0, t1) (ghosts, retired cells)
// are carried over to rho_out unchanged.
template <int WPE>
__global__ void __launch_bounds__(256, WPE) k_ex_advect_faces(AdvPtrs p, double dt, FaceView fc,
                                                         const uint32_t* __restrict__ local_g,
                                                         const uint32_t* __restrict__ pos, uint64_t n,
                                                         double* __restrict__ rho_out, uint64_t t0, uint64_t t1)
{
#pragma clang fp contract(off)
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)xcd_block() * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t q = pos ? pos[i] : (uint32_t)i;
        const uint32_t c = local_g ? local_g[q] : q;  // null: identity (explicit local slots are [0, n_local))
        uint32_t s[6];
#pragma unroll
        for (int k = 0; k < 6; k++) s[k] = fc.ell_slot[k * fc.n + q];
        const double lc3[3] = {p.l[0][c], p.l[1][c], p.l[2][c]};
        const double vc3[3] = {p.v[0][c], p.v[1][c], p.v[2][c]};
        const double rho_c = p.rho[c];
        double acc = p.flux[c];
        double ln0[6], ln1[6], ln2[6], vn[6], rn[6];
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const uint32_t nb = s[k] != 0xffffffffu ? s[k] : c;
            ln0[k] = p.l[0][nb];
            ln1[k] = p.l[1][nb];
            ln2[k] = p.l[2][nb];
            vn[k] = p.v[k >> 1][nb];
            rn[k] = p.rho[nb];
        }
        const double vol = lc3[0] * lc3[1] * lc3[2];
#pragma unroll
        for (int k = 0; k < 6; k++)
            if (s[k] != 0xffffffffu)
                acc += face_term_v((k & 1) ? (k >> 1) + 1 : -((k >> 1) + 1), dt, vol, lc3, vc3, rho_c, ln0[k], ln1[k],
                                   ln2[k], vn[k], rn[k]);
        if (*fc.over)
            for (uint64_t e = fc.o_base[q], e1 = e + fc.o_cnt[q]; e < e1; e++)
                acc += face_term(p, c, fc.o_slot[e], fc.o_dir[e], dt, vol);
        if (!rho_out) {
            p.flux[c] = acc;
        } else {
            rho_out[c] = rho_c + acc;
            if (p.flux[c] != 0.0) p.flux[c] = 0.0;
        }
    }
    if (rho_out)
        for (uint64_t s = t0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; s < t1; s += stride) rho_out[s] = p.rho[s];
}

// k_ex_advect_faces with the per-cell and gathered loads as buffer loads:
// one buffer resource per array and a 32-bit byte offset per lane, instead
// of a 64-bit address per lane and load (the gathers' address arithmetic was
// 68 of the kernel's ~400 VALU instructions per cell).  Arrays below 2 GiB.
__device__ inline __amdgpu_buffer_rsrc_t adv_rsrc(const void* p)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ inline double adv_ld(__amdgpu_buffer_rsrc_t r, uint32_t i)
{
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)(i * 8u), 0, 0));
}

template <int WPE>
__global__ void __launch_bounds__(256, WPE) k_ex_advect_faces_buf(AdvPtrs p, double dt, FaceView fc,
                                                             const uint32_t* __restrict__ pos, uint64_t n,
                                                             double* __restrict__ rho_out, uint64_t t0, uint64_t t1)
{
#pragma clang fp contract(off)
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const __amdgpu_buffer_rsrc_t rr = adv_rsrc(p.rho), rl0 = adv_rsrc(p.l[0]), rl1 = adv_rsrc(p.l[1]),
                                 rl2 = adv_rsrc(p.l[2]), rv0 = adv_rsrc(p.v[0]), rv1 = adv_rsrc(p.v[1]),
                                 rv2 = adv_rsrc(p.v[2]), rf = adv_rsrc(p.flux);
    const __amdgpu_buffer_rsrc_t re = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(fc.ell_slot), 0, 0x7fffffff,
                                                                        0x00020000);
    // XCD-contiguous cells: a cell's neighbors one level-row away were loaded
    // into the same XCD's L2 by the blocks just before it
    for (size_t i = (size_t)xcd_block() * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t q = pos ? pos[i] : (uint32_t)i;
        const uint32_t c = q;  // explicit local slots are [0, n_local)
        uint32_t s[6];
#pragma unroll
        for (int k = 0; k < 6; k++)
            s[k] = __builtin_amdgcn_raw_buffer_load_b32(re, (int)((uint32_t)(k * fc.n + q) * 4u), 0, 0);
        const double lc3[3] = {adv_ld(rl0, c), adv_ld(rl1, c), adv_ld(rl2, c)};
        const double vc3[3] = {adv_ld(rv0, c), adv_ld(rv1, c), adv_ld(rv2, c)};
        const double rho_c = adv_ld(rr, c);
        double acc = adv_ld(rf, c);
        // the overflow's row (faces next to finer cells beyond the first per
        // direction) is read with the first loads and its first entry with the
        // gathers, so a refined cell's chain of dependent loads stays three
        // long instead of five
        const bool over = *fc.over != 0;
        uint64_t ob = 0;
        uint32_t oc = 0;
        if (over) {
            ob = fc.o_base[q];
            oc = fc.o_cnt[q];
        }
        uint32_t nb0 = c;
        int dir0 = 1;
        if (oc) {
            nb0 = fc.o_slot[ob];
            dir0 = fc.o_dir[ob];
        }
        const double vol = lc3[0] * lc3[1] * lc3[2];
        // one axis at a time: its two faces' 10 gathers in flight together,
        // then their terms (10 live neighbor values instead of 30: more waves
        // per SIMD to hide the gathers' latency); the terms are added in face
        // order as before.  An axis no lane of the wave has a face on (z of
        // level-0 cells of a one-cell-thick grid) issues no loads.  (All 30
        // gathers in flight at once measured the same at 183k cells and 7 %
        // slower at 2.56 M.)
#pragma unroll
        for (int ax = 0; ax < 3; ax++) {
            if (!__ballot(s[2 * ax] != 0xffffffffu || s[2 * ax + 1] != 0xffffffffu)) continue;
            const __amdgpu_buffer_rsrc_t rv = ax == 0 ? rv0 : ax == 1 ? rv1 : rv2;
            double ln0[2], ln1[2], ln2[2], vn[2], rn[2];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int k = 2 * ax + h;
                const uint32_t nb = s[k] != 0xffffffffu ? s[k] : c;
                ln0[h] = adv_ld(rl0, nb);
                ln1[h] = adv_ld(rl1, nb);
                ln2[h] = adv_ld(rl2, nb);
                vn[h] = adv_ld(rv, nb);
                rn[h] = adv_ld(rr, nb);
            }
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int k = 2 * ax + h;
                if (s[k] != 0xffffffffu)
                    acc += face_term_v(h ? ax + 1 : -(ax + 1), dt, vol, lc3, vc3, rho_c, ln0[h], ln1[h], ln2[h], vn[h],
                                       rn[h]);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (oc) {  // further faces (finer neighbors), in row order after the six above
            // the first four entries' slots, then their gathers, issued
            // together (a cell next to finer cells has up to four in 2-D); the
            // terms are added in row order
            uint32_t nbo[4] = {nb0, c, c, c};
            int dro[4] = {dir0, 1, 1, 1};
#pragma unroll
            for (int j = 1; j < 4; j++)
                if ((uint32_t)j < oc) {
                    nbo[j] = fc.o_slot[ob + j];
                    dro[j] = fc.o_dir[ob + j];
                }
            double to[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int ax = (dro[j] > 0 ? dro[j] : -dro[j]) - 1;
                const double ln0 = adv_ld(rl0, nbo[j]), ln1 = adv_ld(rl1, nbo[j]), ln2 = adv_ld(rl2, nbo[j]);
                const double vn = adv_ld(ax == 0 ? rv0 : ax == 1 ? rv1 : rv2, nbo[j]), rn = adv_ld(rr, nbo[j]);
                to[j] = face_term_v(dro[j], dt, vol, lc3, vc3, rho_c, ln0, ln1, ln2, vn, rn);
            }
#pragma unroll
            for (int j = 0; j < 4; j++)
                if ((uint32_t)j < oc) acc += to[j];
            for (uint64_t e = ob + 4, e1 = ob + oc; e < e1; e++) {
                const uint32_t nb = fc.o_slot[e];
                const int dir = fc.o_dir[e], ax = (dir > 0 ? dir : -dir) - 1;
                const double ln0 = adv_ld(rl0, nb), ln1 = adv_ld(rl1, nb), ln2 = adv_ld(rl2, nb);
                const double vn = adv_ld(ax == 0 ? rv0 : ax == 1 ? rv1 : rv2, nb), rn = adv_ld(rr, nb);
                acc += face_term_v(dir, dt, vol, lc3, vc3, rho_c, ln0, ln1, ln2, vn, rn);
            }
        }
        if (!rho_out) {
            p.flux[c] = acc;
        } else {
            rho_out[c] = rho_c + acc;
            if (adv_ld(rf, c) != 0.0) p.flux[c] = 0.0;
        }
    }
    if (rho_out)
        for (uint64_t s = t0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; s < t1; s += stride) rho_out[s] = p.rho[s];
}

// check_for_adaptation, tests/advection/adapter.hpp:66-103, and the marks of
// :114-118 in one pass.  The reference maximises each face pair's relative
// density difference into both cells (the neighbor's when it is local); the
// face test on the offsets and the difference are symmetric in the pair and
// a face neighbor's row holds the cell too, so every local cell takes the
// maximum over its own row's faces: no atomics, no cleared array, no second
// launch.
__global__ void __launch_bounds__(256) k_adapt_diff(const double* __restrict__ rho, const uint64_t* __restrict__ st_row,
                                                    const uint32_t* __restrict__ st_slot,
                                                    const int32_t* __restrict__ st_off,
                                                    const uint32_t* __restrict__ local_g,
                                                    const uint8_t* __restrict__ level, int M, uint64_t n, double thr,
                                                    double inc, double sens, int8_t* __restrict__ marks,
                                                    double* __restrict__ out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += stride) {
        const uint32_t c = local_g[q];
        const int lv = level[c];
        const int64_t lc = 1ll << (M - lv);
        const double rc = rho[c];
        double m = 0.0;  // max_diff = 0 (:62-64)
        // (rows of a few face entries: the four-wide row walk measured slower here)
        for (uint64_t e = st_row[q]; e < st_row[q + 1]; e++) {
            const uint32_t nb = st_slot[e];
            const int64_t ln = 1ll << (M - level[nb]);
            const int64_t x = st_off[3 * e], y = st_off[3 * e + 1], z = st_off[3 * e + 2];
            const bool face = ((x == lc || x == -ln) && y == 0 && z == 0) || ((y == lc || y == -ln) && x == 0 && z == 0) ||
                              ((z == lc || z == -ln) && x == 0 && y == 0);
            if (!face) continue;
            const double rn = rho[nb];
            const double diff = fabs(rc - rn) / ((rc < rn ? rc : rn) + thr);
            if (diff > m) m = diff;  // a non-positive or NaN diff never raises it
        }
        // adapter.hpp:114-118
        const double refine_diff = (lv + 1) * inc, unrefine_diff = sens * refine_diff;
        marks[q] = m > refine_diff ? 2 : (m >= unrefine_diff ? 1 : 0);
        if (out) out[q] = m;
    }
}

// k_adapt_diff and k_face_build in one walk of the rows (the rows are most
// of both kernels' bytes: 4 + 12 B per entry), when the solver's face lists
// are stale -- after every rebuild of an adaptive run.  Each entry feeds the
// face lists (face_dir: a shared face) and the adaptation maximum (the
// reference's offset test, a subset of those) as the two kernels do.
__global__ void __launch_bounds__(256) k_adapt_faces(const double* __restrict__ rho, const uint64_t* __restrict__ st_row,
                                                     const uint32_t* __restrict__ st_slot,
                                                     const int32_t* __restrict__ st_off,
                                                     const uint32_t* __restrict__ local_g,
                                                     const uint8_t* __restrict__ level, int M, uint64_t n, double thr,
                                                     double inc, double sens, int8_t* __restrict__ marks,
                                                     double* __restrict__ out, uint32_t* __restrict__ ell_slot,
                                                     uint32_t* __restrict__ o_cnt, uint32_t* __restrict__ o_slot,
                                                     int8_t* __restrict__ o_dir, uint32_t* __restrict__ over)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += stride) {
        const uint32_t c = local_g[q];
        const int lv = level[c];
        const int64_t lc = 1ll << (M - lv);
        const double rc = rho[c];
        double m = 0.0;  // max_diff = 0 (:62-64)
        uint32_t used = 0, k = 0;
        const uint64_t base = st_row[q];
        row_walk4(base, st_row[q + 1], st_slot, st_off, [&](uint64_t, uint32_t nb, int32_t x, int32_t y, int32_t z) {
            const int64_t ln = 1ll << (M - level[nb]);
            const int32_t o[3] = {x, y, z};
            const int dir = face_dir(lc, ln, o);
            if (!dir) return;  // the adaptation's faces are face_dir faces too
            const bool aface = ((x == lc || x == -ln) && y == 0 && z == 0) ||
                               ((y == lc || y == -ln) && x == 0 && z == 0) || ((z == lc || z == -ln) && x == 0 && y == 0);
            if (aface) {
                const double rn = rho[nb];
                const double diff = fabs(rc - rn) / ((rc < rn ? rc : rn) + thr);
                if (diff > m) m = diff;
            }
            const int col = 2 * ((dir > 0 ? dir : -dir) - 1) + (dir > 0 ? 1 : 0);
            if (!(used >> col & 1u)) {
                used |= 1u << col;
                ell_slot[col * n + q] = nb;
                return;
            }
            o_slot[base + k] = nb;
            o_dir[base + k] = (int8_t)dir;
            k++;
        });
        for (int col = 0; col < 6; col++)
            if (!(used >> col & 1u)) ell_slot[col * n + q] = 0xffffffffu;
        o_cnt[q] = k;
        if (__ballot(k > 0) && (threadIdx.x & 63) == 0) atomicOr(over, 1u);
        // adapter.hpp:114-118
        const double refine_diff = (lv + 1) * inc, unrefine_diff = sens * refine_diff;
        marks[q] = m > refine_diff ? 2 : (m >= unrefine_diff ? 1 : 0);
        if (out) out[q] = m;
    }
}

// adapter.hpp:109-176 per sibling group.  The reference's loop inserts and
// erases while it walks the local cells; its outcome per group is: refine
// every cell marked 2; if any sibling is marked 2 nothing else; else keep
// (dont_unrefine) the first sibling marked 1 -- later ones find it recorded
// (:144-150) -- and unrefine cells marked 0 only when no sibling is marked 1
// (a keep erases its siblings' unrefines, :155-157).  Level-0 cells are
// never kept or unrefined (:152, :173).  Local positions are in ascending id
// order and siblings are local (same level-0 ancestor), so "first" is the
// smallest position.  Codes: 0 none, 1 refine, 2 dont_unrefine, 3 unrefine.
// The siblings (dccrg_mapping.hpp:450-471: the parent's children, x fastest)
// are looked up in the leaf bitmap / hash directly; a sibling that is not a
// leaf (refined) or not local takes no part.
__global__ void __launch_bounds__(256) k_adapt_codes(ExView v, const uint64_t* __restrict__ leaves,
                                                     const uint32_t* __restrict__ slot_of_g,
                                                     const uint32_t* __restrict__ local_g,
                                                     const int8_t* __restrict__ marks, uint64_t n,
                                                     uint8_t* __restrict__ code)
{
    const MapParams& mp = v.mp;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += stride) {
        const int m = marks[q];
        const uint64_t c = leaves[local_g[q]];
        uint64_t idx[3];
        int l = 0;
        map_indices(mp, c, idx, &l);
        if (l == 0) {
            code[q] = m == 2 ? 1 : 0;
            continue;
        }
        const uint64_t h = (uint64_t)1 << (mp.max_lvl - l);
        uint64_t p[3];
        for (int d = 0; d < 3; d++) p[d] = idx[d] - idx[d] % (2 * h);
        bool g_ref = false, g_keep = false, earlier_keep = false;
        for (int k = 0; k < 8; k++) {
            const uint64_t ci[3] = {p[0] + (k & 1) * h, p[1] + ((k >> 1) & 1) * h, p[2] + ((k >> 2) & 1) * h};
            const int64_t g = ex_find(v, map_cell(mp, ci, l));
            const uint32_t s = g < 0 ? NO_SLOT : slot_of_g[g];
            if (s >= n) continue;  // refined sibling (not a leaf), or not local
            const int ms = marks[s];
            g_ref |= ms == 2;
            g_keep |= ms == 1;
            earlier_keep |= ms == 1 && (uint64_t)s < q;
        }
        code[q] = m == 2 ? 1 : (m == 1 ? ((!g_ref && !earlier_keep) ? 2 : 0) : ((!g_ref && !g_keep) ? 3 : 0));
    }
}

// uniform grids: the face neighbors present in the neighborhood (mask bit
// 2k / 2k+1 = canonical axis k, -1 / +1), addressed in the slab layout
// rho_out: as k_ex_advect_faces (fused step into the other density buffer;
// storage slots outside [soff + lin0, soff + lin0 + n) listed as [t0, t1) and
// [t2, t3) are carried over)
__global__ void __launch_bounds__(256) k_u_advect(UGeom g, AdvPtrs p, double dt, uint32_t mask, uint64_t lin0,
                                                  uint64_t n, double* __restrict__ rho_out, uint64_t t0, uint64_t t1,
                                                  uint64_t t2, uint64_t t3)
{
#pragma clang fp contract(off)
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const uint64_t soff = (uint64_t)(-g.cbase * (int64_t)g.S);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t lin = lin0 + i;
        int64_t a, b, c;
        ug_decompose(g, lin, a, b, c);
        const uint64_t s = lin + soff;
        const double vol = p.l[0][s] * p.l[1][s] * p.l[2][s];
        double acc = p.flux[s];
        for (int k = 0; k < 3; k++)
            for (int sg = 0; sg < 2; sg++) {
                if (!(mask >> (2 * k + sg) & 1)) continue;
                int32_t d[3] = {0, 0, 0};
                d[k] = sg ? 1 : -1;
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
                const int dir = (sg ? 1 : -1) * (g.perm[k] + 1);
                acc += face_term(p, s, ug_slot(g, a2, b2, c2), dir, dt, vol);
            }
        if (!rho_out) {
            p.flux[s] = acc;
        } else {
            rho_out[s] = p.rho[s] + acc;
            if (p.flux[s] != 0.0) p.flux[s] = 0.0;
        }
    }
    if (rho_out) {
        for (uint64_t s = t0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; s < t1; s += stride) rho_out[s] = p.rho[s];
        for (uint64_t s = t2 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; s < t3; s += stride) rho_out[s] = p.rho[s];
    }
}

// apply_fluxes, solve.hpp:283-293
__global__ void __launch_bounds__(256) k_apply_slots(double* __restrict__ rho, double* __restrict__ flux,
                                                     uint64_t s0, uint64_t n, const uint32_t* __restrict__ slots)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t s = slots ? slots[i] : s0 + i;
        rho[s] += flux[s];
        flux[s] = 0;
    }
}

// order-preserving map of doubles onto uint64 for atomicMin
__device__ inline unsigned long long dkey(double x)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__host__ inline double dunkey(unsigned long long k)
{
    const unsigned long long b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    double x;
    memcpy(&x, &b, 8);
    return x;
}

// max_time_step, solve.hpp:302-320 (local part)
__global__ void __launch_bounds__(256) k_max_dt(AdvPtrs p, uint64_t s0, uint64_t n,
                                                const uint32_t* __restrict__ slots,
                                                unsigned long long* __restrict__ out)
{
    __shared__ unsigned long long red[256];
    unsigned long long m = dkey(DBL_MAX);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t s = slots ? slots[i] : s0 + i;
        for (int d = 0; d < 3; d++) {
            const double t = p.l[d][s] / fabs(p.v[d][s]);
            if (isnormal(t)) {
                const unsigned long long k = dkey(t);
                m = k < m ? k : m;
            }
        }
    }
    red[threadIdx.x] = m;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] = min(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMin(out, red[0]);
}

// velocities and lengths of local cells from their ids (tests/advection/
// adapter.hpp:304-314, initialize.hpp:50-58): Cartesian_Geometry get_length
// and get_center (dccrg_cartesian_geometry.hpp:284-364), solve.hpp:336-342
struct GeoParams {
    double start[3], l0[3];
};

__global__ void __launch_bounds__(256) k_advect_geometry(MapParams mp, GeoParams gp, AdvPtrs p, uint64_t n,
                                                         uint64_t first_id, uint64_t s0,
                                                         const uint64_t* __restrict__ leaves,
                                                         const uint32_t* __restrict__ local_g)
{
#pragma clang fp contract(off)
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const double maxs = (double)((uint64_t)1 << mp.max_lvl);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t id = leaves ? leaves[local_g[i]] : first_id + i;
        const uint64_t s = s0 + i;
        uint64_t idx[3];
        int l = 0;
        map_indices(mp, id, idx, &l);
        const double scale = 1.0 / (double)((uint64_t)1 << l);
        double len[3], ctr[3];
        for (int d = 0; d < 3; d++) {
            len[d] = gp.l0[d] * scale;
            ctr[d] = gp.start[d] + (double)idx[d] * gp.l0[d] / maxs + len[d] / 2;
        }
        double* v0 = (double*)p.v[0];
        double* v1 = (double*)p.v[1];
        double* v2 = (double*)p.v[2];
        v0[s] = -ctr[1] + 0.5;
        v1[s] = ctr[0] - 0.5;
        v2[s] = 0;
        ((double*)p.l[0])[s] = len[0];
        ((double*)p.l[1])[s] = len[1];
        ((double*)p.l[2])[s] = len[2];
    }
}

// parents of removed cells: 0, then += child / 8 for each child in
// ascending id order (adapter.hpp:265-300)
int adv_ptrs(const dccrgx_grid* grid, const dccrgx_advect_fields* f, AdvPtrs* p)
{
    DX_CHECK(f, DCCRGX_EINVAL, "null field set");
    const int32_t ids[8] = {f->density, f->flux, f->vx, f->vy, f->vz, f->length_x, f->length_y, f->length_z};
    for (int i = 0; i < 8; i++) {
        DX_CHECK(ids[i] >= 0 && (size_t)ids[i] < grid->fields.size(), DCCRGX_EINVAL, "bad field %d", ids[i]);
        DX_CHECK(grid->fields[ids[i]].elem == 8 && !grid->fields[ids[i]].variable, DCCRGX_EINVAL,
                 "advection fields are f64 (field %d)", ids[i]);
    }
    DX_CHECK(f->density != f->flux, DCCRGX_EINVAL, "density and flux must be distinct fields");
    auto P = [&](int32_t id) { return (double*)grid->fields[id].ptr; };
    p->rho = P(f->density);
    p->flux = P(f->flux);
    p->v[0] = P(f->vx);
    p->v[1] = P(f->vy);
    p->v[2] = P(f->vz);
    p->l[0] = P(f->length_x);
    p->l[1] = P(f->length_y);
    p->l[2] = P(f->length_z);
    for (int i = 2; i < 8; i++) DX_CHECK(ids[i] != f->flux, DCCRGX_EINVAL, "flux aliases an input field");
    return DCCRGX_OK;
}

// face items of a uniform grid's neighborhood, in canonical axes
uint32_t face_mask(const Hood& h)
{
    uint32_t m = 0;
    for (int32_t k = 0; k < h.K; k++) {
        const int32_t* d = &h.of_c[3 * k];
        const int nz = (d[0] != 0) + (d[1] != 0) + (d[2] != 0);
        if (nz != 1) continue;
        for (int ax = 0; ax < 3; ax++) {
            if (d[ax] == -1) m |= 1u << (2 * ax);
            if (d[ax] == 1) m |= 1u << (2 * ax + 1);
        }
    }
    return m;
}

// local storage runs of a uniform grid: [s0, s0 + n)
void uniform_local_run(const dccrgx_grid* grid, uint64_t* s0, uint64_t* n)
{
    const UGeom& u = grid->g;
    *s0 = u.lo + (uint64_t)(-u.cbase * (int64_t)u.S);
    *n = u.hi - u.lo;
}


// the face lists' storage for n local cells of a neighborhood, the overflow
// flag cleared (stream order)
int alloc_faces(const Hood& h, uint64_t n, hipStream_t st, std::shared_ptr<FaceCache>& out)
{
    auto fc = std::make_shared<FaceCache>();
    fc->n = n;
    const size_t m = std::max<uint64_t>(n, 1), cap = std::max<uint64_t>(h.st_cap, 1);
    DX_HIP(dx_malloc(&fc->ell_slot, 6 * m * 4));
    DX_HIP(dx_malloc(&fc->o_cnt, m * 4));
    DX_HIP(dx_malloc(&fc->o_slot, cap * 4));
    DX_HIP(dx_malloc(&fc->o_dir, cap));
    DX_HIP(dx_malloc(&fc->d_over, 4));
    fc->o_base = h.d_st_row;
    const Fill z[1] = {{fc->d_over, 4, 0}};
    DX_TRY(dx_fill_many(z, 1, st));
    out = std::move(fc);
    return DCCRGX_OK;
}

// build the face lists of a neighborhood's local cells (explicit grids):
// one pass, no synchronisation
int build_faces(const dccrgx_grid* grid, Hood& h)
{
    ExRegion R;
    DX_TRY(explicit_region(grid, h, DCCRGX_REGION_ALL, &R));
    hipStream_t st = grid->ctx->compute;
    std::shared_ptr<FaceCache> fc;
    const uint64_t n = R.n;
    DX_TRY(alloc_faces(h, n, st, fc));
    const int M = grid->map.max_lvl;
    if (n)
        hipLaunchKernelGGL(k_face_build, dim3(grid_for(n)), dim3(256), 0, st, h.d_st_row, h.d_st_slot, h.d_st_off,
                           R.local_slot, R.level, M, n, fc->ell_slot, fc->o_cnt, fc->o_slot, fc->o_dir, fc->d_over);
    DX_HIP(hipGetLastError());
    h.faces = fc;  // the lists are written in stream order before the kernels that read them
    return DCCRGX_OK;
}

// the face-flux kernels over a region; rho_out != null: fused step into
// rho_out, and with `tail` the slots no launch of the step writes are
// carried over (the last launch of a step)
int advect_launch(dccrgx_grid* grid, Hood& h, const AdvPtrs& p, double dt, int32_t region, double* rho_out,
                  bool tail)
{
    hipStream_t st = grid->ctx->compute;
    if (!grid->uniform) {
        ExRegion R;
        DX_TRY(explicit_region(grid, h, region, &R));
        const uint64_t t0 = grid->n_local, t1 = tail && rho_out ? grid->n_slots : t0;
        const uint64_t work = std::max<uint64_t>(R.n, t1 - t0);
        if (!work) return DCCRGX_OK;
        if (!h.faces) DX_TRY(build_faces(grid, h));
        const FaceCache& F = *h.faces;
        const FaceView fv{F.n, F.ell_slot, F.o_base, F.o_cnt, F.o_slot, F.o_dir, F.d_over};
        // explicit grids store local cell q in slot q (explicit.hip): no slot loads
        const uint32_t* rpos = region == DCCRGX_REGION_ALL ? (const uint32_t*)nullptr : R.pos;
        if (grid->n_slots < (1ull << 28) && 6 * F.n < (1ull << 29)) {  // buffer loads: byte offsets below 2 GiB
            hipLaunchKernelGGL(k_ex_advect_faces_buf<1>, dim3(grid_for(work)), dim3(256), 0, st, p, dt, fv, rpos, R.n,
                               rho_out, t0, t1);
        } else {
            hipLaunchKernelGGL(k_ex_advect_faces<1>, dim3(grid_for(work)), dim3(256), 0, st, p, dt, fv,
                               (const uint32_t*)nullptr, rpos, R.n, rho_out, t0, t1);
        }
        DX_HIP(hipGetLastError());
        return DCCRGX_OK;
    }
    const UGeom& u = grid->g;
    const uint32_t mask = face_mask(h);
    uint64_t s0 = 0, nloc = 0;
    uniform_local_run(grid, &s0, &nloc);
    int64_t r[2][2];
    region_slices(grid, h, region, r);
    const int64_t S = (int64_t)u.S;
    int last = -1;
    for (int i = 0; i < 2; i++)
        if (r[i][1] > r[i][0]) last = i;
    for (int i = 0; i < 2; i++) {
        uint64_t l0 = 0, l1 = 0;
        if (r[i][1] > r[i][0]) {
            l0 = std::max<int64_t>((r[i][0] + u.cbase) * S, (int64_t)u.lo);
            l1 = std::min<int64_t>((r[i][1] + u.cbase) * S, (int64_t)u.hi);
            if (l1 < l0) l1 = l0;
        }
        const bool t = tail && rho_out && i == (last < 0 ? 0 : last);
        const uint64_t a0 = 0, a1 = t ? s0 : 0, b0 = s0 + nloc, b1 = t ? grid->n_slots : b0;
        const uint64_t work = std::max<uint64_t>(std::max<uint64_t>(l1 - l0, a1 - a0), b1 - b0);
        if (!work || (!mask && !rho_out)) continue;
        // no face items: the step copies density unchanged (flux + 0 terms)
        hipLaunchKernelGGL(k_u_advect, dim3(grid_for(work)), dim3(256), 0, st, u, p, dt, mask, l0, l1 - l0, rho_out,
                           a0, a1, b0, b1);
        DX_HIP(hipGetLastError());
    }
    return DCCRGX_OK;
}

// the other density buffer of a fused step: a spare of the grid that holds
// n_slots doubles, or a new one
int density_spare(dccrgx_grid* grid, double** out, size_t* bytes)
{
    const size_t need = std::max<uint64_t>(grid->n_slots, 1) * 8;
    auto& sp = grid->spare_bufs;
    size_t best = sp.size();
    for (size_t i = 0; i < sp.size(); i++)
        if (sp[i].second >= need && (best == sp.size() || sp[i].second < sp[best].second)) best = i;
    if (best < sp.size() && sp[best].second <= 2 * need) {
        *out = (double*)sp[best].first;
        *bytes = sp[best].second;
        sp.erase(sp.begin() + best);
        return DCCRGX_OK;
    }
    DX_HIP(dx_malloc(out, need));
    *bytes = need;
    return DCCRGX_OK;
}

}  // namespace

FaceCache::~FaceCache()
{
    FreeBatch fb;
    for (void* q : {(void*)ell_slot, (void*)o_cnt, (void*)o_slot, (void*)o_dir, (void*)d_over}) fb.add(q);
}

}  // namespace dccrgx

using namespace dccrgx;

extern "C" {

int dccrgx_advect_fluxes(dccrgx_grid* grid, int32_t hood_id, const dccrgx_advect_fields* f, double dt,
                         int32_t region)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    DX_CHECK(region >= DCCRGX_REGION_ALL && region <= DCCRGX_REGION_OUTER, DCCRGX_EINVAL, "bad region");
    AdvPtrs p;
    DX_TRY(adv_ptrs(grid, f, &p));
    if (!grid->n_local) return DCCRGX_OK;
    return advect_launch(grid, *h, p, dt, region, nullptr, false);
}

int dccrgx_advect_apply(dccrgx_grid* grid, const dccrgx_advect_fields* f)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    DX_TRY(explicit_host_leaves(grid));
    AdvPtrs p;
    DX_TRY(adv_ptrs(grid, f, &p));
    if (!grid->n_local) return DCCRGX_OK;
    hipStream_t st = grid->ctx->compute;
    uint64_t s0 = 0, n = grid->n_local;
    const uint32_t* slots = nullptr;
    if (grid->uniform) uniform_local_run(grid, &s0, &n);
    else {
        // local cell q lives in slot q on explicit grids (explicit.hip)
        s0 = 0;
        n = grid->ex->n_local();
    }
    hipLaunchKernelGGL(k_apply_slots, dim3(grid_for(n)), dim3(256), 0, st, (double*)p.rho, p.flux, s0, n, slots);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

int dccrgx_advect_max_time_step(dccrgx_grid* grid, const dccrgx_advect_fields* f, double* local_min)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid && local_min, DCCRGX_EINVAL, "null argument");
    AdvPtrs p;
    DX_TRY(adv_ptrs(grid, f, &p));
    *local_min = DBL_MAX;
    if (!grid->n_local) return DCCRGX_OK;
    hipStream_t st = grid->ctx->compute;
    uint64_t s0 = 0, n = grid->n_local;
    const uint32_t* slots = nullptr;
    if (grid->uniform) uniform_local_run(grid, &s0, &n);
    else {
        ExRegion R;
        DX_TRY(explicit_region(grid, grid->hoods.begin()->second, DCCRGX_REGION_ALL, &R));
        slots = R.local_slot;
    }
    unsigned long long* d = nullptr;
    DX_HIP(dx_malloc((void**)&d, 8));
    const unsigned long long init = 0xffffffffffffffffull;  // above every key
    DX_TRY(dx_h2d_async(grid->ctx, d, &init, 8, st));
    hipLaunchKernelGGL(k_max_dt, dim3(std::min<unsigned>(grid_for(n), 1024)), dim3(256), 0, st, p, s0, n, slots, d);
    DX_HIP(hipGetLastError());
    unsigned long long k = 0;
    DX_TRY(dx_d2h(grid->ctx, &k, d, 8, st));
    dx_free(d);
    if (k != init) *local_min = dunkey(k);
    return DCCRGX_OK;
}

}  // extern "C"

namespace dccrgx {
namespace {

// device marks (and optionally the max diffs) of every local cell; the
// caller frees *d_marks_out (left on the compute stream, not synchronised)
int adapt_marks_device(dccrgx_grid* grid, int32_t hood_id, const dccrgx_advect_fields* f, double diff_increase,
                       double diff_threshold, double unrefine_sensitivity, int8_t** d_marks_out, double* max_diff_out)
{
    *d_marks_out = nullptr;
    DX_TRY(amr_ensure_explicit(grid));
    const Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    AdvPtrs p;
    DX_TRY(adv_ptrs(grid, f, &p));
    const uint64_t n = grid->n_local;
    if (!n) return DCCRGX_OK;
    ExRegion R;
    DX_TRY(explicit_region(grid, *h, DCCRGX_REGION_ALL, &R));
    hipStream_t st = grid->ctx->compute;
    int8_t* d_marks = nullptr;
    double* d_diff = nullptr;
    DX_HIP(dx_malloc(&d_marks, n));
    if (max_diff_out) DX_HIP(dx_malloc(&d_diff, n * 8));
    if (!h->faces) {  // the solver's face lists are stale: built in the same walk of the rows
        std::shared_ptr<FaceCache> fc;
        DX_TRY(alloc_faces(*h, n, st, fc));
        hipLaunchKernelGGL(k_adapt_faces, dim3(grid_for(n)), dim3(256), 0, st, p.rho, h->d_st_row, h->d_st_slot,
                           h->d_st_off, R.local_slot, R.level, grid->map.max_lvl, n, diff_threshold, diff_increase,
                           unrefine_sensitivity, d_marks, d_diff, fc->ell_slot, fc->o_cnt, fc->o_slot, fc->o_dir,
                           fc->d_over);
        const_cast<Hood*>(h)->faces = fc;  // written in stream order before the solver's kernels
    } else {
        hipLaunchKernelGGL(k_adapt_diff, dim3(grid_for(n)), dim3(256), 0, st, p.rho, h->d_st_row, h->d_st_slot,
                           h->d_st_off, R.local_slot, R.level, grid->map.max_lvl, n, diff_threshold, diff_increase,
                           unrefine_sensitivity, d_marks, d_diff);
    }
    DX_HIP(hipGetLastError());
    if (max_diff_out) DX_TRY(dx_d2h(grid->ctx, max_diff_out, d_diff, n * 8, st));
    dx_free(d_diff);
    *d_marks_out = d_marks;
    return DCCRGX_OK;
}

}  // namespace
}  // namespace dccrgx

extern "C" {

int dccrgx_advect_adapt_marks(dccrgx_grid* grid, int32_t hood_id, const dccrgx_advect_fields* f,
                              double diff_increase, double diff_threshold, double unrefine_sensitivity,
                              int8_t* marks_out, double* max_diff_out)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid && f && (marks_out || !grid->n_local), DCCRGX_EINVAL, "null argument");
    int8_t* d_marks = nullptr;
    DX_TRY(adapt_marks_device(grid, hood_id, f, diff_increase, diff_threshold, unrefine_sensitivity, &d_marks,
                              max_diff_out));
    if (!d_marks) return DCCRGX_OK;
    hipStream_t st = grid->ctx->compute;
    const int e = dx_d2h(grid->ctx, marks_out, d_marks, grid->n_local, st);
    dx_free(d_marks);
    return e;
}

int dccrgx_advect_adaptation_sets(dccrgx_grid* grid, int32_t hood_id, const dccrgx_advect_fields* f,
                                  double diff_increase, double diff_threshold, double unrefine_sensitivity,
                                  uint64_t* to_refine, uint64_t* not_to_unrefine, uint64_t* to_unrefine, size_t cap,
                                  size_t counts[3])
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid && f && counts, DCCRGX_EINVAL, "null argument");
    counts[0] = counts[1] = counts[2] = 0;
    if (grid->map.max_lvl == 0) return DCCRGX_OK;  // adapter.hpp:57-59
    const uint64_t n = grid->n_local;
    DX_CHECK(cap >= n, DCCRGX_ERANGE, "capacity %zu < %llu local cells", cap, (unsigned long long)n);
    DX_CHECK((to_refine && not_to_unrefine && to_unrefine) || !n, DCCRGX_EINVAL, "null output");
    int8_t* d_marks = nullptr;
    PhaseTimer T("adaptation_sets");
    DX_TRY(adapt_marks_device(grid, hood_id, f, diff_increase, diff_threshold, unrefine_sensitivity, &d_marks,
                              nullptr));
    if (!d_marks) return DCCRGX_OK;
    T.lap("marks");
    hipStream_t st = grid->ctx->compute;
    const Explicit* E = grid->ex;
    uint8_t* d_code = nullptr;
    int s = DCCRGX_OK;
    if (dx_malloc(&d_code, n) != hipSuccess) s = set_error(DCCRGX_ENOMEM, "out of device memory for the adaptation sets");
    if (s == DCCRGX_OK) {
        hipLaunchKernelGGL(k_adapt_codes, dim3(grid_for(n)), dim3(256), 0, st, explicit_view(grid),
                           (const uint64_t*)E->d_leaves, (const uint32_t*)E->d_slot_of_g, (const uint32_t*)E->d_local_g, (const int8_t*)d_marks, n,
                           d_code);
        if (hipGetLastError() != hipSuccess) s = set_error(DCCRGX_EHIP, "adaptation sets failed");
        T.lap("codes");
        uint64_t* out[3] = {to_refine, not_to_unrefine, to_unrefine};
        if (s == DCCRGX_OK) s = amr_dev_codes_to_lists(grid, d_code, n, out, counts);
    }
    for (void* q : {(void*)d_marks, (void*)d_code}) dx_free(q);
    T.lap("lists");
    return s;
}

int dccrgx_advect_adapt_requests(dccrgx_grid* grid, int32_t hood_id, const dccrgx_advect_fields* f,
                                 double diff_increase, double diff_threshold, double unrefine_sensitivity,
                                 size_t counts[3])
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid && f && counts, DCCRGX_EINVAL, "null argument");
    counts[0] = counts[1] = counts[2] = 0;
    if (grid->map.max_lvl == 0) return DCCRGX_OK;  // adapter.hpp:57-59, :190-192
    const uint64_t n = grid->n_local;
    int8_t* d_marks = nullptr;
    PhaseTimer T("adapt_requests");
    DX_TRY(adapt_marks_device(grid, hood_id, f, diff_increase, diff_threshold, unrefine_sensitivity, &d_marks,
                              nullptr));
    if (!d_marks) return DCCRGX_OK;
    hipStream_t st = grid->ctx->compute;
    const Explicit* E = grid->ex;
    uint8_t* d_code = nullptr;
    uint64_t* d_lists = nullptr;
    int s = DCCRGX_OK;
    if (ds_malloc(&d_code, n, st) != hipSuccess || ds_malloc(&d_lists, n * 8, st) != hipSuccess)
        s = set_error(DCCRGX_ENOMEM, "out of device memory for the adaptation sets");
    uint64_t* dev[3] = {nullptr, nullptr, nullptr};
    if (s == DCCRGX_OK) {
        hipLaunchKernelGGL(k_adapt_codes, dim3(grid_for(n)), dim3(256), 0, st, explicit_view(grid),
                           (const uint64_t*)E->d_leaves, (const uint32_t*)E->d_slot_of_g,
                           (const uint32_t*)E->d_local_g, (const int8_t*)d_marks, n, d_code);
        if (hipGetLastError() != hipSuccess) s = set_error(DCCRGX_EHIP, "adaptation sets failed");
        if (s == DCCRGX_OK) s = amr_dev_codes_to_device_lists(grid, d_code, n, d_lists, dev, counts);
    }
    T.lap("lists");
    // adapter.hpp:197-213: refine, dont_unrefine, unrefine requests in this
    // order, each a batch over its ascending device list (the calls' outcome)
    const int32_t kinds[3] = {DCCRGX_AMR_REFINE, DCCRGX_AMR_DONT_UNREFINE, DCCRGX_AMR_UNREFINE};
    if (s == DCCRGX_OK) amr_state(grid);
    if (s == DCCRGX_OK && (counts[0] || counts[1] || counts[2])) {
        const uint64_t* dv[3] = {dev[0], dev[1], dev[2]};
        s = amr_dev_requests_many(grid, 3, kinds, nullptr, dv, counts, nullptr);
    }
    T.lap("requests");
    ds_free(d_code, st);
    ds_free(d_lists, st);
    dx_free(d_marks);
    return s;
}

int dccrgx_advect_set_geometry(dccrgx_grid* grid, const dccrgx_advect_fields* f, const double start[3],
                               const double level_0_cell_length[3])
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid && f && start && level_0_cell_length, DCCRGX_EINVAL, "null argument");
    AdvPtrs p;
    DX_TRY(adv_ptrs(grid, f, &p));
    const uint64_t n = grid->n_local;
    if (!n) return DCCRGX_OK;
    GeoParams gp;
    for (int d = 0; d < 3; d++) {
        gp.start[d] = start[d];
        gp.l0[d] = level_0_cell_length[d];
    }
    uint64_t s0 = 0, nn = n;
    if (grid->uniform) uniform_local_run(grid, &s0, &nn);
    hipLaunchKernelGGL(k_advect_geometry, dim3(grid_for(n)), dim3(256), 0, grid->ctx->compute, grid->map, gp, p, n,
                       grid->first_local, s0, grid->uniform ? (const uint64_t*)nullptr : grid->ex->d_leaves,
                       grid->uniform ? (const uint32_t*)nullptr : grid->ex->d_local_g);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

int dccrgx_amr_copy_from_parents(dccrgx_grid* grid, const int32_t* fields, size_t nf)
{
    DX_CHECK(grid && (fields || !nf), DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    DX_NOT_PENDING(grid);
    if (!grid->amr || grid->amr->new_cells.empty()) return DCCRGX_OK;
    return amr_dev_copy_from_parents(grid, fields, nf);
}

int dccrgx_amr_average_children(dccrgx_grid* grid, const int32_t* fields, size_t nf)
{
    DX_CHECK(grid && (fields || !nf), DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    DX_NOT_PENDING(grid);
    if (!grid->amr || grid->amr->removed.empty()) return DCCRGX_OK;
    return amr_dev_average_children(grid, fields, nf);
}

int dccrgx_amr_adapter_data_rules(dccrgx_grid* grid, const int32_t* fields, size_t nf)
{
    DX_CHECK(grid && (fields || !nf), DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    DX_NOT_PENDING(grid);
    if (!grid->amr || (grid->amr->new_cells.empty() && grid->amr->removed.empty())) return DCCRGX_OK;
    return amr_dev_data_rules(grid, fields, nf);
}

int dccrgx_advect_step(dccrgx_grid* grid, int32_t hood_id, const dccrgx_advect_fields* f, double dt)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid && f, DCCRGX_EINVAL, "null argument");
    // 2d.cpp:321-390: start density halo, inner fluxes, wait, outer fluxes,
    // apply -- fused: the flux kernels write the new density into the other
    // buffer of a double-buffered density (k_ex_advect_faces), one launch
    // per region, and the buffers swap (the density field's device pointer
    // changes, dccrgx.h)
    const int32_t fd = f->density;
    Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    AdvPtrs p;
    DX_TRY(adv_ptrs(grid, f, &p));
    bool remote = false;
    for (const PeerPlan& pp : h->peers) remote |= !pp.send_ids.empty() || !pp.recv_ids.empty();
    DX_TRY(dccrgx_halo_start(grid, hood_id, &fd, 1));
    if (!grid->n_local) return dccrgx_halo_wait(grid, hood_id, DCCRGX_WAIT_ALL);
    double* out = nullptr;
    size_t out_bytes = 0;
    int s = density_spare(grid, &out, &out_bytes);
    if (s != DCCRGX_OK) {
        dccrgx_halo_wait(grid, hood_id, DCCRGX_WAIT_ALL);
        return s;
    }
    if (!remote) {  // nothing to overlap: one launch over every local cell
        s = dccrgx_halo_wait(grid, hood_id, DCCRGX_WAIT_ALL);
        if (s == DCCRGX_OK) s = advect_launch(grid, *h, p, dt, DCCRGX_REGION_ALL, out, true);
    } else {
        s = advect_launch(grid, *h, p, dt, DCCRGX_REGION_INNER, out, false);
        const int w = dccrgx_halo_wait(grid, hood_id, DCCRGX_WAIT_ALL);
        if (s == DCCRGX_OK) s = w;
        if (s == DCCRGX_OK) s = advect_launch(grid, *h, p, dt, DCCRGX_REGION_OUTER, out, true);
    }
    Field& F = grid->fields[fd];
    if (s != DCCRGX_OK) {
        grid->spare_bufs.emplace_back(out, out_bytes);
        return s;
    }
    grid->spare_bufs.emplace_back(F.ptr, F.cap_bytes ? F.cap_bytes : std::max<uint64_t>(grid->n_slots, 1) * 8);
    F.ptr = out;
    F.cap_bytes = out_bytes == std::max<uint64_t>(grid->n_slots, 1) * 8 ? 0 : out_bytes;
    return DCCRGX_OK;
}

}  // extern "C"
