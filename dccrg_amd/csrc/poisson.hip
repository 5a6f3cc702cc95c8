// poisson.hip -- the BiCG Poisson solver of tests/poisson/poisson_solve.hpp
// on the device.
//
// cache_system_info (:827-971) is built with device kernels over the face
// graph (face.hpp): per local cell the kept face neighbors as (slot, code)
// CSR, then the geometric factors of set_scaling_factor (:704-821).  The
// iteration (:251-522) is device-resident: all scalars (r0.r1, p1.Ap0,
// alpha, beta, residual, its minimum, iteration count) live in a device
// state block, reductions are two-level (block partials, then one block in
// a fixed order: deterministic run to run), and every kernel first checks a
// `done` flag, so the host launches batches of iterations and only polls the
// flag between batches.  Across ranks: the remote-neighbor halo (p0, p1) and
// ncclAllReduce of each scalar, the MPI_Allreduce of :349/:426/:486.
//
// Per-cell state is SoA f64 fields of the grid (Poisson_Cell members,
// :44-83), so the halos move exactly the reference's transfer_switch sets:
// SOLVING = p0, p1; GEOMETRY = scaling factor + 6 factors; INIT = solution;
// TYPE = cell type (:94-131).
#include <cfloat>
#include <cmath>
#include <unordered_map>
#include <vector>

#include "face.hpp"

#include "grid.hpp"

namespace dccrgx {
int explicit_face_neighbors(const dccrgx_grid* grid, const uint64_t* cells, size_t n, uint64_t* row,
                            uint64_t* ids, int32_t* dirs, size_t cap, hipStream_t st);
int explicit_slots_of(const dccrgx_grid* grid, const uint64_t* ids, size_t n, int64_t* slots, hipStream_t st);
}  // namespace dccrgx

namespace dccrgx {
namespace {

constexpr double SOLVE = 0, BOUNDARY = 1, SKIP = 2;  // poisson_solve.hpp:160-165
constexpr int RB = 256;                               // reduction block
constexpr int RG = 512;                               // reduction grid (partials)

enum { F_TYPE, F_P0, F_P1, F_R0, F_R1, F_ADP0, F_BEST, F_SF, F_FXP, F_FXN, F_FYP, F_FYN, F_FZP, F_FZN, F_N };

struct PState {
    double dot_r, dot_p, alpha, beta, residual, residual_min, red;
    double pad_;
    uint32_t iteration, done, save, halt, end, pad2_;
};

struct PPtrs {
    const double* type;
    const double* rhs;
    double* sol;
    double* p0;
    double* p1;
    double* r0;
    double* r1;
    double* adp0;
    double* best;
    double* sf;
    double* f[6];  // f_x_pos, f_x_neg, f_y_pos, f_y_neg, f_z_pos, f_z_neg
    const double* len[3];
};

struct PSys {
    uint64_t n;                  // cell_info entries
    const uint64_t* slot;        // storage slot of each
    const uint64_t* row;         // CSR over kept face neighbors
    const uint64_t* nb;          // neighbor slot
    const int32_t* code;         // (dir + 3) | ((rel + 1) << 4)
};

__device__ __forceinline__ int fidx(int dir) { return dir > 0 ? 2 * (dir - 1) : 2 * (-dir - 1) + 1; }

__device__ __forceinline__ double pw(double x, double p) { return p == 2.0 ? x * x : pow(x, p); }

__device__ __forceinline__ void block_partial(double v, double* part)
{
    __shared__ double red[RB];
    red[threadIdx.x] = v;
    __syncthreads();
    for (int w = RB / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// ---- cache_system_info ------------------------------------------------------

// uniform grids: the face graph neighbors (-x, +x, -y, +y, -z, +z of the
// original axes) as slots of the slab layout; count 0..6 per local cell
__global__ void __launch_bounds__(256) k_u_faces(UGeom g, uint64_t lin0, uint64_t n, uint64_t* __restrict__ nb6,
                                                 int32_t* __restrict__ dir6, uint32_t* __restrict__ cnt)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        int64_t a, b, c;
        ug_decompose(g, lin0 + i, a, b, c);
        uint32_t k = 0;
        for (int d = 0; d < 3; d++) {
            int ax = 0;  // canonical axis of original axis d
            for (int q = 0; q < 3; q++)
                if (g.perm[q] == d) ax = q;
            for (int sg = 0; sg < 2; sg++) {
                int32_t dd[3] = {0, 0, 0};
                dd[ax] = sg ? 1 : -1;
                int64_t a2 = a + dd[0], b2 = b + dd[1], c2 = c + dd[2];
                if (a2 < 0 || a2 >= (int64_t)g.LA) {
                    if (!g.perA) continue;
                    a2 = ug_wrap(a2, (int64_t)g.LA);
                }
                if (b2 < 0 || b2 >= (int64_t)g.LB) {
                    if (!g.perB) continue;
                    b2 = ug_wrap(b2, (int64_t)g.LB);
                }
                if ((c2 < 0 || c2 >= (int64_t)g.LC) && !g.perC) continue;
                nb6[6 * i + k] = ug_slot(g, a2, b2, c2);
                dir6[6 * i + k] = sg ? d + 1 : -(d + 1);
                k++;
            }
        }
        cnt[i] = k;
    }
}

// keep rule of :920-937; pass 1 counts, pass 2 writes at row[i]
__global__ void __launch_bounds__(256) k_filter(const double* __restrict__ type, const uint64_t* __restrict__ cslot,
                                                const uint64_t* __restrict__ frow, const uint64_t* __restrict__ fnb,
                                                const int32_t* __restrict__ fdir, const int8_t* __restrict__ frel,
                                                uint64_t n, uint32_t* __restrict__ cnt,
                                                const uint64_t* __restrict__ row, uint64_t* __restrict__ nb,
                                                int32_t* __restrict__ code)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const double tc = type[cslot[i]];
        uint32_t k = 0;
        if (tc != SKIP)
            for (uint64_t e = frow[i]; e < frow[i + 1]; e++) {
                const double tn = type[fnb[e]];
                if (tn == SKIP || (tc == BOUNDARY && tn == BOUNDARY)) continue;
                if (row) {
                    nb[row[i] + k] = fnb[e];
                    code[row[i] + k] = (fdir[e] + 3) | ((frel[e] + 1) << 4);
                }
                k++;
            }
        if (cnt) cnt[i] = k;
    }
}

// set_scaling_factor, :704-821
__global__ void __launch_bounds__(256) k_scaling(PPtrs p, PSys s)
{
#pragma clang fp contract(off)
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < s.n; i += stride) {
        const uint64_t c = s.slot[i];
        const double hx = p.len[0][c] / 2.0, hy = p.len[1][c] / 2.0, hz = p.len[2][c] / 2.0;
        double off[6] = {+2 * hx, -2 * hx, +2 * hy, -2 * hy, +2 * hz, -2 * hz};  // pos/neg per axis
        const double h[3] = {hx, hy, hz};
        for (uint64_t e = s.row[i]; e < s.row[i + 1]; e++) {
            const int dir = (s.code[e] & 15) - 3;
            const int ax = (dir > 0 ? dir : -dir) - 1;
            const double nh = p.len[ax][s.nb[e]] / 2.0;
            if (dir > 0) off[2 * ax] = h[ax] + nh;
            else off[2 * ax + 1] = -1.0 * (h[ax] + nh);
        }
        const double tot[3] = {off[0] - off[1], off[2] - off[3], off[4] - off[5]};
        double f[6] = {0, 0, 0, 0, 0, 0};
        for (uint64_t e = s.row[i]; e < s.row[i + 1]; e++) {
            const int dir = (s.code[e] & 15) - 3;
            const int ax = (dir > 0 ? dir : -dir) - 1;
            if (dir > 0) f[2 * ax] = +2.0 / (off[2 * ax] * tot[ax]);
            else f[2 * ax + 1] = -2.0 / (off[2 * ax + 1] * tot[ax]);
        }
        for (int k = 0; k < 6; k++) p.f[k][c] = f[k];
        p.sf[c] = -f[0] - f[1] - f[2] - f[3] - f[4] - f[5];
    }
}

// ---- solve -------------------------------------------------------------------

// initialize_solver, :976-1056: r0 = rhs - A . solution, p0 = p1 = r1 = r0;
// partial of r0 . r1
__global__ void __launch_bounds__(RB) k_init(PPtrs p, PSys s, double* __restrict__ part)
{
#pragma clang fp contract(off)
    double acc = 0;
    for (size_t i = (size_t)blockIdx.x * RB + threadIdx.x; i < s.n; i += (size_t)gridDim.x * RB) {
        const uint64_t c = s.slot[i];
        if (p.type[c] != SOLVE) continue;
        double r = p.rhs[c] - p.sf[c] * p.sol[c];
        for (uint64_t e = s.row[i]; e < s.row[i + 1]; e++) {
            const int code = s.code[e];
            const int dir = (code & 15) - 3;
            double m = p.f[fidx(dir)][c];
            if ((code >> 4) - 1 > 0) m /= 4.0;
            r -= m * p.sol[s.nb[e]];
        }
        p.r0[c] = r;
        p.p0[c] = r;
        p.p1[c] = r;
        p.r1[c] = r;
        acc += r * r;
    }
    block_partial(acc, part);
}

// A . p0 cached in A_dot_p0 (:283-335); partial of p1 . (A . p0) (:338-345)
__global__ void __launch_bounds__(RB) k_adp0(PPtrs p, PSys s, const PState* __restrict__ S, double* __restrict__ part)
{
#pragma clang fp contract(off)
    if (S->done || S->end) return;
    double acc = 0;
    for (size_t i = (size_t)blockIdx.x * RB + threadIdx.x; i < s.n; i += (size_t)gridDim.x * RB) {
        const uint64_t c = s.slot[i];
        if (p.type[c] != SOLVE) continue;
        double a = p.sf[c] * p.p0[c];
        for (uint64_t e = s.row[i]; e < s.row[i + 1]; e++) {
            const int code = s.code[e];
            double m = p.f[fidx((code & 15) - 3)][c];
            if ((code >> 4) - 1 > 0) m /= 4.0;
            a += m * p.p0[s.nb[e]];
        }
        p.adp0[c] = a;
        acc += p.p1[c] * a;
    }
    block_partial(acc, part);
}

// solution += alpha p0 (:363-368); partial of |r0|^p over all cell_info
// cells (get_residual, :684-697, before r0 is updated)
__global__ void __launch_bounds__(RB) k_sol_res(PPtrs p, PSys s, const PState* __restrict__ S, double pnorm,
                                                double* __restrict__ part)
{
#pragma clang fp contract(off)
    if (S->done) return;
    const double alpha = S->alpha;
    double acc = 0;
    for (size_t i = (size_t)blockIdx.x * RB + threadIdx.x; i < s.n; i += (size_t)gridDim.x * RB) {
        const uint64_t c = s.slot[i];
        if (p.type[c] == SOLVE) p.sol[c] += alpha * p.p0[c];
        acc += pw(fabs(p.r0[c]), pnorm);
    }
    block_partial(acc, part);
}

// best_solution (:378-389); r0 -= alpha A.p0 (:407-412); r1 -= alpha A^T.p1
// with the neighbors' reversed factors (:415-475); partial of r0 . r1
__global__ void __launch_bounds__(RB) k_r(PPtrs p, PSys s, const PState* __restrict__ S, double* __restrict__ part)
{
#pragma clang fp contract(off)
    if (S->done) return;
    const bool save = S->save, halt = S->halt;
    const double alpha = S->alpha;
    double acc = 0;
    for (size_t i = (size_t)blockIdx.x * RB + threadIdx.x; i < s.n; i += (size_t)gridDim.x * RB) {
        const uint64_t c = s.slot[i];
        if (p.type[c] != SOLVE) continue;
        if (save) p.best[c] = p.sol[c];
        if (halt) continue;
        const double r0 = p.r0[c] - alpha * p.adp0[c];
        double a = p.sf[c] * p.p1[c];
        for (uint64_t e = s.row[i]; e < s.row[i + 1]; e++) {
            const int code = s.code[e];
            const uint64_t nb = s.nb[e];
            double m = p.f[fidx(-((code & 15) - 3))][nb];
            if ((code >> 4) - 1 > 0) m /= 4.0;
            a += m * p.p1[nb];
        }
        const double r1 = p.r1[c] - alpha * a;
        p.r0[c] = r0;
        p.r1[c] = r1;
        acc += r0 * r1;
    }
    block_partial(acc, part);
}

// p0 = r0 + beta p0, p1 = r1 + beta p1 (:506-514)
__global__ void __launch_bounds__(RB) k_p(PPtrs p, PSys s, const PState* __restrict__ S)
{
#pragma clang fp contract(off)
    if (S->done) return;
    const double beta = S->beta;
    for (size_t i = (size_t)blockIdx.x * RB + threadIdx.x; i < s.n; i += (size_t)gridDim.x * RB) {
        const uint64_t c = s.slot[i];
        if (p.type[c] != SOLVE) continue;
        p.p0[c] = p.r0[c] + beta * p.p0[c];
        p.p1[c] = p.r1[c] + beta * p.p1[c];
    }
}

// solution = best_solution (:516-521)
__global__ void __launch_bounds__(RB) k_final(PPtrs p, PSys s)
{
    for (size_t i = (size_t)blockIdx.x * RB + threadIdx.x; i < s.n; i += (size_t)gridDim.x * RB) {
        const uint64_t c = s.slot[i];
        if (p.type[c] == SOLVE) p.sol[c] = p.best[c];
    }
}

enum Phase { PH_INIT, PH_ALPHA, PH_RES, PH_BETA, PH_NONE };

// scalar control of one phase (one thread)
__device__ void control(PState* S, int phase, double v, double pnorm, double stop_residual, double increase,
                        uint32_t min_it, uint32_t max_it)
{
    switch (phase) {
    case PH_INIT:
        S->dot_r = v;
        S->residual_min = DBL_MAX;
        S->iteration = 0;
        S->done = S->save = S->halt = S->end = 0;
        break;
    case PH_ALPHA:  // :265-360
        if (S->done) return;
        if (S->end) {
            S->done = 1;
            return;
        }
        S->iteration++;
        S->dot_p = v;
        if (v == 0) {
            S->done = 1;
            return;
        }
        S->alpha = S->dot_r / v;
        break;
    case PH_RES: {  // :370-404
        if (S->done) return;
        const double r = pnorm == 2.0 ? sqrt(v) : pow(v, 1.0 / pnorm);
        S->residual = r;
        S->save = S->residual_min > r;
        if (S->save) S->residual_min = r;
        S->halt = (r <= stop_residual && S->iteration >= min_it) ||
                  (r >= increase * S->residual_min && S->iteration >= min_it);
        break;
    }
    case PH_BETA:  // :477-504, then the loop condition
        if (S->done) return;
        if (S->halt || S->dot_r == 0) {
            S->done = 1;
            return;
        }
        S->beta = v / S->dot_r;
        S->dot_r = v;
        S->end = S->iteration >= max_it;
        break;
    default: break;
    }
}

// partials -> S->red in a fixed order; optionally run the phase control
__global__ void __launch_bounds__(RB) k_finalize(const double* __restrict__ part, int n, PState* S, int phase,
                                                 double pnorm, double stop_residual, double increase,
                                                 uint32_t min_it, uint32_t max_it)
{
    __shared__ double red[RB];
    double a = 0;
    for (int i = threadIdx.x; i < n; i += RB) a += part[i];
    red[threadIdx.x] = a;
    __syncthreads();
    for (int w = RB / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        S->red = red[0];
        if (phase != PH_NONE) control(S, phase, red[0], pnorm, stop_residual, increase, min_it, max_it);
    }
}

__global__ void k_control(PState* S, int phase, double pnorm, double stop_residual, double increase, uint32_t min_it,
                          uint32_t max_it)
{
    control(S, phase, S->red, pnorm, stop_residual, increase, min_it, max_it);
}

// One workgroup runs the whole iteration loop (one rank, no periodic self
// copies, small systems): the same per-cell arithmetic and control as the
// multi-kernel path, block-wide reductions, no launch per phase.
constexpr int SB = 1024;

__device__ double solo_sum(double v, double* red)
{
    red[threadIdx.x] = v;
    __syncthreads();
    for (int w = SB / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
}

__global__ void __launch_bounds__(SB) k_solo(PPtrs p, PSys s, PState* S, double pnorm, double stop_residual,
                                            double increase, uint32_t min_it, uint32_t max_it)
{
#pragma clang fp contract(off)
    __shared__ double red[SB];
    __shared__ PState T;
    if (threadIdx.x == 0) T = *S;
    __syncthreads();
    for (;;) {
        // A . p0 and p1 . (A . p0)
        double acc = 0;
        for (uint64_t i = threadIdx.x; i < s.n; i += SB) {
            const uint64_t c = s.slot[i];
            if (p.type[c] != SOLVE) continue;
            double a = p.sf[c] * p.p0[c];
            for (uint64_t e = s.row[i]; e < s.row[i + 1]; e++) {
                const int code = s.code[e];
                double m = p.f[fidx((code & 15) - 3)][c];
                if ((code >> 4) - 1 > 0) m /= 4.0;
                a += m * p.p0[s.nb[e]];
            }
            p.adp0[c] = a;
            acc += p.p1[c] * a;
        }
        double v = solo_sum(acc, red);
        if (threadIdx.x == 0) control(&T, PH_ALPHA, v, pnorm, stop_residual, increase, min_it, max_it);
        __syncthreads();
        if (T.done) break;
        // solution update and |r0|^p
        acc = 0;
        for (uint64_t i = threadIdx.x; i < s.n; i += SB) {
            const uint64_t c = s.slot[i];
            if (p.type[c] == SOLVE) p.sol[c] += T.alpha * p.p0[c];
            acc += pw(fabs(p.r0[c]), pnorm);
        }
        v = solo_sum(acc, red);
        if (threadIdx.x == 0) control(&T, PH_RES, v, pnorm, stop_residual, increase, min_it, max_it);
        __syncthreads();
        // best solution, r0 and r1, r0 . r1
        acc = 0;
        for (uint64_t i = threadIdx.x; i < s.n; i += SB) {
            const uint64_t c = s.slot[i];
            if (p.type[c] != SOLVE) continue;
            if (T.save) p.best[c] = p.sol[c];
            if (T.halt) continue;
            const double r0 = p.r0[c] - T.alpha * p.adp0[c];
            double a = p.sf[c] * p.p1[c];
            for (uint64_t e = s.row[i]; e < s.row[i + 1]; e++) {
                const int code = s.code[e];
                const uint64_t nb = s.nb[e];
                double m = p.f[fidx(-((code & 15) - 3))][nb];
                if ((code >> 4) - 1 > 0) m /= 4.0;
                a += m * p.p1[nb];
            }
            const double r1 = p.r1[c] - T.alpha * a;
            p.r0[c] = r0;
            p.r1[c] = r1;
            acc += r0 * r1;
        }
        v = solo_sum(acc, red);
        if (threadIdx.x == 0) control(&T, PH_BETA, v, pnorm, stop_residual, increase, min_it, max_it);
        __syncthreads();
        if (T.done) break;
        for (uint64_t i = threadIdx.x; i < s.n; i += SB) {
            const uint64_t c = s.slot[i];
            if (p.type[c] != SOLVE) continue;
            p.p0[c] = p.r0[c] + T.beta * p.p0[c];
            p.p1[c] = p.r1[c] + T.beta * p.p1[c];
        }
        __syncthreads();  // p0, p1 of neighbors are read by the next A . p0
        if (T.end) {
            if (threadIdx.x == 0) T.done = 1;
            break;
        }
    }
    if (threadIdx.x == 0) *S = T;
}

// Small systems (at most SL info cells, one rank): one thread per cell for
// the whole solve, the cell's vectors in registers and the two searched
// directions p0 / p1 in LDS, so A.p0 and A^T.p1 gather from LDS instead of
// global memory.  The first EK face-neighbor entries of a cell live in
// registers with their factors (m of A.p0, the neighbor's reversed factor of
// A^T.p1, each /4 for a finer neighbor, computed once as the per-iteration
// code computes them); a neighbor outside the info cells never changes during
// the solve, so its product with the factor is kept instead.  Further entries
// (at most OVCAP over all cells) sit in LDS the same way.  Sums are per wave (shuffles) then
// over the 16 waves in a fixed order; every thread runs the scalar control on
// its own copy of the state, so no broadcast is needed.  Same arithmetic per
// cell as k_solo; only the summation order of the dot products differs.
// The 2-norm residual only (the reference's default p_of_norm; pow() would
// push the kernel past its registers).
constexpr int SL = 1024;
constexpr int EK = 6;
constexpr int OVCAP = 1024;  // face-neighbor entries beyond EK per cell, all cells together, kept in LDS

// One barrier per sum: successive calls alternate between the two halves of
// ws, so a half is rewritten only after every thread has passed the barrier
// of the call in between (and so has read it).
__device__ __forceinline__ double wg_sum(double v, double* ws, int& par)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    double* w = ws + par * (SL / 64);
    par ^= 1;
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = 0;
#pragma unroll
    for (int k = 0; k < SL / 64; k++) r += w[k];
    return r;
}

__global__ void __launch_bounds__(SL) k_solo_lds(PPtrs p, PSys s, const int32_t* __restrict__ ej, PState* S,
                                                double stop_residual, double increase, uint32_t min_it,
                                                uint32_t max_it)
{
#pragma clang fp contract(off)
    __shared__ double lp0[SL], lp1[SL], ws[2 * SL / 64];
    __shared__ double oma[OVCAP], omt[OVCAP];
    __shared__ int32_t oj[OVCAP];
    __shared__ uint32_t wtot[SL / 64];
    int par = 0;
    const uint32_t i = threadIdx.x;
    const bool have = i < s.n;
    uint64_t c = 0, e0 = 0, e1 = 0;
    bool solve = false;
    double sf = 0, x0 = 0, x1 = 0, r0 = 0, r1 = 0, sol = 0, best = 0, adp = 0;
    int32_t jr[EK];
    double ma[EK], mt[EK];
#pragma unroll
    for (int k = 0; k < EK; k++) {
        jr[k] = -2;  // no entry
        ma[k] = mt[k] = 0;
    }
    if (have) {
        c = s.slot[i];
        solve = p.type[c] == SOLVE;
        sf = p.sf[c];
        x0 = p.p0[c];
        x1 = p.p1[c];
        r0 = p.r0[c];
        r1 = p.r1[c];
        sol = p.sol[c];
        best = p.best[c];
        adp = p.adp0[c];
        e0 = s.row[i];
        e1 = s.row[i + 1];
#pragma unroll
        for (int k = 0; k < EK; k++) {
            const uint64_t e = e0 + k;
            if (e >= e1) continue;
            const int code = s.code[e];
            const int dir = (code & 15) - 3;
            const uint64_t nb = s.nb[e];
            double m = p.f[fidx(dir)][c], m2 = p.f[fidx(-dir)][nb];
            if ((code >> 4) - 1 > 0) {
                m /= 4.0;
                m2 /= 4.0;
            }
            jr[k] = ej[e];
            if (jr[k] >= 0) {
                ma[k] = m;
                mt[k] = m2;
            } else {  // constant neighbor: the products themselves
                ma[k] = m * p.p0[nb];
                mt[k] = m2 * p.p1[nb];
            }
        }
        lp0[i] = x0;
        lp1[i] = x1;
    }
    // entries beyond the first EK of every cell, packed into LDS at this
    // thread's offset (the host launches this kernel only if they fit)
    const uint32_t ov = e1 - e0 > (uint64_t)EK ? (uint32_t)(e1 - e0 - EK) : 0u;
    uint32_t x = ov;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wtot[w] = x;
    __syncthreads();
    uint32_t o0 = x - ov;
    for (int k = 0; k < w; k++) o0 += wtot[k];
    for (uint32_t k = 0; k < ov; k++) {
        const uint64_t e = e0 + EK + k;
        const int code = s.code[e];
        const int dir = (code & 15) - 3;
        const uint64_t nb = s.nb[e];
        double m = p.f[fidx(dir)][c], m2 = p.f[fidx(-dir)][nb];
        if ((code >> 4) - 1 > 0) {
            m /= 4.0;
            m2 /= 4.0;
        }
        const int32_t j = ej[e];
        oj[o0 + k] = j;
        oma[o0 + k] = j >= 0 ? m : m * p.p0[nb];
        omt[o0 + k] = j >= 0 ? m2 : m2 * p.p1[nb];
    }
    __shared__ PState T0;
    if (threadIdx.x == 0) T0 = *S;
    __syncthreads();
    PState T = T0;  // every thread's own copy (a direct load of *S miscompiles at -O2+)
    for (;;) {
        // A . p0 and p1 . (A . p0)
        double acc = 0;
        if (have && solve) {
            double a = sf * x0;
#pragma unroll
            for (int k = 0; k < EK; k++)
                if (jr[k] != -2) a += jr[k] >= 0 ? ma[k] * lp0[jr[k]] : ma[k];
            for (uint32_t k = o0; k < o0 + ov; k++) a += oj[k] >= 0 ? oma[k] * lp0[oj[k]] : oma[k];
            adp = a;
            acc = x1 * a;
        }
        double v = wg_sum(acc, ws, par);
        control(&T, PH_ALPHA, v, 2.0, stop_residual, increase, min_it, max_it);
        if (T.done) break;
        // solution update and |r0|^p over every info cell
        acc = 0;
        if (have) {
            if (solve) sol += T.alpha * x0;
            acc = fabs(r0) * fabs(r0);  // pw(|r0|, 2)
        }
        v = wg_sum(acc, ws, par);
        control(&T, PH_RES, v, 2.0, stop_residual, increase, min_it, max_it);
        // best solution, r0 and r1, r0 . r1
        acc = 0;
        if (have && solve) {
            if (T.save) best = sol;
            if (!T.halt) {
                const double nr0 = r0 - T.alpha * adp;
                double a = sf * x1;
#pragma unroll
                for (int k = 0; k < EK; k++)
                    if (jr[k] != -2) a += jr[k] >= 0 ? mt[k] * lp1[jr[k]] : mt[k];
                for (uint32_t k = o0; k < o0 + ov; k++) a += oj[k] >= 0 ? omt[k] * lp1[oj[k]] : omt[k];
                r1 = r1 - T.alpha * a;
                r0 = nr0;
                acc = r0 * r1;
            }
        }
        v = wg_sum(acc, ws, par);
        control(&T, PH_BETA, v, 2.0, stop_residual, increase, min_it, max_it);
        if (T.done) break;
        if (have && solve) {
            x0 = r0 + T.beta * x0;
            x1 = r1 + T.beta * x1;
            lp0[i] = x0;
            lp1[i] = x1;
        }
        __syncthreads();  // the next A . p0 reads the neighbors' p0
        if (T.end) {
            T.done = 1;
            break;
        }
    }
    if (have && solve) {
        p.sol[c] = sol;
        p.best[c] = best;
        p.p0[c] = x0;
        p.p1[c] = x1;
        p.r0[c] = r0;
        p.r1[c] = r1;
        p.adp0[c] = adp;
    }
    if (threadIdx.x == 0) *S = T;
}

__global__ void __launch_bounds__(256) k_rel(const uint64_t* __restrict__ cells, const uint64_t* __restrict__ row,
                                             const uint64_t* __restrict__ ids, uint64_t n, MapParams mp,
                                             int8_t* __restrict__ rel)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int l = map_level(mp, cells[i]);
        for (uint64_t e = row[i]; e < row[i + 1]; e++) {
            const int nl = map_level(mp, ids[e]);
            rel[e] = nl > l ? 1 : (nl < l ? -1 : 0);
        }
    }
}

__global__ void __launch_bounds__(256) k_u64_from_i64(const int64_t* __restrict__ a, uint64_t n,
                                                      uint64_t* __restrict__ b, int32_t* __restrict__ err)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (a[i] < 0) atomicOr(err, 1);
        b[i] = a[i] < 0 ? 0 : (uint64_t)a[i];
    }
}

unsigned blocks_for(uint64_t n)
{
    uint64_t g = (n + 255) / 256;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, 4096));
}

template <class T>
int dalloc(T** p, size_t n)
{
    *p = nullptr;
    DX_HIP(dx_malloc(p, std::max<size_t>(n, 1) * sizeof(T)));
    return DCCRGX_OK;
}

}  // namespace
}  // namespace dccrgx

using namespace dccrgx;

struct dccrgx_poisson {
    dccrgx_grid* grid = nullptr;
    dccrgx_poisson_params prm{};
    dccrgx_poisson_fields uf{};
    int32_t fid[F_N];
    // cached system
    bool cached = false;
    uint64_t n_info = 0;
    uint64_t *d_slot = nullptr, *d_row = nullptr, *d_nb = nullptr;
    int32_t* d_code = nullptr;
    int32_t* d_ej = nullptr;  // k_solo_lds: info index of each entry's neighbor, -1 outside the info cells
    PState* d_state = nullptr;
    double* d_part = nullptr;

    void free_cache()
    {
        for (void* q : {(void*)d_slot, (void*)d_row, (void*)d_nb, (void*)d_code, (void*)d_ej}) dx_free(q);
        d_slot = d_row = d_nb = nullptr;
        d_code = d_ej = nullptr;
        n_info = 0;
        cached = false;
    }

    PPtrs ptrs() const
    {
        auto F = [&](int32_t id) { return (double*)grid->fields[id].ptr; };
        PPtrs p;
        p.type = F(fid[F_TYPE]);
        p.rhs = F(uf.rhs);
        p.sol = F(uf.solution);
        p.p0 = F(fid[F_P0]);
        p.p1 = F(fid[F_P1]);
        p.r0 = F(fid[F_R0]);
        p.r1 = F(fid[F_R1]);
        p.adp0 = F(fid[F_ADP0]);
        p.best = F(fid[F_BEST]);
        p.sf = F(fid[F_SF]);
        for (int k = 0; k < 6; k++) p.f[k] = F(fid[F_FXP + k]);
        p.len[0] = F(uf.length_x);
        p.len[1] = F(uf.length_y);
        p.len[2] = F(uf.length_z);
        return p;
    }

    PSys sys() const { return PSys{n_info, d_slot, d_row, d_nb, d_code}; }
};

namespace {

int halo(dccrgx_poisson* P, std::initializer_list<int32_t> fields)
{
    std::vector<int32_t> f(fields);
    DX_TRY(dccrgx_halo_start(P->grid, DCCRGX_DEFAULT_NEIGHBORHOOD_ID, f.data(), f.size()));
    return dccrgx_halo_wait(P->grid, DCCRGX_DEFAULT_NEIGHBORHOOD_ID, DCCRGX_WAIT_ALL);
}

// the cross-rank reductions run (several ranks, or the one-GPU test mode
// that drives the multi-rank path through a 1-rank communicator)
bool multi_rank(const Ctx* c) { return c->comm_size > 1 || (c->self_peer && c->has_comm); }

// across ranks: SUM of S->red (MPI_Allreduce in the reference)
int allreduce(dccrgx_poisson* P)
{
    Ctx* c = P->grid->ctx;
    if (!multi_rank(c)) return DCCRGX_OK;
    double* red = &P->d_state->red;
    if (!c->has_comm && c->has_host_tx) {  // host-staged transport (ranks sharing a GPU)
        double v = 0;
        DX_TRY(dx_d2h(c, &v, red, 8, c->compute));
        const int r = c->host_tx.allreduce_f64(c->host_tx.user, &v, 1, 0);
        DX_CHECK(r == 0, DCCRGX_ERCCL, "host transport: allreduce returned %d", r);
        return dx_h2d(c, red, &v, 8, c->compute);
    }
    DX_CHECK(c->has_comm, DCCRGX_ESTATE, "Poisson solve on %d ranks needs the RCCL communicator", c->comm_size);
    DX_RCCL(ncclAllReduce(red, red, 1, ncclFloat64, ncclSum, c->nccl, c->compute));
    return DCCRGX_OK;
}

// reduce partials into S->red and run `phase` (after the cross-rank sum)
int reduce(dccrgx_poisson* P, int phase)
{
    hipStream_t st = P->grid->ctx->compute;
    const dccrgx_poisson_params& q = P->prm;
    const bool multi = multi_rank(P->grid->ctx);
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(RB), 0, st, P->d_part, RG, P->d_state, multi ? (int)PH_NONE : phase,
                       q.p_of_norm, q.stop_residual, q.stop_after_residual_increase, q.min_iterations,
                       q.max_iterations);
    DX_HIP(hipGetLastError());
    if (multi) {
        DX_TRY(allreduce(P));
        hipLaunchKernelGGL(k_control, dim3(1), dim3(1), 0, st, P->d_state, phase, q.p_of_norm, q.stop_residual,
                           q.stop_after_residual_increase, q.min_iterations, q.max_iterations);
        DX_HIP(hipGetLastError());
    }
    return DCCRGX_OK;
}

// cache_system_info, :827-971
int build_cache(dccrgx_poisson* P, const uint64_t* cells, size_t n, const uint64_t* skip, size_t n_skip)
{
    dccrgx_grid* g = P->grid;
    hipStream_t st = g->ctx->compute;
    P->free_cache();
    // local cells (ascending) and their types
    size_t nl = 0;
    std::vector<uint64_t> local(g->n_local);
    DX_TRY(dccrgx_get_cells(g, DCCRGX_DEFAULT_NEIGHBORHOOD_ID, DCCRGX_CELLS_LOCAL, local.data(), local.size(), &nl));
    std::vector<double> type(nl, BOUNDARY);
    auto mark = [&](const uint64_t* ids, size_t k, double t) {
        for (size_t i = 0; i < k; i++) {
            auto it = std::lower_bound(local.begin(), local.end(), ids[i]);
            if (it != local.end() && *it == ids[i]) type[it - local.begin()] = t;
        }
    };
    mark(skip, n_skip, SKIP);
    mark(cells, n, SOLVE);
    DX_TRY(dccrgx_field_write_local(g, P->fid[F_TYPE], type.data(), nl));
    DX_TRY(halo(P, {P->fid[F_TYPE]}));                              // TYPE, :887-888
    DX_TRY(halo(P, {P->uf.length_x, P->uf.length_y, P->uf.length_z}));  // geometry of remote neighbors

    // storage slots of the local cells and their face neighbors
    uint64_t *d_cslot = nullptr, *d_frow = nullptr, *d_fnb = nullptr;
    int32_t* d_fdir = nullptr;
    int8_t* d_frel = nullptr;
    DX_TRY(dalloc(&d_cslot, nl));
    DX_TRY(dalloc(&d_frow, nl + 1));
    std::vector<uint64_t> frow(nl + 1, 0);
    if (g->uniform) {
        const UGeom& u = g->g;
        const uint64_t soff = (uint64_t)(-u.cbase * (int64_t)u.S);
        std::vector<uint64_t> cs(nl);
        for (size_t i = 0; i < nl; i++) cs[i] = u.lo + i + soff;
        DX_HIP(hipMemcpyAsync(d_cslot, cs.data(), nl * 8, hipMemcpyHostToDevice, st));
        uint64_t* d_nb6 = nullptr;
        int32_t* d_dir6 = nullptr;
        uint32_t* d_cnt = nullptr;
        DX_TRY(dalloc(&d_nb6, 6 * nl));
        DX_TRY(dalloc(&d_dir6, 6 * nl));
        DX_TRY(dalloc(&d_cnt, nl));
        if (nl)
            hipLaunchKernelGGL(k_u_faces, dim3(blocks_for(nl)), dim3(256), 0, st, u, u.lo, (uint64_t)nl, d_nb6, d_dir6,
                               d_cnt);
        DX_HIP(hipGetLastError());
        std::vector<uint32_t> cnt(nl);
        std::vector<uint64_t> nb6(6 * nl);
        std::vector<int32_t> dir6(6 * nl);
        if (nl) {
            DX_HIP(hipMemcpyAsync(cnt.data(), d_cnt, nl * 4, hipMemcpyDeviceToHost, st));
            DX_HIP(hipMemcpyAsync(nb6.data(), d_nb6, nl * 48, hipMemcpyDeviceToHost, st));
            DX_HIP(hipMemcpyAsync(dir6.data(), d_dir6, nl * 24, hipMemcpyDeviceToHost, st));
        }
        DX_HIP(hipStreamSynchronize(st));
        std::vector<uint64_t> fnb;
        std::vector<int32_t> fdir;
        for (size_t i = 0; i < nl; i++) {
            for (uint32_t k = 0; k < cnt[i]; k++) {
                fnb.push_back(nb6[6 * i + k]);
                fdir.push_back(dir6[6 * i + k]);
            }
            frow[i + 1] = fnb.size();
        }
        dx_free(d_nb6);
        dx_free(d_dir6);
        dx_free(d_cnt);
        DX_TRY(dalloc(&d_fnb, fnb.size()));
        DX_TRY(dalloc(&d_fdir, fdir.size()));
        DX_TRY(dalloc(&d_frel, fdir.size()));
        if (!fnb.empty()) {
            DX_HIP(hipMemcpyAsync(d_fnb, fnb.data(), fnb.size() * 8, hipMemcpyHostToDevice, st));
            DX_HIP(hipMemcpyAsync(d_fdir, fdir.data(), fdir.size() * 4, hipMemcpyHostToDevice, st));
            DX_HIP(hipMemsetAsync(d_frel, 0, fdir.size(), st));
        }
        DX_HIP(hipMemcpyAsync(d_frow, frow.data(), (nl + 1) * 8, hipMemcpyHostToDevice, st));
        DX_HIP(hipStreamSynchronize(st));
    } else {
        uint64_t* d_cells = nullptr;
        DX_TRY(dalloc(&d_cells, nl));
        if (nl) DX_HIP(hipMemcpyAsync(d_cells, local.data(), nl * 8, hipMemcpyHostToDevice, st));
        DX_TRY(explicit_face_neighbors(g, d_cells, nl, d_frow, nullptr, nullptr, 0, st));
        DX_HIP(hipMemcpyAsync(frow.data(), d_frow, (nl + 1) * 8, hipMemcpyDeviceToHost, st));
        DX_HIP(hipStreamSynchronize(st));
        const uint64_t tot = frow[nl];
        uint64_t* d_fid = nullptr;
        int64_t* d_s = nullptr;
        int32_t* d_err = nullptr;
        DX_TRY(dalloc(&d_fid, tot));
        DX_TRY(dalloc(&d_fdir, tot));
        DX_TRY(dalloc(&d_frel, tot));
        DX_TRY(dalloc(&d_fnb, tot));
        DX_TRY(dalloc(&d_s, std::max<uint64_t>(tot, nl)));
        DX_TRY(dalloc(&d_err, 1));
        DX_HIP(hipMemsetAsync(d_err, 0, 4, st));
        DX_TRY(explicit_face_neighbors(g, d_cells, nl, d_frow, d_fid, d_fdir, tot, st));
        if (nl)
            hipLaunchKernelGGL(k_rel, dim3(blocks_for(nl)), dim3(256), 0, st, d_cells, d_frow, d_fid, (uint64_t)nl,
                               g->map, d_frel);
        DX_TRY(explicit_slots_of(g, d_fid, tot, d_s, st));
        if (tot)
            hipLaunchKernelGGL(k_u64_from_i64, dim3(blocks_for(tot)), dim3(256), 0, st, d_s, tot, d_fnb, d_err);
        DX_TRY(explicit_slots_of(g, d_cells, nl, d_s, st));
        if (nl)
            hipLaunchKernelGGL(k_u64_from_i64, dim3(blocks_for(nl)), dim3(256), 0, st, d_s, (uint64_t)nl, d_cslot,
                               d_err);
        DX_HIP(hipGetLastError());
        int32_t err = 0;
        DX_HIP(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, st));
        DX_HIP(hipStreamSynchronize(st));
        dx_free(d_cells);
        dx_free(d_fid);
        dx_free(d_s);
        dx_free(d_err);
        DX_CHECK(!err, DCCRGX_EINTERNAL, "face neighbor without storage slot");
    }

    // keep rule and cell_info rows (:905-968)
    const double* d_type = (const double*)g->fields[P->fid[F_TYPE]].ptr;
    uint32_t* d_cnt = nullptr;
    DX_TRY(dalloc(&d_cnt, nl));
    if (nl)
        hipLaunchKernelGGL(k_filter, dim3(blocks_for(nl)), dim3(256), 0, st, d_type, d_cslot, d_frow, d_fnb, d_fdir,
                           d_frel, (uint64_t)nl, d_cnt, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                           (int32_t*)nullptr);
    DX_HIP(hipGetLastError());
    std::vector<uint32_t> cnt(nl);
    std::vector<uint64_t> cslot(nl);
    if (nl) {
        DX_HIP(hipMemcpyAsync(cnt.data(), d_cnt, nl * 4, hipMemcpyDeviceToHost, st));
        DX_HIP(hipMemcpyAsync(cslot.data(), d_cslot, nl * 8, hipMemcpyDeviceToHost, st));
    }
    DX_HIP(hipStreamSynchronize(st));
    // cells without kept face neighbors become skip cells (:954-958); the
    // rows of all local cells are written, the info list picks its own
    std::vector<uint64_t> row_all(nl + 1, 0), info_slot, info_row{0};
    bool changed = false;
    for (size_t i = 0; i < nl; i++) {
        row_all[i + 1] = row_all[i] + cnt[i];
        if (type[i] == SKIP) continue;
        if (cnt[i] == 0) {
            type[i] = SKIP;
            changed = true;
            continue;
        }
        info_slot.push_back(cslot[i]);
    }
    uint64_t* d_row_all = nullptr;
    uint64_t* d_nb_all = nullptr;
    int32_t* d_code_all = nullptr;
    DX_TRY(dalloc(&d_row_all, nl + 1));
    DX_TRY(dalloc(&d_nb_all, row_all[nl]));
    DX_TRY(dalloc(&d_code_all, row_all[nl]));
    DX_HIP(hipMemcpyAsync(d_row_all, row_all.data(), (nl + 1) * 8, hipMemcpyHostToDevice, st));
    if (nl)
        hipLaunchKernelGGL(k_filter, dim3(blocks_for(nl)), dim3(256), 0, st, d_type, d_cslot, d_frow, d_fnb, d_fdir,
                           d_frel, (uint64_t)nl, (uint32_t*)nullptr, d_row_all, d_nb_all, d_code_all);
    DX_HIP(hipGetLastError());
    // compact to the info cells (rows of non-info cells are empty anyway
    // except for skip cells, whose count is 0 by the keep rule)
    std::vector<uint64_t> nb_all(row_all[nl]);
    std::vector<int32_t> code_all(row_all[nl]);
    if (row_all[nl]) {
        DX_HIP(hipMemcpyAsync(nb_all.data(), d_nb_all, row_all[nl] * 8, hipMemcpyDeviceToHost, st));
        DX_HIP(hipMemcpyAsync(code_all.data(), d_code_all, row_all[nl] * 4, hipMemcpyDeviceToHost, st));
    }
    DX_HIP(hipStreamSynchronize(st));
    std::vector<uint64_t> nb;
    std::vector<int32_t> code;
    for (size_t i = 0; i < nl; i++) {
        if (type[i] == SKIP) continue;
        for (uint64_t e = row_all[i]; e < row_all[i + 1]; e++) {
            nb.push_back(nb_all[e]);
            code.push_back(code_all[e]);
        }
        info_row.push_back(nb.size());
    }
    for (void* q : {(void*)d_cslot, (void*)d_frow, (void*)d_fnb, (void*)d_fdir, (void*)d_frel, (void*)d_cnt,
                    (void*)d_row_all, (void*)d_nb_all, (void*)d_code_all})
        dx_free(q);
    if (changed) DX_TRY(dccrgx_field_write_local(g, P->fid[F_TYPE], type.data(), nl));

    P->n_info = info_slot.size();
    DX_TRY(dalloc(&P->d_slot, P->n_info));
    DX_TRY(dalloc(&P->d_row, P->n_info + 1));
    DX_TRY(dalloc(&P->d_nb, nb.size()));
    DX_TRY(dalloc(&P->d_code, code.size()));
    if (P->n_info) DX_HIP(hipMemcpyAsync(P->d_slot, info_slot.data(), P->n_info * 8, hipMemcpyHostToDevice, st));
    DX_HIP(hipMemcpyAsync(P->d_row, info_row.data(), info_row.size() * 8, hipMemcpyHostToDevice, st));
    if (!nb.empty()) {
        DX_HIP(hipMemcpyAsync(P->d_nb, nb.data(), nb.size() * 8, hipMemcpyHostToDevice, st));
        DX_HIP(hipMemcpyAsync(P->d_code, code.data(), code.size() * 4, hipMemcpyHostToDevice, st));
    }
    uint64_t overflow = 0;  // entries beyond EK per cell (k_solo_lds keeps them in LDS)
    for (size_t k = 0; k + 1 < info_row.size(); k++)
        overflow += info_row[k + 1] - info_row[k] > (uint64_t)EK ? info_row[k + 1] - info_row[k] - EK : 0;
    if (P->n_info <= (uint64_t)SL && overflow <= (uint64_t)OVCAP) {  // k_solo_lds's neighbor indices
        std::unordered_map<uint64_t, int32_t> info_of;
        for (size_t k = 0; k < info_slot.size(); k++) info_of[info_slot[k]] = (int32_t)k;
        std::vector<int32_t> ej(nb.size());
        for (size_t e = 0; e < nb.size(); e++) {
            auto it = info_of.find(nb[e]);
            ej[e] = it == info_of.end() ? -1 : it->second;
        }
        DX_TRY(dalloc(&P->d_ej, ej.size()));
        if (!ej.empty()) DX_HIP(hipMemcpyAsync(P->d_ej, ej.data(), ej.size() * 4, hipMemcpyHostToDevice, st));
    }
    if (P->n_info)
        hipLaunchKernelGGL(k_scaling, dim3(blocks_for(P->n_info)), dim3(256), 0, st, P->ptrs(), P->sys());
    DX_HIP(hipGetLastError());
    // GEOMETRY, :968-969
    DX_TRY(halo(P, {P->fid[F_SF], P->fid[F_FXP], P->fid[F_FXN], P->fid[F_FYP], P->fid[F_FYN], P->fid[F_FZP],
                    P->fid[F_FZN]}));
    DX_HIP(hipStreamSynchronize(st));
    P->cached = true;
    return DCCRGX_OK;
}

}  // namespace

extern "C" {

int dccrgx_poisson_create(dccrgx_grid* grid, const dccrgx_poisson_params* prm, const dccrgx_poisson_fields* f,
                          dccrgx_poisson** out)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid && f && out, DCCRGX_EINVAL, "null argument");
    const int32_t uf[5] = {f->rhs, f->solution, f->length_x, f->length_y, f->length_z};
    for (int32_t id : uf) {
        DX_CHECK(id >= 0 && (size_t)id < grid->fields.size(), DCCRGX_EINVAL, "bad field %d", id);
        DX_CHECK(grid->fields[id].elem == 8 && !grid->fields[id].variable, DCCRGX_EINVAL,
                 "Poisson fields are f64 (field %d)", id);
    }
    DX_CHECK(f->rhs != f->solution, DCCRGX_EINVAL, "rhs and solution must be distinct fields");
    auto* P = new dccrgx_poisson();
    P->grid = grid;
    P->uf = *f;
    if (prm) P->prm = *prm;
    else P->prm = dccrgx_poisson_params{1000, 0, 1e-15, 2.0, 10.0};  // Poisson_Solve(), :147-155
    int s = DCCRGX_OK;
    for (int k = 0; k < F_N && s == DCCRGX_OK; k++) s = dccrgx_field_create(grid, 8, &P->fid[k]);
    if (s == DCCRGX_OK && dx_malloc(&P->d_state, sizeof(PState)) != hipSuccess) s = DCCRGX_EHIP;
    if (s == DCCRGX_OK && dx_malloc(&P->d_part, RG * sizeof(double)) != hipSuccess) s = DCCRGX_EHIP;
    if (s != DCCRGX_OK) {
        dx_free(P->d_state);
        dx_free(P->d_part);
        delete P;
        return s;
    }
    *out = P;
    return DCCRGX_OK;
}

int dccrgx_poisson_destroy(dccrgx_poisson* P)
{
    if (!P) return DCCRGX_OK;
    P->free_cache();
    dx_free(P->d_state);
    dx_free(P->d_part);
    delete P;
    return DCCRGX_OK;
}

int dccrgx_poisson_field(const dccrgx_poisson* P, int32_t which, int32_t* fid)
{
    DX_CHECK(P && fid && which >= 0 && which < F_N, DCCRGX_EINVAL, "bad argument");
    *fid = P->fid[which];
    return DCCRGX_OK;
}

int dccrgx_poisson_solve(dccrgx_poisson* P, const uint64_t* cells, size_t n, const uint64_t* skip, size_t n_skip,
                         int32_t cache_is_up_to_date, uint32_t* iterations, double* residual_min)
{
    DX_CHECK(P && (cells || !n) && (skip || !n_skip), DCCRGX_EINVAL, "null argument");
    DX_NOT_PENDING(P->grid);
    if (!cache_is_up_to_date || !P->cached) DX_TRY(build_cache(P, cells, n, skip, n_skip));
    hipStream_t st = P->grid->ctx->compute;
    const PPtrs p = P->ptrs();
    const PSys s = P->sys();
    // initialize_solver: INIT halo, r0 = rhs - A x, r0 . r1
    DX_TRY(halo(P, {P->uf.solution}));
    hipLaunchKernelGGL(k_init, dim3(RG), dim3(RB), 0, st, p, s, P->d_part);
    DX_HIP(hipGetLastError());
    DX_TRY(reduce(P, PH_INIT));
    const double pn = P->prm.p_of_norm;
    PState hs{};
    const Hood* dh = find_hood(P->grid, DCCRGX_DEFAULT_NEIGHBORHOOD_ID);
    const bool solo = !multi_rank(P->grid->ctx) && dh && dh->h_self.empty() && P->n_info <= (1u << 16) &&
                      !test_opt(OPT_POISSON_MULTI, 0);
    if (solo) {
        const dccrgx_poisson_params& q = P->prm;
        if (P->d_ej && pn == 2.0 && !test_opt(OPT_POISSON_SOLO_GLOBAL, 0))
            hipLaunchKernelGGL(k_solo_lds, dim3(1), dim3(SL), 0, st, p, s, (const int32_t*)P->d_ej, P->d_state,
                               q.stop_residual, q.stop_after_residual_increase, q.min_iterations, q.max_iterations);
        else
            hipLaunchKernelGGL(k_solo, dim3(1), dim3(SB), 0, st, p, s, P->d_state, pn, q.stop_residual,
                               q.stop_after_residual_increase, q.min_iterations, q.max_iterations);
        DX_HIP(hipGetLastError());
        DX_TRY(dx_d2h(P->grid->ctx, &hs, P->d_state, sizeof(PState), st));
    }
    uint32_t batch = 4;
    for (; !solo;) {
        for (uint32_t k = 0; k < batch; k++) {
            DX_TRY(halo(P, {P->fid[F_P0], P->fid[F_P1]}));  // SOLVING, :279-281
            hipLaunchKernelGGL(k_adp0, dim3(RG), dim3(RB), 0, st, p, s, (const PState*)P->d_state, P->d_part);
            DX_TRY(reduce(P, PH_ALPHA));
            hipLaunchKernelGGL(k_sol_res, dim3(RG), dim3(RB), 0, st, p, s, (const PState*)P->d_state, pn, P->d_part);
            DX_TRY(reduce(P, PH_RES));
            hipLaunchKernelGGL(k_r, dim3(RG), dim3(RB), 0, st, p, s, (const PState*)P->d_state, P->d_part);
            DX_TRY(reduce(P, PH_BETA));
            hipLaunchKernelGGL(k_p, dim3(RG), dim3(RB), 0, st, p, s, (const PState*)P->d_state);
            DX_HIP(hipGetLastError());
        }
        DX_TRY(dx_d2h(P->grid->ctx, &hs, P->d_state, sizeof(PState), st));
        if (hs.done || hs.end) break;
        batch = std::min<uint32_t>(batch * 2, 64);
    }
    hipLaunchKernelGGL(k_final, dim3(RG), dim3(RB), 0, st, p, s);
    DX_HIP(hipGetLastError());
    DX_HIP(hipStreamSynchronize(st));
    if (iterations) *iterations = hs.iteration;
    if (residual_min) *residual_min = hs.residual_min;
    return DCCRGX_OK;
}

}  // extern "C"
