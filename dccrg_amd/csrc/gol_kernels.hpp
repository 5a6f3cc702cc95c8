// gol_kernels.hpp -- the 26-neighbor game-of-life stencil kernels the library
// launches (gol.hip dispatches them; tools/gol_sweep.hip times them against
// the alternative tilings that lost the sweeps).  See gol.hip for the design.
#pragma once
#include "grid.hpp"

namespace dccrgx {

struct GolArgs {
    const uint32_t* in;
    uint32_t* out;
    uint32_t* cnt;
    uint64_t LA, LB, S;
    uint64_t lo, hi;      // local lin range
    int64_t cbase;        // canonical slice of storage slice 0
    int64_t s0, s1;       // storage slices to compute [s0, s1)
    int64_t chunk;        // slices per workgroup
    uint32_t tiles_a, tiles_b;
    int32_t perA, perB;
};

__device__ __forceinline__ uint32_t alive_bit(uint32_t v) { return v != 0u ? 1u : 0u; }

// reference rule, examples/game_of_life.cpp:68-79
__device__ __forceinline__ uint32_t gol_rule(uint32_t count, uint32_t v)
{
    return count == 3u ? 1u : (count == 2u ? v : 0u);
}

// TA x TB tile, NA cells per thread along A (stride 256/ (TB/NB)), NB rows per thread
template <int TA, int TB, int NA, int NB>
__global__ void __launch_bounds__(256) k_gol26(GolArgs g)
{
    constexpr int TXA = TA / NA;           // threads along A
    constexpr int TYB = 256 / TXA;         // threads along B
    static_assert(TYB * NB == TB, "tile shape");
    constexpr int WA = TA + 2, WB = TB + 2;
    constexpr int E = WA * WB;
    constexpr int NL = (E + 255) / 256;    // tile elements loaded per thread
    __shared__ uint32_t tile[2][WB][WA];

    const int t = threadIdx.x;
    const int tx = t % TXA, ty = t / TXA;
    const uint32_t tiles = g.tiles_a * g.tiles_b;
    const uint32_t tile_id = blockIdx.x % tiles;
    const int64_t chunk_id = blockIdx.x / tiles;
    const int64_t a0 = (int64_t)(tile_id % g.tiles_a) * TA;
    const int64_t b0 = (int64_t)(tile_id / g.tiles_a) * TB;
    const int64_t c0 = g.s0 + chunk_id * g.chunk;
    const int64_t c1 = min(g.s1, c0 + g.chunk);
    if (c0 >= c1) return;

    // global element offsets within a plane for this thread's tile loads (-1: zero)
    int64_t goff[NL];
#pragma unroll
    for (int i = 0; i < NL; i++) {
        const int e = t + 256 * i;
        goff[i] = -1;
        if (e < E) {
            const int r = e / WA, q = e - r * WA;
            int64_t a = a0 - 1 + q, b = b0 - 1 + r;
            bool ok = true;
            if (a < 0 || a >= (int64_t)g.LA) {
                if (g.perA) a = ug_wrap(a, (int64_t)g.LA);
                else ok = false;
            }
            if (b < 0 || b >= (int64_t)g.LB) {
                if (g.perB) b = ug_wrap(b, (int64_t)g.LB);
                else ok = false;
            }
            if (ok) goff[i] = a + (int64_t)g.LA * b;
        }
    }
    uint32_t pre[NL];
    auto fetch = [&](int64_t sc) {
        const uint32_t* plane = g.in + (uint64_t)sc * g.S;
#pragma unroll
        for (int i = 0; i < NL; i++) pre[i] = goff[i] >= 0 ? plane[goff[i]] : 0u;
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int i = 0; i < NL; i++) {
            const int e = t + 256 * i;
            if (e < E) (&tile[buf][0][0])[e] = pre[i];
        }
    };
    // 3x3 box sums of the current LDS plane for this thread's cells, and centres
    uint32_t Sx[NB][NA], Vx[NB][NA];
    auto boxsum = [&](int buf) {
#pragma unroll
        for (int i = 0; i < NA; i++) {
            const int q = tx + TXA * i + 1;
            uint32_t hs[NB + 2];
#pragma unroll
            for (int r = 0; r < NB + 2; r++) {
                const int rr = ty * NB + r;
                hs[r] = alive_bit(tile[buf][rr][q - 1]) + alive_bit(tile[buf][rr][q]) +
                        alive_bit(tile[buf][rr][q + 1]);
            }
#pragma unroll
            for (int k = 0; k < NB; k++) {
                Sx[k][i] = hs[k] + hs[k + 1] + hs[k + 2];
                Vx[k][i] = tile[buf][ty * NB + k + 1][q];
            }
        }
    };

    uint32_t Sp[NB][NA], Sc[NB][NA], Vc[NB][NA];
    // prologue: planes c0-1 and c0
    fetch(c0 - 1);
    stash(0);
    fetch(c0);
    __syncthreads();
    boxsum(0);
#pragma unroll
    for (int k = 0; k < NB; k++)
#pragma unroll
        for (int i = 0; i < NA; i++) Sp[k][i] = Sx[k][i];
    stash(1);
    fetch(c0 + 1);
    __syncthreads();
    boxsum(1);
#pragma unroll
    for (int k = 0; k < NB; k++)
#pragma unroll
        for (int i = 0; i < NA; i++) {
            Sc[k][i] = Sx[k][i];
            Vc[k][i] = Vx[k][i];
        }
    int buf = 0;
    for (int64_t c = c0; c < c1; c++) {
        // `pre` holds plane c+1
        stash(buf);
        if (c + 2 <= c1) fetch(c + 2);
        __syncthreads();
        boxsum(buf);
        buf ^= 1;
        const int64_t cg = c + g.cbase;  // canonical slice
#pragma unroll
        for (int k = 0; k < NB; k++) {
            const int64_t b = b0 + ty * NB + k;
#pragma unroll
            for (int i = 0; i < NA; i++) {
                const int64_t a = a0 + tx + TXA * i;
                const uint32_t count = Sp[k][i] + Sc[k][i] + Sx[k][i] - alive_bit(Vc[k][i]);
                if (a < (int64_t)g.LA && b < (int64_t)g.LB) {
                    const uint64_t lin = (uint64_t)a + g.LA * ((uint64_t)b + g.LB * (uint64_t)cg);
                    if (lin >= g.lo && lin < g.hi) {
                        const uint64_t s = (uint64_t)c * g.S + (uint64_t)a + g.LA * (uint64_t)b;
                        g.cnt[s] = count;
                        g.out[s] = gol_rule(count, Vc[k][i]);
                    }
                }
                Sp[k][i] = Sc[k][i];
                Sc[k][i] = Sx[k][i];
                Vc[k][i] = Vx[k][i];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Vectorised 26-neighbor stencil (LA % 4 == 0).  Tile = 256 cells along A x
// NW*RW rows along B; a workgroup is NW waves, wave w owns tile rows
// RW*w..RW*w+RW-1 (the library launches 8 x 4),
// lane l owns cells 4l..4l+3 of each of its rows (one dwordx4 per row per
// plane, loaded once from HBM).  Alive bits of a plane are published to LDS
// packed 4 cells per u32 (one byte each); each lane forms its 3-wide row sums
// with byte-SWAR from its own word and its neighbours' edge bytes, the
// 3x3 plane sums by adding packed rows, and the 27-point sum across the
// planes c-1, c, c+1 held in registers.  Counts <= 27 never carry across
// bytes.  Raw centre values stay in registers for the B3/S23 rule.
// ---------------------------------------------------------------------------
struct Gol4Args {
    const uint32_t* in;
    uint32_t* out;
    uint32_t* cnt;
    uint64_t LA, LB, S;
    uint64_t lo, hi;
    int64_t cbase;
    int64_t s0, s1;
    int64_t chunk;
    uint32_t tiles_a, tiles_b;
    uint32_t nwg;
    int32_t perA, perB;
};

__device__ __forceinline__ uint32_t pack_bits(uint4 v)
{
    return (v.x != 0u ? 1u : 0u) | (v.y != 0u ? 0x100u : 0u) | (v.z != 0u ? 0x10000u : 0u) |
           (v.w != 0u ? 0x1000000u : 0u);
}

// PF: planes in flight (1: the next plane is loaded while the current one is
// computed; 2: two planes ahead, twice the bytes in flight per lane).
// NTL: non-temporal loads for the rows no other tile reads as its apron.
template <int NW, int RW, bool NT = false, int PF = 1, bool NTL = false>
__global__ void __launch_bounds__(64 * NW) k_gol26v(Gol4Args g)
{
    static_assert(PF == 1 || PF == 2, "one or two planes in flight");
    constexpr int TA = 256, TB = NW * RW;
    static_assert(NW >= 2, "apron rows are loaded by the first and last wave");
    __shared__ uint32_t P[2][TB + 2][64];
    __shared__ uint32_t EL[2][TB + 2], ER[2][TB + 2];

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // XCD-aware remap (bijective): workgroups b and b+8 share an XCD; give each
    // XCD a contiguous run of tiles so vertically adjacent tiles (which share
    // apron rows) are served from the same L2.
    const uint32_t bid = blockIdx.x, xcd = bid & 7, q8 = g.nwg >> 3, r8 = g.nwg & 7;
    const uint32_t wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const uint32_t tiles = g.tiles_a * g.tiles_b;
    const uint32_t tile_id = wgid % tiles;
    const int64_t chunk_id = wgid / tiles;
    const int64_t a0 = (int64_t)(tile_id % g.tiles_a) * TA;
    const int64_t b0 = (int64_t)(tile_id / g.tiles_a) * TB;
    const int64_t c0 = g.s0 + chunk_id * g.chunk;
    const int64_t c1 = min(g.s1, c0 + g.chunk);
    if (c0 >= c1) return;

    const int64_t LA = (int64_t)g.LA, LB = (int64_t)g.LB;
    auto wrapA = [&](int64_t a) -> int64_t {  // -1: outside a non-periodic grid
        if (a >= 0 && a < LA) return a;
        return g.perA ? ug_wrap(a, LA) : -1;
    };
    auto wrapB = [&](int64_t b) -> int64_t {
        if (b >= 0 && b < LB) return b;
        return g.perB ? ug_wrap(b, LB) : -1;
    };
    // my vector column and rows (tile rows 1+RW*w+k), plus the apron row of the
    // first / last wave.  In-plane offsets are 32-bit (plane < 2^31 cells) so the
    // loads use a scalar plane base + one VGPR offset; invalid cells (outside a
    // non-periodic grid) load offset 0 and are masked to zero.
    const int64_t av = wrapA(a0 + 4 * lane);
    uint32_t roff[RW + 1], eoff[RW + 1];
    uint32_t rmask = 0, emask = 0;
#pragma unroll
    for (int k = 0; k < RW; k++) {
        const int64_t b = wrapB(b0 + RW * w + k);
        const bool ok = av >= 0 && b >= 0;
        roff[k] = ok ? (uint32_t)(av + LA * b) : 0u;
        rmask |= ok ? (1u << k) : 0u;
    }
    const int xrow = w == 0 ? 0 : (w == NW - 1 ? TB + 1 : -1);  // extra tile row of this wave
    {
        const int64_t b = xrow < 0 ? -1 : wrapB(b0 - 1 + xrow);
        const bool ok = av >= 0 && b >= 0;
        roff[RW] = ok ? (uint32_t)(av + LA * b) : 0u;
        rmask |= ok ? (1u << RW) : 0u;
    }
    // apron columns: lane 0 the left one, lane 63 the right one, for my rows (+ extra row)
    {
        const int64_t ae = lane == 0 ? wrapA(a0 - 1) : (lane == 63 ? wrapA(a0 + TA) : -1);
#pragma unroll
        for (int k = 0; k <= RW; k++) {
            const int64_t b = k < RW ? wrapB(b0 + RW * w + k) : (xrow < 0 ? -1 : wrapB(b0 - 1 + xrow));
            const bool ok = ae >= 0 && b >= 0;
            eoff[k] = ok ? (uint32_t)(ae + LA * b) : 0u;
            emask |= ok ? (1u << k) : 0u;
        }
    }

    uint4 F[RW + 1];       // fetched plane (own rows + extra row)
    uint32_t FE[RW + 1];   // fetched apron scalars
    uint4 F2[RW + 1];      // PF == 2: the plane after
    uint32_t FE2[RW + 1];
    auto fetch_into = [&](int64_t sc, uint4 (&Fd)[RW + 1], uint32_t (&FEd)[RW + 1]) {
        const uint32_t* __restrict__ plane = g.in + (uint64_t)sc * g.S;
#pragma unroll
        for (int k = 0; k <= RW; k++) {
            if (k == RW && xrow < 0) {
                Fd[k] = make_uint4(0, 0, 0, 0);
            } else {
                // tile rows 0 and TB-1 are the neighbouring tiles' aprons
                const bool priv = k < RW && (RW * w + k) != 0 && (RW * w + k) != TB - 1;
                uint4 v;
                if (NTL && priv) {
                    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                    const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(plane + roff[k]));
                    v = make_uint4(x.x, x.y, x.z, x.w);
                } else {
                    v = *reinterpret_cast<const uint4*>(plane + roff[k]);
                }
                Fd[k] = (rmask >> k) & 1u ? v : make_uint4(0, 0, 0, 0);
            }
        }
        if (emask) {
#pragma unroll
            for (int k = 0; k <= RW; k++) FEd[k] = (emask >> k) & 1u ? plane[eoff[k]] : 0u;
        } else {
#pragma unroll
            for (int k = 0; k <= RW; k++) FEd[k] = 0u;
        }
    };
    auto fetch = [&](int64_t sc) { fetch_into(sc, F, FE); };
    auto stash = [&](int buf) {
#pragma unroll
        for (int k = 0; k < RW; k++) P[buf][1 + RW * w + k][lane] = pack_bits(F[k]);
        if (xrow >= 0) P[buf][xrow][lane] = pack_bits(F[RW]);
        if (lane == 0 || lane == 63) {
            uint32_t(*E)[TB + 2] = lane == 0 ? EL : ER;
#pragma unroll
            for (int k = 0; k < RW; k++) E[buf][1 + RW * w + k] = FE[k] != 0u ? 1u : 0u;
            if (xrow >= 0) E[buf][xrow] = FE[RW] != 0u ? 1u : 0u;
        }
    };
    uint32_t Sx[RW], Bx[RW];
    auto plane_sums = [&](int buf) {
        uint32_t h[RW + 2];
        const int ll = lane > 0 ? lane - 1 : 0, lr = lane < 63 ? lane + 1 : 63;
#pragma unroll
        for (int q = 0; q < RW + 2; q++) {
            const int rr = RW * w + q;
            const uint32_t m = P[buf][rr][lane];
            const uint32_t lft = lane > 0 ? (P[buf][rr][ll] >> 24) : EL[buf][rr];
            const uint32_t rgt = lane < 63 ? (P[buf][rr][lr] & 0xffu) : ER[buf][rr];
            h[q] = m + ((m << 8) | lft) + ((m >> 8) | (rgt << 24));
            if (q >= 1 && q <= RW) Bx[q - 1] = m;
        }
#pragma unroll
        for (int k = 0; k < RW; k++) Sx[k] = h[k] + h[k + 1] + h[k + 2];
    };

    uint32_t Sp[RW], Sc[RW], Bc[RW];
    uint4 Vc[RW], Vn[RW];
    fetch(c0 - 1);
    stash(0);
    fetch(c0);
    __syncthreads();
    plane_sums(0);
#pragma unroll
    for (int k = 0; k < RW; k++) Sp[k] = Sx[k];
    stash(1);
#pragma unroll
    for (int k = 0; k < RW; k++) Vc[k] = F[k];
    fetch(c0 + 1);
    if (PF == 2 && c0 + 2 <= c1) fetch_into(c0 + 2, F2, FE2);
    __syncthreads();
    plane_sums(1);
#pragma unroll
    for (int k = 0; k < RW; k++) {
        Sc[k] = Sx[k];
        Bc[k] = Bx[k];
    }
    int buf = 0;
    const uint64_t ua = (uint64_t)(a0 + 4 * lane);
    const bool a_ok = (int64_t)ua < LA;
    for (int64_t c = c0; c < c1; c++) {
        stash(buf);
#pragma unroll
        for (int k = 0; k < RW; k++) Vn[k] = F[k];
        if (PF == 1) {
            if (c + 2 <= c1) fetch(c + 2);
        } else {
#pragma unroll
            for (int k = 0; k <= RW; k++) {
                F[k] = F2[k];
                FE[k] = FE2[k];
            }
            if (c + 3 <= c1) fetch_into(c + 3, F2, FE2);
        }
        __syncthreads();
        plane_sums(buf);
        buf ^= 1;
        // plane c: canonical linear index of its first cell, storage offset
        const uint64_t plin = g.S * (uint64_t)(c + g.cbase);
        const bool full = plin >= g.lo && plin + g.S <= g.hi;  // wave-uniform
        uint32_t* pcnt = g.cnt + (uint64_t)c * g.S;
        uint32_t* pout = g.out + (uint64_t)c * g.S;
#pragma unroll
        for (int k = 0; k < RW; k++) {
            const uint32_t cnt4 = Sp[k] + Sc[k] + Sx[k] - Bc[k];
            const int64_t b = b0 + RW * w + k;
            if (a_ok && b < LB) {
                const uint32_t n0 = cnt4 & 0xffu, n1 = (cnt4 >> 8) & 0xffu, n2 = (cnt4 >> 16) & 0xffu,
                               n3 = cnt4 >> 24;
                const uint4 v = Vc[k];
                const uint4 nc = make_uint4(n0, n1, n2, n3);
                const uint4 nv = make_uint4(gol_rule(n0, v.x), gol_rule(n1, v.y), gol_rule(n2, v.z),
                                            gol_rule(n3, v.w));
                const uint32_t p = (uint32_t)ua + (uint32_t)LA * (uint32_t)b;
                if (full) {
                    if (NT) {
                        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                        const u32x4 xc = {nc.x, nc.y, nc.z, nc.w}, xv = {nv.x, nv.y, nv.z, nv.w};
                        __builtin_nontemporal_store(xc, reinterpret_cast<u32x4*>(pcnt + p));
                        __builtin_nontemporal_store(xv, reinterpret_cast<u32x4*>(pout + p));
                    } else {
                        *reinterpret_cast<uint4*>(pcnt + p) = nc;
                        *reinterpret_cast<uint4*>(pout + p) = nv;
                    }
                } else {
                    const uint32_t ncs[4] = {nc.x, nc.y, nc.z, nc.w}, nvs[4] = {nv.x, nv.y, nv.z, nv.w};
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint64_t lin = plin + p + j;
                        if (lin >= g.lo && lin < g.hi) {
                            pcnt[p + j] = ncs[j];
                            pout[p + j] = nvs[j];
                        }
                    }
                }
            }
            Sp[k] = Sc[k];
            Sc[k] = Sx[k];
            Bc[k] = Bx[k];
            Vc[k] = Vn[k];
        }
    }
}

// Vectorised LB == 1 kernel (2-D grids, LA % 4 == 0): a workgroup owns 256*NW
// cells of a row and marches along C (the y rows); lane = 4 cells (dwordx4),
// packed-byte row sums as in k_gol26v; rows b-1 / b+1 are the row itself
// (periodic B: mult = 3) or absent (mult = 1).
template <int NW, bool NTS = false>
__global__ void __launch_bounds__(64 * NW) k_gol26_rowv(Gol4Args g, uint32_t mult)
{
    constexpr int NT = 64 * NW, TA = 4 * NT;
    __shared__ uint32_t P[2][NT];
    __shared__ uint32_t E[2][2];
    const int t = threadIdx.x;
    const uint32_t bid = blockIdx.x, xcd = bid & 7, q8 = g.nwg >> 3, r8 = g.nwg & 7;
    const uint32_t wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const uint32_t tile_id = wgid % g.tiles_a;
    const int64_t chunk_id = wgid / g.tiles_a;
    const int64_t a0 = (int64_t)tile_id * TA;
    const int64_t c0 = g.s0 + chunk_id * g.chunk;
    const int64_t c1 = min(g.s1, c0 + g.chunk);
    if (c0 >= c1) return;
    const int64_t LA = (int64_t)g.LA;
    auto wrapA = [&](int64_t a) -> int64_t {
        if (a >= 0 && a < LA) return a;
        return g.perA ? ug_wrap(a, LA) : -1;
    };
    const int64_t av = wrapA(a0 + 4 * t);
    const bool vok = av >= 0;
    const uint32_t voff = vok ? (uint32_t)av : 0u;
    const int64_t ae = t == 0 ? wrapA(a0 - 1) : (t == NT - 1 ? wrapA(a0 + TA) : -1);
    const bool eok = ae >= 0;
    const uint32_t eoff = eok ? (uint32_t)ae : 0u;
    uint4 F;
    uint32_t FE;
    auto fetch = [&](int64_t sc) {
        const uint32_t* __restrict__ plane = g.in + (uint64_t)sc * g.S;
        const uint4 v = *reinterpret_cast<const uint4*>(plane + voff);
        F = vok ? v : make_uint4(0, 0, 0, 0);
        FE = eok ? plane[eoff] : 0u;
    };
    auto stash = [&](int buf) {
        P[buf][t] = pack_bits(F);
        if (t == 0) E[buf][0] = FE != 0u ? 1u : 0u;
        if (t == NT - 1) E[buf][1] = FE != 0u ? 1u : 0u;
    };
    uint32_t Sx, Bx;
    auto sums = [&](int buf) {
        const uint32_t m = P[buf][t];
        const uint32_t lft = t > 0 ? (P[buf][t - 1] >> 24) : E[buf][0];
        const uint32_t rgt = t < NT - 1 ? (P[buf][t + 1] & 0xffu) : E[buf][1];
        Sx = mult * (m + ((m << 8) | lft) + ((m >> 8) | (rgt << 24)));
        Bx = m;
    };
    uint32_t Sp, Sc, Bc;
    uint4 Vc, Vn;
    fetch(c0 - 1);
    stash(0);
    fetch(c0);
    __syncthreads();
    sums(0);
    Sp = Sx;
    stash(1);
    Vc = F;
    fetch(c0 + 1);
    __syncthreads();
    sums(1);
    Sc = Sx;
    Bc = Bx;
    int buf = 0;
    const bool a_ok = a0 + 4 * t < LA;
    for (int64_t c = c0; c < c1; c++) {
        stash(buf);
        Vn = F;
        if (c + 2 <= c1) fetch(c + 2);
        __syncthreads();
        sums(buf);
        buf ^= 1;
        const uint32_t cnt4 = Sp + Sc + Sx - Bc;
        if (a_ok) {
            const uint32_t n0 = cnt4 & 0xffu, n1 = (cnt4 >> 8) & 0xffu, n2 = (cnt4 >> 16) & 0xffu, n3 = cnt4 >> 24;
            const uint4 nc = make_uint4(n0, n1, n2, n3);
            const uint4 nv = make_uint4(gol_rule(n0, Vc.x), gol_rule(n1, Vc.y), gol_rule(n2, Vc.z),
                                        gol_rule(n3, Vc.w));
            const uint64_t plin = g.S * (uint64_t)(c + g.cbase);
            const uint32_t p = (uint32_t)(a0 + 4 * t);
            uint32_t* pcnt = g.cnt + (uint64_t)c * g.S;
            uint32_t* pout = g.out + (uint64_t)c * g.S;
            if (plin >= g.lo && plin + g.S <= g.hi) {
                if (NTS) {
                    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                    const u32x4 xc = {nc.x, nc.y, nc.z, nc.w}, xv = {nv.x, nv.y, nv.z, nv.w};
                    __builtin_nontemporal_store(xc, reinterpret_cast<u32x4*>(pcnt + p));
                    __builtin_nontemporal_store(xv, reinterpret_cast<u32x4*>(pout + p));
                } else {
                    *reinterpret_cast<uint4*>(pcnt + p) = nc;
                    *reinterpret_cast<uint4*>(pout + p) = nv;
                }
            } else {
                const uint32_t ncs[4] = {nc.x, nc.y, nc.z, nc.w}, nvs[4] = {nv.x, nv.y, nv.z, nv.w};
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (plin + p + j >= g.lo && plin + p + j < g.hi) {
                        pcnt[p + j] = ncs[j];
                        pout[p + j] = nvs[j];
                    }
            }
        }
        Sp = Sc;
        Sc = Sx;
        Bc = Bx;
        Vc = Vn;
    }
}

// LB == 1 (2-D and 1-D grids): one row per plane; rows b-1 / b+1 are the same
// row (periodic B) or absent.
template <int TA, int NA>
__global__ void __launch_bounds__(256) k_gol26_row(GolArgs g, uint32_t mult)
{
    constexpr int WA = TA + 2;
    constexpr int NL = (WA + 255) / 256;
    __shared__ uint32_t tile[2][WA];
    const int t = threadIdx.x;
    const uint32_t tile_id = blockIdx.x % g.tiles_a;
    const int64_t chunk_id = blockIdx.x / g.tiles_a;
    const int64_t a0 = (int64_t)tile_id * TA;
    const int64_t c0 = g.s0 + chunk_id * g.chunk;
    const int64_t c1 = min(g.s1, c0 + g.chunk);
    if (c0 >= c1) return;
    int64_t goff[NL];
#pragma unroll
    for (int i = 0; i < NL; i++) {
        const int e = t + 256 * i;
        goff[i] = -1;
        if (e < WA) {
            int64_t a = a0 - 1 + e;
            bool ok = true;
            if (a < 0 || a >= (int64_t)g.LA) {
                if (g.perA) a = ug_wrap(a, (int64_t)g.LA);
                else ok = false;
            }
            if (ok) goff[i] = a;
        }
    }
    uint32_t pre[NL];
    auto fetch = [&](int64_t sc) {
        const uint32_t* plane = g.in + (uint64_t)sc * g.S;
#pragma unroll
        for (int i = 0; i < NL; i++) pre[i] = goff[i] >= 0 ? plane[goff[i]] : 0u;
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int i = 0; i < NL; i++) {
            const int e = t + 256 * i;
            if (e < WA) tile[buf][e] = pre[i];
        }
    };
    uint32_t Sx[NA], Vx[NA];
    auto rowsum = [&](int buf) {
#pragma unroll
        for (int i = 0; i < NA; i++) {
            const int q = t + 256 * i + 1;
            Sx[i] = mult * (alive_bit(tile[buf][q - 1]) + alive_bit(tile[buf][q]) +
                            alive_bit(tile[buf][q + 1]));
            Vx[i] = tile[buf][q];
        }
    };
    uint32_t Sp[NA], Sc[NA], Vc[NA];
    fetch(c0 - 1);
    stash(0);
    fetch(c0);
    __syncthreads();
    rowsum(0);
#pragma unroll
    for (int i = 0; i < NA; i++) Sp[i] = Sx[i];
    stash(1);
    fetch(c0 + 1);
    __syncthreads();
    rowsum(1);
#pragma unroll
    for (int i = 0; i < NA; i++) {
        Sc[i] = Sx[i];
        Vc[i] = Vx[i];
    }
    int buf = 0;
    for (int64_t c = c0; c < c1; c++) {
        stash(buf);
        if (c + 2 <= c1) fetch(c + 2);
        __syncthreads();
        rowsum(buf);
        buf ^= 1;
        const int64_t cg = c + g.cbase;
#pragma unroll
        for (int i = 0; i < NA; i++) {
            const int64_t a = a0 + t + 256 * i;
            const uint32_t count = Sp[i] + Sc[i] + Sx[i] - alive_bit(Vc[i]);
            if (a < (int64_t)g.LA) {
                const uint64_t lin = (uint64_t)a + g.LA * (uint64_t)cg;
                if (lin >= g.lo && lin < g.hi) {
                    const uint64_t s = (uint64_t)c * g.S + (uint64_t)a;
                    g.cnt[s] = count;
                    g.out[s] = gol_rule(count, Vc[i]);
                }
            }
            Sp[i] = Sc[i];
            Sc[i] = Sx[i];
            Vc[i] = Vx[i];
        }
    }
}

// slices per workgroup: enough workgroups (`want`) to fill the 256 CUs several
// times over; `forced` > 0 overrides (tests put chunk seams into small grids)
inline int64_t gol_chunk(int64_t nsl, int64_t tiles, int64_t want, int64_t forced)
{
    if (forced > 0) return forced;
    const int64_t chunks = std::max<int64_t>(1, std::min<int64_t>(nsl, (want + tiles - 1) / tiles));
    return (nsl + chunks - 1) / chunks;
}

// launch plan of the vector kernels for a TA x TB tile (cells along A x rows
// along B) over `nsl` slices; nwg == 0 when it does not fit one launch
inline Gol4Args gol4_plan(const GolArgs& a, int TA, int TB, int64_t nsl, int64_t forced_chunk, int64_t want = 8192)
{
    Gol4Args v{};
    v.in = a.in;
    v.out = a.out;
    v.cnt = a.cnt;
    v.LA = a.LA;
    v.LB = a.LB;
    v.S = a.S;
    v.lo = a.lo;
    v.hi = a.hi;
    v.cbase = a.cbase;
    v.s0 = a.s0;
    v.s1 = a.s1;
    v.perA = a.perA;
    v.perB = a.perB;
    v.tiles_a = (uint32_t)((a.LA + TA - 1) / TA);
    v.tiles_b = (uint32_t)((a.LB + TB - 1) / TB);
    const int64_t tiles = (int64_t)v.tiles_a * v.tiles_b;
    v.chunk = gol_chunk(nsl, tiles, want, forced_chunk);
    const int64_t n = tiles * ((nsl + v.chunk - 1) / v.chunk);
    v.nwg = n < (int64_t)UINT32_MAX ? (uint32_t)n : 0u;
    return v;
}

}  // namespace dccrgx
