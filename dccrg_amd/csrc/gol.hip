// gol.hip -- game-of-life stencil over a rank's slab (the user hot loop of
// examples/game_of_life.cpp:54-79 and tests/game_of_life/scalability3d.cpp:
// 136-165, executed on the device with the neighbor gather staged in LDS).
//
// Fast path (the default 26-item cube, i.e. neighborhood length 1): each
// workgroup owns a TA x TB tile of the (A, B) plane and marches along the
// slab axis C.  Every plane is read from HBM once into a double-buffered LDS
// tile (+1 apron in A and B, periodic wrap in index space), the 3x3 box sum
// of the plane is formed from LDS row sums and kept in registers, and the
// 27-point sum of plane c is S(c-1) + S(c) + S(c+1) - centre.  HBM traffic per
// cell: 4 B read (is_alive) + 4 B write (next is_alive) + 4 B write
// (live_neighbor_count) = 12 B -- the algorithmic minimum.
//
// Any other neighborhood (face neighbors, length >= 2, user neighborhoods)
// uses the generic item loop (one lane per cell, neighbor slots computed in
// closed form) -- same results, not bandwidth-optimised.
#include <algorithm>
#include <cstdlib>

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
// 16 rows along B; a workgroup is 4 waves, wave w owns tile rows 4w..4w+3,
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
// Wave-independent 26-neighbor stencil (LA % 4 == 0): every wavefront owns a
// 256-cell x RW-row tile and marches it along C with no workgroup barrier and
// no LDS.  Per plane a lane loads its dwordx4 of the RW own rows and of the
// two apron rows (those come from L2: the neighbouring tiles load them as
// their own rows), packs the alive bits 4 cells per u32, and takes its
// neighbours' edge bytes with cross-lane shuffles; the left / right apron
// cells come from scalar loads of lanes 0 and 63.  The next plane's loads are
// issued right after the current plane's values are taken out of their
// registers, so they overlap the sums and the stores.  Without barriers every
// wave keeps its own loads in flight (k_gol26v's 8-wave workgroups stall the
// CU's memory stream at each plane's __syncthreads).
template <int RW>
__global__ void __launch_bounds__(256) k_gol26w(Gol4Args g)
{
    constexpr int TA = 256, NR = RW + 2;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t bid = blockIdx.x, xcd = bid & 7, q8 = g.nwg >> 3, r8 = g.nwg & 7;
    const uint32_t wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const uint32_t tiles = g.tiles_a * g.tiles_b;
    const uint64_t wave_id = (uint64_t)wgid * 4 + w;
    const uint32_t tile_id = (uint32_t)(wave_id % tiles);
    const int64_t chunk_id = (int64_t)(wave_id / tiles);
    const int64_t a0 = (int64_t)(tile_id % g.tiles_a) * TA;
    const int64_t b0 = (int64_t)(tile_id / g.tiles_a) * RW;
    const int64_t c0 = g.s0 + chunk_id * g.chunk;
    const int64_t c1 = min(g.s1, c0 + g.chunk);
    if (c0 >= c1) return;  // wave-uniform: the whole wave leaves

    const int64_t LA = (int64_t)g.LA, LB = (int64_t)g.LB;
    auto wrapA = [&](int64_t a) -> int64_t {
        if (a >= 0 && a < LA) return a;
        return g.perA ? ug_wrap(a, LA) : -1;
    };
    auto wrapB = [&](int64_t b) -> int64_t {
        if (b >= 0 && b < LB) return b;
        return g.perB ? ug_wrap(b, LB) : -1;
    };
    // rows b0-1 .. b0+RW (r = 0 .. RW+1)
    const int64_t av = wrapA(a0 + 4 * lane);
    const int64_t ae = lane == 0 ? wrapA(a0 - 1) : (lane == 63 ? wrapA(a0 + TA) : -1);
    uint32_t roff[NR], eoff[NR];
    uint32_t rmask = 0, emask = 0;
#pragma unroll
    for (int r = 0; r < NR; r++) {
        const int64_t b = wrapB(b0 - 1 + r);
        const bool ok = av >= 0 && b >= 0;
        roff[r] = ok ? (uint32_t)(av + LA * b) : 0u;
        rmask |= ok ? (1u << r) : 0u;
        const bool eok = ae >= 0 && b >= 0;
        eoff[r] = eok ? (uint32_t)(ae + LA * b) : 0u;
        emask |= eok ? (1u << r) : 0u;
    }

    uint4 F[NR];
    uint32_t FE[NR];
    auto fetch = [&](int64_t sc) {
        const uint32_t* __restrict__ plane = g.in + (uint64_t)sc * g.S;
#pragma unroll
        for (int r = 0; r < NR; r++) {
            const uint4 v = *reinterpret_cast<const uint4*>(plane + roff[r]);
            F[r] = (rmask >> r) & 1u ? v : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < NR; r++) FE[r] = (emask >> r) & 1u ? plane[eoff[r]] : 0u;
    };
    // packed alive bits of the fetched plane and its 3x3 sums for the own
    // rows; nbx: some own cell of the plane holds a raw value other than 0 / 1
    // (then the rule re-reads the raw values instead of using the bits)
    uint32_t Sx[RW], Bx[RW];
    bool nbx = false;
    auto plane_sums = [&]() {
        uint32_t h[NR];
        uint32_t odd = 0;
#pragma unroll
        for (int r = 0; r < NR; r++) {
            const uint32_t m = pack_bits(F[r]);
            const uint32_t up = __shfl_up(m, 1, 64), dn = __shfl_down(m, 1, 64);
            const uint32_t lft = lane > 0 ? (up >> 24) : (FE[r] != 0u ? 1u : 0u);
            const uint32_t rgt = lane < 63 ? (dn & 0xffu) : (FE[r] != 0u ? 1u : 0u);
            h[r] = m + ((m << 8) | lft) + ((m >> 8) | (rgt << 24));
            if (r >= 1 && r <= RW) {
                Bx[r - 1] = m;
                odd |= (F[r].x | F[r].y | F[r].z | F[r].w) >> 1;
            }
        }
        nbx = __any(odd != 0u);
#pragma unroll
        for (int k = 0; k < RW; k++) Sx[k] = h[k] + h[k + 1] + h[k + 2];
    };

    uint32_t Sp[RW], Sc[RW], Bc[RW];
    bool nbc;
    fetch(c0 - 1);
    plane_sums();
#pragma unroll
    for (int k = 0; k < RW; k++) Sp[k] = Sx[k];
    fetch(c0);
    plane_sums();
#pragma unroll
    for (int k = 0; k < RW; k++) {
        Sc[k] = Sx[k];
        Bc[k] = Bx[k];
    }
    nbc = nbx;
    fetch(c0 + 1);
    const uint64_t ua = (uint64_t)(a0 + 4 * lane);
    const bool a_ok = (int64_t)ua < LA;
    for (int64_t c = c0; c < c1; c++) {
        // plane c+1 arrived: take it out of F, then issue plane c+2
        plane_sums();
        if (c + 2 <= c1) fetch(c + 2);
        const uint32_t* __restrict__ pin = g.in + (uint64_t)c * g.S;
        const uint64_t plin = g.S * (uint64_t)(c + g.cbase);
        const bool full = plin >= g.lo && plin + g.S <= g.hi;
        uint32_t* pcnt = g.cnt + (uint64_t)c * g.S;
        uint32_t* pout = g.out + (uint64_t)c * g.S;
#pragma unroll
        for (int k = 0; k < RW; k++) {
            const uint32_t cnt4 = Sp[k] + Sc[k] + Sx[k] - Bc[k];
            const int64_t b = b0 + k;
            if (a_ok && b < LB) {
                const uint32_t n0 = cnt4 & 0xffu, n1 = (cnt4 >> 8) & 0xffu, n2 = (cnt4 >> 16) & 0xffu,
                               n3 = cnt4 >> 24;
                const uint32_t p = (uint32_t)ua + (uint32_t)LA * (uint32_t)b;
                const uint32_t bc = Bc[k];
                // raw centre values: the alive bits unless the plane holds other values
                const uint4 v = nbc ? *reinterpret_cast<const uint4*>(pin + p)
                                    : make_uint4(bc & 1u, (bc >> 8) & 1u, (bc >> 16) & 1u, bc >> 24);
                typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 xc = {n0, n1, n2, n3};
                const u32x4 xv = {gol_rule(n0, v.x), gol_rule(n1, v.y), gol_rule(n2, v.z), gol_rule(n3, v.w)};
                if (full) {
                    __builtin_nontemporal_store(xc, reinterpret_cast<u32x4*>(pcnt + p));
                    __builtin_nontemporal_store(xv, reinterpret_cast<u32x4*>(pout + p));
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint64_t lin = plin + p + j;
                        if (lin >= g.lo && lin < g.hi) {
                            pcnt[p + j] = xc[j];
                            pout[p + j] = xv[j];
                        }
                    }
                }
            }
            Sp[k] = Sc[k];
            Sc[k] = Sx[k];
            Bc[k] = Bx[k];
        }
        nbc = nbx;
    }
}

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

// Wave-independent LB == 1 kernel (2-D grids, LA % 4 == 0): each wave owns a
// 256-cell strip of a row and marches along C on its own -- no LDS tile and
// no barrier.  The horizontal neighbours of a lane's 4 packed cells come from
// the adjacent lanes by cross-lane shuffles; lanes 0 and 63 fetch the strip's
// two apron cells.  Rows are fetched G at a time, G rows ahead of the ones
// being finished, so every wave keeps G dwordx4 loads in flight (the barrier
// per row of k_gol26_rowv capped its memory-level parallelism at one row).
template <int G>
__global__ void __launch_bounds__(256) k_gol2d_wave(Gol4Args g, uint32_t mult)
{
    constexpr int NW = 4;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t bid = blockIdx.x, xcd = bid & 7, q8 = g.nwg >> 3, r8 = g.nwg & 7;
    const uint32_t wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const uint32_t tile_id = wgid % g.tiles_a;
    const int64_t chunk_id = wgid / g.tiles_a;
    const int64_t a0 = ((int64_t)tile_id * NW + w) * 256;
    const int64_t c0 = g.s0 + chunk_id * g.chunk;
    const int64_t c1 = min(g.s1, c0 + g.chunk);
    const int64_t LA = (int64_t)g.LA;
    if (c0 >= c1 || a0 >= LA) return;  // wave-uniform
    auto wrapA = [&](int64_t a) -> int64_t {
        if (a >= 0 && a < LA) return a;
        return g.perA ? ug_wrap(a, LA) : -1;
    };
    const int64_t av = wrapA(a0 + 4 * lane);
    const bool vok = av >= 0;
    const uint32_t voff = vok ? (uint32_t)av : 0u;
    const int64_t ae = lane == 0 ? wrapA(a0 - 1) : (lane == 63 ? wrapA(a0 + 256) : -1);
    const bool eok = ae >= 0;
    const uint32_t eoff = eok ? (uint32_t)ae : 0u;

    uint4 F[G];
    uint32_t FE[G];
    auto fetch_row = [&](int64_t sc, uint4& v, uint32_t& e) {
        const uint32_t* __restrict__ plane = g.in + (uint64_t)sc * g.S;
        const uint4 x = *reinterpret_cast<const uint4*>(plane + voff);
        v = vok ? x : make_uint4(0, 0, 0, 0);
        e = eok ? plane[eoff] : 0u;
    };
    // packed 3-wide row sum of a row (4 cells per lane, one byte each)
    auto hsum = [&](uint32_t m, uint32_t e) -> uint32_t {
        const uint32_t up = __shfl_up(m, 1), dn = __shfl_down(m, 1);
        const uint32_t lft = lane > 0 ? (up >> 24) : (e != 0u ? 1u : 0u);
        const uint32_t rgt = lane < 63 ? (dn & 0xffu) : (e != 0u ? 1u : 0u);
        return mult * (m + ((m << 8) | lft) + ((m >> 8) | (rgt << 24)));
    };
    uint4 Vc;
    uint32_t Hp, Hc, Bc;
    {
        uint4 v;
        uint32_t e;
        fetch_row(c0 - 1, v, e);
        Hp = hsum(pack_bits(v), e);
        fetch_row(c0, Vc, e);
        Bc = pack_bits(Vc);
        Hc = hsum(Bc, e);
    }
#pragma unroll
    for (int j = 0; j < G; j++)
        if (c0 + 1 + j <= c1) fetch_row(c0 + 1 + j, F[j], FE[j]);
    const bool a_ok = a0 + 4 * lane < LA;
    const uint32_t p = (uint32_t)(a0 + 4 * lane);
    for (int64_t c = c0; c < c1; c += G) {
#pragma unroll
        for (int j = 0; j < G; j++) {
            const int64_t r = c + j;  // output row
            const uint32_t Bn = pack_bits(F[j]);
            const uint32_t Hn = hsum(Bn, FE[j]);
            const uint32_t cnt4 = Hp + Hc + Hn - Bc;
            if (a_ok && r < c1) {
                const uint32_t n0 = cnt4 & 0xffu, n1 = (cnt4 >> 8) & 0xffu, n2 = (cnt4 >> 16) & 0xffu,
                               n3 = cnt4 >> 24;
                const uint4 nc = make_uint4(n0, n1, n2, n3);
                const uint4 nv = make_uint4(gol_rule(n0, Vc.x), gol_rule(n1, Vc.y), gol_rule(n2, Vc.z),
                                            gol_rule(n3, Vc.w));
                const uint64_t plin = g.S * (uint64_t)(r + g.cbase);
                uint32_t* pcnt = g.cnt + (uint64_t)r * g.S;
                uint32_t* pout = g.out + (uint64_t)r * g.S;
                if (plin >= g.lo && plin + g.S <= g.hi) {
                    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                    const u32x4 xc = {nc.x, nc.y, nc.z, nc.w}, xv = {nv.x, nv.y, nv.z, nv.w};
                    __builtin_nontemporal_store(xc, reinterpret_cast<u32x4*>(pcnt + p));
                    __builtin_nontemporal_store(xv, reinterpret_cast<u32x4*>(pout + p));
                } else {
                    const uint32_t ncs[4] = {nc.x, nc.y, nc.z, nc.w}, nvs[4] = {nv.x, nv.y, nv.z, nv.w};
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        if (plin + p + q >= g.lo && plin + p + q < g.hi) {
                            pcnt[p + q] = ncs[q];
                            pout[p + q] = nvs[q];
                        }
                }
            }
            Hp = Hc;
            Hc = Hn;
            Bc = Bn;
            Vc = F[j];
            // refill the slot just consumed: row c+G+1+j, G rows ahead
            if (c + G + 1 + j <= c1) fetch_row(c + G + 1 + j, F[j], FE[j]);
        }
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

// generic neighborhood: one lane per local cell, closed-form neighbor slots
__global__ void __launch_bounds__(256) k_gol_items(UGeom g, const uint32_t* __restrict__ in,
                                                   uint32_t* __restrict__ out, uint32_t* __restrict__ cnt,
                                                   const int32_t* __restrict__ items, int K,
                                                   uint64_t lin0, uint64_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const uint64_t soff = (uint64_t)(-g.cbase * (int64_t)g.S);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t lin = lin0 + i;
        int64_t a, b, c;
        ug_decompose(g, lin, a, b, c);
        uint32_t count = 0;
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
            if ((c2 < 0 || c2 >= (int64_t)g.LC) && !g.perC) continue;
            count += alive_bit(in[ug_slot(g, a2, b2, c2)]);
        }
        const uint64_t s = lin + soff;
        cnt[s] = count;
        out[s] = gol_rule(count, in[s]);
    }
}

// deterministic synthetic initial state: alive = splitmix64(id) % 1000 < permille
__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) k_init_hash(uint32_t* __restrict__ f, uint64_t lin0, uint64_t n,
                                                   uint64_t soff, uint32_t permille)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t id = lin0 + i + 1;
        f[lin0 + i + soff] = (splitmix64(id) % 1000u) < permille ? 1u : 0u;
    }
}

static unsigned grid_for(uint64_t n)
{
    uint64_t g = (n + 255) / 256;
    if (g > 256 * 16) g = 256 * 16;
    if (g == 0) g = 1;
    return (unsigned)g;
}

// checksum of a 4-byte field over the local cells: (sum v, sum v * splitmix64(id))
// mod 2^64.  Local position i holds cell ids[i] (explicit grids) or lin0 + i + 1
// (uniform grids, slot lin0 + i + soff).  Per-block partials, then one block
// sums them in a fixed order (no atomics, bit-reproducible).
__global__ void __launch_bounds__(256) k_checksum(const uint32_t* __restrict__ f, uint64_t n, uint64_t lin0,
                                                  uint64_t soff, const uint64_t* __restrict__ ids,
                                                  uint64_t* __restrict__ partial)
{
    uint64_t s0 = 0, s1 = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t v = ids ? f[i] : f[lin0 + i + soff];
        const uint64_t id = ids ? ids[i] : lin0 + i + 1;
        s0 += v;
        s1 += v * splitmix64(id);
    }
    for (int o = 32; o > 0; o >>= 1) {
        s0 += __shfl_down(s0, o, 64);
        s1 += __shfl_down(s1, o, 64);
    }
    __shared__ uint64_t w0[4], w1[4];
    if (threadIdx.x % 64 == 0) {
        w0[threadIdx.x / 64] = s0;
        w1[threadIdx.x / 64] = s1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[2 * blockIdx.x] = w0[0] + w0[1] + w0[2] + w0[3];
        partial[2 * blockIdx.x + 1] = w1[0] + w1[1] + w1[2] + w1[3];
    }
}

__global__ void __launch_bounds__(64) k_checksum_final(const uint64_t* __restrict__ partial, uint32_t nb,
                                                       uint64_t* __restrict__ out)
{
    uint64_t s0 = 0, s1 = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += 64) {
        s0 += partial[2 * b];
        s1 += partial[2 * b + 1];
    }
    for (int o = 32; o > 0; o >>= 1) {
        s0 += __shfl_down(s0, o, 64);
        s1 += __shfl_down(s1, o, 64);
    }
    if (threadIdx.x == 0) {
        out[0] = s0;
        out[1] = s1;
    }
}

// the local cells' ids in slot order, explicit grids (explicit.hip)
int explicit_local_ids(const dccrgx_grid* grid, uint64_t* d_ids, hipStream_t st);

int gol_launch(dccrgx_grid* grid, const Hood& h, const Field& in, const Field& out, const Field& cnt,
               int64_t s0, int64_t s1, hipStream_t st)
{
    const UGeom& u = grid->g;
    if (s1 <= s0 || grid->n_local == 0) return DCCRGX_OK;
    if (!h.cube1) {
        // local lin range of the slices
        const int64_t S = (int64_t)u.S;
        const uint64_t l0 = std::max<int64_t>((s0 + u.cbase) * S, (int64_t)u.lo);
        const uint64_t l1 = std::min<int64_t>((s1 + u.cbase) * S, (int64_t)u.hi);
        if (l1 <= l0) return DCCRGX_OK;
        hipLaunchKernelGGL(k_gol_items, dim3(grid_for(l1 - l0)), dim3(256), 0, st, u,
                           (const uint32_t*)in.ptr, (uint32_t*)out.ptr, (uint32_t*)cnt.ptr, h.d_of_c, h.K,
                           l0, l1 - l0);
        DX_HIP(hipGetLastError());
        return DCCRGX_OK;
    }
    GolArgs a{};
    a.in = (const uint32_t*)in.ptr;
    a.out = (uint32_t*)out.ptr;
    a.cnt = (uint32_t*)cnt.ptr;
    a.LA = u.LA;
    a.LB = u.LB;
    a.S = u.S;
    a.lo = u.lo;
    a.hi = u.hi;
    a.cbase = u.cbase;
    a.s0 = s0;
    a.s1 = s1;
    a.perA = u.perA;
    a.perB = u.perB;
    const int64_t nsl = s1 - s0;
    if (u.LB == 1 && u.LA % 4 == 0 && u.S < (1ull << 31) && !getenv_flag("DCCRGX_GOL_SCALAR")) {
        Gol4Args v{};
        v.in = a.in;
        v.out = a.out;
        v.cnt = a.cnt;
        v.LA = u.LA;
        v.LB = 1;
        v.S = u.S;
        v.lo = u.lo;
        v.hi = u.hi;
        v.cbase = u.cbase;
        v.s0 = s0;
        v.s1 = s1;
        v.perA = u.perA;
        v.perB = u.perB;
        constexpr int NW = 4, TA = 256 * NW;
        // 0: k_gol26_rowv, 1: k_gol26_rowv with non-temporal stores, 4/8/16: k_gol2d_wave<G>
        // (tools/gol2d_sweep.py)
        const int64_t var2 = getenv_int("DCCRGX_GOL2D_VARIANT", 0);
        v.tiles_a = (uint32_t)((u.LA + TA - 1) / TA);
        v.tiles_b = 1;
        int64_t chunk = getenv_int("DCCRGX_GOL_CHUNK", 0);
        if (chunk <= 0) {
            const int64_t want = getenv_int("DCCRGX_GOL_WGS", 8192);
            int64_t chunks = std::max<int64_t>(1, std::min<int64_t>(nsl, (want + v.tiles_a - 1) / v.tiles_a));
            chunk = (nsl + chunks - 1) / chunks;
        }
        v.chunk = chunk;
        const int64_t chunks = (nsl + chunk - 1) / chunk;
        DX_CHECK((int64_t)v.tiles_a * chunks < (int64_t)UINT32_MAX, DCCRGX_EINVAL, "grid too large for one launch");
        v.nwg = (uint32_t)(v.tiles_a * chunks);
        const uint32_t mult = u.perB ? 3u : 1u;
        switch (var2) {
        case 1: hipLaunchKernelGGL((k_gol26_rowv<NW, true>), dim3(v.nwg), dim3(64 * NW), 0, st, v, mult); break;
        case 4: hipLaunchKernelGGL((k_gol2d_wave<4>), dim3(v.nwg), dim3(256), 0, st, v, mult); break;
        case 16: hipLaunchKernelGGL((k_gol2d_wave<16>), dim3(v.nwg), dim3(256), 0, st, v, mult); break;
        case 8: hipLaunchKernelGGL((k_gol2d_wave<8>), dim3(v.nwg), dim3(256), 0, st, v, mult); break;
        default: hipLaunchKernelGGL((k_gol26_rowv<NW>), dim3(v.nwg), dim3(64 * NW), 0, st, v, mult); break;
        }
    } else if (u.LB == 1) {
        constexpr int TA = 1024, NA = 4;
        a.tiles_a = (uint32_t)((u.LA + TA - 1) / TA);
        a.tiles_b = 1;
        int64_t chunks = std::max<int64_t>(1, std::min<int64_t>(nsl, (2048 + a.tiles_a - 1) / a.tiles_a));
        a.chunk = (nsl + chunks - 1) / chunks;
        chunks = (nsl + a.chunk - 1) / a.chunk;
        const uint32_t mult = u.perB ? 3u : 1u;
        hipLaunchKernelGGL((k_gol26_row<TA, NA>), dim3((unsigned)(a.tiles_a * chunks)), dim3(256), 0, st, a,
                           mult);
    } else if (u.LA % 4 == 0 && u.S < (1ull << 31) && !getenv_flag("DCCRGX_GOL_SCALAR")) {
        Gol4Args v{};
        v.in = a.in;
        v.out = a.out;
        v.cnt = a.cnt;
        v.LA = u.LA;
        v.LB = u.LB;
        v.S = u.S;
        v.lo = u.lo;
        v.hi = u.hi;
        v.cbase = u.cbase;
        v.s0 = s0;
        v.s1 = s1;
        v.perA = u.perA;
        v.perB = u.perB;
        // variant: waves per workgroup x rows per wave (tile = 256 x NW*RW)
        // 8 x 4 with non-temporal stores measured fastest on MI355X
        // (tools/gol_sweep.py; profiles/r1_summary.md)
        int64_t var = getenv_int("DCCRGX_GOL_VARIANT", 841);
        // 8 4 1 [P [L]]: 8 waves x 4 rows, NT stores, P planes in flight, L non-temporal loads
        // 9RR: wave-independent tiles of RR rows (k_gol26w)
        if (var != 44 && var != 42 && var != 81 && var != 162 && var != 82 && var != 84 && var != 1621 &&
            var != 8412 && var != 8411 && var != 84121 && var != 84111 && var != 4412 && var != 44121 &&
            var != 904 && var != 906 && var != 908 && var != 912 && var != 916)
            var = 841;
        int NW = 8, RW = 4;  // waves per workgroup (1: independent waves) x rows per wave
        switch (var) {
        case 44: case 4412: case 44121: NW = 4; RW = 4; break;
        case 42: NW = 4; RW = 2; break;
        case 81: NW = 8; RW = 1; break;
        case 82: NW = 8; RW = 2; break;
        case 162: case 1621: NW = 16; RW = 2; break;
        default:
            if (var >= 900 && var < 1000) {
                NW = 1;
                RW = (int)(var - 900);
            }
            break;
        }
        const int TB = NW * RW;
        v.tiles_a = (uint32_t)((u.LA + 255) / 256);
        v.tiles_b = (uint32_t)((u.LB + TB - 1) / TB);
        const int64_t tiles = (int64_t)v.tiles_a * v.tiles_b;
        // slices per workgroup: enough workgroups to fill 256 CUs several times
        int64_t chunk = getenv_int("DCCRGX_GOL_CHUNK", 0);
        if (chunk <= 0) {
            const int64_t want = getenv_int("DCCRGX_GOL_WGS", 8192);
            int64_t chunks = std::max<int64_t>(1, std::min<int64_t>(nsl, (want + tiles - 1) / tiles));
            chunk = (nsl + chunks - 1) / chunks;
        }
        v.chunk = chunk;
        const int64_t chunks = (nsl + chunk - 1) / chunk;
        DX_CHECK(tiles * chunks < (int64_t)UINT32_MAX, DCCRGX_EINVAL, "grid too large for one launch");
        v.nwg = (uint32_t)(tiles * chunks);
        if (NW == 1) v.nwg = (uint32_t)((tiles * chunks + 3) / 4);  // four independent waves per workgroup
        switch (var) {
        case 904: hipLaunchKernelGGL((k_gol26w<4>), dim3(v.nwg), dim3(256), 0, st, v); break;
        case 906: hipLaunchKernelGGL((k_gol26w<6>), dim3(v.nwg), dim3(256), 0, st, v); break;
        case 908: hipLaunchKernelGGL((k_gol26w<8>), dim3(v.nwg), dim3(256), 0, st, v); break;
        case 912: hipLaunchKernelGGL((k_gol26w<12>), dim3(v.nwg), dim3(256), 0, st, v); break;
        case 916: hipLaunchKernelGGL((k_gol26w<16>), dim3(v.nwg), dim3(256), 0, st, v); break;
        case 44: hipLaunchKernelGGL((k_gol26v<4, 4>), dim3(v.nwg), dim3(256), 0, st, v); break;
        case 42: hipLaunchKernelGGL((k_gol26v<4, 2>), dim3(v.nwg), dim3(256), 0, st, v); break;
        case 81: hipLaunchKernelGGL((k_gol26v<8, 1>), dim3(v.nwg), dim3(512), 0, st, v); break;
        case 162: hipLaunchKernelGGL((k_gol26v<16, 2>), dim3(v.nwg), dim3(1024), 0, st, v); break;
        case 82: hipLaunchKernelGGL((k_gol26v<8, 2>), dim3(v.nwg), dim3(512), 0, st, v); break;
        case 84: hipLaunchKernelGGL((k_gol26v<8, 4>), dim3(v.nwg), dim3(512), 0, st, v); break;
        case 1621: hipLaunchKernelGGL((k_gol26v<16, 2, true>), dim3(v.nwg), dim3(1024), 0, st, v); break;
        case 8412: hipLaunchKernelGGL((k_gol26v<8, 4, true, 2>), dim3(v.nwg), dim3(512), 0, st, v); break;
        case 8411: hipLaunchKernelGGL((k_gol26v<8, 4, true, 1, false>), dim3(v.nwg), dim3(512), 0, st, v); break;
        case 84121: hipLaunchKernelGGL((k_gol26v<8, 4, true, 2, true>), dim3(v.nwg), dim3(512), 0, st, v); break;
        case 84111: hipLaunchKernelGGL((k_gol26v<8, 4, true, 1, true>), dim3(v.nwg), dim3(512), 0, st, v); break;
        case 4412: hipLaunchKernelGGL((k_gol26v<4, 4, true, 2>), dim3(v.nwg), dim3(256), 0, st, v); break;
        case 44121: hipLaunchKernelGGL((k_gol26v<4, 4, true, 2, true>), dim3(v.nwg), dim3(256), 0, st, v); break;
        case 841:
        default: hipLaunchKernelGGL((k_gol26v<8, 4, true>), dim3(v.nwg), dim3(512), 0, st, v); break;
        }
    } else {
        constexpr int TA = 64, TB = 16, NA = 1, NB = 4;
        a.tiles_a = (uint32_t)((u.LA + TA - 1) / TA);
        a.tiles_b = (uint32_t)((u.LB + TB - 1) / TB);
        const int64_t tiles = (int64_t)a.tiles_a * a.tiles_b;
        int64_t chunks = std::max<int64_t>(1, std::min<int64_t>(nsl, (2048 + tiles - 1) / tiles));
        a.chunk = (nsl + chunks - 1) / chunks;
        chunks = (nsl + a.chunk - 1) / a.chunk;
        DX_CHECK(tiles * chunks < (int64_t)UINT32_MAX, DCCRGX_EINVAL, "grid too large for one launch");
        hipLaunchKernelGGL((k_gol26<TA, TB, NA, NB>), dim3((unsigned)(tiles * chunks)), dim3(256), 0, st, a);
    }
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

// explicit grids: CSR gather (explicit.hip)
int explicit_gol(dccrgx_grid* grid, const Hood& h, const Field& in, const Field& out, const Field& cnt,
                 int32_t region, hipStream_t st);

struct TimerPool {
    std::vector<hipEvent_t> ev;
    size_t used = 0;
    bool on = false;
};
static std::map<const dccrgx_grid*, TimerPool> g_timers;

static int timed(dccrgx_grid* grid, bool begin, hipStream_t st)
{
    auto it = g_timers.find(grid);
    if (it == g_timers.end() || !it->second.on) return DCCRGX_OK;
    TimerPool& T = it->second;
    if (T.used == T.ev.size()) {
        hipEvent_t e;
        DX_HIP(hipEventCreate(&e));
        T.ev.push_back(e);
    }
    (void)begin;
    DX_HIP(hipEventRecord(T.ev[T.used++], st));
    return DCCRGX_OK;
}

void region_slices(const dccrgx_grid* grid, const Hood& h, int32_t region, int64_t r[2][2])
{
    const UGeom& u = grid->g;
    const int64_t all0 = u.pad, all1 = (int64_t)u.nslices - u.pad;
    r[0][0] = r[0][1] = r[1][0] = r[1][1] = 0;
    if (region == DCCRGX_REGION_ALL) {
        r[0][0] = all0;
        r[0][1] = all1;
    } else if (region == DCCRGX_REGION_INNER) {
        r[0][0] = h.inner_s0;
        r[0][1] = h.inner_s1;
    } else {
        r[0][0] = all0;
        r[0][1] = std::min(h.inner_s0, all1);
        r[1][0] = std::max(h.inner_s1, all0);
        r[1][1] = all1;
        if (h.inner_s1 <= h.inner_s0) {  // no inner slices: everything is outer
            r[0][1] = all1;
            r[1][0] = r[1][1] = 0;
        }
    }
}

static int compute_region(dccrgx_grid* grid, const Hood& h, const Field& in, const Field& out,
                          const Field& cnt, int32_t region, hipStream_t st)
{
    if (!grid->uniform) return explicit_gol(grid, h, in, out, cnt, region, st);
    int64_t r[2][2];
    region_slices(grid, h, region, r);
    for (auto& x : r) {
        if (x[1] <= x[0]) continue;
        DX_TRY(timed(grid, true, st));
        DX_TRY(gol_launch(grid, h, in, out, cnt, x[0], x[1], st));
        DX_TRY(timed(grid, false, st));
    }
    return DCCRGX_OK;
}

}  // namespace dccrgx

using namespace dccrgx;

extern "C" {

static int gol_fields(dccrgx_grid* grid, int32_t a, int32_t b, int32_t c)
{
    const int32_t f[3] = {a, b, c};
    for (int i = 0; i < 3; i++) {
        DX_CHECK(f[i] >= 0 && (size_t)f[i] < grid->fields.size(), DCCRGX_EINVAL, "bad field %d", f[i]);
        DX_CHECK(grid->fields[f[i]].elem == 4 && !grid->fields[f[i]].variable, DCCRGX_EINVAL,
                 "game of life fields are 4-byte");
    }
    DX_CHECK(a != b && a != c && b != c, DCCRGX_EINVAL, "fields must be distinct (double buffered)");
    return DCCRGX_OK;
}

int dccrgx_gol_compute(dccrgx_grid* grid, int32_t hood_id, int32_t fin, int32_t fout, int32_t fcnt,
                       int32_t region)
{
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    const Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    DX_TRY(gol_fields(grid, fin, fout, fcnt));
    DX_CHECK(region >= DCCRGX_REGION_ALL && region <= DCCRGX_REGION_OUTER, DCCRGX_EINVAL, "bad region");
    return compute_region(grid, *h, grid->fields[fin], grid->fields[fout], grid->fields[fcnt], region,
                          grid->ctx->compute);
}

int dccrgx_gol_step(dccrgx_grid* grid, int32_t hood_id, int32_t fin, int32_t fout, int32_t fcnt)
{
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    const Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    DX_TRY(gol_fields(grid, fin, fout, fcnt));
    // scalability3d.cpp:122-166: start halo, inner cells, wait, outer cells
    DX_TRY(dccrgx_halo_start(grid, hood_id, &fin, 1));
    DX_TRY(dccrgx_gol_compute(grid, hood_id, fin, fout, fcnt, DCCRGX_REGION_INNER));
    DX_TRY(dccrgx_halo_wait(grid, hood_id, DCCRGX_WAIT_ALL));
    DX_TRY(dccrgx_gol_compute(grid, hood_id, fin, fout, fcnt, DCCRGX_REGION_OUTER));
    return DCCRGX_OK;
}

int dccrgx_field_init_hash(dccrgx_grid* grid, int32_t fid, uint32_t permille)
{
    DX_CHECK(grid && fid >= 0 && (size_t)fid < grid->fields.size(), DCCRGX_EINVAL, "bad field");
    DX_CHECK(grid->fields[fid].elem == 4, DCCRGX_EINVAL, "4-byte field expected");
    DX_CHECK(grid->uniform, DCCRGX_EINVAL, "uniform grids only");
    if (!grid->n_local) return DCCRGX_OK;
    const uint64_t soff = (uint64_t)(-grid->g.cbase * (int64_t)grid->g.S);
    hipLaunchKernelGGL(k_init_hash, dim3(grid_for(grid->n_local)), dim3(256), 0, grid->ctx->compute,
                       (uint32_t*)grid->fields[fid].ptr, grid->g.lo, grid->n_local, soff, permille);
    DX_HIP(hipGetLastError());
    DX_HIP(hipStreamSynchronize(grid->ctx->compute));
    return DCCRGX_OK;
}

int dccrgx_field_checksum(const dccrgx_grid* grid, int32_t fid, uint64_t out[2])
{
    DX_CHECK(grid && out && fid >= 0 && (size_t)fid < grid->fields.size(), DCCRGX_EINVAL, "bad argument");
    const Field& F = grid->fields[fid];
    DX_CHECK(F.elem == 4 && !F.variable, DCCRGX_EINVAL, "4-byte field expected");
    out[0] = out[1] = 0;
    const uint64_t n = grid->n_local;
    if (!n) return DCCRGX_OK;
    hipStream_t st = grid->ctx->compute;
    const unsigned nb = grid_for(n);
    uint64_t* d = nullptr;
    uint64_t* ids = nullptr;
    DX_HIP(dx_malloc(&d, (2 * (size_t)nb + 2) * 8));
    int s = DCCRGX_OK;
    uint64_t lin0 = 0, soff = 0;
    if (grid->uniform) {
        lin0 = grid->g.lo;
        soff = (uint64_t)(-grid->g.cbase * (int64_t)grid->g.S);
    } else {
        if (dx_malloc(&ids, n * 8) != hipSuccess) s = set_error(DCCRGX_ENOMEM, "checksum: no device memory");
        if (s == DCCRGX_OK) s = explicit_local_ids(grid, ids, st);
    }
    if (s == DCCRGX_OK) {
        hipLaunchKernelGGL(k_checksum, dim3(nb), dim3(256), 0, st, (const uint32_t*)F.ptr, n, lin0, soff,
                           (const uint64_t*)ids, d);
        hipLaunchKernelGGL(k_checksum_final, dim3(1), dim3(64), 0, st, (const uint64_t*)d, nb, d + 2 * nb);
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(out, d + 2 * nb, 16, hipMemcpyDeviceToHost, st) ||
            hipStreamSynchronize(st) != hipSuccess)
            s = set_error(DCCRGX_EHIP, "checksum kernel failed");
    }
    dx_free(ids);
    dx_free(d);
    return s;
}

int dccrgx_kernel_timer(dccrgx_grid* grid, int32_t reset, double* ms, uint64_t* launches)
{
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    TimerPool& T = g_timers[grid];
    if (reset) {
        DX_HIP(hipStreamSynchronize(grid->ctx->compute));
        T.used = 0;
        T.on = reset > 0;
        if (ms) *ms = 0;
        if (launches) *launches = 0;
        return DCCRGX_OK;
    }
    DX_HIP(hipStreamSynchronize(grid->ctx->compute));
    double tot = 0;
    for (size_t i = 0; i + 1 < T.used; i += 2) {
        float x = 0;
        DX_HIP(hipEventElapsedTime(&x, T.ev[i], T.ev[i + 1]));
        tot += x;
    }
    if (ms) *ms = tot;
    if (launches) *launches = T.used / 2;
    return DCCRGX_OK;
}

}  // extern "C"
