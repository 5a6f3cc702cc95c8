// gol_sweep.hip -- the tiling sweep of the 26-neighbor game-of-life stencil,
// kept out of the library: every alternative build of the stencil (tile
// shapes, planes in flight, non-temporal loads, wave-independent tiles, the
// 2-D wave kernels) against the one gol.hip launches, on one synthetic slab.
// Each candidate is first checked bit-exactly against the library's kernel
// (which the host restatement below checks in turn), then timed with HIP
// events; GB/s counts the algorithmic 12 B per cell (is_alive read, next
// is_alive and live_neighbor_count written).
//
//   make -C tools gol_sweep && tools/gol_sweep LA LB C [perA perB [reps]]
//   e.g. tools/gol_sweep 2048 2048 2048 1 1 10   (the bench slab: 2048^3 on one GPU)
//        tools/gol_sweep 16384 1 16384 1 1 20    (2-D 16384^2: LB == 1 kernels)
#include <cstdio>
#include <cstring>
#include <vector>

#include "../dccrg_amd/csrc/gol_kernels.hpp"

namespace dccrgx {

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


}  // namespace dccrgx

using namespace dccrgx;

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

__global__ void k_fill(uint32_t* f, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = i + 0x9e3779b97f4a7c15ull;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        z ^= z >> 31;
        f[i] = (z % 1000) < 350 ? 1u + (uint32_t)((z >> 40) & 7) : 0u;
    }
}

__global__ void k_diff(const uint32_t* a, const uint32_t* b, const uint32_t* c, const uint32_t* d, size_t n,
                       unsigned long long* bad)
{
    unsigned long long k = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        k += (a[i] != b[i]) + (c[i] != d[i]);
    if (k) atomicAdd(bad, k);
}

struct Variant {
    const char* name;
    bool two_d;  // LB == 1 kernels
    void (*launch)(const GolArgs&, int64_t nsl, hipStream_t);
};

template <int NW, int RW, bool NT = false, int PF = 1, bool NTL = false>
static void run_v(const GolArgs& a, int64_t nsl, hipStream_t st)
{
    Gol4Args v = gol4_plan(a, 256, NW * RW, nsl, 0);
    hipLaunchKernelGGL((k_gol26v<NW, RW, NT, PF, NTL>), dim3(v.nwg), dim3(64 * NW), 0, st, v);
}
template <int RW>
static void run_w(const GolArgs& a, int64_t nsl, hipStream_t st)
{
    Gol4Args v = gol4_plan(a, 256, RW, nsl, 0);
    v.nwg = (v.nwg + 3) / 4;  // four independent waves per workgroup
    hipLaunchKernelGGL((k_gol26w<RW>), dim3(v.nwg), dim3(256), 0, st, v);
}
static void run_scalar3(const GolArgs& a0, int64_t nsl, hipStream_t st)
{
    GolArgs a = a0;
    a.tiles_a = (uint32_t)((a.LA + 63) / 64);
    a.tiles_b = (uint32_t)((a.LB + 15) / 16);
    const int64_t tiles = (int64_t)a.tiles_a * a.tiles_b;
    a.chunk = gol_chunk(nsl, tiles, 2048, 0);
    hipLaunchKernelGGL((k_gol26<64, 16, 1, 4>), dim3((unsigned)(tiles * ((nsl + a.chunk - 1) / a.chunk))), dim3(256),
                       0, st, a);
}
template <bool NTS>
static void run_rowv(const GolArgs& a, int64_t nsl, hipStream_t st)
{
    Gol4Args v = gol4_plan(a, 1024, 1, nsl, 0);
    hipLaunchKernelGGL((k_gol26_rowv<4, NTS>), dim3(v.nwg), dim3(256), 0, st, v, a.perB ? 3u : 1u);
}
template <int G>
static void run_2dw(const GolArgs& a, int64_t nsl, hipStream_t st)
{
    Gol4Args v = gol4_plan(a, 1024, 1, nsl, 0);
    hipLaunchKernelGGL((k_gol2d_wave<G>), dim3(v.nwg), dim3(256), 0, st, v, a.perB ? 3u : 1u);
}
static void run_scalar2(const GolArgs& a0, int64_t nsl, hipStream_t st)
{
    GolArgs a = a0;
    a.tiles_a = (uint32_t)((a.LA + 1023) / 1024);
    a.tiles_b = 1;
    a.chunk = gol_chunk(nsl, a.tiles_a, 2048, 0);
    hipLaunchKernelGGL((k_gol26_row<1024, 4>), dim3((unsigned)(a.tiles_a * ((nsl + a.chunk - 1) / a.chunk))),
                       dim3(256), 0, st, a, a.perB ? 3u : 1u);
}

// the library's choice first (gol.hip gol_launch), then the alternatives
static const Variant VARIANTS[] = {
    {"v8x4 nt (library)", false, run_v<8, 4, true>},
    {"v4x4", false, run_v<4, 4>},
    {"v4x2", false, run_v<4, 2>},
    {"v8x1", false, run_v<8, 1>},
    {"v8x2", false, run_v<8, 2>},
    {"v8x4", false, run_v<8, 4>},
    {"v16x2", false, run_v<16, 2>},
    {"v16x2 nt", false, run_v<16, 2, true>},
    {"v8x4 nt pf2", false, run_v<8, 4, true, 2>},
    {"v8x4 nt ntl", false, run_v<8, 4, true, 1, true>},
    {"v8x4 nt pf2 ntl", false, run_v<8, 4, true, 2, true>},
    {"v4x4 nt pf2", false, run_v<4, 4, true, 2>},
    {"v4x4 nt pf2 ntl", false, run_v<4, 4, true, 2, true>},
    {"wave x4", false, run_w<4>},
    {"wave x6", false, run_w<6>},
    {"wave x8", false, run_w<8>},
    {"wave x12", false, run_w<12>},
    {"wave x16", false, run_w<16>},
    {"scalar 64x16", false, run_scalar3},
    {"rowv4 (library)", true, run_rowv<false>},
    {"rowv4 nts", true, run_rowv<true>},
    {"2d wave G4", true, run_2dw<4>},
    {"2d wave G8", true, run_2dw<8>},
    {"2d wave G16", true, run_2dw<16>},
    {"row scalar 1024", true, run_scalar2},
};

// host restatement of the 27-point rule over the padded slab (planes 0 and
// C+1 are the ghost planes), examples/game_of_life.cpp:54-79
static void host_step(const std::vector<uint32_t>& in, std::vector<uint32_t>& out, std::vector<uint32_t>& cnt,
                      int64_t LA, int64_t LB, int64_t C, bool perA, bool perB)
{
    const int64_t S = LA * LB;
    for (int64_t c = 1; c <= C; c++)
        for (int64_t b = 0; b < LB; b++)
            for (int64_t a = 0; a < LA; a++) {
                uint32_t n = 0;
                for (int dc = -1; dc <= 1; dc++)
                    for (int db = -1; db <= 1; db++)
                        for (int da = -1; da <= 1; da++) {
                            if (!da && !db && !dc) continue;
                            int64_t x = a + da, y = b + db;
                            if (x < 0 || x >= LA) {
                                if (!perA) continue;
                                x = (x + LA) % LA;
                            }
                            if (y < 0 || y >= LB) {
                                if (!perB) continue;
                                y = (y + LB) % LB;
                            }
                            n += in[(c + dc) * S + x + LA * y] != 0;
                        }
                const size_t s = c * S + a + LA * b;
                cnt[s] = n;
                out[s] = n == 3 ? 1u : (n == 2 ? in[s] : 0u);
            }
}

int main(int argc, char** argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s LA LB C [perA perB [reps]]\n", argv[0]);
        return 2;
    }
    const int64_t LA = atoll(argv[1]), LB = atoll(argv[2]), C = atoll(argv[3]);
    const bool perA = argc > 4 ? atoi(argv[4]) != 0 : true, perB = argc > 5 ? atoi(argv[5]) != 0 : true;
    const int reps = argc > 6 ? atoi(argv[6]) : 20;
    if (LA % 4 || LA * LB >= (1ll << 31) || LA <= 0 || LB <= 0 || C <= 0) {
        fprintf(stderr, "LA %% 4 == 0 and LA * LB < 2^31 (the vector kernels' domain)\n");
        return 2;
    }
    const int64_t S = LA * LB, N = S * (C + 2);
    uint32_t *in, *out, *cnt, *ref_out, *ref_cnt;
    unsigned long long* d_bad;
    CK(hipMalloc(&d_bad, 8));
    // STAGGER=<bytes> (multiple of 16): out and cnt start that many (twice as
    // many) bytes later than their allocations, to test address aliasing
    const size_t stg = getenv("STAGGER") ? (size_t)atoll(getenv("STAGGER")) & ~(size_t)15 : 0;
    CK(hipMalloc(&in, N * 4 + 2 * stg));
    CK(hipMalloc(&out, N * 4 + 2 * stg));
    CK(hipMalloc(&cnt, N * 4 + 2 * stg));
    out += stg / 4;
    cnt += 2 * stg / 4;
    if (stg) printf("stagger %zu B\n", stg);
    CK(hipMalloc(&ref_out, N * 4));
    CK(hipMalloc(&ref_cnt, N * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, in, (size_t)N);
    CK(hipGetLastError());
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    GolArgs a{};
    a.in = in;
    a.LA = LA;
    a.LB = LB;
    a.S = S;
    a.lo = 0;
    a.hi = S * C;
    a.cbase = -1;  // storage slice 1 is canonical slice 0
    a.s0 = 1;
    a.s1 = C + 1;
    a.perA = perA;
    a.perB = perB;
    const bool two_d = LB == 1;
    const Variant* lib = nullptr;
    for (const Variant& v : VARIANTS)
        if (v.two_d == two_d) {
            lib = &v;
            break;
        }
    // the library kernel's result, checked against the host restatement on small slabs
    CK(hipMemset(ref_out, 0, N * 4));
    CK(hipMemset(ref_cnt, 0, N * 4));
    a.out = ref_out;
    a.cnt = ref_cnt;
    lib->launch(a, C, st);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(st));
    if (N <= (1ll << 26)) {
        std::vector<uint32_t> h_in(N), h_out(N, 0), h_cnt(N, 0), d_out(N), d_cnt(N);
        CK(hipMemcpy(h_in.data(), in, N * 4, hipMemcpyDeviceToHost));
        host_step(h_in, h_out, h_cnt, LA, LB, C, perA, perB);
        CK(hipMemcpy(d_out.data(), ref_out, N * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(d_cnt.data(), ref_cnt, N * 4, hipMemcpyDeviceToHost));
        if (d_out != h_out || d_cnt != h_cnt) {
            fprintf(stderr, "library kernel %s differs from the host restatement\n", lib->name);
            return 1;
        }
        printf("library kernel %s == host restatement (%lld cells)\n", lib->name, (long long)(S * C));
    }
    const double bytes = 12.0 * (double)(S * C);
    int bad = 0;
    for (const Variant& v : VARIANTS) {
        if (v.two_d != two_d) continue;
        CK(hipMemset(out, 0, N * 4));
        CK(hipMemset(cnt, 0, N * 4));
        a.out = out;
        a.cnt = cnt;
        v.launch(a, C, st);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(st));
        // bit-exact against the library kernel
        CK(hipMemset(d_bad, 0, 8));
        hipLaunchKernelGGL(k_diff, dim3(4096), dim3(256), 0, st, out, ref_out, cnt, ref_cnt, (size_t)N, d_bad);
        unsigned long long nbad = 0;
        CK(hipMemcpyAsync(&nbad, d_bad, 8, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        const bool same = nbad == 0;
        bad += !same;
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; r++) v.launch(a, C, st);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-20s %s %9.4f ms %8.1f GB/s\n", v.name, same ? "ok  " : "DIFF", ms, bytes / (ms * 1e6));
    }
    CK(hipFree(in));
    CK(hipFree(out - stg / 4));
    CK(hipFree(cnt - 2 * stg / 4));
    CK(hipFree(ref_out));
    CK(hipFree(ref_cnt));
    CK(hipFree(d_bad));
    return bad ? 1 : 0;
}
