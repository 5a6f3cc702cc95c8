// grid.hip -- uniform implicit grid: block partition, neighborhoods,
// classification and per-peer send/receive lists built on the device with
// wave-ballot / prefix-scan stream compaction, ghost (pad) plans, fields.
//
// Reference behaviour reproduced (ykempf/dccrg):
//   create_level_0_cells      dccrg.hpp:8089-8145  (block partition)
//   initialize_neighborhoods  dccrg.hpp:8017-8076
//   find_neighbors_of / _to   dccrg.hpp:4375-4897  (closed form for one level)
//   update_remote_neighbor_info dccrg.hpp:9131-9409 (inner / outer / remote)
//   recalculate_..._lists     dccrg.hpp:8729-8891  (ascending per-peer lists)
#include <algorithm>
#include <array>
#include <cstring>

#include "grid.hpp"

namespace dccrgx {

// ---------------------------------------------------------------------------
// ordered stream compaction over lin intervals (count -> scan -> fill)
// ---------------------------------------------------------------------------
constexpr int CT = 256;       // threads
constexpr int CI = 16;        // iterations per block
constexpr int TILE = CT * CI;

struct Iv {
    uint64_t first, n;  // lin range [first, first + n)
};

template <class P>
__global__ void __launch_bounds__(CT) k_compact_count(uint64_t first, uint64_t n, P pred,
                                                      uint32_t* __restrict__ counts)
{
    __shared__ uint32_t wsum[CT / 64];
    const uint64_t base = first + (uint64_t)blockIdx.x * TILE;
    uint32_t c = 0;
    for (int it = 0; it < CI; it++) {
        const uint64_t j = (uint64_t)blockIdx.x * TILE + it * CT + threadIdx.x;
        const bool f = j < n && pred(base + it * CT + threadIdx.x);
        c += __popcll(__ballot(f)) * ((threadIdx.x & 63) == 0);
    }
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < CT / 64; w++) t += wsum[w];
        counts[blockIdx.x] = t;
    }
}

template <class P>
__global__ void __launch_bounds__(CT) k_compact_fill(uint64_t first, uint64_t n, P pred,
                                                     const uint64_t* __restrict__ offsets,
                                                     uint64_t* __restrict__ out)
{
    __shared__ uint32_t wsum[CT / 64];
    const uint64_t base = first + (uint64_t)blockIdx.x * TILE;
    uint64_t o = offsets[blockIdx.x];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int it = 0; it < CI; it++) {
        const uint64_t j = (uint64_t)blockIdx.x * TILE + it * CT + threadIdx.x;
        const uint64_t lin = base + it * CT + threadIdx.x;
        const bool f = j < n && pred(lin);
        const uint64_t m = __ballot(f);
        const uint32_t pre = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[w] = __popcll(m);
        __syncthreads();
        uint32_t woff = 0, tot = 0;
        for (int k = 0; k < CT / 64; k++) {
            woff += k < w ? wsum[k] : 0;
            tot += wsum[k];
        }
        if (f) out[o + woff + pre] = lin + 1;  // cell id
        o += tot;
        __syncthreads();
    }
}

// appends the ids (lin+1) in ascending order for which pred holds
template <class P>
static int compact(const std::vector<Iv>& ivs, P pred, std::vector<uint64_t>& out, hipStream_t st)
{
    for (const Iv& iv : ivs) {
        if (iv.n == 0) continue;
        const uint64_t nb = (iv.n + TILE - 1) / TILE;
        uint32_t* d_counts = nullptr;
        uint64_t* d_off = nullptr;
        DX_HIP(dx_malloc(&d_counts, nb * sizeof(uint32_t)));
        hipLaunchKernelGGL(k_compact_count<P>, dim3((unsigned)nb), dim3(CT), 0, st, iv.first, iv.n,
                           pred, d_counts);
        DX_HIP(hipGetLastError());
        std::vector<uint32_t> h(nb);
        DX_HIP(hipMemcpyAsync(h.data(), d_counts, nb * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        DX_HIP(hipStreamSynchronize(st));
        std::vector<uint64_t> off(nb);
        uint64_t tot = 0;
        for (uint64_t b = 0; b < nb; b++) {
            off[b] = tot;
            tot += h[b];
        }
        if (tot) {
            uint64_t* d_out = nullptr;
            DX_HIP(dx_malloc(&d_off, nb * sizeof(uint64_t)));
            DX_HIP(dx_malloc(&d_out, tot * sizeof(uint64_t)));
            DX_HIP(hipMemcpyAsync(d_off, off.data(), nb * sizeof(uint64_t), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_compact_fill<P>, dim3((unsigned)nb), dim3(CT), 0, st, iv.first,
                               iv.n, pred, d_off, d_out);
            DX_HIP(hipGetLastError());
            const size_t old = out.size();
            out.resize(old + tot);
            DX_HIP(hipMemcpyAsync(out.data() + old, d_out, tot * sizeof(uint64_t),
                                  hipMemcpyDeviceToHost, st));
            DX_HIP(hipStreamSynchronize(st));
            dx_free(d_out);
            dx_free(d_off);
        }
        dx_free(d_counts);
    }
    return DCCRGX_OK;
}

// ---------------------------------------------------------------------------
// predicates (uniform grid): one lane per candidate cell, loop over items
// ---------------------------------------------------------------------------
struct PredOuter {  // local cell with a remote neighbors_of or neighbors_to entry
    UGeom g;
    const int32_t* of;
    const int32_t* to;
    int K;
    __device__ bool operator()(uint64_t lin) const
    {
        int64_t a, b, c;
        ug_decompose(g, lin, a, b, c);
        for (int k = 0; k < K; k++) {
            uint64_t n;
            int64_t cu;
            if (ug_neighbor(g, a, b, c, of + 3 * k, n, cu) && !ug_local(g, n)) return true;
            if (ug_neighbor(g, a, b, c, to + 3 * k, n, cu) && !ug_local(g, n)) return true;
        }
        return false;
    }
};

struct PredSend {  // local cell with a neighbors_to entry owned by `peer`
    UGeom g;
    const int32_t* to;
    int K;
    int peer;
    __device__ bool operator()(uint64_t lin) const
    {
        int64_t a, b, c;
        ug_decompose(g, lin, a, b, c);
        for (int k = 0; k < K; k++) {
            uint64_t n;
            int64_t cu;
            if (ug_neighbor(g, a, b, c, to + 3 * k, n, cu) && !ug_local(g, n) && ug_owner(g, n) == peer)
                return true;
        }
        return false;
    }
};

struct PredRecv {  // remote cell that is in neighbors_of of a local cell
    UGeom g;
    const int32_t* to;
    int K;
    __device__ bool operator()(uint64_t lin) const
    {
        int64_t a, b, c;
        ug_decompose(g, lin, a, b, c);
        for (int k = 0; k < K; k++) {
            uint64_t n;
            int64_t cu;
            if (ug_neighbor(g, a, b, c, to + 3 * k, n, cu) && ug_local(g, n)) return true;
        }
        return false;
    }
};

struct PredRemote {  // remote cell in neighbors_of or neighbors_to of a local cell
    UGeom g;
    const int32_t* of;
    const int32_t* to;
    int K;
    __device__ bool operator()(uint64_t lin) const
    {
        int64_t a, b, c;
        ug_decompose(g, lin, a, b, c);
        for (int k = 0; k < K; k++) {
            uint64_t n;
            int64_t cu;
            if (ug_neighbor(g, a, b, c, to + 3 * k, n, cu) && ug_local(g, n)) return true;
            if (ug_neighbor(g, a, b, c, of + 3 * k, n, cu) && ug_local(g, n)) return true;
        }
        return false;
    }
};

// ---------------------------------------------------------------------------
// ghost (pad) plan: what every non-local storage slot holds
// kind: 0 nothing, 1 self copy (val = source slot), 2 received (peer, val = index)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_pad_plan(UGeom g, uint64_t s_first, uint64_t n,
                                                  const uint64_t* __restrict__ recv_ids,
                                                  const uint64_t* __restrict__ peer_off,
                                                  const int32_t* __restrict__ peer_rank, int npeers,
                                                  int8_t* __restrict__ kind, int32_t* __restrict__ pidx,
                                                  uint64_t* __restrict__ val)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t s = s_first + i;
        const uint64_t sc = divide(s, g.dS);
        const uint64_t rem = s - sc * g.S;
        const int64_t cu = (int64_t)sc + g.cbase;
        int8_t k = 0;
        int32_t pi = -1;
        uint64_t v = 0;
        int64_t cw = cu;
        bool ok = true;
        if (cu < 0 || cu >= (int64_t)g.LC) {
            if (!g.perC) ok = false;
            else cw = ug_wrap(cu, (int64_t)g.LC);
        }
        if (ok) {
            const uint64_t lin = rem + g.S * (uint64_t)cw;
            if (ug_local(g, lin)) {
                k = 1;
                v = rem + g.S * (uint64_t)(cw - g.cbase);
            } else {
                const int p = ug_owner(g, lin);
                for (int j = 0; j < npeers; j++) {
                    if (peer_rank[j] != p) continue;
                    uint64_t lo = peer_off[j], hi = peer_off[j + 1];
                    const uint64_t id = lin + 1;
                    while (lo < hi) {
                        const uint64_t mid = (lo + hi) >> 1;
                        if (recv_ids[mid] < id) lo = mid + 1;
                        else hi = mid;
                    }
                    if (lo < peer_off[j + 1] && recv_ids[lo] == id) {
                        k = 2;
                        pi = j;
                        v = lo - peer_off[j];
                    }
                    break;
                }
            }
        }
        kind[i] = k;
        pidx[i] = pi;
        val[i] = v;
    }
}

static unsigned grid_for(uint64_t n)
{
    uint64_t g = (n + 255) / 256;
    if (g > 256 * 16) g = 256 * 16;
    if (g == 0) g = 1;
    return (unsigned)g;
}

template <class T>
static int upload(const std::vector<T>& v, T** d, hipStream_t st)
{
    *d = nullptr;
    if (v.empty()) return DCCRGX_OK;
    DX_HIP(dx_malloc(d, v.size() * sizeof(T)));
    DX_HIP(hipMemcpyAsync(*d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st));
    return DCCRGX_OK;
}

void free_hood(Hood& h)
{
    FreeBatch fb;
    for (void* p : {(void*)h.d_of_c, (void*)h.d_to_c, (void*)h.d_self_dst, (void*)h.d_self_src}) fb.add(p);
    for (PeerPlan& p : h.peers) {
        for (void* q : {(void*)p.d_send_slots, (void*)p.d_unpack_dst, (void*)p.d_unpack_src, p.d_send_buf,
                        p.d_recv_buf})
            fb.add(q);
        free_var_plans(p.var_send, fb);
        free_var_plans(p.var_recv, fb);
    }
    free_var_plans(h.var_self, fb);
    h.d_of_c = h.d_to_c = nullptr;
    h.d_self_dst = h.d_self_src = nullptr;
    h.peers.clear();
    for (void* p : {(void*)h.d_nof_row, (void*)h.d_nof_id, (void*)h.d_nof_off, (void*)h.d_nof_g,
                    (void*)h.d_nto_row, (void*)h.d_nto_g, (void*)h.d_st_row, (void*)h.d_st_slot,
                    (void*)h.d_st_off})
        fb.add(p);
    h.d_st_off = nullptr;
    h.d_nof_row = h.d_nof_id = h.d_nto_row = h.d_st_row = nullptr;
    h.d_nof_off = nullptr;
    h.d_nof_g = h.d_nto_g = h.d_st_slot = nullptr;
    h.n_rows = 0;
    h.faces.reset();
    h.iter.reset();
}

Hood* find_hood(dccrgx_grid* g, int32_t id)
{
    auto it = g->hoods.find(id);
    return it == g->hoods.end() ? nullptr : &it->second;
}

const Hood* find_hood(const dccrgx_grid* g, int32_t id)
{
    auto it = g->hoods.find(id);
    return it == g->hoods.end() ? nullptr : &it->second;
}

static void add_iv(std::vector<Iv>& v, int64_t a, int64_t b, int64_t N)  // [a, b) clipped
{
    a = std::max<int64_t>(a, 0);
    b = std::min<int64_t>(b, N);
    if (a < b) v.push_back({(uint64_t)a, (uint64_t)(b - a)});
}

// sorted disjoint union, minus [ex0, ex1)
static std::vector<Iv> norm_ivs(std::vector<Iv> v, uint64_t ex0, uint64_t ex1)
{
    std::vector<std::pair<uint64_t, uint64_t>> r;
    for (const Iv& x : v) {
        const uint64_t a = x.first, b = x.first + x.n;
        if (b <= ex0 || a >= ex1) r.push_back({a, b});
        else {
            if (a < ex0) r.push_back({a, ex0});
            if (b > ex1) r.push_back({ex1, b});
        }
    }
    std::sort(r.begin(), r.end());
    std::vector<Iv> out;
    for (auto& p : r) {
        if (!out.empty() && p.first <= out.back().first + out.back().n) {
            const uint64_t e = std::max(out.back().first + out.back().n, p.second);
            out.back().n = e - out.back().first;
        } else {
            out.push_back({p.first, p.second - p.first});
        }
    }
    return out;
}

int build_hood(dccrgx_grid* grid, Hood& h)
{
    Ctx* ctx = grid->ctx;
    const UGeom& g = grid->g;
    hipStream_t st = ctx->compute;
    free_hood(h);
    h.outer.clear();
    h.remote.clear();
    h.self_segs.clear();
    h.n_self_scatter = 0;
    h.K = (int32_t)(h.items.size() / 3);
    h.of_c.resize(h.items.size());
    h.to_c.resize(h.items.size());
    for (int k = 0; k < h.K; k++)
        for (int d = 0; d < 3; d++) {
            h.of_c[3 * k + d] = h.items[3 * k + g.perm[d]];
            h.to_c[3 * k + d] = -h.of_c[3 * k + d];
        }
    // the default 26-item cube (any axis order) takes the LDS stencil path
    h.cube1 = false;
    if (h.K == 26) {
        bool all = true;
        for (int k = 0; k < 26 && all; k++) {
            int m = 0;
            for (int d = 0; d < 3; d++) m = std::max(m, std::abs(h.items[3 * k + d]));
            all = (m == 1);
        }
        h.cube1 = all;
    }
    // neighbor counts in closed form (dccrgx_neighbors_of on uniform grids):
    // the full cube of some length, or the six face items
    {
        std::set<std::array<int32_t, 3>> distinct;
        int m = 0;
        bool faces = h.K == 6;
        for (int k = 0; k < h.K; k++) {
            const std::array<int32_t, 3> it = {h.items[3 * k], h.items[3 * k + 1], h.items[3 * k + 2]};
            distinct.insert(it);
            int mk = 0, nz = 0;
            for (int d = 0; d < 3; d++) {
                mk = std::max(mk, std::abs(it[d]));
                nz += it[d] != 0;
            }
            m = std::max(m, mk);
            faces &= mk == 1 && nz == 1;
        }
        const bool unique = (int)distinct.size() == h.K && !distinct.count({0, 0, 0});
        h.count_cube = unique && m >= 1 && h.K == (2 * m + 1) * (2 * m + 1) * (2 * m + 1) - 1 ? m : -1;
        h.count_faces = unique && faces;
    }
    DX_TRY(upload(h.of_c, &h.d_of_c, st));
    DX_TRY(upload(h.to_c, &h.d_to_c, st));
    if (grid->n_local == 0) return DCCRGX_OK;

    const int64_t N = (int64_t)g.N;
    const int64_t W = (int64_t)(g.pad + 1) * (int64_t)g.S;
    const int64_t lo = (int64_t)g.lo, hi = (int64_t)g.hi;

    // local candidates: within W of either end of the local range
    std::vector<Iv> lc;
    add_iv(lc, lo, std::min(hi, lo + W), N);
    add_iv(lc, std::max(lo, hi - W), hi, N);
    lc = norm_ivs(lc, 0, 0);
    // remote candidates
    std::vector<Iv> rc;
    add_iv(rc, lo - W, lo, N);
    add_iv(rc, hi, hi + W, N);
    if (g.perC) {
        add_iv(rc, 0, W, N);
        add_iv(rc, N - W, N, N);
    }
    rc = norm_ivs(rc, (uint64_t)lo, (uint64_t)hi);

    // outer cells (dccrg.hpp:9180-9223)
    DX_TRY(compact(lc, PredOuter{g, h.d_of_c, h.d_to_c, h.K}, h.outer, st));
    // remote cells on the process boundary
    DX_TRY(compact(rc, PredRemote{g, h.d_of_c, h.d_to_c, h.K}, h.remote, st));

    // candidate peers: owners of remote candidates
    std::vector<int> peers;
    for (const Iv& iv : rc) {
        const int p0 = ug_owner(g, iv.first), p1 = ug_owner(g, iv.first + iv.n - 1);
        for (int p = p0; p <= p1; p++)
            if (p != g.rank && part_count(g.part, p) > 0) peers.push_back(p);
    }
    std::sort(peers.begin(), peers.end());
    peers.erase(std::unique(peers.begin(), peers.end()), peers.end());
    for (int p : peers) {
        PeerPlan pp;
        pp.peer = p;
        DX_TRY(compact(lc, PredSend{g, h.d_to_c, h.K, p}, pp.send_ids, st));
        const uint64_t f0 = part_first(g.part, p) - 1, f1 = f0 + part_count(g.part, p);
        std::vector<Iv> pr;
        for (const Iv& iv : rc) {
            const uint64_t a = std::max(iv.first, f0), b = std::min(iv.first + iv.n, f1);
            if (a < b) pr.push_back({a, b - a});
        }
        DX_TRY(compact(pr, PredRecv{g, h.d_to_c, h.K}, pp.recv_ids, st));
        if (!pp.send_ids.empty() || !pp.recv_ids.empty()) h.peers.push_back(std::move(pp));
    }

    // send slots (local cells: slot = lin - cbase * S)
    for (PeerPlan& pp : h.peers) {
        if (pp.send_ids.empty()) continue;
        std::vector<uint64_t> slots(pp.send_ids.size());
        const uint64_t off = (uint64_t)(-g.cbase * (int64_t)g.S);
        for (size_t i = 0; i < slots.size(); i++) slots[i] = pp.send_ids[i] - 1 + off;
        pp.send_direct = true;
        for (size_t i = 1; i < slots.size(); i++)
            if (slots[i] != slots[0] + i) pp.send_direct = false;
        pp.send_slot0 = slots[0];
        if (!pp.send_direct) DX_TRY(upload(slots, &pp.d_send_slots, st));
        pp.h_send_slots = std::move(slots);
    }

    // pad plan over all non-local storage slots
    const uint64_t lo_s = (uint64_t)(lo - g.cbase * (int64_t)g.S);
    const uint64_t hi_s = (uint64_t)(hi - g.cbase * (int64_t)g.S);
    const uint64_t tot_s = g.nslices * g.S;
    std::vector<uint64_t> all_recv, poff(1, 0);
    std::vector<int32_t> prank;
    for (const PeerPlan& pp : h.peers) {
        all_recv.insert(all_recv.end(), pp.recv_ids.begin(), pp.recv_ids.end());
        poff.push_back(all_recv.size());
        prank.push_back(pp.peer);
    }
    uint64_t* d_recv = nullptr;
    uint64_t* d_poff = nullptr;
    int32_t* d_prank = nullptr;
    DX_TRY(upload(all_recv, &d_recv, st));
    DX_TRY(upload(poff, &d_poff, st));
    DX_TRY(upload(prank, &d_prank, st));
    std::vector<std::vector<std::pair<uint64_t, uint64_t>>> unpack(h.peers.size());  // (idx, dst)
    std::vector<std::pair<uint64_t, uint64_t>> self;                                // (dst, src)
    const uint64_t ranges[2][2] = {{0, lo_s}, {hi_s, tot_s}};
    for (auto& r : ranges) {
        const uint64_t n = r[1] - r[0];
        if (n == 0) continue;
        int8_t* d_kind = nullptr;
        int32_t* d_pidx = nullptr;
        uint64_t* d_val = nullptr;
        DX_HIP(dx_malloc(&d_kind, n));
        DX_HIP(dx_malloc(&d_pidx, n * 4));
        DX_HIP(dx_malloc(&d_val, n * 8));
        hipLaunchKernelGGL(k_pad_plan, dim3(grid_for(n)), dim3(256), 0, st, g, r[0], n, d_recv, d_poff,
                           d_prank, (int)prank.size(), d_kind, d_pidx, d_val);
        DX_HIP(hipGetLastError());
        std::vector<int8_t> kind(n);
        std::vector<int32_t> pidx(n);
        std::vector<uint64_t> val(n);
        DX_HIP(hipMemcpyAsync(kind.data(), d_kind, n, hipMemcpyDeviceToHost, st));
        DX_HIP(hipMemcpyAsync(pidx.data(), d_pidx, n * 4, hipMemcpyDeviceToHost, st));
        DX_HIP(hipMemcpyAsync(val.data(), d_val, n * 8, hipMemcpyDeviceToHost, st));
        DX_HIP(hipStreamSynchronize(st));
        dx_free(d_kind);
        dx_free(d_pidx);
        dx_free(d_val);
        for (uint64_t i = 0; i < n; i++) {
            if (kind[i] == 1) self.push_back({r[0] + i, val[i]});
            else if (kind[i] == 2) unpack[pidx[i]].push_back({val[i], r[0] + i});
        }
    }
    dx_free(d_recv);
    dx_free(d_poff);
    dx_free(d_prank);

    for (size_t j = 0; j < h.peers.size(); j++) {
        PeerPlan& pp = h.peers[j];
        auto& u = unpack[j];
        std::stable_sort(u.begin(), u.end());
        pp.recv_direct = !u.empty() && u.size() == pp.recv_ids.size();
        for (size_t i = 0; i < u.size() && pp.recv_direct; i++)
            if (u[i].first != i || u[i].second != u[0].second + i) pp.recv_direct = false;
        DX_CHECK(pp.recv_ids.empty() || !u.empty(), DCCRGX_EINTERNAL,
                 "received cells of peer %d have no ghost slot", pp.peer);
        pp.h_unpack_dst.clear();
        pp.h_unpack_src.clear();
        for (auto& e : u) {
            pp.h_unpack_src.push_back(e.first);
            pp.h_unpack_dst.push_back(e.second);
        }
        if (pp.recv_direct) {
            pp.recv_slot0 = u[0].second;
        } else {
            pp.n_unpack = u.size();
            std::vector<uint64_t> dst(u.size()), src(u.size());
            for (size_t i = 0; i < u.size(); i++) {
                src[i] = u[i].first;
                dst[i] = u[i].second;
            }
            DX_TRY(upload(dst, &pp.d_unpack_dst, st));
            DX_TRY(upload(src, &pp.d_unpack_src, st));
        }
    }
    if (ctx->self_peer && ctx->has_comm && !self.empty()) {
        // own periodic images as messages to this rank (test mode): one
        // peer plan, cells ascending, read from their local slots
        const uint64_t off = (uint64_t)(-g.cbase * (int64_t)g.S);
        PeerPlan pp;
        pp.peer = g.rank;
        for (auto& e : self) pp.send_ids.push_back(e.second - off + 1);
        std::sort(pp.send_ids.begin(), pp.send_ids.end());
        pp.send_ids.erase(std::unique(pp.send_ids.begin(), pp.send_ids.end()), pp.send_ids.end());
        pp.recv_ids = pp.send_ids;
        std::vector<uint64_t> slots(pp.send_ids.size());
        for (size_t i = 0; i < slots.size(); i++) slots[i] = pp.send_ids[i] - 1 + off;
        pp.send_direct = true;
        for (size_t i = 1; i < slots.size(); i++)
            if (slots[i] != slots[0] + i) pp.send_direct = false;
        pp.send_slot0 = slots[0];
        if (!pp.send_direct) DX_TRY(upload(slots, &pp.d_send_slots, st));
        std::vector<std::pair<uint64_t, uint64_t>> u;  // (message index, dst)
        for (auto& e : self) {
            const uint64_t id = e.second - off + 1;
            u.push_back({(uint64_t)(std::lower_bound(pp.send_ids.begin(), pp.send_ids.end(), id) -
                                    pp.send_ids.begin()),
                         e.first});
        }
        std::stable_sort(u.begin(), u.end());
        pp.recv_direct = u.size() == pp.recv_ids.size();
        for (size_t i = 0; i < u.size() && pp.recv_direct; i++)
            if (u[i].first != i || u[i].second != u[0].second + i) pp.recv_direct = false;
        for (auto& e : u) {
            pp.h_unpack_src.push_back(e.first);
            pp.h_unpack_dst.push_back(e.second);
        }
        if (pp.recv_direct) {
            pp.recv_slot0 = u[0].second;
        } else {
            pp.n_unpack = u.size();
            DX_TRY(upload(pp.h_unpack_dst, &pp.d_unpack_dst, st));
            DX_TRY(upload(pp.h_unpack_src, &pp.d_unpack_src, st));
        }
        pp.h_send_slots = std::move(slots);
        auto at = std::lower_bound(h.peers.begin(), h.peers.end(), pp.peer,
                                   [](const PeerPlan& a, int p) { return a.peer < p; });
        h.peers.insert(at, std::move(pp));
        self.clear();
    }
    h.h_self = self;
    {
        FreeBatch fb;
        free_var_plans(h.var_self, fb);  // built for the previous copies
    }
    // self copies: contiguous runs become memcpys when there are few of them
    std::vector<CopySeg> segs;
    for (auto& e : self) {
        if (!segs.empty() && segs.back().dst + segs.back().n == e.first &&
            segs.back().src + segs.back().n == e.second)
            segs.back().n++;
        else
            segs.push_back({e.first, e.second, 1});
    }
    if (segs.size() <= 64) {
        h.self_segs = segs;
    } else {
        h.n_self_scatter = self.size();
        std::vector<uint64_t> dst(self.size()), src(self.size());
        for (size_t i = 0; i < self.size(); i++) {
            dst[i] = self[i].first;
            src[i] = self[i].second;
        }
        DX_TRY(upload(dst, &h.d_self_dst, st));
        DX_TRY(upload(src, &h.d_self_src, st));
    }

    // overlap split: slices whose stencil reads only local or self-copied data
    const int64_t cs = lo / (int64_t)g.S, ce = (hi - 1) / (int64_t)g.S;
    bool remote_pads = false;
    for (const PeerPlan& pp : h.peers) remote_pads |= !pp.recv_ids.empty();
    int64_t c0 = cs, c1 = ce + 1;  // canonical [c0, c1)
    if (remote_pads) {
        const int64_t cA = (lo % (int64_t)g.S == 0) ? cs : cs + 1;
        const int64_t cB = (hi % (int64_t)g.S == 0) ? ce : ce - 1;
        c0 = cA + g.pad;
        c1 = cB - g.pad + 1;
        if (c1 < c0) c1 = c0;
    }
    h.inner_s0 = c0 - g.cbase;
    h.inner_s1 = c1 - g.cbase;
    DX_HIP(hipStreamSynchronize(st));
    return DCCRGX_OK;
}

static int default_items(uint32_t hood_length, std::vector<int32_t>& items)
{
    // dccrg.hpp:8017-8076
    items.clear();
    if (hood_length == 0) {
        const int32_t f[6][3] = {{0, 0, -1}, {0, -1, 0}, {-1, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
        for (auto& it : f) items.insert(items.end(), it, it + 3);
        return DCCRGX_OK;
    }
    const int h = (int)hood_length;
    for (int z = -h; z <= h; z++)
        for (int y = -h; y <= h; y++)
            for (int x = -h; x <= h; x++)
                if (x || y || z) items.insert(items.end(), {x, y, z});
    return DCCRGX_OK;
}

}  // namespace dccrgx

using namespace dccrgx;

static int grid_create(dccrgx_ctx* ctx, const dccrgx_grid_params* prm, const uint64_t* leaves, size_t n_leaves,
                       bool partial, dccrgx_grid** out);

extern "C" {

int dccrgx_grid_create(dccrgx_ctx* ctx, const dccrgx_grid_params* prm, const uint64_t* leaves,
                       size_t n_leaves, dccrgx_grid** out)
{
    return grid_create(ctx, prm, leaves, n_leaves, false, out);
}

}  // extern "C"

// the explicit grid over a box of leaves cut from a larger grid (hybrid.hip)
int dccrgx::grid_create_box(dccrgx_ctx* ctx, const dccrgx_grid_params* prm, const uint64_t* leaves, size_t n,
                            dccrgx_grid** out)
{
    return grid_create(ctx, prm, leaves, n, true, out);
}

static int grid_create(dccrgx_ctx* ctx, const dccrgx_grid_params* prm, const uint64_t* leaves, size_t n_leaves,
                       bool partial, dccrgx_grid** out)
{
    DX_CHECK(ctx && prm && out, DCCRGX_EINVAL, "null argument");
    DX_HIP(hipSetDevice(ctx->device));
    dccrgx_mapping m{};
    std::memcpy(m.length, prm->length, sizeof(m.length));
    m.max_ref_lvl = prm->max_ref_lvl;
    auto grid = std::make_unique<dccrgx_grid>();
    grid->ctx = ctx;
    grid->params = *prm;
    DX_TRY(make_map_params(&m, &grid->map));
    grid->params.max_ref_lvl = grid->map.max_lvl;
    DX_HIP(hipEventCreate(&grid->t0));
    DX_HIP(hipEventCreate(&grid->t1));
    DX_CHECK(prm->partition == DCCRGX_PARTITION_BLOCK || prm->partition == DCCRGX_PARTITION_SFC, DCCRGX_EINVAL,
             "unknown partition %d", (int)prm->partition);
    std::vector<uint64_t> all_level0;
    if (prm->partition == DCCRGX_PARTITION_SFC) {
        DX_TRY(sfc_plan(prm->length, ctx->comm_size, grid->sfc));
        if (!leaves) {  // every level-0 cell, on the explicit layout
            all_level0.resize(grid->map.nlevel0);
            for (uint64_t i = 0; i < all_level0.size(); i++) all_level0[i] = i + 1;
            leaves = all_level0.data();
            n_leaves = all_level0.size();
        }
    }
    if (leaves) {
        grid->uniform = false;
        grid->partial_leaves = partial;
        DX_TRY(explicit_create(grid.get(), leaves, n_leaves));
        *out = grid.release();
        return DCCRGX_OK;
    }
    // uniform implicit grid
    UGeom& g = grid->g;
    const uint64_t* L = prm->length;
    int perm[3];
    if (L[2] > 1) { perm[0] = 0; perm[1] = 1; perm[2] = 2; }
    else if (L[1] > 1) { perm[0] = 0; perm[1] = 2; perm[2] = 1; }
    else { perm[0] = 1; perm[1] = 2; perm[2] = 0; }
    for (int d = 0; d < 3; d++) g.perm[d] = perm[d];
    g.LA = L[perm[0]];
    g.LB = L[perm[1]];
    g.LC = L[perm[2]];
    g.perA = prm->periodic[perm[0]] ? 1 : 0;
    g.perB = prm->periodic[perm[1]] ? 1 : 0;
    g.perC = prm->periodic[perm[2]] ? 1 : 0;
    g.S = g.LA * g.LB;
    g.N = g.S * g.LC;
    g.dA = make_divider(g.LA);
    g.dS = make_divider(g.S);
    g.part = make_partition(g.N, ctx->comm_size);
    g.rank = ctx->rank;
    g.M = grid->map.max_lvl;
    g.pad = (int32_t)std::max<uint32_t>(1, prm->neighborhood_length);
    grid->n_local = part_count(g.part, ctx->rank);
    grid->first_local = grid->n_local ? part_first(g.part, ctx->rank) : 0;
    if (grid->n_local) {
        g.lo = grid->first_local - 1;
        g.hi = g.lo + grid->n_local;
        const int64_t cs = (int64_t)(g.lo / g.S), ce = (int64_t)((g.hi - 1) / g.S);
        g.cbase = cs - g.pad;
        g.nslices = (uint64_t)(ce - cs + 1 + 2 * g.pad);
        grid->n_slots = g.nslices * g.S;
    }
    Hood h;
    h.id = DCCRGX_DEFAULT_NEIGHBORHOOD_ID;
    default_items(prm->neighborhood_length, h.items);
    grid->hoods[h.id] = h;
    DX_TRY(build_hood(grid.get(), grid->hoods[h.id]));
    *out = grid.release();
    return DCCRGX_OK;
}

extern "C" {

int dccrgx_get_process(const dccrgx_grid* grid, const uint64_t* cells, size_t n, int32_t* out)
{
    DX_CHECK(grid && (cells || !n) && (out || !n), DCCRGX_EINVAL, "null argument");
    DX_TRY(explicit_host_leaves(grid));
    for (size_t i = 0; i < n; i++) {
        const uint64_t c = cells[i];
        if (grid->hy) {
            out[i] = hybrid_slot(grid, c) >= 0 ? 0 : -1;
            continue;
        }
        if (grid->uniform) {
            out[i] = (c >= 1 && c <= grid->g.N) ? level0_owner(grid, grid->g.part, c) : -1;
            continue;
        }
        const Explicit* E = grid->ex;
        const int64_t g = E->find(c);
        out[i] = g < 0 ? -1 : E->one_rank ? 0 : E->owner[g];
    }
    return DCCRGX_OK;
}

int dccrgx_grid_destroy(dccrgx_grid* grid)
{
    if (!grid) return DCCRGX_OK;
    hipSetDevice(grid->ctx->device);
    hipStreamSynchronize(grid->ctx->compute);
    hipStreamSynchronize(grid->ctx->comm);
    for (auto& kv : grid->hoods) free_hood(kv.second);
    for (Field& f : grid->fields) dx_free(f.ptr);
    for (auto& b : grid->spare_bufs) dx_free(b.first);
    dx_free(grid->d_sfc_cut);
    hybrid_destroy(grid);
    if (!grid->uniform) explicit_destroy(grid);
    delete grid->spare_host;
    amr_destroy(grid);
    load_state_free(grid);
    hipEventDestroy(grid->t0);
    hipEventDestroy(grid->t1);
    delete grid;
    dx_cache_trim();  // the grid's memory goes back to the device (torch or the user may need it)
    return DCCRGX_OK;
}

int dccrgx_grid_get_info(const dccrgx_grid* grid, dccrgx_grid_info* out)
{
    DX_CHECK(grid && out, DCCRGX_EINVAL, "null argument");
    std::memset(out, 0, sizeof(*out));
    out->n_local = grid->hy ? hybrid_n_local(grid) : grid->n_local;
    out->first_local = grid->first_local;
    out->n_slots = grid->n_slots;
    out->max_ref_lvl = grid->map.max_lvl;
    out->uniform = grid->hy ? 2 : grid->uniform ? 1 : 0;  // 2: uniform layout with refined cells (hybrid.hip)
    out->rank = grid->ctx->rank;
    out->comm_size = grid->ctx->comm_size;
    if (grid->uniform) {
        out->layout[0] = grid->g.LA;
        out->layout[1] = grid->g.LB;
        out->layout[2] = grid->g.nslices;
        out->layout[3] = (uint64_t)grid->g.pad;
    }
    return DCCRGX_OK;
}

int dccrgx_add_neighborhood(dccrgx_grid* grid, int32_t id, const int32_t* items, size_t n)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    // dccrg.hpp:6505-6618
    DX_CHECK(id != DCCRGX_DEFAULT_NEIGHBORHOOD_ID, DCCRGX_EINVAL, "default neighborhood id");
    DX_CHECK(!find_hood(grid, id), DCCRGX_EINVAL, "neighborhood %d exists", id);
    DX_CHECK(items || n == 0, DCCRGX_EINVAL, "null items");
    const uint32_t hl = grid->params.neighborhood_length;
    for (size_t k = 0; k < n; k++) {
        const int32_t* it = items + 3 * k;
        if (hl > 0) {
            for (int d = 0; d < 3; d++)
                DX_CHECK((uint32_t)std::abs(it[d]) <= hl, DCCRGX_EINVAL,
                         "item beyond neighborhood length");
            DX_CHECK(it[0] || it[1] || it[2], DCCRGX_EINVAL, "zero item");
        } else {
            int zeros = 0;
            for (int d = 0; d < 3; d++) {
                zeros += it[d] == 0;
                DX_CHECK(std::abs(it[d]) <= 1, DCCRGX_EINVAL, "item beyond face neighborhood");
            }
            DX_CHECK(zeros == 2, DCCRGX_EINVAL, "not a face item");
        }
    }
    Hood h;
    h.id = id;
    h.items.assign(items, items + 3 * n);
    grid->hoods[id] = h;
    const int s = grid->uniform ? build_hood(grid, grid->hoods[id])
                                : explicit_build_hood(grid, grid->hoods[id]);
    if (s != DCCRGX_OK) {
        free_hood(grid->hoods[id]);
        grid->hoods.erase(id);
    }
    return s;
}

int dccrgx_remove_neighborhood(dccrgx_grid* grid, int32_t id)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    if (id == DCCRGX_DEFAULT_NEIGHBORHOOD_ID) return DCCRGX_OK;  // dccrg.hpp:6685-6687
    Hood* h = find_hood(grid, id);
    if (h) {
        hipStreamSynchronize(grid->ctx->compute);
        hipStreamSynchronize(grid->ctx->comm);
        free_hood(*h);
        grid->hoods.erase(id);
    }
    return DCCRGX_OK;
}

int dccrgx_get_neighborhood(const dccrgx_grid* grid, int32_t id, int32_t* items, size_t cap,
                            size_t* n)
{
    DX_CHECK(grid && n, DCCRGX_EINVAL, "null argument");
    const Hood* h = find_hood(grid, id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", id);
    *n = h->items.size() / 3;
    DX_CHECK(cap >= *n && (items || *n == 0), DCCRGX_ERANGE, "capacity %zu < %zu", cap, *n);
    if (*n) std::memcpy(items, h->items.data(), h->items.size() * sizeof(int32_t));
    return DCCRGX_OK;
}

int dccrgx_get_all_cells(const dccrgx_grid* grid, uint64_t* ids, size_t cap, size_t* n)
{
    DX_CHECK(grid && n, DCCRGX_EINVAL, "null argument");
    DX_TRY(explicit_host_leaves(grid));
    if (!grid->uniform) {
        const std::vector<uint64_t>& L = grid->ex->leaves();
        *n = L.size();
        DX_CHECK(cap >= *n && (ids || !*n), DCCRGX_ERANGE, "capacity");
        std::copy(L.begin(), L.end(), ids);
        return DCCRGX_OK;
    }
    if (grid->hy) {  // one process: every leaf is local
        std::vector<uint64_t> v;
        DX_TRY(hybrid_local_cells(grid, v));
        *n = v.size();
        DX_CHECK(cap >= *n && (ids || !*n), DCCRGX_ERANGE, "capacity");
        std::copy(v.begin(), v.end(), ids);
        return DCCRGX_OK;
    }
    *n = grid->g.N;
    DX_CHECK(cap >= *n && (ids || !*n), DCCRGX_ERANGE, "capacity");
    parallel_ranges(*n, 1u << 16, [ids](size_t b, size_t e) {
        for (size_t i = b; i < e; i++) ids[i] = i + 1;
    });
    return DCCRGX_OK;
}

int dccrgx_get_cells(const dccrgx_grid* grid, int32_t id, int32_t which, uint64_t* ids, size_t cap,
                     size_t* n)
{
    DX_CHECK(grid && n, DCCRGX_EINVAL, "null argument");
    DX_TRY(explicit_host_leaves(grid));
    const Hood* h = find_hood(grid, id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", id);
    if (!grid->uniform) return explicit_get_cells(grid, *h, which, ids, cap, n);
    if (grid->hy) {  // one process: local = inner = every leaf, no outer or remote cells
        if (which == DCCRGX_CELLS_OUTER || which == DCCRGX_CELLS_REMOTE) {
            *n = 0;
            return DCCRGX_OK;
        }
        DX_CHECK(which == DCCRGX_CELLS_LOCAL || which == DCCRGX_CELLS_INNER, DCCRGX_EINVAL, "unknown cell class %d",
                 which);
        std::vector<uint64_t> v;
        DX_TRY(hybrid_local_cells(grid, v));
        *n = v.size();
        DX_CHECK(cap >= *n && (ids || !*n), DCCRGX_ERANGE, "capacity");
        std::copy(v.begin(), v.end(), ids);
        return DCCRGX_OK;
    }
    const uint64_t nl = grid->n_local;
    switch (which) {
    case DCCRGX_CELLS_LOCAL:
        *n = nl;
        DX_CHECK(cap >= *n && (ids || !*n), DCCRGX_ERANGE, "capacity");
        for (uint64_t i = 0; i < nl; i++) ids[i] = grid->first_local + i;
        return DCCRGX_OK;
    case DCCRGX_CELLS_OUTER:
        *n = h->outer.size();
        DX_CHECK(cap >= *n && (ids || !*n), DCCRGX_ERANGE, "capacity");
        std::copy(h->outer.begin(), h->outer.end(), ids);
        return DCCRGX_OK;
    case DCCRGX_CELLS_REMOTE:
        *n = h->remote.size();
        DX_CHECK(cap >= *n && (ids || !*n), DCCRGX_ERANGE, "capacity");
        std::copy(h->remote.begin(), h->remote.end(), ids);
        return DCCRGX_OK;
    case DCCRGX_CELLS_INNER: {
        *n = nl - h->outer.size();
        DX_CHECK(cap >= *n && (ids || !*n), DCCRGX_ERANGE, "capacity");
        size_t w = 0, j = 0;
        for (uint64_t i = 0; i < nl; i++) {
            const uint64_t c = grid->first_local + i;
            while (j < h->outer.size() && h->outer[j] < c) j++;
            if (j < h->outer.size() && h->outer[j] == c) continue;
            ids[w++] = c;
        }
        return DCCRGX_OK;
    }
    default:
        return set_error(DCCRGX_EINVAL, "unknown cell class %d", which);
    }
}

int dccrgx_neighbor_list_stats(const dccrgx_grid* grid, int32_t id, uint64_t out[4])
{
    DX_CHECK(grid && out, DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    DX_TRY(explicit_host_leaves(grid));
    const Hood* h = find_hood(grid, id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", id);
    for (int k = 0; k < 4; k++) out[k] = 0;
    if (grid->uniform || !h->d_nof_row) return DCCRGX_OK;  // closed-form rows: nothing stored
    const uint64_t rows = h->n_rows, nl = grid->ex->n_local();
    uint64_t e[3] = {0, 0, 0};  // neighbors_of, neighbors_to, stencil entries
    hipStream_t st = grid->ctx->compute;
    DX_TRY(dx_d2h(grid->ctx, &e[0], h->d_nof_row + rows, 8, st));
    DX_TRY(dx_d2h(grid->ctx, &e[1], h->d_nto_row + rows, 8, st));
    if (h->d_st_row) DX_TRY(dx_d2h(grid->ctx, &e[2], h->d_st_row + nl, 8, st));
    out[0] = rows;
    out[1] = e[0];
    out[2] = e[1];
    out[3] = (rows + 1) * 8 + e[0] * (8 + 12 + 4)  // neighbors_of: rows, ids, offsets, leaf indices
             + (rows + 1) * 8 + e[1] * 4           // neighbors_to: rows, leaf indices
             + (h->d_st_row ? (nl + 1) * 8 + e[2] * (4 + 12) : 0);  // stencil rows: slots, offsets
    return DCCRGX_OK;
}

int dccrgx_get_peers(const dccrgx_grid* grid, int32_t id, int32_t send, int32_t* peers,
                     uint64_t* counts, size_t cap, size_t* n)
{
    DX_CHECK(grid && n, DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    const Hood* h = find_hood(grid, id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", id);
    size_t w = 0;
    for (const PeerPlan& p : h->peers) {
        const auto& v = send ? p.send_ids : p.recv_ids;
        if (v.empty()) continue;
        if (w < cap) {
            if (peers) peers[w] = p.peer;
            if (counts) counts[w] = v.size();
        }
        w++;
    }
    *n = w;
    DX_CHECK(w <= cap, DCCRGX_ERANGE, "capacity %zu < %zu", cap, w);
    return DCCRGX_OK;
}

int dccrgx_get_peer_cells(const dccrgx_grid* grid, int32_t id, int32_t send, int32_t peer,
                          uint64_t* ids, size_t cap, size_t* n)
{
    DX_CHECK(grid && n, DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    DX_TRY(explicit_host_leaves(grid));
    const Hood* h = find_hood(grid, id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", id);
    *n = 0;
    for (const PeerPlan& p : h->peers) {
        if (p.peer != peer) continue;
        const auto& v = send ? p.send_ids : p.recv_ids;
        *n = v.size();
        DX_CHECK(cap >= *n && (ids || !*n), DCCRGX_ERANGE, "capacity");
        std::copy(v.begin(), v.end(), ids);
    }
    return DCCRGX_OK;
}

}  // extern "C"
