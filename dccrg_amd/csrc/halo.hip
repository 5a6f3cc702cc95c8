// halo.hip -- device SoA field pools and the remote-neighbor halo exchange.
//
// Replaces the reference transfer engine (dccrg.hpp:10726-11209): instead of
// one MPI struct datatype per peer built from every boundary cell's
// get_mpi_datatype(), each registered field is moved as one contiguous RCCL
// message per peer (field-major, cells in ascending id order as in
// dccrg.hpp:8822-8826).  When the per-peer cell run is contiguous in the
// slab layout the message is sent from / received into the field itself
// (no pack, no unpack); otherwise a gather / scatter kernel stages it.
#include <algorithm>
#include <atomic>
#include <cstring>

#include "grid.hpp"

namespace dccrgx {

static unsigned grid_for(uint64_t n)
{
    uint64_t g = (n + 255) / 256;
    if (g > 256 * 16) g = 256 * 16;
    if (g == 0) g = 1;
    return (unsigned)g;
}

// dst[i*E .. ] = src[idx[i]*E ..], elements of E bytes (E multiple of 4 or any)
template <class T>
__global__ void __launch_bounds__(256) k_gather(const T* __restrict__ src, const uint64_t* __restrict__ idx,
                                                uint64_t n, uint32_t words, T* __restrict__ dst)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const uint64_t tot = n * words;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += stride) {
        const uint64_t c = i / words, w = i - c * words;
        dst[i] = src[idx[c] * words + w];
    }
}

// dst[didx[i]*E ..] = src[sidx ? sidx[i] : i]
template <class T>
__global__ void __launch_bounds__(256) k_scatter(const T* __restrict__ src, const uint64_t* __restrict__ sidx,
                                                 const uint64_t* __restrict__ didx, uint64_t n,
                                                 uint32_t words, T* __restrict__ dst)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const uint64_t tot = n * words;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += stride) {
        const uint64_t c = i / words, w = i - c * words;
        const uint64_t s = sidx ? sidx[c] : c;
        dst[didx[c] * words + w] = src[s * words + w];
    }
}

static int launch_gather(const void* src, const uint64_t* idx, uint64_t n, uint32_t elem, void* dst,
                         hipStream_t st)
{
    if (n == 0) return DCCRGX_OK;
    if (elem % 4 == 0)
        hipLaunchKernelGGL(k_gather<uint32_t>, dim3(grid_for(n * (elem / 4))), dim3(256), 0, st,
                           (const uint32_t*)src, idx, n, elem / 4, (uint32_t*)dst);
    else
        hipLaunchKernelGGL(k_gather<uint8_t>, dim3(grid_for(n * elem)), dim3(256), 0, st,
                           (const uint8_t*)src, idx, n, elem, (uint8_t*)dst);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

static int launch_scatter(const void* src, const uint64_t* sidx, const uint64_t* didx, uint64_t n,
                          uint32_t elem, void* dst, hipStream_t st)
{
    if (n == 0) return DCCRGX_OK;
    if (elem % 4 == 0)
        hipLaunchKernelGGL(k_scatter<uint32_t>, dim3(grid_for(n * (elem / 4))), dim3(256), 0, st,
                           (const uint32_t*)src, sidx, didx, n, elem / 4, (uint32_t*)dst);
    else
        hipLaunchKernelGGL(k_scatter<uint8_t>, dim3(grid_for(n * elem)), dim3(256), 0, st,
                           (const uint8_t*)src, sidx, didx, n, elem, (uint8_t*)dst);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

int launch_gather_ext(const void* src, const uint64_t* idx, uint64_t n, uint32_t elem, void* dst,
                      hipStream_t st)
{
    return launch_gather(src, idx, n, elem, dst, st);
}

int launch_scatter_ext(const void* src, const uint64_t* sidx, const uint64_t* didx, uint64_t n,
                       uint32_t elem, void* dst, hipStream_t st)
{
    return launch_scatter(src, sidx, didx, n, elem, dst, st);
}

static int check_fields(const dccrgx_grid* g, const int32_t* f, size_t nf, size_t* bytes_per_cell)
{
    DX_CHECK(f || nf == 0, DCCRGX_EINVAL, "null field list");
    size_t b = 0;
    for (size_t i = 0; i < nf; i++) {
        DX_CHECK(f[i] >= 0 && (size_t)f[i] < g->fields.size(), DCCRGX_EINVAL, "bad field %d", f[i]);
        b += g->fields[f[i]].elem;
    }
    if (bytes_per_cell) *bytes_per_cell = b;
    return DCCRGX_OK;
}

// ---- variable-size fields: byte segments ------------------------------------
using Seg = ByteSeg;

static std::atomic<uint64_t> g_var_epoch{0};
uint64_t next_var_epoch() { return ++g_var_epoch; }

// 16 lanes per segment (four segments per wavefront: cells of a few elements
// are the common case); each group copies in the widest unit its segment's
// addresses and length allow
__global__ void __launch_bounds__(256) k_seg_copy(const Seg* __restrict__ segs, uint64_t n,
                                                  const char* __restrict__ src, char* __restrict__ dst)
{
    constexpr uint32_t G = 16;
    const uint64_t grp = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    const uint32_t lane = threadIdx.x % G;
    const uint64_t groups = (uint64_t)gridDim.x * blockDim.x / G;
    for (uint64_t k = grp; k < n; k += groups) {
        const Seg sg = segs[k];
        const char* a = src + sg.src;
        char* b = dst + sg.dst;
        const uint64_t al = (uint64_t)(uintptr_t)a | (uint64_t)(uintptr_t)b | sg.len;
        if ((al & 15) == 0) {
            for (uint64_t i = lane; i < sg.len / 16; i += G) ((uint4*)b)[i] = ((const uint4*)a)[i];
        } else if ((al & 7) == 0) {
            for (uint64_t i = lane; i < sg.len / 8; i += G) ((uint2*)b)[i] = ((const uint2*)a)[i];
        } else if ((al & 3) == 0) {
            for (uint64_t i = lane; i < sg.len / 4; i += G) ((uint32_t*)b)[i] = ((const uint32_t*)a)[i];
        } else {
            for (uint64_t i = lane; i < sg.len; i += G) b[i] = a[i];
        }
    }
}

static int launch_segs(const Seg* d, uint64_t n, const void* src, void* dst, hipStream_t st)
{
    if (!n) return DCCRGX_OK;
    const uint64_t blocks = std::min<uint64_t>((n + 15) / 16, 4096);
    hipLaunchKernelGGL(k_seg_copy, dim3((unsigned)blocks), dim3(256), 0, st, d, n, (const char*)src, (char*)dst);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

// one-off copies from host-built segments (cell-addressed access, resize)
static int seg_copy(const std::vector<Seg>& segs, const void* src, void* dst, hipStream_t st)
{
    if (segs.empty()) return DCCRGX_OK;
    Seg* d = nullptr;
    DX_HIP(dx_malloc(&d, segs.size() * sizeof(Seg)));
    DX_HIP(hipMemcpyAsync(d, segs.data(), segs.size() * sizeof(Seg), hipMemcpyHostToDevice, st));
    DX_TRY(launch_segs(d, segs.size(), src, dst, st));
    DX_HIP(hipStreamSynchronize(st));
    dx_free(d);
    return DCCRGX_OK;
}

// the cached plan of field fid in `plans`, (re)built by `build` when the
// field's counts changed since
template <class Build>
static int var_plan(dccrgx_grid* g, VarPlans& plans, int32_t fid, Build build, const VarPlan** out)
{
    const Field& F = g->fields[fid];
    VarPlan& P = plans[fid];
    if (P.epoch != F.epoch || !F.epoch) {
        std::vector<Seg> segs;
        uint64_t bytes = 0;
        build(F, segs, bytes);
        dx_free(P.d);  // deferred past the work queued on the library's streams
        P = VarPlan{};
        if (!segs.empty()) {
            DX_HIP(dx_malloc(&P.d, segs.size() * sizeof(Seg)));
            DX_TRY(dx_h2d(g->ctx, P.d, segs.data(), segs.size() * sizeof(Seg), g->ctx->compute));
        }
        P.n = segs.size();
        P.bytes = bytes;
        P.epoch = F.epoch;
    }
    *out = &P;
    return DCCRGX_OK;
}

// first ghost slot of each message cell of peer p
static std::vector<int64_t> first_dst(const PeerPlan& p)
{
    std::vector<int64_t> first(p.recv_ids.size(), -1);
    for (size_t k = 0; k < p.h_unpack_src.size(); k++)
        if (first[p.h_unpack_src[k]] < 0) first[p.h_unpack_src[k]] = (int64_t)p.h_unpack_dst[k];
    return first;
}

// pack plan: cells ascending, each its count[] elements, packed back to back
static int send_plan(dccrgx_grid* g, PeerPlan& p, int32_t fid, const VarPlan** out)
{
    return var_plan(g, p.var_send, fid, [&](const Field& F, std::vector<Seg>& segs, uint64_t& bytes) {
        uint64_t o = 0;
        for (uint64_t s : p.h_send_slots) {
            const uint64_t len = (uint64_t)F.count[s] * F.elem;
            if (len) segs.push_back({F.off[s], o, len});
            o += len;
        }
        bytes = o;
    }, out);
}

// unpack plan: message cell j has the count of its ghost slots (pre-sized by
// the caller); every ghost slot filled from it gets a copy
static int recv_plan(dccrgx_grid* g, PeerPlan& p, int32_t fid, const VarPlan** out)
{
    return var_plan(g, p.var_recv, fid, [&](const Field& F, std::vector<Seg>& segs, uint64_t& bytes) {
        const uint64_t n = p.recv_ids.size();
        const std::vector<int64_t> first = first_dst(p);
        std::vector<uint64_t> pre(n + 1, 0);
        for (uint64_t j = 0; j < n; j++)
            pre[j + 1] = pre[j] + (first[j] >= 0 ? (uint64_t)F.count[first[j]] * F.elem : 0);
        for (size_t k = 0; k < p.h_unpack_dst.size(); k++) {
            const uint64_t d = p.h_unpack_dst[k], j = p.h_unpack_src[k];
            const uint64_t len = std::min<uint64_t>((uint64_t)F.count[d] * F.elem, pre[j + 1] - pre[j]);
            if (len) segs.push_back({pre[j], F.off[d], len});
        }
        bytes = pre[n];
    }, out);
}

// bytes field fid contributes to the message to (send) or from (recv) peer p
static int field_bytes(dccrgx_grid* g, int32_t fid, PeerPlan& p, bool send, size_t* bytes)
{
    const Field& F = g->fields[fid];
    if (!F.variable) {
        *bytes = (send ? p.send_ids.size() : p.recv_ids.size()) * F.elem;
        return DCCRGX_OK;
    }
    const VarPlan* P = nullptr;
    DX_TRY(send ? send_plan(g, p, fid, &P) : recv_plan(g, p, fid, &P));
    *bytes = P->bytes;
    return DCCRGX_OK;
}

static int message_bytes(dccrgx_grid* g, PeerPlan& p, const int32_t* f, size_t nf, bool send, size_t* bytes)
{
    size_t b = 0;
    for (size_t i = 0; i < nf; i++) {
        size_t x = 0;
        DX_TRY(field_bytes(g, f[i], p, send, &x));
        b += x;
    }
    *bytes = b;
    return DCCRGX_OK;
}

static int ensure(void** p, size_t* have, size_t need)
{
    if (*have >= need) return DCCRGX_OK;
    dx_free(*p);
    *p = nullptr;
    *have = 0;
    DX_HIP(dx_malloc(p, need));
    *have = need;
    return DCCRGX_OK;
}

// periodic self copies into pad slots (stream st)
static int self_copy(dccrgx_grid* g, Hood& h, const int32_t* f, size_t nf, hipStream_t st)
{
    for (size_t i = 0; i < nf; i++) {
        const Field& F = g->fields[f[i]];
        if (F.variable) {
            const VarPlan* P = nullptr;
            DX_TRY(var_plan(g, h.var_self, f[i], [&](const Field& G, std::vector<Seg>& segs, uint64_t& bytes) {
                for (auto& e : h.h_self)
                    if (G.count[e.second])
                        segs.push_back({G.off[e.second], G.off[e.first], (uint64_t)G.count[e.second] * G.elem});
                bytes = 0;
            }, &P));
            DX_TRY(launch_segs(P->d, P->n, F.ptr, F.ptr, st));
            continue;
        }
        for (const CopySeg& s : h.self_segs)
            DX_HIP(hipMemcpyAsync((char*)F.ptr + s.dst * F.elem, (char*)F.ptr + s.src * F.elem,
                                  s.n * F.elem, hipMemcpyDeviceToDevice, st));
        DX_TRY(launch_scatter(F.ptr, h.d_self_src, h.d_self_dst, h.n_self_scatter, F.elem, F.ptr, st));
    }
    return DCCRGX_OK;
}

// message layout per peer: field-major, cells ascending
static int pack_peer(dccrgx_grid* g, PeerPlan& p, const int32_t* f, size_t nf, void* dst,
                     hipStream_t st)
{
    const uint64_t n = p.send_ids.size();
    size_t off = 0;
    for (size_t i = 0; i < nf; i++) {
        const Field& F = g->fields[f[i]];
        char* d = (char*)dst + off;
        if (F.variable) {  // cells ascending, each its count[] elements
            const VarPlan* P = nullptr;
            DX_TRY(send_plan(g, p, f[i], &P));
            DX_TRY(launch_segs(P->d, P->n, F.ptr, d, st));
            off += P->bytes;
            continue;
        }
        if (p.send_direct)
            DX_HIP(hipMemcpyAsync(d, (char*)F.ptr + p.send_slot0 * F.elem, n * F.elem,
                                  hipMemcpyDeviceToDevice, st));
        else
            DX_TRY(launch_gather(F.ptr, p.d_send_slots, n, F.elem, d, st));
        off += n * F.elem;
    }
    return DCCRGX_OK;
}

static int unpack_peer(dccrgx_grid* g, PeerPlan& p, const int32_t* f, size_t nf, const void* src,
                       hipStream_t st)
{
    const uint64_t n = p.recv_ids.size();
    size_t off = 0;
    for (size_t i = 0; i < nf; i++) {
        const Field& F = g->fields[f[i]];
        const char* s = (const char*)src + off;
        if (F.variable) {
            const VarPlan* P = nullptr;
            DX_TRY(recv_plan(g, p, f[i], &P));
            DX_TRY(launch_segs(P->d, P->n, s, F.ptr, st));
            off += P->bytes;
            continue;
        }
        if (p.recv_direct)
            DX_HIP(hipMemcpyAsync((char*)F.ptr + p.recv_slot0 * F.elem, s, n * F.elem,
                                  hipMemcpyDeviceToDevice, st));
        else
            DX_TRY(launch_scatter(s, p.d_unpack_src, p.d_unpack_dst, p.n_unpack, F.elem, F.ptr, st));
        off += n * F.elem;
    }
    return DCCRGX_OK;
}

// remote cell lin -> first storage slot holding it (or -1)
__host__ __device__ inline int64_t ghost_slot(const UGeom& g, uint64_t lin)
{
    const uint64_t c = divide(lin, g.dS);
    const uint64_t rem = lin - c * g.S;
    const int64_t c0 = g.cbase, c1 = g.cbase + (int64_t)g.nslices;
    if (!g.perC) {
        if ((int64_t)c >= c0 && (int64_t)c < c1) return (int64_t)(rem + g.S * (uint64_t)((int64_t)c - c0));
        return -1;
    }
    // smallest unwrapped copy c + k*LC >= c0
    int64_t cu = (int64_t)c;
    const int64_t LC = (int64_t)g.LC;
    if (cu < c0) cu += ((c0 - cu + LC - 1) / LC) * LC;
    else cu -= ((cu - c0) / LC) * LC;
    if (cu < c1) return (int64_t)(rem + g.S * (uint64_t)(cu - c0));
    return -1;
}

__global__ void __launch_bounds__(256) k_slots_of(UGeom g, const uint64_t* __restrict__ ids, size_t n,
                                                  int64_t* __restrict__ slots)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t id = ids[i];
        int64_t s = -1;
        if (id >= 1 && id <= g.N) {
            const uint64_t lin = id - 1;
            if (ug_local(g, lin)) s = (int64_t)(lin + (uint64_t)(-g.cbase * (int64_t)g.S));
            else s = ghost_slot(g, lin);
        }
        slots[i] = s;
    }
}

int explicit_slots_of(const dccrgx_grid* grid, const uint64_t* ids, size_t n, int64_t* slots,
                      hipStream_t st);
int64_t explicit_host_slot(const dccrgx_grid* grid, uint64_t id);

// every storage slot holding cell `id` (a uniform grid's periodic images in
// the pad slices included), ascending
static void slots_holding(const dccrgx_grid* grid, uint64_t id, std::vector<uint64_t>& out)
{
    out.clear();
    if (!grid->uniform) {
        const int64_t s = explicit_host_slot(grid, id);
        if (s >= 0) out.push_back((uint64_t)s);
        return;
    }
    const UGeom& g = grid->g;
    if (id < 1 || id > g.N) return;
    const uint64_t lin = id - 1, c = lin / g.S, rem = lin - c * g.S;
    const int64_t c0 = g.cbase, c1 = g.cbase + (int64_t)g.nslices, LC = (int64_t)g.LC;
    int64_t cu = (int64_t)c;
    if (g.perC) {
        if (cu < c0) cu += ((c0 - cu + LC - 1) / LC) * LC;
        else cu -= ((cu - c0) / LC) * LC;
    }
    for (; cu < c1; cu += LC) {
        if (cu >= c0) out.push_back(rem + g.S * (uint64_t)(cu - c0));
        if (!g.perC) break;
    }
}

// the slot read and written for a cell: its own slot if local, else its
// first ghost copy; -1 if this rank stores no copy
static int64_t primary_slot(const dccrgx_grid* grid, uint64_t id)
{
    if (grid->hy) return hybrid_slot(grid, id);
    if (!grid->uniform) return explicit_host_slot(grid, id);
    const UGeom& g = grid->g;
    if (id < 1 || id > g.N) return -1;
    if (ug_local(g, id - 1)) return (int64_t)(id - 1 + (uint64_t)(-g.cbase * (int64_t)g.S));
    return ghost_slot(g, id - 1);
}

int64_t host_primary_slot(const dccrgx_grid* grid, uint64_t id) { return primary_slot(grid, id); }

// One whole update through the host-staged transport (dccrgx_ctx_set_host_transport):
// pack every peer's message on the compute stream (after the queued work),
// copy the messages to host memory, one exchange() call, copy back, unpack.
// Complete on return, so the wait calls have nothing left to do.
static int host_exchange(dccrgx_grid* g, Hood& h, const int32_t* f, size_t nf)
{
    Ctx* c = g->ctx;
    hipStream_t st = c->compute;
    std::vector<int32_t> sp, rp;
    std::vector<const void*> sb;
    std::vector<void*> rb;
    std::vector<uint64_t> sn, rn;
    for (PeerPlan& p : h.peers) {
        if (!p.send_ids.empty()) {
            size_t b = 0;
            DX_TRY(message_bytes(g, p, f, nf, true, &b));
            p.h_send_msg.resize(std::max<size_t>(b, 1));
            if (b) {
                DX_TRY(ensure(&p.d_send_buf, &p.send_buf_bytes, b));
                DX_TRY(pack_peer(g, p, f, nf, p.d_send_buf, st));
                DX_TRY(dx_d2h(c, p.h_send_msg.data(), p.d_send_buf, b, st));
            }
            sp.push_back(p.peer);
            sb.push_back(p.h_send_msg.data());
            sn.push_back(b);
        }
        if (!p.recv_ids.empty()) {
            size_t b = 0;
            DX_TRY(message_bytes(g, p, f, nf, false, &b));
            p.h_recv_msg.resize(std::max<size_t>(b, 1));
            rp.push_back(p.peer);
            rb.push_back(p.h_recv_msg.data());
            rn.push_back(b);
        }
    }
    const int r = c->host_tx.exchange(c->host_tx.user, (int32_t)sp.size(), sp.data(), sb.data(), sn.data(),
                                      (int32_t)rp.size(), rp.data(), rb.data(), rn.data());
    DX_CHECK(r == 0, DCCRGX_ERCCL, "host transport: exchange returned %d", r);
    size_t k = 0;
    for (PeerPlan& p : h.peers) {
        if (p.recv_ids.empty()) continue;
        const size_t b = rn[k++];
        if (!b) continue;
        DX_TRY(ensure(&p.d_recv_buf, &p.recv_buf_bytes, b));
        DX_TRY(dx_h2d(c, p.d_recv_buf, p.h_recv_msg.data(), b, st));
        DX_TRY(unpack_peer(g, p, f, nf, p.d_recv_buf, st));
    }
    return DCCRGX_OK;
}

static int halo_finish(dccrgx_grid* grid, Hood& h, const int32_t* f, size_t nf)
{
    bool var = false;
    for (size_t i = 0; i < nf; i++) var |= grid->fields[f[i]].variable;
    for (PeerPlan& p : h.peers)
        if ((var || !p.recv_direct) && !p.recv_ids.empty())
            DX_TRY(unpack_peer(grid, p, f, nf, p.d_recv_buf, grid->ctx->compute));
    return DCCRGX_OK;
}

}  // namespace dccrgx

using namespace dccrgx;

extern "C" {

int dccrgx_field_create(dccrgx_grid* grid, uint32_t elem, int32_t* fid)
{
    DX_NOT_PENDING(grid);
    DX_CHECK(grid && fid && elem > 0, DCCRGX_EINVAL, "bad argument");
    DX_HIP(hipSetDevice(grid->ctx->device));
    Field F;
    F.elem = elem;
    const size_t bytes = std::max<uint64_t>(grid->n_slots, 1) * elem;
    DX_HIP(dx_malloc(&F.ptr, bytes));
    // ghost slots of cells outside the grid stay zero forever; default-constructed
    // (value-initialised) ghosts as in allocate_copies_of_remote_neighbors, dccrg.hpp:7153-7184
    DX_HIP(hipMemsetAsync(F.ptr, 0, bytes, grid->ctx->compute));
    DX_HIP(hipStreamSynchronize(grid->ctx->compute));
    grid->fields.push_back(F);
    *fid = (int32_t)grid->fields.size() - 1;
    return DCCRGX_OK;
}

int dccrgx_field_device_ptr(const dccrgx_grid* grid, int32_t fid, void** ptr, uint64_t* n_slots)
{
    DX_CHECK(grid && fid >= 0 && (size_t)fid < grid->fields.size(), DCCRGX_EINVAL, "bad field");
    if (ptr) *ptr = grid->fields[fid].ptr;
    if (n_slots) *n_slots = grid->n_slots;
    return DCCRGX_OK;
}

int dccrgx_slots_of(const dccrgx_grid* grid, const uint64_t* ids, size_t n, int64_t* slots, void* stream)
{
    DX_CHECK(grid && (n == 0 || (ids && slots)), DCCRGX_EINVAL, "bad argument");
    hipStream_t st = stream ? (hipStream_t)stream : grid->ctx->compute;
    if (n == 0) return DCCRGX_OK;
    const CallerStream fence(grid->ctx, st);
    if (grid->hy) {  // on the host (refined cells are few; the ids come back in one copy)
        std::vector<uint64_t> h(n);
        std::vector<int64_t> o(n);
        DX_HIP(hipMemcpyAsync(h.data(), ids, n * 8, hipMemcpyDeviceToHost, st));
        DX_HIP(hipStreamSynchronize(st));
        for (size_t i = 0; i < n; i++) o[i] = hybrid_slot(grid, h[i]);
        DX_HIP(hipMemcpyAsync(slots, o.data(), n * 8, hipMemcpyHostToDevice, st));
        DX_HIP(hipStreamSynchronize(st));
        return DCCRGX_OK;
    }
    if (!grid->uniform) return explicit_slots_of(grid, ids, n, slots, st);
    if (grid->n_local == 0) return set_error(DCCRGX_ESTATE, "rank has no cells");
    hipLaunchKernelGGL(k_slots_of, dim3(grid_for(n)), dim3(256), 0, st, grid->g, ids, n, slots);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

// local cells occupy one contiguous slot run in both layouts
static uint64_t local_slot0(const dccrgx_grid* grid)
{
    if (!grid->uniform) return 0;
    return grid->g.lo + (uint64_t)(-grid->g.cbase * (int64_t)grid->g.S);
}

int dccrgx_field_write_local(dccrgx_grid* grid, int32_t fid, const void* host, size_t n)
{
    DX_NOT_PENDING(grid);
    DX_CHECK(grid && fid >= 0 && (size_t)fid < grid->fields.size(), DCCRGX_EINVAL, "bad field");
    DX_CHECK(!grid->fields[fid].variable, DCCRGX_EINVAL, "variable-size field: use dccrgx_field_write_cells");
    if (grid->hy) {
        DX_CHECK(n == hybrid_n_local(grid) && (host || !n), DCCRGX_EINVAL, "expected %llu local values",
                 (unsigned long long)hybrid_n_local(grid));
        return hybrid_local_copy(grid, grid->fields[fid], const_cast<void*>(host), true);
    }
    DX_CHECK(n == grid->n_local && (host || !n), DCCRGX_EINVAL, "expected %llu local values",
             (unsigned long long)grid->n_local);
    if (!n) return DCCRGX_OK;
    const Field& F = grid->fields[fid];
    if (!grid->uniform) return explicit_local_copy(grid, F, const_cast<void*>(host), true);
    return dx_h2d(grid->ctx, (char*)F.ptr + local_slot0(grid) * F.elem, host, n * F.elem, grid->ctx->compute);
}

int dccrgx_field_read_local(const dccrgx_grid* grid, int32_t fid, void* host, size_t n)
{
    DX_CHECK(grid && fid >= 0 && (size_t)fid < grid->fields.size(), DCCRGX_EINVAL, "bad field");
    DX_CHECK(!grid->fields[fid].variable, DCCRGX_EINVAL, "variable-size field: use dccrgx_field_read_cells");
    if (grid->hy) {
        DX_CHECK(n == hybrid_n_local(grid) && (host || !n), DCCRGX_EINVAL, "expected %llu local values",
                 (unsigned long long)hybrid_n_local(grid));
        return hybrid_local_copy(grid, grid->fields[fid], host, false);
    }
    DX_CHECK(n == grid->n_local && (host || !n), DCCRGX_EINVAL, "expected %llu local values",
             (unsigned long long)grid->n_local);
    if (!n) return DCCRGX_OK;
    const Field& F = grid->fields[fid];
    if (!grid->uniform) return explicit_local_copy(grid, F, host, false);
    return dx_d2h(grid->ctx, host, (char*)F.ptr + local_slot0(grid) * F.elem, n * F.elem, grid->ctx->compute);
}

int dccrgx_field_read_remote(const dccrgx_grid* grid, int32_t hood_id, int32_t fid, void* host,
                             size_t n)
{
    DX_CHECK(grid && fid >= 0 && (size_t)fid < grid->fields.size(), DCCRGX_EINVAL, "bad field");
    DX_NO_HYBRID(grid);
    DX_CHECK(!grid->fields[fid].variable, DCCRGX_EINVAL, "variable-size field: use dccrgx_field_read_cells");
    const Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    DX_CHECK(n == h->remote.size() && (host || !n), DCCRGX_EINVAL, "expected %zu remote values",
             h->remote.size());
    if (!n) return DCCRGX_OK;
    hipStream_t st = grid->ctx->compute;
    const Field& F = grid->fields[fid];
    uint64_t* d_ids = nullptr;
    int64_t* d_slots = nullptr;
    void* d_out = nullptr;
    DX_HIP(dx_malloc(&d_ids, n * 8));
    DX_HIP(dx_malloc(&d_slots, n * 8));
    DX_HIP(dx_malloc(&d_out, n * F.elem));
    DX_TRY(dx_h2d(grid->ctx, d_ids, h->remote.data(), n * 8, st));
    DX_TRY(dccrgx_slots_of(grid, d_ids, n, d_slots, st));
    DX_TRY(launch_gather(F.ptr, (const uint64_t*)d_slots, n, F.elem, d_out, st));
    DX_TRY(dx_d2h(grid->ctx, host, d_out, n * F.elem, st));
    dx_free(d_ids);
    dx_free(d_slots);
    dx_free(d_out);
    return DCCRGX_OK;
}

int dccrgx_halo_self(dccrgx_grid* grid, int32_t hood_id, const int32_t* f, size_t nf)
{
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    DX_NO_HYBRID(grid);
    DX_NOT_PENDING(grid);
    Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    DX_TRY(check_fields(grid, f, nf, nullptr));
    return self_copy(grid, *h, f, nf, grid->ctx->compute);
}

int dccrgx_halo_start(dccrgx_grid* grid, int32_t hood_id, const int32_t* f, size_t nf)
{
    DX_NOT_PENDING(grid);
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    Hood* h = find_hood(grid, hood_id);
    // the reference returns false for unknown ids (dccrg.hpp:5055-5060)
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    DX_CHECK(!h->pending, DCCRGX_ESTATE, "halo of neighborhood %d already started", hood_id);
    size_t bpc = 0;
    DX_TRY(check_fields(grid, f, nf, &bpc));
    Ctx* c = grid->ctx;
    DX_TRY(self_copy(grid, *h, f, nf, c->compute));
    bool any = false;
    for (const PeerPlan& p : h->peers) any |= !p.send_ids.empty() || !p.recv_ids.empty();
    if (!any) return DCCRGX_OK;
    if (!c->has_comm && c->has_host_tx) return host_exchange(grid, *h, f, nf);
    DX_CHECK(c->has_comm, DCCRGX_ESTATE,
             "rank %d has remote neighbors but no RCCL communicator (dccrgx_ctx_comm_init)", c->rank);
    // the comm stream starts after everything queued so far on the compute stream
    DX_HIP(hipEventRecord(c->ev_compute, c->compute));
    DX_HIP(hipStreamWaitEvent(c->comm, c->ev_compute, 0));
    bool var = false;
    for (size_t i = 0; i < nf; i++) var |= grid->fields[f[i]].variable;
    for (PeerPlan& p : h->peers) {
        if ((var || !p.send_direct) && !p.send_ids.empty()) {
            size_t b = 0;
            DX_TRY(message_bytes(grid, p, f, nf, true, &b));
            DX_TRY(ensure(&p.d_send_buf, &p.send_buf_bytes, std::max<size_t>(b, 1)));
            DX_TRY(pack_peer(grid, p, f, nf, p.d_send_buf, c->comm));
        }
        if ((var || !p.recv_direct) && !p.recv_ids.empty()) {
            size_t b = 0;
            DX_TRY(message_bytes(grid, p, f, nf, false, &b));
            DX_TRY(ensure(&p.d_recv_buf, &p.recv_buf_bytes, std::max<size_t>(b, 1)));
        }
    }
    // grouped point-to-point: one message per field per peer (xGMI links are
    // point-to-point; z-slab peers are the ring neighbours)
    DX_RCCL(ncclGroupStart());
    for (PeerPlan& p : h->peers) {
        size_t soff = 0, roff = 0;
        for (size_t i = 0; i < nf; i++) {
            const Field& F = grid->fields[f[i]];
            size_t sb = 0, rb = 0;
            DX_TRY(field_bytes(grid, f[i], p, true, &sb));
            DX_TRY(field_bytes(grid, f[i], p, false, &rb));
            if (sb) {
                const void* src = p.send_direct && !var ? (const char*)F.ptr + p.send_slot0 * F.elem
                                                        : (const char*)p.d_send_buf + soff;
                DX_RCCL(ncclSend(src, sb, ncclUint8, p.peer, c->nccl, c->comm));
            }
            if (rb) {
                void* dst = p.recv_direct && !var ? (char*)F.ptr + p.recv_slot0 * F.elem
                                                  : (char*)p.d_recv_buf + roff;
                DX_RCCL(ncclRecv(dst, rb, ncclUint8, p.peer, c->nccl, c->comm));
            }
            soff += sb;
            roff += rb;
        }
    }
    DX_RCCL(ncclGroupEnd());
    DX_HIP(hipEventRecord(c->ev_comm, c->comm));
    h->pending = true;
    h->pending_fields.assign(f, f + nf);
    return DCCRGX_OK;
}

int dccrgx_halo_wait(dccrgx_grid* grid, int32_t hood_id, int32_t which)
{
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    DX_CHECK(which >= DCCRGX_WAIT_ALL && which <= DCCRGX_WAIT_SENDS, DCCRGX_EINVAL, "bad selector");
    if (!h->pending) return DCCRGX_OK;
    Ctx* c = grid->ctx;
    // sends and receives of one RCCL group complete together: any wait
    // completes both (dccrg.hpp:5307-5413 semantics are preserved: after a
    // receive wait the ghosts are current, after a send wait the sent cells
    // may be modified)
    DX_HIP(hipStreamWaitEvent(c->compute, c->ev_comm, 0));
    h->pending = false;
    return halo_finish(grid, *h, h->pending_fields.data(), h->pending_fields.size());
}

int dccrgx_halo_update(dccrgx_grid* grid, int32_t hood_id, const int32_t* f, size_t nf)
{
    DX_TRY(dccrgx_halo_start(grid, hood_id, f, nf));
    return dccrgx_halo_wait(grid, hood_id, DCCRGX_WAIT_ALL);
}

int dccrgx_exchange_start(dccrgx_grid* grid, int32_t hood_id, const void* const* send_host,
                          const uint64_t* send_bytes, void* const* recv_host, const uint64_t* recv_bytes)
{
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    DX_NO_HYBRID(grid);
    DX_NOT_PENDING(grid);
    Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    DX_CHECK(!h->pending, DCCRGX_ESTATE, "transfer of neighborhood %d already started", hood_id);
    Ctx* c = grid->ctx;
    size_t si = 0, ri = 0;
    bool any = false;
    struct Msg { PeerPlan* p; size_t sb, rb; const void* sh; void* rh; };
    std::vector<Msg> msgs;
    for (PeerPlan& p : h->peers) {
        Msg m{&p, 0, 0, nullptr, nullptr};
        if (!p.send_ids.empty()) {
            m.sb = send_bytes[si];
            m.sh = send_host[si++];
        }
        if (!p.recv_ids.empty()) {
            m.rb = recv_bytes[ri];
            m.rh = recv_host[ri++];
        }
        any |= m.sb || m.rb;
        msgs.push_back(m);
    }
    if (!any) return DCCRGX_OK;
    if (!c->has_comm && c->has_host_tx) {  // host-resident payloads: straight to the transport
        std::vector<int32_t> sp, rp;
        std::vector<const void*> sb;
        std::vector<void*> rb;
        std::vector<uint64_t> sn, rn;
        for (Msg& m : msgs) {
            if (!m.p->send_ids.empty()) {
                sp.push_back(m.p->peer);
                sb.push_back(m.sh);
                sn.push_back(m.sb);
            }
            if (!m.p->recv_ids.empty()) {
                rp.push_back(m.p->peer);
                rb.push_back(m.rh);
                rn.push_back(m.rb);
            }
        }
        const int r = c->host_tx.exchange(c->host_tx.user, (int32_t)sp.size(), sp.data(), sb.data(), sn.data(),
                                          (int32_t)rp.size(), rp.data(), rb.data(), rn.data());
        DX_CHECK(r == 0, DCCRGX_ERCCL, "host transport: exchange returned %d", r);
        return DCCRGX_OK;
    }
    DX_CHECK(c->has_comm, DCCRGX_ESTATE, "rank %d has remote neighbors but no RCCL communicator", c->rank);
    for (Msg& m : msgs) {
        if (m.sb) {
            DX_TRY(ensure(&m.p->d_send_buf, &m.p->send_buf_bytes, m.sb));
            DX_HIP(hipMemcpyAsync(m.p->d_send_buf, m.sh, m.sb, hipMemcpyHostToDevice, c->comm));
        }
        if (m.rb) DX_TRY(ensure(&m.p->d_recv_buf, &m.p->recv_buf_bytes, m.rb));
    }
    DX_RCCL(ncclGroupStart());
    for (Msg& m : msgs) {
        if (m.sb) DX_RCCL(ncclSend(m.p->d_send_buf, m.sb, ncclUint8, m.p->peer, c->nccl, c->comm));
        if (m.rb) DX_RCCL(ncclRecv(m.p->d_recv_buf, m.rb, ncclUint8, m.p->peer, c->nccl, c->comm));
    }
    DX_RCCL(ncclGroupEnd());
    for (Msg& m : msgs)
        if (m.rb) DX_HIP(hipMemcpyAsync(m.rh, m.p->d_recv_buf, m.rb, hipMemcpyDeviceToHost, c->comm));
    h->pending = true;
    h->pending_fields.clear();
    return DCCRGX_OK;
}

int dccrgx_exchange_wait(dccrgx_grid* grid, int32_t hood_id)
{
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    DX_NO_HYBRID(grid);
    Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    if (!h->pending) return DCCRGX_OK;
    DX_HIP(hipStreamSynchronize(grid->ctx->comm));
    h->pending = false;
    return DCCRGX_OK;
}

int dccrgx_halo_pack_to(dccrgx_grid* grid, int32_t hood_id, const int32_t* f, size_t nf, int32_t peer,
                        void* dst, size_t cap, size_t* bytes)
{
    DX_CHECK(grid && bytes, DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    DX_NOT_PENDING(grid);
    Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    size_t bpc = 0;
    DX_TRY(check_fields(grid, f, nf, &bpc));
    *bytes = 0;
    for (PeerPlan& p : h->peers) {
        if (p.peer != peer) continue;
        DX_TRY(message_bytes(grid, p, f, nf, true, bytes));
        DX_CHECK(cap >= *bytes, DCCRGX_ERANGE, "capacity %zu < %zu", cap, *bytes);
        DX_TRY(pack_peer(grid, p, f, nf, dst, grid->ctx->compute));
    }
    return DCCRGX_OK;
}

int dccrgx_halo_unpack_from(dccrgx_grid* grid, int32_t hood_id, const int32_t* f, size_t nf,
                            int32_t peer, const void* src, size_t bytes)
{
    DX_CHECK(grid, DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    DX_NOT_PENDING(grid);
    Hood* h = find_hood(grid, hood_id);
    DX_CHECK(h, DCCRGX_ENOTFOUND, "no neighborhood %d", hood_id);
    size_t bpc = 0;
    DX_TRY(check_fields(grid, f, nf, &bpc));
    for (PeerPlan& p : h->peers) {
        if (p.peer != peer) continue;
        size_t want = 0;
        DX_TRY(message_bytes(grid, p, f, nf, false, &want));
        DX_CHECK(bytes == want, DCCRGX_EINVAL, "message is %zu bytes, expected %zu", bytes, want);
        DX_TRY(unpack_peer(grid, p, f, nf, src, grid->ctx->compute));
        return DCCRGX_OK;
    }
    DX_CHECK(bytes == 0, DCCRGX_EINVAL, "no receives from peer %d", peer);
    return DCCRGX_OK;
}

// ---- variable-size cell data and cell-addressed access -----------------------

int dccrgx_field_create_variable(dccrgx_grid* grid, uint32_t elem, int32_t* fid)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid && fid && elem > 0, DCCRGX_EINVAL, "bad argument");
    Field F;
    F.elem = elem;
    F.variable = true;
    F.count.assign(grid->n_slots, 0);
    F.off.assign(grid->n_slots, 0);
    F.pool_bytes = 0;
    F.epoch = next_var_epoch();
    DX_HIP(dx_malloc(&F.ptr, 16));
    grid->fields.push_back(std::move(F));
    *fid = (int32_t)grid->fields.size() - 1;
    return DCCRGX_OK;
}

int dccrgx_field_resize(dccrgx_grid* grid, int32_t fid, const uint64_t* ids, const uint32_t* counts, size_t n)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid && fid >= 0 && (size_t)fid < grid->fields.size(), DCCRGX_EINVAL, "bad field");
    DX_CHECK((ids && counts) || !n, DCCRGX_EINVAL, "null argument");
    Field& F = grid->fields[fid];
    DX_CHECK(F.variable, DCCRGX_EINVAL, "field %d has a fixed size per cell", fid);
    std::vector<uint32_t> cnt = F.count;
    std::vector<uint64_t> s;
    for (size_t i = 0; i < n; i++) {
        slots_holding(grid, ids[i], s);
        DX_CHECK(!s.empty(), DCCRGX_ENOTFOUND, "cell %llu is neither local nor a ghost here",
                 (unsigned long long)ids[i]);
        for (uint64_t x : s) cnt[x] = counts[i];
    }
    std::vector<uint64_t> off(cnt.size());
    uint64_t tot = 0;
    for (size_t k = 0; k < cnt.size(); k++) {
        off[k] = tot;
        tot += (uint64_t)cnt[k] * F.elem;
        tot = (tot + 7) & ~7ull;  // 8-byte aligned cells
    }
    hipStream_t st = grid->ctx->compute;
    void* pool = nullptr;
    DX_HIP(dx_malloc(&pool, std::max<uint64_t>(tot, 16)));
    DX_HIP(hipMemsetAsync(pool, 0, std::max<uint64_t>(tot, 16), st));  // new elements value-initialised
    std::vector<Seg> keep;
    for (size_t k = 0; k < cnt.size(); k++) {
        const uint64_t len = (uint64_t)std::min(cnt[k], F.count[k]) * F.elem;
        if (len) keep.push_back({F.off[k], off[k], len});
    }
    DX_TRY(seg_copy(keep, F.ptr, pool, st));
    DX_HIP(hipStreamSynchronize(st));
    dx_free(F.ptr);
    F.ptr = pool;
    F.pool_bytes = tot;
    F.count.swap(cnt);
    F.off.swap(off);
    F.epoch = next_var_epoch();
    return DCCRGX_OK;
}

int dccrgx_field_get_counts(const dccrgx_grid* grid, int32_t fid, const uint64_t* ids, size_t n, uint32_t* counts)
{
    DX_CHECK(grid && fid >= 0 && (size_t)fid < grid->fields.size(), DCCRGX_EINVAL, "bad field");
    DX_CHECK((ids && counts) || !n, DCCRGX_EINVAL, "null argument");
    const Field& F = grid->fields[fid];
    for (size_t i = 0; i < n; i++) {
        const int64_t s = primary_slot(grid, ids[i]);
        DX_CHECK(s >= 0, DCCRGX_ENOTFOUND, "cell %llu is neither local nor a ghost here", (unsigned long long)ids[i]);
        counts[i] = F.variable ? F.count[s] : 1;
    }
    return DCCRGX_OK;
}

// segments between a packed host-order buffer and the cells' storage
static int cell_segments(const dccrgx_grid* grid, const Field& F, const uint64_t* ids, size_t n, bool to_cells,
                         std::vector<Seg>& segs, uint64_t* total)
{
    uint64_t o = 0;
    for (size_t i = 0; i < n; i++) {
        const int64_t s = primary_slot(grid, ids[i]);
        DX_CHECK(s >= 0, DCCRGX_ENOTFOUND, "cell %llu is neither local nor a ghost here", (unsigned long long)ids[i]);
        const uint64_t len = F.variable ? (uint64_t)F.count[s] * F.elem : F.elem;
        const uint64_t at = F.variable ? F.off[s] : (uint64_t)s * F.elem;
        if (len) segs.push_back(to_cells ? Seg{o, at, len} : Seg{at, o, len});
        o += len;
    }
    *total = o;
    return DCCRGX_OK;
}

int dccrgx_field_write_cells(dccrgx_grid* grid, int32_t fid, const uint64_t* ids, size_t n, const void* data,
                             size_t bytes)
{
    DX_NOT_PENDING(grid);
    DX_CHECK(grid && fid >= 0 && (size_t)fid < grid->fields.size(), DCCRGX_EINVAL, "bad field");
    DX_CHECK(ids || !n, DCCRGX_EINVAL, "null argument");
    const Field& F = grid->fields[fid];
    std::vector<Seg> segs;
    uint64_t tot = 0;
    DX_TRY(cell_segments(grid, F, ids, n, true, segs, &tot));
    DX_CHECK(bytes == tot && (data || !tot), DCCRGX_EINVAL, "%zu bytes given, the cells hold %llu", bytes,
             (unsigned long long)tot);
    if (!tot) return DCCRGX_OK;
    hipStream_t st = grid->ctx->compute;
    void* d = nullptr;
    DX_HIP(dx_malloc(&d, tot));
    DX_HIP(hipMemcpyAsync(d, data, tot, hipMemcpyHostToDevice, st));
    const int s = seg_copy(segs, d, F.ptr, st);
    dx_free(d);
    return s;
}

int dccrgx_field_read_cells(const dccrgx_grid* grid, int32_t fid, const uint64_t* ids, size_t n, void* data,
                            size_t cap, size_t* bytes)
{
    DX_CHECK(grid && bytes && fid >= 0 && (size_t)fid < grid->fields.size(), DCCRGX_EINVAL, "bad argument");
    DX_CHECK(ids || !n, DCCRGX_EINVAL, "null argument");
    const Field& F = grid->fields[fid];
    std::vector<Seg> segs;
    uint64_t tot = 0;
    DX_TRY(cell_segments(grid, F, ids, n, false, segs, &tot));
    *bytes = tot;
    if (!data) return DCCRGX_OK;  // size query
    DX_CHECK(cap >= tot, DCCRGX_ERANGE, "capacity %zu < %llu", cap, (unsigned long long)tot);
    if (!tot) return DCCRGX_OK;
    hipStream_t st = grid->ctx->compute;
    void* d = nullptr;
    DX_HIP(dx_malloc(&d, tot));
    int s = seg_copy(segs, F.ptr, d, st);
    if (s == DCCRGX_OK) {
        DX_HIP(hipMemcpyAsync(data, d, tot, hipMemcpyDeviceToHost, st));
        DX_HIP(hipStreamSynchronize(st));
    }
    dx_free(d);
    return s;
}

}  // extern "C"

