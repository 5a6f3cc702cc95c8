// core.hip -- errors, context, mapping parameters and the batched id<->index
// mapping kernels (dccrg_mapping.hpp re-designed for gfx950: one lane per id,
// magic-number 64-bit division, no loops over levels beyond a branch-free
// compare chain).
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstring>
#include <condition_variable>
#include <exception>
#include <deque>
#include <mutex>
#include <unordered_map>

#include "internal.hpp"

namespace dccrgx {

static thread_local char g_err[1024] = "";

int set_error(int code, const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

void dx_slow_note(const char* what, size_t bytes, double ms)
{
    static const bool on = [] {
        const char* e = std::getenv("DCCRGX_TIMING");
        return e && *e && *e != '0';
    }();
    if (on) std::fprintf(stderr, "[dccrgx] slow %s %zu bytes %.3f ms\n", what, bytes, ms);
}

static int stage_reserve(Ctx* c, size_t bytes)
{
    if (c->stage_bytes >= bytes) return DCCRGX_OK;
    // geometric growth (pinning is slow), at least 4 MiB, at most one chunk
    size_t want = std::min<size_t>(std::max<size_t>({bytes, 2 * c->stage_bytes, 4u << 20}), 64ull << 20);
    if (c->stage) DX_HIP(hipHostFree(c->stage));
    c->stage = nullptr;
    c->stage_dev = nullptr;
    c->stage_bytes = 0;
    // coherent: the gather kernel's stores reach host memory without a cache flush
    DX_HIP(hipHostMalloc(&c->stage, want, hipHostMallocMapped | hipHostMallocCoherent));
    c->stage_bytes = want;
    DX_HIP(hipHostGetDevicePointer(&c->stage_dev, c->stage, 0));
    return DCCRGX_OK;
}

constexpr size_t STAGE_CHUNK = 64ull << 20;

// host copy to / from the pinned stage; large ones split over the host threads
// (one thread copies ~10 GB/s, the leaf list of a 3.5 M-leaf grid is 28 MB)
static void stage_copy(void* dst, const void* src, size_t k)
{
    if (k < (2u << 20)) {
        std::memcpy(dst, src, k);
        return;
    }
    parallel_ranges(k, 1u << 20, [dst, src](size_t b, size_t e) {
        std::memcpy((char*)dst + b, (const char*)src + b, e - b);
    });
}

int dx_h2d(Ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st)
{
    if (!bytes) return DCCRGX_OK;
    DX_TRY(stage_reserve(c, std::min(bytes, STAGE_CHUNK)));
    for (size_t off = 0; off < bytes; off += STAGE_CHUNK) {
        const size_t k = std::min(STAGE_CHUNK, bytes - off);
        stage_copy(c->stage, (const char*)src + off, k);
        DX_HIP(hipMemcpyAsync((char*)dst + off, c->stage, k, hipMemcpyHostToDevice, st));
        DX_HIP(hipStreamSynchronize(st));
    }
    return DCCRGX_OK;
}

int dx_h2d_async(Ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st)
{
    if (!bytes) return DCCRGX_OK;
    if (bytes > Ctx::UP_SLOT_BYTES || st != c->compute) return dx_h2d(c, dst, src, bytes, st);
    if (!c->up) {
        DX_HIP(hipHostMalloc((void**)&c->up, Ctx::UP_SLOTS * Ctx::UP_SLOT_BYTES, hipHostMallocDefault));
        for (int k = 0; k < Ctx::UP_SLOTS; k++) DX_HIP(hipEventCreateWithFlags(&c->up_ev[k], hipEventDisableTiming));
    }
    const int k = c->up_next;
    c->up_next = (k + 1) % Ctx::UP_SLOTS;
    if (c->up_used[k]) DX_HIP(hipEventSynchronize(c->up_ev[k]));  // its previous copy has been read
    char* slot = c->up + (size_t)k * Ctx::UP_SLOT_BYTES;
    std::memcpy(slot, src, bytes);
    DX_HIP(hipMemcpyAsync(dst, slot, bytes, hipMemcpyHostToDevice, st));
    DX_HIP(hipEventRecord(c->up_ev[k], st));
    c->up_used[k] = true;
    return DCCRGX_OK;
}

struct FillArgs {
    uint8_t* p[8];
    uint64_t bytes[8];
    uint32_t word[8];  // the value byte replicated
};

// blockIdx.y: the range; 4-byte stores over the aligned middle, bytes at the ends
__global__ void __launch_bounds__(256) k_fill_many(FillArgs a)
{
    const int r = blockIdx.y;
    uint8_t* p = a.p[r];
    const uint64_t n = a.bytes[r];
    const uint64_t head = std::min<uint64_t>(n, (4 - ((uintptr_t)p & 3)) & 3);
    const uint64_t words = (n - head) / 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t* w = reinterpret_cast<uint32_t*>(p + head);
    for (uint64_t i = t0; i < words; i += stride) w[i] = a.word[r];
    if (t0 < head) p[t0] = (uint8_t)a.word[r];
    const uint64_t tail = head + words * 4;
    if (t0 < n - tail) p[tail + t0] = (uint8_t)a.word[r];
}

int dx_fill_many(const Fill* v, int n, hipStream_t st)
{
    DX_CHECK(n >= 0 && n <= 8, DCCRGX_EINTERNAL, "dx_fill_many: %d ranges", n);
    FillArgs a{};
    uint64_t most = 0;
    int m = 0;
    for (int i = 0; i < n; i++) {
        if (!v[i].bytes) continue;
        a.p[m] = (uint8_t*)v[i].p;
        a.bytes[m] = v[i].bytes;
        a.word[m] = 0x01010101u * v[i].value;
        most = std::max<uint64_t>(most, v[i].bytes / 4 + 4);
        m++;
    }
    if (!m) return DCCRGX_OK;
    const unsigned gx = (unsigned)std::min<uint64_t>((most + 255) / 256, 2048);
    hipLaunchKernelGGL(k_fill_many, dim3(gx, m), dim3(256), 0, st, a);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

constexpr int GATHER_RANGES = 16;
constexpr size_t GATHER_MAX = 1u << 20;

struct GatherArgs {
    const uint8_t* src[GATHER_RANGES];
    uint8_t* dst[GATHER_RANGES];  // in the pinned stage (device address)
    uint64_t bytes[GATHER_RANGES];
};

// blockIdx.y: the range; 4-byte loads / stores when both ends and the size
// allow, bytes otherwise (read-backs of counters and short id lists)
__global__ void __launch_bounds__(256) k_gather_d2h(GatherArgs a)
{
    const int r = blockIdx.y;
    const uint8_t* s = a.src[r];
    uint8_t* d = a.dst[r];
    const uint64_t n = a.bytes[r];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if ((((uintptr_t)s | (uintptr_t)d | n) & 3) == 0) {
        const uint32_t* s4 = reinterpret_cast<const uint32_t*>(s);
        uint32_t* d4 = reinterpret_cast<uint32_t*>(d);
        for (uint64_t i = t0; i < n / 4; i += stride) d4[i] = s4[i];
    } else {
        for (uint64_t i = t0; i < n; i += stride) d[i] = s[i];
    }
}

int dx_d2h_many(Ctx* c, const D2H* v, size_t n, hipStream_t st)
{
    size_t total = 0, nz = 0, most = 0;
    for (size_t i = 0; i < n; i++) {
        total += (v[i].bytes + 15) & ~(size_t)15;
        nz += v[i].bytes ? 1 : 0;
        most = std::max(most, v[i].bytes);
    }
    if (!total) return DCCRGX_OK;
    if (total > STAGE_CHUNK) {  // large: one at a time
        for (size_t i = 0; i < n; i++) DX_TRY(dx_d2h(c, v[i].dst, v[i].src, v[i].bytes, st));
        return DCCRGX_OK;
    }
    DX_TRY(stage_reserve(c, total));
    size_t at = 0;
    if (total <= GATHER_MAX && nz <= (size_t)GATHER_RANGES && c->stage_dev) {
        GatherArgs a{};
        int m = 0;
        for (size_t i = 0; i < n; i++) {
            if (v[i].bytes) {
                a.src[m] = static_cast<const uint8_t*>(v[i].src);
                a.dst[m] = static_cast<uint8_t*>(c->stage_dev) + at;
                a.bytes[m] = v[i].bytes;
                m++;
            }
            at += (v[i].bytes + 15) & ~(size_t)15;
        }
        const unsigned gx = (unsigned)std::min<uint64_t>((most / 4 + 255) / 256 + 1, 256);
        hipLaunchKernelGGL(k_gather_d2h, dim3(gx, m), dim3(256), 0, st, a);
        DX_HIP(hipGetLastError());
    } else {
        for (size_t i = 0; i < n; i++) {
            if (v[i].bytes)
                DX_HIP(hipMemcpyAsync((char*)c->stage + at, v[i].src, v[i].bytes, hipMemcpyDeviceToHost, st));
            at += (v[i].bytes + 15) & ~(size_t)15;
        }
    }
    DX_HIP(hipStreamSynchronize(st));
    at = 0;
    for (size_t i = 0; i < n; i++) {
        if (v[i].bytes) std::memcpy(v[i].dst, (const char*)c->stage + at, v[i].bytes);
        at += (v[i].bytes + 15) & ~(size_t)15;
    }
    return DCCRGX_OK;
}

__global__ void __launch_bounds__(256) k_ident(uint32_t* __restrict__ out, uint64_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = (uint32_t)i;
}

int ctx_identity(Ctx* c, uint64_t n, uint32_t** out, hipStream_t st)
{
    if (n > c->ident_n || !c->ident) {
        const uint64_t cap = std::max<uint64_t>({n + n / 4, 2 * c->ident_n, 1024});
        uint32_t* d = nullptr;
        DX_HIP(dx_malloc(&d, cap * 4));
        hipLaunchKernelGGL(k_ident, dim3((unsigned)std::min<uint64_t>((cap + 255) / 256, 65536)), dim3(256), 0, st, d,
                           cap);
        DX_HIP(hipGetLastError());
        // other streams read it only after this one (the structural calls end in a synchronisation)
        if (c->ident) c->ident_old.push_back(c->ident);
        c->ident = d;
        c->ident_n = cap;
    }
    *out = c->ident;
    return DCCRGX_OK;
}

bool ctx_is_identity(const Ctx* c, const void* p)
{
    if (!p) return false;
    if (p == c->ident) return true;
    for (const uint32_t* q : c->ident_old)
        if (p == q) return true;
    return false;
}

int dx_d2h(Ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st)
{
    if (!bytes) return DCCRGX_OK;
    DX_TRY(stage_reserve(c, std::min(bytes, STAGE_CHUNK)));
    for (size_t off = 0; off < bytes; off += STAGE_CHUNK) {
        const size_t k = std::min(STAGE_CHUNK, bytes - off);
        DX_HIP(hipMemcpyAsync(c->stage, (const char*)src + off, k, hipMemcpyDeviceToHost, st));
        DX_HIP(hipStreamSynchronize(st));
        stage_copy((char*)dst + off, c->stage, k);
    }
    return DCCRGX_OK;
}

// dccrg_mapping.hpp:317-330 (double arithmetic, as the reference)
int max_possible_level(const uint64_t length[3])
{
    const uint64_t grid_length = length[0] * length[1] * length[2];
    int lvl = 0;
    double current_last = 0;
    while (current_last <= double(~uint64_t(0))) {
        current_last += double(grid_length) * std::pow(8.0, double(lvl));
        lvl++;
    }
    return lvl - 2;
}

int make_map_params(const dccrgx_mapping* m, MapParams* out)
{
    DX_CHECK(m && out, DCCRGX_EINVAL, "null mapping");
    DX_CHECK(m->length[0] && m->length[1] && m->length[2], DCCRGX_EINVAL,
             "all lengths must be > 0 (dccrg_length.hpp:97-110)");
    const int maxp = max_possible_level(m->length);
    int M = m->max_ref_lvl < 0 ? maxp : m->max_ref_lvl;
    DX_CHECK(M <= maxp && M < MAX_LEVELS - 2, DCCRGX_EINVAL,
             "maximum refinement level %d exceeds the possible %d", M, maxp);
    MapParams p{};
    std::memcpy(p.length, m->length, sizeof(p.length));
    p.max_lvl = M;
    p.nlevel0 = m->length[0] * m->length[1] * m->length[2];
    uint64_t first = 1;
    for (int l = 0; l < MAX_LEVELS; l++) {
        p.first_id[l] = first;
        if (l <= M) first += p.nlevel0 * ((uint64_t)1 << (3 * l));
    }
    p.last_cell = p.first_id[M + 1] - 1;  // update_last_cell, dccrg_mapping.hpp:679-687
    p.div_lx = make_divider(m->length[0]);
    p.div_lxly = make_divider(m->length[0] * m->length[1]);
    *out = p;
    return DCCRGX_OK;
}

Partition make_partition(uint64_t total, int comm_size)
{
    Partition P{};
    P.total = total;
    P.comm_size = comm_size;
    const uint64_t cs = (uint64_t)comm_size;
    if (total < cs) P.cpp = 1;
    else if (total % cs > 0) P.cpp = total / cs + 1;
    else P.cpp = total / cs;
    P.fewer = P.cpp * cs - total;
    P.split = P.fewer * (P.cpp - 1);
    P.div_cpp = make_divider(P.cpp);
    P.div_cpp1 = make_divider(P.cpp > 1 ? P.cpp - 1 : 1);
    return P;
}

// ---------------------------------------------------------------------------
// mapping kernels
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_ids_to_indices(MapParams p, const uint64_t* __restrict__ ids,
                                                        size_t n, uint64_t* __restrict__ idx3,
                                                        int32_t* __restrict__ lvl)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t o[3];
        int l;
        map_indices(p, ids[i], o, &l);
        if (idx3) {
            idx3[3 * i + 0] = o[0];
            idx3[3 * i + 1] = o[1];
            idx3[3 * i + 2] = o[2];
        }
        if (lvl) lvl[i] = l;
    }
}

// Same results, block-contiguous, U ids per lane per pass: the U loads of a
// lane are issued together, the 3*256*U (x, y, z) triples are staged in LDS
// and leave as one contiguous run of 16-byte non-temporal stores (the triples
// are 24 B apart, so per-lane stores of k_ids_to_indices only fill a third of
// each wave's store span).  U = 2 won the sweep over U = 1, 4, 8
// (profiles/r2_map_variant_sweep.log); k_ids_to_indices takes unaligned outputs.
template <int U>
__global__ void __launch_bounds__(256) k_ids_to_indices_u(MapParams p, const uint64_t* __restrict__ ids,
                                                          size_t n, uint64_t* __restrict__ idx3,
                                                          int32_t* __restrict__ lvl)
{
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    constexpr int B = 256 * U;
    __shared__ uint64_t s[3 * B];
    for (size_t base = (size_t)blockIdx.x * B; base < n; base += (size_t)gridDim.x * B) {
        uint64_t c[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t i = base + k * 256 + threadIdx.x;
            c[k] = i < n ? __builtin_nontemporal_load(ids + i) : 0;
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t i = base + k * 256 + threadIdx.x;
            uint64_t o[3] = {0, 0, 0};
            int l = -1;
            if (i < n) {
                map_indices(p, c[k], o, &l);
                if (lvl) __builtin_nontemporal_store(l, lvl + i);
            }
            const int j = k * 256 + threadIdx.x;
            s[3 * j + 0] = o[0];
            s[3 * j + 1] = o[1];
            s[3 * j + 2] = o[2];
        }
        __syncthreads();
        const size_t cnt = 3 * (n - base < (size_t)B ? n - base : (size_t)B);
        if (cnt == 3 * (size_t)B) {
            u64x2* dst = (u64x2*)(idx3 + 3 * base);
            for (int k = threadIdx.x; k < 3 * B / 2; k += 256) {
                const u64x2 v = {s[2 * k], s[2 * k + 1]};
                __builtin_nontemporal_store(v, dst + k);
            }
        } else {
            for (size_t k = threadIdx.x; k < cnt; k += 256) idx3[3 * base + k] = s[k];
        }
        __syncthreads();
    }
}

// k_ids_to_indices_u with the next pass's ids loaded before this pass is
// computed and stored (one HBM round trip per pass was exposed: the stores
// of a pass wait for the LDS exchange, and the next loads waited for them),
// and the levels staged in LDS too, leaving as 16-byte stores
template <int U>
__global__ void __launch_bounds__(256) k_ids_to_indices_p(MapParams p, const uint64_t* __restrict__ ids,
                                                          size_t n, uint64_t* __restrict__ idx3,
                                                          int32_t* __restrict__ lvl)
{
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    constexpr int B = 256 * U;
    __shared__ __attribute__((aligned(16))) uint64_t s[3 * B];
    __shared__ __attribute__((aligned(16))) int32_t sl[B];
    const size_t step = (size_t)gridDim.x * B;
    size_t base = (size_t)blockIdx.x * B;
    uint64_t c[U];
#pragma unroll
    for (int k = 0; k < U; k++) {
        const size_t i = base + k * 256 + threadIdx.x;
        c[k] = i < n ? __builtin_nontemporal_load(ids + i) : 0;
    }
    for (; base < n; base += step) {
        uint64_t nx[U];
#pragma unroll
        for (int k = 0; k < U; k++) {  // the next pass's ids, in flight while this pass is finished
            const size_t i = base + step + k * 256 + threadIdx.x;
            nx[k] = i < n ? __builtin_nontemporal_load(ids + i) : 0;
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            uint64_t o[3] = {0, 0, 0};
            int l = -1;
            if (base + k * 256 + threadIdx.x < n) map_indices(p, c[k], o, &l);
            const int j = k * 256 + threadIdx.x;
            s[3 * j + 0] = o[0];
            s[3 * j + 1] = o[1];
            s[3 * j + 2] = o[2];
            sl[j] = l;
        }
        __syncthreads();
        const size_t cnt = n - base < (size_t)B ? n - base : (size_t)B;
        if (cnt == (size_t)B) {
            u64x2* dst = (u64x2*)(idx3 + 3 * base);
            for (int k = threadIdx.x; k < 3 * B / 2; k += 256) {
                const u64x2 v = {s[2 * k], s[2 * k + 1]};
                __builtin_nontemporal_store(v, dst + k);
            }
            if (lvl)
                for (int k = threadIdx.x; k < B / 4; k += 256) {
                    const i32x4 v = {sl[4 * k], sl[4 * k + 1], sl[4 * k + 2], sl[4 * k + 3]};
                    __builtin_nontemporal_store(v, (i32x4*)(lvl + base) + k);
                }
        } else {
            for (size_t k = threadIdx.x; k < 3 * cnt; k += 256) idx3[3 * base + k] = s[k];
            if (lvl)
                for (size_t k = threadIdx.x; k < cnt; k += 256) lvl[base + k] = sl[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < U; k++) c[k] = nx[k];
    }
}

__global__ void __launch_bounds__(256) k_indices_to_ids(MapParams p, const uint64_t* __restrict__ idx3,
                                                        const int32_t* __restrict__ lvl, size_t n,
                                                        uint64_t* __restrict__ ids)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t c[3] = {idx3[3 * i], idx3[3 * i + 1], idx3[3 * i + 2]};
        ids[i] = map_cell(p, c, lvl[i]);
    }
}

__global__ void __launch_bounds__(256) k_ids_op(MapParams p, int op, const uint64_t* __restrict__ ids,
                                                size_t n, uint64_t* __restrict__ out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t c = ids[i];
        uint64_t idx[3];
        int l;
        const bool ok = map_indices(p, c, idx, &l);
        uint64_t r = 0;
        switch (op) {
        case DCCRGX_OP_LENGTH_IN_INDICES:  // dccrg_mapping.hpp:298-311
            r = ok ? ((uint64_t)1 << (p.max_lvl - l)) : DCCRGX_ERROR_INDEX;
            break;
        case DCCRGX_OP_PARENT:  // dccrg_mapping.hpp:368-384
            r = !ok ? 0 : (l == 0 ? c : map_cell(p, idx, l - 1));
            break;
        case DCCRGX_OP_LEVEL_0_PARENT:  // dccrg_mapping.hpp:480-494
            r = !ok ? 0 : (l == 0 ? c : map_cell(p, idx, 0));
            break;
        case DCCRGX_OP_CHILD:  // dccrg_mapping.hpp:339-356
            r = !ok ? 0 : (l >= p.max_lvl ? c : map_cell(p, idx, l + 1));
            break;
        }
        out[i] = r;
    }
}

static unsigned grid_for(size_t n)
{
    size_t g = (n + 255) / 256;
    if (g > 256 * 16) g = 256 * 16;  // grid-stride beyond 16 blocks per CU
    if (g == 0) g = 1;
    return (unsigned)g;
}

}  // namespace dccrgx

using namespace dccrgx;

extern "C" {

const char* dccrgx_last_error(void) { return g_err; }
int dccrgx_version(void) { return DCCRGX_VERSION; }

int dccrgx_max_possible_refinement_level(const uint64_t length[3], int32_t* out)
{
    DX_CHECK(length && out, DCCRGX_EINVAL, "null argument");
    *out = max_possible_level(length);
    return DCCRGX_OK;
}

int dccrgx_last_cell(const dccrgx_mapping* map, uint64_t* out)
{
    MapParams p;
    DX_TRY(make_map_params(map, &p));
    *out = p.last_cell;
    return DCCRGX_OK;
}

int dccrgx_map_ids_to_indices(const dccrgx_mapping* map, const uint64_t* ids, size_t n,
                              uint64_t* idx3, int32_t* lvl, void* stream)
{
    MapParams p;
    DX_TRY(make_map_params(map, &p));
    if (n == 0) return DCCRGX_OK;
    DX_CHECK(ids, DCCRGX_EINVAL, "null ids");
    if (idx3 && ((uintptr_t)idx3 & 15) == 0 && ((uintptr_t)lvl & 15) == 0) {
        // one pass per workgroup up to 2^20 workgroups: 2^26 ids 0.475 -> 0.42 ms
        // against 2048 workgroups of 64 passes (tools/map_bench.py A/B,
        // profiles/s11_map_grid_ab.log); the pass prefetch serves larger n
        constexpr size_t per = 256 * 2;
        const unsigned g = (unsigned)std::max<size_t>(1, std::min<size_t>((n + per - 1) / per, 1u << 20));
        hipLaunchKernelGGL(k_ids_to_indices_p<2>, dim3(g), dim3(256), 0, (hipStream_t)stream, p, ids, n, idx3,
                           lvl);
    } else if (idx3 && ((uintptr_t)idx3 & 15) == 0) {
        constexpr size_t per = 256 * 2;
        const unsigned g = (unsigned)std::max<size_t>(1, std::min<size_t>((n + per - 1) / per, 256 * 8));
        hipLaunchKernelGGL(k_ids_to_indices_u<2>, dim3(g), dim3(256), 0, (hipStream_t)stream, p, ids, n, idx3,
                           lvl);
    } else
        hipLaunchKernelGGL(k_ids_to_indices, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, ids, n,
                           idx3, lvl);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

int dccrgx_map_indices_to_ids(const dccrgx_mapping* map, const uint64_t* idx3, const int32_t* lvl,
                              size_t n, uint64_t* ids, void* stream)
{
    MapParams p;
    DX_TRY(make_map_params(map, &p));
    if (n == 0) return DCCRGX_OK;
    DX_CHECK(idx3 && lvl && ids, DCCRGX_EINVAL, "null argument");
    hipLaunchKernelGGL(k_indices_to_ids, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p,
                       idx3, lvl, n, ids);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

int dccrgx_map_ids_op(const dccrgx_mapping* map, int op, const uint64_t* ids, size_t n,
                      uint64_t* out, void* stream)
{
    MapParams p;
    DX_TRY(make_map_params(map, &p));
    DX_CHECK(op >= 0 && op <= DCCRGX_OP_CHILD, DCCRGX_EINVAL, "unknown op %d", op);
    if (n == 0) return DCCRGX_OK;
    DX_CHECK(ids && out, DCCRGX_EINVAL, "null argument");
    hipLaunchKernelGGL(k_ids_op, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, op, ids,
                       n, out);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

int dccrgx_map_host_indices(const dccrgx_mapping* map, uint64_t cell, uint64_t idx3[3], int32_t* lvl)
{
    MapParams p;
    DX_TRY(make_map_params(map, &p));
    DX_CHECK(idx3, DCCRGX_EINVAL, "null output");
    int l;
    map_indices(p, cell, idx3, &l);
    if (lvl) *lvl = l;
    return DCCRGX_OK;
}

int dccrgx_map_host_cell(const dccrgx_mapping* map, const uint64_t idx3[3], int32_t lvl, uint64_t* cell)
{
    MapParams p;
    DX_TRY(make_map_params(map, &p));
    DX_CHECK(idx3 && cell, DCCRGX_EINVAL, "null argument");
    *cell = map_cell(p, idx3, lvl);
    return DCCRGX_OK;
}

}  // extern "C"

namespace dccrgx {
static uint64_t host_op(const MapParams& p, int op, uint64_t c)
{
    uint64_t idx[3];
    int l;
    const bool ok = map_indices(p, c, idx, &l);
    switch (op) {
    case DCCRGX_OP_LENGTH_IN_INDICES: return ok ? ((uint64_t)1 << (p.max_lvl - l)) : DCCRGX_ERROR_INDEX;
    case DCCRGX_OP_PARENT: return !ok ? 0 : (l == 0 ? c : map_cell(p, idx, l - 1));
    case DCCRGX_OP_LEVEL_0_PARENT: return !ok ? 0 : (l == 0 ? c : map_cell(p, idx, 0));
    default: return !ok ? 0 : (l >= p.max_lvl ? c : map_cell(p, idx, l + 1));
    }
}
}  // namespace dccrgx

extern "C" {

int dccrgx_map_host_op(const dccrgx_mapping* map, int op, uint64_t c, uint64_t* out)
{
    MapParams p;
    DX_TRY(make_map_params(map, &p));
    DX_CHECK(out && op >= 0 && op <= DCCRGX_OP_CHILD, DCCRGX_EINVAL, "bad argument");
    *out = host_op(p, op, c);
    return DCCRGX_OK;
}

int dccrgx_map_host_ids_to_indices(const dccrgx_mapping* map, const uint64_t* ids, size_t n, uint64_t* idx3,
                                   int32_t* lvl)
{
    MapParams p;
    DX_TRY(make_map_params(map, &p));
    DX_CHECK(ids || !n, DCCRGX_EINVAL, "null argument");
    for (size_t i = 0; i < n; i++) {
        uint64_t o[3];
        int l;
        map_indices(p, ids[i], o, &l);
        if (idx3) {
            idx3[3 * i] = o[0];
            idx3[3 * i + 1] = o[1];
            idx3[3 * i + 2] = o[2];
        }
        if (lvl) lvl[i] = l;
    }
    return DCCRGX_OK;
}

int dccrgx_map_host_ids_op(const dccrgx_mapping* map, int op, const uint64_t* ids, size_t n, uint64_t* out)
{
    DX_CHECK((ids && out) || !n, DCCRGX_EINVAL, "null argument");
    DX_CHECK(op >= 0 && op <= DCCRGX_OP_CHILD, DCCRGX_EINVAL, "bad op %d", op);
    MapParams p;
    DX_TRY(make_map_params(map, &p));
    for (size_t i = 0; i < n; i++) out[i] = host_op(p, op, ids[i]);
    return DCCRGX_OK;
}

int dccrgx_device_count(int* n)
{
    DX_CHECK(n, DCCRGX_EINVAL, "null output");
    DX_HIP(hipGetDeviceCount(n));
    return DCCRGX_OK;
}

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
}  // extern "C"

namespace dccrgx {
size_t host_threads()
{
    static const size_t nt = [] {
        size_t v = 0;
        for (const char* var : {"DCCRGX_HOST_THREADS", "OMP_NUM_THREADS"}) {
            const char* e = std::getenv(var);
            if (e && std::atoi(e) > 0) {
                v = (size_t)std::atoi(e);
                break;
            }
        }
        if (!v) v = std::max(1u, std::thread::hardware_concurrency());
        return std::min<size_t>(v, 16);
    }();
    return nt;
}

namespace {
// persistent workers for pool_run: each waits for a new generation, runs
// its share, and counts itself done
struct Pool {
    std::mutex m;
    std::condition_variable go, fin;
    std::vector<std::thread> th;
    const std::function<void(size_t)>* job = nullptr;
    std::exception_ptr err;  // the first exception a worker's share threw
    size_t gen = 0, active = 0, pending = 0;
    bool stop = false;
    void ensure(size_t workers)
    {
        while (th.size() < workers) {
            const size_t id = th.size() + 1;
            th.emplace_back([this, id] {
                size_t seen = 0;
                std::unique_lock<std::mutex> lk(m);
                for (;;) {
                    go.wait(lk, [&] { return stop || gen != seen; });
                    if (stop) return;
                    seen = gen;
                    if (id >= active) continue;
                    const std::function<void(size_t)>* j = job;
                    lk.unlock();
                    std::exception_ptr ex;
                    try {
                        (*j)(id);
                    } catch (...) {
                        ex = std::current_exception();
                    }
                    lk.lock();
                    if (ex && !err) err = ex;
                    if (--pending == 0) fin.notify_one();
                }
            });
        }
    }
    ~Pool()
    {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        go.notify_all();
        for (auto& t : th) t.join();
    }
};
Pool& pool()
{
    static Pool p;
    return p;
}
std::mutex g_pool_use;  // one parallel loop at a time
}  // namespace

void pool_run(size_t nt, const std::function<void(size_t)>& job)
{
    std::lock_guard<std::mutex> use(g_pool_use);
    Pool& p = pool();
    {
        std::lock_guard<std::mutex> lk(p.m);
        p.ensure(nt - 1);
        p.job = &job;
        p.active = nt;
        p.pending = nt - 1;
        p.err = nullptr;
        p.gen++;
    }
    p.go.notify_all();
    // every share ends before this returns, also when one throws (the workers
    // hold a pointer to `job`); then the first exception is rethrown
    std::exception_ptr ex;
    try {
        job(0);
    } catch (...) {
        ex = std::current_exception();
    }
    std::unique_lock<std::mutex> lk(p.m);
    p.fin.wait(lk, [&] { return p.pending == 0; });
    if (!ex) ex = p.err;
    p.err = nullptr;
    p.job = nullptr;
    lk.unlock();
    if (ex) std::rethrow_exception(ex);
}

// ---------------------------------------------------------------------------
// caching allocator (internal.hpp)
// ---------------------------------------------------------------------------
namespace {
// blocks up to this size are kept in size classes; larger ones are kept at
// their own size (a view's rows, a rebuild's field arrays), within
// CACHE_MAX_TOTAL, and reused once the library's stream events recorded at the
// free have passed -- work a caller queued on its own stream is not fenced, so
// caller-stream kernels over library buffers must finish before the next
// structural call, which frees and may hand out the block again (as
// include/dccrgx_stencil.hpp states for user stencils)
constexpr size_t CACHE_MAX_BLOCK = 256ull << 20;
constexpr size_t CACHE_MAX_TOTAL = 8ull << 30;     // idle bytes kept at most per device
constexpr size_t STREAM_LIST_MAX = 256ull << 20;   // a stream's own list is made common beyond this
constexpr int MAX_DEV = 64;

size_t size_class(size_t b)
{
    if (b <= 256) return 256;
    size_t c = 256;
    while (c < b) {
        const size_t mid = c + c / 2;  // classes 2^k and 1.5 * 2^k: at most 1/3 unused
        if (mid >= b && mid > c) return mid;
        c <<= 1;
    }
    return c;
}

using Lists = std::map<size_t, std::vector<void*>>;

// blocks freed while work may still use them: reusable by any stream once
// the events recorded on every stream of the device at the free have passed
struct Pending {
    std::vector<std::pair<void*, size_t>> blocks;
    std::vector<hipEvent_t> ev;
    std::vector<hipStream_t> on;  // the stream each event was recorded on
};

struct DevCache {
    std::unordered_map<void*, size_t> live;  // cached-class blocks in use -> class
    Lists idle;                              // reusable by any stream
    std::map<hipStream_t, Lists> by_stream;  // reusable by that stream (stream order)
    std::map<hipStream_t, size_t> stream_bytes;
    std::deque<Pending> pending;
    std::vector<hipEvent_t> ev_pool;
    std::vector<hipStream_t> streams;  // the library's streams on this device (contexts)
    size_t idle_bytes = 0, held_bytes = 0;  // idle; by_stream + pending
};

struct Cache {
    std::mutex m;
    DevCache dev[MAX_DEV];
};

Cache& cache()
{
    static Cache* c = new Cache();  // never destroyed: frees may come during process exit
    return *c;
}

int current_device()
{
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= MAX_DEV) d = 0;
    return d;
}

void* take(Lists& m, size_t cls)
{
    auto it = m.find(cls);
    if (it == m.end() || it->second.empty()) return nullptr;
    void* p = it->second.back();
    it->second.pop_back();
    return p;
}

// large blocks (over CACHE_MAX_BLOCK) are kept at their own size and handed
// out for requests of 80-100 % of it; *got = the block's size
void* take_fit(Lists& m, size_t need, size_t* got)
{
    for (auto it = m.lower_bound(need); it != m.end() && it->first <= need + need / 4; ++it)
        if (!it->second.empty()) {
            void* p = it->second.back();
            it->second.pop_back();
            *got = it->first;
            return p;
        }
    return nullptr;
}

// pending groups whose events have all passed become idle (oldest first)
void drain(DevCache& D)
{
    // hipEventQuery's "not ready" would stay behind as the thread's last
    // error: clear it, unless an earlier error is waiting to be read
    const bool clear = hipPeekAtLastError() == hipSuccess;
    struct Clear {
        bool on;
        ~Clear()
        {
            if (on) (void)hipGetLastError();
        }
    } clear_on_exit{clear};
    while (!D.pending.empty()) {
        Pending& g = D.pending.front();
        for (hipEvent_t e : g.ev)
            if (hipEventQuery(e) != hipSuccess) return;
        for (hipEvent_t e : g.ev) D.ev_pool.push_back(e);  // complete: reusable
        for (auto& b : g.blocks) {
            D.idle[b.second].push_back(b.first);
            D.idle_bytes += b.second;
            D.held_bytes -= b.second;
        }
        D.pending.pop_front();
    }
}

// a pending group of `blocks`: one event on every library stream of the
// device (the library queues work on its contexts' streams only; dx_malloc's
// null-stream allocations are synchronised at once)
void defer(DevCache& D, std::vector<std::pair<void*, size_t>>&& blocks)
{
    Pending g;
    g.blocks = std::move(blocks);
    if (D.streams.empty()) {  // no context: nothing can be in flight on the library's behalf
        for (auto& b : g.blocks) {
            D.idle[b.second].push_back(b.first);
            D.idle_bytes += b.second;
        }
        return;
    }
    for (hipStream_t s : D.streams) {
        hipEvent_t e = nullptr;
        if (!D.ev_pool.empty()) {
            e = D.ev_pool.back();
            D.ev_pool.pop_back();
        } else if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            e = nullptr;
        }
        if (!e || hipEventRecord(e, s) != hipSuccess) {  // cannot fence: wait for the device instead
            if (e) D.ev_pool.push_back(e);
            (void)hipDeviceSynchronize();
            for (hipEvent_t x : g.ev) D.ev_pool.push_back(x);
            g.ev.clear();
            g.on.clear();
            break;
        }
        g.ev.push_back(e);
        g.on.push_back(s);
    }
    for (auto& b : g.blocks) D.held_bytes += b.second;
    D.pending.push_back(std::move(g));
}
}  // namespace

hipError_t dx_cache_alloc(void** p, size_t bytes, hipStream_t st, bool any_stream)
{
    Cache& C = cache();
    // small blocks in size classes; large ones (a view's iteration rows, big
    // grids' lists) at their size rounded to 2 MiB, reused for requests of
    // 80-100 % of a kept block -- a large hipFree waits for the whole device
    const bool large = bytes > CACHE_MAX_BLOCK;
    const size_t cls = large ? (bytes + (2ull << 20) - 1) & ~((2ull << 20) - 1) : size_class(bytes);
    {
        std::lock_guard<std::mutex> lk(C.m);
        DevCache& D = C.dev[current_device()];
        void* q = nullptr;
        size_t got = cls;
        if (!any_stream && !large) {
            auto it = D.by_stream.find(st);
            if (it != D.by_stream.end() && (q = take(it->second, cls))) {
                D.stream_bytes[st] -= cls;
                D.held_bytes -= cls;
            }
        }
        if (!q) {
            drain(D);
            if ((q = large ? take_fit(D.idle, cls, &got) : take(D.idle, cls))) D.idle_bytes -= got;
        }
        if (q) {
            D.live[q] = got;
            *p = q;
            return hipSuccess;
        }
    }
    // hipMalloc, not the stream-ordered pool: the copy engines (SDMA) keep
    // stale translations for pool memory the pool re-maps, so a copy into or
    // out of a fresh hipMallocAsync block can land in the wrong pages
    // (tools/micro/pool_trim_copy.hip: wrong data in 24-39 of 40 rounds with
    // hipMallocAsync on either runtime, none with hipMalloc or with
    // HSA_ENABLE_SDMA=0).  The cache makes the runtime call rare.
    (void)st;
    // a huge array (a headline-size field): the idle cached blocks go back
    // first, so that it is not placed around them
    if (bytes >= (4ull << 30)) dx_cache_trim();
    hipError_t e = hipMalloc(p, cls);
    if (e == hipErrorOutOfMemory) {  // the cache's idle blocks back to the device, then once more
        (void)hipGetLastError();
        dx_cache_trim();
        e = hipMalloc(p, cls);
    }
    if (e != hipSuccess && large) {  // the rounding must not make the difference
        (void)hipGetLastError();
        e = hipMalloc(p, bytes);
        if (e == hipSuccess) {
            std::lock_guard<std::mutex> lk(C.m);
            C.dev[current_device()].live[*p] = bytes;
        }
        return e;
    }
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> lk(C.m);
        C.dev[current_device()].live[*p] = cls;
    }
    return e;
}

void dx_cache_free(void* p, hipStream_t st, bool any_stream)
{
    if (!p) return;
    dx_cache_free_many(&p, 1, st, any_stream);
}

void dx_cache_free_many(void* const* ps, size_t n, hipStream_t st, bool any_stream)
{
    Cache& C = cache();
    std::unique_lock<std::mutex> lk(C.m);
    DevCache& D = C.dev[current_device()];
    std::vector<std::pair<void*, size_t>> blocks;
    std::vector<void*> large;
    std::vector<std::pair<void*, size_t>> big;  // large blocks: fenced for any stream
    for (size_t i = 0; i < n; i++) {
        if (!ps[i]) continue;
        auto it = D.live.find(ps[i]);
        if (it == D.live.end()) {  // not the cache's: back to the pool
            large.push_back(ps[i]);
            continue;
        }
        (it->second > CACHE_MAX_BLOCK ? big : blocks).emplace_back(ps[i], it->second);
        D.live.erase(it);
    }
    if (!big.empty()) {
        std::vector<std::pair<void*, size_t>> keep;
        size_t kept = D.idle_bytes + D.held_bytes;
        for (auto& b : big) {
            if (kept + b.second > CACHE_MAX_TOTAL) {  // the cache stays within its total
                large.push_back(b.first);
                continue;
            }
            kept += b.second;
            keep.push_back(b);
        }
        if (!keep.empty()) defer(D, std::move(keep));
    }
    if (!any_stream) {  // ds_free: reused by `st` in stream order
        size_t& sb = D.stream_bytes[st];
        for (auto& b : blocks) {
            D.by_stream[st][b.second].push_back(b.first);
            sb += b.second;
            D.held_bytes += b.second;
        }
        if (sb > STREAM_LIST_MAX) {  // make them common once `st` has passed this point
            std::vector<std::pair<void*, size_t>> all;
            for (auto& kv : D.by_stream[st])
                for (void* q : kv.second) all.emplace_back(q, kv.first);
            D.by_stream.erase(st);
            D.held_bytes -= sb;
            sb = 0;
            defer(D, std::move(all));
        }
    } else if (!blocks.empty()) {
        if (D.idle_bytes + D.held_bytes > CACHE_MAX_TOTAL) {  // too much kept: return them
            lk.unlock();
            for (auto& b : blocks) (void)hipFree(b.first);  // waits for the device
            lk.lock();
        } else {
            defer(D, std::move(blocks));
        }
    }
    lk.unlock();
    for (void* q : large) (void)hipFree(q);  // waits for the device
}

void dx_cache_trim()
{
    Cache& C = cache();
    std::vector<void*> out;
    {
        std::lock_guard<std::mutex> lk(C.m);
        DevCache& D = C.dev[current_device()];
        if (D.idle_bytes == 0 && D.held_bytes == 0) return;
    }
    (void)hipDeviceSynchronize();  // every pending free has passed
    {
        std::lock_guard<std::mutex> lk(C.m);
        DevCache& D = C.dev[current_device()];
        drain(D);
        for (auto& kv : D.idle)
            for (void* q : kv.second) out.push_back(q);
        D.idle.clear();
        D.idle_bytes = 0;
        for (auto& sl : D.by_stream)
            for (auto& kv : sl.second)
                for (void* q : kv.second) {
                    out.push_back(q);
                    D.held_bytes -= kv.first;
                }
        D.by_stream.clear();
        D.stream_bytes.clear();
    }
    for (void* q : out) (void)hipFree(q);
}

void dx_cache_streams(hipStream_t a, hipStream_t b, bool add)
{
    Cache& C = cache();
    std::lock_guard<std::mutex> lk(C.m);
    DevCache& D = C.dev[current_device()];
    if (!add) {
        // the streams are synchronised and about to be destroyed: events
        // recorded on them are complete, and are destroyed now (querying an
        // event whose stream is gone corrupted the runtime's memory); so are
        // the pooled events, which may have been recorded there last
        for (Pending& g : D.pending)
            for (size_t k = 0; k < g.ev.size();)
                if (g.on[k] == a || g.on[k] == b) {
                    (void)hipEventDestroy(g.ev[k]);
                    g.ev.erase(g.ev.begin() + k);
                    g.on.erase(g.on.begin() + k);
                } else {
                    k++;
                }
        for (hipEvent_t e : D.ev_pool) (void)hipEventDestroy(e);
        D.ev_pool.clear();
        drain(D);
    }
    for (hipStream_t s : {a, b}) {
        if (add) {
            D.streams.push_back(s);
            continue;
        }
        // a destroyed stream (synchronised first): its blocks are common now
        D.streams.erase(std::remove(D.streams.begin(), D.streams.end(), s), D.streams.end());
        auto it = D.by_stream.find(s);
        if (it == D.by_stream.end()) continue;
        for (auto& kv : it->second)
            for (void* q : kv.second) {
                D.idle[kv.first].push_back(q);
                D.idle_bytes += kv.first;
                D.held_bytes -= kv.first;
            }
        D.by_stream.erase(it);
        D.stream_bytes.erase(s);
    }
}

size_t dx_cache_idle_bytes()
{
    Cache& C = cache();
    std::lock_guard<std::mutex> lk(C.m);
    DevCache& D = C.dev[current_device()];
    return D.idle_bytes + D.held_bytes;
}

size_t dx_pool_idle_bytes() { return dx_cache_idle_bytes(); }
}  // namespace dccrgx

extern "C" {

int dccrgx_ctx_create(int device, int rank, int comm_size, dccrgx_ctx** out)
{
    DX_CHECK(out, DCCRGX_EINVAL, "null out");
    DX_CHECK(comm_size >= 1 && rank >= 0 && rank < comm_size, DCCRGX_EINVAL,
             "bad rank %d / comm size %d", rank, comm_size);
    int ndev = 0;
    DX_HIP(hipGetDeviceCount(&ndev));
    DX_CHECK(device >= 0 && device < ndev, DCCRGX_EINVAL, "device %d of %d", device, ndev);
    DX_HIP(hipSetDevice(device));
    auto* c = new dccrgx_ctx();
    c->device = device;
    c->rank = rank;
    c->comm_size = comm_size;
    DX_HIP(hipStreamCreateWithFlags(&c->compute, hipStreamNonBlocking));
    DX_HIP(hipStreamCreateWithFlags(&c->comm, hipStreamNonBlocking));
    DX_HIP(hipEventCreateWithFlags(&c->ev_compute, hipEventDisableTiming));
    DX_HIP(hipEventCreateWithFlags(&c->ev_comm, hipEventDisableTiming));
    DX_HIP(hipEventCreateWithFlags(&c->ev_caller, hipEventDisableTiming));
    DX_HIP(hipEventCreateWithFlags(&c->ev_enter, hipEventDisableTiming));
    dx_cache_streams(c->compute, c->comm, true);  // frees are fenced on these streams
    *out = c;
    return DCCRGX_OK;
}

int dccrgx_ctx_destroy(dccrgx_ctx* c)
{
    if (!c) return DCCRGX_OK;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->compute);
    hipStreamSynchronize(c->comm);
    dx_cache_streams(c->compute, c->comm, false);
    dx_free(c->ident);
    for (uint32_t* q : c->ident_old) dx_free(q);
    dx_cache_trim();
    if (c->has_comm) ncclCommDestroy(c->nccl);
    hipEventDestroy(c->ev_compute);
    hipEventDestroy(c->ev_comm);
    hipEventDestroy(c->ev_caller);
    hipEventDestroy(c->ev_enter);
    for (hipEvent_t e : c->up_ev)  // recorded on the compute stream, which is idle now
        if (e) hipEventDestroy(e);
    hipStreamDestroy(c->compute);
    hipStreamDestroy(c->comm);
    if (c->stage) hipHostFree(c->stage);
    if (c->up) hipHostFree(c->up);
    delete c;
    return DCCRGX_OK;
}

int dccrgx_get_unique_id(uint8_t uid_out[128])
{
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    DX_RCCL(ncclGetUniqueId(&id));
    std::memcpy(uid_out, &id, 128);
    return DCCRGX_OK;
}

int dccrgx_ctx_route_self_through_rccl(dccrgx_ctx* c, int32_t on)
{
    DX_CHECK(c, DCCRGX_EINVAL, "null context");
    c->self_peer = on != 0;
    return DCCRGX_OK;
}

int dccrgx_ctx_set_host_transport(dccrgx_ctx* c, const dccrgx_host_transport* t)
{
    DX_CHECK(c, DCCRGX_EINVAL, "null context");
    if (!t) {
        c->host_tx = dccrgx_host_transport{};
        c->has_host_tx = false;
        return DCCRGX_OK;
    }
    DX_CHECK(t->exchange && t->allreduce_f64, DCCRGX_EINVAL, "transport without exchange / allreduce_f64");
    c->host_tx = *t;
    c->has_host_tx = true;
    return DCCRGX_OK;
}

int dccrgx_ctx_comm_init(dccrgx_ctx* c, const uint8_t uid[128])
{
    DX_CHECK(c && uid, DCCRGX_EINVAL, "null argument");
    DX_CHECK(!c->has_comm, DCCRGX_ESTATE, "communicator already initialised");
    DX_HIP(hipSetDevice(c->device));
    ncclUniqueId id;
    std::memcpy(&id, uid, 128);
    DX_RCCL(ncclCommInitRank(&c->nccl, c->comm_size, id, c->rank));
    c->has_comm = true;
    return DCCRGX_OK;
}

int dccrgx_ctx_compute_stream(dccrgx_ctx* c, void** s)
{
    DX_CHECK(c && s, DCCRGX_EINVAL, "null argument");
    *s = (void*)c->compute;
    return DCCRGX_OK;
}

int dccrgx_ctx_synchronize(dccrgx_ctx* c)
{
    DX_CHECK(c, DCCRGX_EINVAL, "null ctx");
    DX_HIP(hipSetDevice(c->device));
    DX_HIP(hipStreamSynchronize(c->comm));
    DX_HIP(hipStreamSynchronize(c->compute));
    return DCCRGX_OK;
}

}  // extern "C"

// ---- test options (internal.hpp) ------------------------------------------
namespace dccrgx {
namespace {
std::atomic<int64_t> g_test_opt[OPT_COUNT];
std::atomic<bool> g_test_set[OPT_COUNT];
const char* const kTestOptName[OPT_COUNT] = {"gol_scalar",  "gol_chunk",      "poisson_multi",
                                             "poisson_solo_global", "incremental", "ou_small",
                                             "corrupt_ghost", "fail_stop_refining", "check_init", "full_nto",
                                             "hybrid", "ou_walk"};
}  // namespace

int64_t test_opt(TestOpt o, int64_t dflt)
{
#ifdef DCCRGX_NO_TEST_OPTIONS
    (void)o;
    return dflt;
#else
    return g_test_set[o].load(std::memory_order_relaxed) ? g_test_opt[o].load(std::memory_order_relaxed) : dflt;
#endif
}
}  // namespace dccrgx

extern "C" int dccrgx_test_option(const char* name, int64_t value, int32_t set)
{
    using namespace dccrgx;
    DX_CHECK(name, DCCRGX_EINVAL, "null name");
#ifdef DCCRGX_NO_TEST_OPTIONS
    (void)value;
    (void)set;
    return set_error(DCCRGX_EINVAL, "test options are compiled out of this build");
#else
    for (int o = 0; o < OPT_COUNT; o++)
        if (std::strcmp(name, kTestOptName[o]) == 0) {
            g_test_opt[o].store(value);
            g_test_set[o].store(set != 0);
            return DCCRGX_OK;
        }
    return set_error(DCCRGX_EINVAL, "unknown test option '%s'", name);
#endif
}
