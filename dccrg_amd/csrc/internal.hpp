// internal.hpp -- shared internals of libdccrgx.so (MI355X / gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <algorithm>
#include <vector>

#include "dccrgx.h"

namespace dccrgx {

// ---------------------------------------------------------------------------
// errors: thread-local message, status codes from dccrgx.h
// ---------------------------------------------------------------------------
int set_error(int code, const char* fmt, ...);

#define DX_HIP(expr)                                                                    \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return ::dccrgx::set_error(DCCRGX_EHIP, "%s:%d %s: %s", __FILE__, __LINE__, \
                                       #expr, hipGetErrorString(e_));                   \
    } while (0)

#define DX_RCCL(expr)                                                                    \
    do {                                                                                 \
        ncclResult_t r_ = (expr);                                                        \
        if (r_ != ncclSuccess)                                                           \
            return ::dccrgx::set_error(DCCRGX_ERCCL, "%s:%d %s: %s", __FILE__, __LINE__, \
                                       #expr, ncclGetErrorString(r_));                   \
    } while (0)

// Device allocations of the library go through a caching layer over
// hipMalloc (core.hip): an adaptive run frees and allocates grid structures
// every step, and returning them to the driver each time cost tens of ms.
// Blocks up to 256 MiB are kept in size classes when freed and handed out
// again without a runtime call (hipFreeAsync cost ~35 us on torch's bundled
// HIP runtime and an adaptive step freed ~60 scratch buffers -- 2 ms of the
// step, tools/api_census.py); larger blocks are kept at their size (rounded
// to 2 MiB) and reused for requests of 80-100 % of it.  A block freed with
// ds_free on a stream is reused only by that stream (stream order keeps it
// safe); blocks freed with dx_free / FreeBatch (and every large block) are
// reused by any stream once events recorded on every library stream at the
// free have passed -- no host wait, so such a free between a halo's start
// and wait does not block on the exchange.  Blocks freed while the cache
// holds its total limit (8 GiB idle) go back with hipFree, which waits for
// the whole device: such a free between a halo's start and wait stalls the
// host until the exchange is done (grids free them only in structural
// calls).  A hipMalloc that runs out of memory returns the idle blocks first
// and tries again.  The stream-ordered pool (hipMallocAsync) is not used:
// the copy engines keep stale translations for pool memory the pool re-maps,
// and copies into fresh pool blocks landed in the wrong pages
// (tools/micro/pool_trim_copy.hip).
void dx_slow_note(const char* what, size_t bytes, double ms);  // DCCRGX_TIMING: allocations over 1 ms

// idle bytes the cache holds (free for the library's purposes)
size_t dx_pool_idle_bytes();
// return every idle cached block to the device (grid and context teardown)
void dx_cache_trim();

hipError_t dx_cache_alloc(void** p, size_t bytes, hipStream_t st, bool any_stream);
// any_stream: the block becomes reusable by any stream once every library
// stream of the device has passed the free (events, no host wait)
void dx_cache_free(void* p, hipStream_t st, bool any_stream);
void dx_cache_free_many(void* const* ps, size_t n, hipStream_t st, bool any_stream);
// a context's streams join (add) or leave the set the frees are fenced on
void dx_cache_streams(hipStream_t a, hipStream_t b, bool add);
size_t dx_cache_idle_bytes();

template <class T>
inline hipError_t dx_malloc(T** p, size_t bytes)
{
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e = dx_cache_alloc(reinterpret_cast<void**>(p), bytes ? bytes : 1, nullptr, true);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms > 1.0) dx_slow_note("dx_malloc", bytes, ms);
    return e;
}

inline hipError_t dx_free(void* p)
{
    if (p) dx_cache_free(p, nullptr, true);
    return hipSuccess;
}

// Frees of many buffers behind one set of events (structures are released
// together: a neighborhood, an explicit grid's state)
struct FreeBatch {
    std::vector<void*> v;
    void add(void* p)
    {
        if (p) v.push_back(p);
    }
    ~FreeBatch()
    {
        if (!v.empty()) dx_cache_free_many(v.data(), v.size(), nullptr, true);
    }
};

// Stream-ordered allocation for structures built on one stream (neighbor
// lists, scratch of a build): no synchronisation -- the memory is valid for
// work queued on `st` after the call, and a ds_free on `st` returns it once
// the work queued before it is done.  Such memory may later be released
// with dx_free.
template <class T>
inline hipError_t ds_malloc(T** p, size_t bytes, hipStream_t st)
{
    return dx_cache_alloc(reinterpret_cast<void**>(p), bytes ? bytes : 1, st, false);
}

inline hipError_t ds_free(void* p, hipStream_t st)
{
    if (p) dx_cache_free(p, st, false);
    return hipSuccess;
}

#define DX_TRY(expr)                       \
    do {                                   \
        int s_ = (expr);                   \
        if (s_ != DCCRGX_OK) return s_;    \
    } while (0)

#define DX_CHECK(cond, code, ...)                                     \
    do {                                                              \
        if (!(cond)) return ::dccrgx::set_error((code), __VA_ARGS__); \
    } while (0)

// ---------------------------------------------------------------------------
// host phase timing of structural calls (AMR rebuild, neighbor builds):
// DCCRGX_TIMING=1 prints one line per phase to stderr; =2 waits for the
// device before each lap (device time lands in the phase that queued it)
// ---------------------------------------------------------------------------
struct PhaseTimer {
    const char* scope;
    std::chrono::steady_clock::time_point t;
    bool on, sync;
    explicit PhaseTimer(const char* s) : scope(s), t(std::chrono::steady_clock::now())
    {
        const char* e = std::getenv("DCCRGX_TIMING");
        on = e && *e && *e != '0';
        sync = on && *e == '2';
    }
    void lap(const char* what)
    {
        if (!on) return;
        if (sync) (void)hipDeviceSynchronize();
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[dccrgx] %s %s %.3f ms\n", scope, what,
                     std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

// Test options (dccrgx_test_option, core.hip): switches the GPU tests use to
// force a code path the library otherwise picks by size, and fault injection.
// Set explicitly through the C-ABI, never read from the environment; all off
// by default.  A product build may compile them out (-DDCCRGX_NO_TEST_OPTIONS:
// test_opt() returns its default and dccrgx_test_option refuses).
enum TestOpt {
    OPT_GOL_SCALAR,          // LDS-tiled scalar GoL kernels on grids the vector kernels take
    OPT_GOL_CHUNK,           // slices per workgroup of the GoL kernels (chunk seams in small grids)
    OPT_POISSON_MULTI,       // the multi-kernel BiCG for systems one workgroup would take
    OPT_POISSON_SOLO_GLOBAL, // k_solo over global memory instead of k_solo_lds
    OPT_INCREMENTAL,         // 1 / 0: incremental / full neighbor-list rebuilds at any size
    OPT_OU_SMALL,            // queue of override_unrefines' small first pass (overflow retries)
    OPT_CORRUPT_GHOST,       // dccrgx_gol_step marks a ghost cell alive after each exchange
    OPT_FAIL_STOP_REFINING,  // this rank's next stop_refining decisions report ENOMEM (rank + 1)
    OPT_CHECK_INIT,          // explicit grids: check the device leaves and lookups against the host list
    OPT_FULL_NTO,            // one rank: the full neighbors_to transpose after an incremental neighbors_of
    OPT_HYBRID,              // 1: one-process uniform grids refine in place (hybrid.hip) whatever their size
    OPT_OU_WALK,             // 1: override_unrefines walks the face graph (k_ou_walk) instead of k_ou_check
    OPT_COUNT
};
int64_t test_opt(TestOpt o, int64_t dflt);

// ---------------------------------------------------------------------------
// host-side parallel loop for structural work that is independent per item
// (AMR request filtering): [0, n) in contiguous ranges of at least `grain`
// items over up to DCCRGX_HOST_THREADS (else OMP_NUM_THREADS, else the
// hardware's count) threads, capped at 16.  f(begin, end) must only read
// shared state and write disjoint outputs.  The worker threads persist
// between calls (an adaptive run calls this every step; starting 16 threads
// costs more than the work).
// ---------------------------------------------------------------------------
size_t host_threads();
// run job(t) for t in [0, nt) on the pool (t = 0 on the calling thread)
void pool_run(size_t nt, const std::function<void(size_t)>& job);

template <class F>
void parallel_ranges(size_t n, size_t grain, F&& f)
{
    const size_t nt = std::min<size_t>(host_threads(), (n + grain - 1) / std::max<size_t>(grain, 1));
    if (nt <= 1) {
        f((size_t)0, n);
        return;
    }
    const size_t per = (n + nt - 1) / nt;
    pool_run(nt, [&](size_t t) {
        const size_t b = std::min(n, t * per), e = std::min(n, b + per);
        if (b < e) f(b, e);
    });
}

// ---------------------------------------------------------------------------
// 64-bit division by an invariant divisor (Granlund-Montgomery, "unsigned
// division by invariant integers using multiplication", fig. 4.1): 64-bit
// integer division is a long emulated sequence on CDNA, a mul-hi is 4 muls.
// ---------------------------------------------------------------------------
struct Divider {
    uint64_t m;      // magic
    uint32_t sh1;    // min(L, 1)
    uint32_t sh2;    // max(L - 1, 0)
};

inline Divider make_divider(uint64_t d)
{
    Divider r{};
    if (d == 0) d = 1;  // never divided by; keep well defined
    int L = 0;
    while (L < 64 && ((unsigned __int128)1 << L) < d) L++;  // L = ceil(log2 d)
    const unsigned __int128 twoL = (unsigned __int128)1 << L;
    const unsigned __int128 num = (twoL - d) << 64;
    r.m = (uint64_t)(num / d) + 1;
    r.sh1 = L < 1 ? L : 1;
    r.sh2 = L > 1 ? L - 1 : 0;
    return r;
}

#ifdef __HIPCC__
// XCD-aware block order: the dispatcher deals workgroups round-robin over the
// 8 XCDs (block b runs on XCD b % 8); this bijection gives each XCD a
// contiguous run of blocks, so work that reads its neighbors' lines (rows of
// a grid, a stencil's apron) finds them in its own L2
__device__ inline uint32_t xcd_block()
{
    const uint32_t bid = blockIdx.x, nwg = gridDim.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

// One thread's walk over its own row [e, e1) of a stencil row CSR (4-byte
// slots, 3 x 4-byte offsets): once the position is a multiple of four, four
// entries per 16-byte load of slots and three of offsets (lanes on different
// rows: each load is a line per lane, so fewer, wider loads use each line
// for more entries).  fn(entry, slot, x, y, z) in row order.
template <class F>
__device__ inline void row_walk4(uint64_t e, uint64_t e1, const uint32_t* __restrict__ slot,
                                 const int32_t* __restrict__ off, F&& fn)
{
    for (; e < e1 && (e & 3); e++) fn(e, slot[e], off[3 * e], off[3 * e + 1], off[3 * e + 2]);
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    typedef int32_t i4 __attribute__((ext_vector_type(4)));
    for (; e + 4 <= e1; e += 4) {
        const u4 s = *reinterpret_cast<const u4*>(slot + e);
        const i4* po = reinterpret_cast<const i4*>(off + 3 * e);
        const i4 o0 = po[0], o1 = po[1], o2 = po[2];
        fn(e, s.x, o0.x, o0.y, o0.z);
        fn(e + 1, s.y, o0.w, o1.x, o1.y);
        fn(e + 2, s.z, o1.z, o1.w, o2.x);
        fn(e + 3, s.w, o2.y, o2.z, o2.w);
    }
    for (; e < e1; e++) fn(e, slot[e], off[3 * e], off[3 * e + 1], off[3 * e + 2]);
}

// the same over a row of 4-byte values alone: fn(entry, value)
template <class F>
__device__ inline void row_walk4(uint64_t e, uint64_t e1, const uint32_t* __restrict__ val, F&& fn)
{
    for (; e < e1 && (e & 3); e++) fn(e, val[e]);
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    for (; e + 4 <= e1; e += 4) {
        const u4 v = *reinterpret_cast<const u4*>(val + e);
        fn(e, v.x);
        fn(e + 1, v.y);
        fn(e + 2, v.z);
        fn(e + 3, v.w);
    }
    for (; e < e1; e++) fn(e, val[e]);
}
#endif

__host__ __device__ inline uint64_t mulhi64(uint64_t a, uint64_t b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

__host__ __device__ inline uint64_t divide(uint64_t n, const Divider& d)
{
    const uint64_t t1 = mulhi64(d.m, n);
    return (t1 + ((n - t1) >> d.sh1)) >> d.sh2;
}

// ---------------------------------------------------------------------------
// Mapping parameters (dccrg_mapping.hpp) in a form kernels take by value.
// ---------------------------------------------------------------------------
constexpr int MAX_LEVELS = 24;  // > maximum possible refinement level (21) + 2

struct MapParams {
    uint64_t length[3];
    uint64_t first_id[MAX_LEVELS];  // first id of each level (level l .. l+1 boundary)
    uint64_t last_cell;
    uint64_t nlevel0;
    Divider div_lx;    // / length[0]
    Divider div_lxly;  // / (length[0]*length[1])
    int32_t max_lvl;
    int32_t pad_;
};

int make_map_params(const dccrgx_mapping* m, MapParams* out);
int max_possible_level(const uint64_t length[3]);

// Mapping::get_refinement_level, dccrg_mapping.hpp:262-290
__host__ __device__ inline int map_level(const MapParams& p, uint64_t cell)
{
    if (cell == 0 || cell > p.last_cell) return -1;
    // levels are contiguous id ranges: count the level starts <= cell
    // (uniform trip count max_lvl; first_id lives in scalar registers)
    int l = 0;
    for (int k = 1; k <= p.max_lvl; k++) l += cell >= p.first_id[k] ? 1 : 0;
    return l;
}

// Mapping::get_indices, dccrg_mapping.hpp:218-254 (bit-exact; 2 magic divisions)
__host__ __device__ inline bool map_indices(const MapParams& p, uint64_t cell, uint64_t out[3],
                                            int* lvl_out)
{
    const int l = map_level(p, cell);
    if (lvl_out) *lvl_out = l;
    if (l < 0) {
        out[0] = out[1] = out[2] = DCCRGX_ERROR_INDEX;
        return false;
    }
    const uint64_t r = cell - p.first_id[l];
    const uint64_t t = divide(r >> l, p.div_lx);          // r / (Lx 2^l)
    const uint64_t z = divide(r >> (2 * l), p.div_lxly);  // r / (Lx Ly 4^l)
    const uint64_t x = r - t * (p.length[0] << l);
    const uint64_t y = t - z * (p.length[1] << l);
    const int s = p.max_lvl - l;
    out[0] = x << s;
    out[1] = y << s;
    out[2] = z << s;
    return true;
}

// Mapping::get_cell_from_indices, dccrg_mapping.hpp:154-209
__host__ __device__ inline uint64_t map_cell(const MapParams& p, const uint64_t idx[3], int lvl)
{
    const int M = p.max_lvl;
    if (idx[0] >= (p.length[0] << M)) return 0;
    if (idx[1] >= (p.length[1] << M)) return 0;
    if (idx[2] >= (p.length[2] << M)) return 0;
    if (lvl < 0 || lvl > M) return 0;
    const int s = M - lvl;
    const uint64_t lx = p.length[0] << lvl, ly = p.length[1] << lvl;
    return p.first_id[lvl] + (idx[0] >> s) + (idx[1] >> s) * lx + (idx[2] >> s) * lx * ly;
}

__host__ __device__ inline uint64_t map_len_in_indices(const MapParams& p, uint64_t cell)
{
    const int l = map_level(p, cell);
    if (l < 0) return DCCRGX_ERROR_INDEX;
    return (uint64_t)1 << (p.max_lvl - l);
}

// ---------------------------------------------------------------------------
// block partition, dccrg.hpp:8098-8145 (non-SFC)
// ---------------------------------------------------------------------------
struct Partition {
    uint64_t total;   // level-0 cells
    uint64_t cpp;     // cells_per_process
    uint64_t fewer;   // processes with cpp-1 cells
    uint64_t split;   // first 0-based index owned by a "cpp" process = fewer*(cpp-1)
    Divider div_cpp, div_cpp1;
    int32_t comm_size;
    int32_t pad_;
};

Partition make_partition(uint64_t total, int comm_size);

__host__ __device__ inline int part_owner(const Partition& P, uint64_t level0_id)
{
    const uint64_t i = level0_id - 1;
    if (i < P.split) return (int)divide(i, P.div_cpp1);  // cpp-1 > 0 here
    return (int)(P.fewer + divide(i - P.split, P.div_cpp));
}

inline uint64_t part_first(const Partition& P, int rank)  // 1-based first id
{
    const uint64_t r = (uint64_t)rank;
    if (r <= P.fewer) return 1 + r * (P.cpp - 1);
    return 1 + P.split + (r - P.fewer) * P.cpp;
}

inline uint64_t part_count(const Partition& P, int rank)
{
    return (uint64_t)rank < P.fewer ? P.cpp - 1 : P.cpp;
}

// ---------------------------------------------------------------------------
// SFC placement, dccrg.hpp:8147-8220 (USE_SFC; sfc.hip): the level-0 cells in
// Hilbert order get the block partition's per-process counts.  Process r's
// cells are the ones whose key lies in [cut[r-1], cut[r]), so the P-1 cut keys
// are the whole placement: owner = number of cut keys <= the cell's key.
// ---------------------------------------------------------------------------

// Hilbert index of (x, y, z) with `b` bits per axis (Skilling, "Programming
// the Hilbert curve", AIP Conf. Proc. 707, 2004: axes -> transpose, read out
// most significant bit first, X[0] X[1] X[2] per bit; x = X[0])
__host__ __device__ inline uint64_t hilbert3(uint32_t x, uint32_t y, uint32_t z, int b)
{
    uint32_t X[3] = {x, y, z};
    const uint32_t M = 1u << (b - 1);
    for (uint32_t Q = M; Q > 1; Q >>= 1) {  // inverse undo
        const uint32_t P = Q - 1;
        for (int i = 0; i < 3; i++) {
            if (X[i] & Q) {
                X[0] ^= P;
            } else {
                const uint32_t t = (X[0] ^ X[i]) & P;
                X[0] ^= t;
                X[i] ^= t;
            }
        }
    }
    X[1] ^= X[0];  // Gray encode
    X[2] ^= X[1];
    uint32_t t = 0;
    for (uint32_t Q = M; Q > 1; Q >>= 1)
        if (X[2] & Q) t ^= Q - 1;
    for (int i = 0; i < 3; i++) X[i] ^= t;
    uint64_t key = 0;
    for (int bit = b - 1; bit >= 0; bit--)
        for (int i = 0; i < 3; i++) key = (key << 1) | ((X[i] >> bit) & 1u);
    return key;
}

struct SfcCuts {
    const uint64_t* cut;  // ascending; cut[r-1] = key of process r's first cell (r = 1 .. ncut); null: no SFC
    int32_t ncut;         // comm_size - 1
    int32_t bits;         // bits per axis of the Hilbert cube (smallest power of two holding the grid)
    Divider div_lx, div_lxly;  // level-0 extents: x = i % lx, y = (i / lx) % ly, z = i / (lx * ly)
    uint64_t lx, ly;
};

__host__ __device__ inline uint64_t sfc_key(const SfcCuts& s, uint64_t level0_id)
{
    const uint64_t i = level0_id - 1;
    const uint64_t q = divide(i, s.div_lx), z = divide(i, s.div_lxly);
    return hilbert3((uint32_t)(i - q * s.lx), (uint32_t)(q - z * s.ly), (uint32_t)z, s.bits);
}

__host__ __device__ inline int sfc_owner(const SfcCuts& s, uint64_t level0_id)
{
    const uint64_t key = sfc_key(s, level0_id);
    int lo = 0, hi = s.ncut;  // first cut > key
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s.cut[mid] <= key)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
struct Ctx {
    int device = 0, rank = 0, comm_size = 1;
    hipStream_t compute = nullptr, comm = nullptr;
    hipEvent_t ev_compute = nullptr, ev_comm = nullptr;
    hipEvent_t ev_caller = nullptr;  // CallerStream
    hipEvent_t ev_enter = nullptr;   // CallerStream
    ncclComm_t nccl = nullptr;
    bool has_comm = false;
    // test mode (dccrgx_ctx_route_self_through_rccl): a rank's own periodic
    // images travel as RCCL send/recv to itself instead of device copies, so
    // the multi-rank halo path (pack, grouped send/recv, unpack, inner/outer
    // overlap) runs on one GPU through the real communicator
    bool self_peer = false;
    // host-staged transport (dccrgx_ctx_set_host_transport) for ranks without
    // a communicator
    dccrgx_host_transport host_tx{};
    bool has_host_tx = false;
    // pinned bounce buffer of dx_h2d / dx_d2h, and its device address (small
    // read-backs are gathered into it by one kernel, dx_d2h_many)
    void* stage = nullptr;
    void* stage_dev = nullptr;
    size_t stage_bytes = 0;
    // 0, 1, 2, ... on the device, shared by the identity maps of one-rank
    // grids (local position = leaf = slot); grown geometrically, the smaller
    // arrays kept until the context goes (grids may still point into them)
    uint32_t* ident = nullptr;
    uint64_t ident_n = 0;
    std::vector<uint32_t*> ident_old;
    // pinned upload slots of dx_h2d_async: slot k is reused once the event
    // recorded after its copy has passed
    static constexpr int UP_SLOTS = 16;
    static constexpr size_t UP_SLOT_BYTES = 256u << 10;
    char* up = nullptr;
    hipEvent_t up_ev[UP_SLOTS] = {};
    bool up_used[UP_SLOTS] = {};
    int up_next = 0;
};

// Entry points that take a caller's stream queue kernels there which read
// grid-owned buffers (hash, neighbor CSRs, fields).  Freed blocks are fenced
// by events on the library's own streams only (dx_free), so on leaving such
// an entry point the compute stream is made to wait for what the library
// queued on the caller's stream: a later free, rebuild or destroy then covers
// those kernels too.  Only the library's own launches are covered; caller
// kernels reading grid memory (dccrgx_field_device_ptr) must be synchronised
// by the caller before structural calls (dccrgx.h).
struct CallerStream {
    Ctx* c;
    hipStream_t st;
    // the call's work on a caller's stream follows the library's queued work
    // (field writes, steps on the compute stream), and later library work
    // follows it: stream order on both sides, no device-wide wait
    CallerStream(Ctx* c_, hipStream_t s) : c(c_), st(s)
    {
        if (!c || !st || st == c->compute || st == c->comm) return;
        if (hipEventRecord(c->ev_enter, c->compute) == hipSuccess) (void)hipStreamWaitEvent(st, c->ev_enter, 0);
    }
    ~CallerStream()
    {
        if (!c || !st || st == c->compute || st == c->comm) return;
        if (hipEventRecord(c->ev_caller, st) == hipSuccess) (void)hipStreamWaitEvent(c->compute, c->ev_caller, 0);
    }
};

// Host <-> device copies of pageable host memory through the context's pinned
// bounce buffer, in chunks of at most 64 MiB; they return after the copy has
// completed on `st`.  A pageable hipMemcpyAsync of even a few KB stalls for
// ~16 ms now and then on this runtime (seen in the adaptive loop); copies
// from pinned memory do not.
int dx_h2d(Ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st);
int dx_d2h(Ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st);
// A small upload (at most Ctx::UP_SLOT_BYTES) on the context's compute stream
// that returns at once: `src` is copied into a pinned slot, the device copy is
// ordered on the stream like a kernel.  Work on other streams must be ordered
// after it by the caller (the structural calls end in a synchronisation).
// Larger copies and other streams take dx_h2d.
int dx_h2d_async(Ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st);
// several device -> host copies behind one synchronisation; small ones (at
// most 16 ranges, 1 MiB together) are one gather kernel writing the pinned
// stage (a runtime copy of pinned memory is a launch of its own per range)
struct D2H {
    void* dst;
    const void* src;
    size_t bytes;
};
int dx_d2h_many(Ctx* c, const D2H* v, size_t n, hipStream_t st);
// several memsets in one launch (each hipMemsetAsync is a launch of its own
// and costs the host as much as a kernel): at most 8 byte ranges, each set
// to one byte value
struct Fill {
    void* p;
    size_t bytes;
    uint8_t value;
};
int dx_fill_many(const Fill* v, int n, hipStream_t st);
// the context's identity array, at least n entries (one launch when it grows)
int ctx_identity(Ctx* c, uint64_t n, uint32_t** out, hipStream_t st);
// p is (in) one of the context's identity arrays: not to be freed
bool ctx_is_identity(const Ctx* c, const void* p);

}  // namespace dccrgx

struct dccrgx_ctx : dccrgx::Ctx {};
