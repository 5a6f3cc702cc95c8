// grid.hpp -- dccrgx_grid internals: uniform implicit layout, neighborhoods,
// per-peer halo plans, field pools.
#pragma once

#include "flatset.hpp"
#include "internal.hpp"

#include <array>
#include <atomic>
#include <map>
#include <set>
#include <unordered_map>

namespace dccrgx {

// Canonical axes (A fastest, C slowest with extent > 1 unless 1-D) so that
// the 0-based cell index lin = a + LA*(b + LB*c) equals id - 1 for level-0
// cells (dccrg_mapping.hpp:154-209 at level 0).  The block partition
// (dccrg.hpp:8098-8145) then cuts the C axis into slabs: each rank stores its
// slab plus `pad` ghost slices on both sides, addressed with an UNWRAPPED c
// (periodic wrap of A and B is done in index space by the kernels).
struct UGeom {
    uint64_t LA, LB, LC, S;  // S = LA * LB (one slice)
    uint64_t N;              // total level-0 cells
    uint64_t lo, hi;         // local lin range [lo, hi)
    int64_t cbase;           // canonical slice held in storage slice 0
    uint64_t nslices;        // storage slices (local + 2 * pad)
    Divider dA, dS;
    Partition part;
    int32_t perA, perB, perC;
    int32_t rank;
    int32_t M;               // max refinement level (offsets are in units of 2^M)
    int32_t pad;             // ghost slices on each side
    int32_t perm[3];         // canonical axis -> original axis
};

__host__ __device__ inline void ug_decompose(const UGeom& g, uint64_t lin, int64_t& a, int64_t& b,
                                             int64_t& c)
{
    const uint64_t cc = divide(lin, g.dS);
    const uint64_t rem = lin - cc * g.S;
    const uint64_t bb = divide(rem, g.dA);
    a = (int64_t)(rem - bb * g.LA);
    b = (int64_t)bb;
    c = (int64_t)cc;
}

__host__ __device__ inline int64_t ug_wrap(int64_t x, int64_t L)
{
    int64_t r = x % L;
    return r < 0 ? r + L : r;
}

// neighbor of canonical (a,b,c) at item d: wrapped lin and unwrapped c.
// false when the item falls outside a non-periodic grid (dropped, as the
// reference drops it: dccrg.hpp:4670-4672)
__host__ __device__ inline bool ug_neighbor(const UGeom& g, int64_t a, int64_t b, int64_t c,
                                            const int32_t* d, uint64_t& nlin, int64_t& cu)
{
    int64_t a2 = a + d[0], b2 = b + d[1], c2 = c + d[2];
    cu = c2;
    if (a2 < 0 || a2 >= (int64_t)g.LA) {
        if (!g.perA) return false;
        a2 = ug_wrap(a2, (int64_t)g.LA);
    }
    if (b2 < 0 || b2 >= (int64_t)g.LB) {
        if (!g.perB) return false;
        b2 = ug_wrap(b2, (int64_t)g.LB);
    }
    if (c2 < 0 || c2 >= (int64_t)g.LC) {
        if (!g.perC) return false;
        c2 = ug_wrap(c2, (int64_t)g.LC);
    }
    nlin = (uint64_t)a2 + g.LA * ((uint64_t)b2 + g.LB * (uint64_t)c2);
    return true;
}

__host__ __device__ inline bool ug_local(const UGeom& g, uint64_t lin) { return lin >= g.lo && lin < g.hi; }

__host__ __device__ inline int ug_owner(const UGeom& g, uint64_t lin) { return part_owner(g.part, lin + 1); }

// storage slot of canonical (a, b, unwrapped c)
__host__ __device__ inline uint64_t ug_slot(const UGeom& g, int64_t a, int64_t b, int64_t cu)
{
    return (uint64_t)a + g.LA * ((uint64_t)b + g.LB * (uint64_t)(cu - g.cbase));
}

// a byte copy between two device buffers (offsets relative to each)
struct ByteSeg {
    uint64_t src, dst, len;
};

// a variable-size field's byte segments for one copy -- a message's pack or
// unpack, or the periodic self copies -- built from the host count / offset
// mirrors once per count epoch and kept on the device
struct VarPlan {
    uint64_t epoch = 0;  // Field::epoch it was built for (0: none)
    ByteSeg* d = nullptr;
    uint64_t n = 0;      // segments
    uint64_t bytes = 0;  // message bytes of the field (pack: sent, unpack: received)
};
using VarPlans = std::map<int32_t, VarPlan>;  // by field id

// a fresh epoch for a variable field whose counts or offsets changed (never reused)
uint64_t next_var_epoch();

inline void free_var_plans(VarPlans& m, FreeBatch& fb)
{
    for (auto& kv : m) fb.add(kv.second.d);
    m.clear();
}

struct Field {
    void* ptr = nullptr;
    uint32_t elem = 0;
    size_t cap_bytes = 0;  // allocation size when it exceeds n_slots * elem (AMR rebuild), else 0
    // variable-size cell data (tests/variable_data_size): `ptr` is a pool,
    // slot s holds count[s] elements at byte offset off[s] (host mirrors;
    // message sizes are computed from them)
    bool variable = false;
    std::vector<uint32_t> count;
    std::vector<uint64_t> off;
    size_t pool_bytes = 0;
    uint64_t epoch = 0;  // version of count / off (next_var_epoch), keys the cached VarPlans
};

struct PeerPlan {
    int peer = -1;
    // cells this rank sends to `peer` (ascending ids) -- dccrg.hpp:8754-8850
    std::vector<uint64_t> send_ids;
    uint64_t* d_send_slots = nullptr;  // storage slot of each sent cell
    bool send_direct = false;          // slots contiguous: send straight from the field
    uint64_t send_slot0 = 0;
    // cells this rank receives from `peer` (ascending ids) -- dccrg.hpp:8852-8891
    std::vector<uint64_t> recv_ids;
    bool recv_direct = false;          // one ghost slot per cell, contiguous: receive in place
    uint64_t recv_slot0 = 0;
    uint64_t n_unpack = 0;             // (dst slot, message index) pairs otherwise
    uint64_t* d_unpack_dst = nullptr;
    uint64_t* d_unpack_src = nullptr;
    // host copies of the plans (variable-size fields build byte segments
    // from them): slot of each sent cell; (dst slot, message index) of every
    // ghost slot filled from this peer, direct receives included
    std::vector<uint64_t> h_send_slots;
    std::vector<uint64_t> h_unpack_dst, h_unpack_src;
    // staging (allocated on first use, grown as needed)
    void* d_send_buf = nullptr;
    size_t send_buf_bytes = 0;
    void* d_recv_buf = nullptr;
    size_t recv_buf_bytes = 0;
    // host copies of the messages (host-staged transport)
    std::vector<char> h_send_msg, h_recv_msg;
    // variable-size fields: pack / unpack segments per field
    VarPlans var_send, var_recv;
};

struct Explicit;
// the host copy of a leaf list kept on the device (Explicit::leaves())
void explicit_fetch_leaves(const Explicit* E);
// the host copy of an explicit grid's leaf list (fetched once after a device
// rebuild): public entry points that use host lookups call this first, so a
// failing copy is an error code, not an abort (no-op for uniform grids)
int explicit_host_leaves(const dccrgx_grid* grid);

struct Explicit {
    uint64_t n = 0;                 // global leaves
    // Host copies of the leaf list, the local cells and the slot ids.  On one
    // rank the local cells are the leaves and slot k < n holds leaf k, so
    // `local_` stays empty and `slot_ids_` holds only the slots after the
    // leaves (retired cells); after a rebuild decided on the device the leaf
    // list itself stays on the device until host code asks for it (an
    // adaptive step needs none: 3 copies of 8 B per leaf saved per step).
    mutable std::vector<uint64_t> leaves_;  // ascending (valid when host_leaves)
    mutable std::atomic<bool> host_leaves{true};
    Ctx* ctx = nullptr;                     // for the lazy fetch
    bool one_rank = false;                  // local = leaves, slots [0, n) = leaves
    const std::vector<uint64_t>& leaves() const
    {
        if (!host_leaves) explicit_fetch_leaves(this);
        return leaves_;
    }
    uint64_t* d_leaves = nullptr;
    uint64_t* d_keys = nullptr;     // hash keys (0 = empty)
    uint32_t* d_vals = nullptr;     // global index
    uint64_t mask = 0;
    uint64_t* d_bits = nullptr;     // rank bitmap over the id space (instead of the hash)
    uint32_t* d_rank = nullptr;     // leaves before each 64-bit word
    uint64_t nwords = 0;
    Partition part;                 // over level-0 cells
    std::vector<uint64_t> local_;   // ascending local ids (several ranks)
    const std::vector<uint64_t>& local() const { return one_rank ? leaves() : local_; }
    uint64_t n_local() const { return one_rank ? n : local_.size(); }
    std::vector<uint32_t> local_g;  // their global indices (several ranks)
    std::vector<int32_t> owner;     // process of each leaf (level-0 ancestor's, dccrg.hpp:8098-8145;
                                    // several ranks: with one every leaf is rank 0's)
    uint32_t* d_local_g = nullptr;
    // Storage (per rank, not replicated): slots [0, nl) hold the local cells
    // in ascending id order, then ghost copies of remote neighbors (of every
    // neighborhood), then the data of retired cells.  Fields are sized for
    // these slots only, as the reference stores data only for local cells and
    // remote neighbors (dccrg.hpp:7238, 7330).
    std::vector<uint64_t> slot_ids_;                // id held by each slot (one rank: by each slot >= n)
    uint64_t n_slot_ids() const { return one_rank ? n + slot_ids_.size() : slot_ids_.size(); }
    uint64_t slot_id(uint64_t k) const
    {
        if (!one_rank) return slot_ids_[k];
        return k < n ? leaves()[k] : slot_ids_[k - n];
    }
    void push_slot(uint64_t c) { slot_ids_.push_back(c); }
    void truncate_slots(uint64_t ns) { slot_ids_.resize(one_rank ? ns - n : ns); }
    FlatMap32 extra;                                // ghost id -> slot
    std::vector<uint32_t> slot_of_g;                // global leaf index -> slot (NO_SLOT; several ranks)
    bool slot_identity = false;                     // one rank: leaf g in slot g, local_g[g] == g (no host maps)
    uint32_t* d_slot_of_g = nullptr;
    uint32_t* d_local_slot = nullptr;               // local position -> slot (identity)
    uint8_t* d_level = nullptr;                     // refinement level of each slot
    uint64_t d_level_n = 0, d_level_cap = 0;        // levels written, capacity
    bool defer_fields = false;                      // rebuild(): fields are moved afterwards
    struct HoodLists {
        // host copies (explicit_host_lists), made on first use after a build
        bool host_valid = false;
        std::vector<uint64_t> h_nof_row, h_nto_row;
        std::vector<uint32_t> h_nof_g, h_nto_g;
        // single rows fetched for the refinement decisions (explicit_fetch_rows):
        // leaf -> (neighbors_of offset, length, neighbors_to offset, length) in vals
        std::unordered_map<uint32_t, std::array<uint64_t, 4>> row_at;
        std::vector<uint32_t> row_vals;
        std::vector<uint32_t> inner_pos, outer_pos;  // positions in `local`
        bool inner_all = false;                      // one rank: every local cell inner (inner_pos not stored)
        uint32_t* d_inner_pos = nullptr;
        uint32_t* d_outer_pos = nullptr;
        uint32_t* d_all_pos = nullptr;
    };
    std::map<int32_t, HoodLists> hl;
    // host lookups into `leaves` (the AMR request filters and stop_refining
    // query it millions of times per adaptive step): a bucket directory over
    // the id range -- dir[b] = first leaf whose bucket is >= b, ~0.5 leaves
    // per bucket -- narrows each search to a bucket
    // (built on the first lookup after the leaf list changes: an adaptive
    // step on one rank often needs none)
    mutable std::vector<uint32_t> dir;
    mutable uint64_t dir_base = 0;
    mutable int dir_shift = 0;
    mutable bool dir_valid = false;
    void build_dir() const
    {
        dir_valid = true;
        dir.clear();
        const std::vector<uint64_t>& leaves = this->leaves();
        if (leaves.empty()) return;
        dir_base = leaves.front();
        const uint64_t span = leaves.back() - dir_base + 1;
        uint64_t nb = 16;
        while (nb < 2 * leaves.size() && nb < (1ull << 30)) nb <<= 1;
        dir_shift = 0;
        while ((span >> dir_shift) >= nb) dir_shift++;
        nb = (span >> dir_shift) + 1;
        dir.assign(nb + 1, (uint32_t)leaves.size());
        uint64_t b = 0;
        for (size_t i = 0; i < leaves.size(); i++) {
            const uint64_t bi = (leaves[i] - dir_base) >> dir_shift;
            while (b <= bi) dir[b++] = (uint32_t)i;
        }
    }
    // row of leaf g in the neighborhood CSRs, which hold the local cells' rows
    // by local position (= storage slot); -1 for a leaf of another process
    int64_t row_of(uint64_t g) const
    {
        if (slot_identity) return (int64_t)g;
        const uint32_t s = slot_of_g[g];
        return s < n_local() ? (int64_t)s : -1;
    }
    int64_t find(uint64_t c) const  // global index of a leaf, -1 if none
    {
        if (!dir_valid) build_dir();
        const std::vector<uint64_t>& leaves = this->leaves();
        if (dir.empty() || c < dir_base || c > leaves.back()) return -1;
        const uint64_t b = (c - dir_base) >> dir_shift;
        const auto lo = leaves.begin() + dir[b], hi = leaves.begin() + dir[b + 1];
        const auto it = std::lower_bound(lo, hi, c);
        return (it != hi && *it == c) ? (int64_t)(it - leaves.begin()) : -1;
    }
    // data of cells removed by the last stop_refining (refined parents and
    // unrefined children of this rank), readable until
    // clear_refined_unrefined_data (dccrg.hpp:3519-3543, 5550-5567): ascending
    // ids, stored in slots after the ghosts
    std::vector<uint64_t> retired;
    uint64_t ret_slot0 = 0;  // retired[i] is in slot ret_slot0 + i
    int64_t retired_slot(uint64_t id) const
    {
        const auto it = std::lower_bound(retired.begin(), retired.end(), id);
        return it != retired.end() && *it == id ? (int64_t)(ret_slot0 + (it - retired.begin())) : -1;
    }
    // their device copy for slot lookups (amr_dev.hip): ids ascending, then
    // the slot of each (n_ret of each), made by the rebuild that retired them
    uint64_t* d_ret = nullptr;
    uint64_t n_ret = 0;
    // after them in the same allocation: an open-addressing table id -> slot
    // of the same cells (ret_hcap keys, 0 = empty, then ret_hcap slots), so a
    // kernel finds a retired cell's slot in one or two probes instead of a
    // binary search (the data rules of new and removed cells)
    uint64_t ret_hcap = 0;
};

// stop_refining between its two phases (amr.hip)
struct StopTxn;

// pending refinement requests of this rank and the results of the last
// stop_refining (dccrg.hpp:7355-7360, 3483-3543)
struct LoadState;

struct Amr {
    // host view of the four sets (single request calls, amr_requests)
    FlatSet to_refine, not_to_refine, to_unrefine, not_to_unrefine;
    std::vector<uint64_t> new_cells, removed;
    // device view (explicit grids, amr_dev.hip): RF_* flags over the current
    // leaves, and the dont_refine ids that are not leaves.  Each view is
    // refreshed from the other when it is next used.
    uint32_t* d_flags = nullptr;
    uint64_t flags_n = 0, flags_cap = 0;
    std::vector<uint64_t> nr_other;
    bool host_current = true, dev_current = false;
    bool dev_unrefines = true;  // the flags may hold cells_to_unrefine (else erasing them is skipped)
    StopTxn* pending = nullptr;  // a prepared stop_refining awaiting commit or abort
    ~Amr() { (void)dx_free(d_flags); }
};
// a two-phase stop_refining is between prepare and finish: calls that would
// change or read the fields, neighborhoods or halo plans the prepared rebuild
// has already moved must wait for dccrgx_stop_refining_finish
// calls a hybrid grid (hybrid.hip) does not support yet
#define DX_NO_HYBRID(grid)                                                                                   \
    DX_CHECK(!((grid) && (grid)->hy), DCCRGX_ESTATE,                                                         \
             "not supported on a uniform grid with refined cells (hybrid layout, first slice: game of life, " \
             "cell data by id, neighbor queries, level-0 refines and unrefines back to level 0)")
#define DX_NOT_PENDING(grid)                                                                           \
    DX_CHECK(!((grid) && (grid)->amr && (grid)->amr->pending), DCCRGX_ESTATE,                                      \
             "a prepared stop_refining awaits dccrgx_stop_refining_finish")
// amr.hip: the grid's refinement state, made on first use
Amr& amr_state(dccrgx_grid* grid);
// amr_dev.hip
int amr_dev_sync(dccrgx_grid* grid);
int amr_host_sync(dccrgx_grid* grid);
int amr_dev_requests(dccrgx_grid* grid, int32_t kind, const uint64_t* ids, size_t n, int32_t* results);
int amr_dev_requests_ex(dccrgx_grid* grid, int32_t kind, const uint64_t* ids, const uint64_t* dev_ids, size_t n,
                        int32_t* results);
int amr_dev_requests_many(dccrgx_grid* grid, int nk, const int32_t* kinds, const uint64_t* const* ids,
                          const uint64_t* const* dev_ids, const size_t* counts, int32_t* const* results);
int amr_dev_decide(dccrgx_grid* grid, uint64_t** d_leaves_out, uint64_t* n_out, uint64_t* first_out,
                   std::vector<uint64_t>& leaves_host,
                   std::vector<uint64_t>& retired, std::vector<uint64_t>& nr, bool* changed);
// the retired cells' device lookup table (after their slots were assigned)
int amr_dev_retired_table(dccrgx_grid* grid);
// new cells take their parent's value / parents of removed cells the average
// of their children, on the device (tests/advection/adapter.hpp:229-300)
int amr_dev_copy_from_parents(dccrgx_grid* grid, const int32_t* fields, size_t nf);
int amr_dev_average_children(dccrgx_grid* grid, const int32_t* fields, size_t nf);
// both, copies first (one upload, one error read-back)
int amr_dev_data_rules(dccrgx_grid* grid, const int32_t* fields, size_t nf);
// ordered compaction of local cells by code (1..3) into three host lists
int amr_dev_codes_to_lists(dccrgx_grid* grid, const uint8_t* d_code, uint64_t n, uint64_t* out[3], size_t counts[3]);
int amr_dev_codes_to_device_lists(dccrgx_grid* grid, const uint8_t* d_code, uint64_t n, uint64_t* d_out,
                                  uint64_t* dev[3], size_t counts[3]);


struct CopySeg {
    uint64_t dst, src, n;  // contiguous slot run
};

// explicit grids: the face neighbors among a neighborhood's stencil rows,
// per local cell (built on first use by the advection solver, advect.hip).
// The first 6 faces of a cell are stored column-major ([k][local position],
// slot or UINT32_MAX) so a wavefront's loads of face k are independent and
// coalesced; faces beyond 6 (next to finer cells) go to a CSR overflow.
struct FaceCache {
    uint64_t n = 0;
    uint32_t* ell_slot = nullptr;  // 6 columns: the face neighbor in direction -x, +x, -y, +y, -z, +z
    // further face neighbors of cell q: o_cnt[q] entries from o_base[q] (the
    // neighborhood's stencil row offsets: a row's overflow is a subset of it)
    const uint64_t* o_base = nullptr;
    uint32_t* o_cnt = nullptr;
    uint32_t* o_slot = nullptr;
    int8_t* o_dir = nullptr;
    uint32_t* d_over = nullptr;    // device flag: some cell has overflow
    ~FaceCache();
};

// the device user-stencil view's data (stencil.hip, dccrgx_stencil_view_get),
// made on first use after a structural change
struct IterCache {
    int32_t* items = nullptr;      // uniform: 8 per item (a, b, c, mirror, x, y, z, 0), iteration order
    int64_t* delta = nullptr;      // uniform: slot distance of each item
    int32_t reach[3] = {0, 0, 0};  // uniform: largest |item component| per canonical axis
    int32_t shape = 0;             // uniform: DCCRGX_SHAPE_* flags of the items in iteration order
    uint32_t* slot = nullptr;      // explicit: stencil rows regrouped into iteration order
    int32_t* off = nullptr;
    ~IterCache();
};

struct Hood {
    int32_t id = 0;
    std::vector<int32_t> items;    // original (x, y, z) items, hood_of
    std::vector<int32_t> of_c;     // canonical hood_of
    std::vector<int32_t> to_c;     // canonical hood_to = -hood_of (dccrg.hpp:8070-8075)
    int32_t* d_of_c = nullptr;
    int32_t* d_to_c = nullptr;
    int32_t K = 0;
    bool cube1 = false;            // the full 26-item cube: fast stencil path
    int32_t count_cube = -1;       // the full cube of this length (closed-form neighbor counts), else -1
    bool count_faces = false;      // the six face items (closed-form counts)
    // classification, dccrg.hpp:9131-9409
    std::vector<uint64_t> outer;   // ascending
    std::vector<uint64_t> remote;  // ascending
    std::vector<PeerPlan> peers;   // ascending peer rank
    // periodic self copies into pad slots
    std::vector<CopySeg> self_segs;  // contiguous runs (memcpy)
    uint64_t n_self_scatter = 0;     // non-contiguous remainder (kernel)
    uint64_t* d_self_dst = nullptr;
    uint64_t* d_self_src = nullptr;
    std::vector<std::pair<uint64_t, uint64_t>> h_self;  // all (dst, src) self copies
    VarPlans var_self;                                   // their segments per variable-size field
    // slice ranges for the overlap split (storage slice indices, inclusive-exclusive)
    int64_t inner_s0 = 0, inner_s1 = 0;  // fully local and only local reads
    bool pending = false;                // halo started, not waited
    std::vector<int32_t> pending_fields; // fields of the started halo
    // explicit (mixed-level) grids: device CSR over ALL leaves (global index
    // rows), as the reference keeps lists for every cell (dccrg.hpp:8371-8397)
    uint64_t n_rows = 0;
    uint64_t* d_nof_row = nullptr;   // neighbors_of, reference list order
    uint64_t* d_nof_id = nullptr;
    int32_t* d_nof_off = nullptr;    // x, y, z offsets in indices
    uint32_t* d_nof_g = nullptr;     // global leaf index of each entry
    uint64_t* d_nto_row = nullptr;   // neighbors_to, ascending
    uint32_t* d_nto_g = nullptr;
    // stencil rows of local cells: iteration-cache neighbors_of (unique
    // (id, offset) pairs, dccrg.hpp:11570-11712) as storage slots
    uint64_t* d_st_row = nullptr;
    uint32_t* d_st_slot = nullptr;
    uint64_t st_cap = 0;             // entries d_st_slot / d_st_off hold (>= the rows' total)
    int32_t* d_st_off = nullptr;     // x, y, z offset of each stencil entry
    std::shared_ptr<FaceCache> faces;  // advection face lists (explicit grids)
    std::shared_ptr<IterCache> iter;   // user-stencil view (stencil.hip)
};

// Refinement inside a uniform grid (hybrid.hip): the level-0 cells stay in
// the implicit slab layout; refined level-0 cells' children get slots after
// it; the "overlay" -- the leaves whose rows involve a refined cell -- keeps
// its rows (built by an explicit grid over a box of leaves around the refined
// cells), every other leaf's rows stay closed-form.  One process, the
// default neighborhood, refinement of level-0 cells only (first slice).
struct Hybrid {
    std::vector<uint64_t> refined;      // refined level-0 cells, ascending
    std::vector<uint64_t> children;     // their children (the level-1 leaves), ascending
    std::vector<uint64_t> child_slot;   // the storage slot of each
    uint64_t uniform_slots = 0;         // slots of the uniform layout (children after them)
    std::vector<uint64_t> overlay;      // ascending leaves whose rows involve a refined cell
    std::vector<uint32_t> ov_slot;      // the slot of each
    // their iteration-cache rows (dccrg.hpp:11570-11712) as storage slots, host and device
    std::vector<uint64_t> st_row;
    std::vector<uint32_t> st_slot;
    uint64_t* d_st_row = nullptr;
    uint32_t* d_st_slot = nullptr;
    uint32_t* d_ov_slot = nullptr;
    // their neighbors_of (ids, offsets) and neighbors_to (ids) rows, host
    std::vector<uint64_t> nof_row, nof_id, nto_row, nto_id;
    std::vector<int32_t> nof_off;
    int64_t find_child(uint64_t id) const
    {
        const auto it = std::lower_bound(children.begin(), children.end(), id);
        return it != children.end() && *it == id ? (int64_t)(it - children.begin()) : -1;
    }
    int64_t find_overlay(uint64_t id) const
    {
        const auto it = std::lower_bound(overlay.begin(), overlay.end(), id);
        return it != overlay.end() && *it == id ? (int64_t)(it - overlay.begin()) : -1;
    }
    bool is_refined(uint64_t id) const { return std::binary_search(refined.begin(), refined.end(), id); }
};
// an explicit grid over a box of leaves cut from a larger grid (grid.hip)
int grid_create_box(dccrgx_ctx* ctx, const dccrgx_grid_params* prm, const uint64_t* leaves, size_t n,
                    dccrgx_grid** out);
// refine level-0 `cells` (ascending, unique leaves) of a uniform grid in place
// level-0 refines (cells) and unrefines of level-1 groups (their level-0
// parents) of a hybrid grid: new_cells the children made, removed the
// children removed, both ascending
int hybrid_adapt(dccrgx_grid* grid, const std::vector<uint64_t>& cells, const std::vector<uint64_t>& unrefine,
                 std::vector<uint64_t>& new_cells, std::vector<uint64_t>& removed);
// a level-1 cell's level-0 parent and its 8 children (x fastest)
void hybrid_group(const dccrgx_grid* grid, uint64_t child, uint64_t* parent, uint64_t sib[8]);
void hybrid_destroy(dccrgx_grid* grid);
// storage slot of a leaf of a hybrid grid, -1 if the id is not a leaf
int64_t hybrid_slot(const dccrgx_grid* grid, uint64_t id);
// the overlay's game-of-life fix-up after the uniform kernel (gol.hip)
int hybrid_gol(const dccrgx_grid* grid, const void* in, void* out, void* cnt, hipStream_t st);
// neighbors_of / neighbors_to queries of a hybrid grid (device arrays)
int hybrid_neighbors(const dccrgx_grid* grid, int32_t hood_id, bool to, const uint64_t* cells, size_t n,
                     uint64_t* row, uint64_t* ids, int32_t* off3, size_t cap, hipStream_t st);
// local cells of a hybrid grid: count, and values in ascending id order <-> slots
uint64_t hybrid_n_local(const dccrgx_grid* grid);
int hybrid_local_copy(const dccrgx_grid* grid, const Field& F, void* host, bool to_device);
// local cells (ascending) of a hybrid grid
int hybrid_local_cells(const dccrgx_grid* grid, std::vector<uint64_t>& out);
// would the explicit layout of this uniform grid exceed the device (amr.hip)
bool explicit_too_large(const dccrgx_grid* grid);

// the SFC placement of a grid (sfc.hip): O(P) state, no per-cell table
struct SfcPlan {
    std::vector<uint64_t> cut;  // cut[r-1]: Hilbert key of process r's first level-0 cell
    int32_t bits = 0;
    uint64_t length[3] = {0, 0, 0};
    Divider div_lx{}, div_lxly{};
    bool enabled = false;
    bool on() const { return enabled; }
    // the cuts as kernels and host code read them (cut_ptr: host or device copy)
    SfcCuts view(const uint64_t* cut_ptr = nullptr) const
    {
        SfcCuts s{};
        s.cut = cut_ptr ? cut_ptr : cut.data();
        s.ncut = (int32_t)cut.size();
        s.bits = bits;
        s.lx = length[0];
        s.ly = length[1];
        s.div_lx = div_lx;
        s.div_lxly = div_lxly;
        return s;
    }
};
// the placement of `length`'s level-0 cells over comm_size processes (host
// arithmetic over the curve, no device work and no per-cell memory)
int sfc_plan(const uint64_t length[3], int comm_size, SfcPlan& out);

// a rebuild built but not yet adopted (amr.hip rebuild_prepare): the new leaf
// state, neighborhoods and field arrays, held aside while the grid is still
// the old one
struct RebuildTxn {
    Explicit* ex = nullptr;
    std::map<int32_t, Hood> hoods;
    bool uniform = false;
    uint64_t n_local = 0, first_local = 0, n_slots = 0, old_n_slots = 0;
    std::vector<void*> np;    // new array of each field
    std::vector<size_t> cap;  // its capacity in bytes
};

}  // namespace dccrgx

struct dccrgx_grid {
    dccrgx::Ctx* ctx = nullptr;
    dccrgx_grid_params params{};
    dccrgx::MapParams map{};
    bool uniform = true;
    dccrgx::UGeom g{};
    uint64_t n_local = 0, first_local = 0, n_slots = 0;
    std::vector<dccrgx::Field> fields;
    std::map<int32_t, dccrgx::Hood> hoods;
    // explicit grids (explicit.hip)
    dccrgx::Explicit* ex = nullptr;
    // refinement requests and results (amr.hip)
    dccrgx::Amr* amr = nullptr;
    // grid data file being loaded (checkpoint.hip)
    dccrgx::LoadState* load = nullptr;
    // device buffers kept for reuse by the next AMR rebuild (ptr, bytes)
    std::vector<std::pair<void*, size_t>> spare_bufs;
    // host arrays of the previous explicit state, reused by the next rebuild
    // (their capacity: an adaptive run rebuilds every step at similar sizes,
    // and fresh multi-MB vectors cost page faults)
    dccrgx::Explicit* spare_host = nullptr;
    bool rebuilding = false;  // inside amr.hip rebuild_prepare: intermediate synchronisations are skipped
    // refined cells inside a uniform grid (hybrid.hip), or null
    dccrgx::Hybrid* hy = nullptr;
    // the leaves are a box cut from a larger grid (hybrid.hip's box grid):
    // windows outside the box are skipped instead of reported
    bool partial_leaves = false;
    // SFC placement (params.partition): the P - 1 cut keys along the curve
    dccrgx::SfcPlan sfc;
    uint64_t* d_sfc_cut = nullptr;  // their device copy (AMR decisions), made on first use
    // kernel timing (dccrgx_kernel_timer)
    hipEvent_t t0 = nullptr, t1 = nullptr;
    double timed_ms = 0;
    uint64_t timed_launches = 0;
};

namespace dccrgx {
// process of a level-0 cell: the SFC cuts if the grid has them, else the
// block partition P (dccrg.hpp:8098-8145)
inline int level0_owner(const dccrgx_grid* g, const Partition& P, uint64_t l0)
{
    return g->sfc.on() ? sfc_owner(g->sfc.view(), l0) : part_owner(P, l0);
}
Hood* find_hood(dccrgx_grid* g, int32_t id);
const Hood* find_hood(const dccrgx_grid* g, int32_t id);
int build_hood(dccrgx_grid* g, Hood& h);
void free_hood(Hood& h);
int gol_launch(dccrgx_grid* grid, const Hood& h, const Field& in, const Field& out,
               const Field& cnt, int64_t s0, int64_t s1, hipStream_t st);
// uniform grids: storage slice ranges [r[i][0], r[i][1]) of a region
// (DCCRGX_REGION_*; outer cells may form two runs), gol.hip
void region_slices(const dccrgx_grid* grid, const Hood& h, int32_t region, int64_t r[2][2]);
// explicit grids: local cells of a region as positions into the local list
struct ExRegion {
    const uint32_t* pos = nullptr;         // positions in the local cell list
    uint64_t n = 0;
    const uint32_t* local_slot = nullptr;  // local position -> storage slot
    const uint8_t* level = nullptr;        // storage slot -> refinement level
};
constexpr uint32_t NO_SLOT = 0xffffffffu;
int explicit_region(const dccrgx_grid* grid, const Hood& h, int32_t region, ExRegion* out);
// storage slot of each id (-1: none), on the device
int explicit_slots_of(const dccrgx_grid* grid, const uint64_t* ids, size_t n, int64_t* slots, hipStream_t st);
// explicit (mixed refinement level) grids, explicit.hip
int explicit_create(dccrgx_grid* grid, const uint64_t* leaves, size_t n);
void explicit_destroy(dccrgx_grid* grid);
void explicit_free(Explicit* E);
// free E's device memory and keep its host arrays for the next explicit_init
void explicit_recycle(dccrgx_grid* grid, Explicit* E);
void explicit_clear_retired(Explicit* E);
// explicit grids: give `ids` (leaves or retired cells) storage slots if they
// have none, growing every field unless a rebuild defers that
int explicit_add_slots(dccrgx_grid* grid, const std::vector<uint64_t>& ids);
// rebuild(): slots after the ghosts for the retired cells (ascending, unique,
// no leaves), in their order; E->retired becomes `ids`
int explicit_add_retired(dccrgx_grid* grid, const std::vector<uint64_t>& ids);
// rebuild(): old slot (or -1) of every slot of the new layout, device output
int explicit_old_slots(const dccrgx_grid* grid, const Explicit* old, int64_t* d_src, hipStream_t st);
// dst[k] = src[from[k]], or zero where from[k] < 0
int launch_move(const void* src, const int64_t* from, uint64_t n, uint32_t elem, void* dst, hipStream_t st);
// the same for several fields (8-byte elements share one pass over `from`)
int launch_move_many(const void* const* src, void* const* dst, const uint32_t* elem, size_t nf, const int64_t* from,
                     uint64_t n, hipStream_t st);
// the previous leaf set's lists of the same neighborhood and which of its
// leaves are gone (flags & gone_bit): rows of kept leaves that reference no
// gone leaf are copied from `old_h` instead of recomputed (amr.hip rebuild)
constexpr uint32_t AMR_FLAG_GONE = 16u;  // amr_dev.hip RF_GONE: the leaf disappears in the rebuild
struct NofHint {
    const Explicit* old_ex;
    const Hood* old_h;
    const uint32_t* old_flags;
    uint32_t gone_bit;
};
int explicit_build_hood(dccrgx_grid* grid, Hood& h, const NofHint* hint = nullptr);
// the same without the final synchronisation (the caller synchronises: rebuild)
int explicit_build_hood_async(dccrgx_grid* grid, Hood& h, const NofHint* hint = nullptr);
// host copies of a neighborhood's neighbor lists, fetched once per build
int explicit_host_lists(const dccrgx_grid* grid, const Hood& h);
int explicit_host_lists(const dccrgx_grid* grid, int32_t hood_id);
// the neighbors_of / neighbors_to rows of the given leaves (global indices)
// copied to the host row cache of the neighborhood, one gather for all
int explicit_fetch_rows(const dccrgx_grid* grid, const Hood& h, const std::vector<uint32_t>& leaves);
int explicit_get_cells(const dccrgx_grid* grid, const Hood& h, int32_t which, uint64_t* ids,
                       size_t cap, size_t* n);
int explicit_local_copy(const dccrgx_grid* grid, const Field& F, void* host, bool to_device);
// explicit grid state over an ascending leaf list (no neighborhoods built);
// d_leaves: the same list on the device, adopted by the grid (amr_dev.hip);
// on one rank `leaves` may be null: the device list alone, whose first leaf
// is `first_leaf` (the host copy is fetched when host code asks for it)
int explicit_init(dccrgx_grid* grid, const uint64_t* leaves, size_t n, uint64_t* d_leaves = nullptr,
                  std::vector<uint64_t>* take = nullptr,  // take: the vector holding `leaves`, moved from
                  uint64_t first_leaf = 0);
int64_t explicit_host_slot(const dccrgx_grid* grid, uint64_t id);
// the slot read and written for a cell on this rank (-1: none), halo.hip
int64_t host_primary_slot(const dccrgx_grid* grid, uint64_t id);
void amr_destroy(dccrgx_grid* grid);
void load_state_free(dccrgx_grid* grid);
// switch a uniform grid to the explicit layout (amr.hip)
int amr_ensure_explicit(dccrgx_grid* grid);
// device prefix sums (scan.hip): x[0..m) inclusive in place; CSR rows
// (counts in row[1..n] -> row pointers, row[0] = 0, *total = row[n] if given)
int device_inclusive_scan(uint64_t* x, uint64_t m, hipStream_t st);
int device_scan_rows(uint64_t* row, uint64_t n, hipStream_t st, uint64_t* total);
// row[0] = 0, row[i + 1] = cnt[0] + ... + cnt[i] (row: n + 1 entries)
int device_scan_counts(const uint32_t* cnt, uint64_t n, uint64_t* row, hipStream_t st);
int device_scan_rows_total(const uint64_t* row, uint64_t n, hipStream_t st, uint64_t* total);
int launch_gather_ext(const void* src, const uint64_t* idx, uint64_t n, uint32_t elem, void* dst,
                      hipStream_t st);
int launch_scatter_ext(const void* src, const uint64_t* sidx, const uint64_t* didx, uint64_t n,
                       uint32_t elem, void* dst, hipStream_t st);
}  // namespace dccrgx
