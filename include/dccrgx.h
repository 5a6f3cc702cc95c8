/*
 * dccrgx.h -- C-ABI of the MI355X-native dccrg hot path (libdccrgx.so).
 *
 * The reference (ykempf/dccrg) is a header-only C++ template library with no
 * FFI; its drop-in boundary is the public member-function surface of
 * dccrg::Dccrg<Cell_Data, Geometry> plus dccrg::Mapping.  Each export below
 * names the reference interface it replaces (file:line in the reference
 * tree).  The C++ facade include/dccrg_amd.hpp re-implements those member
 * functions on top of these exports; INTEGRATION.md shows the wiring.
 *
 * Conventions:
 *  - every function returns int status, DCCRGX_OK == 0; no exception crosses
 *    the ABI; dccrgx_last_error() returns a thread-local message;
 *  - plain pointers and sizes only; "_dev" pointers are HIP device memory,
 *    "_host" pointers are host memory; streams are hipStream_t passed as void*
 *    (NULL = the context's compute stream); work the library queues on a
 *    caller's stream is ordered before the library's later frees, rebuilds
 *    and destroys (the compute stream waits for it), but the caller's OWN
 *    kernels that read grid memory (dccrgx_field_device_ptr) must be
 *    synchronised by the caller before a structural or destroy call;
 *  - thread-compatible, not thread-safe: one context per host thread;
 *  - device memory of a grid is owned by the grid (SoA field pools).
 */
#ifndef DCCRGX_H
#define DCCRGX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCCRGX_VERSION 1

enum {
    DCCRGX_OK = 0,
    DCCRGX_EINVAL = 1,      /* bad argument (reference: std::invalid_argument / false) */
    DCCRGX_ENOMEM = 2,      /* device or host allocation failed */
    DCCRGX_EHIP = 3,        /* HIP runtime error */
    DCCRGX_ERCCL = 4,       /* RCCL error */
    DCCRGX_ERANGE = 5,      /* output capacity too small; *n holds the needed size */
    DCCRGX_ESTATE = 6,      /* call not valid in the current state */
    DCCRGX_ENOTFOUND = 7,   /* unknown cell / neighborhood id (reference: nullptr / false) */
    DCCRGX_EINTERNAL = 8    /* inconsistent structure (reference: std::runtime_error) */
};

/* dccrg_mapping.hpp:38-41 */
#define DCCRGX_ERROR_CELL ((uint64_t)0)
#define DCCRGX_ERROR_INDEX ((uint64_t)0xFFFFFFFFFFFFFFFFull)
/* dccrg.hpp:99 default_neighborhood_id */
#define DCCRGX_DEFAULT_NEIGHBORHOOD_ID (-0xdcc)

/* cell classes, dccrg.hpp:7594-7718 (inner/outer/local/remote/all_cells) */
enum { DCCRGX_CELLS_LOCAL = 0, DCCRGX_CELLS_INNER = 1, DCCRGX_CELLS_OUTER = 2,
       DCCRGX_CELLS_REMOTE = 3 };

/* halo wait selectors, dccrg.hpp:5307-5413 */
enum { DCCRGX_WAIT_ALL = 0, DCCRGX_WAIT_RECEIVES = 1, DCCRGX_WAIT_SENDS = 2 };

const char* dccrgx_last_error(void);
int dccrgx_version(void);

/* ------------------------------------------------------------------------ *
 * Context: device, compute + communication streams, RCCL communicator.
 * Replaces Dccrg::initialize_mpi (dccrg.hpp:7738-7803): MPI stays only for
 * bootstrap; the data path communicator is RCCL over xGMI.
 * ------------------------------------------------------------------------ */
typedef struct dccrgx_ctx dccrgx_ctx;

int dccrgx_ctx_create(int device, int rank, int comm_size, dccrgx_ctx** out);
int dccrgx_ctx_destroy(dccrgx_ctx* ctx);
/* 128-byte ncclUniqueId; rank 0 creates it, the host bootstrap broadcasts it */
int dccrgx_get_unique_id(uint8_t uid_out[128]);
int dccrgx_ctx_comm_init(dccrgx_ctx* ctx, const uint8_t uid[128]);
/* Test mode, no reference counterpart: grids created afterwards on this
 * context send a rank's own periodic images through RCCL send/recv to itself
 * (a peer plan with peer == rank) instead of device copies, so the whole
 * multi-rank halo path runs on a single GPU.  Needs dccrgx_ctx_comm_init. */
int dccrgx_ctx_route_self_through_rccl(dccrgx_ctx* ctx, int32_t on);
/* Test options (no reference counterpart): process-wide switches the test
 * suite uses to force a code path the library otherwise picks by size, and
 * fault injection; never read from the environment, all off by default.
 * name: "gol_scalar", "gol_chunk" (slices per workgroup), "poisson_multi",
 * "poisson_solo_global", "incremental" (1 / 0), "ou_small" (queue entries),
 * "full_nto" (1: the full neighbors_to transpose in incremental rebuilds),
 * "hybrid" (1: one-process uniform grids refine in place whatever their size),
 * "ou_walk" (1: override_unrefines walks the face graph, the reference's
 * literal algorithm, instead of the equivalent window test),
 * "corrupt_ghost", "fail_stop_refining" (rank + 1), "check_init"; set = 0
 * returns the option to its default.  DCCRGX_EINVAL for an unknown name, or
 * in a build compiled with -DDCCRGX_NO_TEST_OPTIONS. */
int dccrgx_test_option(const char* name, int64_t value, int32_t set);
/* Host-staged transport for ranks that cannot have an RCCL communicator --
 * several processes sharing one GPU, which RCCL refuses ("Duplicate GPU").
 * With no communicator and a transport set, every halo message of a peer is
 * packed on the device (the same plans as the RCCL path), copied to host
 * memory, and one exchange() call moves all messages of the update between
 * the processes (blocking: it returns when every receive buffer is filled);
 * the received bytes are copied back and unpacked.  allreduce_f64 combines
 * the solvers' scalars across ranks (op: 0 sum, 1 min, 2 max), the
 * MPI_Allreduce of tests/poisson/poisson_solve.hpp:349, 426, 486.  The
 * callbacks return 0 on success.  Pass NULL to remove the transport. */
typedef struct {
    void* user;
    int (*exchange)(void* user, int32_t n_send, const int32_t* send_peers, const void* const* send_bufs,
                    const uint64_t* send_bytes, int32_t n_recv, const int32_t* recv_peers,
                    void* const* recv_bufs, const uint64_t* recv_bytes);
    int (*allreduce_f64)(void* user, double* values, int32_t n, int32_t op);
} dccrgx_host_transport;
int dccrgx_ctx_set_host_transport(dccrgx_ctx* ctx, const dccrgx_host_transport* transport);
int dccrgx_ctx_compute_stream(dccrgx_ctx* ctx, void** hip_stream_out);
int dccrgx_ctx_synchronize(dccrgx_ctx* ctx);

/* ------------------------------------------------------------------------ *
 * Batched cell-id mapping (bit-exact with dccrg::Mapping).
 * ------------------------------------------------------------------------ */
typedef struct {
    uint64_t length[3];   /* Grid_Length, dccrg_length.hpp:34-142 */
    int32_t max_ref_lvl;  /* Mapping::max_refinement_level, dccrg_mapping.hpp:664 */
    int32_t reserved;
} dccrgx_mapping;

/* Mapping::get_maximum_possible_refinement_level, dccrg_mapping.hpp:317-330 */
int dccrgx_max_possible_refinement_level(const uint64_t length[3], int32_t* out);
/* Mapping::get_last_cell / update_last_cell, dccrg_mapping.hpp:500-503, 679-687 */
int dccrgx_last_cell(const dccrgx_mapping* map, uint64_t* out);
/* Mapping::get_indices (dccrg_mapping.hpp:218-254) and get_refinement_level
 * (dccrg_mapping.hpp:262-290) for n ids: idx3_dev[3*i..3*i+2], lvl_dev[i];
 * either output may be NULL. */
int dccrgx_map_ids_to_indices(const dccrgx_mapping* map, const uint64_t* ids_dev, size_t n,
                              uint64_t* idx3_dev, int32_t* lvl_dev, void* stream);
/* Mapping::get_cell_from_indices, dccrg_mapping.hpp:154-209 */
int dccrgx_map_indices_to_ids(const dccrgx_mapping* map, const uint64_t* idx3_dev,
                              const int32_t* lvl_dev, size_t n, uint64_t* ids_dev, void* stream);
/* Octree relations, dccrg_mapping.hpp:298-494: op selects the function */
enum { DCCRGX_OP_LENGTH_IN_INDICES = 0, DCCRGX_OP_PARENT = 1, DCCRGX_OP_LEVEL_0_PARENT = 2,
       DCCRGX_OP_CHILD = 3 };
int dccrgx_map_ids_op(const dccrgx_mapping* map, int op, const uint64_t* ids_dev, size_t n,
                      uint64_t* out_dev, void* stream);

/* Scalar host-side forms of the same functions (no device involved), for
 * host code that calls Mapping per cell (tests/game_of_life/solve.hpp:48-51) */
int dccrgx_map_host_indices(const dccrgx_mapping* map, uint64_t cell, uint64_t idx3_out[3],
                            int32_t* lvl_out);
int dccrgx_map_host_cell(const dccrgx_mapping* map, const uint64_t idx3[3], int32_t lvl,
                         uint64_t* cell_out);
int dccrgx_map_host_op(const dccrgx_mapping* map, int op, uint64_t cell, uint64_t* out);
/* host loops of the two above over an array (host memory) */
int dccrgx_map_host_ids_to_indices(const dccrgx_mapping* map, const uint64_t* ids, size_t n,
                                   uint64_t* idx3_out, int32_t* lvl_out);
int dccrgx_map_host_ids_op(const dccrgx_mapping* map, int op, const uint64_t* ids, size_t n, uint64_t* out);
int dccrgx_device_count(int* n_out);

/* ------------------------------------------------------------------------ *
 * Grid: one dccrg grid on this rank.  Replaces Dccrg::initialize
 * (dccrg.hpp:485-562): level-0 creation + block partition (:8089-8145),
 * neighborhoods (:8017-8076), neighbor lists (:8371-8420), boundary
 * classification (:9131-9409), send/receive lists (:8729-8891) and ghost
 * allocation (:7153-7184) -- all built on the device.
 * ------------------------------------------------------------------------ */
typedef struct dccrgx_grid dccrgx_grid;

typedef struct {
    uint64_t length[3];            /* set_initial_length, dccrg.hpp:8242 */
    int32_t max_ref_lvl;           /* set_maximum_refinement_level (<0: max possible), :8276 */
    uint32_t neighborhood_length;  /* set_neighborhood_length, :8328 */
    uint8_t periodic[3];           /* set_periodic, :8305 */
    uint8_t partition;             /* DCCRGX_PARTITION_*: placement of the level-0 cells */
    uint8_t reserved[4];
} dccrgx_grid_params;

/* Placement of the level-0 cells at initialize (create_level_0_cells,
 * dccrg.hpp:8089-8224).  BLOCK: contiguous ids (:8116-8145, the reference's
 * build without USE_SFC).  SFC: the same per-process counts taken along a
 * space-filling curve (the USE_SFC branch :8147-8220; a Hilbert curve, sfc.hip;
 * sfc++'s own curve is not in the reference tree).  The placement is held as
 * the comm_size - 1 cut keys along the curve, not as a per-cell owner table
 * (the reference's replicated cell_process, :7311): a cell's process is the
 * number of cuts <= the Hilbert key of its level-0 ancestor, on the host and
 * on the device.  An SFC grid always uses the explicit layout. */
enum { DCCRGX_PARTITION_BLOCK = 0, DCCRGX_PARTITION_SFC = 1 };
/* the comm_size - 1 cut keys of the SFC placement: cuts_out[r - 1] = the
 * Hilbert key of process r's first level-0 cell (UINT64_MAX if it has none);
 * host arithmetic over the curve, no per-cell work */
int dccrgx_sfc_cuts(const uint64_t length[3], int32_t comm_size, uint64_t* cuts_out);
/* owner of every level-0 cell (index id - 1) under the SFC placement, from the
 * cuts (a listing for tests and tools; ctx is not used) */
int dccrgx_sfc_owners(dccrgx_ctx* ctx, const uint64_t length[3], int32_t comm_size, int32_t* owner_host);
/* the Hilbert key of every level-0 cell (index id - 1), host computation */
int dccrgx_hilbert_keys_host(const uint64_t length[3], uint64_t* keys_out);

typedef struct {
    uint64_t n_local;        /* cells owned by this rank */
    uint64_t first_local;    /* uniform grids: first owned id (0 if none) */
    uint64_t n_slots;        /* slots per field (local + ghost/pad) */
    uint64_t layout[4];      /* uniform: LA, LB, slices in storage, pad slices */
    int32_t max_ref_lvl;     /* effective maximum refinement level */
    int32_t uniform;         /* 1: implicit uniform level-0 grid */
    int32_t rank, comm_size;
} dccrgx_grid_info;

/* leaves_host == NULL: every refinement-level-0 cell exists (implicit uniform
 * grid, arbitrarily large).  Otherwise the replicated set of existing leaf
 * cells (mixed refinement levels); each cell is owned by the rank owning its
 * level-0 parent under params->partition (block or SFC). */
int dccrgx_grid_create(dccrgx_ctx* ctx, const dccrgx_grid_params* params,
                       const uint64_t* leaves_host, size_t n_leaves, dccrgx_grid** out);
int dccrgx_grid_destroy(dccrgx_grid* grid);
int dccrgx_grid_get_info(const dccrgx_grid* grid, dccrgx_grid_info* out);
/* the device neighbor lists neighborhood `hood_id` holds on this rank
 * (explicit grids; the reference keeps neighbors_of / neighbors_to of every
 * cell on every process, dccrg.hpp:8371-8397): out[0] = rows held (this
 * rank's local cells), out[1] = neighbors_of entries, out[2] = neighbors_to
 * entries, out[3] = device bytes of the lists and stencil rows.  Uniform
 * grids store none (closed-form rows): zeros. */
int dccrgx_neighbor_list_stats(const dccrgx_grid* grid, int32_t hood_id, uint64_t out[4]);

/* Dccrg::get_process (dccrg.hpp:5886-5902) for n cells on the host: the
 * process owning each existing cell (the replicated cell_process), -1 for a
 * cell that does not exist */
int dccrgx_get_process(const dccrgx_grid* grid, const uint64_t* cells, size_t n, int32_t* process_out);

/* Dccrg::add_neighborhood / remove_neighborhood, dccrg.hpp:6491-6711
 * (validation as :6573-6618: returns DCCRGX_EINVAL when the reference returns false) */
int dccrgx_add_neighborhood(dccrgx_grid* grid, int32_t hood_id, const int32_t* items3,
                            size_t n_items);
int dccrgx_remove_neighborhood(dccrgx_grid* grid, int32_t hood_id);
/* the neighborhood items (3 ints each) */
int dccrgx_get_neighborhood(const dccrgx_grid* grid, int32_t hood_id, int32_t* items3_out,
                            size_t cap, size_t* n);

/* local/inner/outer/remote cells (dccrg.hpp:7594-7718), ascending ids, host
 * output.  DCCRGX_ERANGE with *n = needed size if cap is too small. */
int dccrgx_get_cells(const dccrgx_grid* grid, int32_t hood_id, int32_t which, uint64_t* ids_host,
                     size_t cap, size_t* n);

/* Dccrg::get_all_cells (dccrg.hpp:3557-3590): every existing leaf cell of the
 * grid (the replicated leaf set; uniform grids: 1..N), ascending, host output.
 * DCCRGX_ERANGE with *n = needed size if cap is too small. */
int dccrgx_get_all_cells(const dccrgx_grid* grid, uint64_t* ids_host, size_t cap, size_t* n);
/* Dccrg::get_neighbors_of (dccrg.hpp:836-883 / find_neighbors_of :4375-4716)
 * for n cells in one batch, computed on the device: CSR in reference list
 * order.  row_ptr_dev has n+1 entries; call with ids_dev == NULL to size. */
int dccrgx_neighbors_of(const dccrgx_grid* grid, int32_t hood_id, const uint64_t* cells_dev,
                        size_t n, uint64_t* row_ptr_dev, uint64_t* ids_dev, int32_t* off3_dev,
                        size_t cap, void* stream);
/* Neighbor gather for user stencils (the iteration cache's neighbor data,
 * Neighbors_Item::data, dccrg.hpp:7404-7456, in get_neighbors_of order): for
 * n LOCAL cells, row pointers as dccrgx_neighbors_of and the element of
 * field_id of every neighbors_of entry, elem bytes each, ghosts read from
 * their copies (update them first).  out == NULL: rows only.
 * DCCRGX_ENOTFOUND if a cell is not local. */
int dccrgx_gather_neighbors(const dccrgx_grid* grid, int32_t hood_id, int32_t field_id, const uint64_t* cells_dev,
                            size_t n, uint64_t* row_ptr_dev, void* out_dev, size_t cap_bytes, void* stream);
/* Device user stencils: the reference's loop over a region's cells and each
 * cell's neighbors_of (examples/game_of_life.cpp:54-79; the iteration cache's
 * Cells_Item / Neighbors_Item {id, data, x, y, z}, dccrg.hpp:7395-7456 and
 * the local/inner/outer cell ranges, :11570-11712) as plain device data that
 * include/dccrgx_stencil.hpp's for_each_cell() launches a caller's device
 * functor over, one thread per cell.  Neighbors come in the iteration cache's
 * order: unique (id, offset) pairs, those that are not also neighbors_to
 * first, each group by ascending (id, x, y, z) (dccrg.hpp:11590-11640).
 * Uniform grids: neighbors in closed form from the canonical geometry
 * (nothing stored); explicit grids: the stencil rows, regrouped into that
 * order on the first call after a structural change.  Neighbor data
 * is read from the field arrays of dccrgx_field_device_ptr at the neighbor's
 * slot (remote neighbors: their ghost copies -- update them first).  Valid
 * until the next structural call (refine, load, new neighborhood).  Regions
 * as dccrgx_gol_compute's: on uniform grids DCCRGX_REGION_INNER is the whole
 * slices whose cells read no ghost copy (a subset of the reference's inner
 * cells) and DCCRGX_REGION_OUTER the rest of the local cells. */
/* dccrgx_stencil_view.shape flags (uniform grids): every item's mirror is an
 * item too (each neighbor is also a neighbor_to); the items are the 26-cell
 * cube of reach 1 / the 6 face items, in their iteration order (the staged
 * launches of include/dccrgx_stencil.hpp then use compile-time offsets) */
enum { DCCRGX_SHAPE_SYMMETRIC = 1, DCCRGX_SHAPE_CUBE1 = 2, DCCRGX_SHAPE_FACES = 4 };
typedef struct dccrgx_stencil_view {
    int32_t kind;     /* 0 uniform (closed form), 1 explicit (stored rows) */
    int32_t n_items;  /* uniform: neighborhood items */
    uint64_t n_cells; /* cells of the region */
    void* stream;     /* the grid's compute stream */
    /* uniform: canonical axes (a fastest, c the partitioned one) */
    uint64_t la, lb, lc;
    uint64_t lo, hi;       /* local range of id - 1 */
    int64_t cbase;         /* canonical slice in storage slice 0 */
    int64_t s0[2], s1[2];  /* storage slice ranges [s0, s1) of the region */
    int32_t per[3];        /* canonical periodicity */
    int32_t perm[3];       /* canonical axis -> x / y / z */
    int32_t scale;         /* offsets in indices of the finest level: 2^max_ref_lvl */
    int32_t reach[3];      /* largest |item component| per canonical axis */
    int32_t nslices;       /* storage slices (local and ghost), la * lb slots each */
    int32_t shape;         /* uniform: DCCRGX_SHAPE_* flags of the items (staged launches) */
    /* n_items x 8 int32, device, in the iteration cache's order for a cell no
     * periodic wrap reaches: canonical (a, b, c) of each item, 1 if its mirror
     * is an item too (the neighbor is also a neighbor_to), the x, y, z offset
     * in indices, 0 */
    const int32_t* items;
    /* n_items int64, device: the slot distance of each item for a cell no
     * grid boundary reaches (a + la * b + la * lb * c) */
    const int64_t* item_delta;
    /* explicit: stencil rows in the iteration cache's order */
    const uint32_t* pos;        /* local positions of the region's cells */
    const uint32_t* local_slot; /* local position -> storage slot */
    const uint32_t* local_g;    /* local position -> leaf index */
    const uint64_t* leaves;     /* leaf ids, ascending */
    const uint64_t* row;        /* stencil rows by local position (n_local + 1) */
    const uint32_t* nbr_slot;   /* storage slot of each entry */
    const int32_t* nbr_off;     /* x, y, z offset of each entry, in indices */
} dccrgx_stencil_view;
int dccrgx_stencil_view_get(const dccrgx_grid* grid, int32_t hood_id, int32_t region, dccrgx_stencil_view* out);
/* Dccrg::get_face_neighbors_of (dccrg.hpp:2828-2955) for n cells: the face
 * graph (update_neighbors_, :9463-9597) neighbor in -x,+x,-y,+y,-z,+z order
 * plus, for a smaller neighbor, its 3 siblings sharing the face; dirs_dev
 * gets -1/+1/-2/+2/-3/+3.  CSR like dccrgx_neighbors_of (<= 24 per cell);
 * DCCRGX_ENOTFOUND if a cell is not an existing leaf (the reference aborts). */
int dccrgx_face_neighbors_of(const dccrgx_grid* grid, const uint64_t* cells_dev, size_t n,
                             uint64_t* row_ptr_dev, uint64_t* ids_dev, int32_t* dirs_dev, size_t cap,
                             void* stream);
int dccrgx_face_neighbors_of_host(const dccrgx_grid* grid, const uint64_t* cells, size_t n,
                                  uint64_t* row_ptr, uint64_t* ids, int32_t* dirs, size_t cap);
/* Dccrg::get_neighbors_to (dccrg.hpp:900-943 / find_neighbors_to :4744-4897),
 * unique ids per cell in ascending order (the reference: unordered). */
int dccrgx_neighbors_to(const dccrgx_grid* grid, int32_t hood_id, const uint64_t* cells_dev,
                        size_t n, uint64_t* row_ptr_dev, uint64_t* ids_dev, size_t cap,
                        void* stream);
/* host-pointer forms of the two batched queries (same results) */
int dccrgx_neighbors_of_host(const dccrgx_grid* grid, int32_t hood_id, const uint64_t* cells_host,
                             size_t n, uint64_t* row_host, uint64_t* ids_host, int32_t* off3_host,
                             size_t cap);
int dccrgx_neighbors_to_host(const dccrgx_grid* grid, int32_t hood_id, const uint64_t* cells_host,
                             size_t n, uint64_t* row_host, uint64_t* ids_host, size_t cap);
/* per-peer ascending send / receive lists (dccrg.hpp:7008-7046, :8729-8891) */
int dccrgx_get_peers(const dccrgx_grid* grid, int32_t hood_id, int32_t send, int32_t* peers_host,
                     uint64_t* counts_host, size_t cap, size_t* n_peers);
int dccrgx_get_peer_cells(const dccrgx_grid* grid, int32_t hood_id, int32_t send, int32_t peer,
                          uint64_t* ids_host, size_t cap, size_t* n);

/* ------------------------------------------------------------------------ *
 * Cell data: device SoA field pools (replace Dccrg::cell_data /
 * remote_neighbors unordered_maps, dccrg.hpp:7238, 7330).
 * ------------------------------------------------------------------------ */
int dccrgx_field_create(dccrgx_grid* grid, uint32_t elem_bytes, int32_t* field_id_out);
/* valid until the next structural call (refine, load) or, for an advection
 * density field, the next dccrgx_advect_step (double-buffered) */
int dccrgx_field_device_ptr(const dccrgx_grid* grid, int32_t field_id, void** ptr_out,
                            uint64_t* n_slots_out);
/* slot of each cell id in every field (-1: no slot on this rank) */
int dccrgx_slots_of(const dccrgx_grid* grid, const uint64_t* ids_dev, size_t n, int64_t* slots_dev,
                    void* stream);
/* copy local cells' values (ascending id order) between host and device */
int dccrgx_field_write_local(dccrgx_grid* grid, int32_t field_id, const void* host, size_t n_local);
int dccrgx_field_read_local(const dccrgx_grid* grid, int32_t field_id, void* host, size_t n_local);
/* ghost copies of the remote cells of a neighborhood (ascending id order) */
int dccrgx_field_read_remote(const dccrgx_grid* grid, int32_t hood_id, int32_t field_id,
                             void* host, size_t n_remote);

/* ------------------------------------------------------------------------ *
 * Remote-neighbor halo exchange.  Replaces update_copies_of_remote_neighbors
 * (dccrg.hpp:978-1014), start_remote_neighbor_copy_updates (:5046-5078),
 * start_..._receives/_sends (:5091-5298), wait_remote_neighbor_copy_updates
 * (:5307-5338), wait_..._sends/_receives (:5347-5413) and the transfer engine
 * (:10726-11209).  Payload = the listed fields of each cell (the MPI datatype
 * of get_mpi_datatype, dccrg_get_cell_datatype.hpp:48-339, becomes a field
 * list); per peer the cells go in ascending id order as in the reference.
 * ------------------------------------------------------------------------ */
int dccrgx_halo_start(dccrgx_grid* grid, int32_t hood_id, const int32_t* field_ids,
                      size_t n_fields);
int dccrgx_halo_wait(dccrgx_grid* grid, int32_t hood_id, int32_t which);
/* start + wait(ALL) */
int dccrgx_halo_update(dccrgx_grid* grid, int32_t hood_id, const int32_t* field_ids,
                       size_t n_fields);
/* Transport-free halo for several ranks driven from ONE process (tests on a
 * single GPU): pack this rank's sends to peer into dst_dev (field-major,
 * ascending ids) / unpack a peer's message into the ghost slots. */
int dccrgx_halo_pack_to(dccrgx_grid* grid, int32_t hood_id, const int32_t* field_ids,
                        size_t n_fields, int32_t peer, void* dst_dev, size_t cap_bytes,
                        size_t* bytes_out);
int dccrgx_halo_unpack_from(dccrgx_grid* grid, int32_t hood_id, const int32_t* field_ids,
                            size_t n_fields, int32_t peer, const void* src_dev, size_t bytes);
/* Byte transport for host-resident cell data (the C++ facade's drop-in path
 * for arbitrary Cell_Data / MPI datatypes, dccrg.hpp:10726-11209): one
 * message per peer, the peers in dccrgx_get_peers order (send=1 for
 * send_host / send_bytes, send=0 for recv_host / recv_bytes), moved with
 * grouped RCCL send/recv through device staging on the communication
 * stream.  Host buffers must stay valid until dccrgx_exchange_wait. */
int dccrgx_exchange_start(dccrgx_grid* grid, int32_t hood_id, const void* const* send_host,
                          const uint64_t* send_bytes, void* const* recv_host,
                          const uint64_t* recv_bytes);
int dccrgx_exchange_wait(dccrgx_grid* grid, int32_t hood_id);
/* periodic self-copies into the ghost/pad slots (part of halo_start) */
int dccrgx_halo_self(dccrgx_grid* grid, int32_t hood_id, const int32_t* field_ids,
                     size_t n_fields);

/* ------------------------------------------------------------------------ *
 * Variable-size cell data (tests/variable_data_size: a Cell_Data whose
 * get_mpi_datatype describes a per-cell number of elements).  A variable
 * field holds count[cell] elements of elem_bytes per cell, zero-initialised
 * on resize like std::vector::resize.  As in the reference, the receiver
 * sizes its ghost copies before a halo (variable_neighbour_data.cpp:95-102);
 * messages carry each cell's elements in ascending id order.
 * ------------------------------------------------------------------------ */
int dccrgx_field_create_variable(dccrgx_grid* grid, uint32_t elem_bytes, int32_t* field_id);
/* set the element counts of cells this rank stores (local cells or ghosts;
 * all storage copies of a cell follow); keeps the leading elements */
int dccrgx_field_resize(dccrgx_grid* grid, int32_t field_id, const uint64_t* ids,
                        const uint32_t* counts, size_t n);
int dccrgx_field_get_counts(const dccrgx_grid* grid, int32_t field_id, const uint64_t* ids, size_t n,
                            uint32_t* counts);
/* cell-addressed access for any field (operator[], dccrg.hpp:768-781): the
 * cells' elements concatenated in the given order, host buffers; a ghost is
 * read from its first copy.  read with data == NULL returns the size. */
int dccrgx_field_write_cells(dccrgx_grid* grid, int32_t field_id, const uint64_t* ids, size_t n,
                             const void* data, size_t bytes);
int dccrgx_field_read_cells(const dccrgx_grid* grid, int32_t field_id, const uint64_t* ids, size_t n,
                            void* data, size_t cap, size_t* bytes);

/* ------------------------------------------------------------------------ *
 * Stencils over local cells.  Game of life as in examples/game_of_life.cpp:
 * 54-79 / tests/game_of_life/scalability3d.cpp:136-165: count live
 * neighbors_of (u32 is_alive > 0), then B3/S23 (count == 3 -> 1, count != 2
 * -> 0).  Double-buffered: alive_in -> (alive_out, count).
 * ------------------------------------------------------------------------ */
enum { DCCRGX_REGION_ALL = 0, DCCRGX_REGION_INNER = 1, DCCRGX_REGION_OUTER = 2 };
int dccrgx_gol_compute(dccrgx_grid* grid, int32_t hood_id, int32_t f_alive_in,
                       int32_t f_alive_out, int32_t f_count, int32_t region);
/* one full step: halo start, inner cells, halo wait, outer cells (the
 * overlap pattern of scalability3d.cpp:122-166); swaps nothing */
int dccrgx_gol_step(dccrgx_grid* grid, int32_t hood_id, int32_t f_alive_in, int32_t f_alive_out,
                    int32_t f_count);
/* The AMR-aware game of life of tests/game_of_life/solve.hpp:40-170 (=
 * solve_optimized.hpp:40-133, "emulating unrefined behaviour" on refined
 * grids): f_data is the test's Cell::data, 9 x u64 per cell (72-byte
 * field, tests/game_of_life/cell.hpp:47).  RECORD lists the distinct level-0
 * parents of live neighbors in data[1..8]; SPREAD_APPLY merges the lists of
 * cells sharing a level-0 parent, then B3/S23 on the number of parents and
 * resets the lists.  The step is RECORD, update_copies_of_remote_neighbors
 * of the field, SPREAD_APPLY (the caller updates the ghosts before, as
 * game_of_life_test.cpp:378-380 does).  The reference's aborts: more than 8
 * parents -> DCCRGX_ERANGE, a dead neighbor's parent already recorded ->
 * DCCRGX_ESTATE. */
enum { DCCRGX_GOLH_RECORD = 1, DCCRGX_GOLH_SPREAD_APPLY = 2 };
int dccrgx_gol_amr_phase(dccrgx_grid* grid, int32_t hood_id, int32_t f_data, int32_t phase);
int dccrgx_gol_amr_step(dccrgx_grid* grid, int32_t hood_id, int32_t f_data);
/* synthetic initial state of a 4-byte field on local cells: 1 where
 * splitmix64(id) % 1000 < permille, else 0 (replaces the rand() loops of
 * tests/game_of_life/scalability3d.cpp:106-114 with an order-independent,
 * reproducible generator) */
int dccrgx_field_init_hash(dccrgx_grid* grid, int32_t field_id, uint32_t permille);
/* checksum of a 4-byte field over this rank's local cells, computed on the
 * device: out[0] = sum of the values, out[1] = sum of value *
 * splitmix64(cell id), both mod 2^64 (the live-cell count of the game of
 * life, and a position-sensitive check of a whole grid without copying it) */
int dccrgx_field_checksum(const dccrgx_grid* grid, int32_t field_id, uint64_t out[2]);
/* time the last dccrgx_gol_compute kernels (HIP events on the compute
 * stream): total ms and launch count since the last reset */
int dccrgx_kernel_timer(dccrgx_grid* grid, int32_t reset, double* ms_out, uint64_t* launches_out);

/* ------------------------------------------------------------------------ *
 * Advection, tests/advection/solve.hpp.  The reference's Cell::data members
 * (cell.hpp:34-44) as separate f64 fields; only `density` changes per step,
 * so the per-step halo moves only that field (transfer_all_data = false,
 * cell.hpp:47-57).  Velocities and lengths of remote neighbors must have
 * been exchanged once (initialize.hpp:60).
 * ------------------------------------------------------------------------ */
typedef struct {
    int32_t density, flux, vx, vy, vz, length_x, length_y, length_z;
} dccrgx_advect_fields;
/* calculate_fluxes(dt, solve_inner, grid, hood), solve.hpp:44-247: adds to
 * `flux` of every local cell of `region` the upwind fluxes through all of
 * its faces found in the neighborhood's neighbors_of (faces detected from
 * offsets and lengths in indices, :73-120).  Gather form: each cell sums its
 * own faces (both directions) instead of scattering into its neighbors;
 * per-face values equal the reference's. */
int dccrgx_advect_fluxes(dccrgx_grid* grid, int32_t hood_id, const dccrgx_advect_fields* f,
                         double dt, int32_t region);
/* apply_fluxes, solve.hpp:283-293: density += flux, flux = 0 (local cells) */
int dccrgx_advect_apply(dccrgx_grid* grid, const dccrgx_advect_fields* f);
/* max_time_step, solve.hpp:302-320, this rank's part: min over local cells
 * and axes of length / |v| where that is a normal number (DBL_MAX if none).
 * The caller reduces with MIN across ranks (:322-332). */
int dccrgx_advect_max_time_step(dccrgx_grid* grid, const dccrgx_advect_fields* f, double* local_min);
/* check_for_adaptation, tests/advection/adapter.hpp:43-176, device part: for
 * every local cell (ascending ids) the maximum relative density difference
 * |a - b| / (min(a, b) + diff_threshold) over the neighbors_of entries the
 * adapter counts as face neighbors (offset == own length or == -neighbor
 * length along one axis, 0 along the others, :70-90), taken over both cells
 * of each pair when the neighbor is local (:98-101); and the decision
 * category: 2 refine (diff > (level + 1) * diff_increase), 1 keep (diff >=
 * unrefine_sensitivity * that), 0 unrefine.  Switches a uniform grid to the
 * explicit layout.  max_diff_out optional. */
int dccrgx_advect_adapt_marks(dccrgx_grid* grid, int32_t hood_id, const dccrgx_advect_fields* f,
                              double diff_increase, double diff_threshold, double unrefine_sensitivity,
                              int8_t* marks_out, double* max_diff_out);
/* check_for_adaptation, tests/advection/adapter.hpp:43-176, complete: the
 * marks above turned into the reference's three sets per sibling group
 * (:109-176) on the device -- to_refine: cells marked 2; not_to_unrefine: the
 * first (lowest id) cell marked 1 of a group without a 2, level > 0;
 * to_unrefine: cells marked 0, level > 0, in a group without a 1 or 2.
 * Each output holds up to `cap` >= local cell count ids, ascending; counts[3]
 * receives the three sizes.  Nothing on a grid with maximum level 0. */
int dccrgx_advect_adaptation_sets(dccrgx_grid* grid, int32_t hood_id, const dccrgx_advect_fields* f,
                                  double diff_increase, double diff_threshold, double unrefine_sensitivity,
                                  uint64_t* to_refine, uint64_t* not_to_unrefine, uint64_t* to_unrefine, size_t cap,
                                  size_t counts[3]);
/* check_for_adaptation followed by the adapter's request loops
 * (tests/advection/adapter.hpp:43-176, then :197-213: refine_completely of
 * to_refine, dont_unrefine of not_to_unrefine, unrefine_completely of
 * to_unrefine, in that order), with the three sets kept on the device: the
 * same request state as dccrgx_advect_adaptation_sets plus
 * dccrgx_amr_request_cells of each set, without the sets' round trip through
 * host memory.  counts[3] receives the three set sizes.  Nothing on a grid
 * with maximum level 0. */
int dccrgx_advect_adapt_requests(dccrgx_grid* grid, int32_t hood_id, const dccrgx_advect_fields* f,
                                 double diff_increase, double diff_threshold, double unrefine_sensitivity,
                                 size_t counts[3]);
/* one step of tests/advection/2d.cpp:321-390: density halo start, inner
 * fluxes, halo wait, outer fluxes, apply -- fused: each cell's face fluxes
 * and the apply are one kernel writing the new density into a second buffer
 * (the same additions in the same order as fluxes + apply, flux left 0), and
 * the two density buffers swap.  The density field's device pointer
 * (dccrgx_field_device_ptr) therefore changes on every step. */
int dccrgx_advect_step(dccrgx_grid* grid, int32_t hood_id, const dccrgx_advect_fields* f, double dt);
/* velocities and lengths of every local cell, adapter.hpp:304-314 /
 * initialize.hpp:50-58: Cartesian_Geometry get_length / get_center
 * (dccrg_cartesian_geometry.hpp:284-364) and solve.hpp:336-342's
 * vx = 0.5 - y, vy = x - 0.5, vz = 0 */
int dccrgx_advect_set_geometry(dccrgx_grid* grid, const dccrgx_advect_fields* f, const double start[3],
                               const double level_0_cell_length[3]);

/* ------------------------------------------------------------------------ *
 * Adaptive mesh refinement (dccrg.hpp:2456-2806, 3483-3543, 5550-5567,
 * 9730-10693).  Request calls set *result to the reference's bool.  A
 * uniform grid switches to the explicit (mixed-level) layout inside the first
 * stop_refining that changes the grid (on every rank together).  stop_refining is collective: every rank passes the union
 * over all ranks of the four request sets (dccrgx_amr_requests on each rank,
 * all-gathered by the caller); the library then evaluates override_refines,
 * induce_refines and override_unrefines on the replicated leaf set and
 * rebuilds the grid on the device.  Field data of surviving cells moves to
 * their new slots, new cells are zero-initialised, and the data of refined
 * parents / removed children stays readable (dccrgx_field_read_cells) until
 * clear_refined_unrefined_data.  Grids with variable-size fields are refused.
 * ------------------------------------------------------------------------ */
enum { DCCRGX_AMR_REFINE = 0, DCCRGX_AMR_DONT_REFINE = 1, DCCRGX_AMR_UNREFINE = 2, DCCRGX_AMR_DONT_UNREFINE = 3 };
/* Dccrg::refine_completely, dccrg.hpp:2456-2548 */
int dccrgx_refine_completely(dccrgx_grid* grid, uint64_t cell, int32_t* result);
/* Dccrg::unrefine_completely, dccrg.hpp:2582-2676 */
int dccrgx_unrefine_completely(dccrgx_grid* grid, uint64_t cell, int32_t* result);
/* Dccrg::dont_unrefine, dccrg.hpp:2701-2760 */
int dccrgx_dont_unrefine(dccrgx_grid* grid, uint64_t cell, int32_t* result);
/* Dccrg::dont_refine, dccrg.hpp:2768-2806 */
int dccrgx_dont_refine(dccrgx_grid* grid, uint64_t cell, int32_t* result);
/* the request call of `kind` (DCCRGX_AMR_*) for each id in order; results
 * optional.  On explicit (mixed-level) grids the whole batch runs on the
 * device (amr_dev.hip) with the results of the calls made in this order. */
int dccrgx_amr_request_cells(dccrgx_grid* grid, int32_t kind, const uint64_t* ids, size_t n, int32_t* results);
/* this rank's pending request set `which` (DCCRGX_AMR_*), ascending; ids == NULL: count only */
int dccrgx_amr_requests(const dccrgx_grid* grid, int32_t which, uint64_t* ids, size_t cap, size_t* n);
/* Dccrg::stop_refining, dccrg.hpp:3483-3507: sets[k] / counts[k] = union over
 * all ranks of request set k; sets == NULL: this rank's own requests (one
 * rank: they are the union; they then never leave the device).  The
 * decisions and the new leaf set are computed on the device; n_new = cells
 * created on this rank */
int dccrgx_stop_refining(dccrgx_grid* grid, const uint64_t* const* sets, const size_t* counts,
                         size_t* n_new);
/* stop_refining in two phases, so that ranks agree before any of them adopts
 * a new leaf set (the reference reaches agreement by All_Gather after each
 * decision phase, dccrg.hpp:9730-10236, and aborts on failure).  prepare =
 * the decisions and the complete new grid state built aside (the grid stays
 * the old one; on failure everything is unwound and the requests stay
 * pending); then every rank all-reduces its status and calls finish with
 * commit = 1 (adopt) when all ranks succeeded, else commit = 0 (drop: old
 * grid, this rank's requests pending).  finish(0) without a prepared
 * stop_refining is a no-op; dccrgx_stop_refining = prepare + finish(1).
 * A uniform grid with refine or unrefine requests switches to the explicit
 * layout at prepare, before the decisions, and stays explicit when the
 * stop_refining is then dropped: same leaves and data, but field device
 * pointers and slots change (take dccrgx_field_device_ptr again).  Between
 * prepare and finish every call that reads or changes the grid's structure
 * or data returns DCCRGX_ESTATE. */
int dccrgx_stop_refining_prepare(dccrgx_grid* grid, const uint64_t* const* sets, const size_t* counts,
                                 size_t* n_new);
int dccrgx_stop_refining_finish(dccrgx_grid* grid, int32_t commit);
/* the cells the last stop_refining created on this rank (ascending; the
 * reference's return value of stop_refining(true)) */
int dccrgx_get_new_cells(const dccrgx_grid* grid, uint64_t* ids, size_t cap, size_t* n);
/* Dccrg::get_removed_cells(true), dccrg.hpp:3519-3543 */
int dccrgx_get_removed_cells(const dccrgx_grid* grid, uint64_t* ids, size_t cap, size_t* n);
/* Dccrg::clear_refined_unrefined_data, dccrg.hpp:5550-5567 */
int dccrgx_clear_refined_unrefined_data(dccrgx_grid* grid);
/* before clear_refined_unrefined_data: every cell the last stop_refining
 * created takes its parent's (refined, retired) values of `fields`
 * (tests/advection/adapter.hpp:229-251) */
int dccrgx_amr_copy_from_parents(dccrgx_grid* grid, const int32_t* fields, size_t nf);
/* before clear_refined_unrefined_data: the parent of removed cells gets 0,
 * then += child / 8 over its children in ascending id order, for each f64
 * field (adapter.hpp:253-300) */
int dccrgx_amr_average_children(dccrgx_grid* grid, const int32_t* fields, size_t nf);
/* both rules above in one call, copies first (the adapter's order,
 * adapter.hpp:229-300): one upload of the two lists, one error read-back */
int dccrgx_amr_adapter_data_rules(dccrgx_grid* grid, const int32_t* fields, size_t nf);

/* ------------------------------------------------------------------------ *
 * Poisson, tests/poisson/poisson_solve.hpp: Poisson_Solve (BiCG over face
 * neighbors, 1/4 weight per smaller face neighbor) with its cell data in the
 * grid's f64 fields.  The solver adds 14 internal fields (Poisson_Cell
 * members, :44-83).  On several ranks the halos and the scalar reductions go
 * over the context's RCCL communicator.
 * ------------------------------------------------------------------------ */
typedef struct dccrgx_poisson dccrgx_poisson;
/* Poisson_Solve(max_iterations, min_iterations, stop_residual, p_of_norm,
 * stop_after_residual_increase, verbose), :147-195 (defaults 1000, 0,
 * 1e-15, 2, 10 with params == NULL) */
typedef struct {
    uint32_t max_iterations, min_iterations;
    double stop_residual, p_of_norm, stop_after_residual_increase;
} dccrgx_poisson_params;
/* user fields: rhs and solution (Poisson_Cell::rhs/solution) and the cell
 * lengths (the geometry's get_length, used by set_scaling_factor :704-821) */
typedef struct {
    int32_t rhs, solution, length_x, length_y, length_z;
} dccrgx_poisson_fields;
enum {
    DCCRGX_POISSON_TYPE = 0, DCCRGX_POISSON_P0, DCCRGX_POISSON_P1, DCCRGX_POISSON_R0, DCCRGX_POISSON_R1,
    DCCRGX_POISSON_A_DOT_P0, DCCRGX_POISSON_BEST_SOLUTION, DCCRGX_POISSON_SCALING_FACTOR,
    DCCRGX_POISSON_F_X_POS, DCCRGX_POISSON_F_X_NEG, DCCRGX_POISSON_F_Y_POS, DCCRGX_POISSON_F_Y_NEG,
    DCCRGX_POISSON_F_Z_POS, DCCRGX_POISSON_F_Z_NEG
};
int dccrgx_poisson_create(dccrgx_grid* grid, const dccrgx_poisson_params* params,
                          const dccrgx_poisson_fields* fields, dccrgx_poisson** out);
int dccrgx_poisson_destroy(dccrgx_poisson* solver);
/* field id of an internal member (DCCRGX_POISSON_*) */
int dccrgx_poisson_field(const dccrgx_poisson* solver, int32_t which, int32_t* field_id);
/* Poisson_Solve::solve(cells, grid, cells_to_skip, cache_is_up_to_date),
 * :251-522: cells/skip are host id lists (non-local ids are ignored).
 * Outputs the iteration count and the minimum residual reached. */
int dccrgx_poisson_solve(dccrgx_poisson* solver, const uint64_t* cells, size_t n_cells,
                         const uint64_t* cells_to_skip, size_t n_skip, int32_t cache_is_up_to_date,
                         uint32_t* iterations, double* residual_min);

/* ------------------------------------------------------------------------ *
 * Grid data files: save_grid_data / load_grid_data (dccrg.hpp:1109-2427),
 * byte-compatible with the reference's layout:
 *   [offset bytes][user header][u64 0x1234567890abcdef][u64 length[3]]
 *   [i32 max_ref_lvl][u32 neighborhood_length][u8 periodic[3]][geometry]
 *   [u64 total cells][(u64 id, u64 absolute offset of its data) x total]
 *   [cell data]
 * rank by rank, each rank's cells in its local order (ascending ids).  A
 * cell's data is the bytes of the given fields in order, no padding -- the
 * packed form of the struct datatype its get_mpi_datatype() would return.
 * Geometry blobs: i32 id (0 No_Geometry; 1 Cartesian + f64 start[3] + f64
 * level_0_cell_length[3]; 2 Stretched + u64 n[3] + coordinates).
 * ------------------------------------------------------------------------ */
typedef struct {
    dccrgx_grid_params params;  /* mapping, neighborhood length, topology */
    uint64_t geometry_bytes;    /* Geometry::data_size() of the stored geometry */
    uint64_t total_cells;
    uint64_t list_offset;       /* absolute offset of the (id, offset) list */
} dccrgx_file_info;
/* bytes between the user header and the cell list */
uint64_t dccrgx_file_preamble_bytes(size_t geometry_bytes);
/* this rank's share of a save: local cells and their data bytes */
int dccrgx_save_sizes(const dccrgx_grid* grid, const int32_t* fields, size_t nf, uint64_t* n_cells,
                      uint64_t* n_bytes);
/* Dccrg::save_grid_data, dccrg.hpp:1109-1712.  Every rank calls it with the
 * same header / geometry / total_cells and its own exclusive prefix sums of
 * dccrgx_save_sizes over lower ranks (cells_before, bytes_before; the
 * caller's all-gather replaces the reference's MPI_Allgather :1490-1530).
 * Rank 0 writes header and preamble; every rank writes its list entries and
 * its cell data (one contiguous range).  The file is not truncated
 * (MPI_MODE_CREATE | MPI_MODE_WRONLY). */
int dccrgx_save_grid_data(const dccrgx_grid* grid, const char* path, uint64_t offset, const void* header,
                          size_t header_bytes, const void* geometry, size_t geometry_bytes, uint64_t total_cells,
                          uint64_t cells_before, uint64_t bytes_before, const int32_t* fields, size_t nf);
/* start_loading_grid_data, first half (dccrg.hpp:1815-2000): header bytes,
 * endianness check, mapping, neighborhood length, topology, geometry (copied
 * out if `geometry` is given) and the cell count */
int dccrgx_file_read_info(const char* path, uint64_t offset, void* header, size_t header_bytes,
                          dccrgx_file_info* info, void* geometry, size_t geometry_cap);
/* start_loading_grid_data, second half (:2002-2105): the grid of the file's
 * cells on this context (each rank gets the cells whose level-0 ancestor it
 * owns, cell_overlaps_local :3603-3622); a file of every level-0 cell gives
 * a uniform grid.  Fields are created afterwards, then loaded: */
int dccrgx_grid_load(dccrgx_ctx* ctx, const char* path, const dccrgx_file_info* info, dccrgx_grid** out);
/* continue_loading_grid_data, :2134-2390: reads the next bytes of every
 * local cell's record into the given fields (variable-size fields take
 * count * elem bytes: size them first, e.g. from a count read by an earlier
 * call) and advances each cell's file offset past them */
int dccrgx_load_cell_data(dccrgx_grid* grid, const int32_t* fields, size_t nf);
/* finish_loading_grid_data, :2402-2426 */
int dccrgx_finish_loading_grid_data(dccrgx_grid* grid);
/* Host-side cell data (the C++ facade keeps Cell_Data on the host): the
 * same save with the local cells' packed records (ascending ids, sizes per
 * cell) given by the caller, and the same continue-load into a host buffer. */
int dccrgx_save_grid_data_host(const dccrgx_grid* grid, const char* path, uint64_t offset, const void* header,
                               size_t header_bytes, const void* geometry, size_t geometry_bytes, uint64_t total_cells,
                               uint64_t cells_before, uint64_t bytes_before, const uint64_t* record_bytes,
                               const void* records, size_t bytes);
int dccrgx_load_cell_records_host(dccrgx_grid* grid, const uint64_t* record_bytes, void* out, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* DCCRGX_H */
