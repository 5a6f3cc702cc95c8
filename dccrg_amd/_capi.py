"""ctypes binding of libdccrgx.so (include/dccrgx.h).

The product path: every call goes to the HIP library; there is no CPU
fallback.  Importing this module on a machine without the built library
raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libdccrgx.so")

DCCRGX_OK = 0
DCCRGX_ENOMEM = 2
DCCRGX_ESTATE = 6
ERROR_CELL = 0
ERROR_INDEX = 0xFFFFFFFFFFFFFFFF
DEFAULT_NEIGHBORHOOD_ID = -0xDCC
CELLS_LOCAL, CELLS_INNER, CELLS_OUTER, CELLS_REMOTE = 0, 1, 2, 3
WAIT_ALL, WAIT_RECEIVES, WAIT_SENDS = 0, 1, 2
REGION_ALL, REGION_INNER, REGION_OUTER = 0, 1, 2
OP_LENGTH_IN_INDICES, OP_PARENT, OP_LEVEL_0_PARENT, OP_CHILD = 0, 1, 2, 3
AMR_REFINE, AMR_DONT_REFINE, AMR_UNREFINE, AMR_DONT_UNREFINE = 0, 1, 2, 3
GOLH_RECORD, GOLH_SPREAD_APPLY = 1, 2
PARTITION_BLOCK, PARTITION_SFC = 0, 1

ERRORS = {1: "EINVAL", 2: "ENOMEM", 3: "EHIP", 4: "ERCCL", 5: "ERANGE", 6: "ESTATE",
          7: "ENOTFOUND", 8: "EINTERNAL"}


class DccrgxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"dccrgx {ERRORS.get(code, code)}: {msg}")
        self.code = code


class Mapping_t(C.Structure):
    _fields_ = [("length", C.c_uint64 * 3), ("max_ref_lvl", C.c_int32), ("reserved", C.c_int32)]


class GridParams_t(C.Structure):
    _fields_ = [("length", C.c_uint64 * 3), ("max_ref_lvl", C.c_int32),
                ("neighborhood_length", C.c_uint32), ("periodic", C.c_uint8 * 3),
                ("partition", C.c_uint8), ("reserved", C.c_uint8 * 4)]


class GridInfo_t(C.Structure):
    _fields_ = [("n_local", C.c_uint64), ("first_local", C.c_uint64), ("n_slots", C.c_uint64),
                ("layout", C.c_uint64 * 4), ("max_ref_lvl", C.c_int32), ("uniform", C.c_int32),
                ("rank", C.c_int32), ("comm_size", C.c_int32)]


class FileInfo_t(C.Structure):
    _fields_ = [("params", GridParams_t), ("geometry_bytes", C.c_uint64), ("total_cells", C.c_uint64),
                ("list_offset", C.c_uint64)]


class StencilView_t(C.Structure):
    """dccrgx_stencil_view (include/dccrgx.h): device data of a user stencil."""
    _fields_ = [("kind", C.c_int32), ("n_items", C.c_int32), ("n_cells", C.c_uint64), ("stream", C.c_void_p),
                ("la", C.c_uint64), ("lb", C.c_uint64), ("lc", C.c_uint64), ("lo", C.c_uint64), ("hi", C.c_uint64),
                ("cbase", C.c_int64), ("s0", C.c_int64 * 2), ("s1", C.c_int64 * 2), ("per", C.c_int32 * 3),
                ("perm", C.c_int32 * 3), ("scale", C.c_int32), ("reach", C.c_int32 * 3), ("nslices", C.c_int32), ("shape", C.c_int32),
                ("items", C.c_void_p), ("item_delta", C.c_void_p), ("pos", C.c_void_p), ("local_slot", C.c_void_p), ("local_g", C.c_void_p),
                ("leaves", C.c_void_p), ("row", C.c_void_p), ("nbr_slot", C.c_void_p), ("nbr_off", C.c_void_p)]


class AdvectFields_t(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("density", "flux", "vx", "vy", "vz",
                                         "length_x", "length_y", "length_z")]


class PoissonParams_t(C.Structure):
    _fields_ = [("max_iterations", C.c_uint32), ("min_iterations", C.c_uint32), ("stop_residual", C.c_double),
                ("p_of_norm", C.c_double), ("stop_after_residual_increase", C.c_double)]


class PoissonFields_t(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("rhs", "solution", "length_x", "length_y", "length_z")]


POISSON_MEMBERS = ("type", "p0", "p1", "r0", "r1", "A_dot_p0", "best_solution", "scaling_factor",
                   "f_x_pos", "f_x_neg", "f_y_pos", "f_y_neg", "f_z_pos", "f_z_neg")


# every symbol include/dccrgx.h declares, with its ctypes signature
_vp = C.c_void_p
_u64p = C.POINTER(C.c_uint64)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_szp = C.POINTER(C.c_size_t)

# dccrgx_host_transport callbacks
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, _vp, C.c_int32, _i32p, C.POINTER(_vp), _u64p, C.c_int32, _i32p,
                          C.POINTER(_vp), _u64p)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, _vp, C.POINTER(C.c_double), C.c_int32, C.c_int32)


class HostTransport_t(C.Structure):
    _fields_ = [("user", _vp), ("exchange", EXCHANGE_FN), ("allreduce_f64", ALLREDUCE_FN)]


SIGNATURES = {
    "dccrgx_last_error": (C.c_char_p, []),
    "dccrgx_version": (C.c_int, []),
    "dccrgx_ctx_create": (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(_vp)]),
    "dccrgx_ctx_destroy": (C.c_int, [_vp]),
    "dccrgx_get_unique_id": (C.c_int, [C.c_char_p]),
    "dccrgx_ctx_comm_init": (C.c_int, [_vp, C.c_char_p]),
    "dccrgx_ctx_route_self_through_rccl": (C.c_int, [_vp, C.c_int32]),
    "dccrgx_test_option": (C.c_int, [C.c_char_p, C.c_int64, C.c_int32]),
    "dccrgx_ctx_compute_stream": (C.c_int, [_vp, C.POINTER(_vp)]),
    "dccrgx_ctx_set_host_transport": (C.c_int, [_vp, C.POINTER(HostTransport_t)]),
    "dccrgx_ctx_synchronize": (C.c_int, [_vp]),
    "dccrgx_max_possible_refinement_level": (C.c_int, [_u64p, _i32p]),
    "dccrgx_last_cell": (C.c_int, [C.POINTER(Mapping_t), _u64p]),
    "dccrgx_map_ids_to_indices": (C.c_int, [C.POINTER(Mapping_t), _vp, C.c_size_t, _vp, _vp, _vp]),
    "dccrgx_map_indices_to_ids": (C.c_int, [C.POINTER(Mapping_t), _vp, _vp, C.c_size_t, _vp, _vp]),
    "dccrgx_map_ids_op": (C.c_int, [C.POINTER(Mapping_t), C.c_int, _vp, C.c_size_t, _vp, _vp]),
    "dccrgx_map_host_indices": (C.c_int, [C.POINTER(Mapping_t), C.c_uint64, _u64p, _i32p]),
    "dccrgx_map_host_cell": (C.c_int, [C.POINTER(Mapping_t), _u64p, C.c_int32, _u64p]),
    "dccrgx_map_host_op": (C.c_int, [C.POINTER(Mapping_t), C.c_int, C.c_uint64, _u64p]),
    "dccrgx_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "dccrgx_map_host_ids_to_indices": (C.c_int, [C.POINTER(Mapping_t), _u64p, C.c_size_t, _u64p, _i32p]),
    "dccrgx_map_host_ids_op": (C.c_int, [C.POINTER(Mapping_t), C.c_int, _u64p, C.c_size_t, _u64p]),
    "dccrgx_neighbors_of_host": (C.c_int, [_vp, C.c_int32, _u64p, C.c_size_t, _u64p, _u64p, _i32p, C.c_size_t]),
    "dccrgx_neighbors_to_host": (C.c_int, [_vp, C.c_int32, _u64p, C.c_size_t, _u64p, _u64p, C.c_size_t]),
    "dccrgx_face_neighbors_of": (C.c_int, [_vp, _vp, C.c_size_t, _vp, _vp, _vp, C.c_size_t, _vp]),
    "dccrgx_face_neighbors_of_host": (C.c_int, [_vp, _u64p, C.c_size_t, _u64p, _u64p, _i32p, C.c_size_t]),
    "dccrgx_exchange_start": (C.c_int, [_vp, C.c_int32, C.POINTER(_vp), _u64p, C.POINTER(_vp), _u64p]),
    "dccrgx_exchange_wait": (C.c_int, [_vp, C.c_int32]),
    "dccrgx_grid_create": (C.c_int, [_vp, C.POINTER(GridParams_t), _u64p, C.c_size_t, C.POINTER(_vp)]),
    "dccrgx_grid_destroy": (C.c_int, [_vp]),
    "dccrgx_grid_get_info": (C.c_int, [_vp, C.POINTER(GridInfo_t)]),
    "dccrgx_add_neighborhood": (C.c_int, [_vp, C.c_int32, _i32p, C.c_size_t]),
    "dccrgx_remove_neighborhood": (C.c_int, [_vp, C.c_int32]),
    "dccrgx_get_neighborhood": (C.c_int, [_vp, C.c_int32, _i32p, C.c_size_t, _szp]),
    "dccrgx_get_cells": (C.c_int, [_vp, C.c_int32, C.c_int32, _u64p, C.c_size_t, _szp]),
    "dccrgx_get_all_cells": (C.c_int, [_vp, _u64p, C.c_size_t, _szp]),
    "dccrgx_neighbors_of": (C.c_int, [_vp, C.c_int32, _vp, C.c_size_t, _vp, _vp, _vp, C.c_size_t, _vp]),
    "dccrgx_neighbors_to": (C.c_int, [_vp, C.c_int32, _vp, C.c_size_t, _vp, _vp, C.c_size_t, _vp]),
    "dccrgx_get_peers": (C.c_int, [_vp, C.c_int32, C.c_int32, _i32p, _u64p, C.c_size_t, _szp]),
    "dccrgx_get_peer_cells": (C.c_int, [_vp, C.c_int32, C.c_int32, C.c_int32, _u64p, C.c_size_t, _szp]),
    "dccrgx_field_create": (C.c_int, [_vp, C.c_uint32, _i32p]),
    "dccrgx_field_device_ptr": (C.c_int, [_vp, C.c_int32, C.POINTER(_vp), _u64p]),
    "dccrgx_slots_of": (C.c_int, [_vp, _vp, C.c_size_t, _vp, _vp]),
    "dccrgx_field_write_local": (C.c_int, [_vp, C.c_int32, _vp, C.c_size_t]),
    "dccrgx_field_read_local": (C.c_int, [_vp, C.c_int32, _vp, C.c_size_t]),
    "dccrgx_field_read_remote": (C.c_int, [_vp, C.c_int32, C.c_int32, _vp, C.c_size_t]),
    "dccrgx_field_create_variable": (C.c_int, [_vp, C.c_uint32, _i32p]),
    "dccrgx_field_resize": (C.c_int, [_vp, C.c_int32, _u64p, C.POINTER(C.c_uint32), C.c_size_t]),
    "dccrgx_field_get_counts": (C.c_int, [_vp, C.c_int32, _u64p, C.c_size_t, C.POINTER(C.c_uint32)]),
    "dccrgx_field_write_cells": (C.c_int, [_vp, C.c_int32, _u64p, C.c_size_t, _vp, C.c_size_t]),
    "dccrgx_field_read_cells": (C.c_int, [_vp, C.c_int32, _u64p, C.c_size_t, _vp, C.c_size_t, _szp]),
    "dccrgx_halo_start": (C.c_int, [_vp, C.c_int32, _i32p, C.c_size_t]),
    "dccrgx_halo_wait": (C.c_int, [_vp, C.c_int32, C.c_int32]),
    "dccrgx_halo_update": (C.c_int, [_vp, C.c_int32, _i32p, C.c_size_t]),
    "dccrgx_halo_pack_to": (C.c_int, [_vp, C.c_int32, _i32p, C.c_size_t, C.c_int32, _vp, C.c_size_t, _szp]),
    "dccrgx_halo_unpack_from": (C.c_int, [_vp, C.c_int32, _i32p, C.c_size_t, C.c_int32, _vp, C.c_size_t]),
    "dccrgx_halo_self": (C.c_int, [_vp, C.c_int32, _i32p, C.c_size_t]),
    "dccrgx_gol_compute": (C.c_int, [_vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
    "dccrgx_gol_step": (C.c_int, [_vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
    "dccrgx_get_process": (C.c_int, [_vp, _u64p, C.c_size_t, _i32p]),
    "dccrgx_gather_neighbors": (C.c_int, [_vp, C.c_int32, C.c_int32, _vp, C.c_size_t, _vp, _vp, C.c_size_t,
                                          _vp]),
    "dccrgx_sfc_owners": (C.c_int, [_vp, _u64p, C.c_int32, _i32p]),
    "dccrgx_sfc_cuts": (C.c_int, [_u64p, C.c_int32, _u64p]),
    "dccrgx_hilbert_keys_host": (C.c_int, [_u64p, _u64p]),
    "dccrgx_gol_amr_phase": (C.c_int, [_vp, C.c_int32, C.c_int32, C.c_int32]),
    "dccrgx_gol_amr_step": (C.c_int, [_vp, C.c_int32, C.c_int32]),
    "dccrgx_field_init_hash": (C.c_int, [_vp, C.c_int32, C.c_uint32]),
    "dccrgx_field_checksum": (C.c_int, [_vp, C.c_int32, _u64p]),
    "dccrgx_kernel_timer": (C.c_int, [_vp, C.c_int32, C.POINTER(C.c_double), _u64p]),
    "dccrgx_advect_fluxes": (C.c_int, [_vp, C.c_int32, C.POINTER(AdvectFields_t), C.c_double, C.c_int32]),
    "dccrgx_advect_apply": (C.c_int, [_vp, C.POINTER(AdvectFields_t)]),
    "dccrgx_advect_max_time_step": (C.c_int, [_vp, C.POINTER(AdvectFields_t), C.POINTER(C.c_double)]),
    "dccrgx_advect_step": (C.c_int, [_vp, C.c_int32, C.POINTER(AdvectFields_t), C.c_double]),
    "dccrgx_poisson_create": (C.c_int, [_vp, C.POINTER(PoissonParams_t), C.POINTER(PoissonFields_t),
                                        C.POINTER(_vp)]),
    "dccrgx_poisson_destroy": (C.c_int, [_vp]),
    "dccrgx_poisson_field": (C.c_int, [_vp, C.c_int32, _i32p]),
    "dccrgx_amr_request_cells": (C.c_int, [_vp, C.c_int32, _u64p, C.c_size_t, _i32p]),
    "dccrgx_advect_adapt_marks": (C.c_int, [_vp, C.c_int32, _vp, C.c_double, C.c_double, C.c_double,
                                            C.POINTER(C.c_int8), C.POINTER(C.c_double)]),
    "dccrgx_advect_adaptation_sets": (C.c_int, [_vp, C.c_int32, _vp, C.c_double, C.c_double, C.c_double,
                                                _u64p, _u64p, _u64p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "dccrgx_refine_completely": (C.c_int, [_vp, C.c_uint64, _i32p]),
    "dccrgx_unrefine_completely": (C.c_int, [_vp, C.c_uint64, _i32p]),
    "dccrgx_dont_unrefine": (C.c_int, [_vp, C.c_uint64, _i32p]),
    "dccrgx_dont_refine": (C.c_int, [_vp, C.c_uint64, _i32p]),
    "dccrgx_amr_requests": (C.c_int, [_vp, C.c_int32, _u64p, C.c_size_t, _szp]),
    "dccrgx_stop_refining": (C.c_int, [_vp, C.POINTER(_u64p), _szp, _szp]),
    "dccrgx_neighbor_list_stats": (C.c_int, [_vp, C.c_int32, C.POINTER(C.c_uint64)]),
    "dccrgx_stencil_view_get": (C.c_int, [_vp, C.c_int32, C.c_int32, C.POINTER(StencilView_t)]),
    "dccrgx_stop_refining_prepare": (C.c_int, [_vp, C.POINTER(_u64p), _szp, _szp]),
    "dccrgx_stop_refining_finish": (C.c_int, [_vp, C.c_int32]),
    "dccrgx_get_new_cells": (C.c_int, [_vp, _u64p, C.c_size_t, _szp]),
    "dccrgx_get_removed_cells": (C.c_int, [_vp, _u64p, C.c_size_t, _szp]),
    "dccrgx_clear_refined_unrefined_data": (C.c_int, [_vp]),
    "dccrgx_poisson_solve": (C.c_int, [_vp, _u64p, C.c_size_t, _u64p, C.c_size_t, C.c_int32,
                                       C.POINTER(C.c_uint32), C.POINTER(C.c_double)]),
    "dccrgx_file_preamble_bytes": (C.c_uint64, [C.c_size_t]),
    "dccrgx_save_sizes": (C.c_int, [_vp, _i32p, C.c_size_t, _u64p, _u64p]),
    "dccrgx_save_grid_data": (C.c_int, [_vp, C.c_char_p, C.c_uint64, _vp, C.c_size_t, _vp, C.c_size_t, C.c_uint64,
                                        C.c_uint64, C.c_uint64, _i32p, C.c_size_t]),
    "dccrgx_file_read_info": (C.c_int, [C.c_char_p, C.c_uint64, _vp, C.c_size_t, C.POINTER(FileInfo_t), _vp,
                                        C.c_size_t]),
    "dccrgx_grid_load": (C.c_int, [_vp, C.c_char_p, C.POINTER(FileInfo_t), C.POINTER(_vp)]),
    "dccrgx_load_cell_data": (C.c_int, [_vp, _i32p, C.c_size_t]),
    "dccrgx_finish_loading_grid_data": (C.c_int, [_vp]),
    "dccrgx_save_grid_data_host": (C.c_int, [_vp, C.c_char_p, C.c_uint64, _vp, C.c_size_t, _vp, C.c_size_t,
                                             C.c_uint64, C.c_uint64, C.c_uint64, _u64p, _vp, C.c_size_t]),
    "dccrgx_load_cell_records_host": (C.c_int, [_vp, _u64p, _vp, C.c_size_t]),
    "dccrgx_advect_set_geometry": (C.c_int, [_vp, C.POINTER(AdvectFields_t), C.POINTER(C.c_double),
                                             C.POINTER(C.c_double)]),
    "dccrgx_amr_copy_from_parents": (C.c_int, [_vp, _i32p, C.c_size_t]),
    "dccrgx_amr_average_children": (C.c_int, [_vp, _i32p, C.c_size_t]),
    "dccrgx_amr_adapter_data_rules": (C.c_int, [_vp, _i32p, C.c_size_t]),
    "dccrgx_advect_adapt_requests": (C.c_int, [_vp, C.c_int32, _vp, C.c_double, C.c_double, C.c_double,
                                               C.POINTER(C.c_size_t)]),
}

_lib = None


def lib():
    """Load libdccrgx.so; raise if it has not been built (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import "
                              f"__graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(status: int):
    if status != DCCRGX_OK:
        raise DccrgxError(status, lib().dccrgx_last_error().decode(errors="replace"))
