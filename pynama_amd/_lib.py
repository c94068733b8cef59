"""ctypes binding of libkle.so (include/kle.h).

The product path has no CPU fallback: if libkle.so cannot be loaded, or a
device call fails, an :class:`Error` is raised (PETSc error codes).
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# KLE_LIBRARY: tools/ A/B scripts point this at the timing-probe build
# (tools/libkle_probe.so, `make -C pynama_amd/csrc probe`); unset = libkle.so
LIBPATH = os.environ.get("KLE_LIBRARY") or os.path.join(_HERE, "libkle.so")


class Error(RuntimeError):
    """petsc4py.PETSc.Error counterpart: carries the PETSc-style error code."""

    def __init__(self, ierr, msg=""):
        self.ierr = ierr
        super().__init__(f"error code {ierr}: {msg}")


i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
vp = C.c_void_p
pvp = C.POINTER(C.c_void_p)


class MeshInfo(C.Structure):
    _fields_ = [("dim", C.c_int), ("ngl", C.c_int), ("rank", C.c_int), ("nranks", C.c_int),
                ("nelem", C.c_int64 * 3), ("lattice", C.c_int64 * 3), ("n_nodes", C.c_int64),
                ("n_elems", C.c_int64), ("node_begin", C.c_int64), ("node_end", C.c_int64),
                ("ext_begin", C.c_int64), ("ext_end", C.c_int64), ("elem_begin", C.c_int64),
                ("elem_end", C.c_int64), ("kind", C.c_int), ("axis", C.c_int)]


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_int, C.c_void_p)
HALO_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_int64, C.c_int, C.POINTER(C.c_double), C.c_int64,
                      C.c_int, C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_double), C.c_int64, C.c_void_p)


EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_double), C.POINTER(C.c_int64),
                          C.POINTER(C.c_double), C.POINTER(C.c_int64), C.c_void_p)


class HostComm(C.Structure):
    _fields_ = [("allreduce", ALLREDUCE_FN), ("halo", HALO_FN), ("user", C.c_void_p), ("exchange", EXCHANGE_FN)]


_SIGS = {
    "kle_version": [],
    "kle_get_unique_id": [C.c_char_p],
    "kle_set_tuning": [C.c_char_p, C.c_int],
    "kle_get_tuning": [C.c_char_p, C.POINTER(C.c_int)],
    "kle_ctx_create": [C.c_int, C.c_int, C.c_int, C.c_char_p, pvp],
    "kle_ctx_create_host_comm": [C.c_int, C.c_int, C.c_int, C.POINTER(HostComm), pvp],
    "kle_ctx_destroy": [vp],
    "kle_ctx_synchronize": [vp],
    "kle_ctx_barrier": [vp],
    "kle_ctx_get_device": [vp, C.POINTER(C.c_int), C.c_char_p, C.c_int, C.POINTER(C.c_int)],
    "kle_ctx_get_comm_info": [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "kle_brick_plan_box": [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int),
                           C.POINTER(C.c_double)],
    "kle_ctx_enable_ipc": [vp],
    "kle_ctx_set_profiling": [vp, C.c_int],
    "kle_ctx_set_profiling_sample": [vp, C.c_int],
    "kle_ctx_set_profiling_filter": [vp, C.c_char_p],
    "kle_ctx_get_kernel_stats": [vp, C.c_char_p, C.POINTER(C.c_int64), C.POINTER(C.c_double)],
    "kle_ctx_reset_kernel_stats": [vp],
    "kle_mesh_create_box": [C.c_int, i64p, f64p, f64p, C.c_int, C.c_int, C.c_int, pvp],
    "kle_mesh_destroy": [vp],
    "kle_mesh_create_unstructured": [C.c_int, C.c_int, C.c_int64, f64p, C.c_int64, i64p, C.c_int64, vp, vp,
                                     C.c_int, C.c_int, pvp],
    "kle_mesh_create_gmsh": [C.c_char_p, C.c_int, C.c_int, C.c_int, pvp],
    "kle_mesh_get_elements": [vp, i64p],
    "kle_set_partitioner": [C.c_int],
    "kle_get_partitioner": [],
    "kle_mesh_get_peers": [vp, C.POINTER(C.c_int), vp, vp, vp, vp],
    "kle_mesh_get_ext_gids": [vp, i64p],
    "kle_mesh_get_info": [vp, C.POINTER(MeshInfo)],
    "kle_mesh_get_conn": [vp, i64p],
    "kle_mesh_get_corners": [vp, f64p],
    "kle_mesh_get_coords": [vp, f64p],
    "kle_mesh_face_nodes": [vp, C.c_uint, vp, C.POINTER(C.c_int64)],
    "kle_mesh_set_dirichlet_faces": [vp, C.c_uint],
    "kle_mesh_set_noslip_dofs": [vp, i64p, C.c_int64, i64p, C.c_int64],
    "kle_mesh_set_noslip_faces": [vp, i32p, C.c_int],
    "kle_mesh_set_dirichlet_nodes": [vp, i64p, C.c_int64],
    "kle_mesh_pattern_size": [vp, C.c_int, C.POINTER(C.c_int64)],
    "kle_mesh_pattern": [vp, C.c_int, i64p, vp],
    "kle_mesh_halo": [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                      C.POINTER(C.c_int64), C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "kle_vec_create_mesh": [vp, vp, C.c_int, pvp],
    "kle_vec_create": [vp, C.c_int64, C.c_int64, pvp],
    "kle_vec_duplicate": [vp, pvp],
    "kle_vec_destroy": [vp],
    "kle_vec_get_sizes": [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)],
    "kle_vec_get_ownership_range": [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)],
    "kle_vec_set": [vp, C.c_double],
    "kle_vec_copy": [vp, vp],
    "kle_vec_axpy": [vp, C.c_double, vp],
    "kle_vec_aypx": [vp, C.c_double, vp],
    "kle_vec_waxpy": [vp, C.c_double, vp, vp],
    "kle_vec_scale": [vp, C.c_double],
    "kle_vec_pointwise_mult": [vp, vp, vp],
    "kle_vec_tensor_square": [vp, C.c_int, vp],
    "kle_vec_reciprocal": [vp],
    "kle_vec_dot": [vp, vp, C.POINTER(C.c_double)],
    "kle_vec_norm2": [vp, C.POINTER(C.c_double)],
    "kle_vec_set_values": [vp, C.c_int64, i64p, f64p, C.c_int],
    "kle_vec_get_values": [vp, C.c_int64, i64p, f64p],
    "kle_vec_get_array": [vp, f64p],
    "kle_vec_set_array": [vp, f64p],
    "kle_vec_restore_array": [vp, f64p],
    "kle_vec_assemble": [vp],
    "kle_vec_ghost_update": [vp],
    "kle_vec_device_ptr": [vp, C.POINTER(C.c_void_p)],
    "kle_assemble_kle": [vp, vp, pvp, pvp, pvp],
    "kle_element_kle": [vp, vp, C.c_int64, f64p, f64p],
    "kle_assemble_operators": [vp, vp, pvp, pvp, pvp],
    "kle_assemble_ns": [vp, vp] + [pvp] * 9,
    "kle_mat_create_aij": [vp, C.c_int64, C.c_int64, C.c_int64, C.c_int64, vp, vp, pvp],
    "kle_mat_create_aij_csr": [vp, C.c_int64, C.c_int64, i64p, i64p, f64p, pvp],
    "kle_mat_set_values": [vp, C.c_int32, i64p, C.c_int32, i64p, f64p, C.c_int],
    "kle_mat_assemble": [vp],
    "kle_mat_destroy": [vp],
    "kle_mat_get_size": [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)],
    "kle_mat_get_local_size": [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)],
    "kle_mat_get_ownership_range": [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)],
    "kle_mat_get_local_nnz": [vp, C.POINTER(C.c_int64)],
    "kle_mat_get_info": [vp, C.c_void_p],  # kle_mat_info* (MatInfo below)
    "kle_mat_mult": [vp, vp, vp],
    "kle_mat_mult_add": [vp, vp, vp, vp],
    "kle_mat_diagonal_scale": [vp, vp, vp],
    "kle_mat_get_diagonal": [vp, vp],
    "kle_mat_axpy": [vp, C.c_double, vp],
    "kle_mat_duplicate": [vp, C.c_int, pvp],
    "kle_mat_get_csr_size": [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)],
    "kle_mat_get_row": [vp, C.c_int64, C.POINTER(C.c_int64), vp, vp],
    "kle_mat_get_csr": [vp, i64p, i64p, f64p],
    "kle_mat_convert_aij": [vp, pvp],
    "kle_set_nb_pad": [C.c_int],
    "kle_mat_set_halo_overlap": [vp, C.c_int],
    "kle_mat_set_spmv_structured": [vp, C.c_int],
    "kle_mat_is_structured": [vp, C.POINTER(C.c_int)],
    "kle_mat_set_symmetric": [vp, C.c_int],
    "kle_mat_get_symmetric": [vp, C.POINTER(C.c_int)],
    "kle_mat_get_sym_bricks": [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_double),
                               C.POINTER(C.c_double)],
    "kle_get_nb_pad": [],
    "kle_set_nb_layout": [C.c_int],
    "kle_get_nb_layout": [],
    "kle_mat_get_format": [vp, C.c_char_p, C.c_int],
    "kle_mat_spmv_bytes": [vp, C.POINTER(C.c_double)],
    "kle_mat_spmv_kernel": [vp, C.c_char_p, C.c_int],
    "kle_mat_time_local_spmv": [vp, vp, vp, C.c_int, C.POINTER(C.c_double)],
    "kle_ksp_create": [vp, pvp],
    "kle_ksp_destroy": [vp],
    "kle_ksp_set_type": [vp, C.c_char_p],
    "kle_ksp_set_pc_type": [vp, C.c_char_p],
    "kle_ksp_set_pc": [vp, C.c_char_p],
    "kle_ksp_set_tolerances": [vp, C.c_double, C.c_double, C.c_double, C.c_int],
    "kle_ksp_set_gmres_restart": [vp, C.c_int],
    "kle_ksp_set_fixed_iterations": [vp, C.c_int],
    "kle_ksp_continue": [vp, vp, vp, C.c_int],
    "kle_ksp_set_cg_single_reduction": [vp, C.c_int],
    "kle_ksp_set_operators": [vp, vp],
    "kle_ksp_set_up": [vp],
    "kle_ksp_solve": [vp, vp, vp],
    "kle_ksp_get_iteration_number": [vp, C.POINTER(C.c_int)],
    "kle_ksp_get_product_kernel": [vp, C.c_char_p, C.c_int],
    "kle_ksp_get_product_bytes": [vp, C.POINTER(C.c_double)],
    "kle_ksp_get_residual_norm": [vp, C.POINTER(C.c_double)],
    "kle_ksp_get_converged_reason": [vp, C.POINTER(C.c_int)],
    "kle_ksp_get_true_relative_residual": [vp, C.POINTER(C.c_double)],
    "kle_ksp_set_corrections": [vp, C.c_int],
    "kle_ksp_get_correction_iterations": [vp, C.POINTER(C.c_int)],
    "kle_ksp_get_correction_reason": [vp, C.POINTER(C.c_int)],
    "kle_mat_move_values": [vp, C.c_longlong, C.c_int],
    "kle_stream_copy_bench": [vp, C.c_int64, C.c_int, C.POINTER(C.c_double)],
    "kle_stream_bench": [vp, C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_double)],
}

_lib = None


def load():
    """Load libkle.so (build it first with __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIBPATH):
        raise Error(56, f"{LIBPATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(LIBPATH)
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_int
    lib.kle_last_error.restype = C.c_char_p
    lib.kle_last_error.argtypes = []
    _lib = lib
    return lib


class MatInfo(C.Structure):
    """kle_mat_info (include/kle.h)."""
    _fields_ = [("m_global", C.c_int64), ("n_global", C.c_int64), ("m_local", C.c_int64),
                ("n_local", C.c_int64), ("nz_used", C.c_int64), ("format", C.c_int),
                ("block_rows", C.c_int), ("block_cols", C.c_int), ("spmv_bytes", C.c_double)]


def exported_symbols():
    return sorted(list(_SIGS) + ["kle_last_error"])


def call(name, *args):
    """Call a kle_* function; raise Error on a non-zero return code."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.kle_last_error()
        raise Error(rc, f"{name}: {msg.decode() if msg else ''}")
    return rc
