"""ctypes binding of the C-ABI in include/hlhgat.h (libhlhgat.so).

The product path has no fallback: if the HIP library is missing or fails to
load, importing :mod:`hlhgat.ops` raises.  ``torch`` is imported first so the
library binds to the HIP runtime torch already loaded (same SONAME
libamdhip64.so.7), which makes torch's device pointers and streams valid
arguments.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede the library load, see module doc)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HLHGAT_LIB", os.path.join(_HERE, "libhlhgat.so"))

c_i32, c_i64, c_f32, c_f64, c_vp, c_sz = (C.c_int32, C.c_int64, C.c_float,
                                           C.c_double, C.c_void_p, C.c_size_t)
P_i64 = C.POINTER(c_i64)
P_f64 = C.POINTER(c_f64)
P_vp = C.POINTER(c_vp)

MAX_COPY_BLOCKS = 64  # HLHGAT_MAX_COPY_BLOCKS

# name -> (restype, argtypes); mirrors include/hlhgat.h exactly
SIGNATURES = {
    "hlhgat_version": (c_i32, []),
    "hlhgat_last_error": (C.c_char_p, []),
    "hlhgat_csr_workspace_bytes": (c_sz, [c_i64]),
    "hlhgat_csr_from_coo": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp,
                                    c_vp, c_vp, c_vp, c_sz, c_vp]),
    "hlhgat_csr_from_sorted_coo": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp,
                                           c_vp, c_vp]),
    "hlhgat_coo_check_sorted": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "hlhgat_incidence_csr": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "hlhgat_halo_tiles": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_i32, c_i32, c_i32, c_vp,
                                  c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, P_i64, P_i64]),
    "hlhgat_graclus": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "hlhgat_mlgc_map": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, P_i64, P_i64]),
    "hlhgat_mlgc_batch": (c_i32, [c_i64, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp,
                                  c_vp]),
    "hlhgat_gather_f32": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    "hlhgat_collate_sizes": (c_i32, [c_vp, c_vp, c_i64, c_vp]),
    "hlhgat_collate": (c_i32, [c_vp, c_vp, c_i64, c_vp]),
    "hlhgat_spmm": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64,
                            c_vp, c_i64, c_vp]),
    "hlhgat_poly_step": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp,
                                 c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_f32,
                                 c_f32, c_f32, c_f32, c_f32, c_f32, c_vp, c_i64, c_vp]),
    "hlhgat_incidence_step": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_i64,
                                      c_i64, c_vp, c_i64, c_f32, c_f32, c_vp, c_i64, c_vp]),
    "hlhgat_poly_basis_fwd": (c_i32, [c_i32, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp,
                                      c_vp, c_i64, c_i64, c_i32, c_vp, c_vp]),
    "hlhgat_poly_basis_bwd": (c_i32, [c_i32, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp,
                                      c_i64, c_i32, c_vp, c_vp]),
    "hlhgat_hodge_factor_work_floats": (c_i64, [c_i64, c_i64]),
    "hlhgat_hodge_spmm": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp]),
    "hlhgat_hodge_poly_step": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp,
                                       c_i64, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32, c_vp,
                                       c_i64, c_vp, c_vp]),
    "hlhgat_poly_basis_fwd_factored": (c_i32, [c_i32, c_vp, c_vp, c_i64, c_i64, c_i32, c_vp,
                                               c_vp, c_vp]),
    "hlhgat_poly_basis_bwd_factored": (c_i32, [c_i32, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp]),
    "hlhgat_hodge_lmax_workspace_bytes": (c_i64, [c_i64, c_i32]),
    "hlhgat_hodge_lmax": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_i32, c_vp, c_vp,
                                  c_i64, c_vp]),
    "hlhgat_bn_bwd_reduce": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64,
                                     c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "hlhgat_eig_pe_workspace_bytes": (c_i64, [c_i64, c_i64, c_i32]),
    "hlhgat_eig_pe": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i32, c_vp,
                              c_i64, c_vp, c_vp, c_i64, c_vp]),
    "hlhgat_hodge_row_sizes": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "hlhgat_hodge_build": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64,
                                   c_vp, c_vp, c_vp, c_i64, c_vp]),
    "hlhgat_proj_fwd": (c_i32, [c_i32, P_vp, P_i64, P_vp, P_i64, P_i64, c_i64, c_i64, c_vp,
                                c_vp, c_i64, c_i32, c_vp]),
    "hlhgat_proj_bwd_data": (c_i32, [c_i32, c_vp, c_i64, P_vp, P_i64, P_i64, c_i64, c_i64,
                                     P_vp, P_i64, c_i32, c_vp]),
    "hlhgat_proj_bwd_weight_workspace_floats": (c_i64, [c_i32, P_i64, c_i64, c_i64, c_i32]),
    "hlhgat_proj_bwd_weight": (c_i32, [c_i32, c_vp, c_i64, P_vp, P_i64, P_i64, c_i64, c_i64,
                                       P_vp, P_i64, c_vp, c_i32, c_vp, c_i64, c_vp]),
    "hlhgat_proj_bwd": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_i32, P_vp, P_i64, P_i64, P_vp,
                                P_i64, c_vp, c_i32, P_vp, P_i64, P_i64, P_vp, P_i64, c_i32,
                                c_vp, c_i64, c_vp]),
    "hlhgat_proj_bwd_defer": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_i32, P_vp, P_i64, P_i64,
                                      P_vp, P_i64, c_vp, c_i32, P_vp, P_i64, P_i64, P_vp, P_i64,
                                      c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "hlhgat_reduce_run": (c_i32, [c_vp, c_vp]),
    "hlhgat_proj_bn_fwd": (c_i32, [c_i32, P_vp, P_i64, P_vp, P_i64, P_i64, c_i64, c_i64, c_vp,
                                   c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32,
                                   c_f32, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "hlhgat_set_proj_bn_fused": (c_i32, [c_i32]),
    "hlhgat_set_proj_bn_split": (c_i32, [c_i32]),
    "hlhgat_set_proj_bwd_rows": (c_i32, [c_i32]),
    "hlhgat_set_gemm_big": (c_i32, [c_i32, c_i64]),
    "hlhgat_proj_bn_fused_capacity": (c_i32, [P_i64]),
    "hlhgat_set_bn_one_launch": (c_i32, [c_i32]),
    "hlhgat_get_bn_one_launch": (c_i32, []),
    "hlhgat_set_bn_wait_us": (c_i32, [C.c_uint32]),
    "hlhgat_set_proj_bn_stamps": (c_i32, [c_vp, c_i64]),
    "hlhgat_bn_giveup_log": (c_i32, [c_vp, c_i32, c_vp]),
    "hlhgat_bn_giveup_reset": (c_i32, []),
    "hlhgat_test_occupy": (c_i32, [c_i32, c_i32, c_i32, C.c_uint32, c_vp]),
    "hlhgat_device_errors": (c_i32, [c_vp]),
    "hlhgat_stream_create": (c_i32, [c_i32, C.c_uint32, c_i32, c_vp, c_i32, c_vp]),
    "hlhgat_stream_cu_mask": (c_i32, [c_vp, c_vp, c_i32]),
    "hlhgat_clear_device_errors": (c_i32, []),
    "hlhgat_bn_wait_timeouts": (c_i32, [c_vp]),
    "hlhgat_edge_gather2": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_f32,
                                    c_f32, c_vp, c_i64, c_vp, c_i64, c_i32, c_vp]),
    "hlhgat_att_score_fwd": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64,
                                     c_f32, c_f32, c_f32, c_i32, c_vp, c_vp]),
    "hlhgat_att_score_bwd": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64,
                                     c_f32, c_f32, c_f32, c_i32, c_vp, c_vp, c_vp, c_vp,
                                     c_vp, c_i64, c_vp]),
    "hlhgat_segment_mean_fwd": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64,
                                        c_vp]),
    "hlhgat_segment_mean_bwd": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64,
                                        c_i64, c_vp]),
    "hlhgat_row_scale_fwd": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "hlhgat_row_scale_bwd": (c_i32, [c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64,
                                     c_vp, c_vp]),
    "hlhgat_edge_absdiff": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64,
                                    c_vp]),
    "hlhgat_pool_mean_bwd": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64,
                                     c_i64, c_vp]),
    "hlhgat_bn_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "hlhgat_bn_apply_running": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_f32,
                                        c_i32, c_vp, c_i64, c_vp]),
    "hlhgat_bn_fwd_train": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                    c_vp, c_f32, c_f32, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp,
                                    c_i64, c_vp]),
    "hlhgat_bn_bwd_train": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64,
                                    c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                                    c_vp]),
    "hlhgat_adam_prepare": (c_i32, [c_vp, c_i64, c_vp, c_vp]),
    "hlhgat_adam_flat_prepared": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_f64, c_f64,
                                          c_f64, c_f64, c_f64, c_vp]),
    "hlhgat_adam_flat": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_f64, c_f64, c_f64,
                                 c_f64, c_f64, c_vp]),
    "hlhgat_bce_logits_fwd": (c_i32, [c_vp, c_vp, c_i64, c_f32, c_vp, c_vp]),
    "hlhgat_bce_logits_bwd": (c_i32, [c_vp, c_vp, c_i64, c_f32, c_vp, c_vp, c_vp]),
    "hlhgat_l1_loss_fwd": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    "hlhgat_l1_loss_bwd": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "hlhgat_bn_sums_len": (c_i64, [c_i64]),
    "hlhgat_bn_sums_fwd": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp,
                                   c_i64, c_vp]),
    "hlhgat_bn_sync_fwd_apply": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i32, c_vp,
                                         c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_i32, c_vp,
                                         c_i64, c_vp, c_vp, c_vp]),
    "hlhgat_bn_sums_bwd": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64,
                                   c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64,
                                   c_vp]),
    "hlhgat_bn_sync_bwd_apply": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp,
                                         c_i64, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_i64,
                                         c_vp]),
    "hlhgat_bn_stats_train": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_f32,
                                      c_f32, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "hlhgat_bn_apply": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i32,
                                c_vp, c_i64, c_vp]),
    "hlhgat_zero_fill": (c_i32, [c_vp, c_sz, c_vp]),
    "hlhgat_copy2d_batched": (c_i32, [c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "hlhgat_prof_enable": (c_i32, [c_i32, c_i32]),
    "hlhgat_prof_reset": (c_i32, []),
    "hlhgat_prof_read": (c_i32, [c_i32, P_i64, P_f64, P_f64, P_f64]),
    "hlhgat_graph_kernel_count": (c_i32, [c_vp, C.c_char_p, P_i64, P_i64]),
}

# constants from include/hlhgat.h
POLY_LAGUERRE, POLY_CHEB, POLY_LAGUERRE_DEMO = 0, 1, 2
SIGMA_SIGMOID, SIGMA_RELU = 0, 1
DEVERR_BN_STATE = 1
DEVERR_HODGE_SIZE = 2
BN_LOG_MAX = 64
PROF_POLY, PROF_PROJ, PROF_HODGE_NODE, PROF_HODGE_EDGE = 0, 1, 2, 3
PROF_PROJ_BWD, PROF_BN_FWD, PROF_BN_BWD, PROF_PROJ_BN = 4, 5, 6, 7
PROF_POLY_ADJ, PROF_INCIDENCE, PROF_GATHER2 = 8, 9, 10
MAX_BLOCKS = 16


class BnGiveup(C.Structure):
    """hlhgat_bn_giveup_t (include/hlhgat.h): one give-up of a one-launch
    BatchNorm workgroup, as it recorded it."""
    _fields_ = [(f, C.c_uint32) for f in ("kernel", "tile", "block", "total", "arrivals", "gen0",
                                          "gen_seen", "wait_us", "outcome")]


class HaloDesc(C.Structure):
    """hlhgat_halo_t (include/hlhgat.h)."""
    _fields_ = [("hdr", c_vp), ("tile_ptr", c_vp), ("halo_ptr", c_vp), ("halo", c_vp), ("srp", c_vp),
                ("lcol", c_vp), ("sval", c_vp), ("n_tiles", c_i64), ("max_halo", c_i32),
                ("max_rows", c_i32), ("max_nnz", c_i32)]


class HodgeFactorDesc(C.Structure):
    """hlhgat_hodge_factor_t (include/hlhgat.h)."""
    _fields_ = [("node_rowptr", c_vp), ("node_edge", c_vp), ("node_sign", c_vp),
                ("node_order", c_vp), ("n_nodes", c_i64), ("ends", c_vp), ("alpha", c_vp),
                ("edge_order", c_vp), ("n_edges", c_i64)]


class PackedGraphsDesc(C.Structure):
    """hlhgat_packed_graphs_t (include/hlhgat.h)."""
    _fields_ = [("n_graphs", c_i64), ("node_ptr", c_vp), ("edge_ptr", c_vp), ("lt_ptr", c_vp),
                ("ls_ptr", c_vp), ("x_t", c_vp), ("f_t", c_i64), ("x_s", c_vp), ("f_s", c_i64),
                ("lt_row", c_vp), ("lt_col", c_vp), ("lt_w", c_vp), ("ls_row", c_vp),
                ("ls_col", c_vp), ("ls_w", c_vp), ("b1_src", c_vp), ("b1_dst", c_vp),
                ("y", c_vp), ("y_dim", c_i64)]


class CollatedDesc(C.Structure):
    """hlhgat_collated_t (include/hlhgat.h)."""
    _fields_ = [("rows_t", c_i64), ("rows_s", c_i64), ("nnz_t", c_i64), ("nnz_s", c_i64),
                ("x_t", c_vp), ("x_s", c_vp), ("edge_index_t", c_vp), ("edge_weight_t", c_vp),
                ("edge_index_s", c_vp), ("edge_weight_s", c_vp), ("edge_index", c_vp),
                ("y", c_vp), ("num_node1", c_vp), ("num_edge1", c_vp), ("csr_rowptr_t", c_vp),
                ("csr_col_t", c_vp), ("csr_rowptr_s", c_vp), ("csr_col_s", c_vp),
                ("inc_rowptr", c_vp), ("inc_eids", c_vp), ("deg_t", c_vp), ("inv_deg_t", c_vp),
                ("seg_ptr_t", c_vp), ("seg_ptr_s", c_vp), ("valid_mask_t", c_vp),
                ("n_t", c_i64), ("n_s", c_i64)]


class HlhgatError(RuntimeError):
    pass


def load(path: str = LIB_PATH) -> C.CDLL:
    if not os.path.exists(path):
        raise ImportError(
            f"hlhgat: HIP library not found at {path}. Build it with "
            f"`python -c 'import __graft_entry__ as g; g.build()'` or "
            f"`make -C hl-hgat_amd/csrc` (hipcc --offload-arch=gfx950).")
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError if a declared symbol is missing
        fn.restype = res
        fn.argtypes = args
    return lib


LIB = load()


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = LIB.hlhgat_last_error().decode(errors="replace")
        raise HlhgatError(f"{what} failed (code {rc}): {msg}")
