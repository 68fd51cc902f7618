"""The C-ABI library loads on a GPU-less host and exports every symbol that
include/hlhgat.h declares (no compute calls here)."""
import ctypes
import os
import re

from conftest import REPO

HEADER = os.path.join(REPO, "include", "hlhgat.h")
LIB = os.path.join(REPO, "hl-hgat_amd", "hlhgat", "libhlhgat.so")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hlhgat_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_hot_path():
    syms = declared_symbols()
    for s in ("hlhgat_spmm", "hlhgat_poly_step", "hlhgat_poly_basis_fwd",
              "hlhgat_poly_basis_bwd", "hlhgat_proj_fwd", "hlhgat_proj_bwd_data",
              "hlhgat_proj_bwd_weight", "hlhgat_edge_gather2", "hlhgat_incidence_csr",
              "hlhgat_att_score_fwd", "hlhgat_att_score_bwd", "hlhgat_csr_from_coo",
              "hlhgat_csr_from_sorted_coo", "hlhgat_segment_mean_fwd"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    import torch  # noqa: F401  (shares the HIP runtime, as the product does)
    lib = ctypes.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_signatures_cover_header():
    import torch  # noqa: F401
    from hlhgat import _lib
    assert set(_lib.SIGNATURES) == set(declared_symbols())
    assert _lib.LIB.hlhgat_version() >= 100


def test_errors_surface_without_gpu():
    """Argument validation runs before any HIP call and reports a message."""
    import torch  # noqa: F401
    from hlhgat import _lib
    rc = _lib.LIB.hlhgat_poly_basis_fwd(7, None, None, None, 10, 0, None, None, None, 1, 1, 3,
                                        None, None)
    assert rc == 1
    assert b"bad kind" in _lib.LIB.hlhgat_last_error()
    rc = _lib.LIB.hlhgat_spmm(None, None, None, 4, 0, None, None, None, 1, 0, None, 1, None)
    assert rc == 1


def test_product_has_no_cpu_fallback():
    import pytest
    import torch
    from hlhgat import ops
    with pytest.raises(RuntimeError, match="ROCm device"):
        ops.linear_blocks([torch.randn(4, 3)], torch.randn(2, 3), None)
