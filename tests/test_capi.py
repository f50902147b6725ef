"""The C-ABI library loads on the CPU and exports exactly what include/kcmc.h declares."""
import ctypes
import os
import re

import numpy as np

from kcmc_amd import _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "kcmc.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(kcmc_\w+)\s*\(", src))


def test_header_declarations_match_binding_table():
    assert _declared() == set(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    for name in _declared():
        assert hasattr(L, name), name
    # dynamic symbol table of the shared object itself
    out = os.popen(f"nm -D --defined-only {_lib.lib_path()}").read()
    for name in _declared():
        assert re.search(rf"\bT {name}\b", out), name


def test_library_has_no_unresolved_internal_symbols():
    """Every kcmc:: symbol one translation unit uses is defined in the library (a helper
    left with internal linkage links into a .so silently and fails only at load time)."""
    out = os.popen(f"nm -D --undefined-only {_lib.lib_path()}").read()
    assert not re.findall(r"\S*kcmc\S*", out), out


def test_abi_version_and_error_reporting():
    L = _lib.load()
    assert L.kcmc_abi_version() == _lib.ABI_VERSION
    out = np.zeros(4, np.int32)
    rc = L.kcmc_hypothesis_table(0, 2, 42, 2, out.ctypes.data_as(ctypes.c_void_p))
    assert rc == _lib.KCMC_EINVAL
    assert b"min_samples" in L.kcmc_last_error()
    h = ctypes.c_void_p()
    assert L.kcmc_create(-1, ctypes.byref(h)) != _lib.KCMC_OK  # no GPU here, or a bad ordinal there
    assert L.kcmc_last_error()


def test_launch_entry_points_validate_before_touching_the_gpu():
    L = _lib.load()
    P = ctypes.c_void_p
    assert L.kcmc_knn2_l2u8(None, None, 1, 32, None, None, 1, 2, None, None, None) == _lib.KCMC_EINVAL
    assert L.kcmc_warp_affine_u16(None, None, None, None, 1, 4, 4, 1, 0, None) == _lib.KCMC_EINVAL
    assert L.kcmc_ransac_rigid(None, None, None, None, None, 0, 1, 10, 1000, 2.0, 1.0, 3, None, None, None, None,
                               None) == _lib.KCMC_EINVAL
    assert L.kcmc_ransac_prepare(None, None, 1, 1000, 42) == _lib.KCMC_EINVAL
    assert L.kcmc_consensus(None, -1, 0, 0, 0, None, None, None, None, None) == _lib.KCMC_EINVAL
    assert L.kcmc_ransac_model(None, 1, None, None, None, None, 0, 1, 10, 1000, 2.0, 1.0, 3, None, None, None,
                               None, None) == _lib.KCMC_EINVAL
    assert L.kcmc_ransac_prepare_samples(None, 3, None, 1, 1000, 42) == _lib.KCMC_EINVAL
    assert L.kcmc_warp_perspective_u16(None, None, None, None, 1, 4, 4, 1, 0, None) == _lib.KCMC_EINVAL
    assert L.kcmc_consensus_vote(None, None, 1, 8, 0, None, None) == _lib.KCMC_EINVAL
    assert L.kcmc_consensus_lookup(None, None, 1, 8, None, 1, None, None, None, None) == _lib.KCMC_EINVAL
    assert L.kcmc_params_boundary(None, None, 1, 6, None, None) == _lib.KCMC_EINVAL
    assert L.kcmc_consensus_merge(None, 0, 8, 1, 1, None, None, None, None) == _lib.KCMC_EINVAL
    assert L.kcmc_memcpy_async(None, None, 8, None) == _lib.KCMC_EINVAL
    # the filter-only entry (knn results from elsewhere)
    assert L.kcmc_match_filter(None, None, None, None, None, None, 1, 8, 0.75, 0.5, 2.0, None, None, None,
                               None) == _lib.KCMC_EINVAL
    del P
