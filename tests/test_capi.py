"""CPU: the native build loads and exposes the full boundary (no GPU compute)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "dpvo_hot.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dpvo_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    import dpvo_amd

    return dpvo_amd.c_abi()


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ["dpvo_corr_forward", "dpvo_corr_backward", "dpvo_patchify_forward",
                 "dpvo_patchify_backward", "dpvo_ba_forward", "dpvo_reproject", "dpvo_neighbors",
                 "dpvo_lie_forward", "dpvo_lie_backward", "dpvo_corr_forward_levels",
                 "dpvo_ba_build_schur", "dpvo_ba_solve_update"]:
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_status_and_version(lib):
    assert lib.dpvo_version().startswith(b"dpvo_hot gfx950")
    assert lib.dpvo_status_string(0) == b"ok"
    assert lib.dpvo_status_string(3) == b"unsupported configuration"


def test_host_side_argument_validation(lib):
    # invalid arguments are rejected before any kernel launch (no GPU needed)
    f = lib.dpvo_corr_forward
    # radius 8 > 7 -> DPVO_ERR_INVALID
    assert f(None, None, None, None, None, 1, 4, 128, 3, 3, 1, 1, 10, 10, 8, 0, None, None) == 1
    # patch of 5x5 = 25 pixels > 16 -> DPVO_ERR_UNSUPPORTED
    assert f(None, None, None, None, None, 1, 4, 128, 5, 5, 1, 1, 10, 10, 3, 0, None, None) == 3
    # zero edges is a no-op success
    assert f(None, None, None, None, None, 1, 0, 128, 3, 3, 1, 1, 10, 10, 3, 0, None, None) == 0
    # BA: t1 < t0 invalid; too many free poses unsupported; workspace too small
    ba_setup = lib.dpvo_ba_setup
    one = ctypes.c_void_p(1)
    assert ba_setup(one, one, one, 10, 100, 5, 4, one, ctypes.c_size_t(1 << 30), None) == 1
    assert ba_setup(one, one, one, 10, 100, 0, 64, one, ctypes.c_size_t(1 << 30), None) == 3
    assert ba_setup(one, one, one, 10, 100, 0, 4, one, ctypes.c_size_t(16), None) == 4
    assert lib.dpvo_lie_forward(2, 0, 0, 4, None, None, None, None) == 3  # RxSO3 not built


def test_workspace_size_grows_with_problem(lib):
    a = lib.dpvo_ba_workspace_bytes(256, 1, 8)
    b = lib.dpvo_ba_workspace_bytes(2048, 1, 12)
    assert 0 < a < b


def test_extension_modules_expose_reference_surface():
    import dpvo_amd

    corr = dpvo_amd.load_extension("cuda_corr")
    ba = dpvo_amd.load_extension("cuda_ba")
    lie = dpvo_amd.load_extension("lietorch_backends")
    for n in ["forward", "backward", "patchify_forward", "patchify_backward"]:
        assert hasattr(corr, n)  # correlation.cpp:57-63
    for n in ["forward", "neighbors", "reproject", "solve_system"]:
        assert hasattr(ba, n)  # ba.cpp:183-189
    for n in ["expm", "expm_backward", "logm", "logm_backward", "inv", "inv_backward", "mul",
              "mul_backward", "adj", "adj_backward", "adjT", "adjT_backward", "act",
              "act_backward", "act4", "act4_backward", "as_matrix", "projector", "Jinv"]:
        assert hasattr(lie, n)  # lietorch.cpp:286-316
    # the import is the in-tree build, not something on site-packages
    assert os.path.realpath(corr.__file__).startswith(os.path.realpath(dpvo_amd.NATIVE_DIR))


def test_cpu_tensors_are_rejected_loudly():
    import torch

    import dpvo_amd

    corr = dpvo_amd.load_extension("cuda_corr")
    f1 = torch.zeros(1, 2, 8, 3, 3)
    f2 = torch.zeros(1, 2, 8, 10, 10)
    co = torch.zeros(1, 1, 2, 3, 3)
    ii = torch.zeros(1, dtype=torch.long)
    with pytest.raises(RuntimeError, match="GPU"):
        corr.forward(f1, f2, co, ii, ii, 3)
