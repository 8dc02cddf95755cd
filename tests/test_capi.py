"""C ABI checks that need no GPU: the library loads, exports every symbol the
public header declares, host helpers match torch, and argument errors come
back as codes + messages (mirroring the reference's TORCH_CHECK /
runtime_error messages, gridencoder.cu:15-18, :392, :409)."""
import ctypes
import os
import re

import pytest
import torch

from conftest import REPO

HEADER = os.path.join(REPO, "include", "samnerf_hip.h")


def header_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(samnerf_\w+)\s*\(", text, re.M)))


def test_header_declares_expected_entry_points():
    syms = header_symbols()
    for s in ["samnerf_grid_encode_forward", "samnerf_grid_encode_backward",
              "samnerf_grad_total_variation", "samnerf_grad_weight_decay",
              "samnerf_sh_encode_forward", "samnerf_sh_encode_backward",
              "samnerf_freq_encode_forward", "samnerf_freq_encode_backward",
              "samnerf_render_forward", "samnerf_sgrid_backward"]:
        assert s in syms


def test_library_exports_every_header_symbol(hip_lib):
    from samnerf_amd import EXPORTED
    syms = header_symbols()
    missing = [s for s in syms if not hasattr(hip_lib, s)]
    assert not missing, missing
    assert sorted(EXPORTED) == syms, "ctypes signature table out of sync with the header"
    assert hip_lib.samnerf_version().startswith(b"samnerf_hip")


@pytest.mark.parametrize("start,end,steps", [(0, 1, 129), (0.5 / 65, 1 - 0.5 / 65, 65),
                                             (0.5 / 33, 1 - 0.5 / 33, 33),
                                             (0.5 / 129, 1 - 0.5 / 129, 129), (0, 511, 512),
                                             (-3.0, 7.25, 97), (2.0, 2.0, 1)])
def test_linspace_host_is_torch_exact(hip_lib, start, end, steps):
    from samnerf_amd.ops import linspace_host
    got = torch.tensor(linspace_host(start, end, steps))
    ref = torch.linspace(start, end, steps)
    assert torch.equal(got, ref)


def test_argument_errors_return_codes_and_messages(hip_lib):
    L = hip_lib
    p = ctypes.c_void_p(64)      # never dereferenced: validation fails first
    rc = L.samnerf_grid_encode_forward(None, p, p, p, 1, 3, 2, 16, 16, 0.5, 16, None, 0, 0, 0, None)
    assert rc == -1 and b"null" in L.samnerf_last_error()
    rc = L.samnerf_grid_encode_forward(p, p, p, p, 4, 3, 3, 16, 16, 0.5, 16, None, 0, 0, 0, None)
    assert rc == -1 and L.samnerf_last_error() == b"GridEncoding: C must be 1, 2, 4, 8, 16 or 32."
    rc = L.samnerf_grid_encode_forward(p, p, p, p, 4, 6, 2, 16, 16, 0.5, 16, None, 0, 0, 0, None)
    assert rc == -1 and L.samnerf_last_error() == b"GridEncoding: D must be 2, 3, 4 or 5."
    rc = L.samnerf_sh_encode_forward(p, p, 4, 3, 9, None, None)
    assert rc == -1 and b"degree in [1, 8]" in L.samnerf_last_error()
    rc = L.samnerf_freq_encode_forward(p, 4, 3, 6, 40, p, None)
    assert rc == -1
    # zero-size work is a successful no-op (no launch)
    assert L.samnerf_grid_encode_forward(p, p, p, p, 0, 3, 2, 16, 16, 0.5, 16, None, 0, 0, 0, None) == 0


def test_render_workspace_size_scales_with_rays(hip_lib):
    from samnerf_amd._lib import SamnerfModel
    m = SamnerfModel()
    m.with_sam = 1
    for i, v in enumerate((128, 64, 32)):
        m.num_steps[i] = v
    a = hip_lib.samnerf_render_workspace_size(ctypes.byref(m), 1024)
    b = hip_lib.samnerf_render_workspace_size(ctypes.byref(m), 2048)
    assert 0 < a < b
    # about 2 KiB of per-ray state + the packed head weights
    assert 1024 * 2000 < a < 1024 * 2100 + 2 * 1024 * 1024


def test_python_shims_reject_non_cuda_tensors(hip_lib):
    import _gridencoder
    import _shencoder
    x = torch.zeros(4, 3)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        _gridencoder.grid_encode_forward(x, torch.zeros(8, 2), torch.zeros(2, dtype=torch.int32),
                                         torch.zeros(1, 4, 2), 4, 3, 2, 1, 1, 1.0, 16, None, 0,
                                         False, 0)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        _shencoder.sh_encode_forward(x, torch.zeros(4, 16), 4, 3, 4, None)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    import samnerf_amd._lib as L
    monkeypatch.setattr(L, "_lib", None)
    monkeypatch.setattr(L, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(L.SamnerfUnavailable, match="no CPU fallback"):
        L.lib()


def test_mask_train_workspace_size_is_model_aware(hip_lib):
    """the adaptive heads (mask_kind 1 / 2) need 2 x 7 x 96 floats
    per ray, not the 'default' head's ~157 KB activation carve."""
    from samnerf_amd._lib import SamnerfModel
    m = SamnerfModel()
    m.with_mask = 1
    n = 4096
    m.mask_kind = 0
    dflt = hip_lib.samnerf_mask_train_workspace_size_model(ctypes.byref(m), n)
    assert dflt == hip_lib.samnerf_mask_train_workspace_size(n)
    assert dflt > 150_000 * n
    for kind in (1, 2):
        m.mask_kind = kind
        assert hip_lib.samnerf_mask_train_workspace_size_model(ctypes.byref(m), n) == 2 * 7 * 96 * 4 * n
