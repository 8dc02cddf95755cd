"""ctypes binding of libsamnerf_hip.so (include/samnerf_hip.h).

The product path has no fallback: if the HIP library is missing or cannot be
loaded, every op raises SamnerfUnavailable with the build command.
"""
import contextlib
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SAMNERF_LIB: another build of the same library (A/B timing of two builds in
# one GPU session); the in-tree build otherwise.
LIB_PATH = os.environ.get("SAMNERF_LIB") or os.path.join(_HERE, "libsamnerf_hip.so")

_u32 = ctypes.c_uint32
_f32 = ctypes.c_float
_f64 = ctypes.c_double
_int = ctypes.c_int
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t


class SamnerfUnavailable(RuntimeError):
    pass


class SamnerfGrid(ctypes.Structure):
    _fields_ = [("embeddings", _vp), ("offsets_host", ctypes.POINTER(ctypes.c_int32)),
                ("num_levels", _u32), ("level_dim", _u32), ("S", _f32),
                ("base_resolution", _u32)]


class SamnerfModel(ctypes.Structure):
    _fields_ = [("grid", SamnerfGrid), ("s_grid", SamnerfGrid), ("prop", SamnerfGrid * 2),
                ("grid_mlp", _vp * 3), ("view_mlp", _vp * 3), ("prop_mlp", (_vp * 2) * 2),
                ("sam_w", _vp * 5), ("sam_b", _vp * 5), ("ln_w", _vp), ("ln_b", _vp),
                ("with_sam", _int), ("aabb", _f32 * 6), ("grid_bound", _f32),
                ("min_near", _f32), ("num_steps", _u32 * 3), ("head_mode", _int),
                ("t_thresh", _f32), ("view_width", _u32),
                ("with_mask", _int), ("mask_kind", _int), ("m_grid", SamnerfGrid), ("mask_w", _vp * 8),
                ("mask_out", _u32),
                ("sum_after_mlp", _int), ("perturb", _vp * 3), ("reuse_packed", _int)]


_SIGS = {
    "samnerf_diag_variants": ([], _int),
    "samnerf_version": ([], ctypes.c_char_p),
    "samnerf_last_error": ([], ctypes.c_char_p),
    "samnerf_grid_encode_forward": ([_vp, _vp, _vp, _vp, _u32, _u32, _u32, _u32, _u32, _f32, _u32,
                                     _vp, _u32, _int, _u32, _vp], _int),
    "samnerf_grid_encode_backward": ([_vp, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _u32, _u32, _f32,
                                      _u32, _vp, _vp, _u32, _int, _u32, _vp], _int),
    "samnerf_grad_total_variation": ([_vp, _vp, _vp, _vp, _f32, _u32, _u32, _u32, _u32, _f32, _u32,
                                      _u32, _int, _vp], _int),
    "samnerf_grad_weight_decay": ([_vp, _vp, _vp, _f32, _u32, _u32, _u32, _vp], _int),
    "samnerf_sh_encode_forward": ([_vp, _vp, _u32, _u32, _u32, _vp, _vp], _int),
    "samnerf_sh_encode_backward": ([_vp, _vp, _u32, _u32, _u32, _vp, _vp, _vp], _int),
    "samnerf_freq_encode_forward": ([_vp, _u32, _u32, _u32, _u32, _vp, _vp], _int),
    "samnerf_freq_encode_backward": ([_vp, _vp, _u32, _u32, _u32, _u32, _vp, _vp], _int),
    "samnerf_get_rays": ([ctypes.POINTER(_f32), _f32, _f32, _f32, _f32, _u32, _u32, _u32, _u32,
                          _vp, _vp, _vp], _int),
    "samnerf_near_far": ([_vp, _vp, _u32, ctypes.POINTER(_f32), _f32, _vp, _vp, _vp], _int),
    "samnerf_contract": ([_vp, _vp, _u32, _vp], _int),
    "samnerf_sample_pdf": ([_vp, _vp, _u32, _u32, _u32, _vp, _vp, _vp], _int),
    "samnerf_composite_weights": ([_vp, _vp, _u32, _u32, _vp, _vp], _int),
    "samnerf_linspace_host": ([_f32, _f32, _u32, ctypes.POINTER(_f32)], None),
    "samnerf_render_workspace_size": ([ctypes.POINTER(SamnerfModel), _u32], _sz),
    "samnerf_render_forward": ([ctypes.POINTER(SamnerfModel), _vp, _vp, _u32, _vp, _u32, _f32,
                                _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp], _int),
    "samnerf_render_forward_tile": ([ctypes.POINTER(SamnerfModel), _vp, _vp, _u32, _vp, _u32, _f32,
                                     _vp, _u32, _int, _vp, _vp, _sz, _vp], _int),
    "samnerf_sgrid_backward": ([ctypes.POINTER(SamnerfModel), _vp, _u32, _vp, _vp, _sz, _vp],
                               _int),
    "samnerf_sgrid_accum_size": ([ctypes.POINTER(SamnerfModel)], _sz),
    "samnerf_sgrid_backward_det": ([ctypes.POINTER(SamnerfModel), _vp, _u32, _vp, _vp, _sz, _vp, _sz, _vp],
                                   _int),
    "samnerf_mask_forward": ([ctypes.POINTER(SamnerfModel), _u32, _vp, _vp, _sz, _vp], _int),
    "samnerf_tile_words": ([], _u32),
    "samnerf_tile_encode": ([_vp, _vp, _vp, _vp, _u32, _vp, _vp], _int),
    "samnerf_tile_decode": ([_vp, _u32, _vp, _vp, _vp, _vp, _vp], _int),
    "samnerf_set_stage_events": ([ctypes.POINTER(_vp), _u32], _int),
    "samnerf_set_taps": ([ctypes.c_void_p, _u32], _int),
    "samnerf_last_forms": ([ctypes.c_void_p, _u32], _int),
    "samnerf_clock_stamp": ([_vp, _vp], _int),
    "samnerf_adam_step": ([ctypes.c_void_p, _u32, _f64, _f64, _f64, _f64, _f64, _u32, _vp], _int),
    "samnerf_rgb_train_workspace_size": ([ctypes.POINTER(SamnerfModel), _u32], _sz),
    "samnerf_rgb_train_step": ([ctypes.POINTER(SamnerfModel), _vp, _vp, _u32, _vp, _u32, _vp,
                                ctypes.c_void_p, _vp, _vp, _vp, _vp, ctypes.c_void_p, _vp, _sz, _vp], _int),
    "samnerf_rgb_train_forward": ([ctypes.POINTER(SamnerfModel), _vp, _vp, _u32, _vp, _u32, _f32, _int,
                                   _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp], _int),
    "samnerf_rgb_train_backward": ([ctypes.POINTER(SamnerfModel), _vp, _vp, _u32, _f32, _int, _vp, _vp,
                                    _vp, _vp, _vp, ctypes.c_void_p, _vp, _sz, _vp], _int),
    "samnerf_sam_head_workspace_size": ([], _sz),
    "samnerf_sam_head_forward": ([ctypes.POINTER(SamnerfModel), _vp, _u32, _vp, _vp, _sz, _vp], _int),
    "samnerf_head_train_workspace_size": ([_u32], _sz),
    "samnerf_head_train_forward": ([ctypes.POINTER(SamnerfModel), _vp, _u32, _vp, _vp, _sz, _vp], _int),
    "samnerf_head_train_backward": ([ctypes.POINTER(SamnerfModel), _vp, _vp, _u32, _vp,
                                     ctypes.POINTER(_vp), ctypes.POINTER(_vp), _vp, _vp, _vp, _sz,
                                     _vp], _int),
    "samnerf_mask_train_workspace_size": ([_u32], _sz),
    "samnerf_mask_train_workspace_size_model": ([ctypes.POINTER(SamnerfModel), _u32], _sz),
    "samnerf_mask_train_forward": ([ctypes.POINTER(SamnerfModel), _u32, _vp, _vp, _sz, _vp, _sz, _vp], _int),
    "samnerf_mask_train_backward": ([ctypes.POINTER(SamnerfModel), _u32, _vp, ctypes.POINTER(_vp), _vp, _vp,
                                     _sz, _vp, _sz, _vp], _int),
}


class SamnerfAdamTensor(ctypes.Structure):
    """samnerf_adam_tensor (include/samnerf_hip.h)."""
    _fields_ = [("param", _vp), ("grad", _vp), ("exp_avg", _vp), ("exp_avg_sq", _vp),
                ("n", ctypes.c_uint64)]


class SamnerfTaps(ctypes.Structure):
    """samnerf_taps (include/samnerf_hip.h): parity-test taps of the render."""
    _fields_ = [("ds0", _vp), ("ds1", _vp), ("w0", _vp), ("w1", _vp), ("bins1", _vp),
                ("bins2", _vp), ("inds1", _vp), ("inds2", _vp), ("sigma2", _vp), ("w2", _vp),
                ("u2", _vp), ("row_stride", _u32), ("rows2", _vp), ("srows", _vp)]


class SamnerfRgbTrainOpts(ctypes.Structure):
    """samnerf_rgb_train_opts (include/samnerf_hip.h)."""
    _fields_ = [("lambda_proposal", _f32), ("lambda_distort", _f32), ("lambda_entropy", _f32),
                ("update_proposal", _int), ("bg_color", _f32)]


class SamnerfRgbGrads(ctypes.Structure):
    """samnerf_rgb_grads (include/samnerf_hip.h)."""
    _fields_ = [("grid", _vp), ("grid_mlp", _vp * 3), ("view_mlp", _vp * 3), ("prop", _vp * 2),
                ("prop_mlp", (_vp * 2) * 2)]


EXPORTED = tuple(_SIGS)
_lib = None


def _load(path, lenient=False):
    if not os.path.exists(path):
        raise SamnerfUnavailable(
            f"{path} is not built; run `python segment-anything-nerf_amd/build.py` "
            "(or __graft_entry__.build()).  There is no CPU fallback.")
    try:
        L = ctypes.CDLL(path)
    except OSError as e:
        raise SamnerfUnavailable(f"cannot load {path}: {e}") from e
    for name, (args, res) in _SIGS.items():
        if lenient and not hasattr(L, name):
            continue                  # an older diagnostic build (tools/diag) lacks newer entry points
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    return L


def lib():
    """Load the HIP library (once).  Raises SamnerfUnavailable if absent."""
    global _lib
    if _lib is None:
        _lib = _load(LIB_PATH, lenient=bool(os.environ.get("SAMNERF_LIB")))
    return _lib


DIAG_LIB_PATH = os.path.join(_HERE, "libsamnerf_hip_diag.so")
_diag = None


@contextlib.contextmanager
def diag_library():
    """Tests and tools only: while the context is active, EVERY call of the
    process (all threads: the swap is of the module-global library handle)
    goes through the diagnostic build (libsamnerf_hip_diag.so), whose kernels
    read the A/B variant switches (SAMNERF_LOOKUP, SAMNERF_FINAL_S, ...) from
    the environment -- the product library has one path per configuration.
    Not for use while product renders run on other threads."""
    global _lib, _diag
    if _diag is None:
        _diag = _load(DIAG_LIB_PATH)
        assert _diag.samnerf_diag_variants() == 1
    prev = lib()
    _lib = _diag
    try:
        yield _diag
    finally:
        _lib = prev


def check(rc, what):
    if rc != 0:
        msg = lib().samnerf_last_error().decode(errors="replace")
        raise RuntimeError(f"{what}: {msg} (code {rc})")


def last_error():
    return lib().samnerf_last_error().decode(errors="replace")
