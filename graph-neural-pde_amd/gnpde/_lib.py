"""ctypes binding of libgnpde.so (the C ABI declared in include/gnpde.h).

The library is built in-tree by ``make -C graph-neural-pde_amd`` (or
``__graft_entry__.build()``).  There is no fallback: if the shared object is
missing or fails to load, every call raises.  This binding is exactly what a
maintainer of the reference would add next to ``src/utils.py`` to reach the
native path (INTEGRATION.md shows it).
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GNPDE_LIB", os.path.join(_HERE, "libgnpde.so"))

STAGE_MAX_OUT = 2
STAGE_MAX_K = 6
STAGE_PRE_K = 2  # operands the fixed-grid epilogues prefetch (csrc/common.hpp kStagePre)
DENSE_BASIS = 5  # the folded dense output's basis polynomials (ABI 8)
DENSE_SLOTS = STAGE_MAX_K + 2  # its operand slots: output 0's base, k[0..5], f


class StageOut(ctypes.Structure):
    """gnpde_stage_out_t: out = cb*base + cf*f + sum_j c[j]*k[j] (k: the stage's shared operands)."""
    _fields_ = [("out", ctypes.c_void_p), ("base", ctypes.c_void_p), ("cb", ctypes.c_float), ("cf", ctypes.c_float),
                ("c", ctypes.c_float * STAGE_MAX_K)]


class StageEpilogue(ctypes.Structure):
    """gnpde_stage_epilogue_t (include/gnpde.h)."""
    _fields_ = [("f_out", ctypes.c_void_p), ("n_out", ctypes.c_int), ("o", StageOut * STAGE_MAX_OUT),
                ("nk", ctypes.c_int), ("k", ctypes.c_void_p * STAGE_MAX_K),
                ("out_rows", ctypes.c_void_p), ("dot_with", ctypes.c_void_p), ("dot_rows", ctypes.c_void_p),
                ("dot_coef", ctypes.c_double), ("dot_accumulate", ctypes.c_int),
                ("err_rows", ctypes.c_void_p), ("err", StageOut), ("err_y0", ctypes.c_void_p), ("err_y1", ctypes.c_int),
                ("atol", ctypes.c_double), ("rtol", ctypes.c_double), ("coef_scale", ctypes.c_void_p),
                ("f_lin", ctypes.c_float), ("unscaled_outs", ctypes.c_int),
                ("dense_out", ctypes.c_void_p), ("dense_rows", ctypes.c_void_p), ("dense_t", ctypes.c_void_p),
                ("dense_dt", ctypes.c_void_p), ("dense_tab", ctypes.c_void_p),
                ("dense_m", (ctypes.c_float * DENSE_SLOTS) * DENSE_BASIS), ("scale_rows", ctypes.c_void_p)]


c_i32p = ctypes.POINTER(ctypes.c_int32)
c_i64p = ctypes.POINTER(ctypes.c_int64)
_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int
_f32 = ctypes.c_float
_f64 = ctypes.c_double
_size = ctypes.c_size_t

# name -> (restype, argtypes); every entry point of include/gnpde.h
SIGNATURES = {
    "gnpde_abi_version": (_int, []),
    "gnpde_last_error": (ctypes.c_char_p, []),
    "gnpde_build_id": (ctypes.c_char_p, []),
    "gnpde_csr_workspace_bytes": (_size, [_i64, _i64, _i64]),
    "gnpde_csr_build": (_int, [_vp, _i64, _i64, _i64, _int, _vp, _vp, _vp, _vp, _size, _vp]),
    "gnpde_gather_weights_f32": (_int, [_vp, _i64, _int, _vp, _vp, _vp]),
    "gnpde_indegree_i32": (_int, [_vp, _i64, _i64, _vp, _vp]),
    "gnpde_mix_weights_f32": (_int, [_vp, _int, _vp, _vp, _i64, _vp, _vp]),
    "gnpde_group_normalize_workspace_bytes": (_size, [_i64]),
    "gnpde_group_normalize_f32": (_int, [_vp, _vp, _i64, _i64, _vp, _vp, _vp, _size, _vp]),
    "gnpde_quantile_workspace_bytes": (_size, [_i64]),
    "gnpde_quantile_f32": (_int, [_vp, _i64, _f64, _vp, _vp, _size, _vp]),
    "gnpde_plan_workspace_bytes": (_size, [_i64]),
    "gnpde_plan_build": (_int, [_vp, _i64, ctypes.c_int32, _vp, _i64, _vp, _i64, c_i64p, c_i64p, c_i64p, _vp,
                                _size, _vp]),
    "gnpde_spmm_rhs_f32": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _int, _vp,
                                  _i64, _vp, _i64, ctypes.POINTER(StageEpilogue), _vp]),
    "gnpde_spmm_rhs_bf16": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _int, _vp,
                                   _i64, _vp, _i64, ctypes.POINTER(StageEpilogue), _vp]),
    "gnpde_attn_ref_rhs_f32": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _i64, _vp, _i64,
                                      _vp, _vp, _int, _vp, _i64, _vp, _i64, ctypes.POINTER(StageEpilogue), _vp]),
    "gnpde_attn_dot_supported": (_int, [_i64, _i64, _i64]),
    "gnpde_attn_dot_workspace_floats": (_i64, [_i64, _i64, _i64]),
    "gnpde_attn_dot_rhs_f32": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp,
                                      _i64, _vp, _vp, _int, _vp, _i64, _vp, _i64, ctypes.POINTER(StageEpilogue), _vp]),
    "gnpde_attn_dot_rhs_bf16": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp,
                                      _i64, _vp, _vp, _int, _vp, _i64, _vp, _i64, ctypes.POINTER(StageEpilogue), _vp]),
    "gnpde_rows_copy": (_int, [_vp, _i64, _i64, _vp, _vp, _vp, _vp]),
    "gnpde_threshold_mask_f32": (_int, [_vp, _i64, _vp, _vp, _vp, _vp]),
    "gnpde_initial_step_workspace_bytes": (_size, []),
    "gnpde_adaptive_control": (_int, [_i64, _vp, _f64, _f64, _f64, _f64, _f64, _vp, _vp, _vp, _vp, _vp, _size, _vp]),
    "gnpde_initial_step_f32": (_int, [_i64, _vp, _vp, _vp, _f64, _f64, _f64, _vp, _vp, _vp, _size, _vp]),
    "gnpde_initial_step_rows": (_int, [_i64, _vp, _vp, _f64, _f64, _vp, _vp, _vp, _size, _vp]),
    "gnpde_initial_step_lin_f32": (_int, [_i64, _vp, _vp, _f64, _f64, _f64, _vp, _vp, _vp, _size, _vp]),
    "gnpde_initial_step_lin_bf16": (_int, [_i64, _vp, _vp, _f64, _f64, _f64, _vp, _vp, _vp, _size, _vp]),
    "gnpde_scaled_sq_sums_f32": (_int, [_i64, _vp, _vp, _vp, _f64, _f64, _vp, _vp, _size, _vp]),
    "gnpde_segment_sums_workspace_bytes": (_size, [_i64]),
    "gnpde_segment_sums_f64": (_int, [_i64, _i64, _vp, _vp, _vp, _size, _vp]),
    "gnpde_compact_items_f32": (_int, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gnpde_initial_step_bf16": (_int, [_i64, _vp, _vp, _vp, _f64, _f64, _f64, _vp, _vp, _vp, _size, _vp]),
    "gnpde_stage_apply_f32": (_int, [_i64, _i64, _i64, _vp, _vp, ctypes.POINTER(StageEpilogue), _vp]),
    "gnpde_stage_apply_bf16": (_int, [_i64, _i64, _i64, _vp, _vp, ctypes.POINTER(StageEpilogue), _vp]),
    "gnpde_seg_long_edges": (_int, []),
    "gnpde_seg_long_pass_edges": (_int, [_i64]),
    "gnpde_linear_f32": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "gnpde_linear_bf16": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "gnpde_linear_wgrad_workspace_bytes": (_size, [_i64, _i64, _i64]),
    "gnpde_linear_wgrad_f32": (_int, [_vp, _i64, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _vp, _size, _vp]),
    "gnpde_keysum_workspace_bytes": (_size, [_i64, _i64, _i64, _i64]),
    "gnpde_ref_scores_f32": (_int, [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp,
                                    _size, _vp]),
    "gnpde_ref_keysum_f32": (_int, [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i64, _vp, _vp, _size, _vp]),
    "gnpde_ref_scores_from_keysum_f32": (_int, [_vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i64, _i64, _vp, _vp,
                                                _size, _vp]),
    "gnpde_softmax_stats_f32": (_int, [_vp, _i64, _vp, _i64, _vp, _int, _int, _i64, _i64, _vp, _vp, _vp, _i64, _f32,
                                       _f32, _vp, _vp, _vp, _vp, _vp]),
    "gnpde_attn_weights_f32": (_int, [_vp, _vp, _i64, _int, _int, _i64, _i64, _vp, _vp, _vp, _i64, _f32, _f32, _vp,
                                      _vp, _vp, _vp]),
    "gnpde_edge_attention_f32": (_int, [_vp, _vp, _vp, _i64, _int, _int, _i64, _i64, _vp, _vp, _vp, _i64, _f32, _f32,
                                        _vp, _vp, _vp, _vp]),
    "gnpde_seg_block_edges": (_int, [_int, _i64, _i64]),
    "gnpde_seg_plan_build": (_int, [_vp, _i64, ctypes.c_int32, _vp, _i64, _vp, _i64, _vp, _i64, c_i64p, c_i64p,
                                    c_i64p]),
    "gnpde_seg_softmax_f32": (_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _int, _int, _int, _i64,
                                     _i64,
                                     _vp, _vp, _vp, _i64, _f32, _f32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gnpde_csr_rowidx": (_int, [_vp, _i64, _i64, _vp, _vp]),
    "gnpde_sddmm_f32": (_int, [_vp, _vp, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _int, _int, _vp, _vp]),
    "gnpde_softmax_backward_f32": (_int, [_vp, _vp, _i64, _i64, _int, _vp, _vp, _vp, _vp]),
    "gnpde_segment_sum_f64": (_int, [_vp, _vp, _i64, _i64, _int, _vp, _vp, _vp]),
    "gnpde_wcolsum_workspace_bytes": (_size, [_i64, _i64, _i64, _int]),
    "gnpde_wcolsum_f64": (_int, [_vp, _i64, _i64, _i64, _i64, _vp, _int, _vp, _vp, _size, _vp]),
    "gnpde_score_input_grad_f32": (_int, [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _int, _vp, _i64, _int, _vp]),
    "gnpde_gather_head_f32": (_int, [_vp, _i64, _int, _int, _vp, _f32, _vp, _vp]),
    "gnpde_rk_combine_f32": (_int, [_i64, _vp, _int, ctypes.POINTER(_vp), ctypes.POINTER(_f64), _f64, _vp, _vp]),
    "gnpde_dot_workspace_bytes": (_size, []),
    "gnpde_dot_f64": (_int, [_i64, _vp, _vp, _vp, _vp, _size, _vp]),
    "gnpde_sum_f64": (_int, [_i64, _vp, _vp, _int, _vp, _size, _vp]),
    "gnpde_self_loops_workspace_bytes": (_size, [_i64, _i64, _i64]),
    "gnpde_self_loops_count": (_int, [_vp, _i64, _i64, c_i64p, _vp, _size, _vp]),
    "gnpde_add_self_loops": (_int, [_vp, _vp, _i64, _i64, _i64, _f32, _i64, _vp, _vp, _vp, _size, _vp]),
    "gnpde_norm_weights_f32": (_int, [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _int, _vp, _vp, _vp]),
    "gnpde_score_grad_f32": (_int, [_vp, _vp, _vp, _i64, _i64, _int, _int, _i64, _i64, _vp, _vp, _i64, _f32, _f32, _vp,
                                    _vp, _i64, _vp, _vp]),
}

# constants mirrored from include/gnpde.h
ABI_VERSION = 8
OK = 0
EINVAL = -1
EHIP = -2
EUNSUPPORTED = -3
EPI_PLAIN = 0
EPI_RHS = 1
ALPHA_SIGMOID = 2
ADD_SOURCE = 4
SCORE_REFERENCE = 0
SCORE_DOT = 1
SCORE_EXP_KERNEL = 2
SCORE_COSINE = 3
SCORE_PEARSON = 4
SCORE_UNIFORM = 5
NORM_RW_ROW = 0
NORM_RW_COL = 1
NORM_GCN = 2

_lock = threading.Lock()
_lib = None


class GnpdeError(RuntimeError):
    pass


def build_id():
    """Source hash compiled into the loaded library (gnpde_build_id)."""
    return load().gnpde_build_id().decode()


def source_hash():
    """Hash of the csrc/ sources and include/gnpde.h of this tree (srchash.py)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gnpde_srchash", os.path.join(os.path.dirname(_HERE), "srchash.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.source_hash()


def load():
    """Load libgnpde.so once; raise GnpdeError (no fallback) if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise GnpdeError(
                "libgnpde.so not found at %s: build it with `make -C graph-neural-pde_amd` or "
                "`python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        ver = lib.gnpde_abi_version()
        if ver != ABI_VERSION:
            raise GnpdeError("libgnpde ABI version %d != expected %d" % (ver, ABI_VERSION))
        _check_fresh(lib)
        _lib = lib
        return lib


def _check_fresh(lib):
    """An in-tree library built from other sources than this tree's csrc/ (a
    stale build with another argument list would shift every argument) is
    refused; GNPDE_ALLOW_STALE=1 downgrades it to a warning."""
    if "GNPDE_LIB" in os.environ:
        return  # an explicitly chosen library: the caller vouches for it
    try:
        src = source_hash()
    except OSError:
        return  # no sources next to the library (an installed copy): nothing to compare
    built = lib.gnpde_build_id().decode()
    if built != src:
        msg = ("libgnpde.so at %s was built from sources %s, this tree's csrc/ hash to %s: rebuild it "
               "(make -C graph-neural-pde_amd)" % (LIB_PATH, built, src))
        if os.environ.get("GNPDE_ALLOW_STALE") == "1":
            import warnings
            warnings.warn(msg)
        else:
            raise GnpdeError(msg)


def call(name, *args):
    """Invoke an entry point; raise GnpdeError with gnpde_last_error() on failure."""
    return check(call_rc(name, *args), name)


def call_rc(name, *args):
    """Invoke an entry point and return its status code (for callers that
    handle GNPDE_EUNSUPPORTED by choosing another device path)."""
    return getattr(load(), name)(*args)


def check(rc, name):
    if rc != 0:
        msg = load().gnpde_last_error().decode(errors="replace")
        raise GnpdeError("%s failed (rc=%d): %s" % (name, rc, msg))
    return rc


def fn(name):
    return getattr(load(), name)
