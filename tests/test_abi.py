"""The C-ABI library loads, exports every symbol include/gnpde.h declares, and
rejects bad arguments with an error code + message before touching the GPU
(these calls validate on the host, so they run without a device)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

import gnpde
from gnpde import _lib

HEADER = os.path.join(ROOT, "include", "gnpde.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gnpde_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_entry_points():
    syms = declared_symbols()
    for must in ("gnpde_csr_build", "gnpde_spmm_rhs_f32", "gnpde_attn_weights_f32", "gnpde_softmax_stats_f32",
                 "gnpde_linear_f32", "gnpde_ref_scores_f32", "gnpde_rk_combine_f32", "gnpde_last_error"):
        assert must in syms


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_every_declared_symbol():
    assert sorted(_lib.SIGNATURES) == declared_symbols()


def test_library_built_from_these_sources():
    """The in-tree libgnpde.so carries the hash of the csrc/ sources it was built
    from (gnpde_build_id); it must be this tree's."""
    info = gnpde.build_info()
    assert info["fresh"], info


def test_abi_version():
    assert _lib.load().gnpde_abi_version() == _lib.ABI_VERSION == 8


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_errors_are_reported_not_raised():
    lib = _lib.load()
    vp = ctypes.c_void_p
    # C = 0 -> EINVAL before any launch
    rc = lib.gnpde_spmm_rhs_f32(vp(0), 0, vp(0), 0, vp(0), vp(0), 0, vp(0), 0, vp(0), 0, vp(0), vp(0), 0, vp(0), 0,
                                vp(0), 0, None, vp(0))
    assert rc == -1
    assert b"C must be" in lib.gnpde_last_error()
    st = _lib.StageEpilogue()
    st.n_out = 3
    rc = lib.gnpde_spmm_rhs_f32(vp(0), 0, vp(0), 0, vp(0), vp(0), 4, vp(16), 4, vp(0), 0, vp(0), vp(0), 0, vp(0), 4,
                                vp(0), 0, ctypes.byref(st), vp(0))
    assert rc == -1 and b"n_out" in lib.gnpde_last_error()
    # the hub partials' 32-bit offsets are checked at the ABI (n_slots is an argument):
    # 2^22 slots x 256 columns x 4 B = 4 GiB -> unsupported; a partials buffer without its slot count -> invalid
    rc = lib.gnpde_spmm_rhs_f32(vp(0), 0, vp(0), 1, vp(0), vp(0), 256, vp(16), 256, vp(0), 0, vp(0), vp(0), 0, vp(64),
                                256, vp(4096), 1 << 22, None, vp(0))
    assert rc == -3 and b"32-bit buffer offsets" in lib.gnpde_last_error()
    rc = lib.gnpde_spmm_rhs_f32(vp(0), 0, vp(0), 1, vp(0), vp(0), 256, vp(16), 256, vp(0), 0, vp(0), vp(0), 0, vp(64),
                                256, vp(4096), 0, None, vp(0))
    assert rc == -1 and b"slot count" in lib.gnpde_last_error()
    rc = lib.gnpde_attn_ref_rhs_f32(vp(0), 0, vp(0), 1, vp(0), vp(0), vp(0), vp(0), vp(0), 2, 256, vp(16), 256, vp(0),
                                    0, vp(0), vp(0), 0, vp(64), 256, vp(4096), 1 << 22, None, vp(0))
    assert rc == -3 and b"32-bit buffer offsets" in lib.gnpde_last_error()
    # the solve entry copy: 16-byte rows only, no aliasing
    rc = lib.gnpde_rows_copy(vp(16), 4, 20, vp(0), vp(64), vp(0), vp(0))
    assert rc == -3 and b"16-byte" in lib.gnpde_last_error()
    rc = lib.gnpde_rows_copy(vp(16), 4, 32, vp(0), vp(16), vp(0), vp(0))
    assert rc == -1 and b"alias" in lib.gnpde_last_error()
    assert lib.gnpde_rows_copy(vp(16), 0, 32, vp(0), vp(64), vp(128), vp(0)) == 0
    # a well-formed stage struct passes validation (no items -> nothing launched):
    # catches a library built against a stale header layout
    st = _lib.StageEpilogue()
    st.n_out = 1
    st.o[0].out, st.o[0].cb, st.o[0].cf = 4096, 1.0, 0.5
    st.nk, st.k[0], st.o[0].c[0] = 1, 8192, 2.0
    rc = lib.gnpde_spmm_rhs_f32(vp(0), 0, vp(0), 0, vp(0), vp(0), 4, vp(16), 4, vp(0), 0, vp(32), vp(0), 1, vp(0), 4,
                                vp(0), 0, ctypes.byref(st), vp(0))
    assert rc == 0, lib.gnpde_last_error()
    # the wide (adaptive) epilogue: error rows need err_y0 and an output or x for y1
    st.err_rows, st.err_y1, st.atol, st.rtol = 16384, -1, 1e-7, 1e-9
    rc = lib.gnpde_spmm_rhs_f32(vp(0), 0, vp(0), 0, vp(0), vp(0), 4, vp(16), 4, vp(0), 0, vp(32), vp(0), 1, vp(0), 4,
                                vp(0), 0, ctypes.byref(st), vp(0))
    assert rc == -1 and b"err_y0" in lib.gnpde_last_error()
    st.err_y0 = 32768
    st.err_y1 = 1
    rc = lib.gnpde_stage_apply_f32(0, 4, 4, vp(0), vp(0), ctypes.byref(st), vp(0))
    assert rc == -1 and b"err_y1" in lib.gnpde_last_error()
    st.err_y1 = 0
    assert lib.gnpde_stage_apply_f32(0, 4, 4, vp(0), vp(0), ctypes.byref(st), vp(0)) == 0
    st.nk = 7
    rc = lib.gnpde_stage_apply_bf16(0, 4, 4, vp(0), vp(0), ctypes.byref(st), vp(0))
    assert rc == -1 and b"nk=7" in lib.gnpde_last_error()
    rc = lib.gnpde_linear_f32(vp(0), 10, 4, 4, vp(0), vp(0), 8, 8, vp(0), 8, vp(0), 0, vp(0))
    assert rc == -1 and b"NULL" in lib.gnpde_last_error()
    rc = lib.gnpde_csr_build(vp(0), 1, 10, 5, 2, vp(0), vp(0), vp(0), vp(0), 0, vp(0))
    assert rc == -1 and b"key_row" in lib.gnpde_last_error()
    rc = lib.gnpde_softmax_stats_f32(vp(0), 0, vp(0), 0, vp(0), 0, 0, 17, 1, vp(0), vp(0), vp(0), 1,
                                     ctypes.c_float(1), ctypes.c_float(1), vp(0), vp(0), vp(0), vp(0), vp(0))
    assert rc == -3 and b"heads" in lib.gnpde_last_error()
    rc = lib.gnpde_rk_combine_f32(16, vp(0), 9, None, None, ctypes.c_double(1.0), vp(1), vp(0))
    assert rc == -3


def test_python_wrapper_raises_with_message():
    with pytest.raises(_lib.GnpdeError, match="rc=-1"):
        _lib.call("gnpde_linear_f32", ctypes.c_void_p(0), 10, 4, 4, ctypes.c_void_p(0), ctypes.c_void_p(0), 8, 8,
                  ctypes.c_void_p(0), 8, ctypes.c_void_p(0), 0, ctypes.c_void_p(0))


def test_stage_struct_layout_matches_header():
    # gnpde_stage_out_t (ABI 3): out, base (8 B each), cb, cf (4 B each), c[6] -> 48 B
    assert ctypes.sizeof(_lib.StageOut) == 8 + 8 + 4 + 4 + 4 * 6
    assert _lib.StageOut.c.offset == 24
    # gnpde_stage_epilogue_t: f_out, n_out (padded to 8), o[2], nk (padded to 8), k[6], out_rows, dot_with,
    # dot_rows, dot_coef, dot_accumulate (padded to 8), err_rows, err, err_y0, err_y1 (padded), atol, rtol
    so = ctypes.sizeof(_lib.StageOut)
    assert _lib.StageEpilogue.nk.offset == 16 + 2 * so
    assert _lib.StageEpilogue.out_rows.offset == 16 + 2 * so + 8 + 48
    assert _lib.StageEpilogue.dot_coef.offset == _lib.StageEpilogue.out_rows.offset + 24
    assert _lib.StageEpilogue.err.offset == _lib.StageEpilogue.dot_coef.offset + 24
    # ... err_y0, err_y1 (padded), atol, rtol, coef_scale, f_lin, unscaled_outs
    assert _lib.StageEpilogue.dense_out.offset == _lib.StageEpilogue.err.offset + so + 8 + 8 + 8 + 8 + 8 + 8
    assert _lib.StageEpilogue.coef_scale.offset == _lib.StageEpilogue.rtol.offset + 8
    assert _lib.StageEpilogue.f_lin.offset == _lib.StageEpilogue.coef_scale.offset + 8
    # unscaled_outs (ABI 6) fills f_lin's padding
    assert _lib.StageEpilogue.unscaled_outs.offset == _lib.StageEpilogue.f_lin.offset + 4
    # ABI 8: dense_out, dense_rows, dense_t, dense_dt, dense_tab, dense_m[5][8] floats
    assert _lib.StageEpilogue.dense_m.offset == _lib.StageEpilogue.dense_out.offset + 5 * 8
    assert _lib.StageEpilogue.scale_rows.offset == _lib.StageEpilogue.dense_m.offset + 5 * 8 * 4
    assert ctypes.sizeof(_lib.StageEpilogue) == _lib.StageEpilogue.scale_rows.offset + 8


def test_workspace_size_queries():
    lib = _lib.load()
    assert lib.gnpde_csr_workspace_bytes(1, 1000, 100) >= 3 * 4000
    assert lib.gnpde_plan_workspace_bytes(100) >= 6 * 404
    assert lib.gnpde_keysum_workspace_bytes(2, 1000, 64, 32) > 0


def test_package_exposes_library_path():
    assert gnpde.native_library_path().endswith("libgnpde.so")


def test_c_header_struct_layout_with_gcc(tmp_path):
    """The ctypes mirror of gnpde_stage_epilogue_t matches what a C compiler lays out."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "gnpde.h"\nint main(void){'
                   'printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(gnpde_stage_out_t),'
                   'offsetof(gnpde_stage_out_t, c), sizeof(gnpde_stage_epilogue_t), offsetof(gnpde_stage_epilogue_t, nk),'
                   'offsetof(gnpde_stage_epilogue_t, k), offsetof(gnpde_stage_epilogue_t, out_rows),'
                   'offsetof(gnpde_stage_epilogue_t, dot_coef), offsetof(gnpde_stage_epilogue_t, dot_accumulate),'
                   'offsetof(gnpde_stage_epilogue_t, err), offsetof(gnpde_stage_epilogue_t, err_y1),'
                   'offsetof(gnpde_stage_epilogue_t, rtol), offsetof(gnpde_stage_epilogue_t, coef_scale),'
                   'offsetof(gnpde_stage_epilogue_t, unscaled_outs));'
                   'printf("%zu %zu %zu %zu\\n", offsetof(gnpde_stage_epilogue_t, dense_out),'
                   'offsetof(gnpde_stage_epilogue_t, dense_tab), offsetof(gnpde_stage_epilogue_t, dense_m),'
                   'offsetof(gnpde_stage_epilogue_t, scale_rows));return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    E = _lib.StageEpilogue
    assert got == [ctypes.sizeof(_lib.StageOut), _lib.StageOut.c.offset, ctypes.sizeof(E), E.nk.offset, E.k.offset,
                   E.out_rows.offset, E.dot_coef.offset, E.dot_accumulate.offset, E.err.offset, E.err_y1.offset,
                   E.rtol.offset, E.coef_scale.offset, E.unscaled_outs.offset, E.dense_out.offset, E.dense_tab.offset,
                   E.dense_m.offset, E.scale_rows.offset]


def test_stale_library_is_refused(monkeypatch):
    """a library built from other sources than this tree (another
    argument list would shift every argument) is refused at load time, not
    only reported by smoke()."""
    lib = _lib.load()
    monkeypatch.setattr(_lib, "source_hash", lambda: "0000000000000000")
    monkeypatch.delenv("GNPDE_LIB", raising=False)
    monkeypatch.delenv("GNPDE_ALLOW_STALE", raising=False)
    with pytest.raises(_lib.GnpdeError, match="rebuild"):
        _lib._check_fresh(lib)
    monkeypatch.setenv("GNPDE_ALLOW_STALE", "1")
    with pytest.warns(UserWarning):
        _lib._check_fresh(lib)
