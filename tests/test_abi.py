"""CPU: libgsr.so (the C ABI) loads and exports every function include/gsr.h declares.

Only argument-validation paths are called here (they return before any HIP call), so no
GPU is needed; compute calls are exercised by the -m gpu tests.
"""
import ctypes
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gsr.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gsr[0-9a-z_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    names = _declared()
    for n in ["gsr3d_project_fwd", "gsr2d_project_fwd", "gsr_bin_offsets", "gsr_bin_sort",
              "gsr3d_raster_fwd", "gsr3d_raster_bwd", "gsr2d_raster_fwd", "gsr2d_raster_bwd",
              "gsr3d_project_bwd", "gsr2d_project_bwd", "gsr_last_error", "gsr_version"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    from gsr import _lib
    lib = _lib.lib()
    for name in _declared():
        assert hasattr(lib, name), f"{name} missing from {_lib.LIB_PATH}"
    assert set(_declared()) == set(_lib.EXPORTS), "ctypes prototypes out of sync with gsr.h"
    assert lib.gsr_version() >= 1
    assert lib.gsr_abi_version() == _lib.ABI_VERSION


def test_abi_version_matches_header():
    from gsr import _lib
    src = open(HEADER).read()
    assert re.search(r"#define GSR_ABI_VERSION (\d+)", src).group(1) == str(_lib.ABI_VERSION)


def test_overflow_bits_match_header():
    from gsr import _lib
    src = open(HEADER).read()
    bits = {int(v): k for k, v in re.findall(r"#define (GSR_OVF_\w+) (\d+)", src)}
    assert set(bits) == set(_lib.OVF_BITS), (bits, _lib.OVF_BITS)


def test_bin_offsets_rejects_bad_caps():
    from gsr import _lib
    lib = _lib.lib()
    caps = _lib.BinCaps(-5, 0, None)
    rc = lib.gsr_bin_offsets(None, 100, None, None, None, None, None, ctypes.byref(caps), None, None)
    assert rc == -1 and b"bad caps" in lib.gsr_last_error()


def test_invalid_arguments_are_reported_not_launched():
    from gsr import _lib
    lib = _lib.lib()
    rc = lib.gsr3d_project_fwd(None, 10, 14, None, None, 0, 64, 64, 0.01, 1e10, 0.0, 0.3, 0, 0, 0, -1,
                               None, None, None, None, None, None, 0, None)
    assert rc == -1 and b"bad N" in lib.gsr_last_error()
    rc = lib.gsr3d_project_fwd(None, 10, 14, None, None, 1, 64, 64, 0.01, 1e10, 0.0, 0.3, 7, 0, 0, -1,
                               None, None, None, None, None, None, 0, None)
    assert rc == -1 and b"radius_mode" in lib.gsr_last_error()
    rc = lib.gsr3d_project_fwd(None, 10, 14, None, None, 1, 64, 64, 0.01, 1e10, 0.0, 0.3, 0, 0, 2, 1,
                               None, None, None, None, None, None, 0, None)
    assert rc == -1 and b"bad band" in lib.gsr_last_error()
    rc = lib.gsr3d_project_fwd(None, 10, 14, None, None, 1, 64, 64, 0.01, 1e10, 0.0, 0.3, 7, 0, 0, -1,
                               None, None, None, None, None, None, 0, None)
    assert rc == -1 and b"radius_mode" in lib.gsr_last_error()
    rc = lib.gsr2d_project_fwd(None, 10, 9, 0, None, 1, 1, 64, 64, 2.0, None, None, None, None, None, 0, None)
    assert rc == -1 and b"eps_cut" in lib.gsr_last_error()
    rc = lib.gsr2d_project_fwd(None, 10, 9, 90, None, 2, 4, 64, 64, 1e-8, None, None, None, None, None, 0, None)
    assert rc == -1 and b"need set_begin" in lib.gsr_last_error()
    rc = lib.gsr2d_project_bwd(None, 10, 9, 0, None, 1, 0, 64, 64, None, None, None, None, None, None, None, None)
    assert rc == -1 and b"bad C" in lib.gsr_last_error()
    rc = lib.gsr_bin_sort(None, None, None, None, None, None, None, 1, 10, 64, 64, 5, 0, 0, 0, 0, 0, 0, None, None, 0, None,
                          None, None)
    assert rc == -1 and b"bad order" in lib.gsr_last_error()
    with pytest.raises(ValueError, match="bad order"):
        _lib.check(rc, "gsr_bin_sort")


def test_layout_switches_validate():
    """The process-wide layout switches accept their documented values only (include/gsr.h:
    gsr_set_fwd_lanes 0/1/4/16, gsr_set_bwd_layout 0/1/2) and leave the setting unchanged on a
    bad value; no GPU call is made."""
    from gsr import _lib
    lib = _lib.lib()
    for v in (0, 1, 2):
        assert lib.gsr_set_bwd_layout(v) == 0
    for v in (-1, 3, 16):
        assert lib.gsr_set_bwd_layout(v) == -1 and b"gsr_set_bwd_layout" in lib.gsr_last_error()
    for v in (0, 1, 4, 16):
        assert lib.gsr_set_fwd_lanes(v) == 0
    for v in (2, 8, -4):
        assert lib.gsr_set_fwd_lanes(v) == -1 and b"gsr_set_fwd_lanes" in lib.gsr_last_error()
    for v in (0, 6, 12, 30):   # gsr_set_fwd_heavy: 0 (off) or a log2 list length in 6..30
        assert lib.gsr_set_fwd_heavy(v) == 0
    for v in (-1, 1, 5, 31):
        assert lib.gsr_set_fwd_heavy(v) == -1 and b"gsr_set_fwd_heavy" in lib.gsr_last_error()
    assert lib.gsr_set_fwd_heavy(0) == 0
    assert lib.gsr_set_bwd_layout(0) == 0 and lib.gsr_set_fwd_lanes(0) == 0


def test_workspace_queries():
    from gsr import _lib
    lib = _lib.lib()
    assert lib.gsr_bin_sort_workspace(1000, 132) >= 16 * 1000


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    from gsr import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.GsrLibraryError):
        _lib.lib()


def test_binding_prototypes_match_header():
    """Every ctypes prototype in gsr/_lib.py has the header's parameter count."""
    import re
    from gsr import _lib
    hdr = open(os.path.join(ROOT, "include", "gsr.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    decls = dict(re.findall(r"\b(gsr\w+)\s*\(([^;{]*?)\)\s*;", hdr, flags=re.S))
    assert set(_lib.EXPORTS) <= set(decls), set(_lib.EXPORTS) - set(decls)
    for name, (_, args) in _lib.EXPORTS.items():
        params = decls[name].strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        assert n == len(args), (name, n, len(args))


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors of gsr_bin_stats / gsr_loss_terms have the C compiler's size and offsets."""
    import shutil
    import subprocess
    from gsr import _lib
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    src = tmp_path / "layout.c"
    structs = {"gsr_bin_stats": _lib.BinStats, "gsr_bin_caps": _lib.BinCaps, "gsr_loss_terms": _lib.LossTerms}
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "gsr.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines += ["return 0;", "}"]
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run([cc, "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], check=True, capture_output=True,
                                                         text=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got[f"{cname} size"]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got[f"{cname} {f}"]) == getattr(py, f).offset, (cname, f)


def test_loss_entry_points_validate():
    from gsr import _lib
    lib = _lib.lib()
    assert lib.gsr_loss_workspace(6, 576, 512) >= 6 * 16
    rc = lib.gsr_loss_iou_l1_fwd(None, None, None, None, 0, 64, 64, 1.0, None, 0, None, None, None, None)
    assert rc == -1 and b"bad C" in lib.gsr_last_error()
    rc = lib.gsr3d_raster_bwd_loss(*([None] * 8), 1, 0, 1, 64, 64, None, None, None, None, None, None, None, None)
    assert rc == -1 and b"loss terms" in lib.gsr_last_error()
