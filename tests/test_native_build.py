"""The HIP kernel library builds for gfx950 and its C ABI matches the ctypes prototypes."""
import glob
import os
import re

from dnn_page_vectors_amd import _build
from dnn_page_vectors_amd.ops._sigs import SIGS


def _codes(args: str) -> str:
    if not args.strip():
        return ""
    out = []
    for a in args.split(","):
        t = a.strip().rsplit(" ", 1)[0]
        out.append("p" if "*" in t else "l" if t == "long" else "u" if "unsigned" in t else "f" if t == "float" else "i")
    return "".join(out)


def test_ctypes_signatures_match_c_declarations():
    src = "".join(open(f).read() for f in glob.glob(os.path.join(_build.CSRC, "kernels", "*.hip")))
    decls = {m.group(1): _codes(m.group(2)) for m in re.finditer(r"PV_API\s+\w+\s+(pv_\w+)\s*\(([^)]*)\)", src)}
    assert decls, "no launchers found"
    for name, codes in decls.items():
        assert name in SIGS, f"{name} missing from ops/_sigs.py"
        assert SIGS[name] == codes, f"{name}: C {codes} vs ctypes {SIGS[name]}"


def test_hip_library_builds_for_gfx950():
    path = _build.build_hip()
    assert os.path.exists(path)
    with open(path, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_debug_kernel_library_builds_with_checks():
    """the PV_CHECK build exists and exports its per-file flag readers."""
    path = _build.build_hip(debug=True)
    with open(path, "rb") as f:
        blob = f.read()
    for unit in ("convfwd", "convbwd", "embed"):
        assert f"pv_debug_{unit}".encode() in blob
    with open(_build.HIP_LIB, "rb") as f:
        assert b"pv_debug_convfwd" not in f.read()  # compiled out of the release library


def test_stale_library_detected(monkeypatch):
    """_native.hip() rebuilds (or, with PAGEVEC_NO_AUTOBUILD=1, refuses) a kernel library whose
    link stamp does not match the tree's sources / headers / flags: any change of an input
    changes the expected stamp."""
    _build.build_hip()
    assert not _build.hip_stale() and _build.hip_stamp()
    monkeypatch.setattr(_build, "HIP_FLAGS", list(_build.HIP_FLAGS) + ["-DPV_STAMP_PROBE=1"])
    assert _build.hip_stale()
