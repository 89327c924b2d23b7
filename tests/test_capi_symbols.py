"""The C-ABI library loads (no GPU needed) and exports exactly what include/fo_hip.h declares;
the ctypes table in fo/_lib.py matches the header's argument counts."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "fo_hip.h")
LIB = os.environ.get("FO_LIB_PATH") or os.path.join(ROOT, "freeze-omni_amd", "fo", "libfo_hip.so")


def header_decls():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    decls = {}
    for m in re.finditer(r"(?:int|long long)\s+(fo_\w+)\s*\(([^;]*?)\)\s*;", txt, flags=re.S):
        args = [a for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        decls[m.group(1)] = len(args)
    return decls


def test_header_matches_ctypes_table():
    from fo import _lib
    decls = header_decls()
    assert set(decls) == set(_lib._SIGS), set(decls) ^ set(_lib._SIGS)
    for name, n in decls.items():
        assert len(_lib._SIGS[name][1]) == n, name


@pytest.mark.skipif(not os.path.exists(LIB), reason="libfo_hip.so not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = set(header_decls()) - exported
    assert not missing, missing
    from fo import _lib
    lib = _lib.load()
    assert lib.fo_version() >= 1
    assert lib.fo_attn_nsplit(257, 8, 4) == 5 and lib.fo_attn_nsplit(100, 64, 14) == 1 and lib.fo_attn_nsplit(1, 1, 1) == 1
    assert _lib.load().fo_gemm_pick_split(1, 224, 18944) == 1   # measured: split-K never pays at >= 48 tiles
    assert _lib.load().fo_gemm_pick_split(1, 4, 4096) > 1
