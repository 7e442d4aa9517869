"""C-ABI boundary checks that need no GPU: libsift_mi.so loads, exports every
symbol include/sift_mi.h declares, and argument validation fails cleanly."""
import ctypes
import os
import re
import subprocess

import pytest
from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "sift_mi.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(sift_mi_[a-z_]+)\s*\(", txt)))


def test_header_matches_binding(pkg):
    from sift_features_amd import _lib
    assert declared_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_all_symbols(pkg):
    L = pkg.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", L._name], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (sift_mi_\w+)", out))
    assert set(declared_symbols()) <= exported


def test_library_is_gfx950_code_object(pkg, tmp_path):
    """The fat binary carries a gfx950 code object (and nothing else)."""
    L = pkg.lib()
    fb = tmp_path / "fatbin.bin"
    subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", L._name,
                    str(tmp_path / "stripped.so")], check=True)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          f"--input={fb}"], capture_output=True, text=True, check=True).stdout.split()
    dev = [t for t in out if not t.startswith("host-")]
    assert dev == ["hipv4-amdgcn-amd-amdhsa--gfx950"], out


def test_version_and_errors_without_device(pkg):
    L = pkg.lib()
    assert b"gfx950" in L.sift_mi_version()
    # null out-pointer is rejected before any device call
    assert L.sift_mi_create(0, 0, None) == -1
    assert b"null" in L.sift_mi_last_error()
    # null contexts are rejected
    assert L.sift_mi_set_chunk(None, 4) == -1
    assert L.sift_mi_fetch(None, None, None, 0) == -1
    assert L.sift_mi_reset_stats(None) == -1
    assert L.sift_mi_set_path_option(None, 0, 1) == -1


def test_library_reads_no_environment(pkg):
    """Path switches are per context (sift_mi_set_path_option): no product
    source reads the environment (no process-global knobs).
    (The binary's one getenv import comes from rocPRIM's headers in
    order.hip's radix sort, not from this code.)"""
    src = os.path.join(ROOT, "sift-features_amd", "csrc")
    for fn in sorted(os.listdir(src)):
        if fn.endswith((".hip", ".cpp", ".h")):
            txt = open(os.path.join(src, fn)).read()
            assert not re.search(r"\bgetenv\s*\(", txt), fn


def test_no_cpu_fallback_in_product(pkg):
    """The product package never imports the oracle or numpy-side SIFT code."""
    pkgdir = os.path.join(ROOT, "sift-features_amd")
    for fn in os.listdir(pkgdir):
        if fn.endswith(".py"):
            src = open(os.path.join(pkgdir, fn)).read()
            assert "oracle" not in src.replace("oracle/", "").lower() or fn == "synth.py", fn
