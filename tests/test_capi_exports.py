"""The C-ABI library loads on a host without a GPU and exports every symbol include/ccmpc.h
declares (no compute calls here)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "ccmpc.h")
LIB = os.path.join(ROOT, "cc-mpc_amd", "ccmpc", "libccmpc.so")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(ccmpc_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_path():
    names = declared_functions()
    for must in ("ccmpc_moments", "ccmpc_minkowski", "ccmpc_affine", "ccmpc_ideal_rollout",
                 "ccmpc_ideal_moments"):
        assert must in names


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB):
        pytest.fail("libccmpc.so missing: run __graft_entry__.build() / make -C cc-mpc_amd/csrc")
    lib = ctypes.CDLL(LIB)
    for name in declared_functions():
        assert hasattr(lib, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (ccmpc_\w+)", nm))
    assert exported == set(declared_functions())


def test_ctypes_binding_covers_header_and_abi():
    from ccmpc import _lib
    assert set(_lib.SIGNATURES) == set(declared_functions())
    lib = _lib.load()                       # host-only calls below; no device work
    assert lib.ccmpc_abi_version() == _lib.ABI_VERSION
    assert lib.ccmpc_status_string(-11) == b"no real tangent (n^T Sigma n <= 0)"
    assert lib.ccmpc_moments_workspace_bytes(8, 4, 20000) > 0
    assert lib.ccmpc_moments_workspace_bytes(41, 4, 20000) == 0        # T > 40 rejected


def test_record_layouts_are_128_bytes():
    from ccmpc import _lib
    assert _lib.HALFSPACE_DTYPE.itemsize == 128
    assert _lib.AFFINE_DTYPE.itemsize == 128
    assert _lib.HALFSPACE_DTYPE.names[-4:] == ("which", "side", "status", "t_tau")


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "cc-mpc_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, flags=re.M), f


def test_cycle_args_struct_matches_the_header():
    """ccmpc._lib.CycleArgs mirrors ccmpc_cycle_args: the same size as the library's, and the
    fields in the header's order (no GPU call: the size query is host code)."""
    import ctypes
    import re
    from ccmpc import _lib
    lib = _lib.load()
    assert lib.ccmpc_cycle_args_size() == ctypes.sizeof(_lib.CycleArgs)
    hdr = open(os.path.join(ROOT, "include", "ccmpc.h")).read()
    body = hdr[hdr.index("typedef struct ccmpc_cycle_args {"):hdr.index("} ccmpc_cycle_args;")]
    names = [n for decl in body.split("{", 1)[1].split(";") if decl.strip()
             for n in re.findall(r"\*?\s*(\w+)\s*(?:,|$)", decl.strip())]
    assert names == [f for f, _ in _lib.CycleArgs._fields_]
