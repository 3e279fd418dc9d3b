"""The C-ABI library loads and exports every entry point include/*.h declares (CPU only: no compute)."""
import ctypes
import os
import re
import subprocess

from mythril_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in ("mgp.h", "mgp_ir.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(mgp_[a-z0-9_]+)\s*\(", src))
    return names


def test_header_declares_the_binding_surface():
    names = _declared()
    assert set(N.EXPORTED_SYMBOLS) == names, names ^ set(N.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = N.lib()
    for name in _declared():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (mgp_[a-z0-9_]+)\b", out))
    assert _declared() <= exported, _declared() - exported


def test_symbols_are_plain_c_abi():
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True).stdout
    for name in _declared():
        assert re.search(rf"\bT {name}$", out, re.M), f"{name} is mangled or missing"


def test_version_and_error_string_without_gpu():
    lib = N.lib()
    assert b"gfx950" in lib.mgp_version()
    assert isinstance(lib.mgp_last_error(None), bytes)
    # NULL-argument guards return MGP_E_ARG instead of crashing
    assert lib.mgp_create(0, None) == N.MGP_E_ARG
    assert lib.mgp_eval_batch(None, None, None, 0, None, 0, 0, None, None) == N.MGP_E_ARG
    assert lib.mgp_keccak256_batch(None, None, 0, 0, 0, None) == N.MGP_E_ARG


def test_lowering_capacity_error_reports_size():
    import numpy as np

    from ._util import pack_states

    nodes, noff, consts, coff = pack_states([([[1, 256, -1, -1, -1, 0, 0], [1, 256, -1, -1, -1, 1, 0],
                                               [41, 1, 0, 1, -1, 0, 0]], [])])
    used = ctypes.c_uint64(0)
    po = np.zeros(2, np.uint64)
    st = np.zeros(1, np.uint8)
    out = np.zeros(2, np.uint32)
    rc = N.lib().mgp_lower(N._ptr(nodes), N._ptr(noff), 1, N._ptr(np.zeros(8, np.uint32)), N._ptr(coff), 0,
                           N._ptr(out), 2, N._ptr(po), N._ptr(st), ctypes.byref(used))
    assert rc == N.MGP_E_CAPACITY and used.value > 2


def test_product_has_no_oracle_dependency():
    """The shipped package must never import the checker."""
    pkg = os.path.join(ROOT, "mythril_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(dirpath, f)).read()
                assert "from oracle" not in src and "import oracle" not in src, f
                assert "liboracle" not in src, f


def test_program_cache_warm_lowers_each_distinct_program_once():
    """mgp_program_cache_warm (host only) puts one program per distinct GPU node list in the
    cache that mgp_check_batch reads; a second warm of the same batch adds none."""
    import corpus
    from mythril_amd import _native as N
    from mythril_amd import front as F

    cs = [c[1] for c in corpus.corpus(48)]
    B = F.Batch(cs + cs[:5])
    n, no, c, co = B.packed(gpu=True)
    distinct = {bytes(n[no[i]:no[i + 1]].tobytes()) + bytes(c[co[i]:co[i + 1]].tobytes()) for i in range(len(no) - 1)}
    N.program_cache_clear()
    N.program_cache_warm(B._h)
    N.program_cache_warm(B._h)
    assert N.program_cache_clear() == len(distinct)
    B.close()
