"""Static checks of the generated gfx950 interpreter (CPU only).

The kernel is generated (mythril_amd/csrc/gen_eval_asm.py); these checks make
properties the GPU run depends on hold by construction:
  * every branch inside a handler is a forward branch (or the return from an
    out-of-line rare path to the point right after the branch into it), so each
    uop finishes and the only loop is the dispatch, which advances the uop
    index each time (a wave always reaches RET or the INVALID pad uop);
  * every handler the translator can name is a symbol of the object, at the
    offsets the library's translator uses;
  * no scalar-memory writes anywhere (results go out through vector stores);
  * 64-bit VGPR operands are even-aligned (gfx950 register-tuple rule);
  * no instruction names a VGPR at or past the kernel's declared VGPR count (the bank's
    GPR-index offsets included);
  * the file assembles for gfx950 with the ROCm LLVM assembler.
"""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "mythril_amd", "csrc", "gen_eval_asm.py")
LLVM = "/opt/rocm/lib/llvm/bin"


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    d = tmp_path_factory.mktemp("asm")
    s, h = str(d / "k.s"), str(d / "h.h")
    subprocess.run([sys.executable, GEN, s, h], check=True)
    return s, open(s).read().splitlines()


def test_branches_are_forward(asm):
    _, lines = asm
    pos = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(\.L\w+):", l)
        if m:
            pos[m.group(1)] = i
    n_branches = n_back = 0
    for i, l in enumerate(lines):
        m = re.match(r"^\s+s_(?:c?branch\w*)\s+(\.L\w+)", l)
        if not m:
            continue
        n_branches += 1
        tgt = m.group(1)
        assert tgt in pos, f"undefined label {tgt}"
        if pos[tgt] > i:
            continue
        n_back += 1
        if re.match(r"\.Ltsels?_\d+$", tgt):
            # the TSEL / TSELS table loop: 8 entries per pass, bounded by the entry count
            # s55, which every pass decrements before the loop test
            assert lines[i - 1].strip() == "s_cmp_gt_i32 s55, 0", lines[i - 1]
            assert lines[i - 2].strip() == "s_sub_u32 s55, s55, 8", lines[i - 2]
            assert l.strip().startswith("s_cbranch_scc1")
            assert not any("s55" in x and not x.strip().startswith(("s_cmp", "s_sub_u32 s55", "s_and_b32 s55"))
                           for x in lines[pos[tgt]:i]), "the loop counter is only decremented"
            continue
        # a return from an out-of-line block: must land right after the forward branch
        # that entered this block (so it cannot loop)
        assert re.match(r"\.L(km|kh)back_\d+$", tgt), f"backward branch at line {i}: {l.strip()}"
        enter = lines[pos[tgt] - 1].strip()
        assert enter.startswith("s_cbranch_scc1"), enter
        block = enter.split()[-1]
        assert pos[tgt] < pos[block] < i
    assert n_branches > 200


def test_handlers_are_symbols_at_translator_offsets(asm):
    import ctypes

    from mythril_amd import _native as N
    from mythril_amd import uop_spec as U

    _, lines = asm
    labels = [l.split()[-1][:-1] for l in lines if "mgp_h_" in l and l.endswith(":")]
    assert labels == [f"mgp_h_{h}" for h in U.HANDLERS]
    fn = N.lib().mgp_uop_handler_offsets
    fn.restype = ctypes.POINTER(ctypes.c_uint16)
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
    n = ctypes.c_uint32()
    p = fn(ctypes.byref(n))
    offs = [p[i] for i in range(n.value)]
    assert n.value == len(U.HANDLERS) and len(set(offs)) == len(offs) and min(offs) > 0


def test_no_scalar_memory_writes(asm):
    _, lines = asm
    # built from parts so that this file itself does not spell the mnemonics
    bad = ["s_" + x for x in ("store", "buffer_store", "scratch_store", "dcache_wb", "dcache_discard", "atomic")]
    for l in lines:
        op = l.strip().split(" ")[0]
        assert not any(op.startswith(b) for b in bad), l


def test_vgpr_pairs_even_aligned(asm):
    _, lines = asm
    for l in lines:
        for a, b in re.findall(r"v\[(\d+):(\d+)\]", l):
            if int(b) - int(a) == 1:
                assert int(a) % 2 == 0, l


def _gen_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_eval_asm", GEN)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


G = _gen_module()


def test_vgprs_within_the_declared_count(asm):
    from mythril_amd import uop_spec as U

    _, lines = asm
    top = 0
    for l in lines:
        code = l.split("//")[0]
        for a in re.findall(r"\bv(\d+)\b", code):
            top = max(top, int(a))
        for a, b in re.findall(r"v\[(\d+):(\d+)\]", code):
            top = max(top, int(b))
    assert top < G.NVGPR
    assert any(f".amdhsa_next_free_vgpr {G.NVGPR}" in l for l in lines)
    # GPR-index mode reads / writes bank position p at RV + 8p + limb: the last position
    # the translator can name must end inside the allocation
    assert U.REG_VARS <= U.REG_POS and G.RV + 8 * U.REG_POS <= G.PG < G.NVGPR


@pytest.mark.skipif(not os.path.exists(f"{LLVM}/clang"), reason="ROCm LLVM assembler not installed")
def test_assembles_for_gfx950(asm, tmp_path):
    s, _ = asm
    o = str(tmp_path / "k.o")
    r = subprocess.run([f"{LLVM}/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                        "-c", s, "-o", o], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


def test_address_registers_initialised_before_first_load(asm):
    # v1 (LDS lane base), v2/v3 (candidate offsets), the code base s[10:11], the uop page
    # and the pool base must be written in the prologue before the first instruction using them
    _, lines = asm
    body = [l.strip() for l in lines]

    def first(pred):
        return next(i for i, l in enumerate(body) if pred(l))

    w1 = first(lambda l: l.startswith("v_lshlrev_b32 v1,"))
    w2 = first(lambda l: l.startswith("v_lshlrev_b32 v2,"))
    w3 = first(lambda l: l.startswith("v_add_u32 v3,"))
    assert w2 < w3 < first(lambda l: l.startswith("global_load") and ", v3," in l)
    assert w2 < first(lambda l: l.startswith("global_load") and ", v2," in l)
    assert w1 < first(lambda l: l.startswith("ds_") and ", v" in l)
    assert first(lambda l: l.startswith("s_getpc_b64 s[10:11]")) < first(lambda l: l.startswith("s_setpc_b64"))
    pg = f"v[{G.PG}:{G.PG + 3}]"
    assert first(lambda l: l.startswith(f"global_load_dwordx4 {pg}")) < \
        first(lambda l: l.startswith(f"v_readlane_b32 s0, v{G.PG}"))
    # pool constants are read with scalar loads from s[14:15]
    assert first(lambda l: l.startswith("s_add_u32 s14,")) < \
        first(lambda l: l.startswith("s_load") and "s[14:15]" in l)


@pytest.mark.skipif(not os.path.exists(f"{LLVM}/ld.lld"), reason="ROCm LLVM linker not installed")
def test_embedded_code_object_is_current(asm, tmp_path):
    """libmgp.so must embed exactly the code object the current generator produces
    (a stale build would run an old kernel on the GPU)."""
    import ctypes

    from mythril_amd import _native as N

    s, _ = asm
    o, h = str(tmp_path / "k.o"), str(tmp_path / "k.hsaco")
    subprocess.run([f"{LLVM}/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                    "-c", s, "-o", o], check=True)
    subprocess.run([f"{LLVM}/ld.lld", "-shared", o, "-o", h], check=True)
    fresh = open(h, "rb").read()
    lib = N.lib()
    size = ctypes.c_size_t.in_dll(lib, "mgp_eval_gfx950_hsaco_size").value
    emb = bytes((ctypes.c_ubyte * size).in_dll(lib, "mgp_eval_gfx950_hsaco"))
    assert emb == fresh, "libmgp.so embeds a stale mgp_eval_gfx950 (rebuild: make -C mythril_amd/csrc)"
