"""Reference interpreter of the uop encoding — TEST INFRASTRUCTURE.

Executes the micro-op programs that mgp_lower appends for the gfx950
assembly interpreter (encoding: mythril_amd/uop_spec.py) at the level of the
kernel's registers — vA / vB / vC 256-bit values, Bool slots, LDS slots — so
that the host translator (csrc/mgp_uop.cpp) can be checked on a CPU-only
machine: eval_dag(DAG) == run_uops(lower(DAG)) for every candidate.  The
assembly handlers implement exactly these register-level semantics.
"""
from __future__ import annotations

from typing import Sequence

from mythril_amd import uop_spec as U

from . import bvsem as S

M256 = (1 << 256) - 1
_NAME_BY_OFF = None


def _names():
    """handler entry offset (w0 fields) -> handler name, from the built library."""
    global _NAME_BY_OFF
    if _NAME_BY_OFF is None:
        import ctypes

        from mythril_amd import _native as N

        _NAME_BY_OFF = {}
        # the direct-dispatch entries first: where a handler has one entry, both tables
        # hold the same offset
        for sym in ("mgp_uop_direct_offsets", "mgp_uop_handler_offsets"):
            fn = getattr(N.lib(), sym)
            fn.restype = ctypes.POINTER(ctypes.c_uint16)
            fn.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
            n = ctypes.c_uint32()
            p = fn(ctypes.byref(n))
            assert n.value == len(U.HANDLERS)
            _NAME_BY_OFF.update({p[i]: U.HANDLERS[i] for i in range(n.value)})
    return _NAME_BY_OFF


def _limbs(words, off) -> int:
    return S.limbs_to_int([int(x) for x in words[off:off + 8]])


def _s256(x: int) -> int:
    return x - (1 << 256) if x >> 255 else x


def _sext(x: int, h: int) -> int:
    return ((x ^ h) - h) & M256


def uop_offset(words, off: int) -> int:
    """Word offset of the uop header of the program at `off` (after the v1 bytecode)."""
    n_ins, n_c = int(words[off]), int(words[off + 1])
    v1 = 4 + 4 * n_ins + 8 * n_c
    return off + ((v1 + 3) & ~3) + 4


def _div(op: int, a: int, b: int) -> int:
    if op == U.DIV_VARIANTS["UDIV"]:
        return M256 if b == 0 else a // b
    if op == U.DIV_VARIANTS["UREM"]:
        return a if b == 0 else a % b
    table = {U.DIV_VARIANTS["SDIV"]: S.bvsdiv, U.DIV_VARIANTS["SREM"]: S.bvsrem, U.DIV_VARIANTS["SMOD"]: S.bvsmod}
    return table[op](a, b, 256)


def run_uops(words: Sequence[int], off: int, xs: Sequence[int]):
    """Run the uop program of the state whose v1 program starts at `off`.

    Returns True/False, or None when either header marks the state unsupported.
    """
    if int(words[off + 3]) & 0xFF:
        return None
    u0 = uop_offset(words, off)
    n_uops, status, pool_bytes = int(words[u0]), int(words[u0 + 1]), int(words[u0 + 2])
    if status:
        return None
    pool0 = u0 + pool_bytes // 4

    n_pool = int(words[u0 + 3]) & 0xFF   # bits 8..13: register variables the program reads

    def pool(idx: int) -> int:
        assert idx < n_pool
        return _limbs(words, pool0 + 8 * idx)

    vA = vB = vC = 0
    KM = KH = 0
    lds = {}
    bools = [False] * U.BOOL_SLOTS
    bools[1] = True

    # register bank (uop_spec.REG_POS positions): position p < REG_VARS holds variable p when
    # the program reads it; the other positions hold register slots
    # (preloaded), else it is a register slot written by REGST stores
    var_mask = (int(words[u0 + 3]) >> 8) & 0xFF
    var_rows = int(words[off + 3]) >> 8   # v1 header: one past the highest variable read
    bank = {p: int(xs[p]) & M256 for p in range(U.REG_VARS) if var_mask >> p & 1}

    # the lane's candidate row: variables, then the spill rows VST writes (mgp_ir.h)
    mem = {}

    def load(kind: str, p: int) -> int:
        if kind == "slot":
            return lds[p]
        if kind == "rvar":
            return bank[p // 8]
        if kind == "var":
            if p in mem:
                return mem[p]
            assert p < len(xs), "read of a spill row before its VST"
            return int(xs[p]) & M256
        return pool(p)

    for pc in range(n_uops):
        w0, w1, w2, w3 = (int(words[u0 + 4 + 4 * pc + k]) for k in range(4))
        assert (pc % U.PAGE_UOPS == U.PAGE_UOPS - 1) == (_names()[w0 & 0xFFFF] == "PAGE"), "page layout"
        names = _names()
        first = names[w0 & 0xFFFF]
        op = names[w0 >> 16]
        pa, pb = w1 & 0xFFFF, w1 >> 16
        if first not in U.BOOL_OPS:
            # mask / sign constants named by the uop (the kernel's handlers load them)
            if w2 & U.F_MASK:
                KM = pool((w2 >> 16) & 0x3F)
            if w2 & U.F_SEXT:
                KH = pool(w3 & 0x3F)
        if first.startswith("XR_"):
            vB = bank[pb // 8]          # fused: vA op bank[B]
            first = op = first[3:]
        elif first.startswith("XS_"):
            vB = lds[pb]                # fused: vA op lds[B]
            first = op = first[3:]
        elif first.startswith("XC_"):
            vB = load("const", pb)      # fused: vA op pool[B]
            first = op = first[3:]
        elif first.startswith("XV_"):   # fused: register-only fetch + op
            _, ka, kb, tgt, op = first.split("_", 4)
            first = f"F_{ka}_{kb}_{tgt}"
        if first.startswith("F_"):
            _, ka, kb, tgt = first.split("_")
            if kb != "none":
                vB = vA if kb == "acc" else load(kb, pb)
            if ka != "acc":
                if tgt == "A":
                    vA = load(ka, pa)
                else:
                    vC = load(ka, pa)
        else:
            op = first
        if op in U.EPI_VARIANTS:   # fixed-epilogue variant: same semantics, flags still in w2
            op = op.rsplit("_", 1)[0]
        sb = (w3 >> U.SHIFT_B_POS) & 31
        if op == "PAGE":
            assert pc % U.PAGE_UOPS == U.PAGE_UOPS - 1, "PAGE must end a 64-uop page"
            continue
        if op == "VST":
            assert (w2 & 0xFFFF) >= max(var_rows, 8), "spill row over a variable the program reads"
            mem[w2 & 0xFFFF] = vA
            continue
        if op in U.BOOL_OPS:
            a, b, c = bools[pa >> 1], bools[pb >> 1], bools[(w2 & 0xFFFF) >> 1]
            if op == "RET":
                return a
            if op == "BAND4":  # AND of four Bool slots (w1 lo/hi, w2 lo/hi)
                bools[w3 >> 17] = a and b and c and bools[(w2 >> 16) >> 1]
                continue
            if op.startswith("BAND4N"):  # the same with the operands of mask m negated
                m = int(op[6:])
                ops4 = [a, b, c, bools[(w2 >> 16) >> 1]]   # not `xs`: load() reads the candidates through it
                bools[w3 >> 17] = all(x != bool(m >> i & 1) for i, x in enumerate(ops4))
                continue
            r = {"BAND": a and b, "BOR": a or b, "BXOR": a != b, "BNOT": not a,
                 "BITE": b if a else c, "BEQ": a == b, "BANDN": a and not b}[op]
            bools[w3 >> 17] = r
            continue
        if op.endswith("_RA") or op.endswith("_RC"):
            base = op[:-3]
            X = vA if op.endswith("_RA") else vC
            Y = vB
            if w2 & U.F_SEXT:
                X, Y = _sext(X, KH), _sext(Y, KH)
            if base == "EQ":
                raw = X == Y
            elif base == "ULT":
                raw = X < Y
            elif base == "UGT":
                raw = X > Y
            elif base == "SLT":
                raw = _s256(X) < _s256(Y)
            elif base == "SGT":
                raw = _s256(X) > _s256(Y)
            elif base == "UADDNO256":
                raw = X + Y > M256
            elif base == "UADDNOW":
                raw = X + Y > KM
            elif base == "UMULNO256":
                raw = X * Y > M256
            elif base == "UMULNOW":
                p = X * Y
                raw = (p >> 256) != 0 or (p & M256) > KM
            else:
                raise ValueError(op)
            r = bool(raw) != bool(w2 & U.F_INVERT)
            if w2 & U.F_BCOMB:  # a folded BAND / BOR with Bool slot w3[15:8]/2
                o = bools[((w3 >> U.BCOMB_POS) & 0xFF) >> 1]
                r = (r or o) if w2 & U.F_BCOMB_OR else (r and o)
            bools[w3 >> 17] = r
            continue
        # BV-producing
        if op == "ITE":
            vA = vA if bools[w3 >> 17] else vB
        elif op.startswith("EQSEL_"):   # select-chain step: vA = (vC == vB) ? Z : vA
            z = load(op[6:], w3 >> 16)
            vA = z if vC == vB else vA
        elif op == "TSEL":              # table of (key, variable) pairs behind the pool
            t0 = pool0 + 2 * (w3 >> 16)
            n_ent = w3 & 0xFFFF
            keys = [int(words[t0 + 2 * i]) for i in range(n_ent)]
            assert len(set(keys)) == n_ent, "TSEL keys must be distinct"
            for i in range(n_ent):
                if vC == keys[i]:
                    vA = load("var", int(words[t0 + 2 * i + 1]))
        elif op == "TSELS":             # keys in LDS / bank slots / candidate rows, chain order
            t0 = pool0 + 2 * (w3 >> 16)
            for i in range(w3 & 0xFFFF):
                kw = int(words[t0 + 2 * i])
                if kw >> 31:
                    key = bank[((kw >> 16) & 0xFF) // 8]
                elif kw >> 30 & 1:
                    key = load("var", (kw >> 16) & 0x3FFF)
                else:
                    key = lds[kw & 0xFFFF]
                if vC == key:
                    vA = load("var", int(words[t0 + 2 * i + 1]))
        elif op in ("ADD", "SUB", "MUL", "AND", "OR", "XOR"):
            vA = {"ADD": vA + vB, "SUB": vA - vB, "MUL": vA * vB, "AND": vA & vB,
                  "OR": vA | vB, "XOR": vA ^ vB}[op] & M256
        elif op in ("SHL", "LSHR", "ASHR"):
            s = vB if vB < 256 else 256
            if op == "SHL":
                vA = (vA << s) & M256
            elif op == "LSHR":
                vA >>= s
            else:
                if w2 & U.F_SEXT:
                    vA = _sext(vA, KH)
                vA = (_s256(vA) >> s) & M256
        elif op == "DIV":
            a, b = vA, vB
            if w2 & U.F_SEXT:
                a, b = _sext(a, KH), _sext(b, KH)
            vA = _div((w2 >> U.DIVOP_POS) & 7, a, b) & M256
        elif op == "NOT":
            vA = ~vA & M256
        elif op == "NEG":
            vA = -vA & M256
        elif op == "MOV":
            pass
        elif op == "SEXT":
            vA = _sext(vA, KH)
        elif op[:4] in ("SHLI", "LSHR", "ASHR") and op[-1].isdigit():
            k = int(op[-1])
            s = 256 if k == 8 else 32 * k + sb
            if op.startswith("SHLI"):
                vA = (vA << s) & M256
            elif op.startswith("LSHRI"):
                vA >>= s
            else:
                if w2 & U.F_SEXT:
                    vA = _sext(vA, KH)
                vA = (_s256(vA) >> s) & M256
        elif op.startswith("CONCAT"):
            k = int(op[-1])
            vA = ((vA << (32 * k + sb)) & M256) | vB
        else:
            raise ValueError(op)
        if w2 & U.F_MASK:
            vA &= KM
        if w2 & U.F_STORE:
            if w2 & U.F_REGST:
                pos = (w2 & 0xFFFF) // 8
                assert not var_mask >> pos & 1, "register slot over a preloaded variable"
                bank[pos] = vA
            else:
                lds[w2 & 0xFFFF] = vA
    raise ValueError("uop program fell off the end without RET")


def first_sat_uops(words, off, cands) -> int:
    for i, xs in enumerate(cands):
        r = run_uops(words, off, xs)
        if r is None:
            return -2
        if r:
            return i
    return -1
