"""z3 / SMT-LIB bit-vector semantics over Python ints — TEST INFRASTRUCTURE.

CPU restatement of what z3 computes for the laser.smt vocabulary the GPU
pre-filter evaluates (reference mythril v0.22.1):

  BitVec.__add__/__sub__/__mul__   bitvec.py:63-94        bvadd/bvsub/bvmul mod 2^w
  BitVec.__truediv__               bitvec.py:96-103       bvsdiv
  UDiv / URem / SRem               bitvec_helper.py:125-152
  << / LShR / >>                   bitvec.py:232-246, bitvec_helper.py:21-22
  < > <= >= (signed)               bitvec.py:138-180
  ULT/UGT/ULE/UGE                  bitvec_helper.py:43-80
  ==, != (zero-extend narrower)    bitvec.py:16-22, 183-216
  If / Concat / Extract            bitvec_helper.py:25-40, 93-122
  BVAddNoOverflow/BVMulNoOverflow/BVSubNoUnderflow (unsigned)  bitvec_helper.py:168-214
  And/Or/Not/Xor                   bool.py:87-123
  Function (uninterpreted)         function.py:7-25; keccak pairs keccak_function_manager.py:56-69

The definitions of bvsdiv/bvsrem/bvsmod follow the SMT-LIB QF_BV theory text
(msb case split), written independently of the HIP kernel's code.
Division-by-zero conventions are SMT-LIB's (x/0 = 2^w-1, x%0 = x) and are NOT
pinned by any reference test ("parity unpinned"); every
other operator is pinned by tests/golden.

Uninterpreted functions: a DAG's UFAPP/UFINV nodes are evaluated under the
lazily built interpretation documented in include/mgp_ir.h — a valid model of
the UF, so any witness found under it is a genuine model.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

# opcode numbers: include/mgp_ir.h
VAR, CONST, TRUE, FALSE = 1, 2, 3, 4
ADD, SUB, MUL, UDIV, UREM, SDIV, SREM, SMOD = 8, 9, 10, 11, 12, 13, 14, 15
AND, OR, XOR, NOT, NEG, SHL, LSHR, ASHR = 16, 17, 18, 19, 20, 21, 22, 23
EXTRACT, CONCAT, ZEXT, SEXT, ITE = 24, 25, 26, 27, 28
EQ, ULT, ULE, UGT, UGE, SLT, SLE, SGT, SGE = 40, 41, 42, 43, 44, 45, 46, 47, 48
UADD_NOOVF, UMUL_NOOVF, USUB_NOUDF = 49, 50, 51
BAND, BOR, BXOR, BNOT, BITE, BEQ = 60, 61, 62, 63, 64, 65
UFAPP, UFINV = 70, 71

BOOL_RESULT = {TRUE, FALSE, EQ, ULT, ULE, UGT, UGE, SLT, SLE, SGT, SGE, UADD_NOOVF, UMUL_NOOVF, USUB_NOUDF,
               BAND, BOR, BXOR, BNOT, BITE, BEQ}


def mask(w: int) -> int:
    return (1 << w) - 1


def msb(x: int, w: int) -> int:
    return (x >> (w - 1)) & 1


def to_signed(x: int, w: int) -> int:
    return x - (1 << w) if msb(x, w) else x


def bvneg(x: int, w: int) -> int:
    return (-x) & mask(w)


def bvudiv(s: int, t: int, w: int) -> int:
    return mask(w) if t == 0 else s // t


def bvurem(s: int, t: int, w: int) -> int:
    return s if t == 0 else s % t


def bvsdiv(s: int, t: int, w: int) -> int:
    ms, mt = msb(s, w), msb(t, w)
    if ms == 0 and mt == 0:
        return bvudiv(s, t, w)
    if ms == 1 and mt == 0:
        return bvneg(bvudiv(bvneg(s, w), t, w), w)
    if ms == 0 and mt == 1:
        return bvneg(bvudiv(s, bvneg(t, w), w), w)
    return bvudiv(bvneg(s, w), bvneg(t, w), w)


def bvsrem(s: int, t: int, w: int) -> int:
    ms, mt = msb(s, w), msb(t, w)
    if ms == 0 and mt == 0:
        return bvurem(s, t, w)
    if ms == 1 and mt == 0:
        return bvneg(bvurem(bvneg(s, w), t, w), w)
    if ms == 0 and mt == 1:
        return bvurem(s, bvneg(t, w), w)
    return bvneg(bvurem(bvneg(s, w), bvneg(t, w), w), w)


def bvsmod(s: int, t: int, w: int) -> int:
    ms, mt = msb(s, w), msb(t, w)
    abs_s = s if ms == 0 else bvneg(s, w)
    abs_t = t if mt == 0 else bvneg(t, w)
    u = bvurem(abs_s, abs_t, w)
    if u == 0:
        return u
    if ms == 0 and mt == 0:
        return u
    if ms == 1 and mt == 0:
        return (bvneg(u, w) + t) & mask(w)
    if ms == 0 and mt == 1:
        return (u + t) & mask(w)
    return bvneg(u, w)


def bvshl(x: int, s: int, w: int) -> int:
    return 0 if s >= w else (x << s) & mask(w)


def bvlshr(x: int, s: int, w: int) -> int:
    return 0 if s >= w else x >> s


def bvashr(x: int, s: int, w: int) -> int:
    if s >= w:
        return mask(w) if msb(x, w) else 0
    return (to_signed(x, w) >> s) & mask(w)


def binop(op: int, x: int, y: int, w: int) -> int:
    m = mask(w)
    if op == ADD:
        return (x + y) & m
    if op == SUB:
        return (x - y) & m
    if op == MUL:
        return (x * y) & m
    if op == UDIV:
        return bvudiv(x, y, w)
    if op == UREM:
        return bvurem(x, y, w)
    if op == SDIV:
        return bvsdiv(x, y, w)
    if op == SREM:
        return bvsrem(x, y, w)
    if op == SMOD:
        return bvsmod(x, y, w)
    if op == AND:
        return x & y
    if op == OR:
        return x | y
    if op == XOR:
        return x ^ y
    if op == SHL:
        return bvshl(x, y, w)
    if op == LSHR:
        return bvlshr(x, y, w)
    if op == ASHR:
        return bvashr(x, y, w)
    raise ValueError(f"not a binary BV op: {op}")


def cmpop(op: int, x: int, y: int, w: int) -> bool:
    if op == EQ:
        return x == y
    if op == ULT:
        return x < y
    if op == ULE:
        return x <= y
    if op == UGT:
        return x > y
    if op == UGE:
        return x >= y
    if op == SLT:
        return to_signed(x, w) < to_signed(y, w)
    if op == SLE:
        return to_signed(x, w) <= to_signed(y, w)
    if op == SGT:
        return to_signed(x, w) > to_signed(y, w)
    if op == SGE:
        return to_signed(x, w) >= to_signed(y, w)
    if op == UADD_NOOVF:
        return x + y < (1 << w)
    if op == UMUL_NOOVF:
        return x * y < (1 << w)
    if op == USUB_NOUDF:
        return y <= x
    raise ValueError(f"not a compare op: {op}")


def limbs_to_int(limbs: Sequence[int]) -> int:
    v = 0
    for i, l in enumerate(limbs):
        v |= (int(l) & 0xFFFFFFFF) << (32 * i)
    return v


def int_to_limbs(v: int, n: int = 8) -> List[int]:
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def wide_read(table: Sequence[int], first: int, w: int) -> int:
    """A w-bit value held in ceil(w/256) consecutive 256-bit entries, low first
    (include/mgp_ir.h "wide values"; w <= 256 is the single entry `first`)."""
    v = 0
    for j in range((w + 255) // 256):
        v |= (int(table[first + j]) & mask(256)) << (256 * j)
    return v & mask(w)


def eval_dag(nodes, consts: Sequence[int], xs: Sequence[int]) -> List:
    """Evaluate a topologically ordered node list.

    nodes: iterable of (op, width, a, b, c, p0, p1) (or a NODE_DTYPE array)
    consts: constant pool (ints); xs: candidate variable values (ints)
    Returns the list of node values (int for BV, bool for Bool).
    """
    vals: List = []
    widths: List[int] = []
    fapps: Dict[int, List[Tuple[int, int]]] = {}
    iapps: Dict[int, List[Tuple[int, int]]] = {}
    for nd in nodes:
        op, w, a, b, c, p0, p1 = (int(nd[0]), int(nd[2]), int(nd[3]), int(nd[4]), int(nd[5]), int(nd[6]),
                                  int(nd[7])) if len(nd) == 8 else tuple(int(v) for v in nd)
        if op in BOOL_RESULT:
            w = 1
        if op == VAR:
            v = wide_read(xs, p0, w)
        elif op == CONST:
            v = wide_read(consts, p0, w)
        elif op == TRUE:
            v = True
        elif op == FALSE:
            v = False
        elif ADD <= op <= ASHR and op not in (NOT, NEG):
            v = binop(op, vals[a], vals[b], w)
        elif op == NOT:
            v = (~vals[a]) & mask(w)
        elif op == NEG:
            v = bvneg(vals[a], w)
        elif op == EXTRACT:
            v = (vals[a] >> p1) & mask(p0 - p1 + 1)
            w = p0 - p1 + 1
        elif op == CONCAT:
            v = (vals[a] << widths[b]) | vals[b]
        elif op == ZEXT:
            v = vals[a]
        elif op == SEXT:
            v = to_signed(vals[a], widths[a]) & mask(w)
        elif op == ITE:
            v = vals[b] if vals[a] else vals[c]
            if isinstance(v, bool):
                w = 1
        elif EQ <= op <= USUB_NOUDF:
            if isinstance(vals[a], bool):
                v = vals[a] == vals[b]
            else:
                v = cmpop(op, vals[a], vals[b], widths[a])
        elif op == BAND:
            v = bool(vals[a] and vals[b])
        elif op == BOR:
            v = bool(vals[a] or vals[b])
        elif op == BXOR:
            v = bool(vals[a]) != bool(vals[b])
        elif op == BNOT:
            v = not vals[a]
        elif op == BITE:
            v = vals[b] if vals[a] else vals[c]
        elif op == BEQ:
            v = bool(vals[a]) == bool(vals[b])
        elif op == UFAPP:
            arg = vals[a]
            v = wide_read(xs, p1, w)
            for (aj, vj) in fapps.get(p0, []):
                if aj == arg:
                    v = vj
                    break
            fapps.setdefault(p0, []).append((arg, v))
        elif op == UFINV:
            arg = vals[a]
            v = None
            for (ak, vk) in iapps.get(p0, []):
                if ak == arg:
                    v = vk
                    break
            if v is None:
                for (aj, vj) in fapps.get(p0, []):
                    if vj == arg:
                        v = aj
                        break
            if v is None:
                v = wide_read(xs, p1, w)
            iapps.setdefault(p0, []).append((arg, v))
        else:
            raise ValueError(f"unknown op {op}")
        vals.append(v)
        widths.append(w)
    return vals


def eval_root(nodes, consts, xs) -> bool:
    return bool(eval_dag(nodes, consts, xs)[-1])


def first_sat(nodes, consts, cands: Sequence[Sequence[int]]) -> int:
    """Lowest candidate index whose assignment satisfies the root, else -1."""
    for i, xs in enumerate(cands):
        if eval_root(nodes, consts, xs):
            return i
    return -1
