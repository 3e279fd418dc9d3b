"""Reference interpreter of the mgp bytecode — TEST INFRASTRUCTURE.

Executes the encoding documented in include/mgp_ir.h instruction by
instruction with Python ints, so the host lowering (mgp_lower) can be checked
on a CPU-only machine: eval_dag(DAG) == run_program(lower(DAG)) for every
candidate.  Operator semantics come from oracle.bvsem.
"""
from __future__ import annotations

from typing import List, Sequence

from . import bvsem as S

K_SLOT, K_CONST, K_ACC, K_VAR = 0, 1, 2, 3
OP_MOV, OP_EQSEL, OP_RET = 80, 81, 90
BOOL_FALSE, BOOL_TRUE = 62, 63
LDS_SLOTS = 32   # MGP_LDS_SLOTS


def _limbs(words, off) -> int:
    return S.limbs_to_int(words[off:off + 8])


def run_program(words: Sequence[int], off: int, xs: Sequence[int]):
    """Run the program at word offset `off` for candidate vars `xs`.

    Returns True/False, or None when the header marks the state unsupported.
    """
    n_ins, n_c, n_slots, status = (int(words[off + k]) for k in range(4))
    if status & 0xFF:
        return None
    ins0 = off + 4
    pool = [_limbs(words, ins0 + 4 * n_ins + 8 * k) for k in range(n_c)]
    slots = {}
    # spill slots (>= LDS_SLOTS) live in the lane's candidate row past its variables
    # (include/mgp_ir.h): a row there must never be a variable the program reads
    max_var = status >> 8
    spill0 = max(max_var, 8)
    rows = {}
    acc = 0
    bools = 1 << BOOL_TRUE

    def bv(o: int) -> int:
        kind, idx = o >> 14, o & 0x3FFF
        if kind == K_ACC:
            return acc
        if kind == K_SLOT:
            if idx >= LDS_SLOTS:
                return rows[spill0 + idx - LDS_SLOTS]
            return slots[idx]
        if kind == K_CONST:
            return pool[idx]
        assert idx < max_var and idx not in rows
        return xs[idx] & S.mask(256)

    def bl(o: int) -> bool:
        return bool((bools >> o) & 1)

    for pc in range(n_ins):
        w0, w1, w2, w3 = (int(words[ins0 + 4 * pc + k]) for k in range(4))
        op = w0 & 0xFF
        width = ((w0 >> 8) & 0xFF) + 1
        dst = ((w0 >> 16) & 0xFF) | ((w3 & 0xFF) << 8)   # BV slots past 255: high bits in w3
        store = (w0 >> 24) & 1
        oa, ob, oc, imm = w1 & 0xFFFF, w1 >> 16, w2 & 0xFFFF, w2 >> 16
        if op == OP_RET:
            return bl(oa)
        if S.BAND <= op <= S.BEQ:
            a, b, c = bl(oa), bl(ob), bl(oc)
            r = {S.BAND: a and b, S.BOR: a or b, S.BXOR: a != b, S.BNOT: not a,
                 S.BITE: b if a else c, S.BEQ: a == b}[op]
            bools = (bools & ~(1 << dst)) | (int(r) << dst)
            continue
        if S.EQ <= op <= S.USUB_NOUDF:
            r = S.cmpop(op, bv(oa), bv(ob), width)
            bools = (bools & ~(1 << dst)) | (int(r) << dst)
            continue
        m = S.mask(width)
        if op == S.ITE:
            r = bv(ob) if bl(oa) else bv(oc)
        elif op == OP_EQSEL:   # select-chain step; operands never name the accumulator
            assert K_ACC not in (oa >> 14, ob >> 14, oc >> 14)
            r = bv(oc) if bv(oa) == bv(ob) else acc
        elif op in (OP_MOV, S.ZEXT):
            r = bv(oa)
        elif op == S.NOT:
            r = ~bv(oa)
        elif op == S.NEG:
            r = -bv(oa)
        elif op == S.EXTRACT:
            r = bv(oa) >> imm
        elif op == S.SEXT:
            r = S.to_signed(bv(oa), imm)
        elif op == S.CONCAT:
            r = (bv(oa) << imm) | bv(ob)
        else:
            r = S.binop(op, bv(oa) & m, bv(ob) & m, width)
        r &= m
        acc = r
        if store:
            if dst >= LDS_SLOTS:
                rows[spill0 + dst - LDS_SLOTS] = r
            else:
                slots[dst] = r
    raise ValueError("program fell off the end without RET")


def first_sat_program(words, off, cands) -> int:
    for i, xs in enumerate(cands):
        r = run_program(words, off, xs)
        if r is None:
            return -2
        if r:
            return i
    return -1
