"""Opcode numbers and encoding constants — Python mirror of include/mgp_ir.h."""
from __future__ import annotations

VAR, CONST, TRUE, FALSE = 1, 2, 3, 4
ADD, SUB, MUL, UDIV, UREM, SDIV, SREM, SMOD = 8, 9, 10, 11, 12, 13, 14, 15
AND, OR, XOR, NOT, NEG, SHL, LSHR, ASHR = 16, 17, 18, 19, 20, 21, 22, 23
EXTRACT, CONCAT, ZEXT, SEXT, ITE = 24, 25, 26, 27, 28
EQ, ULT, ULE, UGT, UGE, SLT, SLE, SGT, SGE = 40, 41, 42, 43, 44, 45, 46, 47, 48
UADD_NOOVF, UMUL_NOOVF, USUB_NOUDF = 49, 50, 51
BAND, BOR, BXOR, BNOT, BITE, BEQ = 60, 61, 62, 63, 64, 65
UFAPP, UFINV = 70, 71
MOV, RET = 80, 90

MAX_WIDTH = 256

OP_NAMES = {v: k for k, v in dict(globals()).items() if k.isupper() and isinstance(v, int) and k != "MAX_WIDTH"}

BOOL_RESULT = frozenset({TRUE, FALSE, EQ, ULT, ULE, UGT, UGE, SLT, SLE, SGT, SGE, UADD_NOOVF, UMUL_NOOVF,
                         USUB_NOUDF, BAND, BOR, BXOR, BNOT, BITE, BEQ})

# nominal INT32 ops per node (same as mgp_synth.cpp nominal_op_cost)
NOMINAL_OPS = {
    ADD: 16, SUB: 16, NEG: 16, MUL: 108, UDIV: 1024, UREM: 1024, SDIV: 1024, SREM: 1024, SMOD: 1024,
    AND: 8, OR: 8, XOR: 8, NOT: 8, SHL: 32, LSHR: 32, ASHR: 32,
    EQ: 16, ULT: 16, ULE: 16, UGT: 16, UGE: 16, SLT: 16, SLE: 16, SGT: 16, SGE: 16,
    UADD_NOOVF: 16, USUB_NOUDF: 16, UMUL_NOOVF: 108, ITE: 8, EXTRACT: 8, CONCAT: 8, ZEXT: 8, SEXT: 8,
    BAND: 1, BOR: 1, BXOR: 1, BNOT: 1, BITE: 1, BEQ: 1, UFAPP: 16, UFINV: 16,
}
