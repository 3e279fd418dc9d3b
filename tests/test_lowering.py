"""Host lowering (mgp_lower, C++) vs the DAG oracle — CPU only.

The bytecode produced for the GPU is executed by oracle.bytecode_ref (an
independent interpreter of the encoding in include/mgp_ir.h) and its uop
re-encoding for the gfx950 assembly interpreter by oracle.uop_ref (register-
level semantics of the handlers, encoding in mythril_amd/uop_spec.py); both
must agree with oracle.bvsem on the DAG for every candidate.
"""
import numpy as np
import pytest

from mythril_amd import _native as N
from mythril_amd import uop_spec as U
from oracle import bvsem as S
from oracle import bytecode_ref as BR
from oracle import uop_ref as UR

from ._util import INTERESTING, cands_from_ints, load_golden, pack_states, state_slice


def _check_states(states, cand_rows, max_slots=0):
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = N.lower(nodes, noff, consts, coff, max_slots=max_slots)
    for s, (nl, cl) in enumerate(states):
        for xs in cand_rows[s]:
            want = S.eval_root(nl, cl, xs)
            got = BR.run_program(words, int(po[s]), xs)
            assert got == want, (s, xs)
            assert UR.run_uops(words, int(po[s]), xs) == want, ("uop", s, xs)
    return words, po, status


def test_synthetic_lowering_matches_dag():
    b = N.synth_generate(0x4D595448, 99, 150, 64, 16)
    words, po, status = N.lower(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
    assert (status == 0).all()
    rng = np.random.default_rng(1)
    for s in range(150):
        nodes, consts = state_slice(b, s)
        rows = [[int(rng.integers(0, 2 ** 63)) << int(rng.integers(0, 190)) for _ in range(6)] for _ in range(6)]
        rows.append([INTERESTING[int(rng.integers(0, len(INTERESTING)))] for _ in range(6)])
        if b["planted"][s]:
            rows.append([S.limbs_to_int(x) for x in b["plant_words"][s]])
        for xs in rows:
            want = S.eval_root(nodes, consts, xs)
            assert BR.run_program(words, int(po[s]), xs) == want, s
            assert UR.run_uops(words, int(po[s]), xs) == want, ("uop", s)


def test_golden_arith_lowering():
    cases = [t for t in load_golden("vm_arith.json") if t["reference_agrees"]][:80]
    states = []
    for t in cases:
        consts = [int(c, 16) for c in t["consts"]]
        node, exp = t["checks"][0]
        nl = [list(n) for n in t["nodes"]]
        cx = consts + [int(exp, 16)]
        nl.append([S.CONST, 256, -1, -1, -1, len(cx) - 1, 0])
        nl.append([S.EQ, 1, node, len(nl) - 1, -1, 0, 0])
        states.append((nl, cx))
    _check_states(states, [[[]]] * len(states))


def test_narrow_widths_and_signed_ops():
    rng = np.random.default_rng(2)
    states, rows = [], []
    for w in (1, 7, 8, 31, 32, 33, 64, 100, 160, 255):
        for op in (S.ADD, S.SUB, S.MUL, S.UDIV, S.UREM, S.SDIV, S.SREM, S.SMOD, S.SHL, S.LSHR, S.ASHR):
            for cmp in (S.SLT, S.ULE, S.SGE, S.EQ, S.UMUL_NOOVF, S.UADD_NOOVF):
                nl = [[S.VAR, w, -1, -1, -1, 0, 0], [S.VAR, w, -1, -1, -1, 1, 0], [op, w, 0, 1, -1, 0, 0],
                      [S.SEXT, 256, 2, -1, -1, 0, 0], [S.EXTRACT, w, 3, -1, -1, w - 1, 0],
                      [cmp, 1, 4, 0, -1, 0, 0]]
                states.append((nl, []))
                rows.append([[int(rng.integers(0, 2 ** 62)) * (1 << int(rng.integers(0, 200))),
                              int(rng.integers(0, 2 ** 62))] for _ in range(4)] + [[(1 << w) - 1, 0],
                                                                                    [1 << (w - 1), (1 << w) - 1]])
    _check_states(states, rows)


def test_concat_extract_ite_bool_ops():
    nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0],
          [S.EXTRACT, 8, 0, -1, -1, 15, 8], [S.EXTRACT, 160, 1, -1, -1, 159, 0],
          [S.CONCAT, 168, 2, 3, -1, 0, 0], [S.ZEXT, 256, 4, -1, -1, 0, 0],
          [S.ULT, 1, 5, 0, -1, 0, 0], [S.ITE, 256, 6, 0, 1, 0, 0],
          [S.EQ, 1, 7, 1, -1, 0, 0], [S.BXOR, 1, 6, 8, -1, 0, 0], [S.BITE, 1, 9, 6, 8, 0, 0],
          [S.TRUE, 1, -1, -1, -1, 0, 0], [S.BEQ, 1, 10, 11, -1, 0, 0], [S.EQ, 1, 12, 9, -1, 0, 0]]
    rows = [[[a, b] for a in INTERESTING[:8] for b in INTERESTING[:8]]]
    _check_states([(nl, [])], rows)


def test_uf_chains():
    # three apps of f, one inverse, consistency must hold in all orders
    nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0], [S.VAR, 256, -1, -1, -1, 2, 0],
          [S.UFAPP, 256, 0, -1, -1, 0, 3], [S.UFAPP, 256, 1, -1, -1, 0, 4], [S.UFAPP, 256, 2, -1, -1, 0, 5],
          [S.UFINV, 256, 4, -1, -1, 0, 6], [S.UFINV, 256, 5, -1, -1, 0, 7],
          [S.EQ, 1, 6, 1, -1, 0, 0], [S.EQ, 1, 3, 5, -1, 0, 0], [S.BOR, 1, 8, 9, -1, 0, 0],
          [S.EQ, 1, 7, 2, -1, 0, 0], [S.BAND, 1, 10, 11, -1, 0, 0]]
    rows = []
    for x0 in (1, 2):
        for x1 in (1, 2, 3):
            for x2 in (1, 3):
                for h in ((10, 10, 10), (10, 11, 12), (10, 11, 10)):
                    rows.append([x0, x1, x2, *h, 1, 2])
    _check_states([(nl, [])], [rows])


def test_uf_constant_arguments_fold():
    # a 32-byte calldata word: 32 selects at constant indices (calldata.py:219-232), one
    # index repeated and one symbolic index read first; constant-vs-constant argument comparisons fold
    # at lowering time, so the state fits the slot budget and agrees with the oracle
    F = 3
    nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.UFAPP, 8, 0, -1, -1, F, 40]]   # x0, calldata[x0]
    sym = 1
    consts = list(range(4, 36)) + [7]
    apps = []
    for i, ci in enumerate(list(range(32)) + [32]):               # last app repeats index 7
        nl.append([S.CONST, 256, -1, -1, -1, ci, 0])
        nl.append([S.UFAPP, 8, len(nl) - 1, -1, -1, F, 1 + i])
        apps.append(len(nl) - 1)
    acc = apps[0]
    for a in apps[1:32]:
        nl.append([S.CONCAT, nl[acc][1] + 8, acc, a, -1, 0, 0])
        acc = len(nl) - 1
    nl.append([S.EQ, 1, apps[32], apps[3], -1, 0, 0])               # f(7) twice: always equal
    e_rep = len(nl) - 1
    nl.append([S.EQ, 1, sym, apps[5], -1, 0, 0])                     # f(x0) == f(9)
    e_sym = len(nl) - 1
    nl.append([S.EXTRACT, 8, acc, -1, -1, 7, 0])
    nl.append([S.EQ, 1, len(nl) - 1, apps[31], -1, 0, 0])            # low byte is f(35)
    nl.append([S.BAND, 1, e_rep, len(nl) - 1, -1, 0, 0])
    nl.append([S.BAND, 1, len(nl) - 1, e_sym, -1, 0, 0])
    rng = np.random.default_rng(17)
    rows = []
    for _ in range(40):
        xs = [int(rng.integers(0, 40))] + [int(rng.integers(0, 4)) for _ in range(41)]
        rows.append(xs)
    rows.append([9] + [1] * 41)
    _, _, status = _check_states([(nl, consts)], [rows])
    assert status[0] == N.ST_OK
    assert S.eval_root(nl, consts, [9] + [1] * 41)


def _live_chain(n):
    # n values each used by two chains that consume them in opposite orders:
    # whatever the schedule, all n are live at once
    nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0]]
    vals = []
    for i in range(n):
        nl.append([S.ADD if i % 2 else S.MUL, 256, len(nl) - 1 if i else 0, i % 2, -1, 0, 0])
        vals.append(len(nl) - 1)
    acc = vals[0]
    for v in vals[1:]:
        nl.append([S.XOR, 256, acc, v, -1, 0, 0])
        acc = len(nl) - 1
    acc2 = vals[-1]
    for v in reversed(vals[:-1]):
        nl.append([S.SUB, 256, acc2, v, -1, 0, 0])
        acc2 = len(nl) - 1
    nl.append([S.ULT, 1, acc, acc2, -1, 0, 0])
    return nl


def _bool_fan(n):
    # n compares that are all live at once (read again in reverse order by a BAND chain
    # after a BOR chain over them): more than the 17 Bool registers of the interpreter
    nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0]]
    cmps = []
    for i in range(n):
        nl.append([S.CONST, 256, -1, -1, -1, i, 0])
        nl.append([S.ULT if i % 2 else S.EQ, 1, len(nl) - 1, i % 2, -1, 0, 0])
        cmps.append(len(nl) - 1)
    acc = cmps[0]
    for c in cmps[1:]:
        nl.append([S.BOR, 1, acc, c, -1, 0, 0])
        acc = len(nl) - 1
    acc2 = cmps[-1]
    for c in reversed(cmps[:-1]):
        nl.append([S.BXOR, 1, acc2, c, -1, 0, 0])
        acc2 = len(nl) - 1
    nl.append([S.BAND, 1, acc, acc2, -1, 0, 0])
    return nl, list(range(3, 3 + 7 * n, 7))


def _header(words, po, s):
    return [int(words[int(po[s]) + k]) for k in range(4)]


def test_many_live_values_spill_to_candidate_rows():
    """Past the LDS slots, BV values spill to the lane's candidate rows past its variables
    (include/mgp_ir.h): a 4-slot cap, 40 and 200 live values all lower and agree with the
    DAG in both encodings (the reference interpreters assert that no spill row is a
    variable the program reads, and that every row is written before it is read);
    300 live values need destinations past slot 255 (high bits in instruction word 3,
    round 4: WalletLibrary's input-order programs need up to 326); past MGP_MAX_SLOTS the
    state is unsupported, never wrong."""
    rows = [[3, 5], [INTERESTING[3], INTERESTING[4]], [0, 2 ** 256 - 1]]
    for n, cap in ((28, 4), (40, 0), (200, 0), (300, 0)):
        nl = _live_chain(n)
        words, po, status = _check_states([(nl, [])], [rows], max_slots=cap)
        assert status[0] == N.ST_OK, (n, cap)
        h = _header(words, po, 0)
        assert h[2] >= 32 if (n > 32 or cap) else True
        assert N.prog_rows(words, po)[0] == (max(h[3] >> 8, 8) + h[2] - 31 if h[2] >= 32 else h[3] >> 8)
    nl = _live_chain(4200)
    nodes, noff, consts, coff = pack_states([(nl, [])])
    words, po, status = N.lower(nodes, noff, consts, coff)
    assert status[0] == N.ST_UNSUPPORTED
    assert BR.run_program(words, int(po[0]), [3, 5]) is None
    assert UR.run_uops(words, int(po[0]), [3, 5]) is None


def test_bool_pressure_demotes_to_bv():
    """More live Bools than the interpreter's 17 registers: the lowering demotes the
    farthest-read ones to 1-bit values (ITE / EQ) and the program still agrees."""
    for n in (16, 24, 60):
        nl, consts = _bool_fan(n)
        rows = [[consts[k], consts[k] + 1] for k in (0, 1, n // 2, n - 1)] + [[0, 0], [5, 2 ** 255]]
        _, _, status = _check_states([(nl, consts)], [rows])
        assert status[0] == N.ST_OK, n


def test_constant_pool_past_64_entries():
    """More than 64 constants: the interpreter's pool has the mask / sign constants first
    (6-bit index fields), then up to 255 entries in all."""
    nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 64, -1, -1, -1, 1, 0]]
    consts = [(k * 0x9E3779B97F4A7C15 + 1) % 2 ** 256 for k in range(150)]
    acc = 0
    for k in range(150):
        nl.append([S.CONST, 256, -1, -1, -1, k, 0])
        nl.append([S.XOR if k % 3 else S.ADD, 256, acc, len(nl) - 1, -1, 0, 0])
        acc = len(nl) - 1
    nl.append([S.EXTRACT, 64, acc, -1, -1, 63, 0])
    nl.append([S.ADD, 64, len(nl) - 1, 1, -1, 0, 0])                   # masked: a width-64 mask constant
    nl.append([S.SLT, 1, len(nl) - 1, 1, -1, 0, 0])                    # signed: a sign constant
    rows = [[7, 9], [INTERESTING[5], 2 ** 63], [0, 2 ** 64 - 1]]
    words, po, status = _check_states([(nl, consts)], [rows])
    assert status[0] == N.ST_OK
    u0 = UR.uop_offset(words, int(po[0]))
    assert int(words[u0 + 3]) & 0xFF > 64


def wide_struct_case():
    # 516-bit and 512-bit values (include/mgp_ir.h "wide values"): VAR over three
    # slots, wide CONST over two pool entries, CONCAT with boundaries that do not
    # line up with 256, EXTRACT (narrow and wide, across pieces), ZEXT, ITE, EQ
    c512 = (0x1234 << 400) | (7 << 255) | 0xABCDEF
    nl = [[S.VAR, 160, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0], [S.VAR, 100, -1, -1, -1, 2, 0],
          [S.CONCAT, 356, 2, 1, -1, 0, 0], [S.CONCAT, 516, 3, 0, -1, 0, 0],        # 4: x2 . x1 . x0
          [S.VAR, 516, -1, -1, -1, 3, 0],                                            # 5: x3,x4,x5 (3 slots)
          [S.EQ, 1, 4, 5, -1, 0, 0],                                                 # 6
          [S.EXTRACT, 200, 4, -1, -1, 299, 100], [S.EXTRACT, 200, 5, -1, -1, 299, 100],
          [S.EQ, 1, 7, 8, -1, 0, 0],                                                 # 9
          [S.EXTRACT, 400, 5, -1, -1, 459, 60], [S.ZEXT, 512, 1, -1, -1, 0, 0],      # 10, 11
          [S.CONST, 512, -1, -1, -1, 0, 0], [S.ULT, 1, 7, 8, -1, 0, 0],              # 12, 13
          [S.ITE, 512, 13, 11, 12, 0, 0], [S.EXTRACT, 512, 5, -1, -1, 511, 0],       # 14, 15
          [S.EQ, 1, 14, 15, -1, 0, 0], [S.EXTRACT, 256, 10, -1, -1, 399, 144],      # 16, 17
          [S.EXTRACT, 256, 5, -1, -1, 459, 204], [S.EQ, 1, 17, 18, -1, 0, 0],        # 18, 19
          [S.BOR, 1, 6, 16, -1, 0, 0], [S.BAND, 1, 20, 19, -1, 0, 0], [S.BOR, 1, 21, 9, -1, 0, 0]]
    consts = [c512 & ((1 << 256) - 1), c512 >> 256]
    rng = np.random.default_rng(7)
    rows = []
    for _ in range(24):
        x = [int(rng.integers(0, 2 ** 62)) << int(rng.integers(0, 190)) for _ in range(6)]
        rows.append(x)
        big = x[0] & ((1 << 160) - 1) | (x[1] << 160) | ((x[2] & ((1 << 100) - 1)) << 416)
        rows.append(x[:3] + [big & ((1 << 256) - 1), (big >> 256) & ((1 << 256) - 1), big >> 512])  # 6 true
        rows.append(x[:3] + [c512 & ((1 << 256) - 1), c512 >> 256, x[5]])                           # 16 via const
        rows.append([x[0], 1 << 255, x[2], x[1], x[1] << 1, x[5]])
    return nl, consts, rows


def test_wide_structural_ops():
    nl, consts, rows = wide_struct_case()
    _, _, status = _check_states([(nl, consts)], [rows])
    assert status[0] == N.ST_OK
    assert sum(S.eval_root(nl, consts, r) for r in rows) >= 24


def wide_arith_cases():
    """ADD / SUB (carry chains), MUL (128-bit limb schoolbook), bitwise ops and unsigned
    compares on 257..776-bit values
    built from 256-bit vars: BVAddNoOverflow's 257-bit expansion
    Extract(256, 256, ZeroExt(1, a) + ZeroExt(1, b)) == 0 among them."""
    states, rows = [], []
    rng = np.random.default_rng(11)
    edge = [0, 1, (1 << 256) - 1, (1 << 256) - 2, 1 << 255, (1 << 255) - 1, 5]
    for w in (257, 300, 512, 516, 776):
        for op in (S.ADD, S.SUB, S.MUL, S.AND, S.OR, S.XOR, S.NOT):
            for cmp in (S.EQ, S.ULT, S.ULE, S.UGT, S.UGE):
                # a = ZeroExt / Concat of vars, b likewise, r = a op b, check cmp(r, c) and Extract(top bit)
                k = w - 256
                nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0],
                      [S.VAR, min(k, 256), -1, -1, -1, 2, 0], [S.VAR, 256, -1, -1, -1, 3, 0],
                      [S.CONCAT, w, 2, 0, -1, 0, 0] if k <= 256 else [S.ZEXT, w, 0, -1, -1, 0, 0],
                      [S.ZEXT, w, 1, -1, -1, 0, 0],
                      [op, w, 4, 5, -1, 0, 0] if op != S.NOT else [S.NOT, w, 4, -1, -1, 0, 0],
                      [S.CONCAT, w, 2, 3, -1, 0, 0] if k <= 256 else [S.ZEXT, w, 3, -1, -1, 0, 0],
                      [cmp, 1, 6, 7, -1, 0, 0], [S.EXTRACT, 1, 6, -1, -1, w - 1, w - 1],
                      [S.EXTRACT, 1, 6, -1, -1, 255, 255], [S.EQ, 1, 9, 10, -1, 0, 0],
                      [S.BOR, 1, 8, 11, -1, 0, 0] if cmp != S.EQ else [S.BAND, 1, 8, 8, -1, 0, 0]]
                states.append((nl, []))
                r = []
                for _ in range(5):
                    xs = [edge[int(rng.integers(0, len(edge)))] if rng.random() < 0.6 else
                          int(rng.integers(0, 2 ** 62)) << int(rng.integers(0, 194)) for _ in range(4)]
                    xs[2] &= (1 << min(k, 256)) - 1
                    r.append(xs)
                # r == c exactly for EQ rows: pick x3 so that Concat(x2, x3) equals the result
                xs = list(r[0])
                vals = S.eval_dag(nl, [], xs)
                res = vals[6]
                if k <= 256:
                    xs[2], xs[3] = res >> 256, res & ((1 << 256) - 1)
                r.append(xs)
                rows.append(r)
    return states, rows


def test_wide_arith_and_compares():
    states, rows = wide_arith_cases()
    _, _, status = _check_states(states, rows)
    assert (status == 0).all()


def test_wide_ops_left_unsupported():
    v0 = [S.VAR, 256, -1, -1, -1, 0, 0]
    for op in (S.UDIV, S.UREM, S.SHL, S.LSHR, S.SLT):
        nl = [v0, [S.CONCAT, 512, 0, 0, -1, 0, 0],
              [op, 1 if op == S.SLT else 512, 1, 1, -1, 0, 0]]
        nl.append([S.BAND, 1, 2, 2, -1, 0, 0] if op == S.SLT else [S.EQ, 1, 2, 1, -1, 0, 0])
        nodes, noff, consts, coff = pack_states([(nl, [])])
        _, _, status = N.lower(nodes, noff, consts, coff)
        assert status[0] == N.ST_UNSUPPORTED, op


def wide_zext_cases():
    """UDIV / UREM / LSHR / ASHR and signed compares on 257..776-bit values whose bits from
    256 up are zero (round 6): ZeroExt of a 256-bit variable, or Concat(0, x) -- the salt
    padding of CREATE2's 776-bit preimage (instructions.py:1707-1721) -- against a divisor /
    shift amount that is zero, one, small, the dividend or anything, with the result's low
    and high halves checked.  -> (states, candidate rows)."""
    states, rows = [], []
    rng = np.random.default_rng(0x776)
    edge = [0, 1, 2, 255, 256, 257, 775, 776, (1 << 256) - 1, 1 << 255, 5]
    for w in (257, 300, 512, 776):
        for op in (S.UDIV, S.UREM, S.LSHR, S.ASHR, S.SLT, S.SLE, S.SGT, S.SGE):
            for shape in range(2):
                nl = [[S.VAR, 256, -1, -1, -1, k, 0] for k in range(4)]                      # 0..3
                nl.append([S.CONST, w - 256, -1, -1, -1, 0, 0])                               # 4: zero pad
                nl.append([S.CONCAT, w, 4, 0, -1, 0, 0] if shape else [S.ZEXT, w, 0, -1, -1, 0, 0])  # 5: a
                nl.append([S.ZEXT, w, 1, -1, -1, 0, 0])                                       # 6: b
                if op in (S.SLT, S.SLE, S.SGT, S.SGE):
                    nl.append([op, 1, 5, 6, -1, 0, 0])                                        # 7
                    nl.append([S.EQ, 1, 2, 3, -1, 0, 0])                                      # 8
                    nl.append([S.BXOR, 1, 7, 8, -1, 0, 0])                                    # 9
                else:
                    nl.append([op, w, 5, 6, -1, 0, 0])                                        # 7: r
                    nl.append([S.EXTRACT, 256, 7, -1, -1, 255, 0])                            # 8: low
                    nl.append([S.EXTRACT, w - 256, 7, -1, -1, w - 1, 256])                    # 9: high
                    nl.append([S.ZEXT, 256, 9, -1, -1, 0, 0] if w - 256 < 256 else [S.EXTRACT, 256, 9, -1, -1, 255, 0])  # 10
                    nl.append([S.EQ, 1, 8, 2, -1, 0, 0])                                      # 11
                    nl.append([S.ULT, 1, 10, 3, -1, 0, 0])                                    # 12
                    nl.append([S.BAND, 1, 11, 12, -1, 0, 0])                                  # 13
                states.append((nl, [0, 0, 0]))
                r = []
                for _ in range(8):
                    xs = [edge[int(rng.integers(0, len(edge)))] if rng.random() < 0.5 else
                          int(rng.integers(0, 2 ** 62)) << int(rng.integers(0, 194)) for _ in range(4)]
                    r.append(xs)
                # make the root true on some rows: the low result and a bound above the high half
                for xs in list(r[:4]):
                    vals = S.eval_dag(nl, [0, 0, 0], xs)
                    ys = list(xs)
                    if op in (S.SLT, S.SLE, S.SGT, S.SGE):
                        ys[3] = ys[2] if not vals[7] else ys[2] ^ 1
                    else:
                        ys[2] = vals[8]
                        ys[3] = (vals[10] + 1) & ((1 << 256) - 1)
                    r.append(ys)
                rows.append(r)
    return states, rows


def test_wide_zero_extended_division_shifts_signed():
    """Wide zero-extended division, right shifts and signed compares lower (round 6) and
    match the DAG semantics (oracle.bvsem) in the bytecode and uop reference interpreters,
    x / 0 = 2^w - 1 in the high pieces included."""
    states, rows = wide_zext_cases()
    _, _, status = _check_states(states, rows)
    assert (status == 0).all()
    assert sum(S.eval_root(nl, cl, xs) for (nl, cl), r in zip(states, rows) for xs in r) > 100


def test_wide_mul_no_overflow_expansion():
    # z3's expansion of BVMulNoOverflow(a, b, False) (bitvec_helper.py:188-199):
    # Extract(511, 256, ZeroExt(256, a) * ZeroExt(256, b)) == 0, against UMUL_NOOVF itself
    nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0],
          [S.ZEXT, 512, 0, -1, -1, 0, 0], [S.ZEXT, 512, 1, -1, -1, 0, 0], [S.MUL, 512, 2, 3, -1, 0, 0],
          [S.EXTRACT, 256, 4, -1, -1, 511, 256], [S.CONST, 256, -1, -1, -1, 0, 0], [S.EQ, 1, 5, 6, -1, 0, 0],
          [S.UMUL_NOOVF, 1, 0, 1, -1, 0, 0], [S.BEQ, 1, 7, 8, -1, 0, 0],
          [S.EXTRACT, 256, 4, -1, -1, 255, 0], [S.MUL, 256, 0, 1, -1, 0, 0], [S.EQ, 1, 10, 11, -1, 0, 0],
          [S.BAND, 1, 9, 12, -1, 0, 0]]
    rng = np.random.default_rng(13)
    rows = [[a, b] for a in INTERESTING for b in INTERESTING[::3]]
    rows += [[int(rng.integers(0, 2 ** 63)) << int(rng.integers(0, 193)),
              int(rng.integers(0, 2 ** 63)) << int(rng.integers(0, 193))] for _ in range(40)]
    _, _, status = _check_states([(nl, [0])], [rows])
    assert status[0] == N.ST_OK
    assert all(S.eval_root(nl, [0], r) for r in rows)  # the expansion agrees with the predicate


def wide_mapping_case():
    # keccak256_512 over Concat(key, slot) and its inverse, as
    # keccak_function_manager.create_keccak builds them (keccak_function_manager.py:122-146):
    # inv(f(k0 . 0)) == k0 . 0, inv(f(k1 . 1)) == k1 . 1, and f(k0 . 0) == f(k1 . 1) must then
    # be impossible (different slots), while f(k0 . 0) == f(k2 . 0) forces k0 == k2
    F = 5
    nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0], [S.VAR, 256, -1, -1, -1, 2, 0],
          [S.CONST, 256, -1, -1, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 1, 0],
          [S.CONCAT, 512, 0, 3, -1, 0, 0], [S.CONCAT, 512, 1, 4, -1, 0, 0], [S.CONCAT, 512, 2, 3, -1, 0, 0],
          [S.UFAPP, 256, 5, -1, -1, F, 3], [S.UFAPP, 256, 6, -1, -1, F, 4], [S.UFAPP, 256, 7, -1, -1, F, 5],
          [S.UFINV, 512, 8, -1, -1, F, 6], [S.UFINV, 512, 9, -1, -1, F, 8], [S.UFINV, 512, 10, -1, -1, F, 10],
          [S.EQ, 1, 11, 5, -1, 0, 0], [S.EQ, 1, 12, 6, -1, 0, 0], [S.EQ, 1, 13, 7, -1, 0, 0],
          [S.BAND, 1, 14, 15, -1, 0, 0], [S.BAND, 1, 17, 16, -1, 0, 0],                 # 17, 18: consistency
          [S.EQ, 1, 8, 9, -1, 0, 0], [S.EQ, 1, 8, 10, -1, 0, 0], [S.EQ, 1, 0, 2, -1, 0, 0],  # 19, 20, 21
          [S.BAND, 1, 18, 19, -1, 0, 0], [S.BXOR, 1, 20, 21, -1, 0, 0],                # 22, 23
          [S.BAND, 1, 18, 23, -1, 0, 0], [S.BOR, 1, 22, 24, -1, 0, 0]]                  # root: never true
    consts = [0, 1]
    rows = []
    for k0 in (3, 1 << 200):
        for k1 in (3, 4):
            for k2 in (3, 1 << 200, 9):
                for h in ((10, 10, 10), (10, 11, 12), (10, 11, 10), (7, 7, 8)):
                    for fr in ((0, 0, 0, 0, 0, 0), (3, 0, 3, 1, 9, 0), (k0, 0, k1, 1, k2, 0)):
                        rows.append([k0, k1, k2, *h, *fr])
    nl_cons = nl[:21] + [[S.BAND, 1, 18, 20, -1, 0, 0]]  # consistent and f(k0.0) == f(k2.0): sat iff k0 == k2 allowed
    return nl, nl_cons, consts, rows


def test_wide_keccak_mapping_uf():
    nl, nl_cons, consts, rows = wide_mapping_case()
    nodes, noff, cpk, coff = pack_states([(nl, consts)])
    words, po, status = N.lower(nodes, noff, cpk, coff)
    assert status[0] == N.ST_OK
    _check_states([(nl, consts), (nl_cons, consts)], [rows, rows])
    assert not any(S.eval_root(nl, consts, r) for r in rows)
    assert any(S.eval_root(nl_cons, consts, r) for r in rows)
    assert all(r[0] == r[2] for r in rows if S.eval_root(nl_cons, consts, r))


@pytest.mark.parametrize("bad", ["wide", "forward_ref", "bool_as_bv", "width_mismatch", "root_bv", "unknown_op"])
def test_malformed_dags_are_unsupported(bad):
    v0 = [S.VAR, 256, -1, -1, -1, 0, 0]
    v1 = [S.VAR, 256, -1, -1, -1, 1, 0]
    nl = {
        "wide": [v0, v1, [S.CONCAT, 512, 0, 1, -1, 0, 0], [S.UDIV, 512, 2, 2, -1, 0, 0],
                 [S.EXTRACT, 1, 3, -1, -1, 0, 0], [S.EQ, 1, 4, 4, -1, 0, 0]],
        "forward_ref": [v0, [S.ULT, 1, 0, 2, -1, 0, 0], v1],
        "bool_as_bv": [v0, [S.ULT, 1, 0, 0, -1, 0, 0], [S.ADD, 256, 0, 1, -1, 0, 0], [S.EQ, 1, 2, 0, -1, 0, 0]],
        "width_mismatch": [v0, [S.VAR, 8, -1, -1, -1, 1, 0], [S.ULT, 1, 0, 1, -1, 0, 0]],
        "root_bv": [v0, v1, [S.ADD, 256, 0, 1, -1, 0, 0]],
        "unknown_op": [v0, [99, 1, 0, 0, -1, 0, 0]],
    }[bad]
    nodes, noff, consts, coff = pack_states([(nl, []), ([v0, v1, [S.ULT, 1, 0, 1, -1, 0, 0]], [])])
    words, po, status = N.lower(nodes, noff, consts, coff)
    assert status[0] == N.ST_UNSUPPORTED and status[1] == N.ST_OK
    assert BR.run_program(words, int(po[0]), [1, 2]) is None
    assert BR.run_program(words, int(po[1]), [1, 2]) is True
    assert UR.run_uops(words, int(po[0]), [1, 2]) is None
    assert UR.run_uops(words, int(po[1]), [1, 2]) is True


def test_empty_batch_and_constant_roots():
    nodes, noff, consts, coff = pack_states([([[S.TRUE, 1, -1, -1, -1, 0, 0]], []),
                                             ([[S.FALSE, 1, -1, -1, -1, 0, 0]], [])])
    words, po, status = N.lower(nodes, noff, consts, coff)
    assert BR.run_program(words, int(po[0]), []) is True
    assert BR.run_program(words, int(po[1]), []) is False
    assert UR.run_uops(words, int(po[0]), []) is True
    assert UR.run_uops(words, int(po[1]), []) is False
    w0, po0, st0 = N.lower(np.zeros(0, dtype=N.NODE_DTYPE), np.zeros(1, np.uint64), np.zeros((0, 8), np.uint32),
                           np.zeros(1, np.uint64))
    assert len(po0) == 1 and w0.size == 0


def test_program_layout_invariants():
    b = N.synth_generate(0x4D595448, 5, 500, 64, 256)
    words, po, status = N.lower(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
    hdr = N.program_headers(words, po)
    assert (po % 4 == 0).all(), "programs must be 16-byte aligned for s_load_dwordx4"
    sizes = 4 + 4 * hdr[:, 0].astype(np.int64) + 8 * hdr[:, 1].astype(np.int64)
    assert (sizes <= (po[1:] - po[:-1]).astype(np.int64)).all()
    assert hdr[:, 2].max() <= 32 and (hdr[:, 3] >> 8 <= b["n_vars"]).all()
    # deterministic
    w2, po2, _ = N.lower(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
    assert np.array_equal(words, w2) and np.array_equal(po, po2)


def test_synthetic_generator_is_deterministic_and_sliceable():
    a = N.synth_generate(0x4D595448, 0, 64, 64, 256)
    b = N.synth_generate(0x4D595448, 32, 32, 64, 256)
    off = int(a["node_offsets"][32])
    assert np.array_equal(a["nodes"][off:], b["nodes"])
    assert np.array_equal(a["planted"][32:], b["planted"])
    assert np.array_equal(a["plant_words"][32:], b["plant_words"])
    ops = N.nominal_ops(a["nodes"], a["node_offsets"])
    assert 1000 < ops.mean() < 6000


def test_c_oracle_wide_values_match_python_oracle():
    """The C oracle (the GPU tests' checker and the CPU baseline) evaluates states with
    values wider than 256 bits on MGP_MAX_WIDE-bit values: it must agree with
    oracle.bvsem on the wide structural, arithmetic and keccak256_512 mapping cases and
    on contract-shaped states with 512-bit mapping preimages (WalletLibrary)."""
    from oracle import coracle

    nl_s, c_s, rows_s = wide_struct_case()
    nl_m, nl_c, c_m, rows_m = wide_mapping_case()
    a_states, a_rows = wide_arith_cases()
    cases = [((nl_s, c_s), rows_s), ((nl_m, c_m), rows_m), ((nl_c, c_m), rows_m)]
    cases += [(st, r) for st, r in zip(a_states, a_rows)]
    for (nl, cl), rows in cases:
        n_vars = max(len(r) for r in rows)
        full = [list(r) + [0] * (n_vars - len(r)) for r in rows]
        nodes, noff, consts, coff = pack_states([(nl, cl)])
        got = coracle.first_sat(nodes, noff, consts, coff, cands_from_ints([full]))
        assert got[0] == S.first_sat(nl, cl, full)


def test_c_oracle_contract_states_match_python_oracle():
    import corpus
    from mythril_amd import dag as D
    from mythril_amd import front as F
    from corpus.keccak_manager import KeccakFunctionManager
    from oracle import coracle

    kfm = KeccakFunctionManager()
    items = corpus.wallet_states(0, kfm)[:3] + [corpus.bectoken_states(k, kfm) for k in range(2)]
    B = F.Batch([list(c[1]) for c in items])
    nv = B.n_vars()
    _, dom = N.refute_domains(*B.packed(), B.var_off)
    cands = N.make_candidates(12, nv, 99, B.var_off, B.var_width, B.hint_off, B.hints, B.alias_off, B.aliases,
                              B.const_off, B.consts, D._FIXED_LIMBS, np.zeros(B.n_states, np.uint8),
                              var_kind=B.var_kind, dom=dom)
    N.guided_candidates(*B.packed(), cands, seed=5, every=2, n_decide=2)
    nodes, noff, consts, coff = B.packed(gpu=True)
    got = coracle.first_sat(nodes, noff, consts, coff, cands)
    for s in range(B.n_states):
        n0, n1 = int(noff[s]), int(noff[s + 1])
        nl = [[int(r[f]) for f in ("op", "width", "a", "b", "c", "p0", "p1")] for r in nodes[n0:n1]]
        cl = [S.limbs_to_int(c) for c in consts[int(coff[s]):int(coff[s + 1])]]
        rows = [[S.limbs_to_int(cands[s, k, v]) for v in range(nv)] for k in range(12)]
        assert got[s] == S.first_sat(nl, cl, rows), s
    B.close()


def test_uf_symbolic_base_offsets_fold():
    """Selects at base + constant (a calldata word at a symbolic ABI offset): two indices
    of one base compare by their constant offsets at lowering time (mod 2^256, nested
    sums flattened), so only selects of different bases are tested at run time."""
    F = 4
    nl = [[S.VAR, 256, -1, -1, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0]]     # B, y
    consts = [4, 36, 2 ** 256 - 1, 0]
    nl += [[S.CONST, 256, -1, -1, -1, k, 0] for k in range(4)]               # 2..5
    nl.append([S.ADD, 256, 2, 0, -1, 0, 0])                                   # 6: 4 + B
    nl.append([S.ADD, 256, 3, 0, -1, 0, 0])                                   # 7: 36 + B
    apps, fresh = [], 10
    for base in (6, 7):
        for i in range(0, 40, 3):
            nl.append([S.CONST, 256, -1, -1, -1, len(consts), 0])
            consts.append(i)
            nl.append([S.ADD, 256, base, len(nl) - 1, -1, 0, 0])             # (c + B) + i
            nl.append([S.UFAPP, 8, len(nl) - 1, -1, -1, F, fresh])
            fresh += 1
            apps.append(len(nl) - 1)
    nl.append([S.ADD, 256, 0, 4, -1, 0, 0])                                   # B + (2^256 - 1) = B - 1
    nl.append([S.UFAPP, 8, len(nl) - 1, -1, -1, F, fresh])
    apps.append(len(nl) - 1)
    nl.append([S.UFAPP, 8, 1, -1, -1, F, fresh + 1])                          # f(y): unknown vs all
    apps.append(len(nl) - 1)
    acc = apps[0]
    for a in apps[1:]:
        nl.append([S.XOR, 8, acc, a, -1, 0, 0])
        acc = len(nl) - 1
    nl.append([S.CONST, 8, -1, -1, -1, len(consts), 0])
    consts.append(0x5A)
    nl.append([S.EQ, 1, acc, len(nl) - 1, -1, 0, 0])
    rng = np.random.default_rng(3)
    rows = []
    for _ in range(30):
        b = int(rng.integers(0, 2 ** 62))
        y = b + int(rng.choice([4, 36, 40, 3, 0, 7, 100])) if rng.random() < 0.7 else int(rng.integers(0, 2 ** 62))
        rows.append([b, y] + [0] * 8 + [int(rng.integers(0, 256)) for _ in range(fresh + 2 - 10)])
    words, po, status = _check_states([(nl, consts)], [rows])
    assert status[0] == N.ST_OK
    # every select has base B except f(y): only f(y) is tested against the others at run time
    n_eq = sum(1 for k in range(int(words[0])) if int(words[4 + 4 * k]) & 0xFF == S.EQ)
    assert n_eq <= 2 * len(apps) + 2, n_eq


def test_bool_folds_uop_reference_matches_oracle():
    """The translator's compare -> BAND/BOR (BCOMB) and BNOT -> BAND (BANDN) folds, run
    through the uop reference interpreter, agree with the C oracle (CPU side of
    tests/test_gpu_parity.py::test_bool_folds_vs_oracle)."""
    from oracle import coracle

    from .test_gpu_parity import _bool_fold_states

    rng = np.random.default_rng(78)
    states = _bool_fold_states(rng, 200)
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = N.lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    n_cand = 12
    vals = rng.integers(0, 256, size=(len(states), n_cand, 3))
    cands = np.zeros((len(states), n_cand, 3, 8), np.uint32)
    cands[..., 0] = vals
    ref = coracle.first_sat(nodes, noff, consts, coff, cands)
    folded = 0
    for s in range(len(states)):
        rows = [[int(x) for x in vals[s, k]] for k in range(n_cand)]
        assert UR.first_sat_uops(words, int(po[s]), rows) == ref[s], s
        u0 = UR.uop_offset(words, int(po[s]))
        folded += sum(bool(int(words[u0 + 6 + 4 * k]) & U.F_BCOMB) for k in range(int(words[u0])))
    assert folded > 100


def test_band4n_folds_uop_reference_matches_oracle():
    """BNOTs read by one AND chain fold into BAND4N<mask>; BNOTs read again elsewhere stay.
    The uop reference interpreter agrees with the C oracle on every candidate, and the fold
    fires (CPU side of tests/test_gpu_parity.py::test_band4n_folds_vs_oracle)."""
    from oracle import coracle

    from .test_gpu_parity import _band4n_states

    rng = np.random.default_rng(92)
    states = _band4n_states(rng, 300)
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = N.lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    n_cand = 12
    vals = rng.integers(0, 256, size=(len(states), n_cand, 3))
    cands = np.zeros((len(states), n_cand, 3, 8), np.uint32)
    cands[..., 0] = vals
    ref = coracle.first_sat(nodes, noff, consts, coff, cands)
    names = UR._names()
    folded = kept = 0
    for s in range(len(states)):
        rows = [[int(x) for x in vals[s, k]] for k in range(n_cand)]
        assert UR.first_sat_uops(words, int(po[s]), rows) == ref[s], s
        u0 = UR.uop_offset(words, int(po[s]))
        for k in range(int(words[u0])):
            nm = names[int(words[u0 + 4 + 4 * k]) & 0xFFFF]
            folded += nm.startswith("BAND4N")
            kept += nm == "BNOT"
    assert folded > 50 and kept > 0, (folded, kept)


def test_band4n_then_hbm_variable_loads_uop_reference():
    """a compare that reads an HBM variable (index >= 6) after a folded BAND4N
    chain.  The uop reference once rebound its candidate row inside the BAND4N branch, so
    every later VAR load read the chain's four Bools; this case fails on that code."""
    from oracle import coracle

    from .test_gpu_parity import _band4n_states

    rng = np.random.default_rng(94)
    states = _band4n_states(rng, 200, late_vars=6)
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = N.lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    n_cand = 12
    vals = rng.integers(0, 256, size=(len(states), n_cand, 9))
    cands = np.zeros((len(states), n_cand, 9, 8), np.uint32)
    cands[..., 0] = vals
    ref = coracle.first_sat(nodes, noff, consts, coff, cands)
    names = UR._names()
    hit = 0
    for s in range(len(states)):
        rows = [[int(x) for x in vals[s, k]] for k in range(n_cand)]
        assert UR.first_sat_uops(words, int(po[s]), rows) == ref[s], s
        u0 = UR.uop_offset(words, int(po[s]))
        seen = False
        for k in range(int(words[u0])):
            nm = names[int(words[u0 + 4 + 4 * k]) & 0xFFFF]
            seen |= nm.startswith("BAND4N")
            hit += seen and "_var_" in nm
    assert hit > 20, hit


def test_select_chain_fusions_uop_reference_matches_oracle():
    """Select chains (EQ + ITE pairs over one key) fused into EQSEL / TSEL / TSELS uops: the
    uop reference interpreter agrees with the C oracle on every candidate, and each fusion
    fires (CPU side of tests/test_gpu_parity.py::test_select_chain_fusions_vs_oracle)."""
    from oracle import coracle

    from .test_gpu_parity import _select_chain_cands, _select_chain_states

    rng = np.random.default_rng(516)
    states = _select_chain_states(rng, 60)
    nodes, noff, consts, coff = pack_states(states)
    words, po, status = N.lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    cands = _select_chain_cands(rng, states, 16)
    ref = coracle.first_sat(nodes, noff, consts, coff, cands)
    names = UR._names()
    seen = {"EQSEL": 0, "TSEL": 0, "TSELS": 0, "row keys": 0}
    for s in range(len(states)):
        rows = [[S.limbs_to_int(cands[s, k, v]) for v in range(cands.shape[2])] for k in range(cands.shape[1])]
        assert UR.first_sat_uops(words, int(po[s]), rows) == ref[s], s
        u0 = UR.uop_offset(words, int(po[s]))
        pool0 = u0 + int(words[u0 + 2]) // 4
        for k in range(int(words[u0])):
            w0, w3 = int(words[u0 + 4 + 4 * k]), int(words[u0 + 7 + 4 * k])
            nm = names[w0 >> 16]
            if nm.startswith("EQSEL"):
                seen["EQSEL"] += 1
            elif nm in seen:
                seen[nm] += 1
            if nm == "TSELS":  # entries whose key is a candidate-row variable (word bit 30)
                t0 = pool0 + 2 * (w3 >> 16)
                seen["row keys"] += sum((int(words[t0 + 2 * i]) >> 30) == 1 for i in range(w3 & 0xFFFF))
    assert all(v > 10 for v in seen.values()), seen
    assert 0 < (ref >= 0).sum() < len(states) or (ref > 0).sum() > 5


def test_contract_select_tables_uop_reference():
    """WalletLibrary's calldata byte tables (TSEL) and symbolic-index Store chains (TSELS)
    through the uop reference interpreter, against the C oracle."""
    import corpus
    from corpus.keccak_manager import KeccakFunctionManager
    from mythril_amd import dag as D
    from mythril_amd import front as F
    from oracle import coracle

    kfm = KeccakFunctionManager()
    items = corpus.wallet_states(0, kfm)[:3]
    B = F.Batch([list(c[1]) for c in items])
    nv = B.n_vars()
    _, dom = N.refute_domains(*B.packed(), B.var_off)
    cands = N.make_candidates(8, nv, 7, B.var_off, B.var_width, B.hint_off, B.hints, B.alias_off, B.aliases,
                              B.const_off, B.consts, D._FIXED_LIMBS, np.zeros(B.n_states, np.uint8),
                              var_kind=B.var_kind, dom=dom)
    nodes, noff, consts, coff = B.packed(gpu=True)
    ref = coracle.first_sat(nodes, noff, consts, coff, cands)
    words, po, status = N.lower(nodes, noff, consts, coff)
    names = UR._names()
    for s in range(B.n_states):
        rows = [[S.limbs_to_int(cands[s, k, v]) for v in range(nv)] for k in range(8)]
        assert UR.first_sat_uops(words, int(po[s]), rows) == ref[s], s
        u0 = UR.uop_offset(words, int(po[s]))
        ops = [names[int(words[u0 + 4 + 4 * k]) >> 16] for k in range(int(words[u0]))]
        assert ops.count("TSEL") > 10 and ops.count("TSELS") > 10, s
    B.close()


def test_uf_byte_tables_both_references_match_oracle():
    """UF chains lowered as v1 EQSEL steps whose selected fresh values are read unmasked
    (EQSEL masks them): the bytecode and uop reference interpreters agree with the oracle on
    candidates with garbage above the 8-bit values; TSEL and TSELS runs fire."""
    from .test_gpu_parity import _uf_byte_table_cands, _uf_byte_table_states

    rng = np.random.default_rng(920)
    states = _uf_byte_table_states(rng, 40)
    cands = _uf_byte_table_cands(rng, states, 12)
    rows = [[[S.limbs_to_int(cands[s, k, v]) for v in range(cands.shape[2])] for k in range(cands.shape[1])]
            for s in range(len(states))]
    words, po, status = _check_states(states, rows)
    assert (status == 0).all()
    names = UR._names()
    seen = set()
    n_eqsel = 0
    for s in range(len(states)):
        o = int(po[s])
        n_eqsel += sum(int(words[o + 4 + 4 * k]) & 0xFF == 81 for k in range(int(words[o])))
        u0 = UR.uop_offset(words, o)
        seen |= {names[int(words[u0 + 4 + 4 * k]) >> 16] for k in range(int(words[u0]))}
    assert n_eqsel > 100 and {"TSEL", "TSELS"} <= seen, (n_eqsel, sorted(seen)[:20])
