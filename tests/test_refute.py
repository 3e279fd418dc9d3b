"""UNSAT pre-check (mgp_refute, host C++) vs the oracle — CPU only.

mgp_refute claims "no assignment satisfies the state" (it replaces the z3
call behind Constraints.is_possible, constraints.py:34-51, for the states it
decides).  A claim is only useful if it is never wrong, so the tests check
soundness against oracle.bvsem / oracle.coracle:

* node by node: for a satisfying assignment, every node's concrete value lies
  inside the abstract value the refuter ends with (known bits and interval),
  and the state is not refuted;
* state by state: no refuted state has a model — exhaustively over all
  assignments for random small-width DAGs over the whole operator set, and by
  candidate search (planted witnesses included) on the synthetic batch;
* hand-written contradictions of the kinds LASER produces are refuted.
"""
import numpy as np
import pytest

from mythril_amd import _native as N
from oracle import bvsem as S
from oracle import coracle

from ._util import node_array, pack_states, random_cands, state_slice

X0 = [S.VAR, 256, -1, -1, -1, 0, 0]
X1 = [S.VAR, 256, -1, -1, -1, 1, 0]


def _refute(states, max_passes=0):
    nodes, noff, consts, coff = pack_states(states)
    return N.refute(nodes, noff, consts, coff, max_passes=max_passes)


def _contains(av_row, v, w, is_bool):
    if is_bool:
        return bool(av_row[32] & (2 if v else 1))
    z = S.limbs_to_int(av_row[0:8])
    o = S.limbs_to_int(av_row[8:16])
    lo = S.limbs_to_int(av_row[16:24])
    hi = S.limbs_to_int(av_row[24:32])
    return (v & z) == 0 and (v & o) == o and lo <= v <= hi and v <= S.mask(w)


def _check_contained(nodes, consts, xs):
    """xs satisfies the root -> not refuted and every node value inside its abstract value."""
    vals = S.eval_dag(nodes, consts, xs)
    assert vals[-1], "test bug: assignment does not satisfy the root"
    arr = nodes if isinstance(nodes, np.ndarray) else node_array(nodes)
    climbs = np.array([S.int_to_limbs(c) for c in consts], dtype=np.uint32).reshape(-1, 8)
    r, av = N.refute_trace(arr, climbs)
    assert r == 0, "refuted a satisfiable state"
    for i, v in enumerate(vals):
        isb = isinstance(v, bool)
        w = 1 if isb else int(arr[i]["width"])
        assert _contains(av[i], v, w, isb), (i, int(arr[i]["op"]), v)


# ------------------------------------------------------------ hand cases
def _st(extra_nodes, consts):
    return ([X0, X1] + extra_nodes, consts)


UNSAT_CASES = {
    # x == 5 and x == 6
    "eq_eq": _st([[S.CONST, 256, -1, -1, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 1, 0],
                  [S.EQ, 1, 0, 2, -1, 0, 0], [S.EQ, 1, 0, 3, -1, 0, 0], [S.BAND, 1, 4, 5, -1, 0, 0]], [5, 6]),
    # x <u 3 and x >u 5
    "ult_ugt": _st([[S.CONST, 256, -1, -1, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 1, 0],
                    [S.ULT, 1, 0, 2, -1, 0, 0], [S.UGT, 1, 0, 3, -1, 0, 0], [S.BAND, 1, 4, 5, -1, 0, 0]], [3, 5]),
    # (x & 1) == 1 and (x & 1) == 0
    "and_bit": _st([[S.CONST, 256, -1, -1, -1, 0, 0], [S.AND, 256, 0, 2, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 1, 0],
                    [S.EQ, 1, 3, 2, -1, 0, 0], [S.EQ, 1, 3, 4, -1, 0, 0], [S.BAND, 1, 5, 6, -1, 0, 0]], [1, 0]),
    # x + 1 == 0 (x = 2^256 - 1) and x <u 10
    "add_wrap": _st([[S.CONST, 256, -1, -1, -1, 0, 0], [S.ADD, 256, 0, 2, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 1, 0],
                     [S.EQ, 1, 3, 4, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 2, 0], [S.ULT, 1, 0, 6, -1, 0, 0],
                     [S.BAND, 1, 5, 7, -1, 0, 0]], [1, 0, 10]),
    # Extract(7, 0, x) == 0x41 and x == 0x42
    "extract": _st([[S.EXTRACT, 8, 0, -1, -1, 7, 0], [S.CONST, 8, -1, -1, -1, 0, 0], [S.EQ, 1, 2, 3, -1, 0, 0],
                    [S.CONST, 256, -1, -1, -1, 1, 0], [S.EQ, 1, 0, 5, -1, 0, 0], [S.BAND, 1, 4, 6, -1, 0, 0]],
                   [0x41, 0x42]),
    # Not(BVAddNoOverflow(x, y, False)) with x <u 10 and y <u 10
    "addnoovf": _st([[S.UADD_NOOVF, 1, 0, 1, -1, 0, 0], [S.BNOT, 1, 2, -1, -1, 0, 0],
                     [S.CONST, 256, -1, -1, -1, 0, 0], [S.ULT, 1, 0, 4, -1, 0, 0], [S.ULT, 1, 1, 4, -1, 0, 0],
                     [S.BAND, 1, 3, 5, -1, 0, 0], [S.BAND, 1, 7, 6, -1, 0, 0]], [10]),
    # jumpi pair: cond and Not(cond) on one path (instructions.py:1556-1562)
    "jumpi_pair": _st([[S.CONST, 256, -1, -1, -1, 0, 0], [S.SUB, 256, 0, 1, -1, 0, 0], [S.EQ, 1, 3, 2, -1, 0, 0],
                       [S.BNOT, 1, 4, -1, -1, 0, 0], [S.BAND, 1, 4, 5, -1, 0, 0]], [0]),
    # calldatasize bound vs byte index: size <u 4 and 35 <u size
    "calldata": _st([[S.CONST, 256, -1, -1, -1, 0, 0], [S.ULT, 1, 0, 2, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 1, 0],
                     [S.ULT, 1, 4, 0, -1, 0, 0], [S.BAND, 1, 3, 5, -1, 0, 0]], [4, 35]),
    # signed: x <s 0 and x >=u 0 and Extract(255,255,x) == 0
    "signed": _st([[S.CONST, 256, -1, -1, -1, 0, 0], [S.SLT, 1, 0, 2, -1, 0, 0], [S.EXTRACT, 1, 0, -1, -1, 255, 255],
                   [S.CONST, 1, -1, -1, -1, 0, 0], [S.EQ, 1, 4, 5, -1, 0, 0], [S.BAND, 1, 3, 6, -1, 0, 0]], [0]),
    # ITE: If(x == 1, 7, 9) == 8
    "ite": _st([[S.CONST, 256, -1, -1, -1, 0, 0], [S.EQ, 1, 0, 2, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 1, 0],
                [S.CONST, 256, -1, -1, -1, 2, 0], [S.ITE, 256, 3, 4, 5, 0, 0], [S.CONST, 256, -1, -1, -1, 3, 0],
                [S.EQ, 1, 6, 7, -1, 0, 0]], [1, 7, 9, 8]),
    # shift: LShR(x, 248) == 0x1ff (the result has at most 8 bits)
    "lshr": _st([[S.CONST, 256, -1, -1, -1, 0, 0], [S.LSHR, 256, 0, 2, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 1, 0],
                 [S.EQ, 1, 3, 4, -1, 0, 0]], [248, 0x1FF]),
    # Concat(x8, y8) == 0x1234 and x8 == 0x13 (8-bit vars)
    "concat": ([[S.VAR, 8, -1, -1, -1, 0, 0], [S.VAR, 8, -1, -1, -1, 1, 0], [S.CONCAT, 16, 0, 1, -1, 0, 0],
                [S.CONST, 16, -1, -1, -1, 0, 0], [S.EQ, 1, 2, 3, -1, 0, 0], [S.CONST, 8, -1, -1, -1, 1, 0],
                [S.EQ, 1, 0, 5, -1, 0, 0], [S.BAND, 1, 4, 6, -1, 0, 0]], [0x1234, 0x13]),
    # literal false
    "false": ([[S.FALSE, 1, -1, -1, -1, 0, 0]], []),
    # SafeMath.sub after its assert: amount <= bal and Not(BVSubNoUnderflow(bal, amount)), amount = x0 * x1
    "sub_atoms": ([X0, X1, [S.VAR, 256, -1, -1, -1, 2, 0], [S.MUL, 256, 0, 1, -1, 0, 0], [S.ULE, 1, 3, 2, -1, 0, 0],
                   [S.USUB_NOUDF, 1, 2, 3, -1, 0, 0], [S.BNOT, 1, 5, -1, -1, 0, 0], [S.BAND, 1, 4, 6, -1, 0, 0]], []),
    # the same query as the smt mirror builds it: UGE/ULE as Or(strict, ==) (bitvec_helper.py:53-80)
    "sub_or_expansion": ([[S.VAR, 256, -1, -1, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 0, 0], [S.UGT, 1, 0, 1, -1, 0, 0],
                          [S.CONST, 256, -1, -1, -1, 1, 0], [S.ULT, 1, 0, 3, -1, 0, 0], [S.EQ, 1, 0, 3, -1, 0, 0],
                          [S.BOR, 1, 4, 5, -1, 0, 0], [S.VAR, 256, -1, -1, -1, 1, 0], [S.UGT, 1, 7, 1, -1, 0, 0],
                          [S.VAR, 256, -1, -1, -1, 2, 0], [S.MUL, 256, 0, 7, -1, 0, 0], [S.UGT, 1, 9, 10, -1, 0, 0],
                          [S.EQ, 1, 9, 10, -1, 0, 0], [S.BOR, 1, 11, 12, -1, 0, 0], [S.ULT, 1, 10, 9, -1, 0, 0],
                          [S.EQ, 1, 10, 9, -1, 0, 0], [S.BOR, 1, 14, 15, -1, 0, 0], [S.USUB_NOUDF, 1, 9, 10, -1, 0, 0],
                          [S.BNOT, 1, 17, -1, -1, 0, 0], [S.BAND, 1, 2, 6, -1, 0, 0], [S.BAND, 1, 19, 8, -1, 0, 0],
                          [S.BAND, 1, 20, 13, -1, 0, 0], [S.BAND, 1, 21, 16, -1, 0, 0], [S.BAND, 1, 22, 18, -1, 0, 0]],
                         [0, 20]),
    # x0 <=u x1 and x1 <=u x0 and x0 == 3 and x1 == 4 (equal by order, different by value)
    "order_eq": _st([[S.ULE, 1, 0, 1, -1, 0, 0], [S.UGE, 1, 0, 1, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 0, 0],
                     [S.EQ, 1, 0, 4, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 1, 0], [S.EQ, 1, 1, 6, -1, 0, 0],
                     [S.BAND, 1, 2, 3, -1, 0, 0], [S.BAND, 1, 8, 5, -1, 0, 0], [S.BAND, 1, 9, 7, -1, 0, 0]], [3, 4]),
    # x0 <s x1 and x0 >=s x1 (no ranges involved)
    "signed_atoms": _st([[S.SLT, 1, 0, 1, -1, 0, 0], [S.SGE, 1, 0, 1, -1, 0, 0], [S.BAND, 1, 2, 3, -1, 0, 0]], []),
    # x0 == x1 and Not(x1 == x0)
    "eq_atoms": _st([[S.EQ, 1, 0, 1, -1, 0, 0], [S.EQ, 1, 1, 0, -1, 0, 0], [S.BNOT, 1, 3, -1, -1, 0, 0],
                     [S.BAND, 1, 2, 4, -1, 0, 0]], []),
}

SAT_CASES = {
    "eq_lt": (_st([[S.CONST, 256, -1, -1, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 1, 0], [S.EQ, 1, 0, 2, -1, 0, 0],
                   [S.ULT, 1, 0, 3, -1, 0, 0], [S.BAND, 1, 4, 5, -1, 0, 0]], [5, 6]), [5, 0]),
    "concat": (([[S.VAR, 8, -1, -1, -1, 0, 0], [S.VAR, 8, -1, -1, -1, 1, 0], [S.CONCAT, 16, 0, 1, -1, 0, 0],
                 [S.CONST, 16, -1, -1, -1, 0, 0], [S.EQ, 1, 2, 3, -1, 0, 0]], [0x1234]), [0x12, 0x34]),
    "mul_noovf": (_st([[S.UMUL_NOOVF, 1, 0, 1, -1, 0, 0], [S.BNOT, 1, 2, -1, -1, 0, 0]], []), [1 << 200, 1 << 100]),
    "sdiv": (_st([[S.SDIV, 256, 0, 1, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 0, 0], [S.EQ, 1, 2, 3, -1, 0, 0]],
                 [(1 << 256) - 1]), [5, 0]),
}


@pytest.mark.parametrize("name", sorted(UNSAT_CASES))
def test_refutes_contradictions(name):
    nl, cl = UNSAT_CASES[name]
    assert _refute([(nl, cl)])[0] == 1


@pytest.mark.parametrize("name", sorted(SAT_CASES))
def test_keeps_satisfiable(name):
    (nl, cl), xs = SAT_CASES[name]
    assert S.eval_root(nl, cl, xs)
    assert _refute([(nl, cl)])[0] == 0
    _check_contained(nl, cl, xs)


def test_unsupported_and_empty():
    bad = ([[S.ADD, 256, 3, 4, -1, 0, 0]], [])
    out = _refute([bad, UNSAT_CASES["eq_eq"]])
    assert list(out) == [-1, 1]
    nodes, noff, consts, coff = pack_states([])
    assert N.refute(nodes, noff, consts, coff).size == 0


def test_wide_values_are_relaxed_soundly():
    """512-bit mapping preimages (include/mgp_ir.h "wide values") are relaxed to fresh
    variables and then tied back piecewise (mgp_refute.cpp piece expansion, round 5): the
    narrow contradiction next to them is refuted, a contradiction that runs through the
    pieces of a wide equality is refuted too, and the satisfiable case is not."""
    # Concat(x0, 0) as keccak256_512 argument, inverse result compared with the preimage
    mapping = [X0, X1, [S.CONST, 256, -1, -1, -1, 0, 0], [S.CONCAT, 512, 0, 2, -1, 0, 0],
               [S.UFAPP, 256, 3, -1, -1, 9, 2], [S.UFINV, 512, 4, -1, -1, 9, 3], [S.EQ, 1, 5, 3, -1, 0, 0],
               [S.EXTRACT, 256, 5, -1, -1, 511, 256], [S.EQ, 1, 7, 1, -1, 0, 0]]          # 6, 8
    unsat = mapping + [[S.CONST, 256, -1, -1, -1, 1, 0], [S.ULT, 1, 0, 9, -1, 0, 0],      # x0 <u 5
                       [S.UGT, 1, 0, 9, -1, 0, 0], [S.BAND, 1, 6, 10, -1, 0, 0],          # x0 >u 5
                       [S.BAND, 1, 12, 11, -1, 0, 0], [S.BAND, 1, 13, 8, -1, 0, 0]]
    sat = mapping + [[S.CONST, 256, -1, -1, -1, 1, 0], [S.ULT, 1, 0, 9, -1, 0, 0],
                     [S.BAND, 1, 6, 10, -1, 0, 0], [S.BAND, 1, 11, 8, -1, 0, 0]]
    # contradictory only through the wide part (inv == Concat(x0, 0) but its high word
    # != x0): the piece expansion equates inv's high piece with x0 and refutes it
    wide_only = mapping + [[S.EQ, 1, 7, 0, -1, 0, 0], [S.BNOT, 1, 9, -1, -1, 0, 0], [S.BAND, 1, 6, 10, -1, 0, 0]]
    out = _refute([(unsat, [0, 5]), (sat, [0, 5]), (wide_only, [0, 5]),
                   ([[S.VAR, 512, -1, -1, -1, 0, 0], [S.EQ, 1, 0, 0, -1, 0, 0]], [])])
    assert list(out) == [1, 0, 1, 0]
    # sat: x0 = 1, x1 = x0 (the inverse returns the preimage), fresh values unused
    xs = [1, 1, 77, 0, 0, 0]
    assert S.eval_root(sat, [0, 5], xs)


# ------------------------------------------- exhaustive small-width DAGs
def _random_small_dag(rng, w=4, n_ops=10):
    """Random DAG over two w-bit vars using the whole operator set; root = AND of 2-3 Bools."""
    nodes, consts = [[S.VAR, w, -1, -1, -1, 0, 0], [S.VAR, w, -1, -1, -1, 1, 0]], []
    bv = {w: [0, 1]}
    bools = []

    def const(width):
        consts.append(int(rng.integers(0, 1 << width)))
        nodes.append([S.CONST, width, -1, -1, -1, len(consts) - 1, 0])
        bv.setdefault(width, []).append(len(nodes) - 1)
        return len(nodes) - 1

    def pick(width):
        pool = bv.get(width, [])
        if not pool or rng.random() < 0.2:
            return const(width)
        return int(pool[int(rng.integers(len(pool)))])

    binops = [S.ADD, S.SUB, S.MUL, S.UDIV, S.UREM, S.SDIV, S.SREM, S.SMOD, S.AND, S.OR, S.XOR, S.SHL, S.LSHR, S.ASHR]
    cmps = [S.EQ, S.ULT, S.ULE, S.UGT, S.UGE, S.SLT, S.SLE, S.SGT, S.SGE, S.UADD_NOOVF, S.UMUL_NOOVF, S.USUB_NOUDF]
    h = w // 2
    for _ in range(n_ops):
        k = rng.random()
        if k < 0.40:
            op = binops[int(rng.integers(len(binops)))]
            a, b = pick(w), pick(w)
            nodes.append([op, w, a, b, -1, 0, 0])
            bv[w].append(len(nodes) - 1)
        elif k < 0.48:
            nodes.append([[S.NOT, S.NEG][int(rng.integers(2))], w, pick(w), -1, -1, 0, 0])
            bv[w].append(len(nodes) - 1)
        elif k < 0.56:
            lo = int(rng.integers(0, w - h + 1))
            nodes.append([S.EXTRACT, h, pick(w), -1, -1, lo + h - 1, lo])
            bv.setdefault(h, []).append(len(nodes) - 1)
        elif k < 0.64:
            op = [S.ZEXT, S.SEXT, S.CONCAT][int(rng.integers(3))]
            if op == S.CONCAT:
                nodes.append([S.CONCAT, w, pick(w - h), pick(h), -1, 0, 0])
            else:
                nodes.append([op, w, pick(h), -1, -1, 0, 0])
            bv[w].append(len(nodes) - 1)
        elif k < 0.70 and bools:
            c = bools[int(rng.integers(len(bools)))]
            nodes.append([S.ITE, w, c, pick(w), pick(w), 0, 0])
            bv[w].append(len(nodes) - 1)
        elif k < 0.92:
            op = cmps[int(rng.integers(len(cmps)))]
            nodes.append([op, 1, pick(w), pick(w), -1, 0, 0])
            bools.append(len(nodes) - 1)
        elif bools:
            op = [S.BAND, S.BOR, S.BXOR, S.BNOT, S.BEQ, S.BITE][int(rng.integers(6))]
            a = bools[int(rng.integers(len(bools)))]
            b = bools[int(rng.integers(len(bools)))]
            c = bools[int(rng.integers(len(bools)))]
            if op == S.BNOT:
                nodes.append([op, 1, a, -1, -1, 0, 0])
            elif op == S.BITE:
                nodes.append([op, 1, a, b, c, 0, 0])
            else:
                nodes.append([op, 1, a, b, -1, 0, 0])
            bools.append(len(nodes) - 1)
    while len(bools) < 2:
        nodes.append([cmps[int(rng.integers(len(cmps)))], 1, pick(w), pick(w), -1, 0, 0])
        bools.append(len(nodes) - 1)
    root = bools[-1]
    for b in bools[-3:-1]:
        nodes.append([S.BAND, 1, root, b, -1, 0, 0])
        root = len(nodes) - 1
    return nodes, consts


@pytest.mark.parametrize("w", [4, 6])
def test_exhaustive_small_width_soundness(w):
    rng = np.random.default_rng(0xBADC0DE + w)
    n = 500 if w == 4 else 160
    states = [_random_small_dag(rng, w=w, n_ops=int(rng.integers(4, 14))) for _ in range(n)]
    verdict = _refute(states)
    refuted = 0
    space = [(x, y) for x in range(1 << w) for y in range(1 << w)]
    for (nl, cl), r in zip(states, verdict):
        assert r in (0, 1)
        models = [xs for xs in space if S.eval_root(nl, cl, xs)]
        if r == 1:
            refuted += 1
            assert not models, "refuted a satisfiable state"
        else:
            for xs in models[:: max(1, len(models) // 3)]:
                _check_contained(nl, cl, xs)
    assert refuted > n // 20  # the pass decides a real share of these


# ------------------------------------------------------- synthetic batch
def test_synthetic_witnesses_inside_abstract_values():
    b = N.synth_generate(0x4D595448, 7, 120, 64, 16)
    checked = 0
    for s in range(120):
        if not b["planted"][s]:
            continue
        nodes, consts = state_slice(b, s)
        _check_contained(nodes, consts, [S.limbs_to_int(x) for x in b["plant_words"][s]])
        checked += 1
    assert checked > 30


def test_synthetic_batch_no_refuted_state_has_a_model():
    n_states, n_cand = 4096, 64
    b = N.synth_generate(0x4D595448, 1 << 20, n_states, 64, n_cand)
    verdict = N.refute(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
    assert set(np.unique(verdict)) <= {0, 1}
    assert not verdict[b["planted"].astype(bool)].any()
    cands = random_cands(np.random.default_rng(3), n_states, n_cand, b["n_vars"])
    for s in range(n_states):
        if b["planted"][s]:
            cands[s, b["plant_idx"][s]] = b["plant_words"][s]
    first = coracle.first_sat(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"], cands)
    assert not ((verdict == 1) & (first >= 0)).any()


# ------------------------------------------------- domain-guided candidates
def test_guided_candidates_decisions_solve_linked_vars():
    # x0 + x1 == 1000 and x0 <u 10: uniform draws never satisfy this; deciding x0 inside
    # [0, 9] and re-running the analysis fixes x1 = 1000 - x0
    nl = [X0, X1, [S.ADD, 256, 0, 1, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 0, 0], [S.EQ, 1, 2, 3, -1, 0, 0],
          [S.CONST, 256, -1, -1, -1, 1, 0], [S.ULT, 1, 0, 5, -1, 0, 0], [S.BAND, 1, 4, 6, -1, 0, 0]]
    cl = [1000, 10]
    nodes, noff, consts, coff = pack_states([(nl, cl)])
    rng = np.random.default_rng(3)
    cands = random_cands(rng, 1, 32, 2)
    before = cands.copy()
    st = N.guided_candidates(nodes, noff, consts, coff, cands, seed=1, every=2, n_decide=4)
    assert st[0] == 0
    assert np.array_equal(cands[:, 1::2], before[:, 1::2]), "rows outside the guided set are left alone"
    rows = [[S.limbs_to_int(cands[0, c, v]) for v in range(2)] for c in range(0, 32, 2)]
    hits = [S.eval_root(nl, cl, r) for r in rows]
    assert all(hits[:4]), rows[:4]        # every decision row is a model here
    assert all(r[0] < 10 for r in rows)   # every guided row lies in the refined domain of x0
    again = before.copy()
    N.guided_candidates(nodes, noff, consts, coff, again, seed=1, every=2, n_decide=4)
    assert np.array_equal(again, cands), "deterministic in the seed"


def test_guided_candidates_rows_per_state():
    """mgp_guided_candidates_rows: a state given r decision rows gets exactly the rows a
    call with n_decide = r writes (decision rows first, plain domain draws after), and
    every state's rows are independent of the other states' counts."""
    b = N.synth_generate(0x5EED, 0, 24, 48, 32)
    nodes, noff, consts, coff = b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"]
    base = random_cands(np.random.default_rng(9), 24, 32, b["n_vars"])
    full, four, mixed = base.copy(), base.copy(), base.copy()
    st8 = N.guided_candidates(nodes, noff, consts, coff, full, seed=3, every=2, n_decide=8)
    st4 = N.guided_candidates(nodes, noff, consts, coff, four, seed=3, every=2, n_decide=4)
    rows = np.array([8 if s % 2 else 4 for s in range(24)], np.uint8)
    stm = N.guided_candidates(nodes, noff, consts, coff, mixed, seed=3, every=2, n_decide=8, rows_per_state=rows)
    assert np.array_equal(st8, st4) and np.array_equal(st8, stm)
    for s in range(24):
        want = full[s] if rows[s] == 8 else four[s]
        assert np.array_equal(mixed[s], want), s
    same = base.copy()
    N.guided_candidates(nodes, noff, consts, coff, same, seed=3, every=2, n_decide=8,
                        rows_per_state=np.full(24, 8, np.uint8))
    assert np.array_equal(same, full)


def test_guided_candidates_status_and_yield_on_synthetic():
    b = N.synth_generate(0x4D595448, 0, 768, 64, 256)
    nodes, noff, consts, coff = b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"]
    nv = b["n_vars"]
    rng = np.random.default_rng(5)
    uni = random_cands(rng, 768, 64, nv, 0.25)
    gd = uni.copy()
    st = N.guided_candidates(nodes, noff, consts, coff, gd, seed=7, every=1, n_decide=16)
    assert np.array_equal(st, N.refute(nodes, noff, consts, coff))
    f_uni = coracle.first_sat(nodes, noff, consts, coff, uni)
    f_gd = coracle.first_sat(nodes, noff, consts, coff, gd)
    assert not ((f_gd >= 0) & (st == 1)).any()
    # the guided rows find witnesses the same number of uniform rows misses
    assert ((f_gd >= 0) & (f_uni < 0)).sum() > 2 * max(1, ((f_uni >= 0) & (f_gd < 0)).sum())


def test_refute_domains_agree_with_refute_and_contain_witnesses():
    """mgp_refute_domains: the same verdicts as mgp_refute, and every planted witness value
    of a non-refuted synthetic state lies inside its variable's exported domain (the
    domains are sound over-approximations, so domain rows never exclude a model)."""
    from mythril_amd import _native as N

    b = N.synth_generate(0x4D595448, 777, 512, 64, 256)
    n = 512
    var_off = np.arange(n + 1, dtype=np.uint64) * b["n_vars"]
    st, dom = N.refute_domains(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"], var_off)
    assert np.array_equal(st, N.refute(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"]))
    checked = 0
    for s in np.nonzero(b["planted"])[0]:
        assert st[s] != 1
        for v in range(b["n_vars"]):
            d = dom[s * b["n_vars"] + v]
            if not d[32]:
                continue
            limb = lambda a: int.from_bytes(np.ascontiguousarray(a).tobytes(), "little")
            z, o, lo, hi = limb(d[0:8]), limb(d[8:16]), limb(d[16:24]), limb(d[24:32])
            x = limb(b["plant_words"][s, v])
            # UF slots hold fresh values that the planted row may not use: check VAR slots only
            if v >= 4:
                continue
            x &= (1 << 256) - 1
            assert lo <= x <= hi and x & z == 0 and x & o == o, (s, v)
            checked += 1
    assert checked > 100


# ------------------------------------------------- UF congruence (pair ties)
def test_uf_congruence_refutes_equal_keys_with_different_values():
    """f(Concat(a, c)) and f(Concat(b, c)) with a == b asserted have equal values (the
    Ackermann axiom of include/mgp_ir.h UFAPP): asserting the values differ is refuted
    (WalletLibrary: the tx-2 sender equal to the initializer reads m_ownerIndex[sender] != 0,
    corpus.py "wallet:initializer not owner"); without a == b it stays open; with the
    arguments structurally different (c vs c') nothing is concluded."""
    A_, B_ = X0, X1
    C0 = [S.CONST, 256, -1, -1, -1, 0, 0]
    C1 = [S.CONST, 256, -1, -1, -1, 1, 0]
    base = [A_, B_, C0, C1,
            [S.CONCAT, 512, 0, 2, -1, 0, 0], [S.CONCAT, 512, 1, 2, -1, 0, 0],      # 4, 5
            [S.UFAPP, 256, 4, -1, -1, 9, 2], [S.UFAPP, 256, 5, -1, -1, 9, 3],      # 6, 7
            [S.EQ, 1, 6, 7, -1, 0, 0], [S.BNOT, 1, 8, -1, -1, 0, 0]]               # 8, 9
    eq_ab = base + [[S.EQ, 1, 0, 1, -1, 0, 0], [S.BAND, 1, 9, 10, -1, 0, 0]]
    free = base + [[S.ULT, 1, 0, 3, -1, 0, 0], [S.BAND, 1, 9, 10, -1, 0, 0]]
    # the keys differ in their constant part: f-values may differ even when a == b
    other = [A_, B_, C0, C1, [S.CONCAT, 512, 0, 2, -1, 0, 0], [S.CONCAT, 512, 1, 3, -1, 0, 0],
             [S.UFAPP, 256, 4, -1, -1, 9, 2], [S.UFAPP, 256, 5, -1, -1, 9, 3],
             [S.EQ, 1, 6, 7, -1, 0, 0], [S.BNOT, 1, 8, -1, -1, 0, 0],
             [S.EQ, 1, 0, 1, -1, 0, 0], [S.BAND, 1, 9, 10, -1, 0, 0]]
    # the value equality reached through a read-over-write ITE (value must be 0, the
    # stored value at the equal key is 1)
    row = base[:8] + [[S.EQ, 1, 6, 7, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 2, 0],
                      [S.ITE, 256, 8, 9, 1, 0, 0], [S.EQ, 1, 10, 2, -1, 0, 0],     # ITE(k2==k1, 1, b) == 0
                      [S.EQ, 1, 0, 1, -1, 0, 0], [S.BAND, 1, 11, 12, -1, 0, 0]]
    out = _refute([(eq_ab, [0, 7]), (free, [0, 7]), (other, [0, 7]), (row, [0, 7, 1])])
    assert list(out) == [1, 0, 0, 1]
    # free: a != b and different fresh values is a model
    assert S.eval_root(free, [0, 7], [1, 2, 5, 6])


def test_uf_congruence_exhaustive_soundness():
    """Random small DAGs over two 3-bit variables and applications of one UF (direct and
    through Concat arguments) with compares, ITEs and Bool structure: no refuted state
    has a model among every assignment of the variables and the fresh UF values
    (C oracle over all 8^k combinations)."""
    rng = np.random.default_rng(0xC0C0)
    w = 3
    states = []
    for _ in range(160):
        nl = [[S.VAR, w, -1, -1, -1, 0, 0], [S.VAR, w, -1, -1, -1, 1, 0]]
        cl = [int(rng.integers(0, 8)) for _ in range(2)]
        nl += [[S.CONST, w, -1, -1, -1, 0, 0], [S.CONST, w, -1, -1, -1, 1, 0]]
        vals, bools = [0, 1, 2, 3], []
        n_uf = 0
        for _ in range(int(rng.integers(6, 14))):
            k = rng.random()
            if k < 0.35 and n_uf < 3:
                a = int(rng.choice(vals))
                if rng.random() < 0.5:     # f(Concat(x, c)) at twice the width, value w bits
                    nl.append([S.CONCAT, 2 * w, a, int(rng.choice([2, 3])), -1, 0, 0])
                    nl.append([S.UFAPP, w, len(nl) - 1, -1, -1, 5, 2 + n_uf])
                    # (2w-bit argument: the function is keyed by its argument width too)
                    nl[-1][5] = 6
                else:
                    nl.append([S.UFAPP, w, a, -1, -1, 5, 2 + n_uf])
                n_uf += 1
                vals.append(len(nl) - 1)
            elif k < 0.55:
                op = [S.ADD, S.XOR, S.SUB][int(rng.integers(3))]
                nl.append([op, w, int(rng.choice(vals)), int(rng.choice(vals)), -1, 0, 0])
                vals.append(len(nl) - 1)
            elif k < 0.65 and bools:
                nl.append([S.ITE, w, int(rng.choice(bools)), int(rng.choice(vals)), int(rng.choice(vals)), 0, 0])
                vals.append(len(nl) - 1)
            elif k < 0.9:
                op = [S.EQ, S.ULT, S.EQ][int(rng.integers(3))]
                nl.append([op, 1, int(rng.choice(vals)), int(rng.choice(vals)), -1, 0, 0])
                bools.append(len(nl) - 1)
            elif bools:
                nl.append([S.BNOT, 1, int(rng.choice(bools)), -1, -1, 0, 0])
                bools.append(len(nl) - 1)
        while len(bools) < 2:
            nl.append([S.EQ, 1, int(rng.choice(vals)), int(rng.choice(vals)), -1, 0, 0])
            bools.append(len(nl) - 1)
        root = bools[-1]
        for b in bools[-4:-1]:
            nl.append([S.BAND, 1, root, b, -1, 0, 0])
            root = len(nl) - 1
        states.append((nl, cl))
    verdict = _refute(states)
    n_vars = 5
    grid = np.array(np.meshgrid(*[np.arange(8)] * n_vars, indexing="ij")).reshape(n_vars, -1).T  # 32768 x 5
    cands = np.zeros((1, grid.shape[0], n_vars, 8), np.uint32)
    cands[0, :, :, 0] = grid
    refuted = 0
    for (nl, cl), r in zip(states, verdict):
        assert r in (0, 1)
        if r != 1:
            continue
        refuted += 1
        nodes, noff, consts, coff = pack_states([(nl, cl)])
        assert coracle.first_sat(nodes, noff, consts, coff, cands)[0] < 0, "refuted a satisfiable state"
    assert refuted > 10


def _congruence_state(rng, w=3):
    """One random term shape T (two operator levels; an ITE's compare adds one more, within
    the congruence depth kCongDepth = 4) instantiated over x0 and over x1 (compares, ITEs,
    adds, a UF application), with x0 = x1 asserted in one of three forms (EQ, ULE both ways, or not at
    all) and T(x0) vs T(x1) constrained to differ (NE, ULT or UGT)."""
    nl = [[S.VAR, w, -1, -1, -1, 0, 0], [S.VAR, w, -1, -1, -1, 1, 0]]
    cl = [int(x) for x in rng.integers(0, 1 << w, size=3)]
    nl += [[S.CONST, w, -1, -1, -1, k, 0] for k in range(3)]   # nodes 2, 3, 4
    n_uf = [0]

    def shape(depth):
        k = rng.random()
        if depth == 0 or k < 0.2:
            return ("v",) if rng.random() < 0.7 else ("c", int(rng.integers(3)))
        if k < 0.45:
            return (["add", "xor", "sub"][int(rng.integers(3))], shape(depth - 1), shape(depth - 1))
        if k < 0.7:
            return ("ite", int(rng.integers(3)), shape(depth - 1), shape(depth - 1), shape(depth - 1))
        if k < 0.85 and n_uf[0] < 1:
            n_uf[0] += 1
            return ("uf", shape(depth - 1))
        return ("not", shape(depth - 1))

    slots = [2]

    def build(t, v):
        if t[0] == "v":
            return v
        if t[0] == "c":
            return 2 + t[1]
        if t[0] in ("add", "xor", "sub"):
            a, b = build(t[1], v), build(t[2], v)
            nl.append([{"add": S.ADD, "xor": S.XOR, "sub": S.SUB}[t[0]], w, a, b, -1, 0, 0])
        elif t[0] == "ite":   # ITE(ULT(T1, c), T2, T3)
            a = build(t[2], v)
            nl.append([S.ULT, 1, a, 2 + t[1], -1, 0, 0])
            c = len(nl) - 1
            b, d = build(t[3], v), build(t[4], v)
            nl.append([S.ITE, w, c, b, d, 0, 0])
        elif t[0] == "uf":
            a = build(t[1], v)
            nl.append([S.UFAPP, w, a, -1, -1, 5, slots[0]])
            slots[0] += 1
        else:
            a = build(t[1], v)
            nl.append([S.NOT, w, a, -1, -1, 0, 0])
        return len(nl) - 1

    t = shape(2)
    t0, t1 = build(t, 0), build(t, 1)
    conj = []
    form = int(rng.integers(3))
    if form == 0:
        nl.append([S.EQ, 1, 0, 1, -1, 0, 0])
        conj.append(len(nl) - 1)
    elif form == 1:
        nl.append([S.ULE, 1, 0, 1, -1, 0, 0])
        conj.append(len(nl) - 1)
        nl.append([S.ULE, 1, 1, 0, -1, 0, 0])
        conj.append(len(nl) - 1)
    rel = int(rng.integers(3))
    nl.append([[S.EQ, S.ULT, S.UGT][rel], 1, t0, t1, -1, 0, 0])
    if rel == 0:
        nl.append([S.BNOT, 1, len(nl) - 1, -1, -1, 0, 0])
    conj.append(len(nl) - 1)
    if rng.random() < 0.5:   # an unrelated side constraint
        nl.append([S.ULT, 1, 0, 2 + int(rng.integers(3)), -1, 0, 0])
        conj.append(len(nl) - 1)
    root = conj[0]
    for c in conj[1:]:
        nl.append([S.BAND, 1, root, c, -1, 0, 0])
        root = len(nl) - 1
    return nl, cl, form


def test_structural_congruence_refutes_calldata_equal_indices():
    """tests/laser/state/calldata_test.py:79-91 at the DAG level: two symbolic calldata loads
    If(i < size, Select(cd, i), 0) at indices asserted equal cannot differ.  Refuted through
    structural congruence (mgp_domain.h Dom::cong): the two ITEs apply one operator to
    operands known equal (the SLT compares over equal indices, the UF applications of one
    function at equal arguments, the same constant)."""
    w = 256
    nl = [[S.VAR, w, -1, -1, -1, 0, 0], [S.VAR, w, -1, -1, -1, 1, 0], [S.EQ, 1, 0, 1, -1, 0, 0],
          [S.VAR, w, -1, -1, -1, 2, 0], [S.SLT, 1, 0, 3, -1, 0, 0], [S.UFAPP, 8, 0, -1, -1, 0, 3],
          [S.CONST, 8, -1, -1, -1, 0, 0], [S.ITE, 8, 4, 5, 6, 0, 0], [S.SLT, 1, 1, 3, -1, 0, 0],
          [S.UFAPP, 8, 1, -1, -1, 0, 4], [S.ITE, 8, 8, 9, 6, 0, 0], [S.EQ, 1, 7, 10, -1, 0, 0],
          [S.BNOT, 1, 11, -1, -1, 0, 0], [S.BAND, 1, 2, 12, -1, 0, 0]]
    # the same without i == j: satisfiable, kept
    free = [r[:] for r in nl]
    free[2] = [S.ULT, 1, 0, 1, -1, 0, 0]
    # different functions (two calldata arrays): no congruence
    other = [r[:] for r in nl]
    other[9] = [S.UFAPP, 8, 1, -1, -1, 1, 4]
    assert list(_refute([(nl, [0]), (free, [0]), (other, [0])])) == [1, 0, 0]


def test_structural_congruence_exhaustive_soundness():
    """Random shapes T instantiated over x0 and x1 (3-bit), T(x0) and T(x1) constrained to
    differ, x0 = x1 asserted as EQ, as ULE both ways, or not at all: no refuted state has a
    model among every assignment of the variables and the UF's fresh values (C oracle over
    all 8^4 combinations), and the asserted-equal states are mostly refuted."""
    rng = np.random.default_rng(0xC0C1)
    states, forms = [], []
    for _ in range(300):
        nl, cl, form = _congruence_state(rng)
        states.append((nl, cl))
        forms.append(form)
    verdict = _refute(states)
    n_vars = 4
    grid = np.array(np.meshgrid(*[np.arange(8)] * n_vars, indexing="ij")).reshape(n_vars, -1).T
    cands = np.zeros((1, grid.shape[0], n_vars, 8), np.uint32)
    cands[0, :, :, 0] = grid
    refuted = {0: 0, 1: 0, 2: 0}
    for (nl, cl), r, form in zip(states, verdict, forms):
        assert r in (0, 1)
        if r != 1:
            continue
        refuted[form] += 1
        nodes, noff, consts, coff = pack_states([(nl, cl)])
        assert coracle.first_sat(nodes, noff, consts, coff, cands)[0] < 0, "refuted a satisfiable state"
    n_form = {f: forms.count(f) for f in (0, 1)}
    assert refuted[0] > 0.8 * n_form[0] and refuted[1] > 0.8 * n_form[1], (refuted, n_form)


def _injective_state(rng, w=3):
    """Applications f(a) with their inverse asserted (inv(f(a)) == a, as the keccak manager
    asserts) -- direct or through Concat(x, c) arguments of twice the width -- with compares
    between the values and between the arguments (six variables: two w-bit variables, two
    application values, two inverse values)."""
    nl = [[S.VAR, w, -1, -1, -1, 0, 0], [S.VAR, w, -1, -1, -1, 1, 0]]
    cl = [int(rng.integers(0, 8)) for _ in range(2)]
    nl += [[S.CONST, w, -1, -1, -1, 0, 0], [S.CONST, w, -1, -1, -1, 1, 0]]
    bools, apps = [], []
    wide = rng.random() < 0.5
    for k in range(2):
        a = int(rng.choice([0, 1, 2, 3]))
        if wide:
            nl.append([S.CONCAT, 2 * w, a, 2, -1, 0, 0])
            a = len(nl) - 1
        nl.append([S.UFAPP, w, a, -1, -1, 7 if wide else 5, 2 + k])
        u = len(nl) - 1
        if rng.random() < 0.85:      # the manager's inv(f(x)) == x
            nl.append([S.UFINV, 2 * w if wide else w, u, -1, -1, 7 if wide else 5, 4 + k])
            nl.append([S.EQ, 1, len(nl) - 1, a, -1, 0, 0])
            bools.append(len(nl) - 1)
        apps.append((u, a))
    (u0, a0), (u1, a1) = apps
    nl.append([S.EQ, 1, u0, u1, -1, 0, 0])
    bools.append(len(nl) - 1)
    if rng.random() < 0.6:          # the arguments differ
        nl.append([S.EQ, 1, a0, a1, -1, 0, 0])
        nl.append([S.BNOT, 1, len(nl) - 1, -1, -1, 0, 0])
        bools.append(len(nl) - 1)
    if rng.random() < 0.5:
        nl.append([[S.ULT, S.EQ, S.UGT][int(rng.integers(3))], 1, int(rng.choice([0, 1])), 3, -1, 0, 0])
        bools.append(len(nl) - 1)
    root = bools[0]
    for b in bools[1:]:
        nl.append([S.BAND, 1, root, b, -1, 0, 0])
        root = len(nl) - 1
    return nl, cl


def test_injectivity_exhaustive_soundness():
    """Applications f(a) with their inverse asserted (inv(f(a)) == a, as the keccak manager
    asserts for every application) -- direct, and through Concat(x, c) arguments of twice the
    width -- with compares between the values and between the arguments: no refuted state
    has a model over all 8^5 assignments of the variables and fresh values (C oracle), and
    the injectivity rule (Dom::injective) refutes `f(a) == f(b) and a != b`."""
    rng = np.random.default_rng(0x1A1)
    w = 3
    states = [_injective_state(rng, w) for _ in range(240)]
    verdict = _refute(states)
    n_vars = 6
    grid = np.array(np.meshgrid(*[np.arange(8)] * n_vars, indexing="ij")).reshape(n_vars, -1).T
    cands = np.zeros((1, grid.shape[0], n_vars, 8), np.uint32)
    cands[0, :, :, 0] = grid
    refuted = 0
    for (nl, cl), r in zip(states, verdict):
        assert r in (0, 1)
        if r != 1:
            continue
        refuted += 1
        nodes, noff, consts, coff = pack_states([(nl, cl)])
        assert coracle.first_sat(nodes, noff, consts, coff, cands)[0] < 0, "refuted a satisfiable state"
    assert refuted > 40, refuted


def _wrap_or_state(rng, w=3):
    """Random DAGs over three w-bit variables mixing ADD / SUB results compared with their
    operands (the wrap-ordering rule), BVAddNoOverflow / BVSubNoUnderflow flags on the same
    operands, and BOR trees of AND-ed compares with constants (the disjunctive hull), plus
    EQ / ITE reads of the bounded nodes."""
    nl = [[S.VAR, w, -1, -1, -1, k, 0] for k in range(3)]
    n_c = 4
    cl = [int(x) for x in rng.integers(0, 1 << w, size=n_c)]
    nl += [[S.CONST, w, -1, -1, -1, k, 0] for k in range(n_c)]   # nodes 3..6
    vals = [0, 1, 2]
    bools = []
    cmps = [S.ULT, S.ULE, S.UGT, S.UGE, S.EQ]

    def const():
        return 3 + int(rng.integers(n_c))

    for _ in range(int(rng.integers(6, 12))):
        k = rng.random()
        if k < 0.3:
            a, b = int(rng.choice(vals)), int(rng.choice(vals))
            op = S.ADD if rng.random() < 0.5 else S.SUB
            nl.append([op, w, a, b, -1, 0, 0])
            r = len(nl) - 1
            vals.append(r)
            # compare the result with an operand, and maybe the flag
            nl.append([cmps[int(rng.integers(4))], 1, r, a if rng.random() < 0.7 else b, -1, 0, 0])
            bools.append(len(nl) - 1)
            if rng.random() < 0.6:
                nl.append([S.UADD_NOOVF if op == S.ADD else S.USUB_NOUDF, 1, a, b, -1, 0, 0])
                if rng.random() < 0.5:
                    nl.append([S.BNOT, 1, len(nl) - 1, -1, -1, 0, 0])
                bools.append(len(nl) - 1)
        elif k < 0.55:
            # Or of 2-3 disjuncts, each an AND of 1-2 compares of one target with constants
            t = int(rng.choice(vals))
            dis = []
            for _ in range(int(rng.integers(2, 4))):
                nl.append([cmps[int(rng.integers(5))], 1, t, const(), -1, 0, 0])
                c = len(nl) - 1
                if rng.random() < 0.5:
                    nl.append([cmps[int(rng.integers(5))], 1, const(), t, -1, 0, 0])
                    nl.append([S.BAND, 1, c, len(nl) - 1, -1, 0, 0])
                    c = len(nl) - 1
                if rng.random() < 0.3:      # ULE's Or(ULT, ==) shape as a conjunct
                    cc = const()
                    nl.append([S.ULT, 1, t, cc, -1, 0, 0])
                    nl.append([S.EQ, 1, t, cc, -1, 0, 0])
                    nl.append([S.BOR, 1, len(nl) - 2, len(nl) - 1, -1, 0, 0])
                    nl.append([S.BAND, 1, c, len(nl) - 1, -1, 0, 0])
                    c = len(nl) - 1
                dis.append(c)
            root = dis[0]
            for d in dis[1:]:
                nl.append([S.BOR, 1, root, d, -1, 0, 0])
                root = len(nl) - 1
            bools.append(root)
        elif k < 0.75:
            nl.append([cmps[int(rng.integers(5))], 1, int(rng.choice(vals)), const() if rng.random() < 0.6
                       else int(rng.choice(vals)), -1, 0, 0])
            bools.append(len(nl) - 1)
        elif bools:
            nl.append([S.ITE, w, int(rng.choice(bools)), int(rng.choice(vals)), const(), 0, 0])
            vals.append(len(nl) - 1)
    while len(bools) < 2:
        nl.append([S.EQ, 1, int(rng.choice(vals)), const(), -1, 0, 0])
        bools.append(len(nl) - 1)
    root = bools[-1]
    for b in bools[-5:-1]:
        nl.append([S.BAND, 1, root, b, -1, 0, 0])
        root = len(nl) - 1
    return nl, cl


def test_wrap_orderings_and_disjunctive_hull_exhaustive_soundness():
    """The wrap-ordering rule (mgp_domain.h Dom::arith_rel) and the disjunctive hull
    (Dom::or_hull): random 3-bit DAGs of their shapes, every refuted state checked over all
    8^3 assignments with the C oracle; both rules must fire (refutations exist)."""
    rng = np.random.default_rng(0xA11CE)
    states = [_wrap_or_state(rng) for _ in range(1500)]
    verdict = _refute(states)
    grid = np.array(np.meshgrid(*[np.arange(8)] * 3, indexing="ij")).reshape(3, -1).T
    cands = np.zeros((1, grid.shape[0], 3, 8), np.uint32)
    cands[0, :, :, 0] = grid
    refuted = 0
    for st, r in zip(states, verdict):
        assert r in (0, 1)
        if r != 1:
            continue
        refuted += 1
        nodes, noff, consts, coff = pack_states([st])
        assert coracle.first_sat(nodes, noff, consts, coff, cands)[0] < 0, "refuted a satisfiable state"
    assert refuted > 100, refuted


def test_wrap_ordering_refutes_safemath_add_overflow():
    """BECToken.sol:25-29 + integer.py:141-147: c = a + b, assert(c >= a) passed, and
    Not(BVAddNoOverflow(a, b)) asserted: contradictory (a wrap makes c < a)."""
    nl = [X0, X1, [S.ADD, 256, 0, 1, -1, 0, 0], [S.UGE, 1, 2, 0, -1, 0, 0],
          [S.UADD_NOOVF, 1, 0, 1, -1, 0, 0], [S.BNOT, 1, 4, -1, -1, 0, 0], [S.BAND, 1, 3, 5, -1, 0, 0]]
    ok = [r[:] for r in nl]
    ok[5] = [S.UADD_NOOVF, 1, 0, 1, -1, 0, 0]      # no overflow: satisfiable
    sub = [X0, X1, [S.SUB, 256, 0, 1, -1, 0, 0], [S.UGT, 1, 2, 0, -1, 0, 0],   # a - b > a ...
           [S.UGE, 1, 0, 1, -1, 0, 0], [S.BAND, 1, 3, 4, -1, 0, 0]]          # ... with b <= a
    assert list(_refute([(nl, []), (ok, []), (sub, [])])) == [1, 0, 1]


def test_disjunctive_hull_separates_keccak_keys_from_small_slots():
    """keccak_function_manager.py:118-146: f(x) in [lo, hi) or f(x) == H; then f(x) == 8 (a
    small storage slot) is refuted, and a Store chain's value at f(x) skips slot 8."""
    lo, hi, H = 1 << 250, (1 << 250) + (1 << 123), (1 << 255) + 12345
    nl = [X0, [S.UFAPP, 256, 0, -1, -1, 0, 1],                              # 1: f(x)
          [S.CONST, 256, -1, -1, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 1, 0],
          [S.CONST, 256, -1, -1, -1, 2, 0], [S.CONST, 256, -1, -1, -1, 3, 0],
          [S.ULT, 1, 2, 1, -1, 0, 0], [S.EQ, 1, 2, 1, -1, 0, 0], [S.BOR, 1, 6, 7, -1, 0, 0],   # 8: lo <= f
          [S.ULT, 1, 1, 3, -1, 0, 0], [S.BAND, 1, 8, 9, -1, 0, 0],               # 10: lo <= f < hi
          [S.EQ, 1, 1, 4, -1, 0, 0], [S.BOR, 1, 10, 11, -1, 0, 0],               # 12: ... or f == H
          [S.EQ, 1, 1, 5, -1, 0, 0], [S.BAND, 1, 12, 13, -1, 0, 0]]              # f == 8
    free = [r[:] for r in nl]
    free[13] = [S.UGT, 1, 1, 5, -1, 0, 0]                                      # f > 8: fine
    assert list(_refute([(nl, [lo, hi, H, 8]), (free, [lo, hi, H, 8])])) == [1, 0]


def test_mul_by_odd_constant_narrows_backward():
    """x * c == k with c odd pins x = k * c^-1 (mod 2^w) on the known low bits of k: with
    x <u 100 that is refuted when c^-1 * k is huge and kept when it is small."""
    C5 = [S.CONST, 256, -1, -1, -1, 0, 0]
    base = [X0, C5, [S.MUL, 256, 0, 1, -1, 0, 0], [S.CONST, 256, -1, -1, -1, 1, 0], [S.EQ, 1, 2, 3, -1, 0, 0],
            [S.CONST, 256, -1, -1, -1, 2, 0], [S.ULT, 1, 0, 5, -1, 0, 0], [S.BAND, 1, 4, 6, -1, 0, 0]]
    out = _refute([(base, [5, 1, 100]), (base, [5, 10, 100]), (base, [6, 1, 100])])
    # 5x = 1: x = 5^-1 mod 2^256 (huge); 5x = 10: x = 2; 6x = 1: even c, 6x is even (no rule
    # needed: the known low bit already contradicts, or the state stays open) -- never
    # refuted when a model exists
    assert out[0] == 1 and out[1] == 0
    assert S.eval_root(base, [5, 10, 100], [2])


# ------------------------------- soak biased to the round-2/3 multiplication rules
def _random_mul_dag(rng, w):
    """Two w-bit variables; products by odd (and some even) constants under EQ and
    compares, BVMulNoOverflow and its negation, sums of products, plus a little Bool
    structure: the shapes backward narrowing through multiplication acts on."""
    nl = [[S.VAR, w, -1, -1, -1, 0, 0], [S.VAR, w, -1, -1, -1, 1, 0]]
    cl = []
    m = (1 << w) - 1

    def const(v):
        cl.append(int(v) & m)
        nl.append([S.CONST, w, -1, -1, -1, len(cl) - 1, 0])
        return len(nl) - 1

    vals, bools = [0, 1], []
    for _ in range(int(rng.integers(3, 9))):
        k = rng.random()
        if k < 0.35:  # x * c, c odd 3/4 of the time
            c = int(rng.integers(0, 1 << w)) | (1 if rng.random() < 0.75 else 0)
            a = int(rng.choice(vals))
            nl.append([S.MUL, w, a, const(c), -1, 0, 0] if rng.random() < 0.5 else [S.MUL, w, const(c), a, -1, 0, 0])
            vals.append(len(nl) - 1)
        elif k < 0.45:
            nl.append([[S.ADD, S.SUB, S.XOR][int(rng.integers(3))], w, int(rng.choice(vals)), int(rng.choice(vals)), -1, 0, 0])
            vals.append(len(nl) - 1)
        elif k < 0.55:
            nl.append([S.UMUL_NOOVF, 1, int(rng.choice(vals)), int(rng.choice(vals)), -1, 0, 0])
            bools.append(len(nl) - 1)
            if rng.random() < 0.6:
                nl.append([S.BNOT, 1, len(nl) - 1, -1, -1, 0, 0])
                bools.append(len(nl) - 1)
        else:  # EQ mostly: product == k
            op = [S.EQ, S.EQ, S.EQ, S.ULT, S.UGT, S.ULE, S.SLT][int(rng.integers(7))]
            a = int(rng.choice(vals[2:] or vals))
            b = const(rng.integers(0, 1 << w)) if rng.random() < 0.7 else int(rng.choice(vals))
            nl.append([op, 1, a, b, -1, 0, 0])
            bools.append(len(nl) - 1)
    while len(bools) < 2:
        nl.append([S.EQ, 1, int(rng.choice(vals)), const(rng.integers(0, 1 << w)), -1, 0, 0])
        bools.append(len(nl) - 1)
    root = bools[-1]
    for b in bools[-4:-1]:
        nl.append([S.BAND, 1, root, b, -1, 0, 0])
        root = len(nl) - 1
    return nl, cl


@pytest.mark.parametrize("w", [4, 6, 8])
def test_exhaustive_soundness_multiplication_shapes(w):
    """Every refuted state has no model over ALL 2^(2w) assignments (C oracle), and the
    product rules really fire: states with `x * odd == k` are refuted in numbers."""
    rng = np.random.default_rng(0x30DD + w)
    n = {4: 600, 6: 400, 8: 200}[w]
    states = [_random_mul_dag(rng, w) for _ in range(n)]
    verdict = _refute(states)
    grid = np.array(np.meshgrid(np.arange(1 << w), np.arange(1 << w), indexing="ij")).reshape(2, -1).T
    cands = np.zeros((1, grid.shape[0], 2, 8), np.uint32)
    cands[0, :, :, 0] = grid
    refuted = unsat = odd_eq_refuted = 0
    for (nl, cl), r in zip(states, verdict):
        assert r in (0, 1)
        nodes, noff, consts, coff = pack_states([(nl, cl)])
        has_model = coracle.first_sat(nodes, noff, consts, coff, cands)[0] >= 0
        unsat += not has_model
        if r == 1:
            refuted += 1
            assert not has_model, "refuted a satisfiable state"
            odd_eq_refuted += any(x[0] == S.EQ and nl[x[2]][0] == S.MUL for x in nl)
    assert refuted > n // 3 and odd_eq_refuted > n // 6, (refuted, odd_eq_refuted, unsat)


def _random_store_chain_dag(rng, w=3):
    """Storage-shaped reads (array.py:16-63 as LASER builds them): Select(Store(Store(a,
    k1, v1), k2, v2), i) = If(i == k2, v2, If(i == k1, v1, a[i])) with a[i] a UF
    application of the base array, several reads of one chain at related indices, and
    constraints on the read values (== / != constants, orderings between reads)."""
    nl = [[S.VAR, w, -1, -1, -1, v, 0] for v in range(4)]        # k1, k2, i, j
    cl = [int(rng.integers(0, 1 << w)) for _ in range(3)]
    nl += [[S.CONST, w, -1, -1, -1, c, 0] for c in range(3)]     # 4, 5, 6
    vals = [0, 1, 2, 3, 4, 5, 6]
    n_uf = 0

    def read(idx):
        nonlocal n_uf
        nl.append([S.UFAPP, w, idx, -1, -1, 9, 4 + n_uf])       # base read a[idx]: fresh value slot 4+
        n_uf += 1
        r = len(nl) - 1
        for k, v in ((0, 4), (1, 5)):                            # oldest store innermost
            nl.append([S.EQ, 1, idx, k, -1, 0, 0])
            nl.append([S.ITE, w, len(nl) - 1, v, r, 0, 0])
            r = len(nl) - 1
        return r

    reads = [read(int(rng.choice([2, 3, 0]))) for _ in range(int(rng.integers(2, 4)))]
    bools = []
    for _ in range(int(rng.integers(2, 5))):
        a = int(rng.choice(reads))
        k = rng.random()
        if k < 0.4:
            nl.append([S.EQ, 1, a, int(rng.choice(vals[4:])), -1, 0, 0])
        elif k < 0.6:
            nl.append([S.EQ, 1, a, int(rng.choice(reads)), -1, 0, 0])
        elif k < 0.8:
            nl.append([S.ULT, 1, a, int(rng.choice(reads + [6])), -1, 0, 0])
        else:
            nl.append([S.EQ, 1, int(rng.choice([0, 1, 2, 3])), int(rng.choice([0, 1, 2, 3])), -1, 0, 0])
        bools.append(len(nl) - 1)
        if rng.random() < 0.4:
            nl.append([S.BNOT, 1, bools[-1], -1, -1, 0, 0])
            bools[-1] = len(nl) - 1
    root = bools[0]
    for b in bools[1:]:
        nl.append([S.BAND, 1, root, b, -1, 0, 0])
        root = len(nl) - 1
    return nl, cl, 4 + n_uf


def test_exhaustive_soundness_store_chains():
    """Read-over-write chains: no refuted state has a model over all
    assignments of the four index variables and every fresh base-read value (2-bit, C
    oracle), and the pre-check does refute a share of them (equal indices force equal
    reads through the ITE chains and UF congruence)."""
    rng = np.random.default_rng(0x570E)
    w = 2
    states = [_random_store_chain_dag(rng, w) for _ in range(240)]
    verdict = _refute([(nl, cl) for nl, cl, _ in states])
    refuted = 0
    for (nl, cl, n_vars), r in zip(states, verdict):
        assert r in (0, 1)
        if r != 1:
            continue
        refuted += 1
        grid = np.array(np.meshgrid(*[np.arange(1 << w)] * n_vars, indexing="ij")).reshape(n_vars, -1).T
        cands = np.zeros((1, grid.shape[0], n_vars, 8), np.uint32)
        cands[0, :, :, 0] = grid
        nodes, noff, consts, coff = pack_states([(nl, cl)])
        assert coracle.first_sat(nodes, noff, consts, coff, cands)[0] < 0, "refuted a satisfiable state"
    assert refuted > 40, refuted


def _alias_state(rng, w=3):
    """Random w-bit DAGs of the shapes the value-alias rule (Dom::same_value) and the case
    split (mgp_refute_split) reason about: select chains on equalities of variables,
    x + 0 / x - 0 / x | 0 / x ^ 0, applications of one function on selected arguments,
    and compares between selected values and applications (ether_thief.py:55-95 in small:
    a balance read through a zero-value transfer against the starting balance)."""
    nl = [[S.VAR, w, -1, -1, -1, k, 0] for k in range(3)]
    cl = [0] + [int(x) for x in rng.integers(0, 1 << w, size=2)]
    nl += [[S.CONST, w, -1, -1, -1, k, 0] for k in range(3)]   # 3: zero, 4, 5
    vals, conds, bools = [0, 1, 2, 4, 5], [], []
    for _ in range(int(rng.integers(2, 4))):
        nl.append([S.EQ, 1, int(rng.integers(0, 3)), int(rng.choice([0, 1, 2, 4, 5])), -1, 0, 0])
        conds.append(len(nl) - 1)
    apps = []
    for _ in range(int(rng.integers(6, 11))):
        k = rng.random()
        if k < 0.35:
            nl.append([S.ITE, w, int(rng.choice(conds)), int(rng.choice(vals)), int(rng.choice(vals)), 0, 0])
        elif k < 0.6:
            nl.append([[S.ADD, S.SUB, S.OR, S.XOR][int(rng.integers(4))], w, int(rng.choice(vals)), 3, -1, 0, 0])
        elif len(apps) < 2:
            nl.append([S.UFAPP, w, int(rng.choice(vals)), -1, -1, 9, 3 + len(apps)])
            apps.append(len(nl) - 1)
        else:
            nl.append([S.ITE, w, int(rng.choice(conds)), int(rng.choice(apps)), int(rng.choice(vals)), 0, 0])
        vals.append(len(nl) - 1)
    for _ in range(int(rng.integers(1, 3))):
        a, b = int(rng.choice(vals[5:] or vals)), int(rng.choice(apps or vals))
        op = [S.UGT, S.ULT, S.EQ][int(rng.integers(3))]
        nl.append([op, 1, a, b, -1, 0, 0])
        if op == S.EQ and rng.random() < 0.5:
            nl.append([S.BNOT, 1, len(nl) - 1, -1, -1, 0, 0])
        bools.append(len(nl) - 1)
    for c in conds:
        if rng.random() < 0.4:
            bools.append(c if rng.random() < 0.5 else (nl.append([S.BNOT, 1, c, -1, -1, 0, 0]) or len(nl) - 1))
    root = bools[0]
    for b in bools[1:]:
        nl.append([S.BAND, 1, root, b, -1, 0, 0])
        root = len(nl) - 1
    return nl, cl


def test_value_alias_and_case_split_exhaustive_soundness():
    """The value-alias rule and one and two levels of case splitting (round 4,
    mgp_refute_split): every state either refutes is checked over all 8^5 assignments of its
    three 3-bit variables and two application values (C oracle, which gives applications
    with equal arguments one value); one level must refute strictly more than the plain
    analysis, and two levels at least what one does."""
    rng = np.random.default_rng(0xE7E)
    states = [_alias_state(rng) for _ in range(700)]
    nodes, noff, consts, coff = pack_states(states)
    plain = N.refute(nodes, noff, consts, coff)
    split = N.refute_split(nodes, noff, consts, coff, max_splits=8)
    split2 = N.refute_split(nodes, noff, consts, coff, max_splits=8, depth=2)
    n_vars = 5
    grid = np.array(np.meshgrid(*[np.arange(8)] * n_vars, indexing="ij")).reshape(n_vars, -1).T
    cands = np.zeros((1, grid.shape[0], n_vars, 8), np.uint32)
    cands[0, :, :, 0] = grid
    n_plain = n_split = n_split2 = 0
    for st, p, s, s2 in zip(states, plain, split, split2):
        assert p in (0, 1) and s in (0, 1) and s2 in (0, 1)
        assert not (p == 1 and s != 1), "the split lost a plain refutation"
        assert not (s == 1 and s2 != 1), "two levels lost a one-level refutation"
        if s2 != 1:
            continue
        n_plain += p == 1
        n_split += s == 1
        n_split2 += 1
        nodes, noff, consts, coff = pack_states([st])
        assert coracle.first_sat(nodes, noff, consts, coff, cands)[0] < 0, "refuted a satisfiable state"
    assert n_plain > 50 and n_split > n_plain and n_split2 >= n_split, (n_plain, n_split, n_split2)


def _transfer_chain_state(rng, w=3):
    """A balance passed through 2-3 conditional transfers (select on an equality of
    addresses between the balance and the balance minus / plus / or / xor an amount that is
    mostly zero) and compared with its start: ether_thief.py:55-95's balance comparisons
    after a run of zero-value transfers, which need one split per transfer."""
    nl = [[S.VAR, w, -1, -1, -1, k, 0] for k in range(4)]
    cl = [0] + [int(x) for x in rng.integers(0, 1 << w, size=2)]
    nl += [[S.CONST, w, -1, -1, -1, k, 0] for k in range(3)]   # 4: zero, 5, 6
    cur = 0
    for _ in range(int(rng.integers(2, 4))):
        a, b = (int(x) for x in rng.choice([1, 2, 3, 5, 6], 2, replace=False))
        nl.append([S.EQ, 1, a, b, -1, 0, 0])
        c = len(nl) - 1
        op = [S.SUB, S.ADD, S.OR, S.XOR][int(rng.integers(4))]
        nl.append([op, w, cur, 4 if rng.random() < 0.85 else int(rng.choice([5, 6])), -1, 0, 0])
        t = len(nl) - 1
        nl.append([S.ITE, w, c, t, cur, 0, 0] if rng.random() < 0.5 else [S.ITE, w, c, cur, t, 0, 0])
        cur = len(nl) - 1
    op = [S.UGT, S.ULT][int(rng.integers(2))]
    nl.append([op, 1, cur, 0, -1, 0, 0] if rng.random() < 0.5 else [op, 1, 0, cur, -1, 0, 0])
    return nl, cl


def test_case_split_depth_exhaustive_soundness():
    """Nested case splits (mgp_refute_split, depth 1..3) on transfer chains: each level
    refutes a superset of the last and strictly more in total, and every refuted state is
    checked over all 8^4 assignments of its four 3-bit variables (C oracle)."""
    rng = np.random.default_rng(0x5917)
    states = [_transfer_chain_state(rng) for _ in range(600)]
    packed = pack_states(states)
    # (without the interval bisection: on 3-bit variables it enumerates every value, so one
    # level with it refutes what three levels of case splits do; its soundness is checked
    # below and in test_bisection_exhaustive_soundness)
    levels = [N.refute(*packed)] + [N.refute_split(*packed, max_splits=8, depth=d, bisect=False) for d in (1, 2, 3)]
    counts = [int((r == 1).sum()) for r in levels]
    for lo, hi in zip(levels, levels[1:]):
        assert ((lo == 1) & (hi != 1)).sum() == 0, "a deeper split lost a refutation"
    assert counts[0] < counts[1] < counts[2] <= counts[3], counts
    n_vars = 4
    grid = np.array(np.meshgrid(*[np.arange(8)] * n_vars, indexing="ij")).reshape(n_vars, -1).T
    cands = np.zeros((1, grid.shape[0], n_vars, 8), np.uint32)
    cands[0, :, :, 0] = grid
    for st, r in zip(states, levels[3]):
        if r == 1:
            assert coracle.first_sat(*pack_states([st]), cands)[0] < 0, "refuted a satisfiable state"
    withb = N.refute_split(*packed, max_splits=8, depth=2)
    assert ((levels[2] == 1) & (withb != 1)).sum() == 0
    for st, r in zip(states, withb):
        if r == 1:
            assert coracle.first_sat(*pack_states([st]), cands)[0] < 0, "bisection refuted a satisfiable state"


def _ratio_state(rng, w=8):
    """x bounded by two constants, then two products of x with constants (wrapping or not)
    divided and compared -- rubixi.sol's payout against the balance share (130-151) -- next
    to a second, free variable in an addition."""
    lo, hi = sorted(int(v) for v in rng.integers(0, 1 << w, size=2))
    c1, c2, d = (int(v) for v in rng.integers(1, 1 << (w // 2), size=3))
    cl = [lo, hi, c1, c2, d]
    nl = [[S.VAR, w, -1, -1, -1, 0, 0], [S.VAR, w, -1, -1, -1, 1, 0]]
    nl += [[S.CONST, w, -1, -1, -1, k, 0] for k in range(5)]                     # 2..6
    nl.append([S.UGE, 1, 0, 2, -1, 0, 0])                                         # 7: x >= lo
    nl.append([S.ULE, 1, 0, 3, -1, 0, 0])                                         # 8: x <= hi
    nl.append([S.MUL, w, 0, 4, -1, 0, 0])                                         # 9
    nl.append([S.MUL, w, 0, 5, -1, 0, 0])                                         # 10
    nl.append([S.UDIV, w, 9, 6, -1, 0, 0])                                        # 11
    nl.append([S.UDIV, w, 10, 6, -1, 0, 0])                                       # 12
    nl.append([S.ADD, w, 11, 1, -1, 0, 0] if rng.random() < 0.3 else [S.ADD, w, 11, 2, -1, 0, 0])  # 13
    nl.append([[S.UGT, S.ULT, S.EQ][int(rng.integers(3))], 1, 13, 12, -1, 0, 0])  # 14
    nl.append([S.BAND, 1, 7, 8, -1, 0, 0])
    nl.append([S.BAND, 1, 15, 14, -1, 0, 0])
    return nl, cl


def test_bisection_exhaustive_soundness():
    """Interval bisection (mgp_refute_split, round 6) on bounded-variable ratio tests over
    8-bit values: it refutes states the case splits alone leave open, and every state it
    refutes has no model over all 2^16 assignments of its two variables (C oracle)."""
    rng = np.random.default_rng(0xB15E)
    states = [_ratio_state(rng) for _ in range(400)]
    packed = pack_states(states)
    nob = N.refute_split(*packed, max_splits=8, depth=2, bisect=False)
    withb = N.refute_split(*packed, max_splits=8, depth=2)
    assert ((nob == 1) & (withb != 1)).sum() == 0
    assert int((withb == 1).sum()) > int((nob == 1).sum()), (int((nob == 1).sum()), int((withb == 1).sum()))
    grid = np.array(np.meshgrid(np.arange(256), np.arange(256), indexing="ij")).reshape(2, -1).T
    cands = np.zeros((1, grid.shape[0], 2, 8), np.uint32)
    cands[0, :, :, 0] = grid
    n_unsat = 0
    for st, r in zip(states, withb):
        unsat = coracle.first_sat(*pack_states([st]), cands)[0] < 0
        n_unsat += unsat
        assert unsat or r != 1, "bisection refuted a satisfiable state"
    # (on this shape it is also complete: 149 of 149 UNSAT states, 137 without it)
    assert int((withb == 1).sum()) == n_unsat, (int((withb == 1).sum()), n_unsat)


def _refund_state(rng, w=3):
    """A balance after a payment and a refund compared with the starting balance, over
    applications of one balance function at a symbolic sender and at a constant address
    (weak_random.sol:18-35 / ether_thief.py:55-95 in small): the sender pays v, gets back
    v - p (or v, or v + p) and the attacker's balance is compared with its start."""
    nl = [[S.VAR, w, -1, -1, -1, k, 0] for k in range(2)]                          # 0 sender, 1 value
    cl = [int(x) for x in rng.integers(0, 1 << w, size=2)]
    nl += [[S.CONST, w, -1, -1, -1, k, 0] for k in range(2)]                       # 2 attacker, 3 price
    nl.append([S.UFAPP, w, 0, -1, -1, 9, 2])                                       # 4 bal(sender)
    nl.append([S.UFAPP, w, 2, -1, -1, 9, 3])                                       # 5 bal(attacker)
    nl.append([S.SUB, w, 4, 1, -1, 0, 0])                                          # 6 bal - v
    refund = int(rng.integers(3))
    nl.append([[S.SUB, S.ADD, S.ADD][refund], w, 1, 3 if refund < 2 else 1, -1, 0, 0])  # 7 v -/+ p (or v + v)
    nl.append([S.ADD, w, 6, 7, -1, 0, 0])                                          # 8 after
    nl.append([S.EQ, 1, 0, 2, -1, 0, 0])                                           # 9 sender == attacker
    nl.append([S.ITE, w, 9, 8, 5, 0, 0])                                           # 10 attacker's balance
    nl.append([[S.UGT, S.ULT, S.EQ][int(rng.integers(3))], 1, 10, 5, -1, 0, 0])    # 11 vs start
    nl.append([S.UGE, 1, 4, 1, -1, 0, 0] if rng.random() < 0.7 else [S.ULT, 1, 1, 4, -1, 0, 0])  # 12
    nl.append([S.UGE, 1, 1, 3, -1, 0, 0])                                          # 13 v >= p
    root = 11
    for extra in (12, 13) + ((9,) if rng.random() < 0.6 else ()):
        nl.append([S.BAND, 1, root, extra, -1, 0, 0])
        root = len(nl) - 1
    return nl, cl


def test_linear_forms_exhaustive_soundness():
    """The linear-form pass (mgp_refute_split, round 6) on payment-and-refund states: it
    refutes states the case splits alone leave open, and every refuted state has no model
    over all 8^4 assignments of its two variables and two application values (C oracle;
    applications with equal arguments get one value)."""
    rng = np.random.default_rng(0x11AE)
    states = [_refund_state(rng) for _ in range(500)]
    packed = pack_states(states)
    nob = N.refute_split(*packed, max_splits=8, depth=2, bisect=False)
    withb = N.refute_split(*packed, max_splits=8, depth=2)
    assert ((nob == 1) & (withb != 1)).sum() == 0
    assert int((withb == 1).sum()) > int((nob == 1).sum()), (int((nob == 1).sum()), int((withb == 1).sum()))
    n_vars = 4
    grid = np.array(np.meshgrid(*[np.arange(8)] * n_vars, indexing="ij")).reshape(n_vars, -1).T
    cands = np.zeros((1, grid.shape[0], n_vars, 8), np.uint32)
    cands[0, :, :, 0] = grid
    for st, r in zip(states, withb):
        if r == 1:
            assert coracle.first_sat(*pack_states([st]), cands)[0] < 0, "linear pass refuted a satisfiable state"


def test_refute_split_argument_range():
    """refute_split packs the atom count (bits 0..15) and the depth (bits 16..19) into one
    C argument: values outside them are refused before the call."""
    import pytest

    nodes, noff, consts, coff = pack_states([_transfer_chain_state(np.random.default_rng(1))])
    for kw in ({"depth": 0}, {"depth": 16}, {"max_splits": 1 << 16}, {"max_splits": -1}):
        with pytest.raises(ValueError):
            N.refute_split(nodes, noff, consts, coff, **kw)
    assert N.refute_split(nodes, noff, consts, coff, max_splits=0).tolist() == N.refute(nodes, noff, consts, coff).tolist()


def _balance_chain_state(rng, w=2):
    """A balances array through 3-5 transfers (corpus.laser's transfer_ether on the laser.smt
    mirror: Store chains of `b[to] = b[to] + v`, `b[from] = b[from] - v`, values mostly 0)
    and ether_thief's `b[a] > start[a]` (ether_thief.py:55-95) or its `==` / `<` variants,
    on w-bit addresses: the shapes Dom::chain_orders walks."""
    from mythril_amd import smt
    from mythril_amd.dag import build_state

    sym = smt.symbol_factory
    addrs = [sym.BitVecSym(f"a{k}", w) for k in range(3)]
    zero = sym.BitVecVal(0, w)
    amt = sym.BitVecSym("amt", w)
    bal = smt.Array("bal", w, w)
    start = __import__("copy").copy(bal)
    cons = []
    for _ in range(int(rng.integers(3, 6))):
        frm, to = (addrs[int(i)] for i in rng.choice(3, 2, replace=False))
        v = zero if rng.random() < 0.8 else amt
        bal[to] = bal[to] + v
        bal[frm] = bal[frm] - v
        if rng.random() < 0.3:
            cons.append(frm == addrs[int(rng.integers(3))])
    a = addrs[int(rng.integers(3))]
    op = int(rng.integers(3))
    cons.append(smt.UGT(bal[a], start[a]) if op == 0 else (smt.ULT(bal[a], start[a]) if op == 1 else
                                                              smt.Not(bal[a] == start[a])))
    st = build_state([c.raw for c in cons])
    return (st.nodes, st.consts), st.n_vars


def test_chain_orders_exhaustive_soundness():
    """Path-sensitive select-chain orderings (round 5, Dom::chain_orders): every state the
    plain pre-check refutes is checked over all assignments of its addresses, amount and
    base-read values (C oracle, equal reads of one array equal), and the plain pre-check
    now refutes the zero-value transfer chains that needed a split per transfer."""
    rng = np.random.default_rng(0xC4A1)
    states = [_balance_chain_state(rng) for _ in range(160)]
    verdict = _refute([s for s, _ in states])
    refuted = 0
    for ((nl, cl), n_vars), r in zip(states, verdict):
        assert r in (0, 1)
        if r != 1:
            continue
        refuted += 1
        grid = np.array(np.meshgrid(*[np.arange(4)] * n_vars, indexing="ij")).reshape(n_vars, -1).T
        cands = np.zeros((1, grid.shape[0], n_vars, 8), np.uint32)
        cands[0, :, :, 0] = grid
        assert coracle.first_sat(*pack_states([(nl, cl)]), cands)[0] < 0, "refuted a satisfiable state"
    assert refuted > 30, refuted


def _random_transfer_dag(rng, w):
    """BECToken's batchTransfer shape (BECToken.sol:254-268, SafeMath.sol): cnt in a small
    range, amount = cnt * value (may wrap), bal >= amount, a receiver balance x and
    sum = x + value with its SafeMath.add overflow test taken either way (or as
    BVAddNoOverflow), x sometimes bal - amount (the sender paying itself)."""
    nl = [[S.VAR, w, -1, -1, -1, v, 0] for v in range(4)]          # cnt, value, bal, x0
    cl = [int(rng.integers(1, 7)), 0, int(rng.integers(1, 1 << (w - 1))), int(rng.integers(0, 1 << w))]
    nl += [[S.CONST, w, -1, -1, -1, c, 0] for c in range(4)]       # 4: cnt bound, 5: 0, 6: bal bound, 7: any
    roots = [len(nl)]
    nl.append([S.UGT, 1, 0, 5, -1, 0, 0])                           # cnt > 0
    roots.append(len(nl))
    nl.append([S.ULE if rng.random() < 0.5 else S.ULT, 1, 0, 4, -1, 0, 0])
    nl.append([S.MUL, w, 0, 1, -1, 0, 0] if rng.random() < 0.5 else [S.MUL, w, 1, 0, -1, 0, 0])
    amount = len(nl) - 1
    roots.append(len(nl))
    nl.append([S.UGE, 1, 2, amount, -1, 0, 0] if rng.random() < 0.5 else [S.ULE, 1, amount, 2, -1, 0, 0])
    if rng.random() < 0.6:
        roots.append(len(nl))
        nl.append([S.ULT, 1, 2, 6, -1, 0, 0])                       # the sender's balance is bounded
    if rng.random() < 0.4:                                          # the receiver is the sender
        nl.append([S.SUB, w, 2, amount, -1, 0, 0])
        x = len(nl) - 1
    else:
        x = 3
        if rng.random() < 0.5:
            roots.append(len(nl))
            nl.append([S.ULT, 1, 3, 7, -1, 0, 0])
    nl.append([S.ADD, w, x, 1, -1, 0, 0] if rng.random() < 0.5 else [S.ADD, w, 1, x, -1, 0, 0])
    s = len(nl) - 1
    k = rng.random()
    if k < 0.4:
        nl.append([S.UGE, 1, s, x, -1, 0, 0])                       # SafeMath.add: assert(c >= a)
        nl.append([S.BNOT, 1, len(nl) - 1, -1, -1, 0, 0])           # ... failing
    elif k < 0.6:
        nl.append([S.UGE, 1, s, x, -1, 0, 0])                       # ... holding
    elif k < 0.8:
        nl.append([S.UADD_NOOVF, 1, x, 1, -1, 0, 0])
        nl.append([S.BNOT, 1, len(nl) - 1, -1, -1, 0, 0])
    else:
        nl.append([S.ULT, 1, s, 7, -1, 0, 0])                       # a bound on the new balance
    roots.append(len(nl) - 1)
    if rng.random() < 0.3:
        roots.append(len(nl))
        nl.append([S.UGT, 1, 1, 7, -1, 0, 0])                       # value bounded below
    r = roots[0]
    for b in roots[1:]:
        nl.append([S.BAND, 1, r, b, -1, 0, 0])
        r = len(nl) - 1
    return nl, cl


@pytest.mark.parametrize("w", [4, 5])
def test_exhaustive_soundness_transfer_shapes(w):
    """Addend bounds once an addition's wrap status is known (a failing SafeMath.add assert
    bounds the addend from below) and products with a small-range operand (cnt * value per
    value of cnt): every refuted state has no model over ALL 2^(4w) assignments (C oracle),
    and the rules refute states in numbers (BECToken's transaction-2 overflow queries)."""
    rng = np.random.default_rng(0x7A5F + w)
    n = {4: 300, 5: 120}[w]
    states = [_random_transfer_dag(rng, w) for _ in range(n)]
    verdict = _refute(states)
    g = np.array(np.meshgrid(*[np.arange(1 << w)] * 4, indexing="ij")).reshape(4, -1).T
    cands = np.zeros((1, g.shape[0], 4, 8), np.uint32)
    cands[0, :, :, 0] = g
    refuted = unsat = 0
    for (nl, cl), r in zip(states, verdict):
        assert r in (0, 1)
        nodes, noff, consts, coff = pack_states([(nl, cl)])
        has_model = coracle.first_sat(nodes, noff, consts, coff, cands)[0] >= 0
        unsat += not has_model
        if r == 1:
            refuted += 1
            assert not has_model, "refuted a satisfiable state"
    assert refuted >= 0.8 * unsat, (refuted, unsat)  # 102 / 102 and 32 / 34 (72 and 18 before the rules)


def test_split_never_refutes_a_planted_synthetic_state():
    """256-bit soundness on random DAGs (the bench's generator, SURVEY §8d op mix): a state with
    a planted satisfying assignment -- checked here by the C oracle -- is never refuted by
    mgp_refute_split at the product's settings (case splits, linear forms, bisection), while
    the split refuter refutes hundreds of the other states."""
    b = N.synth_generate(0x4D595448, 3 << 20, 4096, 64, 256)
    r = N.refute_split(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"], max_splits=8, depth=2)
    planted = np.nonzero(b["planted"])[0]
    assert len(planted) > 1500 and int((r == 1).sum()) > 500
    # the plants are models (one candidate row per planted state)
    sub = planted[:512]
    no, co = b["node_offsets"].astype(np.int64), b["const_offsets"].astype(np.int64)
    nodes = np.concatenate([b["nodes"][no[i]:no[i + 1]] for i in sub])
    consts = np.concatenate([b["consts"][co[i]:co[i + 1]] for i in sub]).reshape(-1, 8)
    noff = np.concatenate([[0], np.cumsum([no[i + 1] - no[i] for i in sub])]).astype(np.uint64)
    coff = np.concatenate([[0], np.cumsum([co[i + 1] - co[i] for i in sub])]).astype(np.uint64)
    cands = np.ascontiguousarray(b["plant_words"][sub][:, None])
    assert (coracle.first_sat(nodes, noff, consts, coff, cands) == 0).all()
    assert int((r[planted] == 1).sum()) == 0
