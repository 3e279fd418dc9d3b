"""oracle.refute_check, the independent re-proof of the product's refutations (VERDICT r5 item
6): the checker itself is sound (every state it re-proves has no model, checked exhaustively
with the C oracle), it never re-proves a query the CPU restatement of the witness rounds
answers with a model, and it replays the product refuter's refutations of restated contracts
from their UNSAT cores.  CPU only; the whole suite's replay is scripts/replay_refutations.py
(profiles/refute_replay_r6.json)."""
import numpy as np
import pytest

from mythril_amd import smt
from oracle import bvsem as S
from oracle import coracle
from oracle import refute_check as RC

from ._util import pack_states
from .test_refute import _injective_state, _random_mul_dag, _random_small_dag, _ratio_state, _refund_state, _transfer_chain_state


def _terms(nodes, consts):
    """A node list (tests/_util format: op, width, a, b, c, p0, p1) -> its root as smt terms:
    Bool nodes get width 0, variables are named by index, UF applications keep the function
    id (their value variable is the C oracle's model of the application)."""
    out = []
    for op, w, a, b, c, p0, p1 in nodes:
        bw = 0 if op in S.BOOL_RESULT or op in (S.BAND, S.BOR, S.BXOR, S.BNOT, S.BITE, S.BEQ) else w
        if op == S.ITE and out[a].width == 0 and w == 1 and out[b].width == 0:
            bw = 0
        args = tuple(out[x] for x in (a, b, c) if x >= 0)
        if op == S.CONST:
            t = smt.mk(op, w, (), (consts[p0] & ((1 << w) - 1),))
        elif op == S.VAR:
            t = smt.mk(op, w, (), (f"x{p0}",))
        elif op == S.EXTRACT:
            t = smt.mk(op, w, args, (p0, p1))
        elif op in (S.UFAPP, S.UFINV):
            t = smt.mk(op, w, args, (p0, f"f{p0}"))
        else:
            t = smt.mk(op, bw, args)
        out.append(t)
    return out[-1]


def _safemath_state(rng, w=4):
    """SafeMath.add's shapes (BECToken.sol): s = a + b (either operand order) compared with one
    of its operands, next to BVAddNoOverflow(a, b) or its negation and a bound on b."""
    nl = [[S.VAR, w, -1, -1, -1, 0, 0], [S.VAR, w, -1, -1, -1, 1, 0]]
    cl = [int(rng.integers(0, 1 << w)) for _ in range(2)]
    nl += [[S.CONST, w, -1, -1, -1, 0, 0], [S.CONST, w, -1, -1, -1, 1, 0]]        # 2, 3
    nl.append([S.ADD, w, 0, 1, -1, 0, 0] if rng.random() < 0.5 else [S.ADD, w, 1, 0, -1, 0, 0])  # 4
    bools = []
    nl.append([S.UADD_NOOVF, 1, 0, 1, -1, 0, 0] if rng.random() < 0.5 else [S.UADD_NOOVF, 1, 1, 0, -1, 0, 0])
    bools.append(len(nl) - 1)
    if rng.random() < 0.5:
        nl.append([S.BNOT, 1, len(nl) - 1, -1, -1, 0, 0])
        bools.append(len(nl) - 1)
    op = [S.UGE, S.UGT, S.ULT, S.ULE, S.EQ][int(rng.integers(5))]
    nl.append([op, 1, 4, int(rng.choice([0, 1])), -1, 0, 0])
    bools.append(len(nl) - 1)
    if rng.random() < 0.5:
        nl.append([[S.ULT, S.UGT, S.EQ][int(rng.integers(3))], 1, 1, int(rng.choice([2, 3])), -1, 0, 0])
        bools.append(len(nl) - 1)
    root = bools[-1]
    for b in bools[-4:-1][::-1]:
        nl.append([S.BAND, 1, root, b, -1, 0, 0])
        root = len(nl) - 1
    return nl, cl


def _no_model(state, n_vars, w):
    grid = np.array(np.meshgrid(*[np.arange(1 << w)] * n_vars, indexing="ij")).reshape(n_vars, -1).T
    cands = np.zeros((1, grid.shape[0], n_vars, 8), np.uint32)
    cands[0, :, :, 0] = grid
    return coracle.first_sat(*pack_states([state]), cands)[0] < 0


@pytest.mark.parametrize("shape", ["random", "transfer", "refund", "ratio", "injective", "mul", "safemath"])
def test_checker_is_sound_exhaustively(shape):
    """Every state the checker re-proves UNSAT has no model over all assignments of its
    variables (and UF application values), and it re-proves a real share of them."""
    rng = np.random.default_rng({"random": 0xC4EC, "transfer": 0x7A5F, "refund": 0x4EF0, "ratio": 0x2A71, "injective": 0x1A1, "mul": 0x30DE, "safemath": 0x5AFE}[shape])
    if shape == "random":
        states = [(_random_small_dag(rng, w=4, n_ops=int(rng.integers(4, 14))), 2, 4) for _ in range(300)]
    elif shape == "transfer":
        states = [(_transfer_chain_state(rng), 4, 3) for _ in range(300)]
    elif shape == "refund":
        states = [(_refund_state(rng), 4, 3) for _ in range(300)]
    elif shape == "ratio":   # rubixi.sol's payout ratios (interval bisection)
        states = [(_ratio_state(rng), 2, 8) for _ in range(150)]
    elif shape == "injective":   # keccak applications with the manager's inverse axiom
        states = [(_injective_state(rng), 6, 3) for _ in range(150)]
    elif shape == "mul":   # products by constants, wrapping (BECToken's cnt * value)
        states = [(_random_mul_dag(rng, 6), 2, 6) for _ in range(300)]
    else:
        states = [(_safemath_state(rng), 2, 4) for _ in range(300)]
    proved = 0
    for st, n_vars, w in states:
        if RC.refute([_terms(*st)], tiers=((2, 8, 20000),)):
            proved += 1
            assert _no_model(st, n_vars, w), f"checker refuted a satisfiable {shape} state"
    assert proved > len(states) // 10, proved


def test_linear_pass_decides_constant_differences():
    """x + 3 > x holds iff x <= 2^w - 4: the pass narrows x (with x >= 2^w - 3 also required
    the state is refuted); f(a) > f(b) with a == b forced by a compare is refuted; x + 1 == x
    is refuted without any split."""
    sym = smt.symbol_factory
    x, a, b = (sym.BitVecSym(n, 8) for n in ("x", "a", "b"))
    c3 = sym.BitVecVal(3, 8)
    assert RC.refute([smt.UGT(x + c3, x).raw, smt.UGE(x, sym.BitVecVal(253, 8)).raw], depth=1)
    assert not RC.refute([smt.UGT(x + c3, x).raw, smt.UGE(x, sym.BitVecVal(252, 8)).raw], depth=1)
    f = smt.Function("f_rc", 8, 8)
    assert RC.refute([(a == b).raw, smt.UGT(f(a), f(b)).raw], depth=1)
    assert not RC.refute([smt.UGT(f(a), f(b)).raw], depth=1)
    assert RC.refute([(x + sym.BitVecVal(1, 8) == x).raw], depth=1)


def _suite(names):
    from oracle.keccak_ref import keccak256

    import corpus

    return corpus.suite(hasher=keccak256, contracts=set(names))


def test_checker_never_refutes_a_witnessed_suite_query():
    """Queries of returnvalue.sol that the CPU restatement of the witness rounds answers with a
    model (C-oracle checked) are never re-proved UNSAT by the checker."""
    from tests import fe_emulate as E

    qs = _suite(["returnvalue"])
    ans, _ = E.suite_answers(qs, witnesses=True)
    sat = [k for k, a in enumerate(ans) if a == "sat"]
    assert len(sat) > 30
    for k in sat[::max(1, len(sat) // 40)]:
        assert not RC.refute(list(qs[k][3]), tiers=((2, 8, 5000),)), qs[k][2]


def test_replays_the_refutations_of_small_contracts():
    """The product refuter's refutations (mgp_refute_split at the product's settings) of five
    contracts are re-proved from their UNSAT cores (mgp_refute_cores) by the checker."""
    from mythril_amd import _native as N
    from mythril_amd import front as F
    from mythril_amd.solver import Prefilter

    qs = _suite(["suicide", "origin", "exceptions", "hashforether", "token"])
    B = F.Batch([list(q[3]) for q in qs])
    p = B.packed()[:4]
    split = N.refute_split(*p, max_splits=Prefilter.SPLIT_REFUTE, depth=Prefilter.SPLIT_DEPTH)
    keep, st = N.refute_cores(*p, np.array([len(q[3]) for q in qs], np.uint32))
    B.close()
    refuted = [k for k in range(len(qs)) if split[k] == 1]
    assert len(refuted) >= 20
    for k in refuted:
        cs = list(qs[k][3])
        if st[k] == 1:
            cs = [c for c, m in zip(cs, keep[k]) if m]
        assert RC.refute(cs), qs[k][2]
