"""The reference's own expectations on the hot path that are not keccak or EVM vectors
(SURVEY.md §8c items 4 and 5), restated through the GPU-first solver surface:

* tests/laser/state/calldata_test.py:41-91 -- SymbolicCalldata / ConcreteCalldata index
  semantics (two `unsat` answers, one concrete-index `unsat`);
* tests/laser/smt/independece_solver_test.py:12-145 -- _get_expr_variables, DependenceBucket,
  DependenceMap, and IndependenceSolver's unsat / unsat-in-second-bucket / sat answers.

Each UNSAT case asserts HOW it is answered: refuted by the host pre-check with no fallback
call (every one of them is), never a GPU witness.  SAT cases must be answered by a GPU
witness the oracle confirms, with no fallback call.  The CPU tests run the same queries
with a stand-in context that finds no witness (the refutations are host code); the GPU
tests run them through the real pipeline.
"""
import numpy as np
import pytest

from mythril_amd import _native as N
from mythril_amd import dag as D
from mythril_amd import solver as SV
from mythril_amd.smt import Array, Function, If, symbol_factory
from oracle import bvsem as S

BVV = symbol_factory.BitVecVal
BVS = symbol_factory.BitVecSym


class SymbolicCalldata:
    """calldata.py:207-236 restated: `_load(i)` = If(i < calldatasize, calldata[i], 0), the
    BitVec `<` being SIGNED (bitvec.py:138-147)."""

    def __init__(self, tx_id):
        self.size = BVS(f"{tx_id}_calldatasize", 256)
        self.calldatasize = self.size
        self._calldata = Array(f"{tx_id}_calldata", 256, 8)

    def __getitem__(self, item):
        item = BVV(item, 256) if isinstance(item, int) else item
        return If(item < self.size, self._calldata[item], BVV(0, 8))


class ConcreteCalldata:
    """calldata.py:135-200 restated for the index load: the concrete byte, 0 past the end
    (a K(256, 8, 0) array with the bytes stored, read at a concrete index)."""

    def __init__(self, tx_id, data):
        self._data = list(data)
        self.calldatasize = BVV(len(self._data), 256)

    def __getitem__(self, item):
        return BVV(self._data[item] if item < len(self._data) else 0, 8)


def _calldata_constrain_index():
    cd = SymbolicCalldata(0)
    return [cd[51] == BVV(1, 8), cd.calldatasize == BVV(50, 256)]           # calldata_test.py:58-76


def _calldata_equal_indices():
    cd = SymbolicCalldata(0)
    a, b = BVS("index_a", 256), BVS("index_b", 256)
    return [a == b, cd[a] != cd[b]]                                          # calldata_test.py:79-91


def _concrete_calldata_constrain_index():
    cd = ConcreteCalldata(0, [1, 4, 7, 3, 7, 2, 9])
    return [cd[2] == BVV(3, 8)]                                              # calldata_test.py:41-55


def _xyzab():
    return [BVS(n, 256) for n in "xyzab"]


def _independence_unsat():
    x, y, z, a, b = _xyzab()
    return [x > y, y == z, y != z, a == b]                                   # independece_solver_test.py:88-105


def _independence_unsat_second_bucket():
    x, y, z, a, b = _xyzab()
    return [x > y, y == z, a == b, a != b]                                   # independece_solver_test.py:108-125


def _independence_sat():
    x, y, z, a, b = _xyzab()
    return [x > y, y == z, a == b]                                           # independece_solver_test.py:128-145


UNSAT = {"calldata_constrain_index": _calldata_constrain_index,
         "calldata_equal_indices": _calldata_equal_indices,
         "concrete_calldata_constrain_index": _concrete_calldata_constrain_index,
         "independence_unsat": _independence_unsat,
         "independence_unsat_in_second_bucket": _independence_unsat_second_bucket}


class CountingBackend(SV.Backend):
    name = "counting"

    def __init__(self):
        self.calls = 0

    def check(self, terms, timeout_ms, minimize=(), maximize=()):
        self.calls += 1
        return SV.unknown, None


def _oracle_confirms(constraints, assignments):
    st = D.build_state([c.raw for c in constraints])
    model = {}
    for a in assignments:
        model.update(a)
    xs = [model.get(name, 0) for (name, _) in st.vars]
    return S.eval_root(st.nodes, st.consts, xs)


# ------------------------------------------------------------------ CPU side
def test_get_expr_variables():
    """independece_solver_test.py:12-40: the leaves of If(x, y, z + b) are x, y, z, b; a
    numeral is no leaf."""
    x = symbol_factory.BoolSym("x")
    y, z, b = BVS("y", 256), BVS("z", 256), BVS("b", 256)
    got = SV._get_expr_variables(If(x, y, z + b).raw)
    assert {"x", "y", "z", "b"} <= set(got)
    assert SV._get_expr_variables((b + BVV(2, 256)).raw) == ["b"]
    # an array select's leaf is the array; a UF application's function is no leaf
    arr, f = Array("cd", 256, 8), Function("keccak256_256", 256, 256)
    assert set(SV._get_expr_variables(arr[y].raw)) == {"cd", "y"}
    assert set(SV._get_expr_variables(f(y).raw)) == {"y"}


def test_create_bucket():
    """independece_solver_test.py:43-53."""
    x = symbol_factory.BoolSym("x")
    bucket = SV.DependenceBucket(["x"], [x.raw])
    assert bucket.variables == ["x"] and bucket.conditions == [x.raw]


def test_dependence_map():
    """independece_solver_test.py:56-85: [x > y, y == z, a == b] -> two buckets, {x, y, z}
    holding the first two conditions and {a, b} holding the third."""
    x, y, z, a, b = _xyzab()
    conditions = [(x > y).raw, (y == z).raw, (a == b).raw]
    dm = SV.DependenceMap()
    for c in conditions:
        dm.add_condition(c)
    assert len(dm.buckets) == 2
    assert set(dm.buckets[0].variables) == {"x", "y", "z"} and len(set(dm.buckets[0].variables)) == 3
    assert conditions[0] in dm.buckets[0].conditions and conditions[1] in dm.buckets[0].conditions
    assert set(dm.buckets[1].variables) == {"a", "b"}
    assert conditions[2] in dm.buckets[1].conditions


@pytest.mark.parametrize("name", sorted(UNSAT))
def test_unsat_pins_are_refuted_on_the_host(name):
    """Every UNSAT expectation is proven by the host pre-check (mgp_refute), the part of the
    pipeline that runs without a GPU; the concrete-index case folds to False on
    construction (laser.smt's simplify)."""
    from mythril_amd.front import Batch

    cs = UNSAT[name]()
    B = Batch([[c.raw for c in cs]])
    assert int(N.refute(*B.packed())[0]) == 1
    B.close()


@pytest.mark.parametrize("name", ["independence_sat"])
def test_sat_pin_is_not_refuted(name):
    from mythril_amd.front import Batch

    B = Batch([[c.raw for c in _independence_sat()]])
    assert int(N.refute(*B.packed())[0]) == 0
    B.close()


# ------------------------------------------------------------------ GPU side
@pytest.fixture()
def backend(mgp_ctx):
    b = CountingBackend()
    old = SV.set_backend(b)
    SV.SolverStatistics().reset()
    SV.unsat_cores().reset()
    SV.enable_gpu(True)
    yield b
    SV.set_backend(old)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(UNSAT))
@pytest.mark.parametrize("solver", ["Solver", "IndependenceSolver"])
def test_unsat_pins_refuted_no_fallback(backend, name, solver):
    """unsat through Solver and IndependenceSolver: refuted, no fallback; no GPU witness
    for the whole query (Solver) or for the contradictory bucket (IndependenceSolver
    batches every bucket, and a satisfiable bucket like {a == b} gets its own witness)."""
    cs = UNSAT[name]()
    s = getattr(SV, solver)()
    s.add(*cs)
    assert s.check() == SV.unsat
    st = SV.SolverStatistics()
    assert backend.calls == 0 and st.query_count == 0
    assert st.refuted >= 1
    if solver == "Solver":
        assert st.gpu_sat == 0
    else:
        dm = SV.DependenceMap()
        for c in cs:
            dm.add_condition(c.raw)
        assert st.gpu_sat + st.refuted == len(dm.buckets)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(UNSAT))
def test_unsat_pins_through_is_possible_and_get_model(backend, name):
    """The prune filter (constraints.py:34-51) drops the state, get_model raises UnsatError
    (analysis/solver.py:27-61), neither calls the fallback."""
    cs = UNSAT[name]()
    assert SV.Constraints(cs).is_possible is False
    with pytest.raises(SV.UnsatError):
        SV.get_model(tuple(cs))
    assert backend.calls == 0


@pytest.mark.gpu
@pytest.mark.parametrize("solver", ["Solver", "IndependenceSolver"])
def test_independence_sat_pin_gpu_witness(backend, solver):
    """independece_solver_test.py:128-145: sat, answered by GPU witnesses (one per bucket
    for IndependenceSolver) that the oracle confirms; no fallback call."""
    cs = _independence_sat()
    s = getattr(SV, solver)()
    s.add(*cs)
    assert s.check() == SV.sat
    assert backend.calls == 0
    m = s.model()
    assert len(m.assignments) == (2 if solver == "IndependenceSolver" else 1)
    assert _oracle_confirms(cs, m.assignments)


@pytest.mark.gpu
def test_prefilter_batch_of_pins(backend):
    """All pins in ONE Prefilter batch: the UNSAT ones refuted, the SAT one a witness."""
    pf = SV.prefilter()
    names = sorted(UNSAT) + ["independence_sat"]
    states = [[c.raw for c in (UNSAT[n]() if n in UNSAT else _independence_sat())] for n in names]
    res = pf.check_states(states)
    assert [r[0] for r in res] == [SV.unsat] * len(UNSAT) + [SV.sat]
    assert backend.calls == 0
    assert _oracle_confirms(_independence_sat(), [res[-1][1]])
    assert np.all([r[1] is None for r in res[:-1]])


def test_state_without_variables_through_refute_domains():
    """A batch whose only state folds to a literal False has no variable slot: the domain
    export (the pipeline's refute step) must accept an empty domain table (the GPU suite
    once failed here with 'mgp_refute failed')."""
    from mythril_amd.front import Batch

    B = Batch([[_concrete_calldata_constrain_index()[0].raw]])
    assert B.n_vars() == 0
    p = B.packed()
    ref, dom = N.refute_domains(*p[:4], B.var_off)
    assert list(ref) == [1] and dom.shape == (0, 33)
    B.close()
