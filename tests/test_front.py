"""Native front end (csrc/mgp_front.cpp via mythril_amd.front.Batch) vs the Python
reference builder (mythril_amd.dag.build_state + pack_states): node for node, constant
for constant, variable tables, candidate hints, aliases, the GPU program's padded-key
strengthening and witness decoding must be identical (CPU only)."""
import numpy as np
import pytest

from mythril_amd import _native as N
from mythril_amd import dag as D
from mythril_amd import front as F
from corpus.keccak_manager import KeccakFunctionManager
from mythril_amd.smt import (Array, And, BVAddNoOverflow, BVMulNoOverflow, BVSubNoUnderflow, Concat, Extract, Function,
                             If, K, LShR, Not, Or, SRem, UDiv, UGE, UGT, ULE, ULT, URem, Xor, symbol_factory)

BVV, BVS = symbol_factory.BitVecVal, symbol_factory.BitVecSym


def _assert_same(states):
    raws = [[c.raw if hasattr(c, "raw") else c for c in st] for st in states]
    B = F.Batch(raws)
    dags = [D.build_state(r) for r in raws]
    p = D.pack_states(dags)
    g = D.pack_states(dags, gpu=True)
    assert np.array_equal(B.nodes, p[0])
    assert np.array_equal(B.gpu_nodes, g[0])
    assert np.array_equal(B.gpu_node_off, g[1])
    assert np.array_equal(B.node_off, p[1])
    assert np.array_equal(B.consts, p[2].reshape(-1, 8))
    assert np.array_equal(B.const_off, p[3])
    assert list(B.flags) == [d.flags for d in dags]
    for s, d in enumerate(dags):
        v0, v1 = int(B.var_off[s]), int(B.var_off[s + 1])
        assert B.var_names(s) == [n for n, _ in d.vars]
        assert list(B.var_width[v0:v1]) == [w for _, w in d.vars]
        assert [vi for vi in range(d.n_vars) if B.var_kind[v0 + vi] == 2] == sorted(d.pinned)
        for vi in range(d.n_vars):
            h = B.hints[int(B.hint_off[v0 + vi]): int(B.hint_off[v0 + vi + 1])]
            assert [int.from_bytes(x.tobytes(), "little") for x in h] == d.hints.get(vi, []), (s, vi)
        a = B.aliases[int(B.alias_off[s]): int(B.alias_off[s + 1])]
        assert [tuple(int(y) for y in x) for x in a] == d.aliases
        words = np.random.default_rng(s).integers(0, 2 ** 32, size=(d.n_vars, 8), dtype=np.uint64).astype(np.uint32)
        assert B.witness_to_model(s, words) == D.witness_to_model(d, words)
    B.close()
    return dags


def test_contract_shaped_states():
    import corpus

    _assert_same([[type("T", (), {"raw": t})() for t in c[1]] for c in corpus.corpus(96)])


def test_operator_zoo_wide_values_arrays_ufs():
    x, y, z = BVS("x", 256), BVS("y", 256), BVS("z", 160)
    w512 = Concat(x, y)
    f = Function("f", 512, 256)
    st = Array("Storage", 256, 256)
    st[x] = y + 1
    st[BVV(7, 256)] = x * y
    kk = K(256, 256, 3)
    kk[y] = BVV(9, 256)
    states = [
        [ULT(x, y), UGT(x + y, BVV(10, 256)), x * y == BVV(6, 256)],
        [UDiv(x, y) == BVV(3, 256), URem(x, BVV(64, 256)) == 0, SRem(x, y) != 0, LShR(x, BVV(3, 256)) == y],
        [Extract(159, 0, x) == z, Concat(z, Extract(95, 0, y)) == x],
        [f(w512) == x, f(Concat(y, x)) == y, Not(BVMulNoOverflow(x, y, False)), BVAddNoOverflow(x, y, False),
         BVSubNoUnderflow(y, x, False)],
        [st[z.raw and Concat(BVV(0, 96), z)] == x, st[BVV(7, 256)] == y, kk[x] == BVV(3, 256)],
        [If(ULT(x, y), x, y) == BVV(5, 256), Or(x == 1, Xor(y == 2, x == y)), x < y, x >= y],
        [],
        [x == x + 0, ULE(x, BVV(100, 256)), UGE(y, BVV(2 ** 255, 256))],
        [w512 == Concat(BVV(1, 256), BVV(2, 256)), ULT(w512, Concat(y, x))],
    ]
    _assert_same(states)


def test_padded_key_equalities_strengthened_by_polarity(monkeypatch):
    from oracle.keccak_ref import keccak256  # no GPU here: concrete hashes from the checker

    monkeypatch.setattr(KeccakFunctionManager, "find_concrete_keccak", staticmethod(
        lambda d: BVV(int.from_bytes(keccak256(d.value.to_bytes(d.size() // 8, "big")), "big"), 256)))
    km = KeccakFunctionManager()
    n1 = BVS("N1", 256)
    o1, c1 = km.create_keccak(BVV(100, 8))    # concrete 8-bit key: its hash joins concrete_hashes
    o0, c0 = km.create_keccak(BVV(100, 256))  # same-width key
    o2, c2 = km.create_keccak(n1)             # symbolic: OR over (f(N1) == H_k and key_k == N1)
    pos = [And(c1, c0, c2), o1 == o2]
    neg = [c2, Not(BVV(5, 8) == BVS("q", 256))]            # padded equality under a negation
    mixed = [Xor(BVV(5, 8) == BVS("q", 256), BVS("r", 256) == 1)]  # both polarities
    none = [BVS("a", 256) == BVV(5, 256)]
    # the padded equality reached only through a BV context: If(eq, 1, 0) == 1, the shape
    # LASER's EQ / ISZERO instructions build: flagged, not left unstrengthened
    from mythril_amd.smt import If
    bvctx = [If(BVV(5, 8) == BVS("q", 256), BVV(1, 256), BVV(0, 256)) == BVV(1, 256)]
    dags = _assert_same([pos, neg, mixed, none, bvctx])
    assert dags[0].flags == 2 and set(dags[0].gpu_ops.values()) == {4}   # FALSE
    assert dags[1].flags == 2 and 3 in dags[1].gpu_ops.values()          # TRUE
    assert dags[2].flags & 1
    assert dags[3].flags == 0 and not dags[3].gpu_ops
    assert dags[4].flags & 1 and not dags[4].gpu_ops


def test_empty_batch_and_state():
    B = F.Batch([])
    assert B.n_states == 0 and len(B.node_off) == 1
    B.close()
    _assert_same([[]])


def test_mixed_corpus_with_pinned_constants():
    """suicide / BECToken / WalletLibrary shapes (corpus.py): several calldata words push the
    constant pool past MGP_FE_POOL_KEEP, so the GPU program pins the rest."""
    import corpus

    dags = _assert_same([[type("T", (), {"raw": t})() for t in c[1]] for c in corpus.corpus(40)])
    assert any(d.flags & 4 for d in dags) and any(d.pinned for d in dags)
    for d in dags:  # the GPU program's front VAR nodes read exactly the pinned slots
        if d.gpu_nodes is not None and d.flags & 4:
            front = [n for n in d.gpu_nodes[: len(d.gpu_nodes) - len(d.nodes)]]
            assert all(n[0] == 1 for n in front) and {n[5] for n in front} <= set(d.pinned)


def test_select_equals_a_build_of_the_selected_states():
    """Batch.select (mgp_fe_select, how Prefilter cuts its candidate-memory groups and retry
    rounds out of one build): every field equals a fresh build of the selected states --
    permuted, repeated and pinned states, an empty selection, a select of a select."""
    import corpus

    cs = [c[1] for c in corpus.corpus(96)]
    B = F.Batch(cs)
    assert (B.flags & 4).any() and not (B.flags & 4).all()  # pinned and unpinned states
    picks = [list(range(0, 96, 3)), [95, 2, 2, 40, 7], [int(i) for i in np.random.default_rng(3).permutation(96)],
             [], [i for i in range(96) if not B.flags[i] & 6]]
    for idx in picks:
        S, R = B.select(idx), F.Batch([cs[i] for i in idx])
        for name in F._FIELDS:
            assert np.array_equal(getattr(S, name), getattr(R, name)), (name, idx[:6])
        if idx:
            sub = list(range(len(idx)))[::-2]
            S2, R2 = S.select(sub), F.Batch([cs[idx[k]] for k in sub])
            for name in F._FIELDS:
                assert np.array_equal(getattr(S2, name), getattr(R2, name)), name
            S2.close()
            R2.close()
        S.close()
        R.close()
    with pytest.raises(N.MgpError):
        B.select([96])
    B.close()
