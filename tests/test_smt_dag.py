"""laser.smt mirror -> DAG -> bytecode, checked against the oracle on CPU."""
import numpy as np

from mythril_amd import _native as N
from mythril_amd import dag as D
from mythril_amd import ir
from mythril_amd.smt import (UGE, UGT, ULE, ULT, And, Array, BVAddNoOverflow, BVMulNoOverflow, BVSubNoUnderflow,
                             Concat, Extract, Function, If, K, LShR, Not, Or, SRem, Sum, UDiv, URem, Xor,
                             symbol_factory)
from oracle import bvsem as S
from oracle import bytecode_ref as BR

BVV = symbol_factory.BitVecVal
BV = symbol_factory.BitVecSym


def _check(constraints, rows_fn, n=40, seed=0):
    st = D.build_state([c.raw for c in constraints])
    nodes, noff, consts, coff = D.pack_states([st])
    words, po, status = N.lower(nodes, noff, consts, coff)
    assert status[0] == 0
    rng = np.random.default_rng(seed)
    cands = D.make_candidates([st], n, max(1, st.n_vars), seed=seed)
    nl = [tuple(int(x) for x in (r["op"], r["flags"], r["width"], r["a"], r["b"], r["c"], r["p0"], r["p1"]))
          for r in nodes]
    nl = [(o, w, a, b, c, p0, p1) for (o, _, w, a, b, c, p0, p1) in nl]
    cl = list(st.consts)
    hits = 0
    for c in range(n):
        xs = [S.limbs_to_int(cands[0, c, v]) for v in range(st.n_vars)]
        want = S.eval_root(nl, cl, xs)
        assert BR.run_program(words, int(po[0]), xs) == want
        hits += want
    return st, hits


def test_operator_semantics_mirror_reference():
    a, b = BV("a", 256), BV("b", 256)
    # BitVec < is SIGNED (bitvec.py:138), / is bvsdiv (bitvec.py:96), >> is bvashr (bitvec.py:240)
    assert (a < b).raw.op == ir.SLT and (a / b).raw.op == ir.SDIV and (a >> b).raw.op == ir.ASHR
    assert ULT(a, b).raw.op == ir.ULT and LShR(a, b).raw.op == ir.LSHR
    # ULE / UGE are Or(ULT, ==) (bitvec_helper.py:53-80)
    assert ULE(a, b).raw.op == ir.BOR and UGE(a, b).raw.op == ir.BOR
    # == pads the narrower side (bitvec.py:16-22)
    e = BV("x", 8) == BV("y", 256)
    assert e.raw.op == ir.EQ and e.raw.args[0].op == ir.ZEXT
    # concrete folding mirrors z3 simplify
    assert (BVV(5, 256) + BVV(7, 256)).value == 12
    assert UDiv(BVV(5, 256), BVV(0, 256)).value == 2 ** 256 - 1
    assert URem(BVV(5, 256), BVV(0, 256)).value == 5
    assert (BVV(2 ** 256 - 1, 256) / BVV(0, 256)).value == 1
    assert SRem(BVV(2 ** 256 - 7, 256), BVV(3, 256)).value == 2 ** 256 - 1
    assert (BVV(1, 256) << BVV(300, 256)).value == 0
    assert (BVV(2 ** 255, 256) >> BVV(300, 256)).value == 2 ** 256 - 1
    assert Extract(15, 8, BVV(0xABCD, 256)).value == 0xAB
    assert Concat(BVV(1, 8), BVV(2, 8)).value == 0x0102
    assert (BVV(3, 256) < BVV(2 ** 256 - 1, 256)).value is False  # 3 < -1 signed
    assert If(True, BVV(1, 256), BVV(2, 256)).value == 1
    assert And(True, BV("q", 256) == 1).symbolic and And(False, BV("q", 256) == 1).is_false


def test_symbolic_mixture_lowering():
    a, b, c = BV("a", 256), BV("b", 256), BV("c", 160)
    cs = [
        ULT(a, BVV(1000, 256)),
        Or(a * b == BVV(24, 256), UGT(b, a)),
        Not(Extract(7, 0, a) == Extract(15, 8, b)),
        BVMulNoOverflow(a, b, False),
        BVAddNoOverflow(a, b, False),
        BVSubNoUnderflow(BVV(2000, 256), a, False),
        Xor(Concat(BVV(0, 96), c) == b, a == BVV(7, 256)),
        If(a < b, UDiv(b, a + 1), SRem(a, b)) != Sum(a, b, BVV(3, 256)),
    ]
    _check(cs, None, n=48)


def test_arrays_read_over_write():
    storage = Array("Storage", 256, 256)
    k, v = BV("k", 256), BV("v", 256)
    storage[BVV(1, 256)] = v
    storage[k] = BVV(9, 256)
    sel = storage[BVV(1, 256)]
    # storage[1] == (k == 1 ? 9 : v)
    st, _ = _check([sel == BVV(9, 256)], None, n=30)
    # storage[1] was written (with v) before the symbolic write: read-over-write resolves it
    # to ITE(k == 1, 9, v) with no read of the base array left
    assert not any(n[0] == ir.UFAPP for n in st.nodes) and any(n[0] == ir.ITE for n in st.nodes)
    kk = K(256, 256, 0)
    kk[k] = v
    _check([kk[BVV(5, 256)] == BVV(0, 256), kk[k] == v], None, n=10)


def test_uf_pairs_and_hints():
    f = Function("f_256", 256, 256)
    inv = Function("f_256-1", 256, 256, inverse_of=f)
    x, y = BV("x", 256), BV("y", 256)
    cs = [inv(f(x)) == x, f(x) == f(y), ULE(BVV(1 << 200, 256), f(x)), URem(f(y), BVV(64, 256)) == 0]
    st, hits = _check(cs, None, n=64)
    assert st.aliases, "x == y style aliases should be harvested"
    assert any(v % 64 == 0 and v >= 1 << 200 for vals in st.hints.values() for v in vals)


def test_bool_symbols_and_constants():
    p = symbol_factory.BoolSym("p")
    x = BV("x", 256)
    _check([Or(p, x == BVV(3, 256)), Not(p) == (x == BVV(3, 256))], None, n=20)
    st = D.build_state([symbol_factory.Bool(True).raw])
    assert st.nodes[-1][0] == ir.TRUE


def test_wide_mapping_preimage_state_lowers_and_candidates_satisfy():
    """keccak256_512(Concat(key, slot)) with the manager's condition (keccak_function_manager.py:122-146):
    the 512-bit preimage and inverse lower to narrow pieces, and the candidates (hints plus
    domain-guided rows) include a model (checked with the CPU uop interpreter, no GPU)."""
    from mythril_amd import _native as N
    from corpus.keccak_manager import KeccakFunctionManager
    from mythril_amd.smt import Concat, ULT, symbol_factory
    from oracle import bvsem as S
    from oracle import uop_ref as UR
    from tests._util import pack_states

    kfm = KeccakFunctionManager()
    key = symbol_factory.BitVecSym("key", 256)
    h, cond = kfm.create_keccak(Concat(key, symbol_factory.BitVecVal(3, 256)))
    st = D.build_state([cond.raw, ULT(key, symbol_factory.BitVecVal(1000, 256)).raw])
    assert st.wide, "inverse result is a wide (512-bit) fresh value"
    (vi, w), = st.wide.items()
    assert w == 512 and st.vars[vi + 1][0].endswith("#1")
    nodes, noff, consts, coff = pack_states([(st.nodes, st.consts)])
    words, po, status = N.lower(nodes, noff, consts, coff)
    assert status[0] == N.ST_OK
    cands = D.make_candidates([st], 64, st.n_vars)
    # as in the product's second round: every other row drawn from the pre-check's domains
    assert N.guided_candidates(nodes, noff, consts, coff, cands, every=2, n_decide=8)[0] == 0
    hits = 0
    for c in range(64):
        xs = [S.limbs_to_int(cands[0, c, v]) for v in range(st.n_vars)]
        want = S.eval_root(st.nodes, st.consts, xs)
        assert UR.run_uops(words, int(po[0]), xs) == want
        hits += want
    assert hits > 0
    model = D.witness_to_model(st, cands[0, 0])
    assert D.model_to_slots(st, model) == [S.limbs_to_int(cands[0, 0, v]) & ((1 << st.vars[v][1]) - 1)
                                           for v in range(st.n_vars)]


def test_native_candidates_layout_and_rows():
    """mgp_make_candidates (via dag.make_candidates): parent row, hint row, alias row,
    width masks, determinism in the seed."""
    from mythril_amd.smt import symbol_factory as sf
    x8, y8, z = sf.BitVecSym("x8", 8), sf.BitVecSym("y8", 8), sf.BitVecSym("z", 256)
    st = D.build_state([(x8 == sf.BitVecVal(0x41, 8)).raw, (x8 == y8).raw, ULT(z, sf.BitVecVal(1000, 256)).raw])
    names = [n for (n, _) in st.vars]
    ix, iy, iz = names.index("x8"), names.index("y8"), names.index("z")
    a = D.make_candidates([st], 64, st.n_vars, seed=9)
    b = D.make_candidates([st], 64, st.n_vars, seed=9)
    assert np.array_equal(a, b)
    assert not np.array_equal(a, D.make_candidates([st], 64, st.n_vars, seed=10))
    assert (a[0, :, ix, 1:] == 0).all() and (a[0, :, ix, 0] <= 0xFF).all()  # 8-bit slots masked
    assert a[0, 0, ix, 0] == 0x41                                           # first hint row
    assert a[0, 1, iy, 0] == 0x41                                           # alias row: y8 := x8
    assert S.limbs_to_int(a[0, 0, iz]) in st.hints[iz]
    p = D.make_candidates([st], 64, st.n_vars, seed=9, parents=[{"z": 7, "x8": 0x41}])
    assert S.limbs_to_int(p[0, 0, iz]) == 7 and p[0, 0, ix, 0] == 0x41 and p[0, 1, ix, 0] == 0x41
    assert sum(S.eval_root(st.nodes, st.consts, [S.limbs_to_int(a[0, c, v]) for v in range(st.n_vars)])
               for c in range(64)) > 0


def test_arena_rows_never_shared_between_live_terms():
    """arena rows are freed by a weakref callback, after every weakref to the
    dying term is cleared, so no thread can fetch a dying term from the intern table and
    keep it alive on a freed row.  Terms are built and dropped by four threads at once;
    afterwards every live interned term owns a distinct row that is not on the free list."""
    import gc
    import threading

    from mythril_amd import smt as M

    def churn(seed):
        x = BV(f"churn_{seed % 2}", 256)
        for i in range(3000):
            t = (x + BVV(i % 97, 256)) * BVV(seed + 1, 256)
            u = ULT(t, BVV(i % 13, 256))
            del t, u

    th = [threading.Thread(target=churn, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    keep = [BV("kept", 256) + BVV(k, 256) for k in range(50)]
    gc.collect()
    live = list(M._INTERN.values())
    tids = [t.tid for t in live]
    assert len(set(tids)) == len(tids)
    assert not set(tids) & set(M.ARENA.free)
    assert all(M._ROW_REFS[t.tid]() is t for t in live)
    assert len(keep) == 50
