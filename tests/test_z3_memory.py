"""Memory of the z3 boundary stays flat over a long analysis.

A `myth analyze` run lowers every path constraint it checks; the walker's AST memo, its
origin / root maps and the term arena must follow the LIVE queries, not every query ever
lowered.  10^5 fresh queries (new constants and shapes, names from a bounded pool, as
LASER's symbol names repeat across states) are lowered and dropped one by one; the
process RSS and the arena's row count must stay flat after warm-up.
"""
import gc
import os
import random

from mythril_amd import smt as T
from mythril_amd import z3_lower as ZL

from . import fake_z3 as z3


def _rss_kib() -> int:
    with open(f"/proc/{os.getpid()}/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1])
    return 0


def _query(rng, names):
    x, y = z3.BitVec(rng.choice(names), 256), z3.BitVec(rng.choice(names), 256)
    c = z3.BitVecVal(rng.getrandbits(256), 256)
    k = z3.BitVecVal(rng.getrandbits(64), 256)
    f = z3.Function("keccak256_256", z3.BitVecSort(256), z3.BitVecSort(256))
    return [z3.ULT(x + c, y), z3.Or(x * k == c, f(y) != c), z3.Extract(7, 0, y ^ c) == z3.BitVecVal(rng.getrandbits(8), 8)]


def _lower_many(n, rng, names):
    for _ in range(n):
        terms = ZL.to_terms(_query(rng, names))
        assert terms is not None and len(terms) == 3
        del terms


def test_lowering_memory_is_flat_over_1e5_queries():
    rng = random.Random(7)
    names = [f"calldata_{i}" for i in range(64)]
    lw = ZL.lowering_for(z3.BitVec("calldata_0", 256))
    lw.max_memo, max_memo = 1 << 13, lw.max_memo  # the bound under test, at a size that cycles often
    _lower_many(20_000, rng, names)  # warm-up: names interned, memo at its cap once
    assert len(lw.memo) <= lw.max_memo + 64
    # the memo is bounded by construction (max_memo ASTs, dropped when full); measure
    # what is left with it empty at both points
    lw.memo.clear()
    gc.collect()
    lw.origin.sweep()
    lw.roots.sweep()
    rss0, rows0 = _rss_kib(), len(T.ARENA.op)
    _lower_many(80_000, rng, names)
    assert len(lw.memo) <= lw.max_memo + 64
    lw.memo.clear()
    gc.collect()
    lw.origin.sweep()
    lw.roots.sweep()
    rss1, rows1 = _rss_kib(), len(T.ARENA.op)
    lw.max_memo = max_memo
    assert rows1 <= rows0 * 1.1 + 1024, (rows0, rows1)
    assert rss1 <= rss0 * 1.10, (rss0, rss1)
    # the maps hold only live terms after a sweep
    assert len(lw.roots) == 0 and len(lw.origin) <= 64 + 1


def test_reused_arena_rows_keep_dags_exact():
    """Rows of dead terms are reused: a term built afterwards can sit in an EARLIER row
    than its arguments, and the native front end must still flatten it exactly as the
    Python builder does."""
    from mythril_amd import ir

    from .test_front import _assert_same

    rng = random.Random(3)
    states, inverted = [], 0
    for k in range(4):
        junk = [T.const(rng.getrandbits(256), 256) for _ in range(300)]
        del junk
        T.ARENA.free.sort()  # any order is valid; ascending makes the next terms take rows downwards
        x, y = T.mk(ir.VAR, 256, (), (f"reuse_x{k}",)), T.mk(ir.VAR, 256, (), (f"reuse_y{k}",))
        s = T.bv_op(ir.ADD, x, T.const(rng.getrandbits(256), 256))
        states.append([T.cmp_op(ir.ULT, s, y), T.cmp_op(ir.EQ, T.bv_op(ir.XOR, s, y), T.const(k, 256))])
        inverted += states[-1][0].tid < x.tid
    assert inverted  # some user really sits in a row before its argument
    _assert_same(states)
