"""Study tool: one restated suite query through the decision rows on the CPU.

usage: python scripts/row_probe.py CONTRACT QUERY_INDEX [n_rows] [--print]

Builds the contract's queries (corpus.suite, CPU Keccak), takes query QUERY_INDEX (its index
within the contract's queries), computes n_rows unseeded decision rows (mgp_decision_rows) and
reports for each row whether it satisfies the GPU formula (the C oracle) and, if not, which
root conjuncts it violates.  --print dumps the query's conjuncts as s-expressions (shared
subterms named once)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import corpus  # noqa: E402
from mythril_amd import _native as N  # noqa: E402
from mythril_amd import dag as D  # noqa: E402
from mythril_amd import front as F  # noqa: E402
from mythril_amd import ir  # noqa: E402
from oracle import bvsem as S  # noqa: E402
from oracle import coracle  # noqa: E402
from oracle.keccak_ref import keccak256  # noqa: E402


def sexpr(roots, max_len=400):
    """Conjuncts as s-expressions; a subterm used more than once is printed once as $k."""
    uses = {}

    def count(t):
        stack = [t]
        while stack:
            x = stack.pop()
            uses[id(x)] = uses.get(id(x), 0) + 1
            if uses[id(x)] == 1:
                stack.extend(x.args)
    for r in roots:
        count(r)
    names = {}
    lines = []

    def show(t, top=False):
        if id(t) in names:
            return names[id(t)]
        op = ir.OP_NAMES.get(t.op, str(t.op))
        if t.op == ir.CONST:
            v = t.params[0]
            s = hex(v) if v > 4096 else str(v)
        elif t.op == ir.VAR:
            s = str(t.params[0])
        else:
            ps = "" if not t.params or t.op in (ir.UFAPP, ir.UFINV) else "[" + ",".join(map(str, t.params)) + "]"
            fn = f"<{t.params[1]}>" if t.op in (ir.UFAPP, ir.UFINV) else ""
            s = f"({op}{ps}{fn} " + " ".join(show(a) for a in t.args) + ")"
        if not top and uses.get(id(t), 0) > 1 and len(s) > 12:
            names[id(t)] = f"${len(names)}"
            lines.append(f"  {names[id(t)]} = {s[:max_len]}")
            return names[id(t)]
        return s
    out = []
    for r in roots:
        out.append(show(r, top=True)[:max_len])
    return lines, out


def node_index(terms):
    """{id(term): node index} as dag.build_state numbers the nodes (same DFS)."""
    memo, n = {}, 0
    for root in terms:
        stack = [(root, False)]
        while stack:
            t, done = stack.pop()
            if id(t) in memo:
                continue
            if done:
                memo[id(t)] = n
                n += 1
                continue
            stack.append((t, True))
            for a in reversed(t.args):
                if id(a) not in memo:
                    stack.append((a, False))
    return memo


def explain(terms, k, vals, memo, depth=3, indent="    "):
    """Print the value of conjunct k's Bool subterms down to `depth` levels."""
    def walk(t, d, pre):
        v = vals[memo[id(t)]]
        op = ir.OP_NAMES.get(t.op, str(t.op))
        s = v if isinstance(v, bool) else hex(v)
        print(f"{pre}{op} = {s}")
        if d > 0 and t.op in (ir.BAND, ir.BOR, ir.BNOT, ir.EQ, ir.ULT, ir.ITE, ir.UGT):
            for a in t.args:
                walk(a, d - 1, pre + "  ")
    walk(terms[k], depth, indent)


def main():
    name, qi = sys.argv[1], int(sys.argv[2])
    n_rows = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3].isdigit() else 8
    qs = corpus.suite(hasher=keccak256, contracts={name})
    q = qs[qi]
    print(q[1], q[2], "expected", q[4], "parent", q[5])
    terms = list(q[3])
    if "--print" in sys.argv:
        lines, roots = sexpr(terms)
        print("\n".join(lines))
        for k, r in enumerate(roots):
            print(f"C{k}: {r}")
    B = F.Batch([terms])
    nv = max(1, B.n_vars())
    rows, mask, st = N.decision_rows(*B.packed(decide=True), nv, 0x1234, n_rows, np.array([n_rows], np.uint8),
                                     state_keys=B.state_key, seed_rows=0)
    ref = N.refute(*B.packed())
    print("refute:", int(ref[0]), "decision status:", int(st[0]), "vars:", B.n_vars(0))
    st_dag = D.build_state(terms)
    # the rows as mgp_check_batch places them (mixture rows 2.., pinned constants kept)
    from tests import fe_emulate as E
    cand = N.make_candidates(n_rows + 2, nv, 0x1234, B.var_off, B.var_width, B.hint_off, B.hints, B.alias_off,
                             B.aliases, B.const_off, B.consts, D._FIXED_LIMBS, np.zeros(1, np.uint8),
                             var_kind=B.var_kind, state_keys=B.state_key)
    E.apply_xrows(B, cand, rows, mask)
    for r in range(n_rows):
        c = cand[0, 2 + r].copy()
        ok = coracle.first_sat(*B.packed(gpu=True), c[None, None])[0]
        first_bad = None
        if ok != 0:
            # the first prefix And(terms[:k+1]) the row falsifies (a prefix DAG numbers its
            # nodes -- and so its UF application names -- as the full one does)
            slots = [int.from_bytes(c[i].tobytes(), "little") for i in range(st_dag.n_vars)]
            model = dict(zip([v[0] for v in st_dag.vars], slots))
            for k in range(len(terms)):
                sd = D.build_state(terms[:k + 1])
                if not S.eval_root(sd.nodes, sd.consts, D.model_to_slots(sd, model)):
                    first_bad = k
                    break
            if first_bad is not None and "--explain" in sys.argv and r == int(os.environ.get("ROW", "0")):
                vals = S.eval_dag(st_dag.nodes, st_dag.consts, D.model_to_slots(st_dag, model))
                explain(terms, first_bad, vals, node_index(terms), depth=int(os.environ.get("DEPTH", "4")))
        print(f"row {r}: {'SAT' if ok == 0 else 'no'}  first violated conjunct {first_bad}  "
              f"decided slots {int(mask[0, r].sum())}")
    B.close()


if __name__ == "__main__":
    main()
