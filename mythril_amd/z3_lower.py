"""z3 AST -> pre-filter terms: the boundary to the reference's own constraints.

In the reference every path constraint is a laser.smt Bool whose ``.raw`` is a z3
BoolRef (mythril/laser/smt/bool.py, constraints.py:41-50).  This walker turns such an
expression (any object with z3py's ExprRef surface) into the hash-consed terms of
mythril_amd.smt, which the native front end (csrc/mgp_front.cpp) flattens for the GPU.
It dispatches on ``decl().kind()`` against the ``Z3_OP_*`` constants of the module the
expression comes from (z3 is not pinned: requirements.txt:30 says ``z3-solver>=4.8.5.0``),
memoises by AST id, and covers the node set LASER builds:

  numerals, Bool / BitVec constants            symbol_factory (smt/__init__.py:83-154)
  bvadd bvsub bvmul bvudiv bvurem bvsdiv bvsrem bvsmod (n-ary, *_i variants), bvneg,
  bvand bvor bvxor bvnot, bvshl bvlshr bvashr, extract, concat, zero/sign_extend,
  repeat, rotate, bvcomp, bvredor/bvredand    bitvec.py:25-253, bitvec_helper.py:10-214
  = distinct ite and or not xor iff implies, unsigned / signed compares
  bvumul_noovfl (newer z3's BVMulNoOverflow)   bitvec_helper.py:183-196
  select / store / const-array (K)             array.py:16-63  -> read-over-write
  unary uninterpreted functions                function.py:7-25 (keccak256_<n>, keccak256_<n>-1)

Anything else raises Unsupported: the caller leaves that state to z3 unchanged.  The
walker also remembers where every variable and uninterpreted application came from
(``origin``), so a GPU witness can be re-checked by z3 (mythril_amd.z3_backend).
"""
from __future__ import annotations

import sys
import weakref
from typing import Dict, List, Optional, Sequence, Tuple

from . import ir
from . import smt as T
from .smt import Function, Term


class Unsupported(Exception):
    """A z3 construct outside the pre-filter's node set (the state stays with z3)."""


_OPS = ("TRUE FALSE EQ DISTINCT ITE AND OR IFF XOR NOT IMPLIES BNUM BNEG BADD BSUB BMUL BSDIV BUDIV BSREM BUREM "
        "BSMOD BSDIV_I BUDIV_I BSREM_I BUREM_I BSMOD_I ULEQ SLEQ UGEQ SGEQ ULT SLT UGT SGT BAND BOR BNOT BXOR "
        "BNAND BNOR BXNOR CONCAT SIGN_EXT ZERO_EXT EXTRACT REPEAT BREDOR BREDAND BCOMP BSHL BLSHR BASHR "
        "ROTATE_LEFT ROTATE_RIGHT BUMUL_NO_OVFL SELECT STORE CONST_ARRAY UNINTERPRETED").split()


class _Array:
    """An array value during the walk: a base array (uninterpreted, by name), a constant
    array K(v), or a store over another array."""

    __slots__ = ("kind", "fn", "expr", "value", "parent", "key", "val")

    def __init__(self, kind, fn=None, expr=None, value=None, parent=None, key=None, val=None):
        self.kind, self.fn, self.expr, self.value = kind, fn, expr, value
        self.parent, self.key, self.val = parent, key, val


class TermMap:
    """term id -> value, for as long as the term lives.

    An entry holds its term weakly: once the term is gone (its arena row may then be
    reused by a new term, smt._Arena.release) the entry reads as absent and is swept.
    Sweeps run when the map has doubled since the last one, so a long analysis keeps
    only the entries of terms that something still holds (amortised O(1) per insert)."""

    def __init__(self):
        self._d: Dict[int, Tuple["weakref.ref[Term]", object]] = {}
        self._sweep_at = 4096

    def setdefault(self, term: Term, value) -> None:
        cur = self._d.get(term.tid)
        if cur is not None and cur[0]() is term:
            return
        self._d[term.tid] = (weakref.ref(term), value)
        if len(self._d) >= self._sweep_at:
            self.sweep()

    def sweep(self) -> None:
        self._d = {k: v for k, v in self._d.items() if v[0]() is not None}
        self._sweep_at = max(4096, 2 * len(self._d))

    def get(self, tid: int, default=None):
        cur = self._d.get(tid)
        if cur is None or cur[0]() is None:
            return default
        return cur[1]

    def __getitem__(self, tid: int):
        cur = self._d.get(tid)
        if cur is None or cur[0]() is None:
            raise KeyError(tid)
        return cur[1]

    def __len__(self) -> int:
        return len(self._d)


class Z3Lowering:
    """z3 expressions of one z3 module -> mythril_amd.smt terms (memoised by AST id).

    Memory stays bounded over a long analysis: the AST memo is dropped whenever it
    passes `max_memo` entries (re-walking an AST gives the same hash-consed terms while
    they live), and `origin` / `roots` forget a term when it dies (TermMap)."""

    max_memo = 1 << 16

    def __init__(self, z3):
        self.z3 = z3
        self.k = {getattr(z3, "Z3_OP_" + n): n for n in _OPS if hasattr(z3, "Z3_OP_" + n)}
        self.memo: Dict[int, object] = {}
        self.funcs: Dict[str, Function] = {}
        # term id -> the z3 expression a variable / uninterpreted application term stands for
        # (a base-array read is (array expr, index expr)), and root term id -> z3 constraint
        self.origin = TermMap()
        self.roots = TermMap()

    # ------------------------------------------------------------------ API
    def lower(self, e) -> Term:
        """One z3 Bool or BitVec expression -> Term (raises Unsupported)."""
        if len(self.memo) > self.max_memo:
            self.memo.clear()  # the terms only the memo held die here ...
            self.origin.sweep()  # ... and so do their map entries (and the z3 ASTs they hold)
            self.roots.sweep()
        r = self._walk(e)
        if isinstance(r, _Array):
            raise Unsupported("array-valued expression")
        return r

    def lower_constraints(self, exprs: Sequence) -> List[Term]:
        out = []
        for e in exprs:
            t = self.lower(e)
            self.roots.setdefault(t, e)
            out.append(t)
        return out

    # ------------------------------------------------------------- helpers
    def _fn(self, name: str, dom: int, rng: int) -> Function:
        """The UF of a z3 function / array name; `<name>-1` is the inverse of `<name>`
        (keccak_function_manager.py:56-69)."""
        f = self.funcs.get(name)
        if f is None:
            if name.endswith("-1") and not name.startswith("array:"):
                fwd = self.funcs.get(name[:-2]) or self._fn(name[:-2], rng, dom)
                f = Function(name, dom, rng, inverse_of=fwd)
            else:
                f = Function(name, dom, rng)
            self.funcs[name] = f
        return f

    def _width(self, e) -> int:
        return int(e.size())

    def _ast_id(self, e) -> int:
        return int(e.get_id())

    def _walk(self, root):
        # memo: AST id -> (the z3 expression, its value).  Holding the expression keeps
        # z3 from recycling the id of a freed AST for a different one.
        stack: List[Tuple[object, bool]] = [(root, False)]
        memo = self.memo
        while stack:
            e, done = stack.pop()
            i = self._ast_id(e)
            if i in memo:
                continue
            kids = list(e.children())
            if not done:
                stack.append((e, True))
                for c in reversed(kids):
                    if self._ast_id(c) not in memo:
                        stack.append((c, False))
                continue
            memo[i] = (e, self._node(e, [memo[self._ast_id(c)][1] for c in kids], kids))
        return memo[self._ast_id(root)][1]

    def _select(self, arr: _Array, idx: Term, idx_expr) -> Term:
        """Read-over-write: select(store(a, k, v), i) = ite(i == k, v, select(a, i))."""
        chain = []
        a = arr
        while a.kind == "store":
            chain.append(a)
            a = a.parent
        if a.kind == "K":
            r = a.value
        else:
            f = a.fn
            r = T.mk(ir.UFAPP, f.range, (idx,), (f.fid, f.name))
            self.origin.setdefault(r, (a.expr, idx_expr))
        for st in reversed(chain):  # oldest store innermost
            r = T.ite(T.cmp_op(ir.EQ, idx, st.key), st.val, r)
        return r

    def _node(self, e, ch: list, kids: list):
        z3 = self.z3
        decl = e.decl()
        kind = self.k.get(decl.kind())
        if kind is None:
            raise Unsupported(f"z3 decl kind {decl.kind()} ({decl.name()})")
        sk = e.sort().kind()
        if kind == "UNINTERPRETED":
            name = str(decl.name())
            if sk == z3.Z3_ARRAY_SORT:
                if ch:
                    raise Unsupported("array-valued function")
                s = e.sort()
                f = self._fn("array:" + name, int(s.domain().size()), int(s.range().size()))
                return _Array("base", fn=f, expr=e)
            if not ch:
                if sk == z3.Z3_BOOL_SORT:
                    v = T.mk(ir.VAR, 1, (), (name,))
                    self.origin.setdefault(v, e)
                    return T.mk(ir.EQ, T.BOOL, (v, T.const(1, 1)))
                if sk != z3.Z3_BV_SORT:
                    raise Unsupported(f"constant of sort kind {sk}")
                v = T.mk(ir.VAR, self._width(e), (), (name,))
                self.origin.setdefault(v, e)
                return v
            if len(ch) != 1 or isinstance(ch[0], _Array) or ch[0].is_bool or sk != z3.Z3_BV_SORT:
                raise Unsupported(f"function {name}/{len(ch)}")
            f = self._fn(name, ch[0].width, self._width(e))
            if f.domain != ch[0].width or f.range != self._width(e):
                raise Unsupported(f"function {name} used at two signatures")
            op = ir.UFINV if f.inverse_of is not None else ir.UFAPP
            r = T.mk(op, f.range, (ch[0],), (f.fid, f.name))
            self.origin.setdefault(r, e)
            return r
        if kind == "SELECT":
            if not isinstance(ch[0], _Array):
                raise Unsupported("select over a non-array")
            return self._select(ch[0], ch[1], kids[1])
        if kind == "STORE":
            if not isinstance(ch[0], _Array) or isinstance(ch[2], _Array):
                raise Unsupported("store of an array value")
            return _Array("store", parent=ch[0], key=ch[1], val=ch[2])
        if kind == "CONST_ARRAY":
            if isinstance(ch[0], _Array):
                raise Unsupported("nested constant array")
            return _Array("K", value=ch[0])
        if any(isinstance(c, _Array) for c in ch):
            raise Unsupported(f"{kind} over an array")
        if kind == "TRUE":
            return T.bconst(True)
        if kind == "FALSE":
            return T.bconst(False)
        if kind == "BNUM":
            return T.const(int(e.as_long()), self._width(e))
        if kind == "NOT":
            return T.b_not(ch[0])
        if kind == "AND":
            return T.b_and(ch)
        if kind == "OR":
            return T.b_or(ch)
        if kind == "IMPLIES":
            return T.b_or([T.b_not(ch[0]), ch[1]])
        if kind in ("XOR", "IFF"):
            a, b = ch
            if T.is_const(a) and T.is_const(b):
                return T.bconst((T.cval(a) != T.cval(b)) == (kind == "XOR"))
            r = T.mk(ir.BXOR, T.BOOL, (a, b))
            return r if kind == "XOR" else T.b_not(r)
        if kind == "EQ":
            return self._eq(ch[0], ch[1])
        if kind == "DISTINCT":
            return T.b_and([T.b_not(self._eq(ch[i], ch[j])) for i in range(len(ch)) for j in range(i + 1, len(ch))])
        if kind == "ITE":
            return T.ite(ch[0], ch[1], ch[2])
        cmps = {"ULT": ir.ULT, "ULEQ": ir.ULE, "UGT": ir.UGT, "UGEQ": ir.UGE, "SLT": ir.SLT, "SLEQ": ir.SLE,
                "SGT": ir.SGT, "SGEQ": ir.SGE, "BUMUL_NO_OVFL": ir.UMUL_NOOVF}
        if kind in cmps:
            return T.cmp_op(cmps[kind], ch[0], ch[1])
        w = self._width(e)
        nary = {"BADD": ir.ADD, "BMUL": ir.MUL, "BAND": ir.AND, "BOR": ir.OR, "BXOR": ir.XOR}
        if kind in nary:
            r = ch[0]
            for c in ch[1:]:
                r = T.bv_op(nary[kind], r, c)
            return r
        binary = {"BSUB": ir.SUB, "BUDIV": ir.UDIV, "BUDIV_I": ir.UDIV, "BUREM": ir.UREM, "BUREM_I": ir.UREM,
                  "BSDIV": ir.SDIV, "BSDIV_I": ir.SDIV, "BSREM": ir.SREM, "BSREM_I": ir.SREM, "BSMOD": ir.SMOD,
                  "BSMOD_I": ir.SMOD, "BSHL": ir.SHL, "BLSHR": ir.LSHR, "BASHR": ir.ASHR}
        if kind in binary:
            return T.bv_op(binary[kind], ch[0], ch[1])
        if kind in ("BNAND", "BNOR", "BXNOR"):
            base = {"BNAND": ir.AND, "BNOR": ir.OR, "BXNOR": ir.XOR}[kind]
            return self._bvnot(T.bv_op(base, ch[0], ch[1]))
        if kind == "BNEG":
            return T.bv_op(ir.SUB, T.const(0, w), ch[0])
        if kind == "BNOT":
            return self._bvnot(ch[0])
        params = [int(p) for p in decl.params()]
        if kind == "EXTRACT":
            return T.extract(params[0], params[1], ch[0])
        if kind == "CONCAT":
            return T.concat(ch)
        if kind == "ZERO_EXT":
            return T.zext(ch[0], ch[0].width + params[0])
        if kind == "SIGN_EXT":
            a = ch[0]
            if params[0] == 0:
                return a
            if a.op == ir.CONST:
                v = T._signed(a.params[0], a.width)
                return T.const(v, a.width + params[0])
            return T.mk(ir.SEXT, a.width + params[0], (a,))
        if kind == "REPEAT":
            return T.concat([ch[0]] * params[0])
        if kind in ("ROTATE_LEFT", "ROTATE_RIGHT"):
            a, n = ch[0], params[0] % ch[0].width
            if kind == "ROTATE_RIGHT":
                n = (a.width - n) % a.width
            if n == 0:
                return a
            return T.concat([T.extract(a.width - n - 1, 0, a), T.extract(a.width - 1, a.width - n, a)])
        if kind == "BCOMP":
            return T.ite(self._eq(ch[0], ch[1]), T.const(1, 1), T.const(0, 1))
        if kind == "BREDOR":
            return T.ite(self._eq(ch[0], T.const(0, ch[0].width)), T.const(0, 1), T.const(1, 1))
        if kind == "BREDAND":
            return T.ite(self._eq(ch[0], T.const(-1, ch[0].width)), T.const(1, 1), T.const(0, 1))
        raise Unsupported(f"z3 op {kind}")

    def _eq(self, a: Term, b: Term) -> Term:
        if a.is_bool or b.is_bool:
            if not (a.is_bool and b.is_bool):
                raise Unsupported("Bool compared with BitVec")
            if T.is_const(a) and T.is_const(b):
                return T.bconst(T.cval(a) == T.cval(b))
            return T.mk(ir.BEQ, T.BOOL, (a, b))
        return T.cmp_op(ir.EQ, a, b)

    @staticmethod
    def _bvnot(a: Term) -> Term:
        if a.op == ir.CONST:
            return T.const(~a.params[0], a.width)
        return T.mk(ir.NOT, a.width, (a,))


_lowerings: Dict[int, Z3Lowering] = {}


def lowering_for(expr) -> Z3Lowering:
    """The walker of the z3 module `expr` belongs to (one per module)."""
    mod = sys.modules.get(type(expr).__module__)
    if mod is None or not hasattr(mod, "Z3_OP_TRUE"):
        raise Unsupported(f"not a z3 expression: {type(expr)!r}")
    w = _lowerings.get(id(mod))
    if w is None:
        w = _lowerings[id(mod)] = Z3Lowering(mod)
    return w


def lowering_of_module(z3) -> Optional[Z3Lowering]:
    """The walker that lowered expressions of the z3 package `z3` (its expressions live in
    a submodule, z3.z3, that shares the package's Solver class)."""
    for w in _lowerings.values():
        if getattr(w.z3, "Solver", None) is getattr(z3, "Solver", 0):
            return w
    return None


def z3_expr_of(t: Term):
    """The z3 expression a term was lowered from (a root constraint, a variable or an
    uninterpreted application; a base-array read becomes Select(array, index)), or None."""
    for w in _lowerings.values():
        e = w.roots.get(t.tid) or w.origin.get(t.tid)
        if e is not None:
            return w.z3.Select(e[0], e[1]) if isinstance(e, tuple) else e
    return None


def is_z3_expr(x) -> bool:
    return hasattr(x, "decl") and hasattr(x, "children") and hasattr(x, "get_id")


def to_terms(constraints: Sequence) -> Optional[List[Term]]:
    """Constraints given as z3 expressions (or laser.smt wrappers around them, `.raw`) ->
    terms, or None when some construct is outside the node set."""
    out = []
    try:
        for c in constraints:
            raw = c.raw if hasattr(c, "raw") and is_z3_expr(c.raw) else c
            out.extend(lowering_for(raw).lower_constraints([raw]))
    except Unsupported:
        return None
    return out
