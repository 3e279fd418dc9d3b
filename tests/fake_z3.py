"""A stand-in for z3py (test infrastructure): z3 is not installed here or on the GPU box.

It reproduces the part of z3py's API the pre-filter's z3 boundary reads
(mythril_amd/z3_lower.py, mythril_amd/z3_backend.py) and the constructors the
reference's laser.smt layer calls (mythril/laser/smt/*.py), with its own
Z3_OP_* numbering, plus a concrete evaluator written from the SMT-LIB bit-vector
semantics (division by zero, signed ops, shifts >= width) so that the walker's output
can be checked against an independent reading of every operator.  The Solver only
decides constraint sets whose free constants are pinned by `x == value` conjuncts
(enough for witness re-checks); anything else is `unknown`.  Results against it are
"parity unpinned" with respect to real z3.
"""
from __future__ import annotations

import itertools
from typing import Dict

Z3_BOOL_SORT, Z3_BV_SORT, Z3_ARRAY_SORT = 1, 4, 5
_names = ("TRUE FALSE EQ DISTINCT ITE AND OR IFF XOR NOT IMPLIES BNUM BNEG BADD BSUB BMUL BSDIV BUDIV BSREM BUREM "
          "BSMOD ULEQ SLEQ UGEQ SGEQ ULT SLT UGT SGT BAND BOR BNOT BXOR CONCAT SIGN_EXT ZERO_EXT EXTRACT REPEAT "
          "BREDOR BREDAND BCOMP BSHL BLSHR BASHR ROTATE_LEFT ROTATE_RIGHT BUMUL_NO_OVFL SELECT STORE CONST_ARRAY "
          "UNINTERPRETED FP_ADD").split()
for _i, _n in enumerate(_names):
    globals()["Z3_OP_" + _n] = 7000 + _i

_ids = itertools.count(1)


class CheckSatResult:
    def __init__(self, s):
        self.s = s

    def __eq__(self, o):
        return isinstance(o, CheckSatResult) and o.s == self.s

    def __repr__(self):
        return self.s


sat, unsat, unknown = CheckSatResult("sat"), CheckSatResult("unsat"), CheckSatResult("unknown")


class SortRef:
    def __init__(self, kind, size=0, dom=None, rng=None):
        self._k, self._size, self._dom, self._rng = kind, size, dom, rng

    def kind(self):
        return self._k

    def size(self):
        return self._size

    def domain(self):
        return self._dom

    def range(self):
        return self._rng


def BitVecSort(w):
    return SortRef(Z3_BV_SORT, w)


def BoolSort():
    return SortRef(Z3_BOOL_SORT)


def ArraySort(d, r):
    return SortRef(Z3_ARRAY_SORT, 0, d, r)


class FuncDeclRef:
    def __init__(self, kind, name, params=(), dom=(), rng=None):
        self._k, self._name, self._params, self._dom, self._rng = kind, name, tuple(params), tuple(dom), rng

    def kind(self):
        return self._k

    def name(self):
        return self._name

    def params(self):
        return list(self._params)

    def arity(self):
        return len(self._dom)

    def __call__(self, *args):
        args = [_bv(a, d.size()) for a, d in zip(args, self._dom)]
        return _mk(self, self._rng, args)


def Function(name, *sorts):
    return FuncDeclRef(Z3_OP_UNINTERPRETED, name, (), sorts[:-1], sorts[-1])


class ExprRef:
    def __init__(self, decl, sort, args):
        self._decl, self._sort, self._args, self._id = decl, sort, list(args), next(_ids)

    def decl(self):
        return self._decl

    def children(self):
        return list(self._args)

    def num_args(self):
        return len(self._args)

    def arg(self, i):
        return self._args[i]

    def get_id(self):
        return self._id

    def sort(self):
        return self._sort

    def size(self):
        return self._sort.size()

    def as_long(self):
        if self._decl.kind() != Z3_OP_BNUM:
            raise AttributeError("not a numeral")
        return self._decl.params()[0]

    def __hash__(self):
        return self._id

    # Bool
    def __eq__(self, o):
        if self._sort.kind() == Z3_BOOL_SORT:
            return _mk(FuncDeclRef(Z3_OP_EQ, "="), BoolSort(), [self, _bool(o)])
        return _mk(FuncDeclRef(Z3_OP_EQ, "="), BoolSort(), [self, _bv(o, self.size())])

    def __ne__(self, o):
        return Not(self == o)

    # BitVec arithmetic (z3py operator meanings)
    def _b(self, kind, name, o, rev=False):
        o = _bv(o, self.size())
        a, b = (o, self) if rev else (self, o)
        return _mk(FuncDeclRef(kind, name), BitVecSort(self.size()), [a, b])

    def __add__(self, o): return self._b(Z3_OP_BADD, "bvadd", o)
    def __radd__(self, o): return self._b(Z3_OP_BADD, "bvadd", o, True)
    def __sub__(self, o): return self._b(Z3_OP_BSUB, "bvsub", o)
    def __rsub__(self, o): return self._b(Z3_OP_BSUB, "bvsub", o, True)
    def __mul__(self, o): return self._b(Z3_OP_BMUL, "bvmul", o)
    def __rmul__(self, o): return self._b(Z3_OP_BMUL, "bvmul", o, True)
    def __truediv__(self, o): return self._b(Z3_OP_BSDIV, "bvsdiv", o)
    def __mod__(self, o): return self._b(Z3_OP_BSMOD, "bvsmod", o)
    def __and__(self, o): return self._b(Z3_OP_BAND, "bvand", o)
    def __or__(self, o): return self._b(Z3_OP_BOR, "bvor", o)
    def __xor__(self, o): return self._b(Z3_OP_BXOR, "bvxor", o)
    def __lshift__(self, o): return self._b(Z3_OP_BSHL, "bvshl", o)
    def __rshift__(self, o): return self._b(Z3_OP_BASHR, "bvashr", o)
    def __neg__(self): return _mk(FuncDeclRef(Z3_OP_BNEG, "bvneg"), self._sort, [self])
    def __invert__(self): return _mk(FuncDeclRef(Z3_OP_BNOT, "bvnot"), self._sort, [self])

    def _c(self, kind, o):
        return _mk(FuncDeclRef(kind, "cmp"), BoolSort(), [self, _bv(o, self.size())])

    def __lt__(self, o): return self._c(Z3_OP_SLT, o)
    def __le__(self, o): return self._c(Z3_OP_SLEQ, o)
    def __gt__(self, o): return self._c(Z3_OP_SGT, o)
    def __ge__(self, o): return self._c(Z3_OP_SGEQ, o)

    # arrays
    def __getitem__(self, i):
        return Select(self, i)


def _mk(decl, sort, args):
    return ExprRef(decl, sort, args)


def _bv(x, w):
    return x if isinstance(x, ExprRef) else BitVecVal(x, w)


def _bool(x):
    return x if isinstance(x, ExprRef) else BoolVal(bool(x))


def BitVec(name, w):
    return _mk(FuncDeclRef(Z3_OP_UNINTERPRETED, name), BitVecSort(w), [])


def BitVecVal(v, w):
    return _mk(FuncDeclRef(Z3_OP_BNUM, "bv", (int(v) % (1 << w), w)), BitVecSort(w), [])


def Bool(name):
    return _mk(FuncDeclRef(Z3_OP_UNINTERPRETED, name), BoolSort(), [])


def BoolVal(b):
    return _mk(FuncDeclRef(Z3_OP_TRUE if b else Z3_OP_FALSE, str(b).lower()), BoolSort(), [])


def Array(name, dom, rng):
    return _mk(FuncDeclRef(Z3_OP_UNINTERPRETED, name), ArraySort(dom, rng), [])


def K(dom, v):
    return _mk(FuncDeclRef(Z3_OP_CONST_ARRAY, "K"), ArraySort(dom, v.sort()), [v])


def Select(a, i):
    return _mk(FuncDeclRef(Z3_OP_SELECT, "select"), a.sort().range(), [a, _bv(i, a.sort().domain().size())])


def Store(a, i, v):
    return _mk(FuncDeclRef(Z3_OP_STORE, "store"), a.sort(),
               [a, _bv(i, a.sort().domain().size()), _bv(v, a.sort().range().size())])


def _nary_bool(kind, name, args):
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        args = args[0]
    return _mk(FuncDeclRef(kind, name), BoolSort(), [_bool(a) for a in args])


def And(*a): return _nary_bool(Z3_OP_AND, "and", a)
def Or(*a): return _nary_bool(Z3_OP_OR, "or", a)
def Not(a): return _mk(FuncDeclRef(Z3_OP_NOT, "not"), BoolSort(), [_bool(a)])
def Xor(a, b): return _mk(FuncDeclRef(Z3_OP_XOR, "xor"), BoolSort(), [_bool(a), _bool(b)])
def Implies(a, b): return _mk(FuncDeclRef(Z3_OP_IMPLIES, "=>"), BoolSort(), [_bool(a), _bool(b)])
def Distinct(*a): return _mk(FuncDeclRef(Z3_OP_DISTINCT, "distinct"), BoolSort(), list(a))


def If(c, a, b):
    if isinstance(a, ExprRef) and a.sort().kind() == Z3_BV_SORT:
        b = _bv(b, a.size())
    elif isinstance(b, ExprRef) and b.sort().kind() == Z3_BV_SORT:
        a = _bv(a, b.size())
    return _mk(FuncDeclRef(Z3_OP_ITE, "if"), a.sort(), [_bool(c), a, b])


def Concat(*a):
    if len(a) == 1 and isinstance(a[0], (list, tuple)):
        a = a[0]
    return _mk(FuncDeclRef(Z3_OP_CONCAT, "concat"), BitVecSort(sum(x.size() for x in a)), list(a))


def Extract(hi, lo, a):
    return _mk(FuncDeclRef(Z3_OP_EXTRACT, "extract", (hi, lo)), BitVecSort(hi - lo + 1), [a])


def ZeroExt(n, a):
    return _mk(FuncDeclRef(Z3_OP_ZERO_EXT, "zero_extend", (n,)), BitVecSort(a.size() + n), [a])


def SignExt(n, a):
    return _mk(FuncDeclRef(Z3_OP_SIGN_EXT, "sign_extend", (n,)), BitVecSort(a.size() + n), [a])


def RepeatBitVec(n, a):
    return _mk(FuncDeclRef(Z3_OP_REPEAT, "repeat", (n,)), BitVecSort(a.size() * n), [a])


def RotateLeft(a, n):
    return _mk(FuncDeclRef(Z3_OP_ROTATE_LEFT, "rotate_left", (n,)), a.sort(), [a])


def RotateRight(a, n):
    return _mk(FuncDeclRef(Z3_OP_ROTATE_RIGHT, "rotate_right", (n,)), a.sort(), [a])


def _bin(kind, name):
    def f(a, b):
        w = a.size() if isinstance(a, ExprRef) else b.size()
        return _mk(FuncDeclRef(kind, name), BitVecSort(w), [_bv(a, w), _bv(b, w)])
    return f


UDiv, URem, SRem, LShR = (_bin(Z3_OP_BUDIV, "bvudiv"), _bin(Z3_OP_BUREM, "bvurem"), _bin(Z3_OP_BSREM, "bvsrem"),
                          _bin(Z3_OP_BLSHR, "bvlshr"))


def _cmp(kind):
    def f(a, b):
        w = a.size() if isinstance(a, ExprRef) else b.size()
        return _mk(FuncDeclRef(kind, "cmp"), BoolSort(), [_bv(a, w), _bv(b, w)])
    return f


ULT, ULE, UGT, UGE = _cmp(Z3_OP_ULT), _cmp(Z3_OP_ULEQ), _cmp(Z3_OP_UGT), _cmp(Z3_OP_UGEQ)


def BVMulNoOverflow(a, b, signed):
    assert not signed
    return _mk(FuncDeclRef(Z3_OP_BUMUL_NO_OVFL, "bvumul_noovfl"), BoolSort(), [a, b])


def BVComp(a, b):
    return _mk(FuncDeclRef(Z3_OP_BCOMP, "bvcomp"), BitVecSort(1), [a, b])


def BVRedOr(a):
    return _mk(FuncDeclRef(Z3_OP_BREDOR, "bvredor"), BitVecSort(1), [a])


def BVRedAnd(a):
    return _mk(FuncDeclRef(Z3_OP_BREDAND, "bvredand"), BitVecSort(1), [a])


def is_true(e):
    return isinstance(e, ExprRef) and e.decl().kind() == Z3_OP_TRUE


def is_false(e):
    return isinstance(e, ExprRef) and e.decl().kind() == Z3_OP_FALSE


def is_bv_value(e):
    return isinstance(e, ExprRef) and e.decl().kind() == Z3_OP_BNUM


# ------------------------------------------------------------- evaluation
def _s(x, w):
    return x - (1 << w) if x >> (w - 1) & 1 else x


def evaluate(e: ExprRef, env: Dict[str, int], funcs: Dict[str, Dict[int, int]], default: int = 0):
    """Concrete value (int, or bool for Bool sort) of e: constants by name from env,
    uninterpreted functions and base arrays by name from funcs[name][arg] (default if
    absent).  SMT-LIB semantics."""
    memo: Dict[int, object] = {}

    def ev(x):
        if x.get_id() in memo:
            return memo[x.get_id()]
        k, a = x.decl().kind(), x.children()
        w = x.size() if x.sort().kind() == Z3_BV_SORT else 0
        m = (1 << w) - 1 if w else 0
        if k == Z3_OP_UNINTERPRETED:
            if not a:
                r = env.get(x.decl().name(), default) if x.sort().kind() != Z3_ARRAY_SORT else ("arr", x.decl().name())
                if x.sort().kind() == Z3_BOOL_SORT:
                    r = bool(r)
            else:
                r = funcs.get(x.decl().name(), {}).get(ev(a[0]), default) & m
        elif k == Z3_OP_BNUM:
            r = x.as_long()
        elif k == Z3_OP_TRUE:
            r = True
        elif k == Z3_OP_FALSE:
            r = False
        elif k == Z3_OP_CONST_ARRAY:
            r = ("K", ev(a[0]))
        elif k == Z3_OP_STORE:
            r = ("store", ev(a[0]), ev(a[1]), ev(a[2]))
        elif k == Z3_OP_SELECT:
            arr, i = ev(a[0]), ev(a[1])
            while arr[0] == "store" and arr[2] != i:
                arr = arr[1]
            if arr[0] == "store":
                r = arr[3]
            elif arr[0] == "K":
                r = arr[1]
            else:
                r = funcs.get("array:" + arr[1], {}).get(i, default) & m
        else:
            v = [ev(c) for c in a]
            r = _op(x, k, v, w, m, a)
        memo[x.get_id()] = r
        return r

    return ev(e)


def _op(x, k, v, w, m, a):
    ow = a[0].size() if a and a[0].sort().kind() == Z3_BV_SORT else 0
    if k == Z3_OP_NOT: return not v[0]
    if k == Z3_OP_AND: return all(v)
    if k == Z3_OP_OR: return any(v)
    if k == Z3_OP_XOR: return v[0] != v[1]
    if k == Z3_OP_IMPLIES: return (not v[0]) or v[1]
    if k == Z3_OP_EQ: return v[0] == v[1]
    if k == Z3_OP_DISTINCT: return len(set(v)) == len(v)
    if k == Z3_OP_ITE: return v[1] if v[0] else v[2]
    if k == Z3_OP_BADD: return sum(v) & m
    if k == Z3_OP_BSUB: return (v[0] - v[1]) & m
    if k == Z3_OP_BMUL:
        r = 1
        for t in v:
            r = r * t & m
        return r
    if k == Z3_OP_BNEG: return -v[0] & m
    if k == Z3_OP_BNOT: return ~v[0] & m
    if k == Z3_OP_BAND: return v[0] & v[1]
    if k == Z3_OP_BOR: return v[0] | v[1]
    if k == Z3_OP_BXOR: return v[0] ^ v[1]
    if k == Z3_OP_BUDIV: return m if v[1] == 0 else v[0] // v[1]
    if k == Z3_OP_BUREM: return v[0] if v[1] == 0 else v[0] % v[1]
    sa, sb = (_s(v[0], ow), _s(v[1], ow)) if len(v) > 1 and ow else (0, 0)
    if k == Z3_OP_BSDIV:
        if sb == 0:
            return 1 if sa < 0 else m
        q = abs(sa) // abs(sb)
        return (q if (sa < 0) == (sb < 0) else -q) & m
    if k == Z3_OP_BSREM:
        if sb == 0:
            return v[0]
        r = abs(sa) % abs(sb)
        return (-r if sa < 0 else r) & m
    if k == Z3_OP_BSMOD:
        if sb == 0:
            return v[0]
        r = abs(sa) % abs(sb)
        if r == 0:
            return 0
        if sa < 0 and sb > 0: return (sb - r) & m
        if sa > 0 and sb < 0: return (sb + r) & m
        if sa < 0 and sb < 0: return -r & m
        return r
    if k == Z3_OP_BSHL: return 0 if v[1] >= w else (v[0] << v[1]) & m
    if k == Z3_OP_BLSHR: return 0 if v[1] >= w else v[0] >> v[1]
    if k == Z3_OP_BASHR: return (_s(v[0], w) >> min(v[1], w)) & m
    if k == Z3_OP_ULT: return v[0] < v[1]
    if k == Z3_OP_ULEQ: return v[0] <= v[1]
    if k == Z3_OP_UGT: return v[0] > v[1]
    if k == Z3_OP_UGEQ: return v[0] >= v[1]
    if k == Z3_OP_SLT: return sa < sb
    if k == Z3_OP_SLEQ: return sa <= sb
    if k == Z3_OP_SGT: return sa > sb
    if k == Z3_OP_SGEQ: return sa >= sb
    if k == Z3_OP_BUMUL_NO_OVFL: return v[0] * v[1] < (1 << ow)
    p = x.decl().params()
    if k == Z3_OP_EXTRACT: return (v[0] >> p[1]) & ((1 << (p[0] - p[1] + 1)) - 1)
    if k == Z3_OP_CONCAT:
        r = 0
        for c, t in zip(a, v):
            r = (r << c.size()) | t
        return r
    if k == Z3_OP_ZERO_EXT: return v[0]
    if k == Z3_OP_SIGN_EXT: return _s(v[0], ow) & m
    if k == Z3_OP_REPEAT:
        r = 0
        for _ in range(p[0]):
            r = (r << ow) | v[0]
        return r
    if k == Z3_OP_ROTATE_LEFT:
        n = p[0] % w
        return ((v[0] << n) | (v[0] >> (w - n))) & m
    if k == Z3_OP_ROTATE_RIGHT:
        n = p[0] % w
        return ((v[0] >> n) | (v[0] << (w - n))) & m
    if k == Z3_OP_BCOMP: return int(v[0] == v[1])
    if k == Z3_OP_BREDOR: return int(v[0] != 0)
    if k == Z3_OP_BREDAND: return int(v[0] == (1 << ow) - 1)
    raise NotImplementedError(k)


def simplify(e):
    return e


class Solver:
    """Decides only when the free constants are pinned by top-level `x == value`
    conjuncts and every read of an array / function is pinned the same way."""

    def __init__(self):
        self.cs = []
        self.timeout = None

    def set(self, key=None, value=None, **kw):
        self.timeout = value if key == "timeout" else kw.get("timeout", self.timeout)

    def set_timeout(self, t):
        self.timeout = t

    def add(self, *cs):
        for c in cs:
            self.cs.extend(c if isinstance(c, (list, tuple)) else [c])

    def check(self):
        env, funcs, rest = {}, {}, []
        for c in self.cs:
            if c.decl().kind() == Z3_OP_EQ and is_bv_value(c.children()[1]):
                lhs, val = c.children()[0], c.children()[1].as_long()
                if lhs.decl().kind() == Z3_OP_UNINTERPRETED and not lhs.children():
                    env[lhs.decl().name()] = val
                    continue
                if lhs.decl().kind() in (Z3_OP_UNINTERPRETED, Z3_OP_SELECT):
                    rest.append(("pin", lhs, val))
                    continue
            if c.decl().kind() == Z3_OP_EQ and c.children()[0].sort().kind() == Z3_BOOL_SORT:
                lhs, rhs = c.children()
                if lhs.decl().kind() == Z3_OP_UNINTERPRETED and not lhs.children() and rhs.decl().kind() in (
                        Z3_OP_TRUE, Z3_OP_FALSE):
                    env[lhs.decl().name()] = int(is_true(rhs))
                    continue
            rest.append(("c", c, None))
        for kind, e, val in rest:  # function / array pins: argument values under env
            if kind != "pin":
                continue
            if e.decl().kind() == Z3_OP_SELECT:
                name = "array:" + e.children()[0].decl().name()
            else:
                name = e.decl().name()
            arg = evaluate(e.children()[-1], env, funcs)
            if funcs.setdefault(name, {}).get(arg, val) != val:
                self._model = None
                return unsat
            funcs[name][arg] = val
        self._env, self._funcs = env, funcs
        try:
            ok = all(evaluate(e, env, funcs) for kind, e, _ in rest if kind == "c")
        except NotImplementedError:  # an operator the stand-in does not model
            return unknown
        return sat if ok else unsat

    def model(self):
        return ModelRef(dict(self._env), dict(self._funcs))


class ModelRef:
    """z3py's ModelRef.eval over the stand-in's decided environment."""

    def __init__(self, env, funcs):
        self.env, self.funcs = env, funcs

    def eval(self, e, model_completion=False):
        if e.sort().kind() == Z3_BOOL_SORT:
            return BoolVal(bool(evaluate(e, self.env, self.funcs)))
        return BitVecVal(evaluate(e, self.env, self.funcs), e.size())


class Optimize(Solver):
    def minimize(self, e):
        pass

    def maximize(self, e):
        pass
