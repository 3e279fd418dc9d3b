"""laser.smt vocabulary over hash-consed terms (no z3) — the host-side mirror.

Mirrors the public surface of the reference's SMT layer
(mythril/laser/smt/__init__.py:1-154, bitvec.py, bitvec_helper.py, bool.py,
function.py, array.py) with the same operator meanings:

  BitVec + - *            bvadd/bvsub/bvmul          bitvec.py:63-94
  BitVec /                bvsdiv (signed!)           bitvec.py:96-103
  < > <= >= on BitVec     SIGNED compares            bitvec.py:138-180
  == / != on BitVec       zero-extend the narrower   bitvec.py:16-22, 183-216
  <<  >>                  bvshl / bvashr             bitvec.py:232-246
  UDiv URem SRem LShR ULT UGT ULE UGE If Concat Extract Sum BV*No*flow
                                                     bitvec_helper.py:10-214
  And Or Not Xor                                     bool.py:87-123
  Function (UF), Array / K (select/store)            function.py, array.py

Terms are DAG nodes (shared structurally), which is exactly what the GPU
lowering consumes (mythril_amd/dag.py).  Concrete sub-terms are folded on
construction — the role z3's simplify() plays in the reference — so
``.value`` / ``.symbolic`` behave like laser.smt's.  Satisfiability is never
decided here: that is the GPU kernel's job (or z3's).
"""
from __future__ import annotations

import hashlib
import weakref
from array import array
from typing import Any, Dict, List, Optional, Sequence, Set, Tuple, Union

from . import ir

Annotations = Set[Any]


class _Arena:
    """Flat table of the live terms: the native DAG builder (mgp_build_states,
    csrc/mgp_front.cpp) walks it instead of the Python objects.

    Per term t: op[t], width[t] (Bool = 0), args[3t..3t+2] (term ids, -1 = none) and
    p[2t], p[2t+1]: VAR (name id, 0), CONST (offset into `limbs`, number of u32 limbs,
    little-endian), EXTRACT (hi, lo), UFAPP / UFINV (function id, function-name id).
    Names are interned in `names`.  The row of a dead term (and a dead constant's limbs)
    goes to a free list and is reused by the next term (`release`), so the table's size
    follows the live terms, not every term ever built.  A live term keeps its arguments
    alive, so no live row ever points at a reused one.
    """

    def __init__(self):
        self.op = array("B")
        self.width = array("I")
        self.args = array("i")
        self.p = array("I")
        self.limbs = array("I")
        self.names: List[str] = []
        self.name_id: Dict[str, int] = {}
        # a stable 64-bit hash of each name's text (blake2b; Python's str hash is salted
        # per process): the native front end keys a state's candidates by its content with
        # names folded in by these, not by the interning order of the ids
        self.name_hash = array("Q")
        self.free: List[int] = []                 # rows of dead terms
        self.free_limbs: Dict[int, List[int]] = {}  # limb count -> offsets of dead constants' limbs

    def intern_name(self, name: str) -> int:
        k = self.name_id.get(name)
        if k is None:
            k = self.name_id[name] = len(self.names)
            self.names.append(name)
            self.name_hash.append(int.from_bytes(hashlib.blake2b(name.encode(), digest_size=8).digest(), "little"))
        return k

    def add(self, op: int, width: int, args: Tuple["Term", ...], params: Tuple) -> int:
        ids = [a.tid for a in args] + [-1, -1, -1]
        p0 = p1 = 0
        if op == ir.VAR:
            p0 = self.intern_name(str(params[0]))
        elif op == ir.CONST:
            n = max(1, (width + 31) // 32)
            limbs = array("I", int(params[0]).to_bytes(4 * n, "little"))
            spare = self.free_limbs.get(n)
            if spare:
                p0 = spare.pop()
                self.limbs[p0:p0 + n] = limbs
            else:
                p0 = len(self.limbs)
                self.limbs.extend(limbs)
            p1 = n
        elif op == ir.EXTRACT:
            p0, p1 = params
        elif op in (ir.UFAPP, ir.UFINV):
            p0, p1 = params[0], self.intern_name(str(params[1]))
        if self.free:
            tid = self.free.pop()
            self.op[tid] = op
            self.width[tid] = width
            self.args[3 * tid:3 * tid + 3] = array("i", ids[:3])
            self.p[2 * tid] = p0
            self.p[2 * tid + 1] = p1
            return tid
        tid = len(self.op)
        self.op.append(op)
        self.width.append(width)
        self.args.extend(ids[:3])
        self.p.append(p0)
        self.p.append(p1)
        return tid

    def release(self, tid: int) -> None:
        """The term of row `tid` is gone: its row (and a constant's limbs) can be reused."""
        if self.op[tid] == ir.CONST:
            self.free_limbs.setdefault(self.p[2 * tid + 1], []).append(self.p[2 * tid])
        self.free.append(tid)

    def live(self) -> int:
        return len(self.op) - len(self.free)


ARENA = _Arena()
_ROW_REFS: Dict[int, "weakref.ref"] = {}   # arena row -> the weakref that frees it


def _free_row(tid: int, ref) -> None:
    try:
        if _ROW_REFS.get(tid) is ref:
            del _ROW_REFS[tid]
            ARENA.release(tid)
    except Exception:  # interpreter shutdown: the module's globals may be gone
        pass


class Term:
    """Hash-consed term node.  op/width/args/params as in include/mgp_ir.h; `tid` is
    its row in the term arena (ARENA) the native DAG builder reads."""

    __slots__ = ("op", "width", "args", "params", "_h", "tid", "__weakref__")

    def __init__(self, op: int, width: int, args: Tuple["Term", ...], params: Tuple):
        self.op = op
        self.width = width
        self.args = args
        self.params = params
        self._h = hash((op, width, tuple(id(a) for a in args), params))
        self.tid = tid = ARENA.add(op, width, args, params)
        # The row is freed by a weakref callback, not by __del__: CPython runs __del__
        # before it clears the term's weakrefs, so another thread could still fetch the
        # dying term from _INTERN (resurrecting it on a freed row); callbacks run after
        # every weakref to the term is cleared, when no lookup can return it any more.
        _ROW_REFS[tid] = weakref.ref(self, lambda r, tid=tid: _free_row(tid, r))

    def __hash__(self):
        return self._h

    def __eq__(self, other):  # structural identity (interned => identity)
        return self is other

    @property
    def is_bool(self) -> bool:
        return self.width == 0

    def __repr__(self):
        return f"Term({ir.OP_NAMES.get(self.op, self.op)}, w={self.width}, params={self.params})"


# Weak values: a term lives as long as something (a constraint list, a parent term, an UNSAT
# core) holds it, as z3 reference-counts its ASTs.  A live term keeps its arguments alive, so
# the id()s in its key stay valid for exactly as long as the entry exists.
_INTERN: "weakref.WeakValueDictionary[Tuple, Term]" = weakref.WeakValueDictionary()


def mk(op: int, width: int, args: Sequence[Term] = (), params: Tuple = ()) -> Term:
    key = (op, width, tuple(id(a) for a in args), params)
    t = _INTERN.get(key)
    if t is None or t.args != tuple(args):
        t = Term(op, width, tuple(args), params)
        _INTERN[key] = t
    return t


BOOL = 0  # width marker of Bool terms


def _mask(w: int) -> int:
    return (1 << w) - 1


def _signed(x: int, w: int) -> int:
    return x - (1 << w) if (x >> (w - 1)) & 1 else x


def const(v: int, w: int) -> Term:
    return mk(ir.CONST, w, (), (int(v) & _mask(w),))


def bconst(b: bool) -> Term:
    return mk(ir.TRUE if b else ir.FALSE, BOOL)


def is_const(t: Term) -> bool:
    return t.op in (ir.CONST, ir.TRUE, ir.FALSE)


def cval(t: Term):
    if t.op == ir.CONST:
        return t.params[0]
    if t.op == ir.TRUE:
        return True
    if t.op == ir.FALSE:
        return False
    return None


# ---------------------------------------------------------- constant folding
def _fold_bin(op: int, x: int, y: int, w: int) -> int:
    m = _mask(w)
    if op == ir.ADD:
        return (x + y) & m
    if op == ir.SUB:
        return (x - y) & m
    if op == ir.MUL:
        return (x * y) & m
    if op == ir.UDIV:
        return m if y == 0 else x // y
    if op == ir.UREM:
        return x if y == 0 else x % y
    if op in (ir.SDIV, ir.SREM, ir.SMOD):
        sx, sy = _signed(x, w), _signed(y, w)
        if op == ir.SDIV:
            if sy == 0:
                return 1 if sx < 0 else m
            q = abs(sx) // abs(sy)
            return (-q if (sx < 0) != (sy < 0) else q) & m
        if op == ir.SREM:
            if sy == 0:
                return x
            r = abs(sx) % abs(sy)
            return (-r if sx < 0 else r) & m
        if sy == 0:
            return x
        r = sx % sy if sy > 0 else -((-sx) % (-sy))  # floor mod: sign follows divisor
        return r & m
    if op == ir.AND:
        return x & y
    if op == ir.OR:
        return x | y
    if op == ir.XOR:
        return x ^ y
    if op == ir.SHL:
        return 0 if y >= w else (x << y) & m
    if op == ir.LSHR:
        return 0 if y >= w else x >> y
    if op == ir.ASHR:
        if y >= w:
            return m if _signed(x, w) < 0 else 0
        return (_signed(x, w) >> y) & m
    raise ValueError(op)


def _fold_cmp(op: int, x: int, y: int, w: int) -> bool:
    sx, sy = _signed(x, w), _signed(y, w)
    return {
        ir.EQ: x == y, ir.ULT: x < y, ir.ULE: x <= y, ir.UGT: x > y, ir.UGE: x >= y,
        ir.SLT: sx < sy, ir.SLE: sx <= sy, ir.SGT: sx > sy, ir.SGE: sx >= sy,
        ir.UADD_NOOVF: x + y < (1 << w), ir.UMUL_NOOVF: x * y < (1 << w), ir.USUB_NOUDF: y <= x,
    }[op]


def bv_op(op: int, a: Term, b: Term) -> Term:
    w = a.width
    if a.width != b.width:
        raise ValueError(f"width mismatch {a.width} vs {b.width}")
    if a.op == ir.CONST and b.op == ir.CONST:
        return const(_fold_bin(op, a.params[0], b.params[0], w), w)
    if op == ir.UDIV and b.op == ir.CONST and b.params[0] and b.params[0] & (b.params[0] - 1) == 0:
        # x / 2^k is a logical shift: z3's simplify() rewrites bvudiv by a power of two so
        # (solc <= 0.5.4 dispatchers: CALLDATALOAD(0) / 2^224, instructions.py:463-477)
        return mk(ir.LSHR, w, (a, const(b.params[0].bit_length() - 1, w)))
    return mk(op, w, (a, b))


def cmp_op(op: int, a: Term, b: Term) -> Term:
    if a.width != b.width:
        raise ValueError(f"width mismatch {a.width} vs {b.width}")
    if a.op == ir.CONST and b.op == ir.CONST:
        return bconst(_fold_cmp(op, a.params[0], b.params[0], a.width))
    if op == ir.EQ and a is b:
        return bconst(True)
    return mk(op, BOOL, (a, b))


def b_and(args: Sequence[Term]) -> Term:
    out: List[Term] = []
    for t in args:
        if t.op == ir.FALSE:
            return bconst(False)
        if t.op != ir.TRUE:
            out.append(t)
    if not out:
        return bconst(True)
    r = out[0]
    for t in out[1:]:
        r = mk(ir.BAND, BOOL, (r, t))
    return r


def b_or(args: Sequence[Term]) -> Term:
    out: List[Term] = []
    for t in args:
        if t.op == ir.TRUE:
            return bconst(True)
        if t.op != ir.FALSE:
            out.append(t)
    if not out:
        return bconst(False)
    r = out[0]
    for t in out[1:]:
        r = mk(ir.BOR, BOOL, (r, t))
    return r


def b_not(a: Term) -> Term:
    if is_const(a):
        return bconst(not cval(a))
    if a.op == ir.BNOT:
        return a.args[0]
    return mk(ir.BNOT, BOOL, (a,))


def ite(c: Term, a: Term, b: Term) -> Term:
    if is_const(c):
        return a if cval(c) else b
    if a is b:
        return a
    if a.is_bool != b.is_bool or (not a.is_bool and a.width != b.width):
        raise ValueError("ite branch sort mismatch")
    return mk(ir.BITE if a.is_bool else ir.ITE, a.width, (c, a, b))


def extract(hi: int, lo: int, a: Term) -> Term:
    w = hi - lo + 1
    if not (0 <= lo <= hi < a.width):
        raise ValueError("bad extract bounds")
    if lo == 0 and w == a.width:
        return a
    if a.op == ir.CONST:
        return const(a.params[0] >> lo, w)
    return mk(ir.EXTRACT, w, (a,), (hi, lo))


def concat(parts: Sequence[Term]) -> Term:
    r = parts[0]
    for p in parts[1:]:
        if r.op == ir.CONST and p.op == ir.CONST:
            r = const((r.params[0] << p.width) | p.params[0], r.width + p.width)
        else:
            r = mk(ir.CONCAT, r.width + p.width, (r, p))
    return r


def zext(a: Term, w: int) -> Term:
    if w == a.width:
        return a
    if a.op == ir.CONST:
        return const(a.params[0], w)
    return mk(ir.ZEXT, w, (a,))


# ------------------------------------------------------------- wrappers
class Expression:
    """laser.smt.Expression: a raw term plus an annotation set (expression.py)."""

    def __init__(self, raw: Term, annotations: Optional[Annotations] = None):
        self.raw = raw
        self._annotations = set(annotations) if annotations else set()

    @property
    def annotations(self) -> Annotations:
        return self._annotations

    def annotate(self, annotation: Any) -> None:
        self._annotations.add(annotation)

    def simplify(self) -> None:
        """Terms are folded on construction; nothing to do."""

    def size(self) -> int:
        return self.raw.width

    def __repr__(self):
        return repr(self.raw)


def _union(*xs) -> Annotations:
    s: Annotations = set()
    for x in xs:
        if isinstance(x, Expression):
            s |= x.annotations
    return s


class Bool(Expression):
    """laser.smt.Bool (bool.py:14-81)."""

    @property
    def is_false(self) -> bool:
        return self.raw.op == ir.FALSE

    @property
    def is_true(self) -> bool:
        return self.raw.op == ir.TRUE

    @property
    def value(self) -> Optional[bool]:
        return True if self.is_true else False if self.is_false else None

    @property
    def symbolic(self) -> bool:
        return self.value is None

    def __eq__(self, other) -> "Bool":  # type: ignore[override]
        o = other.raw if isinstance(other, Expression) else bconst(bool(other))
        if is_const(self.raw) and is_const(o):
            return Bool(bconst(cval(self.raw) == cval(o)), _union(self, other))
        return Bool(mk(ir.BEQ, BOOL, (self.raw, o)), _union(self, other))

    def __ne__(self, other) -> "Bool":  # type: ignore[override]
        return Not(self == other)

    def __bool__(self) -> bool:
        v = self.value
        return v if v is not None else False

    def __hash__(self) -> int:
        return hash(self.raw)


def _coerce(x: Union["BitVec", int], w: int) -> "BitVec":
    return x if isinstance(x, BitVec) else BitVec(const(int(x), w))


def _padded(a: Term, b: Term) -> Tuple[Term, Term]:
    """bitvec.py:16-22: zero-extend the narrower operand.  A narrower constant stays a
    ZEXT node (not folded): z3 sees Concat(BitVecVal(0, k), c) there, and the builder
    treats such a cross-width key equality specially (dag.py, padded equalities)."""
    if a.width < b.width:
        a = mk(ir.ZEXT, b.width, (a,)) if a.op == ir.CONST and b.op != ir.CONST else zext(a, b.width)
    elif b.width < a.width:
        b = mk(ir.ZEXT, a.width, (b,)) if b.op == ir.CONST and a.op != ir.CONST else zext(b, a.width)
    return a, b


class BitVec(Expression):
    """laser.smt.BitVec (bitvec.py:25-253)."""

    @property
    def symbolic(self) -> bool:
        return self.raw.op != ir.CONST

    @property
    def value(self) -> Optional[int]:
        return None if self.symbolic else self.raw.params[0]

    def _bin(self, other, op) -> "BitVec":
        o = _coerce(other, self.size())
        return BitVec(bv_op(op, self.raw, o.raw), _union(self, o))

    def __add__(self, other):
        return self._bin(other, ir.ADD)

    def __radd__(self, other):
        return _coerce(other, self.size())._bin(self, ir.ADD)

    def __sub__(self, other):
        return self._bin(other, ir.SUB)

    def __rsub__(self, other):
        return _coerce(other, self.size())._bin(self, ir.SUB)

    def __mul__(self, other):
        return self._bin(other, ir.MUL)

    def __rmul__(self, other):
        return _coerce(other, self.size())._bin(self, ir.MUL)

    def __truediv__(self, other):
        return self._bin(other, ir.SDIV)

    def __and__(self, other):
        return self._bin(other, ir.AND)

    def __or__(self, other):
        return self._bin(other, ir.OR)

    def __xor__(self, other):
        return self._bin(other, ir.XOR)

    def __lshift__(self, other):
        return self._bin(other, ir.SHL)

    def __rshift__(self, other):
        return self._bin(other, ir.ASHR)

    def _cmp(self, other, op) -> Bool:
        o = _coerce(other, self.size())
        return Bool(cmp_op(op, self.raw, o.raw), _union(self, o))

    def __lt__(self, other):
        return self._cmp(other, ir.SLT)

    def __gt__(self, other):
        return self._cmp(other, ir.SGT)

    def __le__(self, other):
        return self._cmp(other, ir.SLE)

    def __ge__(self, other):
        return self._cmp(other, ir.SGE)

    def __eq__(self, other) -> Bool:  # type: ignore[override]
        o = _coerce(other, self.size())
        a, b = _padded(self.raw, o.raw)
        return Bool(cmp_op(ir.EQ, a, b), _union(self, o))

    def __ne__(self, other) -> Bool:  # type: ignore[override]
        return Not(self.__eq__(other))

    def __hash__(self) -> int:
        return hash(self.raw)


# ------------------------------------------------------- helper functions
def If(a: Union[Bool, bool], b: Union[BitVec, int], c: Union[BitVec, int]) -> BitVec:
    """bitvec_helper.py:25-40 (ints become 256-bit values)."""
    if not isinstance(a, Bool):
        a = Bool(bconst(bool(a)))
    if not isinstance(b, Expression):
        b = BitVec(const(b, 256))
    if not isinstance(c, Expression):
        c = BitVec(const(c, 256))
    r = ite(a.raw, b.raw, c.raw)
    cls = Bool if r.is_bool else BitVec
    return cls(r, _union(a, b, c))


def _cmp_helper(a: BitVec, b: BitVec, op: int) -> Bool:
    return Bool(cmp_op(op, a.raw, b.raw), _union(a, b))


def UGT(a: BitVec, b: BitVec) -> Bool:
    return _cmp_helper(a, b, ir.UGT)


def UGE(a: BitVec, b: BitVec) -> Bool:
    return Or(UGT(a, b), a == b)  # bitvec_helper.py:53-60


def ULT(a: BitVec, b: BitVec) -> Bool:
    return _cmp_helper(a, b, ir.ULT)


def ULE(a: BitVec, b: BitVec) -> Bool:
    return Or(ULT(a, b), a == b)  # bitvec_helper.py:73-80


def Concat(*args) -> BitVec:
    bvs = args[0] if len(args) == 1 and isinstance(args[0], list) else list(args)
    return BitVec(concat([b.raw for b in bvs]), _union(*bvs))


def Extract(high: int, low: int, bv: BitVec) -> BitVec:
    return BitVec(extract(high, low, bv.raw), bv.annotations)


def URem(a: BitVec, b: BitVec) -> BitVec:
    return BitVec(bv_op(ir.UREM, a.raw, b.raw), _union(a, b))


def SRem(a: BitVec, b: BitVec) -> BitVec:
    return BitVec(bv_op(ir.SREM, a.raw, b.raw), _union(a, b))


def UDiv(a: BitVec, b: BitVec) -> BitVec:
    return BitVec(bv_op(ir.UDIV, a.raw, b.raw), _union(a, b))


def LShR(a: BitVec, b: BitVec) -> BitVec:
    return BitVec(bv_op(ir.LSHR, a.raw, b.raw), _union(a, b))


def Sum(*args: BitVec) -> BitVec:
    r = args[0]
    for a in args[1:]:
        r = r + a
    return r


def BVAddNoOverflow(a, b, signed: bool) -> Bool:
    a, b = _coerce(a, 256), _coerce(b, 256)
    if signed:
        raise NotImplementedError("signed BVAddNoOverflow is not on the pre-filter path")
    return _cmp_helper(a, b, ir.UADD_NOOVF)


def BVMulNoOverflow(a, b, signed: bool) -> Bool:
    a, b = _coerce(a, 256), _coerce(b, 256)
    if signed:
        raise NotImplementedError("signed BVMulNoOverflow is not on the pre-filter path")
    return _cmp_helper(a, b, ir.UMUL_NOOVF)


def BVSubNoUnderflow(a, b, signed: bool) -> Bool:
    a, b = _coerce(a, 256), _coerce(b, 256)
    if signed:
        raise NotImplementedError("signed BVSubNoUnderflow is not on the pre-filter path")
    return _cmp_helper(a, b, ir.USUB_NOUDF)


def And(*args: Union[Bool, bool]) -> Bool:
    bs = [a if isinstance(a, Bool) else Bool(bconst(bool(a))) for a in args]
    return Bool(b_and([b.raw for b in bs]), _union(*bs))


def Or(*args: Union[Bool, bool]) -> Bool:
    bs = [a if isinstance(a, Bool) else Bool(bconst(bool(a))) for a in args]
    return Bool(b_or([b.raw for b in bs]), _union(*bs))


def Xor(a: Bool, b: Bool) -> Bool:
    if is_const(a.raw) and is_const(b.raw):
        return Bool(bconst(cval(a.raw) != cval(b.raw)))
    return Bool(mk(ir.BXOR, BOOL, (a.raw, b.raw)), _union(a, b))


def Not(a: Bool) -> Bool:
    return Bool(b_not(a.raw), a.annotations)


def is_true(a: Bool) -> bool:
    return a.raw.op == ir.TRUE


def is_false(a: Bool) -> bool:
    return a.raw.op == ir.FALSE


def simplify(e: Expression) -> Expression:
    return e


# --------------------------------------------------------------- UF / arrays
class Function:
    """Uninterpreted function (function.py:7-25).  `inverse_of` marks a keccak inverse.

    Functions are identified by name and signature, as z3 identifies its declarations: two
    Function("f", 256, 256) objects are one function (one id), and two Array("balance", ...)
    objects read one array -- LASER's world state copies `balances` into `starting_balances`
    and every account's storage is an Array named "Storage" (account.py:28), all of which z3
    sees as the same symbol (mythril_amd.z3_lower interns declarations the same way)."""

    _ids: Dict[Tuple[str, int, int], int] = {}

    def __init__(self, name: str, domain: int, value_range: int, inverse_of: Optional["Function"] = None):
        self.name = name
        self.domain = domain
        self.range = value_range
        self.inverse_of = inverse_of
        if inverse_of is not None:
            self.fid = inverse_of.fid
        else:
            self.fid = Function._ids.setdefault((name, domain, value_range), len(Function._ids))

    def __call__(self, item: BitVec) -> BitVec:
        if item.size() != self.domain:
            raise ValueError(f"{self.name}: argument width {item.size()} != domain {self.domain}")
        op = ir.UFINV if self.inverse_of is not None else ir.UFAPP
        return BitVec(mk(op, self.range, (item.raw,), (self.fid, self.name)), item.annotations)


class BaseArray:
    """Select/Store arrays (array.py:16-63) lowered by read-over-write."""

    def __getitem__(self, item: BitVec) -> BitVec:
        if isinstance(item, slice):
            raise ValueError("Instance of BaseArray, does not support getitem with slices")
        return BitVec(self._select(item.raw))

    def __setitem__(self, key: BitVec, value: Union[BitVec, Bool]) -> None:
        if isinstance(value, Bool):
            value = If(value, 1, 0)
        self._stores = self._stores + ((key.raw, value.raw),)

    def _select(self, idx: Term) -> Term:
        r = self._base(idx)
        for k, v in self._stores:  # oldest first: later stores shadow earlier ones
            r = ite(cmp_op(ir.EQ, idx, k), v, r)
        return r


class Array(BaseArray):
    def __init__(self, name: str, domain: int, value_range: int):
        self.name = name
        self.domain = domain
        self.range = value_range
        self._fn = Function(f"array:{name}", domain, value_range)
        self._stores: Tuple[Tuple[Term, Term], ...] = ()

    def _base(self, idx: Term) -> Term:
        return mk(ir.UFAPP, self.range, (idx,), (self._fn.fid, self._fn.name))


class K(BaseArray):
    def __init__(self, domain: int, value_range: int, value: int):
        self.domain = domain
        self.range = value_range
        self.value = const(value, value_range)
        self._stores = ()

    def _base(self, idx: Term) -> Term:
        return self.value


# ------------------------------------------------------------ symbol factory
class _SymbolFactory:
    """symbol_factory (smt/__init__.py:83-154)."""

    @staticmethod
    def Bool(value: bool, annotations: Optional[Annotations] = None) -> Bool:
        return Bool(bconst(bool(value)), annotations)

    @staticmethod
    def BoolSym(name: str, annotations: Optional[Annotations] = None) -> Bool:
        v = mk(ir.VAR, 1, (), (name,))
        return Bool(mk(ir.EQ, BOOL, (v, const(1, 1))), annotations)

    @staticmethod
    def BitVecVal(value: int, size: int, annotations: Optional[Annotations] = None) -> BitVec:
        return BitVec(const(value, size), annotations)

    @staticmethod
    def BitVecSym(name: str, size: int, annotations: Optional[Annotations] = None) -> BitVec:
        return BitVec(mk(ir.VAR, size, (), (name,)), annotations)


symbol_factory = _SymbolFactory()
