"""Independent re-proof of refutations — TEST INFRASTRUCTURE ONLY.

The product's host pre-check (mythril_amd/csrc/mgp_refute.cpp + mgp_domain.h) claims a
constraint list UNSAT; an unsound claim would drop a satisfiable path (the reference treats
only z3's `unsat` as infeasible, constraints.py:34-51, svm.py:251-255).  This module re-proves
such claims with reasoning of its own, written apart from mgp_domain.h:

  * it reads the hash-consed term DAG (mythril_amd.smt terms), not the native node lists;
  * values are Python ints of any width (no 256-bit limbs, no piece expansion);
  * every transfer function is stated here from the operator's definition in oracle.bvsem
    (SMT-LIB QF_BV semantics, reference bitvec.py / bitvec_helper.py / bool.py);
  * abstract values are unsigned intervals x known bits, Bool truth sets, and the possible
    orderings {<, =, >} of compared operand pairs, propagated over a work list;
  * a linear pass writes every BV node as c + sum(coef * atom) mod 2^w under the decided
    selects (a UF application is one atom per argument form, so congruent reads share it)
    and decides or narrows every compare whose operands differ by a constant;
  * what that leaves open is searched: failed-literal probing, then case splits on Bool atoms
    (operands of required disjunctions, ITE conditions, compares), then interval bisection
    of bounded variables, within a step budget (TIERS: a cheap search, then a deeper one).

A state is re-proved UNSAT when every branch of the search empties some abstract value.
The certificate it checks is the refuter's UNSAT core (mgp_refute_cores: the constraints the
refutation needs), so a re-proof covers the core and therefore the whole list.  What the
search does not close within its budget is reported as unreplayed, not as wrong (only a model
can show a refutation wrong: tests/test_gpu_suite.py's witness checks).  Only tests/ and
scripts/replay_refutations.py import it; tests/test_refute_check.py checks its own soundness
exhaustively on small-width states.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

from . import bvsem as S

# truth sets
BF, BT, BB = 1, 2, 3
# orderings of a pair (x, y)
OLT, OEQ, OGT, OALL = 1, 2, 4, 7

_CMP_U = {S.ULT, S.ULE, S.UGT, S.UGE}
_CMP_S = {S.SLT, S.SLE, S.SGT, S.SGE}
# orderings (x vs y) under which cmp(x, y) is true
_TRUE_ORD = {S.EQ: OEQ, S.ULT: OLT, S.ULE: OLT | OEQ, S.UGT: OGT, S.UGE: OGT | OEQ,
             S.SLT: OLT, S.SLE: OLT | OEQ, S.SGT: OGT, S.SGE: OGT | OEQ, S.USUB_NOUDF: OGT | OEQ}


class Empty(Exception):
    """Some abstract value became empty: the current branch has no model."""


def _mask(w: int) -> int:
    return (1 << w) - 1


def _top(w: int) -> Tuple[int, int, int, int]:
    return (0, _mask(w), 0, 0)


def _exact(v: int, w: int) -> Tuple[int, int, int, int]:
    v &= _mask(w)
    return (v, v, _mask(w) & ~v, v)


def _norm(a, w: int):
    """(lo, hi, z, o): unsigned interval, known-zero and known-one masks.  Re-establishes
    lo >= o, hi <= ~z and the common high prefix of lo / hi as known bits; Empty if none."""
    lo, hi, z, o = a
    m = _mask(w)
    z &= m
    o &= m
    for _ in range(4):
        if z & o:
            raise Empty
        if lo < o:
            lo = o
        if hi > (m & ~z):
            hi = m & ~z
        if lo > hi:
            raise Empty
        k = (lo ^ hi).bit_length()
        pm = m & ~_mask(k)
        nz, no = z | (~lo & pm), o | (lo & pm)
        if (nz, no) == (z, o):
            break
        z, o = nz, no
    if z & o:
        raise Empty
    return (lo, hi, z, o)


def _meet(a, b, w: int):
    return _norm((max(a[0], b[0]), min(a[1], b[1]), a[2] | b[2], a[3] | b[3]), w)


def _hull(a, b):
    return (min(a[0], b[0]), max(a[1], b[1]), a[2] & b[2], a[3] & b[3])


def _is_exact(a) -> bool:
    return a[0] == a[1]


def _known_low(a, b, w: int) -> int:
    """Number of low bits known in both a and b."""
    kn = (a[2] | a[3]) & (b[2] | b[3])
    t = 0
    while t < w and (kn >> t) & 1:
        t += 1
    return t


def _tz(a, w: int) -> int:
    """Trailing bits known zero."""
    t = 0
    while t < w and (a[2] >> t) & 1:
        t += 1
    return t


class Checker:
    """Propagation state of one term DAG (a constraint list) under case splits."""

    CREEP = 24   # changes of one BV node's value per propagation before it is frozen

    def __init__(self, roots: Sequence, budget: int = 200000):
        order: List = []
        index: Dict[int, int] = {}
        stack = [(t, False) for t in reversed(list(roots))]
        while stack:  # post order: operands first
            t, done = stack.pop()
            if id(t) in index:
                continue
            if done:
                index[id(t)] = len(order)
                order.append(t)
                continue
            stack.append((t, True))
            for a in reversed(t.args):
                if id(a) not in index:
                    stack.append((a, False))
        self.t = order
        self.n = len(order)
        self.idx = index
        self.args = [[index[id(a)] for a in t.args] for t in order]
        self.isb = [t.width == 0 for t in order]
        self.w = [t.width for t in order]
        self.users: List[List[int]] = [[] for _ in order]
        for i, aa in enumerate(self.args):
            for a in set(aa):
                self.users[a].append(i)
        self.roots = [index[id(r)] for r in roots]
        # compared operand pairs: (x, y) with x < y -> pair id; per compare node its pair and
        # whether its operands are swapped
        self.pair_of: Dict[Tuple[int, int, bool], int] = {}
        self.cmp_pair: Dict[int, Tuple[int, bool, bool]] = {}
        self.pair_cmps: List[List[int]] = []
        self.pair_xy: List[Tuple[int, int, bool]] = []
        for i, t in enumerate(order):
            if t.op in _TRUE_ORD and len(self.args[i]) == 2 and not self.isb[self.args[i][0]]:
                a, b = self.args[i]
                signed = t.op in _CMP_S
                x, y, sw = (a, b, False) if a <= b else (b, a, True)
                key = (x, y, signed)
                if key not in self.pair_of:
                    self.pair_of[key] = len(self.pair_xy)
                    self.pair_xy.append(key)
                    self.pair_cmps.append([])
                p = self.pair_of[key]
                self.cmp_pair[i] = (p, sw, signed)
                self.pair_cmps[p].append(i)
        # EQ nodes share the "=" ordering with both the unsigned and the signed pair
        self.eq_twin: Dict[int, int] = {}
        for (x, y, signed), p in self.pair_of.items():
            q = self.pair_of.get((x, y, not signed))
            if q is not None:
                self.eq_twin[p] = q
        # UF applications by function: congruence (equal arguments -> equal values)
        self.ufs: Dict[Tuple[int, object], List[int]] = {}
        for i, t in enumerate(order):
            if t.op in (S.UFAPP, S.UFINV):
                self.ufs.setdefault((t.op, t.params[0]), []).append(i)
        self.uf_peers: Dict[int, List[int]] = {}
        for apps in self.ufs.values():
            if 1 < len(apps) <= 64:
                for i in apps:
                    self.uf_peers[i] = [j for j in apps if j != i]
        # BVAddNoOverflow nodes by their (unordered) operand pair
        self.noovf: Dict[Tuple[int, int], int] = {}
        for i, t in enumerate(order):
            if t.op == S.UADD_NOOVF and len(self.args[i]) == 2:
                a, b = self.args[i]
                self.noovf[(min(a, b), max(a, b))] = i
        # injective applications: f(x) with the keccak manager's inverse axiom
        # f^-1(f(x)) == x among the constraints (keccak_function_manager.py:102-146); while
        # the axiom node holds, f(x) == f(y) implies x == y
        self.inj: Dict[object, List[Tuple[int, int]]] = {}
        for e, t in enumerate(order):
            if t.op != S.EQ or len(self.args[e]) != 2:
                continue
            for u, x in (self.args[e], self.args[e][::-1]):
                tu = order[u]
                if tu.op == S.UFINV and order[self.args[u][0]].op == S.UFAPP:
                    a = self.args[u][0]
                    if self.args[a][0] == x and order[a].params[0] == tu.params[0]:
                        self.inj.setdefault(tu.params[0], []).append((a, e))
        self.budget = budget
        self.steps = 0
        self.creep: Dict[int, int] = {}
        self.atom_node: Dict = {}
        self.av: List = [None] * self.n
        self.pairs: List[int] = [OALL] * len(self.pair_xy)
        for i, t in enumerate(order):
            self.av[i] = BB if self.isb[i] else _top(t.width)

    # ------------------------------------------------------------ state
    def snapshot(self):
        return (list(self.av), list(self.pairs))

    def restore(self, s) -> None:
        self.av, self.pairs = list(s[0]), list(s[1])

    def _set(self, i: int, v, work: List[int]) -> None:
        if self.isb[i]:
            nv = self.av[i] & v
            if not nv:
                raise Empty
        else:
            nv = _meet(self.av[i], v, self.w[i])
            if nv != self.av[i]:
                # a cycle of compares can narrow an interval by one per lap (x > y with x and y
                # congruent); past CREEP changes in one propagation the node keeps its value
                # (a sound over-approximation) and the linear pass decides the cycle
                c = self.creep.get(i, 0) + 1
                self.creep[i] = c
                if c > self.CREEP:
                    return
        if nv != self.av[i]:
            self.av[i] = nv
            work.append(i)

    def _set_pair(self, p: int, s: int, work: List[int]) -> None:
        ns = self.pairs[p] & s
        if not ns:
            raise Empty
        if ns != self.pairs[p]:
            self.pairs[p] = ns
            work.extend(self.pair_cmps[p])
            x, y, _ = self.pair_xy[p]
            work.append(x)
            work.append(y)
            q = self.eq_twin.get(p)
            if q is not None:  # "=" is one fact for the unsigned and the signed pair
                if not ns & OEQ and self.pairs[q] & OEQ:
                    self._set_pair(q, OALL & ~OEQ, work)
                if ns == OEQ and self.pairs[q] != OEQ:
                    self._set_pair(q, OEQ, work)

    # ------------------------------------------------------------ forward
    def forward(self, i: int):
        """The value node i can take given its operands' abstract values."""
        t = self.t[i]
        op, w, ar = t.op, t.width, self.args[i]
        av = self.av
        if op == S.CONST:
            return _exact(t.params[0], w)
        if op == S.TRUE:
            return BT
        if op == S.FALSE:
            return BF
        if op in (S.VAR, S.UFAPP, S.UFINV):
            return _top(w)
        if self.isb[i]:
            return self._forward_bool(i, op, ar)
        m = _mask(w)
        if op == S.ITE:
            c = av[ar[0]]
            if c == BT:
                return av[ar[1]]
            if c == BF:
                return av[ar[2]]
            return _hull(av[ar[1]], av[ar[2]])
        a = av[ar[0]]
        if op == S.EXTRACT:
            hi_b, lo_b = t.params
            n = hi_b - lo_b + 1
            mn = _mask(n)
            z, o = (a[2] >> lo_b) & mn, (a[3] >> lo_b) & mn
            if (a[0] >> (hi_b + 1)) == (a[1] >> (hi_b + 1)):
                return (((a[0] >> lo_b) & mn), ((a[1] >> lo_b) & mn), z, o)
            return (0, mn, z, o)
        if op == S.ZEXT:
            wa = self.w[ar[0]]
            return (a[0], a[1], a[2] | (m & ~_mask(wa)), a[3])
        if op == S.SEXT:
            wa = self.w[ar[0]]
            if (a[2] >> (wa - 1)) & 1:  # sign known 0
                return (a[0], a[1], a[2] | (m & ~_mask(wa)), a[3])
            if (a[3] >> (wa - 1)) & 1:  # sign known 1
                ext = m & ~_mask(wa)
                return (a[0] | ext, a[1] | ext, a[2], a[3] | ext)
            return (0, m, a[2] & _mask(wa - 1), a[3] & _mask(wa - 1))
        if op == S.NOT:
            return (m - a[1], m - a[0], a[3], a[2])
        if op == S.NEG:
            if _is_exact(a):
                return _exact(-a[0], w)
            return _top(w)
        b = av[ar[1]] if len(ar) > 1 else None
        if op == S.CONCAT:
            wb = self.w[ar[1]]
            return ((a[0] << wb) | b[0], (a[1] << wb) | b[1], (a[2] << wb) | b[2], (a[3] << wb) | b[3])
        if _is_exact(a) and _is_exact(b) and S.ADD <= op <= S.ASHR:
            return _exact(S.binop(op, a[0], b[0], w), w)
        if op == S.ADD:
            k = _known_low(a, b, w)
            low = (a[3] + b[3]) & _mask(k)
            z, o = _mask(k) & ~low, low
            if a[1] + b[1] <= m:
                return (a[0] + b[0], a[1] + b[1], z, o)
            if a[0] + b[0] > m:
                return (a[0] + b[0] - m - 1, a[1] + b[1] - m - 1, z, o)
            return (0, m, z, o)
        if op == S.SUB:
            k = _known_low(a, b, w)
            low = (a[3] - b[3]) & _mask(k)
            z, o = _mask(k) & ~low, low
            if a[0] >= b[1] or not self._pair_ord(ar[0], ar[1]) & OLT:  # a >= b: no wrap
                return (max(0, a[0] - b[1]), a[1] - b[0], z, o)
            if a[1] < b[0]:
                return (a[0] - b[1] + m + 1, a[1] - b[0] + m + 1, z, o)
            return (0, m, z, o)
        if op == S.MUL:
            tz = min(w, _tz(a, w) + _tz(b, w))
            z = _mask(tz)
            if a[1] * b[1] <= m:
                return (a[0] * b[0], a[1] * b[1], z, 0)
            return (0, m, z, 0)
        if op == S.UDIV:
            if b[0] > 0:
                return (a[0] // b[1], a[1] // b[0], 0, 0)
            return _top(w)
        if op == S.UREM:
            if _is_exact(b) and b[0] and not b[0] & (b[0] - 1):   # x % 2^k = x & (2^k - 1)
                k = b[0] - 1
                return (0, min(a[1], k), (a[2] & k) | (m & ~k), a[3] & k)
            if b[0] > 0:
                return (0, min(a[1], b[1] - 1), 0, 0)
            return (0, a[1], 0, 0)
        if op == S.AND:
            return (0, min(a[1], b[1]), a[2] | b[2], a[3] & b[3])
        if op == S.OR:
            return (max(a[0], b[0]), m, a[2] & b[2], a[3] | b[3])
        if op == S.XOR:
            return (0, m, (a[2] & b[2]) | (a[3] & b[3]), (a[2] & b[3]) | (a[3] & b[2]))
        if op in (S.SHL, S.LSHR) and _is_exact(b):
            s = b[0]
            if s >= w:
                return _exact(0, w)
            if op == S.SHL:
                z, o = ((a[2] << s) | _mask(s)) & m, (a[3] << s) & m
                if (a[1] << s) <= m:
                    return (a[0] << s, a[1] << s, z, o)
                return (0, m, z, o)
            return (a[0] >> s, a[1] >> s, (a[2] >> s) | (m & ~(m >> s)), a[3] >> s)
        if op == S.LSHR:
            return (0, a[1], 0, 0)
        return _top(w)

    def _forward_bool(self, i: int, op: int, ar):
        av = self.av
        if op == S.BNOT:
            c = av[ar[0]]
            return (BT if c & BF else 0) | (BF if c & BT else 0)
        if op in (S.BAND, S.BOR, S.BXOR, S.BEQ):
            a, b = av[ar[0]], av[ar[1]]
            out = 0
            for x in (False, True):
                if not a & (BT if x else BF):
                    continue
                for y in (False, True):
                    if not b & (BT if y else BF):
                        continue
                    r = (x and y) if op == S.BAND else (x or y) if op == S.BOR else (x != y) if op == S.BXOR else (x == y)
                    out |= BT if r else BF
            return out
        if op == S.BITE:
            c = av[ar[0]]
            if c == BT:
                return av[ar[1]]
            if c == BF:
                return av[ar[2]]
            return av[ar[1]] | av[ar[2]]
        if op in _TRUE_ORD or op in (S.UADD_NOOVF, S.UMUL_NOOVF):
            a, b = av[ar[0]], av[ar[1]]
            if isinstance(a, int):  # Bool == Bool through EQ
                return self._forward_bool(i, S.BEQ, ar)
            w = self.w[ar[0]]
            out = BB
            if op == S.UADD_NOOVF:
                if a[1] + b[1] <= _mask(w):
                    out = BT
                elif a[0] + b[0] > _mask(w):
                    out = BF
                return out
            if op == S.UMUL_NOOVF:
                if a[1] * b[1] <= _mask(w):
                    out = BT
                elif a[0] * b[0] > _mask(w):
                    out = BF
                return out
            ords = self._orders(a, b, w, op in _CMP_S)
            cp = self.cmp_pair.get(i)
            if cp is not None:
                p, sw, _ = cp
                ps = self.pairs[p]
                ords &= _swap(ps) if sw else ps
            t_ord = _TRUE_ORD[op]
            if op == S.USUB_NOUDF:  # BVSubNoUnderflow(a, b): b <= a, i.e. a >= b
                t_ord = OGT | OEQ
            out = 0
            if ords & t_ord:
                out |= BT
            if ords & ~t_ord & OALL:
                out |= BF
            if not out:
                raise Empty
            return out
        return BB

    def _pair_ord(self, a: int, b: int, signed: bool = False) -> int:
        """The orderings of node a vs node b the compared-pair facts allow (OALL if the two
        are never compared)."""
        if a == b:
            return OEQ
        x, y = (a, b) if a < b else (b, a)
        p = self.pair_of.get((x, y, signed))
        if p is None:
            return OALL
        return self.pairs[p] if a < b else _swap(self.pairs[p])

    @staticmethod
    def _orders(a, b, w: int, signed: bool) -> int:
        """Orderings of x vs y possible for x in a, y in b."""
        if signed:
            a, b = _flip(a, w), _flip(b, w)
        s = 0
        if a[0] < b[1]:
            s |= OLT
        if a[1] > b[0]:
            s |= OGT
        if max(a[0], b[0]) <= min(a[1], b[1]) and not ((a[3] & b[2]) | (a[2] & b[3])):
            s |= OEQ
        return s

    # ------------------------------------------------------------ backward
    def backward(self, i: int, work: List[int]) -> None:
        """Narrow node i's operands (and pair orderings) by node i's abstract value."""
        t = self.t[i]
        op, ar, v = t.op, self.args[i], self.av[i]
        av = self.av
        if self.isb[i]:
            if op == S.BNOT:
                self._set(ar[0], (BT if v & BF else 0) | (BF if v & BT else 0), work)
            elif op == S.BAND:
                if v == BT:
                    self._set(ar[0], BT, work)
                    self._set(ar[1], BT, work)
                elif v == BF:
                    for x, y in ((0, 1), (1, 0)):
                        if av[ar[x]] == BT:
                            self._set(ar[y], BF, work)
            elif op == S.BOR:
                if v == BF:
                    self._set(ar[0], BF, work)
                    self._set(ar[1], BF, work)
                elif v == BT:
                    for x, y in ((0, 1), (1, 0)):
                        if av[ar[x]] == BF:
                            self._set(ar[y], BT, work)
                    self._or_of_compares(ar, work)
            elif op in (S.BXOR, S.BEQ) or (op == S.EQ and self.isb[ar[0]]):
                if v != BB:
                    same = (v == BT) == (op != S.BXOR)
                    for x, y in ((0, 1), (1, 0)):
                        c = av[ar[x]]
                        if c != BB:
                            self._set(ar[y], c if same else (BB ^ c), work)
            elif op == S.BITE:
                c = av[ar[0]]
                if c == BT:
                    self._set(ar[1], v, work)
                elif c == BF:
                    self._set(ar[2], v, work)
                else:
                    if not av[ar[1]] & v:
                        self._set(ar[0], BF, work)
                    if not av[ar[2]] & v:
                        self._set(ar[0], BT, work)
            elif op in _TRUE_ORD or op in (S.UADD_NOOVF, S.UMUL_NOOVF):
                if v != BB:
                    self._backward_cmp(i, op, ar, v == BT, work)
            return
        w = t.width
        m = _mask(w)
        if op == S.ITE:
            c = av[ar[0]]
            if c == BT:
                self._set(ar[1], v, work)
            elif c == BF:
                self._set(ar[2], v, work)
            else:
                for br, bad in ((1, BF), (2, BT)):
                    try:
                        _meet(av[ar[br]], v, w)
                    except Empty:
                        self._set(ar[0], bad, work)
            return
        if op in (S.CONST, S.VAR, S.UFAPP, S.UFINV):
            if op in (S.UFAPP, S.UFINV):
                self._congruence(i, work)
            return
        a = av[ar[0]]
        if op == S.EXTRACT:
            hi_b, lo_b = t.params
            wa = self.w[ar[0]]
            self._set(ar[0], (0, _mask(wa), v[2] << lo_b, v[3] << lo_b), work)
            return
        if op == S.ZEXT:
            wa = self.w[ar[0]]
            if v[1] >> wa:
                self._set(ar[0], (v[0] if v[0] <= _mask(wa) else _mask(wa) + 1, _mask(wa), v[2], v[3]), work)
            else:
                self._set(ar[0], (v[0], v[1], v[2], v[3]), work)
            return
        if op == S.NOT:
            self._set(ar[0], (m - v[1], m - v[0], v[3], v[2]), work)
            return
        if op == S.CONCAT:
            wb = self.w[ar[1]]
            mb = _mask(wb)
            self._set(ar[0], (v[0] >> wb, v[1] >> wb, v[2] >> wb, v[3] >> wb), work)
            if (v[0] >> wb) == (v[1] >> wb):
                self._set(ar[1], (v[0] & mb, v[1] & mb, v[2] & mb, v[3] & mb), work)
            else:
                self._set(ar[1], (0, mb, v[2] & mb, v[3] & mb), work)
            return
        if len(ar) < 2:
            return
        b = av[ar[1]]
        if op == S.ADD:
            for x, y in ((0, 1), (1, 0)):
                o = av[ar[y]]
                if _is_exact(o):
                    c = o[0]
                    if v[0] >= c:
                        self._set(ar[x], (v[0] - c, v[1] - c, 0, 0), work)
                    elif v[1] < c:
                        self._set(ar[x], (v[0] - c + m + 1, v[1] - c + m + 1, 0, 0), work)
                    if _is_exact(v):
                        self._set(ar[x], _exact(v[0] - c, w), work)
            return
        if op == S.SUB:  # r = a - b: a = r + b, b = a - r
            if _is_exact(b):
                c = b[0]
                if v[1] + c <= m:
                    self._set(ar[0], (v[0] + c, v[1] + c, 0, 0), work)
                elif v[0] + c > m:
                    self._set(ar[0], (v[0] + c - m - 1, v[1] + c - m - 1, 0, 0), work)
            if _is_exact(a) and _is_exact(v):
                self._set(ar[1], _exact(a[0] - v[0], w), work)
            if _is_exact(b) and _is_exact(v):
                self._set(ar[0], _exact(v[0] + b[0], w), work)
            return
        if op == S.AND:
            for x, y in ((0, 1), (1, 0)):
                o = av[ar[y]]
                self._set(ar[x], (v[0], m, v[2] & o[3], v[3]), work)
            return
        if op == S.UREM and _is_exact(b) and b[0] and not b[0] & (b[0] - 1):
            k = b[0] - 1   # x % 2^k: the low k bits of x are the result's
            self._set(ar[0], (0, m, v[2] & k, v[3] & k), work)
            return
        if op == S.OR:
            for x, y in ((0, 1), (1, 0)):
                o = av[ar[y]]
                self._set(ar[x], (0, v[1], v[2], v[3] & o[2]), work)
            return
        if op == S.XOR:
            for x, y in ((0, 1), (1, 0)):
                o = av[ar[y]]
                # bit known in r and in the other operand: known here
                z = (v[2] & o[2]) | (v[3] & o[3])
                one = (v[3] & o[2]) | (v[2] & o[3])
                self._set(ar[x], (0, m, z, one), work)
            return
        if op in (S.SHL, S.LSHR) and _is_exact(b) and b[0] < w:
            s = b[0]
            if op == S.LSHR:  # r = a >> s: a's bits s.. are r's bits 0..
                self._set(ar[0], (0, m, (v[2] << s) & m, (v[3] << s) & m), work)
            else:  # r = a << s: a's bits 0..w-s are r's bits s..
                self._set(ar[0], (0, m, v[2] >> s, v[3] >> s), work)
            return
        if op == S.MUL:
            # x * c = r (mod 2^w) with c exact: x * c = j * 2^w + r for some wrap count j, so
            # x lies in the union over j of [(j * 2^w + r.lo) / c, (j * 2^w + r.hi) / c]
            # (rounded inwards) within x's interval; x gets the hull of the non-empty pieces
            for x, y in ((0, 1), (1, 0)):
                o = av[ar[y]]
                if not _is_exact(o) or o[0] == 0:
                    continue
                c, xv = o[0], av[ar[x]]
                j0, j1 = xv[0] * c >> w, xv[1] * c >> w
                if j1 - j0 > 64:
                    continue
                lo = hi = None
                for j in range(j0, j1 + 1):
                    plo = max(xv[0], -(-((j << w) + v[0]) // c))
                    phi = min(xv[1], ((j << w) + v[1]) // c)
                    if plo <= phi:
                        lo = plo if lo is None else lo
                        hi = phi
                if lo is None:
                    raise Empty
                self._set(ar[x], (lo, hi, 0, 0), work)
            return

    def _or_of_compares(self, ar, work: List[int]) -> None:
        """Or(cmp1(x, y), cmp2(x, y)) required true on one operand pair (ULE's and UGE's
        Or(ULT, ==) expansions, bitvec_helper.py:53-80): the pair's orderings are within the
        union of the two compares' true orderings."""
        c0, c1 = self.cmp_pair.get(ar[0]), self.cmp_pair.get(ar[1])
        if c0 is None or c1 is None or c0[0] != c1[0]:
            return
        p = c0[0]
        u = 0
        for k, (_, sw, _) in ((ar[0], c0), (ar[1], c1)):
            op = self.t[k].op
            o = OGT | OEQ if op == S.USUB_NOUDF else _TRUE_ORD[op]
            u |= _swap(o) if sw else o
        self._set_pair(p, u, work)
        x, y, signed = self.pair_xy[p]
        self._narrow_by_order(x, y, self.pairs[p], signed, work)

    def _backward_cmp(self, i: int, op: int, ar, truth: bool, work: List[int]) -> None:
        av = self.av
        x, y = ar
        a, b = av[x], av[y]
        w = self.w[x]
        m = _mask(w)
        if op == S.UADD_NOOVF:
            if truth:  # a + b <= m
                self._set(x, (0, m - b[0], 0, 0), work)
                self._set(y, (0, m - a[0], 0, 0), work)
            else:  # a + b > m
                self._set(x, (max(0, m + 1 - b[1]), m, 0, 0), work)
                self._set(y, (max(0, m + 1 - a[1]), m, 0, 0), work)
            return
        if op == S.UMUL_NOOVF:
            if truth:
                if b[0] > 0:
                    self._set(x, (0, m // b[0], 0, 0), work)
                if a[0] > 0:
                    self._set(y, (0, m // a[0], 0, 0), work)
            else:
                if b[1] == 0 or a[1] == 0:
                    raise Empty
                self._set(x, (-(-(m + 1) // b[1]), m, 0, 0), work)
                self._set(y, (-(-(m + 1) // a[1]), m, 0, 0), work)
            return
        t_ord = _TRUE_ORD[op]
        if op == S.USUB_NOUDF:
            t_ord = OGT | OEQ
        want = t_ord if truth else OALL & ~t_ord
        cp = self.cmp_pair.get(i)
        if cp is not None:
            p, sw, _ = cp
            self._set_pair(p, _swap(want) if sw else want, work)
            ps = self.pairs[p]
            want &= _swap(ps) if sw else ps
        self._narrow_by_order(x, y, want, op in _CMP_S, work)

    def _narrow_by_order(self, x: int, y: int, want: int, signed: bool, work: List[int]) -> None:
        av = self.av
        a, b = av[x], av[y]
        w = self.w[x]
        if want == OEQ:
            self._set(x, b, work)
            self._set(y, self.av[x], work)
            return
        if signed:
            fa, fb = _flip(a, w), _flip(b, w)
            if fa is None or fb is None:
                return
            na, nb = _order_bounds(fa, fb, want)
            if na is not None:
                self._set(x, _unflip(na, w), work)
            if nb is not None:
                self._set(y, _unflip(nb, w), work)
            return
        na, nb = _order_bounds(a, b, want)
        if na is not None:
            self._set(x, na, work)
        if nb is not None:
            self._set(y, nb, work)
        if not want & OEQ and _is_exact(b):
            c = b[0]
            aa = self.av[x]
            if aa[0] == c:
                self._set(x, (c + 1, aa[1], 0, 0), work)
            elif aa[1] == c:
                self._set(x, (aa[0], c - 1, 0, 0), work)
        if not want & OEQ and _is_exact(self.av[x]):
            c = self.av[x][0]
            bb = self.av[y]
            if bb[0] == c:
                self._set(y, (c + 1, bb[1], 0, 0), work)
            elif bb[1] == c:
                self._set(y, (bb[0], c - 1, 0, 0), work)

    def _congruence(self, i: int, work: List[int]) -> None:
        """f(a) and f(b) of one function: a == b (same term, or equal exact values) gives
        f(a) == f(b); f(a) and f(b) known different gives a != b (by values only)."""
        peers = self.uf_peers.get(i)
        if not peers:
            return
        ai = self.args[i][0]
        for j in peers:
            aj = self.args[j][0]
            p = self.pair_of.get((min(ai, aj), max(ai, aj), False))
            if ai == aj or (_is_exact(self.av[ai]) and self.av[ai] == self.av[aj]) or \
                    (p is not None and self.pairs[p] == OEQ):
                self._set(j, self.av[i], work)
                self._set(i, self.av[j], work)

    # ------------------------------------------------------------ linear forms
    def _forms(self) -> List:
        """Every BV node's value as c + sum(coef * atom) mod 2^w under the current abstract
        values: exact nodes are constants, decided ITEs are their chosen branch, ADD / SUB /
        NEG / NOT and MUL by an exact value combine their operands' forms; a UF application is
        the atom (function, form of its argument), so f(x) and f(y) with equal argument forms
        are one atom; a node whose compared pair is known "=" takes its partner's form; any
        other node is an atom of its own.  None for Bool nodes."""
        forms: List = [None] * self.n
        av = self.av
        self.atom_node: Dict = {}
        self.steps += self.n // 4   # a pass over the DAG counts against the step budget
        # a compared pair known equal: the later node takes the earlier one's form
        rep: Dict[int, int] = {}
        for p, (x, y, _) in enumerate(self.pair_xy):
            if self.pairs[p] == OEQ and x != y and not self.isb[x]:
                rep[y] = min(x, rep.get(y, x))
        for i in range(self.n):
            if self.isb[i]:
                continue
            t, w, ar = self.t[i], self.w[i], self.args[i]
            m = _mask(w)
            a = av[i]
            op = t.op
            f = None
            if _is_exact(a):
                f = (a[0], {})
            elif op == S.ITE and av[ar[0]] in (BT, BF):
                f = forms[ar[1] if av[ar[0]] == BT else ar[2]]
            elif op in (S.ADD, S.SUB):
                f = _lin_add(forms[ar[0]], forms[ar[1]], -1 if op == S.SUB else 1, m)
            elif op == S.NEG:
                f = _lin_scale(forms[ar[0]], m, m)
            elif op == S.NOT:  # ~x = -x - 1
                f = _lin_add((m, {}), forms[ar[0]], -1, m)
            elif op == S.MUL:
                for x, y in ((0, 1), (1, 0)):
                    if _is_exact(av[ar[x]]):
                        f = _lin_scale(forms[ar[y]], av[ar[x]][0], m)
                        break
            elif op in (S.UFAPP, S.UFINV):
                fa = forms[ar[0]]
                key = ("u", op, repr(t.params), _form_key(fa) if fa is not None else ("n", ar[0]))
                self.atom_node.setdefault(key, i)
                f = (0, {key: 1})
            if f is None or len(f[1]) > 24:
                f = (0, {("n", i): 1})
            j = rep.get(i)
            if j is not None:  # known equal to node j: one form (a constant difference is a contradiction)
                d = _lin_add(f, forms[j], -1, m)
                if not d[1] and d[0]:
                    raise Empty
                f = forms[j]
            forms[i] = f
        return forms

    def _diff_range(self, d, m: int):
        """The integer range of a difference form d = k + sum(c * atom) with every atom in its
        interval (a coefficient above m / 2 counts as negative), or None if it leaves [0, m]."""
        lo = hi = d[0]
        for key, c in d[1].items():
            i = key[1] if key[0] == "n" else self.atom_node.get(key)
            if i is None:
                return None
            a = self.av[i]
            if c <= m // 2:
                lo += c * a[0]
                hi += c * a[1]
            else:
                c = m + 1 - c
                lo -= c * a[1]
                hi -= c * a[0]
        if lo < 0 or hi > m:
            return None
        return lo, hi

    def linear(self, work: List[int]) -> None:
        """Compares whose operands' forms differ by a constant k: x = y + k mod 2^w, so x > y
        iff k != 0 and y + k does not wrap (y <= 2^w - 1 - k), x < y iff it wraps, x == y iff
        k == 0.  That bounds the pair's orderings (and so the compare's truth, open or not) by
        y's interval; a compare required true or false narrows y's interval to the side it
        needs (or empties the branch).  A difference that is not constant but whose atoms'
        intervals keep it inside [lo, hi] within [0, 2^w - 1] (x = y + D, D in [lo, hi]) bounds
        the orderings the same way: "=" only if lo == 0, ">" if y + max(lo, 1) can stay below
        2^w, "<" only if y + hi can wrap (either operand order)."""
        forms = self._forms()
        av = self.av
        self._injective(forms, work)
        for i, (p, sw, signed) in self.cmp_pair.items():
            x, y = self.args[i]
            fx, fy = forms[x], forms[y]
            if fx is None or fy is None:
                continue
            w = self.w[x]
            m = _mask(w)
            d = _lin_add(fx, fy, -1, m)
            k = None
            if not d[1]:
                k = d[0]
                if k == 0:
                    poss = OEQ
                elif signed:
                    poss = OLT | OGT
                else:
                    yv = av[y]
                    poss = (OGT if yv[0] <= m - k else 0) | (OLT if yv[1] > m - k else 0)
            elif signed:
                continue
            else:
                r = self._diff_range(d, m)
                flip = False
                if r is None:
                    r = self._diff_range(_lin_scale(d, m, m), m)   # y - x
                    flip = True
                    if r is None:
                        continue
                lo, hi = r
                base = x if flip else y   # the operand D is added to
                b = av[base]
                poss = (OEQ if lo == 0 else 0) | \
                    (OGT if hi > 0 and b[0] + max(lo, 1) <= m else 0) | \
                    (OLT if b[1] + hi > m else 0)
                # D is one node d and BVAddNoOverflow(base, d) is decided: the sum wraps (x < y)
                # or it does not (x >= y) -- bitvec_helper.py's SafeMath-style overflow checks
                dd = _lin_scale(d, m, m) if flip else d
                if dd[0] == 0 and len(dd[1]) == 1:
                    (key, coef), = dd[1].items()
                    if coef == 1 and key[0] == "n":
                        t = self.noovf.get((min(base, key[1]), max(base, key[1])))
                        if t is not None and av[t] == BT:
                            poss &= OGT | OEQ
                        elif t is not None and av[t] == BF:
                            poss &= OLT
                if flip:
                    poss = _swap(poss)
            self._set_pair(p, _swap(poss) if sw else poss, work)
            op = self.t[i].op
            t_ord = OGT | OEQ if op == S.USUB_NOUDF else _TRUE_ORD[op]
            self._set(i, (BT if poss & t_ord else 0) | (BF if poss & ~t_ord & OALL else 0), work)
            v = av[i]
            if k is None or k == 0 or signed or v not in (BT, BF):
                continue
            want = (t_ord if v == BT else OALL & ~t_ord) & (OLT | OGT)
            if want == OGT:      # y + k must not wrap
                self._set(y, (0, m - k, 0, 0), work)
            elif want == OLT:    # y + k must wrap
                self._set(y, (m - k + 1, m, 0, 0), work)
            elif not want:
                raise Empty

    def _differ(self, a: int, b: int, forms) -> bool:
        """Nodes a and b can never be equal: their forms differ by a non-zero constant, their
        compared pair excludes "=", or their abstract values cannot meet."""
        if a == b:
            return False
        fa, fb = forms[a], forms[b]
        if fa is not None and fb is not None:
            d = _lin_add(fa, fb, -1, _mask(self.w[a]))
            if not d[1]:
                return d[0] != 0
        if not self._pair_ord(a, b) & OEQ:
            return True
        return not self._orders(self.av[a], self.av[b], self.w[a], False) & OEQ

    def _injective(self, forms, work: List[int]) -> None:
        """Two applications of an injective function (inverse axiom required true): equal
        values with different arguments empty the branch; different arguments exclude "=" from
        every compare of one application with a value the other is known to equal; equal
        values make the arguments equal."""
        av = self.av
        for apps in self.inj.values():
            live = [a for a, e in apps if av[e] == BT]
            for x in range(len(live)):
                for y in range(x + 1, len(live)):
                    i, j = live[x], live[y]
                    ai, aj = self.args[i][0], self.args[j][0]
                    same_val = (_is_exact(av[i]) and av[i] == av[j]) or self._pair_ord(i, j) == OEQ
                    if self._differ(ai, aj, forms):
                        if same_val:
                            raise Empty
                        for k, o in ((i, j), (j, i)):
                            if not _is_exact(av[o]):
                                continue
                            for c in self.users[k]:
                                cp = self.cmp_pair.get(c)
                                if cp is None:
                                    continue
                                other = [z for z in self.args[c] if z != k]
                                if other and _is_exact(av[other[0]]) and av[other[0]][0] == av[o][0]:
                                    pp, sw, _ = cp
                                    self._set_pair(pp, OALL & ~OEQ, work)
                    elif same_val and self.w[ai] == self.w[aj]:
                        self._set(ai, av[aj], work)
                        self._set(aj, av[ai], work)

    def saturate(self, seeds: Optional[List[int]] = None, rounds: int = 4) -> None:
        """propagate, then the linear pass and propagation again while it narrows something."""
        self.propagate(seeds)
        for _ in range(rounds):
            if self.steps > self.budget:
                return
            work: List[int] = []
            self.linear(work)
            if not work:
                return
            self.propagate(work)

    # ------------------------------------------------------------ driver
    def propagate(self, seeds: Optional[List[int]] = None) -> None:
        """Work-list propagation to a fixpoint (or the step budget); Empty if refuted."""
        work: List[int] = list(range(self.n)) if seeds is None else list(seeds)
        self.creep = {}
        if seeds is None:
            for r in self.roots:
                self._set(r, BT, work)
        head = 0
        while head < len(work):
            i = work[head]
            head += 1
            if head > 4096:  # compact the queue
                work = work[head:]
                head = 0
            self.steps += 1
            if self.steps > self.budget:
                return
            fv = self.forward(i)
            self._set(i, fv, work)
            self.backward(i, work)
            for u in self.users[i]:
                nf = self.forward(u)
                old = self.av[u]
                self._set(u, nf, work)
                if self.av[u] == old:
                    self.backward(u, work)

    def atoms(self) -> List[int]:
        """Open Bool nodes worth a case split, nearest the roots first: operands of
        disjunctions that must hold, ITE conditions, compares."""
        out, seen = [], set()
        for i in reversed(range(self.n)):
            t = self.t[i]
            if t.op == S.BOR and self.av[i] == BT:
                for a in self.args[i]:
                    if self.av[a] == BB and a not in seen:
                        seen.add(a)
                        out.append(a)
        # ITE conditions: those of ITEs that feed arithmetic or compares before those that
        # only assemble bytes (a calldata word's CONCAT of per-byte "in bounds" selects)
        late = []
        for i in reversed(range(self.n)):
            t = self.t[i]
            if t.op in (S.ITE, S.BITE):
                c = self.args[i][0]
                if self.av[c] == BB and c not in seen:
                    seen.add(c)
                    if self.users[i] and all(self.t[u].op in (S.CONCAT, S.EXTRACT) for u in self.users[i]):
                        late.append(c)
                    else:
                        out.append(c)
        out.extend(late)
        for i in reversed(range(self.n)):
            if self.isb[i] and self.av[i] == BB and i not in seen and self.t[i].op in _TRUE_ORD:
                seen.add(i)
                out.append(i)
        return out


def _lin_add(f, g, sign: int, m: int):
    """f + sign * g of two linear forms mod m + 1 (None if either is None)."""
    if f is None or g is None:
        return None
    c = (f[0] + sign * g[0]) & m
    out = dict(f[1])
    for a, k in g[1].items():
        nk = (out.get(a, 0) + sign * k) & m
        if nk:
            out[a] = nk
        else:
            out.pop(a, None)
    return (c, out)


def _lin_scale(f, k: int, m: int):
    if f is None:
        return None
    out = {}
    for a, c in f[1].items():
        nc = (c * k) & m
        if nc:
            out[a] = nc
    return ((f[0] * k) & m, out)


def _form_key(f):
    return (f[0], tuple(sorted(f[1].items())))


def _swap(s: int) -> int:
    return (s & OEQ) | ((s & OLT) << 2) | ((s & OGT) >> 2)


def _flip(a, w: int):
    """Signed order -> unsigned order: x ^ 2^(w-1) (the sign bit must be known or the
    interval must not straddle it for the bounds to carry over)."""
    sb = 1 << (w - 1)
    z, o = a[2], a[3]
    nz = (z & ~sb) | (sb if o & sb else 0)
    no = (o & ~sb) | (sb if z & sb else 0)
    if (a[0] & sb) == (a[1] & sb):
        return (a[0] ^ sb, a[1] ^ sb, nz, no)
    return (0, _mask(w), nz, no)


def _unflip(a, w: int):
    return _flip(a, w)


def _order_bounds(a, b, want: int):
    """Bounds on x (in a) and y (in b) under the orderings `want` of x vs y."""
    if want == OLT:
        return (a[0], min(a[1], b[1] - 1), 0, 0), (max(b[0], a[0] + 1), b[1], 0, 0)
    if want == OLT | OEQ:
        return (a[0], min(a[1], b[1]), 0, 0), (max(b[0], a[0]), b[1], 0, 0)
    if want == OGT:
        return (max(a[0], b[0] + 1), a[1], 0, 0), (b[0], min(b[1], a[1] - 1), 0, 0)
    if want == OGT | OEQ:
        return (max(a[0], b[0]), a[1], 0, 0), (b[0], min(b[1], a[1]), 0, 0)
    return None, None


TIERS = ((2, 8, 60000), (3, 8, 600000))   # (split depth, atoms per level, step budget)


def refute(roots: Sequence, depth: int = 0, max_atoms: int = 8, budget: int = 0, tiers=None) -> bool:
    """True iff the conjunction of `roots` (smt terms) is re-proved UNSAT: propagation with the
    linear pass, failed-literal probing, then case splits on up to max_atoms open atoms per
    level, `depth` levels, within `budget` propagation steps.  With depth 0 the TIERS run in
    turn (a cheap search first, a deeper one for what it leaves)."""
    for d, na, b in tiers or (((depth, max_atoms, budget or 200000),) if depth else TIERS):
        if _refute_once(roots, d, na, b):
            return True
    return False


def _refute_once(roots: Sequence, depth: int, max_atoms: int, budget: int) -> bool:
    try:
        C = Checker(roots, budget)
    except RecursionError:  # pragma: no cover
        return False
    try:
        C.saturate()
    except Empty:
        return True
    if C.steps > C.budget:
        return False
    base = C.snapshot()
    if _split(C, depth, max_atoms):
        return True
    C.restore(base)
    C.steps = 0   # the bisection gets a budget of its own
    return _bisect(C, BISECT_LEVELS)


BISECT_LEVELS = 8


def _bisect(C: Checker, levels: int, max_vars: int = 4) -> bool:
    """Interval bisection: a node (a variable, a calldata word, ...) whose interval the
    propagation bounded is cut in halves, each half propagated (with the linear pass), `levels` deep; refuted when every
    leaf empties.  Bit-length midpoints first (a range over several orders of magnitude), then
    arithmetic ones."""
    cands = []
    for i in range(C.n):
        if C.t[i].op not in (S.CONST, S.ITE) and not C.isb[i]:
            lo, hi = C.av[i][0], C.av[i][1]
            if lo != hi and (lo > 0 or hi < _mask(C.w[i])):
                cands.append((C.t[i].op != S.VAR, hi - lo, i))   # variables first
    base = C.snapshot()
    for _, _, i in sorted(cands)[:max_vars]:
        if _halves(C, i, levels):
            return True
        C.restore(base)
        if C.steps > C.budget:
            return False
    return False


def _halves(C: Checker, i: int, levels: int) -> bool:
    lo, hi = C.av[i][0], C.av[i][1]
    if levels <= 0 or lo == hi:
        return False
    bl, bh = lo.bit_length(), hi.bit_length()
    mid = (1 << ((bl + bh) // 2)) - 1 if bh > bl + 1 else (lo + hi) // 2
    mid = min(max(mid, lo), hi - 1)
    base = C.snapshot()
    for part in ((lo, mid), (mid + 1, hi)):
        C.restore(base)
        try:
            work: List[int] = []
            C._set(i, (part[0], part[1], 0, 0), work)
            C.saturate(work)
        except Empty:
            continue
        if C.steps > C.budget or not _halves(C, i, levels - 1):
            C.restore(base)
            return False
    C.restore(base)
    return True


def _probe(C: Checker, max_probe: int):
    """Failed-literal probing: an atom one of whose sides empties is fixed to the other side at
    no depth cost, until no probed atom is forced.  -> True if both sides of an atom empty
    (refuted), None if the step budget ran out, False otherwise (C holds the forced state)."""
    while True:
        base = C.snapshot()
        forced = False
        for a in C.atoms()[:max_probe]:
            open_sides = []
            for side in (BT, BF):
                C.restore(base)
                try:
                    work: List[int] = []
                    C._set(a, side, work)
                    C.saturate(work)
                    open_sides.append(side)
                except Empty:
                    pass
                if C.steps > C.budget:
                    C.restore(base)
                    return None
            if not open_sides:
                return True
            if len(open_sides) == 1:
                C.restore(base)
                work = []
                C._set(a, open_sides[0], work)
                C.saturate(work)
                forced = True
                break
        if not forced:
            C.restore(base)
            return False


def _split(C: Checker, depth: int, max_atoms: int) -> bool:
    r = _probe(C, 2 * max_atoms)
    if r is not False:
        return bool(r)
    if depth <= 0:
        return False
    base = C.snapshot()
    for a in C.atoms()[:max_atoms]:
        closed = True
        for side in (BT, BF):
            C.restore(base)
            try:
                work: List[int] = []
                C._set(a, side, work)
                C.saturate(work)
            except Empty:
                continue
            if C.steps > C.budget or not _split(C, depth - 1, max_atoms):
                closed = False
                break
        C.restore(base)
        if closed:
            return True
        if C.steps > C.budget:
            return False
    return False
