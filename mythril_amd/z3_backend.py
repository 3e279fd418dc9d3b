"""z3 as the pre-filter's fallback solver, and z3's evaluator as the witness re-check.

The reference answers every query with z3 (analysis/solver.py:37-61 builds an
``Optimize``, constraints.py:41-50 a ``Solver`` with a 100 ms timeout).  Behind
``solver.set_backend(Z3Backend())`` this adapter does the same for the states the GPU
and the host pre-check leave open, with the reference's own z3 constraints: terms that
came from z3 (mythril_amd.z3_lower) are mapped back to the expressions they were
lowered from, so z3 sees exactly what it would have seen without the pre-filter.

``recheck(terms, witness)`` re-checks a GPU witness with z3 before it is trusted
(BASELINE.json north_star): every variable, uninterpreted application and base-array
read the witness assigns is pinned to its value, and z3 must answer sat for the
original constraints under those pins — an evaluation, not a search.  A witness z3
rejects is dropped and the query goes to the fallback unchanged.  Terms built by the
laser.smt mirror (no z3 origin) cannot be re-checked and are reported as such.

``recheck_refutation(terms)`` is the same audit for the UNSAT side: a refutation by
the host pre-check (mgp_refute) answers unsat with no z3 call, which is a deliberate
divergence from the reference for states z3 would time out on.  With
``recheck_refutations=f`` > 0 a deterministic fraction f of the refuted states (every
state when f = 1) is also put to z3 with the reference's timeout; a z3 `sat` there is a
pre-check soundness bug, counted in SolverStatistics.refute_disagreements, and z3's
answer wins.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

from . import solver as SV
from . import z3_lower


class Z3Backend(SV.Backend):
    name = "z3"

    def __init__(self, z3=None, recheck_timeout_ms: int = 1000, recheck_refutations: float = 0.0,
                 refutation_timeout_ms: int = 10000):
        if z3 is None:
            import z3  # noqa: F811  (the reference's dependency, requirements.txt:30)
        if not 0.0 <= recheck_refutations <= 1.0:
            raise ValueError("recheck_refutations is a fraction in [0, 1]")
        self.z3 = z3
        self.recheck_timeout_ms = recheck_timeout_ms
        self.rechecks = 0
        self.recheck_failures = 0
        self.recheck_refutations = recheck_refutations
        self.refutation_timeout_ms = refutation_timeout_ms
        self._refutations_seen = 0

    # ------------------------------------------------------------ helpers
    def _lowering(self) -> Optional[z3_lower.Z3Lowering]:
        return z3_lower.lowering_of_module(self.z3)

    def _exprs(self, terms) -> Optional[list]:
        lw = self._lowering()
        if lw is None:
            return None
        out = []
        for t in terms:
            e = lw.roots.get(t.tid)
            if e is None:
                return None
            out.append(e)
        return out

    def _objective(self, t):
        lw = self._lowering()
        e = None if lw is None else (lw.roots.get(t.tid) or lw.origin.get(t.tid))
        return None if isinstance(e, tuple) else e

    # ----------------------------------------------------------- Backend
    def check(self, terms: Sequence, timeout_ms: int, minimize=(), maximize=()) -> Tuple[str, Optional[SV.Model]]:
        """analysis/solver.py:37-61 (Optimize + objectives) / constraints.py:41-50 (Solver)."""
        z3 = self.z3
        exprs = self._exprs(terms)
        if exprs is None:
            return SV.unknown, None
        s = z3.Optimize() if (minimize or maximize) else z3.Solver()
        s.set("timeout", int(timeout_ms))
        s.add(*exprs)
        for objs, fn in ((minimize, "minimize"), (maximize, "maximize")):
            for t in objs:
                e = self._objective(t)
                if e is None:
                    return SV.unknown, None
                getattr(s, fn)(e)
        r = s.check()
        if r == z3.sat:
            return SV.sat, SV.Model([], raw=s.model())
        if r == z3.unsat:
            return SV.unsat, None
        return SV.unknown, None

    def check_raw(self, raw_constraints: Sequence, lowered: Sequence, timeout_ms: int, minimize=(),
                  maximize=()) -> Tuple[str, Optional[SV.Model]]:
        """A query the pre-filter could not lower: z3 on the caller's own constraints
        (laser.smt wrappers or z3 expressions) plus the lowered part."""
        z3 = self.z3
        low = self._exprs(lowered) if lowered else []
        if low is None:
            return SV.unknown, None
        exprs = [getattr(c, "raw", c) for c in raw_constraints] + low
        s = z3.Optimize() if (minimize or maximize) else z3.Solver()
        s.set("timeout", int(timeout_ms))
        s.add(*exprs)
        for objs, fn in ((minimize, "minimize"), (maximize, "maximize")):
            for t in objs:
                e = self._objective(t) if not z3_lower.is_z3_expr(getattr(t, "raw", t)) else getattr(t, "raw", t)
                if e is None:
                    return SV.unknown, None
                getattr(s, fn)(e)
        r = s.check()
        if r == z3.sat:
            return SV.sat, SV.Model([], raw=s.model())
        return (SV.unsat, None) if r == z3.unsat else (SV.unknown, None)

    def recheck(self, terms: Sequence, witness) -> Optional[bool]:
        """True: z3 confirms the witness; False: z3 rejects it; None: not checkable (terms
        without a z3 origin, or a witness that is not a GPU slot witness)."""
        z3 = self.z3
        lw = self._lowering()
        exprs = self._exprs(terms)
        if exprs is None or lw is None or not hasattr(witness, "_vt"):
            return None
        vt, v0, v1 = witness._vt, witness._v0, witness._v1
        vals = [int.from_bytes(bytes(witness.vals[i].tobytes()), "little") for i in range(v1 - v0)]
        pins = []
        i = 0
        while i < v1 - v0:
            full = int(vt.var_full[v0 + i])
            k = max(1, (full + 255) // 256)
            if int(vt.var_kind[v0 + i]) == 2:  # pinned constant of the GPU program
                i += k
                continue
            value = 0
            for j in range(k):
                value |= (vals[i + j] & ((1 << int(vt.var_width[v0 + i + j])) - 1)) << (256 * j)
            e = lw.origin.get(int(vt.var_tid[v0 + i]))
            if isinstance(e, tuple):  # a base-array read: (array, index)
                e = z3.Select(e[0], e[1])
            if e is None:
                return None
            if e.sort().kind() == z3.Z3_BOOL_SORT:
                pins.append(e == z3.BoolVal(bool(value)))
            else:
                pins.append(e == z3.BitVecVal(value, e.size()))
            i += k
        s = z3.Solver()
        s.set("timeout", self.recheck_timeout_ms)
        s.add(*(exprs + pins))
        self.rechecks += 1
        ok = s.check() == z3.sat
        if not ok:
            self.recheck_failures += 1
        return ok

    def recheck_refutation(self, terms: Sequence) -> Optional[Tuple[str, Optional[SV.Model]]]:
        """z3's answer for a state the pre-check refuted, for the sampled fraction
        `recheck_refutations` of them (the k-th refutation is sampled when floor(k f)
        steps); None when not sampled or not checkable (terms without a z3 origin)."""
        f = self.recheck_refutations
        if f <= 0.0:
            return None
        k = self._refutations_seen = self._refutations_seen + 1
        if int(k * f) == int((k - 1) * f):
            return None
        if self._exprs(terms) is None:
            return None
        return self.check(terms, self.refutation_timeout_ms)
