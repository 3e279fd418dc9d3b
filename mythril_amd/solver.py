"""GPU-first satisfiability front end — mirror of the reference's solver surface.

Mirrors, with the same names, argument meaning and error behaviour:

  get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True)
      mythril/analysis/solver.py:27-61 — returns a Model or raises UnsatError
      (on unsat AND on unknown/timeout); literal False -> UnsatError; Python
      bools are dropped; lru_cache'd on the hashable constraint tuple.
  Constraints.is_possible
      mythril/laser/ethereum/state/constraints.py:30-51 — cached bit; unknown
      counts as possible.
  Solver / Optimize / SolverStatistics
      mythril/laser/smt/solver/solver.py:15-105, solver_statistics.py:8-43 —
      query_count counts every check() that reaches the fallback solver.
  IndependenceSolver / DependenceMap / DependenceBucket
      mythril/laser/smt/solver/independence_solver.py:10-153 — buckets of
      constraints that share no variable, checked separately (one GPU batch).

What changes is the order: a batch of states is first evaluated on the GPU
(libmgp.so) against candidate assignments; a witness PROVES satisfiability
(`sat`).  A state without a witness goes through the host UNSAT pre-check
(mgp_refute: known bits x intervals with backward narrowing, sound), which
PROVES `unsat` for the shallow contradictions.  Everything else — no witness
and no refutation, unsupported DAG, and the model of every minimize/maximize
query (tx-sequence model values must stay bit-identical to z3's,
solver.py:88-136) — goes to the fallback backend unchanged.  The
fallback is z3 (mythril_amd.z3_backend, where z3 is installed); without it the
answer is `unknown`, which each caller maps exactly as the reference does.
"""
from __future__ import annotations

import collections
import os
import threading
import time
from functools import lru_cache
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Set, Tuple, Union

import numpy as np

from . import dag as D
from . import ir
from .smt import Bool, Expression, Term, bconst

sat, unsat, unknown = "sat", "unsat", "unknown"


class UnsatError(Exception):
    """mythril/exceptions.py:16."""


class _Singleton(type):
    _inst: Dict[type, object] = {}
    _lock = threading.Lock()

    def __call__(cls, *a, **k):
        with cls._lock:
            if cls not in cls._inst:
                cls._inst[cls] = super().__call__(*a, **k)
        return cls._inst[cls]


class SolverStatistics(metaclass=_Singleton):
    """solver_statistics.py:29-43 plus the pre-filter's own counters."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.enabled = True
        self.query_count = 0      # checks that reached the fallback solver (the reference's "z3 calls")
        self.solver_time = 0.0
        self.gpu_queries = 0      # states sent to the GPU
        self.gpu_sat = 0          # states proven SAT by a GPU witness
        self.gpu_undecided = 0
        self.refuted = 0          # states proven UNSAT by the host pre-check (mgp_refute)
        self.core_hits = 0        # states UNSAT because they contain a known UNSAT core
        self.gpu_retry = 0        # states given a second, larger candidate round
        self.gpu_time = 0.0
        self.gpu_batches = 0
        self.rechecks = 0         # GPU witnesses re-checked by the fallback's evaluator (z3)
        self.recheck_rejects = 0  # ... and rejected (the query then went to the fallback)
        self.not_lowerable = 0    # queries with a construct outside the node set
        self.refute_rechecks = 0       # host refutations the fallback re-asked (Z3Backend.recheck_refutations)
        self.refute_disagreements = 0  # ... that it answered sat: a pre-check soundness bug, z3 wins

    def __repr__(self):
        return (f"Query count: {self.query_count} \nSolver time: {self.solver_time}\n"
                f"GPU queries: {self.gpu_queries} (sat {self.gpu_sat}, refuted {self.refuted}, "
                f"undecided {self.gpu_undecided}, "
                f"{self.gpu_batches} batches, {self.gpu_time:.3f}s)")


def stat_smt_query(func: Callable):
    stats = SolverStatistics()

    def wrapper(*args, **kwargs):
        if not stats.enabled:
            return func(*args, **kwargs)
        stats.query_count += 1
        t = time.time()
        try:
            return func(*args, **kwargs)
        finally:
            stats.solver_time += time.time() - t

    return wrapper


class Model:
    """laser.smt.Model (model.py:6-59) over a {variable name: value} assignment."""

    def __init__(self, assignments: Optional[Sequence[Dict[str, int]]] = None, raw=None):
        self.assignments: List[Dict[str, int]] = list(assignments or [])
        self.raw = raw  # a fallback solver's native model, when it produced this one

    def decls(self) -> List[str]:
        out: List[str] = []
        for a in self.assignments:
            out.extend(a.keys())
        return out

    def __getitem__(self, item):
        if isinstance(item, int):
            return self.decls()[item]
        name = item.raw.params[0] if isinstance(item, Expression) else item
        for a in self.assignments:
            if name in a:
                return a[name]
        return None

    def eval(self, expression, model_completion: bool = False):
        """model.py:45-59.  Either kind of model answers with a value that has z3's
        `.as_long()` (a z3 numeral from a fallback model, a ModelValue from a GPU witness),
        so reference callers work with both; None = not determined by this model."""
        t = expression.raw if isinstance(expression, Expression) else expression
        if self.raw is not None and hasattr(self.raw, "eval"):  # a z3 model from the fallback
            if isinstance(t, Term):  # a mirror term: the z3 expression it was lowered from
                from . import z3_lower

                z = z3_lower.z3_expr_of(t)
                if z is None:
                    return None
                t = z
            return self.raw.eval(t, model_completion=model_completion)
        if isinstance(t, Term):
            if t.op == 2:  # CONST
                return ModelValue(t.params[0])
            if t.op == 1:  # VAR
                v = self[str(t.params[0])]
                if v is None:
                    return ModelValue(0) if model_completion else None
                return ModelValue(v)
        return None


class ModelValue(int):
    """An integer model value with z3's numeral accessor (BitVecNumRef.as_long)."""

    def as_long(self) -> int:
        return int(self)


# --------------------------------------------------------------- backends
class Backend:
    """Fallback solver interface: check(terms, timeout_ms, minimize, maximize) -> (result, Model|None).

    The base class is the null backend of an installation without z3: every query it gets
    is `unknown`, which each caller maps exactly as the reference maps a z3 timeout
    (is_possible -> True, get_model -> UnsatError).  It says so once, loudly; install
    z3 and ``set_backend(mythril_amd.z3_backend.Z3Backend())`` for the real fallback."""

    name = "none"
    _warned = False

    def check(self, terms: Sequence[Term], timeout_ms: int, minimize=(), maximize=()) -> Tuple[str, Optional[Model]]:
        if type(self) is Backend and not Backend._warned:
            Backend._warned = True
            import warnings

            warnings.warn("mythril_amd: no fallback solver set; queries the GPU and the host pre-check "
                          "leave open answer 'unknown' (set_backend(z3_backend.Z3Backend()) where z3 exists)",
                          RuntimeWarning, stacklevel=3)
        return unknown, None

    def check_raw(self, raw_constraints: Sequence, lowered: Sequence[Term], timeout_ms: int, minimize=(),
                  maximize=()) -> Tuple[str, Optional[Model]]:
        """A query with constraints the pre-filter could not lower (given as the caller's
        own objects) -- only a backend that understands them (z3) can answer."""
        return unknown, None


_backend: Backend = Backend()


def set_backend(b: Backend) -> Backend:
    global _backend
    old, _backend = _backend, b
    return old


def get_backend() -> Backend:
    return _backend


# ------------------------------------------------------------ UNSAT cores
class UnsatCores:
    """Constraint sets known to be UNSAT (refuted by mgp_refute, or unsat from the fallback).

    A conjunction only gets stronger as constraints are added (a child's Constraints
    extends its parent's, constraints.py:67-85), so a state whose constraint set contains
    a stored set is UNSAT with no analysis at all ("prefix/core
    cache").  Refuted sets are first shrunk to a core (`shrink`), which then also covers
    other paths that repeat the same contradiction.  Terms are hash-consed, so set
    membership is identity of the interned constraint terms.

    Thread safety: a background shrink (flush(background=True)) works on a snapshot of the
    term arena taken on the caller's thread (the arena's arrays may be reallocated while
    the worker's native calls run without the GIL), and its cores are stored under the
    cache lock only if no reset() happened since the snapshot.
    """

    HALVINGS = 3  # halving rounds before the single deletions (shrink_many)
    HALVE_MIN = 8  # shortest list a halving round tries

    def __init__(self, max_sets: int = 1 << 14):
        self.max_sets = max_sets
        self._lock = threading.RLock()
        self.reset()

    def reset(self) -> None:
        with self._lock:
            self.sets: List[frozenset] = []
            self.index: Dict[Term, List[int]] = {}  # every stored set under ONE of its members
            self.pending: List[list] = []  # refuted lists not yet shrunk (Prefilter.core_batch)
            self.gen = getattr(self, "gen", 0) + 1  # a background shrink of an older generation is dropped
            self._worker = getattr(self, "_worker", None)

    def add_pending(self, lists: Sequence[list]) -> None:
        with self._lock:
            self.pending.extend(lists)

    def flush(self, N, background: bool = False) -> None:
        """Shrink the pending refuted constraint lists to cores (one batched shrink_many)
        and store them; background=True runs it on a worker thread (the native calls
        release the GIL) unless one is still running, which then keeps them pending."""
        if not self.pending:
            return
        if background:
            if self._worker is not None and self._worker.is_alive():
                return
            from .smt import ARENA

            with self._lock:
                pending, self.pending, gen = self.pending, [], self.gen
            snap = _ArenaSnapshot(ARENA)  # on this thread: the worker never reads the live arena

            def work():
                # a small OpenMP team: the foreground calls keep the rest of the cores
                N.lib().mgp_set_thread_omp(max(1, N.lib().mgp_set_thread_omp(0) // 4))
                cores = UnsatCores.shrink_many(N, pending, arena=snap)
                with self._lock:
                    if self.gen == gen:
                        for core in cores:
                            self.add(core)

            self._worker = threading.Thread(target=work, name="mgp-unsat-cores", daemon=True)
            self._worker.start()
            return
        self.join()
        with self._lock:
            pending, self.pending = self.pending, []
        for core in UnsatCores.shrink_many(N, pending):
            self.add(core)

    def join(self) -> None:
        """Wait for a background shrink."""
        if self._worker is not None:
            self._worker.join()
            self._worker = None

    def covered(self, terms: Iterable[Term]) -> bool:
        s = set(terms)
        with self._lock:
            for t in s:
                for k in self.index.get(t, ()):
                    if self.sets[k] <= s:
                        return True
        return False

    def add(self, core: Iterable[Term]) -> None:
        fs = frozenset(core)
        with self._lock:
            if not fs or len(self.sets) >= self.max_sets or self.covered(fs):
                return
            self.sets.append(fs)
            anchor = min(fs, key=lambda t: len(self.index.get(t, ())))
            self.index.setdefault(anchor, []).append(len(self.sets) - 1)

    @staticmethod
    def shrink(N, terms: Sequence[Term], max_terms: int = 32) -> List[Term]:
        """Deletion-based core of one refuted constraint list (see shrink_many)."""
        return UnsatCores.shrink_many(N, [terms], max_terms)[0]

    @staticmethod
    def shrink_many(N, lists: Sequence[Sequence[Term]], max_terms: int = 32, arena=None) -> List[List[Term]]:
        """Cores of many refuted constraint lists in one native call (mgp_build_states once
        per list, then mgp_refute_cores): per list up to HALVINGS rounds keep the first or
        second half when it alone is refuted, then greedy single deletions (lists of at most
        max_terms) drop every constraint the refutation does not need; each trial re-runs
        the analysis on the list's one DAG with only the kept constraints required.  Every
        set returned is one the refuter refuted (a list it does not refute comes back
        whole).  `arena`: the term arena to read (a snapshot for a background shrink;
        default the live one)."""
        from .front import Batch

        lists = [list(dict.fromkeys(t)) for t in lists]
        if not lists:
            return []
        # a batch's refuted states repeat lists (LASER's forks re-add one constraint list on
        # several paths; the 1 024 corpus refutes 213 lists, 63 of them distinct): each
        # distinct list is shrunk once
        first: Dict[tuple, int] = {}
        for t in lists:
            first.setdefault(tuple(t), len(first))
        uniq = [list(k) for k in first]
        B = Batch(uniq, arena=arena) if arena is not None else Batch(uniq)
        try:
            keep, status = N.refute_cores(*B.packed()[:4], np.array([len(t) for t in uniq], np.uint32),
                                          halvings=UnsatCores.HALVINGS, max_single=max_terms)
        finally:
            B.close()
        cores = [[t[i] for i in range(len(t)) if m[i]] if st == 1 else t for t, m, st in zip(uniq, keep, status)]
        return [list(cores[first[tuple(t)]]) for t in lists]


class _ArenaSnapshot:
    """A copy of the term arena's arrays (front.Batch reads these through raw pointers)."""

    def __init__(self, A):
        from array import array

        self.op, self.width, self.args = array("B", A.op), array("I", A.width), array("i", A.args)
        self.p, self.limbs, self.name_hash = array("I", A.p), array("I", A.limbs), array("Q", A.name_hash)


_cores = UnsatCores()


def unsat_cores() -> UnsatCores:
    return _cores


# ------------------------------------------------------------- GPU stage
class Prefilter:
    """Batched GPU witness search over states: one libmgp context per device.

    Answers are a function of each state's content only.  Candidate streams are keyed
    by the state's content key (mgp_build_states MGP_FE_STATE_KEY) and a fixed seed,
    every open state gets the same second round (decision rows within a per-state work
    cap, not a wall-clock budget), so a state is SAT / refuted / undecided the same way
    in any batch, in any order, on any number of host threads or devices.

    devices=[d0, d1, ...]: one context and one host thread per device; a batch is
    hash-sharded over them by state content key (distributed.shard_of) and the results
    are merged in input order (BASELINE config 4)."""

    # second witness round for the states the first round and the pre-check leave open:
    # RETRY_CAND device-generated candidates (a new seed, domain rows) whose first
    # DECIDE_ROWS mixture rows are host decision rows (mgp_decision_rows)
    RETRY_CAND = 256
    DECIDE_ROWS = 4
    DECIDE_MIN_ROWS = 2
    # per-state work cap of the decision rows: variables x DAG nodes x rows (a deterministic
    # count; the largest WalletLibrary state of the corpus needs 1.8 M at four rows)
    DECIDE_MAX_UNITS = 1 << 25
    # decision rows seeded with the parent witness (bit mask of rows; states without a parent
    # witness decide every row unseeded)
    SEED_ROWS = 0x3
    # the states both witness rounds leave open get case splits on their open select
    # conditions (mgp_refute_split) before they go to the fallback: at most SPLIT_REFUTE of
    # them per state (0 = off), nested SPLIT_DEPTH levels.  Depth 2 refutes 11 more of the
    # tuned contracts' ether_thief / etherstore queries than depth 1 (calls.sol 32 -> 21 z3
    # calls) and costs ~7x the split time of the states that reach it
    SPLIT_REFUTE = 8
    SPLIT_DEPTH = 2
    SMALL_BATCH = 16   # at most this many states: the first-round rows overlap the lowering
    # a state of more than this many DAG nodes gets its decision rows in the FIRST round
    # (seed ROWS_FIRST_SEED; the retry round draws new ones): large contract states
    # (WalletLibrary's 600-1 500 nodes) are rarely decided by the mixture alone (148 of the
    # corpus' 344), and their rows cost less than a second GPU round on 12-30 k-instruction
    # programs.  A rule on the state alone (tests/fe_emulate.py restates it)
    ROWS_FIRST_NODES = 600
    ROWS_FIRST_SEED = 0x3C6EF372
    # rows per large state in the first round, from decision row ROWS_FIRST_FROM: row 1 (the
    # greedy select-branch row, parent-seeded) decides all 344 large corpus states alone, as
    # rows 0-1 and rows 0-3 do (row 0 alone: 148 stay open, tests/fe_emulate.py), at half the
    # host time of two rows; the retry round still gets DECIDE_ROWS from row 0
    ROWS_FIRST_FROM = 1
    ROWS_FIRST_ROWS = 1
    # pinned host staging of mgp_check_batch reserved per context (programs + tables of one
    # batch go up through it: WalletLibrary's lowered programs are ~0.45 MB each)
    HOST_STAGING = 256 << 20

    # pipelines > 1: that many contexts per device, each with its own host thread and a share
    # of the OpenMP threads; a batch of at least PIPELINE_MIN states is hash-sharded over them
    # (as over devices), so one shard's GPU rounds run while another's host stages (DAG build,
    # decision rows, lowering, pre-check) run -- the answers are the single pipeline's, every
    # state's being a function of its content.  Off by default: on a
    # 16-thread host the two half teams cost more than the overlap hides (the 1 024-state call
    # 119 -> 221-272 ms, bench frontend.pipelines2)
    PIPELINE_MIN = 128
    MIN_GROUPS = 1
    GROUP_MIN_STATES = 256

    def __init__(self, device: int = 0, n_cand: int = 256, seed: int = 0x4D595448,
                 devices: Optional[Sequence[int]] = None, pipelines: int = 1):
        from . import _native as N

        self._N = N
        self.devices = list(devices) if devices is not None else [device]
        if not self.devices:
            raise ValueError("Prefilter needs at least one device")
        if pipelines < 1:
            raise ValueError("Prefilter needs at least one pipeline per device")
        self.pipelines = pipelines
        self.ctxs = [N.Context(d) for d in self.devices for _ in range(pipelines)]
        self.ctx = self.ctxs[0]
        self.n_cand = n_cand
        self.seed = seed
        self.refute = True  # host UNSAT pre-check (mgp_refute) on every GPU miss
        self.retry_cand = self.RETRY_CAND  # 0 (or <= n_cand) = no second round
        self.decide_rows = self.DECIDE_ROWS
        self.decide_max_units = self.DECIDE_MAX_UNITS
        self.seed_rows = self.SEED_ROWS
        self.split_refute = self.SPLIT_REFUTE
        self.split_depth = self.SPLIT_DEPTH
        self.rows_first_nodes = self.ROWS_FIRST_NODES
        self.cand_bytes = 1 << 30  # candidate memory of one witness round (larger batches are split)
        # a call of >= GROUP_MIN_STATES states runs as at least min_groups groups, so that the
        # pipeline has a next round's host stages to overlap with each GPU round
        self.min_groups = self.MIN_GROUPS
        # the pipeline's pinned host staging and candidate block, sized once here instead of
        # on the first large batch (pinning a few hundred MB of host memory takes tens of ms)
        # (MGP_HOST_STAGING_MB lowers the reserve for several ranks on one device; a reserve
        # that fails leaves the buffers to grow lazily on the first large batch)
        staging = int(os.environ.get("MGP_HOST_STAGING_MB", self.HOST_STAGING >> 20)) << 20
        for c in self.ctxs:
            reserve = getattr(c, "reserve", None)  # (test doubles of the context have none)
            if reserve is not None and staging > 0:
                try:
                    reserve(staging, self.cand_bytes)
                except N.MgpError:
                    pass
        # refuted constraint lists wait in the core cache and are shrunk to cores together
        # once core_batch of them are pending (flush_cores): one batched shrink instead of
        # one per call keeps the deletion trials off the latency of small calls
        self.core_batch = 32
        # shrink on a worker thread (off the caller's latency) only when the caller leaves
        # the host idle between calls: back to back, its OpenMP team competes with the next
        # call's (the bench's first-round pass fell from 3 850 to 2 680 states/s with it on)
        self.core_async = False
        self._tls = threading.local()  # per-thread stage profile (sharded batches)
        self.last_times = None     # mgp_check_batch stage times (ms) of the last batch
        self.last_profile = None   # host + GPU stage split of the last batch (bench frontend_latency)

    def close(self) -> None:
        for c in self.ctxs:
            c.close()

    def check_states(self, states: Sequence[Sequence[Term]],
                     parents: Optional[Sequence[Optional[Dict[str, int]]]] = None) -> List[Tuple[str, Optional[Dict[str, int]]]]:
        """-> per state ('sat', assignment), ('unsat', None) or ('undecided', None).

        'sat' = a GPU witness (a model); 'unsat' = proven by the host pre-check
        (mgp_refute: known bits x intervals, sound); everything else is
        'undecided' and goes to the fallback solver.
        """
        if not states:
            return []
        stats = SolverStatistics()
        t0 = time.time()
        # states that contain a known UNSAT core need no analysis
        hit = [self.refute and _cores.covered(s) for s in states]
        if any(hit):
            stats.core_hits += sum(hit)
            rest = [s for s, h in zip(states, hit) if not h]
            rest_par = None if parents is None else [p for p, h in zip(parents, hit) if not h]
            sub = iter(self.check_states(rest, rest_par) if rest else [])
            return [(unsat, None) if h else next(sub) for h in hit]
        if len(self.ctxs) > 1 and len(states) > 1 and (len(self.devices) > 1 or len(states) >= self.PIPELINE_MIN):
            out, refuted = self._check_sharded(states, parents)
        else:
            out, refuted = self._check_native(self.ctx, states, parents)
        if refuted:
            _cores.add_pending([list(states[i]) for i in refuted])
            if len(_cores.pending) >= self.core_batch:
                tr = time.perf_counter()
                _cores.flush(self._N, background=self.core_async)
                if self.last_profile is not None:
                    self.last_profile["cores_ms"] = 1e3 * (time.perf_counter() - tr)
        stats.gpu_batches += 1
        stats.gpu_queries += len(states)
        stats.gpu_sat += sum(1 for r in out if r[0] == sat)
        stats.refuted += sum(1 for r in out if r[0] == unsat)
        stats.gpu_undecided += sum(1 for r in out if r[0] == "undecided")
        stats.gpu_time += time.time() - t0
        return out

    def shard(self, states: Sequence[Sequence[Term]]) -> np.ndarray:
        """Device index (into self.devices) of every state: hash of its content key."""
        from .distributed import shard_of
        from .front import Batch

        B = Batch(states)
        keys = np.array(B.state_key, dtype=np.uint64)
        B.close()
        return shard_of(keys, len(self.ctxs))

    def _check_sharded(self, states, parents):
        """One host thread per device, each running the whole pipeline on its hash shard
        (the native calls release the GIL); results merged in input order."""
        owner = self.shard(states)
        parts = [np.nonzero(owner == g)[0] for g in range(len(self.ctxs))]
        results: List = [None] * len(self.ctxs)
        profs: List = [None] * len(self.ctxs)
        errors: List = []
        # several pipelines on one host: each thread's OpenMP team gets its share of the cores
        # (one full team per thread oversubscribes them)
        lib = self._N.lib()
        share = max(1, lib.mgp_set_thread_omp(0) * len(self.devices) // len(self.ctxs)) \
            if self.pipelines > 1 else 0

        def work(g):
            idx = parts[g]
            try:
                if share:
                    lib.mgp_set_thread_omp(share)
                results[g] = self._check_native(self.ctxs[g], [states[i] for i in idx],
                                                None if parents is None else [parents[i] for i in idx])
                profs[g] = getattr(self._tls, "profile", None)
            except BaseException as e:  # re-raised on the caller's thread
                errors.append(e)

        threads = [threading.Thread(target=work, args=(g,), name=f"mgp-ctx{g}")
                   for g in range(len(self.ctxs)) if len(parts[g])]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            raise errors[0]
        self.last_profile = dict(_sum_profiles([p for p in profs if p]), shards=sum(1 for p in parts if len(p)))
        out: List = [None] * len(states)
        refuted: List[int] = []
        for g, idx in enumerate(parts):
            if not len(idx):
                continue
            sub, sub_ref = results[g]
            for k, i in enumerate(idx):
                out[int(i)] = sub[k]
            refuted.extend(int(idx[k]) for k in sub_ref)
        return out, sorted(refuted)

    def _check_native(self, ctx, states, parents):
        """One native front-end batch (mgp_build_states) through the witness rounds on `ctx`
        (GPU witnesses; host refutations) and the split refuter for what is left.  ->
        (results, indices of the refuted states).  A batch whose candidate block would pass
        `cand_bytes` runs as groups of similar variable counts, cut out of the one build
        (Batch.select).  The rounds are pipelined (mgp_check_submit / mgp_check_finish, two in
        flight): a round's host stages -- decision rows, lowering, pre-check, staging -- run
        while the previous round is on the GPU, and a group's second round is queued when its
        first round finishes.  The answers do not change: candidates are keyed by content."""
        from .front import Batch

        tb = time.perf_counter()
        B = Batch(states)
        n = len(states)
        prof = {"states": n, "build_ms": 1e3 * (time.perf_counter() - tb)}
        nv = np.diff(B.var_off).astype(np.int64)
        n_vars = max(1, int(nv.max()) if len(nv) else 1)
        parts = self.min_groups if n >= self.GROUP_MIN_STATES else 1
        groups = self._groups(nv, self.n_cand, -(-n // parts) if parts > 1 else 0) \
            if n > 1 and (parts > 1 or n * self.n_cand * n_vars * 32 > self.cand_bytes) else [list(range(n))]
        first = np.full(n, -1, np.int32)
        proven = np.zeros(n, np.int8)
        witnesses: Dict[int, object] = {}
        jobs = collections.deque(_Round("first", grp, B if len(groups) == 1 else B.select(grp), len(groups) > 1,
                                        None if parents is None else [parents[i] for i in grp])
                                 for grp in groups)
        inflight: collections.deque = collections.deque()
        try:
            while jobs or inflight:
                if jobs and len(inflight) < 2:
                    job = jobs.popleft()
                    self._submit_round(ctx, job, prof)
                    inflight.append(job)
                    continue
                job = inflight.popleft()
                jobs.extend(self._finish_round(job, first, proven, witnesses, prof))
        finally:
            for job in inflight:  # an error: drain what is in flight before the batches go
                try:
                    job.pending.finish()
                except Exception:
                    pass
            for job in list(jobs) + list(inflight):
                job.close()
        left = [i for i in range(n) if first[i] < 0 and proven[i] != 1]
        if left and self.refute and self.split_refute > 0:
            ts = time.perf_counter()
            LB = B.select(left)
            rs = self._N.refute_split(*LB.packed()[:4], max_splits=self.split_refute, depth=self.split_depth)
            LB.close()
            for k, i in enumerate(left):
                if rs[k] == 1:
                    proven[i] = 1
            prof["split_ms"] = 1e3 * (time.perf_counter() - ts)
            prof["split_refuted"] = int((rs == 1).sum())
        tr = time.perf_counter()
        out: List[Tuple[str, Optional[object]]] = []
        refuted = []
        for i in range(n):
            if first[i] >= 0:
                if proven[i] == 1:  # a witness and an UNSAT proof cannot both hold
                    raise RuntimeError(f"mgp_refute refuted state {i} that has a GPU witness (soundness bug)")
                out.append((sat, witnesses[i]))
            elif proven[i] == 1:
                out.append((unsat, None))
                refuted.append(i)
            else:
                out.append(("undecided", None))
        B.close()
        prof["results_ms"] = 1e3 * (time.perf_counter() - tr)
        prof["cores_ms"] = 0.0
        if len(groups) > 1:
            prof["groups"] = len(groups)
        self.last_profile = prof
        self._tls.profile = prof
        return out, refuted

    _STAGES = ("lower_ms", "refute_ms", "upload_launch_ms", "gpu_wait_ms", "copy_back_ms")

    def _submit_round(self, ctx, job: "_Round", prof: dict) -> None:
        """Host half of a witness round: its explicit rows (the first round's decision rows of
        large states; the second round's decision rows), then mgp_check_submit."""
        td = time.perf_counter()
        if job.kind == "first":
            xrows = self._first_round_rows(job.batch, job.parents, ctx)
            if xrows is not None:
                prof["rows_first_ms"] = prof.get("rows_first_ms", 0.0) + 1e3 * (time.perf_counter() - td)
            job.pending = job.batch.submit(ctx, self.n_cand, self.seed, job.parents, refute=self.refute, xrows=xrows)
            for name, t in zip(self._STAGES[:3], job.pending.times[:3]):
                prof[name] = prof.get(name, 0.0) + float(t)
        else:
            rows, mask = self._decision_rows(self._rows_args(job.batch, job.parents), self._seed2())
            prof["decide_host_ms"] = prof.get("decide_host_ms", 0.0) + 1e3 * (time.perf_counter() - td)
            # (the second round's candidates carry no parent row: its decision rows are seeded
            # with the parents' values instead, mgp_decision_rows_seeded)
            job.pending = job.batch.submit(ctx, self._n2(), self._seed2(), refute=self.refute, xrows=(rows, mask))
            r2 = prof.setdefault("round2_stages", {})
            for name, t in zip(("lower", "refute", "upload_launch"), job.pending.times[:3]):
                r2[name] = r2.get(name, 0.0) + float(t)
        prof["pipelined_rounds"] = prof.get("pipelined_rounds", 0) + 1

    def _finish_round(self, job: "_Round", first, proven, witnesses, prof) -> List["_Round"]:
        """Collect a round's answers into first / proven / witnesses; a first round returns the
        second round(s) for its open states (none when retry_cand is 0)."""
        from .front import FE_SAT_UNSAFE

        f, w, ref, times = job.pending.finish()
        if job.kind == "first":
            for name, t in zip(self._STAGES[3:], times[3:5]):
                prof[name] = prof.get(name, 0.0) + float(t)
        else:
            r2 = prof.setdefault("round2_stages", {})
            for name, t in zip(("gpu_wait", "copy_back"), times[3:5]):
                r2[name] = r2.get(name, 0.0) + float(t)
        tr = time.perf_counter()
        unsafe = (job.batch.flags & FE_SAT_UNSAFE) != 0
        G = job.idx
        follow: List[_Round] = []
        if job.kind == "first":
            f = f.copy()
            f[unsafe & (f >= 0)] = -1  # no GPU SAT answer for those (mgp_front.cpp)
            for k, i in enumerate(G):
                first[i] = f[k]
                if ref[k] == 1:
                    proven[i] = 1
            sat_k = [k for k in range(len(G)) if f[k] >= 0]
            for k, wt in zip(sat_k, job.batch.witnesses(sat_k, w)):
                witnesses[G[k]] = wt
            retry = [k for k in range(len(G)) if f[k] == -1 and ref[k] != 1]
            prof["retry_states"] = prof.get("retry_states", 0) + len(retry)
            if retry and self.retry_cand > 0:
                SolverStatistics().gpu_retry += len(retry)
                follow = self._retry_rounds(job, retry)
        else:
            found = 0
            for k, i in enumerate(G):
                if f[k] >= 0 and not unsafe[k]:
                    first[i] = f[k]
                    witnesses[i] = job.batch.witness(k, w[k])
                    found += 1
            prof["retry_sat"] = prof.get("retry_sat", 0) + found
        job.close()
        prof["collect_ms"] = prof.get("collect_ms", 0.0) + 1e3 * (time.perf_counter() - tr)
        return follow

    def _n2(self) -> int:
        return max(64, self.retry_cand // 64 * 64)

    def _seed2(self) -> int:
        return (self.seed + 0x7F4A7C15) & (2 ** 64 - 1)

    def _retry_rounds(self, job: "_Round", retry: List[int]) -> List["_Round"]:
        """The second witness round of a first round's open states (local indices `retry`):
        host decision rows (mgp_decision_rows, each variable fixed in turn and the analysis
        re-propagated) placed in the first mixture rows of a device-generated round with a
        new seed, one round per candidate-memory group.  A state with a parent witness gets
        SEED_ROWS of its rows seeded with the parent's values (mgp_decision_rows_seeded):
        the draws then only decide what the child's new constraint brought in."""
        n2 = self._n2()
        SB = job.batch.select(retry)
        nv = np.diff(SB.var_off).astype(np.int64)
        groups = self._groups(nv, n2) if len(retry) * n2 * max(1, int(nv.max())) * 32 > self.cand_bytes \
            else [list(range(len(retry)))]
        par = job.parents
        out = []
        for grp in groups:
            GB = SB if len(groups) == 1 else SB.select(grp)
            out.append(_Round("retry", [job.idx[retry[k]] for k in grp], GB, True,
                              None if par is None else [par[retry[k]] for k in grp]))
        if len(groups) > 1:
            SB.close()
        return out

    def flush_cores(self) -> None:
        """Shrink the pending refuted constraint lists to cores and store them (waits for
        a background shrink first)."""
        _cores.flush(self._N)

    def _groups(self, nv: np.ndarray, n_cand: int, max_len: int = 0) -> List[List[int]]:
        """Indices grouped by variable count so that each group's candidate block fits cand_bytes
        (and, max_len > 0, each group holds at most max_len states)."""
        order = sorted(range(len(nv)), key=lambda i: (int(nv[i]), i))
        groups: List[List[int]] = []
        grp: List[int] = []
        for i in order:
            w = max(1, int(nv[i]))
            if grp and ((len(grp) + 1) * n_cand * w * 32 > self.cand_bytes or 0 < max_len <= len(grp)):
                groups.append(grp)
                grp = []
            grp.append(i)
        if grp:
            groups.append(grp)
        return groups

    def rows_per_state(self, B) -> np.ndarray:
        """Decision rows each state of batch B gets: DECIDE_ROWS while variables x nodes x rows
        stays within decide_max_units, else DECIDE_MIN_ROWS if that fits, else none -- a rule
        on the state alone, so its answer does not depend on the rest of the batch."""
        units = np.diff(B.var_off).astype(np.float64) * np.diff(B.node_off).astype(np.float64)
        rows = np.where(units * self.decide_rows <= self.decide_max_units, self.decide_rows,
                        np.where(units * self.DECIDE_MIN_ROWS <= self.decide_max_units, self.DECIDE_MIN_ROWS, 0))
        return rows.astype(np.uint8)

    def _rows_args(self, GB, parents):
        """The inputs of mgp_decision_rows for batch GB (parent-seeded rows when a parent
        witness is given)."""
        from .front import seed_arrays

        gv = max(1, GB.n_vars())
        seeds = seed_arrays(GB, parents) if parents is not None and any(p is not None for p in parents) else None
        if seeds is not None and seeds[0].shape[1] != gv:
            seeds = None
        return list(GB.packed(decide=True)), gv, self.rows_per_state(GB), GB.state_key, seeds

    def _decision_rows(self, args, seed2, n_rows=None, row0=0):
        packed, gv, rps, keys, seeds = args
        n_rows = self.decide_rows if n_rows is None else n_rows
        rows, mask, _ = self._N.decision_rows(*packed, gv, seed2, n_rows, np.minimum(rps, n_rows).astype(np.uint8),
                                              state_keys=keys, seeds=seeds, seed_rows=self.seed_rows, row0=row0)
        return rows, mask

    def _first_round_rows(self, B, parents, ctx):
        """Decision rows of B's states above rows_first_nodes nodes (None if there are none),
        for the first round's mixture rows."""
        if self.decide_rows <= 0 or self.rows_first_nodes <= 0 or B.n_states == 0:
            return None
        big = np.diff(B.node_off) > self.rows_first_nodes
        if not big.any():
            return None
        packed, gv, rps, keys, seeds = self._rows_args(B, parents)
        rps = np.where(big, rps, 0).astype(np.uint8)
        seed1 = (self.seed + self.ROWS_FIRST_SEED) & (2 ** 64 - 1)
        out: dict = {}

        row0 = min(self.ROWS_FIRST_FROM, max(0, self.decide_rows - 1))

        def work():
            try:
                out["rows"] = self._decision_rows((packed, gv, rps, keys, seeds), seed1,
                                                  n_rows=min(self.decide_rows - row0, self.ROWS_FIRST_ROWS), row0=row0)
            except BaseException as e:
                out["error"] = e

        if B.n_states > self.SMALL_BATCH:
            # a large batch keeps every host thread busy in either stage: run them in turn
            # (two OpenMP teams on the same cores slowed the 128-state call 36 -> 75 ms; on half
            # the threads each they tied with running in turn, profiles/fe_overlap_ab_r4.json)
            return work() or self._rows_or_raise(out)
        # a small batch: the rows on a host thread while this one lowers the batch's programs
        # into the program cache (mgp_program_cache_warm); mgp_check_batch then finds them
        t = threading.Thread(target=work, name="mgp-first-round-rows", daemon=True)
        t.start()
        try:
            self._N.program_cache_warm(B._h)
        finally:
            t.join()
        return self._rows_or_raise(out)

    @staticmethod
    def _rows_or_raise(out: dict):
        if "error" in out:
            raise out["error"]
        return out["rows"]


class _Round:
    """One witness round of a Prefilter batch: the global indices of its states, their
    batch (owned: closed once the round is collected), their parent witnesses and, once
    submitted, the pending GPU round."""

    def __init__(self, kind: str, idx: List[int], batch, owned: bool, parents):
        self.kind, self.idx, self.batch, self.owned, self.parents = kind, idx, batch, owned, parents
        self.pending = None

    def close(self) -> None:
        if self.owned and self.batch is not None:
            self.batch.close()
        self.batch = None


def _sum_profiles(profs: List[dict]) -> dict:
    """Stage profile of a batch run as sub-batches: numeric stages summed (nested dicts
    too), flags OR-ed, and the sub-batch count recorded."""
    out: dict = {"groups": len(profs)}
    for p in profs:
        for k, v in p.items():
            if isinstance(v, dict):
                out[k] = _sum_profiles_into(out.get(k, {}), v)
            elif isinstance(v, bool):
                out[k] = bool(out.get(k, False)) or v
            elif isinstance(v, (int, float)):
                out[k] = out.get(k, 0) + v
    return out


def _sum_profiles_into(acc: dict, p: dict) -> dict:
    for k, v in p.items():
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            acc[k] = acc.get(k, 0) + v
    return acc


_prefilter: Optional[Prefilter] = None
_enabled = True


def prefilter() -> Optional[Prefilter]:
    """The process-wide GPU stage (None when disabled)."""
    global _prefilter
    if not _enabled:
        return None
    if _prefilter is None:
        _prefilter = Prefilter()
    return _prefilter


def enable_gpu(flag: bool = True) -> None:
    global _enabled
    _enabled = flag


class NotLowerable(Exception):
    """A constraint outside the pre-filter's node set (z3_lower.Unsupported): the query
    goes to the fallback solver unchanged."""


def _terms(constraints: Iterable) -> List[Term]:
    """Constraints as pre-filter terms: laser.smt mirror expressions (.raw Term), the
    reference's own laser.smt wrappers or bare z3 expressions (lowered by
    mythril_amd.z3_lower), Python bools."""
    from . import z3_lower

    out = []
    for c in constraints:
        if isinstance(c, bool):
            out.append(bconst(c))
        elif isinstance(c, Expression):
            out.append(c.raw)
        elif isinstance(c, Term):
            out.append(c)
        else:
            raw = getattr(c, "raw", c)
            if not z3_lower.is_z3_expr(raw):
                raise NotLowerable(f"unknown constraint type {type(c)!r}")
            t = z3_lower.to_terms([raw])
            if t is None:
                raise NotLowerable("z3 construct outside the node set")
            out.extend(t)
    return out


def _recheck(terms: Sequence[Term], witness) -> bool:
    """A GPU witness is trusted unless the fallback backend can re-check it and rejects it
    (Z3Backend.recheck: z3's evaluator on the original constraints)."""
    rc = getattr(get_backend(), "recheck", None)
    if rc is None:
        return True
    ok = rc(terms, witness)
    stats = SolverStatistics()
    stats.rechecks += ok is not None
    if ok is False:
        stats.recheck_rejects += 1
        return False
    return True


def _confirm_refutation(terms: Sequence[Term]) -> Tuple[bool, Optional[Model]]:
    """-> (refutation stands, model).  A backend that audits refutations
    (Z3Backend(recheck_refutations=f)) answers for a sampled fraction of them; a `sat`
    from it overrides the pre-check and is counted as a disagreement."""
    rc = getattr(get_backend(), "recheck_refutation", None)
    if rc is None:
        return True, None
    r = rc(terms)
    if r is None:
        return True, None
    stats = SolverStatistics()
    stats.refute_rechecks += 1
    if r[0] == sat:
        stats.refute_disagreements += 1
        _cores.reset()  # cores shrunk by the same pre-check are suspect too
        import warnings

        warnings.warn("mythril_amd: the fallback solver found a model for a state the host pre-check "
                      "refuted (mgp_refute soundness bug); using the fallback's answer", RuntimeWarning, stacklevel=3)
        return False, r[1]
    return True, None


# ------------------------------------------------------------ Solver API
class BaseSolver:
    def __init__(self):
        self.constraints: List[Term] = []
        self.raw_constraints: List = []  # constraints the pre-filter cannot lower
        self.lowerable = True
        self.timeout = 10000
        self._model: Optional[Model] = None

    def set_timeout(self, timeout: int) -> None:
        self.timeout = timeout

    def add(self, *constraints) -> None:
        flat = []
        for c in constraints:
            flat.extend(c if isinstance(c, (list, tuple)) else [c])
        try:
            self.constraints.extend(_terms(flat))
        except NotLowerable:
            self.lowerable = False
            SolverStatistics().not_lowerable += 1
            self.raw_constraints.extend(flat)

    append = add

    def model(self) -> Model:
        return self._model


class Solver(BaseSolver):
    """GPU witness first, then the fallback solver (counted in SolverStatistics.query_count)."""

    def check(self, *args) -> str:
        pf = prefilter() if self.lowerable else None
        if pf is not None:
            res, assign = pf.check_states([self.constraints])[0]
            if res == sat and _recheck(self.constraints, assign):
                self._model = Model([assign])
                return sat
            if res == unsat:
                stands, model = _confirm_refutation(self.constraints)
                self._model = model
                return unsat if stands else sat
        return self._fallback()

    @stat_smt_query
    def _fallback(self) -> str:
        if not self.lowerable:
            r, m = get_backend().check_raw(self.raw_constraints, self.constraints, self.timeout)
            self._model = m
            return r
        r, m = get_backend().check(self.constraints, self.timeout)
        self._model = m
        if r == unsat:
            _cores.add(self.constraints)
        return r

    def reset(self) -> None:
        self.constraints = []


class Optimize(BaseSolver):
    """Optimize: minimised model values come from the fallback solver (they are reported
    verbatim); a state the pre-check refutes is unsat without it."""

    def __init__(self):
        super().__init__()
        self._min: List[Term] = []
        self._max: List[Term] = []

    def minimize(self, e) -> None:
        self._min.append(e.raw if isinstance(e, Expression) else e)

    def maximize(self, e) -> None:
        self._max.append(e.raw if isinstance(e, Expression) else e)

    def check(self, *args) -> str:
        pf = prefilter() if self.lowerable else None
        if pf is not None:
            res, assign = pf.check_states([self.constraints])[0]
            if res == unsat:  # no model exists, whatever the objectives
                stands, _ = _confirm_refutation(self.constraints)
                if stands:
                    self._model = None
                    return unsat
                return self._fallback()
            if res == sat and not self._min and not self._max and _recheck(self.constraints, assign):
                self._model = Model([assign])
                return sat
        return self._fallback()

    @stat_smt_query
    def _fallback(self) -> str:
        if not self.lowerable:
            r, m = get_backend().check_raw(self.raw_constraints, self.constraints, self.timeout, tuple(self._min),
                                           tuple(self._max))
            self._model = m
            return r
        r, m = get_backend().check(self.constraints, self.timeout, tuple(self._min), tuple(self._max))
        self._model = m
        if r == unsat:
            _cores.add(self.constraints)
        return r


def _get_expr_variables(t: Term) -> List[str]:
    """independence_solver.py:10-22 over terms: the leaves of the expression that are not
    bit-vector numerals, by name.  z3's leaves are constants (BitVec / Bool symbols, the
    array constant under a Select, and the Bool literals True / False); a UF application's
    function symbol is no child, so it is no leaf.  Here an array select is a UFAPP of the
    function ``array:<name>`` (smt.Array), whose leaf is the array itself."""
    out: List[str] = []
    seen: Set[int] = set()
    stack = [t]
    while stack:
        u = stack.pop()
        if id(u) in seen:
            continue
        seen.add(id(u))
        if u.op == ir.VAR:
            out.append(str(u.params[0]))
        elif u.op in (ir.TRUE, ir.FALSE):
            out.append("True" if u.op == ir.TRUE else "False")
        elif u.op == ir.UFAPP and str(u.params[1]).startswith("array:"):
            out.append(str(u.params[1])[len("array:"):])
        stack.extend(u.args)
    return out


class DependenceBucket:
    """independence_solver.py:25-35: conditions that share variables."""

    def __init__(self, variables=None, conditions=None):
        self.variables: List[str] = variables or []
        self.conditions: List[Term] = conditions or []


class DependenceMap:
    """independence_solver.py:38-83: buckets of conditions, merged when they share a variable."""

    def __init__(self):
        self.buckets: List[DependenceBucket] = []
        self.variable_map: Dict[str, DependenceBucket] = {}

    def add_condition(self, condition: Term) -> None:
        variables = list(dict.fromkeys(_get_expr_variables(condition)))
        relevant = [b for b in self.buckets if any(self.variable_map.get(v) is b for v in variables)]
        new_bucket = DependenceBucket(variables, [condition])
        self.buckets.append(new_bucket)
        if relevant:
            relevant.append(new_bucket)
            new_bucket = self._merge_buckets(relevant)
        for v in new_bucket.variables:
            self.variable_map[v] = new_bucket

    def _merge_buckets(self, bucket_list: List[DependenceBucket]) -> DependenceBucket:
        variables: List[str] = []
        conditions: List[Term] = []
        for b in bucket_list:
            self.buckets.remove(b)
            variables += b.variables
            conditions += b.conditions
        merged = DependenceBucket(variables, conditions)
        self.buckets.append(merged)
        return merged


class IndependenceSolver(BaseSolver):
    """independence_solver.py:86-153: the constraints split into buckets that share no
    variable, each checked on its own, the first non-sat bucket's answer returned.  GPU
    first: all buckets go to the pre-filter as ONE batch (a bucket is a state); a bucket
    with a witness is sat, a refuted one unsat; the buckets left open go to the fallback
    in bucket order, inside one counted check (the reference decorates check() itself
    with stat_smt_query, so one IndependenceSolver.check is at most one query)."""

    def __init__(self):
        super().__init__()
        self.models: List[Dict[str, int]] = []

    def check(self, *args) -> str:
        if not self.lowerable:
            return self._fallback_raw()
        dm = DependenceMap()
        for c in self.constraints:
            dm.add_condition(c)
        buckets = dm.buckets
        pf = prefilter()
        answers = pf.check_states([b.conditions for b in buckets]) if pf is not None and buckets else \
            [("undecided", None)] * len(buckets)
        self.models = []
        open_from = None
        for k, (b, (res, assign)) in enumerate(zip(buckets, answers)):
            if res == sat and _recheck(b.conditions, assign):
                self.models.append(assign)
                continue
            if res == unsat and _confirm_refutation(b.conditions)[0]:
                self._model = None
                return unsat
            open_from = k
            break
        if open_from is not None:
            return self._fallback_buckets(buckets[open_from:], answers[open_from:])
        self._model = Model(self.models)
        return sat

    @stat_smt_query
    def _fallback_buckets(self, buckets, answers) -> str:
        for b, (res, assign) in zip(buckets, answers):
            if res == sat and _recheck(b.conditions, assign):
                self.models.append(assign)
                continue
            if res == unsat and _confirm_refutation(b.conditions)[0]:
                self._model = None
                return unsat
            r, m = get_backend().check(b.conditions, self.timeout)
            if r != sat:
                if r == unsat:
                    _cores.add(b.conditions)
                self._model = None
                return r
            self.models.extend(m.assignments if m is not None else [])
        self._model = Model(self.models)
        return sat

    @stat_smt_query
    def _fallback_raw(self) -> str:
        r, m = get_backend().check_raw(self.raw_constraints, self.constraints, self.timeout)
        self._model = m
        return r

    def reset(self) -> None:
        self.constraints = []

    def pop(self, num) -> None:
        self.constraints.pop(num)


class _Clock:
    """time_handler (laser/ethereum/time_handler.py:5-18) stand-in: ms left of the execution budget."""

    def __init__(self):
        self.deadline: Optional[float] = None

    def start_execution(self, seconds: float) -> None:
        self.deadline = time.time() + seconds

    def time_remaining(self) -> float:
        return 1e12 if self.deadline is None else (self.deadline - time.time()) * 1000.0


time_handler = _Clock()
solver_timeout_ms = 10000  # analysis_args.solver_timeout default (analysis_args.py:11)


@lru_cache(maxsize=2 ** 23)
def get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True) -> Model:
    """analysis/solver.py:27-61 with a GPU witness stage for SAT-only queries."""
    timeout = solver_timeout_ms
    if enforce_execution_time:
        timeout = min(timeout, time_handler.time_remaining() - 500)
        if timeout <= 0:
            raise UnsatError
    for c in constraints:
        if type(c) == bool and not c:
            raise UnsatError
    constraints = [c for c in constraints if type(c) != bool]
    s = Optimize()
    s.set_timeout(int(timeout))
    for c in constraints:
        s.add(c)
    for e in minimize:
        s.minimize(e)
    for e in maximize:
        s.maximize(e)
    result = s.check()
    if result == sat:
        return s.model()
    raise UnsatError


class Constraints(list):
    """constraints.py:10-126 with a GPU-first is_possible and witness inheritance."""

    def __init__(self, constraint_list: Optional[List] = None, is_possible: Optional[bool] = None,
                 witness: Optional[Dict[str, int]] = None):
        constraint_list = self._get_smt_bool_list(constraint_list or [])
        super().__init__(constraint_list)
        self._default_timeout = 100
        self._is_possible = is_possible
        self.witness = witness  # last satisfying assignment seen (parent's for a fresh child)

    @property
    def is_possible(self) -> bool:
        if self._is_possible is not None:
            return self._is_possible
        batch_is_possible([self])
        return bool(self._is_possible)

    def append(self, constraint) -> None:
        super().append(constraint if isinstance(constraint, Bool) else Bool(bconst(bool(constraint))))
        self._is_possible = None

    def pop(self, index: int = -1) -> None:
        raise NotImplementedError

    @property
    def as_list(self) -> List[Bool]:
        return self[:]

    def __copy__(self) -> "Constraints":
        return Constraints(super().copy(), is_possible=self._is_possible, witness=self.witness)

    def copy(self) -> "Constraints":
        return self.__copy__()

    def __deepcopy__(self, memodict=None) -> "Constraints":
        return self.__copy__()

    def __add__(self, constraints) -> "Constraints":
        lst = super().__add__(self._get_smt_bool_list(constraints))
        return Constraints(constraint_list=lst, is_possible=None, witness=self.witness)

    def __iadd__(self, constraints) -> "Constraints":
        super().__iadd__(self._get_smt_bool_list(constraints))
        self._is_possible = None
        return self

    @staticmethod
    def _get_smt_bool_list(constraints) -> List[Bool]:
        return [c if isinstance(c, Bool) else Bool(bconst(bool(c))) for c in constraints]

    def __hash__(self):
        return tuple(self[:]).__hash__()


def batch_is_possible(items: Sequence[Constraints]) -> List[bool]:
    """The prune filter of LaserEVM.exec (svm.py:251-255) over a whole worklist.

    One GPU batch for every uncached entry; an entry with a witness is possible,
    an entry the host pre-check proves UNSAT is not, and every other entry goes
    through the reference's single-query path (100 ms fallback check, unknown ->
    possible, constraints.py:42-51).
    """
    todo = [c for c in items if getattr(c, "_is_possible", None) is None]
    pf = prefilter()
    results: List[Tuple[str, Optional[Dict[str, int]]]] = [("undecided", None)] * len(todo)
    lowered: List[Optional[List[Term]]] = []
    for c in todo:
        try:
            lowered.append(_terms(c))
        except NotLowerable:  # counted by the fallback Solver.add below
            lowered.append(None)
    idx = [k for k, t in enumerate(lowered) if t is not None]
    if pf is not None and idx:
        sub = pf.check_states([lowered[k] for k in idx], parents=[getattr(todo[k], "witness", None) for k in idx])
        for k, r in zip(idx, sub):
            results[k] = r
    for c, t, (res, assign) in zip(todo, lowered, results):
        if res == sat and _recheck(t, assign):
            c._is_possible = True
            c.witness = assign
            continue
        if res == unsat:
            stands, model = _confirm_refutation(t)
            c._is_possible = not stands
            continue
        s = Solver()
        s.set_timeout(c._default_timeout)
        s.add(*c)
        r = s._fallback()
        c._is_possible = r != unsat
    return [bool(c._is_possible) for c in items]
