"""A restatement of how LASER asks its solver questions (test and benchmark infrastructure).

No solc / z3 / mythril exists here or on the GPU box, so `myth analyze` cannot run.  This
module restates, over the laser.smt mirror (mythril_amd.smt), the part of a `myth analyze
<contract> -t N` run that produces solver queries, so that the pre-filter can be measured
on every contract of solidity_examples/ with each query tagged by how the reference asks it:

* ``prune``  -- Constraints.is_possible at the prune filter (svm.py:251-255), one per
  successor whose constraint list changed: both successors of a symbolic JUMPI
  (instructions.py:1556-1610), the first step of every transaction (the setup constraints of
  transaction/symbolic.py:165-167 and transaction_models.py:129-133 reset the cache), every
  SHA3 (instructions.py:1037) and every ether transfer (instructions.py:66-87);
* ``model``  -- a SAT-only get_model (analysis/solver.py:27-61): MutationPruner
  (mutation_pruner.py:55-83), the integer module's ostate check (integer.py:288-297),
  ether_thief (ether_thief.py:76-80), state_change_external_calls (120-145, 189-198);
* ``dep``    -- DependencyPruner's `get_model((loc == dep,))` (below), a SAT-only get_model
  on one equality of two storage locations, no path constraints;
* ``txseq``  -- get_transaction_sequence (analysis/solver.py:88-136): get_model with the
  minimisation constraints (242-282) and minimize objectives, so a SAT answer is ONE z3
  Optimize call whatever the GPU finds (its model values go into the report); an UNSAT one
  is zero calls when the host pre-check refutes it.

What is restated (by reading the reference and the contracts; no reference run pins it):
the solc dispatcher (calldatasize < 4, one selector compare per function, callvalue == 0
for non-payable functions), `require` / `if` / `assert` as JUMPIs, storage through one
Store chain per run (read-over-write), mappings through the keccak manager, ether
transfers, the modules' hook points and caches (DetectionModule.cache by address; the
integer module's ostate sets; potential issues checked at transaction end,
potential_issues.py:75-108), and MutationPruner's filter between transactions.
What is approximated or left out, and why:

* DependencyPruner (dependency_pruner.py, loaded by default, analysis/symbolic.py:139-140) is
  restated over the JUMPI successors as its basic blocks: from the second message call on, a
  successor whose block this path saw before runs only if some storage location written in
  the previous transaction can equal a location read on paths through the block -- one
  ``dep`` query `get_model((loc == dep,))` per pair (dependency_pruner.py:134-187, lru-cached
  like every get_model) -- and a pruned successor asks nothing more (PluginSkipState drops it
  before the prune filter, svm.py:614-631);
* compiler-internal arithmetic (memory pointers, ABI offsets) carries no integer-module
  annotation here; only source-level ADD / SUB / MUL / EXP do;
* feasibility of every branch is decided by reading (`t=` / `f=` at each site), as the
  reference would learn it from z3; each query carries that expectation ("sat" / "unsat",
  or None where reading does not decide it), and the bench reports any contradiction;
* open states carried into the next transaction are capped per run (`max_open`), in
  generation order, so `-t 3` stays a few thousand queries.

The queries of one run are `Analysis.queries`: (kind, label, terms, expected, parent)
tuples; `parent` links a query to the prune query that established the asking state, so a
consumer can hand the parent's witness to the pre-filter as the plugin does.
"""
from __future__ import annotations

import copy
import itertools
import json
import os
from typing import Dict, List, Optional, Sequence, Tuple

from mythril_amd.smt import (And, Array, BVAddNoOverflow, BVMulNoOverflow, BVSubNoUnderflow, Concat, Extract, If,
                             K, Not, Or, UDiv, UGE, UGT, ULE, ULT, is_false, is_true, symbol_factory)

BVV, BVS = symbol_factory.BitVecVal, symbol_factory.BitVecSym
CREATOR = 0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE
ATTACKER = 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF
SOMEGUY = 0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA
ACTORS = (CREATOR, ATTACKER, SOMEGUY)                     # transaction/symbolic.py:22-67
CONTRACT_ADDRESS = 0x0901D12EBE1B195E5AA8748E62BD7734AE19B51F  # the analysed account (LASER's default)
ETHER = 10 ** 18
GSTIPEND = 2300


def _bv(x, w: int = 256):
    return BVV(x, w) if isinstance(x, int) else x


def _exp(ok: Optional[bool]) -> Optional[str]:
    """feasibility by reading -> the query's expectation (None: reading does not decide it)."""
    return None if ok is None else ("sat" if ok else "unsat")


class Tx:
    """One symbolic transaction: calldata, sender, value (transaction/symbolic.py:70-191)."""

    def __init__(self, tid: int, creation: bool = False):
        self.tid = tid
        self.creation = creation
        self.calldata = Array(f"{tid}_calldata", 256, 8)
        self.size = BVS(f"{tid}_calldatasize", 256)
        self.sender = BVV(CREATOR, 256) if creation else BVS(f"sender_{tid}", 256)
        self.value = BVS(f"call_value{tid}", 256)

    def env(self, name: str):
        """GlobalState.new_bitvec (instructions.py: timestamp, coinbase, gas, ...): '<tid>_<name>'."""
        return BVS(f"{self.tid}_{name}", 256)

    def byte(self, idx):
        """calldata.py:219-232: If(idx < calldatasize, calldata[idx], 0) -- a SIGNED `<`."""
        i = _bv(idx)
        return If(i < self.size, self.calldata[i], BVV(0, 8))

    def word(self, off):
        base = _bv(off)
        return Concat(*[self.byte(base + i) for i in range(32)])

    def arg(self, k: int):
        return self.word(4 + 32 * k)

    def address_arg(self, k: int):
        """an `address` parameter: the low 160 bits of its word (solc 0.5 masks, no check)."""
        return Concat(BVV(0, 96), Extract(159, 0, self.arg(k)))


class DepAnn:
    """plugin_annotations.py:17-49 DependencyAnnotation: the blocks on this path, the storage
    locations it read (this transaction) and wrote (per iteration), whether it made a call."""

    def __init__(self):
        self.loaded: list = []
        self.written: Dict[int, list] = {}
        self.has_call = False
        self.path: list = [0]
        self.seen: set = set()

    def copy(self) -> "DepAnn":
        d = DepAnn.__new__(DepAnn)
        d.loaded = list(self.loaded)
        d.written = {k: list(v) for k, v in self.written.items()}
        d.has_call = self.has_call
        d.path = list(self.path)
        d.seen = set(self.seen)
        return d


def _same_term(a, b) -> bool:
    return a.raw is b.raw


def _add_loc(lst: list, loc) -> None:
    if not any(_same_term(loc, x) for x in lst):
        lst.append(loc)


class World:
    """The world state a path carries: the contract's storage (one Store chain) and the
    balances (world_state.py:33); `starting` are the balances before any transaction."""

    def __init__(self):
        # a created contract's storage is concrete: K(0) (transaction_models.py:205, account.py:26)
        self.storage = K(256, 256, 0)
        self.balances = Array("balance", 256, 256)
        self.starting = copy.copy(self.balances)   # starting_balances: the same array, no stores
        self.txs: List[Tx] = []
        self.cons: list = []   # world_state.constraints: they carry over into the next transaction
        self.qid = -1          # the query that established the state this world was opened from
        self.dep = DepAnn()    # DependencyAnnotation handed to the next transaction's states

    def fork(self) -> "World":
        w = World.__new__(World)
        w.storage = copy.copy(self.storage)
        w.balances = copy.copy(self.balances)
        w.starting = self.starting
        w.txs = list(self.txs)
        w.cons = list(self.cons)
        w.qid = self.qid
        w.dep = self.dep.copy()
        return w


class Analysis:
    """One `myth analyze <contract> -t tx_count` restated: its queries, module caches and
    the open states between transactions."""

    def __init__(self, name: str, kfm, tx_count: int, max_open: int = 6):
        self.name = name
        self.kfm = kfm
        self.tx_count = tx_count
        self.max_open = max_open
        # (kind, label, terms, expected, parent): parent = the index of the prune query that
        # established the asking state (its witness is the plugin's first candidate), or -1
        self.queries: List[Tuple[str, str, tuple, Optional[str], int]] = []
        self.cache: Dict[str, set] = {}        # DetectionModule.cache per module
        self.ostate_sat: set = set()           # integer.py: _ostates_satisfiable / _unsatisfiable
        self.ostate_unsat: set = set()
        self.next_tid = 1
        self.decide = refuter()
        self._decided: Dict[tuple, bool] = {}
        # DependencyPruner (dependency_pruner.py:83-96): per block, the storage locations read
        # and written on paths through it and whether a call was made; `iteration` counts the
        # transactions as start_sym_trans does (the creation transaction is 1, reset to 0 when
        # it ends, so message call k is iteration k)
        self.dep_sloads: Dict[object, list] = {}
        self.dep_sstores: Dict[object, list] = {}
        self.dep_calls: set = set()
        self.iteration = 0

    def tid(self) -> int:
        t = self.next_tid
        self.next_tid += 1
        return t

    def ask(self, kind: str, label: str, cons: Sequence, expected: Optional[str], parent: int = -1) -> bool:
        """Record one solver query; returns whether the reference's solver finds it
        satisfiable: the expectation by reading, or -- where reading does not decide it --
        "not refuted by the host pre-check" (a refutation is a proof, so z3 answers unsat
        there too and LASER drops the state; an unrefuted query is followed, which can only
        add queries the pre-filter then fails to refute)."""
        terms = tuple(c.raw for c in cons)
        self.queries.append((kind, f"{self.name}:{label}", terms, expected, parent))
        if expected is not None:
            return expected != "unsat"
        return not self.refuted(terms)

    def refuted(self, terms: tuple) -> bool:
        if self.decide is None:
            return False
        r = self._decided.get(terms)
        if r is None:
            r = self._decided[terms] = bool(self.decide(terms))
        return r

    def cached(self, module: str, addr: str) -> bool:
        return addr in self.cache.get(module, ())

    def found(self, module: str, addr: str) -> None:
        self.cache.setdefault(module, set()).add(addr)


def refuter():
    """The host UNSAT pre-check as a decider for branches and module queries that reading
    leaves open: terms -> refuted?  It is the product's strongest setting (mgp_refute_split
    with Prefilter's case splits and interval bisection, CPU code): a refutation is a proof,
    so z3 answers unsat there and LASER drops the state -- a weaker decider would follow
    branches the reference never reaches and count their queries on both sides."""
    from mythril_amd import _native as N
    from mythril_amd.front import Batch
    from mythril_amd.solver import Prefilter

    cache = refute_cache()

    def decide(terms: tuple) -> bool:
        B = Batch([list(terms)])
        try:
            key = f"{int(B.state_key[0]):016x}"
            r = cache.get(key)
            if r is None:
                r = cache[key] = int(N.refute_split(*B.packed()[:4], max_splits=Prefilter.SPLIT_REFUTE,
                                                    depth=Prefilter.SPLIT_DEPTH)[0]) == 1
            return r
        finally:
            B.close()
    return decide


# The stream generator's refutations, by state content key (mgp_build_states
# MGP_FE_STATE_KEY), computed by the refuter itself and kept in corpus/refute_cache.json so
# that a suite() call does not re-run a minute of case splits on states it has decided before
# (`python -m corpus.laser` rewrites it).  The file carries a hash of the refuter's sources and
# settings: after any change to them it is ignored and every decision is recomputed live.
_CACHE_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "refute_cache.json")
_CACHE: Optional[Dict[str, bool]] = None


def _refuter_version() -> str:
    import hashlib

    from mythril_amd.solver import Prefilter

    h = hashlib.sha256(f"{Prefilter.SPLIT_REFUTE}/{Prefilter.SPLIT_DEPTH}".encode())
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mythril_amd", "csrc")
    for f in ("mgp_refute.cpp", "mgp_domain.h", "mgp_bv.h", "mgp_front.cpp"):
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:32]


def refute_cache() -> Dict[str, bool]:
    global _CACHE
    if _CACHE is None:
        _CACHE = {}
        try:
            with open(_CACHE_PATH) as f:
                blob = json.load(f)
            if blob.get("version") == _refuter_version():
                _CACHE = {k: bool(v) for k, v in blob["decisions"].items()}
        except (OSError, ValueError, KeyError):
            pass
    return _CACHE


def save_refute_cache() -> int:
    with open(_CACHE_PATH, "w") as f:
        json.dump({"version": _refuter_version(), "decisions": {k: int(v) for k, v in sorted(refute_cache().items())}},
                  f, separators=(",", ":"))
    return len(refute_cache())


if __name__ == "__main__":
    import corpus
    from corpus import laser as _L  # the module suite() uses (this file runs as __main__)

    from oracle.keccak_ref import keccak256  # CPU Keccak for the manager's concrete hashes

    for mo in (6, 12, 24):
        corpus.suite(hasher=keccak256, max_open=mo, contracts=None if mo == 6 else {"wallet"})
    print(f"{_L.save_refute_cache()} decisions -> {_L._CACHE_PATH}")


class OverflowAnn:
    """integer.py OverUnderflowAnnotation: the state at the op and the overflow condition."""

    _keys = itertools.count()

    def __init__(self, site: str, cons: list, cond, sat: Optional[bool], sat_at_end: Optional[bool]):
        self.key = next(OverflowAnn._keys)   # the ostate's identity (integer.py's ostate sets)
        self.site, self.cons, self.cond = site, cons, cond
        self.qid = -1
        self.sat, self.sat_at_end = sat, sat_at_end


class Path:
    """A GlobalState restated: constraints, world, current transaction, module annotations."""

    def __init__(self, run: Analysis, world: World, tx: Tx, fn: str):
        self.run, self.world, self.tx, self.fn = run, world, tx, fn
        self.cons: list = []
        self.taint: Dict[object, List[OverflowAnn]] = {}  # term -> annotations on that value
        self.sinks: List[OverflowAnn] = []              # annotations that reached a sink
        self.retvals: List[Tuple[str, object, bool]] = []
        self.call_sites: List[str] = []
        self.sc_calls: List[Tuple[list, object, object, bool]] = []  # state_change annotations
        self.potential: List[Tuple[str, str, list, Optional[str]]] = []
        self.mutated = False
        self.selfdestructed = False
        self.qid = -1   # the prune query that established this state (corpus parent links)
        self.dep = world.dep.copy()
        # dropped by DependencyPruner (PluginSkipState): the contract code still walks it
        # (its successors are dead too) but it asks nothing and opens no world state
        self.dead = False

    def _ask(self, kind: str, label: str, cons: Sequence, expected: Optional[str], establishes: bool = False,
             parent: Optional[int] = None) -> bool:
        if self.dead:
            return False
        i = len(self.run.queries)
        r = self.run.ask(kind, label, cons, expected, self.qid if parent is None else parent)
        if establishes:
            self.qid = i
        return r

    def fork(self) -> "Path":
        p = copy.copy(self)
        p.world = self.world.fork()
        p.cons = list(self.cons)
        p.taint = dict(self.taint)
        p.sinks = list(self.sinks)
        p.retvals = list(self.retvals)
        p.call_sites = list(self.call_sites)
        p.sc_calls = list(self.sc_calls)
        p.potential = list(self.potential)
        p.dep = self.dep.copy()
        return p

    # -------------------------------------------------------------- constraints
    def append(self, c, label: str, sat: Optional[bool] = True) -> bool:
        """world_state.constraints.append + the next step's prune query."""
        self.cons.append(c)
        return self._ask("prune", label, self.cons, _exp(sat), establishes=True)

    def branch(self, cond, label: str, t: Optional[bool] = True, f: Optional[bool] = True, origin: bool = False,
               predictable: bool = False) -> Tuple[Optional["Path"], Optional["Path"]]:
        """JUMPI (instructions.py:1533-1610): the module pre-hooks, then both successors,
        each prune-checked; `t` / `f` say which one is feasible (by reading)."""
        if self.dead:
            return self.fork(), self.fork()
        self._sink(cond)
        if origin and not self.run.cached("origin", label) and \
                self._ask("txseq", f"origin@{label}", self._txseq(self.cons), "sat"):
            self.run.found("origin", label)
        if predictable and not self.run.cached("predictable", label) and \
                self._ask("txseq", f"predictable@{label}", self._txseq(self.cons), "sat"):
            self.run.found("predictable", label)
        if is_true(cond) or is_false(cond):
            # a concrete condition: one successor, with the literal True appended
            # (instructions.py:1556-1610), so it is still prune-checked once
            q = self.fork()
            q.cons.append(symbol_factory.Bool(True))
            if not q._dep_block(f"{label}:{'T' if is_true(cond) else 'F'}"):
                q.dead = True
            q._ask("prune", f"{label}:const", q.cons, "sat", establishes=True)
            return (q, None) if is_true(cond) else (None, q)
        succ = []
        for want, ok in ((cond, t), (Not(cond), f)):
            q = self.fork()
            q.cons.append(want)
            # the JUMPI post-hooks (DependencyPruner) run on both successors before the
            # prune filter asks about either (svm.py:320-331, 251-255)
            keep = q._dep_block(f"{label}:{'T' if want is cond else 'F'}")
            succ.append((q, want, ok, keep))
        out = []
        for q, want, ok, keep in succ:
            if not keep:  # PluginSkipState: no prune query, the state is gone
                q.dead = True
                out.append(q)
                continue
            live = q._ask("prune", f"{label}:{'T' if want is cond else 'F'}", q.cons, _exp(ok), establishes=True)
            out.append(q if live else None)
        return out[0], out[1]

    # -------------------------------------------------------------- DependencyPruner
    def _dep_block(self, block) -> bool:
        """jumpi_hook + _check_basic_block (dependency_pruner.py:202-221, 287-310): the block
        joins this path; from iteration 2 on, a block this path has seen runs only if
        wanna_execute says so.  False = PluginSkipState."""
        run, d = self.run, self.dep
        d.path.append(block)
        if run.iteration < 2:
            return True
        if block not in d.seen:
            d.seen.add(block)
            return True
        return self._wanna_execute(block)

    def _wanna_execute(self, block) -> bool:
        """dependency_pruner.py:134-187.  (Its storage_accessed_global branch compares block
        offsets with storage locations and never matches; it is left out.)"""
        run, d = self.run, self.dep
        if block in run.dep_calls:
            return True
        if block not in run.dep_sloads:
            return False
        deps = run.dep_sloads[block]
        for loc in d.written.get(run.iteration - 1, []):
            for dep in list(deps) + list(d.loaded):
                if self._dep_query(loc, dep, block):
                    return True
        return False

    def _dep_query(self, loc, dep, block) -> bool:
        """get_model((location == dependency,)): one SAT-only query on one unfolded equality
        (z3 gets `loc == dep` as written, so distinct location pairs are distinct calls)."""
        from mythril_amd import ir
        from mythril_amd.smt import Bool, mk

        eq = Bool(mk(ir.EQ, 0, (loc.raw, dep.raw)))
        exp = None
        if loc.raw.op == ir.CONST and dep.raw.op == ir.CONST:
            exp = "sat" if loc.raw.params[0] == dep.raw.params[0] else "unsat"
        elif loc.raw is dep.raw:
            exp = "sat"
        return self._ask("dep", f"dependency@{block}", [eq], exp)

    def _dep_sload(self, key) -> None:
        """sload_hook (dependency_pruner.py:247-259)."""
        if self.dead:
            return
        run, d = self.run, self.dep
        _add_loc(d.loaded, key)
        for b in d.path:
            _add_loc(run.dep_sloads.setdefault(b, []), key)

    def _dep_sstore(self, key) -> None:
        """sstore_hook (dependency_pruner.py:238-245)."""
        if self.dead:
            return
        run, d = self.run, self.dep
        for b in d.path:
            _add_loc(run.dep_sstores.setdefault(b, []), key)
        _add_loc(d.written.setdefault(run.iteration, []), key)

    def _dep_call(self) -> None:
        """call_hook (dependency_pruner.py:261-267)."""
        if self.dead:
            return
        for b in self.dep.path:
            if b in self.run.dep_sstores:
                self.run.dep_calls.add(b)
        self.dep.has_call = True

    def _dep_end(self) -> None:
        """_transaction_end at STOP / RETURN (dependency_pruner.py:269-285), then the
        world-state hook: the annotation goes on with path [0] and nothing loaded
        (dependency_pruner.py:312-330)."""
        if self.dead:
            return
        for k in self.dep.loaded:
            for b in self.dep.path:
                _add_loc(self.run.dep_sloads.setdefault(b, []), k)
        if self.dep.has_call:
            self._dep_call()

    def require(self, cond, label: str, t: Optional[bool] = True, f: Optional[bool] = True, **kw) -> Optional["Path"]:
        """require(cond): the false successor reverts (nothing more is asked on it)."""
        return self.branch(cond, label, t, f, **kw)[0]

    def assert_(self, cond, label: str, t: Optional[bool] = True, f: Optional[bool] = True) -> Optional["Path"]:
        """assert(cond): the false successor reaches INVALID (ASSERT_FAIL), where the
        exceptions module asks for a transaction sequence (exceptions.py:55)."""
        ok, bad = self.branch(cond, label, t, f)
        if bad is not None and not self.run.cached("exceptions", label):
            if bad._ask("txseq", f"assert_fail@{label}", bad._txseq(bad.cons), _exp(f)):
                self.run.found("exceptions", label)
        return ok

    # -------------------------------------------------------------- arithmetic
    def _ann(self, r, site: str, cond, sat, sat_at_end):
        if not self.run.cached("integer", site):
            a = OverflowAnn(site, list(self.cons), cond, sat, sat_at_end)
            a.qid = self.qid
            self.taint[r.raw] = self.taint.get(r.raw, []) + [a]
        return r

    def add(self, a, b, site: str, sat: Optional[bool] = True, sat_at_end="same"):
        """ADD pre-hook: Not(BVAddNoOverflow(a, b, False)) annotates the result (integer.py)."""
        a, b = _bv(a), _bv(b)
        return self._ann(a + b, site, Not(BVAddNoOverflow(a, b, False)), sat, sat if sat_at_end == "same" else sat_at_end)

    def sub(self, a, b, site: str, sat: Optional[bool] = True, sat_at_end="same"):
        a, b = _bv(a), _bv(b)
        return self._ann(a - b, site, Not(BVSubNoUnderflow(a, b, False)), sat, sat if sat_at_end == "same" else sat_at_end)

    def mul(self, a, b, site: str, sat: Optional[bool] = True, sat_at_end="same"):
        a, b = _bv(a), _bv(b)
        return self._ann(a * b, site, Not(BVMulNoOverflow(a, b, False)), sat, sat if sat_at_end == "same" else sat_at_end)

    def _sink(self, value) -> None:
        """SSTORE / JUMPI / CALL / RETURN pre-hooks: annotations on the value (and on any
        sub-term it was computed from: laser.smt unions operand annotations) reach a sink."""
        if not self.taint:
            return
        seen, stack = set(), [value.raw]
        while stack:
            t = stack.pop()
            if id(t) in seen:
                continue
            seen.add(id(t))
            for a in self.taint.get(t, ()):
                if a not in self.sinks:
                    self.sinks.append(a)
            stack.extend(t.args)

    # -------------------------------------------------------------- storage
    def sload(self, key):
        self._dep_sload(_bv(key))
        return self.world.storage[_bv(key)]

    def sstore(self, key, value) -> None:
        value = _bv(value)
        self._sink(value)
        self._state_access("sstore")
        self._dep_sstore(_bv(key))
        self.world.storage[_bv(key)] = value
        self.mutated = True

    def mapping(self, key, slot, label: str):
        """m[key] at `slot` (a slot number, or the hash of an outer mapping's entry): SHA3
        over Concat(key, slot) -- the keccak manager's condition is appended
        (instructions.py:1037), so the next step is prune-checked."""
        h, cond = self.run.kfm.create_keccak(Concat(_bv(key), _bv(slot)))
        self.append(cond, f"sha3@{label}")
        return h

    def sha3_word(self, x, label: str):
        """keccak256 of one 32-byte word: a dynamic array's data location keccak(slot)."""
        h, cond = self.run.kfm.create_keccak(_bv(x))
        self.append(cond, f"sha3@{label}")
        return h

    def _state_access(self, label: str) -> None:
        """state_change_external_calls: a storage access after a recorded external call asks
        for a transaction sequence (state_change_external_calls.py:40-75)."""
        for call_cons, gas, to, user in self.sc_calls:
            site = f"{self.fn}:{label}"
            if self.run.cached("state_change", site):
                continue
            extra = [UGT(gas, BVV(2300, 256)), Or(UGT(to, BVV(16, 256)), to == BVV(0, 256))]
            if user:
                extra.append(to == BVV(ATTACKER, 256))
            if self._ask("txseq", f"state_change@{site}", self._txseq(self.cons + extra), "sat"):
                self.run.found("state_change", site)

    # -------------------------------------------------------------- calls
    def call(self, to, value, gas, label: str, gas_ok: Optional[bool] = True, to_attacker: Optional[bool] = True,
             value_pos: Optional[bool] = True, thief="skip"):
        """CALL to an account without code (every callee here): the module pre-hooks
        (external_calls, state_change, integer, multiple_sends), transfer_ether
        (instructions.py:66-87, one constraint + prune query), a fresh retval, then the
        post-hooks (ether_thief, unchecked_retval).  `gas_ok` / `to_attacker` /
        `value_pos` / `thief` are the answers by reading."""
        to, value, gas = _bv(to), _bv(value), _bv(gas)
        run = self.run
        self._dep_call()
        self._sink(value)
        self._state_access(f"call@{label}")
        # external_calls.py:83-110: gas > 2300 and to == attacker -> a potential issue
        if not run.cached("external_calls", label):
            extra = [UGT(gas, BVV(2300, 256)), to == BVV(ATTACKER, 256)]
            exp = _exp(False if gas_ok is False or to_attacker is False else (None if gas_ok is None or to_attacker is None else True))
            if self._ask("txseq", f"external_call@{label}", self._txseq(self.cons + extra), exp):
                self.potential.append(("external_calls", label, extra, exp))
        # state_change_external_calls.py:171-198: _balance_change, then _add_external_call
        if value.raw.op != 2:  # a symbolic value
            self._ask("model", f"balance_change@{label}", self.cons + [UGT(value, BVV(0, 256))],
                    _exp(value_pos))
        ext = [UGT(gas, BVV(2300, 256)), Or(UGT(to, BVV(16, 256)), to == BVV(0, 256))]
        if self._ask("model", f"add_external_call@{label}", self.cons + ext, _exp(gas_ok)):
            user = self._ask("model", f"external_call_attacker@{label}",
                           self.cons + ext + [to == BVV(ATTACKER, 256)], _exp(to_attacker))
            self.sc_calls.append((list(self.cons), gas, to, user))
        self.call_sites.append(label)
        # transfer_ether
        this = BVV(CONTRACT_ADDRESS, 256)
        self.append(UGE(self.world.balances[this], value), f"transfer@{label}")
        self.world.balances[to] = self.world.balances[to] + value
        self.world.balances[this] = self.world.balances[this] - value
        self.mutated = True   # MutationPruner's CALL pre-hook
        retval = self.tx.env(f"retval_{label}")
        self.retvals.append((label, retval, True))
        # ether_thief.py:55-95 (post-hook): the attacker's balance grew, attacker is sender
        if thief != "skip" and not run.cached("ether_thief", label):
            extra = [UGT(self.world.balances[BVV(ATTACKER, 256)], self.world.starting[BVV(ATTACKER, 256)]),
                     self.tx.sender == BVV(ATTACKER, 256)]
            exp = _exp(thief)
            if self._ask("model", f"ether_thief@{label}", self.cons + extra, exp):
                self.potential.append(("ether_thief", label, extra, exp))
        return retval

    def selfdestruct(self, to, label: str, attacker_to: Optional[bool], reachable: Optional[bool] = True) -> None:
        """suicide.py:60-110: the attacker query, then (if unsat) the plain one."""
        to = _bv(to)
        self.selfdestructed = True   # SUICIDE ends the transaction (no STOP / RETURN hooks)
        if self.run.cached("suicide", label):
            return
        who = [And(t.sender == BVV(ATTACKER, 256), t.sender == t.sender) for t in self.world.txs if not t.creation]
        q1 = self._ask("txseq", f"suicide_attacker@{label}", self._txseq(self.cons + who + [to == BVV(ATTACKER, 256)]),
                          _exp(attacker_to))
        if q1 or self._ask("txseq", f"suicide@{label}", self._txseq(self.cons + who),
                              _exp(reachable)):
            self.run.found("suicide", label)

    # -------------------------------------------------------------- transaction end
    def _txseq(self, cons: list) -> list:
        """analysis/solver.py:242-282: calldatasize <= 5000 and the starting-balance caps of
        every transaction's caller, and a cap on every account (creator, attacker, someguy,
        the contract)."""
        out = list(cons)
        for t in self.world.txs:
            if not t.creation:
                out.append(UGE(BVV(5000, 256), t.size))
            out.append(UGE(BVV(10 ** 21, 256), self.world.starting[t.sender]))
        for a in ACTORS + (CONTRACT_ADDRESS,):
            out.append(UGE(BVV(10 ** 20, 256), self.world.starting[BVV(a, 256)]))
        return out

    def stop(self, label: str = "stop") -> Optional["Path"]:
        """STOP / RETURN: the modules' pre-hooks, check_potential_issues (potential_issues.py:
        75-108), then add_world_state with MutationPruner's filter (mutation_pruner.py:55-83).
        Returns the path when its world state opens the next transaction."""
        run = self.run
        if self.dead:
            return None
        # unchecked_retval.py:80-110: one transaction sequence per recorded retval
        for site, rv, free in ([] if self.selfdestructed else self.retvals):
            if run.cached("unchecked_retval", site):
                continue
            if self._ask("txseq", f"unchecked_retval@{site}", self._txseq(self.cons + [rv == BVV(0, 256)]),
                       _exp(free)):
                run.found("unchecked_retval", site)
        # multiple_sends.py:60-100: every call after the first
        for site in ([] if self.selfdestructed else self.call_sites[1:]):
            if run.cached("multiple_sends", site):
                continue
            if self._ask("txseq", f"multiple_sends@{site}", self._txseq(self.cons), "sat"):
                run.found("multiple_sends", site)
                break
        # integer.py:263-330
        for a in ([] if self.selfdestructed else self.sinks):
            if run.cached("integer", a.site) or a.key in run.ostate_unsat:
                continue
            if a.key not in run.ostate_sat:
                if self._ask("model", f"overflow@{a.site}", a.cons + [a.cond], _exp(a.sat), parent=a.qid):
                    run.ostate_sat.add(a.key)
                else:
                    run.ostate_unsat.add(a.key)
                    continue
            if self._ask("txseq", f"overflow_issue@{a.site}", self._txseq(self.cons + [a.cond]),
                       _exp(a.sat_at_end)):
                run.found("integer", a.site)
        # check_potential_issues
        for module, site, extra, exp in self.potential:
            if run.cached(module, site):
                continue
            if self._ask("txseq", f"potential_{module}@{site}", self._txseq(self.cons + extra), exp):
                run.found(module, site)
        self.world.cons = list(self.cons)   # the open world state keeps the path's constraints
        self.world.qid = self.qid
        self._dep_end()
        self.dep.path = [0]
        self.dep.loaded = []
        self.world.dep = self.dep
        if self.tx.creation:
            return self
        # MutationPruner: keep a world state that mutated, or whose callvalue can be > 0
        # (non-payable: the dispatcher pinned callvalue to 0; payable: it depends on the path)
        payable = self._ask("model", f"mutation_pruner@{label}", self.cons + [UGT(self.tx.value, BVV(0, 256))],
                          None if self.payable else "unsat")
        return self if (payable or self.mutated) else None

    payable = False


class Contract:
    """A contract restated: functions (selector, payable, body), fallback, constructor.

    A body is `body(p) -> list of end paths` (paths that reached STOP / RETURN); a path that
    reverts is simply not returned."""

    name = "?"
    tx_count = 2
    functions: List[Tuple[str, int, bool, object]] = []  # (name, selector, payable, body)
    fallback = None             # (payable, body) or None: a revert
    fallback_payable = False

    def constructor(self, p: Path) -> List[Path]:
        return [p]


def start_tx(run: Analysis, world: World, creation: bool = False, index: int = 0) -> Path:
    """_setup_global_state_for_execution + initial_global_state: sender among the ACTORS,
    it can pay the value, the value moves (transaction_models.py:110-133)."""
    tx = Tx(run.tid(), creation)
    tx.index = index   # 0: the creation transaction, k: the k-th message call
    run.iteration = 1 if creation else index   # start_sym_trans (the creation's is reset after it)
    w = world.fork()
    w.txs.append(tx)
    p = Path(run, w, tx, "constructor" if creation else "dispatcher")
    p.cons = list(w.cons)
    p.cons.append(Or(*[tx.sender == BVV(a, 256) for a in ACTORS]))
    this = BVV(CONTRACT_ADDRESS, 256)
    p.cons.append(UGE(w.balances[tx.sender], tx.value))
    w.balances[this] = w.balances[this] + tx.value
    w.balances[tx.sender] = w.balances[tx.sender] - tx.value
    p.qid = w.qid
    p._ask("prune", "tx_start", p.cons, "sat", establishes=True)
    return p


def dispatch(contract: Contract, p: Path) -> List[Path]:
    """The solc dispatcher: calldatasize < 4 -> fallback; the selector compared with every
    function's in order; a non-payable function's callvalue check; no match -> fallback."""
    tx = p.tx
    ends: List[Path] = []
    short, rest = p.branch(ULT(tx.size, BVV(4, 256)), "dispatch:size<4")
    sel = UDiv(tx.word(0), BVV(1 << 224, 256)) & BVV(0xFFFFFFFF, 256)
    for name, sig, payable, body in contract.functions:
        if rest is None:
            break
        hit, rest = rest.branch(sel == BVV(sig, 256), f"dispatch:{name}")
        if hit is None:
            continue
        hit.fn = name
        hit.payable = payable
        if not payable:
            hit = hit.require(tx.value == BVV(0, 256), f"{name}:callvalue")
            if hit is None:
                continue
        ends.extend(body(hit))
    for q in (short, rest):
        if q is None or contract.fallback is None:
            continue
        q.fn = "fallback"
        q.payable = contract.fallback_payable
        if not contract.fallback_payable:
            q = q.require(tx.value == BVV(0, 256), "fallback:callvalue")
            if q is None:
                continue
        ends.extend(contract.fallback(q))
    return ends


def analyze(contract: Contract, kfm, tx_count: Optional[int] = None, max_open: int = 6) -> Analysis:
    """Creation transaction, then `tx_count` message-call rounds from every open state."""
    run = Analysis(contract.name, kfm, tx_count or contract.tx_count, max_open)
    p = start_tx(run, World(), creation=True)
    opened = []
    for q in contract.constructor(p):
        r = q.stop("constructor_end")
        if r is not None:
            opened.append(r.world)
    for k in range(run.tx_count):
        nxt = []
        for w in opened[:run.max_open]:
            p = start_tx(run, w, index=k + 1)
            for q in dispatch(contract, p):
                r = q.stop(f"{q.fn}_end")
                if r is not None:
                    nxt.append(r.world)
        opened = nxt
    return run
