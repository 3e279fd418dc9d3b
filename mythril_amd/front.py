"""Native front end: a batch of states' constraint terms -> packed DAGs, variable tables, hints.

`Batch(term_lists)` hands the term arena (smt.ARENA) and the root term ids of every
state to `mgp_build_states` (csrc/mgp_front.cpp, OpenMP over states) and exposes
the result as numpy views: exactly the arrays mythril_amd/dag.py build_state +
pack_states (+ make_candidates' flattened tables) produce in Python, which stay as
the reference implementation the tests pin this one against.  Replaces, per batch,
the per-state re-adding of every constraint to a fresh z3 solver that
Constraints.is_possible (constraints.py:34-51) and get_model (analysis/solver.py:
37-50) do.
"""
from __future__ import annotations

import ctypes
from collections.abc import Mapping
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _native as N
from .smt import ARENA, Term

FE_SAT_UNSAFE = 0x1
FE_STRENGTHENED = 0x2

# include/mgp.h enum mgp_fe_field -> (index, dtype, items per entry)
_FIELDS = {
    "nodes": (0, N.NODE_DTYPE, 1), "gpu_nodes": (1, N.NODE_DTYPE, 1), "node_off": (2, np.uint64, 1),
    "consts": (3, np.uint32, 8), "const_off": (4, np.uint64, 1), "var_off": (5, np.uint64, 1),
    "var_width": (6, np.uint32, 1), "var_full": (7, np.uint32, 1), "var_name": (8, np.uint32, 1),
    "var_aux": (9, np.uint32, 1), "var_kind": (10, np.uint8, 1), "hint_off": (11, np.uint64, 1),
    "hints": (12, np.uint32, 8), "alias_off": (13, np.uint64, 1), "aliases": (14, np.uint32, 2),
    "flags": (15, np.uint8, 1), "var_key": (16, np.uint64, 1), "gpu_node_off": (17, np.uint64, 1),
    "var_tid": (18, np.int32, 1), "state_key": (19, np.uint64, 1), "dec_nodes": (20, N.NODE_DTYPE, 1),
}
_VAR_TABLES = ("var_off", "var_width", "var_full", "var_name", "var_aux", "var_kind", "var_key", "var_tid")
FIXED_POOL_LIMBS = None  # dag._FIXED_LIMBS (set lazily: dag imports the native module too)


def _arena_ptr(a) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.buffer_info()[0])


class Batch:
    """Flattened constraint DAGs of n states (owned by the native batch object)."""

    def __init__(self, term_lists: Sequence[Sequence[Term]], arena=None):
        """arena: the term arena to read (smt.ARENA, or a snapshot of it with the same
        arrays for a builder running off the thread that creates terms)."""
        L = N.lib()
        roots = np.fromiter((t.tid for lst in term_lists for t in lst), dtype=np.int32)
        off = np.zeros(len(term_lists) + 1, np.uint64)
        if len(term_lists):
            off[1:] = np.cumsum([len(lst) for lst in term_lists])
        if roots.size == 0:
            roots = np.zeros(1, np.int32)
        self.n_states = len(term_lists)
        self._vt = None
        self._h = ctypes.c_void_p()
        A = ARENA if arena is None else arena
        rc = L.mgp_build_states(_arena_ptr(A.op), _arena_ptr(A.width), _arena_ptr(A.args), _arena_ptr(A.p),
                                len(A.op), _arena_ptr(A.limbs), len(A.limbs), N._ptr(roots), N._ptr(off),
                                self.n_states, _arena_ptr(A.name_hash) if len(A.name_hash) else None,
                                len(A.name_hash), ctypes.byref(self._h))
        N._check(rc)
        self._load_fields()

    def select(self, idx: Sequence[int]) -> "Batch":
        """States idx of this batch as a batch of their own (mgp_fe_select: the arrays a
        build of those states would give, without walking the term arena again)."""
        ix = np.ascontiguousarray(np.asarray(idx, dtype=np.uint32).reshape(-1))
        out = Batch.__new__(Batch)
        out.n_states = int(ix.size)
        out._vt = None
        out._h = ctypes.c_void_p()
        N._check(N.lib().mgp_fe_select(self._h, N._ptr(ix) if ix.size else None, ix.size, ctypes.byref(out._h)))
        out._load_fields()
        return out

    def _load_fields(self) -> None:
        L = N.lib()
        for name, (idx, dt, per) in _FIELDS.items():
            p, n = ctypes.c_void_p(), ctypes.c_uint64()
            N._check(L.mgp_fe_get(self._h, idx, ctypes.byref(p), ctypes.byref(n)))
            cnt = int(n.value)
            if cnt == 0 or not p.value:
                arr = np.zeros((0, per) if per > 1 else 0, dtype=dt)
            else:
                buf = (ctypes.c_char * (cnt * np.dtype(dt).itemsize)).from_address(p.value)
                arr = np.frombuffer(buf, dtype=dt)
                if per > 1:
                    arr = arr.reshape(-1, per)
            setattr(self, name, arr)

    def var_tables(self) -> "VarTables":
        """Owned copies of the variable tables (witnesses outlive the native batch)."""
        if self._vt is None:
            self._vt = VarTables(*(np.array(getattr(self, k)) for k in _VAR_TABLES))
        return self._vt

    def check(self, ctx, n_cand: int, seed: int, parents: Optional[Sequence] = None, refute: bool = True,
              xrows=None):
        """-> (first_sat i32[n], witness u32[n, n_vars, 8], refuted i8[n], stage ms[5]) through the
        context's check_batch (mgp_check_batch on a libmgp context).  xrows = (rows u32 [n, k,
        nv, 8], mask u8 [n, k, nv]): explicit rows placed in the first k mixture rows."""
        return ctx.check_batch(self, n_cand, seed, parents, refute, xrows)

    def submit(self, ctx, n_cand: int, seed: int, parents: Optional[Sequence] = None, refute: bool = True,
               xrows=None):
        """The host half of check (mgp_check_submit on a libmgp context): lowering, pre-check
        and staging now, the GPU round enqueued; -> a pending round whose finish() returns
        check's tuple.  A context without submit_batch (a test double) answers at once."""
        sub = getattr(ctx, "submit_batch", None)
        if sub is None:
            return _Answered(ctx.check_batch(self, n_cand, seed, parents, refute, xrows))
        return sub(self, n_cand, seed, parents, refute, xrows)

    def _native_args(self, n_cand: int, seed: int, parents, xrows):
        """The batch-side arguments of mgp_check_batch / mgp_check_submit."""
        global FIXED_POOL_LIMBS
        if FIXED_POOL_LIMBS is None:
            from .dag import _FIXED_LIMBS

            FIXED_POOL_LIMBS = np.ascontiguousarray(_FIXED_LIMBS, dtype=np.uint32)
        n = self.n_states
        pk = pv = po = None
        if parents is not None and any(p is not None for p in parents):
            ks, vs, cnt = [], [], []
            for p in parents:
                k, v = parent_arrays(p)
                ks.append(k)
                vs.append(v)
                cnt.append(len(k))
            pk = np.ascontiguousarray(np.concatenate(ks), dtype=np.uint64)
            pv = np.ascontiguousarray(np.concatenate(vs).reshape(-1, 8), dtype=np.uint32)
            po = np.zeros(n + 1, np.uint64)
            po[1:] = np.cumsum(cnt)
            if pk.size == 0:
                pk, pv = np.zeros(1, np.uint64), np.zeros((1, 8), np.uint32)
        xr, xm, nx, nxv = self._xrows(xrows)
        # (the arrays stay referenced by the caller until the native call returns)
        return (pk, pv, po, xr, xm), (self._h, n_cand, seed & (2 ** 64 - 1), N._ptr(FIXED_POOL_LIMBS),
                                      len(FIXED_POOL_LIMBS), N._ptr(pk), N._ptr(pv), N._ptr(po),
                                      N._ptr(self.var_key) if pk is not None else None,
                                      N._ptr(xr), N._ptr(xm), nx, nxv)

    def _check_native(self, ctx, n_cand: int, seed: int, parents: Optional[Sequence] = None, refute: bool = True,
                      xrows=None):
        """mgp_check_batch on libmgp context `ctx`."""
        n = self.n_states
        n_vars = max(1, self.n_vars())
        first = np.full(n, N.MGP_NO_SAT, np.int32)
        wit = np.zeros((n, n_vars, 8), np.uint32)
        ref = np.zeros(max(n, 1), np.int8)
        times = np.zeros(5, np.float64)
        nv = ctypes.c_uint32(0)
        keep, args = self._native_args(n_cand, seed, parents, xrows)
        rc = N.lib().mgp_check_batch(ctx._h, *args, 0 if refute else 1, N._ptr(first), N._ptr(wit), N._ptr(ref),
                                     ctypes.byref(nv), N._ptr(times))
        N._check(rc, ctx._h)
        return first, wit, ref[:n], times

    def _submit_native(self, ctx, n_cand: int, seed: int, parents: Optional[Sequence] = None, refute: bool = True,
                       xrows=None) -> "PendingRound":
        """mgp_check_submit on libmgp context `ctx`."""
        n = self.n_states
        ref = np.zeros(max(n, 1), np.int8)
        times = np.zeros(5, np.float64)
        nv = ctypes.c_uint32(0)
        ticket = ctypes.c_int32(-1)
        keep, args = self._native_args(n_cand, seed, parents, xrows)
        rc = N.lib().mgp_check_submit(ctx._h, *args, 0 if refute else 1, N._ptr(ref), ctypes.byref(nv),
                                      N._ptr(times), ctypes.byref(ticket))
        N._check(rc, ctx._h)
        del keep
        return PendingRound(ctx, ticket.value, n, max(1, self.n_vars()), ref[:n], times)

    def _xrows(self, xrows):
        if xrows is None:
            return None, None, 0, 0
        rows, mask = xrows
        rows = np.ascontiguousarray(rows, dtype=np.uint32)
        mask = np.ascontiguousarray(mask, dtype=np.uint8)
        if rows.ndim != 4 or rows.shape[0] != self.n_states or rows.shape[3] != 8 or mask.shape != rows.shape[:3]:
            raise ValueError("xrows must be (rows u32 [n_states, k, n_vars, 8], mask u8 [n_states, k, n_vars])")
        if rows.shape[1] == 0 or rows.shape[2] == 0:
            return None, None, 0, 0
        return rows, mask, rows.shape[1], rows.shape[2]

    def device_candidates(self, ctx, n_cand: int, n_vars: int, seed: int, dom=None, xrows=None) -> np.ndarray:
        """Test hook (mgp_fe_candidates): the GPU-generated first-round candidates, returned in
        the host layout [state][cand][var][8] of mgp_make_candidates."""
        global FIXED_POOL_LIMBS
        if FIXED_POOL_LIMBS is None:
            from .dag import _FIXED_LIMBS

            FIXED_POOL_LIMBS = np.ascontiguousarray(_FIXED_LIMBS, dtype=np.uint32)
        n = self.n_states
        dev = np.zeros((n, n_vars, 2, n_cand, 4), np.uint32)
        xr, xm, nx, nxv = self._xrows(xrows)
        N._check(N.lib().mgp_fe_candidates(ctx._h, self._h, n_cand, n_vars, seed & (2 ** 64 - 1),
                                           N._ptr(FIXED_POOL_LIMBS), len(FIXED_POOL_LIMBS),
                                           None if dom is None else N._ptr(np.ascontiguousarray(dom, np.uint32)),
                                           N._ptr(xr), N._ptr(xm), nx, nxv, N._ptr(dev)), ctx._h)
        return np.ascontiguousarray(dev.transpose(0, 3, 1, 2, 4).reshape(n, n_cand, n_vars, 8))

    def witness(self, s: int, words: np.ndarray) -> "SlotWitness":
        """State s's witness (words [n_vars, 8]) as a lazily decoded {name: value} mapping."""
        vt = self.var_tables()
        v0, v1 = int(vt.var_off[s]), int(vt.var_off[s + 1])
        return SlotWitness(vt, v0, v1, words[: v1 - v0])

    def witnesses(self, idx: Sequence[int], words: np.ndarray) -> List["SlotWitness"]:
        """Witnesses of states idx (words [n, n_vars, 8] indexed by state): Batch.witness in
        bulk, with the slot offsets read in one numpy gather (a 1 024-state answer list)."""
        vt = self.var_tables()
        ix = np.asarray(idx, dtype=np.int64)
        v0s, v1s = vt.var_off[ix].tolist(), vt.var_off[ix + 1].tolist()
        return [SlotWitness(vt, a, b, words[i, : b - a]) for i, a, b in zip(ix.tolist(), v0s, v1s)]

    def close(self) -> None:
        if self._h:
            N.lib().mgp_fe_free(self._h)
            self._h = ctypes.c_void_p()
            for name in _FIELDS:
                setattr(self, name, None)

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ views
    def packed(self, gpu: bool = False, decide: bool = False):
        """(nodes, node_offsets, consts [n, 8], const_offsets) as dag.pack_states; gpu=True
        gives the program the GPU evaluates (padded key equalities strengthened, excess
        constants pinned); decide=True the strengthened formula on the original node
        indices, which witness searches aim at (never refutations: it implies the
        original formula, not the other way round)."""
        if gpu:
            return self.gpu_nodes, self.gpu_node_off, self.consts, self.const_off
        if decide:
            return self.dec_nodes, self.node_off, self.consts, self.const_off
        return self.nodes, self.node_off, self.consts, self.const_off

    def n_vars(self, s: Optional[int] = None) -> int:
        if s is None:
            return int(np.diff(self.var_off).max()) if self.n_states else 0
        return int(self.var_off[s + 1] - self.var_off[s])

    def var_names(self, s: int) -> List[str]:
        """dag.StateDag.vars names of state s (`name`, `name#j`, `fn@node`)."""
        out = []
        j = 0
        for v in range(int(self.var_off[s]), int(self.var_off[s + 1])):
            j = 0 if self.var_full[v] else j + 1  # slot index within a wide value
            kind = int(self.var_kind[v])
            if kind == 2:
                nm = f"#pool{int(self.var_aux[v])}"
            else:
                nm = ARENA.names[int(self.var_name[v])]
                if kind:
                    nm = f"{nm}@{int(self.var_aux[v])}"
            out.append(nm if j == 0 else f"{nm}#{j}")
        return out

    def witness_to_model(self, s: int, words: np.ndarray) -> Dict[str, int]:
        """Witness words [n_vars, 8] of state s -> {name: value} (dag.witness_to_model)."""
        v0, v1 = int(self.var_off[s]), int(self.var_off[s + 1])
        w = np.ascontiguousarray(words[: v1 - v0], dtype=np.uint32)
        vals = [int.from_bytes(w[i].tobytes(), "little") for i in range(v1 - v0)]
        return _decode(self.var_width, self.var_full, self.var_name, self.var_aux, self.var_kind, v0, v1, vals)


class PendingRound:
    """A witness round submitted with mgp_check_submit; finish() waits for its GPU work and
    returns (first_sat, witness, refuted, stage ms[5]) as Batch.check does."""

    def __init__(self, ctx, ticket: int, n: int, n_vars: int, refuted: np.ndarray, times: np.ndarray):
        self.ctx, self.ticket, self.n, self.n_vars = ctx, ticket, n, n_vars
        self.refuted, self.times = refuted, times
        self._out = None

    def finish(self):
        if self._out is None:
            first = np.full(self.n, N.MGP_NO_SAT, np.int32)
            wit = np.zeros((self.n, self.n_vars, 8), np.uint32)
            N._check(N.lib().mgp_check_finish(self.ctx._h, self.ticket, N._ptr(first), N._ptr(wit),
                                              N._ptr(self.times[3:])), self.ctx._h)
            self._out = (first, wit, self.refuted, self.times)
        return self._out


class _Answered:
    """A round answered at submission (a context without mgp_check_submit)."""

    def __init__(self, out):
        self._out = out
        self.times = out[3]

    def finish(self):
        return self._out


class VarTables:
    """Owned copies of a batch's per-slot variable tables."""

    def __init__(self, var_off, var_width, var_full, var_name, var_aux, var_kind, var_key, var_tid):
        self.var_off, self.var_width, self.var_full = var_off, var_width, var_full
        self.var_name, self.var_aux, self.var_kind, self.var_key = var_name, var_aux, var_kind, var_key
        self.var_tid = var_tid


class SlotWitness(Mapping):
    """A GPU witness: slot keys + 8-limb values, decoded to {name: int} on first access
    (dag.witness_to_model semantics).  Children reuse `keys`/`vals` directly as their
    parent-witness row (mgp_check_batch)."""

    __slots__ = ("_vt", "_v0", "_v1", "vals", "_d")

    def __init__(self, vt: VarTables, v0: int, v1: int, vals: np.ndarray):
        self._vt, self._v0, self._v1, self.vals, self._d = vt, v0, v1, vals, None

    @property
    def keys_array(self) -> np.ndarray:
        return self._vt.var_key[self._v0: self._v1]

    def _dict(self) -> Dict[str, int]:
        if self._d is None:
            vt, v0, v1 = self._vt, self._v0, self._v1
            vals = [int.from_bytes(np.ascontiguousarray(self.vals[i]).tobytes(), "little") for i in range(v1 - v0)]
            self._d = _decode(vt.var_width, vt.var_full, vt.var_name, vt.var_aux, vt.var_kind, v0, v1, vals)
        return self._d

    def __getitem__(self, k):
        return self._dict()[k]

    def __iter__(self):
        return iter(self._dict())

    def __len__(self):
        return len(self._dict())

    def __repr__(self):
        return f"SlotWitness({self._dict()!r})"


_KIND_UF = 1 << 63


def _decode(var_width, var_full, var_name, var_aux, var_kind, v0: int, v1: int, vals) -> Dict[str, int]:
    """Slot values of one state -> {name: value} (dag.witness_to_model): a wide value joined
    from its pieces, fresh UF values as `fn@node`, pinned constants left out."""
    d: Dict[str, int] = {}
    i = 0
    while i < v1 - v0:
        full = int(var_full[v0 + i])
        k = max(1, (full + 255) // 256)
        kind = int(var_kind[v0 + i])
        if kind != 2:
            nm = ARENA.names[int(var_name[v0 + i])]
            if kind:
                nm = f"{nm}@{int(var_aux[v0 + i])}"
            pieces = [vals[i + j] & ((1 << int(var_width[v0 + i + j])) - 1) for j in range(k)]
            d[nm] = sum(p << (256 * j) for j, p in enumerate(pieces))
        i += k
    return d


def parent_arrays(p) -> "tuple[np.ndarray, np.ndarray]":
    """(slot keys u64[k], values u32[k, 8]) of a parent witness: a SlotWitness as is; a
    {name: value} dict (e.g. a fallback solver's model) by name -- `name`, `fn@node`,
    a value wider than 256 bits spread over its pieces."""
    if p is None:
        return np.zeros(0, np.uint64), np.zeros((0, 8), np.uint32)
    if isinstance(p, SlotWitness):
        return p.keys_array, np.ascontiguousarray(p.vals, dtype=np.uint32).reshape(-1, 8)
    keys: List[int] = []
    vals: List[bytes] = []
    for name, value in p.items():
        if not isinstance(value, int):
            continue
        uf = "@" in name and name.rsplit("@", 1)[1].isdigit()
        base, node = (name.rsplit("@", 1)[0], int(name.rsplit("@", 1)[1])) if uf else (name, 0)
        nid = ARENA.name_id.get(base)
        if nid is None:
            continue
        value &= (1 << 2048) - 1
        for j in range(max(1, (value.bit_length() + 255) // 256)):
            piece = (value >> (256 * j)) & ((1 << 256) - 1)
            keys.append((_KIND_UF | (nid << 32) | ((node & 0xFFFFFF) << 8) | j) if uf else ((nid << 32) | j))
            vals.append(piece.to_bytes(32, "little"))
    if not keys:
        return np.zeros(0, np.uint64), np.zeros((0, 8), np.uint32)
    return np.array(keys, np.uint64), np.frombuffer(b"".join(vals), np.uint32).reshape(-1, 8)


def seed_arrays(B: "Batch", parents: Sequence) -> "tuple[np.ndarray, np.ndarray]":
    """Per state of batch B, its parent witness's values on B's variable slots, matched by
    slot key as mgp_check_batch matches the parent row: (vals u32 [n, n_vars, 8], mask u8
    [n, n_vars]) for mgp_decision_rows_seeded."""
    n, nv = B.n_states, max(1, B.n_vars())
    vals = np.zeros((n, nv, 8), np.uint32)
    mask = np.zeros((n, nv), np.uint8)
    for s, p in enumerate(parents):
        if p is None:
            continue
        pk, pv = parent_arrays(p)
        if pk.size == 0:
            continue
        v0, v1 = int(B.var_off[s]), int(B.var_off[s + 1])
        keys = np.asarray(B.var_key[v0:v1], dtype=np.uint64)
        order = np.argsort(pk, kind="stable")
        sk = pk[order]
        pos = np.searchsorted(sk, keys)
        pos = np.minimum(pos, len(sk) - 1)
        hit = (sk[pos] == keys) & (keys != np.uint64(0xFFFFFFFFFFFFFFFF))
        idx = np.nonzero(hit)[0]
        vals[s, idx] = pv[order[pos[idx]]]
        mask[s, idx] = 1
    return vals, mask

