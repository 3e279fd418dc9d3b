"""ctypes binding of libmgp.so (include/mgp.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (``make -C
mythril_amd/csrc``) and lives next to this file.  There is deliberately no
fallback: if the library is missing or cannot load, every entry point raises
``NativeUnavailable`` — the product path never silently evaluates constraints
on the CPU.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MGP_LIB_PATH: an alternative build of the same library (A/B measurements of kernel variants)
LIB_PATH = os.environ.get("MGP_LIB_PATH") or os.path.join(_HERE, "libmgp.so")

# include/mgp_ir.h : mgp_node (24 bytes)
NODE_DTYPE = np.dtype(
    [
        ("op", "u1"),
        ("flags", "u1"),
        ("width", "<u2"),
        ("a", "<i4"),
        ("b", "<i4"),
        ("c", "<i4"),
        ("p0", "<u4"),
        ("p1", "<u4"),
    ]
)
assert NODE_DTYPE.itemsize == 24

MGP_OK = 0
MGP_E_ARG = -1
MGP_E_HIP = -2
MGP_E_NOMEM = -3
MGP_E_CAPACITY = -4

MGP_NO_SAT = -1
MGP_UNDECIDED = -2
MGP_EVAL_FAULT = -3  # internal inconsistency (never expected); treated as undecided
ST_OK = 0
ST_UNSUPPORTED = 1


class NativeUnavailable(RuntimeError):
    """libmgp.so is missing or failed to load (no CPU fallback exists)."""


class MgpError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mgp error {code}: {msg}")
        self.code = code


_lib = None
_lib_lock = threading.Lock()

_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_I32 = ctypes.c_int32


def _bind(lib):
    sig = {
        "mgp_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_P)]),
        "mgp_destroy": (None, [_P]),
        "mgp_last_error": (ctypes.c_char_p, [_P]),
        "mgp_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
        "mgp_version": (ctypes.c_char_p, []),
        "mgp_lower": (ctypes.c_int, [_P, _P, _U32, _P, _P, _U32, _P, _U64, _P, _P, _P]),
        "mgp_eval_batch": (ctypes.c_int, [_P, _P, _P, _U32, _P, _U32, _U32, _P, _P]),
        "mgp_eval_batch_dev": (ctypes.c_int, [_P, _P, _U32, _P, _U32, _U32, _U32, _P, _P, _P, _P, _P, _P, _U32, _P]),
        "mgp_plan_buckets": (ctypes.c_int, [_P, _P, _U32, _P, _P, _P, _U32]),
        "mgp_fill_candidates_dev": (ctypes.c_int, [_P, _P, _U32, _U64, _U64, _P, _U32, _U32, _P]),
        "mgp_plant_candidates_dev": (ctypes.c_int, [_P, _U32, _U32, _U32, _P, _P, _P, _U32, _P]),
        "mgp_keccak256_batch": (ctypes.c_int, [_P, _P, _U64, _U32, _U32, _P]),
        "mgp_keccak256_dev": (ctypes.c_int, [_P, _U64, _U32, _U32, _P, _P]),
        "mgp_fill_mapping_preimages_dev": (ctypes.c_int, [_P, _U64, _U64, _U64, _P]),
        "mgp_synth_generate": (ctypes.c_int, [_U64, _U64, _U32, _U32, _U32, _P, _P, _P, _P, _P, _P, _P]),
        "mgp_synth_set_ablate": (ctypes.c_int, [ctypes.c_int]),
        "mgp_nominal_ops": (ctypes.c_int, [_P, _P, _U32, _P]),
        "mgp_probe_valu_dev": (ctypes.c_int, [_U32, _U32, _P, _P, _P]),
        "mgp_set_eval_engine": (ctypes.c_int, [ctypes.c_int]),
        "mgp_set_keccak_engine": (ctypes.c_int, [ctypes.c_int]),
        "mgp_set_thread_omp": (ctypes.c_int, [ctypes.c_int]),
        "mgp_set_eval_diag": (ctypes.c_int, [_P]),
        "mgp_refute": (ctypes.c_int, [_P, _P, _U32, _P, _P, _U32, _P]),
        "mgp_refute_split": (ctypes.c_int, [_P, _P, _U32, _P, _P, _U32, _U32, _P]),
        "mgp_refute_cores": (ctypes.c_int, [_P, _P, _U32, _P, _P, _P, _U32, _U32, _U32, _P, _P]),
        "mgp_refute_trace": (ctypes.c_int, [_P, _U64, _P, _U64, _U32, _P]),
        "mgp_guided_candidates": (ctypes.c_int, [_P, _P, _U32, _P, _P, _U32, _U32, _U32, _U64, _U32, _U32, _P, _P]),
        "mgp_guided_candidates_rows": (ctypes.c_int, [_P, _P, _U32, _P, _P, _U32, _U32, _U32, _U64, _U32, _U32, _P, _P,
                                                      _P]),
        "mgp_make_candidates": (ctypes.c_int, [_U32, _U32, _U32, _U64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _U32,
                                               _P, _P, _P, _P]),
        "mgp_decision_rows": (ctypes.c_int, [_P, _P, _U32, _P, _P, _U32, _U32, _U64, _P, _U32, _P, _P, _P, _P]),
        "mgp_decision_rows_seeded": (ctypes.c_int, [_P, _P, _U32, _P, _P, _U32, _U32, _U64, _P, _U32, _P, _P, _P,
                                                    _U32, _P, _P, _P]),
        "mgp_decision_rows_from": (ctypes.c_int, [_P, _P, _U32, _P, _P, _U32, _U32, _U64, _P, _U32, _U32, _P, _P,
                                                  _P, _U32, _P, _P, _P]),
        "mgp_refute_domains": (ctypes.c_int, [_P, _P, _U32, _P, _P, _P, _U32, _P, _P]),
        "mgp_build_states": (ctypes.c_int, [_P, _P, _P, _P, _U64, _P, _U64, _P, _P, _U32, _P, _U64,
                                            ctypes.POINTER(_P)]),
        "mgp_fe_get": (ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(_P), ctypes.POINTER(_U64)]),
        "mgp_fe_free": (None, [_P]),
        "mgp_fe_select": (ctypes.c_int, [_P, _P, _U32, ctypes.POINTER(_P)]),
        "mgp_check_submit": (ctypes.c_int, [_P, _P, _U32, _U64, _P, _U32, _P, _P, _P, _P, _P, _P, _U32, _U32, _U32,
                                            _P, _P, _P, _P]),
        "mgp_check_finish": (ctypes.c_int, [_P, _I32, _P, _P, _P]),
        "mgp_pipeline_reserve": (ctypes.c_int, [_P, _U64, _U64]),
        "mgp_check_batch": (ctypes.c_int, [_P, _P, _U32, _U64, _P, _U32, _P, _P, _P, _P, _P, _P, _U32, _U32, _U32,
                                           _P, _P, _P, _P, _P]),
        "mgp_fe_candidates": (ctypes.c_int, [_P, _P, _U32, _U32, _U64, _P, _U32, _P, _P, _P, _U32, _U32, _P]),
        "mgp_program_cache_clear": (_U64, []),
        "mgp_program_cache_warm": (ctypes.c_int, [_P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def lib():
    """Load libmgp.so once; raise NativeUnavailable loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeUnavailable(
                    f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                    "(the GPU pre-filter has no CPU fallback)"
                )
            try:
                _lib = _bind(ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL))
            except OSError as e:  # pragma: no cover - depends on the box
                raise NativeUnavailable(f"cannot load {LIB_PATH}: {e}") from e
    return _lib


EXPORTED_SYMBOLS = (
    "mgp_create",
    "mgp_destroy",
    "mgp_last_error",
    "mgp_device_count",
    "mgp_version",
    "mgp_lower",
    "mgp_eval_batch",
    "mgp_eval_batch_dev",
    "mgp_plan_buckets",
    "mgp_fill_candidates_dev",
    "mgp_plant_candidates_dev",
    "mgp_keccak256_batch",
    "mgp_keccak256_dev",
    "mgp_fill_mapping_preimages_dev",
    "mgp_synth_generate",
    "mgp_synth_set_ablate",
    "mgp_nominal_ops",
    "mgp_probe_valu_dev",
    "mgp_set_eval_engine",
    "mgp_set_keccak_engine",
    "mgp_set_thread_omp",
    "mgp_set_eval_diag",
    "mgp_refute",
    "mgp_refute_split",
    "mgp_refute_cores",
    "mgp_refute_trace",
    "mgp_guided_candidates",
    "mgp_guided_candidates_rows",
    "mgp_make_candidates",
    "mgp_decision_rows",
    "mgp_decision_rows_seeded",
    "mgp_decision_rows_from",
    "mgp_refute_domains",
    "mgp_build_states",
    "mgp_fe_get",
    "mgp_fe_free",
    "mgp_fe_select",
    "mgp_check_batch",
    "mgp_check_submit",
    "mgp_check_finish",
    "mgp_pipeline_reserve",
    "mgp_fe_candidates",
    "mgp_program_cache_clear",
    "mgp_program_cache_warm",
)


def program_cache_warm(batch_handle) -> None:
    """Lower a native front-end batch's GPU programs into the program cache (host only)."""
    _check(lib().mgp_program_cache_warm(batch_handle))


def program_cache_clear() -> int:
    """Empty mgp_check_batch's cache of lowered programs (cold measurements, tests)."""
    return int(lib().mgp_program_cache_clear())


ENGINE_HIP, ENGINE_ASM = 1, 2
ENGINES = {"hip": ENGINE_HIP, "asm": ENGINE_ASM}


def set_eval_engine(name: Optional[str] = None) -> str:
    """Select the evaluation kernel ('asm' = hand-written gfx950 interpreter, default;
    'hip' = HIP C++ interpreter); returns the engine in use."""
    cur = lib().mgp_set_eval_engine(ENGINES[name] if name else 0)
    return {v: k for k, v in ENGINES.items()}[cur]


KECCAK_ENGINES = {"hip": 1, "asm": 2, "asm_dx": 3}


def set_keccak_engine(name: Optional[str] = None) -> str:
    """Select the 64-byte Keccak kernel ('asm' = hand-allocated mgp_keccak64_gfx950,
    default; 'asm_dx' = its theta-through-D variant; 'hip' = compiler-allocated
    mgp_keccak64_kernel); returns the one in use."""
    cur = lib().mgp_set_keccak_engine(KECCAK_ENGINES[name] if name else 0)
    return {v: k for k, v in KECCAK_ENGINES.items()}[cur]


def _ptr(a: Optional[np.ndarray]):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays passed to libmgp must be C-contiguous"
    return ctypes.c_void_p(a.ctypes.data)


def _check(rc: int, ctx=None):
    if rc != MGP_OK:
        msg = lib().mgp_last_error(ctx)
        raise MgpError(rc, msg.decode() if msg else "")


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().mgp_device_count(ctypes.byref(n))
    return n.value if rc == MGP_OK else 0


# ------------------------------------------------------------------ lowering
def lower(
    nodes: np.ndarray,
    node_offsets: np.ndarray,
    consts: np.ndarray,
    const_offsets: np.ndarray,
    max_slots: int = 0,
) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Lower node lists to bytecode -> (words u32, prog_offsets u64, status u8)."""
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    node_offsets = np.ascontiguousarray(node_offsets, dtype=np.uint64)
    consts = np.ascontiguousarray(consts, dtype=np.uint32).reshape(-1)
    if consts.size == 0:
        consts = np.zeros(8, dtype=np.uint32)
    const_offsets = np.ascontiguousarray(const_offsets, dtype=np.uint64)
    n_states = len(node_offsets) - 1
    prog_offsets = np.zeros(n_states + 1, dtype=np.uint64)
    status = np.zeros(max(n_states, 1), dtype=np.uint8)
    used = ctypes.c_uint64(0)
    cap = int(len(nodes)) * 16 + n_states * 64 + 64
    L = lib()
    for _ in range(2):
        words = np.zeros(cap, dtype=np.uint32)
        rc = L.mgp_lower(
            _ptr(nodes), _ptr(node_offsets), n_states, _ptr(consts), _ptr(const_offsets), max_slots,
            _ptr(words), cap, _ptr(prog_offsets), _ptr(status), ctypes.byref(used),
        )
        if rc == MGP_E_CAPACITY:
            cap = int(used.value)
            continue
        _check(rc)
        return words[: int(used.value)], prog_offsets, status[:n_states]
    raise MgpError(MGP_E_CAPACITY, "lowering capacity")


LDS_SLOTS = 32  # include/mgp_ir.h MGP_LDS_SLOTS


def prog_rows(words: np.ndarray, prog_offsets: np.ndarray) -> np.ndarray:
    """Candidate rows each lowered program needs (include/mgp_ir.h MGP_PROG_VARS): the
    variables it reads, plus the spill rows of a program with more live values than
    LDS slots.  A device candidate block for mgp_eval_batch_dev needs the maximum."""
    h = np.asarray(words, dtype=np.uint64)[np.asarray(prog_offsets[:-1], dtype=np.int64)[:, None] + np.arange(4)]
    max_var = h[:, 3] >> np.uint64(8)
    spill = np.maximum(max_var, 8) + h[:, 2] - LDS_SLOTS + 1
    ok = (h[:, 3] & np.uint64(0xFF)) == 0
    return np.where(ok & (h[:, 2] >= LDS_SLOTS), spill, np.where(ok, max_var, 0)).astype(np.int64)


def make_candidates(n_cand: int, n_vars: int, seed: int, var_off, var_width, hint_off, hints, alias_off, aliases,
                    const_off, consts, fixed_pool, has_parent, var_kind=None, dom=None, state_keys=None) -> np.ndarray:
    """mgp_make_candidates over flattened per-state tables -> uint32 [n_states, n_cand, n_vars, 8]
    (state_keys: per-state stream tags, front.Batch.state_key; None = the state index)."""
    def u(a, dt):
        a = np.ascontiguousarray(a, dtype=dt)
        return a if a.size else np.zeros(8, dtype=dt)
    n_states = len(var_off) - 1
    out = np.empty((n_states, n_cand, n_vars, 8), dtype=np.uint32)
    fixed = u(fixed_pool, np.uint32)
    _check(lib().mgp_make_candidates(n_states, n_cand, n_vars, seed & (2 ** 64 - 1), _ptr(u(var_off, np.uint64)),
                                     _ptr(u(var_width, np.uint32)),
                                     None if var_kind is None else _ptr(u(var_kind, np.uint8)),
                                     _ptr(u(hint_off, np.uint64)),
                                     _ptr(u(hints, np.uint32)), _ptr(u(alias_off, np.uint64)),
                                     _ptr(u(aliases, np.uint32)), _ptr(u(const_off, np.uint64)),
                                     _ptr(u(consts, np.uint32)), _ptr(fixed), len(fixed_pool),
                                     _ptr(u(has_parent, np.uint8)),
                                     None if dom is None else _ptr(np.ascontiguousarray(dom, dtype=np.uint32)),
                                     None if state_keys is None else _ptr(np.ascontiguousarray(state_keys, np.uint64)),
                                     _ptr(out)))
    return out


def decision_rows(nodes, node_offsets, consts, const_offsets, n_vars: int, seed: int, n_decide: int,
                  rows_per_state: Optional[np.ndarray] = None, state_keys: Optional[np.ndarray] = None,
                  max_passes: int = 0, seeds=None, seed_rows: int = 0, row0: int = 0):
    """mgp_decision_rows -> (rows u32 [n, n_decide, n_vars, 8], mask u8 [n, n_decide, n_vars], status i8[n]);
    seeds = (vals u32
    [n, n_vars, 8], mask u8 [n, n_vars]): parent values the rows in `seed_rows` (a bit mask)
    fix first (mgp_decision_rows_seeded); row0 > 0: output row k is decision row row0 + k
    (mgp_decision_rows_from)."""
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    node_offsets = np.ascontiguousarray(node_offsets, dtype=np.uint64)
    consts = np.ascontiguousarray(consts, dtype=np.uint32).reshape(-1)
    if consts.size == 0:
        consts = np.zeros(8, dtype=np.uint32)
    const_offsets = np.ascontiguousarray(const_offsets, dtype=np.uint64)
    n_states = len(node_offsets) - 1
    rows = np.zeros((n_states, n_decide, n_vars, 8), np.uint32)
    mask = np.zeros((n_states, n_decide, n_vars), np.uint8)
    out = np.zeros(max(n_states, 1), np.int8)
    rps = None
    if rows_per_state is not None:
        rps = np.ascontiguousarray(np.minimum(rows_per_state, 255), dtype=np.uint8)
        if rps.shape != (n_states,):
            raise ValueError("rows_per_state must hold one entry per state")
    keys = None if state_keys is None else np.ascontiguousarray(state_keys, dtype=np.uint64)
    if keys is not None and keys.shape != (n_states,):
        raise ValueError("state_keys must hold one entry per state")
    args = (_ptr(nodes), _ptr(node_offsets), n_states, _ptr(consts), _ptr(const_offsets), max_passes, n_vars,
            seed & (2 ** 64 - 1), _ptr(keys), n_decide, _ptr(rps), _ptr(rows) if rows.size else None,
            _ptr(mask) if mask.size else None, _ptr(out))
    if seeds is not None or row0:
        sv = sm = None
        if seeds is not None:
            sv = np.ascontiguousarray(seeds[0], dtype=np.uint32)
            sm = np.ascontiguousarray(seeds[1], dtype=np.uint8)
            if sv.shape != (n_states, n_vars, 8) or sm.shape != (n_states, n_vars):
                raise ValueError("seeds must be (vals u32 [n_states, n_vars, 8], mask u8 [n_states, n_vars])")
        sa = (None if sv is None else _ptr(sv), None if sm is None else _ptr(sm), seed_rows)
        if row0:
            _check(lib().mgp_decision_rows_from(*(args[:9] + (int(row0),) + args[9:11] + sa + args[11:])))
        else:
            _check(lib().mgp_decision_rows_seeded(*(args[:11] + sa + args[11:])))
        return rows, mask, out[:n_states]
    _check(lib().mgp_decision_rows(*args))
    return rows, mask, out[:n_states]


def refute_domains(nodes, node_offsets, consts, const_offsets, var_off, max_passes: int = 0):
    """mgp_refute + per-slot refined abstract values -> (status int8[n], dom uint32[n_slots, 33])."""
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    node_offsets = np.ascontiguousarray(node_offsets, dtype=np.uint64)
    consts = np.ascontiguousarray(consts, dtype=np.uint32).reshape(-1)
    if consts.size == 0:
        consts = np.zeros(8, dtype=np.uint32)
    const_offsets = np.ascontiguousarray(const_offsets, dtype=np.uint64)
    var_off = np.ascontiguousarray(var_off, dtype=np.uint64)
    n_states = len(node_offsets) - 1
    out = np.zeros(max(n_states, 1), dtype=np.int8)
    dom = np.zeros((max(int(var_off[-1]), 1), 33), dtype=np.uint32)
    _check(lib().mgp_refute_domains(_ptr(nodes), _ptr(node_offsets), n_states, _ptr(consts), _ptr(const_offsets),
                                    _ptr(var_off), max_passes, _ptr(out), _ptr(dom)))
    return out[:n_states], dom[: int(var_off[-1])]


def guided_candidates(nodes: np.ndarray, node_offsets: np.ndarray, consts: np.ndarray, const_offsets: np.ndarray,
                      cands: np.ndarray, seed: int = 0x4D595448, every: int = 2, n_decide: int = 16,
                      max_passes: int = 0, rows_per_state: Optional[np.ndarray] = None) -> np.ndarray:
    """Overwrite rows 0, every, 2*every, ... of cands (uint32 [n_states, n_cand, n_vars, 8], in place)
    with draws from each variable's refined abstract value, the first n_decide of them by
    decisions (include/mgp.h); -> int8 status per state as refute()."""
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    node_offsets = np.ascontiguousarray(node_offsets, dtype=np.uint64)
    consts = np.ascontiguousarray(consts, dtype=np.uint32).reshape(-1)
    if consts.size == 0:
        consts = np.zeros(8, dtype=np.uint32)
    const_offsets = np.ascontiguousarray(const_offsets, dtype=np.uint64)
    n_states = len(node_offsets) - 1
    if cands.dtype != np.uint32 or not cands.flags.c_contiguous or cands.ndim != 4 or cands.shape[0] != n_states \
            or cands.shape[3] != 8:
        raise ValueError("cands must be a C-contiguous uint32 [n_states, n_cand, n_vars, 8] array")
    out = np.zeros(max(n_states, 1), dtype=np.int8)
    if rows_per_state is None:
        _check(lib().mgp_guided_candidates(_ptr(nodes), _ptr(node_offsets), n_states, _ptr(consts),
                                           _ptr(const_offsets), max_passes, cands.shape[1], cands.shape[2],
                                           seed & (2 ** 64 - 1), every, n_decide, _ptr(cands), _ptr(out)))
    else:
        rows = np.ascontiguousarray(np.minimum(rows_per_state, 255), dtype=np.uint8)
        if rows.shape != (n_states,):
            raise ValueError("rows_per_state must hold one entry per state")
        _check(lib().mgp_guided_candidates_rows(_ptr(nodes), _ptr(node_offsets), n_states, _ptr(consts),
                                                _ptr(const_offsets), max_passes, cands.shape[1], cands.shape[2],
                                                seed & (2 ** 64 - 1), every, n_decide, _ptr(rows), _ptr(cands),
                                                _ptr(out)))
    return out[:n_states]


def refute(nodes: np.ndarray, node_offsets: np.ndarray, consts: np.ndarray, const_offsets: np.ndarray,
           max_passes: int = 0) -> np.ndarray:
    """Sound UNSAT pre-check per state -> int8 (1 proven UNSAT, 0 not refuted, -1 not analysed)."""
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    node_offsets = np.ascontiguousarray(node_offsets, dtype=np.uint64)
    consts = np.ascontiguousarray(consts, dtype=np.uint32).reshape(-1)
    if consts.size == 0:
        consts = np.zeros(8, dtype=np.uint32)
    const_offsets = np.ascontiguousarray(const_offsets, dtype=np.uint64)
    n_states = len(node_offsets) - 1
    out = np.zeros(max(n_states, 1), dtype=np.int8)
    _check(lib().mgp_refute(_ptr(nodes), _ptr(node_offsets), n_states, _ptr(consts), _ptr(const_offsets),
                            max_passes, _ptr(out)))
    return out[:n_states]


def refute_split(nodes: np.ndarray, node_offsets: np.ndarray, consts: np.ndarray, const_offsets: np.ndarray,
                 max_splits: int = 8, max_passes: int = 0, depth: int = 1, bisect: bool = True) -> np.ndarray:
    """refute + case splits on open select conditions (mgp_refute_split): at most
    max_splits conditions per state, nested `depth` levels (1..15); then (bisect) interval
    bisection of bounded variables."""
    if not 0 <= max_splits < (1 << 16) or not 1 <= depth <= 15:
        raise ValueError(f"refute_split: max_splits {max_splits} / depth {depth} out of range")
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    node_offsets = np.ascontiguousarray(node_offsets, dtype=np.uint64)
    consts = np.ascontiguousarray(consts, dtype=np.uint32).reshape(-1)
    if consts.size == 0:
        consts = np.zeros(8, dtype=np.uint32)
    const_offsets = np.ascontiguousarray(const_offsets, dtype=np.uint64)
    n_states = len(node_offsets) - 1
    out = np.zeros(max(n_states, 1), dtype=np.int8)
    _check(lib().mgp_refute_split(_ptr(nodes), _ptr(node_offsets), n_states, _ptr(consts), _ptr(const_offsets),
                                  max_passes, max_splits | (depth << 16) | (0 if bisect else 1 << 20), _ptr(out)))
    return out[:n_states]


def refute_cores(nodes: np.ndarray, node_offsets: np.ndarray, consts: np.ndarray, const_offsets: np.ndarray,
                 n_roots: np.ndarray, max_passes: int = 0, halvings: int = 3, max_single: int = 32):
    """mgp_refute_cores: the core of each refuted constraint list whose DAG these are (the
    lists' constraint counts in n_roots) -> (list of u8 keep masks, status i8 [n])."""
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    node_offsets = np.ascontiguousarray(node_offsets, dtype=np.uint64)
    consts = np.ascontiguousarray(consts, dtype=np.uint32).reshape(-1)
    if consts.size == 0:
        consts = np.zeros(8, dtype=np.uint32)
    const_offsets = np.ascontiguousarray(const_offsets, dtype=np.uint64)
    n_roots = np.ascontiguousarray(n_roots, dtype=np.uint32)
    n_states = len(node_offsets) - 1
    if n_roots.shape != (n_states,):
        raise ValueError("n_roots must hold one count per state")
    keep = np.zeros(max(int(n_roots.sum()), 1), dtype=np.uint8)
    out = np.zeros(max(n_states, 1), dtype=np.int8)
    _check(lib().mgp_refute_cores(_ptr(nodes), _ptr(node_offsets), n_states, _ptr(consts), _ptr(const_offsets),
                                  _ptr(n_roots), max_passes, halvings, max_single, _ptr(keep), _ptr(out)))
    off = np.concatenate([[0], np.cumsum(n_roots)]).astype(np.int64)
    return [keep[off[k]:off[k + 1]] for k in range(n_states)], out[:n_states]


def refute_trace(nodes: np.ndarray, consts: np.ndarray, max_passes: int = 0):
    """One state's refined abstract values -> (verdict, (n_nodes, 33) u32 array)."""
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    consts = np.ascontiguousarray(consts, dtype=np.uint32).reshape(-1)
    if consts.size == 0:
        consts = np.zeros(8, dtype=np.uint32)
    out = np.zeros((max(len(nodes), 1), 33), dtype=np.uint32)
    r = lib().mgp_refute_trace(_ptr(nodes), len(nodes), _ptr(consts), consts.size // 8, max_passes, _ptr(out))
    return int(r), out[: len(nodes)]


def program_headers(words: np.ndarray, prog_offsets: np.ndarray) -> np.ndarray:
    """(n_states, 4) header words: n_ins, n_consts, n_slots, status|vars<<8."""
    idx = prog_offsets[:-1].astype(np.int64)
    return np.stack([words[idx + k] for k in range(4)], axis=1)


# ------------------------------------------------------------------ context
class Context:
    """One libmgp context (device + HIP stream + device buffers)."""

    def __init__(self, device: int = 0):
        self._h = ctypes.c_void_p()
        _check(lib().mgp_create(device, ctypes.byref(self._h)))
        self.device = device

    def close(self):
        if self._h:
            lib().mgp_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def eval_batch(self, words, prog_offsets, cands: np.ndarray, want_witness: bool = True):
        """cands: uint32 [n_states, n_cand, n_vars, 8].  -> (first_sat i32, witness u32 [n,n_vars,8])."""
        words = np.ascontiguousarray(words, dtype=np.uint32)
        prog_offsets = np.ascontiguousarray(prog_offsets, dtype=np.uint64)
        cands = np.ascontiguousarray(cands, dtype=np.uint32)
        n_states, n_cand, n_vars, limbs = cands.shape
        assert limbs == 8 and len(prog_offsets) == n_states + 1
        first = np.full(n_states, MGP_NO_SAT, dtype=np.int32)
        wit = np.zeros((n_states, n_vars, 8), dtype=np.uint32) if want_witness else None
        rc = lib().mgp_eval_batch(
            self._h, _ptr(words), _ptr(prog_offsets), n_states, _ptr(cands), n_cand, n_vars,
            _ptr(first), _ptr(wit),
        )
        _check(rc, self._h)
        return first, wit

    def reserve(self, host_bytes: int, cand_bytes: int) -> None:
        """mgp_pipeline_reserve: size the pipeline's pinned staging and candidate block now."""
        _check(lib().mgp_pipeline_reserve(self._h, int(host_bytes), int(cand_bytes)), self._h)

    def check_batch(self, batch, n_cand: int, seed: int, parents=None, refute: bool = True, xrows=None):
        """A front-end batch (mythril_amd.front.Batch) through mgp_check_batch."""
        return batch._check_native(self, n_cand, seed, parents, refute, xrows)

    def submit_batch(self, batch, n_cand: int, seed: int, parents=None, refute: bool = True, xrows=None):
        """mgp_check_submit: the host stages of check_batch now, the GPU round enqueued; ->
        front.PendingRound (finish() = mgp_check_finish).  At most two in flight."""
        return batch._submit_native(self, n_cand, seed, parents, refute, xrows)

    def keccak256(self, data: np.ndarray, length: int, stride: int) -> np.ndarray:
        data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        n = 0 if stride == 0 else (len(data) - length) // stride + 1 if len(data) >= length else 0
        return self.keccak256_n(data, n, length, stride)

    def keccak256_n(self, data: np.ndarray, n: int, length: int, stride: int) -> np.ndarray:
        data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        if n and len(data) < (n - 1) * stride + length:
            raise ValueError("input buffer too small")
        out = np.zeros((n, 32), dtype=np.uint8)
        if n == 0:
            return out
        if data.size == 0:
            data = np.zeros(1, dtype=np.uint8)
        _check(lib().mgp_keccak256_batch(self._h, _ptr(data), n, length, stride, _ptr(out)), self._h)
        return out


# ------------------------------------------------------------- synthetic
SYNTH_VARS = 6


def synth_set_ablate(mode: int) -> None:
    """mgp_synth_set_ablate: 0 none, 1 divisions drawn as ADD, 2 MUL, 3 both."""
    _check(lib().mgp_synth_set_ablate(int(mode)))


def synth_generate(seed: int, state_base: int, n_states: int, n_nodes: int = 64, n_cand: int = 256):
    """Synthetic DAG batch -> dict(nodes, node_offsets, consts, const_offsets, planted, plant_idx, plant_words)."""
    stride = n_nodes + 32
    nodes = np.zeros(n_states * stride, dtype=NODE_DTYPE)
    node_offsets = np.zeros(n_states + 1, dtype=np.uint64)
    consts = np.zeros((n_states * 16, 8), dtype=np.uint32)
    const_offsets = np.zeros(n_states + 1, dtype=np.uint64)
    planted = np.zeros(n_states, dtype=np.uint8)
    plant_idx = np.zeros(n_states, dtype=np.uint32)
    plant_words = np.zeros((n_states, SYNTH_VARS, 8), dtype=np.uint32)
    _check(
        lib().mgp_synth_generate(
            seed, state_base, n_states, n_nodes, n_cand, _ptr(nodes), _ptr(node_offsets), _ptr(consts),
            _ptr(const_offsets), _ptr(planted), _ptr(plant_idx), _ptr(plant_words),
        )
    )
    return {
        "nodes": nodes[: int(node_offsets[-1])],
        "node_offsets": node_offsets,
        "consts": consts[: int(const_offsets[-1])],
        "const_offsets": const_offsets,
        "planted": planted,
        "plant_idx": plant_idx,
        "plant_words": plant_words,
        "n_vars": SYNTH_VARS,
    }


def nominal_ops(nodes: np.ndarray, node_offsets: np.ndarray) -> np.ndarray:
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    node_offsets = np.ascontiguousarray(node_offsets, dtype=np.uint64)
    n = len(node_offsets) - 1
    out = np.zeros(max(n, 1), dtype=np.uint64)
    _check(lib().mgp_nominal_ops(_ptr(nodes), _ptr(node_offsets), n, _ptr(out)))
    return out[:n]


# ---------------------------------------------------- device-pointer API
def plan_buckets(words: np.ndarray, prog_offsets: np.ndarray, max_buckets: int = 256):
    """-> (order u32[n], bounds u32[nb+1], slots u32[nb]) grouping states by LDS slot count."""
    words = np.ascontiguousarray(words, dtype=np.uint32)
    prog_offsets = np.ascontiguousarray(prog_offsets, dtype=np.uint64)
    n = len(prog_offsets) - 1
    order = np.zeros(max(n, 1), dtype=np.uint32)
    bounds = np.zeros(max_buckets + 1, dtype=np.uint32)
    slots = np.zeros(max_buckets, dtype=np.uint32)
    nb = lib().mgp_plan_buckets(_ptr(words), _ptr(prog_offsets), n, _ptr(order), _ptr(bounds), _ptr(slots),
                                max_buckets)
    if nb < 0:
        _check(nb)
    return order[:n], bounds[: nb + 1].copy(), slots[:nb].copy()


def eval_batch_dev(d_words, d_offs, n_states, d_cands, n_cand, n_vars, n_slots, d_first, d_wit, d_scratch,
                   stream, d_order=None, bounds: Optional[np.ndarray] = None, slots: Optional[np.ndarray] = None) -> None:
    nb = 0 if bounds is None else len(slots)
    _check(
        lib().mgp_eval_batch_dev(
            d_words, d_offs, n_states, d_cands, n_cand, n_vars, n_slots, d_first, d_wit, d_scratch, d_order,
            _ptr(bounds) if nb else None, _ptr(slots) if nb else None, nb, stream
        )
    )


def fill_candidates_dev(d_words, d_offs, n_states, state_base, seed, d_cands, n_cand, n_vars, stream) -> None:
    _check(lib().mgp_fill_candidates_dev(d_words, d_offs, n_states, state_base, seed, d_cands, n_cand, n_vars,
                                         stream))


def plant_candidates_dev(d_cands, n_states, n_cand, n_vars, d_pstate, d_pidx, d_pwords, n_plant, stream) -> None:
    _check(lib().mgp_plant_candidates_dev(d_cands, n_states, n_cand, n_vars, d_pstate, d_pidx, d_pwords, n_plant,
                                          stream))


def keccak256_dev(d_in, n, length, stride, d_out, stream) -> None:
    _check(lib().mgp_keccak256_dev(d_in, n, length, stride, d_out, stream))


def fill_mapping_preimages_dev(d_out, first, n, seed, stream) -> None:
    _check(lib().mgp_fill_mapping_preimages_dev(d_out, first, n, seed, stream))


def probe_valu_dev(iters, blocks, d_sink, stream) -> int:
    ops = ctypes.c_uint64(0)
    _check(lib().mgp_probe_valu_dev(iters, blocks, d_sink, ctypes.byref(ops), stream))
    return int(ops.value)
