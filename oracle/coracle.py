"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE / CPU BASELINE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P, U32, U64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        L.oracle_first_sat.argtypes = [P, P, U32, P, P, P, U32, U32, P, ctypes.c_int]
        L.oracle_first_sat.restype = ctypes.c_int
        L.oracle_keccak256.argtypes = [P, U64, U32, U32, P]
        L.oracle_keccak256.restype = ctypes.c_int
        L.oracle_mapping_preimages.argtypes = [P, U64, U64, U64]
        L.oracle_mapping_preimages.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def first_sat(nodes, node_offsets, consts, const_offsets, cands, full=False) -> np.ndarray:
    """cands uint32 [n_states, n_cand, n_vars, 8] (host AoS)."""
    nodes = np.ascontiguousarray(nodes)
    node_offsets = np.ascontiguousarray(node_offsets, dtype=np.uint64)
    consts = np.ascontiguousarray(consts, dtype=np.uint32).reshape(-1)
    if consts.size == 0:
        consts = np.zeros(8, dtype=np.uint32)
    const_offsets = np.ascontiguousarray(const_offsets, dtype=np.uint64)
    cands = np.ascontiguousarray(cands, dtype=np.uint32)
    n_states, n_cand, n_vars, _ = cands.shape
    out = np.zeros(n_states, dtype=np.int32)
    lib().oracle_first_sat(_p(nodes), _p(node_offsets), n_states, _p(consts), _p(const_offsets), _p(cands),
                           n_cand, n_vars, _p(out), 1 if full else 0)
    return out


def keccak256(data: np.ndarray, n: int, length: int, stride: int) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    if data.size == 0:
        data = np.zeros(1, dtype=np.uint8)
    out = np.zeros((n, 32), dtype=np.uint8)
    lib().oracle_keccak256(_p(data), n, length, stride, _p(out))
    return out


def mapping_preimages(first: int, n: int, seed: int) -> np.ndarray:
    out = np.zeros((n, 64), dtype=np.uint8)
    lib().oracle_mapping_preimages(_p(out), first, n, seed)
    return out
