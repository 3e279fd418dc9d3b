"""Shared helpers for the parity tests (tests only)."""
from __future__ import annotations

import json
import os
from typing import List, Sequence, Tuple

import numpy as np

from mythril_amd import _native as N
from oracle import bvsem as S

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def node_array(nodes: Sequence[Sequence[int]]) -> np.ndarray:
    arr = np.zeros(len(nodes), dtype=N.NODE_DTYPE)
    for i, (op, w, a, b, c, p0, p1) in enumerate(nodes):
        arr[i] = (op, 0, w, a, b, c, p0, p1)
    return arr


def pack_states(states: List[Tuple[Sequence[Sequence[int]], Sequence[int]]]):
    """states: list of (node list, const ints) -> (nodes, node_offsets, consts u32[n,8], const_offsets)."""
    nodes, noff, consts, coff = [], [0], [], [0]
    for nl, cl in states:
        nodes.append(node_array(nl))
        noff.append(noff[-1] + len(nl))
        for c in cl:
            consts.append(S.int_to_limbs(int(c)))
        coff.append(coff[-1] + len(cl))
    nodes = np.concatenate(nodes) if nodes else np.zeros(0, dtype=N.NODE_DTYPE)
    consts = np.array(consts, dtype=np.uint32).reshape(-1, 8) if consts else np.zeros((0, 8), dtype=np.uint32)
    return nodes, np.array(noff, dtype=np.uint64), consts, np.array(coff, dtype=np.uint64)


def state_slice(batch, s: int):
    n0, n1 = int(batch["node_offsets"][s]), int(batch["node_offsets"][s + 1])
    c0, c1 = int(batch["const_offsets"][s]), int(batch["const_offsets"][s + 1])
    nodes = batch["nodes"][n0:n1]
    consts = [S.limbs_to_int(c) for c in batch["consts"][c0:c1]]
    return nodes, consts


def cands_from_ints(rows: Sequence[Sequence[Sequence[int]]]) -> np.ndarray:
    """rows[state][cand][var] ints -> uint32 [n_states, n_cand, n_vars, 8]."""
    n_s, n_c, n_v = len(rows), len(rows[0]), len(rows[0][0])
    out = np.zeros((n_s, n_c, n_v, 8), dtype=np.uint32)
    for s in range(n_s):
        for c in range(n_c):
            for v in range(n_v):
                out[s, c, v] = S.int_to_limbs(int(rows[s][c][v]))
    return out


INTERESTING = [0, 1, 2, (1 << 256) - 1, 1 << 255, (1 << 255) - 1, (1 << 160) - 1, 1 << 128,
               0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF, 0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE,
               (1 << 256) - 2, 255, 256, 257, 31, 32, 0xFFFFFFFF, 1 << 32, 1 << 64]


def random_cands(rng: np.random.Generator, n_states: int, n_cand: int, n_vars: int,
                 interesting_frac: float = 0.3) -> np.ndarray:
    c = rng.integers(0, 2 ** 32, size=(n_states, n_cand, n_vars, 8), dtype=np.uint64).astype(np.uint32)
    pick = rng.random((n_states, n_cand, n_vars)) < interesting_frac
    idx = rng.integers(0, len(INTERESTING), size=(n_states, n_cand, n_vars))
    table = np.array([S.int_to_limbs(v) for v in INTERESTING], dtype=np.uint32)
    c[pick] = table[idx[pick]]
    return c
