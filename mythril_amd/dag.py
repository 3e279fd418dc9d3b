"""Terms -> per-state constraint DAGs (include/mgp_ir.h node lists) and candidates.

`build_state` flattens the conjunction of a state's path constraints
(mythril/laser/ethereum/state/constraints.py:10-126 holds them as a list of
Bool) into a topologically ordered node list with a constant pool and a
variable table.  Every uninterpreted-function application (keccak256_<n>,
its inverse, base-array selects) gets a fresh candidate variable — the
Ackermann encoding the HIP path evaluates (mgp_lower.cpp).

`make_candidates` builds the candidate assignments one state is evaluated on:
the parent state's witness first (a successor only adds constraints to its
parent, svm.py:251-255 / instructions.py:1533-1610), then assignments
harvested from the DAG's own constants (x == c, x +- 1 around compared
constants, LASER's actor addresses transaction/symbolic.py:22-27, keccak
interval bases keccak_function_manager.py:118-146), then uniform values.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import ir
from ._native import NODE_DTYPE
from .smt import Term

ACTORS = (0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE, 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,
          0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA)
SPECIAL = (0, 1, 2, (1 << 256) - 1, 1 << 255, (1 << 160) - 1, 10 ** 18, 10 ** 20)


@dataclass
class StateDag:
    nodes: List[Tuple[int, int, int, int, int, int, int]] = field(default_factory=list)
    consts: List[int] = field(default_factory=list)
    vars: List[Tuple[str, int]] = field(default_factory=list)  # (name, width); index = var index
    var_terms: List[Optional[Term]] = field(default_factory=list)
    hints: Dict[int, List[int]] = field(default_factory=dict)  # var index -> harvested values
    aliases: List[Tuple[int, int]] = field(default_factory=list)  # (dst var, src var) from x == y
    # wide values (> 256 bits, include/mgp_ir.h): first slot -> full width; the value
    # occupies ceil(width/256) consecutive var slots / pool entries, low 256 bits first
    wide: Dict[int, int] = field(default_factory=dict)
    # padded key equalities (csrc/mgp_front.cpp): node index -> TRUE/FALSE op in the GPU
    # program; flags bit 0 = such an equality under both polarities (no GPU SAT answer)
    gpu_ops: Dict[int, int] = field(default_factory=dict)  # node -> TRUE / FALSE
    flags: int = 0
    # pinned constants (csrc/mgp_front.cpp pin_constants): var slots of the GPU program
    # holding a pool constant in every candidate row
    pinned: Dict[int, int] = field(default_factory=dict)  # slot -> value
    gpu_nodes: Optional[List[Tuple[int, int, int, int, int, int, int]]] = None  # when it differs from nodes

    @property
    def n_vars(self) -> int:
        return len(self.vars)


def build_state(constraints: Sequence[Term]) -> StateDag:
    """Flatten And(constraints) into a StateDag (root = last node, Bool)."""
    d = StateDag()
    memo: Dict[int, int] = {}
    var_idx: Dict[Tuple[str, int], int] = {}
    const_idx: Dict[Tuple[int, int], int] = {}

    def new_var(name: str, width: int, term: Optional[Term]) -> int:
        key = (name, width)
        if key not in var_idx:
            var_idx[key] = len(d.vars)
            if width > 256:
                d.wide[len(d.vars)] = width
            for j, off in enumerate(range(0, width, 256)):
                d.vars.append((name if j == 0 else f"{name}#{j}", min(256, width - off)))
                d.var_terms.append(term if j == 0 else None)
        return var_idx[key]

    def emit(t: Term) -> int:
        ch = [memo[id(a)] for a in t.args]
        a, b, c = (ch + [-1, -1, -1])[:3]
        w = 1 if t.width == 0 else t.width
        p0 = p1 = 0
        op = t.op
        if op == ir.VAR:
            p0 = new_var(str(t.params[0]), w, t)
        elif op == ir.CONST:
            v = t.params[0]
            k = (w + 255) // 256
            if (v, k) not in const_idx:
                const_idx[(v, k)] = len(d.consts)
                d.consts.extend((v >> (256 * j)) & ((1 << 256) - 1) for j in range(k))
            p0 = const_idx[(v, k)]
        elif op == ir.EXTRACT:
            p0, p1 = t.params
        elif op in (ir.UFAPP, ir.UFINV):
            fid, name = t.params
            p0 = fid
            p1 = new_var(f"{name}@{len(d.nodes)}", w, None)
        d.nodes.append((op, w, a, b, c, p0, p1))
        return len(d.nodes) - 1

    roots: List[int] = []
    for root in constraints:
        stack: List[Tuple[Term, bool]] = [(root, False)]
        while stack:
            t, done = stack.pop()
            if id(t) in memo:
                continue
            if done:
                memo[id(t)] = emit(t)
                continue
            stack.append((t, True))
            for a in reversed(t.args):
                if id(a) not in memo:
                    stack.append((a, False))
        roots.append(memo[id(root)])
    if not roots:
        d.nodes.append((ir.TRUE, 1, -1, -1, -1, 0, 0))
    else:
        r = roots[0]
        for x in roots[1:]:
            d.nodes.append((ir.BAND, 1, r, x, -1, 0, 0))
            r = len(d.nodes) - 1
        if r != len(d.nodes) - 1:  # root must be the last node
            d.nodes.append((ir.BAND, 1, r, r, -1, 0, 0))
    _harvest_hints(d)
    _strengthen_padded(d)
    _pin_constants(d)
    if d.gpu_ops and d.gpu_nodes is None:
        d.gpu_nodes = list(d.nodes)
    if d.gpu_ops:
        shift = len(d.gpu_nodes) - len(d.nodes)
        for i, op in d.gpu_ops.items():
            d.gpu_nodes[shift + i] = (op, 1, -1, -1, -1, 0, 0)
    return d


POOL_KEEP = 48  # include/mgp.h MGP_FE_POOL_KEEP


def _pin_constants(d: StateDag) -> None:
    """Pool entries from POOL_KEEP on are pinned in the GPU program (csrc/mgp_front.cpp
    pin_constants; the gfx950 interpreter holds <= 64 constants): operand uses other than
    a UF argument read a VAR node placed in front of the program, of a pinned slot."""
    if len(d.consts) <= POOL_KEEP:
        return
    nodes = d.nodes
    pinned = [n[0] == ir.CONST and n[5] + (n[1] + 255) // 256 > POOL_KEEP for n in nodes]
    if not any(pinned):
        return
    other = [False] * len(nodes)
    for (op, w, a, b, c, p0, p1) in nodes:
        for k, x in enumerate((a, b, c)):
            if x < 0 or not pinned[x] or (k == 0 and op in (ir.UFAPP, ir.UFINV)):
                continue
            other[x] = True
    slot_of: Dict[int, int] = {}
    front: Dict[int, int] = {}
    pre = []
    for i, (op, w, a, b, c, p0, p1) in enumerate(nodes):
        if not other[i]:
            continue
        k = (w + 255) // 256
        if p0 not in slot_of:
            slot_of[p0] = len(d.vars)
            if k > 1:
                d.wide[len(d.vars)] = w
            for j in range(k):
                d.pinned[len(d.vars)] = d.consts[p0 + j]
                d.hints[len(d.vars)] = [d.consts[p0 + j]]
                d.vars.append((f"#pool{p0}" if j == 0 else f"#pool{p0}#{j}", min(256, w - 256 * j)))
                d.var_terms.append(None)
        front[i] = len(pre)
        pre.append((ir.VAR, w, -1, -1, -1, slot_of[p0], 0))
    if not pre:
        return
    P = len(pre)
    out = list(pre)
    for (op, w, a, b, c, p0, p1) in nodes:
        ops = []
        for k, x in enumerate((a, b, c)):
            if x < 0:
                ops.append(x)
            elif x in front and not (k == 0 and op in (ir.UFAPP, ir.UFINV)):
                ops.append(front[x])
            else:
                ops.append(x + P)
        out.append((op, w, ops[0], ops[1], ops[2], p0, p1))
    d.gpu_nodes = out
    d.flags |= 4


def _is_padded_eq(nodes, n) -> bool:
    """EQ(ZEXT(CONST), x) with x not constant: a narrower constant key compared with a
    wider value (bitvec.py:16-22, keccak_function_manager.py:141-145)."""
    op, w, a, b = n[0], n[1], n[2], n[3]
    if op != ir.EQ or a < 0 or b < 0:
        return False

    def zc(x):
        return nodes[x][0] == ir.ZEXT and nodes[x][2] >= 0 and nodes[nodes[x][2]][0] == ir.CONST

    return (zc(a) and nodes[b][0] != ir.CONST) or (zc(b) and nodes[a][0] != ir.CONST)


def _strengthen_padded(d: StateDag) -> None:
    """Polarity of every padded key equality from the root; positive -> FALSE, negative ->
    TRUE in the GPU program (a stronger formula: its witnesses are models with or without
    those disjuncts), both -> flags |= 1 (csrc/mgp_front.cpp explains why)."""
    nodes = d.nodes
    if not any(_is_padded_eq(nodes, n) for n in nodes):
        return
    pol = [0] * len(nodes)
    pol[-1] = 1
    for i in range(len(nodes) - 1, -1, -1):
        p = pol[i]
        if not p:
            continue
        op, _, a, b, c = nodes[i][:5]
        if op in (ir.BAND, ir.BOR):
            for x in (a, b):
                if x >= 0:
                    pol[x] |= p
        elif op == ir.BNOT:
            pol[a] |= ((p & 1) << 1) | (p >> 1)
        elif op in (ir.BXOR, ir.BEQ):
            pol[a] |= 3
            pol[b] |= 3
        elif op == ir.BITE:
            pol[a] |= 3
            pol[b] |= p
            pol[c] |= p
        else:
            # a node the pass does not model (a compare, a BV ITE, a BV operator, a UF
            # application): its operands -- a padded equality under If(eq, 1, 0) == 1,
            # the shape LASER's EQ / ISZERO build -- are reached with both polarities
            for x in (a, b, c):
                if x >= 0:
                    pol[x] |= 3
    for i, n in enumerate(nodes):
        if pol[i] and _is_padded_eq(nodes, n):
            if pol[i] == 3:
                d.flags |= 1
            else:
                d.gpu_ops[i] = ir.FALSE if pol[i] == 1 else ir.TRUE
                d.flags |= 2


def _var_of(nodes, x) -> int:
    op = nodes[x][0]
    if op == ir.VAR:
        return nodes[x][5]
    if op in (ir.UFAPP, ir.UFINV):
        return nodes[x][6]
    return -1


def _harvest_hints(d: StateDag) -> None:
    """x == c -> x := c ; x <op> c -> c-1, c, c+1 and 64-aligned neighbours (keccak
    intervals, keccak_function_manager.py:135-140) ; x == y -> alias pair."""
    nodes = d.nodes
    for (op, w, a, b, c, p0, p1) in nodes:
        if a < 0 or b < 0:
            continue
        if op in (ir.MUL, ir.UMUL_NOOVF):
            # wrap hints: x * c -> floor((2^w-1)/c) and +1 (csrc/mgp_front.cpp wrap_hints)
            wa = nodes[a][1]
            for x, y in ((a, b), (b, a)):
                vi = _var_of(nodes, x)
                if vi < 0 or nodes[y][0] != ir.CONST or wa > 256 or wa < 2:
                    continue
                m = (1 << wa) - 1
                cv = d.consts[nodes[y][5]] & m
                if cv < 2:
                    continue
                q = m // cv
                d.hints.setdefault(vi, []).extend([q, (q + 1) & m])
        if op < ir.EQ or op > ir.USUB_NOUDF:
            continue
        va, vb = _var_of(nodes, a), _var_of(nodes, b)
        if op == ir.EQ and va >= 0 and vb >= 0 and va != vb:
            d.aliases.append((va, vb))
            d.aliases.append((vb, va))
        for vi, y in ((va, b), (vb, a)):
            if vi < 0 or nodes[y][0] != ir.CONST or nodes[a][1] > 256:
                continue
            cv = d.consts[nodes[y][5]]
            m = (1 << nodes[a][1]) - 1
            if op == ir.EQ:
                vals = [cv]
            else:
                up = (cv + 63) & ~63 & m
                vals = [up, (up + 64) & m, cv, (cv - 1) & m, (cv + 1) & m]
            d.hints.setdefault(vi, []).extend(vals)


def pack_states(states: Sequence[StateDag], gpu: bool = False):
    """-> (nodes NODE_DTYPE, node_offsets u64, consts u32[n,8], const_offsets u64);
    gpu=True: the GPU program (padded key equalities replaced, see _strengthen_padded)."""
    lists = [(s.gpu_nodes if gpu and s.gpu_nodes is not None else s.nodes) for s in states]
    n_nodes = sum(len(x) for x in lists)
    nodes = np.zeros(n_nodes, dtype=NODE_DTYPE)
    noff = np.zeros(len(states) + 1, dtype=np.uint64)
    n_c = sum(len(s.consts) for s in states)
    consts = np.zeros((n_c, 8), dtype=np.uint32)
    coff = np.zeros(len(states) + 1, dtype=np.uint64)
    i = j = 0
    for k, s in enumerate(states):
        for (op, w, a, b, c, p0, p1) in lists[k]:
            nodes[i] = (op, 0, w, a, b, c, p0, p1)
            i += 1
        for v in s.consts:
            consts[j] = [(v >> (32 * l)) & 0xFFFFFFFF for l in range(8)] if v < (1 << 256) else 0
            j += 1
        noff[k + 1] = i
        coff[k + 1] = j
    return nodes, noff, consts, coff


def _to_limbs(v: int) -> List[int]:
    return [(v >> (32 * l)) & 0xFFFFFFFF for l in range(8)]


_M256 = (1 << 256) - 1


def _limbs_of(values: Sequence[int]) -> np.ndarray:
    """ints -> uint32 [n, 8] little-endian limbs (low 256 bits)."""
    if not values:
        return np.zeros((0, 8), dtype=np.uint32)
    b = b"".join((int(v) & _M256).to_bytes(32, "little") for v in values)
    return np.frombuffer(b, dtype=np.uint32).reshape(-1, 8).copy()


def _width_mask(w: int) -> np.ndarray:
    return _limbs_of([(1 << min(w, 256)) - 1])[0]


_FIXED_POOL = ACTORS + SPECIAL


_FIXED_LIMBS = _limbs_of(list(_FIXED_POOL))


def make_candidates(states: Sequence[StateDag], n_cand: int, n_vars: int, seed: int = 0x4D595448,
                    parents: Optional[Sequence[Optional[Dict[str, int]]]] = None) -> np.ndarray:
    """uint32 [n_states, n_cand, n_vars, 8] candidate assignments (host layout of mgp_eval_batch).

    c0 parent witness (if any), c1 first hint of every var, c2 = c1 with every
    x == y alias applied, then a seeded mixture per var: 35 % harvested hint,
    25 % pool (state constants +-1, actors, boundary values), 15 % alias of an
    equal-width var, 25 % uniform.  Generated natively (mgp_make_candidates,
    OpenMP over states) from the flattened per-state tables built here.
    """
    from . import _native as N

    n = len(states)
    var_off = np.zeros(n + 1, np.uint64)
    const_off = np.zeros(n + 1, np.uint64)
    alias_off = np.zeros(n + 1, np.uint64)
    widths: List[int] = []
    hint_counts: List[int] = []
    hint_vals: List[int] = []
    alias_pairs: List[Tuple[int, int]] = []
    const_vals: List[int] = []
    for s, st in enumerate(states):
        widths.extend(w for (_, w) in st.vars)
        for vi in range(st.n_vars):
            h = st.hints.get(vi) or ()
            hint_counts.append(len(h))
            hint_vals.extend(h)
        alias_pairs.extend(st.aliases)
        const_vals.extend(st.consts)
        var_off[s + 1] = len(widths)
        alias_off[s + 1] = len(alias_pairs)
        const_off[s + 1] = len(const_vals)
    hint_off = np.zeros(len(hint_counts) + 1, np.uint64)
    hint_off[1:] = np.cumsum(hint_counts)
    has_parent = np.array([bool(parents is not None and parents[s]) for s in range(n)], dtype=np.uint8)
    kinds = np.array([2 if vi in st.pinned else 0 for st in states for vi in range(st.n_vars)], np.uint8)
    out = N.make_candidates(n_cand, n_vars, seed, var_off, np.array(widths, np.uint32), hint_off,
                            _limbs_of(hint_vals), alias_off, np.array(alias_pairs, np.uint32).reshape(-1, 2),
                            const_off, _limbs_of(const_vals), _FIXED_LIMBS, has_parent, var_kind=kinds)
    if parents is not None:
        for s, st in enumerate(states):
            if not parents[s] or n_cand == 0:
                continue
            for vi, (name, w) in enumerate(st.vars):
                if name in parents[s]:
                    pv = parents[s][name]
                    for j in range((st.wide.get(vi, w) + 255) // 256):  # wide: its later slots too
                        out[s, 0, vi + j] = _limbs_of([(pv >> (256 * j)) & ((1 << st.vars[vi + j][1]) - 1)])[0]
    return out


def witness_to_model(st: StateDag, words: np.ndarray) -> Dict[str, int]:
    """Witness words [n_vars, 8] -> {var name: value masked to its width} (free vars only)."""
    model: Dict[str, int] = {}
    vals = []
    for vi, (name, w) in enumerate(st.vars):
        v = 0
        for l in range(8):
            v |= int(words[vi, l]) << (32 * l)
        vals.append(v & ((1 << w) - 1))
    skip = set()
    for vi, w in st.wide.items():
        k = (w + 255) // 256
        skip.update(range(vi + 1, vi + k))
        if vi not in st.pinned:
            model[st.vars[vi][0]] = sum(vals[vi + j] << (256 * j) for j in range(k))
    for vi, (name, w) in enumerate(st.vars):
        if vi not in skip and vi not in st.wide and vi not in st.pinned:
            model[name] = vals[vi]
    return model


def model_to_slots(st: StateDag, model: Dict[str, int]) -> List[int]:
    """{var name: value} -> one int per var slot (a wide var spread over its slots);
    the inverse of witness_to_model, missing names read as 0."""
    out = [0] * st.n_vars
    rest = set()
    for vi, w in st.wide.items():
        v = model.get(st.vars[vi][0], 0)
        for j in range((w + 255) // 256):
            out[vi + j] = (v >> (256 * j)) & ((1 << st.vars[vi + j][1]) - 1)
            rest.add(vi + j)
    for vi, (name, w) in enumerate(st.vars):
        if vi not in rest:
            out[vi] = model.get(name, 0) & ((1 << w) - 1)
    return out


def nominal_ops(st: StateDag) -> int:
    return sum(ir.NOMINAL_OPS.get(n[0], 0) for n in st.nodes)
