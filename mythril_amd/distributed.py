"""Multi-GPU sharding of the pre-filter (one process per GPU, torch.distributed).

States are independent: state `s` belongs to rank
`hash64(s) mod world`, so every rank evaluates its shard with no data-path
collective.  The single exchange step is gathering the per-state first-SAT
words (and, on request, witnesses) to the host-owning rank — RCCL `gather`
over xGMI with backend "nccl" (= RCCL on ROCm), `gloo` on CPU for tests.
Keccak batches split into contiguous index ranges.

Division-heavy DAGs cost ~10x a cheap one, so equal-count hash
shards can leave one GPU with much more work.  `balanced_shards` is the
rebalancing option of SURVEY.md §8e done without moving data after the fact:
every rank holds the batch's per-state cost estimate (nominal ops,
`_native.nominal_ops`) and computes the same cost-balanced assignment locally
(sort by cost, snake order over ranks), so no collective is needed to agree.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

_M64 = (1 << 64) - 1


def hash64(x: int) -> int:
    """splitmix64 finaliser — deterministic across processes (unlike hash())."""
    z = (x + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def shard_of(state_ids: Sequence[int], world: int) -> np.ndarray:
    """Owning rank of each state id."""
    ids = np.asarray(state_ids, dtype=np.uint64)
    z = ids + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return (z % np.uint64(world)).astype(np.int64)


def local_indices(state_ids: Sequence[int], rank: int, world: int) -> np.ndarray:
    """Positions (into state_ids) of the states this rank evaluates."""
    return np.nonzero(shard_of(state_ids, world) == rank)[0]


def balanced_shards(costs: Sequence[float], world: int) -> np.ndarray:
    """Owning rank of each state so that per-rank cost sums are even.

    States sorted by cost (descending, ties by index) are dealt to ranks in snake
    order 0..W-1, W-1..0, ...; deterministic, so every rank computes the same map.
    The heaviest rank exceeds the mean by at most the largest single cost.
    """
    c = np.asarray(costs, dtype=np.float64)
    order = np.lexsort((np.arange(len(c)), -c))
    pos = np.arange(len(c)) % (2 * world)
    lane = np.where(pos < world, pos, 2 * world - 1 - pos)
    owner = np.empty(len(c), dtype=np.int64)
    owner[order] = lane
    return owner


def keccak_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [first, first+count) slice of a Keccak batch for this rank."""
    base, rem = divmod(n_total, world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


def gather_first_sat(local_idx: np.ndarray, local_first: np.ndarray, n_total: int, dst: int = 0,
                     device=None) -> Optional[np.ndarray]:
    """Assemble the global first-SAT array on rank `dst` (None elsewhere).

    Shards differ in size, so sizes are exchanged first and every rank pads to
    the largest shard; one gather of (index, first_sat) pairs follows.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    rank = dist.get_rank()
    dev = device if device is not None else torch.device("cpu")
    n_local = torch.tensor([len(local_idx)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(sizes, n_local)
    cap = int(max(int(s.item()) for s in sizes))
    buf = torch.full((2, max(cap, 1)), -1, dtype=torch.int64, device=dev)
    if len(local_idx):
        buf[0, : len(local_idx)] = torch.as_tensor(np.asarray(local_idx, dtype=np.int64), device=dev)
        buf[1, : len(local_idx)] = torch.as_tensor(np.asarray(local_first, dtype=np.int64), device=dev)
    recv = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, recv, dst=dst)
    if rank != dst:
        return None
    out = np.full(n_total, -3, dtype=np.int64)  # -3: no rank reported this state
    for r, t in enumerate(recv):
        k = int(sizes[r].item())
        a = t.cpu().numpy()
        out[a[0, :k]] = a[1, :k]
    return out.astype(np.int32)


def run_sharded(state_ids: Sequence[int], evaluate: Callable[[np.ndarray], np.ndarray], dst: int = 0,
                device=None, costs: Optional[Sequence[float]] = None) -> Optional[np.ndarray]:
    """Evaluate this rank's shard with `evaluate(positions) -> first_sat` and gather to `dst`.

    Shards are hash shards, or cost-balanced shards when per-state `costs` are given."""
    import torch.distributed as dist

    rank, world = dist.get_rank(), dist.get_world_size()
    if costs is not None:
        idx = np.nonzero(balanced_shards(costs, world) == rank)[0]
    else:
        idx = local_indices(state_ids, rank, world)
    first = evaluate(idx) if len(idx) else np.zeros(0, dtype=np.int32)
    return gather_first_sat(idx, first, len(state_ids), dst=dst, device=device)


def gather_witnesses(ids, first, wit, dst: int = 0):
    """Gather the SAT states' (global id, first-SAT index, witness words) to rank `dst` -- the
    second half of SURVEY.md §8e's exchange step (first-SAT words for every state, witness
    words only for the SAT ones).

    ids (int64 [n]), first (int32 [n]) and wit (int32 [n, n_vars * 8]) are this rank's
    states as torch tensors on the process group's device (CUDA for "nccl" = RCCL, CPU for
    gloo).  Only rows with first >= 0 travel: the counts are exchanged, every rank pads to
    the largest count, one gather of the index / first pairs and one of the witness rows
    follow.  -> on dst (ids np.int64 [k], first np.int32 [k], witness np.int32 [k, n_vars*8],
    bytes received), None elsewhere."""
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    sat = torch.nonzero(first >= 0).flatten()
    k_local = torch.tensor([int(sat.numel())], dtype=torch.int64, device=first.device)
    counts = [torch.zeros_like(k_local) for _ in range(world)]
    dist.all_gather(counts, k_local)
    cap = max(1, max(int(c.item()) for c in counts))
    width = int(wit.shape[1]) if wit.dim() == 2 else 0
    head = torch.full((2, cap), -1, dtype=torch.int64, device=first.device)
    rows = torch.zeros((cap, max(width, 1)), dtype=torch.int32, device=first.device)
    n = int(sat.numel())
    if n:
        head[0, :n] = ids[sat].to(torch.int64)
        head[1, :n] = first[sat].to(torch.int64)
        if width:
            rows[:n, :width] = wit[sat]
    h_recv = [torch.empty_like(head) for _ in range(world)] if rank == dst else None
    r_recv = [torch.empty_like(rows) for _ in range(world)] if rank == dst else None
    dist.gather(head, h_recv, dst=dst)
    dist.gather(rows, r_recv, dst=dst)
    if rank != dst:
        return None
    out_ids, out_first, out_rows = [], [], []
    for r in range(world):
        k = int(counts[r].item())
        a = h_recv[r].cpu().numpy()
        out_ids.append(a[0, :k])
        out_first.append(a[1, :k])
        out_rows.append(r_recv[r].cpu().numpy()[:k, :width])
    nbytes = sum((head.numel() * 8 + rows.numel() * 4) for _ in range(world))
    return (np.concatenate(out_ids), np.concatenate(out_first).astype(np.int32),
            np.concatenate(out_rows).astype(np.int32), nbytes)
