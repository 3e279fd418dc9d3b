"""Multi-process sharding + gather (world size 2, gloo, CPU) — mirrors the RCCL path of bench.py.

Each rank evaluates the states its hash shard owns (here with the CPU oracle
standing in for the kernel, since this runs without a GPU) and rank 0 must
reassemble exactly the single-process result.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from mythril_amd import _native as N
from mythril_amd import distributed as D
from oracle import coracle

from ._util import random_cands


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(n_states=300, n_cand=24):
    b = N.synth_generate(0x4D595448, 4242, n_states, 64, n_cand)
    cands = random_cands(np.random.default_rng(3), n_states, n_cand, b["n_vars"])
    for s in range(n_states):
        if b["planted"][s]:
            cands[s, b["plant_idx"][s]] = b["plant_words"][s]
    return b, cands


def _slice(b, cands, idx):
    no, co = b["node_offsets"], b["const_offsets"]
    nodes = np.concatenate([b["nodes"][int(no[s]):int(no[s + 1])] for s in idx])
    consts = np.concatenate([b["consts"][int(co[s]):int(co[s + 1])] for s in idx])
    noff = np.concatenate([[0], np.cumsum([int(no[s + 1] - no[s]) for s in idx])]).astype(np.uint64)
    coff = np.concatenate([[0], np.cumsum([int(co[s + 1] - co[s]) for s in idx])]).astype(np.uint64)
    return nodes, noff, consts, coff, np.ascontiguousarray(cands[idx])


def _worker(rank, world, port, out_path, balanced=False):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, cands = _batch()
    ids = np.arange(len(b["planted"])) + 10_000  # global state ids

    def evaluate(idx):
        return coracle.first_sat(*_slice(b, cands, idx))

    costs = N.nominal_ops(b["nodes"], b["node_offsets"]) if balanced else None
    res = D.run_sharded(ids, evaluate, dst=0, costs=costs)
    if rank == 0:
        np.save(out_path, res)
    dist.barrier()
    dist.destroy_process_group()


def _wit_worker(rank, world, port, out_path):
    """Each rank evaluates its hash shard, then rank 0 gathers the SAT states' first-SAT
    index and witness words (distributed.gather_witnesses, the §8e exchange step)."""
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, cands = _batch()
    ids = np.arange(len(b["planted"])) + 10_000
    idx = D.local_indices(ids, rank, world)
    first = coracle.first_sat(*_slice(b, cands, idx)) if len(idx) else np.zeros(0, np.int32)
    n_vars = cands.shape[2]
    wit = np.zeros((len(idx), n_vars * 8), np.int32)
    for k, s in enumerate(idx):
        if first[k] >= 0:
            wit[k] = cands[s, first[k]].reshape(-1).view(np.int32)
    res = D.gather_witnesses(torch.as_tensor(ids[idx].astype(np.int64)), torch.as_tensor(first.astype(np.int32)),
                             torch.as_tensor(wit), dst=0)
    if rank == 0:
        np.savez(out_path, ids=res[0], first=res[1], rows=res[2], nbytes=res[3])
    else:
        assert res is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_two_rank_witness_gather_matches_single_process(tmp_path):
    """The gathered witnesses are the single-process witnesses: every SAT state once, with
    its lowest satisfying candidate row (the witness the kernel writes)."""
    out = str(tmp_path / "wit.npz")
    mp.spawn(_wit_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    b, cands = _batch()
    want = coracle.first_sat(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"], cands)
    sat = np.nonzero(want >= 0)[0]
    order = np.argsort(got["ids"])
    assert np.array_equal(got["ids"][order] - 10_000, sat)
    assert np.array_equal(got["first"][order], want[sat])
    rows = got["rows"][order].view(np.uint32).reshape(len(sat), cands.shape[2], 8)
    assert np.array_equal(rows, cands[sat, want[sat]])
    assert int(got["nbytes"]) > 0


def test_hash_sharding_is_a_partition():
    ids = np.arange(10_000)
    for world in (1, 2, 4, 8):
        owners = D.shard_of(ids, world)
        assert owners.min() >= 0 and owners.max() < world
        counts = np.bincount(owners, minlength=world)
        assert counts.sum() == len(ids) and counts.min() > 0.8 * len(ids) / world
        parts = np.concatenate([D.local_indices(ids, r, world) for r in range(world)])
        assert np.array_equal(np.sort(parts), ids)
    # deterministic and process independent: the vectorised map is splitmix64 (hash64), whose
    # first output for 0 is the published constant
    assert D.hash64(0) == 0xE220A8397B1DCDAF
    big = 1 << 62
    assert [int(x) for x in D.shard_of(np.arange(64), big)] == [D.hash64(i) % big for i in range(64)]


def test_keccak_ranges_cover_exactly():
    for n, world in ((10, 3), (1 << 20, 8), (7, 8)):
        spans = [D.keccak_range(n, r, world) for r in range(world)]
        assert spans[0][0] == 0 and sum(c for _, c in spans) == n
        for (f0, c0), (f1, _) in zip(spans, spans[1:]):
            assert f0 + c0 == f1


def test_cost_balanced_shards():
    b = N.synth_generate(0x4D595448, 0, 4096, 64, 256)
    costs = N.nominal_ops(b["nodes"], b["node_offsets"]).astype(np.float64)
    for world in (1, 2, 4, 8):
        owner = D.balanced_shards(costs, world)
        assert owner.min() >= 0 and owner.max() < world
        load = np.bincount(owner, weights=costs, minlength=world)
        assert load.max() - load.mean() <= costs.max()
        assert np.array_equal(owner, D.balanced_shards(costs, world)), "deterministic"
        hash_load = np.bincount(D.shard_of(np.arange(4096), world), weights=costs, minlength=world)
        assert load.max() <= hash_load.max()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("balanced", [False, True])
def test_two_rank_gather_matches_single_process(tmp_path, balanced):
    out = str(tmp_path / "gathered.npy")
    mp.spawn(_worker, args=(2, _free_port(), out, balanced), nprocs=2, join=True)
    got = np.load(out)
    b, cands = _batch()
    want = coracle.first_sat(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"], cands)
    assert np.array_equal(got, want)


def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` without a torchrun environment starts 2 ranks itself (before any
    GPU call); --dry-run keeps it on CPU/gloo.  Rank 0's line reports the world size the
    process group formed and each rank's contiguous shard."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run",
                        "--states", "64"], capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["world_size_seen"] == 2 and line["dry_run"]
    assert [x["first_state"] for x in line["ranks"]] == [0, 64]
    assert all(x["states"] == 64 and x["lowered_ok"] == 64 for x in line["ranks"])
