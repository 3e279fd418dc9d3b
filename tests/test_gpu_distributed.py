"""Multi-process sharding + gather with the real kernel (world size 2, gloo for the exchange,
both ranks on the one GPU of the test box) -- the product path of SURVEY §8e with the HIP
interpreter evaluating each rank's hash shard, where tests/test_distributed.py stands the C
oracle in for it.  Rank 0 must reassemble exactly the single-process GPU result (and the
oracle's), first-SAT words and witness rows alike.  (RCCL needs one GPU per rank, so the
exchange runs on gloo here; the driver's 8-GPU scaling run exercises RCCL.)"""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from mythril_amd import _native as N
from mythril_amd import distributed as D
from oracle import coracle

from .test_distributed import _batch, _free_port, _slice

pytestmark = pytest.mark.gpu


def _gpu_eval(ctx, b, cands, idx):
    nodes, noff, consts, coff, c = _slice(b, cands, idx)
    words, po, status = N.lower(nodes, noff, consts, coff)
    assert (status == 0).all()
    return ctx.eval_batch(words, po, c)


def _worker(rank, world, port, out_path):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = N.Context(0)
    try:
        b, cands = _batch()
        ids = np.arange(len(b["planted"])) + 10_000
        first_all = D.run_sharded(ids, lambda idx: _gpu_eval(ctx, b, cands, idx)[0], dst=0)
        idx = D.local_indices(ids, rank, world)
        first, wit = _gpu_eval(ctx, b, cands, idx) if len(idx) else (np.zeros(0, np.int32), None)
        n_vars = cands.shape[2]
        w = (np.zeros((0, n_vars * 8), np.int32) if wit is None
             else np.ascontiguousarray(wit.reshape(len(idx), -1)[:, : n_vars * 8]).view(np.int32))
        res = D.gather_witnesses(torch.as_tensor(ids[idx].astype(np.int64)), torch.as_tensor(first.astype(np.int32)),
                                 torch.as_tensor(w), dst=0)
        if rank == 0:
            np.savez(out_path, first_all=first_all, ids=res[0], first=res[1], rows=res[2])
        dist.barrier()
    finally:
        ctx.close()
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_ranks_on_the_gpu_match_single_process(tmp_path, mgp_ctx):
    out = str(tmp_path / "gpu2.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    b, cands = _batch()
    want = coracle.first_sat(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"], cands)
    single, _ = _gpu_eval(mgp_ctx, b, cands, np.arange(len(want)))
    assert np.array_equal(single, want)
    assert np.array_equal(got["first_all"], want)
    sat = np.nonzero(want >= 0)[0]
    order = np.argsort(got["ids"])
    assert np.array_equal(got["ids"][order] - 10_000, sat)
    assert np.array_equal(got["first"][order], want[sat])
    rows = got["rows"][order].view(np.uint32).reshape(len(sat), cands.shape[2], 8)
    assert np.array_equal(rows, cands[sat, want[sat]])
