"""Disagreement signature of the two GPU engines on the full-size bench workload.

Runs the hand-written gfx950 interpreter and the HIP C++ interpreter over the
2^20-state bench batch (tests/test_gpu_fullsize.py's setup) with the libmgp.so
named by MGP_LIB_PATH and prints the number of states whose first_sat differs
and the first few of them.  Used to match a candidate handler defect against
the r3n failure record (39339 states, first [1 30 32 58 75]) by building the
defect into a separate library and comparing signatures.
"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from mythril_amd import _native as N  # noqa: E402

SEED = 0x4D595448


def _run(dev, d_words, d_po, words, po, n_states, d_cands, n_cand, n_vars, engine):
    old = N.set_eval_engine()
    N.set_eval_engine(engine)
    try:
        order, bounds, slots = N.plan_buckets(words, po)
        hdr = N.program_headers(words, po)
        d_order = torch.from_numpy(order.view(np.int32)).to(dev)
        d_first = torch.empty(n_states, dtype=torch.int32, device=dev)
        d_wit = torch.empty(n_states * n_vars * 8, dtype=torch.int32, device=dev)
        d_scratch = torch.empty(n_states * ((n_cand + 63) // 64), dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev)
        N.eval_batch_dev(d_words.data_ptr(), d_po.data_ptr(), n_states, d_cands.data_ptr(), n_cand, n_vars,
                         int(hdr[:, 2].max()), d_first.data_ptr(), d_wit.data_ptr(), d_scratch.data_ptr(),
                         stream.cuda_stream, d_order.data_ptr(), bounds, slots)
        torch.cuda.synchronize(dev)
        return d_first.cpu().numpy()
    finally:
        N.set_eval_engine(old)


def main():
    dev = torch.device("cuda", 0)
    N.Context(0)
    n_states, n_cand, n_nodes = 1 << 20, 256, 64
    b = N.synth_generate(SEED, 0, n_states, n_nodes, n_cand)
    n_vars = b["n_vars"]
    words, po, status = N.lower(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
    assert (status == 0).all()
    d_words = torch.from_numpy(words.view(np.int32)).to(dev)
    d_po = torch.from_numpy(po.view(np.int64)).to(dev)
    d_cands = torch.empty(n_states * n_vars * 2 * n_cand * 4, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    N.fill_candidates_dev(d_words.data_ptr(), d_po.data_ptr(), n_states, 0, SEED, d_cands.data_ptr(), n_cand,
                          n_vars, stream)
    pl = np.nonzero(b["planted"])[0].astype(np.uint32)
    d_ps = torch.from_numpy(pl.view(np.int32)).to(dev)
    d_pi = torch.from_numpy(b["plant_idx"][pl].view(np.int32)).to(dev)
    d_pw = torch.from_numpy(np.ascontiguousarray(b["plant_words"][pl]).view(np.int32)).to(dev)
    N.plant_candidates_dev(d_cands.data_ptr(), n_states, n_cand, n_vars, d_ps.data_ptr(), d_pi.data_ptr(),
                           d_pw.data_ptr(), len(pl), stream)
    first = _run(dev, d_words, d_po, words, po, n_states, d_cands, n_cand, n_vars, "asm")
    first_hip = _run(dev, d_words, d_po, words, po, n_states, d_cands, n_cand, n_vars, "hip")
    diff = np.nonzero(first != first_hip)[0]
    print(json.dumps({"lib": N.LIB_PATH, "disagree": int(diff.size), "first": diff[:8].tolist()}), flush=True)


if __name__ == "__main__":
    main()
