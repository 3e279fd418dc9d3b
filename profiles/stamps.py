#!/usr/bin/env python3
"""Per-wave clock stamps of the interpreter on the bench workload (GPU, diagnostic).

Runs bench.py's synthetic batch once with mgp_set_eval_diag and reports, per wave,
the prologue (entry -> first uop dispatch) and the program run (first dispatch -> RET)
in shader clocks, split into descriptor / page+pool+variable loads / decode, overall
and per v1 slot count.
    python profiles/stamps.py [--states 262144]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import _native as N  # noqa: E402

SEED = 0x4D595448


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--states", type=int, default=1 << 18)
    ap.add_argument("--dump", default="", help="write per-wave stamps to this .npz")
    args = ap.parse_args()
    import torch

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    n_states, n_cand = args.states, 256
    b = N.synth_generate(SEED, 0, n_states, 64, n_cand)
    words, po, status = N.lower(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
    hdr = N.program_headers(words, po)
    n_vars = b["n_vars"]
    d_words = torch.from_numpy(words.view(np.int32)).to(dev)
    d_po = torch.from_numpy(po.view(np.int64)).to(dev)
    d_cands = torch.empty(n_states * n_vars * 2 * n_cand * 4, dtype=torch.int32, device=dev)
    N.fill_candidates_dev(vp(d_words), vp(d_po), n_states, 0, SEED, vp(d_cands), n_cand, n_vars, sh)
    order, bounds, bslots = N.plan_buckets(words, po)
    d_order = torch.from_numpy(order.view(np.int32)).to(dev)
    n_chunks = n_cand // 64
    d_first = torch.empty(n_states, dtype=torch.int32, device=dev)
    d_wit = torch.empty(n_states * n_vars * 8, dtype=torch.int32, device=dev)
    d_scratch = torch.empty(n_states * n_chunks, dtype=torch.int32, device=dev)
    d_diag = torch.zeros(n_states * n_chunks * 4, dtype=torch.int32, device=dev)

    def step():
        N.eval_batch_dev(vp(d_words), vp(d_po), n_states, vp(d_cands), n_cand, n_vars, int(hdr[:, 2].max()),
                         vp(d_first), vp(d_wit), vp(d_scratch), sh, vp(d_order), bounds, bslots)

    step()
    N.lib().mgp_set_eval_diag(vp(d_diag))
    step()
    torch.cuda.synchronize(dev)
    N.lib().mgp_set_eval_diag(None)
    d = d_diag.cpu().numpy().view(np.uint32).reshape(n_states, n_chunks, 4).astype(np.float64)
    desc, loads, disp, run = d[:, :, 0], d[:, :, 1], d[:, :, 2], d[:, :, 3]
    ok = run > 0
    pro = desc + loads + disp
    res = {"waves": int(ok.sum()),
           "desc_med": float(np.median(desc[ok])), "loads_med": float(np.median(loads[ok])),
           "dispatch_med": float(np.median(disp[ok])), "prologue_med": float(np.median(pro[ok])),
           "run_med": float(np.median(run[ok])), "run_mean": float(run[ok].mean()),
           "prologue_share": float(pro[ok].sum() / (pro[ok].sum() + run[ok].sum()))}
    print(json.dumps(res))
    if args.dump:
        np.savez_compressed(args.dump, desc=d[:, :, 0], loads=d[:, :, 1], disp=d[:, :, 2], run=d[:, :, 3],
                            slots=hdr[:, 2])
    slots = hdr[:, 2]
    uops = None
    for sl in np.unique(slots):
        m = (slots == sl)[:, None] & ok
        if m.sum() < 100:
            continue
        print(f"v1 slots {int(sl):2d}: waves {int(m.sum()):7d}  desc {np.median(desc[m]):6.0f}  loads "
              f"{np.median(loads[m]):6.0f}  dispatch {np.median(disp[m]):5.0f}  run med {np.median(run[m]):7.0f}")
    del uops


if __name__ == "__main__":
    main()
