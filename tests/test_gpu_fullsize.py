"""Full-size parity: the bench workload itself (SURVEY.md §8d config 3, 2^20 states x
64-node DAGs x 256 candidates), device-resident exactly as bench.py runs it.

At this size the CPU oracle cannot evaluate every candidate in test time, so the
checks are size-independent properties plus oracle checks on samples:

* the two independent GPU engines (hand-written gfx950 interpreter, HIP C++
  interpreter) agree on first_sat for every state;
* every planted witness is found, at or before its planted index;
* sampled SAT states: the reported witness equals the candidate at first_sat and
  the oracle confirms it satisfies the state; sampled states' first_sat equals the
  oracle's first-SAT scan over all 256 of their device candidates;
* the host UNSAT pre-check (plain, and the split refuter on 32 768 states) refutes no state
  that has a GPU witness.
"""
import numpy as np
import pytest

from mythril_amd import _native as N
from oracle import coracle

pytestmark = pytest.mark.gpu

SEED = 0x4D595448


def _run(torch, dev, d_words, d_po, words, po, n_states, d_cands, n_cand, n_vars, engine):
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
        return d_first.cpu().numpy(), d_wit
    finally:
        N.set_eval_engine(old)


def _host_cands(torch, d_cands, states, n_cand, n_vars):
    """Device layout [state][var][half][cand][4] -> host [state][cand][var][8] for the given states."""
    per = n_vars * 2 * n_cand * 4
    idx = torch.from_numpy(np.asarray(states, dtype=np.int64)).to(d_cands.device)
    blk = d_cands.view(-1, per).index_select(0, idx).cpu().numpy().view(np.uint32)
    return np.ascontiguousarray(
        blk.reshape(len(states), n_vars, 2, n_cand, 4).transpose(0, 3, 1, 2, 4).reshape(len(states), n_cand, n_vars, 8))


def _sub_batch(b, states):
    nodes, noff, consts, coff = [], [0], [], [0]
    for s in states:
        n0, n1 = int(b["node_offsets"][s]), int(b["node_offsets"][s + 1])
        c0, c1 = int(b["const_offsets"][s]), int(b["const_offsets"][s + 1])
        nodes.append(b["nodes"][n0:n1])
        consts.append(b["consts"][c0:c1])
        noff.append(noff[-1] + n1 - n0)
        coff.append(coff[-1] + c1 - c0)
    return (np.concatenate(nodes), np.array(noff, np.uint64), np.concatenate(consts).reshape(-1, 8),
            np.array(coff, np.uint64))


def test_bench_workload_full_size(mgp_ctx):
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
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

    first, d_wit = _run(torch, dev, d_words, d_po, words, po, n_states, d_cands, n_cand, n_vars, "asm")
    first_hip, _ = _run(torch, dev, d_words, d_po, words, po, n_states, d_cands, n_cand, n_vars, "hip")
    diff = np.nonzero(first != first_hip)[0]
    assert diff.size == 0, f"engines disagree on {diff.size} states, e.g. {diff[:5]}"
    assert (first >= -1).all()
    assert (first[pl] >= 0).all() and (first[pl] <= b["plant_idx"][pl].astype(np.int64)).all()

    rng = np.random.default_rng(7)
    sample = np.sort(rng.choice(n_states, size=3072, replace=False))
    hc = _host_cands(torch, d_cands, sample, n_cand, n_vars)
    sub = _sub_batch(b, sample)
    ref = coracle.first_sat(*sub, hc)
    assert np.array_equal(first[sample], ref)
    wit = d_wit.view(n_states, n_vars, 8).index_select(
        0, torch.from_numpy(sample.astype(np.int64)).to(dev)).cpu().numpy().view(np.uint32)
    for k in np.nonzero(ref >= 0)[0]:
        assert (wit[k] == hc[k, ref[k]]).all()

    verdict = N.refute(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
    assert not ((verdict == 1) & (first >= 0)).any()
    assert (verdict[first < 0] == 1).any()
    # the split refuter (case splits, linear forms, interval bisection) on the first 32 768
    # states: no GPU-witnessed state refuted, and more refuted than by the plain analysis
    k = 1 << 15
    v2 = N.refute_split(b["nodes"][: int(b["node_offsets"][k])], b["node_offsets"][: k + 1], b["consts"],
                        b["const_offsets"][: k + 1], max_splits=8, depth=2)
    assert not ((v2 == 1) & (first[:k] >= 0)).any()
    assert int((v2 == 1).sum()) > int((verdict[:k] == 1).sum())
