#!/usr/bin/env python3
"""Benchmark of the MI355X satisfiability pre-filter (BASELINE.json metric).

A *step* = one pass of the HIP constraint-evaluation kernel over the whole
synthetic batch resident in HBM: n_states x n_cand candidate-model evaluations
(2^20 states x 64-op-node 256-bit DAGs x 256
candidates per GPU), followed by the first-SAT reduction and — for N > 1 — the
RCCL gather of the per-state first-SAT words to rank 0.  Weak scaling: every
rank owns its own contiguous 2^20-state id range (state ids rank*2^20 + i).

Printed (rank 0, one JSON line): whole-job candidate-model evals/s, the
roofline object of the eval kernel (INT32 VALU bound: nominal ops from the
committed per-op table / measured kernel time, priced against the measured
v_add_u32 probe and, as `frac_spec`, against the 78.6 Tops/s spec peak), its
HBM fraction, the CPU baseline (oracle/c restatement, OpenMP over the host
cores, timed on a bounded sample whose first-SAT words must equal the GPU's),
and the batched Keccak-256 line (config 5; the first 65 536 digests and a
1-in-2^20 sample of the rest are checked against the oracle).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--states S] [--cand C]

With --gpus N > 1 and no torchrun environment, bench.py launches N ranks itself
(torch.distributed.run on 127.0.0.1, before any GPU call) and exits with their
status.  --dry-run replaces the GPU work by a CPU pass over the same shards on
gloo (launcher / rank plumbing test).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "candidate-model evals/sec (1/2/4/8 GPU) + myth analyze wall-clock, z3 calls"
SEED = 0x4D595448
# INT32 VALU: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 Tops/s (MI355X_MICROARCH.md: 4 SIMD-32 per CU,
# a wave64 VALU op issues over 2 cycles).  SURVEY.md's 39.3 counts 64 lanes/CU/clk, half the SIMD width;
# bench.py prices against the v_add_u32 probe (mgp_probe_valu_dev) it measures on the box.
VALU_PEAK_TOPS = 256 * 128 * 2.4e9 / 1e12
KECCAK_KERNEL = {"asm": "mgp_keccak64_gfx950", "asm_dx": "mgp_keccak64_gfx950_dx", "hip": "mgp_keccak64_kernel"}
HBM_PEAK_GBS = 8000.0
KECCAK_OPS_PER_HASH = 7458  # SURVEY.md §8d (310/round x 24 + absorb)
KECCAK_BYTES_PER_HASH = 96
ENGINE_KERNEL = {"asm": "mgp_eval_gfx950", "hip": "mgp_eval_kernel"}


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def vp(t):
    return ctypes.c_void_p(t.data_ptr())


def _slice_states(b, idx):
    """Node lists / constant pools of the states idx of a synthetic batch, repacked."""
    no, co = b["node_offsets"].astype(np.int64), b["const_offsets"].astype(np.int64)
    nl = [b["nodes"][no[i]: no[i + 1]] for i in idx]
    cl = [b["consts"][co[i]: co[i + 1]] for i in idx]
    so = np.zeros(len(idx) + 1, np.uint64)
    so[1:] = np.cumsum([len(x) for x in nl])
    sco = np.zeros(len(idx) + 1, np.uint64)
    sco[1:] = np.cumsum([len(x) for x in cl])
    return np.concatenate(nl), so, np.concatenate(cl).reshape(-1, 8), sco


def _contract_states(n: int):
    """n path-constraint lists of the mixed contract corpus (corpus.py): suicide.sol kill,
    BECToken.sol batchTransfer (overflow / underflow queries) and WalletLibrary.sol
    initWallet -> kill (prune queries along tx 2 and the suicide module's query)."""
    import corpus

    return [c[1] for c in corpus.corpus(n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--states", type=int, default=1 << 20)
    ap.add_argument("--cand", type=int, default=256)
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--keccak", type=int, default=1 << 30, help="hashes per GPU (0 = skip)")
    ap.add_argument("--keccak-chunk", type=int, default=1 << 26)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--refute-sample", type=int, default=1 << 17,
                    help="states of the rank-0 batch run through the host UNSAT pre-check (0 = skip)")
    ap.add_argument("--suite", type=int, default=1, help="the 13-contract solidity_examples suite (0 = skip)")
    ap.add_argument("--suite-open-sweep", type=int, default=1,
                    help="WalletLibrary -t 3 at max_open 6 / 12 / 24 open states between transactions (0 = skip)")
    ap.add_argument("--div-split", type=int, default=1, help="time the division-free twin batch (0 = skip)")
    ap.add_argument("--frontend", type=int, default=1024,
                    help="contract-shaped states through the full Prefilter front end (0 = skip)")
    ap.add_argument("--guided-sample", type=int, default=1 << 16,
                    help="open states of that sample given the domain-guided second witness round")
    ap.add_argument("--keccak-sample-every", type=int, default=1 << 20,
                    help="beyond the first 65 536, check one digest in this many against the oracle")
    ap.add_argument("--detail", default=None,
                    help="path of the full JSON record (default profiles/bench_detail_r6.json)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: gloo ranks run the shard plumbing on CPU and rank 0 prints one line")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launched without torchrun: start the N ranks here, before anything touches the GPU
        sys.exit(launch_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    from mythril_amd import _native as N

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        return dry_run(args, world, rank)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        world = dist.get_world_size()  # the world RCCL actually formed
    N.lib()  # loud failure if the HIP library is missing

    # ---------------------------------------------------------- workload
    n_states, n_cand, n_nodes = args.states, args.cand, args.nodes
    base = rank * n_states
    t0 = time.time()
    b = N.synth_generate(SEED, base, n_states, n_nodes, n_cand)
    words, po, status = N.lower(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
    hdr = N.program_headers(words, po)
    n_slots = int(hdr[:, 2].max())
    n_vars = b["n_vars"]
    ops_state = N.nominal_ops(b["nodes"], b["node_offsets"]).astype(np.float64)
    log(f"rank {rank}: generated+lowered {n_states} states in {time.time() - t0:.1f}s; "
        f"slots max {n_slots}, ins mean {hdr[:, 0].mean():.1f}, unsupported {(status != 0).sum()}")

    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)
    d_words = torch.from_numpy(words.view(np.int32)).to(dev)
    d_po = torch.from_numpy(po.view(np.int64)).to(dev)
    n_cand_words = n_states * n_vars * 2 * n_cand * 4
    d_cands = torch.empty(n_cand_words, dtype=torch.int32, device=dev)
    N.fill_candidates_dev(vp(d_words), vp(d_po), n_states, base, SEED, vp(d_cands), n_cand, n_vars, sh)
    pl = np.nonzero(b["planted"])[0].astype(np.uint32)
    d_pstate = torch.from_numpy(pl.view(np.int32)).to(dev)
    d_pidx = torch.from_numpy(b["plant_idx"][pl].view(np.int32)).to(dev)
    d_pwords = torch.from_numpy(np.ascontiguousarray(b["plant_words"][pl]).view(np.int32)).to(dev)
    N.plant_candidates_dev(vp(d_cands), n_states, n_cand, n_vars, vp(d_pstate), vp(d_pidx), vp(d_pwords),
                           len(pl), sh)
    order, bounds, bslots = N.plan_buckets(words, po)
    d_order = torch.from_numpy(order.view(np.int32)).to(dev)
    log(f"rank {rank}: {len(bslots)} slot buckets: " +
        ", ".join(f"{int(sl)}:{int(bounds[i + 1] - bounds[i])}" for i, sl in enumerate(bslots)))
    n_chunks = (n_cand + 63) // 64
    d_first = torch.empty(n_states, dtype=torch.int32, device=dev)
    d_wit = torch.empty(n_states * n_vars * 8, dtype=torch.int32, device=dev)
    d_scratch = torch.empty(n_states * n_chunks, dtype=torch.int32, device=dev)
    gather_buf = [torch.empty_like(d_first) for _ in range(world)] if (world > 1 and rank == 0) else None
    torch.cuda.synchronize(dev)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        N.eval_batch_dev(vp(d_words), vp(d_po), n_states, vp(d_cands), n_cand, n_vars, n_slots, vp(d_first),
                         vp(d_wit), vp(d_scratch), sh, vp(d_order), bounds, bslots)
        if ev is not None:
            ev[1].record(stream)
        if world > 1:
            dist.gather(d_first, gather_buf if rank == 0 else None, dst=0)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    valu_peak = measure_valu_peak(N, torch, dev, stream, sh)
    log(f"rank {rank}: measured INT32 VALU peak {valu_peak:.1f} Tops/s (derived {VALU_PEAK_TOPS:.1f})")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    kern_ms = float(np.mean([a.elapsed_time(bb) for a, bb in evs]))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # the rest of the §8e exchange step, outside the timed steps (which gather first-SAT
    # words only): the SAT states' witness words to rank 0 (distributed.gather_witnesses)
    gather = None
    if world > 1:
        from mythril_amd import distributed as DIST

        ids_t = torch.arange(base, base + n_states, dtype=torch.int64, device=dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        tg = time.perf_counter()
        gres = DIST.gather_witnesses(ids_t, d_first, d_wit.view(n_states, n_vars * 8), dst=0)
        torch.cuda.synchronize(dev)
        gms = 1e3 * (time.perf_counter() - tg)
        if rank == 0:
            gather = {"witness_states": int(len(gres[0])), "gather_bytes": int(gres[3]), "gather_ms": gms,
                      "first_sat_bytes_per_step": 4 * n_states * world,
                      "note": "RCCL gather of (state id, first-SAT, witness words) of every SAT state to rank 0"}
    first = d_first.cpu().numpy()
    sat = int((first >= 0).sum())
    planted_ok = bool(np.all(first[pl] >= 0) and np.all(first[pl] <= b["plant_idx"][pl].astype(np.int64)))
    evals_rank = n_states * n_cand
    value = world * evals_rank * args.steps / elapsed
    ops_launch = float(ops_state.sum()) * n_cand
    achieved_tops = ops_launch / (kern_ms * 1e-3) / 1e12
    bytes_launch = (n_cand_words * 4 + words.nbytes + po.nbytes + n_states * n_chunks * 4 * 2 + n_states * 4
                    + sat * n_vars * 32)
    achieved_gbs = bytes_launch / (kern_ms * 1e-3) / 1e9
    log(f"rank {rank}: kernel {kern_ms:.2f} ms/launch, step {1e3 * elapsed / args.steps:.2f} ms, SAT {sat}/{n_states}, "
        f"planted found {planted_ok}")

    # Division split: the same states with every division drawn as an ADD
    # (mgp_synth_set_ablate; the random stream is unchanged otherwise), timed on the same
    # candidates.  div_share = the part of a launch the divisions take; frac_nondiv = the
    # nominal ops of the division-free DAGs per second of their launch, against the spec
    # peak -- the roofline of everything but the 1024-op division pricing.
    div_split = None
    if args.div_split and rank == 0:
        N.synth_set_ablate(1)
        try:
            b2 = N.synth_generate(SEED, base, n_states, n_nodes, n_cand)
        finally:
            N.synth_set_ablate(0)
        w2, po2, _ = N.lower(b2["nodes"], b2["node_offsets"], b2["consts"], b2["const_offsets"])
        ops2 = N.nominal_ops(b2["nodes"], b2["node_offsets"]).astype(np.float64)
        slots2 = int(N.program_headers(w2, po2)[:, 2].max())
        order2, bounds2, bslots2 = N.plan_buckets(w2, po2)
        d_w2 = torch.from_numpy(w2.view(np.int32)).to(dev)
        d_po2 = torch.from_numpy(po2.view(np.int64)).to(dev)
        d_order2 = torch.from_numpy(order2.view(np.int32)).to(dev)
        ev2 = []
        for k in range(args.warmup + args.steps):
            e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            e[0].record(stream)
            N.eval_batch_dev(vp(d_w2), vp(d_po2), n_states, vp(d_cands), n_cand, n_vars, slots2, vp(d_first),
                             vp(d_wit), vp(d_scratch), sh, vp(d_order2), bounds2, bslots2)
            e[1].record(stream)
            if k >= args.warmup:
                ev2.append(e)
        torch.cuda.synchronize(dev)
        t2 = float(np.mean([a.elapsed_time(bb) for a, bb in ev2]))
        ops_nondiv = float(ops2.sum()) * n_cand
        div_split = {"launch_ms_nodiv": t2, "div_share": 1.0 - t2 / kern_ms,
                     "ops_per_eval_nodiv": float(ops2.mean()),
                     "achieved_nondiv": ops_nondiv / (t2 * 1e-3) / 1e12,
                     "frac_nondiv": ops_nondiv / (t2 * 1e-3) / 1e12 / VALU_PEAK_TOPS}
        del d_w2, d_po2, d_order2
        log(f"rank {rank}: division split {div_split}")

    # HBM bytes and issued VALU instructions per step from the committed rocprofv3 PMC
    # run of the same workload (profiles/collect.sh -> analyze.py -> profiles/eval_pmc.json)
    traffic, valu_busy = None, None
    pmc_path = os.path.join(ROOT, "profiles", "eval_pmc.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pm = json.load(f)
            if (pm.get("states") == n_states and pm.get("cand") == n_cand
                    and pm.get("kernel") == ENGINE_KERNEL[N.set_eval_engine()]):
                traffic = pm.get("hbm_bytes_per_launch")
                if pm.get("valu_wave_insts_per_step"):
                    valu_busy = {"issued_int32_lane_ops_per_s": pm["valu_wave_insts_per_step"] * 64 / (kern_ms * 1e-3),
                                 "source": pm.get("source")}
        except (OSError, ValueError):
            traffic = None

    # ---------------------------------------------------------- Keccak
    keccak = None
    if args.keccak > 0:
        nk, chunk = args.keccak, min(args.keccak_chunk, args.keccak)
        kfirst = rank * nk
        d_pre = torch.empty(nk * 64, dtype=torch.uint8, device=dev)
        d_dig = torch.empty(nk * 32, dtype=torch.uint8, device=dev)
        N.fill_mapping_preimages_dev(vp(d_pre), kfirst, nk, SEED, sh)
        torch.cuda.synchronize(dev)

        def kpass(evl=None):
            for off in range(0, nk, chunk):
                m = min(chunk, nk - off)
                if evl is not None:
                    evl.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                    evl[-1][0].record(stream)
                N.keccak256_dev(ctypes.c_void_p(d_pre.data_ptr() + off * 64), m, 64, 64,
                                ctypes.c_void_p(d_dig.data_ptr() + off * 32), sh)
                if evl is not None:
                    evl[-1][1].record(stream)

        kpass()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        kevs = []
        tk = time.perf_counter()
        ksteps = max(1, min(args.steps, 3))
        for _ in range(ksteps):
            kpass(kevs)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        kel = time.perf_counter() - tk
        if world > 1:
            t = torch.tensor([kel], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            kel = float(t.item())
        kms = float(np.mean([a.elapsed_time(bb) for a, bb in kevs]))
        k_rate = world * nk * ksteps / kel
        k_verified = verify_keccak(d_pre, d_dig, kfirst, nk, args.keccak_sample_every)
        if world > 1:
            t = torch.tensor([k_verified["checked"], k_verified["mismatches"]], dtype=torch.int64, device=dev)
            dist.all_reduce(t)
            k_verified.update(checked=int(t[0]), mismatches=int(t[1]), ranks=world)
        log(f"keccak verification: {k_verified}")
        if k_verified["mismatches"]:
            raise RuntimeError(f"keccak digests differ from the oracle: {k_verified}")
        # A/B: the same passes on the other 64-byte kernel (compiler-allocated HIP vs the
        # hand-allocated gfx950 one), timed the same way; digests were verified above
        k_engine = N.set_keccak_engine()
        k_ab = {}
        for other in ("asm", "asm_dx", "hip"):
            if other == k_engine:
                continue
            N.set_keccak_engine(other)
            kpass()
            torch.cuda.synchronize(dev)
            kevs_o = []
            for _ in range(ksteps):
                kpass(kevs_o)
            torch.cuda.synchronize(dev)
            kms_o = float(np.mean([a.elapsed_time(bb) for a, bb in kevs_o]))
            k_ab[other] = {"launch_ms": kms_o, "hashes_per_s_per_gpu": chunk / (kms_o * 1e-3)}
        N.set_keccak_engine(k_engine)
        k_tops = chunk * KECCAK_OPS_PER_HASH / (kms * 1e-3) / 1e12
        k_gbs = chunk * KECCAK_BYTES_PER_HASH / (kms * 1e-3) / 1e9
        # HBM bytes and issued VALU lane-ops per hash from the committed rocprofv3 PMC run
        # (profiles/collect.sh -> analyze.py -> profiles/keccak_pmc.json)
        k_traffic, k_issued = None, None
        kp = os.path.join(ROOT, "profiles", "keccak_pmc.json")
        if os.path.exists(kp):
            try:
                with open(kp) as f:
                    km = json.load(f)
                if km.get("kernel") != KECCAK_KERNEL[k_engine]:  # a profile of the other kernel says nothing here
                    km = {}
                if km.get("hbm_bytes_per_hash") and k_traffic is None:
                    k_traffic = km["hbm_bytes_per_hash"] * chunk
                if km.get("valu_lane_ops_per_hash"):
                    iss = km["valu_lane_ops_per_hash"] * chunk / (kms * 1e-3) / 1e12
                    k_issued = {"lane_ops_per_hash": km["valu_lane_ops_per_hash"], "achieved": iss,
                                "peak": VALU_PEAK_TOPS, "unit": "TOP/s", "frac": iss / VALU_PEAK_TOPS,
                                "peak_measured": valu_peak, "frac_measured": iss / valu_peak,
                                "source": km.get("source")}
            except (OSError, ValueError):
                pass
        if k_issued is None and k_engine != "hip":
            # the hand-allocated kernel is straight-line code: every VALU instruction of its
            # source issues exactly once per wave (one hash per lane)
            sys.path.insert(0, os.path.join(ROOT, "mythril_amd", "csrc"))
            import gen_keccak_asm

            theta = dict(gen_keccak_asm.VARIANTS)[KECCAK_KERNEL[k_engine]]
            n_valu = sum(1 for ln in gen_keccak_asm.generate(theta=theta)[0].split("\n") if ln.strip().startswith("v_"))
            n_valu += 8  # prologue: index, bound compare, address arithmetic (the digest gather is in the body)
            iss = n_valu * chunk / (kms * 1e-3) / 1e12
            k_issued = {"lane_ops_per_hash": n_valu, "achieved": iss, "peak": VALU_PEAK_TOPS, "unit": "TOP/s",
                        "frac": iss / VALU_PEAK_TOPS, "peak_measured": valu_peak, "frac_measured": iss / valu_peak,
                        "source": "static count of mgp_keccak64_gfx950 (straight-line: each VALU instruction "
                                  "issues once per wave)"}
        keccak = {
            "metric": "keccak256 hashes/s (64-byte mapping-slot preimages)",
            "value": k_rate,
            "unit": "hashes/s",
            "hashes_per_gpu": nk,
            "ms_per_pass": 1e3 * kel / ksteps,
            "engine": k_engine,
            "kernel": KECCAK_KERNEL[k_engine],
            "ab_other_engines": k_ab,
            # frac = ISSUED VALU lane-ops (PMC, profiles/keccak_pmc.json) over the spec peak: a
            # true fraction (<= 1).  The nominal-op rate (7 458 ops/hash) counts
            # ops that v_bitop3 / v_alignbit fold into one instruction, so it can pass the peak;
            # it is kept as nominal_achieved / nominal_frac.
            "roofline": {"bound": "valu", "achieved": k_issued["achieved"] if k_issued else None,
                         "peak": VALU_PEAK_TOPS, "unit": "TOP/s",
                         "frac": k_issued["frac"] if k_issued else None, "traffic": k_traffic,
                         "ops": "issued VALU lane-ops per hash (PMC SQ_INSTS_VALU x 64) x hashes",
                         "nominal_achieved": k_tops, "nominal_frac": k_tops / VALU_PEAK_TOPS,
                         "kernel": KECCAK_KERNEL[k_engine], "launch_ms": kms, "hashes_per_launch": chunk},
            "valu_issued": k_issued,
            "verified": k_verified,
            "roofline_hbm": {"achieved": k_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": k_gbs / HBM_PEAK_GBS},
        }
        del d_pre, d_dig

    # ------------------------------------------- solver-call accounting (host pre-check)
    # Of a sample of the batch: states with a GPU witness (SAT, no solver call), states the
    # host pre-check proves UNSAT (mgp_refute, no solver call), and the rest, which the
    # integrated path hands to z3 (SURVEY.md 8d "z3 calls").  Not part of the timed step.
    prefilter = None
    if rank == 0 and args.refute_sample > 0:
        ns = min(n_states, args.refute_sample)
        tr = time.perf_counter()
        ver = N.refute(b["nodes"][: int(b["node_offsets"][ns])], b["node_offsets"][: ns + 1], b["consts"],
                       b["const_offsets"][: ns + 1])
        dtr = time.perf_counter() - tr
        sat_s, ref_s = first[:ns] >= 0, ver == 1
        if (sat_s & ref_s).any():
            raise RuntimeError("mgp_refute refuted a state with a GPU witness (soundness bug)")
        # the split refuter (case splits, linear forms, bisection) against the GPU witnesses of
        # the first 32 768 states: a 256-bit soundness check on random DAGs
        ns2 = min(ns, 1 << 15)
        ts2 = time.perf_counter()
        ver2 = N.refute_split(b["nodes"][: int(b["node_offsets"][ns2])], b["node_offsets"][: ns2 + 1], b["consts"],
                              b["const_offsets"][: ns2 + 1], max_splits=8, depth=2)
        split_check = {"states": ns2, "refuted": int((ver2 == 1).sum()),
                       "refuted_with_gpu_witness": int(((ver2 == 1) & (first[:ns2] >= 0)).sum()),
                       "seconds": time.perf_counter() - ts2}
        if split_check["refuted_with_gpu_witness"]:
            raise RuntimeError(f"mgp_refute_split refuted states with a GPU witness: {split_check}")
        fallback = int(ns - sat_s.sum() - ref_s.sum())
        # second witness round on the states still open: candidates drawn from the pre-check's
        # refined domains, 32 rows by decisions (mgp_guided_candidates), the rest uniform
        open_idx = np.nonzero(~sat_s & ~ref_s)[0][: args.guided_sample]
        guided = None
        if len(open_idx):
            tg = time.perf_counter()
            sn, so, sc, sco = _slice_states(b, open_idx)
            gw, gpo, _ = N.lower(sn, so, sc, sco)
            g_cand = 128
            gc = np.random.default_rng(SEED).integers(0, 2 ** 32, size=(len(open_idx), g_cand, n_vars, 8),
                                                      dtype=np.uint32)
            gst = N.guided_candidates(sn, so, sc, sco, gc, seed=SEED, every=2, n_decide=32)
            dgen = time.perf_counter() - tg
            gctx = N.Context(local)
            gfirst, _ = gctx.eval_batch(gw, gpo, gc)
            gctx.close()
            if ((gfirst >= 0) & (gst == 1)).any():
                raise RuntimeError("mgp_refute refuted a state with a GPU witness (soundness bug)")
            found = int((gfirst >= 0).sum())
            left = fallback - found if len(open_idx) == fallback else None
            guided = {"open_states": len(open_idx), "candidates": g_cand, "decision_rows": 32,
                      "gpu_sat": found, "fallback_after": left,
                      "solver_call_reduction": (ns / max(1, left)) if left is not None else None,
                      "host_states_per_s": len(open_idx) / dgen, "seconds": time.perf_counter() - tg}
        prefilter = {"sample_states": ns, "gpu_sat": int(sat_s.sum()), "refuted": int(ref_s.sum()),
                     "fallback": fallback, "solver_call_reduction": ns / max(1, fallback),
                     "refute_states_per_s": ns / dtr, "refute_threads": _threads(),
                     "guided_round": guided, "split_check": split_check,
                     "note": "synthetic DAGs (random ops), not solidity_examples; reduction = states / states "
                             "left for z3 after GPU witnesses and host refutations (guided_round: after the "
                             "second, domain-guided witness round as well)"}
        log(f"prefilter: {prefilter}")

    # ------------------------------------------ front end (host + GPU) on contract-shaped states
    # The product path of Constraints.is_possible / get_model for a batch: DAG build, lowering,
    # candidates, GPU evaluation, pre-check, guided second round.  Not part of the timed step.
    frontend = None
    if rank == 0 and args.frontend > 0:
        from mythril_amd import solver as SV

        pf = SV.Prefilter(device=local)
        cs = _contract_states(args.frontend)
        pf.check_states(cs[:64])  # warm-up (kernels loaded, host pools touched)
        # three cold calls (no UNSAT core and no lowered program from an earlier call answers
        # any of them); the median is the reported rate, the first call is kept beside it,
        # and every call must give the same answers
        fe_calls = []
        for rep in range(3):
            SV.unsat_cores().reset()
            pf._N.program_cache_clear()
            SV.SolverStatistics().reset()
            tf = time.perf_counter()
            res = pf.check_states(cs)
            fe_calls.append((time.perf_counter() - tf, [r[0] for r in res], pf.last_profile,
                             SV.SolverStatistics().refuted, SV.SolverStatistics().core_hits))
        kinds = fe_calls[0][1]
        if any(c[1] != kinds for c in fe_calls):
            raise RuntimeError("front end: cold calls on one batch gave different answers")
        med_call = sorted(fe_calls, key=lambda c: c[0])[1]
        dtf = med_call[0]
        import collections

        import corpus

        items = corpus.corpus(len(cs))
        labels = [c[0] for c in items]
        by_shape = collections.defaultdict(collections.Counter)
        for lab, k in zip(labels, kinds):
            by_shape[lab.split(":")[0]][k] += 1
        # answers against the corpus' by-construction expectations (corpus.py): a "sat" on an
        # expected-unsat state would be a wrong answer, an "unsat" on an expected-sat one too
        expect = {"expected_unsat": 0, "expected_unsat_refuted": 0, "expected_sat": 0, "expected_sat_witness": 0,
                  "contradicted": 0}
        for (_, _, e), k in zip(items, kinds):
            if e == "unsat":
                expect["expected_unsat"] += 1
                expect["expected_unsat_refuted"] += k == SV.unsat
                expect["contradicted"] += k == SV.sat
            elif e == "sat":
                expect["expected_sat"] += 1
                expect["expected_sat_witness"] += k == SV.sat
                expect["contradicted"] += k == SV.unsat
        if expect["contradicted"]:
            raise RuntimeError(f"front end contradicts the corpus expectations: {expect}")
        frontend = {"states": len(cs), "seconds": dtf, "states_per_s": len(cs) / dtf,
                    "calls_seconds": [round(c[0], 4) for c in fe_calls], "first_call_seconds": fe_calls[0][0],
                    "sat": kinds.count(SV.sat), "unsat": kinds.count(SV.unsat),
                    "refuted": med_call[3], "core_hits": med_call[4],
                    "undecided": kinds.count("undecided"), "candidates": pf.n_cand,
                    "solver_call_reduction": len(cs) / max(1, kinds.count("undecided")), "expectations": expect,
                    "by_contract": {k: dict(v) for k, v in by_shape.items()},
                    "stages_ms": med_call[2], "latency": frontend_latency(pf, SV, cs),
                    "latency_2_by_contract": {
                        k: frontend_latency(pf, SV, [c for c, lab in zip(cs, labels) if lab.startswith(k)], sizes=(2,))
                        for k in ("suicide", "bectoken", "wallet")},
                    "shape": "mixed corpus (corpus.py): suicide.sol kill, BECToken.sol batchTransfer, "
                             "WalletLibrary.sol initWallet -> kill"}
        # the same batch, cold, with the first GPU round and the host pre-check only (no
        # retry round, no host decision rows): the throughput end of the policy
        SV.unsat_cores().reset()
        pf._N.program_cache_clear()
        keep_retry, pf.retry_cand = pf.retry_cand, 0
        tf = time.perf_counter()
        res1 = pf.check_states(cs)
        dt1 = time.perf_counter() - tf
        pf.retry_cand = keep_retry
        k1 = [r[0] for r in res1]
        frontend["first_round_only"] = {"seconds": dt1, "states_per_s": len(cs) / dt1, "sat": k1.count(SV.sat),
                                        "unsat": k1.count(SV.unsat), "undecided": k1.count("undecided"),
                                        "solver_call_reduction": len(cs) / max(1, k1.count("undecided")),
                                        "stages_ms": pf.last_profile}
        # A/B: the same cold batch with the UNSAT-core shrink on a worker thread (a quarter of
        # the OpenMP threads), then the default policy's result vector is compared
        SV.unsat_cores().reset()
        pf._N.program_cache_clear()
        pf.core_async = True
        tf = time.perf_counter()
        res_a = pf.check_states(cs)
        dta = time.perf_counter() - tf
        SV.unsat_cores().join()
        pf.core_async = False
        frontend["core_async"] = {"seconds": dta, "states_per_s": len(cs) / dta,
                                  "same_answers": [r[0] for r in res_a] == kinds}
        # A/B: the candidate-memory cap of one witness round (batches past it run as
        # sub-batches one after another), the default against 4x it
        keep_cb = pf.cand_bytes
        for tag, cb in (("cand_cap_x4", 4 * keep_cb), ("cand_cap_default", keep_cb)):
            SV.unsat_cores().reset()
            pf._N.program_cache_clear()
            pf.cand_bytes = cb
            tf = time.perf_counter()
            res_c = pf.check_states(cs)
            dtc = time.perf_counter() - tf
            frontend[tag] = {"cand_bytes": cb, "seconds": dtc, "states_per_s": len(cs) / dtc,
                             "same_answers": [r[0] for r in res_c] == kinds, "stages_ms": pf.last_profile}
        pf.cand_bytes = keep_cb
        # A/B: the call cut into at least 2 / 4 groups (Prefilter.min_groups), so that more of
        # each GPU round overlaps the next group's host stages; medians of 3 cold calls
        keep_mg = pf.min_groups
        frontend["min_groups"] = {}
        for mg in (2, 4):
            pf.min_groups = mg
            runs = []
            for rep in range(3):
                SV.unsat_cores().reset()
                pf._N.program_cache_clear()
                tf = time.perf_counter()
                res_g = pf.check_states(cs)
                runs.append((time.perf_counter() - tf, [r[0] for r in res_g], pf.last_profile))
            medg = sorted(runs, key=lambda c: c[0])[1]
            frontend["min_groups"][str(mg)] = {"seconds": medg[0], "states_per_s": len(cs) / medg[0],
                                               "calls_seconds": [round(c[0], 4) for c in runs],
                                               "same_answers": all(c[1] == kinds for c in runs),
                                               "stages_ms": medg[2]}
            if not frontend["min_groups"][str(mg)]["same_answers"]:
                raise RuntimeError(f"front end: min_groups={mg} gave other answers")
        pf.min_groups = keep_mg
        pf.ctx.close()
        # two pipelines on the one GPU (Prefilter(pipelines=2)): the batch hash-sharded over two
        # contexts, each on its own host thread with half the OpenMP threads, so that one
        # shard's GPU round overlaps the other's host stages; GPU busy =
        # the sum of the two shards' GPU waits and launch stages over the call's wall time
        pf2 = SV.Prefilter(devices=[local], pipelines=2)
        pf2.check_states(cs[:256])
        p2 = []
        for rep in range(3):
            SV.unsat_cores().reset()
            pf2._N.program_cache_clear()
            tf = time.perf_counter()
            res2 = pf2.check_states(cs)
            p2.append((time.perf_counter() - tf, [r[0] for r in res2], pf2.last_profile))
        pf2.close()
        med2 = sorted(p2, key=lambda c: c[0])[1]
        frontend["pipelines2"] = {"seconds": med2[0], "states_per_s": len(cs) / med2[0],
                                  "calls_seconds": [round(c[0], 4) for c in p2],
                                  "same_answers": all(c[1] == kinds for c in p2), "stages_ms": med2[2]}
        if not frontend["pipelines2"]["same_answers"]:
            raise RuntimeError("front end: two pipelines gave other answers than one")
        log(f"frontend: {frontend}")

    # ------------------------------------ the 13 solidity_examples contracts (configs 1, 2, 4 + 10 more)
    # Every query a `myth analyze <contract> -t N` run asks, restated by corpus.laser /
    # corpus.contracts and tagged prune / SAT-only get_model / get_transaction_sequence, through
    # the product Prefilter cold, one batch per contract.  z3 calls are counted the honest way
    # (corpus.account): a tx-sequence query is a z3 Optimize call unless refuted.
    suite = None
    if rank == 0 and args.suite:
        from mythril_amd import solver as SV

        import corpus

        tg = time.perf_counter()
        qs = corpus.suite()
        gen_s = time.perf_counter() - tg
        pf = SV.Prefilter(device=local)
        pf.check_states([list(q[3]) for q in qs[:64]])        # warm-up (kernels loaded, pools touched)
        SV.unsat_cores().reset()
        pf._N.program_cache_clear()
        SV.SolverStatistics().reset()
        t_all = time.perf_counter()
        answers, _ = corpus.answer(pf, qs)   # level by level along parent links, parent witnesses passed
        dt_all = time.perf_counter() - t_all
        acc = corpus.account(qs, answers)
        if acc["all"]["contradicted"]:
            raise RuntimeError(f"suite answers contradict the expectations: {acc['all']}")
        # the UNSAT side against the SAT side: no query the GPU answered
        # with a model (a proof of SAT) may be refuted by the refuter at either setting or be
        # covered by a stored UNSAT core; and no refuted sat-if-reachable query lacks a
        # refuted ancestor (corpus.account counts that as a contradiction)
        from mythril_amd.front import Batch

        ts = time.perf_counter()
        sat_idx = [k for k, a in enumerate(answers) if a == "sat"]
        SB = Batch([list(qs[k][3]) for k in sat_idx])
        try:
            packed = SB.packed()[:4]
            r_plain = N.refute(*packed)
            r_split = N.refute_split(*packed, max_splits=SV.Prefilter.SPLIT_REFUTE, depth=SV.Prefilter.SPLIT_DEPTH)
        finally:
            SB.close()
        SV.unsat_cores().flush(N)
        # ... and every refutation audited by a wider witness search (1 024 candidates per state
        # from another seed, no pre-check): a model it finds would make that refutation unsound
        unsat_idx = [k for k, a in enumerate(answers) if a == "unsat"]
        auditor = SV.Prefilter(device=local, n_cand=1024, seed=0xA0D17)
        auditor.refute, auditor.retry_cand, auditor.rows_first_nodes, auditor.split_refute = False, 0, 0, 0
        audit = auditor.check_states([list(qs[k][3]) for k in unsat_idx]) if unsat_idx else []
        auditor.close()
        soundness = {"witnessed": len(sat_idx), "refuted_plain": int((r_plain == 1).sum()),
                     "refutations_audited": len(unsat_idx), "audit_candidates": 1024,
                     "audit_models_found": sum(1 for a, _ in audit if a == "sat"),
                     "refuted_split": int((r_split == 1).sum()),
                     "core_covered": int(sum(SV.unsat_cores().covered(qs[k][3]) for k in sat_idx)),
                     **{f: acc["all"][f] for f in ("sat_if_reachable", "refuted_with_sat_expectation_if_reachable",
                                                   "sat_expectations_dropped")},
                     "seconds": time.perf_counter() - ts}
        log(f"suite soundness: {soundness}")
        if (soundness["refuted_plain"] or soundness["refuted_split"] or soundness["core_covered"]
                or soundness["audit_models_found"]):
            raise RuntimeError(f"the refuter claims UNSAT for witnessed suite queries: {soundness}")
        suite = dict(acc, queries=len(qs), seconds=dt_all, queries_per_s=len(qs) / dt_all, generate_s=gen_s,
                     soundness=soundness,
                     held_out_contracts=sorted(corpus.held_out()),
                     note="queries restated by reading the reference (corpus/laser.py, corpus/contracts.py); "
                          "ref_calls = restated reference calls (the z3 calls the restated run makes, get_model "
                          "lru-deduplicated), z3_calls = undecided prune/model/dep queries + every tx-sequence "
                          "query not refuted; dep = DependencyPruner's get_model((loc == dep,))")
        # the issues SURVEY §8d expects by reading for configs 1, 2 and 4: every query of the module
        # that reports them, with the product's answers ("sat" = a GPU witness: the state exists,
        # so z3 finds the transaction sequence and the issue is reported by both paths)
        suite["config_issues"] = {lab: [a for q, a in zip(qs, answers) if q[2].startswith(lab)] for lab in (
            "suicide:suicide@kill:selfdestruct", "bectoken:overflow_issue@batchTransfer:mul",
            "wallet:suicide_attacker@kill:selfdestruct")}
        # the two held-out contracts no round-6 mechanism was studied on (rubixi and weak_random
        # were opened for the root-cause analysis): the generality check
        suite["frozen"] = {n: {k: acc["by_contract"][n][k] for k in ("ref_calls", "z3_calls", "reduction")}
                           for n in ("timelock", "token") if n in acc["by_contract"]}
        # WalletLibrary -t 3 (config 4, "state explosion") as the open states carried between
        # transactions grow: max_open 6 (the suite's cap) / 12 / 24
        if args.suite_open_sweep:
            sweep = {}
            for mo in (6, 12, 24):
                tg = time.perf_counter()
                wq = corpus.suite(max_open=mo, contracts={"wallet"})
                g = time.perf_counter() - tg
                SV.unsat_cores().reset()
                pf._N.program_cache_clear()
                t0 = time.perf_counter()
                wa, _ = corpus.answer(pf, wq)
                dt = time.perf_counter() - t0
                wacc = corpus.account(wq, wa)["all"]
                if wacc["contradicted"]:
                    raise RuntimeError(f"wallet max_open={mo} contradicts the expectations: {wacc}")
                sweep[str(mo)] = dict(wacc, seconds=dt, generate_s=g)
                log(f"suite wallet max_open={mo}: {json.dumps(sweep[str(mo)])}")
            suite["wallet_max_open"] = sweep
        pf.ctx.close()
        log(f"suite: {json.dumps(suite['all'])} held_out {json.dumps(suite['held_out'])}")

    # ---------------------------------------------------------- CPU baseline
    cpu = None
    if rank == 0 and not args.no_cpu:
        cpu = cpu_baseline(b, d_cands, n_states, n_cand, n_vars, args.cpu_seconds, evals_rank / (kern_ms * 1e-3),
                           first, status)
        if keccak is not None:
            keccak["cpu_baseline"] = cpu_keccak(args.cpu_seconds / 2)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded DAG generator + Philox candidates, 50% planted witnesses)",
            "config": {
                "workload": "synthetic: 1M states x 64-node 256-bit constraint DAGs x 256 candidate assignments"
                if n_states == 1 << 20 and n_cand == 256 else f"synthetic: {n_states} states x {n_nodes} nodes x {n_cand} cand",
                "states_per_gpu": n_states, "candidates": n_cand, "op_nodes": n_nodes, "n_vars": n_vars,
                "parallelism": f"dp{world} (contiguous state-id shards, {n_states} per rank; RCCL gather of "
                               "first-SAT)",
                "lds_slots": n_slots, "nominal_ops_per_eval": float(ops_state.mean()),
            },
            # peak = the spec INT32 VALU peak (MI355X_MICROARCH.md); the box's v_add_u32 probe is
            # reported beside it (peak_measured / frac_measured)
            "roofline": {"bound": "valu", "achieved": achieved_tops, "peak": VALU_PEAK_TOPS, "unit": "TOP/s",
                         "frac": achieved_tops / VALU_PEAK_TOPS, "traffic": traffic, "peak_measured": valu_peak,
                         "frac_measured": achieved_tops / valu_peak, "frac_spec": achieved_tops / VALU_PEAK_TOPS,
                         "ops": "nominal INT32 ops of the live DAG nodes (SURVEY.md 8d table) x candidates",
                         "kernel": ENGINE_KERNEL[N.set_eval_engine()] + "(+finalize)", "launch_ms": kern_ms,
                         "evals_per_launch": evals_rank,
                         **({} if div_split is None else {
                             "frac_nondiv": div_split["frac_nondiv"], "div_share": div_split["div_share"],
                             "div_split": div_split})},
            "roofline_hbm": {"achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": achieved_gbs / HBM_PEAK_GBS, "bytes_per_launch": bytes_launch},
            # VALU busy: every issued VALU instruction (dispatch/decode overhead included) x 64 lanes
            "valu_busy": None if valu_busy is None else dict(
                valu_busy, frac=valu_busy["issued_int32_lane_ops_per_s"] / (valu_peak * 1e12),
                frac_spec=valu_busy["issued_int32_lane_ops_per_s"] / (VALU_PEAK_TOPS * 1e12)),
            "cpu_baseline": cpu,
            "results": {"sat_states": sat, "planted_states": int(len(pl)), "planted_found": planted_ok},
            "keccak": keccak,
            "prefilter": prefilter,
            "frontend": frontend,
            "suite": suite,
            "gather": gather,
        }
        # the full record (suite by contract, wallet sweep, latency and stage splits, A/B legs)
        # goes to a side file; stdout carries the headline line the driver parses (< 12 KB)
        detail = args.detail or os.path.join(ROOT, "profiles", "bench_detail_r6.json")
        try:
            os.makedirs(os.path.dirname(os.path.abspath(detail)), exist_ok=True)
            with open(detail, "w") as f:
                json.dump(line, f, indent=1)
        except OSError as e:
            log(f"detail file {detail} not written: {e}")
            detail = None
        head = headline(line, detail)
        text = json.dumps(head)
        if len(text) > HEADLINE_MAX_BYTES:
            raise RuntimeError(f"headline JSON line is {len(text)} bytes (> {HEADLINE_MAX_BYTES})")
        print(text, flush=True)
    if world > 1:
        dist.destroy_process_group()


HEADLINE_MAX_BYTES = 12000
_SUITE_KEYS = ("contracts", "queries", "ref_calls", "z3_calls", "reduction", "contradicted")


def _pick(d, keys):
    return None if d is None else {k: d[k] for k in keys if k in d}


def headline(line: dict, detail_path) -> dict:
    """The driver's one-line record: the contract keys, the eval kernel's roofline and CPU
    baseline, and one level of the Keccak / front-end / suite results.  Everything else
    stays in the detail file whose path it names."""
    head = {k: line[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")}
    rf = dict(line["roofline"])
    rf.pop("div_split", None)
    head["roofline"] = rf
    head["roofline_hbm"] = line["roofline_hbm"]
    head["valu_busy"] = line["valu_busy"]
    head["cpu_baseline"] = line["cpu_baseline"]
    head["results"] = line["results"]
    k = line.get("keccak")
    if k is not None:
        krf = {x: k["roofline"][x] for x in ("bound", "achieved", "peak", "unit", "frac", "traffic", "ops",
                                             "kernel", "launch_ms", "hashes_per_launch")}
        head["keccak"] = {"metric": k["metric"], "value": k["value"], "unit": k["unit"],
                          "hashes_per_gpu": k["hashes_per_gpu"], "roofline": krf,
                          "verified_mismatches": k["verified"]["mismatches"],
                          "verified_checked": k["verified"]["checked"],
                          "cpu_baseline": _pick(k.get("cpu_baseline"), ("value", "unit", "cores", "kind", "sample"))}
    fe = line.get("frontend")
    if fe is not None:
        head["frontend"] = {**_pick(fe, ("states", "seconds", "states_per_s", "first_call_seconds", "sat", "unsat",
                                         "undecided", "solver_call_reduction")),
                            "contradicted": fe["expectations"]["contradicted"],
                            "gpu_wait_ms": fe["stages_ms"].get("gpu_wait_ms"),
                            **({"pipelines2_seconds": fe["pipelines2"]["seconds"],
                                "pipelines2_states_per_s": fe["pipelines2"]["states_per_s"]}
                               if "pipelines2" in fe else {}),
                            "latency_ms": {str(r["states"]): round(r["ms_per_call"], 3) for r in fe["latency"]}}
    pf = line.get("prefilter")
    if pf is not None:
        head["prefilter"] = _pick(pf, ("sample_states", "gpu_sat", "refuted", "fallback", "solver_call_reduction"))
        if pf.get("split_check"):
            head["prefilter"]["split_check"] = _pick(pf["split_check"], ("states", "refuted", "refuted_with_gpu_witness"))
    su = line.get("suite")
    if su is not None:
        head["suite"] = {part: _pick(su.get(part), _SUITE_KEYS) for part in ("all", "tuned", "held_out")}
        head["suite"]["seconds"] = su.get("seconds")
        for extra in ("soundness", "frozen", "config_issues"):
            if extra in su:
                head["suite"][extra] = su[extra]
    head["gather"] = line.get("gather")
    head["detail"] = None if detail_path is None else os.path.relpath(detail_path, ROOT)
    return head


def measure_valu_peak(N, torch, dev, stream, sh) -> float:
    """Best of 3 timed v_add_u32 probe launches (Tops/s)."""
    sink = torch.zeros(4096, dtype=torch.int32, device=dev)
    best = 0.0
    for it in range(4):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        ops = N.probe_valu_dev(400, 4096, vp(sink), sh)
        b.record(stream)
        torch.cuda.synchronize(dev)
        if it:
            best = max(best, ops / (a.elapsed_time(b) * 1e-3) / 1e12)
    return best


def _threads() -> int:
    v = os.environ.get("OMP_NUM_THREADS")
    if v and v.isdigit():
        return int(v)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


def cpu_baseline(b, d_cands, n_states, n_cand, n_vars, target_s, gpu_rate, gpu_first, status):
    """Time the C oracle (OpenMP, all candidates evaluated) on a bounded sample of the same batch,
    and check that its first-SAT words equal the GPU's for every sampled state (a free full-size
    parity check: the sample is the head of the timed batch)."""
    from oracle import coracle

    def sample(k):
        # device layout [s][v][h][c][4] -> host AoS [s][c][v][8]
        words_per_state = n_vars * 2 * n_cand * 4
        dv = d_cands[: k * words_per_state].cpu().numpy().view(np.uint32)
        dv = dv.reshape(k, n_vars, 2, n_cand, 4).transpose(0, 3, 1, 2, 4).reshape(k, n_cand, n_vars, 8)
        sub_off = b["node_offsets"][: k + 1]
        sub_coff = b["const_offsets"][: k + 1]
        return (b["nodes"][: int(sub_off[-1])], sub_off, b["consts"][: int(sub_coff[-1])], sub_coff,
                np.ascontiguousarray(dv))

    k = min(256, n_states)
    t_used = 0.0
    while True:
        nodes, no, cs, co, cands = sample(k)
        t = time.perf_counter()
        ref = coracle.first_sat(nodes, no, cs, co, cands, full=True)
        t_used = time.perf_counter() - t
        if t_used >= target_s * 0.5 or k >= n_states:
            break
        k = min(n_states, int(k * min(8.0, max(2.0, target_s / max(t_used, 1e-3)))))
    rate = k * n_cand / t_used
    ok = status[:k] == 0
    diff = int((np.asarray(ref)[ok] != gpu_first[:k][ok]).sum())
    log(f"cpu baseline: {k} states x {n_cand} cand in {t_used:.1f}s = {rate:.3g} evals/s; "
        f"first-SAT parity {int(ok.sum()) - diff}/{int(ok.sum())}")
    if diff:
        raise RuntimeError(f"{diff} of {int(ok.sum())} sampled states: GPU first-SAT differs from the oracle")
    return {"value": rate, "unit": "evals/s", "cores": _threads(), "kind": "port",
            "sample": f"first {k} states of the rank-0 batch x {n_cand} candidates (all evaluated), "
                      f"oracle/c/oracle.c DAG evaluator, OpenMP", "seconds": t_used,
            "gpu_over_cpu": gpu_rate / rate, "parity_states": int(ok.sum()), "parity_mismatches": diff}


def frontend_latency(pf, SV, cs, sizes=(1, 2, 16, 128, 1024)):
    """Wall time of one Prefilter.check_states call at LASER-like batch sizes (a JUMPI
    fork hands the prune filter <= 2 successors, svm.py:251-255) up to a full worklist,
    cold (no UNSAT core cached), median of repeated calls, with the stage split."""
    out = []
    for n in sizes:
        if n > len(cs):
            break
        reps = max(3, min(30, 2048 // n))
        walls, profs = [], []
        for r in range(reps):
            SV.unsat_cores().reset()
            pf._N.program_cache_clear()  # cold: no lowered program reused across calls
            sub = cs[(r * n) % max(1, len(cs) - n + 1):][:n]
            t = time.perf_counter()
            pf.check_states(sub)
            walls.append(1e3 * (time.perf_counter() - t))
            profs.append(pf.last_profile or {})
        med = int(np.argsort(walls)[len(walls) // 2])
        row = {"states": n, "ms_per_call": walls[med], "states_per_s": 1e3 * n / walls[med], "reps": reps}
        row.update({k: round(v, 3) for k, v in profs[med].items() if k.endswith("_ms")})
        out.append(row)
    return out


def verify_keccak(d_pre, d_dig, kfirst, nk, every):
    """The first 65 536 digests of this rank's range and one in `every` after that (at a
    seeded offset inside each block), bit-exact against the C oracle on the same preimages
    (SURVEY.md 8d config-5 verification protocol)."""
    from oracle import coracle

    head = min(nk, 1 << 16)
    pre = coracle.mapping_preimages(kfirst, head, SEED)
    got = d_dig[: head * 32].cpu().numpy().reshape(head, 32)
    bad = int((got != coracle.keccak256(pre.reshape(-1), head, 64, 64)).any(axis=1).sum())
    gpu_pre_bad = int((d_pre[: head * 64].cpu().numpy().reshape(head, 64) != pre).any(axis=1).sum())
    idx = np.arange(head, nk, max(1, every), dtype=np.int64)
    if len(idx):
        idx = idx + np.random.default_rng(SEED + kfirst).integers(0, max(1, every), size=len(idx))
        idx = idx[idx < nk]
    sampled = 0
    if len(idx):
        import torch

        d_idx = torch.from_numpy(idx).to(d_dig.device)
        got_s = d_dig.view(nk, 32).index_select(0, d_idx).cpu().numpy()
        pre_s = np.concatenate([coracle.mapping_preimages(kfirst + int(i), 1, SEED) for i in idx])
        bad += int((got_s != coracle.keccak256(pre_s.reshape(-1), len(idx), 64, 64)).any(axis=1).sum())
        sampled = len(idx)
    return {"checked": head + sampled, "first": head, "sampled": sampled, "sample_every": every,
            "mismatches": bad + gpu_pre_bad, "against": "oracle/c keccak256 + mapping_preimages"}


def launch_ranks(n: int) -> int:
    """torch.distributed.run with n ranks on this node (127.0.0.1), this script's own argv."""
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log(f"launching {n} ranks: {' '.join(cmd[1:6])} ...")
    return subprocess.call(cmd, env=dict(os.environ))


def dry_run(args, world: int, rank: int):
    """CPU-only pass of the rank plumbing: every rank builds and lowers its own contiguous
    shard of a small synthetic batch, rank 0 gathers the per-rank counts over gloo and prints
    one line (n_gpus = the world size the process group formed)."""
    import torch
    import torch.distributed as dist

    from mythril_amd import _native as N

    dist.init_process_group("gloo")
    world = dist.get_world_size()
    n_states = min(args.states, 256)
    base = rank * n_states
    b = N.synth_generate(SEED, base, n_states, args.nodes, args.cand)
    words, po, status = N.lower(b["nodes"], b["node_offsets"], b["consts"], b["const_offsets"])
    mine = torch.tensor([rank, base, n_states, int((status == 0).sum()), int(words.size)], dtype=torch.int64)
    out = [torch.zeros_like(mine) for _ in range(world)] if rank == 0 else None
    dist.gather(mine, out, dst=0)
    if rank == 0:
        ranks = [t.tolist() for t in out]
        print(json.dumps({"metric": METRIC, "value": None, "unit": "evals/s", "n_gpus": world, "dry_run": True,
                          "world_size_seen": world, "ranks": [{"rank": r[0], "first_state": r[1], "states": r[2],
                                                               "lowered_ok": r[3], "words": r[4]} for r in ranks],
                          "config": {"parallelism": f"dp{world} (contiguous state-id shards, gloo dry run)"}}),
              flush=True)
    dist.destroy_process_group()


def cpu_keccak(target_s):
    from oracle import coracle

    n = 1 << 20
    pre = coracle.mapping_preimages(0, n, SEED)
    while True:
        t = time.perf_counter()
        coracle.keccak256(pre, n, 64, 64)
        dt = time.perf_counter() - t
        if dt >= target_s * 0.5 or n >= 1 << 26:
            break
        n = min(1 << 26, int(n * max(2.0, target_s / max(dt, 1e-3))))
        pre = coracle.mapping_preimages(0, n, SEED)
    rate = n / dt
    log(f"cpu keccak: {n} hashes in {dt:.1f}s = {rate:.3g}/s")
    return {"value": rate, "unit": "hashes/s", "cores": _threads(), "kind": "port",
            "sample": f"{n} mapping-slot preimages, oracle/c/oracle.c keccak256, OpenMP", "seconds": dt}


if __name__ == "__main__":
    main()
