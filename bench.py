"""Benchmark: matched Reserve assignments/s at a 10M-unit queue (BASELINE.json).

One step = one batch of R=65,536 hanging Reserves (config 2 / metric shape:
4 types, prio ~ U[0,1024), 70% one type / 20% two / 10% wildcard) matched
against an HBM-resident 10M-unit work queue through the C ABI
(adlbq_reserve_batch_device), followed by SS_UNRESERVE of every matched unit
(adlbq_unreserve_batch_device) so each step sees the same queue.  Each step
uses a different pre-staged request batch.  Inputs are resident in HBM before
the timed region.

Multi-GPU (torchrun, one process per GPU): every rank is an independent ADLB
server shard with its own 10M-unit queue and its own Reserve stream (the
reference shards queues by server); no collective touches the data
path (weak scaling).  The barrier / max-over-ranks timing is measurement only.

The JSON line carries the roofline of the matching pipeline measured with HIP
events on the launch stream, and the CPU baseline: the oracle (this repo's
linked-list restatement of the reference xq scans) timed on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
STAGES = ["prep", "hist", "thresholds", "prefix", "select", "sort", "targeted", "rank", "chain", "finalize", "park"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--units", type=int, default=10_000_000)
    ap.add_argument("--reserves", type=int, default=65_536)
    ap.add_argument("--types", type=int, default=4)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--equal-prio", action="store_true", help="config-2 variant: all priorities equal")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-stage HIP event timing")
    return ap.parse_args()


def cpu_baseline(w, budget_s: float) -> dict:
    """The oracle (repo restatement of xq's linked-list scans, one core) on the
    same queue: build it once, then time Reserves from the same batch until the
    budget is used.  Per-Reserve cost is ~constant (pinned units are still
    visited), so the sample rate is the rate of the whole batch."""
    import oracle
    from adlb_amd import synth
    o = oracle.Oracle("own")
    o.init(w.user_types, w.num_app_ranks)
    o.replay(synth.put_events(w))
    done, t0 = 0, time.perf_counter()
    chunk = 4
    while time.perf_counter() - t0 < budget_s and done < w.n_reserves:
        k = min(chunk, w.n_reserves - done)
        o.replay(synth.reserve_events(w.r_rank[done:done + k], w.r_types[done:done + k],
                                      w.r_hang[done:done + k]))
        done += k
    el = time.perf_counter() - t0
    return {"value": done / el, "unit": "assignments/s", "cores": 1, "kind": "port",
            "sample": f"first {done} Reserves of the step-0 batch on a {w.n_units}-unit queue "
                      f"({el:.1f} s, oracle/liboracle.so: linked-list restatement of xq.c scans)"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from adlb_amd import synth
    from adlb_amd.server import Server

    R, N = args.reserves, args.units
    w = synth.config2(n_units=N, n_types=args.types, n_reserves=R, seed=args.seed + 1000 * rank,
                      equal_prio=args.equal_prio)
    srv = Server(w.user_types, w.num_app_ranks, max_units=N, device=local)
    # one explicit stream for the library and the torch glue ops (the handle's
    # own stream is non-blocking and would not order against torch's null stream)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    srv.set_stream(stream.cuda_stream)
    units = np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(N, -1),
                      np.zeros(N), np.full(N, -1), np.full(N, -1)], axis=1).astype(np.int32)
    srv.put_batch(units)
    del units
    nb = args.steps + args.warmup
    rng = np.random.default_rng(args.seed + 7 + rank)
    reqs = np.empty((nb, R, 18), np.int32)
    for b in range(nb):
        reqs[b, :, 0] = np.arange(R, dtype=np.int32)
        reqs[b, :, 1] = 1
        reqs[b, :, 2:] = synth.type_vectors(rng, w.user_types, R) if b else w.r_types
    d_reqs = torch.from_numpy(reqs).to(dev)
    d_resp = torch.empty((nb, R, 12), dtype=torch.int32, device=dev)
    d_trip = torch.empty((R, 3), dtype=torch.int32, device=dev)
    d_trip[:, 0] = torch.arange(R, dtype=torch.int32, device=dev)
    d_trip[:, 2] = -1
    torch.cuda.synchronize()

    def step(b):
        srv.reserve_batch_device(R, d_reqs[b].data_ptr(), d_resp[b].data_ptr())
        r = d_resp[b]
        # SS_UNRESERVE every matched unit (wqseqno <= 0 rows are ignored by the kernel)
        torch.where(r[:, 0] == 1, r[:, 5], torch.full_like(r[:, 5], -1), out=d_trip[:, 1])
        srv.unreserve_batch_device(R, d_trip.data_ptr())

    for b in range(args.warmup):
        step(b)
    torch.cuda.synchronize()
    if not args.no_profile:
        srv.profile(True)
        for s in STAGES:
            srv.profile_read(s)  # drain warmup
        base = {s: srv.profile_read(s) for s in STAGES}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(args.warmup, nb):
        step(b)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    matched = int((d_resp[args.warmup:, :, 0] == 1).sum().item())
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        m = torch.tensor([matched], dtype=torch.int64, device=dev)
        dist.all_reduce(m, op=dist.ReduceOp.SUM)
        matched = int(m.item())

    stages = {}
    if not args.no_profile:
        for s in STAGES:
            ms, n = srv.profile_read(s)
            ms0, n0 = base[s]
            if n - n0:
                stages[s] = round((ms - ms0) / (n - n0), 4)
    live = srv.last_scan_units()
    alg_bytes = 16 * live + (72 + 8 + 4) * R          # per matching batch
    batch_ms = sum(stages.values()) if stages else el * 1e3 / args.steps
    scan_ms = stages.get("hist", 0) + stages.get("select", 0)
    dominant = max(stages, key=stages.get) if stages else "batch"
    res = {
        "metric": "matched Reserve assignments/sec at 10M-unit queue",
        "value": matched / el,
        "unit": "assignments/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (seeded config-2 queue and Reserve batches, adlb_amd/synth.py)",
        "config": {"workload": f"config2-metric: {N} units/shard, {args.types} types, prio U[0,1024), "
                               f"{R} hanging Reserves/step (70/20/10 single/pair/wildcard), "
                               f"step = reserve batch + unreserve of matched units",
                   "units_per_shard": N, "reserves_per_step": R, "parallelism": f"shards{world}"},
        "roofline": {
            "bound": "hbm",
            "kernel": "reserve-batch pipeline (all stages of one batch)",
            "achieved": round(alg_bytes / (batch_ms * 1e-3) / 1e9, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(alg_bytes / (batch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": None,
            "algorithmic_bytes": alg_bytes,
            "scan_kernels_GBs": round(16 * live / (scan_ms * 1e-3) / 1e9, 1) if scan_ms else None,
        },
        "stages_ms": stages,
        "chain_rounds_last_batch": srv.stat("chain_rounds"),
        "candidates_last_batch": srv.stat("candidates"),
        "dominant_stage": dominant,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(w, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(res), flush=True)
    srv.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
