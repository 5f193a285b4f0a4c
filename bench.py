"""Benchmark: matched Reserve assignments/s at a 10M-unit queue (BASELINE.json).

One step = one batch of R=65,536 hanging Reserves (config 2 / metric shape:
4 types, prio ~ U[0,1024), 70% one type / 20% two / 10% wildcard) matched
against an HBM-resident 10M-unit work queue through the C ABI
(adlbq_reserve_batch_device), followed by SS_UNRESERVE of every matched unit
(adlbq_unreserve_resp_device) so each step sees the same queue.  Each step
uses a different pre-staged request batch.  Inputs are resident in HBM before
the timed region.

Multi-GPU (torchrun, one process per GPU): every rank is an independent ADLB
server shard with its own 10M-unit queue and its own Reserve stream (the
reference shards queues by server); no collective touches the data
path (weak scaling).  The barrier / max-over-ranks timing is measurement only.

The JSON line carries, per kernel of the reserve batch, the average launch
time measured with HIP events recorded on the launch stream around each launch
(adlbq_profile_*), the algorithmic bytes of that kernel and the
HBM traffic from two separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KB,
FETCH_SIZE doubled per the gfx950 correction) run as child processes before
this process touches the GPU.  `roofline` is the dominant kernel (largest
average launch time).  `cpu_baseline` is the oracle (this repo's linked-list
restatement of the reference xq scans) timed on a bounded sample.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ADLBQ_RESERVE_INTS = 18  # include/adlbq.h

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
STAGES = ["hist", "thresholds", "select", "sort", "targeted", "rank", "chain", "finalize"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process unless set (0: HIP's default)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--units", type=int, default=10_000_000)
    ap.add_argument("--reserves", type=int, default=65_536)
    ap.add_argument("--types", type=int, default=4)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--equal-prio", action="store_true", help="config-2 variant: all priorities equal")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of each CPU baseline sample")
    ap.add_argument("--cpu-cores", type=int, default=min(16, len(os.sched_getaffinity(0))),
                    help="CPU baseline processes (the GPU box's CPU share is 16 per GPU)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-stage HIP event timing")
    ap.add_argument("--profile-every", type=int, default=10,
                    help="timed region: HIP events around the dominant kernel on every n-th batch")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--no-config3", action="store_true", help="skip the config-3 steal-round measurement")
    ap.add_argument("--c3-servers", type=int, default=8, help="config 3: server shards per GPU")
    ap.add_argument("--c3-units", type=int, default=1_562_500, help="config 3: units per server shard")
    ap.add_argument("--c3-reserves", type=int, default=8192, help="config 3: Reserves per shard per step")
    ap.add_argument("--c3-k", type=int, default=1024, help="config 3: exported units per type per shard")
    ap.add_argument("--c3-steps", type=int, default=40)
    ap.add_argument("--c3-rqcap", type=int, default=2048, help="config 3: parked Reserves per shard a round considers (~820 park per step)")
    ap.add_argument("--c3-threads", type=int, default=0, help="config 3: enqueue the shards' batches from threads")
    ap.add_argument("--c3-streams", type=int, default=1,
                    help="config 3: HIP streams the GPU's shards share (round robin); 0 = one per shard")
    ap.add_argument("--c3-group", type=int, default=1,
                    help="config 3: every shard's Reserve batch as one launch per kernel (adlbq_reserve_group_device)")
    ap.add_argument("--c3-warmup", type=int, default=8, help="config 3: untimed steps (rq and export buffers grow)")
    ap.add_argument("--c3-parts", action="store_true", help="config 3: synchronise and time each part of every step")
    ap.add_argument("--config3-only", action="store_true", help="only the config-3 leg (profiling)")
    ap.add_argument("--c3-param", action="append", default=[], metavar="NAME=V",
                    help="config 3: adlbq_set_param on every shard (repeatable)")
    ap.add_argument("--no-config4", action="store_true", help="skip the config-4 measurement")
    ap.add_argument("--no-config2", action="store_true", help="skip the config-2 (1M-unit) leg")
    ap.add_argument("--c2-units", type=int, default=1_000_000, help="config 2: units")
    ap.add_argument("--c2-steps", type=int, default=20, help="config 2: timed steps")
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 stream measurement")
    ap.add_argument("--no-wide", action="store_true", help="skip the more-than-64-types leg")
    ap.add_argument("--diag-same-batch", action="store_true",
                    help="diagnostic: every metric step on the same request / response buffers (cache residency)")
    ap.add_argument("--wide-only", action="store_true", help="only the more-than-64-types leg")
    ap.add_argument("--wide-types", type=int, default=100)
    ap.add_argument("--wide-units", type=int, default=200_000)
    ap.add_argument("--wide-reserves", type=int, default=4096)
    ap.add_argument("--config5-only", action="store_true", help="only the config-5 leg")
    ap.add_argument("--c5-shards", type=int, default=8, help="config 5: server shards (one steal group)")
    ap.add_argument("--c5-ranks", type=int, default=4096, help="config 5: app ranks")
    ap.add_argument("--c5-events", type=int, default=10_000_000, help="config 5: events over all shards")
    ap.add_argument("--c5-round-every", type=int, default=10_000, help="config 5: events between steal rounds")
    ap.add_argument("--c5-k", type=int, default=64, help="config 5: steal export depth per (shard, type)")
    ap.add_argument("--c5-q0", type=int, default=128, help="config 5: generator's target queue depth")
    ap.add_argument("--config4-only", action="store_true", help="only the config-4 leg (profiling)")
    ap.add_argument("--c4-units", type=int, default=10_000_000, help="config 4: units (80%% targeted)")
    ap.add_argument("--c4-steps", type=int, default=5)
    ap.add_argument("--c4-puts", type=int, default=2048,
                    help="config 4: Puts per step before the Reserve batch (same mix: 80%% targeted), so the "
                         "targeted index update is timed")
    ap.add_argument("--c4-chain-passes", type=int, default=None,
                    help="config 4: in-launch neighbour passes of the ordered choice's round 0 (adlbq 'chain_passes')")
    ap.add_argument("--c4-chain-rounds", type=int, default=None,
                    help="config 4: ordered-choice round launches after round 0 (adlbq 'chain_rounds')")
    ap.add_argument("--chain-rounds", type=int, default=None, help="metric leg: adlbq 'chain_rounds'")
    ap.add_argument("--no-host-path", action="store_true",
                    help="metric leg: skip the host-buffer (PCIe-inclusive) adlbq_reserve_batch measurement")
    ap.add_argument("--chain-per-batch", action="store_true",
                    help="metric leg: the chain's counters of every timed batch (untimed replay)")
    ap.add_argument("--chain-stamps", action="store_true",
                    help="metric leg: after the timed region, one batch with the chain's phase stamps (diagnostic)")
    ap.add_argument("--c4-chain-modes", type=int, default=None, help="config 4: adlbq 'chain_modes'")
    ap.add_argument("--chain-passes", type=int, default=None, help="metric leg: adlbq 'chain_passes'")
    ap.add_argument("--chain-modes", type=int, default=None, help="metric leg: adlbq 'chain_modes'")
    ap.add_argument("--rank-in-select", type=int, default=None, help="metric leg: adlbq 'rank_in_select'")
    ap.add_argument("--chain-warm", type=int, default=None, help="metric leg: adlbq 'chain_warm' (0, 256, 512)")
    ap.add_argument("--c4-param", action="append", default=[], metavar="NAME=V",
                    help="config-4 leg: any adlbq_set_param (diagnostics), repeatable")
    ap.add_argument("--kernel-stamps", action="store_true", help="diagnostic: phase stamps of passes 1 and 2 (us)")
    ap.add_argument("--diag-first", action="store_true",
                    help="diagnostic (never a reported number): host sections of the first timed step")
    ap.add_argument("--param", action="append", default=[], metavar="NAME=V",
                    help="metric leg: any adlbq_set_param (diagnostics), repeatable")
    ap.add_argument("--c4-chain-stats", action="store_true",
                    help="config 4: after the timed region, replay each batch alone and report its chain counters")
    return ap.parse_args()


# stage (adlbq_profile_read name) -> kernel symbol of that launch
KERNEL_OF = {"hist": "k_prep_hist", "thresholds": "k_thresholds",
             "select": "k_select_wave", "sort": "k_keybits + merged hipcub radix sort",
             "targeted": "k_targeted_idx", "rank": "k_rank", "chain": "k_chain0", "finalize": "k_finalize"}


def _kernel_base(name: str) -> str:
    n = name.strip().strip('"')
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0]


def pmc_traffic(args) -> dict | None:
    """HBM bytes per launch of each kernel from two rocprofv3 PMC passes over a
    short run of the same workload (child processes; this process has not
    touched the GPU yet).  FETCH_SIZE/WRITE_SIZE are KB; FETCH_SIZE is doubled
    (gfx950 reports half of wide streaming reads, MI355X_MICROARCH.md).  The mean
    over the steady-state launches (the first launch of each kernel dropped)."""
    prof = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3")
                                         else None)
    if prof is None:
        return None
    child = [sys.executable, os.path.abspath(__file__), "--steps", "2", "--warmup", "1", "--no-cpu", "--no-pmc",
             "--no-config3", "--no-config4", "--no-config5", "--no-wide",
             "--no-profile", "--no-host-path", "--units", str(args.units), "--reserves", str(args.reserves), "--types",
             str(args.types), "--seed", str(args.seed)] + (["--equal-prio"] if args.equal_prio else [])
    out = {}
    tmp = tempfile.mkdtemp(prefix="adlbq_pmc_")
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr)
            r = subprocess.run([prof, "--pmc", ctr, "-d", d, "-o", "run", "--output-format", "csv", "--"] + child,
                               stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=600,
                               env=dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp")))
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if r.returncode != 0 or not files:
                return None
            per = {}
            for row in csv.DictReader(open(files[0])):
                per.setdefault(_kernel_base(row["Kernel_Name"]), []).append(float(row["Counter_Value"]))
            scale = 2048.0 if ctr == "FETCH_SIZE" else 1024.0
            for k, v in per.items():
                v = v[1:] if len(v) > 1 else v
                out.setdefault(k, {})[ctr] = scale * sum(v) / len(v)
    except (OSError, subprocess.SubprocessError, KeyError, ValueError):
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return {k: v.get("FETCH_SIZE", 0.0) + v.get("WRITE_SIZE", 0.0) for k, v in out.items()
            if "FETCH_SIZE" in v and "WRITE_SIZE" in v}


def traffic_of(pmc, stage):
    if not pmc:
        return None
    # the select stage is k_select_wave (T <= 8), else k_select_open
    for want in (KERNEL_OF[stage], "k_select_open") if stage == "select" else (KERNEL_OF[stage],):
        hits = [v for k, v in pmc.items() if k == want or k.startswith(want + "_small<") or k.startswith(want + "<")]
        if len(hits) == 1:
            return round(hits[0])
    return None


def _exact_check():
    """tests/exact_check.py: the size-independent parity checker (test
    infrastructure; run after the timed region on one timed batch per leg)."""
    d = os.path.join(ROOT, "tests")
    if d not in sys.path:
        sys.path.insert(0, d)
    import exact_check
    return exact_check


def parity_of(fn) -> dict:
    """{"parity": True, "parity_detail": ...} if fn() returns, else False with the failure."""
    try:
        return {"parity": True, "parity_detail": fn()}
    except AssertionError as e:
        return {"parity": False, "parity_detail": f"AssertionError: {e}"}


def all_ranks_true(ok: bool) -> bool:
    import torch
    import torch.distributed as dist
    from adlb_amd import shards
    t = torch.tensor([1 if ok else 0], dtype=torch.int64, device=shards._dev_of(dist.get_backend()))
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def check_units(ec, w, seq, avail, reqs18, resp, server_rank):
    """One Reserve batch against the sequential result (exact_check.check_batch,
    every TA_RESERVE_RESP field)."""
    n = w.u_type.size
    common = np.empty((n, 3), np.int32)
    common[:, 0], common[:, 1:] = 0, -1
    return ec.check_batch(w.user_types, w.u_type, w.u_prio, w.u_target, seq, avail, reqs18[:, 0], reqs18[:, 2:],
                          reqs18[:, 1], resp, u_len=w.u_len, u_answer=w.u_answer, u_common=common,
                          server_rank=server_rank)


def cpu_baseline(w, budget_s: float, seed: int, cores: int, equal_prio: bool = False) -> dict:
    """The CPU baseline on the GPU box's host: the reference's
    own src/xq.c (oracle/_ref/libxqref.so, built from /root/reference in the
    build container; this repo's restatement oracle/liboracle.so when that is
    absent) on the metric queue.  Per-Reserve cost is ~constant (pinned units
    are still visited), so a sample's rate is the batch's rate.
      value            `cores` independent processes, each with its own replica
                       of the whole queue (aggregate Reserves/s);
      one_core         one process, one replica;
      sharded          the ADLB-natural split: `cores` servers with 1/cores of
                       the units each, Reserves routed round robin;
    ns_per_node = seconds per Reserve / (2 x units held): the reference scans
    the list twice per Reserve (xq.c:219-247 then 190-217)."""
    import multiprocessing as mp
    import oracle
    from oracle.baseline import sample
    N, T, R = w.n_units, int(w.user_types.size), w.n_reserves

    def pick(units):
        # the reference build holds its queue under adlb.c's own allocation cap (max_malloc =
        # 500 MB until ADLB_Server runs, adlb.c:218, 3439-3452): ~140 B per unit with payload
        return "ref" if oracle.available("ref") and units * 150 < 4.5e8 else "own"

    def summary(res, what, kind):
        done = sum(r[0] for r in res)
        rate = sum(r[0] / r[1] for r in res if r[1] > 0)
        per = [r[1] / max(r[0], 1) / (2.0 * r[2]) * 1e9 for r in res]
        src = ("oracle/_ref/libxqref.so (the reference's src/xq.c, compiled in the build container)" if kind == "ref"
               else "oracle/liboracle.so (this repo's restatement of xq.c)")
        return {"value": rate, "unit": "assignments/s", "cores": len(res), "reserves_timed": done,
                "kind": "reference" if kind == "ref" else "port", "ns_per_node": round(float(np.median(per)), 3),
                "sample": f"{what}; {src}"}

    k1, ks = pick(N), pick(N // max(cores, 1))
    one = summary([sample((k1, N, T, R, seed, equal_prio, 0, 1, budget_s))],
                  f"first Reserves of the step-0 batch on the {N}-unit queue, one process, {budget_s:.0f} s", k1)
    ctx = mp.get_context("spawn")  # this process holds the GPU: no fork
    lim = 10 * budget_s + 300
    with ctx.Pool(cores) as pool:
        rep = summary(pool.map_async(sample, [(k1, N, T, R, seed, equal_prio, 0, 1, budget_s)] * cores).get(lim),
                      f"{cores} processes x one {N}-unit replica each, {budget_s:.0f} s each", k1)
        shd = summary(pool.map_async(sample, [(ks, N, T, R, seed, equal_prio, c, cores, budget_s)
                                              for c in range(cores)]).get(lim),
                      f"{cores} server processes x {N // cores} units (units and Reserves dealt round robin), "
                      f"{budget_s:.0f} s each", ks)
    return {"value": rep["value"], "unit": "assignments/s", "cores": cores, "kind": rep["kind"],
            "sample": rep["sample"], "ns_per_node": rep["ns_per_node"],
            "one_core": one, "sharded": shd,
            "host_cpus": {"affinity": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count()}}


def cpu_baseline_config(name, jobs, budget_s: float, what: str, units_per_proc: int) -> dict:
    """CPU baselines of configs 3 and 4 on the GPU box's host (BASELINE.md:
    configs 2-5 in one table): len(jobs) processes in parallel, each building
    its queue in the reference's own xq.c (oracle/_ref/libxqref.so) where
    adlb.c's allocation cap allows, this repo's restatement otherwise, and
    timing Reserves of the same workload for budget_s seconds.  value =
    aggregate Reserves/s; ns_per_node as cpu_baseline."""
    import multiprocessing as mp
    from oracle.baseline import sample
    ctx = mp.get_context("spawn")  # this process holds the GPU: no fork
    with ctx.Pool(len(jobs)) as pool:
        res = pool.map_async(sample, jobs).get(10 * budget_s + 600)
    kind = jobs[0][1]
    rate = sum(r[0] / r[1] for r in res if r[1] > 0)
    per = [r[1] / max(r[0], 1) / (2.0 * r[2]) * 1e9 for r in res]
    src = ("oracle/_ref/libxqref.so (the reference's src/xq.c, compiled in the build container)" if kind == "ref"
           else "oracle/liboracle.so (this repo's restatement of xq.c)")
    return {"value": rate, "unit": "assignments/s", "cores": len(jobs), "kind": "reference" if kind == "ref" else "port",
            "reserves_timed": int(sum(r[0] for r in res)), "ns_per_node": round(float(np.median(per)), 3),
            "units_per_process": units_per_proc, "sample": f"{name}: {what}; {src}; {budget_s:.0f} s each"}


def _ref_fits(units: int) -> str:
    import oracle
    # adlb.c's max_malloc is 500 MB until ADLB_Server runs (adlb.c:218, 3439-3452): ~150 B per unit with payload
    return "ref" if oracle.available("ref") and units * 150 < 4.5e8 else "own"


def bench_config3(args, torch, dist, world, rank, local, dev):
    """Config 3: c3_servers server shards per GPU (64 over 8
    GPUs), c3_units units each, per-shard type skew so ~10% of the Reserves
    have no local match.  One step = every shard's Reserve batch (concurrent
    streams), then one steal round over all shards (device top-k export, one
    all-gather over RCCL, the merge, grants), then SS_UNRESERVE of every
    matched and stolen unit so each step sees the same queues.  Reports
    (local + stolen assignments) / s and the steal round's share."""
    from adlb_amd import shards, synth
    from adlb_amd.server import ReserveGroup, Server

    SL, N, R, k = args.c3_servers, args.c3_units, args.c3_reserves, args.c3_k
    S, T = SL * world, 4
    W3 = max(1, args.c3_warmup)
    nb = args.c3_steps + W3
    srvs, streams, d_reqs, d_resp, wks, h_reqs = [], [], [], [], [], []
    for j in range(SL):
        idx = rank * SL + j
        w = synth.config3_shard(idx, S, N, T, R, seed=args.seed)
        srv = Server(w.user_types, w.num_app_ranks, S, idx, max_units=N, device=local)
        for kv in args.c3_param:
            k_, v_ = kv.split("=", 1)
            srv.set_param(k_, int(v_))
        nst = args.c3_streams if args.c3_streams > 0 else SL
        st = streams[j % nst] if j >= nst else torch.cuda.Stream(dev)
        srv.set_stream(st.cuda_stream)
        srv.put_batch(np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(N, -1),
                                np.zeros(N), np.full(N, -1), np.full(N, -1)], axis=1).astype(np.int32))
        rng = np.random.default_rng(args.seed + 31 * idx)
        reqs = np.empty((nb, R, 18), np.int32)
        for b in range(nb):
            reqs[b, :, 0] = w.r_rank
            reqs[b, :, 1] = 1
            reqs[b, :, 2:] = synth.config3_types(rng, T, idx, R) if b else w.r_types
        with torch.cuda.stream(st):
            d_reqs.append(torch.from_numpy(reqs).to(dev))
            d_resp.append(torch.empty((nb, R, 12), dtype=torch.int32, device=dev))
        srvs.append(srv)
        streams.append(st)
        wks.append(w)
        h_reqs.append(reqs)
    torch.cuda.synchronize()
    keep, parts, sparts = [], {"batches": 0.0, "steal": 0.0, "unreserve": 0.0}, {}

    group = shards.StealGroup(srvs, k, rqcap=args.c3_rqcap)
    pool = ThreadPoolExecutor(max_workers=len(srvs)) if args.c3_threads else None

    class Res:
        def __init__(self, decided, settled):
            self.decided, self.settled = decided, settled

    # device pointers of every (shard, batch) once: no tensor views inside the timed loop
    p_req = [[d_reqs[j][b].data_ptr() for b in range(nb)] for j in range(len(srvs))]
    p_resp = [[d_resp[j][b].data_ptr() for b in range(nb)] for j in range(len(srvs))]

    def enqueue(j, b):
        srvs[j].reserve_batch_device(R, p_req[j][b], p_resp[j][b])

    rgroup = ReserveGroup(srvs) if args.c3_group else None
    packed = ([rgroup.pack([R] * len(srvs), [p_req[j][b] for j in range(len(srvs))],
                           [p_resp[j][b] for j in range(len(srvs))]) for b in range(nb)] if rgroup else None)

    def step(b, timed_parts=False):
        t0 = time.perf_counter()
        if rgroup is not None:
            rgroup.reserve_device(packed=packed[b])
        elif pool is not None:
            list(pool.map(lambda j: enqueue(j, b), range(len(srvs))))
        else:
            for j in range(len(srvs)):
                enqueue(j, b)
        if timed_parts:
            parts["batches_enqueue"] = parts.get("batches_enqueue", 0.0) + time.perf_counter() - t0
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        tm = sparts if timed_parts else None
        nd, ns = group.round(timing=tm)
        t2 = time.perf_counter()
        if rgroup is not None:
            rgroup.unreserve_resp_device(packed=packed[b])
        else:
            for j, srv in enumerate(srvs):
                srv.unreserve_resp_device(R, p_req[j][b], p_resp[j][b])
        group.unreserve_grants()
        if timed_parts:
            for key in ("copy_ns", "merge_ns", "apply_ns"):
                sparts["settle_" + key[:-3]] = sparts.get("settle_" + key[:-3], 0.0) + group.stat(key) * 1e-9
        if timed_parts:
            torch.cuda.synchronize()
            parts["batches"] += t1 - t0
            parts["steal"] += t2 - t1
            parts["unreserve"] += time.perf_counter() - t2
        return Res(nd, ns)

    for b in range(W3):                  # warm-up
        step(b)
    torch.cuda.synchronize()
    keep.clear()
    if args.c3_parts:                    # per-part timing, synchronised (untimed)
        for b in range(W3, nb):
            step(b, timed_parts=True)
        torch.cuda.synchronize()
        keep.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    HACC = ("tables", "rq_cap", "rq_waits", "rq_reclaims", "scan_cap", "sort", "total")
    HACC_MS = ("tables", "rq_cap", "scan_cap", "sort", "total")
    hacc0 = {k: sum(srv.stat("hacc:" + k) for srv in srvs) for k in HACC}
    t0 = time.perf_counter()
    settled = decided = 0
    for b in range(W3, nb):
        r = step(b)
        settled += r.settled
        decided += r.decided
    last_round = r
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    local_matched = int(sum(int((d[W3:, :, 0] == 1).sum().item()) for d in d_resp))
    parked = int(sum(int((d[W3:, :, 0] == 0).sum().item()) for d in d_resp))
    if world > 1:
        el, local_matched = shards.reduce_step_timing(el, local_matched)
        _, parked = shards.reduce_step_timing(0.0, parked)
    steps = nb - W3
    out = {
        "workload": f"config3: {S} server shards ({SL}/GPU) x {N} units, {T} types with one type missing per "
                    f"shard, {R} Reserves/shard/step (~10% only the missing type), steal round k={k}, rqcap={args.c3_rqcap}"
                    + (", the shards' batches as one launch per kernel" if rgroup else ""),
        "value": (local_matched + settled) / el,
        "unit": "assignments/s",
        "ms_per_step": el * 1e3 / steps,
        "local_matched_per_step": local_matched / steps,
        "parked_per_step": parked / steps,
        "stolen_per_step": settled / steps,
        "decided_per_step": decided / steps,
        "parts_ms_per_step": ({kk: round(v * 1e3 / (nb - W3), 3) for kk, v in {**parts, **sparts}.items()}
                              if args.c3_parts else None),
        "reserve_host_sections_ms_per_step": {k: round((sum(srv.stat("hacc:" + k) for srv in srvs) - hacc0[k]) / 1e6
                                                       / (nb - W3), 4) for k in HACC if k in HACC_MS},
        "reserve_host_counts_per_step": {k: round((sum(srv.stat("hacc:" + k) for srv in srvs) - hacc0[k]) / (nb - W3), 3)
                                         for k in HACC if k not in HACC_MS},
        "scaling": "weak",
    }
    out["rq_per_shard"] = {"cap": [srv.stat("rq_cap") for srv in srvs],
                           "slots": [srv.stat("rq_slots") for srv in srvs],
                           "device_reclaims": [srv.stat("rq_reclaims") for srv in srvs],
                           "sync_reclaims": [srv.stat("hacc:rq_reclaims") for srv in srvs],
                           "waits": [srv.stat("hacc:rq_waits") for srv in srvs],
                           "last_wait": [{k: srv.stat("hacc:rqw_" + k) for k in ("need", "cap", "landed", "snap_rq_n",
                                                                                "since", "stale")} for srv in srvs[:2]]}
    bg, bd = group.check()
    out["steal_check"] = {"bad_grants": bg, "bad_deletes": bd}
    par = parity_of(lambda: config3_parity(_exact_check(), wks, h_reqs, d_resp, nb - 1, group, last_round,
                                           rank * SL, S, decided, settled, nb - W3))
    if world > 1:
        par["parity"] = all_ranks_true(par["parity"])
    out.update(par)
    if not par["parity"]:
        out["value"] = None
    group.close()
    if pool is not None:
        pool.shutdown()
    for srv in srvs:
        srv.close()
    return out


def config3_parity(ec, wks, h_reqs, d_resp, b, group, last, idx0, S, decided, settled, steps):
    """The last timed step of the config-3 leg: every local shard's Reserve
    batch against the sequential result, then the steal round that followed
    it against the serial RFR exchanges (exact_check.serial_steal_expect).
    Needs a clean state before that step: every round decided and settled all
    parked Reserves (so none was left parked) and every match and grant was
    unreserved."""
    R = h_reqs[0].shape[1]
    resp = [d[b].cpu().numpy() for d in d_resp]
    nparked = sum(int((r[:, 0] == 0).sum()) for r in resp)
    assert decided == settled, f"{decided - settled} decided Reserves were not settled (left parked)"
    assert last.decided == last.settled, "the checked round left Reserves parked"
    out = {"batches": []}
    for j, (w, rq, r) in enumerate(zip(wks, h_reqs, resp)):
        n = w.u_type.size
        out["batches"].append(check_units(ec, w, np.arange(1, n + 1, dtype=np.int64), np.ones(n, bool), rq[b], r,
                                          w.num_app_ranks + idx0 + j)["matched"])
    if S != len(wks):  # several processes: the round's other shards are not held here
        out["round"] = "per-process batches only (the round spans other processes' shards)"
        return out
    assert last.decided == nparked, "the checked round did not consider every parked Reserve"
    shards_ = []
    for j, (w, rq, r) in enumerate(zip(wks, h_reqs, resp)):
        n = w.u_type.size
        taken = np.zeros(n, bool)
        taken[r[r[:, 0] == 1, 5] - 1] = True
        park = np.nonzero(r[:, 0] == 0)[0]
        rows = np.empty((park.size, 18), np.int32)
        rows[:, 0], rows[:, 1], rows[:, 2:] = r[park, 10], rq[b][park, 0], rq[b][park, 2:]
        rows = rows[np.argsort(rows[:, 0], kind="stable")]
        assert (w.u_target < 0).all()
        shards_.append({"type": w.u_type, "prio": w.u_prio, "seq": np.arange(1, n + 1), "len": w.u_len,
                        "answer": w.u_answer, "avail": ~taken, "rq": rows})
    exp = ec.serial_steal_expect(wks[0].user_types, wks[0].num_app_ranks, shards_, last.decided)
    got = group.responses()
    assert got.shape == exp.shape, f"round: {got.shape[0]} settlements, serial model {exp.shape[0]}"
    assert np.array_equal(got, exp), "round settlements differ from the serial RFR exchanges"
    out["round_settled"] = int(exp.shape[0])
    return out


def host_latency_table(srv, torch, dev, reqs, d_reqs, d_resp, sizes=(1, 16, 256, 4096), reps=20):
    """Latency of the synchronous host-buffer entry point libadlb.so calls
    (adlbq_reserve_batch: requests from host memory, responses back) against
    the batch size R, on the metric queue: median and p90 over `reps` calls of
    the first R Reserves of one batch, each followed (untimed) by SS_UNRESERVE
    of its matches so every call sees the same queue."""
    out = []
    for r in sizes:
        if r > reqs.shape[0]:
            continue
        sub = np.ascontiguousarray(reqs[:r])
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            resp = srv.reserve_batch(sub)
            ts.append(time.perf_counter() - t)
            d_resp[:r].copy_(torch.from_numpy(resp).to(dev))
            srv.unreserve_resp_device(r, d_reqs.data_ptr(), d_resp.data_ptr())
            srv.sync()
        ts = np.sort(np.array(ts)) * 1e3
        out.append({"R": r, "ms_median": round(float(np.median(ts)), 4),
                    "ms_p90": round(float(ts[int(0.9 * (len(ts) - 1))]), 4),
                    "assignments_per_s_median": round(r / (float(np.median(ts)) * 1e-3), 1)})
    return out


def zipf_type_sets(rng, n_types, R, lo=1, hi=4):
    """(R, 16) request vectors of lo..hi distinct types drawn without replacement
    with Zipf(1.1) weights (Gumbel top-k: the same law as synth.type_vectors with
    ntypes_range, vectorised), padded with -2."""
    from adlb_amd import synth
    w = synth.zipf_weights(n_types)
    keys = np.log(w)[None, :] + rng.gumbel(size=(R, n_types))
    order = np.argsort(-keys, axis=1)[:, :hi].astype(np.int32)
    k = rng.integers(lo, hi + 1, size=R)
    out = np.full((R, 16), -2, np.int32)
    for c in range(hi):
        sel = k > c
        out[sel, c] = order[sel, c]
    return out


def bench_config5(args, torch, dist, world, rank, local, dev):
    """Config 5 at its SURVEY §8(d) shape: S server shards serving tsp.c-style
    branch-and-bound streams (oracle/gen_c5.c: work Puts at prio 1+len, bound
    updates at prio 999999999 targeted to their home shard, Reserves {2, 1} /
    {1} / wildcard that mostly hang, Gets on the holding shard), ~c5_events
    events in all, and every c5_round_every events a qmstat snapshot exchange
    and a steal round over all shards (SS_RFR, adlb.c:1802-1933).  The streams
    react to outcomes and steals, so they are recorded first with the oracle as
    every shard (untimed; the C generator); the engine then serves them through
    adlbsrv_replay_rounds (adlb_replay.cpp): one host thread and HIP stream per
    shard issuing device-side batches with no host sync per call, one
    steal-group round (export depth c5_k) at each marker.  Every output and
    every steal is checked against the oracle's.  Reports events/s; the CPU
    figure is the oracle serving the same stream (generator in the loop)."""
    import oracle
    from adlb_amd import replay, shards
    from adlb_amd.server import Server
    S, A = args.c5_shards, args.c5_ranks
    kw = dict(n_shards=S, n_ranks=A, round_every=args.c5_round_every, k=args.c5_k, q0=args.c5_q0)
    t0 = time.perf_counter()
    d = oracle.gen_config5(n_events=args.c5_events, seed=args.seed + 101 * rank, **kw)
    gen_s = time.perf_counter() - t0
    warm = oracle.gen_config5(n_events=min(args.c5_events, 100_000), seed=args.seed + 7 + 101 * rank, **kw)
    c5_stats = {}

    def run(dd, closed=False, cl_stats=None):
        srvs = [Server(dd["user_types"], A, S, s_, max_units=1 << 16, device=local) for s_ in range(S)]
        try:
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            w0 = time.perf_counter()
            got, steals, sec, calls = replay.replay_rounds(srvs, dd["traces"], k=args.c5_k, rqcap=A, closed=closed,
                                                           stats=cl_stats)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            wall_s = time.perf_counter() - w0
            # reserve batches served by the one-workgroup choice, and the host sections of the reserve call (ms)
            c5_stats.clear()
            c5_stats["small_batches"] = sum(s_.stat("small_batches") for s_ in srvs)
            dg = [sum(s_.stat(f"diag{k}") for s_ in srvs) for k in range(8)]
            c5_stats["small_units_per_call"] = round(dg[0] / max(dg[4], 1), 1)
            c5_stats["small_reserves_per_call"] = round(dg[1] / max(dg[4], 1), 1)
            c5_stats["small_us_to_sorted"] = round(dg[2] / max(dg[4], 1) / 100, 2)  # 100 MHz constant clock
            c5_stats["small_us_serial"] = round(dg[3] / max(dg[4], 1) / 100, 2)
            # k_put_match_blk over the run (first chunk of each batch with something parked)
            c5_stats["put_match_staged_entries"] = dg[5]
            c5_stats["put_match_stage_ms"] = round(dg[6] / 1e5, 1)
            c5_stats["put_match_match_ms"] = round(dg[7] / 1e5, 1)
            for sec_name in ("total", "tindex", "l_scan", "l_rank", "l_chain", "l_fin", "tables", "sort"):
                c5_stats["host_ms_" + sec_name] = round(sum(s_.stat("hacc:" + sec_name) for s_ in srvs) / 1e6, 1)
            return got, steals, sec, calls, wall_s
        finally:
            for s_ in srvs:
                s_.close()

    run(warm)  # kernels loaded, pools sized
    got, steals, sec, calls, wall = run(d)
    st_key = lambda a: np.sort(np.ascontiguousarray(a).view([("", a.dtype)] * 15), axis=0)

    def parity(got_, steals_):
        same_ = all(np.array_equal(g, e) for g, e in zip(got_, d["outputs"]))
        same_st = steals_.shape == d["steals"].shape and np.array_equal(st_key(steals_), st_key(d["steals"]))
        return bool(same_), bool(same_st)

    same, same_steals = parity(got, steals)
    ok = bool(same and same_steals)
    total = int(d["events"])
    el = sec
    # closed loop: every Get waits for the reply it depends on and takes its wqseqno from it
    cl = {}
    try:
        run(warm, closed=True)
        got_c, steals_c, sec_c, _, _ = run(d, closed=True, cl_stats=cl)
        same_c, same_steals_c = parity(got_c, steals_c)
        ok_c = same_c and same_steals_c and cl.get("wqseqno_mismatch", 1) == 0
        el_c = sec_c
    except RuntimeError as e:  # reported in the line (value null, parity false), not a lost bench line
        cl["error"] = str(e)
        ok_c, el_c = False, 0.0
    if world > 1:
        el_c, _ = shards.reduce_step_timing(el_c, total)
        ok_c = all_ranks_true(ok_c)
        el, total = shards.reduce_step_timing(el, total)
        ok = all_ranks_true(ok)
    closed_loop = {"value": total / el_c if ok_c else None, "unit": "events/s", "seconds": round(el_c, 4),
                   "parity": bool(ok_c), **cl,
                   "note": "each Get issued only after the TA_RESERVE_RESP (or put-side match, or steal answer) it "
                           "depends on has landed in mapped host memory, its wqseqno taken from that reply "
                           "(tsp.c:157-162); Puts and Reserves as in the open-loop run"}
    cpu_sh = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu_sh = cpu_baseline_c5(d, A, S)
    return {"workload": f"config5: {S} server shards x tsp-style streams ({A} app ranks, {int(d['events'])} events, "
                        f"a qmstat exchange + steal round every {args.c5_round_every} events: {int(d['rounds'])} rounds, "
                        f"{d['steals'].shape[0]} steals, {int(d['stopped'])} stopped at export depth {args.c5_k}) "
                        f"per GPU; one host thread + HIP stream per shard, no host sync per call",
            "value": total / el if ok else None, "unit": "events/s", "seconds": el,
            "wall_incl_staging_s": round(wall, 4), "events": total, "calls": int(sum(calls)),
            "events_per_call": round(int(d["events"]) / max(int(sum(calls)), 1), 2),
            "host_seconds": replay.last_rounds_prof(),
            "engine": dict(c5_stats),
            "parity": ok, "parity_outputs": bool(same), "parity_steals": bool(same_steals),
            "closed_loop": closed_loop,
            "cpu_baseline": cpu_sh,
            "cpu_generator_events_per_s": int(d["events"]) / gen_s,
            "cpu_generator_note": "the stream generator (gen_c5.c) with the oracle serving every shard, one core: "
                                  "generation cost included, not a server baseline",
            "scaling": "weak"}


def cpu_baseline_c5(d, A, S) -> dict:
    """Config 5's CPU baseline in the ADLB-natural layout: S server processes,
    one per shard, each replaying its own shard's stream with its part of every
    steal round inlined (oracle/gen_c5.c xtrace: its SS_RFR answers as donor,
    its rq deletions as requester) through this repo's restatement of xq.c /
    adlb.c's handlers (oracle/liboracle.so), in parallel.  value = the stream's
    events / the slowest process's seconds.  No MPI messaging is charged, so
    this favours the CPU."""
    import multiprocessing as mp
    import tempfile
    from oracle.baseline import c5_shard
    tmp = tempfile.mkdtemp(prefix="c5cpu_")
    try:
        jobs = []
        for s_ in range(S):
            path = os.path.join(tmp, f"x{s_}.npy")
            np.save(path, d["xtraces"][s_])
            jobs.append((path, d["user_types"], A, S, s_))
        ctx = mp.get_context("spawn")  # this process holds the GPU: no fork
        with ctx.Pool(S) as pool:
            res = pool.map_async(c5_shard, jobs).get(1200)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    slowest = max(r[1] for r in res)
    return {"value": int(d["events"]) / slowest, "unit": "events/s", "cores": S, "kind": "port",
            "seconds_slowest": round(slowest, 4), "seconds_per_process": [round(r[1], 4) for r in res],
            "host_cpus": {"affinity": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count()},
            "sample": f"the whole config-5 stream ({int(d['events'])} events): {S} server processes, one per shard, "
                      f"each replaying its shard's events and its part of every steal round through "
                      f"oracle/liboracle.so (this repo's restatement of xq.c / adlb.c's handlers); no MPI cost"}


def bench_config2(args, torch, dist, world, rank, local, dev):
    """BASELINE config 2 at its own size: a 1,000,000-unit queue (4 types, prio
    U[0,1024), all untargeted) against 65,536 hanging Reserves per step; a step
    = the Reserve batch + the SS_UNRESERVE of its matches (as the metric leg),
    inputs resident in HBM, args.c2_steps timed steps after args.warmup.  The
    last timed batch is checked against the sequential result."""
    from adlb_amd import shards, synth
    from adlb_amd.server import Server
    R, N = args.reserves, args.c2_units
    w = synth.config2(n_units=N, n_types=args.types, n_reserves=R, seed=shards.shard_seed(args.seed + 20, rank))
    srv = Server(w.user_types, w.num_app_ranks, world, rank, max_units=N, device=local)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    srv.set_stream(stream.cuda_stream)
    try:
        units = np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(N, -1), np.zeros(N),
                          np.full(N, -1), np.full(N, -1)], axis=1).astype(np.int32)
        srv.put_batch(units)
        del units
        W2, K2 = max(args.warmup, 1), args.c2_steps
        nb = W2 + K2
        rng = np.random.default_rng(args.seed + 27 + rank)
        reqs = np.empty((nb, R, 18), np.int32)
        for b in range(nb):
            reqs[b, :, 0] = np.arange(R, dtype=np.int32)
            reqs[b, :, 1] = 1
            reqs[b, :, 2:] = synth.type_vectors(rng, w.user_types, R) if b else w.r_types
        d_reqs = torch.from_numpy(reqs).to(dev)
        d_resp = torch.empty((nb, R, 12), dtype=torch.int32, device=dev)
        p_req = [d_reqs[b].data_ptr() for b in range(nb)]
        p_resp = [d_resp[b].data_ptr() for b in range(nb)]

        def step(b):
            srv.reserve_batch_device(R, p_req[b], p_resp[b])
            srv.unreserve_resp_device(R, p_req[b], p_resp[b])

        for b in range(W2):
            step(b)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for b in range(W2, nb):
            step(b)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        matched = int((d_resp[W2:, :, 0] == 1).sum().item())
        if world > 1:
            el, matched = shards.reduce_step_timing(el, matched)
        ec = _exact_check()
        par = parity_of(lambda: check_units(ec, w, np.arange(1, N + 1, dtype=np.int64), np.ones(N, bool),
                                            reqs[nb - 1], d_resp[nb - 1].cpu().numpy(), w.num_app_ranks + rank))
        if world > 1:
            par["parity"] = all_ranks_true(par["parity"])
        return {"workload": f"config2: {N} units/shard, {args.types} types, prio U[0,1024), {R} hanging Reserves/step "
                            f"(70/20/10 single/pair/wildcard), step = reserve batch + unreserve of matched units",
                "value": matched / el if par["parity"] else None, "unit": "assignments/s", "steps": K2,
                "warmup": W2, "ms_per_step": el * 1e3 / K2, **par, "scaling": "weak"}
    finally:
        srv.close()


def bench_wide(args, torch, dev):
    """More than 64 work types (the sorted-runs Reserve path, adlbq_wide.hip):
    a config-2-shaped queue with args.wide_types types; a step = one Reserve
    batch + the unreserve of its matches.  The first batch is checked against
    the oracle (the restatement of xq.c, on the same trace)."""
    import oracle
    from adlb_amd import synth
    from adlb_amd.server import Server
    N, R, T = args.wide_units, args.wide_reserves, args.wide_types
    w = synth.config2(n_units=N, n_types=T, n_reserves=R, seed=args.seed + 90, prio_hi=1024)
    reqs = np.concatenate([w.r_rank[:, None], w.r_hang[:, None].astype(np.int32), w.r_types], axis=1).astype(np.int32)
    units = np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(N, -1), np.zeros(N),
                      np.full(N, -1), np.full(N, -1)], axis=1).astype(np.int32)
    with Server(w.user_types, w.num_app_ranks, max_units=N) as srv:
        srv.put_batch(units)
        d_req = torch.from_numpy(reqs).to(dev)
        d_resp = torch.empty((R, 12), dtype=torch.int32, device=dev)
        first = None
        for _ in range(2):  # warm-up (buffers sized), then the checked batch's answers
            srv.reserve_batch_device(R, d_req.data_ptr(), d_resp.data_ptr())
            torch.cuda.synchronize()
            first = d_resp.cpu().numpy().copy()
            srv.unreserve_resp_device(R, d_req.data_ptr(), d_resp.data_ptr())
        torch.cuda.synchronize()
        steps = 5
        t0 = time.perf_counter()
        for _ in range(steps):
            srv.reserve_batch_device(R, d_req.data_ptr(), d_resp.data_ptr())
            srv.unreserve_resp_device(R, d_req.data_ptr(), d_resp.data_ptr())
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    o = oracle.Oracle("own")
    o.init(w.user_types, w.num_app_ranks)
    exp = np.asarray(synth.split_outputs(o.replay(synth.workload_trace(w)))[N:], np.int32)
    same = bool(np.array_equal(first[:, :10], exp[:, :10]))
    matched = int((first[:, 0] == 1).sum())
    return {"workload": f"{T} work types (sorted-runs path): {N} untargeted units, prio U[0,1024), {R} hanging "
                        f"Reserves (70/20/10 single/pair/wildcard); step = reserve batch + unreserve",
            "value": matched * steps / el if same else None, "unit": "assignments/s",
            "ms_per_step": el * 1e3 / steps, "matched_per_step": matched, "parity": same}


def config4_parity(ec, w, puts, applied, reqs, d_resp, d_pout, b, R, server_rank):
    """Batch b (the last timed one) of the config-4 leg against the sequential
    result over the queue it saw: the initial units, then every Put batch in
    the order it went in (wqseqnos in that order), all unpinned (no Reserve
    ever parked, so no Put matched one, and every match was unreserved)."""
    from adlb_amd import synth
    allr = d_resp[:, :, 0].cpu().numpy()
    assert (allr == 1).all(), "a Reserve parked: the queue state before the batch is not reconstructible here"
    if puts is not None and applied:
        pz = np.concatenate([puts[i] for i in applied])
        n0 = w.u_type.size
        po = d_pout.cpu().numpy()
        last = puts[applied[-1]].shape[0]
        assert (po[:, 0] == np.arange(n0 + pz.shape[0] - last + 1, n0 + pz.shape[0] + 1)).all(), "Put wqseqnos"
        assert (po[:, 1] == -1).all(), "a Put matched a parked Reserve"
        w = synth.Workload(user_types=w.user_types, num_app_ranks=w.num_app_ranks,
                           u_type=np.concatenate([w.u_type, pz[:, 0]]), u_prio=np.concatenate([w.u_prio, pz[:, 1]]),
                           u_target=np.concatenate([w.u_target, pz[:, 3]]),
                           u_answer=np.concatenate([w.u_answer, pz[:, 2]]), u_len=np.concatenate([w.u_len, pz[:, 4]]),
                           r_rank=w.r_rank, r_types=w.r_types, r_hang=w.r_hang, name="config4")
    n = w.u_type.size
    return check_units(ec, w, np.arange(1, n + 1, dtype=np.int64), np.ones(n, bool), reqs[b], d_resp[b].cpu().numpy(),
                       server_rank)


def bench_config4(args, torch, dist, world, rank, local, dev):
    """Config 4: c4_units units with 80% targeted (target ~
    Zipf(1.1) over 1,024 app ranks), 32 types with Zipf(1.1) popularity, prio ~
    U[0, 2^16); 65,536 hanging Reserves per step from ranks U[0, 1024) with 1-4
    Zipf types each, a different pre-staged batch per step.  A step = the
    reserve batch (pre-targeted scan per rank bucket, then the untargeted
    scan, wide-T chain) + SS_UNRESERVE of every match, so each step sees the
    same queue.  Reports matched assignments/s and the per-stage times."""
    from adlb_amd import shards, synth
    from adlb_amd.server import Server

    R, N, W4 = args.reserves, args.c4_units, 2
    nb = args.c4_steps + W4
    w = synth.config4(n_units=N, n_reserves=R, seed=shards.shard_seed(args.seed + 40, rank))
    srv = Server(w.user_types, w.num_app_ranks, world, rank, max_units=N, device=local)
    stream = torch.cuda.Stream(dev)
    srv.set_stream(stream.cuda_stream)
    if args.c4_chain_passes is not None:
        srv.set_param("chain_passes", args.c4_chain_passes)
    if args.c4_chain_modes is not None:
        srv.set_param("chain_modes", args.c4_chain_modes)
    if args.c4_chain_rounds is not None:
        srv.set_param("chain_rounds", args.c4_chain_rounds)
    for kv in args.c4_param:
        k_, v_ = kv.split("=", 1)
        srv.set_param(k_, int(v_))
    srv.put_batch(np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(N, -1),
                            np.zeros(N), np.full(N, -1), np.full(N, -1)], axis=1).astype(np.int32))
    rng = np.random.default_rng(args.seed + 41 + rank)
    reqs = np.empty((nb, R, 18), np.int32)
    for b in range(nb):
        reqs[b, :, 0] = rng.integers(0, w.num_app_ranks, size=R)
        reqs[b, :, 1] = 1
        reqs[b, :, 2:] = zipf_type_sets(rng, len(w.user_types), R) if b else w.r_types
    with torch.cuda.stream(stream):
        d_reqs = torch.from_numpy(reqs).to(dev)
        d_resp = torch.empty((nb, R, 12), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    P = args.c4_puts
    puts = None
    if P > 0:  # each step's new units, drawn like the queue (targets, types, prios)
        wp = synth.config4(n_units=nb * P, n_reserves=1, seed=shards.shard_seed(args.seed + 43, rank))
        puts = np.stack([wp.u_type, wp.u_prio, wp.u_answer, wp.u_target, wp.u_len, np.full(nb * P, -1),
                         np.zeros(nb * P), np.full(nb * P, -1), np.full(nb * P, -1)], axis=1).astype(np.int32)
        puts = puts.reshape(nb, P, 9)
        with torch.cuda.stream(stream):
            d_pout = torch.empty((P, 3), dtype=torch.int32, device=dev)

    host_parts = {"put": 0.0, "reserve": 0.0, "unreserve": 0.0}
    applied = []  # put batches in the order they went in (wqseqnos follow it)

    p_req = [d_reqs[b].data_ptr() for b in range(nb)]  # no tensor views inside the timed loop
    p_resp = [d_resp[b].data_ptr() for b in range(nb)]
    p_pout = d_pout.data_ptr() if puts is not None else 0

    def step(b):
        t0 = time.perf_counter()
        if puts is not None:  # device-resident results: no host round trip
            srv.put_batch_device(puts[b], p_pout)
            applied.append(b)
        t1 = time.perf_counter()
        srv.reserve_batch_device(R, p_req[b], p_resp[b])
        t2 = time.perf_counter()
        srv.unreserve_resp_device(R, p_req[b], p_resp[b])
        host_parts["put"] += t1 - t0
        host_parts["reserve"] += t2 - t1
        host_parts["unreserve"] += time.perf_counter() - t2

    for b in range(W4):
        step(b)
    torch.cuda.synchronize()
    srv.profile(True)
    base = {st: srv.profile_read(st) for st in STAGES}
    hbase = {st: srv.stat("host_ns:" + st) for st in (*STAGES, "pre", "scan", "tindex")}
    step(W4 - 1)
    stages, stages_host = {}, {}
    for st in STAGES:
        ms, n = srv.profile_read(st)
        if n - base[st][1]:
            stages[st] = round((ms - base[st][0]) / (n - base[st][1]), 4)
            stages_host[st] = round((srv.stat("host_ns:" + st) - hbase[st]) / 1e6 / (n - base[st][1]), 4)
    for st in ("pre", "scan", "tindex"):  # host-only parts of the reserve call (one profiled step)
        stages_host[st] = round((srv.stat("host_ns:" + st) - hbase.get(st, 0)) / 1e6, 4)
    srv.profile(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    HACC = ("req_cap", "tables", "tables_wait", "rq_cap", "scan_cap", "tindex", "tindex_wait", "ti_keys", "ti_sort",
            "ti_wait", "ti_alloc", "ti_fill", "ti_devptr", "ti_launch", "ti_stage", "ti_delta", "sort", "total")
    hacc0 = {k: srv.stat("hacc:" + k) for k in HACC}
    t0 = time.perf_counter()
    host = 0.0
    for k in host_parts:
        host_parts[k] = 0.0
    for b in range(W4, nb):
        th = time.perf_counter()
        step(b)
        host += time.perf_counter() - th
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    matched = int((d_resp[W4:, :, 0] == 1).sum().item())
    if world > 1:
        el, matched = shards.reduce_step_timing(el, matched)
    steps = nb - W4
    par = parity_of(lambda: config4_parity(_exact_check(), w, puts, applied, reqs, d_resp, d_pout, nb - 1, R,
                                           w.num_app_ranks + rank))
    if world > 1:
        par["parity"] = all_ranks_true(par["parity"])
    per_batch = []
    if args.c4_chain_stats:
        for b in range(W4, nb):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            step(b)
            torch.cuda.synchronize()
            per_batch.append({"ms": round((time.perf_counter() - t1) * 1e3, 3),
                              **{k: srv.stat(k) for k in ("chain_rounds", "chain_passes", "chain_recomputed",
                                                          "chain_fallback", "chain_timeouts")}})
    out = {
        "workload": f"config4: {N} units/shard (80% targeted, Zipf(1.1) over 1024 ranks), 32 Zipf types, "
                    f"prio U[0,2^16), {R} hanging Reserves/step with 1-4 types, {P} Puts (same mix) before each",
        "targeted_index": {"merges": srv.stat("tindex_merges"), "rebuilds": srv.stat("tindex_rebuilds")},
        "candidate_sort": {"planned": srv.stat("sort_async"), "planned_radix": srv.stat("sort_radix"),
                           "plan_missed": srv.stat("sort_async_bad"),
                           "device_sorted_lists": srv.stat("device_sorted_lists"),
                           "keyrank": srv.stat("keyrank"), "keyrank_failed": srv.stat("keyrank_failed"),
                           "keyrank_why": srv.stat("keyrank_why"), "keyrank_maxbin": srv.stat("keyrank_maxbin"),
                           "candidates": srv.stat("candidates")},
        "value": matched / el if par["parity"] else None,
        **par,
        "unit": "assignments/s",
        "ms_per_step": el * 1e3 / steps,
        "matched_per_step": matched / steps,
        "host_call_ms_per_step": round(host * 1e3 / steps, 3),
        "host_call_parts_ms": {k: round(v * 1e3 / steps, 3) for k, v in host_parts.items()},
        "stages_ms": stages,
        "stages_host_ms": stages_host,
        "reserve_host_sections_ms": {k: round((srv.stat("hacc:" + k) - hacc0[k]) / 1e6 / max(nb - W4, 1), 4)
                                     for k in HACC},
        "scaling": "weak",
    }
    if per_batch:
        out["chain_per_batch"] = per_batch
    srv.close()
    return out


def main():
    args = parse()
    world0 = int(os.environ.get("WORLD_SIZE", "1"))
    pmc = None
    if world0 == 1 and not args.no_pmc:
        pmc = pmc_traffic(args)  # before this process initialises the GPU
    # one hardware queue per server shard's stream (HIP's default is 4): config 3's
    # 8 shards and config 5's 8 streams then run side by side instead of 2 per queue
    if args.hw_queues > 0 and "GPU_MAX_HW_QUEUES" not in os.environ:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # ADLB_BENCH_REHEARSE=1: rehearse the multi-rank path on fewer GPUs than ranks
    # (gloo, ranks folded onto the visible devices); timings then mean nothing
    rehearse = os.environ.get("ADLB_BENCH_REHEARSE") == "1"
    if world > 1:
        dist.init_process_group("gloo" if rehearse else "nccl")
    if rehearse:
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from adlb_amd import shards, synth
    from adlb_amd.server import Server

    if args.config4_only:
        out = bench_config4(args, torch, dist, world, rank, local, dev)
        if rank == 0:
            print(json.dumps({"config4": out}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    if args.wide_only:
        if rank == 0:
            print(json.dumps({"wide_types": bench_wide(args, torch, dev)}), flush=True)
        return
    if args.config5_only:
        out = bench_config5(args, torch, dist, world, rank, local, dev)
        if rank == 0:
            print(json.dumps({"config5": out}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    if args.config3_only:
        out = bench_config3(args, torch, dist, world, rank, local, dev)
        if rank == 0:
            print(json.dumps({"config3": out}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    R, N = args.reserves, args.units
    w = synth.config2(n_units=N, n_types=args.types, n_reserves=R, seed=shards.shard_seed(args.seed, rank),
                      equal_prio=args.equal_prio)
    srv = Server(w.user_types, w.num_app_ranks, world, rank, max_units=N, device=local)
    if args.chain_passes is not None:
        srv.set_param("chain_passes", args.chain_passes)
    if args.chain_warm is not None:
        srv.set_param("chain_warm", args.chain_warm)
    if args.chain_modes is not None:
        srv.set_param("chain_modes", args.chain_modes)
    if args.chain_rounds is not None:
        srv.set_param("chain_rounds", args.chain_rounds)
    if args.rank_in_select is not None:
        srv.set_param("rank_in_select", args.rank_in_select)
    for kv in args.param:
        k, v = kv.split("=", 1)
        srv.set_param(k, int(v))
    # one explicit stream for the library and the torch glue ops (the handle's
    # own stream is non-blocking and would not order against torch's null stream)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    srv.set_stream(stream.cuda_stream)
    units = np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(N, -1),
                      np.zeros(N), np.full(N, -1), np.full(N, -1)], axis=1).astype(np.int32)
    srv.put_batch(units)
    del units
    if world > 1:
        shards.exchange_qmstat(srv)  # the qmstat table every shard's donor choice reads (untimed)
    nb = args.steps + args.warmup
    rng = np.random.default_rng(args.seed + 7 + rank)
    reqs = np.empty((nb, R, 18), np.int32)
    for b in range(nb):
        reqs[b, :, 0] = np.arange(R, dtype=np.int32)
        reqs[b, :, 1] = 1
        reqs[b, :, 2:] = synth.type_vectors(rng, w.user_types, R) if b else w.r_types
    d_reqs = torch.from_numpy(reqs).to(dev)
    d_resp = torch.empty((nb, R, 12), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    p_req = [d_reqs[b].data_ptr() for b in range(nb)]  # no tensor views inside the timed loop
    p_resp = [d_resp[b].data_ptr() for b in range(nb)]
    if args.diag_same_batch:  # diagnostic only (never a reported number): every step on batch 0's buffers
        p_req = [p_req[0]] * nb
        p_resp = [p_resp[0]] * nb

    def step(b):
        srv.reserve_batch_device(R, p_req[b], p_resp[b])
        # SS_UNRESERVE every matched unit, straight from the batch's responses
        srv.unreserve_resp_device(R, p_req[b], p_resp[b])

    for b in range(args.warmup):
        step(b)
    torch.cuda.synchronize()
    stages, dominant, dom_timed = {}, None, None
    if not args.no_profile:
        # per-stage breakdown, untimed: HIP events around every stage's launches
        srv.profile(True)
        base = {s: srv.profile_read(s) for s in STAGES}
        for i in range(min(args.steps, 10)):
            step(i % max(args.warmup, 1))
        for s in STAGES:
            ms, n = srv.profile_read(s)
            ms0, n0 = base[s]
            if n - n0:
                stages[s] = round((ms - ms0) / (n - n0), 4)
        dominant = max(stages, key=stages.get) if stages else None
        # the timed region carries events around the dominant stage only
        srv.profile_only(dominant)
        # every n-th timed batch carries the two events (each event record holds
        # the queue ~5 us behind the kernel before it)
        srv.set_param("profile_every", args.profile_every)
        base_dom = srv.profile_read(dominant)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    HACC_M = ("req_cap", "tables", "rq_cap", "scan_cap", "l_scan", "sort", "l_rank", "l_chain", "l_fin", "total")
    HACC_D = ("ls_pre", "ls_hist", "ls_thr", "ls_sel")  # diagnostic only (--diag-first)
    hacc0 = {k: srv.stat("hacc:" + k) for k in HACC_M + HACC_D}
    t_enq = []
    t0 = time.perf_counter()
    first_sections = None
    for b in range(args.warmup, nb):
        if args.diag_first and b == args.warmup + 1:  # diagnostic only: host sections of the first timed step
            first_sections = {k: round((srv.stat("hacc:" + k) - hacc0[k]) / 1e3, 1) for k in HACC_M + HACC_D}
        step(b)
        t_enq.append(time.perf_counter())
    t_submit = time.perf_counter() - t0  # host time to enqueue the K steps
    torch.cuda.synchronize()
    t_sync = time.perf_counter()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    host_sections = {k: round((srv.stat("hacc:" + k) - hacc0[k]) / 1e6 / max(args.steps, 1), 4) for k in HACC_M}
    # where the timed region's host time went: the first step's enqueue, the rest, the final wait
    enqueue_ms = {"first": round((t_enq[0] - t0) * 1e3, 4) if t_enq else None,
                  "rest_per_step": round((t_enq[-1] - t_enq[0]) * 1e3 / max(len(t_enq) - 1, 1), 4) if t_enq else None,
                  "sync_wait": round((t_sync - t_enq[-1]) * 1e3, 4) if t_enq else None}
    matched = int((d_resp[args.warmup:, :, 0] == 1).sum().item())
    if world > 1:
        el, matched = shards.reduce_step_timing(el, matched)
    if dominant:
        ms, n = srv.profile_read(dominant)
        if n - base_dom[1]:
            dom_timed = round((ms - base_dom[0]) / (n - base_dom[1]), 4)
            stages[dominant] = dom_timed
    # parity gate: the last timed batch against the sequential
    # result, untimed; every earlier matched unit was unreserved before it
    ec = _exact_check()
    par = parity_of(lambda: check_units(ec, w, np.arange(1, N + 1, dtype=np.int64), np.ones(N, bool), reqs[nb - 1],
                                        d_resp[nb - 1].cpu().numpy(), w.num_app_ranks + rank))
    par["parity_batch"] = nb - 1
    if world > 1:
        par["parity"] = all_ranks_true(par["parity"])

    # the host-buffer boundary (adlbq_reserve_batch: requests from host memory,
    # responses back, synchronous): the PCIe-inclusive rate, reported beside
    # `value`, never as it (untimed by the driver's clock)
    host_path = None
    if not args.no_host_path:
        hb = min(args.steps, 10)
        torch.cuda.synchronize()
        t_res = 0.0
        t1 = time.perf_counter()
        for i in range(hb):
            b = args.warmup + i % max(args.steps, 1)
            th = time.perf_counter()
            resp = srv.reserve_batch(reqs[b])
            t_res += time.perf_counter() - th
            d_resp[b].copy_(torch.from_numpy(resp).to(dev))  # restore the queue from these responses
            torch.cuda.synchronize()
            srv.unreserve_resp_device(R, d_reqs[b].data_ptr(), d_resp[b].data_ptr())
            srv.sync()
        host_path = {"entry": "adlbq_reserve_batch (host buffers, synchronous)",
                     "ms_per_batch": round(t_res * 1e3 / hb, 4),
                     "assignments_per_s": round(int((d_resp[args.warmup:args.warmup + hb, :, 0] == 1).sum().item())
                                                / t_res, 1) if t_res else None,
                     "bytes_over_pcie_per_batch": (ADLBQ_RESERVE_INTS * 4 + 12 * 4) * R,
                     "step_ms_with_restore": round((time.perf_counter() - t1) * 1e3 / hb, 4)}
        host_path["latency_vs_batch"] = host_latency_table(srv, torch, dev, reqs[args.warmup], d_reqs[args.warmup],
                                                           d_resp[args.warmup])

    chain_batches = None
    if args.chain_per_batch:  # untimed: the timed batches again, one at a time, with the chain's counters
        chain_batches = []
        for b in range(args.warmup, nb):
            srv.reserve_batch_device(R, d_reqs[b].data_ptr(), d_resp[b].data_ptr())
            srv.sync()
            chain_batches.append([srv.stat("chain_" + k) for k in ("passes", "recomputed", "fallback", "timeouts")])
            srv.unreserve_resp_device(R, d_reqs[b].data_ptr(), d_resp[b].data_ptr())
        srv.sync()
    phases = None
    if args.chain_stamps:
        srv.set_param("chain_stamps", 1)
        step(args.warmup)
        torch.cuda.synchronize()
        phases = {f"phase{k}": (srv.stat(f"chain_phase{k}"), srv.stat(f"chain_phase{k}_max")) for k in range(1, 8)}
        phases["clock_mhz_pass1"] = srv.stat("chain_phase2_mhz")
        phases["start_spread"] = srv.stat("chain_start_spread")
        phases["end_abs"] = srv.stat("chain_end_abs")
        srv.set_param("chain_stamps", 0)
    if args.kernel_stamps:
        # diagnostic: per-workgroup phase stamps of pass 1 (hist) and pass 2 (select) of one batch
        srv.set_param("kernel_stamps", 1)
        step(1)
        torch.cuda.synchronize()
        phases = dict(phases or {})
        for w in ("hist", "sel"):
            phases[w] = {k: srv.stat(f"kst_{w}_{k}") / 1000.0 for k in ("1", "2", "3", "start", "span")}
            phases[w]["startp"] = [srv.stat(f"kst_{w}_startp{q}") / 1000.0 for q in (10, 25, 50, 75, 90, 99)]
            phases[w]["endp"] = [srv.stat(f"kst_{w}_endp{q}") / 1000.0 for q in (10, 25, 50, 75, 90, 99)]
        srv.set_param("kernel_stamps", 0)
    live = srv.last_scan_units()
    # algorithmic bytes per launch: SURVEY §8(d)'s 16 B per live
    # unit for the open-bucket scan (hist + select together), 20 B per Reserve
    # for the ordered-choice chain (8 B type mask + 4 B targeted result read,
    # 4 B choice written, 4 B candidate rank read), 72+8+4 B per Reserve for the
    # batch as a whole (request record, assignment output, pin write).
    alg = {"chain": 20 * R, "scan": 16 * live, "batch": 16 * live + (72 + 8 + 4) * R}
    batch_ms = sum(stages.values()) if stages else el * 1e3 / args.steps
    kernels = {}
    for st, ms in stages.items():
        kernels[st] = {"kernel": KERNEL_OF[st], "ms": ms, "traffic": traffic_of(pmc, st)}

    def roof(bytes_, ms, traffic, kernel):
        a = bytes_ / (ms * 1e-3) / 1e9 if ms else None
        return {"bound": "hbm", "kernel": kernel, "achieved": round(a, 2) if a else None, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(a / HBM_PEAK_GBS, 6) if a else None, "traffic": traffic,
                "algorithmic_bytes": bytes_, "launch_ms": ms}

    if dominant == "chain":
        roofline = roof(alg["chain"], stages["chain"], kernels["chain"]["traffic"], KERNEL_OF["chain"])
    elif dominant in ("hist", "select"):
        roofline = roof(alg["scan"] / 2, stages[dominant], kernels[dominant]["traffic"], KERNEL_OF[dominant])
    elif dominant:
        roofline = roof(alg["batch"] * stages[dominant] / batch_ms, stages[dominant], kernels[dominant]["traffic"],
                        KERNEL_OF[dominant])
    else:
        roofline = roof(alg["batch"], batch_ms, None, "reserve batch (unprofiled)")
    scan_ms = stages.get("hist", 0) + stages.get("select", 0)
    scan_tr = [kernels[k]["traffic"] for k in ("hist", "select") if k in kernels]
    res = {
        "metric": "matched Reserve assignments/sec at 10M-unit queue",
        "value": matched / el if par["parity"] else None,   # no number without parity
        **par,
        "unit": "assignments/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el * 1e3 / args.steps,
        "host_submit_ms_per_step": round(t_submit * 1e3 / args.steps, 4),
        "timed_region_host_ms": enqueue_ms,
        **({"diag_first_step_host_us": first_sections} if first_sections else {}),
        "reserve_host_sections_ms_per_step": host_sections,
        "host_buffer_path": host_path,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (seeded config-2 queue and Reserve batches, adlb_amd/synth.py)",
        "config": {"workload": f"config2-metric: {N} units/shard, {args.types} types, prio U[0,1024), "
                               f"{R} hanging Reserves/step (70/20/10 single/pair/wildcard), "
                               f"step = reserve batch + unreserve of matched units",
                   "units_per_shard": N, "reserves_per_step": R, "parallelism": f"shards{world}"},
        "roofline": roofline,
        "roofline_scan": roof(alg["scan"], scan_ms, sum(scan_tr) if scan_tr and None not in scan_tr else None,
                              "k_prep_hist + k_select_wave (time includes the request preparation)") if scan_ms else None,
        "roofline_batch": roof(alg["batch"], batch_ms, None, "all reserve-batch kernels"),
        "kernels_ms": kernels,
        "chain_last_batch": {k: srv.stat("chain_" + k) for k in ("rounds", "passes", "recomputed", "fallback",
                                                                  "timeouts")},
        "candidates_last_batch": srv.stat("candidates"),
        "rank_in_select_last_batch": srv.stat("rank_fast"),
    }
    if phases:
        res["chain_phases_ns"] = phases
    if chain_batches is not None:
        res["chain_per_batch"] = {"fields": ["passes", "recomputed", "fallback", "timeouts"], "batches": chain_batches}
    srv.close()
    del d_reqs, d_resp
    if not args.no_config2:
        try:
            res["config2"] = bench_config2(args, torch, dist, world, rank, local, dev)
        except Exception as e:  # reported, not fatal: the metric line above stands
            res["config2"] = {"error": f"{type(e).__name__}: {e}"}
    if not args.no_config3:
        try:
            res["config3"] = bench_config3(args, torch, dist, world, rank, local, dev)
        except Exception as e:  # reported, not fatal: the metric line above stands
            res["config3"] = {"error": f"{type(e).__name__}: {e}"}
    if not args.no_config4:
        try:
            res["config4"] = bench_config4(args, torch, dist, world, rank, local, dev)
        except Exception as e:  # reported, not fatal
            res["config4"] = {"error": f"{type(e).__name__}: {e}"}
    if not args.no_config5:
        try:
            res["config5"] = bench_config5(args, torch, dist, world, rank, local, dev)
        except Exception as e:  # reported, not fatal
            res["config5"] = {"error": f"{type(e).__name__}: {e}"}
    if not args.no_wide:
        try:
            res["wide_types"] = bench_wide(args, torch, dev)
        except Exception as e:  # reported, not fatal
            res["wide_types"] = {"error": f"{type(e).__name__}: {e}"}
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(w, args.cpu_seconds, shards.shard_seed(args.seed, rank),
                                           args.cpu_cores, args.equal_prio)
        c3 = res.get("config3")
        if isinstance(c3, dict) and "error" not in c3:
            # the shard layout: one server process per shard, each shard as the GPU leg builds it
            S = args.c3_servers * world
            ncp = min(args.cpu_cores, S)
            kind = _ref_fits(args.c3_units)
            jobs = [("config3", kind, j, S, args.c3_units, args.c3_reserves, args.seed, args.cpu_seconds)
                    for j in range(ncp)]
            c3["cpu_baseline"] = cpu_baseline_config(
                "config3", jobs, args.cpu_seconds,
                f"{ncp} server processes, shards 0..{ncp - 1} of {S} ({args.c3_units} units each, the GPU leg's "
                f"queues and first Reserve batches; local matching only, no steal round)", args.c3_units)
        c4 = res.get("config4")
        if isinstance(c4, dict) and "error" not in c4:
            kind = _ref_fits(args.c4_units)
            jobs = [("config4", kind, args.c4_units, args.reserves, shards.shard_seed(args.seed + 40, 0),
                     args.cpu_seconds)] * args.cpu_cores
            c4["cpu_baseline"] = cpu_baseline_config(
                "config4", jobs, args.cpu_seconds,
                f"{args.cpu_cores} processes x one replica of the {args.c4_units}-unit config-4 queue (80% targeted, "
                f"32 types; the GPU leg's queue and first Reserve batch, no Puts between Reserves)", args.c4_units)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
