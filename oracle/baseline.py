"""TEST INFRASTRUCTURE ONLY -- one process of bench.py's cpu_baseline leg.

Imported by the bench's spawned worker processes (a module path, so spawn
can find it), never by adlb_amd/.
"""
import time


def sample(job):
    """One CPU baseline process: build the queue (all of it, or shard c of C:
    units u with u % C == c in order, the Reserves r with r % C == c) in the
    oracle and time Reserves until the budget is spent.  Returns (Reserves
    done, seconds, units held).

    job = (kind, n_units, n_types, n_reserves, seed, equal_prio, c, C, budget)
    for the config-2 / metric queue, or ("config3", kind, shard, n_shards,
    n_units, n_reserves, seed, budget): config-3 server shard `shard` as
    bench.py's leg builds it, or ("config4", kind, n_units, n_reserves, seed,
    budget): the config-4 queue (80% targeted, 32 Zipf types) with its first
    Reserve batch."""
    import oracle
    from adlb_amd import synth
    if job[0] == "config3":
        _, kind, shard, S, n_units, n_reserves, seed, budget = job
        w = synth.config3_shard(shard, S, n_units, 4, n_reserves, seed=seed)
        return _time(oracle, synth, kind, w, budget, num_servers=S, idx=shard)
    if job[0] == "config4":
        _, kind, n_units, n_reserves, seed, budget = job
        w = synth.config4(n_units=n_units, n_reserves=n_reserves, seed=seed)
        return _time(oracle, synth, kind, w, budget)
    kind, n_units, n_types, n_reserves, seed, eq, c, C, budget = job
    w = synth.config2(n_units=n_units, n_types=n_types, n_reserves=n_reserves, seed=seed, equal_prio=eq)
    if C > 1:
        for f in ("u_type", "u_prio", "u_answer", "u_target", "u_len"):
            setattr(w, f, getattr(w, f)[c::C])
        for f in ("r_rank", "r_types", "r_hang"):
            setattr(w, f, getattr(w, f)[c::C])
    return _time(oracle, synth, kind, w, budget)


def _time(oracle, synth, kind, w, budget, num_servers=1, idx=0):
    o = oracle.Oracle(kind)
    o.init(w.user_types, w.num_app_ranks, num_servers, idx)
    o.replay(synth.put_events(w))
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget and done < w.n_reserves:
        k = min(4, w.n_reserves - done)
        o.replay(synth.reserve_events(w.r_rank[done:done + k], w.r_types[done:done + k], w.r_hang[done:done + k]))
        done += k
    return done, time.perf_counter() - t0, w.n_units


def c5_shard(job):
    """One server process of the config-5 CPU baseline: shard s's expanded
    trace (oracle/gen_c5.c xtrace: its events plus its part of every steal
    round) replayed alone through the oracle, as one ADLB server process
    serves its own queue.  job = (path of the .npy trace, user_types,
    num_app_ranks, num_servers, s).  Returns (events, seconds)."""
    import numpy as np

    import oracle
    path, ut, A, S, s = job
    tr = np.load(path, mmap_mode="r")
    tr = np.ascontiguousarray(tr, dtype=np.int32)
    o = oracle.Oracle("own")
    o.init(ut, A, S, s)
    cap = oracle.output_bound(tr, o.ntypes)
    out = np.empty(cap, dtype=np.int32)
    t0 = time.perf_counter()
    n = o.lib.orc_replay(tr.ctypes.data, tr.size, out.ctypes.data, cap)
    sec = time.perf_counter() - t0
    if n < 0:
        raise ValueError(f"oracle: shard {s} trace rejected (rc={n})")
    return int(tr.size), sec
