"""TEST INFRASTRUCTURE ONLY -- one process of bench.py's cpu_baseline leg.

Imported by the bench's spawned worker processes (a module path, so spawn
can find it), never by adlb_amd/.
"""
import time


def sample(job):
    """One CPU baseline process: build the queue (all of it, or shard c of C:
    units u with u % C == c in order, the Reserves r with r % C == c) in the
    oracle and time Reserves until the budget is spent.  Returns (Reserves
    done, seconds, units held)."""
    kind, n_units, n_types, n_reserves, seed, eq, c, C, budget = job
    import oracle
    from adlb_amd import synth
    w = synth.config2(n_units=n_units, n_types=n_types, n_reserves=n_reserves, seed=seed, equal_prio=eq)
    if C > 1:
        for f in ("u_type", "u_prio", "u_answer", "u_target", "u_len"):
            setattr(w, f, getattr(w, f)[c::C])
        for f in ("r_rank", "r_types", "r_hang"):
            setattr(w, f, getattr(w, f)[c::C])
    o = oracle.Oracle(kind)
    o.init(w.user_types, w.num_app_ranks)
    o.replay(synth.put_events(w))
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget and done < w.n_reserves:
        k = min(4, w.n_reserves - done)
        o.replay(synth.reserve_events(w.r_rank[done:done + k], w.r_types[done:done + k], w.r_hang[done:done + k]))
        done += k
    return done, time.perf_counter() - t0, w.n_units
