"""Diagnostic: the bench's config-5 flow (all handles alive) with per-shard comparison."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from adlb_amd import replay, synth  # noqa: E402
from adlb_amd.server import Server  # noqa: E402

A, S, seed = 512, 8, int(os.environ.get("SEED", "0"))
traces, expect = [], []
for idx in range(S):
    o = oracle.Oracle("own", private=True)
    o.init([1, 2], A, S, idx)
    traces.append(np.ascontiguousarray(synth.config5_stream(lambda ev: synth.split_outputs(o.replay(ev)), n_ranks=A,
                                                            n_rounds=60, n_servers=S, my_idx=idx,
                                                            seed=seed + 17 * idx, n_seed_units=4 * A), np.int32))
for idx, tr in enumerate(traces):
    o = oracle.Oracle("own", private=True)
    o.init([1, 2], A, S, idx)
    expect.append(o.replay(tr))
srvs = [Server([1, 2], A, S, i, max_units=1 << 16) for i in range(S)]
with Server([1, 2], A, S, 0, max_units=1 << 16) as tmp:
    replay.replay(tmp, traces[0][: min(traces[0].size, 20000)])
for i, (srv, tr) in enumerate(zip(srvs, traces)):
    g = replay.replay(srv, tr)
    same = np.array_equal(g, expect[i])
    msg = ""
    if not same:
        gs, es = synth.split_outputs(g), synth.split_outputs(expect[i])
        k = next((j for j, (x, y) in enumerate(zip(gs, es)) if list(x) != list(y)), None)
        msg = f"first differing output {k}: got {list(gs[k]) if k is not None else None} exp {list(es[k]) if k is not None else None} (lens {len(gs)} {len(es)})"
    print(i, same, msg, srv.stat("tindex_merges"), srv.stat("tindex_rebuilds"), flush=True)
