"""Diagnostic: the failing config-5 shard replayed whole under put-match variants."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from adlb_amd import replay, synth  # noqa: E402
from adlb_amd.server import Server  # noqa: E402

A, S, seed, idx = 512, 8, 2, 3
o = oracle.Oracle("own", private=True)
o.init([1, 2], A, S, idx)
tr = np.ascontiguousarray(synth.config5_stream(lambda ev: synth.split_outputs(o.replay(ev)), n_ranks=A, n_rounds=60,
                                               n_servers=S, my_idx=idx, seed=seed + 17 * idx, n_seed_units=4 * A),
                          np.int32)
o = oracle.Oracle("own", private=True)
o.init([1, 2], A, S, idx)
exp = o.replay(tr)
for params in ({}, {"put_match_block": 0}, {"put_always_match": 1}, {"put_always_match": 1, "put_match_block": 0}):
    with Server([1, 2], A, S, idx, max_units=1 << 16) as srv:
        for k, v in params.items():
            srv.set_param(k, v)
        g = replay.replay(srv, tr)
    gs, es = synth.split_outputs(g), synth.split_outputs(exp)
    k = next((j for j, (x, y) in enumerate(zip(gs, es)) if list(x) != list(y)), None)
    print(params, "identical" if k is None else f"first diff {k}: got {list(gs[k])} exp {list(es[k])}", flush=True)
