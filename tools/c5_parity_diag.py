"""Diagnostic: first event where the GPU replay of a config-5 stream differs from the oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from adlb_amd import replay, synth  # noqa: E402
from adlb_amd.server import Server  # noqa: E402

A, S = 512, 8
for idx in range(S):
    o = oracle.Oracle("own", private=True)
    o.init([1, 2], A, S, idx)
    tr = synth.config5_stream(lambda ev: synth.split_outputs(o.replay(ev)), n_ranks=A, n_rounds=60, n_servers=S,
                              my_idx=idx, seed=int(os.environ.get('SEED', '0')) + 17 * idx, n_seed_units=4 * A)
    tr = np.ascontiguousarray(tr, np.int32)
    o2 = oracle.Oracle("own", private=True)
    o2.init([1, 2], A, S, idx)
    with Server([1, 2], A, S, idx, max_units=1 << 16) as srv:
        # replay run by run, comparing as we go
        pos = 0
        for op, a in replay._runs(tr, 2):
            w = 1 + a.shape[1]
            seg = np.concatenate([np.full((a.shape[0], 1), op, np.int32), a], axis=1).ravel()
            g = replay.replay(srv, seg)
            e = o2.replay(seg)
            if not np.array_equal(g, e):
                gs, es = synth.split_outputs(g), synth.split_outputs(e)
                k = next(i for i, (x, y) in enumerate(zip(gs, es)) if list(x) != list(y))
                print(f"shard {idx}: op {op} run of {a.shape[0]} at event {pos}: item {k}: got {list(gs[k])} "
                      f"expected {list(es[k])}; args {a[k].tolist()}; merges {srv.stat('tindex_merges')} "
                      f"rebuilds {srv.stat('tindex_rebuilds')}", flush=True)
                break
            pos += a.shape[0]
        else:
            print(f"shard {idx}: identical ({pos} events)", flush=True)
