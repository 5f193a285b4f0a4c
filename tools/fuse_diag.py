"""Fused-finalize diagnostic: the full-size config-2 batch with fuse_finalize on/off;
duplicates (requests sharing a unit) by segment, and the chain counters."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from adlb_amd import synth
from adlb_amd.server import Server
import torch

w = synth.config2(n_units=10_000_000, n_reserves=65_536, seed=7)
units = np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(w.n_units, -1), np.zeros(w.n_units),
                  np.full(w.n_units, -1), np.full(w.n_units, -1)], axis=1).astype(np.int32)
reqs = np.concatenate([w.r_rank[:, None], w.r_hang[:, None].astype(np.int32), w.r_types], axis=1).astype(np.int32)
for fuse in (int(a) for a in sys.argv[1:] or ["1", "0"]):
    with Server(w.user_types, w.num_app_ranks, max_units=w.n_units) as s:
        s.set_param("fuse_finalize", fuse)
        s.put_batch(units)
        for b in range(3):
            resp = s.reserve_batch(reqs)
            m = np.nonzero(resp[:, 0] == 1)[0]
            seqs = resp[m, 5]
            u, inv, cnt = np.unique(seqs, return_inverse=True, return_counts=True)
            dup = m[cnt[inv] > 1]
            st = {k: s.stat(k) for k in ("chain_passes", "chain_recomputed", "chain_fallback", "chain_timeouts",
                                         "rank_fast", "batch_failed")}
            print(f"fuse={fuse} batch={b} matched={m.size} dups={dup.size} segs={sorted(set((dup // 256).tolist()))[:20]} "
                  f"first={dup[:8].tolist()} stats={st}", flush=True)
            if m.size:
                trip = torch.tensor(np.stack([w.r_rank[m], resp[m, 5], np.full(m.size, -1)], axis=1)
                                    .astype(np.int32).ravel(), device="cuda")
                torch.cuda.synchronize()
                s.unreserve_batch_device(m.size, trip.data_ptr())
                s.sync()
