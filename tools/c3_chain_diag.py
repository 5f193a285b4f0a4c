"""Diagnostic: the ordered-choice kernel on one config-3 shard (GPU).
Prints per-batch chain statistics and phase stamps for p_remote in {0.1, 0}.
  python tools/c3_chain_diag.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from adlb_amd import synth  # noqa: E402
from adlb_amd.server import Server  # noqa: E402

STATS = ["chain_rounds", "chain_passes", "chain_recomputed", "chain_fallback", "chain_timeouts", "parked",
         "rank_fast", "candidates"] + [f"chain_phase{k}" for k in range(1, 6)] + [f"chain_phase{k}_max" for k in range(1, 6)]

for p_remote in (0.1, 0.0):
    for shard in (0, 1):
        w = synth.config3_shard(shard, 64, 1_562_500, 4, 8192, seed=3, p_remote=p_remote)
        srv = Server(w.user_types, w.num_app_ranks, 64, shard, max_units=w.n_units, device=0)
        srv.put_batch(np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(w.n_units, -1),
                                np.zeros(w.n_units), np.full(w.n_units, -1), np.full(w.n_units, -1)],
                               axis=1).astype(np.int32))
        srv.set_param("chain_stamps", 1)
        reqs = np.empty((8192, 18), np.int32)
        reqs[:, 0] = w.r_rank
        reqs[:, 1] = 1
        reqs[:, 2:] = w.r_types
        d_req = torch.from_numpy(reqs).cuda()
        d_resp = torch.empty((8192, 12), dtype=torch.int32, device="cuda")
        for it in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            srv.reserve_batch_device(8192, d_req.data_ptr(), d_resp.data_ptr())
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) * 1e3
            st = {k: srv.stat(k) for k in STATS}
            print(f"p_remote {p_remote} shard {shard} it {it}: {el:.3f} ms", st, flush=True)
            srv.unreserve_resp_device(8192, d_req.data_ptr(), d_resp.data_ptr())
            # parked requests stay on rq; drop them so every batch sees the same queue
            rq = srv.rq_export()
            if rq.shape[0]:
                srv.rq_delete_batch(rq[:, 0])
        srv.close()
