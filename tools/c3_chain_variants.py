"""Diagnostic: chain parameters on one config-3 shard (GPU)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from adlb_amd import synth  # noqa: E402
from adlb_amd.server import Server  # noqa: E402

w = synth.config3_shard(1, 64, 1_562_500, 4, 8192, seed=3, p_remote=float(os.environ.get("PREMOTE", "0.1")))
srv = Server(w.user_types, w.num_app_ranks, 64, 1, max_units=w.n_units, device=0)
srv.put_batch(np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(w.n_units, -1),
                        np.zeros(w.n_units), np.full(w.n_units, -1), np.full(w.n_units, -1)], axis=1).astype(np.int32))
reqs = np.empty((8192, 18), np.int32)
reqs[:, 0] = w.r_rank
reqs[:, 1] = 1
reqs[:, 2:] = w.r_types
d_req = torch.from_numpy(reqs).cuda()
d_resp = torch.empty((8192, 12), dtype=torch.int32, device="cuda")
ref = None
for P, K, modes, warm in [(3, -1, -1, -1), (8, -1, -1, -1), (3, 4, 0, -1), (3, 4, -1, -1), (3, -1, -1, 0),
                          (3, -1, -1, 512), (8, 8, 0, -1)]:
    srv.set_param("chain_passes", P)
    srv.set_param("chain_rounds", K)
    srv.set_param("chain_modes", modes)
    srv.set_param("chain_warm", warm)
    ts = []
    for it in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        srv.reserve_batch_device(8192, d_req.data_ptr(), d_resp.data_ptr())
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
        st = {k: srv.stat(k) for k in ["chain_rounds", "chain_recomputed", "chain_fallback", "parked"]}
        out = d_resp.cpu().numpy()[:, :10].copy()
        if ref is None:
            ref = out
        assert np.array_equal(out, ref), "results differ across parameters"
        srv.unreserve_resp_device(8192, d_req.data_ptr(), d_resp.data_ptr())
        rq = srv.rq_export()
        if rq.shape[0]:
            srv.rq_delete_batch(rq[:, 0])
    print(f"P={P} K={K} modes={modes} warm={warm}: ms {min(ts):.3f}", st, flush=True)
srv.close()
