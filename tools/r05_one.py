"""Round 5: latency of one-Reserve batches (adlbq_reserve_batch, host buffers) on the
10M-unit metric queue, with the engine's host-section timers; run under rocprofv3
--kernel-trace for the kernel's own duration."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), ".."))
from adlb_amd import synth  # noqa: E402
from adlb_amd.server import Server  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
# "sparse" as the second argument: priorities over [0, 2^20) and nothing returned between the Reserves
# (a taken unit is usually the only one at its priority: the anchor goes stale after every Reserve)
SPARSE = len(sys.argv) > 2 and sys.argv[2] == "sparse"
w = synth.config2(n_units=N, n_reserves=64, seed=2, prio_hi=(1 << 20) if SPARSE else 1024)
srv = Server(w.user_types, w.num_app_ranks, 1, 0, max_units=N, device=0)
for kv in sys.argv[3 if SPARSE else 2:]:  # NAME=V engine parameters (A/B)
    k_, v_ = kv.split("=", 1)
    srv.set_param(k_, int(v_))
units = np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(N, -1), np.zeros(N),
                  np.full(N, -1), np.full(N, -1)], axis=1).astype(np.int32)
srv.put_batch(units)
srv.sync()
reqs = np.zeros((64, 18), np.int32)
reqs[:, 0] = np.arange(64)
reqs[:, 1] = 1
reqs[:, 2:] = w.r_types
d_reqs = torch.from_numpy(reqs).to("cuda:0")
d_resp = torch.empty((64, 12), dtype=torch.int32, device="cuda:0")
H = ("req_cap", "tables", "rq_cap", "scan_cap", "l_scan", "total")
ts, h0 = [], {k: srv.stat("hacc:" + k) for k in H}
for i in range(60):
    sub = np.ascontiguousarray(reqs[i % 64:i % 64 + 1])
    t = time.perf_counter()
    resp = srv.reserve_batch(sub)
    ts.append(time.perf_counter() - t)
    if not SPARSE:
        d_resp[:1].copy_(torch.from_numpy(resp).to("cuda:0"))
        srv.unreserve_resp_device(1, d_reqs[i % 64:].data_ptr(), d_resp.data_ptr())
        srv.sync()
print("R=1 latency median %.1f us, p10 %.1f, p90 %.1f" % tuple(np.percentile(np.array(ts[10:]) * 1e6, [50, 10, 90])))
print("host sections per call (us):", {k: round((srv.stat("hacc:" + k) - h0[k]) / 1e3 / 60, 1) for k in H})
print("one_batches", srv.stat("one_batches"))
