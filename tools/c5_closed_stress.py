"""Closed-loop config-5 replay (adlbsrv_replay_rounds2) over several seeds, each against the oracle; a
failing seed is replayed open loop to tell a driver-side failure from an engine result."""
import os
import sys
import traceback

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_gpu_config5 import _check  # noqa: E402

seeds = [int(x) for x in sys.argv[1:]] or list(range(5, 13))
fails = 0
for sd in seeds:
    try:
        d = _check(S=4, A=1024, n_events=200_000, k=64, q0=128, seed=sd, closed=True)
        print(f"seed {sd}: closed ok {d['closed_stats']}", flush=True)
    except Exception as e:  # noqa: BLE001
        fails += 1
        print(f"seed {sd}: closed FAILED: {e}", flush=True)
        try:
            _check(S=4, A=1024, n_events=200_000, k=64, q0=128, seed=sd, closed=False)
            print(f"seed {sd}: open loop ok", flush=True)
        except Exception as e2:  # noqa: BLE001
            print(f"seed {sd}: open loop FAILED too: {e2}", flush=True)
print("failures", fails, "of", len(seeds))
