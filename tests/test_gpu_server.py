"""Config 1: the ADLB server on the GPU engine.

1. Replay: the inbound event streams the reference server handled while
   running `mpirun -np 4 nq -n 8 -q` (1 server) and `-np 6 ... -n 9 -nservers 2`
   (2 servers) -- recorded by oracle/gen_nq.py -- go through the repo's server
   core (adlb_amd/csrc/adlb_core.cpp over the adlbq GPU engine), and every
   reply must equal what the reference server sent: every TA_RESERVE_RESP
   (rc, type, prio, len, answer rank, wqseqno, server), every Get's length
   and payload bytes, every put ack, every info answer, every SS_RFR, in the
   same order.  Runs of Reserves / Gets are replayed as one batch (batch=True)
   and one by one.
2. Drop-in: the reference's examples/nq.c, compiled unchanged against
   include/adlb/adlb.h and linked to adlb_amd/libadlb.so (oracle/_ref/nq_amd,
   built in the build container), under mpirun: 92 and 352 solutions.
"""
import os
import subprocess

import pytest

from nq_fixture import Fixture, compare, replay

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
FIXTURES = ["nq_np4_n8.npz", "nq_np6_n9_s2_r4.npz", "nq_np6_n9_s2_r5.npz"]
NQ_AMD = os.path.join(ROOT, "oracle", "_ref", "nq_amd")
MPIRUN = "/opt/conda/bin/mpirun"


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [True, False])
@pytest.mark.parametrize("name", FIXTURES)
def test_nq_event_stream_replay(name, batch):
    from adlb_amd.core import Core
    fx = Fixture(os.path.join(GOLD, name))
    with Core(fx.types, fx.A, fx.S, fx.me, max_malloc=fx.max_malloc, device=0) as core:
        got = replay(core, fx, batch=batch)
        assert core.num_parked() == 0
    err = compare(got, fx.expected())
    assert err is None, f"{name}: {err}"


def _run_nq(np_, args, timeout=240):
    if not os.path.exists(NQ_AMD):
        pytest.skip("oracle/_ref/nq_amd not built (needs the reference sources in the build container)")
    env = dict(os.environ, ADLB_DEVICE="0")
    r = subprocess.run([MPIRUN, "-np", str(np_), NQ_AMD, *args], env=env, capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, f"rc={r.returncode}\nstdout:\n{r.stdout[-3000:]}\nstderr:\n{r.stderr[-3000:]}"
    return r.stdout


@pytest.mark.gpu
def test_nq_one_server_92():
    out = _run_nq(4, ["-n", "8", "-q"])
    assert "found 92 solutions" in out, out[-2000:]


@pytest.mark.gpu
def test_nq_two_servers_352():
    out = _run_nq(6, ["-n", "9", "-q", "-nservers", "2"])
    assert "found 352 solutions" in out, out[-2000:]
