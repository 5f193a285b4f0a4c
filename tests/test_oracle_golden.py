"""The oracle (oracle/liboracle.so, this repo's CPU restatement) reproduces the
golden vectors generated from the reference's own src/xq.c (oracle/gen_golden.py)."""
import glob
import os

import numpy as np
import pytest

import oracle
from adlb_amd import synth

# server event streams (nq_*, mix_*: oracle/gen_nq.py) are replayed by test_gpu_server.py
GOLD = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz"))
              if not os.path.basename(p).startswith(("nq_", "mix_")))


def load(path):
    d = np.load(path, allow_pickle=False)
    return d["user_types"], d["cfg"], d["trace"], d["expected"]


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p)[:-4] for p in GOLD])
def test_oracle_matches_reference_golden(path):
    ut, cfg, trace, expected = load(path)
    o = oracle.Oracle("own")
    o.init(ut, int(cfg[0]), int(cfg[1]), int(cfg[2]))
    out = o.replay(trace)
    assert out.size == expected.size
    bad = np.nonzero(out != expected)[0]
    assert bad.size == 0, f"first mismatch at output int {bad[0]}"


def test_golden_set_is_complete():
    names = {os.path.basename(p)[:-4] for p in GOLD}
    for must in ["t01_tie_seqno", "t03_pretargeted", "t06_lowest", "t08_rq_fifo",
                 "t13_donor", "t16_wild_nonzero", "c2_n20k_r4k", "c2_eqprio_n20k_r4k", "c4_n30k_r2k", "c5_stream",
                 "w100_c2_park_puts", "w100_c4", "w200_get_unreserve"]:
        assert must in names


@pytest.mark.skipif(not oracle.available("ref"), reason="reference build only in build container")
def test_own_vs_ref_random_small():
    """Fresh random traces (not stored): own restatement == reference xq.c."""
    for seed in range(3):
        w = synth.config4(n_units=3000, n_reserves=512, n_ranks=16, n_types=6, seed=100 + seed)
        tr = synth.workload_trace(w)
        outs = []
        for kind in ("own", "ref"):
            o = oracle.Oracle(kind)
            o.init(w.user_types, w.num_app_ranks)
            outs.append(o.replay(tr))
        assert np.array_equal(outs[0], outs[1])


def test_tsp_fixtures_consistent():
    """tests/golden/tsp_m*.txt are gen_tsp.py's seeded matrices, and the
    recorded reference bdist (oracle/_ref/tsp under mpirun, tsp.c:262) equals
    the Held-Karp optimum of each matrix."""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import gen_tsp
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(gold, "tsp_expected.json")) as f:
        exp = json.load(f)
    assert set(exp) == {f"tsp_m{n}.txt" for n in gen_tsp.SIZES}
    for name, rec in exp.items():
        with open(os.path.join(gold, name)) as f:
            v = np.array(f.read().split(), dtype=np.int64)
        n = int(v[0])
        d = v[1:].reshape(n, n)
        np.testing.assert_array_equal(d, gen_tsp.matrix(n))
        assert rec["reference_bdist"] == rec["held_karp"] == gen_tsp.held_karp(d)
