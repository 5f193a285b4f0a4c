"""Fixtures for the relinked examples/tsp.c.

Writes seeded distance matrices in tsp.c's stdin format (tsp.c:89-103: the
city count, then the n x n matrix row by row; a 0 off the diagonal never
occurs here) to tests/golden/tsp_m<n>.txt and tests/golden/tsp_expected.json
with, per matrix:

* ``held_karp``: the optimal tour length from city 0 computed here by the
  Held-Karp dynamic programme (independent of ADLB), with tsp.c's convention
  that a 0 entry costs 999999999 (tsp.c:99-100);
* ``reference_bdist``: what the reference build prints as ``bdist``
  (tsp.c:262) when run as ``mpirun -np 5 oracle/_ref/tsp -nservers 2 <
  matrix`` -- oracle/_ref/tsp is the reference's examples/tsp.c + src/adlb.c +
  src/xq.c compiled where they lie (oracle/Makefile, ``_ref/%``).  Recorded
  only when the reference build is present (build container).

The relinked binary (oracle/_ref/tsp_amd: tsp.c unchanged against
include/adlb/adlb.h and adlb_amd/libadlb.so) must print the same bdist
(tests/test_gpu_server.py::test_tsp_relinked).  Run:  python tests/golden/gen_tsp.py
"""
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_TSP = os.path.join(ROOT, "oracle", "_ref", "tsp")
MPIRUN = "/opt/conda/bin/mpirun"
SIZES = (9, 10, 11)


def matrix(n: int) -> np.ndarray:
    rng = np.random.default_rng(20261017 + n)
    d = rng.integers(1, 100, size=(n, n))
    np.fill_diagonal(d, 0)
    return d


def held_karp(d: np.ndarray) -> int:
    n = d.shape[0]
    D = d.astype(np.int64).copy()
    D[D == 0] = 999999999
    INF = 1 << 60
    full = 1 << n
    dp = np.full((full, n), INF, dtype=np.int64)
    dp[1, 0] = 0
    for S in range(1, full, 2):          # subsets containing city 0
        row = dp[S]
        for j in np.nonzero(row < INF)[0]:
            v = row[j]
            for k in range(1, n):
                if not (S >> k) & 1:
                    T = S | (1 << k)
                    if v + D[j, k] < dp[T, k]:
                        dp[T, k] = v + D[j, k]
    return int(min(dp[full - 1, j] + D[j, 0] for j in range(1, n)))


def main():
    out = {}
    for n in SIZES:
        d = matrix(n)
        name = f"tsp_m{n}.txt"
        with open(os.path.join(HERE, name), "w") as f:
            f.write(f"{n}\n")
            for r in d:
                f.write(" ".join(str(int(x)) for x in r) + "\n")
        rec = {"n": n, "held_karp": held_karp(d)}
        if os.path.exists(REF_TSP):
            with open(os.path.join(HERE, name)) as f:
                r = subprocess.run([MPIRUN, "-np", "5", REF_TSP, "-nservers", "2"], stdin=f, capture_output=True,
                                   text=True, timeout=600)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("bdist ")]
            assert r.returncode == 0 and line, r.stdout[-2000:]
            rec["reference_bdist"] = int(line[0].split()[1])
            rec["reference_cmd"] = "mpirun -np 5 oracle/_ref/tsp -nservers 2 < tests/golden/" + name
            assert rec["reference_bdist"] == rec["held_karp"], rec
        out[name] = rec
        print(name, rec)
    with open(os.path.join(HERE, "tsp_expected.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
