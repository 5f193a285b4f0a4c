"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports
every entry point include/adlbq.h declares, and the Python mirror covers them.
No compute calls here (no GPU in the build container)."""
import os
import shutil
import subprocess
import tempfile

import pytest

from adlb_amd import _lib


def test_library_built_for_gfx950():
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build() first"
    # --offloading extracts the device images next to its input: work on a copy
    with tempfile.TemporaryDirectory() as d:
        lib = shutil.copy(_lib.LIB_PATH, d)
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", lib],
                             capture_output=True, text=True, cwd=d)
    txt = out.stdout + out.stderr
    assert "gfx950" in txt


def test_exports_every_header_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in _lib.header_symbols() if s not in exported]
    assert not missing, missing


def test_binding_signatures_cover_header():
    assert set(_lib.header_symbols()) == set(_lib.SIGNATURES)


def test_library_loads_and_reports_version():
    lib = _lib.load()
    assert lib.adlbq_version().startswith(b"adlbq")


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.AdlbqError):
        _lib.load()


def test_replay_run_splitting():
    import numpy as np
    from adlb_amd import replay, synth
    w = synth.config2(n_units=10, n_reserves=4, seed=0)
    tr = np.concatenate([synth.put_events(w), synth.reserve_events(w.r_rank, w.r_types, w.r_hang),
                         synth.simple_events(synth.OP_INFO), synth.put_events(w, 0, 2)])
    runs = list(replay._runs(tr, 4))
    assert [r[0] for r in runs] == [synth.OP_PUT, synth.OP_RESERVE, synth.OP_INFO, synth.OP_PUT]
    assert [r[1].shape for r in runs] == [(10, 9), (4, 18), (1, 0), (2, 9)]
