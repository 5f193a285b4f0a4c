"""Serialised global loads in the gfx950 code of the HIP sources: for every
kernel, the global loads followed within two instructions by
`s_waitcnt vmcnt(0)` (a load the code waits for at once -- fine in a pointer
chase, a bug where the loads were meant to be in flight together, e.g. a load
under a per-lane condition whose result the compiler merges at the join).

usage: python tools/asm_waits.py [min_count] [file.hip ...]   (default 4, every adlbq_*.hip)
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "adlb_amd", "csrc")


def kernel_waits(asm: str):
    lines = asm.splitlines()
    out = []
    for i, line in enumerate(lines):
        m = re.match(r"^(_Z\S+):\s", line)
        if not m:
            continue
        e = i
        while e < len(lines) and not lines[e].startswith(".Lfunc_end"):
            e += 1
        at = [k - i for k in range(i, e) if "global_load" in lines[k]
              and any("s_waitcnt vmcnt(0)" in lines[q] for q in range(k + 1, min(k + 3, e)))]
        out.append((m.group(1), at))
    return out


def main(argv):
    lim = int(argv[1]) if len(argv) > 1 else 4
    files = argv[2:] or sorted(glob.glob(os.path.join(CSRC, "adlbq_*.hip")))
    with tempfile.TemporaryDirectory() as td:
        for f in files:
            s = os.path.join(td, os.path.basename(f) + ".s")
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                            "-I" + os.path.join(CSRC, "..", "..", "include"), "--cuda-device-only", "-S", f,
                            "-o", s], check=True, capture_output=True)
            for name, at in kernel_waits(open(s).read()):
                if len(at) >= lim:
                    print(f"{os.path.basename(f)}  {len(at):3d}  {name[:90]}")


if __name__ == "__main__":
    main(sys.argv)
