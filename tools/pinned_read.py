"""Host read speed of pinned (hipHostMalloc) memory vs pageable memory, MB/s (diagnostic)."""
import time

import numpy as np
import torch

n = 1 << 22  # 16 MB of int32
a = torch.empty(n, dtype=torch.int32, pin_memory=True)
a.numpy()[:] = 1
b = np.ones(n, dtype=np.int32)
for name, arr in (("pinned", a.numpy()), ("pageable", b)):
    arr.sum()
    t = time.perf_counter()
    for _ in range(5):
        s = int(arr.sum())
    el = (time.perf_counter() - t) / 5
    print(f"{name}: {arr.nbytes / el / 1e6:.0f} MB/s (sum {s})")
