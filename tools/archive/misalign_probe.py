#!/usr/bin/env python3
"""Read-only and mix HBM probe (tools/libhbm_probe.so) with every input
shifted by 0/4/8/12 bytes (or mixed 4/8/12): does a misaligned 16-B lane
load cost bandwidth by itself?  One JSON line per case."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import hbm_probe as H  # noqa: E402

n, nbytes = 8, 1 << 30
raw = [torch.empty((nbytes + 4096) // 4, device="cuda").uniform_() for _ in range(n + 1)]
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for name, offs in (("aligned", [0] * n), ("all+4", [4] * n), ("all+8", [8] * n), ("all+12", [12] * n),
                   ("mixed 4/8/12", [4, 8, 12, 4, 8, 12, 4, 8]), ("aligned", [0] * n)):
    tab = (ctypes.c_void_p * n)(*[raw[k].data_ptr() + offs[k] for k in range(n)])
    for mode in (1, 0):
        def fn():
            rc = H.LIB.probe_run(mode, 256, 4, 2, 2, 0, 1024, tab, n, ctypes.c_void_p(raw[n].data_ptr()), nbytes, stream)
            assert rc == 0, rc
        t = min(H.timeit(fn) for _ in range(3))
        moved = (n + 1) * nbytes if mode == 0 else n * nbytes
        print(json.dumps({"case": name, "offsets": offs, "mode": ["mix", "read"][mode], "GBps": round(moved / t / 1e9, 1)}),
              flush=True)
