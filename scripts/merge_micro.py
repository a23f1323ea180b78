"""Micro-benchmark of the segmented merge sort (csrc/fz_segsort.h) through fz_spearman_index_seg,
whose first step sorts every segment: run under rocprofv3 --kernel-trace to read the per-round
kernel times.  Cases: one 20M-value segment (13 merge rounds), 1,000 segments of 16,384 values
(2 rounds), 5,000 segments of 8,192 (1 round)."""
import ctypes as C
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from tse_amd import engine as E  # noqa: E402

eng = E.Engine(0)
rng = np.random.default_rng(1)
for name, lens in (("one_20M", [20_000_000]), ("1000x16384", [16384] * 1000), ("5000x8192", [8192] * 5000)):
    n = int(sum(lens))
    x = torch.from_numpy(rng.random(n)).to(eng.dev)
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)).to(eng.dev)
    S = len(lens)
    rho = torch.empty(S, dtype=torch.float64, device=eng.dev)
    p = torch.empty(S, dtype=torch.float64, device=eng.dev)
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        E._check(eng.lib, eng.lib.fz_spearman_index_seg(eng.ctx, C.c_void_p(x.data_ptr()), n, C.c_void_p(offs.data_ptr()),
                                                       S, max(lens), C.c_void_p(rho.data_ptr()), C.c_void_p(p.data_ptr())))
        torch.cuda.synchronize()
        print(name, rep, f"{(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
eng.close()
