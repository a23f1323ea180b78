"""k_series_small micro-benchmark (spearmanr(range(n), x) + shapiro(x) of one series of <= 4,096
values in one workgroup, fz_series_tests): per-call time from HIP events, and with a
FZ_SERIES_TIMING variant (scripts/build_variants.sh sertime -DFZ_SERIES_TIMING) the workgroup's
phase stamps (us): sort network, Spearman (its p-value on thread 0), Shapiro-Wilk (its p-value).

usage: python scripts/series_micro.py [libfz path]"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from tse_amd import engine as E
    path = sys.argv[1] if len(sys.argv) > 1 else E.LIB_PATH
    eng = E.Engine(0, lib_path=path)
    torch = eng.torch
    timing = hasattr(eng.lib, "fz_debug_series_timing")
    rng = np.random.default_rng(5)
    for n in (300, 1000, 2960, 4096):
        a = np.round(rng.normal(50, 10, n), 3)
        x = torch.from_numpy(a).to(eng.dev)
        out = torch.zeros(4, dtype=torch.float64, device=eng.dev)
        f = eng.lib.fz_series_tests
        for _ in range(3):
            f(eng.ctx, C.c_void_p(x.data_ptr()), n, C.c_void_p(out.data_ptr()))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f(eng.ctx, C.c_void_p(x.data_ptr()), n, C.c_void_p(out.data_ptr()))
        e1.record()
        torch.cuda.synchronize()
        row = {"n": n, "us": round(e0.elapsed_time(e1) / 20 * 1e3, 2), "out": [float(v) for v in out.cpu()]}
        if timing:
            buf = (C.c_ulonglong * 8)()
            eng.lib.fz_debug_series_timing(buf)
            t = [int(v) for v in buf]
            row["phase_us"] = [round((t[i] - t[i - 1]) / 100.0, 2) for i in range(1, 4)]
            if all(t[4:8]):  # the Shapiro-Wilk pass: normal scores' sum, first sums, second sums, p-value
                seq = [t[2], t[4], t[5], t[6], t[7]]
                row["shapiro_us"] = [round((seq[i] - seq[i - 1]) / 100.0, 2) for i in range(1, 5)]
        print(json.dumps(row), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
