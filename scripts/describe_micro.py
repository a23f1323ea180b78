"""describe-by-selection micro-benchmark (k_describe_sel, one workgroup per sample): per-launch time
from the library's HIP-event probe on samples shaped like the ones the analyses describe (RQ3's
integer total-line differences, coverage deltas, rates), checked against numpy; with
TIMING=1 and the FZ_DESC_TIMING variant (scripts/build_variants.sh desctime -DFZ_DESC_TIMING)
also the workgroup's phase stamps (wall clock, 100 MHz ticks):
  0 start  1 stats pass  2 squares pass  3 select setup  4 histogram  5 gather / wide bounds
  6 narrow ranks  7 refinement rounds  8 final gather  9 written

usage: python scripts/describe_micro.py [libfz path]"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def samples():
    rng = np.random.default_rng(3)
    yield "ints9022", np.round(rng.normal(0, 60, 9022))
    yield "normal1000", rng.normal(0, 0.6, 1000)
    yield "normal1500", rng.normal(0, 0.6, 1500)
    yield "normal2000", rng.normal(0, 0.6, 2000)
    yield "ints4000", np.round(rng.normal(0, 60, 4000))
    yield "normal6000", rng.normal(0, 0.6, 6000)
    yield "normal12000", rng.normal(0, 0.6, 12000)
    yield "normal60000", rng.normal(0, 0.6, 60000)
    yield "rates3000", np.round(rng.uniform(0, 100, 3000), 2)
    yield "const5000", np.full(5000, 7.0)


def main():
    from tse_amd import engine as E
    path = sys.argv[1] if len(sys.argv) > 1 else E.LIB_PATH
    eng = E.Engine(0, lib_path=path)
    torch = eng.torch
    timing = os.environ.get("TIMING") and hasattr(eng.lib, "fz_debug_desc_timing")
    for name, a in samples():
        x = torch.from_numpy(a).to(eng.dev)
        d = eng.describe(x)
        ok = abs(d.median - float(np.median(a))) <= 1e-12 * max(1.0, abs(float(np.median(a)))) and \
            abs(d.q1 - float(np.percentile(a, 25))) <= 1e-9 * max(1.0, abs(float(np.percentile(a, 25))))
        eng.probe_begin("describe_select")
        for _ in range(20):
            eng.describe(x)
        eng.synchronize()
        launches, ms, _ = eng.probe_end()
        row = {"sample": name, "n": len(a), "ok": bool(ok), "us": round(ms / max(launches, 1) * 1e3, 2)}
        if timing:
            import ctypes as C
            buf = (C.c_ulonglong * 32)()
            eng.lib.fz_debug_desc_timing(buf)
            t = [int(v) for v in buf[:32]]
            row["phase_us"] = [round((t[i] - t[i - 1]) / 100.0, 2) for i in range(1, 10)]
            # every stamp relative to the start (us; stamps 10-13 inside the first selection step,
            # 16-21 / 22-27 the first two refinement rounds; stale values from earlier samples
            # where a phase did not run)
            row["stamps_us"] = {i: round((t[i] - t[0]) / 100.0, 2) for i in range(1, 32) if t[i] >= t[0]}
        print(json.dumps(row), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
