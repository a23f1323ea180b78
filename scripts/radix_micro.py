"""Radix-pass micro-benchmark: sort N (key, value) pairs with each libfz build variant and report
the per-pass kernel time (the library's HIP-event probe around every k_onesweep launch) and the
algorithmic rate (24 B per pair per pass).  Also checks every variant's result against numpy's
stable argsort.

usage: python scripts/radix_micro.py [variant ...]      (variants from scripts/build_variants.sh)
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
VDIR = os.path.join(REPO, "tse-replication-package-1-million-fuzzing-sessions_amd", "csrc", "build", "variants")


def main():
    from tse_amd import engine as E
    names = sys.argv[1:] or sorted(f[6:-3] for f in os.listdir(VDIR) if f.startswith("libfz_"))
    sizes = [int(x) for x in os.environ.get("SIZES", "262144,650000,1000000,4000000,16000000").split(",")]
    bits = int(os.environ.get("BITS", "32"))
    reps = int(os.environ.get("REPS", "10"))
    probe = os.environ.get("PROBE", "radix_scatter")
    rng = np.random.default_rng(1)
    data = {n: rng.integers(0, 1 << bits, size=n, dtype=np.uint64) for n in sizes}
    if os.environ.get("KIND") == "sorted":
        data = {n: np.sort(v) for n, v in data.items()}
    for name in names:
        eng = E.Engine(0, lib_path=os.path.join(VDIR, f"libfz_{name}.so"))
        torch = eng.torch
        row = {"variant": name}
        for n in sizes:
            k = data[n]
            dk0 = torch.from_numpy(k.view(np.int64)).to(eng.dev)
            dv0 = torch.arange(n, dtype=torch.int32, device=eng.dev)
            dk, dv = dk0.clone(), dv0.clone()
            eng.radix_sort(dk, dv, bits)
            eng.synchronize()
            if n <= 4_000_000 and not os.environ.get("NOCHECK"):
                order = np.argsort(k, kind="stable")
                ok = (np.array_equal(dk.cpu().numpy().view(np.uint64), k[order])
                      and np.array_equal(dv.cpu().numpy(), order.astype(np.int32)))
                if not ok:
                    row[str(n)] = "MISMATCH"
                    continue
            eng.probe_begin(probe)
            for _ in range(reps):
                dk.copy_(dk0)
                dv.copy_(dv0)
                eng.radix_sort(dk, dv, bits)
            eng.synchronize()
            launches, ms, nbytes = eng.probe_end()
            us = ms / launches * 1e3
            row[str(n)] = {"launches": launches // reps, "us_per_pass": round(us, 2), "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1)}
        print(json.dumps(row), flush=True)
        eng.close()




def timing(name="timing", n=650000, bits=32):
    """Phase stamps (µs after the launch's first tile started) of tiles 0, mid, last of one pass
    in a FZ_OS_TIMING build: entry, ranked, block scans, look-back, LDS staged, written."""
    import ctypes as C
    from tse_amd import engine as E
    eng = E.Engine(0, lib_path=os.path.join(VDIR, f"libfz_{name}.so"))
    torch = eng.torch
    f = eng.lib.fz_debug_os_timing
    f.argtypes = [C.POINTER(C.c_ulonglong)]
    buf = (C.c_ulonglong * 25)()
    for n_ in (n, 16_000_000):
        k = np.random.default_rng(2).integers(0, 1 << bits, size=n_, dtype=np.uint64)
        for rep in range(3):
            dk = torch.from_numpy(k.view(np.int64)).to(eng.dev)
            dv = torch.arange(n_, dtype=torch.int32, device=eng.dev)
            eng.synchronize()
            f(buf)  # resets first-stamp
            eng.radix_sort(dk, dv, 8)  # one pass
            f(buf)
            t0 = buf[24]
            rows = [[round((buf[s * 8 + p] - t0) / 100.0, 2) for p in (0, 6, 1, 2, 3, 4, 5)] for s in range(3)]
            print(json.dumps({"n": n_, "rep": rep, "tile0": rows[0], "mid": rows[1], "last": rows[2]}), flush=True)


if __name__ == "__main__":
    if os.environ.get("TIMING"):
        timing(os.environ["TIMING"])
    else:
        main()
