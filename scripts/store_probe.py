"""Where the store build's time goes at a configuration: the host time of fz_store_build (it returns
after its one counter read-back, with the gather still running), the GPU time to the end of the
build, and the same for back-to-back builds (the bench's steps).

usage: python scripts/store_probe.py [--config c2] [--reps 20]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import tse_amd.synth as synth
    from tse_amd import engine as E
    t = synth.generate(synth.config(args.config))
    eng = E.Engine(0)
    eng.upload(t)
    torch = eng.torch
    for _ in range(3):
        eng.build_store()
    eng.synchronize()
    host, total = [], []
    for _ in range(args.reps):
        eng.synchronize()
        t0 = time.perf_counter()
        eng.build_store()
        t1 = time.perf_counter()
        eng.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e3)
        total.append((t2 - t0) * 1e3)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    eng.synchronize()
    t0 = time.perf_counter()
    ev0.record(eng.stream)
    for _ in range(args.reps):
        eng.build_store()
    ev1.record(eng.stream)
    eng.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / args.reps
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    print(json.dumps({"config": args.config, "host_ms_to_return": round(med(host), 4),
                      "ms_to_idle": round(med(total), 4), "back_to_back_ms": round(wall, 4),
                      "back_to_back_gpu_ms": round(ev0.elapsed_time(ev1) / args.reps, 4)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
