"""Build-log analysis throughput: synthetic Cloud Build logs resident in
HBM through fz_buildlog (line split + per-line classification + per-log fold), plus the host's
srcmap extraction and build_infos assembly (tse_amd.buildlog.analyze), against the oracle's
per-line Python restatement of buildlog_analysis() on a sample (one core).  Prints one JSON line.

usage: python scripts/bench_buildlog.py [--logs 4000] [--repeat 8] [--steps 5]"""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--logs", type=int, default=4000)
    ap.add_argument("--repeat", type=int, default=8, help="the generated batch is repeated this many times")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu-sample", type=int, default=300)
    args = ap.parse_args()
    from tse_amd import buildlog, synth_logs
    from tse_amd import engine as E

    batch = synth_logs.make_batch(11, args.logs, mean_lines=400)
    batch = [(r, t) for r, t in batch if t and len(t.splitlines()) != 1]  # no IndexError logs in the timed batch
    rows = [r for r, _ in batch] * args.repeat
    texts = [t for _, t in batch] * args.repeat
    raws = [t.encode("utf-8") for t in texts]
    offs = np.zeros(len(raws) + 1, dtype=np.int64)
    np.cumsum([len(r) for r in raws], out=offs[1:])
    blob = b"".join(raws)
    n_lines = sum(len(t.splitlines()) for t in texts[:len(batch)]) * args.repeat
    eng = E.Engine(0)
    torch = eng.torch
    dev = eng.dev
    d_text = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    d_offs = torch.from_numpy(offs).to(dev)
    n = len(raws)
    i32 = lambda k: torch.empty(max(k, 1), dtype=torch.int32, device=dev)  # noqa: E731
    i64 = lambda k: torch.empty(max(k, 1), dtype=torch.int64, device=dev)  # noqa: E731
    cap = len(blob) // 16
    bufs = {"log_type": i32(n), "log_result": i32(n), "log_status": i32(n), "log_proj_off": i64(n),
            "log_proj_len": i32(n), "log_line0": i64(n), "n_lines": i64(1), "ev_line": i64(cap), "ev_start": i64(cap),
            "ev_len": i32(cap), "ev_flags": i32(cap), "n_events": i64(1)}
    o = E.FzBuildlogOut(**{k: C.c_void_p(v.data_ptr()) for k, v in bufs.items()}, event_cap=cap)

    def step():
        E._check(eng.lib, eng.lib.fz_buildlog(eng.ctx, C.c_void_p(d_text.data_ptr()), len(blob),
                                              offs.ctypes.data_as(C.c_void_p), C.c_void_p(d_offs.data_ptr()), n,
                                              C.byref(o)))
    step()
    torch.cuda.synchronize()
    assert int(bufs["n_lines"].item()) == n_lines
    eng.probe_begin("buildlog_classify,buildlog_lines")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    eng.probe_end()
    kern = {}
    for k in ("buildlog_classify", "buildlog_lines"):
        launches, ms, b = eng.probe_get(k)
        if launches:
            kern[k] = {"avg_launch_us": round(ms / launches * 1e3, 1), "GBps": round(b / (ms * 1e-3) / 1e9, 1),
                       "frac": round(b / (ms * 1e-3) / 1e9 / 8000.0, 4)}
    # whole drop-in call (upload of the texts, kernels, host srcmap extraction, dict assembly)
    t1 = time.perf_counter()
    res = buildlog.analyze(eng, rows[:len(batch)], texts[:len(batch)])
    t_full = time.perf_counter() - t1
    eng.close()
    # CPU: the oracle (per-line Python regexes, the reference's own algorithm) on a sample
    from oracle import buildlog_oracle as bo
    sample = batch[:args.cpu_sample]
    t2 = time.perf_counter()
    for r, t in sample:
        bo.build_infos(r, t)
    t_cpu = time.perf_counter() - t2
    cpu_lines = sum(len(t.splitlines()) for _, t in sample)
    ach = len(blob) / dt / 1e9
    print(json.dumps({
        "metric": "build-log lines/s (fz_buildlog: split + classify + fold, text resident in HBM)",
        "value": round(n_lines / dt, 1), "unit": "lines/s", "logs": n, "lines": n_lines, "bytes": len(blob),
        "ms_per_batch": round(dt * 1e3, 3), "text_GBps": round(ach, 1),
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": 8000.0, "unit": "GB/s",
                     "frac": round(ach / 8000.0, 4), "note": "whole call (3 text passes: count, write, classify)"},
        "kernels": kern,
        "dropin_analyze_s_per_log": round(t_full / len(batch), 6), "dropin_logs": len(batch), "results": len(res),
        "cpu_baseline": {"value": round(cpu_lines / t_cpu, 1), "unit": "lines/s", "cores": 1, "kind": "port",
                         "sample": f"oracle/buildlog_oracle.py on {len(sample)} logs ({cpu_lines} lines, {t_cpu:.1f} s)"}}),
          flush=True)


if __name__ == "__main__":
    main()
