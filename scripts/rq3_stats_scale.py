"""Time fz_rq3_stats on the config-2 RQ3 samples replicated x1 / x2 / x4 / x8 (what every rank of
the sharded step recomputes after the all-gather at world size N)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    import tse_amd.synth as synth
    from tse_amd import engine as E
    from tse_amd import parallel as par
    t = synth.generate(synth.config("c2"))
    eng = E.Engine(0)
    eng.upload(t)
    eng.build_store()
    sh = par.GpuRQ3Shard(eng)
    part = sh.run()
    det_pct, det_tot, non_pct = part["det_pct"], part["det_tot"], part["non_pct"]
    print("det", det_pct.numel(), "non", non_pct.numel(), flush=True)
    for k in (1, 2, 4, 8):
        a, b, c = det_pct.repeat(k), det_tot.repeat(k), non_pct.repeat(k)
        for _ in range(2):
            sh.stats(a, b, c)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            sh.stats(a, b, c)
        torch.cuda.synchronize()
        print(f"x{k}: {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
