"""All six analyses on a ten-times config-2 table (10,000 projects: ~19 M buildlog rows, ~9.5 M
coverage rows, ~650 k issues) - RQ1 / RQ2-add / RQ3 / RQ4a at a size the coverage-only configs 3 / 5
never reach - every output against the multi-core C++ restatement of the six scripts
(oracle/cpu/fz_cpu.cpp, held to the numpy oracle on the golden cases by test_cpu_baseline.py):
integers exact, fp64 within 1e-9 relative."""
import os

import pytest

import tse_amd.synth as synth
from oracle import cpu_baseline as cb
from test_cpu_baseline import check_port
from tse_amd.rq import compute

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]


def test_scaled_c2_all_analyses_vs_cpu_port(engine):
    t = synth.generate(synth.config("c2", n_projects=10_000))
    assert t.n_rows > 25_000_000 and len(t.i_project) > 500_000
    engine.upload(t)
    engine.build_store()
    res = {"rq1": compute.rq1(engine), "rq2_count": compute.rq2_count(engine), "rq2_add": compute.rq2_add(engine),
           "rq3": compute.rq3(engine), "rq4a": compute.rq4a(engine), "rq4b": compute.rq4b(engine)}
    engine.tables = None
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or 16), os.cpu_count() or 1))
    out, _ = cb.run(cb.HostTables(t), threads=threads)
    check_port(out, res)
