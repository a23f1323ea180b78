"""The drop-in at the reference's own invocation (run_all_analysis.sh:13-46): from a working
directory laid out like the reference checkout, `python3 program/research_questions/<rq>.py` with
no arguments, one process per script, reads ./data/columnar and writes the reference's stdout and
files under ./data/result_data - compared with the golden outputs of the unmodified reference
scripts on the same tables."""
import os
import subprocess
import sys

import pytest

import goldens
from tse_amd import store
from tse_amd.rq import scripts

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_paths_argumentless(tmp_path):
    work = tmp_path / "checkout"
    (work / "data").mkdir(parents=True)
    os.symlink(os.path.join(REPO, "program"), work / "program")
    store.save_columnar(goldens.tables("tiny"), str(work / "data" / "columnar"))
    env = {k: v for k, v in os.environ.items() if k not in ("FZ_DATA", "FZ_ENGINE_ROOT")}
    env["FZ_FIGURES"] = "0"
    for name in scripts.SCRIPTS:
        p = subprocess.run([sys.executable, f"program/research_questions/{name}.py"], cwd=work, env=env,
                           capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, name + "\n" + p.stderr[-3000:]
        errs = goldens.compare_lines(p.stdout, goldens.text("tiny", name), rtol=1e-9)
        assert not errs, name + "\n" + "\n".join(errs)
    root = os.path.join(goldens.GOLDEN, "tiny", "result_data")
    n = 0
    for dp, _, fns in os.walk(root):
        for fn in fns:
            rel = os.path.relpath(os.path.join(dp, fn), root)
            if rel.endswith("manifest.json") or "rq4_gc_introduction_iteration" in rel:
                continue  # (row order of that file is a dict order of the reference; test_gpu_scripts)
            rel = rel[:-3] if rel.endswith(".gz") else rel
            assert (work / "data" / "result_data" / rel).read_bytes() == goldens.file_bytes("tiny", rel), rel
            n += 1
    assert n >= 10
