"""End-to-end drop-in check on the GPU: the six script runners, fed from a columnar directory on
disk (store.save_columnar), write the reference's files under <cwd>/data/result_data and print its
stdout - compared with the golden fixtures produced by the unmodified reference scripts."""
import io
import os

import pandas as pd
import pytest

import goldens
from tse_amd import store
from tse_amd.rq import scripts

pytestmark = pytest.mark.gpu


def test_all_scripts_tiny(engine, tmp_path, monkeypatch, capsys):
    t0 = goldens.tables("tiny")
    store.save_columnar(t0, str(tmp_path / "col"))
    monkeypatch.setenv("FZ_DATA", str(tmp_path / "col"))
    t = scripts.load_tables()
    work = tmp_path / "work"
    work.mkdir()
    announced = []
    for name in scripts.SCRIPTS:
        capsys.readouterr()
        r = scripts.run(name, engine, t, cwd=str(work), figures=True)  # figures: side process, joined
        announced += [p for p, _ in r.figures]
        out = capsys.readouterr().out
        errs = goldens.compare_lines(out, goldens.text("tiny", name), rtol=1e-9)
        assert not errs, name + "\n" + "\n".join(errs)
    root = os.path.join(goldens.GOLDEN, "tiny", "result_data")
    n = 0
    for dp, _, fns in os.walk(root):
        for fn in fns:
            rel = os.path.relpath(os.path.join(dp, fn), root)
            if rel.endswith("manifest.json"):
                continue
            rel = rel[:-3] if rel.endswith(".gz") else rel
            ours = (work / "data" / "result_data" / rel).read_bytes()
            gold = goldens.file_bytes("tiny", rel)
            if rel.endswith("rq4_gc_introduction_iteration.csv"):
                a, b = pd.read_csv(io.BytesIO(ours)), pd.read_csv(io.BytesIO(gold))
                assert sorted(zip(a.Project, a.Introduction_Iteration)) == sorted(zip(b.Project, b.Introduction_Iteration))
            else:
                assert ours == gold, rel
            n += 1
    assert n >= 10
    for p in announced:  # the PDFs the reference writes (drawn from the libfz results)
        with open(work / p, "rb") as f:
            assert f.read(5) == b"%PDF-", p


def test_all_scripts_medium_figures(engine, tmp_path):
    """Every figure of the medium case drawn from the GPU results (rq2 per-project trends included)."""
    t = goldens.tables("medium")
    pdfs = 0
    for name in scripts.SCRIPTS:
        r = scripts.run(name, engine, t, cwd=str(tmp_path), figures=True)
        for p, _ in r.figures:
            assert (tmp_path / p).read_bytes()[:5] == b"%PDF-", p
    for dp, _, fns in os.walk(tmp_path / "data" / "result_data"):
        pdfs += sum(fn.endswith(".pdf") for fn in fns)
    assert pdfs >= 12
