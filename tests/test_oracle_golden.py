"""The CPU oracle, rendered, reproduces the reference's own outputs (golden fixtures).

Golden fixtures were produced by running the unmodified reference scripts on the same
synthetic tables (tests/golden/make_goldens.py).  This pins the oracle (and the renderer)
before either is used to judge the GPU path.
"""
import hashlib
import io

import numpy as np
import pandas as pd
import pytest

import goldens
from oracle import rq_oracle as orc
from tse_amd.rq import render

CASES = goldens.CASES


def _check_files(case, rendered, prefix):
    import os
    root = os.path.join(goldens.GOLDEN, case, "result_data")
    n = 0
    for dp, _, fns in os.walk(root):
        for fn in fns:
            rel = os.path.relpath(os.path.join(dp, fn), root)
            if rel.endswith(".gz"):
                rel = rel[:-3]
            if not rel.startswith(prefix) or rel.endswith("manifest.json") or "change_analysis/" in rel:
                continue
            key = "data/result_data/" + rel
            assert key in rendered.files, f"missing output {key}"
            gold = goldens.file_bytes(case, rel)
            ours = rendered.files[key]
            if rel.endswith("rq4_gc_introduction_iteration.csv"):
                # tie order comes from Python set iteration + unstable sort in the reference
                a = pd.read_csv(io.BytesIO(ours))
                b = pd.read_csv(io.BytesIO(gold))
                assert list(a["Introduction_Iteration"]) == list(b["Introduction_Iteration"])
                assert sorted(zip(a.Project, a.Introduction_Iteration)) == sorted(zip(b.Project, b.Introduction_Iteration))
            else:
                assert ours == gold, f"{key} differs"
            n += 1
    return n


def _check_log(case, script, rendered):
    gl = goldens.golden_log(case, script).split("\n")
    ol = goldens.render_log(rendered).split("\n")
    # the Top/Bottom-5 tables inherit tie order from set iteration: compare their iteration column only
    def strip_tables(lines):
        out, skip = [], False
        for ln in lines:
            if "Projects (Earliest" in ln or "Projects (Latest" in ln:
                out.append(ln)
                skip = True
                continue
            if skip and (ln.startswith("[") and not ln.startswith("[RESULT]")):
                skip = False
            if skip:
                toks = ln.split()
                out.append(toks[-1] if toks else "")
                continue
            out.append(ln)
        return out
    errs = goldens.compare_lines("\n".join(strip_tables(ol)), "\n".join(strip_tables(gl)), rtol=0)
    assert not errs, "\n".join(errs)


@pytest.mark.parametrize("case", CASES)
def test_rq1(case):
    t = goldens.tables(case)
    r = render.rq1(orc.rq1(t), t)
    errs = goldens.compare_lines(r.text(), goldens.text(case, "rq1_detection_rate"))
    assert not errs, "\n".join(errs)
    assert _check_files(case, r, "rq1/") == 2


@pytest.mark.parametrize("case", CASES)
def test_rq2_count(case):
    t = goldens.tables(case)
    r = render.rq2_count(orc.rq2_count(t), t)
    errs = goldens.compare_lines(r.text(), goldens.text(case, "rq2_coverage_count"))
    assert not errs, "\n".join(errs)
    assert _check_files(case, r, "rq2/") == 1


@pytest.mark.parametrize("case", CASES)
def test_rq2_add(case):
    t = goldens.tables(case)
    r = render.rq2_add(orc.rq2_add(t), t)
    errs = goldens.compare_lines(r.text(), goldens.text(case, "rq2_coverage_and_added"))
    assert not errs, "\n".join(errs)
    _check_files(case, r, "rq3/all_coverage")
    man = goldens.manifest(case)
    ours = {k.split("/")[-1]: hashlib.sha256(v).hexdigest() for k, v in r.files.items() if "change_analysis/" in k}
    assert ours == man


@pytest.mark.parametrize("case", CASES)
def test_rq3(case):
    t = goldens.tables(case)
    r = render.rq3(orc.rq3(t), t)
    errs = goldens.compare_lines(r.text(), goldens.text(case, "rq3_diff_coverage_at_detection"))
    assert not errs, "\n".join(errs)
    assert _check_files(case, r, "rq3/detected") + _check_files(case, r, "rq3/non_detected") == 2


@pytest.mark.parametrize("case", CASES)
def test_rq4a(case):
    t = goldens.tables(case)
    r = render.rq4a(orc.rq4a(t), t)
    errs = goldens.compare_lines(r.text(), goldens.text(case, "rq4a_bug"))
    assert not errs, "\n".join(errs)
    _check_log(case, "rq4a_bug", r)
    assert _check_files(case, r, "rq4/") == 2


@pytest.mark.parametrize("case", CASES)
def test_rq4b(case):
    t = goldens.tables(case)
    res = orc.rq4b(t)
    r = render.rq4b(res, t, n_eligible=len(orc.eligible_projects(t)))
    errs = goldens.compare_lines(r.text(), goldens.text(case, "rq4b_coverage"))
    assert not errs, "\n".join(errs)
    _check_log(case, "rq4b_coverage", r)
