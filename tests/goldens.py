"""Helpers to load golden fixtures (``tests/golden/<case>/``) and compare rendered output."""
from __future__ import annotations

import gzip
import json
import os
import re
from functools import lru_cache

import numpy as np

import tse_amd.synth as synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["tiny", "medium"]
SCRIPTS = ["rq1_detection_rate", "rq2_coverage_count", "rq2_coverage_and_added",
           "rq3_diff_coverage_at_detection", "rq4a_bug", "rq4b_coverage"]


@lru_cache(maxsize=4)
def tables(case):
    """The synthetic table of a golden case ('tiny', 'medium', or 'tiny+<edge>' of null_edges)."""
    import null_edges
    with open(os.path.join(GOLDEN, case, "meta.json")) as f:
        meta = json.load(f)
    base, edge = null_edges.split(case)
    t = synth.generate(synth.config(base))
    if edge:
        t = null_edges.apply(t, edge)
    fp = null_edges.fingerprint(t) if edge else synth.table_fingerprint(t)
    assert fp == meta["fingerprint"], \
        f"synthetic tables for '{case}' drifted from the golden fixture; regenerate goldens"
    return t


def returncode(case, script):
    with open(os.path.join(GOLDEN, case, "meta.json")) as f:
        return json.load(f)["scripts"][script]["returncode"]


def text(case, script, stream="stdout"):
    with open(os.path.join(GOLDEN, case, script, f"{stream}.txt")) as f:
        return f.read()


def file_bytes(case, rel):
    p = os.path.join(GOLDEN, case, "result_data", rel)
    if os.path.exists(p):
        with open(p, "rb") as f:
            return f.read()
    if os.path.exists(p + ".gz"):
        with gzip.open(p + ".gz", "rb") as f:
            return f.read()
    return None


def manifest(case):
    p = os.path.join(GOLDEN, case, "result_data", "rq3", "change_analysis_manifest.json")
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f)


_NUM = re.compile(r"[-+]?(?:\d[\d,]*\.?\d*(?:[eE][-+]?\d+)?|\.\d+(?:[eE][-+]?\d+)?|nan|inf)")


def _tokens(line):
    out, pos = [], 0
    for m in _NUM.finditer(line):
        out.append(("s", line[pos:m.start()]))
        out.append(("n", m.group(0)))
        pos = m.end()
    out.append(("s", line[pos:]))
    return out


def _sig_digits(tok: str) -> int:
    mant = tok.lower().split("e")[0].lstrip("+-").replace(",", "").replace(".", "").lstrip("0")
    return len(mant)


def _close(a: str, b: str, rtol: float) -> bool:
    """Numeric tokens compare exactly, except full-precision values (>= 12 significant digits, e.g.
    repr(np.float64) of a statistic), which may differ within rtol: an fp64 statistic that agrees
    to 1e-9 relative can print different trailing digits, but a rounded value (.2f/.4f, counts,
    percentages) must print the same digits."""
    if a == b:
        return True
    try:
        x, y = float(a.replace(",", "")), float(b.replace(",", ""))
    except ValueError:
        return False
    if np.isnan(x) and np.isnan(y):
        return True
    if min(_sig_digits(a), _sig_digits(b)) < 12:
        return False
    return abs(x - y) <= rtol * max(abs(x), abs(y))


def compare_lines(ours, golden, rtol=0.0):
    """Line-by-line compare; only full-precision numeric tokens may differ (within rtol)."""
    lo, lg = ours.rstrip("\n").split("\n"), golden.rstrip("\n").split("\n")
    errs = []
    if len(lo) != len(lg):
        errs.append(f"line count {len(lo)} != {len(lg)}")
    for k, (a, b) in enumerate(zip(lo, lg)):
        if a == b:
            continue
        ta, tb = _tokens(a), _tokens(b)
        ok = len(ta) == len(tb) and all(
            (x[0] == y[0]) and (x[1] == y[1] if x[0] == "s" else (rtol > 0 and _close(x[1], y[1], rtol)))
            for x, y in zip(ta, tb))
        if not ok:
            errs.append(f"line {k}: ours={a!r}\n         gold={b!r}")
        if len(errs) > 10:
            break
    return errs


_TS = re.compile(r"^\d{4}-\d\d-\d\d \d\d:\d\d:\d\d ")


def golden_log(case, script):
    """stderr of the reference with timestamps stripped and tqdm remnants dropped."""
    out = []
    for ln in text(case, script, "stderr").split("\n"):
        if not ln.strip():
            continue
        out.append(_TS.sub("", ln))
    return "\n".join(out) + "\n"


def render_log(rendered):
    out = list(rendered.preamble_stderr)
    for lvl, msg in rendered.log:
        lines = f"[{lvl}] {msg}".split("\n")
        out.extend(ln for ln in lines if ln.strip())
    return "\n".join(out) + "\n"
