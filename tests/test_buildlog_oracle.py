"""The build-log oracle (oracle/buildlog_oracle.py) against the reference's own
buildlog_analysis() outputs on the committed synthetic logs (tests/golden/buildlog)."""
import gzip
import json
import os

import pytest

from oracle import buildlog_oracle as bo

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "buildlog")


def load():
    with gzip.open(os.path.join(HERE, "logs.json.gz"), "rt") as f:
        logs = json.load(f)["logs"]
    with gzip.open(os.path.join(HERE, "expected.json.gz"), "rt") as f:
        exp = json.load(f)
    return logs, exp


def test_oracle_matches_reference_outputs():
    logs, exp = load()
    assert len(logs) == len(exp) >= 300
    kinds = set()
    for lg, want in zip(logs, exp):
        if "raises" in want:
            with pytest.raises(getattr(__builtins__, want["raises"], Exception) if isinstance(__builtins__, dict)
                               else getattr(__import__("builtins"), want["raises"])):
                bo.build_infos(lg["row"], lg["text"])
            continue
        got = bo.build_infos(lg["row"], lg["text"])
        got["timecreated"] = str(got["timecreated"])
        assert got == want, lg["row"]["name"]
        kinds.add((want["build_type"], want["result"]))
    # the batch exercises every outcome of both fields
    assert {b for b, _ in kinds} >= {"", "Fuzzing", "Coverage", "Unknown", "coverage"}
    assert {r for _, r in kinds} >= {"Error", "Success", "Unknown"}
