"""Golden vectors for the build-log analysis: the reference's own
``buildlog_analysis(row)`` (program/preparation/4_get_buildlog_analysis.py:14-246), imported
unmodified from /root/reference with ``requests.get`` replaced by a stub that serves synthetic log
texts (tse_amd.synth_logs; the real logs live on storage.googleapis.com), run on every log of a
seeded batch.  Writes logs.json.gz (metadata rows + texts) and expected.json.gz (the returned
dicts, or the exception the reference raises).  Run in the build container only:

    python tests/golden/buildlog/make_buildlog_goldens.py
"""
import contextlib
import gzip
import importlib.util
import io
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, REPO)
REF = "/root/reference/program/preparation/4_get_buildlog_analysis.py"

import tse_amd  # noqa: E402,F401
from tse_amd import synth_logs  # noqa: E402


class _Resp:
    def __init__(self, text):
        self.text = text

    def raise_for_status(self):
        if self.text is None:
            raise RuntimeError("404 Client Error")


def main(seed=20241016, n_logs=300, mean_lines=150):
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
    cwd = os.getcwd()
    os.chdir("/tmp")  # the module creates its SAVE_FOLDER relative to the working directory
    try:
        spec = importlib.util.spec_from_file_location("ref_buildlog", REF)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        os.chdir(cwd)
    batch = synth_logs.make_batch(seed, n_logs, mean_lines)
    batch.append(({**batch[0][0], "name": "download-fails"}, None))
    texts = {}
    mod.requests.get = lambda url: _Resp(texts[url])
    expected = []
    for row, text in batch:
        texts[row["medialink"]] = text
        with contextlib.redirect_stdout(io.StringIO()):
            try:
                out = mod.buildlog_analysis(row)
                out["timecreated"] = str(out["timecreated"])
                expected.append(out)
            except Exception as e:  # noqa: BLE001
                expected.append({"raises": type(e).__name__})
    with gzip.open(os.path.join(HERE, "logs.json.gz"), "wt") as f:
        json.dump({"seed": seed, "logs": [{"row": r, "text": t} for r, t in batch]}, f)
    with gzip.open(os.path.join(HERE, "expected.json.gz"), "wt") as f:
        json.dump(expected, f, indent=0)
    print(len(batch), "logs;", sum("raises" in e for e in expected), "raise")


if __name__ == "__main__":
    main()
