"""Build-log analysis on the GPU: the drop-in for ``buildlog_analysis(row)`` and ``main()`` of
``program/preparation/4_get_buildlog_analysis.py`` for logs already on
disk (the reference downloads each one with ``requests.get``, :44-52 - network, out of scope).

``analyze(eng, rows, texts)`` uploads a whole batch of log texts to HBM once and runs ``fz_buildlog``
(csrc/fz_buildlog.hip): str.splitlines() lines, per-line pattern classification and a per-log fold
give project / build_type / result; the host then extracts the srcmap entries (jq_inplace lines
and JSON blocks, :162-214) from the few lines the kernel lists, and assembles the reference's
``build_infos`` dicts (:29-42, 218-223).  A log of exactly one line makes the reference raise
IndexError (:230): ``analyze`` raises it too (``errors="raise"``) or returns the exception object
in that log's slot (``errors="keep"``).
"""
from __future__ import annotations

import ctypes as C
import json
import os
import re
from typing import List, Optional, Sequence

import numpy as np

from . import engine as E

BUILD_TYPES = ["", "coverage", "introspector", "Fuzzing", "Unknown", "Introspector", "Coverage"]  # FZ_BT_*
RESULTS = ["", "Error", "Success", "Unknown"]                                                      # FZ_BR_*
BL_SKIP, BL_JQ, BL_OPEN, BL_CLOSE = 1 << 2, 1 << 8, 1 << 9, 1 << 10

# the srcmap patterns of :64-65, 166-170 (host side: the lines the kernel lists)
_JQ = re.compile(r"jq_inplace [^ ]+ '(.*?)'")
_JSON_LINE = re.compile(r"Step #\d+:\s?(.*)")
_JQ_PATH = re.compile(r'"(.+?)"\s*=')
_JQ_TYPE = re.compile(r'type:\s*"(.+?)"')
_JQ_URL = re.compile(r'url:\s*"(.+?)"')
_JQ_REV = re.compile(r'rev:\s*"(.+?)"')


class _Sources:
    def __init__(self):
        self.paths: List[str] = []
        self.types: List[str] = []
        self.urls: List[str] = []
        self.revs: List[str] = []

    def jq(self, line: str) -> None:
        m = _JQ.search(line)
        if not m:
            return
        c = m.group(1)
        parts = (_JQ_PATH.search(c), _JQ_TYPE.search(c), _JQ_URL.search(c), _JQ_REV.search(c))
        if all(parts):
            self.paths.append(parts[0].group(1))
            self.types.append(parts[1].group(1))
            self.urls.append(parts[2].group(1))
            self.revs.append(parts[3].group(1))

    def block(self, lines: List[str]) -> None:
        """A "Step #N: {" ... '}' block (:183-214): group(1) of every line joined, parsed as JSON."""
        text = "".join(m.group(1) for m in (_JSON_LINE.search(x) for x in lines) if m)
        try:
            parsed = json.loads(text)
        except json.JSONDecodeError:
            return
        for path, d in parsed.items():
            self.paths.append(path)
            self.types.append(d.get("type", ""))
            self.urls.append(d.get("url", ""))
            self.revs.append(d.get("rev", ""))


def _sources(raw: bytes, ev_line, ev_start, ev_len, ev_flags, skip_lines) -> _Sources:
    """The jq / JSON state machine of :162-214 over one log's listed lines (in line order)."""
    src = _Sources()
    open_k = -1
    for k in range(len(ev_line)):
        f = int(ev_flags[k])
        if f & BL_SKIP:
            continue
        if f & BL_JQ:
            src.jq(raw[ev_start[k]:ev_start[k] + ev_len[k]].decode("utf-8"))
        if open_k < 0:
            if f & BL_OPEN:
                open_k = k
            continue
        if f & BL_CLOSE:  # the block: every line from the opening one to this one, skip lines left out
            a, b = int(ev_start[open_k]), int(ev_start[k] + ev_len[k])
            lines = raw[a:b].decode("utf-8").splitlines()
            l0 = int(ev_line[open_k])
            assert len(lines) == int(ev_line[k]) - l0 + 1
            src.block([x for i, x in enumerate(lines) if (l0 + i) not in skip_lines])
            open_k = -1
    return src


def analyze(eng: "E.Engine", rows: Sequence[dict], texts: Sequence[Optional[str]], errors: str = "raise") -> list:
    """build_infos of every (metadata row, log text) pair; text None = the download failed (the
    reference returns the defaults, :50-52)."""
    import pandas as pd
    torch = eng.torch
    raws = [b"" if t is None else t.encode("utf-8") for t in texts]
    offs = np.zeros(len(raws) + 1, dtype=np.int64)
    np.cumsum([len(r) for r in raws], out=offs[1:])
    blob = b"".join(raws)
    n = len(raws)
    dev = eng.dev
    d_text = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev) if blob else torch.zeros(1, dtype=torch.uint8,
                                                                                                   device=dev)
    d_offs = torch.from_numpy(offs).to(dev)
    i32 = lambda k: torch.empty(max(k, 1), dtype=torch.int32, device=dev)  # noqa: E731
    i64 = lambda k: torch.empty(max(k, 1), dtype=torch.int64, device=dev)  # noqa: E731
    outs = {"log_type": i32(n), "log_result": i32(n), "log_status": i32(n), "log_proj_off": i64(n),
            "log_proj_len": i32(n), "log_line0": i64(n), "n_lines": i64(1), "n_events": i64(1)}
    cap = max(1024, len(blob) // 256)
    while True:
        ev = {"ev_line": i64(cap), "ev_start": i64(cap), "ev_len": i32(cap),
              "ev_flags": torch.empty(cap, dtype=torch.int32, device=dev)}
        o = E.FzBuildlogOut(**{k: C.c_void_p(v.data_ptr()) for k, v in {**outs, **ev}.items()}, event_cap=cap)
        E._check(eng.lib, eng.lib.fz_buildlog(eng.ctx, C.c_void_p(d_text.data_ptr()), len(blob),
                                              offs.ctypes.data_as(C.c_void_p), C.c_void_p(d_offs.data_ptr()), n,
                                              C.byref(o)))
        n_ev = int(outs["n_events"].item())
        if n_ev <= cap:
            break
        cap = n_ev
    host = {k: v[:n].cpu().numpy() for k, v in outs.items() if k.startswith("log_")}
    evh = {k: v[:n_ev].cpu().numpy() for k, v in ev.items()}
    order = np.argsort(evh["ev_line"], kind="stable")
    evh = {k: v[order] for k, v in evh.items()}
    bounds = np.searchsorted(evh["ev_line"], np.append(host["log_line0"], np.iinfo(np.int64).max))
    out = []
    for g, (row, text) in enumerate(zip(rows, texts)):
        try:
            tc = pd.to_datetime(row["timecreated"])
        except Exception:  # noqa: BLE001  (:25-27: printed, the analysis goes on with None)
            tc = None
        info = {"id": row["name"], "size": int(row["size"]), "project": "", "build_type": "", "result": "",
                "timecreated": tc, "modules": [], "path": [], "revisions": [], "types": [], "repo_urls": [],
                "download_link": row["medialink"]}
        st = int(host["log_status"][g])
        if text is None or st == 1:
            out.append(info)
            continue
        if st == 2:
            err = IndexError("list index out of range")
            if errors == "raise":
                raise err
            out.append(err)
            continue
        a, b = bounds[g], bounds[g + 1]
        ev_g = {k: v[a:b] for k, v in evh.items()}
        skip = set(ev_g["ev_line"][(ev_g["ev_flags"] & BL_SKIP) != 0].tolist())
        src = _sources(blob, ev_g["ev_line"], ev_g["ev_start"], ev_g["ev_len"], ev_g["ev_flags"], skip)
        po = int(host["log_proj_off"][g])
        info.update(project=blob[po:po + int(host["log_proj_len"][g])].decode("utf-8") if po >= 0 else "",
                    build_type=BUILD_TYPES[int(host["log_type"][g])], result=RESULTS[int(host["log_result"][g])],
                    modules=[p.split("/")[-1].capitalize() for p in src.paths], path=src.paths,
                    revisions=src.revs, types=src.types, repo_urls=src.urls)
        out.append(info)
    return out


def main(csv_path: str = "data/processed_data/csv/buildlog_metadata.csv",
         save_folder: str = "data/processed_data/csv/buildlog_analyzed_batches", log_dir: Optional[str] = None,
         limit: Optional[int] = 10) -> int:
    """main() of the reference (:249-288) over logs already downloaded into ``log_dir`` (default
    $FZ_BUILDLOG_DIR, else data/buildlogs) as log-<name>.txt; ``limit`` = the first 10 unprocessed
    rows as there (None: all of them, one GPU batch)."""
    import glob

    import pandas as pd
    log_dir = log_dir or os.environ.get("FZ_BUILDLOG_DIR", os.path.join("data", "buildlogs"))
    os.makedirs(save_folder, exist_ok=True)
    try:
        df = pd.read_csv(csv_path)
    except FileNotFoundError:
        print(f"Error: CSV file not found: {csv_path}")
        return 0
    if not all(c in df.columns for c in ["name", "selflink", "medialink", "size", "timecreated"]):
        print("CSV is missing required columns")
        return 0
    done = set()
    for fp in glob.glob(os.path.join(save_folder, "*.csv")):
        try:
            prev = pd.read_csv(fp)
            if "id" in prev.columns:
                done.update(prev["id"].dropna().tolist())
        except Exception as e:  # noqa: BLE001
            print(f"Failed to load: {fp}, {e}")
    df = df[~df["name"].isin(done)]
    if df.empty:
        print("No new data to process.")
        return 0
    print(f"Processing first {limit} items from unprocessed data (total {len(df)}items)" if limit else
          f"Processing all {len(df)} unprocessed items")
    part = df.head(limit) if limit else df
    rows = part.to_dict("records")
    texts = []
    for r in rows:
        fp = os.path.join(log_dir, f"log-{r['name']}.txt")
        texts.append(open(fp, encoding="utf-8", newline="").read() if os.path.exists(fp) else None)
    eng = E.Engine(0)
    try:
        results = analyze(eng, rows, texts)
    finally:
        eng.close()
    if results:
        save = os.path.join(save_folder, f"batch_debug_{len(results)}_items.csv")
        pd.DataFrame(results).to_csv(save, index=False)
        print(f"\n💾 Saved {len(results)} entries to {save}")
    return 0
