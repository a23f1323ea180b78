"""CPU ORACLE (test infrastructure only - see oracle/__init__.py).

Restatement of the build-log analysis of the reference's preparation step,
``program/preparation/4_get_buildlog_analysis.py:14-246`` (``buildlog_analysis(row)``), for a log
whose text is already at hand (the reference downloads it with ``requests.get`` at :44-52; the
network part is out of scope).  Written as the GPU path computes it: every line is classified on
its own (``classify``), then one fold per log combines the line events (``fold``):

* project      - the first line with an image or GCS match, the image preferred (:84-98);
* build_type   - lines either SET a value (a "Starting Step" line :101-118, or the last of the
                 intro / html / base-runner / compile matches of a line :120-149), or apply the
                 PUSH DONE rule "Fuzzing unless Coverage / Introspector" (:150-152), or nothing;
                 "Starting Step" lines with an empty / srcmap / build step skip the rest of the
                 line's processing (:104-105);
* paths etc.   - jq_inplace lines (:163-180) and "Step #N: {" ... "}" blocks parsed as JSON
                 (:183-214), in line order; modules = last path component, capitalised (:219);
* result       - from the last 200 lines (:228-237).

Reference quirks kept: the ERROR pattern ``\\nERROR.*`` (:70) can never match a line from
``splitlines()`` (no per-line Error type); the per-line ``result`` variable (:153-159) is never
stored; a log of exactly one line raises IndexError at ``lines[-2]`` (:230); a JSON block ends at
the first line ending with '}' (so multi-line inner objects never parse); ``.`` in the patterns'
``gcr.io`` matches any character.

Pinned by tests/golden/buildlog (make_buildlog_goldens.py runs the reference's own function on
synthetic logs).
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field
from typing import List, Optional

IMAGE = re.compile(r"Already have image: gcr\.io/oss-fuzz/([^\s:]+)")
GCS = re.compile(r"No URLs matched: gs://oss-fuzz-coverage/([^/]+)/textcov_reports")
STEP = re.compile(r"Starting Step #\d+\s*(.*)")                      # matched at the line start
INTRO = re.compile(r"Step #(\d+): Pulling image: gcr.io/oss-fuzz-base/base-runner")
HTML = re.compile(r"/report/.*\.html")
BASE_RUNNER = re.compile(r"Unable to find image 'gcr.io/oss-fuzz-base/base-runner:latest' locally")
PUSH_DONE = re.compile(r"PUSH\s*DONE", re.DOTALL)
COMPILE = re.compile(r"compile-(.*)-(.*)-x86_64")
JQ = re.compile(r"jq_inplace [^ ]+ '(.*?)'")
JSON_LINE = re.compile(r"Step #\d+:\s?(.*)")
FUZZ_STEPS = ("address-x86_64", "undefined-x86_64", "memory-x86_64", "none-x86_64", "address-i386")


@dataclass
class LineEvent:
    image: Optional[str] = None
    gcs: Optional[str] = None
    skip: bool = False          # "Starting Step" line that ends the line's processing
    set_to: Optional[str] = None
    push_done: bool = False     # the PUSH DONE rule applies after set_to
    jq: Optional[str] = None    # jq_inplace payload


def classify(line: str) -> LineEvent:
    ev = LineEvent()
    m = IMAGE.search(line)
    ev.image = m.group(1) if m else None
    m = GCS.search(line)
    ev.gcs = m.group(1) if m else None
    m = STEP.match(line)
    if m:
        text = m.group(1).strip().replace('"', "")
        if text == "" or "srcmap" in text or "build" in text:
            ev.skip = True
            return ev
        if "coverage" in text:
            ev.set_to = "coverage"
        elif "introspector" in text:
            ev.set_to = "introspector"
        elif any(k in text for k in FUZZ_STEPS):
            ev.set_to = "Fuzzing"
        else:
            ev.set_to = "Unknown"
    else:
        m = INTRO.search(line)
        if m:
            ev.set_to = {"0": "Introspector", "4": "Coverage", "5": "Fuzzing"}.get(m.group(1), "Unknown")
        if HTML.search(line):
            ev.set_to = "Coverage"
        if BASE_RUNNER.search(line):
            ev.set_to = "Fuzzing"
        m = COMPILE.search(line)
        if m:
            ev.set_to = {"address": "Fuzzing", "memory": "Fuzzing", "undefined": "Fuzzing", "none": "Fuzzing",
                         "coverage": "Coverage", "introspector": "Introspector"}.get(m.group(2), "Unknown")
        ev.push_done = PUSH_DONE.search(line) is not None
    m = JQ.search(line)
    ev.jq = m.group(1) if m else None
    return ev


def push_done_rule(state: str) -> str:
    return state if state in ("Coverage", "Introspector") else "Fuzzing"


@dataclass
class LogResult:
    project: str = ""
    build_type: str = ""
    result: str = ""
    paths: List[str] = field(default_factory=list)
    types: List[str] = field(default_factory=list)
    repo_urls: List[str] = field(default_factory=list)
    revisions: List[str] = field(default_factory=list)

    @property
    def modules(self) -> List[str]:
        return [p.split("/")[-1].capitalize() for p in self.paths]


def _jq_fields(res: LogResult, content: str) -> None:
    path = re.search(r'"(.+?)"\s*=', content)
    typ = re.search(r'type:\s*"(.+?)"', content)
    url = re.search(r'url:\s*"(.+?)"', content)
    rev = re.search(r'rev:\s*"(.+?)"', content)
    if path and typ and url and rev:
        res.paths.append(path.group(1))
        res.types.append(typ.group(1))
        res.repo_urls.append(url.group(1))
        res.revisions.append(rev.group(1))


def sources(res: LogResult, lines: List[str], events: List[LineEvent]) -> None:
    """jq_inplace lines and JSON blocks, in line order (4_get_buildlog_analysis.py:162-214)."""
    collecting, parts = False, []
    for line, ev in zip(lines, events):
        if ev.skip:
            continue
        if ev.jq is not None:
            _jq_fields(res, ev.jq)
        if not collecting and "{" in line and line.strip().endswith("{"):
            m = JSON_LINE.search(line)
            if m and m.group(1).strip() == "{":
                collecting, parts = True, [m.group(1)]
                continue
        if collecting:
            m = JSON_LINE.search(line)
            if m:
                parts.append(m.group(1))
            if line.strip().endswith("}"):
                collecting = False
                try:
                    block = json.loads("".join(parts))
                    for path, d in block.items():
                        res.paths.append(path)
                        res.types.append(d.get("type", ""))
                        res.repo_urls.append(d.get("url", ""))
                        res.revisions.append(d.get("rev", ""))
                except json.JSONDecodeError:
                    pass
                parts = []


def tail_result(lines: List[str]) -> str:
    """4_get_buildlog_analysis.py:228-237 (len(lines) == 1 raises IndexError, as there)."""
    tail = [x.strip() for x in lines[-200:]]
    if "ERROR" in lines[-2] or "ERROR" in tail:
        return "Error"
    if "PUSH" in tail and "DONE" in tail:
        return "Success"
    if "ERROR: context deadline exceeded" in tail:
        return "Error"
    return "Unknown"


def fold(lines: List[str], events: List[LineEvent]) -> LogResult:
    res = LogResult()
    for ev in events:
        name = ev.image or ev.gcs
        if name:
            res.project = name
            break
    state = ""
    for ev in events:
        if ev.set_to is not None:
            state = ev.set_to
        if ev.push_done:
            state = push_done_rule(state)
    res.build_type = state
    sources(res, lines, events)
    res.result = tail_result(lines)
    return res


def analyze_text(text: str) -> LogResult:
    """One log's text -> the fields buildlog_analysis() fills (empty log: all defaults, :54-55)."""
    lines = text.splitlines()
    if not lines:
        return LogResult()
    return fold(lines, [classify(x) for x in lines])


def build_infos(row: dict, text: Optional[str]) -> dict:
    """The dict buildlog_analysis(row) returns (:29-42, 218-223), text None = download failed."""
    import pandas as pd
    try:
        tc = pd.to_datetime(row["timecreated"])
    except Exception:  # noqa: BLE001  (the reference prints and continues, :25-27)
        tc = None
    out = {"id": row["name"], "size": int(row["size"]), "project": "", "build_type": "", "result": "",
           "timecreated": tc, "modules": [], "path": [], "revisions": [], "types": [], "repo_urls": [],
           "download_link": row["medialink"]}
    if text is None:
        return out
    r = analyze_text(text)
    if not text.splitlines():
        return out
    out.update(project=r.project, build_type=r.build_type, result=r.result, modules=r.modules, path=r.paths,
               revisions=r.revisions, types=r.types, repo_urls=r.repo_urls)
    return out
