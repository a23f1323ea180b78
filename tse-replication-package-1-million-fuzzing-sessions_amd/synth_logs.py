"""Synthetic OSS-Fuzz Cloud Build logs (the inputs of 4_get_buildlog_analysis.py, which downloads
them from storage.googleapis.com - unavailable offline).  Deterministic per seed.  Each log mixes
the line shapes the analysis looks for (image / GCS project lines, "Starting Step" lines of every
kind, base-runner pulls, coverage report links, compile step names, PUSH / DONE / ERROR tails,
srcmap jq_inplace lines and JSON blocks - parseable and not) with filler build output, CRLF / CR /
form-feed line breaks and non-ASCII text, so every branch and quirk of the analysis is exercised.
"""
from __future__ import annotations

import random
from typing import List, Tuple

ENGINES = ["libfuzzer", "afl", "honggfuzz", "centipede"]
SANITIZERS = ["address", "undefined", "memory", "none", "coverage", "introspector", "dataflow"]


def _hex(r: random.Random, n: int) -> str:
    return "".join(r.choice("0123456789abcdef") for _ in range(n))


def _project(r: random.Random) -> str:
    return r.choice(["abseil-cpp", "libpng", "zlib", "openssl", "curl", "sqlite3", "json-c", "libxml2", "re2",
                     "ffmpeg", "harfbuzz", "php", "boringssl", "mruby", "tinyxml2"])


def _filler(r: random.Random, step: int) -> str:
    k = r.randrange(9)
    if k == 0:
        return f"Step #{step}: [{r.randrange(100):3d}%] Building CXX object src/CMakeFiles/x.dir/f{r.randrange(999)}.cc.o"
    if k == 1:
        return f"Step #{step}: {_hex(r, 12)}: Pull complete"
    if k == 2:
        return f"Step #{step}: INFO: Seed: {r.randrange(1 << 31)}"
    if k == 3:
        return f"Step #{step}: #{r.randrange(10 ** 6)}\tNEW    cov: {r.randrange(9999)} ft: {r.randrange(9999)}"
    if k == 4:
        return f"Step #{step}: Ünïcödé lïne — {r.randrange(100)} ✓"
    if k == 5:
        return f"Step #{step}: Digest: sha256:{_hex(r, 64)}"
    if k == 6:
        return f"Step #{step}: Status: Downloaded newer image for gcr.io/oss-fuzz-base/base-builder:latest"
    if k == 7:
        return ""
    return f"Step #{step}:   {'x' * r.randrange(40)} }} {{ '{r.randrange(9)}'"


def _step_name(r: random.Random) -> str:
    k = r.randrange(10)
    if k == 0:
        return ""
    if k == 1:
        return ' - "srcmap"'
    if k == 2:
        return f' - "build-check-{r.choice(ENGINES)}-{r.choice(SANITIZERS)}-x86_64"'
    if k == 3:
        return f' - "compile-{r.choice(ENGINES)}-{r.choice(SANITIZERS)}-x86_64"'
    if k == 4:
        return f' - "compile-{r.choice(ENGINES)}-address-i386"'
    if k == 5:
        return ' - "introspector"'
    if k == 6:
        return ' - "upload-coverage"'
    if k == 7:
        return f' - "{r.choice(["push", "tests", "zip", "gsutil"])}"'
    if k == 8:
        return '   "  "   '
    return f' - "{r.choice(["compile", "run"])}-{r.choice(SANITIZERS)}-x86_64"'


def _srcmap_jq(r: random.Random, proj: str, step: int) -> str:
    path = f"/src/{proj if r.random() < 0.6 else _project(r) + '-' + _hex(r, 3)}"
    ok = r.random() < 0.8
    fields = [f'type: "git"', f'url: "https://github.com/x/{proj}.git"', f'rev: "{_hex(r, 40)}"']
    if not ok:
        fields.pop(r.randrange(3))
    return f"Step #{step}: + jq_inplace /tmp/file{_hex(r, 6)} '.\"{path}\" = {{ {', '.join(fields)} }}'"


def _srcmap_json(r: random.Random, proj: str, step: int) -> List[str]:
    n = 1 + r.randrange(3)
    if r.random() < 0.6:  # one line per entry: the block parses
        body = []
        for k in range(n):
            sep = "," if k < n - 1 else ""
            body.append(f'Step #{step}:   "/src/{proj}{k}": {{"type": "git", "url": "https://g/{proj}{k}", '
                        f'"rev": "{_hex(r, 40)}"}}{sep}')
        return [f"Step #{step}: {{"] + body + [f"Step #{step}: }}"]
    out = [f"Step #{step}:{' ' if r.random() < 0.5 else ''}{{"]  # nested lines: ends at the inner '}'
    for k in range(n):
        out += [f'Step #{step}:   "/src/{proj}{k}": {{', f'Step #{step}:     "type": "git",',
                f'Step #{step}:     "rev": "{_hex(r, 8)}"', f"Step #{step}:   }}" + ("," if k < n - 1 else "")]
    return out + [f"Step #{step}: }}"]


def _special(r: random.Random, proj: str, step: int) -> List[str]:
    k = r.randrange(16)
    if k == 0:
        return [f"Step #{step}: Already have image: gcr.io/oss-fuzz/{proj}{':latest' if r.random() < 0.5 else ''}"]
    if k == 1:
        return [f"Step #{step}: CommandException: No URLs matched: gs://oss-fuzz-coverage/{proj}/textcov_reports/"
                f"2024{r.randrange(10, 13)}{r.randrange(10, 29)}/*"]
    if k == 2:
        return [f"Starting Step #{step}{_step_name(r)}"]
    if k == 3:
        return [f"Step #{r.choice([0, 4, 5, 7, 12])}: Pulling image: gcr.io/oss-fuzz-base/base-runner"]
    if k == 4:
        return [f"Step #{step}: Coverage report: https://storage.googleapis.com/oss-fuzz-coverage/{proj}/reports/"
                f"2024/linux/report/index.html"]
    if k == 5:
        return [f"Step #{step}: Unable to find image 'gcr.io/oss-fuzz-base/base-runner:latest' locally"]
    if k == 6:
        return [f"Step #{step} - \"compile-{r.choice(ENGINES)}-{r.choice(SANITIZERS)}-x86_64\": done"]
    if k == 7:
        return [r.choice(["PUSH", "DONE", "PUSH DONE", "PUSHDONE", " PUSH ", "ERROR", "ERROR: context deadline exceeded",
                          f"Step #{step}: ERROR: build step failed"])]
    if k == 8:
        return [_srcmap_jq(r, proj, step)]
    if k == 9:
        return _srcmap_json(r, proj, step)
    if k == 10:
        return [f"Step #{step}: Pulling image: gcrXio/oss-fuzz-base/base-runner"]  # '.' matches any char
    if k == 11:
        return [f"Step #{step}: compile-a-b-c-x86_64 and compile-{r.choice(SANITIZERS)}-x86_64-x86_64"]
    if k == 12:
        return [f"Starting Step #{step} \"compile-{r.choice(ENGINES)}-coverage-x86_64\""]
    if k == 13:
        return [f"Step #{step}: Already have image: gcr.io/oss-fuzz/{_project(r)} and No URLs matched: "
                f"gs://oss-fuzz-coverage/{_project(r)}/textcov_reports"]
    if k == 14:
        return ["PUSH", "DONE"]
    return [f"Step #{step}: PUSH\t DONE"]


def make_log(r: random.Random, n_lines: int) -> str:
    proj = _project(r)
    lines: List[str] = [f'starting build "{_hex(r, 8)}-{_hex(r, 4)}"', "", "FETCHSOURCE", "BUILD"]
    step = 0
    while len(lines) < n_lines:
        if r.random() < 0.05:
            step += 1
        lines += _special(r, proj, step) if r.random() < 0.25 else [_filler(r, step)]
    lines = lines[:n_lines]
    seps = []
    for _ in lines:
        x = r.random()
        seps.append("\n" if x < 0.9 else "\r\n" if x < 0.95 else "\r" if x < 0.97 else "\x0c" if x < 0.98
                    else "\x1e" if x < 0.99 else " ")
    text = "".join(a + b for a, b in zip(lines, seps))
    return text if r.random() < 0.8 else text.rstrip("\n\r\x0c\x1e ")


def make_batch(seed: int, n_logs: int, mean_lines: int = 400) -> List[Tuple[dict, str]]:
    """(metadata row of buildlog_metadata.csv, log text) pairs; a few empty / one-line logs."""
    r = random.Random(seed)
    out = []
    for k in range(n_logs):
        name = f"{_hex(r, 8)}-{_hex(r, 4)}-{_hex(r, 4)}-{_hex(r, 4)}-{_hex(r, 12)}"
        row = {"name": name, "selflink": f"https://www.googleapis.com/storage/v1/b/oss-fuzz-build-logs/o/log-{name}.txt",
               "medialink": f"https://storage.googleapis.com/download/storage/v1/b/oss-fuzz-build-logs/o/log-{name}.txt",
               "size": r.randrange(1000, 10 ** 7),
               "timecreated": f"2024-{r.randrange(1, 13):02d}-{r.randrange(1, 29):02d}T{r.randrange(24):02d}:"
                              f"{r.randrange(60):02d}:{r.randrange(60):02d}.{r.randrange(1000):03d}Z"}
        x = r.random()
        if x < 0.02:
            text = ""
        elif x < 0.04:
            text = "\n\n\n"
        elif x < 0.05:
            text = f"Step #0: Already have image: gcr.io/oss-fuzz/{_project(r)}\n"  # one line: lines[-2] raises
        else:
            text = make_log(r, max(2, int(r.expovariate(1.0 / mean_lines))))
        out.append((row, text))
    return out
