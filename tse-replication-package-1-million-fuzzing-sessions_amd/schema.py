"""Columnar layout of the four session tables the RQ scripts read.

The reference keeps these tables in PostgreSQL (schema inferred in SURVEY.md section 8(c);
columns named in ``program/__module/queries1.py:18-55,120-129,289-295`` and
``program/preparation/3_get_coverage_data.py:132``).  The engine keeps them as typed
columns, one numpy array per column on the host and one device buffer per column in HBM:

* every timestamp is an ``int64`` count of microseconds since 1970-01-01 of the *naive*
  value stored in the database (RQ4 treats naive values as UTC, ``rq4a_bug.py:137``);
  a NULL timestamp is ``TS_NULL`` (sorts last, fails every ``<``/``>`` predicate);
* ``project`` is dictionary-encoded in byte order, so id order == ``ORDER BY project``
  under a C/BINARY collation;
* ``build_type``, ``result`` and ``status`` are small integer codes into per-table
  vocabularies whose first entries are the literals the SQL filters compare against;
* ``modules`` / ``revisions`` are ids into string pools; ``rev_canon`` is the id of the
  canonical token multiset ``sorted(s[1:-2].split(','))`` RQ3 compares
  (``rq3_diff_coverage_at_detection.py:280``);
* nullable integers carry a validity mask.
"""
from __future__ import annotations

import datetime as _dt
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

TS_NULL = np.iinfo(np.int64).max
US_PER_DAY = 86_400_000_000
EPOCH = _dt.datetime(1970, 1, 1)

# vocabularies: fixed leading entries, dataset-specific strings appended after them
BUILD_TYPES = ["Fuzzing", "Coverage"]
RESULTS = ["Finish", "Halfway", "HalfWay", "Error"]
STATUSES = ["Fixed", "Fixed (Verified)"]
BT_FUZZING, BT_COVERAGE = 0, 1
R_FINISH, R_HALFWAY_LOWER, R_HALFWAY_UPPER, R_ERROR = 0, 1, 2, 3
CODE_NULL = 255

LIMIT_DATE = "2025-01-08"          # queries1.py:3 (repeated inline in every script)
RQ3_LIMIT_DATE = "2025-01-09"      # rq3_diff_coverage_at_detection.py:262-263


def ts_from_str(s: str) -> int:
    """'YYYY-MM-DD[ HH:MM:SS[.ffffff]]' -> int64 microseconds (naive)."""
    if len(s) == 10:
        d = _dt.datetime.strptime(s, "%Y-%m-%d")
    elif "." in s:
        d = _dt.datetime.strptime(s, "%Y-%m-%d %H:%M:%S.%f")
    else:
        d = _dt.datetime.strptime(s, "%Y-%m-%d %H:%M:%S")
    return dt_to_us(d)


def dt_to_us(d: _dt.datetime) -> int:
    delta = d - EPOCH
    return (delta.days * 86400 + delta.seconds) * 1_000_000 + delta.microseconds


def us_to_dt(us: int) -> _dt.datetime:
    return EPOCH + _dt.timedelta(microseconds=int(us))


def day_floor(us):
    """Start of the calendar day (``x.date()``) in microseconds."""
    return (np.asarray(us, dtype=np.int64) // US_PER_DAY) * US_PER_DAY


LIMIT_US = ts_from_str(LIMIT_DATE)
RQ3_LIMIT_US = ts_from_str(RQ3_LIMIT_DATE)


@dataclass
class Tables:
    """Host-side columnar image of buildlog_data, total_coverage, issues, project_info
    plus the RQ4 corpus CSV (``data/processed_data/csv/project_corpus_analysis.csv``)."""

    projects: List[str]
    # buildlog_data
    b_project: np.ndarray            # uint32
    b_type: np.ndarray               # uint8 codes into build_types
    b_result: np.ndarray             # uint8 codes into results (CODE_NULL = NULL)
    b_time: np.ndarray               # int64 us (TS_NULL = NULL)
    b_modules: np.ndarray            # int32 ids into modules_pool (-1 = NULL)
    b_revisions: np.ndarray          # int32 ids into revisions_pool (-1 = NULL)
    b_name: np.ndarray               # object array of str (or None)
    modules_pool: List[Optional[str]]
    revisions_pool: List[Optional[str]]
    # total_coverage
    c_project: np.ndarray            # uint32
    c_date: np.ndarray               # int64 us
    c_coverage: np.ndarray           # float64 (0.0 where NULL)
    c_coverage_valid: np.ndarray     # bool
    c_covered: np.ndarray            # int64 (0 where NULL)
    c_covered_valid: np.ndarray      # bool
    c_total: np.ndarray              # int64 (0 where NULL)
    c_total_valid: np.ndarray        # bool
    # issues
    i_number: np.ndarray             # int64
    i_project: np.ndarray            # uint32
    i_rts: np.ndarray                # int64 us (TS_NULL = NULL)
    i_status: np.ndarray             # uint8 codes into statuses
    i_new_id: np.ndarray             # int64
    # project_info
    pi_project: np.ndarray           # uint32 ids of projects present in project_info
    pi_first_commit: np.ndarray      # int64 us
    # vocabularies
    build_types: List[str] = field(default_factory=lambda: list(BUILD_TYPES))
    results: List[str] = field(default_factory=lambda: list(RESULTS))
    statuses: List[str] = field(default_factory=lambda: list(STATUSES))
    # RQ4 corpus CSV, verbatim text (parsed by the RQ4 host code exactly as pandas does)
    corpus_csv: str = ""
    # derived encodings (group_key / rev_canon / corpus columns), computed once per table and
    # persisted by store.save_columnar; each entry is keyed by the identity of the inputs it was
    # derived from, so a table rebuilt around new arrays (a shard, a renamed copy) recomputes
    derived: dict = field(default_factory=dict, compare=False, repr=False)

    def cached(self, name, inputs, make):
        hit = self.derived.get(name)
        if hit is not None and len(hit[0]) == len(inputs) and all(a is b for a, b in zip(hit[0], inputs)):
            return hit[1]
        value = make()
        self.derived[name] = (tuple(inputs), value)  # holds the inputs: identity stays meaningful
        return value

    @property
    def n_rows(self) -> int:
        """Session rows = buildlog_data + total_coverage + issues."""
        return int(len(self.b_project) + len(self.c_project) + len(self.i_project))

    def rev_canon(self) -> np.ndarray:
        """Per-build id of ``sorted(rev[1:-2].split(','))`` (rq3:280); -1 for NULL."""
        return self.cached("rev_canon", (self.b_revisions, self.revisions_pool), self._rev_canon)

    def _rev_canon(self) -> np.ndarray:
        canon_of_pool = np.full(len(self.revisions_pool), -1, dtype=np.int32)
        seen = {}
        for k, s in enumerate(self.revisions_pool):
            if s is None:
                continue
            key = tuple(sorted(s[1:-2].split(",")))
            canon_of_pool[k] = seen.setdefault(key, len(seen))
        out = np.full(len(self.b_revisions), -1, dtype=np.int32)
        ok = self.b_revisions >= 0
        out[ok] = canon_of_pool[self.b_revisions[ok]]
        return out.astype(np.int32)

    def group_key(self) -> np.ndarray:
        """Per-build id of ``str(modules) + '_' + str(revisions)`` (rq2_coverage_and_added.py:129)."""
        return self.cached("group_key", (self.b_modules, self.b_revisions, self.modules_pool, self.revisions_pool),
                           self._group_key)

    def _group_key(self) -> np.ndarray:
        m = np.where(self.b_modules >= 0, self.b_modules, len(self.modules_pool)).astype(np.int64)
        r = np.where(self.b_revisions >= 0, self.b_revisions, len(self.revisions_pool)).astype(np.int64)
        # the key is the concatenated TEXT: str(None) == 'None', and 'a_b'+'_'+'c' == 'a'+'_'+'b_c'
        mp = list(self.modules_pool) + [None]
        rp = list(self.revisions_pool) + [None]
        pair = m * (len(rp) + 1) + r
        upair, inv = np.unique(pair, return_inverse=True)
        text_id = {}
        ids = np.empty(len(upair), dtype=np.int32)
        for k, pv in enumerate(upair.tolist()):
            s = str(mp[pv // (len(rp) + 1)]) + "_" + str(rp[pv % (len(rp) + 1)])
            ids[k] = text_id.setdefault(s, len(text_id))
        return ids[inv.reshape(-1)].astype(np.int32)
