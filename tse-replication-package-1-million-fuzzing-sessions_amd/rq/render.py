"""Text rendering: result object -> the exact stdout / log lines / CSV bytes of the reference.

Every ``print`` and ``logger`` call below mirrors one in the reference script (cited per
function); CSV files are written with ``csv.writer`` (``\\r\\n`` line ends, ``str()`` of
each cell) like the reference.  A ``Rendered`` holds:

* ``stdout``  - what the reference prints;
* ``log``     - (level, message) records the reference sends to ``logging`` (stderr);
* ``files``   - {path relative to the run directory: bytes}.
"""
from __future__ import annotations

import csv
import io
import os
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import numpy as np
import pandas as pd

from ..schema import CODE_NULL, Tables, us_to_dt
from . import common, writer
from .results import (Describe, RQ1Result, RQ2AddResult, RQ2CountResult, RQ3Result, RQ4aResult,
                      RQ4bResult)

VENN_WARNING = ("Optional package 'matplotlib-venn' not found — Venn diagram will be skipped. "
                "Install with: pip install matplotlib-venn")


@dataclass
class Rendered:
    stdout: List[str] = field(default_factory=list)
    log: List[Tuple[str, str]] = field(default_factory=list)
    files: Dict[str, bytes] = field(default_factory=dict)
    figures: List[Tuple[str, object]] = field(default_factory=list)   # (path, callable) drawn on demand
    preamble_stderr: List[str] = field(default_factory=list)          # raw stderr before logging config

    def p(self, *args, sep=" "):
        self.stdout.append(sep.join(str(a) for a in args))

    def info(self, msg):
        self.log.append(("INFO", msg))

    def warning(self, msg):
        self.log.append(("WARNING", msg))

    def text(self) -> str:
        return "\n".join(self.stdout) + ("\n" if self.stdout else "")


def csv_bytes(rows, header=None) -> bytes:
    buf = io.StringIO(newline="")
    w = csv.writer(buf)
    if header is not None:
        w.writerow(header)
    w.writerows(rows)
    return buf.getvalue().encode("utf-8")


def _dt(us) -> str:
    return str(us_to_dt(us))


def _result_str(t: Tables, code):
    return None if code == CODE_NULL else t.results[code]


# ------------------------------------------------------------------------------------- RQ1
def rq1_late_lines(d: Describe) -> List[str]:
    """rq1_detection_rate.py:262-268: the late-stage block (first line starts with a newline)."""
    if d.min_nonzero is None:
        raise ValueError("min() arg is an empty sequence")   # the reference raises here (:264)
    return ["\nAnalysis of detection rates from iteration 26 onwards (for paper replication):",
            f"  - Min/Max: {d.min:.2f}% / {d.max:.2f}%",
            f"value min and than 0 {d.min_nonzero}",
            f"  - IQR (25th-75th percentile): {d.q1:.2f}% - {d.q3:.2f}%",
            f"  - Median: {d.median:.2f}%",
            f"  - Mean: {d.mean:.2f}%",
            f"  - Zero count: {d.n_zero/d.count*100:.2f}%({d.n_zero}/{d.count})"]


def rq1(r: RQ1Result, t: Tables) -> Rendered:
    """rq1_detection_rate.py:127-268 (collect_and_analyze_data) and :308-348 (main)."""
    o = Rendered()
    o.p(f"Found {r.n_issues_lim:,} issues from {r.n_issues_lim_projects:,} projects before 2025-01-08. (in study design)")
    o.p(f"Found {r.n_fixed_lim:,} fixed issues from {r.n_fixed_lim_projects:,} projects before 2025-01-08. (in study design)")
    o.p(f"Found {len(r.eligible):,} projects with at least 365 coverage reports (corresponds to 878 projects in study design).")
    o.p(f"Found {r.n_without_matching:,} issues without matching build.")
    o.p(f"Fetched {r.n_target:,} fixed issues from {r.n_target_projects:,} target projects.")
    o.p("\n[Phase 1/3] Counting the number of projects per fuzzing iteration...")
    o.p(f"{len(r.eligible):,} projects have {r.total_fuzz_builds:,} successful fuzzing builds. (in abstract)")
    n = len(r.matched_issue)
    o.p(f"\n[Phase 2/3] Mapping {n:,} vulnerability issues to fuzzing iterations...")
    o.p(f"(These are from {r.n_matched_projects:,} unique projects, corresponding to {n:,} issues from 808 projects in the paper).")
    o.p(f"linked {n:,}({n / r.n_target*100:.2f}%) issues to buildlog data. {n}/{r.n_target}")
    keys, rates, first_down, late = common.rq1_rates(r.iter_total, r.iter_detected, r.min_project_threshold)
    o.p("\n[Phase 3/3] Filtering and finalizing data...")
    o.p(f"Removing {len(r.iter_total) - len(keys):,} iterations with fewer than {r.min_project_threshold:,} projects.")
    o.p(f"Retained {len(keys):,} iterations for the final analysis (corresponds to 2,263rd session in the paper).")
    o.p("Aggregating final data for plotting...")
    for i, rate in enumerate(rates[:first_down]):
        o.p(f"{i+1}: {rate:.4f}%")
    if late:
        for line in rq1_late_lines(r.late):
            o.p(line)
    out_dir = "data/result_data/rq1"
    raw_path = os.path.join(out_dir, "rq1_raw_issues_for_analysis.csv")
    stats_path = os.path.join(out_dir, "rq1_detection_rate_stats.csv")
    if n == 0:
        o.p("No issue data to save.")
    else:
        rows = []
        for i, b in zip(r.matched_issue.tolist(), r.matched_build.tolist()):
            rows.append([int(t.i_number[i]), t.projects[t.i_project[i]], _dt(t.i_rts[i]), _dt(t.b_time[b]),
                         t.build_types[t.b_type[b]], _result_str(t, t.b_result[b]), t.b_name[b],
                         _pool(t.modules_pool, t.b_modules[b]), _pool(t.revisions_pool, t.b_revisions[b])])
        o.files[raw_path] = csv_bytes(rows, [f"issue_{i}" for i in range(9)])
        o.p(f"Saved raw issue data to: {raw_path}")
    o.files[stats_path] = csv_bytes(
        [[k, int(r.iter_total[k - 1]), int(r.iter_detected[k - 1])] for k in keys],
        ["Iteration", "Total_Projects", "Detected_Projects_Count"])
    o.p(f"Saved aggregated statistics to: {stats_path}")
    if not keys:
        o.p("No data available to create the graph.")
    else:
        pdf = os.path.join(out_dir, "rq1_detection_rate.pdf")
        o.figures.append((pdf, ("rq1", keys, rates, [int(r.iter_total[k - 1]) for k in keys])))
        o.p(f"Saved detection rate graph to: {pdf}")
    return o


def _pool(pool, k):
    return None if k < 0 else pool[k]


# ------------------------------------------------------------------------------- RQ2 count
def rq2_count(r: RQ2CountResult, t: Tables) -> Rendered:
    """rq2_coverage_count.py:244-483."""
    o = Rendered()
    out_dir = "data/result_data/rq2"
    o.p("--- Main process started ---")
    o.p(f"\n--- Starting to process {len(r.eligible)} projects ---")
    processed = r.raw_n > 0
    corr = r.corr
    for p, c in zip(r.eligible[processed].tolist(), corr.tolist()):
        if not np.isnan(c) and abs(c) > 0.5:
            o.figures.append((os.path.join(out_dir, "projects", f"{c:.4f}_{t.projects[p]}.pdf"), ("rq2_project", p)))
    o.p("\n--- Project processing finished ---\n")
    o.p("\n--- Analysis of Project Coverage Normality (Shapiro-Wilk) ---")
    tested = int(np.sum(r.n_trend >= 3))
    normal = int(np.sum((r.n_trend >= 3) & (r.sw_p > 0.05)))
    if tested > 0:
        o.p(f"Projects tested for normality (N >= 3 sessions): {tested}")
        o.p(f"Projects whose coverage trend follows normal distribution (p > 0.05): {normal}")
        o.p(f"Percentage of normally distributed projects: {(normal / tested) * 100:.2f}%")
    else:
        o.p("No projects had sufficient data (N >= 3) for normality testing.")
    csv_path = os.path.join(out_dir, "coverage_by_session_index.csv")
    o.p(f"Saving coverage data per session index to: {csv_path}")
    offs = r.session_offsets
    nrows = len(offs) - 1
    if writer.lib() is not None:  # the same bytes from the native writer (rq/writer.py)
        o.files[csv_path] = writer.float_rows(r.session_values, offs)
    else:
        vals = r.session_values.tolist()
        o.files[csv_path] = csv_bytes([vals[offs[i]:offs[i + 1]] for i in range(nrows)])
    o.p(f"Successfully saved. Total rows (max sessions): {nrows}")
    o.p("\n--- Analysis of All Project Correlations ---")
    valid = corr[~np.isnan(corr)]
    o.p(f"Total projects processed: {len(corr)}")
    o.p(f"Number of projects with valid correlation: {len(valid)}")
    o.p(f"Average correlation: {r.corr_mean:.4f}, Median correlation: {r.corr_median:.4f}")
    o.p(f"Correlation histogram saved to: {os.path.join(out_dir, 'all_project_corr_hist.pdf')}")
    o.p("\n--- Generating Boxplot of Coverage vs. Session Count ---")
    o.p(f"Number of sessions with >= 100 projects: {len(r.ge100)}")
    o.p(f"Boxplot saved to: {os.path.join(out_dir, 'session_coverage_boxplot.pdf')}")
    o.p("\n--- Correlation of Average/Median Coverage over Time ---")
    if len(r.median_trend) > 1:
        s, pv = r.spearman_median
        o.p("Spearman correlation (Session Index vs. Median):",
            f"SignificanceResult(statistic={np.float64(s)!r}, pvalue={np.float64(pv)!r})")
    else:
        o.p("Not enough data points to calculate correlation of coverage trends.")
    o.p("\n--- Normality Test for Median Trend (Shapiro-Wilk) ---")
    if len(r.median_trend) >= 3:
        o.p(f"Shapiro-Wilk test for 'median_trend' (N={len(r.median_trend)}): p-value = {r.shapiro_median_p:.4f}")
        if r.shapiro_median_p > 0.05:
            o.p("-> The distribution of median coverage values (median_trend) CAN be considered normal.")
        else:
            o.p("-> The distribution of median coverage values (median_trend) is NOT normal.")
    else:
        o.p(f"Not enough median values (N={len(r.median_trend)}, required >= 3) to run Shapiro-Wilk test.")
    o.p("Generating average/median line plot...")
    o.p(f"Line plot saved to: {os.path.join(out_dir, 'average_median_lineplot.pdf')}")
    o.p("\n--- Generating Coverage Distribution Trend Plot ---")
    if len(r.ge100) == 0:
        o.p("Warning: No session data provided. Skipping distribution trend plot.")
    else:
        o.p(f"Generating coverage distribution trend plot... (Data points: {len(r.ge100)} sessions)")
        o.p("Calculating percentiles for distribution plot...")
        o.p(f"Coverage distribution trend plot saved to: {os.path.join(out_dir, 'session_coverage_distribution_trend.pdf')}")
    o.p("\n--- Main process finished ---")
    return o


# --------------------------------------------------------------------------------- RQ2 add
def rq2_add(r: RQ2AddResult, t: Tables) -> Rendered:
    """rq2_coverage_and_added.py:73-283 (writes into data/result_data/rq3/)."""
    o = Rendered()
    out_dir = "data/result_data/rq3"
    o.p("--- Main process started for RQ3 ---")
    o.p("--- RQ3 Coverage Change Analysis Started ---")
    if len(r.projects) == 0:
        o.p("Warning: No projects found satisfying the criteria (coverage >= 365 sessions). Exiting.")
        o.p("\n--- Main process finished for RQ3 ---")
        return o
    o.p(f"\n--- Starting to process {len(r.projects)} projects ---")
    header = ['project', 'timecreated_i', 'modules_i', 'revisions_i', 'timecreated_i+1', 'modules_i+1',
              'revisions_i+1', 'covered_line_i', 'total_line_i', 'covered_line_i+1', 'total_line_i+1',
              'diff_total_line', 'diff_coverage']

    def cell(c, col, p):
        if c < 0:
            return np.nan
        if col == "covered":
            valid, v, isf = t.c_covered_valid[c], t.c_covered[c], r.covered_is_float[p]
        else:
            valid, v, isf = t.c_total_valid[c], t.c_total[c], r.total_is_float[p]
        if not valid:
            return np.nan
        return float(v) if isf else int(v)

    if writer.lib() is not None:  # every row formatted once, natively (rq/writer.py)
        body, row_end = writer.change_rows(r, t)
        hb = csv_bytes([], header)
        rp = np.asarray(r.row_project, dtype=np.int64)
        if len(rp):
            starts = np.concatenate([[0], row_end[:-1]])
            first = np.concatenate([[True], rp[1:] != rp[:-1]])  # runs of one project
            run_at = np.nonzero(first)[0]
            run_end = np.concatenate([run_at[1:], [len(rp)]])
            pieces = {}
            for a, b in zip(run_at.tolist(), run_end.tolist()):
                pieces.setdefault(int(rp[a]), []).append(body[int(starts[a]):int(row_end[b - 1])])
            for p, parts in pieces.items():
                o.files[os.path.join(out_dir, "change_analysis", f"{t.projects[p]}.csv")] = hb + b"".join(parts)
        o.p("\n--- Project processing finished ---\n")
        if len(rp):
            path = os.path.join(out_dir, "all_coverage_change_analysis.csv")
            o.files[path] = hb + body
            o.p(f"All project change analysis saved to: {path}")
        o.p("\n--- Main process finished for RQ3 ---")
        return o
    all_rows = []
    per_project = {}
    for k in range(len(r.row_project)):
        p = int(r.row_project[k])
        e, s, f = int(r.row_end_build[k]), int(r.row_start_build[k]), int(r.row_first_build[k])
        ci, ci1 = int(r.row_cov_i[k]), int(r.row_cov_i1[k])
        dtot = r.diff_total[k]
        if np.isnan(dtot):
            dtot_c = np.nan
        else:
            dtot_c = float(dtot) if r.total_is_float[p] else int(dtot)
        row = [t.projects[p], _dt(t.b_time[e]), _pool(t.modules_pool, t.b_modules[f]),
               _pool(t.revisions_pool, t.b_revisions[f]), _dt(t.b_time[s]), _pool(t.modules_pool, t.b_modules[s]),
               _pool(t.revisions_pool, t.b_revisions[s]), cell(ci, "covered", p), cell(ci, "total", p),
               cell(ci1, "covered", p), cell(ci1, "total", p), dtot_c, float(r.diff_coverage[k])]
        all_rows.append(row)
        per_project.setdefault(p, []).append(row)
    for p, rows in per_project.items():
        o.files[os.path.join(out_dir, "change_analysis", f"{t.projects[p]}.csv")] = csv_bytes(rows, header)
    o.p("\n--- Project processing finished ---\n")
    if all_rows:
        path = os.path.join(out_dir, "all_coverage_change_analysis.csv")
        o.files[path] = csv_bytes(all_rows, header)
        o.p(f"All project change analysis saved to: {path}")
    o.p("\n--- Main process finished for RQ3 ---")
    return o


# ------------------------------------------------------------------------------------- RQ3
def _summary(o: Rendered, d: Describe, name: str):
    """rq3_diff_coverage_at_detection.py:25-66."""
    o.p(f"\n--- Summary Statistics for '{name}' Group ---")
    if d is None or d.count == 0:
        o.p("No data available.")
        return
    pos = d.n_pos / d.count * 100
    zero = d.n_zero / d.count * 100
    neg = d.n_neg / d.count * 100
    o.p("+--------------------------+----------------------+")
    o.p("| Metric                   | Value                |")
    o.p("+--------------------------+----------------------+")
    o.p(f"| Count                    | {d.count:<20} |")
    o.p(f"| Positive Change Rate (%) | {f'{pos:.2f}':<20} |")
    o.p(f"| Zero Change Rate (%)     | {f'{zero:.2f}':<20} |")
    o.p(f"| Negative Change Rate (%) | {f'{neg:.2f}':<20} |")
    o.p(f"| Mean                     | {f'{d.mean:.4f}':<20} |")
    o.p(f"| Median                   | {f'{d.median:.4f}':<20} |")
    o.p(f"| Std. Deviation           | {f'{d.std:.4f}':<20} |")
    o.p(f"| Min                      | {f'{d.min:.4f}':<20} |")
    o.p(f"| Q1                       | {f'{d.q1:.4f}':<20} |")
    o.p(f"| Q3                       | {f'{d.q3:.4f}':<20} |")
    o.p(f"| Max                      | {f'{d.max:.4f}':<20} |")
    o.p("+--------------------------+----------------------+")


def rq3(r: RQ3Result, t: Tables) -> Rendered:
    """rq3_diff_coverage_at_detection.py:202-360."""
    o = Rendered()
    out_dir = "data/result_data/rq3"
    o.p("--- RQ3 Analysis Started ---")
    o.p(f"Fetched {r.n_all_issues} fixed issues from target projects.")
    o.p(f"\nFound {len(r.det_pct)} instances of coverage change on bug detection.")
    det_path = os.path.join(out_dir, "detected_coverage_changes.csv")
    non_path = os.path.join(out_dir, "non_detected_coverage_changes.csv")
    hdr = ['CoverageChangePercent', 'CoveredLinesChange', 'TotalLinesChange']
    o.files[det_path] = csv_bytes(zip(r.det_pct.tolist(), r.det_cov.tolist(), r.det_tot.tolist()), hdr)
    o.p(f"Saved detected changes data to {det_path}")
    o.files[non_path] = csv_bytes(zip(r.non_pct.tolist(), r.non_cov.tolist(), r.non_tot.tolist()), hdr)
    o.p(f"Saved non-detected changes data to {non_path}")
    _summary(o, r.desc_detected, "Detected")
    _summary(o, r.desc_non, "Not Detected")
    _summary(o, r.desc_det_total, "Detected Total")
    sig = np.array([15, 10, 5, 2.5, 1])
    for name, ad in (("Detected", r.anderson_det), ("Not Detected", r.anderson_non)):
        if ad is None:
            raise ValueError("anderson: empty input")        # the reference raises on empty data
        o.p(name)
        o.p("Test statistic (A²):", np.float64(ad[0]))
        o.p("Critical values:", np.asarray(ad[1]))
        o.p("Significance levels (%):", sig)
    o.p(f"Levene's test statistic: {r.levene[0]:.4f}")
    o.p(f"P-value: {r.levene[1]:.4f}")
    o.p(f"Brunner-Munzel W statistic: {r.brunnermunzel[0]:.4f}")
    o.p(f"P-value: {r.brunnermunzel[1]:.4f}")
    o.p("--- Generating comparison plots ---")
    o.p(f"Box plot saved to {os.path.join(out_dir, 'coverage_diff_boxplot.pdf')}")
    o.p(f"Histograms saved to {os.path.join(out_dir, 'coverage_diff_histograms.pdf')}")
    o.p("\n--- RQ3 Analysis Finished ---")
    return o


# ------------------------------------------------------------------------------------ RQ4a
def _gname(g):
    return {'group1': 'Group A (No Corpus)', 'group2': 'Group B (Initial Corpus)',
            'group3': 'Group D (1-5 Day Corpus)', 'group4': 'Group C (>5 Day Corpus)'}[g]


_TREND_HDR = ['Iteration', 'G1_Total_Projects', 'G1_Detected_Count', 'G1_Detection_Rate_pct',
              'G2_Total_Projects', 'G2_Detected_Count', 'G2_Detection_Rate_pct']


def rq4a_trend_lines(rows, after) -> List[str]:
    """rq4a_bug.py:698-747: superiority count, first iteration below 5 %, median / IQR after it,
    from the kept trend rows and the finishing statistics (``after[g] = (median, iqr)`` or None)."""
    out = []
    df = pd.DataFrame(rows, columns=_TREND_HDR)
    sup = int(np.sum(df['G2_Detection_Rate_pct'] > df['G1_Detection_Rate_pct']))
    tot = len(df)
    out.append(f"Count of Group B exceeding Group A within valid data range: {sup}/{tot} "
               f"({(sup / tot) * 100 if tot > 0 else 0:.2f}%)")
    g1r = df['G1_Detection_Rate_pct'].tolist()
    g2r = df['G2_Detection_Rate_pct'].tolist()

    def first5(rates):
        for idx, rate in enumerate(rates):
            if rate < 5:
                return idx
        return len(rates)
    f1, f2 = first5(g1r), first5(g2r)
    for name, f, rates in (("Group A", f1, g1r), ("Group B", f2, g2r)):
        if f < len(rates):
            out.append(f"{name}: {df.iloc[f]['Iteration']}th iteration fell below 5% (value: {rates[f]:.2f}%)")
        else:
            out.append(f"{name}: No iteration fell below 5%")
    for name, key in (("Group A", "g1"), ("Group B", "g2")):
        a = after[key]
        if a is not None:
            out.append(f"{name}: median {a[0]:.2f}, IQR {a[1]:.2f}")
            out.append(f"{name}: Last valid data count {df.iloc[-1]['Iteration']}th")
        else:
            out.append(f"{name}: No data below 5%")
    return out


def rq4a_intro_lines(n_pos, intro_stats) -> List[str]:
    """rq4a_bug.py:281-285 (the N > 0 introduction iterations' summary)."""
    mean, med, mn, mxx = intro_stats
    return [f"[RESULT] Introduction Iteration (N={n_pos}):", f"  - Mean: {mean:.2f}", f"  - Median: {med:.1f}",
            f"  - Min: {mn}", f"  - Max: {mxx}"]


def rq4a(r: RQ4aResult, t: Tables, cwd: str = "<WORK>") -> Rendered:
    """rq4a_bug.py:653-882."""
    o = Rendered()
    o.preamble_stderr.append(VENN_WARNING)
    out_dir = os.path.join(cwd, "data/result_data/rq4/bug")
    g = r.groups
    o.info("--- Starting RQ4 Bug Detection Trend Analysis ---")
    o.info("Graph save format: pdf")
    o.info(f"Projects categorized: G1={len(g['group1'])}, G2={len(g['group2'])}, G3={len(g['group3'])}, G4={len(g['group4'])}")
    o.info("Processing G1 and G2 projects for detection trend...")
    o.info("Processing G4 projects for pre/post analysis (Fixed N filtering)...")
    # calculate_and_save_stats (:156-207)
    g1_keys = [i + 1 for i in range(len(r.g1_total)) if r.g1_total[i] > 0 or r.g1_det[i] > 0]
    g2_keys = [i + 1 for i in range(len(r.g2_total)) if r.g2_total[i] > 0 or r.g2_det[i] > 0]
    mx = max(max(g1_keys, default=0), max(g2_keys, default=0))
    o.info(f"Max iteration found in data: {mx}")
    rows = common.rq4a_rows(r.g1_total, r.g1_det, r.g2_total, r.g2_det)
    o.info(f"Filtering iterations with fewer than 100 projects in either group. Retained {len(rows)} iterations.")
    o.info("\n--- G1/G2 Detection Trend Statistics ---")
    o.info(f"| {'Iter':<4} | {'G1 Total':<8} | {'G1 Rate':<7} | {'G2 Total':<8} | {'G2 Rate':<7} |")
    o.info(f"|{'-'*6}|{'-'*10}|{'-'*9}|{'-'*10}|{'-'*9}|")
    for row in rows:
        if row[0] <= 100:
            o.info(f"| {row[0]:<4} | {row[1]:<8} | {row[3]:>6.2f}% | {row[4]:<8} | {row[6]:>6.2f}% |")
    o.files["data/result_data/rq4/bug/rq4_g1_g2_detection_trend.csv"] = csv_bytes(rows, _TREND_HDR)
    o.info(f"Saved G1/G2 trend statistics to: {os.path.join(out_dir, 'rq4_g1_g2_detection_trend.csv')}")
    o.p(f"Groups used: {_gname('group1')} ({len(g['group1'])} projects), {_gname('group2')} ({len(g['group2'])} projects)")
    for line in rq4a_trend_lines(rows, r.after):
        o.p(line)
    tot = len(rows)
    mv = int(rows[-1][0]) if tot else 0
    o.p(f"\n[Graph Limit Info] Max iteration where both groups maintained >= 100 projects: {mv}")
    o.p("Data around end:")
    if mv > 0:
        o.p(f"{mv}: Group A {int(r.g1_total[mv - 1])}, Group B {int(r.g2_total[mv - 1])}")
    nx = mv + 1
    g1n = nx in g1_keys
    g2n = nx in g2_keys
    if g1n or g2n:
        a = int(r.g1_total[nx - 1]) if g1n else 0
        b = int(r.g2_total[nx - 1]) if g2n else 0
        o.p(f"{nx}: Group A {a}, Group B {b} (Outside filter)")
    else:
        o.p(f"(No data exists after iteration {mv})")
    if tot == 0:
        o.warning("No data available to create the trend graph.")
    else:
        o.info(f"Saved detection rate trend graph to: {os.path.join(out_dir, 'rq4_g1_g2_detection_trend.pdf')}")
    # analyze_g4_corpus_introduction_iteration (:246-299)
    o.info("\n--- Analyzing Group C Corpus Introduction Iteration ---")
    intro = sorted(r.intro, key=lambda x: (x[1], t.projects[x[0]]))
    dfi = pd.DataFrame([(t.projects[p], k) for p, k in intro], columns=['Project', 'Introduction_Iteration'])
    o.info(f"[RESULT] Total Group C Projects analyzed: {len(dfi)}")
    if r.intro_stats is not None:
        for line in rq4a_intro_lines(int((dfi['Introduction_Iteration'] > 0).sum()), r.intro_stats):
            o.info(line)
    else:
        o.info("[RESULT] No projects found with corpus introduction after the first fuzzing session.")
    o.files["data/result_data/rq4/bug/rq4_gc_introduction_iteration.csv"] = dfi.to_csv(index=False).encode()
    o.info(f"Saved Group C introduction iteration data to: {os.path.join(out_dir, 'rq4_gc_introduction_iteration.csv')}")
    o.info("\n[RESULT] Top 5 Projects (Earliest Corpus Introduction):")
    o.info(dfi.head(5).to_string(index=False))
    o.info("\n[RESULT] Bottom 5 Projects (Latest Corpus Introduction):")
    o.info(dfi.tail(5).to_string(index=False))
    # analyze_g4_trend (:417-510)
    N = 7
    pre_rate, post_rate = r.g4_overall
    if not r.has_g4_transition:
        o.warning("Skipping G4 Trend Analysis: No data available.")
        pre_rate = post_rate = 0
    else:
        o.info("\n--- Group C (Introduced Corpus) Pre-N/Post-N Trend Analysis (Fixed n) ---")
        o.info(f"| {'Step':<7} | {'n (Total)':<9} | {'DetCnt':<6} | {'Rate':<6} |")
        o.info(f"|{'-'*9}|{'-'*11}|{'-'*8}|{'-'*8}|")
        for step in sorted(r.g4_steps):
            n_total, det = r.g4_steps[step]
            if n_total == 0:
                continue
            rate = (det / n_total) * 100
            label = f"{'Pre' if step < 0 else 'Post'}-{abs(step)}"
            o.info(f"| {label:<7} | {n_total:<9} | {det:<6} | {rate:>5.2f}% |")
        o.info(f"Saved Group C trend graph to: {os.path.join(out_dir, 'rq4_gc_detection_trend.pdf')}")
    # analyze_and_report_g4_delta (:634-650)
    o.info("\n--- Group C Corpus Introduction Effect Analysis ---")
    o.info(f"Number of Projects: {r.n_g4_analyzed}")
    o.info(f"Average Pre-Introduction Detection Rate:  {pre_rate:.2f}%")
    o.info(f"Average Post-Introduction Detection Rate: {post_rate:.2f}%")
    delta = post_rate - pre_rate
    o.info(f"Effect (Post - Pre): {delta:+.2f} points")
    if pre_rate > 0:
        o.info(f"Relative Improvement: {(delta / pre_rate) * 100:+.2f}%")
    else:
        o.info("Relative Improvement: Undefined (Pre-rate is 0%)")
    # report_g4_pre_post_transition (:806-882)
    if r.has_g4_transition:
        both, pre_only, post_only, neither = r.g4_transition
        o.p("\n=== Group C Pre/Post Detection Transition ===")
        o.p(f"Total Projects: {sum(r.g4_transition)}")
        o.p(f" (i)-(iii) Detected in Pre AND Detected in Post: {both}")
        o.p(f" (i)-(iv)  Detected in Pre AND NOT Detected in Post: {pre_only}")
        o.p(f" (ii)-(iii) NOT Detected in Pre AND Detected in Post: {post_only}")
        o.p(f" (ii)-(iv)  NOT Detected in Pre AND NOT Detected in Post: {neither}")
        o.p(f" Sum check: {both + pre_only + post_only + neither}")
        o.p("=============================================\n")
        o.warning("Optional package 'matplotlib-venn' not found — skipping Venn diagram. "
                  "Install with: pip install matplotlib-venn")
    o.p(f"Valid project count for Group C: {r.n_g4_analyzed}")
    o.info("\n--- RQ4 Bug Detection Trend Analysis Finished ---")
    return o


# ------------------------------------------------------------------------------------ RQ4b
def rq4b(r: RQ4bResult, t: Tables, n_eligible: int, cwd: str = "<WORK>") -> Rendered:
    """rq4b_coverage.py:1209-1261."""
    o = Rendered()
    out_dir = os.path.join(cwd, "data/result_data/rq4/coverage")
    o.info(f"Using Current Working Directory: {cwd}")
    o.info(f"Added to sys.path: {os.path.join(cwd, 'program/__module')}")
    o.info("Connecting to DB to fetch eligible projects (RQ1 criteria)...")
    o.info(f"Found {n_eligible} eligible projects in DB.")
    o.info(f"Loading corpus analysis data from '{os.path.join(cwd, 'data/processed_data/csv/project_corpus_analysis.csv')}'...")
    g1, g2, g3, g4 = r.group_counts
    o.p("\n=== Number of Projects by Group ===")
    o.p(f"Group 1 (No Corpus): {g1} projects")
    o.p(f"Group 2 (Same Time): {g2} projects")
    o.p(f"Group 3 (< 7 day): {g3} projects")
    o.p(f"Group 4 (>= 7 day): {g4} projects")
    o.p(f"Total: {g1 + g2 + g3 + g4} projects\n")
    # analyze_g2_g1_trends (:910-1015)
    o.p("\n=== Analysis 3: G2 vs G1 Coverage Trend Analysis ===")
    last = r.last_valid_idx
    if last != -1:
        o.info(f"Filtering analysis up to session {last+1} (Limit: BOTH G1 and G2 >= 100).")
        o.info(f"At limit ({last+1}): G1 Count={int(r.c1[last])}, G2 Count={int(r.c2[last])}")
        if last + 1 < len(r.c1):
            o.info(f"Next ({last+2}): G1 Count={int(r.c1[last+1])}, G2 Count={int(r.c2[last+1])}")
    else:
        o.warning("No sessions met the condition (Either G1 or G2 >= 100). No summary reported.")
    # summarize_p_value_trends_and_stats (:799-908)
    o.info("Summarizing trends and stats...")
    pv = r.p_bm[:last + 1].tolist()
    if len(pv) == 0:
        o.warning("No valid data to summarize.")
    else:
        valid_p = [p for p in pv if not np.isnan(p)]
        sig = sum(1 for p in valid_p if p < 0.05)
        o.p("\n=== Trend Analysis Summary (Trend Summary) ===")
        o.p(f"Target Valid Period: 1 ~ {len(pv)} Sessions")
        if valid_p:
            o.p(f"Brunner-Munzel Test Significant Difference (p<0.05) Rate: {sig}/{len(valid_p)} ({sig/len(valid_p)*100:.2f}%)")
            first = next(((i + 1, p) for i, p in enumerate(pv) if not np.isnan(p) and p < 0.05), None)
            if first is not None:
                o.p(f"First significant difference detected at: {first[0]}th session (p={first[1]:.4e})")
            else:
                o.p("No significant difference detected.")
        else:
            o.p("Brunner-Munzel Test: No valid calculation results")
        n, wins, _, _ = common.rq4b_compare(r.g2_q[:last + 1].tolist(), r.g1_q[:last + 1].tolist())
        if n > 0:
            o.p(f"Group B > Group A Ratio (N={n}):")
            o.p(f"  - Q1               : {wins[0]}/{n} ({wins[0]/n*100:.2f}%)")
            o.p(f"  - Median           : {wins[1]}/{n} ({wins[1]/n*100:.2f}%)")
            o.p(f"  - Q3               : {wins[2]}/{n} ({wins[2]/n*100:.2f}%)")
            o.p(f"\nSpearman Rank Correlation with Coverage Measurement Count (N={n}):")
            labels = ["Q1", "Median", "Q3"]
            for k, (c, p) in enumerate(r.spearman6):
                if k == 0:
                    o.p(" [Group A (No Corpus)]")
                if k == 3:
                    o.p(" [Group B (Initial Corpus)]")
                o.p(f"  - {labels[k % 3]:<15} : corr={c:.4f}, p-value={p:.4e}")
        else:
            o.p("Stats Comparison: No valid data")
        o.p("============================================\n")
    # get_coverage_deltas (:725-797)
    o.p("\n=== Analysis 2: Pre/Post Corpus Introduction Difference Analysis (Group C: Strict Filter Applied) ===")
    o.p(f"Number of projects meeting conditions and analyzed: {r.n_delta_projects}")
    # analyze_g2_vs_g1_initial_coverage (:248-313)
    o.p("\n=== Analysis 1: G2 vs G1 Initial Coverage Comparison ===")
    o.p("Groups used: Group 2 (G2) vs Group 1 (G1)")
    o.p(f"Number of Group 2 projects: {r.n_g2}")
    o.p(f"Number of Group 1 projects: {r.n_g1}\n")
    if len(r.init_g2) > 0 and len(r.init_g1) > 0:
        o.info(f"[RESULT] Mann-Whitney U (G2 vs G1): p-value={r.mwu_p:.4f}")
        o.info(f"[RESULT] Cliff's Delta: {r.cliff:.4f}")
        o.info(f"[RESULT] Brunner-Munzel (G2 vs G1): p-value={r.bm[1]:.4f}, BM-statistic={r.bm[0]:.4f}")
        o.info(f"[RESULT] Levene's Test (G2 vs G1): p-value={r.levene[1]:.4f}, statistic={r.levene[0]:.4f}")
        st = {'n_g2': len(r.init_g2), 'n_g1': len(r.init_g1), 'mannwhitney_p_two_sided': float(r.mwu_p),
              'cliffs_delta': float(r.cliff), 'brunner_stat': float(r.bm[0]), 'brunner_p': float(r.bm[1]),
              'levene_stat': float(r.levene[0]), 'levene_p': float(r.levene[1])}
        o.info(f"Initial coverage stats: {st}")
    # plot_coverage_deltas (:1041-1118)
    if r.n_delta_projects > 0:
        o.p("\n--- Coverage Median for Each Step (Group C) ---")
        for i in reversed(range(7)):
            lab = f"Pre-{i+1}"
            o.p(f" {lab:<7}: {r.pre_median[i]:.2f} (N={len(r.pre_cov[i])})")
        for i in range(7):
            lab = f"Post-{i+1}"
            o.p(f" {lab:<7}: {r.post_median[i]:.2f} (N={len(r.post_cov[i])})")
        o.p("----------------------------------\n")
    # plot_g2_g1_comparative_boxplot (:491-637)
    o.info("Generating G2 vs G1 Comparative Boxplot...")
    c1_0 = int(r.extra.get("c1_0", r.c1[0] if len(r.c1) else 0))
    c2_0 = int(r.extra.get("c2_0", r.c2[0] if len(r.c2) else 0))
    if c1_0 < 100 or c2_0 < 100:
        o.warning("No sufficient data for boxplot.")
    else:
        o.info(f"Saved comparative boxplot to {os.path.join(out_dir, 'g2_g1_boxplot_comparison.pdf')}")
    o.info("--- Analysis Finished ---")
    return o
