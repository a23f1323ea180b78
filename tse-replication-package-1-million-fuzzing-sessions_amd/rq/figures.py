"""The reference's figures (PDF), drawn off the critical path.

The analyses' numbers come from the GPU; the figures are host matplotlib, as in the reference, and
run in a side process after the tables and stdout are written (``scripts.run(..., figures=True)``).
Each ``spec_*`` function extracts what one script's figures show from its result object (small
host arrays, picklable); ``draw(spec, cwd)`` renders them to the reference's paths:

* rq1   ``rq1/rq1_detection_rate.pdf``                       (rq1_detection_rate.py:46-98)
* rq2   ``rq2/projects/{rho:.4f}_{project}.pdf`` per |rho| > 0.5, ``all_project_corr_hist.pdf``,
        ``session_coverage_boxplot.pdf``, ``average_median_lineplot.pdf``,
        ``session_coverage_distribution_trend.pdf``         (rq2_coverage_count.py:23-242, 325-480)
* rq3   ``rq3/coverage_diff_boxplot.pdf``, ``coverage_diff_histograms.pdf``, ``detected.pdf``,
        ``non_detected.pdf``                                 (rq3_diff_coverage_at_detection.py:70-198, 355-358)
* rq4a  ``rq4/bug/rq4_g1_g2_detection_trend.pdf``, ``rq4_gc_detection_trend.pdf`` (rq4a_bug.py:210-243, 417-510)
* rq4b  ``rq4/coverage/coverage_delta_timeseries_linear.pdf``, ``g2_g1_boxplot_comparison.pdf``
        (rq4b_coverage.py:1041-1118, 491-637)

PDF bytes are not a parity target (matplotlib embeds dates and versions); the figures show the same
series over the same axes.
"""
from __future__ import annotations

import os

import numpy as np

from ..schema import LIMIT_US, Tables


# ---------------------------------------------------------------------------------------- specs
def spec_rq1(r) -> dict:
    from .common import rq1_rates
    keys, rates, _, _ = rq1_rates(r.iter_total, r.iter_detected, r.min_project_threshold)
    return {"kind": "rq1", "rates": np.asarray(rates), "totals": np.array([int(r.iter_total[k - 1]) for k in keys])}


def _trend_index(t: Tables):
    """GET_TOTAL_COVERAGE_EACH_PROJECT (queries1.py:120-129) rows of every project, by (project,
    date): the row ids and each project's [start, end) in them (one sort for all projects)."""
    m = t.c_coverage_valid & (t.c_coverage != 0) & (t.c_date < LIMIT_US)
    idx = np.nonzero(m)[0]
    idx = idx[np.lexsort((t.c_date[idx], t.c_project[idx]))]
    proj = t.c_project[idx].astype(np.int64)
    ids = np.arange(len(t.projects))
    return idx, np.searchsorted(proj, ids, "left"), np.searchsorted(proj, ids, "right")


def spec_rq2_count(r, t: Tables) -> dict:
    processed = r.eligible[r.raw_n > 0]
    projects = []
    idx, start, end = _trend_index(t)
    for p, c in zip(processed.tolist(), r.corr.tolist()):
        if not np.isnan(c) and abs(c) > 0.5:                      # rq2_coverage_count.py:325-327
            rows = idx[start[p]:end[p]]
            projects.append((f"{c:.4f}_{t.projects[p]}", t.c_covered[rows].astype(np.float64),
                             t.c_total[rows].astype(np.float64)))
    offs = np.asarray(r.session_offsets)
    K = len(r.ge100)
    step = [i for i in range(0, K, 100)]                          # every 100th session (:396-398)
    box = [np.asarray(r.session_values[offs[i]:offs[i + 1]]) for i in step]
    return {"kind": "rq2", "projects": projects, "corr": np.asarray(r.corr[~np.isnan(r.corr)]),
            "box": box, "box_idx": step, "average": np.asarray(r.average_trend),
            "median": np.asarray(r.median_trend), "pct": np.asarray(r.dist_percentiles),
            "mean": np.asarray(r.dist_mean), "sizes": np.diff(offs)[:K]}


def spec_rq3(r) -> dict:
    return {"kind": "rq3", "det": np.asarray(r.det_pct), "non": np.asarray(r.non_pct)}


def spec_rq4a(r) -> dict:
    from .common import rq4a_rows
    rows = rq4a_rows(r.g1_total, r.g1_det, r.g2_total, r.g2_det)
    steps = sorted(r.g4_steps.items())
    return {"kind": "rq4a", "iters": np.array([x[0] for x in rows]), "g1": np.array([x[3] for x in rows]),
            "g2": np.array([x[6] for x in rows]), "steps": steps, "has_g4": bool(r.has_g4_transition)}


def spec_rq4b(r, t: Tables) -> dict:
    from .common import corpus_groups
    pre = [np.asarray(x) for x in r.pre_cov]
    post = [np.asarray(x) for x in r.post_cov]
    deltas = [pre[0] - pre[i] for i in range(6, 0, -1)] + [post[i] - pre[0] for i in range(7)] if r.n_delta_projects \
        else []
    # session boxplots of G2 vs G1 (every BOXPLOT_STEP = 100th session with >= 100 values in both groups)
    elig = np.nonzero(np.bincount(t.c_project[t.c_coverage_valid & (t.c_coverage > 0) & (t.c_date < LIMIT_US)]
                                  .astype(np.int64), minlength=len(t.projects)) >= 365)[0]
    groups, _ = corpus_groups(t, elig, add_missing_to_g1=False)
    m = t.c_coverage_valid & (t.c_coverage > 0) & (t.c_date < LIMIT_US)
    idx = np.nonzero(m)[0]
    idx = idx[np.lexsort((t.c_date[idx], t.c_project[idx]))]
    proj = t.c_project[idx].astype(np.int64)
    start = np.searchsorted(proj, np.arange(len(t.projects)), "left")
    end = np.searchsorted(proj, np.arange(len(t.projects)), "right")
    sessions = [i for i in range(0, r.last_valid_idx + 1, 100)] if r.last_valid_idx >= 0 else []

    def values(g, i):
        ps = [p for p in groups[g] if end[p] - start[p] > i]
        return t.c_coverage[idx[[start[p] + i for p in ps]]] if ps else np.zeros(0)
    box = [(i, values("group2", i), values("group1", i)) for i in sessions]
    return {"kind": "rq4b", "deltas": deltas, "box": box}


# ---------------------------------------------------------------------------------------- drawing
def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def _save(fig, path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    fig.savefig(path, format="pdf", bbox_inches="tight")


def draw(spec: dict, cwd: str) -> list:
    """Render one script's figures under cwd; returns the written paths."""
    plt = _plt()
    out = []
    kind = spec["kind"]
    base = os.path.join(cwd, "data", "result_data")
    if kind == "rq1" and len(spec["rates"]):
        fig, ax1 = plt.subplots(figsize=(5, 3))
        ax2 = ax1.twinx()
        ax1.set_zorder(ax2.get_zorder() + 1)
        ax1.patch.set_visible(False)
        x = np.arange(len(spec["rates"]))
        ax1.plot(x, spec["rates"], color="b", marker="o", markersize=1.0, linewidth=1)
        ax1.set_ylabel("Percentage of Projects Detecting Bugs")
        ax1.set_xlabel("Fuzzing Session")
        ax2.bar(x, spec["totals"], color="#88c778", alpha=0.6)
        ax2.set_ylabel("Number of Projects")
        out.append(os.path.join(base, "rq1", "rq1_detection_rate.pdf"))
        _save(fig, out[-1])
        plt.close(fig)
    elif kind in ("rq2", "rq2_projects"):
        d = os.path.join(base, "rq2")
        for name, cov, tot in spec["projects"]:
            fig, ax1 = plt.subplots(figsize=(5, 3))
            ax2 = ax1.twinx()
            ax1.set_zorder(ax2.get_zorder() + 1)
            ax1.patch.set_visible(False)
            x = np.arange(len(cov))
            pct = np.divide(cov, tot, out=np.zeros_like(cov), where=tot != 0) * 100
            ax2.fill_between(x, 0, tot, alpha=0.5, label="Total Lines")
            ax2.fill_between(x, 0, cov, alpha=0.9, label="Covered Lines")
            ax2.set_ylabel("Number of Lines")
            ax1.plot(x, pct, color="red", alpha=0.7, linewidth=1.3, label="Coverage (%)")
            ax1.set_ylim(0, 105)
            ax1.set_ylabel("Coverage (%)")
            ax1.set_xlabel("Coverage Measurement Count")
            out.append(os.path.join(d, "projects", name + ".pdf"))
            _save(fig, out[-1])
            plt.close(fig)
        if kind == "rq2_projects":
            return out
        fig = plt.figure(figsize=(5, 3))
        plt.hist(spec["corr"], bins=40, color="skyblue", edgecolor="black", alpha=0.8)
        plt.xlabel("Correlation")
        plt.ylabel("Frequency")
        out.append(os.path.join(d, "all_project_corr_hist.pdf"))
        _save(fig, out[-1])
        plt.close(fig)
        if spec["box"]:
            fig, ax1 = plt.subplots(figsize=(7.5, 4.5))
            ax2 = ax1.twinx()
            ax1.set_zorder(ax2.get_zorder() + 1)
            ax1.patch.set_visible(False)
            pos = np.arange(1, len(spec["box"]) + 1)
            ax2.bar(pos, [len(b) for b in spec["box"]], color="#88c778", alpha=0.6)
            ax2.set_ylabel("Number of Projects")
            ax1.boxplot(spec["box"], positions=pos, patch_artist=True)
            ax1.scatter(pos, [np.mean(b) for b in spec["box"]], color="#215F9A", marker="^", s=8, zorder=4)
            ax1.set_ylim(0, 100)
            ax1.set_ylabel("Coverage (%)")
            ax1.set_xlabel("Coverage Measurement Count")
            ax1.set_xticks(pos)
            ax1.set_xticklabels([str(i + 1) for i in spec["box_idx"]], rotation=45)
            out.append(os.path.join(d, "session_coverage_boxplot.pdf"))
            _save(fig, out[-1])
            plt.close(fig)
        fig = plt.figure(figsize=(6, 4))
        x = np.arange(len(spec["average"]))
        plt.plot(x, spec["average"], label="Average", marker="o", color="blue", markersize=1, linewidth=1)
        plt.plot(x, spec["median"], label="Median", marker="o", color="green", markersize=1, linewidth=1)
        plt.xlabel("Session Index")
        plt.ylabel("Coverage (%)")
        plt.legend()
        out.append(os.path.join(d, "average_median_lineplot.pdf"))
        _save(fig, out[-1])
        plt.close(fig)
        if len(spec["mean"]):
            fig, (ax_n, ax_c) = plt.subplots(2, 1, figsize=(10, 6), sharex=True,
                                             gridspec_kw={"height_ratios": [1, 3]})
            x = np.arange(len(spec["mean"]))
            ax_n.plot(x, spec["sizes"], linewidth=1.5)
            ax_n.set_ylabel("#Projects")
            ax_n.set_title("Coverage Percentage across Fuzzing Sessions")
            p5, p25, p50, p75, p95 = spec["pct"]
            ax_c.fill_between(x, p25, p75, alpha=0.35, label="Percentile 25-75%")
            ax_c.fill_between(x, p5, p95, alpha=0.28)
            ax_c.plot(x, p5, color="#6889df", linewidth=1.3, label="Percentile 5-95%")
            ax_c.plot(x, p95, color="#6889df", linewidth=1.3)
            ax_c.plot(x, p50, color="#2ca02c", linewidth=2, label="Median")
            ax_c.plot(x, spec["mean"], color="#ffb43b", linewidth=2, label="Mean")
            ax_c.set_ylim(0, 100)
            ax_c.set_ylabel("Line Coverage %")
            ax_c.set_xlabel("Coverage Measurement Count (Sessions)")
            ax_c.legend(loc="lower center", ncol=4, frameon=False)
            out.append(os.path.join(d, "session_coverage_distribution_trend.pdf"))
            _save(fig, out[-1])
            plt.close(fig)
    elif kind == "rq3":
        d = os.path.join(base, "rq3")
        det, non = spec["det"], spec["non"]
        fig = plt.figure(figsize=(4, 3))
        plt.boxplot([det, non], patch_artist=True, tick_labels=["Detected", "Not Detected"], showfliers=True)
        plt.ylabel("Coverage Difference (%)")
        plt.yscale("symlog", linthresh=0.01)
        out.append(os.path.join(d, "coverage_diff_boxplot.pdf"))
        _save(fig, out[-1])
        plt.close(fig)
        fig, (a1, a2) = plt.subplots(1, 2, figsize=(8, 3), sharey=True, sharex=True)
        bins = np.linspace(-5, 5, 51)
        a1.hist(det, bins=bins, color="skyblue", edgecolor="black")
        a1.set_title("Detected")
        a2.hist(non, bins=bins, color="salmon", edgecolor="black")
        a2.set_title("Not Detected")
        for a in (a1, a2):
            a.set_xlabel("Coverage Difference (%)")
        a1.set_ylabel("Frequency")
        out.append(os.path.join(d, "coverage_diff_histograms.pdf"))
        _save(fig, out[-1])
        plt.close(fig)
        for name, v in (("detected.pdf", det), ("non_detected.pdf", non)):
            fig = plt.figure(figsize=(2.0, 2.5))
            if len(v):
                plt.boxplot(v, patch_artist=True, widths=0.5, showfliers=True)
                plt.scatter(1, np.mean(v), marker="^", s=15, zorder=3)
            plt.yscale("symlog", linthresh=0.01)
            plt.ylabel("Coverage Difference")
            plt.xticks([])
            out.append(os.path.join(d, name))
            _save(fig, out[-1])
            plt.close(fig)
    elif kind == "rq4a":
        d = os.path.join(base, "rq4", "bug")
        if len(spec["iters"]):
            fig = plt.figure(figsize=(5, 3))
            plt.plot(spec["iters"], spec["g1"], linewidth=1, marker="o", markersize=1, label="Group A (No Corpus)")
            plt.plot(spec["iters"], spec["g2"], linewidth=1, marker="o", markersize=1, alpha=0.7,
                     label="Group B (Initial Corpus)")
            plt.xlabel("Fuzzing Session")
            plt.ylabel("Percentage of Projects Detecting Bugs")
            plt.legend()
            out.append(os.path.join(d, "rq4_g1_g2_detection_trend.pdf"))
            _save(fig, out[-1])
            plt.close(fig)
        if spec["has_g4"]:
            labels, rates = [], []
            for step, (n, det) in spec["steps"]:
                if n:
                    labels.append(f"{'Pre' if step < 0 else 'Post'}-{abs(step)}")
                    rates.append(det / n * 100)
            fig = plt.figure(figsize=(5, 3))
            plt.plot(range(len(rates)), rates, marker="o")
            plt.xticks(range(len(rates)), labels, rotation=45)
            plt.ylabel("Detection Rate (%)")
            out.append(os.path.join(d, "rq4_gc_detection_trend.pdf"))
            _save(fig, out[-1])
            plt.close(fig)
    elif kind == "rq4b":
        d = os.path.join(base, "rq4", "coverage")
        if spec["deltas"]:
            fig = plt.figure(figsize=(5, 3))
            plt.boxplot(spec["deltas"], positions=range(len(spec["deltas"])), showfliers=False)
            plt.xticks(range(len(spec["deltas"])), [f"Pre-{k}" for k in range(6, 0, -1)]
                       + [f"Post-{k}" for k in range(7)], rotation=45)
            plt.ylim(-50, 50)
            plt.ylabel("Coverage Delta (Relative to Pre-1)")
            plt.xlabel("Time Step (t)")
            plt.axhline(0, ls="--", color="black", linewidth=1.0)
            out.append(os.path.join(d, "coverage_delta_timeseries_linear.pdf"))
            _save(fig, out[-1])
            plt.close(fig)
        if spec["box"]:
            fig, ax = plt.subplots(figsize=(5, 3))
            pos = np.arange(len(spec["box"]))
            ax.boxplot([b[2] for b in spec["box"]], positions=pos - 0.2, widths=0.35, showfliers=False)
            ax.boxplot([b[1] for b in spec["box"]], positions=pos + 0.2, widths=0.35, showfliers=False)
            ax.set_xticks(pos)
            ax.set_xticklabels([str(b[0] + 1) for b in spec["box"]], rotation=45)
            ax.set_ylabel("Coverage (%)")
            ax.set_xlabel("Fuzzing Session")
            out.append(os.path.join(d, "g2_g1_boxplot_comparison.pdf"))
            _save(fig, out[-1])
            plt.close(fig)
    return out


def spec(name: str, r, t: Tables) -> dict:
    """The figure data of one drop-in script's result object."""
    if name == "rq1_detection_rate":
        return spec_rq1(r)
    if name == "rq2_coverage_count":
        return spec_rq2_count(r, t)
    if name == "rq3_diff_coverage_at_detection":
        return spec_rq3(r)
    if name == "rq4a_bug":
        return spec_rq4a(r)
    if name == "rq4b_coverage":
        return spec_rq4b(r, t)
    return {"kind": "none"}     # rq2_coverage_and_added draws nothing


def split(specs, workers: int):
    """The specs cut into `workers` lists of about equal drawing work: the per-project trend
    figures of RQ2 (hundreds of PDFs, rq2_coverage_count.py:325-327) are dealt round-robin."""
    parts = [[] for _ in range(max(1, workers))]
    for sp in specs:
        if sp.get("kind") == "rq2" and len(parts) > 1 and len(sp["projects"]) > 1:
            pr = sp["projects"]
            parts[0].append(dict(sp, projects=pr[0::len(parts)]))
            for w in range(1, len(parts)):
                if pr[w::len(parts)]:
                    parts[w].append({"kind": "rq2_projects", "projects": pr[w::len(parts)]})
        else:
            parts[0].append(sp)
    return [p for p in parts if p]


def figure_workers() -> int:
    return max(1, min(8, int(os.environ.get("FZ_FIGURE_WORKERS", os.cpu_count() or 1))))


def draw_in_side_process(specs, cwd: str, workers: int = 1):
    """Start child interpreters that draw the figures (the GPU process never runs matplotlib);
    returns the Process list (join() them before exiting)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    procs = []
    for part in split(specs, workers):
        p = ctx.Process(target=_draw_all, args=(part, cwd), daemon=False)
        p.start()
        procs.append(p)
    return procs


def _draw_all(specs, cwd):
    for s in specs:
        draw(s, cwd)
