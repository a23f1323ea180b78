"""Drop-in at the reference's own path: `python3 program/research_questions/rq3_diff_coverage_at_detection.py` from the
repository root, no arguments (run_all_analysis.sh), runs the MI355X engine's rq3_diff_coverage_at_detection
(tse_amd.rq.scripts) - same stdout, logs, CSVs and figures under ./data/result_data.  Tables:
$FZ_DATA, else ./data/columnar, else the dump ./data/database/backup_clean.sql (converted to
./data/columnar on first use).  The engine is found at $FZ_ENGINE_ROOT or two levels above this file."""
import os
import sys

_root = os.environ.get("FZ_ENGINE_ROOT") or os.path.dirname(os.path.dirname(os.path.dirname(os.path.realpath(__file__))))
if _root not in sys.path:
    sys.path.insert(0, _root)

from tse_amd.rq import scripts  # noqa: E402

if __name__ == "__main__":
    sys.exit(scripts.main_one("rq3_diff_coverage_at_detection"))
