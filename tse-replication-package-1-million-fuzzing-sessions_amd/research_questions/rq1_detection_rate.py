"""Drop-in for program/research_questions/rq1_detection_rate.py - main() at rq1_detection_rate.py:308-348 (collect_and_analyze_data :101-269).

Same stdout, log records and output files under ./data/result_data; the analysis runs on the GPU
through libfz (tse_amd.rq.compute), the tables come from $FZ_DATA (tse_amd.rq.scripts.load_tables).
"""
import sys

from tse_amd.rq import scripts


def main():
    scripts.run("rq1_detection_rate")


if __name__ == "__main__":
    sys.exit(main())
