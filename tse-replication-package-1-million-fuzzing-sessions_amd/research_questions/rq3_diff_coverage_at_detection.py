"""Drop-in for program/research_questions/rq3_diff_coverage_at_detection.py - main() at rq3_diff_coverage_at_detection.py:202-360.

Same stdout, log records and output files under ./data/result_data; the analysis runs on the GPU
through libfz (tse_amd.rq.compute), the tables come from $FZ_DATA (tse_amd.rq.scripts.load_tables).
"""
import sys

from tse_amd.rq import scripts


def main():
    scripts.run("rq3_diff_coverage_at_detection")


if __name__ == "__main__":
    sys.exit(main())
