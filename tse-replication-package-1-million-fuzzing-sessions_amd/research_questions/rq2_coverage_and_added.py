"""Drop-in for program/research_questions/rq2_coverage_and_added.py - main() at rq2_coverage_and_added.py:241-283 (analyze_coverage_change :73-238).

Same stdout, log records and output files under ./data/result_data; the analysis runs on the GPU
through libfz (tse_amd.rq.compute), the tables come from $FZ_DATA (tse_amd.rq.scripts.load_tables).
"""
import sys

from tse_amd.rq import scripts


def main():
    scripts.run("rq2_coverage_and_added")


if __name__ == "__main__":
    sys.exit(main())
