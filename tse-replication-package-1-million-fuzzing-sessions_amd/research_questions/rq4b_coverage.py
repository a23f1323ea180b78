"""Drop-in for program/research_questions/rq4b_coverage.py - main() at rq4b_coverage.py:1209-1261.

Same stdout, log records and output files under ./data/result_data; the analysis runs on the GPU
through libfz (tse_amd.rq.compute), the tables come from $FZ_DATA (tse_amd.rq.scripts.load_tables).
"""
import sys

from tse_amd.rq import scripts


def main():
    scripts.run("rq4b_coverage")


if __name__ == "__main__":
    sys.exit(main())
