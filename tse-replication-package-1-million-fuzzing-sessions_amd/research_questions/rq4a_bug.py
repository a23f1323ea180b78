"""Drop-in for program/research_questions/rq4a_bug.py - main() at rq4a_bug.py:653-884.

Same stdout, log records and output files under ./data/result_data; the analysis runs on the GPU
through libfz (tse_amd.rq.compute), the tables come from $FZ_DATA (tse_amd.rq.scripts.load_tables).
"""
import sys

from tse_amd.rq import scripts


def main():
    scripts.run("rq4a_bug")


if __name__ == "__main__":
    sys.exit(main())
