"""CPU ORACLE - TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker / CPU baseline - never as the product path.

``rq_oracle`` restates the reference's analysis (SQL + Python loops of
``program/research_questions/*.py`` and ``program/__module/queries1.py``) as numpy over the
columnar ``Tables``, calling numpy / scipy exactly where the reference calls them (numpy
2.2.6 / scipy 1.15.3 in this image; the reference's ``requirements.txt`` pins nothing).

Pinning: the oracle is checked against golden fixtures produced by running the UNMODIFIED
reference scripts on the same synthetic tables (``tests/golden/make_goldens.py``; recipe in
SURVEY.md Appendix A) and against the reference's own shipped outputs
(``data/result_data/**`` known-answer tests).
"""
