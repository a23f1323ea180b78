"""The six reference analysis scripts re-expressed on the engine.

Each script is split in two halves so the numbers can be checked independently of the text:

* ``compute`` (``tse_amd.rq.compute``) runs the hot path on the GPU through ``libfz`` and
  returns a plain result object (``tse_amd.rq.results``);
* ``render`` (``tse_amd.rq.render``) turns a result object into exactly the stdout lines and
  output files the reference script writes.

The CPU oracle (``oracle/``) produces the same result objects, so a test can compare
GPU-vs-oracle numbers field by field and oracle-vs-golden text byte by byte.
"""
