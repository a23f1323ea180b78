"""MI355X-native engine for the RQ1-RQ4 analytics of the 1M-fuzzing-sessions replication package.

Import as ``tse_amd`` (see the repo-root shim ``tse_amd.py``).

Layers
------
schema   columnar table layout (enums, dictionary-encoded strings, int64 microsecond timestamps)
synth    synthetic session tables with the shipped schema
store    columnar store on disk + sqlite/CSV ingest (the drop-in replacement for ``dbFile.DB``)
engine   ctypes binding of ``libfz.so`` (HIP kernels, C-ABI in ``include/fz.h``)
rq       the six analysis scripts re-expressed on the engine (same outputs as the reference)
"""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# FZ_LIB_PATH: an alternative build of the same library (tuning variants, scripts/build_variants.sh)
LIB_PATH = os.environ.get("FZ_LIB_PATH") or os.path.join(PKG_DIR, "lib", "libfz.so")

__all__ = ["PKG_DIR", "LIB_PATH"]
