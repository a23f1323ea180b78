"""CPU checks of the drop-in boundary: libfz.so loads and exports every symbol include/fz.h declares
(no compute call - there is no GPU here), and the ctypes struct layouts match the header."""
import ctypes as C
import os
import re

import pytest

import tse_amd
from tse_amd import engine as E

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "fz.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(fz_\w+)\s*\(", src, re.M)))


def test_header_declares_bound_symbols():
    decl = _declared()
    assert decl, "no declarations parsed"
    assert sorted(E.SIGNATURES) == decl


def test_library_exports_every_symbol():
    if not os.path.exists(tse_amd.LIB_PATH):
        pytest.skip("libfz.so not built (run __graft_entry__.build())")
    lib = E.load_library()
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.fz_abi_version() == 1


def test_struct_sizes():
    # fz_tables: 4 int64 sizes + 16 pointers + n_projects; fz_describe: 13 x 8 bytes
    assert C.sizeof(E.FzTables) == 8 * (1 + 1 + 6 + 1 + 6 + 1 + 4 + 1)
    assert C.sizeof(E.FzDescribe) == 8 * E.DESCRIBE_DOUBLES
    assert C.sizeof(E.FzStoreStats) == 8 * 6


def test_engine_refuses_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        E.Engine(0)
