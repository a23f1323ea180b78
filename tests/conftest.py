"""pytest configuration: the ``gpu`` marker and shared fixtures.

CPU tests (``-m "not gpu"``) cover the oracle against the golden fixtures, the host logic
and the C-ABI symbol table; GPU tests (``-m gpu``) run the HIP path through ``libfz.so``.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import tse_amd  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through libfz.so)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def engine():
    """One libfz context on cuda:0 for the whole GPU test session (fails loudly without a GPU)."""
    from tse_amd import engine as E
    eng = E.Engine(0)
    yield eng
    eng.close()


@pytest.fixture(scope="session")
def engine_for(engine):
    """engine_for(case): the engine with that golden case's tables uploaded and the store built."""
    import goldens

    def get(case):
        t = goldens.tables(case)  # cached: the same object while the case's tables are loaded
        if engine.tables is None or engine.tables.host is not t:
            engine.upload(t)
            engine.build_store()
        return engine
    return get
