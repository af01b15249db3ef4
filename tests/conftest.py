import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device; run with -m gpu")


class _LazyCases(dict):
    """Golden cases loaded on first access (the cfg3 B=128 case regenerates ~1 GB of replay)."""

    def __missing__(self, name):
        from tests.golden_utils import Case, CASE_NAMES
        assert name in CASE_NAMES, name
        self[name] = Case(name)
        return self[name]


@pytest.fixture(scope="session")
def golden_cases():
    return _LazyCases()
