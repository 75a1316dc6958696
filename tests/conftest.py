"""pytest configuration: the `gpu` marker and import paths (repo root, package dir, oracle/)."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "duckdb-robust-predicate-transfer_amd")
for p in (REPO, PKG, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librpt_gpu.so on cuda:0)")


@pytest.fixture(scope="session")
def golden():
    import golden_util

    return golden_util.Golden()
