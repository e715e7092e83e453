"""Shared test setup.

* `gpu` marker: tests that need an MI355X (run on the GPU box with -m gpu).
* sys.path: the CPU oracle binding (oracle/pyoracle.py, test infrastructure)
  and the engine binding (fhe-sorting_amd/fhesort.py).
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, 'oracle'), os.path.join(REPO, 'fhe-sorting_amd'), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an AMD MI355X (gfx950) GPU')
    config.addinivalue_line('markers', 'slow: long-running CPU test')
