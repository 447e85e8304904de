"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs on a CPU-only host (oracle vs golden fixtures, host logic,
C-ABI loading, gloo multi-process sharding); `-m gpu` runs the HIP parity
tests on an MI355X.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "delta-node_amd"), ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — parity tests of the HIP path")
    config.addinivalue_line("markers", "slow: full-size (2^24) cases")
