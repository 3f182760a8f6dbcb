"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs on CPU only (oracle vs reference goldens, host logic, C ABI
symbol table, gloo multi-process); `-m gpu` runs the parity tests through the
C ABI on an MI355X.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "storage-benchmarks_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")
