"""Run bench.py against another build of librsgpu.so (same-box A/B of two
library builds; tool, not product):
    python3 tools/ab_lib.py LIB.so [bench.py arguments...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "storage-benchmarks_amd"))
import rsgpu  # noqa: E402

rsgpu.LIB_PATH = os.path.abspath(sys.argv[1])
import bench  # noqa: E402

sys.exit(bench.main(sys.argv[2:]))
