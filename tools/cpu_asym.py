"""CPU baseline asymmetry diagnostic (run on the GPU box's host): times the
AVX2 port data kernel of oracle/_ref over the encode's and the decode's
source sets (oracle/ref_driver.c ref_cpu_asym), then the bench's own
cpu_bench sample for comparison.  Test infrastructure, CPU only."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle_lib import Reference  # noqa: E402

L = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libisal_ref.so"))
t = (C.c_double * 5)()
L.ref_cpu_asym(64, 32, 1000000, 3, t)
names = ["encode_block_with", "decode_block_with", "decode data kernel again",
         "encode data kernel again", "decode data kernel, fresh outputs"]
res = {n: v for n, v in zip(names, t)}
t2 = (C.c_double * 5)()
L.ref_cpu_asym_thread(64, 32, 1000000, 3, t2)
res["on a pthread"] = {n: v for n, v in zip(names, t2)}
res["cpu_bench_1thread"] = Reference().cpu_bench(64, 32, 1000000, 1, 3, kernel=1)
L.ref_cpu_asym(64, 32, 1000000, 3, t)
res["main thread again"] = {n: v for n, v in zip(names, t)}
print(json.dumps(res, indent=1))
