"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE CSVs into HBM bytes per launch.

FETCH_SIZE and WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced streaming read (MI355X_MICROARCH.md, HBM section),
so traffic = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (per dispatch, averaged
over the dispatches of the same kernel).

usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON
"""
import csv
import json
import sys
from collections import defaultdict


def name_of(kernel: str) -> str:
    if "k_rs_bs<" in kernel:
        return "k_rs_bs(syndrome)" if kernel.split(">")[0].rstrip().endswith("true") else "k_rs_bs(encode)"
    if "k_rs_jitw" in kernel:  # rs_jit.h Wide<R, CS>
        return "k_rs_jit%s(decode)" % ("16" if "Wide<16" in kernel else "12" if "Wide<12" in kernel else "10")
    if "k_rs_jit" in kernel:
        return "k_rs_jit(encode)" if "true>" in kernel.split("(")[0] else "k_rs_jit(decode)"
    if "k_rs_tc" in kernel:  # the bench's only k_rs_tc launch is the one-matrix decode
        return "k_rs_tc(decode)"
    if "k_dot_generic" in kernel:
        return "k_dot_generic(solve)"
    if "k_rs_encode_lh" in kernel:
        return "k_rs_encode_lh"
    if "k_decode_prepare_syn" in kernel:
        return "k_decode_prepare_syn"
    if "k_decode_prepare" in kernel:
        return "k_decode_prepare"
    return kernel.split("(")[0]


def load(path, counter):
    acc = defaultdict(list)
    per_dispatch = defaultdict(float)
    kname = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        per_dispatch[r["Dispatch_Id"]] += float(r["Counter_Value"])
        kname[r["Dispatch_Id"]] = name_of(r["Kernel_Name"])
    for d, v in per_dispatch.items():
        acc[kname[d]].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    f = load(sys.argv[1], "FETCH_SIZE")
    w = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in set(f) | set(w):
        out[k] = 2 * f.get(k, 0.0) * 1024 + w.get(k, 0.0) * 1024
    out["_note"] = "bytes per launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH half-count)"
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
