"""Average rocprofv3 PMC counters per kernel over the pass directories of
tools/pmc_sq.sh.  usage: python3 tools/pmc_summary.py gpurun_out/sq_TAG"""
import csv
import glob
import sys
from collections import defaultdict


def short(k: str) -> str:
    if "k_rs_jitw" in k:  # rs_jit.h Wide<R, CS>
        return "k_rs_jit%s(decode)" % ("16" if "Wide<16" in k else "12" if "Wide<12" in k else "10")
    if "k_rs_jit" in k:  # <NW, true>: the shared-program encode
        return "k_rs_jit(encode)" if "true>" in k.split("(")[0] else "k_rs_jit(decode)"
    for key in ("k_rs_tc", "k_rs_jit", "k_rs_bs", "k_dot_generic",
                "k_decode_prepare_syn", "k_fill_synth"):
        if key in k:
            return key
    return k.split("(")[0][:40]


def main():
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(sys.argv[1] + "/pass*/run_counter_collection.csv"):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        for (d, c), v in per.items():
            acc[names[d]][c].append(v)
    for k, cs in sorted(acc.items()):
        print(k)
        for c, vs in sorted(cs.items()):
            print(f"   {c:28s} {sum(vs) / len(vs):16.4g}")


if __name__ == "__main__":
    main()
