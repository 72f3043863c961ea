"""Per-kernel mean of the PMC counters in rocprofv3 --pmc pass directories (tools/ab_pmc.sh):
the closed-loop kernel and the dispatch-order / staging kernels around it, in KiB for FETCH_SIZE
and WRITE_SIZE.  Usage: python tools/pmc_kernels.py OUT.json PASS_DIR...   """
import collections
import csv
import glob
import json
import os
import sys

KERNELS = ("closed_loop", "unpermute", "invert", "order")


def summarise(path):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"].split("(")[0][:70]
        acc[(k, row["Counter_Name"])].append(float(row["Counter_Value"]))
    return {"%s|%s" % (k, c): dict(n=len(v), mean_kib=sum(v) / len(v))
            for (k, c), v in acc.items() if any(s in k for s in KERNELS)}


def main():
    out = {}
    for d in sys.argv[2:]:
        f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
        out[os.path.basename(d.rstrip("/"))] = summarise(f)
    with open(sys.argv[1], "w") as fh:
        json.dump(out, fh, indent=1)
    for name, v in out.items():
        for k, s in v.items():
            print("%-10s %-72s %9.1f" % (name, k, s["mean_kib"]))


if __name__ == "__main__":
    main()
