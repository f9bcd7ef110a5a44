"""Summarise rocprofv3 --pmc CSV output per kernel (sum over dispatches,
then per dispatch).  python tools/pmc_csv.py <dir containing *counter_collection.csv>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    for sub in sorted(os.listdir(root)):
        files = glob.glob(os.path.join(root, sub, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        agg = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        for f in files:
            for r in csv.DictReader(open(f)):
                k = r.get("Kernel_Name", "?")
                if "igemm" not in k and "conv" not in k and "gemm" not in k:
                    continue
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        for k, d in agg.items():
            n = max(1, len(disp[k]))
            print(f"[{sub}] {k[:90]}  ({n} dispatches)")
            for c in sorted(d):
                print(f"    {c:28s} {d[c] / n:14.4g}")


if __name__ == "__main__":
    main()
