"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value per kernel
name over its dispatches (all passes under DIR merged).   python tools/pmc_summary.py DIR"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name") or row.get("Kernel-Name") or row.get("KernelName")
                acc[k[:120]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        if "sysml" not in k and "row_k" not in k:
            continue
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.4g}   (n={len(v)})")


if __name__ == "__main__":
    main()
