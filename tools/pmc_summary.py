#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value per kernel (per
dispatch), for the kernels matching a pattern.  Usage: pmc_summary.py <csv>... [--match rocfm]"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="rocfm|rocprim")
    a = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in a.csv:
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name", "")
                if not re.search(a.match, name):
                    continue
                short = re.sub(r"\(.*", "", name).replace("void ", "")[-70:]
                key = (r.get("Dispatch_Id"), r.get("Counter_Name"))
                acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        print(k)
        for c, vals in sorted(cs.items()):
            print(f"    {c:28s} {sum(vals) / len(vals):14.1f}   (n={len(vals)})")


if __name__ == "__main__":
    main()
