#!/usr/bin/env python3
"""Timeline of the last few training steps from a rocprofv3 kernel_trace.csv.

    python tools/trace_steps.py gpurun_out/prof/x_kernel_trace.csv [--anchor deepfm_rows] [--steps 3]

Steps are delimited by the anchor kernel (one launch per step); prints each kernel's start offset
from the step's anchor, duration, queue and a short name, plus per-step span and gap totals.
"""
import argparse
import csv
import re


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"<.*", "", n) if "rocprim" not in n else "rocprim::" + re.findall(r"detail::(\w+)", name)[0] \
        if re.findall(r"detail::(\w+)", name) else n
    n = n.replace("void ", "").replace("rocfm::", "").replace("(anonymous namespace)::", "")
    return n[-60:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--anchor", default="deepfm_rows")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]))
    rows.sort()
    anchors = [i for i, r in enumerate(rows) if a.anchor in r[3]]
    if len(anchors) < a.steps + 2:
        print("not enough steps")
        return
    sel = anchors[-(a.steps + 1):]
    for s0, s1 in zip(sel[:-1], sel[1:]):
        t0 = rows[s0][0]
        print(f"--- step: {(rows[s1][0] - t0) / 1e3:.1f} us between anchors")
        busy_end = t0
        for st, en, q, name in rows[s0:s1]:
            print(f"  {(st - t0) / 1e3:8.1f} +{(en - st) / 1e3:6.1f}  q{q:>2}  {short(name)}")


if __name__ == "__main__":
    main()
