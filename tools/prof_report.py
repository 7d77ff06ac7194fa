#!/usr/bin/env python3
"""Markdown report from a rocprofv3 --kernel-trace --stats --output-format csv run:
top kernels by total time and the per-step kernel timeline of the last steps.

    python tools/prof_report.py gpurun_out/prof/x  --title "..." [--anchor deepfm_rows] > profiles/x.md
"""
import argparse
import csv
import glob
import os
import re
import subprocess
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", name).replace("void ", "")
    if "rocprim" in n:
        m = re.findall(r"detail::(\w+)", name)
        return "rocprim::" + (m[1] if len(m) > 1 else m[0] if m else "kernel")
    n = re.sub(r"<(.{60,})>", "<…>", n)
    return n.replace("rocfm::", "").replace("(anonymous namespace)::", "")[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix", help="directory + output prefix, e.g. gpurun_out/prof15/single")
    ap.add_argument("--title", default="")
    ap.add_argument("--anchor", default="deepfm_rows")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    stats = a.prefix + "_kernel_stats.csv"
    trace = a.prefix + "_kernel_trace.csv"
    print(f"# {a.title or os.path.basename(a.prefix)}\n")
    print("Source: `rocprofv3 --kernel-trace --stats` on one MI355X. Kernel durations under the profiler "
          "include its per-dispatch overhead (≈1-2 µs); treat them as upper bounds.\n")
    if os.path.exists(trace):  # steady state: the last `window` steps of the trace only
        ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                    for r in csv.DictReader(open(trace)))
        anchors = [i for i, e in enumerate(ev) if a.anchor in e[2]]
        sel = ev[anchors[-min(len(anchors), 65)]:anchors[-1]] if len(anchors) > 2 else ev
        nsteps = max(1, min(len(anchors), 65) - 1)
        agg = {}
        for st, en, nm in sel:
            k = short(nm)
            c, t = agg.get(k, (0, 0))
            agg[k] = (c + 1, t + (en - st))
        tot = sum(t for _, t in agg.values())
        print(f"Steady state: the last {nsteps} steps of the timed region.\n")
        print("| kernel | calls/step | avg µs | share of kernel time |\n|---|---|---|---|")
        for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[: a.top]:
            print(f"| `{k}` | {c / nsteps:.2f} | {t / c / 1e3:.2f} | {t / tot * 100:.1f}% |")
        span = (sel[-1][1] - sel[0][0]) / 1e3 / nsteps if sel else 0
        print(f"\nWall time per step under the profiler: {span:.1f} µs.")
    else:
        rows = list(csv.DictReader(open(stats)))
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        print("| kernel | calls | avg µs | total % |\n|---|---|---|---|")
        for r in rows[: a.top]:
            print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                  f"{float(r['TotalDurationNs']) / tot * 100:.1f} |")
    if os.path.exists(trace):
        out = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "trace_steps.py"), trace,
                              "--anchor", a.anchor, "--steps", str(a.steps)], capture_output=True, text=True).stdout
        print("\n## Steady-state step timeline (µs from the step's first kernel; queue)\n\n```")
        print(out.rstrip())
        print("```")


if __name__ == "__main__":
    main()
