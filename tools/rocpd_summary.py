"""Summarise a rocprofv3 rocpd database (``--kernel-trace`` run): per-kernel count / total / mean
device time, and — over the last N dispatches of the busiest kernel's stream — the gaps between
consecutive kernels.  Usage: python tools/rocpd_summary.py <results.db> [--steps N]."""
import argparse
import collections
import re
import sqlite3


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"<.*", "", name)
    return name.split("::")[-1][:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=2000, help="dispatches (all streams) for the timeline stats")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    by = collections.defaultdict(list)
    for n, s, e, st in rows:
        by[short(n)].append((e - s) / 1e3)
    tot = sum(sum(v) for v in by.values())
    print(f"{'kernel':<50}{'calls':>8}{'total ms':>11}{'mean us':>10}{'share':>8}{'p50':>8}{'p90':>8}{'max':>8}")
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        q = sorted(v)
        print(f"{k:<50}{len(v):>8}{sum(v) / 1e3:>11.2f}{sum(v) / len(v):>10.2f}{100 * sum(v) / tot:>7.1f}%"
              f"{q[len(q) // 2]:>8.2f}{q[min(len(q) - 1, (9 * len(q)) // 10)]:>8.2f}{q[-1]:>8.2f}")
    # timeline of the last dispatches: busy time (union of kernel intervals) vs wall span
    tail = rows[-a.last:]
    if tail:
        iv = sorted((s, e) for _, s, e, _ in tail)
        busy, cs, ce = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        span = iv[-1][1] - iv[0][0]
        print(f"last {len(tail)} dispatches: span {span / 1e3:.1f} us, GPU busy (any kernel) {busy / 1e3:.1f} us "
              f"({100 * busy / span:.1f} %)")


if __name__ == "__main__":
    main()
