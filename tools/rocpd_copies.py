"""Summarise the memory copies of a rocprofv3 rocpd database (``--memory-copy-trace``): per copy
kind / direction, count, bytes, time and rate, plus whether any ran as a kernel (blit) — and, per
step-kernel name, the mean duration of its dispatches that overlapped an H2D copy vs those that did
not.  Usage: python tools/rocpd_copies.py <results.db> [--kernels deepfm_rows,step_tail]"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--kernels", default="deepfm_rows,step_tail")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    names = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
    print("tables/views:", ", ".join(sorted(n for n in names if "copy" in n.lower() or n in ("kernels",))))
    view = next((n for n in ("memory_copies", "memory_copy", "rocpd_memory_copy") if n in names), None)
    if view is None:
        print("no memory-copy table")
        return
    cols = [r[1] for r in con.execute(f"pragma table_info({view})")]
    print("columns:", ", ".join(cols))
    want = [c for c in ("name", "start", "end", "size", "src_agent_type", "dst_agent_type", "stream_id",
                        "queue_id", "src_agent_abs_index", "dst_agent_abs_index") if c in cols]
    rows = con.execute(f"select {', '.join(want)} from {view} order by start").fetchall()
    idx = {c: i for i, c in enumerate(want)}
    by = collections.defaultdict(lambda: [0, 0, 0.0])
    h2d = []
    for r in rows:
        key = (r[idx["name"]] if "name" in idx else "?",
               r[idx["src_agent_type"]] if "src_agent_type" in idx else "?",
               r[idx["dst_agent_type"]] if "dst_agent_type" in idx else "?")
        b = by[key]
        b[0] += 1
        b[1] += int(r[idx["size"]]) if "size" in idx and r[idx["size"]] is not None else 0
        dt = (r[idx["end"]] - r[idx["start"]]) / 1e3
        b[2] += dt
        if "CPU" in str(key[1]).upper() and "GPU" in str(key[2]).upper():
            h2d.append((r[idx["start"]], r[idx["end"]]))
    print(f"{'copy':<48}{'calls':>7}{'MB':>10}{'ms':>9}{'GB/s':>8}")
    for k, (n, by_, ms) in sorted(by.items(), key=lambda kv: -kv[1][2]):
        print(f"{str(k)[:48]:<48}{n:>7}{by_ / 1e6:>10.1f}{ms / 1e3:>9.2f}{(by_ / 1e9) / max(ms / 1e6, 1e-12):>8.1f}")
    krows = con.execute("select name, start, end from kernels order by start").fetchall()
    blit = [k for k in krows if "copyBuffer" in k[0] or "rocclr" in k[0]]
    print(f"blit (shader) copy kernels: {len(blit)}")
    h2d.sort()
    for kn in a.kernels.split(","):
        over, clear = [], []
        j = 0
        for n, s, e in krows:
            if kn not in n:
                continue
            while j < len(h2d) and h2d[j][1] < s:
                j += 1
            hit = j < len(h2d) and h2d[j][0] < e
            (over if hit else clear).append((e - s) / 1e3)
        if over or clear:
            f = lambda v: f"{sum(v) / len(v):.2f} us (n={len(v)})" if v else "—"  # noqa: E731
            print(f"{kn}: during an H2D copy {f(over)}; otherwise {f(clear)}")


if __name__ == "__main__":
    main()
