"""Print one line per bench JSON file in a directory: µs/step, M examples/s, planned-tail workgroups.
Usage: python tools/bench_table.py <dir>"""
import glob
import json
import os
import sys


def main():
    for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
        try:
            d = json.loads([ln for ln in open(f) if ln.startswith("{")][-1])
        except (IndexError, ValueError):
            print(f"{os.path.basename(f)[:-5]:<22} (no JSON line)")
            continue
        print(f"{os.path.basename(f)[:-5]:<22} {d['ms_per_step'] * 1000:7.1f} us {d['value'] / 1e6:7.2f} M  "
              f"nw={d.get('config', {}).get('emb_plan_workgroups')}")


if __name__ == "__main__":
    main()
