#!/usr/bin/env python3
"""Kernel timeline from a rocprofv3 --kernel-trace CSV: the last N launches with
start (us, from the first listed), duration and the gap to the previous launch's end.

    python tools/kernel_timeline.py PATH/TO/run_kernel_trace.csv [--last 24]
"""
import argparse
import csv
import re
import statistics


def short(name):
    m = re.match(r"(?:void )?(?:\(anonymous namespace\)::)?([A-Za-z_0-9]+)", name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=24)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    sel = rows[-a.last:]
    t0 = sel[0][0]
    prev = None
    gaps = {}
    for s, e, n in sel:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} gap {gap:6.1f}  {n}")
        if prev is not None:
            gaps.setdefault(n, []).append(gap)
        prev = e
    durs = {}
    for s, e, n in rows:
        durs.setdefault(n, []).append((e - s) / 1e3)
    print("# per kernel over the whole trace: launches, median duration us, median gap before it us")
    for n, d in sorted(durs.items()):
        g = gaps.get(n)
        print(f"#  {n:24s} {len(d):6d} {statistics.median(d):9.1f} {statistics.median(g) if g else float('nan'):7.1f}")


if __name__ == "__main__":
    main()
