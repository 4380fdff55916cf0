"""Summarise a rocprofv3 --kernel-trace CSV: per kernel, launches, mean duration and the mean
idle gap from the previous kernel's end to its start (same queue order), plus the busy fraction
of the traced window.  Usage: python tools/trace_gaps.py <..._kernel_trace.csv> [name-filter]"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = [r for r in rows if filt in r["Kernel_Name"]] if filt else rows
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    dur, gap, n = defaultdict(float), defaultdict(float), defaultdict(int)
    prev_end = None
    busy = 0
    for s, e, name in ev:
        key = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:70]
        n[key] += 1
        dur[key] += e - s
        busy += e - s
        if prev_end is not None:
            gap[key] += max(0, s - prev_end)
        prev_end = e
    for k in sorted(n, key=lambda k: -dur[k]):
        print(f"{k:70s} n {n[k]:6d}  dur {dur[k] / n[k] / 1e3:8.2f} us  gap-before {gap[k] / n[k] / 1e3:8.2f} us")
    if ev:
        span = ev[-1][1] - ev[0][0]
        print(f"window {span / 1e3:.1f} us, kernels busy {busy / span:.1%}")


if __name__ == "__main__":
    main()
