#!/usr/bin/env python3
"""The bench's timed requests out of a rocprofv3 kernel trace (rocprofv3 --kernel-trace
--output-format csv of `python bench.py --no-cpu --no-calib --steps K --warmup W`).

bench.py issues, on one stream and in this order, for the configured request shape:
  1 correctness-check request (device path), max(5, min(K, 50)) host-API requests (the same
  kernels), the pre-warm's requests (round 5: the line's prewarm.requests), W warm-up requests,
  K timed requests, then HIP-event-timed requests and the side legs.
Every one of them is a request-shaped dispatch (the same kernel(s) and grid).  This script picks
the request-shaped dispatches (the most frequent (kernel, grid) of the COS kernels), takes the
K timed ones (after the requests above, --bench reads the pre-warm's count from the line; a
request of several kernels is counted once per its first kernel) and reports their mean / median device duration and the wall
span of the timed window per request -- the number comparable to bench.py's ms_per_step.

usage: python tools/request_trace.py TRACE.csv --steps K --warmup W [--bench LINE.json] [--out JSON]
"""
import argparse
import collections
import csv
import json
import re
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--bench", help="the run's JSON line (its prewarm.requests)")
    ap.add_argument("--grid", type=int, help="the request's grid (threads); default: the most "
                    "frequent COS dispatch shape")
    ap.add_argument("--out")
    a = ap.parse_args()
    n_pre = 0
    if a.bench:
        with open(a.bench) as fh:
            line = json.loads(fh.read().strip().splitlines()[-1])
        n_pre = int(line.get("prewarm", {}).get("requests", 0))
    rows = []
    with open(a.trace) as fh:
        for r in csv.DictReader(fh):
            if "cos_" not in r["Kernel_Name"] and "table_prologue" not in r["Kernel_Name"]:
                continue
            m = re.search(r"(\w+)(?:<[^>]*>)?\(", r["Kernel_Name"])
            name = m.group(1) if m else r["Kernel_Name"]
            rows.append((int(r["Dispatch_Id"]), name,
                         int(r["Grid_Size_X"]), int(r["Start_Timestamp"]),
                         int(r["End_Timestamp"])))
    rows.sort()
    if a.grid:
        rows = [r for r in rows if r[2] == a.grid]
    shape = collections.Counter((k, g) for _, k, g, _, _ in rows).most_common()
    # a request = one dispatch of each kernel of the dominant shape(s) with the same count
    top = shape[0][1]
    kinds = [s for s, c in shape if c == top]
    first = kinds[0]
    reqs, cur = [], None
    for d, k, g, s, e in rows:
        if (k, g) not in kinds:
            continue
        if (k, g) == first:
            cur = [s, e, e - s]
            reqs.append(cur)
        elif cur is not None:
            cur[1] = e
            cur[2] += e - s
    lo = 1 + max(5, min(a.steps, 50)) + n_pre + a.warmup
    hi = lo + a.steps
    timed = reqs[lo:hi]
    durs = [t[2] / 1e3 for t in timed]          # device time of the request's kernels, us
    span = (timed[-1][1] - timed[0][0]) / 1e3 / len(timed)
    out = {"kernels": [f"{k} grid {g}" for k, g in kinds], "requests_in_trace": len(reqs),
           "timed_requests": len(timed), "timed_positions": [lo, hi],
           "device_us_mean": statistics.mean(durs), "device_us_median": statistics.median(durs),
           "device_us_min": min(durs), "device_us_max": max(durs),
           "wall_span_us_per_request": span,
           "all_requests_device_us_mean": statistics.mean(t[2] / 1e3 for t in reqs)}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
