"""Turn a round's rocprofv3 outputs (tools/gpu_profile.sh, merged into gpurun_out/prof/) into the
committed evidence under profiles/:

  profiles/<tag>_<config>_kernel_stats.csv   rocprofv3 --stats summary, verbatim
  profiles/<tag>_<config>_pmc.csv            per-kernel medians of every PMC counter collected
  profiles/pmc_traffic.json                  per config: HBM bytes per request (read by bench.py)
  profiles/<tag>_summary.md                  the same numbers as a table

HBM bytes follow MI355X_MICROARCH.md's rocprofv3 section: FETCH_SIZE and WRITE_SIZE come from
separate passes and are in KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide coalesced
read, so it is doubled.  A request is one cos_fused_kernel launch (latency-bound requests) or one
cos_table_kernel + one option-kernel launch (large requests): whichever the config spends its
time in.

usage: python tools/summarize_profiles.py --tag r01 [--src gpurun_out/prof]
"""
import argparse
import collections
import csv
import glob
import gzip
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("loss_partials_kernel", "cos_fused_kernel", "cos_table_kernel", "cos_option_small_kernel", "cos_option_kernel",
           "table_prologue_kernel", "cos_gen_kernel")


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def median(v):
    v = sorted(v)
    n = len(v)
    return v[n // 2] if n % 2 else 0.5 * (v[n // 2 - 1] + v[n // 2])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "prof"))
    ap.add_argument("--configs", default="c2,c3")
    args = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    tpath = os.path.join(prof, "pmc_traffic.json")
    traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
    md = [f"# Profile summary {args.tag}", "",
          "One request = cos_fused_kernel (every maturity group one tile: C1-C4; on grids of "
          ">= 8,192 blocks, C4, preceded by table_prologue_kernel), cos_gen_kernel (generator "
          "grids, C5: one fused small-tile launch per batch), or cos_table_kernel + the option "
          "kernel (--path split; cos_option_kernel for multi-tile groups, "
          "cos_option_small_kernel for large calls on <=16-option tiles). Durations: "
          "rocprofv3 --kernel-trace --stats average; counters: per-launch medians of separate "
          "--pmc passes.", ""]
    for c in args.configs.split(","):
        stats = os.path.join(args.src, f"{args.tag}_{c}_stats_kernel_stats.csv")
        if not os.path.exists(stats):
            print("missing", stats)
            continue
        shutil.copy(stats, os.path.join(prof, f"{args.tag}_{c}_kernel_stats.csv"))
        # per kernel family, the average of its dominant template instantiation (C4's 5-wave
        # fused build next to one 4-wave spot-check call), the total over all of them
        avg, total, top = {}, {}, {}
        for r in csv.DictReader(open(stats)):
            k = short(r["Name"])
            if k:
                tot = float(r["TotalDurationNs"])
                total[k] = total.get(k, 0.0) + tot
                if tot > top.get(k, -1.0):
                    top[k] = tot
                    avg[k] = float(r["AverageNs"])
        # the request's kernels: the fused kernel if the config spends its time there, else the
        # table kernel + whichever option-kernel variant dominates (the others only serve the
        # bench's small spot-check calls)
        if total.get("cos_gen_kernel", 0.0) >= max(total.values()):
            req_kernels = ("cos_gen_kernel",)             # generator grids: one fused launch
        elif total.get("cos_fused_kernel", 0.0) >= max(total.values()):
            # large fused grids run table_prologue_kernel ahead of the fused kernel
            pro = total.get("table_prologue_kernel", 0.0) >= 0.01 * total["cos_fused_kernel"]
            # multi-round loss requests sum their tiles' partials in a launch of their own
            fin = total.get("loss_partials_kernel", 0.0) >= 0.001 * total["cos_fused_kernel"]
            req_kernels = ((("table_prologue_kernel",) if pro else ()) + ("cos_fused_kernel",)
                           + (("loss_partials_kernel",) if fin else ()))
        else:
            opt = max((k for k in ("cos_option_small_kernel", "cos_option_kernel") if k in total),
                      key=lambda k: total[k])
            req_kernels = ("cos_table_kernel", opt)
        vals = collections.defaultdict(list)
        for f in glob.glob(os.path.join(args.src, f"{args.tag}_{c}_pmc*_counter_collection.csv*")):
            fh = gzip.open(f, "rt") if f.endswith(".gz") else open(f)
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                if k:
                    vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        med = {key: median(v) for key, v in vals.items()}
        with open(os.path.join(prof, f"{args.tag}_{c}_pmc.csv"), "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["kernel", "counter", "median_per_launch", "launches"])
            for (k, ctr), v in sorted(med.items()):
                w.writerow([k, ctr, v, len(vals[(k, ctr)])])
        per_kernel = {}
        for k in req_kernels:
            fetch = med.get((k, "FETCH_SIZE"))
            write = med.get((k, "WRITE_SIZE"))
            e = {"avg_ns": avg.get(k)}
            if fetch is not None and write is not None:
                e["fetch_bytes_x2"] = 2.0 * fetch * 1024.0
                e["fetch_bytes"] = e["fetch_bytes_x2"]
                e["write_bytes"] = write * 1024.0
            sized = [med.get((k, f"TCC_EA0_RDREQ_{b}B_sum")) for b in (32, 64, 128)]
            if all(x is not None for x in sized):
                # the L2's memory-side read requests by size: the fetched bytes exactly (the x2
                # of FETCH_SIZE is calibrated for 16-B-per-lane streaming reads only)
                e["fetch_bytes"] = 32.0 * sized[0] + 64.0 * sized[1] + 128.0 * sized[2]
                e["fetch_basis"] = "TCC_EA0_RDREQ_{32,64,128}B x size"
            for n in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_DRAM_sum", "TCC_EA0_RDREQ_DRAM_32B_sum",
                      "TCC_EA0_WRREQ_DRAM_sum", "TCC_EA0_WRREQ_64B_sum"):
                if (k, n) in med:
                    e[n] = med[(k, n)]
            f64 = [med.get((k, n)) for n in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                             "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")]
            if all(x is not None for x in f64):
                # executed fp64 flops: 64 lanes per wave instruction, fma = 2
                e["exec_fp64_flop"] = 64.0 * (2 * f64[0] + f64[1] + f64[2] + f64[3])
                e["valu_insts"] = med.get((k, "SQ_INSTS_VALU"))
            for n in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_BUSY_CYCLES", "SQ_WAVES"):
                if (k, n) in med:
                    e[n] = med[(k, n)]
            per_kernel[k] = e
        hbm = None
        if all("fetch_bytes" in per_kernel[k] for k in req_kernels):
            hbm = sum(per_kernel[k]["fetch_bytes"] + per_kernel[k]["write_bytes"]
                      for k in req_kernels)
        req_ns = sum(per_kernel[k]["avg_ns"] or 0.0 for k in req_kernels)
        traffic[c] = {"round": args.tag, "hbm_bytes_per_launch": hbm, "request_avg_ns": req_ns,
                      "kernels": per_kernel,
                      "note": "fetched bytes from the L2's read requests by size (32/64/128 B) "
                              "where collected, else FETCH_SIZE x2 (gfx950); + WRITE_SIZE; the "
                              "request's kernels"}
        md += [f"## {c}", "", "| kernel | avg us | fetch MB | write MB | exec fp64 GFLOP | "
               "exec fp64 TFLOP/s | wait_any/wave_cycles |", "|---|---|---|---|---|---|---|"]
        for k in req_kernels:
            e = per_kernel[k]
            t = (e["avg_ns"] or 0) * 1e-9
            ef = e.get("exec_fp64_flop")
            wa = (e["SQ_WAIT_ANY"] / e["SQ_WAVE_CYCLES"]) if e.get("SQ_WAVE_CYCLES") else None
            md.append(f"| {k} | {t * 1e6:.2f} | {e.get('fetch_bytes', 0) / 1e6:.3f} | "
                      f"{e.get('write_bytes', 0) / 1e6:.3f} | "
                      f"{(ef or 0) / 1e9:.3f} | {(ef or 0) / t / 1e12 if t else 0:.2f} | "
                      f"{'%.3f' % wa if wa is not None else '-'} |")
        md += ["", f"request: {req_ns / 1e3:.2f} us, HBM/fabric bytes {hbm / 1e6 if hbm else 0:.3f} MB",
               ""]
    json.dump(traffic, open(tpath, "w"), indent=1)
    open(os.path.join(prof, f"{args.tag}_summary.md"), "w").write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
