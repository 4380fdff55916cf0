#!/usr/bin/env python3
"""Per-basic-block instruction counts of one kernel in the gfx950 assembly (`make asm` writes
/tmp/dhcos_asm/dh_kernels-hip-amdgcn-amd-amdhsa-gfx950.s), with loops marked from their back
edges: the static half of a VALU budget (multiply each block by its trip count).

usage: python tools/isa_blocks.py KERNEL_SUBSTRING [--asm FILE] [--min 1]
"""
import argparse
import re

ASM = "/tmp/dhcos_asm/dh_kernels-hip-amdgcn-amd-amdhsa-gfx950.s"


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "br"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel")
    ap.add_argument("--asm", default=ASM)
    ap.add_argument("--min", type=int, default=1, help="hide blocks with fewer VALU")
    a = ap.parse_args()
    lines = open(a.asm).read().split("\n")
    start = next(i for i, l in enumerate(lines)
                 if l.endswith(":") is False and a.kernel in l and l.split(":")[0].startswith("_Z")
                 and not l.startswith("\t"))
    name = lines[start].split(":")[0]
    blocks, cur = [], {"label": "entry", "line": start, "n": {}, "ops": [], "targets": [],
                       "comment": ""}
    for i in range(start + 1, len(lines)):
        l = lines[i]
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):(.*)", l)
        if m:
            blocks.append(cur)
            cur = {"label": m.group(1), "line": i, "n": {}, "ops": [], "targets": [],
                   "comment": m.group(2).strip()}
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")):
            if s.startswith("; %bb") or "Loop" in s:
                cur["comment"] += " " + s
            continue
        op = s.split()[0]
        c = classify(op)
        if c:
            cur["n"][c] = cur["n"].get(c, 0) + 1
            cur["ops"].append(op)
        if c == "br":
            t = s.split()[-1]
            if t.startswith(".LBB"):
                cur["targets"].append(t)
    blocks.append(cur)
    idx = {b["label"]: k for k, b in enumerate(blocks)}
    loops = []
    for k, b in enumerate(blocks):
        for t in b["targets"]:
            if t in idx and idx[t] <= k:
                loops.append((idx[t], k))
    print(name)
    tot = {}
    for k, b in enumerate(blocks):
        for c, v in b["n"].items():
            tot[c] = tot.get(c, 0) + v
        depth = sum(1 for s, e in loops if s <= k <= e)
        if b["n"].get("valu", 0) < a.min and not any(s == k for s, e in loops):
            continue
        head = "".join(f" [loop {s}-{e}]" for s, e in loops if s == k)
        print(f"{k:4d} {b['label']:>12} line {b['line']:6d} depth {depth} "
              f"valu {b['n'].get('valu', 0):4d} salu {b['n'].get('salu', 0):3d} "
              f"lds {b['n'].get('lds', 0):3d} vmem {b['n'].get('vmem', 0):3d}{head} "
              f"{b['comment'][:60]}")
    print("total", tot)
    for s, e in loops:
        v = sum(blocks[k]["n"].get("valu", 0) for k in range(s, e + 1))
        print(f"loop {s}-{e}: {v} VALU over its blocks")


if __name__ == "__main__":
    main()
