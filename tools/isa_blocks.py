"""Per-basic-block instruction mix of one kernel in a hipcc --save-temps .s file.

Usage: python tools/isa_blocks.py <file.s> <kernel-name-substring> [--min 40]
Prints each basic block with >= --min instructions: label, #instr, #VALU, #fp64 VALU, #SALU,
#LDS, #VMEM, backward-branch target (loops)."""
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 40
    lines = open(path).read().splitlines()
    start = None
    for i, ln in enumerate(lines):
        if re.match(r"^_Z\S*:", ln) and name in ln:
            start = i
            break
    if start is None:
        sys.exit("kernel not found")
    blocks, cur, label = [], [], lines[start].rstrip(":")
    order = {}
    for ln in lines[start + 1:]:
        if ln.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            blocks.append((label, cur))
            label, cur = m.group(1), []
            continue
        s = ln.strip()
        if not s or s.startswith((";", ".", "//")):
            continue
        cur.append(s)
    blocks.append((label, cur))
    for idx, (lb, _) in enumerate(blocks):
        order[lb] = idx
    tot = dict(n=0, valu=0, f64=0)
    for idx, (lb, ins) in enumerate(blocks):
        ops = [i.split()[0] for i in ins]
        valu = [o for o in ops if o.startswith("v_")]
        f64 = [o for o in valu if "f64" in o]
        salu = [o for o in ops if o.startswith("s_")]
        lds = [o for o in ops if o.startswith("ds_")]
        vmem = [o for o in ops if o.startswith(("global_", "buffer_", "flat_", "scratch_"))]
        back = ""
        for i in ins:
            m = re.match(r"s_(cbranch_\w+|branch)\s+(\.LBB\S+)", i)
            if m and order.get(m.group(2), 1 << 30) <= idx:
                back = f"loop->{m.group(2)}"
        tot["n"] += len(ops)
        tot["valu"] += len(valu)
        tot["f64"] += len(f64)
        if len(ops) >= mn or back:
            trans = [o for o in valu if o.startswith(("v_rcp", "v_rsq", "v_sqrt", "v_exp", "v_log", "v_sin", "v_cos", "v_frexp", "v_ldexp"))]
            print(f"{lb:22s} n={len(ops):5d} valu={len(valu):5d} f64={len(f64):5d} "
                  f"trans={len(trans):3d} salu={len(salu):4d} lds={len(lds):3d} vmem={len(vmem):3d} {back}")
    print("total", tot)


if __name__ == "__main__":
    main()
