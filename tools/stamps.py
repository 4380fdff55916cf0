"""Phase breakdown of the option kernel from in-kernel s_memtime stamps (diagnostic build).

Usage:  make -C option-pricing-ffn-lbfgs_amd/csrc stamps
        python tools/stamps.py [--config c2] [--mode loss|price]
Stamps per block of cos_option_kernel: [0] start, [1] table + option data staged,
[2] options priced (incl. clamp path), [3] loss hand-off done; of the cos_table_kernel block with
the same index: [4] start, [5] truncation range + CF constants ready, [6] CF loop done, [7] end.
s_memtime is per XCD, so only
differences inside one block are meaningful; read shares, not absolute lengths.
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DHCOS_LIB"] = os.environ.get("STAMPS_LIB") or os.path.join(
    ROOT, "option-pricing-ffn-lbfgs_amd", "dhcos", "libdhcos_stamps.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "option-pricing-ffn-lbfgs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import bench  # noqa: E402
from dhcos.calibrator import DoubleHestonJumpCalibrator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--mode", default="loss")
    ap.add_argument("--path", type=int, default=0, help="0 auto, 1 split, 2 fused")
    ap.add_argument("--dump", default="", help="save the raw [blocks, 8] stamps (.npy)")
    ap.add_argument("--dev", action="store_true",
                    help="params / outputs in device memory (loss_dev), as the bench and the "
                         "device L-BFGS driver run; default: the host API (zero-copy params)")
    ap.add_argument("--timeline", action="store_true",
                    help="fused kernel: the blocks' residency (slot 23, s_memrealtime, 100 MHz) "
                         "as resident-block counts over the launch")
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    opts, S0, r = bench.make_surface(cfg["nK"], cfg["nT"], N=cfg["N"], put_itm=cfg["put_itm"])
    cal = DoubleHestonJumpCalibrator(S0, r, opts, N=cfg["N"])
    surf = cal._get_surface()
    host = bench.step_params(cal, 2, cfg["starts"], seed=0)
    for _ in range(3):
        surf.loss_terms(host[0], cfg["N"])
    surf.ctx.set_path(args.path)
    if args.dev:
        d_p = torch.from_numpy(np.ascontiguousarray(host[1])).cuda()
        d_sse = torch.empty(d_p.shape[0], dtype=torch.float64, device="cuda")
        d_bad = torch.empty(d_p.shape[0], dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        for _ in range(3):
            surf.loss_dev(d_p.data_ptr(), d_p.shape[0], d_sse.data_ptr(), d_bad.data_ptr(),
                          N=cfg["N"])
        surf.ctx.synchronize()
    surf.ctx.debug_stamps(True)
    if args.dev:
        surf.loss_dev(d_p.data_ptr(), d_p.shape[0], d_sse.data_ptr(), d_bad.data_ptr(), N=cfg["N"])
        surf.ctx.synchronize()
    elif args.mode == "loss":
        surf.loss_terms(host[1], cfg["N"])
    else:
        surf.price(host[1], cfg["N"])
    st = surf.ctx.read_stamps().astype(np.int64)
    surf.ctx.debug_stamps(False)
    if args.dump:
        np.save(args.dump, st)
    if surf.ctx.last_path == 2:          # cos_fused_kernel: stamps 0..5 of every block
        st = st[st[:, 0] > 0]
        print(f"{args.config} {args.mode}: fused-kernel blocks {len(st)}")
        names = ["prologue+stage", "cf+clamp", "consts+rot", "sums", "loss"]
        for i, nm in enumerate(names):
            c = st[:, i + 1] - st[:, i]
            print(f"  {nm:15s} median {np.median(c):8.0f}  p90 {np.percentile(c, 90):8.0f}  "
                  f"max {c.max():8.0f} cycles")
        life = st[:, 5] - st[:, 0]
        print(f"  lifetime median {np.median(life):8.0f}  max {life.max():8.0f}")
        detail = [("prologue (thread 0)", 0, 8), ("p: record+T in", 0, 31), ("p: range", 31, 28),
                  ("p: exps+consts", 28, 30), ("p: to end", 30, 8), ("staging wait", 8, 1),
                  ("cf: consts load", 1, 6), ("cf: clamp scan", 1, 29), ("cf: after scan", 29, 6), ("cf: entries", 6, 7), ("cf: clamp+barrier", 7, 2),
                  ("cf: start w1 - w0", 6, 19), ("cf: start w3 - w0", 6, 20),
                  ("cf: end w1 - w0", 7, 16), ("cf: end w2 - w0", 7, 17),
                  ("cf: end w3 - w0", 7, 18), ("cf: clamp loop w0", 7, 21),
                  ("cf: w1 at barrier - w0 CF end", 7, 22),
                  ("sums: setup", 3, 9),
                  ("sums: angle loop", 9, 10), ("sums: butterfly", 10, 11),
                  ("sums: finalise", 11, 4), ("loss: barrier", 4, 13), ("loss: wave sums", 13, 14),
                  ("loss: store drain", 14, 15), ("loss: ticket", 15, 12), ("loss: last", 12, 5)]
        for nm, i0, i1 in detail:
            # blocks that skip a phase (e.g. the prologue's "p:" stamps on blocks that load their
            # constants formed ahead) leave its stamps at 0: only blocks with both stamps count
            both = (st[:, i0] > 0) & (st[:, i1] > 0)
            if not both.any():
                continue
            c = (st[both, i1] - st[both, i0]).astype(np.int64)
            print(f"    {nm:20s} median {np.median(c):8.0f}  p90 {np.percentile(c, 90):8.0f}"
                  + (f"  ({both.sum()} blocks)" if not both.all() else ""))
        if args.timeline:
            timeline(st[:, 23])
            hw = st[:, 24:28].astype(np.int64)
            simd = (hw >> 4) & 3
            cu = (hw >> 8) & 15
            print("  SIMD of wave w (HW_ID bits 5:4), share of blocks per SIMD 0..3:")
            for w in range(4):
                sh = [np.mean(simd[:, w] == k) for k in range(4)]
                print(f"    wave {w}: " + "  ".join(f"{x:.2f}" for x in sh))
            print(f"  waves of a block on one CU: {np.mean((cu == cu[:, :1]).all(axis=1)):.3f}")
            # co-resident blocks: the same XCD (block id mod 8, round-robin dispatch), shader
            # engine / array and CU; their block-id differences and whether their waves share SIMDs
            se = (hw[:, 0] >> 13) & 3
            sh = (hw[:, 0] >> 12) & 1
            key = (np.arange(len(st)) % 8) * 10000 + se * 1000 + sh * 100 + cu[:, 0]
            groups = collections.defaultdict(list)
            for b, k in enumerate(key):
                groups[int(k)].append(b)
            sizes = collections.Counter(len(v) for v in groups.values())
            diffs = collections.Counter()
            rot = collections.Counter()
            same = []
            for v in groups.values():
                if len(v) == 2:
                    diffs[v[1] - v[0]] += 1
                    same.append(np.mean(simd[v[0]] == simd[v[1]]))
                    rot[int((simd[v[1], 0] - simd[v[0], 0]) % 4)] += 1
            print(f"  blocks per CU: {dict(sorted(sizes.items()))}; id differences of CU pairs "
                  f"(most common): {diffs.most_common(4)}; pairs' waves on the same SIMD: "
                  f"{np.mean(same) if same else float('nan'):.2f}; SIMD offset of the later block's "
                  f"wave 0: {dict(sorted(rot.items()))}")
            life = st[:, 5] - st[:, 0]
            ng = surf.n_groups if hasattr(surf, "n_groups") else cfg["nT"]
            g = np.arange(len(st)) % ng
            print(f"  lifetime (cycles) by maturity group ({ng} groups, group 0 = shortest T):")
            for lo in range(0, ng, max(1, ng // 10)):
                sel = (g >= lo) & (g < lo + max(1, ng // 10))
                print(f"    groups {lo:3d}..: median {np.median(life[sel]):8.0f}  "
                      f"p90 {np.percentile(life[sel], 90):8.0f}  "
                      f"cf {np.median(st[sel, 2] - st[sel, 1]):7.0f}  "
                      f"sums {np.median(st[sel, 4] - st[sel, 3]):7.0f}")
        return
    tb = st[st[:, 4] > 0]
    print(f"{args.config} {args.mode}: table-kernel blocks {len(tb)}")
    for nm, c in zip(["consts", "cf loop", "reduce"], [tb[:, 5] - tb[:, 4], tb[:, 6] - tb[:, 5],
                                                      tb[:, 7] - tb[:, 6]]):
        print(f"  {nm:8s} median {np.median(c):8.0f}  p90 {np.percentile(c, 90):8.0f}  "
              f"max {c.max():8.0f} cycles")
    st = st[st[:, 0] > 0]
    print(f"{args.config} {args.mode}: option-kernel blocks {len(st)}")
    for nm, c in zip(["stage", "options", "loss"], [st[:, 1] - st[:, 0], st[:, 2] - st[:, 1],
                                                     st[:, 3] - st[:, 2]]):
        print(f"  {nm:8s} median {np.median(c):8.0f}  p90 {np.percentile(c, 90):8.0f}  "
              f"max {c.max():8.0f} cycles")
    life = st[:, 3] - st[:, 0]
    print(f"  lifetime median {np.median(life):8.0f}  max {life.max():8.0f}")


def timeline(rt):
    """Resident fused blocks over the launch from the 100 MHz start/end stamps (10 ns ticks)."""
    # the slot is read as int64: mask the shifted start, or a start stamp with bit 31 set comes back
    # negative (and every residency as 2^32 ticks)
    t0 = ((rt >> 32) & 0xffffffff).astype(np.int64)
    t1 = (rt & 0xffffffff).astype(np.int64)
    t1 = np.where(t1 < t0, t1 + (1 << 32), t1)
    base = t0.min()
    t0, t1 = t0 - base, t1 - base
    span = t1.max()
    print(f"  timeline: {len(t0)} blocks over {span * 0.01:.2f} us; last start at "
          f"{t0.max() * 0.01:.2f} us; block residency median {np.median(t1 - t0) * 0.01:.2f} us "
          f"(p10 {np.percentile(t1 - t0, 10) * 0.01:.2f}, max {(t1 - t0).max() * 0.01:.2f})")
    nb = 40
    edges = np.linspace(0, span, nb + 1)
    mids = 0.5 * (edges[1:] + edges[:-1])
    res = [int(np.sum((t0 <= m) & (t1 > m))) for m in mids]
    peak = max(res)
    for m, c in zip(mids, res):
        print(f"    {m * 0.01:7.2f} us  {c:5d} {'#' * int(60 * c / max(peak, 1))}")
    # work-conserving estimate: the residency integral at the peak count
    busy = float(np.sum(t1 - t0))
    print(f"  resident-block integral / (peak {peak} x span): {busy / (peak * span):.3f}")


if __name__ == "__main__":
    main()
