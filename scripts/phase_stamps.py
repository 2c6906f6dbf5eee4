"""Per-phase timing of sgld_step_kernel from in-kernel s_memtime stamps (diagnostic build path:
stamps are written only by gpt_sgld_session_stamps launches).  Usage on the GPU box:
    python scripts/phase_stamps.py [--chains C] [--steps S]
"""
import argparse
import ctypes as C
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHAIN_NAMES = {1: "prologue (tables, U, rows)", 2: "batch loop", 3: "w update",
               4: "U noise + drive", 5: "proj + geod grams", 6: "expm x2", 7: "tmpU, norm, U write"}
NAMES = {1: "P0 stage", 2: "P1 V-phase", 3: "w-block gradw / U stage", 4: "P2 gradU (+barrier)",
         5: "proj gram+mom", 6: "geod grams", 7: "expm x2", 8: "tmpU+norm", 9: "U write+idx",
         10: "P5 next temp"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--n", type=int, default=500)
    ap.add_argument("--r", type=int, default=5)
    ap.add_argument("--m", type=int, default=50)
    ap.add_argument("--sgd", action="store_true", help="langevin=False (no noise draws)")
    ap.add_argument("--N", type=int, default=10000, help="training rows used (phi footprint)")
    ap.add_argument("--engine", default="grid", choices=["grid", "chain"])
    args = ap.parse_args()
    import torch
    import bench
    from gpt_amd import GPT_SGLD as G
    from gpt_amd._lib import check, lib
    from gpt_amd.session import SGLDSession, feature_device
    dev = torch.device("cuda", 0)
    n, D, r, Q, m = args.n, 8, args.r, 200, args.m
    Xtr, ytr, _, _, _ = bench.kin40k(D)
    Xtr, ytr = Xtr[:args.N], ytr[:args.N]
    ls = np.array([2.5242, 2.3376, 1.3630, 1.4949, 1.6022, 1.1366, 1.1964, 1.7028])
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    phi = feature_device(tt(Xtr.T), tt(ls), 1.042, math.sqrt(n / Q ** (1 / D)), tt(Z.T), tt(b.T))
    y = tt(ytr)
    s = SGLDSession(phi, y, I, r, Q, m, 1e-5, 1e-8, 0.0476, 0, 3, list(range(1, args.chains + 1)),
                    store=False, langevin=not args.sgd, engine=args.engine)
    s.run(50)
    s.sync()
    if args.engine == "chain":
        # the library sizes every step's slice for D+1 workgroups per chain; chain-engine
        # workgroup c writes slot c of it
        out = np.zeros((args.steps, (D + 1) * args.chains, 16), dtype=np.int64)
        check(lib().gpt_sgld_session_stamps(s._h, args.steps, out.ctypes.data_as(C.POINTER(C.c_int64))))
        out_all = out
        lp = out[:, args.chains:2 * args.chains, :]
        out = out[:, :args.chains, :]
        tot = np.median((out[..., 7] - out[..., 0]).ravel())
        print("chain engine: median cycles per phase (wave 0), batch of %d rows" % m)
        order = [1, 2, 3, 4, 5, 6, 7]
        prev = 0
        for i in order:
            v = np.median((out[..., i] - out[..., prev]).ravel())
            print("  %2d %-28s %8.0f cyc  %5.1f%%" % (i, CHAIN_NAMES[i], v, 100 * v / tot))
            prev = i
        print("  total %.0f cycles" % tot)
        arr = out[..., 8:16] - out[..., 0:1]
        print("  per-wave arrival at the end-of-step barrier (cycles from start):",
              " ".join("%d" % v for v in np.median(arr.reshape(-1, 8), axis=0)))
        if (lp[..., 7] > 0).all():
            names = ["vmcnt wait (row DMA)", "(a) rows LDS->regs", "(b) temp + reductions",
                     "barrier 1", "(c) V task", "barrier 2", "(e) residual, A, gradU"]
            for wv, base in (("wave 0", 0), ("wave 4", 8)):
                d = np.median(lp[..., base + 1:base + 8] - lp[..., base:base + 7], axis=(0, 1))
                print("  loop group 10, %s: " % wv + ", ".join("%s %d" % (nm, v) for nm, v in zip(names, d))
                      + "  (total %d)" % np.median(lp[..., base + 7] - lp[..., base]))
            print("  wave 4 starts the group %d cycles after wave 0"
                  % np.median(lp[..., 8] - lp[..., 0]))
        sp = np.concatenate([out_all[:, 2 * args.chains:3 * args.chains, :],
                             out_all[:, 3 * args.chains:4 * args.chains, :]], axis=2)
        # sp[..., 0:8] wave 0 slots 0-7, [8:16] wave 4 slots 0-7, [16:24] wave 0 slots 8-15,
        # [24:32] wave 4 slots 8-15
        if (sp[..., 0] > 0).all():
            snames = ["", "gwp barrier", "w update", "next batch idx/y + DMA", "noise+drive",
                      "proj", "geod grams", "expm 2r", "expm r", "F", "U.F pass", "mom.F pass + norms",
                      "norm sums", "normalise", "(unused)", "end barrier + U write"][:16]
            for wv, cols in (("wave 0", list(range(0, 8)) + list(range(16, 24))),
                             ("wave 4", list(range(8, 16)) + list(range(24, 32)))):
                ts = sp[..., cols]
                parts = []
                for i in range(1, 16):
                    if i == 14 or not (ts[..., i] > 0).all():
                        continue
                    j = i - 1
                    while j == 14 or not (ts[..., j] > 0).all():
                        j -= 1
                    parts.append("%s %d" % (snames[i], np.median(ts[..., i] - ts[..., j])))
                print("  Stiefel phase, %s (cycles): %s" % (wv, ", ".join(parts)))
                print("    %s: w-start %d cycles after wave 0's, end at +%d" % (
                    wv, np.median(ts[..., 0] - sp[..., 0]), np.median(ts[..., 15] - ts[..., 0])))
        for nm, row in (("expm 2r", 4), ("expm r", 5)):
            xs = out_all[:, row * args.chains:(row + 1) * args.chains, :]
            if (xs[..., 11:15] > 0).all():
                dx = np.median((xs[..., 12:15] - xs[..., 11:14]).reshape(-1, 3), axis=0)
                degs, cnt = np.unique(xs[..., 10], return_counts=True)
                print("  %s (wave 0): products %d, solve %d, squarings %d cycles; degree/scaling %s"
                      % ((nm,) + tuple(dx) + (dict(zip(degs.tolist(), cnt.tolist())),)))
        print("event-timed step kernel: %.2f us" % s.time_steps(20))
        return
    KB = D                                                       # k-blocks per chain
    nb = (KB + 1) * args.chains
    out = np.zeros((args.steps, nb, 16), dtype=np.int64)
    check(lib().gpt_sgld_session_stamps(s._h, args.steps, out.ctypes.data_as(C.POINTER(C.c_int64))))
    kblocks = out.reshape(args.steps, args.chains, KB + 1, 16)[:, :, :KB, :]
    wblocks = out.reshape(args.steps, args.chains, KB + 1, 16)[:, :, KB, :]
    print("k-blocks: median cycles per phase (stamp[i] - stamp[i-1])")
    prev = 0
    tot = np.median((kblocks[..., 10] - kblocks[..., 0]).ravel())
    for i in range(1, 11):
        d = kblocks[..., i] - kblocks[..., prev]
        ok = kblocks[..., i] > 0
        if ok.any():
            v = np.median(d[ok])
            print("  %2d %-26s %8.0f cyc  %5.1f%%" % (i, NAMES[i], v, 100 * v / tot))
            prev = i
    print("  total k-block %.0f cycles" % tot)
    xs = kblocks[..., 11:15]
    if (xs > 0).all():
        dx = np.median((xs[..., 1:] - xs[..., :-1]).reshape(-1, 3), axis=0)
        print("  expm(2r x 2r) inside: products %.0f, solve %.0f, squarings %.0f cycles" % tuple(dx))
        el = kblocks[..., 15] - kblocks[..., 12]
        if (kblocks[..., 15] > 0).all():
            print("  solve: elimination %.0f cycles, back substitution %.0f"
                  % (np.median(el), np.median(kblocks[..., 13] - kblocks[..., 15])))
    dw = np.median((wblocks[..., 3] - wblocks[..., 0]).ravel())
    print("w-block total %.0f cycles (V-phase %.0f)" % (dw, np.median((wblocks[..., 2] - wblocks[..., 0]).ravel())))
    t_us = s.time_steps(20)
    print("event-timed step kernel: %.2f us" % t_us)


if __name__ == "__main__":
    main()
