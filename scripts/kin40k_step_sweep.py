"""Step-size sweep at a kin40k shape on the GPU: one 256-chain session, a grid
of (εw, εU) pairs set per chain with gpt_sgld_session_set_hyper, every chain run for the
reference's 200 epochs (kin40kExperiment.jl:74), the epoch-end samples of the last 50 epochs
predicted on the 30 000 test rows (:78-87).  Per pair: chains that hit the geodesic NaN
bail-out (GPT_SGLD.jl:422-424), the median chain's epoch-200 test RMSE and last-50 curve mean,
and the ensemble RMSE of the pair's surviving chains' mean prediction.

    python scripts/kin40k_step_sweep.py --n 500 --r 5 --epsw 1e-5,3e-5,1e-4 --epsU 1e-8,1e-7 \
        --out gpurun_out/sweep.json
"""
import argparse
import itertools
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=500)
    ap.add_argument("--r", type=int, default=5)
    ap.add_argument("--chains", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=200)
    ap.add_argument("--last", type=int, default=50)
    ap.add_argument("--epsw", default="1e-5,2e-5,5e-5,1e-4")
    ap.add_argument("--epsU", default="1e-8,3e-8,1e-7,3e-7")
    ap.add_argument("--seed0", type=int, default=1001, help="first chain seed")
    ap.add_argument("--engine", default="auto")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch
    import bench
    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import SGLDSession, feature_device, pred_device

    dev = torch.device("cuda", 0)
    n, D, r, Q, m, sv = args.n, 8, args.r, 200, 50, 0.0476
    Xtr, ytr, Xte, yte, ysd = bench.kin40k(D)
    N, Nte = Xtr.shape[0], Xte.shape[0]
    nb = -(-N // m)
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    scale = math.sqrt(n / Q ** (1.0 / D))
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    ls = tt(np.array(bench.KIN40K_LS))
    phi = feature_device(tt(Xtr.T), ls, 1.0420, scale, tt(Z.T), tt(b.T))
    phite = feature_device(tt(Xte.T), ls, 1.0420, scale, tt(Z.T), tt(b.T))
    pairs = list(itertools.product([float(x) for x in args.epsw.split(",")],
                                   [float(x) for x in args.epsU.split(",")]))
    C = args.chains
    per = C // len(pairs)
    assert per >= 1, "more pairs than chains"
    C = per * len(pairs)
    last = min(args.last, args.epochs)
    sess = SGLDSession(phi, tt(ytr), I, r, Q, m, pairs[0][0], pairs[0][1], sv, args.epochs - last,
                       last, list(range(args.seed0, args.seed0 + C)), store_every=nb, store=True,
                       engine=args.engine)
    for c in range(C):
        ew, eu = pairs[c // per]
        sess.set_hyper(c, ew, eu, sv)
    t0 = time.perf_counter()
    sess.run(sess.total_steps)
    sess.sync()
    train_s = time.perf_counter() - t0
    I0 = torch.from_numpy(np.asfortranarray(I - 1).ravel(order="F").astype(np.int32)).to(dev)
    yte_d = tt(yte)
    fh = torch.empty((last, Nte), dtype=torch.float64, device=dev)
    res = []
    for p, (ew, eu) in enumerate(pairs):
        finals, means, bailed = [], [], 0
        fsum = torch.zeros(Nte, dtype=torch.float64, device=dev)
        cnt = 0
        for c in range(p * per, (p + 1) * per):
            if sess.status(c) != 0:
                bailed += 1
                continue
            _, _, ws, Us, ns = sess.device_state(c)
            pred_device(ws, Us, I0, phite, n, D, Nte, r, Q, ns, fh)
            err = fh[:ns] - yte_d[None, :]
            curve = (ysd * torch.sqrt((err * err).mean(dim=1))).cpu().numpy()
            finals.append(float(curve[-1]))
            means.append(float(curve.mean()))
            fsum += fh[:ns].sum(dim=0)
            cnt += ns
        d = dict(epsw=ew, epsU=eu, chains=per, bailed=bailed)
        if finals:
            fm = (fsum / cnt).cpu().numpy()
            d.update(median_final=float(np.median(finals)), median_last50=float(np.median(means)),
                     min_final=float(np.min(finals)), max_final=float(np.max(finals)),
                     ensemble_rmse=float(ysd * math.sqrt(np.mean((fm - yte) ** 2))))
        res.append(d)
        print(json.dumps(d), flush=True)
    out = dict(n=n, D=D, r=r, Q=Q, m=m, epochs=args.epochs, last=last, engine=sess.info()["engine"],
               chains=C, train_s=train_s, seed0=args.seed0, pairs=res,
               reference=dict(file="testRMSE_kin40k.h5 (n = 150, r = 20)", final=0.2385,
                              last50_curve_mean=0.2448))
    sess.close()
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
