"""Per-phase shader cycles of the wave engine (wave.hip WSTAMP slots, s_memtime) at
kin40kExperiment.jl's configuration (n = 150, D = 8, r = 20, Q = 200, m = 50).

    python scripts/wave_stamps.py [--chains 256] [--steps 4]
"""
import argparse
import ctypes as C
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DIM = ["stage", "gradU", "drive+noise", "M gram", "mom+S", "park+X1", "expm r", "X0+expm 2r",
       "F", "tmpU+norm+write", "phidotU next"]
VPH = ["V+fhat", "gradw+w", "coef"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=256)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--n", type=int, default=150)
    ap.add_argument("--r", type=int, default=20)
    ap.add_argument("--epsU", type=float, default=1e-7)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    import bench
    from gpt_amd import GPT_SGLD as G
    from gpt_amd._lib import check, lib
    from gpt_amd.session import SGLDSession, feature_device
    dev = torch.device("cuda", 0)
    n, D, r, Q, m = args.n, 8, args.r, 200, 50
    Xtr, ytr, _, _, _ = bench.kin40k(D)
    ls = np.array(bench.WORKLOADS["kin40k"][3])
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    phi = feature_device(tt(Xtr.T), tt(ls), 1.0420, math.sqrt(n / Q ** (1.0 / D)), tt(Z.T), tt(b.T))
    Cn = args.chains
    s = SGLDSession(phi, tt(ytr), I, r, Q, m, 1e-5, args.epsU, 0.0476, 0, 3, list(range(1, Cn + 1)),
                    store=False, engine="wave")
    s.run(20)
    s.sync()
    W = (D + 1) * Cn
    out = np.zeros((args.steps, W, 16), dtype=np.int64)
    check(lib().gpt_sgld_session_stamps(s._h, args.steps, out.ctypes.data_as(C.POINTER(C.c_int64))))
    alive = [c for c in range(Cn) if s.status(c) == 0]
    s.close()
    res = {}
    rows = np.array([[c * (D + 1) + k for k in range(D)] for c in alive]).ravel()
    dim = out[:, rows, :12].reshape(-1, 12).astype(np.float64)
    ok = (dim > 0).all(axis=1)
    d = np.diff(dim[ok], axis=1)
    res["dim_cycles_median"] = {nm: float(np.median(d[:, i])) for i, nm in enumerate(DIM)}
    res["dim_total_median"] = float(np.median(dim[ok, 11] - dim[ok, 0]))
    # inside the expm: products (to slot 12 / 14), solve (to 13 / 15)
    ex = out[:, rows, :].reshape(-1, 16).astype(np.float64)
    okx = (ex[:, [6, 7, 8, 12, 13, 14, 15]] > 0).all(axis=1)
    e = ex[okx]
    res["expm_r"] = {"poly": float(np.median(e[:, 14] - e[:, 6])), "solve": float(np.median(e[:, 15] - e[:, 14])),
                     "rest": float(np.median(e[:, 7] - e[:, 15]))}
    res["expm_2r"] = {"X0+poly": float(np.median(e[:, 12] - e[:, 7])), "solve": float(np.median(e[:, 13] - e[:, 12])),
                      "rest": float(np.median(e[:, 8] - e[:, 13]))}
    vrows = np.array([c * (D + 1) + D for c in alive])
    vp = out[:, vrows, :5].reshape(-1, 5).astype(np.float64)
    okv = (vp > 0).all(axis=1)
    dv = np.diff(vp[okv][:, :4], axis=1)
    res["vphase_cycles_median"] = {nm: float(np.median(dv[:, i])) for i, nm in enumerate(VPH)}
    res["vphase_stage_cycles_median"] = float(np.median(vp[okv][:, 4] - vp[okv][:, 0]))
    # launch spans (first entry to last exit, per step) in shader ticks
    spans = []
    for st in range(args.steps):
        a = out[st, rows, 0]
        z = out[st, rows, 11]
        a, z = a[a > 0], z[z > 0]
        if a.size and z.size:
            spans.append(float(z.max() - a.min()))
    res["dim_launch_span_median"] = float(np.median(spans)) if spans else None
    res["chains_alive"] = len(alive)
    print(json.dumps(res, indent=1))
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
