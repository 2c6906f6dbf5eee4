"""Wave engine against the oracle on kin40k data at kin40kExperiment.jl's shape (n = 150, r = 20),
step by step (every step stored): prints the relative error of each stored w / U sample, so a
divergence shows the step where it starts.

    python scripts/wave_check.py [--N 600] [--epochs 2] [--engine wave]
"""
import argparse
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=600)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--engine", default="wave")
    ap.add_argument("--epsw", type=float, default=1e-4)
    ap.add_argument("--epsU", type=float, default=1e-7)
    ap.add_argument("--seed", type=int, default=3)
    args = ap.parse_args()
    import bench
    from gpt_amd import GPT_SGLD as G
    from oracle import gpt_sgld_ref as R
    n, D, r, Q, m = 150, 8, 20, 200, 50
    Xtr, ytr, _, _, _ = bench.kin40k(D)
    Xtr, ytr = Xtr[:args.N], ytr[:args.N]
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    phi = R.feature(Xtr, np.array(bench.KIN40K_LS), 1.0420, math.sqrt(n / Q ** (1.0 / D)), Z, b)
    ws, Us, dg = G.GPTregression(phi, ytr, 0.0476, I, r, Q, m, args.epsw, args.epsU, 0, args.epochs,
                                 args.seed, diag=True, engine=args.engine)
    wo, Uo, info = R.GPTregression(phi, ytr, 0.0476, I, r, Q, m, args.epsw, args.epsU, 0,
                                   args.epochs, args.seed, record=True)
    print("oracle status", info["status"], "gpu all-zero", not ws.any())
    T = ws.shape[1]
    gw = np.array(info["gradw_norm"])
    for t in range(T):
        ew = np.abs(ws[:, t] - wo[:, t]).max() / max(np.abs(wo[:, t]).max(), 1e-300)
        eu = np.abs(Us[..., t] - Uo[..., t]).max() / max(np.abs(Uo[..., t]).max(), 1e-300)
        eg = abs(dg[0, t] - gw[t]) / max(abs(gw[t]), 1e-300) if t < gw.size else float("nan")
        print("step %3d  w %.2e  U %.2e  gradw %.2e  |w| %.3e" % (t, ew, eu, eg, np.abs(wo[:, t]).max()))




def multichain(argv):
    """python scripts/wave_check.py multi [C] [steps]: chain c of a C-chain session vs a one-chain
    session of its seed (bitwise) and the oracle, on the kin40k subset."""
    import torch
    import bench
    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import SGLDSession
    from oracle import gpt_sgld_ref as R
    Cn = int(argv[0]) if argv else 8
    steps = int(argv[1]) if len(argv) > 1 else 24
    n, D, r, Q, m, Nsub = 150, 8, 20, 200, 50, 600
    Xtr, ytr, _, _, _ = bench.kin40k(D)
    Xtr, ytr = Xtr[:Nsub], ytr[:Nsub]
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    phi = R.feature(Xtr, np.array(bench.KIN40K_LS), 1.0420, math.sqrt(n / Q ** (1.0 / D)), Z, b)
    dev = torch.device("cuda", 0)
    phit = torch.from_numpy(np.ascontiguousarray(phi.transpose(2, 1, 0))).to(dev)
    yt = torch.from_numpy(np.ascontiguousarray(ytr)).to(dev)
    nb = -(-Nsub // m)
    ep = -(-steps // nb)
    s = SGLDSession(phit, yt, I, r, Q, m, 1e-4, 1e-7, 0.0476, 0, ep, list(range(1, Cn + 1)),
                    store=True, engine="wave")
    s.run(steps)
    s.sync()
    for c in range(Cn):
        ws, Us, st = s.fetch(c)
        s1 = SGLDSession(phit, yt, I, r, Q, m, 1e-4, 1e-7, 0.0476, 0, ep, [c + 1], store=True,
                         engine="wave")
        s1.run(steps)
        s1.sync()
        w1, U1, st1 = s1.fetch(0)
        s1.close()
        wo, Uo, info = R.GPTregression(phi, ytr, 0.0476, I, r, Q, m, 1e-4, 1e-7, 0, ep, c + 1,
                                       max_steps=steps)
        k = min(steps, ws.shape[1])
        print("chain %d status %d single %d oracle %d  |multi-single| %.2e  multi-oracle w %.2e U %.2e"
              % (c, st, st1, info["status"], np.abs(ws[:, :k] - w1[:, :k]).max(),
                 np.abs(ws[:, :k] - wo[:, :k]).max() / np.abs(wo[:, :k]).max(),
                 np.abs(Us[..., :k] - Uo[..., :k]).max()), flush=True)
    s.close()


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "multi":
    multichain(sys.argv[2:])
    sys.exit(0)


if __name__ == "__main__":
    main()
