"""Step time of the r = 20 engines at kin40kExperiment.jl's configuration (n = 150, D = 8, r = 20,
Q = 200, m = 50): chain-steps/s for several chain counts on the wave and grid engines.

    python scripts/wave_probe.py [--chains 256,10,1] [--engines wave,grid] [--steps 200]
"""
import argparse
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
    ap.add_argument("--chains", default="256,10,1")
    ap.add_argument("--engines", default="wave,grid")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--n", type=int, default=150)
    ap.add_argument("--r", type=int, default=20)
    ap.add_argument("--epsw", type=float, default=1e-4)
    ap.add_argument("--epsU", type=float, default=1e-7)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    import bench
    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import SGLDSession, feature_device
    dev = torch.device("cuda", 0)
    n, D, r, Q, m = args.n, 8, args.r, 200, 50
    Xtr, ytr, Xte, yte, ysd = bench.kin40k(D)
    ls = np.array(bench.WORKLOADS["kin40k"][3])
    scale = math.sqrt(n / Q ** (1.0 / D))
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    phi = feature_device(tt(Xtr.T), tt(ls), 1.0420, scale, tt(Z.T), tt(b.T))
    y = tt(ytr)
    torch.cuda.synchronize()
    nb = -(-Xtr.shape[0] // m)
    res = []
    for eng in args.engines.split(","):
        for C in [int(x) for x in args.chains.split(",")]:
            if eng == "grid" and C > 64:
                continue
            epochs = 2 + -(-(3 * args.steps) // nb)
            s = SGLDSession(phi, y, I, r, Q, m, args.epsw, args.epsU, 0.0476, 0, epochs,
                            list(range(1, C + 1)), store=False, engine=eng)
            s.run(50)
            s.prepare(args.steps)
            s.sync()
            t0 = time.perf_counter()
            s.run(args.steps)
            s.sync()
            dt = time.perf_counter() - t0
            k_us = s.time_steps(20)
            st = [s.status(c) for c in range(C)]
            d = dict(engine=s.info()["engine"], chains=C, us_per_step=1e6 * dt / args.steps,
                     chain_steps_per_s=C * args.steps / dt, event_us=k_us,
                     bailed=sum(1 for x in st if x))
            print(json.dumps(d), flush=True)
            res.append(d)
            s.close()
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
