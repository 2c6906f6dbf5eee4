"""Wall time per sweep of GPT_fullw_gibbs (100k_movielensExperiment.jl:1032-1129) at BASELINE
config 5's r = 20 on fold 1, bench.py's parameter line (signal_var = σ_u = 0.5,
σ_w = ‖w_init‖_F / r, avg = true, param_seed 10); run under `rocprofv3 --kernel-trace --stats`
for the per-kernel split of a sweep.

    python scripts/time_gibbs.py [--sweeps 40] [--r 20]
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
    ap.add_argument("--sweeps", type=int, default=40)
    ap.add_argument("--r", type=int, default=20)
    args = ap.parse_args()
    from gpt_amd import movielens
    d = np.load(os.path.join(ROOT, "tests", "golden", "ml100k.npz"))
    tr, te, ud, md, mu, sd = movielens.fold(d, 1)
    r = args.r
    wg = np.random.default_rng(10).standard_normal((r, r))
    sw = math.sqrt((wg ** 2).sum()) / r
    movielens.GPT_fullw_gibbs(tr, ud, md, te, 0.5, 0.5, sw, wg, 1, 2, 1, 10, mu, sd, avg=True)
    t0 = time.perf_counter()
    go = movielens.GPT_fullw_gibbs(tr, ud, md, te, 0.5, 0.5, sw, wg, 0, args.sweeps, 1, 10, mu, sd,
                                   avg=True)
    dt = time.perf_counter() - t0
    print(json.dumps(dict(r=r, sweeps=args.sweeps, seconds=dt, ms_per_sweep=1e3 * dt / args.sweeps,
                          test_rmse_final=float(np.asarray(go[5])[-1]))), flush=True)


if __name__ == "__main__":
    main()
