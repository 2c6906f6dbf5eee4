"""Wall time of the live MovieLens experiment's 5-fold call (GPT_fullw_sideinfo_folds, r = 20,
100k_movielensExperiment.jl:723-739) for A/B runs of two library builds (GPTSGLD_LIB):

    GPTSGLD_LIB=gpt_amd/libgptsgld_head.so python scripts/ml_ab.py [--epochs 20] [--r 20]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--r", type=int, default=20)
    args = ap.parse_args()
    import bench
    from gpt_amd import movielens
    cfg = bench.ML_CONFIG
    d = np.load(os.path.join(ROOT, "tests", "golden", "ml100k.npz"))
    folds = [movielens.fold(d, i) for i in range(1, 6)]
    w0 = np.random.default_rng(17).standard_normal((args.r, args.r))

    def run(E):
        return movielens.GPT_fullw_sideinfo_folds(
            [f[0] for f in folds], folds[0][2], folds[0][3], [f[1] for f in folds],
            cfg["signal_var"], cfg["sigma_u"], cfg["sigma_w"], w0, cfg["m"], cfg["epsw"],
            cfg["epsU"], cfg["a"], cfg["b"], cfg["c"], 0, E, cfg["param_seed"],
            [f[4] for f in folds], [f[5] for f in folds])

    run(2)
    t0 = time.perf_counter()
    outs = run(args.epochs)
    dt = time.perf_counter() - t0
    nb = -(-folds[0][0].shape[0] // cfg["m"])
    print("lib %s: %d epochs in %.3f s = %.1f ms/epoch, %.0f fold-steps/s; min test RMSE %s"
          % (os.environ.get("GPTSGLD_LIB", "default"), args.epochs, dt, 1e3 * dt / args.epochs,
             5 * nb * args.epochs / dt, [round(float(o[5].min()), 5) for o in outs]))


if __name__ == "__main__":
    main()
