"""Wall-clock of the MovieLens-100k CF samplers on the GPU (config 5): the live GPT_fullw_sideinfo
run of 100k_movielensExperiment.jl:723-730 (fold 1, r = 15 or --r, m = 100) and one GPT_fullw_gibbs
sweep, printed as one JSON line.  Usage: python scripts/time_movielens.py [--epochs E]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--r", type=int, default=15, help="rank (BASELINE config 5 is r = 20)")
    args = ap.parse_args()
    from gpt_amd import movielens
    d = np.load(os.path.join(ROOT, "tests", "golden", "ml100k.npz"))
    tr, te, ud, md, mu, sd = movielens.fold(d, 1)
    w0 = np.random.default_rng(17).standard_normal((args.r, args.r))
    movielens.GPT_fullw_sideinfo(tr, ud, md, te, 0.8, 0.1, 1.0, w0, 100, 1e-4, 1e-6, 0.5, 0.25,
                                 0.5, 0, 1, 17, mu, sd)                        # warm-up / load
    t = time.perf_counter()
    out = movielens.GPT_fullw_sideinfo(tr, ud, md, te, 0.8, 0.1, 1.0, w0, 100, 1e-4, 1e-6, 0.5,
                                       0.25, 0.5, 0, args.epochs, 17, mu, sd)
    ts = (time.perf_counter() - t) / args.epochs
    t = time.perf_counter()
    g = movielens.GPT_fullw_gibbs(tr, ud, md, te, 0.8, 0.5, 1.0, w0, 0, 2, 1, 17, mu, sd)
    tg = (time.perf_counter() - t) / 2
    # the five folds of :733-736: separate calls vs one launch per epoch for all folds
    fl = [movielens.fold(d, i) for i in range(1, 6)]
    args5 = (0.8, 0.1, 1.0, w0, 100, 1e-4, 1e-6, 0.5, 0.25, 0.5, 0, args.epochs, 17)
    t = time.perf_counter()
    for f in fl:
        movielens.GPT_fullw_sideinfo(f[0], ud, md, f[1], *args5, f[4], f[5])
    t_sep = (time.perf_counter() - t) / args.epochs
    t = time.perf_counter()
    o5 = movielens.GPT_fullw_sideinfo_folds([f[0] for f in fl], ud, md, [f[1] for f in fl], *args5,
                                            [f[4] for f in fl], [f[5] for f in fl])
    t_fold = (time.perf_counter() - t) / args.epochs
    print(json.dumps({"workload": "ml-100k fold 1, r=%d" % args.r, "sideinfo_sgd_s_per_epoch": ts,
                      "sideinfo_steps_per_s": 800 / ts, "sideinfo_testRMSE": list(out[5]),
                      "gibbs_s_per_sweep": tg, "gibbs_testRMSE": list(g[5]),
                      "five_folds_separate_s_per_epoch": t_sep,
                      "five_folds_one_launch_s_per_epoch": t_fold,
                      "five_folds_steps_per_s": 5 * 800 / t_fold,
                      "five_folds_testRMSE_last": [float(o[5][args.epochs - 1]) for o in o5]}))


if __name__ == "__main__":
    main()
