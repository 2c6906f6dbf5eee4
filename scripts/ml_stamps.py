"""Per-phase shader cycles of the MovieLens epoch kernel (cf_epoch_kernel) at the live
configuration of 100k_movielensExperiment.jl:723-739 (5 folds, r = 20, m = 100): medians over
fold 0's first 64 steps (GPTSGLD_CF_STAMPS, gpt_cf_last_stamps).

    python scripts/ml_stamps.py [--r 20]
    GPTSGLD_LIB=gpt_amd/libgptsgld_diag.so python scripts/ml_stamps.py   (+ per-wave sub-phases)
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PH = ["batch", "masks+links", "sums", "sum*w", "residual", "gradw+rows", "moves U,V"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--r", type=int, default=20)
    args = ap.parse_args()
    os.environ["GPTSGLD_CF_STAMPS"] = "1"
    import bench
    from gpt_amd import movielens
    from gpt_amd._lib import lib
    cfg = bench.ML_CONFIG
    d = np.load(os.path.join(ROOT, "tests", "golden", "ml100k.npz"))
    folds = [movielens.fold(d, i) for i in range(1, 6)]
    w0 = np.random.default_rng(17).standard_normal((args.r, args.r))
    movielens.GPT_fullw_sideinfo_folds(
        [f[0] for f in folds], folds[0][2], folds[0][3], [f[1] for f in folds], cfg["signal_var"],
        cfg["sigma_u"], cfg["sigma_w"], w0, cfg["m"], cfg["epsw"], cfg["epsU"], cfg["a"], cfg["b"],
        cfg["c"], 0, 1, cfg["param_seed"], [f[4] for f in folds], [f[5] for f in folds])
    st = np.zeros(64 * 72, dtype=np.int64)
    n = lib().gpt_cf_last_stamps(st.ctypes.data_as(C.POINTER(C.c_int64)), st.size)
    slots = n // 64
    full = st[:n].reshape(64, slots).astype(np.float64)
    full = full[(full[:, :8] > 0).all(axis=1)]
    st = full[:, :8]
    if slots > 8:
        # diagnostic build (CF_WSTAMPS): per wave, cycles after the step's sums-phase start
        # (stamp 2) to the end of its sums loop, and after the gradient phase's start (stamp 5) to
        # the end of its gradw tiles, its feature tiles and its gradient rows
        ws = full[:, 8:].reshape(len(full), 16, 4)
        print("per wave (median over steps): sums-loop end | gradw end | ftiles end | rows end")
        for wv in range(16):
            print("  wave %2d  %7.0f  %7.0f  %7.0f  %7.0f" % (
                wv, np.median(ws[:, wv, 0] - st[:, 2]), np.median(ws[:, wv, 1] - st[:, 5]),
                np.median(ws[:, wv, 2] - st[:, 5]), np.median(ws[:, wv, 3] - st[:, 5])))
    d = np.diff(st, axis=1)
    tot = np.median(st[1:, 0] - st[:-1, 0])
    print("steps", len(st), "median cycles per step", tot)
    for i, nm in enumerate(PH):
        print("  %-14s %8.0f" % (nm, np.median(d[:, i])))
    print("  %-14s %8.0f" % ("w copy+next", tot - np.median(st[:, 7] - st[:, 0])))


if __name__ == "__main__":
    main()
