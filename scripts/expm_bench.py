"""Shader cycles of the wave engine's 2r x 2r Padé expm as geod calls it (three LDS slots, r result
columns), per Padé degree: geodesic-shaped matrices t·[A −S; I A] scaled to 1-norms in each
degree's range, one wave per matrix (gpt_debug_expm_stamps), medians of the polynomial and solve
phases.  Two launch shapes: one matrix per CU (no LDS contention) and four per CU (as the engine
runs them).

    python scripts/expm_bench.py [--nn 40] [--count 1024]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def mats(nn, count, target, seed):
    r = nn // 2
    rng = np.random.default_rng(seed)
    out = np.empty((count, nn, nn))
    for c in range(count):
        B = rng.standard_normal((r, r))
        A = (B - B.T) / 2
        W = rng.standard_normal((3 * r, r))
        T = np.block([[A, -(W.T @ W)], [np.eye(r), A]])
        out[c] = T * (target / np.abs(T).sum(axis=0).max())
    return np.ascontiguousarray(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nn", type=int, default=40)
    ap.add_argument("--count", type=int, default=1024)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)
    from gpt_amd import _lib
    res = {}
    for deg, target in ((3, 0.01), (5, 0.13), (7, 0.6), (9, 1.5), (13, 4.4), (13, 20.0)):
        for count in (256, args.count):
            A = mats(args.nn, count, target, deg)
            st = np.zeros((count, 4), dtype=np.int64)
            _lib.check(_lib.lib().gpt_debug_expm_stamps(args.nn, count, A.ctypes.data_as(_lib.P_D),
                                                        st.ctypes.data_as(C.POINTER(C.c_int64))))
            d = np.diff(st, axis=1).astype(float)
            key = "deg%d_norm%g_%d" % (deg, target, count)
            res[key] = {"poly": float(np.median(d[:, 0])), "solve": float(np.median(d[:, 1])),
                        "rest": float(np.median(d[:, 2])),
                        "total": float(np.median(st[:, 3] - st[:, 0]))}
            print(key, res[key], flush=True)
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
