"""Time the stacked-sample prediction (MFMA GEMM + V-phase) on the GPU.

    python scripts/time_pred.py [--S 256] [--n 500] [--r 5] [--Ntest 30000]
Prints ms per call and the GEMM's fp64 TFLOP/s for each GPTSGLD_PRED_VPHASE (pairs, rows) asked
for.  (Rounds 3-5 also compared GEMM wave tiles and a tile V-phase; those switches were removed
from the library in round 6 with the 4 x 4 tile kept.)
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", type=int, default=256)
    ap.add_argument("--n", type=int, default=500)
    ap.add_argument("--r", type=int, default=5)
    ap.add_argument("--D", type=int, default=8)
    ap.add_argument("--Q", type=int, default=200)
    ap.add_argument("--Ntest", type=int, default=30000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--vphases", default="pairs,rows",
                    help="GPTSGLD_PRED_VPHASE values to compare (pairs, rows)")
    a = ap.parse_args()
    import torch
    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import pred_device
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    phi = torch.randn(a.Ntest * a.D * a.n, dtype=torch.float64, device=dev, generator=g) * 0.05
    U = torch.randn(a.S, a.n * a.r * a.D, dtype=torch.float64, device=dev, generator=g) * 0.05
    w = torch.randn(a.S, a.Q, dtype=torch.float64, device=dev, generator=g)
    I = G.samplenz(a.r, a.D, a.Q, 3)
    I0 = torch.from_numpy(np.asfortranarray(I - 1).ravel(order="F").astype(np.int32)).to(dev)
    f = torch.empty(a.S, a.Ntest, dtype=torch.float64, device=dev)
    flop = 2.0 * a.S * a.r * a.n * a.D * a.Ntest
    ref = None
    for vp in a.vphases.split(","):
        os.environ["GPTSGLD_PRED_VPHASE"] = vp
        pred_device(w.data_ptr(), U.data_ptr(), I0, phi, a.n, a.D, a.Ntest, a.r, a.Q, a.S, f)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            pred_device(w.data_ptr(), U.data_ptr(), I0, phi, a.n, a.D, a.Ntest, a.r, a.Q, a.S, f)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        if ref is None:
            ref = f.clone()
        d = (f - ref).abs().max().item() / ref.abs().max().item()
        print("vphase %s: %.3f ms per call (GEMM + V-phase), GEMM flop / call time %.1f "
              "TFLOP/s, max rel diff vs the first %.1e" % (vp, ms, flop / ms / 1e9, d), flush=True)


if __name__ == "__main__":
    main()
