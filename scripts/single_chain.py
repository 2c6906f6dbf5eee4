"""Single-chain latency sweep: one kin40k-shaped chain (the bench shape: D=8, n=500, r=5, Q=200, m=50)
on the grid engine and on the split engine at each batch-slice count S.

Prints one JSON line per configuration: steps/s over `--steps` graph-replayed steps after a warm-up,
plus the per-launch kernel time from hipEvents (session.time_steps).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4000)
    ap.add_argument("--warmup", type=int, default=400)
    ap.add_argument("--splits", default="0,2,3,4,5,6,7,8")
    args = ap.parse_args()
    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import SGLDSession
    dev = torch.device("cuda", 0)
    N, D, n, r, Q, m = 36000, 8, 500, 5, 200, 50
    rng = np.random.default_rng(3)
    phi = torch.from_numpy(rng.standard_normal((N, D, n)) * 0.1).to(dev)
    y = torch.from_numpy(rng.standard_normal(N)).to(dev)
    I = G.samplenz(r, D, Q, 17)
    nb = -(-N // m)
    need = args.warmup + args.steps + 64
    epochs = -(-need // nb) + 1
    for s in [int(v) for v in args.splits.split(",")]:
        if s == 0:
            os.environ.pop("GPTSGLD_SPLIT", None)
            engine = "grid"
        else:
            os.environ["GPTSGLD_SPLIT"] = str(s)
            engine = "split"
        s1 = SGLDSession(phi, y, I, r, Q, m, 1e-5, 1e-8, 0.0476, 0, epochs, [7], store_every=nb,
                         store=False, engine=engine)
        s1.run(args.warmup)
        s1.prepare(args.steps)
        s1.sync()
        t1 = time.perf_counter()
        s1.run(args.steps)
        s1.sync()
        sps = args.steps / (time.perf_counter() - t1)
        k_us = s1.time_steps(64)
        info = s1.info()
        s1.close()
        print(json.dumps({"split": s, "engine": info["engine"], "workgroups": info.get("workgroups"),
                          "steps_per_s": round(sps, 1), "kernel_us": k_us}), flush=True)
    os.environ.pop("GPTSGLD_SPLIT", None)


if __name__ == "__main__":
    main()
