"""Config 4's literal form (one chain per GPU) at the kin40k bench shape on each step engine that
takes it: µs per step by hipEvents around a prepared 2 000-step run after a 1 s clock warm-up.

    python scripts/single_chain_ab.py [--engines grid wave] [--chains 1]
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
    ap.add_argument("--engines", nargs="+", default=["grid", "wave"])
    ap.add_argument("--chains", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch
    import bench
    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import SGLDSession, feature_device
    dev = torch.device("cuda", 0)
    n, D, r, Q, m = 500, 8, 5, 200, 50
    Xtr, ytr, _, _, _ = bench.kin40k(D)
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    phi = feature_device(tt(Xtr.T), tt(np.array(bench.KIN40K_LS)), 1.042,
                         math.sqrt(n / Q ** (1 / D)), tt(Z.T), tt(b.T))
    y = tt(ytr)
    st = torch.cuda.Stream(device=dev)
    out = {}
    for rep in range(args.reps):
        for eng in args.engines:
            s = SGLDSession(phi, y, I, r, Q, m, 1e-5, 1e-8, 0.0476, 0, 400,
                            [7 + c for c in range(args.chains)], store=False, engine=eng,
                            stream=st.cuda_stream)
            info = s.info()
            tw = time.perf_counter()
            while time.perf_counter() - tw < 0.5:
                s.run(200)
                s.sync()
            s.prepare(args.steps)
            s.sync()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            s.run(args.steps)
            e1.record(st)
            s.sync()
            us = 1000.0 * e0.elapsed_time(e1) / args.steps
            ok = all(s.status(c) == 0 for c in range(args.chains))
            s.close()
            out.setdefault(eng, []).append(us)
            print(json.dumps(dict(engine=eng, info=info, us_per_step=us,
                                  steps_per_s=args.chains * 1e6 / us, alive=ok)), flush=True)
    print(json.dumps({k: min(v) for k, v in out.items()}))


if __name__ == "__main__":
    main()
