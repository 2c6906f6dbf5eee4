"""The geodesic bail-out step (GPT_SGLD.jl:23-26, 422-424) of diverging chains in the two CPU
restatements (oracle/cpu C++ loops; oracle/gpt_sgld_ref.py numpy/LAPACK), on kin40kExperiment.jl's
shape (n = 150, r = 20, εw = 1e-4, εU = 1e-7, seeds 1..32, two epochs) and on the bench shape
(n = 500, r = 5, εw = 1e-5, εU = 1e-8, seeds 5001..5032, two epochs), with each bailing chain's
largest ‖t·[A −S; I A]‖₁ per step before it bails (the expm scaling it forces).

    python scripts/bail_steps_cpu.py profiles/r6_bail_steps.json
"""
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out):
    import bench
    from gpt_amd import GPT_SGLD as G
    from oracle import cpu_lib
    from oracle import gpt_sgld_ref as R
    Xtr, ytr, _, _, _ = bench.kin40k(8)
    D, Q, m = 8, 200, 50
    res = {}
    for name, n, r, ew, eu, seeds in (("kin40k_ref", 150, 20, 1e-4, 1e-7, range(1, 33)),
                                      ("bench", 500, 5, 1e-5, 1e-8, range(5001, 5033))):
        I = G.samplenz(r, D, Q, 17)
        Z, b = G.feature_inputs(n, D, 17)
        phi = R.feature(Xtr, np.array(bench.KIN40K_LS), 1.0420, math.sqrt(n / Q ** (1.0 / D)), Z, b)
        sd = np.array(list(seeds), dtype=np.uint64)
        cpu = cpu_lib.GPTregression_chains(phi, ytr, 0.0476, I, r, Q, m, ew, eu, 0, 2, sd,
                                           threads=os.cpu_count())
        cpp = {int(s): int(c) for s, st, c in zip(sd, cpu["status"], cpu["chain_steps"]) if st}
        npy, norms = {}, {}
        orig = R.geod
        for s, st in cpp.items():
            trace = []

            def geod(U, mom, t, _trace=trace):
                A = U.T @ mom
                T = np.block([[A, -(mom.T @ mom)], [np.eye(U.shape[1]), A]])
                _trace.append(float(np.abs(t * T).sum(axis=0).max()))
                return orig(U, mom, t)
            R.geod = geod
            try:
                with np.errstate(all="ignore"):
                    _, _, info = R.GPTregression(phi, ytr, 0.0476, I, r, Q, m, ew, eu, 0, 1, s,
                                                 max_steps=st + 1)
            finally:
                R.geod = orig
            npy[s] = int(info.get("bail_step", 0))
            norms[s] = ["%.3g" % max(trace[k * D:(k + 1) * D]) for k in range(len(trace) // D)]
        res[name] = dict(n=n, r=r, epsw=ew, epsU=eu, seeds=[int(x) for x in sd], cpp=cpp, numpy=npy,
                         max_expm_norm_per_step=norms)
        print(name, "C++", cpp, "numpy", npy, flush=True)
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
