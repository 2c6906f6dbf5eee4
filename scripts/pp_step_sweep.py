"""PowerPlant config 2 (D = 4, n = 500, r = 5, Q = 200, m = 256, ℓ = 1.4332,
σ² = 0.2299²) step-size sweep on the C++ oracle restatement (oracle/cpu, CPU only): per-epoch
test-RMSE curves of independent chains for each (εw, εU) pair, against testRMSE_PP.h5 (final
4.145, last-50 mean 4.146).  VERDICT r3 item 3: is the +1-3 % bias of the bench pair (1e-5, 1e-8)
a step-size effect?

    python scripts/pp_step_sweep.py [--epochs 200] [--chains 4] [--procs 8] [--out F.json]
"""
import argparse
import itertools
import json
import math
import os
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _setup(fseed=17):
    import bench
    from gpt_amd import GPT_SGLD as G
    from oracle import gpt_sgld_ref as R
    n, D, r, Q = 500, 4, 5, 200
    Xtr, ytr, Xte, yte, ysd = bench.powerplant(D)
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, fseed)
    scale = math.sqrt(n / Q ** (1.0 / D))
    phi = R.feature(Xtr, np.full(D, 1.4332), 1.0, scale, Z, b)
    phite = R.feature(Xte, np.full(D, 1.4332), 1.0, scale, Z, b)
    return dict(phi=phi, phite=phite, ytr=ytr, yte=yte, ysd=ysd, I=I, n=n, D=D, r=r, Q=Q)


_P = {}


def run_one(job):
    from oracle import cpu_lib
    epsw, epsU, seed, epochs, m, fseed = job
    if fseed not in _P:
        _P[fseed] = _setup(fseed)
    p = _P[fseed]
    N = p["phi"].shape[2]
    nb = -(-N // m)
    o = cpu_lib.GPTregression_chains(p["phi"], p["ytr"], 0.2299 ** 2, p["I"], p["r"], p["Q"], m,
                                     epsw, epsU, 0, epochs, [seed], threads=1, store_every=nb,
                                     stores=True)
    if o["status"][0] != 0:
        return dict(epsw=epsw, epsU=epsU, seed=seed, fseed=fseed, bailed=True)
    f, _ = cpu_lib.pred(o["w_store"], o["U_store"], p["I"], p["phite"], threads=1)
    curve = p["ysd"] * np.sqrt(((f - p["yte"][None, :]) ** 2).mean(axis=1))
    return dict(epsw=epsw, epsU=epsU, seed=seed, fseed=fseed, bailed=False, final=float(curve[-1]),
                last50=float(curve[-50:].mean()), first=float(curve[0]),
                curve=curve[::10].tolist())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=200)
    ap.add_argument("--chains", type=int, default=4)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--epsw", default="1e-5,2e-5,5e-5,1e-4")
    ap.add_argument("--epsU", default="1e-8,1e-7")
    ap.add_argument("--fseeds", default="17", help="feature (Z, b) seeds: the RFF draw")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    ew = [float(x) for x in args.epsw.split(",")]
    eu = [float(x) for x in args.epsU.split(",")]
    fs = [int(x) for x in args.fseeds.split(",")]
    jobs = [(a, b, s, args.epochs, args.m, f) for a, b in itertools.product(ew, eu) for f in fs
            for s in range(1, args.chains + 1)]
    with Pool(args.procs) as pool:
        res = pool.map(run_one, jobs)
    ref = np.load(os.path.join(ROOT, "tests", "golden", "ref_curves.npz"))["testRMSE_PP"]
    summary = []
    for a, b, f in itertools.product(ew, eu, fs):
        rs = [x for x in res if x["epsw"] == a and x["epsU"] == b and x["fseed"] == f]
        ok = [x for x in rs if not x["bailed"]]
        d = dict(epsw=a, epsU=b, fseed=f, chains=len(rs), bailed=len(rs) - len(ok))
        if ok:
            d.update(median_final=float(np.median([x["final"] for x in ok])),
                     median_last50=float(np.median([x["last50"] for x in ok])),
                     last50=[round(x["last50"], 4) for x in ok])
            d["last50_vs_ref"] = d["median_last50"] / float(ref[-50:].mean()) - 1.0
        summary.append(d)
        print(json.dumps(d), flush=True)
    if args.out:
        json.dump(dict(reference=dict(final=float(ref[-1]), last50=float(ref[-50:].mean())),
                       summary=summary, runs=res), open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
