"""Round-6 probe: the bench shape's geodesic bail-outs and long-horizon states
on the GPU against the C++ restatement (oracle/cpu, test infrastructure).

  python scripts/bail_probe.py OUT.json

(a) kin40k bench shape (n = 500, D = 8, r = 5, Q = 200, m = 50, εw = 1e-5, εU = 1e-8, chain
    engine), seeds 5001..5032 over 200 epochs: which chains bail out and at which step, on the GPU
    (diagnostic rows: the last step with a gradient norm) and in the restatement (chain_steps).
(b) the same shape, seeds 1..256, chains 0 / 97 / 255 after K steps against the restatement.
(c) kin40kExperiment.jl's shape (n = 150, r = 20, εw = 1e-4, εU = 1e-7, wave engine), seeds 1..32
    over 2 epochs: bail-outs and the surviving chains' states against the restatement.
"""
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def main(out):
    import torch
    import bench
    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import SGLDSession, feature_device
    from oracle import cpu_lib
    dev = torch.device("cuda", 0)
    res = {}
    Xtr, ytr, _, _, _ = bench.kin40k(8)
    ls = np.array(bench.KIN40K_LS)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    N, D, Q, m = Xtr.shape[0], 8, 200, 50
    nb = -(-N // m)
    # ---- (a) + (b): bench shape
    n, r, ew, eu, sv = 500, 5, 1e-5, 1e-8, 0.0476
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    phi = feature_device(tt(Xtr.T), tt(ls), 1.0420, math.sqrt(n / Q ** (1.0 / D)), tt(Z.T), tt(b.T))
    y = tt(ytr)
    torch.cuda.synchronize()
    phi_np = np.asfortranarray(phi.cpu().numpy().transpose(2, 1, 0))
    seeds = list(range(5001, 5033))
    E = int(os.environ.get("PROBE_EPOCHS", "200"))
    t0 = time.time()
    s = SGLDSession(phi, y, I, r, Q, m, ew, eu, sv, 0, E, seeds, store=False, engine="chain")
    s.run(E * nb); s.sync()
    st_plain = [s.status(c) for c in range(len(seeds))]
    s.close()
    s = SGLDSession(phi, y, I, r, Q, m, ew, eu, sv, 0, E, seeds, store=False, diag=True,
                    engine="chain")
    s.run(E * nb); s.sync()
    gpu = []
    for c in range(len(seeds)):
        dg = np.zeros((1 + D, s.total_steps), order="F")
        import ctypes as C
        from gpt_amd import _lib
        stv = C.c_int32(0)
        _lib.check(_lib.lib().gpt_sgld_session_fetch(s._h, c, None, None,
                                                     dg.ctypes.data_as(_lib.P_D), C.byref(stv)))
        nz = np.flatnonzero(dg[0])
        gpu.append(dict(seed=seeds[c], status=int(stv.value), status_nodiag=st_plain[c],
                        last_step=int(nz[-1]) if nz.size else -1,
                        gradw_last=[float(x) for x in dg[0, max(0, nz[-1] - 3):nz[-1] + 1]]
                        if nz.size else []))
    s.close()
    res["a_gpu_s"] = time.time() - t0
    res["a_gpu"] = [g for g in gpu if g["status"] or g["status_nodiag"]]
    print("GPU bail-outs:", res["a_gpu"], flush=True)
    t0 = time.time()
    cpu = cpu_lib.GPTregression_chains(phi_np, ytr, sv, I, r, Q, m, ew, eu, 0, E,
                                       np.array(seeds, dtype=np.uint64), threads=16)
    res["a_cpu_s"] = time.time() - t0
    res["a_cpu"] = [dict(seed=seeds[c], status=int(cpu["status"][c]),
                         steps=int(cpu["chain_steps"][c])) for c in range(len(seeds))
                    if cpu["status"][c]]
    print("CPU bail-outs:", res["a_cpu"], "in %.1f s" % res["a_cpu_s"], flush=True)
    json.dump(res, open(out, "w"), indent=1)
    # ---- (b) long-horizon states, 256-chain launch
    probe = [0, 97, 255]
    res["b"] = {}
    for K in (200, 1000):
        s = SGLDSession(phi, y, I, r, Q, m, ew, eu, sv, 0, -(-K // nb), list(range(1, 257)),
                        store=False, engine="chain")
        s.run(K); s.sync()
        w_all = torch.empty((256, Q), dtype=torch.float64, device=dev)
        U_all = torch.empty((256, n * r * D), dtype=torch.float64, device=dev)
        s.gather_state(0, 256, w_all, U_all); s.sync()
        s.close()
        wn, Un = w_all.cpu().numpy(), U_all.cpu().numpy()
        o = cpu_lib.GPTregression_chains(phi_np, ytr, sv, I, r, Q, m, ew, eu, 0, -(-K // nb),
                                         np.array([c + 1 for c in probe], dtype=np.uint64),
                                         threads=3, max_steps=K)
        res["b"][K] = [dict(chain=c, w=rel(wn[c], o["w"][:, i]),
                            U=rel(Un[c], o["U"][..., i].ravel(order="F")))
                       for i, c in enumerate(probe)]
        print("K=%d" % K, res["b"][K], flush=True)
    json.dump(res, open(out, "w"), indent=1)
    # ---- (c) wave engine at kin40kExperiment.jl's shape
    n, r = 150, 20
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    from oracle import gpt_sgld_ref as R
    phi2 = R.feature(Xtr, ls, 1.0420, math.sqrt(n / Q ** (1.0 / D)), Z, b)
    seeds = list(range(1, 33))
    cpu = cpu_lib.GPTregression_chains(phi2, ytr, sv, I, r, Q, m, 1e-4, 1e-7, 0, 2,
                                       np.array(seeds, dtype=np.uint64), threads=16)
    phi_d = torch.from_numpy(np.ascontiguousarray(np.transpose(phi2, (2, 1, 0)))).to(dev)
    s = SGLDSession(phi_d, y, I, r, Q, m, 1e-4, 1e-7, sv, 0, 2, seeds, store=False)
    s.run(2 * nb); s.sync()
    w_all = torch.empty((32, Q), dtype=torch.float64, device=dev)
    U_all = torch.empty((32, n * r * D), dtype=torch.float64, device=dev)
    s.gather_state(0, 32, w_all, U_all); s.sync()
    stg = [s.status(c) for c in range(32)]
    s.close()
    wn, Un = w_all.cpu().numpy(), U_all.cpu().numpy()
    res["c"] = [dict(seed=seeds[c], gpu=stg[c], cpu=int(cpu["status"][c]),
                     cpu_steps=int(cpu["chain_steps"][c]),
                     w=rel(wn[c], cpu["w"][:, c]) if stg[c] == 0 and cpu["status"][c] == 0 else None,
                     U=rel(Un[c], cpu["U"][..., c].ravel(order="F"))
                     if stg[c] == 0 and cpu["status"][c] == 0 else None) for c in range(32)]
    print("wave:", res["c"], flush=True)
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
