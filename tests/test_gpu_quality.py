"""Quality parity at the BASELINE configurations, on the GPU.

* kin40k at the reference's own configuration (kin40kExperiment.jl:38-51,67-91: n = 150, r = 20,
  Q = 200, m = 50, εw = 1e-4, εU = 1e-7, random length scales 1 + 0.2·randn per sweep): the
  per-epoch test-RMSE curves of ten sweeps against the reference's recorded curve
  (testRMSE_kin40k.h5 -> tests/golden/ref_curves.npz).  Julia's RNG stream is not reproducible,
  so this is a band, not a per-value match: every surviving sweep within [0.85, 1.2]x the
  reference curve over epochs 5-30 and the median within 10 % at epoch 30.  Sweeps that take the
  geodesic NaN bail-out (GPT_SGLD.jl:422-424) are counted, as the reference's logs count
  `RMSE=NaN` runs (DataRecords.txt:61,71,75,91); at least 6 of 10 must survive.
* BASELINE config 1 (PowerPlantNoTensorExperiment.jl:5-42): full-theta SGLD on PowerPlant rows
  1-5000, n = 2000 features, m = 50, εθ = 1.1e-4, 100 epochs — the whole trajectory against the
  oracle (<= 1e-9 relative) and the script's "testRMSE with averaged pred" (epochs 60-100, :62-63)
  against the exact-GP ceiling 4.0056 (DataRecords.txt:19): within [3.95, 4.35].
* BASELINE config 5 at r = 20 (100k_movielensExperiment.jl): GPT_fullw_sideinfo for one epoch of
  fold 1 (80 000 ratings; the live configuration of :723-730 at r = 20) and an SGLD + Stiefel run,
  and GPT_fullw_gibbs (r² = 400 Kronecker design), against the oracle.

Converged quality against every curve the reference holds (the metric is
"steps/s + test RMSE"): kin40k over the reference's full 200 epochs (testRMSE_kin40k.h5),
PowerPlant config 2 over 200 epochs (testRMSE_PP.h5, vanilla and RMSprop), MovieLens
GPT_fullw_gibbs over 1 000 sweeps (fullWresults.h5).  Julia's RNG stream is not reproducible,
so these are statistical bands, stated in each test; the measured values are written to
gpurun_out/quality_r3.json.
"""
import json
import math
import os

import numpy as np
import pytest

from oracle import gpt_sgld_ref as R

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _record(key, val):
    """Append a measured quality value to gpurun_out/quality_r3.json (evidence for DESIGN.md)."""
    path = os.path.join(ROOT, "gpurun_out", "quality_r3.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    d = json.load(open(path)) if os.path.exists(path) else {}
    d[key] = val
    json.dump(d, open(path, "w"), indent=1)


def rel(a, b):
    a = np.asarray(a); b = np.asarray(b)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def stiefel_errors(sess, chains, n, r, D):
    """max_k |U_kᵀU_k − I| of the current U of each chain (device state, gathered).  The step
    kernels take geod's A = Uᵀmom as (M − Mᵀ)/2 from the projection's M = UᵀW (chain and wave
    engines) and the grid engine S from the same identity (GPT_SGLD.jl:19-22 replaced): both hold
    only on the manifold, so the invariant is asserted after the long runs that rely on them."""
    import torch
    dev = torch.device("cuda", 0)
    out = []
    for c in chains:
        w_t = torch.empty((1, sess.Q), dtype=torch.float64, device=dev)
        U_t = torch.empty((1, n * r * D), dtype=torch.float64, device=dev)
        sess.gather_state(c, 1, w_t, U_t)
        sess.sync()
        U = U_t.cpu().numpy().reshape((D, r, n)).transpose(2, 1, 0)      # Julia (n, r, D)
        out.append(max(float(np.abs(U[:, :, k].T @ U[:, :, k] - np.eye(r)).max())
                       for k in range(D)))
    return out


def _numpy_bail_steps(phi, y, sv, I, r, Q, m, epsw, epsU, cpp_steps):
    """The numpy restatement's (oracle/gpt_sgld_ref.py, GPT_SGLD.jl:345-448 line by line, numpy /
    LAPACK arithmetic) 1-based bail-out step of each seed the C++ restatement bails out, run a step
    past the C++ one (0: no bail-out by then)."""
    import torch
    if isinstance(phi, torch.Tensor):
        phi = np.asfortranarray(phi.cpu().numpy().transpose(2, 1, 0))
    out = {}
    for seed, st in cpp_steps.items():
        with np.errstate(all="ignore"):
            _, _, info = R.GPTregression(phi, y, sv, I, r, Q, m, epsw, epsU, 0, 1, seed,
                                         max_steps=st + 1)
        out[seed] = int(info.get("bail_step", 0))
    return out


def _assert_bail_steps(gpu, cpp, npy):
    """A diverging chain bails out where its geodesic's expm first holds a NaN (GPT_SGLD.jl:23-26).
    Its steps before that grow ‖t·[A −S; I A]‖₁ to 1e22-1e27, so expm! scales by 2^-70…2^-89 and
    squares 70-89 times: whether the squarings of a matrix whose exact exponential is bounded end in
    an overflow (a NaN, that step) or in finite values (U overflows in tmpU instead, and the NaN
    input bails out the next step) turns on the last bits of the Padé result, i.e. on the order of
    the floating-point sums.  The two CPU restatements (C++ loops; numpy/LAPACK) differ from each
    other by one step on some seeds for that reason (round 6: kin40k_ref seeds 1, 3, 19, 20, 21;
    profiles/r6_bail_steps.json), and the reference's own step would follow its BLAS.  So: the same
    chains bail out (asserted by the caller), each within one step of both restatements."""
    assert set(gpu) == set(cpp) == set(npy), (gpu, cpp, npy)
    for s in gpu:
        assert abs(gpu[s] - cpp[s]) <= 1 and abs(gpu[s] - npy[s]) <= 1, (s, gpu, cpp, npy)


def test_kin40k_reference_configuration_tracks_reference_curve():
    """kin40kExperiment.jl:38-91 over its full 200 epochs (10 sweeps, r = 20, n = 150) against
    testRMSE_kin40k.h5: bands in the assertions below."""
    import torch
    from bench import kin40k
    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import SGLDSession, feature_device, pred_device

    dev = torch.device("cuda", 0)
    n, D, r, Q, m, epochs, sweeps = 150, 8, 20, 200, 50, 200, 10
    Xtr, ytr, Xte, yte, ysd = kin40k(D)
    N, Nte = Xtr.shape[0], Xte.shape[0]
    nb = -(-N // m)
    I = G.samplenz(r, D, Q, 17)                                 # kin40kExperiment.jl:44
    scale = math.sqrt(n / Q ** (1.0 / D))                       # :45
    Z, b = G.feature_inputs(n, D, 17)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    Xtr_d, Xte_d, Z_d, b_d = tt(Xtr.T), tt(Xte.T), tt(Z.T), tt(b.T)
    phis, phites = [], []
    for j in range(1, sweeps + 1):                              # :67-72
        g = np.random.default_rng(j)
        ls = np.ones(D) + 0.2 * g.standard_normal(D)
        srbf = 1 + 0.2 * g.standard_normal()
        phis.append(feature_device(Xtr_d, tt(ls), srbf, scale, Z_d, b_d))
        phites.append(feature_device(Xte_d, tt(ls), srbf, scale, Z_d, b_d))
    sess = SGLDSession(phis, tt(ytr), I, r, Q, m, 1e-4, 1e-7, 0.0476, 0, epochs,
                       list(range(1, sweeps + 1)), store_every=nb, store=True)
    engine = sess.info()["engine"]
    sess.run(epochs * nb)
    sess.sync()
    alive_c = [c for c in range(sweeps) if sess.status(c) == 0]
    st_err = stiefel_errors(sess, alive_c, n, r, D)
    I0 = torch.from_numpy(np.asfortranarray(I - 1).ravel(order="F").astype(np.int32)).to(dev)
    yte_d = tt(yte)
    fh = torch.empty((epochs, Nte), dtype=torch.float64, device=dev)
    ref = np.load(os.path.join(ROOT, "tests", "golden", "ref_curves.npz"))["testRMSE_kin40k"]
    curves, alive = [], 0
    for c in range(sweeps):
        if sess.status(c) != 0:                               # NaN bail-out: zero stores
            continue
        alive += 1
        _, _, ws, Us, ns = sess.device_state(c)
        assert ns == epochs
        pred_device(ws, Us, I0, phites[c], n, D, Nte, r, Q, epochs, fh)
        err = fh - yte_d[None, :]
        curves.append((ysd * torch.sqrt((err * err).mean(dim=1))).cpu().numpy())   # :83
    sess.close()
    assert alive >= 6, "only %d of %d sweeps survived" % (alive, sweeps)
    # the manifold invariant behind the kernels' Gram identities, after 40 000 steps
    assert max(st_err) <= 1e-10, st_err
    curves = np.array(curves)
    final, last50 = curves[:, -1], curves[:, -50:].mean(axis=1)
    _record("kin40k_reference_config", dict(
        engine=engine, stiefel_err=st_err,
        sweeps=sweeps, survived=alive, epochs=epochs, final=final.tolist(),
        last50_curve_mean=last50.tolist(), median_final=float(np.median(final)),
        median_last50=float(np.median(last50)), ref_final=float(ref[-1]),
        ref_last50=float(ref[-50:].mean()), median_curve=np.median(curves, axis=0).tolist()))
    ratio = curves[:, 4:30] / ref[4:30][None, :]
    assert ratio.min() >= 0.85 and ratio.max() <= 1.2, (ratio.min(), ratio.max())
    assert abs(np.median(curves[:, 29]) / ref[29] - 1.0) <= 0.10
    assert np.all(curves[:, 29] < curves[:, 0])                 # every sweep learns
    # converged (kin40kExperiment.jl:74-90; the reference's 200-epoch curve ends at 0.2385, its
    # last 50 epochs average 0.2448).  Nothing here was tuned: the step sizes, hyper-parameter
    # draws and sweep seeds 1..10 are the script's own (:50-51, :67-72).  The band is the spread of
    # the sweeps themselves: the 8 surviving finals have s.d. 0.0075 (3.1 % of 0.2385; round 5,
    # gpurun_out/quality_r3.json), so the median's standard error is ≈ 1.25·3.1 %/√8 ≈ 1.4 % and
    # 3 % is about two of them; measured +0.3 % (final) and −2.4 % (last-50 mean).  Every surviving
    # sweep's final within ±10 % (three s.d.; measured 0.937-1.030).
    assert abs(np.median(final) / ref[-1] - 1.0) <= 0.03, (np.median(final), ref[-1])
    assert abs(np.median(last50) / ref[-50:].mean() - 1.0) <= 0.03, np.median(last50)
    assert np.all(final >= 0.9 * ref[-1]) and np.all(final <= 1.1 * ref[-1]), final


def test_kin40k_bench_shape_converged_quality():
    """The headline metric's "+ test RMSE" at its own shape (n = 500, D = 8, r = 5, Q = 200,
    m = 50, the bench's step pair, chain engine), 32 chains over the reference's 200 epochs.  No
    reference curve exists at r = 5; the bands come from the round-5 sweep (scripts/
    kin40k_step_sweep.py, profiles/r5c_kin40k_sweep*.json, other chain seeds): at r = 5 the median
    chain's epoch-200 RMSE sits at 0.344-0.36 for every stable (εw, εU) pair and for n = 150 as
    well as n = 500, while r = 20 at n = 150 reaches 0.238-0.243 at the same pairs (the reference:
    0.2385) — the gap to the reference is the rank's capacity, not mixing.
    Bail-outs (GPT_SGLD.jl:422-424) are pinned to the oracle, not banded: the chains that bail out
    over the 200 epochs are exactly the ones the C++ restatement (oracle/cpu, same Philox streams)
    bails out over its first two epochs, each at the same step.  Round 5 first ran this test with
    `bailed == 0` and it failed on MI355X (seed 5032); round 6 ran all 32 seeds through the
    restatement for the full 200 epochs (profiles/r6a_bail_probe.json, 76 s on 16 cores): it bails
    out seed 5032 alone, at its third step (the initial w draw sends |gradw| 2e6 -> 6e11 -> 1e25),
    exactly as the chain kernel does.  Bands on the survivors: the median chain's epoch-200 value
    and last-50 curve mean within [0.33, 0.38]; every chain below its own epoch-1 value; the
    ensemble of the last 50 epoch-end samples of the surviving chains at most 0.30."""
    import torch
    import bench
    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import SGLDSession, feature_device, pred_device
    from oracle import cpu_lib
    dev = torch.device("cuda", 0)
    _, D, m, ls, srbf, sv, _, n, r, epsw, epsU = bench.WORKLOADS["kin40k"]
    Q, epochs, chains = 200, 200, 32
    Xtr, ytr, Xte, yte, ysd = bench.kin40k(D)
    Nte = Xte.shape[0]
    nb = -(-Xtr.shape[0] // m)
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    scale = math.sqrt(n / Q ** (1.0 / D))
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    phi = feature_device(tt(Xtr.T), tt(np.array(ls)), srbf, scale, tt(Z.T), tt(b.T))
    phite = feature_device(tt(Xte.T), tt(np.array(ls)), srbf, scale, tt(Z.T), tt(b.T))
    seeds = list(range(5001, 5001 + chains))
    sess = SGLDSession(phi, tt(ytr), I, r, Q, m, epsw, epsU, sv, 0, epochs, seeds,
                       store_every=nb, store=True, engine="chain")
    sess.run(epochs * nb)
    sess.sync()
    # the oracle's bail-outs over two epochs, and the step each one bails out at
    phi_np = np.asfortranarray(phi.cpu().numpy().transpose(2, 1, 0))
    cpu = cpu_lib.GPTregression_chains(phi_np, ytr, sv, I, r, Q, m, epsw, epsU, 0, 2,
                                       np.array(seeds, dtype=np.uint64), threads=16)
    want = {seeds[c]: int(cpu["chain_steps"][c]) for c in range(chains) if cpu["status"][c]}
    np_steps = _numpy_bail_steps(phi_np, ytr, sv, I, r, Q, m, epsw, epsU, want)
    I0 = torch.from_numpy(np.asfortranarray(I - 1).ravel(order="F").astype(np.int32)).to(dev)
    yte_d = tt(yte)
    fh = torch.empty((epochs, Nte), dtype=torch.float64, device=dev)
    fsum = torch.zeros(Nte, dtype=torch.float64, device=dev)
    curves, got = [], []
    for c in range(chains):
        if sess.status(c) != 0:
            got.append(seeds[c])
            continue
        _, _, ws, Us, ns = sess.device_state(c)
        assert ns == epochs
        pred_device(ws, Us, I0, phite, n, D, Nte, r, Q, epochs, fh)
        err = fh - yte_d[None, :]
        curves.append((ysd * torch.sqrt((err * err).mean(dim=1))).cpu().numpy())
        fsum += fh[-50:].sum(dim=0)
    sess.close()
    bailed = len(got)
    assert sorted(want) == got, (got, want)
    # the bail-out step on the device: the last step with a gradient norm in the diagnostic rows
    bad = [c for c in range(chains) if seeds[c] in want]
    if bad:
        sd = SGLDSession(phi, tt(ytr), I, r, Q, m, epsw, epsU, sv, 0, 2, [seeds[c] for c in bad],
                         store=False, diag=True, engine="chain")
        sd.run(2 * nb)
        sd.sync()
        steps = {seeds[c]: sd.bail_step(i) for i, c in enumerate(bad)}
        sd.close()
        _assert_bail_steps(steps, want, np_steps)
    curves = np.array(curves)
    fmean = (fsum / (50 * len(curves))).cpu().numpy()
    ens = float(ysd * math.sqrt(np.mean((fmean - yte) ** 2)))
    final, last50 = curves[:, -1], curves[:, -50:].mean(axis=1)
    _record("kin40k_bench_shape", dict(chains=chains, bailed=bailed, epsw=epsw, epsU=epsU,
                                       bailed_seeds=got, oracle_bail_steps=want,
                                       numpy_bail_steps=np_steps,
                                       final=final.tolist(),
                                       last50_curve_mean=last50.tolist(), ensemble_rmse=ens,
                                       median_final=float(np.median(final)),
                                       median_last50=float(np.median(last50))))
    assert 0.33 <= np.median(final) <= 0.38, np.median(final)
    assert 0.33 <= np.median(last50) <= 0.38, np.median(last50)
    assert np.all(final < curves[:, 0])
    assert ens <= 0.30, ens


def test_gpnt_sgld_config1_powerplant_full_run():
    from bench import powerplant
    from gpt_amd import GPT_SGLD as G
    Xtr, ytr, Xte, yte, ysd = powerplant(4)                      # :5-26 (whitened, 5000 rows)
    n, m, eps, epochs = 2000, 50, 0.00011, 100
    phi = G.featureNotensor(Xtr, n, 1.4332, 1.0, 17)             # :32
    phite = G.featureNotensor(Xte, n, 1.4332, 1.0, 17)           # :33
    Z, b = R.seeded_feature_inputs(n, 4, 17)
    phi_o = R.featureNotensor(Xtr, 1.4332, 1.0, Z, b[:, 0])
    assert rel(phi, phi_o) < 1e-14                  # same argument bits; cos differs by ulps
    got = G.GPNT_SGLD(phi, ytr, 0.2299 ** 2, 1.0, m, eps, 0, 0, epochs, 1)    # :42
    want = R.GPNT_SGLD(phi, ytr, 0.2299 ** 2, 1.0, m, eps, 0, 0, epochs, 1)
    assert got.shape == want.shape == (n, epochs * 100)
    assert rel(got, want) < 1e-9
    nb = 100
    fh = np.stack([phite.T @ got[:, nb * e - 1] for e in range(1, epochs + 1)], axis=1)   # :53-56
    mean_fhat = fh[:, 59:100].mean(axis=1)                                               # :62
    rmse = ysd * math.sqrt(np.mean((mean_fhat - yte) ** 2))                              # :63
    assert 3.95 <= rmse <= 4.35, rmse


def _ml(ntr, nte, fold=1):
    from gpt_amd import movielens
    d = np.load(os.path.join(ROOT, "tests", "golden", "ml100k.npz"))
    tr, te, ud, md, mu, sd = movielens.fold(d, fold)
    return tr[:ntr], te[:nte], ud, md, mu, sd


@pytest.mark.parametrize("ntr,nte,m,ep,lang,stf,epsU", [
    (80000, 20000, 100, 1, False, False, 1e-6),          # live configuration of :723-730, r = 20
    (6000, 1500, 64, 2, True, True, 1e-4),               # SGLD + Stiefel
])
def test_movielens_sideinfo_r20_matches_oracle(ntr, nte, m, ep, lang, stf, epsU):
    from gpt_amd import movielens
    from oracle import movielens_ref as M
    tr, te, ud, md, mu, sd = _ml(ntr, nte)
    w0 = np.random.default_rng(17).standard_normal((20, 20))
    args = (tr, ud, md, te, 0.8, 0.1, 1.0, w0, m, 1e-4, epsU, 0.5, 0.25, 0.5, 0, ep, 17, mu, sd)
    got = movielens.GPT_fullw_sideinfo(*args, langevin=lang, stiefel=stf)
    want = M.GPT_fullw_sideinfo(*args, langevin=lang, stiefel=stf)
    for g, w_ in zip(got[:3], want[:3]):
        assert rel(g, w_) < 1e-8, rel(g, w_)
    assert np.abs(got[3] - want[3]).max() < 1e-8
    assert np.all(np.abs(got[5] - want[5]) <= 1e-9 * want[5])
    assert 0.8 < got[5][0] < 1.4                                 # rating-scale test RMSE


def test_movielens_gibbs_r20_matches_oracle():
    from gpt_amd import movielens
    from oracle import movielens_ref as M
    tr, te, ud, md, mu, sd = _ml(6000, 1500)
    w0 = np.random.default_rng(9).standard_normal((20, 20))
    args = (tr, ud, md, te, 0.8, 0.5, 1.0, w0, 0, 2, 1, 17, mu, sd)
    got = movielens.GPT_fullw_gibbs(*args)
    want = M.GPT_fullw_gibbs(*args)
    for g, w_ in zip(got[:3], want[:3]):
        assert rel(g, w_) < 1e-8, rel(g, w_)
    assert np.abs(got[3] - want[3]).max() < 1e-8
    assert np.all(np.abs(got[5] - want[5]) <= 1e-9 * want[5])


def _pp_curves(seeds, epochs, epsw, epsU, rms=None, m=256):
    """Per-epoch test-RMSE curves (original units) of independent PowerPlant chains at BASELINE
    config 2 (rows 1-5000 train / 4568 test, D = 4, n = 500, r = 5, Q = 200,
    ℓ = 1.4332, σ_RBF = 1, σ² = 0.2299², PowerPlantDataExperiment.jl:14-37), the epoch-end sample
    of every epoch predicted on the test rows (:196-209)."""
    import torch
    from bench import powerplant
    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import SGLDSession, feature_device, pred_device
    dev = torch.device("cuda", 0)
    n, D, r, Q = 500, 4, 5, 200
    Xtr, ytr, Xte, yte, ysd = powerplant(D)
    N, Nte = Xtr.shape[0], Xte.shape[0]
    nb = -(-N // m)
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    scale = math.sqrt(n / Q ** (1.0 / D))
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    ls = tt(np.full(D, 1.4332))
    phi = feature_device(tt(Xtr.T), ls, 1.0, scale, tt(Z.T), tt(b.T))
    phite = feature_device(tt(Xte.T), ls, 1.0, scale, tt(Z.T), tt(b.T))
    sess = SGLDSession(phi, tt(ytr), I, r, Q, m, epsw, epsU, 0.2299 ** 2, 0, epochs, seeds,
                       store_every=nb, store=True, engine="grid" if rms else "auto")
    if rms:
        sess.set_rmsprop(*rms)
    sess.run(epochs * nb)
    sess.sync()
    alive_c = [c for c in range(len(seeds)) if sess.status(c) == 0]
    st_err = stiefel_errors(sess, alive_c, n, r, D)
    assert max(st_err or [0.0]) <= 1e-10, st_err    # the manifold invariant after 4 000 steps
    I0 = torch.from_numpy(np.asfortranarray(I - 1).ravel(order="F").astype(np.int32)).to(dev)
    yte_d = tt(yte)
    fh = torch.empty((epochs, Nte), dtype=torch.float64, device=dev)
    curves, bailed = [], 0
    for c in range(len(seeds)):
        if sess.status(c) != 0:
            bailed += 1
            continue
        _, _, ws, Us, ns = sess.device_state(c)
        pred_device(ws, Us, I0, phite, n, D, Nte, r, Q, epochs, fh)
        err = fh - yte_d[None, :]
        curves.append((ysd * torch.sqrt((err * err).mean(dim=1))).cpu().numpy())
    sess.close()
    return np.array(curves), bailed


def test_powerplant_config2_converged_tracks_reference_curve():
    """BASELINE config 2 over 200 epochs against testRMSE_PP.h5 `testRMSE` (the vanilla SGLD
    block, PowerPlantDataExperiment.jl:196-209: 4.904 at epoch 1, 4.145 at epoch 200, last 50
    epochs 4.146).  The run that wrote the file is not recoverable from the script (it now reads
    maxepoch = 100, r = 20, m = 10; its commented step sizes εw = 1e-4, εU = 1e-7 at :59-60
    bail out or land 6 % high at n = 500, r = 5).  The step sizes are the round-4 oracle sweep's
    (scripts/pp_step_sweep.py, profiles/r4_pp_step_sweep*.json: 200 epochs, 8 chains per pair):
    the bench's old pair εw = 1e-5, εU = 1e-8 lands +3.1 % high, εU <= 3e-9 too little U motion
    (+4-8 %), εU >= 1e-7 too much noise (+3-6 %, bail-outs), the best stable pair εw = 5e-5,
    εU = 2e-8 +1.1 % — within the spread of the random-feature draw itself (feature seeds 17-21:
    +1.1 % to +2.2 % at one pair).  16 chains at that pair, with chain seeds 101-116: the sweep
    picked the pair on seeds 1-8, so these bands are not fitted to the chains they test (ADVICE
    r4).  Bands: at most one bail-out — the measured rate at this pair is 4 of 512 chains
    (profiles/r4pp_bench.json), so a 16-chain run sees one with probability ≈ 12 % and two with
    ≈ 0.6 %; the median chain's last-50-epoch curve mean within 2 % of 4.146 and its epoch-200
    value within 3 % of 4.145; every chain within [0.95, 1.08]x of the reference's epoch-200 value
    and below its own epoch-1 value."""
    ref = np.load(os.path.join(ROOT, "tests", "golden", "ref_curves.npz"))["testRMSE_PP"]
    curves, bailed = _pp_curves(list(range(101, 117)), 200, 5e-5, 2e-8)
    final, last50 = curves[:, -1], curves[:, -50:].mean(axis=1)
    _record("powerplant_config2", dict(chains=16, bailed=bailed, final=final.tolist(),
                                       last50_curve_mean=last50.tolist(),
                                       median_curve=np.median(curves, axis=0).tolist(),
                                       ref_final=float(ref[-1]), ref_last50=float(ref[-50:].mean())))
    assert bailed <= 1
    assert abs(np.median(last50) / ref[-50:].mean() - 1.0) <= 0.02, np.median(last50)
    assert abs(np.median(final) / ref[-1] - 1.0) <= 0.03, np.median(final)
    assert np.all(final >= 0.95 * ref[-1]) and np.all(final <= 1.08 * ref[-1]), final
    assert np.all(final < curves[:, 0])


def test_powerplant_rmsprop_converged_tracks_reference_curve():
    """GPT_SGLDERM_RMSprop at config 2 over 200 epochs against testRMSE_PP.h5 `testRMSE2` (the
    RMSprop block, PowerPlantDataExperiment.jl:211-224: 5.864 at epoch 1, 4.100 at epoch 200,
    last 50 epochs 4.134) with α = 0.99 (the script's commented value, :62), 8 chains.  The
    script's commented ε = 1e-4 (:61) and every ε down to 1e-7 diverge at this shape in the oracle
    restatement and on the GPU alike (RMSprop divides ε by √(moving average of ĝ²) + 1e-5, so the
    first steps are up to 1e5·ε; scripts/probe_rmsprop_pp.py, round 3); ε = 1e-8 is the largest
    that converges.  Bands as the vanilla test: median last-50 mean within 5 %, median final
    within 6 %, every chain within [0.9, 1.15]x of the reference's final value."""
    ref = np.load(os.path.join(ROOT, "tests", "golden", "ref_curves.npz"))["testRMSE2_PP"]
    curves, bailed = _pp_curves(list(range(1, 9)), 200, 1e-8, 1e-8, rms=(1e-8, 0.99))
    assert bailed == 0, "%d of 8 chains hit the geodesic NaN bail-out" % bailed
    final, last50 = curves[:, -1], curves[:, -50:].mean(axis=1)
    _record("powerplant_config2_rmsprop", dict(chains=8, bailed=bailed, final=final.tolist(),
                                               last50_curve_mean=last50.tolist(),
                                               median_curve=np.median(curves, axis=0).tolist(),
                                               ref_final=float(ref[-1]),
                                               ref_last50=float(ref[-50:].mean())))
    assert bailed == 0
    assert abs(np.median(last50) / ref[-50:].mean() - 1.0) <= 0.05, np.median(last50)
    assert abs(np.median(final) / ref[-1] - 1.0) <= 0.06, np.median(final)
    assert np.all(final >= 0.9 * ref[-1]) and np.all(final <= 1.15 * ref[-1]), final


def test_movielens_fullw_gibbs_converged_tracks_reference_curve():
    """GPT_fullw_gibbs (100k_movielensExperiment.jl:1032-1129) over 1 000 sweeps against
    fullWresults.h5 `testRMSE` (the running-average test RMSE, avg = true: 1.630 after the first
    kept sweep, 1.129 after 100, 0.9543 after 1 000, minimum 0.9531), the run of the parameter
    line at :743: r = 15, signal_var = 0.5, sigma_u = 0.5, sigma_w = ‖w_init‖_F / r, burnin = 15,
    maxepoch = 1000, param_seed = 10, avg = true (:752).  Not recoverable from the script:
    n_samples (commented out at :743; 1 here) and the ratings of that run (fold 1 u1.base /
    u1.test here).  The reference's early curve is far slower than this run's (1.63 -> 1.13 over
    the first 100 kept sweeps against 1.05 -> 0.925 here: its first samples were much worse, and
    the running average carries them), so the band is on the converged end only: the final
    running-average RMSE within 4 % of 0.9543 (measured round 3: 0.9234, -3.2 %), the minimum
    within 4 % of 0.9531, the curve decreasing from the first kept sweep to the last and flat
    over the last 500 sweeps (within 0.5 %), i.e. converged."""
    from gpt_amd import movielens
    ref = np.load(os.path.join(ROOT, "tests", "golden", "ref_curves.npz"))["fullW_testRMSE"]
    tr, te, ud, md, mu, sd = _ml(80000, 20000)
    r = 15
    w0 = np.random.default_rng(10).standard_normal((r, r))
    sigma_w = math.sqrt((w0 ** 2).sum()) / r
    got = movielens.GPT_fullw_gibbs(tr, ud, md, te, 0.5, 0.5, sigma_w, w0, 15, 1000, 1, 10, mu, sd,
                                    avg=True)
    test_rmse = np.asarray(got[5])
    _record("movielens_fullw_gibbs", dict(curve=test_rmse[::10].tolist(), final=float(test_rmse[-1]),
                                          min=float(test_rmse.min()), ref_final=float(ref[-1]),
                                          ref_min=float(ref.min()),
                                          ref_curve=ref[::10].tolist()))
    assert abs(test_rmse[-1] / ref[-1] - 1.0) <= 0.04, test_rmse[-1]
    assert abs(test_rmse.min() / ref.min() - 1.0) <= 0.04, test_rmse.min()
    assert test_rmse[-1] < test_rmse[0]
    tail = test_rmse[500:]
    assert tail.max() / tail.min() - 1.0 <= 0.005, (tail.min(), tail.max())


def test_kin40k_ref_bailouts_match_oracle():
    """The geodesic NaN bail-out (GPT_SGLD.jl:422-424) at kin40kExperiment.jl's own step pair
    (εw = 1e-4, εU = 1e-7; n = 150, r = 20, D = 8, Q = 200, m = 50, the wave engine): the chains
    that bail out in the first two epochs are exactly the ones the oracle's C++ restatement
    (oracle/cpu/gpt_sgld_cpu.cpp, same Philox streams and seeds) bails out — the bail-out rate is
    the reference algorithm's, not the engine's (7 of these 32 seeds at this pair on this data,
    the rate the bench's 256-chain run shows over 200 epochs: 32 of 256), each at the oracle's
    step; and every surviving chain's w and U after the 400 steps equal the restatement's within
    1e-8 (round 6 measured at most 4.7e-11 for w and 2.2e-12 for U, profiles/r6a_bail_probe.json).
    The diagnostic rows (diag = True) only add stores of the gradient norms."""
    import torch
    import bench
    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import SGLDSession
    from oracle import cpu_lib
    Xtr, ytr, _, _, _ = bench.kin40k(8)
    n, D, r, Q, m, epochs, C = 150, 8, 20, 200, 50, 2, 32
    I = G.samplenz(r, D, Q, 17)
    scale = math.sqrt(n / Q ** (1.0 / D))
    Z, b = G.feature_inputs(n, D, 17)
    phi = R.feature(Xtr, np.array(bench.KIN40K_LS), 1.0420, scale, Z, b)
    seeds = list(range(1, C + 1))
    cpu = cpu_lib.GPTregression_chains(phi, ytr, 0.0476, I, r, Q, m, 1e-4, 1e-7, 0, epochs,
                                       np.array(seeds, dtype=np.uint64), threads=16)
    want = sorted(int(s) for s, st in zip(seeds, cpu["status"]) if st != 0)
    dev = torch.device("cuda", 0)
    phi_d = torch.from_numpy(np.ascontiguousarray(np.transpose(phi, (2, 1, 0)))).to(dev)
    y_d = torch.from_numpy(np.ascontiguousarray(ytr)).to(dev)
    sess = SGLDSession(phi_d, y_d, I, r, Q, m, 1e-4, 1e-7, 0.0476, 0, epochs, seeds, store=False,
                       diag=True)
    assert sess.info()["engine"] == "wave"
    sess.run(epochs * sess.numbatches)
    sess.sync()
    got = sorted(s for c, s in enumerate(seeds) if sess.status(c) != 0)
    steps = {seeds[c]: sess.bail_step(c) for c in range(C) if sess.status(c) != 0}
    np_steps = _numpy_bail_steps(phi, ytr, 0.0476, I, r, Q, m, 1e-4, 1e-7,
                                 {seeds[c]: int(cpu["chain_steps"][c]) for c in range(C)
                                  if cpu["status"][c]})
    w_all = torch.empty((C, Q), dtype=torch.float64, device=dev)
    U_all = torch.empty((C, n * r * D), dtype=torch.float64, device=dev)
    sess.gather_state(0, C, w_all, U_all)
    sess.sync()
    sess.close()
    wn, Un = w_all.cpu().numpy(), U_all.cpu().numpy()
    errs = [(rel(wn[c], cpu["w"][:, c]), rel(Un[c], cpu["U"][..., c].ravel(order="F")))
            for c in range(C) if seeds[c] not in got and cpu["status"][c] == 0]
    want_steps = {seeds[c]: int(cpu["chain_steps"][c]) for c in range(C) if cpu["status"][c]}
    _record("kin40k_ref_bailouts", dict(chains=C, epochs=epochs, gpu=got, oracle=want,
                                        gpu_steps=steps, oracle_steps=want_steps,
                                        numpy_steps=np_steps,
                                        max_w_rel=max(e[0] for e in errs),
                                        max_U_rel=max(e[1] for e in errs)))
    assert len(want) >= 1, "the pair no longer bails out on this data: the test needs new seeds"
    assert got == want, (got, want)
    _assert_bail_steps(steps, want_steps, np_steps)
    assert len(errs) == C - len(want)
    assert max(e[0] for e in errs) <= 1e-8 and max(e[1] for e in errs) <= 1e-8, errs
