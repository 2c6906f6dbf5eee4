"""GPU parity: libgptsgld.so (HIP, gfx950) against the CPU oracle on identical inputs, seeds,
Philox streams and permutations.

Tolerances (fp64 path; the GPU sums in a different order and uses leave-one-out products
instead of computeU_phi's division, GPT_SGLD.jl:253):
  features                       max |Δ| <= 1e-14·|c|  (same argument bits; libm cos differs by a few ulp)
  pred / fhat                    max |Δ| <= 1e-12·max|f|
  sampler trajectories           max |Δ| <= 1e-8·max|x| over every stored w and U sample
  per-step gradient norms        relative <= 1e-9
  test RMSE                      relative <= 1e-10
"""
import math

import numpy as np
import pytest

from oracle import gpt_sgld_ref as R

pytestmark = pytest.mark.gpu


def G():
    from gpt_amd import GPT_SGLD
    return GPT_SGLD


def rel(a, b):
    a = np.asarray(a); b = np.asarray(b)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def make_problem(n, D, N, r, Q, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((N, D))
    Z = rng.standard_normal((n, D))
    b = 2 * np.pi * rng.random((n, D))
    ls = 1.0 + 0.2 * rng.standard_normal(D)
    scale = math.sqrt(n / Q ** (1.0 / D))
    phi = R.feature(X, ls, 1.0, scale, Z, b)
    I = R.samplenz(r, D, Q, seed + 1)
    w, U = R.init_state(n, r, D, Q, seed + 2)
    y = R.pred(w, U, I, phi) + 0.05 * rng.standard_normal(N)
    return dict(X=X, Z=Z, b=b, ls=ls, scale=scale, phi=phi, I=I, y=y)


# ----------------------------------------------------------------------------- features
def test_feature_matches_oracle():
    rng = np.random.default_rng(1)
    N, D, n = 300, 5, 64
    X = rng.standard_normal((N, D)); Z = rng.standard_normal((n, D)); b = 2 * np.pi * rng.random((n, D))
    ls = 1 + 0.2 * rng.standard_normal(D)
    got = G().feature(X, ls, 1.3, 2.0, Z, b)
    want = R.feature(X, ls, 1.3, 2.0, Z, b)
    assert got.shape == (n, D, N)
    assert np.abs(got - want).max() <= 1e-14 * np.abs(want).max()


def test_feature_seeded_generation_c():
    rng = np.random.default_rng(2)
    X = rng.standard_normal((50, 4))
    got = G().feature(X, 20, [1.2, 1.1, 0.9, 1.4], 1.05, 17, 3.0)
    Z, b = R.seeded_feature_inputs(20, 4, 17)
    want = R.feature(X, [1.2, 1.1, 0.9, 1.4], 1.05, 3.0, Z, b)
    assert rel(got, want) < 2e-15


def test_feature_generation_a():
    """feature(X,n,length_scale,seed) of GPT_SGLD_p.jl:40-54: b = randn, Z/ℓ, sqrt(2/n), no σ."""
    rng = np.random.default_rng(4)
    X = rng.standard_normal((70, 3))
    got = G().feature(X, 24, 1.3, 11)
    want = R.feature_gen_a(X, 24, 1.3, 11)
    assert got.shape == (24, 3, 70)
    assert np.abs(got - want).max() <= 1e-14 * np.abs(want).max()


@pytest.mark.parametrize("N,seed,epochs", [(1, 3, 2), (2, 5, 3), (97, 1, 4), (5000, 17, 3),
                                           (10000, 1001, 3), (13632, 2, 2), (20011, 7, 2)])
def test_epoch_orders_match_oracle(N, seed, epochs):
    """Device epoch orders (order.hip: parallel Fisher–Yates by reservations, LDS up to 13 632
    rows, global workspace beyond) == the oracle's sequential randperm composed per epoch
    (GPT_SGLD.jl:373-374), bit for bit."""
    from oracle import philox as px
    got = G().epoch_orders(N, seed, epochs)
    order = np.arange(N)
    for e in range(epochs):
        order = order[px.randperm(N, seed, e)]
        assert np.array_equal(got[:, e], order), "epoch %d" % e


def test_feature_notensor_matches_oracle():
    rng = np.random.default_rng(3)
    N, D, n = 200, 4, 96
    X = rng.standard_normal((N, D)); Z = rng.standard_normal((n, D)); b = 2 * np.pi * rng.random(n)
    got = G().featureNotensor(X, 1.4332, 1.0, Z, b)
    want = R.featureNotensor(X, 1.4332, 1.0, Z, b)
    assert rel(got, want) < 2e-15


# ----------------------------------------------------------------------------- prediction
@pytest.mark.parametrize("tag,expected", [("5D", 0.03125), ("10D", 0.0258)])
def test_pred_on_reference_fixture(tag, expected):
    from conftest import load_golden
    d = load_golden("tensor_synth_%s.npz" % tag)
    f = G().pred(d["w"], d["U"], d["I"], d["phi"])
    want = R.pred(d["w"], d["U"], d["I"], d["phi"])
    assert rel(f, want) < 1e-12
    assert abs(np.std(d["y3"] - f) - expected) < 5e-4


def test_pred_mean_and_rmse():
    p = make_problem(40, 4, 300, 3, 20, seed=5)
    rng = np.random.default_rng(9)
    S = 4
    ws = rng.standard_normal((20, S))
    Us = np.stack([R.init_state(40, 3, 4, 20, 100 + s)[1] for s in range(S)], axis=3)
    mean, rm = G().pred_mean(ws, Us, p["I"], p["phi"], p["y"], scale=2.5)
    want = R.posterior_mean_pred(ws, Us, p["I"], p["phi"])
    assert rel(mean, want) < 1e-12
    assert rm == pytest.approx(R.rmse(p["y"], want, 2.5), rel=1e-10)


@pytest.mark.parametrize("n,D,Nt,r,Q,S", [
    (41, 3, 200, 5, 30, 30),       # odd n (8-B operand loads), 3 c-tiles of the S·r GEMM, ragged rows
    (150, 8, 130, 20, 200, 4),     # the reference's kin40k rank (r = 20, n = 150)
    (500, 8, 700, 5, 200, 40),     # bench shape, 4 c-tiles, 11 row tiles
])
def test_pred_stacked_samples_mfma(n, D, Nt, r, Q, S):
    """pred over S stacked samples (fp64-MFMA phidotU GEMM M = S·r, N = Ntest, K = n, then the
    V-phase) against the oracle's pred of every sample."""
    rng = np.random.default_rng(n + S)
    X = rng.standard_normal((Nt, D)); Z = rng.standard_normal((n, D)); b = 2 * np.pi * rng.random((n, D))
    phi = R.feature(X, 1.0 + 0.1 * rng.random(D), 1.0, math.sqrt(n / Q ** (1.0 / D)), Z, b)
    I = R.samplenz(r, D, Q, 5)
    ws = rng.standard_normal((Q, S))
    Us = np.stack([R.init_state(n, r, D, Q, 50 + s)[1] for s in range(S)], axis=3)
    yt = rng.standard_normal(Nt)
    mean, rm = G().pred_mean(ws, Us.reshape((n, r, D * S), order="F"), I, phi, yt, scale=1.3)
    f = np.stack([R.pred(ws[:, s], Us[..., s], I, phi) for s in range(S)])
    assert rel(mean, f.mean(axis=0)) < 1e-12
    assert rm == pytest.approx(R.rmse(yt, f.mean(axis=0), 1.3), rel=1e-10)
    f1 = G().pred(ws[:, S - 1], Us[..., S - 1], I, phi)
    assert rel(f1, f[S - 1]) < 1e-12


@pytest.mark.parametrize("D", [3, 8])
def test_pred_vphase_pairs_equals_rows(D, monkeypatch):
    """The pair-table V-phase (default, r <= 5) and the lanes-as-rows V-phase
    (GPTSGLD_PRED_VPHASE=rows) give the same predictions up to the association of the D factors."""
    n, Nt, r, Q, S = 64, 777, 5, 60, 6
    rng = np.random.default_rng(D)
    X = rng.standard_normal((Nt, D)); Z = rng.standard_normal((n, D)); b = 2 * np.pi * rng.random((n, D))
    phi = R.feature(X, 1.0 + 0.1 * rng.random(D), 1.0, math.sqrt(n / Q ** (1.0 / D)), Z, b)
    I = R.samplenz(r, D, Q, 7)
    ws = rng.standard_normal((Q, S))
    Us = np.stack([R.init_state(n, r, D, Q, 70 + s)[1] for s in range(S)], axis=3)
    yt = rng.standard_normal(Nt)
    Uf = Us.reshape((n, r, D * S), order="F")
    mean_p, _ = G().pred_mean(ws, Uf, I, phi, yt)
    monkeypatch.setenv("GPTSGLD_PRED_VPHASE", "rows")
    mean_r, _ = G().pred_mean(ws, Uf, I, phi, yt)
    monkeypatch.delenv("GPTSGLD_PRED_VPHASE")
    assert rel(mean_p, mean_r) < 1e-13
    f = np.stack([R.pred(ws[:, s], Us[..., s], I, phi) for s in range(S)])
    assert rel(mean_p, f.mean(axis=0)) < 1e-12


# ----------------------------------------------------------------------------- sampler
CASES = {
    # name: (n, D, N, r, Q, m, burnin, maxepoch, store_every, langevin, stiefel)
    "small": (16, 3, 40, 2, 6, 8, 1, 2, 1, True, True),
    "ragged_thin": (24, 4, 37, 3, 10, 8, 0, 3, 5, True, True),
    "sgd": (16, 3, 40, 2, 6, 8, 0, 2, 1, False, True),
    "euclid": (16, 3, 40, 2, 6, 8, 0, 2, 1, True, False),
    "kin40k_shape": (500, 8, 200, 5, 200, 50, 0, 1, 1, True, True),
    "wide_batch": (64, 4, 300, 4, 30, 100, 0, 1, 1, True, True),
    "rank10": (100, 4, 120, 10, 60, 30, 0, 1, 1, True, True),
    "ref_kin40k_rank20": (150, 8, 100, 20, 200, 50, 0, 1, 1, True, True),
    "batch256": (96, 4, 600, 5, 80, 256, 0, 1, 1, True, True),
    "powerplant_shape": (500, 4, 600, 5, 200, 256, 0, 2, 1, True, True),   # D <= 4 build, J = 8, 2 V tasks/wave
    # odd shapes of the chain engine at D >= 5: half-filled 64-row blocks, ragged batches,
    # the n = 512 / Q = 256 maxima (a 64-member run), thinning after burn-in
    "c2_d5_half128": (200, 5, 90, 3, 70, 20, 0, 2, 1, True, True),      # J2 = 2, ragged last batch
    "c2_n258_thin": (258, 6, 60, 4, 130, 15, 1, 2, 3, True, True),      # 2 rows in the second half
    "c2_n512_q256": (512, 8, 70, 5, 256, 33, 0, 1, 1, True, True),      # full halves, 8 V tasks, odd m
    "c2_r2_d7": (300, 7, 64, 2, 100, 16, 0, 2, 2, True, True),
    # edge shapes: a last batch of one row (an odd row group), one input dimension, odd n with
    # one 64-row block (4-B row staging), odd n past one block (the chain engine declines: grid)
    "last_row_alone": (24, 2, 41, 2, 4, 8, 0, 2, 1, True, True),
    "d1": (32, 1, 30, 3, 3, 7, 0, 2, 1, True, True),
    "n17_odd": (17, 3, 40, 2, 6, 8, 0, 2, 1, True, True),
    "n101_odd": (101, 2, 33, 3, 9, 10, 0, 2, 1, True, True),
    # more than 8 input dimensions: the grid engine's lane-per-q V-phase tile (the column-lane
    # form and the chain engine stop at D = 8), split into slices of 7 / 8 rows
    "d12": (40, 12, 80, 2, 24, 15, 0, 2, 1, True, True),
    # wave engine shapes (wave.hip, r > 5): one 64-row block, ragged thinned batches after burn-in,
    # four row blocks (J = 4), odd n with odd 2r, the 2r = 32 one-pass solve at the m = 64 maximum,
    # 12 input dimensions at r = 20
    "w_r6_d3": (40, 3, 70, 6, 30, 16, 0, 2, 1, True, True),
    "w_r8_thin": (96, 4, 55, 8, 50, 12, 1, 2, 3, True, True),
    "w_r12_n200": (200, 5, 64, 12, 100, 32, 0, 1, 1, True, True),
    "w_r15_odd": (77, 6, 40, 15, 90, 9, 0, 2, 1, True, True),
    "w_r16_m64": (130, 4, 130, 16, 120, 64, 0, 1, 1, True, True),
    "w_r20_d12": (64, 12, 30, 20, 60, 10, 0, 1, 1, True, True),
}


def _chain_ok(n, D, r, lang, stf):
    """Shapes the chain engine (chain.hip) takes; the grid engine (sgld.hip) takes all."""
    return lang and stf and D <= 8 and r <= 5 and n <= 512 and (n <= 64 or n % 2 == 0)


def _shape(name):
    return [CASES[name][i] for i in (0, 1, 3, 9, 10)]


WAVE_RANKS = (6, 8, 10, 12, 15, 16, 20)


def _wave_ok(name):
    """Shapes the wave engine (wave.hip) takes: SGLD + Stiefel at an instantiated r > 5,
    3r <= n <= 256, m <= 64."""
    n, D, N, r, Q, m, burnin, maxepoch, se, lang, stf = CASES[name]
    return lang and stf and r in WAVE_RANKS and 3 * r <= n <= 256 and m <= 64


ENGINE_CASES = [(name, eng) for name in CASES for eng in ("grid", "chain", "wave")
                if (eng == "grid" and not name.startswith("w_"))
                or (eng == "chain" and _chain_ok(*_shape(name)))
                or (eng == "wave" and _wave_ok(name))]


@pytest.mark.parametrize("name,engine", ENGINE_CASES)
def test_sampler_trajectory_matches_oracle(name, engine):
    n, D, N, r, Q, m, burnin, maxepoch, se, lang, stf = CASES[name]
    p = make_problem(n, D, N, r, Q, seed=11)
    kw = dict(langevin=lang, stiefel=stf, store_every=se, engine=engine)
    epsw, epsU, sv, seed = 1e-4, 1e-6, 0.05, 23
    ws, Us, dg = G().GPTregression(p["phi"], p["y"], sv, p["I"], r, Q, m, epsw, epsU, burnin,
                                   maxepoch, seed, diag=True, **kw)
    kw.pop("engine")
    wo, Uo, info = R.GPTregression(p["phi"], p["y"], sv, p["I"], r, Q, m, epsw, epsU, burnin,
                                   maxepoch, seed, record=True, **kw)
    assert info["status"] == 0
    assert ws.shape == wo.shape and Us.shape == Uo.shape
    assert rel(ws, wo) < 1e-8, rel(ws, wo)
    assert rel(Us, Uo) < 1e-8, rel(Us, Uo)
    gw = np.array(info["gradw_norm"]); gU = np.array(info["gradU_norm"]).T
    assert rel(dg[0], gw) < 1e-9
    assert rel(dg[1:], gU) < 1e-9
    if stf:
        for s in range(Us.shape[3]):
            for k in range(D):
                Uk = Us[:, :, k, s]
                assert np.abs(Uk.T @ Uk - np.eye(r)).max() < 1e-10


@pytest.mark.parametrize("name", [c for c, e in ENGINE_CASES if e == "chain"])
def test_chain_trajectory_without_diagnostics(name):
    """The chain engine with no per-step gradient-norm buffer (the diag writes compiled in but
    skipped, the production configuration): same samples as the oracle."""
    n, D, N, r, Q, m, burnin, maxepoch, se, lang, stf = CASES[name]
    p = make_problem(n, D, N, r, Q, seed=11)
    epsw, epsU, sv, seed = 1e-4, 1e-6, 0.05, 23
    ws, Us = G().GPTregression(p["phi"], p["y"], sv, p["I"], r, Q, m, epsw, epsU, burnin,
                               maxepoch, seed, langevin=lang, stiefel=stf, store_every=se,
                               engine="chain")
    wo, Uo, info = R.GPTregression(p["phi"], p["y"], sv, p["I"], r, Q, m, epsw, epsU, burnin,
                                   maxepoch, seed, langevin=lang, stiefel=stf, store_every=se)
    assert info["status"] == 0
    assert rel(ws, wo) < 1e-8, rel(ws, wo)
    assert rel(Us, Uo) < 1e-8, rel(Us, Uo)


RMS_CASES = {
    # name: (n, D, N, r, Q, m, burnin, maxepoch, epsilon)
    "small": (16, 3, 40, 2, 6, 8, 1, 2, 1e-5),
    "ragged": (24, 4, 37, 3, 10, 8, 0, 3, 1e-5),
    # At ε = 1e-5 this shape is ill-conditioned in the oracle itself: a 1e-15 relative
    # perturbation of U_init grows to 8e-8 in three steps (one RMSprop geodesic step of
    # t = √mean(εU) ≈ 0.06 over momenta of norm ≈ 20).  ε = 1e-6 keeps it at 2e-12.
    "kin40k_shape": (500, 8, 150, 5, 200, 50, 0, 1, 1e-6),
}


@pytest.mark.parametrize("name", list(RMS_CASES))
def test_rmsprop_trajectory_matches_oracle(name):
    """GPT_SGLDERM_RMSprop (GPT_SGLD.jl:1121-1237) against the oracle restatement."""
    n, D, N, r, Q, m, burnin, maxepoch, eps = RMS_CASES[name]
    p = make_problem(n, D, N, r, Q, seed=13)
    alpha, sv, seed = 0.9, 0.05, 29
    ws, Us, dg = G().GPT_SGLDERM_RMSprop(p["phi"], p["y"], sv, p["I"], r, Q, m, eps, alpha, burnin,
                                         maxepoch, seed, diag=True)
    wo, Uo, info = R.GPT_SGLDERM_RMSprop(p["phi"], p["y"], sv, p["I"], r, Q, m, eps, alpha, burnin,
                                         maxepoch, seed, record=True)
    assert info["status"] == 0
    assert rel(ws, wo) < 1e-8, rel(ws, wo)
    assert rel(Us, Uo) < 1e-8, rel(Us, Uo)
    assert rel(dg[0], np.array(info["gradw_norm"])) < 1e-9
    assert rel(dg[1:], np.array(info["gradU_norm"]).T) < 1e-9


def test_rmsprop_set_after_prepare_runs_rmsprop_steps():
    """Graphs prepared before set_rmsprop captured plain SGLD steps; set_rmsprop drops them, so
    the run that follows takes RMSprop steps (the stale graphs used to be replayed)."""
    import torch
    from gpt_amd.session import SGLDSession
    n, D, N, r, Q, m, burnin, maxepoch, eps = RMS_CASES["small"]
    p = make_problem(n, D, N, r, Q, seed=13)
    alpha, sv, seed = 0.9, 0.05, 29
    dev = torch.device("cuda", 0)
    phi = torch.from_numpy(np.ascontiguousarray(np.asarray(p["phi"]).transpose(2, 1, 0))).to(dev)
    y = torch.from_numpy(np.ascontiguousarray(np.asarray(p["y"], dtype=np.float64))).to(dev)
    s = SGLDSession(phi, y, p["I"], r, Q, m, eps, eps, sv, burnin, maxepoch, [seed],
                    engine="grid")
    s.prepare(s.total_steps)
    s.set_rmsprop(eps, alpha)
    s.run(s.total_steps)
    ws, Us, st = s.fetch(0)
    s.close()
    wo, Uo, info = R.GPT_SGLDERM_RMSprop(p["phi"], p["y"], sv, p["I"], r, Q, m, eps, alpha, burnin,
                                         maxepoch, seed)
    assert st == 0 and info["status"] == 0
    assert rel(ws, wo) < 1e-8, rel(ws, wo)
    assert rel(Us, Uo) < 1e-8, rel(Us, Uo)


def test_pred_mean_x_fused_features():
    """Fused feature+pred (§8(f) per-epoch evaluation) equals pred_mean over materialised
    features, and the per-sample RMSE curve matches the oracle."""
    rng = np.random.default_rng(21)
    n, D, Nt, r, Q, S = 40, 4, 333, 3, 20, 3
    X = rng.standard_normal((Nt, D)); Z = rng.standard_normal((n, D)); b = 2 * np.pi * rng.random((n, D))
    ls = 1 + 0.2 * rng.standard_normal(D)
    I = R.samplenz(r, D, Q, 3)
    ws = rng.standard_normal((Q, S))
    Us = np.stack([R.init_state(n, r, D, Q, 10 + s)[1] for s in range(S)], axis=3)
    yt = rng.standard_normal(Nt)
    mean, rm, srm = G().pred_mean_x(ws, Us.reshape((n, r, D * S), order="F"), I, X, yt, ls, 1.1,
                                    2.0, Z, b, scale=1.7)
    phi = G().feature(X, ls, 1.1, 2.0, Z, b)
    mean2, rm2 = G().pred_mean(ws, Us.reshape((n, r, D * S), order="F"), I, phi, yt, scale=1.7)
    # pred_mean runs the stacked-sample MFMA GEMM (another summation order than the fused tile)
    assert rel(mean, mean2) < 1e-13 and abs(rm - rm2) <= 1e-13 * rm2
    phio = R.feature(X, ls, 1.1, 2.0, Z, b)
    f = np.stack([R.pred(ws[:, s], Us[..., s], I, phio) for s in range(S)])
    assert rel(mean, f.mean(axis=0)) < 1e-12
    want = 1.7 * np.sqrt(((f - yt) ** 2).mean(axis=1))
    assert np.abs(srm - want).max() <= 1e-12 * want.max()


CLS_CASES = {
    # name: (n, D, N, r, Q, m, C, burnin, maxepoch, langevin, stiefel)
    "binary_sgld_stiefel": (16, 4, 60, 3, 20, 10, 2, 0, 2, True, True),
    "three_class_ragged": (24, 3, 45, 2, 8, 16, 3, 1, 1, True, True),
    "binary_sgd_stiefel": (16, 4, 60, 3, 20, 10, 2, 0, 1, False, True),
    "binary_sgld_euclid": (16, 4, 60, 3, 20, 10, 2, 0, 1, True, False),
    "binary_sgd_euclid": (16, 4, 60, 3, 20, 10, 2, 0, 1, False, False),
}


@pytest.mark.parametrize("name", list(CLS_CASES))
def test_classification_matches_oracle(name):
    """GPTclassification (GPT_SGLD.jl:452-680): softmax residuals over the classes, two moves
    per step, all four langevin/stiefel variants of the second move."""
    n, D, N, r, Q, m, ncls, burnin, maxepoch, lang, stf = CLS_CASES[name]
    p = make_problem(n, D, N, r, Q, seed=23)
    f = p["y"] - np.median(p["y"])
    y = (1 + np.clip(np.floor((f - f.min()) / (np.ptp(f) + 1e-12) * ncls), 0, ncls - 1)).astype(float)
    assert int(y.max()) == ncls and int(y.min()) == 1
    epsw, epsU, seed = 1e-4, 1e-6, 41
    ws, Us, dg = G().GPTclassification(p["phi"], y, p["I"], r, Q, m, epsw, epsU, burnin, maxepoch,
                                       seed, langevin=lang, stiefel=stf, diag=True)
    wo, Uo, info = R.GPTclassification(p["phi"], y, p["I"], r, Q, m, epsw, epsU, burnin, maxepoch,
                                       seed, langevin=lang, stiefel=stf, record=True)
    assert info["status"] == 0
    assert ws.shape == (Q, ncls, maxepoch * (-(-N // m)))
    assert rel(ws, wo) < 1e-8, rel(ws, wo)
    assert rel(Us, Uo) < 1e-8, rel(Us, Uo)
    gw = np.array(info["gradw_norm"])                  # (steps, C)
    gu = np.array(info["gradU_norm"])                  # (steps, C, D)
    assert rel(dg[0], gw) < 1e-9
    assert rel(np.moveaxis(dg[1:], 0, 2), gu) < 1e-9


GMC_CASES = {
    # name: (n, D, N, r, Q, L, burnin, maxepoch, signal_var, eps)
    "accepting": (8, 3, 40, 2, 5, 5, 1, 5, 1.0, 1e-2),
    "rejecting": (8, 3, 40, 2, 5, 5, 1, 7, 1.0, 1e-1),   # epochs 1, 4, 6, 7 rejected (w restored)
    "powerplant_like": (20, 4, 300, 5, 40, 4, 0, 2, 1.0, 1e-3),
}


def _gmc_problem(n, D, N, r, Q):
    rng = np.random.default_rng(3)
    phi = rng.standard_normal((n, D, N)) * 0.5
    I = R.samplenz(r, D, Q, 1)
    w, U = R.init_state(n, r, D, Q, 3)
    return phi, R.pred(w, U, I, phi) + 0.1 * rng.standard_normal(N), I


@pytest.mark.parametrize("name", list(GMC_CASES))
def test_gmc_matches_oracle(name):
    """GPT_GMC (GPT_SGLD.jl:684-805): full-batch leapfrog with geodboth, Metropolis step."""
    n, D, N, r, Q, L, burnin, maxepoch, sv, eps = GMC_CASES[name]
    phi, y, I = _gmc_problem(n, D, N, r, Q)
    ws, Us, acc = G().GPT_GMC(phi, y, sv, I, r, Q, eps, eps, burnin, maxepoch, L, 7)
    wo, Uo, acco = R.GPT_GMC(phi, y, sv, I, r, Q, eps, eps, burnin, maxepoch, L, 7)
    assert rel(ws, wo) < 1e-8, rel(ws, wo)
    assert rel(Us, Uo) < 1e-8, rel(Us, Uo)
    assert np.all(np.abs(acc - acco) <= 1e-7 * np.maximum(np.abs(acco), 1e-3))


def test_gmc_geodesic_nan_bailout():
    """A diverging geodesic returns zero stores and NaN acceptance probabilities (:757)."""
    phi, y, I = _gmc_problem(8, 3, 40, 2, 5)
    ws, Us, acc = G().GPT_GMC(phi, y, 0.1, I, 2, 5, 0.3, 0.3, 1, 3, 5, 7)
    wo, Uo, acco = R.GPT_GMC(phi, y, 0.1, I, 2, 5, 0.3, 0.3, 1, 3, 5, 7)
    assert np.isnan(acco).all() and np.isnan(acc).all()
    assert not ws.any() and not Us.any()


WONLY_CASES = {
    # name: (n, D, N, r, Q, m, burnin, maxepoch, epsw)
    "small": (16, 3, 40, 2, 6, 8, 1, 2, 1e-4),
    "ragged": (24, 4, 37, 3, 10, 8, 0, 3, 1e-4),
    "kin40k_shape": (500, 8, 150, 5, 200, 50, 1, 1, 1e-5),
}


@pytest.mark.parametrize("name", list(WONLY_CASES))
def test_sgldermw_matches_oracle(name):
    """GPT_SGLDERMw (GPT_SGLD.jl:1065-1118): w-only SGLD with the Stiefel U held fixed."""
    n, D, N, r, Q, m, burnin, maxepoch, eps = WONLY_CASES[name]
    p = make_problem(n, D, N, r, Q, seed=17)
    sv, seed = 0.05, 31
    ws, U, gn = G().GPT_SGLDERMw(p["phi"], p["y"], sv, p["I"], r, Q, m, eps, burnin, maxepoch, seed,
                                 diag=True)
    wo, Uo, info = R.GPT_SGLDERMw(p["phi"], p["y"], sv, p["I"], r, Q, m, eps, burnin, maxepoch,
                                  seed, record=True)
    assert rel(U, Uo) < 1e-14
    assert rel(ws, wo) < 1e-9, rel(ws, wo)
    assert rel(gn, np.array(info["gradw_norm"])) < 1e-9


def test_sgldERM_generation_a_mapping():
    n, D, N, r, Q, m = 12, 3, 30, 2, 6, 10
    p = make_problem(n, D, N, r, Q, seed=4)
    ws, Us = G().GPT_SGLDERM(p["phi"], p["y"], 0.3, p["I"], r, Q, m, 1e-6, 1e-6, 0, 2, 3)
    wo, Uo, _ = R.GPT_SGLDERM(p["phi"], p["y"], 0.3, p["I"], r, Q, m, 1e-6, 1e-6, 0, 2, 3)
    assert rel(ws, wo) < 1e-8 and rel(Us, Uo) < 1e-8


@pytest.mark.parametrize("engine", ["grid", "chain", "wave"])
def test_injected_initial_state(engine):
    n, D, N, r, Q, m = (12, 3, 30, 2, 6, 10) if engine != "wave" else (24, 3, 30, 6, 6, 10)
    p = make_problem(n, D, N, r, Q, seed=8)
    rng = np.random.default_rng(0)
    w0 = rng.standard_normal(Q)
    _, U0 = R.init_state(n, r, D, Q, 999)
    ws, Us = G().GPTregression(p["phi"], p["y"], 0.1, p["I"], r, Q, m, 1e-4, 1e-6, 0, 1, 4,
                               w_init=w0, U_init=U0, engine=engine)
    wo, Uo, _ = R.GPTregression(p["phi"], p["y"], 0.1, p["I"], r, Q, m, 1e-4, 1e-6, 0, 1, 4,
                                w_init=w0, U_init=U0)
    assert rel(ws, wo) < 1e-8 and rel(Us, Uo) < 1e-8


@pytest.mark.parametrize("engine", ["grid", "chain", "wave"])
def test_nan_geodesic_bailout_zero_fills(capsys, engine):
    n, D, N, r, Q, m = (12, 3, 30, 2, 6, 10) if engine != "wave" else (24, 3, 30, 6, 6, 10)
    p = make_problem(n, D, N, r, Q, seed=6)
    ws, Us = G().GPTregression(p["phi"], p["y"], 0.1, p["I"], r, Q, m, 1e-4, 1e300, 0, 2, 3,
                               engine=engine)
    assert not ws.any() and not Us.any()
    assert "Get NaN when moving along Geodesic" in capsys.readouterr().out
    _, _, info = R.GPTregression(p["phi"], p["y"], 0.1, p["I"], r, Q, m, 1e-4, 1e300, 0, 2, 3)
    assert info["status"] == 1


def test_bad_dims_raise():
    from gpt_amd._lib import GPTError
    p = make_problem(8, 3, 20, 2, 5, seed=1)
    with pytest.raises((GPTError, ValueError)):
        G().GPTregression(p["phi"], p["y"], 0.1, p["I"], 7, 5, 4, 1e-4, 1e-6, 0, 1, 1)  # r=7
    with pytest.raises((GPTError, ValueError)):
        G().GPTregression(p["phi"], p["y"], 0.1, p["I"], 2, 5000, 4, 1e-4, 1e-6, 0, 1, 1)


def test_gpnt_sgld_matches_oracle():
    rng = np.random.default_rng(12)
    N, D, n = 120, 4, 80
    X = rng.standard_normal((N, D)); Z = rng.standard_normal((n, D)); b = 2 * np.pi * rng.random(n)
    phi = R.featureNotensor(X, 1.4, 1.0, Z, b)
    y = rng.standard_normal(N)
    got = G().GPNT_SGLD(phi, y, 0.05, 1.0, 25, 1e-4, 0.1, 1, 2, 5)
    want = R.GPNT_SGLD(phi, y, 0.05, 1.0, 25, 1e-4, 0.1, 1, 2, 5)
    assert got.shape == want.shape
    assert rel(got, want) < 1e-9


@pytest.mark.parametrize("engine", ["grid", "chain", "wave"])
def test_multichain_session_equals_single_runs(engine):
    import torch
    from gpt_amd.session import SGLDSession
    n, D, N, r, Q, m = (32, 4, 60, 3, 12, 16) if engine != "wave" else (32, 4, 60, 6, 12, 16)
    p = make_problem(n, D, N, r, Q, seed=21)
    phi_t = torch.from_numpy(np.ascontiguousarray(p["phi"].transpose(2, 1, 0))).cuda()
    y_t = torch.from_numpy(p["y"]).cuda()
    seeds = [3, 4, 5]
    s = SGLDSession(phi_t, y_t, p["I"], r, Q, m, 1e-4, 1e-6, 0.05, 0, 2, seeds, store_every=2,
                    engine=engine)
    assert s.info()["engine"] == engine
    s.run(3)          # partial chunk (direct launches)
    s.prepare(4)      # graphs for the next 4 steps: the epoch's last step + 3 of the next epoch
    s.run(4)          # replays them (an epoch-order build inside the second graph)
    s.run(10 ** 9)    # the rest
    s.sync()
    for c, sd in enumerate(seeds):
        ws, Us, st = s.fetch(c)
        wo, Uo, _ = R.GPTregression(p["phi"], p["y"], 0.05, p["I"], r, Q, m, 1e-4, 1e-6, 0, 2, sd,
                                    store_every=2)
        assert st == 0 and rel(ws, wo) < 1e-8 and rel(Us, Uo) < 1e-8
    s.close()


@pytest.mark.parametrize("shape", ["kin40k_ref_sweeps", "bench_chain_engine"])
def test_regression_chains_equals_session(shape):
    """gpt_sgld_regression_chains (the host-array multi-chain entry the Julia shim binds for
    kin40kExperiment.jl:67-74's sweep block) against a device session of the same chains: the
    stores are bitwise equal.  kin40k_ref_sweeps: the script's shape (n = 150, r = 20, m = 50,
    εw = 1e-4, εU = 1e-7; the wave engine), ten sweeps, each its own phi from its own length scales
    and σ_RBF (:68-72), two epochs of epoch-end samples.  bench_chain_engine: the metric's shape
    (n = 500, r = 5) on the chain engine, four chains on one phi with per-chain εw / εU / σ²."""
    import torch
    import bench
    from gpt_amd import GPT_SGLD as GG
    from gpt_amd.session import SGLDSession
    Xtr, ytr, _, _, _ = bench.kin40k(8)
    D, Q, m = 8, 200, 50
    nb = -(-ytr.size // m)
    if shape == "kin40k_ref_sweeps":
        n, r, engine, C, epochs = 150, 20, None, 10, 2
        I = GG.samplenz(r, D, Q, 17)
        Z, b = GG.feature_inputs(n, D, 17)
        scale = math.sqrt(n / Q ** (1.0 / D))
        phis = []
        for j in range(1, C + 1):
            g = np.random.default_rng(j)
            ls = np.ones(D) + 0.2 * g.standard_normal(D)
            phis.append(GG.feature(Xtr, ls, 1 + 0.2 * g.standard_normal(), scale, Z, b))
        ew, eu, sv = 1e-4, 1e-7, 0.0476
        hyper = None
    else:
        n, r, engine, C, epochs = 500, 5, "chain", 4, 1
        I = GG.samplenz(r, D, Q, 17)
        Z, b = GG.feature_inputs(n, D, 17)
        phis = GG.feature(Xtr, np.array(bench.KIN40K_LS), 1.0420, math.sqrt(n / Q ** (1.0 / D)), Z, b)
        ew, eu, sv = [1e-5, 2e-5, 1e-5, 5e-6], [1e-8, 1e-8, 2e-8, 5e-9], [0.0476, 0.05, 0.0476, 0.04]
        hyper = list(zip(ew, eu, sv))
    seeds = list(range(1, C + 1))
    got = GG.GPTregression_chains(phis, ytr, sv, I, r, Q, m, ew, eu, 0, epochs, seeds,
                                  store_every=nb, engine=engine)
    plist = phis if isinstance(phis, list) else [phis]
    dphi = [torch.from_numpy(np.ascontiguousarray(np.transpose(p, (2, 1, 0)))).cuda() for p in plist]
    y_d = torch.from_numpy(np.ascontiguousarray(ytr)).cuda()
    s = SGLDSession(dphi, y_d, I, r, Q, m, ew if hyper is None else ew[0],
                    eu if hyper is None else eu[0], sv if hyper is None else sv[0], 0, epochs, seeds,
                    store_every=nb, store=True, engine=engine or "auto")
    assert s.info()["engine"] == ("wave" if engine is None else engine)
    if hyper:
        for c, (a, bb, v) in enumerate(hyper):
            s.set_hyper(c, a, bb, v)
    s.run(epochs * nb)
    s.sync()
    alive = 0
    for c in range(C):
        ws, Us, st = s.fetch(c)
        gw, gU, gst = got[c]
        assert gst == st, (c, gst, st)
        assert np.array_equal(gw, ws) and np.array_equal(gU, Us), c
        alive += st == 0
    s.close()
    assert alive >= C // 2


@pytest.mark.parametrize("engine", ["grid", "chain", "wave"])
def test_epoch_order_ring_over_many_epochs(engine):
    """Seven epochs of a ragged N (nb = 4) with every epoch-end sample stored: the two-slot order
    ring (order.hip) must hand each epoch its own composed permutation, through direct launches
    and graph replays alike."""
    n, D, N, r, Q, m = (24, 3, 29, 3, 10, 8) if engine != "wave" else (24, 3, 29, 6, 10, 8)
    p = make_problem(n, D, N, r, Q, seed=31)
    got_w, got_U = G().GPTregression(p["phi"], p["y"], 0.05, p["I"], r, Q, m, 1e-4, 1e-6, 1, 6, 9,
                                     store_every=2, engine=engine)
    wo, Uo, info = R.GPTregression(p["phi"], p["y"], 0.05, p["I"], r, Q, m, 1e-4, 1e-6, 1, 6, 9,
                                   store_every=2)
    assert info["status"] == 0
    assert rel(got_w, wo) < 1e-8 and rel(got_U, Uo) < 1e-8


def test_engine_selection():
    """One chain at the kin40k shape runs the grid engine (D + 1 workgroups, the shorter step);
    r = 20 at the reference's kin40k shape runs the wave engine by default; the removed split
    engine is rejected."""
    import torch
    from gpt_amd._lib import GPTError
    from gpt_amd.session import SGLDSession
    dev = torch.device("cuda", 0)
    for (n, D, N, r, Q, m), want in [((500, 8, 200, 5, 200, 50), "grid"),
                                     ((150, 8, 100, 20, 200, 50), "wave")]:
        p = make_problem(n, D, N, r, Q, seed=3)
        phi = torch.from_numpy(np.ascontiguousarray(np.asarray(p["phi"]).transpose(2, 1, 0))).to(dev)
        y = torch.from_numpy(np.ascontiguousarray(np.asarray(p["y"], dtype=np.float64))).to(dev)
        s = SGLDSession(phi, y, p["I"], r, Q, m, 1e-4, 1e-6, 0.05, 0, 1, [5])
        info = s.info()
        s.close()
        assert info["engine"] == want
        if want == "grid":
            assert info["workgroups"] == D + 1
        else:
            assert info["workgroups"] == D and info["threads"] == 64
    with pytest.raises(GPTError):
        import ctypes as C
        from gpt_amd import _lib
        from gpt_amd.GPT_SGLD import make_config
        cfg = make_config(16, 3, 40, 2, 6, 8, 1e-4, 1e-6, 0.05, 1.0, 0, 1, 0, True, True, 1, 0)
        p = make_problem(16, 3, 40, 2, 6, seed=1)
        phi = torch.from_numpy(np.ascontiguousarray(np.asarray(p["phi"]).transpose(2, 1, 0))).to(dev)
        y = torch.from_numpy(np.ascontiguousarray(np.asarray(p["y"], dtype=np.float64))).to(dev)
        I = np.asfortranarray(np.asarray(p["I"], dtype=np.int32))
        h = C.c_void_p()
        _lib.check(_lib.lib().gpt_sgld_session_create(
            C.byref(cfg), 1, (C.c_uint64 * 1)(1), (C.c_void_p * 1)(phi.data_ptr()),
            (C.c_void_p * 1)(y.data_ptr()), I.ctypes.data_as(_lib.P_I32), 1 | 64, None, C.byref(h)))


@pytest.mark.parametrize("env_engine", ["chain", "wave"])
def test_explicit_engine_flags_beat_environment(monkeypatch, env_engine):
    """GPTSGLD_ENGINE applies only when no engine bit is set: w-only steps (bit 16),
    classification (bit 32) and an explicit grid request (bit 2) stay on the grid engine, the only
    one that implements them, and still match the oracle."""
    import torch
    from gpt_amd.session import SGLDSession
    monkeypatch.setenv("GPTSGLD_ENGINE", env_engine)
    n, D, N, r, Q, m, burnin, maxepoch, eps = WONLY_CASES["small"]
    p = make_problem(n, D, N, r, Q, seed=17)
    ws, U, gn = G().GPT_SGLDERMw(p["phi"], p["y"], 0.05, p["I"], r, Q, m, eps, burnin, maxepoch,
                                 31, diag=True)
    wo, Uo, info = R.GPT_SGLDERMw(p["phi"], p["y"], 0.05, p["I"], r, Q, m, eps, burnin, maxepoch,
                                  31, record=True)
    assert rel(ws, wo) < 1e-9 and rel(U, Uo) < 1e-14
    n, D, N, r, Q, m, ncls, burnin, maxepoch, lang, stf = CLS_CASES["binary_sgld_stiefel"]
    p = make_problem(n, D, N, r, Q, seed=23)
    f = p["y"] - np.median(p["y"])
    y = (1 + np.clip(np.floor((f - f.min()) / (np.ptp(f) + 1e-12) * ncls), 0, ncls - 1)).astype(float)
    ws, Us = G().GPTclassification(p["phi"], y, p["I"], r, Q, m, 1e-4, 1e-6, burnin, maxepoch, 41)
    wo, Uo, _ = R.GPTclassification(p["phi"], y, p["I"], r, Q, m, 1e-4, 1e-6, burnin, maxepoch, 41)
    assert rel(ws, wo) < 1e-8 and rel(Us, Uo) < 1e-8
    n, D, N, r, Q, m = 32, 4, 60, 3, 12, 16
    p = make_problem(n, D, N, r, Q, seed=21)
    phi = torch.from_numpy(np.ascontiguousarray(p["phi"].transpose(2, 1, 0))).cuda()
    s = SGLDSession(phi, torch.from_numpy(p["y"]).cuda(), p["I"], r, Q, m, 1e-4, 1e-6, 0.05, 0, 1,
                    [3], engine="grid")
    assert s.info()["engine"] == "grid"
    s.close()


def test_chain_engine_declines_odd_n_past_one_block():
    """Odd n > 64 cannot use the chain engine's 16-B row staging: forcing it fails loudly
    (GPT_ERR_BAD_DIMS) and the default selection runs the grid engine (n101_odd above)."""
    from gpt_amd._lib import GPTError
    n, D, N, r, Q, m, burnin, maxepoch, se, lang, stf = CASES["n101_odd"]
    p = make_problem(n, D, N, r, Q, seed=11)
    with pytest.raises(GPTError):
        G().GPTregression(p["phi"], p["y"], 0.05, p["I"], r, Q, m, 1e-4, 1e-6, burnin, maxepoch,
                          23, store_every=se, engine="chain")


@pytest.mark.parametrize("nn", [12, 20, 24, 30, 40])
@pytest.mark.parametrize("mode", [0, 1])
def test_device_expm_all_pade_degrees(nn, mode):
    """The device expm (mode 0: the wave engine's register-blocked Padé, wave.hip; mode 1: the grid
    and chain engines' wave_expm) against the oracle's restatement of Julia Base expm! on
    geodesic-shaped matrices t·[A −S; I A] (A skew, S symmetric PSD) whose 1-norms cover every
    branch: degrees 3, 5, 7, 9 and 13 with and without the 2^-s scaling."""
    import ctypes as C
    from gpt_amd import _lib
    r = nn // 2
    rng = np.random.default_rng(nn)
    mats, want = [], []
    for target in [0.01, 0.2, 0.6, 1.5, 2.0, 4.4, 9.0, 40.0]:
        B = rng.standard_normal((r, r))
        A = (B - B.T) / 2
        Wm = rng.standard_normal((3 * r, r))
        S = Wm.T @ Wm
        T = np.block([[A, -S], [np.eye(r), A]])
        X = T * (target / np.abs(T).sum(axis=0).max())
        mats.append(X)
        want.append(R.expm(X))
    Ah = np.ascontiguousarray(np.stack(mats))
    E = np.zeros_like(Ah)
    bad = np.zeros(len(mats), dtype=np.int32)
    _lib.check(_lib.lib().gpt_debug_expm(nn, len(mats), mode, Ah.ctypes.data_as(_lib.P_D),
                                         E.ctypes.data_as(_lib.P_D), bad.ctypes.data_as(_lib.P_I32)))
    assert not bad.any()
    for c in range(len(mats)):
        assert rel(E[c], want[c]) < 1e-12, (c, rel(E[c], want[c]))


def test_injected_U_off_the_manifold_is_rejected():
    """On the Stiefel path the kernels take geod's A = Uᵀmom from the projection's Gram (valid for
    UᵀU = I only): a U_init with non-orthonormal columns is refused (GPT_ERR_BAD_DIMS)."""
    from gpt_amd._lib import GPTError
    n, D, N, r, Q, m = 12, 3, 30, 2, 6, 10
    p = make_problem(n, D, N, r, Q, seed=8)
    _, U0 = R.init_state(n, r, D, Q, 999)
    with pytest.raises(GPTError):
        G().GPTregression(p["phi"], p["y"], 0.1, p["I"], r, Q, m, 1e-4, 1e-6, 0, 1, 4,
                          U_init=1.01 * U0)
    # Euclidean runs take any U
    G().GPTregression(p["phi"], p["y"], 0.1, p["I"], r, Q, m, 1e-4, 1e-6, 0, 1, 4,
                      U_init=1.01 * U0, stiefel=False)
