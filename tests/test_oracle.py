"""CPU tests: the oracle pinned against the reference's own fixtures and methods.

- TensorSynthData{5D,10D}100N.h5 (MakeSynthData.jl:6-27): y_k = pred(w,U,I,phi) + N(0,σ_k²).
  Residual std of y3 (σ² = 1e-3) must be ≈ sqrt(1e-3) and U orthonormal — pins pred, phidotU,
  computeV, computefhat and the column-major layouts.
- Diagnostic_gradients.jl:131-158: analytic gradients vs finite differences (here central
  differences with a stated tolerance instead of printing the std of the differences).
- Julia Base expm! vs scipy.linalg.expm; Philox4x32-10 vs the Random123 known-answer vectors.
"""
import math

import numpy as np
import pytest
import scipy.linalg

from oracle import gpt_sgld_ref as R
from oracle import philox as px


@pytest.mark.parametrize("tag,expected", [("5D", 0.03125), ("10D", 0.0258)])
def test_pred_pinned_by_fixture(tag, expected):
    from conftest import load_golden
    d = load_golden("tensor_synth_%s.npz" % tag)
    f = R.pred(d["w"], d["U"], d["I"], d["phi"])
    res = d["y3"] - f
    assert abs(np.std(res) - expected) < 5e-4
    # y1 (σ²=0.1) and y2 (σ²=0.01) residuals scale with their noise levels
    assert 0.2 < np.std(d["y1"] - f) < 0.45
    assert 0.06 < np.std(d["y2"] - f) < 0.14
    U = d["U"]
    for k in range(U.shape[2]):
        assert np.abs(U[:, :, k].T @ U[:, :, k] - np.eye(U.shape[1])).max() < 1e-12
    # phi bound: |phi| <= sqrt(2)*scale/sqrt(n) with scale = sqrt(n/Q^(1/D))
    n, D, N = d["phi"].shape
    Q = len(d["w"])
    bound = math.sqrt(2.0 / n) * math.sqrt(n / Q ** (1.0 / D))
    assert np.abs(d["phi"]).max() <= bound * (1 + 1e-12)


def test_phidotU_layout_against_fixture():
    from conftest import load_golden
    d = load_golden("tensor_synth_5D.npz")
    phi, U = d["phi"], d["U"]
    temp = R.phidotU(U, phi)
    k, l, i = 3, 1, 17
    assert temp[k, l, i] == pytest.approx(float(np.dot(phi[:, k, i], U[:, l, k])), rel=1e-14)


def test_finite_difference_gradients():
    from conftest import load_golden
    d = load_golden("tensor_synth_5D.npz")
    phi, w, U, I, y = d["phi"], d["w"], d["U"], d["I"], d["y3"]
    sigma = math.sqrt(1e-3)
    N = phi.shape[2]
    g = R.gradients(phi, y, w, U, I, N, sigma ** 2, sigma_w=1e150)   # likelihood part only (prior term ~1e-300)
    h = 1e-6
    fdw = np.array([(R.loglik(phi, y, w + h * e, U, I, sigma) - R.loglik(phi, y, w - h * e, U, I, sigma)) / (2 * h)
                    for e in np.eye(len(w))])
    assert np.abs(fdw - g["gradw"]).max() <= 1e-7 * np.abs(g["gradw"]).max()
    fdU = np.zeros_like(U)
    for idx in np.ndindex(U.shape):
        Up = U.copy(); Up[idx] += h
        Um = U.copy(); Um[idx] -= h
        fdU[idx] = (R.loglik(phi, y, w, Up, I, sigma) - R.loglik(phi, y, w, Um, I, sigma)) / (2 * h)
    assert np.abs(fdU - g["gradU"]).max() <= 1e-7 * np.abs(g["gradU"]).max()


@pytest.mark.parametrize("scale", [1e-4, 0.01, 0.2, 0.6, 1.5, 3.0, 40.0])
def test_expm_matches_scipy(scale):
    rng = np.random.default_rng(int(scale * 1000))
    A = rng.standard_normal((10, 10)) * scale
    ref = scipy.linalg.expm(A)
    assert np.abs(R.expm(A) - ref).max() <= 1e-13 * max(1.0, np.abs(ref).max()) * max(1, scale)


def test_geod_stays_on_stiefel():
    rng = np.random.default_rng(3)
    w, U = R.init_state(40, 4, 1, 3, 7)
    U = U[:, :, 0]
    mom = R.proj(U, rng.standard_normal(U.shape))
    Un, ok = R.geod(U, mom, 0.05)
    assert ok
    assert np.abs(Un.T @ Un - np.eye(4)).max() < 1e-12
    with np.errstate(all="ignore"):
        bad, ok = R.geod(U, U * 1e4, 1.0)   # exp(1e4) overflows -> NaN in E
    assert not ok and not bad.any()


def test_philox_known_answers():
    kat = [((0, 0, 0, 0), 0, (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, 0xffffffffffffffff, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0x299f31d0 << 32) | 0xa4093822,
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in kat:
        got = tuple(int(x) for x in px.philox4x32(*ctr, key))
        assert got == want


def test_normals_and_perm_statistics():
    z = px.normals(200001, 11, 0, px.W_NOISE, 0)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    p = px.randperm(1000, 5, 3)
    assert sorted(p.tolist()) == list(range(1000))
    assert not (p == np.arange(1000)).all()


def test_samplenz_distinct_digits():
    I = R.samplenz(5, 8, 200, 17)
    assert I.shape == (200, 8) and I.min() >= 1 and I.max() <= 5
    L = sum((I[:, k].astype(np.int64) - 1) * 5 ** k for k in range(8))
    assert len(set(L.tolist())) == 200


def test_oracle_sampler_runs_and_zero_fills_on_nan():
    rng = np.random.default_rng(0)
    n, D, N, r, Q = 6, 3, 20, 2, 5
    phi = np.asfortranarray(rng.standard_normal((n, D, N)) * 0.3)
    y = rng.standard_normal(N)
    I = R.samplenz(r, D, Q, 1)
    ws, Us, info = R.GPTregression(phi, y, 0.1, I, r, Q, 7, 1e-3, 1e-3, 1, 2, 5)
    assert info["status"] == 0 and ws.shape == (Q, 2 * 3) and np.isfinite(Us).all()
    ws, Us, info = R.GPTregression(phi, y, 0.1, I, r, Q, 7, 1e-3, 1e300, 0, 1, 5)
    assert info["status"] == 1 and not ws.any() and not Us.any()


def test_reference_curves_fixture():
    from conftest import load_golden
    c = load_golden("ref_curves.npz")
    assert c["testRMSE_kin40k"].shape == (200,)
    assert abs(c["testRMSE_kin40k"][-1] - 0.2385) < 1e-3
    assert abs(c["testRMSE_kin40k"][-50:].mean() - 0.2448) < 2e-3 or c["testRMSE_kin40k"][-50:].mean() > 0.2
    assert abs(c["testRMSE_PP"][-1] - 4.1446) < 1e-3


def test_rmsprop_oracle_first_step_and_invariants():
    """GPT_SGLDERM_RMSprop (GPT_SGLD.jl:1121-1237): the first w update restated by hand from the
    shared gradient pieces, Stiefel invariance of every stored U."""
    import math
    from oracle import philox as px
    rng = np.random.default_rng(5)
    n, D, N, r, Q, m = 10, 3, 30, 2, 6, 10
    X = rng.standard_normal((N, D)); Z = rng.standard_normal((n, D)); b = 2 * np.pi * rng.random((n, D))
    phi = R.feature(X, np.ones(D), 1.0, 2.0, Z, b)
    I = R.samplenz(r, D, Q, 4)
    y = rng.standard_normal(N)
    eps, alpha, sv, seed = 1e-3, 0.9, 0.2, 7
    ws, Us, info = R.GPT_SGLDERM_RMSprop(phi, y, sv, I, r, Q, m, eps, alpha, 0, 2, seed)
    assert info["status"] == 0
    w0, U0 = R.init_state(n, r, D, Q, seed)
    idx = px.randperm(N, seed, 0)[:m]
    temp = R.phidotU(U0, phi[:, :, idx])
    V = R.computeV(temp, I)
    res = y[idx] - V.T @ w0
    gr = V @ res / (m * sv)
    gw = (1 - alpha) * gr ** 2
    ew = eps / (np.sqrt(gw) + R.RMS_LAMBDA)
    w1 = w0 + ew * (N * gr - w0) / 2 + np.sqrt(ew) * px.normals(Q, seed, 0, px.W_NOISE, 0)
    assert np.allclose(ws[:, 0], w1, rtol=1e-13, atol=1e-13)
    for s in range(Us.shape[3]):
        for k in range(D):
            assert np.abs(Us[:, :, k, s].T @ Us[:, :, k, s] - np.eye(r)).max() < 1e-10
