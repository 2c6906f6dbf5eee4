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


@pytest.mark.parametrize("n,D,r,Q,N,m,epsw,epsU,steps", [
    (40, 3, 2, 10, 120, 20, 1e-3, 1e-4, 60),
    (150, 4, 10, 60, 300, 50, 1e-4, 1e-6, 30),
    (64, 2, 3, 20, 200, 30, 1e-3, 1e-2, 80),
])
def test_geod_grams_from_projection_identity(monkeypatch, n, D, r, Q, N, m, epsw, epsU, steps):
    """The step kernels form geod's A = Uᵀmom (GPT_SGLD.jl:19-37) as (M − Mᵀ)/2 from the
    projection's M = UᵀW (chain engine; S = momᵀmom from its own pass) and S as
    G − MᵀMs − Ms·M + Ms·Ms from the drive's Gram G = WᵀW (grid engine), which hold for UᵀU = I.
    Whole oracle trajectories with the identities substituted agree with the reference form
    within 1e-12 relative (measured ≤ 1.2e-14), far inside the 1e-8 GPU parity tolerance."""
    rng = np.random.default_rng(0)
    phi = rng.standard_normal((n, D, N)) * math.sqrt(2.0 / n)
    y = rng.standard_normal(N)
    I = np.stack([rng.integers(0, r, Q) for _ in range(D)], axis=1)
    ep = -(-steps * m // N) + 1
    w0, U0, _ = R.GPTregression(phi, y, 0.1, I, r, Q, m, epsw, epsU, 0, ep, 7, max_steps=steps)
    cache = {}
    orig_expm = R.expm

    def proj(U, V):
        M = U.T @ V
        Ms = (M + M.T) / 2
        cache.update(M=M, Ms=Ms, G=V.T @ V)
        return V - U @ Ms

    def geod(U, mom, t):
        n_, r_ = U.shape
        M, Ms, G = cache["M"], cache["Ms"], cache["G"]
        A = (M - M.T) / 2
        S = G - M.T @ Ms - Ms @ M + Ms @ Ms
        T = np.block([[A, -S], [np.eye(r_), A]])
        E = orig_expm(t * T)
        tmpU = (np.hstack([U, mom]) @ E[:, :r_]) @ orig_expm(-t * A)
        return tmpU / np.linalg.norm(tmpU, axis=0)[None, :], True

    monkeypatch.setattr(R, "proj", proj)
    monkeypatch.setattr(R, "geod", geod)
    w1, U1, _ = R.GPTregression(phi, y, 0.1, I, r, Q, m, epsw, epsU, 0, ep, 7, max_steps=steps)
    rel = lambda a, b: np.abs(a[..., :steps] - b[..., :steps]).max() / np.abs(b[..., :steps]).max()
    assert rel(w1, w0) < 1e-12 and rel(U1, U0) < 1e-12, (rel(w1, w0), rel(U1, U0))


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


def _gibbs_literal(b, y, sigma, n, r, q, iters, burnin, seed, I):
    """TGP.jl:37-86 written as the reference's element-wise comprehensions (tiny sizes only),
    with the same Philox draws and the same zero-initialised absent runs as the oracle."""
    _, D, N = b.shape
    su2, sw2 = 1.0 / r, float(r) ** D / q
    U = R.tgp_init_U(n, r, D, seed)
    dot = lambda k, l, j: sum(U[a, l - 1, k] * b[a, k, j] for a in range(n))     # noqa: E731
    Ws, Us = [], []
    for it in range(1, iters + 1):
        V = np.array([[math.prod(dot(d, I[i, d], j) for d in range(D)) for j in range(N)]
                      for i in range(q)])
        M = V @ V.T / sigma ** 2 + np.eye(q) / sw2
        mu = np.linalg.solve(M, V @ y / sigma ** 2)
        Lt = np.linalg.cholesky(M).T                                          # chol(M, :U)
        W = np.linalg.solve(Lt, px.normals(q, seed, it - 1, px.TGP_W_NOISE, 0)) + mu
        if it > burnin:
            Ws.append(W.copy()); Us.append(U.copy())
        for k in range(D):
            Vk = np.array([[V[l, j] / dot(k, I[l, k], j) for j in range(N)] for l in range(q)])
            Vkk = W[:, None] * Vk
            C = np.zeros((r, N))
            for l in set(I[:, k]):
                C[l - 1, :] = Vkk[I[:, k] == l, :].sum(axis=0)
            Ck = np.array([[C[row // n, j] * b[row % n, k, j] for j in range(N)]
                           for row in range(n * r)])                          # repeat ⊙ repmat
            Mu = Ck @ Ck.T / sigma ** 2 + np.eye(n * r) / su2
            z = px.normals(n * r, seed, it - 1, px.TGP_U_NOISE, k)
            x = np.linalg.solve(Mu, z) + np.linalg.solve(Mu, Ck @ y / sigma ** 2)
            U[:, :, k] = x.reshape((n, r), order="F")
            V = np.array([[Vk[l, j] * dot(k, I[l, k], j) for j in range(N)] for l in range(q)])
    return np.array(Ws).T, np.moveaxis(np.array(Us), 0, -1)


def test_tgp_gibbs_oracle_matches_literal_restatement():
    """The vectorised GPT_inf restatement against TGP.jl's comprehension form (tiny sizes)."""
    rng = np.random.default_rng(5)
    n, D, N, r, q, sigma = 4, 3, 9, 2, 5, 0.4
    b = rng.standard_normal((n, D, N))
    y = rng.standard_normal(N)
    I = R.tgp_draw_I(q, D, r, 11)
    W, U, I2 = R.GPT_inf(b, y, sigma, n, r, q, 3, 1, 11, I=I)
    Wl, Ul = _gibbs_literal(b, y, sigma, n, r, q, 3, 1, 11, I)
    assert (I2 == I).all()
    assert np.abs(W - Wl).max() <= 1e-10 * np.abs(Wl).max()
    assert np.abs(U - Ul).max() <= 1e-10 * np.abs(Ul).max()


def test_tgp_draws_and_conditional_mean():
    """I in 1..r with every value used; U init scale sqrt(1/r); the W draw is centred on the
    posterior mean with covariance M⁻¹ (checked through whitening by chol(M)ᵀ)."""
    I = R.tgp_draw_I(400, 3, 5, 3)
    assert I.min() == 1 and I.max() == 5 and I.shape == (400, 3)
    assert abs(np.bincount(I.ravel())[1:].mean() - 240) < 1e-9
    U = R.tgp_init_U(200, 5, 2, 3)
    assert abs(U.std() - math.sqrt(1 / 5)) < 0.02
    rng = np.random.default_rng(6)
    n, D, N, r, q, sigma = 5, 2, 40, 3, 7, 0.3
    b = rng.standard_normal((n, D, N))
    y = rng.standard_normal(N)
    I = R.tgp_draw_I(q, D, r, 4)
    W, U, _ = R.GPT_inf(b, y, sigma, n, r, q, 1, 0, 4, I=I)
    V = R.tgp_V(U[..., 0], I, b)
    M = V @ V.T / sigma ** 2 + np.eye(q) * q / r ** D
    mu = np.linalg.solve(M, V @ y / sigma ** 2)
    z = np.linalg.cholesky(M).T @ (W[:, 0] - mu)
    assert np.abs(z - px.normals(q, 4, 0, px.TGP_W_NOISE, 0)).max() < 1e-9


def test_sgldermw_oracle_keeps_U_and_matches_first_step():
    rng = np.random.default_rng(8)
    n, D, N, r, Q, m = 6, 2, 20, 2, 3, 10
    phi = rng.standard_normal((n, D, N))
    y = rng.standard_normal(N)
    I = R.samplenz(r, D, Q, 2)
    ws, U, info = R.GPT_SGLDERMw(phi, y, 0.3, I, r, Q, m, 1e-3, 0, 1, 5, record=True)
    w0, U0 = R.init_state(n, r, D, Q, 5, True, 1.0)
    assert np.array_equal(U, U0)
    idx = np.arange(N)[px.randperm(N, 5, 0)][:m]
    V = R.computeV(R.phidotU(U0, phi[:, :, idx]), I)
    g = (N / m) * V @ (y[idx] - V.T @ w0) / 0.3 - w0
    w1 = w0 + 1e-3 * g / 2 + math.sqrt(1e-3) * px.normals(Q, 5, 0, px.W_NOISE, 0)
    assert np.allclose(ws[:, 0], w1, rtol=0, atol=1e-13)
    assert abs(info["gradw_norm"][0] - np.linalg.norm(g)) < 1e-10 * np.linalg.norm(g)


def test_classification_oracle_first_step_and_softmax_gradient():
    """GPTclassification restatement: class-0 init equals GPTregression's (Stiefel), the
    residual is [y = c] − softmax, and the gradient matches finite differences of the
    multinomial log-likelihood Σ_i fhat[i, y_i] − logsumexp_i (the reference's check, :568-602)."""
    rng = np.random.default_rng(12)
    n, D, N, r, Q = 6, 2, 12, 2, 3
    phi = rng.standard_normal((n, D, N))
    I = R.samplenz(r, D, Q, 4)
    w, U = R.init_state_cls(n, r, D, Q, 3, 9)
    w0, U0 = R.init_state(n, r, D, Q, 9)
    assert np.array_equal(w[:, 0], w0) and np.array_equal(U[..., 0], U0)
    y = np.array([1, 2, 3] * 4)

    def ll(wc):
        f = np.stack([R.computefhat(R.computeV(R.phidotU(U[..., c], phi), I), wc[:, c])
                      for c in range(3)], axis=1)
        return sum(f[i, y[i] - 1] - R.logsumexp(f[i]) for i in range(N))
    f = np.stack([R.computefhat(R.computeV(R.phidotU(U[..., c], phi), I), w[:, c]) for c in range(3)], axis=1)
    lse = np.array([R.logsumexp(f[i]) for i in range(N)])
    c = 1
    res = (y == c + 1) - np.exp(f[:, c] - lse)
    gw, gU = R.gradients_res(phi, res, w[:, c], U[..., c], I, N)
    q, h = 2, 1e-6
    wp = w.copy(); wp[q, c] += h
    wm = w.copy(); wm[q, c] -= h
    fd = (ll(wp) - ll(wm)) / (2 * h)
    assert abs((gw[q] + w[q, c]) - fd) < 1e-6 * max(1.0, abs(fd))   # N/B = 1 here


def test_gmc_oracle_energy_conservation_and_w_only_rejection():
    """GPT_GMC restatement: the leapfrog conserves H to O(ε) (acceptance → 1 as ε → 0), and a
    rejected epoch restores w but keeps U's proposal (the reference's U_old aliasing)."""
    rng = np.random.default_rng(3)
    n, D, N, r, Q = 8, 3, 40, 2, 5
    phi = rng.standard_normal((n, D, N)) * 0.5
    I = R.samplenz(r, D, Q, 1)
    w, U = R.init_state(n, r, D, Q, 3)
    y = R.pred(w, U, I, phi) + 0.1 * rng.standard_normal(N)
    _, _, acc = R.GPT_GMC(phi, y, 1.0, I, r, Q, 1e-7, 1e-7, 0, 2, 3, 7)
    assert np.all(np.abs(acc - 1) < 1e-3)
    ws, Us, acc = R.GPT_GMC(phi, y, 1.0, I, r, Q, 0.1, 0.1, 0, 1, 5, 7)
    u = px.uniform(7, 0, px.GMC_U, 0)
    w0, U0 = R.init_state(n, r, D, Q, 7)
    assert u > acc[0]                                   # this epoch is rejected
    assert np.array_equal(ws[:, 0], w0)                 # w restored
    assert not np.allclose(Us[..., 0], U0)              # U keeps the proposal


def test_kronecker_precision_from_user_statistics():
    """The identity behind the device's w | U, V system (cf.hip cfg_wprec / cfg_wrhs, GPT_fullw_gibbs
    :1088-1093): with Kron[i, a·r + b] = V[m_i, a]·U[u_i, b], Kronᵀ·Kron[(a,b), (a',b')] =
    Σ_u H_u[a,a']·U[u,b]·U[u,b'] (H_u = Σ_{i∈u} V[m_i]ᵀV[m_i]) and Kronᵀ·y[(a,b)] = Σ_u h_u[a]·U[u,b]
    (h_u = Σ_{i∈u} y_i V[m_i]), here on random ratings with users that rate nothing."""
    rng = np.random.default_rng(5)
    n1, n2, r, N = 30, 40, 4, 500
    users = rng.integers(0, n1 - 3, N)
    movies = rng.integers(0, n2, N)
    y = rng.standard_normal(N)
    U = rng.standard_normal((n1, r))
    V = rng.standard_normal((n2, r))
    K = (V[movies][:, :, None] * U[users][:, None, :]).reshape((N, r * r))
    H = np.zeros((n1, r, r))
    h = np.zeros((n1, r))
    for i in range(N):
        H[users[i]] += np.outer(V[movies[i]], V[movies[i]])
        h[users[i]] += y[i] * V[movies[i]]
    P = np.einsum("ub,uc->ubc", U, U)
    Z = np.einsum("uad,ubc->abdc", H, P).reshape(r * r, r * r)     # [(a,b), (a',b')]
    rhs = np.einsum("ua,ub->ab", h, U).reshape(r * r)
    assert np.abs(Z - K.T @ K).max() <= 1e-12 * np.abs(K.T @ K).max()
    assert np.abs(rhs - K.T @ y).max() <= 1e-12 * np.abs(K.T @ y).max()


def test_movielens_cpp_port_matches_numpy_restatement():
    """oracle/cpu/movielens_cpu.cpp (the MovieLens CPU baseline of bench.py) against
    oracle/movielens_ref.py's GPT_fullw_sideinfo (SGD) over two epochs of a small problem."""
    from oracle import cpu_lib
    from oracle import movielens_ref as M
    from oracle import philox as px
    rng = np.random.default_rng(3)
    n1, n2, D1, D2, r, N, Nt, m, seed = 30, 40, 5, 4, 4, 300, 50, 16, 17
    ud = (rng.random((n1, D1)) < 0.3).astype(float)
    md = (rng.random((n2, D2)) < 0.3).astype(float)

    def ratings(n):
        return np.column_stack([rng.integers(1, n1 + 1, n), rng.integers(1, n2 + 1, n),
                                rng.standard_normal(n)])
    R, Rt = ratings(N), ratings(Nt)
    w0 = 0.3 * rng.standard_normal((r, r))
    want = M.GPT_fullw_sideinfo(R, ud, md, Rt, 0.8, 0.1, 1.0, w0, m, 1e-3, 1e-3, 0.5, 0.25, 0.5, 0,
                                2, seed, 0.0, 1.0)
    U0 = M.init_uv(n1 + D1, r, seed, 0, False, 0.1)
    V0 = M.init_uv(n2 + D2, r, seed, 1, False, 0.1)
    perms = np.stack([px.randperm(N, seed, e) for e in range(2)])
    _, outs = cpu_lib.cf_sgd_folds([(R, Rt)], ud, md, [perms], w0, U0, V0, 0.8, 0.1, 1.0, m, 1e-3,
                                   1e-3, 0.5, 0.25, 0.5)
    w, U, V, sse = outs[0]
    for got, ref in ((w, want[0][:, :, 1]), (U, want[1][:, :, 1]), (V, want[2][:, :, 1])):
        assert np.abs(got - ref).max() <= 1e-12 * np.abs(ref).max()
    pred = M.predict(Rt, U, V, w, *M.side_rows(ud, md), 0.5, 0.25, 0.5)
    assert sse[1, 1] == pytest.approx(np.sum((Rt[:, 2] - pred) ** 2), rel=1e-12)
    # the lazy prior-decay move (the GPU's one-launch epoch, cf.hip domove = 2): the same numbers
    _, outs_l = cpu_lib.cf_sgd_folds([(R, Rt)], ud, md, [perms], w0, U0, V0, 0.8, 0.1, 1.0, m,
                                     1e-3, 1e-3, 0.5, 0.25, 0.5, lazy=True)
    for got, ref in zip(outs_l[0], outs[0]):
        assert np.abs(got - ref).max() <= 1e-12 * np.abs(ref).max()
