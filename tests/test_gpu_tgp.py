"""GPU parity of the tensor-GP Gibbs sampler (TGP.jl:37-108, §8 a25) against the oracle.

Same b, y, I, seed and Philox draws on both sides.  Tolerances (fp64): the device sums the
SYRKs on the matrix cores in 16×4 blocks and factors with a right-looking Cholesky, so the
precision matrices agree to ~1e-14 relative and the draws to ~cond(M)·1e-16:
  W and U samples            max |Δ| <= 1e-8·max|x|
  features                   max |Δ| <= 1e-14·max|phi|
  TensorRes RMSE             relative <= 1e-9
"""
import math

import numpy as np
import pytest

from oracle import gpt_sgld_ref as R

pytestmark = pytest.mark.gpu


def T():
    from gpt_amd import TGP
    return TGP


def rel(a, b):
    a = np.asarray(a); b = np.asarray(b)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def data(N, D, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((N, D)) * rng.uniform(0.5, 3.0, D) + rng.uniform(-2, 2, D)
    y = np.sin(X).sum(axis=1) + 0.1 * rng.standard_normal(N)
    return X, y


def oracle_b(X, n, sigmaRBF, gen):
    Z, b = R.seeded_feature_inputs(n, X.shape[1], gen)
    return R.feature(X, sigmaRBF, 1.0, 1.0, Z, b)


def test_tgp_feature_row():
    X, _ = data(3, 4, 0)
    got = T().feature(X[1], 12, 1.4332, 123)
    want = oracle_b(X[1:2], 12, 1.4332, 123)[:, :, 0]
    assert got.shape == (12, 4)
    assert rel(got, want) < 1e-14


CASES = {
    # name: (n, D, N, r, q, sigma, iters, burnin)
    "unit_test_shape": (10, 4, 300, 5, 100, 0.2299, 3, 1),        # UnitTest.jl:15 at N=300
    "ragged": (7, 3, 131, 3, 20, 0.3, 4, 2),
    "wide_u": (40, 4, 257, 5, 37, 0.25, 2, 0),                     # nr = 200 (13 MFMA tiles)
}


@pytest.mark.parametrize("name", list(CASES))
def test_gibbs_matches_oracle(name):
    n, D, N, r, q, sigma, iters, burnin = CASES[name]
    X, y = data(N, D, 7)
    gen, sigmaRBF = 123, 1.4332
    W, U, I = T().GPT_inf(X, y, sigma, n, r, sigmaRBF, q, gen, iters, burnin)
    b = oracle_b(R.datawhitening(X), n, sigmaRBF, gen)
    Wo, Uo, Io = R.GPT_inf(b, R.datawhitening(y), sigma, n, r, q, iters, burnin, gen)
    assert (I == Io).all()
    assert W.shape == (q, iters - burnin) and U.shape == (n, r, D, iters - burnin)
    assert rel(W, Wo) < 1e-8, rel(W, Wo)
    assert rel(U, Uo) < 1e-8, rel(U, Uo)


def test_gibbs_fixed_I_and_errors():
    n, D, N, r, q = 6, 2, 80, 2, 4
    X, y = data(N, D, 3)
    I = np.array([[1, 2], [2, 2], [1, 1], [2, 1]], dtype=np.int32)
    W, U, I2 = T().GPT_inf(X, y, 0.3, n, r, 1.0, q, 5, 2, 0, I=I)
    assert (I2 == I).all()
    b = oracle_b(R.datawhitening(X), n, 1.0, 5)
    Wo, Uo, _ = R.GPT_inf(b, R.datawhitening(y), 0.3, n, r, q, 2, 0, 5, I=I)
    assert rel(W, Wo) < 1e-8 and rel(U, Uo) < 1e-8
    from gpt_amd._lib import GPTError
    with pytest.raises(GPTError):
        T().GPT_inf(X, y, 0.3, n, r, 1.0, q, 5, 2, 0, I=I + 5)            # I out of 1..r
    with pytest.raises(GPTError):
        T().GPT_inf(X, y, 0.3, n, 7, 1.0, q, 5, 2, 0)                     # rank not instantiated


def test_tensor_res_matches_oracle():
    n, D, N, r, q, sigma, iters, burnin = 10, 4, 300, 5, 100, 0.2299, 3, 1
    X, y = data(N + 120, D, 9)
    Xtr, ytr, Xte, yte = X[:N], y[:N], X[N:], y[N:]
    got = T().TensorRes(Xtr, ytr, sigma, n, r, 1.4332, q, 123, iters, burnin, Xte, yte)
    b = oracle_b(R.datawhitening(Xtr), n, 1.4332, 123)
    W, U, I = R.GPT_inf(b, R.datawhitening(ytr), sigma, n, r, q, iters, burnin, 123)
    bt = oracle_b(R.datawhitening(Xte), n, 1.4332, 123)
    yfit = np.mean([R.pred(W[:, s], U[..., s], I, bt) for s in range(W.shape[1])], axis=0)
    want = yte.std(ddof=1) * math.sqrt(np.mean((yfit - R.datawhitening(yte)) ** 2))
    assert abs(got - want) <= 1e-9 * want
    assert 0 < got < 2 * yte.std(ddof=1)
