"""The C++ fp64 CPU restatement (oracle/cpu/gpt_sgld_cpu.cpp, the bench's CPU baseline) against
the numpy oracle: same inputs, same Philox streams and permutations -> the same trajectory.

Tolerance: stores <= 1e-10 relative (both fp64; summation order differs, and the numpy oracle
divides in computeU_phi the same way)."""
import math

import numpy as np
import pytest

from oracle import gpt_sgld_ref as R

cpu = pytest.importorskip("oracle.cpu_lib")


def _problem(n, D, N, r, Q, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((N, D))
    Z = rng.standard_normal((n, D))
    b = 2 * np.pi * rng.random((n, D))
    phi = R.feature(X, 1.0 + 0.2 * rng.standard_normal(D), 1.0, math.sqrt(n / Q ** (1.0 / D)), Z, b)
    I = R.samplenz(r, D, Q, seed + 1)
    w, U = R.init_state(n, r, D, Q, seed + 2)
    y = R.pred(w, U, I, phi) + 0.05 * rng.standard_normal(N)
    return phi, y, I


@pytest.mark.parametrize("n,D,N,r,Q,m,epochs", [(24, 3, 50, 3, 12, 16, 2), (40, 4, 37, 5, 30, 10, 2),
                                                (16, 2, 20, 2, 4, 20, 3)])
def test_cpu_restatement_matches_oracle(n, D, N, r, Q, m, epochs):
    phi, y, I = _problem(n, D, N, r, Q)
    wo, Uo, info = R.GPTregression(phi, y, 0.05, I, r, Q, m, 1e-4, 1e-6, 1, epochs - 1, 7)
    got = cpu.GPTregression_chains(phi, y, 0.05, I, r, Q, m, 1e-4, 1e-6, 1, epochs - 1, [7],
                                   stores=True)
    assert got["status"][0] == 0 == info["status"]
    assert np.abs(got["w_store"] - wo).max() <= 1e-10 * np.abs(wo).max()
    assert np.abs(got["U_store"] - Uo).max() <= 1e-10 * np.abs(Uo).max()
    assert np.abs(got["w"][:, 0] - wo[:, -1]).max() <= 1e-10 * np.abs(wo).max()


def test_cpu_chains_are_independent_of_threading():
    phi, y, I = _problem(24, 3, 40, 3, 12)
    one = cpu.GPTregression_chains(phi, y, 0.05, I, 3, 12, 10, 1e-4, 1e-6, 0, 2, [1, 2, 3], threads=1)
    many = cpu.GPTregression_chains(phi, y, 0.05, I, 3, 12, 10, 1e-4, 1e-6, 0, 2, [1, 2, 3], threads=3)
    assert np.array_equal(one["w"], many["w"]) and np.array_equal(one["U"], many["U"])
    single = cpu.GPTregression_chains(phi, y, 0.05, I, 3, 12, 10, 1e-4, 1e-6, 0, 2, [2])
    assert np.array_equal(single["w"][:, 0], many["w"][:, 1])
    assert one["steps"] == 3 * 8


def test_cpu_nan_bailout_zero_fills():
    phi, y, I = _problem(16, 2, 20, 2, 4)
    got = cpu.GPTregression_chains(phi, y * 1e8, 1e-12, I, 2, 4, 5, 1.0, 1.0, 0, 2, [3], stores=True)
    wo, Uo, info = R.GPTregression(phi, y * 1e8, 1e-12, I, 2, 4, 5, 1.0, 1.0, 0, 2, 3)
    assert info["status"] == 1 and got["status"][0] == 1
    assert not got["w_store"].any() and not got["U_store"].any()


def test_cpu_pred_matches_oracle():
    """The CPU prediction baseline (gptcpu_pred) is pred of GPT_SGLD.jl:233-243 per sample."""
    rng = np.random.default_rng(5)
    n, D, Nt, r, Q, S = 20, 3, 57, 4, 30, 3
    phi = np.asfortranarray(rng.standard_normal((n, D, Nt)) * 0.3)
    w = rng.standard_normal((Q, S))
    U = rng.standard_normal((n, r, D, S)) * 0.3
    I = rng.integers(1, r + 1, size=(Q, D)).astype(np.int32)
    f, sec = cpu.pred(w, U, I, phi, threads=2)
    for s in range(S):
        want = R.pred(w[:, s], U[..., s], I, phi)
        assert np.abs(f[s] - want).max() <= 1e-12 * np.abs(want).max()
    assert sec >= 0.0
