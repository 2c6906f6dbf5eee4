"""GPU parity of the MovieLens-100k tensor CF sampler (GPT_fullw_sideinfo,
100k_movielensExperiment.jl:409-551; §8(f) item 1, BASELINE config 5) against the oracle.

Data: the reference's ml-100k files as processed by :561-586 (tests/golden/ml100k.npz, built by
scripts/make_ml100k_fixture.py).  Tolerances (fp64; the device sums gradient rows and feature
sums in the reference's rating order but forms (e·sumV)·wᵀ as e·(sumV·wᵀ)):
  w / U / V stores       max |Δ| <= 1e-8·max|x|
  test predictions       max |Δ| <= 1e-8 (rating scale)
  train / test RMSE      relative <= 1e-9
"""
import os

import numpy as np
import pytest

from oracle import movielens_ref as M

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "ml100k.npz")


def rel(a, b):
    a = np.asarray(a); b = np.asarray(b)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def problem(ntr, nte, fold=1):
    from gpt_amd import movielens
    d = np.load(GOLD)
    tr, te, ud, md, mu, sd = movielens.fold(d, fold)
    return tr[:ntr], te[:nte], ud, md, mu, sd


CASES = {
    # name: (ntrain, ntest, r, m, epochs, burnin, langevin, stiefel, avg, epsw, epsU)
    "sgd_euclid_live": (3000, 1000, 4, 100, 2, 0, False, False, False, 1e-4, 1e-6),
    "sgld_euclid_avg": (2950, 800, 5, 64, 3, 1, True, False, True, 1e-4, 1e-6),
    "sgd_stiefel": (3000, 1000, 4, 100, 2, 0, False, True, False, 1e-4, 1e-4),
    "sgld_stiefel": (2950, 800, 3, 64, 2, 0, True, True, True, 1e-4, 1e-4),
}


@pytest.mark.parametrize("name", list(CASES))
def test_fullw_sideinfo_matches_oracle(name):
    from gpt_amd import movielens
    ntr, nte, r, m, ep, bi, lang, stf, avg, epsw, epsU = CASES[name]
    tr, te, ud, md, mu, sd = problem(ntr, nte)
    w0 = np.random.default_rng(5).standard_normal((r, r))
    args = (tr, ud, md, te, 0.8, 0.1, 1.0, w0, m, epsw, epsU, 0.5, 0.25, 0.5, bi, ep, 17, mu, sd)
    got = movielens.GPT_fullw_sideinfo(*args, langevin=lang, stiefel=stf, avg=avg)
    want = M.GPT_fullw_sideinfo(*args, langevin=lang, stiefel=stf, avg=avg)
    for g, w_, tol in zip(got[:3], want[:3], (1e-8, 1e-8, 1e-8)):
        assert rel(g, w_) < tol, rel(g, w_)
    assert np.abs(got[3] - want[3]).max() < 1e-8
    assert np.all(np.abs(got[4] - want[4]) <= 1e-9 * want[4])
    assert np.all(np.abs(got[5] - want[5]) <= 1e-9 * want[5])


@pytest.mark.parametrize("lang", [False, True])
def test_fullw_sideinfo_wide_side_information(lang):
    """More than 64 side-information columns per side (synthetic 0/1 features appended to the
    ml-100k ones: 28 + 40 user, 18 + 50 movie columns) take the kernel's CSR path instead of the
    64-bit feature masks; against the oracle."""
    from gpt_amd import movielens
    tr, te, ud, md, mu, sd = problem(3000, 1000)
    rng = np.random.default_rng(11)
    ud2 = np.hstack([ud, (rng.random((ud.shape[0], 40)) < 0.05).astype(np.float64)])
    md2 = np.hstack([md, (rng.random((md.shape[0], 50)) < 0.05).astype(np.float64)])
    assert ud2.shape[1] > 64 and md2.shape[1] > 64
    w0 = np.random.default_rng(5).standard_normal((4, 4))
    args = (tr, ud2, md2, te, 0.8, 0.1, 1.0, w0, 100, 1e-4, 1e-6, 0.5, 0.25, 0.5, 0, 2, 17, mu, sd)
    got = movielens.GPT_fullw_sideinfo(*args, langevin=lang)
    want = M.GPT_fullw_sideinfo(*args, langevin=lang)
    for g, w_ in zip(got[:3], want[:3]):
        assert rel(g, w_) < 1e-8, rel(g, w_)
    assert np.all(np.abs(got[5] - want[5]) <= 1e-9 * want[5])


@pytest.mark.parametrize("m,r,cols", [(200, 4, None), (1100, 1, 1)])
def test_fullw_sideinfo_lazy_move_wide_batches(m, r, cols):
    """The lazy SGD move (cf_epoch_kernel domove = 2, the default for SGD on the feature-mask path)
    past the bitonic-link batch (B <= 128): m = 200 takes the per-pair link walk; m = 1100
    (> 1024 threads) also loads its batches without the prefetch — its LDS carve fits only at
    r = 1 with one side-information column per side (the first of ml-100k's).  Against the
    oracle's dense per-step move, with the launch mode asserted."""
    from gpt_amd import movielens
    tr, te, ud, md, mu, sd = problem(3300, 1000)
    if cols:
        ud, md = np.ascontiguousarray(ud[:, :cols]), np.ascontiguousarray(md[:, :cols])
    w0 = np.random.default_rng(5).standard_normal((r, r))
    args = (tr, ud, md, te, 0.8, 0.1, 1.0, w0, m, 1e-4, 1e-6, 0.5, 0.25, 0.5, 0, 2, 17, mu, sd)
    got = movielens.GPT_fullw_sideinfo(*args)
    assert movielens.last_timing()["mode"] == 2
    want = M.GPT_fullw_sideinfo(*args)
    for g, w_ in zip(got[:3], want[:3]):
        assert rel(g, w_) < 1e-8, rel(g, w_)
    assert np.abs(got[3] - want[3]).max() < 1e-8
    assert np.all(np.abs(got[5] - want[5]) <= 1e-9 * want[5])


def test_fullw_sideinfo_lazy_equals_eager_move(monkeypatch):
    """The lazy SGD move (m·c^Δ for the rows a batch skips) against the per-step dense move of
    every row (GPTSGLD_CF_LAZY=0: a batch-phase launch and a row-parallel move launch per step, the
    reference's order of operations), 2 epochs of the live configuration's shape on 20 000
    ratings at r = 20: stores within the 1e-8 store tolerance, test RMSE within 1e-9."""
    from gpt_amd import movielens
    tr, te, ud, md, mu, sd = problem(20000, 5000)
    w0 = np.random.default_rng(17).standard_normal((20, 20))
    args = (tr, ud, md, te, 0.8, 0.1, 1.0, w0, 100, 1e-4, 1e-6, 0.5, 0.25, 0.5, 0, 2, 17, mu, sd)
    lazy = movielens.GPT_fullw_sideinfo(*args)
    assert movielens.last_timing()["mode"] == 2
    monkeypatch.setenv("GPTSGLD_CF_LAZY", "0")
    eager = movielens.GPT_fullw_sideinfo(*args)
    assert movielens.last_timing()["mode"] == 0
    for g, w_ in zip(lazy[:3], eager[:3]):
        assert rel(g, w_) < 1e-8, rel(g, w_)
    assert np.all(np.abs(lazy[5] - eager[5]) <= 1e-9 * eager[5])


def test_fullw_sideinfo_live_config_full_fold():
    """The live run of :723-730 (r = 15, m = 100, SGD, a/b/c = 0.5/0.25/0.5) for one epoch of
    fold 1 (80 000 ratings), against the oracle."""
    from gpt_amd import movielens
    tr, te, ud, md, mu, sd = problem(80000, 20000)
    w0 = np.random.default_rng(17).standard_normal((15, 15))
    args = (tr, ud, md, te, 0.8, 0.1, 1.0, w0, 100, 1e-4, 1e-6, 0.5, 0.25, 0.5, 0, 1, 17, mu, sd)
    got = movielens.GPT_fullw_sideinfo(*args)
    want = M.GPT_fullw_sideinfo(*args)
    assert rel(got[0], want[0]) < 1e-8 and rel(got[1], want[1]) < 1e-8 and rel(got[2], want[2]) < 1e-8
    assert abs(got[5][0] - want[5][0]) <= 1e-9 * want[5][0]
    assert 0.8 < got[5][0] < 1.3                      # test RMSE on the 1..5 rating scale


GIBBS_CASES = {
    # name: (ntrain, ntest, r, burnin, maxepoch, n_samples, avg, rotated_w)
    "plain": (3000, 1000, 4, 0, 2, 1, False, False),
    "avg_rotated": (2500, 700, 3, 1, 2, 2, True, True),
    "r15_fold": (6000, 1500, 15, 0, 1, 1, False, False),      # r = 15 of :723 (r² = 225 design)
}


@pytest.mark.parametrize("name", list(GIBBS_CASES))
def test_fullw_gibbs_matches_oracle(name):
    """GPT_fullw_gibbs (100k_movielensExperiment.jl:1032-1129): per-user / per-movie r × r
    conditionals in one wave each, w | U, V through the fp64-MFMA SYRK of the Kronecker design."""
    from gpt_amd import movielens
    ntr, nte, r, bi, ep, ns, avg, rot = GIBBS_CASES[name]
    tr, te, ud, md, mu, sd = problem(ntr, nte)
    w0 = np.random.default_rng(9).standard_normal((r, r))
    args = (tr, ud, md, te, 0.8, 0.5, 1.0, w0, bi, ep, ns, 17, mu, sd)
    got = movielens.GPT_fullw_gibbs(*args, avg=avg, rotated_w=rot)
    want = M.GPT_fullw_gibbs(*args, avg=avg, rotated_w=rot)
    for g, w_ in zip(got[:3], want[:3]):
        assert rel(g, w_) < 1e-8, rel(g, w_)
    assert np.abs(got[3] - want[3]).max() < 1e-8
    assert np.all(np.abs(got[4] - want[4]) <= 1e-9 * want[4])
    assert np.all(np.abs(got[5] - want[5]) <= 1e-9 * want[5])


# The other CF variants of 100k_movielensExperiment.jl: GPT_fixw_sideinfo (:282-404), GPT_fullw
# (:160-279), GPT_fixw (:56-156) on the same device kernels (w fixed / no feature rows / their
# own U, V initialisations), GPT_fixw_gibbs (:945-1028) on the Gibbs kernels without the w draw.
VARIANT_CASES = {
    # name: (ntrain, ntest, r, m, epochs, burnin, langevin, stiefel, avg, epsU)
    "sgd_euclid": (3000, 1000, 4, 100, 2, 0, False, False, False, 1e-6),
    "sgld_euclid_avg": (2950, 800, 5, 64, 3, 1, True, False, True, 1e-6),
    "sgld_stiefel": (2950, 800, 3, 64, 2, 0, True, True, True, 1e-4),
}


def _check_tail(got, want):
    """(…, testpred_store, trainRMSE, testRMSE) tails of the variant tuples."""
    assert np.abs(got[-3] - want[-3]).max() < 1e-8
    assert np.all(np.abs(got[-2] - want[-2]) <= 1e-9 * want[-2])
    assert np.all(np.abs(got[-1] - want[-1]) <= 1e-9 * want[-1])


@pytest.mark.parametrize("name", list(VARIANT_CASES))
def test_fixw_sideinfo_matches_oracle(name):
    from gpt_amd import movielens
    ntr, nte, r, m, ep, bi, lang, stf, avg, epsU = VARIANT_CASES[name]
    tr, te, ud, md, mu, sd = problem(ntr, nte)
    w = np.random.default_rng(6).standard_normal((r, r))
    args = (tr, ud, md, te, 0.8, 0.1, w, m, epsU, 0.5, 0.25, 0.5, bi, ep, 17, mu, sd)
    got = movielens.GPT_fixw_sideinfo(*args, langevin=lang, stiefel=stf, avg=avg)
    want = M.GPT_fixw_sideinfo(*args, langevin=lang, stiefel=stf, avg=avg)
    assert len(got) == len(want) == 5
    assert got[0].shape == (ud.shape[0] + ud.shape[1], r, ep)
    for g, w_ in zip(got[:2], want[:2]):
        assert rel(g, w_) < 1e-8, rel(g, w_)
    _check_tail(got, want)


@pytest.mark.parametrize("name", list(VARIANT_CASES))
def test_fullw_no_side_matches_oracle(name):
    from gpt_amd import movielens
    ntr, nte, r, m, ep, bi, lang, stf, avg, epsU = VARIANT_CASES[name]
    tr, te, ud, md, mu, sd = problem(ntr, nte)
    w0 = np.random.default_rng(7).standard_normal((r, r))
    args = (tr, ud, md, te, 0.8, 0.1, 1.0, w0, m, 1e-4, epsU, bi, ep, 17, mu, sd)
    got = movielens.GPT_fullw(*args, langevin=lang, stiefel=stf, avg=avg)
    want = M.GPT_fullw(*args, langevin=lang, stiefel=stf, avg=avg)
    assert got[1].shape == (ud.shape[0], r, ep)                   # no feature rows
    for g, w_ in zip(got[:3], want[:3]):
        assert rel(g, w_) < 1e-8, rel(g, w_)
    _check_tail(got, want)


@pytest.mark.parametrize("name", list(VARIANT_CASES))
def test_fixw_no_side_matches_oracle(name):
    from gpt_amd import movielens
    ntr, nte, r, m, ep, bi, lang, stf, avg, epsU = VARIANT_CASES[name]
    tr, te, ud, md, mu, sd = problem(ntr, nte)
    w = np.random.default_rng(8).standard_normal((r, r))
    args = (tr, ud, md, te, 0.8, 0.1, w, m, epsU, bi, ep, 17, mu, sd)
    got = movielens.GPT_fixw(*args, langevin=lang, stiefel=stf, avg=avg)
    want = M.GPT_fixw(*args, langevin=lang, stiefel=stf, avg=avg)
    assert len(got) == 5 and got[0].shape == (ud.shape[0], r, ep)
    for g, w_ in zip(got[:2], want[:2]):
        assert rel(g, w_) < 1e-8, rel(g, w_)
    _check_tail(got, want)


@pytest.mark.parametrize("rotated", [False, True])
def test_fixw_gibbs_matches_oracle(rotated):
    from gpt_amd import movielens
    tr, te, ud, md, mu, sd = problem(3000, 800)
    w = np.random.default_rng(9).standard_normal((4, 4))
    args = (tr, ud, md, te, 0.8, 0.5, w, 1, 2, 2, 17, mu, sd)
    got = movielens.GPT_fixw_gibbs(*args, avg=True, rotated_w=rotated)
    want = M.GPT_fixw_gibbs(*args, avg=True, rotated_w=rotated)
    assert len(got) == 5
    for g, w_ in zip(got[:2], want[:2]):
        assert rel(g, w_) < 1e-8, rel(g, w_)
    _check_tail(got, want)


@pytest.mark.parametrize("lang,stf,avg", [(False, False, False), (True, True, True)])
def test_sideinfo_folds_equal_separate_runs(lang, stf, avg):
    """The folds loop of :733-736 as one launch per epoch (gpt_cf_fullw_sideinfo_folds) gives
    every fold exactly the values of its own GPT_fullw_sideinfo call (bit-identical: the same
    kernels, one chain per fold)."""
    from gpt_amd import movielens
    d = np.load(GOLD)
    folds = [movielens.fold(d, i) for i in (1, 2, 3)]
    trs = [f[0][:3000] for f in folds]
    tes = [f[1][:700 + 50 * i] for i, f in enumerate(folds)]       # test sets of different sizes
    ud, md = folds[0][2], folds[0][3]
    mus = [f[4] for f in folds]
    sds = [f[5] for f in folds]
    w0 = np.random.default_rng(5).standard_normal((4, 4))
    epsU = 1e-4 if stf else 1e-6
    common = (0.8, 0.1, 1.0, w0, 100, 1e-4, epsU, 0.5, 0.25, 0.5, 0, 3, 17)
    got = movielens.GPT_fullw_sideinfo_folds(trs, ud, md, tes, *common, mus, sds, langevin=lang,
                                             stiefel=stf, avg=avg)
    assert len(got) == 3
    for f in range(3):
        want = movielens.GPT_fullw_sideinfo(trs[f], ud, md, tes[f], *common, mus[f], sds[f],
                                            langevin=lang, stiefel=stf, avg=avg)
        for g, w_ in zip(got[f], want):
            assert g.shape == w_.shape
            assert np.array_equal(g, w_)


@pytest.mark.parametrize("p", [1, 5, 16, 17, 100, 225, 400, 1023, 1024, 1100])
def test_gaussian_draw_blocked_cholesky_and_solves(p):
    """The Gibbs samplers' Gaussian conditional draw (tgp.hip gaussian_draw_prec: blocked MFMA
    Cholesky + blocked triangular solves for p <= 1024, the column kernels past it) against numpy:
    out = L⁻ᵀz + M⁻¹x for M = L·Lᵀ, z the Philox normals of the draw's stream.  Sizes: one panel
    and partial panels (1, 5, 16, 17), the TGP / MovieLens sizes (100, 225 = 15², 400 = 20²), the
    blocked limit (1023, 1024) and the fallback (1100)."""
    import ctypes as C
    from gpt_amd import _lib
    from oracle import philox as px
    rng = np.random.default_rng(p)
    A = rng.standard_normal((p, p + 3))
    M = np.asfortranarray(A @ A.T / p + 0.5 * np.eye(p))
    x = rng.standard_normal(p)
    out = np.zeros(p)
    st = np.zeros(1, dtype=np.int32)
    _lib.check(_lib.lib().gpt_debug_gaussian_draw(p, M.ctypes.data_as(_lib.P_D),
                                                  x.ctypes.data_as(_lib.P_D), 11, 3, 7, 0,
                                                  out.ctypes.data_as(_lib.P_D),
                                                  st.ctypes.data_as(_lib.P_I32)))
    assert st[0] == 0
    z = px.normals(p, 11, 3, 7, 0)
    L = np.linalg.cholesky(M)
    want = np.linalg.solve(L.T, z) + np.linalg.solve(M, x)
    assert np.abs(out - want).max() <= 1e-10 * np.abs(want).max(), np.abs(out - want).max()


def test_gaussian_draw_flags_non_spd():
    """A precision with a non-positive pivot sets the status (PosDefException in the reference)."""
    from gpt_amd import _lib
    p = 40
    M = np.asfortranarray(-np.eye(p))
    x = np.zeros(p)
    out = np.zeros(p)
    st = np.zeros(1, dtype=np.int32)
    _lib.check(_lib.lib().gpt_debug_gaussian_draw(p, M.ctypes.data_as(_lib.P_D),
                                                  x.ctypes.data_as(_lib.P_D), 1, 0, 0, 0,
                                                  out.ctypes.data_as(_lib.P_D),
                                                  st.ctypes.data_as(_lib.P_I32)))
    assert st[0] == 1
