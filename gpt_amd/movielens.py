"""MovieLens-100k tensor collaborative filtering (100k_movielensExperiment.jl, §8(f) item 1 /
BASELINE config 5) on libgptsgld.so.

    GPT_fullw_sideinfo(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, sigma_w,
                       w_init, m, epsw, epsU, a, b, c, burnin, maxepoch, param_seed,
                       ytrainMean, ytrainStd; langevin=False, stiefel=False, avg=False)
                                                             100k_movielensExperiment.jl:409-551
    GPT_fullw_gibbs(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, sigma_w,
                    w_init, burnin, maxepoch, n_samples, param_seed, ytrainMean, ytrainStd;
                    avg=False, rotated_w=False)              100k_movielensExperiment.jl:1032-1129
    GPT_fullw_sideinfo_folds(Ratings, UserData, MovieData, Ratingtests, ..., ytrainMeans,
                             ytrainStds; ...)   the folds loop of :733-736 as one device launch
                                                per epoch (a list of per-fold result tuples)
    GPT_fixw_sideinfo(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, w, m, epsU,
                      a, b, c, burnin, maxepoch, param_seed, ytrainMean, ytrainStd;
                      langevin, stiefel, avg)                  :282-404
    GPT_fullw(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, sigma_w, w_init, m,
              epsw, epsU, burnin, maxepoch, param_seed, ytrainMean, ytrainStd;
              langevin, stiefel, avg)                          :160-279
    GPT_fixw(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, w, m, epsU, burnin,
             maxepoch, param_seed, ytrainMean, ytrainStd; langevin, stiefel, avg)     :56-156
    GPT_fixw_gibbs(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, w, burnin,
                   maxepoch, n_samples, param_seed, ytrainMean, ytrainStd; avg, rotated_w)
                                                             :945-1028
    fold(data, i)     the standardised u{i}.base / u{i}.test split of :566-576

Same argument meaning and return tuple as the reference: (w_store, U_store, V_store,
testpred_store, trainRMSEvec, testRMSEvec), without w_store for the fixed-w variants.  ``data`` is the mapping written by
scripts/make_ml100k_fixture.py (ratings per fold, the processed UserData / MovieData of
:578-584).  Randomness follows the framework's Philox contract (oracle/movielens_ref.py).
"""
import ctypes as C

import numpy as np

from ._lib import P_D, check, lib
from . import _lib

__all__ = ["GPT_fullw_sideinfo", "GPT_fullw_sideinfo_folds", "GPT_fixw_sideinfo", "GPT_fullw", "GPT_fixw", "GPT_fullw_gibbs",
           "GPT_fixw_gibbs", "fold"]


def _f64(a):
    return np.asfortranarray(np.asarray(a, dtype=np.float64))


def _ptr(a):
    return a.ctypes.data_as(P_D)


def fold(data, i):
    """(Ratingtrain, Ratingtest, UserData, MovieData, ytrainMean, ytrainStd) of fold i (1..5),
    ratings standardised with the training mean / std (:570-575)."""
    tr = np.asarray(data["u%d_base" % i], dtype=np.float64).copy()
    te = np.asarray(data["u%d_test" % i], dtype=np.float64).copy()
    mu, sd = tr[:, 2].mean(), tr[:, 2].std(ddof=1)
    tr[:, 2] = (tr[:, 2] - mu) / sd
    te[:, 2] = (te[:, 2] - mu) / sd
    return (tr, te, np.asarray(data["user_data"], dtype=np.float64),
            np.asarray(data["movie_data"], dtype=np.float64), mu, sd)


def GPT_fullw_sideinfo(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, sigma_w,
                       w_init, m, epsw, epsU, a, b, c, burnin, maxepoch, param_seed, ytrainMean,
                       ytrainStd, langevin=False, stiefel=False, avg=False):
    Rt = _f64(Rating)
    Rs = _f64(Ratingtest)
    Ud = _f64(UserData)
    Md = _f64(MovieData)
    w0 = _f64(w_init)
    N, Ntest = Rt.shape[0], Rs.shape[0]
    n1, D1 = Ud.shape
    n2, D2 = Md.shape
    r = w0.shape[0]
    if Rt.shape[1] < 3 or Rs.shape[1] < 3 or w0.shape != (r, r):
        raise ValueError("Rating / Ratingtest need (user, movie, rating) columns; w_init is r x r")
    w_store = np.zeros((r, r, maxepoch), order="F")
    U_store = np.zeros((n1 + D1, r, maxepoch), order="F")
    V_store = np.zeros((n2 + D2, r, maxepoch), order="F")
    tps = np.zeros((Ntest, maxepoch), order="F")
    trm = np.zeros(maxepoch)
    tsm = np.zeros(maxepoch)
    code = lib().gpt_cf_fullw_sideinfo(
        _ptr(Rt), N, N, _ptr(Ud), n1, D1, _ptr(Md), n2, D2, _ptr(Rs), Ntest, Ntest,
        float(signal_var), float(sigma_u), float(sigma_w), _ptr(w0), r, int(m), float(epsw),
        float(epsU), float(a), float(b), float(c), int(burnin), int(maxepoch),
        int(param_seed) & (2 ** 64 - 1), float(ytrainMean), float(ytrainStd), int(bool(langevin)),
        int(bool(stiefel)), int(bool(avg)), _ptr(w_store), _ptr(U_store), _ptr(V_store),
        _ptr(tps), _ptr(trm), _ptr(tsm))
    if code == _lib.GPT_ERR_NAN_GEODESIC:
        print("Get NaN when moving along Geodesic. Try smaller epsU")
    else:
        check(code)
    return w_store, U_store, V_store, tps, trm, tsm


def GPT_fullw_gibbs(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, sigma_w, w_init,
                    burnin, maxepoch, n_samples, param_seed, ytrainMean, ytrainStd, avg=False,
                    rotated_w=False):
    Rt = _f64(Rating)
    Rs = _f64(Ratingtest)
    w0 = _f64(w_init)
    N, Ntest = Rt.shape[0], Rs.shape[0]
    n1, n2 = np.shape(UserData)[0], np.shape(MovieData)[0]
    r = w0.shape[0]
    w_store = np.zeros((r, r, maxepoch), order="F")
    U_store = np.zeros((n1, r, maxepoch), order="F")
    V_store = np.zeros((n2, r, maxepoch), order="F")
    tps = np.zeros((Ntest, maxepoch), order="F")
    trm = np.zeros(maxepoch)
    tsm = np.zeros(maxepoch)
    check(lib().gpt_cf_fullw_gibbs(
        _ptr(Rt), N, N, n1, n2, _ptr(Rs), Ntest, Ntest, float(signal_var), float(sigma_u),
        float(sigma_w), _ptr(w0), r, int(burnin), int(maxepoch), int(n_samples),
        int(param_seed) & (2 ** 64 - 1), float(ytrainMean), float(ytrainStd), int(bool(avg)),
        int(bool(rotated_w)), _ptr(w_store), _ptr(U_store), _ptr(V_store), _ptr(tps), _ptr(trm),
        _ptr(tsm)))
    return w_store, U_store, V_store, tps, trm, tsm


def _sgd_common(Rating, Ratingtest, w, maxepoch):
    Rt, Rs, w0 = _f64(Rating), _f64(Ratingtest), _f64(w)
    r = w0.shape[0]
    if Rt.shape[1] < 3 or Rs.shape[1] < 3 or w0.shape != (r, r):
        raise ValueError("Rating / Ratingtest need (user, movie, rating) columns; w is r x r")
    Ntest = Rs.shape[0]
    return (Rt, Rs, w0, r, np.zeros((Ntest, maxepoch), order="F"), np.zeros(maxepoch),
            np.zeros(maxepoch))


def _nan_or_check(code):
    if code == _lib.GPT_ERR_NAN_GEODESIC:
        print("Get NaN when moving along Geodesic. Try smaller epsU")
    else:
        check(code)


def GPT_fixw_sideinfo(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, w, m, epsU,
                      a, b, c, burnin, maxepoch, param_seed, ytrainMean, ytrainStd,
                      langevin=False, stiefel=False, avg=False):
    """100k_movielensExperiment.jl:282-404 -> (U_store, V_store, testpred_store, trainRMSEvec,
    testRMSEvec)."""
    Rt, Rs, w0, r, tps, trm, tsm = _sgd_common(Rating, Ratingtest, w, maxepoch)
    Ud, Md = _f64(UserData), _f64(MovieData)
    n1, D1 = Ud.shape
    n2, D2 = Md.shape
    U_store = np.zeros((n1 + D1, r, maxepoch), order="F")
    V_store = np.zeros((n2 + D2, r, maxepoch), order="F")
    _nan_or_check(lib().gpt_cf_fixw_sideinfo(
        _ptr(Rt), Rt.shape[0], Rt.shape[0], _ptr(Ud), n1, D1, _ptr(Md), n2, D2, _ptr(Rs),
        Rs.shape[0], Rs.shape[0], float(signal_var), float(sigma_u), _ptr(w0), r, int(m),
        float(epsU), float(a), float(b), float(c), int(burnin), int(maxepoch),
        int(param_seed) & (2 ** 64 - 1), float(ytrainMean), float(ytrainStd), int(bool(langevin)),
        int(bool(stiefel)), int(bool(avg)), _ptr(U_store), _ptr(V_store), _ptr(tps), _ptr(trm),
        _ptr(tsm)))
    return U_store, V_store, tps, trm, tsm


def GPT_fullw(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, sigma_w, w_init, m,
              epsw, epsU, burnin, maxepoch, param_seed, ytrainMean, ytrainStd, langevin=False,
              stiefel=False, avg=False):
    """100k_movielensExperiment.jl:160-279 (no side information) -> (w_store, U_store, V_store,
    testpred_store, trainRMSEvec, testRMSEvec)."""
    Rt, Rs, w0, r, tps, trm, tsm = _sgd_common(Rating, Ratingtest, w_init, maxepoch)
    n1, n2 = np.shape(UserData)[0], np.shape(MovieData)[0]
    w_store = np.zeros((r, r, maxepoch), order="F")
    U_store = np.zeros((n1, r, maxepoch), order="F")
    V_store = np.zeros((n2, r, maxepoch), order="F")
    _nan_or_check(lib().gpt_cf_fullw(
        _ptr(Rt), Rt.shape[0], Rt.shape[0], n1, n2, _ptr(Rs), Rs.shape[0], Rs.shape[0],
        float(signal_var), float(sigma_u), float(sigma_w), _ptr(w0), r, int(m), float(epsw),
        float(epsU), int(burnin), int(maxepoch), int(param_seed) & (2 ** 64 - 1),
        float(ytrainMean), float(ytrainStd), int(bool(langevin)), int(bool(stiefel)),
        int(bool(avg)), _ptr(w_store), _ptr(U_store), _ptr(V_store), _ptr(tps), _ptr(trm),
        _ptr(tsm)))
    return w_store, U_store, V_store, tps, trm, tsm


def GPT_fixw(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, w, m, epsU, burnin,
             maxepoch, param_seed, ytrainMean, ytrainStd, langevin=False, stiefel=False,
             avg=False):
    """100k_movielensExperiment.jl:56-156 (no side information, w fixed) -> (U_store, V_store,
    testpred_store, trainRMSEvec, testRMSEvec)."""
    Rt, Rs, w0, r, tps, trm, tsm = _sgd_common(Rating, Ratingtest, w, maxepoch)
    n1, n2 = np.shape(UserData)[0], np.shape(MovieData)[0]
    U_store = np.zeros((n1, r, maxepoch), order="F")
    V_store = np.zeros((n2, r, maxepoch), order="F")
    _nan_or_check(lib().gpt_cf_fixw(
        _ptr(Rt), Rt.shape[0], Rt.shape[0], n1, n2, _ptr(Rs), Rs.shape[0], Rs.shape[0],
        float(signal_var), float(sigma_u), _ptr(w0), r, int(m), float(epsU), int(burnin),
        int(maxepoch), int(param_seed) & (2 ** 64 - 1), float(ytrainMean), float(ytrainStd),
        int(bool(langevin)), int(bool(stiefel)), int(bool(avg)), _ptr(U_store), _ptr(V_store),
        _ptr(tps), _ptr(trm), _ptr(tsm)))
    return U_store, V_store, tps, trm, tsm


def GPT_fixw_gibbs(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, w, burnin,
                   maxepoch, n_samples, param_seed, ytrainMean, ytrainStd, avg=False,
                   rotated_w=False):
    """100k_movielensExperiment.jl:945-1028 -> (U_store, V_store, testpred_store, trainRMSEvec,
    testRMSEvec)."""
    Rt, Rs, w0, r, tps, trm, tsm = _sgd_common(Rating, Ratingtest, w, maxepoch)
    n1, n2 = np.shape(UserData)[0], np.shape(MovieData)[0]
    U_store = np.zeros((n1, r, maxepoch), order="F")
    V_store = np.zeros((n2, r, maxepoch), order="F")
    check(lib().gpt_cf_fixw_gibbs(
        _ptr(Rt), Rt.shape[0], Rt.shape[0], n1, n2, _ptr(Rs), Rs.shape[0], Rs.shape[0],
        float(signal_var), float(sigma_u), _ptr(w0), r, int(burnin), int(maxepoch),
        int(n_samples), int(param_seed) & (2 ** 64 - 1), float(ytrainMean), float(ytrainStd),
        int(bool(avg)), int(bool(rotated_w)), _ptr(U_store), _ptr(V_store), _ptr(tps), _ptr(trm),
        _ptr(tsm)))
    return U_store, V_store, tps, trm, tsm


def last_timing():
    """Device time of the last CF SGD / SGLD call on this thread (gpt_cf_last_timing): dict with
    epoch_ms (cf_epoch_kernel launches), eval_ms (cf_eval_kernel), epochs, fold_steps and mode
    (gpt_cf_last_mode: 0 batch-phase + move launches per step, 1 Stiefel epoch launch, 2 lazy SGD
    epoch launch)."""
    em, vm = C.c_double(), C.c_double()
    ne, fs = C.c_int64(), C.c_int64()
    check(lib().gpt_cf_last_timing(C.byref(em), C.byref(vm), C.byref(ne), C.byref(fs)))
    mode = C.c_int32()
    check(lib().gpt_cf_last_mode(C.byref(mode)))
    return dict(epoch_ms=em.value, eval_ms=vm.value, epochs=ne.value, fold_steps=fs.value,
                mode=mode.value)


def GPT_fullw_sideinfo_folds(Ratings, UserData, MovieData, Ratingtests, signal_var, sigma_u,
                             sigma_w, w_init, m, epsw, epsU, a, b, c, burnin, maxepoch, param_seed,
                             ytrainMeans, ytrainStds, langevin=False, stiefel=False, avg=False):
    """The per-fold loop of 100k_movielensExperiment.jl:733-736 (GPT_fullw_sideinfo on fold i
    with its own ratings and ytrainMean[i] / ytrainStd[i], one param_seed) with the folds as
    sibling chains of one device launch per epoch.  Returns one (w_store, U_store, V_store,
    testpred_store, trainRMSEvec, testRMSEvec) tuple per fold — the same values as separate
    GPT_fullw_sideinfo calls; a fold that hit the geodesic NaN keeps zero parameter stores."""
    F = len(Ratings)
    if len(Ratingtests) != F or len(ytrainMeans) != F or len(ytrainStds) != F:
        raise ValueError("one test set, ytrainMean and ytrainStd per fold")
    Rts = [_f64(R) for R in Ratings]
    Rss = [_f64(R) for R in Ratingtests]
    Ud, Md, w0 = _f64(UserData), _f64(MovieData), _f64(w_init)
    n1, D1 = Ud.shape
    n2, D2 = Md.shape
    r = w0.shape[0]
    outs = []
    for Rs in Rss:
        outs.append((np.zeros((r, r, maxepoch), order="F"),
                     np.zeros((n1 + D1, r, maxepoch), order="F"),
                     np.zeros((n2 + D2, r, maxepoch), order="F"),
                     np.zeros((Rs.shape[0], maxepoch), order="F"), np.zeros(maxepoch),
                     np.zeros(maxepoch)))
    PP = C.c_void_p * F
    ptrs = lambda arrs: PP(*[a.ctypes.data for a in arrs])
    Ns = np.array([R.shape[0] for R in Rts], dtype=np.int64)
    Nts = np.array([R.shape[0] for R in Rss], dtype=np.int64)
    ym = _f64(np.asarray(ytrainMeans, dtype=np.float64))
    ys = _f64(np.asarray(ytrainStds, dtype=np.float64))
    st = np.zeros(F, dtype=np.int32)
    code = lib().gpt_cf_fullw_sideinfo_folds(
        F, ptrs(Rts), Ns.ctypes.data, ptrs(Rss), Nts.ctypes.data, _ptr(Ud), n1, D1, _ptr(Md), n2,
        D2, float(signal_var), float(sigma_u), float(sigma_w), _ptr(w0), r, int(m), float(epsw),
        float(epsU), float(a), float(b), float(c), int(burnin), int(maxepoch),
        int(param_seed) & (2 ** 64 - 1), _ptr(ym), _ptr(ys), int(bool(langevin)),
        int(bool(stiefel)), int(bool(avg)), ptrs([o[0] for o in outs]),
        ptrs([o[1] for o in outs]), ptrs([o[2] for o in outs]), ptrs([o[3] for o in outs]),
        ptrs([o[4] for o in outs]), ptrs([o[5] for o in outs]),
        st.ctypes.data_as(_lib.P_I32))
    _nan_or_check(code)
    return outs
