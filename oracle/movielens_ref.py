"""CPU oracle for the MovieLens-100k tensor CF model (100k_movielensExperiment.jl, §8(f) item 1).

TEST INFRASTRUCTURE — NOT PRODUCT CODE.  Only ``tests/`` may import this module; the product
path (``gpt_amd.movielens`` + ``libgptsgld.so``) never touches ``oracle/``.

``GPT_fullw_sideinfo`` restates 100k_movielensExperiment.jl:409-551 rating by rating, with the
framework's Philox streams in place of Julia's MersenneTwister (oracle/philox.py):
  * epoch permutation: ``randperm(N, seed, epoch-1)`` of the ORIGINAL ratings (:451-452 — not
    cumulative, unlike GPTregression's ``phi=phi[:,:,perm]``);
  * U, V init (:424-428): Stiefel polar factor of Z = randn(r, rows) with Z on (CF_UV_INIT, 0/1)
    (element a + r·row), or sigma_u·randn(rows, r) on the same streams (element row + rows·l);
  * noise: w on (step, CF_W_NOISE, 0) (element i + r·j), U/V on (step, CF_UV_NOISE, 0/1) in
    u_noise's layout (element l + RE·row, RE = r rounded up to even).
Row indices are 0-based here: user u -> U row u, user feature f -> U row n1 + f (Uidx, :430-437).
"""
import math

import numpy as np

from . import gpt_sgld_ref as R
from . import philox as px


def side_rows(user_data, movie_data):
    """Uidx / Vidx of :430-437 (0-based rows of U and V)."""
    n1, n2 = user_data.shape[0], movie_data.shape[0]
    uidx = [n1 + np.flatnonzero(user_data[u]) for u in range(n1)]
    vidx = [n2 + np.flatnonzero(movie_data[v]) for v in range(n2)]
    return uidx, vidx


def cutoff(pred):
    """:49-52 — clamp predictions to [1, 5]."""
    return np.clip(pred, 1.0, 5.0)


def uv_noise(rows, r, seed, step, which):
    re = r + (r & 1)
    return px.normals(re * rows, seed, step, px.CF_UV_NOISE, which).reshape((rows, re))[:, :r]


def init_uv(rows, r, seed, which, stiefel, sigma_u, mode="side"):
    """U / V init: "side" (GPT_fullw_sideinfo :424-428) Stiefel polar factor or σ_u·randn;
    "sigma" (GPT_fixw*, :67 / :294) σ_u·randn also when stiefel; "unit" (GPT_fullw :175-180)
    polar factor or randn."""
    if stiefel and mode != "sigma":
        z = px.normals(r * rows, seed, 0, px.CF_UV_INIT, which).reshape((r, rows), order="F")
        return np.asfortranarray(R.stiefel_init(z))
    z = px.normals(rows * r, seed, 0, px.CF_UV_INIT, which).reshape((rows, r), order="F")
    return z if mode == "unit" else sigma_u * z


def predict(ratings, U, V, w, uidx, vidx, a, b, c):
    """a·sum((sumU*w).*sumV) for every (user, movie) row of ``ratings`` (:526-529)."""
    out = np.empty(len(ratings))
    for i, (u, v) in enumerate(ratings[:, :2].astype(np.int64) - 1):
        sumU = U[u] + b * U[uidx[u]].sum(axis=0)
        sumV = V[v] + c * V[vidx[v]].sum(axis=0)
        out[i] = a * np.sum((sumU @ w) * sumV)
    return out


def GPT_fullw_sideinfo(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, sigma_w,
                       w_init, m, epsw, epsU, a, b, c, burnin, maxepoch, param_seed, ytrainMean,
                       ytrainStd, langevin=False, stiefel=False, avg=False, fixw=False,
                       init="side"):
    """100k_movielensExperiment.jl:409-551 (fixw / init: the other SGD variants, below).  Rating (N, 3+) holds 1-based user / movie ids and
    the standardised rating.  Returns (w_store (r, r, T), U_store (n1+D1, r, T), V_store,
    testpred_store (Ntest, T), trainRMSEvec (T), testRMSEvec (T)), T = maxepoch; entries of
    epochs after an early stop (:545-547) stay 0 (10 for testRMSEvec, as :441)."""
    Rating = np.asarray(Rating, dtype=np.float64)
    Ratingtest = np.asarray(Ratingtest, dtype=np.float64)
    N, Ntest = len(Rating), len(Ratingtest)
    n1, D1 = UserData.shape
    n2, D2 = MovieData.shape
    nb = -(-N // m)
    w = np.array(w_init, dtype=np.float64, order="F")
    r = w.shape[0]
    w_store = np.zeros((r, r, maxepoch), order="F")
    U_store = np.zeros((n1 + D1, r, maxepoch), order="F")
    V_store = np.zeros((n2 + D2, r, maxepoch), order="F")
    testpred_store = np.zeros((Ntest, maxepoch), order="F")
    U = init_uv(n1 + D1, r, param_seed, 0, stiefel, sigma_u, init)
    V = init_uv(n2 + D2, r, param_seed, 1, stiefel, sigma_u, init)
    uidx, vidx = side_rows(UserData, MovieData)
    trainRMSE = np.zeros(maxepoch)
    testRMSE = 10.0 * np.ones(maxepoch)
    trainpred, testpred = np.zeros(N), np.zeros(Ntest)
    counter = testcounter = 0
    sq, sqw = math.sqrt(epsU), math.sqrt(epsw)
    step = 0

    def bail():
        return (np.zeros_like(w_store), np.zeros_like(U_store), np.zeros_like(V_store),
                testpred_store, trainRMSE, testRMSE)

    for epoch in range(1, burnin + maxepoch + 1):
        shuffled = Rating[px.randperm(N, param_seed, epoch - 1)]
        for batch in range(nb):
            br = shuffled[m * batch: min(m * (batch + 1), N)]
            B = len(br)
            gradw = np.zeros((r, r))
            gradU = np.zeros((n1 + D1, r))
            gradV = np.zeros((n2 + D2, r))
            for ii in range(B):
                u, v, rating = int(br[ii, 0]) - 1, int(br[ii, 1]) - 1, br[ii, 2]
                sumU = U[u] + b * U[uidx[u]].sum(axis=0)
                sumV = V[v] + c * V[vidx[v]].sum(axis=0)
                t = sumU @ w
                e = rating - a * np.sum(t * sumV)
                Utemp = (e * sumV) @ w.T
                Vtemp = (e * sumU) @ w
                gradw += e * np.outer(sumU, sumV) / signal_var          # kron(sumV', sumU')
                gradU[u] += a * Utemp / signal_var
                gradV[v] += a * Vtemp / signal_var
                gradU[uidx[u]] += a * b * Utemp / signal_var
                gradV[vidx[v]] += a * c * Vtemp / signal_var
            gradw = gradw * N / B - w / sigma_w ** 2
            gradU *= N / B
            gradV *= N / B
            if not fixw:                                             # GPT_fixw*: w is fixed
                w = w + epsw * gradw / 2
                if langevin:
                    w = w + sqw * px.normals(r * r, param_seed, step, px.CF_W_NOISE, 0).reshape((r, r), order="F")
            new = []
            for which, (M, G) in enumerate(((U, gradU), (V, gradV))):
                xi = uv_noise(M.shape[0], r, param_seed, step, which)
                if stiefel:
                    mom = R.proj(M, sq * G / 2 + (xi if langevin else 0.0))
                    Mn, ok = R.geod(M, mom, sq)
                    if not ok:
                        return bail()
                else:
                    Mn = M + epsU * (G - M / sigma_u ** 2) / 2
                    if langevin:
                        Mn = Mn + sq * xi
                new.append(Mn)
            U, V = new
            step += 1
        if epoch > burnin:
            s = epoch - burnin - 1
            w_store[:, :, s] = w
            U_store[:, :, s] = U
            V_store[:, :, s] = V
            if not avg:
                counter = 0
            trainpred = (trainpred * counter + predict(Rating, U, V, w, uidx, vidx, a, b, c)) / (counter + 1)
            ft = cutoff(trainpred * ytrainStd + ytrainMean)
            trainRMSE[s] = math.sqrt(np.sum((ytrainStd * Rating[:, 2] + ytrainMean - ft) ** 2) / N)
            testpred = (testpred * counter + predict(Ratingtest, U, V, w, uidx, vidx, a, b, c)) / (counter + 1)
            fs = cutoff(testpred * ytrainStd + ytrainMean)
            testpred_store[:, s] = fs
            testRMSE[s] = math.sqrt(np.sum((ytrainStd * Ratingtest[:, 2] + ytrainMean - fs) ** 2) / Ntest)
            counter += 1
            if epoch > 1 and s > 0 and testRMSE[s] > testRMSE[s - 1]:
                testcounter += 1
            else:
                testcounter = 0
        if testcounter >= 5:
            break
    return w_store, U_store, V_store, testpred_store, trainRMSE, testRMSE


def GPT_fixw_sideinfo(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, w, m, epsU,
                      a, b, c, burnin, maxepoch, param_seed, ytrainMean, ytrainStd,
                      langevin=False, stiefel=False, avg=False):
    """100k_movielensExperiment.jl:282-404: GPT_fullw_sideinfo with w fixed (no gradw, no w
    step) and U, V = σ_u·randn (:294, also under stiefel).  Returns (U_store, V_store,
    testpred_store, trainRMSE, testRMSE)."""
    out = GPT_fullw_sideinfo(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, 1.0, w,
                             m, 0.0, epsU, a, b, c, burnin, maxepoch, param_seed, ytrainMean,
                             ytrainStd, langevin, stiefel, avg, fixw=True, init="sigma")
    return out[1:]


def _no_side(UserData, MovieData):
    return np.zeros((np.shape(UserData)[0], 0)), np.zeros((np.shape(MovieData)[0], 0))


def GPT_fullw(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, sigma_w, w_init, m,
              epsw, epsU, burnin, maxepoch, param_seed, ytrainMean, ytrainStd, langevin=False,
              stiefel=False, avg=False):
    """100k_movielensExperiment.jl:160-279: no side information — pred = sum((U[user,:]*w).*
    V[movie,:]), gradw = kron(V[movie,:]', U[user,:]') (= the side-information model at a = 1,
    b = c = 0 with no feature rows); U, V = randn or the Stiefel polar init (:175-180)."""
    ud, md = _no_side(UserData, MovieData)
    return GPT_fullw_sideinfo(Rating, ud, md, Ratingtest, signal_var, sigma_u, sigma_w, w_init, m,
                              epsw, epsU, 1.0, 0.0, 0.0, burnin, maxepoch, param_seed, ytrainMean,
                              ytrainStd, langevin, stiefel, avg, init="unit")


def GPT_fixw(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, w, m, epsU, burnin,
             maxepoch, param_seed, ytrainMean, ytrainStd, langevin=False, stiefel=False,
             avg=False):
    """100k_movielensExperiment.jl:56-156: no side information, w fixed, U, V = σ_u·randn.
    Returns (U_store, V_store, testpred_store, trainRMSE, testRMSE)."""
    ud, md = _no_side(UserData, MovieData)
    out = GPT_fullw_sideinfo(Rating, ud, md, Ratingtest, signal_var, sigma_u, 1.0, w, m, 0.0,
                             epsU, 1.0, 0.0, 0.0, burnin, maxepoch, param_seed, ytrainMean,
                             ytrainStd, langevin, stiefel, avg, fixw=True, init="sigma")
    return out[1:]


def GPT_fixw_gibbs(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, w, burnin,
                   maxepoch, n_samples, param_seed, ytrainMean, ytrainStd, avg=False,
                   rotated_w=False):
    """100k_movielensExperiment.jl:945-1028: the user / movie conditionals of GPT_fullw_gibbs
    with w fixed (no w draw).  Returns (U_store, V_store, testpred_store, trainRMSE, testRMSE)."""
    out = GPT_fullw_gibbs(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, 1.0, w,
                          burnin, maxepoch, n_samples, param_seed, ytrainMean, ytrainStd, avg,
                          rotated_w, fixw=True)
    return out[1:]


def GPT_fullw_gibbs(Rating, UserData, MovieData, Ratingtest, signal_var, sigma_u, sigma_w, w_init,
                    burnin, maxepoch, n_samples, param_seed, ytrainMean, ytrainStd, avg=False,
                    rotated_w=False, fixw=False):
    r"""100k_movielensExperiment.jl:1032-1129 — Gibbs sampling of the tensor CF model without
    side information: per sweep every user row U_i | V, w, every movie row V_j | U, w (r × r
    Gaussian conditionals through chol(·,:U)), then w | U, V with the N × r² Kronecker design
    (kron(V[movie,:], U[user,:]) rows, r² × r² conditional).  Draws (framework contract):
    Q = qr(randn(r,r)) on (CFG_INIT, 0), U = σ_u·randn(n1, r) on (CFG_INIT, 1), V on (CFG_INIT, 2);
    sweep g (counted from 0 over the run) draws user i's z on (g, CFG_U, i), movie j's on
    (g, CFG_V, j) and w's on (g, CFG_W, 0).  ``\`` (a general LU solve in the reference) is taken
    through the Cholesky factor.  ytrainMean / ytrainStd are arguments (the reference reads the
    script's globals, :1100); the train prediction is a running average like the test one (the
    reference re-allocates it uninitialised every epoch, :1098, which only matters when avg).
    Returns (w_store (r,r,T), U_store (n1,r,T), V_store (n2,r,T), testpred_store, trainRMSE,
    testRMSE)."""
    Rating = np.asarray(Rating, dtype=np.float64)
    Ratingtest = np.asarray(Ratingtest, dtype=np.float64)
    N, Ntest = len(Rating), len(Ratingtest)
    n1, n2 = UserData.shape[0], MovieData.shape[0]
    w0 = np.array(w_init, dtype=np.float64, order="F")
    r = w0.shape[0]
    Qm, _ = np.linalg.qr(px.normals(r * r, param_seed, 0, px.CFG_INIT, 0).reshape((r, r), order="F"))
    U = sigma_u * px.normals(n1 * r, param_seed, 0, px.CFG_INIT, 1).reshape((n1, r), order="F")
    V = sigma_u * px.normals(n2 * r, param_seed, 0, px.CFG_INIT, 2).reshape((n2, r), order="F")
    if rotated_w:
        w = Qm @ w0
        U = U @ Qm.T
    else:
        w = w0.copy()
    users = Rating[:, 0].astype(np.int64) - 1
    movies = Rating[:, 1].astype(np.int64) - 1
    y = Rating[:, 2]
    w_store = np.zeros((r, r, maxepoch), order="F")
    U_store = np.zeros((n1, r, maxepoch), order="F")
    V_store = np.zeros((n2, r, maxepoch), order="F")
    testpred_store = np.zeros((Ntest, maxepoch), order="F")
    trainRMSE, testRMSE = np.zeros(maxepoch), np.zeros(maxepoch)
    trainpred, testpred = np.zeros(N), np.zeros(Ntest)
    counter = 0
    sweep = 0

    def draw(prec, rhs, z):
        L = np.linalg.cholesky(prec)
        mu = np.linalg.solve(L.T, np.linalg.solve(L, rhs)) / signal_var
        return np.linalg.solve(L.T, z) + mu

    for epoch in range(1, burnin + maxepoch + 1):
        for _ in range(n_samples):
            for i in range(n1):                                                 # :1060-1071
                sel = users == i
                if sel.any():
                    X = V[movies[sel]] @ w.T
                    prec = X.T @ X / signal_var + np.eye(r) / sigma_u ** 2
                    U[i] = draw(prec, X.T @ y[sel], px.normals(r, param_seed, sweep, px.CFG_U, i))
            for j in range(n2):                                                 # :1074-1085
                sel = movies == j
                if sel.any():
                    X = U[users[sel]] @ w
                    prec = X.T @ X / signal_var + np.eye(r) / sigma_u ** 2
                    V[j] = draw(prec, X.T @ y[sel], px.normals(r, param_seed, sweep, px.CFG_V, j))
            if not fixw:
                K = (V[movies][:, :, None] * U[users][:, None, :]).reshape((N, r * r))   # kron(V, U)
                prec = K.T @ K / signal_var + np.eye(r * r) / sigma_w ** 2              # :1092
                w = draw(prec, K.T @ y, px.normals(r * r, param_seed, sweep, px.CFG_W, 0)).reshape(
                    (r, r), order="F")
            sweep += 1
        if epoch > burnin:
            s = epoch - burnin - 1
            w_store[:, :, s] = w
            U_store[:, :, s] = U
            V_store[:, :, s] = V
            if not avg:
                counter = 0
            ptr = np.einsum("ik,kj,ij->i", U[users], w, V[movies])
            trainpred = (trainpred * counter + ptr) / (counter + 1)
            ft = cutoff(trainpred * ytrainStd + ytrainMean)
            trainRMSE[s] = math.sqrt(np.sum((ytrainStd * y + ytrainMean - ft) ** 2) / N)
            tu = Ratingtest[:, 0].astype(np.int64) - 1
            tm = Ratingtest[:, 1].astype(np.int64) - 1
            pte = np.einsum("ik,kj,ij->i", U[tu], w, V[tm])
            testpred = (testpred * counter + pte) / (counter + 1)
            fs = cutoff(testpred * ytrainStd + ytrainMean)
            testpred_store[:, s] = fs
            testRMSE[s] = math.sqrt(np.sum((ytrainStd * Ratingtest[:, 2] + ytrainMean - fs) ** 2) / Ntest)
            counter += 1
    return w_store, U_store, V_store, testpred_store, trainRMSE, testRMSE
