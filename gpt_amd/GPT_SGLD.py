"""Python mirror of the reference's ``GPT_SGLD`` / ``GPT_SGLD_p`` Julia module API, running on
libgptsgld.so (HIP, gfx950).

Same function names, argument meaning, return values and error behaviour as the reference:

    feature(X, length_scale, sigma_RBF, phi_scale, Z, b)      GPT_SGLD.jl:71    (Gen D)
    feature(X, n, length_scale, sigma_RBF, seed, scale)       kin40kExperiment.jl:71 (Gen C)
    feature(X, n, length_scale, seed)                         GPT_SGLD_p.jl:40  (Gen A: b=randn)
    featureNotensor(X, length_scale, sigma_RBF, Z, b)         GPT_SGLD.jl:109   (Gen D)
    featureNotensor(X, n, length_scale, sigma_RBF, seed)      PowerPlantNoTensorExperiment.jl:32
    samplenz(r, D, Q, seed)                                   GPT_SGLD_p.jl:57
    GPTregression(phi, y, signal_var, I, r, Q, m, epsw, epsU, burnin, maxepoch[, param_seed];
                  langevin, stiefel)                          GPT_SGLD.jl:345
    GPT_SGLDERM(phi, y, sigma, I, r, Q, m, epsw, epsU, burnin, maxepoch)  GPT_SGLD_p.jl:146
    GPT_SGLDERMw(phi, y, signal_var, I, r, Q, m, epsw, burnin, maxepoch)  GPT_SGLD.jl:1065
    GPTclassification(phi, y, I, r, Q, m, epsw, epsU, burnin, maxepoch[, param_seed];
                      langevin, stiefel)                      GPT_SGLD.jl:452
    GPT_GMC(phi, y, signal_var, I, r, Q, epsw, epsU, burnin, maxepoch, L, param_seed)
                                                              GPT_SGLD.jl:684
    pred(w, U, I, phitest)                                    GPT_SGLD.jl:233
    RMSE(w_store, U_store, I, phitest, ytest)                 GPT_SGLD_p.jl:124
    pred_mean_x(w_store, U_store, I, Xtest, ytest, ls, σ, scale, Z, b)  fused feature + pred
    GPNT_SGLD(phi, y, signal_var, sigma_theta, m, eps_theta, decay_rate, burnin, maxepoch,
              param_seed)                                     GPT_SGLD.jl:809
    datawhitening(X), proj, geod are not on the device path (host prep / inside the kernel).

Arrays follow Julia's column-major layout: ``phi`` is (n, D, N) Fortran-ordered, ``U`` is
(n, r, D), ``I`` is (Q, D) Int32 1-based.  Like the reference, a NaN in the geodesic prints
"Get NaN when moving along Geodesic. Try smaller epsU" and returns all-zero stores
(GPT_SGLD.jl:23-26,422-424); bad dimensions raise (the reference's ``error(...)``).

RNG: Julia's MersenneTwister stream is replaced by the framework's Philox contract
(oracle/philox.py documents it); seeds play the same role (``srand(param_seed)``).
"""
import contextlib
import math
import os

import numpy as np

from . import _lib
from ._lib import C, P_D, P_I32, P_U64, SGLDConfig, check, lib


def _f64(a):
    return np.asfortranarray(np.asarray(a, dtype=np.float64))


def _ptr(a, t=P_D):
    return a.ctypes.data_as(t)


# ------------------------------------------------------------------ data preparation (host)
def datawhitening(X):
    """GPT_SGLD.jl:62-67 — per-column (x - mean)/std, n-1 denominator (host-side data prep)."""
    X = np.array(X, dtype=np.float64, copy=True)
    if X.ndim == 1:
        return (X - X.mean()) / X.std(ddof=1)
    return (X - X.mean(axis=0)) / X.std(axis=0, ddof=1)


# ------------------------------------------------------------------ features
def feature_inputs(n, D, seed):
    """Seeded ``Z = randn(n,D)``, ``b = 2π·rand(n,D)`` (Generation-C feature wrapper)."""
    Z = np.empty((n, D), order="F")
    b = np.empty((n, D), order="F")
    check(lib().gpt_feature_inputs(n, D, int(seed) & (2 ** 64 - 1), _ptr(Z), _ptr(b)))
    return Z, b


def feature_inputs_a(n, D, seed):
    """Seeded Generation-A inputs (GPT_SGLD_p.jl:40-54): ``Z = randn(n,D)``, ``b = randn(n,D)``."""
    Z = np.empty((n, D), order="F")
    b = np.empty((n, D), order="F")
    check(lib().gpt_feature_inputs_a(n, D, int(seed) & (2 ** 64 - 1), _ptr(Z), _ptr(b)))
    return Z, b


def epoch_orders(N, seed, epochs):
    """Row order of every epoch of a chain with ``param_seed`` = seed (randperm + phi[:,:,perm],
    GPT_SGLD.jl:373-374), built on the device: (N, epochs) int32, 0-based."""
    out = np.empty((int(N), int(epochs)), dtype=np.int32, order="F")
    check(lib().gpt_epoch_orders(int(N), int(seed) & (2 ** 64 - 1), int(epochs), _ptr(out, P_I32)))
    return out


def _feature_D(X, length_scale, sigma_RBF, phi_scale, Z, b):
    X = _f64(X)
    N, D = X.shape
    Z = _f64(Z)
    n = Z.shape[0]
    if Z.shape != (n, D):
        raise ValueError("Z must be (n, D)")
    b = _f64(np.asarray(b, dtype=np.float64).reshape((n, D), order="F"))
    ls = _f64(np.atleast_1d(length_scale))
    if ls.size not in (1, D):
        raise ValueError("dimensions of X and length_scale do not match")
    phi = np.empty((n, D, N), order="F")
    check(lib().gpt_feature(_ptr(X), N, D, _ptr(ls), ls.size, float(sigma_RBF), float(phi_scale),
                            _ptr(Z), _ptr(b), n, _ptr(phi)))
    return phi


def feature(X, *args):
    """Random Fourier features of the tensor model (all reference generations, see module doc)."""
    if len(args) == 5 and np.ndim(args[3]) == 2:          # Gen D: ls, σ, phi_scale, Z, b
        return _feature_D(X, *args)
    if len(args) == 5:                                    # Gen C: n, ls, σ, seed, scale
        n, ls, sigma, seed, scale = args
        Z, b = feature_inputs(int(n), np.shape(X)[1], seed)
        return _feature_D(X, ls, sigma, scale, Z, b)
    if len(args) == 4:                                    # Gen B: n, ls, seed, scale
        n, ls, seed, scale = args
        Z, b = feature_inputs(int(n), np.shape(X)[1], seed)
        return _feature_D(X, ls, 1.0, scale, Z, b)
    if len(args) == 3:                                    # Gen A: n, ls, seed
        # GPT_SGLD_p.jl:40-54: Z = randn(n,D)/length_scale, b = randn(n,D), phi = sqrt(2/n)·
        # cos(X[i,k]·Z[j,k] + b[j,k]) — no sigma_RBF / scale; Z/ℓ is formed first as there (the
        # kernel's argument X·Z'/1 is then the same double)
        n, ls, seed = args
        if np.size(ls) != 1:
            raise TypeError("feature(X,n,length_scale,seed): length_scale is a scalar (GPT_SGLD_p.jl:40)")
        Z, b = feature_inputs_a(int(n), np.shape(X)[1], seed)
        return _feature_D(X, 1.0, 1.0, 1.0, Z / float(np.ravel(ls)[0]), b)
    raise TypeError("feature: unsupported argument list")


def featureNotensor(X, *args):
    """Full-theta RFF features (GPT_SGLD.jl:109-120); Gen C form draws Z, b from ``seed``."""
    X = _f64(X)
    N, D = X.shape
    if len(args) != 4:
        raise TypeError("featureNotensor: unsupported argument list")
    if np.ndim(args[2]) != 2:                             # Gen C: n, ls, σ, seed
        return featureNotensor_seeded(X, *args)
    ls, sigma, Z, b = args                                # Gen D: ls, σ, Z, b
    Z = _f64(Z)
    b = _f64(np.asarray(b, dtype=np.float64).ravel())
    n = Z.shape[0]
    if Z.shape != (n, D) or b.size != n:
        raise ValueError("Z must be (n, D) and b of length n")
    ls = _f64(np.atleast_1d(ls))
    phi = np.empty((n, N), order="F")
    check(lib().gpt_feature_notensor(_ptr(X), N, D, _ptr(ls), ls.size, float(sigma), _ptr(Z),
                                     _ptr(b), n, _ptr(phi)))
    return phi


def featureNotensor_seeded(X, n, length_scale, sigma_RBF, seed):
    """Generation-C ``featureNotensor(X,n,ls,σ,seed)``: Z=randn(n,D), b=2π·rand(n)."""
    X = _f64(X)
    Z, b = feature_inputs(int(n), X.shape[1], seed)
    return featureNotensor(X, length_scale, sigma_RBF, Z, b[:, 0])


# ------------------------------------------------------------------ sparse core locations
def samplenz(r, D, Q, seed=0):
    """Q distinct lattice points of [r]^D (GPT_SGLD.jl:181-190), 1-based Int32 (Q, D)."""
    I = np.empty((Q, D), dtype=np.int32, order="F")
    check(lib().gpt_samplenz(r, D, Q, int(seed) & (2 ** 64 - 1), _ptr(I, P_I32)))
    return I


# ------------------------------------------------------------------ sampler
def make_config(n, D, N, r, Q, m, epsw, epsU, signal_var, sigma_w, burnin, maxepoch, seed,
                langevin=True, stiefel=True, store_every=1, max_steps=0):
    return SGLDConfig(n=n, D=D, N=N, r=r, Q=Q, m=m, epsw=float(epsw), epsU=float(epsU),
                      signal_var=float(signal_var), sigma_w=float(sigma_w), burnin=burnin,
                      maxepoch=maxepoch, seed=int(seed) & (2 ** 64 - 1), langevin=int(bool(langevin)),
                      stiefel=int(bool(stiefel)), store_every=store_every, max_steps=max_steps)


def init_state(n, r, D, Q, seed, stiefel=True, sigma_w=1.0):
    """Initial (w, U) GPTregression draws for ``param_seed`` (GPT_SGLD.jl:357-369)."""
    cfg = make_config(n, D, 1, r, Q, 1, 0, 0, 1.0, sigma_w, 0, 1, seed, stiefel=stiefel)
    w = np.empty(Q)
    U = np.empty((n, r, D), order="F")
    check(lib().gpt_sgld_init(C.byref(cfg), _ptr(w), _ptr(U)))
    return w, U


@contextlib.contextmanager
def _engine_env(engine):
    """GPTSGLD_ENGINE for the duration of one host-API call (the library reads it at session
    creation; include/gptsgld.h gpt_sgld_session_info)."""
    if engine is None:
        yield
        return
    if engine not in ("grid", "chain", "wave", "auto"):
        raise ValueError("engine must be 'grid', 'chain', 'wave' or 'auto'")
    old = os.environ.get("GPTSGLD_ENGINE")
    os.environ["GPTSGLD_ENGINE"] = engine
    try:
        yield
    finally:
        if old is None:
            del os.environ["GPTSGLD_ENGINE"]
        else:
            os.environ["GPTSGLD_ENGINE"] = old


def GPTregression(phi, y, signal_var, I, r, Q, m, epsw, epsU, burnin, maxepoch, param_seed=0,
                  langevin=True, stiefel=True, sigma_w=1.0, store_every=1, max_steps=0,
                  w_init=None, U_init=None, diag=False, engine=None):
    """Tensor-GP regression sampler (GPT_SGLD.jl:345-448).  Returns (w_store, U_store)
    [, diag]; ``diag`` = per-step [‖gradw‖, ‖gradU_1‖, …] ((1+D) × steps).
    ``engine`` ("grid" | "chain" | "wave" | None = library default) selects the step kernel."""
    phi = _f64(phi)
    n, D, N = phi.shape
    y = _f64(np.asarray(y, dtype=np.float64).ravel())
    if y.size != N:
        raise ValueError("phi and y disagree on N")
    I = np.asfortranarray(np.asarray(I, dtype=np.int32))
    if I.shape != (Q, D):
        raise ValueError("I must be (Q, D)")
    cfg = make_config(n, D, N, r, Q, m, epsw, epsU, signal_var, sigma_w, burnin, maxepoch,
                      param_seed, langevin, stiefel, store_every, max_steps)
    nb = -(-N // m)
    T = (maxepoch * nb) // store_every
    w_store = np.zeros((Q, T), order="F")
    U_store = np.zeros((n, r, D, T), order="F")
    total = (burnin + maxepoch) * nb if max_steps <= 0 else min((burnin + maxepoch) * nb, max_steps)
    dg = np.zeros((1 + D, total), order="F") if diag else None
    wi = _f64(w_init) if w_init is not None else None
    Ui = _f64(U_init) if U_init is not None else None
    with _engine_env(engine):
        code = lib().gpt_sgld_regression(C.byref(cfg), _ptr(phi), _ptr(y), _ptr(I, P_I32),
                                         _ptr(wi) if wi is not None else None,
                                         _ptr(Ui) if Ui is not None else None,
                                         _ptr(w_store), _ptr(U_store), _ptr(dg) if diag else None)
    if code == _lib.GPT_ERR_NAN_GEODESIC:
        print("Get NaN when moving along Geodesic. Try smaller epsU")
        w_store[:] = 0.0
        U_store[:] = 0.0
    else:
        check(code)
    return (w_store, U_store, dg) if diag else (w_store, U_store)


def GPTregression_chains(phis, y, signal_var, I, r, Q, m, epsw, epsU, burnin, maxepoch, seeds,
                         sigma_w=1.0, store_every=1, max_steps=0, engine=None):
    """Independent GPTregression chains in one call (gpt_sgld_regression_chains): the
    ``@parallel for j=1:10`` sweep block of kin40kExperiment.jl:67-74 (``phis`` a list with one
    phi per chain, each from its own length scales / sigma_RBF) or posterior chains on one phi
    (``phis`` a single array).  ``epsw``, ``epsU``, ``signal_var``: a scalar or one value per
    chain.  Returns a list of (w_store, U_store, status) per chain; status 1 = the geodesic NaN
    bail-out (that chain's stores are zeros, GPT_SGLD.jl:422-424)."""
    seeds = [int(s) & (2 ** 64 - 1) for s in seeds]
    nch = len(seeds)
    if not isinstance(phis, (list, tuple)):
        phis = [phis] * nch
    if len(phis) != nch:
        raise ValueError("one phi per chain, or one shared phi")
    uniq = {}
    for p in phis:                                  # one host copy per distinct array
        if id(p) not in uniq:
            uniq[id(p)] = _f64(p)
    ph = [uniq[id(p)] for p in phis]
    n, D, N = ph[0].shape
    if any(p.shape != (n, D, N) for p in ph):
        raise ValueError("every phi must have the same (n, D, N)")
    y = _f64(np.asarray(y, dtype=np.float64).ravel())
    if y.size != N:
        raise ValueError("phi and y disagree on N")
    I = np.asfortranarray(np.asarray(I, dtype=np.int32))
    if I.shape != (Q, D):
        raise ValueError("I must be (Q, D)")

    def per_chain(v):
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(v, dtype=np.float64), (nch,)))
        return a, _ptr(a)
    ew, ew_p = per_chain(epsw)
    eu, eu_p = per_chain(epsU)
    sv, sv_p = per_chain(signal_var)
    cfg = make_config(n, D, N, r, Q, m, ew[0], eu[0], sv[0], sigma_w, burnin, maxepoch, 0, True,
                      True, store_every, max_steps)
    T = (maxepoch * (-(-N // m))) // store_every
    ws = [np.zeros((Q, T), order="F") for _ in range(nch)]
    Us = [np.zeros((n, r, D, T), order="F") for _ in range(nch)]
    st = np.zeros(nch, dtype=np.int32)
    arr = lambda xs: (P_D * nch)(*[_ptr(x) for x in xs])
    sd = np.array(seeds, dtype=np.uint64)
    with _engine_env(engine):
        check(lib().gpt_sgld_regression_chains(C.byref(cfg), nch, sd.ctypes.data_as(P_U64),
                                               arr(ph), arr([y] * nch), _ptr(I, P_I32), ew_p,
                                               eu_p, sv_p, arr(ws), arr(Us), _ptr(st, P_I32)))
    return [(ws[c], Us[c], int(st[c])) for c in range(nch)]


def GPT_SGLDERM_RMSprop(phi, y, signal_var, I, r, Q, m, epsilon, alpha, burnin, maxepoch,
                        param_seed=0, w_init=None, U_init=None, diag=False):
    """SGLD with RMSprop step sizes (GPT_SGLD.jl:1121-1237).  Returns (w_store, U_store)
    [, diag]; on the geodesic NaN bail-out prints the reference's message and returns zeros."""
    phi = _f64(phi)
    n, D, N = phi.shape
    y = _f64(np.asarray(y, dtype=np.float64).ravel())
    if y.size != N:
        raise ValueError("phi and y disagree on N")
    I = np.asfortranarray(np.asarray(I, dtype=np.int32))
    if I.shape != (Q, D):
        raise ValueError("I must be (Q, D)")
    cfg = make_config(n, D, N, r, Q, m, epsilon, epsilon, signal_var, 1.0, burnin, maxepoch,
                      param_seed, True, True, 1, 0)
    nb = -(-N // m)
    T = maxepoch * nb
    w_store = np.zeros((Q, T), order="F")
    U_store = np.zeros((n, r, D, T), order="F")
    dg = np.zeros((1 + D, (burnin + maxepoch) * nb), order="F") if diag else None
    wi = _f64(w_init) if w_init is not None else None
    Ui = _f64(U_init) if U_init is not None else None
    code = lib().gpt_sgld_rmsprop(C.byref(cfg), float(epsilon), float(alpha), _ptr(phi), _ptr(y),
                                  _ptr(I, P_I32), _ptr(wi) if wi is not None else None,
                                  _ptr(Ui) if Ui is not None else None, _ptr(w_store),
                                  _ptr(U_store), _ptr(dg) if diag else None)
    if code == _lib.GPT_ERR_NAN_GEODESIC:
        print("Get NaN when moving along Geodesic. Try smaller epsU")
        w_store[:] = 0.0
        U_store[:] = 0.0
    else:
        check(code)
    return (w_store, U_store, dg) if diag else (w_store, U_store)


def GPT_SGLDERMw(phi, y, signal_var, I, r, Q, m, epsw, burnin, maxepoch, param_seed=0,
                 w_init=None, U_init=None, diag=False):
    """SGLD on w with U fixed at its uniform Stiefel draw (GPT_SGLD.jl:1065-1118).  Returns
    (w_store, U) [, gradw norms per step]."""
    phi = _f64(phi)
    n, D, N = phi.shape
    y = _f64(np.asarray(y, dtype=np.float64).ravel())
    if y.size != N:
        raise ValueError("phi and y disagree on N")
    I = np.asfortranarray(np.asarray(I, dtype=np.int32))
    if I.shape != (Q, D):
        raise ValueError("I must be (Q, D)")
    cfg = make_config(n, D, N, r, Q, m, epsw, 0.0, signal_var, 1.0, burnin, maxepoch,
                      param_seed, True, True, 1, 0)
    nb = -(-N // m)
    w_store = np.zeros((Q, maxepoch * nb), order="F")
    U = np.zeros((n, r, D), order="F")
    dg = np.zeros((1 + D, (burnin + maxepoch) * nb), order="F") if diag else None
    wi = _f64(w_init) if w_init is not None else None
    Ui = _f64(U_init) if U_init is not None else None
    check(lib().gpt_sgld_wonly(C.byref(cfg), _ptr(phi), _ptr(y), _ptr(I, P_I32),
                               _ptr(wi) if wi is not None else None,
                               _ptr(Ui) if Ui is not None else None, _ptr(w_store), _ptr(U),
                               _ptr(dg) if diag else None))
    return (w_store, U, dg[0].copy()) if diag else (w_store, U)


def GPTclassification(phi, y, I, r, Q, m, epsw, epsU, burnin, maxepoch, param_seed=0,
                      langevin=True, stiefel=True, w_init=None, U_init=None, diag=False):
    """Softmax tensor-GP classifier (GPT_SGLD.jl:452-680), labels y in 1..C.  Returns
    (w_store (Q, C, T), U_store (n, r, D, C, T)) [, diag (1+D, steps, C)]; on the geodesic NaN
    bail-out prints the reference's message and returns zeros."""
    phi = _f64(phi)
    n, D, N = phi.shape
    y = _f64(np.asarray(y, dtype=np.float64).ravel())
    if y.size != N:
        raise ValueError("phi and y disagree on N")
    ncls = int(y.max() - y.min() + 1)
    I = np.asfortranarray(np.asarray(I, dtype=np.int32))
    if I.shape != (Q, D):
        raise ValueError("I must be (Q, D)")
    cfg = make_config(n, D, N, r, Q, m, epsw, epsU, 1.0, 1.0, burnin, maxepoch, param_seed,
                      langevin, stiefel, 1, 0)
    nb = -(-N // m)
    T = maxepoch * nb
    w_store = np.zeros((Q, ncls, T), order="F")
    U_store = np.zeros((n, r, D, ncls, T), order="F")
    dg = np.zeros((1 + D, (burnin + maxepoch) * nb, ncls), order="F") if diag else None
    wi = _f64(w_init) if w_init is not None else None
    Ui = _f64(U_init) if U_init is not None else None
    code = lib().gpt_sgld_classification(C.byref(cfg), _ptr(phi), _ptr(y), _ptr(I, P_I32),
                                         _ptr(wi) if wi is not None else None,
                                         _ptr(Ui) if Ui is not None else None, _ptr(w_store),
                                         _ptr(U_store), _ptr(dg) if diag else None)
    if code == _lib.GPT_ERR_NAN_GEODESIC:
        print("Get NaN when moving along Geodesic. Try smaller epsU")
    else:
        check(code)
    return (w_store, U_store, dg) if diag else (w_store, U_store)


def GPT_GMC(phi, y, signal_var, I, r, Q, epsw, epsU, burnin, maxepoch, L, param_seed=0,
            w_init=None, U_init=None):
    """Geodesic Monte Carlo (GPT_SGLD.jl:684-805).  Returns (w_store (Q, maxepoch),
    U_store (n, r, D, maxepoch), accept_prob (burnin+maxepoch)); on the geodesic NaN bail-out
    prints the reference's message and returns zeros and NaN probabilities."""
    phi = _f64(phi)
    n, D, N = phi.shape
    y = _f64(np.asarray(y, dtype=np.float64).ravel())
    if y.size != N:
        raise ValueError("phi and y disagree on N")
    I = np.asfortranarray(np.asarray(I, dtype=np.int32))
    if I.shape != (Q, D):
        raise ValueError("I must be (Q, D)")
    w_store = np.zeros((Q, maxepoch), order="F")
    U_store = np.zeros((n, r, D, maxepoch), order="F")
    acc = np.zeros(burnin + maxepoch)
    wi = _f64(w_init) if w_init is not None else None
    Ui = _f64(U_init) if U_init is not None else None
    code = lib().gpt_gmc(_ptr(phi), _ptr(y), n, D, N, r, Q, _ptr(I, P_I32), float(signal_var),
                         float(epsw), float(epsU), int(burnin), int(maxepoch), int(L),
                         int(param_seed) & (2 ** 64 - 1), _ptr(wi) if wi is not None else None,
                         _ptr(Ui) if Ui is not None else None, _ptr(w_store), _ptr(U_store),
                         _ptr(acc))
    if code == _lib.GPT_ERR_NAN_GEODESIC:
        print("Get NaN when moving along Geodesic. Try smaller epsU")
    else:
        check(code)
    return w_store, U_store, acc


def GPT_SGLDERM(phi, y, sigma, I, r, Q, m, epsw, epsU, burnin, maxepoch, param_seed=0, **kw):
    """Generation A/B sampler (GPT_SGLD_p.jl:146-243): ``sigma`` is the noise s.d. and the
    prior s.d. of w is sqrt(n^D/Q) (:155)."""
    n, D, _ = np.shape(phi)
    return GPTregression(phi, y, float(sigma) ** 2, I, r, Q, m, epsw, epsU, burnin, maxepoch,
                         param_seed, sigma_w=math.sqrt(float(n) ** D / Q), **kw)


# ------------------------------------------------------------------ prediction
def pred(w, U, I, phitest):
    """fhat = pred(w, U, I, phitest) (GPT_SGLD.jl:233-243)."""
    phitest = _f64(phitest)
    n, D, Nt = phitest.shape
    U = _f64(U)
    r = U.shape[1]
    w = _f64(np.asarray(w, dtype=np.float64).ravel())
    I = np.asfortranarray(np.asarray(I, dtype=np.int32))
    out = np.empty(Nt)
    check(lib().gpt_pred(_ptr(w), _ptr(U), _ptr(I, P_I32), _ptr(phitest), n, D, Nt, r, w.size,
                         _ptr(out)))
    return out


def pred_mean(w_store, U_store, I, phitest, ytest, scale=1.0):
    """Posterior-mean prediction over the stored samples and its RMSE·scale
    (GPT_SGLD_p.jl:124-132; kin40kExperiment.jl:80-87).  Returns (meanfhat, rmse)."""
    phitest = _f64(phitest)
    n, D, Nt = phitest.shape
    w_store = _f64(w_store)
    U_store = _f64(U_store)
    Q, S = w_store.shape
    r = U_store.shape[1]
    I = np.asfortranarray(np.asarray(I, dtype=np.int32))
    yt = _f64(np.asarray(ytest, dtype=np.float64).ravel())
    mean = np.empty(Nt)
    rm = C.c_double(0.0)
    check(lib().gpt_pred_mean(_ptr(w_store), _ptr(U_store), _ptr(I, P_I32), _ptr(phitest), _ptr(yt),
                              n, D, Nt, r, Q, S, float(scale), _ptr(mean), C.byref(rm)))
    return mean, rm.value


def pred_mean_x(w_store, U_store, I, Xtest, ytest, length_scale, sigma_RBF, phi_scale, Z, b,
                scale=1.0):
    """pred_mean with the test features formed inside the prediction kernel from Xtest (no
    n·D·Ntest phitest array; same doubles as ``feature(Xtest, length_scale, sigma_RBF,
    phi_scale, Z, b)``).  Returns (meanfhat, rmse, per-sample rmse) — the last is the
    ``testRMSE`` curve of kin40kExperiment.jl:78-83 when the samples are the epoch ends."""
    X = _f64(Xtest)
    Nt, D = X.shape
    Z = _f64(Z)
    n = Z.shape[0]
    b = _f64(np.asarray(b, dtype=np.float64).reshape((n, D), order="F"))
    ls = _f64(np.atleast_1d(length_scale))
    w_store = _f64(w_store)
    U_store = _f64(U_store)
    Q, S = w_store.shape
    r = U_store.shape[1]
    I = np.asfortranarray(np.asarray(I, dtype=np.int32))
    yt = _f64(np.asarray(ytest, dtype=np.float64).ravel())
    mean = np.empty(Nt)
    srm = np.empty(S)
    rm = C.c_double(0.0)
    check(lib().gpt_pred_mean_x(_ptr(w_store), _ptr(U_store), _ptr(I, P_I32), _ptr(X), _ptr(yt), Nt,
                                D, _ptr(ls), ls.size, float(sigma_RBF), float(phi_scale), _ptr(Z),
                                _ptr(b), n, r, Q, S, float(scale), _ptr(mean), C.byref(rm),
                                _ptr(srm)))
    return mean, rm.value, srm


def RMSE(w_store, U_store, I, phitest, ytest):
    """GPT_SGLD_p.jl:124-132: RMSE of the mean prediction over ALL stored samples."""
    return pred_mean(w_store, U_store, I, phitest, ytest)[1]


# ------------------------------------------------------------------ full-theta model
def GPNT_SGLD(phi, y, signal_var, sigma_theta, m, eps_theta, decay_rate, burnin, maxepoch,
              param_seed=0):
    """Full-theta RFF SGLD (GPT_SGLD.jl:809-847).  Returns theta_store (n, T); on NaN prints
    the reference's message and returns zeros(n) (:840-843)."""
    phi = _f64(phi)
    n, N = phi.shape
    y = _f64(np.asarray(y, dtype=np.float64).ravel())
    nb = -(-N // m)
    out = np.empty((n, (maxepoch + burnin) * nb), order="F")
    code = lib().gpt_gpnt_sgld(_ptr(phi), _ptr(y), n, N, float(signal_var), float(sigma_theta), m,
                               float(eps_theta), float(decay_rate), burnin, maxepoch,
                               int(param_seed) & (2 ** 64 - 1), _ptr(out))
    if code == _lib.GPT_ERR_NAN_THETA:
        print("Get NaN in theta. Try smaller epsilon")
        return np.zeros(n)
    check(code)
    return out
