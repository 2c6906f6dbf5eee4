"""Python mirror of the reference's ``TGP`` Julia module (TGP.jl) — the tensor GP fitted by Gibbs
sampling — running on libgptsgld.so (HIP, gfx950).

    feature(x, n, sigmaRBF, generator)                       TGP.jl:6-14
    datawhitening(x)                                         TGP.jl:16-21
    GPT_inf(X, y, sigma, n, r, sigmaRBF, q, generator, num_iterations, burnin)   TGP.jl:37-86
    TensorRes(Xtrain, ytrain, sigma, n, r, sigmaRBF, q, generator, num_iterations, burnin, X, y)
                                                             TGP.jl:89-108

``feature`` reseeds its generator on every call (``srand(generator)``, TGP.jl:8), so every row
gets the same Z, b: here Z = randn(n, D)/sigmaRBF and b = rand(n, D) come from the Philox
feature streams of ``generator`` and all N rows are mapped in one device launch.  The Gibbs
sweeps (GPT_inf) run on the device (gpt_tgp_gibbs); the sampler's own draws (U init, I, the W
and U noise) use the TGP Philox streams of the same seed (oracle/philox.py).  A precision
matrix that fails Cholesky raises like Julia's PosDefException.
"""
import numpy as np

from ._lib import C, P_D, P_I32, check, lib
from .GPT_SGLD import _f64, _feature_D, _ptr, datawhitening, feature_inputs, pred_mean

__all__ = ["feature", "datawhitening", "GPT_inf", "TensorRes"]


def _features(X, n, sigmaRBF, generator):
    """b (n, D, N): row i is ``feature(X[i,:], n, sigmaRBF, generator)`` (TGP.jl:45-46)."""
    X = _f64(np.atleast_2d(X))
    Z, b = feature_inputs(int(n), X.shape[1], generator)
    return _feature_D(X, float(sigmaRBF), 1.0, 1.0, Z, b)


def feature(x, n, sigmaRBF, generator):
    """phi (n, D) = sqrt(2/n)·cos(x .* Z/sigmaRBF + 2π b) for one input row (TGP.jl:6-14)."""
    x = np.asarray(x, dtype=np.float64).reshape(1, -1)
    return np.asfortranarray(_features(x, n, sigmaRBF, generator)[:, :, 0])


def _gibbs(b, y, sigma, n, r, q, generator, num_iterations, burnin, I=None):
    n_, D, N = b.shape
    if n_ != n:
        raise ValueError("b rows must equal n")
    y = _f64(np.asarray(y, dtype=np.float64).ravel())
    if y.size != N:
        raise ValueError("y must have N entries")
    T = int(num_iterations) - int(burnin)
    W = np.empty((q, T), order="F")
    U = np.empty((n, r, D, T), order="F")
    Iout = np.empty((q, D), dtype=np.int32, order="F")
    Iin = None
    if I is not None:
        Iin = np.asfortranarray(np.asarray(I, dtype=np.int32))
        if Iin.shape != (q, D):
            raise ValueError("I must be (q, D)")
    check(lib().gpt_tgp_gibbs(_ptr(b), _ptr(y), n, D, N, r, q, float(sigma), int(num_iterations),
                              int(burnin), int(generator) & (2 ** 64 - 1),
                              _ptr(Iin, P_I32) if Iin is not None else None, _ptr(W), _ptr(U),
                              _ptr(Iout, P_I32)))
    return W, U, Iout


def GPT_inf(X, y, sigma, n, r, sigmaRBF, q, generator, num_iterations, burnin, I=None):
    """Gibbs sampler of the tensor GP (TGP.jl:37-86).  Whitens X and y, maps features and runs
    ``num_iterations`` sweeps; returns (W_array (q, T), V_array (n, r, D, T), I (q, D)) with
    T = num_iterations - burnin.  ``I`` (optional) fixes the core indices instead of drawing
    them (TGP.jl:50)."""
    X = datawhitening(np.asarray(X, dtype=np.float64))
    y = datawhitening(np.asarray(y, dtype=np.float64).ravel())
    b = _features(X, n, sigmaRBF, generator)
    return _gibbs(b, y, sigma, int(n), int(r), int(q), generator, num_iterations, burnin, I)


def TensorRes(Xtrain, ytrain, sigma, n, r, sigmaRBF, q, generator, num_iterations, burnin, X, y,
              I=None):
    """Test RMSE of the posterior-mean fit over the kept Gibbs sweeps (TGP.jl:89-108):
    ``std(y)·sqrt(mean((yfit - whiten(y))²))``."""
    W, U, I = GPT_inf(Xtrain, ytrain, sigma, n, r, sigmaRBF, q, generator, num_iterations, burnin,
                      I)
    y = np.asarray(y, dtype=np.float64).ravel()
    ystd = y.std(ddof=1)
    Xw = datawhitening(np.asarray(X, dtype=np.float64))
    yw = datawhitening(y)
    b = _features(Xw, n, sigmaRBF, generator)
    D = b.shape[1]
    U_store = np.asfortranarray(U.reshape((n, r, D * U.shape[3]), order="F"))
    return pred_mean(W, U_store, I, b, yw, scale=ystd)[1]
