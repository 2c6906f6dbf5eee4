"""ctypes binding of oracle/_build/libgptcpu.so — the C++ fp64 restatement of GPT_SGLD.jl:345-448.

TEST INFRASTRUCTURE and CPU BASELINE.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import anything under ``oracle/``; the product path
(``gpt_amd``) never does.  Built by ``make -C oracle`` (``__graft_entry__.build()``).
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libgptcpu.so")
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("%s missing: run `make -C oracle`" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        P_D = C.POINTER(C.c_double)
        L.gptcpu_regression.restype = C.c_longlong
        L.gptcpu_regression.argtypes = [C.POINTER(C.c_int64), P_D, P_D, P_D, C.POINTER(C.c_int32),
                                        C.c_int, C.POINTER(C.c_uint64), C.c_int, P_D, P_D, P_D, P_D,
                                        C.POINTER(C.c_int32), P_D, C.POINTER(C.c_int64)]
        L.gptcpu_cf_sgd.restype = C.c_double
        PP_I = C.POINTER(C.POINTER(C.c_int32))
        PP_D = C.POINTER(C.POINTER(C.c_double))
        L.gptcpu_cf_sgd.argtypes = [C.c_int, C.POINTER(C.c_int64), P_D] + [C.POINTER(C.c_int32)] * 4 + \
            [PP_I, PP_I, PP_D, PP_I, PP_I, PP_I, PP_D, PP_D, PP_D, PP_D, PP_D, C.c_int]
        L.gptcpu_max_threads.restype = C.c_int
        L.gptcpu_pred.restype = None
        L.gptcpu_pred.argtypes = [C.c_int64] * 6 + [P_D, P_D, P_D, C.POINTER(C.c_int32), C.c_int,
                                                    P_D, P_D]
        _LIB = L
    return _LIB


def _p(a, t=C.c_double):
    return a.ctypes.data_as(C.POINTER(t)) if a is not None else None


def GPTregression_chains(phi, y, signal_var, I, r, Q, m, epsw, epsU, burnin, maxepoch, seeds,
                         threads=1, sigma_w=1.0, store_every=1, max_steps=0, stores=False):
    """Independent GPTregression chains (one per seed) on ``threads`` OpenMP threads.
    Returns dict(w (Q, C), U (n, r, D, C), status (C,), chain_steps (C,): the steps each chain
    took, a bail-out step included, steps, seconds[, w_store, U_store of chain 0])."""
    phi = np.asfortranarray(phi, dtype=np.float64)
    n, D, N = phi.shape
    y = np.ascontiguousarray(np.ravel(y), dtype=np.float64)
    I = np.asfortranarray(I, dtype=np.int32)
    seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
    nch = len(seeds)
    icfg = np.array([n, D, N, r, Q, m, burnin, maxepoch, store_every, max_steps], dtype=np.int64)
    dcfg = np.array([epsw, epsU, signal_var, sigma_w], dtype=np.float64)
    w = np.zeros((Q, nch), order="F")
    U = np.zeros((n, r, D, nch), order="F")
    nb = -(-N // m)
    T = (maxepoch * nb) // store_every
    ws = np.zeros((Q, T), order="F") if stores else None
    Us = np.zeros((n, r, D, T), order="F") if stores else None
    st = np.zeros(nch, dtype=np.int32)
    cs = np.zeros(nch, dtype=np.int64)
    sec = C.c_double(0.0)
    steps = lib().gptcpu_regression(_p(icfg, C.c_int64), _p(dcfg), _p(phi), _p(y), _p(I, C.c_int32),
                                    nch, _p(seeds, C.c_uint64), int(threads), _p(w), _p(U), _p(ws),
                                    _p(Us), _p(st, C.c_int32), C.byref(sec),
                                    _p(cs, C.c_int64))
    if steps < 0:
        raise ValueError("gptcpu_regression: unsupported configuration")
    out = dict(w=w, U=U, status=st, chain_steps=cs, steps=int(steps), seconds=sec.value)
    if stores:
        out.update(w_store=ws, U_store=Us)
    return out


def pred(w, U, I, phitest, threads=1):
    """pred (GPT_SGLD.jl:233-243) of S samples: w (Q, S), U (n, r, D, S), phitest (n, D, Ntest)
    in the reference layouts.  Returns (fhat (S, Ntest), seconds)."""
    phitest = np.asfortranarray(phitest, dtype=np.float64)
    n, D, Nt = phitest.shape
    w = np.asfortranarray(np.asarray(w, dtype=np.float64).reshape(w.shape[0], -1))
    Q, S = w.shape
    U = np.asfortranarray(np.asarray(U, dtype=np.float64).reshape(n, -1, D, S))
    r = U.shape[1]
    I = np.asfortranarray(I, dtype=np.int32)
    f = np.zeros((S, Nt))
    sec = C.c_double(0.0)
    lib().gptcpu_pred(n, D, Nt, r, Q, S, _p(phitest), _p(w), _p(U), _p(I, C.c_int32), int(threads),
                      _p(f), C.byref(sec))
    return f, sec.value


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _csr(data, base):
    """CSR of the feature rows of each user / movie (absolute U / V rows base + f)."""
    ptr, fe = [0], []
    for row in np.asarray(data):
        fe.extend(int(base + f) for f in np.flatnonzero(row))
        ptr.append(len(fe))
    return np.array(ptr, dtype=np.int32), np.array(fe if fe else [0], dtype=np.int32)


def cf_sgd_folds(folds, UserData, MovieData, perms, w0, U0, V0, signal_var, sigma_u, sigma_w, m,
                 epsw, epsU, a, b, c, threads=1, lazy=False):
    """GPT_fullw_sideinfo SGD epochs (langevin = stiefel = false) of every fold on ``threads``
    OpenMP threads, from the given state: folds = [(Rating, Ratingtest)] (1-based ids,
    standardised ratings), perms[f] = (epochs, N) 0-based orders, w0 (r, r), U0 / V0 (rows, r)
    row-major starting states shared by the folds.  ``lazy``: the GPU's lazy prior-decay move
    (rows outside a batch read as M·c^Δ) instead of the reference's dense per-step move of every
    row.  Returns (seconds, [(w, U, V, sse (epochs, 2))])."""
    L = lib()
    nf = len(folds)
    n1, D1 = np.asarray(UserData).shape
    n2, D2 = np.asarray(MovieData).shape
    r = np.asarray(w0).shape[0]
    uptr, ufe = _csr(UserData, n1)
    vptr, vfe = _csr(MovieData, n2)
    keep, outs = [], []
    arr = {k: [] for k in ("u", "m", "y", "p", "tu", "tm", "ty", "w", "U", "V", "s")}
    N = len(folds[0][0])
    Nt = min(len(f[1]) for f in folds)
    epochs = np.asarray(perms[0]).shape[0]
    for f, (Rt, Rs) in enumerate(folds):
        Rt = np.asarray(Rt, dtype=np.float64)
        Rs = np.asarray(Rs, dtype=np.float64)[:Nt]
        d = dict(u=np.ascontiguousarray(Rt[:, 0] - 1, dtype=np.int32),
                 m=np.ascontiguousarray(Rt[:, 1] - 1, dtype=np.int32),
                 y=np.ascontiguousarray(Rt[:, 2]),
                 p=np.ascontiguousarray(perms[f], dtype=np.int32),
                 tu=np.ascontiguousarray(Rs[:, 0] - 1, dtype=np.int32),
                 tm=np.ascontiguousarray(Rs[:, 1] - 1, dtype=np.int32),
                 ty=np.ascontiguousarray(Rs[:, 2]),
                 w=np.array(w0, dtype=np.float64, order="F"),
                 U=np.array(U0, dtype=np.float64, order="C"),
                 V=np.array(V0, dtype=np.float64, order="C"),
                 s=np.zeros((epochs, 2)))
        keep.append(d)
        for k in arr:
            t = C.c_int32 if d[k].dtype == np.int32 else C.c_double
            arr[k].append(_p(d[k], t))
    def pp(k, t):
        return (C.POINTER(t) * nf)(*arr[k])
    icfg = np.array([N, Nt, n1, D1, n2, D2, r, m, epochs, int(bool(lazy))], dtype=np.int64)
    dcfg = np.array([signal_var, sigma_u, sigma_w, epsw, epsU, a, b, c], dtype=np.float64)
    sec = L.gptcpu_cf_sgd(nf, _p(icfg, C.c_int64), _p(dcfg), _p(uptr, C.c_int32), _p(ufe, C.c_int32),
                          _p(vptr, C.c_int32), _p(vfe, C.c_int32), pp("u", C.c_int32),
                          pp("m", C.c_int32), pp("y", C.c_double), pp("p", C.c_int32),
                          pp("tu", C.c_int32), pp("tm", C.c_int32), pp("ty", C.c_double),
                          pp("w", C.c_double), pp("U", C.c_double), pp("V", C.c_double),
                          pp("s", C.c_double), int(threads))
    for d in keep:
        outs.append((d["w"], d["U"], d["V"], d["s"]))
    return sec, outs
