"""CPU oracle: a numpy fp64 restatement of the reference tensor-GP SGLD path.

TEST INFRASTRUCTURE — NOT PRODUCT CODE.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import this module.  The product path
(``gpt_amd`` + ``libgptsgld.so``) never imports, links or executes anything under
``oracle/``.

Every function restates the Julia reference line for line (citations are
``/root/reference/<file>:<line>``).  Arrays use Julia's column-major semantics: a Julia
``phi[j,k,i]`` is ``phi[j, k, i]`` here with ``order='F'`` storage, ``I`` is 1-based
Int32 exactly as ``samplenz`` returns it.

Randomness: the reference draws from Julia's global MersenneTwister, which cannot be
reproduced without Julia.  All draws here come from the Philox streams of
``oracle/philox.py`` (the same contract the HIP kernels implement), consumed at the same
points in the same order as the reference.  Pinning: ``pred``/``phidotU``/
``computeV``/``computefhat`` and the column-major layouts are pinned by the reference's
own fixtures ``TensorSynthData{5D,10D}100N.h5`` (tests/golden); the gradients by the
finite-difference method of ``Diagnostic_gradients.jl:131-158``; ``expm`` by the Padé
algorithm of Julia Base 0.3 ``expm!`` (cross-checked against scipy); RNG-dependent
trajectories are parity-unpinned against Julia and pinned against this oracle.
"""
import math
import numpy as np

from . import philox as px


# --------------------------------------------------------------------------- data prep
def datawhitening(X):
    """GPT_SGLD.jl:62-67 — centre each column and divide by its (n-1) std."""
    X = np.array(X, dtype=np.float64, copy=True)
    if X.ndim == 1:
        return (X - X.mean()) / X.std(ddof=1)
    for i in range(X.shape[1]):
        X[:, i] = (X[:, i] - X[:, i].mean()) / X[:, i].std(ddof=1)
    return X


# --------------------------------------------------------------------------- features
def feature(X, length_scale, sigma_RBF, phi_scale, Z, b):
    """GPT_SGLD.jl:71-84.  phi[j,k,i] = c·cos(X[i,k]·Zt[j,k] + b[j,k]),
    Zt = scale(Z, 1./length_scale), c = phi_scale·σ^(1/D)·sqrt(2/n)."""
    X = np.asarray(X, dtype=np.float64)
    N, D = X.shape
    Z = np.asarray(Z, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64).reshape(Z.shape, order="F")
    n = Z.shape[0]
    ls = np.broadcast_to(np.asarray(length_scale, dtype=np.float64), (D,))
    Zt = Z * (1.0 / ls)[None, :]
    arg = X.T[None, :, :] * Zt[:, :, None] + b[:, :, None]          # (n, D, N)
    c = phi_scale * sigma_RBF ** (1.0 / D) * math.sqrt(2.0 / n)
    return np.asfortranarray(c * np.cos(arg))


def featureNotensor(X, length_scale, sigma_RBF, Z, b):
    """GPT_SGLD.jl:109-120.  phi[j,i] = sqrt(2/n)·σ·cos(Σ_k X[i,k]·Zt[j,k] + b[j])."""
    X = np.asarray(X, dtype=np.float64)
    N, D = X.shape
    Z = np.asarray(Z, dtype=np.float64)
    n = Z.shape[0]
    ls = np.broadcast_to(np.asarray(length_scale, dtype=np.float64), (D,))
    Zt = Z * (1.0 / ls)[None, :]
    s = np.zeros((n, N))
    for k in range(D):                       # sum(X[i,:].*Zt[j,:]) left to right
        s = s + Zt[:, k:k + 1] * X[None, :, k]
    return np.asfortranarray(math.sqrt(2.0 / n) * sigma_RBF * np.cos(s + np.asarray(b, float).reshape(n, 1)))


def seeded_feature_inputs(n, D, seed):
    """Generation-C seeded ``feature(X,n,ls,σ,seed,scale)``: Z=randn(n,D),
    b=2π·rand(n,D) drawn from the framework's streams (W_INIT/U_INIT reused with c3 tags)."""
    Z = px.normals(n * D, seed, 0, 9, 0).reshape((n, D), order="F")
    x0, x1, _, _ = px.philox4x32(np.arange(n * D, dtype=np.uint32), 0, 10, 0, seed)
    b = 2.0 * np.pi * px._u53(x0, x1).reshape((n, D), order="F")
    return Z, b


def seeded_feature_inputs_a(n, D, seed):
    """Generation-A seeded inputs (GPT_SGLD_p.jl:43-45): Z=randn(n,D) (the Gen-C Z stream),
    b=randn(n,D) on the FEAT_B stream with c3 = 1."""
    Z = px.normals(n * D, seed, 0, 9, 0).reshape((n, D), order="F")
    b = px.normals(n * D, seed, 0, 10, 1).reshape((n, D), order="F")
    return Z, b


def feature_gen_a(X, n, length_scale, seed):
    """GPT_SGLD_p.jl:40-54, line by line: Z = randn(n,D)/length_scale, b = randn(n,D),
    phi[j,k,i] = cos(X[i,k]*Z[j,k] + b[j,k]), return sqrt(2/n)*phi (no sigma_RBF, no scale)."""
    X = np.asarray(X, dtype=np.float64)
    N, D = X.shape
    Z, b = seeded_feature_inputs_a(n, D, seed)
    Z = Z / float(length_scale)
    phi = np.cos(X.T[None, :, :] * Z[:, :, None] + b[:, :, None])
    return np.asfortranarray(math.sqrt(2.0 / n) * phi)


# --------------------------------------------------------------------------- samplenz
def samplenz_from_L(L, r, D):
    """GPT_SGLD.jl:181-190 body given the drawn lattice indices L:
    I[q,:] = digits(L[q], r, D) + 1 (little-endian base-r digits)."""
    L = np.asarray(L, dtype=np.int64)
    I = np.empty((len(L), D), dtype=np.int32, order="F")
    for q, v in enumerate(L):
        v = int(v)
        for k in range(D):
            I[q, k] = v % r + 1
            v //= r
    return I


def sample_lattice(r, D, Q, seed):
    """``sample(0:(r^D-1), Q, replace=false)`` restated as a sparse partial Fisher–Yates on
    the SAMPLENZ stream (c2=8): position i swaps with i + floor(u64·(M-i)/2^64)."""
    M = int(r) ** int(D)
    if Q > M:
        raise ValueError("Q must be <= r^D")
    x0, x1, _, _ = px.philox4x32(np.arange(Q, dtype=np.uint32), 0, 8, 0, seed)
    swapped = {}
    L = []
    for i in range(Q):
        u = (int(x0[i]) << 32) | int(x1[i])
        j = i + ((u * (M - i)) >> 64)
        vi = swapped.get(i, i)
        vj = swapped.get(j, j)
        swapped[i], swapped[j] = vj, vi
        L.append(vj)
    return np.array(L, dtype=np.int64)


def samplenz(r, D, Q, seed):
    """Gen-A/C ``samplenz(r,D,Q,seed)`` (GPT_SGLD_p.jl:57-67) on the framework stream."""
    return samplenz_from_L(sample_lattice(r, D, Q, seed), r, D)


# --------------------------------------------------------------------------- forward
def phidotU(U, phi):
    """GPT_SGLD.jl:193-205.  temp[k,l,i] = dot(phi[:,k,i], U[:,l,k])."""
    return np.einsum("jki,jlk->kli", phi, U)


def computeV(temp, I):
    """GPT_SGLD.jl:208-220.  V[q,i] = prod_k temp[k, I[q,k], i] (product in k order)."""
    Q, D = I.shape
    V = np.ones((Q, temp.shape[2]))
    for k in range(D):
        V = V * temp[k, I[:, k] - 1, :]
    return V


def computefhat(V, w):
    """GPT_SGLD.jl:223-230.  fhat[i] = dot(V[:,i], w)."""
    return V.T @ w


def pred(w, U, I, phitest):
    """GPT_SGLD.jl:233-243."""
    return computefhat(computeV(phidotU(U, phitest), I), w)


def computeU_phi(V, temp, I):
    """GPT_SGLD.jl:246-258.  U_phi[q,i,k] = V[q,i] / temp[k, I[q,k], i]."""
    Q, D = I.shape
    out = np.empty((Q, V.shape[1], D))
    for k in range(D):
        out[:, :, k] = V / temp[k, I[:, k] - 1, :]
    return out


def computeA(U_phi, w, I, r):
    """GPT_SGLD.jl:261-273.  A[l,k,i] = sum_{q: I[q,k]=l} U_phi[q,i,k]·w[q]."""
    Q, B, D = U_phi.shape
    A = np.zeros((r, D, B))
    for k in range(D):
        for l in np.unique(I[:, k]):
            idx = np.nonzero(I[:, k] == l)[0]
            A[l - 1, k, :] = w[idx] @ U_phi[idx, :, k]
    return A


def computePsi(A, phi):
    """GPT_SGLD.jl:276-286.  Psi[:,i,k] = kron(A[:,k,i], phi[:,k,i])."""
    r, D, B = A.shape
    n = phi.shape[0]
    Psi = np.empty((n * r, B, D))
    for k in range(D):
        # kron(a, p)[(l)*n + j] = a[l]*p[j]
        Psi[:, :, k] = (A[:, k, None, :] * phi[None, :, k, :]).reshape(n * r, B)
    return Psi


def gradients(phi_batch, y_batch, w, U, I, N, signal_var, sigma_w=1.0):
    """GPT_SGLD.jl:384-408: temp, V, fhat, gradw, U_phi, A, Psi, gradU for one minibatch."""
    n, D, B = phi_batch.shape
    r = U.shape[1]
    temp = phidotU(U, phi_batch)
    V = computeV(temp, I)
    fhat = computefhat(V, w)
    res = y_batch - fhat
    gradw = (N / B) * (V @ res) / signal_var - w / sigma_w ** 2
    U_phi = computeU_phi(V, temp, I)
    A = computeA(U_phi, w, I, r)
    Psi = computePsi(A, phi_batch)
    gradU = np.empty((n, r, D))
    for k in range(D):
        # reshape((N/B)*Psi_k*(y-fhat)/σ², n, r) — Julia column-major reshape
        gradU[:, :, k] = ((N / B) * (Psi[:, :, k] @ res) / signal_var).reshape((n, r), order="F")
    return dict(temp=temp, V=V, fhat=fhat, gradw=gradw, A=A, gradU=gradU)


def loglik(phi, y, w, U, I, sigma):
    """Diagnostic_gradients.jl:5-37 — log p(y|x,w,U) (for finite-difference checks)."""
    fhat = pred(w, U, I, phi)
    return -np.linalg.norm(y - fhat) ** 2 / (2 * sigma ** 2)


# --------------------------------------------------------------------------- Stiefel
def proj(U, V):
    """GPT_SGLD.jl:14-16."""
    return V - U @ (U.T @ V + V.T @ U) / 2


_PADE = {
    3: [120.0, 60.0, 12.0, 1.0],
    5: [30240.0, 15120.0, 3360.0, 420.0, 30.0, 1.0],
    7: [17297280.0, 8648640.0, 1995840.0, 277200.0, 25200.0, 1512.0, 56.0, 1.0],
    9: [17643225600.0, 8821612800.0, 2075673600.0, 302702400.0, 30270240.0,
        2162160.0, 110880.0, 3960.0, 90.0, 1.0],
    13: [64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
         1187353796428800.0, 129060195264000.0, 10559470521600.0, 670442572800.0,
         33522128640.0, 1323241920.0, 40840800.0, 960960.0, 16380.0, 182.0, 1.0],
}


def expm(A):
    """Matrix exponential by Padé scaling-and-squaring, restating Julia Base 0.3
    ``expm!`` (Higham 2005; thresholds 0.015/0.25/0.95/2.1 and 5.4 as in Julia Base,
    without the LAPACK ``gebal`` balancing step, which does not change the result)."""
    A = np.array(A, dtype=np.float64)
    n = A.shape[0]
    Id = np.eye(n)
    nA = np.abs(A).sum(axis=0).max() if n else 0.0
    if not np.isfinite(nA):
        # Julia's ceil(Int, log2(nA/5.4)) would throw here; the framework takes geod's
        # NaN bail-out instead (documented in DESIGN.md).
        return np.full((n, n), np.nan)
    if nA <= 2.1:
        if nA > 0.95:
            C = _PADE[9]
        elif nA > 0.25:
            C = _PADE[7]
        elif nA > 0.015:
            C = _PADE[5]
        else:
            C = _PADE[3]
        A2 = A @ A
        P = Id.copy()
        U = C[1] * P
        V = C[0] * P
        for k in range(1, (len(C) - 1) // 2 + 1):
            k2 = 2 * k
            P = P @ A2
            U = U + C[k2 + 1] * P
            V = V + C[k2] * P
        U = A @ U
        X = np.linalg.solve(V - U, V + U)
    else:
        s = math.log2(nA / 5.4)
        si = int(math.ceil(s)) if s > 0 else 0
        if s > 0:
            A = A / (2.0 ** si)
        C = _PADE[13]
        A2 = A @ A
        A4 = A2 @ A2
        A6 = A2 @ A4
        U = A @ (A6 @ (C[13] * A6 + C[11] * A4 + C[9] * A2)
                 + C[7] * A6 + C[5] * A4 + C[3] * A2 + C[1] * Id)
        V = A6 @ (C[12] * A6 + C[10] * A4 + C[8] * A2) + C[6] * A6 + C[4] * A4 + C[2] * A2 + C[0] * Id
        X = np.linalg.solve(V - U, V + U)
        for _ in range(si):
            X = X @ X
    return X


def geod(U, mom, t):
    """GPT_SGLD.jl:19-37.  Returns (U_new, ok); ok=False reproduces the NaN bail-out
    (``println`` + ``zeros(n,r)``)."""
    n, r = U.shape
    A = U.T @ mom
    T = np.block([[A, -(mom.T @ mom)], [np.eye(r), A]])
    with np.errstate(all="ignore"):
        E = expm(t * T)
    if np.isnan(E).any():
        return np.zeros((n, r)), False
    mexp = expm(-t * A)
    tmpU = (np.hstack([U, mom]) @ E[:, :r]) @ mexp
    return tmpU / np.linalg.norm(tmpU, axis=0)[None, :], True


def stiefel_init(Zr_n):
    """GPT_SGLD.jl:365-366: U_k = transpose(sqrtm(Z*Z') \\ Z) = Z'(ZZ')^(-1/2)."""
    Z = Zr_n
    evals, evecs = np.linalg.eigh(Z @ Z.T)
    inv_sqrt = (evecs / np.sqrt(evals)[None, :]) @ evecs.T
    return Z.T @ inv_sqrt


def u_noise(n, r, seed, step, k):
    """U-noise contract of stream (step, U_NOISE, k): the quad layout of ``philox.unoise_quads``
    (one Philox block per four normals: column l of rows λ + 64·(4q + i)).  Stands in for
    Julia's ``randn(n, r)`` at GPT_SGLD.jl:420 / ``randn(n, r, D)`` at :426."""
    return px.unoise_quads(n, r, seed, step, px.U_NOISE, k)


def init_state(n, r, D, Q, seed, stiefel=True, sigma_w=1.0):
    """GPT_SGLD.jl:357-369 on the framework streams: w = σ_w·randn(Q); U_k polar factor of
    Z = randn(r, n) (Stiefel) or randn(n,r)/sqrt(n) (non-Stiefel)."""
    w = sigma_w * px.normals(Q, seed, 0, px.W_INIT, 0)
    U = np.empty((n, r, D), order="F")
    for k in range(D):
        z = px.normals(r * n, seed, 0, px.U_INIT, k)
        if stiefel:
            U[:, :, k] = stiefel_init(z.reshape((r, n), order="F"))
        else:
            U[:, :, k] = z.reshape((r, n), order="F").T / math.sqrt(n)
    return w, U


# --------------------------------------------------------------------------- sampler
def GPTregression(phi, y, signal_var, I, r, Q, m, epsw, epsU, burnin, maxepoch, param_seed,
                  langevin=True, stiefel=True, sigma_w=1.0, store_every=1,
                  w_init=None, U_init=None, max_steps=None, record=False):
    """GPT_SGLD.jl:345-448 (Generation D).  Returns (w_store, U_store, info).

    ``store_every`` = 1 is the reference (a sample after every post-burn-in step);
    ``store_every`` = numbatches keeps the epoch-end samples the scripts consume
    (kin40kExperiment.jl:79).  ``max_steps`` truncates the run (for parity tests).
    ``info`` holds the status (0 ok, 1 NaN in geodesic; then bail_step, the 1-based step) and,
    with ``record``, per-step gradient norms and fhat.
    """
    phi = np.asarray(phi, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).ravel()
    n, D, N = phi.shape
    numbatches = -(-N // m)
    if w_init is None or U_init is None:
        w0, U0 = init_state(n, r, D, Q, param_seed, stiefel, sigma_w)
    w = np.array(w0 if w_init is None else w_init, dtype=np.float64)
    U = np.array(U0 if U_init is None else U_init, dtype=np.float64, order="F")
    nstore = (maxepoch * numbatches) // store_every
    w_store = np.zeros((Q, nstore), order="F")
    U_store = np.zeros((n, r, D, nstore), order="F")
    info = dict(status=0, gradw_norm=[], gradU_norm=[], fhat=[])
    order = np.arange(N)
    step = 0
    for epoch in range(1, burnin + maxepoch + 1):
        perm = px.randperm(N, param_seed, epoch - 1)
        order = order[perm]                      # phi=phi[:,:,perm]; y=y[perm] (cumulative)
        for batch in range(1, numbatches + 1):
            if max_steps is not None and step >= max_steps:
                return w_store, U_store, info
            idx = order[m * (batch - 1): min(m * batch, N)]
            phi_b = phi[:, :, idx]
            y_b = y[idx]
            g = gradients(phi_b, y_b, w, U, I, N, signal_var, sigma_w)
            if record:
                info["gradw_norm"].append(np.linalg.norm(g["gradw"]))
                info["gradU_norm"].append([np.linalg.norm(g["gradU"][:, :, k]) for k in range(D)])
                info["fhat"].append(g["fhat"].copy())
            if langevin:
                w = w + epsw * g["gradw"] / 2 + math.sqrt(epsw) * px.normals(Q, param_seed, step, px.W_NOISE, 0)
            else:
                w = w + epsw * g["gradw"] / 2
            if stiefel:
                for k in range(D):
                    xi = u_noise(n, r, param_seed, step, k)
                    drive = math.sqrt(epsU) * g["gradU"][:, :, k] / 2
                    mom = proj(U[:, :, k], drive + xi if langevin else drive)
                    Un, ok = geod(U[:, :, k], mom, math.sqrt(epsU))
                    if not ok:
                        info["status"] = 1
                        info["bail_step"] = step + 1          # 1-based step of the bail-out
                        return np.zeros_like(w_store), np.zeros_like(U_store), info
                    U[:, :, k] = Un
            else:
                upd = epsU * (g["gradU"] - n * U) / 2
                if langevin:
                    xi = np.stack([u_noise(n, r, param_seed, step, k) for k in range(D)], axis=2)
                    upd = upd + math.sqrt(epsU) * xi
                U = U + upd
            if epoch > burnin:
                s = (epoch - burnin - 1) * numbatches + (batch - 1)
                if (s + 1) % store_every == 0:
                    slot = (s + 1) // store_every - 1
                    w_store[:, slot] = w
                    U_store[:, :, :, slot] = U
            step += 1
    return w_store, U_store, info


def GPT_SGLDERMw(phi, y, signal_var, I, r, Q, m, epsw, burnin, maxepoch, param_seed=0,
                 w_init=None, U_init=None, max_steps=None, record=False):
    """GPT_SGLD.jl:1065-1118 — SGLD on w alone, U fixed at its uniform Stiefel draw (σ_w = 1).
    Same init, permutations and w-noise stream as GPTregression; returns (w_store, U, info)
    with w_store (Q, maxepoch·numbatches)."""
    phi = np.asarray(phi, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).ravel()
    n, D, N = phi.shape
    numbatches = -(-N // m)
    if w_init is None or U_init is None:
        w0, U0 = init_state(n, r, D, Q, param_seed, True, 1.0)
    w = np.array(w0 if w_init is None else w_init, dtype=np.float64)
    U = np.array(U0 if U_init is None else U_init, dtype=np.float64, order="F")
    w_store = np.zeros((Q, maxepoch * numbatches), order="F")
    info = dict(status=0, gradw_norm=[])
    order = np.arange(N)
    step = 0
    for epoch in range(1, burnin + maxepoch + 1):
        order = order[px.randperm(N, param_seed, epoch - 1)]
        for batch in range(1, numbatches + 1):
            if max_steps is not None and step >= max_steps:
                return w_store, U, info
            idx = order[m * (batch - 1): min(m * batch, N)]
            V = computeV(phidotU(U, phi[:, :, idx]), I)                       # :1095-1098
            fhat = V.T @ w                                                      # :1101
            gradw = (N / len(idx)) * V @ (y[idx] - fhat) / signal_var - w      # :1104
            if record:
                info["gradw_norm"].append(np.linalg.norm(gradw))
            w = w + epsw * gradw / 2 + math.sqrt(epsw) * px.normals(Q, param_seed, step, px.W_NOISE, 0)
            if epoch > burnin:
                w_store[:, (epoch - burnin - 1) * numbatches + batch - 1] = w
            step += 1
    return w_store, U, info


def init_state_cls(n, r, D, Q, ncls, seed, stiefel=True, sigma_w=1.0):
    """GPT_SGLD.jl:463-477: w = σ_w·randn(Q, C); U[:,:,k,c] uniform on the Stiefel manifold, or
    randn(n, r, D, C) (unscaled, unlike GPTregression).  Class c draws its w on (W_INIT, c) and
    U_k on (U_INIT, k + D·c) — class 0 is GPTregression's init."""
    w = np.empty((Q, ncls), order="F")
    U = np.empty((n, r, D, ncls), order="F")
    for c in range(ncls):
        w[:, c] = sigma_w * px.normals(Q, seed, 0, px.W_INIT, c)
        for k in range(D):
            z = px.normals(r * n, seed, 0, px.U_INIT, k + D * c).reshape((r, n), order="F")
            U[:, :, k, c] = stiefel_init(z) if stiefel else z.T
    return w, U


def logsumexp(x):
    """max(x) + log(sum(exp(x - max(x)))) (the logsumexp the reference calls at :513)."""
    u = np.max(x)
    return u + math.log(np.sum(np.exp(x - u)))


def gradients_res(phi_batch, res, w, U, I, N):
    """gradw = (N/B)·V·res − w and gradU_k = (N/B)·Ψ_k·res (σ_w = 1, no noise variance): the
    regression gradients with the residual supplied (GPTclassification's [y_i = c] − p_ic)."""
    n, D, B = phi_batch.shape
    r = U.shape[1]
    temp = phidotU(U, phi_batch)
    V = computeV(temp, I)
    gradw = (N / B) * (V @ res) - w
    A = computeA(computeU_phi(V, temp, I), w, I, r)
    Psi = computePsi(A, phi_batch)
    gradU = np.empty((n, r, D))
    for k in range(D):
        gradU[:, :, k] = ((N / B) * (Psi[:, :, k] @ res)).reshape((n, r), order="F")
    return gradw, gradU


def GPTclassification(phi, y, I, r, Q, m, epsw, epsU, burnin, maxepoch, param_seed,
                      langevin=True, stiefel=True, w_init=None, U_init=None, max_steps=None,
                      record=False):
    """GPT_SGLD.jl:452-680: softmax tensor-GP classifier, labels y in 1..C, σ_w = 1.

    Per minibatch: fhat[i,c] = V_cᵀw_c for every class, p_ic = exp(fhat_ic − logsumexp_i),
    residual [y_i = c] − p_ic, gradw/gradU as gradients_res.  As in the reference, w and U are
    moved TWICE with the same gradients: an unconditional SGLD + Stiefel-geodesic step (:624-636)
    and then the step selected by langevin/stiefel (:638-671), the second from the first's U.
    Noise contract: w of class c pass p on (step, W_NOISE, 2c + p); U_k of class c pass p on
    (step, U_NOISE, k + D·(2c + p)) with u_noise's layout.  Returns (w_store (Q, C, T),
    U_store (n, r, D, C, T), info); a NaN in a geodesic returns zeros like :632-634."""
    phi = np.asarray(phi, dtype=np.float64)
    yl = np.asarray(y).ravel().astype(np.int64)
    n, D, N = phi.shape
    ncls = int(yl.max() - yl.min() + 1)
    nb = -(-N // m)
    if w_init is None or U_init is None:
        w0, U0 = init_state_cls(n, r, D, Q, ncls, param_seed, stiefel, 1.0)
    w = np.array(w0 if w_init is None else w_init, dtype=np.float64, order="F")
    U = np.array(U0 if U_init is None else U_init, dtype=np.float64, order="F")
    T = maxepoch * nb
    w_store = np.zeros((Q, ncls, T), order="F")
    U_store = np.zeros((n, r, D, ncls, T), order="F")
    info = dict(status=0, gradw_norm=[], gradU_norm=[])
    order = np.arange(N)
    step = 0
    sq, sqw = math.sqrt(epsU), math.sqrt(epsw)

    def zeros():
        info["status"] = 1
        return np.zeros_like(w_store), np.zeros_like(U_store), info

    for epoch in range(1, burnin + maxepoch + 1):
        order = order[px.randperm(N, param_seed, epoch - 1)]
        for batch in range(1, nb + 1):
            if max_steps is not None and step >= max_steps:
                return w_store, U_store, info
            idx = order[m * (batch - 1): min(m * batch, N)]
            pb, yb = phi[:, :, idx], yl[idx]
            B = len(idx)
            fhat = np.stack([computefhat(computeV(phidotU(U[..., c], pb), I), w[:, c])
                             for c in range(ncls)], axis=1)                    # (B, C) :496-506
            lse = np.array([logsumexp(fhat[i, :]) for i in range(B)])
            gw, gU = [], []
            for c in range(ncls):
                res = (yb == c + 1).astype(np.float64) - np.exp(fhat[:, c] - lse)
                a, b = gradients_res(pb, res, w[:, c], U[..., c], I, N)
                gw.append(a)
                gU.append(b)
            if record:
                info["gradw_norm"].append([np.linalg.norm(g) for g in gw])
                info["gradU_norm"].append([[np.linalg.norm(gU[c][:, :, k]) for k in range(D)]
                                           for c in range(ncls)])
            for p in range(2):
                for c in range(ncls):
                    noise = (p == 0 or langevin)
                    w[:, c] += epsw * gw[c] / 2
                    if noise:
                        w[:, c] += sqw * px.normals(Q, param_seed, step, px.W_NOISE, 2 * c + p)
                for c in range(ncls):
                    for k in range(D):
                        xi = u_noise(n, r, param_seed, step, k + D * (2 * c + p))
                        G = gU[c][:, :, k]
                        if p == 0 or stiefel:
                            drive = sq * G / 2 + (xi if (p == 0 or langevin) else 0.0)
                            Un, ok = geod(U[:, :, k, c], proj(U[:, :, k, c], drive), sq)
                            if not ok:
                                return zeros()
                            U[:, :, k, c] = Un
                        else:
                            upd = epsU * (G - n * U[:, :, k, c]) / 2
                            if langevin:
                                upd = upd + sq * xi
                            U[:, :, k, c] = U[:, :, k, c] + upd
            if epoch > burnin:
                s = (epoch - burnin - 1) * nb + batch - 1
                w_store[:, :, s] = w
                U_store[:, :, :, :, s] = U
            step += 1
    return w_store, U_store, info


def geodboth(U, mom, t):
    """GPT_SGLD.jl:40-59: geodesic end point AND its velocity; (zeros, zeros, False) on NaN."""
    n, r = U.shape
    A = U.T @ mom
    T = np.block([[A, -(mom.T @ mom)], [np.eye(r), A]])
    with np.errstate(all="ignore"):
        E = expm(t * T)
    if np.isnan(E).any():
        return np.zeros((n, r)), np.zeros((n, r)), False
    mexp = expm(-t * A)
    X = np.hstack([U, mom])
    tmpU = (X @ E[:, :r]) @ mexp
    tmpV = (X @ E[:, r:]) @ mexp
    return tmpU / np.linalg.norm(tmpU, axis=0)[None, :], tmpV, True


def full_gradients(phi, y, w, U, I, signal_var):
    """GPT_GMC's full-data gradients (GPT_SGLD.jl:718-739): gradw = V(y−fhat)/σ² − w (σ_w = 1),
    gradU_k = Ψ_k(y−fhat)/σ²; also fhat."""
    n, D, N = phi.shape
    r = U.shape[1]
    temp = phidotU(U, phi)
    V = computeV(temp, I)
    fhat = computefhat(V, w)
    res = y - fhat
    gradw = V @ res / signal_var - w
    Psi = computePsi(computeA(computeU_phi(V, temp, I), w, I, r), phi)
    gradU = np.empty((n, r, D))
    for k in range(D):
        gradU[:, :, k] = (Psi[:, :, k] @ res / signal_var).reshape((n, r), order="F")
    return gradw, gradU, fhat


def GPT_GMC(phi, y, signal_var, I, r, Q, epsw, epsU, burnin, maxepoch, L, param_seed,
            w_init=None, U_init=None):
    """GPT_SGLD.jl:684-805 — geodesic Monte Carlo (full-batch HMC with the Stiefel geodesic
    flow for U), σ_w = 1.  Per epoch: p ~ N(0, I) (GMC_P stream), mom_k = proj(U_k, ξ) (GMC_MOM,
    u_noise layout), L leapfrog steps (half kick, drift: w += √εw·p and geodboth, half kick),
    H = −|w|²/2 − |y−fhat|²/(2σ²) − |mom|²/2 − |p|²/2, accept_prob = exp(H − H_old), reject
    when u > accept_prob (u on GMC_U).  As in the reference, a rejection restores w only:
    ``U_old = U`` aliases the array that the leapfrog updates in place (:710, :754), so U keeps
    its proposal.  Returns (w_store (Q, maxepoch), U_store (n, r, D, maxepoch), accept_prob);
    a NaN in a geodesic returns zeros and NaN accept probabilities (:757)."""
    phi = np.asarray(phi, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).ravel()
    n, D, N = phi.shape
    if w_init is None or U_init is None:
        w0, U0 = init_state(n, r, D, Q, param_seed, True, 1.0)
    w = np.array(w0 if w_init is None else w_init, dtype=np.float64)
    U = np.array(U0 if U_init is None else U_init, dtype=np.float64, order="F")
    w_store = np.zeros((Q, maxepoch), order="F")
    U_store = np.zeros((n, r, D, maxepoch), order="F")
    acc = np.zeros(maxepoch + burnin)
    sw, su = math.sqrt(epsw), math.sqrt(epsU)
    re = r + (r & 1)
    for epoch in range(1, burnin + maxepoch + 1):
        w_old = w
        p = px.normals(Q, param_seed, epoch - 1, px.GMC_P, 0)
        mom = np.empty((n, r, D), order="F")
        for k in range(D):
            xi = px.normals(re * n, param_seed, epoch - 1, px.GMC_MOM, k).reshape((n, re))[:, :r]
            mom[:, :, k] = proj(U[:, :, k], xi)
        H_old = (-np.sum(w * w) / 2 - np.linalg.norm(y - pred(w, U, I, phi)) ** 2 / (2 * signal_var)
                 - np.sum(mom * mom) / 2 - np.sum(p * p) / 2)
        gw, gU, fhat = full_gradients(phi, y, w, U, I, signal_var)
        for _ in range(L):
            p = p + sw * gw / 2
            for k in range(D):
                mom[:, :, k] = proj(U[:, :, k], mom[:, :, k] + su * gU[:, :, k] / 2)
            w = w + sw * p
            for k in range(D):
                Un, Vn, ok = geodboth(U[:, :, k], mom[:, :, k], su)
                if not ok:
                    return (np.zeros((Q, maxepoch)), np.zeros((n, r, D, maxepoch)),
                            np.full(maxepoch + burnin, np.nan))
                U[:, :, k], mom[:, :, k] = Un, Vn
            gw, gU, fhat = full_gradients(phi, y, w, U, I, signal_var)   # also the next kick's
            p = p + sw * gw / 2
            for k in range(D):
                mom[:, :, k] = proj(U[:, :, k], mom[:, :, k] + su * gU[:, :, k] / 2)
        H = (-np.sum(w * w) / 2 - np.linalg.norm(y - fhat) ** 2 / (2 * signal_var)
             - np.sum(mom * mom) / 2 - np.sum(p * p) / 2)
        acc[epoch - 1] = math.exp(H - H_old)
        if px.uniform(param_seed, epoch - 1, px.GMC_U, 0) > acc[epoch - 1]:
            w = w_old                                       # U stays (reference aliasing)
        if epoch > burnin:
            w_store[:, epoch - burnin - 1] = w
            U_store[:, :, :, epoch - burnin - 1] = U
    return w_store, U_store, acc


RMS_LAMBDA = 1e-5   # GPT_SGLD.jl:1146 smoothing constant


def GPT_SGLDERM_RMSprop(phi, y, signal_var, I, r, Q, m, epsilon, alpha, burnin, maxepoch,
                        param_seed=0, w_init=None, U_init=None, max_steps=None, record=False):
    """GPT_SGLD.jl:1121-1237 — SGLD with RMSprop-preconditioned step sizes (σ_w = 1).

    Differences from GPTregression, all as in the reference: the moving averages
    gw = α·gw + (1-α)·ĝw², gU = α·gU + (1-α)·ĝU² of the squared *per-sample mean* gradients
    (ĝw = V·res/(B·σ²) :1182, ĝU = Ψ_k·res/(B·σ²) :1212); per-entry step sizes
    εw = ε/(√gw + λ) (:1186) and one scalar step per dimension εU_k = mean(ε/(√gU_k + λ)) (:1218);
    **w is updated before computeA** (:1193 vs :1199), so A (and gradU) use the new w.
    Noise streams and permutations follow the framework contract of GPTregression.
    """
    phi = np.asarray(phi, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).ravel()
    n, D, N = phi.shape
    numbatches = -(-N // m)
    if w_init is None or U_init is None:
        w0, U0 = init_state(n, r, D, Q, param_seed, True, 1.0)
    w = np.array(w0 if w_init is None else w_init, dtype=np.float64)
    U = np.array(U0 if U_init is None else U_init, dtype=np.float64, order="F")
    nstore = maxepoch * numbatches
    w_store = np.zeros((Q, nstore), order="F")
    U_store = np.zeros((n, r, D, nstore), order="F")
    gw = np.zeros(Q)
    gU = np.zeros((n, r, D), order="F")
    info = dict(status=0, gradw_norm=[], gradU_norm=[])
    order = np.arange(N)
    step = 0
    for epoch in range(1, burnin + maxepoch + 1):
        order = order[px.randperm(N, param_seed, epoch - 1)]
        for batch in range(1, numbatches + 1):
            if max_steps is not None and step >= max_steps:
                return w_store, U_store, info
            idx = order[m * (batch - 1): min(m * batch, N)]
            phi_b = phi[:, :, idx]
            y_b = y[idx]
            B = len(idx)
            temp = phidotU(U, phi_b)
            V = computeV(temp, I)
            fhat = computefhat(V, w)
            res = y_b - fhat
            gradw = (1.0 / B) * (V @ res) / signal_var                       # :1182
            gw = alpha * gw + (1 - alpha) * gradw ** 2                          # :1185
            epsw = epsilon / (np.sqrt(gw) + RMS_LAMBDA)                         # :1186
            gradw = N * gradw - w                                               # :1190 (σ_w = 1)
            w = w + epsw * gradw / 2 + np.sqrt(epsw) * px.normals(Q, param_seed, step, px.W_NOISE, 0)
            U_phi = computeU_phi(V, temp, I)
            A = computeA(U_phi, w, I, r)                                        # new w (:1199)
            Psi = computePsi(A, phi_b)
            gradU = np.empty((n, r, D), order="F")
            for k in range(D):
                gradU[:, :, k] = ((1.0 / B) * (Psi[:, :, k] @ res) / signal_var).reshape((n, r), order="F")
            gU = alpha * gU + (1 - alpha) * gradU ** 2                          # :1216
            epsU = epsilon / (np.sqrt(gU) + RMS_LAMBDA)                         # :1217
            meanepsU = epsU.mean(axis=(0, 1))                                   # :1218
            gradU = gradU * N                                                   # :1227
            if record:
                info["gradw_norm"].append(np.linalg.norm(gradw))
                info["gradU_norm"].append([np.linalg.norm(gradU[:, :, k]) for k in range(D)])
            for k in range(D):
                sk = math.sqrt(meanepsU[k])
                mom = proj(U[:, :, k], sk * gradU[:, :, k] / 2 + u_noise(n, r, param_seed, step, k))
                Un, ok = geod(U[:, :, k], mom, sk)
                if not ok:
                    info["status"] = 1
                    return np.zeros_like(w_store), np.zeros_like(U_store), info
                U[:, :, k] = Un
            if epoch > burnin:
                s = (epoch - burnin - 1) * numbatches + (batch - 1)
                w_store[:, s] = w
                U_store[:, :, :, s] = U
            step += 1
    return w_store, U_store, info


def GPT_SGLDERM(phi, y, sigma, I, r, Q, m, epsw, epsU, burnin, maxepoch, param_seed=0, **kw):
    """GPT_SGLD_p.jl:146-243 (Generations A/B): ``sigma`` is the noise s.d. and
    σ_w = sqrt(n^D/Q) (:155).  Follows GPTregression's batch labels (the ``y[batch]`` slip
    at :222 is not reproduced)."""
    n, D, _ = np.asarray(phi).shape
    return GPTregression(phi, y, sigma ** 2, I, r, Q, m, epsw, epsU, burnin, maxepoch, param_seed,
                         sigma_w=math.sqrt(float(n) ** D / Q), **kw)


def GPNT_SGLD(phi, y, signal_var, sigma_theta, m, eps_theta, decay_rate, burnin, maxepoch, param_seed):
    """GPT_SGLD.jl:809-847 — full-theta RFF SGLD (config 1).  Returns theta_store (n, T)
    or zeros(n) on NaN (:840-843)."""
    phi = np.asarray(phi, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).ravel()
    n, N = phi.shape
    numbatches = -(-N // m)
    theta = sigma_theta * px.normals(n, param_seed, 0, px.THETA_INIT, 0)
    store = np.empty((n, (maxepoch + burnin) * numbatches), order="F")
    order = np.arange(N)
    t = 0
    for epoch in range(1, maxepoch + burnin + 1):
        order = order[px.randperm(N, param_seed, epoch - 1)]
        for batch in range(1, numbatches + 1):
            t += 1
            idx = order[m * (batch - 1): min(m * batch, N)]
            pb = phi[:, idx]
            yb = y[idx]
            B = len(idx)
            eps = eps_theta * t ** (-decay_rate)
            grad = -theta / sigma_theta ** 2 + (N / B) * (pb @ (yb - pb.T @ theta)) / signal_var
            theta = theta + eps * grad / 2 + math.sqrt(eps) * px.normals(n, param_seed, t - 1, px.THETA_NOISE, 0)
            store[:, t - 1] = theta
            if np.isnan(theta).any():
                return np.zeros(n)
    return store


# --------------------------------------------------------------------------- evaluation
def rmse(ytest, fhat, scale=1.0):
    """kin40kExperiment.jl:83 — ytrainStd·‖ytest − pred‖/sqrt(Ntest)."""
    ytest = np.asarray(ytest, dtype=np.float64).ravel()
    return scale * np.linalg.norm(ytest - fhat) / math.sqrt(len(ytest))


def posterior_mean_pred(w_store, U_store, I, phitest, cols=None):
    """GPT_SGLD_p.jl:124-132 (``RMSE``): mean of pred over stored samples (all, or ``cols``)."""
    cols = range(w_store.shape[1]) if cols is None else cols
    acc = None
    cnt = 0
    for s in cols:
        p = pred(w_store[:, s], U_store[:, :, :, s], I, phitest)
        acc = p if acc is None else acc + p
        cnt += 1
    return acc / cnt


# --------------------------------------------------------------------------- TGP Gibbs (a25)
def tgp_draw_I(q, D, r, seed):
    """TGP.jl:50 ``I = rand(DiscreteUniform(1, r), q, D)`` on the TGP_I stream: entry e = i + q·d
    is 1 + floor(x0·r / 2^32) of Philox block e (with replacement, unlike samplenz)."""
    x0, _, _, _ = px.philox4x32(np.arange(q * D, dtype=np.uint32), 0, px.TGP_I, 0, seed)
    return (1 + ((x0.astype(np.uint64) * np.uint64(r)) >> np.uint64(32))).astype(np.int32).reshape(
        (q, D), order="F")


def tgp_init_U(n, r, D, seed):
    """TGP.jl:48-49: U_d = sqrt(1/r)·randn(n, r) (TGP_U_INIT stream, tag d)."""
    U = np.empty((n, r, D), order="F")
    for d in range(D):
        U[:, :, d] = math.sqrt(1.0 / r) * px.normals(n * r, seed, 0, px.TGP_U_INIT, d).reshape(
            (n, r), order="F")
    return U


def tgp_V(U, I, b):
    """TGP.jl:55: V[i,j] = Π_d U_d[:, I[i,d]]ᵀ b[:, d, j]  (q × N)."""
    return computeV(phidotU(U, b), I)


def GPT_inf(b, y, sigma, n, r, q, num_iterations, burnin, seed, I=None):
    r"""TGP.jl:37-86 (Gibbs sweep of the tensor GP) on whitened data: ``b`` (n, D, N) is the
    feature array of TGP.feature (TGP.jl:6-14) and ``y`` (N) the whitened targets.

    Per sweep: W ~ N(Mu_w, invSigma_w⁻¹) through the upper Cholesky factor (:57-59); for each k
    the leave-one-out C (r × N, run sums over I[:,k]), Ck = C ⊗ b_k, invSigma_U = CkCkᵀ/σ² + r·I,
    U_k = invSigma_U⁻¹ z + Mu_U (:76-79 — ``factorize(invSigma_U) \ randn`` solves, as in the
    reference) and V refreshed with the new U_k (:81).  Runs C[l,:] of values l absent from
    I[:,k] are uninitialised in the reference (Array(Float64,r,N)); here they are 0.
    Returns (W_array (q, T), V_array (n, r, D, T), I), T = num_iterations - burnin."""
    from scipy.linalg import solve_triangular
    b = np.asarray(b, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).ravel()
    _, D, N = b.shape
    sigma_u = math.sqrt(1.0 / r)
    sigma_w = math.sqrt(float(r) ** D / q)
    U = tgp_init_U(n, r, D, seed)
    if I is None:
        I = tgp_draw_I(q, D, r, seed)
    T = num_iterations - burnin
    W_array = np.zeros((q, T), order="F")
    V_array = np.zeros((n, r, D, T), order="F")
    s2 = sigma ** 2
    for it in range(1, num_iterations + 1):
        temp = phidotU(U, b)
        V = computeV(temp, I)
        inv_w = V @ V.T / s2 + np.eye(q) / sigma_w ** 2
        L = np.linalg.cholesky(inv_w)
        mu = solve_triangular(L.T, solve_triangular(L, V @ y / s2, lower=True), lower=False)
        z = px.normals(q, seed, it - 1, px.TGP_W_NOISE, 0)
        W = solve_triangular(L.T, z, lower=False) + mu                         # chol(·,:U) \ z
        if it > burnin:
            W_array[:, it - burnin - 1] = W
            V_array[:, :, :, it - burnin - 1] = U
        for k in range(D):
            tk = temp[k, I[:, k] - 1, :]                                        # (q, N)
            Vk = V / tk
            Vkk = W[:, None] * Vk
            C = np.zeros((r, N))
            for l in range(1, r + 1):
                sel = I[:, k] == l
                if sel.any():
                    C[l - 1, :] = Vkk[sel, :].sum(axis=0)
            Ck = (C[:, None, :] * b[None, :, k, :]).reshape((r * n, N))          # row (l, j) -> l·n + j
            inv_u = Ck @ Ck.T / s2 + np.eye(n * r) / sigma_u ** 2
            Lu = np.linalg.cholesky(inv_u)
            rhs = Ck @ y / s2
            zu = px.normals(n * r, seed, it - 1, px.TGP_U_NOISE, k)
            x = solve_triangular(Lu.T, solve_triangular(Lu, rhs + zu, lower=True), lower=False)
            U[:, :, k] = x.reshape((n, r), order="F")
            temp[k] = U[:, :, k].T @ b[:, k, :]
            V = Vk * temp[k, I[:, k] - 1, :]
    return W_array, V_array, I
