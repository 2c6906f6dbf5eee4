"""Philox4x32-10 random streams — the RNG contract shared by the HIP path and the oracle.

TEST INFRASTRUCTURE.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import anything under ``oracle/``; the product path
(``gpt_amd``) never does.

Julia's MersenneTwister/Ziggurat stream (``srand``/``randn``/``randperm``,
GPT_SGLD.jl:357,360,365,373,412,420) cannot be reproduced here (no Julia), so the
framework defines its own counter-based streams.  The *consumption points* follow the
reference one for one (SURVEY.md §8(a) "RNG consumption order"):

    stream        counter (c0, c1, c2, c3)           reference draw
    ------------  ---------------------------------  -------------------------------
    W_INIT        (e>>1, 0,      W_INIT,  0)           w = randn(Q)          :360
    U_INIT        (e>>1, 0,      U_INIT,  k)           Z = randn(r, n)       :365
    PERM          (i,    epoch,  PERM,    0)           randperm(N)           :373
    W_NOISE       (e>>1, step,   W_NOISE, 0)           randn(Q)              :412
    U_NOISE       (c0,   step,   U_NOISE, k)           randn(n, r)           :420
                  quads: ξ[λ + 64(4q+i), l] for i < 4 from c0 = (l·NQ + q)·64 + λ,
                  NQ = ceil(ceil(n/64)/4) (see ``unoise_quads``)
    THETA_INIT    (e>>1, 0,      TH_INIT, 0)           theta = randn(n)      :815
    THETA_NOISE   (e>>1, t,      TH_NOISE,0)           randn(n)              :836

key = (seed & 0xffffffff, seed >> 32).  Element ``e`` of a normal stream comes from the
Philox block at c0 = e>>1: two 53-bit uniforms u1, u2 and the Box–Muller pair
(z0, z1) = sqrt(-2 ln u1)·(cos 2πu2, sin 2πu2); element e takes z0 if e is even, z1 if
odd.  Column-major element order matches Julia's ``randn(r, n)`` / ``randn(n, r)``.
``randperm`` is Fisher–Yates from the top: for i = N-1 … 1, j = floor(u32(i)·(i+1)/2^32),
swap(p[i], p[j]).
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

W_INIT, U_INIT, PERM, W_NOISE, U_NOISE, THETA_INIT, THETA_NOISE = 1, 2, 3, 4, 5, 6, 7
# TGP Gibbs (TGP.jl:37-86): U init, the core index draw, and the two Gaussian draws per sweep
TGP_U_INIT, TGP_I, TGP_W_NOISE, TGP_U_NOISE = 11, 12, 13, 14
# GPT_GMC (GPT_SGLD.jl:684-805): momentum of w, momentum of U, the accept/reject uniform
GMC_P, GMC_MOM, GMC_U = 15, 16, 17
# MovieLens tensor CF (100k_movielensExperiment.jl:409-551): U/V init, w noise, U/V noise
CF_UV_INIT, CF_W_NOISE, CF_UV_NOISE = 18, 19, 20
# GPT_fullw_gibbs (100k_movielensExperiment.jl:1032-1129): init (QR draw, U, V), per-sweep draws
CFG_INIT, CFG_U, CFG_V, CFG_W = 21, 22, 23, 24


def philox4x32(c0, c1, c2, c3, seed):
    """Vectorised Philox4x32-10.  c* are uint32 arrays (broadcastable); returns 4 uint32 arrays."""
    c0 = np.asarray(c0, dtype=np.uint32)
    c1 = np.asarray(c1, dtype=np.uint32)
    c2 = np.asarray(c2, dtype=np.uint32)
    c3 = np.asarray(c3, dtype=np.uint32)
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    c0 = c0.copy(); c1 = c1.copy(); c2 = c2.copy(); c3 = c3.copy()
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    k0 = np.uint32(seed & 0xFFFFFFFF)
    k1 = np.uint32(seed >> 32)
    with np.errstate(over="ignore"):
        for rnd in range(10):
            if rnd > 0:
                k0 = np.uint32((int(k0) + int(W0)) & 0xFFFFFFFF)
                k1 = np.uint32((int(k1) + int(W1)) & 0xFFFFFFFF)
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & MASK32).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & MASK32).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return c0, c1, c2, c3


def _u53(a, b):
    """Two uint32 words -> uniform double in (0, 1) with 53 random bits."""
    return ((a >> np.uint32(5)).astype(np.float64) * 67108864.0
            + (b >> np.uint32(6)).astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)


def normals(count, seed, c1, c2, c3):
    """``count`` standard normals of stream (c1, c2, c3) — element e at index e."""
    count = int(count)
    nblk = (count + 1) // 2
    x0, x1, x2, x3 = philox4x32(np.arange(nblk, dtype=np.uint32), c1, c2, c3, seed)
    u1 = _u53(x0, x1)
    u2 = _u53(x2, x3)
    rad = np.sqrt(-2.0 * np.log(u1))
    th = 2.0 * np.pi * u2
    z = np.empty(2 * nblk, dtype=np.float64)
    z[0::2] = rad * np.cos(th)
    z[1::2] = rad * np.sin(th)
    return z[:count]


def _u32(x):
    """One uint32 word -> uniform double in (0, 1): (x + 1/2)·2^-32."""
    return (x.astype(np.float64) + 0.5) * (1.0 / 4294967296.0)


def unoise_quads(n, r, seed, c1, c2, c3):
    """The n×r noise matrix of the U_NOISE contract (gpt_common.h normal_quad).  Rows come in
    blocks of 64 (row j = λ + 64·b); Philox block c0 = (l·NQ + q)·64 + λ, NQ = ceil(ceil(n/64)/4),
    gives column l of rows λ + 64·(4q + i), i = 0..3, as two Box–Muller pairs of 32-bit
    uniforms u(x) = (x + 1/2)·2^-32: (z0, z1) = sqrt(-2 ln u(x0))·(cos 2πu(x1), sin 2πu(x1)) and
    (z2, z3) from (x2, x3).  Rows >= n are dropped."""
    n, r = int(n), int(r)
    nq = (-(-n // 64) + 3) // 4
    c0 = np.arange(r * nq * 64, dtype=np.uint32)
    x0, x1, x2, x3 = philox4x32(c0, c1, c2, c3, seed)
    ra = np.sqrt(-2.0 * np.log(_u32(x0)))
    rb = np.sqrt(-2.0 * np.log(_u32(x2)))
    ta, tb = 2.0 * np.pi * _u32(x1), 2.0 * np.pi * _u32(x3)
    z = np.stack([ra * np.cos(ta), ra * np.sin(ta), rb * np.cos(tb), rb * np.sin(tb)])  # (4, cnt)
    idx = np.arange(r * nq * 64)
    l, q, lam = idx // (nq * 64), (idx // 64) % nq, idx % 64
    out = np.empty((nq * 4 * 64, r))
    for i in range(4):
        out[lam + 64 * (4 * q + i), l] = z[i]
    return out[:n]


def uniform(seed, c1, c2, c3):
    """One uniform on (0, 1): u53 of the first two words of Philox block 0 of (c1, c2, c3)."""
    x0, x1, _, _ = philox4x32(np.zeros(1, dtype=np.uint32), c1, c2, c3, seed)
    return float(_u53(x0, x1)[0])


def randperm(N, seed, epoch):
    """0-based permutation of range(N) (Fisher–Yates, PERM stream of ``epoch``)."""
    N = int(N)
    p = np.arange(N, dtype=np.int64)
    if N <= 1:
        return p
    i = np.arange(N, dtype=np.uint32)
    x0, _, _, _ = philox4x32(i, epoch, PERM, 0, seed)
    x0 = x0.astype(np.uint64)
    for ii in range(N - 1, 0, -1):
        j = int((int(x0[ii]) * (ii + 1)) >> 32)
        p[ii], p[j] = p[j], p[ii]
    return p
