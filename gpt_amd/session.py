"""Device-resident multi-chain SGLD sessions (the benchmark and multi-GPU path).

Inputs stay in HBM as torch tensors (PyTorch is only the allocator/stream plumbing); every
chain step runs in libgptsgld.so's fused HIP kernel.  Chains share the configuration and
may share or own their (phi, y) (a hyper-parameter sweep gives each chain its own phi, as
kin40kExperiment.jl:67-72 does; posterior chains share one, BASELINE config 4).
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import SGLDConfig, check, lib
from .GPT_SGLD import make_config


# store_flags bits selecting the step engine (include/gptsgld.h, gpt_sgld_session_info)
ENGINES = {"auto": 0, "grid": 4, "chain": 8, "wave": 128}
ENGINE_NAMES = {0: "grid", 1: "chain", 3: "wave"}


class SGLDSession:
    def __init__(self, phis, ys, I, r, Q, m, epsw, epsU, signal_var, burnin, maxepoch, seeds,
                 sigma_w=1.0, langevin=True, stiefel=True, store_every=1, max_steps=0,
                 store=True, diag=False, stream=None, engine="auto"):
        import torch
        if not isinstance(phis, (list, tuple)):
            phis = [phis]
        if not isinstance(ys, (list, tuple)):
            ys = [ys]
        seeds = list(seeds)
        nch = len(seeds)
        if len(phis) == 1 and nch > 1:
            phis = phis * nch
        if len(ys) == 1 and nch > 1:
            ys = ys * nch
        if len(phis) != nch or len(ys) != nch:
            raise ValueError("need one (phi, y) per chain or a shared one")
        for p in phis:
            if p.dtype != torch.float64 or not p.is_cuda or p.dim() != 3 or not p.is_contiguous():
                raise ValueError("phi must be a contiguous float64 device tensor of torch shape "
                                 "(N, D, n) == Julia phi (n, D, N)")
        N, D, n = phis[0].shape     # torch (N, D, n) row-major == Julia (n, D, N) column-major
        self._keep = (phis, ys)
        self.n, self.D, self.N, self.r, self.Q, self.m = int(n), int(D), int(N), r, Q, m
        self.nchains = nch
        I = np.asfortranarray(np.asarray(I, dtype=np.int32))
        self.cfg = make_config(self.n, self.D, self.N, r, Q, m, epsw, epsU, signal_var, sigma_w,
                               burnin, maxepoch, 0, langevin, stiefel, store_every, max_steps)
        pp = (C.c_void_p * nch)(*[p.data_ptr() for p in phis])
        yy = (C.c_void_p * nch)(*[y.data_ptr() for y in ys])
        sd = (C.c_uint64 * nch)(*[int(s) & (2 ** 64 - 1) for s in seeds])
        h = C.c_void_p()
        if engine not in ENGINES:
            raise ValueError("engine must be one of %s" % sorted(ENGINES))
        flags = (1 if store else 0) | (2 if diag else 0) | ENGINES[engine]
        st = C.c_void_p(stream) if stream else None
        check(lib().gpt_sgld_session_create(C.byref(self.cfg), nch, sd, pp, yy,
                                            I.ctypes.data_as(_lib.P_I32), flags, st, C.byref(h)))
        self._h = h
        self.numbatches = -(-self.N // m)
        total = (burnin + maxepoch) * self.numbatches
        self.total_steps = total if max_steps <= 0 else min(total, max_steps)
        self.nstore = (maxepoch * self.numbatches) // store_every

    def set_hyper(self, chain, epsw, epsU, signal_var, sigma_w=1.0):
        check(lib().gpt_sgld_session_set_hyper(self._h, chain, float(epsw), float(epsU),
                                               float(signal_var), float(sigma_w)))

    def set_rmsprop(self, epsilon, alpha):
        """Switch this (grid-engine) session to GPT_SGLDERM_RMSprop steps (GPT_SGLD.jl:1121)."""
        check(lib().gpt_sgld_session_set_rmsprop(self._h, float(epsilon), float(alpha)))

    def run(self, nsteps):
        check(lib().gpt_sgld_session_run(self._h, int(nsteps)))

    def prepare(self, nsteps):
        """Capture the graphs the next ``run(nsteps)`` replays (nothing runs): a timed run then
        launches graphs only."""
        check(lib().gpt_sgld_session_prepare(self._h, int(nsteps)))

    def time_steps(self, nsteps):
        """Run nsteps un-captured steps with a hipEvent pair around every step-kernel launch;
        returns the mean step-kernel duration in microseconds."""
        avg = C.c_double(0.0)
        check(lib().gpt_sgld_session_time_steps(self._h, int(nsteps), C.byref(avg)))
        return avg.value

    def info(self):
        """dict(engine, lds_bytes, threads, workgroups) of the step launch."""
        out = (C.c_int64 * 4)()
        check(lib().gpt_sgld_session_info(self._h, out))
        return dict(engine=ENGINE_NAMES.get(out[0], str(out[0])), lds_bytes=out[1],
                    threads=out[2], workgroups=out[3])

    def sync(self):
        check(lib().gpt_sgld_session_sync(self._h))

    @property
    def steps_done(self):
        return int(lib().gpt_sgld_session_steps_done(self._h))

    def device_state(self, chain):
        w = C.c_void_p(); U = C.c_void_p(); ws = C.c_void_p(); Us = C.c_void_p(); ns = C.c_int64()
        check(lib().gpt_sgld_session_state(self._h, chain, C.byref(w), C.byref(U), C.byref(ws),
                                           C.byref(Us), C.byref(ns)))
        return w.value, U.value, ws.value, Us.value, ns.value

    def gather_state(self, first, count, w_out, U_out):
        """Current (w, U) of chains first..first+count-1 into device tensors w_out (count, Q) and
        U_out (count, n*r*D), on the session stream (call sync() before another stream reads)."""
        check(lib().gpt_sgld_session_gather_state(self._h, first, count,
                                                  C.c_void_p(w_out.data_ptr()),
                                                  C.c_void_p(U_out.data_ptr())))

    def status(self, chain):
        """GPT_OK, or GPT_ERR_NAN_GEODESIC when chain hit the geodesic bail-out (4 bytes copied)."""
        st = C.c_int32(0)
        check(lib().gpt_sgld_session_fetch(self._h, chain, None, None, None, C.byref(st)))
        return st.value

    def fetch(self, chain, diag=False):
        """(w_store, U_store, status[, diag]) of one chain, host numpy in Julia layout."""
        ws = np.zeros((self.Q, self.nstore), order="F")
        Us = np.zeros((self.n, self.r, self.D, self.nstore), order="F")
        dg = np.zeros((1 + self.D, self.total_steps), order="F") if diag else None
        st = C.c_int32(0)
        check(lib().gpt_sgld_session_fetch(self._h, chain, ws.ctypes.data_as(_lib.P_D),
                                           Us.ctypes.data_as(_lib.P_D),
                                           dg.ctypes.data_as(_lib.P_D) if diag else None,
                                           C.byref(st)))
        return (ws, Us, st.value, dg) if diag else (ws, Us, st.value)

    def diagnostics(self, chain):
        """(diag (1 + D, total_steps), status) of one chain of a session created with diag=True:
        per step [‖gradw‖, ‖gradU_1‖ … ‖gradU_D‖] (engine-dependent rows; zero past a bail-out)."""
        dg = np.zeros((1 + self.D, self.total_steps), order="F")
        st = C.c_int32(0)
        check(lib().gpt_sgld_session_fetch(self._h, chain, None, None,
                                           dg.ctypes.data_as(_lib.P_D), C.byref(st)))
        return dg, st.value

    def bail_step(self, chain):
        """1-based step at which a bailed-out chain hit the geodesic NaN (GPT_SGLD.jl:422-424):
        the last step with a gradient norm in the diagnostic rows; 0 for a live chain."""
        dg, st = self.diagnostics(chain)
        if st == 0:
            return 0
        nz = np.flatnonzero(dg[0])
        return int(nz[-1]) + 1 if nz.size else 0

    def close(self):
        if getattr(self, "_h", None):
            lib().gpt_sgld_session_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def feature_device(X, length_scale, sigma_RBF, phi_scale, Z, b, stream=None):
    """phi on the device (torch (N, D, n) == Julia (n, D, N)) from device tensors X (N, D)
    [Julia column-major => torch (D, N)], Z/b (n, D) [torch (D, n)], length_scale (D,)."""
    import torch
    D, N = X.shape
    n = Z.shape[1]
    phi = torch.empty((N, D, n), dtype=torch.float64, device=X.device)
    check(lib().gpt_feature_dev(C.c_void_p(X.data_ptr()), N, D, C.c_void_p(length_scale.data_ptr()),
                                D, float(sigma_RBF), float(phi_scale), C.c_void_p(Z.data_ptr()),
                                C.c_void_p(b.data_ptr()), n, C.c_void_p(phi.data_ptr()),
                                C.c_void_p(stream) if stream else None))
    return phi


def pred_device_timed(w_ptr, U_ptr, I0_dev, phitest, n, D, Ntest, r, Q, S, fhat_out):
    """pred_device on the null stream with per-phase event timing: (gemm_ms, vphase_ms)."""
    ms = np.zeros(2)
    check(lib().gpt_pred_dev_timed(C.c_void_p(w_ptr), C.c_void_p(U_ptr),
                                   C.c_void_p(I0_dev.data_ptr()), C.c_void_p(phitest.data_ptr()),
                                   n, D, Ntest, r, Q, S, C.c_void_p(fhat_out.data_ptr()), None,
                                   ms.ctypes.data_as(_lib.P_D)))
    return float(ms[0]), float(ms[1])


def pred_device(w_ptr, U_ptr, I0_dev, phitest, n, D, Ntest, r, Q, S, fhat_out, stream=None):
    """fhat (Ntest, S) on the device from S consecutive samples at w_ptr / U_ptr."""
    check(lib().gpt_pred_dev(C.c_void_p(w_ptr), C.c_void_p(U_ptr), C.c_void_p(I0_dev.data_ptr()),
                             C.c_void_p(phitest.data_ptr()), n, D, Ntest, r, Q, S,
                             C.c_void_p(fhat_out.data_ptr()), C.c_void_p(stream) if stream else None))


VPHASE_KERNELS = {0: "pred_vphase_pairs_kernel", 1: "pred_vphase_rows_pf_kernel",
                  2: "pred_vphase_rows_kernel", 4: "pred_kernel (direct, no separate V-phase)"}


def pred_last_vphase():
    """Name of the V-phase kernel the last prediction call on this thread launched
    (gpt_pred_last_vphase), or None before any call."""
    k = C.c_int32(-1)
    check(lib().gpt_pred_last_vphase(C.byref(k)))
    return VPHASE_KERNELS.get(k.value)
