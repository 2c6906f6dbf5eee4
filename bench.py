"""Benchmark: SGLD steps/s of the tensor-GP sampler on kin40k (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--chains C] ...
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workload (BASELINE config 3/4): kin40k — Ntrain = 10 000 rows (the reference's
own kin40k_train files, whitened as kin40kExperiment.jl:25-37), D = 8, n = 500 random
features per dimension, rank r = 5, Q = 200, minibatch m = 50, σ² = 0.0476, ℓ/σ_RBF of
kin40kExperiment.jl:22-23, εw = 1e-5, εU = 1e-8 (the script's 1e-4 / 1e-7 diverge at n = 500,
r = 5 in the oracle and on the GPU alike).  phi (320 MB) is built on the device by
the feature kernel and stays resident in HBM.  Each GPU runs C independent posterior chains
(seeds differ, phi shared — BASELINE config 4 has one chain per GPU; C chains per GPU is the
same thing with the GPU filled).  A "step" is one SGLD step of one chain over one minibatch;
value = chain-steps/s summed over all chains and GPUs (weak scaling: work per GPU fixed).
After the timed region each GPU predicts the 30 000 test rows with its chains' final
samples; ranks all-reduce (RCCL) the predictive mean and rank 0 reports the ensemble RMSE.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_MFMA_PEAK_TFS = 78.6     # MI355X dense FP64 matrix peak (AMD spec; v_mfma_f64_16x16x4f64)
FP64_PEAK_TFLOPS = 78.6        # MI355X fp64 vector/matrix peak (spec)


def kin40k(D):
    d = np.load(os.path.join(ROOT, "tests", "golden", "kin40k.npz"))
    Xtr, ytr, Xte, yte = d["Xtrain"], d["ytrain"].ravel(), d["Xtest"], d["ytest"].ravel()
    mu, sd = Xtr.mean(axis=0), Xtr.std(axis=0, ddof=1)
    ymu, ysd = ytr.mean(), ytr.std(ddof=1)
    Xtr = (Xtr - mu) / sd                       # datawhitening (GPT_SGLD.jl:62-67)
    Xte = (Xte - mu) / sd                       # kin40kExperiment.jl:36
    return Xtr[:, :D], (ytr - ymu) / ysd, Xte[:, :D], (yte - ymu) / ysd, ysd


def powerplant(D, ntrain=5000):
    """BASELINE config 2 (SURVEY §8 canonical shapes): Folds5x2_pp.csv rows 1..5000 train, the
    other 4568 test, whitened with the train moments as PowerPlantDataExperiment.jl:25-37."""
    d = np.load(os.path.join(ROOT, "tests", "golden", "powerplant.npz"))["data"]
    Xtr, ytr, Xte, yte = d[:ntrain, :D], d[:ntrain, D], d[ntrain:, :D], d[ntrain:, D]
    mu, sd = Xtr.mean(axis=0), Xtr.std(axis=0, ddof=1)
    ymu, ysd = ytr.mean(), ytr.std(ddof=1)
    return (Xtr - mu) / sd, (ytr - ymu) / ysd, (Xte - mu) / sd, (yte - ymu) / ysd, ysd


KIN40K_LS = [2.5242, 2.3376, 1.3630, 1.4949, 1.6022, 1.1366, 1.1964, 1.7028]
WORKLOADS = {
    # name: (loader, D, minibatch, length scales, sigma_RBF, signal_var, description,
    #        defaults n, r, epsw, epsU)
    "kin40k": (kin40k, 8, 50, KIN40K_LS, 1.0420, 0.0476, "kin40k tensor-GP SGLD (GPTregression)",
               500, 5, 1e-5, 1e-8),
    # the configuration kin40kExperiment.jl itself runs (:38-51: n = 150, r = 20, Q = 200, m = 50,
    # εw = 1e-4, εU = 1e-7) — the only kin40k shape with a reference test-RMSE curve
    # (testRMSE_kin40k.h5): the wave engine (wave.hip)
    "kin40k_ref": (kin40k, 8, 50, KIN40K_LS, 1.0420, 0.0476,
                   "kin40k tensor-GP SGLD at kin40kExperiment.jl's configuration (GPTregression)",
                   150, 20, 1e-4, 1e-7),
    # εw = 5e-5, εU = 2e-8: the round-4 oracle sweep's best stable pair at this shape
    # (scripts/pp_step_sweep.py; tests/test_gpu_quality.py)
    "powerplant": (powerplant, 4, 256, [1.4332] * 4, 1.0, 0.2299 ** 2,
                   "PowerPlant tensor-GP SGLD (GPTregression), BASELINE config 2", 500, 5, 5e-5, 2e-8),
}
METRICS = {
    "kin40k": "SGLD steps/sec (kin40k, n_feat=500/dim, r=5)",
    "kin40k_ref": "SGLD steps/sec + test RMSE (kin40kExperiment.jl: n_feat=150/dim, r=20, m=50)",
    "powerplant": "SGLD steps/sec (PowerPlant, n_feat=500/dim, r=5, minibatch 256)",
}
KERNELS = {"chain": "chain_kernel<%d,J,2>", "grid": "sgld_step_kernel<%d>",
           "wave": "wv_vphase_kernel<%d> + wv_dim_kernel<%d,J>"}
KERNEL_LAUNCHES = {"chain": "one chain_kernel launch runs the steps up to the end of an epoch",
                   "grid": "one sgld_step_kernel launch per step",
                   "wave": "two launches per step: wv_vphase_kernel, then wv_dim_kernel"}
KERNEL_US_NOTE = ("device time per step of all chains: one hipEvent pair on the session stream "
                  "around the %d timed steps' graph launches (kernel gaps inside the graphs "
                  "included), / steps; %s")


def profile_marker(stream):
    """A ~2 µs spin kernel on `stream`, launched outside the timed region on both sides of it:
    scripts/prof_timed.py takes the dispatches between the two markers of a kernel trace as the
    timed steps."""
    import torch
    with torch.cuda.stream(stream):
        torch.cuda._sleep(4000)


def algorithmic_bytes_per_step(n, D, B, r, Q):
    """8·(n·D·B + B + 2·n·r·D + 2·Q) + 4·Q·D bytes per SGLD step."""
    return 8 * (n * D * B + B + 2 * n * r * D + 2 * Q) + 4 * Q * D


def algorithmic_flops_per_step(n, D, B, r, Q):
    """4nrDB + 3QDB + 4QB + D(14nr² + 2·30·(2r)³) flops per SGLD step (the last
    term prices geod's two expm at 30 (2r)³-products, a generous Padé count)."""
    return 4 * n * r * D * B + 3 * Q * D * B + 4 * Q * B + D * (14 * n * r * r + 2 * 30 * (2 * r) ** 3)


def executed_flops_per_step(n, D, B, r, Q):
    """The flops the wave engine executes per step at the Padé degree the kin40k runs take (5 for
    the 2r x 2r expm: three products, an LU and the r right-hand sides geod reads; degree 3 for the
    r x r one: two products, an LU with r right-hand sides), for comparison with the §8(d) count:
    phidotU + gradU 4nrDB, V / A 3QDB, fhat / gradw 4QB, proj + Grams + tmpU D·(2nr² · 5 + 2·2nr·r),
    the expm D·(3·2(2r)³ + (2/3)(2r)³ + 2(2r)²·r + 2·2r³ + (8/3)r³)."""
    nn = 2 * r
    expm = 3 * 2 * nn ** 3 + 2 * nn ** 3 / 3 + 2 * nn ** 2 * r + 2 * 2 * r ** 3 + 8 * r ** 3 / 3
    return (4 * n * r * D * B + 3 * Q * D * B + 4 * Q * B
            + D * (2 * n * r * r * 5 + 2 * 2 * n * r * r + expm))


def _cpu_threads():
    """Host threads for the CPU baseline: the box's CPU share (OMP_NUM_THREADS is set to it on
    the GPU box), else every CPU this process may run on."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:                               # pragma: no cover
        return os.cpu_count() or 1


def cpu_baseline(phi_np, y_np, I, args, seconds):
    """The C++ fp64 restatement of GPT_SGLD.jl:345-448 (oracle/cpu, test infrastructure) on the
    same workload, bounded to about ``seconds`` of wall time: 1 chain on 1 core, then T chains on
    T cores (OpenMP over chains).  Falls back to the numpy oracle (1 core) when the
    library was not built."""
    N = phi_np.shape[2]
    nb = -(-N // args.m)
    try:
        from oracle import cpu_lib
        cpu_lib.lib()
    except Exception as exc:                             # pragma: no cover
        cpu_lib = None
        why = str(exc)
    if cpu_lib is None:
        from oracle import gpt_sgld_ref as R
        steps = 20
        t0 = time.perf_counter()
        R.GPTregression(phi_np, y_np, args.signal_var, I, args.r, args.Q, args.m, args.epsw,
                        args.epsU, 0, -(-steps // nb), 1, max_steps=steps, store_every=nb)
        dt = time.perf_counter() - t0
        return dict(value=steps / dt, unit="SGLD steps/s (1 chain)", cores=1, kind="port",
                    sample="numpy oracle, %d steps (C++ restatement unavailable: %s)" % (steps, why))

    def run(chains, threads, steps):
        epochs = -(-steps // nb)
        o = cpu_lib.GPTregression_chains(phi_np, y_np, args.signal_var, I, args.r, args.Q, args.m,
                                         args.epsw, args.epsU, 0, epochs,
                                         [1000 + c for c in range(chains)], threads=threads,
                                         store_every=epochs * nb, max_steps=steps)
        return o["steps"] / o["seconds"], o["steps"], o["seconds"]

    probe, _, _ = run(1, 1, 20)
    s1 = max(20, int(probe * 0.3 * seconds))
    one, st1, dt1 = run(1, 1, s1)
    T = _cpu_threads()
    sT = max(10, int(one * 0.6 * seconds))               # per chain: ~0.6·seconds if T cores scale
    allc, stT, dtT = run(T, T, sT)
    return dict(value=allc, unit="chain-steps/s (%d chains on %d cores)" % (T, T), cores=T,
                kind="port", single_core_steps_per_s=one, nproc=os.cpu_count(),
                cpu_model=cpu_lib.cpu_model(),
                sample="oracle/cpu/gpt_sgld_cpu.cpp (C++ fp64 restatement of GPT_SGLD.jl:345-448, "
                       "OpenMP over chains, no BLAS) on the %s config (n=%d, D=%d, r=%d, Q=%d, m=%d): "
                       "1 chain x %d steps on 1 core in %.1f s; %d chains x %d steps on %d cores in "
                       "%.1f s" % (args.workload, args.n, args.D, args.r, args.Q, args.m, st1, dt1,
                                   T, sT, T, dtT))


def cpu_pred_baseline(phi_te, w_all, U_all, fh, I, n, D, r, seconds):
    """CPU side of the stacked-sample prediction (BASELINE.md:34): the C++ restatement of pred
    (GPT_SGLD.jl:233-243, oracle/cpu) over all test rows for as many of the GPU's samples as fit
    about seconds/4 on the host's cores, checked against the GPU's fhat of the same samples;
    reported per sample and extrapolated to the GPU call's sample count."""
    from oracle import cpu_lib
    T = _cpu_threads()
    pt = np.asfortranarray(phi_te.cpu().numpy().transpose(2, 1, 0))     # (n, D, Ntest)
    Nte, Stot = pt.shape[2], w_all.shape[0]
    wn, Un = w_all.cpu().numpy(), U_all.cpu().numpy()
    def sample_args(S):
        return (np.asfortranarray(wn[:S].T),
                np.reshape(Un[:S].T, (n, r, D, S), order="F"))
    w1, U1 = sample_args(1)
    _, sec1 = cpu_lib.pred(w1, U1, I, pt, threads=T)
    S = int(max(1, min(Stot, (0.25 * seconds) / max(sec1, 1e-6))))
    wS, US = sample_args(S)
    f, secS = cpu_lib.pred(wS, US, I, pt, threads=T)
    ref = fh[:S].cpu().numpy()
    return dict(ms_per_sample=1e3 * secS / S, samples_timed=S, Ntest=int(Nte), cores=T,
                ms_est_for_gpu_call=1e3 * secS / S * Stot, gpu_call_samples=int(Stot),
                max_rel_diff_vs_gpu=float(np.abs(f - ref).max() / np.abs(ref).max()),
                sample="oracle/cpu gptcpu_pred (pred of GPT_SGLD.jl:233-243, OpenMP over test "
                       "rows) on %d of the GPU call's samples x %d test rows, %d cores"
                       % (S, Nte, T))


def cpu_b256_baseline(phi_np, y_np, I, args, seconds):
    """BASELINE.md:35's minibatch-256 variant of the CPU chain (1 chain, 1 core, ~seconds/6)."""
    from oracle import cpu_lib
    N = phi_np.shape[2]
    nb = -(-N // 256)
    def run(steps):
        o = cpu_lib.GPTregression_chains(phi_np, y_np, args.signal_var, I, args.r, args.Q, 256,
                                         args.epsw, args.epsU, 0, -(-steps // nb), [1000],
                                         threads=1, store_every=(-(-steps // nb)) * nb,
                                         max_steps=steps)
        return o["steps"] / o["seconds"], o["steps"], o["seconds"]
    probe, _, _ = run(4)
    sps, st, dt = run(max(4, int(probe * seconds / 6)))
    return dict(value=sps, unit="SGLD steps/s (1 chain, 1 core, minibatch 256)", steps=st,
                seconds=dt)


def chain_seeds(rank, C):
    """param_seed of chain c on this rank: rank·C + c + 1 — distinct over all ranks and chains
    (kin40kExperiment.jl:68 seeds its chains 1..J)."""
    return [rank * C + c + 1 for c in range(C)]


def scratch_seeds(rank, C):
    """Seeds of the clock warm-up's scratch chains (disjoint from chain_seeds at any world size)."""
    return [(1 << 40) + rank * C + c for c in range(C)]


def launch_command(argv, nproc, port, script=None):
    """The torchrun command bench.py re-runs itself under for --gpus N > 1 (one rank per GPU)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            "--nproc-per-node", str(nproc), "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(script or __file__)] + list(argv)


def self_launch(argv, nproc, script=None):
    """Start N ranks as a child torchrun and return its exit code.  Called before anything in
    this process touches the GPU (no exec: a child process)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(launch_command(argv, nproc, port, script), env=env)


def max_over_ranks(dt, device=None):
    """Slowest rank's wall time (the timed region's value is whole-job work over this)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return dt
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def compose_line(v):
    """The bench's JSON line (rank 0) from the measured values in namespace v.  Every N keeps the
    same fields: cpu_baseline (rank 0's host cores), kernel_us per rank, the single-chain pass."""
    a = v.args
    pred_tfs = v.pred_flop / (v.pred_ms * 1e-3) / 1e12
    gemm_tfs = v.pred_flop / (v.gemm_ms * 1e-3) / 1e12
    return {
        "metric": METRICS[a.workload],
        "value": v.value,
        "unit": "chain-steps/s",
        "n_gpus": v.world,
        "world_size_seen": v.world_seen,
        "steps": a.steps,
        "warmup": a.warmup,
        "clock_warm_ms": v.warm_ms,
        "ms_per_step": v.ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("the reference's %s files (tests/golden/%s.npz), whitened; features on device"
                 % (v.dataset, v.dataset)),
        "config": {"workload": v.wdesc, "Ntrain": v.N, "Ntest": v.Nte,
                   "D": v.D, "n_features": v.n, "r": v.r, "Q": v.Q, "minibatch": v.m,
                   "chains_per_gpu": v.C, "chains_alive_after_timed_steps": v.alive,
                   "epsw": a.epsw, "epsU": a.epsU,
                   "signal_var": a.signal_var, "parallelism": "chains%dx%d" % (v.C, v.world),
                   "engine": v.info["engine"], "workgroups_per_launch": v.info["workgroups"],
                   "threads_per_workgroup": v.info["threads"], "lds_bytes": v.info["lds_bytes"]},
        "roofline": dict(v.roof, **{
                     "traffic": v.traffic, "traffic_source": v.traffic_src,
                     "kernel": KERNELS[v.info["engine"]].replace("%d", str(v.r)),
                     "kernel_us": v.k_us,
                     "kernel_us_per_rank": v.k_us_ranks,
                     "kernel_us_note": KERNEL_US_NOTE % (a.steps, KERNEL_LAUNCHES[v.info["engine"]]),
                     "algorithmic_bytes_per_launch": v.bytes_launch,
                     "algorithmic_bytes_per_step": v.bytes_launch,
                     "steps_run_per_chain": v.steps_run}),
        "cpu_baseline": v.cpu,
        "test_rmse": v.quality["test_rmse"],
        "test_rmse_note": v.quality["note"],
        "quality": v.quality,
        "allreduce_ms": v.allreduce_ms,
        "timed_region_host_us": v.host_us,
        "pred": {"samples": v.npred, "Ntest": v.Nte, "ms": v.pred_ms, "gemm_flop": v.pred_flop,
                 "achieved_tflops": pred_tfs, "peak_tflops": FP64_MFMA_PEAK_TFS,
                 "frac": pred_tfs / FP64_MFMA_PEAK_TFS,
                 "kernels": "pred_temp_mfma_kernel (v_mfma_f64_16x16x4f64) + %s" % v.vphase_kernel,
                 "note": "whole stacked-sample call timed with events (GEMM + V-phase), median of 5 calls after 3 warm-up calls (the GEMM's clock settles over the first calls: 6.1, 5.6, 5.3 ms in profiles/r5ak_kernel_stats.csv's trace)",
                 "gemm_ms": v.gemm_ms, "vphase_ms": v.vphase_ms,
                 "gemm_roofline": {"bound": "mfma", "achieved": gemm_tfs,
                                   "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                                   "frac": gemm_tfs / FP64_MFMA_PEAK_TFS},
                 "final_state_ensemble_rmse": v.rmse_final},
        "single_chain": v.single,
        "single_chain_steps_per_s": v.single["steps_per_s"] if v.single else None,
    }


ML_CONFIG = dict(signal_var=0.8, sigma_u=0.1, sigma_w=1.0, m=100, epsw=1e-4, epsU=1e-6, a=0.5,
                 b=0.25, c=0.5, burnin=0, maxepoch=200, param_seed=17)


def movielens_bytes_per_step(ud, md, m, r):
    """Algorithmic HBM bytes of one GPT_fullw_sideinfo minibatch step (100k_movielensExperiment.jl
    :455-507; cf_epoch_kernel): the batch's (user, movie, rating) triples, the U / V rows and
    side-feature rows its sums read (mean feature count per user / movie), the gradient rows
    written (at most 2m + D1 + D2), and the dense move of every row of U and V (the prior term
    moves all rows: read M and G, write M and zero G)."""
    n1, D1 = ud.shape
    n2, D2 = md.shape
    fu, fv = float(ud.sum(axis=1).mean()), float(md.sum(axis=1).mean())
    gather = m * (4 + 4 + 8 + 4) + 8 * m * r * (2 + fu + fv)
    grads = 8 * r * (2 * m + D1 + D2)
    move = 4 * 8 * r * (n1 + D1 + n2 + D2)
    return gather + grads + move


def movielens_lazy_bytes_per_step(ud, md, m, r, nb):
    """HBM bytes per minibatch step of the lazy SGD path (cf_epoch_kernel domove = 2, one launch per
    epoch): the batch's triples and both feature masks, the batch's U / V rows read (the feature
    rows live in LDS for the launch), the touched rows' move (read + write), and the per-epoch
    flush of every row (read + write) and the feature rows' load / store, spread over the epoch's
    nb steps."""
    n1, D1 = ud.shape
    n2, D2 = md.shape
    gather = m * (4 + 4 + 8 + 8 + 8) + 8 * m * r * 2
    moved = 2 * 8 * r * 2 * m
    epoch = 2 * 8 * r * (n1 + D1 + n2 + D2) + 2 * 8 * r * (D1 + D2)
    return gather + moved + epoch / nb


def gibbs_flops_per_sweep(N, n1, n2, r):
    """fp64 flops of one GPT_fullw_gibbs sweep as cf.hip / tgp.hip run it: the user / movie
    conditionals (per rating the X row, 2r^2, and the precision update, 2r^2; per row an r x r
    Cholesky and two solves), the w | U, V statistics (2r^2 per rating), the precision GEMM
    Z = H^T P (2 p^2 n1, p = r^2), the right-hand side (2 p n1), the p x p Cholesky (p^3 / 3 FMAs)
    and three triangular solves (p^2 each)."""
    p = r * r
    rows = 2 * N * 4 * r * r + (n1 + n2) * (2 * r ** 3 / 3 + 4 * r * r)
    stats = 2 * N * r * r
    wsys = 2 * p * p * n1 + 2 * p * n1 + 2 * p ** 3 / 3 + 3 * 2 * p * p
    return rows + stats + wsys


def movielens_cpu_baseline(folds, w0, cfg, epochs=12):
    """The C++ fp64 restatement of GPT_fullw_sideinfo's SGD epochs (oracle/cpu/movielens_cpu.cpp,
    the reference's dense per-step move of every row; checked against oracle/movielens_ref.py by
    tests/test_oracle.py) on the same 5 folds, one OpenMP thread per fold, ``epochs`` epochs from
    the same starting state, each epoch's train / test evaluation included; plus one fold on one
    core for the per-core rate."""
    from oracle import cpu_lib
    from oracle import movielens_ref as M
    from oracle import philox as px
    r = np.asarray(w0).shape[0]
    ud, md = folds[0][2], folds[0][3]
    n1, D1 = ud.shape
    n2, D2 = md.shape
    U0 = M.init_uv(n1 + D1, r, cfg["param_seed"], 0, False, cfg["sigma_u"])
    V0 = M.init_uv(n2 + D2, r, cfg["param_seed"], 1, False, cfg["sigma_u"])
    N = folds[0][0].shape[0]
    perms = np.stack([px.randperm(N, cfg["param_seed"], e) for e in range(epochs)])
    args = (ud, md)
    hyper = (w0, U0, V0, cfg["signal_var"], cfg["sigma_u"], cfg["sigma_w"], cfg["m"], cfg["epsw"],
             cfg["epsU"], cfg["a"], cfg["b"], cfg["c"])
    nb = -(-N // cfg["m"])
    nf = len(folds)

    def leg(lazy, E):
        sec1, _ = cpu_lib.cf_sgd_folds([(folds[0][0], folds[0][1])], *args, [perms[:2]], *hyper,
                                       threads=1, lazy=lazy)
        sec, _ = cpu_lib.cf_sgd_folds([(f[0], f[1]) for f in folds], *args, [perms[:E]] * nf,
                                      *hyper, threads=nf, lazy=lazy)
        return nf * E * nb / sec, 2 * nb / sec1, sec, sec1
    # the GPU's algorithm (the lazy prior-decay move) is the fair baseline; the reference's dense
    # per-step move of every row beside it
    v, v1, sec, sec1 = leg(True, epochs)
    d, d1, dsec, dsec1 = leg(False, epochs)
    return dict(value=v, unit="fold-steps/s (%d folds on %d cores)" % (nf, nf),
                cores=nf, kind="port", single_core_steps_per_s=v1,
                sample="oracle/cpu/movielens_cpu.cpp run_fold_lazy (C++ fp64 restatement of "
                       "100k_movielensExperiment.jl:409-551, SGD, with the GPU's lazy prior-decay "
                       "move: rows outside a batch read as M*c^k, the same arithmetic regrouped) on "
                       "the %d folds, %d epochs = %d minibatch steps per fold plus each epoch's "
                       "train / test evaluation, one OpenMP thread per fold, in %.1f s; fold 1 alone "
                       "on 1 core for 2 epochs in %.2f s" % (nf, epochs, epochs * nb, sec, sec1),
                reference_dense_moves=dict(
                    value=d, unit="fold-steps/s (%d folds on %d cores)" % (nf, nf),
                    single_core_steps_per_s=d1,
                    sample="run_fold: the reference's dense per-step move of every U / V row "
                           "(:481-507), same folds and epochs, in %.1f s; fold 1 on 1 core for 2 "
                           "epochs in %.2f s" % (dsec, dsec1)))


def movielens_main(args):
    """bench.py --workload movielens: the live experiment of 100k_movielensExperiment.jl:723-739
    (GPT_fullw_sideinfo on the 5 ml-100k folds, SGD, σ_u = 0.1, σ² = 0.8, εU = 1e-6, εw = 1e-4,
    a, b, c = 0.5, 0.25, 0.5, m = 100, 200 epochs, param_seed 17) at BASELINE config 5's r = 20
    (the script runs r = 15; --r).  The folds run as sibling chains of one cf_epoch_kernel launch
    per epoch (gpt_cf_fullw_sideinfo_folds); value = minibatch steps summed over the folds / wall
    time of the whole call (host evaluation, stores and early stop included); roofline from the
    device time of each epoch's launches (hipEvents inside the library, gpt_cf_last_timing).  N > 1:
    every rank runs the experiment with its own param_seed (replicas, no collective)."""
    import torch
    import torch.distributed as dist
    from gpt_amd import movielens
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    cfg = dict(ML_CONFIG)
    r = args.r if args.r is not None else 20
    epochs = args.epochs
    cfg["param_seed"] += rank
    d = np.load(os.path.join(ROOT, "tests", "golden", "ml100k.npz"))
    folds = [movielens.fold(d, i) for i in range(1, 6)]
    trs, tes = [f[0] for f in folds], [f[1] for f in folds]
    ud, md = folds[0][2], folds[0][3]
    mus, sds = [f[4] for f in folds], [f[5] for f in folds]
    w0 = cfg["sigma_w"] * np.random.default_rng(cfg["param_seed"]).standard_normal((r, r))

    def run(E):
        return movielens.GPT_fullw_sideinfo_folds(
            trs, ud, md, tes, cfg["signal_var"], cfg["sigma_u"], cfg["sigma_w"], w0, cfg["m"],
            cfg["epsw"], cfg["epsU"], cfg["a"], cfg["b"], cfg["c"], cfg["burnin"], E,
            cfg["param_seed"], mus, sds)

    run(max(1, args.warmup_epochs))                  # warm-up: kernels loaded, clocks up
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = run(epochs)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    tm = movielens.last_timing()
    dt = max_over_ranks(wall, dev)
    steps_all = gather_over_ranks(float(tm["fold_steps"]), dev)
    value = sum(steps_all) / dt
    mins = [float(o[5].min()) for o in outs]
    nbat = -(-trs[0].shape[0] // cfg["m"])
    bdense = movielens_bytes_per_step(ud, md, cfg["m"], r)
    lazy = tm.get("mode", 0) == 2
    bstep = movielens_lazy_bytes_per_step(ud, md, cfg["m"], r, nbat) if lazy else bdense
    ep_us = 1e3 * tm["epoch_ms"] / max(tm["epochs"], 1)
    steps_per_launch = tm["fold_steps"] / max(tm["epochs"], 1)
    achieved = bstep * steps_per_launch / (ep_us * 1e-6) / 1e9
    # config 5's other sampler (BASELINE: "full-W Gibbs vs SGLD"): GPT_fullw_gibbs on fold 1 with
    # the parameter line of :743-752 (signal_var = σ_u = 0.5, σ_w = ‖w_init‖_F / r, burnin 15,
    # avg = true, param_seed 10) at r = 20, timed on the wall clock (whole sweeps, host
    # bookkeeping included), with the running-average test RMSE beside fullWresults.h5's (r = 15)
    gibbs = None
    if rank == 0:
        tr1, te1, ud1, md1, mu1, sd1 = folds[0]
        wg = np.random.default_rng(10).standard_normal((r, r))
        sw_g = math.sqrt((wg ** 2).sum()) / r
        gsweeps = args.gibbs_sweeps
        movielens.GPT_fullw_gibbs(tr1, ud1, md1, te1, 0.5, 0.5, sw_g, wg, 1, 2, 1, 10, mu1, sd1,
                                  avg=True)                       # warm-up
        tg = time.perf_counter()
        go = movielens.GPT_fullw_gibbs(tr1, ud1, md1, te1, 0.5, 0.5, sw_g, wg, 15, gsweeps, 1, 10,
                                       mu1, sd1, avg=True)
        dtg = time.perf_counter() - tg
        refg = np.load(os.path.join(ROOT, "tests", "golden", "ref_curves.npz"))["fullW_testRMSE"]
        curve = np.asarray(go[5])
        gibbs = {"sampler": "GPT_fullw_gibbs (100k_movielensExperiment.jl:1032-1129), fold 1, r=%d" % r,
                 "sweeps": 15 + gsweeps, "seconds": dtg, "sweeps_per_s": (15 + gsweeps) / dtg,
                 "ms_per_sweep": 1e3 * dtg / (15 + gsweeps),
                 "roofline": {"bound": "mfma", "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                              "flops_per_sweep": gibbs_flops_per_sweep(tr1.shape[0], ud1.shape[0],
                                                                       md1.shape[0], r),
                              "kernel": "whole sweep (chol_blk_kernel, cfg_rows_kernel x 3, "
                                        "cfg_wprec_kernel, trsv_blk_kernel x 3, ...)",
                              "note": "latency-bound: the 400 x 400 Cholesky's 25 serial panels "
                                      "are 0.50 of 1.35 ms of kernels per sweep "
                                      "(profiles/r5r_gibbs_kernel_stats.csv)"},
                 "test_rmse_running_avg_final": float(curve[-1]),
                 "test_rmse_running_avg_min": float(curve.min()),
                 "reference_fullWresults_h5_r15": {"at_same_sweep": float(refg[min(gsweeps, len(refg)) - 1]),
                                                    "final_1000": float(refg[-1]), "min": float(refg.min())}}
        gr = gibbs["roofline"]
        gr["achieved"] = gr["flops_per_sweep"] / (1e-3 * gibbs["ms_per_sweep"]) / 1e12
        gr["frac"] = gr["achieved"] / gr["peak"]
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = movielens_cpu_baseline(folds, w0, cfg)
    if rank == 0:
        nb = -(-trs[0].shape[0] // cfg["m"])
        out = {
            "metric": "GPT_fullw_sideinfo minibatch steps/sec + test RMSE (100k_movielensExperiment.jl, "
                      "5 folds, r=%d)" % r,
            "value": value, "unit": "fold-steps/s", "n_gpus": world, "steps": int(tm["fold_steps"]),
            "warmup": int(max(1, args.warmup_epochs)) * nb * len(folds),
            "ms_per_step": 1e3 * dt / max(1, tm["fold_steps"] / len(folds)),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "ml-100k u1..u5 base/test + u.user / u.item side information "
                    "(tests/golden/ml100k.npz), ratings standardised per fold",
            "config": {"workload": "GPT_fullw_sideinfo, 5 folds as sibling chains (SGD: "
                                   "langevin = stiefel = false, :733-736)",
                       "r": r, "epochs": epochs, "folds": len(folds), "Ntrain": int(trs[0].shape[0]),
                       "Ntest": int(tes[0].shape[0]), "users": int(ud.shape[0]), "movies": int(md.shape[0]),
                       "D1": int(ud.shape[1]), "D2": int(md.shape[1]), **cfg,
                       "parallelism": "folds%dx%d" % (len(folds), world)},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": ("cf_gather_kernel + cf_epoch_kernel<%d, lazy move> (one launch "
                                    "per epoch: %d minibatch steps per fold workgroup)" % (r, nb))
                                   if lazy else
                                   ("cf_gather_kernel + %d x (cf_epoch_kernel<%d> batch phase + "
                                    "cf_move_kernel<%d>)" % (nb, r, r)),
                         "kernel_us": ep_us, "kernel_us_note": "per epoch of every live fold's %d "
                         "minibatch steps, hipEvents inside gpt_cf_fullw_sideinfo_folds around the "
                         "epoch's launches (%s)" % (nb, "one epoch launch, one workgroup per fold, "
                         "the lazy SGD move: rows outside a batch only decay and are read as m*c^k"
                         if lazy else "one batch-phase launch, one workgroup per fold, and one "
                         "row-parallel move launch per step"),
                         "launch_mode": int(tm.get("mode", 0)),
                         "survey_8d_bytes_per_step": bdense,
                         "survey_8d_note": "the reference's dense per-step move of every U / V row "
                                           "(read M, G; write M, G) priced in",
                         "eval_kernel_us": 1e3 * tm["eval_ms"] / max(tm["epochs"], 1),
                         "algorithmic_bytes_per_step": bstep,
                         "algorithmic_bytes_per_launch": bstep * steps_per_launch,
                         "device_fraction_of_wall": (tm["epoch_ms"] + tm["eval_ms"]) / (1e3 * wall)},
            "cpu_baseline": cpu,
            "test_rmse": float(np.mean(mins)),
            "test_rmse_note": "meantestRMSE of :735-737: mean over the folds of each fold's minimum "
                              "per-epoch test RMSE (rating units, predictions cut off to [1, 5])",
            "gibbs": gibbs,
            "quality": {"min_test_rmse_per_fold": mins,
                        "epochs_run_per_fold": [int((o[4] > 0).sum()) for o in outs],
                        "final_train_rmse_per_fold": [float(o[4][o[4] > 0][-1]) if (o[4] > 0).any()
                                                      else None for o in outs]},
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def gather_over_ranks(x, device=None):
    """[x of rank 0, .., x of rank N-1] (every rank gets the list)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [x]
    t = torch.tensor([x], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--chains", type=int, default=0,
                    help="independent chains per GPU (0: one per CU for the chain engine, two at "
                         "D <= 4; CUs // (D+1) for the grid engine, D+1 workgroups per chain)")
    ap.add_argument("--engine", default="auto", choices=["auto", "grid", "chain", "wave"])
    ap.add_argument("--workload", default="kin40k", choices=sorted(WORKLOADS) + ["movielens"],
                    help="kin40k (BASELINE configs 3/4, the metric's workload), kin40k_ref "
                         "(kin40kExperiment.jl's n=150, r=20), powerplant (config 2) or movielens "
                         "(config 5: GPT_fullw_sideinfo over the 5 ml-100k folds)")
    ap.add_argument("--warmup-epochs", type=int, default=2, help="movielens: warm-up call's epochs")
    ap.add_argument("--gibbs-sweeps", type=int, default=200,
                    help="movielens: kept sweeps of the full-W Gibbs leg (after 15 burn-in)")
    ap.add_argument("--n", type=int, default=None, help="default: the workload's (500 / 150)")
    ap.add_argument("--D", type=int, default=None, help="default: the workload's D (8 / 4)")
    ap.add_argument("--r", type=int, default=None, help="default: the workload's (5 / 20)")
    ap.add_argument("--Q", type=int, default=200)
    ap.add_argument("--m", type=int, default=None, help="minibatch (default: 50 / 256)")
    # kin40kExperiment.jl:50-51 uses εw=1e-4, εU=1e-7 at n=150, r=20; under the restated
    # GPT_SGLD.jl update both the oracle and the GPU path diverge there (w Hessian λmax≈3e5),
    # so the benchmark uses the largest stable pair found by the oracle sweep.
    ap.add_argument("--epsw", type=float, default=None, help="default: the workload's")
    ap.add_argument("--epsU", type=float, default=None, help="default: the workload's")
    ap.add_argument("--signal_var", type=float, default=None, help="default: the workload's")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--clock-warm-ms", type=float, default=1000.0,
                    help="untimed GPU clock warm-up on a scratch session before the warmup steps")
    ap.add_argument("--epochs", type=int, default=200,
                    help="epochs every chain runs in total (kin40kExperiment.jl:74: maxepoch 200); "
                         "the steps after the timed region finish them for the converged test RMSE")
    ap.add_argument("--last-epochs", type=int, default=50,
                    help="epoch-end samples per chain in the posterior mean (kin40kExperiment.jl:80-87)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-single-chain", dest="single_chain", action="store_false",
                    help="skip the C=1 latency pass (one chain on one CU)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: re-run under torchrun before any HIP call in this process
        raise SystemExit(self_launch(sys.argv[1:], args.gpus))
    if args.workload == "movielens":
        return movielens_main(args)
    loader, wD, wm, wls, sigma_rbf, wsv, wdesc, wn, wr, wew, weu = WORKLOADS[args.workload]
    for k_, v_ in (("n", wn), ("r", wr), ("epsw", wew), ("epsU", weu)):
        if getattr(args, k_) is None:
            setattr(args, k_, v_)
    if args.D is None:
        args.D = wD
    if args.m is None:
        args.m = wm
    if args.signal_var is None:
        args.signal_var = wsv

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import SGLDSession, feature_device, pred_device

    n, D, r, Q, m = args.n, args.D, args.r, args.Q, args.m
    Xtr, ytr, Xte, yte, ysd = loader(D)
    N, Nte = Xtr.shape[0], Xte.shape[0]
    ls = np.array(wls)[:D]
    scale = math.sqrt(n / Q ** (1.0 / D))                 # kin40kExperiment.jl:45
    I = G.samplenz(r, D, Q, 17)                           # :44 (seed 17)
    Z, b = G.feature_inputs(n, D, 17)                     # Gen-C seeded feature inputs
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    phi_tr = feature_device(tt(Xtr.T), tt(ls), sigma_rbf, scale, tt(Z.T), tt(b.T))
    phi_te = feature_device(tt(Xte.T), tt(ls), sigma_rbf, scale, tt(Z.T), tt(b.T))
    y_tr = tt(ytr)
    torch.cuda.synchronize()

    nb = -(-N // m)
    C = args.chains
    if C <= 0:
        # filling the GPU: the chain engine whenever it takes the shape (one chain's session
        # would pick the grid engine, the single-chain latency choice); past r = 5 the wave engine
        # (one chain per CU: 256 chains = 2048 dimension waves, two per SIMD)
        eng = "grid"
        if args.engine == "wave" or (args.engine == "auto" and r > 5):
            eng = "wave"
        elif args.engine in ("auto", "chain"):
            from gpt_amd._lib import GPTError
            try:
                probe = SGLDSession(phi_tr, y_tr, I, r, Q, m, args.epsw, args.epsU,
                                    args.signal_var, 0, 1, [1], store=False, engine="chain")
                eng = "chain"
                probe.close()
            except GPTError:
                if args.engine == "chain":
                    raise
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        # chain engine: one chain per CU, two at D <= 4 (4-wave build, 80 KB of LDS);
        # grid engine: D+1 workgroups per chain
        C = ((cus * (2 if D <= 4 else 1)) if eng == "chain"
             else (cus if eng == "wave" else max(1, cus // (D + 1))))
    need = args.warmup + args.steps
    epochs = -(-need // nb) + 1
    epochs_total = max(args.epochs, epochs)
    last = max(1, min(args.last_epochs, epochs_total))
    seeds = chain_seeds(rank, C)
    # burn-in = all but the last `last` epochs: the timed steps store nothing, the epoch-end
    # samples of the last epochs feed the converged posterior mean.  The session runs on a torch
    # stream of ours, so hipEvents recorded on it bracket exactly the timed steps' launches
    tstream = torch.cuda.Stream(device=dev)
    sess = SGLDSession(phi_tr, y_tr, I, r, Q, m, args.epsw, args.epsU, args.signal_var,
                       epochs_total - last, last, seeds, store_every=nb, store=True,
                       engine=args.engine, stream=tstream.cuda_stream)
    info = sess.info()
    sess.run(args.warmup)
    sess.prepare(args.steps)           # capture the timed steps' graphs outside the timed region
    sess.sync()
    warm_ms = 0.0
    warm_steps = 0                     # chain steps of the scratch session (profile accounting)
    sw = None
    if args.clock_warm_ms > 0:
        # Bring the GPU to its sustained clock right before the timed region.  The chain kernel's
        # cycles per step are fixed (≈216 k); its time per step follows the shader clock, which
        # drops during any idle gap of a millisecond or more (host work, frees) and takes
        # milliseconds to ramp back (scripts/timeline.py: 2.09 GHz after a gap, 2.33-2.39 GHz
        # under sustained load).  The driver's 20 timed steps are ~2 ms, so without this they
        # would measure the ramp.  A scratch session of the same shape and chain count runs the
        # same work (the timed chains' state is untouched) and stays allocated until the timed
        # region is over, so no free (a device synchronisation) sits between it and the timing.
        ep_warm = 2 + int(args.clock_warm_ms / 15.0)
        sw = SGLDSession(phi_tr, y_tr, I, r, Q, m, args.epsw, args.epsU, args.signal_var, 0,
                         ep_warm, scratch_seeds(rank, C), store=False, engine=args.engine)
        tw = time.perf_counter()
        while ((time.perf_counter() - tw) * 1000.0 < args.clock_warm_ms
               and sw.steps_done < sw.total_steps):
            ns = min(nb, sw.total_steps - sw.steps_done)
            sw.run(ns)
            sw.sync()
            warm_steps += ns
        warm_ms = (time.perf_counter() - tw) * 1000.0
    # a marker dispatch before and after the timed region (outside it), so a kernel trace of this
    # command isolates the timed steps' dispatches (scripts/prof_timed.py)
    profile_marker(tstream)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    pc = time.perf_counter
    t0 = pc()
    ev0.record(tstream)
    t1 = pc()
    sess.run(args.steps)
    t2 = pc()
    ev1.record(tstream)
    t3 = pc()
    # one device synchronisation closes the region: the session runs on tstream, which it drains
    # (a separate hipStreamSynchronize first measured 3-83 µs more, scripts/host_overhead.py)
    t4 = pc()
    torch.cuda.synchronize()
    t5 = pc()
    if world > 1:
        dist.barrier()
    dt_rank = pc() - t0
    host_us = {"ev0_record": 1e6 * (t1 - t0), "run_call": 1e6 * (t2 - t1),
               "ev1_record": 1e6 * (t3 - t2), "device_sync": 1e6 * (t5 - t4)}
    profile_marker(tstream)
    # device time of the timed steps on the session stream (the graph launches of the timed
    # region, gaps between their kernels included): <= the wall time above by construction
    k_us = 1000.0 * ev0.elapsed_time(ev1) / args.steps
    host_us["wall_minus_event_total"] = 1e6 * dt_rank - 1000.0 * ev0.elapsed_time(ev1)
    # chains that hit the geodesic NaN bail-out (GPT_SGLD.jl:422-424) stop stepping; at the
    # reference's own kin40k configuration (εw = 1e-4, εU = 1e-7) about one chain in eight does,
    # as in the reference, and PowerPlant's εw = 5e-5 / εU = 2e-8 loses a few of 512.  Only the
    # chains still alive after the timed steps are counted (a chain that bailed inside the timed
    # region did part of its steps: not counted, conservative).
    bad = [c for c in range(C) if sess.status(c) != 0]
    alive = C - len(bad)
    if alive == 0:
        raise SystemExit("chains %s hit the geodesic NaN bail-out: the timed steps were no-ops" % bad)
    dt = max_over_ranks(dt_rank, dev)
    total_steps = sum(gather_over_ranks(float(alive * args.steps), dev))
    value = total_steps / dt
    ms_per_step = 1000.0 * dt / args.steps

    if sw is not None:
        sw.close()
    k_us_ranks = gather_over_ranks(k_us, dev)
    B = m
    bytes_launch = alive * algorithmic_bytes_per_step(n, D, B, r, Q)
    achieved = bytes_launch / (k_us * 1e-6) / 1e9
    if info["engine"] == "wave":
        # r = 20: fp64-compute bound.  Primary figure: the flops the engine executes at the Padé
        # degree these runs take; §8(d)'s count (which prices geod's two expm at 30 (2r)³
        # products each) beside it
        fl = alive * algorithmic_flops_per_step(n, D, B, r, Q)
        ex = alive * executed_flops_per_step(n, D, B, r, Q)
        tf = ex / (k_us * 1e-6) / 1e12
        roof = {"bound": "fp64", "achieved": tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": tf / FP64_PEAK_TFLOPS, "flops_per_step": ex,
                "flops_basis": "executed (Padé degree 5 / 3, r right-hand sides; "
                               "bench.executed_flops_per_step)",
                "survey_8d_flops_per_step": fl,
                "survey_8d_frac": fl / (k_us * 1e-6) / 1e12 / FP64_PEAK_TFLOPS,
                "survey_8d_note": "SURVEY §8(d) count, pricing each expm at 30 (2r)^3 products",
                "hbm_achieved_GBs": achieved, "hbm_frac": achieved / HBM_PEAK_GBS}
    else:
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS}
    # HBM traffic per launch is a PMC quantity (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, gfx950
    # FETCH doubling): it cannot be read inside this run, so it comes from the stored profile of
    # the same shape, with its tag (scripts/pmc_chain.sh -> profiles/pmc_traffic.json)
    traffic, traffic_src = None, None
    if os.path.exists(args.pmc):
        try:
            pm = json.load(open(args.pmc))
            key = "C%d_n%d_D%d_r%d_Q%d_m%d" % (C, n, D, r, Q, m)
            ent = pm.get(key, {})
            traffic = ent.get("hbm_bytes_per_launch")
            if traffic is not None:
                traffic_src = "stored PMC profile %s[%s] (%s)" % (
                    os.path.relpath(args.pmc, ROOT), key, ent.get("source", "untagged"))
        except Exception:
            traffic = None

    # ---- quality leg (the metric's "+ test RMSE"): every chain finishes its epochs_total epochs
    # (kin40kExperiment.jl:74) and the ensemble prediction is the mean over every chain's last
    # `last` epoch-end samples (:80-87), all-reduced over ranks (RCCL, config 4)
    from gpt_amd.ensemble import combine_predictive_mean, rmse as ens_rmse
    I0 = torch.from_numpy(np.asfortranarray(I - 1).ravel(order="F").astype(np.int32)).to(dev)
    tq = time.perf_counter()
    sess.run(sess.total_steps)
    sess.sync()
    quality_train_s = time.perf_counter() - tq
    status = [sess.status(c) for c in range(C)]
    fsum_q = torch.zeros(Nte, dtype=torch.float64, device=dev)
    cnt = 0
    fhq = torch.empty((last, Nte), dtype=torch.float64, device=dev)
    yte_d = torch.from_numpy(np.ascontiguousarray(yte)).to(dev)
    finals, curve_means = [], []
    for c in range(C):
        if status[c] != 0:
            continue
        _, _, ws, Us, ns = sess.device_state(c)
        pred_device(ws, Us, I0, phi_te, n, D, Nte, r, Q, ns, fhq)
        fsum_q += fhq[:ns].sum(dim=0)
        cnt += ns
        # this chain's per-epoch test-RMSE curve over its last epochs (kin40kExperiment.jl:83)
        err = fhq[:ns] - yte_d[None, :]
        curve = (ysd * torch.sqrt((err * err).mean(dim=1))).cpu().numpy()
        finals.append(float(curve[-1]))
        curve_means.append(float(curve.mean()))
    torch.cuda.synchronize()
    fmean_q = combine_predictive_mean(fsum_q, cnt)
    rmse_conv = ens_rmse(yte, fmean_q.cpu().numpy(), ysd)
    quality = {"test_rmse": rmse_conv, "epochs": epochs_total, "samples_per_chain": last,
               "chains": C * world, "bailed_out": int(sum(1 for x in status if x != 0)),
               "train_s": quality_train_s,
               "chain_final_rmse_median": float(np.median(finals)) if finals else None,
               "chain_curve_mean_median": float(np.median(curve_means)) if curve_means else None,
               "note": "RMSE (original units, ytrainStd x) of the mean prediction over the last %d "
                       "epoch-end samples of every chain after %d epochs (kin40kExperiment.jl:74-87); "
                       "chain_final_rmse_median / chain_curve_mean_median: the median chain's "
                       "epoch-%d test RMSE and its curve's mean over the last %d epochs (rank 0's "
                       "chains)" % (last, epochs_total, epochs_total, last)}
    if args.workload == "kin40k_ref":
        ref = np.load(os.path.join(ROOT, "tests", "golden", "ref_curves.npz"))["testRMSE_kin40k"]
        quality["reference"] = {"file": "testRMSE_kin40k.h5 (tests/golden/ref_curves.npz)",
                                "final": float(ref[-1]), "last50_curve_mean": float(ref[-50:].mean())}

    # posterior predictive over every chain's final state as ONE stacked-sample prediction
    # (fp64-MFMA phidotU GEMM with M = S·r, N = Ntest, K = n per dimension, then the V-phase)
    w_all = torch.empty((C, Q), dtype=torch.float64, device=dev)
    U_all = torch.empty((C, n * r * D), dtype=torch.float64, device=dev)
    sess.gather_state(0, C, w_all, U_all)
    sess.sync()
    live = [c for c in range(C) if status[c] == 0]      # a bailed-out chain's state is undefined
    if len(live) < C:
        li = torch.tensor(live, dtype=torch.long, device=dev)
        w_all, U_all = w_all[li].contiguous(), U_all[li].contiguous()
    npred = len(live)
    fh = torch.empty((npred, Nte), dtype=torch.float64, device=dev)
    for _ in range(3):                                # warm-up: pool, kernels, the clock under MFMA load
        pred_device(w_all.data_ptr(), U_all.data_ptr(), I0, phi_te, n, D, Nte, r, Q, npred, fh)
    torch.cuda.synchronize()
    pred_times = []                                   # the median of five steady-state calls
    for _ in range(5):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        pred_device(w_all.data_ptr(), U_all.data_ptr(), I0, phi_te, n, D, Nte, r, Q, npred, fh)
        ev1.record()
        torch.cuda.synchronize()
        pred_times.append(ev0.elapsed_time(ev1))
    pred_ms = sorted(pred_times)[2]
    pred_flop = 2.0 * npred * r * n * D * Nte             # the GEMM (dominant); V-phase excluded
    from gpt_amd.session import pred_device_timed, pred_last_vphase
    vphase_kernel = pred_last_vphase()               # the kernel the calls above launched
    gemm_ms, vphase_ms = pred_device_timed(w_all.data_ptr(), U_all.data_ptr(), I0, phi_te, n, D,
                                           Nte, r, Q, npred, fh)
    fsum = fh.sum(dim=0)
    combine_predictive_mean(torch.zeros_like(fsum), 1)   # warm-up (communicator setup, kernels)
    torch.cuda.synchronize()
    ta = time.perf_counter()
    fmean = combine_predictive_mean(fsum, npred)     # RCCL all-reduce across ranks (config 4)
    torch.cuda.synchronize()
    allreduce_ms = 1000.0 * (time.perf_counter() - ta)
    rmse_final = ens_rmse(yte, fmean.cpu().numpy(), ysd)

    single = None
    if args.single_chain and rank == 0:
        s1st = torch.cuda.Stream(device=dev)
        s1 = SGLDSession(phi_tr, y_tr, I, r, Q, m, args.epsw, args.epsU, args.signal_var, 0,
                         epochs, [7], store_every=nb, store=False, engine=args.engine,
                         stream=s1st.cuda_stream)
        s1.run(args.warmup)
        s1.prepare(args.steps)
        s1.sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t1 = time.perf_counter(); e0.record(s1st); s1.run(args.steps); e1.record(s1st); s1.sync()
        sps = args.steps / (time.perf_counter() - t1)
        s1_us = 1000.0 * e0.elapsed_time(e1) / args.steps
        b1 = algorithmic_bytes_per_step(n, D, m, r, Q)
        single = {"steps_per_s": sps, "engine": s1.info()["engine"], "kernel_us": s1_us,
                  "roofline_frac": (b1 / (s1_us * 1e-6) / 1e9 / HBM_PEAK_GBS) if s1_us else None}
        s1.close()

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:          # host cores of rank 0's box, any N
        phi_np = np.asfortranarray(phi_tr.cpu().numpy().transpose(2, 1, 0))
        cpu = cpu_baseline(phi_np, ytr, I, args, args.cpu_seconds)
        if cpu is not None and "single_core_steps_per_s" in cpu:      # the C++ restatement ran
            cpu["pred"] = cpu_pred_baseline(phi_te, w_all, U_all, fh, I, n, D, r, args.cpu_seconds)
            cpu["minibatch_256"] = cpu_b256_baseline(phi_np, ytr, I, args, args.cpu_seconds)

    if rank == 0:
        import types
        world_seen = dist.get_world_size() if world > 1 else 1
        steps_run = sess.total_steps + warm_steps
        out = compose_line(types.SimpleNamespace(
            args=args, value=value, world=world, world_seen=world_seen, warm_ms=warm_ms,
            ms_per_step=ms_per_step, wdesc=wdesc, N=N, Nte=Nte, D=D, n=n, r=r, Q=Q, m=m, C=C,
            info=info, roof=roof, alive=alive, traffic=traffic, traffic_src=traffic_src, k_us=k_us,
            dataset=loader.__name__,
            k_us_ranks=k_us_ranks, bytes_launch=bytes_launch, steps_run=steps_run, cpu=cpu,
            quality=quality, allreduce_ms=allreduce_ms, npred=npred, pred_ms=pred_ms,
            pred_flop=pred_flop, gemm_ms=gemm_ms, vphase_ms=vphase_ms, rmse_final=rmse_final,
            vphase_kernel=vphase_kernel, host_us=host_us,
            single=single))
        print(json.dumps(out))
    sess.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
