"""Reproduce / rule out the host SIGSEGV of round 4 (VERDICT r4 "What's weak" #1): a 256-chain
wave-engine session at kin40k_ref's shape (n = 150, r = 20, εw = 1e-4, εU = 1e-7, epoch-end
samples stored) whose whole 200-epoch run is ONE gpt_sgld_session_run call — bench.py's quality
leg — meant to be run under `rocprofv3 --kernel-trace --stats`.

A background thread copies /proc/self/maps to --maps every 0.25 s while the main thread sits in
the run() call (ctypes releases the GIL), so the addresses of a crash's stack trace (printed by
the profiler's failure handler) can be resolved to libraries and offsets afterwards
(scripts/symbolize_trace.py).  GPTSGLD_MAX_INFLIGHT selects how many epoch chunks the session
lets into the stream at once (0 = unbounded, the round-4 behaviour).

    rocprofv3 --kernel-trace --stats -d gpurun_out/x -o x -- \
        python -u scripts/refprof_repro.py --maps gpurun_out/maps.txt
"""
import argparse
import math
import os
import shutil
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=200)
    ap.add_argument("--chains", type=int, default=256)
    ap.add_argument("--maps", default=os.path.join(ROOT, "gpurun_out", "repro_maps.txt"))
    args = ap.parse_args()

    import torch
    import bench
    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import SGLDSession, feature_device

    n, D, r, Q, m = 150, 8, 20, 200, 50
    Xtr, ytr, _, _, _ = bench.kin40k(D)
    ls = np.array(bench.KIN40K_LS)
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    phi = feature_device(tt(Xtr.T), tt(ls), 1.0420, math.sqrt(n / Q ** (1.0 / D)), tt(Z.T), tt(b.T))
    y = tt(ytr)
    nb = -(-ytr.size // m)
    last = min(50, args.epochs)
    sess = SGLDSession(phi, y, I, r, Q, m, 1e-4, 1e-7, 0.0476, args.epochs - last, last,
                       list(range(1, args.chains + 1)), store_every=nb, store=True, engine="wave")
    sess.run(nb)                                  # first epoch: every library is loaded now
    sess.sync()

    stop = threading.Event()
    tmp = args.maps + ".tmp"

    def dump():
        while not stop.is_set():
            try:
                shutil.copyfile("/proc/self/maps", tmp)
                os.replace(tmp, args.maps)
            except OSError:
                pass
            stop.wait(0.25)

    th = threading.Thread(target=dump, daemon=True)
    th.start()
    t0 = time.perf_counter()
    print("run: %d steps in one call, GPTSGLD_MAX_INFLIGHT=%s" %
          (sess.total_steps - sess.steps_done, os.environ.get("GPTSGLD_MAX_INFLIGHT", "default")),
          flush=True)
    sess.run(sess.total_steps)
    t1 = time.perf_counter()
    sess.sync()
    t2 = time.perf_counter()
    stop.set()
    th.join()
    alive = sum(1 for c in range(args.chains) if sess.status(c) == 0)
    print("enqueue %.2f s, drain %.2f s, %d of %d chains alive" % (t1 - t0, t2 - t1, alive,
                                                                 args.chains), flush=True)
    sess.close()


if __name__ == "__main__":
    main()
