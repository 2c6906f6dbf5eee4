"""Host time around the driver's timed region (bench.py --steps 20): wall clock minus the hipEvent
span of the same 20-step launch, for variants of the region's host calls (diagnostic).

    python scripts/host_overhead.py [--reps 12] [--out FILE]

bench  : t0; ev0.record; sess.run(20) [prepared graph]; ev1.record; sess.sync(); torch.cuda.synchronize()
nosync : the same without sess.sync() (torch.cuda.synchronize() drains the session stream too)
direct : sess.run(20) without a prepared graph (direct kernel launches)
spin   : the session stream polled (hipStreamQuery) instead of hipStreamSynchronize
noev   : no events: sess.run(20); torch.cuda.synchronize() (wall only)
Each rep runs the variants in turn on the bench's 256-chain kin40k session, with 40 ms of steps
between reps to hold the clock.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--out", default=None)
    ap.add_argument("--spin-flags", action="store_true",
                    help="hipSetDeviceFlags(hipDeviceScheduleSpin) after torch's device init")
    args = ap.parse_args()
    import torch
    import bench
    from gpt_amd import GPT_SGLD as G
    from gpt_amd.session import SGLDSession, feature_device
    dev = torch.device("cuda", 0)
    n, D, r, Q, m = 500, 8, 5, 200, 50
    Xtr, ytr, _, _, _ = bench.kin40k(D)
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    phi = feature_device(tt(Xtr.T), tt(np.array(bench.KIN40K_LS)), 1.042,
                         math.sqrt(n / Q ** (1 / D)), tt(Z.T), tt(b.T))
    y = tt(ytr)
    if args.spin_flags:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(1), flush=True)
    tstream = torch.cuda.Stream(device=dev)
    sess = SGLDSession(phi, y, I, r, Q, m, 1e-5, 1e-8, 0.0476, 0, 200, list(range(1, 257)),
                       store=False, engine="chain", stream=tstream.cuda_stream)
    sw = SGLDSession(phi, y, I, r, Q, m, 1e-5, 1e-8, 0.0476, 0, 200, [10 ** 6 + c for c in range(256)],
                     store=False, engine="chain")
    nb = 200

    def warm(ms):
        t = time.perf_counter()
        while (time.perf_counter() - t) * 1e3 < ms:
            sw.run(nb)
            sw.sync()

    def region(kind):
        # keep the 20 steps inside one epoch (one launch), as the driver's steps 5-24
        pos = sess.steps_done % nb
        if pos + 20 > nb or pos < 5:
            sess.run((nb - pos) % nb + 5)
            sess.sync()
        if kind != "direct":
            sess.prepare(20)
        sess.sync()
        warm(40)
        bench.profile_marker(tstream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        if kind == "noev":
            sess.run(20)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e6, None
        e0.record(tstream)
        sess.run(20)
        e1.record(tstream)
        if kind == "spin":
            while not tstream.query():
                pass
        elif kind != "nosync":
            sess.sync()
        t4 = time.perf_counter()
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        wall = (t5 - t0) * 1e6
        devsync[kind].append((t5 - t4) * 1e6)
        return wall, 1e3 * e0.elapsed_time(e1)

    warm(300)
    kinds = ["bench", "nosync", "spin", "direct", "noev"]
    devsync = {k: [] for k in kinds}
    res = {k: [] for k in kinds}
    for _ in range(args.reps):
        for k in kinds:
            res[k].append(region(k))
    out = {}
    for k in kinds:
        walls = np.array([w for w, _ in res[k]])
        evs = np.array([e for _, e in res[k] if e is not None])
        out[k] = dict(walls=[round(float(x), 1) for x in walls],
                      device_sync_us=[round(float(x), 1) for x in devsync[k]],
                      hosts=[round(float(w - e), 1) for w, e in res[k] if e is not None],
                      wall_us_median=float(np.median(walls)), wall_us_min=float(walls.min()),
                      event_us_median=float(np.median(evs)) if evs.size else None,
                      host_us_median=float(np.median(walls - evs)) if evs.size else None,
                      host_us_min=float((walls - evs).min()) if evs.size else None)
        print(k, json.dumps(out[k]), flush=True)
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)
    sess.close()
    sw.close()


if __name__ == "__main__":
    main()
