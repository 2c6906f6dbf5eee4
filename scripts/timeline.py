"""Per-step timeline of every chain-engine workgroup (diagnostic library libgptsgld_tl.so,
`make -C gpt_amd/csrc timeline`): where a launch's time goes beyond steps x per-step time.

    GPTSGLD_LIB=gpt_amd/libgptsgld_tl.so python scripts/timeline.py [--out FILE]

Runs the bench's kin40k workload (256 chains, n = 500, D = 8, r = 5, m = 50) in the bench's
order (clock warm-up, 5 warm-up steps, then the 20 steps the driver times), recording for every
workgroup s_memrealtime (100 MHz) and s_memtime (shader clock) at entry, prologue end and the
end of each step, plus HW_ID / XCC_ID.  The same is then recorded for launches later in the run
(after an idle gap, late in the epoch, 100-step and epoch-long launches).  Per launch it reports
dispatch skew, prologue time, per-step time (mean and max over chains), the tail (last chain's
end - median chain's end), the shader clock, and the event time of the launch.
"""
import argparse
import ctypes as C
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

RT_HZ = 100e6          # s_memrealtime: the 100 MHz constant clock


def analyse(tl, nsteps, ev_us, tag):
    C_, S = tl.shape[0], tl.shape[1]
    rt = tl[:, 0:2 * (nsteps + 2):2].astype(np.float64)        # (chains, 2 + nsteps)
    mt = tl[:, 1:2 * (nsteps + 2):2].astype(np.float64)
    hw = tl[:, S - 2].astype(np.int64)
    xcc = tl[:, S - 1].astype(np.int64) & 0xF
    t0 = rt[:, 0].min()
    us = (rt - t0) / RT_HZ * 1e6                                 # µs since the first entry
    entry, pro = us[:, 0], us[:, 1]
    ends = us[:, 2:]
    step = np.diff(us[:, 1:], axis=1)                            # per chain, per step
    mhz = np.diff(mt[:, 1:], axis=1) / np.maximum(np.diff(rt[:, 1:], axis=1), 1) * 100.0
    last = ends[:, -1]
    per_xcc = {}
    for x in np.unique(xcc):
        sel = xcc == x
        per_xcc[int(x)] = dict(chains=int(sel.sum()), mean_end_us=float(last[sel].mean()),
                               max_end_us=float(last[sel].max()),
                               mean_step_us=float(step[sel].mean()),
                               clock_mhz_median=float(np.median(mhz[sel])),
                               cycles_per_step_median=float(np.median(np.diff(mt[sel][:, 1:], axis=1))),
                               prologue_us_mean=float((pro - entry)[sel].mean()))
    out = dict(
        tag=tag, steps=nsteps, chains=C_, event_us=ev_us,
        event_us_per_step=ev_us / nsteps,
        span_us=float(last.max()),
        dispatch_skew_us=float(entry.max() - entry.min()),
        prologue_us_mean=float((pro - entry).mean()), prologue_us_max=float((pro - entry).max()),
        first_step_us_mean=float(step[:, 0].mean()),
        step_us_mean=float(step.mean()),
        step_us_mean_after_first=float(step[:, 1:].mean()) if nsteps > 1 else None,
        step_us_by_index_mean=[float(x) for x in step.mean(axis=0)[:25]],
        step_us_by_index_max=[float(x) for x in step.max(axis=0)[:25]],
        chain_total_us_min=float((last - entry).min()),
        chain_total_us_median=float(np.median(last - entry)),
        chain_total_us_max=float((last - entry).max()),
        end_us_median=float(np.median(last)), end_us_max=float(last.max()),
        tail_us=float(last.max() - np.median(last)),
        clock_mhz_median=float(np.median(mhz)), clock_mhz_min=float(mhz.min()),
        clock_mhz_first_step=float(np.median(mhz[:, 0])),
        clock_mhz_last_step=float(np.median(mhz[:, -1])),
        slowest_chains=[int(c) for c in np.argsort(-(last))[:8]],
        slowest_hw=[(int(xcc[c]), int((hw[c] >> 8) & 0xF), int((hw[c] >> 13) & 0x7))
                    for c in np.argsort(-(last))[:8]],
        per_xcc=per_xcc,
    )
    # how the launch's span splits: dispatch + prologue + nsteps x median step + tail
    med_step = float(np.median(step))
    out["median_step_us"] = med_step
    out["span_minus_steps_us"] = float(last.max() - nsteps * med_step)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "timeline.json"))
    ap.add_argument("--chains", type=int, default=256)
    args = ap.parse_args()
    import torch
    import bench
    from gpt_amd import GPT_SGLD as G
    from gpt_amd._lib import check, lib
    from gpt_amd.session import SGLDSession, feature_device
    dev = torch.device("cuda", 0)
    n, D, r, Q, m = 500, 8, 5, 200, 50
    Xtr, ytr, _, _, _ = bench.kin40k(D)
    ls = np.array([2.5242, 2.3376, 1.3630, 1.4949, 1.6022, 1.1366, 1.1964, 1.7028])
    I = G.samplenz(r, D, Q, 17)
    Z, b = G.feature_inputs(n, D, 17)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    phi = feature_device(tt(Xtr.T), tt(ls), 1.042, math.sqrt(n / Q ** (1 / D)), tt(Z.T), tt(b.T))
    y = tt(ytr)
    torch.cuda.synchronize()
    S = int(lib().gpt_sgld_timeline_slots())
    Cn = args.chains
    nb = 200

    def timeline(sess, k, tag):
        out = np.zeros((Cn, S), dtype=np.int64)
        ev = C.c_double(0.0)
        check(lib().gpt_sgld_session_timeline(sess._h, k, out.ctypes.data_as(C.POINTER(C.c_int64)),
                                              C.byref(ev)))
        if not out[:, 0].all():
            raise SystemExit("timeline empty: run with GPTSGLD_LIB=gpt_amd/libgptsgld_tl.so")
        return analyse(out, k, ev.value, tag)

    res = []
    sess = SGLDSession(phi, y, I, r, Q, m, 1e-5, 1e-8, 0.0476, 0, 8, [c + 1 for c in range(Cn)],
                       store=False, engine="chain")
    # bench order: 300 ms of clock warm-up on a scratch session, 5 warm-up steps, then the timed 20
    sw = SGLDSession(phi, y, I, r, Q, m, 1e-5, 1e-8, 0.0476, 0, 2, [10 ** 6 + c for c in range(Cn)],
                     store=False, engine="chain")
    tw = time.perf_counter()
    while time.perf_counter() - tw < 0.3 and sw.steps_done < sw.total_steps:
        sw.run(min(nb, sw.total_steps - sw.steps_done)); sw.sync()
    sw.close()
    sess.run(5); sess.sync()
    res.append(timeline(sess, 20, "driver form: steps 5-24 right after 5 warm-up steps"))
    print(json.dumps(res[-1])[:400], flush=True)
    res.append(timeline(sess, 20, "steps 25-44, back to back"))
    time.sleep(0.01)
    res.append(timeline(sess, 20, "steps 45-64 after a 10 ms idle gap"))
    sess.run(nb - 65 + 4 * nb + 5); sess.sync()             # to step 1005 (epoch 5)
    res.append(timeline(sess, 20, "steps 1005-1024 (epoch 5)"))
    res.append(timeline(sess, 100, "steps 1025-1124: a 100-step launch"))
    sess.run(nb - 125); sess.sync()                          # epoch 6 start
    res.append(timeline(sess, 200, "steps 1200-1399: an epoch-long launch"))
    res.append(timeline(sess, 20, "steps 1400-1419 (new epoch: order kernel before)"))
    sess.close()
    for x in res:
        print(json.dumps({k: v for k, v in x.items() if not k.startswith("step_us_by")}), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
