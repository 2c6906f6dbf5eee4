"""Shader-clock cycles per SGLD step of chain-engine ablation libraries (scripts/ablation_build.sh),
256 chains at the bench shape: one process per library (a library per process), each measuring
s_memtime deltas per step over a 200-step launch after a warm-up.  Clock-independent, so variants
measured minutes apart compare directly.

    python scripts/ablation_run.py base nonoise ...   (on the GPU box)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, math, sys, time
import numpy as np
sys.path.insert(0, %(root)r)
import ctypes as C
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
Cn = 256
S = int(lib().gpt_sgld_timeline_slots())
s = SGLDSession(phi, y, I, r, Q, m, 1e-5, 1e-8, 0.0476, 0, 4, [c + 1 for c in range(Cn)],
                store=False, engine="chain")
s.run(200); s.sync()                      # warm-up epoch (clock, caches)
out = np.zeros((Cn, S), dtype=np.int64)
ev = C.c_double(0.0)
check(lib().gpt_sgld_session_timeline(s._h, 200, out.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(ev)))
# slots: 0 entry, 1 prologue end, 2 + s end of step s (CHAIN_TIMELINE=2 builds: the last only)
rt = out[:, [2, 2 * 201]].astype(float); mt = out[:, [3, 2 * 201 + 1]].astype(float)
cyc = np.diff(mt, axis=1) / 200.0         # per chain: prologue end -> last step end, per step
us = np.diff(rt, axis=1) / 100.0 / 200.0
print(json.dumps(dict(cycles_per_step_median=float(np.median(cyc)), cycles_per_step_mean=float(cyc.mean()),
                      us_per_step_median=float(np.median(us)), event_us_per_step=ev.value / 200,
                      clock_mhz=float(np.median(cyc / np.maximum(us, 1e-9))))))
"""


def main():
    res = {}
    for name in sys.argv[1:]:
        lib = os.path.join(ROOT, "gpt_amd", "libgptsgld.so" if name == "product"
                           else "libgptsgld_abl_%s.so" % name)
        env = dict(os.environ, GPTSGLD_LIB=lib)
        p = subprocess.run([sys.executable, "-c", CHILD % dict(root=ROOT)], env=env,
                           capture_output=True, text=True, timeout=240)
        line = [x for x in p.stdout.splitlines() if x.startswith("{")]
        res[name] = json.loads(line[-1]) if line else dict(error=p.stderr[-800:])
        print(name, res[name], flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "ablation.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
