"""Probe: GPT_SGLDERM_RMSprop at PowerPlant config 2 for a few ε (which converge, and where)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_gpu_quality import _pp_curves  # noqa: E402

ref = np.load(os.path.join(ROOT, "tests", "golden", "ref_curves.npz"))["testRMSE2_PP"]
out = {}
CFGS = [(float(a), int(b)) for a, b in (x.split(":") for x in sys.argv[1:])] or \
    [(3e-5, 256), (1e-5, 256), (3e-6, 256), (1e-6, 256)]
for eps, m in CFGS:
    curves, bailed = _pp_curves(list(range(1, 5)), 200, eps, eps, rms=(eps, 0.99), m=m)
    d = dict(bailed=bailed)
    if len(curves):
        d.update(final=curves[:, -1].tolist(), last50=curves[:, -50:].mean(axis=1).tolist(),
                 first=curves[:, 0].tolist())
    out["%g:%d" % (eps, m)] = d
    print(eps, m, d, flush=True)
print("ref", ref[0], ref[-1], ref[-50:].mean())
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "probe_rmsprop_pp.json"), "w"), indent=1)
