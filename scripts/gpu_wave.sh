#!/bin/bash
# Wave engine iteration: parity cases, phase stamps (16 / 256 chains), r = 20 throughput probe.
# Output tag: $1 (files gpurun_out/<tag>_*).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-w}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wave or selection" > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/wave_stamps.py --chains 16 --steps 4 --out gpurun_out/${T}_stamps16.json > gpurun_out/${T}_stamps.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/wave_stamps.py --chains 256 --steps 4 --out gpurun_out/${T}_stamps256.json >> gpurun_out/${T}_stamps.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/wave_probe.py --chains 256,10 --engines wave --steps 200 --out gpurun_out/${T}_probe.json > gpurun_out/${T}_probe.log 2>&1 || exit $?
python3 - "$T" <<'PY'
import json, sys
T = sys.argv[1]
for c in (16, 256):
    d = json.load(open("gpurun_out/%s_stamps%d.json" % (T, c)))
    print(c, "dim", int(d["dim_total_median"]), {k: int(v) for k, v in d["dim_cycles_median"].items()})
    print(c, "vph", {k: int(v) for k, v in d["vphase_cycles_median"].items()})
    print(c, "expm_r", d["expm_r"], "expm_2r", d["expm_2r"])
for d in json.load(open("gpurun_out/%s_probe.json" % T)):
    print(d)
PY
