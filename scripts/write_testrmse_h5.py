"""Write the per-sweep test-RMSE curves as the reference's HDF5 files (§8(f) item 2).

    /opt/conda/bin/python3.9 scripts/write_testrmse_h5.py CURVES.npz [--outdir DIR] [--prefix testRMSE_kin40k]

kin40kExperiment.jl:88-90 writes one file per sweep j, `testRMSE_kin40k$j.h5`, holding the dataset
`testRMSE` (Float64, length maxepoch).  scripts/kin40k_experiment.py saves the device run's curves
as an .npz (array `testRMSE`, sweeps x epochs) because the image's /usr/bin/python3 has no h5py;
this converter runs under the container's /opt/conda python (h5py 3.3) and writes the same file
names, dataset name, dtype and shape as the reference (checked against
/root/reference/testRMSE_kin40k.h5 when that file is present: dataset `testRMSE`, {200}, double).
A NaN-bailed sweep (all-zero stores) keeps its curve as computed, as the reference would.
"""
import argparse
import os
import sys

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("curves")
    ap.add_argument("--outdir", default=".")
    ap.add_argument("--prefix", default="testRMSE_kin40k")
    ap.add_argument("--check", default="/root/reference/testRMSE_kin40k.h5",
                    help="reference file whose dataset layout the output must match (if present)")
    args = ap.parse_args()
    try:
        import h5py
    except ImportError:
        sys.exit("h5py is not importable by %s: run this with /opt/conda/bin/python3.9" % sys.executable)
    curves = np.atleast_2d(np.load(args.curves)["testRMSE"]).astype(np.float64)
    os.makedirs(args.outdir, exist_ok=True)
    paths = []
    for j, c in enumerate(curves, start=1):                 # @parallel for j=1:10 (:67)
        path = os.path.join(args.outdir, "%s%d.h5" % (args.prefix, j))
        with h5py.File(path, "w") as f:                     # h5open(..., "w") / write(file, "testRMSE", ...)
            f.create_dataset("testRMSE", data=np.ascontiguousarray(c))
        paths.append(path)
    if os.path.exists(args.check):
        with h5py.File(args.check, "r") as ref, h5py.File(paths[0], "r") as got:
            r, g = ref["testRMSE"], got["testRMSE"]
            assert list(ref.keys()) == list(got.keys()) == ["testRMSE"]
            assert r.dtype == g.dtype and r.ndim == g.ndim == 1, (r.dtype, g.dtype, r.shape, g.shape)
    print("\n".join(paths))


if __name__ == "__main__":
    main()
