"""Regenerate the committed golden fixtures from the reference's own data files.

Run in the survey container (needs h5py, which only /opt/conda/bin/python3.9 has):

    /opt/conda/bin/python3.9 tests/golden/make_golden.py /root/reference

Outputs (all small, data only — inputs and expected outputs, no reference source):
  tensor_synth_5D.npz / tensor_synth_10D.npz  TensorSynthData{5D,10D}100N.h5 (written by
      MakeSynthData.jl:6-27 with fhatdraw, GPT_SGLD.jl:323-342): X, w, U, I, phi,
      length_scale, y1..y3 — pins pred() and the column-major layouts end to end.
  kin40k.npz          kin40k_{train,test}_{data,labels}.txt (config 3/4 inputs)
  powerplant.npz      Folds5x2_pp.csv (bare-CR line endings; configs 1/2 inputs)
  ref_curves.npz      testRMSE_kin40k.h5:testRMSE, testRMSE_PP.h5:testRMSE,testRMSE2
      (the reference's recorded learning curves — statistical anchors)

h5py reports Julia arrays with reversed dimensions; every array is transposed back to
Julia's (column-major) index order here, so fixture[a, b, c] == julia[a+1, b+1, c+1].
"""
import os
import sys

import numpy as np


def julia_order(a):
    a = np.asarray(a)
    return np.asfortranarray(a.transpose(tuple(range(a.ndim))[::-1]))


def main(ref):
    import h5py
    out = os.path.dirname(os.path.abspath(__file__))
    for tag in ("5D", "10D"):
        with h5py.File(os.path.join(ref, "TensorSynthData%s100N.h5" % tag), "r") as f:
            d = {k: julia_order(f[k][()]) for k in f.keys()}
        np.savez(os.path.join(out, "tensor_synth_%s.npz" % tag), **d)
    rd = lambda name: np.loadtxt(os.path.join(ref, name), dtype=np.float64)
    np.savez_compressed(os.path.join(out, "kin40k.npz"),
                        Xtrain=rd("kin40k_train_data.txt"), ytrain=rd("kin40k_train_labels.txt"),
                        Xtest=rd("kin40k_test_data.txt"), ytest=rd("kin40k_test_labels.txt"))
    with open(os.path.join(ref, "Folds5x2_pp.csv"), "rb") as f:
        lines = f.read().decode().replace("\r\n", "\n").replace("\r", "\n").strip().split("\n")
    data = np.array([[float(v) for v in ln.split(",")] for ln in lines[1:]], dtype=np.float64)
    np.savez_compressed(os.path.join(out, "powerplant.npz"), data=data)
    curves = {}
    with h5py.File(os.path.join(ref, "testRMSE_kin40k.h5"), "r") as f:
        curves["testRMSE_kin40k"] = f["testRMSE"][()]
    with h5py.File(os.path.join(ref, "testRMSE_PP.h5"), "r") as f:
        curves["testRMSE_PP"] = f["testRMSE"][()]
        curves["testRMSE2_PP"] = f["testRMSE2"][()]
    with h5py.File(os.path.join(ref, "fullWresults.h5"), "r") as f:     # GPT_fullw_gibbs curves
        curves["fullW_testRMSE"] = f["testRMSE"][()]
        curves["fullW_trainRMSE"] = f["trainRMSE"][()]
    np.savez(os.path.join(out, "ref_curves.npz"), **curves)
    print("wrote fixtures to", out)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
