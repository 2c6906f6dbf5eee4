"""Build tests/golden/ml100k.npz from the reference's MovieLens-100k files (data only).

Follows the data processing of 100k_movielensExperiment.jl:561-586:
  * ratings u{1..5}.{base,test}: (user, movie, rating) columns (timestamps dropped);
  * UserData: age binned by bin_age (:43-46: quintile edges, first edge >= age), then dummy
    columns for age bin / gender / occupation with sorted levels (getdummy :8-21), id and zip
    dropped (:580-583)  -> 943 x 28;
  * MovieData: the 19 genre flags minus the first ("unknown"), id dropped (:581-584) -> 1682 x 18.
Usage: python scripts/make_ml100k_fixture.py /root/reference/ml-100k
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bin_age(age):
    q = np.quantile(age, [0.2, 0.4, 0.6, 0.8, 1.0])          # Julia's default (type 7)
    return np.array([int(np.argmin(q < x)) + 1 for x in age])  # indmin(q .< x)


def main(src):
    users = [l.rstrip("\n").split("|") for l in open(os.path.join(src, "u.user"), encoding="latin-1")]
    age = np.array([float(u[1]) for u in users])
    ab = bin_age(age)
    cols = []
    for vals in (list(ab), [u[2] for u in users], [u[3] for u in users]):
        levels = sorted(set(vals))
        cols.append(np.array([[1 if v == lv else 0 for lv in levels] for v in vals], dtype=np.uint8))
    user_data = np.hstack(cols)
    items = [l.rstrip("\n").split("|") for l in open(os.path.join(src, "u.item"), encoding="latin-1")]
    genres = np.array([[int(x) for x in it[5:24]] for it in items], dtype=np.uint8)
    movie_data = genres[:, 1:]
    out = dict(user_data=user_data, movie_data=movie_data)
    for i in range(1, 6):
        for part in ("base", "test"):
            a = np.loadtxt(os.path.join(src, "u%d.%s" % (i, part)), dtype=np.int64)
            out["u%d_%s" % (i, part)] = a[:, :3].astype(np.int16)
    dst = os.path.join(ROOT, "tests", "golden", "ml100k.npz")
    np.savez_compressed(dst, **out)
    print(dst, user_data.shape, movie_data.shape, os.path.getsize(dst))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/ml-100k")
