// C++ fp64 restatement of GPT_fullw_sideinfo's SGD epochs (100k_movielensExperiment.jl:409-551
// with langevin = stiefel = false, the live experiment of :723-739), folds in parallel on OpenMP
// threads.
//
// TEST INFRASTRUCTURE and CPU BASELINE (bench.py --workload movielens `cpu_baseline`), not product
// code; checked against oracle/movielens_ref.py by tests/test_oracle.py.  Follows the reference's
// dense arithmetic: per minibatch the gradient matrices of every U / V row are zeroed, the batch's
// ratings add their rows (:455-477), and every row then takes its step (:481-507); per epoch the
// train and test predictions (:526-539) are formed and their squared errors summed.  run_fold_lazy
// is the same arithmetic with the GPU's lazy prior-decay move (the fair CPU baseline of that path).
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct Fold {
  const int32_t* user;     // N, 0-based
  const int32_t* movie;
  const double* rating;    // standardised
  const int32_t* perm;     // epochs × N: each epoch's order
  const int32_t* tuser;    // Ntest
  const int32_t* tmovie;
  const double* trating;
  double* w;               // r × r, w[i + r·j]
  double* U;               // (n1 + D1) × r, row-major
  double* V;               // (n2 + D2) × r
  double* sse;             // epochs × 2 (train, test)
};

struct Cfg {
  int N, Ntest, n1, D1, n2, D2, r, m, epochs;
  double signal_var, sigma_u, sigma_w, epsw, epsU, a, b, c;
  const int32_t *uptr, *ufe, *vptr, *vfe;   // CSR feature rows (absolute row indices)
};

// sumU / sumV of one (user, movie) pair (:462)
void sums(const Cfg& g, const Fold& f, int u, int v, double* su, double* sv) {
  const int r = g.r;
  for (int l = 0; l < r; ++l) {
    double s = 0.0;
    for (int z = g.uptr[u]; z < g.uptr[u + 1]; ++z) s += f.U[(size_t)g.ufe[z] * r + l];
    su[l] = f.U[(size_t)u * r + l] + g.b * s;
    s = 0.0;
    for (int z = g.vptr[v]; z < g.vptr[v + 1]; ++z) s += f.V[(size_t)g.vfe[z] * r + l];
    sv[l] = f.V[(size_t)v * r + l] + g.c * s;
  }
}

double predict(const Cfg& g, const Fold& f, int u, int v, double* su, double* sv) {
  sums(g, f, u, v, su, sv);
  const int r = g.r;
  double p = 0.0;
  for (int j = 0; j < r; ++j) {
    double t = 0.0;
    for (int i = 0; i < r; ++i) t += su[i] * f.w[i + r * j];
    p += t * sv[j];
  }
  return g.a * p;
}

void run_fold(const Cfg& g, const Fold& f) {
  const int r = g.r, rowsU = g.n1 + g.D1, rowsV = g.n2 + g.D2;
  std::vector<double> gw((size_t)r * r), gU((size_t)rowsU * r), gV((size_t)rowsV * r);
  std::vector<double> su(r), sv(r), t(r), ut(r), vt(r);
  const int nb = (g.N + g.m - 1) / g.m;
  const double su2 = g.sigma_u * g.sigma_u, sw2 = g.sigma_w * g.sigma_w;
  for (int ep = 0; ep < g.epochs; ++ep) {
    const int32_t* perm = f.perm + (size_t)ep * g.N;
    for (int bt = 0; bt < nb; ++bt) {
      const int i0 = bt * g.m, B = std::min(g.m, g.N - i0);
      std::fill(gw.begin(), gw.end(), 0.0);
      std::fill(gU.begin(), gU.end(), 0.0);
      std::fill(gV.begin(), gV.end(), 0.0);
      for (int ii = 0; ii < B; ++ii) {
        const int k = perm[i0 + ii], u = f.user[k], v = f.movie[k];
        sums(g, f, u, v, su.data(), sv.data());
        double p = 0.0;
        for (int j = 0; j < r; ++j) {
          double s = 0.0;
          for (int i = 0; i < r; ++i) s += su[i] * f.w[i + r * j];
          t[j] = s;
          p += s * sv[j];
        }
        const double e = f.rating[k] - g.a * p;
        for (int i = 0; i < r; ++i) {                       // Utemp = (e·sumV)·wᵀ, Vtemp = (e·sumU)·w
          double s1 = 0.0, s2 = 0.0;
          for (int j = 0; j < r; ++j) {
            s1 += e * sv[j] * f.w[i + r * j];
            s2 += e * su[j] * f.w[j + r * i];
          }
          ut[i] = s1;
          vt[i] = s2;
        }
        for (int j = 0; j < r; ++j)
          for (int i = 0; i < r; ++i) gw[i + r * j] += e * su[i] * sv[j] / g.signal_var;
        const double ca = g.a / g.signal_var;
        for (int l = 0; l < r; ++l) {
          gU[(size_t)u * r + l] += ca * ut[l];
          gV[(size_t)v * r + l] += ca * vt[l];
        }
        for (int z = g.uptr[u]; z < g.uptr[u + 1]; ++z)
          for (int l = 0; l < r; ++l) gU[(size_t)g.ufe[z] * r + l] += ca * g.b * ut[l];
        for (int z = g.vptr[v]; z < g.vptr[v + 1]; ++z)
          for (int l = 0; l < r; ++l) gV[(size_t)g.vfe[z] * r + l] += ca * g.c * vt[l];
      }
      const double cN = (double)g.N / (double)B;
      for (int o = 0; o < r * r; ++o) f.w[o] += g.epsw * (gw[o] * cN - f.w[o] / sw2) / 2;
      for (size_t o = 0; o < gU.size(); ++o) f.U[o] += g.epsU * (gU[o] * cN - f.U[o] / su2) / 2;
      for (size_t o = 0; o < gV.size(); ++o) f.V[o] += g.epsU * (gV[o] * cN - f.V[o] / su2) / 2;
    }
    double s0 = 0.0, s1 = 0.0;                               // the epoch's evaluation (:526-539)
    for (int k = 0; k < g.N; ++k) {
      const double d = f.rating[k] - predict(g, f, f.user[k], f.movie[k], su.data(), sv.data());
      s0 += d * d;
    }
    for (int k = 0; k < g.Ntest; ++k) {
      const double d = f.trating[k] - predict(g, f, f.tuser[k], f.tmovie[k], su.data(), sv.data());
      s1 += d * d;
    }
    f.sse[2 * ep] = s0;
    f.sse[2 * ep + 1] = s1;
  }
}

// The same epochs with the lazy prior-decay move the GPU's one-launch epoch uses (cf.hip,
// cf_epoch_kernel domove = 2): a row outside a minibatch has a zero gradient, so its step
// M ← M + εU·(0 − M/σ_u²)/2 only scales it by c = 1 − εU/(2σ_u²).  Each row keeps the step it
// was last brought to (cur) and is read as M·c^Δ; the rows a batch touches (its users, movies and
// their side-feature rows) are brought to the current step, take the full step and are marked one
// step ahead; at the epoch's end every row is brought to the epoch's last step (its evaluation
// reads them).  The same arithmetic regrouped (powers of c instead of repeated products): the
// fair CPU counterpart of the GPU's algorithm, beside the reference's dense moves above.
void run_fold_lazy(const Cfg& g, const Fold& f) {
  const int r = g.r, rowsU = g.n1 + g.D1, rowsV = g.n2 + g.D2;
  const int nb = (g.N + g.m - 1) / g.m;
  const double su2 = g.sigma_u * g.sigma_u, sw2 = g.sigma_w * g.sigma_w;
  const double cdec = 1.0 - g.epsU / (2.0 * su2);
  std::vector<double> cpow((size_t)nb + 2, 1.0);
  for (int d = 1; d <= nb + 1; ++d) cpow[d] = cpow[d - 1] * cdec;
  std::vector<double> gw((size_t)r * r), gU((size_t)rowsU * r, 0.0), gV((size_t)rowsV * r, 0.0);
  std::vector<double> su(r), sv(r), t(r), ut(r), vt(r);
  std::vector<int> curU(rowsU, 0), curV(rowsV, 0), listU, listV;
  std::vector<char> inU(rowsU, 0), inV(rowsV, 0);
  auto touch = [&](int row, int j, double* M, std::vector<int>& cur, std::vector<char>& in,
                   std::vector<int>& list) {
    if (in[row]) return;
    in[row] = 1;
    list.push_back(row);
    const int d = j - cur[row];
    if (d > 0)
      for (int l = 0; l < r; ++l) M[(size_t)row * r + l] *= cpow[d];
    cur[row] = j;
  };
  for (int ep = 0; ep < g.epochs; ++ep) {
    const int32_t* perm = f.perm + (size_t)ep * g.N;
    std::fill(curU.begin(), curU.end(), 0);
    std::fill(curV.begin(), curV.end(), 0);
    for (int bt = 0; bt < nb; ++bt) {
      const int i0 = bt * g.m, B = std::min(g.m, g.N - i0);
      listU.clear();
      listV.clear();
      for (int ii = 0; ii < B; ++ii) {
        const int k = perm[i0 + ii], u = f.user[k], v = f.movie[k];
        touch(u, bt, f.U, curU, inU, listU);
        for (int z = g.uptr[u]; z < g.uptr[u + 1]; ++z) touch(g.ufe[z], bt, f.U, curU, inU, listU);
        touch(v, bt, f.V, curV, inV, listV);
        for (int z = g.vptr[v]; z < g.vptr[v + 1]; ++z) touch(g.vfe[z], bt, f.V, curV, inV, listV);
      }
      std::fill(gw.begin(), gw.end(), 0.0);
      for (int ii = 0; ii < B; ++ii) {
        const int k = perm[i0 + ii], u = f.user[k], v = f.movie[k];
        sums(g, f, u, v, su.data(), sv.data());
        double p = 0.0;
        for (int j = 0; j < r; ++j) {
          double s = 0.0;
          for (int i = 0; i < r; ++i) s += su[i] * f.w[i + r * j];
          t[j] = s;
          p += s * sv[j];
        }
        const double e = f.rating[k] - g.a * p;
        for (int i = 0; i < r; ++i) {
          double s1 = 0.0, s2 = 0.0;
          for (int j = 0; j < r; ++j) {
            s1 += e * sv[j] * f.w[i + r * j];
            s2 += e * su[j] * f.w[j + r * i];
          }
          ut[i] = s1;
          vt[i] = s2;
        }
        for (int j = 0; j < r; ++j)
          for (int i = 0; i < r; ++i) gw[i + r * j] += e * su[i] * sv[j] / g.signal_var;
        const double ca = g.a / g.signal_var;
        for (int l = 0; l < r; ++l) {
          gU[(size_t)u * r + l] += ca * ut[l];
          gV[(size_t)v * r + l] += ca * vt[l];
        }
        for (int z = g.uptr[u]; z < g.uptr[u + 1]; ++z)
          for (int l = 0; l < r; ++l) gU[(size_t)g.ufe[z] * r + l] += ca * g.b * ut[l];
        for (int z = g.vptr[v]; z < g.vptr[v + 1]; ++z)
          for (int l = 0; l < r; ++l) gV[(size_t)g.vfe[z] * r + l] += ca * g.c * vt[l];
      }
      const double cN = (double)g.N / (double)B;
      for (int o = 0; o < r * r; ++o) f.w[o] += g.epsw * (gw[o] * cN - f.w[o] / sw2) / 2;
      for (int row : listU) {
        for (int l = 0; l < r; ++l) {
          double& M = f.U[(size_t)row * r + l];
          double& G = gU[(size_t)row * r + l];
          M += g.epsU * (G * cN - M / su2) / 2;
          G = 0.0;
        }
        curU[row] = bt + 1;
        inU[row] = 0;
      }
      for (int row : listV) {
        for (int l = 0; l < r; ++l) {
          double& M = f.V[(size_t)row * r + l];
          double& G = gV[(size_t)row * r + l];
          M += g.epsU * (G * cN - M / su2) / 2;
          G = 0.0;
        }
        curV[row] = bt + 1;
        inV[row] = 0;
      }
    }
    for (int row = 0; row < rowsU; ++row)               // every row as of the epoch's end
      for (int l = 0; l < r; ++l) f.U[(size_t)row * r + l] *= cpow[nb - curU[row]];
    for (int row = 0; row < rowsV; ++row)
      for (int l = 0; l < r; ++l) f.V[(size_t)row * r + l] *= cpow[nb - curV[row]];
    double s0 = 0.0, s1 = 0.0;
    for (int k = 0; k < g.N; ++k) {
      const double d = f.rating[k] - predict(g, f, f.user[k], f.movie[k], su.data(), sv.data());
      s0 += d * d;
    }
    for (int k = 0; k < g.Ntest; ++k) {
      const double d = f.trating[k] - predict(g, f, f.tuser[k], f.tmovie[k], su.data(), sv.data());
      s1 += d * d;
    }
    f.sse[2 * ep] = s0;
    f.sse[2 * ep + 1] = s1;
  }
}

}  // namespace

extern "C" {

// icfg: N, Ntest, n1, D1, n2, D2, r, m, epochs, lazy (1: run_fold_lazy, the GPU's move; 0: the
// reference's dense moves); dcfg: signal_var, sigma_u, sigma_w, epsw, epsU, a, b, c.  Per fold f
// (arrays of nf pointers): ids / ratings / perms / test set / state (in-out) / sse (epochs × 2).
// Returns the wall seconds of the epochs (folds on `threads` threads).
double gptcpu_cf_sgd(int nf, const int64_t* icfg, const double* dcfg, const int32_t* uptr,
                     const int32_t* ufe, const int32_t* vptr, const int32_t* vfe,
                     const int32_t* const* user, const int32_t* const* movie,
                     const double* const* rating, const int32_t* const* perm,
                     const int32_t* const* tuser, const int32_t* const* tmovie,
                     const double* const* trating, double* const* w, double* const* U,
                     double* const* V, double* const* sse, int threads) {
  Cfg g{};
  g.N = (int)icfg[0]; g.Ntest = (int)icfg[1]; g.n1 = (int)icfg[2]; g.D1 = (int)icfg[3];
  g.n2 = (int)icfg[4]; g.D2 = (int)icfg[5]; g.r = (int)icfg[6]; g.m = (int)icfg[7];
  g.epochs = (int)icfg[8];
  const bool lazy = icfg[9] != 0;
  g.signal_var = dcfg[0]; g.sigma_u = dcfg[1]; g.sigma_w = dcfg[2]; g.epsw = dcfg[3];
  g.epsU = dcfg[4]; g.a = dcfg[5]; g.b = dcfg[6]; g.c = dcfg[7];
  g.uptr = uptr; g.ufe = ufe; g.vptr = vptr; g.vfe = vfe;
  std::vector<Fold> folds(nf);
  for (int f = 0; f < nf; ++f)
    folds[f] = Fold{user[f], movie[f], rating[f], perm[f], tuser[f], tmovie[f], trating[f],
                    w[f], U[f], V[f], sse[f]};
  const auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1)
  for (int f = 0; f < nf; ++f) {
    if (lazy) run_fold_lazy(g, folds[f]);
    else run_fold(g, folds[f]);
  }
  const auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}

}  // extern "C"
