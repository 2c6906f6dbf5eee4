// gpt_sgld_cpu.cpp — C++ fp64 restatement of the reference's SGLD loop, GPT_SGLD.jl:345-448.
//
// TEST INFRASTRUCTURE and CPU BASELINE.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg load this library (oracle/_build/libgptcpu.so); the product path (gpt_amd/,
// libgptsgld.so) never does.  It is the on-box CPU restatement SURVEY.md §7.2 / §8(d) call for:
// the reference's loop order, one chain per OpenMP thread (chains are independent, as the
// reference's `@parallel for` sweeps, kin40kExperiment.jl:67), no BLAS.  Its random draws follow
// the framework's Philox contract (oracle/philox.py), so on the same inputs it reproduces the
// numpy oracle (tests/test_cpu_baseline.py) and, through it, the GPU path.
//
// Per step (GPT_SGLD.jl line numbers):
//   idx = order[batch]                                     :379-381 (gather by index, no copy)
//   temp[k,l,i] = dot(phi[:,k,i], U[:,l,k])                :384 phidotU :193-205
//   V[q,i] = Π_k temp[k, I[q,k], i]                        :387 computeV :208-220
//   fhat[i] = dot(V[:,i], w)                               :390 computefhat :223-230
//   gradw = (N/B)·V(y−fhat)/σ² − w/σ_w²                    :393
//   U_phi[q,i,k] = V[q,i]/temp[k,I[q,k],i]                 :396 computeU_phi :246-258
//   A[l,k,i] = Σ_{q: I[q,k]=l} U_phi[q,i,k]·w[q]          :399 computeA :261-273
//   gradU_k = (N/B)/σ²·Σ_i kron(A[:,k,i], phi[:,k,i])·res_i :402-408 (Psi·res, Psi not stored)
//   w += εw/2·gradw + √εw·ξ                                :411-414
//   U_k = geod(U_k, proj(U_k, √εU/2·gradU_k + ζ_k), √εU)   :417-424 (proj :14-16, geod :19-37)
//   store w, U after burn-in                               :441-444 (every store_every-th step)
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

// ---------------------------------------------------------------- Philox contract (philox.py)
struct U4 { uint32_t x, y, z, w; };
enum : uint32_t { kWInit = 1, kUInit = 2, kPerm = 3, kWNoise = 4, kUNoise = 5 };

inline U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
  }
  return U4{c0, c1, c2, c3};
}
inline double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6) + 0.5) * (1.0 / 9007199254740992.0);
}
// element e of normal stream (c1, c2, c3): Box–Muller on the block c0 = e >> 1
inline double normal_at(uint64_t seed, uint32_t e, uint32_t c1, uint32_t c2, uint32_t c3) {
  const U4 x = philox(e >> 1, c1, c2, c3, seed);
  const double rad = std::sqrt(-2.0 * std::log(u53(x.x, x.y)));
  const double th = 6.283185307179586 * u53(x.z, x.w);
  return (e & 1u) ? rad * std::sin(th) : rad * std::cos(th);
}
// elements 2·c0 and 2·c0+1 of the stream (one Box–Muller pair)
inline void normal_pair(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                        double& z0, double& z1) {
  const U4 x = philox(c0, c1, c2, c3, seed);
  const double rad = std::sqrt(-2.0 * std::log(u53(x.x, x.y)));
  const double th = 6.283185307179586 * u53(x.z, x.w);
  z0 = rad * std::cos(th);
  z1 = rad * std::sin(th);
}

// U-noise contract (gpt_common.h normal_quad / oracle/philox.py unoise_quads): Philox block
// c0 = (l·NQ + q)·64 + λ gives column l of rows λ + 64·(4q + i), i < 4, from 32-bit uniforms.
inline double u32u(uint32_t x) { return ((double)x + 0.5) * (1.0 / 4294967296.0); }
inline void unoise_quads(int n, int r, uint64_t seed, uint32_t c1, uint32_t c2, uint32_t c3,
                         double* xi /* n×r column-major */) {
  const int nq = ((n + 63) / 64 + 3) / 4;
  for (int l = 0; l < r; ++l)
    for (int q = 0; q < nq; ++q)
      for (int lam = 0; lam < 64; ++lam) {
        const U4 x = philox((uint32_t)((l * nq + q) * 64 + lam), c1, c2, c3, seed);
        const double ra = std::sqrt(-2.0 * std::log(u32u(x.x)));
        const double rb = std::sqrt(-2.0 * std::log(u32u(x.z)));
        const double ta = 6.283185307179586 * u32u(x.y), tb = 6.283185307179586 * u32u(x.w);
        const double z[4] = {ra * std::cos(ta), ra * std::sin(ta), rb * std::cos(tb), rb * std::sin(tb)};
        for (int i = 0; i < 4; ++i) {
          const int j = lam + 64 * (4 * q + i);
          if (j < n) xi[j + (size_t)n * l] = z[i];
        }
      }
}

// ---------------------------------------------------------------- small dense helpers
// Column-major n×c matrices.  C = A(m×k)·B(k×c)
void matmul(int m, int k, int c, const double* A, const double* B, double* C) {
  for (int j = 0; j < c; ++j)
    for (int i = 0; i < m; ++i) {
      double s = 0.0;
      for (int t = 0; t < k; ++t) s += A[i + (size_t)m * t] * B[t + (size_t)k * j];
      C[i + (size_t)m * j] = s;
    }
}

// Solve M·X = B (p×p, p×p) by Gaussian elimination with partial pivoting (LAPACK gesv order).
void solve(int p, std::vector<double> M, std::vector<double>& B) {
  std::vector<int> piv(p);
  for (int c = 0; c < p; ++c) {
    int r = c;
    for (int i = c + 1; i < p; ++i)
      if (std::fabs(M[i + p * c]) > std::fabs(M[r + p * c])) r = i;
    if (r != c) {
      for (int j = 0; j < p; ++j) std::swap(M[c + p * j], M[r + p * j]);
      for (int j = 0; j < p; ++j) std::swap(B[c + p * j], B[r + p * j]);
    }
    const double d = M[c + p * c];
    for (int i = c + 1; i < p; ++i) {
      const double f = M[i + p * c] / d;
      M[i + p * c] = f;
      for (int j = c + 1; j < p; ++j) M[i + p * j] -= f * M[c + p * j];
      for (int j = 0; j < p; ++j) B[i + p * j] -= f * B[c + p * j];
    }
  }
  for (int j = 0; j < p; ++j)
    for (int i = p - 1; i >= 0; --i) {
      double s = B[i + p * j];
      for (int t = i + 1; t < p; ++t) s -= M[i + p * t] * B[t + p * j];
      B[i + p * j] = s / M[i + p * i];
    }
}

// expm by Padé scaling-and-squaring with Julia Base 0.3 expm! thresholds (oracle gpt_sgld_ref.expm).
bool expm(int p, const double* Ain, std::vector<double>& X) {
  static const double c3[] = {120.0, 60.0, 12.0, 1.0};
  static const double c5[] = {30240.0, 15120.0, 3360.0, 420.0, 30.0, 1.0};
  static const double c7[] = {17297280.0, 8648640.0, 1995840.0, 277200.0, 25200.0, 1512.0, 56.0, 1.0};
  static const double c9[] = {17643225600.0, 8821612800.0, 2075673600.0, 302702400.0, 30270240.0,
                              2162160.0, 110880.0, 3960.0, 90.0, 1.0};
  static const double c13[] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
                               1187353796428800.0, 129060195264000.0, 10559470521600.0,
                               670442572800.0, 33522128640.0, 1323241920.0, 40840800.0, 960960.0,
                               16380.0, 182.0, 1.0};
  const size_t pp = (size_t)p * p;
  std::vector<double> A(Ain, Ain + pp), Id(pp, 0.0);
  for (int i = 0; i < p; ++i) Id[i + p * i] = 1.0;
  double nA = 0.0;
  for (int j = 0; j < p; ++j) {
    double s = 0.0;
    for (int i = 0; i < p; ++i) s += std::fabs(A[i + p * j]);
    nA = std::max(nA, s);
  }
  X.assign(pp, NAN);
  if (!std::isfinite(nA)) return false;
  std::vector<double> A2(pp), Uu(pp), V(pp), T(pp);
  int si = 0;
  if (nA <= 2.1) {
    const double* C; int nc;
    if (nA > 0.95) { C = c9; nc = 10; } else if (nA > 0.25) { C = c7; nc = 8; }
    else if (nA > 0.015) { C = c5; nc = 6; } else { C = c3; nc = 4; }
    matmul(p, p, p, A.data(), A.data(), A2.data());
    std::vector<double> P = Id;
    for (size_t x = 0; x < pp; ++x) { Uu[x] = C[1] * P[x]; V[x] = C[0] * P[x]; }
    for (int k = 1; k <= (nc - 1) / 2; ++k) {
      matmul(p, p, p, P.data(), A2.data(), T.data());
      P = T;
      for (size_t x = 0; x < pp; ++x) { Uu[x] += C[2 * k + 1] * P[x]; V[x] += C[2 * k] * P[x]; }
    }
    matmul(p, p, p, A.data(), Uu.data(), T.data());
    Uu = T;
  } else {
    const double s = std::log2(nA / 5.4);
    si = s > 0 ? (int)std::ceil(s) : 0;
    if (s > 0)
      for (auto& a : A) a /= std::pow(2.0, si);
    const double* C = c13;
    std::vector<double> A4(pp), A6(pp), W(pp);
    matmul(p, p, p, A.data(), A.data(), A2.data());
    matmul(p, p, p, A2.data(), A2.data(), A4.data());
    matmul(p, p, p, A2.data(), A4.data(), A6.data());
    for (size_t x = 0; x < pp; ++x) W[x] = C[13] * A6[x] + C[11] * A4[x] + C[9] * A2[x];
    matmul(p, p, p, A6.data(), W.data(), T.data());
    for (size_t x = 0; x < pp; ++x) T[x] += C[7] * A6[x] + C[5] * A4[x] + C[3] * A2[x] + C[1] * Id[x];
    matmul(p, p, p, A.data(), T.data(), Uu.data());
    for (size_t x = 0; x < pp; ++x) W[x] = C[12] * A6[x] + C[10] * A4[x] + C[8] * A2[x];
    matmul(p, p, p, A6.data(), W.data(), V.data());
    for (size_t x = 0; x < pp; ++x) V[x] += C[6] * A6[x] + C[4] * A4[x] + C[2] * A2[x] + C[0] * Id[x];
  }
  std::vector<double> M(pp);
  X.resize(pp);
  for (size_t x = 0; x < pp; ++x) { M[x] = V[x] - Uu[x]; X[x] = V[x] + Uu[x]; }
  solve(p, M, X);
  for (int q = 0; q < si; ++q) {
    matmul(p, p, p, X.data(), X.data(), T.data());
    X = T;
  }
  for (double v : X)
    if (std::isnan(v)) return false;
  return true;
}

// Cyclic Jacobi eigen-decomposition of a symmetric r×r matrix (row-major).
void jacobi(int r, std::vector<double>& A, std::vector<double>& V, std::vector<double>& ev) {
  V.assign((size_t)r * r, 0.0);
  for (int i = 0; i < r; ++i) V[i * r + i] = 1.0;
  for (int sweep = 0; sweep < 100; ++sweep) {
    double off = 0.0, tot = 0.0;
    for (int i = 0; i < r; ++i)
      for (int j = 0; j < r; ++j) {
        tot += A[i * r + j] * A[i * r + j];
        if (i != j) off += A[i * r + j] * A[i * r + j];
      }
    if (off <= 1e-32 * tot) break;
    for (int p = 0; p < r; ++p)
      for (int q = p + 1; q < r; ++q) {
        const double apq = A[p * r + q];
        if (apq == 0.0) continue;
        const double th = (A[q * r + q] - A[p * r + p]) / (2.0 * apq);
        const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < r; ++k) {
          const double akp = A[k * r + p], akq = A[k * r + q];
          A[k * r + p] = c * akp - s * akq; A[k * r + q] = s * akp + c * akq;
        }
        for (int k = 0; k < r; ++k) {
          const double apk = A[p * r + k], aqk = A[q * r + k];
          A[p * r + k] = c * apk - s * aqk; A[q * r + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < r; ++k) {
          const double vkp = V[k * r + p], vkq = V[k * r + q];
          V[k * r + p] = c * vkp - s * vkq; V[k * r + q] = s * vkp + c * vkq;
        }
      }
  }
  ev.resize(r);
  for (int i = 0; i < r; ++i) ev[i] = A[i * r + i];
}

// GPT_SGLD.jl:357-369: w = σ_w·randn(Q); U_k = Zᵀ(ZZᵀ)^(-1/2), Z = randn(r, n).
void init_state(int n, int r, int D, int Q, uint64_t seed, double sigma_w, double* w, double* U) {
  for (int q = 0; q < Q; ++q) w[q] = sigma_w * normal_at(seed, q, 0, kWInit, 0);
  std::vector<double> Z((size_t)r * n), G, Vv, ev;
  for (int k = 0; k < D; ++k) {
    for (int e = 0; e < r * n; ++e) Z[e] = normal_at(seed, e, 0, kUInit, k);
    G.assign((size_t)r * r, 0.0);
    for (int a = 0; a < r; ++a)
      for (int c = 0; c < r; ++c) {
        double s = 0.0;
        for (int j = 0; j < n; ++j) s += Z[a + (size_t)r * j] * Z[c + (size_t)r * j];
        G[a * r + c] = s;
      }
    jacobi(r, G, Vv, ev);
    std::vector<double> S((size_t)r * r, 0.0);
    for (int a = 0; a < r; ++a)
      for (int c = 0; c < r; ++c) {
        double s = 0.0;
        for (int z = 0; z < r; ++z) s += Vv[a * r + z] * Vv[c * r + z] / std::sqrt(ev[z]);
        S[a * r + c] = s;
      }
    double* Uk = U + (size_t)n * r * k;
    for (int j = 0; j < n; ++j)
      for (int c = 0; c < r; ++c) {
        double s = 0.0;
        for (int a = 0; a < r; ++a) s += Z[a + (size_t)r * j] * S[a * r + c];
        Uk[j + (size_t)n * c] = s;
      }
  }
}

// randperm(N) on the PERM stream of `epoch` (Fisher–Yates from the top, oracle/philox.py).
void randperm(int N, uint64_t seed, int epoch, std::vector<int32_t>& p) {
  p.resize(N);
  for (int i = 0; i < N; ++i) p[i] = i;
  for (int i = N - 1; i >= 1; --i) {
    const uint32_t x = philox((uint32_t)i, (uint32_t)epoch, kPerm, 0, seed).x;
    std::swap(p[i], p[(int)(((uint64_t)x * (uint64_t)(i + 1)) >> 32)]);
  }
}

struct Cfg {
  int64_t n, D, N, r, Q, m;
  double epsw, epsU, signal_var, sigma_w;
  int64_t burnin, maxepoch, store_every, max_steps;
};

// One chain, GPT_SGLD.jl:345-448 (SGLD + Stiefel).  Returns 0, or 1 on the geodesic NaN bail-out
// (stores zero-filled as :422-424).  w_out/U_out: the final state; stores may be null.
int run_chain(const Cfg& c, const double* phi, const double* y, const int32_t* I1, uint64_t seed,
              double* w_out, double* U_out, double* w_store, double* U_store, long long* steps) {
  const int n = (int)c.n, D = (int)c.D, N = (int)c.N, r = (int)c.r, Q = (int)c.Q, m = (int)c.m;
  const long long nb = (N + m - 1) / m;
  const long long nstore = (c.maxepoch * nb) / c.store_every;
  const long long total = c.max_steps > 0 ? std::min<long long>(c.max_steps, (c.burnin + c.maxepoch) * nb)
                                          : (c.burnin + c.maxepoch) * nb;
  std::vector<double> w(Q), U((size_t)n * r * D);
  init_state(n, r, D, Q, seed, c.sigma_w, w.data(), U.data());
  std::vector<int32_t> I0((size_t)Q * D);
  for (size_t x = 0; x < I0.size(); ++x) I0[x] = I1[x] - 1;
  std::vector<int32_t> order(N), perm, nxt(N);
  for (int i = 0; i < N; ++i) order[i] = i;
  std::vector<double> temp((size_t)D * r * m), V((size_t)Q * m), fhat(m), res(m), gradw(Q),
      Uphi((size_t)Q * m), A((size_t)r * D * m), gradU((size_t)n * r), mom((size_t)n * r),
      M1((size_t)r * r), T((size_t)2 * r * 2 * r), E, mx, tmp((size_t)n * r);
  long long t = 0;
  for (int epoch = 1; epoch <= c.burnin + c.maxepoch && t < total; ++epoch) {
    randperm(N, seed, epoch - 1, perm);                        // :373-374, cumulative
    for (int i = 0; i < N; ++i) nxt[i] = order[perm[i]];
    order.swap(nxt);
    for (long long batch = 0; batch < nb && t < total; ++batch, ++t) {
      const int start = (int)(batch * m), B = std::min(m, N - start);
      const int32_t* idx = order.data() + start;
      // phidotU (:193-205): temp[k,l,i]
      for (int i = 0; i < B; ++i)
        for (int k = 0; k < D; ++k) {
          const double* pk = phi + (size_t)n * (k + (size_t)D * idx[i]);
          for (int l = 0; l < r; ++l) {
            const double* ul = U.data() + (size_t)n * (l + (size_t)r * k);
            double s = 0.0;
#pragma omp simd reduction(+ : s)
            for (int j = 0; j < n; ++j) s += pk[j] * ul[j];     // dot (a BLAS ddot in Julia)
            temp[k + (size_t)D * (l + (size_t)r * i)] = s;
          }
        }
      // computeV (:208-220), computefhat (:223-230)
      for (int i = 0; i < B; ++i) {
        double f = 0.0;
        for (int q = 0; q < Q; ++q) {
          double v = 1.0;
          for (int k = 0; k < D; ++k) v *= temp[k + (size_t)D * (I0[q + (size_t)Q * k] + (size_t)r * i)];
          V[q + (size_t)Q * i] = v;
          f += v * w[q];
        }
        fhat[i] = f;
        res[i] = y[idx[i]] - f;
      }
      // gradw (:393)
      const double cN = (double)N / (double)B;
      for (int q = 0; q < Q; ++q) {
        double s = 0.0;
        for (int i = 0; i < B; ++i) s += V[q + (size_t)Q * i] * res[i];
        gradw[q] = cN * s / c.signal_var - w[q] / (c.sigma_w * c.sigma_w);
      }
      // computeU_phi (:246-258) and computeA (:261-273), dimension by dimension
      std::fill(A.begin(), A.end(), 0.0);
      for (int k = 0; k < D; ++k) {
        for (int i = 0; i < B; ++i)
          for (int q = 0; q < Q; ++q)
            Uphi[q + (size_t)Q * i] =
                V[q + (size_t)Q * i] / temp[k + (size_t)D * (I0[q + (size_t)Q * k] + (size_t)r * i)];
        for (int i = 0; i < B; ++i)
          for (int q = 0; q < Q; ++q)
            A[I0[q + (size_t)Q * k] + (size_t)r * (k + (size_t)D * i)] += Uphi[q + (size_t)Q * i] * w[q];
      }
      // w update (:411-414): the old w formed A above
      const double sqw = std::sqrt(c.epsw);
      for (int q = 0; q < Q; q += 2) {
        double z0, z1;
        normal_pair(seed, (uint32_t)(q >> 1), (uint32_t)t, kWNoise, 0, z0, z1);
        w[q] += c.epsw * gradw[q] / 2 + sqw * z0;
        if (q + 1 < Q) w[q + 1] += c.epsw * gradw[q + 1] / 2 + sqw * z1;
      }
      const double cU = cN / c.signal_var, sq = std::sqrt(c.epsU);
      for (int k = 0; k < D; ++k) {
        // gradU_k = reshape((N/B)·Psi_k·res/σ², n, r), Psi_k[:,i] = kron(A[:,k,i], phi[:,k,i])
        std::fill(gradU.begin(), gradU.end(), 0.0);
        for (int i = 0; i < B; ++i) {
          const double* pk = phi + (size_t)n * (k + (size_t)D * idx[i]);
          for (int l = 0; l < r; ++l) {
            const double a = A[l + (size_t)r * (k + (size_t)D * i)] * res[i];
            double* g = gradU.data() + (size_t)n * l;
            for (int j = 0; j < n; ++j) g[j] += pk[j] * a;
          }
        }
        double* Uk = U.data() + (size_t)n * r * k;
        // drive = √εU·gradU/2 + ζ (:420), ζ on the quad contract of (t, U_NOISE, k)
        unoise_quads(n, r, seed, (uint32_t)t, kUNoise, (uint32_t)k, mom.data());
        for (size_t e = 0; e < (size_t)n * r; ++e) mom[e] = sq * (cU * gradU[e]) / 2 + mom[e];
        // proj (:14-16): mom − U(Uᵀmom + momᵀU)/2
        for (int a = 0; a < r; ++a)
          for (int b = 0; b < r; ++b) {
            double s = 0.0;
#pragma omp simd reduction(+ : s)
            for (int j = 0; j < n; ++j) s += Uk[j + (size_t)n * a] * mom[j + (size_t)n * b];
            M1[a + (size_t)r * b] = s;
          }
        for (int j = 0; j < n; ++j)
          for (int b = 0; b < r; ++b) {
            double s = 0.0;
            for (int a = 0; a < r; ++a) s += Uk[j + (size_t)n * a] * (M1[a + (size_t)r * b] + M1[b + (size_t)r * a]);
            tmp[j + (size_t)n * b] = mom[j + (size_t)n * b] - s / 2;
          }
        mom.swap(tmp);
        // geod (:19-37): A = Uᵀmom, S = momᵀmom, E = expm(t[A −S; I A]), expm(−tA)
        const int p = 2 * r;
        std::vector<double> Ag((size_t)r * r), Sg((size_t)r * r);
        for (int a = 0; a < r; ++a)
          for (int b = 0; b < r; ++b) {
            double s0 = 0.0, s1 = 0.0;
#pragma omp simd reduction(+ : s0, s1)
            for (int j = 0; j < n; ++j) {
              s0 += Uk[j + (size_t)n * a] * mom[j + (size_t)n * b];
              s1 += mom[j + (size_t)n * a] * mom[j + (size_t)n * b];
            }
            Ag[a + (size_t)r * b] = s0; Sg[a + (size_t)r * b] = s1;
          }
        for (int a = 0; a < p; ++a)
          for (int b = 0; b < p; ++b) {
            double v;
            if (a < r) v = b < r ? Ag[a + r * b] : -Sg[a + r * (b - r)];
            else v = b < r ? (a - r == b ? 1.0 : 0.0) : Ag[(a - r) + r * (b - r)];
            T[a + (size_t)p * b] = sq * v;
          }
        // :23-26: only E is checked (a NaN in expm(−tA) reaches U and bails out the next step)
        const bool ok = expm(p, T.data(), E);
        std::vector<double> mA((size_t)r * r);
        for (size_t x = 0; x < mA.size(); ++x) mA[x] = -sq * Ag[x];
        if (ok) (void)expm(r, mA.data(), mx);
        if (!ok) {
          if (w_store) std::memset(w_store, 0, sizeof(double) * Q * nstore);
          if (U_store) std::memset(U_store, 0, sizeof(double) * (size_t)n * r * D * nstore);
          *steps = t + 1;
          return 1;
        }
        // tmpU = [U mom]·E[:,1:r]·expm(−tA), then unit columns
        for (int j = 0; j < n; ++j) {
          double z[64];
          for (int b = 0; b < r; ++b) {
            double s = 0.0;
            for (int a = 0; a < r; ++a) s += Uk[j + (size_t)n * a] * E[a + (size_t)p * b];
            for (int a = 0; a < r; ++a) s += mom[j + (size_t)n * a] * E[r + a + (size_t)p * b];
            z[b] = s;
          }
          for (int b = 0; b < r; ++b) {
            double s = 0.0;
            for (int a = 0; a < r; ++a) s += z[a] * mx[a + (size_t)r * b];
            tmp[j + (size_t)n * b] = s;
          }
        }
        for (int b = 0; b < r; ++b) {
          double s = 0.0;
          for (int j = 0; j < n; ++j) s += tmp[j + (size_t)n * b] * tmp[j + (size_t)n * b];
          const double nrm = std::sqrt(s);
          for (int j = 0; j < n; ++j) Uk[j + (size_t)n * b] = tmp[j + (size_t)n * b] / nrm;
        }
      }
      if (epoch > c.burnin) {                                      // :441-444
        const long long s = (epoch - c.burnin - 1) * nb + batch;
        if ((s + 1) % c.store_every == 0) {
          const long long slot = (s + 1) / c.store_every - 1;
          if (w_store) std::memcpy(w_store + (size_t)slot * Q, w.data(), sizeof(double) * Q);
          if (U_store) std::memcpy(U_store + (size_t)slot * n * r * D, U.data(), sizeof(double) * U.size());
        }
      }
    }
  }
  if (w_out) std::memcpy(w_out, w.data(), sizeof(double) * Q);
  if (U_out) std::memcpy(U_out, U.data(), sizeof(double) * U.size());
  *steps = t;
  return 0;
}

}  // namespace

extern "C" {

// GPTregression (GPT_SGLD.jl:345-448) for `nchains` independent chains (seeds[c]) on `threads`
// OpenMP threads, one chain per thread at a time.  cfg = {n, D, N, r, Q, m, burnin, maxepoch,
// store_every, max_steps} as int64 and {epsw, epsU, signal_var, sigma_w} as double.  w_out
// (Q, nchains), U_out (n·r·D, nchains) final states; w_store / U_store (nullable) chain 0's stores
// in the reference's layout; status[c]: 0 or 1 (geodesic NaN); chain_steps[c] (nullable): the steps
// chain c took (a bailed chain counts its bail-out step).  *seconds: wall time of the chain loop;
// returns the total number of steps taken.
long long gptcpu_regression(const int64_t* icfg, const double* dcfg, const double* phi,
                            const double* y, const int32_t* I, int nchains, const uint64_t* seeds,
                            int threads, double* w_out, double* U_out, double* w_store,
                            double* U_store, int32_t* status, double* seconds,
                            int64_t* chain_steps) {
  Cfg c;
  c.n = icfg[0]; c.D = icfg[1]; c.N = icfg[2]; c.r = icfg[3]; c.Q = icfg[4]; c.m = icfg[5];
  c.burnin = icfg[6]; c.maxepoch = icfg[7]; c.store_every = icfg[8]; c.max_steps = icfg[9];
  c.epsw = dcfg[0]; c.epsU = dcfg[1]; c.signal_var = dcfg[2]; c.sigma_w = dcfg[3];
  if (c.r > 32 || c.r < 1 || c.store_every < 1) return -1;
  const size_t nrD = (size_t)c.n * c.r * c.D;
  long long total = 0;
  const auto t0 = std::chrono::steady_clock::now();
#ifdef _OPENMP
  if (threads < 1) threads = omp_get_max_threads();
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(+ : total)
#endif
  for (int ch = 0; ch < nchains; ++ch) {
    long long st = 0;
    const int rc = run_chain(c, phi, y, I, seeds[ch], w_out ? w_out + (size_t)ch * c.Q : nullptr,
                             U_out ? U_out + (size_t)ch * nrD : nullptr, ch == 0 ? w_store : nullptr,
                             ch == 0 ? U_store : nullptr, &st);
    if (status) status[ch] = rc;
    if (chain_steps) chain_steps[ch] = st;
    total += st;
  }
  *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return total;
}

// pred (GPT_SGLD.jl:233-243) for S samples over Ntest rows: fhat[s·Ntest + i] =
// Σ_q w_s[q]·Π_k temp[k, I[q,k], i], temp = phidotU(U_s, phitest) (:193-205, :208-230), with
// phitest in the reference layout (n, D, Ntest), w (Q, S), U (n·r·D, S).  OpenMP over test
// rows; *seconds: wall time.  The CPU side of the stacked-sample prediction (BASELINE.md:34).
void gptcpu_pred(int64_t n, int64_t D, int64_t Ntest, int64_t r, int64_t Q, int64_t S,
                 const double* phitest, const double* w, const double* U, const int32_t* I,
                 int threads, double* fhat, double* seconds) {
  const auto t0 = std::chrono::steady_clock::now();
  const size_t nrD = (size_t)n * r * D;
#ifdef _OPENMP
  if (threads < 1) threads = omp_get_max_threads();
#pragma omp parallel num_threads(threads)
#endif
  {
    std::vector<double> temp((size_t)D * r);
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
    for (long long i = 0; i < Ntest; ++i)
      for (int64_t s = 0; s < S; ++s) {
        const double* Us = U + (size_t)s * nrD;
        for (int64_t k = 0; k < D; ++k) {
          const double* pk = phitest + (size_t)n * (k + (size_t)D * i);
          for (int64_t l = 0; l < r; ++l) {
            const double* ul = Us + (size_t)n * (l + (size_t)r * k);
            double a = 0.0;
#pragma omp simd reduction(+ : a)
            for (int64_t j = 0; j < n; ++j) a += pk[j] * ul[j];
            temp[k + (size_t)D * l] = a;
          }
        }
        double f = 0.0;
        for (int64_t q = 0; q < Q; ++q) {
          double v = 1.0;
          for (int64_t k = 0; k < D; ++k) v *= temp[k + (size_t)D * (I[q + (size_t)Q * k] - 1)];
          f += v * w[q + (size_t)Q * s];
        }
        fhat[(size_t)s * Ntest + i] = f;
      }
  }
  *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int gptcpu_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

}  // extern "C"
