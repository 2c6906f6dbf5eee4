// Device building blocks shared by the step, prediction and init kernels (gfx950, wave64).
#pragma once
#include "gpt_internal.h"

namespace gpt {

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// Order LDS traffic between the lanes of ONE wave (no workgroup barrier).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

// Sum of one value per thread over the workgroup; every thread gets the total.
// Uses red[0..kNW); deterministic order.
__device__ __forceinline__ double blk_sum(double v, double* red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < kNW; ++w) s += red[w];
  __syncthreads();
  return s;
}

// Butterfly "transpose-reduce" across the 64 lanes of a wave: each lane starts with NV
// partial values; afterwards lane λ holds in v[0] the wave total of value (λ >> (6-P)),
// P = log2(NV).  Costs NV-1 exchanged doubles per lane instead of NV·6 for NV separate
// wave reductions.
template <int NV>
struct Butterfly {
  static constexpr int P = NV == 8 ? 3 : (NV == 16 ? 4 : (NV == 32 ? 5 : 6));
  // One halving round at a compile-time stage S (keeps every index static: no scratch).
  template <int S>
  __device__ __forceinline__ static void round(double (&v)[NV], int lane) {
    if constexpr (S < P) {
      constexpr int off = 32 >> S;
      constexpr int h = NV >> (S + 1);
      const bool up = (lane & off) != 0;
#pragma unroll
      for (int u = 0; u < h; ++u) {
        const double send = up ? v[u] : v[u + h];
        const double keep = up ? v[u + h] : v[u];
        v[u] = keep + __shfl_xor(send, off, 64);
      }
      round<S + 1>(v, lane);
    } else if constexpr (S < 6) {
      v[0] += __shfl_xor(v[0], 32 >> S, 64);
      round<S + 1>(v, lane);
    }
  }
  __device__ __forceinline__ static void run(double (&v)[NV], int lane) { round<0>(v, lane); }
};

template <int R>
struct RCfg {
  static constexpr int ICH = (64 / R) < 8 ? (64 / R) : 8;   // batch columns per wave pass
  static constexpr int NVR = ICH * R;
  static constexpr int NV = NVR <= 8 ? 8 : (NVR <= 16 ? 16 : (NVR <= 32 ? 32 : 64));
};

// temp[l][i] = Σ_j phi[koff + row(i)*rstride + j] · U_l[l*NP + j]   (GPT_SGLD.jl:193-205)
// for i < Bt, row(i) = idx_l[i].  Lanes stride over j (coalesced 512-B loads), wave w takes
// columns i = base + w + kNW·ii; partials are combined with one Butterfly per pass.
// U_l rows must be zero-padded for j in [n, NP).
template <int R, class Out>
__device__ __forceinline__ void phidotU_tile(const double* __restrict__ phi, long long koff,
                                             long long rstride, const int* idx_l, int Bt,
                                             int n, int NP, const double* U_l, Out out) {
  using C = RCfg<R>;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int SH = 6 - Butterfly<C::NV>::P;
  for (int base = 0; base < Bt; base += kNW * C::ICH) {
    double v[C::NV];
#pragma unroll
    for (int u = 0; u < C::NV; ++u) v[u] = 0.0;
    const double* rowp[C::ICH];
#pragma unroll
    for (int ii = 0; ii < C::ICH; ++ii) {
      const int i = min(base + wv + kNW * ii, Bt - 1);
      rowp[ii] = phi + koff + (long long)uni(idx_l[i]) * rstride;
    }
    const int JS = NP >> 6;
#pragma unroll 2
    for (int s = 0; s < JS; ++s) {
      const int j = lane + 64 * s;
      const int jc = min(j, n - 1);
      double p[C::ICH];
#pragma unroll
      for (int ii = 0; ii < C::ICH; ++ii) p[ii] = rowp[ii][jc];
      double u[R];
#pragma unroll
      for (int l = 0; l < R; ++l) u[l] = U_l[l * NP + j];
#pragma unroll
      for (int ii = 0; ii < C::ICH; ++ii)
#pragma unroll
        for (int l = 0; l < R; ++l) v[ii * R + l] = fma(p[ii], u[l], v[ii * R + l]);
    }
    Butterfly<C::NV>::run(v, lane);
    const int vi = lane >> SH;
    if ((lane & ((1 << SH) - 1)) == 0 && vi < C::NVR) {
      const int ii = vi / R, l = vi - (vi / R) * R;
      const int i = base + wv + kNW * ii;
      if (i < Bt) out(l, i, v[0]);
    }
  }
}

// V-phase partials for columns [ic, ic+64) (lane = column): over q = wave, wave+kNW, …
//   V[q,i]  = Π_k temp[k, I[q,k], i]                 (GPT_SGLD.jl:208-220, same k order)
//   fh     += w[q]·V[q,i]                            (:223-230)
//   a[l]   += w[q]·Π_{k'≠kown} temp[k', I[q,k'], i]  for l = I[q,kown]   (:246-273, no division)
// writes red[(wave*(1+R) + comp)*64 + lane]; comp 0 = fh, 1+l = a[l].
template <int R>
__device__ __forceinline__ void vphase_partials(const double* temp_l, int MP, const int* I_l,
                                                const double* w_l, int Q, int D, int kown,
                                                int ic, int Bt, double* red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = min(ic + lane, Bt - 1);
  double fh = 0.0;
  double a[R];
#pragma unroll
  for (int l = 0; l < R; ++l) a[l] = 0.0;
  for (int q = wv; q < Q; q += kNW) {
    const int* Iq = I_l + q * D;
    double v = 1.0, vk = 1.0;
#pragma unroll
    for (int kk = 0; kk < kDMax; ++kk) {
      if (kk < D) {
        const double tv = temp_l[(kk * R + uni(Iq[kk])) * MP + i];
        v *= tv;
        if (kk != kown) vk *= tv;
      }
    }
    const double wq = w_l[q];
    fh = fma(wq, v, fh);
    if (kown >= 0) {
      const int lk = uni(Iq[kown]);
      const double cc = wq * vk;
#pragma unroll
      for (int l = 0; l < R; ++l)
        if (l == lk) a[l] += cc;
    }
  }
  red[(wv * (1 + R)) * 64 + lane] = fh;
  if (kown >= 0) {
#pragma unroll
    for (int l = 0; l < R; ++l) red[(wv * (1 + R) + 1 + l) * 64 + lane] = a[l];
  }
}

// Gram products over j < n of LDS rows (stride NP), lanes = outputs, waves = j slices.
//  mode 0: out[a*R+b] = Σ_j X[a][j]·Y[b][j]                      (R² outputs)
//  mode 1: out[a*R+b] = Σ X[a]Y[b];  out[R²+a*R+b] = Σ Y[a]Y[b]   (2R² outputs)
//  mode 2: out[l] = Σ_j X[l][j]²                                   (R outputs)
template <int R>
__device__ __forceinline__ void blk_gram(const double* X, const double* Y, int NP, int n,
                                         int mode, double* out, double* red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nout = mode == 0 ? R * R : (mode == 1 ? 2 * R * R : R);
  const int chunk = (n + kNW - 1) / kNW;
  const int j0 = wv * chunk, j1 = min(n, j0 + chunk);
  for (int o = lane; o < nout; o += 64) {
    const double* xa;
    const double* yb;
    if (mode == 2) { xa = X + o * NP; yb = xa; }
    else {
      const int oo = o < R * R ? o : o - R * R;
      const int a = oo / R, b = oo - a * R;
      xa = (o < R * R ? X : Y) + a * NP;
      yb = Y + b * NP;
    }
    double s = 0.0;
    for (int j = j0; j < j1; ++j) s = fma(xa[j], yb[j], s);
    red[wv * nout + o] = s;
  }
  __syncthreads();
  for (int o = threadIdx.x; o < nout; o += kNT) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kNW; ++w) s += red[w * nout + o];
    out[o] = s;
  }
  __syncthreads();
}

// ---------------------------------------------------------------- small dense algebra (1 wave)
__device__ __forceinline__ void wave_mm(const double* A, const double* B, double* C, int nn) {
  const int lane = threadIdx.x & 63;
  for (int o = lane; o < nn * nn; o += 64) {
    const int i = o / nn, j = o - i * nn;
    double s = 0.0;
    for (int t = 0; t < nn; ++t) s = fma(A[i * nn + t], B[t * nn + j], s);
    C[o] = s;
  }
  wave_sync();
}

// Solve M·X = X0 in place (X holds X0 on entry), partial pivoting (LAPACK gesv semantics:
// largest |pivot|, first index on ties, multipliers scaled by 1/pivot).
__device__ __forceinline__ void wave_solve(double* M, double* X, int nn) {
  const int lane = threadIdx.x & 63;
  for (int c = 0; c < nn; ++c) {
    double best = -1.0;
    int bi = c;
    if (lane >= c && lane < nn) { best = fabs(M[lane * nn + c]); bi = lane; }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double ob = __shfl_xor(best, off, 64);
      const int oi = __shfl_xor(bi, off, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    bi = uni(bi);
    if (bi != c) {
      for (int col = lane; col < nn; col += 64) {
        double t0 = M[c * nn + col]; M[c * nn + col] = M[bi * nn + col]; M[bi * nn + col] = t0;
        double t1 = X[c * nn + col]; X[c * nn + col] = X[bi * nn + col]; X[bi * nn + col] = t1;
      }
      wave_sync();
    }
    const double rp = 1.0 / M[c * nn + c];
    const int rows = nn - c - 1;
    // row updates: M[row][col>c] and X[row][*]
    const int wcols = (nn - c - 1) + nn;
    for (int o = lane; o < rows * wcols; o += 64) {
      const int rr = c + 1 + o / wcols, cc = o - (o / wcols) * wcols;
      const double f = M[rr * nn + c] * rp;
      if (cc < nn - c - 1) {
        const int col = c + 1 + cc;
        M[rr * nn + col] -= f * M[c * nn + col];
      } else {
        const int col = cc - (nn - c - 1);
        X[rr * nn + col] -= f * X[c * nn + col];
      }
    }
    wave_sync();
  }
  for (int c = nn - 1; c >= 0; --c) {
    for (int col = lane; col < nn; col += 64) {
      double s = X[c * nn + col];
      for (int t = c + 1; t < nn; ++t) s -= M[c * nn + t] * X[t * nn + col];
      X[c * nn + col] = s / M[c * nn + c];
    }
    wave_sync();
  }
}

// X = expm(A) for an nn×nn matrix held in S[0..nn²) (row-major; overwritten).  Padé
// scaling-and-squaring of Julia Base 0.3 expm! (Higham 2005; thresholds 0.015/0.25/0.95/2.1,
// 13th order above, θ13 = 5.4).  Scratch S: 8 nn² doubles; result at S + 8 nn².
// Returns true if the result contains a NaN (the geod bail-out of GPT_SGLD.jl:23-26).
__device__ bool wave_expm(double* S, int nn) {
  const int lane = threadIdx.x & 63;
  const int q = nn * nn;
  double* A = S;
  double* A2 = S + q;
  double* A4 = S + 2 * q;
  double* A6 = S + 3 * q;
  double* U = S + 4 * q;
  double* V = S + 5 * q;
  double* T = S + 6 * q;
  double* M = S + 7 * q;
  double* X = S + 8 * q;
  double cs = 0.0;
  if (lane < nn)
    for (int i = 0; i < nn; ++i) cs += fabs(A[i * nn + lane]);
  const double nA = wave_max(cs);
  int si = 0;
  if (nA <= 2.1) {
    double C[10];
    int deg;
    if (nA > 0.95) {
      const double c9[10] = {17643225600.0, 8821612800.0, 2075673600.0, 302702400.0, 30270240.0,
                             2162160.0, 110880.0, 3960.0, 90.0, 1.0};
      for (int z = 0; z < 10; ++z) C[z] = c9[z];
      deg = 9;
    } else if (nA > 0.25) {
      const double c7[8] = {17297280.0, 8648640.0, 1995840.0, 277200.0, 25200.0, 1512.0, 56.0, 1.0};
      for (int z = 0; z < 8; ++z) C[z] = c7[z];
      deg = 7;
    } else if (nA > 0.015) {
      const double c5[6] = {30240.0, 15120.0, 3360.0, 420.0, 30.0, 1.0};
      for (int z = 0; z < 6; ++z) C[z] = c5[z];
      deg = 5;
    } else {
      const double c3[4] = {120.0, 60.0, 12.0, 1.0};
      for (int z = 0; z < 4; ++z) C[z] = c3[z];
      deg = 3;
    }
    wave_mm(A, A, A2, nn);
    for (int o = lane; o < q; o += 64) {
      const double id = (o / nn == o - (o / nn) * nn) ? 1.0 : 0.0;
      T[o] = id;
      U[o] = C[1] * id;
      V[o] = C[0] * id;
    }
    wave_sync();
    for (int kk = 1; kk <= (deg - 1) / 2; ++kk) {
      wave_mm(T, A2, A4, nn);  // P = P·A2  (A4 is free scratch here)
      for (int o = lane; o < q; o += 64) {
        const double p = A4[o];
        T[o] = p;
        U[o] = U[o] + C[2 * kk + 1] * p;
        V[o] = V[o] + C[2 * kk] * p;
      }
      wave_sync();
    }
    wave_mm(A, U, A6, nn);
    for (int o = lane; o < q; o += 64) U[o] = A6[o];
    wave_sync();
  } else {
    const double s = log2(nA / 5.4);
    si = (s > 0.0) ? (s < 60.0 ? (int)ceil(s) : 60) : 0;
    if (!(nA == nA)) si = 0;
    if (si > 0) {
      const double sc = ldexp(1.0, -si);
      for (int o = lane; o < q; o += 64) A[o] *= sc;
      wave_sync();
    }
    const double c[14] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
                          1187353796428800.0, 129060195264000.0, 10559470521600.0,
                          670442572800.0, 33522128640.0, 1323241920.0, 40840800.0, 960960.0,
                          16380.0, 182.0, 1.0};
    wave_mm(A, A, A2, nn);
    wave_mm(A2, A2, A4, nn);
    wave_mm(A2, A4, A6, nn);
    for (int o = lane; o < q; o += 64) T[o] = c[13] * A6[o] + c[11] * A4[o] + c[9] * A2[o];
    wave_sync();
    wave_mm(A6, T, M, nn);
    for (int o = lane; o < q; o += 64) {
      const double id = (o / nn == o - (o / nn) * nn) ? 1.0 : 0.0;
      M[o] = M[o] + c[7] * A6[o] + c[5] * A4[o] + c[3] * A2[o] + c[1] * id;
      T[o] = c[12] * A6[o] + c[10] * A4[o] + c[8] * A2[o];
    }
    wave_sync();
    wave_mm(A, M, U, nn);
    wave_mm(A6, T, V, nn);
    for (int o = lane; o < q; o += 64) {
      const double id = (o / nn == o - (o / nn) * nn) ? 1.0 : 0.0;
      V[o] = V[o] + c[6] * A6[o] + c[4] * A4[o] + c[2] * A2[o] + c[0] * id;
    }
    wave_sync();
  }
  for (int o = lane; o < q; o += 64) {
    M[o] = V[o] - U[o];
    X[o] = V[o] + U[o];
  }
  wave_sync();
  wave_solve(M, X, nn);
  for (int z = 0; z < si; ++z) {
    wave_mm(X, X, T, nn);
    for (int o = lane; o < q; o += 64) X[o] = T[o];
    wave_sync();
  }
  bool bad = false;
  for (int o = lane; o < q; o += 64) bad |= (X[o] != X[o]);
  return __any(bad);
}

}  // namespace gpt
