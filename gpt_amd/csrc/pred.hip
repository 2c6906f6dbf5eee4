// Test-set prediction and RMSE reductions (GPT_SGLD.jl:233-243; GPT_SGLD_p.jl:124-132;
// kin40kExperiment.jl:78-87).
#include "device_util.h"

namespace gpt {

// fhat[s*Ntest + i] = pred(w_s, U_s, I, phitest)[i] for a 64-column tile × one sample.
template <int R>
__global__ __launch_bounds__(kNT) void pred_kernel(const double* __restrict__ w,
                                                   const double* __restrict__ U,
                                                   const int32_t* __restrict__ I0,
                                                   const double* __restrict__ phitest, int n,
                                                   int D, long long Ntest, int Q,
                                                   double* __restrict__ fhat) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int MP = 65;
  const int NP = ((n + 63) / 64) * 64, NS = NP + 1;
  size_t o = 0;
  double* temp_l = (double*)(smem + o); o = al16(o + 8 * (size_t)D * R * MP);
  int* I_l = (int*)(smem + o);          o = al16(o + 4 * (size_t)Q * D);
  double* w_l = (double*)(smem + o);    o = al16(o + 8 * (size_t)Q);
  int* idx_l = (int*)(smem + o);        o = al16(o + 4 * 64);
  double* U_l = (double*)(smem + o);
  const int tid = threadIdx.x;
  const int s = blockIdx.y;
  const long long i0 = (long long)blockIdx.x * 64;
  const int Bt = (int)min((long long)64, Ntest - i0);
  const double* ws = w + (size_t)s * Q;
  const double* Us = U + (size_t)s * n * R * D;
  for (int x = tid; x < Q * D; x += kNT) I_l[x] = I0[x];     // transposed: kk*Q + q
  for (int q = tid; q < Q; q += kNT) w_l[q] = ws[q];
  for (int i = tid; i < 64; i += kNT) idx_l[i] = (int)(i0 + min(i, Bt - 1));
  for (int kk = 0; kk < D; ++kk) {
    __syncthreads();
    const double* Uk = Us + (size_t)n * R * kk;
    for (int x = tid; x < R * NP; x += kNT) {
      const int l = x / NP, j = x - l * NP;
      U_l[l * NS + j] = j < n ? Uk[j + (size_t)n * l] : 0.0;
    }
    __syncthreads();
    phidotU_tile<R>(phitest, (long long)n * kk, (long long)n * D, nullptr, (int)i0, Bt, n, NP, NS,
                    U_l,
                    [&](int l, int i, double v) { temp_l[(kk * R + l) * MP + i] = v; });
  }
  __syncthreads();
  vphase_tile<R, VCfg<R>::ICV_MAX>(temp_l, MP, I_l, w_l, Q, D, 0, Bt, [&](int comp, int i, double v) {
    if (comp == 0) fhat[(size_t)s * Ntest + i0 + i] = v;
  });
}

size_t pred_lds_bytes(int n, int D, int r, int Q);

// phidotU_tile with the feature rows formed on the fly, in feature_kernel's arithmetic (the same
// doubles as a materialised phi): temp[l][i] = Σ_j c·cos(X[i0+i, k]·zt[j] + bj[j]) · U_l[l][j],
// zt = Z[:,k]·(1/ls[k]) and bj = b[:,k] staged (zero-padded to NP) in LDS.
template <int R, class Out>
__device__ __forceinline__ void featdotU_tile(const double* __restrict__ Xk, double c,
                                              const double* zt, const double* bj, long long rowbase,
                                              int Bt, int NP, int NS, const double* U_l, Out out) {
  using Cf = RCfg<R>;
  const int lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6);
  constexpr int SH = 6 - Butterfly<Cf::NV>::P;
  for (int base = 0; base < Bt; base += kNW * Cf::ICH) {
    double v[Cf::NV];
#pragma unroll
    for (int u = 0; u < Cf::NV; ++u) v[u] = 0.0;
    double xv[Cf::ICH];
#pragma unroll
    for (int ii = 0; ii < Cf::ICH; ++ii)
      xv[ii] = gptr(Xk)[rowbase + min(base + wv + kNW * ii, Bt - 1)];
    const int JS = NP >> 6;
#pragma unroll 2
    for (int s2 = 0; s2 < JS; ++s2) {
      const int j = lane + 64 * s2;
      const double z = zt[j], bb = bj[j];
      double u[R];
#pragma unroll
      for (int l = 0; l < R; ++l) u[l] = U_l[l * NS + j];
#pragma unroll
      for (int ii = 0; ii < Cf::ICH; ++ii) {
        const double p = c * cos(__dadd_rn(__dmul_rn(xv[ii], z), bb));
#pragma unroll
        for (int l = 0; l < R; ++l) v[ii * R + l] = fma(p, u[l], v[ii * R + l]);
      }
    }
    Butterfly<Cf::NV>::run(v, lane);
    const int vi = lane >> SH;
    if ((lane & ((1 << SH) - 1)) == 0 && vi < Cf::NVR) {
      const int ii = vi / R, l = vi - (vi / R) * R;
      const int i = base + wv + kNW * ii;
      if (i < Bt) out(l, i, v[0]);
    }
  }
}

// pred_kernel over features formed from Xtest (N × D column-major) instead of a stored phitest.
template <int R>
__global__ __launch_bounds__(kNT) void pred_x_kernel(const double* __restrict__ w,
                                                     const double* __restrict__ U,
                                                     const int32_t* __restrict__ I0,
                                                     const double* __restrict__ X,
                                                     const double* __restrict__ ls,
                                                     const double* __restrict__ Z,
                                                     const double* __restrict__ bfe, double c,
                                                     int n, int D, long long Ntest, int Q,
                                                     double* __restrict__ fhat) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int MP = 65;
  const int NP = ((n + 63) / 64) * 64, NS = NP + 1;
  size_t o = 0;
  double* temp_l = (double*)(smem + o); o = al16(o + 8 * (size_t)D * R * MP);
  int* I_l = (int*)(smem + o);          o = al16(o + 4 * (size_t)Q * D);
  double* w_l = (double*)(smem + o);    o = al16(o + 8 * (size_t)Q);
  double* zt_l = (double*)(smem + o);   o = al16(o + 8 * (size_t)NP);
  double* bj_l = (double*)(smem + o);   o = al16(o + 8 * (size_t)NP);
  double* U_l = (double*)(smem + o);
  const int tid = threadIdx.x;
  const int s = blockIdx.y;
  const long long i0 = (long long)blockIdx.x * 64;
  const int Bt = (int)min((long long)64, Ntest - i0);
  const double* ws = w + (size_t)s * Q;
  const double* Us = U + (size_t)s * n * R * D;
  for (int x = tid; x < Q * D; x += kNT) I_l[x] = I0[x];
  for (int q = tid; q < Q; q += kNT) w_l[q] = ws[q];
  for (int kk = 0; kk < D; ++kk) {
    __syncthreads();
    const double* Uk = Us + (size_t)n * R * kk;
    for (int x = tid; x < R * NP; x += kNT) {
      const int l = x / NP, j = x - l * NP;
      U_l[l * NS + j] = j < n ? Uk[j + (size_t)n * l] : 0.0;
    }
    const double ils = 1.0 / ls[kk];
    for (int j = tid; j < NP; j += kNT) {
      zt_l[j] = j < n ? __dmul_rn(Z[j + (size_t)n * kk], ils) : 0.0;
      bj_l[j] = j < n ? bfe[j + (size_t)n * kk] : 0.0;
    }
    __syncthreads();
    featdotU_tile<R>(X + (size_t)Ntest * kk, c, zt_l, bj_l, i0, Bt, NP, NS, U_l,
                     [&](int l, int i, double v) { temp_l[(kk * R + l) * MP + i] = v; });
  }
  __syncthreads();
  vphase_tile<R, VCfg<R>::ICV_MAX>(temp_l, MP, I_l, w_l, Q, D, 0, Bt, [&](int comp, int i, double v) {
    if (comp == 0) fhat[(size_t)s * Ntest + i0 + i] = v;
  });
}

size_t pred_x_lds_bytes(int n, int D, int r, int Q) {
  return pred_lds_bytes(n, D, r, Q) + 2 * al16(8 * (size_t)(((n + 63) / 64) * 64));
}

size_t pred_lds_bytes(int n, int D, int r, int Q) {
  size_t o = 0;
  o = al16(o + 8 * (size_t)D * r * 65);
  o = al16(o + 4 * (size_t)Q * D);
  o = al16(o + 8 * (size_t)Q);
  o = al16(o + 4 * 64);
  o = al16(o + 8 * (size_t)r * (((n + 63) / 64) * 64 + 1));
  return o;
}

// mean_out[i] = (1/S) Σ_s fhat[s,i];  sse_out[0] = Σ_i (ytest_i − mean_i)²;
// sse_out[1+s] = Σ_i (ytest_i − fhat[s,i])²   (per-sample test error for testRMSE curves)
__global__ __launch_bounds__(kNT) void mean_sse_kernel(const double* __restrict__ fhat,
                                                       const double* __restrict__ ytest,
                                                       long long Ntest, int S,
                                                       double* __restrict__ mean_out,
                                                       double* __restrict__ sse_out) {
  __shared__ double red[kNW];
  const int s = blockIdx.x;  // block 0..S-1: per-sample SSE; block S: posterior mean
  double acc = 0.0;
  if (s < S) {
    const double* f = fhat + (size_t)s * Ntest;
    for (long long i = threadIdx.x; i < Ntest; i += kNT) {
      const double d = ytest[i] - f[i];
      acc = fma(d, d, acc);
    }
  } else {
    for (long long i = threadIdx.x; i < Ntest; i += kNT) {
      double m = 0.0;
      for (int z = 0; z < S; ++z) m += fhat[(size_t)z * Ntest + i];
      m /= S;
      if (mean_out) mean_out[i] = m;
      const double d = ytest[i] - m;
      acc = fma(d, d, acc);
    }
  }
  const double tot = blk_sum(acc, red);
  if (threadIdx.x == 0) sse_out[s < S ? 1 + s : 0] = tot;
}

#define GPT_RANKS(X) X(1) X(2) X(3) X(4) X(5) X(6) X(8) X(10) X(12) X(15) X(16) X(20)

hipError_t launch_pred(const double* w, const double* U, const int32_t* I0, const double* phitest,
                       int n, int D, long long Ntest, int r, int Q, int S, double* fhat,
                       hipStream_t st) {
  if (Ntest <= 0 || S <= 0) return hipSuccess;
  const size_t lds = pred_lds_bytes(n, D, r, Q);
  dim3 grid((unsigned)((Ntest + 63) / 64), S);
  switch (r) {
#define CASE(RR)                                                                             \
  case RR: {                                                                                 \
    static bool attr = false;                                                                \
    if (!attr) {                                                                             \
      hipError_t e = hipFuncSetAttribute((const void*)pred_kernel<RR>,                        \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
      if (e != hipSuccess) return e;                                                         \
      attr = true;                                                                           \
    }                                                                                        \
    hipLaunchKernelGGL(pred_kernel<RR>, grid, dim3(kNT), lds, st, w, U, I0, phitest, n, D,   \
                       Ntest, Q, fhat);                                                      \
  } break;
    GPT_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_pred_x(const double* w, const double* U, const int32_t* I0, const double* X,
                         const double* ls, const double* Z, const double* bfe, double c, int n,
                         int D, long long Ntest, int r, int Q, int S, double* fhat,
                         hipStream_t st) {
  if (Ntest <= 0 || S <= 0) return hipSuccess;
  const size_t lds = pred_x_lds_bytes(n, D, r, Q);
  dim3 grid((unsigned)((Ntest + 63) / 64), S);
  switch (r) {
#define CASE(RR)                                                                             \
  case RR: {                                                                                 \
    static bool attr = false;                                                                \
    if (!attr) {                                                                             \
      hipError_t e = hipFuncSetAttribute((const void*)pred_x_kernel<RR>,                      \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
      if (e != hipSuccess) return e;                                                         \
      attr = true;                                                                           \
    }                                                                                        \
    hipLaunchKernelGGL(pred_x_kernel<RR>, grid, dim3(kNT), lds, st, w, U, I0, X, ls, Z, bfe, c, \
                       n, D, Ntest, Q, fhat);                                                \
  } break;
    GPT_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_mean_rmse(const double* fhat, const double* ytest, long long Ntest, int S,
                            double* mean_out, double* sse_out, hipStream_t st) {
  hipLaunchKernelGGL(mean_sse_kernel, dim3(S + 1), dim3(kNT), 0, st, fhat, ytest, Ntest, S,
                     mean_out, sse_out);
  return hipGetLastError();
}

}  // namespace gpt
