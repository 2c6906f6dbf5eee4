// Tensor-GP Gibbs sweep (TGP.jl:37-86, `GPT_inf`) for MI355X (gfx950).
//
// A sweep draws W | U from its Gaussian conditional (q × q) and then each U_k | W, U_{-k}
// (nr × nr).  The dense parts are SYRKs with a long inner dimension (K = N samples), done on the
// fp64 matrix cores (v_mfma_f64_16x16x4f64), and Cholesky factorisations / triangular solves of
// the q × q and nr × nr precision matrices, done by one workgroup each (they are small:
// q ≈ 100, nr <= ~1000 in the reference's use, `UnitTest.jl:15-28`).  The feature contractions
// reuse the phidotU tile of the SGLD path.
#include "device_util.h"

namespace gpt {

typedef double d4 __attribute__((ext_vector_type(4)));

// temp[(d·R + l)·N + i] = U_dᵀ b[:, d, i] for d = d0 + blockIdx.y, rows i of a 64-row tile.
template <int R>
__global__ __launch_bounds__(kNT) void tgp_temp_kernel(const double* __restrict__ U,
                                                       const double* __restrict__ b, int n, int D,
                                                       long long N, int d0,
                                                       double* __restrict__ temp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int NP = ((n + 63) / 64) * 64, NS = NP + 1;
  double* U_l = (double*)smem;
  const int tid = threadIdx.x, d = d0 + blockIdx.y;
  const long long i0 = (long long)blockIdx.x * 64;
  const int Bt = (int)min((long long)64, N - i0);
  const double* Ud = U + (size_t)n * R * d;
  for (int x = tid; x < R * NP; x += kNT) {
    const int l = x / NP, j = x - l * NP;
    U_l[l * NS + j] = j < n ? Ud[j + (size_t)n * l] : 0.0;
  }
  __syncthreads();
  phidotU_tile<R>(b, (long long)n * d, (long long)n * D, nullptr, (int)i0, Bt, n, NP, NS, U_l,
                  [&](int l, int i, double v) { temp[((size_t)d * R + l) * N + i0 + i] = v; });
}

// V[q + Q·i] = Π_d temp[(d·R + I0[q + Q·d])·N + i]   (TGP.jl:55, product in d order)
__global__ void tgp_v_kernel(const double* __restrict__ temp, const int32_t* __restrict__ I0,
                             int Q, int D, int R, long long N, double* __restrict__ V) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)Q * N) return;
  const int q = (int)(e % Q);
  const long long i = e / Q;
  double v = 1.0;
  for (int d = 0; d < D; ++d) v *= temp[((size_t)d * R + I0[q + Q * d]) * N + i];
  V[e] = v;
}

// C[l + R·i] = Σ_{q: I[q,k]=l} W_q · V[q,i] / temp[k, I[q,k], i]   (TGP.jl:72-77, q ascending)
__global__ void tgp_c_kernel(const double* __restrict__ V, const double* __restrict__ W,
                             const double* __restrict__ temp, const int32_t* __restrict__ I0,
                             int Q, int R, long long N, int k, double* __restrict__ Cm) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)R * N) return;
  const int l = (int)(e % R);
  const long long i = e / R;
  const double tk = temp[((size_t)k * R + l) * N + i];
  double s = 0.0;
  for (int q = 0; q < Q; ++q)
    if (I0[q + Q * k] == l) s += W[q] * (V[q + (size_t)Q * i] / tk);
  Cm[e] = s;
}

// Ck[(l·n + j) + nr·i] = C[l + R·i] · b[j + n·(k + D·i)]   (TGP.jl:78, Kronecker rows)
__global__ void tgp_ck_kernel(const double* __restrict__ Cm, const double* __restrict__ b, int n,
                              int D, int R, long long N, int k, double* __restrict__ Ck) {
  const long long nr = (long long)n * R;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nr * N) return;
  const long long i = e / nr;
  const int row = (int)(e - i * nr), l = row / n, j = row - l * n;
  Ck[e] = Cm[l + (size_t)R * i] * b[j + (size_t)n * (k + (size_t)D * i)];
}

// V[q,i] = (V[q,i] / told[k, I[q,k], i]) · tnew[I[q,k], i]   (TGP.jl:76, :81)
__global__ void tgp_vupd_kernel(double* __restrict__ V, const double* __restrict__ temp,
                                const double* __restrict__ tnew, const int32_t* __restrict__ I0,
                                int Q, int R, long long N, int k) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)Q * N) return;
  const int q = (int)(e % Q);
  const long long i = e / Q;
  const int l = I0[q + Q * k];
  V[e] = (V[e] / temp[((size_t)k * R + l) * N + i]) * tnew[(size_t)l * N + i];
}

// M (lower 16×16 tiles, column-major p × p) = alpha · A Aᵀ + beta · I, A column-major p × N.
// One wave per tile pair (ta >= tb); fp64 MFMA 16×16×4: lane λ feeds A[ta·16 + (λ&15), k0 + (λ>>4)]
// and A[tb·16 + (λ&15), k0 + (λ>>4)] and receives D[(λ>>4) + 4r, λ&15].
__global__ __launch_bounds__(256) void syrk_mfma_kernel(const double* __restrict__ A, int p,
                                                        long long N, double alpha, double beta,
                                                        double* __restrict__ M) {
  const int lane = threadIdx.x & 63;
  const long long pair = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int T = (p + 15) / 16;
  if (pair >= (long long)T * (T + 1) / 2) return;
  int ta = (int)((sqrt(8.0 * (double)pair + 1.0) - 1.0) / 2.0);
  while ((long long)ta * (ta + 1) / 2 > pair) --ta;
  while ((long long)(ta + 1) * (ta + 2) / 2 <= pair) ++ta;
  const int tb = (int)(pair - (long long)ta * (ta + 1) / 2);
  const int ra = ta * 16 + (lane & 15), rb = tb * 16 + (lane & 15), kl = lane >> 4;
  const bool oka = ra < p, okb = rb < p;
  const double* pa = A + (oka ? ra : 0);
  const double* pb = A + (okb ? rb : 0);
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  long long k0 = 0;
  for (; k0 + 16 <= N; k0 += 16) {
    double av[4], bv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long kk = k0 + 4 * u + kl;
      av[u] = oka ? pa[(size_t)p * kk] : 0.0;
      bv[u] = okb ? pb[(size_t)p * kk] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc, 0, 0, 0);
  }
  for (; k0 < N; k0 += 4) {
    const long long kk = k0 + kl;
    const double av = (oka && kk < N) ? pa[(size_t)p * kk] : 0.0;
    const double bv = (okb && kk < N) ? pb[(size_t)p * kk] : 0.0;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
  }
  const int col = tb * 16 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = ta * 16 + (lane >> 4) + 4 * r;
    if (row < p && col < p) M[row + (size_t)p * col] = alpha * acc[r] + (row == col ? beta : 0.0);
  }
}

// out[a] = alpha · Σ_i A[a + p·i] · y[i]
__global__ void gemv_kernel(const double* __restrict__ A, int p, long long N,
                            const double* __restrict__ y, double alpha, double* __restrict__ out) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= p) return;
  double s = 0.0;
  for (long long i = 0; i < N; ++i) s = fma(A[a + (size_t)p * i], y[i], s);
  out[a] = alpha * s;
}

__global__ void axpy_kernel(double* __restrict__ x, const double* __restrict__ z, int p) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a < p) x[a] += z[a];
}

// z[e] = element e of Philox normal stream (c1, c2, c3)
__global__ void normals_kernel(double* __restrict__ z, int cnt, uint64_t seed, uint32_t c1,
                               uint32_t c2, uint32_t c3) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < cnt) z[e] = normal_at(seed, (uint32_t)e, c1, c2, c3);
}

// In-place lower Cholesky of the SPD matrix M (column-major p × p, lower triangle read), one
// workgroup: right-looking, column by column.  status = 1 if a pivot is not positive.
constexpr int kTgpNT = 1024;
__global__ __launch_bounds__(kTgpNT) void chol_kernel(double* __restrict__ M, int p,
                                                      int32_t* __restrict__ status) {
  __shared__ double piv;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = kTgpNT / 64;
  for (int j = 0; j < p; ++j) {
    if (tid == 0) {
      const double d = M[j + (size_t)p * j];
      if (!(d > 0.0)) *status = 1;
      piv = sqrt(d);
      M[j + (size_t)p * j] = piv;
    }
    __syncthreads();
    const double pv = piv;
    for (int i = j + 1 + tid; i < p; i += kTgpNT) M[i + (size_t)p * j] /= pv;
    __syncthreads();
    for (int c = j + 1 + wv; c < p; c += nw) {
      const double mc = M[c + (size_t)p * j];
      for (int i = c + lane; i < p; i += 64) M[i + (size_t)p * c] -= M[i + (size_t)p * j] * mc;
    }
    __syncthreads();
  }
}

// x := L⁻¹ x (trans = 0) or L⁻ᵀ x (trans = 1), L lower (column-major p × p); one workgroup.
__global__ __launch_bounds__(kTgpNT) void trsv_kernel(const double* __restrict__ L, int p,
                                                      double* __restrict__ x, int trans) {
  __shared__ double xj;
  const int tid = threadIdx.x;
  if (!trans) {
    for (int j = 0; j < p; ++j) {
      if (tid == 0) { xj = x[j] / L[j + (size_t)p * j]; x[j] = xj; }
      __syncthreads();
      const double v = xj;
      for (int i = j + 1 + tid; i < p; i += kTgpNT) x[i] -= L[i + (size_t)p * j] * v;
      __syncthreads();
    }
  } else {
    for (int j = p - 1; j >= 0; --j) {
      if (tid == 0) { xj = x[j] / L[j + (size_t)p * j]; x[j] = xj; }
      __syncthreads();
      const double v = xj;
      for (int i = tid; i < j; i += kTgpNT) x[i] -= L[j + (size_t)p * i] * v;
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------------------ host side
#define GPT_TGP_RANKS(X) X(1) X(2) X(3) X(4) X(5) X(6) X(8) X(10) X(12) X(15) X(16) X(20)

static hipError_t launch_tgp_temp(const double* U, const double* b, int n, int D, long long N,
                                  int r, int d0, int nd, double* temp, hipStream_t st) {
  const size_t lds = 8 * (size_t)r * (((n + 63) / 64) * 64 + 1);
  dim3 grid((unsigned)((N + 63) / 64), nd);
  switch (r) {
#define CASE(RR)                                                                             \
  case RR:                                                                                   \
    hipLaunchKernelGGL(tgp_temp_kernel<RR>, grid, dim3(kNT), lds, st, U, b, n, D, N, d0, temp); \
    break;
    GPT_TGP_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

static unsigned nblk(long long cnt, int t) { return (unsigned)((cnt + t - 1) / t); }

// One Gibbs sweep driver.  All pointers device; W_hist (q × T), U_hist (n·r·D × T).
hipError_t tgp_gibbs(const double* b, const double* y, int n, int D, long long N, int r, int q,
                     double sigma, int iters, int burnin, uint64_t seed, const int32_t* I0,
                     double* U, double* W_hist, double* U_hist, int32_t* status, hipStream_t st) {
  const int nr = n * r, pm = std::max(q, nr);
  const double s2 = sigma * sigma;
  const double sigma_u2 = 1.0 / r, sigma_w2 = std::pow((double)r, (double)D) / q;
  double *temp = nullptr, *V = nullptr, *Cm = nullptr, *Ck = nullptr, *M = nullptr, *x = nullptr,
         *z = nullptr, *W = nullptr, *tnew = nullptr;
  hipError_t e = hipSuccess;
  auto al = [&](double** p, size_t cnt) {
    if (e == hipSuccess) e = hipMallocAsync((void**)p, 8 * (cnt ? cnt : 1), st);
  };
  al(&temp, (size_t)D * r * N); al(&V, (size_t)q * N); al(&Cm, (size_t)r * N);
  al(&Ck, (size_t)nr * N); al(&M, (size_t)pm * pm); al(&x, pm); al(&z, pm); al(&W, q);
  al(&tnew, (size_t)r * N);
  for (int it = 1; it <= iters && e == hipSuccess; ++it) {
    e = launch_tgp_temp(U, b, n, D, N, r, 0, D, temp, st);
    if (e != hipSuccess) break;
    hipLaunchKernelGGL(tgp_v_kernel, nblk((long long)q * N, 256), 256, 0, st, temp, I0, q, D, r, N, V);
    // W | U  (TGP.jl:57-59)
    const int Tq = (q + 15) / 16;
    hipLaunchKernelGGL(syrk_mfma_kernel, nblk((long long)Tq * (Tq + 1) / 2, 4), 256, 0, st, V, q, N,
                       1.0 / s2, 1.0 / sigma_w2, M);
    hipLaunchKernelGGL(gemv_kernel, nblk(q, 256), 256, 0, st, V, q, N, y, 1.0 / s2, x);
    hipLaunchKernelGGL(chol_kernel, 1, kTgpNT, 0, st, M, q, status);
    hipLaunchKernelGGL(trsv_kernel, 1, kTgpNT, 0, st, M, q, x, 0);
    hipLaunchKernelGGL(normals_kernel, nblk(q, 256), 256, 0, st, z, q, seed, (uint32_t)(it - 1),
                       (uint32_t)kTgpWNoise, 0u);
    hipLaunchKernelGGL(axpy_kernel, nblk(q, 256), 256, 0, st, x, z, q);
    hipLaunchKernelGGL(trsv_kernel, 1, kTgpNT, 0, st, M, q, x, 1);   // W = L⁻ᵀ(L⁻¹ rhs + z)
    e = hipMemcpyAsync(W, x, 8 * (size_t)q, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) break;
    if (it > burnin) {
      e = hipMemcpyAsync(W_hist + (size_t)q * (it - burnin - 1), W, 8 * (size_t)q,
                         hipMemcpyDeviceToDevice, st);
      if (e == hipSuccess)
        e = hipMemcpyAsync(U_hist + (size_t)nr * D * (it - burnin - 1), U, 8 * (size_t)nr * D,
                           hipMemcpyDeviceToDevice, st);
      if (e != hipSuccess) break;
    }
    // U_k | W, U_{-k}  (TGP.jl:71-82)
    const int Tu = (nr + 15) / 16;
    for (int k = 0; k < D && e == hipSuccess; ++k) {
      hipLaunchKernelGGL(tgp_c_kernel, nblk((long long)r * N, 256), 256, 0, st, V, W, temp, I0, q, r,
                         N, k, Cm);
      hipLaunchKernelGGL(tgp_ck_kernel, nblk((long long)nr * N, 256), 256, 0, st, Cm, b, n, D, r, N,
                         k, Ck);
      hipLaunchKernelGGL(syrk_mfma_kernel, nblk((long long)Tu * (Tu + 1) / 2, 4), 256, 0, st, Ck, nr,
                         N, 1.0 / s2, 1.0 / sigma_u2, M);
      hipLaunchKernelGGL(gemv_kernel, nblk(nr, 256), 256, 0, st, Ck, nr, N, y, 1.0 / s2, x);
      hipLaunchKernelGGL(normals_kernel, nblk(nr, 256), 256, 0, st, z, nr, seed, (uint32_t)(it - 1),
                         (uint32_t)kTgpUNoise, (uint32_t)k);
      hipLaunchKernelGGL(axpy_kernel, nblk(nr, 256), 256, 0, st, x, z, nr);
      hipLaunchKernelGGL(chol_kernel, 1, kTgpNT, 0, st, M, nr, status);
      hipLaunchKernelGGL(trsv_kernel, 1, kTgpNT, 0, st, M, nr, x, 0);
      hipLaunchKernelGGL(trsv_kernel, 1, kTgpNT, 0, st, M, nr, x, 1);   // U_k = M⁻¹(rhs + z)
      e = hipMemcpyAsync(U + (size_t)nr * k, x, 8 * (size_t)nr, hipMemcpyDeviceToDevice, st);
      if (e != hipSuccess) break;
      e = launch_tgp_temp(U, b, n, D, N, r, k, 1, tnew - (size_t)k * r * N, st);
      if (e != hipSuccess) break;
      hipLaunchKernelGGL(tgp_vupd_kernel, nblk((long long)q * N, 256), 256, 0, st, V, temp, tnew, I0,
                         q, r, N, k);
      e = hipMemcpyAsync(temp + (size_t)k * r * N, tnew, 8 * (size_t)r * N,
                         hipMemcpyDeviceToDevice, st);
    }
    if (e == hipSuccess) e = hipGetLastError();
  }
  for (double* p : {temp, V, Cm, Ck, M, x, z, W, tnew})
    if (p) (void)hipFreeAsync(p, st);
  return e;
}

}  // namespace gpt
