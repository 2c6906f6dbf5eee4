// Random-Fourier-feature maps (GPT_SGLD.jl:71-84, 109-120) and the full-theta SGLD step
// (GPNT_SGLD, GPT_SGLD.jl:809-847).
#include "device_util.h"

namespace gpt {

// phi[j + n(k + D i)] = c · cos(X[i + N k] · (Z[j + n k] · (1/ls[k])) + b[j + n k]).
// The argument is formed with round-to-nearest multiplies/adds (no FMA contraction) so it is
// the same double the reference forms; only cos differs (≤1 ulp between libms).
__global__ __launch_bounds__(256) void feature_kernel(const double* __restrict__ X, long long N,
                                                      int D, const double* __restrict__ ls,
                                                      double c, const double* __restrict__ Z,
                                                      const double* __restrict__ b, int n,
                                                      double* __restrict__ phi) {
  const long long total = (long long)n * D * N;
  for (long long x = (long long)blockIdx.x * blockDim.x + threadIdx.x; x < total;
       x += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(x % n);
    const long long rest = x / n;
    const int k = (int)(rest % D);
    const long long i = rest / D;
    const double zt = __dmul_rn(Z[j + (long long)n * k], 1.0 / ls[k]);
    const double arg = __dadd_rn(__dmul_rn(X[i + N * k], zt), b[j + (long long)n * k]);
    phi[x] = c * cos(arg);
  }
}

// phi[j + n i] = c · cos(Σ_k X[i,k]·Zt[j,k] + b[j]),  c = sqrt(2/n)·σ  (sum in k order).
__global__ __launch_bounds__(256) void feature_notensor_kernel(
    const double* __restrict__ X, long long N, int D, const double* __restrict__ ls, double c,
    const double* __restrict__ Z, const double* __restrict__ b, int n, double* __restrict__ phi) {
  const long long total = (long long)n * N;
  for (long long x = (long long)blockIdx.x * blockDim.x + threadIdx.x; x < total;
       x += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(x % n);
    const long long i = x / n;
    double s = 0.0;
    for (int k = 0; k < D; ++k)
      s = __dadd_rn(s, __dmul_rn(X[i + N * k], __dmul_rn(Z[j + (long long)n * k], 1.0 / ls[k])));
    phi[x] = c * cos(__dadd_rn(s, b[j]));
  }
}

hipError_t launch_feature(const double* X, long long N, int D, const double* ls, double c,
                          const double* Z, const double* b, int n, double* phi, hipStream_t st) {
  const long long total = (long long)n * D * N;
  const int blocks = (int)min((total + 255) / 256, (long long)256 * 16);
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(feature_kernel, dim3(blocks), dim3(256), 0, st, X, N, D, ls, c, Z, b, n, phi);
  return hipGetLastError();
}

hipError_t launch_feature_notensor(const double* X, long long N, int D, const double* ls,
                                   double c, const double* Z, const double* b, int n,
                                   double* phi, hipStream_t st) {
  const long long total = (long long)n * N;
  const int blocks = (int)min((total + 255) / 256, (long long)256 * 16);
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(feature_notensor_kernel, dim3(blocks), dim3(256), 0, st, X, N, D, ls, c, Z,
                     b, n, phi);
  return hipGetLastError();
}

// One full-theta SGLD step (GPT_SGLD.jl:826-843) in one workgroup:
//   res = y_B − Φ_Bᵀθ ;  θ += ε_t/2·(−θ/σθ² + (N/B)Φ_B res/σ²) + sqrt(ε_t)·ξ ;  store θ.
__global__ __launch_bounds__(kNT) void gpnt_step_kernel(
    const double* __restrict__ phi, const double* __restrict__ y,
    const int32_t* __restrict__ order, int n, int N, int m, int nb, long long total,
    double signal_var, double sigma_theta, double eps_theta, double decay_rate, uint64_t seed,
    double* __restrict__ theta, double* __restrict__ store, int32_t* __restrict__ status,
    const long long* __restrict__ tbase, int t_local) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const long long t = tbase[0] + t_local;
  if (t >= total) return;
  if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int e = (int)(t / nb), b = (int)(t - (long long)e * nb);
  const int start = b * m;
  const int Bt = min(m, N - start);
  int* idx_l = (int*)smem;
  double* res_l = (double*)(smem + al16(4 * (size_t)m));
  double* red = res_l + ((m + 1) & ~1);
  const int32_t* ord = order + (size_t)e * N + start;
  for (int i = tid; i < Bt; i += kNT) idx_l[i] = ord[i];
  __syncthreads();
  // Φ_Bᵀθ: lanes over features j (coalesced), 64 batch columns per pass, Butterfly over lanes.
  for (int base = 0; base < Bt; base += 64) {
    double v[64];
#pragma unroll
    for (int u = 0; u < 64; ++u) v[u] = 0.0;
    for (int j = wv * 64 + lane; j < n; j += kNT) {
      const double th = theta[j];
#pragma unroll
      for (int u = 0; u < 64; ++u) {
        const int i = min(base + u, Bt - 1);
        v[u] = fma(phi[(long long)uni(idx_l[i]) * n + j], th, v[u]);
      }
    }
    Butterfly<64>::run(v, lane);
    red[wv * 64 + lane] = v[0];
    __syncthreads();
    if (tid < 64 && base + tid < Bt) {
      double s = 0.0;
#pragma unroll
      for (int w2 = 0; w2 < kNW; ++w2) s += red[w2 * 64 + tid];
      res_l[base + tid] = y[idx_l[base + tid]] - s;
    }
    __syncthreads();
  }
  const double eps = eps_theta * pow((double)(t + 1), -decay_rate);
  const double cN = (double)N / (double)Bt;
  const double isg2 = 1.0 / (sigma_theta * sigma_theta);
  bool bad = false;
  double* out = store ? store + (size_t)t * n : nullptr;
  for (int j = tid; j < n; j += kNT) {
    double g = 0.0;
    for (int i = 0; i < Bt; ++i) g = fma(phi[(long long)uni(idx_l[i]) * n + j], res_l[i], g);
    const double th = theta[j];
    const double grad = -th * isg2 + cN * g / signal_var;
    const double nt = th + (eps * grad / 2 +
                            sqrt(eps) * normal_at(seed, (uint32_t)j, (uint32_t)t, kThetaNoise, 0));
    theta[j] = nt;
    if (out) out[j] = nt;
    bad |= (nt != nt);
  }
  if (__syncthreads_or(bad) && tid == 0)
    __hip_atomic_store(status, GPT_ERR_NAN_THETA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

hipError_t launch_gpnt(const double* phi, const double* y, const int32_t* order, int n, int N,
                       int m, int nb, long long total, double signal_var, double sigma_theta,
                       double eps_theta, double decay_rate, uint64_t seed, double* theta,
                       double* theta_store, int32_t* status, const long long* tbase, int t_local,
                       hipStream_t st) {
  const size_t lds = al16(4 * (size_t)m) + 8 * (size_t)(((m + 1) & ~1) + kNW * 64);
  hipLaunchKernelGGL(gpnt_step_kernel, dim3(1), dim3(kNT), lds, st, phi, y, order, n, N, m, nb,
                     total, signal_var, sigma_theta, eps_theta, decay_rate, seed, theta,
                     theta_store, status, tbase, t_local);
  return hipGetLastError();
}

}  // namespace gpt
