// v_mfma_f64_16x16x4f64 issue rate and dependent latency on gfx950 (diagnostic).
// One workgroup per CU, W waves per workgroup (W/4 per SIMD), each wave running NIT passes of
// C independent accumulation chains; s_memtime around the loop of every wave.
//   hipcc --offload-arch=gfx950 -O3 scripts/mfma_f64_bench.hip -o /tmp/mfma_f64_bench
//   /tmp/mfma_f64_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int C>
__global__ void bench(long long* out, double* sink, int nit) {
  const int lane = threadIdx.x & 63;
  double a = 1.0 + lane * 1e-9, b = 1.0 - lane * 1e-9;
  d4 acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = d4{0.0, 0.0, 0.0, (double)c};
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < nit; ++i) {
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) s += acc[c][0] + acc[c][3];
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_mfma_f64_4x4x4f64 (four 4 × 4 blocks, K = 4, one double per lane in and out)
template <int C>
__global__ void bench4(long long* out, double* sink, int nit) {
  const int lane = threadIdx.x & 63;
  double a = 1.0 + lane * 1e-9, b = 1.0 - lane * 1e-9;
  double acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = (double)c;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < nit; ++i) {
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) s += acc[c];
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int C>
static void run4(int W, int nit) {
  const int nb = 256;
  long long* d_out;
  double* d_sink;
  (void)hipMalloc(&d_out, sizeof(long long) * nb * W);
  (void)hipMalloc(&d_sink, sizeof(double) * nb * W * 64);
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL(bench4<C>, dim3(nb), dim3(64 * W), 0, 0, d_out, d_sink, nit);
  (void)hipDeviceSynchronize();
  std::vector<long long> h(nb * W);
  (void)hipMemcpy(h.data(), d_out, sizeof(long long) * nb * W, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  const double per_wave = (double)h[h.size() / 2] / ((double)nit * C);
  printf("4x4x4 f64: waves/WG %2d chains %d : %.1f cycles per MFMA of a wave, %.1f per MFMA per SIMD\n",
         W, C, per_wave, per_wave / std::max(1, W / 4));
  (void)hipFree(d_out);
  (void)hipFree(d_sink);
}

// The MovieLens feature-tile pass: 12 LDS reads, one wait, 8 VALU operand ops, 4 chained MFMAs
// whose sources the next pass's reads and VALU overwrite (PP = 1), or the same with the next
// pass's reads issued before this pass's MFMAs into a second register set (PP = 2).
template <int PP>
__global__ void pass_bench(long long* out, double* sink, int nit) {
  __shared__ double T[100 * 20];
  __shared__ unsigned long long mk[100];
  __shared__ double er[100];
  const int tid = threadIdx.x, lane = tid & 63, rl = lane & 15, kl = lane >> 4;
  for (int i = tid; i < 2000; i += blockDim.x) T[i] = 1.0 + i * 1e-6;
  for (int i = tid; i < 100; i += blockDim.x) { mk[i] = 0x5555555555555555ull ^ i; er[i] = 0.5 + i * 1e-3; }
  __syncthreads();
  const int B = 100, R = 20, fa = rl, lb = rl;
  d4 acc = d4{0.0, 0.0, 0.0, 0.0};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < nit; ++it) {
    if (PP == 1) {
      for (int k0 = 0; k0 < B; k0 += 16) {
        unsigned long long mr[4];
        double e4[4], t4[4], av[4], bv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int kc = min(k0 + 4 * u + kl, B - 1);
          mr[u] = mk[kc]; e4[u] = er[kc]; t4[u] = T[kc * R + lb];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          av[u] = (double)((unsigned)(mr[u] >> fa) & 1u & (unsigned)(k0 + 4 * u + kl < B));
          bv[u] = e4[u] * t4[u];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc, 0, 0, 0);
      }
    } else {
      double av[2][4], bv[2][4];
      auto ld = [&](int k0, double (&a)[4], double (&b)[4]) {
        unsigned long long mr[4];
        double e4[4], t4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int kc = min(k0 + 4 * u + kl, B - 1);
          mr[u] = mk[kc]; e4[u] = er[kc]; t4[u] = T[kc * R + lb];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a[u] = (double)((unsigned)(mr[u] >> fa) & 1u & (unsigned)(k0 + 4 * u + kl < B));
          b[u] = e4[u] * t4[u];
        }
      };
      ld(0, av[0], bv[0]);
      for (int k0 = 0; k0 < B; k0 += 32) {
        ld(k0 + 16, av[1], bv[1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[0][u], bv[0][u], acc, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        ld(k0 + 32, av[0], bv[0]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[1][u], bv[1][u], acc, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[blockIdx.x * (blockDim.x / 64) + (tid >> 6)] = t1 - t0;
  sink[blockIdx.x * blockDim.x + tid] = acc[0] + acc[3];
}

template <int PP>
static void run_pass(int W, int nit) {
  const int nb = 256;
  long long* d_out;
  double* d_sink;
  (void)hipMalloc(&d_out, sizeof(long long) * nb * W);
  (void)hipMalloc(&d_sink, sizeof(double) * nb * W * 64);
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL(pass_bench<PP>, dim3(nb), dim3(64 * W), 0, 0, d_out, d_sink, nit);
  (void)hipDeviceSynchronize();
  std::vector<long long> h(nb * W);
  (void)hipMemcpy(h.data(), d_out, sizeof(long long) * nb * W, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  const int passes = PP == 1 ? 7 : 8;
  printf("feature-tile pass (%s), waves/WG %2d: %.0f cycles per tile of a wave (%d passes)\n",
         PP == 1 ? "as in cf.hip" : "pipelined  ", W, (double)h[h.size() / 2] / nit, passes);
  (void)hipFree(d_out);
  (void)hipFree(d_sink);
}

template <int C>
static void run(int W, int nit) {
  const int nb = 256;
  long long* d_out;
  double* d_sink;
  (void)hipMalloc(&d_out, sizeof(long long) * nb * W);
  (void)hipMalloc(&d_sink, sizeof(double) * nb * W * 64);
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL(bench<C>, dim3(nb), dim3(64 * W), 0, 0, d_out, d_sink, nit);
  (void)hipDeviceSynchronize();
  std::vector<long long> h(nb * W);
  (void)hipMemcpy(h.data(), d_out, sizeof(long long) * nb * W, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  const double med = (double)h[h.size() / 2];
  // cycles per MFMA of one wave; per SIMD (W/4 waves share a SIMD)
  const double per_wave = med / ((double)nit * C);
  printf("waves/WG %2d (per SIMD %d)  chains %d : %.1f cycles per MFMA of a wave, %.1f per MFMA per SIMD\n",
         W, std::max(1, W / 4), C, per_wave, per_wave / std::max(1, W / 4));
  (void)hipFree(d_out);
  (void)hipFree(d_sink);
}

int main() {
  const int nit = 512;
  for (int W : {1, 4, 8, 16}) {
    run<1>(W, nit);
    run<2>(W, nit);
    run<4>(W, nit);
  }
  for (int W : {1, 4, 16}) {
    run4<1>(W, nit);
    run4<4>(W, nit);
  }
  for (int W : {1, 4, 8, 16}) {
    run_pass<1>(W, 64);
    run_pass<2>(W, 64);
  }
  return 0;
}
