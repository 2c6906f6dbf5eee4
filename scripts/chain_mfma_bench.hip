// The chain engine's two per-wave contractions on the VALU (as chain.hip runs them) and on the
// fp64 matrix cores (v_mfma_f64_16x16x4f64), at the bench shape: one wave per (chain, dimension),
// 8 waves per workgroup, 256 workgroups (2 048 waves, two per SIMD, as chain_kernel<5,8,2,8>);
// per "step" each wave takes a batch of B = 50 rows of phi (n = 500 doubles each, random rows of
// a 10 000-row table) and forms
//   phidotU  temp[i, l]  = Σ_j phi[row_i, j] · U[j, l]                (B × r, K = n)
//   gradU    G[j, l]    += Σ_i phi[row_i, j] · c[i, l]  with c = temp (n × r, K = B)
// VALU form: the chain kernel's register layout (lane λ holds rows j = λ + 64·jj of U and G, the
// batch streamed two rows at a time, each row loaded once and used by both contractions, the G·R
// partial dots reduced over the wave by an xor butterfly).  MFMA form: phidotU as 16-row tiles of
// the batch (A = phi rows, K = n, B = U with r = 5 padded to 16 columns), gradU as 16-row tiles of
// n (A = phi columns, K = the batch rows, B = c); c through LDS, U from global memory (beside c
// it does not fit the workgroup's LDS); G accumulates in memory (its 32 tiles do not fit registers).
// Diagnostic, not part of the library:
//   hipcc --offload-arch=gfx950 -O3 scripts/chain_mfma_bench.hip -o diagbin/chain_mfma_bench
//   diagbin/chain_mfma_bench [steps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

constexpr int kN = 500, kR = 5, kB = 50, kJ = 8, kRows = 10000, kWaves = 8, kWG = 256;
typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int row_of(int wave, int step, int i) {
  unsigned h = (unsigned)(wave * 7919 + step * 104729 + i * 1299709);
  h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
  return (int)(h % kRows);
}

__device__ __forceinline__ double xsum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---------------------------------------------------------------- VALU form
__global__ __launch_bounds__(512, 1) void valu_kernel(const double* __restrict__ phi,
                                                     const double* __restrict__ U0, int steps,
                                                     double* __restrict__ out, long long* cyc) {
  const int lane = threadIdx.x & 63, wave = blockIdx.x * kWaves + (threadIdx.x >> 6);
  double u[kJ][kR], g[kJ][kR];
#pragma unroll
  for (int jj = 0; jj < kJ; ++jj)
#pragma unroll
    for (int l = 0; l < kR; ++l) {
      const int j = lane + 64 * jj;
      u[jj][l] = j < kN ? U0[(size_t)(wave % 64) * kN * kR + l * kN + j] : 0.0;
      g[jj][l] = 0.0;
    }
  double chk = 0.0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < steps; ++s) {
    for (int i0 = 0; i0 < kB; i0 += 2) {
      double p[2][kJ];
#pragma unroll
      for (int gg = 0; gg < 2; ++gg) {
        const double* rp = phi + (size_t)row_of(wave, s, i0 + gg) * kN;
#pragma unroll
        for (int jj = 0; jj < kJ; ++jj) {
          const int j = lane + 64 * jj;
          p[gg][jj] = rp[j < kN ? j : kN - 1];
        }
      }
      double t[2][kR];
#pragma unroll
      for (int gg = 0; gg < 2; ++gg)
#pragma unroll
        for (int l = 0; l < kR; ++l) {
          double v = 0.0;
#pragma unroll
          for (int jj = 0; jj < kJ; ++jj) v = fma(p[gg][jj], u[jj][l], v);
          t[gg][l] = xsum(v);
        }
#pragma unroll
      for (int gg = 0; gg < 2; ++gg)
#pragma unroll
        for (int jj = 0; jj < kJ; ++jj)
#pragma unroll
          for (int l = 0; l < kR; ++l) g[jj][l] = fma(p[gg][jj], t[gg][l], g[jj][l]);
#pragma unroll
      for (int gg = 0; gg < 2; ++gg)
#pragma unroll
        for (int l = 0; l < kR; ++l) chk += t[gg][l];
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  double gs = 0.0;
#pragma unroll
  for (int jj = 0; jj < kJ; ++jj)
#pragma unroll
    for (int l = 0; l < kR; ++l) gs += (lane + 64 * jj < kN) ? g[jj][l] : 0.0;
  gs = xsum(gs);
  if (lane == 0) {
    out[2 * wave] = chk;
    out[2 * wave + 1] = gs;
    cyc[wave] = t1 - t0;
  }
}

// ---------------------------------------------------------------- MFMA form
__global__ __launch_bounds__(512, 1) void mfma_kernel(const double* __restrict__ phi,
                                                     const double* __restrict__ U0, int steps,
                                                     double* __restrict__ out, long long* cyc,
                                                     double* __restrict__ gmem) {
  // U (20 KB per wave) does not fit beside c in the workgroup's LDS: B operands of phidotU come
  // from global memory (L1 / L2 resident)
  __shared__ double cl[kWaves][64 * 16];            // c = temp rows (padded 64 × 16)
  __shared__ int rl[kWaves][64];
  const int lane = threadIdx.x & 63, w8 = threadIdx.x >> 6, wave = blockIdx.x * kWaves + w8;
  const double* Ug = U0 + (size_t)(wave % 64) * kN * kR;
  double* G = gmem + (size_t)wave * kN * 16;         // zeroed by the host before the launch
  const int r16 = lane & 15, k4 = lane >> 4;
  double chk = 0.0;
  __builtin_amdgcn_wave_barrier();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < steps; ++s) {
    rl[w8][lane] = lane < kB ? row_of(wave, s, lane) : row_of(wave, s, kB - 1);
    __builtin_amdgcn_wave_barrier();
    // phidotU: four 16-row tiles of the batch, K = n in steps of 4 (125 MFMAs per tile)
#pragma unroll 1
    for (int t = 0; t < 4; ++t) {
      const double* rp = phi + (size_t)rl[w8][16 * t + r16] * kN;
      d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 5
      for (int kk = 0; kk < kN / 4; ++kk) {
        const int j = 4 * kk + k4;
        const double a = rp[j];
        const double b = r16 < kR ? Ug[r16 * kN + j] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
      }
      // D[k4 + 4·v][r16] = temp[16t + k4 + 4·v][r16]
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int i = 16 * t + k4 + 4 * v;
        const double x = (i < kB && r16 < kR) ? acc[v] : 0.0;
        cl[w8][i * 16 + r16] = x;
        chk += x;
      }
    }
    __builtin_amdgcn_wave_barrier();
    // gradU: 32 tiles of 16 rows of n (500 -> 512), K = the batch rows in steps of 4 (13 MFMAs)
#pragma unroll 1
    for (int t = 0; t < 32; ++t) {
      const int j = 16 * t + r16;
      d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kb = 0; kb < 13; ++kb) {
        const int i = 4 * kb + k4;
        const double a = (i < kB && j < kN) ? phi[(size_t)rl[w8][i] * kN + j] : 0.0;
        const double b = cl[w8][i * 16 + r16];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
      }
      // D[k4 + 4·v][r16] = G-increment[16t + k4 + 4·v][l = r16]
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int jj = 16 * t + k4 + 4 * v;
        if (jj < kN) {            // read-modify-write past the L1 (the line may hold the old G)
          double* gp = G + jj * 16 + r16;
          const double cur = __hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(gp, cur + acc[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
  }
  __threadfence_block();
  const long long t1 = __builtin_amdgcn_s_memtime();
  double gs = 0.0;
  for (int o = lane; o < kN * 16; o += 64)
    gs += (o % 16) < kR ? __hip_atomic_load(G + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
  gs = xsum(gs);
  chk = xsum(chk) ;
  if (lane == 0) {
    out[2 * wave] = chk;
    out[2 * wave + 1] = gs;
    cyc[wave] = t1 - t0;
  }
}

int main(int argc, char** argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 20;
  const int W = kWG * kWaves;
  std::vector<double> hphi((size_t)kRows * kN), hU((size_t)64 * kN * kR);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xffff) / 65536.0 - 0.5; };
  for (auto& x : hphi) x = rnd();
  for (auto& x : hU) x = rnd() * 0.1;
  double *dphi, *dU, *dout, *dG;
  long long* dcyc;
  (void)hipMalloc(&dphi, 8 * hphi.size());
  (void)hipMalloc(&dU, 8 * hU.size());
  (void)hipMalloc(&dout, 16 * W);
  (void)hipMalloc(&dcyc, 8 * W);
  (void)hipMalloc(&dG, (size_t)8 * W * kN * 16);
  (void)hipMemcpy(dphi, hphi.data(), 8 * hphi.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(dU, hU.data(), 8 * hU.size(), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  std::vector<double> ov(2 * W), om(2 * W);
  std::vector<long long> cv(W), cm(W);
  for (int rep = 0; rep < 3; ++rep) {
    float msv = 0.f, msm = 0.f;
    hipLaunchKernelGGL(valu_kernel, dim3(kWG), dim3(512), 0, 0, dphi, dU, 2, dout, dcyc);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(valu_kernel, dim3(kWG), dim3(512), 0, 0, dphi, dU, steps, dout, dcyc);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&msv, e0, e1);
    (void)hipMemcpy(ov.data(), dout, 16 * W, hipMemcpyDeviceToHost);
    (void)hipMemcpy(cv.data(), dcyc, 8 * W, hipMemcpyDeviceToHost);
    (void)hipMemset(dG, 0, (size_t)8 * W * kN * 16);
    hipLaunchKernelGGL(mfma_kernel, dim3(kWG), dim3(512), 0, 0, dphi, dU, 2, dout, dcyc, dG);
    (void)hipMemset(dG, 0, (size_t)8 * W * kN * 16);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_kernel, dim3(kWG), dim3(512), 0, 0, dphi, dU, steps, dout, dcyc, dG);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&msm, e0, e1);
    (void)hipMemcpy(om.data(), dout, 16 * W, hipMemcpyDeviceToHost);
    (void)hipMemcpy(cm.data(), dcyc, 8 * W, hipMemcpyDeviceToHost);
    double dt = 0.0, dg = 0.0;
    for (int w = 0; w < W; ++w) {
      dt = std::max(dt, std::fabs(ov[2 * w] - om[2 * w]) / std::max(1e-30, std::fabs(ov[2 * w])));
      dg = std::max(dg, std::fabs(ov[2 * w + 1] - om[2 * w + 1]) / std::max(1e-30, std::fabs(ov[2 * w + 1])));
    }
    std::vector<long long> a(cv), b(cm);
    std::nth_element(a.begin(), a.begin() + W / 2, a.end());
    std::nth_element(b.begin(), b.begin() + W / 2, b.end());
    if (rep == 0) printf("wave 0: VALU temp-sum %.6e gradU-sum %.6e | MFMA %.6e %.6e\n", ov[0], ov[1], om[0], om[1]);
    printf("steps %d  VALU %.1f us/step (%lld cycles/step median)  MFMA %.1f us/step (%lld cycles/step)"
           "  max rel diff temp-sum %.1e gradU-sum %.1e\n", steps, 1e3 * msv / steps,
           a[W / 2] / steps, 1e3 * msm / steps, b[W / 2] / steps, dt, dg);
  }
  return 0;
}
