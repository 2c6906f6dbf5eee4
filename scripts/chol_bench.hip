// Standalone timing of the dense Gibbs solves (tgp.hip): blocked Cholesky and the triangular
// solves on a random SPD matrix of size p, with per-panel phase stamps of the Cholesky
// (GPT_CHOL_STAMPS build).  Diagnostic only (not part of the library):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DGPT_CHOL_STAMPS=1 -I gpt_amd/csrc \
//         scripts/chol_bench.hip -o /tmp/chol_bench && /tmp/chol_bench 400
#include "../gpt_amd/csrc/tgp.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

using namespace gpt;

int main(int argc, char** argv) {
  const int p = argc > 1 ? std::atoi(argv[1]) : 400;
  std::vector<double> A((size_t)p * p), M((size_t)p * p);
  unsigned s = 12345;
  for (auto& v : A) { s = s * 1103515245u + 12345u; v = ((s >> 8) & 0xffff) / 65536.0 - 0.5; }
  for (int i = 0; i < p; ++i)
    for (int j = 0; j < p; ++j) {
      double t = 0.0;
      for (int k = 0; k < p; ++k) t += A[i + (size_t)p * k] * A[j + (size_t)p * k];
      M[i + (size_t)p * j] = t + (i == j ? p : 0.0);
    }
  double *dM, *dM0, *dx;
  int32_t* dst;
  (void)hipMalloc(&dM, 8 * M.size()); (void)hipMalloc(&dM0, 8 * M.size());
  (void)hipMalloc(&dx, 8 * p); (void)hipMalloc(&dst, 4);
  (void)hipMemcpy(dM0, M.data(), 8 * M.size(), hipMemcpyHostToDevice);
  (void)hipMemset(dst, 0, 4);
  std::vector<double> x(p, 1.0);
  hipEvent_t e0, e1, e2, e3, e4;
  hipEventCreate(&e0); hipEventCreate(&e1); hipEventCreate(&e2); hipEventCreate(&e3); hipEventCreate(&e4);
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipMemcpy(dM, dM0, 8 * M.size(), hipMemcpyDeviceToDevice);
    (void)hipMemcpy(dx, x.data(), 8 * p, hipMemcpyHostToDevice);
    hipEventRecord(e0, 0);
    launch_chol(dM, p, dst, 0);
    hipEventRecord(e1, 0);
    launch_trsv(dM, p, dx, 0, 0);
    hipEventRecord(e2, 0);
    launch_trsv(dM, p, dx, 1, 0);
    hipEventRecord(e3, 0);
    hipEventSynchronize(e3);
    float a, b, c;
    hipEventElapsedTime(&a, e0, e1); hipEventElapsedTime(&b, e1, e2); hipEventElapsedTime(&c, e2, e3);
    std::printf("p=%d chol %.1f us  trsv %.1f us  trsvT %.1f us\n", p, 1e3 * a, 1e3 * b, 1e3 * c);
  }
  // residual of M x = 1
  std::vector<double> sol(p);
  (void)hipMemcpy(sol.data(), dx, 8 * p, hipMemcpyDeviceToHost);
  double r = 0.0;
  for (int i = 0; i < p; ++i) {
    double t = 0.0;
    for (int j = 0; j < p; ++j) t += M[i + (size_t)p * j] * sol[j];
    r = std::fmax(r, std::fabs(t - 1.0));
  }
  int32_t st = 0;
  (void)hipMemcpy(&st, dst, 4, hipMemcpyDeviceToHost);
  std::printf("max |M x - 1| = %.3e, status %d\n", r, st);
#if GPT_CHOL_STAMPS
  long long stp[64 * 8];
  (void)hipMemcpyFromSymbol(stp, HIP_SYMBOL(g_chol_stamps), sizeof(stp));
  const char* nm[6] = {"load", "diag", "solve", "write", "trail", "barrier"};
  long long tot[6] = {0};
  const int np = (p + kCholNB - 1) / kCholNB;
  for (int q = 0; q < np && q < 64; ++q)
    for (int ph = 0; ph < 6; ++ph) tot[ph] += stp[q * 8 + ph + 1] - stp[q * 8 + ph];
  for (int ph = 0; ph < 6; ++ph) std::printf("  %-8s %lld cycles (%d panels)\n", nm[ph], tot[ph], np);
#endif
  return 0;
}
