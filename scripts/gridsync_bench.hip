// Cost of a grid-wide barrier on MI355X (diagnostic, not part of the library): a cooperative
// launch of G workgroups runs `iters` cooperative_groups grid syncs, and a hand-rolled barrier
// (agent-scope relaxed atomic arrival counter + polling, s_sleep between polls) for comparison.
//   hipcc --offload-arch=gfx950 -O3 scripts/gridsync_bench.hip -o diagbin/gridsync_bench
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <cstdio>
#include <cstdlib>
namespace cg = cooperative_groups;

__global__ void cg_sync_kernel(int iters, long long* out) {
  cg::grid_group g = cg::this_grid();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) g.sync();
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = t1 - t0;
}

__global__ void atomic_sync_kernel(int iters, unsigned* ctr, long long* out) {
  const long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned G = gridDim.x;
  for (int i = 0; i < iters; ++i) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = G * (unsigned)(i + 1);
      while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target)
        __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = t1 - t0;
}

int main(int argc, char** argv) {
  const int iters = 2000;
  long long* d_out;
  unsigned* d_ctr;
  (void)hipMalloc(&d_out, 8);
  (void)hipMalloc(&d_ctr, 4);
  int grids[] = {9, 32, 128, 256};
  for (int G : grids) {
    for (int threads : {256, 512}) {
      void* args[] = {(void*)&iters, (void*)&d_out};
      hipError_t e = hipLaunchCooperativeKernel((const void*)cg_sync_kernel, dim3(G), dim3(threads), args, 0, 0);
      (void)hipDeviceSynchronize();
      long long cyc = 0;
      (void)hipMemcpy(&cyc, d_out, 8, hipMemcpyDeviceToHost);
      (void)hipMemset(d_ctr, 0, 4);
      hipLaunchKernelGGL(atomic_sync_kernel, dim3(G), dim3(threads), 0, 0, iters, d_ctr, d_out);
      (void)hipDeviceSynchronize();
      long long cyc2 = 0;
      (void)hipMemcpy(&cyc2, d_out, 8, hipMemcpyDeviceToHost);
      std::printf("G=%3d threads=%d  cg grid.sync: %s %.0f cycles each   atomic barrier: %.0f cycles each\n",
                  G, threads, e == hipSuccess ? "ok" : hipGetErrorString(e), (double)cyc / iters,
                  (double)cyc2 / iters);
    }
  }
  return 0;
}
