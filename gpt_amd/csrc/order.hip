// Epoch orders on the device (GPT_SGLD.jl:373-374: perm = randperm(N); phi = phi[:,:,perm]).
//
// The reference permutes phi in place every epoch, so the permutations compose: batch slot i of
// epoch e reads row order_e[i] = order_{e-1}[perm_e[i]] (order_{-1} = identity).  perm_e is the
// framework's Fisher–Yates contract (oracle/philox.py randperm): for i = N-1 … 1,
// swap(p[i], p[j_i]) with j_i = ⌊x0(i, e, PERM, 0)·(i+1)/2^32⌋.
//
// Each chain keeps a two-slot ring of orders (ChainDesc::order, 2·N int32): slot e&1 holds
// order_e.  The session builds order_{e+1} right before the first step of epoch e (the grid engine's
// last step of epoch e already reads the next epoch's first batch), when slot (e+1)&1 — order_{e-1}
// — has no reader left.  So nothing is generated on the host and the device holds 2·N ints per
// chain whatever the number of epochs.
//
// The swaps are applied in parallel by deterministic reservations (Shun, Gu, Blelloch, Fineman,
// Gibbons, SODA 2015): every round, each pending swap i writes max(i) into the reservation words of
// both of its positions; a swap holding both commits.  Every swap that precedes i in the sequential
// order (a larger index) and touches one of i's positions has committed already — it would hold the
// reservation otherwise — and every pending one that touches them has a smaller index and waits, so
// the result is the sequential shuffle bit for bit.  The largest pending index always commits; N =
// 10 000 takes 29 rounds.  One 1024-thread workgroup per chain; p, the reservations and j live in
// LDS up to 13 632 rows (12 B per row), in a global workspace beyond.
#include "gpt_internal.h"

namespace gpt {

constexpr int kOrdNT = 1024;
constexpr int kOrdLdsMax = 160 * 1024 - 256;       // dynamic LDS beside the kernel's static words
constexpr int kOrdLdsRows = kOrdLdsMax / 12;

template <bool LDS>
struct OrdMem {
  // LDS words are plain; global words are accessed at agent scope so that no access is served by
  // a stale L1 line next to the L2 atomics (the workgroup owns its workspace, but the reservation
  // atomics execute in L2).
  static __device__ __forceinline__ int ld(const int32_t* a) {
    if constexpr (LDS) return *a;
    else return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  static __device__ __forceinline__ void st(int32_t* a, int v) {
    if constexpr (LDS) *a = v;
    else __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  static __device__ __forceinline__ void amax(int32_t* a, int v) {
    if constexpr (LDS) atomicMax(a, v);
    else __hip_atomic_fetch_max(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
};

// e_fixed >= 0: build order_{e_fixed}.  Otherwise build order_{e+1} for the epoch e of step
// tbase[0] + t_local (launched before that step, which is the first of its epoch).
template <bool LDS>
__global__ __launch_bounds__(kOrdNT) void epoch_order_kernel(const ChainDesc* chains, int N, int nb,
                                                              long long total_steps,
                                                              const long long* tbase, int t_local,
                                                              int e_fixed, int32_t* ws) {
  extern __shared__ __attribute__((aligned(16))) int32_t osm[];
  __shared__ int remaining;
  __shared__ int wdone[kOrdNT / 64];
  using M = OrdMem<LDS>;
  const ChainDesc C = chains[blockIdx.x];
  int e = e_fixed;
  if (e < 0) {
    const long long t = tbase[0] + t_local;
    e = (int)(t / nb) + 1;
    if ((long long)e * nb >= total_steps) return;   // no step of the run reads this epoch
  }
  int32_t* p = LDS ? osm : ws + (size_t)blockIdx.x * 3 * N;
  int32_t* R = p + N;
  int32_t* J = R + N;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < N; i += kOrdNT) {
    M::st(p + i, i);
    M::st(R + i, -1);
    int j = -1;                                       // position 0 has no swap of its own
    if (i > 0) {
      const uint32_t x = philox4x32((uint32_t)i, (uint32_t)e, kPerm, 0, C.seed).x;
      j = (int)(((uint64_t)x * (uint64_t)(i + 1)) >> 32);
    }
    M::st(J + i, j);
  }
  if (tid == 0) remaining = N - 1;
  __syncthreads();
  while (remaining > 0) {
    for (int i = tid; i < N; i += kOrdNT) {           // reserve both positions of every pending swap
      const int j = M::ld(J + i);
      if (j >= 0) {
        M::amax(R + i, i);
        M::amax(R + j, i);
      }
    }
    __syncthreads();
    int done = 0;
    for (int i = tid; i < N; i += kOrdNT) {           // commit the swaps that hold both
      const int j = M::ld(J + i);
      if (j >= 0 && M::ld(R + i) == i && M::ld(R + j) == i) {
        const int pi = M::ld(p + i), pj = M::ld(p + j);
        M::st(p + i, pj);
        M::st(p + j, pi);
        M::st(J + i, -1);
        ++done;
      }
    }
    __syncthreads();
    for (int i = tid; i < N; i += kOrdNT) M::st(R + i, -1);
    for (int o = 32; o >= 1; o >>= 1) done += __shfl_xor(done, o);
    if (lane == 0) wdone[wv] = done;
    __syncthreads();
    if (tid == 0) {
      int s = 0;
      for (int w = 0; w < kOrdNT / 64; ++w) s += wdone[w];
      remaining -= s;
    }
    __syncthreads();
  }
  // compose: order_e[i] = order_{e-1}[perm_e[i]]
  int32_t* out = C.order + (size_t)(e & 1) * N;
  const int32_t* prev = C.order + (size_t)((e + 1) & 1) * N;
  for (int i = tid; i < N; i += kOrdNT) {
    const int pi = M::ld(p + i);
    out[i] = e == 0 ? pi : prev[pi];
  }
}

bool epoch_order_in_lds(int N) { return N <= kOrdLdsRows; }
size_t epoch_order_ws_ints(int N, int nchains) {
  return epoch_order_in_lds(N) ? 0 : (size_t)3 * N * nchains;
}

hipError_t launch_epoch_order(const ChainDesc* chains, int nchains, int N, int nb,
                              long long total_steps, const long long* tbase, int t_local,
                              int e_fixed, int32_t* ws, hipStream_t st) {
  if (N < 1) return hipSuccess;
  if (epoch_order_in_lds(N)) {
    static std::atomic<uint64_t> attr{0};
    hipError_t e = set_max_lds_once((const void*)epoch_order_kernel<true>, kOrdLdsMax, attr);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(epoch_order_kernel<true>, dim3(nchains), dim3(kOrdNT), (size_t)12 * N, st,
                       chains, N, nb, total_steps, tbase, t_local, e_fixed, nullptr);
  } else {
    if (!ws) return hipErrorInvalidValue;
    hipLaunchKernelGGL(epoch_order_kernel<false>, dim3(nchains), dim3(kOrdNT), 0, st, chains, N,
                       nb, total_steps, tbase, t_local, e_fixed, ws);
  }
  return hipGetLastError();
}

}  // namespace gpt
