// Tensor-GP Gibbs sweep (TGP.jl:37-86, `GPT_inf`) for MI355X (gfx950).
//
// A sweep draws W | U from its Gaussian conditional (q × q) and then each U_k | W, U_{-k}
// (nr × nr).  The dense parts are SYRKs with a long inner dimension (K = N samples), done on the
// fp64 matrix cores (v_mfma_f64_16x16x4f64), and Cholesky factorisations / triangular solves of
// the q × q and nr × nr precision matrices, done by one workgroup each (they are small:
// q ≈ 100, nr <= ~1000 in the reference's use, `UnitTest.jl:15-28`).  The feature contractions
// reuse the phidotU tile of the SGLD path.
#include "device_util.h"
#include <cstdio>

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

// out[a] = alpha · Σ_i A[a + p·i] · y[i] in two launches: partial sums over column chunks of
// kGemvCh (threads over a: every load of a column is coalesced; one thread per a, as the round-4
// kernel had, ran 80 000 serial loads on 2 workgroups: 19.5 ms per MovieLens w draw), then the
// chunks added in chunk order (deterministic).
constexpr int kGemvCh = 256;
__global__ __launch_bounds__(256) void gemv_part_kernel(const double* __restrict__ A, int p,
                                                        long long N, const double* __restrict__ y,
                                                        double* __restrict__ part) {
  const int a = blockIdx.y * 256 + threadIdx.x;
  const long long i0 = (long long)blockIdx.x * kGemvCh;
  const int cnt = (int)min((long long)kGemvCh, N - i0);
  if (a >= p) return;
  const double* col = A + (size_t)p * i0 + a;
  double s = 0.0;
#pragma unroll 8
  for (int i = 0; i < cnt; ++i) s = fma(col[(size_t)p * i], y[i0 + i], s);
  part[(size_t)blockIdx.x * p + a] = s;
}
__global__ __launch_bounds__(256) void gemv_fin_kernel(const double* __restrict__ part, int p,
                                                       int nch, double alpha,
                                                       double* __restrict__ out) {
  const int a = blockIdx.x * 256 + threadIdx.x;
  if (a >= p) return;
  double s = 0.0;
  for (int c = 0; c < nch; ++c) s += part[(size_t)c * p + a];
  out[a] = alpha * s;
}

static hipError_t launch_gemv(const double* A, int p, long long N, const double* y, double alpha,
                              double* out, hipStream_t st) {
  const int nch = (int)((N + kGemvCh - 1) / kGemvCh);
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, 8 * (size_t)nch * p, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gemv_part_kernel, dim3(nch, (p + 255) / 256), dim3(256), 0, st, A, p, N, y,
                     part);
  hipLaunchKernelGGL(gemv_fin_kernel, dim3((p + 255) / 256), dim3(256), 0, st, part, p, nch, alpha,
                     out);
  e = hipGetLastError();
  (void)hipFreeAsync(part, st);
  return e;
}

__global__ void axpy_kernel(double* __restrict__ x, const double* __restrict__ z, int p) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a < p) x[a] += z[a];
}

__global__ void gmc_sum_kernel(const double* __restrict__ a, const double* __restrict__ b,
                               double* __restrict__ out, int p) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < p) out[e] = a[e] + b[e];
}

// z[e] = element e of Philox normal stream (c1, c2, c3)
__global__ void normals_kernel(double* __restrict__ z, int cnt, uint64_t seed, uint32_t c1,
                               uint32_t c2, uint32_t c3) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < cnt) z[e] = normal_at(seed, (uint32_t)e, c1, c2, c3);
}

// In-place lower Cholesky of the SPD matrix M (column-major p × p, lower triangle read), one
// workgroup: right-looking, column by column (p > kCholPMax; chol_blk_kernel below otherwise).
// status = 1 if a pivot is not positive.
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

// Blocked form for p <= kCholPMax, one workgroup of kTgpNT threads, panels of kCholNB columns
// (the p = 400 w precision of GPT_fullw_gibbs at r = 20 took 5.3 ms with the column kernel):
//  1. the panel (rows j0..p-1) -> LDS, rows padded to kCholS doubles (conflict-free per lane row);
//  2. wave 0 factors the diagonal block in registers (lane i holds row i; pivots and multipliers
//     broadcast by v_readlane);
//  3. every thread solves one panel row against it (L21 = A21·L11⁻ᵀ);
//  4. the trailing lower triangle takes the rank-kCholNB update: a wave task is 64 consecutive
//     rows (lane = row, its panel row in registers) × 4 consecutive columns (their panel rows read
//     as LDS broadcasts), a coalesced read-modify-write of M per column.
// The factor is also written transposed into the upper triangle (Lᵀ, row j of L = column j of
// the upper part), which the transposed solve reads column-wise (trsv_blk_kernel).
constexpr int kCholNB = 16;
constexpr int kCholS = 18;
constexpr int kCholPMax = 1024;
#ifndef GPT_CHOL_STAMPS
#define GPT_CHOL_STAMPS 0
#endif
#ifndef GPT_CHOL_EXP
#define GPT_CHOL_EXP 0              // diagnostic builds: 1 no C loads, 2 no C stores, 3 no MFMA
#endif
#if GPT_CHOL_STAMPS
__device__ long long g_chol_stamps[64 * 8];       // per panel: phase-end shader clocks (thread 0)
#define CHOL_STAMP(ph) do { if (tid == 0 && j0 / kCholNB < 64) g_chol_stamps[(j0 / kCholNB) * 8 + (ph)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define CHOL_STAMP(ph) do {} while (0)
#endif
__global__ __launch_bounds__(kTgpNT) void chol_blk_kernel(double* __restrict__ M, int p,
                                                          int32_t* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) double Pn[kCholPMax * kCholS];   // 144 KB
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int j0 = 0; j0 < p; j0 += kCholNB) {
    CHOL_STAMP(0);
    // a last panel narrower than kCholNB is padded with identity columns: the padded block
    // factors to [L11 0; 0 I] and its zero columns add nothing below, so no step needs a guard
    const int nb = min(kCholNB, p - j0), rows = p - j0;
    for (int e = tid; e < rows * kCholNB; e += kTgpNT) {        // panel -> LDS (coalesced over i)
      const int jj = e / rows, i = e - jj * rows;
      Pn[i * kCholS + jj] = jj < nb ? M[(size_t)(j0 + i) + (size_t)p * (j0 + jj)]
                                    : (i == jj ? 1.0 : 0.0);
    }
    __syncthreads();
    CHOL_STAMP(1);
    if (wv == 0) {                                               // diagonal block, one wave
      // dpotf2's form: the pivot's square root, then its reciprocal scales the column
      double rw[kCholNB];
#pragma unroll
      for (int k = 0; k < kCholNB; ++k)
        rw[k] = lane < nb ? Pn[lane * kCholS + k] : (k == lane ? 1.0 : 0.0);
      bool bad = false;
      double rdg = 0.0;                                          // lane j: 1 / L[j][j]
#pragma unroll
      for (int j = 0; j < kCholNB; ++j) {
        const double d = readlane_d(rw[j], j);
        bad |= !(d > 0.0);
        const double pv = sqrt(d), rp = 1.0 / pv;
        if (lane == j) { rw[j] = pv; rdg = rp; }
        if (lane > j) rw[j] = rw[j] * rp;
#pragma unroll
        for (int k = j + 1; k < kCholNB; ++k) {
          const double lkj = readlane_d(rw[j], k);
          if (lane >= k) rw[k] -= rw[j] * lkj;
        }
      }
      if (lane == 0 && bad) *status = 1;
      if (lane < kCholNB) {
#pragma unroll
        for (int k = 0; k < kCholNB; ++k) Pn[lane * kCholS + k] = k <= lane ? rw[k] : 0.0;
        Pn[lane * kCholS + kCholNB] = rdg;                       // the row's pad slot
      }
    }
    __syncthreads();
    CHOL_STAMP(2);
    for (int i = kCholNB + tid; i < rows; i += kTgpNT) {        // L21 = A21 · L11⁻ᵀ, a row each
      double x[kCholNB];
#pragma unroll
      for (int j = 0; j < kCholNB; ++j) {
        double s2 = Pn[i * kCholS + j];
#pragma unroll
        for (int k = 0; k < j; ++k) s2 -= x[k] * Pn[j * kCholS + k];
        x[j] = s2 * Pn[j * kCholS + kCholNB];
      }
#pragma unroll
      for (int j = 0; j < kCholNB; ++j) Pn[i * kCholS + j] = x[j];
    }
    __syncthreads();
    CHOL_STAMP(3);
    for (int e = tid; e < rows * nb; e += kTgpNT) {             // the factored panel -> M (L)
      const int jj = e / rows, i = e - jj * rows;
      if (i >= jj) M[(size_t)(j0 + i) + (size_t)p * (j0 + jj)] = Pn[i * kCholS + jj];
    }
    for (int e = tid; e < rows * kCholNB; e += kTgpNT) {        // and transposed (Lᵀ), row-wise
      const int i = e / kCholNB, jj = e - i * kCholNB;
      if (jj < nb && i >= jj) M[(size_t)(j0 + jj) + (size_t)p * (j0 + i)] = Pn[i * kCholS + jj];
    }
    CHOL_STAMP(4);
    // trailing update of rows / cols j0+16 .. p-1 (lower triangle): C -= L21·L21ᵀ in 16 × 16
    // tiles on the fp64 matrix cores (v_mfma_f64_16x16x4f64, K = 16 in four steps), one tile
    // per wave at a time; lane λ feeds L21[tile row λ&15][k0 + (λ>>4)] for both operands and
    // holds C[(λ>>4) + 4q][λ&15] (as syrk_mfma_kernel)
    const int rem = rows - kCholNB;
    if (rem > 0) {
      // the MFMA computes the tile transposed (first operand from the column tile), so lane λ
      // holds C[r0 + (λ&15)][c0 + (λ>>4) + 4q]: each load / store of C covers 16 consecutive rows
      // of 4 columns (a few cache lines) instead of 16 columns
      const int T = (rem + 15) / 16, npair = T * (T + 1) / 2;
      const int li = lane & 15, lk = lane >> 4;
      constexpr int PW = 4;                                      // tiles of a wave in flight
      for (int t0 = wv; t0 < npair; t0 += PW * (kTgpNT / 64)) {
        int r0[PW], c0[PW];
        d4 acc[PW];
#pragma unroll
        for (int w4 = 0; w4 < PW; ++w4) {
          const int t = min(t0 + w4 * (kTgpNT / 64), npair - 1);
          int ti = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) / 2.0);
          while (ti * (ti + 1) / 2 > t) --ti;
          while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
          const int tj = t - ti * (ti + 1) / 2;
          r0[w4] = kCholNB + 16 * ti;                            // panel-relative
          c0[w4] = kCholNB + 16 * tj;
          const int row = r0[w4] + li;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int col = c0[w4] + lk + 4 * q;
#if GPT_CHOL_EXP == 1
            acc[w4][q] = 0.0 * row * col;
#else
            acc[w4][q] = (row < rows && col < rows) ? M[(size_t)(j0 + row) + (size_t)p * (j0 + col)]
                                                    : 0.0;
#endif
          }
        }
#pragma unroll
        for (int w4 = 0; w4 < PW; ++w4) {
          const int ra = min(r0[w4] + li, rows - 1), rb = min(c0[w4] + li, rows - 1);
#pragma unroll
          for (int s4 = 0; s4 < kCholNB / 4; ++s4) {
            const double av = -Pn[rb * kCholS + 4 * s4 + lk];
            const double bv = Pn[ra * kCholS + 4 * s4 + lk];
#if GPT_CHOL_EXP == 3
            acc[w4][0] += av * bv;
#else
            acc[w4] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[w4], 0, 0, 0);
#endif
          }
        }
#pragma unroll
        for (int w4 = 0; w4 < PW; ++w4) {
          if (t0 + w4 * (kTgpNT / 64) >= npair) break;
          const int row = r0[w4] + li;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int col = c0[w4] + lk + 4 * q;
#if GPT_CHOL_EXP == 2
            if (row < rows && col < rows && row >= col && acc[w4][q] == 12345.678)
#else
            if (row < rows && col < rows && row >= col)
#endif
              M[(size_t)(j0 + row) + (size_t)p * (j0 + col)] = acc[w4][q];
          }
        }
      }
    }
    CHOL_STAMP(5);
    __syncthreads();
    CHOL_STAMP(6);
  }
}

// x := L⁻¹ x (TRANS = 0) or L⁻ᵀ x (TRANS = 1) after chol_blk_kernel (L in the lower triangle, Lᵀ
// in the upper one), p <= kCholPMax, one workgroup of 256 threads with x in LDS, in blocks of
// kCholNB columns: wave 0 solves the block's triangle in registers (lane = row, pivots broadcast
// by v_readlane), then every thread updates its rows with the block's kCholNB solved values
// (column-major reads, coalesced over the rows).  The same operations in the same order as the
// column kernel (trsv_kernel): identical doubles, two block barriers per kCholNB columns instead
// of two per column.
template <int TRANS>
__global__ __launch_bounds__(256) void trsv_blk_kernel(const double* __restrict__ L, int p,
                                                       double* __restrict__ x) {
  constexpr int RPT = kCholPMax / 256;              // rows per thread
  __shared__ double xs[kCholPMax];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < p; i += 256) xs[i] = x[i];
  const int nblk = (p + kCholNB - 1) / kCholNB;
  // forward: blocks in order; transposed: from the last block (its rows jb0 .. jb1-1) down
  auto range = [&](int bi, int& jb0, int& jb1) {
    jb0 = TRANS ? max(0, p - (bi + 1) * kCholNB) : bi * kCholNB;
    jb1 = TRANS ? p - bi * kCholNB : min(p, jb0 + kCholNB);
  };
  // lane r (< nb) of wave 0 holds row jb0 + r of the block's triangle: forward,
  // L[jb0+r][jb0+k] (k <= r); transposed, Lᵀ[jb0+r][jb0+k] = L[jb0+k][jb0+r] from the upper part
  // (k >= r).  Loaded one block ahead.
  double rw[kCholNB];
  auto load_tri = [&](int bi) {
    int jb0, jb1;
    range(bi, jb0, jb1);
    const int nb = jb1 - jb0, rr = jb0 + min(lane, nb - 1);
#pragma unroll
    for (int k = 0; k < kCholNB; ++k) rw[k] = k < nb ? L[(size_t)rr + (size_t)p * (jb0 + k)] : 1.0;
  };
  if (wv == 0) load_tri(0);
  __syncthreads();
  for (int bi = 0; bi < nblk; ++bi) {
    int jb0, jb1;
    range(bi, jb0, jb1);
    const int nb = jb1 - jb0;
    // this thread's rectangle entries, in flight while wave 0 solves the triangle
    const int r0 = TRANS ? 0 : jb1, r1 = TRANS ? jb0 : p;
    double lr[RPT][kCholNB];
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const int i = min(r0 + tid + 256 * u, p - 1);
#pragma unroll
      for (int k = 0; k < kCholNB; ++k)
        lr[u][k] = (k < nb && r0 + tid + 256 * u < r1) ? L[(size_t)i + (size_t)p * (jb0 + k)] : 0.0;
    }
    if (wv == 0) {
      double xv = lane < nb ? xs[jb0 + lane] : 0.0;
      if (!TRANS) {
#pragma unroll
        for (int j = 0; j < kCholNB; ++j) {
          if (j < nb) {
            const double xj = readlane_d(xv, j) / readlane_d(rw[j], j);
            if (lane == j) xv = xj;
            if (lane > j) xv -= rw[j] * xj;
          }
        }
      } else {
#pragma unroll
        for (int j = kCholNB - 1; j >= 0; --j) {
          if (j < nb) {
            const double xj = readlane_d(xv, j) / readlane_d(rw[j], j);
            if (lane == j) xv = xj;
            if (lane < j) xv -= rw[j] * xj;
          }
        }
      }
      if (lane < nb) xs[jb0 + lane] = xv;
      if (bi + 1 < nblk) load_tri(bi + 1);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const int i = r0 + tid + 256 * u;
      if (i < r1) {
        double s2 = xs[i];
        if (!TRANS) {
#pragma unroll
          for (int k = 0; k < kCholNB; ++k)
            if (k < nb) s2 -= lr[u][k] * xs[jb0 + k];
        } else {
#pragma unroll
          for (int k = kCholNB - 1; k >= 0; --k)
            if (k < nb) s2 -= lr[u][k] * xs[jb0 + k];
        }
        xs[i] = s2;
      }
    }
    __syncthreads();
  }
  for (int i = tid; i < p; i += 256) x[i] = xs[i];
}

static void launch_chol(double* M, int p, int32_t* status, hipStream_t st) {
  if (p <= kCholPMax)
    hipLaunchKernelGGL(chol_blk_kernel, 1, kTgpNT, 0, st, M, p, status);
  else
    hipLaunchKernelGGL(chol_kernel, 1, kTgpNT, 0, st, M, p, status);
}

// triangular solve against launch_chol's factor (the blocked forms go together: trsv_blk reads
// the transposed factor chol_blk leaves in the upper triangle)
static void launch_trsv(const double* M, int p, double* x, int trans, hipStream_t st) {
  if (p <= kCholPMax) {
    if (trans) hipLaunchKernelGGL(trsv_blk_kernel<1>, 1, 256, 0, st, M, p, x);
    else hipLaunchKernelGGL(trsv_blk_kernel<0>, 1, 256, 0, st, M, p, x);
  } else {
    hipLaunchKernelGGL(trsv_kernel, 1, kTgpNT, 0, st, M, p, x, trans);
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
    e = launch_gemv(V, q, N, y, 1.0 / s2, x, st);
    if (e != hipSuccess) break;
    launch_chol(M, q, status, st);
    launch_trsv(M, q, x, 0, st);
    hipLaunchKernelGGL(normals_kernel, nblk(q, 256), 256, 0, st, z, q, seed, (uint32_t)(it - 1),
                       (uint32_t)kTgpWNoise, 0u);
    hipLaunchKernelGGL(axpy_kernel, nblk(q, 256), 256, 0, st, x, z, q);
    launch_trsv(M, q, x, 1, st);   // W = L⁻ᵀ(L⁻¹ rhs + z)
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
      e = launch_gemv(Ck, nr, N, y, 1.0 / s2, x, st);
      if (e != hipSuccess) break;
      hipLaunchKernelGGL(normals_kernel, nblk(nr, 256), 256, 0, st, z, nr, seed, (uint32_t)(it - 1),
                         (uint32_t)kTgpUNoise, (uint32_t)k);
      hipLaunchKernelGGL(axpy_kernel, nblk(nr, 256), 256, 0, st, x, z, nr);
      launch_chol(M, nr, status, st);
      launch_trsv(M, nr, x, 0, st);
      launch_trsv(M, nr, x, 1, st);   // U_k = M⁻¹(rhs + z)
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

// out = L⁻ᵀz + M⁻¹x for the SPD precision M = L·Lᵀ (column-major p × p, factored in place) and
// z on the Philox normal stream (c1, c2, c3): the Gaussian conditional draw of a linear-Gaussian
// block (GPT_fullw_gibbs w | U, V, 100k_movielensExperiment.jl:1087-1094: mu = M \ rhs, then
// chol(M,:U) \ randn + mu).  Scratch: x (p, overwritten with the mean), z (p).
hipError_t gaussian_draw_prec(double* M, int p, double* x, uint64_t seed, uint32_t c1, uint32_t c2,
                              uint32_t c3, double* z, double* out, int32_t* status, hipStream_t st) {
  launch_chol(M, p, status, st);
  launch_trsv(M, p, x, 0, st);
  launch_trsv(M, p, x, 1, st);          // mu = M⁻¹x
  hipLaunchKernelGGL(normals_kernel, nblk(p, 256), 256, 0, st, z, p, seed, c1, c2, c3);
  launch_trsv(M, p, z, 1, st);          // L⁻ᵀz
  hipLaunchKernelGGL(gmc_sum_kernel, nblk(p, 256), 256, 0, st, z, x, out, p);
  return hipGetLastError();
}

// The same draw with M = alpha·A·Aᵀ + beta·I and x = ysc·A·y formed from the dense design A
// (p × N column-major).  Scratch: M (p²), x, z (p).
hipError_t gaussian_draw_dense(const double* A, int p, long long N, const double* y, double alpha,
                               double beta, double ysc, uint64_t seed, uint32_t c1, uint32_t c2,
                               uint32_t c3, double* M, double* x, double* z, double* out,
                               int32_t* status, hipStream_t st) {
  const int T = (p + 15) / 16;
  hipLaunchKernelGGL(syrk_mfma_kernel, nblk((long long)T * (T + 1) / 2, 4), 256, 0, st, A, p, N,
                     alpha, beta, M);
  hipError_t e = launch_gemv(A, p, N, y, ysc, x, st);
  if (e != hipSuccess) return e;
  return gaussian_draw_prec(M, p, x, seed, c1, c2, c3, z, out, status, st);
}

// ============================================================================ GPT_GMC
// Geodesic Monte Carlo (GPT_SGLD.jl:684-805): full-batch gradients from the same kernels as the
// Gibbs sweep (temp over all N rows, V, the leave-one-out run sums C), then per-dimension
// workgroups for the Stiefel kicks (proj) and the geodesic drift (geodboth, :40-59).

// fhat[i] = Σ_q V[q,i]·w[q] (q ascending); res[i] = y[i] − fhat[i]
__global__ void gmc_fhat_kernel(const double* __restrict__ V, const double* __restrict__ w,
                                const double* __restrict__ y, int Q, long long N,
                                double* __restrict__ fhat, double* __restrict__ res) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  double s = 0.0;
  for (int q = 0; q < Q; ++q) s = fma(V[q + (size_t)Q * i], w[q], s);
  fhat[i] = s;
  res[i] = y[i] - s;
}

// gw[q] = Σ_i V[q,i]·res[i] / σ² − w[q]   (σ_w = 1, GPT_SGLD.jl:725)
__global__ void gmc_gradw_kernel(const double* __restrict__ V, const double* __restrict__ res,
                                 const double* __restrict__ w, int Q, long long N, double inv_s2,
                                 double* __restrict__ gw) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  double s = 0.0;
  for (long long i = 0; i < N; ++i) s = fma(V[q + (size_t)Q * i], res[i], s);
  gw[q] = s * inv_s2 - w[q];
}

// gU[j + n·l] = Σ_i C[l,i]·res[i]·phi[j,k,i] / σ²   (Ψ_k·res, :733-736)
__global__ void gmc_gradU_kernel(const double* __restrict__ Cm, const double* __restrict__ res,
                                 const double* __restrict__ phi, int n, int D, int R, long long N,
                                 int k, double inv_s2, double* __restrict__ gU) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * R) return;
  const int l = e / n, j = e - l * n;
  double s = 0.0;
  for (long long i = 0; i < N; ++i)
    s = fma(Cm[l + (size_t)R * i] * res[i], phi[j + (size_t)n * (k + (size_t)D * i)], s);
  gU[e] = s * inv_s2;
}

__global__ void gmc_axpy_kernel(double* __restrict__ x, const double* __restrict__ z, double a,
                                int cnt) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < cnt) x[e] += a * z[e];
}

// Kick of U's momentum (one workgroup per dimension k): mom_k = proj(U_k, X), X = mom_k + c·gU_k,
// or X = ξ (GMC_MOM stream, u_noise layout) when init (the fresh momentum of :711-713).
template <int R>
__global__ __launch_bounds__(kNT) void gmc_kick_kernel(const double* __restrict__ U,
                                                       double* __restrict__ mom,
                                                       const double* __restrict__ gU, double c,
                                                       int n, int init, uint64_t seed,
                                                       uint32_t epoch) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* Ul = (double*)smem;                 // n × R column-major
  double* Xl = Ul + (size_t)n * R;
  double* Ml = Xl + (size_t)n * R;            // R × R: Ml[a·R + b] = Σ_j U[j,a]·X[j,b]
  const int k = blockIdx.x, tid = threadIdx.x;
  const size_t off = (size_t)n * R * k;
  constexpr int RE = R + (R & 1);
  for (int e = tid; e < n * R; e += kNT) {
    Ul[e] = U[off + e];
    if (!init) Xl[e] = mom[off + e] + c * gU[off + e];
  }
  if (init) {
    for (int c0 = tid; c0 < (n * RE) / 2; c0 += kNT) {
      double z0, z1;
      normal_pair(seed, (uint32_t)c0, epoch, kGmcMom, (uint32_t)k, z0, z1);
      const int e0 = 2 * c0, j = e0 / RE, l = e0 - j * RE;   // element l + RE·j
      if (l < R) Xl[j + (size_t)n * l] = z0;
      if (l + 1 < R) Xl[j + (size_t)n * (l + 1)] = z1;
    }
  }
  __syncthreads();
  for (int e = tid; e < R * R; e += kNT) {
    const int a = e / R, b = e - a * R;
    double s = 0.0;
    for (int j = 0; j < n; ++j) s = fma(Ul[j + (size_t)n * a], Xl[j + (size_t)n * b], s);
    Ml[e] = s;
  }
  __syncthreads();
  for (int j = tid; j < n; j += kNT) {
#pragma unroll
    for (int b = 0; b < R; ++b) {
      double s = 0.0;
#pragma unroll
      for (int a = 0; a < R; ++a) s = fma(Ul[j + (size_t)n * a], Ml[a * R + b] + Ml[b * R + a], s);
      mom[off + j + (size_t)n * b] = Xl[j + (size_t)n * b] - s / 2;
    }
  }
}

// Drift of U_k along its geodesic for time t (geodboth, :40-59), one workgroup per dimension:
// E = expm(t[A −S; I A]) (wave 0), expm(−tA) (wave 1), U ← normalise([U mom]·E[:,1:r]·expm(−tA)),
// mom ← [U mom]·E[:,r+1:2r]·expm(−tA).  status = 1 on a NaN in E.
template <int R>
__global__ __launch_bounds__(kNT) void gmc_geod_kernel(double* __restrict__ U,
                                                       double* __restrict__ mom, double t, int n,
                                                       int32_t* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NN = 2 * R;
  double* Ul = (double*)smem;
  double* Ml = Ul + (size_t)n * R;
  double* Ag = Ml + (size_t)n * R;           // R × R   Uᵀmom
  double* Sg = Ag + R * R;                   // R × R   momᵀmom
  double* X0 = Sg + R * R;                   // 7·NN² expm scratch (E at X0 + NN²)
  double* X1 = X0 + 7 * NN * NN;             // 7·R² expm scratch (expm(−tA) at X1 + R²)
  double* F = X1 + 7 * R * R;                // NN × NN: [E[:,1:r]·mx | E[:,r+1:2r]·mx]
  double* nr = F + NN * NN;                  // R column norms
  int& bad = *(int*)(nr + R);                // NaN flag of the expm
  const int k = blockIdx.x, tid = threadIdx.x, wv = tid >> 6;
  const size_t off = (size_t)n * R * k;
  for (int e = tid; e < n * R; e += kNT) { Ul[e] = U[off + e]; Ml[e] = mom[off + e]; }
  if (tid == 0) bad = 0;
  __syncthreads();
  for (int e = tid; e < 2 * R * R; e += kNT) {
    const int g = e / (R * R), ab = e - g * R * R, a = ab / R, b = ab - a * R;
    const double* P = g ? Ml : Ul;
    double s = 0.0;
    for (int j = 0; j < n; ++j) s = fma(P[j + (size_t)n * a], Ml[j + (size_t)n * b], s);
    (g ? Sg : Ag)[ab] = s;
  }
  __syncthreads();
  if (wv == 0) {
    for (int o = tid; o < NN * NN; o += 64) {
      const int i = o / NN, j = o - i * NN;
      double v;
      if (i < R) v = j < R ? Ag[i * R + j] : -Sg[i * R + (j - R)];
      else v = j < R ? (i - R == j ? 1.0 : 0.0) : Ag[(i - R) * R + (j - R)];
      X0[o] = t * v;
    }
    wave_sync();
    if (wave_expm<NN>(X0) && tid == 0) bad = 1;
  } else if (wv == 1) {
    const int ln = tid & 63;
    for (int o = ln; o < R * R; o += 64) X1[o] = -t * Ag[o];
    wave_sync();
    wave_expm<R>(X1);
  }
  __syncthreads();
  if (bad) {
    if (tid == 0) *status = 1;
    return;
  }
  const double* E = X0 + NN * NN;
  const double* mx = X1 + R * R;
  for (int o = tid; o < NN * NN; o += kNT) {       // F[a][h·R + l] = Σ_c E[a][h·R + c]·mx[c][l]
    const int a = o / NN, hl = o - a * NN, h = hl / R, l = hl - h * R;
    double s = 0.0;
#pragma unroll
    for (int c2 = 0; c2 < R; ++c2) s = fma(E[a * NN + h * R + c2], mx[c2 * R + l], s);
    F[o] = s;
  }
  __syncthreads();
  for (int j = tid; j < n; j += kNT) {
    double x[NN];
#pragma unroll
    for (int a = 0; a < R; ++a) { x[a] = Ul[j + (size_t)n * a]; x[R + a] = Ml[j + (size_t)n * a]; }
#pragma unroll
    for (int hl = 0; hl < NN; ++hl) {
      double s = 0.0;
#pragma unroll
      for (int a = 0; a < NN; ++a) s = fma(x[a], F[a * NN + hl], s);
      if (hl < R) Ul[j + (size_t)n * hl] = s;                 // tmpU (normalised below)
      else mom[off + j + (size_t)n * (hl - R)] = s;           // tmpV
    }
  }
  __syncthreads();
  for (int l = tid; l < R; l += kNT) {
    double s = 0.0;
    for (int j = 0; j < n; ++j) s = fma(Ul[j + (size_t)n * l], Ul[j + (size_t)n * l], s);
    nr[l] = sqrt(s);
  }
  __syncthreads();
  for (int e = tid; e < n * R; e += kNT) U[off + e] = Ul[e] / nr[e / n];
}

// out[0] = −|w|²/2 − |res|²/(2σ²) − |mom|²/2 − |p|²/2   (H, GPT_SGLD.jl:714, :795)
__global__ __launch_bounds__(kNT) void gmc_energy_kernel(const double* __restrict__ w,
                                                         const double* __restrict__ p, int Q,
                                                         const double* __restrict__ res,
                                                         long long N, const double* __restrict__ mom,
                                                         long long nm, double inv_2s2,
                                                         double* __restrict__ out) {
  __shared__ double red[kNW];
  double a = 0.0, b = 0.0, c = 0.0, d = 0.0;
  for (int q = threadIdx.x; q < Q; q += kNT) { a = fma(w[q], w[q], a); d = fma(p[q], p[q], d); }
  for (long long i = threadIdx.x; i < N; i += kNT) b = fma(res[i], res[i], b);
  for (long long e = threadIdx.x; e < nm; e += kNT) c = fma(mom[e], mom[e], c);
  const double sa = blk_sum(a, red), sb = blk_sum(b, red), sc = blk_sum(c, red), sd = blk_sum(d, red);
  if (threadIdx.x == 0) out[0] = -sa / 2 - sb * inv_2s2 - sc / 2 - sd / 2;
}

static size_t gmc_kick_lds(int n, int r) { return 8 * ((size_t)2 * n * r + (size_t)r * r); }
static size_t gmc_geod_lds(int n, int r) {
  return 8 * ((size_t)2 * n * r + 2 * (size_t)r * r + 7 * 4 * (size_t)r * r + 7 * (size_t)r * r +
              4 * (size_t)r * r + r + 1);
}

bool gmc_supported(int n, int r) {
  return gmc_geod_lds(n, r) <= 160 * 1024 && gmc_kick_lds(n, r) <= 160 * 1024;
}

static hipError_t launch_gmc_kick(const double* U, double* mom, const double* gU, double c, int n,
                                  int D, int r, int init, uint64_t seed, uint32_t epoch,
                                  hipStream_t st) {
  const size_t lds = gmc_kick_lds(n, r);
  switch (r) {
#define CASE(RR)                                                                              \
  case RR: {                                                                                  \
    static std::atomic<uint64_t> attr{0};                                                         \
    hipError_t e = set_max_lds_once((const void*)gmc_kick_kernel<RR>, 160 * 1024, attr);          \
    if (e != hipSuccess) return e;                                                                \
    hipLaunchKernelGGL(gmc_kick_kernel<RR>, dim3(D), dim3(kNT), lds, st, U, mom, gU, c, n, init, \
                       seed, epoch);                                                          \
  } break;
    GPT_TGP_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

static hipError_t launch_gmc_geod(double* U, double* mom, double t, int n, int D, int r,
                                  int32_t* status, hipStream_t st) {
  const size_t lds = gmc_geod_lds(n, r);
  switch (r) {
#define CASE(RR)                                                                              \
  case RR: {                                                                                  \
    static std::atomic<uint64_t> attr{0};                                                         \
    hipError_t e = set_max_lds_once((const void*)gmc_geod_kernel<RR>, 160 * 1024, attr);          \
    if (e != hipSuccess) return e;                                                                \
    hipLaunchKernelGGL(gmc_geod_kernel<RR>, dim3(D), dim3(kNT), lds, st, U, mom, t, n, status); \
  } break;
    GPT_TGP_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Full-data gradients at (w, U): fhat/res, gw, gU (all device; scratch temp (D·r·N), V (Q·N),
// Cm (r·N)).
static hipError_t gmc_gradients(const double* phi, const double* y, const int32_t* I0,
                                 const double* w, const double* U, int n, int D, long long N,
                                 int r, int Q, double inv_s2, double* temp, double* V, double* Cm,
                                 double* fhat, double* res, double* gw, double* gU,
                                 hipStream_t st) {
  hipError_t e = launch_tgp_temp(U, phi, n, D, N, r, 0, D, temp, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(tgp_v_kernel, nblk((long long)Q * N, 256), 256, 0, st, temp, I0, Q, D, r, N, V);
  hipLaunchKernelGGL(gmc_fhat_kernel, nblk(N, 256), 256, 0, st, V, w, y, Q, N, fhat, res);
  hipLaunchKernelGGL(gmc_gradw_kernel, nblk(Q, 64), 64, 0, st, V, res, w, Q, N, inv_s2, gw);
  for (int k = 0; k < D; ++k) {
    hipLaunchKernelGGL(tgp_c_kernel, nblk((long long)r * N, 256), 256, 0, st, V, w, temp, I0, Q, r,
                       N, k, Cm);
    hipLaunchKernelGGL(gmc_gradU_kernel, nblk((long long)n * r, 64), 64, 0, st, Cm, res, phi, n, D,
                       r, N, k, inv_s2, gU + (size_t)n * r * k);
  }
  return hipGetLastError();
}

hipError_t gmc_run(const double* phi, const double* y, const int32_t* I0, int n, int D,
                   long long N, int r, int Q, double signal_var, double epsw, double epsU,
                   int burnin, int maxepoch, int L, uint64_t seed, double* w, double* U,
                   double* w_store, double* U_store, double* accept, int32_t* status,
                   hipStream_t st) {
  const size_t nm = (size_t)n * r * D;
  const double inv_s2 = 1.0 / signal_var, sw = sqrt(epsw), su = sqrt(epsU);
  double *temp = nullptr, *V = nullptr, *Cm = nullptr, *fhat = nullptr, *res = nullptr,
         *gw = nullptr, *gU = nullptr, *p = nullptr, *mom = nullptr, *w_old = nullptr, *Hd = nullptr;
  hipError_t e = hipSuccess;
  auto al = [&](double** q, size_t cnt) {
    if (e == hipSuccess) e = hipMallocAsync((void**)q, 8 * (cnt ? cnt : 1), st);
  };
  al(&temp, (size_t)D * r * N); al(&V, (size_t)Q * N); al(&Cm, (size_t)r * N); al(&fhat, N);
  al(&res, N); al(&gw, Q); al(&gU, nm); al(&p, Q); al(&mom, nm); al(&w_old, Q); al(&Hd, 2);
#define GMC_CK(stage)                                                                        \
  do {                                                                                       \
    if (e == hipSuccess) e = hipGetLastError();                                              \
    if (e != hipSuccess) {                                                                   \
      fprintf(stderr, "gpt_gmc: %s failed: %s\n", stage, hipGetErrorString(e));              \
    }                                                                                        \
  } while (0)
  GMC_CK("alloc");
  auto grads = [&]() {
    return gmc_gradients(phi, y, I0, w, U, n, D, N, r, Q, inv_s2, temp, V, Cm, fhat, res, gw, gU, st);
  };
  auto kick = [&]() {
    hipLaunchKernelGGL(gmc_axpy_kernel, nblk(Q, 256), 256, 0, st, p, gw, sw / 2, Q);
    return launch_gmc_kick(U, mom, gU, su / 2, n, D, r, 0, seed, 0, st);
  };
  for (int epoch = 1; epoch <= burnin + maxepoch && e == hipSuccess; ++epoch) {
    e = hipMemcpyAsync(w_old, w, 8 * (size_t)Q, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) break;
    hipLaunchKernelGGL(normals_kernel, nblk(Q, 256), 256, 0, st, p, Q, seed, (uint32_t)(epoch - 1),
                       (uint32_t)kGmcP, 0u);
    e = launch_gmc_kick(U, mom, nullptr, 0.0, n, D, r, 1, seed, (uint32_t)(epoch - 1), st);
    GMC_CK("momentum draw");
    if (e == hipSuccess) e = grads();
    GMC_CK("gradients");
    if (e != hipSuccess) break;
    hipLaunchKernelGGL(gmc_energy_kernel, 1, kNT, 0, st, w, p, Q, res, N, mom, (long long)nm,
                       inv_s2 / 2, Hd);
    for (int l = 0; l < L && e == hipSuccess; ++l) {
      e = kick();
      if (e != hipSuccess) break;
      hipLaunchKernelGGL(gmc_axpy_kernel, nblk(Q, 256), 256, 0, st, w, p, sw, Q);
      GMC_CK("kick/drift");
      if (e == hipSuccess) e = launch_gmc_geod(U, mom, su, n, D, r, status, st);
      GMC_CK("geodesic");
      if (e == hipSuccess) e = grads();
      GMC_CK("gradients");
      if (e == hipSuccess) e = kick();
      GMC_CK("kick");
    }
    if (e != hipSuccess) break;
    hipLaunchKernelGGL(gmc_energy_kernel, 1, kNT, 0, st, w, p, Q, res, N, mom, (long long)nm,
                       inv_s2 / 2, Hd + 1);
    double H[2];
    int32_t bad = 0;
    e = hipMemcpyAsync(H, Hd, 16, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(&bad, status, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    GMC_CK("energy");
    if (e != hipSuccess || bad) break;
    const double ap = exp(H[1] - H[0]);
    accept[epoch - 1] = ap;
    const U4 x = philox4x32(0u, (uint32_t)(epoch - 1), kGmcU, 0u, seed);
    if (u53(x.x, x.y) > ap)                  // reject: w only (U_old aliases U, :710/:798-800)
      e = hipMemcpyAsync(w, w_old, 8 * (size_t)Q, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess && epoch > burnin) {
      e = hipMemcpyAsync(w_store + (size_t)Q * (epoch - burnin - 1), w, 8 * (size_t)Q,
                         hipMemcpyDeviceToHost, st);
      if (e == hipSuccess)
        e = hipMemcpyAsync(U_store + nm * (epoch - burnin - 1), U, 8 * nm, hipMemcpyDeviceToHost, st);
    }
  }
  GMC_CK("stores");
#undef GMC_CK
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  for (double* q : {temp, V, Cm, fhat, res, gw, gU, p, mom, w_old, Hd})
    if (q) (void)hipFreeAsync(q, st);
  (void)hipStreamSynchronize(st);
  return e;
}

}  // namespace gpt
