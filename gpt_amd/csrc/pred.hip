// Test-set prediction and RMSE reductions (GPT_SGLD.jl:233-243; GPT_SGLD_p.jl:124-132;
// kin40kExperiment.jl:78-87).
#include <mutex>

#include "device_util.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

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

// ---- stacked-sample prediction on the fp64 matrix cores (GPT_SGLD.jl:233-243 over S samples)
//
// phidotU of S samples at once is one GEMM per dimension k:
//   T[s][i/64][k·R + l][i%64] = Σ_j U_s[j, l, k] · phi[j, k, i]     (M = S·R, N = Ntest, K = n)
// (tile-contiguous: the V-phase reads a (sample, 64 rows) tile's D·R rows as one block)
// run on v_mfma_f64_16x16x4f64, then the V-phase (computeV / computefhat) per (sample, 64-row tile)
// reads its R·D temp rows.  Both operands are K(j)-contiguous; lane λ feeds the K pair
// j0 + 2(λ>>4) + {0,1} of row/column λ&15 as one 16-B load and the two halves go to two MFMAs
// (any K order common to A and B is the same sum).  A workgroup = 4 waves = a 64(c) × 64(i)
// tile, each wave 2 × 2 MFMA tiles.  Workgroups are numbered so that the c-tiles of one
// (i-tile, k) land on the same XCD (dispatch is round-robin over the 8 XCDs): phi[:, k, tile] is
// then fetched into one L2 and reused there by every c-tile.
typedef double pd4 __attribute__((ext_vector_type(4)));
typedef double pd2 __attribute__((ext_vector_type(2)));
constexpr int kXcds = 8;

template <bool V2, int TM, int TN>
__global__ __launch_bounds__(256) void pred_temp_mfma_kernel(const double* __restrict__ U,
                                                             const double* __restrict__ phi,
                                                             int n, int D, int R,
                                                             long long Ntest, int S,
                                                             double* __restrict__ T,
                                                             long long nti64) {
  constexpr int WC = 32 * TM, WI = 32 * TN;        // workgroup tile (2 × 2 waves of 16TM × 16TN)
  const int SR = S * R;
  const int nct = (SR + WC - 1) / WC;
  const long long nit = (Ntest + WI - 1) / WI;
  const long long total = (long long)nct * nit * D;
  const long long per = ((long long)gridDim.x) / kXcds;
  const long long logical = (long long)(blockIdx.x % kXcds) * per + blockIdx.x / kXcds;
  if (logical >= total) return;
  const int ct = (int)(logical % nct);
  const long long rest = logical / nct;
  const long long it = rest % nit;
  const int k = (int)(rest / nit);
  const int lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6), kl = lane >> 4;
  const int cw = ct * WC + (wv & 1) * 16 * TM;
  const long long iw = it * WI + (wv >> 1) * 16 * TN;
  const __attribute__((address_space(1))) double* pa[TM];
  const __attribute__((address_space(1))) double* pb[TN];
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    const int c = cw + 16 * t + (lane & 15);
    const int cc = c < SR ? c : 0, sm = cc / R, l = cc - sm * R;
    pa[t] = gptr(U + (size_t)sm * n * R * D + (size_t)n * (l + R * k));
  }
#pragma unroll
  for (int u = 0; u < TN; ++u) {
    const long long i = iw + 16 * u + (lane & 15);
    pb[u] = gptr(phi + (size_t)n * (k + (size_t)D * (i < Ntest ? i : 0)));
  }
  pd4 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u) acc[t][u] = pd4{0.0, 0.0, 0.0, 0.0};
  // Branch- and select-free operand loads in the K loop (address clamped in-row): lanes of
  // columns c >= S·R or rows i >= Ntest read row 0 and only feed outputs that are never stored,
  // so the loaded values go straight into the MFMAs and the loads of one step stay in flight
  // across the other step's MFMAs.  Only the K tail (j >= n) is zeroed, after the loop.
  auto ld = [&](const __attribute__((address_space(1))) double* p, int j, double& x0, double& x1) {
    if constexpr (V2) {              // n even: j even, rows 16-B aligned
      const pd2 v = *(const __attribute__((address_space(1))) pd2*)(p + min(j, n - 2));
      x0 = v[0]; x1 = v[1];
    } else {
      x0 = p[min(j, n - 1)];
      x1 = p[min(j + 1, n - 1)];
    }
  };
  struct Ops { double a0[TM], a1[TM], b0[TN], b1[TN]; };
  auto load = [&](int j, Ops& o) {
#pragma unroll
    for (int t = 0; t < TM; ++t) ld(pa[t], j, o.a0[t], o.a1[t]);
#pragma unroll
    for (int u = 0; u < TN; ++u) ld(pb[u], j, o.b0[u], o.b1[u]);
  };
  auto ktail = [&](int j, Ops& o) {    // zero the A halves past n (one operand suffices)
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      o.a0[t] = j < n ? o.a0[t] : 0.0;
      o.a1[t] = j + 1 < n ? o.a1[t] : 0.0;
    }
  };
  // every accumulator with the even K half, then with the odd one (TM·TN >= 4 independent MFMAs
  // between two on one accumulator)
  auto mma = [&](const Ops& o) {
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.a0[t], o.b0[u], acc[t][u], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.a1[t], o.b1[u], acc[t][u], 0, 0, 0);
  };
  // two K steps of 8 per iteration over the full 16-blocks, ping-ponging two operand sets: one
  // step's loads are in flight while the other step's MFMAs run; then the masked tail
  const int nfull = n & ~15;
  Ops X, Y;
  load(2 * kl, X);
  for (int j0 = 0; j0 < nfull; j0 += 16) {
    load(j0 + 8 + 2 * kl, Y);
    mma(X);
    load(j0 + 16 + 2 * kl, X);
    mma(Y);
  }
  if (nfull < n) {
    load(nfull + 8 + 2 * kl, Y);
    ktail(nfull + 2 * kl, X);
    ktail(nfull + 8 + 2 * kl, Y);
    mma(X);
    mma(Y);
  }
  // D[row = (λ>>4) + 4·reg][col = λ&15]: row ↔ c, col ↔ i (16 consecutive i per store)
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int c = cw + 16 * t + kl + 4 * reg;
        const long long i = iw + 16 * u + (lane & 15);
        if (c < SR && i < Ntest) {
          const int sm = c / R, l = c - sm * R;
          gptr_w(T)[((((size_t)sm * nti64 + (size_t)(i >> 6)) * D + k) * R + l) * 64 + (i & 63)] =
              acc[t][u][reg];
        }
      }
}

// V-phase over the stacked temp with lanes as test rows: one wave = (sample s, 64 rows); the
// wave stages its D·R temp rows (64 doubles each, coalesced) into LDS, then for every core entry q
// the D factors temp[k, I[q,k]] are lane-contiguous LDS reads (no bank conflicts) at offsets the
// whole wave shares, taken from a (q, k) table by scalar loads.
__global__ void pred_offs_kernel(const int32_t* __restrict__ I0, int Q, int D, int R,
                                 int32_t* __restrict__ offs) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= Q * D) return;
  const int q = x / D, k = x - q * D;
  offs[x] = (int32_t)((k * R + I0[q + Q * k]) * 64);
}

// kRowsWaves waves share one (sample, 64 rows) tile: they stage its D·R temp rows together and
// split the core entries (contiguous ranges of q), adding their partial sums in wave order.  With
// one wave per tile (round 4) a tile's 82 KB of LDS at r = 20, D = 8 left one wave per CU: 7.7 ms
// per 224-sample call, against the 7.1 ms GEMM.
constexpr int kRowsWaves = 16;
__global__ __launch_bounds__(64 * kRowsWaves) void pred_vphase_rows_kernel(
    const double* __restrict__ w, const double* __restrict__ T, const int32_t* __restrict__ offs,
    int D, int R, long long Ntest, int Q, double* __restrict__ fhat) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* tl = (double*)smem;                       // [k·R + l][64]
  double* part = tl + (size_t)D * R * 64;           // [wave][64]
  const int lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6);
  const int s = blockIdx.y;
  const long long i0 = (long long)blockIdx.x * 64;
  const long long i = i0 + lane;
  const bool ok = i < Ntest;
  const double* Ts = T + ((size_t)s * ((Ntest + 63) / 64) + blockIdx.x) * D * R * 64 + lane;
  for (int row = wv; row < D * R; row += kRowsWaves) tl[row * 64 + lane] = gptr(Ts)[(size_t)row * 64];
  __syncthreads();
  const auto* ofq = cptr(offs);
  const auto* wq = cptr(w + (size_t)s * Q);
  const int qa = Q * wv / kRowsWaves, qb = Q * (wv + 1) / kRowsWaves;
  double f0 = 0.0, f1 = 0.0;
  int q = qa;
  for (; q + 2 <= qb; q += 2) {
    double v0 = wq[q], v1 = wq[q + 1];
    for (int k = 0; k < D; ++k) {
      v0 *= tl[ofq[q * D + k] + lane];
      v1 *= tl[ofq[(q + 1) * D + k] + lane];
    }
    f0 += v0;
    f1 += v1;
  }
  if (q < qb) {
    double v0 = wq[q];
    for (int k = 0; k < D; ++k) v0 *= tl[ofq[q * D + k] + lane];
    f0 += v0;
  }
  part[wv * 64 + lane] = f0 + f1;
  __syncthreads();
  if (wv == 0) {
    double f = part[lane];
#pragma unroll
    for (int x = 1; x < kRowsWaves; ++x) f += part[x * 64 + lane];
    if (ok) fhat[(size_t)s * Ntest + i] = f;
  }
}

// The rows V-phase as a persistent loop over (sample, 64-row) tiles: every workgroup (one per CU,
// the tile's D·R rows take ~80 KB of LDS at r = 20) keeps the rows of its next two tiles in
// flight in registers (up to 16 per lane and wave each) while its waves run the current tile's
// core entries from LDS, so the tiles' HBM reads overlap the LDS work instead of alternating with
// it (one tile ahead behind __syncthreads, which waits for them: 3.7 ms per 224-sample call).  DD > 0: D as a
// compile-time constant, so a core entry's D offsets are one scalar load and its D LDS reads are
// issued together (with a runtime D each factor waited for its offset's scalar load and then its
// LDS read, one after the other: 4.2 ms of a 10.9 ms call at r = 20).  The core-entry loop and the
// partial sums are the rows kernel's (the same doubles).
// NW waves per workgroup, NPW prefetched rows per wave.  16 waves (the launch uses 16) measured
// 3.48 ms per 224-sample r = 20 call against 5.06 ms with 8 waves whose core-entry loop keeps each
// pair's 2·D LDS reads in flight together (`profiles/r5ah_rows_vphase_waves.txt`): the tile
// stream needs the memory parallelism of 16 waves more than the loop needs the registers.
template <int DD, int NW, int NPW>
__global__ __launch_bounds__(64 * NW) void pred_vphase_rows_pf_kernel(
    const double* __restrict__ w, const double* __restrict__ T, const int32_t* __restrict__ offs,
    int Drt, int R, long long Ntest, int Q, double* __restrict__ fhat, int S) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int D = DD > 0 ? DD : Drt;
  double* tl = (double*)smem;                       // [k·R + l][64]
  double* part = tl + (size_t)D * R * 64;           // [wave][64]
  // the core entries' offsets (Q·D, the same for every tile) and the tile's sample's w (Q) in
  // LDS: the entry loop reads them as wave-uniform LDS broadcasts, in order with its data reads
  // (as scalar loads each pair waited for its offsets — the lgkm counter is shared — and the w
  // lines of every new sample missed the scalar cache)
  int* ofl = (int*)(part + NW * 64);
  double* wl = (double*)(ofl + ((Q * (DD > 0 ? DD : Drt) + 3) & ~3));
  const int lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6);
  const int DR = D * R;
  for (int x = threadIdx.x; x < Q * D; x += 64 * NW) ofl[x] = offs[x];
  const long long nti = (Ntest + 63) / 64, ntiles = nti * S;
  // two register buffers: the rows of tile t + 2G are loaded while tile t runs and tile t + G
  // waits in the other buffer; the barriers inside the loop wait for LDS only (s_barrier after
  // lgkmcnt(0)), so these loads stay in flight across them (__syncthreads would wait for them)
  double nxa[NPW + 1], nxb[NPW + 1];                // + the sample's w entry of this thread
  const bool wreg = Q <= 64 * NW;                    // w rides with the rows (else loaded at park)
  auto fetch = [&](long long tile, double (&nx)[NPW + 1]) {
    const int s = (int)(tile / nti);
    if (wreg) nx[NPW] = w[(size_t)s * Q + min((int)threadIdx.x, Q - 1)];
    const long long i0 = (tile - (long long)s * nti) * 64, i = i0 + lane;
    const double* Ts = T + (size_t)tile * DR * 64 + lane;    // the tile's rows: one block
#pragma unroll
    for (int x = 0; x < NPW; ++x) {
      const int row = wv + NW * x;
      if (row < DR) nx[x] = gptr(Ts)[(size_t)row * 64];
    }
  };
  auto park = [&](const double (&nx)[NPW + 1], long long tile) {
#pragma unroll
    for (int x = 0; x < NPW; ++x) {
      const int row = wv + NW * x;
      if (row < DR) tl[row * 64 + lane] = nx[x];
    }
    if (wreg) {
      if ((int)threadIdx.x < Q) wl[threadIdx.x] = nx[NPW];
    } else {
      for (int x = threadIdx.x; x < Q; x += 64 * NW) wl[x] = w[(size_t)(tile / nti) * Q + x];
    }
  };
  auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  const int* ofq = ofl;
  const int qa = Q * wv / NW, qb = Q * (wv + 1) / NW;
  const long long G = gridDim.x;
  // tile t from LDS; loads of t + 2G into ld; t + G (in pk) parked at the end
  auto body = [&](long long tile, double (&ld)[NPW + 1], const double (&pk)[NPW + 1]) {
    if (tile + 2 * G < ntiles) fetch(tile + 2 * G, ld);
    const int s = (int)(tile / nti);
    const long long i = (tile - (long long)s * nti) * 64 + lane;
    const double* wq = wl;
    double f0 = 0.0, f1 = 0.0;
    int q = qa;
    for (; q + 2 <= qb; q += 2) {
      double v0 = wq[q], v1 = wq[q + 1];
      if constexpr (DD > 0) {
        int o0[DD], o1[DD];
#pragma unroll
        for (int k = 0; k < DD; ++k) { o0[k] = ofq[q * DD + k]; o1[k] = ofq[(q + 1) * DD + k]; }
        double t0[DD], t1[DD];
#pragma unroll
        for (int k = 0; k < DD; ++k) { t0[k] = tl[o0[k] + lane]; t1[k] = tl[o1[k] + lane]; }
#pragma unroll
        for (int k = 0; k < DD; ++k) { v0 *= t0[k]; v1 *= t1[k]; }
      } else {
        for (int k = 0; k < D; ++k) {
          v0 *= tl[ofq[q * D + k] + lane];
          v1 *= tl[ofq[(q + 1) * D + k] + lane];
        }
      }
      f0 += v0;
      f1 += v1;
    }
    if (q < qb) {
      double v0 = wq[q];
      for (int k = 0; k < D; ++k) v0 *= tl[ofq[q * D + k] + lane];
      f0 += v0;
    }
    part[wv * 64 + lane] = f0 + f1;
    lds_barrier();                                   // every wave is done with tl and part
    if (wv == 0) {
      double f = part[lane];
#pragma unroll
      for (int x = 1; x < NW; ++x) f += part[x * 64 + lane];
      if (i < Ntest) fhat[(size_t)s * Ntest + i] = f;
    }
    if (tile + G < ntiles) park(pk, tile + G);
    lds_barrier();
  };
  long long tile = blockIdx.x;
  if (tile >= ntiles) return;
  fetch(tile, nxa);
  if (tile + G < ntiles) fetch(tile + G, nxb);
  park(nxa, tile);
  __syncthreads();
  for (;;) {
    body(tile, nxa, nxb);
    tile += G;
    if (tile >= ntiles) break;
    body(tile, nxb, nxa);
    tile += G;
    if (tile >= ntiles) break;
  }
}

// V-phase with pair tables: the D factors of V[q, i] are taken two dimensions at a time from
// per-test-row tables PP_t[a·r + b] = temp[2t, a]·temp[2t+1, b] (an odd last dimension keeps its r
// rows), built once per (sample, 64 rows) workgroup, so a core entry costs ⌈D/2⌉ lane-contiguous LDS
// reads instead of D — the rows kernel above is bound by exactly those reads (64 lanes × 8 B at
// 128 B/clk per CU).  Four waves split the core entries; their partial sums are added in wave
// order.  V = Π_t PP_t associates the D factors pairwise (the oracle multiplies them in k order):
// the two differ by rounding only.
constexpr int kPairWaves = 4;
static int pred_pair_tables(int D) { return (D + 1) / 2; }
static int pred_pair_rows(int D, int r) { return (D / 2) * r * r + (D & 1) * r; }
static size_t pred_pairs_lds_bytes(int D, int r) {
  return 8 * (size_t)pred_pair_rows(D, r) * 64 + 8 * (size_t)kPairWaves * 64;
}

// offp[q·NT + t]: LDS offset (doubles) of core entry q's factor in table t
__global__ void pred_pair_offs_kernel(const int32_t* __restrict__ I0, int Q, int D, int R,
                                      int32_t* __restrict__ offp) {
  const int NT = (D + 1) / 2;
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= Q * NT) return;
  const int q = x / NT, t = x - q * NT;
  const int a = I0[q + Q * (2 * t)];
  const int row = 2 * t + 1 < D ? t * R * R + a * R + I0[q + Q * (2 * t + 1)]
                                : t * R * R + a;    // the odd last dimension: r rows
  offp[x] = row * 64;
}

template <int NT>
__global__ __launch_bounds__(64 * kPairWaves) void pred_vphase_pairs_kernel(
    const double* __restrict__ w, const double* __restrict__ T, const int32_t* __restrict__ offp,
    int D, int R, long long Ntest, int Q, double* __restrict__ fhat, long long ldF) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* pp = (double*)smem;                                   // [row][64]
  const int tid = threadIdx.x, lane = tid & 63, wv = uni(tid >> 6);
  const int s = blockIdx.y;
  const long long i0 = (long long)blockIdx.x * 64;
  const long long i = i0 + lane;
  const bool ok = i < Ntest;
  const double* Ts = T + ((size_t)s * ((Ntest + 63) / 64) + blockIdx.x) * D * R * 64 + lane;
  const int rows = (D / 2) * R * R + (D & 1) * R;
  double* red = pp + (size_t)rows * 64;
  // tables: wave w builds tables w, w + 4, ..; the 2·R temp rows of a table (512 contiguous
  // bytes each) are loaded together, then the R² products go to LDS
  for (int t = wv; t < NT; t += kPairWaves) {
    double a[5], b[5];
    const bool two = 2 * t + 1 < D;
#pragma unroll
    for (int x = 0; x < 5; ++x) {
      a[x] = x < R ? gptr(Ts)[(size_t)((2 * t) * R + x) * 64] : 0.0;
      b[x] = (x < R && two) ? gptr(Ts)[(size_t)((2 * t + 1) * R + x) * 64] : 1.0;
    }
    double* dst = pp + (size_t)t * R * R * 64 + lane;
    if (two) {
#pragma unroll
      for (int x = 0; x < 5; ++x)
#pragma unroll
        for (int y = 0; y < 5; ++y)
          if (x < R && y < R) dst[(x * R + y) * 64] = a[x] * b[y];
    } else {
#pragma unroll
      for (int x = 0; x < 5; ++x)
        if (x < R) dst[x * 64] = a[x];
    }
  }
  __syncthreads();
  const auto* of = cptr(offp);
  const auto* wq = cptr(w + (size_t)s * Q);
  const int qa = (Q * wv) / kPairWaves, qb = (Q * (wv + 1)) / kPairWaves;
  double f0 = 0.0, f1 = 0.0;
  int q = qa;
  for (; q + 2 <= qb; q += 2) {
    double v0 = pp[of[q * NT] + lane], v1 = pp[of[(q + 1) * NT] + lane];
#pragma unroll
    for (int t = 1; t < NT; ++t) {
      v0 *= pp[of[q * NT + t] + lane];
      v1 *= pp[of[(q + 1) * NT + t] + lane];
    }
    f0 = fma(wq[q], v0, f0);
    f1 = fma(wq[q + 1], v1, f1);
  }
  if (q < qb) {
    double v0 = pp[of[q * NT] + lane];
#pragma unroll
    for (int t = 1; t < NT; ++t) v0 *= pp[of[q * NT + t] + lane];
    f0 = fma(wq[q], v0, f0);
  }
  red[wv * 64 + lane] = f0 + f1;
  __syncthreads();
  if (wv == 0 && ok) {
    double f = red[lane];
#pragma unroll
    for (int x = 1; x < kPairWaves; ++x) f += red[x * 64 + lane];
    fhat[(size_t)s * ldF + i] = f;
  }
}


// Workgroup tile of the stacked-sample GEMM: a wave tile of 16·TM c × 16·TN i (TM = TN = 4).
template <int TM, int TN>
static void launch_pred_gemm_t(const double* Us, const double* phitest, int n, int D, int r,
                               long long Ntest, int Sc, double* T, hipStream_t st,
                               long long nti64) {
  const long long total = (long long)((Sc * r + 32 * TM - 1) / (32 * TM)) *
                          ((Ntest + 32 * TN - 1) / (32 * TN)) * D;
  const unsigned grid = (unsigned)((total + kXcds - 1) / kXcds * kXcds);
  if ((n & 1) == 0)
    hipLaunchKernelGGL((pred_temp_mfma_kernel<true, TM, TN>), dim3(grid), dim3(256), 0, st, Us,
                       phitest, n, D, r, Ntest, Sc, T, nti64);
  else
    hipLaunchKernelGGL((pred_temp_mfma_kernel<false, TM, TN>), dim3(grid), dim3(256), 0, st, Us,
                       phitest, n, D, r, Ntest, Sc, T, nti64);
}

static hipError_t launch_pred_gemm(const double* Us, const double* phitest, int n, int D, int r,
                                   long long Ntest, int Sc, double* T, hipStream_t st,
                                   long long nti64 = -1) {
  if (nti64 < 0) nti64 = (Ntest + 63) / 64;
  // 4 × 4 MFMA tiles per wave (the 2 × 2, 4 × 2 and 2 × 4 variants measured slower, round 3)
  launch_pred_gemm_t<4, 4>(Us, phitest, n, D, r, Ntest, Sc, T, st, nti64);
  return hipGetLastError();
}

template <int NN>
static hipError_t launch_vphase_pairs(const double* w, const double* T, const int32_t* offp, int D,
                                      int r, long long rows, int Q, double* fhat, int Sc,
                                      long long ldF, size_t plds, hipStream_t st) {
  static std::atomic<uint64_t> attr{0};
  hipError_t e = set_max_lds_once((const void*)pred_vphase_pairs_kernel<NN>, 160 * 1024, attr);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(pred_vphase_pairs_kernel<NN>, dim3((unsigned)((rows + 63) / 64), Sc),
                     dim3(64 * kPairWaves), plds, st, w, T, offp, D, r, rows, Q, fhat, ldF);
  return hipGetLastError();
}

static hipError_t vphase_pairs(int NTp, const double* w, const double* T, const int32_t* offp,
                               int D, int r, long long rows, int Q, double* fhat, int Sc,
                               long long ldF, size_t plds, hipStream_t st) {
  switch (NTp) {
#define PCASE(NN) \
    case NN: return launch_vphase_pairs<NN>(w, T, offp, D, r, rows, Q, fhat, Sc, ldF, plds, st);
    PCASE(1) PCASE(2) PCASE(3) PCASE(4) PCASE(5) PCASE(6) PCASE(7) PCASE(8)
#undef PCASE
    default: return hipErrorInvalidValue;
  }
}

// Which V-phase kernel the last prediction call on this thread launched (gpt_pred_last_vphase):
// 0 pred_vphase_pairs_kernel, 1 pred_vphase_rows_pf_kernel, 2 pred_vphase_rows_kernel,
// 4 pred_kernel (direct, no separate V-phase).
static thread_local int g_pred_vphase = -1;
int pred_last_vphase() { return g_pred_vphase; }

// The rows V-phase: the persistent prefetching kernel while a tile's D·R rows fit 16 per wave and
// its LDS fits a CU (as many workgroups as the LDS lets every CU hold), else the
// one-tile-per-workgroup kernel.
constexpr int kRowsPfWaves = 16;
template <int DD, int NPW, int NW = kRowsPfWaves>
static hipError_t launch_rows_pf(const double* w, const double* T, const int32_t* offs, int D, int r,
                                 long long Ntest, int Q, double* fhat, int Sc, hipStream_t st) {
  static std::atomic<uint64_t> attr{0};
  hipError_t e =
      set_max_lds_once((const void*)pred_vphase_rows_pf_kernel<DD, NW, NPW>, 160 * 1024, attr);
  if (e != hipSuccess) return e;
  g_pred_vphase = 1;
  int dev = 0, cus = 0;
  e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  const size_t lds = 8 * (size_t)D * r * 64 + 8 * (size_t)NW * 64 + 4 * (((size_t)Q * D + 3) & ~3) +
                     8 * (size_t)Q;
  const long long per_cu = std::max<long long>(1, (long long)(160 * 1024) / (long long)lds);
  const long long ntiles = (Ntest + 63) / 64 * (long long)Sc;
  const unsigned grid = (unsigned)std::min<long long>(ntiles, per_cu * cus);
  hipLaunchKernelGGL((pred_vphase_rows_pf_kernel<DD, NW, NPW>), dim3(grid), dim3(64 * NW), lds, st,
                     w, T, offs, D, r, Ntest, Q, fhat, Sc);
  return hipGetLastError();
}

static hipError_t launch_vphase_rows(const double* w, const double* T, const int32_t* offs, int D,
                                     int r, long long Ntest, int Q, double* fhat, int Sc,
                                     size_t rlds, hipStream_t st) {
  // (the persistent kernel's LDS: the tile's rows, the wave partials, the entries' offsets and
  // the sample's w — a large core (Q·D) can push it past one CU's 160 KB)
  const size_t pf_lds = 8 * (size_t)D * r * 64 + 8 * (size_t)kRowsPfWaves * 64 +
                        4 * (((size_t)Q * D + 3) & ~(size_t)3) + 8 * (size_t)Q;
  if (D * r <= kRowsPfWaves * 16 && pf_lds <= 160 * 1024) {
    // rows per wave: 10 (D·r ≤ 160: kin40kExperiment.jl's D = 8, r = 20) or 16
    if (D * r <= kRowsPfWaves * 10) {
      switch (D) {
#define DCASE(X) case X: return launch_rows_pf<X, 10>(w, T, offs, D, r, Ntest, Q, fhat, Sc, st);
        DCASE(2) DCASE(3) DCASE(4) DCASE(5) DCASE(6) DCASE(7) DCASE(8) DCASE(9) DCASE(10) DCASE(12)
#undef DCASE
        default: return launch_rows_pf<0, 10>(w, T, offs, D, r, Ntest, Q, fhat, Sc, st);
      }
    }
    return launch_rows_pf<0, 16>(w, T, offs, D, r, Ntest, Q, fhat, Sc, st);
  }
  if (rlds > 64 * 1024) {
    static std::atomic<uint64_t> attr{0};
    const hipError_t e = set_max_lds_once((const void*)pred_vphase_rows_kernel, 160 * 1024, attr);
    if (e != hipSuccess) return e;
  }
  g_pred_vphase = 2;
  hipLaunchKernelGGL(pred_vphase_rows_kernel, dim3((unsigned)((Ntest + 63) / 64), Sc),
                     dim3(64 * kRowsWaves), rlds, st, w, T, offs, D, r, Ntest, Q, fhat);
  return hipGetLastError();
}

// The prediction's pass buffers come from a private stream-ordered pool per device that keeps its
// memory between calls (release threshold ∞: the default threshold 0 unmapped and remapped the
// ~GBs of every call, ≈0.45 ms of a 7 ms call) without changing the device's default pool for the
// rest of the process; gpt_pred_trim_pool() returns it.
static std::mutex g_pred_pool_mu;
static hipMemPool_t g_pred_pool[64] = {};

static hipError_t pred_pool(hipMemPool_t* out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(g_pred_pool_mu);
  hipMemPool_t& p = g_pred_pool[dev & 63];
  if (!p) {
    hipMemPoolProps props = {};
    props.allocType = hipMemAllocationTypePinned;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    e = hipMemPoolCreate(&p, &props);
    if (e != hipSuccess) { p = nullptr; return e; }
    uint64_t thr = ~0ull;
    e = hipMemPoolSetAttribute(p, hipMemPoolAttrReleaseThreshold, &thr);
    if (e != hipSuccess) return e;
  }
  *out = p;
  return hipSuccess;
}

hipError_t pred_trim_pools() {
  std::lock_guard<std::mutex> lk(g_pred_pool_mu);
  for (auto& p : g_pred_pool)
    if (p) {
      const hipError_t e = hipMemPoolTrimTo(p, 0);
      if (e != hipSuccess) return e;
    }
  return hipSuccess;
}

static hipError_t launch_pred_mfma(const double* w, const double* U, const int32_t* I0,
                                   const double* phitest, int n, int D, long long Ntest, int r,
                                   int Q, int S, double* fhat, hipStream_t st,
                                   PredPhaseTiming* timing) {
  struct Events {                          // destroyed on every exit path
    hipEvent_t e[3] = {nullptr, nullptr, nullptr};
    ~Events() { for (auto x : e) if (x) (void)hipEventDestroy(x); }
  } evs;
  hipEvent_t* ev = evs.e;
  if (timing)
    for (int i = 0; i < 3; ++i) {
      const hipError_t ee = hipEventCreate(&ev[i]);
      if (ee != hipSuccess) return ee;
    }
  // temp of up to ~8 GiB of samples per pass; a pass of several workgroup tiles takes a multiple of
  // 128 / gcd(128, r) samples, so its S·r columns fill whole 128-column tiles (no MFMA padding)
  // T per sample: (Ntest / 64 tiles) × (D·r rows) × 64 doubles, tile-contiguous, so a V-phase
  // tile's rows are one block (row-major [D·r][Ntest] made each tile 160 strided 512-B reads at
  // r = 20: 1.9 TB/s, 4.1 ms of the 224-sample call with no arithmetic at all)
  const size_t per_sample = 8 * (size_t)D * r * (size_t)((Ntest + 63) / 64 * 64);
  int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)S, ((size_t)8 << 30) / per_sample));
  int unit = 1;
  {
    int g = 128, b = r;
    while (b) { const int t = g % b; g = b; b = t; }
    unit = 128 / g;
    if (chunk < S && chunk >= unit) chunk = chunk / unit * unit;
  }
  hipMemPool_t pool = nullptr;
  hipError_t e = pred_pool(&pool);
  if (e != hipSuccess) return e;
  double* T = nullptr;
  const int NTp = pred_pair_tables(D);
  size_t tbytes = 0;
  for (;;) {          // out of device memory: halve the pass (whole 128-column tiles while it can)
    tbytes = (per_sample * chunk + 255) / 256 * 256;
    e = hipMallocFromPoolAsync((void**)&T, tbytes + 4 * (size_t)Q * D + 4 * (size_t)Q * NTp, pool,
                               st);
    if (e != hipErrorOutOfMemory || chunk == 1) break;
    (void)hipGetLastError();
    chunk = chunk / 2 >= unit ? chunk / 2 / unit * unit : std::max(1, chunk / 2);
  }
  if (e != hipSuccess) return e;
  int32_t* offs = (int32_t*)((char*)T + tbytes);
  int32_t* offp = offs + (size_t)Q * D;
  const size_t rlds = 8 * (size_t)D * r * 64 + 8 * (size_t)kRowsWaves * 64;
  // V-phase variant: "pairs" (default where the tables fit: ⌈D/2⌉ ≤ 8 and ≤ 96 KB), else "rows";
  // GPTSGLD_PRED_VPHASE=rows forces the rows form (tests/test_gpu_parity.py compares the two)
  const int vmode = [] {
    const char* ev = std::getenv("GPTSGLD_PRED_VPHASE");
    return (ev && std::strcmp(ev, "rows") == 0) ? 1 : 0;
  }();
  const size_t plds = pred_pairs_lds_bytes(D, r);
  const bool pairs = vmode == 0 && r <= 5 && NTp <= 8 && plds <= 96 * 1024;
  for (int s0 = 0; s0 < S && e == hipSuccess; s0 += chunk) {
    const int Sc = std::min(chunk, S - s0);
    const double* Us = U + (size_t)s0 * n * r * D;
    if (timing) (void)hipEventRecord(ev[0], st);
    e = launch_pred_gemm(Us, phitest, n, D, r, Ntest, Sc, T, st);
    if (e != hipSuccess) break;
    if (s0 == 0) {
      // the V-phase's offset table, launched behind the first GEMM (its launch latency then hides
      // under the GEMM instead of delaying it)
      if (pairs)
        hipLaunchKernelGGL(pred_pair_offs_kernel, dim3((Q * NTp + 255) / 256), dim3(256), 0, st, I0,
                           Q, D, r, offp);
      else
        hipLaunchKernelGGL(pred_offs_kernel, dim3((Q * D + 255) / 256), dim3(256), 0, st, I0, Q, D,
                           r, offs);
    }
    if (timing) (void)hipEventRecord(ev[1], st);
    if (pairs) {
      g_pred_vphase = 0;
      e = vphase_pairs(NTp, w + (size_t)s0 * Q, T, offp, D, r, Ntest, Q, fhat + (size_t)s0 * Ntest,
                       Sc, Ntest, plds, st);
      if (timing && e == hipSuccess) {
        (void)hipEventRecord(ev[2], st);
        (void)hipEventSynchronize(ev[2]);
        float a = 0.f, b = 0.f;
        (void)hipEventElapsedTime(&a, ev[0], ev[1]);
        (void)hipEventElapsedTime(&b, ev[1], ev[2]);
        timing->gemm_ms += a;
        timing->vphase_ms += b;
      }
      continue;
    }
    e = launch_vphase_rows(w + (size_t)s0 * Q, T, offs, D, r, Ntest, Q, fhat + (size_t)s0 * Ntest,
                           Sc, rlds, st);
    if (timing && e == hipSuccess) {
      (void)hipEventRecord(ev[2], st);
      (void)hipEventSynchronize(ev[2]);
      float a = 0.f, b = 0.f;
      (void)hipEventElapsedTime(&a, ev[0], ev[1]);
      (void)hipEventElapsedTime(&b, ev[1], ev[2]);
      timing->gemm_ms += a;
      timing->vphase_ms += b;
    }
  }
  const hipError_t ef = hipFreeAsync(T, st);
  return e != hipSuccess ? e : ef;
}

static hipError_t launch_pred_direct(const double* w, const double* U, const int32_t* I0, const double* phitest,
                       int n, int D, long long Ntest, int r, int Q, int S, double* fhat,
                       hipStream_t st) {
  if (Ntest <= 0 || S <= 0) return hipSuccess;
  const size_t lds = pred_lds_bytes(n, D, r, Q);
  dim3 grid((unsigned)((Ntest + 63) / 64), S);
  switch (r) {
#define CASE(RR)                                                                             \
  case RR: {                                                                                 \
    static std::atomic<uint64_t> attr{0};                                                         \
    hipError_t e = set_max_lds_once((const void*)pred_kernel<RR>, 160 * 1024, attr);              \
    if (e != hipSuccess) return e;                                                                \
    hipLaunchKernelGGL(pred_kernel<RR>, grid, dim3(kNT), lds, st, w, U, I0, phitest, n, D,   \
                       Ntest, Q, fhat);                                                      \
  } break;
    GPT_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Prediction over S stored samples: the MFMA path (stacked-sample GEMM + V-phase) by default;
// GPTSGLD_PRED=direct selects the per-sample streaming kernel (pred_kernel) for comparison.
hipError_t launch_pred(const double* w, const double* U, const int32_t* I0, const double* phitest,
                       int n, int D, long long Ntest, int r, int Q, int S, double* fhat,
                       hipStream_t st, PredPhaseTiming* timing) {
  if (Ntest <= 0 || S <= 0) return hipSuccess;
  static const bool direct = [] {
    const char* ev = std::getenv("GPTSGLD_PRED");
    return ev && std::strcmp(ev, "direct") == 0;
  }();
  if (direct) {
    g_pred_vphase = 4;
    return launch_pred_direct(w, U, I0, phitest, n, D, Ntest, r, Q, S, fhat, st);
  }
  return launch_pred_mfma(w, U, I0, phitest, n, D, Ntest, r, Q, S, fhat, st, timing);
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
    static std::atomic<uint64_t> attr{0};                                                         \
    hipError_t e = set_max_lds_once((const void*)pred_x_kernel<RR>, 160 * 1024, attr);            \
    if (e != hipSuccess) return e;                                                                \
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
