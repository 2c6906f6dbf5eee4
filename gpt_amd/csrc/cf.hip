// MovieLens-100k tensor collaborative filtering with side information (§8(f) item 1):
// GPT_fullw_sideinfo, 100k_movielensExperiment.jl:409-551.
//
// Model: rating(user, movie) ≈ a · sumUᵀ w sumV with sumU = U[user] + b·Σ U[user's feature rows],
// sumV = V[movie] + c·Σ V[movie's feature rows] (U: (n1+D1) × r, V: (n2+D2) × r, w: r × r).
// Per minibatch, one workgroup per chain (fold) forms the ratings' sums and residuals in LDS, the
// w step, and the gradient rows (users / movies in the batch and their feature rows) summed in
// rating order — deterministic, no atomics — into zeroed dense gradient buffers; then every row of
// U and V takes its SGD / SGLD step (the prior term moves all rows): for the Euclidean variants in
// a row-parallel launch over the whole GPU (cf_move_kernel), for the Stiefel ones (projection +
// geodesic, Grams over every row) inside the same workgroup, which then runs the whole epoch.  A
// second kernel predicts every train / test rating after the epoch (running averages, cutoff,
// squared errors per block).
#include "device_util.h"

namespace gpt {

#define GPT_CF_RANKS(X) X(1) X(2) X(3) X(4) X(5) X(6) X(8) X(10) X(12) X(15) X(16) X(20)

constexpr int kCfNT = 1024;
constexpr int kCfNW = kCfNT / 64;
typedef double pd4 __attribute__((ext_vector_type(4)));

// Diagnostic phase stamps of the epoch kernel (P.stamps, gpt_cf_last_stamps): thread 0 of chain 0
// records s_memtime after the barrier closing each phase of the first kCfStampSteps steps.
#define CF_STAMP(bt, slot)                                                                   \
  do {                                                                                       \
    if (P.stamps && blockIdx.x == 0 && threadIdx.x == 0 && (bt) < kCfStampSteps)            \
      P.stamps[(size_t)(bt) * kCfStampSlots + (slot)] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)

// Per-wave sub-phase stamps (diagnostic builds with CF_WSTAMPS): lane 0 of every wave of chain 0,
// slots 8 + 4·wave + i of the step's stamp row.
#if CF_WSTAMPS
#define CF_WSTAMP(bt, i)                                                                      \
  do {                                                                                        \
    if (P.stamps && blockIdx.x == 0 && (threadIdx.x & 63) == 0 && (bt) < kCfStampSteps)      \
      P.stamps[(size_t)(bt) * kCfStampSlots + 8 + 4 * (threadIdx.x >> 6) + (i)] =             \
          (long long)__builtin_amdgcn_s_memtime();                                           \
  } while (0)
#define CF_EXP(bit) ((P.exp & (bit)) != 0)
#else
#define CF_WSTAMP(bt, i) do {} while (0)
#define CF_EXP(bit) false
#endif

// Sum of A[:, a]·B[:, b] over `rows` for every (a, b) < r², one wave per entry (wave sums).
__device__ void cf_gram(const double* A, const double* B, int rows, int r, double* out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int e = wv; e < r * r; e += kCfNW) {
    const int a = e / r, b = e - a * r;
    double s = 0.0;
    for (int row = lane; row < rows; row += 64)
      s = fma(gptr(A)[row + (size_t)rows * a], gptr(B)[row + (size_t)rows * b], s);
    s = wave_sum(s);
    if (lane == 0) out[e] = s;
  }
}

// One U or V step (the update block of :481-507) on matrix M with gradient rows G (zeroed
// afterwards).  which = 0 (U) / 1 (V) selects the noise stream.
template <int R>
__device__ bool cf_move(const CfParams& P, double* M, double* G, int rows, int which,
                        long long step, double* scr) {
  const int tid = threadIdx.x, wv = tid >> 6;
  constexpr int RE = R + (R & 1);
  const double sq = sqrt(P.epsU);
  const uint32_t st = (uint32_t)step;
  if (!P.stiefel) {
    const double su2 = P.sigma_u * P.sigma_u;
    for (int o = tid; o < rows * (RE / 2); o += kCfNT) {
      const int lp = o / rows, row = o - lp * rows;       // consecutive rows: coalesced
      double z[2] = {0.0, 0.0};
      if (P.langevin)
        normal_pair(P.seed, (uint32_t)((2 * lp + RE * row) >> 1), st, kCfUVNoise, (uint32_t)which,
                    z[0], z[1]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int l = 2 * lp + h;
        if (l >= R) break;
        const size_t e = row + (size_t)rows * l;
        const double m0 = gptr(M)[e];
        double mn = m0 + P.epsU * (gptr(G)[e] - m0 / su2) / 2;
        if (P.langevin) mn = mn + sq * z[h];
        gptr_w(M)[e] = mn;
        gptr_w(G)[e] = 0.0;
      }
    }
    __syncthreads();
    return true;
  }
  // Stiefel: mom = proj(M, √εU·G/2 [+ ξ]) (GPT_SGLD.jl:14-16), M = geod(M, mom, √εU) (:19-37)
  constexpr int NN = 2 * R;
  double* Mg = scr;                 // R²
  double* Ag = Mg + R * R;          // R²
  double* Sg = Ag + R * R;          // R²
  double* X0 = Sg + R * R;          // 7 NN²
  double* X1 = X0 + 7 * NN * NN;    // 7 R²
  double* F = X1 + 7 * R * R;       // NN × R
  double* nr = F + NN * R;          // R
  int* flag = (int*)(nr + R);
  for (int o = tid; o < rows * (RE / 2); o += kCfNT) {
    const int lp = o / rows, row = o - lp * rows;       // consecutive rows: coalesced
    double z[2] = {0.0, 0.0};
    if (P.langevin)
      normal_pair(P.seed, (uint32_t)((2 * lp + RE * row) >> 1), st, kCfUVNoise, (uint32_t)which,
                  z[0], z[1]);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int l = 2 * lp + h;
      if (l >= R) break;
      const size_t e = row + (size_t)rows * l;
      gptr_w(G)[e] = sq * gptr(G)[e] / 2 + z[h];
    }
  }
  if (tid == 0) flag[0] = 0;
  __syncthreads();
  cf_gram(M, G, rows, R, Mg);
  __syncthreads();
  for (int row = tid; row < rows; row += kCfNT) {
    // an offset the compiler cannot see through: the R² Gram entries are read from LDS per row
    // rather than hoisted out of the row loop into registers (at r = 20 that spilled thousands
    // of values)
    int zo = 0;
    asm volatile("" : "+v"(zo));
    double x[R], u[R];
#pragma unroll
    for (int l = 0; l < R; ++l) {
      u[l] = gptr(M)[row + (size_t)rows * l];
      x[l] = gptr(G)[row + (size_t)rows * l];
    }
#pragma unroll
    for (int bb = 0; bb < R; ++bb) {
      double s = 0.0;
#pragma unroll
      for (int a2 = 0; a2 < R; ++a2) s = fma(u[a2], Mg[zo + a2 * R + bb] + Mg[zo + bb * R + a2], s);
      gptr_w(G)[row + (size_t)rows * bb] = x[bb] - s / 2;
    }
  }
  __syncthreads();
  cf_gram(M, G, rows, R, Ag);
  cf_gram(G, G, rows, R, Sg);
  __syncthreads();
  const double tt = sq;
  if (wv == 0) {
    for (int o = tid; o < NN * NN; o += 64) {
      const int i = o / NN, j = o - i * NN;
      double v;
      if (i < R) v = j < R ? Ag[i * R + j] : -Sg[i * R + (j - R)];
      else v = j < R ? (i - R == j ? 1.0 : 0.0) : Ag[(i - R) * R + (j - R)];
      X0[o] = tt * v;
    }
    wave_sync();
    if (wave_expm<NN, false>(X0) && tid == 0) flag[0] = 1;   // 1024-thread block: LDS GEPP
  } else if (wv == 1) {
    const int ln = tid & 63;
    for (int o = ln; o < R * R; o += 64) X1[o] = -tt * Ag[o];
    wave_sync();
    wave_expm<R>(X1);
  }
  __syncthreads();
  if (flag[0]) return false;
  const double* E = X0 + NN * NN;
  const double* mx = X1 + R * R;
  for (int o = tid; o < NN * R; o += kCfNT) {
    const int a2 = o / R, l = o - a2 * R;
    double s = 0.0;
#pragma unroll
    for (int c2 = 0; c2 < R; ++c2) s = fma(E[a2 * NN + c2], mx[c2 * R + l], s);
    F[o] = s;
  }
  __syncthreads();
  for (int row = tid; row < rows; row += kCfNT) {
    int zo = 0;                       // F read from LDS per row (see the proj loop)
    asm volatile("" : "+v"(zo));
    double x[NN];
#pragma unroll
    for (int l = 0; l < R; ++l) {
      x[l] = gptr(M)[row + (size_t)rows * l];
      x[R + l] = gptr(G)[row + (size_t)rows * l];
    }
#pragma unroll
    for (int l = 0; l < R; ++l) {
      double s = 0.0;
#pragma unroll
      for (int a2 = 0; a2 < NN; ++a2) s = fma(x[a2], F[zo + a2 * R + l], s);
      gptr_w(M)[row + (size_t)rows * l] = s;
      gptr_w(G)[row + (size_t)rows * l] = 0.0;
    }
  }
  __syncthreads();
  {
    const int lane = tid & 63;
    for (int l = wv; l < R; l += kCfNW) {
      double s = 0.0;
      for (int row = lane; row < rows; row += 64) {
        const double v = gptr(M)[row + (size_t)rows * l];
        s = fma(v, v, s);
      }
      s = wave_sum(s);
      if (lane == 0) nr[l] = sqrt(s);
    }
  }
  __syncthreads();
  for (int o = tid; o < rows * R; o += kCfNT) {
    const int l = o / rows;
    gptr_w(M)[o] = gptr(M)[o] / nr[l];
  }
  __syncthreads();
  return true;
}

// The SGD / SGLD move of U and V without the Stiefel geometry (the update block of :481-507 with
// stiefel = false) touches every row independently, so it runs outside the epoch kernel's single
// workgroup: grid (blocks, folds), one (row, column pair) per thread, the same doubles and noise
// indices as cf_move.  G rows are zeroed for the next batch.
// With at most 8 folds the grid is XCD-aware: workgroup x runs on XCD x mod 8 (round-robin
// dispatch), so fold f's rows are moved by workgroups of XCD f — the XCD of the fold's epoch
// workgroup (blockIdx.x = f), whose next batch then reads U and V from its own L2.
template <int R>
__global__ __launch_bounds__(256) void cf_move_kernel(CfParams P, const CfChain* chains,
                                                      const long long* step_base, long long step,
                                                      int nchains) {
  if (step_base) step += *step_base;                 // graph replays: the epoch's first step
  int fold, blk;
  if (nchains <= 8) {
    fold = blockIdx.x & 7;
    blk = blockIdx.x >> 3;
    if (fold >= nchains) return;
  } else {
    fold = blockIdx.y;
    blk = blockIdx.x;
  }
  const CfChain C = chains[fold];
  if (__hip_atomic_load(C.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  constexpr int RE = R + (R & 1);
  const int nU = P.rowsU * (RE / 2);
  const int o0 = blk * 256 + threadIdx.x;
  if (o0 >= nU + P.rowsV * (RE / 2)) return;
  const int which = o0 >= nU ? 1 : 0;
  const int o = o0 - which * nU;
  const int rows = which ? P.rowsV : P.rowsU;
  double* M = which ? C.V : C.U;
  double* G = which ? C.GV : C.GU;
  const int lp = o / rows, row = o - lp * rows;
  const double su2 = P.sigma_u * P.sigma_u;
  double z[2] = {0.0, 0.0};
  if (P.langevin)
    normal_pair(P.seed, (uint32_t)((2 * lp + RE * row) >> 1), (uint32_t)step, kCfUVNoise,
                (uint32_t)which, z[0], z[1]);
  const double sq = sqrt(P.epsU);
  double m0[2], g0[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int l = min(2 * lp + h, R - 1);
    m0[h] = gptr(M)[row + (size_t)rows * l];
    g0[h] = gptr(G)[row + (size_t)rows * l];
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int l = 2 * lp + h;
    if (l >= R) break;
    const size_t e = row + (size_t)rows * l;
    double mn = m0[h] + P.epsU * (g0[h] - m0[h] / su2) / 2;
    if (P.langevin) mn = mn + sq * z[h];
    gptr_w(M)[e] = mn;
    gptr_w(G)[e] = 0.0;
  }
}

// The value of lane λ ^ j (j < 64, a power of two) without an LDS round trip: DPP within rows
// (quad_perm for 1, 2; row_ror 4 / 12 picked per lane for 4; row_ror 8), v_permlane16/32_swap
// across rows.  Which rotation / swap slot holds the partner is read off the lane ids themselves
// (XorSel, formed once).
struct XorSel { bool r4, s16, s32; };
__device__ __forceinline__ XorSel xor_sel(int lane) {
  XorSel x;
  x.r4 = __builtin_amdgcn_mov_dpp(lane, 0x124, 0xF, 0xF, false) == (lane ^ 4);
  x.s16 = (int)__builtin_amdgcn_permlane16_swap((unsigned)lane, (unsigned)lane, false, false)[0] ==
          (lane ^ 16);
  x.s32 = (int)__builtin_amdgcn_permlane32_swap((unsigned)lane, (unsigned)lane, false, false)[0] ==
          (lane ^ 32);
  return x;
}
__device__ __forceinline__ int xor_lane(int v, int j, const XorSel& x) {
  if (j == 1) return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);      // quad_perm 1,0,3,2
  if (j == 2) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);      // quad_perm 2,3,0,1
  if (j == 8) return __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);     // row_ror 8
  if (j == 4) {
    const int a = __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false);         // row_ror 4
    const int b = __builtin_amdgcn_mov_dpp(v, 0x12C, 0xF, 0xF, false);         // row_ror 12
    return x.r4 ? a : b;
  }
  const auto sw = j == 16 ? __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false)
                          : __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
  return (int)((j == 16 ? x.s16 : x.s32) ? sw[0] : sw[1]);
}

// Lazy move's row-major working copy: column-major M (rows × R, the session's layout) -> Mr
// (row r at Mr[r·R .. r·R + R−1]) through an LDS tile of TR rows; eight loads per thread in
// flight.  Every thread of the block calls it (block barriers inside).
template <int R>
__device__ void cf_rows_in(const double* M, double* Mr, int rows, double* tile, int TR) {
  const int tid = threadIdx.x;
  for (int r0 = 0; r0 < rows; r0 += TR) {
    const int nr = min(TR, rows - r0), ne = nr * R;
    for (int o0 = tid; o0 < ne; o0 += 8 * kCfNT) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int o = min(o0 + u * kCfNT, ne - 1), l = o / nr, rr = o - l * nr;
        v[u] = gptr(M)[r0 + rr + (size_t)rows * l];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int o = o0 + u * kCfNT, l = o / nr, rr = o - l * nr;
        if (o < ne) tile[rr * R + l] = v[u];
      }
    }
    __syncthreads();
    for (int o = tid; o < ne; o += kCfNT) gptr_w(Mr)[(size_t)r0 * R + o] = tile[o];
    __syncthreads();
  }
}

// ... and back at the launch's end: row r of M = (its value as of step cur[r]) · c^(nb − cur[r]),
// the feature rows (r >= base) from Fl, the others from Mr.
template <int R>
__device__ void cf_rows_out(const double* Mr, double* M, int rows, int base, const double* Fl,
                            const int* cur, const double* cpow, int nb, double* tile, int TR) {
  const int tid = threadIdx.x;
  for (int r0 = 0; r0 < rows; r0 += TR) {
    const int nr = min(TR, rows - r0), ne = nr * R;
    for (int o0 = tid; o0 < ne; o0 += 8 * kCfNT) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int o = min(o0 + u * kCfNT, ne - 1), row = r0 + o / R;
        v[u] = row >= base ? Fl[(row - base) * R + o % R] : gptr(Mr)[(size_t)r0 * R + o];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int o = o0 + u * kCfNT;
        if (o < ne) tile[o] = v[u] * cpow[nb - cur[r0 + o / R]];
      }
    }
    __syncthreads();
    for (int o = tid; o < ne; o += kCfNT) {
      const int l = o / nr, rr = o - l * nr;
      gptr_w(M)[r0 + rr + (size_t)rows * l] = tile[rr * R + l];
    }
    __syncthreads();
  }
}

// Byte offset of the lazy move's tables (cpow, cur) in the epoch kernel's LDS: past the batch
// carve of the masks path (w, wn, sU, sV, tU, tV, er, umk, vmk, us, ms, unx, vnx, fcnt, flist).
GPT_HD size_t cf_lazy_offset(int r, int m, int nfeat) {
  const size_t b = 8 * (2 * (size_t)r * r + 4 * (size_t)m * r + m) + 16 * (size_t)m +
                   4 * (4 * (size_t)m + (size_t)nfeat) + 2 * (size_t)nfeat * m;
  return (b + 15) / 16 * 16;
}

// domove = 0: only the batch phase of each step (sums, residuals, gradw + the w step, the
// gradient rows); the caller launches cf_move_kernel between steps.  1: the Stiefel move in the
// workgroup after every batch phase.  2: the lazy SGD move (below).  A template argument, so the
// batch-phase variants are not register-allocated around the Stiefel move's arrays.  bt0: the
// launch's first batch of the epoch, step0 its step.
template <int R, int domove>
__global__ __launch_bounds__(kCfNT) void cf_epoch_kernel(CfParams P, const CfChain* chains,
                                                         const long long* step_base,
                                                         long long step0, int bt0, int nb) {

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const CfChain C = chains[blockIdx.x];
  const int tid = threadIdx.x, m = P.m, N = C.N;
  double* w_l = (double*)smem;                  // R²
  double* wn_l = w_l + R * R;                   // R²
  double* sU = wn_l + R * R;                    // m × R   sumU of each batch rating
  double* sV = sU + (size_t)m * R;              // m × R
  double* tU = sV + (size_t)m * R;              // m × R   sumU·w
  double* tV = tU + (size_t)m * R;              // m × R   w·sumVᵀ
  double* er = tV + (size_t)m * R;              // m       rating, then residual
  // side-information bitmasks of the batch's users / movies (D1, D2 <= 64: the feature rows of a
  // rating without walking the CSR lists in global memory every time)
  uint64_t* umk = (uint64_t*)(er + m);          // m
  uint64_t* vmk = umk + m;                      // m
  int* us = (int*)(vmk + m);                    // m
  int* ms = us + m;                             // m
  // per batch position ii of each side: (next position with the same user / movie) + 1, or 0,
  // with bit 16 set when ii is that id's first position in the batch (its gradient row's owner)
  int* unx = ms + m;                            // m
  int* vnx = unx + m;                           // m
  const bool masks = P.D1 <= 64 && P.D2 <= 64;
  // with the masks: per feature row (users' D1, then movies' D2) the batch positions carrying it,
  // ascending (fcnt of them), so its gradient sums only those ratings
  int* fcnt = vnx + m;                          // D1 + D2
  unsigned short* flist = (unsigned short*)(fcnt + P.D1 + P.D2);   // (D1 + D2) × m
  // Stiefel scratch of the U / V moves: aliases the batch buffers (sU .. ms), which are dead from
  // the barrier before the moves until the next batch reloads them (r = 20 fits 160 KB this way)
  double* scr = sU;
  if (__hip_atomic_load(C.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  if (step_base) step0 += *step_base;                // graph replays: the epoch's first step
  for (int o = tid; o < R * R; o += kCfNT) w_l[o] = C.w[o];
  const double is2 = 1.0 / P.signal_var;
  // domove = 2 (SGD, the masks path): the lazy move.  A row whose gradient is zero in a step only
  // decays, m ← m + εU·(0 − m/σ_u²)/2 = m·c (c = 1 − εU/(2σ_u²)), so a row is stored as of the
  // step it last moved (cur: U rows, then V rows, launch-local steps) and read as m·c^Δ (cpow,
  // Δ = 0 … nb); the rows of a batch take the full move in the batch phase itself, the rest are
  // brought to the launch's last step at its end.  One launch per epoch, no gradient buffers.
  constexpr bool lazy = domove == 2;
  const double su2 = P.sigma_u * P.sigma_u;
  // The feature rows (users' D1, then movies' D2) stay in LDS for the launch: Fl as of their
  // step in cur, Fc their values at the current step (formed once per step), hit the features the
  // batch carries (their rows move this step).
  const int nfeat = P.D1 + P.D2;
  double* cpow = nullptr;
  int* cur = nullptr;
  double* Fl = nullptr;
  double* Fc = nullptr;
  unsigned long long* hit = nullptr;
  double* mcl = nullptr;   // the batch's own U / V rows as of this step, [side][ii][l] (sums phase)
  if (lazy) {
    const size_t o0 = cf_lazy_offset(R, m, nfeat);
    cpow = (double*)(smem + o0);
    cur = (int*)(cpow + nb + 1);
    Fl = (double*)(smem + ((o0 + 8 * ((size_t)nb + 1) + 4 * (size_t)(P.rowsU + P.rowsV) + 15) / 16 * 16));
    Fc = Fl + nfeat * R;
    hit = (unsigned long long*)(Fc + nfeat * R);
    mcl = (double*)(hit + 2);                          // 2 · m · R
    // c^d by binary powering (the host takes this path only for 0 < c < 1)
    const double c1 = 1.0 - P.epsU / (2 * su2);
    for (int d = tid; d <= nb; d += kCfNT) {
      double p = 1.0, b = c1;
      for (int e = d; e > 0; e >>= 1) {
        if (e & 1) p *= b;
        b *= b;
      }
      cpow[d] = p;
    }
    for (int o = tid; o < P.rowsU + P.rowsV; o += kCfNT) cur[o] = 0;
    for (int o = tid; o < nfeat * R; o += kCfNT) {
      const int fo = o / R, l = o - fo * R, side = fo >= P.D1 ? 1 : 0, f = fo - side * P.D1;
      Fl[o] = gptr(side ? C.V : C.U)[(side ? P.n2 : P.n1) + f + (size_t)(side ? P.rowsV : P.rowsU) * l];
    }
    // Row-major working copies of U and V for the launch, in the gradient buffers (the lazy move
    // has none): a rating's r entries are then one contiguous run for the sums phase's gathers and
    // the moves' stores, where the session's column-major layout spreads them over r cache lines.
    // Transposed through the batch buffers, which are free until the first batch.
    const int TR = (int)((cf_lazy_offset(R, m, nfeat) - 16 * (size_t)R * R) / (8 * R));
    cf_rows_in<R>(C.U, C.GU, P.rowsU, sU, TR);
    cf_rows_in<R>(C.V, C.GV, P.rowsV, sU, TR);
  }
  // lazy path: the next batch's (user, movie, rating) of thread tid < m are loaded during this
  // step's gradient phase and their feature masks after it, so the batch and mask phases of the
  // next step wait for no global memory (the barriers between them wait for LDS only)
  int pf_u = 0, pf_m = 0;
  double pf_r = 0.0;
  uint64_t pf_mu = 0, pf_mm = 0;
  auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  for (int bt = bt0; bt < bt0 + nb; ++bt) {
    CF_STAMP(bt, 0);
    const long long step = step0 + (bt - bt0);
    const int jl = bt - bt0;                           // launch-local step (lazy move)
    const int B = min(m, N - bt * m);
    const double cN = (double)N / (double)B;
    const bool pref = lazy && bt > bt0 && m <= kCfNT;  // this batch was prefetched
    if (pref) {
      if (tid < B) {
        us[tid] = pf_u;
        ms[tid] = pf_m;
        er[tid] = pf_r;
        umk[tid] = pf_mu;
        vmk[tid] = pf_mm;
      }
    } else {
      for (int ii = tid; ii < B; ii += kCfNT) {
        us[ii] = C.ep_user[bt * m + ii];              // the epoch's order (cf_gather_kernel)
        ms[ii] = C.ep_movie[bt * m + ii];
        er[ii] = C.ep_rating[bt * m + ii];
      }
    }
    if (lazy && tid < 2) hit[tid] = 0ull;
    if (pref) lds_barrier(); else __syncthreads();
    CF_STAMP(bt, 1);
    // per (side, ii): the feature bitmask, the first-occurrence flag and the next occurrence
    if (B <= 128) {
      // the links by sorting: wave `side` sorts the 128 keys (id << 8 | position) of its side
      // (two per lane, bitonic, lane exchanges by DPP / permlane), so equal ids end up adjacent in
      // ascending position: a key's successor with the same id is its next occurrence, and a key
      // whose predecessor differs is the first (the round-4 form compared every pair, 11.6 k
      // cycles of the step); the masks go to LDS from the other waves
      const int wv = uni(tid >> 6), lane = tid & 63;
      if (wv < 2) {
        const int* ids = wv ? ms : us;
        int k0 = lane < B ? (ids[lane] << 8) | lane : 0x7fffffff;
        int k1 = lane + 64 < B ? (ids[lane + 64] << 8) | (lane + 64) : 0x7fffffff;
        const XorSel xs = xor_sel(lane);
#pragma unroll
        for (int k = 2; k <= 128; k <<= 1) {
#pragma unroll
          for (int j = k >> 1; j > 0; j >>= 1) {
            if (j == 64) {                             // (k = 128: ascending everywhere)
              const int lo = min(k0, k1), hi = max(k0, k1);
              k0 = lo;
              k1 = hi;
            } else {
              // (DPP / permlane exchanges: __shfl_xor's ds_bpermute round trips made the 28
              // stages a 4.4 k-cycle latency chain)
              const int o0 = xor_lane(k0, j, xs), o1 = xor_lane(k1, j, xs);
              const bool low = (lane & j) == 0;        // this element is the lower of its pair
              const bool asc0 = (lane & k) == 0, asc1 = ((lane + 64) & k) == 0;
              k0 = (low == asc0) ? min(k0, o0) : max(k0, o0);
              k1 = (low == asc1) ? min(k1, o1) : max(k1, o1);
            }
          }
        }
        // neighbours in sorted order: e = lane (k0) and e = 64 + lane (k1)
        const int p0 = __shfl(k0, (lane + 63) & 63), p1 = __shfl(k1, (lane + 63) & 63);
        const int n0 = __shfl(k0, (lane + 1) & 63), n1 = __shfl(k1, (lane + 1) & 63);
        const int last0 = __shfl(k0, 63), first1 = __shfl(k1, 0);   // with every lane active
        const int prev0 = lane == 0 ? 0x7fffffff : p0, prev1 = lane == 0 ? last0 : p1;
        const int next0 = lane == 63 ? first1 : n0, next1 = lane == 63 ? 0x7fffffff : n1;
        int* nxl = wv ? vnx : unx;
        auto link = [&](int key, int prev, int next) {
          if (key == 0x7fffffff) return;
          const bool first = (prev >> 8) != (key >> 8) || prev == 0x7fffffff;
          const int nx = (next != 0x7fffffff && (next >> 8) == (key >> 8)) ? (next & 0xff) : -1;
          nxl[key & 0xff] = (nx + 1) | (first ? 1 << 16 : 0);
        };
        link(k0, prev0, next0);
        link(k1, prev1, next1);
      } else if (masks) {
        for (int o = tid - 128; o < 2 * B; o += kCfNT - 128) {
          const int side = o >= B ? 1 : 0, ii = o - side * B;
          const int id = (side ? ms : us)[ii];
          const uint64_t mk = pref ? (side ? vmk : umk)[ii] : (side ? P.vmask : P.umask)[id];
          if (!pref) (side ? vmk : umk)[ii] = mk;
          if (lazy) __hip_atomic_fetch_or(hit + side, (unsigned long long)mk, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    } else
    for (int o = tid; o < 2 * B; o += kCfNT) {
      const int side = o >= B ? 1 : 0, ii = o - side * B;
      const int* ids = side ? ms : us;
      const int id = ids[ii];
      if (masks) {
        const uint64_t mk = pref ? (side ? vmk : umk)[ii] : (side ? P.vmask : P.umask)[id];
        if (!pref) (side ? vmk : umk)[ii] = mk;
        if (lazy) __hip_atomic_fetch_or(hit + side, (unsigned long long)mk, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      bool first = true;
      int nx = -1;
      for (int z0 = 0; z0 < B; z0 += 8) {              // eight ids read before they are compared
        int iz[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) iz[u] = z0 + u < B ? ids[z0 + u] : -1;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int z = z0 + u;
          const bool same = iz[u] == id;
          first &= !(same && z < ii);
          if (same && z > ii && nx < 0) nx = z;
        }
      }
      (side ? vnx : unx)[ii] = (nx + 1) | (first ? 1 << 16 : 0);
    }
    if (lazy)                                         // the feature rows as of this step
      for (int o = tid; o < nfeat * R; o += kCfNT) {
        const int fo = o / R, side = fo >= P.D1 ? 1 : 0;
        const int row = (side ? P.rowsU + P.n2 - P.D1 : P.n1) + fo;
        Fc[o] = Fl[o] * cpow[jl - cur[row]];
      }
    __syncthreads();
    CF_STAMP(bt, 2);
    // sumU = U[user,:] + b·sum(U[uidx,:],1), sumV likewise (:462); the feature rows in ascending
    // order (find(UserData[i,:]), the CSR order).  With the masks: four (rating, column) items
    // per thread and pass, every item's row loads issued before any sum (one memory latency per
    // pass instead of one per item)
    if (lazy) {
      // the rating's own row from memory (as of this step), its feature rows from Fc, added in
      // ascending order from 0 as the masks path below does
      // four items per thread and pass: every item's row load, decay and first three feature
      // values are read before any sum (a user carries 3 features, 97 % of the rated movies 1-3;
      // the rest, if any, after)
      for (int o0 = tid; o0 < 2 * B * R; o0 += 4 * kCfNT) {
        double mv[4], cp[4], fv[4][3];
        uint64_t rest[4];
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          const int o = min(o0 + k4 * kCfNT, 2 * B * R - 1);
          const int side = o >= B * R ? 1 : 0, x = o - side * (B * R), ii = x / R, l = x - ii * R;
          const int id = side ? ms[ii] : us[ii];
          mv[k4] = gptr(side ? C.GV : C.GU)[(size_t)id * R + l];     // row-major copy
          cp[k4] = cpow[jl - cur[(side ? P.rowsU : 0) + id]];
          const double* Fs = Fc + (side ? P.D1 * R : 0) + l;
          uint64_t mk = (side ? vmk : umk)[ii];
#pragma unroll
          for (int u = 0; u < 3; ++u) {
            const bool h = mk != 0;
            const double xf = Fs[(h ? __ffsll((long long)mk) - 1 : 0) * R];
            fv[k4][u] = h ? xf : 0.0;                   // + 0.0: the sum is unchanged
            mk &= mk - 1;
          }
          rest[k4] = mk;
        }
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          const int o = o0 + k4 * kCfNT;
          if (o >= 2 * B * R) break;
          const int side = o >= B * R ? 1 : 0, x = o - side * (B * R), ii = x / R, l = x - ii * R;
          const double mcur = mv[k4] * cp[k4];
          mcl[o] = mcur;                                 // o = (side·B + ii)·R + l
          double f = 0.0;
#pragma unroll
          for (int u = 0; u < 3; ++u) f += fv[k4][u];
          uint64_t mk = rest[k4];
          const double* Fs = Fc + (side ? P.D1 * R : 0) + l;
          while (mk) {
            const int fb = __ffsll((long long)mk) - 1;
            mk &= mk - 1;
            f += Fs[fb * R];
          }
          (side ? sV : sU)[ii * R + l] = mcur + (side ? P.c : P.b) * f;
        }
      }
    } else if (masks) {
      for (int o0 = tid; o0 < 2 * B * R; o0 += 4 * kCfNT) {
        double fv[4][4], mv[4];
        bool fh[4][4], ok[4];
        uint64_t rest[4];
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          const int o = o0 + k4 * kCfNT;
          ok[k4] = o < 2 * B * R;
          const int oc = ok[k4] ? o : o0;
          const int side = oc >= B * R ? 1 : 0, x = oc - side * (B * R), ii = x / R, l = x - ii * R;
          const double* M = side ? C.V : C.U;
          const int rows = side ? P.rowsV : P.rowsU;
          const int id = side ? ms[ii] : us[ii];
          const int base = side ? P.n2 : P.n1;
          uint64_t mk = (side ? vmk : umk)[ii];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            fh[k4][u] = mk != 0;
            const int fb = fh[k4][u] ? __ffsll((long long)mk) - 1 : 0;
            fv[k4][u] = fh[k4][u] ? gptr(M)[base + fb + (size_t)rows * l] : 0.0;
            mk &= mk - 1;
          }
          rest[k4] = mk;
          mv[k4] = gptr(M)[id + (size_t)rows * l];
        }
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          if (!ok[k4]) continue;
          const int o = o0 + k4 * kCfNT;
          const int side = o >= B * R ? 1 : 0, x = o - side * (B * R), ii = x / R, l = x - ii * R;
          const double* M = side ? C.V : C.U;
          const int rows = side ? P.rowsV : P.rowsU;
          const int base = side ? P.n2 : P.n1;
          double f = 0.0;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (fh[k4][u]) f += fv[k4][u];
          uint64_t mk = rest[k4];
          while (mk) {
            const int fb = __ffsll((long long)mk) - 1;
            mk &= mk - 1;
            f += gptr(M)[base + fb + (size_t)rows * l];
          }
          (side ? sV : sU)[ii * R + l] = mv[k4] + (side ? P.c : P.b) * f;
        }
      }
    } else {
      for (int o = tid; o < 2 * B * R; o += kCfNT) {
        const int side = o >= B * R ? 1 : 0, x = o - side * (B * R), ii = x / R, l = x - ii * R;
        const double* M = side ? C.V : C.U;
        const int rows = side ? P.rowsV : P.rowsU;
        const int id = side ? ms[ii] : us[ii];
        const int32_t* ptr = side ? P.vptr : P.uptr;
        const int32_t* fe = side ? P.vfe : P.ufe;
        double f = 0.0;
        for (int z = ptr[id]; z < ptr[id + 1]; ++z) f += gptr(M)[fe[z] + (size_t)rows * l];
        (side ? sV : sU)[ii * R + l] = gptr(M)[id + (size_t)rows * l] + (side ? P.c : P.b) * f;
      }
    }
    CF_WSTAMP(bt, 0);
    if (masks && !lazy)
      for (int o = tid; o < P.D1 + P.D2; o += kCfNT) {
        const int side = o >= P.D1 ? 1 : 0, f = o - side * P.D1;
        const uint64_t* mk = side ? vmk : umk;
        unsigned short* lst = flist + (size_t)o * m;
        int c = 0;
        for (int z0 = 0; z0 < B; z0 += 8) {
          uint64_t m8[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) m8[u] = z0 + u < B ? mk[z0 + u] : 0ull;
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if ((m8[u] >> f) & 1ull) lst[c++] = (unsigned short)(z0 + u);
        }
        fcnt[o] = c;
      }
    __syncthreads();
    CF_STAMP(bt, 3);
    // (sumU*w)[ii, :] and (sumV*w')[ii, :] on the fp64 matrix cores: one wave per (side, 16-rating
    // tile), ⌈R/16⌉ column tiles, K = R in steps of 4 (v_mfma_f64_16x16x4f64; lane λ feeds
    // A[λ&15][k0 + (λ>>4)] = sumX[rating][k] and B[k0 + (λ>>4)][λ&15] = w entry; rows past B and
    // columns past R read clamped addresses and are not stored, K past R is zero)
    {
      constexpr int NTc = (R + 15) / 16;
      const int lane = tid & 63, wv = uni(tid >> 6), mts = (B + 15) / 16;
      const int rl = lane & 15, kl = lane >> 4;
      for (int t = wv; t < 2 * mts; t += kCfNW) {
        const int side = t >= mts ? 1 : 0, m0 = (t - side * mts) * 16;
        int zo = 0;                        // opaque: addresses formed per tile, not hoisted out of
        asm volatile("" : "+v"(zo));       // the step loop into spilled registers
        const double* S = (side ? sV : sU) + zo;
        const double* wz = w_l + zo;
        const int arow = min(m0 + rl, B - 1);
        pd4 acc[NTc];
#pragma unroll
        for (int nt = 0; nt < NTc; ++nt) acc[nt] = pd4{0.0, 0.0, 0.0, 0.0};
        // every operand read before the first MFMA (KS·(1 + NTc) reads in flight; the scheduling
        // barrier keeps the compiler from pairing each MFMA with a read and its wait)
        constexpr int KS = (R + 3) / 4;
        double av[KS], bv[KS][NTc];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int k = 4 * ks + kl, kc = min(k, R - 1);
          const double x = S[arow * R + kc];            // unconditional read, then a select
          av[ks] = k < R ? x : 0.0;
#pragma unroll
          for (int nt = 0; nt < NTc; ++nt) {
            const int n = min(nt * 16 + rl, R - 1);
            bv[ks][nt] = side ? wz[n + R * kc] : wz[kc + R * n];
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
          for (int nt = 0; nt < NTc; ++nt)
            acc[nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ks], bv[ks][nt], acc[nt], 0, 0, 0);
        double* Tt = side ? tV : tU;
#pragma unroll
        for (int nt = 0; nt < NTc; ++nt)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int row = m0 + kl + 4 * q, col = nt * 16 + rl;
            if (row < B && col < R) Tt[row * R + col] = acc[nt][q];
          }
      }
    }
    __syncthreads();
    CF_STAMP(bt, 4);
    for (int ii = tid; ii < B; ii += kCfNT) {       // residual rating − a·sum((sumU*w).*sumV)
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < R; ++j) s = fma(tU[ii * R + j], sV[ii * R + j], s);
      er[ii] = er[ii] - P.a * s;
    }
    __syncthreads();
    CF_STAMP(bt, 5);
    const int Bn = bt + 1 < bt0 + nb ? min(m, N - (bt + 1) * m) : 0;
    if (lazy && m <= kCfNT && tid < Bn) {             // the next batch, in flight under the gradients
      pf_u = C.ep_user[(bt + 1) * m + tid];
      pf_m = C.ep_movie[(bt + 1) * m + tid];
      pf_r = C.ep_rating[(bt + 1) * m + tid];
    }
    // gradw (:466, :473-477) and the w step of :479-483 into wn
    // (GPT_fixw / GPT_fixw_sideinfo, :56-156 / :282-404: w is fixed — no gradw, no step)
    // gradw[i, j] = Σ_ii sumU[ii, i]·(er_ii·sumV[ii, j]) on the fp64 matrix cores: one wave per
    // 16 × 16 tile of w, K = the batch's ratings in steps of 4 (past B: zero); then the w step of
    // :479-483 per entry.  (The round-4 form summed er·(sumU·sumV)·is2 rating by rating per entry:
    // the same sum, rounded differently.)
    if (CF_EXP(2)) __builtin_amdgcn_s_setprio(2);
    if (!P.fixw && !CF_EXP(8)) {
      constexpr int NTw = (R + 15) / 16;
      const int lane = tid & 63, wv = uni(tid >> 6), rl = lane & 15, kl = lane >> 4;
      for (int t = wv; t < NTw * NTw; t += kCfNW) {
        const int it = t / NTw, jt = t - it * NTw;
        const int ia = min(it * 16 + rl, R - 1), jb = min(jt * 16 + rl, R - 1);
        int zo = 0;                        // (as above)
        asm volatile("" : "+v"(zo));
        const double* sUz = sU + zo;
        const double* sVz = sV + zo;
        const double* erz = er + zo;
        pd4 acc = pd4{0.0, 0.0, 0.0, 0.0};
        // four K steps per pass, every LDS read of the pass issued before its MFMAs (reads
        // unconditional at clamped rows, the operand past B selected to zero: no branch around
        // a read, which had left each step's read latency in front of its MFMA)
        for (int k0 = 0; k0 < B; k0 += 16) {
          double x4[4], er4[4], s4[4], av[4], bv[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int kc = min(k0 + 4 * u + kl, B - 1);
            x4[u] = sUz[kc * R + ia];
            er4[u] = erz[kc];
            s4[u] = sVz[kc * R + jb];
          }
          __builtin_amdgcn_sched_barrier(0);             // reads, operands, MFMAs in that order
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            av[u] = k0 + 4 * u + kl < B ? x4[u] : 0.0;
            bv[u] = er4[u] * s4[u];
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int u = 0; u < 4; ++u)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = it * 16 + kl + 4 * q, j = jt * 16 + rl;
          if (i < R && j < R) {
            const int ow = i + R * j;
            const double G = acc[q] * is2 * cN - w_l[ow] / (P.sigma_w * P.sigma_w);
            double wn = w_l[ow] + P.epsw * G / 2;
            if (P.langevin)
              wn = wn + sqrt(P.epsw) * normal_at(P.seed, (uint32_t)ow, (uint32_t)step, kCfWNoise, 0);
            wn_l[ow] = wn;
          }
        }
      }
    } else {
      for (int o = tid; o < R * R; o += kCfNT) wn_l[o] = w_l[o];
    }
    CF_WSTAMP(bt, 1);
    if (lazy && !CF_EXP(4)) {
      // feature rows: G[f, l] = Σ_ii [f ∈ mask_ii]·er_ii·T[ii, l] on the fp64 matrix cores (one
      // wave per 16 features × 16 columns of a side, K = the ratings; A = the mask bit as 0 / 1),
      // then the move of every feature the batch carries, in LDS (Fl).  Before the gradient rows:
      // the tiles' MFMA chains then overlap the rows' VALU / LDS work of the other waves of each
      // SIMD (after them, the tiles of two waves per SIMD ran alone at the end of the phase)
      constexpr int LT = (R + 15) / 16;
      const int lane = tid & 63, wv = uni(tid >> 6), rl = lane & 15, kl = lane >> 4;
      const int FT1 = (P.D1 + 15) / 16, FT2 = (P.D2 + 15) / 16;
      // tiles from the last wave down, so they do not queue behind gradw's tiles on waves 0, 1, ..
      // (one tile per wave: all LT column tiles of 16 features on one wave, their chains
      // interleaved, measured slower — 15.8-17.1 k against 10.9-15.6 k cycles)
      for (int t = kCfNW - 1 - wv; t < (FT1 + FT2) * LT; t += kCfNW) {
        const int ft = t / LT, lt = t - ft * LT, side = ft >= FT1 ? 1 : 0;
        const int f0 = (ft - side * FT1) * 16, Ds = side ? P.D2 : P.D1;
        int zo = 0;
        asm volatile("" : "+v"(zo));
        const uint64_t* mk = (side ? vmk : umk) + zo;
        const double* T = (side ? tU : tV) + zo;
        const double* erz = er + zo;
        const int fa = f0 + rl, lb = min(lt * 16 + rl, R - 1);
        pd4 acc = pd4{0.0, 0.0, 0.0, 0.0};
        for (int k0 = 0; k0 < B; k0 += 16) {            // (four K steps per pass, as gradw's)
          // the pass's twelve reads issued together, then the operands, then the MFMAs (the
          // scheduling barriers keep the compiler from interleaving them one step at a time)
          uint64_t mr[4];
          double er4[4], t4[4], av[4], bv[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int kc = min(k0 + 4 * u + kl, B - 1);
            mr[u] = mk[kc];
            er4[u] = erz[kc];
            t4[u] = T[kc * R + lb];
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            // the bit as arithmetic, no select: a select let the compiler sink the mask read
            // under a branch
            const unsigned bit = (unsigned)(mr[u] >> fa) & 1u & (unsigned)(k0 + 4 * u + kl < B);
            av[u] = (double)bit;
            bv[u] = er4[u] * t4[u];
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int u = 0; u < 4; ++u)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc, 0, 0, 0);
        }
        const double ab = P.a * (side ? P.c : P.b);
        const unsigned long long hs = hit[side];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int f = f0 + kl + 4 * q, l = lt * 16 + rl;
          if (f < Ds && l < R && ((hs >> f) & 1ull)) {
            const int o = ((side ? P.D1 : 0) + f) * R + l;
            const double g = ab * acc[q] * is2, m0 = Fc[o];
            Fl[o] = m0 + P.epsU * (g * cN - m0 / su2) / 2;
          }
        }
      }
    }
    CF_WSTAMP(bt, 2);
    if (CF_EXP(2)) __builtin_amdgcn_s_setprio(0);
    // gradient rows in rating order (:467-471): the first rating of a user / movie in the batch
    // sums its row; feature rows sum over the ratings whose user / movie carries them
    // (the same-id positions of a first occurrence are walked through the next links, ascending)
    // (four items per thread with their reads batched measured slower: 260.5-261.3 k against
    // 268.3-268.5 k fold-steps/s, profiles/r6_ml_ab.txt)
    for (int o = tid; o < (CF_EXP(1) ? 0 : 2 * B * R); o += kCfNT) {
      const int side = o >= B * R ? 1 : 0, x = o - side * (B * R), ii = x / R, l = x - ii * R;
      const int* nxl = side ? vnx : unx;
      if (!(nxl[ii] >> 16)) continue;
      const int id = (side ? ms : us)[ii];
      const double* T = side ? tU : tV;     // Vtemp = e·(sumU*w), Utemp = e·(sumV*w')
      double g = 0.0;
      for (int z = ii; z >= 0; z = (nxl[z] & 0xFFFF) - 1) g += P.a * (er[z] * T[z * R + l]) * is2;
      const size_t e = id + (size_t)(side ? P.rowsV : P.rowsU) * l;
      if (lazy) {                                     // the row's move of this step (cf_move)
        const double m0 = mcl[o];                     // the value the sums phase read (no update since)
        gptr_w(side ? C.GV : C.GU)[(size_t)id * R + l] = m0 + P.epsU * (g * cN - m0 / su2) / 2;
      } else {
        gptr_w(side ? C.GV : C.GU)[e] = g * cN;
      }
    }
    CF_WSTAMP(bt, 3);
    for (int o = tid; o < (lazy ? 0 : (P.D1 + P.D2) * R); o += kCfNT) {
      const int side = o >= P.D1 * R ? 1 : 0;
      const int x = side ? o - P.D1 * R : o, f = x / R, l = x - f * R;
      const int* ids = side ? ms : us;
      const int row = (side ? P.n2 : P.n1) + f;
      const double ab = P.a * (side ? P.c : P.b);
      const double* T = side ? tU : tV;
      double g = 0.0;
      bool hit = false;
      if (masks) {
        const int fo = side ? P.D1 + f : f;
        const unsigned short* lst = flist + (size_t)fo * m;
        const int c = fcnt[fo];
        hit = c > 0;
        int x = 0;
        for (; x + 4 <= c; x += 4) {                    // four list entries' reads in flight
          int z4[4];
          double t4[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) z4[u] = lst[x + u];
#pragma unroll
          for (int u = 0; u < 4; ++u) t4[u] = ab * (er[z4[u]] * T[z4[u] * R + l]) * is2;
#pragma unroll
          for (int u = 0; u < 4; ++u) g += t4[u];
        }
        for (; x < c; ++x) {
          const int z = lst[x];
          g += ab * (er[z] * T[z * R + l]) * is2;
        }
      } else {
        const int32_t* ptr = side ? P.vptr : P.uptr;
        const int32_t* fe = side ? P.vfe : P.ufe;
        for (int z = 0; z < B; ++z) {
          const int id = ids[z];
          bool has = false;
          for (int q = ptr[id]; q < ptr[id + 1]; ++q) has |= fe[q] == row;
          if (has) { g += ab * (er[z] * T[z * R + l]) * is2; hit = true; }
        }
      }
      if (hit) gptr_w(side ? C.GV : C.GU)[row + (size_t)(side ? P.rowsV : P.rowsU) * l] = g * cN;
    }
    __syncthreads();
    CF_STAMP(bt, 6);
    if (lazy && m <= kCfNT && tid < Bn) {             // ... and its feature masks
      pf_mu = P.umask[pf_u];
      pf_mm = P.vmask[pf_m];
    }
    if (lazy) {                                       // the moved rows are current as of jl + 1
      for (int o = tid; o < 2 * B; o += kCfNT) {
        const int side = o >= B ? 1 : 0, ii = o - side * B;
        if ((side ? vnx : unx)[ii] >> 16) cur[(side ? P.rowsU : 0) + (side ? ms : us)[ii]] = jl + 1;
      }
      for (int o = tid; o < P.D1 + P.D2; o += kCfNT) {
        const int side = o >= P.D1 ? 1 : 0, f = o - side * P.D1;
        if ((hit[side] >> f) & 1ull) cur[(side ? P.rowsU + P.n2 : P.n1) + f] = jl + 1;
      }
    }
    if (domove == 1 && (!cf_move<R>(P, C.U, C.GU, P.rowsU, 0, step, scr) ||
                   !cf_move<R>(P, C.V, C.GV, P.rowsV, 1, step, scr))) {
      if (tid == 0) __hip_atomic_store(C.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    CF_STAMP(bt, 7);
    for (int o = tid; o < R * R; o += kCfNT) w_l[o] = wn_l[o];
    if (lazy) lds_barrier(); else __syncthreads();    // (no global writes since the last fence)
  }
  if (lazy) {                                         // every row brought to the launch's end
    const int TR = (int)((cf_lazy_offset(R, m, nfeat) - 16 * (size_t)R * R) / (8 * R));
    cf_rows_out<R>(C.GU, C.U, P.rowsU, P.n1, Fl, cur, cpow, nb, sU, TR);
    cf_rows_out<R>(C.GV, C.V, P.rowsV, P.n2, Fl + P.D1 * R, cur + P.rowsU, cpow, nb, sU, TR);
  }
  for (int o = tid; o < R * R; o += kCfNT) C.w[o] = w_l[o];
}

// Every train (blockIdx.y = 0) / test (1) rating of a chain: running average of a·sumUᵀw sumV
// (:526-529, :536-539), de-standardised and cut off, squared error summed per block into
// C.sse[2·blockIdx.x + set] (the host adds the partials in order).
template <int R>
__global__ __launch_bounds__(256) void cf_eval_kernel(CfParams P, const CfChain* chains, int counter) {
  __shared__ double red[4];
  const CfChain C = chains[blockIdx.z];
  // a stopped (early stop) or bailed-out fold keeps its last predictions
  if (__hip_atomic_load(C.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  const double ymean = C.ymean, ystd = C.ystd;
  const int set = blockIdx.y;
  const int n = set ? C.Ntest : C.N;
  const int i = blockIdx.x * 256 + threadIdx.x;
  double se = 0.0;
  if (i < n) {
    const int u = set ? C.te_user[i] : C.tr_user[i];
    const int v = set ? C.te_movie[i] : C.tr_movie[i];
    double su[R], sv[R];
#pragma unroll
    for (int l = 0; l < R; ++l) {
      double f = 0.0;
      for (int z = P.uptr[u]; z < P.uptr[u + 1]; ++z) f += C.U[P.ufe[z] + (size_t)P.rowsU * l];
      su[l] = C.U[u + (size_t)P.rowsU * l] + P.b * f;
      double g = 0.0;
      for (int z = P.vptr[v]; z < P.vptr[v + 1]; ++z) g += C.V[P.vfe[z] + (size_t)P.rowsV * l];
      sv[l] = C.V[v + (size_t)P.rowsV * l] + P.c * g;
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      double t = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) t = fma(su[k], C.w[k + R * j], t);
      s = fma(t, sv[j], s);
    }
    const double pred = P.a * s;
    double* run = set ? C.testpred : C.trainpred;
    const double avgp = (run[i] * counter + pred) / (counter + 1);
    run[i] = avgp;
    const double fin = fmin(fmax(avgp * ystd + ymean, 1.0), 5.0);
    const double d = ystd * (set ? C.te_rating[i] : C.tr_rating[i]) + ymean - fin;
    se = d * d;
  }
  se = wave_sum(se);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) red[wv] = se;
  __syncthreads();
  if (threadIdx.x == 0) C.sse[2 * blockIdx.x + set] = red[0] + red[1] + red[2] + red[3];
}

// ============================================================================ GPT_fullw_gibbs
// 100k_movielensExperiment.jl:1032-1129.  One wave per user (side 0) / movie (side 1): the
// conditional of its row given the other side and w — X = V[Ni,:]·wᵀ (users) or U[Nj,:]·w
// (movies), precision XᵀX/σ² + I/σ_u², in-wave Cholesky, row = chol(·,:U) \ z +
// (precision \ Xᵀy)/σ² (:1063-1070, :1077-1084).  status = 1: not SPD.
// The row's ratings go in chunks of 64: lane λ gathers rating zc + λ's other-side row and forms
// its X row (all 64 gathers in flight; the round-4 kernel formed one X row at a time behind two
// dependent global loads, 0.84 ms per launch for the movie with the most ratings), the rows wait
// in LDS, then the precision / right-hand side accumulate rating by rating in the same order and
// with the same fma chains as before (identical doubles).
// MODE 1 (w | U, V statistics, no draw): X = V[Ni,:] itself; writes H_u = Σ_i V[m_i,:]ᵀV[m_i,:]
// (R², entry a + R·a') and h_u = Σ_i y_i V[m_i,:] (R) per user, zeros for a user without ratings.
template <int R, int MODE>
__global__ __launch_bounds__(256) void cfg_rows_kernel(int side, const double* __restrict__ W,
                                                       const double* __restrict__ Oth, int rows_oth,
                                                       double* __restrict__ Me, int rows_me,
                                                       const int32_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ lst,
                                                       const int32_t* __restrict__ other,
                                                       const double* __restrict__ y,
                                                       double signal_var, double su2,
                                                       uint64_t seed, uint32_t sweep,
                                                       uint32_t stream, int32_t* __restrict__ status,
                                                       double* __restrict__ Hout,
                                                       double* __restrict__ hout) {
  constexpr int NE = (R * R + 63) / 64;
  __shared__ double Ls[4][R * R], rh[4][R], zs[4][R], Ws[R * R];
  __shared__ double Xs[4][64 * R + 64];             // a chunk's X rows | their y
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (MODE == 0)
    for (int e = threadIdx.x; e < R * R; e += 256) Ws[e] = W[e];
  __syncthreads();
  const int ent = blockIdx.x * 4 + wv;
  if (ent >= rows_me) return;                       // whole waves only: no block barriers below
  const int z0 = ptr[ent], z1 = ptr[ent + 1];
  double acc[NE];
#pragma unroll
  for (int t = 0; t < NE; ++t) acc[t] = 0.0;
  double racc = 0.0;
  if (MODE == 0 && z0 == z1) return;                // no ratings: the row is left as it is
  double* X = Xs[wv];
  double* Y = X + 64 * R;
  // this lane's precision entries e = lane + 64t as (row, column) offsets into an X row; entries
  // past R² read X[0]·X[0] and are never stored (no branch inside the rating loop)
  int oa[NE], ob[NE];
#pragma unroll
  for (int t = 0; t < NE; ++t) {
    const int e = min(lane + 64 * t, R * R);
    oa[t] = e < R * R ? e % R : 0;
    ob[t] = e < R * R ? e / R : 0;
  }
  const int ol = lane < R ? lane : 0;
  for (int zc = z0; zc < z1; zc += 64) {
    const int cnt = min(64, z1 - zc);
    if (lane < cnt) {
      const int ri = lst[zc + lane], o = other[ri];
      double orow[R];
#pragma unroll
      for (int b = 0; b < R; ++b) orow[b] = Oth[o + (size_t)rows_oth * b];
      if (MODE == 1) {
#pragma unroll
        for (int a = 0; a < R; ++a) X[lane * R + a] = orow[a];
      } else if (side == 0) {
#pragma unroll
        for (int a = 0; a < R; ++a) {
          double s2 = 0.0;
#pragma unroll
          for (int b = 0; b < R; ++b) s2 = fma(orow[b], Ws[a + R * b], s2);
          X[lane * R + a] = s2;
        }
      } else {
#pragma unroll
        for (int a = 0; a < R; ++a) {
          double s2 = 0.0;
#pragma unroll
          for (int k = 0; k < R; ++k) s2 = fma(orow[k], Ws[k + R * a], s2);
          X[lane * R + a] = s2;
        }
      }
      Y[lane] = y[ri];
    }
    wave_sync();
    // ratings in order (the same fma chain per entry as rating-by-rating), four per pass so their
    // LDS reads are in flight together
    int zz = 0;
    for (; zz + 4 <= cnt; zz += 4) {
      double xa[4][NE], xb[4][NE], xl[4], yy[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double* x = X + (zz + q) * R;
#pragma unroll
        for (int t = 0; t < NE; ++t) { xa[q][t] = x[oa[t]]; xb[q][t] = x[ob[t]]; }
        xl[q] = x[ol];
        yy[q] = Y[zz + q];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int t = 0; t < NE; ++t) acc[t] = fma(xa[q][t], xb[q][t], acc[t]);
        racc = fma(xl[q], yy[q], racc);
      }
    }
    for (; zz < cnt; ++zz) {
      const double* x = X + zz * R;
#pragma unroll
      for (int t = 0; t < NE; ++t) acc[t] = fma(x[oa[t]], x[ob[t]], acc[t]);
      racc = fma(x[ol], Y[zz], racc);
    }
    wave_sync();
  }
  if (MODE == 1) {
#pragma unroll
    for (int t = 0; t < NE; ++t) {
      const int e = lane + 64 * t;
      if (e < R * R) Hout[(size_t)ent * R * R + e] = acc[t];
    }
    if (lane < R) hout[(size_t)ent * R + lane] = racc;
    return;
  }
  double* A = Ls[wv];
#pragma unroll
  for (int t = 0; t < NE; ++t) {
    const int e = lane + 64 * t;
    if (e < R * R) A[e] = acc[t] / signal_var + ((e % R) == (e / R) ? 1.0 / su2 : 0.0);
  }
  if (lane < R) {
    rh[wv][lane] = racc;
    zs[wv][lane] = normal_at(seed, (uint32_t)lane, sweep, stream, (uint32_t)ent);
  }
  wave_sync();
  // lower Cholesky with lane i holding row i (A[i + R·k]); pivots and multipliers broadcast by
  // v_readlane — the column loop's operations in its order (identical doubles)
  bool bad = false;
  {
    double rw[R];
#pragma unroll
    for (int k = 0; k < R; ++k) rw[k] = A[ol + R * k];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const double d = readlane_d(rw[j], j);
      bad |= !(d > 0.0);
      const double pv = sqrt(d);
      if (lane == j) rw[j] = pv;
      if (lane > j) rw[j] /= pv;
#pragma unroll
      for (int k = j + 1; k < R; ++k) {
        const double lkj = readlane_d(rw[j], k);
        if (lane >= k) rw[k] -= rw[j] * lkj;
      }
    }
    if (lane < R)
#pragma unroll
      for (int k = 0; k < R; ++k)
        if (k <= lane) A[lane + R * k] = rw[k];
  }
  wave_sync();
  if (lane == 0) {
    if (bad) *status = 1;
    double* rb = rh[wv];
    double* zb = zs[wv];
    for (int i = 0; i < R; ++i) {                   // L⁻¹ rhs
      double s2 = rb[i];
      for (int k = 0; k < i; ++k) s2 -= A[i + R * k] * rb[k];
      rb[i] = s2 / A[i + R * i];
    }
    for (int i = R - 1; i >= 0; --i) {              // L⁻ᵀ (L⁻¹ rhs) and L⁻ᵀ z
      double s2 = rb[i], s3 = zb[i];
      for (int k = i + 1; k < R; ++k) {
        s2 -= A[k + R * i] * rb[k];
        s3 -= A[k + R * i] * zb[k];
      }
      rb[i] = s2 / A[i + R * i];
      zb[i] = s3 / A[i + R * i];
    }
    for (int a = 0; a < R; ++a) Me[ent + (size_t)rows_me * a] = zb[a] + rb[a] / signal_var;
  }
}

// The w | U, V precision without the N × R² Kronecker design (:1088-1092): grouping the ratings
// by user, Kronᵀ·Kron[(a,b), (a',b')] = Σ_i V[m_i,a]U[u_i,b]V[m_i,a']U[u_i,b'] =
// Σ_u H_u[a,a']·U[u,b]U[u,b'], i.e. Z = Hᵀ·P with H (n1 × R², MODE-1 rows) and P_u = U[u,:]ᵀU[u,:]
// (n1 × R²): a GEMM with K = n1 (0.3 GFLOP at r = 20 against the 12.8 GFLOP SYRK of the 256 MB
// design).  Block = a 64 × 64 tile of Z over one K slice (blockIdx.z), 4 × 4 outputs per thread;
// partial tiles go to Zp[slice] and cfg_wprec_fin_kernel adds the slices in order.
constexpr int kWpTile = 64, kWpKc = 16, kWpSlices = 4;
template <int R>
__global__ __launch_bounds__(256) void cfg_wprec_kernel(const double* __restrict__ H,
                                                        const double* __restrict__ U, int n1,
                                                        double* __restrict__ Zp) {
  constexpr int P = R * R;
  __shared__ __attribute__((aligned(16))) double Hs[kWpKc][kWpTile], Ps[kWpKc][kWpTile];
  __shared__ double Us[kWpKc][R];
  const int tid = threadIdx.x, tr = tid & 15, tc = tid >> 4;
  const int e0 = blockIdx.x * kWpTile, f0 = blockIdx.y * kWpTile;
  const int per = (n1 + kWpSlices - 1) / kWpSlices;
  const int u0 = blockIdx.z * per, u1 = min(n1, u0 + per);
  double acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;
  for (int uc = u0; uc < u1; uc += kWpKc) {
    const int cnt = min(kWpKc, u1 - uc);
    for (int x = tid; x < kWpKc * R; x += 256) {
      const int k = x / R, b = x - k * R;
      Us[k][b] = k < cnt ? U[(uc + k) + (size_t)n1 * b] : 0.0;
    }
    for (int x = tid; x < kWpKc * kWpTile; x += 256) {
      const int k = x / kWpTile, c = x - k * kWpTile;
      Hs[k][c] = (k < cnt && e0 + c < P) ? H[(size_t)(uc + k) * P + e0 + c] : 0.0;
    }
    __syncthreads();
    for (int x = tid; x < kWpKc * kWpTile; x += 256) {
      const int k = x / kWpTile, c = x - k * kWpTile, f = min(f0 + c, P - 1);
      Ps[k][c] = Us[k][f % R] * Us[k][f / R];
    }
    __syncthreads();
    for (int k = 0; k < cnt; ++k) {
      double h[4], q[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { h[i] = Hs[k][tr + 16 * i]; q[i] = Ps[k][tc + 16 * i]; }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fma(h[i], q[j], acc[i][j]);
    }
    __syncthreads();
  }
  double* Z = Zp + (size_t)blockIdx.z * P * P;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = e0 + tr + 16 * i, f = f0 + tc + 16 * j;
      if (e < P && f < P) Z[(size_t)e + (size_t)P * f] = acc[i][j];
    }
}

// M[(a·R + b) + p·(a'·R + b')] = alpha·Σ_slices Z[(a + R·a') + p·(b + R·b')] + beta·δ, p = R²
template <int R>
__global__ __launch_bounds__(256) void cfg_wprec_fin_kernel(const double* __restrict__ Zp,
                                                            double alpha, double beta,
                                                            double* __restrict__ M) {
  constexpr int P = R * R;
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= P * P) return;
  const int c = o % P, c2 = o / P;
  const int a = c / R, b = c - a * R, a2 = c2 / R, b2 = c2 - a2 * R;
  const size_t zi = (size_t)(a + R * a2) + (size_t)P * (b + R * b2);
  double s = Zp[zi];
#pragma unroll
  for (int sl = 1; sl < kWpSlices; ++sl) s += Zp[(size_t)sl * P * P + zi];
  M[o] = alpha * s + (c == c2 ? beta : 0.0);
}

// x[a·R + b] = ysc·Σ_u h_u[a]·U[u,b]  (Kronᵀ·y, :1093), one workgroup, users in order
template <int R>
__global__ __launch_bounds__(512) void cfg_wrhs_kernel(const double* __restrict__ hv,
                                                       const double* __restrict__ U, int n1,
                                                       double ysc, double* __restrict__ x) {
  __shared__ double hs[64][R], us[64][R];
  const int tid = threadIdx.x, a = tid / R, b = tid - a * R;
  double s = 0.0;
  for (int uc = 0; uc < n1; uc += 64) {
    const int cnt = min(64, n1 - uc);
    for (int e = tid; e < 64 * R; e += 512) {
      const int k = e / R, l = e - k * R;
      hs[k][l] = k < cnt ? hv[(size_t)(uc + k) * R + l] : 0.0;
      us[k][l] = k < cnt ? U[(uc + k) + (size_t)n1 * l] : 0.0;
    }
    __syncthreads();
    if (tid < R * R)
      for (int k = 0; k < cnt; ++k) s = fma(hs[k][a], us[k][b], s);
    __syncthreads();
  }
  if (tid < R * R) x[tid] = ysc * s;
}

hipError_t launch_cfg_rows(int side, int r, const double* W, const double* Oth, int rows_oth,
                           double* Me, int rows_me, const int32_t* ptr, const int32_t* lst,
                           const int32_t* other, const double* y, double signal_var, double su2,
                           uint64_t seed, uint32_t sweep, uint32_t stream, int32_t* status,
                           hipStream_t st) {
  switch (r) {
#define CASE(RR)                                                                              \
  case RR:                                                                                    \
    hipLaunchKernelGGL((cfg_rows_kernel<RR, 0>), dim3((rows_me + 3) / 4), dim3(256), 0, st,   \
                       side, W, Oth, rows_oth, Me, rows_me, ptr, lst, other, y, signal_var,   \
                       su2, seed, sweep, stream, status, nullptr, nullptr);                   \
    break;
    GPT_CF_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// w | U, V (GPT_fullw_gibbs :1088-1094): precision M = Kronᵀ·Kron/σ² + I/σ_w² and rhs x =
// Kronᵀ·y/σ² from per-user statistics.  Scratch: H (n1·r²), h (n1·r), Zp (kWpSlices·r⁴).
size_t cfg_wsystem_scratch_dbl(int r, int n1) {
  return (size_t)n1 * r * r + (size_t)n1 * r + (size_t)kWpSlices * r * r * r * r;
}

hipError_t launch_cfg_wsystem(int r, const double* U, int n1, const double* V, int n2,
                              const int32_t* uptr, const int32_t* ulst, const int32_t* movies,
                              const double* y, double alpha, double beta, double ysc,
                              double* scratch, double* M, double* x, hipStream_t st) {
  const int p = r * r;
  double* H = scratch;
  double* hv = H + (size_t)n1 * p;
  double* Zp = hv + (size_t)n1 * r;
  switch (r) {
#define CASE(RR)                                                                              \
  case RR:                                                                                    \
    hipLaunchKernelGGL((cfg_rows_kernel<RR, 1>), dim3((n1 + 3) / 4), dim3(256), 0, st, 0,      \
                       nullptr, V, n2, nullptr, n1, uptr, ulst, movies, y, 1.0, 1.0,          \
                       (uint64_t)0, 0u, 0u, nullptr, H, hv);                                  \
    hipLaunchKernelGGL(cfg_wprec_kernel<RR>,                                                  \
                       dim3((p + kWpTile - 1) / kWpTile, (p + kWpTile - 1) / kWpTile,        \
                            kWpSlices), dim3(256), 0, st, H, U, n1, Zp);                      \
    hipLaunchKernelGGL(cfg_wprec_fin_kernel<RR>, dim3((p * p + 255) / 256), dim3(256), 0, st, \
                       Zp, alpha, beta, M);                                                   \
    hipLaunchKernelGGL(cfg_wrhs_kernel<RR>, dim3(1), dim3(512), 0, st, hv, U, n1, ysc, x);    \
    break;
    GPT_CF_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Per sweep kept (GPT_fullw_gibbs / GPT_fixw_gibbs bookkeeping, :1097-1118): the train / test
// RMSE from the evaluation kernel's block partials (added in block order, as the host used to),
// and the cut-off de-standardised test prediction of the sweep.
__global__ __launch_bounds__(256) void cfg_keep_kernel(const CfChain* __restrict__ chains,
                                                       int neval, double* __restrict__ rmse,
                                                       double* __restrict__ tp_out) {
  const CfChain C = chains[0];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < C.Ntest)
    tp_out[i] = fmin(fmax(C.testpred[i] * C.ystd + C.ymean, 1.0), 5.0);
  if (i == 0) {
    double s0 = 0.0, s1 = 0.0;
    for (int z = 0; z < neval; ++z) { s0 += C.sse[2 * z]; s1 += C.sse[2 * z + 1]; }
    rmse[0] = sqrt(s0 / (double)C.N);
    rmse[1] = sqrt(s1 / (double)C.Ntest);
  }
}

hipError_t launch_cfg_keep(const CfChain* chains, int Ntest, int neval, double* rmse,
                           double* tp_out, hipStream_t st) {
  hipLaunchKernelGGL(cfg_keep_kernel, dim3((Ntest + 255) / 256), dim3(256), 0, st, chains, neval,
                     rmse, tp_out);
  return hipGetLastError();
}

// The per-feature rating lists (fcnt, flist) sit last in the batch carve and exist only on the
// bitmask path (D1, D2 <= 64); the CSR path sizes them to zero.
size_t cf_lds_bytes(int r, int m, int nfeat, bool masks) {
  const size_t lists = masks ? 4 * (size_t)nfeat + 2 * (size_t)nfeat * m : 0;
  const size_t base = 8 * (2 * (size_t)r * r + 4 * (size_t)m * r + m) + 16 * (size_t)m +
                      4 * (4 * (size_t)m + 2) + lists + 16;
  const size_t nn = 2 * (size_t)r;
  const size_t stf = 8 * (3 * (size_t)r * r + 7 * nn * nn + 7 * (size_t)r * r + nn * r + r) + 16;
  const size_t moves = 8 * 2 * (size_t)r * r + stf;      // w | wn | Stiefel scratch over the batch
  return al16(base > moves ? base : moves);
}


// LDS of the lazy-move epoch launch (domove = 2): the batch carve, then cpow[0..nb], cur[rows],
// the feature rows Fl, Fc (nfeat × r each) and the two hit masks
size_t cf_lazy_lds_bytes(int r, int m, int nfeat, int rows, int nb) {
  return al16(cf_lazy_offset(r, m, nfeat) + 8 * ((size_t)nb + 1) + 4 * (size_t)rows) +
         16 * (size_t)nfeat * r + 16 + 16 + 16 * (size_t)m * r;
}

bool cf_rank_supported(int r) {
  switch (r) {
#define CASE(RR) case RR:
    GPT_CF_RANKS(CASE)
#undef CASE
    return true;
    default: return false;
  }
}

template <int RR, int DM>
static hipError_t launch_cf_epoch_t(const CfParams& P, const CfChain* chains, int nchains,
                                    long long step0, int bt0, int nb, size_t lds, hipStream_t st,
                                    const long long* step_base) {
  static std::atomic<uint64_t> attr{0};
  hipError_t e = set_max_lds_once((const void*)cf_epoch_kernel<RR, DM>, 160 * 1024, attr);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((cf_epoch_kernel<RR, DM>), dim3(nchains), dim3(kCfNT), lds, st, P, chains,
                     step_base, step0, bt0, nb);
  return hipGetLastError();
}

hipError_t launch_cf_epoch(const CfParams& P, const CfChain* chains, int nchains, long long step0,
                           int bt0, int nb, int domove, hipStream_t st,
                           const long long* step_base) {
  size_t lds = cf_lds_bytes(P.r, P.m, P.D1 + P.D2, P.D1 <= 64 && P.D2 <= 64);
  if (domove == 2)
    lds = std::max(lds, cf_lazy_lds_bytes(P.r, P.m, P.D1 + P.D2, P.rowsU + P.rowsV, nb));
  switch (P.r) {
#define CASE(RR)                                                                              \
  case RR:                                                                                    \
    if (domove == 1)                                                                          \
      return launch_cf_epoch_t<RR, 1>(P, chains, nchains, step0, bt0, nb, lds, st, step_base); \
    if (domove == 2)                                                                          \
      return launch_cf_epoch_t<RR, 2>(P, chains, nchains, step0, bt0, nb, lds, st, step_base); \
    return launch_cf_epoch_t<RR, 0>(P, chains, nchains, step0, bt0, nb, lds, st, step_base);
    GPT_CF_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
}

// The training ratings of every fold in this epoch's order, once per epoch (the batch kernels
// then read their minibatch contiguously instead of through the permutation).
__global__ __launch_bounds__(256) void cf_gather_kernel(const CfChain* chains, int N) {
  const CfChain C = chains[blockIdx.y];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  const int idx = C.perm[i];
  C.ep_user[i] = C.tr_user[idx];
  C.ep_movie[i] = C.tr_movie[idx];
  C.ep_rating[i] = C.tr_rating[idx];
}

hipError_t launch_cf_gather(const CfChain* chains, int nchains, int N, hipStream_t st) {
  hipLaunchKernelGGL(cf_gather_kernel, dim3((unsigned)((N + 255) / 256), nchains), dim3(256), 0,
                     st, chains, N);
  return hipGetLastError();
}

hipError_t launch_cf_move(const CfParams& P, const CfChain* chains, int nchains, long long step,
                          hipStream_t st, const long long* step_base) {
  const int RE = P.r + (P.r & 1);
  const unsigned blocks = (unsigned)(((long long)(P.rowsU + P.rowsV) * (RE / 2) + 255) / 256);
  const dim3 grid = nchains <= 8 ? dim3(8 * blocks) : dim3(blocks, nchains);
  switch (P.r) {
#define CASE(RR)                                                                              \
  case RR:                                                                                    \
    hipLaunchKernelGGL(cf_move_kernel<RR>, grid, dim3(256), 0, st, P, chains, step_base, step, \
                       nchains);                                                              \
    break;
    GPT_CF_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_cf_eval(const CfParams& P, const CfChain* chains, int nchains, int nmax,
                          int counter, hipStream_t st) {
  dim3 grid((unsigned)((nmax + 255) / 256), 2, nchains);
  switch (P.r) {
#define CASE(RR)                                                                              \
  case RR:                                                                                    \
    hipLaunchKernelGGL(cf_eval_kernel<RR>, grid, dim3(256), 0, st, P, chains, counter);        \
    break;
    GPT_CF_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace gpt
