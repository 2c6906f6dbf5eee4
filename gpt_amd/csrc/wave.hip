// Wave engine for MI355X (gfx950): the SGLD step at ranks past the chain engine (r > 5 — the
// reference's own kin40k configuration runs r = 20 at n = 150, kin40kExperiment.jl:38-51).
//
// At r = 20 one chain's U and its drive take 2·n·r·D doubles (384 KB at n = 150, D = 8): more
// than a CU holds next to eight concurrent 40 × 40 Padé expm.  So a step is two launches:
//
//   wv_vphase_kernel  one workgroup (8 waves) per chain: temp of the batch (formed by the previous
//                     launch) -> V, fhat, residual (computeV / computefhat, GPT_SGLD.jl:208-230),
//                     gradw and the Langevin w step (:393, 411-414), and the core sums
//                     coef[k][i][l] = A[l,k,i]·res_i of every dimension (computeU_phi / computeA,
//                     :246-273) — the only cross-dimension coupling of a step
//   wv_dim_kernel     one wave per (chain, dimension k), 4 waves per CU (one per SIMD, the whole
//                     512-entry register file each): gradU^(k) = Φ_k·coef_k (computePsi + Psi·res
//                     without Psi, :276-408), the Langevin drive, proj (:14-16), geod (:19-37: the
//                     2r × 2r and r × r Padé expm with the matrices in registers and three LDS
//                     operand slots), the U write, and temp[k] of the NEXT batch (phidotU,
//                     :193-205; fp64 MFMA tiles for even n) for the next step's V-phase
//
// The kernel boundary carries the V-phase -> gradU dependency and the temp of the next step; an
// epoch of launches is one hipGraph (capi.hip).  φ rows are read twice per step (gradU here, the
// next step's phidotU one launch later): at r = 20 the step is fp64-compute bound (§8(d): ≈42.5
// MFLOP against 0.9 MB per chain-step), not HBM bound.
#include "device_util.h"

namespace gpt {

// ------------------------------------------------------------ register-blocked NN × NN matrices
// wave_mm's blocked layout: lane (bi, bj) of an NB × NB grid owns the BS × BS block at
// (bi·BS, bj·BS); lanes past NB² hold a duplicate that is never stored.  A product accumulates
// Σ_t A[i,t]·B[t,j] in t order, the doubles of wave_mm.
template <int NN>
struct Blk {
  static constexpr int BS = (NN + 7) / 8, NB = (NN + BS - 1) / BS;
  double v[BS][BS];
};

template <int NN>
__device__ __forceinline__ void blk_origin(int lane, int& i0, int& j0) {
  constexpr int BS = Blk<NN>::BS, NB = Blk<NN>::NB;
  i0 = min(lane / NB, NB - 1) * BS;
  j0 = (lane % NB) * BS;
}

// C = A·B for row-major NN × NN LDS operands
template <int NN>
__device__ __forceinline__ void blk_mm(const double* A, const double* B, Blk<NN>& C, int lane) {
  constexpr int BS = Blk<NN>::BS;
  int i0, j0;
  blk_origin<NN>(lane, i0, j0);
#pragma unroll
  for (int x = 0; x < BS; ++x)
#pragma unroll
    for (int y = 0; y < BS; ++y) C.v[x][y] = 0.0;
#pragma unroll 4
  for (int t = 0; t < NN; ++t) {
    double a[BS], b[BS];
#pragma unroll
    for (int x = 0; x < BS; ++x) {
      a[x] = A[min(i0 + x, NN - 1) * NN + t];
      b[x] = B[t * NN + min(j0 + x, NN - 1)];
    }
#pragma unroll
    for (int x = 0; x < BS; ++x)
#pragma unroll
      for (int y = 0; y < BS; ++y) C.v[x][y] = fma(a[x], b[y], C.v[x][y]);
  }
}

template <int NN>
__device__ __forceinline__ void blk_st(double* C, const Blk<NN>& B, int lane) {
  constexpr int BS = Blk<NN>::BS, NB = Blk<NN>::NB;
  int i0, j0;
  blk_origin<NN>(lane, i0, j0);
  if (lane < NB * NB) {
#pragma unroll
    for (int x = 0; x < BS; ++x)
#pragma unroll
      for (int y = 0; y < BS; ++y)
        if (i0 + x < NN && j0 + y < NN) C[(i0 + x) * NN + j0 + y] = B.v[x][y];
  }
}

template <int NN>
__device__ __forceinline__ double blk_id(int lane, int x, int y) {
  int i0, j0;
  blk_origin<NN>(lane, i0, j0);
  return i0 + x == j0 + y ? 1.0 : 0.0;
}

// Solve M·X = X0 (X holds X0) for column diagonally dominant M with 32 < NN <= 64: wave_solve_dd's
// one-pass register LU (Gaussian elimination that partial pivoting provably leaves unswapped;
// multipliers and pivot rows broadcast by v_readlane, no LDS round trip between pivots) in
// ⌈NN / (64 − NN)⌉ passes, each over [M | the next 64 − NN columns of X] with one column per
// lane.  M is re-factored in every pass with the same operations, so every column sees exactly
// the doubles of wave_solve_dd.  (The two-pass wave_solve_dd2 parks the factors in LDS and
// writes a pivot's multipliers from one lane: 75 k cycles at NN = 40; two columns per lane in
// one pass spilled ~1 400 VGPRs.)  Returns false (nothing written) when M is not diagonally
// dominant.
template <int NN>
__device__ __forceinline__ void wv_solve_dd_pass(const double* M, double* X, double* Us, int xo,
                                                 int lane) {
  constexpr int NX = 64 - NN;                            // right-hand sides per pass
  const bool xl = lane >= NN;
  const int xc = min(xo + lane - NN, NN - 1);            // this lane's X column (clamped)
  const bool xw = xl && xo + lane - NN < NN;             // ... and whether it is written
  double col[NN];
#pragma unroll
  for (int i = 0; i < NN; ++i) col[i] = xl ? X[i * NN + xc] : M[i * NN + min(lane, NN - 1)];
  double rpv[NN];
#pragma unroll
  for (int p = 0; p < NN; ++p) {                        // forward elimination (getrf + L solve):
    const double rp = rcp_nr(readlane_d(col[p], p));    // each lane scales its own pivot-row
    rpv[p] = rp;                                         // entry once, so a row update is one
    const double g = col[p] * rp;                        // broadcast and one FMA
#pragma unroll
    for (int i = p + 1; i < NN; ++i) col[i] = fma(-readlane_d(col[i], p), g, col[i]);
  }
  // back substitution, column-oriented: U's columns go to the scratch slot (lane k writes column
  // k), so U[0..k-1][k] comes as broadcast LDS reads (two entries per read) instead of 2k readlanes
  if (lane < NN) {
#pragma unroll
    for (int i = 0; i < NN; i += 2) *(double2*)(Us + lane * NN + i) = make_double2(col[i], col[i + 1]);
  }
  wave_sync();
#pragma unroll
  for (int k = NN - 1; k >= 0; --k) {
    double u[NN];
#pragma unroll
    for (int i = 0; i < k; i += 2) {
      const double2 u2 = *(const double2*)(Us + k * NN + i);
      u[i] = u2.x;
      if (i + 1 < k) u[i + 1] = u2.y;
    }
    if (xl) {
      col[k] = col[k] * rpv[k];
#pragma unroll
      for (int i = 0; i < k; ++i) col[i] -= col[k] * u[i];
    }
  }
  wave_sync();                                           // every lane has read its X column
  if (xw) {
#pragma unroll
    for (int i = 0; i < NN; ++i) X[i * NN + xc] = col[i];
  }
  wave_sync();
  (void)NX;
}

template <int NN>
__device__ __forceinline__ bool wv_solve_dd_passes(const double* M, double* X, double* Us, int lane,
                                                   int ncols) {
  static_assert(NN > 32 && NN < 64 && NN % 2 == 0, "one X column per lane beside M's");
  bool dd = true;
  {
    const int lc = min(lane, NN - 1);
    double off = 0.0;
#pragma unroll
    for (int i = 0; i < NN; ++i)
      if (i != lc) off += fabs(M[i * NN + lc]);
    dd = lane >= NN || fabs(M[lc * NN + lc]) > off;
  }
  if (!__all(dd)) return false;
#pragma unroll 1
  for (int xo = 0; xo < ncols; xo += 64 - NN) wv_solve_dd_pass<NN>(M, X, Us, xo, lane);
  return true;
}

// expm(S0) (NN × NN, row-major in LDS slot S0; overwritten) into slot S1, S2 scratch: the Padé
// scaling-and-squaring of wave_expm (Julia Base 0.3 expm!: degrees 3/5/7/9 below ‖A‖₁ = 2.1,
// degree 13 with 2^-s scaling above), with the polynomial terms in registers.  Returns true if
// the result holds a NaN (the geod bail-out, GPT_SGLD.jl:23-26).  ncols < NN: only columns
// [0, ncols) of the result are wanted (geod reads E[:, 1:r]); without squarings (‖A‖₁ <= 5.4) the
// solve then takes those right-hand sides only — each column's operations are the full solve's,
// so they are the same doubles — and the NaN check covers them (with squarings every column is
// solved and checked).
template <int NN>
__device__ __forceinline__ bool wv_expm(double* S0, double* S1, double* S2, int lane,
                                        long long* st = nullptr, int ncols = NN) {
  constexpr int BS = Blk<NN>::BS;
  double cs = 0.0;
  {
    const int lc = min(lane, NN - 1);
#pragma unroll
    for (int i = 0; i < NN; ++i) cs += fabs(S0[i * NN + lc]);
    if (lane >= NN) cs = 0.0;
  }
  // a non-finite ‖A‖₁ (an Inf or NaN entry): the oracle's NaN result (Julia's expm! would throw at
  // ceil(Int, log2(nA/5.4))), i.e. geod's bail-out; wave_max (fmax) alone would drop a NaN column
  if (__any(!(cs <= 1.79769313486231570e308))) return true;
  const double nA = wave_max(cs);
  int si = 0;
  Blk<NN> U, V;
  if (nA <= 2.1) {
    const int deg = nA > 0.95 ? 9 : (nA > 0.25 ? 7 : (nA > 0.015 ? 5 : 3));
    const double* C = kPade[(deg - 3) / 2];
    Blk<NN> T;
    blk_mm<NN>(S0, S0, T, lane);                        // A2
    blk_st<NN>(S1, T, lane);
    {
      const double c0 = C[0], c1 = C[1], cu = C[3], cv = C[2];
#pragma unroll
      for (int x = 0; x < BS; ++x)
#pragma unroll
        for (int y = 0; y < BS; ++y) {
          const double id = blk_id<NN>(lane, x, y);
          U.v[x][y] = c1 * id + cu * T.v[x][y];
          V.v[x][y] = c0 * id + cv * T.v[x][y];
        }
    }
    wave_sync();
    for (int kk = 2; kk <= (deg - 1) / 2; ++kk) {       // P = P·A2
      Blk<NN> Pk;
      if (kk == 2) {
        blk_mm<NN>(S1, S1, Pk, lane);
      } else {
        blk_st<NN>(S2, T, lane);
        wave_sync();
        blk_mm<NN>(S2, S1, Pk, lane);
        wave_sync();                                     // S2 is read before the next store
      }
      const double cu = C[2 * kk + 1], cv = C[2 * kk];
#pragma unroll
      for (int x = 0; x < BS; ++x)
#pragma unroll
        for (int y = 0; y < BS; ++y) {
          T.v[x][y] = Pk.v[x][y];
          U.v[x][y] = U.v[x][y] + cu * Pk.v[x][y];
          V.v[x][y] = V.v[x][y] + cv * Pk.v[x][y];
        }
    }
    blk_st<NN>(S2, U, lane);                             // U = A·U
    wave_sync();
    blk_mm<NN>(S0, S2, U, lane);
  } else {
    // as many squarings as Julia's expm! takes (no cap: a capped scaling leaves ‖A/2^s‖ > 5.4, and
    // the Padé-13 result then differs from the reference's where a diverging chain is about to bail
    // out; ‖A‖₁ <= DBL_MAX bounds si by 1022)
    const double s = log2(nA / 5.4);
    si = (s > 0.0) ? (int)ceil(s) : 0;
    if (si > 0) {
      const double sc = ldexp(1.0, -si);
      for (int o = lane; o < NN * NN; o += 64) S0[o] *= sc;
      wave_sync();
    }
    constexpr double c[14] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
                              1187353796428800.0, 129060195264000.0, 10559470521600.0,
                              670442572800.0, 33522128640.0, 1323241920.0, 40840800.0, 960960.0,
                              16380.0, 182.0, 1.0};
    Blk<NN> A2, A4, A6, T;
    blk_mm<NN>(S0, S0, A2, lane);
    blk_st<NN>(S1, A2, lane);
    wave_sync();
    blk_mm<NN>(S1, S1, A4, lane);
    blk_st<NN>(S2, A4, lane);
    wave_sync();
    blk_mm<NN>(S1, S2, A6, lane);
    wave_sync();
#pragma unroll
    for (int x = 0; x < BS; ++x)
#pragma unroll
      for (int y = 0; y < BS; ++y)
        T.v[x][y] = c[13] * A6.v[x][y] + c[11] * A4.v[x][y] + c[9] * A2.v[x][y];
    blk_st<NN>(S1, A6, lane);
    blk_st<NN>(S2, T, lane);
    wave_sync();
    blk_mm<NN>(S1, S2, V, lane);                         // A6·inner
    wave_sync();
#pragma unroll
    for (int x = 0; x < BS; ++x)
#pragma unroll
      for (int y = 0; y < BS; ++y) {
        const double id = blk_id<NN>(lane, x, y);
        V.v[x][y] = V.v[x][y] + c[7] * A6.v[x][y] + c[5] * A4.v[x][y] + c[3] * A2.v[x][y] + c[1] * id;
        T.v[x][y] = c[12] * A6.v[x][y] + c[10] * A4.v[x][y] + c[8] * A2.v[x][y];
      }
    blk_st<NN>(S2, V, lane);
    wave_sync();
    blk_mm<NN>(S0, S2, U, lane);                         // U = A·(A6·inner + …)
    wave_sync();
    blk_st<NN>(S2, T, lane);
    wave_sync();
    blk_mm<NN>(S1, S2, V, lane);                         // V = A6·(…)
#pragma unroll
    for (int x = 0; x < BS; ++x)
#pragma unroll
      for (int y = 0; y < BS; ++y) {
        const double id = blk_id<NN>(lane, x, y);
        V.v[x][y] = V.v[x][y] + c[6] * A6.v[x][y] + c[4] * A4.v[x][y] + c[2] * A2.v[x][y] + c[0] * id;
      }
  }
  wave_sync();                                           // every operand read is done
  if (st && lane == 0) st[0] = (long long)__builtin_amdgcn_s_memtime();
  {
    Blk<NN> M;
#pragma unroll
    for (int x = 0; x < BS; ++x)
#pragma unroll
      for (int y = 0; y < BS; ++y) {
        M.v[x][y] = V.v[x][y] - U.v[x][y];
        U.v[x][y] = V.v[x][y] + U.v[x][y];
      }
    blk_st<NN>(S0, M, lane);
    blk_st<NN>(S1, U, lane);
  }
  wave_sync();
  bool solved = false;
  const int nc = si > 0 ? NN : ncols;
  if constexpr (2 * NN <= 64) solved = wave_solve_dd<NN>(S0, S1);
  else if constexpr (NN <= 64) solved = wv_solve_dd_passes<NN>(S0, S1, S2, lane, nc);
  if (!solved) wave_solve<NN>(S0, S1);
  if (st && lane == 0) st[1] = (long long)__builtin_amdgcn_s_memtime();
  for (int z = 0; z < si; ++z) {
    Blk<NN> P2;
    blk_mm<NN>(S1, S1, P2, lane);
    wave_sync();
    blk_st<NN>(S1, P2, lane);
    wave_sync();
  }
  bool bad = false;
#pragma unroll
  for (int o0 = 0; o0 < NN * NN; o0 += 64) {            // every read in flight at once
    const int o = o0 + lane;
    if (o < NN * NN) bad |= (o % NN < nc) && (S1[o] != S1[o]);
  }
  return __any(bad);
}

// dst[o] = src[o] for o < cnt (global -> LDS) by threads t of nth: UNR loads in flight per thread
// before their stores (a plain loop waits for every load before its store: one memory latency
// per 64 · nth doubles).
template <int UNR, class T>
__device__ __forceinline__ void copy_to_lds(T* dst, const T* src, int cnt, int t, int nth) {
  for (int o0 = 0; o0 < cnt; o0 += UNR * nth) {
    T v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int o = o0 + u * nth + t;
      v[u] = gptr(src)[o < cnt ? o : cnt - 1];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int o = o0 + u * nth + t;
      if (o < cnt) dst[o] = v[u];
    }
  }
}

// copy_to_lds of doubles as 16-B pairs when the count and both addresses allow (half the loads,
// half the memory round trips for the same UNR)
typedef double dpair __attribute__((ext_vector_type(2)));
template <int UNR>
__device__ __forceinline__ void copy_to_lds_d2(double* dst, const double* src, int cnt, int t,
                                               int nth) {
  if (((cnt | (int)((uintptr_t)src >> 3) | (int)((uintptr_t)dst >> 3)) & 1) == 0)
    copy_to_lds<UNR>((dpair*)dst, (const dpair*)src, cnt / 2, t, nth);
  else
    copy_to_lds<UNR>(dst, src, cnt, t, nth);
}

// Wave totals of NV per-lane values (exact-count butterfly) written to dst[0..NV).
template <int NV>
__device__ __forceinline__ void wv_sum_to_lds(double (&v)[NV], double* dst, int lane) {
  obf_run<NV, NV>(v, lane);
  int vi;
  bool wr;
  obf_index<NV>(lane, vi, wr);
  if (wr) dst[vi] = v[0];
}

// (chain, dimension) of workgroup x of the dimension launch: the D waves of chain c go to the
// XCD that runs chain c's V-phase workgroup (workgroups are dealt to the 8 XCDs round robin), so
// temp and coef cross an L2 only through the kernel boundary's write-back, never between XCDs.
__device__ __forceinline__ void wv_map(int x, int nchains, int D, int& c, int& k) {
  if ((nchains & 7) == 0) {
    const int xcd = x & 7, s = x >> 3;
    c = xcd + 8 * (s / D);
    k = s - (s / D) * D;
  } else {
    c = x / D;
    k = x - c * D;
  }
}

// LDS doubles of one dimension wave: three (2r)² operand slots for the geodesic's expm, or the
// staged U^(k) (n·r) plus coef_k / the r × r Grams when those need more.
GPT_HD int wv_dim_lds_dbl(int n, int r, int m) {
  const int slots = 12 * r * r;
  const int mp = (m + 7) / 8 * 8;                       // coef_k rows padded to the gradU row ring
  const int pre = n * r + (mp * r > 4 * r * r ? mp * r : 4 * r * r);
  return slots > pre ? slots : pre;
}

// The V-phase tables (16-bit, wave_tables): [q·D + k] = (k·r + I[q,k])·m, then the run members of
// every dimension (q with I[q,k] = l, q order, runs in l order), then the D·(r+1) run starts;
// padded to whole 16-B vectors.
GPT_HD int wv_table_shorts(int D, int r, int Q) { return (Q * D + D * Q + D * (r + 1) + 7) / 8 * 8; }

// The V-phase workgroup's LDS (doubles): temp of the batch, V (stride m|1), w, y, res, fhat
// partials, a reduction row and (16-B aligned) the tables.
GPT_HD int wv_vphase_tab_dbl(int D, int r, int Q, int m) {
  return (D * r * m + (Q + 1) * (m | 1) + Q + 1 + 2 * 64 + 8 * 64 + 8 + 1) & ~1;
}
GPT_HD int wv_vphase_lds_dbl(int D, int r, int Q, int m) {
  return wv_vphase_tab_dbl(D, r, Q, m) + wv_table_shorts(D, r, Q) / 4;
}

constexpr int kWvMaxM = 64;            // minibatch rows: one per lane of the V-phase

// U-noise columns per pass of the drive loop (independent Philox chains interleaved)
#ifndef WV_NOISE_UNR
#define WV_NOISE_UNR 4
#endif
#define WV_STR(x) #x
#define WV_UNROLL(n) _Pragma(WV_STR(unroll n))

// Phase stamps (gpt_sgld_session_stamps; s_memtime): dimension wave (c, k) in row c·(D+1) + k,
// the chain's V-phase workgroup in row c·(D+1) + D.
#define WSTAMP(row, slot)                                                                   \
  do {                                                                                      \
    if (P.stamps && lane == 0)                                                              \
      P.stamps[(size_t)(row) * kStamps + (slot)] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)

// ------------------------------------------------------------------------------ V-phase launch
template <int R>
__global__ __launch_bounds__(512) void wv_vphase_kernel(StepParams P,
                                                        const ChainDesc* __restrict__ chains,
                                                        const long long* __restrict__ tbase,
                                                        int t_local) {
  extern __shared__ __attribute__((aligned(16))) double wv_sm[];
  const ChainDesc* Cp = chains + blockIdx.x;
  const long long t = tbase[0] + t_local;
  if (t >= P.total_steps) return;
  if (__hip_atomic_load(Cp->status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = uni(tid >> 6);
  const int D = P.D, Q = P.Q, m = P.m, MV = m | 1;
  const int srow = (int)blockIdx.x * (D + 1) + D;
  if (wv == 0) WSTAMP(srow, 0);
  double* temp_l = wv_sm;                             // [(k·R + l)·m + i]
  double* V_l = temp_l + D * R * m;                   // [q·MV + i]; row Q = 0 (run padding)
  double* w_l = V_l + (Q + 1) * MV;                   // w_Q = 0
  double* y_l = w_l + Q + 1;
  double* res_l = y_l + 64;
  double* fpart = res_l + 64;                         // [wave·64 + i]
  double* red = fpart + 8 * 64;
  // 16-bit tables: [q·D + k] = (k·R + I[q,k])·m (< 2^16, wave_supported), the run members
  // (wave_tables), then the run starts
  unsigned short* toff_l = (unsigned short*)(wv_sm + wv_vphase_tab_dbl(D, R, Q, m));
  unsigned short* mem_l = toff_l + Q * D;
  unsigned short* seg_l = mem_l + D * Q;

  const int e = (int)(t / P.nb), b = (int)(t - (long long)e * P.nb);
  const int Bt = min(m, P.N - b * m);
  const int32_t* ord = Cp->order + (size_t)(e & 1) * P.N + (size_t)b * m;
  {
    const double* tsrc = Cp->temp + (size_t)(t & 1) * D * R * m;
    copy_to_lds_d2<8>(temp_l, tsrc, D * R * m, tid, 512);
    const double* wsrc = Cp->w + (size_t)(t & 1) * Q;
    for (int q = tid; q < Q; q += 512) w_l[q] = gptr(wsrc)[q];
    if (tid == 0) w_l[Q] = 0.0;
    for (int i = tid; i < MV; i += 512) V_l[Q * MV + i] = 0.0;
    if (tid < 64) y_l[tid] = tid < Bt ? gptr(Cp->y)[gptr(ord)[tid]] : 0.0;
    copy_to_lds<4>((long long*)toff_l, (const long long*)P.wvtab, wv_table_shorts(D, R, Q) / 4, tid,
                   512);
  }
  __syncthreads();
  if (wv == 0) WSTAMP(srow, 4);
  // V[q,i] = Π_k temp[k, I[q,k], i] in k order (computeV) and w_q·V partial sums of fhat:
  // lanes = batch rows, waves = slices of the core entries
  const int i = lane, ic = min(lane, Bt - 1);
  {
    // V[q, i] = Π_k temp[k, I[q,k], i] left to right (1.0 times the first factor is exact);
    // four q per pass with their stores after all reads, so the reads of one pass are in flight
    // together (a store in between would order every later read behind it)
    auto vq = [&](int q) {
      const unsigned short* to = toff_l + q * D;
      double x = 1.0;
      if (D == 8) {                                   // the 8 offsets of q in one 16-B read
        const uint4 o4 = *(const uint4*)to;
        const unsigned ow[4] = {o4.x, o4.y, o4.z, o4.w};
        double t8[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) t8[kk] = temp_l[((ow[kk >> 1] >> (16 * (kk & 1))) & 0xffffu) + ic];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) x *= t8[kk];
        return x;
      }
      for (int k0 = 0; k0 < D; k0 += 8) {
        double t8[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) t8[kk] = k0 + kk < D ? temp_l[to[k0 + kk] + ic] : 1.0;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) x *= t8[kk];
      }
      return x;
    };
    const int Qw = (Q + 7) / 8, qa = wv * Qw, qb = min(Q, qa + Qw);
    double f = 0.0;
    int q = qa;
    for (; q + 4 <= qb; q += 4) {
      double v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = vq(q + u);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (i < Bt) V_l[(q + u) * MV + i] = v[u];
        f = fma(w_l[q + u], v[u], f);
      }
    }
    for (; q < qb; ++q) {
      const double v = vq(q);
      if (i < Bt) V_l[q * MV + i] = v;
      f = fma(w_l[q], v, f);
    }
    fpart[wv * 64 + lane] = f;
  }
  __syncthreads();
  if (wv == 0) WSTAMP(srow, 1);
  if (tid < 64) {
    double fh = 0.0;
#pragma unroll
    for (int w2 = 0; w2 < 8; ++w2) fh += fpart[w2 * 64 + tid];
    res_l[tid] = tid < Bt ? y_l[tid] - fh : 0.0;
  }
  __syncthreads();
  const double cN = (double)P.N / (double)Bt;
  const long long post = t - P.burnin_steps;
  const bool store = post >= 0 && ((post + 1) % P.store_every) == 0;
  const long long slot = store ? (post + 1) / P.store_every - 1 : 0;
  {
    // gradw and the Langevin step on w (GPT_SGLD.jl:393, 411-414): threads over q
    const double sv = Cp->signal_var, sw = Cp->sigma_w, epsw = Cp->epsw;
    const double inv_sw2 = 1.0 / (sw * sw), sqe = sqrt(epsw);
    double gn2 = 0.0;
    for (int q = tid; q < Q; q += 512) {
      double g = 0.0;
      for (int ii = 0; ii < Bt; ++ii) g = fma(V_l[q * MV + ii], res_l[ii], g);
      const double wq = w_l[q];
      const double gradw = cN * g / sv - wq * inv_sw2;
      double step = epsw * gradw / 2;
      step += sqe * normal_at(Cp->seed, (uint32_t)q, (uint32_t)t, kWNoise, 0);
      const double wn = wq + step;
      gptr_w(Cp->w)[(size_t)((t + 1) & 1) * Q + q] = wn;
      if (store && Cp->w_store) gptr_w(Cp->w_store)[(size_t)slot * Q + q] = wn;
      gn2 = fma(gradw, gradw, gn2);
    }
    if (Cp->diag) {
      gn2 = wave_sum(gn2);
      if (lane == 0) red[wv] = gn2;
    }
  }
  if (wv == 0) WSTAMP(srow, 2);
  // coef[k][i][l] = A[l,k,i]·res_i, A = (Σ_{q: I[q,k]=l} w_q·V[q,i]) / temp[k,l,i] (computeU_phi +
  // computeA with the old w, :396-399): waves over (k, l), lanes = rows, members in q order
  {
    double* cf = Cp->coef;
    for (int p = wv; p < D * R; p += 8) {
      const int k = p / R, l = p - k * R;
      const int s0 = seg_l[k * (R + 1) + l], s1 = seg_l[k * (R + 1) + l + 1];
      const unsigned short* mk = mem_l + k * Q;
      double a = 0.0;
      for (int s = s0; s < s1; s += 4) {               // members 4 at a time (past the run: q = Q,
        int q4[4];                                      // a zero row and a zero weight)
#pragma unroll
        for (int u = 0; u < 4; ++u) q4[u] = s + u < s1 ? mk[s + u] : Q;
        double wv4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) wv4[u] = w_l[q4[u]] * V_l[q4[u] * MV + ic];
#pragma unroll
        for (int u = 0; u < 4; ++u) a += wv4[u];
      }
      const double cval = (a * rcp_nr(temp_l[p * m + ic])) * res_l[ic];
      if (i < Bt) gptr_w(cf)[((size_t)k * m + i) * R + l] = cval;
    }
  }
  if (wv == 0) WSTAMP(srow, 3);
  if (Cp->diag) {
    __syncthreads();
    if (tid == 0) {
      double s = 0.0;
      for (int w2 = 0; w2 < 8; ++w2) s += red[w2];
      Cp->diag[(size_t)t * (1 + D)] = sqrt(s);
    }
  }
}

// ---------------------------------------------------------------------------- dimension launch
// init != 0: only temp of the batch of step t with the stored U (the first step of a run).
typedef double pd4 __attribute__((ext_vector_type(4)));
typedef double pd2 __attribute__((ext_vector_type(2)));
// the dimension wave's U^(k) staging slot (column-major, stride n) at the start of its LDS
__device__ __forceinline__ double* U_lds_base(double* sm) { return sm; }

template <int R, int J>
__global__ __launch_bounds__(64, 1) void wv_dim_kernel(StepParams P,
                                                       const ChainDesc* __restrict__ chains,
                                                       const long long* __restrict__ tbase,
                                                       int t_local, int nchains, int init) {
  extern __shared__ __attribute__((aligned(16))) double wv_sm[];
  constexpr int NN = 2 * R, SL = NN * NN, PF = 8;       // PF: batch rows in flight
  int c, k;
  wv_map(blockIdx.x, nchains, P.D, c, k);
  const ChainDesc* Cp = chains + c;
  const long long t = tbase[0] + t_local;
  if (t >= P.total_steps) return;
  if (__hip_atomic_load(Cp->status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  const int lane = lane_id();
  const int n = P.n, D = P.D, m = P.m;
  const int srow = c * (D + 1) + k;
  WSTAMP(srow, 0);
  const size_t rstride = (size_t)n * D;
  const double* phik = Cp->phi + (size_t)n * k;
  double* Ug = Cp->U + (size_t)n * R * k;
  int jc[J];
  bool jok[J];
#pragma unroll
  for (int jj = 0; jj < J; ++jj) {
    jc[jj] = min(lane + 64 * jj, n - 1);
    jok[jj] = lane + 64 * jj < n;
  }
  double u[J][R];                                       // U^(k) rows of this lane

  // phidotU (GPT_SGLD.jl:193-205) of the Bn rows at ordn into temp slot tdst: two rows at a time,
  // 2R partial dots per lane reduced by one exact-count butterfly (the two rows' exchanges
  // interleave); PF rows' loads in flight
  auto phidotU = [&](const int32_t* ordn, int Bn, double* tdst) {
    const int myrow = gptr(ordn)[min(lane, Bn - 1)];
    const RowPtr rp(phik, myrow, (long long)rstride);
    double ring[PF][J];
#pragma unroll
    for (int x = 0; x < PF; ++x)
#pragma unroll
      for (int jj = 0; jj < J; ++jj) ring[x][jj] = rp.at(min(x, Bn - 1))[jc[jj]];
    for (int i0 = 0; i0 < Bn; i0 += PF) {
#pragma unroll
      for (int x = 0; x < PF; x += 2) {
        double p[2][J];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int jj = 0; jj < J; ++jj) p[h][jj] = ring[x + h][jj];
          const int inext = min(i0 + x + h + PF, Bn - 1);
#pragma unroll
          for (int jj = 0; jj < J; ++jj) ring[x + h][jj] = rp.at(inext)[jc[jj]];
        }
        if (i0 + x < Bn) {
          double v[2 * R];
#pragma unroll
          for (int l = 0; l < 2 * R; ++l) v[l] = 0.0;
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int jj = 0; jj < J; ++jj)
#pragma unroll
              for (int l = 0; l < R; ++l) v[h * R + l] = fma(p[h][jj], u[jj][l], v[h * R + l]);
          obf_run<2 * R, 2 * R>(v, lane);
          int vi;
          bool wr;
          obf_index<2 * R>(lane, vi, wr);
          const int h = vi >= R ? 1 : 0, l = vi - h * R;
          if (wr && i0 + x + h < Bn) gptr_w(tdst)[((size_t)k * R + l) * m + i0 + x + h] = v[0];
        }
      }
    }
  };

  // phidotU on the fp64 matrix cores (n even): temp[k][l][i] = Σ_j U[j][l]·φ[row_i][k][j] as
  // ⌈R/16⌉ × 4 tiles of v_mfma_f64_16x16x4f64 (M = l, N = the ≤ 64 batch rows, K = j); A = Uᵀ from
  // U^(k) staged in LDS (column-major, stride n), B = φ rows straight from memory.  Lane λ feeds
  // the K pair j0 + 2(λ>>4) + {0,1} of row / column λ&15 as one 16-B read, the halves to two
  // MFMAs (as pred_temp_mfma_kernel); columns l >= R and rows i >= Bn read clamped addresses and
  // only feed outputs that are never stored, the K tail j >= n is zeroed on the A side.
  constexpr int TT = (R + 15) / 16;
  auto phidotU_mfma = [&](const int32_t* ordn, int Bn, double* tdst) {
    const int kl = lane >> 4, c16 = lane & 15;
    const double* pa[TT];
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) pa[tt] = U_lds_base(wv_sm) + (size_t)n * min(16 * tt + c16, R - 1);
    const __attribute__((address_space(1))) double* pb[4];
#pragma unroll
    for (int uu = 0; uu < 4; ++uu)
      pb[uu] = gptr(phik + (size_t)gptr(ordn)[min(16 * uu + c16, Bn - 1)] * rstride);
    struct Ops { pd2 a[TT], b[4]; };
    auto load = [&](int j, Ops& o) {
      const int jj = min(j, n - 2);
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) {
        const pd2 v = *(const pd2*)(pa[tt] + jj);
        o.a[tt] = pd2{j < n ? v[0] : 0.0, j + 1 < n ? v[1] : 0.0};
      }
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) o.b[uu] = *(const __attribute__((address_space(1))) pd2*)(pb[uu] + jj);
    };
    pd4 acc[TT][4];
#pragma unroll
    for (int tt = 0; tt < TT; ++tt)
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) acc[tt][uu] = pd4{0.0, 0.0, 0.0, 0.0};
    auto mma = [&](const Ops& o) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int tt = 0; tt < TT; ++tt)
#pragma unroll
          for (int uu = 0; uu < 4; ++uu)
            acc[tt][uu] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.a[tt][h], o.b[uu][h], acc[tt][uu], 0, 0, 0);
    };
    // K chunks of 8 through a ring of 4 operand sets (three chunks' loads in flight under each
    // chunk's MFMAs); the chunk count is rounded up to the ring (chunks past n have zero A), so
    // the loop has no branch that would make the compiler wait for every outstanding load
    constexpr int NB = 4;
    Ops ring[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) load(8 * q + 2 * kl, ring[q]);
    const int nch = ((n + 7) / 8 + NB - 1) / NB * NB;
    for (int c0 = 0; c0 < nch; c0 += NB) {
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        mma(ring[q]);
        load(8 * (c0 + q + NB) + 2 * kl, ring[q]);
      }
    }
    // D[row = kl + 4·reg][col = c16]: row ↔ l, col ↔ batch row
#pragma unroll
    for (int tt = 0; tt < TT; ++tt)
#pragma unroll
      for (int uu = 0; uu < 4; ++uu)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int l = 16 * tt + kl + 4 * reg, i = 16 * uu + c16;
          if (l < R && i < Bn) gptr_w(tdst)[((size_t)k * R + l) * m + i] = acc[tt][uu][reg];
        }
  };
  // U^(k) rows of the lane's registers into the LDS staging slot (column-major, stride n)
  auto u_to_lds = [&]() {
    double* Ul = U_lds_base(wv_sm);
#pragma unroll
    for (int jj = 0; jj < J; ++jj)
      if (jok[jj]) {
#pragma unroll
        for (int l = 0; l < R; ++l) Ul[jc[jj] + (size_t)n * l] = u[jj][l];
      }
    wave_sync();
  };

  const int e = (int)(t / P.nb), bb = (int)(t - (long long)e * P.nb);
  const int Bt = min(m, P.N - bb * m);
  const int32_t* ord = Cp->order + (size_t)(e & 1) * P.N + (size_t)bb * m;
  if (init) {
#pragma unroll
    for (int jj = 0; jj < J; ++jj)
#pragma unroll
      for (int l = 0; l < R; ++l) u[jj][l] = jok[jj] ? gptr(Ug)[jc[jj] + (size_t)n * l] : 0.0;
    if ((n & 1) == 0) {
      u_to_lds();
      phidotU_mfma(ord, Bt, Cp->temp + (size_t)(t & 1) * D * R * m);
    } else {
      phidotU(ord, Bt, Cp->temp + (size_t)(t & 1) * D * R * m);
    }
    return;
  }
  WSTAMP(srow, 1);

  // ---- stage U^(k) (column-major, stride n) and coef_k (row i: R values) in LDS
  double* U_l = wv_sm;
  double* cf_l = U_l + n * R;
  double* sctab = wv_sm + wv_dim_lds_dbl(n, R, m);
  sincos_tab_fill(sctab, lane, 64);
  copy_to_lds_d2<12>(U_l, Ug, n * R, lane, 64);
  copy_to_lds_d2<8>(cf_l, Cp->coef + (size_t)k * m * R, Bt * R, lane, 64);
  for (int o = Bt * R + lane; o < (Bt + PF - 1) / PF * PF * R; o += 64) cf_l[o] = 0.0;
  wave_sync();

  // ---- gradU^(k) = (N/B)/σ² Σ_i φ[:,k,i]·coef[k][i][:]  (GPT_SGLD.jl:396-408)
  double g[J][R];
#pragma unroll
  for (int jj = 0; jj < J; ++jj)
#pragma unroll
    for (int l = 0; l < R; ++l) g[jj][l] = 0.0;
  {
    const int myrow = gptr(ord)[min(lane, Bt - 1)];
    const RowPtr rp(phik, myrow, (long long)rstride);
    double ring[PF][J];
#pragma unroll
    for (int x = 0; x < PF; ++x)
#pragma unroll
      for (int jj = 0; jj < J; ++jj) ring[x][jj] = rp.at(min(x, Bt - 1))[jc[jj]];
    for (int i0 = 0; i0 < Bt; i0 += PF) {
#pragma unroll
      for (int x = 0; x < PF; ++x) {
        double p[J];
#pragma unroll
        for (int jj = 0; jj < J; ++jj) p[jj] = ring[x][jj];
        const int inext = min(i0 + x + PF, Bt - 1);
#pragma unroll
        for (int jj = 0; jj < J; ++jj) ring[x][jj] = rp.at(inext)[jc[jj]];
        {
          // no per-row branch (coef rows past Bt are zero: +0 added to each sum, exact), so the
          // row ring's loads stay in flight across rows (a branch made the compiler wait for
          // every outstanding load); the row's R coefficients are read together, waited for once
          const double* ci = cf_l + (i0 + x) * R;
          double c[R];
#pragma unroll
          for (int l = 0; l < R; ++l) c[l] = ci[l];
#pragma unroll
          for (int l = 0; l < R; ++l) asm volatile("" : "+v"(c[l]));
#pragma unroll
          for (int l = 0; l < R; ++l)
#pragma unroll
            for (int jj = 0; jj < J; ++jj) g[jj][l] = fma(p[jj], c[l], g[jj][l]);
        }
      }
    }
  }
  WSTAMP(srow, 2);
  const double cN = (double)P.N / (double)Bt;
  const double cU = cN / Cp->signal_var;
  const double sq = sqrt(Cp->epsU);
  // ---- Langevin drive √εU/2·gradU + ζ (:420), ζ on the U-noise quad contract (gpt_common.h)
  {
    double gu2 = 0.0;
    constexpr int NQJ = (J + 3) / 4;
    const int NQ = unoise_nq(n);
    const uint64_t seed = Cp->seed;
    WV_UNROLL(WV_NOISE_UNR)
    for (int l = 0; l < R; ++l) {
#pragma unroll
      for (int q = 0; q < NQJ; ++q) {
        double z[4];
        normal_quad_tab<4>(seed, (uint32_t)((l * NQ + q) * 64 + lane), (uint32_t)t, kUNoise,
                           (uint32_t)k, sctab, z);
#pragma unroll
        for (int L = 0; L < R; ++L) {
          if (l == L) {
#pragma unroll
            for (int i2 = 0; i2 < 4; ++i2) {
              const int jj = 4 * q + i2;
              if (jj < J) {
                const double Gv = jok[jj] ? g[jj][L] * cU : 0.0;
                gu2 = fma(Gv, Gv, gu2);
                g[jj][L] = jok[jj] ? sq * Gv / 2 + z[i2] : 0.0;
              }
            }
          }
        }
      }
    }
    if (Cp->diag) {
      gu2 = wave_sum(gu2);
      if (lane == 0) Cp->diag[(size_t)t * (1 + D) + 1 + k] = sqrt(gu2);
    }
  }
  WSTAMP(srow, 3);
  // ---- proj (:14-16): M = UᵀW, mom = W − U·(M + Mᵀ)/2; geod Grams A = (M − Mᵀ)/2 (UᵀU = I),
  //      S = momᵀmom (:19-22)
  double* Mg = cf_l;                                     // coef_k is consumed
  double* Ms = Mg + R * R;
  double* Sg = Ms + R * R;
  double* Ag = Sg + R * R;
#pragma unroll 1
  for (int a = 0; a < R; ++a) {
    double ua[J];
#pragma unroll
    for (int jj = 0; jj < J; ++jj) ua[jj] = jok[jj] ? U_l[jc[jj] + n * a] : 0.0;
    double v[R];
#pragma unroll
    for (int b2 = 0; b2 < R; ++b2) {
      double s = 0.0;
#pragma unroll
      for (int jj = 0; jj < J; ++jj) s = fma(ua[jj], g[jj][b2], s);
      v[b2] = s;
    }
    wv_sum_to_lds<R>(v, Mg + a * R, lane);
  }
  wave_sync();
  for (int o = lane; o < R * R; o += 64) {
    const int a = o / R, b2 = o - a * R;
    Ms[o] = Mg[o] + Mg[b2 * R + a];
  }
  wave_sync();
  WSTAMP(srow, 4);
#pragma unroll
  for (int jj = 0; jj < J; ++jj) {
    double s[R];
#pragma unroll
    for (int b2 = 0; b2 < R; ++b2) s[b2] = 0.0;
#pragma unroll 2
    for (int a = 0; a < R; ++a) {
      const double ua = jok[jj] ? U_l[jc[jj] + n * a] : 0.0;
#pragma unroll
      for (int b2 = 0; b2 < R; ++b2) s[b2] = fma(ua, Ms[a * R + b2], s[b2]);
    }
#pragma unroll
    for (int b2 = 0; b2 < R; ++b2) g[jj][b2] = g[jj][b2] - s[b2] / 2;
  }
  // S[a][b] for b >= a, rows a and R−1−a in one exact-count butterfly of R + 1 values (static a:
  // g stays in registers — g[jj][a] with a runtime a put the whole drive in scratch memory)
#pragma unroll
  for (int p = 0; p < (R + 1) / 2; ++p) {
    const int a1 = p, a2 = R - 1 - p, n1 = R - a1;
    const bool two = a2 > a1;
    double v[R + 1];
#pragma unroll
    for (int x = 0; x < R + 1; ++x) {
      const int a = x < n1 ? a1 : a2, b2 = x < n1 ? a1 + x : a2 + (x - n1);
      double s1 = 0.0;
      if (x < n1 || (two && b2 < R)) {
#pragma unroll
        for (int jj = 0; jj < J; ++jj) s1 = fma(g[jj][a], g[jj][b2], s1);
      }
      v[x] = s1;
    }
    obf_run<R + 1, R + 1>(v, lane);
    int vi;
    bool wr;
    obf_index<R + 1>(lane, vi, wr);
    if (wr) {
      if (vi < n1) Sg[a1 * R + a1 + vi] = v[0];
      else if (two && a2 + (vi - n1) < R) Sg[a2 * R + a2 + (vi - n1)] = v[0];
    }
  }
  wave_sync();
  for (int o = lane; o < R * R; o += 64) {
    const int i2 = o / R, b2 = o - i2 * R;
    Ag[o] = (Mg[o] - Mg[b2 * R + i2]) / 2;
    if (i2 > b2) Sg[o] = Sg[b2 * R + i2];
  }
  WSTAMP(srow, 5);
  // mom leaves the registers for the expm (the chain's park area, column-major like U)
  double* park = Cp->park + (size_t)n * R * k;
#pragma unroll
  for (int jj = 0; jj < J; ++jj)
    if (jok[jj]) {
#pragma unroll
      for (int l = 0; l < R; ++l) gptr_w(park)[jc[jj] + (size_t)n * l] = g[jj][l];
    }
  wave_sync();
  // ---- geod (:19-37): expm(−tA) first (its r × r scratch below Mg), kept in registers across
  //      the 2r × 2r expm of t·[A −S; I A], which takes all three slots
  double* S0 = wv_sm;
  double* S1 = S0 + SL;
  double* S2 = S1 + SL;
  const double tt = sq;
  bool bad;
  constexpr int MXL = (R * R + 63) / 64;
  double mxr[MXL];
  {
    double* X1 = wv_sm;                                  // 3 r² doubles, below Mg (n >= 3r)
    double* X1b = X1 + R * R;
    double* X1c = X1b + R * R;
    for (int o = lane; o < R * R; o += 64) X1[o] = -tt * Ag[o];
    wave_sync();
    WSTAMP(srow, 6);
    wv_expm<R>(X1, X1b, X1c, lane, P.stamps ? P.stamps + (size_t)srow * kStamps + 14 : nullptr);
    WSTAMP(srow, 7);
#pragma unroll
    for (int x = 0; x < MXL; ++x) mxr[x] = X1b[min(lane + 64 * x, R * R - 1)];
    wave_sync();                                         // X1b is read before slot 0 covers it
    // X0 = t·[A −S; I A] into slot 0 (Ag / Sg sit past slot 0: n >= 3r, wave_supported)
    for (int o = lane; o < NN * NN; o += 64) {
      const int i2 = o / NN, j2 = o - i2 * NN;
      double v;
      if (i2 < R) v = j2 < R ? Ag[i2 * R + j2] : -Sg[i2 * R + (j2 - R)];
      else v = j2 < R ? (i2 - R == j2 ? 1.0 : 0.0) : Ag[(i2 - R) * R + (j2 - R)];
      S0[o] = tt * v;
    }
    wave_sync();
    bad = wv_expm<NN>(S0, S1, S2, lane, P.stamps ? P.stamps + (size_t)srow * kStamps + 12 : nullptr,
                      R);
  }
  WSTAMP(srow, 8);
  // F = E[:, 1:r]·expm(−tA) (2r × r) into slot 0; expm(−tA) back to LDS at slot 2
  double* mx = S2;
  double* F = S0;
#pragma unroll
  for (int x = 0; x < MXL; ++x)
    if (lane + 64 * x < R * R) mx[lane + 64 * x] = mxr[x];
  wave_sync();
  // one row of F per lane (a = lane < 2r): R independent fma chains, each over c2 in order (the
  // same doubles as one output per lane and pass); the expm(−tA) rows are wave-uniform reads
  if (lane < NN) {
    const int a = lane;
    double acc[R];
#pragma unroll
    for (int l = 0; l < R; ++l) acc[l] = 0.0;
#pragma unroll 2
    for (int c2 = 0; c2 < R; ++c2) {
      const double e = S1[a * NN + c2];
#pragma unroll
      for (int l = 0; l < R; ++l) acc[l] = fma(e, mx[c2 * R + l], acc[l]);
    }
#pragma unroll
    for (int l = 0; l < R; ++l) F[a * R + l] = acc[l];
  }
  wave_sync();
  if (bad) {                                             // NaN in the geodesic (:422-424)
    if (lane == 0) __hip_atomic_store(Cp->status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  WSTAMP(srow, 9);
  // ---- tmpU = [U mom]·F row by row (:35 with the two products associated the other way), then
  //      the column normalisation
  // (a outer: each F row is read from LDS once for the J rows of the lane; the [U mom] values
  // of four a at a time are in flight)
#pragma unroll
  for (int jj = 0; jj < J; ++jj)
#pragma unroll
    for (int l = 0; l < R; ++l) u[jj][l] = 0.0;
#pragma unroll
  for (int a0 = 0; a0 < 2 * R; a0 += 4) {
    double x[4][J];
#pragma unroll
    for (int da = 0; da < 4; ++da)
#pragma unroll
      for (int jj = 0; jj < J; ++jj) {
        const int a = a0 + da;
        const double* src = a < R ? Ug + (size_t)n * a : park + (size_t)n * (a - R);
        x[da][jj] = a < 2 * R ? gptr(src)[jc[jj]] : 0.0;
      }
#pragma unroll
    for (int da = 0; da < 4; ++da) {
      const int a = a0 + da;
      if (a < 2 * R) {
        double f[R];
#pragma unroll
        for (int l = 0; l < R; ++l) f[l] = F[a * R + l];
#pragma unroll
        for (int jj = 0; jj < J; ++jj) {
          const double xa = jok[jj] ? x[da][jj] : 0.0;
#pragma unroll
          for (int l = 0; l < R; ++l) u[jj][l] = fma(xa, f[l], u[jj][l]);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  double nrm[R];
#pragma unroll
  for (int l = 0; l < R; ++l) {
    nrm[l] = 0.0;
#pragma unroll
    for (int jj = 0; jj < J; ++jj) nrm[l] = fma(u[jj][l], u[jj][l], nrm[l]);
  }
  double* nr = S2 + R * R;
  wv_sum_to_lds<R>(nrm, nr, lane);
  wave_sync();
#pragma unroll
  for (int l = 0; l < R; ++l) {
    const double isc = 1.0 / sqrt(nr[l]);
#pragma unroll
    for (int jj = 0; jj < J; ++jj) u[jj][l] = u[jj][l] * isc;
  }
  // ---- U^(k) and its sample store (GPT_SGLD.jl:441-444)
  {
    const long long post = t - P.burnin_steps;
    const bool store = post >= 0 && ((post + 1) % P.store_every) == 0;
    const long long slot = store ? (post + 1) / P.store_every - 1 : 0;
    double* Us = (store && Cp->U_store) ? Cp->U_store + ((size_t)slot * D + k) * n * R : nullptr;
#pragma unroll
    for (int jj = 0; jj < J; ++jj)
      if (jok[jj]) {
#pragma unroll
        for (int l = 0; l < R; ++l) {
          gptr_w(Ug)[jc[jj] + (size_t)n * l] = u[jj][l];
          if (Us) gptr_w(Us)[jc[jj] + (size_t)n * l] = u[jj][l];
        }
      }
  }
  WSTAMP(srow, 10);
  // ---- temp[k] of the next batch with the new U^(k)
  const long long t1 = t + 1;
  if (t1 < P.total_steps) {
    const int e1 = (int)(t1 / P.nb), b1 = (int)(t1 - (long long)e1 * P.nb);
    const int B1 = min(m, P.N - b1 * m);
    const int32_t* ord1 = Cp->order + (size_t)(e1 & 1) * P.N + (size_t)b1 * m;
    double* tdst = Cp->temp + (size_t)(t1 & 1) * D * R * m;
    if ((n & 1) == 0) {
      wave_sync();                                       // every read of the slot is done
      u_to_lds();
      phidotU_mfma(ord1, B1, tdst);
    } else {
      phidotU(ord1, B1, tdst);
    }
  }
  WSTAMP(srow, 11);
}

// ------------------------------------------------------------------------------------ host side
#define GPT_WV_CFGS(X) X(6) X(8) X(10) X(12) X(15) X(16) X(20)

static int wv_J(int n) { return n <= 64 ? 1 : (n <= 128 ? 2 : (n <= 192 ? 3 : (n <= 256 ? 4 : 0))); }

// + the U noise's two 16-entry (sin, cos) tables (fm_sincos_tab2) past everything else
size_t wv_dim_lds_bytes(int n, int r, int m) { return 8 * ((size_t)wv_dim_lds_dbl(n, r, m) + 64); }
size_t wv_vphase_lds_bytes(int D, int r, int Q, int m) {
  return 8 * (size_t)wv_vphase_lds_dbl(D, r, Q, m);
}

bool wave_supported(int n, int D, int r, int Q, int m, bool langevin, bool stiefel) {
  if (!langevin || !stiefel) return false;        // SGD / Euclidean variants: grid engine
  bool inst = false;
#define CASE(RR) inst |= (r == RR);
  GPT_WV_CFGS(CASE)
#undef CASE
  if (!inst || wv_J(n) == 0 || m > kWvMaxM || D < 1 || D > kDMax) return false;
  if (3 * r * r > n * r) return false;            // expm(−tA)'s scratch below the Grams
  if ((long long)D * r * m >= 65536 || Q >= 65536) return false;   // 16-bit V-phase tables
  return wv_vphase_lds_bytes(D, r, Q, m) <= 160 * 1024 && wv_dim_lds_bytes(n, r, m) <= 160 * 1024;
}

// D·Q members of every run (core entries q with I[q,k] = l, in q order, runs in l order), then
// the D·(r+1) run starts.
void wave_tables(const std::vector<int32_t>& I0, int Q, int D, int r, int m,
                 std::vector<uint16_t>& out) {
  out.assign((size_t)wv_table_shorts(D, r, Q), 0);
  for (int q = 0; q < Q; ++q)
    for (int k = 0; k < D; ++k)
      out[(size_t)q * D + k] = (uint16_t)((k * r + I0[q + (size_t)Q * k]) * m);
  uint16_t* mem = out.data() + (size_t)Q * D;
  for (int k = 0; k < D; ++k) {
    int pos = 0;
    uint16_t* seg = mem + (size_t)D * Q + (size_t)k * (r + 1);
    for (int l = 0; l < r; ++l) {
      seg[l] = (uint16_t)pos;
      for (int q = 0; q < Q; ++q)
        if (I0[q + (size_t)Q * k] == l) mem[(size_t)k * Q + pos++] = (uint16_t)q;
    }
    seg[r] = (uint16_t)pos;
  }
}

hipError_t launch_wave(const StepParams& P, const ChainDesc* chains, int nchains,
                       const long long* tbase, int t_local, bool init, hipStream_t st) {
  const int J = wv_J(P.n);
  const size_t ldsv = wv_vphase_lds_bytes(P.D, P.r, P.Q, P.m);
  const size_t ldsd = wv_dim_lds_bytes(P.n, P.r, P.m);
#define CASE_J(RR, JJ)                                                                        \
  if (J == JJ) {                                                                              \
    static std::atomic<uint64_t> attr{0};                                                     \
    hipError_t e = set_max_lds_once((const void*)wv_dim_kernel<RR, JJ>, 160 * 1024, attr);    \
    if (e != hipSuccess) return e;                                                            \
    hipLaunchKernelGGL((wv_dim_kernel<RR, JJ>), dim3(nchains * P.D), dim3(64), ldsd, st, P,   \
                       chains, tbase, t_local, nchains, init ? 1 : 0);                        \
    return hipGetLastError();                                                                 \
  }
#define CASE(RR)                                                                              \
  if (P.r == RR) {                                                                            \
    if (!init) {                                                                              \
      static std::atomic<uint64_t> attr{0};                                                   \
      hipError_t e = set_max_lds_once((const void*)wv_vphase_kernel<RR>, 160 * 1024, attr);   \
      if (e != hipSuccess) return e;                                                          \
      hipLaunchKernelGGL((wv_vphase_kernel<RR>), dim3(nchains), dim3(512), ldsv, st, P,       \
                         chains, tbase, t_local);                                             \
      e = hipGetLastError();                                                                  \
      if (e != hipSuccess) return e;                                                          \
    }                                                                                         \
    CASE_J(RR, 1) CASE_J(RR, 2) CASE_J(RR, 3) CASE_J(RR, 4)                                   \
    return hipErrorInvalidValue;                                                              \
  }
  GPT_WV_CFGS(CASE)
#undef CASE
#undef CASE_J
  return hipErrorInvalidValue;
}

}  // namespace gpt

// ------------------------------------------------------------------------ expm unit check (tests)
namespace gpt {
// One wave per matrix: wv_expm (mode 0) or the grid engine's wave_expm (mode 1) of an NN × NN
// row-major matrix; NaN flags in bad.  Mode 2 (timing, gpt_debug_expm_stamps): wv_expm as geod
// calls it (three slots, the first NN/2 result columns) with s_memtime stamps per matrix in
// st[4·m + 0..3]: entry, polynomial done, solve done, exit.
template <int NN>
__global__ __launch_bounds__(64) void wv_expm_check_kernel(const double* A, double* E, int32_t* bad,
                                                           int mode, long long* st) {
  extern __shared__ __attribute__((aligned(16))) double wv_sm[];
  const int lane = lane_id();
  const double* a = A + (size_t)blockIdx.x * NN * NN;
  double* S0 = wv_sm;
  for (int o = lane; o < NN * NN; o += 64) S0[o] = a[o];
  wave_sync();
  bool b;
  const double* res;
  long long* sm = st ? st + 4 * (size_t)blockIdx.x : nullptr;
  if (sm && lane == 0) sm[0] = (long long)__builtin_amdgcn_s_memtime();
  if (mode == 2) {
    b = wv_expm<NN>(S0, S0 + NN * NN, S0 + 2 * NN * NN, lane, sm ? sm + 1 : nullptr, NN / 2);
    if (sm && lane == 0) sm[3] = (long long)__builtin_amdgcn_s_memtime();
    res = S0 + NN * NN;
  } else if (mode == 0) {
    b = wv_expm<NN>(S0, S0 + NN * NN, S0 + 2 * NN * NN, lane);
    res = S0 + NN * NN;
  } else {
    b = wave_expm<NN>(S0);
    res = S0 + NN * NN;
  }
  wave_sync();
  for (int o = lane; o < NN * NN; o += 64) E[(size_t)blockIdx.x * NN * NN + o] = res[o];
  if (lane == 0) bad[blockIdx.x] = b ? 1 : 0;
}

hipError_t launch_expm_check(int nn, int count, const double* A, double* E, int32_t* bad, int mode,
                             hipStream_t st, long long* stamps) {
#define CASE(NNV)                                                                               \
  if (nn == NNV) {                                                                              \
    const size_t lds = 8 * (size_t)(mode == 2 ? 3 : 7) * NNV * NNV;                             \
    hipError_t e = hipFuncSetAttribute((const void*)wv_expm_check_kernel<NNV>,                 \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
    if (e != hipSuccess) return e;                                                              \
    hipLaunchKernelGGL(wv_expm_check_kernel<NNV>, dim3(count), dim3(64), lds, st, A, E, bad,    \
                       mode, stamps);                                                           \
    return hipGetLastError();                                                                   \
  }
  CASE(12) CASE(16) CASE(20) CASE(24) CASE(30) CASE(32) CASE(40)
#undef CASE
  return hipErrorInvalidValue;
}
}  // namespace gpt
