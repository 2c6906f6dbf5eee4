// Fused tensor-GP SGLD step for MI355X (gfx950).
//
// One launch = one SGLD step (GPT_SGLD.jl:377-445) of every chain.  Grid (D+1, chains):
//   block k < D : owns U^(k) (n×r, in LDS).  Recomputes V/fhat/residual (cheap, identical in
//                 every block), forms A[:,k,:] without the division of computeU_phi, streams
//                 phi[:,k,batch] once for gradU^(k) (Psi is never materialised), does the
//                 Stiefel projection + geodesic (two Padé expm on two waves), writes U^(k),
//                 and — fused — streams phi[:,k,next batch] to produce temp[k,:,:] of the NEXT
//                 step with the new U^(k).
//   block D     : owns w: gradw from V and the residual, the Langevin update and w_store.
// The only grid-wide dependency of a step (every block needs temp of all k) is carried by the
// kernel boundary; temp/w are ping-ponged by step parity.  The host captures an epoch of
// launches in a hipGraph.
#include "device_util.h"

namespace gpt {

// Diagnostic phase stamps (only when P.stamps != nullptr): thread 0 records s_memtime after
// the workgroup barrier that closes a phase.
#define STAMP(slot)                                                                        \
  do {                                                                                     \
    if (P.stamps && tid == 0)                                                              \
      P.stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * kStamps + (slot)] =         \
          (long long)__builtin_amdgcn_s_memtime();                                         \
  } while (0)

#ifndef GPT_TOUCH
#define GPT_TOUCH 1       // L2 touch of the next batch's rows during the V-phase
#endif
#ifndef VPHASE_COLS
#define VPHASE_COLS 1     // the column-lane V-phase (vphase_cols) where the LDS has its scratch
#endif
#ifndef GPT_VHALF
#define GPT_VHALF 1         // vphase_cols_half for batches / slices of <= 32 columns
#endif
#ifndef GPT_EXP_P2NOCOEF
#define GPT_EXP_P2NOCOEF 0   // diagnostics only (wrong results): P2 without its coefficient reads
#endif
#ifndef GPT_EXP_P2NOLOAD
#define GPT_EXP_P2NOLOAD 0   // diagnostics only (wrong results): P2 without its row loads
#endif
constexpr int kTouch = 4;   // row pairs per wave: 2·kNW·kTouch = 64 rows >= the minibatch

template <int R>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(GPT_WPE))) void sgld_step_kernel(StepParams P,
                                                        const ChainDesc* __restrict__ chains,
                                                        const long long* __restrict__ tbase,
                                                        int t_local, int kbase) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const ChainDesc C = chains[blockIdx.y];
  // kbase = D: the RMSprop w phase (one workgroup); kbase = D + 1: the class-fhat pass of
  // GPTclassification (one workgroup per class, before the step launch).
  const int k = (int)blockIdx.x + kbase;
  const int tid = threadIdx.x, wv = uni(tid >> 6);
  const long long t = tbase[0] + t_local;
  if (t >= P.total_steps) return;
  if (__hip_atomic_load(C.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;

  const int n = P.n, D = P.D, Q = P.Q, m = P.m;
  const StepLayout L = step_layout(n, D, R, Q, m);
  const int MP = L.MP, NP = L.NP, NS = L.NS;
  const bool vcols = VPHASE_COLS && P.vtab && k <= D;   // not the class-fhat pass (k = D + 1)
  int* IT_l = (int*)(smem + L.o_I);            // I transposed: kk*Q + q
  double* w_l = (double*)(smem + L.o_w);
  int* idx_l = (int*)(smem + L.o_idx);
  double* y_l = (double*)(smem + L.o_y);
  double* res_l = (double*)(smem + L.o_res);
  double* coef_l = (double*)(smem + L.o_coef);
  double* gram = (double*)(smem + L.o_gram);
  double* Ec = (double*)(smem + L.o_Ec);       // E[:, 0:r] (2r × r)
  double* mx = (double*)(smem + L.o_mx);       // expm(-t·A) (r × r)
  double* temp_l = (double*)(smem + L.o_temp);
  double* W_l = (double*)(smem + L.o_W);
  double* U_l = (double*)(smem + L.o_U);
  double* red = (double*)(smem + L.o_red);

  const int e = (int)(t / P.nb), b = (int)(t - (long long)e * P.nb);
  const int start = b * m;
  const int Bt = min(m, P.N - start);
  const int32_t* ord = C.order + (size_t)(e & 1) * P.N + start;
  const bool wblock = (k == D);
  const long long t1 = t + 1;
  const int e1 = (int)(t1 / P.nb), b1 = (int)(t1 - (long long)e1 * P.nb);
  const int s1 = b1 * m;
  const bool has_next = t1 < P.total_steps;
  const int B1 = has_next ? min(m, P.N - s1) : 0;
  const int32_t* ord1 = C.order + (size_t)((has_next ? e1 : e) & 1) * P.N + (has_next ? s1 : start);
  const int Bs = Bt, Bsn = B1;         // this workgroup's batch columns and next-batch columns
  // the element loops' divisors (fast_div: no runtime integer division per element)
  const FastDiv fdMP = fast_div(MP), fdNP = fast_div(NP), fdBs = fast_div(Bs), fdn = fast_div(n),
                fdNQ = fast_div(64 * unoise_nq(n));
  // rows of the next batch this lane touches into L2 during the V-phase (P5 streams them at the
  // end of the step): lanes 0-31 / 32-63 of wave w cover rows 2(w + kNW·x) + {0, 1}
  int trow[kTouch];
  const bool touch = GPT_TOUCH && k < D && has_next && Bsn > 0;
  if (touch) {
#pragma unroll
    for (int x = 0; x < kTouch; ++x) {
      const int i = 2 * (wv + kNW * x) + ((tid & 63) >> 5);
      trow[x] = gptr(ord1)[min(i, Bsn - 1)];         // past the batch: its last row again
    }
  }
  STAMP(0);

  // ---- P0: stage temp (this batch), I, w, batch rows and targets
  {
    const double* tsrc = C.temp + (size_t)(t & 1) * D * R * m;
    for (int o = tid; o < D * R * MP; o += kNT) {   // zero tail: unrolled reads run past Bs
      const int row = fdiv(o, fdMP), i = o - row * MP;
      temp_l[o] = i < Bs ? gptr(tsrc)[row * m + i] : 0.0;
    }
    for (int i = tid; i < MP; i += kNT) res_l[i] = 0.0;
    if (!(vcols && k < D))       // read by the w block's gradw and vphase_tile only
      for (int o = tid; o < Q * D; o += kNT) IT_l[o] = gptr(P.I0)[o];   // I0 is already q + Q*k
    // RMSprop U phase: A uses the new w written by the w phase (GPT_SGLD.jl:1193-1199)
    const double* wsrc = C.w + (size_t)(((P.rms && k < D) ? t + 1 : t) & 1) * Q;
    for (int q = tid; q < Q; q += kNT) w_l[q] = gptr(wsrc)[q];
    for (int i = tid; i < Bs; i += kNT) {
      const int row = gptr(ord)[i];
      idx_l[i] = row;
      y_l[i] = gptr(C.y)[row];
    }
    for (int o = tid; o < R * MP; o += kNT) coef_l[o] = 0.0;
    if (vcols) {
      double* ones = (double*)(smem + L.o_ones);
      for (int i = tid; i < MP; i += kNT) ones[i] = 1.0;
      const int4* tg = (const int4*)(P.vtab + (size_t)k * Q * 16);
      int4* tl = (int4*)(smem + L.o_vtab);
      for (int o = tid; o < 4 * Q; o += kNT) tl[o] = tg[o];
    }
  }
  __syncthreads();
  STAMP(1);

  const long long koff = (long long)n * k, rstride = (long long)n * D;
  // one 4-B load per 128-B line of the rows: the lines reach this XCD's L2 while the V-phase below
  // works from LDS only; the loaded words are consumed (an empty asm) only after the V-phase, so
  // their wait sits at its end (checked in the ISA: an LDS-DMA touch instead puts a vmcnt wait in
  // front of the V-phase's LDS reads, and so did batching P0's loads ahead of it)
  int tv[kTouch];
  if (touch) {
    const unsigned o = min(32u * (unsigned)(tid & 31), 2u * n - 1u);   // in 4-B words
#pragma unroll
    for (int x = 0; x < kTouch; ++x)
      tv[x] = gptr((const int*)(C.phi + koff + (long long)trow[x] * rstride))[o];
    asm volatile("" ::: "memory");
  }
  // ---- P1: V, fhat, residual, A[:,k,:] (GPT_SGLD.jl:384-399)
  {
    auto vout = [&](int comp, int i, double v) {
      if (comp == 0) res_l[i] = P.ncls ? v : y_l[i] - v;      // classification: fhat itself
      else coef_l[(comp - 1) * MP + i] = v;
    };
    if (vcols) {
      double* vred = (double*)(smem + L.o_vred);
      const int32_t* tab = (const int32_t*)(smem + L.o_vtab);
      if (Bs <= 32 && GPT_VHALF) {        // a small batch: two q per pass
        if (k < D) vphase_cols_half<R, true>(temp_l, tab, w_l, Q, Bs, vred, vout);
        else vphase_cols_half<R, false>(temp_l, tab, w_l, Q, Bs, vred, vout);
      } else if (k < D) {
        vphase_cols<R, true>(temp_l, tab, w_l, Q, Bs, vred, vout);
      } else {
        vphase_cols<R, false>(temp_l, tab, w_l, Q, Bs, vred, vout);
      }
    } else if (Bs <= kNW * VCfg<R>::ICV_SMALL)
      vphase_tile<R, VCfg<R>::ICV_SMALL>(temp_l, MP, IT_l, w_l, Q, D, k >= D ? 0 : k, Bs, vout);
    else
      vphase_tile<R, VCfg<R>::ICV_MAX>(temp_l, MP, IT_l, w_l, Q, D, k >= D ? 0 : k, Bs, vout);
  }
  if (touch) {
#pragma unroll
    for (int x = 0; x < kTouch; ++x) asm volatile("" ::"v"(tv[x]));
  }
  __syncthreads();
  STAMP(2);

  if (P.ncls) {
    const int cls = blockIdx.y % P.ncls;
    if (k == D + 1) {               // class-fhat pass: fhat of this class for its siblings
      for (int i = tid; i < Bt; i += kNT) gptr_w(C.res)[i] = res_l[i];
      return;
    }
    // softmax residual [y_i = c] − exp(fhat_ic − logsumexp_i fhat_i·) (GPT_SGLD.jl:509-526)
    const ChainDesc* sib = chains + (blockIdx.y - cls);
    for (int i = tid; i < Bt; i += kNT) {
      double u = -INFINITY;
      for (int c2 = 0; c2 < P.ncls; ++c2) u = fmax(u, gptr(sib[c2].res)[i]);
      double se = 0.0;
      for (int c2 = 0; c2 < P.ncls; ++c2) se += exp(gptr(sib[c2].res)[i] - u);
      const double lse = u + log(se);
      res_l[i] = ((int)y_l[i] == cls + 1 ? 1.0 : 0.0) - exp(gptr(sib[cls].res)[i] - lse);
    }
    __syncthreads();
  }

  const double cN = (double)P.N / (double)Bt;
  const long long post = t - P.burnin_steps;
  const bool store = post >= 0 && ((post + 1) % P.store_every) == 0;
  const long long slot = store ? (post + 1) / P.store_every - 1 : 0;

  if (wblock && P.rms) {
    // ---- RMSprop w phase (GPT_SGLD.jl:1182-1193): per-entry step sizes from the moving average
    //      of squared per-sample gradients; the residuals go to the U phase (which sees new w)
    for (int i = tid; i < Bt; i += kNT) gptr_w(C.res)[i] = res_l[i];
    double gn2 = 0.0;
    const double cR = 1.0 / ((double)Bt * C.signal_var);
    for (int q = tid; q < Q; q += kNT) {
      double g = 0.0;
      for (int i0 = 0; i0 < Bt; i0 += 16) {
        double vv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) vv[u] = 1.0;
        for (int kk = 0; kk < D; ++kk) {
          const double* row = temp_l + (kk * R + IT_l[kk * Q + q]) * MP + i0;
#pragma unroll
          for (int u = 0; u < 16; ++u) vv[u] *= row[u];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) g = fma(vv[u], res_l[i0 + u], g);
      }
      const double gr = g * cR;                                   // ĝw (:1182)
      const double gwq = P.rms_alpha * gptr(C.gw)[q] + (1.0 - P.rms_alpha) * gr * gr;
      gptr_w(C.gw)[q] = gwq;
      const double ew = P.rms_eps / (sqrt(gwq) + kRmsLambda);     // :1186
      const double wq = w_l[q];
      const double gradw = (double)P.N * gr - wq;                 // :1190 (σ_w = 1)
      const double wn = wq + ew * gradw / 2 +
                        sqrt(ew) * normal_at(C.seed, (uint32_t)q, (uint32_t)t, kWNoise, 0);
      gptr_w(C.w)[(size_t)((t + 1) & 1) * Q + q] = wn;
      if (store && C.w_store) gptr_w(C.w_store)[(size_t)slot * Q + q] = wn;
      gn2 = fma(gradw, gradw, gn2);
    }
    __syncthreads();
    if (C.diag) {
      const double tot = blk_sum(gn2, red);
      if (tid == 0) C.diag[(size_t)t * (1 + D)] = sqrt(tot);
    }
    return;
  }

  if (wblock) {
    // ---- gradw and the Langevin step on w (GPT_SGLD.jl:393, 411-414)
    double gn2 = 0.0;
    const double inv_sw2 = 1.0 / (C.sigma_w * C.sigma_w);
    const double sqe = sqrt(C.epsw);
    for (int q = tid; q < Q; q += kNT) {
      double g = 0.0;
      for (int i0 = 0; i0 < Bt; i0 += 16) {
        double vv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) vv[u] = 1.0;
        for (int kk = 0; kk < D; ++kk) {
          const double* row = temp_l + (kk * R + IT_l[kk * Q + q]) * MP + i0;
#pragma unroll
          for (int u = 0; u < 16; ++u) vv[u] *= row[u];      // MP covers i0+15 (zero tail)
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) g = fma(vv[u], res_l[i0 + u], g);   // res zero-padded
      }
      const double wq = w_l[q];
      const double gradw = cN * g / C.signal_var - wq * inv_sw2;
      double wn;
      if (P.ncls) {                 // two moves with the same gradient (GPT_SGLD.jl:624, :639-642)
        const int cls = blockIdx.y % P.ncls;
        const double w1 = wq + (C.epsw * gradw / 2 +
                                sqe * normal_at(C.seed, (uint32_t)q, (uint32_t)t, kWNoise, 2 * cls));
        double step = C.epsw * gradw / 2;
        if (P.langevin)
          step += sqe * normal_at(C.seed, (uint32_t)q, (uint32_t)t, kWNoise, 2 * cls + 1);
        wn = w1 + step;
      } else {
        double step = C.epsw * gradw / 2;
        if (P.langevin) step += sqe * normal_at(C.seed, (uint32_t)q, (uint32_t)t, kWNoise, 0);
        wn = wq + step;
      }
      gptr_w(C.w)[(size_t)((t + 1) & 1) * Q + q] = wn;
      if (store && C.w_store) gptr_w(C.w_store)[(size_t)slot * Q + q] = wn;
      gn2 = fma(gradw, gradw, gn2);
    }
    __syncthreads();
    STAMP(3);
    if (C.diag) {
      __syncthreads();
      const double tot = blk_sum(gn2, red);     // temp_l is dead after the barrier
      if (tid == 0) C.diag[(size_t)t * (1 + D)] = sqrt(tot);
    }
    return;
  }

  if (P.rms) {   // the residuals are the w phase's (old w); V above used the new w for A only
    for (int i = tid; i < Bt; i += kNT) res_l[i] = gptr(C.res)[i];
    __syncthreads();
  }
  // coef[l][i] = A[l][i]·res[i]; stage U^(k) (the union slot of temp_l is free now)
  for (int o = tid; o < R * Bs; o += kNT) {
    const int l = fdiv(o, fdBs), i = o - l * Bs;
    coef_l[l * MP + i] *= res_l[i];
  }
  const double* Ug = C.U + (size_t)n * R * k;
  // W_l starts as the Langevin noise ξ of the drive (quad contract, gpt_common.h): the quads are
  // spread over the threads here, so P2's thread-per-row drive reads its ξ[j, :] from LDS
  const bool noise0 = (P.langevin || P.ncls) && !P.rms;
  for (int o = tid; o < R * NP; o += kNT) {
    const int l = fdiv(o, fdNP), j = o - l * NP;
    U_l[l * NS + j] = j < n ? gptr(Ug)[j + (size_t)n * l] : 0.0;
    if (j >= n || !noise0) W_l[l * NS + j] = 0.0;
  }
  if (noise0) {
    const uint32_t c3 = P.ncls ? (uint32_t)(k + D * 2 * (blockIdx.y % P.ncls)) : (uint32_t)k;
    const int NQ = unoise_nq(n);
    for (int qd = tid; qd < R * NQ * 64; qd += kNT) {
      const int l = fdiv(qd, fdNQ), q = (qd >> 6) - l * NQ, lam = qd & 63;
      double z[4];
      normal_quad<4>(C.seed, (uint32_t)qd, (uint32_t)t, kUNoise, c3, z);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = lam + 64 * (4 * q + i);
        if (j < n) W_l[l * NS + j] = z[i];
      }
    }
  }
  __syncthreads();
  STAMP(3);

  // ---- P2: gradU^(k) = (N/B)/σ² Σ_i phi[:,k,i] (A[:,k,i] res_i)ᵀ   (GPT_SGLD.jl:396-408)
  const double cU = cN / C.signal_var;
  const double sq = sqrt(C.epsU);
  double gn2 = 0.0, esum = 0.0;
  // Uniform trip count (j clamped, writes masked): every lane takes part in the row-vector
  // load below, so v_readlane never reads a lane that skipped it.
  // the drive of row j from its gradient sums acc[l] = Σ_i phi[j,k,i]·A[l,k,i]·res_i
  auto drive = [&](int j, const double (&acc)[R]) {
    if (P.rms) {                  // :1212-1227: ĝU, moving average, N·ĝU kept until εU_k is known
#pragma unroll
      for (int l = 0; l < R; ++l) {
        const double gr = acc[l] / ((double)Bt * C.signal_var);
        const size_t e = (size_t)n * R * k + (size_t)n * l + j;
        const double gu = P.rms_alpha * gptr(C.gU)[e] + (1.0 - P.rms_alpha) * gr * gr;
        gptr_w(C.gU)[e] = gu;
        esum += P.rms_eps / (sqrt(gu) + kRmsLambda);
        const double G = (double)P.N * gr;
        gn2 = fma(G, G, gn2);
        W_l[l * NS + j] = G;
      }
    } else {
#pragma unroll
      for (int l = 0; l < R; ++l) {
        const double G = acc[l] * cU;
        gn2 = fma(G, G, gn2);
        if (P.ncls) gptr_w(C.gU)[(size_t)n * R * k + (size_t)n * l + j] = G;   // second move
        if (P.stiefel || P.ncls) {
          W_l[l * NS + j] = sq * G / 2 + W_l[l * NS + j];         // :420 drive (W_l held ξ)
        } else {                                                  // :426 / :437
          const double u = U_l[l * NS + j];
          U_l[l * NS + j] = u + (C.epsU * (G - n * u) / 2 + sq * W_l[l * NS + j]);
        }
      }
    }
  };
  for (int j0 = 0; j0 < n; j0 += kNT) {
    const int j = j0 + tid;
    const bool jok = j < n;
    const int jc = jok ? j : n - 1;
    double acc[R];
#pragma unroll
    for (int l = 0; l < R; ++l) acc[l] = 0.0;
    for (int i0 = 0; i0 < Bs; i0 += 32) {
      // lane u: address of the row of column i0+u (columns past Bs: the clamped row), formed
      // once per lane and broadcast as two 32-bit halves (no per-row 64-bit SALU multiply)
      const RowPtr rp(C.phi + koff, idx_l[min(i0 + (tid & 63), Bs - 1)], rstride);   // P0's rows
      double p[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) p[u] = GPT_EXP_P2NOLOAD ? 1e-3 * (u + jc) : rp.at(u)[jc];
#pragma unroll
      for (int u = 0; u < 32; ++u)
#pragma unroll
        for (int l = 0; l < R; ++l)
          acc[l] = fma(p[u], GPT_EXP_P2NOCOEF ? 1e-3 * (l + u) : coef_l[l * MP + i0 + u], acc[l]);
    }
    if (jok) drive(j, acc);
  }
  if (C.diag) {
    const double tot = blk_sum(gn2, red);
    if (tid == 0) C.diag[(size_t)t * (1 + D) + 1 + k] = sqrt(tot);
  }
  double sk = sq;                 // geodesic time: √εU, or √mean(εU_k) under RMSprop (:1218)
  if (P.rms) {
    __syncthreads();
    sk = sqrt(blk_sum(esum, red) / ((double)n * R));
    const int NQ = unoise_nq(n);
    for (int qd = tid; qd < R * NQ * 64; qd += kNT) {   // drive √εU_k·gradU/2 + ξ (:1231)
      const int l = fdiv(qd, fdNQ), q = (qd >> 6) - l * NQ, lam = qd & 63;
      double z[4];
      normal_quad<4>(C.seed, (uint32_t)qd, (uint32_t)t, kUNoise, (uint32_t)k, z);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = lam + 64 * (4 * q + i);
        if (j < n) W_l[l * NS + j] = sk * W_l[l * NS + j] / 2 + z[i];
      }
    }
  }
  __syncthreads();
  STAMP(4);

  // GPTclassification moves U twice with one gradient: pass 0 is SGLD + Stiefel whatever the
  // flags (GPT_SGLD.jl:627-636), pass 1 the langevin/stiefel variant from pass 0's U (:643-671)
  const int npass = P.ncls ? 2 : 1;
  for (int pass = 0; pass < npass; ++pass) {
  if (pass == 1) {
    // pass 0's U is the "old U" of pass 1 (re-read from HBM when it is not kept in LDS)
    for (int o = tid; o < R * n; o += kNT) {
      const int l = fdiv(o, fdn), j = o - l * n;
      gptr_w(C.U + (size_t)n * R * k)[o] = U_l[l * NS + j];
    }
    const uint32_t c3 = (uint32_t)(k + D * (2 * (blockIdx.y % P.ncls) + 1));
    const int NQ = unoise_nq(n);
    for (int qd = tid; qd < R * NQ * 64; qd += kNT) {
      const int l = fdiv(qd, fdNQ), q = (qd >> 6) - l * NQ, lam = qd & 63;
      double z[4] = {0.0, 0.0, 0.0, 0.0};
      if (P.langevin) normal_quad<4>(C.seed, (uint32_t)qd, (uint32_t)t, kUNoise, c3, z);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = lam + 64 * (4 * q + i);
        if (j >= n) break;
        const double G = gptr(C.gU)[(size_t)n * R * k + (size_t)n * l + j];
        if (P.stiefel) {
          W_l[l * NS + j] = sq * G / 2 + z[i];
        } else {
          const double u = U_l[l * NS + j];
          U_l[l * NS + j] = u + (C.epsU * (G - n * u) / 2 + sq * z[i]);
        }
      }
    }
    __syncthreads();
  }
  if (pass == 0 ? (P.stiefel || P.ncls) : P.stiefel) {
    double* Mg = gram;              // r×r   M = Uᵀ·drive
    double* Gg = gram + R * R;      // r×r   G = driveᵀ·drive
    double* Ag = gram + 2 * R * R;  // r×r   A = Uᵀ·mom
    double* Sg = gram + 3 * R * R;  // r×r   S = momᵀ·mom
    int* flag = (int*)(gram + 4 * R * R + R);
    // ---- proj (GPT_SGLD.jl:14-16): mom = V − U(UᵀV + VᵀU)/2, and the geod Grams (:19-37).  On the
    // Stiefel manifold (UᵀU = I: every move of a stiefel run is a geodesic from a Stiefel init) they
    // come from the same Gram pass: A = Uᵀmom = (M − Mᵀ)/2 and
    // S = momᵀmom = G − MᵀMs − Ms·M + Ms·Ms (M = UᵀV, G = VᵀV, Ms = (M + Mᵀ)/2), so no second pass
    // over mom (the oracle's reference form agrees to ≤ 1.2e-14 relative over whole trajectories,
    // tests/test_oracle.py).  GPTclassification's pass 0 with stiefel = false moves a U that the
    // Euclidean pass 1 took off the manifold: there A and S come from mom as the reference does.
    const bool onm = P.stiefel != 0;
    blk_gram<R>(U_l, W_l, NS, n, onm ? 1 : 0, Mg, red);
    if (onm) {
      for (int o = tid; o < R * R; o += kNT) {
        const int i = o / R, b = o - i * R;
        double s = Gg[min(i, b) * R + max(i, b)];
        for (int c = 0; c < R; ++c) {
          const double mci = Mg[c * R + i], mic = Mg[i * R + c];
          const double mcb = Mg[c * R + b], mbc = Mg[b * R + c];
          const double msic = (mic + mci) / 2, mscb = (mcb + mbc) / 2;
          s = fma(-mci, mscb, s);
          s = fma(-msic, mcb, s);
          s = fma(msic, mscb, s);
        }
        Sg[o] = s;
        Ag[o] = (Mg[o] - Mg[b * R + i]) / 2;
      }
    }
    for (int j = tid; j < n; j += kNT) {
      double vj[R], uj[R];
#pragma unroll
      for (int l = 0; l < R; ++l) { vj[l] = W_l[l * NS + j]; uj[l] = U_l[l * NS + j]; }
#pragma unroll
      for (int bb = 0; bb < R; ++bb) {
        double s = 0.0;
#pragma unroll
        for (int a = 0; a < R; ++a) s = fma(uj[a], Mg[a * R + bb] + Mg[bb * R + a], s);
        W_l[bb * NS + j] = vj[bb] - s / 2;
      }
    }
    __syncthreads();
    STAMP(5);
    if (!onm) blk_gram<R>(U_l, W_l, NS, n, 1, Ag, red);   // Ag = Uᵀmom, Sg = momᵀmom
    STAMP(6);
    const double tt = sk;
    const int nn = 2 * R;
    double* X0 = (double*)(smem + L.o_x0);     // U_l / red are dead from here to the update
    double* X1 = (double*)(smem + L.o_x1);
    if (wv == 0) {
      for (int o = tid; o < nn * nn; o += 64) {
        const int i = o / nn, j = o - i * nn;
        double v;
        if (i < R) v = j < R ? Ag[i * R + j] : -Sg[i * R + (j - R)];
        else v = j < R ? (i - R == j ? 1.0 : 0.0) : Ag[(i - R) * R + (j - R)];
        X0[o] = tt * v;
      }
      wave_sync();
      const bool bad = wave_expm<2 * R>(
          X0, P.stamps ? P.stamps + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * kStamps : nullptr);
      for (int o = tid; o < nn * R; o += 64) {
        const int a = o / R, l = o - a * R;
        Ec[o] = X0[nn * nn + a * nn + l];
      }
      if (tid == 0) flag[0] = bad ? 1 : 0;
      wave_sync();
    }
    if (wv == (L.conc ? 1 : 0)) {
      const int ln = tid & 63;
      for (int o = ln; o < R * R; o += 64) X1[o] = -tt * Ag[o];
      wave_sync();
      wave_expm<R>(X1);
      for (int o = ln; o < R * R; o += 64) mx[o] = X1[R * R + o];
    }
    __syncthreads();
    STAMP(7);
    if (flag[0]) {
      if (tid == 0) __hip_atomic_store(C.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if constexpr (R <= 8) {
      // tmpU = ([U mom]·E[:,1:r])·expm(-tA)   (old U re-read from HBM/L2; mom in W_l); each thread
      // keeps the squares of its rows, the column norms are one butterfly per wave and a wave-order
      // sum (no Gram pass over W_l), and a thread normalises the rows it wrote
      constexpr int NVN = R <= 8 ? 8 : (R <= 16 ? 16 : 32);
      double sq2[NVN];
  #pragma unroll
      for (int l = 0; l < NVN; ++l) sq2[l] = 0.0;
      for (int j = tid; j < n; j += kNT) {
        double x[2 * R];
  #pragma unroll
        for (int l = 0; l < R; ++l) {
          x[l] = L.keepU ? U_l[l * NS + j] : gptr(Ug)[j + (size_t)n * l];
          x[R + l] = W_l[l * NS + j];
        }
        double row1[R];
  #pragma unroll
        for (int l = 0; l < R; ++l) {
          double s = 0.0;
  #pragma unroll
          for (int a = 0; a < 2 * R; ++a) s = fma(x[a], Ec[a * R + l], s);
          row1[l] = s;
        }
  #pragma unroll
        for (int l = 0; l < R; ++l) {
          double s = 0.0;
  #pragma unroll
          for (int c2 = 0; c2 < R; ++c2) s = fma(row1[c2], mx[c2 * R + l], s);
          W_l[l * NS + j] = s;
          sq2[l] = fma(s, s, sq2[l]);
        }
      }
      {
        constexpr int SHN = 6 - Butterfly<NVN>::P;
        const int ln = tid & 63;
        Butterfly<NVN>::run(sq2, ln);
        const int vi = ln >> SHN;
        if ((ln & ((1 << SHN) - 1)) == 0 && vi < R) red[wv * NVN + vi] = sq2[0];
      }
      __syncthreads();
      double cn[R];
  #pragma unroll
      for (int l = 0; l < R; ++l) {
        double a = 0.0;
  #pragma unroll
        for (int w = 0; w < kNW; ++w) a += red[w * NVN + l];
        cn[l] = sqrt(a);
      }
      for (int j = tid; j < NP; j += kNT) {
  #pragma unroll
        for (int l = 0; l < R; ++l) U_l[l * NS + j] = j < n ? W_l[l * NS + j] / cn[l] : 0.0;
      }
    } else {   // r > 8: the Gram pass (the butterfly's partials would spill)
      // tmpU = ([U mom]·E[:,1:r])·expm(-tA)   (old U re-read from HBM/L2; mom in W_l)
      for (int j = tid; j < n; j += kNT) {
        double x[2 * R];
  #pragma unroll
        for (int l = 0; l < R; ++l) {
          x[l] = L.keepU ? U_l[l * NS + j] : gptr(Ug)[j + (size_t)n * l];
          x[R + l] = W_l[l * NS + j];
        }
        double row1[R];
  #pragma unroll
        for (int l = 0; l < R; ++l) {
          double s = 0.0;
  #pragma unroll
          for (int a = 0; a < 2 * R; ++a) s = fma(x[a], Ec[a * R + l], s);
          row1[l] = s;
        }
  #pragma unroll
        for (int l = 0; l < R; ++l) {
          double s = 0.0;
  #pragma unroll
          for (int c2 = 0; c2 < R; ++c2) s = fma(row1[c2], mx[c2 * R + l], s);
          W_l[l * NS + j] = s;
        }
      }
      __syncthreads();
      double* nrm = gram + 4 * R * R; // r
      blk_gram<R>(W_l, W_l, NS, n, 2, nrm, red);
      for (int o = tid; o < R * NP; o += kNT) {
        const int l = fdiv(o, fdNP), j = o - l * NP;
        U_l[l * NS + j] = j < n ? W_l[l * NS + j] / sqrt(nrm[l]) : 0.0;
      }
    }
    __syncthreads();
    STAMP(8);
  }
  }  // pass

  // ---- write U^(k) (and the sample store, GPT_SGLD.jl:441-444)
  {
    double* Uk = C.U + (size_t)n * R * k;
    double* Us = (store && C.U_store) ? C.U_store + ((size_t)slot * D + k) * n * R : nullptr;
    for (int o = tid; o < R * n; o += kNT) {
      const int l = fdiv(o, fdn), j = o - l * n;
      const double u = U_l[l * NS + j];
      gptr_w(Uk)[o] = u;
      if (Us) gptr_w(Us)[o] = u;
    }
  }

  // ---- P5: temp[k,:,:] of the next step with the new U^(k) (phidotU, GPT_SGLD.jl:193-205)
  if (has_next) {
    __syncthreads();
    STAMP(9);
    double* tdst = C.temp + (size_t)(t1 & 1) * D * R * m + (size_t)k * R * m;
    auto p5out = [&](int l, int i, double v) { gptr_w(tdst)[l * m + i] = v; };
    // the fewest batch columns per wave pass that cover the (slice of the) next batch in one pass
    // (fewer row loads, and at <= 32 values a half-size butterfly)
    if constexpr (RCfgX<R, 4>::ICH != RCfgX<R, 8>::ICH) {
      if (Bsn <= kNW * RCfgX<R, 4>::ICH) {
        phidotU_tile<R, decltype(p5out), 4>(C.phi, koff, rstride, ord1, 0, Bsn, n, NP, NS,
                                            U_l, p5out);
      } else if (Bsn <= kNW * RCfgX<R, 7>::ICH) {
        phidotU_tile<R, decltype(p5out), 7>(C.phi, koff, rstride, ord1, 0, Bsn, n, NP, NS,
                                            U_l, p5out);
      } else {
        phidotU_tile<R>(C.phi, koff, rstride, ord1, 0, Bsn, n, NP, NS, U_l, p5out);
      }
    } else {
      phidotU_tile<R>(C.phi, koff, rstride, ord1, 0, Bsn, n, NP, NS, U_l, p5out);
    }
    __syncthreads();
    STAMP(10);
  }
}

// temp of the first step of a run (or after a restart): phidotU of batch t with U as stored.
template <int R>
__global__ __launch_bounds__(kNT) void temp_init_kernel(StepParams P,
                                                        const ChainDesc* __restrict__ chains,
                                                        const long long* __restrict__ tbase,
                                                        int t_local) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const ChainDesc C = chains[blockIdx.y];
  const int k = blockIdx.x, tid = threadIdx.x;
  const long long t = tbase[0] + t_local;
  if (t >= P.total_steps) return;
  const int n = P.n, D = P.D, m = P.m;
  const StepLayout L = step_layout(n, D, R, P.Q, m);
  const int NP = L.NP, NS = L.NS;
  const FastDiv fdNP = fast_div(NP);
  double* U_l = (double*)(smem + L.o_U);
  const int e = (int)(t / P.nb), b = (int)(t - (long long)e * P.nb);
  const int start = b * m;
  const int Bt = min(m, P.N - start);
  const int32_t* ord = C.order + (size_t)(e & 1) * P.N + start;
  const double* Uk = C.U + (size_t)n * R * k;
  for (int o = tid; o < R * NP; o += kNT) {
    const int l = fdiv(o, fdNP), j = o - l * NP;
    U_l[l * NS + j] = j < n ? Uk[j + (size_t)n * l] : 0.0;
  }
  __syncthreads();
  double* tdst = C.temp + (size_t)(t & 1) * D * R * m + (size_t)k * R * m;
  phidotU_tile<R>(C.phi, (long long)n * k, (long long)n * D, ord, 0, Bt, n, NP, NS, U_l,
                  [&](int l, int i, double v) { tdst[l * m + i] = v; });
}

__global__ void advance_kernel(long long* tbase, long long by) {
  if (threadIdx.x == 0 && blockIdx.x == 0) tbase[0] += by;
}

#define GPT_RANKS(X) X(1) X(2) X(3) X(4) X(5) X(6) X(8) X(10) X(12) X(15) X(16) X(20)

void vphase_cols_tables(const std::vector<int32_t>& I0, int n, int D, int r, int Q, int m,
                        std::vector<int32_t>& out) {
  const StepLayout L = step_layout(n, D, r, Q, m);
  const int ones = (int)((L.o_ones - L.o_temp) / 8), MP = L.MP;
  out.assign((size_t)(D + 1) * Q * 16, 0);
  for (int k = 0; k <= D; ++k)
    for (int q = 0; q < Q; ++q) {
      int32_t* e = out.data() + ((size_t)k * Q + q) * 16;
      for (int s = 0; s < 8; ++s) {
        int kk = -1;
        if (k == D) kk = s < D ? s : -1;                 // w block: all factors in k order
        else if (s == 7) kk = k;                         // own factor last
        else if (s < D - 1) kk = s < k ? s : s + 1;      // the others in k order
        e[s] = kk < 0 ? ones : (kk * r + I0[q + (size_t)Q * kk]) * MP;
      }
      e[8] = k < D ? I0[q + (size_t)Q * k] : 0;
    }
}

bool rank_supported(int r) {
  switch (r) {
#define CASE(RR) case RR:
    GPT_RANKS(CASE)
#undef CASE
    return true;
    default: return false;
  }
}

hipError_t launch_temp_init(const StepParams& P, const ChainDesc* chains, int nchains,
                            const long long* tbase, hipStream_t st) {
  const StepLayout L = step_layout(P.n, P.D, P.r, P.Q, P.m);
  dim3 grid(P.D, nchains);
  switch (P.r) {
#define CASE(RR)                                                                           \
  case RR:                                                                                 \
    hipLaunchKernelGGL(temp_init_kernel<RR>, grid, dim3(kNT), L.bytes, st, P, chains, tbase, 0); \
    break;
    GPT_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_step(const StepParams& P, const ChainDesc* chains, int nchains,
                       const long long* tbase, int t_local, hipStream_t st) {
  const StepLayout L = step_layout(P.n, P.D, P.r, P.Q, P.m);
  dim3 grid(P.D + 1, nchains);
  switch (P.r) {
#define CASE(RR)                                                                              \
  case RR:                                                                                    \
    hipLaunchKernelGGL(sgld_step_kernel<RR>, grid, dim3(kNT), L.bytes, st, P, chains, tbase,  \
                       t_local, 0);                                                           \
    break;
    GPT_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_step_rms(const StepParams& P, const ChainDesc* chains, int nchains,
                           const long long* tbase, int t_local, hipStream_t st) {
  const StepLayout L = step_layout(P.n, P.D, P.r, P.Q, P.m);
  switch (P.r) {
#define CASE(RR)                                                                              \
  case RR:                                                                                    \
    hipLaunchKernelGGL(sgld_step_kernel<RR>, dim3(1, nchains), dim3(kNT), L.bytes, st, P,     \
                       chains, tbase, t_local, P.D);                                          \
    hipLaunchKernelGGL(sgld_step_kernel<RR>, dim3(P.D, nchains), dim3(kNT), L.bytes, st, P,   \
                       chains, tbase, t_local, 0);                                            \
    break;
    GPT_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// GPT_SGLDERMw (GPT_SGLD.jl:1065-1118): U never moves, so each step is temp of its batch with the
// fixed U (temp_init_kernel) followed by the w block alone.
hipError_t launch_step_wonly(const StepParams& P, const ChainDesc* chains, int nchains,
                             const long long* tbase, int t_local, hipStream_t st) {
  const StepLayout L = step_layout(P.n, P.D, P.r, P.Q, P.m);
  switch (P.r) {
#define CASE(RR)                                                                              \
  case RR:                                                                                    \
    hipLaunchKernelGGL(temp_init_kernel<RR>, dim3(P.D, nchains), dim3(kNT), L.bytes, st, P,   \
                       chains, tbase, t_local);                                               \
    hipLaunchKernelGGL(sgld_step_kernel<RR>, dim3(1, nchains), dim3(kNT), L.bytes, st, P,     \
                       chains, tbase, t_local, P.D);                                          \
    break;
    GPT_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// GPTclassification: the class-fhat pass (one workgroup per class) then the step of every class.
hipError_t launch_step_cls(const StepParams& P, const ChainDesc* chains, int nchains,
                           const long long* tbase, int t_local, hipStream_t st) {
  const StepLayout L = step_layout(P.n, P.D, P.r, P.Q, P.m);
  switch (P.r) {
#define CASE(RR)                                                                              \
  case RR:                                                                                    \
    hipLaunchKernelGGL(sgld_step_kernel<RR>, dim3(1, nchains), dim3(kNT), L.bytes, st, P,     \
                       chains, tbase, t_local, P.D + 1);                                      \
    hipLaunchKernelGGL(sgld_step_kernel<RR>, dim3(P.D + 1, nchains), dim3(kNT), L.bytes, st,  \
                       P, chains, tbase, t_local, 0);                                         \
    break;
    GPT_RANKS(CASE)
#undef CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_advance(long long* tbase, long long by, hipStream_t st) {
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(64), 0, st, tbase, by);
  return hipGetLastError();
}

// Opt the kernels into >64 KiB of dynamic LDS once per process.
hipError_t set_lds_limits() {
  static std::atomic<uint64_t> done{0};
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (done.load(std::memory_order_acquire) & (1ull << (dev & 63))) return hipSuccess;
#define CASE(RR)                                                                              \
  e = hipFuncSetAttribute((const void*)sgld_step_kernel<RR>,                                   \
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);            \
  if (e != hipSuccess) return e;                                                              \
  e = hipFuncSetAttribute((const void*)temp_init_kernel<RR>,                                   \
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);            \
  if (e != hipSuccess) return e;
  GPT_RANKS(CASE)
#undef CASE
  done.fetch_or(1ull << (dev & 63), std::memory_order_acq_rel);
  return e;
}

}  // namespace gpt
