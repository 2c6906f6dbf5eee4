// Chain-resident SGLD engine for MI355X (gfx950): one workgroup per chain.
//
// Workgroup = D waves; wave k owns U^(k) (n×r) in REGISTERS for the step (lane λ holds rows
// j = λ + 64·jj, jj < J).  A step (GPT_SGLD.jl:377-445) streams its minibatch G rows at a time;
// each row slice phi[:,k,row] is read from HBM ONCE — staged into this wave's LDS slice by
// LDS-DMA (global_load_lds) one group ahead — and used twice from registers:
//   (b) temp[k,:,row]  = phi[:,k,row]ᵀ U^(k)                    (phidotU, :193-205)
//   (c) V, fhat and the core sums A[:,k,row] for the G rows, all waves together
//       (computeV / computefhat / computeU_phi / computeA, :208-273)
//   (e) gradU^(k) += phi[:,k,row] · (A[:,k,row]·res_row)ᵀ        (computePsi + Psi·res, :276-408)
// The grid engine (sgld.hip) reads the batch twice.  After the batch: the w update (block-wide)
// and, per wave with no block barrier, the Langevin drive, Stiefel projection, geodesic (two Padé
// expm on the wave) and renormalisation of U^(k) in registers.
//
// The core sums A[l,k,row] = Σ_{q: I[q,k]=l} w_q·V_q/temp[k,l,row] are formed as
// (Σ_{q in run (k,l)} w_q·V_q) · (1/temp[k,l,row]): the V tasks write w_q·V_q once per (row, q)
// and the run members (host table runq, q ascending) are gathered by 8-lane groups — fixed
// order, no atomics, and 1/temp is formed once per (k, l, row) when temp is.
#include "device_util.h"

namespace gpt {

// Variants measured and dropped in rounds 1-3 (DESIGN.md keeps the numbers) are no longer
// switchable here: LDS-scratch (b) reductions, padded butterflies, other row-staging points,
// double-buffered staging, L2 touches of the next batch, wave priorities, the fused M + G Gram.
constexpr int kChainBufs = 1;     // row-staging buffers
constexpr int kChainDMax = 8;     // waves per workgroup (one per input dimension)
constexpr int kChainTPW8 = 1;     // V tasks per wave at J = 8, D > 4
constexpr int kChainTasks = 2;    // V-phase tasks per wave (NCH·G <= tasks·D); J = 8: kChainTPW8
constexpr int kChainG = 2;        // batch rows per group (G = 3 spills 60 VGPRs)
constexpr int kChainQPL = 4;      // q chunks of 64 (Q <= 64·kChainQPL)
constexpr int kChainQP = 64 * kChainQPL;
constexpr int kChainRun = 64;     // members per run (core entries with one value of I[·,k])
constexpr int kChainRunS = 72;    // reduction scratch stride (doubles): 8-lane readers of rows
                                  // l, l+1.. hit disjoint LDS bank ranges (72·2 dwords ≡ 16 banks)
constexpr int kChainQS = 264;     // w·V row stride; slot kChainQP of a row is a constant 0

constexpr int kChainMMax = 256;   // largest minibatch the engine takes

// Per-wave scratch after the batch: S0 = max(expm<2r> scratch, noise slots) | E[:,1:r] | grams.
GPT_HD constexpr int chain_scratch_dbl(int r) {
  const int s0a = 7 * 4 * r * r, s0b = 64 * 8;     // expm scratch | noise slots (8 row blocks)
  return (s0a > s0b ? s0a : s0b) + 2 * r * r + 3 * r * r + r;
}
GPT_HD constexpr int al16c(int x) { return (x + 15) & ~15; }

// LDS carve of chain_kernel<R, J, G>, fixed at compile time: every table is sized for the
// engine's maxima (kChainDMax dimensions, Q <= kChainQP, m <= kChainMMax), so every LDS address
// is a constant and none of them occupies a scalar register (the kernel sits at the SGPR limit).
template <int R, int G, int WV = kChainDMax>
struct ChainLds {
  static constexpr int DRG = kChainDMax * R * G;          // temp entries of a slot
  static constexpr int TS = 2 * (DRG + G);                // temp | ones(G) | 1/temp | ones(G)
  static constexpr int NTMAX = kChainQPL * G;             // V tasks at Q = kChainQP
  static constexpr int o_IT = 0;                                         // int[kChainDMax][Q]
  static constexpr int o_w = al16c(o_IT + 4 * kChainQP * kChainDMax);    // double[Q]
  static constexpr int o_idx = al16c(o_w + 8 * kChainQP);                // int[m]
  static constexpr int o_y = al16c(o_idx + 4 * kChainMMax);              // double[m]
  static constexpr int o_temp = al16c(o_y + 8 * kChainMMax);             // 2 slots
  static constexpr int o_fp = al16c(o_temp + 8 * 2 * TS);
  static constexpr int o_gwp = al16c(o_fp + 8 * kChainQPL * G);
  static constexpr int o_misc = al16c(o_gwp + 8 * NTMAX * 64);
  static constexpr int o_touch = al16c(o_misc + 8 * 16);                // 256 B DMA sink
  static constexpr int o_un = al16c(o_touch + 256);
  // union: w·V rows [row][q] (stride kChainQS) + per-wave reduction scratch (batch loop) |
  // per-wave post-batch scratch
  // (per-wave parts sized for the WV waves of the build: at WV = 4 the carve plus the row staging
  // stays under 80 KB, two chains per CU)
  static constexpr int L_dbl = G * kChainQS + WV * G * R * kChainRunS;
  static constexpr int x_dbl = chain_scratch_dbl(R);
  // after the union: the U noise's (sin, cos)(2πi/256) table (WV = 8 builds; the WV = 4 carve
  // stays under 80 KB for two chains per CU and draws its angles by polynomial)
  static constexpr int o_tab = al16c(o_un + 8 * (L_dbl > x_dbl * WV ? L_dbl : x_dbl * WV));
  static constexpr bool tab = WV == kChainDMax;
  static constexpr int bytes = al16c(o_tab + (tab ? 8 * 64 : 0));
};

// Timeline of every workgroup in P.stamps (gpt_sgld_session_timeline; kTimeline slots per block).
// 2 (product): entry, prologue end and the launch's last step end, plus HW_ID / XCC_ID — the
// per-launch dispatch skew, prologue and per-chain span, and shader cycles per step independent
// of the clock (scripts/ablation_run.py).  The step loop itself carries no stamp code, and this
// build is also the faster allocation: 217 k shader cycles per 256-chain step and no scratch
// reload in the batch loop, against 69 spilled VGPRs with ten reloads per row group when the
// entry / exit stamps are left out too (round 3).  1 (make timeline): every step end as well.
#ifndef CHAIN_TIMELINE
#define CHAIN_TIMELINE 2
#endif

#ifndef CHAIN_SSTAMP
#define CHAIN_SSTAMP 0            // diagnostic builds only (make diag): Stiefel sub-phase stamps
#endif
// Phase / loop stamps (gpt_sgld_session_stamps): compiled into the diagnostic builds only.  The
// product kernel without them takes 217 k instead of 236 k shader cycles per 256-chain step
// (scripts/ablation_run.py, round 3) although the allocator then reports 65 spilled VGPRs
// instead of 20: the stamps' branches split the step into blocks the scheduler could not
// overlap across.
#ifndef CHAIN_STAMPS
#define CHAIN_STAMPS CHAIN_SSTAMP
#endif
#define CHAIN_FENCE() do {} while (0)
// Post-batch wave priorities.  The two waves of a SIMD (dimensions k and k + 4) run the same
// per-wave Stiefel phase after the batch; with equal priority the older wave runs ahead and its
// partner finishes the phase alone, every latency exposed.  Waves k >= 4 take priority 1 for the
// w update and the U noise, waves k < 4 from the projection through the 2r × 2r expm, waves
// k >= 4 again from expm(−tA) to the end of the step: 201.0 k → 196.8 k shader cycles per 256-chain
// step (−2.1 %, two alternating A/B rounds, profiles/r6_chain_priority_ab.txt); a fixed priority
// (+1 %), a flip at every sub-phase (+4 %) and other flip points (−0.1 … −1.2 %) measured worse.
// CHAIN_PRIO=0 builds the equal-priority kernel for comparison.
#ifndef CHAIN_PRIO
#define CHAIN_PRIO 2
#endif
#define CHAIN_SETPRIO(hi_upper)                                                             \
  do {                                                                                      \
    if (CHAIN_PRIO) {                                                                       \
      if ((k >= 4) == (hi_upper)) __builtin_amdgcn_s_setprio(1);                            \
      else __builtin_amdgcn_s_setprio(0);                                                   \
    }                                                                                       \
  } while (0)
#if !CHAIN_STAMPS
#define CSTAMP(slot) CHAIN_FENCE()
#endif
#if CHAIN_TIMELINE
// slot i of the block's timeline: {s_memrealtime (100 MHz constant clock), s_memtime (shader
// clock)}; 0 = entry, 1 = prologue end, 2 + s = end of the launch's step s.
#define TSTAMP_ANY(i)                                                                       \
  do {                                                                                      \
    if (P.tline && tid == 0 && (i) < kTimelineSteps + 2) {                                  \
      long long* ts_ = P.tline + (size_t)blockIdx.x * kTimeline + 2 * (i);                  \
      ts_[0] = (long long)__builtin_amdgcn_s_memrealtime();                                \
      ts_[1] = (long long)__builtin_amdgcn_s_memtime();                                    \
    }                                                                                       \
  } while (0)
#else
#define TSTAMP_ANY(i) do {} while (0)
#endif
// CHAIN_TIMELINE = 1: every step end; = 2: entry, prologue end and the launch's last step end only
// (no stamp code inside the step loop, so the loop compiles as in the product kernel)
#if CHAIN_TIMELINE == 1
#define TSTAMP(i) TSTAMP_ANY(i)
#else
#define TSTAMP(i) do {} while (0)
#endif
#if CHAIN_STAMPS
#define CSTAMP(slot)                                                                        \
  do {                                                                                      \
    if (P.stamps && tid == 0)                                                               \
      P.stamps[(size_t)blockIdx.x * kStamps + (slot)] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
#endif

// Loop sub-phase stamps (diagnostic runs only): waves 0 and 4 (one SIMD) at one row group, in the
// stamp row gridDim.x + blockIdx.x (the library sizes the stamp buffer for D+1 rows per chain).
#if CHAIN_STAMPS
#define LSTAMP(slot)                                                                        \
  do {                                                                                      \
    if (P.stamps && g0 == 20 && lane == 0 && (k == 0 || k == 4))                            \
      P.stamps[(size_t)(gridDim.x + blockIdx.x) * kStamps + (k ? 8 : 0) + (slot)] =         \
          (long long)__builtin_amdgcn_s_memtime();                                         \
  } while (0)
#else
#define LSTAMP(slot) CHAIN_FENCE()
#endif

// Stiefel sub-phase stamps (diagnostic runs only): waves 0 and 4 of every step, slot i < 16 in
// stamp row (2 + i/8)·gridDim.x + blockIdx.x (columns i%8, +8 for wave 4).
#define SSTAMP(slot)                                                                        \
  do {                                                                                      \
    if ((slot) == 4) CHAIN_SETPRIO(false);  /* after the U noise: waves k < 4 first */      \
    if ((slot) == 7) CHAIN_SETPRIO(true);   /* after the 2r x 2r expm: waves k >= 4 */     \
    if (CHAIN_SSTAMP && P.stamps && lane == 0 && (k == 0 || k == 4))                                        \
      P.stamps[(size_t)((2 + (slot) / 8) * gridDim.x + blockIdx.x) * kStamps + (k ? 8 : 0) + \
               (slot) % 8] = (long long)__builtin_amdgcn_s_memtime();                       \
  } while (0)

// Workgroup barrier that orders LDS only: an LDS-DMA prefetch stays in flight across it
// (__syncthreads() would also drain vmcnt).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// WV: waves per workgroup the build is bounded for — kChainDMax, or 4 for D <= 4, where one wave
// per SIMD leaves the register file to two V tasks per wave even at J = 8 (PowerPlant, D = 4,
// minibatch 256: 8 tasks per row group).
template <int R, int J, int G, int WV>
__global__ __launch_bounds__(64 * WV, WV == 4 ? 2 : 1) void chain_kernel(StepParams P,
                                                                const ChainDesc* chains,
                                                                const long long* __restrict__ tbase,
                                                                int t_local, int nsteps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ __attribute__((aligned(16))) double pbuf[kChainBufs * WV * G * 64 * J];   // row staging
  // Chain fields are read through Cp at their point of use (scalar loads) rather than held in
  // SGPRs across the batch loop, where SGPR pressure spills into VGPR lanes.
  const ChainDesc* Cp = chains + blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, k = uni(tid >> 6);
  const int n = P.n, D = P.D, Q = P.Q, m = P.m, NTH = 64 * D;
  using L = ChainLds<R, G, WV>;
  const int NCH = (Q + 63) / 64, NT = NCH * G;                  // q chunks of 64, V tasks
  int* IT_l = (int*)(smem + L::o_IT);
  double* w_l = (double*)(smem + L::o_w);
  int* idx_l = (int*)(smem + L::o_idx);
  double* y_l = (double*)(smem + L::o_y);
  double* temp_l = (double*)(smem + L::o_temp);
  double* fp_l = (double*)(smem + L::o_fp);
  double* gwp_l = (double*)(smem + L::o_gwp);
  double* misc = (double*)(smem + L::o_misc);
  int* flag = (int*)(misc + 8);
  double* wVr = (double*)(smem + L::o_un);                      // w_q·V_q per batch row
  double* X = (double*)(smem + L::o_un) + k * L::x_dbl;         // this wave's scratch
  double* xi_l = X;                                             // noise slots (before expm)
  double* pw0 = pbuf + k * (kChainBufs * G * 64 * J);           // this wave's staged rows
  [[maybe_unused]] double* bscr = wVr + G * kChainQS + k * G * R * kChainRunS;   // per row

  // steps t0 .. tend-1 of this chain in one launch (a chunk of at most one epoch): U^(k) stays in
  // registers and w in LDS between steps; the next batch's rows and targets are fetched during
  // the previous step's Stiefel phase
  TSTAMP_ANY(0);
#if CHAIN_TIMELINE
  if (P.tline && tid == 0) {            // where the workgroup runs: HW_ID and XCC_ID
    long long* ts_ = P.tline + (size_t)blockIdx.x * kTimeline + kTimeline - 2;
    ts_[0] = (long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    ts_[1] = (long long)__builtin_amdgcn_s_getreg((31 << 11) | 20);
  }
#endif
  const long long t0 = tbase[0] + t_local;
  if (t0 >= P.total_steps) return;
  if (__hip_atomic_load(Cp->status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  CSTAMP(0);
  const long long tend = min(P.total_steps, t0 + (long long)nsteps);

  // batch of step tt: its rows of the epoch order and its length
  auto batch_of = [&](long long tt, int& bt) -> const int32_t* {
    const int ee = (int)(tt / P.nb), bb = (int)(tt - (long long)ee * P.nb);
    bt = min(m, P.N - bb * m);
    return Cp->order + (size_t)(ee & 1) * P.N + (size_t)bb * m;
  };
  long long t = t0;
  int Bt;
  const int32_t* ord = batch_of(t, Bt);
  const long long koff = (long long)n * k, rstride = (long long)n * D;
  const double* phi_k = uni_ptr(Cp->phi) + koff;
  // Stage rows g0n .. g0n+G-1 of this wave's dimension into pw (lane-linear LDS image: double j
  // of row gg at pw[gg·64J + j]); bytes past the row end are clamped in-row and never read.
  auto stage_rows = [&](const int (&rows)[G], int ln, double* pw) {
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      const char* rb = (const char*)(phi_k + (long long)rows[gg] * rstride);
      __attribute__((address_space(3))) double* dst =
          (__attribute__((address_space(3))) double*)(pw + gg * 64 * J);
      if constexpr (J >= 2) {           // n even (chain_supported): 16-B pieces, J/2 per row
#pragma unroll
        for (int s = 0; s < J / 2; ++s) {
          const unsigned o = min(16u * ln + 1024u * s, 8u * n - 16u);
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(rb + o),
                                           (__attribute__((address_space(3))) void*)(dst + 128 * s),
                                           16, 0, 0);
        }
      } else {                          // n <= 64: 4-B pieces, 2 per row
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const unsigned o = min(4u * ln + 256u * s, 8u * n - 4u);
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(rb + o),
                                           (__attribute__((address_space(3))) void*)(dst + 32 * s),
                                           4, 0, 0);
        }
      }
    }
  };
  auto stage = [&](int g0n, int ln, double* pw) {
    int rows[G];
#pragma unroll
    for (int gg = 0; gg < G; ++gg) rows[gg] = uni(idx_l[min(g0n + gg, Bt - 1)]);
    // no LDS read between the DMA issues: a DS read after a pending LDS-DMA may be ordered
    // behind it (vmcnt) by the compiler
    stage_rows(rows, ln, pw);
  };
  {
    // the first group's rows go out before the prologue's own loads (row indices from global)
    int rows0[G];
#pragma unroll
    for (int gg = 0; gg < G; ++gg) rows0[gg] = gptr(ord)[min(gg, Bt - 1)];
    stage_rows(rows0, lane, pw0);
  }

  // ---- prologue: index tables, w, batch rows, and U^(k) into registers
  constexpr int DRG = L::DRG;           // temp entries of all kChainDMax dimensions
  {
    // IT_l[kk·Q+q]: temp index (kk·R + I[q,kk])·G of the core entry (+gg at use); rows kk >= D
    // point at the ones slot.
    for (int o = tid; o < Q * kChainDMax; o += NTH) {
      const int kk = o / Q, q = o - kk * Q;
      IT_l[o] = kk < D ? (kk * R + gptr(P.I0)[q + Q * kk]) * G : DRG;
    }
    for (int o = tid; o < G; o += NTH) wVr[o * kChainQS + kChainQP] = 0.0;   // gather zero slots
    for (int o = tid; o < 2 * G; o += NTH) {                     // ones slots of both temp slots
      temp_l[o / G * L::TS + DRG + o % G] = 1.0;
      temp_l[o / G * L::TS + 2 * DRG + G + o % G] = 1.0;
    }
    for (int o = tid; o < kChainQPL * G; o += NTH) fp_l[o] = 0.0;
  }
  if constexpr (L::tab) sincos_tab_fill((double*)(smem + L::o_tab), tid, NTH);
  for (int q = tid; q < Q; q += NTH) w_l[q] = gptr(Cp->w)[(size_t)(t0 & 1) * Q + q];
  if (tid == 0) flag[0] = 0;
  {
    const double* yv = Cp->y;
    for (int i = tid; i < Bt; i += NTH) {
      const int row = gptr(ord)[i];
      idx_l[i] = row;
      y_l[i] = gptr(yv)[row];
    }
  }
  double u[J][R];
  {
    const double* Ug = Cp->U + (size_t)n * R * k;
#pragma unroll
    for (int jj = 0; jj < J; ++jj) {
      const int j = lane + 64 * jj;
      const int jc = min(j, n - 1);          // unconditional in-bounds loads, padding rows zeroed
#pragma unroll
      for (int l = 0; l < R; ++l) {
        const double x = gptr(Ug + (size_t)n * l)[jc];
        u[jj][l] = j < n ? x : 0.0;
      }
    }
  }
  __syncthreads();
  CSTAMP(1);
  TSTAMP_ANY(1);



  constexpr int TPW = (J >= 8 && WV > 4) ? kChainTPW8 : kChainTasks;   // J = 8, D > 4: one task
  for (;;) {                             // ---------------------------------- one SGLD step
  // thread ids formed inside the step from v_mbcnt (not threadIdx.x): per-lane addresses are not
  // hoisted out of the step loop, and v0 need not be kept — the register-bound kernel used to spill
  // it and reload it (and values derived from it) in the Stiefel phase, each reload a vmcnt(0)
  // wait behind the next batch's row DMA (−4 % step time)
  const int lane = lane_id(), tid = 64 * k + lane;
  for (int o = tid; o < G; o += NTH) wVr[o * kChainQS + kChainQP] = 0.0;   // gather zero slots
  // (re-derived every step rather than held across the Stiefel phase, where registers are short)
  // this wave's V-task temp indices (< 256, four per register), fixed for the step
  unsigned itp[TPW][kChainDMax / 4];
#pragma unroll
  for (int x = 0; x < TPW; ++x) {
    const int task = k + D * x;
    const int c = task < NT ? task % NCH : 0;
    const int qq = min(64 * c + lane, Q - 1);
#pragma unroll
    for (int h = 0; h < kChainDMax / 4; ++h) {
      unsigned v = 0;
#pragma unroll
      for (int b4 = 0; b4 < 4; ++b4) v |= (unsigned)IT_l[(4 * h + b4) * Q + qq] << (8 * b4);
      itp[x][h] = v;
    }
  }
  // this lane's run members for the core sums of dimension k: lane 8l+s gathers members
  // s, s+8, .., s+56 of run (k, l) (two 16-bit q indices per register)
  unsigned gq[4];
  {
    const int rl0 = min(lane >> 3, R - 1), rs0 = lane & 7;
    const int32_t* rq = P.runq + ((size_t)k * R + rl0) * kChainRun + rs0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      gq[i] = (unsigned)gptr(rq)[16 * i] | ((unsigned)gptr(rq)[16 * i + 8] << 16);
  }
  double acc[J][R];
#pragma unroll
  for (int jj = 0; jj < J; ++jj)
#pragma unroll
    for (int l = 0; l < R; ++l) acc[jj][l] = 0.0;
  double vsave[TPW], gw[TPW];
#pragma unroll
  for (int x = 0; x < TPW; ++x) { vsave[x] = 0.0; gw[x] = 0.0; }

  int slot = 0;
  for (int g0 = 0; g0 < Bt; g0 += G, slot ^= 1) {
    // lane id the compiler cannot see through: per-lane addresses are recomputed inside the
    // loop instead of being hoisted into registers that stay live across it
    int ln = lane;
    asm volatile("" : "+v"(ln));
    LSTAMP(0);
    // (a) this wave's staged rows -> registers, then stage the next group behind them
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    LSTAMP(1);
    double* pw = pw0;
    double p[G][J];
#pragma unroll
    for (int gg = 0; gg < G; ++gg)
#pragma unroll
      for (int jj = 0; jj < J; ++jj)
        p[gg][jj] = pw[gg * 64 * J + ln + 64 * jj];   // j >= n: finite in-row values, u = 0 there
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    LSTAMP(2);
    // (b) temp[k,l,row] and 1/temp for the G rows: R partial dots per lane, reduced through this
    // wave's LDS scratch by 8-lane groups (lane 8l+s sums 8 partials of output l, DPP finishes)
    double* tsl = temp_l + slot * L::TS;
    const int rl = min(ln >> 3, R - 1);
    {
      // the G·R partial dots of this lane, reduced over the wave by one register butterfly
      // (permlane swaps + DPP, no LDS round trip) over exactly G·R values (obf_run)
      double v[G * R];
#pragma unroll
      for (int x = 0; x < G * R; ++x) v[x] = 0.0;
#pragma unroll
      for (int gg = 0; gg < G; ++gg)
#pragma unroll
        for (int jj = 0; jj < J; ++jj)
#pragma unroll
          for (int l = 0; l < R; ++l) v[gg * R + l] = fma(p[gg][jj], u[jj][l], v[gg * R + l]);
      obf_run<G * R, G * R>(v, ln);
      int vi;
      bool wr;
      obf_index<G * R>(ln, vi, wr);
      if (wr) {
        const int gg = vi / R, l = vi - gg * R;
        tsl[(k * R + l) * G + gg] = v[0];
        tsl[DRG + G + (k * R + l) * G + gg] = rcp_nr(v[0]);
      }
    }
    // the next group's rows are staged here, behind (b) (measured best of five placements)
    if (g0 + G < Bt) stage(g0 + G, ln, pw);
    LSTAMP(3);
    lds_barrier();
    LSTAMP(4);
    // (c) V tasks: task = gg·NCH + c covers q = 64c + lane of batch column g0+gg
#pragma unroll
    for (int x = 0; x < TPW; ++x) {
      const int task = k + D * x;
      if (task >= NT) break;
      const int gg = task / NCH, c = task - gg * NCH;
      const int q = 64 * c + ln;
      const bool ok = q < Q;
      const int qq = ok ? q : 0;
      // every LDS read of the task in flight at once: kChainDMax dimensions, no guards (rows
      // kk >= D of the table hit the ones slots)
      double tv[kChainDMax];                       // Π_k temp (computeV), as a product tree
#pragma unroll
      for (int kk = 0; kk < kChainDMax; ++kk)
        tv[kk] = tsl[((itp[x][kk >> 2] >> (8 * (kk & 3))) & 0xff) + gg];
      static_assert(kChainDMax == 8, "product tree below is written for 8 dimensions");
      const double V = ((tv[0] * tv[1]) * (tv[2] * tv[3])) * ((tv[4] * tv[5]) * (tv[6] * tv[7]));
      const double wV = ok ? w_l[qq] * V : 0.0;
      if (ok) wVr[gg * kChainQS + q] = wV;         // w_q·V_q, gathered by the run sums in (e)
      vsave[x] = ok ? V : 0.0;
      const double fs = wave_sum(wV);
      if (lane == 0) fp_l[gg * kChainQPL + c] = fs;
    }
    LSTAMP(5);
    lds_barrier();
    LSTAMP(6);
    // (e) residuals, A[:,k,·]·res, and the gradU / gradw accumulation
    double res[G];
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      double f = fp_l[gg * kChainQPL];
#pragma unroll
      for (int c = 1; c < kChainQPL; ++c) f += fp_l[gg * kChainQPL + c];   // unused chunks are 0
      res[gg] = (g0 + gg < Bt) ? y_l[g0 + gg] - f : 0.0;
    }
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      // A[l,k,row] = (Σ_{q in run (k,l)} w_q·V_q) / temp[k,l,row] (computeU_phi + computeA,
      // :248-273): lane 8l+s sums members s, s+8, .., the 8-lane group finishes with DPP; lane
      // 8l then holds A[l]
      const double* wr = wVr + gg * kChainQS;
      double a = wr[gq[0] & 0xffff];
#pragma unroll
      for (int i = 1; i < 8; ++i) a += wr[(gq[i >> 1] >> (16 * (i & 1))) & 0xffff];
      // A·res formed on every lane before the broadcast (same two products as A then ·res)
      a = (group8_sum(a) * tsl[DRG + G + (k * R + rl) * G + gg]) * res[gg];
      double cc[R];
#pragma unroll
      for (int l = 0; l < R; ++l) cc[l] = readlane_d(a, 8 * l);
#pragma unroll
      for (int jj = 0; jj < J; ++jj) {
        const double pv = p[gg][jj];
#pragma unroll
        for (int l = 0; l < R; ++l) acc[jj][l] = fma(pv, cc[l], acc[jj][l]);
      }
    }
#pragma unroll
    for (int x = 0; x < TPW; ++x) {
      const int task = k + D * x;
      if (task >= NT) break;
      const int gg = task / NCH;
      double rr = res[0];
#pragma unroll
      for (int g2 = 1; g2 < G; ++g2) if (gg == g2) rr = res[g2];
      gw[x] = fma(vsave[x], rr, gw[x]);
    }
    LSTAMP(7);
  }
  CSTAMP(2);

  // loaded after the batch loop (see Cp), through a pointer the compiler cannot see through, so
  // that the load is not hoisted out of the step loop (the fields would then hold ~40 SGPRs)
  const ChainDesc* Cq = Cp;
  asm volatile("" : "+s"(Cq));
  const ChainDesc C = *Cq;
  const double cN = (double)P.N / (double)Bt;
  const long long post = t - P.burnin_steps;
  const bool store = post >= 0 && ((post + 1) % P.store_every) == 0;
  const long long slot_s = store ? (post + 1) / P.store_every - 1 : 0;

  // ---- w: gradw and the Langevin step (GPT_SGLD.jl:393, 411-414)
#pragma unroll
  for (int x = 0; x < TPW; ++x) {
    const int task = k + D * x;
    if (task >= NT) break;
    gwp_l[task * 64 + lane] = gw[x];
  }
  SSTAMP(0);
  __syncthreads();
  SSTAMP(1);
  CHAIN_SETPRIO(true);
  {
    const double inv_sw2 = 1.0 / (C.sigma_w * C.sigma_w);
    const double sqe = sqrt(C.epsw);
    double gn2 = 0.0;
#pragma unroll 1
    for (int q = tid; q < Q; q += NTH) {
      const int c = q >> 6, ln = q & 63;
      double g = 0.0;
      for (int gg = 0; gg < G; ++gg) g += gwp_l[(gg * NCH + c) * 64 + ln];
      const double wq = w_l[q];
      const double gradw = cN * g / C.signal_var - wq * inv_sw2;
      double step = C.epsw * gradw / 2;
      step += sqe * normal_at(C.seed, (uint32_t)q, (uint32_t)t, kWNoise, 0);
      const double wn = wq + step;
      w_l[q] = wn;
      if (t + 1 == tend) gptr_w(C.w)[(size_t)((t + 1) & 1) * Q + q] = wn;
      if (store && C.w_store) gptr_w(C.w_store)[(size_t)slot_s * Q + q] = wn;
      gn2 = fma(gradw, gradw, gn2);
    }
    if (C.diag) {
      gn2 = wave_sum(gn2);
      if (lane == 0) misc[k] = gn2;
    }
  }
  SSTAMP(2);
  int Bn = 0;
  const int32_t* ordn = nullptr;
  if (t + 1 < tend) {
    // every wave is past the batch loop: the next batch's indices, targets and first rows
    ordn = batch_of(t + 1, Bn);
    for (int i = tid; i < Bn; i += NTH) {
      const int row = gptr(ordn)[i];
      idx_l[i] = row;
      y_l[i] = gptr(Cp->y)[row];
    }
    int rows0[G];
#pragma unroll
    for (int gg = 0; gg < G; ++gg) rows0[gg] = gptr(ordn)[min(gg, Bn - 1)];
    stage_rows(rows0, lane, pw0);
  }
  CSTAMP(3);
  SSTAMP(3);

  // ---- U^(k): gradient, Langevin drive, Stiefel projection + geodesic (per wave)
  const double cU = cN / C.signal_var;
  const double sq = sqrt(C.epsU);
  double gu2 = 0.0;
  // U noise on the quad contract (gpt_common.h): lane λ's rows λ + 64·jj are exactly the rows of
  // its quads, so every Box–Muller output is used.  One non-unrolled column loop (register-light
  // Philox/Box–Muller body, values through this lane's LDS slots); the column's drive is applied
  // under a uniform branch so the accumulator registers keep static indices.
  {
    constexpr int NQJ = (J + 3) / 4;
    constexpr int NZ = J >= 4 ? 4 : 2;
    const int NQ = unoise_nq(n);
#pragma unroll 1
    for (int l = 0; l < R; ++l) {
#pragma unroll
      for (int q = 0; q < NQJ; ++q) {
        double z[4];
        if constexpr (L::tab)
          normal_quad_tab<NZ>(C.seed, (uint32_t)((l * NQ + q) * 64 + lane), (uint32_t)t, kUNoise,
                              (uint32_t)k, (const double*)(smem + L::o_tab), z);
        else
          normal_quad<NZ>(C.seed, (uint32_t)((l * NQ + q) * 64 + lane), (uint32_t)t, kUNoise,
                          (uint32_t)k, z);
#pragma unroll
        for (int i = 0; i < NZ; ++i)
          if (4 * q + i < J) xi_l[(4 * q + i) * 64 + lane] = z[i];
      }
#pragma unroll
      for (int L = 0; L < R; ++L) {
        if (l == L) {
#pragma unroll
          for (int jj = 0; jj < J; ++jj) {
            const int j = lane + 64 * jj;
            const double Gv = j < n ? acc[jj][L] * cU : 0.0;
            gu2 = fma(Gv, Gv, gu2);
            acc[jj][L] = j < n ? sq * Gv / 2 + xi_l[jj * 64 + lane] : 0.0;    // :420 drive
          }
        }
      }
    }
  }
  if (C.diag) {
    gu2 = wave_sum(gu2);
    if (lane == 0) C.diag[(size_t)t * (1 + D) + 1 + k] = sqrt(gu2);
  }
  CSTAMP(4);
  SSTAMP(4);
  {
    constexpr int NN = 2 * R;
    constexpr int S0 = (7 * NN * NN > 64 * 8) ? 7 * NN * NN : 64 * 8;
    double* X0 = X;                          // expm scratch (7·NN²), reused for expm(−tA)
    double* Ec = X + S0;                     // E[:, 0:r]  (NN × R)
    double* Mg = Ec + NN * R;                // UᵀW, then Ag | Sg | nrm
    double* Ag = Mg + R * R;
    double* Sg = Ag + R * R;
    double* nr = Sg + R * R;
    wave_sync();                             // noise slots (aliasing X0) are consumed
    // proj (GPT_SGLD.jl:14-16): M = UᵀW, mom = W − U·Ms with Ms = (M + Mᵀ)/2; geod (:19-37)
    // needs A = Uᵀmom and S = momᵀmom.  With UᵀU = I, A = (M − Mᵀ)/2 and
    // S = G − MᵀMs − Ms·M + Ms·Ms for the drive's Gram G = WᵀW (the oracle's reference form
    // agrees to ≤ 1.2e-14 relative over whole trajectories, tests/test_oracle.py), so Uᵀmom
    // needs no pass over the rows.  M, then S = momᵀmom from a second pass after mom (M and G
    // from one pass spilled u into the batch loop, round 3).
#pragma unroll
    for (int a = 0; a < R; ++a) {
      double v[R];
#pragma unroll
      for (int bb = 0; bb < R; ++bb) {
        double s0 = 0.0;
#pragma unroll
        for (int jj = 0; jj < J; ++jj) s0 = fma(u[jj][a], acc[jj][bb], s0);
        v[bb] = s0;
      }
      wave_sum_to_lds<R>(v, Mg + a * R);
    }
    wave_sync();
    SSTAMP(5);
#pragma unroll
    for (int bb = 0; bb < R; ++bb) {
      double ms[R];
#pragma unroll
      for (int a = 0; a < R; ++a) ms[a] = Mg[a * R + bb] + Mg[bb * R + a];
#pragma unroll
      for (int jj = 0; jj < J; ++jj) {
        double s = 0.0;
#pragma unroll
        for (int a = 0; a < R; ++a) s = fma(u[jj][a], ms[a], s);
        acc[jj][bb] = acc[jj][bb] - s / 2;
      }
    }
      CSTAMP(5);
      SSTAMP(6);
      {
#pragma unroll
        for (int a = 0; a < R; ++a) {
          double v[R];
#pragma unroll
          for (int bb = 0; bb < R; ++bb) {
            double s1 = 0.0;
            if (bb >= a)
#pragma unroll
              for (int jj = 0; jj < J; ++jj) s1 = fma(acc[jj][a], acc[jj][bb], s1);
            v[bb] = s1;
          }
          wave_sum_to_lds<R>(v, Sg + a * R);    // S[a][b] valid for b >= a
        }
        wave_sync();
        for (int o = lane; o < R * R; o += 64) {
          const int i = o / R, b = o - i * R;
          Ag[o] = (Mg[o] - Mg[b * R + i]) / 2;
          if (i > b) Sg[o] = Sg[b * R + i];
        }
      }
      wave_sync();
      const double tt = sq;
      for (int o = lane; o < NN * NN; o += 64) {
        const int i = o / NN, j = o - i * NN;
        double v;
        if (i < R) v = j < R ? Ag[i * R + j] : -Sg[i * R + (j - R)];
        else v = j < R ? (i - R == j ? 1.0 : 0.0) : Ag[(i - R) * R + (j - R)];
        X0[o] = tt * v;
      }
      wave_sync();
      long long* xst = (CHAIN_SSTAMP && P.stamps && k == 0)
                           ? P.stamps + (size_t)(4 * gridDim.x + blockIdx.x) * kStamps : nullptr;
      const bool bad = wave_expm<NN>(X0, xst);
      SSTAMP(7);
      for (int o = lane; o < NN * R; o += 64) {
        const int a = o / R, l = o - a * R;
        Ec[o] = X0[NN * NN + a * NN + l];
      }
      wave_sync();
      double* X1 = X0;                        // expm(−tA) in the same scratch
      for (int o = lane; o < R * R; o += 64) X1[o] = -tt * Ag[o];
      wave_sync();
      wave_expm<R>(X1, xst ? xst + (size_t)gridDim.x * kStamps : nullptr);
      if (bad && lane == 0) flag[0] = 1;
      CSTAMP(6);
      SSTAMP(8);
      const double* mx = X1 + R * R;          // expm(−tA)
      // F = E[:,1:r]·expm(−tA) (NN × R, on the wave), then tmpU = [U mom]·F row by row
      // (GPT_SGLD.jl:35 with the two products associated the other way), then normalisation
      double* F = Mg;                         // grams are dead: reuse their slots
      wave_sync();
      for (int o = lane; o < NN * R; o += 64) {
        const int a = o / R, l = o - a * R;
        double s = 0.0;
#pragma unroll
        for (int c2 = 0; c2 < R; ++c2) s = fma(Ec[a * R + c2], mx[c2 * R + l], s);
        F[o] = s;
      }
      wave_sync();
      SSTAMP(9);
      // two passes with R×R halves of F in registers: U·F[0:r,:] in place, then += mom·F[r:2r,:]
      // (each F value read from LDS once per wave)
      {
        double Fh[R * R];
#pragma unroll
        for (int x = 0; x < R * R; ++x) Fh[x] = F[x];
#pragma unroll
        for (int jj = 0; jj < J; ++jj) {
          double o[R];
#pragma unroll
          for (int l = 0; l < R; ++l) o[l] = 0.0;
#pragma unroll
          for (int a = 0; a < R; ++a)
#pragma unroll
            for (int l = 0; l < R; ++l) o[l] = fma(u[jj][a], Fh[a * R + l], o[l]);
#pragma unroll
          for (int l = 0; l < R; ++l) u[jj][l] = o[l];
        }
      }
      SSTAMP(10);
      double nrm[R];
#pragma unroll
      for (int l = 0; l < R; ++l) nrm[l] = 0.0;
      {
        double Fh[R * R];
#pragma unroll
        for (int x = 0; x < R * R; ++x) Fh[x] = F[R * R + x];
#pragma unroll
        for (int jj = 0; jj < J; ++jj) {
#pragma unroll
          for (int a = 0; a < R; ++a)
#pragma unroll
            for (int l = 0; l < R; ++l) u[jj][l] = fma(acc[jj][a], Fh[a * R + l], u[jj][l]);
#pragma unroll
          for (int l = 0; l < R; ++l) nrm[l] = fma(u[jj][l], u[jj][l], nrm[l]);
        }
      }
      SSTAMP(11);
      wave_sum_to_lds<R>(nrm, nr);
      wave_sync();
      SSTAMP(12);
#pragma unroll
      for (int l = 0; l < R; ++l) {
        const double isc = 1.0 / sqrt(nr[l]);
#pragma unroll
        for (int jj = 0; jj < J; ++jj) u[jj][l] = u[jj][l] * isc;
      }
    }
    SSTAMP(13);
    if (CHAIN_PRIO) __builtin_amdgcn_s_setprio(0);
    if (CHAIN_STAMPS && P.stamps && lane == 0)   // per-wave arrival at the end-of-step barrier
    P.stamps[(size_t)blockIdx.x * kStamps + 8 + k] = (long long)__builtin_amdgcn_s_memtime();
  __syncthreads();                      // w_l, flag and the gradw partials are complete
    if (C.diag && tid == 0) {
      double s = 0.0;
      for (int w2 = 0; w2 < D; ++w2) s += misc[w2];
      C.diag[(size_t)t * (1 + D)] = sqrt(s);
    }
    if (flag[0]) {                        // NaN in the geodesic: the chain stops (:422-424)
      if (tid == 0) __hip_atomic_store(C.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    double* Uk = (t + 1 == tend) ? C.U + (size_t)n * R * k : nullptr;
    double* Us = (store && C.U_store) ? C.U_store + ((size_t)slot_s * D + k) * n * R : nullptr;
#pragma unroll
    for (int jj = 0; jj < J; ++jj) {
      const int j = lane + 64 * jj;
      if (j < n)
#pragma unroll
        for (int l = 0; l < R; ++l) {
          if (Uk) gptr_w(Uk)[j + (size_t)n * l] = u[jj][l];
          if (Us) gptr_w(Us)[j + (size_t)n * l] = u[jj][l];
        }
    }
    CSTAMP(7);
    SSTAMP(15);
    TSTAMP(2 + (int)(t - t0));
    if (++t >= tend) break;
    ord = ordn;
    Bt = Bn;
  }
#if CHAIN_TIMELINE == 2
  TSTAMP_ANY(2 + (int)(tend - 1 - t0));
#endif
}

// ------------------------------------------------------------------------------ host side
#define GPT_CHAIN_CFGS(X) \
  X(1, 1) X(1, 2) X(1, 4) X(1, 8) X(2, 1) X(2, 2) X(2, 4) X(2, 8) X(3, 1) X(3, 2) X(3, 4) X(3, 8) \
  X(4, 1) X(4, 2) X(4, 4) X(4, 8) X(5, 1) X(5, 2) X(5, 4) X(5, 8)

// Static LDS of chain_kernel<R, J, G>: the row staging buffer.
static int chain_wv(int D) { return D <= 4 ? 4 : kChainDMax; }
static size_t chain_static_lds(int J, int WV) { return 8 * (size_t)kChainBufs * WV * kChainG * 64 * J; }

static int chain_J(int n) { return n <= 64 ? 1 : (n <= 128 ? 2 : (n <= 256 ? 4 : (n <= 512 ? 8 : 0))); }

size_t chain_lds_bytes(int n, int D, int r, int Q, int m) {
  (void)n; (void)Q; (void)m;
  const bool w4 = chain_wv(D) == 4;
  switch (r) {
    case 1: return w4 ? ChainLds<1, kChainG, 4>::bytes : ChainLds<1, kChainG>::bytes;
    case 2: return w4 ? ChainLds<2, kChainG, 4>::bytes : ChainLds<2, kChainG>::bytes;
    case 3: return w4 ? ChainLds<3, kChainG, 4>::bytes : ChainLds<3, kChainG>::bytes;
    case 4: return w4 ? ChainLds<4, kChainG, 4>::bytes : ChainLds<4, kChainG>::bytes;
    case 5: return w4 ? ChainLds<5, kChainG, 4>::bytes : ChainLds<5, kChainG>::bytes;
    default: return (size_t)1 << 30;
  }
}

bool chain_supported(int n, int D, int r, int Q, int m, bool langevin, bool stiefel, int max_run) {
  if (max_run > kChainRun) return false;  // a run of core entries must fit its 64 slots
  if (!langevin || !stiefel) return false;   // SGD / Euclidean variants run on the grid engine
  if (D < 1 || D > kChainDMax || r < 1 || r > 5 || chain_J(n) == 0) return false;
  if (chain_J(n) >= 2 && (n & 1)) return false;   // 16-B row staging needs 16-B aligned rows
  if (Q > kChainQP || m > kChainMMax) return false;   // the fixed LDS carve's maxima
  const int NT = (Q + 63) / 64 * kChainG;
  if (NT > ((chain_J(n) >= 8 && D > 4) ? kChainTPW8 : kChainTasks) * D) return false;
  return chain_lds_bytes(n, D, r, Q, m) + chain_static_lds(chain_J(n), chain_wv(D)) <= 160 * 1024;
}

hipError_t launch_chain(const StepParams& P, const ChainDesc* chains, int nchains,
                        const long long* tbase, int t_local, int nsteps, hipStream_t st) {
  const int J = chain_J(P.n);
  const size_t lds = chain_lds_bytes(P.n, P.D, P.r, P.Q, P.m);
  dim3 grid(nchains), block(64 * P.D);
#define CASE_W(RR, JJ, WW)                                                                    \
  if (P.r == RR && J == JJ && (P.D <= 4) == (WW == 4)) {                                      \
    static std::atomic<uint64_t> attr{0};                                                     \
    hipError_t e = set_max_lds_once((const void*)chain_kernel<RR, JJ, kChainG, WW>,           \
                                    (int)(160 * 1024 - chain_static_lds(JJ, WW)), attr);      \
    if (e != hipSuccess) return e;                                                            \
    hipLaunchKernelGGL((chain_kernel<RR, JJ, kChainG, WW>), grid, block, lds, st, P, chains, tbase, \
                       t_local, nsteps);                                                      \
    return hipGetLastError();                                                                 \
  }
#define CASE(RR, JJ) CASE_W(RR, JJ, kChainDMax) CASE_W(RR, JJ, 4)
  GPT_CHAIN_CFGS(CASE)
#undef CASE
#undef CASE_W
  return hipErrorInvalidValue;
}

}  // namespace gpt
