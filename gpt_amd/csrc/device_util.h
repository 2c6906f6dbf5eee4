// Device building blocks shared by the step, prediction and init kernels (gfx950, wave64).
#pragma once
#include "gpt_internal.h"

namespace gpt {

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
// A pointer known to be wave-uniform, held in SGPRs.
template <class T>
__device__ __forceinline__ T* uni_ptr(T* p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (T*)(((unsigned long long)hi << 32) | lo);
}

// Lane id (0..63) from v_mbcnt, formed where it is used: nothing has to keep threadIdx.x (v0)
// alive, which long kernels would otherwise spill to scratch and reload — each reload a vmcnt(0)
// wait behind every load still in flight.
__device__ __forceinline__ int lane_id() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// Order LDS traffic between the lanes of ONE wave (no workgroup barrier).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- cross-lane exchanges without LDS (gfx950): v_permlane32/16_swap and DPP row/quad moves.
// xch<OFF>(a, b): lane λ returns a(λ) + [partner's b] where λ keeps a and sends b (partner of λ at
// "distance" OFF; for OFF = 4 the partner is the row_half_mirror lane, which also differs in bit 2).
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  // every control used here is a full permutation within a row, so no lane keeps its old
  // value: mov_dpp (old = undef) needs no zero-initialised destination
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int OFF>
__device__ __forceinline__ double dpp_partner(double v) {
  static_assert(OFF == 8 || OFF == 4 || OFF == 2 || OFF == 1, "DPP partner offset");
  if constexpr (OFF == 8) return dpp_d<0x128>(v);        // row_ror:8   (λ ^ 8 within a row)
  else if constexpr (OFF == 4) return dpp_d<0x141>(v);   // row_half_mirror (bit 2 flips)
  else if constexpr (OFF == 2) return dpp_d<0x4E>(v);    // quad_perm [2,3,0,1]
  else return dpp_d<0xB1>(v);                            // quad_perm [1,0,3,2]
}
// Pair exchange for the halving butterfly round at lane bit OFF: lanes with the bit clear keep
// `lo` and receive the partner's `lo`; lanes with it set keep `hi` and receive the partner's
// `hi`; returns keep + received.
template <int OFF>
__device__ __forceinline__ double pair_sum(double lo, double hi, int lane) {
  if constexpr (OFF == 32 || OFF == 16) {
    const long long a = __double_as_longlong(lo), b = __double_as_longlong(hi);
    unsigned al = (unsigned)a, ah = (unsigned)(a >> 32), bl = (unsigned)b, bh = (unsigned)(b >> 32);
    if constexpr (OFF == 32) {
      auto l2 = __builtin_amdgcn_permlane32_swap(al, bl, false, false);
      auto h2 = __builtin_amdgcn_permlane32_swap(ah, bh, false, false);
      al = l2[0]; bl = l2[1]; ah = h2[0]; bh = h2[1];
    } else {
      auto l2 = __builtin_amdgcn_permlane16_swap(al, bl, false, false);
      auto h2 = __builtin_amdgcn_permlane16_swap(ah, bh, false, false);
      al = l2[0]; bl = l2[1]; ah = h2[0]; bh = h2[1];
    }
    // lower half now holds (own lo, partner lo), upper half (partner hi, own hi)
    return __longlong_as_double(((long long)ah << 32) | al) +
           __longlong_as_double(((long long)bh << 32) | bl);
  } else {
    const bool up = (lane & OFF) != 0;
    const double send = up ? lo : hi;
    const double keep = up ? hi : lo;
    return keep + dpp_partner<OFF>(send);
  }
}
// v + partner's v (single-value round).
template <int OFF>
__device__ __forceinline__ double self_sum(double v, int lane) {
  if constexpr (OFF == 32 || OFF == 16) return pair_sum<OFF>(v, v, lane);
  else return v + dpp_partner<OFF>(v);
}

// Sum over aligned groups of 8 lanes (every lane of the group gets it): DPP only.
__device__ __forceinline__ double group8_sum(double v) {
  v += dpp_partner<1>(v);
  v += dpp_partner<2>(v);
  return v + dpp_partner<4>(v);     // row_half_mirror pairs the two quads of the group
}

// floor(x / d) for a divisor fixed over a loop: one v_mul_hi_u32 (and a select for d = 1)
// instead of the ~30 VALU instructions of a runtime integer division.  M = ⌈2³²/d⌉ =
// ⌊(2³² − 1)/d⌋ + 1 (one 32-bit division where the divisor is formed); exact whenever
// x·d ≤ 2³²: with x = qd + r, x·M/2³² = q + r/d + x·δ/(d·2³²), δ = M·d − 2³² < d, so the
// fraction stays below 1.  (d = 1 would need M = 2³²: m = 0 marks it.)
struct FastDiv {
  uint32_t m;
};
__device__ __forceinline__ FastDiv fast_div(int d) {
  return FastDiv{d == 1 ? 0u : 0xFFFFFFFFu / (uint32_t)d + 1u};
}
__device__ __forceinline__ int fdiv(int x, FastDiv f) {
  return f.m ? (int)__umulhi((uint32_t)x, f.m) : x;
}

// 1/x from the hardware reciprocal plus two Newton steps (within 1 ulp; 5 VALU ops instead of
// the ~10 of an IEEE division).
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

__device__ __forceinline__ double wave_sum(double v) {
  const int lane = threadIdx.x & 63;
  v = self_sum<32>(v, lane);
  v = self_sum<16>(v, lane);
  v = self_sum<8>(v, lane);
  v = self_sum<4>(v, lane);
  v = self_sum<2>(v, lane);
  return self_sum<1>(v, lane);
}

// max(v, partner's v) for the exchange pattern of wave_sum (permlane swaps across 32 / 16, DPP
// within rows) — no LDS round trip (a __shfl_xor of a double is two ds_bpermute per stage).
template <int OFF>
__device__ __forceinline__ double self_max(double v) {
  if constexpr (OFF == 32 || OFF == 16) {
    const long long a = __double_as_longlong(v);
    const unsigned lo = (unsigned)a, hi = (unsigned)(a >> 32);
    // swapping (v, v): each lane ends up with {own v, partner's v} in its two slots
    const auto l2 = OFF == 32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                              : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h2 = OFF == 32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                              : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const double x0 = __longlong_as_double(((long long)h2[0] << 32) | (unsigned)l2[0]);
    const double x1 = __longlong_as_double(((long long)h2[1] << 32) | (unsigned)l2[1]);
    return fmax(x0, x1);
  } else {
    return fmax(v, dpp_partner<OFF>(v));
  }
}

__device__ __forceinline__ double wave_max(double v) {
  v = self_max<32>(v);
  v = self_max<16>(v);
  v = self_max<8>(v);
  v = self_max<4>(v);
  v = self_max<2>(v);
  return self_max<1>(v);
}

// Sum of one value per thread over the workgroup; every thread gets the total.
// Uses red[0..kNW); deterministic order.
__device__ __forceinline__ double blk_sum(double v, double* red) {
  const int lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6);
  v = wave_sum(v);
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < kNW; ++w) s += red[w];
  __syncthreads();
  return s;
}

// Butterfly "transpose-reduce" across the 64 lanes of a wave: each lane starts with NV
// partial values; afterwards lane λ holds in v[0] the wave total of value (λ >> (6-P)),
// P = log2(NV).  Costs NV-1 exchanged doubles per lane instead of NV·6 for NV separate
// wave reductions.
template <int NV>
struct Butterfly {
  static constexpr int P = NV == 8 ? 3 : (NV == 16 ? 4 : (NV == 32 ? 5 : 6));
  // One halving round at a compile-time stage S (keeps every index static: no scratch).
  template <int S>
  __device__ __forceinline__ static void round(double (&v)[NV], int lane) {
    if constexpr (S < P) {
      constexpr int off = 32 >> S;
      constexpr int h = NV >> (S + 1);
#pragma unroll
      for (int u = 0; u < h; ++u) v[u] = pair_sum<off>(v[u], v[u + h], lane);
      round<S + 1>(v, lane);
    } else if constexpr (S < 6) {
      v[0] = self_sum<(32 >> S)>(v[0], lane);
      round<S + 1>(v, lane);
    }
  }
  __device__ __forceinline__ static void run(double (&v)[NV], int lane) { round<0>(v, lane); }
};

// Butterfly for any count NV of values (no padding to a power of two): at each of the 6 lane
// stages the NV values pair up (NV/2 exchanges; an odd last value is summed with its partner's
// copy and kept by both), leaving ⌈NV/2⌉.  For NV = 10 that is 47 VALU instructions against 63
// for Butterfly<16>.  obf_index gives the value a lane holds in v[0] afterwards and whether the
// lane is that value's one writer.
template <int N0, int NV, int S = 0>
__device__ __forceinline__ void obf_run(double (&v)[N0], int lane) {
  if constexpr (S < 6) {
    constexpr int off = 32 >> S, H = NV / 2;
#pragma unroll
    for (int u = 0; u < H; ++u) v[u] = pair_sum<off>(v[u], v[u + H], lane);
    if constexpr (NV & 1) v[H] = self_sum<off>(v[NV - 1], lane);
    obf_run<N0, H + (NV & 1), S + 1>(v, lane);
  }
}
template <int NV, int S = 0>
__device__ __forceinline__ void obf_index(int lane, int& idx, bool& wr) {
  if constexpr (S < 6) {
    constexpr int H = NV / 2;
    int j;
    bool w;
    obf_index<H + (NV & 1), S + 1>(lane, j, w);
    const bool bit = ((lane >> (5 - S)) & 1) != 0;
    if (j < H) { idx = bit ? j + H : j; wr = w; }
    else { idx = NV - 1; wr = w && !bit; }
  } else {
    idx = 0;
    wr = true;
  }
}

template <int R, int ICHX = 8>
struct RCfgX {
  static constexpr int ICH = (64 / R) < ICHX ? (64 / R) : ICHX;   // batch columns per wave pass
  static constexpr int NVR = ICH * R;
  static constexpr int NV = NVR <= 8 ? 8 : (NVR <= 16 ? 16 : (NVR <= 32 ? 32 : 64));
};
template <int R>
struct RCfg {
  static constexpr int ICH = (64 / R) < 8 ? (64 / R) : 8;   // batch columns per wave pass
  static constexpr int NVR = ICH * R;
  static constexpr int NV = NVR <= 8 ? 8 : (NVR <= 16 ? 16 : (NVR <= 32 ? 32 : 64));
};

// temp[l][i] = Σ_j phi[koff + row(i)*rstride + j] · U_l[l*NP + j]   (GPT_SGLD.jl:193-205)
// for i < Bt (rows from ordp, see batch_rows_lane).  Lanes stride over j (coalesced 512-B loads), wave w takes
// columns i = base + w + kNW·ii; partials are combined with one Butterfly per pass.
// U_l rows (stride NS) must be zero-padded for j in [n, NP).
// Row of batch column (base + lane) for every lane: one coalesced load per 64 columns; single
// rows are then broadcast with v_readlane (no per-column memory round trip).  ordp == nullptr
// means the identity map row = rowbase + column (prediction over a contiguous test range).
__device__ __forceinline__ int batch_rows_lane(const int32_t* ordp, int rowbase, int base, int Bt) {
  const int lane = threadIdx.x & 63;
  const int i = min(base + lane, Bt - 1);
  return ordp ? gptr(ordp)[i] : rowbase + i;
}

// Per-lane row addresses base + row·stride of a wave's rows, read back one lane at a time (a
// uniform lane index) as two v_readlane halves: a scalar address, so the row's load is the
// saddr + 32-bit lane offset form with no per-row 64-bit address arithmetic.
struct RowPtr {
  unsigned lo, hi;
  __device__ __forceinline__ RowPtr(const double* base, int row, long long stride) {
    const unsigned long long v = (unsigned long long)(base + (long long)row * stride);
    lo = (unsigned)v;
    hi = (unsigned)(v >> 32);
  }
  __device__ __forceinline__ const __attribute__((address_space(1))) double* at(int u) const {
    return (const __attribute__((address_space(1))) double*)(
        ((unsigned long long)__builtin_amdgcn_readlane(hi, u) << 32) |
        (unsigned)__builtin_amdgcn_readlane(lo, u));
  }
};

template <int R, class Out, int ICHX = 8>
__device__ __forceinline__ void phidotU_tile(const double* __restrict__ phi, long long koff,
                                             long long rstride, const int32_t* ordp, int rowbase,
                                             int Bt, int n, int NP, int NS, const double* U_l,
                                             Out out) {
  using C = RCfgX<R, ICHX>;
  const int lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6);
  constexpr int SH = 6 - Butterfly<C::NV>::P;
  for (int base = 0; base < Bt; base += kNW * C::ICH) {
    double v[C::NV];
#pragma unroll
    for (int u = 0; u < C::NV; ++u) v[u] = 0.0;
    const RowPtr rp(phi + koff, batch_rows_lane(ordp, rowbase, base, Bt), rstride);   // <= 64 columns
    const __attribute__((address_space(1))) double* rowp[C::ICH];
#pragma unroll
    for (int ii = 0; ii < C::ICH; ++ii) rowp[ii] = rp.at(min(wv + kNW * ii, 63));
    const int JS = NP >> 6;
#pragma unroll 4
    for (int s = 0; s < JS; ++s) {
      const int j = lane + 64 * s;
      const int jc = min(j, n - 1);
      double p[C::ICH];
#pragma unroll
      for (int ii = 0; ii < C::ICH; ++ii) p[ii] = rowp[ii][jc];
      double u[R];
#pragma unroll
      for (int l = 0; l < R; ++l) u[l] = U_l[l * NS + j];
#pragma unroll
      for (int ii = 0; ii < C::ICH; ++ii)
#pragma unroll
        for (int l = 0; l < R; ++l) v[ii * R + l] = fma(p[ii], u[l], v[ii * R + l]);
    }
    Butterfly<C::NV>::run(v, lane);
    const int vi = lane >> SH;
    if ((lane & ((1 << SH) - 1)) == 0 && vi < C::NVR) {
      const int ii = vi / R, l = vi - (vi / R) * R;
      const int i = base + wv + kNW * ii;
      if (i < Bt) out(l, i, v[0]);
    }
  }
}

// V-phase over a batch (lanes = core entries q, strided by 64; waves = batch columns
// i = base + wave + kNW·ii).  For each column, with NC = 1 + R values per column:
//   val[0]   = Σ_q w[q]·V[q,i],  V[q,i] = Π_k temp[k, I[q,k], i]      (GPT_SGLD.jl:208-230, k order)
//   val[1+l] = Σ_{q: I[q,kown]=l} w[q]·Π_{k≠kown} temp[k, I[q,k], i]   (:246-273 without the
//              division of computeU_phi — a leave-one-out product)
// reduced over q by one Butterfly per pass (no cross-wave traffic).  IT_l is I transposed
// (kk·Q + q, conflict-free per-lane reads).  out(comp, i, value) is called once per value.
template <int R>
struct VCfg {
  static constexpr int NC = 1 + R;
  static constexpr int ICV_MAX = (64 / NC) < 12 ? (64 / NC) : 12;   // columns per wave pass
  static constexpr int ICV_SMALL = ICV_MAX < 7 ? ICV_MAX : 7;      // batches <= 56 in one pass
};

template <int R, int ICV, class Out>
__device__ __forceinline__ void vphase_tile(const double* temp_l, int MP, const int* IT_l,
                                            const double* w_l, int Q, int D, int kown, int Bt,
                                            Out out) {
  constexpr int NC = 1 + R;
  const int lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6);
  for (int base = 0; base < Bt; base += kNW * ICV) {
    const int nii = min(ICV, (Bt - base - wv + kNW - 1) / kNW);
    int col[ICV];
#pragma unroll
    for (int ii = 0; ii < ICV; ++ii) col[ii] = min(base + wv + kNW * ii, Bt - 1);
    double v[64];
#pragma unroll
    for (int u = 0; u < 64; ++u) v[u] = 0.0;
    for (int q0 = 0; q0 < Q; q0 += 64) {
      const int q = q0 + lane;
      const bool ok = q < Q;
      const int qq = ok ? q : 0;
      const double wq = ok ? w_l[qq] : 0.0;
      const int lk = IT_l[kown * Q + qq];
      double vv[ICV], vk[ICV];
#pragma unroll
      for (int ii = 0; ii < ICV; ++ii) { vv[ii] = 1.0; vk[ii] = 1.0; }
      // k outer (same product order as computeV), the ICV column loads of one k in flight
      for (int kk = 0; kk < D; ++kk) {
        const double* row = temp_l + (kk * R + IT_l[kk * Q + qq]) * MP;
        double tv[ICV];
#pragma unroll
        for (int ii = 0; ii < ICV; ++ii) tv[ii] = row[col[ii]];
        if (kk != kown) {
#pragma unroll
          for (int ii = 0; ii < ICV; ++ii) { vv[ii] *= tv[ii]; vk[ii] *= tv[ii]; }
        } else {
#pragma unroll
          for (int ii = 0; ii < ICV; ++ii) vv[ii] *= tv[ii];
        }
      }
#pragma unroll
      for (int ii = 0; ii < ICV; ++ii) {
        v[ii * NC] = fma(wq, vv[ii], v[ii * NC]);
        const double cc = wq * vk[ii];
#pragma unroll
        for (int l = 0; l < R; ++l) v[ii * NC + 1 + l] += (l == lk) ? cc : 0.0;
      }
    }
    Butterfly<64>::run(v, lane);
    const int ii = lane / NC, comp = lane - ii * NC;
    if (ii < nii) out(comp, base + wv + kNW * ii, v[0]);
  }
}

// The V-phase of vphase_tile in the column-lane form (the step kernel's latency path): lanes =
// batch columns i = c0 + lane, waves = contiguous slices of the core entries q.  q is wave-uniform,
// so every temp read is one contiguous 512-B row segment (no gather, no transpose-reduce), and
// the LDS table entry of q (vphase_cols_tables, 16 ints) is three broadcast reads: the 8 temp row offsets
// of its factors — the D−1 factors k ≠ kown in k order, ones-row padding, the kown factor last —
// and I[q, kown].  val[1+l] gets the leave-one-out product, val[0] = that product · temp[kown]
// (the w block's table has all D factors in k order).  VPHASE_QU entries per pass (one measured
// fastest: the eight reads of one entry are in flight together, more entries only lengthen the
// pass).  The per-wave partial sums (NC per column) meet in vred (kNW·NC·64 doubles) and are
// summed in wave order.
#ifndef VPHASE_QU
#define VPHASE_QU 1          // core entries per pass of vphase_cols (1: 15.6 k cycles, 2: 16.8 k, 4: 17.5 k)
#endif
template <int R, bool WITHA, class Out>
__device__ __forceinline__ void vphase_cols(const double* temp_l, const int32_t* tab,
                                            const double* w_l, int Q, int Bt, double* vred,
                                            Out out) {
  constexpr int NC = WITHA ? 1 + R : 1;
  constexpr int QU = VPHASE_QU;
  const int lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6);
  const int Qw = (Q + kNW - 1) / kNW;
  const int qa = wv * Qw, qb = min(Q, qa + Qw);
  for (int c0 = 0; c0 < Bt; c0 += 64) {
    const double* tcol = temp_l + min(c0 + lane, Bt - 1);
    double f = 0.0, a[R];
#pragma unroll
    for (int l = 0; l < R; ++l) a[l] = 0.0;
    for (int q0 = qa; q0 < qb; q0 += QU) {
      double vk[QU], t7[QU], wq[QU];
      int lk[QU];
#pragma unroll
      for (int u = 0; u < QU; ++u) {
        const int q = min(q0 + u, qb - 1);             // past the slice: weight 0
        const int4 e0 = *(const int4*)(tab + 16 * q), e1 = *(const int4*)(tab + 16 * q + 4);
        wq[u] = q0 + u < qb ? w_l[q] : 0.0;
        const double t0 = tcol[e0.x], t1 = tcol[e0.y], t2 = tcol[e0.z], t3 = tcol[e0.w];
        const double t4 = tcol[e1.x], t5 = tcol[e1.y], t6 = tcol[e1.z];
        t7[u] = tcol[e1.w];
        vk[u] = ((((((t0 * t1) * t2) * t3) * t4) * t5) * t6);
        lk[u] = WITHA ? uni(tab[16 * q + 8]) : 0;
      }
#pragma unroll
      for (int u = 0; u < QU; ++u) {
        f = fma(wq[u], vk[u] * t7[u], f);
        if (WITHA) {
          const double cc = wq[u] * vk[u];
#pragma unroll
          for (int l = 0; l < R; ++l)
            if (l == lk[u]) a[l] += cc;
        }
      }
    }
    vred[wv * NC * 64 + lane] = f;
    if (WITHA) {
#pragma unroll
      for (int l = 0; l < R; ++l) vred[(wv * NC + 1 + l) * 64 + lane] = a[l];
    }
    __syncthreads();
    for (int o = threadIdx.x; o < NC * 64; o += kNT) {
      const int comp = o >> 6, ln = o & 63;
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < kNW; ++w) s += vred[(w * NC + comp) * 64 + ln];
      if (c0 + ln < Bt) out(comp, c0 + ln, s);
    }
    __syncthreads();
  }
}

// vphase_cols for a batch (slice) of at most 32 columns: the two half-waves take alternate core
// entries (lanes λ and λ + 32 hold the same column), so a wave walks its slice of q in half the
// passes; the halves' partial sums meet by one permlane swap (even-q sum + odd-q sum).  A's row
// differs between the halves, so it is selected per lane.
template <int R, bool WITHA, class Out>
__device__ __forceinline__ void vphase_cols_half(const double* temp_l, const int32_t* tab,
                                                 const double* w_l, int Q, int Bt, double* vred,
                                                 Out out) {
  constexpr int NC = WITHA ? 1 + R : 1;
  const int lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6), h = lane >> 5;
  const int Qw = (Q + kNW - 1) / kNW;
  const int qa = wv * Qw, qb = min(Q, qa + Qw);
  const double* tcol = temp_l + min(lane & 31, Bt - 1);
  double f = 0.0, a[R];
#pragma unroll
  for (int l = 0; l < R; ++l) a[l] = 0.0;
  for (int q0 = qa; q0 < qb; q0 += 2) {
    const bool ok = q0 + h < qb;
    const int q = ok ? q0 + h : q0;
    const int4 e0 = *(const int4*)(tab + 16 * q), e1 = *(const int4*)(tab + 16 * q + 4);
    const double wq = ok ? w_l[q] : 0.0;
    const double t0 = tcol[e0.x], t1 = tcol[e0.y], t2 = tcol[e0.z], t3 = tcol[e0.w];
    const double t4 = tcol[e1.x], t5 = tcol[e1.y], t6 = tcol[e1.z], t7 = tcol[e1.w];
    const double vk = ((((((t0 * t1) * t2) * t3) * t4) * t5) * t6);
    f = fma(wq, vk * t7, f);
    if (WITHA) {
      const int lk = tab[16 * q + 8];
      const double cc = wq * vk;
#pragma unroll
      for (int l = 0; l < R; ++l) a[l] += (l == lk) ? cc : 0.0;
    }
  }
  f = self_sum<32>(f, lane);
  vred[wv * NC * 64 + lane] = f;
  if (WITHA) {
#pragma unroll
    for (int l = 0; l < R; ++l) vred[(wv * NC + 1 + l) * 64 + lane] = self_sum<32>(a[l], lane);
  }
  __syncthreads();
  for (int o = threadIdx.x; o < NC * 64; o += kNT) {
    const int comp = o >> 6, ln = o & 63;
    double sacc = 0.0;
#pragma unroll
    for (int w = 0; w < kNW; ++w) sacc += vred[(w * NC + comp) * 64 + ln];
    if (ln < Bt) out(comp, ln, sacc);
  }
  __syncthreads();
}

// Gram products over j < n of LDS rows (stride NP), lanes = outputs, waves = j slices.
//  mode 0: out[a*R+b] = Σ_j X[a][j]·Y[b][j]                      (R² outputs)
//  mode 1: out[a*R+b] = Σ X[a]Y[b];  out[R²+a*R+b] = Σ Y[a]Y[b]   (2R² outputs)
//  mode 2: out[l] = Σ_j X[l][j]²                                   (R outputs)
template <int R>
__device__ __forceinline__ void blk_gram(const double* X, const double* Y, int NP, int n,
                                         int mode, double* out, double* red) {
  const int lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6);
  const int nout = mode == 0 ? R * R : (mode == 1 ? 2 * R * R : R);
  const int chunk = (n + kNW - 1) / kNW;
  const int j0 = wv * chunk, j1 = min(n, j0 + chunk);
  for (int o = lane; o < nout; o += 64) {
    const double* xa;
    const double* yb;
    if (mode == 2) { xa = X + o * NP; yb = xa; }
    else {
      const int oo = o < R * R ? o : o - R * R;
      const int a = oo / R, b = oo - a * R;
      xa = (o < R * R ? X : Y) + a * NP;
      yb = Y + b * NP;
    }
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int j = j0;
    for (; j + 8 <= j1; j += 8) {
      double x[8], y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) { x[u] = xa[j + u]; y[u] = yb[j + u]; }
      s0 = fma(x[0], y[0], s0); s1 = fma(x[1], y[1], s1); s2 = fma(x[2], y[2], s2); s3 = fma(x[3], y[3], s3);
      s0 = fma(x[4], y[4], s0); s1 = fma(x[5], y[5], s1); s2 = fma(x[6], y[6], s2); s3 = fma(x[7], y[7], s3);
    }
    for (; j < j1; ++j) s0 = fma(xa[j], yb[j], s0);
    red[wv * nout + o] = (s0 + s1) + (s2 + s3);
  }
  __syncthreads();
  for (int o = threadIdx.x; o < nout; o += kNT) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kNW; ++w) s += red[w * nout + o];
    out[o] = s;
  }
  __syncthreads();
}

// blk_gram's outputs formed row-parallel (R <= 8): thread t takes rows j = t + kNT·x, forms its
// products for every output, and each wave reduces them with one butterfly; the per-wave totals
// meet in red (kNW·NVG doubles) and are summed in wave order by the threads that own an output.
// Same modes and outputs as blk_gram; far shorter dependency chains than its lane-per-output
// j loops.  Two block barriers.
template <int R>
__device__ __forceinline__ void blk_gram_rows(const double* X, const double* Y, int NP, int n,
                                              int mode, double* out, double* red) {
  static_assert(R <= 8, "row-parallel Gram: R <= 8");
  constexpr int NVG = 2 * R * R <= 8 ? 8 : (2 * R * R <= 16 ? 16 : (2 * R * R <= 32 ? 32 : 64));
  const int lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6);
  const int nout = mode == 0 ? R * R : (mode == 1 ? 2 * R * R : R);
  double v[NVG];
#pragma unroll
  for (int x = 0; x < NVG; ++x) v[x] = 0.0;
  for (int j = threadIdx.x; j < n; j += kNT) {
    double xa[R], yb[R];
#pragma unroll
    for (int a = 0; a < R; ++a) { xa[a] = X[a * NP + j]; yb[a] = Y[a * NP + j]; }
    if (mode == 2) {
#pragma unroll
      for (int a = 0; a < R; ++a) v[a] = fma(xa[a], xa[a], v[a]);
    } else {
#pragma unroll
      for (int a = 0; a < R; ++a)
#pragma unroll
        for (int b = 0; b < R; ++b) {
          v[a * R + b] = fma(xa[a], yb[b], v[a * R + b]);
          if (2 * R * R <= NVG && mode == 1) v[R * R + a * R + b] = fma(yb[a], yb[b], v[R * R + a * R + b]);
        }
    }
  }
  constexpr int SH = 6 - Butterfly<NVG>::P;
  Butterfly<NVG>::run(v, lane);
  const int vi = lane >> SH;
  if ((lane & ((1 << SH) - 1)) == 0 && vi < nout) red[wv * NVG + vi] = v[0];
  __syncthreads();
  for (int o = threadIdx.x; o < nout; o += kNT) {
    double sacc = 0.0;
#pragma unroll
    for (int w = 0; w < kNW; ++w) sacc += red[w * NVG + o];
    out[o] = sacc;
  }
  __syncthreads();
}

// ---------------------------------------------------------------- small dense algebra (1 wave)
// Padé numerator coefficients b_0..b_m of degrees 3, 5, 7, 9 (Higham 2005, Julia Base expm!).
__constant__ double kPade[4][10] = {
    {120.0, 60.0, 12.0, 1.0},
    {30240.0, 15120.0, 3360.0, 420.0, 30.0, 1.0},
    {17297280.0, 8648640.0, 1995840.0, 277200.0, 25200.0, 1512.0, 56.0, 1.0},
    {17643225600.0, 8821612800.0, 2075673600.0, 302702400.0, 30270240.0, 2162160.0, 110880.0,
     3960.0, 90.0, 1.0}};

// NN is compile-time so every inner product is unrolled with all its LDS reads in flight.
// wave_mm takes the register-blocked form from this size up (NN = 10, the r = 5 geodesic: 25
// lanes with 2 × 2 blocks, one pass instead of two passes of 64 + 36 lane-outputs)
#ifndef GPT_WAVE_MM_BLOCKED
#define GPT_WAVE_MM_BLOCKED 10
#endif
constexpr int kWaveMmBlocked = GPT_WAVE_MM_BLOCKED;
template <int NN>
__device__ __forceinline__ void wave_mm(const double* A, const double* B, double* C) {
  const int lane = threadIdx.x & 63;
  if constexpr (NN >= kWaveMmBlocked) {
    // register-blocked: lane (bi, bj) of an NB × NB grid owns a BS × BS block of C, so each LDS
    // value read feeds BS FMAs (NN = 40: 5 × 5 blocks, 0.4 reads per FMA instead of 2).  Every
    // output is still Σ_t A[i,t]·B[t,j] accumulated in t order — the same doubles as below.
    constexpr int BS = (NN + 7) / 8, NB = (NN + BS - 1) / BS;
    if (lane < NB * NB) {
      const int i0 = (lane / NB) * BS, j0 = (lane % NB) * BS;
      double acc[BS][BS];
#pragma unroll
      for (int x = 0; x < BS; ++x)
#pragma unroll
        for (int y = 0; y < BS; ++y) acc[x][y] = 0.0;
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
          for (int y = 0; y < BS; ++y) acc[x][y] = fma(a[x], b[y], acc[x][y]);
      }
#pragma unroll
      for (int x = 0; x < BS; ++x)
#pragma unroll
        for (int y = 0; y < BS; ++y)
          if (i0 + x < NN && j0 + y < NN) C[(i0 + x) * NN + j0 + y] = acc[x][y];
    }
    wave_sync();
    return;
  }
  for (int o = lane; o < NN * NN; o += 64) {
    const int i = o / NN, j = o - i * NN;
    double a[NN], b[NN];
#pragma unroll
    for (int t = 0; t < NN; ++t) { a[t] = A[i * NN + t]; b[t] = B[t * NN + j]; }
    double s = 0.0;
#pragma unroll
    for (int t = 0; t < NN; ++t) s = fma(a[t], b[t], s);
    C[o] = s;
  }
  wave_sync();
}

// Solve M·X = X0 in place (X holds X0 on entry), partial pivoting (LAPACK gesv semantics:
// largest |pivot|, first index on ties, multipliers scaled by 1/pivot).
// Large systems (NN >= 16: the 2r x 2r Padé solve at r >= 8) are compiled out of line so the
// elimination gets its own register allocation instead of the caller's, which at r = 20 is already
// at the VGPR limit and spilled the block buffers to scratch inside the row loop.
template <int NN>
__device__ __forceinline__ void wave_solve_body(double* M, double* X, long long* st);
template <int NN>
__device__ __noinline__ void wave_solve_ool(double* M, double* X, long long* st) {
  __builtin_assume(__builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void*)M));
  __builtin_assume(__builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void*)X));
  wave_solve_body<NN>(M, X, st);               // M, X are LDS (see wave_expm): ds_*, not flat_*
}
template <int NN>
__device__ __forceinline__ void wave_solve(double* M, double* X, long long* st = nullptr) {
  if constexpr (NN >= 16) wave_solve_ool<NN>(M, X, st);
  else wave_solve_body<NN>(M, X, st);
}
template <int NN>
__device__ __forceinline__ void wave_solve_body(double* M, double* X, long long* st) {
  const int lane = threadIdx.x & 63;
  // strictly column diagonally dominant M: partial pivoting never swaps (dominance survives
  // elimination), so the pivot search can be skipped with identical results
  bool dd = true;
  if (lane < NN) {
    double off = 0.0;
    for (int i = 0; i < NN; ++i)
      if (i != lane) off += fabs(M[i * NN + lane]);
    dd = fabs(M[lane * NN + lane]) > off;
  }
  const bool nopiv = __all(dd);
  for (int c = 0; c < NN; ++c) {
    int bi = c;
    if (!nopiv) {
      const double mine = (lane >= c && lane < NN) ? fabs(M[lane * NN + c]) : -1.0;
      const double best = wave_max(mine);
      const unsigned long long hit = __ballot(mine == best && lane >= c && lane < NN);
      bi = hit ? (int)__ffsll((long long)hit) - 1 : c;
    }
    if (bi != c) {
      for (int col = lane; col < NN; col += 64) {
        double t0 = M[c * NN + col]; M[c * NN + col] = M[bi * NN + col]; M[bi * NN + col] = t0;
        double t1 = X[c * NN + col]; X[c * NN + col] = X[bi * NN + col]; X[bi * NN + col] = t1;
      }
      wave_sync();
    }
    const double rp = 1.0 / M[c * NN + c];
    // lanes over the columns of [M | X] right of the pivot, rows in a uniform loop: the
    // multiplier M[rr,c]·rp is a broadcast read and no lane divides indices (same arithmetic
    // per element as a lanes-over-elements sweep)
    const int mcols = NN - c - 1, wcols = mcols + NN;
    // a lane owns column cc = lane and, when [M | X] has more than 64 columns right of the pivot,
    // cc + 64 too; both are updated in the same pass over the rows, which go in blocks of 8 with
    // all reads of a block issued before its writes (the columns and the multiplier column never
    // alias, but the compiler cannot know: one row at a time would serialise on LDS latency)
    if (lane < wcols) {
      const int cb = lane + 64;
      const bool two = cb < wcols;
      double* pa = lane < mcols ? M + (c + 1 + lane) : X + (lane - mcols);
      double* pb = two ? (cb < mcols ? M + (c + 1 + cb) : X + (cb - mcols)) : pa;
      const double piva = pa[c * NN], pivb = pb[c * NN];
      for (int r0 = c + 1; r0 < NN; r0 += 8) {
        double fv[8], ca[8], cbv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int rr = min(r0 + u, NN - 1);
          fv[u] = M[rr * NN + c];
          ca[u] = pa[rr * NN];
          cbv[u] = pb[rr * NN];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const double f = fv[u] * rp;
          if (r0 + u < NN) {
            pa[(r0 + u) * NN] = ca[u] - f * piva;
            if (two) pb[(r0 + u) * NN] = cbv[u] - f * pivb;
          }
        }
      }
    }
    wave_sync();
  }
  if (st && lane == 0) st[15] = (long long)__builtin_amdgcn_s_memtime();   // diagnostic stamp
  // back substitution: lanes over columns of X; the row of M and the solved rows stay in regs
  for (int col = lane; col < NN; col += 64) {
    double x[NN];
#pragma unroll
    for (int t = 0; t < NN; ++t) x[t] = X[t * NN + col];
#pragma unroll
    for (int c = NN - 1; c >= 0; --c) {
      double s = x[c];
#pragma unroll
      for (int t = c + 1; t < NN; ++t) s -= M[c * NN + t] * x[t];
      x[c] = s / M[c * NN + c];
    }
#pragma unroll
    for (int t = 0; t < NN; ++t) X[t * NN + col] = x[t];
  }
  wave_sync();
}

// Wave-wide sums of NV per-lane values written to dst[0..NV) (and, with dst2, values NV..2NV-1
// to dst2[0..NV)); the caller orders the LDS writes with wave_sync().
template <int NV>
__device__ __forceinline__ void wave_sum_to_lds(double (&v)[NV], double* dst) {
  constexpr int NB = NV <= 8 ? 8 : (NV <= 16 ? 16 : (NV <= 32 ? 32 : 64));
  const int lane = lane_id();
  double b[NB];
#pragma unroll
  for (int x = 0; x < NB; ++x) b[x] = x < NV ? v[x] : 0.0;
  Butterfly<NB>::run(b, lane);
  constexpr int SH = 6 - Butterfly<NB>::P;
  const int vi = lane >> SH;
  if ((lane & ((1 << SH) - 1)) == 0 && vi < NV) dst[vi] = b[0];
}
template <int NV>
__device__ __forceinline__ void wave_sum_to_lds(double (&v)[2 * NV], double* dst, double* dst2) {
  constexpr int NB = 2 * NV <= 8 ? 8 : (2 * NV <= 16 ? 16 : (2 * NV <= 32 ? 32 : 64));
  const int lane = lane_id();
  double b[NB];
#pragma unroll
  for (int x = 0; x < NB; ++x) b[x] = x < 2 * NV ? v[x] : 0.0;
  Butterfly<NB>::run(b, lane);
  constexpr int SH = 6 - Butterfly<NB>::P;
  const int vi = lane >> SH;
  if ((lane & ((1 << SH) - 1)) == 0 && vi < 2 * NV) {
    if (vi < NV) dst[vi] = b[0];
    else dst2[vi - NV] = b[0];
  }
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Solve M·X = X0 (X holds X0) for column diagonally dominant M: Gaussian elimination with
// partial pivoting provably never swaps rows there, so the arithmetic of wave_solve is
// reproduced without the pivot searches.  Lanes own columns of [M | X] in registers; pivot
// rows and multipliers are broadcast with v_readlane (no LDS round trips).  Returns false
// (nothing written) when M is not diagonally dominant — the caller then pivots.
template <int NN>
__device__ __forceinline__ bool wave_solve_dd(const double* M, double* X) {
  const int lane = threadIdx.x & 63;
  bool dd = true;
  if (lane < NN) {
    double off = 0.0;
#pragma unroll
    for (int i = 0; i < NN; ++i)
      if (i != lane) off += fabs(M[i * NN + lane]);
    dd = fabs(M[lane * NN + lane]) > off;
  }
  if (!__all(dd)) return false;
  double col[NN];
#pragma unroll
  for (int i = 0; i < NN; ++i) {
    const int c = lane < NN ? lane : lane - NN;
    col[i] = lane < NN ? M[i * NN + c] : (lane < 2 * NN ? X[i * NN + c] : 0.0);
  }
  // the reciprocal of each pivot (Newton-refined, within 1 ulp) scales both the multipliers and
  // the back substitution: no division on the elimination's critical path
  double rpv[NN];
#pragma unroll
  for (int p = 0; p < NN; ++p) {              // forward elimination (getrf + L solve)
    const double rp = rcp_nr(readlane_d(col[p], p));
    rpv[p] = rp;
#pragma unroll
    for (int i = p + 1; i < NN; ++i) {
      const double f = readlane_d(col[i], p) * rp;
      col[i] -= f * col[p];
    }
  }
  const bool xl = lane >= NN;                 // only the right-hand-side lanes back-substitute
#pragma unroll
  for (int k = NN - 1; k >= 0; --k) {         // back substitution, column-oriented (trsm)
    double u[NN];
#pragma unroll
    for (int i = 0; i < k; ++i) u[i] = readlane_d(col[i], k);    // U[0..k-1][k] from lane k
    if (xl) {
      col[k] = col[k] * rpv[k];
#pragma unroll
      for (int i = 0; i < k; ++i) col[i] -= col[k] * u[i];
    }
  }
  wave_sync();
  if (lane >= NN && lane < 2 * NN) {
#pragma unroll
    for (int i = 0; i < NN; ++i) X[i * NN + lane - NN] = col[i];
  }
  wave_sync();
  return true;
}

// wave_solve_dd for 32 < NN <= 64, where [M | X] has more columns than the wave has lanes: the
// factorisation and the right-hand sides go in two passes of one column per lane, with the
// factors kept in LDS between them (F, NN² doubles: multipliers below the diagonal, U above it,
// the Newton-refined pivot reciprocals on it).  Every column sees exactly the operations of
// wave_solve_dd (the pivot lane's multipliers are the doubles the other lanes would form).
template <int NN>
__device__ __noinline__ bool wave_solve_dd2(const double* Mg, double* Xg, double* Fg) {
  static_assert(NN > 32 && NN <= 64, "two-pass register LU");
  typedef __attribute__((address_space(3))) double lds_d;   // LDS arguments: ds_*, not flat_*
  const lds_d* M = (const lds_d*)Mg;
  lds_d* X = (lds_d*)Xg;
  lds_d* F = (lds_d*)Fg;
  const int lane = lane_id();
  bool dd = true;
  if (lane < NN) {
    double off = 0.0;
#pragma unroll
    for (int i = 0; i < NN; ++i)
      if (i != lane) off += fabs(M[i * NN + lane]);
    dd = fabs(M[lane * NN + lane]) > off;
  }
  if (!__all(dd)) return false;
  double col[NN];
#pragma unroll
  for (int i = 0; i < NN; ++i) col[i] = M[i * NN + (lane < NN ? lane : 0)];
#pragma unroll
  for (int p = 0; p < NN; ++p) {              // getrf: the pivot lane writes its multipliers
    if (lane == p) {
      const double rp = rcp_nr(col[p]);
      F[p * NN + p] = rp;
#pragma unroll
      for (int i = p + 1; i < NN; ++i) F[i * NN + p] = col[i] * rp;
    }
    wave_sync();
#pragma unroll
    for (int i = p + 1; i < NN; ++i) col[i] -= F[i * NN + p] * col[p];
  }
#pragma unroll
  for (int i = 0; i < NN - 1; ++i)            // U above the diagonal: column k from lane k
    if (i < lane && lane < NN) F[i * NN + lane] = col[i];
  wave_sync();
#pragma unroll
  for (int i = 0; i < NN; ++i) col[i] = X[i * NN + (lane < NN ? lane : 0)];
  // Each step's factor reads hang off an offset that depends on the previous step's result: the
  // scheduler cannot issue all NN² reads up front (which spilled ~1 200 values at 256 VGPRs).
#pragma unroll
  for (int p = 0; p < NN; ++p) {              // L solve
    int zo = 0;
    asm volatile("" : "+v"(zo) : "v"(col[p]));
#pragma unroll
    for (int i = p + 1; i < NN; ++i) col[i] -= F[zo + i * NN + p] * col[p];
  }
#pragma unroll
  for (int k = NN - 1; k >= 0; --k) {         // back substitution
    int zo = 0;
    asm volatile("" : "+v"(zo) : "v"(col[k]));
    col[k] = col[k] * F[zo + k * NN + k];
#pragma unroll
    for (int i = 0; i < k; ++i) col[i] -= col[k] * F[zo + i * NN + k];
  }
  wave_sync();
  if (lane < NN) {
#pragma unroll
    for (int i = 0; i < NN; ++i) X[i * NN + lane] = col[i];
  }
  wave_sync();
  return true;
}

// expm(A) for an NN×NN matrix held in S[0..NN²) (row-major; overwritten).  Padé
// scaling-and-squaring of Julia Base 0.3 expm! (Higham 2005; thresholds 0.015/0.25/0.95/2.1,
// 13th order above, θ13 = 5.4).  Scratch S: 7 NN² doubles; the result is left at S + NN².
// Returns true if the result contains a NaN (the geod bail-out of GPT_SGLD.jl:23-26).
// kRegLU2 = false keeps the LDS GEPP for 32 < NN <= 64 (callers at a 128-VGPR budget, where the
// two-pass register LU spills).
template <int NN, bool kRegLU2 = true>
__device__ bool wave_expm(double* S, long long* st = nullptr) {
  // S is LDS (every caller's expm scratch): said so, the compiler infers the local address space
  // for everything derived from it and emits ds_* instead of flat_* (this function is compiled
  // out of line, where the caller's address space is not visible)
  __builtin_assume(__builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void*)S));
  const int lane = threadIdx.x & 63;
  // diagnostic stamps (slots 11-14 of the caller's stamp row; grid engine stamp builds only)
#define GPT_XST(i)                                                        \
  do {                                                                    \
    if (st && lane == 0) st[i] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
  GPT_XST(11);
  constexpr int q = NN * NN;
  double* A = S;
  double* A2 = S + q;
  double* A4 = S + 2 * q;
  double* A6 = S + 3 * q;
  double* U = S + 4 * q;
  double* V = S + 5 * q;
  double* T = S + 6 * q;
  double cs = 0.0;
  if (lane < NN) {
#pragma unroll
    for (int i = 0; i < NN; ++i) cs += fabs(A[i * NN + lane]);
  }
  // a non-finite ‖A‖₁ (an Inf or NaN entry): the oracle's NaN result (Julia's expm! would throw at
  // ceil(Int, log2(nA/5.4))), i.e. geod's bail-out; wave_max (fmax) alone would drop a NaN column
  if (__any(!(cs <= 1.79769313486231570e308))) return true;
  const double nA = wave_max(cs);
  int si = 0;
  if (nA <= 2.1) {
    const int deg = nA > 0.95 ? 9 : (nA > 0.25 ? 7 : (nA > 0.015 ? 5 : 3));
    if (st && lane == 0) st[10] = deg;
    const double* C = kPade[(deg - 3) / 2];   // wave-uniform: scalar loads from constant memory
    wave_mm<NN>(A, A, A2);
    const double c0 = C[0], c1 = C[1];
    for (int o = lane; o < q; o += 64) {
      const double id = (o / NN == o - (o / NN) * NN) ? 1.0 : 0.0;
      T[o] = id;
      U[o] = c1 * id;
      V[o] = c0 * id;
    }
    wave_sync();
    for (int kk = 1; kk <= (deg - 1) / 2; ++kk) {
      if (kk > 1) wave_mm<NN>(T, A2, A4);   // P = P·A2 (A4 is free scratch here); P1 = A2
      const double* Pk = kk > 1 ? A4 : A2;
      const double cu = C[2 * kk + 1], cv = C[2 * kk];
      for (int o = lane; o < q; o += 64) {
        const double p = Pk[o];
        T[o] = p;
        U[o] = U[o] + cu * p;
        V[o] = V[o] + cv * p;
      }
      wave_sync();
    }
    wave_mm<NN>(A, U, A6);
    for (int o = lane; o < q; o += 64) U[o] = A6[o];
    wave_sync();
  } else {
    // as many squarings as Julia's expm! takes (no cap; ‖A‖₁ <= DBL_MAX bounds si by 1022)
    const double s = log2(nA / 5.4);
    si = (s > 0.0) ? (int)ceil(s) : 0;
    if (st && lane == 0) st[10] = 13 + 100 * si;
    if (si > 0) {
      const double sc = ldexp(1.0, -si);
      for (int o = lane; o < q; o += 64) A[o] *= sc;
      wave_sync();
    }
    constexpr double c[14] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
                              1187353796428800.0, 129060195264000.0, 10559470521600.0,
                              670442572800.0, 33522128640.0, 1323241920.0, 40840800.0, 960960.0,
                              16380.0, 182.0, 1.0};
    wave_mm<NN>(A, A, A2);
    wave_mm<NN>(A2, A2, A4);
    wave_mm<NN>(A2, A4, A6);
    for (int o = lane; o < q; o += 64) T[o] = c[13] * A6[o] + c[11] * A4[o] + c[9] * A2[o];
    wave_sync();
    wave_mm<NN>(A6, T, V);               // V used as scratch for A6·inner
    for (int o = lane; o < q; o += 64) {
      const double id = (o / NN == o - (o / NN) * NN) ? 1.0 : 0.0;
      V[o] = V[o] + c[7] * A6[o] + c[5] * A4[o] + c[3] * A2[o] + c[1] * id;
      T[o] = c[12] * A6[o] + c[10] * A4[o] + c[8] * A2[o];
    }
    wave_sync();
    wave_mm<NN>(A, V, U);                // U = A·(A6·inner + …)
    wave_mm<NN>(A6, T, V);               // V = A6·(…)
    for (int o = lane; o < q; o += 64) {
      const double id = (o / NN == o - (o / NN) * NN) ? 1.0 : 0.0;
      V[o] = V[o] + c[6] * A6[o] + c[4] * A4[o] + c[2] * A2[o] + c[0] * id;
    }
    wave_sync();
  }
  GPT_XST(12);
  double* M = A4;      // dead from here on
  double* X = A2;
  for (int o = lane; o < q; o += 64) {
    M[o] = V[o] - U[o];
    X[o] = V[o] + U[o];
  }
  wave_sync();
  bool solved = false;
  if constexpr (2 * NN <= 64) solved = wave_solve_dd<NN>(M, X);
  else if constexpr (kRegLU2 && NN <= 64) solved = wave_solve_dd2<NN>(M, X, U);   // U, V dead here
  if (!solved) wave_solve<NN>(M, X, st);
  GPT_XST(13);
  for (int z = 0; z < si; ++z) {
    wave_mm<NN>(X, X, T);
    for (int o = lane; o < q; o += 64) X[o] = T[o];
    wave_sync();
  }
  GPT_XST(14);
#undef GPT_XST
  bool bad = false;
  for (int o = lane; o < q; o += 64) bad |= (X[o] != X[o]);
  return __any(bad);
}

}  // namespace gpt
