// Shared device/host helpers for libgptsgld: Philox4x32-10 streams, wave reductions.
//
// The Philox stream layout is the framework's RNG contract (see oracle/philox.py for the
// table).  It replaces Julia's global MersenneTwister draws at GPT_SGLD.jl:357-420; the
// consumption points are the reference's, the bits are ours.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GPT_HD __host__ __device__ __forceinline__
#include "fastmath.h"

namespace gpt {

enum Stream : uint32_t {
  kWInit = 1, kUInit = 2, kPerm = 3, kWNoise = 4, kUNoise = 5,
  kThetaInit = 6, kThetaNoise = 7, kSampleNZ = 8, kFeatZ = 9, kFeatB = 10,
  kTgpUInit = 11, kTgpI = 12, kTgpWNoise = 13, kTgpUNoise = 14,
  kGmcP = 15, kGmcMom = 16, kGmcU = 17,
  kCfUVInit = 18, kCfWNoise = 19, kCfUVNoise = 20,
  kCfgInit = 21, kCfgU = 22, kCfgV = 23, kCfgW = 24
};

struct U4 { uint32_t x, y, z, w; };

GPT_HD U4 philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
#if defined(__HIP_DEVICE_COMPILE__)
    // three-input xor in one v_bitop3_b32 (gfx950; truth table 0x96)
    const uint32_t n0 = __builtin_amdgcn_bitop3_b32(hi1, c1, k0, 0x96);
    const uint32_t n2 = __builtin_amdgcn_bitop3_b32(hi0, c3, k1, 0x96);
#else
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
#endif
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  return U4{c0, c1, c2, c3};
}

GPT_HD double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6) + 0.5) * (1.0 / 9007199254740992.0);
}

__constant__ double kFmCoef[31] = GPT_FM_COEF;

// The Box–Muller coefficient table behind a pointer the compiler cannot see through: the
// coefficients are scalar-loaded where used rather than hoisted into registers.
__device__ __forceinline__ const __attribute__((address_space(4))) double* fm_coef() {
  const __attribute__((address_space(4))) double* c =
      (const __attribute__((address_space(4))) double*)kFmCoef;
  asm volatile("" : "+s"(c));
  return c;
}

// Element e of normal stream (c1, c2, c3): Box–Muller on the block at c0 = e>>1.
// (log / sincos(2πu) from fastmath.h; host-side draws use libm in capi.hip.)
__device__ __forceinline__ double normal_at(uint64_t seed, uint32_t e, uint32_t c1, uint32_t c2,
                                            uint32_t c3) {
  const U4 x = philox4x32(e >> 1, c1, c2, c3, seed);
  const double u1 = u53(x.x, x.y), u2 = u53(x.z, x.w);
  const auto c = fm_coef();
  const double rad = fm_sqrt_pos(-2.0 * fm_log_c(u1, c));
  double sn, cs;
  fm_sincos_2pi_c(u2, sn, cs, c);
  return (e & 1u) ? rad * sn : rad * cs;
}

// Both Box–Muller outputs of the block at c0 (elements 2·c0 and 2·c0+1 of the stream).
__device__ __forceinline__ void normal_pair(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2,
                                            uint32_t c3, double& z0, double& z1) {
  const U4 x = philox4x32(c0, c1, c2, c3, seed);
  const double u1 = u53(x.x, x.y), u2 = u53(x.z, x.w);
  const auto c = fm_coef();
  const double rad = fm_sqrt_pos(-2.0 * fm_log_c(u1, c));
  double sn, cs;
  fm_sincos_2pi_c(u2, sn, cs, c);
  z0 = rad * cs;
  z1 = rad * sn;
}

// U-noise contract (oracle/philox.py, U_NOISE): rows of the n×r noise matrix of one dimension
// come in blocks of 64 (row j = λ + 64·b); the Philox block at
//   c0 = (l·NQ + q)·64 + λ,   NQ = ⌈⌈n/64⌉/4⌉,
// gives column l of rows λ + 64·(4q + i), i = 0..3, as two Box–Muller pairs of 32-bit uniforms:
//   (z0, z1) = √(−2 ln u(x0))·(cos 2πu(x1), sin 2πu(x1)),  (z2, z3) likewise from (x2, x3),
//   u(x) = (x + ½)·2⁻³².  Rows ≥ n are dropped.
// One Philox call feeds four normals, and a wave whose lane λ owns rows λ + 64·b (the chain
// engine) draws exactly its own elements.
GPT_HD int unoise_nq(int n) { return ((n + 63) / 64 + 3) / 4; }
GPT_HD double u32u(uint32_t x) { return ((double)x + 0.5) * (1.0 / 4294967296.0); }

// NZ = 4: both pairs; NZ = 2: the first pair only (blocks 4q+2, 4q+3 past the last row block).
template <int NZ>
__device__ __forceinline__ void normal_quad(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2,
                                            uint32_t c3, double* z) {
  const U4 x = philox4x32(c0, c1, c2, c3, seed);
  const auto c = fm_coef();
  {
    const double rad = fm_sqrt_pos(-2.0 * fm_log_c(u32u(x.x), c));
    double sn, cs;
    fm_sincos_2pi_c(u32u(x.y), sn, cs, c);
    z[0] = rad * cs;
    z[1] = rad * sn;
  }
  if constexpr (NZ == 4) {
    const double rad = fm_sqrt_pos(-2.0 * fm_log_c(u32u(x.z), c));
    double sn, cs;
    fm_sincos_2pi_c(u32u(x.w), sn, cs, c);
    z[2] = rad * cs;
    z[3] = rad * sn;
  }
}

// normal_quad with the angles from fm_sincos_tab2 (two 16-entry tables in LDS, filled by
// sincos_tab_fill): the same streams to within 3 ulp
template <int NZ>
__device__ __forceinline__ void normal_quad_tab(uint64_t seed, uint32_t c0, uint32_t c1,
                                                uint32_t c2, uint32_t c3, const double* tab,
                                                double* z) {
  const U4 x = philox4x32(c0, c1, c2, c3, seed);
  const auto c = fm_coef();
  {
    const double rad = fm_sqrt_pos(-2.0 * fm_log_c(u32u(x.x), c));
    double sn, cs;
    fm_sincos_tab2(x.y, tab, sn, cs, c);
    z[0] = rad * cs;
    z[1] = rad * sn;
  }
  if constexpr (NZ == 4) {
    const double rad = fm_sqrt_pos(-2.0 * fm_log_c(u32u(x.z), c));
    double sn, cs;
    fm_sincos_tab2(x.w, tab, sn, cs, c);
    z[2] = rad * cs;
    z[3] = rad * sn;
  }
}
// (sin, cos)(2πj/16) into tab[2j], tab[2j + 1] and (sin, cos)(2πj/256) into tab[32 + 2j],
// tab[33 + 2j], j < 16 (fm_sincos_tab2)
__device__ __forceinline__ void sincos_tab_fill(double* tab, int tid, int nth) {
  const auto c = fm_coef();
  for (int i = tid; i < 32; i += nth) {
    double sn, cs;
    fm_sincos_2pi_c((double)(i & 15) * (i < 16 ? 1.0 / 16.0 : 1.0 / 256.0), sn, cs, c);
    tab[2 * i] = sn;
    tab[2 * i + 1] = cs;
  }
}

// Global-address-space view of a pointer (global_load/global_store instead of flat_*, which
// would also count against lgkmcnt and serialise behind LDS traffic).
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gptr(const T* p) {
  return (const __attribute__((address_space(1))) T*)p;
}
// Constant-address-space view: uniform indices become scalar (s_load) loads.
template <class T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* cptr(const T* p) {
  return (const __attribute__((address_space(4))) T*)p;
}
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gptr_w(T* p) {
  return (__attribute__((address_space(1))) T*)p;
}

}  // namespace gpt
