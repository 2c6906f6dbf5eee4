// Internal declarations shared by the libgptsgld translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>
#include <string>
#include <vector>
#include "gpt_common.h"
#include "../../include/gptsgld.h"

namespace gpt {

#ifndef GPT_NT
#define GPT_NT 512
#endif
#ifndef GPT_WPE
#define GPT_WPE 2
#endif
constexpr int kNT = GPT_NT;        // threads per workgroup (waves of 64)
constexpr int kNW = kNT / 64;      // waves per workgroup
constexpr int kDMax = 16;          // max input dimensions D handled by the kernels
constexpr int kEngineGrid = 0;     // sgld.hip: grid (D+1, chains), two batch reads per step
constexpr int kEngineChain = 1;    // chain.hip: one workgroup per chain, one batch read per step
constexpr int kEngineWave = 3;     // wave.hip: per step a V-phase workgroup per chain, then one
                                   // wave per (chain, dimension) (ranks past the chain engine)

// Per-chain device state.  All pointers are device pointers.
struct ChainDesc {
  const double* phi;     // n*D*N   training features, Julia layout
  const double* y;       // N       training targets
  int32_t* order;        // 2*N     ring of cumulative epoch orders (0-based rows): order_e at
                         //         (e&1)*N, built on the device (order.hip)
  double* w;             // 2*Q     ping-pong: w_t at (t&1)*Q
  double* U;             // n*r*D   current Stiefel factors (block k owns slice k)
  double* temp;          // 2*D*r*m ping-pong temp[k,l,i] of the NEXT batch
  double* w_store;       // Q*nstore or nullptr
  double* U_store;       // n*r*D*nstore or nullptr
  double* diag;          // (1+D)*steps per-step gradient norms or nullptr
  int32_t* status;       // 0 ok, 1 NaN in geodesic
  uint64_t seed;
  double epsw, epsU, signal_var, sigma_w;   // per-chain hyper-parameters (sweeps)
  double* gw;            // RMSprop (GPT_SGLD.jl:1121): Q moving average of squared gradw
  double* gU;            //   n*r*D moving average of squared gradU
  double* res;           //   m residuals of the step (written by the w phase)
  double* coef;          // wave engine: D*m*r core sums A[l,k,i]*res_i of the step, [(k*m + i)*r + l]
  double* park;          //   n*r*D the Stiefel momentum while the geodesic's expm holds the registers
};

struct StepParams {
  int n, D, N, r, Q, m, nb;       // nb = numbatches = ceil(N/m)
  int burnin_steps;               // burnin*nb
  long long total_steps;
  int store_every;
  int langevin, stiefel;
  const int32_t* I0;              // Q*D 0-based, layout q + Q*k
  const int32_t* runq;            // chain engine: runq[(k*r + l)*64 + s] = s-th q (ascending) with
                                  // I[q,k] = l, or 256 (a zero slot) past the run's end
  const int32_t* vtab;            // grid engine, column-lane V-phase: per workgroup kind (k < D,
                                  // w block = D) and core entry q, 16 ints: 8 temp row offsets
                                  // and I[q, k] (vphase_cols_tables), or null (vphase_tile)
  const uint16_t* wvtab;          // wave engine: V-phase temp offsets, run members, run starts
                                  // (16-bit, wave_tables)
  long long* stamps;              // diagnostic builds: s_memtime per phase per block, else null
  long long* tline;               // chain engine: per-workgroup timeline (kTimeline per block) or null
  int rms;                        // 1: GPT_SGLDERM_RMSprop steps (grid engine, two launches)
  int wonly;                      // 1: GPT_SGLDERMw steps (w alone, U fixed; grid engine)
  int ncls;                       // >= 2: GPTclassification, chains are the classes of one
                                  // model (grid engine; ChainDesc.res = class fhat, .gU = gradU)
  double rms_eps, rms_alpha;      // its epsilon and moving-average coefficient
};
constexpr int kStamps = 16;       // stamp slots per block
constexpr int kTimelineSteps = 512;                 // timeline diagnostics: steps per launch
constexpr int kTimeline = 2 * (kTimelineSteps + 2) + 2;   // int64 per block (+ HW_ID, XCC_ID)
constexpr double kRmsLambda = 1e-5;   // RMSprop smoothing (GPT_SGLD.jl:1146)

GPT_HD size_t al16(size_t x) { return (x + 15) & ~size_t(15); }

// LDS carve of the step kernel (bytes), shared by host (size) and device (offsets).
// Persistent part (whole launch) + a union whose tenants change by phase:
//   V-phase : temp_l                                     (D·R·MP)
//   grads   : W_l | U_l | redG                           (R·NP, R·NP, kNW·max(R²,8))
//   expm    : W_l | expm0 (7·(2R)²) | expm1 (7·R²)       (U_l/redG dead; old U re-read from HBM)
//   update  : W_l | U_l | redG                           (new U; P5 reads U_l)
struct StepLayout {
  int MP, NP, NS, conc, keepU, vcols;   // NP: n padded to 64 (loop range), NS = NP+1 row stride
  size_t o_I, o_w, o_idx, o_y, o_res, o_coef, o_gram, o_Ec, o_mx, o_un;
  size_t o_temp, o_W, o_U, o_red, o_x0, o_x1, o_ones, o_vred, o_vtab, bytes;
};

GPT_HD StepLayout step_layout(int n, int D, int r, int Q, int m) {
  StepLayout L;
  L.MP = ((m + 31) / 32) * 32 + 1;   // odd (bank spread); covers 32-wide unrolled reads
  L.NP = ((n + 63) / 64) * 64;
  L.NS = L.NP + 1;                   // odd stride: rows of U_l/W_l on different banks
  size_t o = 0;
  L.o_I = o;    o = al16(o + 4 * (size_t)Q * D);
  L.o_w = o;    o = al16(o + 8 * (size_t)Q);
  L.o_idx = o;  o = al16(o + 4 * (size_t)m);
  L.o_y = o;    o = al16(o + 8 * (size_t)m);
  L.o_res = o;  o = al16(o + 8 * (size_t)L.MP);
  L.o_coef = o; o = al16(o + 8 * (size_t)r * L.MP);
  L.o_gram = o; o = al16(o + 8 * (size_t)(4 * r * r + r + 2));
  L.o_Ec = o;   o = al16(o + 8 * (size_t)(2 * r * r));
  L.o_mx = o;   o = al16(o + 8 * (size_t)(r * r));
  L.o_un = o;
  const size_t nrp = 8 * (size_t)r * L.NS;
  // Gram scratch: kNW rows of 2r² (blk_gram), padded to the butterfly width of blk_gram_rows
  const int g2 = 2 * r * r, g2p = g2 <= 8 ? 8 : (g2 <= 16 ? 16 : (g2 <= 32 ? 32 : (g2 <= 64 ? 64 : g2)));
  const size_t red = 8 * (size_t)kNW * g2p;
  const size_t x0 = 8 * (size_t)7 * 4 * r * r, x1 = 8 * (size_t)7 * r * r;
  L.o_temp = o;
  L.o_W = o;
  L.o_U = o + nrp;
  L.o_red = L.o_U + nrp;
  const size_t un_v = 8 * (size_t)D * r * L.MP;
  const size_t un_g = 2 * nrp + red;
  size_t un = un_v > un_g ? un_v : un_g;
  const size_t cap = 160 * 1024;
  // Preferred: expm scratch after red with U_l kept (old U stays in LDS for tmpU), both expm
  // concurrent.  Fallbacks alias the scratch over U_l/red, then run the two expm in turn.
  if (al16(o + (un > 2 * nrp + red + x0 + x1 ? un : 2 * nrp + red + x0 + x1)) <= cap) {
    L.keepU = 1; L.conc = 1;
    L.o_x0 = L.o_red + red; L.o_x1 = L.o_x0 + x0;
    if (2 * nrp + red + x0 + x1 > un) un = 2 * nrp + red + x0 + x1;
  } else {
    L.keepU = 0;
    L.o_x0 = o + nrp;
    L.conc = (al16(o + (un > nrp + x0 + x1 ? un : nrp + x0 + x1)) <= cap) ? 1 : 0;
    L.o_x1 = L.conc ? L.o_x0 + x0 : L.o_x0;
    const size_t ux = L.conc ? nrp + x0 + x1 : nrp + x0;
    if (ux > un) un = ux;
  }
  // the column-lane V-phase (vphase_cols, D <= 8) keeps after temp_l a row of MP ones, its
  // per-wave partial sums (kNW·(1+r)·64 doubles) and its table (16 ints per q), when that still
  // fits the LDS; otherwise the step uses vphase_tile
  L.o_ones = o + al16(un_v);
  L.o_vred = L.o_ones + al16(8 * (size_t)L.MP);
  L.o_vtab = L.o_vred + 8 * (size_t)kNW * (1 + r) * 64;
  const size_t vend = L.o_vtab + 64 * (size_t)Q - o;
  if (D <= 8 && vend > un && al16(o + vend) <= cap) un = vend;
  L.vcols = (D <= 8 && vend <= un) ? 1 : 0;
  L.bytes = al16(o + un);
  return L;
}

// Raise a kernel's dynamic-LDS limit once per device.  Thread-safe: host threads (one per GPU, or
// several sessions) may race to set the same attribute, which is idempotent; the latch only
// skips the call once a device has it.
inline hipError_t set_max_lds_once(const void* fn, int bytes, std::atomic<uint64_t>& latch) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const uint64_t bit = 1ull << (dev & 63);
  if (latch.load(std::memory_order_acquire) & bit) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) latch.fetch_or(bit, std::memory_order_acq_rel);
  return e;
}

// Host helpers (capi.hip / sgld.hip)
void set_error(const std::string& msg);
int hip_fail(hipError_t e, const char* what);

// Launch wrappers implemented in sgld.hip / pred.hip / feature.hip
hipError_t launch_temp_init(const StepParams& P, const ChainDesc* chains, int nchains,
                            const long long* tbase, hipStream_t st);
hipError_t launch_step(const StepParams& P, const ChainDesc* chains, int nchains,
                       const long long* tbase, int t_local, hipStream_t st);
// RMSprop step = w phase (one workgroup per chain) then U phase (D workgroups per chain)
hipError_t launch_step_wonly(const StepParams& P, const ChainDesc* chains, int nchains,
                             const long long* tbase, int t_local, hipStream_t st);
hipError_t launch_step_cls(const StepParams& P, const ChainDesc* chains, int nchains,
                           const long long* tbase, int t_local, hipStream_t st);
hipError_t launch_step_rms(const StepParams& P, const ChainDesc* chains, int nchains,
                           const long long* tbase, int t_local, hipStream_t st);
hipError_t launch_advance(long long* tbase, long long by, hipStream_t st);
// Epoch orders (order.hip): e_fixed >= 0 builds order_{e_fixed}; e_fixed < 0 builds order_{e+1}
// for the epoch e of step tbase[0] + t_local.  ws: epoch_order_ws_ints(N, nchains) ints (0 when
// the shuffle fits LDS).
bool epoch_order_in_lds(int N);
size_t epoch_order_ws_ints(int N, int nchains);
hipError_t launch_epoch_order(const ChainDesc* chains, int nchains, int N, int nb,
                              long long total_steps, const long long* tbase, int t_local,
                              int e_fixed, int32_t* ws, hipStream_t st);
bool rank_supported(int r);
// vphase_cols' tables for a session (step_layout(n, D, r, Q, m).vcols): (D+1)·Q·16 ints
void vphase_cols_tables(const std::vector<int32_t>& I0, int n, int D, int r, int Q, int m,
                        std::vector<int32_t>& out);

// Chain-resident engine (chain.hip): one workgroup per chain, many steps per launch.
bool chain_supported(int n, int D, int r, int Q, int m, bool langevin, bool stiefel,
                     int max_run = 0);
size_t chain_lds_bytes(int n, int D, int r, int Q, int m);
// nsteps consecutive steps per launch (steps t .. t+nsteps-1 of one epoch at most)
hipError_t launch_chain(const StepParams& P, const ChainDesc* chains, int nchains,
                        const long long* tbase, int t_local, int nsteps, hipStream_t st);

// Wave engine (wave.hip): two launches per step (V-phase per chain, then a wave per dimension);
// init = the first step's temp only.
bool wave_supported(int n, int D, int r, int Q, int m, bool langevin, bool stiefel);
void wave_tables(const std::vector<int32_t>& I0, int Q, int D, int r, int m,
                 std::vector<uint16_t>& out);
size_t wv_dim_lds_bytes(int n, int r, int m);
size_t wv_vphase_lds_bytes(int D, int r, int Q, int m);
hipError_t launch_wave(const StepParams& P, const ChainDesc* chains, int nchains,
                       const long long* tbase, int t_local, bool init, hipStream_t st);
hipError_t launch_expm_check(int nn, int count, const double* A, double* E, int32_t* bad, int mode,
                             hipStream_t st, long long* stamps = nullptr);


hipError_t launch_pred_x(const double* w, const double* U, const int32_t* I0, const double* X,
                         const double* ls, const double* Z, const double* bfe, double c, int n,
                         int D, long long Ntest, int r, int Q, int S, double* fhat, hipStream_t st);
size_t pred_x_lds_bytes(int n, int D, int r, int Q);
// Per-phase event timing of the stacked-sample prediction (diagnostics / the benchmark):
// gemm_ms / vphase_ms accumulate over the sample chunks of one call.
struct PredPhaseTiming { double gemm_ms = 0.0, vphase_ms = 0.0; };
int pred_last_vphase();
hipError_t launch_pred(const double* w, const double* U, const int32_t* I0, const double* phitest,
                       int n, int D, long long Ntest, int r, int Q, int S, double* fhat,
                       hipStream_t st, PredPhaseTiming* timing = nullptr);
hipError_t pred_trim_pools();      // return the prediction pool's memory (gpt_pred_trim_pool)
hipError_t launch_mean_rmse(const double* fhat, const double* ytest, long long Ntest, int S,
                            double* mean_out, double* sse_out, hipStream_t st);
hipError_t launch_feature(const double* X, long long N, int D, const double* ls, double c,
                          const double* Z, const double* b, int n, double* phi, hipStream_t st);
hipError_t launch_feature_notensor(const double* X, long long N, int D, const double* ls,
                                   double c, const double* Z, const double* b, int n,
                                   double* phi, hipStream_t st);
// MovieLens tensor CF (cf.hip, 100k_movielensExperiment.jl:409-551)
struct CfParams {
  int n1, D1, n2, D2, r, m, rowsU, rowsV;
  double a, b, c, signal_var, sigma_u, sigma_w, epsw, epsU;
  int langevin, stiefel;
  int fixw;              // GPT_fixw*: w is a fixed argument (no gradw, no w step)
  uint64_t seed;
  const int32_t* uptr;   // n1+1 CSR offsets into ufe: the feature rows (n1 + f) of each user
  const int32_t* ufe;
  const int32_t* vptr;   // n2+1
  const int32_t* vfe;
  const uint64_t* umask;   // n1: bitmask of each user's feature rows (D1 <= 64), else null
  const uint64_t* vmask;   // n2
  long long* stamps;     // diagnostics: kCfStampSteps x kCfStampSlots s_memtime of chain 0, or null
  int exp;               // diagnostic builds only (CF_WSTAMPS): timing experiments, GPTSGLD_CF_EXP
};
// CF_WSTAMPS (diagnostic builds, make diag): 4 more stamps per wave of the 16 (cf.hip CF_WSTAMP)
#ifndef CF_WSTAMPS
#define CF_WSTAMPS 0
#endif
constexpr int kCfStampSteps = 64, kCfStampSlots = CF_WSTAMPS ? 8 + 4 * 16 : 8;

struct CfChain {
  const int32_t* tr_user;   // N   0-based ids
  const int32_t* tr_movie;
  const double* tr_rating;  // N   standardised
  const int32_t* te_user;   // Ntest
  const int32_t* te_movie;
  const double* te_rating;
  int N, Ntest;
  const int32_t* perm;      // N   this epoch's permutation (0-based rows of the ratings)
  int32_t* ep_user;         // N   the training ratings in this epoch's order (cf_gather_kernel)
  int32_t* ep_movie;
  double* ep_rating;
  double* w;                // r*r column-major
  double* U;                // rowsU*r column-major
  double* V;                // rowsV*r
  double* GU;               // rowsU*r zeroed scratch (gradient rows / momentum)
  double* GV;
  double ymean, ystd;       // ytrainMean / ytrainStd of the chain's fold (evaluation)
  double* trainpred;        // N      running averages (avg)
  double* testpred;         // Ntest
  double* sse;              // 2 * gridDim.x partial sums of the eval kernel
  int32_t* status;
};

size_t cf_lds_bytes(int r, int m, int nfeat, bool masks);
size_t cf_lazy_lds_bytes(int r, int m, int nfeat, int rows, int nb);
bool cf_rank_supported(int r);
hipError_t launch_cf_epoch(const CfParams& P, const CfChain* chains, int nchains, long long step0,
                           int bt0, int nb, int domove, hipStream_t st,
                           const long long* step_base = nullptr);
hipError_t launch_cf_gather(const CfChain* chains, int nchains, int N, hipStream_t st);
hipError_t launch_cf_move(const CfParams& P, const CfChain* chains, int nchains, long long step,
                          hipStream_t st, const long long* step_base = nullptr);
hipError_t launch_cf_eval(const CfParams& P, const CfChain* chains, int nchains, int nmax,
                          int counter, hipStream_t st);
hipError_t launch_cfg_rows(int side, int r, const double* W, const double* Oth, int rows_oth,
                           double* Me, int rows_me, const int32_t* ptr, const int32_t* lst,
                           const int32_t* other, const double* y, double signal_var, double su2,
                           uint64_t seed, uint32_t sweep, uint32_t stream, int32_t* status,
                           hipStream_t st);
size_t cfg_wsystem_scratch_dbl(int r, int n1);
hipError_t launch_cfg_wsystem(int r, const double* U, int n1, const double* V, int n2,
                              const int32_t* uptr, const int32_t* ulst, const int32_t* movies,
                              const double* y, double alpha, double beta, double ysc,
                              double* scratch, double* M, double* x, hipStream_t st);
hipError_t launch_cfg_keep(const CfChain* chains, int Ntest, int neval, double* rmse,
                           double* tp_out, hipStream_t st);
hipError_t gaussian_draw_prec(double* M, int p, double* x, uint64_t seed, uint32_t c1, uint32_t c2,
                              uint32_t c3, double* z, double* out, int32_t* status, hipStream_t st);
hipError_t gaussian_draw_dense(const double* A, int p, long long N, const double* y, double alpha,
                               double beta, double ysc, uint64_t seed, uint32_t c1, uint32_t c2,
                               uint32_t c3, double* M, double* x, double* z, double* out,
                               int32_t* status, hipStream_t st);
bool gmc_supported(int n, int r);
hipError_t gmc_run(const double* phi, const double* y, const int32_t* I0, int n, int D,
                   long long N, int r, int Q, double signal_var, double epsw, double epsU,
                   int burnin, int maxepoch, int L, uint64_t seed, double* w, double* U,
                   double* w_store, double* U_store, double* accept, int32_t* status,
                   hipStream_t st);
hipError_t tgp_gibbs(const double* b, const double* y, int n, int D, long long N, int r, int q,
                     double sigma, int iters, int burnin, uint64_t seed, const int32_t* I0,
                     double* U, double* W_hist, double* U_hist, int32_t* status, hipStream_t st);
hipError_t launch_gpnt(const double* phi, const double* y, const int32_t* order, int n, int N,
                       int m, int nb, long long total, double signal_var, double sigma_theta,
                       double eps_theta, double decay_rate, uint64_t seed, double* theta,
                       double* theta_store, int32_t* status, const long long* tbase, int t_local,
                       hipStream_t st);

// Host-side Philox consumers (init / permutations / samplenz)
void host_init_state(int n, int r, int D, int Q, uint64_t seed, bool stiefel, double sigma_w,
                     double* w, double* U, int cls = 0, bool cls_init = false);
void host_epoch_orders(int N, uint64_t seed, int epochs, int32_t* out);  // E*N cumulative

}  // namespace gpt
