/* gptsgld.h — C ABI of libgptsgld.so, the MI355X-native tensor-GP SGLD path.
 *
 * Drop-in boundary for the Julia module API that the reference's experiment scripts import
 * with `@everywhere using GPT_SGLD` (kin40kExperiment.jl:3).  Each entry point below names
 * the reference function it replaces (file:line under hyunjik11/GPT).  INTEGRATION.md shows
 * the Julia `ccall` shim and the Python ctypes binding.
 *
 * Conventions:
 *  - Arrays are Julia column-major: phi[j,k,i] at j + n*(k + D*i); U[j,l,k] at j + n*(l + r*k);
 *    I[q,k] (Int32, 1-based, values 1..r) at q + Q*k; X[i,k] at i + N*k; Float64 everywhere.
 *  - The caller allocates every output (zero-copy with `ccall(..., Ptr{Float64})`).  The
 *    library owns only device scratch.
 *  - Return value: GPT_OK, or an error code; gpt_last_error() has a thread-local message.
 *    GPT_ERR_NAN_GEODESIC mirrors GPT_SGLD.jl:23-26,422-424: the sample stores are zero-filled.
 *  - Host-pointer entry points copy to the device, run, and copy back (PCIe included).
 *    The *_dev entry points take device pointers and a hipStream_t (as void*) and are what the
 *    benchmark times (inputs resident in HBM).
 *  - Reentrant: no global state except the per-thread error string.
 */
#ifndef GPTSGLD_H
#define GPTSGLD_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPT_OK 0
#define GPT_ERR_NAN_GEODESIC 1
#define GPT_ERR_BAD_DIMS 2
#define GPT_ERR_HIP 3
#define GPT_ERR_NAN_THETA 4
#define GPT_ERR_NOT_SPD 5      /* a Gibbs precision matrix failed Cholesky (PosDefException) */

/* Sampler configuration: the scalar arguments of GPTregression (GPT_SGLD.jl:345) plus the
 * framework's store policy.  sigma_w = 1 is Generation C/D (GPT_SGLD.jl:354); Generation A/B
 * (GPT_SGLDERM, GPT_SGLD_p.jl:155) passes sigma_w = sqrt(n^D/Q) and signal_var = sigma^2. */
typedef struct gpt_sgld_config {
  int64_t n;          /* random features per input dimension (reference `n`)            */
  int64_t D;          /* input dimensions                                               */
  int64_t N;          /* training rows                                                  */
  int64_t r;          /* Stiefel rank                                                   */
  int64_t Q;          /* non-zeros of the sparse Tucker core                            */
  int64_t m;          /* minibatch size (reference `m`)                                 */
  double epsw, epsU;  /* SGLD step sizes                                                */
  double signal_var;  /* observation noise variance                                     */
  double sigma_w;     /* prior s.d. of w                                                */
  int64_t burnin, maxepoch;
  uint64_t seed;      /* param_seed: Philox key of every draw of this chain             */
  int32_t langevin;   /* 1 = SGLD (noise), 0 = SGD                                      */
  int32_t stiefel;    /* 1 = geodesic Stiefel update, 0 = Euclidean update of U         */
  int64_t store_every;/* 1 = reference (every post-burn-in step); numbatches = epoch ends */
  int64_t max_steps;  /* 0 = run all (burnin+maxepoch)*numbatches steps                  */
} gpt_sgld_config;

/* ---- features ------------------------------------------------------------------------ */
/* feature(X,length_scale,sigma_RBF,phi_scale,Z,b)  GPT_SGLD.jl:71-84  -> phi (n,D,N) */
int gpt_feature(const double* X, int64_t N, int64_t D, const double* length_scale,
                int64_t ls_len, double sigma_rbf, double phi_scale, const double* Z,
                const double* b, int64_t n, double* phi_out);
/* featureNotensor(X,length_scale,sigma_RBF,Z,b)  GPT_SGLD.jl:109-120  -> phi (n,N) */
int gpt_feature_notensor(const double* X, int64_t N, int64_t D, const double* length_scale,
                         int64_t ls_len, double sigma_rbf, const double* Z, const double* b,
                         int64_t n, double* phi_out);
/* Device form of gpt_feature (all pointers device, hip_stream may be NULL). */
int gpt_feature_dev(const double* X_dev, int64_t N, int64_t D, const double* ls_dev,
                    int64_t ls_len, double sigma_rbf, double phi_scale, const double* Z_dev,
                    const double* b_dev, int64_t n, double* phi_dev, void* hip_stream);
/* seeded Generation-C inputs of feature(X,n,ls,σ,seed,scale): Z=randn(n,D), b=2π·rand(n,D) */
int gpt_feature_inputs(int64_t n, int64_t D, uint64_t seed, double* Z_out, double* b_out);
/* seeded Generation-A inputs of feature(X,n,length_scale,seed)  GPT_SGLD_p.jl:40-54:
 * Z = randn(n,D) (the Gen-C Z stream), b = randn(n,D) (its own stream); the caller applies
 * Z/length_scale and scale sqrt(2/n) with sigma = 1 (gpt_feature with phi_scale = 1). */
int gpt_feature_inputs_a(int64_t n, int64_t D, uint64_t seed, double* Z_out, double* b_out);

/* samplenz(r,D,Q,seed)  GPT_SGLD.jl:181-190 / GPT_SGLD_p.jl:57-67  -> I (Q,D) Int32 1-based */
int gpt_samplenz(int64_t r, int64_t D, int64_t Q, uint64_t seed, int32_t* I_out);

/* Initial state of GPTregression (GPT_SGLD.jl:357-369): w (Q), U (n,r,D). */
int gpt_sgld_init(const gpt_sgld_config* cfg, double* w_out, double* U_out);

/* ---- sampler ------------------------------------------------------------------------- */
/* GPTregression(phi,y,signal_var,I,r,Q,m,epsw,epsU,burnin,maxepoch,param_seed;langevin,stiefel)
 * GPT_SGLD.jl:345-448 (also GPT_SGLDERM, GPT_SGLD_p.jl:146-243, via sigma_w/signal_var).
 * w_init/U_init: NULL = draw from the seed (the reference's srand(param_seed) path).  With
 * stiefel, U_init must have orthonormal columns per dimension (as the reference's init does): the
 * geodesic takes Uᵀmom as (M − Mᵀ)/2 from the projection's M = UᵀW, which holds on the manifold.
 * w_store (Q,T), U_store (n,r,D,T) with T = maxepoch*numbatches/store_every.
 * diag (nullable): per step [‖gradw‖, ‖gradU_1‖ … ‖gradU_D‖] ((1+D) x steps). */
int gpt_sgld_regression(const gpt_sgld_config* cfg, const double* phi, const double* y,
                        const int32_t* I, const double* w_init, const double* U_init,
                        double* w_store, double* U_store, double* diag);

/* Independent GPTregression chains in one call, from host arrays (kin40kExperiment.jl:67-74: the
 * `@parallel for j=1:10` sweep block, every sweep its own phi from its own length scales and
 * sigma_RBF; or posterior chains sharing one phi, BASELINE config 4).  It builds a device session
 * internally, so the multi-chain engines (chain engine r <= 5, wave engine r = 6..20; the grid
 * engine while nchains·(D+1) workgroups fit the CUs; GPTSGLD_ENGINE overrides) serve a host that
 * has no device memory of its own (the Julia shim).  phi[c] (n,D,N), y[c] (N): chain c's inputs
 * (pointers may repeat; each distinct array is copied to the device once).  seeds[c]: param_seed.
 * epsw / epsU / signal_var: NULL = cfg's value for every chain, else one per chain (sigma_w is
 * cfg's).  w_store[c] (Q,T), U_store[c] (n,r,D,T), T = maxepoch*numbatches/store_every, as
 * gpt_sgld_regression (both NULL: no stores).  status[c]: GPT_OK, or GPT_ERR_NAN_GEODESIC with
 * that chain's stores zero-filled (GPT_SGLD.jl:422-424); the return value is GPT_OK when every
 * chain ran to its end or bailed out. */
int gpt_sgld_regression_chains(const gpt_sgld_config* cfg, int32_t nchains, const uint64_t* seeds,
                               const double* const* phi, const double* const* y, const int32_t* I,
                               const double* epsw, const double* epsU, const double* signal_var,
                               double* const* w_store, double* const* U_store, int32_t* status);

/* GPT_SGLDERM_RMSprop(phi,y,signal_var,I,r,Q,m,epsilon,alpha,burnin,maxepoch)
 * GPT_SGLD.jl:1121-1237: per-entry RMSprop step sizes for w, one averaged step per U^(k), w
 * updated before A.  cfg's epsw/epsU/sigma_w are not used (sigma_w = 1 as in the reference);
 * cfg->langevin and cfg->stiefel must be 1.  Runs on the grid engine. */
/* GPT_SGLDERMw(phi,y,signal_var,I,r,Q,m,epsw,burnin,maxepoch)  GPT_SGLD.jl:1065-1118: SGLD on w
 * alone, U fixed at its uniform Stiefel draw (cfg: stiefel = langevin = 1, sigma_w = 1; epsU is
 * unused).  w_store (Q, maxepoch*numbatches), U_out (n, r, D) = the fixed U, diag row 0 = |gradw|
 * per step.  Runs on the grid engine (store_flags bit 4 in a session). */
int gpt_sgld_wonly(const gpt_sgld_config* cfg, const double* phi, const double* y, const int32_t* I,
                   const double* w_init, const double* U_init, double* w_store, double* U_out,
                   double* diag);
/* GPTclassification(phi,y,I,r,Q,m,epsw,epsU,burnin,maxepoch,param_seed;langevin,stiefel)
 * GPT_SGLD.jl:452-680: softmax tensor-GP classifier; y holds labels 1..C (as doubles).  cfg:
 * signal_var / sigma_w are not used (the model has no noise variance, sigma_w = 1).  Optional
 * w_init (Q, C) / U_init (n, r, D, C).  w_store (Q, C, maxepoch*numbatches), U_store
 * (n, r, D, C, ...); diag (1+D, steps, C) per-class gradient norms.  As the reference, w and U
 * move twice per step with one gradient (an SGLD + Stiefel move, then the langevin/stiefel
 * variant).  Grid engine (store_flags bit 5 in a session: the chains are the C classes). */
int gpt_sgld_classification(const gpt_sgld_config* cfg, const double* phi, const double* y,
                            const int32_t* I, const double* w_init, const double* U_init,
                            double* w_store, double* U_store, double* diag);
int gpt_sgld_rmsprop(const gpt_sgld_config* cfg, double epsilon, double alpha, const double* phi,
                     const double* y, const int32_t* I, const double* w_init,
                     const double* U_init, double* w_store, double* U_store, double* diag);

/* Multi-chain, device-resident session (benchmark / multi-GPU path).  Chains share the
 * config except seed; chain c reads phi_dev[c], y_dev[c] (device pointers; may alias). */
typedef struct gpt_sgld_session gpt_sgld_session;
int gpt_sgld_session_create(const gpt_sgld_config* cfg, int32_t nchains, const uint64_t* seeds,
                            const double* const* phi_dev, const double* const* y_dev,
                            const int32_t* I_host, int32_t store_on_device, void* hip_stream,
                            gpt_sgld_session** out);
/* Per-chain step sizes / variances (a hyper-parameter sweep, kin40kExperiment.jl:67-74);
 * call before the first run. */
int gpt_sgld_session_set_hyper(gpt_sgld_session* s, int32_t chain, double epsw, double epsU,
                               double signal_var, double sigma_w);
/* Queue `nsteps` SGLD steps of every chain on the session stream (asynchronous).  Whole epochs
 * replay one captured hipGraph; partial chunks replay a graph when one was prepared for them. */
int gpt_sgld_session_run(gpt_sgld_session* s, int64_t nsteps);
/* Capture (without running) the graphs a following gpt_sgld_session_run(s, nsteps) will replay,
 * so that run launches no individual kernels and pays no capture inside a timed region. */
int gpt_sgld_session_prepare(gpt_sgld_session* s, int64_t nsteps);
/* Switch a grid-engine session (store_flags bit 2) to GPT_SGLDERM_RMSprop steps; call before
 * the first run. */
int gpt_sgld_session_set_rmsprop(gpt_sgld_session* s, double epsilon, double alpha);
int gpt_sgld_session_sync(gpt_sgld_session* s);
/* Device pointers of chain c's current state and stores (for pred / collectives). */
int gpt_sgld_session_state(gpt_sgld_session* s, int32_t chain, double** w_dev, double** U_dev,
                           double** w_store_dev, double** U_store_dev, int64_t* nstore);
/* Current state of chains first .. first+count-1 packed on the device for stacked-sample
 * prediction (gpt_pred_dev with S = count): w_dev_out (Q, count), U_dev_out (n*r*D, count).
 * Ordered on the session stream. */
int gpt_sgld_session_gather_state(gpt_sgld_session* s, int32_t first, int32_t count,
                                  double* w_dev_out, double* U_dev_out);
int64_t gpt_sgld_session_steps_done(gpt_sgld_session* s);
/* Run `nsteps` steps WITHOUT graph capture, bracketing every step-kernel launch with hipEvents;
 * *avg_us = mean step-kernel duration (the roofline's per-launch time).  Synchronises. */
int gpt_sgld_session_time_steps(gpt_sgld_session* s, int64_t nsteps, double* avg_us);
/* Diagnostic: run nsteps un-captured steps recording s_memtime (shader-clock ticks)
 * stamps per phase; out = nsteps x W x 16 int64 (0 = phase not reached), W = the workgroups of
 * one step ((D+1)*nchains, grid engine; gpt_sgld_session_info). */
int gpt_sgld_session_stamps(gpt_sgld_session* s, int64_t nsteps, int64_t* out);
/* Diagnostic (chain engine): ONE launch of nsteps steps (within the current epoch, <= 512);
 * out = nchains x gpt_sgld_timeline_slots() int64: per block {s_memrealtime, s_memtime} at slot
 * 0 = entry, 1 = prologue end and 2 + s = end of step s, then HW_ID and XCC_ID.  The product
 * library fills slots 0, 1 and the last step's; the timeline build (`make timeline`) every step.
 * *event_us = the launch's hipEvent time. */
int64_t gpt_sgld_timeline_slots(void);
/* Test entry: E = expm(A) for `count` row-major nn x nn host matrices (nn in {12,16,20,24,30,32,
 * 40}) on the device: mode 0 the wave engine's register-blocked Padé (wave.hip wv_expm), mode 1 the
 * grid engine's wave_expm; bad[c] = 1 when E_c holds a NaN (the geodesic bail-out test). */
int gpt_debug_expm(int32_t nn, int32_t count, int32_t mode, const double* A, double* E,
                   int32_t* bad);
/* Test entry: the Gaussian conditional draw of the Gibbs samplers (tgp.hip gaussian_draw_prec,
 * GPT_fullw_gibbs w | U, V at 100k_movielensExperiment.jl:1092-1094, TGP.jl:61-63): M (p × p,
 * column-major, SPD; its lower triangle is read) = L·Lᵀ, out = L⁻ᵀz + M⁻¹x with z the Philox
 * normals (seed, c1, c2, c3) of element e = 0..p-1; *status = 1 if M is not positive definite. */
int gpt_debug_gaussian_draw(int32_t p, const double* M, const double* x, uint64_t seed, uint32_t c1,
                            uint32_t c2, uint32_t c3, double* out, int32_t* status);
/* Timing of the wave engine's expm as geod calls it (three LDS slots, the first nn/2 result
 * columns), one wave per matrix: stamps[4·m + 0..3] = s_memtime at entry, after the Padé
 * polynomial, after the solve, at exit (diagnostics; scripts/expm_bench.py). */
int gpt_debug_expm_stamps(int32_t nn, int32_t count, const double* A, int64_t* stamps);
int gpt_sgld_session_timeline(gpt_sgld_session* s, int64_t nsteps, int64_t* out, double* event_us);
/* Copy chain c's stores / status back (status: GPT_OK or GPT_ERR_NAN_GEODESIC; stores are
 * zero-filled for a non-zero status). */
int gpt_sgld_session_fetch(gpt_sgld_session* s, int32_t chain, double* w_store, double* U_store,
                           double* diag, int32_t* status);
void gpt_sgld_session_destroy(gpt_sgld_session* s);
/* out[4] = {engine, LDS bytes per workgroup, threads per workgroup, workgroups per step launch}.
 * Engines: 0 grid (sgld.hip: D+1 workgroups per chain, one step per launch), 1 chain (chain.hip:
 * one workgroup per chain, up to an epoch of steps per launch; r <= 5), 3 wave (wave.hip: per
 * step a V-phase workgroup per chain, then one wave per (chain, dimension); the figures are the
 * dimension launch's).  Engine 2 (the round-3 split engine) was removed.
 * store_flags of gpt_sgld_session_create: bit0 stores, bit1 diagnostics, bit2 force the grid
 * engine, bit3 force the chain engine, bit7 force the wave engine (bit6, the split engine, is
 * rejected).  Default: the chain engine whenever the shape allows it (few chains: the grid engine
 * while nchains*(D+1) workgroups fit the GPU's CUs), else the wave engine whenever the shape
 * allows it (SGLD + Stiefel, r in {6,8,10,12,15,16,20}, 3r <= n <= 256, m <= 64), else the grid
 * engine; GPTSGLD_ENGINE=grid|chain|wave overrides the default. */
int gpt_sgld_session_info(gpt_sgld_session* s, int64_t* out);

/* ---- prediction ---------------------------------------------------------------------- */
/* pred(w,U,I,phitest)  GPT_SGLD.jl:233-243  -> fhat (Ntest) */
int gpt_pred(const double* w, const double* U, const int32_t* I, const double* phitest,
             int64_t n, int64_t D, int64_t Ntest, int64_t r, int64_t Q, double* fhat_out);
/* Device form over S stored samples: fhat_dev (Ntest,S) = pred of each sample.
 * I_dev is 0-based Int32 (Q,D). */
int gpt_pred_dev(const double* w_dev, const double* U_dev, const int32_t* I0_dev,
                 const double* phitest_dev, int64_t n, int64_t D, int64_t Ntest, int64_t r,
                 int64_t Q, int64_t S, double* fhat_dev, void* hip_stream);
/* The stacked-sample prediction keeps its pass buffers (up to 8 GiB) in a private stream-ordered
 * pool between calls; this returns that memory to the device. */
int gpt_pred_trim_pool(void);
/* gpt_pred_dev with per-phase event timing (diagnostics / the benchmark): ms_out[0] = the
 * phidotU GEMM (fp64 MFMA) kernels, ms_out[1] = the V-phase kernels, summed over the sample
 * chunks of the call; synchronises hip_stream. */
int gpt_pred_dev_timed(const double* w_dev, const double* U_dev, const int32_t* I0_dev,
                       const double* phitest_dev, int64_t n, int64_t D, int64_t Ntest, int64_t r,
                       int64_t Q, int64_t S, double* fhat_dev, void* hip_stream, double* ms_out);
/* The V-phase kernel the last gpt_pred* call on this thread launched (measurement, no reference
 * counterpart): 0 pred_vphase_pairs_kernel, 1 pred_vphase_rows_pf_kernel, 2 pred_vphase_rows_kernel,
 * 4 pred_kernel (the direct path, no separate V-phase); -1 before any call. */
int gpt_pred_last_vphase(int32_t* kind);
/* Posterior-mean prediction over S samples + RMSE (GPT_SGLD_p.jl:124-132,
 * kin40kExperiment.jl:80-87): mean_out (Ntest), returns rmse*scale in *rmse_out. */
int gpt_pred_mean(const double* w_store, const double* U_store, const int32_t* I,
                  const double* phitest, const double* ytest, int64_t n, int64_t D,
                  int64_t Ntest, int64_t r, int64_t Q, int64_t S, double scale,
                  double* mean_out, double* rmse_out);

/* Fused feature + posterior-mean prediction (§8(f) per-epoch evaluation, kin40kExperiment.jl:78-87):
 * the test features phi = feature(Xtest, length_scale, sigma_rbf, phi_scale, Z, b) are formed
 * inside the prediction kernel (no n*D*Ntest phitest array; the same doubles gpt_feature makes).
 * Xtest (Ntest, D) column-major.  mean_out (Ntest) and *rmse_out as gpt_pred_mean;
 * sample_rmse_out (S, optional) = scale*||ytest - pred(sample s)||/sqrt(Ntest), the testRMSE curve. */
int gpt_pred_mean_x(const double* w_store, const double* U_store, const int32_t* I,
                    const double* Xtest, const double* ytest, int64_t Ntest, int64_t D,
                    const double* length_scale, int64_t ls_len, double sigma_rbf, double phi_scale,
                    const double* Z, const double* b, int64_t n, int64_t r, int64_t Q, int64_t S,
                    double scale, double* mean_out, double* rmse_out, double* sample_rmse_out);

/* ---- full-theta model (config 1) ----------------------------------------------------- */
/* GPNT_SGLD(phi,y,signal_var,sigma_theta,m,eps_theta,decay_rate,burnin,maxepoch,param_seed)
 * GPT_SGLD.jl:809-847 -> theta_store (n, (maxepoch+burnin)*numbatches) */
int gpt_gpnt_sgld(const double* phi, const double* y, int64_t n, int64_t N, double signal_var,
                  double sigma_theta, int64_t m, double eps_theta, double decay_rate,
                  int64_t burnin, int64_t maxepoch, uint64_t seed, double* theta_store);

/* ---- tensor-GP Gibbs sampler (§8 a25) ----------------------------------------------- */
/* GPT_inf(b,y,sigma,n,r,q,num_iterations,burnin) TGP.jl:37-86 on whitened data.
 * b (n, D, N) column-major feature array (TGP.feature, TGP.jl:6-14), y (N).
 * I (q, D) 1-based core indices; NULL draws them (TGP.jl:50) on the TGP_I Philox stream, and
 * I_out (optional) receives the indices used.  U starts at sqrt(1/r)·randn (TGP.jl:48-49,
 * TGP_U_INIT stream).  W_out (q, T), U_out (n, r, D, T), T = num_iterations - burnin: the W
 * draw of each kept sweep and the U it was drawn against (TGP.jl:60-63).
 * Returns GPT_ERR_NOT_SPD when a precision matrix is not positive definite. */
int gpt_tgp_gibbs(const double* b, const double* y, int64_t n, int64_t D, int64_t N, int64_t r,
                  int64_t q, double sigma, int64_t num_iterations, int64_t burnin, uint64_t seed,
                  const int32_t* I, double* W_out, double* U_out, int32_t* I_out);

/* ---- geodesic Monte Carlo (§8(f) item 4) ------------------------------------------- */
/* GPT_GMC(phi,y,signal_var,I,r,Q,epsw,epsU,burnin,maxepoch,L,param_seed)  GPT_SGLD.jl:684-805:
 * full-batch HMC with L leapfrog steps per epoch (Stiefel geodesic drift for U, geodboth
 * :40-59), sigma_w = 1.  w_store (Q, maxepoch), U_store (n, r, D, maxepoch), accept_prob
 * (burnin+maxepoch).  As the reference, a rejection restores w only (U_old aliases U there).
 * Optional w_init (Q) / U_init (n, r, D).  GPT_ERR_NAN_GEODESIC: zero stores, NaN accept_prob. */
int gpt_gmc(const double* phi, const double* y, int64_t n, int64_t D, int64_t N, int64_t r,
            int64_t Q, const int32_t* I, double signal_var, double epsw, double epsU,
            int64_t burnin, int64_t maxepoch, int64_t L, uint64_t seed, const double* w_init,
            const double* U_init, double* w_store, double* U_store, double* accept_prob);

/* ---- MovieLens-100k tensor CF with side information (§8(f) item 1, config 5) -------- */
/* GPT_fullw_sideinfo(Rating,UserData,MovieData,Ratingtest,signal_var,sigma_u,sigma_w,w_init,m,
 *   epsw,epsU,a,b,c,burnin,maxepoch,param_seed,ytrainMean,ytrainStd;langevin,stiefel,avg)
 * 100k_movielensExperiment.jl:409-551.  Rating (N x >=3, leading dimension ldr, column-major):
 * 1-based user, movie, standardised rating; Ratingtest likewise (ldt).  UserData (n1 x D1),
 * MovieData (n2 x D2) column-major 0/1 side information; w_init (r x r).  Outputs (caller-
 * allocated, column-major): w_store (r,r,maxepoch), U_store (n1+D1,r,maxepoch), V_store
 * (n2+D2,r,maxepoch), testpred_store (Ntest,maxepoch), trainRMSE / testRMSE (maxepoch; epochs
 * after the early stop of :545-547 keep 0 / 10).  GPT_ERR_NAN_GEODESIC: zero parameter stores. */
int gpt_cf_fullw_sideinfo(const double* Rating, int64_t N, int64_t ldr, const double* UserData,
                          int64_t n1, int64_t D1, const double* MovieData, int64_t n2, int64_t D2,
                          const double* Ratingtest, int64_t Ntest, int64_t ldt, double signal_var,
                          double sigma_u, double sigma_w, const double* w_init, int64_t r, int64_t m,
                          double epsw, double epsU, double a, double b, double c, int64_t burnin,
                          int64_t maxepoch, uint64_t seed, double ytrainMean, double ytrainStd,
                          int32_t langevin, int32_t stiefel, int32_t avg, double* w_store,
                          double* U_store, double* V_store, double* testpred_store,
                          double* trainRMSE, double* testRMSE);

/* GPT_fullw_gibbs(Rating,UserData,MovieData,Ratingtest,signal_var,sigma_u,sigma_w,w_init,burnin,
 *   maxepoch,n_samples,param_seed;avg,rotated_w)  100k_movielensExperiment.jl:1032-1129: Gibbs
 * sweeps of the CF model without side information (U: n1 x r, V: n2 x r rows | the rest, then
 * w | U, V through the N x r^2 Kronecker design).  n1 / n2 are size(UserData,1) / size(MovieData,1);
 * ytrainMean / ytrainStd are arguments (the reference reads script globals).  Outputs as
 * gpt_cf_fullw_sideinfo with U_store (n1,r,maxepoch), V_store (n2,r,maxepoch).
 * GPT_ERR_NOT_SPD on a non positive definite precision (Julia's PosDefException): detected within
 * two epochs of the failed Cholesky, and every output array is zeroed (the reference returns none). */
int gpt_cf_fullw_gibbs(const double* Rating, int64_t N, int64_t ldr, int64_t n1, int64_t n2,
                       const double* Ratingtest, int64_t Ntest, int64_t ldt, double signal_var,
                       double sigma_u, double sigma_w, const double* w_init, int64_t r,
                       int64_t burnin, int64_t maxepoch, int64_t n_samples, uint64_t seed,
                       double ytrainMean, double ytrainStd, int32_t avg, int32_t rotated_w,
                       double* w_store, double* U_store, double* V_store, double* testpred_store,
                       double* trainRMSE, double* testRMSE);

/* The folds of 100k_movielensExperiment.jl:733-736 (`@parallel for i=1:5` over
 * GPT_fullw_sideinfo(Ratingtrain[:,:,i], ..., Ratingtest[:,:,i], ..., ytrainMean[i],
 * ytrainStd[i])) as F sibling chains of one device launch per epoch: fold f reads Rating[f]
 * (N[f] x >=3, column-major, leading dimension N[f]) and Ratingtest[f] (Ntest[f] x >=3) and
 * writes w_store[f] .. testRMSE[f] exactly as F separate gpt_cf_fullw_sideinfo calls with the
 * same param_seed would (same init, per-epoch permutation and early stop, per fold); every fold
 * has the same N.  status[f] (optional): GPT_OK or GPT_ERR_NAN_GEODESIC for that fold; the return
 * value is GPT_ERR_NAN_GEODESIC when any fold bailed out. */
int gpt_cf_fullw_sideinfo_folds(int64_t F, const double* const* Rating, const int64_t* N,
                                const double* const* Ratingtest, const int64_t* Ntest,
                                const double* UserData, int64_t n1, int64_t D1,
                                const double* MovieData, int64_t n2, int64_t D2, double signal_var,
                                double sigma_u, double sigma_w, const double* w_init, int64_t r,
                                int64_t m, double epsw, double epsU, double a, double b, double c,
                                int64_t burnin, int64_t maxepoch, uint64_t seed,
                                const double* ytrainMean, const double* ytrainStd,
                                int32_t langevin, int32_t stiefel, int32_t avg,
                                double* const* w_store, double* const* U_store,
                                double* const* V_store, double* const* testpred_store,
                                double* const* trainRMSE, double* const* testRMSE, int32_t* status);

/* Device time of the last CF SGD / SGLD run (any gpt_cf_* SGD entry, fixw / sideinfo / folds)
 * on the calling thread: hipEvents around each epoch launch (cf_epoch_kernel, every live fold's
 * minibatch steps of one epoch) and each evaluation launch (cf_eval_kernel); epochs = epoch
 * launches, fold_steps = minibatch steps summed over the folds live in each launch.  No
 * reference counterpart (measurement, bench.py --workload movielens). */
int gpt_cf_last_timing(double* epoch_ms, double* eval_ms, int64_t* epochs, int64_t* fold_steps);
/* How the last CF SGD / SGLD call on this thread launched its epochs: 0 = per minibatch a
 * batch-phase launch (one workgroup per fold) and a row-parallel move launch; 1 = one launch per
 * epoch with the Stiefel move inside (stiefel = 1); 2 = one launch per epoch with the lazy SGD
 * move (langevin = stiefel = 0 on the feature-mask path: rows outside a batch only decay, read as
 * m·c^Δ).  No reference counterpart (measurement). */
int gpt_cf_last_mode(int32_t* mode);
/* With GPTSGLD_CF_STAMPS set, the last CF SGD call recorded s_memtime at the 8 phase boundaries
 * of fold 0's first 64 steps of its first epoch (batch load, masks / links, sums, sum·w,
 * residuals, gradients, U / V moves): copies up to cap of them (64 x 8, step-major) and returns
 * how many there are (0 without the variable).  Diagnostics. */
int64_t gpt_cf_last_stamps(int64_t* out, int64_t cap);

/* The other SGD / SGLD variants of the CF model (same Rating / Ratingtest / output conventions
 * as gpt_cf_fullw_sideinfo; the NaN bail-out zeroes the parameter stores):
 *   GPT_fixw_sideinfo(Rating,UserData,MovieData,Ratingtest,signal_var,sigma_u,w,m,epsU,a,b,c,
 *     burnin,maxepoch,param_seed,ytrainMean,ytrainStd;langevin,stiefel,avg)
 *     100k_movielensExperiment.jl:282-404 — w fixed, U,V = sigma_u*randn (also when stiefel);
 *     returns U_store (n1+D1,r,T), V_store, testpred_store, trainRMSE, testRMSE.
 *   GPT_fullw(Rating,UserData,MovieData,Ratingtest,signal_var,sigma_u,sigma_w,w_init,m,epsw,epsU,
 *     burnin,maxepoch,param_seed,ytrainMean,ytrainStd;langevin,stiefel,avg)
 *     :160-279 — no side information (pred = sum((U[user,:]*w).*V[movie,:])), U,V = randn or
 *     the Stiefel polar init; returns w_store (r,r,T), U_store (n1,r,T), V_store (n2,r,T), ...
 *   GPT_fixw(Rating,UserData,MovieData,Ratingtest,signal_var,sigma_u,w,m,epsU,burnin,maxepoch,
 *     param_seed,ytrainMean,ytrainStd;langevin,stiefel,avg)
 *     :56-156 — no side information, w fixed, U,V = sigma_u*randn; returns U_store (n1,r,T), ...
 * (The reference's bail-out of GPT_fullw / GPT_fixw returns a 3-tuple of zero arrays; these
 * entry points keep the normal outputs with zeroed parameter stores and GPT_ERR_NAN_GEODESIC.) */
int gpt_cf_fixw_sideinfo(const double* Rating, int64_t N, int64_t ldr, const double* UserData,
                         int64_t n1, int64_t D1, const double* MovieData, int64_t n2, int64_t D2,
                         const double* Ratingtest, int64_t Ntest, int64_t ldt, double signal_var,
                         double sigma_u, const double* w, int64_t r, int64_t m, double epsU,
                         double a, double b, double c, int64_t burnin, int64_t maxepoch,
                         uint64_t seed, double ytrainMean, double ytrainStd, int32_t langevin,
                         int32_t stiefel, int32_t avg, double* U_store, double* V_store,
                         double* testpred_store, double* trainRMSE, double* testRMSE);
int gpt_cf_fullw(const double* Rating, int64_t N, int64_t ldr, int64_t n1, int64_t n2,
                 const double* Ratingtest, int64_t Ntest, int64_t ldt, double signal_var,
                 double sigma_u, double sigma_w, const double* w_init, int64_t r, int64_t m,
                 double epsw, double epsU, int64_t burnin, int64_t maxepoch, uint64_t seed,
                 double ytrainMean, double ytrainStd, int32_t langevin, int32_t stiefel,
                 int32_t avg, double* w_store, double* U_store, double* V_store,
                 double* testpred_store, double* trainRMSE, double* testRMSE);
int gpt_cf_fixw(const double* Rating, int64_t N, int64_t ldr, int64_t n1, int64_t n2,
                const double* Ratingtest, int64_t Ntest, int64_t ldt, double signal_var,
                double sigma_u, const double* w, int64_t r, int64_t m, double epsU, int64_t burnin,
                int64_t maxepoch, uint64_t seed, double ytrainMean, double ytrainStd,
                int32_t langevin, int32_t stiefel, int32_t avg, double* U_store, double* V_store,
                double* testpred_store, double* trainRMSE, double* testRMSE);

/* GPT_fixw_gibbs(Rating,UserData,MovieData,Ratingtest,signal_var,sigma_u,w,burnin,maxepoch,
 *   n_samples,param_seed;avg,rotated_w)  100k_movielensExperiment.jl:945-1028: the user / movie
 * Gibbs conditionals of gpt_cf_fullw_gibbs with w fixed (no w draw); returns U_store (n1,r,T),
 * V_store (n2,r,T), testpred_store, trainRMSE, testRMSE. */
int gpt_cf_fixw_gibbs(const double* Rating, int64_t N, int64_t ldr, int64_t n1, int64_t n2,
                      const double* Ratingtest, int64_t Ntest, int64_t ldt, double signal_var,
                      double sigma_u, const double* w, int64_t r, int64_t burnin,
                      int64_t maxepoch, int64_t n_samples, uint64_t seed, double ytrainMean,
                      double ytrainStd, int32_t avg, int32_t rotated_w, double* U_store,
                      double* V_store, double* testpred_store, double* trainRMSE,
                      double* testRMSE);

/* randperm(N) + phi = phi[:,:,perm] of GPT_SGLD.jl:373-374 for `epochs` epochs of one chain,
 * built on the device by the sessions' own kernel: out (N, epochs) column-major, 0-based rows
 * of the composed order (order_e = order_{e-1}[perm_e]). */
int gpt_epoch_orders(int64_t N, uint64_t seed, int64_t epochs, int32_t* out);

const char* gpt_last_error(void);
/* LDS bytes one step workgroup needs for this shape (must be <= 163840). */
int64_t gpt_sgld_lds_bytes(int64_t n, int64_t D, int64_t r, int64_t Q, int64_t m);
int gpt_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* GPTSGLD_H */
