// Host side of libgptsgld.so: the C ABI of include/gptsgld.h.
//
// Replaces the Julia module API of GPT_SGLD.jl (feature :71, featureNotensor :109, samplenz :181,
// GPTregression :345, pred :233, GPNT_SGLD :809) and GPT_SGLD_p.jl (GPT_SGLDERM :146, RMSE :124).
// All arithmetic of the sampler runs in the HIP kernels; the host only validates arguments,
// draws the one-time initial state and the epoch permutations from the Philox contract (the
// reference does the same draws on the CPU, GPT_SGLD.jl:357-373), moves buffers and launches.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "gpt_internal.h"

namespace gpt {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
int hip_fail(hipError_t e, const char* what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return GPT_ERR_HIP;
}
hipError_t set_lds_limits();
size_t pred_lds_bytes(int n, int D, int r, int Q);

#define HIPCHK(call)                                   \
  do {                                                 \
    hipError_t _e = (call);                            \
    if (_e != hipSuccess) return hip_fail(_e, #call);  \
  } while (0)

// ------------------------------------------------------------------ host Philox consumers
static double host_normal(uint64_t seed, uint32_t e, uint32_t c1, uint32_t c2, uint32_t c3) {
  const U4 x = philox4x32(e >> 1, c1, c2, c3, seed);
  const double u1 = u53(x.x, x.y), u2 = u53(x.z, x.w);
  const double rad = std::sqrt(-2.0 * std::log(u1));
  const double th = 6.283185307179586 * u2;
  return (e & 1u) ? rad * std::sin(th) : rad * std::cos(th);
}

// Cyclic Jacobi eigendecomposition of a symmetric r×r matrix (row-major, destroyed).
static void jacobi_eig(int r, std::vector<double>& A, std::vector<double>& V,
                       std::vector<double>& ev) {
  V.assign((size_t)r * r, 0.0);
  for (int i = 0; i < r; ++i) V[i * r + i] = 1.0;
  for (int sweep = 0; sweep < 100; ++sweep) {
    double off = 0.0, tot = 0.0;
    for (int i = 0; i < r; ++i)
      for (int j = 0; j < r; ++j) {
        tot += A[i * r + j] * A[i * r + j];
        if (i != j) off += A[i * r + j] * A[i * r + j];
      }
    if (off <= 1e-32 * tot) break;
    for (int p = 0; p < r; ++p)
      for (int q = p + 1; q < r; ++q) {
        const double apq = A[p * r + q];
        if (apq == 0.0) continue;
        const double theta = (A[q * r + q] - A[p * r + p]) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < r; ++k) {  // A = Jᵀ A J
          const double akp = A[k * r + p], akq = A[k * r + q];
          A[k * r + p] = c * akp - s * akq;
          A[k * r + q] = s * akp + c * akq;
        }
        for (int k = 0; k < r; ++k) {
          const double apk = A[p * r + k], aqk = A[q * r + k];
          A[p * r + k] = c * apk - s * aqk;
          A[q * r + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < r; ++k) {
          const double vkp = V[k * r + p], vkq = V[k * r + q];
          V[k * r + p] = c * vkp - s * vkq;
          V[k * r + q] = s * vkp + c * vkq;
        }
      }
  }
  ev.resize(r);
  for (int i = 0; i < r; ++i) ev[i] = A[i * r + i];
}

// GPT_SGLD.jl:357-369: w = σ_w·randn(Q); U_k = Zᵀ(ZZᵀ)^(-1/2), Z = randn(r,n)  (or randn/√n).
// Uniform draw on the Stiefel manifold from Z (r × n, element a + r·j): Uk (n × r, column-major)
// = Zᵀ(ZZᵀ)^(-1/2), the polar factor (transpose(sqrtm(Z*Z') \\ Z), GPT_SGLD.jl:365-366).
static void host_stiefel_polar(const double* Z, int r, int n, double* Uk) {
  std::vector<double> G((size_t)r * r, 0.0), Vv, ev;
  for (int a = 0; a < r; ++a)
    for (int c = 0; c < r; ++c) {
      double s = 0.0;
      for (int j = 0; j < n; ++j) s += Z[a + (size_t)r * j] * Z[c + (size_t)r * j];
      G[a * r + c] = s;
    }
  jacobi_eig(r, G, Vv, ev);
  std::vector<double> S((size_t)r * r, 0.0);  // (ZZᵀ)^(-1/2)
  for (int a = 0; a < r; ++a)
    for (int c = 0; c < r; ++c) {
      double s = 0.0;
      for (int z = 0; z < r; ++z) s += Vv[a * r + z] * Vv[c * r + z] / std::sqrt(ev[z]);
      S[a * r + c] = s;
    }
  for (int j = 0; j < n; ++j)
    for (int c = 0; c < r; ++c) {
      double s = 0.0;
      for (int a = 0; a < r; ++a) s += Z[a + (size_t)r * j] * S[a * r + c];
      Uk[j + (size_t)n * c] = s;
    }
}

// Class cls of GPTclassification (GPT_SGLD.jl:463-477) draws w on (W_INIT, cls) and U_k on
// (U_INIT, k + D·cls), and its non-Stiefel U is randn unscaled (cls_init).
void host_init_state(int n, int r, int D, int Q, uint64_t seed, bool stiefel, double sigma_w,
                     double* w, double* U, int cls, bool cls_init) {
  for (int q = 0; q < Q; ++q) w[q] = sigma_w * host_normal(seed, q, 0, kWInit, (uint32_t)cls);
  std::vector<double> Z((size_t)r * n);
  for (int k = 0; k < D; ++k) {
    for (int e = 0; e < r * n; ++e) Z[e] = host_normal(seed, e, 0, kUInit, (uint32_t)(k + D * cls));  // Z[a + r*j]
    double* Uk = U + (size_t)n * r * k;
    if (!stiefel) {
      for (int j = 0; j < n; ++j)
        for (int a = 0; a < r; ++a) Uk[j + (size_t)n * a] = cls_init ? Z[a + (size_t)r * j] : Z[a + (size_t)r * j] / std::sqrt((double)n);
      continue;
    }
    host_stiefel_polar(Z.data(), r, n, Uk);
  }
}

// Cumulative epoch orders on the host (GPNT_SGLD only; sessions build them on the device, order.hip):
// phi=phi[:,:,perm] every epoch composes the permutations (GPT_SGLD.jl:373-374);
// order_e = order_{e-1}[perm_e], perm_e Fisher–Yates on the PERM stream.
void host_epoch_orders(int N, uint64_t seed, int epochs, int32_t* out) {
  std::vector<int32_t> cur(N), p(N);
  for (int i = 0; i < N; ++i) cur[i] = i;
  for (int e = 0; e < epochs; ++e) {
    for (int i = 0; i < N; ++i) p[i] = i;
    for (int i = N - 1; i >= 1; --i) {
      const uint32_t x = philox4x32((uint32_t)i, (uint32_t)e, kPerm, 0, seed).x;
      const int j = (int)(((uint64_t)x * (uint64_t)(i + 1)) >> 32);
      std::swap(p[i], p[j]);
    }
    int32_t* o = out + (size_t)e * N;
    for (int i = 0; i < N; ++i) o[i] = cur[p[i]];
    std::memcpy(cur.data(), o, sizeof(int32_t) * N);
  }
}

struct DevMem {
  void* p = nullptr;
  DevMem() = default;
  DevMem(const DevMem&) = delete;
  DevMem& operator=(const DevMem&) = delete;
  ~DevMem() { if (p) (void)hipFree(p); }
  hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 16); }
  template <class T> T* as() const { return (T*)p; }
};

static bool valid_cfg(const gpt_sgld_config* c) {
  if (!c) { set_error("null config"); return false; }
  if (c->n < 1 || c->D < 1 || c->N < 1 || c->r < 1 || c->Q < 1 || c->m < 1) {
    set_error("dimensions must be positive"); return false;
  }
  if (c->D > kDMax) { set_error("D > 16 is not supported by the kernels"); return false; }
  if (!rank_supported((int)c->r)) {
    set_error("rank r not instantiated (supported: 1-6,8,10,12,15,16,20)"); return false;
  }
  if (c->n > (1 << 20) || c->N > (1LL << 31) - 1 || c->Q > (1 << 20)) {
    set_error("dimension too large"); return false;
  }
  double rD = std::pow((double)c->r, (double)c->D);
  if ((double)c->Q > rD) { set_error("Q must be <= r^D"); return false; }
  if (c->store_every < 1) { set_error("store_every must be >= 1"); return false; }
  if (!(c->signal_var > 0) || !(c->sigma_w > 0)) { set_error("variances must be > 0"); return false; }
  const StepLayout L = step_layout((int)c->n, (int)c->D, (int)c->r, (int)c->Q, (int)c->m);
  const bool chain_ok = chain_supported((int)c->n, (int)c->D, (int)c->r, (int)c->Q, (int)c->m,
                                        c->langevin != 0, c->stiefel != 0);
  const bool wave_ok = wave_supported((int)c->n, (int)c->D, (int)c->r, (int)c->Q, (int)c->m,
                                       c->langevin != 0, c->stiefel != 0);
  if (L.bytes > 160 * 1024 && !chain_ok && !wave_ok) {
    set_error("working set exceeds 160 KiB LDS (n*r, Q*D or m too large)"); return false;
  }
  return true;
}

}  // namespace gpt

using namespace gpt;

// ====================================================================== session
struct gpt_sgld_session {
  gpt_sgld_config cfg{};
  int nchains = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  StepParams P{};
  long long numbatches = 0, total_steps = 0, steps_done = 0, nstore = 0;
  int epochs = 0;
  DevMem I0, chains_d, tbase, status;
  std::vector<std::unique_ptr<DevMem>> chain_mem;
  std::vector<ChainDesc> chains_h;
  bool temp_ready = false;
  // Captured step sequences, keyed by where they start in an epoch (b0 = first step % numbatches,
  // which fixes where the epoch-order builds sit) and their length.  A replay reads the step
  // counter from the device, so one graph serves every epoch.
  struct GraphEnt { long long b0; int len; hipGraph_t g; hipGraphExec_t x; };
  std::vector<GraphEnt> graphs;
  bool ran = false;                   // a step has been enqueued (RMSprop must be set before)
  int graph_steps = 0;                // canonical chunk: one epoch (<= 512 steps)
  DevMem ord_ws;                      // epoch-order workspace when a shuffle exceeds LDS
  bool store = false, diag = false;
  int engine = 0;                     // kEngineGrid / kEngineChain / kEngineWave
  DevMem runq;
  DevMem wvtab;                       // wave engine: run members and starts (wave_tables)
  DevMem vtab;                        // grid engine: vphase_cols tables
  // Bounded in-flight work (gpt_sgld_session_run): an event after every chunk it enqueues, and
  // before the chunk that would put more than max_inflight chunks (<= one epoch each) in the
  // stream, a wait for the oldest.  A 200-epoch run() used to enqueue all 200 epoch graphs
  // (80 000 kernel dispatches on the wave engine) before the first finished.
  int max_inflight = 8;               // GPTSGLD_MAX_INFLIGHT; 0 = unbounded
  std::vector<hipEvent_t> inflight;
  long long chunks_enqueued = 0;
};

// Engine choice: store_flags bit 2 (or bit 4 / 5, w-only steps / classification) forces the grid
// engine (sgld.hip), bit 3 the chain engine (chain.hip), bit 7 the wave engine (wave.hip);
// otherwise GPTSGLD_ENGINE=grid|chain|wave; otherwise the chain engine whenever it supports the
// shape, else the wave engine (ranks past the chain engine), else the grid engine.  Few chains
// of a chain-engine shape go to the grid engine (D+1 workgroups per chain: the shorter step) as
// long as every chain's workgroups fit the GPU at once.  (Engine 2, the round-3 split engine —
// the grid engine with the batch in slices and an in-kernel barrier — measured slower at every
// slice count and was removed in round 4; bit 6 / "split" are rejected.)
static int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return cus;
}

static int pick_engine(const gpt_sgld_config* c, const int32_t* I_host, int32_t flags,
                       int nchains, int* engine) {
  int max_run = 0;                    // longest run of core entries sharing one I[·,k] value
  for (int k = 0; k < (int)c->D; ++k) {
    std::vector<int> cnt((size_t)c->r + 1, 0);
    for (int q = 0; q < (int)c->Q; ++q) max_run = std::max(max_run, ++cnt[I_host[q + c->Q * k]]);
  }
  const bool chain_ok = chain_supported((int)c->n, (int)c->D, (int)c->r, (int)c->Q, (int)c->m,
                                        c->langevin != 0, c->stiefel != 0, max_run);
  const bool grid_ok =
      step_layout((int)c->n, (int)c->D, (int)c->r, (int)c->Q, (int)c->m).bytes <= 160 * 1024;
  const bool wave_ok = wave_supported((int)c->n, (int)c->D, (int)c->r, (int)c->Q, (int)c->m,
                                      c->langevin != 0, c->stiefel != 0);
  if (flags & 64) { set_error("the split engine (store_flags bit 6) was removed"); return GPT_ERR_BAD_DIMS; }
  // explicit store_flags win over the environment: bits 4/16/32 (RMSprop-capable sessions, w-only
  // steps, classification) exist only on the grid engine
  int want = -1;
  if (flags & (4 | 16 | 32)) want = kEngineGrid;
  else if (flags & 8) want = kEngineChain;
  else if (flags & 128) want = kEngineWave;
  else if (const char* ev = std::getenv("GPTSGLD_ENGINE")) {
    if (!std::strcmp(ev, "grid")) want = kEngineGrid;
    else if (!std::strcmp(ev, "chain")) want = kEngineChain;
    else if (!std::strcmp(ev, "split")) {
      set_error("the split engine (GPTSGLD_ENGINE=split) was removed"); return GPT_ERR_BAD_DIMS;
    }
    else if (!std::strcmp(ev, "wave")) want = kEngineWave;
  }
  if (want == kEngineWave && !wave_ok) {
    set_error("wave engine does not support this shape (needs SGLD+Stiefel, r in {6,8,10,12,15,"
              "16,20}, 3r <= n <= 256, m <= 64, the V-phase working set within 160 KiB LDS)");
    return GPT_ERR_BAD_DIMS;
  }
  if (want == kEngineChain && !chain_ok) {
    set_error("chain engine does not support this shape (needs D<=8, r<=5, n<=512 (even if >64), "
              "Q<=256, SGLD+Stiefel, <=64 core entries per I[.,k] value)");
    return GPT_ERR_BAD_DIMS;
  }
  if (want == kEngineGrid && !grid_ok) {
    set_error("grid engine: working set exceeds 160 KiB LDS"); return GPT_ERR_BAD_DIMS;
  }
  // few chains: the grid engine's D+1 workgroups per chain (the shorter step)
  // ranks past the chain engine: the wave engine (its step is shorter than the grid engine's even
  // for one chain: the geodesic's expm runs on every dimension's wave at once)
  if (want < 0 && !chain_ok && wave_ok) want = kEngineWave;
  if (want < 0 && grid_ok && (long long)nchains * (c->D + 1) <= device_cus()) want = kEngineGrid;
  *engine = want >= 0 ? want : (chain_ok ? kEngineChain : kEngineGrid);
  return GPT_OK;
}

// Chain engine tables: for every dimension k the core entries ordered by (I[q,k], q):
// pos[q + Q*k] = rank of q, seg[k*(r+1) + l] = first rank with I[q,k] = l (0-based).
// Run members of the chain engine's core sums (see gpt_internal.h StepParams::runq).
static void chain_runq(const std::vector<int32_t>& I0, int Q, int D, int r,
                       std::vector<int32_t>& out) {
  out.assign((size_t)D * r * 64, 256);
  for (int k = 0; k < D; ++k) {
    std::vector<int> cnt(r, 0);
    for (int q = 0; q < Q; ++q) {
      const int l = I0[q + (size_t)Q * k];
      out[((size_t)k * r + l) * 64 + cnt[l]++] = q;   // max run <= 64 (chain_supported)
    }
  }
}

extern "C" const char* gpt_last_error(void) { return g_err.c_str(); }

extern "C" int64_t gpt_sgld_lds_bytes(int64_t n, int64_t D, int64_t r, int64_t Q, int64_t m) {
  return (int64_t)step_layout((int)n, (int)D, (int)r, (int)Q, (int)m).bytes;
}

extern "C" int gpt_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

// Steps t_local .. t_local+nsteps-1 of the sequence being enqueued (nsteps > 1 only on the chain
// engine, within one epoch: every other kernel is one step per launch).
static hipError_t session_launch(gpt_sgld_session* s, const StepParams& P, int t_local,
                                 int nsteps = 1) {
  if (P.ncls)
    return launch_step_cls(P, s->chains_d.as<ChainDesc>(), s->nchains, s->tbase.as<long long>(),
                           t_local, s->stream);
  if (P.wonly)
    return launch_step_wonly(P, s->chains_d.as<ChainDesc>(), s->nchains, s->tbase.as<long long>(),
                             t_local, s->stream);
  if (P.rms)
    return launch_step_rms(P, s->chains_d.as<ChainDesc>(), s->nchains, s->tbase.as<long long>(),
                           t_local, s->stream);
  if (s->engine == kEngineChain)
    return launch_chain(P, s->chains_d.as<ChainDesc>(), s->nchains, s->tbase.as<long long>(),
                        t_local, nsteps, s->stream);
  if (s->engine == kEngineWave)
    return launch_wave(P, s->chains_d.as<ChainDesc>(), s->nchains, s->tbase.as<long long>(),
                       t_local, false, s->stream);
  return launch_step(P, s->chains_d.as<ChainDesc>(), s->nchains, s->tbase.as<long long>(),
                     t_local, s->stream);
}

// temp of the first step (grid engine only: the chain engine forms temp inside its step).
static int session_prime(gpt_sgld_session* s) {
  if (s->engine == kEngineChain || s->temp_ready) return GPT_OK;
  hipError_t e = s->engine == kEngineWave
                     ? launch_wave(s->P, s->chains_d.as<ChainDesc>(), s->nchains,
                                   s->tbase.as<long long>(), 0, true, s->stream)
                     : launch_temp_init(s->P, s->chains_d.as<ChainDesc>(), s->nchains,
                                        s->tbase.as<long long>(), s->stream);
  if (e != hipSuccess) return hip_fail(e, "launch_temp_init");
  s->temp_ready = true;
  return GPT_OK;
}

// Before the first step of epoch e, order_{e+1} goes into the ring slot order_{e-1} leaves
// (order.hip).  t_host = the step's index as the host counts it: in a captured sequence only its
// position in the epoch matters (the kernel reads the step counter from the device).
static hipError_t session_epoch_order(gpt_sgld_session* s, long long t_host, int t_local) {
  if (t_host % s->P.nb != 0) return hipSuccess;
  return launch_epoch_order(s->chains_d.as<ChainDesc>(), s->nchains, s->P.N, s->P.nb,
                            s->total_steps, s->tbase.as<long long>(), t_local, -1,
                            s->ord_ws.as<int32_t>(), s->stream);
}

// Steps of one epoch at most that one launch runs from host step t_host (chain engine: the rest of
// the epoch within `left`; other engines: 1).
static int session_span(const gpt_sgld_session* s, long long t_host, long long left) {
  if (s->engine != kEngineChain || s->P.rms || s->P.wonly || s->P.ncls) return 1;
  return (int)std::min<long long>(left, s->P.nb - t_host % s->P.nb);
}

static int session_enqueue(gpt_sgld_session* s, int count) {
  s->ran = true;
  for (int i = 0; i < count;) {
    hipError_t e = session_epoch_order(s, s->steps_done + i, i);
    if (e != hipSuccess) return hip_fail(e, "launch_epoch_order");
    const int span = session_span(s, s->steps_done + i, count - i);
    e = session_launch(s, s->P, i, span);
    if (e != hipSuccess) return hip_fail(e, "launch_step");
    i += span;
  }
  hipError_t e = launch_advance(s->tbase.as<long long>(), count, s->stream);
  if (e != hipSuccess) return hip_fail(e, "launch_advance");
  return GPT_OK;
}

extern "C" int gpt_sgld_session_create(const gpt_sgld_config* cfg, int32_t nchains,
                                       const uint64_t* seeds, const double* const* phi_dev,
                                       const double* const* y_dev, const int32_t* I_host,
                                       int32_t store_flags, void* hip_stream,
                                       gpt_sgld_session** out) {
  if (!out) { set_error("null out"); return GPT_ERR_BAD_DIMS; }
  *out = nullptr;
  if (!valid_cfg(cfg)) return GPT_ERR_BAD_DIMS;
  if (nchains < 1 || !seeds || !phi_dev || !y_dev || !I_host) {
    set_error("bad chain arguments"); return GPT_ERR_BAD_DIMS;
  }
  const int n = (int)cfg->n, D = (int)cfg->D, N = (int)cfg->N, r = (int)cfg->r, Q = (int)cfg->Q,
            m = (int)cfg->m;
  for (long long x = 0; x < (long long)Q * D; ++x)
    if (I_host[x] < 1 || I_host[x] > r) { set_error("I entries must be in 1..r"); return GPT_ERR_BAD_DIMS; }
  hipError_t he = set_lds_limits();
  if (he != hipSuccess) return hip_fail(he, "hipFuncSetAttribute");

  std::unique_ptr<gpt_sgld_session> s(new gpt_sgld_session());
  {
    const int rc = pick_engine(cfg, I_host, store_flags, nchains, &s->engine);
    if (rc != GPT_OK) return rc;
  }
  s->cfg = *cfg;
  s->nchains = nchains;
  s->numbatches = (N + m - 1) / m;
  s->epochs = (int)(cfg->burnin + cfg->maxepoch);
  s->total_steps = (long long)s->epochs * s->numbatches;
  if (cfg->max_steps > 0) s->total_steps = std::min<long long>(s->total_steps, cfg->max_steps);
  s->nstore = (cfg->maxepoch * s->numbatches) / cfg->store_every;
  s->store = (store_flags & 1) != 0;
  s->diag = (store_flags & 2) != 0;
  if (hip_stream) s->stream = (hipStream_t)hip_stream;
  else {
    HIPCHK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    s->own_stream = true;
  }
  StepParams& P = s->P;
  P.n = n; P.D = D; P.N = N; P.r = r; P.Q = Q; P.m = m; P.nb = (int)s->numbatches;
  P.burnin_steps = (int)(cfg->burnin * s->numbatches);
  P.total_steps = s->total_steps;
  P.store_every = (int)cfg->store_every;
  P.langevin = cfg->langevin; P.stiefel = cfg->stiefel;

  std::vector<int32_t> I0((size_t)Q * D);
  for (size_t x = 0; x < I0.size(); ++x) I0[x] = I_host[x] - 1;
  HIPCHK(s->I0.alloc(sizeof(int32_t) * I0.size()));
  HIPCHK(hipMemcpy(s->I0.p, I0.data(), sizeof(int32_t) * I0.size(), hipMemcpyHostToDevice));
  P.I0 = s->I0.as<int32_t>();
  P.runq = nullptr;
  if (s->engine == kEngineChain) {
    std::vector<int32_t> rq;
    chain_runq(I0, Q, D, r, rq);
    HIPCHK(s->runq.alloc(sizeof(int32_t) * rq.size()));
    HIPCHK(hipMemcpy(s->runq.p, rq.data(), sizeof(int32_t) * rq.size(), hipMemcpyHostToDevice));
    P.runq = s->runq.as<int32_t>();
  }
  P.wvtab = nullptr;
  if (s->engine == kEngineWave) {
    std::vector<uint16_t> wt;
    wave_tables(I0, Q, D, r, m, wt);
    HIPCHK(s->wvtab.alloc(sizeof(uint16_t) * wt.size()));
    HIPCHK(hipMemcpy(s->wvtab.p, wt.data(), sizeof(uint16_t) * wt.size(), hipMemcpyHostToDevice));
    P.wvtab = s->wvtab.as<uint16_t>();
  }
  P.vtab = nullptr;
  if (s->engine != kEngineChain && s->engine != kEngineWave && step_layout(n, D, r, Q, m).vcols) {
    std::vector<int32_t> vt;
    vphase_cols_tables(I0, n, D, r, Q, m, vt);
    HIPCHK(s->vtab.alloc(sizeof(int32_t) * vt.size()));
    HIPCHK(hipMemcpy(s->vtab.p, vt.data(), sizeof(int32_t) * vt.size(), hipMemcpyHostToDevice));
    P.vtab = s->vtab.as<int32_t>();
  }
  P.stamps = nullptr;
  P.tline = nullptr;
  P.rms = 0; P.rms_eps = 0.0; P.rms_alpha = 0.0;
  P.wonly = (store_flags & 16) ? 1 : 0;
  P.ncls = (store_flags & 32) ? nchains : 0;
  HIPCHK(s->tbase.alloc(sizeof(long long)));
  HIPCHK(hipMemset(s->tbase.p, 0, sizeof(long long)));
  HIPCHK(s->status.alloc(sizeof(int32_t) * nchains));
  HIPCHK(hipMemset(s->status.p, 0, sizeof(int32_t) * nchains));

  constexpr size_t a = 256;
  auto up = [](size_t x) { return (x + a - 1) / a * a; };
  const size_t b_w = up(8 * 2 * (size_t)Q), b_U = up(8 * (size_t)n * r * D),
               b_temp = up(8 * 2 * (size_t)D * r * m),
               b_ord = up(4 * 2 * (size_t)N),
               b_ws = s->store ? up(8 * (size_t)Q * s->nstore) : 0,
               b_Us = s->store ? up(8 * (size_t)n * r * D * s->nstore) : 0,
               b_dg = s->diag ? up(8 * (size_t)(1 + D) * s->total_steps) : 0,
               b_wv = s->engine == kEngineWave ? up(8 * (size_t)D * m * r) + up(8 * (size_t)n * r * D) : 0;
  std::vector<double> w0(Q), U0((size_t)n * r * D);
  s->chains_h.resize(nchains);
  for (int c = 0; c < nchains; ++c) {
    std::unique_ptr<DevMem> mem(new DevMem());
    HIPCHK(mem->alloc(b_w + b_U + b_temp + b_ord + b_ws + b_Us + b_dg + b_wv));
    char* base = mem->as<char>();
    ChainDesc& C = s->chains_h[c];
    C.phi = phi_dev[c];
    C.y = y_dev[c];
    C.w = (double*)base;
    C.U = (double*)(base + b_w);
    C.temp = (double*)(base + b_w + b_U);
    C.order = (int32_t*)(base + b_w + b_U + b_temp);
    C.w_store = s->store ? (double*)(base + b_w + b_U + b_temp + b_ord) : nullptr;
    C.U_store = s->store ? (double*)(base + b_w + b_U + b_temp + b_ord + b_ws) : nullptr;
    C.diag = s->diag ? (double*)(base + b_w + b_U + b_temp + b_ord + b_ws + b_Us) : nullptr;
    C.status = s->status.as<int32_t>() + c;
    C.seed = seeds[c];
    C.gw = C.gU = C.res = nullptr;
    C.coef = C.park = nullptr;
    if (b_wv) {
      char* wv = base + b_w + b_U + b_temp + b_ord + b_ws + b_Us + b_dg;
      C.coef = (double*)wv;
      C.park = (double*)(wv + up(8 * (size_t)D * m * r));
    }
    C.epsw = cfg->epsw; C.epsU = cfg->epsU; C.signal_var = cfg->signal_var; C.sigma_w = cfg->sigma_w;
    host_init_state(n, r, D, Q, seeds[c], cfg->stiefel != 0, cfg->sigma_w, w0.data(), U0.data());
    HIPCHK(hipMemcpy(C.w, w0.data(), 8 * (size_t)Q, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(C.U, U0.data(), 8 * U0.size(), hipMemcpyHostToDevice));
    if (s->store) HIPCHK(hipMemset(C.w_store, 0, b_ws + b_Us));
    if (s->diag) HIPCHK(hipMemset(C.diag, 0, b_dg));
    s->chain_mem.push_back(std::move(mem));
  }
  HIPCHK(s->chains_d.alloc(sizeof(ChainDesc) * nchains));
  HIPCHK(hipMemcpy(s->chains_d.p, s->chains_h.data(), sizeof(ChainDesc) * nchains,
                   hipMemcpyHostToDevice));
  // order_0 of every chain (the first step builds order_1, session_epoch_order)
  if (const size_t wsi = epoch_order_ws_ints(N, nchains)) HIPCHK(s->ord_ws.alloc(4 * wsi));
  HIPCHK(launch_epoch_order(s->chains_d.as<ChainDesc>(), nchains, N, (int)s->numbatches,
                            s->total_steps, s->tbase.as<long long>(), 0, 0, s->ord_ws.as<int32_t>(),
                            s->stream));
  s->graph_steps = (int)std::min<long long>(std::max<long long>(s->numbatches, 1), 512);
  if (const char* ev = std::getenv("GPTSGLD_MAX_INFLIGHT")) s->max_inflight = std::max(0, std::atoi(ev));
  *out = s.release();
  return GPT_OK;
}

// Overwrite chain c's initial state (w_init/U_init injection of the host API).  On the Stiefel
// path the kernels take geod's A = Uᵀmom as (M − Mᵀ)/2 (and the grid engine S from the Gram
// identity), which holds only for UᵀU = I: a U_init off the manifold is rejected.
static int session_set_state(gpt_sgld_session* s, int c, const double* w, const double* U) {
  const ChainDesc& C = s->chains_h[c];
  if (U && s->cfg.stiefel) {
    const int n = s->P.n, r = s->P.r, D = s->P.D;
    for (int k = 0; k < D; ++k) {
      const double* Uk = U + (size_t)n * r * k;
      for (int a = 0; a < r; ++a)
        for (int b = a; b < r; ++b) {
          double g = 0.0;
          for (int j = 0; j < n; ++j) g += Uk[j + (size_t)n * a] * Uk[j + (size_t)n * b];
          if (std::fabs(g - (a == b ? 1.0 : 0.0)) > 1e-10) {
            set_error("U_init must have orthonormal columns in every dimension (max |U_kᵀU_k - I| "
                      "<= 1e-10) on the Stiefel path");
            return GPT_ERR_BAD_DIMS;
          }
        }
    }
  }
  if (w) HIPCHK(hipMemcpy(C.w, w, 8 * (size_t)s->P.Q, hipMemcpyHostToDevice));
  if (U) HIPCHK(hipMemcpy(C.U, U, 8 * (size_t)s->P.n * s->P.r * s->P.D, hipMemcpyHostToDevice));
  s->temp_ready = false;
  return GPT_OK;
}

extern "C" int gpt_sgld_session_set_hyper(gpt_sgld_session* s, int32_t chain, double epsw,
                                          double epsU, double signal_var, double sigma_w) {
  if (!s || chain < 0 || chain >= s->nchains) { set_error("bad chain"); return GPT_ERR_BAD_DIMS; }
  if (!(signal_var > 0) || !(sigma_w > 0)) { set_error("variances must be > 0"); return GPT_ERR_BAD_DIMS; }
  ChainDesc& C = s->chains_h[chain];
  C.epsw = epsw; C.epsU = epsU; C.signal_var = signal_var; C.sigma_w = sigma_w;
  HIPCHK(hipMemcpy(s->chains_d.as<ChainDesc>() + chain, &C, sizeof(ChainDesc), hipMemcpyHostToDevice));
  return GPT_OK;
}

// Destroy every captured graph (after the stream has drained: a launched graph may still run).
static void session_drop_graphs(gpt_sgld_session* s) {
  if (s->graphs.empty()) return;
  (void)hipStreamSynchronize(s->stream);
  for (auto& g : s->graphs) {
    (void)hipGraphExecDestroy(g.x);
    (void)hipGraphDestroy(g.g);
  }
  s->graphs.clear();
}

// Per-chain zeroed gw (Q) | gU (n·r·D) | res (m) buffers of the RMSprop and classification steps.
static int session_alloc_aux(gpt_sgld_session* s) {
  const StepParams& P = s->P;
  const size_t bq = 8 * (size_t)P.Q, bu = 8 * (size_t)P.n * P.r * P.D, br = 8 * (size_t)P.m;
  for (int c = 0; c < s->nchains; ++c) {
    std::unique_ptr<DevMem> mem(new DevMem());
    HIPCHK(mem->alloc(bq + bu + br));
    HIPCHK(hipMemset(mem->p, 0, bq + bu + br));
    ChainDesc& C = s->chains_h[c];
    C.gw = mem->as<double>();
    C.gU = C.gw + P.Q;
    C.res = C.gU + (size_t)P.n * P.r * P.D;
    s->chain_mem.push_back(std::move(mem));
  }
  HIPCHK(hipMemcpy(s->chains_d.p, s->chains_h.data(), sizeof(ChainDesc) * s->nchains,
                   hipMemcpyHostToDevice));
  return GPT_OK;
}

extern "C" int gpt_sgld_session_set_rmsprop(gpt_sgld_session* s, double epsilon, double alpha) {
  if (!s) { set_error("null session"); return GPT_ERR_BAD_DIMS; }
  if (s->engine != kEngineGrid) {
    set_error("RMSprop steps run on the grid engine: create the session with store_flags bit 2");
    return GPT_ERR_BAD_DIMS;
  }
  if (!s->cfg.stiefel || !s->cfg.langevin) {
    set_error("GPT_SGLDERM_RMSprop is the SGLD + Stiefel sampler (langevin = stiefel = 1)");
    return GPT_ERR_BAD_DIMS;
  }
  if (s->steps_done != 0 || s->ran) { set_error("set RMSprop before the first run"); return GPT_ERR_BAD_DIMS; }
  if (!(epsilon > 0) || !(alpha >= 0 && alpha < 1)) {
    set_error("RMSprop needs epsilon > 0 and 0 <= alpha < 1"); return GPT_ERR_BAD_DIMS;
  }
  const int rc = session_alloc_aux(s);     // moving averages start at 0 (:1143-1144)
  if (rc != GPT_OK) return rc;
  s->P.rms = 1; s->P.rms_eps = epsilon; s->P.rms_alpha = alpha;
  // graphs prepared before this call (gpt_sgld_session_prepare) captured plain SGLD steps: drop
  // them so the next run captures RMSprop steps
  session_drop_graphs(s);
  return GPT_OK;
}

// The graph replaying `len` steps from a start at b0 = step % numbatches (captured on first use).
static int session_graph(gpt_sgld_session* s, int len, hipGraphExec_t* out) {
  const long long b0 = s->steps_done % s->P.nb;
  for (auto& g : s->graphs)
    if (g.b0 == b0 && g.len == len) { *out = g.x; return GPT_OK; }
  if (s->graphs.size() >= 16) {                // bounded cache: drop the oldest
    HIPCHK(hipStreamSynchronize(s->stream));   // it may still be running (launches are async)
    (void)hipGraphExecDestroy(s->graphs.front().x);
    (void)hipGraphDestroy(s->graphs.front().g);
    s->graphs.erase(s->graphs.begin());
  }
  HIPCHK(hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal));
  int rc = session_enqueue(s, len);
  hipGraph_t g = nullptr;
  hipError_t ee = hipStreamEndCapture(s->stream, &g);
  if (rc != GPT_OK) { if (g) (void)hipGraphDestroy(g); return rc; }
  if (ee != hipSuccess) return hip_fail(ee, "hipStreamEndCapture");
  hipGraphExec_t x = nullptr;
  ee = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
  if (ee != hipSuccess) { (void)hipGraphDestroy(g); return hip_fail(ee, "hipGraphInstantiate"); }
  s->graphs.push_back({b0, len, g, x});
  // upload now (ordered on the session stream), so a graph prepared ahead of a timed region does
  // not pay its first-launch upload inside it
  HIPCHK(hipGraphUpload(x, s->stream));
  *out = x;
  return GPT_OK;
}

// Chunks of a run of n steps from the current step: up to the end of the current epoch, then whole
// epochs (graph_steps), then the remainder.
static int session_next_chunk(const gpt_sgld_session* s, long long remaining, long long at) {
  const long long to_epoch_end = s->graph_steps - (at % s->P.nb) % s->graph_steps;
  return (int)std::min<long long>(remaining, to_epoch_end);
}

// Before enqueueing a chunk: wait until fewer than max_inflight chunks are outstanding.
static int session_throttle(gpt_sgld_session* s) {
  if (s->max_inflight <= 0) return GPT_OK;
  if (s->inflight.empty()) {
    s->inflight.assign(s->max_inflight, nullptr);
    for (auto& e : s->inflight) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  if (s->chunks_enqueued >= s->max_inflight)
    HIPCHK(hipEventSynchronize(s->inflight[s->chunks_enqueued % s->max_inflight]));
  return GPT_OK;
}

// After enqueueing a chunk: mark its end in the ring slot the throttle waits on later.
static int session_mark(gpt_sgld_session* s) {
  if (s->max_inflight <= 0) return GPT_OK;
  HIPCHK(hipEventRecord(s->inflight[s->chunks_enqueued % s->max_inflight], s->stream));
  ++s->chunks_enqueued;
  return GPT_OK;
}

extern "C" int gpt_sgld_session_run(gpt_sgld_session* s, int64_t nsteps) {
  if (!s) { set_error("null session"); return GPT_ERR_BAD_DIMS; }
  long long remaining = std::min<long long>(nsteps, s->total_steps - s->steps_done);
  if (remaining <= 0) return GPT_OK;
  {
    const int rc = session_prime(s);
    if (rc != GPT_OK) return rc;
  }
  while (remaining > 0) {
    {
      const int rc = session_throttle(s);
      if (rc != GPT_OK) return rc;
    }
    const int chunk = session_next_chunk(s, remaining, s->steps_done);
    // a whole canonical chunk, or any chunk prepared beforehand (gpt_sgld_session_prepare), runs as
    // one graph; other partial chunks are launched directly
    const long long b0 = s->steps_done % s->P.nb;
    bool cached = false;
    for (auto& g : s->graphs) cached |= (g.b0 == b0 && g.len == chunk);
    if (chunk == s->graph_steps || cached) {
      hipGraphExec_t x = nullptr;
      const int rc = session_graph(s, chunk, &x);
      if (rc != GPT_OK) return rc;
      HIPCHK(hipGraphLaunch(x, s->stream));
      s->ran = true;
    } else {
      const int rc = session_enqueue(s, chunk);
      if (rc != GPT_OK) return rc;
    }
    s->steps_done += chunk;
    remaining -= chunk;
    {
      const int rc = session_mark(s);
      if (rc != GPT_OK) return rc;
    }
  }
  return GPT_OK;
}

extern "C" int gpt_sgld_session_prepare(gpt_sgld_session* s, int64_t nsteps) {
  if (!s) { set_error("null session"); return GPT_ERR_BAD_DIMS; }
  long long remaining = std::min<long long>(nsteps, s->total_steps - s->steps_done);
  const long long saved = s->steps_done;
  const bool ran = s->ran;
  int rc = GPT_OK;
  while (remaining > 0 && rc == GPT_OK) {  // the same chunking as gpt_sgld_session_run
    const int chunk = session_next_chunk(s, remaining, s->steps_done);
    hipGraphExec_t x = nullptr;
    rc = session_graph(s, chunk, &x);
    s->steps_done += chunk;
    remaining -= chunk;
  }
  s->steps_done = saved;                   // capture enqueues nothing: the position is unchanged
  s->ran = ran;
  return rc;
}

extern "C" int gpt_sgld_session_time_steps(gpt_sgld_session* s, int64_t nsteps, double* avg_us) {
  if (!s) { set_error("null session"); return GPT_ERR_BAD_DIMS; }
  const long long cnt = std::min<long long>(nsteps, s->total_steps - s->steps_done);
  if (avg_us) *avg_us = 0.0;
  if (cnt <= 0) return GPT_OK;
  {
    const int rc = session_prime(s);
    if (rc != GPT_OK) return rc;
  }
  struct Events {                          // destroyed on every exit path
    std::vector<hipEvent_t> v;
    ~Events() { for (auto e : v) if (e) (void)hipEventDestroy(e); }
  } evs;
  evs.v.assign(2 * cnt, nullptr);
  std::vector<hipEvent_t>& ev = evs.v;
  for (auto& e : ev) HIPCHK(hipEventCreate(&e));
  int rc = GPT_OK;
  s->ran = true;
  // one event pair per launch (a launch runs `span` steps on the chain engine)
  long long nl = 0;
  for (long long i = 0; i < cnt && rc == GPT_OK; ++nl) {
    hipError_t eo = session_epoch_order(s, s->steps_done + i, (int)i);   // outside the event pair
    if (eo != hipSuccess) return hip_fail(eo, "launch_epoch_order");
    const int span = session_span(s, s->steps_done + i, cnt - i);
    HIPCHK(hipEventRecord(ev[2 * nl], s->stream));
    hipError_t e = session_launch(s, s->P, (int)i, span);
    if (e != hipSuccess) rc = hip_fail(e, "launch_step");
    HIPCHK(hipEventRecord(ev[2 * nl + 1], s->stream));
    i += span;
  }
  if (rc == GPT_OK) {
    hipError_t e = launch_advance(s->tbase.as<long long>(), cnt, s->stream);
    if (e != hipSuccess) rc = hip_fail(e, "launch_advance");
  }
  HIPCHK(hipStreamSynchronize(s->stream));
  double tot = 0.0;
  for (long long i = 0; i < nl; ++i) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
    tot += ms;
  }
  if (rc != GPT_OK) return rc;
  s->steps_done += cnt;
  if (avg_us) *avg_us = 1000.0 * tot / (double)cnt;
  return GPT_OK;
}

extern "C" int gpt_sgld_session_stamps(gpt_sgld_session* s, int64_t nsteps, int64_t* out) {
  if (!s || !out) { set_error("null argument"); return GPT_ERR_BAD_DIMS; }
  const long long cnt = std::min<long long>(nsteps, s->total_steps - s->steps_done);
  if (cnt <= 0) return GPT_OK;
  {
    const int rc = session_prime(s);
    if (rc != GPT_OK) return rc;
  }
  // one slot row per workgroup of a step: D+1 per chain
  const size_t per = (size_t)(s->P.D + 1) * s->nchains * kStamps;
  DevMem buf;
  HIPCHK(buf.alloc(8 * per * cnt));
  HIPCHK(hipMemset(buf.p, 0, 8 * per * cnt));
  StepParams P = s->P;
  s->ran = true;
  for (long long i = 0; i < cnt; ++i) {
    P.stamps = buf.as<long long>() + per * i;
    hipError_t eo = session_epoch_order(s, s->steps_done + i, (int)i);
    if (eo != hipSuccess) return hip_fail(eo, "launch_epoch_order");
    hipError_t e = session_launch(s, P, (int)i);
    if (e != hipSuccess) return hip_fail(e, "launch_step");
  }
  hipError_t e = launch_advance(s->tbase.as<long long>(), cnt, s->stream);
  if (e != hipSuccess) return hip_fail(e, "launch_advance");
  HIPCHK(hipStreamSynchronize(s->stream));
  HIPCHK(hipMemcpy(out, buf.p, 8 * per * cnt, hipMemcpyDeviceToHost));
  s->steps_done += cnt;
  return GPT_OK;
}

extern "C" int64_t gpt_sgld_timeline_slots(void) { return kTimeline; }

// Test entry: expm of `count` row-major nn × nn host matrices on the device, by the wave engine's
// register-blocked Padé (mode 0) or the grid engine's wave_expm (mode 1).
extern "C" int gpt_debug_expm(int32_t nn, int32_t count, int32_t mode, const double* A, double* E,
                              int32_t* bad) {
  if (count < 1 || !A || !E || !bad) { set_error("bad arguments"); return GPT_ERR_BAD_DIMS; }
  const size_t b = 8 * (size_t)nn * nn * count;
  DevMem dA, dE, dB;
  HIPCHK(dA.alloc(b));
  HIPCHK(dE.alloc(b));
  HIPCHK(dB.alloc(4 * (size_t)count));
  HIPCHK(hipMemcpy(dA.p, A, b, hipMemcpyHostToDevice));
  hipError_t e = launch_expm_check(nn, count, dA.as<double>(), dE.as<double>(), dB.as<int32_t>(),
                                   mode, nullptr);
  if (e == hipErrorInvalidValue) { set_error("nn not instantiated"); return GPT_ERR_BAD_DIMS; }
  HIPCHK(e);
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(E, dE.p, b, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(bad, dB.p, 4 * (size_t)count, hipMemcpyDeviceToHost));
  return GPT_OK;
}

extern "C" int gpt_debug_gaussian_draw(int32_t p, const double* M, const double* x, uint64_t seed,
                                       uint32_t c1, uint32_t c2, uint32_t c3, double* out,
                                       int32_t* status) {
  if (p < 1 || !M || !x || !out || !status) { set_error("bad arguments"); return GPT_ERR_BAD_DIMS; }
  DevMem dM, dx, dz, dout, dst;
  HIPCHK(dM.alloc(8 * (size_t)p * p));
  HIPCHK(dx.alloc(8 * (size_t)p));
  HIPCHK(dz.alloc(8 * (size_t)p));
  HIPCHK(dout.alloc(8 * (size_t)p));
  HIPCHK(dst.alloc(4));
  HIPCHK(hipMemcpy(dM.p, M, 8 * (size_t)p * p, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dx.p, x, 8 * (size_t)p, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(dst.p, 0, 4));
  HIPCHK(gaussian_draw_prec(dM.as<double>(), p, dx.as<double>(), seed, c1, c2, c3, dz.as<double>(),
                            dout.as<double>(), dst.as<int32_t>(), nullptr));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, dout.p, 8 * (size_t)p, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(status, dst.p, 4, hipMemcpyDeviceToHost));
  return GPT_OK;
}

extern "C" int gpt_debug_expm_stamps(int32_t nn, int32_t count, const double* A, int64_t* stamps) {
  if (count < 1 || !A || !stamps) { set_error("bad arguments"); return GPT_ERR_BAD_DIMS; }
  const size_t b = 8 * (size_t)nn * nn * count;
  DevMem dA, dE, dB, dS;
  HIPCHK(dA.alloc(b));
  HIPCHK(dE.alloc(b));
  HIPCHK(dB.alloc(4 * (size_t)count));
  HIPCHK(dS.alloc(32 * (size_t)count));
  HIPCHK(hipMemcpy(dA.p, A, b, hipMemcpyHostToDevice));
  hipError_t e = launch_expm_check(nn, count, dA.as<double>(), dE.as<double>(), dB.as<int32_t>(), 2,
                                   nullptr, dS.as<long long>());
  if (e == hipErrorInvalidValue) { set_error("nn not instantiated"); return GPT_ERR_BAD_DIMS; }
  HIPCHK(e);
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(stamps, dS.p, 32 * (size_t)count, hipMemcpyDeviceToHost));
  return GPT_OK;
}

extern "C" int gpt_sgld_session_timeline(gpt_sgld_session* s, int64_t nsteps, int64_t* out,
                                         double* event_us) {
  if (!s || !out) { set_error("null argument"); return GPT_ERR_BAD_DIMS; }
  if (s->engine != kEngineChain) { set_error("timeline: chain engine only"); return GPT_ERR_BAD_DIMS; }
  const long long left = s->total_steps - s->steps_done;
  const int span = session_span(s, s->steps_done, std::min<long long>(nsteps, left));
  if (nsteps < 1 || span != nsteps || nsteps > kTimelineSteps) {
    set_error("timeline: nsteps must be one launch (within the epoch and the run, <= 512)");
    return GPT_ERR_BAD_DIMS;
  }
  const size_t per = (size_t)kTimeline * s->nchains;
  DevMem buf;
  HIPCHK(buf.alloc(8 * per));
  HIPCHK(hipMemsetAsync(buf.p, 0, 8 * per, s->stream));
  StepParams P = s->P;
  P.tline = buf.as<long long>();
  s->ran = true;
  hipError_t eo = session_epoch_order(s, s->steps_done, 0);
  if (eo != hipSuccess) return hip_fail(eo, "launch_epoch_order");
  hipEvent_t e0 = nullptr, e1 = nullptr;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  hipError_t e = hipEventRecord(e0, s->stream);
  if (e == hipSuccess) e = session_launch(s, P, 0, (int)nsteps);
  if (e == hipSuccess) e = hipEventRecord(e1, s->stream);
  if (e == hipSuccess) e = launch_advance(s->tbase.as<long long>(), nsteps, s->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  float ms = 0.f;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (e != hipSuccess) return hip_fail(e, "timeline launch");
  if (event_us) *event_us = 1000.0 * ms;
  HIPCHK(hipMemcpy(out, buf.p, 8 * per, hipMemcpyDeviceToHost));
  s->steps_done += nsteps;
  return GPT_OK;
}

extern "C" int gpt_sgld_session_info(gpt_sgld_session* s, int64_t* out) {
  if (!s || !out) { set_error("null argument"); return GPT_ERR_BAD_DIMS; }
  const StepParams& P = s->P;
  out[0] = s->engine;
  if (s->engine == kEngineChain) {
    out[1] = (int64_t)chain_lds_bytes(P.n, P.D, P.r, P.Q, P.m);
    out[2] = 64 * P.D;
    out[3] = s->nchains;
  } else if (s->engine == kEngineWave) {     // the dimension launch (the V-phase: one per chain)
    out[1] = (int64_t)wv_dim_lds_bytes(P.n, P.r, P.m);
    out[2] = 64;
    out[3] = (int64_t)P.D * s->nchains;
  } else {
    out[1] = (int64_t)step_layout(P.n, P.D, P.r, P.Q, P.m).bytes;
    out[2] = kNT;
    out[3] = (int64_t)(P.D + 1) * s->nchains;
  }
  return GPT_OK;
}

extern "C" int gpt_sgld_session_sync(gpt_sgld_session* s) {
  if (!s) return GPT_ERR_BAD_DIMS;
  HIPCHK(hipStreamSynchronize(s->stream));
  return GPT_OK;
}

extern "C" int64_t gpt_sgld_session_steps_done(gpt_sgld_session* s) { return s ? s->steps_done : -1; }

extern "C" int gpt_sgld_session_state(gpt_sgld_session* s, int32_t chain, double** w_dev,
                                      double** U_dev, double** w_store_dev, double** U_store_dev,
                                      int64_t* nstore) {
  if (!s || chain < 0 || chain >= s->nchains) { set_error("bad chain"); return GPT_ERR_BAD_DIMS; }
  const ChainDesc& C = s->chains_h[chain];
  // current w lives in the ping-pong slot of the next step
  if (w_dev) *w_dev = C.w + (size_t)(s->steps_done & 1) * s->P.Q;
  if (U_dev) *U_dev = C.U;
  if (w_store_dev) *w_store_dev = C.w_store;
  if (U_store_dev) *U_store_dev = C.U_store;
  if (nstore) *nstore = s->nstore;
  return GPT_OK;
}

extern "C" int gpt_sgld_session_gather_state(gpt_sgld_session* s, int32_t first, int32_t count,
                                             double* w_dev_out, double* U_dev_out) {
  if (!s || first < 0 || count < 0 || first + count > s->nchains || (count && (!w_dev_out || !U_dev_out))) {
    set_error("bad chain range"); return GPT_ERR_BAD_DIMS;
  }
  const size_t Q = (size_t)s->P.Q, nrD = (size_t)s->P.n * s->P.r * s->P.D;
  for (int32_t c = 0; c < count; ++c) {
    const ChainDesc& C = s->chains_h[first + c];
    HIPCHK(hipMemcpyAsync(w_dev_out + c * Q, C.w + (size_t)(s->steps_done & 1) * Q, 8 * Q,
                          hipMemcpyDeviceToDevice, s->stream));
    HIPCHK(hipMemcpyAsync(U_dev_out + c * nrD, C.U, 8 * nrD, hipMemcpyDeviceToDevice, s->stream));
  }
  return GPT_OK;
}

extern "C" int gpt_sgld_session_fetch(gpt_sgld_session* s, int32_t chain, double* w_store,
                                      double* U_store, double* diag, int32_t* status) {
  if (!s || chain < 0 || chain >= s->nchains) { set_error("bad chain"); return GPT_ERR_BAD_DIMS; }
  HIPCHK(hipStreamSynchronize(s->stream));
  const ChainDesc& C = s->chains_h[chain];
  int32_t st = 0;
  HIPCHK(hipMemcpy(&st, C.status, sizeof(int32_t), hipMemcpyDeviceToHost));
  if (status) *status = st;
  const size_t nws = (size_t)s->P.Q * s->nstore, nus = (size_t)s->P.n * s->P.r * s->P.D * s->nstore;
  if (w_store) {
    if (!s->store) { set_error("session created without stores"); return GPT_ERR_BAD_DIMS; }
    if (st) std::memset(w_store, 0, 8 * nws);  // GPT_SGLD.jl:422-424
    else HIPCHK(hipMemcpy(w_store, C.w_store, 8 * nws, hipMemcpyDeviceToHost));
  }
  if (U_store) {
    if (!s->store) { set_error("session created without stores"); return GPT_ERR_BAD_DIMS; }
    if (st) std::memset(U_store, 0, 8 * nus);
    else HIPCHK(hipMemcpy(U_store, C.U_store, 8 * nus, hipMemcpyDeviceToHost));
  }
  if (diag) {
    if (!s->diag) { set_error("session created without diagnostics"); return GPT_ERR_BAD_DIMS; }
    HIPCHK(hipMemcpy(diag, C.diag, 8 * (size_t)(1 + s->P.D) * s->total_steps, hipMemcpyDeviceToHost));
  }
  return GPT_OK;
}

extern "C" void gpt_sgld_session_destroy(gpt_sgld_session* s) {
  if (!s) return;
  (void)hipStreamSynchronize(s->stream);
  session_drop_graphs(s);
  for (auto e : s->inflight) if (e) (void)hipEventDestroy(e);
  if (s->own_stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

// ====================================================================== host-pointer API
extern "C" int gpt_sgld_init(const gpt_sgld_config* cfg, double* w_out, double* U_out) {
  if (!valid_cfg(cfg)) return GPT_ERR_BAD_DIMS;
  host_init_state((int)cfg->n, (int)cfg->r, (int)cfg->D, (int)cfg->Q, cfg->seed, cfg->stiefel != 0,
                  cfg->sigma_w, w_out, U_out);
  return GPT_OK;
}

// Shared driver of the host-pointer samplers: one chain, device copies of phi / y, the run, the
// stores back (zero-filled + GPT_ERR_NAN_GEODESIC on the geodesic bail-out, GPT_SGLD.jl:422-424).
static int host_sampler(const gpt_sgld_config* cfg, const double* phi, const double* y,
                        const int32_t* I, const double* w_init, const double* U_init,
                        double* w_store, double* U_store, double* diag, int extra_flags,
                        double rms_eps, double rms_alpha, double* U_final = nullptr) {
  if (!valid_cfg(cfg)) return GPT_ERR_BAD_DIMS;
  if (!phi || !y || !I) { set_error("null input"); return GPT_ERR_BAD_DIMS; }
  const size_t nphi = (size_t)cfg->n * cfg->D * cfg->N;
  DevMem dphi, dy;
  HIPCHK(dphi.alloc(8 * nphi));
  HIPCHK(dy.alloc(8 * (size_t)cfg->N));
  HIPCHK(hipMemcpy(dphi.p, phi, 8 * nphi, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dy.p, y, 8 * (size_t)cfg->N, hipMemcpyHostToDevice));
  const double* pp = dphi.as<double>();
  const double* yy = dy.as<double>();
  gpt_sgld_session* s = nullptr;
  const int flags = ((w_store || U_store) ? 1 : 0) | (diag ? 2 : 0) | extra_flags;
  int rc = gpt_sgld_session_create(cfg, 1, &cfg->seed, &pp, &yy, I, flags, nullptr, &s);
  if (rc != GPT_OK) return rc;
  std::unique_ptr<gpt_sgld_session, void (*)(gpt_sgld_session*)> guard(s, gpt_sgld_session_destroy);
  if (rms_eps > 0) {
    rc = gpt_sgld_session_set_rmsprop(s, rms_eps, rms_alpha);
    if (rc != GPT_OK) return rc;
  }
  if (w_init || U_init) {
    rc = session_set_state(s, 0, w_init, U_init);
    if (rc != GPT_OK) return rc;
  }
  rc = gpt_sgld_session_run(s, s->total_steps);
  if (rc != GPT_OK) return rc;
  int32_t st = 0;
  rc = gpt_sgld_session_fetch(s, 0, w_store, U_store, diag, &st);
  if (rc != GPT_OK) return rc;
  if (st) {
    set_error("Get NaN when moving along Geodesic. Try smaller epsU");
    return GPT_ERR_NAN_GEODESIC;
  }
  if (U_final)
    HIPCHK(hipMemcpy(U_final, s->chains_h[0].U, 8 * (size_t)cfg->n * cfg->r * cfg->D,
                     hipMemcpyDeviceToHost));
  return GPT_OK;
}

extern "C" int gpt_sgld_regression(const gpt_sgld_config* cfg, const double* phi, const double* y,
                                   const int32_t* I, const double* w_init, const double* U_init,
                                   double* w_store, double* U_store, double* diag) {
  return host_sampler(cfg, phi, y, I, w_init, U_init, w_store, U_store, diag, 0, 0.0, 0.0);
}

// Independent chains from host arrays through one device session (the chain / wave engines that
// the device-pointer session API reaches): kin40kExperiment.jl:67-74's sweep block, every sweep
// its own phi and hyper-parameters, or posterior chains on one phi.  Each distinct phi / y array is
// copied to the device once (the pointers may repeat).
extern "C" int gpt_sgld_regression_chains(const gpt_sgld_config* cfg, int32_t nchains,
                                          const uint64_t* seeds, const double* const* phi,
                                          const double* const* y, const int32_t* I,
                                          const double* epsw, const double* epsU,
                                          const double* signal_var, double* const* w_store,
                                          double* const* U_store, int32_t* status) {
  if (!valid_cfg(cfg)) return GPT_ERR_BAD_DIMS;
  if (nchains < 1 || !seeds || !phi || !y || !I || !status) {
    set_error("gpt_sgld_regression_chains: null or empty arguments");
    return GPT_ERR_BAD_DIMS;
  }
  const bool stores = w_store || U_store;
  for (int c = 0; c < nchains; ++c) {
    if (!phi[c] || !y[c] || (w_store && !w_store[c]) || (U_store && !U_store[c])) {
      set_error("gpt_sgld_regression_chains: null per-chain pointer");
      return GPT_ERR_BAD_DIMS;
    }
  }
  const size_t nphi = (size_t)cfg->n * cfg->D * cfg->N;
  // one device copy per distinct host array
  std::vector<std::unique_ptr<DevMem>> mem;
  std::unordered_map<const double*, const double*> dev_of;
  auto upload = [&](const double* h, size_t count, const double** out) -> int {
    auto it = dev_of.find(h);
    if (it != dev_of.end()) { *out = it->second; return GPT_OK; }
    std::unique_ptr<DevMem> m(new DevMem());
    HIPCHK(m->alloc(8 * count));
    HIPCHK(hipMemcpy(m->p, h, 8 * count, hipMemcpyHostToDevice));
    *out = m->as<double>();
    dev_of[h] = *out;
    mem.push_back(std::move(m));
    return GPT_OK;
  };
  std::vector<const double*> dphi(nchains), dy(nchains);
  for (int c = 0; c < nchains; ++c) {
    int rc = upload(phi[c], nphi, &dphi[c]);
    if (rc == GPT_OK) rc = upload(y[c], (size_t)cfg->N, &dy[c]);
    if (rc != GPT_OK) return rc;
  }
  gpt_sgld_session* s = nullptr;
  int rc = gpt_sgld_session_create(cfg, nchains, seeds, dphi.data(), dy.data(), I, stores ? 1 : 0,
                                   nullptr, &s);
  if (rc != GPT_OK) return rc;
  std::unique_ptr<gpt_sgld_session, void (*)(gpt_sgld_session*)> guard(s, gpt_sgld_session_destroy);
  if (epsw || epsU || signal_var)
    for (int c = 0; c < nchains; ++c) {
      rc = gpt_sgld_session_set_hyper(s, c, epsw ? epsw[c] : cfg->epsw, epsU ? epsU[c] : cfg->epsU,
                                      signal_var ? signal_var[c] : cfg->signal_var, cfg->sigma_w);
      if (rc != GPT_OK) return rc;
    }
  rc = gpt_sgld_session_run(s, s->total_steps);
  if (rc != GPT_OK) return rc;
  for (int c = 0; c < nchains; ++c) {
    rc = gpt_sgld_session_fetch(s, c, w_store ? w_store[c] : nullptr, U_store ? U_store[c] : nullptr,
                                nullptr, &status[c]);
    if (rc != GPT_OK) return rc;
  }
  return GPT_OK;
}

extern "C" int gpt_sgld_rmsprop(const gpt_sgld_config* cfg, double epsilon, double alpha,
                                const double* phi, const double* y, const int32_t* I,
                                const double* w_init, const double* U_init, double* w_store,
                                double* U_store, double* diag) {
  if (!(epsilon > 0)) { set_error("RMSprop needs epsilon > 0"); return GPT_ERR_BAD_DIMS; }
  return host_sampler(cfg, phi, y, I, w_init, U_init, w_store, U_store, diag, 4, epsilon, alpha);
}

extern "C" int gpt_sgld_wonly(const gpt_sgld_config* cfg, const double* phi, const double* y,
                              const int32_t* I, const double* w_init, const double* U_init,
                              double* w_store, double* U_out, double* diag) {
  if (!cfg || !cfg->stiefel || !cfg->langevin) {
    set_error("GPT_SGLDERMw: U is a uniform Stiefel draw and w takes SGLD steps (stiefel = langevin = 1)");
    return GPT_ERR_BAD_DIMS;
  }
  return host_sampler(cfg, phi, y, I, w_init, U_init, w_store, nullptr, diag, 16, 0.0, 0.0, U_out);
}

extern "C" int gpt_sgld_classification(const gpt_sgld_config* cfg, const double* phi,
                                       const double* y, const int32_t* I, const double* w_init,
                                       const double* U_init, double* w_store, double* U_store,
                                       double* diag) {
  if (!valid_cfg(cfg)) return GPT_ERR_BAD_DIMS;
  if (!phi || !y || !I) { set_error("null input"); return GPT_ERR_BAD_DIMS; }
  const int64_t N = cfg->N, Q = cfg->Q, nur = cfg->n * cfg->r * cfg->D;
  long long lo = 0, hi = 0;
  for (int64_t i = 0; i < N; ++i) {
    const double v = y[i];
    if (v != std::floor(v)) { set_error("class labels must be integers"); return GPT_ERR_BAD_DIMS; }
    lo = i ? std::min(lo, (long long)v) : (long long)v;
    hi = i ? std::max(hi, (long long)v) : (long long)v;
  }
  if (lo != 1 || hi > 64) {
    set_error("class labels must be 1..C (C <= 64): they index the classes (GPT_SGLD.jl:520)");
    return GPT_ERR_BAD_DIMS;
  }
  const int ncls = (int)hi;
  const size_t nphi = (size_t)cfg->n * cfg->D * N;
  DevMem dphi, dy;
  HIPCHK(dphi.alloc(8 * nphi));
  HIPCHK(dy.alloc(8 * (size_t)N));
  HIPCHK(hipMemcpy(dphi.p, phi, 8 * nphi, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dy.p, y, 8 * (size_t)N, hipMemcpyHostToDevice));
  std::vector<uint64_t> seeds(ncls, cfg->seed);
  std::vector<const double*> pp(ncls, dphi.as<double>()), yy(ncls, dy.as<double>());
  gpt_sgld_session* s = nullptr;
  const int flags = ((w_store || U_store) ? 1 : 0) | (diag ? 2 : 0) | 32;
  int rc = gpt_sgld_session_create(cfg, ncls, seeds.data(), pp.data(), yy.data(), I, flags, nullptr, &s);
  if (rc != GPT_OK) return rc;
  std::unique_ptr<gpt_sgld_session, void (*)(gpt_sgld_session*)> guard(s, gpt_sgld_session_destroy);
  rc = session_alloc_aux(s);
  if (rc != GPT_OK) return rc;
  std::vector<double> w0((size_t)Q), U0((size_t)nur);
  for (int c = 0; c < ncls; ++c) {
    rc = gpt_sgld_session_set_hyper(s, c, cfg->epsw, cfg->epsU, 1.0, 1.0);   // no noise variance
    if (rc != GPT_OK) return rc;
    if (w_init && U_init) {
      rc = session_set_state(s, c, w_init + (size_t)Q * c, U_init + (size_t)nur * c);
    } else {
      host_init_state((int)cfg->n, (int)cfg->r, (int)cfg->D, (int)Q, cfg->seed, cfg->stiefel != 0,
                      1.0, w0.data(), U0.data(), c, true);
      rc = session_set_state(s, c, w0.data(), U0.data());
    }
    if (rc != GPT_OK) return rc;
  }
  rc = gpt_sgld_session_run(s, s->total_steps);
  if (rc != GPT_OK) return rc;
  const int64_t T = s->nstore, steps = s->total_steps;
  std::vector<double> wb(w_store ? (size_t)Q * T : 0), Ub(U_store ? (size_t)nur * T : 0),
      db(diag ? (size_t)(1 + cfg->D) * steps : 0);
  bool bad = false;
  for (int c = 0; c < ncls; ++c) {
    int32_t st = 0;
    rc = gpt_sgld_session_fetch(s, c, w_store ? wb.data() : nullptr, U_store ? Ub.data() : nullptr,
                                diag ? db.data() : nullptr, &st);
    if (rc != GPT_OK) return rc;
    bad |= st != 0;
    for (int64_t z = 0; z < T; ++z) {      // (Q, C, T) and (n, r, D, C, T) column-major
      if (w_store) std::memcpy(w_store + ((size_t)z * ncls + c) * Q, wb.data() + (size_t)z * Q, 8 * Q);
      if (U_store) std::memcpy(U_store + ((size_t)z * ncls + c) * nur, Ub.data() + (size_t)z * nur, 8 * nur);
    }
    if (diag) std::memcpy(diag + (size_t)c * db.size(), db.data(), 8 * db.size());
  }
  if (bad) {                               // GPT_SGLD.jl:632-634: zero stores
    if (w_store) std::memset(w_store, 0, 8 * (size_t)Q * ncls * T);
    if (U_store) std::memset(U_store, 0, 8 * (size_t)nur * ncls * T);
    set_error("Get NaN when moving along Geodesic. Try smaller epsU");
    return GPT_ERR_NAN_GEODESIC;
  }
  return GPT_OK;
}

extern "C" int gpt_samplenz(int64_t r, int64_t D, int64_t Q, uint64_t seed, int32_t* I_out) {
  if (r < 1 || D < 1 || Q < 1 || !I_out) { set_error("bad samplenz arguments"); return GPT_ERR_BAD_DIMS; }
  unsigned __int128 M = 1;
  for (int k = 0; k < D; ++k) {
    M *= (unsigned __int128)r;
    if (M > ((unsigned __int128)1 << 62)) { set_error("r^D too large"); return GPT_ERR_BAD_DIMS; }
  }
  if ((unsigned __int128)Q > M) { set_error("Q must be <= r^D"); return GPT_ERR_BAD_DIMS; }
  const uint64_t MM = (uint64_t)M;
  std::unordered_map<uint64_t, uint64_t> sw;
  auto get = [&sw](uint64_t x) { auto it = sw.find(x); return it == sw.end() ? x : it->second; };
  for (int64_t i = 0; i < Q; ++i) {
    const U4 x = philox4x32((uint32_t)i, 0, kSampleNZ, 0, seed);
    const uint64_t u = ((uint64_t)x.x << 32) | x.y;
    const uint64_t j = (uint64_t)i + (uint64_t)(((unsigned __int128)u * (MM - (uint64_t)i)) >> 64);
    const uint64_t vi = get(i), vj = get(j);
    sw[i] = vj;
    sw[j] = vi;
    uint64_t v = vj;  // L[i]; I[i,:] = digits(L, r, D) + 1
    for (int64_t k = 0; k < D; ++k) {
      I_out[i + Q * k] = (int32_t)(v % (uint64_t)r) + 1;
      v /= (uint64_t)r;
    }
  }
  return GPT_OK;
}

extern "C" int gpt_feature_inputs(int64_t n, int64_t D, uint64_t seed, double* Z_out, double* b_out) {
  if (n < 1 || D < 1) { set_error("bad dims"); return GPT_ERR_BAD_DIMS; }
  for (int64_t e = 0; e < n * D; ++e) {
    if (Z_out) Z_out[e] = host_normal(seed, (uint32_t)e, 0, kFeatZ, 0);
    if (b_out) {
      const U4 x = philox4x32((uint32_t)e, 0, kFeatB, 0, seed);
      b_out[e] = 2.0 * 3.141592653589793 * u53(x.x, x.y);
    }
  }
  return GPT_OK;
}

// Generation-A feature inputs (GPT_SGLD_p.jl:40-54): Z = randn(n,D) (the Gen-C Z stream) and
// b = randn(n,D) on the FEAT_B stream with c3 = 1 (Gen C draws b = 2π·rand on c3 = 0).
extern "C" int gpt_feature_inputs_a(int64_t n, int64_t D, uint64_t seed, double* Z_out, double* b_out) {
  if (n < 1 || D < 1) { set_error("bad dims"); return GPT_ERR_BAD_DIMS; }
  for (int64_t e = 0; e < n * D; ++e) {
    if (Z_out) Z_out[e] = host_normal(seed, (uint32_t)e, 0, kFeatZ, 0);
    if (b_out) b_out[e] = host_normal(seed, (uint32_t)e, 0, kFeatB, 1);
  }
  return GPT_OK;
}

// randperm(N) + phi = phi[:,:,perm] (GPT_SGLD.jl:373-374) for `epochs` epochs, built on the device
// by the sampler's own kernel (order.hip).  out: (N, epochs) column-major, 0-based rows.
extern "C" int gpt_epoch_orders(int64_t N, uint64_t seed, int64_t epochs, int32_t* out) {
  if (N < 1 || N > (1LL << 31) - 1 || epochs < 0 || epochs > (1 << 20) || (epochs && !out)) {
    set_error("bad epoch-order arguments"); return GPT_ERR_BAD_DIMS;
  }
  DevMem ring, cd, ws;
  HIPCHK(ring.alloc(8 * (size_t)N));
  ChainDesc C{};
  C.order = ring.as<int32_t>();
  C.seed = seed;
  HIPCHK(cd.alloc(sizeof(ChainDesc)));
  HIPCHK(hipMemcpy(cd.p, &C, sizeof(ChainDesc), hipMemcpyHostToDevice));
  if (const size_t wsi = epoch_order_ws_ints((int)N, 1)) HIPCHK(ws.alloc(4 * wsi));
  for (int64_t e = 0; e < epochs; ++e) {
    HIPCHK(launch_epoch_order(cd.as<ChainDesc>(), 1, (int)N, 1, 0, nullptr, 0, (int)e,
                              ws.as<int32_t>(), nullptr));
    HIPCHK(hipMemcpy(out + (size_t)e * N, ring.as<int32_t>() + (size_t)(e & 1) * N, 4 * (size_t)N,
                     hipMemcpyDeviceToHost));
  }
  return GPT_OK;
}

static int feature_common(bool tensor, const double* X, int64_t N, int64_t D, const double* ls,
                          int64_t ls_len, double sigma_rbf, double phi_scale, const double* Z,
                          const double* b, int64_t n, double* phi_out) {
  if (!X || !ls || !Z || !b || !phi_out || N < 1 || D < 1 || n < 1) {
    set_error("bad feature arguments"); return GPT_ERR_BAD_DIMS;
  }
  if (ls_len != 1 && ls_len != D) {
    set_error("dimensions of X and length_scale do not match"); return GPT_ERR_BAD_DIMS;
  }
  std::vector<double> lsv(D);
  for (int64_t k = 0; k < D; ++k) lsv[k] = ls[ls_len == 1 ? 0 : k];
  const size_t nphi = tensor ? (size_t)n * D * N : (size_t)n * N;
  const size_t nb = tensor ? (size_t)n * D : (size_t)n;
  DevMem dX, dls, dZ, db, dphi;
  HIPCHK(dX.alloc(8 * (size_t)N * D));
  HIPCHK(dls.alloc(8 * (size_t)D));
  HIPCHK(dZ.alloc(8 * (size_t)n * D));
  HIPCHK(db.alloc(8 * nb));
  HIPCHK(dphi.alloc(8 * nphi));
  HIPCHK(hipMemcpy(dX.p, X, 8 * (size_t)N * D, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dls.p, lsv.data(), 8 * (size_t)D, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dZ.p, Z, 8 * (size_t)n * D, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(db.p, b, 8 * nb, hipMemcpyHostToDevice));
  hipError_t e;
  if (tensor) {
    const double c = phi_scale * std::pow(sigma_rbf, 1.0 / (double)D) * std::sqrt(2.0 / (double)n);
    e = launch_feature(dX.as<double>(), N, (int)D, dls.as<double>(), c, dZ.as<double>(),
                       db.as<double>(), (int)n, dphi.as<double>(), nullptr);
  } else {
    const double c = std::sqrt(2.0 / (double)n) * sigma_rbf;
    e = launch_feature_notensor(dX.as<double>(), N, (int)D, dls.as<double>(), c, dZ.as<double>(),
                                db.as<double>(), (int)n, dphi.as<double>(), nullptr);
  }
  if (e != hipSuccess) return hip_fail(e, "feature kernel");
  HIPCHK(hipMemcpy(phi_out, dphi.p, 8 * nphi, hipMemcpyDeviceToHost));
  return GPT_OK;
}

extern "C" int gpt_feature_dev(const double* X_dev, int64_t N, int64_t D, const double* ls_dev,
                               int64_t ls_len, double sigma_rbf, double phi_scale,
                               const double* Z_dev, const double* b_dev, int64_t n, double* phi_dev,
                               void* hip_stream) {
  if (!X_dev || !ls_dev || !Z_dev || !b_dev || !phi_dev || N < 1 || D < 1 || n < 1 || ls_len != D) {
    set_error("bad gpt_feature_dev arguments (ls_len must equal D)"); return GPT_ERR_BAD_DIMS;
  }
  const double c = phi_scale * std::pow(sigma_rbf, 1.0 / (double)D) * std::sqrt(2.0 / (double)n);
  hipError_t e = launch_feature(X_dev, N, (int)D, ls_dev, c, Z_dev, b_dev, (int)n, phi_dev,
                                (hipStream_t)hip_stream);
  if (e != hipSuccess) return hip_fail(e, "feature kernel");
  return GPT_OK;
}

extern "C" int gpt_feature(const double* X, int64_t N, int64_t D, const double* length_scale,
                           int64_t ls_len, double sigma_rbf, double phi_scale, const double* Z,
                           const double* b, int64_t n, double* phi_out) {
  return feature_common(true, X, N, D, length_scale, ls_len, sigma_rbf, phi_scale, Z, b, n, phi_out);
}

extern "C" int gpt_feature_notensor(const double* X, int64_t N, int64_t D, const double* length_scale,
                                    int64_t ls_len, double sigma_rbf, const double* Z,
                                    const double* b, int64_t n, double* phi_out) {
  return feature_common(false, X, N, D, length_scale, ls_len, sigma_rbf, 1.0, Z, b, n, phi_out);
}

static bool valid_pred(int64_t n, int64_t D, int64_t Ntest, int64_t r, int64_t Q) {
  if (n < 1 || D < 1 || Ntest < 0 || r < 1 || Q < 1) { set_error("bad pred dims"); return false; }
  if (D > kDMax) { set_error("D > 16 unsupported"); return false; }
  if (!rank_supported((int)r)) { set_error("rank not instantiated"); return false; }
  if (pred_lds_bytes((int)n, (int)D, (int)r, (int)Q) > 160 * 1024) { set_error("pred LDS too large"); return false; }
  return true;
}

extern "C" int gpt_pred_dev(const double* w_dev, const double* U_dev, const int32_t* I0_dev,
                            const double* phitest_dev, int64_t n, int64_t D, int64_t Ntest,
                            int64_t r, int64_t Q, int64_t S, double* fhat_dev, void* hip_stream) {
  if (!valid_pred(n, D, Ntest, r, Q)) return GPT_ERR_BAD_DIMS;
  hipError_t e = launch_pred(w_dev, U_dev, I0_dev, phitest_dev, (int)n, (int)D, Ntest, (int)r,
                             (int)Q, (int)S, fhat_dev, (hipStream_t)hip_stream);
  if (e != hipSuccess) return hip_fail(e, "pred kernel");
  return GPT_OK;
}

extern "C" int gpt_pred_trim_pool(void) {
  HIPCHK(pred_trim_pools());
  return GPT_OK;
}

extern "C" int gpt_pred_dev_timed(const double* w_dev, const double* U_dev, const int32_t* I0_dev,
                                  const double* phitest_dev, int64_t n, int64_t D, int64_t Ntest,
                                  int64_t r, int64_t Q, int64_t S, double* fhat_dev,
                                  void* hip_stream, double* ms_out) {
  if (!valid_pred(n, D, Ntest, r, Q)) return GPT_ERR_BAD_DIMS;
  if (!ms_out) { set_error("gpt_pred_dev_timed: ms_out is null"); return GPT_ERR_BAD_DIMS; }
  PredPhaseTiming tm;
  hipError_t e = launch_pred(w_dev, U_dev, I0_dev, phitest_dev, (int)n, (int)D, Ntest, (int)r,
                             (int)Q, (int)S, fhat_dev, (hipStream_t)hip_stream, &tm);
  if (e != hipSuccess) return hip_fail(e, "pred kernel");
  HIPCHK(hipStreamSynchronize((hipStream_t)hip_stream));
  ms_out[0] = tm.gemm_ms;
  ms_out[1] = tm.vphase_ms;
  return GPT_OK;
}

static int pred_host(const double* w, const double* U, const int32_t* I, const double* phitest,
                     const double* ytest, int64_t n, int64_t D, int64_t Ntest, int64_t r,
                     int64_t Q, int64_t S, double scale, double* fhat_out, double* mean_out,
                     double* rmse_out) {
  if (!valid_pred(n, D, Ntest, r, Q) || S < 1) return GPT_ERR_BAD_DIMS;
  std::vector<int32_t> I0((size_t)Q * D);
  for (size_t x = 0; x < I0.size(); ++x) {
    if (I[x] < 1 || I[x] > r) { set_error("I entries must be in 1..r"); return GPT_ERR_BAD_DIMS; }
    I0[x] = I[x] - 1;
  }
  DevMem dw, dU, dI, dphi, df, dy, dmean, dsse;
  HIPCHK(dw.alloc(8 * (size_t)Q * S));
  HIPCHK(dU.alloc(8 * (size_t)n * r * D * S));
  HIPCHK(dI.alloc(4 * I0.size()));
  HIPCHK(dphi.alloc(8 * (size_t)n * D * Ntest));
  HIPCHK(df.alloc(8 * (size_t)Ntest * S));
  HIPCHK(hipMemcpy(dw.p, w, 8 * (size_t)Q * S, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dU.p, U, 8 * (size_t)n * r * D * S, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dI.p, I0.data(), 4 * I0.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dphi.p, phitest, 8 * (size_t)n * D * Ntest, hipMemcpyHostToDevice));
  int rc = gpt_pred_dev(dw.as<double>(), dU.as<double>(), dI.as<int32_t>(), dphi.as<double>(), n,
                        D, Ntest, r, Q, S, df.as<double>(), nullptr);
  if (rc != GPT_OK) return rc;
  if (fhat_out) HIPCHK(hipMemcpy(fhat_out, df.p, 8 * (size_t)Ntest * S, hipMemcpyDeviceToHost));
  if (ytest) {
    HIPCHK(dy.alloc(8 * (size_t)Ntest));
    HIPCHK(dmean.alloc(8 * (size_t)Ntest));
    HIPCHK(dsse.alloc(8 * (size_t)(S + 1)));
    HIPCHK(hipMemcpy(dy.p, ytest, 8 * (size_t)Ntest, hipMemcpyHostToDevice));
    hipError_t e = launch_mean_rmse(df.as<double>(), dy.as<double>(), Ntest, (int)S,
                                    dmean.as<double>(), dsse.as<double>(), nullptr);
    if (e != hipSuccess) return hip_fail(e, "mean/sse kernel");
    double sse = 0.0;
    HIPCHK(hipMemcpy(&sse, dsse.p, 8, hipMemcpyDeviceToHost));
    if (mean_out) HIPCHK(hipMemcpy(mean_out, dmean.p, 8 * (size_t)Ntest, hipMemcpyDeviceToHost));
    if (rmse_out) *rmse_out = scale * std::sqrt(sse / (double)Ntest);
  }
  HIPCHK(hipDeviceSynchronize());
  return GPT_OK;
}

extern "C" int gpt_pred(const double* w, const double* U, const int32_t* I, const double* phitest,
                        int64_t n, int64_t D, int64_t Ntest, int64_t r, int64_t Q, double* fhat_out) {
  return pred_host(w, U, I, phitest, nullptr, n, D, Ntest, r, Q, 1, 1.0, fhat_out, nullptr, nullptr);
}

extern "C" int gpt_pred_mean(const double* w_store, const double* U_store, const int32_t* I,
                             const double* phitest, const double* ytest, int64_t n, int64_t D,
                             int64_t Ntest, int64_t r, int64_t Q, int64_t S, double scale,
                             double* mean_out, double* rmse_out) {
  if (!ytest) { set_error("ytest required"); return GPT_ERR_BAD_DIMS; }
  return pred_host(w_store, U_store, I, phitest, ytest, n, D, Ntest, r, Q, S, scale, nullptr,
                   mean_out, rmse_out);
}

extern "C" int gpt_pred_mean_x(const double* w_store, const double* U_store, const int32_t* I,
                               const double* Xtest, const double* ytest, int64_t Ntest, int64_t D,
                               const double* length_scale, int64_t ls_len, double sigma_rbf,
                               double phi_scale, const double* Z, const double* b, int64_t n,
                               int64_t r, int64_t Q, int64_t S, double scale, double* mean_out,
                               double* rmse_out, double* sample_rmse_out) {
  if (!w_store || !U_store || !I || !Xtest || !ytest || !length_scale || !Z || !b || S < 1) {
    set_error("bad pred_mean_x arguments"); return GPT_ERR_BAD_DIMS;
  }
  if (ls_len != 1 && ls_len != D) {
    set_error("dimensions of X and length_scale do not match"); return GPT_ERR_BAD_DIMS;
  }
  if (!valid_pred(n, D, Ntest, r, Q)) return GPT_ERR_BAD_DIMS;
  if (pred_x_lds_bytes((int)n, (int)D, (int)r, (int)Q) > 160 * 1024) {
    set_error("pred LDS too large"); return GPT_ERR_BAD_DIMS;
  }
  std::vector<int32_t> I0((size_t)Q * D);
  for (size_t x = 0; x < I0.size(); ++x) {
    if (I[x] < 1 || I[x] > r) { set_error("I entries must be in 1..r"); return GPT_ERR_BAD_DIMS; }
    I0[x] = I[x] - 1;
  }
  std::vector<double> lsv(D);
  for (int64_t k = 0; k < D; ++k) lsv[k] = length_scale[ls_len == 1 ? 0 : k];
  const double c = phi_scale * std::pow(sigma_rbf, 1.0 / (double)D) * std::sqrt(2.0 / (double)n);
  DevMem dw, dU, dI, dX, dls, dZ, db, df, dy, dmean, dsse;
  HIPCHK(dw.alloc(8 * (size_t)Q * S));
  HIPCHK(dU.alloc(8 * (size_t)n * r * D * S));
  HIPCHK(dI.alloc(4 * I0.size()));
  HIPCHK(dX.alloc(8 * (size_t)Ntest * D));
  HIPCHK(dls.alloc(8 * (size_t)D));
  HIPCHK(dZ.alloc(8 * (size_t)n * D));
  HIPCHK(db.alloc(8 * (size_t)n * D));
  HIPCHK(df.alloc(8 * (size_t)Ntest * S));
  HIPCHK(dy.alloc(8 * (size_t)Ntest));
  HIPCHK(dmean.alloc(8 * (size_t)Ntest));
  HIPCHK(dsse.alloc(8 * (size_t)(S + 1)));
  HIPCHK(hipMemcpy(dw.p, w_store, 8 * (size_t)Q * S, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dU.p, U_store, 8 * (size_t)n * r * D * S, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dI.p, I0.data(), 4 * I0.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dX.p, Xtest, 8 * (size_t)Ntest * D, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dls.p, lsv.data(), 8 * (size_t)D, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dZ.p, Z, 8 * (size_t)n * D, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(db.p, b, 8 * (size_t)n * D, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dy.p, ytest, 8 * (size_t)Ntest, hipMemcpyHostToDevice));
  // Default: the test features are formed once on the device (feature_kernel, the same doubles
  // as gpt_feature) and every sample is predicted by the stacked-sample MFMA path, which reads
  // them through L2 per group of samples.  GPTSGLD_PRED=direct: pred_x_kernel, which forms the
  // features inside every sample's prediction tile (no phitest array).
  const char* pev = std::getenv("GPTSGLD_PRED");
  hipError_t e;
  DevMem dphi;
  if (pev && std::strcmp(pev, "direct") == 0) {
    e = launch_pred_x(dw.as<double>(), dU.as<double>(), dI.as<int32_t>(), dX.as<double>(),
                      dls.as<double>(), dZ.as<double>(), db.as<double>(), c, (int)n, (int)D,
                      Ntest, (int)r, (int)Q, (int)S, df.as<double>(), nullptr);
    if (e != hipSuccess) return hip_fail(e, "pred_x kernel");
  } else {
    HIPCHK(dphi.alloc(8 * (size_t)n * D * Ntest));
    e = launch_feature(dX.as<double>(), Ntest, (int)D, dls.as<double>(), c, dZ.as<double>(),
                       db.as<double>(), (int)n, dphi.as<double>(), nullptr);
    if (e != hipSuccess) return hip_fail(e, "feature kernel");
    e = launch_pred(dw.as<double>(), dU.as<double>(), dI.as<int32_t>(), dphi.as<double>(), (int)n,
                    (int)D, Ntest, (int)r, (int)Q, (int)S, df.as<double>(), nullptr);
    if (e != hipSuccess) return hip_fail(e, "pred kernels");
  }
  e = launch_mean_rmse(df.as<double>(), dy.as<double>(), Ntest, (int)S, dmean.as<double>(),
                       dsse.as<double>(), nullptr);
  if (e != hipSuccess) return hip_fail(e, "mean/sse kernel");
  std::vector<double> sse((size_t)S + 1);
  HIPCHK(hipMemcpy(sse.data(), dsse.p, 8 * sse.size(), hipMemcpyDeviceToHost));
  if (mean_out) HIPCHK(hipMemcpy(mean_out, dmean.p, 8 * (size_t)Ntest, hipMemcpyDeviceToHost));
  if (rmse_out) *rmse_out = scale * std::sqrt(sse[0] / (double)Ntest);
  if (sample_rmse_out)
    for (int64_t z = 0; z < S; ++z) sample_rmse_out[z] = scale * std::sqrt(sse[1 + z] / (double)Ntest);
  return GPT_OK;
}

extern "C" int gpt_gpnt_sgld(const double* phi, const double* y, int64_t n, int64_t N,
                             double signal_var, double sigma_theta, int64_t m, double eps_theta,
                             double decay_rate, int64_t burnin, int64_t maxepoch, uint64_t seed,
                             double* theta_store) {
  if (!phi || !y || !theta_store || n < 1 || N < 1 || m < 1 || burnin < 0 || maxepoch < 0) {
    set_error("bad GPNT_SGLD arguments"); return GPT_ERR_BAD_DIMS;
  }
  const long long nb = (N + m - 1) / m;
  const int epochs = (int)(burnin + maxepoch);
  const long long total = (long long)epochs * nb;
  std::vector<double> th0(n);
  for (int64_t j = 0; j < n; ++j) th0[j] = sigma_theta * host_normal(seed, (uint32_t)j, 0, kThetaInit, 0);
  std::vector<int32_t> ord((size_t)epochs * N);
  host_epoch_orders((int)N, seed, epochs, ord.data());
  DevMem dphi, dy, dord, dth, dst, dstat, dtb;
  HIPCHK(dphi.alloc(8 * (size_t)n * N));
  HIPCHK(dy.alloc(8 * (size_t)N));
  HIPCHK(dord.alloc(4 * ord.size()));
  HIPCHK(dth.alloc(8 * (size_t)n));
  HIPCHK(dst.alloc(8 * (size_t)n * total));
  HIPCHK(dstat.alloc(4));
  HIPCHK(dtb.alloc(8));
  HIPCHK(hipMemcpy(dphi.p, phi, 8 * (size_t)n * N, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dy.p, y, 8 * (size_t)N, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dord.p, ord.data(), 4 * ord.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dth.p, th0.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(dstat.p, 0, 4));
  HIPCHK(hipMemset(dtb.p, 0, 8));
  for (long long t = 0; t < total; ++t) {
    hipError_t e = launch_gpnt(dphi.as<double>(), dy.as<double>(), dord.as<int32_t>(), (int)n, (int)N,
                               (int)m, (int)nb, total, signal_var, sigma_theta, eps_theta, decay_rate,
                               seed, dth.as<double>(), dst.as<double>(), dstat.as<int32_t>(),
                               dtb.as<long long>(), (int)t, nullptr);
    if (e != hipSuccess) return hip_fail(e, "gpnt kernel");
  }
  int32_t st = 0;
  HIPCHK(hipMemcpy(&st, dstat.p, 4, hipMemcpyDeviceToHost));
  if (st) {
    std::memset(theta_store, 0, 8 * (size_t)n * total);
    set_error("Get NaN in theta. Try smaller epsilon");
    return GPT_ERR_NAN_THETA;
  }
  HIPCHK(hipMemcpy(theta_store, dst.p, 8 * (size_t)n * total, hipMemcpyDeviceToHost));
  return GPT_OK;
}

extern "C" int gpt_tgp_gibbs(const double* b, const double* y, int64_t n, int64_t D, int64_t N,
                             int64_t r, int64_t q, double sigma, int64_t num_iterations,
                             int64_t burnin, uint64_t seed, const int32_t* I, double* W_out,
                             double* U_out, int32_t* I_out) {
  if (!b || !y || !W_out || !U_out || n < 1 || D < 1 || N < 1 || q < 1 || burnin < 0 ||
      num_iterations <= burnin || !(sigma > 0)) {
    set_error("bad GPT_inf arguments"); return GPT_ERR_BAD_DIMS;
  }
  if (!rank_supported((int)r)) { set_error("rank r not instantiated (supported: 1-6,8,10,12,15,16,20)"); return GPT_ERR_BAD_DIMS; }
  if (n * r > 8192 || q > 8192 || (double)n * D * N > 2e9) { set_error("dimension too large"); return GPT_ERR_BAD_DIMS; }
  std::vector<int32_t> I0((size_t)q * D);
  for (int64_t e = 0; e < q * D; ++e) {
    int32_t v;
    if (I) {
      v = I[e];
      if (v < 1 || v > r) { set_error("I entries must be in 1..r"); return GPT_ERR_BAD_DIMS; }
    } else {
      const U4 x = philox4x32((uint32_t)e, 0, kTgpI, 0, seed);
      v = 1 + (int32_t)(((uint64_t)x.x * (uint64_t)r) >> 32);
    }
    if (I_out) I_out[e] = v;
    I0[e] = v - 1;
  }
  const int64_t nr = n * r, T = num_iterations - burnin;
  std::vector<double> U0((size_t)nr * D);
  const double su = std::sqrt(1.0 / (double)r);
  for (int64_t d = 0; d < D; ++d)
    for (int64_t e = 0; e < nr; ++e) U0[d * nr + e] = su * host_normal(seed, (uint32_t)e, 0, kTgpUInit, (uint32_t)d);
  DevMem db, dy, dI, dU, dW, dUh, dst;
  HIPCHK(db.alloc(8 * (size_t)n * D * N));
  HIPCHK(dy.alloc(8 * (size_t)N));
  HIPCHK(dI.alloc(4 * I0.size()));
  HIPCHK(dU.alloc(8 * U0.size()));
  HIPCHK(dW.alloc(8 * (size_t)q * T));
  HIPCHK(dUh.alloc(8 * (size_t)nr * D * T));
  HIPCHK(dst.alloc(4));
  HIPCHK(hipMemcpy(db.p, b, 8 * (size_t)n * D * N, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dy.p, y, 8 * (size_t)N, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dI.p, I0.data(), 4 * I0.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dU.p, U0.data(), 8 * U0.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemset(dst.p, 0, 4));
  hipError_t e = tgp_gibbs(db.as<double>(), dy.as<double>(), (int)n, (int)D, N, (int)r, (int)q, sigma,
                           (int)num_iterations, (int)burnin, seed, dI.as<int32_t>(), dU.as<double>(),
                           dW.as<double>(), dUh.as<double>(), dst.as<int32_t>(), nullptr);
  if (e != hipSuccess) return hip_fail(e, "tgp gibbs");
  HIPCHK(hipStreamSynchronize(nullptr));
  int32_t stt = 0;
  HIPCHK(hipMemcpy(&stt, dst.p, 4, hipMemcpyDeviceToHost));
  if (stt) { set_error("PosDefException: Gibbs precision matrix not positive definite"); return GPT_ERR_NOT_SPD; }
  HIPCHK(hipMemcpy(W_out, dW.p, 8 * (size_t)q * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(U_out, dUh.p, 8 * (size_t)nr * D * T, hipMemcpyDeviceToHost));
  return GPT_OK;
}

extern "C" int gpt_gmc(const double* phi, const double* y, int64_t n, int64_t D, int64_t N,
                       int64_t r, int64_t Q, const int32_t* I, double signal_var, double epsw,
                       double epsU, int64_t burnin, int64_t maxepoch, int64_t L, uint64_t seed,
                       const double* w_init, const double* U_init, double* w_store,
                       double* U_store, double* accept_prob) {
  if (!phi || !y || !I || !w_store || !U_store || !accept_prob || n < 1 || D < 1 || N < 1 ||
      Q < 1 || burnin < 0 || maxepoch < 0 || L < 1 || !(signal_var > 0)) {
    set_error("bad GPT_GMC arguments"); return GPT_ERR_BAD_DIMS;
  }
  if (!rank_supported((int)r) || !gmc_supported((int)n, (int)r)) {
    set_error("GPT_GMC: rank not instantiated or n*r too large for one workgroup's LDS");
    return GPT_ERR_BAD_DIMS;
  }
  std::vector<int32_t> I0((size_t)Q * D);
  for (size_t x = 0; x < I0.size(); ++x) {
    if (I[x] < 1 || I[x] > r) { set_error("I entries must be in 1..r"); return GPT_ERR_BAD_DIMS; }
    I0[x] = I[x] - 1;
  }
  const size_t nm = (size_t)n * r * D, nphi = (size_t)n * D * N;
  std::vector<double> w0((size_t)Q), U0(nm);
  host_init_state((int)n, (int)r, (int)D, (int)Q, seed, true, 1.0, w0.data(), U0.data());
  if (w_init) std::memcpy(w0.data(), w_init, 8 * (size_t)Q);
  if (U_init) std::memcpy(U0.data(), U_init, 8 * nm);
  DevMem dphi, dy, dI, dw, dU, dst;
  HIPCHK(dphi.alloc(8 * nphi));
  HIPCHK(dy.alloc(8 * (size_t)N));
  HIPCHK(dI.alloc(4 * I0.size()));
  HIPCHK(dw.alloc(8 * (size_t)Q));
  HIPCHK(dU.alloc(8 * nm));
  HIPCHK(dst.alloc(4));
  HIPCHK(hipMemcpy(dphi.p, phi, 8 * nphi, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dy.p, y, 8 * (size_t)N, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dI.p, I0.data(), 4 * I0.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dw.p, w0.data(), 8 * (size_t)Q, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dU.p, U0.data(), 8 * nm, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(dst.p, 0, 4));
  std::memset(w_store, 0, 8 * (size_t)Q * maxepoch);
  std::memset(U_store, 0, 8 * nm * maxepoch);
  hipError_t e = gmc_run(dphi.as<double>(), dy.as<double>(), dI.as<int32_t>(), (int)n, (int)D, N,
                         (int)r, (int)Q, signal_var, epsw, epsU, (int)burnin, (int)maxepoch, (int)L,
                         seed, dw.as<double>(), dU.as<double>(), w_store, U_store, accept_prob,
                         dst.as<int32_t>(), nullptr);
  if (e != hipSuccess) return hip_fail(e, "GPT_GMC");
  int32_t bad = 0;
  HIPCHK(hipMemcpy(&bad, dst.p, 4, hipMemcpyDeviceToHost));
  if (bad) {                         // GPT_SGLD.jl:757: zeros and NaN acceptance probabilities
    std::memset(w_store, 0, 8 * (size_t)Q * maxepoch);
    std::memset(U_store, 0, 8 * nm * maxepoch);
    for (int64_t z = 0; z < burnin + maxepoch; ++z) accept_prob[z] = std::nan("");
    set_error("Get NaN when moving along Geodesic. Try smaller epsU");
    return GPT_ERR_NAN_GEODESIC;
  }
  return GPT_OK;
}

// Non-cumulative epoch permutation randperm(N) on the PERM stream of `epoch` (the shuffles of
// 100k_movielensExperiment.jl:451-452 permute the original ratings every epoch).
static void host_randperm(int N, uint64_t seed, int epoch, int32_t* p) {
  for (int i = 0; i < N; ++i) p[i] = i;
  for (int i = N - 1; i >= 1; --i) {
    const uint32_t x = philox4x32((uint32_t)i, (uint32_t)epoch, kPerm, 0, seed).x;
    const int j = (int)(((uint64_t)x * (uint64_t)(i + 1)) >> 32);
    std::swap(p[i], p[j]);
  }
}

static void cf_features(const double* X, int n, int D, int rowbase, std::vector<int32_t>& ptr,
                        std::vector<int32_t>& fe) {
  ptr.assign((size_t)n + 1, 0);
  fe.clear();
  for (int i = 0; i < n; ++i) {
    for (int f = 0; f < D; ++f)
      if (X[i + (size_t)n * f] != 0.0) fe.push_back(rowbase + f);   // find(Data[i,:]) (:430-437)
    ptr[i + 1] = (int32_t)fe.size();
  }
  if (fe.empty()) fe.push_back(0);
}

// U, V initialisation of the SGD / SGLD CF samplers (the reference's variants differ):
//   kCfInitSide  GPT_fullw_sideinfo :424-428  stiefel ? polar(randn(r,rows)) : σ_u·randn(rows,r)
//   kCfInitSigma GPT_fixw / GPT_fixw_sideinfo :67 / :294  σ_u·randn(rows,r) (also when stiefel)
//   kCfInitUnit  GPT_fullw :175-180           stiefel ? polar(randn(r,rows)) : randn(rows,r)
enum CfInit { kCfInitSide = 0, kCfInitSigma = 1, kCfInitUnit = 2 };

// One fold's ratings and outputs of a CF run (column-major, caller-owned).
struct CfFold {
  const double* Rating; int64_t N, ldr;
  const double* Ratingtest; int64_t Ntest, ldt;
  double ymean, ystd;
  double *w_store, *U_store, *V_store, *testpred_store, *trainRMSE, *testRMSE;
  int32_t status;                  // out: GPT_OK or GPT_ERR_NAN_GEODESIC
};

// SGD / SGLD runs of the tensor CF model (the body of every GPT_*w* SGD variant) for F folds at
// once: the folds are sibling chains of one cf_epoch_kernel launch per epoch (the reference runs
// them as `@parallel for i=1:5`, 100k_movielensExperiment.jl:733-736), each with its own ratings,
// permutation, state, evaluation and early stop (:541-547); a fold that stops or bails out is
// skipped by later launches.  The folds share the side information, hyper-parameters and seed,
// hence the initial U, V (as separate calls with one param_seed do) and the per-epoch
// permutation; every fold has the same number of training ratings.  fixw keeps w at w_init
// (w_store may then be null); D1 = D2 = 0 with a = 1, b = c = 0 is the model without side
// information.
// Device time of the last CF SGD run on this thread (gpt_cf_last_timing): hipEvents around each
// epoch / eval launch, read after the per-epoch status copy that synchronises anyway.
struct CfTiming { double epoch_ms, eval_ms; int64_t epochs, evals, fold_steps; };
static thread_local CfTiming g_cf_timing{};
static thread_local int32_t g_cf_mode = 0;      // gpt_cf_last_mode
// GPTSGLD_CF_STAMPS=1: per-phase s_memtime of fold 0's first epoch (gpt_cf_last_stamps)
static thread_local std::vector<long long> g_cf_stamps;

static int cf_sgd_run(
    const char* name, std::vector<CfFold>& folds, const double* UserData, int64_t n1, int64_t D1,
    const double* MovieData, int64_t n2, int64_t D2, double signal_var, double sigma_u,
    double sigma_w, const double* w_init, int64_t r, int64_t m, double epsw, double epsU, double a,
    double b, double c, int64_t burnin, int64_t maxepoch, uint64_t seed, int32_t langevin,
    int32_t stiefel, int32_t avg, bool fixw, CfInit init) {
  const int F = (int)folds.size();
  bool ok = F >= 1 && (D1 == 0 || UserData) && (D2 == 0 || MovieData) && w_init && n1 >= 1 &&
            n2 >= 1 && D1 >= 0 && D2 >= 0 && m >= 1 && burnin >= 0 && maxepoch >= 0 &&
            signal_var > 0 && sigma_u > 0 && sigma_w > 0;
  for (const CfFold& f : folds)
    ok = ok && f.Rating && f.Ratingtest && (fixw || f.w_store) && f.U_store && f.V_store &&
         f.testpred_store && f.trainRMSE && f.testRMSE && f.N >= 1 && f.Ntest >= 1 &&
         f.ldr >= f.N && f.ldt >= f.Ntest && f.N == folds[0].N;
  if (!ok) { set_error(std::string("bad ") + name + " arguments"); return GPT_ERR_BAD_DIMS; }
  if (!cf_rank_supported((int)r) || cf_lds_bytes((int)r, (int)m, (int)(D1 + D2), D1 <= 64 && D2 <= 64) > 160 * 1024) {
    set_error(std::string(name) + ": rank not instantiated (1-6,8,10,12,15,16,20) or minibatch too large");
    return GPT_ERR_BAD_DIMS;
  }
  const int64_t N = folds[0].N;
  const int rowsU = (int)(n1 + D1), rowsV = (int)(n2 + D2);
  std::vector<int32_t> uptr, ufe, vptr, vfe;
  cf_features(UserData, (int)n1, (int)D1, (int)n1, uptr, ufe);
  cf_features(MovieData, (int)n2, (int)D2, (int)n2, vptr, vfe);
  // U, V init (:424-428 / :67 / :175-180, see CfInit)
  std::vector<double> U0((size_t)rowsU * r), V0((size_t)rowsV * r);
  for (int which = 0; which < 2; ++which) {
    const int rows = which ? rowsV : rowsU;
    double* M = which ? V0.data() : U0.data();
    std::vector<double> Z((size_t)rows * r);
    for (size_t e = 0; e < Z.size(); ++e) Z[e] = host_normal(seed, (uint32_t)e, 0, kCfUVInit, (uint32_t)which);
    if (stiefel && init != kCfInitSigma) host_stiefel_polar(Z.data(), (int)r, rows, M);
    else if (init == kCfInitUnit) for (size_t e = 0; e < Z.size(); ++e) M[e] = Z[e];
    else for (size_t e = 0; e < Z.size(); ++e) M[e] = sigma_u * Z[e];
  }
  const size_t nU = U0.size(), nV = V0.size(), rr = (size_t)r * r;
  const int nbatch = (int)((N + m - 1) / m);
  int64_t ntmax = 0;
  for (const CfFold& f : folds) ntmax = std::max(ntmax, f.Ntest);
  const int nmax = (int)std::max(N, ntmax);
  const int neval = (nmax + 255) / 256;
  DevMem d_up, d_uf, d_vp, d_vf, d_perm, d_ch;
  HIPCHK(d_up.alloc(4 * uptr.size())); HIPCHK(d_uf.alloc(4 * ufe.size()));
  HIPCHK(d_vp.alloc(4 * vptr.size())); HIPCHK(d_vf.alloc(4 * vfe.size()));
  HIPCHK(d_perm.alloc(4 * N)); HIPCHK(d_ch.alloc(sizeof(CfChain) * F));
  HIPCHK(hipMemcpy(d_up.p, uptr.data(), 4 * uptr.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_uf.p, ufe.data(), 4 * ufe.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_vp.p, vptr.data(), 4 * vptr.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_vf.p, vfe.data(), 4 * vfe.size(), hipMemcpyHostToDevice));
  // per fold: ratings, state, scratch, running predictions, SSE partials, status
  std::vector<std::unique_ptr<DevMem>> mem;
  std::vector<CfChain> ch(F);
  std::vector<int32_t*> d_st(F);
  std::vector<double*> d_w(F), d_U(F), d_V(F), d_sse(F), d_tep(F);
  for (int f = 0; f < F; ++f) {
    const CfFold& fd = folds[f];
    const int64_t Nt = fd.Ntest;
    std::vector<int32_t> tu(N), tm(N), eu(Nt), em(Nt);
    std::vector<double> tr(N), er(Nt);
    for (int64_t i = 0; i < N; ++i) {
      tu[i] = (int32_t)fd.Rating[i] - 1; tm[i] = (int32_t)fd.Rating[i + fd.ldr] - 1;
      tr[i] = fd.Rating[i + 2 * fd.ldr];
      if (tu[i] < 0 || tu[i] >= n1 || tm[i] < 0 || tm[i] >= n2) { set_error("rating ids out of range"); return GPT_ERR_BAD_DIMS; }
    }
    for (int64_t i = 0; i < Nt; ++i) {
      eu[i] = (int32_t)fd.Ratingtest[i] - 1; em[i] = (int32_t)fd.Ratingtest[i + fd.ldt] - 1;
      er[i] = fd.Ratingtest[i + 2 * fd.ldt];
      if (eu[i] < 0 || eu[i] >= n1 || em[i] < 0 || em[i] >= n2) { set_error("test rating ids out of range"); return GPT_ERR_BAD_DIMS; }
    }
    // one allocation per fold: ids (int32) first, then doubles (8-B aligned offsets)
    const size_t ints = (size_t)(4 * N + 2 * Nt + 2);
    const size_t dbl0 = (ints * 4 + 15) / 16 * 2;                     // in doubles
    const size_t ndbl = (size_t)N + Nt + rr + 2 * nU + 2 * nV + N + Nt + 2 * (size_t)neval + N;
    std::unique_ptr<DevMem> dm(new DevMem());
    HIPCHK(dm->alloc(8 * (dbl0 + ndbl)));
    int32_t* ip = dm->as<int32_t>();
    double* dp = dm->as<double>() + dbl0;
    CfChain& C = ch[f];
    C.tr_user = ip; C.tr_movie = ip + N; C.te_user = ip + 2 * N; C.te_movie = ip + 2 * N + Nt;
    d_st[f] = ip + 2 * N + 2 * Nt;
    C.tr_rating = dp; C.te_rating = dp + N;
    C.w = dp + N + Nt; C.U = C.w + rr; C.V = C.U + nU; C.GU = C.V + nV; C.GV = C.GU + nU;
    C.trainpred = C.GV + nV; C.testpred = C.trainpred + N; C.sse = C.testpred + Nt;
    C.ep_user = ip + 2 * N + 2 * Nt + 2; C.ep_movie = C.ep_user + N;
    C.ep_rating = C.sse + 2 * (size_t)neval;
    C.N = (int)N; C.Ntest = (int)Nt; C.perm = d_perm.as<int32_t>();
    C.status = d_st[f]; C.ymean = fd.ymean; C.ystd = fd.ystd;
    d_w[f] = C.w; d_U[f] = C.U; d_V[f] = C.V; d_sse[f] = C.sse; d_tep[f] = C.testpred;
    HIPCHK(hipMemcpy((void*)C.tr_user, tu.data(), 4 * N, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy((void*)C.tr_movie, tm.data(), 4 * N, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy((void*)C.te_user, eu.data(), 4 * Nt, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy((void*)C.te_movie, em.data(), 4 * Nt, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy((void*)C.tr_rating, tr.data(), 8 * N, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy((void*)C.te_rating, er.data(), 8 * Nt, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(C.w, w_init, 8 * rr, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(C.U, U0.data(), 8 * nU, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(C.V, V0.data(), 8 * nV, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(C.GU, 0, 8 * (nU + nV)));                             // GU, GV
    HIPCHK(hipMemset(C.trainpred, 0, 8 * (size_t)(N + Nt)));
    HIPCHK(hipMemset(d_st[f], 0, 4));
    mem.push_back(std::move(dm));
  }
  HIPCHK(hipMemcpy(d_ch.p, ch.data(), sizeof(CfChain) * F, hipMemcpyHostToDevice));
  CfParams P{};
  P.n1 = (int)n1; P.D1 = (int)D1; P.n2 = (int)n2; P.D2 = (int)D2; P.r = (int)r; P.m = (int)m;
  P.rowsU = rowsU; P.rowsV = rowsV;
  P.a = a; P.b = b; P.c = c; P.signal_var = signal_var; P.sigma_u = sigma_u; P.sigma_w = sigma_w;
  P.epsw = epsw; P.epsU = epsU; P.langevin = langevin; P.stiefel = stiefel; P.seed = seed;
  P.fixw = fixw ? 1 : 0;
  P.uptr = d_up.as<int32_t>(); P.ufe = d_uf.as<int32_t>(); P.vptr = d_vp.as<int32_t>(); P.vfe = d_vf.as<int32_t>();
  DevMem d_masks;
  if (D1 <= 64 && D2 <= 64) {    // each user's / movie's feature rows as one 64-bit mask
    std::vector<uint64_t> mk((size_t)(n1 + n2), 0);
    for (int64_t i = 0; i < n1; ++i)
      for (int z = uptr[i]; z < uptr[i + 1]; ++z) mk[i] |= 1ull << (ufe[z] - n1);
    for (int64_t i = 0; i < n2; ++i)
      for (int z = vptr[i]; z < vptr[i + 1]; ++z) mk[n1 + i] |= 1ull << (vfe[z] - n2);
    HIPCHK(d_masks.alloc(8 * mk.size()));
    HIPCHK(hipMemcpy(d_masks.p, mk.data(), 8 * mk.size(), hipMemcpyHostToDevice));
    P.umask = d_masks.as<uint64_t>();
    P.vmask = P.umask + n1;
  }
  DevMem d_stamps;
  const bool want_stamps = std::getenv("GPTSGLD_CF_STAMPS") != nullptr;
  g_cf_stamps.clear();
  if (want_stamps) {
    HIPCHK(d_stamps.alloc(8 * (size_t)kCfStampSteps * kCfStampSlots));
    HIPCHK(hipMemset(d_stamps.p, 0, 8 * (size_t)kCfStampSteps * kCfStampSlots));
    P.stamps = d_stamps.as<long long>();
  }
#if CF_WSTAMPS
  if (std::getenv("GPTSGLD_CF_EXP")) P.exp = std::atoi(std::getenv("GPTSGLD_CF_EXP"));
#endif
  for (CfFold& fd : folds) {
    if (fd.w_store) std::memset(fd.w_store, 0, 8 * rr * maxepoch);
    std::memset(fd.U_store, 0, 8 * nU * maxepoch);
    std::memset(fd.V_store, 0, 8 * nV * maxepoch);
    std::memset(fd.testpred_store, 0, 8 * (size_t)fd.Ntest * maxepoch);
    std::memset(fd.trainRMSE, 0, 8 * (size_t)maxepoch);
    for (int64_t z = 0; z < maxepoch; ++z) fd.testRMSE[z] = 10.0;            // :441
    fd.status = GPT_OK;
  }
  std::vector<int32_t> perm(N);
  std::vector<double> sse(2 * (size_t)neval), tp(ntmax);
  std::vector<char> live(F, 1);
  std::vector<int> testcounter(F, 0);
  int counter = 0, nlive = F;
  long long step_base_host = 0;                      // graph replays' epoch base: read by the copy
                                                     // below, alive until the epoch's event sync
  const int32_t stopped = 2;                         // skips the fold in later launches
  struct Events {
    hipEvent_t e[4] = {nullptr, nullptr, nullptr, nullptr};
    ~Events() { for (auto x : e) if (x) (void)hipEventDestroy(x); }
  } evs;
  for (auto& x : evs.e) HIPCHK(hipEventCreate(&x));
  // the run's own stream; the SGD / SGLD path replays one captured graph per epoch (gather + the
  // epoch's batch-phase / move launch pairs), its steps counted from a device-side epoch base
  struct RunStream {
    hipStream_t s = nullptr;
    hipGraph_t g = nullptr;
    hipGraphExec_t x = nullptr;
    ~RunStream() {
      if (s) (void)hipStreamSynchronize(s);
      if (x) (void)hipGraphExecDestroy(x);
      if (g) (void)hipGraphDestroy(g);
      if (s) (void)hipStreamDestroy(s);
    }
  } rs;
  HIPCHK(hipStreamCreateWithFlags(&rs.s, hipStreamNonBlocking));
  hipStream_t st = rs.s;
  HIPCHK(hipStreamSynchronize(nullptr));             // the set-up copies / memsets are done
  DevMem d_step;
  HIPCHK(d_step.alloc(sizeof(long long)));
  g_cf_timing = CfTiming{};
  // SGD (no Langevin noise, no Stiefel geometry) on the feature-mask path: the lazy move, one
  // launch per epoch (cf_epoch_kernel domove = 2); GPTSGLD_CF_LAZY=0 keeps the batch-phase / move
  // launch pairs
  // (the decay factor c = 1 − εU/(2σ_u²) of a skipped row must lie in (0, 1): the kernel reads a
  // row Δ steps behind as m·c^Δ; outside that range the eager move keeps the reference's numbers)
  const double cdecay = 1.0 - P.epsU / (2.0 * P.sigma_u * P.sigma_u);
  const bool lazy = !stiefel && !langevin && P.umask != nullptr && cdecay > 0.0 && cdecay < 1.0 &&
                    cf_lazy_lds_bytes((int)r, (int)m, (int)(D1 + D2), rowsU + rowsV, nbatch) <=
                        160 * 1024 &&
                    !(std::getenv("GPTSGLD_CF_LAZY") && std::strcmp(std::getenv("GPTSGLD_CF_LAZY"), "0") == 0);
  g_cf_mode = stiefel ? 1 : (lazy ? 2 : 0);
  for (int64_t epoch = 1; epoch <= burnin + maxepoch && nlive > 0; ++epoch) {
    host_randperm((int)N, seed, (int)(epoch - 1), perm.data());
    HIPCHK(hipMemcpy(d_perm.p, perm.data(), 4 * N, hipMemcpyHostToDevice));
    hipError_t e = hipSuccess;
    if (stiefel || lazy) {
      // the Stiefel move needs Grams over every row, the lazy SGD move needs none of the rows
      // outside the batch: the whole epoch in one workgroup per fold, one launch
      HIPCHK(hipEventRecord(evs.e[0], st));
      e = launch_cf_gather(d_ch.as<CfChain>(), F, (int)N, st);
      if (e == hipSuccess)
        e = launch_cf_epoch(P, d_ch.as<CfChain>(), F, (epoch - 1) * nbatch, 0, nbatch,
                            stiefel ? 1 : 2, st);
    } else if (P.stamps) {
      // the stamped first epoch: direct launches (the stamp buffer is dropped after it)
      HIPCHK(hipEventRecord(evs.e[0], st));
      e = launch_cf_gather(d_ch.as<CfChain>(), F, (int)N, st);
      for (int b = 0; b < nbatch && e == hipSuccess; ++b) {
        const long long step = (epoch - 1) * nbatch + b;
        e = launch_cf_epoch(P, d_ch.as<CfChain>(), F, step, b, 1, 0, st);
        if (e == hipSuccess) e = launch_cf_move(P, d_ch.as<CfChain>(), F, step, st);
      }
    } else {
      // per minibatch: the batch phase (one workgroup per fold), then the row-parallel move of U
      // and V over the whole GPU (cf_move_kernel) — an epoch of them as one graph
      if (!rs.x) {
        HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        e = launch_cf_gather(d_ch.as<CfChain>(), F, (int)N, st);
        for (int b = 0; b < nbatch && e == hipSuccess; ++b) {
          e = launch_cf_epoch(P, d_ch.as<CfChain>(), F, b, b, 1, 0, st, d_step.as<long long>());
          if (e == hipSuccess)
            e = launch_cf_move(P, d_ch.as<CfChain>(), F, b, st, d_step.as<long long>());
        }
        const hipError_t ec = hipStreamEndCapture(st, &rs.g);
        if (e != hipSuccess) return hip_fail(e, "cf epoch capture");
        if (ec != hipSuccess) return hip_fail(ec, "hipStreamEndCapture");
        HIPCHK(hipGraphInstantiate(&rs.x, rs.g, nullptr, nullptr, 0));
      }
      step_base_host = (epoch - 1) * nbatch;
      HIPCHK(hipMemcpyAsync(d_step.p, &step_base_host, sizeof(long long), hipMemcpyHostToDevice, st));
      HIPCHK(hipEventRecord(evs.e[0], st));
      e = hipGraphLaunch(rs.x, st);
    }
    if (e != hipSuccess) return hip_fail(e, "cf epoch kernel");
    HIPCHK(hipEventRecord(evs.e[1], st));
    HIPCHK(hipEventSynchronize(evs.e[1]));
    if (P.stamps) {                // the first epoch only
      g_cf_stamps.resize((size_t)kCfStampSteps * kCfStampSlots);
      HIPCHK(hipMemcpy(g_cf_stamps.data(), P.stamps, 8 * g_cf_stamps.size(), hipMemcpyDeviceToHost));
      P.stamps = nullptr;
    }
    {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, evs.e[0], evs.e[1]));
      g_cf_timing.epoch_ms += ms;
      g_cf_timing.epochs += 1;
      g_cf_timing.fold_steps += (int64_t)nlive * nbatch;
    }
    for (int f = 0; f < F; ++f) {
      if (!live[f]) continue;
      int32_t bad = 0;
      HIPCHK(hipMemcpy(&bad, d_st[f], 4, hipMemcpyDeviceToHost));
      if (bad) {                     // :490-492 — zero parameter stores, curves as they are
        CfFold& fd = folds[f];
        if (fd.w_store) std::memset(fd.w_store, 0, 8 * rr * maxepoch);
        std::memset(fd.U_store, 0, 8 * nU * maxepoch);
        std::memset(fd.V_store, 0, 8 * nV * maxepoch);
        fd.status = GPT_ERR_NAN_GEODESIC;
        live[f] = 0; --nlive;
      }
    }
    if (epoch > burnin && nlive > 0) {
      const int64_t s2 = epoch - burnin - 1;
      if (!avg) counter = 0;
      HIPCHK(hipEventRecord(evs.e[2], st));
      e = launch_cf_eval(P, d_ch.as<CfChain>(), F, nmax, counter, st);
      if (e != hipSuccess) return hip_fail(e, "cf eval kernel");
      HIPCHK(hipEventRecord(evs.e[3], st));
      HIPCHK(hipEventSynchronize(evs.e[3]));
      {
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, evs.e[2], evs.e[3]));
        g_cf_timing.eval_ms += ms;
        g_cf_timing.evals += 1;
      }
      for (int f = 0; f < F; ++f) {
        if (!live[f]) continue;
        CfFold& fd = folds[f];
        if (fd.w_store) HIPCHK(hipMemcpy(fd.w_store + rr * s2, d_w[f], 8 * rr, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(fd.U_store + nU * s2, d_U[f], 8 * nU, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(fd.V_store + nV * s2, d_V[f], 8 * nV, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(sse.data(), d_sse[f], 16 * (size_t)neval, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(tp.data(), d_tep[f], 8 * fd.Ntest, hipMemcpyDeviceToHost));
        double st0 = 0.0, st1 = 0.0;
        for (int z = 0; z < neval; ++z) { st0 += sse[2 * z]; st1 += sse[2 * z + 1]; }
        fd.trainRMSE[s2] = std::sqrt(st0 / (double)N);
        fd.testRMSE[s2] = std::sqrt(st1 / (double)fd.Ntest);
        for (int64_t i = 0; i < fd.Ntest; ++i)
          fd.testpred_store[(size_t)fd.Ntest * s2 + i] =
              std::min(std::max(tp[i] * fd.ystd + fd.ymean, 1.0), 5.0);
        // :541-547 (the reference compares with the previous epoch's entry; none at s2 = 0)
        if (epoch > 1 && s2 > 0 && fd.testRMSE[s2] > fd.testRMSE[s2 - 1]) testcounter[f] += 1;
        else testcounter[f] = 0;
        if (testcounter[f] >= 5) {
          HIPCHK(hipMemcpy(d_st[f], &stopped, 4, hipMemcpyHostToDevice));
          live[f] = 0; --nlive;
        }
      }
      counter += 1;
    }
  }
  for (const CfFold& fd : folds)
    if (fd.status != GPT_OK) {
      set_error("Get NaN when moving along Geodesic. Try smaller epsU");
      return GPT_ERR_NAN_GEODESIC;
    }
  return GPT_OK;
}

// one fold (the reference functions' own signature)
static int cf_sgd_one(const char* name, const double* Rating, int64_t N, int64_t ldr,
                      const double* UserData, int64_t n1, int64_t D1, const double* MovieData,
                      int64_t n2, int64_t D2, const double* Ratingtest, int64_t Ntest, int64_t ldt,
                      double signal_var, double sigma_u, double sigma_w, const double* w_init,
                      int64_t r, int64_t m, double epsw, double epsU, double a, double b, double c,
                      int64_t burnin, int64_t maxepoch, uint64_t seed, double ytrainMean,
                      double ytrainStd, int32_t langevin, int32_t stiefel, int32_t avg, bool fixw,
                      CfInit init, double* w_store, double* U_store, double* V_store,
                      double* testpred_store, double* trainRMSE, double* testRMSE) {
  std::vector<CfFold> folds(1);
  folds[0] = CfFold{Rating, N, ldr, Ratingtest, Ntest, ldt, ytrainMean, ytrainStd, w_store, U_store,
                    V_store, testpred_store, trainRMSE, testRMSE, GPT_OK};
  return cf_sgd_run(name, folds, UserData, n1, D1, MovieData, n2, D2, signal_var, sigma_u, sigma_w,
                    w_init, r, m, epsw, epsU, a, b, c, burnin, maxepoch, seed, langevin, stiefel,
                    avg, fixw, init);
}

extern "C" int gpt_cf_fullw_sideinfo(
    const double* Rating, int64_t N, int64_t ldr, const double* UserData, int64_t n1, int64_t D1,
    const double* MovieData, int64_t n2, int64_t D2, const double* Ratingtest, int64_t Ntest,
    int64_t ldt, double signal_var, double sigma_u, double sigma_w, const double* w_init, int64_t r,
    int64_t m, double epsw, double epsU, double a, double b, double c, int64_t burnin,
    int64_t maxepoch, uint64_t seed, double ytrainMean, double ytrainStd, int32_t langevin,
    int32_t stiefel, int32_t avg, double* w_store, double* U_store, double* V_store,
    double* testpred_store, double* trainRMSE, double* testRMSE) {
  return cf_sgd_one("GPT_fullw_sideinfo", Rating, N, ldr, UserData, n1, D1, MovieData, n2, D2,
                    Ratingtest, Ntest, ldt, signal_var, sigma_u, sigma_w, w_init, r, m, epsw, epsU,
                    a, b, c, burnin, maxepoch, seed, ytrainMean, ytrainStd, langevin, stiefel, avg,
                    false, kCfInitSide, w_store, U_store, V_store, testpred_store, trainRMSE,
                    testRMSE);
}

extern "C" int gpt_cf_fullw_sideinfo_folds(
    int64_t F, const double* const* Rating, const int64_t* N, const double* const* Ratingtest,
    const int64_t* Ntest, const double* UserData, int64_t n1, int64_t D1, const double* MovieData,
    int64_t n2, int64_t D2, double signal_var, double sigma_u, double sigma_w,
    const double* w_init, int64_t r, int64_t m, double epsw, double epsU, double a, double b,
    double c, int64_t burnin, int64_t maxepoch, uint64_t seed, const double* ytrainMean,
    const double* ytrainStd, int32_t langevin, int32_t stiefel, int32_t avg,
    double* const* w_store, double* const* U_store, double* const* V_store,
    double* const* testpred_store, double* const* trainRMSE, double* const* testRMSE,
    int32_t* status) {
  if (F < 1 || F > 65535 || !Rating || !N || !Ratingtest || !Ntest || !ytrainMean || !ytrainStd ||
      !w_store || !U_store || !V_store || !testpred_store || !trainRMSE || !testRMSE) {
    set_error("bad GPT_fullw_sideinfo_folds arguments"); return GPT_ERR_BAD_DIMS;
  }
  std::vector<CfFold> folds(F);
  for (int64_t f = 0; f < F; ++f)
    folds[f] = CfFold{Rating[f], N[f], N[f], Ratingtest[f], Ntest[f], Ntest[f], ytrainMean[f],
                      ytrainStd[f], w_store[f], U_store[f], V_store[f], testpred_store[f],
                      trainRMSE[f], testRMSE[f], GPT_OK};
  const int rc = cf_sgd_run("GPT_fullw_sideinfo_folds", folds, UserData, n1, D1, MovieData, n2, D2,
                            signal_var, sigma_u, sigma_w, w_init, r, m, epsw, epsU, a, b, c,
                            burnin, maxepoch, seed, langevin, stiefel, avg, false, kCfInitSide);
  if (status)
    for (int64_t f = 0; f < F; ++f) status[f] = folds[f].status;
  return rc;
}

extern "C" int gpt_cf_last_timing(double* epoch_ms, double* eval_ms, int64_t* epochs,
                                   int64_t* fold_steps) {
  if (!epoch_ms || !eval_ms || !epochs || !fold_steps) {
    set_error("gpt_cf_last_timing: null output"); return GPT_ERR_BAD_DIMS;
  }
  *epoch_ms = g_cf_timing.epoch_ms;
  *eval_ms = g_cf_timing.eval_ms;
  *epochs = g_cf_timing.epochs;
  *fold_steps = g_cf_timing.fold_steps;
  return GPT_OK;
}

extern "C" int gpt_pred_last_vphase(int32_t* kind) {
  if (!kind) { set_error("gpt_pred_last_vphase: null output"); return GPT_ERR_BAD_DIMS; }
  *kind = pred_last_vphase();
  return GPT_OK;
}

extern "C" int gpt_cf_last_mode(int32_t* mode) {
  if (!mode) { set_error("gpt_cf_last_mode: null output"); return GPT_ERR_BAD_DIMS; }
  *mode = g_cf_mode;
  return GPT_OK;
}

extern "C" int64_t gpt_cf_last_stamps(int64_t* out, int64_t cap) {
  const int64_t n = (int64_t)g_cf_stamps.size();
  if (out)
    for (int64_t i = 0; i < std::min(n, cap); ++i) out[i] = g_cf_stamps[(size_t)i];
  return n;
}

extern "C" int gpt_cf_fixw_sideinfo(
    const double* Rating, int64_t N, int64_t ldr, const double* UserData, int64_t n1, int64_t D1,
    const double* MovieData, int64_t n2, int64_t D2, const double* Ratingtest, int64_t Ntest,
    int64_t ldt, double signal_var, double sigma_u, const double* w, int64_t r, int64_t m,
    double epsU, double a, double b, double c, int64_t burnin, int64_t maxepoch, uint64_t seed,
    double ytrainMean, double ytrainStd, int32_t langevin, int32_t stiefel, int32_t avg,
    double* U_store, double* V_store, double* testpred_store, double* trainRMSE,
    double* testRMSE) {
  return cf_sgd_one("GPT_fixw_sideinfo", Rating, N, ldr, UserData, n1, D1, MovieData, n2, D2,
                    Ratingtest, Ntest, ldt, signal_var, sigma_u, 1.0, w, r, m, 0.0, epsU, a, b, c,
                    burnin, maxepoch, seed, ytrainMean, ytrainStd, langevin, stiefel, avg, true,
                    kCfInitSigma, nullptr, U_store, V_store, testpred_store, trainRMSE, testRMSE);
}

extern "C" int gpt_cf_fullw(const double* Rating, int64_t N, int64_t ldr, int64_t n1, int64_t n2,
                            const double* Ratingtest, int64_t Ntest, int64_t ldt,
                            double signal_var, double sigma_u, double sigma_w,
                            const double* w_init, int64_t r, int64_t m, double epsw, double epsU,
                            int64_t burnin, int64_t maxepoch, uint64_t seed, double ytrainMean,
                            double ytrainStd, int32_t langevin, int32_t stiefel, int32_t avg,
                            double* w_store, double* U_store, double* V_store,
                            double* testpred_store, double* trainRMSE, double* testRMSE) {
  return cf_sgd_one("GPT_fullw", Rating, N, ldr, nullptr, n1, 0, nullptr, n2, 0, Ratingtest,
                    Ntest, ldt, signal_var, sigma_u, sigma_w, w_init, r, m, epsw, epsU, 1.0, 0.0,
                    0.0, burnin, maxepoch, seed, ytrainMean, ytrainStd, langevin, stiefel, avg,
                    false, kCfInitUnit, w_store, U_store, V_store, testpred_store, trainRMSE,
                    testRMSE);
}

extern "C" int gpt_cf_fixw(const double* Rating, int64_t N, int64_t ldr, int64_t n1, int64_t n2,
                           const double* Ratingtest, int64_t Ntest, int64_t ldt, double signal_var,
                           double sigma_u, const double* w, int64_t r, int64_t m, double epsU,
                           int64_t burnin, int64_t maxepoch, uint64_t seed, double ytrainMean,
                           double ytrainStd, int32_t langevin, int32_t stiefel, int32_t avg,
                           double* U_store, double* V_store, double* testpred_store,
                           double* trainRMSE, double* testRMSE) {
  return cf_sgd_one("GPT_fixw", Rating, N, ldr, nullptr, n1, 0, nullptr, n2, 0, Ratingtest, Ntest,
                    ldt, signal_var, sigma_u, 1.0, w, r, m, 0.0, epsU, 1.0, 0.0, 0.0, burnin,
                    maxepoch, seed, ytrainMean, ytrainStd, langevin, stiefel, avg, true,
                    kCfInitSigma, nullptr, U_store, V_store, testpred_store, trainRMSE, testRMSE);
}

// Q of a Householder QR (LAPACK dgeqr2 + dorg2r conventions), r × r column-major in place.
static void host_qr_q(int r, std::vector<double>& A) {
  std::vector<double> tau(r, 0.0);
  for (int k = 0; k < r; ++k) {
    double xn = 0.0;
    for (int i = k + 1; i < r; ++i) xn = std::hypot(xn, A[i + (size_t)r * k]);
    const double alpha = A[k + (size_t)r * k];
    if (xn == 0.0) { tau[k] = 0.0; continue; }
    const double beta = -std::copysign(std::hypot(alpha, xn), alpha);
    tau[k] = (beta - alpha) / beta;
    const double sc = 1.0 / (alpha - beta);
    for (int i = k + 1; i < r; ++i) A[i + (size_t)r * k] *= sc;
    A[k + (size_t)r * k] = beta;
    for (int j = k + 1; j < r; ++j) {            // apply H_k to the trailing columns
      double s = A[k + (size_t)r * j];
      for (int i = k + 1; i < r; ++i) s += A[i + (size_t)r * k] * A[i + (size_t)r * j];
      s *= tau[k];
      A[k + (size_t)r * j] -= s;
      for (int i = k + 1; i < r; ++i) A[i + (size_t)r * j] -= s * A[i + (size_t)r * k];
    }
  }
  std::vector<double> Qm((size_t)r * r, 0.0);
  for (int i = 0; i < r; ++i) Qm[i + (size_t)r * i] = 1.0;
  for (int k = r - 1; k >= 0; --k) {             // Q = H_0 … H_{r-1} applied to I (dorg2r)
    for (int j = k; j < r; ++j) {
      double s = Qm[k + (size_t)r * j];
      for (int i = k + 1; i < r; ++i) s += A[i + (size_t)r * k] * Qm[i + (size_t)r * j];
      s *= tau[k];
      Qm[k + (size_t)r * j] -= s;
      for (int i = k + 1; i < r; ++i) Qm[i + (size_t)r * j] -= s * A[i + (size_t)r * k];
    }
  }
  A.swap(Qm);
}

// Gibbs sweeps of the CF model without side information (GPT_fullw_gibbs; fixw: GPT_fixw_gibbs,
// :945-1028 — the same user / movie conditionals, no w draw, w_store may be null).
static int cf_gibbs_run(
    const char* name, const double* Rating, int64_t N, int64_t ldr, int64_t n1, int64_t n2,
    const double* Ratingtest, int64_t Ntest, int64_t ldt, double signal_var, double sigma_u,
    double sigma_w, const double* w_init, int64_t r, int64_t burnin, int64_t maxepoch,
    int64_t n_samples, uint64_t seed, double ytrainMean, double ytrainStd, int32_t avg,
    int32_t rotated_w, bool fixw, double* w_store, double* U_store, double* V_store,
    double* testpred_store, double* trainRMSE, double* testRMSE) {
  if (!Rating || !Ratingtest || !w_init || (!fixw && !w_store) || !U_store || !V_store || !testpred_store ||
      !trainRMSE || !testRMSE || N < 1 || Ntest < 1 || ldr < N || ldt < Ntest || n1 < 1 || n2 < 1 ||
      burnin < 0 || maxepoch < 0 || n_samples < 1 || !(signal_var > 0) || !(sigma_u > 0) ||
      !(sigma_w > 0)) {
    set_error(std::string("bad ") + name + " arguments"); return GPT_ERR_BAD_DIMS;
  }
  if (!cf_rank_supported((int)r) || r * r > 1024) {
    set_error(std::string(name) + ": rank not instantiated (1-6,8,10,12,15,16,20)"); return GPT_ERR_BAD_DIMS;
  }
  std::vector<int32_t> tu(N), tm(N), eu(Ntest), em(Ntest);
  std::vector<double> tr(N), er(Ntest);
  for (int64_t i = 0; i < N; ++i) {
    tu[i] = (int32_t)Rating[i] - 1; tm[i] = (int32_t)Rating[i + ldr] - 1; tr[i] = Rating[i + 2 * ldr];
    if (tu[i] < 0 || tu[i] >= n1 || tm[i] < 0 || tm[i] >= n2) { set_error("rating ids out of range"); return GPT_ERR_BAD_DIMS; }
  }
  for (int64_t i = 0; i < Ntest; ++i) {
    eu[i] = (int32_t)Ratingtest[i] - 1; em[i] = (int32_t)Ratingtest[i + ldt] - 1; er[i] = Ratingtest[i + 2 * ldt];
    if (eu[i] < 0 || eu[i] >= n1 || em[i] < 0 || em[i] >= n2) { set_error("test rating ids out of range"); return GPT_ERR_BAD_DIMS; }
  }
  // ratings of each user / movie in Rating order (idx = (Rating[:,1].==i), :1061)
  std::vector<int32_t> uptr(n1 + 1, 0), mptr(n2 + 1, 0), ulst(N), mlst(N);
  for (int64_t i = 0; i < N; ++i) { uptr[tu[i] + 1]++; mptr[tm[i] + 1]++; }
  for (int64_t i = 0; i < n1; ++i) uptr[i + 1] += uptr[i];
  for (int64_t i = 0; i < n2; ++i) mptr[i + 1] += mptr[i];
  {
    std::vector<int32_t> cu(uptr.begin(), uptr.end() - 1), cm(mptr.begin(), mptr.end() - 1);
    for (int64_t i = 0; i < N; ++i) { ulst[cu[tu[i]]++] = (int32_t)i; mlst[cm[tm[i]]++] = (int32_t)i; }
  }
  // init (:1047-1053): Q = qr(randn(r,r)), U = σ_u·randn(n1,r), V = σ_u·randn(n2,r)
  const size_t rr = (size_t)r * r, nU = (size_t)n1 * r, nV = (size_t)n2 * r;
  std::vector<double> Qm(rr), U0(nU), V0(nV), w0(w_init, w_init + rr);
  for (size_t e = 0; e < rr; ++e) Qm[e] = host_normal(seed, (uint32_t)e, 0, kCfgInit, 0);
  for (size_t e = 0; e < nU; ++e) U0[e] = sigma_u * host_normal(seed, (uint32_t)e, 0, kCfgInit, 1);
  for (size_t e = 0; e < nV; ++e) V0[e] = sigma_u * host_normal(seed, (uint32_t)e, 0, kCfgInit, 2);
  host_qr_q((int)r, Qm);
  if (rotated_w) {                                // w = Q·w_init; U = U·Q'
    for (int64_t i = 0; i < r; ++i)
      for (int64_t j = 0; j < r; ++j) {
        double s = 0.0;
        for (int64_t k = 0; k < r; ++k) s += Qm[i + r * k] * w_init[k + r * j];
        w0[i + r * j] = s;
      }
    std::vector<double> U1(nU);
    for (int64_t i = 0; i < n1; ++i)
      for (int64_t j = 0; j < r; ++j) {
        double s = 0.0;
        for (int64_t k = 0; k < r; ++k) s += U0[i + n1 * k] * Qm[j + r * k];
        U1[i + n1 * j] = s;
      }
    U0.swap(U1);
  }
  const int p = (int)rr;
  const int neval = (int)((std::max(N, Ntest) + 255) / 256);
  DevMem d_tu, d_tm, d_tr, d_eu, d_em, d_er, d_up, d_mp, d_ul, d_ml, d_w, d_U, d_V, d_M, d_x,
      d_z, d_trp, d_tep, d_sse, d_st, d_ch, d_zu, d_zv, d_ws, d_keep;
  HIPCHK(d_tu.alloc(4 * N)); HIPCHK(d_tm.alloc(4 * N)); HIPCHK(d_tr.alloc(8 * N));
  HIPCHK(d_eu.alloc(4 * Ntest)); HIPCHK(d_em.alloc(4 * Ntest)); HIPCHK(d_er.alloc(8 * Ntest));
  HIPCHK(d_up.alloc(4 * uptr.size())); HIPCHK(d_mp.alloc(4 * mptr.size()));
  HIPCHK(d_ul.alloc(4 * N)); HIPCHK(d_ml.alloc(4 * N));
  HIPCHK(d_w.alloc(8 * rr)); HIPCHK(d_U.alloc(8 * nU)); HIPCHK(d_V.alloc(8 * nV));
  HIPCHK(d_M.alloc(8 * rr * rr)); HIPCHK(d_x.alloc(8 * rr));
  HIPCHK(d_z.alloc(8 * rr)); HIPCHK(d_trp.alloc(8 * N)); HIPCHK(d_tep.alloc(8 * Ntest));
  HIPCHK(d_sse.alloc(16 * (size_t)neval)); HIPCHK(d_st.alloc(4)); HIPCHK(d_ch.alloc(sizeof(CfChain)));
  HIPCHK(d_zu.alloc(4 * (n1 + 1))); HIPCHK(d_zv.alloc(4 * (n2 + 1)));
  HIPCHK(d_ws.alloc(8 * cfg_wsystem_scratch_dbl((int)r, (int)n1)));
  HIPCHK(hipMemcpy(d_tu.p, tu.data(), 4 * N, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_tm.p, tm.data(), 4 * N, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_tr.p, tr.data(), 8 * N, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_eu.p, eu.data(), 4 * Ntest, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_em.p, em.data(), 4 * Ntest, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_er.p, er.data(), 8 * Ntest, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_up.p, uptr.data(), 4 * uptr.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_mp.p, mptr.data(), 4 * mptr.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_ul.p, ulst.data(), 4 * N, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_ml.p, mlst.data(), 4 * N, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_w.p, w0.data(), 8 * rr, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_U.p, U0.data(), 8 * nU, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_V.p, V0.data(), 8 * nV, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(d_trp.p, 0, 8 * N)); HIPCHK(hipMemset(d_tep.p, 0, 8 * Ntest));
  HIPCHK(hipMemset(d_st.p, 0, 4));
  HIPCHK(hipMemset(d_zu.p, 0, 4 * (n1 + 1))); HIPCHK(hipMemset(d_zv.p, 0, 4 * (n2 + 1)));
  // prediction without side information: a = 1, b = c = 0, empty feature lists (:1101-1102)
  CfParams P{};
  P.n1 = (int)n1; P.D1 = 0; P.n2 = (int)n2; P.D2 = 0; P.r = (int)r; P.m = 1;
  P.rowsU = (int)n1; P.rowsV = (int)n2; P.a = 1.0; P.b = 0.0; P.c = 0.0;
  P.signal_var = signal_var; P.sigma_u = sigma_u; P.sigma_w = sigma_w; P.seed = seed;
  P.uptr = d_zu.as<int32_t>(); P.ufe = d_zu.as<int32_t>(); P.vptr = d_zv.as<int32_t>(); P.vfe = d_zv.as<int32_t>();
  CfChain Cc{};
  Cc.tr_user = d_tu.as<int32_t>(); Cc.tr_movie = d_tm.as<int32_t>(); Cc.tr_rating = d_tr.as<double>();
  Cc.te_user = d_eu.as<int32_t>(); Cc.te_movie = d_em.as<int32_t>(); Cc.te_rating = d_er.as<double>();
  Cc.N = (int)N; Cc.Ntest = (int)Ntest; Cc.w = d_w.as<double>(); Cc.U = d_U.as<double>();
  Cc.V = d_V.as<double>(); Cc.trainpred = d_trp.as<double>(); Cc.testpred = d_tep.as<double>();
  Cc.sse = d_sse.as<double>(); Cc.status = d_st.as<int32_t>();
  Cc.ymean = ytrainMean; Cc.ystd = ytrainStd;
  HIPCHK(hipMemcpy(d_ch.p, &Cc, sizeof(CfChain), hipMemcpyHostToDevice));
  if (w_store) std::memset(w_store, 0, 8 * rr * maxepoch);
  std::memset(U_store, 0, 8 * nU * maxepoch);
  std::memset(V_store, 0, 8 * nV * maxepoch);
  std::memset(testpred_store, 0, 8 * (size_t)Ntest * maxepoch);
  std::memset(trainRMSE, 0, 8 * (size_t)maxepoch);
  std::memset(testRMSE, 0, 8 * (size_t)maxepoch);
  // Kept sweeps are recorded on the device (w | U | V | test prediction | the two RMSEs per sweep,
  // up to ~1 GiB of sweeps at a time) and copied to the caller's arrays in chunks: no host
  // synchronisation inside a chunk (the round-4 loop copied and synchronised every sweep).
  const size_t kb = rr + nU + nV + (size_t)Ntest + 2;              // doubles per kept sweep
  const int64_t chunkE = std::max<int64_t>(1, std::min<int64_t>(std::max<int64_t>(maxepoch, 1),
                                                                 (int64_t)((1ull << 27) / kb)));
  HIPCHK(d_keep.alloc(8 * kb * chunkE));
  double* kw = d_keep.as<double>();
  double* kU = kw + rr * chunkE;
  double* kV = kU + nU * chunkE;
  double* ktp = kV + nV * chunkE;
  double* krm = ktp + (size_t)Ntest * chunkE;
  std::vector<double> rm(2 * (size_t)chunkE);
  int64_t flushed = 0;                              // kept sweeps already in the caller's arrays
  // Julia throws PosDefException (no outputs): every output array is zeroed before the error
  auto not_spd = [&]() -> int {
    if (w_store) std::memset(w_store, 0, 8 * rr * maxepoch);
    std::memset(U_store, 0, 8 * nU * maxepoch);
    std::memset(V_store, 0, 8 * nV * maxepoch);
    std::memset(testpred_store, 0, 8 * (size_t)Ntest * maxepoch);
    std::memset(trainRMSE, 0, 8 * (size_t)maxepoch);
    std::memset(testRMSE, 0, 8 * (size_t)maxepoch);
    set_error("PosDefException: a Gibbs precision matrix is not positive definite");
    return GPT_ERR_NOT_SPD;
  };
  // The status word after every epoch's sweeps is copied into pinned memory behind them and read
  // one epoch later, so a failed Cholesky stops the sampler within two epochs without a full
  // synchronisation per epoch.
  struct StatusRing {
    int32_t* h = nullptr;
    hipEvent_t e[2] = {nullptr, nullptr};
    ~StatusRing() {
      for (auto x : e) if (x) (void)hipEventDestroy(x);
      if (h) (void)hipHostFree(h);
    }
  } sr;
  HIPCHK(hipHostMalloc((void**)&sr.h, 2 * sizeof(int32_t), hipHostMallocDefault));
  sr.h[0] = sr.h[1] = 0;
  for (auto& x : sr.e) HIPCHK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  auto flush = [&](int64_t upto) -> int {
    HIPCHK(hipStreamSynchronize(nullptr));
    int32_t bad = 0;
    HIPCHK(hipMemcpy(&bad, d_st.p, 4, hipMemcpyDeviceToHost));
    if (bad) return not_spd();
    const int64_t c = upto - flushed;
    if (c <= 0) return GPT_OK;
    if (w_store) HIPCHK(hipMemcpy(w_store + rr * flushed, kw, 8 * rr * c, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(U_store + nU * flushed, kU, 8 * nU * c, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(V_store + nV * flushed, kV, 8 * nV * c, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(testpred_store + (size_t)Ntest * flushed, ktp, 8 * (size_t)Ntest * c,
                     hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(rm.data(), krm, 16 * c, hipMemcpyDeviceToHost));
    for (int64_t s2 = 0; s2 < c; ++s2) {
      trainRMSE[flushed + s2] = rm[2 * s2];
      testRMSE[flushed + s2] = rm[2 * s2 + 1];
    }
    flushed = upto;
    return GPT_OK;
  };
  const double su2 = sigma_u * sigma_u;
  int counter = 0;
  uint32_t sweep = 0;
  for (int64_t epoch = 1; epoch <= burnin + maxepoch; ++epoch) {
    for (int64_t g = 0; g < n_samples; ++g, ++sweep) {
      hipError_t e = launch_cfg_rows(0, (int)r, d_w.as<double>(), d_V.as<double>(), (int)n2,
                                     d_U.as<double>(), (int)n1, d_up.as<int32_t>(), d_ul.as<int32_t>(),
                                     d_tm.as<int32_t>(), d_tr.as<double>(), signal_var, su2, seed,
                                     sweep, kCfgU, d_st.as<int32_t>(), nullptr);
      if (e == hipSuccess)
        e = launch_cfg_rows(1, (int)r, d_w.as<double>(), d_U.as<double>(), (int)n1, d_V.as<double>(),
                            (int)n2, d_mp.as<int32_t>(), d_ml.as<int32_t>(), d_tu.as<int32_t>(),
                            d_tr.as<double>(), signal_var, su2, seed, sweep, kCfgV,
                            d_st.as<int32_t>(), nullptr);
      if (e == hipSuccess && !fixw)
        e = launch_cfg_wsystem((int)r, d_U.as<double>(), (int)n1, d_V.as<double>(), (int)n2,
                               d_up.as<int32_t>(), d_ul.as<int32_t>(), d_tm.as<int32_t>(),
                               d_tr.as<double>(), 1.0 / signal_var, 1.0 / (sigma_w * sigma_w),
                               1.0 / signal_var, d_ws.as<double>(), d_M.as<double>(),
                               d_x.as<double>(), nullptr);
      if (e == hipSuccess && !fixw)
        e = gaussian_draw_prec(d_M.as<double>(), p, d_x.as<double>(), seed, sweep, kCfgW, 0,
                               d_z.as<double>(), d_w.as<double>(), d_st.as<int32_t>(), nullptr);
      if (e != hipSuccess) return hip_fail(e, name);
    }
    if (epoch > burnin) {
      const int64_t s2 = epoch - burnin - 1, slot = (s2 - flushed);
      if (w_store) HIPCHK(hipMemcpyAsync(kw + rr * slot, d_w.p, 8 * rr, hipMemcpyDeviceToDevice, nullptr));
      HIPCHK(hipMemcpyAsync(kU + nU * slot, d_U.p, 8 * nU, hipMemcpyDeviceToDevice, nullptr));
      HIPCHK(hipMemcpyAsync(kV + nV * slot, d_V.p, 8 * nV, hipMemcpyDeviceToDevice, nullptr));
      if (!avg) counter = 0;
      hipError_t e = launch_cf_eval(P, d_ch.as<CfChain>(), 1, (int)std::max(N, Ntest), counter,
                                    nullptr);
      if (e == hipSuccess)
        e = launch_cfg_keep(d_ch.as<CfChain>(), (int)Ntest, neval, krm + 2 * slot,
                            ktp + (size_t)Ntest * slot, nullptr);
      if (e != hipSuccess) return hip_fail(e, "cf eval kernel");
      counter += 1;
      if (slot + 1 == chunkE) {
        const int rc = flush(s2 + 1);
        if (rc != GPT_OK) return rc;
      }
    }
    const int ring = (int)(epoch & 1);
    HIPCHK(hipMemcpyAsync(sr.h + ring, d_st.p, 4, hipMemcpyDeviceToHost, nullptr));
    HIPCHK(hipEventRecord(sr.e[ring], nullptr));
    if (epoch > 1) {                        // the previous epoch's status, one epoch behind
      HIPCHK(hipEventSynchronize(sr.e[ring ^ 1]));
      if (sr.h[ring ^ 1]) {
        HIPCHK(hipStreamSynchronize(nullptr));
        return not_spd();
      }
    }
  }
  return flush(maxepoch);
}

extern "C" int gpt_cf_fullw_gibbs(
    const double* Rating, int64_t N, int64_t ldr, int64_t n1, int64_t n2, const double* Ratingtest,
    int64_t Ntest, int64_t ldt, double signal_var, double sigma_u, double sigma_w,
    const double* w_init, int64_t r, int64_t burnin, int64_t maxepoch, int64_t n_samples,
    uint64_t seed, double ytrainMean, double ytrainStd, int32_t avg, int32_t rotated_w,
    double* w_store, double* U_store, double* V_store, double* testpred_store, double* trainRMSE,
    double* testRMSE) {
  return cf_gibbs_run("GPT_fullw_gibbs", Rating, N, ldr, n1, n2, Ratingtest, Ntest, ldt,
                      signal_var, sigma_u, sigma_w, w_init, r, burnin, maxepoch, n_samples, seed,
                      ytrainMean, ytrainStd, avg, rotated_w, false, w_store, U_store, V_store,
                      testpred_store, trainRMSE, testRMSE);
}

extern "C" int gpt_cf_fixw_gibbs(
    const double* Rating, int64_t N, int64_t ldr, int64_t n1, int64_t n2, const double* Ratingtest,
    int64_t Ntest, int64_t ldt, double signal_var, double sigma_u, const double* w, int64_t r,
    int64_t burnin, int64_t maxepoch, int64_t n_samples, uint64_t seed, double ytrainMean,
    double ytrainStd, int32_t avg, int32_t rotated_w, double* U_store, double* V_store,
    double* testpred_store, double* trainRMSE, double* testRMSE) {
  return cf_gibbs_run("GPT_fixw_gibbs", Rating, N, ldr, n1, n2, Ratingtest, Ntest, ldt,
                      signal_var, sigma_u, 1.0, w, r, burnin, maxepoch, n_samples, seed,
                      ytrainMean, ytrainStd, avg, rotated_w, true, nullptr, U_store, V_store,
                      testpred_store, trainRMSE, testRMSE);
}
