// hbx_api.hip -- the extern "C" boundary declared in include/hbx.h.
//
// Plans own twiddle / transfer-function tables (built once in float64 on the
// host) and a per-job workspace.  Entry points only enqueue work on the given
// stream: no allocation, copy or synchronisation happens inside a launch
// function after the plan exists, so callers may capture them in hipGraphs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "hbx.h"
#include "hbx_internal.hpp"

using hbx::EnvDev;
using hbx::EnvParams;
using hbx::JobDesc;
using hbx::PlanDev;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HBX_HIP(expr)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return fail(HBX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
  } while (0)

}  // namespace

struct hbx_plan {
  hbx_optics_t optics;
  PlanDev pd;
  int device;
  int max_jobs;
  size_t ws_bytes;
  JobDesc* jobs;          // [max_jobs]
  JobDesc* full_jobs;     // [max_jobs] (env i / G, group i % G): the jobs of every full propagation
                          // without env ids, built once (ABI v14: one launch fewer per tt.simulate)
  float* job_inten;       // [max_jobs][N][N]
  int32_t* accept_flag;   // [max_jobs]
  int32_t* err;           // [1]
  double* delta;          // [max_jobs] psnr change per step (importance rewards)
  // flip-map workspace (lazy, hbx_flip_map)
  float2* map_field = nullptr;   // [CH][N][N]
  float* map_inten = nullptr;    // [G][N][N]
  double* map_stats = nullptr;   // [G][3] + psnr
  float2* map_q = nullptr;       // [G][4][N][N] h-side spectra
  double* map_d4 = nullptr;      // [G]
  double* map_part = nullptr;    // [G][64]
  float2* map_x = nullptr;       // [4P + P/2 + 1][N][N]
  float2* map_s = nullptr;       // same size: FFT scratch
  float2* map_y = nullptr;       // [P + P/2 + 1][N][N]
  double* walk_partial = nullptr;  // [kWalkMaxK x blocks][2] (lazy, hbx_dbs_walk_psf)
  size_t walk_partial_elems = 0;
  int* walk_counter = nullptr;     // fused walk step: arrival tickets [9] (zero between launches)
  int walk_split = 0;              // HBX_WALK_SPLIT=1: three-launch batches for every K
  int walk_persist = 0;            // HBX_WALK_PERSIST=1: one cooperative launch per walk call
  int32_t* planes_ticket = nullptr;  // hbx_dbs_walk_planes: the fused decision's arrival counter
  int32_t* walk_ring = nullptr;      // (r06) its candidate-slot ring base (WalkPlanesArgs::ring)
  uint8_t* walk_phase = nullptr;     // (r06) [max_jobs] what each job slot still needs (::phase)
};

namespace {

int check_plan(hbx_plan_t p) {
  if (!p) return fail(HBX_ERR_INVALID, "null plan");
  return HBX_OK;
}

double fftfreq(int k, int n, double d) {
  const int kk = (k < (n + 1) / 2) ? k : k - n;  // numpy.fft.fftfreq ordering
  return (double)kk / ((double)n * d);
}

std::complex<double> transfer(const hbx_optics_t& o, double wl, double fx, double fy) {
  const double f2 = fx * fx + fy * fy;
  if (o.tf_kind == HBX_TF_ASM) {
    const double arg = 1.0 / (wl * wl) - f2;
    if (arg <= 0.0) return {0.0, 0.0};
    // |U|^2 is blind to the global phase 2 pi z / wl; keep it anyway (double).
    const double ph = 2.0 * M_PI * o.z * std::sqrt(arg);
    return {std::cos(ph), std::sin(ph)};
  }
  const double ph = 2.0 * M_PI * o.z / wl - M_PI * wl * o.z * f2;
  return {std::cos(ph), std::sin(ph)};
}

}  // namespace

extern "C" {

int hbx_abi_version(void) { return HBX_ABI_VERSION; }

int hbx_host_alloc(size_t bytes, void** host, void** device) {
  if (!host || !device || bytes == 0) return fail(HBX_ERR_INVALID, "hbx_host_alloc: null pointer or zero size");
  *host = nullptr;
  *device = nullptr;
  void* h = nullptr;
  // portable: a rank's process may run on any device (LOCAL_RANK), not the current one at alloc
  if (hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess || !h)
    return fail(HBX_ERR_NOMEM, "hipHostMalloc");
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
    (void)hipHostFree(h);
    return fail(HBX_ERR_HIP, "hipHostGetDevicePointer");
  }
  *host = h;
  *device = d;
  return HBX_OK;
}

int hbx_host_free(void* host) {
  if (!host) return HBX_OK;
  HBX_HIP(hipHostFree(host));
  return HBX_OK;
}

const char* hbx_last_error(void) { return g_last_error.c_str(); }

int hbx_plan_create(hbx_plan_t* out, const hbx_optics_t* o, int32_t max_jobs, int32_t device) {
  if (!out || !o) return fail(HBX_ERR_INVALID, "null argument");
  *out = nullptr;
  if (o->height != o->width) return fail(HBX_ERR_UNSUPPORTED, "only square N x N masks are built");
  int R = 0;
  if (o->height == 1024) R = 32;
  else if (o->height == 256) R = 16;
  else if (o->height == 64) R = 8;
  else if (o->height == 896) R = 0;   // crop of a 1024 mask: generic 28 x 32 path
  else return fail(HBX_ERR_UNSUPPORTED, "N must be 64, 256, 896 or 1024");
  if (o->groups < 1 || o->groups > HBX_MAX_GROUPS) return fail(HBX_ERR_INVALID, "groups out of range");
  if (o->planes < 2 || (o->planes % 2)) return fail(HBX_ERR_INVALID, "planes must be even and >= 2");
  if (max_jobs < o->groups) return fail(HBX_ERR_INVALID, "max_jobs must be >= groups");
  if (o->tf_kind != HBX_TF_ASM && o->tf_kind != HBX_TF_FRESNEL) return fail(HBX_ERR_INVALID, "tf_kind");
  if (o->field_kind != HBX_FIELD_AMPLITUDE && o->field_kind != HBX_FIELD_PHASE)
    return fail(HBX_ERR_INVALID, "field_kind");
  if (o->rel_scale != HBX_REL_NONE && o->rel_scale != HBX_REL_LSQ) return fail(HBX_ERR_INVALID, "rel_scale");
  for (int g = 0; g < o->groups; ++g)
    if (!(o->wavelength[g] > 0.0)) return fail(HBX_ERR_INVALID, "wavelength must be > 0");
  if (!(o->dx > 0.0) || !(o->dy > 0.0)) return fail(HBX_ERR_INVALID, "pixel pitch must be > 0");

  HBX_HIP(hipSetDevice(device));
  hbx_plan* p = new (std::nothrow) hbx_plan();
  if (!p) return fail(HBX_ERR_NOMEM, "host allocation");
  std::memset(p, 0, sizeof(*p));
  p->optics = *o;
  p->device = device;
  p->max_jobs = max_jobs;
  const int N = o->height, G = o->groups, P = o->planes;
  PlanDev& pd = p->pd;
  pd.R = R; pd.N = N; pd.G = G; pd.P = P;
  if (o->field_kind == HBX_FIELD_AMPLITUDE) { pd.va = 0.0f; pd.vb = 1.0f; }
  else { pd.va = 1.0f; pd.vb = -2.0f; }

  // host tables in float64, rounded once to complex64
  std::vector<float2> tw((size_t)N);
  for (int k1 = 0; k1 < R; ++k1)
    for (int t = 0; t < R; ++t) {
      const double a = -2.0 * M_PI * (double)((t * k1) % N) / (double)N;
      tw[(size_t)k1 * R + t] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
  if (R == 0)   // N = 896: [k1 < 28][t < 32] = W896^{t k1}
    for (int k1 = 0; k1 < 28; ++k1)
      for (int t = 0; t < 32; ++t) {
        const double a = -2.0 * M_PI * (double)(t * k1) / (double)N;
        tw[(size_t)k1 * 32 + t] = make_float2((float)std::cos(a), (float)std::sin(a));
      }
  {
    const char* ev = std::getenv("HBX_WALK_SPLIT");   // A/B switch: the v5 three-launch walk batches
    p->walk_split = (ev && ev[0] && ev[0] != '0') ? 1 : 0;
    const char* ep = std::getenv("HBX_WALK_PERSIST");   // the persistent fused walk (r03, measured)
    p->walk_persist = (ep && ep[0] && ep[0] != '0') ? 1 : 0;
  }
  const size_t hrow = (size_t)(N / 2 + 1) * N;
  std::vector<float2> ht((size_t)G * hrow);
  // ifft2 normalisation, and 1/2: the row passes write 2 A (their Hermitian split drops its
  // 0.5 factors, r06), the column passes multiply by H / 2 -- powers of two, so every product
  // and so B are the bits of A x H (hbx_passes.hip, pass 1).  Only the column passes read ht.
  const double scale = 0.5 / ((double)N * (double)N);
  for (int g = 0; g < G; ++g)
    for (int kx = 0; kx <= N / 2; ++kx) {
      const double fx = fftfreq(kx, N, o->dx);
      for (int ky = 0; ky < N; ++ky) {
        const double fy = fftfreq(ky, N, o->dy);
        const std::complex<double> h = transfer(*o, o->wavelength[g], fx, fy) * scale;
        ht[g * hrow + (size_t)kx * N + ky] = make_float2((float)h.real(), (float)h.imag());
      }
    }
  // partial slots per job: row blocks of the last pass (8 rows each on the generic path)
  const int RB = R ? N / (256 / R) : N / 8;
  // the generic path ping-pongs full planes between A and B
  const size_t ws_a_bytes = (size_t)max_jobs * P * (R ? hbx::plane_a_elems(R) : (size_t)N * N) * sizeof(float2);
  const size_t ws_b_bytes = (size_t)max_jobs * P * (R ? hbx::plane_b_elems(R) : (size_t)N * N) * sizeof(float2);
  p->ws_bytes = ws_a_bytes + ws_b_bytes;
  auto cleanup = [&](int code, const std::string& msg) {
    hbx_plan_destroy(p);
    return fail(code, msg);
  };
  if (hipMalloc(&pd.tw, tw.size() * sizeof(float2)) != hipSuccess) return cleanup(HBX_ERR_NOMEM, "tw");
  if (hipMalloc(&pd.htab, ht.size() * sizeof(float2)) != hipSuccess) return cleanup(HBX_ERR_NOMEM, "htab");
  if (hipMalloc(&pd.ws_a, ws_a_bytes) != hipSuccess) return cleanup(HBX_ERR_NOMEM, "workspace A");
  if (hipMalloc(&pd.ws_b, ws_b_bytes) != hipSuccess) return cleanup(HBX_ERR_NOMEM, "workspace B");
  if (hipMalloc(&pd.partial, (size_t)max_jobs * RB * 3 * sizeof(double)) != hipSuccess)
    return cleanup(HBX_ERR_NOMEM, "partial");
  if (hipMalloc(&pd.job_stats, (size_t)max_jobs * 3 * sizeof(double)) != hipSuccess)
    return cleanup(HBX_ERR_NOMEM, "job_stats");
  if (hipMalloc(&p->jobs, (size_t)max_jobs * sizeof(JobDesc)) != hipSuccess) return cleanup(HBX_ERR_NOMEM, "jobs");
  if (hipMalloc(&p->full_jobs, (size_t)max_jobs * sizeof(JobDesc)) != hipSuccess)
    return cleanup(HBX_ERR_NOMEM, "full jobs");
  // the plane-cache walk's arrival counter (zero between launches; its user resets it): allocated
  // and zeroed here, not on a walk's first call (no blocking memset inside a hot / captured call)
  if (hipMalloc(&p->planes_ticket, 64) != hipSuccess) return cleanup(HBX_ERR_NOMEM, "walk ticket");
  if (hipMalloc(&p->walk_ring, 64) != hipSuccess) return cleanup(HBX_ERR_NOMEM, "walk ring");
  if (hipMalloc(&p->walk_phase, (size_t)max_jobs) != hipSuccess) return cleanup(HBX_ERR_NOMEM, "walk phase");
  if (hipMalloc(&p->accept_flag, (size_t)max_jobs * sizeof(int32_t)) != hipSuccess)
    return cleanup(HBX_ERR_NOMEM, "accept_flag");
  if (hipMalloc(&p->err, sizeof(int32_t)) != hipSuccess) return cleanup(HBX_ERR_NOMEM, "err");
  if (hipMalloc(&p->delta, (size_t)max_jobs * sizeof(double)) != hipSuccess) return cleanup(HBX_ERR_NOMEM, "delta");
  if (hipMalloc(&pd.psf_partial, (size_t)max_jobs * hbx::kPsfBlocks * 2 * sizeof(double)) != hipSuccess)
    return cleanup(HBX_ERR_NOMEM, "psf partials");
  if (hipMalloc(&pd.psf_order, (size_t)max_jobs * sizeof(int32_t)) != hipSuccess)
    return cleanup(HBX_ERR_NOMEM, "psf order");
  if (hipMalloc(&pd.zero_row, (size_t)N * sizeof(float)) != hipSuccess) return cleanup(HBX_ERR_NOMEM, "zero row");
  if (hipMemcpy(pd.tw, tw.data(), tw.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(pd.htab, ht.data(), ht.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(p->err, 0, sizeof(int32_t)) != hipSuccess ||
      hipMemset(pd.zero_row, 0, (size_t)N * sizeof(float)) != hipSuccess ||
      hipMemset(p->planes_ticket, 0, 64) != hipSuccess ||
      hipMemset(p->walk_ring, 0, 64) != hipSuccess ||
      hipMemset(p->walk_phase, 0, (size_t)max_jobs) != hipSuccess ||
      hbx::launch_jobs_full(nullptr, max_jobs / G, G, p->full_jobs, nullptr) != hipSuccess ||
      hipStreamSynchronize(nullptr) != hipSuccess)
    return cleanup(HBX_ERR_HIP, "table upload");
  *out = p;
  return HBX_OK;
}

int hbx_plan_destroy(hbx_plan_t p) {
  if (!p) return HBX_OK;
  (void)hipSetDevice(p->device);
  if (p->pd.tw) (void)hipFree(p->pd.tw);
  if (p->pd.htab) (void)hipFree(p->pd.htab);
  if (p->pd.ws_a) (void)hipFree(p->pd.ws_a);
  if (p->pd.ws_b) (void)hipFree(p->pd.ws_b);
  if (p->pd.partial) (void)hipFree(p->pd.partial);
  if (p->pd.job_stats) (void)hipFree(p->pd.job_stats);
  if (p->jobs) (void)hipFree(p->jobs);
  if (p->full_jobs) (void)hipFree(p->full_jobs);
  if (p->job_inten) (void)hipFree(p->job_inten);
  if (p->accept_flag) (void)hipFree(p->accept_flag);
  if (p->err) (void)hipFree(p->err);
  if (p->delta) (void)hipFree(p->delta);
  if (p->pd.hpsf) (void)hipFree(p->pd.hpsf);
  if (p->pd.psf_partial) (void)hipFree(p->pd.psf_partial);
  if (p->walk_partial) (void)hipFree(p->walk_partial);
  if (p->walk_counter) (void)hipFree(p->walk_counter);
  if (p->planes_ticket) (void)hipFree(p->planes_ticket);
  if (p->walk_ring) (void)hipFree(p->walk_ring);
  if (p->walk_phase) (void)hipFree(p->walk_phase);
  if (p->pd.psf_order) (void)hipFree(p->pd.psf_order);
  if (p->pd.zero_row) (void)hipFree(p->pd.zero_row);
  for (void* q : {(void*)p->map_field, (void*)p->map_inten, (void*)p->map_stats, (void*)p->map_q,
                  (void*)p->map_d4, (void*)p->map_part, (void*)p->map_x, (void*)p->map_s, (void*)p->map_y})
    if (q) (void)hipFree(q);
  hbx_plan_set_timing(p, 0);
  delete p;
  return HBX_OK;
}

size_t hbx_plan_workspace_bytes(hbx_plan_t p) { return p ? p->ws_bytes : 0; }

int hbx_plan_set_precision(hbx_plan_t p, int32_t precision) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (precision < HBX_PRECISION_F32 || precision > HBX_PRECISION_F16_STORE)
    return fail(HBX_ERR_INVALID, "precision must be HBX_PRECISION_F32, _BF16_STORE or _F16_STORE");
  if (precision != HBX_PRECISION_F32 && p->pd.R == 0)
    return fail(HBX_ERR_UNSUPPORTED, "reduced-precision intermediates: N = 64 / 256 / 1024 only");
  p->pd.store_kind = precision;
  return HBX_OK;
}

int hbx_plan_precision(hbx_plan_t p) {
  int rc = check_plan(p);
  if (rc) return rc;
  return p->pd.store_kind;
}

int hbx_plan_pipeline(hbx_plan_t p) {
  int rc = check_plan(p);
  if (rc) return rc;
  return HBX_PIPE_THREE_PASS;   // the only pipeline built since ABI v8
}

}  // extern "C"

namespace {

int ensure_job_inten(hbx_plan_t p) {
  if (p->job_inten) return HBX_OK;
  const size_t bytes = (size_t)p->max_jobs * p->pd.N * p->pd.N * sizeof(float);
  if (hipMalloc(&p->job_inten, bytes) != hipSuccess) return fail(HBX_ERR_NOMEM, "job intensity buffer");
  return HBX_OK;
}

double pixel_count(const hbx_plan_t p) {
  return (double)p->pd.G * (double)p->pd.N * (double)p->pd.N;
}

// Single-pixel fields h_g = IFFT2(H_g), computed once with the exact FFT path:
// one env whose mask has only pixel (0, 0) of plane g*P set, propagated as an
// amplitude field (va = 0, vb = 1) whatever the plan's field encoding, so
// plane g*P's output field is h_g.  Allocates: call outside graph capture.
int ensure_hpsf(hbx_plan_t p, hipStream_t st) {
  PlanDev& pd = p->pd;
  if (pd.hpsf) return HBX_OK;
  const int N = pd.N, G = pd.G, P = pd.P, CH = G * P;
  const size_t hw = (size_t)N * N;
  uint64_t* mask = nullptr;
  float* target = nullptr;
  float2* field = nullptr;
  float2* h = nullptr;
  auto release = [&]() {
    if (mask) (void)hipFree(mask);
    if (target) (void)hipFree(target);
    if (field) (void)hipFree(field);
  };
  if (hipMalloc(&mask, (size_t)CH * N * (N / 64) * sizeof(uint64_t)) != hipSuccess ||
      hipMalloc(&target, (size_t)G * hw * sizeof(float)) != hipSuccess ||
      hipMalloc(&field, (size_t)CH * hw * sizeof(float2)) != hipSuccess ||
      hipMalloc(&h, (size_t)G * hw * sizeof(float2)) != hipSuccess) {
    release();
    if (h) (void)hipFree(h);
    return fail(HBX_ERR_NOMEM, "single-pixel field tables");
  }
  std::vector<uint64_t> m((size_t)CH * N * (N / 64), 0);
  for (int g = 0; g < G; ++g) m[(size_t)g * P * N * (N / 64)] = 1ull;  // pixel (0,0) of plane g*P
  if (hipMemcpyAsync(mask, m.data(), m.size() * sizeof(uint64_t), hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemsetAsync(target, 0, (size_t)G * hw * sizeof(float), st) != hipSuccess) {
    release();
    (void)hipFree(h);
    return fail(HBX_ERR_HIP, "single-pixel field setup");
  }
  PlanDev amp = pd;
  amp.va = 0.0f;
  amp.vb = 1.0f;
  amp.timer = nullptr;
  amp.store_kind = HBX_PRECISION_F32;   // h is a table of the product path, whatever the plan's precision
  hipError_t e = hbx::launch_jobs_full(nullptr, 1, G, p->jobs, st);
  if (e == hipSuccess)
    e = hbx::run_jobs(amp, p->jobs, G, reinterpret_cast<const uint32_t*>(mask), target, nullptr, field, st);
  for (int g = 0; g < G && e == hipSuccess; ++g)
    e = hipMemcpyAsync(h + (size_t)g * hw, field + (size_t)g * P * hw, hw * sizeof(float2),
                       hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  release();
  if (e != hipSuccess) {
    (void)hipFree(h);
    return fail(HBX_ERR_HIP, std::string("single-pixel field: ") + hipGetErrorString(e));
  }
  pd.hpsf = h;
  return HBX_OK;
}

EnvDev env_dev(const hbx_env_buffers_t* e) {
  EnvDev d;
  d.mask = e->mask; d.record = e->record; d.target = e->target; d.chan_stats = e->chan_stats;
  d.init_psnr = e->init_psnr; d.prev_psnr = e->prev_psnr; d.max_psnr_diff = e->max_psnr_diff;
  d.steps = e->steps; d.flip_count = e->flip_count; d.sustained = e->sustained;
  d.imp_changes = e->imp_changes; d.imp_values = e->imp_values; d.t_psnr_diff = e->t_psnr_diff;
  d.imp_count = e->imp_count;
  d.state_bytes = e->state_bytes;
  d.recon_pending = e->recon_pending;
  d.plane_slot = (e->plane_inten && e->plane_slot) ? e->plane_slot : nullptr;
  d.error = e->error;
  d.error_host = e->error_host;
  return d;
}

EnvDev env_offset(const EnvDev& d, size_t e0, int CH, int G, int N) {
  EnvDev o = d;
  const size_t mwords = (size_t)CH * N * (N / 64);
  o.mask = d.mask + e0 * mwords;
  o.record = d.record ? d.record + e0 * (size_t)CH * N * N : nullptr;
  o.target = d.target + e0 * (size_t)G * N * N;
  o.chan_stats = d.chan_stats + e0 * G * 3;
  o.init_psnr = d.init_psnr + e0;
  o.prev_psnr = d.prev_psnr + e0;
  o.max_psnr_diff = d.max_psnr_diff + e0;
  o.steps = d.steps + e0;
  o.flip_count = d.flip_count + e0;
  o.sustained = d.sustained + e0;
  o.imp_changes = d.imp_changes ? d.imp_changes + e0 * (size_t)d.imp_count : nullptr;
  o.imp_values = d.imp_values ? d.imp_values + e0 * (size_t)d.imp_count : nullptr;
  o.t_psnr_diff = d.t_psnr_diff ? d.t_psnr_diff + e0 : nullptr;
  o.state_bytes = d.state_bytes ? d.state_bytes + e0 * (size_t)CH * N * N : nullptr;
  o.recon_pending = d.recon_pending ? d.recon_pending + e0 : nullptr;
  o.plane_slot = d.plane_slot ? d.plane_slot + e0 * (size_t)(CH + 2) : nullptr;
  return o;
}

// the observation buffers a step writes need the caches they mirror
int check_obs_buffers(const hbx_env_buffers_t* e) {
  if (e->recon && (!e->intensity || !e->recon_pending))
    return fail(HBX_ERR_INVALID, "env.recon needs env.intensity and env.recon_pending");
  return HBX_OK;
}

// full propagation of n_ids envs (absolute ids from env_ids, or 0..n_ids-1)
int propagate_full(hbx_plan_t p, const uint64_t* mask, const float* target, const int32_t* env_ids,
                   int n_ids, float* intensity, double* chan_stats, double* psnr, const EnvDev* env,
                   float2* field, hipStream_t st, float* plane_pool = nullptr, int32_t* plane_slot = nullptr,
                   int spares = 1) {
  const PlanDev& pd = p->pd;
  const int CHs = pd.G * pd.P + 2 * spares;   // plane-cache slots per env
  if (plane_pool) {                           // identity slots, then every plane's |U|^2 into its slot
    if (pd.R != 32 && pd.R != 16 && pd.R != 0)
      return fail(HBX_ERR_UNSUPPORTED, "plane cache: N = 1024, 896 or 256 only");
    HBX_HIP(hbx::launch_plane_slot_init(env_ids, n_ids, plane_slot, CHs, st));
  }
  const int G = pd.G;
  const int chunk = p->max_jobs / G;
  if (intensity) {
    int rc = ensure_job_inten(p);
    if (rc) return rc;
  }
  EnvDev dummy;
  std::memset(&dummy, 0, sizeof(dummy));
  for (int i0 = 0; i0 < n_ids; i0 += chunk) {
    const int n = std::min(chunk, n_ids - i0);
    // with env_ids the jobs carry absolute env ids; without, ids are chunk-local
    // and every per-env buffer is offset by i0 instead
    // with env ids the jobs are built per chunk; without, they are the plan's constant table
    JobDesc* jobs = env_ids ? p->jobs : p->full_jobs;
    if (env_ids) HBX_HIP(hbx::launch_jobs_full(env_ids + i0, n, G, jobs, st));
    const size_t mwords = (size_t)G * pd.P * pd.N * (pd.N / 64);
    const uint64_t* m = env_ids ? mask : mask + (size_t)i0 * mwords;
    const float* tg = (env_ids || !target) ? target : target + (size_t)i0 * G * pd.N * pd.N;
    float2* fo = field ? (env_ids ? field : field + (size_t)i0 * G * pd.P * pd.N * pd.N) : nullptr;
    PlanDev pdx = pd;
    if (plane_pool) {
      pdx.plane_mode = hbx::kPlanesFill;
      pdx.plane_spares = spares;
      pdx.plane_pool = env_ids ? plane_pool : plane_pool + (size_t)i0 * CHs * pd.N * pd.N;
      pdx.plane_slot = env_ids ? plane_slot : plane_slot + (size_t)i0 * CHs;
    }
    HBX_HIP(hbx::run_jobs(pdx, jobs, n * G, reinterpret_cast<const uint32_t*>(m), tg,
                          intensity ? p->job_inten : nullptr, fo, st));
    double* cs = (env_ids || !chan_stats) ? chan_stats : chan_stats + (size_t)i0 * G * 3;
    double* ps = psnr ? (env_ids ? psnr : psnr + i0) : nullptr;
    EnvDev ed = dummy;
    if (env) ed = env_ids ? *env : env_offset(*env, i0, G * pd.P, G, pd.N);
    if (cs || ps || env)   // tt.simulate alone (fields only) has nothing to finalize
      HBX_HIP(hbx::launch_full_finalize(jobs, pd.job_stats, n, G, cs, ps, pixel_count(p),
                                        p->optics.rel_scale, p->optics.peak, ed, env ? 1 : 0, st));
    if (intensity) {
      float* cache = env_ids ? intensity : intensity + (size_t)i0 * G * pd.N * pd.N;
      HBX_HIP(hbx::launch_scatter_intensity(jobs, n * G, p->job_inten, cache, G,
                                            (size_t)pd.N * pd.N, nullptr, st));
    }
  }
  return HBX_OK;
}

}  // namespace

extern "C" {

int hbx_propagate(hbx_plan_t p, const uint64_t* mask, const float* target, int32_t n_env,
                  float* intensity, double* chan_stats, double* psnr, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (n_env <= 0) return n_env == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "n_env");  // empty: null buffers allowed
  if (!mask || !target || !chan_stats) return fail(HBX_ERR_INVALID, "null buffer");
  HBX_HIP(hipSetDevice(p->device));
  return propagate_full(p, mask, target, nullptr, n_env, intensity, chan_stats, psnr, nullptr,
                        nullptr, (hipStream_t)stream);
}

int hbx_simulate(hbx_plan_t p, const uint64_t* mask, int32_t n_env, float* field, float* intensity,
                 void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (n_env <= 0) return n_env == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "n_env");
  if (!mask || !field) return fail(HBX_ERR_INVALID, "null buffer");
  HBX_HIP(hipSetDevice(p->device));
  return propagate_full(p, mask, nullptr, nullptr, n_env, intensity, nullptr, nullptr, nullptr,
                        reinterpret_cast<float2*>(field), (hipStream_t)stream);
}

int hbx_psnr(hbx_plan_t p, const double* chan_stats, int32_t n_env, double* psnr, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (n_env <= 0) return n_env == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "n_env");
  if (!chan_stats || !psnr) return fail(HBX_ERR_INVALID, "null buffer");
  HBX_HIP(hipSetDevice(p->device));
  HBX_HIP(hbx::launch_psnr(chan_stats, n_env, p->pd.G, psnr, pixel_count(p), p->optics.rel_scale,
                           p->optics.peak, (hipStream_t)stream));
  return HBX_OK;
}

int hbx_env_reset(hbx_plan_t p, const hbx_env_buffers_t* e, int32_t n_env, const int32_t* env_ids,
                  int32_t n_ids, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (!e || !e->mask || !e->target || !e->chan_stats || !e->init_psnr || !e->prev_psnr ||
      !e->max_psnr_diff || !e->steps || !e->flip_count || !e->sustained)
    return fail(HBX_ERR_INVALID, "env buffers incomplete");
  if (n_env < 0) return fail(HBX_ERR_INVALID, "n_env");
  const int n = env_ids ? n_ids : n_env;
  if (n <= 0) return HBX_OK;
  HBX_HIP(hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  const PlanDev& pd = p->pd;
  const int CH = pd.G * pd.P;
  if (e->record)
    HBX_HIP(hbx::launch_zero_record(e->record, env_ids, n, (size_t)CH * pd.N * pd.N, st));
  if (e->field) {
    if (!e->intensity) return fail(HBX_ERR_INVALID, "env.field needs env.intensity");
    rc = ensure_hpsf(p, st);
    if (rc) return rc;
  }
  rc = check_obs_buffers(e);
  if (rc) return rc;
  EnvDev ed = env_dev(e);
  const bool planes = e->plane_inten && e->plane_slot;
  if ((e->plane_inten != nullptr) != (e->plane_slot != nullptr))
    return fail(HBX_ERR_INVALID, "plane cache: give both plane_inten and plane_slot");
  if (planes && e->field) return fail(HBX_ERR_INVALID, "plane cache and env.field (incremental mode) are exclusive");
  rc = propagate_full(p, e->mask, e->target, env_ids, n, e->intensity, e->chan_stats, nullptr, &ed,
                      reinterpret_cast<float2*>(e->field), st, planes ? e->plane_inten : nullptr,
                      planes ? e->plane_slot : nullptr);
  if (rc) return rc;
  HBX_HIP(hbx::launch_obs_sync(env_ids, n, e->mask, e->state_bytes, e->intensity, e->recon, e->recon_pending,
                               0, CH, pd.G, (size_t)pd.N * pd.N, st));
  return HBX_OK;
}

int hbx_env_obs_sync(hbx_plan_t p, const hbx_env_buffers_t* e, int32_t n_env, const int32_t* env_ids,
                     int32_t n_ids, int32_t what, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (!e) return fail(HBX_ERR_INVALID, "null env buffers");
  if (what == HBX_OBS_SETTLE) {
    if (!e->recon || !e->intensity || !e->recon_pending)
      return fail(HBX_ERR_INVALID, "HBX_OBS_SETTLE needs recon, intensity and recon_pending");
    if (n_env < 0) return fail(HBX_ERR_INVALID, "n_env");
    const int n = env_ids ? n_ids : n_env;
    if (n <= 0) return n == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "n_ids");
    if (p->pd.G == 1) return HBX_OK;   // (ABI v12) nothing is ever pending with one group
    HBX_HIP(hipSetDevice(p->device));
    HBX_HIP(hbx::launch_obs_settle(env_ids, n, e->intensity, e->recon, e->recon_pending, p->pd.G,
                                   (size_t)p->pd.N * p->pd.N, (hipStream_t)stream));
    return HBX_OK;
  }
  if (what & ~(HBX_OBS_STATE | HBX_OBS_RECON | HBX_OBS_RESOLVE))
    return fail(HBX_ERR_INVALID, "what: HBX_OBS_STATE | HBX_OBS_RECON | HBX_OBS_RESOLVE, or HBX_OBS_SETTLE alone");
  if ((what & HBX_OBS_RESOLVE) && !(what & HBX_OBS_RECON))
    return fail(HBX_ERR_INVALID, "HBX_OBS_RESOLVE is a modifier of HBX_OBS_RECON");
  const bool st_on = (what & HBX_OBS_STATE) != 0, rc_on = (what & HBX_OBS_RECON) != 0;
  if (st_on && (!e->mask || !e->state_bytes)) return fail(HBX_ERR_INVALID, "HBX_OBS_STATE needs mask and state_bytes");
  if (rc_on && (!e->recon || !e->intensity || !e->recon_pending))
    return fail(HBX_ERR_INVALID, "HBX_OBS_RECON needs recon, intensity and recon_pending");
  if (n_env < 0) return fail(HBX_ERR_INVALID, "n_env");
  const int n = env_ids ? n_ids : n_env;
  if (n <= 0) return n == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "n_ids");
  HBX_HIP(hipSetDevice(p->device));
  const PlanDev& pd = p->pd;
  if (rc_on && pd.G == 1) {
    // (ABI v12) one group: the step keeps no accepted-intensity cache, so the accepted state's
    // intensity is re-propagated from the mask (the same kernels: the bits the steps compute)
    if (!e->target) return fail(HBX_ERR_INVALID, "HBX_OBS_RECON needs env.target");
    int rc2 = propagate_full(p, e->mask, e->target, env_ids, n, e->intensity, nullptr, nullptr, nullptr, nullptr,
                             (hipStream_t)stream);
    if (rc2) return rc2;
  }
  HBX_HIP(hbx::launch_obs_sync(env_ids, n, e->mask, st_on ? e->state_bytes : nullptr, e->intensity,
                               rc_on ? e->recon : nullptr, e->recon_pending, (what & HBX_OBS_RESOLVE) ? 1 : 0,
                               pd.G * pd.P, pd.G,
                               (size_t)pd.N * pd.N, (hipStream_t)stream));
  return HBX_OK;
}

int hbx_field_refresh(hbx_plan_t p, const hbx_env_buffers_t* e, int32_t n_env, const int32_t* env_ids,
                      int32_t n_ids, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  const bool planes = e && e->plane_inten && e->plane_slot && !e->field;
  if (planes) {   // ABI v9: rebuild the plane cache (and chan_stats / intensity) of the listed envs
    if (!e->mask || !e->target || !e->chan_stats)
      return fail(HBX_ERR_INVALID, "plane-cache refresh needs mask, target and chan_stats");
    const int n = env_ids ? n_ids : n_env;
    if (n <= 0) return n == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "n_env");
    HBX_HIP(hipSetDevice(p->device));
    return propagate_full(p, e->mask, e->target, env_ids, n, e->intensity, e->chan_stats, nullptr, nullptr,
                          nullptr, (hipStream_t)stream, e->plane_inten, e->plane_slot);
  }
  if (!e || !e->mask || !e->target || !e->chan_stats || !e->intensity || !e->field)
    return fail(HBX_ERR_INVALID, "refresh needs mask, target, chan_stats, intensity and field");
  const int n = env_ids ? n_ids : n_env;
  if (n <= 0) return n == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "n_env");
  HBX_HIP(hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  rc = ensure_hpsf(p, st);
  if (rc) return rc;
  return propagate_full(p, e->mask, e->target, env_ids, n, e->intensity, e->chan_stats, nullptr, nullptr,
                        reinterpret_cast<float2*>(e->field), st);
}

int hbx_env_step_psf(hbx_plan_t p, const hbx_env_buffers_t* e, const hbx_env_params_t* prm,
                     int32_t n_env, const int64_t* actions, double* reward, double* psnr,
                     uint8_t* accepted, uint8_t* terminated, uint8_t* truncated, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (!e || !prm || !actions || !e->mask || !e->target || !e->chan_stats || !e->init_psnr ||
      !e->prev_psnr || !e->max_psnr_diff || !e->steps || !e->flip_count || !e->sustained ||
      !e->intensity || !e->field)
    return fail(HBX_ERR_INVALID, "env buffers incomplete (incremental mode needs field + intensity)");
  if (!p->pd.hpsf) return fail(HBX_ERR_INVALID, "incremental mode: call hbx_env_reset with env.field first");
  if (e->recon) return fail(HBX_ERR_INVALID, "env.recon (the pre-rollback recon_image) needs the FFT-mode step");
  if (prm->accept_rule != HBX_ACCEPT_ENV && prm->accept_rule != HBX_ACCEPT_DBS)
    return fail(HBX_ERR_INVALID, "accept_rule");
  if (prm->reward_kind != HBX_REWARD_PSNR && prm->reward_kind != HBX_REWARD_IMPORTANCE)
    return fail(HBX_ERR_INVALID, "reward_kind");
  if (prm->reward_kind == HBX_REWARD_IMPORTANCE && (!e->imp_changes || !e->imp_values || e->imp_count <= 0))
    return fail(HBX_ERR_INVALID, "importance rewards need imp_changes, imp_values and imp_count > 0");
  if (n_env <= 0) return n_env == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "n_env");
  HBX_HIP(hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  const PlanDev& pd = p->pd;
  const int N = pd.N, G = pd.G, P = pd.P, CH = G * P;
  const size_t hw = (size_t)N * N;
  EnvParams ep;
  ep.max_steps = prm->max_steps; ep.t_psnr = prm->t_psnr; ep.t_steps = prm->t_steps;
  ep.t_psnr_diff = prm->t_psnr_diff; ep.reward_weight = prm->reward_weight;
  ep.accept_rule = prm->accept_rule;
  ep.reward_kind = prm->reward_kind;
  EnvDev base = env_dev(e);
  base.plane_slot = nullptr;   // the incremental step leaves a plane cache alone (the modes are exclusive)
  for (int b0 = 0; b0 < n_env; b0 += p->max_jobs) {
    const int n = std::min(p->max_jobs, n_env - b0);
    const EnvDev ed = env_offset(base, b0, CH, G, N);
    float2* fld = reinterpret_cast<float2*>(e->field) + (size_t)b0 * CH * hw;
    float* inten = e->intensity + (size_t)b0 * G * hw;
    // the job decode rides in k_psf_order's launch (actions -> jobs, then the colour sort)
    HBX_HIP(hbx::launch_psf_eval(pd, p->jobs, n, ed.mask, fld, inten, ed.target, ed.chan_stats, st, actions + b0,
                                 e->error ? e->error : p->err));
    HBX_HIP(hbx::launch_env_step_finalize(p->jobs, pd.job_stats, n, G, P, N, N, ed, ep, pixel_count(p),
                                          p->optics.rel_scale, p->optics.peak,
                                          reward ? reward + b0 : nullptr, psnr ? psnr + b0 : nullptr,
                                          accepted ? accepted + b0 : nullptr,
                                          terminated ? terminated + b0 : nullptr,
                                          truncated ? truncated + b0 : nullptr, p->accept_flag, p->delta,
                                          st));
    HBX_HIP(hbx::launch_psf_commit(pd, p->jobs, n, ed.mask, fld, inten, p->accept_flag, st));
  }
  return HBX_OK;
}

int hbx_env_step(hbx_plan_t p, const hbx_env_buffers_t* e, const hbx_env_params_t* prm,
                 int32_t n_env, const int64_t* actions, double* reward, double* psnr,
                 uint8_t* accepted, uint8_t* terminated, uint8_t* truncated, float* group_intensity,
                 void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (!e || !prm || !actions || !e->mask || !e->target || !e->chan_stats || !e->init_psnr ||
      !e->prev_psnr || !e->max_psnr_diff || !e->steps || !e->flip_count || !e->sustained)
    return fail(HBX_ERR_INVALID, "env buffers incomplete");
  if (prm->accept_rule != HBX_ACCEPT_ENV && prm->accept_rule != HBX_ACCEPT_DBS)
    return fail(HBX_ERR_INVALID, "accept_rule");
  if (prm->reward_kind != HBX_REWARD_PSNR && prm->reward_kind != HBX_REWARD_IMPORTANCE)
    return fail(HBX_ERR_INVALID, "reward_kind");
  if (prm->reward_kind == HBX_REWARD_IMPORTANCE && (!e->imp_changes || !e->imp_values || e->imp_count <= 0))
    return fail(HBX_ERR_INVALID, "importance rewards need imp_changes, imp_values and imp_count > 0");
  if (n_env <= 0) return n_env == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "n_env");
  HBX_HIP(hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  const PlanDev& pd = p->pd;
  const int N = pd.N, G = pd.G, P = pd.P, CH = G * P;
  const size_t hw = (size_t)N * N;
  rc = check_obs_buffers(e);
  if (rc) return rc;
  if (e->recon && group_intensity)
    return fail(HBX_ERR_INVALID, "give group_intensity or env.recon, not both (recon holds the stepped group)");
  const bool to_recon = e->recon != nullptr;
  const bool want_inten = !to_recon && (group_intensity || e->intensity);
  if (want_inten) {
    rc = ensure_job_inten(p);
    if (rc) return rc;
  }
  PlanDev pdx = p->pd;            // with recon, k_rowinv writes the stepped group straight into it
  pdx.inten_by_env = to_recon ? 1 : 0;
  if ((e->plane_inten != nullptr) != (e->plane_slot != nullptr))
    return fail(HBX_ERR_INVALID, "plane cache: give both plane_inten and plane_slot");
  const bool planes = e->plane_inten != nullptr;
  if (planes && pd.R != 32 && pd.R != 16 && pd.R != 0)
    return fail(HBX_ERR_UNSUPPORTED, "plane cache: N = 1024, 896 or 256 only");
  if (planes) pdx.plane_mode = hbx::kPlanesStep;
  EnvParams ep;
  ep.max_steps = prm->max_steps; ep.t_psnr = prm->t_psnr; ep.t_steps = prm->t_steps;
  ep.t_psnr_diff = prm->t_psnr_diff; ep.reward_weight = prm->reward_weight;
  ep.accept_rule = prm->accept_rule;
  ep.reward_kind = prm->reward_kind;
  EnvDev base = env_dev(e);
  if (!base.error) base.error = p->err;   // the word k_jobs_from_actions sets
  // (ABI v12) one colour group: every step rewrites recon whole, so nothing is ever restored from
  // the intensity cache -- no pending reconcile, no copies (hbx.h, recon_pending)
  if (to_recon && G == 1) base.recon_pending = nullptr;
  for (int b0 = 0; b0 < n_env; b0 += p->max_jobs) {
    const int n = std::min(p->max_jobs, n_env - b0);
    const EnvDev ed = env_offset(base, b0, CH, G, N);
    float* rec = to_recon ? e->recon + (size_t)b0 * G * hw : nullptr;
    if (planes) {
      pdx.plane_pool = e->plane_inten + (size_t)b0 * (CH + 2) * hw;
      pdx.plane_slot = e->plane_slot + (size_t)b0 * (CH + 2);
    }
    // the previous step's group: recon and intensity agree again before it is overwritten -- in
    // k_rowinv_d's epilogue at N = 1024 / 256 (no launch of its own), else k_recon_reconcile
    const bool fuse_rc = to_recon && ed.recon_pending && (pd.R == 32 || pd.R == 16);
    pdx.rc_pending = fuse_rc ? ed.recon_pending : nullptr;
    pdx.rc_cache = fuse_rc ? e->intensity + (size_t)b0 * G * hw : nullptr;
    // N = 1024 / 256: the finalize kernel sums the row-block partials itself (no k_reduce_partials)
    pdx.skip_reduce = (pd.R == 32 || pd.R == 16) ? 1 : 0;
    if (to_recon && ed.recon_pending && !fuse_rc)
      HBX_HIP(hbx::launch_recon_reconcile(ed.recon_pending, rec, e->intensity + (size_t)b0 * G * hw, n, G, hw, st));
    if (pdx.skip_reduce) {     // N = 1024 / 256: the first pass decodes the actions itself
      pdx.actions = actions + b0;
      pdx.act_err = e->error ? e->error : p->err;
    } else {
      HBX_HIP(hbx::launch_jobs_from_actions(actions + b0, n, N, N, P, CH, p->jobs, e->error ? e->error : p->err, st));
    }
    HBX_HIP(hbx::run_jobs(pdx, p->jobs, n, reinterpret_cast<const uint32_t*>(ed.mask), ed.target,
                          to_recon ? rec : (want_inten ? p->job_inten : nullptr), nullptr, st));
    HBX_HIP(hbx::launch_env_step_finalize(p->jobs, pd.job_stats, n, G, P, N, N, ed, ep, pixel_count(p),
                                          p->optics.rel_scale, p->optics.peak,
                                          reward ? reward + b0 : nullptr, psnr ? psnr + b0 : nullptr,
                                          accepted ? accepted + b0 : nullptr,
                                          terminated ? terminated + b0 : nullptr,
                                          truncated ? truncated + b0 : nullptr, p->accept_flag, p->delta,
                                          st, pdx.skip_reduce ? pd.partial : nullptr,
                                          pdx.skip_reduce ? pd.N / (256 / pd.R) : 0));
    if (group_intensity)
      HBX_HIP(hipMemcpyAsync(group_intensity + (size_t)b0 * hw, p->job_inten, (size_t)n * hw * sizeof(float),
                             hipMemcpyDeviceToDevice, st));
    if (e->intensity && !to_recon)
      HBX_HIP(hbx::launch_scatter_intensity(p->jobs, n, p->job_inten, e->intensity + (size_t)b0 * G * hw, G,
                                            hw, p->accept_flag, st));
  }
  return HBX_OK;
}

int hbx_step(hbx_plan_t p, uint64_t* mask, const int64_t* actions, int32_t n_env, const float* target,
             double* chan_stats, double* prev_psnr, double* psnr_out, uint8_t* accepted,
             int32_t accept_rule, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (accept_rule != HBX_ACCEPT_ENV && accept_rule != HBX_ACCEPT_DBS) return fail(HBX_ERR_INVALID, "accept_rule");
  if (n_env <= 0) return n_env == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "n_env");
  if (!mask || !actions || !target || !chan_stats || !prev_psnr) return fail(HBX_ERR_INVALID, "null buffer");
  HBX_HIP(hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  const PlanDev& pd = p->pd;
  const int N = pd.N, G = pd.G, P = pd.P, CH = G * P;
  for (int b0 = 0; b0 < n_env; b0 += p->max_jobs) {
    const int n = std::min(p->max_jobs, n_env - b0);
    uint64_t* m = mask + (size_t)b0 * CH * N * (N / 64);
    const float* tg = target + (size_t)b0 * G * N * N;
    HBX_HIP(hbx::launch_jobs_from_actions(actions + b0, n, N, N, P, CH, p->jobs, p->err, st));
    HBX_HIP(hbx::run_jobs(pd, p->jobs, n, reinterpret_cast<const uint32_t*>(m), tg, nullptr, nullptr, st));
    HBX_HIP(hbx::launch_dbs_step_finalize(p->jobs, pd.job_stats, n, G, P, N, N, m,
                                          chan_stats + (size_t)b0 * G * 3, prev_psnr + b0,
                                          psnr_out ? psnr_out + b0 : nullptr,
                                          accepted ? accepted + b0 : nullptr, accept_rule,
                                          pixel_count(p), p->optics.rel_scale, p->optics.peak, st));
  }
  return HBX_OK;
}

int hbx_eval_flips(hbx_plan_t p, const uint64_t* base_mask, const float* target,
                   const double* base_chan_stats, const int64_t* flips, int32_t K, double* psnr_out,
                   double* group_stats, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (K <= 0) return K == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "K");  // empty batch: null buffers allowed
  if (!base_mask || !target || !base_chan_stats || !flips || !psnr_out)
    return fail(HBX_ERR_INVALID, "null buffer");
  HBX_HIP(hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  const PlanDev& pd = p->pd;
  const int N = pd.N, G = pd.G, P = pd.P, CH = G * P;
  for (int k0 = 0; k0 < K; k0 += p->max_jobs) {
    const int n = std::min(p->max_jobs, K - k0);
    HBX_HIP(hbx::launch_jobs_from_flips(flips + k0, n, N, N, P, CH, p->jobs, st));
    HBX_HIP(hbx::run_jobs(pd, p->jobs, n, reinterpret_cast<const uint32_t*>(base_mask), target, nullptr,
                          nullptr, st));
    HBX_HIP(hbx::launch_eval_finalize(p->jobs, pd.job_stats, n, G, base_chan_stats, psnr_out + k0,
                                      group_stats ? group_stats + (size_t)k0 * 3 : nullptr,
                                      pixel_count(p), p->optics.rel_scale, p->optics.peak, st));
  }
  return HBX_OK;
}

namespace {
int ensure_map(hbx_plan_t p, hipStream_t st) {
  if (p->map_y) return HBX_OK;
  int rc = ensure_hpsf(p, st);
  if (rc) return rc;
  PlanDev& pd = p->pd;
  const size_t hw = (size_t)pd.N * pd.N;
  const int G = pd.G, P = pd.P, CH = G * P;
  const size_t nx = 4 * P + P / 2 + 1, ny = P + P / 2 + 1;
  const size_t ns = std::max(nx, (size_t)4 * G);
  if (hipMalloc(&p->map_field, CH * hw * sizeof(float2)) != hipSuccess ||
      hipMalloc(&p->map_inten, G * hw * sizeof(float)) != hipSuccess ||
      hipMalloc(&p->map_stats, (size_t)(3 * G + 1) * sizeof(double)) != hipSuccess ||
      hipMalloc(&p->map_q, (size_t)4 * G * hw * sizeof(float2)) != hipSuccess ||
      hipMalloc(&p->map_d4, (size_t)G * sizeof(double)) != hipSuccess ||
      hipMalloc(&p->map_part, (size_t)G * 64 * sizeof(double)) != hipSuccess ||
      hipMalloc(&p->map_x, std::max(nx, ny) * hw * sizeof(float2)) != hipSuccess ||
      hipMalloc(&p->map_s, ns * hw * sizeof(float2)) != hipSuccess ||
      hipMalloc(&p->map_y, ny * hw * sizeof(float2)) != hipSuccess) {
    for (void** q : {(void**)&p->map_field, (void**)&p->map_inten, (void**)&p->map_stats, (void**)&p->map_q,
                     (void**)&p->map_d4, (void**)&p->map_part, (void**)&p->map_x, (void**)&p->map_s,
                     (void**)&p->map_y})
      if (*q) { (void)hipFree(*q); *q = nullptr; }
    return fail(HBX_ERR_NOMEM, "flip-map workspace");
  }
  HBX_HIP(hbx::map_prepare_h(pd, p->map_q, p->map_s, p->map_part, p->map_d4, st));
  return HBX_OK;
}
}  // namespace

int hbx_flip_map(hbx_plan_t p, const uint64_t* mask, const float* target, float* dpsnr, double* base_psnr,
                 void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (!mask || !target || !dpsnr) return fail(HBX_ERR_INVALID, "flip map needs mask, target and dpsnr");
  if (p->pd.P % 2) return fail(HBX_ERR_INVALID, "flip map needs an even plane count");
  if (p->max_jobs < p->pd.G) return fail(HBX_ERR_INVALID, "flip map needs max_jobs >= groups");
  HBX_HIP(hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  rc = ensure_map(p, st);
  if (rc) return rc;
  const PlanDev& pd = p->pd;
  const int G = pd.G;
  double* stats = p->map_stats;
  rc = propagate_full(p, mask, target, nullptr, 1, p->map_inten, stats, stats + 3 * G, nullptr,
                      p->map_field, st);
  if (rc) return rc;
  for (int g = 0; g < G; ++g)
    HBX_HIP(hbx::map_group(pd, g, p->map_field, p->map_inten, target, mask, stats, p->map_q, p->map_d4,
                           p->map_x, p->map_s, p->map_y, dpsnr, pixel_count(p), p->optics.rel_scale,
                           p->optics.peak, st));
  if (base_psnr)
    HBX_HIP(hipMemcpyAsync(base_psnr, stats + 3 * G, sizeof(double), hipMemcpyDeviceToDevice, st));
  return HBX_OK;
}

int hbx_commit_flip(hbx_plan_t p, uint64_t* base_mask, double* base_chan_stats, double* prev_psnr,
                    const int64_t* flips, const double* psnr_out, const double* group_stats,
                    const int32_t* k, int32_t K, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (K <= 0) return K == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "K");
  if (!base_mask || !base_chan_stats || !prev_psnr || !flips || !psnr_out || !group_stats || !k)
    return fail(HBX_ERR_INVALID, "null buffer");
  HBX_HIP(hipSetDevice(p->device));
  const PlanDev& pd = p->pd;
  HBX_HIP(hbx::launch_commit_flip(base_mask, base_chan_stats, prev_psnr, flips, psnr_out, group_stats, k,
                                  K, pd.G, pd.P, pd.N, pd.N, (hipStream_t)stream));
  return HBX_OK;
}

int hbx_planes_fill(hbx_plan_t p, const uint64_t* mask, const float* target, float* plane_inten,
                    int32_t* plane_slot, int32_t n_spare_pairs, double* chan_stats, double* psnr, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (!mask || !target || !plane_inten || !plane_slot || !chan_stats)
    return fail(HBX_ERR_INVALID, "planes fill needs mask, target, plane_inten, plane_slot and chan_stats");
  if (n_spare_pairs < 1) return fail(HBX_ERR_INVALID, "n_spare_pairs >= 1");
  if (p->max_jobs < p->pd.G) return fail(HBX_ERR_INVALID, "planes fill needs max_jobs >= groups");
  HBX_HIP(hipSetDevice(p->device));
  return propagate_full(p, mask, target, nullptr, 1, nullptr, chan_stats, psnr, nullptr, nullptr,
                        (hipStream_t)stream, plane_inten, plane_slot, n_spare_pairs);
}

int hbx_eval_flips_planes(hbx_plan_t p, const uint64_t* base_mask, const float* target,
                          const double* base_chan_stats, float* plane_inten, const int32_t* plane_slot,
                          int32_t n_spare_pairs, const int64_t* flips, int32_t K, double* psnr_out,
                          double* group_stats, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (K <= 0) return K == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "K");
  if (!base_mask || !target || !base_chan_stats || !plane_inten || !plane_slot || !flips || !psnr_out)
    return fail(HBX_ERR_INVALID, "null buffer");
  if (p->pd.R != 32 && p->pd.R != 16 && p->pd.R != 0)
    return fail(HBX_ERR_UNSUPPORTED, "plane cache: N = 1024, 896 or 256 only");
  if (K > n_spare_pairs) return fail(HBX_ERR_INVALID, "K > n_spare_pairs: every candidate needs its own spare pair");
  HBX_HIP(hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  const PlanDev& pd = p->pd;
  const int N = pd.N, G = pd.G, P = pd.P, CH = G * P;
  PlanDev pdx = pd;
  pdx.plane_mode = hbx::kPlanesStep;
  pdx.plane_pool = plane_inten;
  pdx.plane_slot = plane_slot;
  pdx.plane_spares = n_spare_pairs;   // > 1: spare pair = candidate index (1: K = 1, pair 0)
  for (int k0 = 0; k0 < K; k0 += p->max_jobs) {
    const int n = std::min(p->max_jobs, K - k0);
    pdx.spare_base = k0;
    HBX_HIP(hbx::launch_jobs_from_flips(flips + k0, n, N, N, P, CH, p->jobs, st));
    HBX_HIP(hbx::run_jobs(pdx, p->jobs, n, reinterpret_cast<const uint32_t*>(base_mask), target, nullptr,
                          nullptr, st));
    HBX_HIP(hbx::launch_eval_finalize(p->jobs, pd.job_stats, n, G, base_chan_stats, psnr_out + k0,
                                      group_stats ? group_stats + (size_t)k0 * 3 : nullptr,
                                      pixel_count(p), p->optics.rel_scale, p->optics.peak, st));
  }
  return HBX_OK;
}

int hbx_commit_flip_planes(hbx_plan_t p, uint64_t* base_mask, double* base_chan_stats, double* prev_psnr,
                           int32_t* plane_slot, int32_t n_spare_pairs, const int64_t* flips,
                           const double* psnr_out, const double* group_stats, const int32_t* k, int32_t K,
                           void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (K <= 0) return K == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "K");
  if (!base_mask || !base_chan_stats || !prev_psnr || !plane_slot || !flips || !psnr_out || !group_stats || !k)
    return fail(HBX_ERR_INVALID, "null buffer");
  if (K > n_spare_pairs) return fail(HBX_ERR_INVALID, "K > n_spare_pairs");
  HBX_HIP(hipSetDevice(p->device));
  const PlanDev& pd = p->pd;
  HBX_HIP(hbx::launch_commit_flip(base_mask, base_chan_stats, prev_psnr, flips, psnr_out, group_stats, k,
                                  K, pd.G, pd.P, pd.N, pd.N, (hipStream_t)stream, plane_slot));
  return HBX_OK;
}

int hbx_dbs_walk_planes(hbx_plan_t p, uint64_t* base_mask, const float* target, double* base_chan_stats,
                        float* plane_inten, int32_t* plane_slot, int32_t n_spare_pairs, const int64_t* order,
                        int64_t n_order, hbx_dbs_walk_t* walk, int64_t* accept_pos, double* accept_psnr,
                        int64_t accept_cap, int32_t K, int32_t batches, void* stream) {
  return hbx_dbs_walk_planes_fill(p, base_mask, target, base_chan_stats, plane_inten, plane_slot, n_spare_pairs,
                                  order, n_order, walk, accept_pos, accept_psnr, accept_cap, K, batches, nullptr,
                                  0, 0, stream);
}

int hbx_dbs_walk_planes_fill(hbx_plan_t p, uint64_t* base_mask, const float* target, double* base_chan_stats,
                             float* plane_inten, int32_t* plane_slot, int32_t n_spare_pairs, const int64_t* order,
                             int64_t n_order, hbx_dbs_walk_t* walk, int64_t* accept_pos, double* accept_psnr,
                             int64_t accept_cap, int32_t K, int32_t batches, int64_t* fill_count,
                             int64_t fill_target, int64_t fill_tol, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (!base_mask || !target || !base_chan_stats || !plane_inten || !plane_slot || !order || !walk)
    return fail(HBX_ERR_INVALID, "null buffer");
  if (accept_cap < 0 || (accept_cap > 0 && (!accept_pos || !accept_psnr)))
    return fail(HBX_ERR_INVALID, "accept log");
  if (p->pd.R != 32 && p->pd.R != 16 && p->pd.R != 0)
    return fail(HBX_ERR_UNSUPPORTED, "plane cache: N = 1024, 896 or 256 only");
  if (K < 1 || K > 256 || K > p->max_jobs || K > n_spare_pairs)
    return fail(HBX_ERR_INVALID, "K must be in [1, min(256, max_jobs, n_spare_pairs)]");
  if (batches < 0 || n_order < 0) return fail(HBX_ERR_INVALID, "batches / n_order");
  if (fill_count && (fill_tol < 0 || fill_target < 0 ||
                     fill_target > (int64_t)p->pd.P * p->pd.N * p->pd.N))
    return fail(HBX_ERR_INVALID, "fill_target in [0, P*H*W] and fill_tol >= 0");
  HBX_HIP(hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  const PlanDev& pd = p->pd;
  PlanDev pdx = pd;
  pdx.plane_mode = hbx::kPlanesStep;
  pdx.plane_pool = plane_inten;
  pdx.plane_slot = plane_slot;
  pdx.plane_spares = n_spare_pairs;
  pdx.spare_base = 0;
  pdx.skip_reduce = 1;                     // the decision reduces the row-block partials itself
  const int RB = pd.R ? pd.N / (256 / pd.R) : pd.N / 8;
  hbx::WalkPlanesArgs wa;
  wa.w = walk; wa.order = order; wa.jobs = p->jobs; wa.partial = pd.partial; wa.mask = base_mask;
  wa.base_stats = base_chan_stats; wa.plane_slot = plane_slot; wa.accept_pos = accept_pos;
  wa.accept_psnr = accept_psnr; wa.accept_cap = accept_cap; wa.ticket = p->planes_ticket;
  wa.RB = RB; wa.K = K; wa.G = pd.G; wa.P = pd.P; wa.H = pd.N; wa.W = pd.N;
  wa.count = pixel_count(p); wa.rel_scale = p->optics.rel_scale; wa.peak = p->optics.peak;
  wa.fill_count = fill_count; wa.fill_target = fill_target; wa.fill_tol = fill_tol;
  // (r05) each batch's decision runs in the last-arriving k_rowinv_d workgroup of that batch
  // (k_rowinv_d<R, true>): three launches per batch instead of four.  (r06) N = 896: the decision
  // in a launch of its own behind each batch (k_walk_planes, decide = 1)
  const bool fused = pd.R != 0;
  pdx.walk_planes = fused ? &wa : nullptr;
  // (r06) candidates a batch propagated but did not visit keep their job slot, their pair's B and,
  // when their colour group saw no accept, their partials: the next batch skips those passes for
  // them (fused decision only; the 896 path decides in its own launch and re-propagates)
  // (the decision keeps the accepted (group, pair)s as bits < 48 of one word: G * P / 2 <= 48)
  if (fused && pd.G * pd.P / 2 <= 48 && !std::getenv("HBX_WALK_NO_RETAIN")) {
    wa.ring = p->walk_ring;
    wa.phase = p->walk_phase;
    pdx.walk_phase = p->walk_phase;
  }
  HBX_HIP(hbx::launch_walk_planes(wa, 0, st));   // this call's first batch of jobs, from the walk state
  for (int b = 0; b < batches; ++b) {
    HBX_HIP(hbx::run_jobs(pdx, p->jobs, K, reinterpret_cast<const uint32_t*>(base_mask), target, nullptr,
                          nullptr, st));
    if (!fused) HBX_HIP(hbx::launch_walk_planes(wa, 1, st));
  }
  return HBX_OK;
}

int hbx_eval_flips_psf(hbx_plan_t p, const uint64_t* base_mask, const float* target,
                       const double* base_chan_stats, const float* field, const float* intensity,
                       const int64_t* flips, int32_t K, double* psnr_out, double* group_stats,
                       void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (K <= 0) return K == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "K");
  if (!base_mask || !target || !base_chan_stats || !field || !intensity || !flips || !psnr_out)
    return fail(HBX_ERR_INVALID, "null buffer");
  HBX_HIP(hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  rc = ensure_hpsf(p, st);
  if (rc) return rc;
  const PlanDev& pd = p->pd;
  const int N = pd.N, G = pd.G, P = pd.P, CH = G * P;
  for (int k0 = 0; k0 < K; k0 += p->max_jobs) {
    const int n = std::min(p->max_jobs, K - k0);
    HBX_HIP(hbx::launch_jobs_from_flips(flips + k0, n, N, N, P, CH, p->jobs, st));
    HBX_HIP(hbx::launch_psf_eval(pd, p->jobs, n, base_mask, reinterpret_cast<const float2*>(field), intensity,
                                 target, base_chan_stats, st));
    HBX_HIP(hbx::launch_eval_finalize(p->jobs, pd.job_stats, n, G, base_chan_stats, psnr_out + k0,
                                      group_stats ? group_stats + (size_t)k0 * 3 : nullptr,
                                      pixel_count(p), p->optics.rel_scale, p->optics.peak, st));
  }
  return HBX_OK;
}

int hbx_commit_flip_psf(hbx_plan_t p, uint64_t* base_mask, double* base_chan_stats, double* prev_psnr,
                        float* field, float* intensity, const int64_t* flips, const double* psnr_out,
                        const double* group_stats, const int32_t* k, int32_t K, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (K <= 0) return K == 0 ? HBX_OK : fail(HBX_ERR_INVALID, "K");
  if (!base_mask || !base_chan_stats || !prev_psnr || !field || !intensity || !flips || !psnr_out ||
      !group_stats || !k)
    return fail(HBX_ERR_INVALID, "null buffer");
  HBX_HIP(hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  rc = ensure_hpsf(p, st);
  if (rc) return rc;
  const PlanDev& pd = p->pd;
  const int N = pd.N, G = pd.G, P = pd.P, CH = G * P;
  // toggle the mask bit first: the field update's delta is read from the new bit
  HBX_HIP(hbx::launch_commit_flip(base_mask, base_chan_stats, prev_psnr, flips, psnr_out, group_stats, k,
                                  K, G, P, N, N, st));
  HBX_HIP(hbx::launch_job_from_flip_k(flips, k, K, N, N, P, CH, p->jobs, pd.psf_order, p->accept_flag, st));
  // psf_order is already {0}: launch_psf_commit visits the single job
  HBX_HIP(hbx::launch_psf_commit(pd, p->jobs, 1, base_mask, reinterpret_cast<float2*>(field), intensity,
                                 p->accept_flag, st));
  return HBX_OK;
}

int hbx_dbs_walk_psf(hbx_plan_t p, uint64_t* base_mask, const float* target, double* base_chan_stats,
                     float* field, float* intensity, const int64_t* order, int64_t n_order,
                     hbx_dbs_walk_t* walk,
                     int64_t* accept_pos, double* accept_psnr, int64_t accept_cap, int32_t K,
                     int32_t batches, void* stream) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (!base_mask || !target || !base_chan_stats || !field || !intensity || !order || !walk)
    return fail(HBX_ERR_INVALID, "null buffer");
  if (accept_cap < 0 || (accept_cap > 0 && (!accept_pos || !accept_psnr)))
    return fail(HBX_ERR_INVALID, "accept log");
  if (K < 1 || K > hbx::kWalkMaxK) return fail(HBX_ERR_INVALID, "K must be in [1, 256]");
  if (batches < 0) return fail(HBX_ERR_INVALID, "batches");
  if (n_order < 0) return fail(HBX_ERR_INVALID, "n_order");
  HBX_HIP(hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  rc = ensure_hpsf(p, st);
  if (rc) return rc;
  const PlanDev& pd = p->pd;
  // sized once for every K, so the buffer never moves: launches captured into a
  // graph (one per K) stay valid
  size_t need = (size_t)hbx::walk_step_blocks(pd.N) * hbx::kWalkStepMaxTerms;
  for (int k = 1; k <= hbx::kWalkMaxK; ++k)
    need = std::max(need, (size_t)k * hbx::walk_blocks_per_job(pd.N, k) * 2);
  if (!p->walk_counter) {   // allocation: first call only, outside capture
    if (hipMalloc(&p->walk_counter, hbx::kWalkScratchBytes) != hipSuccess) return fail(HBX_ERR_NOMEM, "walk scratch");
    if (hipMemset(p->walk_counter, 0, hbx::kWalkScratchBytes) != hipSuccess) return fail(HBX_ERR_HIP, "walk scratch");
  }
  if (need > p->walk_partial_elems) {   // allocation: first call only, outside capture
    if (p->walk_partial) (void)hipFree(p->walk_partial);
    p->walk_partial = nullptr;
    p->walk_partial_elems = 0;
    if (hipMalloc(&p->walk_partial, need * sizeof(double)) != hipSuccess)
      return fail(HBX_ERR_NOMEM, "walk partials");
    p->walk_partial_elems = need;
  }
  hbx::WalkLaunch l;
  l.mask = base_mask;
  l.target = target;
  l.base_stats = base_chan_stats;
  l.field = reinterpret_cast<float2*>(field);
  l.inten = intensity;
  l.order = order;
  l.n_order = n_order;
  l.walk = walk;
  l.log_pos = accept_pos;
  l.log_psnr = accept_psnr;
  l.log_cap = accept_cap;
  l.partial = p->walk_partial;
  l.counter = p->walk_counter;
  l.fused = p->walk_split ? 0 : 1;
  l.persist = p->walk_persist;
  l.K = K;
  l.batches = batches;
  l.count = pixel_count(p);
  l.peak = p->optics.peak;
  l.rel = p->optics.rel_scale;
  // the decoded next actions a previous launch left are keyed on (position, order
  // pointer); a new call may bring new order contents at the same address: invalidate
  HBX_HIP(hipMemsetAsync(p->walk_counter + hbx::kWalkCounters, 0xff, sizeof(int64_t), st));
  HBX_HIP(hipMemsetAsync(p->walk_counter + hbx::kWalkAbort, 0, sizeof(int), st));   // persistent walk
  HBX_HIP(hbx::launch_walk(pd, l, st));
  return HBX_OK;
}

}  // extern "C"

extern "C" {

int hbx_plan_set_timing(hbx_plan_t p, int32_t capacity) { return hbx_plan_set_timing_sampled(p, capacity, 1); }

int hbx_plan_set_timing_sampled(hbx_plan_t p, int32_t capacity, int32_t every) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (capacity < 0) return fail(HBX_ERR_INVALID, "capacity");
  if (every < 1) return fail(HBX_ERR_INVALID, "every");
  (void)hipSetDevice(p->device);
  hbx::PassTimer* tm = p->pd.timer;
  if (tm) {
    for (int k = 0; k < hbx::kNumPasses; ++k) {
      for (int i = 0; i < 2 * tm->capacity; ++i) (void)hipEventDestroy(tm->ev[k][i]);
      delete[] tm->ev[k];
    }
    delete tm;
    p->pd.timer = nullptr;
  }
  if (capacity == 0) return HBX_OK;
  tm = new (std::nothrow) hbx::PassTimer();
  if (!tm) return fail(HBX_ERR_NOMEM, "timer");
  // on any failure below, destroy exactly the events created so far
  auto undo = [tm](int passes_done, int events_in_pass) {
    for (int k = 0; k <= passes_done && k < hbx::kNumPasses; ++k) {
      if (!tm->ev[k]) continue;
      const int n = k < passes_done ? 2 * tm->capacity : events_in_pass;
      for (int i = 0; i < n; ++i) (void)hipEventDestroy(tm->ev[k][i]);
      delete[] tm->ev[k];
    }
    delete tm;
  };
  tm->capacity = capacity;
  tm->every = every;
  for (int k = 0; k < hbx::kNumPasses; ++k) {
    tm->ev[k] = new (std::nothrow) hipEvent_t[2 * (size_t)capacity];
    if (!tm->ev[k]) {
      undo(k, 0);
      return fail(HBX_ERR_NOMEM, "timer events");
    }
    for (int i = 0; i < 2 * capacity; ++i) {
      const hipError_t e = hipEventCreate(&tm->ev[k][i]);
      if (e != hipSuccess) {
        undo(k, i);
        return fail(HBX_ERR_HIP, std::string("hipEventCreate: ") + hipGetErrorString(e));
      }
    }
  }
  p->pd.timer = tm;
  return HBX_OK;
}

int hbx_plan_read_timing(hbx_plan_t p, double* ms_total, int64_t* launches, int64_t* jobs) {
  int rc = check_plan(p);
  if (rc) return rc;
  if (!ms_total || !launches) return fail(HBX_ERR_INVALID, "null output");
  hbx::PassTimer* tm = p->pd.timer;
  for (int k = 0; k < hbx::kNumPasses; ++k) {
    ms_total[k] = 0.0;
    launches[k] = 0;
    if (jobs) jobs[k] = 0;
  }
  if (!tm) return fail(HBX_ERR_INVALID, "timing not enabled");
  (void)hipSetDevice(p->device);
  for (int k = 0; k < hbx::kNumPasses; ++k) {
    double tot = 0.0;
    for (int i = 0; i < tm->count[k]; ++i) {
      HBX_HIP(hipEventSynchronize(tm->ev[k][2 * i + 1]));
      float ms = 0.0f;
      HBX_HIP(hipEventElapsedTime(&ms, tm->ev[k][2 * i], tm->ev[k][2 * i + 1]));
      tot += ms;
    }
    ms_total[k] = tot;
    launches[k] = tm->count[k];
    if (jobs) jobs[k] = tm->jobs[k];
    tm->count[k] = 0;
    tm->calls[k] = 0;
    tm->jobs[k] = 0;
  }
  return HBX_OK;
}

int hbx_pack_mask(const void* src, int32_t src_kind, int64_t n_values, int32_t mode, double threshold,
                  uint64_t* bits, int32_t* error, void* stream) {
  if (n_values < 0 || n_values % 64) return fail(HBX_ERR_INVALID, "hbx_pack_mask: n_values must be a multiple of 64");
  if (n_values == 0) return HBX_OK;
  if (!src || !bits) return fail(HBX_ERR_INVALID, "hbx_pack_mask: null buffer");
  if (mode != HBX_PACK_BINARY && mode != HBX_PACK_THRESHOLD)
    return fail(HBX_ERR_INVALID, "hbx_pack_mask: mode must be HBX_PACK_BINARY or HBX_PACK_THRESHOLD");
  const uintptr_t align = src_kind == HBX_SRC_U8 ? 4 : src_kind == HBX_SRC_F32 ? 16 : src_kind == HBX_SRC_F64 ? 32 : 0;
  if (!align) return fail(HBX_ERR_INVALID, "hbx_pack_mask: src_kind must be HBX_SRC_U8, _F32 or _F64");
  if ((uintptr_t)src % align) return fail(HBX_ERR_INVALID, "hbx_pack_mask: src is not aligned to its vector load");
  if ((uintptr_t)bits % 8) return fail(HBX_ERR_INVALID, "hbx_pack_mask: bits is not 8-byte aligned");
  HBX_HIP(hbx::launch_pack_mask(src, src_kind, n_values / 64, mode, threshold, bits, error, (hipStream_t)stream));
  return HBX_OK;
}

int hbx_rel_stats(const void* x, const void* y, int32_t src_kind, int64_t n, int32_t rel_scale, double peak,
                  double* workspace, double* out, void* stream) {
  static_assert(HBX_REL_WORKSPACE_DOUBLES >= 3 * 1024, "workspace holds 3 doubles per partial slot");
  if (n <= 0) return fail(HBX_ERR_INVALID, "hbx_rel_stats: n must be > 0");
  if (!x || !y || !workspace || !out) return fail(HBX_ERR_INVALID, "hbx_rel_stats: null buffer");
  if (src_kind != HBX_SRC_F32 && src_kind != HBX_SRC_F64)
    return fail(HBX_ERR_INVALID, "hbx_rel_stats: src_kind must be HBX_SRC_F32 or HBX_SRC_F64");
  if (rel_scale != HBX_REL_NONE && rel_scale != HBX_REL_LSQ) return fail(HBX_ERR_INVALID, "hbx_rel_stats: rel_scale");
  if (3 * hbx::rel_partial_slots() > HBX_REL_WORKSPACE_DOUBLES) return fail(HBX_ERR_INVALID, "workspace size");
  HBX_HIP(hbx::launch_rel_stats(x, y, src_kind, n, (double)n, rel_scale, peak, workspace, out, (hipStream_t)stream));
  return HBX_OK;
}

}  // extern "C"
