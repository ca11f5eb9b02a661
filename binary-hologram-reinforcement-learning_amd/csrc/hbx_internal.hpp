// hbx_internal.hpp -- types shared by the kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include "hbx.h"

namespace hbx {

// tt.relativeLoss(.., tm.get_PSNR) from the channel sums (env.py:174):
// lsq scale s = sum IT / sum I^2, mse = mean((s I - T)^2), psnr = 10 log10(peak^2 / mse)
__device__ __forceinline__ double psnr_from(double sxy, double sxx, double syy, double count,
                                            int rel_scale, double peak) {
  double mse;
  if (rel_scale == 1) mse = (sxx > 0.0) ? (syy - sxy * sxy / sxx) / count : syy / count;
  else mse = (sxx - 2.0 * sxy + syy) / count;
  if (!(mse > 0.0)) return INFINITY;
  return 10.0 * log10(peak * peak / mse);
}

// Increment of one pixel's plane-mean intensity when a flip adds delta * h to
// its field u: (|u + delta h|^2 - |u|^2) / P = delta (2 Re(u conj h) + delta |h|^2) / P,
// formed without the two squares, so its f32 error is relative to the
// increment itself (differencing the squares loses it to the rounding of |u|^2
// wherever |h| << |u|, i.e. almost everywhere: ~1e-10 dB of noise per 1024x24
// candidate).  Incremental-field kernels (hbx_psf.hip, hbx_walk.hip).
__device__ __forceinline__ float flip_dI(float ur, float ui, float hr, float hi, float delta, float invp) {
  const float re = fmaf(ur, hr, ui * hi);
  const float hh = fmaf(hr, hr, hi * hi);
  return delta * fmaf(delta, hh, 2.0f * re) * invp;
}

// One colour-group propagation: env index (plan-local), group, optional flip.
struct JobDesc {
  int32_t env;         // < 0: invalid job (skipped, outputs neutral)
  int32_t group;
  int32_t flip_plane;  // plane within the group, -1 = no flip
  int32_t flip_pix;    // row * W + col
};

// env.py:157-161: action -> (channel, pixel) of env b; an action outside [0, CH*hw) is an
// invalid job (env -1).  Shared by k_jobs_from_actions and the first pass's fused decode.
__host__ __device__ __forceinline__ JobDesc job_of_action(int64_t a, int b, int64_t hw, int P, int CH) {
  JobDesc jd;
  if (a < 0 || a >= (int64_t)CH * hw) {
    jd.env = -1; jd.group = 0; jd.flip_plane = -1; jd.flip_pix = 0;
  } else {
    const int ch = (int)(a / hw);
    jd.env = b;
    jd.group = ch / P;
    jd.flip_plane = ch % P;
    jd.flip_pix = (int)(a % hw);
  }
  return jd;
}

// Intermediate layout of the fused N = R^2 path (hbx_passes.hip).  The row
// passes run blocks of row_nt(R) = 256 threads = panel_rows(R) rows; a plane of
// L lines is stored as N / PAN panels [L][PAN], panel q at q * PAN * L.  A is
// kept in panels of the row block height (8 rows at N = 1024: every k_rowfwd
// store is contiguous -- 0.69 ms for the 128-job A vs 1.19 ms as 64-B pieces of
// line-major A, tools/membw2.hip -- and k_col2's line reads cost nothing), B in
// panels of 16 rows (k_col2 writes 128-B pieces; 8-row B panels made its
// stores cost 1 ms more, 32 / 64 rows or a pad between panels were slower too:
// DESIGN.md 4).
constexpr int kPanelA = 8;
constexpr int kPanelB = 16;
__host__ __device__ constexpr int row_nt(int R) { return 256; }
__host__ __device__ constexpr int panel_rows(int R) { return row_nt(R) / R; }
__host__ __device__ constexpr int pan_of(int R, int rows) {
  return rows <= 0 || rows >= R * R ? R * R : (rows < panel_rows(R) ? panel_rows(R) : rows);
}
__host__ __device__ constexpr int pan_a(int R) { return pan_of(R, kPanelA); }
__host__ __device__ constexpr int pan_b(int R) { return pan_of(R, kPanelB); }
__host__ __device__ constexpr int panel_stride(int R, int L, int PAN) { return L * PAN; }
// float2 elements per intermediate plane: A (half spectrum, N/2 lines), B (N lines)
__host__ __device__ constexpr size_t plane_a_elems(int R) {
  return (size_t)(R * R / pan_a(R)) * panel_stride(R, R * R / 2, pan_a(R));
}
__host__ __device__ constexpr size_t plane_b_elems(int R) {
  return (size_t)(R * R / pan_b(R)) * panel_stride(R, R * R, pan_b(R));
}

// Line kx of a panel-layout plane as addressed by lane t of an R-lane group:
// element y = t + R jj sits at byte offset voff(t, kx) + joff(jj) from the
// plane base (joff is a compile-time constant per jj: an SGPR or immediate
// offset of a buffer instruction, so one address VGPR serves the whole line).
template <int R, int L, int PAN>
struct PanelLine {
  static constexpr int PS = panel_stride(R, L, PAN);
  // element (line, y) of the plane
  __device__ __forceinline__ static constexpr size_t at(int line, int y) {
    return (size_t)(y / PAN) * PS + (size_t)line * PAN + y % PAN;
  }
  __device__ __forceinline__ static int voff(int t, int kx) {
    if constexpr (R > PAN) return ((t / PAN) * PS + kx * PAN + t % PAN) * 8;
    else return (kx * PAN + t) * 8;
  }
  __device__ __forceinline__ static constexpr int joff(int jj) {
    if constexpr (R > PAN) return jj * (R / PAN) * PS * 8;
    else return (((R * jj) / PAN) * PS + (R * jj) % PAN) * 8;
  }
};

// Optional hipEvent pairs around every `every`-th pass launch (hbx_plan_set_timing*).
constexpr int kNumPasses = 5;  // rowfwd, col, rowinv, psf_eval, psf_commit
struct PassTimer {
  int capacity = 0;
  int every = 1;
  int count[kNumPasses] = {};
  int64_t calls[kNumPasses] = {};   // launches seen (recorded or not)
  bool open[kNumPasses] = {};       // begin() recorded, end() pending
  int64_t jobs[kNumPasses] = {};
  hipEvent_t* ev[kNumPasses] = {};  // [2 * capacity] start/stop
  __host__ void begin(int pass, hipStream_t st) {
    open[pass] = capacity && count[pass] < capacity && calls[pass] % every == 0;
    if (open[pass]) (void)hipEventRecord(ev[pass][2 * count[pass]], st);
  }
  __host__ void end(int pass, int n_jobs, hipStream_t st) {
    ++calls[pass];
    if (open[pass]) {
      (void)hipEventRecord(ev[pass][2 * count[pass] + 1], st);
      ++count[pass];
      jobs[pass] += n_jobs;
      open[pass] = false;
    }
  }
};

// the FFT-mode plane-cache walk's decision (hbx_walk_planes.hpp): everything it reads and writes
struct WalkPlanesArgs {
  hbx_dbs_walk_t* w;
  const int64_t* order;
  JobDesc* jobs;
  const double* partial;     // [K][RB][3] row-block partials of the batch just propagated
  uint64_t* mask;
  double* base_stats;
  int32_t* plane_slot;
  int64_t* accept_pos;
  double* accept_psnr;
  int64_t accept_cap;
  int32_t* ticket;           // fused decision: arrival counter of the k_rowinv_d workgroups
  int RB, K, G, P, H, W;
  double count;
  int rel_scale;
  double peak;
  // (ABI v13, extension) on-pixel ratio constraint: per-group on-pixel counts (nullptr = off),
  // the target count and the tolerance (hbx_dbs_walk_planes_fill)
  int64_t* fill_count = nullptr;
  int64_t fill_target = 0;
  int64_t fill_tol = 0;
  // (r06) candidate retention across batches (fused decision only; nullptr = off): the batch's
  // candidate i sits in job slot (*ring + i) % K, and phase[slot] tells the passes what a slot
  // still needs -- 0 everything, 1 only k_rowinv_d (its pair's B is still valid), 2 nothing (its
  // partials and fresh pair are still valid).  Slots are kept by the candidates a batch propagated
  // but did not visit (hbx_walk_planes.hpp)
  int32_t* ring = nullptr;
  uint8_t* phase = nullptr;
};

struct PlanDev {
  int R;               // N = R * R; 0: N = 896 = 28 x 32 (generic path)
  int N, G, P;
  float va, vb;        // field = va + vb * bit
  float2* tw;          // [N]  W_N^{t k1} at [k1 * R + t]; N = 1024 appends the
                       // whole-wave tables [16][64] W1024^{L k1}, [16][4] W64^{l0 m1}
  float2* htab;        // [G][N/2 + 1][N]  H(kx, ky) / (2 N^2): the row passes write 2 A
  float2* ws_a;        // [max_jobs][P][N/2][N]  half spectrum after k_rowfwd (line kx, over y)
  float2* ws_b;        // [max_jobs][P][N][N]    after k_col (line kx, over y)
  double* partial;     // [max_jobs][N / (256/R)][3]
  double* job_stats;   // [max_jobs][3]
  float2* hpsf;        // [G][N][N] single-pixel field h_g = IFFT2(H_g) (lazy, incremental mode)
  double* psf_partial; // [max_jobs][kPsfBlocks][2]
  int32_t* psf_order;  // [max_jobs] jobs sorted by colour group (launch order)
  float* zero_row;     // [N] zeros: the target row of a propagation without a target
  int store_kind;      // HBX_PRECISION_*: rounding of the pass intermediates (0 = f32, the product)
  int inten_by_env;    // intensity output rows: 0 = job-major [job][N][N]; 1 = env-major
                       // [env][G][N][N] at (job.env, job.group) (the obs recon buffer, ABI v8)
  PassTimer* timer;    // nullable
  // plane-cached FFT mode (ABI v9; N = 1024 / 256), set per call on a copy of the plan's PlanDev:
  //   kPlanesOff    no plane cache
  //   kPlanesFill   full propagation: every plane's |U_p|^2 also goes to its pool slot
  //   kPlanesStep   env step: only the flipped plane's pair is propagated, the other planes'
  //                 |U_q|^2 come from the pool (k_rowinv_d sums them in the same plane order,
  //                 so the group intensity is the FFT mode's bit for bit); the pair's fresh
  //                 |U|^2 go to the env's two spare slots (swapped in on accept)
  int plane_mode;
  float* plane_pool;         // [env][CH + 2S][N][N] f32 per-plane |U|^2 (env ids as the jobs carry them)
  const int32_t* plane_slot; // [env][CH + 2S] pool slot of every plane; [CH + 2s], [CH + 2s + 1] = spare pair s
  int plane_spares;          // S: spare pairs per env (0 / 1: the env step's one pair).  S > 1 (ABI v10,
                             // hbx_eval_flips_planes): candidate j of a launch writes its pair to spare
  int spare_base;            // pair spare_base + j, so K candidates of one base keep K fresh pairs
  // (r04) env step with the recon observation at N = 1024 / 256: k_rowinv_d applies the previous
  // step's recon / intensity-cache reconcile (recon_pending, env-major like inten_out) itself
  const int32_t* rc_pending; // [env] nullable
  float* rc_cache;           // [env][G][N][N] the intensity cache
  int skip_reduce = 0;       // 1: leave the per-row-block partials (a caller reduces them itself)
  const uint8_t* walk_phase = nullptr;           // (r06) per job slot: 0 all passes, 1 k_rowinv_d only,
                                                 // 2 none (WalkPlanesArgs::phase; nullptr = all)
  const WalkPlanesArgs* walk_planes = nullptr;   // (r05) plane-cache walk batch: the last k_rowinv_d
                                                 // workgroup decides (hbx_walk_planes.hpp)
  // env step at N = 1024 / 256: the first pass decodes the actions itself (no k_jobs_from_actions
  // launch) and one of its workgroups per job writes the JobDesc the later passes read
  const int64_t* actions = nullptr;
  int32_t* act_err = nullptr;
};
constexpr int kPlanesOff = 0, kPlanesFill = 1, kPlanesStep = 2;

constexpr int kPsfBlocks = 128;   // blocks per job of the incremental-field kernels
                                  // (measured 128 > 256 > 64 > 32, profiles/r01_psf_blocks_ab.txt)

struct EnvDev {
  uint64_t* mask;
  int8_t* record;
  const float* target;
  double* chan_stats;
  double* init_psnr;
  double* prev_psnr;
  double* max_psnr_diff;
  int64_t* steps;
  int64_t* flip_count;
  int64_t* sustained;
  const double* imp_changes;  // [B][imp_count] (importance rewards)
  const double* imp_values;
  const double* t_psnr_diff;  // [B] nullable
  int imp_count;
  int8_t* state_bytes;        // [B][CH][H][W] obs["state"] mirror of the mask bits (nullable, ABI v8)
  int32_t* recon_pending;     // [B] group the next step reconciles (nullable; with recon)
  int32_t* plane_slot;        // [B][CH + 2] plane-cache slots (nullable, ABI v9): an accepted step
                              // swaps the flipped pair's slots with the two spares
  const int32_t* error;       // the sticky error word (nullable)
  int32_t* error_host;        // its mirror, written by the env-step finalize (nullable, ABI v11)
};

struct EnvParams {
  int64_t max_steps;
  double t_psnr;
  int64_t t_steps;
  double t_psnr_diff;
  double reward_weight;
  int32_t accept_rule;
  int32_t reward_kind;  // 0 env.py, 1 env_group.py
};

// field_out (nullable): [env][G*P][N][N] complex field of every propagated plane
hipError_t run_jobs(const PlanDev& pd, const JobDesc* jobs, int n_jobs, const uint32_t* mask,
                    const float* target, float* inten_out, float2* field_out, hipStream_t st);
// fused three-pass propagation at N = 896 (hbx_passes896.hip)
hipError_t run_jobs_896(const PlanDev& pd, const JobDesc* jobs, int n_jobs, const uint32_t* mask,
                        const float* target, float* inten_out, float2* field_out, hipStream_t st);
// 2-D FFT of n_planes [N][N] complex planes in a (result in a; b is scratch of
// the same size).  Unnormalised both ways.
hipError_t run_fft2d(const PlanDev& pd, float2* a, float2* b, int n_planes, bool inverse,
                     hipStream_t st);
// flip map (hbx_map.hip): h-side spectra q [G][4][N][N] + sum |h|^4 per group,
// then one group's dPSNR map [P][N][N] into out + g*P*N*N
hipError_t map_prepare_h(const PlanDev& pd, float2* q, float2* scratch, double* part, double* d4,
                         hipStream_t st);
hipError_t map_group(const PlanDev& pd, int g, const float2* field, const float* inten,
                     const float* target, const uint64_t* mask, const double* stats, const float2* q,
                     const double* d4, float2* X, float2* S, float2* Y, float* out, double count, int rel,
                     double peak, hipStream_t st);
hipError_t launch_psf_eval(const PlanDev& pd, const JobDesc* jobs, int n_jobs, const uint64_t* mask,
                           const float2* field, const float* inten, const float* target,
                           const double* chan_stats, hipStream_t st, const int64_t* actions = nullptr,
                           int32_t* err = nullptr);
// device-resident greedy DBS walk (hbx_walk.hip)
struct WalkLaunch {
  uint64_t* mask;
  const float* target;
  double* base_stats;
  float2* field;
  float* inten;
  const int64_t* order;
  int64_t n_order;   // length of order: the walk never visits past min(walk->total, n_order)
  hbx_dbs_walk_t* walk;
  int64_t* log_pos;
  double* log_psnr;
  int64_t log_cap;
  double* partial;   // split batch: [K][walk_blocks_per_job(N, K)][2]; fused step: [blocks][terms]
  int* counter;      // fused step: walk scratch (kWalkScratchBytes): tickets, then WalkPre
  int fused;         // 1: one k_walk_step launch per batch when K has a fused variant
  int persist;       // 1 (with fused): one cooperative launch runs all `batches` (grid barrier per batch)
  int K, batches;
  double count, peak;
  int rel;
};
constexpr int kWalkMaxK = 256;
int walk_blocks_per_job(int N, int K);
int walk_step_blocks(int N);
bool walk_fused_k(int K);
constexpr int kWalkStepMaxTerms = 26;   // 2 K + 3 K (K-1) / 2 at K = 4: max over the fused variants
// fused-step scratch: int counters [kWalkCounters] (arrival tickets [0, kWalkTickets),
// zero between launches), then the WalkPre the deciding block leaves for the next launch
constexpr int kWalkCounters = 16;
constexpr int kWalkTickets = 9;
constexpr int kWalkGen = 12;             // persistent walk: generation word (bumped per decided batch)
constexpr int kWalkAbort = 13;           //   and the abort word (a grid barrier timed out)
constexpr unsigned kWalkSpinMax = 1u << 20;   // polls (each ~1-2 us) before a waiting block gives up
constexpr int kWalkPreMax = 4;          // the largest fused K
struct WalkPre {
  int64_t pos;              // valid for this walk position (-1: invalid; cleared per API call)
  const int64_t* order;     //   and this order array
  int32_t n;                // actions filled
  int32_t pad;
  int32_t ch[kWalkPreMax];   // order[pos + j] decoded: channel (-1: not a valid action) ...
  int32_t pix[kWalkPreMax];  //   ... and pixel
  float delta[kWalkPreMax];  // vb (1 - 2 bit) of each action's pixel before its flip
  float cdelta[2];           // the pending commits' vb (2 bit - 1) after their flips
};
constexpr size_t kWalkScratchBytes = kWalkCounters * sizeof(int) + sizeof(WalkPre);
hipError_t launch_walk(const PlanDev& pd, const WalkLaunch& l, hipStream_t st);
hipError_t launch_psf_commit(const PlanDev& pd, const JobDesc* jobs, int n_jobs, const uint64_t* mask,
                             float2* field, float* inten, const int32_t* accept_flag, hipStream_t st);
hipError_t launch_jobs_from_actions(const int64_t* actions, int n, int H, int W, int P, int CH,
                                    JobDesc* jobs, int32_t* err, hipStream_t st);
hipError_t launch_jobs_from_flips(const int64_t* flips, int K, int H, int W, int P, int CH,
                                  JobDesc* jobs, hipStream_t st);
hipError_t launch_job_from_flip_k(const int64_t* flips, const int32_t* k, int K, int H, int W, int P, int CH,
                                  JobDesc* jobs, int32_t* order, int32_t* accept, hipStream_t st);
hipError_t launch_jobs_full(const int32_t* env_ids, int n_ids, int G, JobDesc* jobs, hipStream_t st);
hipError_t launch_full_finalize(const JobDesc* jobs, const double* job_stats, int n_ids, int G,
                                double* chan_stats, double* psnr, double count, int rel, double peak,
                                const EnvDev& env, int reset, hipStream_t st);
hipError_t launch_env_step_finalize(const JobDesc* jobs, const double* job_stats, int n, int G,
                                    int P, int H, int W, const EnvDev& env, const EnvParams& prm,
                                    double count, int rel, double peak, double* reward, double* psnr,
                                    uint8_t* acc, uint8_t* term, uint8_t* trunc, int32_t* accept_flag,
                                    double* delta_scratch, hipStream_t st,
                                    const double* partial = nullptr, int RB = 0);
hipError_t launch_dbs_step_finalize(const JobDesc* jobs, const double* job_stats, int n, int G, int P,
                                    int H, int W, uint64_t* mask, double* chan_stats, double* prev,
                                    double* psnr, uint8_t* acc, int rule, double count, int rel,
                                    double peak, hipStream_t st);
hipError_t launch_eval_finalize(const JobDesc* jobs, const double* job_stats, int K, int G,
                                const double* base_stats, double* psnr, double* gstats, double count,
                                int rel, double peak, hipStream_t st);
hipError_t launch_commit_flip(uint64_t* mask, double* stats, double* prev, const int64_t* flips,
                              const double* psnr, const double* gstats, const int32_t* k, int K,
                              int G, int P, int H, int W, hipStream_t st, int32_t* plane_slot = nullptr);
hipError_t launch_zero_record(int8_t* record, const int32_t* env_ids, int n_ids, size_t per_env,
                              hipStream_t st);
hipError_t launch_scatter_intensity(const JobDesc* jobs, int n_jobs, const float* src, float* cache,
                                    int G, size_t hw, const int32_t* accept_flag, hipStream_t st);
hipError_t launch_psnr(const double* chan_stats, int n, int G, double* psnr, double count, int rel,
                       double peak, hipStream_t st);
// observation mirrors (ABI v8): reconcile the previous step's group between recon and
// intensity (recon_pending), and rebuild state_bytes / recon of listed envs
hipError_t launch_recon_reconcile(const int32_t* pending, float* recon, float* intensity, int n, int G,
                                  size_t hw, hipStream_t st);
// plane cache (ABI v9): slot[env][i] = i for the listed envs (env_ids nullable: 0 .. n_ids - 1)
hipError_t launch_walk_planes(const WalkPlanesArgs& a, int decide, hipStream_t st);
hipError_t launch_plane_slot_init(const int32_t* env_ids, int n_ids, int32_t* slot, int CHS, hipStream_t st);
hipError_t launch_obs_sync(const int32_t* env_ids, int n_ids, const uint64_t* mask, int8_t* state_bytes,
                           float* intensity, float* recon, int32_t* pending, int resolve, int CH, int G, size_t hw,
                           hipStream_t st);
hipError_t launch_obs_settle(const int32_t* env_ids, int n_ids, float* intensity, const float* recon,
                             int32_t* pending, int G, size_t hw, hipStream_t st);
// (ABI v14) hbx_pack.hip: mask values -> bits, and relativeLoss statistics
hipError_t launch_pack_mask(const void* src, int kind, int64_t n_words, int mode, double thr, uint64_t* bits,
                            int32_t* err, hipStream_t st);
int rel_partial_slots();
hipError_t launch_rel_stats(const void* x, const void* y, int kind, int64_t n, double count, int rel_scale,
                            double peak, double* part, double* out, hipStream_t st);

}  // namespace hbx
