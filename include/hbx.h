/*
 * hbx.h -- C-ABI of the MI355X-native binary-hologram hot path (libhbx.so).
 *
 * The reference (songyb111-gachon/binary-hologram-reinforcement-learning) is
 * pure Python: its hot path is a chain of torch ops behind the third-party
 * `torchOptics` API (tt.Tensor / tt.simulate / tt.relativeLoss / tm.get_PSNR)
 * called from gymnasium envs and DBS drivers.  This header is the boundary
 * those call sites bind to once the hot path is native.  Each entry point
 * names the reference interface it replaces (file:line under the reference).
 *
 * Conventions
 *   - Every buffer argument is a caller-owned DEVICE pointer (e.g. a
 *     torch-ROCm tensor's data_ptr()), contiguous, in the layout stated.
 *   - Masks are bit-packed: uint64 words [..][H][W/64], bit j of word w is
 *     pixel column 64*w + j (little-endian).  W % 64 == 0.
 *   - All calls are asynchronous on `stream` (a hipStream_t; NULL = default).
 *     A plan is bound to one device and is not re-entrant: one plan per
 *     stream / per GPU process.
 *   - Return 0 on success, a negative HBX_ERR_* code otherwise; the message
 *     is in hbx_last_error() (thread-local).  No C++ exception crosses it.
 *   - Channel c of an env belongs to colour group g = c / planes; group g
 *     propagates with wavelength[g]  (env_1024_24.py:135-147).
 */
#ifndef HBX_H
#define HBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HBX_ABI_VERSION 14

#define HBX_OK 0
#define HBX_ERR_INVALID (-1)     /* bad argument / shape                          */
#define HBX_ERR_HIP (-2)         /* HIP runtime error                             */
#define HBX_ERR_UNSUPPORTED (-3) /* size not built (N must be 64, 256, 896, 1024)  */
#define HBX_ERR_NOMEM (-4)       /* workspace allocation failed                   */

/* Transfer function (tt.simulate, env.py:172; SURVEY a4 assumptions as switches) */
#define HBX_TF_ASM 0       /* exact angular spectrum, evanescent cut              */
#define HBX_TF_FRESNEL 1   /* Fresnel transfer function                           */
/* Mask -> field (env.py:170-171) */
#define HBX_FIELD_AMPLITUDE 0 /* u = m in {0,1}  (literal reference)              */
#define HBX_FIELD_PHASE 1     /* u = exp(i pi m) in {+1,-1}                       */
/* tt.relativeLoss scale (env.py:174) */
#define HBX_REL_NONE 0
#define HBX_REL_LSQ 1      /* s = sum(I T)/sum(I^2) over every channel            */
/* accept rule */
#define HBX_ACCEPT_ENV 0   /* roll back iff delta < 0   (env.py:191)              */
#define HBX_ACCEPT_DBS 1   /* accept iff psnr > prev    (DBS_1024_24.py:355)      */
/* reward: env.py:188-254 (RW * change, cubic success / max-steps bonuses)
 * or env_group.py:250-318 (importance rank of the nearest sampled change,
 * linear success / max-steps bonuses 100 - (200/1500) (steps - 1000)). */
#define HBX_REWARD_PSNR 0
#define HBX_REWARD_IMPORTANCE 1

#define HBX_MAX_GROUPS 4

/* Optics of one plan; replaces tt.Tensor meta {'dx','wl'} + simulate's z
 * (env.py:124,172; env_1024_24.py:135-138; DBS_1024_24.py:230-233). */
typedef struct hbx_optics {
  int32_t height;                        /* N (64, 256, 896 or 1024), square */
  int32_t width;                         /* == height                         */
  int32_t groups;                        /* G: 1 mono, 3 RGB                  */
  int32_t planes;                        /* P planes per group (even)         */
  double wavelength[HBX_MAX_GROUPS];     /* metres, per group                 */
  double dx, dy;                         /* pixel pitch, metres               */
  double z;                              /* propagation distance, metres      */
  int32_t tf_kind;                       /* HBX_TF_*                          */
  int32_t field_kind;                    /* HBX_FIELD_*                       */
  int32_t rel_scale;                     /* HBX_REL_*                         */
  int32_t reserved;
  double peak;                           /* PSNR peak (1.0)                   */
} hbx_optics_t;

/* Device-resident state of B environments (BinaryHologramEnv attributes,
 * env.py:65-81: state, state_record, previous/initial psnr, counters). */
typedef struct hbx_env_buffers {
  uint64_t* mask;          /* [B][G*P][H][W/64]  env.state                    */
  int8_t* record;          /* [B][G*P][H][W]     env.state_record (nullable)  */
  const float* target;     /* [B][G][H][W]       target image                 */
  double* chan_stats;      /* [B][G][3]          sum I*T, sum I^2, sum T^2    */
  double* init_psnr;       /* [B]                env.initial_psnr             */
  double* prev_psnr;       /* [B]                env.previous_psnr            */
  double* max_psnr_diff;   /* [B]                env.max_psnr_diff            */
  int64_t* steps;          /* [B]                env.steps                    */
  int64_t* flip_count;     /* [B]                env.flip_count               */
  int64_t* sustained;      /* [B]                env.psnr_sustained_steps     */
  float* intensity;        /* [B][G][H][W] cached group means (nullable;
                              required by the incremental-field mode)          */
  int32_t* error;          /* [1] sticky device error word (nullable)         */
  float* field;            /* [B][G*P][H][W][2] complex64 propagated field of
                              every plane (nullable; incremental-field mode)   */
  /* env_group.py importance rewards (HBX_REWARD_IMPORTANCE only):            */
  const double* imp_changes;  /* [B][imp_count] psnr_change_list (env_group.py:90-120) */
  const double* imp_values;   /* [B][imp_count] importance_ranks (env_group.py:121-143) */
  const double* t_psnr_diff;  /* [B] per-env T_PSNR_DIFF (dynamic threshold,
                                 env_group.py:198; nullable -> params value)  */
  int32_t imp_count;          /* 10000 in the reference                       */
  int32_t reserved;
  /* ABI v8: zero-copy observations (env.py:135-140,176-181).  The reference
   * hands out env.state itself as obs["state"] and the stepped reconstruction
   * as obs["recon_image"]; these buffers are those observations, kept current
   * by reset and step so a caller can alias them instead of rebuilding them. */
  int8_t* state_bytes;     /* [B][G*P][H][W] 0/1 = the mask bits as int8:
                              obs["state"] (nullable).  Written by hbx_env_reset
                              / hbx_env_obs_sync and by the accepted flip of
                              every step (both modes).                        */
  float* recon;            /* [B][G][H][W] obs["recon_image"] (nullable; FFT
                              mode only; needs intensity and recon_pending).
                              After hbx_env_step the stepped group holds the
                              stepped (pre-rollback) intensity, env.py:179,
                              written there by the propagation itself; the
                              other groups hold the cached accepted ones.     */
  int32_t* recon_pending;  /* [B] internal: the group the next step reconciles
                              between recon and intensity (+g+1: accepted,
                              recon -> intensity; -(g+1): rolled back,
                              intensity -> recon; 0: none).  With recon given,
                              env->intensity of the last stepped group is
                              current only after that reconcile.
                              ABI v12: with ONE colour group (G = 1) every step
                              rewrites recon whole and nothing is ever restored,
                              so no reconcile runs: recon_pending stays 0 and
                              env->intensity keeps the last reset's / sync's
                              values (HBX_OBS_RECON re-propagates it).        */
  /* ABI v9: plane-cached FFT mode (N = 1024 / 256; both non-null, with
   * hbx_env_reset / hbx_field_refresh filling them).  A step changes ONE plane
   * of the touched group, and the FFT mode's re-propagation of the other plane
   * pairs reproduces their |U_q|^2 bit for bit (deterministic kernels), so the
   * step propagates only the flipped plane's pair and sums the cached planes
   * in the same plane order: the group intensity, statistics, PSNR, reward and
   * every decision are the FFT mode's bit for bit (env.py:170-174 work, 1/4 of
   * the propagation).  The pair is propagated, not the flipped plane alone:
   * k_rowfwd transforms two planes as the real and imaginary parts of one
   * complex FFT, so the partner's rounding sees the flipped plane and its bits
   * change too.  Both fresh |U|^2 go to the env's two spare slots and are
   * swapped in on accept (rollback: nothing to undo). */
  float* plane_inten;      /* [B][G*P + 2][H][W] f32 pool of per-plane |U|^2  */
  int32_t* plane_slot;     /* [B][G*P + 2] pool slot of each plane; [G*P] and
                              [G*P + 1] are the spares (caller-owned, filled
                              by reset)                                       */
  /* ABI v11: one-copy-free step readback.  hbx_env_step's last kernel copies
   * *error here (nullable; typically host memory from hbx_host_alloc, given by
   * its device address), so a caller whose reward / psnr / flag outputs also
   * live in such memory reads the whole step result on the host once the
   * stream work is complete, with no device-to-host copy. */
  int32_t* error_host;
} hbx_env_buffers_t;

/* BinaryHologramEnv.__init__ keyword arguments (env.py:38) + RW (env.py:29). */
typedef struct hbx_env_params {
  int64_t max_steps;       /* 10000 */
  double t_psnr;           /* 30    */
  int64_t t_steps;         /* 1     */
  double t_psnr_diff;      /* 0.1   */
  double reward_weight;    /* 800   */
  int32_t accept_rule;     /* HBX_ACCEPT_ENV */
  int32_t reward_kind;     /* HBX_REWARD_PSNR (env.py) | HBX_REWARD_IMPORTANCE (env_group.py) */
} hbx_env_params_t;

typedef struct hbx_plan* hbx_plan_t;

/* Library identity. */
int hbx_abi_version(void);
const char* hbx_last_error(void);

/* ABI v11: page-locked host memory that the GPU reads and writes directly
 * (mapped, coherent).  *host is the CPU address, *device the address to pass
 * to kernels (the step outputs of hbx_env_step, env->error_host).  The
 * reference's VecEnv hands numpy rewards / dones to SB3 every step
 * (train-PPO.py:296-322, env.py:259): the step kernels write them here and the
 * host reads them without a copy engine round trip.  Free with hbx_host_free. */
int hbx_host_alloc(size_t bytes, void** host, void** device);
int hbx_host_free(void* host);

/* Plan: owns twiddles, transfer-function tables and a workspace for up to
 * `max_jobs` concurrent group propagations (P * 12 * N^2 bytes per job:
 * 96 MiB at N = 1024, P = 8; hbx_plan_workspace_bytes gives the total).
 * Replaces the per-call setup hidden inside tt.simulate (env.py:172). */
int hbx_plan_create(hbx_plan_t* plan, const hbx_optics_t* optics, int32_t max_jobs,
                    int32_t device);
int hbx_plan_destroy(hbx_plan_t plan);
size_t hbx_plan_workspace_bytes(hbx_plan_t plan);
/* Propagation pipeline the plan runs (ABI v4): which kernels fill the pass
 * timer slots HBX_PASS_ROWFWD / HBX_PASS_COL below.  Since ABI v8 always
 *   HBX_PIPE_THREE_PASS  k_rowfwd -> k_col2 -> k_rowinv (N = 64, 256, 896, 1024; N = 896 runs
 *                        the fused mixed-radix 28 x 32 kernels of the same three passes)
 * (the r01 / r02 bits -> column pass and composed generic-N pipelines, values 1 and 2, were
 * measured slower and removed). */
#define HBX_PIPE_THREE_PASS 0
int hbx_plan_pipeline(hbx_plan_t plan);

/* Full propagation of every group of n_env masks (env.py:123-133 reset path,
 * env_1024_24.py:149-166, DBS_1024_24.py:244-257):
 *   intensity[B][G][H][W] = mean_p |IFFT2(FFT2(u_p) H_g)|^2   (nullable)
 *   chan_stats[B][G][3]   = per-channel sum I*T, sum I^2, sum T^2
 *   psnr[B]               = relativeLoss(rgb, target, get_PSNR)  (nullable)  */
int hbx_propagate(hbx_plan_t plan, const uint64_t* mask, const float* target, int32_t n_env,
                  float* intensity, double* chan_stats, double* psnr, void* stream);

/* tt.simulate(tt.Tensor(mask, meta), z) (env.py:170-172; DBS_1024_24.py:
 * 326-328) for binary masks: the propagated complex field of every plane,
 *   field[B][G*P][H][W][2] = IFFT2(FFT2(u) H_g)   (complex64, re/im pairs)
 * and optionally the plane-mean intensity[B][G][H][W] (nullable). */
int hbx_simulate(hbx_plan_t plan, const uint64_t* mask, int32_t n_env, float* field,
                 float* intensity, void* stream);

/* PSNR from per-channel statistics (tt.relativeLoss(.., tm.get_PSNR),
 * env.py:174): chan_stats[B][G][3] -> psnr[B]. */
int hbx_psnr(hbx_plan_t plan, const double* chan_stats, int32_t n_env, double* psnr,
             void* stream);

/* Env reset tail (env.py:120-133): given env.mask already thresholded and
 * env.target set for the listed envs (env_ids nullable = all n_env), propagate
 * every group, fill chan_stats / intensity (and env.field when non-null),
 * set init_psnr = prev_psnr and zero steps / flip_count / sustained / record,
 * max_psnr_diff = -inf. */
int hbx_env_reset(hbx_plan_t plan, const hbx_env_buffers_t* env, int32_t n_env,
                  const int32_t* env_ids, int32_t n_ids, void* stream);

/* Batched env.step(action) (env.py:154-259 mono; DBS_1024_24.py:313-422
 * per-flip RGB with cached other-group statistics).  One action per env:
 * decode (env.py:157-161), flip + record, re-propagate the touched colour
 * group, relative PSNR, reward = RW * delta, rollback / bonus / termination.
 *   reward, psnr [B] f64; accepted, terminated, truncated [B] u8 (nullable; device
 *   addresses, e.g. of hbx_host_alloc'd host-mapped memory -- ABI v11: the kernels then
 *   write the results straight to the host, readable once the stream work is done)
 *   group_intensity [B][H][W] f32: the stepped (pre-rollback) group mean
 *   (nullable; not together with env->recon, which already holds it).
 * With env->recon (ABI v8) the last pass writes the stepped intensity straight
 * into recon[b][g] and the step starts by reconciling the previous step's
 * group (one N^2 f32 copy per env); without it, accepted steps refresh
 * env->intensity[b][g] when that cache is non-null.  env->state_bytes, when
 * non-null, follows every accepted flip. */
int hbx_env_step(hbx_plan_t plan, const hbx_env_buffers_t* env, const hbx_env_params_t* params,
                 int32_t n_env, const int64_t* actions, double* reward, double* psnr,
                 uint8_t* accepted, uint8_t* terminated, uint8_t* truncated,
                 float* group_intensity, void* stream);

/* DBS primitive (SURVEY 8b hbx_step): one candidate flip per env evaluated
 * against prev_psnr and applied iff accepted (accept_rule), without the
 * env's reward bookkeeping (DBS.py:247-294). */
int hbx_step(hbx_plan_t plan, uint64_t* mask, const int64_t* actions, int32_t n_env,
             const float* target, double* chan_stats, double* prev_psnr, double* psnr_out,
             uint8_t* accepted, int32_t accept_rule, void* stream);

/* Independent trial flips against ONE fixed base env (probe sweep
 * DBS_1024_24-128.py:310-373, range.py:294-335, env_group.py:96-120 and the
 * speculative batches of greedy DBS): for k < K
 *   psnr_out[k]      = PSNR with pixel flips[k] toggled
 *   group_stats[k][3] = stats of the touched group (nullable)            */
int hbx_eval_flips(hbx_plan_t plan, const uint64_t* base_mask, const float* target,
                   const double* base_chan_stats, const int64_t* flips, int32_t K,
                   double* psnr_out, double* group_stats, void* stream);

/* PSNR change of EVERY single-pixel flip of one env against its current
 * state, all CH*H*W of them at once (the full probe sweep
 * DBS_1024_24-128.py:310-373 / range.py:294-335 and env_group.py:90-143's
 * sampled importance pass, without one propagation per flip):
 *   dpsnr[c][r][col] = PSNR(state with (c, r, col) toggled) - PSNR(state)
 * By linearity a flip adds delta * h_g(. - x0) to one plane's field, so the
 * new (sum I T, sum I^2) are correlations of functions of the fields, the
 * intensity and the target with functions of the single-pixel field h_g,
 * evaluated with 2-D FFTs (hbx_map.hip).  mask [CH][H][W/64], target
 * [G][H][W] (one env), dpsnr [CH][H][W] f32, base_psnr (nullable) f64. */
int hbx_flip_map(hbx_plan_t plan, const uint64_t* mask, const float* target, float* dpsnr,
                 double* base_psnr, void* stream);

/* Commit one accepted candidate of hbx_eval_flips into the base env:
 * toggle mask bit `flips[k]`, chan_stats[g] = group_stats[k], prev_psnr =
 * psnr_out[k].  Device-side; `k` is a device int32 (from the host or a
 * device search); K (ABI v6) is the length of flips / psnr_out / group_stats:
 * a k outside [0, K) commits nothing. */
int hbx_commit_flip(hbx_plan_t plan, uint64_t* base_mask, double* base_chan_stats,
                    double* prev_psnr, const int64_t* flips, const double* psnr_out,
                    const double* group_stats, const int32_t* k, int32_t K, void* stream);

/* (ABI v10) hbx_eval_flips / hbx_commit_flip with the base env's per-plane
 * |U_p|^2 cached (N = 1024 / 256): the speculative greedy DBS of
 * DBS_1024_24.py:313-363 in the FFT mode, bit for bit, at a fraction of the
 * bytes.  A candidate flips one plane, so only that plane's PAIR (the two
 * planes one complex row FFT carries) is propagated; the group intensity sums
 * the cached planes and the pair's fresh ones in the FFT mode's plane order,
 * i.e. the same f32 sum.  Candidate k writes its pair's fresh |U|^2 to spare
 * pair k of the pool; committing candidate k swaps that pair's slots in.
 *   plane_inten [CH + 2 S][H][W] f32, plane_slot [CH + 2 S] int32 (S =
 *   n_spare_pairs >= K): filled by hbx_planes_fill from the base mask
 *   (identity slots, every plane's |U|^2, the base chan_stats / psnr).
 * Replaces the per-flip tt.simulate of the whole colour group
 * (DBS_1024_24.py:326-332) in speculative batches. */
int hbx_planes_fill(hbx_plan_t plan, const uint64_t* mask, const float* target, float* plane_inten,
                    int32_t* plane_slot, int32_t n_spare_pairs, double* chan_stats, double* psnr,
                    void* stream);
int hbx_eval_flips_planes(hbx_plan_t plan, const uint64_t* base_mask, const float* target,
                          const double* base_chan_stats, float* plane_inten, const int32_t* plane_slot,
                          int32_t n_spare_pairs, const int64_t* flips, int32_t K, double* psnr_out,
                          double* group_stats, void* stream);
int hbx_commit_flip_planes(hbx_plan_t plan, uint64_t* base_mask, double* base_chan_stats,
                           double* prev_psnr, int32_t* plane_slot, int32_t n_spare_pairs,
                           const int64_t* flips, const double* psnr_out, const double* group_stats,
                           const int32_t* k, int32_t K, void* stream);


/* hbx_eval_flips / hbx_commit_flip on the incremental-field path: the base
 * env additionally carries its per-plane field [CH][H][W][2] and group
 * intensities [G][H][W] (hbx_simulate), so a candidate costs one streaming
 * pass over one plane (no FFT) -- the speculative greedy DBS of
 * DBS_1024_24.py:313-422 at ~16 B/px per candidate.  The commit also rewrites
 * the accepted plane's field and its group intensity. */
int hbx_eval_flips_psf(hbx_plan_t plan, const uint64_t* base_mask, const float* target,
                       const double* base_chan_stats, const float* field, const float* intensity,
                       const int64_t* flips, int32_t K, double* psnr_out, double* group_stats,
                       void* stream);
int hbx_commit_flip_psf(hbx_plan_t plan, uint64_t* base_mask, double* base_chan_stats,
                        double* prev_psnr, float* field, float* intensity, const int64_t* flips,
                        const double* psnr_out, const double* group_stats, const int32_t* k,
                        int32_t K, void* stream);

/* Device-resident greedy DBS walk (ABI v5): the whole loop of DBS.py:247-294 /
 * DBS_1024_24.py:313-422 -- visit order[pos..], keep a flip iff PSNR strictly
 * improves -- as speculative batches that never return to the host.  Each
 * batch evaluates the next K candidates on the incremental-field path (as
 * hbx_eval_flips_psf); a one-block launch picks the first improving one in
 * visiting order, toggles its mask bit, updates base_chan_stats and the walk
 * state and appends (position, psnr) to the accept log; a third launch
 * rewrites the accepted plane's field and group intensity.  `batches` batches
 * are enqueued per call with no host synchronisation; batches after the walk
 * is done (or halted) cost three empty launches.  The accept sequence is the
 * serial loop's: every candidate before an accepted one was evaluated against
 * exactly the state the serial loop would have had.
 *
 * ABI v7: for K in 1..4 a batch is ONE launch (k_walk_step):
 * it first applies the previous batch's accepted flip(s) to field / intensity,
 * evaluates the K candidates on the updated state, and its last-arriving
 * workgroup decides; for K = 2..4 it also resolves the first candidate after
 * the first accept against the state WITH that accept (exact pairwise terms),
 * so a batch takes up to two accepts of the serial loop.  The accepted flips of
 * a batch therefore reach field / intensity in the NEXT launch: after the walk
 * is done make one more call (batches >= 1; it only commits).  K > 4 runs the
 * three-launch batch of ABI v5 (eval / decide / commit; also selected for every
 * K by HBX_WALK_SPLIT=1 in the environment at plan creation); a call that
 * switches from the one-launch to the three-launch form first issues one
 * commit-only step for the pending accepts.
 *
 * The walk state lives in DEVICE memory (caller-owned; commit_ch = -1,
 * commit2_ch1 = 0, split_ch1 = 0 and the counters zero at the start); the caller reads it back
 * between calls.  When halt == 1 (after every refresh_every-th accept) the
 * caller re-propagates field, intensity and base_chan_stats exactly
 * (hbx_simulate / hbx_propagate) -- the mask already holds every accepted flip,
 * so it also drops pending commits (commit_ch = -1, commit2_ch1 = 0) -- sets
 * prev_psnr to the exact PSNR and clears halt.
 * n_order (ABI v6) is the length of `order`: the walk never visits past
 * min(walk->total, n_order).
 * The walk's partial sums, arrival counters and decoded next actions live in
 * plan-owned scratch: at most one walk per plan may be in flight at a time
 * (walks of several images side by side need one plan each, as
 * hbx.dbs.greedy_many enforces); each call re-derives the decoded actions
 * from `order` once, so a new walk on the same plan needs no reset.
 *
 * Candidate evaluation is in increment form: each candidate's f64 partials
 * are sum dI T and sum (2 I + dI) dI with dI = delta (2 Re(U conj h) +
 * delta |h|^2) / P formed in f32 per pixel, added to base_chan_stats -- the
 * decision carries the increment's own f32 precision (~1e-13 dB at 1024x24),
 * not the rounding of full-image sums. */
typedef struct hbx_dbs_walk {
  int64_t pos;             /* next position of `order` to visit                  */
  int64_t total;           /* positions to visit (order length or a prefix)      */
  int64_t accepted;        /* accepts so far (log entries written: min(., cap))  */
  int64_t batches;         /* speculative batches evaluated                      */
  double prev_psnr;        /* PSNR of the current base                           */
  double init_psnr;        /* PSNR at the start of the walk                      */
  double last_psnr;        /* PSNR of the last visited candidate                 */
  double stop_diff;        /* DBS_ratio_0.5.py:366-372 early stop threshold      */
  int32_t stop_enabled;    /* 1: done once prev_psnr - init_psnr >= stop_diff    */
  int32_t refresh_every;   /* halt after every refresh_every-th accept (0: never) */
  int32_t done;            /* 1: pos == total, or stopped early                  */
  int32_t halt;            /* 1: paused for an exact refresh (caller clears)     */
  int32_t stopped_early;
  int32_t commit_ch;       /* internal: pending commit channel, -1 = none        */
  int32_t commit_pix;      /* internal                                           */
  int32_t commit2_ch1;     /* internal (ABI v7): channel + 1 of a second pending
                              commit, 0 = none                                   */
  int32_t commit_pix2;     /* internal                                           */
  int32_t split_ch1;       /* internal (ABI v7): channel + 1 of the split batch's
                              accept, applied within the batch, 0 = none          */
  int32_t split_pix;       /* internal                                           */
  int32_t fault;           /* (r03) 1: a persistent walk launch's grid barrier timed
                              out (done is set too; the state is unreliable)     */
} hbx_dbs_walk_t;
int hbx_dbs_walk_psf(hbx_plan_t plan, uint64_t* base_mask, const float* target,
                     double* base_chan_stats, float* field, float* intensity, const int64_t* order,
                     int64_t n_order, hbx_dbs_walk_t* walk, int64_t* accept_pos, double* accept_psnr,
                     int64_t accept_cap, int32_t K, int32_t batches, void* stream);

/* (ABI v10) The same greedy DBS with the decision on the device: `batches`
 * speculative batches of K candidates (order[pos .. pos + K)) are enqueued
 * without a host round trip; after each batch's propagation one block forms
 * the K PSNRs (as hbx_eval_flips_planes), commits the first strict improvement
 * (as hbx_commit_flip_planes) into base_mask / base_chan_stats / plane_slot,
 * logs it (accept_pos / accept_psnr, up to accept_cap) and advances the walk
 * state (hbx_dbs_walk_t: pos, total, accepted, batches, prev / init / last
 * PSNR, stop_enabled / stop_diff, done, stopped_early; the incremental-walk
 * fields are unused).  Batches after `done` are no-ops.  K <= n_spare_pairs,
 * max_jobs and 256.  The accept sequence and every logged PSNR are the
 * host-decided batches' (and the full re-propagation's) bit for bit. */
int hbx_dbs_walk_planes(hbx_plan_t plan, uint64_t* base_mask, const float* target,
                        double* base_chan_stats, float* plane_inten, int32_t* plane_slot,
                        int32_t n_spare_pairs, const int64_t* order, int64_t n_order,
                        hbx_dbs_walk_t* walk, int64_t* accept_pos, double* accept_psnr,
                        int64_t accept_cap, int32_t K, int32_t batches, void* stream);

/* (ABI v13) EXTENSION, no reference counterpart (DBS_ratio_0.5.py has no on-pixel
 * constraint; BASELINE configs[4] names one): hbx_dbs_walk_planes under an on-pixel ratio
 * constraint.  fill_count[G] (device, caller-initialised) holds each colour group's on-pixel
 * count over its P planes; a candidate that moves group g's count C by d = +1 (pixel 0 -> 1) or
 * -1 is admissible iff |C + d - fill_target| <= fill_tol or |C + d - fill_target| < |C -
 * fill_target|.  An inadmissible candidate is visited and rejected without a propagation (no
 * PSNR); an accepted one updates fill_count.  fill_count NULL: hbx_dbs_walk_planes.  The
 * host-decided batches of hbx.dbs.greedy(..., fill_ratio=) apply the same rule. */
int hbx_dbs_walk_planes_fill(hbx_plan_t plan, uint64_t* base_mask, const float* target,
                             double* base_chan_stats, float* plane_inten, int32_t* plane_slot,
                             int32_t n_spare_pairs, const int64_t* order, int64_t n_order,
                             hbx_dbs_walk_t* walk, int64_t* accept_pos, double* accept_psnr,
                             int64_t accept_cap, int32_t K, int32_t batches, int64_t* fill_count,
                             int64_t fill_target, int64_t fill_tol, void* stream);

/* Incremental-field ("PSF") mode (reported separately from
 * the FFT-mode headline).  tt.simulate is linear, so flipping pixel (c, r, col)
 * changes only plane c's field, by delta * h_g shifted to (r, col), where
 * h_g = IFFT2(H_g) is the single-pixel field and delta = vb * (1 - 2 bit_old):
 *   U_c' = U_c + delta h_g(y - r, x - col),  I_g' = I_g + (|U_c'|^2 - |U_c|^2) / P
 * The step streams U_c, I_g and the target channel once (no FFT), then the
 * same reward / accept / rollback tail as hbx_env_step; accepted steps
 * rewrite U_c and I_g.  Requires env->field and env->intensity, filled by
 * hbx_env_reset (or hbx_field_refresh) with the exact FFT path. */
int hbx_env_step_psf(hbx_plan_t plan, const hbx_env_buffers_t* env, const hbx_env_params_t* params,
                     int32_t n_env, const int64_t* actions, double* reward, double* psnr,
                     uint8_t* accepted, uint8_t* terminated, uint8_t* truncated, void* stream);

/* (ABI v8) Rebuild the observation mirrors of the listed envs (env_ids
 * nullable = all n_env) from the state they mirror:
 *   HBX_OBS_STATE  state_bytes <- the mask bits
 *   HBX_OBS_RECON  recon <- intensity, recon_pending <- 0; the intensity cache is
 *                  taken as authoritative (it was just rewritten: reset, checkpoint load).
 *                  ABI v12, G = 1: intensity is first re-propagated from the mask (the
 *                  step keeps no cache at one group; needs env->target)
 *   HBX_OBS_RESOLVE (ABI v10, with HBX_OBS_RECON) apply the last step's pending
 *                  reconcile first: after an accepted step the stepped group's new
 *                  intensity lives in recon only (recon_pending = group + 1), so that
 *                  group goes recon -> intensity and the others intensity -> recon.
 *                  Use it to re-sync mid-episode without rewriting intensity.
 *   HBX_OBS_SETTLE (ABI v11, alone) the accepted half of that reconcile only: envs
 *                  whose last step was accepted (recon_pending > 0) copy the stepped
 *                  group recon -> intensity and clear recon_pending; recon is not
 *                  touched (it is still the observation the step returned), rolled-back
 *                  envs keep their pending restore for the next step.  A VecEnv queues
 *                  it right behind the step's readback, so the copy runs while the host
 *                  turns the step around instead of inside the next step's k_rowinv.
 *                  ABI v12: a no-op at G = 1 (nothing is pending).
 * hbx_env_reset does both for the envs it resets; a caller that restores
 * masks or intensities by itself (checkpoint load) calls it after. */
#define HBX_OBS_STATE 1
#define HBX_OBS_RECON 2
#define HBX_OBS_RESOLVE 4
#define HBX_OBS_SETTLE 8
int hbx_env_obs_sync(hbx_plan_t plan, const hbx_env_buffers_t* env, int32_t n_env,
                     const int32_t* env_ids, int32_t n_ids, int32_t what, void* stream);

/* Exact re-propagation (FFT path) of env->field, env->intensity and
 * env->chan_stats for the listed envs (bounds the fp32 drift of the
 * incremental updates; counters and PSNR history are left untouched).
 * ABI v9: with env->plane_inten / plane_slot (and no field) it rebuilds the
 * plane cache instead (after a checkpoint load). */
int hbx_field_refresh(hbx_plan_t plan, const hbx_env_buffers_t* env, int32_t n_env,
                      const int32_t* env_ids, int32_t n_ids, void* stream);

/* Precision of the propagation intermediates (ABI v6; SURVEY 8d cfg 5,
 * DBS_ratio_0.5.py fp32-vs-bf16 sweep).  HBX_PRECISION_F32 is the product
 * path.  HBX_PRECISION_BF16_STORE / HBX_PRECISION_F16_STORE round every value
 * written to the two pass intermediates (row spectrum, column-pass output) to
 * bf16 / fp16 -- the numerics of half-width intermediate storage, measured
 * against f32 by tools/precision_sweep.py and bench.py (layout and traffic
 * stay f32).  N = 64 / 256 / 1024 three-pass path only (HBX_ERR_UNSUPPORTED
 * elsewhere). */
#define HBX_PRECISION_F32 0
#define HBX_PRECISION_BF16_STORE 1
#define HBX_PRECISION_F16_STORE 2
int hbx_plan_set_precision(hbx_plan_t plan, int32_t precision);
int hbx_plan_precision(hbx_plan_t plan);

/* Optional device timing of the three propagation passes (hipEvents recorded
 * on the launch stream around every pass launch; not for graph capture).
 * capacity = max launches recorded per pass before hbx_plan_read_timing;
 * 0 disables.  Replaces debug_env.py:165-306's per-phase time.time() prints. */
#define HBX_PASS_ROWFWD 0
#define HBX_PASS_COL 1
#define HBX_PASS_ROWINV 2
#define HBX_PASS_PSF_EVAL 3
#define HBX_PASS_PSF_COMMIT 4
#define HBX_NUM_PASSES 5
int hbx_plan_set_timing(hbx_plan_t plan, int32_t capacity);
/* As hbx_plan_set_timing, recording only every `every`-th launch of each pass
 * (every >= 1; 1 = hbx_plan_set_timing).  Each event pair costs a few us of
 * stream time (the record's release), a visible share of a 0.35 ms 256x256x8
 * step: sampling keeps the timed loop's step time within noise of an untimed
 * one while the recorded launches are still those of that loop. */
int hbx_plan_set_timing_sampled(hbx_plan_t plan, int32_t capacity, int32_t every);
/* Waits for the recorded events; ms_total[HBX_NUM_PASSES] = summed kernel
 * time, launches[HBX_NUM_PASSES], jobs[HBX_NUM_PASSES] = summed jobs per
 * launch; then clears the record. */
int hbx_plan_read_timing(hbx_plan_t plan, double* ms_total, int64_t* launches, int64_t* jobs);

/* (ABI v14) Mask -> bits on the device, one streaming pass (hbx_pack.hip).  Replaces the
 * per-call host / torch work in front of every propagation: env reset's `state =
 * (pre_model >= 0.5)` (env.py:120, env_1024_24.py:120-124) and the float / int8 mask that
 * tt.simulate receives (env.py:123,170-171 `tt.Tensor(torch.tensor(state, float32))`;
 * DBS_1024_24.py:326-327).
 *   src      `n_values` contiguous values of kind src_kind (HBX_SRC_U8: bool / int8 / uint8
 *            bytes; HBX_SRC_F32; HBX_SRC_F64), aligned to 4 (u8) / 16 (f32) / 32 (f64) bytes;
 *            n_values % 64 == 0 (rows of W values with W % 64 == 0 are contiguous words)
 *   bits     n_values / 64 words in the mask layout above (bit j of word w = value 64 w + j)
 *   mode     HBX_PACK_BINARY: bit = (v != 0); a value that is not 0 or 1 (NaN included)
 *            stores 1 into *error (nullable; any address the kernel may write, e.g. host
 *            memory from hbx_host_alloc, so the check needs no device -> host copy).
 *            HBX_PACK_THRESHOLD: bit = (v >= threshold) (NaN -> 0, as torch's `>=`).
 * Runs on the current device, asynchronously on `stream`; no plan needed. */
#define HBX_SRC_U8 0
#define HBX_SRC_F32 1
#define HBX_SRC_F64 2
#define HBX_PACK_BINARY 0
#define HBX_PACK_THRESHOLD 1
int hbx_pack_mask(const void* src, int32_t src_kind, int64_t n_values, int32_t mode, double threshold,
                  uint64_t* bits, int32_t* error, void* stream);

/* (ABI v14) tt.relativeLoss(x, y, tm.get_PSNR / F.mse_loss) (env.py:131-132,174;
 * DBS_1024_24.py:332,342,352) in one fixed-order f64 reduction: x, y `n` contiguous values
 * of kind HBX_SRC_F32 or HBX_SRC_F64 (both the same kind);
 *   out[5] = {sum x y, sum x^2, sum y^2, PSNR, MSE}  with the plans' rel_scale rule
 *   (HBX_REL_LSQ: s = sum xy / sum x^2, MSE = mean((s x - y)^2); HBX_REL_NONE: s = 1) and
 *   PSNR = 10 log10(peak^2 / MSE) (+inf at MSE <= 0).
 * `workspace` holds HBX_REL_WORKSPACE_DOUBLES doubles (device); `out` any address the kernel
 * may write (host-mapped memory reads back without a copy). */
#define HBX_REL_WORKSPACE_DOUBLES 3072
int hbx_rel_stats(const void* x, const void* y, int32_t src_kind, int64_t n, int32_t rel_scale, double peak,
                  double* workspace, double* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HBX_H */
