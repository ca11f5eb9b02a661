// hbx_kernels.hip -- HIP kernels of the binary-hologram hot path (gfx950).
//
// This file: the small per-job / per-env kernels that turn the propagation
// passes' partial sums (hbx_passes.hip) into PSNR / reward / accept-rollback
// (env.py:154-259) on the device -- no host sync per step.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "hbx_fft.hpp"
#include "hbx_internal.hpp"
#include "hbx_walk_planes.hpp"

namespace hbx {

// ---------------------------------------------------------------------------
// Small per-job / per-env kernels
// ---------------------------------------------------------------------------
// jobs from actions: one job per env (env.py:157-161 decode)
__global__ void k_jobs_from_actions(const int64_t* __restrict__ actions, int n, int H, int W,
                                    int P, int CH, JobDesc* __restrict__ jobs,
                                    int32_t* __restrict__ err) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const JobDesc jd = job_of_action(actions[b], b, (int64_t)H * W, P, CH);
  if (jd.env < 0 && err) atomicOr(err, 1);
  jobs[b] = jd;
}

// flip jobs against one base env (probe sweep / speculative DBS)
__global__ void k_jobs_from_flips(const int64_t* __restrict__ flips, int K, int H, int W, int P,
                                  int CH, JobDesc* __restrict__ jobs) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const int64_t a = flips[k];
  const int64_t hw = (int64_t)H * W;
  JobDesc jd;
  if (a < 0 || a >= (int64_t)CH * hw) {
    jd.env = -1; jd.group = 0; jd.flip_plane = -1; jd.flip_pix = 0;
  } else {
    const int ch = (int)(a / hw);
    jd.env = 0; jd.group = ch / P; jd.flip_plane = ch % P; jd.flip_pix = (int)(a % hw);
  }
  jobs[k] = jd;
}

// the one job of candidate flips[*k] (commit of a speculative batch)
__global__ void k_job_from_flip_k(const int64_t* __restrict__ flips, const int32_t* __restrict__ k, int K,
                                  int H, int W, int P, int CH, JobDesc* __restrict__ jobs,
                                  int32_t* __restrict__ order, int32_t* __restrict__ accept) {
  const int kk = *k;
  const int64_t a = (kk >= 0 && kk < K) ? flips[kk] : -1;   // k outside [0, K): nothing to commit
  const int64_t hw = (int64_t)H * W;
  JobDesc jd;
  if (a < 0 || a >= (int64_t)CH * hw) {
    jd.env = -1; jd.group = 0; jd.flip_plane = -1; jd.flip_pix = 0;
  } else {
    const int ch = (int)(a / hw);
    jd.env = 0; jd.group = ch / P; jd.flip_plane = ch % P; jd.flip_pix = (int)(a % hw);
  }
  jobs[0] = jd;
  order[0] = 0;
  accept[0] = jd.env >= 0 ? 1 : 0;
}

// full-propagation jobs: (env_ids[i], g) for all groups
__global__ void k_jobs_full(const int32_t* __restrict__ env_ids, int n_ids, int G,
                            JobDesc* __restrict__ jobs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ids * G) return;
  const int e = env_ids ? env_ids[i / G] : i / G;
  JobDesc jd;
  jd.env = e; jd.group = i % G; jd.flip_plane = -1; jd.flip_pix = 0;
  jobs[i] = jd;
}

// sum the row-block partials of every job (fixed order) -> job_stats[j][3]
// grid (n_jobs), one wave per job: the wave stages the job's row-block partials in LDS with
// coalesced loads, then lane 0 adds them in row-block order (the fixed order every result
// depends on, bit for bit).  One thread per job walking its 3 KB of partials took ~20 us
// per 128-job launch (rocprofv3, profiles/r02_final4/kernel_stats.csv).
__global__ __launch_bounds__(64) void k_reduce_partials(const double* __restrict__ partial, int n_jobs, int RB,
                                                        double* __restrict__ job_stats) {
  constexpr int CHUNK = 768;   // doubles per staging round (a multiple of 3)
  __shared__ double s[CHUNK];
  const int j = blockIdx.x;
  if (j >= n_jobs) return;
  // lane k < 3 carries sum k (a separate chain per statistic, each in row-block order)
  const int k = threadIdx.x;
  double acc = 0.0;
  const double* p = partial + (size_t)j * RB * 3;
  for (int c0 = 0; c0 < 3 * RB; c0 += CHUNK) {
    const int n = 3 * RB - c0 < CHUNK ? 3 * RB - c0 : CHUNK;
    for (int i = threadIdx.x; i < n; i += 64) s[i] = p[c0 + i];
    __syncthreads();
    if (k < 3)
#pragma unroll 8
      for (int i = k; i < n; i += 3) acc += s[i];
    __syncthreads();
  }
  if (k < 3) job_stats[3 * j + k] = acc;
}

// scatter full-propagation job stats into chan_stats[env][g]; psnr per env
__global__ void k_full_finalize(const JobDesc* __restrict__ jobs, const double* __restrict__ job_stats,
                                int n_ids, int G, double* __restrict__ chan_stats,
                                double* __restrict__ psnr, double count, int rel_scale, double peak,
                                EnvDev env, int reset) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ids) return;
  const int e = jobs[i * G].env;
  double sxy = 0.0, sxx = 0.0, syy = 0.0;
  for (int g = 0; g < G; ++g) {
    const double* s = job_stats + 3 * (size_t)(i * G + g);
    if (chan_stats) {
      double* d = chan_stats + ((size_t)e * G + g) * 3;
      d[0] = s[0]; d[1] = s[1]; d[2] = s[2];
    }
    sxy += s[0]; sxx += s[1]; syy += s[2];
  }
  const double ps = psnr_from(sxy, sxx, syy, count, rel_scale, peak);
  if (psnr) psnr[e] = ps;
  if (reset) {
    env.init_psnr[e] = ps;
    env.prev_psnr[e] = ps;
    env.max_psnr_diff[e] = -INFINITY;
    env.steps[e] = 0;
    env.flip_count[e] = 0;
    env.sustained[e] = 0;
  }
}

__device__ __forceinline__ double success_cubic(double s, double c0) {
  // env.py:230-235 / 249-254
  return 1828.57 * (s * s * s) - 3733.33 * (s * s) + 2800.0 * s - c0;
}

// env.step tail (env.py:155-259) for one env per thread
__global__ void k_env_step_finalize(const JobDesc* __restrict__ jobs,
                                    const double* __restrict__ job_stats, int n, int G, int P,
                                    int H, int W, EnvDev env, EnvParams prm, double count,
                                    int rel_scale, double peak, double* __restrict__ reward_out,
                                    double* __restrict__ psnr_out, uint8_t* __restrict__ acc_out,
                                    uint8_t* __restrict__ term_out, uint8_t* __restrict__ trunc_out,
                                    int32_t* __restrict__ accept_flag, double* __restrict__ delta_out,
                                    const double* __restrict__ partial, int RB) {
  __shared__ double s_part[768];
  __shared__ double s_js[3];
  int b;
  const double* js;
  if (partial) {
    // k_reduce_partials fused (one launch per step less): one wave per env sums its job's
    // row-block partials in row-block order (k_reduce_partials' order bit for bit), lane 0
    // finalizes
    b = blockIdx.x;
    const int k = threadIdx.x;
    double acc = 0.0;
    const double* p = partial + (size_t)b * RB * 3;
    for (int c0 = 0; c0 < 3 * RB; c0 += 768) {
      const int m = 3 * RB - c0 < 768 ? 3 * RB - c0 : 768;
      for (int i = k; i < m; i += 64) s_part[i] = p[c0 + i];
      __syncthreads();
      if (k < 3)
#pragma unroll 8
        for (int i = k; i < m; i += 3) acc += s_part[i];
      __syncthreads();
    }
    if (k < 3) s_js[k] = acc;
    __syncthreads();
    if (k != 0 || b >= n) return;
    js = s_js;
  } else {
    b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n) return;
    js = job_stats + 3 * (size_t)b;
  }
  // the error word is final here: every kernel of the step that sets it (k_jobs_from_actions, or
  // at N = 1024 / 256 the fused first pass's decode) ran before this one.  Mirror it next to the
  // step outputs (ABI v11); a later error source must run before this kernel, which stays the
  // last one of the step that reads the word
  if (b == 0 && env.error_host) env.error_host[0] = env.error ? env.error[0] : 0;
  const JobDesc jb = jobs[b];
  if (delta_out) delta_out[b] = NAN;   // no importance lookup for an invalid job
  if (jb.env < 0) {
    if (reward_out) reward_out[b] = 0.0;
    if (psnr_out) psnr_out[b] = env.prev_psnr[b];
    if (acc_out) acc_out[b] = 0;
    if (term_out) term_out[b] = 0;
    if (trunc_out) trunc_out[b] = 0;
    if (accept_flag) accept_flag[b] = 0;
    // recon_pending stays: an invalid job propagates nothing, so the previous step's reconcile
    // (fused into k_rowinv_d, which skips invalid jobs) is still owed and the next valid step
    // applies it (the separate k_recon_reconcile of the other sizes is idempotent)
    return;
  }
  const int g = jb.group;
  const int ch = g * P + jb.flip_plane;
  const int CH = G * P;
  const int64_t steps = env.steps[b] + 1;            // env.py:155
  env.steps[b] = steps;
  if (env.record) {                                   // env.py:165 (int8 wraps like numpy)
    int8_t* r = env.record + ((size_t)b * CH + ch) * (size_t)H * W + jb.flip_pix;
    *r = (int8_t)(*r + 1);
  }
  int64_t flips = env.flip_count[b] + 1;             // env.py:167
  double* st = env.chan_stats + (size_t)b * G * 3;
  double sxy = 0.0, sxx = 0.0, syy = 0.0;
  for (int gg = 0; gg < G; ++gg) {
    if (gg == g) { sxy += js[0]; sxx += js[1]; syy += js[2]; }
    else { sxy += st[3 * gg]; sxx += st[3 * gg + 1]; syy += st[3 * gg + 2]; }
  }
  const double psnr_after = psnr_from(sxy, sxx, syy, count, rel_scale, peak);
  const double change = psnr_after - env.prev_psnr[b];   // env.py:184
  const double diff = psnr_after - env.init_psnr[b];     // env.py:185
  const bool importance = prm.reward_kind == 1;
  // env.py:188 / env_group.py:254-255 (the importance term is added by
  // k_importance_reward from delta_out; here only the bonuses accumulate)
  double reward = importance ? 0.0 : change * prm.reward_weight;
  if (delta_out) delta_out[b] = change;
  const double tpd = env.t_psnr_diff ? env.t_psnr_diff[b] : prm.t_psnr_diff;   // env_group.py:198
  const bool reject = (prm.accept_rule == 0) ? (change < 0.0) : !(change > 0.0);
  bool term = false, trunc = false;
  if (reject) {                                           // env.py:191-196
    flips -= 1;
  } else {
    uint64_t* word = env.mask + ((size_t)b * CH + ch) * (size_t)H * (W / 64) + (size_t)(jb.flip_pix / W) * (W / 64) +
                     (jb.flip_pix % W) / 64;
    const uint64_t nw = *word ^ (1ull << ((jb.flip_pix % W) & 63));
    *word = nw;
    if (env.state_bytes)                                 // obs["state"] mirror (env.py:177 hands out self.state)
      env.state_bytes[((size_t)b * CH + ch) * (size_t)H * W + jb.flip_pix] = (int8_t)((nw >> ((jb.flip_pix % W) & 63)) & 1ull);
    st[3 * g] = js[0]; st[3 * g + 1] = js[1]; st[3 * g + 2] = js[2];
    if (env.plane_slot) {   // plane cache: the flipped pair's fresh |U|^2 (in the spares) become current
      int32_t* s = env.plane_slot + (size_t)b * (CH + 2);
      const int pa = g * P + (jb.flip_plane & ~1);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int32_t cur = s[pa + i];
        s[pa + i] = s[CH + i];
        s[CH + i] = cur;
      }
    }
    env.max_psnr_diff[b] = fmax(env.max_psnr_diff[b], diff);     // env.py:198
    const double sr = (double)flips / (double)steps;              // env.py:200
    env.prev_psnr[b] = psnr_after;                                // env.py:214
    int64_t sus = env.sustained[b];
    // env_group.py:292-315: linear in the step count instead of the cubic in sr
    const double lin = 100.0 + (-200.0 / 1500.0) * (double)(steps - 1000);
    if (diff >= tpd || (psnr_after >= prm.t_psnr && diff < 0.1)) {
      sus += 1;                                                   // env.py:225
      if (sus >= prm.t_steps && diff >= tpd) reward += importance ? lin : success_cubic(sr, 595.2);
    }
    env.sustained[b] = sus;
    if (steps >= prm.max_steps)                                   // env.py:249-254
      reward += importance ? lin : success_cubic(sr, 595.24);
    term = steps >= prm.max_steps || sus >= prm.t_steps;                // env.py:257
    trunc = steps >= prm.max_steps;                                     // env.py:258
  }
  env.flip_count[b] = flips;
  if (reward_out) reward_out[b] = reward;
  if (psnr_out) psnr_out[b] = psnr_after;
  if (acc_out) acc_out[b] = reject ? 0 : 1;
  if (term_out) term_out[b] = term ? 1 : 0;
  if (trunc_out) trunc_out[b] = trunc ? 1 : 0;
  if (accept_flag) accept_flag[b] = reject ? 0 : 1;
  if (env.recon_pending) env.recon_pending[b] = reject ? -(g + 1) : (g + 1);
}

// env_group.py:254-255: reward = importance_ranks[argmin |psnr_change_list -
// change|] (first index on ties, as np.argmin), one block per env
__global__ void k_importance_reward(const double* __restrict__ delta, const double* __restrict__ changes,
                                    const double* __restrict__ values, int K, int n,
                                    double* __restrict__ reward) {
  const int b = blockIdx.x;
  if (b >= n) return;
  const double c = delta[b];
  if (c != c) return;   // invalid job
  const double* lst = changes + (size_t)b * K;
  double best = INFINITY;
  int bi = K;
  for (int i = threadIdx.x; i < K; i += blockDim.x) {
    const double d = fabs(lst[i] - c);
    if (d < best) { best = d; bi = i; }   // i increases: first index kept on ties
  }
  __shared__ double sd[256];
  __shared__ int si[256];
  sd[threadIdx.x] = best;
  si[threadIdx.x] = bi;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const double d2 = sd[threadIdx.x + o];
      const int i2 = si[threadIdx.x + o];
      if (d2 < sd[threadIdx.x] || (d2 == sd[threadIdx.x] && i2 < si[threadIdx.x])) {
        sd[threadIdx.x] = d2;
        si[threadIdx.x] = i2;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && si[0] < K) reward[b] += values[(size_t)b * K + si[0]];
}

// DBS primitive: accept iff rule, no reward bookkeeping
__global__ void k_dbs_step_finalize(const JobDesc* __restrict__ jobs,
                                    const double* __restrict__ job_stats, int n, int G, int P,
                                    int H, int W, uint64_t* __restrict__ mask,
                                    double* __restrict__ chan_stats, double* __restrict__ prev,
                                    double* __restrict__ psnr_out, uint8_t* __restrict__ acc_out,
                                    int accept_rule, double count, int rel_scale, double peak) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const JobDesc jb = jobs[b];
  if (jb.env < 0) {
    if (psnr_out) psnr_out[b] = prev[b];
    if (acc_out) acc_out[b] = 0;
    return;
  }
  const int g = jb.group, CH = G * P, ch = g * P + jb.flip_plane;
  double* st = chan_stats + (size_t)b * G * 3;
  const double* js = job_stats + 3 * (size_t)b;
  double sxy = 0.0, sxx = 0.0, syy = 0.0;
  for (int gg = 0; gg < G; ++gg) {
    if (gg == g) { sxy += js[0]; sxx += js[1]; syy += js[2]; }
    else { sxy += st[3 * gg]; sxx += st[3 * gg + 1]; syy += st[3 * gg + 2]; }
  }
  const double ps = psnr_from(sxy, sxx, syy, count, rel_scale, peak);
  const double change = ps - prev[b];
  const bool ok = (accept_rule == 0) ? !(change < 0.0) : (change > 0.0);
  if (ok) {
    mask[((size_t)b * CH + ch) * (size_t)H * (W / 64) + (size_t)(jb.flip_pix / W) * (W / 64) +
         (jb.flip_pix % W) / 64] ^= (1ull << ((jb.flip_pix % W) & 63));
    st[3 * g] = js[0]; st[3 * g + 1] = js[1]; st[3 * g + 2] = js[2];
    prev[b] = ps;
  }
  if (psnr_out) psnr_out[b] = ps;
  if (acc_out) acc_out[b] = ok ? 1 : 0;
}

// probe / speculative candidates against one base env
__global__ void k_eval_finalize(const JobDesc* __restrict__ jobs, const double* __restrict__ job_stats,
                                int K, int G, const double* __restrict__ base_stats,
                                double* __restrict__ psnr_out, double* __restrict__ group_stats,
                                double count, int rel_scale, double peak) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const JobDesc jb = jobs[k];
  const double* js = job_stats + 3 * (size_t)k;
  if (jb.env < 0) {
    psnr_out[k] = NAN;
    if (group_stats) { group_stats[3 * k] = 0.0; group_stats[3 * k + 1] = 0.0; group_stats[3 * k + 2] = 0.0; }
    return;
  }
  double sxy = 0.0, sxx = 0.0, syy = 0.0;
  for (int gg = 0; gg < G; ++gg) {
    if (gg == jb.group) { sxy += js[0]; sxx += js[1]; syy += js[2]; }
    else { sxy += base_stats[3 * gg]; sxx += base_stats[3 * gg + 1]; syy += base_stats[3 * gg + 2]; }
  }
  psnr_out[k] = psnr_from(sxy, sxx, syy, count, rel_scale, peak);
  if (group_stats) { group_stats[3 * k] = js[0]; group_stats[3 * k + 1] = js[1]; group_stats[3 * k + 2] = js[2]; }
}

__global__ void k_commit_flip(uint64_t* __restrict__ mask, double* __restrict__ base_stats,
                              double* __restrict__ prev, const int64_t* __restrict__ flips,
                              const double* __restrict__ psnr, const double* __restrict__ gstats,
                              const int32_t* __restrict__ kp, int K, int G, int P, int H, int W,
                              int32_t* __restrict__ plane_slot) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int k = *kp;
  if (k < 0 || k >= K) return;
  const int64_t a = flips[k];
  const int64_t hw = (int64_t)H * W;
  if (a < 0 || a >= (int64_t)G * P * hw) return;
  const int ch = (int)(a / hw);
  const int pix = (int)(a % hw);
  const int g = ch / P;
  mask[(size_t)ch * H * (W / 64) + (size_t)(pix / W) * (W / 64) + (pix % W) / 64] ^=
      (1ull << ((pix % W) & 63));
  base_stats[3 * g] = gstats[3 * k];
  base_stats[3 * g + 1] = gstats[3 * k + 1];
  base_stats[3 * g + 2] = gstats[3 * k + 2];
  *prev = psnr[k];
  if (plane_slot) {   // plane cache (ABI v10): candidate k's fresh pair (spare pair k) becomes current
    const int CH = G * P, pa = g * P + ((ch % P) & ~1);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int32_t cur = plane_slot[pa + i];
      plane_slot[pa + i] = plane_slot[CH + 2 * k + i];
      plane_slot[CH + 2 * k + i] = cur;
    }
  }
}

// Device-decided greedy DBS in the FFT mode with the base state's plane cache (ABI v10,
// hbx_dbs_walk_planes): the decision (hbx_walk_planes.hpp walk_planes_decide) in a launch of its
// own -- each call's first batch of jobs (decide = 0).  Since r05 the per-batch decision runs in
// the last-arriving workgroup of the batch's k_rowinv_d launch instead (one launch per batch less).
__global__ void k_walk_planes(WalkPlanesArgs a, int decide) {
  __shared__ __attribute__((aligned(16))) char lds[walk_planes_lds_bytes(128)];
  walk_planes_decide<false>(a, decide, lds);
}

hipError_t launch_walk_planes(const WalkPlanesArgs& a, int decide, hipStream_t st) {
  if (a.RB > 128 || a.K > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_walk_planes, dim3(1), dim3(256), 0, st, a, decide);
  return hipGetLastError();
}

// zero record planes of reset envs
__global__ void k_zero_record(int8_t* __restrict__ record, const int32_t* __restrict__ env_ids,
                              int n_ids, size_t per_env) {
  const size_t n16 = per_env / 16;
  const int i = blockIdx.y;
  if (i >= n_ids) return;
  const int e = env_ids ? env_ids[i] : i;
  uint4* base = reinterpret_cast<uint4*>(record + (size_t)e * per_env);
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < n16; k += (size_t)gridDim.x * blockDim.x)
    base[k] = make_uint4(0, 0, 0, 0);
}

// copy job intensities [n_jobs][H][W] into the env cache [B][G][H][W] (full or accepted steps)
__global__ void k_scatter_intensity(const JobDesc* __restrict__ jobs, const float* __restrict__ src,
                                    float* __restrict__ cache, int G, size_t hw,
                                    const int32_t* __restrict__ accept_flag) {
  const int j = blockIdx.y;
  const JobDesc jb = jobs[j];
  if (jb.env < 0) return;
  if (accept_flag && accept_flag[j] == 0) return;
  const float4* s = reinterpret_cast<const float4*>(src + (size_t)j * hw);
  float4* d = reinterpret_cast<float4*>(cache + ((size_t)jb.env * G + jb.group) * hw);
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < hw / 4; k += (size_t)gridDim.x * blockDim.x)
    d[k] = s[k];
}

// obs["recon_image"] (ABI v8): the previous step left its group's stepped intensity in
// recon[b][g]; before this step overwrites a group, make the two caches agree again --
// accepted (+g+1): intensity[b][g] <- recon[b][g]; rolled back (-(g+1)): recon[b][g] <-
// intensity[b][g] (env.py:191-196 restores the state; the obs of the NEXT step shows the
// restored means of the groups it does not touch).  grid (x, n envs)
__global__ void k_recon_reconcile(const int32_t* __restrict__ pending, float* __restrict__ recon,
                                  float* __restrict__ intensity, int G, size_t hw) {
  const int b = blockIdx.y;
  const int p = pending[b];
  if (p == 0) return;
  const int g = (p > 0 ? p : -p) - 1;
  const size_t off = ((size_t)b * G + g) * hw;
  const float4* s = reinterpret_cast<const float4*>((p > 0 ? recon : intensity) + off);
  float4* d = reinterpret_cast<float4*>((p > 0 ? intensity : recon) + off);
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < hw / 4; k += (size_t)gridDim.x * blockDim.x)
    d[k] = s[k];
}

// rebuild the observation mirrors of listed envs: state_bytes from the mask bits (one
// 64-bit word -> 64 bytes per thread), recon <- intensity (pending cleared by k_pending_clear
// after this launch: every block of an env reads pending first).  resolve (HBX_OBS_RESOLVE):
// an accepted step's pending reconcile (pending = g + 1: recon holds group g's new intensity,
// the intensity cache the old one) is applied first, i.e. group g goes recon -> intensity; without
// it intensity is authoritative (reset / checkpoint load rewrote it).  grid (x, n_ids)
__global__ void k_obs_sync(const int32_t* __restrict__ env_ids, const uint64_t* __restrict__ mask,
                           int8_t* __restrict__ state_bytes, float* __restrict__ intensity,
                           float* __restrict__ recon, const int32_t* __restrict__ pending, int resolve, int CH,
                           int G, size_t hw) {
  const int i = blockIdx.y;
  const int e = env_ids ? env_ids[i] : i;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t t0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (state_bytes) {
    const size_t words = (size_t)CH * hw / 64;
    const uint64_t* m = mask + (size_t)e * words;
    uint4* o = reinterpret_cast<uint4*>(state_bytes + (size_t)e * CH * hw);
    for (size_t w = t0; w < words; w += stride) {
      const uint64_t x = m[w];
      uint32_t q[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {    // bytes 4k .. 4k+3 = bits 4k .. 4k+3
        const uint32_t n = (uint32_t)(x >> (4 * k)) & 0xfu;
        q[k] = (n & 1u) | ((n & 2u) << 7) | ((n & 4u) << 14) | ((n & 8u) << 21);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) o[4 * w + k] = make_uint4(q[4 * k], q[4 * k + 1], q[4 * k + 2], q[4 * k + 3]);
    }
  }
  if (recon) {
    const int p = (resolve && pending) ? pending[e] : 0;
    const size_t gacc = p > 0 ? (size_t)(p - 1) : (size_t)G;     // G: no group goes recon -> intensity
    float4* in4 = reinterpret_cast<float4*>(intensity + (size_t)e * G * hw);
    float4* rc4 = reinterpret_cast<float4*>(recon + (size_t)e * G * hw);
    for (size_t k = t0; k < (size_t)G * hw / 4; k += stride) {
      if (k / (hw / 4) == gacc) in4[k] = rc4[k];
      else rc4[k] = in4[k];
    }
  }
}
// HBX_OBS_SETTLE: an accepted last step's group recon -> intensity (recon untouched); then
// k_pending_settled clears those pendings (a separate launch: every block of k_obs_settle reads
// the pending word first).  grid (x, n_ids)
__global__ void k_obs_settle(const int32_t* __restrict__ env_ids, float* __restrict__ intensity,
                             const float* __restrict__ recon, const int32_t* __restrict__ pending, int G,
                             size_t hw) {
  const int e = env_ids ? env_ids[blockIdx.y] : (int)blockIdx.y;
  const int p = pending[e];
  if (p <= 0) return;
  const size_t off = ((size_t)e * G + (p - 1)) * hw / 4;
  const float4* src = reinterpret_cast<const float4*>(recon) + off;
  float4* dst = reinterpret_cast<float4*>(intensity) + off;
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < hw / 4; k += (size_t)gridDim.x * blockDim.x)
    dst[k] = src[k];
}
__global__ void k_pending_settled(const int32_t* __restrict__ env_ids, int n_ids, int32_t* __restrict__ pending) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ids) return;
  const int e = env_ids ? env_ids[i] : i;
  if (pending[e] > 0) pending[e] = 0;
}
__global__ void k_pending_clear(const int32_t* __restrict__ env_ids, int n_ids, int32_t* __restrict__ pending) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_ids) pending[env_ids ? env_ids[i] : i] = 0;
}

// psnr from chan_stats
__global__ void k_psnr(const double* __restrict__ chan_stats, int n, int G, double* __restrict__ psnr,
                       double count, int rel_scale, double peak) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  double sxy = 0.0, sxx = 0.0, syy = 0.0;
  for (int g = 0; g < G; ++g) {
    const double* s = chan_stats + ((size_t)b * G + g) * 3;
    sxy += s[0]; sxx += s[1]; syy += s[2];
  }
  psnr[b] = psnr_from(sxy, sxx, syy, count, rel_scale, peak);
}

hipError_t launch_jobs_from_actions(const int64_t* actions, int n, int H, int W, int P, int CH,
                                    JobDesc* jobs, int32_t* err, hipStream_t st) {
  hipLaunchKernelGGL(k_jobs_from_actions, dim3((n + 127) / 128), dim3(128), 0, st, actions, n, H,
                     W, P, CH, jobs, err);
  return hipGetLastError();
}
hipError_t launch_jobs_from_flips(const int64_t* flips, int K, int H, int W, int P, int CH,
                                  JobDesc* jobs, hipStream_t st) {
  hipLaunchKernelGGL(k_jobs_from_flips, dim3((K + 127) / 128), dim3(128), 0, st, flips, K, H, W, P,
                     CH, jobs);
  return hipGetLastError();
}
hipError_t launch_job_from_flip_k(const int64_t* flips, const int32_t* k, int K, int H, int W, int P, int CH,
                                  JobDesc* jobs, int32_t* order, int32_t* accept, hipStream_t st) {
  hipLaunchKernelGGL(k_job_from_flip_k, dim3(1), dim3(1), 0, st, flips, k, K, H, W, P, CH, jobs, order, accept);
  return hipGetLastError();
}
hipError_t launch_jobs_full(const int32_t* env_ids, int n_ids, int G, JobDesc* jobs, hipStream_t st) {
  const int n = n_ids * G;
  hipLaunchKernelGGL(k_jobs_full, dim3((n + 127) / 128), dim3(128), 0, st, env_ids, n_ids, G, jobs);
  return hipGetLastError();
}
hipError_t launch_full_finalize(const JobDesc* jobs, const double* job_stats, int n_ids, int G,
                                double* chan_stats, double* psnr, double count, int rel, double peak,
                                const EnvDev& env, int reset, hipStream_t st) {
  hipLaunchKernelGGL(k_full_finalize, dim3((n_ids + 63) / 64), dim3(64), 0, st, jobs, job_stats,
                     n_ids, G, chan_stats, psnr, count, rel, peak, env, reset);
  return hipGetLastError();
}
hipError_t launch_env_step_finalize(const JobDesc* jobs, const double* job_stats, int n, int G,
                                    int P, int H, int W, const EnvDev& env, const EnvParams& prm,
                                    double count, int rel, double peak, double* reward, double* psnr,
                                    uint8_t* acc, uint8_t* term, uint8_t* trunc, int32_t* accept_flag,
                                    double* delta_scratch, hipStream_t st, const double* partial, int RB) {
  const bool imp = prm.reward_kind == 1 && reward && env.imp_changes && env.imp_values && env.imp_count > 0;
  hipLaunchKernelGGL(k_env_step_finalize, dim3(partial ? n : (n + 63) / 64), dim3(64), 0, st, jobs, job_stats, n,
                     G, P, H, W, env, prm, count, rel, peak, reward, psnr, acc, term, trunc,
                     accept_flag, imp ? delta_scratch : nullptr, partial, RB);
  if (imp)
    hipLaunchKernelGGL(k_importance_reward, dim3(n), dim3(256), 0, st, delta_scratch, env.imp_changes,
                       env.imp_values, env.imp_count, n, reward);
  return hipGetLastError();
}
hipError_t launch_dbs_step_finalize(const JobDesc* jobs, const double* job_stats, int n, int G, int P,
                                    int H, int W, uint64_t* mask, double* chan_stats, double* prev,
                                    double* psnr, uint8_t* acc, int rule, double count, int rel,
                                    double peak, hipStream_t st) {
  hipLaunchKernelGGL(k_dbs_step_finalize, dim3((n + 63) / 64), dim3(64), 0, st, jobs, job_stats, n, G,
                     P, H, W, mask, chan_stats, prev, psnr, acc, rule, count, rel, peak);
  return hipGetLastError();
}
hipError_t launch_eval_finalize(const JobDesc* jobs, const double* job_stats, int K, int G,
                                const double* base_stats, double* psnr, double* gstats, double count,
                                int rel, double peak, hipStream_t st) {
  hipLaunchKernelGGL(k_eval_finalize, dim3((K + 63) / 64), dim3(64), 0, st, jobs, job_stats, K, G,
                     base_stats, psnr, gstats, count, rel, peak);
  return hipGetLastError();
}
hipError_t launch_commit_flip(uint64_t* mask, double* stats, double* prev, const int64_t* flips,
                              const double* psnr, const double* gstats, const int32_t* k, int K,
                              int G, int P, int H, int W, hipStream_t st, int32_t* plane_slot) {
  hipLaunchKernelGGL(k_commit_flip, dim3(1), dim3(64), 0, st, mask, stats, prev, flips, psnr, gstats,
                     k, K, G, P, H, W, plane_slot);
  return hipGetLastError();
}
hipError_t launch_zero_record(int8_t* record, const int32_t* env_ids, int n_ids, size_t per_env,
                              hipStream_t st) {
  hipLaunchKernelGGL(k_zero_record, dim3(64, n_ids), dim3(256), 0, st, record, env_ids, n_ids, per_env);
  return hipGetLastError();
}
hipError_t launch_scatter_intensity(const JobDesc* jobs, int n_jobs, const float* src, float* cache,
                                    int G, size_t hw, const int32_t* accept_flag, hipStream_t st) {
  hipLaunchKernelGGL(k_scatter_intensity, dim3(64, n_jobs), dim3(256), 0, st, jobs, src, cache, G, hw,
                     accept_flag);
  return hipGetLastError();
}
hipError_t launch_recon_reconcile(const int32_t* pending, float* recon, float* intensity, int n, int G,
                                  size_t hw, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_recon_reconcile, dim3(32, n), dim3(256), 0, st, pending, recon, intensity, G, hw);
  return hipGetLastError();
}
// plane cache (ABI v9): identity slots of the listed envs (the fill pass writes plane i to slot i,
// the spares are slots CH and CH + 1)
__global__ void k_plane_slot_init(const int32_t* __restrict__ env_ids, int n_ids, int32_t* __restrict__ slot,
                                  int CHS) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ids * CHS) return;
  const int k = i / CHS, c = i % CHS;
  const int e = env_ids ? env_ids[k] : k;
  slot[(size_t)e * CHS + c] = c;
}

hipError_t launch_plane_slot_init(const int32_t* env_ids, int n_ids, int32_t* slot, int CHS, hipStream_t st) {
  const int n = n_ids * CHS;
  hipLaunchKernelGGL(k_plane_slot_init, dim3((n + 255) / 256), dim3(256), 0, st, env_ids, n_ids, slot, CHS);
  return hipGetLastError();
}

hipError_t launch_obs_sync(const int32_t* env_ids, int n_ids, const uint64_t* mask, int8_t* state_bytes,
                           float* intensity, float* recon, int32_t* pending, int resolve, int CH, int G, size_t hw,
                           hipStream_t st) {
  if (n_ids <= 0 || (!state_bytes && !recon)) return hipSuccess;
  hipLaunchKernelGGL(k_obs_sync, dim3(64, n_ids), dim3(256), 0, st, env_ids, mask, state_bytes, intensity, recon,
                     pending, resolve, CH, G, hw);
  if (recon && pending)
    hipLaunchKernelGGL(k_pending_clear, dim3((n_ids + 255) / 256), dim3(256), 0, st, env_ids, n_ids, pending);
  return hipGetLastError();
}
hipError_t launch_obs_settle(const int32_t* env_ids, int n_ids, float* intensity, const float* recon,
                             int32_t* pending, int G, size_t hw, hipStream_t st) {
  if (n_ids <= 0) return hipSuccess;
  const unsigned gx = (unsigned)std::min<size_t>(32, (hw / 4 + 255) / 256);
  hipLaunchKernelGGL(k_obs_settle, dim3(gx, n_ids), dim3(256), 0, st, env_ids, intensity, recon, pending, G, hw);
  hipLaunchKernelGGL(k_pending_settled, dim3((n_ids + 255) / 256), dim3(256), 0, st, env_ids, n_ids, pending);
  return hipGetLastError();
}
hipError_t launch_psnr(const double* chan_stats, int n, int G, double* psnr, double count, int rel,
                       double peak, hipStream_t st) {
  hipLaunchKernelGGL(k_psnr, dim3((n + 63) / 64), dim3(64), 0, st, chan_stats, n, G, psnr, count, rel,
                     peak);
  return hipGetLastError();
}

}  // namespace hbx
