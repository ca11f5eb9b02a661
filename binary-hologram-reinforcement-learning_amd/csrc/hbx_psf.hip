// hbx_psf.hip -- incremental-field ("PSF") mode kernels (gfx950).
//
// tt.simulate is linear in the field, so flipping pixel (c, r, col) of a mask
// whose plane-c field U_c is known changes only that plane:
//   U_c'(y, x) = U_c(y, x) + delta * h_g((y - r) mod N, (x - col) mod N)
//   I_g'(y, x) = I_g(y, x) + (|U_c'|^2 - |U_c|^2) / P
// with h_g = IFFT2(H_g) the field of a single unit pixel (computed once by
// the exact FFT path) and delta = vb * (1 - 2 bit_old) the change of the
// field value (amplitude: +-1, phase: -+2).  A step therefore streams U_c
// (8 B/px), I_g (4 B/px) and the target channel (4 B/px) once -- no FFT --
// and the relative-PSNR sums come out of the same pass as the flip's
// INCREMENTS sum dI T and sum (2 I + dI) dI (f64), added to the cached f64
// channel sums: the decision then carries the increment's own f32 precision
// (~1e-13 dB at 1024 x 24) instead of the rounding of a full-image sum.  h_g is even in x
// and y (H_g depends on fx^2 and fy^2), so only its quadrant [0, N/2]^2 is
// read (folded offsets): 2.1 MB per group at N = 1024, which stays in an
// XCD's 4-MB L2 when the launch visits the jobs grouped by colour group
// (k_psf_order) -- instead of 8 MB per job streamed from the Infinity Cache.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbx_internal.hpp"

namespace hbx {

namespace {

__device__ __forceinline__ float flip_delta(const uint64_t* mask, const JobDesc& jb, int N, int P,
                                            int CH, float vb, bool after_flip) {
  const int c = jb.group * P + jb.flip_plane;
  const int r = jb.flip_pix / N, col = jb.flip_pix % N;
  const uint64_t w = mask[(((size_t)jb.env * CH + c) * N + r) * (N / 64) + col / 64];
  const int bit = (int)((w >> (col & 63)) & 1ull);
  // before the flip: delta = vb (1 - 2 bit_old); after it: bit_new = 1 - bit_old
  return after_flip ? vb * (float)(2 * bit - 1) : vb * (float)(1 - 2 * bit);
}

// |d| mod N folded into [0, N/2] (h is even in each coordinate)
__device__ __forceinline__ int fold(int d, int N) {
  d = (N & (N - 1)) ? ((d % N) + N) % N : (d & (N - 1));   // N = 896 is not a power of 2
  return d <= N / 2 ? d : N - d;
}

template <int BLK>
__device__ __forceinline__ void block_sum2(double& a, double& b, double (*red)[2]) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    b += __shfl_xor(b, off, 64);
  }
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) { red[w][0] = a; red[w][1] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    a = 0.0; b = 0.0;
    for (int i = 0; i < BLK / 64; ++i) { a += red[i][0]; b += red[i][1]; }
  }
}

}  // namespace

// stable counting sort of the jobs by colour group (one block of 256 threads):
// launches then visit one group's jobs after another, so h_g stays L2-resident.
// Job j goes to (jobs of smaller groups) + (jobs of its group before it), both
// from per-wave ballots over chunks of 256 jobs -- the order of the serial
// sort, without its 2 * n_jobs dependent loads (34 us per 128-job step as one
// thread, rocprofv3 profiles/r02_final4/kernel_stats.csv).  Jobs without an env
// count as group 0, as before.
// With actions != nullptr the same launch first decodes the env-step actions into the
// jobs (k_jobs_from_actions' rule, env.py:157-161), saving the env step one launch.
__global__ __launch_bounds__(256) void k_psf_order(JobDesc* __restrict__ jobs, int n_jobs, int G,
                                                   int32_t* __restrict__ order, const int64_t* __restrict__ actions,
                                                   int N, int P, int32_t* __restrict__ err) {
  constexpr int W = 256 / 64;
  __shared__ int wc[W][8];   // this chunk's jobs per wave and group
  __shared__ int run[8];     // jobs per group in the chunks before this one
  __shared__ int base[8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  for (int pass = 0; pass < 2; ++pass) {
    if (threadIdx.x < 8) run[threadIdx.x] = 0;
    __syncthreads();
    for (int c0 = 0; c0 < n_jobs; c0 += 256) {
      const int j = c0 + (int)threadIdx.x;
      int g = -1;
      if (j < n_jobs) {
        if (actions) {   // decode (both passes: registers only; the jobs are written once)
          const int64_t a = actions[j];
          const int64_t hw = (int64_t)N * N;
          JobDesc jd;
          if (a < 0 || a >= (int64_t)G * P * hw) {
            jd.env = -1; jd.group = 0; jd.flip_plane = -1; jd.flip_pix = 0;
            if (pass == 0 && err) atomicOr(err, 1);
          } else {
            const int ch = (int)(a / hw);
            jd.env = j; jd.group = ch / P; jd.flip_plane = ch % P; jd.flip_pix = (int)(a % hw);
          }
          if (pass == 0) jobs[j] = jd;
          g = jd.group;
        } else {
          g = jobs[j].env >= 0 ? jobs[j].group : 0;
        }
      }
      int mine = 0;
      for (int gg = 0; gg < G; ++gg) {
        const uint64_t m = __ballot(g == gg);
        if (lane == 0) wc[w][gg] = __popcll(m);
        if (g == gg) mine = __popcll(m & below);
      }
      __syncthreads();
      if (pass == 1 && g >= 0) {
        int pos = base[g] + run[g] + mine;
        for (int ww = 0; ww < w; ++ww) pos += wc[ww][g];
        order[pos] = j;
      }
      __syncthreads();
      if ((int)threadIdx.x < G) {
        int s = 0;
        for (int ww = 0; ww < W; ++ww) s += wc[ww][threadIdx.x];
        run[threadIdx.x] += s;
      }
      __syncthreads();
    }
    if (pass == 0 && threadIdx.x == 0) {
      int acc = 0;
      for (int gg = 0; gg < G; ++gg) { base[gg] = acc; acc += run[gg]; }
    }
    __syncthreads();
  }
}

// grid (kPsfBlocks, n_jobs); each thread walks single pixels
__global__ __launch_bounds__(256) void k_psf_eval(const JobDesc* __restrict__ jobs,
                                                  const int32_t* __restrict__ order,
                                                  const uint64_t* __restrict__ mask,
                                                  const float2* __restrict__ field,
                                                  const float* __restrict__ inten,
                                                  const float* __restrict__ target,
                                                  const float2* __restrict__ hpsf, int N, int P,
                                                  int G, float vb, double* __restrict__ partial) {
  __shared__ double red[4][2];
  const int j = order[blockIdx.y];
  const JobDesc jb = jobs[j];
  double sxy = 0.0, sxx = 0.0;
  if (jb.env >= 0) {
    const int CH = G * P;
    const int g = jb.group;
    const int r = jb.flip_pix / N, col = jb.flip_pix % N;
    const float delta = flip_delta(mask, jb, N, P, CH, vb, false);
    const float invp = 1.0f / (float)P;
    const size_t hw = (size_t)N * N;
    const float2* h = hpsf + (size_t)g * hw;
    // one pixel per lane: the shifted h reads coalesce per wave (measured 0.457 -> 0.445 and
    // 0.427 -> 0.419 ms per 128-job launch against four pixels per lane, r01)
    const float2* U2 = field + ((size_t)jb.env * CH + g * P + jb.flip_plane) * hw;
    const float* I1 = inten + ((size_t)jb.env * G + g) * hw;
    const float* T1 = target + ((size_t)jb.env * G + g) * hw;
    const int npx = (int)hw;
#pragma unroll 4
    for (int q = blockIdx.x * 256 + threadIdx.x; q < npx; q += kPsfBlocks * 256) {
      const int y = q / N, x = q % N;
      // the once-read streams are non-temporal, so they do not push h_g out of the L2:
      // measured 0.409 -> 0.367 ms per 128-job launch
      typedef float f2v __attribute__((ext_vector_type(2)));
      const f2v uv = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(U2 + q));
      const float2 u = make_float2(uv.x, uv.y);
      const float iv = __builtin_nontemporal_load(I1 + q), tv = __builtin_nontemporal_load(T1 + q);
      const float2 hv = h[(size_t)fold(y - r, N) * N + fold(x - col, N)];
      const float dI = flip_dI(u.x, u.y, hv.x, hv.y, delta, invp);
      sxy = fma((double)dI, (double)tv, sxy);
      sxx = fma((double)fmaf(2.0f, iv, dI), (double)dI, sxx);
    }
  }
  block_sum2<256>(sxy, sxx, red);
  if (threadIdx.x == 0) {
    double* o = partial + ((size_t)j * kPsfBlocks + blockIdx.x) * 2;
    o[0] = sxy; o[1] = sxx;
  }
}

// fixed-order reduction of the block partials (the flip's increments of sum IT
// and sum I^2) added to the cached channel statistics; sum T^2 of the touched
// channel is unchanged by a flip
// grid (n_jobs), one wave per job: coalesced staging of the block partials in LDS, then
// lane 0 adds them in block order (as k_reduce_partials)
__global__ __launch_bounds__(64) void k_psf_reduce(const JobDesc* __restrict__ jobs, const double* __restrict__ partial,
                                                   int n_jobs, int G, const double* __restrict__ chan_stats,
                                                   double* __restrict__ job_stats) {
  __shared__ double s[2 * kPsfBlocks];
  const int j = blockIdx.x;
  if (j >= n_jobs) return;
  const double* p = partial + (size_t)j * kPsfBlocks * 2;
  for (int i = threadIdx.x; i < 2 * kPsfBlocks; i += 64) s[i] = p[i];
  __syncthreads();
  // lanes 0 and 1 carry the two sums, each in block order; lane 0 then writes both
  double acc = 0.0;
  if (threadIdx.x < 2) {
#pragma unroll 8
    for (int i = threadIdx.x; i < 2 * kPsfBlocks; i += 2) acc += s[i];
  }
  const double b = __shfl(acc, 1, 64);
  if (threadIdx.x != 0) return;
  const double a = acc;
  const JobDesc jb = jobs[j];
  if (jb.env < 0) {
    job_stats[3 * j] = job_stats[3 * j + 1] = job_stats[3 * j + 2] = 0.0;
    return;
  }
  // the partials are the flip's increments; the flipped group's sums are base + increment
  const double* base = chan_stats + ((size_t)jb.env * G + jb.group) * 3;
  job_stats[3 * j] = base[0] + a;
  job_stats[3 * j + 1] = base[1] + b;
  job_stats[3 * j + 2] = base[2];
}

// accepted envs: rewrite U_c and I_g (the mask bit is already flipped)
__global__ __launch_bounds__(256) void k_psf_commit(const JobDesc* __restrict__ jobs,
                                                    const int32_t* __restrict__ order,
                                                    const uint64_t* __restrict__ mask,
                                                    float2* __restrict__ field,
                                                    float* __restrict__ inten,
                                                    const float2* __restrict__ hpsf,
                                                    const int32_t* __restrict__ accept_flag, int N,
                                                    int P, int G, float vb) {
  const int j = order[blockIdx.y];
  const JobDesc jb = jobs[j];
  if (jb.env < 0 || accept_flag[j] == 0) return;
  const int CH = G * P;
  const int g = jb.group;
  const int r = jb.flip_pix / N, col = jb.flip_pix % N;
  const float delta = flip_delta(mask, jb, N, P, CH, vb, true);
  const float invp = 1.0f / (float)P;
  const size_t hw = (size_t)N * N;
  const float2* h = hpsf + (size_t)g * hw;
  // one pixel per lane, as k_psf_eval (coalesced shifted-h reads): 0.292 -> 0.287 ms per
  // 128-job step against four pixels per lane (profiles/r02/psf_commit_px1_ab.txt)
  float2* U2 = field + ((size_t)jb.env * CH + g * P + jb.flip_plane) * hw;
  float* I1 = inten + ((size_t)jb.env * G + g) * hw;
#pragma unroll 4
  for (int q = blockIdx.x * 256 + threadIdx.x; q < (int)hw; q += kPsfBlocks * 256) {
    const int y = q / N, x = q % N;
    float2 u = U2[q];
    float iv = I1[q];
    const float2 hv = h[(size_t)fold(y - r, N) * N + fold(x - col, N)];
    iv += flip_dI(u.x, u.y, hv.x, hv.y, delta, invp);
    u.x = fmaf(delta, hv.x, u.x);
    u.y = fmaf(delta, hv.y, u.y);
    U2[q] = u;
    I1[q] = iv;
  }
}

hipError_t launch_psf_eval(const PlanDev& pd, const JobDesc* jobs, int n_jobs, const uint64_t* mask,
                           const float2* field, const float* inten, const float* target,
                           const double* chan_stats, hipStream_t st, const int64_t* actions, int32_t* err) {
  PassTimer* tm = pd.timer;
  hipLaunchKernelGGL(k_psf_order, dim3(1), dim3(256), 0, st, const_cast<JobDesc*>(jobs), n_jobs, pd.G, pd.psf_order,
                     actions, pd.N, pd.P, err);
  if (tm) tm->begin(3, st);
  hipLaunchKernelGGL(k_psf_eval, dim3(kPsfBlocks, n_jobs), dim3(256), 0, st, jobs, pd.psf_order, mask, field, inten,
                     target, pd.hpsf, pd.N, pd.P, pd.G, pd.vb, pd.psf_partial);
  if (tm) tm->end(3, n_jobs, st);
  hipLaunchKernelGGL(k_psf_reduce, dim3(n_jobs), dim3(64), 0, st, jobs, pd.psf_partial,
                     n_jobs, pd.G, chan_stats, pd.job_stats);
  return hipGetLastError();
}

hipError_t launch_psf_commit(const PlanDev& pd, const JobDesc* jobs, int n_jobs, const uint64_t* mask,
                             float2* field, float* inten, const int32_t* accept_flag, hipStream_t st) {
  PassTimer* tm = pd.timer;
  if (tm) tm->begin(4, st);
  hipLaunchKernelGGL(k_psf_commit, dim3(kPsfBlocks, n_jobs), dim3(256), 0, st, jobs, pd.psf_order, mask, field, inten,
                     pd.hpsf, accept_flag, pd.N, pd.P, pd.G, pd.vb);
  if (tm) tm->end(4, n_jobs, st);
  return hipGetLastError();
}

}  // namespace hbx
