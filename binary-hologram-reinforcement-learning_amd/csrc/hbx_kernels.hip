// hbx_kernels.hip -- HIP kernels of the binary-hologram hot path (gfx950).
//
// One "job" = one colour group (P planes, N x N) of one env propagated with an
// optional single-pixel flip applied on the fly.  A job runs through three
// passes over a per-job workspace ws[job][P][N][N] (complex64, in place):
//
//   k_rowfwd  bits -> real row FFTs, two planes packed into one complex FFT,
//             Hermitian split, half spectrum (kx < N/2; Nyquist packed into
//             the imaginary part of kx = 0)                          [write N^2/2]
//   k_col     per strip of SW half-spectrum columns (LDS [N][SW+1]):
//             column FFT -> x H(kx,ky) (and the mirrored column N-kx
//             through Hermitian symmetry) -> two inverse column FFTs [read N^2/2, write N^2]
//   k_rowinv  per row, all P planes: inverse row FFT, |U|^2, plane mean,
//             f64 partial sums (I*T, I^2, T^2) against the target   [read N^2 + target]
//
// then tiny per-env kernels turn the partial sums into PSNR / reward /
// accept-rollback (env.py:154-259) on the device -- no host sync per step.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "hbx_fft.hpp"
#include "hbx_internal.hpp"

namespace hbx {

// ---------------------------------------------------------------------------
// Pass 1: forward row FFT of two bit-planes (real) packed as one complex FFT.
// Block = 256 threads = 256/R lane groups; group -> (job, plane pair, row).
// ---------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(256) void k_rowfwd(const JobDesc* __restrict__ jobs,
                                                const uint32_t* __restrict__ mask,
                                                float2* __restrict__ ws,
                                                const float2* __restrict__ tw_glob, int P,
                                                int CH, float va, float vb) {
  constexpr int N = R * R;
  constexpr int GPB = 256 / R;     // lane groups (rows) per block
  constexpr int WPR = N / 32;      // 32-bit words per mask row
  __shared__ float2 tw[N];
  __shared__ float2 scratch[GPB * R * (R + 1)];

  for (int i = threadIdx.x; i < N; i += 256) tw[i] = tw_glob[i];
  __syncthreads();

  const int grp = threadIdx.x / R;
  const int t = threadIdx.x % R;
  const int lane_base = (threadIdx.x & 63) - t;
  constexpr int RB = N / GPB;     // row blocks per plane pair
  int bid = blockIdx.x;
  const int rb = bid % RB;
  bid /= RB;
  const int q = bid % (P / 2);
  const int j = bid / (P / 2);
  const JobDesc jb = jobs[j];
  if (jb.env < 0) return;  // invalid job (uniform per block)
  const int y = rb * GPB + grp;
  const int pa = 2 * q, pb = 2 * q + 1;
  const int ca = jb.group * P + pa;

  const uint32_t* rowa = mask + ((size_t)jb.env * CH + ca) * N * WPR + (size_t)y * WPR;
  const uint32_t* rowb = rowa + (size_t)N * WPR;
  uint32_t wa[WPR], wb[WPR];
  if constexpr (WPR % 4 == 0) {
#pragma unroll
    for (int i = 0; i < WPR / 4; ++i) {
      const uint4 a = reinterpret_cast<const uint4*>(rowa)[i];
      const uint4 b = reinterpret_cast<const uint4*>(rowb)[i];
      wa[4 * i] = a.x; wa[4 * i + 1] = a.y; wa[4 * i + 2] = a.z; wa[4 * i + 3] = a.w;
      wb[4 * i] = b.x; wb[4 * i + 1] = b.y; wb[4 * i + 2] = b.z; wb[4 * i + 3] = b.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < WPR; ++i) { wa[i] = rowa[i]; wb[i] = rowb[i]; }
  }
  // on-the-fly single-pixel flip of this job (env.py:164)
  if (jb.flip_plane >= 0 && jb.flip_pix / N == y) {
    const int col = jb.flip_pix % N;
    const uint32_t bit = 1u << (col & 31);
#pragma unroll
    for (int i = 0; i < WPR; ++i) {
      if (i == (col >> 5)) {
        if (jb.flip_plane == pa) wa[i] ^= bit;
        if (jb.flip_plane == pb) wb[i] ^= bit;
      }
    }
  }
  float2 v[R];
#pragma unroll
  for (int jj = 0; jj < R; ++jj) {
    const int w = (R * jj) >> 5;
    const int sh = ((R * jj) & 31) + t;
    v[jj].x = fmaf(vb, (float)((wa[w] >> sh) & 1u), va);
    v[jj].y = fmaf(vb, (float)((wb[w] >> sh) & 1u), va);
  }
  PaddedScratch<R> sc{scratch + grp * R * (R + 1)};
  fft_group<R, false>(v, t, sc, tw);

  // Hermitian split: F_a = (Z + conj Z(-k))/2, F_b = -i (Z - conj Z(-k))/2
  float2* outa = ws + (((size_t)j * P + pa) * N + y) * N;
  float2* outb = outa + (size_t)N * N;
  const float2 zny = v[R / 2];  // Z[N/2] on lane 0
#pragma unroll
  for (int k2 = 0; k2 < R / 2; ++k2) {
    const float2 z = v[k2];
    const float2 m = mirror_conj<R>(v, k2, t, lane_base);
    float2 fa = make_float2(0.5f * (z.x + m.x), 0.5f * (z.y + m.y));
    float2 fb = make_float2(0.5f * (z.y - m.y), -0.5f * (z.x - m.x));
    if (k2 == 0 && t == 0) {  // DC and Nyquist are real: pack Nyquist in .y
      fa = make_float2(z.x, zny.x);
      fb = make_float2(z.y, zny.y);
    }
    outa[t + R * k2] = fa;
    outb[t + R * k2] = fb;
  }
}

// ---------------------------------------------------------------------------
// Pass 2: column pass on a strip of SW = 256/R half-spectrum columns.
// ---------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(256) void k_col(const JobDesc* __restrict__ jobs,
                                             float2* __restrict__ ws,
                                             const float2* __restrict__ htab,
                                             const float2* __restrict__ tw_glob, int P) {
  constexpr int N = R * R;
  constexpr int SW = 256 / R;         // columns per strip
  constexpr int PITCH = SW + 1;
  constexpr int NSTRIP = (N / 2) / SW;
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  float2* tw = smem;                  // [N]
  float2* strip = smem + N;           // [N][PITCH]

  int bid = blockIdx.x;
  const int s = bid % NSTRIP;
  bid /= NSTRIP;
  const int p = bid % P;
  const int j = bid / P;
  const JobDesc jb = jobs[j];
  if (jb.env < 0) return;
  const int x0 = s * SW;
  float2* plane = ws + ((size_t)j * P + p) * N * N;

  for (int i = threadIdx.x; i < N; i += 256) tw[i] = tw_glob[i];
  for (int i = threadIdx.x; i < N * SW; i += 256) {
    const int yy = i / SW, c = i % SW;
    strip[yy * PITCH + c] = plane[(size_t)yy * N + x0 + c];
  }
  __syncthreads();

  const int c = threadIdx.x / R;
  const int t = threadIdx.x % R;
  const int lane_base = (threadIdx.x & 63) - t;
  const int kx = x0 + c;
  float2 v[R];
#pragma unroll
  for (int jj = 0; jj < R; ++jj) v[jj] = strip[(t + R * jj) * PITCH + c];
  ColumnScratch<R, PITCH> sc{strip + c};
  fft_group<R, false>(v, t, sc, tw);

  const float2* hg = htab + (size_t)jb.group * (N / 2 + 1) * N;
  // kx != 0: G(kx) = F H(kx), G(N-kx) = conj F(kx,-ky) H(kx)   (H even in fx)
  // kx == 0: the packed column z = F(0,y) + i F(N/2,y) (both real sequences)
  //          splits into F(0) = (Z + M)/2 and F(N/2) = -i (Z - M)/2.
  // Branch-free so the lane shuffles never run under divergent control flow.
  const bool dc = (kx == 0);
  const float2* h1p = hg + (dc ? 0 : (size_t)kx * N);
  const float2* h2p = dc ? hg + (size_t)(N / 2) * N : h1p;
  float2 g1[R], g2[R];
#pragma unroll
  for (int k2 = 0; k2 < R; ++k2) {
    const float2 z = v[k2];
    const float2 m = mirror_conj<R>(v, k2, t, lane_base);
    const float2 a1 = dc ? make_float2(0.5f * (z.x + m.x), 0.5f * (z.y + m.y)) : z;
    const float2 a2 = dc ? make_float2(0.5f * (z.y - m.y), -0.5f * (z.x - m.x)) : m;
    g1[k2] = cmul(a1, h1p[t + R * k2]);
    g2[k2] = cmul(a2, h2p[t + R * k2]);
  }
  fft_group<R, true>(g1, t, sc, tw);
  fft_group<R, true>(g2, t, sc, tw);

  // direct columns: kx -> kx
#pragma unroll
  for (int k2 = 0; k2 < R; ++k2) strip[(t + R * k2) * PITCH + c] = g1[k2];
  __syncthreads();
  for (int i = threadIdx.x; i < N * SW; i += 256) {
    const int yy = i / SW, cc = i % SW;
    plane[(size_t)yy * N + x0 + cc] = strip[yy * PITCH + cc];
  }
  __syncthreads();
  // mirrored columns: kx -> N - kx (kx = 0 -> N/2)
#pragma unroll
  for (int k2 = 0; k2 < R; ++k2) strip[(t + R * k2) * PITCH + c] = g2[k2];
  __syncthreads();
  for (int i = threadIdx.x; i < N * SW; i += 256) {
    const int yy = i / SW, cc = i % SW;
    const int kk = x0 + cc;
    const int xm = (kk == 0) ? (N / 2) : (N - kk);
    plane[(size_t)yy * N + xm] = strip[yy * PITCH + cc];
  }
}

// ---------------------------------------------------------------------------
// Pass 3: inverse row FFT of all P planes of a row, |U|^2 plane mean and
// f64 partial sums against the target row.
// ---------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(256) void k_rowinv(const JobDesc* __restrict__ jobs,
                                                const float2* __restrict__ ws,
                                                const float* __restrict__ target,
                                                const float2* __restrict__ tw_glob, int P, int G,
                                                double* __restrict__ partial,
                                                float* __restrict__ inten_out) {
  constexpr int N = R * R;
  constexpr int GPB = 256 / R;
  constexpr int RB = N / GPB;
  __shared__ float2 tw[N];
  __shared__ float2 scratch[GPB * R * (R + 1)];
  __shared__ double red[GPB][3];

  for (int i = threadIdx.x; i < N; i += 256) tw[i] = tw_glob[i];
  __syncthreads();

  const int grp = threadIdx.x / R;
  const int t = threadIdx.x % R;
  const int rb = blockIdx.x % RB;
  const int j = blockIdx.x / RB;
  const JobDesc jb = jobs[j];
  if (jb.env < 0) {
    if (threadIdx.x == 0) {
      double* o = partial + ((size_t)j * RB + rb) * 3;
      o[0] = 0.0; o[1] = 0.0; o[2] = 0.0;
    }
    return;
  }
  const int y = rb * GPB + grp;
  PaddedScratch<R> sc{scratch + grp * R * (R + 1)};

  float acc[R];
#pragma unroll
  for (int k = 0; k < R; ++k) acc[k] = 0.0f;
  for (int p = 0; p < P; ++p) {
    const float2* row = ws + (((size_t)j * P + p) * N + y) * N;
    float2 v[R];
#pragma unroll
    for (int jj = 0; jj < R; ++jj) v[jj] = row[t + R * jj];
    fft_group<R, true>(v, t, sc, tw);
#pragma unroll
    for (int k = 0; k < R; ++k) acc[k] += norm2(v[k]);
  }
  const float invp = 1.0f / (float)P;
  const float* trow = target + (((size_t)jb.env * G + jb.group) * N + y) * N;
  double sxy = 0.0, sxx = 0.0, syy = 0.0;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const float I = acc[k] * invp;
    const float T = trow[t + R * k];
    sxy = fma((double)I, (double)T, sxy);
    sxx = fma((double)I, (double)I, sxx);
    syy = fma((double)T, (double)T, syy);
    acc[k] = I;
  }
  if (inten_out) {
    float* orow = inten_out + ((size_t)j * N + y) * N;
#pragma unroll
    for (int k = 0; k < R; ++k) orow[t + R * k] = acc[k];
  }
  // reduce over the R lanes of the group (fixed butterfly order -> deterministic)
#pragma unroll
  for (int off = R / 2; off >= 1; off >>= 1) {
    sxy += __shfl_xor(sxy, off, 64);
    sxx += __shfl_xor(sxx, off, 64);
    syy += __shfl_xor(syy, off, 64);
  }
  if (t == 0) { red[grp][0] = sxy; red[grp][1] = sxx; red[grp][2] = syy; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0, cc = 0.0;
    for (int g = 0; g < GPB; ++g) { a += red[g][0]; b += red[g][1]; cc += red[g][2]; }
    double* o = partial + ((size_t)j * RB + rb) * 3;
    o[0] = a; o[1] = b; o[2] = cc;
  }
}

// ---------------------------------------------------------------------------
// Small per-job / per-env kernels
// ---------------------------------------------------------------------------
__device__ __forceinline__ double psnr_from(double sxy, double sxx, double syy, double count,
                                            int rel_scale, double peak) {
  double mse;
  if (rel_scale == 1) mse = (sxx > 0.0) ? (syy - sxy * sxy / sxx) / count : syy / count;
  else mse = (sxx - 2.0 * sxy + syy) / count;
  if (!(mse > 0.0)) return INFINITY;
  return 10.0 * log10(peak * peak / mse);
}

// jobs from actions: one job per env (env.py:157-161 decode)
__global__ void k_jobs_from_actions(const int64_t* __restrict__ actions, int n, int H, int W,
                                    int P, int CH, JobDesc* __restrict__ jobs,
                                    int32_t* __restrict__ err) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const int64_t a = actions[b];
  const int64_t hw = (int64_t)H * W;
  JobDesc jd;
  if (a < 0 || a >= (int64_t)CH * hw) {
    jd.env = -1; jd.group = 0; jd.flip_plane = -1; jd.flip_pix = 0;
    if (err) atomicOr(err, 1);
  } else {
    const int ch = (int)(a / hw);
    jd.env = b;
    jd.group = ch / P;
    jd.flip_plane = ch % P;
    jd.flip_pix = (int)(a % hw);
  }
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
__global__ void k_reduce_partials(const double* __restrict__ partial, int n_jobs, int RB,
                                  double* __restrict__ job_stats) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_jobs) return;
  double a = 0.0, b = 0.0, c = 0.0;
  const double* p = partial + (size_t)j * RB * 3;
  for (int r = 0; r < RB; ++r) { a += p[3 * r]; b += p[3 * r + 1]; c += p[3 * r + 2]; }
  job_stats[3 * j] = a; job_stats[3 * j + 1] = b; job_stats[3 * j + 2] = c;
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
    double* d = chan_stats + ((size_t)e * G + g) * 3;
    d[0] = s[0]; d[1] = s[1]; d[2] = s[2];
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
                                    int32_t* __restrict__ accept_flag) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const JobDesc jb = jobs[b];
  if (jb.env < 0) {
    if (reward_out) reward_out[b] = 0.0;
    if (psnr_out) psnr_out[b] = env.prev_psnr[b];
    if (acc_out) acc_out[b] = 0;
    if (term_out) term_out[b] = 0;
    if (trunc_out) trunc_out[b] = 0;
    if (accept_flag) accept_flag[b] = 0;
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
  const double* js = job_stats + 3 * (size_t)b;
  double sxy = 0.0, sxx = 0.0, syy = 0.0;
  for (int gg = 0; gg < G; ++gg) {
    if (gg == g) { sxy += js[0]; sxx += js[1]; syy += js[2]; }
    else { sxy += st[3 * gg]; sxx += st[3 * gg + 1]; syy += st[3 * gg + 2]; }
  }
  const double psnr_after = psnr_from(sxy, sxx, syy, count, rel_scale, peak);
  const double change = psnr_after - env.prev_psnr[b];   // env.py:184
  const double diff = psnr_after - env.init_psnr[b];     // env.py:185
  double reward = change * prm.reward_weight;            // env.py:188
  const bool reject = (prm.accept_rule == 0) ? (change < 0.0) : !(change > 0.0);
  bool term = false, trunc = false;
  if (reject) {                                           // env.py:191-196
    flips -= 1;
  } else {
    env.mask[((size_t)b * CH + ch) * (size_t)H * (W / 64) + (size_t)(jb.flip_pix / W) * (W / 64) +
             (jb.flip_pix % W) / 64] ^= (1ull << ((jb.flip_pix % W) & 63));
    st[3 * g] = js[0]; st[3 * g + 1] = js[1]; st[3 * g + 2] = js[2];
    env.max_psnr_diff[b] = fmax(env.max_psnr_diff[b], diff);     // env.py:198
    const double sr = (double)flips / (double)steps;              // env.py:200
    env.prev_psnr[b] = psnr_after;                                // env.py:214
    int64_t sus = env.sustained[b];
    if (diff >= prm.t_psnr_diff || (psnr_after >= prm.t_psnr && diff < 0.1)) {
      sus += 1;                                                   // env.py:225
      if (sus >= prm.t_steps && diff >= prm.t_psnr_diff) reward += success_cubic(sr, 595.2);
    }
    env.sustained[b] = sus;
    if (steps >= prm.max_steps) reward += success_cubic(sr, 595.24);   // env.py:249-254
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
                              const int32_t* __restrict__ kp, int K, int G, int P, int H, int W) {
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

// ---------------------------------------------------------------------------
// Host-side launch helpers (called from hbx_api.cpp)
// ---------------------------------------------------------------------------
template <int R>
static hipError_t launch_passes(const PlanDev& pd, const JobDesc* jobs, int n_jobs,
                                const uint32_t* mask, const float* target, float* inten_out,
                                hipStream_t st) {
  constexpr int N = R * R;
  constexpr int GPB = 256 / R;
  constexpr int SW = 256 / R;
  const int P = pd.P;
  const int CH = pd.G * pd.P;
  PassTimer* tm = pd.timer;
  {
    const unsigned blocks = (unsigned)n_jobs * (P / 2) * (N / GPB);
    if (tm) tm->begin(0, st);
    hipLaunchKernelGGL(k_rowfwd<R>, dim3(blocks), dim3(256), 0, st, jobs, mask, pd.ws, pd.tw, P,
                       CH, pd.va, pd.vb);
    if (tm) tm->end(0, n_jobs, st);
  }
  {
    const unsigned blocks = (unsigned)n_jobs * P * ((N / 2) / SW);
    const size_t lds = (size_t)(N + N * (SW + 1)) * sizeof(float2);
    if (tm) tm->begin(1, st);
    hipLaunchKernelGGL(k_col<R>, dim3(blocks), dim3(256), lds, st, jobs, pd.ws, pd.htab, pd.tw, P);
    if (tm) tm->end(1, n_jobs, st);
  }
  {
    const unsigned blocks = (unsigned)n_jobs * (N / GPB);
    if (tm) tm->begin(2, st);
    hipLaunchKernelGGL(k_rowinv<R>, dim3(blocks), dim3(256), 0, st, jobs, pd.ws, target, pd.tw,
                       P, pd.G, pd.partial, inten_out);
    if (tm) tm->end(2, n_jobs, st);
  }
  {
    const int RB = N / GPB;
    hipLaunchKernelGGL(k_reduce_partials, dim3((n_jobs + 63) / 64), dim3(64), 0, st, pd.partial,
                       n_jobs, RB, pd.job_stats);
  }
  return hipGetLastError();
}

hipError_t run_jobs(const PlanDev& pd, const JobDesc* jobs, int n_jobs, const uint32_t* mask,
                    const float* target, float* inten_out, hipStream_t st) {
  switch (pd.R) {
    case 32: return launch_passes<32>(pd, jobs, n_jobs, mask, target, inten_out, st);
    case 16: return launch_passes<16>(pd, jobs, n_jobs, mask, target, inten_out, st);
    case 8: return launch_passes<8>(pd, jobs, n_jobs, mask, target, inten_out, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t col_kernel_lds(int R, size_t* bytes) {
  const int N = R * R, SW = 256 / R;
  *bytes = (size_t)(N + N * (SW + 1)) * sizeof(float2);
  hipError_t e = hipSuccess;
  switch (R) {
    case 32: e = hipFuncSetAttribute((const void*)k_col<32>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)*bytes); break;
    case 16: e = hipFuncSetAttribute((const void*)k_col<16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)*bytes); break;
    case 8: e = hipFuncSetAttribute((const void*)k_col<8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)*bytes); break;
    default: return hipErrorInvalidValue;
  }
  return e;
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
                                    hipStream_t st) {
  hipLaunchKernelGGL(k_env_step_finalize, dim3((n + 63) / 64), dim3(64), 0, st, jobs, job_stats, n,
                     G, P, H, W, env, prm, count, rel, peak, reward, psnr, acc, term, trunc,
                     accept_flag);
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
                              int G, int P, int H, int W, hipStream_t st) {
  hipLaunchKernelGGL(k_commit_flip, dim3(1), dim3(64), 0, st, mask, stats, prev, flips, psnr, gstats,
                     k, K, G, P, H, W);
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
hipError_t launch_psnr(const double* chan_stats, int n, int G, double* psnr, double count, int rel,
                       double peak, hipStream_t st) {
  hipLaunchKernelGGL(k_psnr, dim3((n + 63) / 64), dim3(64), 0, st, chan_stats, n, G, psnr, count, rel,
                     peak);
  return hipGetLastError();
}

}  // namespace hbx
