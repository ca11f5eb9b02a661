// hbx_generic.hip -- propagation of colour groups at N = 896 (the 64-pixel
// crop of a 1024 mask that env_1024_24_128.py:144-149 and
// DBS_1024_24-128.py:210-216 propagate).  896 = 28 x 32 is not a square of a
// power of two, so instead of the fused three-pass pipeline the propagation
// is composed from the transposing row-FFT kernel (k_fft_rt896, mixed-radix
// 28 x 32 lane-group FFT) and three elementwise kernels:
//   k_gen_prep    bits (+ the job's flip) -> field planes          [write 8 N^2 B / plane]
//   2-D FFT       two transposing row passes                      [2 x (8 + 8) N^2 B]
//   k_gen_tf      x H(kx, ky) / N^2 (H even in fx: half table)    [8 + 8 N^2 B]
//   inverse 2-D FFT                                               [2 x (8 + 8) N^2 B]
//   k_gen_reduce  |U|^2 plane mean, f64 partials of (I T, I^2, T^2) per row block,
//                 optional intensity / field outputs
// The job / partial / finalize interfaces are those of the fused path, so the
// env step, eval_flips, flip map and incremental mode all run unchanged.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbx_fft.hpp"
#include "hbx_internal.hpp"

namespace hbx {

namespace {

constexpr int kGenRows = 8;   // rows per reduce block (partial slots per job = N / 8)

__global__ void k_gen_prep(const JobDesc* __restrict__ jobs, const uint64_t* __restrict__ mask,
                           float2* __restrict__ X, int N, int P, int CH, float va, float vb) {
  const size_t hw = (size_t)N * N;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const int jp = blockIdx.y;        // job * P + plane
  if (i >= hw) return;
  const int j = jp / P, p = jp % P;
  const JobDesc jb = jobs[j];
  float2* o = X + (size_t)jp * hw;
  if (jb.env < 0) { o[i] = make_float2(0.f, 0.f); return; }
  const int y = (int)(i / N), x = (int)(i % N);
  const uint64_t w = mask[(((size_t)jb.env * CH + jb.group * P + p) * N + y) * (N / 64) + (x >> 6)];
  int bit = (int)((w >> (x & 63)) & 1ull);
  if (jb.flip_plane == p && jb.flip_pix == (int)i) bit ^= 1;        // env.py:164, on the fly
  o[i] = make_float2(fmaf(vb, (float)bit, va), 0.f);
}

// spectrum [ky][kx] (natural orientation after two transposing passes)
__global__ void k_gen_tf(const JobDesc* __restrict__ jobs, float2* __restrict__ X,
                         const float2* __restrict__ htab, int N, int P) {
  const size_t hw = (size_t)N * N;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const int jp = blockIdx.y;
  if (i >= hw) return;
  const JobDesc jb = jobs[jp / P];
  if (jb.env < 0) return;
  const int ky = (int)(i / N), kx = (int)(i % N);
  const int fx = kx <= N / 2 ? kx : N - kx;
  const float2 h = htab[((size_t)jb.group * (N / 2 + 1) + fx) * N + ky];
  X[(size_t)jp * hw + i] = cmul(X[(size_t)jp * hw + i], h);
}

// one block per (job, 8-row block): intensity, stats partials, optional outputs
__global__ __launch_bounds__(256) void k_gen_reduce(const JobDesc* __restrict__ jobs,
                                                    const float2* __restrict__ U,
                                                    const float* __restrict__ target, int N, int P, int G,
                                                    double* __restrict__ partial,
                                                    float* __restrict__ inten_out,
                                                    float2* __restrict__ field_out) {
  __shared__ double red[4][3];
  const int RB = N / kGenRows;
  const int rb = blockIdx.x % RB, j = blockIdx.x / RB;
  const JobDesc jb = jobs[j];
  const size_t hw = (size_t)N * N;
  double sxy = 0.0, sxx = 0.0, syy = 0.0;
  if (jb.env >= 0) {
    const float invp = 1.0f / (float)P;
    for (int e = threadIdx.x; e < kGenRows * N; e += 256) {
      const size_t i = (size_t)rb * kGenRows * N + e;
      float acc = 0.0f;
      for (int p = 0; p < P; ++p) {
        const float2 u = U[((size_t)j * P + p) * hw + i];
        acc = fmaf(u.x, u.x, fmaf(u.y, u.y, acc));
        if (field_out) field_out[(((size_t)jb.env * G + jb.group) * P + p) * hw + i] = u;
      }
      const float I = acc * invp;
      const float T = target ? target[((size_t)jb.env * G + jb.group) * hw + i] : 0.0f;
      sxy = fma((double)I, (double)T, sxy);
      sxx = fma((double)I, (double)I, sxx);
      syy = fma((double)T, (double)T, syy);
      if (inten_out) inten_out[(size_t)j * hw + i] = I;
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    sxy += __shfl_xor(sxy, off, 64);
    sxx += __shfl_xor(sxx, off, 64);
    syy += __shfl_xor(syy, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x / 64][0] = sxy; red[threadIdx.x / 64][1] = sxx; red[threadIdx.x / 64][2] = syy;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0, c = 0.0;
    for (int w = 0; w < 4; ++w) { a += red[w][0]; b += red[w][1]; c += red[w][2]; }
    double* o = partial + ((size_t)j * RB + rb) * 3;
    o[0] = a; o[1] = b; o[2] = c;
  }
}

}  // namespace

__global__ void k_reduce_partials(const double* __restrict__ partial, int n_jobs, int RB,
                                  double* __restrict__ job_stats);

hipError_t run_jobs_generic(const PlanDev& pd, const JobDesc* jobs, int n_jobs, const uint64_t* mask,
                            const float* target, float* inten_out, float2* field_out, hipStream_t st) {
  const int N = pd.N, P = pd.P, CH = pd.G * P;
  const size_t hw = (size_t)N * N;
  const unsigned pb = (unsigned)((hw + 255) / 256);
  const int planes = n_jobs * P;
  float2* X = pd.ws_a;
  float2* S = pd.ws_b;
  PassTimer* tm = pd.timer;
  if (tm) tm->begin(0, st);
  hipLaunchKernelGGL(k_gen_prep, dim3(pb, planes), dim3(256), 0, st, jobs, mask, X, N, P, CH, pd.va, pd.vb);
  hipError_t e = run_fft2d(pd, X, S, planes, false, st);
  if (tm) tm->end(0, n_jobs, st);
  if (e != hipSuccess) return e;
  if (tm) tm->begin(1, st);
  hipLaunchKernelGGL(k_gen_tf, dim3(pb, planes), dim3(256), 0, st, jobs, X, pd.htab, N, P);
  e = run_fft2d(pd, X, S, planes, true, st);
  if (tm) tm->end(1, n_jobs, st);
  if (e != hipSuccess) return e;
  const int RB = N / kGenRows;
  if (tm) tm->begin(2, st);
  hipLaunchKernelGGL(k_gen_reduce, dim3((unsigned)(n_jobs * RB)), dim3(256), 0, st, jobs, X, target, N, P,
                     pd.G, pd.partial, inten_out, field_out);
  if (tm) tm->end(2, n_jobs, st);
  hipLaunchKernelGGL(k_reduce_partials, dim3(n_jobs), dim3(64), 0, st, pd.partial, n_jobs, RB,
                     pd.job_stats);
  return hipGetLastError();
}

}  // namespace hbx
