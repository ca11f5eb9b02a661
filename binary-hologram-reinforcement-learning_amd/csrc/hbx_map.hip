// hbx_map.hip -- every single-pixel flip's PSNR change against a fixed state,
// by correlation (the probe sweep DBS_1024_24-128.py:310-373 / range.py:294-335
// and env_group.py:90-143's importance pass, without one propagation per flip).
//
// A flip of pixel x0 in plane p of group g adds delta * h(x - x0) to that
// plane's field U (h = the single-pixel field of the group, delta = vb (1 - 2 b),
// s = 1 - 2 b the flip sign).  With I the group intensity (mean over the P
// planes of |U|^2), T the target channel and C[f, q](x0) = sum_x f(x) q(x - x0):
//   dI         = (2 Re(conj U delta h') + delta^2 |h'|^2) / P,   h' = h(. - x0)
//   S1 = sum T dI            = s (2 vb / P) Re C[T conj U, h] + (vb^2 / P) C[T, |h|^2]
//   S2 = sum (2 I dI + dI^2) = s [(4 vb / P) Re C[I conj U, h] + (4 vb^3 / P^2) Re C[conj U, |h|^2 h]]
//        + (2 vb^2 / P) C[I, |h|^2] + (2 vb^2 / P^2) Re(C[|U|^2, |h|^2] + C[conj U^2, h^2])
//        + vb^4 / P^2 sum |h|^4
// and the flipped state's statistics are (Sxy + S1, Sxx + S2, Syy) -- exactly
// the quantities an env-step or an eval_flips job sums, for all N^2 pixels of a
// plane at once.  Each correlation is IFFT(F(k) Q(-k)) / N^2 with F = FFT(f),
// Q = FFT(q); real-valued outputs are packed two per complex inverse transform
// by Hermitian symmetrisation.
//
// Per group: 4P + P/2 + 1 forward 2-D FFTs of the data side (T conj U, I conj U,
// conj U, conj U^2 per plane, |U|^2 in plane pairs, T + i I), 3P/2 + 1 inverse
// ones; the h side (h, |h|^2, |h|^2 h, h^2) is transformed once per plan.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbx_fft.hpp"
#include "hbx_internal.hpp"

namespace hbx {

namespace {

__device__ __forceinline__ double psnr_of(double sxy, double sxx, double syy, double count,
                                          int rel_scale, double peak) {
  double mse;
  if (rel_scale == 1) mse = (sxx > 0.0) ? (syy - sxy * sxy / sxx) / count : syy / count;
  else mse = (sxx - 2.0 * sxy + syy) / count;
  if (!(mse > 0.0)) return INFINITY;
  return 10.0 * log10(peak * peak / mse);
}

__device__ __forceinline__ size_t neg_index(size_t i, int N) {  // (-ky, -kx) mod N
  const int ky = (int)(i / N), kx = (int)(i % N);
  return (size_t)((N - ky) % N) * N + ((N - kx) % N);
}

// h-side functions of every group: [g][4][N][N] = h, |h|^2, |h|^2 h, h^2
__global__ void k_map_hprep(const float2* __restrict__ h, float2* __restrict__ q, int G, size_t hw) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= (size_t)G * hw) return;
  const size_t g = i / hw, x = i % hw;
  const float2 v = h[i];
  const float a = norm2(v);
  float2* o = q + g * 4 * hw + x;
  o[0] = v;
  o[hw] = make_float2(a, 0.0f);
  o[2 * hw] = make_float2(a * v.x, a * v.y);
  o[3 * hw] = make_float2(v.x * v.x - v.y * v.y, 2.0f * v.x * v.y);
}

// per-block f64 partial sums of |h|^4 (fixed order -> reproducible)
__global__ void k_map_h4_partial(const float2* __restrict__ h, size_t hw, double* __restrict__ part) {
  __shared__ double red[256];
  const float2* hg = h + (size_t)blockIdx.y * hw;
  double acc = 0.0;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < hw; i += (size_t)gridDim.x * 256) {
    const double a = (double)norm2(hg[i]);
    acc = fma(a, a, acc);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.y * gridDim.x + blockIdx.x] = red[0];
}

__global__ void k_map_h4_final(const double* __restrict__ part, int nb, int G, double* __restrict__ d4) {
  const int g = threadIdx.x;
  if (g >= G) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += part[g * nb + b];
  d4[g] = s;
}

// data-side functions of group g: X[0,P) T conj U, [P,2P) I conj U, [2P,3P) conj U,
// [3P,4P) conj U^2, [4P, 4P+P/2) |U_2q|^2 + i |U_2q+1|^2, [4P+P/2] T + i I
__global__ void k_map_prep(const float2* __restrict__ field, const float* __restrict__ inten,
                           const float* __restrict__ target, float2* __restrict__ X, int P, size_t hw) {
  const size_t x = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (x >= hw) return;
  const float I = inten[x], T = target[x];
  float prev = 0.0f;
  for (int p = 0; p < P; ++p) {
    const float2 u = field[(size_t)p * hw + x];
    const float2 uc = make_float2(u.x, -u.y);
    X[(size_t)p * hw + x] = make_float2(T * uc.x, T * uc.y);
    X[(size_t)(P + p) * hw + x] = make_float2(I * uc.x, I * uc.y);
    X[(size_t)(2 * P + p) * hw + x] = uc;
    X[(size_t)(3 * P + p) * hw + x] = make_float2(uc.x * uc.x - uc.y * uc.y, 2.0f * uc.x * uc.y);
    const float a = norm2(u);
    if (p & 1) X[(size_t)(4 * P + p / 2) * hw + x] = make_float2(prev, a);
    prev = a;
  }
  X[(size_t)(4 * P + P / 2) * hw + x] = make_float2(T, I);
}

// Spectral products (all scaled by 1/N^2):
//   Y[p]      = Herm(X0 Q1~) + i Herm(c2a X1 Q1~ + c2b X2 Q3~)        p < P
//   Y[P + q]  = Herm(A_2q Q2~ + X3_2q Q4~) + i Herm(A_2q+1 Q2~ + X3_2q+1 Q4~)
//   Y[P+P/2]  = X5 Q2~
// with Qn~(k) = Qn(-k), Herm(Z)(k) = (Z(k) + conj Z(-k)) / 2 and A_2q, A_2q+1 the
// spectra of the two real planes packed in X4[q].
__global__ void k_map_combine(const float2* __restrict__ X, const float2* __restrict__ Q,
                              float2* __restrict__ Y, int P, int N, float c2a, float c2b, float inv_n2) {
  const size_t hw = (size_t)N * N;
  const size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const int plane = blockIdx.y;  // 0 .. P + P/2
  if (k >= hw) return;
  const size_t kn = neg_index(k, N);
  const float2* Q1 = Q;
  const float2* Q2 = Q + hw;
  const float2* Q3 = Q + 2 * hw;
  const float2* Q4 = Q + 3 * hw;
  float2 out;
  if (plane < P) {
    const float2* X0 = X + (size_t)plane * hw;
    const float2* X1 = X + (size_t)(P + plane) * hw;
    const float2* X2 = X + (size_t)(2 * P + plane) * hw;
    // Za(k) and Za(-k) for the two products
    const float2 q1k = Q1[kn], q1n = Q1[k], q3k = Q3[kn], q3n = Q3[k];
    const float2 a_k = cmul(X0[k], q1k), a_n = cmul(X0[kn], q1n);
    const float2 b_k = cadd(cscale(cmul(X1[k], q1k), c2a), cscale(cmul(X2[k], q3k), c2b));
    const float2 b_n = cadd(cscale(cmul(X1[kn], q1n), c2a), cscale(cmul(X2[kn], q3n), c2b));
    const float2 ha = make_float2(0.5f * (a_k.x + a_n.x), 0.5f * (a_k.y - a_n.y));
    const float2 hb = make_float2(0.5f * (b_k.x + b_n.x), 0.5f * (b_k.y - b_n.y));
    out = make_float2(ha.x - hb.y, ha.y + hb.x);   // ha + i hb
  } else if (plane < P + P / 2) {
    const int q = plane - P;
    const float2* Z = X + (size_t)(4 * P + q) * hw;
    const float2* X3a = X + (size_t)(3 * P + 2 * q) * hw;
    const float2* X3b = X3a + hw;
    const float2 zk = Z[k], zn = Z[kn];
    // A(k) = (Z(k) + conj Z(-k)) / 2, B(k) = (Z(k) - conj Z(-k)) / (2i); A(-k) = conj A(k)
    const float2 A = make_float2(0.5f * (zk.x + zn.x), 0.5f * (zk.y - zn.y));
    const float2 B = make_float2(0.5f * (zk.y + zn.y), -0.5f * (zk.x - zn.x));
    const float2 q2k = Q2[kn], q2n = Q2[k], q4k = Q4[kn], q4n = Q4[k];
    const float2 a_k = cadd(cmul(A, q2k), cmul(X3a[k], q4k));
    const float2 a_n = cadd(cmul(conjf2(A), q2n), cmul(X3a[kn], q4n));
    const float2 b_k = cadd(cmul(B, q2k), cmul(X3b[k], q4k));
    const float2 b_n = cadd(cmul(conjf2(B), q2n), cmul(X3b[kn], q4n));
    const float2 ha = make_float2(0.5f * (a_k.x + a_n.x), 0.5f * (a_k.y - a_n.y));
    const float2 hb = make_float2(0.5f * (b_k.x + b_n.x), 0.5f * (b_k.y - b_n.y));
    out = make_float2(ha.x - hb.y, ha.y + hb.x);
  } else {
    out = cmul(X[(size_t)(4 * P + P / 2) * hw + k], Q2[kn]);
  }
  Y[(size_t)plane * hw + k] = cscale(out, inv_n2);
}

// PSNR change of every flip of group g's planes
__global__ void k_map_final(const float2* __restrict__ Y, const uint64_t* __restrict__ mask,
                            const double* __restrict__ stats /* [G][3] */, const double* __restrict__ d4,
                            float* __restrict__ out, int g, int G, int P, int N, float vb, double count,
                            int rel, double peak) {
  const size_t hw = (size_t)N * N;
  const size_t x = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const int p = blockIdx.y;
  if (x >= hw) return;
  double sxy = 0.0, sxx = 0.0, syy = 0.0;
  for (int c = 0; c < G; ++c) { sxy += stats[3 * c]; sxx += stats[3 * c + 1]; syy += stats[3 * c + 2]; }
  const double base = psnr_of(sxy, sxx, syy, count, rel, peak);
  const int ch = g * P + p;
  const int y = (int)(x / N), col = (int)(x % N);
  const uint64_t w = mask[((size_t)ch * N + y) * (N / 64) + (col >> 6)];
  const double s = ((w >> (col & 63)) & 1ull) ? -1.0 : 1.0;
  const float2 e12 = Y[(size_t)p * hw + x];
  const float2 e3p = Y[(size_t)(P + p / 2) * hw + x];
  const float2 bb = Y[(size_t)(P + P / 2) * hw + x];
  const double e1 = e12.x, e2 = e12.y, e3 = (p & 1) ? e3p.y : e3p.x, b1 = bb.x, b2 = bb.y;
  const double v = vb, v2 = v * v, Pd = (double)P;
  const double s1 = (s * 2.0 * v * e1 + v2 * b1) / Pd;
  const double s2 = s * e2 + 2.0 * v2 / Pd * b2 + 2.0 * v2 / (Pd * Pd) * e3 + v2 * v2 * d4[g] / (Pd * Pd);
  out[(size_t)ch * hw + x] = (float)(psnr_of(sxy + s1, sxx + s2, syy, count, rel, peak) - base);
}

}  // namespace

hipError_t map_prepare_h(const PlanDev& pd, float2* q, float2* scratch, double* part, double* d4,
                         hipStream_t st) {
  const size_t hw = (size_t)pd.N * pd.N;
  const int G = pd.G;
  hipLaunchKernelGGL(k_map_hprep, dim3((unsigned)((G * hw + 255) / 256)), dim3(256), 0, st, pd.hpsf, q, G, hw);
  constexpr int NB = 64;
  hipLaunchKernelGGL(k_map_h4_partial, dim3(NB, G), dim3(256), 0, st, pd.hpsf, hw, part);
  hipLaunchKernelGGL(k_map_h4_final, dim3(1), dim3(64), 0, st, part, NB, G, d4);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return run_fft2d(pd, q, scratch, 4 * G, false, st);
}

hipError_t map_group(const PlanDev& pd, int g, const float2* field, const float* inten,
                     const float* target, const uint64_t* mask, const double* stats, const float2* q,
                     const double* d4, float2* X, float2* S, float2* Y, float* out, double count, int rel,
                     double peak, hipStream_t st) {
  const int N = pd.N, P = pd.P, G = pd.G;
  const size_t hw = (size_t)N * N;
  const int nx = 4 * P + P / 2 + 1, ny = P + P / 2 + 1;
  const unsigned pb = (unsigned)((hw + 255) / 256);
  hipLaunchKernelGGL(k_map_prep, dim3(pb), dim3(256), 0, st, field + (size_t)g * P * hw, inten + (size_t)g * hw,
                     target + (size_t)g * hw, X, P, hw);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = run_fft2d(pd, X, S, nx, false, st);
  if (e != hipSuccess) return e;
  const float vb = pd.vb, Pf = (float)P;
  hipLaunchKernelGGL(k_map_combine, dim3(pb, ny), dim3(256), 0, st, X, q + (size_t)g * 4 * hw, Y, P, N,
                     4.0f * vb / Pf, 4.0f * vb * vb * vb / (Pf * Pf), 1.0f / (float)hw);
  e = hipGetLastError();
  if (e == hipSuccess) e = run_fft2d(pd, Y, X, ny, true, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_map_final, dim3(pb, P), dim3(256), 0, st, Y, mask, stats, d4, out, g, G, P, N, vb, count,
                     rel, peak);
  return hipGetLastError();
}

}  // namespace hbx
