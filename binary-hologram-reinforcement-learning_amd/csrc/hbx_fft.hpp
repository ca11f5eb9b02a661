// hbx_fft.hpp -- in-register / LDS FFT building blocks for gfx950 (wave64).
//
// An N = R*R point complex FFT is done by a "lane group" of R lanes of one
// wavefront (R = 32 -> two 1024-point FFTs per wave; R = 16 -> four 256-point;
// R = 8 -> eight 64-point).  Four-step decomposition n = t + R*j,
// k = k1 + R*k2:
//   X[k1 + R k2] = sum_t W_R^{t k2} W_N^{t k1} sum_j x[t + R j] W_R^{j k1}
// Lane t holds x[t + R j] in v[j] (so loads of a row are coalesced: for a
// fixed j the R lanes read R consecutive elements), runs an R-point DFT in
// registers, multiplies by W_N^{t k1}, transposes through LDS (one write, one
// read, conflict-free), runs the second R-point DFT and ends holding
// X[t + R k2] in v[k2] -- natural order, so stores coalesce the same way.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hbx {

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
// a * conj(b)
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, a.y * b.y), fmaf(a.y, b.x, -a.x * b.y));
}
__device__ __forceinline__ float2 conjf2(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float norm2(float2 a) { return fmaf(a.x, a.x, a.y * a.y); }

// cos / sin of 2*pi*k/32 for k = 0..8 (first octant; the rest by symmetry).
// Literal constants so fully unrolled code folds them into immediates.
__device__ __forceinline__ float c32(int k) {
  switch (k & 31) {
    case 0: return 1.0f;
    case 1: return 0.98078528040323044913f;
    case 2: return 0.92387953251128675613f;
    case 3: return 0.83146961230254523708f;
    case 4: return 0.70710678118654752440f;
    case 5: return 0.55557023301960222474f;
    case 6: return 0.38268343236508977173f;
    case 7: return 0.19509032201612826785f;
    case 8: return 0.0f;
    case 9: return -0.19509032201612826785f;
    case 10: return -0.38268343236508977173f;
    case 11: return -0.55557023301960222474f;
    case 12: return -0.70710678118654752440f;
    case 13: return -0.83146961230254523708f;
    case 14: return -0.92387953251128675613f;
    case 15: return -0.98078528040323044913f;
    case 16: return -1.0f;
    case 17: return -0.98078528040323044913f;
    case 18: return -0.92387953251128675613f;
    case 19: return -0.83146961230254523708f;
    case 20: return -0.70710678118654752440f;
    case 21: return -0.55557023301960222474f;
    case 22: return -0.38268343236508977173f;
    case 23: return -0.19509032201612826785f;
    case 24: return 0.0f;
    case 25: return 0.19509032201612826785f;
    case 26: return 0.38268343236508977173f;
    case 27: return 0.55557023301960222474f;
    case 28: return 0.70710678118654752440f;
    case 29: return 0.83146961230254523708f;
    case 30: return 0.92387953251128675613f;
    default: return 0.98078528040323044913f;
  }
}
__device__ __forceinline__ float s32(int k) { return c32(k - 8); }  // sin(x) = cos(x - pi/2)

// Multiply d by W_M^k = exp(-+ 2 pi i k / M), M | 32, k compile-time after unrolling.
template <bool INV>
__device__ __forceinline__ float2 twiddle_const(float2 d, int k, int M) {
  const int k32 = (k * (32 / M)) & 31;  // exponent in units of 2pi/32
  if (k32 == 0) return d;
  if (k32 == 8) return INV ? make_float2(-d.y, d.x) : make_float2(d.y, -d.x);   // *(+i) / *(-i)
  if (k32 == 16) return make_float2(-d.x, -d.y);
  if (k32 == 24) return INV ? make_float2(d.y, -d.x) : make_float2(-d.y, d.x);
  const float c = c32(k32), s = s32(k32);
  if (k32 == 4 || k32 == 12 || k32 == 20 || k32 == 28) {
    // |c| == |s| == sqrt(1/2): 2 mul + 2 add
    const float ws = INV ? s : -s;
    return make_float2(c * d.x - ws * d.y, c * d.y + ws * d.x);
  }
  const float ws = INV ? s : -s;
  return make_float2(fmaf(c, d.x, -ws * d.y), fmaf(c, d.y, ws * d.x));
}

__host__ __device__ constexpr int ilog2c(int n) { return n <= 1 ? 0 : 1 + ilog2c(n / 2); }
__host__ __device__ constexpr int bitrev(int x, int bits) {
  int r = 0;
  for (int i = 0; i < bits; ++i) r |= ((x >> i) & 1) << (bits - 1 - i);
  return r;
}

// In-register R-point DFT (R in {4, 8, 16, 32}), radix-2 DIF, natural-order out.
// forward: X[k] = sum_n x[n] exp(-2 pi i n k / R); inverse: + sign, no scaling.
template <int R, bool INV>
__device__ __forceinline__ void dft_reg(float2 (&v)[R]) {
#pragma unroll
  for (int span = R / 2; span >= 1; span >>= 1) {
#pragma unroll
    for (int start = 0; start < R; start += 2 * span) {
#pragma unroll
      for (int k = 0; k < span; ++k) {
        const float2 a = v[start + k], b = v[start + k + span];
        v[start + k] = cadd(a, b);
        v[start + k + span] = twiddle_const<INV>(csub(a, b), k, 2 * span);
      }
    }
  }
  // DIF leaves X[k] at position bitrev(k): permute (register renaming only)
  float2 tmp[R];
#pragma unroll
  for (int k = 0; k < R; ++k) tmp[k] = v[bitrev(k, ilog2c(R))];
#pragma unroll
  for (int k = 0; k < R; ++k) v[k] = tmp[k];
}

// Wave-level ordering of LDS traffic between lanes of one wavefront.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup barrier that orders LDS only: outstanding GLOBAL loads (register
// prefetches) stay in flight across it, unlike __syncthreads().
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Scratch layout for the transpose: a padded [R][R+1] tile private to a lane group.
template <int R>
struct PaddedScratch {
  float2* base;
  __device__ __forceinline__ float2* at(int t, int k1) const { return base + t * (R + 1) + k1; }
};

// Scratch that lives in the slots of one column of an LDS strip [N][SW+1]:
// slot(t, k1) = R*k1 + ((t + k1) mod R)  -> conflict-free both ways.
template <int R, int PITCH>
struct ColumnScratch {
  float2* col;  // &strip[0 * PITCH + c]
  __device__ __forceinline__ float2* at(int t, int k1) const {
    return col + (R * k1 + ((t + k1) & (R - 1))) * PITCH;
  }
};

// Full N = R*R point FFT by R lanes.  v[j] = x[t + R j] in, v[k2] = X[t + R k2] out.
// tw: LDS table [k1][t] = W_N^{t k1} (forward sign).
template <int R, bool INV, class Scratch>
__device__ __forceinline__ void fft_group(float2 (&v)[R], int t, const Scratch& sc, const float2* tw) {
  // keep the twiddle loads local to each FFT: without this barrier the
  // compiler CSEs / hoists them across calls and pins 2R VGPRs for good
  asm volatile("" ::: "memory");
#ifdef HBX_NO_FFT  // access-pattern ceiling experiments only (tools/): data moves, no arithmetic
  return;
#endif
  dft_reg<R, INV>(v);
#pragma unroll
  for (int k1 = 1; k1 < R; ++k1) {
    const float2 w = tw[k1 * R + t];
    v[k1] = INV ? cmulc(v[k1], w) : cmul(v[k1], w);
  }
  wave_sync();  // previous users of the scratch are done
#pragma unroll
  for (int k1 = 0; k1 < R; ++k1) *sc.at(t, k1) = v[k1];
  wave_sync();
#pragma unroll
  for (int tt = 0; tt < R; ++tt) v[tt] = *sc.at(tt, t);
  wave_sync();
  dft_reg<R, INV>(v);
}

// Value of conj(X[N - k]) for k = t + R*k2, fetched from the lane group that
// holds it (lane (R - t) mod R, register R-1-k2; lane 0 keeps its own
// register (R - k2) mod R).  `lane_base` is the first lane of the group.
template <int R>
__device__ __forceinline__ float2 mirror_conj(const float2 (&v)[R], int k2, int t, int lane_base) {
  const int src = lane_base + ((R - t) & (R - 1));
  const float2 other = v[R - 1 - k2];
  float2 p;
  p.x = __shfl(other.x, src, 64);
  p.y = __shfl(other.y, src, 64);
  const float2 own = v[(R - k2) & (R - 1)];
  const float2 z = (t == 0) ? own : p;
  return conjf2(z);
}

}  // namespace hbx
