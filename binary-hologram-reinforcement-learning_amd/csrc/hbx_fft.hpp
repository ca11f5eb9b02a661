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

#include <type_traits>
#include <utility>

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

__host__ __device__ constexpr int ilog2c(int n) { return n <= 1 ? 0 : 1 + ilog2c(n / 2); }
__host__ __device__ constexpr int bitrev(int x, int bits) {
  int r = 0;
  for (int i = 0; i < bits; ++i) r |= ((x >> i) & 1) << (bits - 1 - i);
  return r;
}

// ---------------------------------------------------------------------------
// Packed-f32 complex arithmetic (gfx950 VOP3P: one v_pk_* instruction works on
// both halves of a 64-bit register pair, at the issue cost of one f32 op).
// op_sel / op_sel_hi pick the source half feeding the low / high result and
// neg_lo / neg_hi negate it, so the swaps and sign flips of the +-i twiddles
// and of a complex product cost nothing extra:
//   a * w       = v_pk_mul (a, w.xx) ; v_pk_fma(-a.y|a.x, w.yy, .)   2 instr.
//   (a - b)(-i) = (a.y - b.y, b.x - a.x)                           1 instr.
// The asm statements are not volatile: the compiler schedules them freely.
// ---------------------------------------------------------------------------
typedef float pk2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ pk2 to_pk(float2 a) { return (pk2){a.x, a.y}; }
__device__ __forceinline__ float2 from_pk(pk2 a) { return make_float2(a.x, a.y); }

// a * w (w in VGPRs)
__device__ __forceinline__ pk2 pk_cmul(pk2 a, pk2 w) {
  pk2 t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(w));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
      : "=v"(r) : "v"(a), "v"(w), "v"(t));
  return r;
}
// a * conj(w)
__device__ __forceinline__ pk2 pk_cmulc(pk2 a, pk2 w) {
  pk2 t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(w));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]"
      : "=v"(r) : "v"(a), "v"(w), "v"(t));
  return r;
}
// a * (C + iS) where C / S are one half of the register pair P, possibly
// swapped (SW) and negated (N1 for C, N2 for S) -- all folded into op_sel /
// neg modifiers, so the 4 first-octant pairs P_r = (cos, sin)(2 pi r / 32),
// r = 1..4, serve every compile-time twiddle of a 32-point DFT
template <bool SW, bool N1, bool N2>
__device__ __forceinline__ pk2 pk_cmul_sel(pk2 a, pk2 P) {
  pk2 t, r;
  if constexpr (!SW && !N1) asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(P));
  if constexpr (!SW && N1) asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(t) : "v"(a), "v"(P));
  if constexpr (SW && !N1) asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(t) : "v"(a), "v"(P));
  if constexpr (SW && N1) asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(t) : "v"(a), "v"(P));
  if constexpr (!SW && !N2)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]" : "=v"(r) : "v"(a), "v"(P), "v"(t));
  if constexpr (!SW && N2)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,1,0] neg_hi:[0,1,0]" : "=v"(r) : "v"(a), "v"(P), "v"(t));
  if constexpr (SW && !N2)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[1,0,0]" : "=v"(r) : "v"(a), "v"(P), "v"(t));
  if constexpr (SW && N2)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[1,1,0] neg_hi:[0,1,0]" : "=v"(r) : "v"(a), "v"(P), "v"(t));
  return r;
}

// first-octant pair P_r, r = 1..4
__device__ __forceinline__ pk2 octant_pair(int r) { return (pk2){c32(r), s32(r)}; }

// (a - b) * (-i) = (a.y - b.y, b.x - a.x)
__device__ __forceinline__ pk2 pk_sub_mul_mi(pk2 a, pk2 b) {
  pk2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_lo:[0,1] neg_hi:[1,0]"
      : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// (a - b) * (+i) = (b.y - a.y, a.x - b.x)
__device__ __forceinline__ pk2 pk_sub_mul_pi(pk2 a, pk2 b) {
  pk2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_lo:[1,0] neg_hi:[0,1]"
      : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// (a - b) * W_M^k (forward) or W_M^-k (INV), k / M compile-time after unrolling
template <bool INV, int K32>
__device__ __forceinline__ pk2 pk_sub_twiddle_k(pk2 a, pk2 b) {
  constexpr int k32 = K32 & 31;   // exponent in units of 2pi/32
  if constexpr (k32 == 0) return a - b;
  else if constexpr (k32 == 16) return b - a;
  else if constexpr (k32 == 8) return INV ? pk_sub_mul_pi(a, b) : pk_sub_mul_mi(a, b);
  else if constexpr (k32 == 24) return INV ? pk_sub_mul_mi(a, b) : pk_sub_mul_pi(a, b);
  else {
    // theta = 2 pi (8 q + r) / 32: (cos, sin) theta from P_r (r <= 4) or swap(P_8-r),
    // rotated by quadrant q; forward twiddles use -sin
    constexpr int q = k32 / 8, r = k32 % 8;
    constexpr bool swA = r > 4;
    constexpr bool sw = swA != (q % 2 == 1);
    constexpr bool n1 = (q == 1 || q == 2);
    constexpr bool n2 = (q == 2 || q == 3) != !INV;
    return pk_cmul_sel<sw, n1, n2>(a - b, octant_pair(swA ? 8 - r : r));
  }
}

template <int R, bool INV, int SPAN, int K>
__device__ __forceinline__ void dft_stage_bfly(pk2 (&w)[R], int start) {
  const pk2 a = w[start + K], b = w[start + K + SPAN];
  w[start + K] = a + b;
  w[start + K + SPAN] = pk_sub_twiddle_k<INV, K * (32 / (2 * SPAN))>(a, b);
}

template <int R, bool INV, int SPAN, int... Ks>
__device__ __forceinline__ void dft_stage(pk2 (&w)[R], std::integer_sequence<int, Ks...>) {
#pragma unroll
  for (int start = 0; start < R; start += 2 * SPAN) (dft_stage_bfly<R, INV, SPAN, Ks>(w, start), ...);
}

template <int R, bool INV, int SPAN>
__device__ __forceinline__ void dft_stages(pk2 (&w)[R]) {
  dft_stage<R, INV, SPAN>(w, std::make_integer_sequence<int, SPAN>{});
  if constexpr (SPAN > 1) dft_stages<R, INV, SPAN / 2>(w);
}

// In-register R-point DFT (R in {4, 8, 16, 32}), radix-2 DIF, natural-order out.
// forward: X[k] = sum_n x[n] exp(-2 pi i n k / R); inverse: + sign, no scaling.
// Packed f32: R/2 log2 R butterflies of one v_pk_add + one packed (sub x twiddle)
// (1 instruction for 1, -1, +-i; 3 otherwise) -- half the VALU of scalar f32.
template <int R, bool INV>
__device__ __forceinline__ void dft_reg(pk2 (&w)[R]) {
  dft_stages<R, INV, R / 2>(w);
  // DIF leaves X[k] at position bitrev(k): permute (register renaming only)
  pk2 tmp[R];
#pragma unroll
  for (int k = 0; k < R; ++k) tmp[k] = w[bitrev(k, ilog2c(R))];
#pragma unroll
  for (int k = 0; k < R; ++k) w[k] = tmp[k];
}

// scalar-f32 variant (lower register pressure: the column pass keeps two
// lines in registers and spills with the packed one)
template <bool INV>
__device__ __forceinline__ float2 twiddle_const(float2 d, int k, int M) {
  const int k32 = (k * (32 / M)) & 31;  // exponent in units of 2pi/32
  if (k32 == 0) return d;
  if (k32 == 8) return INV ? make_float2(-d.y, d.x) : make_float2(d.y, -d.x);   // *(+i) / *(-i)
  if (k32 == 16) return make_float2(-d.x, -d.y);
  if (k32 == 24) return INV ? make_float2(d.y, -d.x) : make_float2(-d.y, d.x);
  const float c = c32(k32), s = s32(k32);
  const float ws = INV ? s : -s;
  return make_float2(fmaf(c, d.x, -ws * d.y), fmaf(c, d.y, ws * d.x));
}

template <int R, bool INV>
__device__ __forceinline__ void dft_reg_scalar(float2 (&v)[R]) {
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
  float2 tmp[R];
#pragma unroll
  for (int k = 0; k < R; ++k) tmp[k] = v[bitrev(k, ilog2c(R))];
#pragma unroll
  for (int k = 0; k < R; ++k) v[k] = tmp[k];
}

template <int R, bool INV>
__device__ __forceinline__ void dft_reg(float2 (&v)[R]) {
  pk2 w[R];
#pragma unroll
  for (int k = 0; k < R; ++k) w[k] = to_pk(v[k]);
  dft_reg<R, INV>(w);
#pragma unroll
  for (int k = 0; k < R; ++k) v[k] = from_pk(w[k]);
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
// tw: LDS table [k1][t] = W_N^{t k1} (forward sign).  Element type float2 or
// pk2 (pk2 arrays keep the whole FFT in packed register pairs, no copies).
template <class T>
__device__ __forceinline__ pk2 ld_pk(const T& a) {
  if constexpr (std::is_same<T, pk2>::value) return a; else return to_pk(a);
}
template <class T>
__device__ __forceinline__ T st_pk(pk2 a) {
  if constexpr (std::is_same<T, pk2>::value) return a; else return from_pk(a);
}

// fft_group in two halves: s1 = the first DFT over j and the twiddles (registers and the
// LDS twiddle table only), s2 = the transpose through the group's scratch and the second
// DFT.  A kernel that shares the scratch with other work can sit a barrier between them.
template <int R, bool INV, bool SCALAR = false, class T>
__device__ __forceinline__ void fft_group_s1(T (&v)[R], int t, const float2* tw) {
  asm volatile("" ::: "memory");
  if constexpr (SCALAR) {
    static_assert(std::is_same<T, float2>::value, "scalar FFT works on float2");
    dft_reg_scalar<R, INV>(v);
#pragma unroll
    for (int k1 = 1; k1 < R; ++k1) {
      const float2 w = tw[k1 * R + t];
      v[k1] = INV ? cmulc(v[k1], w) : cmul(v[k1], w);
    }
  } else {
    dft_reg<R, INV>(v);
#pragma unroll
    for (int k1 = 1; k1 < R; ++k1) {
      const pk2 w = to_pk(tw[k1 * R + t]);
      v[k1] = st_pk<T>(INV ? pk_cmulc(ld_pk(v[k1]), w) : pk_cmul(ld_pk(v[k1]), w));
    }
  }
}
template <int R, bool INV, bool SCALAR = false, class Scratch, class T>
__device__ __forceinline__ void fft_group_s2(T (&v)[R], int t, const Scratch& sc) {
  wave_sync();  // previous users of the scratch are done
#pragma unroll
  for (int k1 = 0; k1 < R; ++k1) *reinterpret_cast<T*>(sc.at(t, k1)) = v[k1];
  wave_sync();
#pragma unroll
  for (int tt = 0; tt < R; ++tt) v[tt] = *reinterpret_cast<const T*>(sc.at(tt, t));
  wave_sync();
  if constexpr (SCALAR) dft_reg_scalar<R, INV>(v);
  else dft_reg<R, INV>(v);
}

template <int R, bool INV, bool SCALAR = false, class Scratch, class T>
__device__ __forceinline__ void fft_group(T (&v)[R], int t, const Scratch& sc, const float2* tw) {
  // keep the twiddle loads local to each FFT: without this barrier the
  // compiler CSEs / hoists them across calls and pins 2R VGPRs for good
  asm volatile("" ::: "memory");
  if constexpr (SCALAR) {
    static_assert(std::is_same<T, float2>::value, "scalar FFT works on float2");
    dft_reg_scalar<R, INV>(v);
#pragma unroll
    for (int k1 = 1; k1 < R; ++k1) {
      const float2 w = tw[k1 * R + t];
      v[k1] = INV ? cmulc(v[k1], w) : cmul(v[k1], w);
    }
  } else {
    dft_reg<R, INV>(v);
#pragma unroll
    for (int k1 = 1; k1 < R; ++k1) {
      const pk2 w = to_pk(tw[k1 * R + t]);
      v[k1] = st_pk<T>(INV ? pk_cmulc(ld_pk(v[k1]), w) : pk_cmul(ld_pk(v[k1]), w));
    }
  }
  wave_sync();  // previous users of the scratch are done
#pragma unroll
  for (int k1 = 0; k1 < R; ++k1) *reinterpret_cast<T*>(sc.at(t, k1)) = v[k1];
  wave_sync();
#pragma unroll
  for (int tt = 0; tt < R; ++tt) v[tt] = *reinterpret_cast<const T*>(sc.at(tt, t));
  wave_sync();
  if constexpr (SCALAR) dft_reg_scalar<R, INV>(v);
  else dft_reg<R, INV>(v);
}

// fft_group with half the scratch: the transpose moves the real parts, then the
// imaginary parts, through a private [R][R+1] FLOAT tile (4.2 KB per group at
// R = 32 instead of 8.4 KB).  Same result, bit for bit: only the LDS hand-off
// differs.  Each half of v is overwritten only after the whole group has
// written it out (wave_sync), so no extra registers are held.
template <int R, bool INV, bool SCALAR = false, class T>
__device__ __forceinline__ void fft_group_split(T (&v)[R], int t, float* sc, const float2* tw) {
  asm volatile("" ::: "memory");
  if constexpr (SCALAR) {
    static_assert(std::is_same<T, float2>::value, "scalar FFT works on float2");
    dft_reg_scalar<R, INV>(v);
#pragma unroll
    for (int k1 = 1; k1 < R; ++k1) {
      const float2 w = tw[k1 * R + t];
      v[k1] = INV ? cmulc(v[k1], w) : cmul(v[k1], w);
    }
  } else {
    dft_reg<R, INV>(v);
#pragma unroll
    for (int k1 = 1; k1 < R; ++k1) {
      const pk2 w = to_pk(tw[k1 * R + t]);
      v[k1] = st_pk<T>(INV ? pk_cmulc(ld_pk(v[k1]), w) : pk_cmul(ld_pk(v[k1]), w));
    }
  }
  wave_sync();  // previous users of the scratch are done
#pragma unroll
  for (int k1 = 0; k1 < R; ++k1) sc[t * (R + 1) + k1] = v[k1].x;
  wave_sync();
#pragma unroll
  for (int tt = 0; tt < R; ++tt) v[tt].x = sc[tt * (R + 1) + t];
  wave_sync();
#pragma unroll
  for (int k1 = 0; k1 < R; ++k1) sc[t * (R + 1) + k1] = v[k1].y;
  wave_sync();
#pragma unroll
  for (int tt = 0; tt < R; ++tt) v[tt].y = sc[tt * (R + 1) + t];
  wave_sync();
  if constexpr (SCALAR) dft_reg_scalar<R, INV>(v);
  else dft_reg<R, INV>(v);
}

template <int J>
__device__ __forceinline__ uint32_t bit_transpose_level(uint32_t x, int t) {
  constexpr uint32_t m = J == 16 ? 0x0000ffffu : J == 8 ? 0x00ff00ffu : J == 4 ? 0x0f0f0f0fu
                       : J == 2 ? 0x33333333u : 0x55555555u;
  const uint32_t y = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, (J << 10) | 0x1f);
  const bool hi = (t & J) != 0;
  const uint32_t lo_v = hi ? y : x, hi_v = hi ? x : y;
  const uint32_t d = ((lo_v >> J) ^ hi_v) & m;
  return x ^ (hi ? d : (d << J));
}
// The value of lane t ^ J (J < 32) of the lane's 32-lane group, without the LDS pipe (r05): DPP
// quad permutes for J = 1, 2, row rotations for J = 4 (two, one per half of each 8-lane run), 8,
// and gfx950's v_permlane16_swap for J = 16.  ds_swizzle (bit_transpose_level) costs an LDS
// round trip per level, five dependent ones per transpose (k_rowfwd32: SQ_WAIT_INST_LDS twice
// SQ_ACTIVE_INST_LDS).  tools/lane_xor_test.hip checks every J against ds_swizzle.
template <int J>
__device__ __forceinline__ uint32_t lane_xor(uint32_t x, int t) {
  if constexpr (J == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xf, 0xf, false);    // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xf, 0xf, false);    // quad_perm [2,3,0,1]
  } else if constexpr (J == 4) {
    const uint32_t a = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x124, 0xf, 0xf, false);   // row_ror:4
    const uint32_t b = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x12C, 0xf, 0xf, false);   // row_ror:12
    return (t & 4) ? a : b;
  } else if constexpr (J == 8) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xf, 0xf, false);   // row_ror:8
  } else {
    static_assert(J == 16, "lane_xor: J in {1, 2, 4, 8, 16}");
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (t & 16) ? r[0] : r[1];
  }
}

template <int J>
__device__ __forceinline__ uint32_t bit_transpose_level_dpp(uint32_t x, int t) {
  constexpr uint32_t m = J == 16 ? 0x0000ffffu : J == 8 ? 0x00ff00ffu : J == 4 ? 0x0f0f0f0fu
                       : J == 2 ? 0x33333333u : 0x55555555u;
  const uint32_t y = lane_xor<J>(x, t);
  const bool hi = (t & J) != 0;
  const uint32_t lo_v = hi ? y : x, hi_v = hi ? x : y;
  const uint32_t d = ((lo_v >> J) ^ hi_v) & m;
  return x ^ (hi ? d : (d << J));
}

// 32 x 32 bit transpose across a 32-lane group: bit r of lane t's result = bit t of lane r's x
__device__ __forceinline__ uint32_t group_bit_transpose(uint32_t x, int t) {
  x = bit_transpose_level_dpp<16>(x, t);
  x = bit_transpose_level_dpp<8>(x, t);
  x = bit_transpose_level_dpp<4>(x, t);
  x = bit_transpose_level_dpp<2>(x, t);
  return bit_transpose_level_dpp<1>(x, t);
}
// the ds_swizzle form (r02-r04), kept as the reference of tools/lane_xor_test.hip
__device__ __forceinline__ uint32_t group_bit_transpose_swizzle(uint32_t x, int t) {
  x = bit_transpose_level<16>(x, t);
  x = bit_transpose_level<8>(x, t);
  x = bit_transpose_level<4>(x, t);
  x = bit_transpose_level<2>(x, t);
  return bit_transpose_level<1>(x, t);
}

// ---------------------------------------------------------------------------
// Mirror-paired lane order of k_rowfwd32's second FFT stage (r05).  The Hermitian split needs
// conj Z[N - k] next to Z[k]; with lane t holding k1 = t (k = k1 + 32 k2) the partner lane is
// 32 - t: a cross-lane gather (two ds_bpermute per value, 32 per row block).  Reading column
// k1 = kMirrorK1[t] of the transposed tile instead puts k1 and 32 - k1 on the lane pair
// (2m, 2m + 1): the partner is lane t ^ 1, a DPP quad permute.  Lanes 0 / 1 hold k1 = 0 / 16,
// their own mirrors.  Which pair sits in which half of the group is chosen so the plane tile's
// lane-row writes (tile_pos<32, 8> of line k1 + 32 k2) stay conflict-free for the 16-lane
// service of ds_write_b64 (tools/lds_swizzle_model.py mirror_pair_order, exhaustive over splits).
static __constant__ const int kMirrorK1[32] = {0, 16, 1, 31, 3, 29, 4, 28, 5, 27, 7, 25, 8, 24, 12, 20,
                                               2, 30, 6, 26, 9, 23, 10, 22, 11, 21, 13, 19, 14, 18, 15, 17};
__device__ __forceinline__ int mirror_k1(int t) { return kMirrorK1[t & 31]; }

// fft_group_split (R = 32, packed) with the second stage in mirror-paired lane order: lane t
// ends up holding X[k1 + 32 k2] for k1 = mirror_k1(t) (passed in), k2 = 0..31.
template <bool INV, class T>
__device__ __forceinline__ void fft_group_split_mirror(T (&v)[32], int t, int k1, float* sc, const float2* tw) {
  asm volatile("" ::: "memory");
  dft_reg<32, INV>(v);
#pragma unroll
  for (int j = 1; j < 32; ++j) {
    const pk2 w = to_pk(tw[j * 32 + t]);
    v[j] = st_pk<T>(INV ? pk_cmulc(ld_pk(v[j]), w) : pk_cmul(ld_pk(v[j]), w));
  }
  wave_sync();
#pragma unroll
  for (int j = 0; j < 32; ++j) sc[t * 33 + j] = v[j].x;
  wave_sync();
#pragma unroll
  for (int tt = 0; tt < 32; ++tt) v[tt].x = sc[tt * 33 + k1];
  wave_sync();
#pragma unroll
  for (int j = 0; j < 32; ++j) sc[t * 33 + j] = v[j].y;
  wave_sync();
#pragma unroll
  for (int tt = 0; tt < 32; ++tt) v[tt].y = sc[tt * 33 + k1];
  wave_sync();
  dft_reg<32, INV>(v);
}

// conj(X[N - k]) for k = k1 + 32 k2 in the mirror-paired order: lane t ^ 1's register 31 - k2
// (DPP), lane 0 (k1 = 0) its own register (32 - k2) mod 32, lane 1 (k1 = 16) its own 31 - k2
template <class T>
__device__ __forceinline__ float2 mirror_conj_paired(const T (&v)[32], int k2, int t) {
  const float2 a = make_float2(v[31 - k2].x, v[31 - k2].y);
  float2 p;
  p.x = __uint_as_float((uint32_t)__builtin_amdgcn_mov_dpp((int)__float_as_uint(a.x), 0xB1, 0xf, 0xf, false));
  p.y = __uint_as_float((uint32_t)__builtin_amdgcn_mov_dpp((int)__float_as_uint(a.y), 0xB1, 0xf, 0xf, false));
  const float2 own0 = make_float2(v[(32 - k2) & 31].x, v[(32 - k2) & 31].y);
  const float2 z = t == 0 ? own0 : (t == 1 ? a : p);
  return conjf2(z);
}

// Value of conj(X[N - k]) for k = t + R*k2, fetched from the lane group that
// holds it (lane (R - t) mod R, register R-1-k2; lane 0 keeps its own
// register (R - k2) mod R).  `lane_base` is the first lane of the group.
template <int R, class T>
__device__ __forceinline__ float2 mirror_conj(const T (&v)[R], int k2, int t, int lane_base) {
  const int src = lane_base + ((R - t) & (R - 1));
  const float2 other = make_float2(v[R - 1 - k2].x, v[R - 1 - k2].y);
  float2 p;
  p.x = __shfl(other.x, src, 64);
  p.y = __shfl(other.y, src, 64);
  const float2 own = make_float2(v[(R - k2) & (R - 1)].x, v[(R - k2) & (R - 1)].y);
  const float2 z = (t == 0) ? own : p;
  return conjf2(z);
}

// ---------------------------------------------------------------------------
// N = 896 (the 64-pixel crop of a 1024 mask, env_1024_24_128.py:144-149):
// 896 = 28 x 32, so a 32-lane group does a four-step with 28 registers in the
// first stage and 32 in the second:
//   natural layout: lane t < 32, register j < 28 holds x[t + 32 j]
//   slot layout:    lane k1 < 28, register k2 < 32 holds X[k1 + 28 k2]
// The 28-point DFT is Good-Thomas (28 = 4 x 7, coprime: no twiddles, only
// index maps n = (7 n1 + 4 n2) mod 28, k = (21 k1 + 8 k2) mod 28); the
// 7-point DFT pairs x_m with x_{7-m}.  Lanes 28..31 carry no data in the slot
// layout (their registers are don't-care).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float c7(int k) {
  switch (((k % 7) + 7) % 7) {
    case 0: return 1.0f;
    case 1: case 6: return 0.62348980185873353053f;
    case 2: case 5: return -0.22252093395631440429f;
    default: return -0.90096886790241912624f;
  }
}
__device__ __forceinline__ float s7(int k) {   // sin(2 pi k / 7)
  switch (((k % 7) + 7) % 7) {
    case 0: return 0.0f;
    case 1: return 0.78183148246802980871f;
    case 2: return 0.97492791218182360702f;
    case 3: return 0.43388373911755812048f;
    case 4: return -0.43388373911755812048f;
    case 5: return -0.97492791218182360702f;
    default: return -0.78183148246802980871f;
  }
}

// in-place 7-point DFT of x[0..6] (forward: exp(-2 pi i n k / 7))
template <bool INV>
__device__ __forceinline__ void dft7(float2 (&x)[7]) {
  float2 a[4], b[4];
#pragma unroll
  for (int m = 1; m <= 3; ++m) { a[m] = cadd(x[m], x[7 - m]); b[m] = csub(x[m], x[7 - m]); }
  const float2 x0 = x[0];
  x[0] = cadd(x0, cadd(a[1], cadd(a[2], a[3])));
#pragma unroll
  for (int k = 1; k <= 3; ++k) {
    float2 u = x0, w = make_float2(0.f, 0.f);
#pragma unroll
    for (int m = 1; m <= 3; ++m) {
      const float c = c7(m * k), sn = s7(m * k);
      u = make_float2(fmaf(c, a[m].x, u.x), fmaf(c, a[m].y, u.y));
      w = make_float2(fmaf(sn, b[m].x, w.x), fmaf(sn, b[m].y, w.y));
    }
    // forward: X[k] = u - i w, X[7-k] = u + i w ; inverse swaps them
    const float2 miw = make_float2(w.y, -w.x);
    x[k] = INV ? csub(u, miw) : cadd(u, miw);
    x[7 - k] = INV ? cadd(u, miw) : csub(u, miw);
  }
}

template <bool INV>
__device__ __forceinline__ void dft4(float2& x0, float2& x1, float2& x2, float2& x3) {
  const float2 t0 = cadd(x0, x2), t1 = csub(x0, x2), t2 = cadd(x1, x3), t3 = csub(x1, x3);
  // forward: X1 = t1 - i t3, X3 = t1 + i t3
  const float2 mi3 = INV ? make_float2(-t3.y, t3.x) : make_float2(t3.y, -t3.x);
  x0 = cadd(t0, t2);
  x2 = csub(t0, t2);
  x1 = cadd(t1, mi3);
  x3 = csub(t1, mi3);
}

// 28-point DFT of v[0..27], natural order in and out (Good-Thomas 4 x 7)
template <bool INV>
__device__ __forceinline__ void dft28(float2 (&v)[32]) {
  float2 y[4][7];
#pragma unroll
  for (int n2 = 0; n2 < 7; ++n2) {
    float2 e0 = v[(4 * n2) % 28], e1 = v[(7 + 4 * n2) % 28];
    float2 e2 = v[(14 + 4 * n2) % 28], e3 = v[(21 + 4 * n2) % 28];
    dft4<INV>(e0, e1, e2, e3);
    y[0][n2] = e0; y[1][n2] = e1; y[2][n2] = e2; y[3][n2] = e3;
  }
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    dft7<INV>(y[k1]);
#pragma unroll
    for (int k2 = 0; k2 < 7; ++k2) v[(21 * k1 + 8 * k2) % 28] = y[k1][k2];
  }
}

// Packed-f32 variants (two floats per VALU op: v_pk_add / v_pk_fma with a
// broadcast constant): half the VALU of the scalar radix-4 / radix-7 stages.
__device__ __forceinline__ pk2 pk_mul_mi(pk2 a) { return (pk2){a.y, -a.x}; }   // a * (-i)
__device__ __forceinline__ pk2 pk_mul_pi(pk2 a) { return (pk2){-a.y, a.x}; }   // a * (+i)

template <bool INV>
__device__ __forceinline__ void dft7_pk(pk2 (&x)[7]) {
  pk2 a[4], b[4];
#pragma unroll
  for (int m = 1; m <= 3; ++m) { a[m] = x[m] + x[7 - m]; b[m] = x[m] - x[7 - m]; }
  const pk2 x0 = x[0];
  x[0] = x0 + (a[1] + (a[2] + a[3]));
#pragma unroll
  for (int k = 1; k <= 3; ++k) {
    pk2 u = x0, w = (pk2){0.f, 0.f};
#pragma unroll
    for (int m = 1; m <= 3; ++m) {
      const float c = c7(m * k), sn = s7(m * k);
      u = __builtin_elementwise_fma((pk2){c, c}, a[m], u);
      w = __builtin_elementwise_fma((pk2){sn, sn}, b[m], w);
    }
    const pk2 miw = pk_mul_mi(w);
    x[k] = INV ? u - miw : u + miw;
    x[7 - k] = INV ? u + miw : u - miw;
  }
}

template <bool INV>
__device__ __forceinline__ void dft4_pk(pk2& x0, pk2& x1, pk2& x2, pk2& x3) {
  const pk2 t0 = x0 + x2, t1 = x0 - x2, t2 = x1 + x3, t3 = x1 - x3;
  const pk2 mi3 = INV ? pk_mul_pi(t3) : pk_mul_mi(t3);
  x0 = t0 + t2;
  x2 = t0 - t2;
  x1 = t1 + mi3;
  x3 = t1 - mi3;
}

template <bool INV>
__device__ __forceinline__ void dft28_pk(float2 (&v)[32]) {
  pk2 y[4][7];
#pragma unroll
  for (int n2 = 0; n2 < 7; ++n2) {
    pk2 e0 = to_pk(v[(4 * n2) % 28]), e1 = to_pk(v[(7 + 4 * n2) % 28]);
    pk2 e2 = to_pk(v[(14 + 4 * n2) % 28]), e3 = to_pk(v[(21 + 4 * n2) % 28]);
    dft4_pk<INV>(e0, e1, e2, e3);
    y[0][n2] = e0; y[1][n2] = e1; y[2][n2] = e2; y[3][n2] = e3;
  }
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    dft7_pk<INV>(y[k1]);
#pragma unroll
    for (int k2 = 0; k2 < 7; ++k2) v[(21 * k1 + 8 * k2) % 28] = from_pk(y[k1][k2]);
  }
}

// 896-point FFT by 32 lanes, natural layout in -> slot layout out.
// tw896: LDS [k1 < 28][t < 32] = W896^{t k1} (forward sign); INV conjugates.
// SCALAR: scalar-f32 32-point DFTs (fewer live registers than the packed ones
// when a kernel keeps two lines in flight).  _s1 = the 28-point DFTs and twiddles
// (registers and the twiddle table only), _s2 = the transpose through the group's
// scratch and the 32-point DFTs: a kernel that shares the scratch can sit a block
// barrier between them (k_col896).
template <bool INV, bool SCALAR = false>
__device__ __forceinline__ void fft896_ns_s1(float2 (&v)[32], int t, const float2* tw896) {
  asm volatile("" ::: "memory");
  if constexpr (SCALAR) {
    dft28<INV>(v);
#pragma unroll
    for (int k1 = 1; k1 < 28; ++k1) {
      const float2 w = tw896[k1 * 32 + t];
      v[k1] = INV ? cmulc(v[k1], w) : cmul(v[k1], w);
    }
  } else {
    dft28_pk<INV>(v);
#pragma unroll
    for (int k1 = 1; k1 < 28; ++k1) {
      const pk2 w = to_pk(tw896[k1 * 32 + t]);
      v[k1] = from_pk(INV ? pk_cmulc(to_pk(v[k1]), w) : pk_cmul(to_pk(v[k1]), w));
    }
  }
}
template <bool INV, bool SCALAR = false, class Scratch>
__device__ __forceinline__ void fft896_ns_s2(float2 (&v)[32], int t, const Scratch& sc) {
  wave_sync();
#pragma unroll
  for (int k1 = 0; k1 < 28; ++k1) *sc.at(t, k1) = v[k1];
  wave_sync();
  // lane k1 (< 28) gathers A'[t][k1] for t = 0..31; lanes 28..31 read columns 28..31 of the
  // padded tile (in range, never written here: don't-care values, as before).  r05: they read
  // column 0 until r04, the same bank as lane 16 under the 16-lane service of the ds_read2_b64
  // the compiler emits (64 extra LDS cycles per wave and transpose; k_col896's counter,
  // tools/lds_swizzle_model.py col896_conflicts)
  const int k1 = t;
#pragma unroll
  for (int tt = 0; tt < 32; ++tt) v[tt] = *sc.at(tt, k1);
  wave_sync();
  if constexpr (SCALAR) dft_reg_scalar<32, INV>(v);
  else dft_reg<32, INV>(v);
}
template <bool INV, bool SCALAR = false, class Scratch>
__device__ __forceinline__ void fft896_ns(float2 (&v)[32], int t, const Scratch& sc, const float2* tw896) {
  fft896_ns_s1<INV, SCALAR>(v, t, tw896);
  fft896_ns_s2<INV, SCALAR>(v, t, sc);
}

// fft896_ns with half the scratch (r04, k_rowfwd896 at three workgroups per CU): the transpose
// moves the real parts, then the imaginary parts, through a private [32][33] FLOAT tile
// (fft_group_split's scheme).  Same arithmetic, bit-identical result.
template <bool INV>
__device__ __forceinline__ void fft896_ns_split(float2 (&v)[32], int t, float* sc, const float2* tw896) {
  asm volatile("" ::: "memory");
  dft28_pk<INV>(v);
#pragma unroll
  for (int k1 = 1; k1 < 28; ++k1) {
    const pk2 w = to_pk(tw896[k1 * 32 + t]);
    v[k1] = from_pk(INV ? pk_cmulc(to_pk(v[k1]), w) : pk_cmul(to_pk(v[k1]), w));
  }
  const int k1 = t < 28 ? t : 0;
  wave_sync();
#pragma unroll
  for (int j = 0; j < 28; ++j) sc[t * 33 + j] = v[j].x;
  wave_sync();
#pragma unroll
  for (int tt = 0; tt < 32; ++tt) v[tt].x = sc[tt * 33 + k1];
  wave_sync();
#pragma unroll
  for (int j = 0; j < 28; ++j) sc[t * 33 + j] = v[j].y;
  wave_sync();
#pragma unroll
  for (int tt = 0; tt < 32; ++tt) v[tt].y = sc[tt * 33 + k1];
  wave_sync();
  dft_reg<32, INV>(v);
}

// 896-point FFT by 32 lanes, slot layout in -> natural layout out (adjoint of
// fft896_ns: the same stages in reverse order with the opposite sign); _s1 = the
// 32-point DFTs in registers, _s2 = transpose, twiddles, 28-point DFTs
template <bool INV, bool SCALAR = false>
__device__ __forceinline__ void fft896_sn_s1(float2 (&v)[32]) {
  asm volatile("" ::: "memory");
  if constexpr (SCALAR) dft_reg_scalar<32, INV>(v);   // over k2 -> index t (the natural lane)
  else dft_reg<32, INV>(v);
}
template <bool INV, bool SCALAR = false, class Scratch>
__device__ __forceinline__ void fft896_sn_s2(float2 (&v)[32], int t, const Scratch& sc, const float2* tw896) {
  wave_sync();
  // lane k1 (< 28) holds B[k1][t] for t = 0..31 in v[t]
  if (t < 28) {
#pragma unroll
    for (int tt = 0; tt < 32; ++tt) *sc.at(tt, t) = v[tt];
  }
  wave_sync();
#pragma unroll
  for (int k1 = 0; k1 < 28; ++k1) v[k1] = *sc.at(t, k1);
  wave_sync();
  if constexpr (SCALAR) {
#pragma unroll
    for (int k1 = 1; k1 < 28; ++k1) {
      const float2 w = tw896[k1 * 32 + t];
      v[k1] = INV ? cmulc(v[k1], w) : cmul(v[k1], w);
    }
    dft28<INV>(v);              // over k1 -> register j: x[t + 32 j]
  } else {
#pragma unroll
    for (int k1 = 1; k1 < 28; ++k1) {
      const pk2 w = to_pk(tw896[k1 * 32 + t]);
      v[k1] = from_pk(INV ? pk_cmulc(to_pk(v[k1]), w) : pk_cmul(to_pk(v[k1]), w));
    }
    dft28_pk<INV>(v);
  }
}
template <bool INV, bool SCALAR = false, class Scratch>
__device__ __forceinline__ void fft896_sn(float2 (&v)[32], int t, const Scratch& sc, const float2* tw896) {
  fft896_sn_s1<INV, SCALAR>(v);
  fft896_sn_s2<INV, SCALAR>(v, t, sc, tw896);
}

}  // namespace hbx
