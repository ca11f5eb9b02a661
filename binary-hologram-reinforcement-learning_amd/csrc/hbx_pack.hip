// hbx_pack.hip -- the device side of the operator shim's per-call work (gfx950).
//
// k_pack_mask: mask values -> the bit-packed words every propagation reads (include/hbx.h
//   layout).  The reference builds its field from a float / int8 mask on every call
//   (env.py:120-123,170-171: `pre_model >= 0.5`, `torch.tensor(state, dtype=float32)`;
//   DBS_1024_24.py:326-327); here one streaming pass turns it into 1 bit per pixel.  Each wave
//   packs 4 words (256 values) per iteration: lane l loads values 4l .. 4l+3 with one vector
//   load (u32 / float4 / 2 x double2), four wave64 ballots give bit l of "value 4l + k is on"
//   for k = 0..3, and lane i < 4 interleaves the four 16-bit slices i of the ballots into word i
//   (word i bit 4j + k = ballot_k bit 16i + j).  HBM-bound: 1 / 4 / 8 bytes read and 1/8 byte
//   written per pixel.  The binary check of tt.simulate (a value not 0 or 1) is a ballot too:
//   one store of 1 into a caller word (device or host-mapped memory), no host sync.
// k_rel_partials / k_rel_final: tt.relativeLoss(x, y, tm.get_PSNR) (env.py:132,174;
//   DBS_1024_24.py:332) as sufficient statistics sum xy, sum x^2, sum y^2 in f64 (the products
//   formed in f64, as torch's x.double() * y.double()), a fixed-order two-stage reduction
//   (deterministic), then the same PSNR / MSE formula as the env kernels (psnr_from).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "hbx.h"
#include "hbx_internal.hpp"

namespace hbx {

namespace {

// every 4th bit of a 64-bit word from a 16-bit value: bit j -> bit 4j
__device__ __forceinline__ uint64_t spread4(uint64_t x) {
  x &= 0xffffull;
  x = (x | (x << 24)) & 0x000000ff000000ffull;
  x = (x | (x << 12)) & 0x000f000f000f000full;
  x = (x | (x << 6)) & 0x0303030303030303ull;
  x = (x | (x << 3)) & 0x1111111111111111ull;
  return x;
}

// the four values 4l .. 4l+3 of one lane as floats / doubles + the binary check
struct Quad {
  bool on[4];
  bool bad;
};

template <int KIND>
__device__ __forceinline__ Quad load_quad(const void* __restrict__ src, int64_t q, int mode, double thr) {
  Quad r;
  r.bad = false;
  if constexpr (KIND == HBX_SRC_U8) {
    const uint32_t v = reinterpret_cast<const uint32_t*>(src)[q];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t b = (v >> (8 * k)) & 0xffu;
      r.on[k] = mode == HBX_PACK_THRESHOLD ? ((double)b >= thr) : (b != 0u);
    }
    r.bad = (v & 0xfefefefeu) != 0u;
  } else if constexpr (KIND == HBX_SRC_F32) {
    const float4 v = reinterpret_cast<const float4*>(src)[q];
    const float e[4] = {v.x, v.y, v.z, v.w};
    const float tf = (float)thr;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      r.on[k] = mode == HBX_PACK_THRESHOLD ? (e[k] >= tf) : (e[k] != 0.0f);
      r.bad |= !(e[k] == 0.0f || e[k] == 1.0f);
    }
  } else {
    const double2 a = reinterpret_cast<const double2*>(src)[2 * q];
    const double2 b = reinterpret_cast<const double2*>(src)[2 * q + 1];
    const double e[4] = {a.x, a.y, b.x, b.y};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      r.on[k] = mode == HBX_PACK_THRESHOLD ? (e[k] >= thr) : (e[k] != 0.0);
      r.bad |= !(e[k] == 0.0 || e[k] == 1.0);
    }
  }
  return r;
}

// grid-stride over groups of 4 words; n_words words (= values / 64).  A group past the end
// (n_words % 4 != 0) loads nothing for its missing words: their lanes report off / valid.
template <int KIND>
__global__ __launch_bounds__(256) void k_pack_mask(const void* __restrict__ src, int64_t n_words, int mode,
                                                   double thr, uint64_t* __restrict__ bits,
                                                   int32_t* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int64_t n_groups = (n_words + 3) / 4;
  const int64_t stride = (int64_t)gridDim.x * (blockDim.x >> 6);
  bool bad = false;
  for (int64_t g = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); g < n_groups; g += stride) {
    const int64_t w_lane = 4 * g + (lane >> 4);   // the word this lane's four values belong to
    Quad v;
    if (w_lane < n_words) {
      v = load_quad<KIND>(src, 64 * g + lane, mode, thr);
    } else {
      v.on[0] = v.on[1] = v.on[2] = v.on[3] = false;
      v.bad = false;
    }
    bad |= v.bad;
    const uint64_t b0 = __ballot(v.on[0]), b1 = __ballot(v.on[1]);
    const uint64_t b2 = __ballot(v.on[2]), b3 = __ballot(v.on[3]);
    if (lane < 4 && 4 * g + lane < n_words) {
      const int s = 16 * lane;
      bits[4 * g + lane] = spread4(b0 >> s) | (spread4(b1 >> s) << 1) | (spread4(b2 >> s) << 2) |
                           (spread4(b3 >> s) << 3);
    }
  }
  if (err && mode == HBX_PACK_BINARY && __ballot(bad) != 0ull && lane == 0) *err = 1;
}

constexpr int kRelBlocks = 1024;   // partial slots of the relativeLoss reduction (fixed: deterministic)

template <typename T>
__global__ __launch_bounds__(256) void k_rel_partials(const T* __restrict__ x, const T* __restrict__ y, int64_t n,
                                                      double* __restrict__ part) {
  __shared__ double s[3][4];
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * per;
  const int64_t i1 = i0 + per < n ? i0 + per : n;
  double sxy = 0.0, sxx = 0.0, syy = 0.0;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const double a = (double)x[i], b = (double)y[i];
    sxy = fma(a, b, sxy);
    sxx = fma(a, a, sxx);
    syy = fma(b, b, syy);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sxy += __shfl_xor(sxy, o);
    sxx += __shfl_xor(sxx, o);
    syy += __shfl_xor(syy, o);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { s[0][w] = sxy; s[1][w] = sxx; s[2][w] = syy; }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int k = threadIdx.x;
    part[3 * blockIdx.x + k] = ((s[k][0] + s[k][1]) + s[k][2]) + s[k][3];
  }
}

// one wave: the partials in fixed order, then out = {sum xy, sum x^2, sum y^2, psnr, mse}
__global__ __launch_bounds__(64) void k_rel_final(const double* __restrict__ part, int n_part, double count,
                                                  int rel_scale, double peak, double* __restrict__ out) {
  double a[3] = {0.0, 0.0, 0.0};
  for (int i = threadIdx.x; i < n_part; i += 64)
#pragma unroll
    for (int k = 0; k < 3; ++k) a[k] += part[3 * i + k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int k = 0; k < 3; ++k) a[k] += __shfl_xor(a[k], o);
  if (threadIdx.x == 0) {
    const double sxy = a[0], sxx = a[1], syy = a[2];
    double mse;
    if (rel_scale == HBX_REL_LSQ) mse = (sxx > 0.0) ? (syy - sxy * sxy / sxx) / count : syy / count;
    else mse = (sxx - 2.0 * sxy + syy) / count;
    out[0] = sxy;
    out[1] = sxx;
    out[2] = syy;
    out[3] = psnr_from(sxy, sxx, syy, count, rel_scale, peak);
    out[4] = mse;
  }
}

}  // namespace

hipError_t launch_pack_mask(const void* src, int kind, int64_t n_words, int mode, double thr, uint64_t* bits,
                            int32_t* err, hipStream_t st) {
  if (n_words <= 0) return hipSuccess;
  const int64_t groups = (n_words + 3) / 4;
  const int64_t want = (groups + 3) / 4;   // 4 waves per workgroup
  const unsigned blocks = (unsigned)(want < 256 * 8 ? want : 256 * 8);
  switch (kind) {
    case HBX_SRC_U8:
      hipLaunchKernelGGL(k_pack_mask<HBX_SRC_U8>, dim3(blocks), dim3(256), 0, st, src, n_words, mode, thr, bits, err);
      break;
    case HBX_SRC_F32:
      hipLaunchKernelGGL(k_pack_mask<HBX_SRC_F32>, dim3(blocks), dim3(256), 0, st, src, n_words, mode, thr, bits, err);
      break;
    case HBX_SRC_F64:
      hipLaunchKernelGGL(k_pack_mask<HBX_SRC_F64>, dim3(blocks), dim3(256), 0, st, src, n_words, mode, thr, bits, err);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

int rel_partial_slots() { return kRelBlocks; }

hipError_t launch_rel_stats(const void* x, const void* y, int kind, int64_t n, double count, int rel_scale,
                            double peak, double* part, double* out, hipStream_t st) {
  const int64_t want = (n + 4095) / 4096;   // >= 4096 values per workgroup
  const unsigned blocks = (unsigned)(want < 1 ? 1 : (want < kRelBlocks ? want : kRelBlocks));
  if (kind == HBX_SRC_F32)
    hipLaunchKernelGGL(k_rel_partials<float>, dim3(blocks), dim3(256), 0, st, static_cast<const float*>(x),
                       static_cast<const float*>(y), n, part);
  else if (kind == HBX_SRC_F64)
    hipLaunchKernelGGL(k_rel_partials<double>, dim3(blocks), dim3(256), 0, st, static_cast<const double*>(x),
                       static_cast<const double*>(y), n, part);
  else
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_rel_final, dim3(1), dim3(64), 0, st, part, (int)blocks, count, rel_scale, peak, out);
  return hipGetLastError();
}

}  // namespace hbx
