// hbx_rowcol.hpp -- helpers shared by the row / column passes (hbx_passes.hip,
// hbx_passes896.hip): LDS tile swizzle, XCD-aware row-block order, buffer
// descriptors of wave-uniform planes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbx_fft.hpp"

namespace hbx {

// Position of element (line, r) in an LDS tile [line][GPB rows], r XOR-swizzled
// by a function of (line mod R) only: lane t of a group reading line t + R*j
// then addresses base_t + j*R*GPB (immediate offsets, no per-j address VGPRs),
// ds_read_b64 is conflict-free and ds_write_b64 at most 2-way (checked
// exhaustively for R = 8, 16, 32).
template <int R, int GPB = 256 / R>
__device__ __forceinline__ int tile_pos(int line, int r) {
  if constexpr (GPB == 16) {
    // 16 rows (512-thread blocks, N = 1024): swizzle (line mod 16) ^ bit 4 of
    // line -- conflict-free for the lane-row reads / writes and the 16-B chunk
    // writes; the chunk reads of k_rowfwd stay 2-way (checked exhaustively)
    return line * GPB + (r ^ (((line & 15) ^ ((line >> 4) & 1)) & (GPB - 1)));
  } else if constexpr (R == 32 && GPB == 8) {
    // q ^ 5 b1 (q = bits 2-4 of line, b1 = bit 1): the lane-row reads stay
    // conflict-free (bijective in q for fixed line mod 4) and the two b64
    // writes -- lane rows t + 32 k2 (16-lane groups: bijective in bits 1-3)
    // and the 16-B chunk pairs of 4 consecutive lines (the b1 term flips the
    // parity) -- lose their 2-way conflicts (tools/lds_swizzle_model.py)
    return line * GPB + (r ^ ((((line & 31) >> 2) ^ (((line >> 1) & 1) * 5)) & 7));
  } else {
    constexpr int SR = ilog2c(32 / GPB);
    constexpr int SL = ilog2c(GPB / 8);
    return line * GPB + (r ^ ((((line & (R - 1)) >> SR) << SL) & (GPB - 1)));
  }
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// buffer descriptor of a wave-uniform plane (cdna_hip_programming.md T8 recipe)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const void* base, unsigned bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* p = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ float2 buf_ld2(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
}

__device__ __forceinline__ void buf_st2(float2 v, __amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rs, voff, soff, 0);
}

// The once-touched intermediate streams: loads keep the default cache policy (non-temporal
// loads slowed k_rowinv 1.80 -> 2.21 ms, r01); the row spectrum A and the column output B are
// STORED non-temporal since r03 -- with B in slot tiles and A read by k_col2 right after,
// default-policy stores left their dirty lines in the Infinity Cache to be written back during
// the next pass (N = 1024 headline 24.9k -> 25.9k (B) -> 26.1k (A and B) on one box; N = 256
// k_rowinv 0.140 -> 0.100 ms).  (r01, before the tiles: nt A stores 1.17 -> 1.27 ms.)
__device__ __forceinline__ float2 buf_ld2s(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
}
__device__ __forceinline__ void buf_st2s(float2 v, __amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rs, voff, soff, 0);
}
__device__ __forceinline__ float4 ld_stream4(const float2* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st_stream4(float2* p, float4 v) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4*>(p));
}
// cache-policy bit of buffer instructions (gfx950 aux operand): nt = non-temporal
constexpr int kBufNT = 2;

// Workgroups b, b+8, b+16, ... land on the same XCD (round-robin dispatch over
// the 8 XCDs; placement is a speed hint only, never relied on for
// correctness).  The row passes touch 64-B pieces of every 8-KB line, the
// piece for rows y0..y0+7: keep GS consecutive row blocks on one XCD so each
// line is read / written as GS*64 contiguous bytes through one L2.  Measured
// on 1024x24, 128 envs (k_rowfwd / k_rowinv ms): no remap 1.34 / 2.75,
// GS=2 1.18 / 2.43, GS=4 1.17 / 2.40, GS=8 1.12 / 2.08, GS=16 1.12 / 1.98.
constexpr int kXcdGroup = 16;
template <int RB>
__device__ __forceinline__ int xcd_pair(int bid) {
  constexpr int GS = (RB / 8 < kXcdGroup) ? RB / 8 : kXcdGroup;
  constexpr int SPAN = 8 * (GS > 0 ? GS : 1);
  if constexpr (GS > 1 && RB % SPAN == 0)
    return (bid / SPAN) * SPAN + (bid % 8) * GS + (bid / 8) % GS;
  else return bid;
}

}  // namespace hbx
