// hbx_rowcol.hpp -- helpers shared by the row / column passes (hbx_passes.hip,
// hbx_passes896.hip): LDS tile swizzle, XCD-aware row-block order, buffer
// descriptors of wave-uniform planes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

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

// Field value of mask bit sh of word w for the row passes: va + vb * bit (hbx_api.hip's field
// kinds: amplitude 0 / 1, binary phase exp(i pi bit) = +-1).  The two kinds the plans use are
// built from the bit with two integer ops instead of extract + convert + fma (the same f32
// values bit for bit: fmaf(1, b, 0) = b, fmaf(-2, b, 1) = +-1.0f = 0x3F800000 with the sign
// bit b).  r06: k_rowfwd32 1,311 -> ~1,250 VALU and 168 -> 152 VGPRs per row block,
// 0.874-0.887 -> 0.852-0.873 ms alternated 4x on one box (profiles/r06/rowfwd_bitop_ab_r06o.txt).
enum { kFieldAmp = 0, kFieldPhase = 1, kFieldAny = 2 };
template <int FK>
__device__ __forceinline__ float bit_value(uint32_t w, int sh, float va, float vb) {
  if constexpr (FK == kFieldAmp) return (float)((w >> sh) & 1u);
  else if constexpr (FK == kFieldPhase) return __uint_as_float(((w << (31 - sh)) & 0x80000000u) | 0x3F800000u);
  else return fmaf(vb, (float)((w >> sh) & 1u), va);
}
// f(integral_constant<int, FK>) under a uniform branch on the plan's (va, vb)
template <class F>
__device__ __forceinline__ void with_field_kind(float va, float vb, F&& f) {
  if (va == 0.0f && vb == 1.0f) f(std::integral_constant<int, kFieldAmp>{});
  else if (va == 1.0f && vb == -2.0f) f(std::integral_constant<int, kFieldPhase>{});
  else f(std::integral_constant<int, kFieldAny>{});
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

// ---------------------------------------------------------------------------
// Staged slot-tile stores of the column passes (k_col2 at N = 1024 / 256, k_col896 since r04):
// the output line sets of a block (TL lines: group g = slot g of slot tile st, TileB) go out
// through the groups' FFT scratch regions.  The writer puts row y of its line at col2_pos(g / 2,
// y) of its OWN region (no block barrier); after a block barrier col2_stage_store stores the set
// as 16-B chunks (slots 2 sp, 2 sp + 1 from regions 2 sp, 2 sp + 1) in memory order -- one
// contiguous run per 16-row band.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int R>
constexpr int col2_region_stride() { return R * (R + 1) > R * R + 32 ? R * (R + 1) : R * R + 32; }
template <int R>
__device__ __forceinline__ float2* col2_region(float2* scratch, int g) {
  return scratch + g * col2_region_stride<R>();
}
// Where row y of slot pair sp's regions sits.  The readers (col2_stage_store) load the rows
// y0 = band * 16 + (tid / NSP) % 16 of the NSP = TL / 2 slot pairs sp = tid % NSP; gfx950 serves
// the compiler's ds_read2(st64)_b64 as 16-lane groups over 32 banks (16 float2: NSP pairs x
// 16 / NSP rows) and a ds_read_b64 as 32-lane groups over 64 banks (NSP pairs x 32 / NSP rows).
// A constant shift per pair cannot serve both (r03's (sp * 64 / TL) was the 64-bank one; the
// compiler emits read2st64, and rocprofv3 counted 67.1 M SQ_LDS_BANK_CONFLICT cycles per 128-job
// k_col2 launch = 8 extra cycles on each of the 32 stage reads per wave and line).  Shift sp by
// 32 / TL float2 and flip row bit 4 (+16 banks) when row bit HB (the bit splitting a 32-lane
// group's rows in halves) is set, except for the last pair: conflict-free in both models, and
// the writers' 16-lane runs of consecutive rows stay conflict-free (tools/lds_swizzle_model.py
// checks all three; found by exhaustive search over this family).
template <int R>
__device__ __forceinline__ int col2_pos(int sp, int y) {
  constexpr int TL = 256 / R, NSP = TL / 2, HB = ilog2c(16 / NSP);
  return sp * (32 / TL) + (y ^ ((((y >> HB) & 1) && sp != NSP - 1) ? 16 : 0));
}

template <int R, int N = R * R>
__device__ __forceinline__ void col2_stage_store(const float2* scratch, __amdgpu_buffer_rsrc_t rb, int st) {
  constexpr int TL = 256 / R, CH = N * TL / 2;   // 16-B chunks per line set (N = 896: R = 32's geometry)
  static_assert(CH % 256 == 0, "whole chunk rounds");
  // chunk c = tid + 256 i: band c / (8 TL) = tid / (8 TL) + (32 / TL) i, row (tid / (TL / 2)) % 16,
  // slot pair tid % (TL / 2); memory offset = lane part + i (32 / TL) 16 N + st 16 TL (soffset)
  const int tid = threadIdx.x, sp = tid % (TL / 2);
  const int band0 = tid / (8 * TL), r = (tid / (TL / 2)) % 16;
  const int y0 = band0 * 16 + r;
  // rows y0 + (32 / TL) 16 i differ from y0 in bits >= 5 only, so col2_pos moves with them
  static_assert((32 / TL) * 16 >= 32, "stage rows step past the swizzled bits");
  const float2* lo_r = col2_region<R>(const_cast<float2*>(scratch), 2 * sp) + col2_pos<R>(sp, y0);
  const float2* hi_r = col2_region<R>(const_cast<float2*>(scratch), 2 * sp + 1) + col2_pos<R>(sp, y0);
  const int voff = (band0 * 16 * N + r * TL + 2 * sp) * 8;
#pragma unroll
  for (int i = 0; i < CH / 256; ++i) {
    const float2 lo = lo_r[(32 / TL) * 16 * i];   // (rounded by col2_stage_write under SK)
    const float2 hi = hi_r[(32 / TL) * 16 * i];
    const u32x4 o = {__float_as_uint(lo.x), __float_as_uint(lo.y), __float_as_uint(hi.x), __float_as_uint(hi.y)};
    // non-temporal (nt): B streams out without taking Infinity-Cache residency, so its write-back
    // no longer lands on top of k_rowinv's reads (r03: N = 256 k_col2 0.143 -> 0.128 ms and
    // k_rowinv 0.140 -> 0.126; N = 1024 2.70 -> 2.66 and 1.474 -> 1.419).
    // soffset stays the literal 0, the whole offset rides in voffset: LLVM's gfx950 hazard
    // recognizer inserts the 2 wait states a VALU write of a >64-bit store's data VGPRs needs
    // only when the MUBUF soffset is not a register -- with an SGPR soffset (r03) it assumed no
    // hazard and scheduled such writes right behind the store, the cause of the r03 bf16
    // non-determinism and of the ITER = 1 wrong B rows (tools/hazard_scan.py
    // now rejects any wide buffer store with a register soffset)
    __builtin_amdgcn_raw_buffer_store_b128(o, rb, voff + (st * 16 * TL + i * (32 / TL) * 16 * N) * 8, 0, kBufNT);
  }
}

}  // namespace hbx
