// hbx_colbits.hip -- N = 1024 propagation without the row-spectrum intermediate.
//
// The three-pass path (hbx_passes.hip) writes the half spectrum A of every
// plane (4 N^2 B) in k_rowfwd and reads it back in the column pass: 64 MB of
// the 207 MB a 1024 x 8 job moves.  A is a function of 128 KB of mask bits,
// so here the column pass rebuilds the lines it needs from the bits instead:
//
//   k_bits_t   per plane row: the 32 x 32 bit transpose T(y, n2) = bits
//              {x = 32 n1 + n2} (bit n1), lane shuffles, flip applied; each
//              T word stored as 8 nibble-table offsets (one byte each)
//                                                    [read N^2/8, write N^2/4 B]
//   k_colbits  one block per (plane, spectral class): the 16 lines
//              kx = c + 64 m (m = 0..15) of class c are
//                F(c + 64 m, y) = sum_{n2<16} W16^{m n2} y_c(n2)
//                y_c(n2) = W1024^{c n2} (g(n2) + W64^c g(n2 + 16))
//                g(n2)   = sum_{n1<32} bit(32 n1 + n2) W32^{c n1}
//              (x = 32 n1 + n2; kx x = 32 c n1 + c n2 + 64 m n2 mod 1024).
//              g(n2) is 8 lookups in nibble tables of class c (16 entries
//              each: one LDS bank pair per entry, so the random lookups of a
//              lane group never conflict), then a 16-point DFT in registers
//              gives the 16 lines of one row.  Lines go through an LDS
//              staging area [16][1024] into the column layout, and each lane
//              group continues exactly like k_col2: FFT over y -> x H / x conj H
//              -> two inverse FFTs -> B lines kx and N - kx.
//                                                    [read N^2/4 (L2), write 8 N^2 B]
// Classes c = 1..31 carry 16 input lines each; their upper lines kx > 512
// are the Hermitian partners of class 64 - c, so classes 33..63 are never
// run.  Classes 0 and 32 (8 lines each, g shared: W32^{32 n1} = 1) share one
// block; its line kx = 0 carries F(0) + i F(512) like A's line 0.
//
// k_rowinv (hbx_passes.hip) then reads B unchanged.  Per 1024 x 8 job the
// path moves ~ 2 MB (bits, T) + 64 MB (B write) + 68 MB (B + target read)
// instead of 207 MB.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbx_fft.hpp"
#include "hbx_internal.hpp"

namespace hbx {

namespace {

constexpr int kN = 1024;
constexpr int kR = 32;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t cb_rsrc(const void* base, unsigned bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* p = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, 0x00020000);
}
typedef unsigned int cb_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2 cb_ld2(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
}
__device__ __forceinline__ void cb_st2(float2 v, __amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(cb_u32x2, v), rs, voff, soff, 0);
}

// nibble k of a 32-bit T word -> byte k of the code, value nibble * 8 (the
// byte offset of the entry in nibble table k)
__device__ __forceinline__ uint32_t nib_code(uint32_t v16) {
  // v16: 16 bits -> 4 bytes, byte k = ((v16 >> 4k) & 15) << 3
  uint32_t r = (v16 & 0xFu) | ((v16 & 0xF0u) << 4) | ((v16 & 0xF00u) << 8) | ((v16 & 0xF000u) << 12);
  return r << 3;
}

}  // namespace

// ---------------------------------------------------------------------------
// k_bits_t: 64 rows of one plane per 256-thread block.  A wave holds two rows
// (lanes 0-31, 32-63), lane n1 the 32-bit word n1; five xor-shuffle stages
// transpose the 32 x 32 bit block so lane n2 ends with T(n2) (bit n1 = bit n2
// of word n1).  Output tenc[plane][i < 16][y] (16 B) = codes of T(i), T(i+16).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bits_t(const JobDesc* __restrict__ jobs,
                                                const uint32_t* __restrict__ mask,
                                                uint4* __restrict__ tenc, int P, int CH) {
  constexpr int ROWS = 64;
  __shared__ uint2 tile[16][ROWS][2];
  const int bid = blockIdx.x;
  const int rb = bid % (kN / ROWS);
  const int pl = bid / (kN / ROWS);
  const int j = pl / P, p = pl % P;
  const JobDesc jb = jobs[j];
  if (jb.env < 0) return;
  const uint32_t* src = mask + ((size_t)jb.env * CH + (size_t)jb.group * P + p) * kN * 32;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int n1 = lane & 31;
  const bool flip_here = jb.flip_plane == p;
  const int fy = jb.flip_pix / kN, fx = jb.flip_pix % kN;
  for (int it = 0; it < ROWS / 8; ++it) {
    const int r = it * 8 + wave * 2 + (lane >> 5);
    const int y = rb * ROWS + r;
    uint32_t x = src[(size_t)y * 32 + n1];
    if (flip_here && fy == y && (fx >> 5) == n1) x ^= 1u << (fx & 31);   // env.py:164
#pragma unroll
    for (int st = 0; st < 5; ++st) {
      const int s = 16 >> st;
      const uint32_t m = st == 0 ? 0x0000FFFFu : st == 1 ? 0x00FF00FFu : st == 2 ? 0x0F0F0F0Fu
                       : st == 3 ? 0x33333333u : 0x55555555u;
      const uint32_t q = (uint32_t)__shfl_xor((int)x, s, 64);
      x = (n1 & s) ? ((x & ~m) | ((q >> s) & m)) : ((x & m) | ((q & m) << s));
    }
    // lane n2 = n1 now holds T(n2)
    tile[n1 & 15][r][n1 >> 4] = make_uint2(nib_code(x & 0xFFFFu), nib_code(x >> 16));
  }
  __syncthreads();
  uint4* dst = tenc + (size_t)pl * 16 * kN + rb * ROWS;
#pragma unroll
  for (int k = 0; k < 16 * ROWS / 256; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int i = e / ROWS, r = e % ROWS;
    const uint2 a = tile[i][r][0], b = tile[i][r][1];
    dst[(size_t)i * kN + r] = make_uint4(a.x, a.y, b.x, b.y);
  }
}

// ---------------------------------------------------------------------------
// k_colbits: 256 threads (8 lane groups) per block, two blocks per CU, so one
// block's row phase (LDS lookups) overlaps the other's column phase (HBM
// stores).  The block's 16 lines are processed in two batches of 8: the row
// phase stages batch 1 in LDS [8][1024] and keeps batch 2 in registers (4
// rows x 8 lines per thread) until batch 1's lines are done.
// LDS: twiddles (8 KB) + one region that is the staging area plus the class
// tables, then the 8 lane groups' transpose scratch (the k_col2 footprint).
// ---------------------------------------------------------------------------
constexpr int kNT = 256;
constexpr int kGrp = kNT / kR;                        // 8 lane groups
constexpr int kRows = kN / kNT;                       // rows per thread in the row phase
constexpr int kStage = kGrp * kN;                     // float2
constexpr int kScr = kGrp * kR * (kR + 1);            // float2
constexpr int kTabF2 = 128 + 2 * 17;                  // nibble tables + two fold sets
constexpr int kRegion = (kStage + kTabF2 > kScr) ? kStage + kTabF2 : kScr;

// 8 lookups: sum of the nibble-table entries selected by the 8 code bytes
__device__ __forceinline__ pk2 nib_sum(const float2* tab, uint32_t lo, uint32_t hi) {
#ifdef HBX_CB_NO_LOOKUP   // timing experiment: arithmetic stand-in for the 8 LDS lookups
  return (pk2){__uint_as_float(lo & 0x3f0f0f0fu), __uint_as_float(hi & 0x3f0f0f0fu)};
#endif
  const char* tb = reinterpret_cast<const char*>(tab);
  pk2 s0 = to_pk(*reinterpret_cast<const float2*>(tb + 0 * 128 + (lo & 0xFFu)));
  pk2 s1 = to_pk(*reinterpret_cast<const float2*>(tb + 1 * 128 + ((lo >> 8) & 0xFFu)));
  pk2 s2 = to_pk(*reinterpret_cast<const float2*>(tb + 2 * 128 + ((lo >> 16) & 0xFFu)));
  pk2 s3 = to_pk(*reinterpret_cast<const float2*>(tb + 3 * 128 + (lo >> 24)));
  pk2 s4 = to_pk(*reinterpret_cast<const float2*>(tb + 4 * 128 + (hi & 0xFFu)));
  pk2 s5 = to_pk(*reinterpret_cast<const float2*>(tb + 5 * 128 + ((hi >> 8) & 0xFFu)));
  pk2 s6 = to_pk(*reinterpret_cast<const float2*>(tb + 6 * 128 + ((hi >> 16) & 0xFFu)));
  pk2 s7 = to_pk(*reinterpret_cast<const float2*>(tb + 7 * 128 + (hi >> 24)));
  return ((s0 + s1) + (s2 + s3)) + ((s4 + s5) + (s6 + s7));
}

// one input line through the column pass (as k_col2): FFT over y -> x H and
// x conj H -> two inverse FFTs -> B lines kx and N - kx (N/2 for dc)
__device__ __forceinline__ void col_line(float2 (&v)[kR], int kx, bool dc, int t,
                                         const PaddedScratch<kR>& sc, const float2* tw,
                                         __amdgpu_buffer_rsrc_t rh, __amdgpu_buffer_rsrc_t rb) {
  using PB = PanelLine<kR, kN, pan_b(kR)>;
  const float2* mrow = sc.at((kR - t) & (kR - 1), 0) + (t == 0 ? 1 : 0) + (kR - 1);
  const int hrow = kx <= kN / 2 ? kx : kN - kx;   // H is even in fx
  const int vh = (hrow * kN + t) * 8;
  fft_group<kR, false, true>(v, t, sc, tw);
  wave_sync();
  if (!dc) {
#pragma unroll
    for (int c8 = 0; c8 < kR; c8 += 8) {
      float2 hb[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) hb[i] = cb_ld2(rh, vh, (c8 + i) * kR * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int k2 = c8 + i;
        const float2 w = cmulc(v[k2], hb[i]);
        *sc.at(t, k2) = w;
        if (k2 == 0) *sc.at(t, kR) = w;
        v[k2] = cmul(v[k2], hb[i]);
      }
    }
  } else {
#pragma unroll
    for (int k2 = 0; k2 < kR; ++k2) *sc.at(t, k2) = v[k2];
    *sc.at(t, kR) = v[0];
  }
  wave_sync();
  float2 m[kR];
#pragma unroll
  for (int k2 = 0; k2 < kR; ++k2) m[k2] = conjf2(mrow[-k2]);
  if (dc) {   // (Z + M)/2 H(0) -> line 0, -i (Z - M)/2 H(N/2) -> line N/2
    const int vn = ((kN / 2) * kN + t) * 8;
#pragma unroll
    for (int k2 = 0; k2 < kR; ++k2) {
      const float2 z = v[k2], mm = m[k2];
      v[k2] = cmul(make_float2(0.5f * (z.x + mm.x), 0.5f * (z.y + mm.y)), cb_ld2(rh, vh, k2 * kR * 8));
      m[k2] = cmul(make_float2(0.5f * (z.y - mm.y), -0.5f * (z.x - mm.x)), cb_ld2(rh, vn, k2 * kR * 8));
    }
  }
  fft_group<kR, true, true>(v, t, sc, tw);
  {
    const int vo = PB::voff(t, kx);
#pragma unroll
    for (int k2 = 0; k2 < kR; ++k2) cb_st2(v[k2], rb, vo, PB::joff(k2));
  }
  fft_group<kR, true, true>(m, t, sc, tw);
  {
    const int vo = PB::voff(t, dc ? kN / 2 : kN - kx);
#pragma unroll
    for (int k2 = 0; k2 < kR; ++k2) cb_st2(m[k2], rb, vo, PB::joff(k2));
  }
}

__global__ __launch_bounds__(kNT, 2) void k_colbits(const JobDesc* __restrict__ jobs,
                                                    const uint4* __restrict__ tenc,
                                                    float2* __restrict__ ws_b,
                                                    const float2* __restrict__ htab,
                                                    const float2* __restrict__ tw_glob, int P,
                                                    int n_jobs, float va, float vb) {
  __shared__ float2 tw[kN];
  __shared__ __attribute__((aligned(16))) float2 region[kRegion];
  float2* stage = region;
  float2* tab = region + kStage;          // [8][16] nibble tables (x vb)
  float2* fold = tab + 128;               // [2][17]: W1024^{c n2} (n2 < 16), W64^c

  // block -> (job, plane, slot): with n_jobs % 8 == 0, XCD x (blocks b = x mod 8)
  // takes whole jobs j = x mod 8, so a job's planes reuse one group's H rows
  // and a plane's 32 blocks share its T plane in one L2 (speed hint only)
  const int NB = 32 * P;                  // blocks per job
  int b = blockIdx.x, j, rem;
  if ((n_jobs & 7) == 0) {
    const int x = b & 7, r = b >> 3;
    j = x + 8 * (r / NB);
    rem = r % NB;
  } else {
    j = b / NB;
    rem = b % NB;
  }
  const int p = rem / 32;
  const int s = rem % 32;                 // class slot: 0 = classes {0, 32}, else class s
  const JobDesc jb = jobs[j];
  if (jb.env < 0) return;                 // uniform per block
  const int pl = j * P + p;

  for (int i = threadIdx.x; i < kN; i += kNT) tw[i] = tw_glob[i];
  {
    const float2* ct = tw_glob + kTwClassOff + s * kTwClassStride;   // class s (s = 0: k1 = 0)
    if (threadIdx.x < 128) tab[threadIdx.x] = make_float2(vb * ct[threadIdx.x].x, vb * ct[threadIdx.x].y);
    else if (threadIdx.x < 128 + 17) fold[threadIdx.x - 128] = ct[threadIdx.x];
    else if (threadIdx.x < 128 + 34) {   // merged block: class 32's fold set
      const float2* c32t = tw_glob + kTwClassOff + 32 * kTwClassStride;
      fold[threadIdx.x - 128] = c32t[threadIdx.x - 17];
    }
  }
  __syncthreads();

  // ---- row phase: the block's 16 lines of every row; batch 1 -> staging, batch 2 -> held
  const uint4* tp = tenc + (size_t)pl * 16 * kN;
  const bool merged = (s == 0);
  float2 held[kRows][8];
#ifndef HBX_CB_NO_P1   // timing experiment: column phase alone
#pragma unroll
  for (int rr = 0; rr < kRows; ++rr) {
    const int y = threadIdx.x + kNT * rr;
    uint4 e[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) e[i] = tp[(size_t)i * kN + y];
    if (!merged) {
      const pk2 w64 = to_pk(fold[16]);
      pk2 acc[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const pk2 ga = nib_sum(tab, e[i].x, e[i].y);
        const pk2 gb = nib_sum(tab, e[i].z, e[i].w);
        acc[i] = pk_cmul(ga + pk_cmul(gb, w64), to_pk(fold[i]));
        asm volatile("" ::: "memory");   // keep the lookup addresses of one chunk live at a time
      }
      dft_reg<16, false>(acc);
#pragma unroll
      for (int m = 0; m < 8; ++m) stage[m * kN + y] = from_pk(acc[m]);
#pragma unroll
      for (int m = 0; m < 8; ++m) held[rr][m] = from_pk(acc[8 + m]);
    } else {
      pk2 a0[16], a32[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const pk2 ga = nib_sum(tab, e[i].x, e[i].y);
        const pk2 gb = nib_sum(tab, e[i].z, e[i].w);
        a0[i] = ga + gb;                                    // class 0: W1024^0 = W64^0 = 1
        a32[i] = pk_cmul(ga - gb, to_pk(fold[17 + i]));    // class 32: W64^32 = -1
        asm volatile("" ::: "memory");
      }
      dft_reg<16, false>(a0);
      dft_reg<16, false>(a32);
      // line 0 slot: F(0) + i F(512), both real (va: the constant field's DC)
      stage[y] = make_float2(a0[0].x + va * (float)kN, a0[8].x);
#pragma unroll
      for (int m = 1; m < 8; ++m) stage[m * kN + y] = from_pk(a0[m]);
#pragma unroll
      for (int m = 0; m < 8; ++m) held[rr][m] = from_pk(a32[m]);
    }
  }
#else
#pragma unroll
  for (int rr = 0; rr < kRows; ++rr)
#pragma unroll
    for (int m = 0; m < 8; ++m) held[rr][m] = make_float2(0.f, 0.f);
#endif
  __syncthreads();
#ifdef HBX_CB_NO_P2   // timing experiment: row phase alone (values kept live)
  if (threadIdx.x == 0) {
    float2 a = stage[s * 37 + 5];
#pragma unroll
    for (int rr = 0; rr < kRows; ++rr)
#pragma unroll
      for (int m = 0; m < 8; ++m) a = cadd(a, held[rr][m]);
    ws_b[(size_t)pl * plane_b_elems(kR) + s] = a;
  }
  return;
#endif

  // ---- column phase: one lane group per line, two batches
  const int grp = threadIdx.x / kR;
  const int t = threadIdx.x % kR;
  const __amdgpu_buffer_rsrc_t rb = cb_rsrc(ws_b + (size_t)pl * plane_b_elems(kR), plane_b_elems(kR) * 8);
  const __amdgpu_buffer_rsrc_t rh = cb_rsrc(htab + (size_t)jb.group * (kN / 2 + 1) * kN, (kN / 2 + 1) * kN * 8);
  const PaddedScratch<kR> sc{region + grp * kR * (kR + 1)};
  float2 v[kR];
#pragma unroll
  for (int jj = 0; jj < kR; ++jj) v[jj] = stage[grp * kN + t + kR * jj];
  lds_barrier();   // staging consumed: the region becomes the transpose scratch
  col_line(v, merged ? 64 * grp : s + 64 * grp, merged && grp == 0, t, sc, tw, rh, rb);

  lds_barrier();   // every group is done with its scratch: stage batch 2
#pragma unroll
  for (int rr = 0; rr < kRows; ++rr)
#pragma unroll
    for (int m = 0; m < 8; ++m) stage[m * kN + threadIdx.x + kNT * rr] = held[rr][m];
  lds_barrier();
#pragma unroll
  for (int jj = 0; jj < kR; ++jj) v[jj] = stage[grp * kN + t + kR * jj];
  lds_barrier();
  col_line(v, merged ? 32 + 64 * grp : s + 64 * (8 + grp), false, t, sc, tw, rh, rb);
}

hipError_t launch_colbits(const PlanDev& pd, const JobDesc* jobs, int n_jobs, const uint32_t* mask,
                          hipStream_t st) {
  const int P = pd.P;
  uint4* tenc = reinterpret_cast<uint4*>(pd.ws_a);   // 2 MB per job, inside A's 32 MB
  PassTimer* tm = pd.timer;
  if (tm) tm->begin(0, st);
  hipLaunchKernelGGL(k_bits_t, dim3((unsigned)n_jobs * P * (kN / 64)), dim3(256), 0, st, jobs, mask, tenc, P,
                     pd.G * P);
  if (tm) tm->end(0, n_jobs, st);
  if (tm) tm->begin(1, st);
  hipLaunchKernelGGL(k_colbits, dim3((unsigned)n_jobs * P * 32), dim3(kNT), 0, st, jobs, tenc, pd.ws_b, pd.htab,
                     pd.tw, P, n_jobs, pd.va, pd.vb);
  if (tm) tm->end(1, n_jobs, st);
  return hipGetLastError();
}

}  // namespace hbx
