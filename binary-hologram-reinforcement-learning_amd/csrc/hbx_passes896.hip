// hbx_passes896.hip -- the fused three-pass propagation at N = 896, the
// 64-pixel centre crop of a 1024 mask that env_1024_24_128.py:144-149 and
// DBS_1024_24-128.py:210-216 propagate.
//
// Same structure as the N = R^2 passes (hbx_passes.hip), on the 28 x 32
// lane-group FFT of hbx_fft.hpp (natural layout: lane t < 32, register j < 28
// holds x[t + 32 j]; slot layout: lane k1 < 28, register k2 < 32 holds
// X[k1 + 28 k2]):
//
//   k_rowfwd896  8 rows of a plane pair per block: bits -> one complex FFT
//                per row pair (plane a real, plane b imaginary) -> Hermitian
//                split -> half spectrum kx < 448 (Nyquist in Im of kx = 0) ->
//                LDS tile transpose -> A[kx][y0..y0+8)   [read N^2/8, write 4 N^2 B per plane]
//   k_col896     one lane group per half-spectrum line kx: FFT over y ->
//                x H and x conj H (H even in fx and ky) -> two IFFTs -> B lines
//                kx and N - kx (448 for kx = 0)           [read 4 N^2, write 8 N^2]
//   k_rowinv896  8 rows per block, all P planes: LDS tile transpose of the B
//                rows (next plane prefetched) -> IFFT over kx -> |U|^2 -> plane
//                mean -> f64 partials of (I T, I^2, T^2)  [read 8 N^2 per plane + 4 N^2]
//
// A is [kx < 448][y], B is [kx < 896][y] (column-major lines).  It replaced
// a composed path (2-D FFTs around a transfer-function pass, removed in r03),
// which moved ~10 plane-sized round trips per job instead of 3.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbx_fft.hpp"
#include "hbx_internal.hpp"
#include "hbx_rowcol.hpp"

namespace hbx {

namespace {

constexpr int kN = 896;
constexpr int kR = 32;                         // lanes per group
constexpr int kL = 28;                         // slot lanes / natural registers
constexpr int kGPB = 8;                        // rows (lines) per 256-thread block
constexpr int kRB = kN / kGPB;                 // 112 row blocks
constexpr int kHalf = kN / 2;                  // 448 half-spectrum lines
constexpr size_t kPlaneA = (size_t)kHalf * kN;
constexpr size_t kPlaneB = (size_t)kN * kN;
constexpr int kSCR = kGPB * kR * (kR + 1);     // padded transpose scratch
constexpr int kWPR = kN / 32;                  // 32-bit mask words per row (28)
static_assert(kN * kGPB <= kSCR, "the row tile must fit in the scratch area");

// conj Z[N - k] for the slot-layout element k = k1 + 28 k2 (lane k1 < 28,
// register k2): lane 28 - k1, register 31 - k2; lane 0 keeps its own
// register (32 - k2) mod 32.  Lanes 28..31 get don't-care values.
__device__ __forceinline__ float2 mirror_conj896(const float2 (&v)[32], int k2, int t, int lane_base) {
  const int src = lane_base + ((t > 0 && t < kL) ? kL - t : 0);
  float2 p;
  p.x = __shfl(v[31 - k2].x, src, 64);
  p.y = __shfl(v[31 - k2].y, src, 64);
  const float2 own = v[(32 - k2) & 31];
  return conjf2(t == 0 ? own : p);
}

}  // namespace

// ---------------------------------------------------------------------------
// Pass 1 (r04: k_rowfwd32's scheme at 896)
// ---------------------------------------------------------------------------
// A at 896 is stored in panels of the row block height, [y / 8][kx < 448][y % 8] (r01-r03:
// line-major [kx][y], i.e. 64-B pieces of every line per row block -- the access shape that
// replayed at 1.19-1.24 ms against 0.69 ms for contiguous panels at N = 1024, DESIGN.md 4;
// k_rowfwd896 ran at 0.40 of 8 TB/s).  A row block now writes one contiguous 28-KB panel per
// plane, and k_col896's lane groups read 64-B pieces of 8 consecutive y.
__host__ __device__ constexpr size_t a896_at(int kx, int y) {
  return (size_t)(y >> 3) * (kHalf * kGPB) + (size_t)kx * kGPB + (y & 7);
}

// Three workgroups per CU, as k_rowfwd32 (hbx_passes.hip): lane t < 28 loads mask word t of
// its row (lanes 28..31 re-load word 27; their bits land in bits 28..31 of the transposed
// words, x >= 896, never used) and group_bit_transpose hands lane t bit t of every word;
// the FFT transposes real then imaginary parts through a 4.2-KB float tile per group
// (fft896_ns_split); the Hermitian split goes out one plane at a time through a 28-KB tile
// aliasing those FFT tiles; each workgroup walks RIT896 row blocks of one plane pair with the
// next rows' words loaded before the stores; A is stored non-temporal.
// Tile of one plane's half spectrum [kx < 448][8 rows] for k_rowfwd896, row r XOR-swizzled by
// a function of kx mod 28: the lane-row writes (lane t: kx = t + 28 k2) then address one
// lane base + k2 * 28 * 8 (tile_pos<32, 8>'s swizzle keys on kx mod 32, which pinned 16 address
// VGPRs and spilled at three workgroups per CU), and are conflict-free; the 16-B chunk reads
// are conflict-free as 16-lane read2 and 16 extra cycles per 56 reads as ds_read_b64
// (exhaustive search over ((m >> a) & 7) ^ b * bit c of m, tools/lds_swizzle_model.py)
__device__ __forceinline__ int tile896_pos(int kx, int r) {
  const int m = kx % kL;
  return kx * kGPB + (r ^ ((((m >> 2) & 7) ^ (((m >> 1) & 1) * 5)) & 7));
}

// row blocks per workgroup (112 / 8 = 14 per pair).  r04 A/B (profiles/r04/rit896_ab_r04g.txt,
// crop k_rowfwd896 per 128-job launch): 2 -> 0.731 ms, 4 -> 0.728-0.731, 7 -> 0.711, 8 -> 0.704
constexpr int kRit896 = 8;
static_assert(kRB % kRit896 == 0, "row-block walk");

__global__ __launch_bounds__(256, 3) void k_rowfwd896(const JobDesc* __restrict__ jobs,
                                                      const uint32_t* __restrict__ mask,
                                                      float2* __restrict__ ws_a,
                                                      const float2* __restrict__ tw_glob, int P, int CH,
                                                      float va, float vb, int pair_step) {
  constexpr int SCRF = kGPB * kR * (kR + 1);      // floats: 8 FFT tiles (33.8 KB)
  static_assert(kHalf * kGPB * 2 <= SCRF, "one plane's tile must fit in the FFT tiles");
  constexpr int RBW = kRB / kRit896;
  __shared__ float2 tw[kN];
  __shared__ __attribute__((aligned(16))) float lds[SCRF];
  for (int i = threadIdx.x; i < kN; i += 256) tw[i] = tw_glob[i];

  const int grp = threadIdx.x / kR;
  const int t = threadIdx.x % kR;
  const int lane_base = (threadIdx.x & 63) - t;
  int bid = blockIdx.x;
  const int rbw = bid % RBW;
  bid /= RBW;
  const int npair = pair_step ? 1 : P / 2;   // (r06) plane-cached step: only the flipped plane's pair
  const int j = bid / npair;
  const JobDesc jb = jobs[j];
  if (jb.env < 0) return;  // uniform per block
  const int q = pair_step ? (jb.flip_plane >> 1) : bid % npair;
  const int pa = 2 * q, pb = 2 * q + 1;
  const uint32_t* plane_a = mask + ((size_t)jb.env * CH + jb.group * P + pa) * kN * kWPR;
  const int wt = t < kWPR ? t : kWPR - 1;
  uint32_t wa, wb;
  auto load_row = [&](int y) {
    wa = plane_a[(size_t)y * kWPR + wt];
    wb = plane_a[(size_t)(kN + y) * kWPR + wt];
  };
  load_row(rbw * kRit896 * kGPB + grp);
  __syncthreads();  // tw visible

  float2* base = ws_a + ((size_t)j * P + pa) * kPlaneA;
  float2* tile = reinterpret_cast<float2*>(lds);
  constexpr int CHUNKS = kHalf * kGPB / 2;      // 16-B chunks of one plane's panel (1792)
  static_assert(CHUNKS % 256 == 0, "chunking");
#pragma unroll 1
  for (int it = 0; it < kRit896; ++it) {
    const int y0 = (rbw * kRit896 + it) * kGPB;
    const int y = y0 + grp;
    uint32_t ta = group_bit_transpose(wa, t);   // bit r = pixel x = t + 32 r of the row
    uint32_t tb = group_bit_transpose(wb, t);
    if (jb.flip_plane >= 0 && jb.flip_pix / kN == y) {  // env.py:164 flip, on the fly
      const int col = jb.flip_pix % kN;
      if (t == (col & 31)) {
        if (jb.flip_plane == pa) ta ^= 1u << (col >> 5);
        if (jb.flip_plane == pb) tb ^= 1u << (col >> 5);
      }
    }
    float2 v[32];
    with_field_kind(va, vb, [&](auto fk) {
#pragma unroll
      for (int jj = 0; jj < kL; ++jj)
        v[jj] = make_float2(bit_value<fk()>(ta, jj, va, vb), bit_value<fk()>(tb, jj, va, vb));
    });
#pragma unroll
    for (int jj = kL; jj < 32; ++jj) v[jj] = make_float2(0.f, 0.f);
    // next rows' words (the last iteration re-reads its own row: no conditional load)
    load_row(it + 1 < kRit896 ? y + kGPB : y);
    if (it > 0) lds_barrier();   // every group has read the previous plane-b tile
    fft896_ns_split<false>(v, t, lds + grp * kR * (kR + 1), tw);

    // Hermitian split of the slot-layout spectrum (kx = t + 28 k2 < 448: k2 < 16): plane a
    // now, plane b kept in registers for the second tile
    float2 fb[16];
    lds_barrier();    // every group is done with its FFT tile: reuse as the plane tile
    const float2 zny = v[16];  // Z[448] on lane 0
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) {
      const float2 z = v[k2];
      const float2 m = mirror_conj896(v, k2, t, lane_base);
      float2 fa = make_float2(z.x + m.x, z.y + m.y);       // 2 A (htab holds H / 2)
      fb[k2] = make_float2(z.y - m.y, m.x - z.x);
      if (k2 == 0 && t == 0) {  // DC and Nyquist of a real row are real
        fa = make_float2(z.x + z.x, zny.x + zny.x);
        fb[k2] = make_float2(z.y + z.y, zny.y + zny.y);
      }
      if (t < kL) tile[tile896_pos(t + kL * k2, grp)] = fa;
    }
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) {
      if (pl == 1) {
        lds_barrier();   // plane a's tile has been read
#pragma unroll
        for (int k2 = 0; k2 < 16; ++k2)
          if (t < kL) tile[tile896_pos(t + kL * k2, grp)] = fb[k2];
      }
      lds_barrier();
      float2* panel = base + (size_t)pl * kPlaneA + a896_at(0, y0);
#pragma unroll
      for (int i = 0; i < CHUNKS / 256; ++i) {
        const int c = threadIdx.x + 256 * i;
        const int r2 = (c % (kGPB / 2)) * 2;
        const int line = c / (kGPB / 2);
        // rows r2, r2 + 1 of the line sit in one aligned 16-B pair (the XOR swizzle permutes whole
        // pairs; its bit 0 swaps the two halves): one ds_read_b128, whose 16-lane groups cover
        // four whole lines -- conflict-free for any swizzle inside a line (r05; two ds_read_b64
        // cost 16 extra LDS cycles per 56 reads, 1.8 M per 128-job launch)
        const int p0 = tile896_pos(line, r2);
        const float4 ab = *reinterpret_cast<const float4*>(tile + (p0 & ~1));
        const bool sw = (p0 & 1) != 0;
        st_stream4(panel + 2 * c, sw ? make_float4(ab.z, ab.w, ab.x, ab.y) : ab);   // = a896_at(line, y0 + r2)
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Pass 2 (r04: k_col2's scheme at 896): one lane group per input line and both of its
// output lines.  FFT over y -> Z (slot layout); H(kx, ky) for ky <= 448 only (17 of 32
// registers; H is even in ky, the other 15 come mirrored through the group's scratch);
// v <- Z H -> IFFT -> B line kx; w <- Z conj H -> IFFT -> conj -> B line N - kx (the
// conjugate-even identity of k_col2, no mirror of the line).  kx = 0: (Z + M)/2 H(0) ->
// line 0, -i (Z - M)/2 H(448) -> line 448 with M = conj Z(-ky) from a register shuffle.
// XCD-aware lines: the 8 line blocks of a plane are blockIdx % 8, i.e. one per XCD (blocks
// are dispatched round-robin over the 8 XCDs; placement is a speed hint only), so an XCD
// touches only its 56 of the 448 H rows of each colour group -- 0.2 MB per group in its
// 4-MB L2 instead of the whole 3.2-MB table (r03: 1.22x the algorithmic bytes, the H rows
// re-fetched across jobs of different colour groups).
// ---------------------------------------------------------------------------
constexpr int kColIter = 7;
constexpr int kColLB = kHalf / (kGPB * kColIter);   // 8 line blocks per plane = one per XCD
static_assert(kHalf % (kGPB * kColIter) == 0 && kColLB == 8, "line blocking");

// each group writes its output line (natural layout: lane t, register j -> row t + 32 j) into its
// own scratch region at col2_pos (hbx_rowcol.hpp); rows 32 apart share a lane base
__device__ __forceinline__ void col896_stage_write(const float2 (&v)[32], float sy, float2* scratch, int grp,
                                                   int t) {
  float2* base = col2_region<kR>(scratch, grp) + col2_pos<kR>(grp >> 1, t);
#pragma unroll
  for (int jj = 0; jj < kL; ++jj) base[kR * jj] = make_float2(v[jj].x, sy * v[jj].y);
}

__global__ __launch_bounds__(256, 2) void k_col896(const JobDesc* __restrict__ jobs,
                                                   const float2* __restrict__ ws_a,
                                                   float2* __restrict__ ws_b,
                                                   const float2* __restrict__ htab,
                                                   const float2* __restrict__ tw_glob, int P, int pair_step) {
  __shared__ float2 tw[kN];
  __shared__ float2 scratch[kSCR];
  for (int i = threadIdx.x; i < kN; i += 256) tw[i] = tw_glob[i];

  const int grp = threadIdx.x / kR;
  const int t = threadIdx.x % kR;
  const int lane_base = (threadIdx.x & 63) - t;
  int bid = blockIdx.x;
  const int lb = bid % kColLB;
  bid /= kColLB;
  const int np = pair_step ? 2 : P;     // (r06) plane-cached step: the flipped plane's pair only
  const int j = bid / np;
  const JobDesc jb = jobs[j];
  if (jb.env < 0) return;
  const int p = pair_step ? (jb.flip_plane & ~1) + bid % 2 : bid % np;
  const __amdgpu_buffer_rsrc_t ra = plane_rsrc(ws_a + ((size_t)j * P + p) * kPlaneA, (unsigned)(kPlaneA * 8));
  const __amdgpu_buffer_rsrc_t rb = plane_rsrc(ws_b + ((size_t)j * P + p) * kPlaneB, (unsigned)(kPlaneB * 8));
  const __amdgpu_buffer_rsrc_t rh = plane_rsrc(htab + (size_t)jb.group * (kHalf + 1) * kN,
                                               (unsigned)((kHalf + 1) * kN * 8));
  static_assert(col2_region_stride<kR>() == kR * (kR + 1), "stage regions are the FFT scratch regions");
  float2* const hs = scratch + grp * kR * (kR + 1);
  const PaddedScratch<kR> sc{hs};
  const int k1 = t < kL ? t : 0;   // slot lane (28..31 carry don't-care values)
  // the mirror of ky = k1 + 28 k2 (k2 > 16) is 896 - ky = (28 - k1) + 28 (31 - k2), lane 0:
  // 28 (32 - k2); the group writes its ky <= 448 values as hs[k2 * 28 + lane] (lanes < 28; r05:
  // rows of 28, not 32 -- with 32 lane 0's read hit lane 12's bank, 30 extra LDS cycles per wave
  // and line; lanes 28..31 read don't-care values on the four banks no other lane uses)
  const float2* hm = hs + (t == 0 ? kL : ((kL - t) & 31));
  // A line kx of a panel plane as seen by lane t: y = t + 32 jj -> a896_at(kx, t) + jj * 4 panels
  const int lane_a = (int)a896_at(0, t) * 8;
  constexpr int JSTEP = 4 * kHalf * kGPB * 8;   // bytes between registers jj and jj + 1
  constexpr int KSTEP = kColLB * kGPB;
  const int kx0 = lb * kGPB + grp;

  float2 v[32];
#pragma unroll
  for (int jj = 0; jj < kL; ++jj) v[jj] = buf_ld2s(ra, lane_a + kx0 * kGPB * 8, jj * JSTEP);
#pragma unroll
  for (int jj = kL; jj < 32; ++jj) v[jj] = make_float2(0.f, 0.f);
  lds_barrier();  // tw visible (the line loads stay in flight)

#pragma unroll 1
  for (int it = 0; it < kColIter; ++it) {
    const int kx = kx0 + it * KSTEP;
    const bool dc = (kx == 0);
    const int vh = (kx * kN + k1) * 8;   // H(kx, ky = k1 + 28 k2) at vh + k2 * 28 * 8
    float2 hb[32];
    fft896_ns_s1<false, true>(v, t, tw);
    if (!dc) {   // H(kx, ky <= 448), in flight under the transpose
#pragma unroll
      for (int i = 0; i <= 16; ++i) hb[i] = buf_ld2(rh, vh, i * kL * 8);
    }
    if (it > 0) lds_barrier();   // the previous iteration's second set has been read out
    fft896_ns_s2<false, true>(v, t, sc);
    float2 w[32];
    if (!dc) {
      wave_sync();
      if (t < kL) {
#pragma unroll
        for (int i = 0; i <= 16; ++i) hs[i * kL + t] = hb[i];
      }
      wave_sync();
#pragma unroll
      for (int i = 17; i < 32; ++i) hb[i] = hm[(31 - i) * kL];
      wave_sync();
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        w[i] = cmulc(v[i], hb[i]);
        v[i] = cmul(v[i], hb[i]);
      }
    } else {
      const int vn = (kHalf * kN + k1) * 8;
#pragma unroll
      for (int k2 = 0; k2 < 32; ++k2) w[k2] = mirror_conj896(v, k2, t, lane_base);
#pragma unroll
      for (int k2 = 0; k2 < 32; ++k2) {
        const float2 z = v[k2], mm = w[k2];
        v[k2] = cmul(make_float2(0.5f * (z.x + mm.x), 0.5f * (z.y + mm.y)), buf_ld2(rh, vh, k2 * kL * 8));
        w[k2] = cmul(make_float2(0.5f * (z.y - mm.y), -0.5f * (z.x - mm.x)), buf_ld2(rh, vn, k2 * kL * 8));
      }
    }
    fft896_sn<true, true>(v, t, sc, tw);
    // B in 1-KB slot tiles (r04, as N = 1024): the block's 8 lines kxb .. kxb + 7 are slot tile
    // kxb / 8; their mirrors N - kx (448 for kx = 0) are slots 448 + kx, tile 56 + kxb / 8
    const int kxb = kx - grp;
    col896_stage_write(v, 1.0f, scratch, grp, t);
    lds_barrier();
    col2_stage_store<kR, kN>(scratch, rb, kxb / kGPB);
    if (it + 1 < kColIter) {  // next line in flight under the second inverse FFT
#pragma unroll
      for (int jj = 0; jj < kL; ++jj) v[jj] = buf_ld2s(ra, lane_a + (kx + KSTEP) * kGPB * 8, jj * JSTEP);
#pragma unroll
      for (int jj = kL; jj < 32; ++jj) v[jj] = make_float2(0.f, 0.f);
    }
    fft896_sn_s1<true, true>(w);
    lds_barrier();   // the first set has been read out: the regions are the FFTs' again
    fft896_sn_s2<true, true>(w, t, sc, tw);
    col896_stage_write(w, dc ? 1.0f : -1.0f, scratch, grp, t);   // line N - kx = conj IFFT(Z conj H)
    lds_barrier();
    col2_stage_store<kR, kN>(scratch, rb, (kHalf + kxb) / kGPB);
  }
}

// ---------------------------------------------------------------------------
// Pass 3 (r04: k_rowinv_d's scheme at 896): 8 rows per block, all P planes; every lane loads
// its own FFT input straight from B's slot tiles -- no LDS tile, no block barrier in the plane
// loop (r01-r03: an LDS tile transpose of 64-B line pieces between three block barriers per
// plane, 0.56-0.59 of 8 TB/s).  The group for row y needs, in slot layout, lane k1 < 28 and
// register k2 < 32: kx = k1 + 28 k2, i.e. slot s = kx (kx <= 448) or 1344 - kx (kx > 448):
//   k2 = 2 m + b < 16:          s = 28 b + k1 + 56 m        -> lane base lo[b] + m * 7 tiles
//   k2 = 31 - (2 m + b) > 16:   s = 476 - k1 + 28 b + 56 m  -> lane base hi[b] + m * 7 tiles
//   k2 = 16:                    lane 0: s = 448 (Nyquist line), lanes k1 > 0: hi[1] + 7 * 7 tiles
// (56 slots = 7 whole 8-slot tiles, so every offset is the lane base plus a constant).  Eight
// consecutive lanes read a 64-B tile row; a wave's two rows are adjacent: 128 B.
// ---------------------------------------------------------------------------
constexpr bool kInvScalar = false;   // packed DFTs (one line live)

template <bool LEAN>
__global__ __launch_bounds__(256, 2) void k_rowinv896(const JobDesc* __restrict__ jobs,
                                                      const float2* __restrict__ ws_b,
                                                      const float* __restrict__ target,
                                                      const float2* __restrict__ tw_glob, int P, int G,
                                                      double* __restrict__ partial,
                                                      float* __restrict__ inten_out,
                                                      float2* __restrict__ field_out, size_t tmask,
                                                      int inten_by_env, int plane_mode,
                                                      float* __restrict__ plane_pool,
                                                      const int32_t* __restrict__ plane_slot, int plane_spares,
                                                      int spare_base) {
  constexpr int TL = 8;                           // slots per tile (1-KB tiles, as N = 1024)
  if constexpr (LEAN) {   // (r06) the plain FFT-mode launch: no plane-cache / field code (as k_rowinv_d)
    plane_mode = kPlanesOff;
    field_out = nullptr;
  }
  __shared__ float2 tw[kN];
  __shared__ float2 scratch[kSCR];
  __shared__ double red[kGPB][3];
  for (int i = threadIdx.x; i < kN; i += 256) tw[i] = tw_glob[i];

  const int grp = threadIdx.x / kR;
  const int t = threadIdx.x % kR;
  const int bid = xcd_pair<kRB>(blockIdx.x);
  const int rb = bid % kRB;
  const int j = bid / kRB;
  const JobDesc jb = jobs[j];
  if (jb.env < 0) {
    if (threadIdx.x == 0) {
      double* o = partial + ((size_t)j * kRB + rb) * 3;
      o[0] = 0.0; o[1] = 0.0; o[2] = 0.0;
    }
    return;
  }
  const int y = rb * kGPB + grp;
  const __amdgpu_buffer_rsrc_t rs = plane_rsrc(ws_b + (size_t)j * P * kPlaneB, (unsigned)((size_t)P * kPlaneB * 8));
  const int k1 = t < kL ? t : 0;                  // lanes 28..31 mirror lane 0 (don't-care values)
  const int yb = (y >> 4) * 16 * kN + (y & 15) * TL;
  auto at = [&](int slot) { return (yb + (slot / TL) * 16 * TL + slot % TL) * 8; };   // bytes
  const int lo0 = at(k1), lo1 = at(28 + k1);
  const int hi0 = at(476 - k1), hi1 = at(504 - k1);
  constexpr int MS = 7 * 16 * TL * 8;             // bytes per m: 7 tiles
  const int mid = k1 == 0 ? at(kHalf) : hi1 + 7 * MS;
  auto load_plane = [&](float2 (&v)[32], int p) {
    const int po = p * (int)(kPlaneB * 8);
#pragma unroll
    for (int k2 = 0; k2 < 32; ++k2) {
      if (k2 < 16) v[k2] = buf_ld2s(rs, (k2 & 1) ? lo1 : lo0, po + (k2 >> 1) * MS);
      else if (k2 == 16) v[k2] = buf_ld2s(rs, mid, po);
      else {
        const int q = 31 - k2;
        v[k2] = buf_ld2s(rs, (q & 1) ? hi1 : hi0, po + (q >> 1) * MS);
      }
    }
  };
  float acc[kL];
#pragma unroll
  for (int k = 0; k < kL; ++k) acc[k] = 0.0f;
  const PaddedScratch<kR> sc{scratch + grp * kR * (kR + 1)};
  // (r06) plane cache, as k_rowinv_d (hbx_passes.hip): slots of this env's planes, pool rows of this
  // lane group's row y; every plane's |U_p|^2 goes to its slot on a fill, the flipped pair's two to
  // the job's spare pair on a step, and a step adds the cached planes in the FFT mode's plane order
  const int CH = G * P;
  const int CHS = CH + 2 * (plane_spares > 1 ? plane_spares : 1);
  const int spare = CH + 2 * (plane_spares > 1 ? spare_base + j : 0);
  const int32_t* slots = plane_slot ? plane_slot + (size_t)jb.env * CHS : nullptr;
  auto pool_row = [&](int slot) { return plane_pool + (((size_t)jb.env * CHS + slot) * kN + y) * kN; };
  auto finish_plane = [&](float2 (&v)[32], int p) {
    fft896_sn<true, kInvScalar>(v, t, sc, tw);      // slot layout in, natural out: x = t + 32 j
    float f[kL];
#pragma unroll
    for (int k = 0; k < kL; ++k) {
      f[k] = fmaf(v[k].x, v[k].x, v[k].y * v[k].y);
      acc[k] += f[k];
    }
    if (field_out) {  // exact field of this plane (incremental mode init / refresh)
      float2* frow = field_out + (((size_t)jb.env * G * P + jb.group * P + p) * kN + y) * kN;
#pragma unroll
      for (int k = 0; k < kL; ++k) frow[t + kR * k] = v[k];
    }
    if (plane_mode != kPlanesOff) {
      float* orow = pool_row(slots[plane_mode == kPlanesFill ? jb.group * P + p : spare + (p & 1)]);
#pragma unroll
      for (int k = 0; k < kL; ++k) __builtin_nontemporal_store(f[k], orow + t + kR * k);
    }
  };
  auto add_cached = [&](int q) {
    const float* crow = pool_row(slots[jb.group * P + q]);
    float c[kL];
#pragma unroll
    for (int k = 0; k < kL; ++k) c[k] = __builtin_nontemporal_load(crow + t + kR * k);
#pragma unroll
    for (int k = 0; k < kL; ++k) acc[k] += c[k];
  };
  float2 v[32];
  if (plane_mode == kPlanesStep) {   // only the flipped plane's pair is in B
    const int pa = jb.flip_plane & ~1;
    load_plane(v, pa);
    __syncthreads();  // tw visible
#pragma unroll 1
    for (int q = 0; q < pa; ++q) add_cached(q);
    finish_plane(v, pa);
    load_plane(v, pa + 1);
    finish_plane(v, pa + 1);
#pragma unroll 1
    for (int q = pa + 2; q < P; ++q) add_cached(q);
  } else {
    load_plane(v, 0);
    __syncthreads();  // tw visible
#pragma unroll 1
    for (int p = 0; p < P; ++p) {
      finish_plane(v, p);
      load_plane(v, p + 1 < P ? p + 1 : p);   // unconditional: the last round re-reads plane P - 1
    }
  }

  const float invp = 1.0f / (float)P;
  const float* trow = target + ((((size_t)jb.env * G + jb.group) * kN + y) * kN & tmask);
  double sxy = 0.0, sxx = 0.0, syy = 0.0;
#pragma unroll
  for (int k = 0; k < kL; ++k) {
    const float I = acc[k] * invp;
    const float T = trow[t + kR * k];
    sxy = fma((double)I, (double)T, sxy);
    sxx = fma((double)I, (double)I, sxx);
    syy = fma((double)T, (double)T, syy);
    acc[k] = I;
  }
  if (inten_out) {
    const size_t slot = inten_by_env ? (size_t)jb.env * G + jb.group : (size_t)j;
    float* orow = inten_out + (slot * kN + y) * kN;
#pragma unroll
    for (int k = 0; k < kL; ++k) orow[t + kR * k] = acc[k];
  }
#pragma unroll
  for (int off = kR / 2; off >= 1; off >>= 1) {
    sxy += __shfl_xor(sxy, off, 64);
    sxx += __shfl_xor(sxx, off, 64);
    syy += __shfl_xor(syy, off, 64);
  }
  if (t == 0) { red[grp][0] = sxy; red[grp][1] = sxx; red[grp][2] = syy; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0, cc = 0.0;
    for (int g = 0; g < kGPB; ++g) { a += red[g][0]; b += red[g][1]; cc += red[g][2]; }
    double* o = partial + ((size_t)j * kRB + rb) * 3;
    o[0] = a; o[1] = b; o[2] = cc;
  }
}

__global__ void k_reduce_partials(const double* __restrict__ partial, int n_jobs, int RB,
                                  double* __restrict__ job_stats);

hipError_t run_jobs_896(const PlanDev& pd, const JobDesc* jobs, int n_jobs, const uint32_t* mask,
                        const float* target, float* inten_out, float2* field_out, hipStream_t st) {
  const int P = pd.P;
  const int CH = pd.G * pd.P;
  PassTimer* tm = pd.timer;
  // (r06) plane-cached mode at 896: a fill writes every plane's |U|^2, a step propagates the
  // flipped plane's pair only (the walk's decision runs in a launch of its own at 896)
  const int pair = pd.plane_mode == kPlanesStep ? 1 : 0;
  if (pd.plane_mode != kPlanesOff && (!pd.plane_pool || !pd.plane_slot)) return hipErrorInvalidValue;
  if (tm) tm->begin(0, st);
  hipLaunchKernelGGL(k_rowfwd896, dim3((unsigned)n_jobs * (pair ? 1 : P / 2) * (kRB / kRit896)), dim3(256), 0, st,
                     jobs, mask, pd.ws_a, pd.tw, P, CH, pd.va, pd.vb, pair);
  if (tm) tm->end(0, n_jobs, st);
  if (tm) tm->begin(1, st);
  hipLaunchKernelGGL(k_col896, dim3((unsigned)n_jobs * (pair ? 2 : P) * kColLB), dim3(256), 0, st, jobs, pd.ws_a,
                     pd.ws_b, pd.htab, pd.tw, P, pair);
  if (tm) tm->end(1, n_jobs, st);
  if (tm) tm->begin(2, st);
  // (r06) the plain FFT-mode launch gets the lean instantiation (profiles/r06/rowinv896_lean_ab_r06i.txt)
  const bool lean = pd.plane_mode == kPlanesOff && !field_out;
  if (lean)
    hipLaunchKernelGGL(k_rowinv896<true>, dim3((unsigned)n_jobs * kRB), dim3(256), 0, st, jobs, pd.ws_b,
                       target ? target : pd.zero_row, pd.tw, P, pd.G, pd.partial, inten_out, field_out,
                       target ? ~(size_t)0 : (size_t)0, pd.inten_by_env, pd.plane_mode, pd.plane_pool, pd.plane_slot,
                       pd.plane_spares, pd.spare_base);
  else
    hipLaunchKernelGGL(k_rowinv896<false>, dim3((unsigned)n_jobs * kRB), dim3(256), 0, st, jobs, pd.ws_b,
                       target ? target : pd.zero_row, pd.tw, P, pd.G, pd.partial, inten_out, field_out,
                       target ? ~(size_t)0 : (size_t)0, pd.inten_by_env, pd.plane_mode, pd.plane_pool, pd.plane_slot,
                       pd.plane_spares, pd.spare_base);
  if (tm) tm->end(2, n_jobs, st);
  hipLaunchKernelGGL(k_reduce_partials, dim3(n_jobs), dim3(64), 0, st, pd.partial, n_jobs, kRB,
                     pd.job_stats);
  return hipGetLastError();
}

}  // namespace hbx
