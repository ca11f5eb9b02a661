// hbx_passes.hip -- the three propagation passes (gfx950, wave64).
//
// One "job" = one colour group (P planes, N x N) of one env, propagated with
// an optional single-pixel flip applied on the fly (env.py:164-172).  The
// intermediates are organised by spectral LINE kx (the N values over y), so
// the column pass streams whole lines and the two transposes a 2-D FFT needs
// live in LDS tiles of the row passes.  A is stored in panels of the row block
// height ([y / 8][kx][y % 8] at N = 1024: every k_rowfwd row block writes one
// contiguous 64-KB panel per plane pair); B in panels of 16 rows
// ([y / 16][kx][y % 16], hbx_internal.hpp), which gives
// the column pass 256-B pieces to write and the row inverse pass 128-B pieces
// to read (measured: 1-2 % over column-major B; 8-row panels made the column
// pass's scattered 64-B writes cost 1 ms).
//
//   k_rowfwd  GPB rows of a plane pair per block: bits -> one complex FFT per
//             row pair (plane a real, plane b imaginary) -> Hermitian split ->
//             half spectrum kx < N/2 (Nyquist packed in Im of kx = 0), stored doubled:
//             2 A, the split's 0.5 factors dropped (r06) and folded into htab = H / 2 ->
//             LDS tile transpose -> A panel y0 / GPB       [HBM: read N^2/8 B, write 4 N^2 B per plane]
//   k_col2    one lane group per half-spectrum line kx: FFT over y -> x H and
//             x conj H (H is even in fx and ky) -> two IFFTs -> B lines kx
//             and N - kx (N/2 for kx = 0); buffer loads / stores with one
//             address VGPR per line; the next input line is prefetched under
//             the second IFFT                                    [read 4 N^2, write 8 N^2]
//   k_rowinv  GPB rows per block, all P planes: LDS tile transpose of the B
//             rows y0..y0+GPB (next plane's tile prefetched into registers
//             behind LDS-only barriers) -> IFFT over kx -> |U|^2 -> plane
//             mean -> f64 partials of (I*T, I^2, T^2) vs the target row   [read 8 N^2 per plane + 4 N^2]
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbx_fft.hpp"
#include "hbx_internal.hpp"
#include "hbx_rowcol.hpp"
#include "hbx_walk_planes.hpp"

namespace hbx {

// Precision study (SURVEY 8d cfg 5, hbx_plan_set_precision): SK = HBX_PRECISION_BF16_STORE /
// _F16_STORE rounds every value written to the two pass intermediates (row spectrum,
// column-pass output) to bf16 / fp16, i.e. the numerics of half-width intermediate storage
// (the layout stays f32).  SK = HBX_PRECISION_F32 is the product path (no rounding code).
template <int SK>
__device__ __forceinline__ float2 store_round(float2 v) {
  if constexpr (SK == HBX_PRECISION_BF16_STORE) {
    auto r = [](float x) {
      uint32_t u = __float_as_uint(x);
      u += 0x7fffu + ((u >> 16) & 1u);   // round to nearest even
      return __uint_as_float(u & 0xffff0000u);
    };
    return make_float2(r(v.x), r(v.y));
  } else if constexpr (SK == HBX_PRECISION_F16_STORE) {
    return make_float2((float)(_Float16)v.x, (float)(_Float16)v.y);
  } else {
    return v;
  }
}

// The row passes' A stores: A is stored doubled (2 A, see htab), so the fp16 study rounds 0.5 v to
// fp16 and doubles it back -- the fp16 value of A itself (fp16 subnormals are not scale-invariant);
// bf16 shares f32's exponent range, where doubling commutes with rounding.
template <int SK>
__device__ __forceinline__ float2 store_round_a(float2 v) {
  if constexpr (SK == HBX_PRECISION_F16_STORE) {
    return make_float2(2.0f * (float)(_Float16)(0.5f * v.x), 2.0f * (float)(_Float16)(0.5f * v.y));
  } else {
    return store_round<SK>(v);
  }
}

// Threads per block of the row passes (row_nt, hbx_internal.hpp).  512-thread
// row blocks (16 rows) were measured slower at N = 1024 -- one 143-KB block per
// CU, whose barriers stall the whole CU: k_rowfwd 1.17 -> 1.54 ms, k_rowinv
// 2.01 -> 2.62 ms.
template <int R>
constexpr int kRowNT = row_nt(R);

// Intermediate layout (hbx_internal.hpp): panels of PAN = kRowNT / R rows, the
// row passes' block height.  A plane of L lines (L = N/2 for A, N for B) is
// N / PAN panels [L][PAN], element (line, y) at (y / PAN) * PS + line * PAN +
// y % PAN with PS = panel_stride(R, L).  A row block then writes (k_rowfwd)
// or reads (k_rowinv) ONE contiguous L * PAN * 8-B panel, while a column-pass
// lane group sees line kx as 64-B pieces of PAN consecutive y -- two adjacent
// lines per wave, so whole 128-B lines per wave instruction.
template <int R>
constexpr int kPanel = panel_rows(R);

template <int R>
using LayoutA = PanelLine<R, R * R / 2, pan_a(R)>;
template <int R>
using LayoutB = PanelLine<R, R * R, pan_b(R)>;

// B at N = 1024 and 256 (r03): tiles [y / 16][s / TL][16 rows][TL slots], TL = 256 / R
// (1 KB at N = 1024, 2 KB at N = 256), of the line SLOT
//   s(kx) = kx (kx <= N/2),  3N/2 - kx (kx > N/2),
// so the two output line sets of a k_col2 block -- its TL lines kx0 .. kx0 + TL - 1 and their
// mirrors N - kx0 - TL + 1 .. N - kx0 (N/2 for kx = 0) -- each fill one aligned tile, which
// the block writes as one contiguous run per 16-row band (staged through LDS), and a
// k_rowinv_d block reads 64-B (N = 1024) / 128-B (N = 256) runs per row straight into its
// FFT layout.  Replayed without arithmetic (tools/membw3.hip, N = 1024): k_col2's movement
// 2.39-2.43 ms (16-row panels 2.41-2.47), k_rowinv's 1.37-1.40 ms (1.62-1.65): DESIGN.md 4.
template <int R>
struct TileB {
  static constexpr int N = R * R, TL = 256 / R;
  __device__ static constexpr int at(int s, int y) {   // float2 offset of (slot s, row y)
    return (y >> 4) * 16 * N + (s / TL) * 16 * TL + (y & 15) * TL + s % TL;
  }
};
template <int R>
constexpr bool kTiledB = R == 32 || R == 16;



// ---------------------------------------------------------------------------
// Pass 1
// ---------------------------------------------------------------------------
// Row blocks per k_rowfwd workgroup (rowfwd_iters): a workgroup walks RIT
// consecutive row blocks of one plane pair, so the stores of block i stay in
// flight under the bit loads and row FFTs of block i + 1 (the next rows' mask
// words are prefetched before the stores are issued: vmcnt counts loads and
// stores in order, so waiting for them never waits for the stores).  With one
// row block per workgroup the load -> FFT -> LDS tile -> store chain of the
// two co-resident workgroups ran nearly serial.
template <int R>
constexpr int rowfwd_iters() { return R == 32 ? 4 : (R == 16 ? 2 : 1); }   // N = 256: 2 (r03,
// with nt A stores: 0.0634 -> 0.0585 ms; 4 row blocks 0.0611)

// The job of workgroup's job index j: jobs[j], or (actions non-null: the env step) decoded from
// actions[j] here, the workgroup with rbw = 0 of the job's first pair writing it to jobs[j] for
// the later passes and flagging an invalid action in *err
__device__ __forceinline__ JobDesc first_pass_job(const JobDesc* jobs, const int64_t* actions, int32_t* err,
                                                  int j, bool writer, int64_t hw, int P, int CH) {
  if (!actions) return jobs[j];
  const JobDesc jb = job_of_action(actions[j], j, hw, P, CH);
  if (writer && threadIdx.x == 0) {
    const_cast<JobDesc*>(jobs)[j] = jb;
    if (jb.env < 0 && err) atomicOr(err, 1);
  }
  return jb;
}

template <int R, int NT, int SK, int RIT = rowfwd_iters<R>()>
__global__ __launch_bounds__(NT, 512 / NT) void k_rowfwd(const JobDesc* jobs,
                                                   const uint32_t* __restrict__ mask,
                                                   float2* __restrict__ ws_a,
                                                   const float2* __restrict__ tw_glob, int P,
                                                   int CH, float va, float vb, int pair_step,
                                                   const int64_t* __restrict__ actions, int32_t* err,
                                                   const uint8_t* __restrict__ phase) {
  constexpr int N = R * R;
  constexpr int GPB = NT / R;          // rows per row block
  constexpr int WPR = N / 32;           // 32-bit mask words per row
  constexpr int SCR = GPB * R * (R + 1);
  static_assert(N * GPB <= SCR, "tile must fit in the scratch area");
  __shared__ float2 tw[N];
  __shared__ __attribute__((aligned(16))) float2 lds[SCR];

  for (int i = threadIdx.x; i < N; i += NT) tw[i] = tw_glob[i];

  const int grp = threadIdx.x / R;
  const int t = threadIdx.x % R;
  const int lane_base = (threadIdx.x & 63) - t;
  constexpr int RB = N / GPB;
  constexpr int RBW = RB / RIT;        // workgroups per plane pair
  int bid = RIT == 1 ? xcd_pair<RB>(blockIdx.x) : (int)blockIdx.x;
  const int rbw = bid % RBW;
  bid /= RBW;
  const int npair = pair_step ? 1 : P / 2;   // plane-cached step: only the flipped plane's pair
  const int j = bid / npair;
  const JobDesc jb = first_pass_job(jobs, actions, err, j, rbw == 0 && bid % npair == 0, (int64_t)N * N, P, CH);
  if (jb.env < 0 || (phase && phase[j])) return;  // uniform per block (a walk slot whose A / B are kept)
  const int q = pair_step ? (jb.flip_plane >> 1) : bid % npair;
  const int pa = 2 * q, pb = 2 * q + 1;
  const uint32_t* plane_a = mask + ((size_t)jb.env * CH + jb.group * P + pa) * N * WPR;
  uint32_t wa[WPR], wb[WPR];
  auto load_row = [&](int y) {
    const uint32_t* rowa = plane_a + (size_t)y * WPR;
    const uint32_t* rowb = rowa + (size_t)N * WPR;
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
  };
  load_row(rbw * RIT * GPB + grp);
  __syncthreads();  // tw visible

  constexpr size_t PLA = plane_a_elems(R);
  float2* base = ws_a + ((size_t)j * P + pa) * PLA;
#pragma unroll 1
  for (int it = 0; it < RIT; ++it) {
    const int y0 = (rbw * RIT + it) * GPB;
    const int y = y0 + grp;
    if (jb.flip_plane >= 0 && jb.flip_pix / N == y) {  // env.py:164 flip, on the fly
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
    pk2 v[R];
    with_field_kind(va, vb, [&](auto fk) {
#pragma unroll
      for (int jj = 0; jj < R; ++jj) {
        const int w = (R * jj) >> 5;
        const int sh = ((R * jj) & 31) + t;
        v[jj] = (pk2){bit_value<fk()>(wa[w], sh, va, vb), bit_value<fk()>(wb[w], sh, va, vb)};
      }
    });
    if constexpr (RIT > 1) {
      // next rows' words (the last iteration re-reads its own row: no conditional load)
      load_row(it + 1 < RIT ? y + GPB : y);
      if (it > 0) lds_barrier();   // every group has read the previous tile: scratch reusable
    }
    fft_group<R, false>(v, t, PaddedScratch<R>{lds + grp * R * (R + 1)}, tw);
    lds_barrier();    // every group is done with its scratch: reuse as the tile

    // Hermitian split -> tile[plane][kx][row]
    float2* tile = lds;
    const float2 zny = from_pk(v[R / 2]);  // Z[N/2] on lane 0
#pragma unroll
    for (int k2 = 0; k2 < R / 2; ++k2) {
      const float2 z = from_pk(v[k2]);
      const float2 m = mirror_conj<R>(v, k2, t, lane_base);
      float2 fa = make_float2(z.x + m.x, z.y + m.y);       // 2 A (htab holds H / 2)
      float2 fb = make_float2(z.y - m.y, m.x - z.x);
      if (k2 == 0 && t == 0) {  // DC and Nyquist of a real row are real
        fa = make_float2(z.x + z.x, zny.x + zny.x);
        fb = make_float2(z.y + z.y, zny.y + zny.y);
      }
      const int kx = t + R * k2;
      tile[tile_pos<R, GPB>(kx, grp)] = fa;
      tile[tile_pos<R, GPB>(N / 2 + kx, grp)] = fb;
    }
    lds_barrier();
    // store tile lines: A[pa|pb][kx][y0 .. y0+GPB), 16 B per thread per chunk
    constexpr int CHUNKS = N * GPB / 2;
    static_assert(CHUNKS % NT == 0, "chunking");
#pragma unroll
    for (int i = 0; i < CHUNKS / NT; ++i) {
      const int c = threadIdx.x + NT * i;
      const int r2 = (c % (GPB / 2)) * 2;
      const int line = c / (GPB / 2);  // pl * N/2 + kx : A planes pa, pb are adjacent
      float2 a, b;
      if constexpr (GPB == 16) {
        // (r05) rows r2, r2 + 1 sit in one aligned 16-B pair (the swizzle XORs whole pairs, its
        // bit 0 swaps the halves): one ds_read_b128 from a single lane base (the swizzle keys on
        // bits 0-4 of the line, which the chunk rounds i leave alone), conflict-free in the
        // 4 x 16-lane model; the two ds_read_b64 it replaces were 2-way (0.79 M extra LDS cycles
        // per 128-job launch at N = 256, profiles/r05/prof_mono_r05t); time unchanged (0.0587-0.0589
        // vs 0.0587-0.0588 ms, profiles/r05/rowfwd16_ab_r05u.txt)
        const int p0 = tile_pos<R, GPB>(line, r2);
        const float4 ab = *reinterpret_cast<const float4*>(tile + (p0 & ~1));
        const bool sw = (p0 & 1) != 0;
        a = sw ? make_float2(ab.z, ab.w) : make_float2(ab.x, ab.y);
        b = sw ? make_float2(ab.x, ab.y) : make_float2(ab.z, ab.w);
      } else {
        a = tile[tile_pos<R, GPB>(line, r2)];
        b = tile[tile_pos<R, GPB>(line, r2 + 1)];
      }
      a = store_round_a<SK>(a);
      b = store_round_a<SK>(b);
      const int pl = line / (N / 2);
      // panel layout: (line, y0 + r2) of plane pl -> contiguous 16-B chunks of the panel
      st_stream4(base + (size_t)pl * PLA + LayoutA<R>::at(line - pl * (N / 2), y0 + r2),
                 make_float4(a.x, a.y, b.x, b.y));
    }
  }
}

// k_rowfwd at N = 1024 with three workgroups per CU (the wide kernel above: 216 VGPRs,
// 75.8 KB LDS, two).  The pass is bound by how many row blocks' stores a CU keeps in
// flight, not by its arithmetic (the whole launch is ~75 us of VALU issue), so:
//  * lane t loads ONE mask word of its row per plane (word t) and a 32 x 32 bit
//    transpose across the group (five ds_swizzle levels) hands it bit t of every
//    word -- the 64 VGPRs of whole-row words the wide kernel keeps for its prefetch
//    are two here;
//  * the FFT transposes real and imaginary parts through a 4.2-KB float tile per
//    group (fft_group_split), and the Hermitian split goes out one plane at a time
//    through a 32-KB tile that aliases those FFT tiles: 8 KB twiddles + 33.8 KB.
// Same arithmetic as k_rowfwd, so the A it writes is bit-identical.
template <int SK, int RIT = rowfwd_iters<32>()>
__global__ __launch_bounds__(256, 3) void k_rowfwd32(const JobDesc* jobs,
                                                     const uint32_t* __restrict__ mask,
                                                     float2* __restrict__ ws_a,
                                                     const float2* __restrict__ tw_glob, int P, int CH,
                                                     float va, float vb, int pair_step,
                                                     const int64_t* __restrict__ actions, int32_t* err,
                                                     const uint8_t* __restrict__ phase) {
  constexpr int R = 32, NT = 256, N = R * R;
  constexpr int GPB = NT / R;          // 8 rows per row block
  constexpr int WPR = N / 32;          // 32 mask words per row = one per lane
  constexpr int SCRF = GPB * R * (R + 1);               // floats: 8 FFT tiles
  static_assert((N / 2) * GPB * 2 <= SCRF, "one plane's tile must fit in the FFT tiles");
  __shared__ float2 tw[N];
  __shared__ __attribute__((aligned(16))) float lds[SCRF];

  for (int i = threadIdx.x; i < N; i += NT) tw[i] = tw_glob[i];

  const int grp = threadIdx.x / R;
  const int t = threadIdx.x % R;
  const int k1 = mirror_k1(t);         // r05: the second FFT stage in mirror-paired lane order
  constexpr int RB = N / GPB;
  constexpr int RBW = RB / RIT;
  int bid = RIT == 1 ? xcd_pair<RB>(blockIdx.x) : (int)blockIdx.x;
  const int rbw = bid % RBW;
  bid /= RBW;
  const int npair = pair_step ? 1 : P / 2;   // plane-cached step: only the flipped plane's pair
  const int j = bid / npair;
  const JobDesc jb = first_pass_job(jobs, actions, err, j, rbw == 0 && bid % npair == 0, (int64_t)N * N, P, CH);
  if (jb.env < 0 || (phase && phase[j])) return;  // uniform per block (a walk slot whose A / B are kept)
  const int q = pair_step ? (jb.flip_plane >> 1) : bid % npair;
  const int pa = 2 * q, pb = 2 * q + 1;
  const uint32_t* plane_a = mask + ((size_t)jb.env * CH + jb.group * P + pa) * N * WPR;
  uint32_t wa, wb;
  auto load_row = [&](int y) {
    wa = plane_a[(size_t)y * WPR + t];
    wb = plane_a[(size_t)(N + y) * WPR + t];
  };
  load_row(rbw * RIT * GPB + grp);
  __syncthreads();  // tw visible

  constexpr size_t PLA = plane_a_elems(R);
  float2* base = ws_a + ((size_t)j * P + pa) * PLA;
  float2* tile = reinterpret_cast<float2*>(lds);
#pragma unroll 1
  for (int it = 0; it < RIT; ++it) {
    const int y0 = (rbw * RIT + it) * GPB;
    const int y = y0 + grp;
    // bit r of ta / tb = pixel x = t + 32 r of the row
    uint32_t ta = group_bit_transpose(wa, t);
    uint32_t tb = group_bit_transpose(wb, t);
    if (jb.flip_plane >= 0 && jb.flip_pix / N == y) {  // env.py:164 flip, on the fly
      const int col = jb.flip_pix % N;
      if (t == (col & 31)) {
        if (jb.flip_plane == pa) ta ^= 1u << (col >> 5);
        if (jb.flip_plane == pb) tb ^= 1u << (col >> 5);
      }
    }
    pk2 v[R];
    with_field_kind(va, vb, [&](auto fk) {
#pragma unroll
      for (int jj = 0; jj < R; ++jj)
        v[jj] = (pk2){bit_value<fk()>(ta, jj, va, vb), bit_value<fk()>(tb, jj, va, vb)};
    });
    if constexpr (RIT > 1) {
      // next rows' words (the last iteration re-reads its own row: no conditional load)
      load_row(it + 1 < RIT ? y + GPB : y);
      if (it > 0) lds_barrier();   // every group has read the previous plane-b tile
    }
    // lane t now holds Z[k1 + 32 k2] (k1 = mirror_k1(t)): the mirror partner is lane t ^ 1
    fft_group_split_mirror<false>(v, t, k1, lds + grp * R * (R + 1), tw);

    // Hermitian split: plane a now, plane b kept in registers for the second tile
    float2 fb[R / 2];
    lds_barrier();    // every group is done with its FFT tile: reuse as the plane tile
    const float2 zny = from_pk(v[R / 2]);  // Z[N/2] on lane 0 (k1 = 0)
#pragma unroll
    for (int k2 = 0; k2 < R / 2; ++k2) {
      const float2 z = from_pk(v[k2]);
      const float2 m = mirror_conj_paired(v, k2, t);
      float2 fa = make_float2(z.x + m.x, z.y + m.y);       // 2 A (htab holds H / 2)
      fb[k2] = make_float2(z.y - m.y, m.x - z.x);
      if (k2 == 0 && t == 0) {  // DC and Nyquist of a real row are real
        fa = make_float2(z.x + z.x, zny.x + zny.x);
        fb[k2] = make_float2(z.y + z.y, zny.y + zny.y);
      }
      tile[tile_pos<R, GPB>(k1 + R * k2, grp)] = fa;
    }
    constexpr int CHUNKS = (N / 2) * GPB / 2;   // 16-B chunks of one plane's panel
    static_assert(CHUNKS % NT == 0, "chunking");
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) {
      if (pl == 1) {
        lds_barrier();   // plane a's tile has been read
#pragma unroll
        for (int k2 = 0; k2 < R / 2; ++k2) tile[tile_pos<R, GPB>(k1 + R * k2, grp)] = fb[k2];
      }
      lds_barrier();
#pragma unroll
      for (int i = 0; i < CHUNKS / NT; ++i) {
        const int c = threadIdx.x + NT * i;
        const int r2 = (c % (GPB / 2)) * 2;
        const int line = c / (GPB / 2);
        const float2 a = store_round_a<SK>(tile[tile_pos<R, GPB>(line, r2)]);
        const float2 b = store_round_a<SK>(tile[tile_pos<R, GPB>(line, r2 + 1)]);
        st_stream4(base + (size_t)pl * PLA + LayoutA<R>::at(line, y0 + r2), make_float4(a.x, a.y, b.x, b.y));
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Pass 2
// ---------------------------------------------------------------------------
// Column pass, one lane group per input line and both of its output lines:
// forward FFT over y -> Z; Z H and W = Z conj H from the same H(kx, .) row (H
// is even in fx and fy); inverse FFT of Z H -> B line kx.  H is even in ky, so
//   IFFT_y(M H)(y) = conj IFFT_y(Z conj H)(y),   M(ky) = conj Z(-ky),
// i.e. B line N - kx is the conjugate of the inverse FFT of W, formed in
// registers from the same H values (no LDS mirror of the line).  Only kx = 0 needs M itself
// ((Z + M)/2 and (Z - M)/2 are the transforms of the two real lines packed into
// A line 0: a register shuffle, mirror_conj; -> lines 0 and N/2).  One forward
// FFT per input line, one A read, one read of half the H row (N = 1024 / 256: H is even
// in ky, the other half comes mirrored through the group's scratch); the FFT and H hand-offs
// stay inside the group's own scratch (wave_sync only).  The next line's loads go into v
// as soon as line kx is stored and fly under the second inverse FFT.
// Scalar-f32 FFTs: with two lines in registers the packed variant spills.
// Measured and removed: the round-1 LDS mirror, packed DFTs,
// three workgroups per CU, H issued ahead, B panels of 8 / 32 / 64 rows.
//
// Lines per lane group.  Measured r03: N = 1024 ITER 2 / 4 / 8 = 2.94 / 2.72 / 2.76 ms (with the
// nt B stores, r03i: 2.82 / 2.58-2.60 / 2.68-2.70).  N = 256: ITER 4 = 0.152 ms, 2 = 0.144.  r03's
// ITER = 1 build wrote wrong B rows; the cause was the wide-store data hazard of the SGPR-soffset
// stage stores.  Rebuilt with the soffset-0 stores (r04) it is exact (the 256 flip
// map / mono / plane tests, profiles/r04/iter1_tests_r04b.txt) and no faster (0.1445-0.1447 ms vs
// 0.1432-0.1445 for ITER = 2, profiles/r04/iter1_ab_r04b.txt), so ITER = 2 stays; small launches
// use ITER = 1 (launch_passes' kSmallBlocks).
template <int R>
__host__ __device__ constexpr int col2_iters() { return R == 32 ? 4 : (R == 16 ? 2 : 1); }

// N = 1024 / 256: the output line sets of a k_col2 block (TL lines: group g = slot g of
// slot tile st, TileB) go out through the FFT scratch.  col2_stage_write: each group
// writes its line (imaginary part times sy) into its OWN scratch region (the group's FFT
// is done with it; no block barrier), row y at col2_pos(g / 2, y).  After a block barrier,
// col2_stage_store: the block stores the set as 16-B chunks (slots 2 sp, 2 sp + 1 from
// regions 2 sp, 2 sp + 1) in memory order -- one contiguous run per 16-row band.
template <int R, int SK>
__device__ __forceinline__ void col2_stage_write(const float2 (&v)[R], float sy, float2* scratch, int grp, int t) {
  // row y = t + R k2: col2_pos only touches bits < 5, so rows R q apart with R q a multiple of
  // 32 share a lane base (constant offsets, the stores pair into ds_write2_b64)
  constexpr int PQ = R >= 32 ? 1 : 32 / R;
  float2* reg = col2_region<R>(scratch, grp);
  float2* base[PQ];
#pragma unroll
  for (int q = 0; q < PQ; ++q) base[q] = reg + col2_pos<R>(grp >> 1, t + R * q);
#pragma unroll
  for (int q = 0; q < PQ; ++q) {
#pragma unroll
    for (int k2 = q; k2 < R; k2 += PQ) base[q][R * (k2 - q)] = store_round<SK>(make_float2(v[k2].x, sy * v[k2].y));
  }
}

template <int R, int SK, int ITER = col2_iters<R>()>
__global__ __launch_bounds__(256, 2) void k_col2(const JobDesc* __restrict__ jobs,
                                                 const float2* __restrict__ ws_a,
                                                 float2* __restrict__ ws_b,
                                                 const float2* __restrict__ htab,
                                                 const float2* __restrict__ tw_glob, int P,
                                                 int pair_step, const uint8_t* __restrict__ phase) {
  constexpr int N = R * R;
  constexpr int GPB = 256 / R;          // lane groups (= input lines) per block iteration
  constexpr int LB = (N / 2) / (GPB * ITER);
  static_assert((N / 2) % (GPB * ITER) == 0, "line blocking");
  __shared__ float2 tw[N];
  constexpr int RS = kTiledB<R> ? col2_region_stride<R>() : R * (R + 1);   // per-group scratch region
  __shared__ float2 scratch[GPB * RS];

  for (int i = threadIdx.x; i < N; i += 256) tw[i] = tw_glob[i];

  const int grp = threadIdx.x / R;
  const int t = threadIdx.x % R;
  const int lane_base = (threadIdx.x & 63) - t;
  int bid = blockIdx.x;
  const int lb = bid % LB;
  bid /= LB;
  const int np = pair_step ? 2 : P;     // plane-cached step: the flipped plane's pair only
  const int j = bid / np;
  const JobDesc jb = jobs[j];
  if (jb.env < 0 || (phase && phase[j])) return;   // (a walk slot whose B is kept)
  const int p = pair_step ? (jb.flip_plane & ~1) + bid % 2 : bid % np;
  using PA = LayoutA<R>;   // A planes: N/2 lines
  using PB = LayoutB<R>;   // B planes: N lines
  const __amdgpu_buffer_rsrc_t ra = plane_rsrc(ws_a + ((size_t)j * P + p) * plane_a_elems(R), plane_a_elems(R) * 8);
  const __amdgpu_buffer_rsrc_t rb = plane_rsrc(ws_b + ((size_t)j * P + p) * plane_b_elems(R), plane_b_elems(R) * 8);
  // H rows of this group, natural [kx][ky]: element (kx, t + R k2) at (kx N + t) * 8 + k2 * R * 8
  const __amdgpu_buffer_rsrc_t rh = plane_rsrc(htab + (size_t)jb.group * (N / 2 + 1) * N, (N / 2 + 1) * N * 8);
  const PaddedScratch<R> sc{scratch + grp * RS};
  // the LB blocks of a plane run side by side: at iteration it they hold lines
  // it * LB * GPB + [0, LB * GPB), i.e. whole contiguous stretches of every panel
  constexpr int KSTEP = LB * GPB;
  const int kx0 = lb * GPB + grp;

  float2 v[R];
  {
    const int vo = PA::voff(t, kx0);
#pragma unroll
    for (int jj = 0; jj < R; ++jj) v[jj] = buf_ld2s(ra, vo, PA::joff(jj));
  }
  lds_barrier();  // tw visible (the line loads stay in flight)

#pragma unroll 1
  for (int it = 0; it < ITER; ++it) {
    const int kx = kx0 + it * KSTEP;
    const bool dc = (kx == 0);
    const int vh = (kx * N + t) * 8;
    // H(kx, .) of this line (N = 1024 / 256: the R/2 + 1 values of ky <= N/2 only, mirrored
    // below), issued before the second FFT stage so the loads fly under it
    constexpr int HP = kTiledB<R> ? R / 2 + 1 : 0;
    float2 hb[R];
    if constexpr (kTiledB<R>) {
      fft_group_s1<R, false, true>(v, t, tw);
      if (!dc) {
#pragma unroll
        for (int i = 0; i < HP; ++i) hb[i] = buf_ld2(rh, vh, i * R * 8);
      }
      if (it > 0) lds_barrier();   // the previous iteration's second set has been read out
      fft_group_s2<R, false, true>(v, t, sc);
    } else {
      fft_group<R, false, true>(v, t, sc, tw);
    }
    float2 w[R];
    if (!dc) {   // v <- Z H, w <- Z conj H
      if constexpr (kTiledB<R>) {
        // H(kx, N - ky) = H(kx, ky): lane t holds ky = t + R k2, whose mirror N - ky sits on
        // lane (R - t) mod R at k2' = R - 1 - k2 (lane 0: its own k2' = R - k2).  The group's
        // loads of k2 <= R/2 go through its FFT scratch (free between the forward and the
        // inverse FFT) and come back mirrored: 17 H loads per line instead of 32 at N = 1024,
        // k_col2 2.67 -> 2.58 ms
        float2* hs = scratch + grp * RS;
        wave_sync();
#pragma unroll
        for (int i = 0; i <= R / 2; ++i) hs[i * R + t] = hb[i];
        wave_sync();
        const float2* hm = hs + (t == 0 ? R : 0) + ((R - t) & (R - 1));
#pragma unroll
        for (int i = R / 2 + 1; i < R; ++i) hb[i] = hm[(R - 1 - i) * R];
        wave_sync();
      } else {
#pragma unroll
        for (int i = 0; i < R; ++i) hb[i] = buf_ld2(rh, vh, i * R * 8);
      }
#pragma unroll
      for (int i = 0; i < R; ++i) {
        w[i] = cmulc(v[i], hb[i]);
        v[i] = cmul(v[i], hb[i]);
      }
    } else {     // kx = 0: (Z + M)/2 H(0) -> line 0, -i (Z - M)/2 H(N/2) -> line N/2
      const int vn = ((N / 2) * N + t) * 8;
#pragma unroll
      for (int k2 = 0; k2 < R; ++k2) w[k2] = mirror_conj<R>(v, k2, t, lane_base);
#pragma unroll
      for (int k2 = 0; k2 < R; ++k2) {
        const float2 z = v[k2], mm = w[k2];
        v[k2] = cmul(make_float2(0.5f * (z.x + mm.x), 0.5f * (z.y + mm.y)), buf_ld2(rh, vh, k2 * R * 8));
        w[k2] = cmul(make_float2(0.5f * (z.y - mm.y), -0.5f * (z.x - mm.x)), buf_ld2(rh, vn, k2 * R * 8));
      }
    }
    fft_group<R, true, true>(v, t, sc, tw);
    const float sy = dc ? 1.0f : -1.0f;   // line N - kx = conj IFFT(W)
    if constexpr (kTiledB<R>) {
      const int kxb = kx - grp;            // the block's GPB lines: slot tile kxb / GPB
      col2_stage_write<R, SK>(v, 1.0f, scratch, grp, t);
      lds_barrier();
      col2_stage_store<R>(scratch, rb, kxb / GPB);
      if (it + 1 < ITER) {  // next line in flight under the second inverse FFT
        const int vo = PA::voff(t, kx + KSTEP);
#pragma unroll
        for (int jj = 0; jj < R; ++jj) v[jj] = buf_ld2s(ra, vo, PA::joff(jj));
      }
      fft_group_s1<R, true, true>(w, t, tw);
      lds_barrier();   // the first set has been read out: the regions are the FFTs' again
      fft_group_s2<R, true, true>(w, t, sc);
      col2_stage_write<R, SK>(w, sy, scratch, grp, t);
      lds_barrier();
      col2_stage_store<R>(scratch, rb, (N / 2 + kxb) / GPB);
    } else {
      {
        const int vo = PB::voff(t, kx);
#pragma unroll
        for (int k2 = 0; k2 < R; ++k2) buf_st2s(store_round<SK>(v[k2]), rb, vo, PB::joff(k2));
      }
      if (it + 1 < ITER) {  // next line in flight under the second inverse FFT
        const int vo = PA::voff(t, kx + KSTEP);
#pragma unroll
        for (int jj = 0; jj < R; ++jj) v[jj] = buf_ld2s(ra, vo, PA::joff(jj));
      }
      fft_group<R, true, true>(w, t, sc, tw);
      {
        const int vo = PB::voff(t, dc ? N / 2 : N - kx);
#pragma unroll
        for (int k2 = 0; k2 < R; ++k2)
          buf_st2s(store_round<SK>(make_float2(w[k2].x, sy * w[k2].y)), rb, vo, PB::joff(k2));
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Pass 3
// ---------------------------------------------------------------------------
// k_rowinv's tail: plane mean, f64 partials of (I*T, I^2, T^2) against the target row,
// fixed-order reduction over the group's lanes and the block's rows.
template <int R, int GPB, bool SC1 = false, bool TPRE = false>
__device__ __forceinline__ void rowinv_epilogue(float (&acc)[R], int P, int G, const JobDesc& jb, int j, int y,
                                                int rb, int grp, int t, const float* __restrict__ target,
                                                size_t tmask, float* __restrict__ inten_out, int inten_by_env,
                                                double* __restrict__ partial, double (&red)[GPB][3],
                                                const int32_t* __restrict__ rc_pending = nullptr,
                                                float* __restrict__ rc_cache = nullptr,
                                                const float* tpre = nullptr) {
  constexpr int N = R * R;
  constexpr int RB = N / GPB;
  const float invp = 1.0f / (float)P;
  // tmask = 0 points every row at the plan's zero row (no target): the loads
  // stay unconditional, so they issue early like the rest of the stream
  const float* trow = target + ((((size_t)jb.env * G + jb.group) * N + y) * N & tmask);
  double sxy = 0.0, sxx = 0.0, syy = 0.0;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const float I = acc[k] * invp;
    const float T = TPRE ? tpre[k] : trow[t + R * k];   // TPRE: the caller loaded the row ahead
    sxy = fma((double)I, (double)T, sxy);
    sxx = fma((double)I, (double)I, sxx);
    syy = fma((double)T, (double)T, syy);
    acc[k] = I;
  }
  if (inten_out) {
    const size_t slot = inten_by_env ? (size_t)jb.env * G + jb.group : (size_t)j;
    float* orow = inten_out + (slot * N + y) * N;
    if (rc_pending) {
      // (r04) the previous step's recon / intensity-cache reconcile of this env, fused here
      // instead of its own launch before the step (k_recon_reconcile): the previous step left
      // group gp's new intensity in recon only (p > 0, accepted: recon -> cache) or its stepped
      // intensity in recon (p < 0, rolled back: cache -> recon).  Row y of group gp is moved
      // by the lane group of row y; when gp is this step's group, an accepted row is read out
      // before this step overwrites it and a rolled-back one needs nothing.
      const int p = rc_pending[jb.env];
      if (p != 0) {
        const int gp = (p > 0 ? p : -p) - 1;
        const size_t grow = (((size_t)jb.env * G + gp) * N + y) * N;
        if (p > 0) {
#pragma unroll
          for (int k = 0; k < R; ++k) rc_cache[grow + t + R * k] = inten_out[grow + t + R * k];
        } else if (gp != jb.group) {
#pragma unroll
          for (int k = 0; k < R; ++k) inten_out[grow + t + R * k] = rc_cache[grow + t + R * k];
        }
      }
    }
    if (inten_by_env) {
      // obs["recon_image"] (r05): streamed out non-temporal -- nothing on the device reads it
      // before the next step rewrites it (the settle copy at G > 1 takes the accepted half)
#pragma unroll
      for (int k = 0; k < R; ++k) __builtin_nontemporal_store(acc[k], orow + t + R * k);
    } else {
#pragma unroll
      for (int k = 0; k < R; ++k) orow[t + R * k] = acc[k];
    }
  }
  // reduce over the R lanes of the group, fixed order -> bitwise reproducible
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
    if constexpr (SC1) {   // read by the deciding workgroup of this launch (walk_planes_arrive)
      const __amdgpu_buffer_rsrc_t ro = walk_planes_rsrc(o, 24);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, a), ro, 0, 0, kSc1Bit);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, b), ro, 8, 0, kSc1Bit);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, cc), ro, 16, 0, kSc1Bit);
    } else {
      o[0] = a; o[1] = b; o[2] = cc;
    }
  }
}

// k_rowinv at N = 1024 / 256 (r03): every lane loads its own FFT input straight from
// the tiled B (TileB) -- lane t of group g (row y0 + g) needs kx = t + R jj, which for TL
// consecutive lanes is TL consecutive slots of one tile row (64 B at N = 1024: the two rows
// of a wave are adjacent, 128 B; 128 B at N = 256: a wave's four rows are one 512-B run),
// so no LDS tile and no block barrier sit in the plane loop: the group's FFT transpose
// (wave_sync) is its only LDS traffic.  The next plane's loads are issued as soon as this
// plane's FFT is done (two blocks per CU cover them; a second register set for a plane in
// flight took one block per CU and measured 1.80 ms against 1.47).  The r02
// kernel staged every plane through an LDS tile between three block barriers (1.80 ms).
template <int R, bool WALK = false, bool LEAN = false>
__global__ __launch_bounds__(256, 2) void k_rowinv_d(const JobDesc* __restrict__ jobs,
                                                     const float2* __restrict__ ws_b,
                                                     const float* __restrict__ target,
                                                     const float2* __restrict__ tw_glob, int P, int G,
                                                     double* __restrict__ partial, float* __restrict__ inten_out,
                                                     float2* __restrict__ field_out, size_t tmask, int inten_by_env,
                                                     int plane_mode, float* __restrict__ plane_pool,
                                                     const int32_t* __restrict__ plane_slot, int plane_spares,
                                                     int spare_base, const int32_t* __restrict__ rc_pending,
                                                     float* __restrict__ rc_cache, WalkPlanesArgs wk) {
  constexpr int N = R * R, GPB = 256 / R, RB = N / GPB, TL = 256 / R;
  static_assert(!WALK || walk_planes_lds_bytes(RB) <= GPB * R * (R + 1) * 8, "the decision's LDS fits the scratch");
  __shared__ float2 tw[N];
  __shared__ float2 scratch[GPB * R * (R + 1)];
  __shared__ double red[GPB][3];
  for (int i = threadIdx.x; i < N; i += 256) tw[i] = tw_glob[i];

  const int grp = threadIdx.x / R;
  const int t = threadIdx.x % R;
  const int bid = xcd_pair<RB>(blockIdx.x);
  const int rb = bid % RB;
  const int j = bid / RB;
  const JobDesc jb = jobs[j];
  if constexpr (WALK) {
    if (wk.phase && wk.phase[j] == 2) {   // (r06) a kept walk slot: its partials and fresh pair stand
      walk_planes_arrive(wk, reinterpret_cast<char*>(scratch));
      return;
    }
  }
  if (jb.env < 0) {
    if (threadIdx.x == 0) {
      double* o = partial + ((size_t)j * RB + rb) * 3;
      if constexpr (WALK) {
        const __amdgpu_buffer_rsrc_t ro = walk_planes_rsrc(o, 24);
        for (int i = 0; i < 3; ++i) __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, ro, 8 * i, 0, kSc1Bit);
      } else {
        o[0] = 0.0; o[1] = 0.0; o[2] = 0.0;
      }
    }
    if constexpr (WALK) walk_planes_arrive(wk, reinterpret_cast<char*>(scratch));
    return;
  }
  if constexpr (LEAN) {   // the plain FFT-mode launch: no plane cache, field, reconcile or walk code
    plane_mode = kPlanesOff;
    field_out = nullptr;
    rc_pending = nullptr;
    rc_cache = nullptr;
  }
  const int y = rb * GPB + grp;
  constexpr int PLB = N * N;                 // float2 per B plane
  const __amdgpu_buffer_rsrc_t rs = plane_rsrc(ws_b + (size_t)j * P * PLB, (unsigned)((size_t)P * PLB * 8));
  // lane bases (bytes) of this row, slot s at TileB<R>::at(s, y):
  //   jj < R/2 (and kx = N/2 for t = 0): s = kx = t + R jj -> lo + 16 R jj float2
  //   jj >= R/2 otherwise: s = 3N/2 - kx -> hi - 16 R jj, written hiB + 16 R (R - 1 - jj)
  //   so every offset stays non-negative
  constexpr int JS = 16 * R * 8;             // bytes per jj
  const int yb = (y >> 4) * 16 * N + (y & 15) * TL;
  const int m = t / TL, u = t % TL;
  const int lo = (yb + m * 16 * TL + u) * 8;
  const int hiB = (yb + (u ? (3 * N / (2 * TL) - m - 1) * 16 * TL + TL - u : (3 * N / (2 * TL) - m) * 16 * TL) -
                   16 * R * (R - 1)) * 8;
  const int vmid = t == 0 ? lo + JS * (R / 2) : hiB + JS * (R / 2 - 1);
  auto load_plane = [&](pk2 (&v)[R], int p) {
    const int po = p * PLB * 8;
#pragma unroll
    for (int jj = 0; jj < R; ++jj) {
      const int vo = jj < R / 2 ? lo : (jj == R / 2 ? vmid : hiB);
      const int so = po + (jj < R / 2 ? JS * jj : (jj == R / 2 ? 0 : JS * (R - 1 - jj)));
      v[jj] = to_pk(buf_ld2s(rs, vo, so));
    }
  };
  float acc[R];
#pragma unroll
  for (int k = 0; k < R; ++k) acc[k] = 0.0f;
  const PaddedScratch<R> sc{scratch + grp * R * (R + 1)};
  // plane cache (ABI v9): slots of this env's planes, pool rows of this lane group's row y
  const int CH = G * P;
  const int CHS = CH + 2 * (plane_spares > 1 ? plane_spares : 1);   // pool slots per env
  const int spare = CH + 2 * (plane_spares > 1 ? spare_base + j : 0);  // this job's fresh pair
  const int32_t* slots = plane_slot ? plane_slot + (size_t)jb.env * CHS : nullptr;
  auto pool_row = [&](int slot) { return plane_pool + (((size_t)jb.env * CHS + slot) * N + y) * N; };
  auto finish_plane = [&](pk2 (&v)[R], int p) {
    fft_group<R, true>(v, t, sc, tw);
    float f[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      f[k] = fmaf(v[k].x, v[k].x, v[k].y * v[k].y);
      acc[k] += f[k];
    }
    if (field_out) {  // exact field of this plane (incremental mode init / refresh)
      float2* frow = field_out + (((size_t)jb.env * G * P + jb.group * P + p) * N + y) * N;
#pragma unroll
      for (int k = 0; k < R; ++k) frow[t + R * k] = from_pk(v[k]);
    }
    // |U_p|^2 to the plane cache: every plane on a fill; on a step both planes of the flipped pair
    // go to the two spares -- the partner's bits change too (the pair is ONE complex row FFT, so
    // its rounding sees the flipped plane), which is why a step keeps both
    if (plane_mode != kPlanesOff) {
      float* orow = pool_row(slots[plane_mode == kPlanesFill ? jb.group * P + p : spare + (p & 1)]);
#pragma unroll
      for (int k = 0; k < R; ++k) __builtin_nontemporal_store(f[k], orow + t + R * k);
    }
  };
  // a cached plane's |U_q|^2 added in its place in the plane order (the sum is the FFT mode's
  // sum bit for bit: acc = ((0 + c_0) + c_1) + ..., each c_q the same f32 value)
  auto add_cached = [&](int q) {
    const float* crow = pool_row(slots[jb.group * P + q]);
    float c[R];
#pragma unroll
    for (int k = 0; k < R; ++k) c[k] = __builtin_nontemporal_load(crow + t + R * k);
#pragma unroll
    for (int k = 0; k < R; ++k) acc[k] += c[k];
  };
  pk2 va[R];
  if (plane_mode == kPlanesStep) {   // only the flipped plane's pair is in B
    const int pa = jb.flip_plane & ~1;
    load_plane(va, pa);
    __syncthreads();  // tw visible
#pragma unroll 1
    for (int q = 0; q < pa; ++q) add_cached(q);
    finish_plane(va, pa);
    load_plane(va, pa + 1);
    finish_plane(va, pa + 1);
#pragma unroll 1
    for (int q = pa + 2; q < P; ++q) add_cached(q);
    rowinv_epilogue<R, GPB, WALK>(acc, P, G, jb, j, y, rb, grp, t, target, tmask, inten_out, inten_by_env, partial,
                                  red, rc_pending, rc_cache);
    if constexpr (WALK) {
      __syncthreads();   // every group is done with its scratch region: the decision's LDS
      walk_planes_arrive(wk, reinterpret_cast<char*>(scratch));
    }
    return;
  }
  load_plane(va, 0);
  __syncthreads();  // tw visible
  if constexpr (R == 16) {   // N = 256: registers to spare -- the next plane in flight under this one's FFT
    pk2 vb[R];
#pragma unroll 1
    for (int p = 0; p < P; p += 2) {         // P is even (hbx_plan_create)
      load_plane(vb, p + 1);
      finish_plane(va, p);
      load_plane(va, p + 2 < P ? p + 2 : p + 1);
      finish_plane(vb, p + 1);
    }
  } else if constexpr (LEAN) {
    // (r06) the last plane peeled: its FFT runs with the target row's loads in flight instead of a
    // re-read of plane P - 1 (the loads the tail waited for; 32 more VGPRs fit the lean kernel)
#pragma unroll 1
    for (int p = 0; p < P - 1; ++p) {
      finish_plane(va, p);
      load_plane(va, p + 1);
    }
    const float* trow = target + ((((size_t)jb.env * G + jb.group) * N + y) * N & tmask);
    float tv[R];
#pragma unroll
    for (int k = 0; k < R; ++k) tv[k] = trow[t + R * k];
    finish_plane(va, P - 1);
    rowinv_epilogue<R, GPB, false, true>(acc, P, G, jb, j, y, rb, grp, t, target, tmask, inten_out, inten_by_env,
                                         partial, red, rc_pending, rc_cache, tv);
    return;
  } else {
#pragma unroll 1
    for (int p = 0; p < P; ++p) {
      finish_plane(va, p);
      load_plane(va, p + 1 < P ? p + 1 : p);   // unconditional: the last round re-reads plane P - 1
    }
  }
  rowinv_epilogue<R, GPB>(acc, P, G, jb, j, y, rb, grp, t, target, tmask, inten_out, inten_by_env, partial, red,
                           rc_pending, rc_cache);
}

template <int R, int NT>
__global__ __launch_bounds__(NT, 512 / NT) void k_rowinv(const JobDesc* __restrict__ jobs,
                                                   const float2* __restrict__ ws_b,
                                                   const float* __restrict__ target,
                                                   const float2* __restrict__ tw_glob, int P,
                                                   int G, double* __restrict__ partial,
                                                   float* __restrict__ inten_out,
                                                   float2* __restrict__ field_out,
                                                   size_t tmask, int inten_by_env) {
  constexpr int N = R * R;
  constexpr int GPB = NT / R;          // rows per block
  constexpr int RB = N / GPB;
  constexpr int CH16 = N * GPB / 2;     // 16-B chunks per plane tile
  constexpr int PER = CH16 / NT;
  static_assert(CH16 % NT == 0, "chunking");
  constexpr int SCR = GPB * R * (R + 1);   // padded transpose scratch reuses the tile
  __shared__ float2 tw[N];
  __shared__ __attribute__((aligned(16))) float2 tile[SCR > N * GPB ? SCR : N * GPB];
  __shared__ double red[GPB][3];

  for (int i = threadIdx.x; i < N; i += NT) tw[i] = tw_glob[i];

  const int grp = threadIdx.x / R;
  const int t = threadIdx.x % R;
  const int bid = xcd_pair<RB>(blockIdx.x);
  const int rb = bid % RB;
  const int j = bid / RB;
  const JobDesc jb = jobs[j];
  if (jb.env < 0) {
    if (threadIdx.x == 0) {
      double* o = partial + ((size_t)j * RB + rb) * 3;
      o[0] = 0.0; o[1] = 0.0; o[2] = 0.0;
    }
    return;
  }
  const int y0 = rb * GPB;
  const int y = y0 + grp;
  constexpr size_t PLB = plane_b_elems(R);
  const float2* jbase = ws_b + (size_t)j * P * PLB;

  float4 pre[PER];   // this thread's share of a plane tile, one plane ahead
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = threadIdx.x + NT * i;
    const int line = c / (GPB / 2), r2 = (c % (GPB / 2)) * 2;
    pre[i] = ld_stream4(jbase + LayoutB<R>::at(line, y0 + r2));
  }
  float acc[R];
#pragma unroll
  for (int k = 0; k < R; ++k) acc[k] = 0.0f;

#pragma unroll 1
  for (int p = 0; p < P; ++p) {
    lds_barrier();  // previous plane's scratch use is over (also publishes tw)
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + NT * i;
      const int line = c / (GPB / 2), r2 = (c % (GPB / 2)) * 2;
      tile[tile_pos<R, GPB>(line, r2)] = make_float2(pre[i].x, pre[i].y);
      tile[tile_pos<R, GPB>(line, r2 + 1)] = make_float2(pre[i].z, pre[i].w);
    }
    if (p + 1 < P) {  // next plane's tile in flight under this plane's FFT
      const float2* nb = jbase + (size_t)(p + 1) * PLB;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int c = threadIdx.x + NT * i;
        const int line = c / (GPB / 2), r2 = (c % (GPB / 2)) * 2;
        pre[i] = ld_stream4(nb + LayoutB<R>::at(line, y0 + r2));
      }
    }
    lds_barrier();
    pk2 v[R];
#pragma unroll
    for (int jj = 0; jj < R; ++jj) v[jj] = to_pk(tile[tile_pos<R, GPB>(t + R * jj, grp)]);
    lds_barrier();  // tile consumed: reuse it as transpose scratch
    fft_group<R, true>(v, t, PaddedScratch<R>{tile + grp * R * (R + 1)}, tw);
#pragma unroll
    for (int k = 0; k < R; ++k) acc[k] += fmaf(v[k].x, v[k].x, v[k].y * v[k].y);
    if (field_out) {  // exact field of this plane (incremental mode init / refresh)
      float2* frow = field_out + (((size_t)jb.env * G * P + jb.group * P + p) * N + y) * N;
#pragma unroll
      for (int k = 0; k < R; ++k) frow[t + R * k] = from_pk(v[k]);
    }
  }

  rowinv_epilogue<R, GPB>(acc, P, G, jb, j, y, rb, grp, t, target, tmask, inten_out, inten_by_env, partial, red);
}

// ---------------------------------------------------------------------------
// Generic complex 2-D FFT (flip-map correlations): a row pass that writes its
// result transposed.  in [n][N][N] row-major -> out[n][k][y] = FFT_x in[n][y][x];
// two applications give the 2-D transform in natural orientation.  Same
// 32-lane group FFT and LDS tile transpose as k_rowfwd (64-B pieces of each
// output line, XCD-grouped row blocks).  INV: + sign, no 1/N^2.
// ---------------------------------------------------------------------------
template <int R, bool INV>
__global__ __launch_bounds__(256, 2) void k_fft_rt(const float2* __restrict__ in,
                                                   float2* __restrict__ out,
                                                   const float2* __restrict__ tw_glob) {
  constexpr int N = R * R;
  constexpr int GPB = 256 / R;
  constexpr int SCR = GPB * R * (R + 1);
  static_assert(N * GPB <= SCR, "tile must fit in the scratch area");
  constexpr int RB = N / GPB;
  __shared__ float2 tw[N];
  __shared__ __attribute__((aligned(16))) float2 lds[SCR];
  for (int i = threadIdx.x; i < N; i += 256) tw[i] = tw_glob[i];
  const int grp = threadIdx.x / R;
  const int t = threadIdx.x % R;
  int bid = xcd_pair<RB>(blockIdx.x);
  const int rb = bid % RB;
  const int plane = bid / RB;
  const int y0 = rb * GPB;
  const float2* row = in + ((size_t)plane * N + y0 + grp) * N + t;
  float2 v[R];
#pragma unroll
  for (int j = 0; j < R; ++j) v[j] = row[R * j];
  __syncthreads();  // tw visible
  fft_group<R, INV>(v, t, PaddedScratch<R>{lds + grp * R * (R + 1)}, tw);
  lds_barrier();    // scratch reused as the tile [k][row]
#pragma unroll
  for (int k2 = 0; k2 < R; ++k2) lds[tile_pos<R>(t + R * k2, grp)] = v[k2];
  lds_barrier();
  float2* base = out + (size_t)plane * N * N;
  constexpr int CHUNKS = N * GPB / 2;
#pragma unroll
  for (int i = 0; i < CHUNKS / 256; ++i) {
    const int c = threadIdx.x + 256 * i;
    const int r2 = (c % (GPB / 2)) * 2;
    const int line = c / (GPB / 2);
    const float2 a = lds[tile_pos<R>(line, r2)];
    const float2 b = lds[tile_pos<R>(line, r2 + 1)];
    *reinterpret_cast<float4*>(base + (size_t)line * N + y0 + r2) = make_float4(a.x, a.y, b.x, b.y);
  }
}

template <int R>
static hipError_t launch_fft2d(const PlanDev& pd, float2* a, float2* b, int n_planes, bool inverse,
                               hipStream_t st) {
  constexpr int N = R * R;
  const unsigned blocks = (unsigned)n_planes * (N / (256 / R));
  for (int pass = 0; pass < 2; ++pass) {
    const float2* src = pass == 0 ? a : b;
    float2* dst = pass == 0 ? b : a;
    if (inverse)
      hipLaunchKernelGGL((k_fft_rt<R, true>), dim3(blocks), dim3(256), 0, st, src, dst, pd.tw);
    else
      hipLaunchKernelGGL((k_fft_rt<R, false>), dim3(blocks), dim3(256), 0, st, src, dst, pd.tw);
  }
  return hipGetLastError();
}

// N = 896 (crop of a 1024 mask): the same transposing row pass on the 28 x 32
// lane-group FFT (natural layout in, slot layout out: lane k1 < 28 writes
// X[k1 + 28 k2] into the tile)
template <bool INV>
__global__ __launch_bounds__(256, 2) void k_fft_rt896(const float2* __restrict__ in,
                                                      float2* __restrict__ out,
                                                      const float2* __restrict__ tw_glob) {
  constexpr int N = 896, R = 32, GPB = 8, RB = N / GPB;
  constexpr int SCR = GPB * R * (R + 1);
  static_assert(N * GPB <= SCR, "tile must fit in the scratch area");
  __shared__ float2 tw[N];
  __shared__ __attribute__((aligned(16))) float2 lds[SCR];
  for (int i = threadIdx.x; i < N; i += 256) tw[i] = tw_glob[i];
  const int grp = threadIdx.x / R;
  const int t = threadIdx.x % R;
  int bid = xcd_pair<RB>(blockIdx.x);
  const int rb = bid % RB;
  const int plane = bid / RB;
  const int y0 = rb * GPB;
  const float2* row = in + ((size_t)plane * N + y0 + grp) * N + t;
  float2 v[32];
#pragma unroll
  for (int j = 0; j < 28; ++j) v[j] = row[R * j];
  __syncthreads();  // tw visible
  fft896_ns<INV>(v, t, PaddedScratch<R>{lds + grp * R * (R + 1)}, tw);
  lds_barrier();
  if (t < 28) {
#pragma unroll
    for (int k2 = 0; k2 < 32; ++k2) lds[tile_pos<R, GPB>(t + 28 * k2, grp)] = v[k2];
  }
  lds_barrier();
  float2* base = out + (size_t)plane * N * N;
  constexpr int CHUNKS = N * GPB / 2;
  static_assert(CHUNKS % 256 == 0, "chunking");
#pragma unroll
  for (int i = 0; i < CHUNKS / 256; ++i) {
    const int c = threadIdx.x + 256 * i;
    const int r2 = (c % (GPB / 2)) * 2;
    const int line = c / (GPB / 2);
    const float2 a = lds[tile_pos<R, GPB>(line, r2)];
    const float2 b = lds[tile_pos<R, GPB>(line, r2 + 1)];
    *reinterpret_cast<float4*>(base + (size_t)line * N + y0 + r2) = make_float4(a.x, a.y, b.x, b.y);
  }
}

hipError_t run_fft2d(const PlanDev& pd, float2* a, float2* b, int n_planes, bool inverse,
                     hipStream_t st) {
  if (n_planes <= 0) return hipSuccess;
  if (pd.R == 0) {   // N = 896
    const unsigned blocks = (unsigned)n_planes * (896 / 8);
    for (int pass = 0; pass < 2; ++pass) {
      const float2* src = pass == 0 ? a : b;
      float2* dst = pass == 0 ? b : a;
      if (inverse) hipLaunchKernelGGL((k_fft_rt896<true>), dim3(blocks), dim3(256), 0, st, src, dst, pd.tw);
      else hipLaunchKernelGGL((k_fft_rt896<false>), dim3(blocks), dim3(256), 0, st, src, dst, pd.tw);
    }
    return hipGetLastError();
  }
  switch (pd.R) {
    case 32: return launch_fft2d<32>(pd, a, b, n_planes, inverse, st);
    case 16: return launch_fft2d<16>(pd, a, b, n_planes, inverse, st);
    case 8: return launch_fft2d<8>(pd, a, b, n_planes, inverse, st);
    default: return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------
// launch sequence for one batch of jobs
// ---------------------------------------------------------------------------
__global__ void k_reduce_partials(const double* __restrict__ partial, int n_jobs, int RB,
                                  double* __restrict__ job_stats);

template <int R, int SK>
static hipError_t launch_passes(const PlanDev& pd, const JobDesc* jobs, int n_jobs,
                                const uint32_t* mask, const float* target, float* inten_out,
                                float2* field_out, hipStream_t st) {
  constexpr int N = R * R;
  constexpr int GPB = 256 / R;
  const int P = pd.P;
  const int CH = pd.G * pd.P;
  PassTimer* tm = pd.timer;
  const int pair = pd.plane_mode == kPlanesStep ? 1 : 0;
  if (pd.plane_mode != kPlanesOff && (!kTiledB<R> || !pd.plane_pool || !pd.plane_slot)) return hipErrorInvalidValue;
  // Small batches (greedy DBS, a few candidates per launch): the walk-per-workgroup loops
  // (rowfwd_iters row blocks, col2_iters lines) trade parallelism for store overlap, which pays
  // only when the launch fills the chip many times over.  Below kSmallBlocks workgroups the
  // launch runs one row block / one line per workgroup instead -- the same arithmetic, so
  // bit-identical results (tests/test_gpu_dbs_headline.py plane-cache / full re-propagation).
  constexpr unsigned kSmallBlocks = 2048;
  const unsigned rf_blocks = (unsigned)n_jobs * (pair ? 1 : P / 2) * (N / (kRowNT<R> / R)) / rowfwd_iters<R>();
  const unsigned col_blocks = (unsigned)n_jobs * (pair ? 2 : P) * ((N / 2) / (GPB * col2_iters<R>()));
  const bool small = kTiledB<R> && rf_blocks < kSmallBlocks && col_blocks < kSmallBlocks;
  {
    if (tm) tm->begin(0, st);
    if constexpr (R == 32) {
      if (small)
        hipLaunchKernelGGL((k_rowfwd32<SK, 1>), dim3(rf_blocks * rowfwd_iters<R>()), dim3(256), 0, st, jobs, mask,
                           pd.ws_a, pd.tw, P, CH, pd.va, pd.vb, pair, pd.actions, pd.act_err, pd.walk_phase);
      else
        hipLaunchKernelGGL((k_rowfwd32<SK>), dim3(rf_blocks), dim3(256), 0, st, jobs, mask, pd.ws_a, pd.tw, P, CH,
                           pd.va, pd.vb, pair, pd.actions, pd.act_err, pd.walk_phase);
    } else if constexpr (kTiledB<R>) {
      if (small)
        hipLaunchKernelGGL((k_rowfwd<R, kRowNT<R>, SK, 1>), dim3(rf_blocks * rowfwd_iters<R>()), dim3(kRowNT<R>), 0,
                           st, jobs, mask, pd.ws_a, pd.tw, P, CH, pd.va, pd.vb, pair, pd.actions, pd.act_err, pd.walk_phase);
      else
        hipLaunchKernelGGL((k_rowfwd<R, kRowNT<R>, SK>), dim3(rf_blocks), dim3(kRowNT<R>), 0, st, jobs, mask,
                           pd.ws_a, pd.tw, P, CH, pd.va, pd.vb, pair, pd.actions, pd.act_err, pd.walk_phase);
    } else {
      hipLaunchKernelGGL((k_rowfwd<R, kRowNT<R>, SK>), dim3(rf_blocks), dim3(kRowNT<R>), 0, st, jobs, mask, pd.ws_a,
                         pd.tw, P, CH, pd.va, pd.vb, pair, pd.actions, pd.act_err, pd.walk_phase);
    }
    if (tm) tm->end(0, n_jobs, st);
  }
  {
    if (tm) tm->begin(1, st);
    if constexpr (kTiledB<R>) {
      if (small)
        hipLaunchKernelGGL((k_col2<R, SK, 1>), dim3(col_blocks * col2_iters<R>()), dim3(256), 0, st, jobs, pd.ws_a,
                           pd.ws_b, pd.htab, pd.tw, P, pair, pd.walk_phase);
      else
        hipLaunchKernelGGL((k_col2<R, SK>), dim3(col_blocks), dim3(256), 0, st, jobs, pd.ws_a, pd.ws_b, pd.htab,
                           pd.tw, P, pair, pd.walk_phase);
    } else {
      hipLaunchKernelGGL((k_col2<R, SK>), dim3(col_blocks), dim3(256), 0, st, jobs, pd.ws_a, pd.ws_b, pd.htab,
                         pd.tw, P, pair, pd.walk_phase);
    }
    if (tm) tm->end(1, n_jobs, st);
  }
  {
    const unsigned blocks = (unsigned)n_jobs * (N / (kRowNT<R> / R));
    if (tm) tm->begin(2, st);
    if constexpr (kTiledB<R>) {
      if (pd.walk_planes) {   // (r05) a plane-cache walk batch: the last workgroup decides
        if (pd.plane_mode != kPlanesStep) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_rowinv_d<R, true>), dim3(blocks), dim3(256), 0, st, jobs, pd.ws_b,
                           target ? target : pd.zero_row, pd.tw, P, pd.G, pd.partial, inten_out, field_out,
                           target ? ~(size_t)0 : (size_t)0, pd.inten_by_env, pd.plane_mode, pd.plane_pool,
                           pd.plane_slot, pd.plane_spares, pd.spare_base, pd.rc_pending, pd.rc_cache,
                           *pd.walk_planes);
      } else if (pd.plane_mode == kPlanesOff && !field_out && !pd.rc_pending) {
        // (r06) the plain FFT-mode launch (the headline): its own instantiation without the plane
        // cache / field / reconcile / walk code -- 1,687 instead of 4,988 instructions; same
        // arithmetic and bits, k_rowinv 1.465-1.515 -> 1.444-1.457 ms alternated on one box
        // (profiles/r06/rowinv_lean_ab_r06e.txt)
        hipLaunchKernelGGL((k_rowinv_d<R, false, true>), dim3(blocks), dim3(256), 0, st, jobs, pd.ws_b,
                           target ? target : pd.zero_row, pd.tw, P, pd.G, pd.partial, inten_out, field_out,
                           target ? ~(size_t)0 : (size_t)0, pd.inten_by_env, pd.plane_mode, pd.plane_pool,
                           pd.plane_slot, pd.plane_spares, pd.spare_base, pd.rc_pending, pd.rc_cache,
                           WalkPlanesArgs{});
      } else {
        hipLaunchKernelGGL((k_rowinv_d<R>), dim3(blocks), dim3(256), 0, st, jobs, pd.ws_b,
                           target ? target : pd.zero_row, pd.tw, P, pd.G, pd.partial, inten_out, field_out,
                           target ? ~(size_t)0 : (size_t)0, pd.inten_by_env, pd.plane_mode, pd.plane_pool,
                           pd.plane_slot, pd.plane_spares, pd.spare_base, pd.rc_pending, pd.rc_cache,
                           WalkPlanesArgs{});
      }
    }
    else
      hipLaunchKernelGGL((k_rowinv<R, kRowNT<R>>), dim3(blocks), dim3(kRowNT<R>), 0, st, jobs, pd.ws_b,
                         target ? target : pd.zero_row, pd.tw, P, pd.G, pd.partial, inten_out,
                         field_out, target ? ~(size_t)0 : (size_t)0, pd.inten_by_env);
    if (tm) tm->end(2, n_jobs, st);
  }
  if (!pd.skip_reduce)
    hipLaunchKernelGGL(k_reduce_partials, dim3(n_jobs), dim3(64), 0, st, pd.partial,
                       n_jobs, N / (kRowNT<R> / R), pd.job_stats);
  return hipGetLastError();
}

hipError_t run_jobs(const PlanDev& pd, const JobDesc* jobs, int n_jobs, const uint32_t* mask,
                    const float* target, float* inten_out, float2* field_out, hipStream_t st) {
  if (pd.R == 0) return run_jobs_896(pd, jobs, n_jobs, mask, target, inten_out, field_out, st);
  switch (pd.R * 4 + pd.store_kind) {
#define HBX_PASSES_CASE(R_, SK_) \
    case R_ * 4 + SK_: return launch_passes<R_, SK_>(pd, jobs, n_jobs, mask, target, inten_out, field_out, st);
    HBX_PASSES_CASE(32, HBX_PRECISION_F32)
    HBX_PASSES_CASE(32, HBX_PRECISION_BF16_STORE)
    HBX_PASSES_CASE(32, HBX_PRECISION_F16_STORE)
    HBX_PASSES_CASE(16, HBX_PRECISION_F32)
    HBX_PASSES_CASE(16, HBX_PRECISION_BF16_STORE)
    HBX_PASSES_CASE(16, HBX_PRECISION_F16_STORE)
    HBX_PASSES_CASE(8, HBX_PRECISION_F32)
    HBX_PASSES_CASE(8, HBX_PRECISION_BF16_STORE)
    HBX_PASSES_CASE(8, HBX_PRECISION_F16_STORE)
#undef HBX_PASSES_CASE
    default: return hipErrorInvalidValue;
  }
}

}  // namespace hbx
