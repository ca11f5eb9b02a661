// membw3.hip -- r03 access-shape study for the B intermediate (k_col2 -> k_rowinv),
// replayed without arithmetic (the pass structure, barriers and LDS hand-offs kept):
//
//   col2_A8_B16       today's k_col2 movement: 8 lines per block, A 8-row panels read
//                     8 B / lane, B lines kx and N - kx written 8 B / lane into 16-row panels
//   col2_A8_B8_lds    B in 8-row panels, each output line set staged through a 64-KB LDS
//                     tile (block barrier) and written as 16-B lanes: one wave instruction =
//                     two 512-B panel runs (the block's 8 lines x 8 rows)
//   col2_A8_B16_lds   the same staging into 16-row panels (1-KB panel runs)
//   rowinv_pan<PAN>   k_rowinv's loads: 8 rows per block (all 8 planes of a job), XCD-grouped
//   mall_read<MB>     Infinity-Cache read rate: write a MB-sized buffer, then read it back
//
// build: hipcc -O3 --offload-arch=gfx950 tools/membw3.hip -o tools/membw3
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int N = 1024, R = 32, P = 8;

__device__ __forceinline__ int xcd_group(int bid) {
  constexpr int GS = 16, SPAN = 8 * GS;
  return (bid / SPAN) * SPAN + (bid % 8) * GS + (bid / 8) % GS;
}

template <int PAN, int L>
__device__ __forceinline__ size_t pan_at(int line, int y) {
  return (size_t)(y / PAN) * L * PAN + (size_t)line * PAN + y % PAN;
}

__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__global__ void k_r1w2_flat(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const float4 v = a[i];
  b[i] = v;
  b[i + n] = make_float4(v.y, v.x, v.w, v.z);
}
__global__ void k_read_flat(const float4* __restrict__ a, float* out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const float4 v = a[i];
  if (v.x + v.y + v.z + v.w == 12345.f) out[0] = 1.f;
}
__global__ void k_write_flat(float4* __restrict__ a) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  a[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

// today's movement
template <int PAN>
__global__ __launch_bounds__(256, 2) void k_col2_direct(const float2* __restrict__ A, float2* __restrict__ B) {
  constexpr int GPB = 8, ITER = 4, LB = (N / 2) / (GPB * ITER), KSTEP = LB * GPB;
  constexpr size_t PLA = (size_t)(N / 2) * N, PLB = (size_t)N * N;
  const int grp = threadIdx.x / R, t = threadIdx.x % R;
  int bid = blockIdx.x;
  const int lb = bid % LB;
  bid /= LB;
  const float2* a = A + (size_t)bid * PLA;
  float2* b = B + (size_t)bid * PLB;
  for (int it = 0; it < ITER; ++it) {
    const int kx = lb * GPB + grp + it * KSTEP;
    float2 v[R];
#pragma unroll
    for (int jj = 0; jj < R; ++jj) v[jj] = a[pan_at<8, N / 2>(kx, t + R * jj)];
    const int k2 = kx == 0 ? N / 2 : N - kx;
#pragma unroll
    for (int jj = 0; jj < R; ++jj) b[pan_at<PAN, N>(kx, t + R * jj)] = v[jj];
#pragma unroll
    for (int jj = 0; jj < R; ++jj) b[pan_at<PAN, N>(k2, t + R * jj)] = make_float2(v[jj].y, v[jj].x);
  }
}

// staged: the block's 8 lines of one output set go through an LDS tile, then 16-B lanes
// PAN = 8: tile [q 128][slot 8][r 8], slot = (g + q) % 8 (conflict-free b64 writes and
// b128 reads); memory run per panel = the 8 lines x 8 rows = 512 B
// PAN = 16: tile [q 64][slot 8][r 16], run per panel 1 KB
template <int PAN>
__device__ __forceinline__ void staged_store(float2* __restrict__ b, float2* tile, const float2 (&v)[R], int lines0,
                                             bool reversed, int grp, int t) {
  constexpr int Q = N / PAN;               // panels
  constexpr int ROW = 8 * PAN;             // float2 per panel row of the tile
  lds_barrier();   // the previous use of the tile is over
#pragma unroll
  for (int k2 = 0; k2 < R; ++k2) {
    const int y = t + R * k2;
    const int q = y / PAN, r = y % PAN;
    tile[q * ROW + ((grp + q) & 7) * PAN + r] = v[k2];
  }
  lds_barrier();
  // chunk c (16 B): q = c / (4 PAN), slot line g = (c / (PAN / 2)) % 8, pair rp = c % (PAN / 2)
  constexpr int CH = Q * 8 * PAN / 2;      // chunks per line set = 4096
#pragma unroll
  for (int i = 0; i < CH / 256; ++i) {
    const int c = threadIdx.x + 256 * i;
    const int q = c / (4 * PAN);
    const int g = (c / (PAN / 2)) % 8;
    const int rp = c % (PAN / 2);
    const float4 w = *reinterpret_cast<const float4*>(tile + q * ROW + ((g + q) & 7) * PAN + 2 * rp);
    // reversed: the block's lines run N - kx0 - 7 .. N - kx0 in memory order
    const int line = reversed ? lines0 - 7 + g : lines0 + g;
    const int gg = reversed ? 7 - g : g;   // (data of group gg lands at line lines0 - gg)
    (void)gg;
    *reinterpret_cast<float4*>(b + (size_t)q * N * PAN + (size_t)line * PAN + 2 * rp) = w;
  }
}

template <int PAN>
__global__ __launch_bounds__(256, 2) void k_col2_lds(const float2* __restrict__ A, float2* __restrict__ B) {
  constexpr int GPB = 8, ITER = 4, LB = (N / 2) / (GPB * ITER), KSTEP = LB * GPB;
  constexpr size_t PLA = (size_t)(N / 2) * N, PLB = (size_t)N * N;
  __shared__ __attribute__((aligned(16))) float2 tile[N * 8];
  const int grp = threadIdx.x / R, t = threadIdx.x % R;
  int bid = blockIdx.x;
  const int lb = bid % LB;
  bid /= LB;
  const float2* a = A + (size_t)bid * PLA;
  float2* b = B + (size_t)bid * PLB;
  for (int it = 0; it < ITER; ++it) {
    const int kx0 = lb * GPB + it * KSTEP;
    const int kx = kx0 + grp;
    float2 v[R];
#pragma unroll
    for (int jj = 0; jj < R; ++jj) v[jj] = a[pan_at<8, N / 2>(kx, t + R * jj)];
    staged_store<PAN>(b, tile, v, kx0, false, grp, t);
#pragma unroll
    for (int jj = 0; jj < R; ++jj) v[jj] = make_float2(v[jj].y, v[jj].x);
    // second set: lines N - kx0 - 7 .. N - kx0 (kx0 = 0 -> lines N/2 .. : approximated as N - 8)
    staged_store<PAN>(b, tile, v, kx0 == 0 ? N - 1 : N - kx0, true, grp, t);
  }
}

// tiled B: [y / 16][kx / TL][16 rows][TL lines] (TL = 8: 1-KB tiles; 16: 2-KB tiles).
// k_col2 with GL = TL lines per block iteration (GL lane groups), staged through LDS:
// per 16-row band one tile of TL lines x 16 rows contiguous.
template <int TL>
__device__ __forceinline__ size_t tile_at(int line, int y) {
  return ((size_t)(y / 16) * (N / TL) + line / TL) * (16 * TL) + (y % 16) * TL + line % TL;
}
template <int TL, int PA = 8>
__global__ __launch_bounds__(TL * 32, 1) void k_col2_tiled(const float2* __restrict__ A, float2* __restrict__ B) {
  constexpr int NT = TL * 32, ITER = 4, LB = (N / 2) / (TL * ITER), KSTEP = LB * TL;
  constexpr size_t PLA = (size_t)(N / 2) * N, PLB = (size_t)N * N;
  __shared__ __attribute__((aligned(16))) float2 tile[N * TL];   // [band 64][16 rows][TL] (+ swizzle)
  const int grp = threadIdx.x / R, t = threadIdx.x % R;
  int bid = blockIdx.x;
  const int lb = bid % LB;
  bid /= LB;
  const float2* a = A + (size_t)bid * PLA;
  float2* b = B + (size_t)bid * PLB;
  for (int it = 0; it < ITER; ++it) {
    const int kx0 = lb * TL + it * KSTEP;
    const int kx = kx0 + grp;
    float2 v[R];
#pragma unroll
    for (int jj = 0; jj < R; ++jj) v[jj] = a[pan_at<PA, N / 2>(kx, t + R * jj)];
    for (int set = 0; set < 2; ++set) {
      lds_barrier();
      // tile element (band, r, l): band * 16 TL + r * TL + (l ^ (r & (TL - 1)))  (xor swizzle on the line)
#pragma unroll
      for (int k2 = 0; k2 < R; ++k2) {
        const int y = t + R * k2;
        const int band = y / 16, r = y % 16;
        tile[band * 16 * TL + r * TL + (grp ^ (r & (TL - 1)))] = v[k2];
      }
      lds_barrier();
      constexpr int CH = N * TL / 2;   // 16-B chunks of the line set
#pragma unroll
      for (int i = 0; i < CH / NT; ++i) {
        const int c = threadIdx.x + NT * i;
        const int band = c / (8 * TL), r = (c / (TL / 2)) % 16, lp = (c % (TL / 2)) * 2;
        const float2 w0 = tile[band * 16 * TL + r * TL + (lp ^ (r & (TL - 1)))];
        const float2 w1 = tile[band * 16 * TL + r * TL + ((lp + 1) ^ (r & (TL - 1)))];
        const int line0 = set == 0 ? kx0 : (kx0 == 0 ? N - TL : N - kx0 - TL);
        *reinterpret_cast<float4*>(b + ((size_t)band * (N / TL) + line0 / TL) * (16 * TL) + r * TL + lp) =
            make_float4(w0.x, w0.y, w1.x, w1.y);
      }
#pragma unroll
      for (int jj = 0; jj < R; ++jj) v[jj] = make_float2(v[jj].y, v[jj].x);
    }
  }
}
// T8 written directly from the FFT layout (no LDS): lane t (line kx, row y = t + 32 k2)
// stores 8 B; SWAP: lanes t and t + 32 (lines kx, kx + 1 of a wave) exchange halves so
// each lane stores 16 B = (row y, slots kx, kx + 1)
template <bool SWAP>
__global__ __launch_bounds__(256, 2) void k_col2_t8_direct(const float2* __restrict__ A, float2* __restrict__ B) {
  constexpr int GPB = 8, ITER = 4, LB = (N / 2) / (GPB * ITER), KSTEP = LB * GPB;
  constexpr size_t PLA = (size_t)(N / 2) * N, PLB = (size_t)N * N;
  const int grp = threadIdx.x / R, t = threadIdx.x % R;
  int bid = blockIdx.x;
  const int lb = bid % LB;
  bid /= LB;
  const float2* a = A + (size_t)bid * PLA;
  float2* b = B + (size_t)bid * PLB;
  const bool upper = (threadIdx.x & 32) != 0;
  for (int it = 0; it < ITER; ++it) {
    const int kx0 = lb * GPB + it * KSTEP;
    const int kx = kx0 + grp;
    float2 v[R];
#pragma unroll
    for (int jj = 0; jj < R; ++jj) v[jj] = a[pan_at<8, N / 2>(kx, t + R * jj)];
    for (int set = 0; set < 2; ++set) {
      const int s = set == 0 ? kx : N / 2 + kx;
      if (!SWAP) {
#pragma unroll
        for (int k2 = 0; k2 < R; ++k2) {
          const int y = t + R * k2;
          b[tile_at<8>(s, y)] = v[k2];
        }
      } else {
        // pair registers k2 (lanes < 32 keep it) and k2 + 1 (lanes >= 32 keep it)
#pragma unroll
        for (int k2 = 0; k2 < R; k2 += 2) {
          const float2 mine = upper ? v[k2 + 1] : v[k2];     // what this lane keeps
          const float2 give = upper ? v[k2] : v[k2 + 1];     // what the partner keeps
          float2 other;
          other.x = __shfl_xor(give.x, 32, 64);
          other.y = __shfl_xor(give.y, 32, 64);
          // lane < 32: row y = t + 32 k2, lines (kx, kx + 1) = (mine, other); lane >= 32: row t + 32 (k2 + 1),
          // lines (kx - 1, kx) = (other, mine)
          const int y = t + R * (upper ? k2 + 1 : k2);
          const int s0 = upper ? s - 1 : s;
          const float4 w = upper ? make_float4(other.x, other.y, mine.x, mine.y)
                                 : make_float4(mine.x, mine.y, other.x, other.y);
          *reinterpret_cast<float4*>(b + tile_at<8>(s0, y)) = w;
        }
      }
#pragma unroll
      for (int jj = 0; jj < R; ++jj) v[jj] = make_float2(v[jj].y, v[jj].x);
    }
  }
}

// k_rowinv's loads from the tiled B: 8 rows per block -> per tile the 8-row half: TL * 8 * 8 B contiguous
template <int TL>
__global__ __launch_bounds__(256, 2) void k_rowinv_tiled(const float2* __restrict__ B, float* out) {
  constexpr int G = 8, RB = N / G, CH16 = N * G / 2;
  const int bid = xcd_group(blockIdx.x);
  const int rb = bid % RB;
  const int job = bid / RB;
  const int y0 = rb * G;
  float acc = 0.f;
  for (int p = 0; p < P; ++p) {
    const float2* b = B + ((size_t)job * P + p) * N * N;
#pragma unroll 4
    for (int i = 0; i < CH16 / 256; ++i) {
      const int c = threadIdx.x + 256 * i;     // chunk: tile c / (4 TL), row (c / (TL / 2)) % 8, line pair
      const int tl = c / (4 * TL), r = (c / (TL / 2)) % 8, lp = (c % (TL / 2)) * 2;
      const float4 v = *reinterpret_cast<const float4*>(b + tile_at<TL>(tl * TL + lp, y0 + r));
      acc += v.x + v.y + v.z + v.w;
    }
  }
  if (acc == 12345.f) out[0] = acc;
}

// k_rowinv's direct lane loads (lane t of group g: kx = t + 32 jj, row y0 + g, 8 B) from
// B in 16-row panels [y / 16][kx][16] -- no LDS tile, no barrier; two planes in flight
__global__ __launch_bounds__(256, 2) void k_rowinv_direct_pan16(const float2* __restrict__ B, float* out) {
  constexpr int G = 8, RB = N / G;
  const int bid = xcd_group(blockIdx.x);
  const int rb = bid % RB;
  const int job = bid / RB;
  const int grp = threadIdx.x / R, t = threadIdx.x % R;
  const int y = rb * G + grp;
  float acc = 0.f;
  for (int p = 0; p < P; ++p) {
    const float2* b = B + ((size_t)job * P + p) * N * N + (size_t)(y / 16) * N * 16 + y % 16;
    float2 v[R];
#pragma unroll
    for (int jj = 0; jj < R; ++jj) v[jj] = b[(size_t)(t + R * jj) * 16];
#pragma unroll
    for (int jj = 0; jj < R; ++jj) acc += v[jj].x + v[jj].y;
  }
  if (acc == 12345.f) out[0] = acc;
}
// the same from the 1-KB slot tiles (k_rowinv32's loads): kx = t + 32 jj, lower slots only (timing)
__global__ __launch_bounds__(256, 2) void k_rowinv_direct_t8(const float2* __restrict__ B, float* out) {
  constexpr int G = 8, RB = N / G;
  const int bid = xcd_group(blockIdx.x);
  const int rb = bid % RB;
  const int job = bid / RB;
  const int grp = threadIdx.x / R, t = threadIdx.x % R;
  const int y = rb * G + grp;
  float acc = 0.f;
  for (int p = 0; p < P; ++p) {
    const float2* b = B + ((size_t)job * P + p) * N * N;
    float2 v[R];
#pragma unroll
    for (int jj = 0; jj < R; ++jj) v[jj] = b[tile_at<8>((t + R * jj) % N, y)];
#pragma unroll
    for (int jj = 0; jj < R; ++jj) acc += v[jj].x + v[jj].y;
  }
  if (acc == 12345.f) out[0] = acc;
}

template <int PAN>
__global__ __launch_bounds__(256, 2) void k_rowinv_rows(const float2* __restrict__ B, float* out) {
  constexpr int G = 8, RB = N / G, CH16 = N * G / 2;
  const int bid = xcd_group(blockIdx.x);
  const int rb = bid % RB;
  const int job = bid / RB;
  const int y0 = rb * G;
  float acc = 0.f;
  for (int p = 0; p < P; ++p) {
    const float2* b = B + ((size_t)job * P + p) * N * N;
#pragma unroll 4
    for (int i = 0; i < CH16 / 256; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int line = c / (G / 2), r2 = (c % (G / 2)) * 2;
      const int y = y0 + r2;
      const float4 v = *reinterpret_cast<const float4*>(b + (size_t)(y / PAN) * N * PAN + (size_t)line * PAN + y % PAN);
      acc += v.x + v.y + v.z + v.w;
    }
  }
  if (acc == 12345.f) out[0] = acc;
}

// (r06) channel de-aliasing: pad every B band (128 KB at TL = 8) by PADB float2 and every A panel
// (32 KB) by PADA float2, so the 1-KB pieces of one block (B: 64 bands at the band stride; A: 4
// panels per 32 rows) stop landing on the same HBM channel
template <int PADB, int PADA>
__global__ __launch_bounds__(256, 2) void k_col2_pad(const float2* __restrict__ A, float2* __restrict__ B) {
  constexpr int TL = 8, NT = 256, ITER = 4, LB = (N / 2) / (TL * ITER), KSTEP = LB * TL;
  constexpr size_t PLA = (size_t)(N / 2) * N + (size_t)(N / 8) * PADA, PLB = (size_t)N * N + (size_t)(N / 16) * PADB;
  __shared__ __attribute__((aligned(16))) float2 tile[N * TL];
  const int grp = threadIdx.x / R, t = threadIdx.x % R;
  int bid = blockIdx.x;
  const int lb = bid % LB;
  bid /= LB;
  const float2* a = A + (size_t)bid * PLA;
  float2* b = B + (size_t)bid * PLB;
  for (int it = 0; it < ITER; ++it) {
    const int kx0 = lb * TL + it * KSTEP;
    const int kx = kx0 + grp;
    float2 v[R];
#pragma unroll
    for (int jj = 0; jj < R; ++jj) {
      const int y = t + R * jj;
      v[jj] = a[pan_at<8, N / 2>(kx, y) + (size_t)(y / 8) * PADA];
    }
    for (int set = 0; set < 2; ++set) {
      lds_barrier();
#pragma unroll
      for (int k2 = 0; k2 < R; ++k2) {
        const int y = t + R * k2;
        const int band = y / 16, r = y % 16;
        tile[band * 16 * TL + r * TL + (grp ^ (r & (TL - 1)))] = v[k2];
      }
      lds_barrier();
      constexpr int CH = N * TL / 2;
#pragma unroll
      for (int i = 0; i < CH / NT; ++i) {
        const int c = threadIdx.x + NT * i;
        const int band = c / (8 * TL), r = (c / (TL / 2)) % 16, lp = (c % (TL / 2)) * 2;
        const float2 w0 = tile[band * 16 * TL + r * TL + (lp ^ (r & (TL - 1)))];
        const float2 w1 = tile[band * 16 * TL + r * TL + ((lp + 1) ^ (r & (TL - 1)))];
        const int line0 = set == 0 ? kx0 : (kx0 == 0 ? N - TL : N - kx0 - TL);
        *reinterpret_cast<float4*>(b + ((size_t)band * (N / TL) + line0 / TL) * (16 * TL) + (size_t)band * PADB +
                                   r * TL + lp) = make_float4(w0.x, w0.y, w1.x, w1.y);
      }
#pragma unroll
      for (int jj = 0; jj < R; ++jj) v[jj] = make_float2(v[jj].y, v[jj].x);
    }
  }
}

int main() {
  const int jobs = 128;
  const size_t a_bytes = (size_t)jobs * P * (N / 2) * N * 8;   // 4.29 GB
  const size_t a_alloc = a_bytes + (size_t)jobs * P * (N / 8) * 64 * 8 + (1 << 20);   // + A panel pads
  const size_t b_bytes = 2 * a_bytes + (size_t)jobs * P * (N / 16) * 512 * 8 + (1 << 20);   // 8.59 GB + pads
  float2 *A, *B;
  float* o;
  if (hipMalloc(&A, a_alloc) != hipSuccess || hipMalloc(&B, b_bytes) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(A, 0, a_alloc);
  (void)hipMemset(B, 0, b_bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto time = [&](const char* name, double moved, auto launch) {
    launch();
    (void)hipDeviceSynchronize();
    float best = 1e30f, sum = 0.f;
    const int reps = 7;
    for (int r = 0; r < reps; ++r) {
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
      sum += ms;
    }
    printf("{\"kernel\": \"%s\", \"GBs_best\": %.1f, \"GBs_avg\": %.1f, \"ms_best\": %.4f, \"bytes\": %.0f}\n", name,
           moved / (best * 1e-3) / 1e9, moved / (sum / reps * 1e-3) / 1e9, best, moved);
    fflush(stdout);
  };
  const size_t n16 = a_bytes / 16;
  const unsigned g16 = (unsigned)(n16 / 256);
  time("flat_r1w2", 3.0 * a_bytes,
       [&] { hipLaunchKernelGGL(k_r1w2_flat, g16, 256, 0, 0, (const float4*)A, (float4*)B, n16); });
  const unsigned gcol = jobs * P * 16;
  for (int rep = 0; rep < 2; ++rep) {
    time("col2_T8", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_tiled<8>), gcol, 256, 0, 0, A, B); });
    time("col2_pad_0_0", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pad<0, 0>), gcol, 256, 0, 0, A, B); });
    time("col2_pad_128_0", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pad<128, 0>), gcol, 256, 0, 0, A, B); });
    time("col2_pad_256_0", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pad<256, 0>), gcol, 256, 0, 0, A, B); });
    time("col2_pad_512_0", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pad<512, 0>), gcol, 256, 0, 0, A, B); });
    time("col2_pad_0_32", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pad<0, 32>), gcol, 256, 0, 0, A, B); });
    time("col2_pad_0_64", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pad<0, 64>), gcol, 256, 0, 0, A, B); });
    time("col2_pad_128_32", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pad<128, 32>), gcol, 256, 0, 0, A, B); });
    time("col2_pad_256_64", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pad<256, 64>), gcol, 256, 0, 0, A, B); });
    time("flat_r1w2", 3.0 * a_bytes,
         [&] { hipLaunchKernelGGL(k_r1w2_flat, g16, 256, 0, 0, (const float4*)A, (float4*)B, n16); });
  }
  return 0;
}
