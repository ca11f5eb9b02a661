// membw2.hip -- streaming ceilings measured with FLAT kernels (one 16-B element per
// thread, grid = elements / 256, no grid-stride loop) and the data movement of the
// hbx passes replayed without their arithmetic, so the pass efficiency claims in
// DESIGN.md rest on measured ceilings of the same access shapes.
//
//   flat_read / flat_write / flat_copy (r1w1) / flat_r1w2 (one read, two written
//   streams)                                         -- the chip's streaming ceilings
//   col2_pan<PAN>   k_col2's movement: per block 8 lines kx of one plane, 4 iterations;
//                   read A line kx (8 KB contiguous, 8 B per lane, 32 loads per lane),
//                   write B lines kx and N - kx in panels of PAN rows
//   rowfwd_rows<G>  k_rowfwd's stores: G rows per block -> 8 G-byte pieces of every
//                   line of the line-major A plane pair
//   rowinv_rows<G>  k_rowinv's loads: G rows of every line of 8 B planes in 16-row panels
//
// build: hipcc -O3 --offload-arch=gfx950 tools/membw2.hip -o tools/membw2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

constexpr int N = 1024, R = 32, P = 8;

__global__ void k_read_flat(const float4* __restrict__ a, float* out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const float4 v = a[i];
  if (v.x + v.y + v.z + v.w == 12345.f) out[0] = 1.f;
}
__global__ void k_write_flat(float4* __restrict__ a) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  a[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}
__global__ void k_copy_flat(const float4* __restrict__ a, float4* __restrict__ b) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  b[i] = a[i];
}
__global__ void k_r1w2_flat(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const float4 v = a[i];
  b[i] = v;
  b[i + n] = make_float4(v.y, v.x, v.w, v.z);
}
// 8 B per lane, flat
__global__ void k_write8_flat(float2* __restrict__ a) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  a[i] = make_float2(1.f, (float)i);
}
__global__ void k_r1w2_8_flat(const float2* __restrict__ a, float2* __restrict__ b, size_t n) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const float2 v = a[i];
  b[i] = v;
  b[i + n] = make_float2(v.y, v.x);
}

// k_col2 replayed: grid = jobs * P * LB, LB = 16; block = 8 lane groups of 32 lanes
// element (line, y) of a plane of L lines stored in panels of PAN rows
template <int PAN, int L>
__device__ __forceinline__ size_t pan_at(int line, int y) {
  return (size_t)(y / PAN) * L * PAN + (size_t)line * PAN + y % PAN;
}

// XCD-aware grouping of consecutive row blocks (hbx_rowcol.hpp xcd_pair, GS = 16)
__device__ __forceinline__ int xcd_group(int bid) {
  constexpr int GS = 16, SPAN = 8 * GS;
  return (bid / SPAN) * SPAN + (bid % 8) * GS + (bid / 8) % GS;
}

template <int PANA, int PAN, int ITER = 4>
__global__ __launch_bounds__(256, 2) void k_col2_pan(const float2* __restrict__ A, float2* __restrict__ B) {
  constexpr int GPB = 8, LB = (N / 2) / (GPB * ITER), KSTEP = LB * GPB;
  constexpr size_t PLA = (size_t)(N / 2) * N, PLB = (size_t)N * N;
  const int grp = threadIdx.x / R, t = threadIdx.x % R;
  int bid = blockIdx.x;
  const int lb = bid % LB;
  bid /= LB;   // plane index (job * P + p)
  const float2* a = A + (size_t)bid * PLA;
  float2* b = B + (size_t)bid * PLB;
  for (int it = 0; it < ITER; ++it) {
    const int kx = lb * GPB + grp + it * KSTEP;
    float2 v[R];
#pragma unroll
    for (int jj = 0; jj < R; ++jj) v[jj] = a[pan_at<PANA, N / 2>(kx, t + R * jj)];
    const int k2 = kx == 0 ? N / 2 : N - kx;
#pragma unroll
    for (int jj = 0; jj < R; ++jj) {
      const int y = t + R * jj;
      b[(size_t)(y / PAN) * N * PAN + (size_t)kx * PAN + y % PAN] = v[jj];
    }
#pragma unroll
    for (int jj = 0; jj < R; ++jj) {
      const int y = t + R * jj;
      b[(size_t)(y / PAN) * N * PAN + (size_t)k2 * PAN + y % PAN] = make_float2(v[jj].y, v[jj].x);
    }
  }
}

// k_col2's movement with 16 B per lane: lane t of a group holds y = 2t, 2t+1 (+ 64 jj)
template <int PANA, int PAN>
__global__ __launch_bounds__(256, 2) void k_col2_pan16B(const float2* __restrict__ A, float2* __restrict__ B) {
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
    float4 v[R / 2];
#pragma unroll
    for (int jj = 0; jj < R / 2; ++jj)
      v[jj] = *reinterpret_cast<const float4*>(a + pan_at<PANA, N / 2>(kx, 2 * t + 2 * R * jj));
    const int k2 = kx == 0 ? N / 2 : N - kx;
#pragma unroll
    for (int jj = 0; jj < R / 2; ++jj) {
      const int y = 2 * t + 2 * R * jj;
      *reinterpret_cast<float4*>(b + (size_t)(y / PAN) * N * PAN + (size_t)kx * PAN + y % PAN) = v[jj];
    }
#pragma unroll
    for (int jj = 0; jj < R / 2; ++jj) {
      const int y = 2 * t + 2 * R * jj;
      *reinterpret_cast<float4*>(b + (size_t)(y / PAN) * N * PAN + (size_t)k2 * PAN + y % PAN) =
          make_float4(v[jj].y, v[jj].x, v[jj].w, v[jj].z);
    }
  }
}

// k_col2's movement, 8 B per lane, whole A line loaded but B stored per 64 lanes: a wave
// = ONE line (64 lanes x 8 B = 512 B contiguous per instruction)
template <int PANA, int PAN>
__global__ __launch_bounds__(256, 2) void k_col2_wave(const float2* __restrict__ A, float2* __restrict__ B) {
  constexpr int WPB = 4, ITER = 8, LB = (N / 2) / (WPB * ITER), KSTEP = LB * WPB;
  constexpr size_t PLA = (size_t)(N / 2) * N, PLB = (size_t)N * N;
  const int w = threadIdx.x / 64, l = threadIdx.x % 64;
  int bid = blockIdx.x;
  const int lb = bid % LB;
  bid /= LB;
  const float2* a = A + (size_t)bid * PLA;
  float2* b = B + (size_t)bid * PLB;
  for (int it = 0; it < ITER; ++it) {
    const int kx = lb * WPB + w + it * KSTEP;
    float2 v[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) v[jj] = a[pan_at<PANA, N / 2>(kx, l + 64 * jj)];
    const int k2 = kx == 0 ? N / 2 : N - kx;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      const int y = l + 64 * jj;
      b[(size_t)(y / PAN) * N * PAN + (size_t)kx * PAN + y % PAN] = v[jj];
    }
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      const int y = l + 64 * jj;
      b[(size_t)(y / PAN) * N * PAN + (size_t)k2 * PAN + y % PAN] = make_float2(v[jj].y, v[jj].x);
    }
  }
}

// k_rowfwd's stores: block = G rows of a plane pair (2 x N/2 lines of N y, line-major),
// 16 B (two y) per thread per chunk; consecutive blocks = consecutive row blocks
template <int G>
__global__ __launch_bounds__(256, 2) void k_rowfwd_rows(float2* __restrict__ A) {
  constexpr int RB = N / G, CHUNKS = N * G / 2;
  const int rb = blockIdx.x % RB;
  const int pair = blockIdx.x / RB;
  float2* base = A + (size_t)pair * 2 * (N / 2) * N;
  const int y0 = rb * G;
#pragma unroll 4
  for (int i = 0; i < CHUNKS / 256; ++i) {
    const int c = threadIdx.x + 256 * i;
    const int r2 = (c % (G / 2)) * 2;
    const int line = c / (G / 2);
    *reinterpret_cast<float4*>(base + (size_t)line * N + y0 + r2) = make_float4(1.f, 2.f, (float)c, (float)i);
  }
}

// k_rowfwd's stores into A stored in panels of PAN = G rows: one contiguous panel per block
template <int G, bool XCD>
__global__ __launch_bounds__(256, 2) void k_rowfwd_panel(float2* __restrict__ A) {
  constexpr int RB = N / G, CHUNKS = N * G / 2;
  const int bid = XCD ? xcd_group(blockIdx.x) : blockIdx.x;
  const int rb = bid % RB;
  const int pair = bid / RB;
  float2* base = A + (size_t)pair * 2 * (N / 2) * N;
  const int y0 = rb * G;
#pragma unroll 4
  for (int i = 0; i < CHUNKS / 256; ++i) {
    const int c = threadIdx.x + 256 * i;
    const int r2 = (c % (G / 2)) * 2;
    const int line = c / (G / 2);   // 0 .. N-1: plane (line / (N/2)), line % (N/2)
    const int pl = line / (N / 2);
    *reinterpret_cast<float4*>(base + (size_t)pl * (N / 2) * N + pan_at<G, N / 2>(line % (N / 2), y0 + r2)) =
        make_float4(1.f, 2.f, (float)c, (float)i);
  }
}

// k_rowinv's loads: block = G rows, all P planes of one job; B planes in panels of PAN rows
template <int G, int PAN = 16, bool XCD = false>
__global__ __launch_bounds__(256, 2) void k_rowinv_rows(const float2* __restrict__ B, float* out) {
  constexpr int RB = N / G, CH16 = N * G / 2;
  const int bid = XCD ? xcd_group(blockIdx.x) : blockIdx.x;
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

int main(int argc, char** argv) {
  const int jobs = 128;
  const size_t a_bytes = (size_t)jobs * P * (N / 2) * N * 8;   // 4.29 GB: A of 128 jobs
  const size_t b_bytes = 2 * a_bytes;                           // 8.59 GB: B of 128 jobs
  float2 *A, *B;
  float* o;
  if (hipMalloc(&A, a_bytes) != hipSuccess || hipMalloc(&B, b_bytes) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(A, 0, a_bytes);
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
  const size_t n16 = a_bytes / 16;            // float4 elements of A
  const unsigned g16 = (unsigned)(n16 / 256);
  time("flat_read", (double)a_bytes, [&] { hipLaunchKernelGGL(k_read_flat, g16, 256, 0, 0, (const float4*)A, o); });
  time("flat_write", (double)a_bytes, [&] { hipLaunchKernelGGL(k_write_flat, g16, 256, 0, 0, (float4*)A); });
  time("flat_write8", (double)a_bytes, [&] { hipLaunchKernelGGL(k_write8_flat, 2 * g16, 256, 0, 0, A); });
  time("flat_copy_r1w1", 2.0 * a_bytes,
       [&] { hipLaunchKernelGGL(k_copy_flat, g16, 256, 0, 0, (const float4*)A, (float4*)B); });
  time("flat_r1w2", 3.0 * a_bytes,
       [&] { hipLaunchKernelGGL(k_r1w2_flat, g16, 256, 0, 0, (const float4*)A, (float4*)B, n16); });
  time("flat_r1w2_8B", 3.0 * a_bytes,
       [&] { hipLaunchKernelGGL(k_r1w2_8_flat, 2 * g16, 256, 0, 0, A, B, 2 * n16); });
  const unsigned gcol = jobs * P * 16;
#define COL2(PA_, PB_) time("col2_A" #PA_ "_B" #PB_, 3.0 * a_bytes, \
                            [&] { hipLaunchKernelGGL((k_col2_pan<PA_, PB_>), gcol, 256, 0, 0, A, B); })
  COL2(1024, 16); COL2(1024, 32); COL2(1024, 64); COL2(1024, 1024);
  COL2(8, 16); COL2(16, 16); COL2(32, 16); COL2(8, 8); COL2(16, 32); COL2(8, 32);
#define COL2W(PA_, PB_) time("col2w_A" #PA_ "_B" #PB_, 3.0 * a_bytes, \
                             [&] { hipLaunchKernelGGL((k_col2_wave<PA_, PB_>), gcol, 256, 0, 0, A, B); })
#define COL2Q(PA_, PB_) time("col2_16B_A" #PA_ "_B" #PB_, 3.0 * a_bytes, \
                             [&] { hipLaunchKernelGGL((k_col2_pan16B<PA_, PB_>), gcol, 256, 0, 0, A, B); })
  for (int reps = 0; reps < 1; ++reps) {
    time("col2_A8_B16_it1", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pan<8, 16, 1>), gcol * 4, 256, 0, 0, A, B); });
    time("col2_A8_B16_it2", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pan<8, 16, 2>), gcol * 2, 256, 0, 0, A, B); });
    time("col2_A8_B16_it8", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pan<8, 16, 8>), gcol / 2, 256, 0, 0, A, B); });
    time("col2_A8_B16_it16", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pan<8, 16, 16>), gcol / 4, 256, 0, 0, A, B); });
    time("col2_A8_B64_it1", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pan<8, 64, 1>), gcol * 4, 256, 0, 0, A, B); });
    time("col2_A8_B1024_it1", 3.0 * a_bytes, [&] { hipLaunchKernelGGL((k_col2_pan<8, 1024, 1>), gcol * 4, 256, 0, 0, A, B); });
  }
  const unsigned gfw8 = jobs * (P / 2) * (N / 8), gfw16 = jobs * (P / 2) * (N / 16);
  time("rowfwd_panel8", (double)a_bytes, [&] { hipLaunchKernelGGL((k_rowfwd_panel<8, false>), gfw8, 256, 0, 0, A); });
  time("rowfwd_panel8_xcd", (double)a_bytes, [&] { hipLaunchKernelGGL((k_rowfwd_panel<8, true>), gfw8, 256, 0, 0, A); });
  time("rowfwd_panel16", (double)a_bytes, [&] { hipLaunchKernelGGL((k_rowfwd_panel<16, false>), gfw16, 256, 0, 0, A); });
  time("rowinv_rows8_pan8", (double)b_bytes,
       [&] { hipLaunchKernelGGL((k_rowinv_rows<8, 8>), jobs * (N / 8), 256, 0, 0, B, o); });
  time("rowinv_rows8_pan16_xcd", (double)b_bytes,
       [&] { hipLaunchKernelGGL((k_rowinv_rows<8, 16, true>), jobs * (N / 8), 256, 0, 0, B, o); });
  time("rowinv_rows8_pan8_xcd", (double)b_bytes,
       [&] { hipLaunchKernelGGL((k_rowinv_rows<8, 8, true>), jobs * (N / 8), 256, 0, 0, B, o); });
  time("rowfwd_rows8", (double)a_bytes,
       [&] { hipLaunchKernelGGL(k_rowfwd_rows<8>, jobs * (P / 2) * (N / 8), 256, 0, 0, A); });
  time("rowfwd_rows16", (double)a_bytes,
       [&] { hipLaunchKernelGGL(k_rowfwd_rows<16>, jobs * (P / 2) * (N / 16), 256, 0, 0, A); });
  time("rowfwd_rows32", (double)a_bytes,
       [&] { hipLaunchKernelGGL(k_rowfwd_rows<32>, jobs * (P / 2) * (N / 32), 256, 0, 0, A); });
  time("rowinv_rows8", (double)b_bytes, [&] { hipLaunchKernelGGL(k_rowinv_rows<8>, jobs * (N / 8), 256, 0, 0, B, o); });
  time("rowinv_rows16", (double)b_bytes,
       [&] { hipLaunchKernelGGL(k_rowinv_rows<16>, jobs * (N / 16), 256, 0, 0, B, o); });
  return 0;
}
