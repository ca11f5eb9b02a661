// membw256.hip -- read-rate floor of N = 256 k_rowinv_d's access pattern, without arithmetic.
//   linear<G>   570 MB read as G blocks x 256 threads, 16-B lanes, contiguous chunk per block
//   rowinv<RI>  k_rowinv_d<16>'s loads: per block 16 rows (one 16-row band) x 8 planes of a
//               job, lane t of group g: 16 x 8-B loads (tile layout), two planes in flight
// build: hipcc -O3 --offload-arch=gfx950 tools/membw256.hip -o tools/membw256
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

typedef float float2v __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_linear(const float4* __restrict__ in, size_t per_block, float* out) {
  const float4* p = in + blockIdx.x * per_block;
  float4 a = {0, 0, 0, 0};
  for (size_t i = threadIdx.x; i < per_block; i += 256 * 4) {
    float4 v0 = p[i], v1 = p[i + 256], v2 = p[i + 512], v3 = p[i + 768];
    a.x += v0.x + v1.x + v2.x + v3.x;
    a.y += v0.y + v1.y + v2.y + v3.y;
  }
  if (a.x == 12345.f) out[0] = a.y;
}

// B of J jobs: [J][P = 8][256 x 256 float2], tiled [y/16][s/16][16 rows][16 slots]
template <int RI>
__global__ __launch_bounds__(256, 2) void k_rowinv(const float2v* __restrict__ b, float* out) {
  constexpr int R = 16, N = 256, TL = 16, P = 8, RB = 16, PLB = N * N;
  const int grp = threadIdx.x / R, t = threadIdx.x % R;
  const int bid = blockIdx.x;
  const int rb0 = (bid % (RB / RI)) * RI, j = bid / (RB / RI);
  const float2v* base = b + (size_t)j * P * PLB;
  const int y = rb0 * 16 + grp;
  const int yb = (y >> 4) * 16 * N + (y & 15) * TL;
  float acc = 0.f;
  for (int it = 0; it < RI; ++it) {
    for (int p = 0; p < P; ++p) {
      const float2v* pl = base + (size_t)p * PLB + it * 16 * N + yb;
      float2v v[R];
#pragma unroll
      for (int jj = 0; jj < R; ++jj) v[jj] = pl[jj * 16 * TL + t];
#pragma unroll
      for (int jj = 0; jj < R; ++jj) acc += v[jj].x * v[jj].x + v[jj].y;
    }
  }
  if (acc == 12345.f) out[0] = acc;
}

int main() {
  const size_t J = 128, bytes = J * 8 * 256 * 256 * 8;   // 512 MiB
  void* buf;
  float* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 5; ++w) launch();
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int r = 0; r < 20; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    printf("%-16s %.4f ms  %.0f GB/s\n", name, best, bytes / (best * 1e-3) / 1e9);
  };
  for (int G : {512, 1024, 2048, 4096, 8192, 16384}) {
    char nm[32];
    snprintf(nm, sizeof nm, "linear<%d>", G);
    const size_t per = bytes / 16 / G;
    run(nm, [&] { hipLaunchKernelGGL(k_linear, dim3(G), dim3(256), 0, 0, (const float4*)buf, per, out); });
  }
  run("rowinv<1>", [&] { hipLaunchKernelGGL(k_rowinv<1>, dim3(J * 16), dim3(256), 0, 0, (const float2v*)buf, out); });
  run("rowinv<2>", [&] { hipLaunchKernelGGL(k_rowinv<2>, dim3(J * 8), dim3(256), 0, 0, (const float2v*)buf, out); });
  run("rowinv<4>", [&] { hipLaunchKernelGGL(k_rowinv<4>, dim3(J * 4), dim3(256), 0, 0, (const float2v*)buf, out); });
  return 0;
}
