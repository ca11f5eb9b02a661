// membw.hip -- HBM bandwidth calibration for the traffic mixes of the hbx passes.
// read-only, write-only, copy (1 read : 1 write), and 1 read : 2 writes (the
// column pass).  16-B per lane, grid-stride, large buffers (>> 256 MiB L3).
// build: hipcc -O3 --offload-arch=gfx950 tools/membw.hip -o tools/membw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_read(const float4* __restrict__ a, size_t n, float* out) {
  float4 acc = make_float4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[0] = 1.f;
}
__global__ void k_write(float4* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_float4(1, 2, 3, (float)i);
}
__global__ void k_copy(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}
__global__ void k_r1w2(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    b[2 * i] = v;
    b[2 * i + 1] = make_float4(v.y, v.x, v.w, v.z);
  }
}

// 8 B per lane (float2): the column pass's access width
__global__ void k_read8(const float2* __restrict__ a, size_t n, float* out) {
  float2 acc = make_float2(0, 0);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float2 v = a[i];
    acc.x += v.x; acc.y += v.y;
  }
  if (acc.x + acc.y == 12345.f) out[0] = 1.f;
}
__global__ void k_write8(float2* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_float2(1, (float)i);
}
__global__ void k_copy8(const float2* __restrict__ a, float2* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}
// one element per thread, no grid-stride loop (grid = n / 256)
__global__ void k_copy_flat(const float4* __restrict__ a, float4* __restrict__ b) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  b[i] = a[i];
}

int main() {
  const size_t bytes = (size_t)4 << 30;  // 4 GiB per buffer
  const size_t n = bytes / sizeof(float4);
  float4 *a, *b;
  float* o;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, 2 * bytes) != hipSuccess ||
      hipMalloc(&o, 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
  (void)hipMemset(a, 0, bytes);
  (void)hipMemset(b, 0, 2 * bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = 256 * 16, block = 256;
  auto time = [&](const char* name, double moved, auto launch) {
    launch();
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("{\"kernel\": \"%s\", \"GBs\": %.1f, \"ms\": %.3f}\n", name, moved / (best * 1e-3) / 1e9, best);
  };
  time("read", (double)bytes, [&] { hipLaunchKernelGGL(k_read, grid, block, 0, 0, a, n, o); });
  time("write", (double)bytes, [&] { hipLaunchKernelGGL(k_write, grid, block, 0, 0, a, n); });
  time("copy_r1w1", 2.0 * bytes, [&] { hipLaunchKernelGGL(k_copy, grid, block, 0, 0, a, b, n); });
  time("r1w2", 3.0 * bytes, [&] { hipLaunchKernelGGL(k_r1w2, grid, block, 0, 0, a, b, n); });
  time("read8", (double)bytes, [&] { hipLaunchKernelGGL(k_read8, grid, block, 0, 0, (const float2*)a, 2 * n, o); });
  time("write8", (double)bytes, [&] { hipLaunchKernelGGL(k_write8, grid, block, 0, 0, (float2*)a, 2 * n); });
  time("copy8_r1w1", 2.0 * bytes, [&] { hipLaunchKernelGGL(k_copy8, grid, block, 0, 0, (const float2*)a, (float2*)b, 2 * n); });
  time("copy_flat_r1w1", 2.0 * bytes, [&] { hipLaunchKernelGGL(k_copy_flat, (unsigned)(n / 256), block, 0, 0, a, b); });
  for (int g : {1024, 2048, 8192, 16384}) {
    char nm[64];
    snprintf(nm, sizeof nm, "copy_r1w1_grid%d", g);
    time(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL(k_copy, g, block, 0, 0, a, b, n); });
  }
  return 0;
}
