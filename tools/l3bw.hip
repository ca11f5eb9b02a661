// l3bw.hip -- does a chunked launch schedule keep the pass intermediates in the
// 256 MiB Infinity Cache?  Emulates the three-pass traffic of one env step:
//   k1: read a small input slice (mask bits), write A (S bytes)
//   k2: read A, write B (2 S bytes)
//   k3: read B (2 S bytes), reduce to a scalar
// over TOTAL bytes of A-equivalent work, split into chunks of S bytes that
// reuse the same A / B buffers.  Prints the effective rate (algorithmic bytes
// of k1+k2+k3 / wall time) per chunk size, plus per-kernel averages.
// build: hipcc -O3 --offload-arch=gfx950 tools/l3bw.hip -o tools/l3bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

__global__ void k1(const float4* __restrict__ in, float4* __restrict__ a, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = in[i / 64];   // 1/64 of the output volume read (bit-packed masks)
    a[i] = make_float4(v.x + (float)i, v.y, v.z, v.w);
  }
}
__global__ void k2(const float4* __restrict__ a, float4* __restrict__ b, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    b[2 * i] = v;
    b[2 * i + 1] = make_float4(v.y, v.x, v.w, v.z);
  }
}
__global__ void k3(const float4* __restrict__ b, size_t n4, float* out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < 2 * n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = b[i];
    acc += v.x * v.x + v.y * v.y + v.z + v.w;
  }
  if (acc == 12345.f) out[0] = acc;
}

int main(int argc, char** argv) {
  const size_t total = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 4096ull) << 20;   // MiB of A
  const size_t chunks_mb[] = {16, 32, 48, 64, 96, 128, 192, 256, 512, 4096};
  float4 *in, *a, *b;
  float* out;
  const size_t max_chunk = 4096ull << 20;
  CHECK(hipMalloc(&in, total / 64 + 4096));
  CHECK(hipMalloc(&a, max_chunk));
  CHECK(hipMalloc(&b, 2 * max_chunk));
  CHECK(hipMalloc(&out, 4));
  CHECK(hipMemset(in, 0, total / 64 + 4096));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int blocks = 256 * 8, nt = 256;
  for (size_t cm : chunks_mb) {
    const size_t S = cm << 20;
    if (S > total) continue;
    const size_t n4 = S / 16;
    const size_t nchunks = total / S;
    for (int rep = 0; rep < 3; ++rep) {
      CHECK(hipEventRecord(e0, 0));
      for (size_t c = 0; c < nchunks; ++c) {
        hipLaunchKernelGGL(k1, dim3(blocks), dim3(nt), 0, 0, in + c * (n4 / 64), a, n4);
        hipLaunchKernelGGL(k2, dim3(blocks), dim3(nt), 0, 0, a, b, n4);
        hipLaunchKernelGGL(k3, dim3(blocks), dim3(nt), 0, 0, b, n4, out);
      }
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double bytes = (double)nchunks * (double)S * (1.0 / 64 + 1 + 1 + 2 + 2 + 0);
      if (rep == 2)
        std::printf("chunk %5zu MiB x %5zu: %8.3f ms  %7.1f GB/s effective (k1 w S, k2 r S w 2S, k3 r 2S)\n", cm,
                    nchunks, ms, bytes / (ms * 1e6));
    }
  }
  return 0;
}
