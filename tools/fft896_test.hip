// fft896_test.hip -- checks the 896-point lane-group FFT (hbx_fft.hpp,
// fft896_ns / fft896_sn) against a double-precision DFT on the host.
//   hipcc -O3 -std=c++17 -fno-slp-vectorize --offload-arch=gfx950 tools/fft896_test.hip -o tools/fft896_test
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../binary-hologram-reinforcement-learning_amd/csrc/hbx_fft.hpp"

using namespace hbx;
constexpr int N = 896;

__global__ __launch_bounds__(256) void k_test(const float2* x, float2* X, float2* xr, const float2* twg) {
  __shared__ float2 tw[N];
  __shared__ float2 scratch[8 * 32 * 33];
  for (int i = threadIdx.x; i < N; i += 256) tw[i] = twg[i];
  __syncthreads();
  const int grp = threadIdx.x / 32, t = threadIdx.x % 32;
  const int line = blockIdx.x * 8 + grp;
  const PaddedScratch<32> sc{scratch + grp * 32 * 33};
  float2 v[32];
  for (int j = 0; j < 28; ++j) v[j] = x[line * N + t + 32 * j];
  fft896_ns<false>(v, t, sc, tw);
  if (t < 28)
    for (int k2 = 0; k2 < 32; ++k2) X[line * N + t + 28 * k2] = v[k2];
  __syncthreads();
  if (t < 28)
    for (int k2 = 0; k2 < 32; ++k2) v[k2] = X[line * N + t + 28 * k2];
  fft896_sn<true>(v, t, sc, tw);
  for (int j = 0; j < 28; ++j) xr[line * N + t + 32 * j] = v[j];
}

int main() {
  const int lines = 8;
  std::vector<float2> x(lines * N), X(lines * N), xr(lines * N), tw(N);
  srand(3);
  for (auto& e : x) e = make_float2(rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f);
  for (int k1 = 0; k1 < 28; ++k1)
    for (int t = 0; t < 32; ++t) {
      const double a = -2.0 * M_PI * (double)(t * k1) / N;
      tw[k1 * 32 + t] = make_float2((float)cos(a), (float)sin(a));
    }
  float2 *dx, *dX, *dxr, *dt;
  (void)hipMalloc(&dx, x.size() * 8); (void)hipMalloc(&dX, x.size() * 8);
  (void)hipMalloc(&dxr, x.size() * 8); (void)hipMalloc(&dt, N * 8);
  (void)hipMemcpy(dx, x.data(), x.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dt, tw.data(), N * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_test, dim3(lines / 8), dim3(256), 0, 0, dx, dX, dxr, dt);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
  (void)hipMemcpy(X.data(), dX, x.size() * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(xr.data(), dxr, x.size() * 8, hipMemcpyDeviceToHost);
  double ef = 0, ei = 0, mag = 0;
  for (int l = 0; l < lines; ++l)
    for (int k = 0; k < N; ++k) {
      double re = 0, im = 0;
      for (int n = 0; n < N; ++n) {
        const double a = -2.0 * M_PI * (double)((long)n * k % N) / N;
        const float2 e = x[l * N + n];
        re += e.x * cos(a) - e.y * sin(a);
        im += e.x * sin(a) + e.y * cos(a);
      }
      ef = fmax(ef, hypot(re - X[l * N + k].x, im - X[l * N + k].y));
      mag = fmax(mag, hypot(re, im));
      ei = fmax(ei, hypot(xr[l * N + k].x / N - x[l * N + k].x, xr[l * N + k].y / N - x[l * N + k].y));
    }
  printf("{\"fwd_max_abs_err\": %.3e, \"spectrum_max\": %.3e, \"roundtrip_max_abs_err\": %.3e}\n", ef, mag, ei);
  return (ef < 1e-4 * mag && ei < 1e-5) ? 0 : 1;
}
