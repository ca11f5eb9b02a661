// lane_xor_test.hip -- checks hbx_fft.hpp's DPP / permlane lane exchanges (r05) against the
// ds_swizzle forms they replace: lane_xor<J> for J = 1..16, and the whole 32 x 32 group bit
// transpose against the swizzle transpose and a host reference.  Build:
//   hipcc -O3 --offload-arch=gfx950 -I binary-hologram-reinforcement-learning_amd/csrc tools/lane_xor_test.hip -o tools/lane_xor_test
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "hbx_fft.hpp"

using namespace hbx;

template <int J>
__device__ uint32_t swz(uint32_t x) { return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, (J << 10) | 0x1f); }

__global__ void k(const uint32_t* in, uint32_t* out) {
  const int lane = threadIdx.x, t = lane % 32;
  const uint32_t x = in[blockIdx.x * 64 + lane];
  uint32_t* o = out + (size_t)blockIdx.x * 64 * 12 + lane * 12;
  o[0] = lane_xor<1>(x, t);  o[1] = swz<1>(x);
  o[2] = lane_xor<2>(x, t);  o[3] = swz<2>(x);
  o[4] = lane_xor<4>(x, t);  o[5] = swz<4>(x);
  o[6] = lane_xor<8>(x, t);  o[7] = swz<8>(x);
  o[8] = lane_xor<16>(x, t); o[9] = swz<16>(x);
  o[10] = group_bit_transpose(x, t);
  o[11] = group_bit_transpose_swizzle(x, t);
}

int main() {
  const int blocks = 64, n = blocks * 64;
  uint32_t* h = (uint32_t*)malloc(n * 4);
  uint32_t* r = (uint32_t*)malloc((size_t)n * 12 * 4);
  srand(7);
  for (int i = 0; i < n; ++i) h[i] = ((uint32_t)rand() << 16) ^ (uint32_t)rand() ^ (i & 1 ? 0x80000001u : 0);
  uint32_t *din, *dout;
  if (hipMalloc(&din, n * 4) || hipMalloc(&dout, (size_t)n * 12 * 4)) { printf("alloc failed\n"); return 2; }
  (void)hipMemcpy(din, h, n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, din, dout);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
  (void)hipMemcpy(r, dout, (size_t)n * 12 * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  const int Js[5] = {1, 2, 4, 8, 16};
  for (int b = 0; b < blocks; ++b)
    for (int lane = 0; lane < 64; ++lane) {
      const uint32_t* o = r + ((size_t)b * 64 + lane) * 12;
      for (int q = 0; q < 5; ++q) {
        const uint32_t want = h[b * 64 + (lane ^ Js[q])];
        if (o[2 * q] != want || o[2 * q + 1] != want) {
          if (bad < 10) printf("J=%d block %d lane %d: dpp %08x swizzle %08x want %08x\n", Js[q], b, lane, o[2 * q], o[2 * q + 1], want);
          ++bad;
        }
      }
      uint32_t want = 0;   // bit r of lane t = bit t of lane r (same 32-lane group)
      const int g0 = lane & 32, t = lane & 31;
      for (int rr = 0; rr < 32; ++rr) want |= ((h[b * 64 + g0 + rr] >> t) & 1u) << rr;
      if (o[10] != want || o[11] != want) {
        if (bad < 10) printf("transpose block %d lane %d: dpp %08x swizzle %08x want %08x\n", b, lane, o[10], o[11], want);
        ++bad;
      }
    }
  printf("lane_xor_test: %d mismatches over %d lanes\n", bad, n);
  return bad ? 1 : 0;
}
