/* A host program in plain C on the C-ABI alone (include/hbx.h + the HIP runtime's C API, no
 * Python, no torch): what a cgo / JNI / N-API binding of the reference's env.step would drive
 * (env.py:90-259, train-PPO.py:296-322).  B envs of the 256x256x8 mono env:
 *   hbx_plan_create -> hbx_env_reset -> n_steps x hbx_env_step (results written by the step
 *   kernels into hbx_host_alloc'd host-mapped memory) -> checks:
 *   - every reward finite, some steps accepted and some rolled back;
 *   - prev_psnr of every env equals hbx_propagate + hbx_psnr of its current mask (the FFT mode
 *     re-propagates the touched group every step, so the two agree to the last bits);
 *   - an out-of-range action sets the error word mirrored into host memory (env->error_host).
 * Prints one line "env_step_host: ... OK" and exits 0, or prints the failed check and exits 1.
 * Built by __graft_entry__.build() (gcc, -lhbx -lamdhip64); run by tests/test_gpu_c_host.py. */
#define _POSIX_C_SOURCE 199309L
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "hbx.h"

#define CHECK_HIP(x)                                                          \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d HIP %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                               \
    }                                                                         \
  } while (0)
#define CHECK_HBX(x)                                                          \
  do {                                                                        \
    int r_ = (x);                                                             \
    if (r_ != HBX_OK) {                                                       \
      fprintf(stderr, "%s:%d hbx %d: %s\n", __FILE__, __LINE__, r_, hbx_last_error()); \
      return 1;                                                               \
    }                                                                         \
  } while (0)
#define EXPECT(c)                                                             \
  do {                                                                        \
    if (!(c)) {                                                               \
      fprintf(stderr, "%s:%d check failed: %s\n", __FILE__, __LINE__, #c);     \
      return 1;                                                               \
    }                                                                         \
  } while (0)

static uint64_t rng_state = 0x9e3779b97f4a7c15ull;
static uint64_t rng_next(void) {   /* splitmix64 */
  uint64_t z = (rng_state += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

static void* dalloc(size_t bytes) {
  void* p = NULL;
  if (hipMalloc(&p, bytes) != hipSuccess) return NULL;
  if (hipMemset(p, 0, bytes) != hipSuccess) return NULL;
  return p;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 16;
  const int n_steps = argc > 2 ? atoi(argv[2]) : 200;
  const int N = 256, G = 1, P = 8, CH = G * P;
  const size_t hw = (size_t)N * N;
  EXPECT(hbx_abi_version() == HBX_ABI_VERSION);

  hbx_optics_t o;
  memset(&o, 0, sizeof(o));
  o.height = N; o.width = N; o.groups = G; o.planes = P;
  o.wavelength[0] = 515e-9;                      /* env.py:124 */
  o.dx = o.dy = 7.56e-6; o.z = 2e-3;             /* env.py:124,172 */
  o.tf_kind = HBX_TF_ASM; o.field_kind = HBX_FIELD_AMPLITUDE; o.rel_scale = HBX_REL_LSQ; o.peak = 1.0;
  hbx_plan_t plan = NULL;
  CHECK_HBX(hbx_plan_create(&plan, &o, B, 0));

  /* env buffers (caller-owned device memory) */
  const size_t mwords = (size_t)B * CH * N * (N / 64);
  hbx_env_buffers_t e;
  memset(&e, 0, sizeof(e));
  e.mask = (uint64_t*)dalloc(mwords * 8);
  e.record = (int8_t*)dalloc((size_t)B * CH * hw);
  float* target = (float*)dalloc((size_t)B * G * hw * 4);
  e.target = target;
  e.chan_stats = (double*)dalloc((size_t)B * G * 3 * 8);
  e.init_psnr = (double*)dalloc((size_t)B * 8);
  e.prev_psnr = (double*)dalloc((size_t)B * 8);
  e.max_psnr_diff = (double*)dalloc((size_t)B * 8);
  e.steps = (int64_t*)dalloc((size_t)B * 8);
  e.flip_count = (int64_t*)dalloc((size_t)B * 8);
  e.sustained = (int64_t*)dalloc((size_t)B * 8);
  e.error = (int32_t*)dalloc(8);
  EXPECT(e.mask && e.record && target && e.chan_stats && e.init_psnr && e.prev_psnr && e.max_psnr_diff &&
         e.steps && e.flip_count && e.sustained && e.error);

  /* synthetic inputs: ~50 % fill masks (env.py:120 threshold of a U[0,1) pre-model), U[0,1) targets */
  uint64_t* hmask = (uint64_t*)malloc(mwords * 8);
  float* htgt = (float*)malloc((size_t)B * G * hw * 4);
  for (size_t i = 0; i < mwords; ++i) hmask[i] = rng_next();
  for (size_t i = 0; i < (size_t)B * G * hw; ++i) htgt[i] = (float)((rng_next() >> 40) * (1.0 / 16777216.0));
  CHECK_HIP(hipMemcpy(e.mask, hmask, mwords * 8, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(target, htgt, (size_t)B * G * hw * 4, hipMemcpyHostToDevice));

  hipStream_t st;
  CHECK_HIP(hipStreamCreate(&st));
  CHECK_HBX(hbx_env_reset(plan, &e, B, NULL, 0, st));

  /* the step's results land in host-mapped memory (ABI v11): reward | psnr | acc | term | trunc | error */
  const size_t eoff = ((size_t)B * 19 + 7) / 8 * 8;   /* the error word, 8-byte aligned */
  const size_t row = eoff + 8;
  void *hrow = NULL, *drow = NULL;
  CHECK_HBX(hbx_host_alloc(row, &hrow, &drow));
  uint8_t* h = (uint8_t*)hrow;
  char* d = (char*)drow;
  e.error_host = (int32_t*)(d + eoff);

  hbx_env_params_t prm;
  memset(&prm, 0, sizeof(prm));
  prm.max_steps = 1000000000; prm.t_psnr = 1e9; prm.t_steps = 1; prm.t_psnr_diff = 1e9;   /* no episode ends */
  prm.reward_weight = 800.0; prm.accept_rule = HBX_ACCEPT_ENV; prm.reward_kind = HBX_REWARD_PSNR;

  int64_t* hact = (int64_t*)malloc((size_t)B * 8);
  int64_t* dact = (int64_t*)dalloc((size_t)B * 8);
  EXPECT(hact && dact);
  long n_acc = 0, n_rej = 0;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int s = 0; s < n_steps; ++s) {
    for (int b = 0; b < B; ++b) hact[b] = (int64_t)(rng_next() % ((uint64_t)CH * hw));
    CHECK_HIP(hipMemcpyAsync(dact, hact, (size_t)B * 8, hipMemcpyHostToDevice, st));
    CHECK_HBX(hbx_env_step(plan, &e, &prm, B, dact, (double*)d, (double*)(d + 8 * (size_t)B),
                           (uint8_t*)(d + 16 * (size_t)B), (uint8_t*)(d + 17 * (size_t)B),
                           (uint8_t*)(d + 18 * (size_t)B), NULL, st));
    CHECK_HIP(hipStreamSynchronize(st));
    const double* rew = (const double*)h;
    for (int b = 0; b < B; ++b) {
      EXPECT(isfinite(rew[b]));
      if (h[16 * (size_t)B + b]) ++n_acc; else ++n_rej;
    }
    EXPECT(*(const int32_t*)(h + eoff) == 0);
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  const double sec = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
  EXPECT(n_acc > 0 && n_rej > 0);

  /* prev_psnr == a fresh propagation of the current masks */
  double* stats = (double*)dalloc((size_t)B * G * 3 * 8);
  double* dps = (double*)dalloc((size_t)B * 8);
  EXPECT(stats && dps);
  CHECK_HBX(hbx_propagate(plan, e.mask, target, B, NULL, stats, dps, st));
  CHECK_HIP(hipStreamSynchronize(st));
  double* fresh = (double*)malloc((size_t)B * 8);
  double* prev = (double*)malloc((size_t)B * 8);
  CHECK_HIP(hipMemcpy(fresh, dps, (size_t)B * 8, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(prev, e.prev_psnr, (size_t)B * 8, hipMemcpyDeviceToHost));
  double worst = 0.0;
  for (int b = 0; b < B; ++b) worst = fmax(worst, fabs(fresh[b] - prev[b]));
  EXPECT(worst <= 1e-9);

  /* an out-of-range action: the step itself succeeds, the mirrored error word says why */
  hact[0] = (int64_t)CH * (int64_t)hw;
  CHECK_HIP(hipMemcpyAsync(dact, hact, (size_t)B * 8, hipMemcpyHostToDevice, st));
  CHECK_HBX(hbx_env_step(plan, &e, &prm, B, dact, (double*)d, (double*)(d + 8 * (size_t)B),
                         (uint8_t*)(d + 16 * (size_t)B), (uint8_t*)(d + 17 * (size_t)B),
                         (uint8_t*)(d + 18 * (size_t)B), NULL, st));
  CHECK_HIP(hipStreamSynchronize(st));
  EXPECT(*(const int32_t*)(h + eoff) != 0);
  EXPECT(h[16 * (size_t)B + 0] == 0);   /* the offending env's step is a no-op */

  /* HBX_OBS_SETTLE validates its buffers before the one-group no-op, so argument errors
   * are the same at every G (this plan has G = 1 and the env no recon / intensity / recon_pending) */
  EXPECT(hbx_env_obs_sync(plan, &e, B, NULL, 0, HBX_OBS_SETTLE, st) == HBX_ERR_INVALID);
  EXPECT(strstr(hbx_last_error(), "HBX_OBS_SETTLE") != NULL);

  /* (ABI v14) the pack kernel from plain C: 0/1 bytes -> words, and the binary check's word */
  {
    const size_t nv = 4 * 64 + 64;           /* 5 words: a ragged last group of the kernel */
    uint8_t hv[320];
    for (size_t i = 0; i < nv; ++i) hv[i] = (uint8_t)((i * 7 + i / 3) % 2);
    uint8_t* dv = (uint8_t*)dalloc(nv);
    uint64_t* dw = (uint64_t*)dalloc(5 * 8);
    EXPECT(dv && dw);
    CHECK_HIP(hipMemcpy(dv, hv, nv, hipMemcpyHostToDevice));
    int32_t* herr = (int32_t*)(h + eoff);
    *herr = 0;
    CHECK_HBX(hbx_pack_mask(dv, HBX_SRC_U8, (int64_t)nv, HBX_PACK_BINARY, 0.0, dw, (int32_t*)(d + eoff), st));
    CHECK_HIP(hipStreamSynchronize(st));
    uint64_t hw5[5];
    CHECK_HIP(hipMemcpy(hw5, dw, sizeof hw5, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < nv; ++i) EXPECT(((hw5[i / 64] >> (i % 64)) & 1u) == hv[i]);
    EXPECT(*herr == 0);
    hv[nv - 1] = 2;
    CHECK_HIP(hipMemcpy(dv, hv, nv, hipMemcpyHostToDevice));
    CHECK_HBX(hbx_pack_mask(dv, HBX_SRC_U8, (int64_t)nv, HBX_PACK_BINARY, 0.0, dw, (int32_t*)(d + eoff), st));
    CHECK_HIP(hipStreamSynchronize(st));
    EXPECT(*herr == 1);
  }

  printf("env_step_host: %d envs x %d steps of 256x256x8 in %.3f s (%.0f env-steps/s incl. one host "
         "round trip per step), %ld accepted / %ld rolled back, max |prev_psnr - fresh| = %.3g dB, OK\n",
         B, n_steps, sec, B * n_steps / sec, n_acc, n_rej, worst);
  CHECK_HBX(hbx_host_free(hrow));
  CHECK_HBX(hbx_plan_destroy(plan));
  CHECK_HIP(hipStreamDestroy(st));
  return 0;
}
