/* Host-side checks of the C-ABI error paths (sanitizers on host
 * code only).  Built with clang -fsanitize=address against libhbx_asan.so
 * (the library with its host code ASan-instrumented) by
 * tests/test_abi.py::test_abi_error_paths_under_asan; needs no GPU: every
 * call below fails argument validation (or device selection) before any
 * kernel launch. */
#include <stdio.h>
#include <string.h>

#include "hbx.h"

static int fails = 0;
#define CHECK(cond)                                                      \
  do {                                                                   \
    if (!(cond)) {                                                       \
      printf("FAIL line %d: %s (last error: %s)\n", __LINE__, #cond,     \
             hbx_last_error());                                          \
      fails++;                                                           \
    }                                                                    \
  } while (0)

static hbx_optics_t rgb(int n) {
  hbx_optics_t o;
  memset(&o, 0, sizeof o);
  o.height = o.width = n;
  o.groups = 3;
  o.planes = 8;
  o.wavelength[0] = 638e-9;
  o.wavelength[1] = 515e-9;
  o.wavelength[2] = 450e-9;
  o.dx = o.dy = 7.56e-6;
  o.z = 2e-3;
  o.tf_kind = HBX_TF_ASM;
  o.field_kind = HBX_FIELD_AMPLITUDE;
  o.rel_scale = HBX_REL_LSQ;
  o.peak = 1.0;
  return o;
}

int main(void) {
  CHECK(hbx_abi_version() == HBX_ABI_VERSION);
  /* every entry point rejects a null plan */
  CHECK(hbx_propagate(NULL, NULL, NULL, 1, NULL, NULL, NULL, NULL) == HBX_ERR_INVALID);
  CHECK(strstr(hbx_last_error(), "null plan") != NULL);
  CHECK(hbx_simulate(NULL, NULL, 1, NULL, NULL, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_psnr(NULL, NULL, 0, NULL, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_env_reset(NULL, NULL, 0, NULL, 0, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_env_step(NULL, NULL, NULL, 0, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_env_step_psf(NULL, NULL, NULL, 0, NULL, NULL, NULL, NULL, NULL, NULL, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_field_refresh(NULL, NULL, 0, NULL, 0, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_env_obs_sync(NULL, NULL, 0, NULL, 0, HBX_OBS_STATE, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_step(NULL, NULL, NULL, 0, NULL, NULL, NULL, NULL, NULL, 0, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_eval_flips(NULL, NULL, NULL, NULL, NULL, 1, NULL, NULL, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_eval_flips_psf(NULL, NULL, NULL, NULL, NULL, NULL, NULL, 1, NULL, NULL, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_commit_flip(NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, 1, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_commit_flip_psf(NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, 1, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_flip_map(NULL, NULL, NULL, NULL, NULL, NULL) == HBX_ERR_INVALID);
  {
    void *h = (void*)1, *d = (void*)1;
    CHECK(hbx_host_alloc(0, &h, &d) == HBX_ERR_INVALID);   /* no HIP call before the checks */
    CHECK(h == (void*)1 && d == (void*)1);
    CHECK(hbx_host_alloc(64, NULL, &d) == HBX_ERR_INVALID);
    CHECK(hbx_host_free(NULL) == HBX_OK);
  }
  CHECK(hbx_planes_fill(NULL, NULL, NULL, NULL, NULL, 1, NULL, NULL, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_eval_flips_planes(NULL, NULL, NULL, NULL, NULL, NULL, 1, NULL, 1, NULL, NULL, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_commit_flip_planes(NULL, NULL, NULL, NULL, NULL, 1, NULL, NULL, NULL, NULL, 1, NULL) ==
        HBX_ERR_INVALID);
  CHECK(hbx_env_obs_sync(NULL, NULL, 0, NULL, 0, HBX_OBS_RECON | HBX_OBS_RESOLVE, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_env_obs_sync(NULL, NULL, 0, NULL, 0, HBX_OBS_SETTLE, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_dbs_walk_planes(NULL, NULL, NULL, NULL, NULL, NULL, 1, NULL, 0, NULL, NULL, NULL, 0, 1, 1, NULL) ==
        HBX_ERR_INVALID);
  CHECK(hbx_dbs_walk_planes_fill(NULL, NULL, NULL, NULL, NULL, NULL, 1, NULL, 0, NULL, NULL, NULL, 0, 1, 1, NULL, 0,
                                 0, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_dbs_walk_psf(NULL, NULL, NULL, NULL, NULL, NULL, NULL, 0, NULL, NULL, NULL, 0, 1, 1, NULL) ==
        HBX_ERR_INVALID);
  CHECK(hbx_plan_pipeline(NULL) == HBX_ERR_INVALID);
  CHECK(hbx_plan_set_precision(NULL, HBX_PRECISION_BF16_STORE) == HBX_ERR_INVALID);
  CHECK(hbx_plan_precision(NULL) == HBX_ERR_INVALID);
  CHECK(hbx_plan_set_timing(NULL, 4) == HBX_ERR_INVALID);
  CHECK(hbx_plan_set_timing_sampled(NULL, 4, 2) == HBX_ERR_INVALID);
  CHECK(hbx_plan_read_timing(NULL, NULL, NULL, NULL) == HBX_ERR_INVALID);
  CHECK(hbx_plan_workspace_bytes(NULL) == 0);
  CHECK(hbx_plan_destroy(NULL) == HBX_OK);

  /* (ABI v14) pack / relativeLoss: argument validation before any launch */
  {
    static double buf[8];   /* 32-byte aligned enough for every kind; never dereferenced */
    void* src = (void*)(((unsigned long)buf + 31) & ~31ul);
    uint64_t* bits = (uint64_t*)src;
    CHECK(hbx_pack_mask(src, HBX_SRC_F32, 0, HBX_PACK_BINARY, 0.0, bits, NULL, NULL) == HBX_OK); /* empty */
    CHECK(hbx_pack_mask(src, HBX_SRC_F32, 100, HBX_PACK_BINARY, 0.0, bits, NULL, NULL) == HBX_ERR_INVALID);
    CHECK(strstr(hbx_last_error(), "multiple of 64") != NULL);
    CHECK(hbx_pack_mask(NULL, HBX_SRC_F32, 64, HBX_PACK_BINARY, 0.0, bits, NULL, NULL) == HBX_ERR_INVALID);
    CHECK(hbx_pack_mask(src, HBX_SRC_F32, 64, HBX_PACK_BINARY, 0.0, NULL, NULL, NULL) == HBX_ERR_INVALID);
    CHECK(hbx_pack_mask(src, 7, 64, HBX_PACK_BINARY, 0.0, bits, NULL, NULL) == HBX_ERR_INVALID);
    CHECK(hbx_pack_mask(src, HBX_SRC_F32, 64, 5, 0.0, bits, NULL, NULL) == HBX_ERR_INVALID);
    CHECK(hbx_pack_mask((char*)src + 4, HBX_SRC_F32, 64, HBX_PACK_BINARY, 0.0, bits, NULL, NULL) ==
          HBX_ERR_INVALID);
    CHECK(strstr(hbx_last_error(), "aligned") != NULL);
    CHECK(hbx_pack_mask((char*)src + 16, HBX_SRC_F64, 64, HBX_PACK_THRESHOLD, 0.5, bits, NULL, NULL) ==
          HBX_ERR_INVALID);
    CHECK(hbx_pack_mask((char*)src + 2, HBX_SRC_U8, 64, HBX_PACK_BINARY, 0.0, bits, NULL, NULL) ==
          HBX_ERR_INVALID);
    CHECK(hbx_rel_stats(src, src, HBX_SRC_F32, 0, HBX_REL_LSQ, 1.0, buf, buf, NULL) == HBX_ERR_INVALID);
    CHECK(hbx_rel_stats(NULL, src, HBX_SRC_F32, 64, HBX_REL_LSQ, 1.0, buf, buf, NULL) == HBX_ERR_INVALID);
    CHECK(hbx_rel_stats(src, src, HBX_SRC_F32, 64, HBX_REL_LSQ, 1.0, NULL, buf, NULL) == HBX_ERR_INVALID);
    CHECK(hbx_rel_stats(src, src, HBX_SRC_U8, 64, HBX_REL_LSQ, 1.0, buf, buf, NULL) == HBX_ERR_INVALID);
    CHECK(hbx_rel_stats(src, src, HBX_SRC_F32, 64, 3, 1.0, buf, buf, NULL) == HBX_ERR_INVALID);
  }

  /* plan validation happens before any device call */
  hbx_plan_t p = NULL;
  hbx_optics_t o = rgb(1024);
  CHECK(hbx_plan_create(NULL, &o, 3, 0) == HBX_ERR_INVALID);
  CHECK(hbx_plan_create(&p, NULL, 3, 0) == HBX_ERR_INVALID && p == NULL);
  o = rgb(100);
  CHECK(hbx_plan_create(&p, &o, 3, 0) == HBX_ERR_UNSUPPORTED && p == NULL);
  o = rgb(1024);
  o.width = 512;
  CHECK(hbx_plan_create(&p, &o, 3, 0) == HBX_ERR_UNSUPPORTED);
  o = rgb(1024);
  o.groups = 0;
  CHECK(hbx_plan_create(&p, &o, 3, 0) == HBX_ERR_INVALID);
  o.groups = HBX_MAX_GROUPS + 1;
  CHECK(hbx_plan_create(&p, &o, 8, 0) == HBX_ERR_INVALID);
  o = rgb(1024);
  o.planes = 7;
  CHECK(hbx_plan_create(&p, &o, 3, 0) == HBX_ERR_INVALID);
  o = rgb(1024);
  CHECK(hbx_plan_create(&p, &o, 2, 0) == HBX_ERR_INVALID);   /* max_jobs < groups */
  o.tf_kind = 7;
  CHECK(hbx_plan_create(&p, &o, 3, 0) == HBX_ERR_INVALID);
  o = rgb(1024);
  o.field_kind = -1;
  CHECK(hbx_plan_create(&p, &o, 3, 0) == HBX_ERR_INVALID);
  o = rgb(1024);
  o.rel_scale = 2;
  CHECK(hbx_plan_create(&p, &o, 3, 0) == HBX_ERR_INVALID);
  o = rgb(1024);
  o.wavelength[1] = 0.0;
  CHECK(hbx_plan_create(&p, &o, 3, 0) == HBX_ERR_INVALID);
  o = rgb(1024);
  o.dx = -1.0;
  CHECK(hbx_plan_create(&p, &o, 3, 0) == HBX_ERR_INVALID);
  CHECK(p == NULL);
  /* a valid plan on a device that does not exist: an HIP error, never a crash */
  o = rgb(64);
  o.planes = 2;
  CHECK(hbx_plan_create(&p, &o, 3, 4096) == HBX_ERR_HIP && p == NULL);
  CHECK(strlen(hbx_last_error()) > 0);

  printf(fails ? "FAILED %d\n" : "OK\n", fails);
  return fails != 0;
}
