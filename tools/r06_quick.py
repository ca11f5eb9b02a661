"""r06 quick A/B on one GPU: the torchOptics shim loop vs the torch.fft reference step
(bench.shim_dbs_loop / torch_reference_step), the reset cost before / after hbx_pack_mask, and
the numpy-observation step (bench.vecenv_step_obs_numpy).  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    from hbx.plan import mono_config, rgb_config
    out = {}
    what = sys.argv[1:] or ["shim", "reset", "numpy"]
    if "shim" in what:
        for rep in range(2):
            out[f"torch_reference_step_{rep}"] = bench.torch_reference_step(256, 300, 20)["value"]
            out[f"shim_dbs_loop_{rep}"] = bench.shim_dbs_loop(256, 300, 20)["value"]
        print(json.dumps(out), flush=True)
    if "reset" in what:
        out["reset_1024x24"] = bench.reset_cost(rgb_config(1024))
        print(json.dumps(out), flush=True)
    if "lazy" in what:
        mono = mono_config(256)
        g = torch.Generator(device="cuda").manual_seed(3)
        pres = [torch.rand((8, 256, 256), generator=g, device="cuda") for _ in range(128)]
        tgts = [torch.rand((1, 256, 256), generator=g, device="cuda") for _ in range(128)]
        for fmt in ("torch", "lazy"):
            r = bench.vecenv_step_obs(mono, 128, 240, 5, lambda i: tgts[i], lambda i: pres[i], 0.33, 12,
                                      obs_format=fmt)
            out[f"vecenv_step_obs_{fmt}"] = {k: r[k] for k in ("ms_per_step", "pure_device_step_ms",
                                                              "overhead_vs_pure_device_step")}
        print(json.dumps(out), flush=True)
    if "numpy" in what:
        mono = mono_config(256)
        g = torch.Generator(device="cuda").manual_seed(3)
        pres = [torch.rand((8, 256, 256), generator=g, device="cuda") for _ in range(128)]
        tgts = [torch.rand((1, 256, 256), generator=g, device="cuda") for _ in range(128)]
        out["vecenv_step_obs_numpy"] = bench.vecenv_step_obs_numpy(mono, 128, 30, 5, lambda i: tgts[i],
                                                                   lambda i: pres[i], 13)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
