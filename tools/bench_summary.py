"""One-screen summary of a bench.py JSON line: python tools/bench_summary.py gpurun_out/<tag>/bench.json"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pk = 8000.0


def passes(p):
    return " ".join(f"{k} {v['avg_ms']:.4f}ms/{v['achieved_GBs'] / pk:.3f}" for k, v in p.items())


print(f"headline {d['value']:.0f} {d['unit']} ({d['ms_per_step']} ms/step) roofline {d['roofline']['kernel']} "
      f"frac {d['roofline']['frac']} traffic {d['roofline'].get('traffic')} ranks {d.get('ranks_seen')}")
print("  passes", passes(d["passes"]))
print("  step_alg_frac", d.get("step_alg_frac"), "psnr_delta", d.get("psnr_delta_vs_numpy"))
if "vecenv_step_obs" in d:
    o = d["vecenv_step_obs"]
    print(f"  vecenv_step_obs {o['value']:.0f} ({o['ms_per_step']} ms, overhead {o['obs_overhead_frac']})")
cb = d.get("cpu_baseline")
if cb:
    print(f"  cpu_baseline {cb['value']} {cb['unit']} x{cb['cores']} {cb['kind']}")
m = d.get("ppo_mono_256")
if m:
    print(f"mono256 {m['value']:.0f} ({m['ms_per_step']} ms) roofline {m.get('roofline', {}).get('frac')}")
    print("  passes", passes(m["passes"]))
    if "vecenv_step_obs" in m:
        print(f"  vecenv_step_obs overhead {m['vecenv_step_obs']['obs_overhead_frac']}")
for k in ("incremental_psf_mode", "dbs_greedy", "probe_sweep", "precision_sweep"):
    if k in d:
        s = json.dumps(d[k])
        print(f"{k}: {s[:300]}")
