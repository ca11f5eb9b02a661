import sys, time, numpy as np, torch
sys.path.insert(0, "binary-hologram-reinforcement-learning_amd"); sys.path.insert(0, ".")
import hbx
from oracle import hbx_oracle as O
from tests.test_gpu_parity import dev_cfg, to_dev_bits
for n, mk in ((256, lambda: O.mono_config(256)), (64, lambda: O.rgb_config(64, planes=2))):
    ocfg = mk(); pre, tgt = O.synthetic_inputs(ocfg, 41)
    env = O.OracleEnv(ocfg); base = env.reset(pre, tgt)
    plan = hbx.Plan(dev_cfg(ocfg), max_jobs=64)
    bits = to_dev_bits(O.pack_mask((pre >= 0.5).astype(np.uint8)))
    dmap, b = plan.flip_map(bits, torch.from_numpy(tgt).cuda())
    flat = dmap.reshape(-1).cpu().numpy().astype(np.float64)
    s = np.random.default_rng(1).integers(0, flat.size, 64)
    want = np.array([env.evaluate_flip(int(a))[0] - base for a in s])
    print(n, "max|err|", np.max(np.abs(flat[s] - want)), "max|delta|", np.max(np.abs(want)), "rel", np.max(np.abs(flat[s]-want))/np.max(np.abs(want)))
ocfg = O.rgb_config(1024); pre, tgt = O.synthetic_inputs(ocfg, 5)
plan = hbx.Plan(dev_cfg(ocfg), max_jobs=8)
bits = to_dev_bits(O.pack_mask((pre >= 0.5).astype(np.uint8))); t = torch.from_numpy(tgt).cuda()
dmap, b = plan.flip_map(bits, t); torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5): plan.flip_map(bits, t, out=dmap)
torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 5
print(f"1024x24 flip map: {dt*1e3:.2f} ms for {24*1024*1024} flips -> {24*1024*1024/dt/1e9:.2f} Gflips/s")
env = O.OracleEnv(ocfg); base = env.reset(pre, tgt)
s = np.array([0, 5*1024*1024 + 77, 13*1024*1024+512*1024+3, 23*1024*1024+999])
want = np.array([env.evaluate_flip(int(a))[0] - base for a in s])
got = dmap.reshape(-1)[torch.from_numpy(s).cuda()].double().cpu().numpy()
print("1024 vs oracle:", np.abs(got - want), want)
