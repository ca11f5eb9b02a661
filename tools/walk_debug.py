"""Debug helper: run the device walk on the 64x64x(3x2) DBS fixture and print the
walk state after every chunk (pos, accepted, batches, done, halt, pending commits)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd"))
import numpy as np
import torch

import hbx
from hbx import dbs
from oracle import hbx_oracle as O

d = np.load(os.path.join(ROOT, "tests/golden/dbs_trace_64.npz"))
cfg = hbx.OpticsConfig(64, 64, 3, 2, O.WL_RGB)
plan = hbx.Plan(cfg, max_jobs=64)
mask = hbx.pack_bits(torch.from_numpy(d["pre_model"]).cuda() >= 0.5)
tgt = torch.from_numpy(d["target"]).cuda()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
t0 = time.time()


def prog(pos, acc, prev, secs):
    print(f"chunk: pos {pos} accepted {acc} prev {prev:.6f} t {secs:.3f}", flush=True)
    if time.time() - t0 > 30:
        print("giving up", flush=True)
        os._exit(3)


res = dbs.greedy(plan, mask, tgt, d["order"][:n], mode="psf", progress=prog)
want = np.nonzero(d["accepted"][:n])[0]
print("accepts", len(res.accepted_positions), "want", len(want), "equal",
      np.array_equal(np.array(res.accepted_positions), want), flush=True)
