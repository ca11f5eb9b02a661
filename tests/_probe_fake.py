"""Test infrastructure: a CPU stand-in for hbx.Plan whose propagate /
eval_flips are answered by the float64 oracle, so host drivers that only
need those two calls (hbx.dbs.probe / probe_sharded) run over gloo without a
GPU (tests/test_dist.py)."""
import numpy as np
import torch

from oracle import hbx_oracle as O


class OraclePlan:
    def __init__(self, ocfg):
        self.ocfg = ocfg
        self.cfg = ocfg
        self.device = torch.device("cpu")

    def _env(self, mask, target):
        m = O.unpack_mask(mask.numpy().view("<u8"), self.ocfg.width).astype(np.float32)
        env = O.OracleEnv(self.ocfg)
        env.reset(m, target.numpy())
        return env

    def propagate(self, mask, target, want_intensity=False, stream=None):
        env = self._env(mask[0], target[0])
        return None, torch.from_numpy(env.stats.copy())[None], torch.tensor([env.initial_psnr])

    def eval_flips(self, mask, target, base_stats, flips, out, gst, stream=None):
        env = self._env(mask, target)
        for i, a in enumerate(flips.tolist()):
            ps, g, _, st = env.evaluate_flip(int(a))
            out[i] = ps
            gst[i] = torch.from_numpy(st[g])
        return out, gst


def probe_inputs():
    ocfg = O.rgb_config(64, planes=2)
    pre, tgt = O.synthetic_inputs(ocfg, 5)
    mask = torch.from_numpy(O.pack_mask((pre >= 0.5).astype(np.uint8)).view(np.int64))
    flips = np.random.default_rng(9).integers(0, ocfg.channels * 64 * 64, 90)
    return ocfg, pre, torch.from_numpy(tgt), mask, flips
