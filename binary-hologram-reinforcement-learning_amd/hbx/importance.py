"""env_group.py importance rewards.

At reset the reference flips 10 000 random pixels one at a time against the
fresh state, records each PSNR change (env_group.py:90-120), maps the change
ranks through a degree-5 polynomial (env_group.py:121-143) and sets the
dynamic success threshold T_PSNR_DIFF = (sum of the positive changes) / 4
(env_group.py:198).  Every step's reward is then the importance value of the
sampled change nearest to the step's change (env_group.py:254-255), computed
on the device (hbx_env_step, HBX_REWARD_IMPORTANCE).

Here the 10 000 changes are read out of the all-flip map (hbx_flip_map) of the
reset state instead of 10 000 propagations.  Ties in the ranking (the same
pixel drawn twice) are ordered by draw index (stable sort); the reference's
np.argsort default leaves that order unspecified.
"""
from __future__ import annotations

import numpy as np

STEP_POLY = np.array([10000, 9000, 8000, 5000, 2500, 1])     # env_group.py:121
REWARDS_POLY = np.array([-0.5, -0.48, -0.45, -0.35, 0, 1])   # env_group.py:122


def rank_polynomial() -> np.poly1d:
    """The degree-5 interpolant through (STEP_POLY, REWARDS_POLY) (env_group.py:123-125)."""
    return np.poly1d(np.polyfit(STEP_POLY, REWARDS_POLY, len(STEP_POLY) - 1))


def importance_values(changes: np.ndarray):
    """(importance_ranks[n], T_PSNR_DIFF) for the sampled PSNR changes:
    rank r of the ascending sort maps to x = 10000 - 9999 r / (n - 1)
    (env_group.py:132-141), importance = poly(x)."""
    c = np.asarray(changes, np.float64)
    n = c.shape[0]
    poly = rank_polynomial()
    order = np.argsort(c, kind="stable")
    ranks = np.empty(n, np.float64)
    x = 10000 - (10000 - 1) * (np.arange(n) / max(n - 1, 1))
    ranks[order] = poly(x)
    return ranks, float(np.sum(c[c > 0])) / 4.0
