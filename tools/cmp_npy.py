"""Where two [env][plane][y][x](complex) arrays differ: python tools/cmp_npy.py a.npy b.npy"""
import collections
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
d = np.abs(a - b)
if d.ndim == 5:
    d = d.sum(-1)
print(a.shape, a.dtype, "max", d.max())
bad = np.argwhere(d > 1e-5)
print(len(bad))
for axis, name in enumerate(("envs", "planes", "rows", "cols")):
    if len(bad):
        print(name, collections.Counter(bad[:, axis]).most_common(12))
