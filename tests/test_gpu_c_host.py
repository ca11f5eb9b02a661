"""The C-ABI driven from plain C (tests/c/env_step_host.c, built by __graft_entry__.build()):
plan -> reset -> 200 steps of 16 envs at 256x256x8 with the results written by the step kernels
into hbx_host_alloc'd memory, prev_psnr against a fresh hbx_propagate of the final masks, and an
out-of-range action reported through the mirrored error word -- the path a cgo / JNI / N-API
binding of env.step would take."""
import os
import subprocess

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

EXE = os.path.join(ROOT, "binary-hologram-reinforcement-learning_amd", "hbx", "env_step_host")


def test_env_step_from_c():
    assert os.path.exists(EXE), "build first: python -c 'import __graft_entry__ as g; g.build()'"
    out = subprocess.run([EXE, "16", "200"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr + out.stdout
    assert out.stdout.strip().endswith("OK"), out.stdout
