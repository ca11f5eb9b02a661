"""HostObsMirror (obs_format="numpy", r06) bookkeeping on the CPU: the ping-pong host sets, the
catch-up of the deltas and reset rows a set missed, invalidation.  A stand-in env holds CPU
tensors and applies env.py:164-181's rules itself (the "device"); the mirror must hand out, after
every call, arrays equal to that state, and must leave the arrays it returned one call earlier
untouched (SB3 adds `_last_obs` to its rollout buffer after the next env.step)."""
from types import SimpleNamespace

import numpy as np
import torch

from hbx.env import OBS_KEYS, HostObsMirror
from hbx.plan import OpticsConfig


class _FakeVec:
    def __init__(self, B=5, N=64, G=1, P=2, seed=0):
        self.cfg = OpticsConfig(N, N, G, P, (515e-9,) * G)
        self.num_envs, self.device, self.obs_keys = B, torch.device("cpu"), OBS_KEYS
        self.rng = np.random.default_rng(seed)
        CH = G * P
        self.state = SimpleNamespace(
            record=torch.zeros((B, CH, N, N), dtype=torch.int8),
            state_bytes=torch.zeros((B, CH, N, N), dtype=torch.int8),
            pre_model=torch.zeros((B, CH, N, N), dtype=torch.float32),
            target=torch.zeros((B, G, N, N), dtype=torch.float32),
            recon=torch.zeros((B, G, N, N), dtype=torch.float32))
        for i in range(B):
            self.reset_env(i)

    def reset_env(self, i):
        st, c = self.state, self.cfg
        pre = torch.from_numpy(self.rng.random((c.channels, c.height, c.width), np.float32))
        st.pre_model[i] = pre
        st.state_bytes[i] = (pre >= 0.5).to(torch.int8)
        st.record[i] = 0
        st.target[i] = torch.from_numpy(self.rng.random((c.groups, c.height, c.width), np.float32))
        st.recon[i] = torch.from_numpy(self.rng.random((c.groups, c.height, c.width), np.float32))

    def step(self, actions, accepted):
        st, c = self.state, self.cfg
        for b, a in enumerate(actions.tolist()):
            ch, pix = divmod(a, c.height * c.width)
            r, col = divmod(pix, c.width)
            st.record[b, ch, r, col] += 1
            if accepted[b]:
                st.state_bytes[b, ch, r, col] ^= 1
        st.recon.copy_(torch.from_numpy(self.rng.random(tuple(st.recon.shape), np.float32)))

    def want(self):
        st = self.state
        return {"state_record": st.record.numpy()[:, None], "state": st.state_bytes.numpy()[:, None],
                "pre_model": st.pre_model.numpy()[:, None], "target_image": st.target.numpy()[:, None],
                "recon_image": st.recon.numpy()[:, None]}


def _check(obs, want, what):
    for k in OBS_KEYS:
        assert np.array_equal(obs[k], want[k]), (what, k)


def test_mirror_pingpong_steps_resets_and_invalidation():
    vec = _FakeVec()
    m = HostObsMirror(vec)
    m.begin()
    m.reset_rows(range(vec.num_envs))
    obs = m.obs()
    _check(obs, vec.want(), "reset")
    held, held_copy = obs, {k: v.copy() for k, v in obs.items()}
    npx = vec.cfg.channels * vec.cfg.height * vec.cfg.width
    for s in range(60):
        m.begin()
        acts = vec.rng.integers(0, npx, vec.num_envs)
        acc = vec.rng.random(vec.num_envs) < 0.5
        vec.step(acts, acc)
        m.queue_recon()
        m.step_delta(acts, acc.astype(np.uint8))
        if s % 7 == 3:                               # an auto-reset of a subset inside the step
            ids = sorted(set(vec.rng.integers(0, vec.num_envs, 2).tolist()))
            for i in ids:
                vec.reset_env(i)
            m.reset_rows(ids)
        obs = m.obs()
        _check(obs, vec.want(), s)
        for k in OBS_KEYS:                           # the previous call's arrays are untouched
            assert np.array_equal(held[k], held_copy[k]), (s, k)
        assert all(obs[k] is not held[k] for k in OBS_KEYS)
        held, held_copy = obs, {k: v.copy() for k, v in obs.items()}
        if s == 40:                                  # a bare device step between two steps: re-copy
            acts2 = vec.rng.integers(0, npx, vec.num_envs)
            vec.step(acts2, np.ones(vec.num_envs, bool))
            m.invalidate()
    # a reset-only call (env_method('reset')) between steps
    m.begin()
    vec.reset_env(1)
    m.reset_rows([1])
    m.sync_recon()
    _check(m.obs(), vec.want(), "env_method reset")


def test_mirror_int8_record_wraps_like_numpy():
    vec = _FakeVec(B=1, N=64, P=2)
    m = HostObsMirror(vec)
    m.begin()
    m.reset_rows([0])
    for _ in range(300):                             # the same pixel 300 times: int8 wraps
        m.begin()
        vec.step(np.array([5]), np.array([False]))
        m.queue_recon()
        m.step_delta(np.array([5]), np.array([0], np.uint8))
    assert m.obs()["state_record"][0, 0, 0, 0, 5] == np.int8(300 - 256)
    _check(m.obs(), vec.want(), "wrap")


def test_lazyobs_undo_log_restores_older_values():
    """LazyObs (obs_format="lazy", r06): an unread state / state_record key is kept by an undo log
    of the later steps' one-byte changes instead of a device copy; reading it after k more steps
    gives the values it was created with (int8 record wrap included); past UNDO_MAX steps the key
    is materialised."""
    from hbx.env import LazyObs
    rng = np.random.default_rng(4)
    B, CH, N = 3, 2, 8
    rec = torch.from_numpy(rng.integers(-128, 128, (B, CH, N, N)).astype(np.int8))
    rec[0, 1, 2, 3] = 127                                # wraps on the next +1
    st = torch.from_numpy((rng.random((B, CH, N, N)) < 0.5).astype(np.int8))
    want = {"state_record": rec.numpy()[:, None].copy(), "state": st.numpy()[:, None].copy()}
    lz = LazyObs({"state_record": rec.unsqueeze(1), "state": st.unsqueeze(1)})
    assert lz._track(("state", "state_record"))
    for step in range(LazyObs.UNDO_MAX):
        b = np.arange(B)
        c, r, col = rng.integers(0, CH, B), rng.integers(0, N, B), rng.integers(0, N, B)
        if step == 0:
            c[0], r[0], col[0] = 1, 2, 3
        acc = (rng.random(B) < 0.5).astype(np.int8)
        for i in range(B):                               # the "device" step
            rec[i, c[i], r[i], col[i]] += 1
            st[i, c[i], r[i], col[i]] ^= int(acc[i])
        lz._record((b, c, r, col, acc))
    assert np.array_equal(lz["state"], want["state"])
    assert np.array_equal(lz["state_record"], want["state_record"])
    lz2 = LazyObs({"state": st.unsqueeze(1)})
    lz2._track(("state",))
    snap = st.numpy()[:, None].copy()
    for _ in range(LazyObs.UNDO_MAX + 1):                # one past the bound: materialised then
        st[:, 0, 0, 0] ^= 1
        lz2._record((np.arange(B), np.zeros(B, np.int64), np.zeros(B, np.int64), np.zeros(B, np.int64),
                     np.ones(B, np.int8)))
    assert not lz2._tracked and np.array_equal(lz2["state"], snap)
