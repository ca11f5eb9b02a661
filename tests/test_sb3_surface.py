"""HologramVecEnv as the VecEnv SB3 consumes: train-PPO.py:296-322
passes the env to PPO("MultiInputPolicy", ...), whose rollout collection calls
step_async / step_wait and assigns every observation key into a DictRolloutBuffer
(`buffer[key][pos] = np.array(obs[key])`); optimize_hyperparameter.py:317-318 wraps it
with make_vec_env / VecNormalize, which read num_envs / observation_space and call
get_attr / set_attr / env_method / seed.  stable-baselines3 is not installed in this
image, so the buffer assignment is replayed here, and the subclassing branch is run
against a stand-in `stable_baselines3.common.vec_env.VecEnv` module."""
import importlib
import sys
import types

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import hbx_oracle as O  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm GPU")
    import hbx
    hbx.load_library()
    yield


def _make(obs_format, B=3, max_steps=4, **kw):
    import hbx
    from hbx.env import HologramVecEnv
    ocfg = O.OpticsConfig(64, 64, 3, 2, O.WL_RGB)
    ins = [O.synthetic_inputs(ocfg, 70 + i) for i in range(B)]
    cfg = hbx.OpticsConfig(64, 64, 3, 2, O.WL_RGB)
    return HologramVecEnv(cfg, B, lambda i: ins[i][1], pre_model_source=lambda i: ins[i][0],
                          max_steps=max_steps, obs_format=obs_format, **kw), ins


def test_rollout_buffer_assignment_numpy_obs():
    env, _ = _make("numpy")
    n_steps, B = 16, env.num_envs
    space = env.observation_space
    buf = {k: np.zeros((n_steps, B) + tuple(space[k].shape), dtype=space[k].dtype) for k in space.keys()}
    rewards = np.zeros((n_steps, B), np.float32)
    dones_seen = 0
    obs = env.reset()
    space.seed(0)
    env.action_space.seed(0)
    for pos in range(n_steps):
        for k in buf:                                   # DictRolloutBuffer.add
            buf[k][pos] = np.array(obs[k])
        actions = np.array([env.action_space.sample() for _ in range(B)])
        env.step_async(actions)
        obs, rew, dones, infos = env.step_wait()
        assert isinstance(rew, np.ndarray) and rew.dtype == np.float32 and rew.shape == (B,)
        assert dones.dtype == bool and len(infos) == B
        rewards[pos] = rew
        for i in np.nonzero(dones)[0]:
            dones_seen += 1
            term = infos[i]["terminal_observation"]
            assert set(term) == set(space.keys())
            assert all(isinstance(v, np.ndarray) and v.shape == space[k].shape for k, v in term.items())
            assert "TimeLimit.truncated" in infos[i]
    assert dones_seen >= B                              # max_steps=4 over 16 steps: every env finished
    assert buf["state"].dtype == np.int8 and buf["recon_image"].shape == (n_steps, B, 1, 3, 64, 64)
    assert np.all((buf["state"] == 0) | (buf["state"] == 1))
    env.close()


def test_vecenv_method_surface():
    env, ins = _make("lazy")
    obs = env.reset()
    from hbx.env import LazyObs
    assert isinstance(obs, LazyObs)
    assert isinstance(obs.device("state"), torch.Tensor)          # no copy needed
    st = obs["state"]
    assert isinstance(st, np.ndarray) and st.shape == (3, 1, 6, 64, 64)
    assert np.array_equal(st[1, 0], (ins[1][0] >= 0.5).astype(np.int8))
    init = env.get_attr("initial_psnr")
    assert len(init) == 3 and all(isinstance(v, float) for v in init)
    assert env.get_attr("initial_psnr", indices=[2]) == init[2:]
    assert env.get_attr("render_mode") == [None, None, None]
    env.set_attr("T_PSNR", 25.0)
    assert env.get_attr("T_PSNR") == [25.0] * 3
    with pytest.raises(ValueError):
        env.set_attr("max_steps", 9, indices=[0])
    with pytest.raises(AttributeError):
        env.set_attr("steps", 0)
    env.step(np.array([5, 6, 7]))
    assert env.get_attr("steps") == [1, 1, 1]
    out = env.env_method("reset", indices=[1])
    assert len(out) == 1 and out[0]["state"].shape == (1, 6, 64, 64)
    assert env.get_attr("steps") == [1, 0, 1]
    assert env.env_is_wrapped(object) == [False] * 3
    assert env.seed(3) == [3, 4, 5]
    assert env.get_images() == [None] * 3 and env.render() is None
    env.close()


def test_subclasses_sb3_vecenv_when_importable(monkeypatch):
    """With stable_baselines3 importable, HologramVecEnv is a VecEnv subclass and
    runs VecEnv.__init__ (stand-in module: the real one is not installed here)."""
    calls = {}

    class VecEnv:                                        # the attributes SB3 2.x's __init__ sets
        def __init__(self, num_envs, observation_space, action_space):
            calls["init"] = (num_envs, observation_space, action_space)
            self.num_envs = num_envs
            self.observation_space = observation_space
            self.action_space = action_space
            self.reset_infos = [{} for _ in range(num_envs)]
            self._seeds = [None for _ in range(num_envs)]
            self._options = [{} for _ in range(num_envs)]
            self.render_mode = None

    mods = {name: types.ModuleType(name) for name in
            ("stable_baselines3", "stable_baselines3.common", "stable_baselines3.common.vec_env")}
    mods["stable_baselines3.common.vec_env"].VecEnv = VecEnv
    for name, m in mods.items():
        monkeypatch.setitem(sys.modules, name, m)
    import hbx.env as henv
    try:
        henv = importlib.reload(henv)
        assert henv.HAVE_SB3 and issubclass(henv.HologramVecEnv, VecEnv)
        env, _ = _make("numpy")
        assert isinstance(env, VecEnv) and calls["init"][0] == 3
        assert calls["init"][1] is env.observation_space
        obs = env.reset()
        assert obs["state"].shape == (3, 1, 6, 64, 64)
        env.close()
    finally:
        monkeypatch.undo()
        importlib.reload(henv)
