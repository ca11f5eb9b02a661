"""RCCL (torch.distributed "nccl") on the one MI355X of a test box: a world of
one built with hbx.dist.init(force=True), device-bound, running every
collective the multi-GPU path uses -- the per-step metric gather to rank 0
(StepMetricGather / gather_to_rank0), the max-over-ranks timer, describe_world,
the sharded probe sweep's histogram all-reduce and greedy_dataset's summary
gather -- each compared with the world-less result (the caller is
train-PPO.py:296-322 with 128 envs per GPU, BASELINE configs[3]).  So the
first 8-GPU run is not the first time the nccl branches execute."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import hbx_oracle as O  # noqa: E402


def _inputs():
    import hbx
    ocfg = O.OpticsConfig(64, 64, 3, 2, O.WL_RGB)
    cfg = hbx.OpticsConfig(ocfg.height, ocfg.width, ocfg.groups, ocfg.planes, tuple(ocfg.wavelengths),
                           ocfg.dx, ocfg.dy, ocfg.z, ocfg.tf_kind, ocfg.field_kind, ocfg.rel_scale, ocfg.peak)
    return ocfg, cfg


def _run_all(tmp, tag):
    """Every collective of the multi-GPU path, on device tensors; returns comparable values."""
    import hbx
    from hbx import dbs
    from hbx import dist as hd
    from hbx.env import HologramVecEnv
    dev = torch.device("cuda", 0)
    ocfg, cfg = _inputs()
    out = {}
    # per-step metric gather of a real 4-env VecEnv, 5 steps gathered every 3; the step
    # kernel writes its outputs straight into the gather's byte rows (slot())
    ins = [O.synthetic_inputs(ocfg, 40 + i) for i in range(4)]
    vec = HologramVecEnv(cfg, 4, lambda i: ins[i][1], pre_model_source=lambda i: ins[i][0],
                         obs_keys=(), auto_reset=False)
    vec.reset()
    acts = torch.from_numpy(np.random.default_rng(5).integers(0, ocfg.channels * 64 * 64, (5, 4))).to(dev)
    mg = hd.StepMetricGather(4, every=3, device=dev)
    single = []
    for k in range(5):
        slot = mg.slot()
        r, ps, acc, term, trunc = vec.step_device(acts[k], out=slot)
        assert all(a.data_ptr() == b.data_ptr() for a, b in zip((r, ps, acc, term, trunc), slot))
        single.append(hd.gather_to_rank0(hd.pack_step_metrics(r, ps, acc, term, trunc)).cpu().numpy())
        mg.add(r, ps, acc, term, trunc)
    mg.flush()
    vec.close()
    out["steps"] = np.stack(single)
    out["blocks"] = [b.cpu().numpy() for b in mg.gathered]
    out["max"] = hd.max_over_ranks(1.25, dev)
    out["world"] = hd.describe_world(dev)
    # sharded probe sweep: one 31-double all-reduce
    pre, tgt = O.synthetic_inputs(ocfg, 7)
    flips = np.random.default_rng(8).integers(0, ocfg.channels * 64 * 64, 300)
    plan = hbx.Plan(cfg, max_jobs=256)
    mask = hbx.pack_bits(torch.from_numpy(pre).cuda() >= 0.5)
    pr = dbs.probe_sharded(plan, mask, torch.from_numpy(tgt).cuda(), flips, pre_model=pre)
    plan.close()
    out["probe"] = (pr.shard, pr.attempted_bins.tolist(), pr.improved_bins.tolist(), pr.delta_bins.tolist(),
                    pr.improved_total, pr.psnr.tolist())
    # greedy_dataset: per-image summaries gathered to rank 0
    dins = [O.synthetic_inputs(ocfg, 80 + i) for i in range(2)]
    orders = [np.random.default_rng(90 + i).permutation(ocfg.channels * 64 * 64)[:600] for i in range(2)]

    def load(i):
        return hbx.pack_bits(torch.from_numpy(dins[i][0]).cuda() >= 0.5), torch.from_numpy(dins[i][1]).cuda()

    rows = dbs.greedy_dataset(2, load, lambda i: orders[i], lambda: hbx.Plan(cfg, max_jobs=cfg.groups),
                              per_gpu=2, save_dir=str(tmp / tag))
    out["dataset"] = [{k: v for k, v in r.items() if k != "seconds"} for r in rows]
    return out


def test_rccl_world1_collectives_equal_worldless(tmp_path):
    import hbx
    from hbx import dist as hd
    hbx.load_library()
    assert not hd.active(), "another test left a process group behind"
    want = _run_all(tmp_path, "plain")
    assert want["world"] == [[0, 1, 0, "none"]]
    hd.init(backend="nccl", force=True)
    try:
        assert hd.active() and hd.backend() == "nccl"
        got = _run_all(tmp_path, "rccl")
        assert got["world"] == [[0, 1, 0, "nccl"]]
        assert np.array_equal(got["steps"], want["steps"])
        assert len(got["blocks"]) == len(want["blocks"]) == 2
        for a, b in zip(got["blocks"], want["blocks"]):
            assert np.array_equal(a, b)
        assert np.array_equal(np.concatenate(got["blocks"]), want["steps"])
        assert got["max"] == want["max"] == 1.25
        assert got["probe"] == want["probe"]
        assert got["dataset"] == want["dataset"] and [r["image"] for r in got["dataset"]] == [0, 1]
        hd.barrier()
    finally:
        hd.shutdown()
    assert not hd.active()
