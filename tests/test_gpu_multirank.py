"""Multi-rank product path on one MI355X: two ranks share cuda:0 over gloo (RCCL needs one GPU per
rank; the driver's 8-GPU run covers RCCL itself). Each rank builds its agents from DIFFERENT synthetic
weights; after ShardedEvaluationPipeline's broadcast every rank must compute with rank 0's weights,
including the encoder's host layer table (split-f16 exponents), so the gathered outputs equal
per-shard EvaluationPipeline runs with rank 0's weights (each shard is a reference call
on its sub-batch)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _cfg(seed):
    from genpose2_amd.config import GenPoseConfig
    return GenPoseConfig(device=DEV, sampling_steps=20, eval_repeat_num=20, noise_seed=4, seed=seed)


def _batch(total):
    from genpose2_amd import synthetic
    pts, center = synthetic.make_batch(12, total, 1024)
    return {"pts": torch.from_numpy(pts).to(DEV), "pts_center": torch.from_numpy(center).to(DEV)}


def _worker(rank, world, port, out_dir, total, ckpt):
    import torch.distributed as dist
    from genpose2_amd.runner import ShardedEvaluationPipeline
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        pipe = ShardedEvaluationPipeline(_cfg(seed=0 if rank == 0 else 99), with_scale=True)
        if ckpt:   # rank 0 alone reads a checkpoint (seed 7 weights), then broadcasts it
            pipe.load_ckpt(score=ckpt if rank == 0 else "/nonexistent/on/this/rank.pth")
        got = pipe.run(_batch(total))
        if rank == 0:
            for k in ("pred_pose", "pts_feat", "energy", "aggregated", "length"):
                np.save(os.path.join(out_dir, f"{k}.npy"), getattr(got, k).cpu().numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("with_ckpt", [False, True])
def test_two_ranks_mismatched_seeds_equal_rank0_weights(tmp_path, with_ckpt):
    import torch.multiprocessing as mp
    from conftest import write_reference_checkpoint
    from genpose2_amd import shard
    from genpose2_amd.runner import EvaluationPipeline
    total, world = 5, 2
    ckpt = write_reference_checkpoint(str(tmp_path / "score.pth"), "score", seed=7) if with_ckpt else ""
    port = 29300 + (os.getpid() + int(with_ckpt)) % 600
    mp.spawn(_worker, args=(world, port, str(tmp_path), total, ckpt), nprocs=world, join=True)
    batch = _batch(total)
    parts = []
    for r in range(world):
        lo, hi = shard.shard_range(total, world, r)
        ref = EvaluationPipeline(_cfg(seed=0), with_scale=True)
        if with_ckpt:
            ref.score_agent.load_ckpt(model_dir=ckpt, model_path=True, load_model_only=True)
        parts.append(ref.run({k: v[lo:hi] for k, v in batch.items()}))
    # every output's agreement first (per object), so a mismatch names what diverged, then the exact bar
    report = {}
    for k in ("pred_pose", "pts_feat", "energy", "aggregated", "length"):
        want = torch.cat([getattr(p, k) for p in parts]).cpu().numpy()
        got = np.load(tmp_path / f"{k}.npy")
        report[k] = [int(i) for i in range(want.shape[0]) if not np.array_equal(got[i], want[i])]
    print("objects differing from the per-shard reference:", report)
    for k in ("pred_pose", "pts_feat", "energy", "aggregated", "length"):
        want = torch.cat([getattr(p, k) for p in parts]).cpu().numpy()
        np.testing.assert_array_equal(np.load(tmp_path / f"{k}.npy"), want, err_msg=k)


def _cfg_global(k):
    from genpose2_amd.config import GenPoseConfig
    return GenPoseConfig(device=DEV, sampling_steps=20, eval_repeat_num=k, noise_seed=4, seed=0)


def _global_worker(rank, world, port, out_dir, total, k):
    import torch.distributed as dist
    from genpose2_amd.runner import ShardedEvaluationPipeline
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        pipe = ShardedEvaluationPipeline(_cfg_global(k), global_batch=True)
        got = pipe.run(_batch(total))
        # negative control: the default semantics (each shard a reference call on its sub-batch)
        own = ShardedEvaluationPipeline(_cfg_global(k), with_energy=False).run(_batch(total))
        if rank == 0:
            for key in ("pred_pose", "energy", "aggregated"):
                np.save(os.path.join(out_dir, f"{key}.npy"), getattr(got, key).cpu().numpy())
            np.save(os.path.join(out_dir, "per_shard_pred_pose.npy"), own.pred_pose.cpu().numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total,k", [(6, 16), (5, 16), (132, 64)])
def test_global_batch_two_ranks_equal_one_call(tmp_path, total, k):
    """Global-batch PC sampling (ShardedEvaluationPipeline(global_batch=True), gp_pc_sample_global): two ranks
    sharing cuda:0 over gloo, each sampling its block of objects with the Langevin grad_norm averaged over
    BOTH shards' rows (one partials all-gather per step), the prior and the device noise drawn for the whole
    batch, give bit for bit what ONE EvaluationPipeline call on the whole batch gives -- the reference's
    single cond_pc_sampler call (samplers.py:143-144). Shards of whole tiles (16-row tiles; 64-row tiles at
    132 x 64 rows) and a short last shard (5 objects: 3 + 2)."""
    import torch.multiprocessing as mp
    from genpose2_amd.runner import EvaluationPipeline
    world = 2
    port = 29400 + (os.getpid() + total) % 500
    mp.spawn(_global_worker, args=(world, port, str(tmp_path), total, k), nprocs=world, join=True)
    ref = EvaluationPipeline(_cfg_global(k)).run(_batch(total))
    for key in ("pred_pose", "energy", "aggregated"):
        np.testing.assert_array_equal(np.load(tmp_path / f"{key}.npy"), getattr(ref, key).cpu().numpy(), err_msg=key)
    assert not np.array_equal(np.load(tmp_path / "per_shard_pred_pose.npy"), ref.pred_pose.cpu().numpy())


def _cfg_global_ode(k, steps):
    from genpose2_amd.config import GenPoseConfig
    return GenPoseConfig(device=DEV, sampler_mode=["ode"], sampling_steps=steps, T0=0.55, eval_repeat_num=k,
                         noise_seed=4, seed=0)


def _global_ode_worker(rank, world, port, out_dir, total, k, steps):
    import torch.distributed as dist
    from genpose2_amd.runner import ShardedEvaluationPipeline
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        torch.manual_seed(21)
        pipe = ShardedEvaluationPipeline(_cfg_global_ode(k, steps), with_energy=False, global_batch=True)
        got = pipe.run(_batch(total))
        nfev = pipe.local.score_agent.last_nfev
        torch.manual_seed(21)
        own = ShardedEvaluationPipeline(_cfg_global_ode(k, steps), with_energy=False).run(_batch(total))
        np.save(os.path.join(out_dir, f"nfev_{rank}.npy"), np.array(nfev))
        if rank == 0:
            np.save(os.path.join(out_dir, "pred_pose.npy"), got.pred_pose.cpu().numpy())
            np.save(os.path.join(out_dir, "per_shard_pred_pose.npy"), own.pred_pose.cpu().numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total,k,steps", [(6, 16, None), (5, 16, 100), (132, 64, None)])
def test_global_batch_ode_two_ranks_equal_one_call(tmp_path, total, k, steps):
    """Global-batch ODE sampling (GlobalDeviceRk45 + gp_ode_auto_attempt_global): two ranks sharing cuda:0 over
    gloo integrate their blocks of objects with select_initial_step's norms over the whole batch's y0 / f0 / f1
    (gathered once) and every RK45 attempt's error norm over both shards' partials (one all-gather per attempt),
    so both ranks take the single call's accept / reject decisions: the gathered poses and nfev equal ONE
    solve_ivp call on the whole batch (samplers.py:226-234) bit for bit. T0 = 0.55 with t_eval unset and
    with 100 steps (dense output at eps); whole-tile shards and a short last shard; the per-shard default
    semantics differ (negative control)."""
    import torch.multiprocessing as mp
    from genpose2_amd.runner import EvaluationPipeline
    world = 2
    port = 29200 + (os.getpid() + total + (steps or 0)) % 90
    mp.spawn(_global_ode_worker, args=(world, port, str(tmp_path), total, k, steps), nprocs=world, join=True)
    torch.manual_seed(21)
    pipe = EvaluationPipeline(_cfg_global_ode(k, steps), with_energy=False)
    ref = pipe.run(_batch(total))
    got = np.load(tmp_path / "pred_pose.npy")
    np.testing.assert_array_equal(got, ref.pred_pose.cpu().numpy())
    assert int(np.load(tmp_path / "nfev_0.npy")) == int(np.load(tmp_path / "nfev_1.npy")) == pipe.score_agent.last_nfev
    assert not np.array_equal(np.load(tmp_path / "per_shard_pred_pose.npy"), ref.pred_pose.cpu().numpy())
