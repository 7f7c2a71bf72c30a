"""Counterpart of runners/evaluation_single.py.

Stages, in the reference's order:
  inference_score  (:78-120)  PoseNet(score).pred_func -> pred_pose (B,K,9), pts_feat
  inference_energy (:123-157) PoseNet(energy).get_energy(T=1e-5) -> (B,K,2)
  aggregate_pose   (:160-219) sort by energy, top retain_ratio*K, quaternion average (+DBSCAN)
  inference_scale  (:222-288) PoseNet(scale).pred_scale_func(axes=aggregated R, pts_feat), or the
                              bounding box of the points in the aggregated frame without a ScaleNet

Two forms:
  * ``EvaluationPipeline``: one batch through all stages with in-memory hand-off (the energy
    encoder overlapped with the score sampler on a side stream);
  * the reference's file-backed stage functions with the same pickle hand-off format
    (evaluation_single.py:120,157,219,254,288) and ``process_batch``
    (datasets/datasets_omni6dpose.py:674-754), so a run against a real dataloader writes and reads
    the same stage files. The reference reads the module globals ``cfg`` and ``dataloader``; here
    they are arguments.
"""
from __future__ import annotations

import os
import pickle
from dataclasses import dataclass
from typing import Dict, Iterable, Optional

import torch

from . import aggregate
from . import device as dev
from .agent import PoseNet
from .config import GenPoseConfig


@dataclass
class StageOutputs:
    pred_pose: torch.Tensor
    pts_feat: torch.Tensor
    energy: Optional[torch.Tensor] = None
    aggregated: Optional[torch.Tensor] = None
    length: Optional[torch.Tensor] = None


class EvaluationPipeline:
    def __init__(self, cfg: GenPoseConfig, with_energy: bool = True, with_scale: bool = False):
        self.cfg = cfg
        self.score_agent = PoseNet(cfg.copy(agent_type="score")).eval()
        self.energy_agent = PoseNet(cfg.copy(agent_type="energy")).eval() if with_energy else None
        self.scale_agent = PoseNet(cfg.copy(agent_type="scale")).eval() if with_scale else None
        self._side = None

    def run(self, batch: Dict[str, torch.Tensor]) -> StageOutputs:
        """One batch through the stages. The energy network's point encoder depends only on the
        points, so it runs on a side stream concurrently with the score sampler (started after the
        score encoder, whose kernels want the whole chip) and is joined before the energy evaluation."""
        cfg = self.cfg
        data = dict(batch)
        edata = None
        if self.energy_agent is not None:
            main = torch.cuda.current_stream(batch["pts"].device)
            if self._side is None:
                self._side = torch.cuda.Stream(device=batch["pts"].device)
            # the energy encoder's inputs: the points, and for --dino pointwise the image branch's
            edata = {k: batch[k] for k in ("pts", "pts_center", "roi_rgb", "roi_xs", "roi_ys", "dino_layers",
                                           "point_rgb_feat") if k in batch}

            # one geometry pass (FPS, centroids, ball lists of every level) for both Light encoders
            self.score_agent.encode_geometry(data)
            if "enc_geometry" in data:
                edata["enc_geometry"] = data["enc_geometry"]

            def start_energy_encoder():   # after the score encoder, beside the sampler
                self._side.wait_stream(main)
                with torch.cuda.stream(self._side):
                    self.energy_agent.encode_func(edata)
            self.score_agent.after_encode = start_energy_encoder
        try:
            pred_pose, _ = self.score_agent.pred_func(data=data, repeat_num=cfg.eval_repeat_num, T0=cfg.T0,
                                                      return_average_res=False, return_process=False)
        finally:
            self.score_agent.after_encode = None
        out = StageOutputs(pred_pose=pred_pose, pts_feat=data["pts_feat"])
        if self.energy_agent is not None:
            main.wait_stream(self._side)
            edata["pts_feat"].record_stream(main)
            if "_energy_pobj" in edata:
                edata["_energy_pobj"][1].record_stream(main)
            out.energy = self.energy_agent.get_energy(data=edata, pose_samples=pred_pose, T=1e-5, mode="test",
                                                      extract_feature=False)
        energy = out.energy if out.energy is not None else torch.ones(*pred_pose.shape[:2], 2,
                                                                      device=pred_pose.device)
        out.aggregated = aggregate.aggregate_pose(pred_pose, energy, cfg.retain_ratio, cfg.clustering,
                                                  cfg.clustering_eps, cfg.clustering_minpts,
                                                  retain_num=int(cfg.eval_repeat_num * cfg.retain_ratio))
        if self.scale_agent is not None:
            sdata = {"pts_feat": out.pts_feat, "rgb_feat": None,
                     "axes": out.aggregated[:, :3, :3].contiguous()}
            _, out.length = self.scale_agent.pred_scale_func(sdata)
        return out


# ============================================================================ process_batch

class ShardedEvaluationPipeline:
    """EvaluationPipeline over one process group (config 4: B=2048 objects over 8 GPUs).

    Every rank holds the same agents; their packed weights (device buffers and the host layer tables)
    are broadcast from ``src`` (RCCL over xGMI) at construction and by ``sync_weights``, so weights
    loaded on ``src`` alone (``load_ckpt`` then ``sync_weights``) reach every GPU. ``run`` takes the WHOLE
    batch on every rank, processes the rank's contiguous object block (shard.shard_range) with no
    collective on the sampling path -- each shard is a reference call on its sub-batch -- and gathers
    pred_pose, pts_feat, energy, aggregated and length back in object order on every rank (dst=None)
    or on ``dst`` only. ``global_batch=True`` makes the shards one reference call on the whole batch instead
    (shard.GlobalBatch): the PC sampler's Langevin grad_norm over every shard's rows (one all-gather of the
    score-norm partials per step) with the prior and device noise drawn for the whole batch; the ODE sampler's
    select_initial_step norms over the whole batch's state (three one-time all-gathers) and every RK45
    attempt's error norm over every shard's partials (one all-gather per attempt)."""

    def __init__(self, cfg: GenPoseConfig, with_energy: bool = True, with_scale: bool = False, src: int = 0,
                 global_batch: bool = False):
        self.local = EvaluationPipeline(cfg, with_energy, with_scale)
        self.src = src
        self.global_batch = global_batch
        self.sync_weights()

    def agents(self):
        return [a for a in (self.local.score_agent, self.local.energy_agent, self.local.scale_agent) if a is not None]

    def load_ckpt(self, score: Optional[str] = None, energy: Optional[str] = None, scale: Optional[str] = None) -> None:
        """Load reference checkpoints on ``src`` only (paths may not exist on the other ranks), then
        broadcast them to every rank. A failure on ``src`` (missing file, key mismatch) is broadcast
        first and raised on every rank, so no rank is left waiting in the weight broadcast."""
        import torch.distributed as dist
        err = [None]
        if dist.get_rank() == self.src:
            try:
                for a, p in ((self.local.score_agent, score), (self.local.energy_agent, energy),
                             (self.local.scale_agent, scale)):
                    if a is not None and p:
                        a.load_ckpt(model_dir=p, model_path=True, load_model_only=True)
            except Exception as e:   # noqa: BLE001 -- re-raised below, on every rank
                err[0] = f"{type(e).__name__}: {e}"
        dist.broadcast_object_list(err, src=self.src)
        if err[0] is not None:
            raise RuntimeError(f"load_ckpt failed on rank {self.src}: {err[0]}")
        self.sync_weights()

    def sync_weights(self) -> None:
        """Every agent's weights from ``src`` to all ranks (buffers + host tables; shard.broadcast_agent)."""
        from . import shard
        for a in self.agents():
            shard.broadcast_agent(a, src=self.src)

    def run(self, batch: Dict[str, torch.Tensor], dst: Optional[int] = None) -> Optional[StageOutputs]:
        import torch.distributed as dist
        from . import arch, shard
        total = int(batch["pts"].shape[0])
        lo, hi = shard.shard_range(total, dist.get_world_size(), dist.get_rank())
        K = self.local.cfg.eval_repeat_num
        if self.global_batch:
            self.local.score_agent.global_batch = shard.GlobalBatch.of(total)   # raises on an empty shard
        if hi > lo:
            # per-object tensors, and lists of them (the DINOv3 layers of --dino pointwise)
            try:
                out = self.local.run({k: [t[lo:hi] for t in v] if isinstance(v, (list, tuple)) else v[lo:hi]
                                      for k, v in batch.items()})
            finally:
                self.local.score_agent.global_batch = None
        else:   # more ranks than objects: an empty shard still joins the gathers
            d = batch["pts"].device
            z = lambda *s: torch.zeros(s, dtype=torch.float32, device=d)  # noqa: E731
            out = StageOutputs(pred_pose=z(0, K, arch.POSE_DIM), pts_feat=z(0, arch.PTS_FEAT_DIM),
                               energy=z(0, K, 2) if self.local.energy_agent is not None else None,
                               aggregated=z(0, 4, 4), length=z(0, 3) if self.local.scale_agent is not None else None)
        g = shard.gather_outputs({"pred_pose": out.pred_pose, "pts_feat": out.pts_feat, "energy": out.energy,
                                  "aggregated": out.aggregated, "length": out.length}, total, dst)
        return None if g is None else StageOutputs(**g)

def process_batch(batch_sample: Dict, device, pose_mode: str = "rot_matrix", PTS_AUG_PARAMS=None) -> Dict:
    """process_batch (datasets_omni6dpose.py:674-754) for inference: the keys the pose-candidate
    path reads. ``pts`` = ``pcl_in`` on the device (un-normalised camera-frame points,
    ``pts_color`` the same tensor as in the reference), ``pts_center`` = mean over the points by
    gp_points_mean (:746-752). ``sym_info`` and the ``roi_*`` keys are passed through unchanged:
    only the DINO branches read them (out of scope), so they are not copied to the device.
    ``gt_pose`` ([rot6 | t]) is added when the batch carries ``rotation``/``translation``.
    Training-time augmentation (``PTS_AUG_PARAMS``) is out of scope."""
    if pose_mode != "rot_matrix":
        raise NotImplementedError(f"pose_mode {pose_mode}: only rot_matrix is built")
    if PTS_AUG_PARAMS is not None:
        raise NotImplementedError("training-time point augmentation is out of scope")
    pts = batch_sample["pcl_in"].to(device=device, dtype=torch.float32).contiguous()
    out = {"pts": pts, "pts_color": pts, "pts_center": dev.points_mean(pts)}
    for key in ("sym_info", "roi_rgb", "roi_xs", "roi_ys", "roi_center_dir"):
        if key in batch_sample:
            out[key] = batch_sample[key]
    if "rotation" in batch_sample and "translation" in batch_sample:
        R = batch_sample["rotation"].to(device=device, dtype=torch.float32)
        # get_pose_representation(.., "rot_matrix") = matrix_to_rotation_6d(R^T): the first two columns of R
        # (misc.py:189-192)
        rot6 = torch.cat([R[:, :, 0], R[:, :, 1]], dim=-1)
        out["gt_pose"] = torch.cat([rot6, batch_sample["translation"].to(device=device, dtype=torch.float32)], -1)
    return out


# ============================================================================ file-backed stages
def _agent(cfg: GenPoseConfig, agent_type: str, ckpt: Optional[str]) -> PoseNet:
    agent = PoseNet(cfg.copy(agent_type=agent_type))
    if ckpt:
        agent.load_ckpt(model_dir=ckpt, model_path=True, load_model_only=True)
    return agent.eval()


def inference_score(cfg: GenPoseConfig, dataloader: Iterable, save_path: str, agent: Optional[PoseNet] = None):
    """evaluation_single.py:78-120 -> pickle (all_pred_pose [per batch (B,K,9) on the device],
    all_score_feature [per batch {"pts_feat": (B,1024) cpu, "rgb_feat": None}])."""
    if os.path.exists(save_path):
        return
    agent = agent or _agent(cfg, "score", cfg.pretrained_score_model_path)
    all_pred_pose, all_score_feature = [], []
    for test_batch in dataloader:
        batch_sample = process_batch(test_batch, cfg.device, cfg.pose_mode)
        pred_pose, _ = agent.pred_func(data=batch_sample, repeat_num=cfg.eval_repeat_num, T0=cfg.T0,
                                       return_average_res=False, return_process=False)
        all_pred_pose.append(pred_pose)
        all_score_feature.append({"pts_feat": batch_sample["pts_feat"].cpu(),
                                  "rgb_feat": None if batch_sample["rgb_feat"] is None
                                  else batch_sample["rgb_feat"].cpu()})
    with open(save_path, "wb") as f:
        pickle.dump((all_pred_pose, all_score_feature), f)


def _load(path: str):
    # stage files are written by the functions above (or by the reference runner): trusted input
    with open(path, "rb") as f:
        return pickle.load(f)


def inference_energy(cfg: GenPoseConfig, dataloader: Iterable, score_path: str, save_path: str,
                     agent: Optional[PoseNet] = None):
    """evaluation_single.py:123-157 -> pickle all_pred_energy [per batch (B,K,2) cpu]."""
    if os.path.exists(save_path):
        return
    assert os.path.exists(score_path)
    all_pred_pose, _ = _load(score_path)
    agent = agent or _agent(cfg, "energy", cfg.pretrained_energy_model_path)
    all_pred_energy = []
    for i, test_batch in enumerate(dataloader):
        batch_sample = process_batch(test_batch, cfg.device, cfg.pose_mode)
        pred_energy = agent.get_energy(data=batch_sample, pose_samples=all_pred_pose[i], T=1e-5, mode="test",
                                       extract_feature=True)
        all_pred_energy.append(pred_energy.cpu())
    with open(save_path, "wb") as f:
        pickle.dump(all_pred_energy, f)


def aggregate_pose(cfg: GenPoseConfig, score_path: str, energy_path: Optional[str], save_path: str):
    """evaluation_single.py:160-219 -> pickle all_aggregated_pose [per batch (B,4,4) cpu]; one
    gp_rank_aggregate launch per batch. Without an energy file every candidate has energy 1."""
    if os.path.exists(save_path):
        return
    assert os.path.exists(score_path)
    all_pred_pose, _ = _load(score_path)
    if energy_path is not None:
        assert os.path.exists(energy_path)
        all_pred_energy = _load(energy_path)
    else:
        all_pred_energy = [torch.ones(*(p.shape[:2]), 2) for p in all_pred_pose]
    all_aggregated_pose = []
    for pred_pose, pred_energy in zip(all_pred_pose, all_pred_energy):
        dev_ = pred_pose.device if pred_pose.is_cuda else torch.device(cfg.device)
        agg = aggregate.aggregate_pose(pred_pose.to(dev_), pred_energy.to(dev_), cfg.retain_ratio,
                                       cfg.clustering, cfg.clustering_eps, cfg.clustering_minpts,
                                       retain_num=int(cfg.eval_repeat_num * cfg.retain_ratio))   # :180
        all_aggregated_pose.append(agg.cpu())
    with open(save_path, "wb") as f:
        pickle.dump(all_aggregated_pose, f)


def inference_scale(cfg: GenPoseConfig, dataloader: Iterable, score_path: str, aggregate_path: str,
                    save_path: str, agent: Optional[PoseNet] = None):
    """evaluation_single.py:222-288 -> pickle (all_final_pose [per batch (B,4,4) cpu],
    all_final_length [per batch (B,3) cpu]). Without cfg.pretrained_scale_model_path (and no agent)
    the lengths are the bounding box of the points in the aggregated frame (gp_bbox_length) and
    the poses are the aggregated ones (:229-254)."""
    if os.path.exists(save_path):
        return
    assert os.path.exists(score_path)
    _, all_score_feature = _load(score_path)
    assert os.path.exists(aggregate_path)
    all_aggregated_pose = _load(aggregate_path)
    if agent is None and cfg.pretrained_scale_model_path is None:
        all_final_length = []
        for i, test_batch in enumerate(dataloader):
            pcl = test_batch["pcl_in"].to(device=cfg.device, dtype=torch.float32)
            length = dev.bbox_length(pcl, all_aggregated_pose[i].to(cfg.device))
            all_final_length.append(length.cpu())
        with open(save_path, "wb") as f:
            pickle.dump((all_aggregated_pose, all_final_length), f)
        return
    agent = agent or _agent(cfg, "scale", cfg.pretrained_scale_model_path)
    all_final_pose, all_final_length = [], []
    for i, test_batch in enumerate(dataloader):
        batch_sample = process_batch(test_batch, cfg.device, cfg.pose_mode)
        batch_sample.update({k: (None if v is None else v.to(cfg.device)) for k, v in all_score_feature[i].items()})
        batch_sample["axes"] = all_aggregated_pose[i][:, :3, :3].to(cfg.device).contiguous()
        cal_mat, length = agent.pred_scale_func(batch_sample)
        final_pose = all_aggregated_pose[i].clone()
        final_pose[:, :3, :3] = cal_mat.cpu()
        all_final_pose.append(final_pose.cpu())
        all_final_length.append(length.cpu())
    with open(save_path, "wb") as f:
        pickle.dump((all_final_pose, all_final_length), f)
