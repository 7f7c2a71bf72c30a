"""Harness counterpart of runners/evaluation_single.py on synthetic batches.

Stages, in the reference's order, with in-memory hand-off instead of the pickles between them
(evaluation_single.py:120,157,219,288):
  inference_score  (:78-120)  PoseNet(score).pred_func -> pred_pose (B,K,9), pts_feat
  inference_energy (:123-157) PoseNet(energy).get_energy(T=1e-5) -> (B,K,2)
  aggregate_pose   (:160-219) sort by energy, top retain_ratio*K, quaternion average (+DBSCAN)
  inference_scale  (:222-288) PoseNet(scale).pred_scale_func(axes=aggregated R, pts_feat)
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import torch

from . import aggregate
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
            edata = {"pts": batch["pts"], "pts_center": batch["pts_center"]}

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
            out.energy = self.energy_agent.get_energy(data=edata, pose_samples=pred_pose, T=1e-5, mode="test",
                                                      extract_feature=False)
        energy = out.energy if out.energy is not None else torch.ones(*pred_pose.shape[:2], 2,
                                                                      device=pred_pose.device)
        out.aggregated = aggregate.aggregate_pose(pred_pose, energy, cfg.retain_ratio, cfg.clustering,
                                                  cfg.clustering_eps, cfg.clustering_minpts)
        if self.scale_agent is not None:
            sdata = {"pts_feat": out.pts_feat, "rgb_feat": None,
                     "axes": out.aggregated[:, :3, :3].contiguous()}
            _, out.length = self.scale_agent.pred_scale_func(sdata)
        return out
