"""Explicit configuration object for the pose-candidate path.

Mirrors the flags of the reference's argparse config (``configs/config.py:5-135``) that
select or parameterise the hot path, with the same names and defaults, but without parsing
``sys.argv`` at import time (the reference parses at import, ``pointnet2.py:28``).
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import List, Optional


@dataclass
class GenPoseConfig:
    # model selection (configs/config.py:28-42)
    agent_type: str = "score"              # score | energy | scale
    sampler_mode: List[str] = field(default_factory=lambda: ["pc"])
    sampling_steps: Optional[int] = 500
    sde_mode: str = "ve"
    pose_mode: str = "rot_matrix"
    regression_head: str = "Rx_Ry_and_T"
    pointnet2_params: str = "light"
    pts_encoder: str = "pointnet2"
    energy_mode: str = "IP"
    s_theta_mode: str = "score"
    norm_energy: str = "identical"
    dino: str = "none"
    scale_embedding: int = 180
    num_points: int = 1024
    device: str = "cuda"
    # evaluation (configs/config.py:77-127)
    eval_repeat_num: int = 50
    T0: float = 1.0
    clustering: int = 1
    clustering_eps: float = 0.05
    clustering_minpts: float = 0.1667
    retain_ratio: float = 0.4
    save_video: bool = False
    batch_size: int = 192
    seed: int = 0
    # checkpoint paths (configs/config.py:51-53)
    pretrained_score_model_path: Optional[str] = None
    pretrained_energy_model_path: Optional[str] = None
    pretrained_scale_model_path: Optional[str] = None
    # build-specific knobs (no reference counterpart)
    noise: str = "philox"                  # philox (device RNG) | injected (parity buffers)
    noise_seed: int = 0

    def copy(self, **kw) -> "GenPoseConfig":
        return replace(self, **kw)

    def validate(self) -> None:
        """Reject configurations outside the built path with the reference's exception type
        (``NotImplementedError``, e.g. ``posenet.py:345``, ``scorenet.py:177``)."""
        if self.agent_type not in ("score", "energy", "scale"):
            raise NotImplementedError(f"agent_type {self.agent_type}")
        if self.sde_mode != "ve":
            raise NotImplementedError(f"sde_mode {self.sde_mode} (only 've' is on the path)")
        if self.pose_mode != "rot_matrix" or self.regression_head != "Rx_Ry_and_T":
            raise NotImplementedError("only pose_mode=rot_matrix / Rx_Ry_and_T are built")
        if self.dino not in ("none", "pointwise"):
            raise NotImplementedError("dino 'global' needs the DINOv3 backbone's global head (out of scope); "
                                      "'pointwise' takes the backbone's intermediate layers as data['dino_layers'] "
                                      "(or a backbone in PoseNet.dino)")
        if self.pts_encoder != "pointnet2" or self.pointnet2_params != "light":
            raise NotImplementedError("only pointnet2 'light' encoder is built")
        if self.sampler_mode[0] not in ("pc", "ode"):
            raise NotImplementedError(f"sampler {self.sampler_mode[0]}")
        if (self.energy_mode, self.s_theta_mode, self.norm_energy) != ("IP", "score", "identical"):
            raise NotImplementedError("only the IP/score/identical energy is built")
        if self.noise not in ("philox", "injected"):
            raise ValueError(f"noise {self.noise}")
