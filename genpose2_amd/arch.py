"""Architecture constants of the GenPose++ hot path (``--dino none`` configuration).

Everything here is a fact about the reference model, restated as data so that the host
packer, the oracle and the kernels agree on one description:

* PointNet++ MSG "Light" encoder: ``networks/pts_encoder/pointnet2.py:77-89`` selected at
  ``:123-130``; channel bookkeeping ``pointnet2.py:219-236`` (+3 xyz channels per level,
  ``pointnet2_modules.py:118-119``).
* Score / energy heads: ``networks/gf_algorithms/scorenet.py:135-209`` and
  ``energynet.py:55-120`` (``Rx_Ry_and_T`` heads, ``pose_mode="rot_matrix"``).
* VE SDE constants: ``networks/gf_algorithms/sde.py:110-119``.
* ScaleNet: ``networks/scalenet.py:12-31``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Tuple

# ---------------------------------------------------------------- encoder (Light cfg)
NPOINTS: List[Optional[int]] = [512, 256, 128, 64, None]
RADII: List[Tuple[Optional[float], Optional[float]]] = [
    (0.01, 0.02), (0.02, 0.04), (0.04, 0.08), (0.08, 0.16), (None, None)]
NSAMPLES: List[Tuple[Optional[int], Optional[int]]] = [
    (16, 32), (16, 32), (16, 32), (16, 32), (None, None)]
MLPS: List[List[List[int]]] = [
    [[16, 16, 32], [32, 32, 64]],
    [[64, 64, 128], [64, 96, 128]],
    [[128, 196, 256], [128, 196, 256]],
    [[256, 256, 512], [256, 384, 512]],
    [[512, 512], [512, 512]],
]
N_LEVELS = len(NPOINTS)
BN_EPS = 1e-5  # nn.BatchNorm2d default, pytorch_utils.py:_BNBase
PTS_FEAT_DIM = 1024


@dataclass(frozen=True)
class SABranch:
    level: int
    branch: int
    npoint: Optional[int]      # None -> GroupAll
    radius: Optional[float]
    nsample: Optional[int]
    widths: Tuple[int, ...]    # (c_in incl. +3 xyz, h1, ..., c_out)
    out_offset: int            # channel offset of this branch in the level output


def sa_branches() -> List[List[SABranch]]:
    """Per level, per branch layer widths (``pointnet2.py:219-236``)."""
    levels = []
    c_in = 0  # Pointnet2ClsMSG(input_channels=0)
    for lv in range(N_LEVELS):
        branches = []
        off = 0
        for b, mlp in enumerate(MLPS[lv]):
            widths = (c_in + 3,) + tuple(mlp)
            branches.append(SABranch(lv, b, NPOINTS[lv], RADII[lv][b], NSAMPLES[lv][b],
                                     widths, off))
            off += mlp[-1]
        levels.append(branches)
        c_in = off
    return levels


def level_out_channels(level: int) -> int:
    return sum(m[-1] for m in MLPS[level])


# ---------------------------------------------------------------- DINO-pointwise fused encoder
# Pointnet2ClsMSGFus(input_channels=384) (pointnet2.py:255-388; selected by --dino pointwise,
# posenet.py:75-77): the Light SA levels with 384 per-point image-feature channels entering level 0,
# a relative-PE transformer block after every level (attention.py:414-533, bias 648-735) and a gated
# fusion of the (index-interpolated) image features before levels 1..4 (attention.py:224-325).
DINO_DIM = 384
FUS_HEADS = 8             # TransformerBlockWithRelativePE(channel_out, num_heads=8)
FUS_FF_MULT = 4           # linear1: d -> 4d
FUS_PE_HID = 16           # distance / direction encoders: Linear(1|3, 16) -> ReLU -> Linear(16, 8)
FUS_REDUCTION = 4         # GatedAttentionFusion reduction_ratio
FUS_SPATIAL_K = 7         # spatial attention Conv1d(2, 1, 7, padding=3)
LN_EPS = 1e-5             # nn.LayerNorm default

# ImgEncoder(dino_dim=384, num_patches=256, patch_size=16) over DINOv3's intermediate layers [2, 6, 11]
# (posenet.py:64, :137-143; networks/img_encoder/img_encoder.py) and the patch -> point gather
# pos = (roi_xs // 14) * 16 + roi_ys // 14, clamped (posenet.py:146-192)
IMG_PATCHES = 256
IMG_GRID = 16                         # h = w = sqrt(num_patches)
IMG_LAYERS = (2, 6, 11)               # get_intermediate_layers(n=[2, 6, 11], norm=True)
IMG_PATCH_PX = 14                     # roi_xs // 14, roi_ys // 14
IMG_REL_EMB = (2 * (IMG_GRID - 1)) ** 2   # nn.Embedding(max_rel * max_rel, dim // 4): 900 rows


def fus_sa_branches() -> List[List[SABranch]]:
    """sa_branches() with the 384 image-feature channels entering level 0 (pointnet2.py:281-285:
    channel_in starts at input_channels and is the previous level's channel_out afterwards)."""
    levels = []
    c_in = DINO_DIM
    for lv in range(N_LEVELS):
        branches, off = [], 0
        for b, mlp in enumerate(MLPS[lv]):
            branches.append(SABranch(lv, b, NPOINTS[lv], RADII[lv][b], NSAMPLES[lv][b],
                                     (c_in + 3,) + tuple(mlp), off))
            off += mlp[-1]
        levels.append(branches)
        c_in = off
    return levels


def fus_level_points(level: int, n_points: int) -> int:
    """Points (tokens) of level `level`'s output: npoint, or 1 after GroupAll."""
    return NPOINTS[level] if NPOINTS[level] is not None else 1


# ---------------------------------------------------------------- score / energy net
POSE_DIM = 9          # rot_matrix: 6D rotation + translation (genpose_utils.py:21-38)
POSE_HID = 256        # pose_encoder 9->256->256
T_EMB = 128           # GaussianFourierProjection(embed_dim=128) -> Linear(128,128)
GFP_HALF = 64
GFP_SCALE = 30.0
HEAD_HID = 256        # each of the 3 heads: Linear(1408,256) -> ReLU -> Linear(256,3)
N_HEADS = 3
HEAD_IN = PTS_FEAT_DIM + T_EMB + POSE_HID  # 1408, concat order [pts, t, pose] (scorenet.py:249)
HEAD_NAMES = ("fusion_tail_rot_x", "fusion_tail_rot_y", "fusion_tail_trans")

# ---------------------------------------------------------------- VE SDE (sde.py:110-119)
SIGMA_MIN = 0.01
SIGMA_MAX = 50.0
SAMPLING_EPS = 1e-5
SDE_T = 1.0
SNR = 0.16            # cond_pc_sampler default (samplers.py:119)
# sqrt(2 * (log(sigma_max) - log(sigma_min))) as the reference forms it (sde.py:24-26)
DIFFUSION_SCALE = math.sqrt(2.0 * (math.log(SIGMA_MAX) - math.log(SIGMA_MIN)))

# ---------------------------------------------------------------- ScaleNet
SCALE_EMB = 180       # --scale_embedding default (configs/config.py:42)
SCALE_HID = 256

# ---------------------------------------------------------------- FLOP accounting
def score_flops_per_candidate_step() -> int:
    """Hoisted score-MLP FLOPs per candidate-step: 2*(9*256+256*256+256*768+768*3)."""
    return 2 * (POSE_DIM * POSE_HID + POSE_HID * POSE_HID + POSE_HID * N_HEADS * HEAD_HID
                + N_HEADS * HEAD_HID * 3)


def encoder_flops_per_object(n_points: int = 1024) -> int:
    """Dense MAC count of the SA MLPs per object, x2 (GroupAll head included)."""
    macs = 0
    for lv, branches in enumerate(sa_branches()):
        for br in branches:
            rows = (br.npoint * br.nsample) if br.npoint is not None else NPOINTS[lv - 1]
            w = br.widths
            macs += rows * sum(w[i] * w[i + 1] for i in range(len(w) - 1))
    return 2 * macs
