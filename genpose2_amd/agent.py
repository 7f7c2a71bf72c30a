"""``PoseNet``-compatible inference agent (networks/posenet_agent.py:52) on the MI355X path.

Drop-in for the inference members the evaluation runner uses
(runners/evaluation_single.py:83-104, 129-152, 258-280): ``__init__(cfg)``, ``load_ckpt``,
``eval``, ``pred_func``, ``get_energy``, ``pred_scale_func`` -- same signatures, argument
meaning, return shapes/dtypes and data-dict side effects. Training members are out of scope.

Every computation runs in libgenpose_hip.so; this class only moves tensors and scalars.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from . import aggregate, arch, device as dev, sde, weights
from .config import GenPoseConfig
from .ode import DeviceRk45, GlobalDeviceRk45, rk45_device, rk45_drive, time_scalars


def _as_config(cfg) -> GenPoseConfig:
    if isinstance(cfg, GenPoseConfig):
        return cfg
    base = GenPoseConfig()
    kw = {f: getattr(cfg, f) for f in base.__dataclass_fields__ if hasattr(cfg, f)}
    return base.copy(**kw)


class NoiseFeed:
    """Injected standard-normal draws for parity runs: ``prior`` (R,9) replaces the prior
    ``torch.randn`` (sde.py:34); ``z1``/``z2`` (T,R,9) replace the two ``randn_like`` per PC step
    (samplers.py:148,166)."""

    def __init__(self, prior: torch.Tensor, z1: Optional[torch.Tensor] = None, z2: Optional[torch.Tensor] = None):
        self.prior, self.z1, self.z2 = prior, z1, z2


class PoseNet:
    def __init__(self, cfg):
        self.cfg = _as_config(cfg)
        self.cfg.validate()
        self.device = torch.device(self.cfg.device)
        if self.device.type != "cuda":
            raise ValueError("genpose2_amd runs on a HIP device only (cfg.device must be 'cuda[:i]')")
        self.is_testing = False
        self.pts_feature = False
        self.noise_feed: Optional[NoiseFeed] = None
        self._calls = 0
        self.after_encode = None                   # optional callable run by pred_func after the encoder
        self._geom_stream = None                   # encode_geometry's side stream (DINO-pointwise)
        self.ode_host_control = False              # ODE: True runs the RK45 controller on the host
        self.ode_trace: Optional[list] = None      # ODE: a list receives [t, h, error norm] per step attempt
                                                   # (host controller)
        self._denoise_scalars = {}                 # ODE: (eps, steps) -> the denoise step's scalars
        self.global_batch = None                   # shard.GlobalBatch: this call is one shard of a global-batch
                                                   # PC / ODE call (runner.ShardedEvaluationPipeline(global_batch=True))
        self._gen = torch.Generator(device=self.device)
        self._gen.manual_seed(self.cfg.noise_seed)
        self.weights_source = f"synthetic(seed={self.cfg.seed})"
        # --dino pointwise: the frozen DINOv3 backbone (posenet.py:56-62) is not part of this build; a caller
        # that has it sets it here (an object with the reference's get_intermediate_layers), or passes its
        # output as data["dino_layers"]
        self.dino = None
        self._build(weights.synthetic_state_dict(self.weights_kind, seed=self.cfg.seed))

    @property
    def pointwise(self) -> bool:
        """--dino pointwise: the Pointnet2ClsMSGFus encoder (posenet.py:75-77) over per-point features."""
        return self.cfg.dino == "pointwise" and self.cfg.agent_type in ("score", "energy")

    @property
    def weights_kind(self) -> str:
        return self.cfg.agent_type + ("_pointwise" if self.pointwise else "")

    # ------------------------------------------------------------------ model construction
    def _build(self, sd: weights.StateDict) -> None:
        if self.pointwise:
            # a --dino pointwise checkpoint also holds the frozen DINOv3 backbone (posenet.py:56-62): its
            # intermediate layers are this path's input (data["dino_layers"], or self.dino)
            sd = {k: v for k, v in sd.items() if not k.startswith("dino.")}
        weights.check_keys(sd, self.weights_kind)
        self.state_dict = sd
        self._pc_cache = {}                        # T -> (step table, tproj); energy t -> time row
        if self.cfg.agent_type in ("score", "energy"):
            if self.pointwise:
                from .fus_encoder import FusEncoderModel
                from .img_encoder import ImgEncoderModel
                self.encoder = FusEncoderModel(sd, self.device)
                self.img_encoder = ImgEncoderModel(sd, self.device)
            else:
                self.encoder = dev.EncoderModel(sd, self.device)
            self.heads = dev.HeadModel(sd, self.device)
            self.scale = None
        else:
            self.encoder = self.heads = None
            self.scale = dev.ScaleModel(sd, self.device)

    def load_ckpt(self, name=None, model_dir=None, model_path=False, load_model_only=False):
        """posenet_agent.py:171-203 path resolution; loads with torch.load(weights_only=True)."""
        if not model_path:
            if name not in ("latest", "best"):
                name = "ckpt_epoch{}".format(name)
            load_path = os.path.join(model_dir if model_dir is not None else "./results/ckpts/debug",
                                     "{}.pth".format(name))
        else:
            load_path = model_dir
        sd = weights.load_checkpoint(load_path)
        self._build(sd)
        self.weights_source = load_path

    def eval(self):
        self.is_testing = True
        return self

    def train(self, mode: bool = True):
        raise NotImplementedError("training is out of scope for the MI355X inference path")

    # ------------------------------------------------------------------ helpers
    def _draw_prior(self, R: int) -> torch.Tensor:
        if self.noise_feed is not None:
            return self.noise_feed.prior.to(self.device, torch.float32).reshape(R, arch.POSE_DIM)
        return torch.randn((R, arch.POSE_DIM), generator=self._gen, device=self.device, dtype=torch.float32)

    def _pc_table(self, T: int):
        """Step table and per-step head projections for T steps: fixed by T and the weights, so
        built once (the H2D copy of the time grid would otherwise stall the host behind the
        encoder on every call)."""
        c = self._pc_cache.get(T)
        if c is None:
            tab = sde.pc_step_table(T)
            c = (tab, self.heads.time_proj(torch.from_numpy(tab[:, 0]).to(self.device)))
            self._pc_cache[T] = c
        return c

    def dino_layers(self, data):
        """The DINOv3 intermediate layers of posenet.py:138-144: data["dino_layers"] (three (B, 256, 384)
        tensors), or self.dino.get_intermediate_layers(roi_rgb, ...) when a backbone is set."""
        layers = data.get("dino_layers")
        if layers is not None:
            return layers
        if self.dino is None or data.get("roi_rgb") is None:
            raise KeyError("dino 'pointwise' needs data['dino_layers'] (the DINOv3 backbone's intermediate layers "
                           "[2, 6, 11], three (B, 256, 384) tensors) or a backbone in PoseNet.dino with data['roi_rgb']")
        return self.dino.get_intermediate_layers(data["roi_rgb"], n=list(arch.IMG_LAYERS), reshape=False, norm=True,
                                                 return_class_token=False)

    def _encode(self, data) -> torch.Tensor:
        if self.pointwise:
            # posenet.py:136-197: ImgEncoder over the backbone's layers, the patch -> point gather at
            # roi_xs / roi_ys, then Pointnet2ClsMSGFus over [pts | rgb_feat]. data["point_rgb_feat"]
            # (B, N, 384) skips the image branch with per-point features computed elsewhere.
            rgb = data.get("point_rgb_feat")
            if rgb is None:
                feat = self.img_encoder.forward(self.dino_layers(data))
                rgb = self.img_encoder.gather(feat, data["roi_xs"], data["roi_ys"])
            return self.encoder.forward(data["pts"], rgb, geometry=data.get("enc_geometry"))
        return self.encoder.forward(data["pts"], geometry=data.get("enc_geometry"))

    @torch.no_grad()
    def encode_geometry(self, data):
        """data["enc_geometry"]: FPS indices, centroids and ball lists of data["pts"] for every level, in
        this agent's encoder workspace. Every agent of the same encoder family (Light or DINO-pointwise) that
        encodes the same points (the ScoreNet and EnergyNet of one batch) then runs only its MLPs; valid until
        this agent encodes again. The DINO-pointwise geometry runs on a side stream after the current stream's
        work: the image branches (ImgEncoder, patch gather) do not read it and start beside it, and the fused
        encoders wait for its event before their first level."""
        if not self.pointwise:
            data["enc_geometry"] = self.encoder.geometry(data["pts"])
            return
        if self._geom_stream is None:
            self._geom_stream = torch.cuda.Stream(device=self.device)
        gs = self._geom_stream
        pts = data["pts"]
        self.encoder.workspace(pts.shape[0], pts.shape[1])   # allocated (if it grows) on the caller's stream
        gs.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(gs):
            data["enc_geometry"] = self.encoder.geometry(data["pts"])
        data["pts"].record_stream(gs)

    @torch.no_grad()
    def encode_func(self, data):
        """posenet_agent.py:385-387: data["pts_feat"] (no rgb branch with dino 'none')."""
        data["pts_feat"] = self._encode(data)
        data["rgb_feat"] = None
        if self.cfg.agent_type == "energy":
            # get_energy(extract_feature=False)'s object projection formed here, on the encoder's stream
            # (the runner runs it beside the score sampler), keyed by the feature tensor it came from
            data["_energy_pobj"] = (data["pts_feat"], self.heads.object_proj(data["pts_feat"]))

    @staticmethod
    def per_object_energy_t(bs: int) -> torch.Tensor:
        """get_energy(T=None)'s per-object times: (randint(1e-5 * 1e5, 1e-4 * 1e5, (bs, 1)) as float32) / 1e5
        from torch's default generator (posenet_agent.py:677-685), shape (bs,)."""
        return (torch.randint(1, 10, (bs, 1)).to(torch.float32) / 1e5).view(bs)

    def _energy_time_row(self, t: float):
        """The head-1 time row and sigma of t, cached with the weights (_pc_cache is reset when they
        change): evaluation calls get_energy with the same T = 1e-5 for every batch."""
        key = ("energy_t", t)
        c = self._pc_cache.get(key)
        if c is None:
            c = self._time_row_and_sigma(self.heads, t)
            self._pc_cache[key] = c
        return c

    @staticmethod
    def _time_row_and_sigma(heads: dev.HeadModel, t: float):
        t32 = torch.tensor([t], dtype=torch.float32)
        sig = float(sde.sigma(t32)[0])
        return heads.time_proj(t32.to(heads.device)), sig

    # ------------------------------------------------------------------ pred_func
    @torch.no_grad()
    def pred_func(self, data, repeat_num, save_path="./visualization_results", return_average_res=False,
                  init_x: torch.Tensor = None, T0=None, return_process=False, extract_feature=True):
        """posenet_agent.py:490-584. extract_feature=False takes data["pts_feat"] from an earlier
        encode_func (as get_energy's flag does), so a serving loop can encode the next batch on a
        side stream while this one samples."""
        if self.cfg.agent_type != "score":
            raise NotImplementedError("pred_func needs agent_type='score'")
        self.is_testing = True
        feat = self._encode(data) if extract_feature else dev.require_device_tensor(data["pts_feat"], "pts_feat")
        data["pts_feat"] = feat
        data["rgb_feat"] = None                    # dino none (posenet.py:316-318)
        if self.after_encode is not None:          # pipeline hook: start side-stream work here
            self.after_encode()
        bs = data["pts"].shape[0]
        K = int(repeat_num)
        R = bs * K
        self.pts_feature = True
        center = dev.require_device_tensor(data["pts_center"], "pts_center")
        pobj = self.heads.object_proj(feat)
        rep_init = None if init_x is None else init_x.to(self.device).unsqueeze(1).repeat(1, K, 1).view(R, -1)
        mode = self.cfg.sampler_mode[0]
        self._calls += 1
        if mode == "pc":
            T = int(self.cfg.sampling_steps)
            tab, tproj = self._pc_table(T)
            gb = self.global_batch
            if rep_init is None and gb is not None:   # this shard's rows of the whole batch's prior draw
                if self.noise_feed is not None:
                    raise ValueError("global-batch sampling draws the prior itself (noise_feed not supported)")
                x = (self._draw_prior(gb.total * K)[gb.lo * K:gb.hi * K] * sde.prior_sigma(arch.SDE_T)).contiguous()
            elif rep_init is None:   # prior((R,9)) at T=1 (sde.py:30-34); init_x used as-is (samplers.py:128)
                x = (self._draw_prior(R) * sde.prior_sigma(arch.SDE_T)).contiguous()
            else:
                x = rep_init.to(torch.float32).contiguous().clone()
            z1 = z2 = None
            if self.noise_feed is not None and self.noise_feed.z1 is not None:
                z1 = self.noise_feed.z1.to(self.device, torch.float32).contiguous()
                z2 = self.noise_feed.z2.to(self.device, torch.float32).contiguous()
            seed = (self.cfg.noise_seed * 1000003 + self._calls) & 0xFFFFFFFFFFFF
            want_xs = bool(return_process or self.cfg.save_video)
            res, q, xs = self.heads.pc_sample(pobj, tproj, tab, x, K, center, z1, z2, seed=seed, want_xs=want_xs,
                                              global_batch=gb)
            pred_pose = res.view(bs, K, -1)
            pred_q = q.view(bs, K, -1)
            in_process = xs.view(bs, K, T, -1) if xs is not None else None
        elif mode == "ode":
            pred_pose, pred_q, in_process = self._ode(pobj, center, bs, K, rep_init, T0,
                                                      bool(return_process or self.cfg.save_video))
        else:
            raise NotImplementedError(mode)
        self.pts_feature = False
        if return_average_res:
            avg = torch.zeros((bs, 7), dtype=torch.float32, device=self.device)   # torch.zeros((bs, 7)): fp32 (:560)
            avg[:, :4] = aggregate.average_quaternion_batch(pred_q[:, :, :4])
            avg[:, 4:] = torch.mean(pred_q[:, :, 4:], dim=1)
            if return_process:
                return pred_pose, pred_q, avg, in_process
            return pred_pose, pred_q, avg
        if return_process:
            return [pred_pose, in_process]
        return pred_pose, pred_q

    def _ode(self, pobj, center, bs, K, rep_init, T0, want_process=False):
        """cond_ode_sampler (samplers.py:180-258) on device: RK45 stages, error norms and dense
        output are HIP launches (genpose2_amd/ode.py DeviceRk45); the controller runs scipy's step
        logic on host scalars. Returns (pose (B,K,9) fp64, q (B,K,7) fp64, process or None)."""
        R = bs * K
        T0 = arch.SDE_T if T0 is None else float(T0)
        eps = arch.SAMPLING_EPS
        steps = self.cfg.sampling_steps
        gb = self.global_batch
        if gb is None:
            x0 = self._draw_prior(R) * sde.prior_sigma(T0)
        else:   # this shard's rows of the whole batch's prior draw
            if want_process or self.ode_host_control or self.ode_trace is not None:
                raise NotImplementedError("global-batch ODE sampling runs the device step controller only "
                                          "(no return_process / save_video, host control or trace)")
            if self.noise_feed is not None:
                raise ValueError("global-batch sampling draws the prior itself (noise_feed not supported)")
            x0 = self._draw_prior(gb.total * K)[gb.lo * K:gb.hi * K] * sde.prior_sigma(T0)
        if rep_init is not None:
            x0 = rep_init.to(torch.float32) + x0
        t_eval = None if steps is None else np.linspace(T0, eps, steps)
        if gb is not None:
            # one solve on the whole batch: the error norms over every shard's rows (GlobalDeviceRk45)
            be = GlobalDeviceRk45(self.heads, pobj, x0.to(self.device), K, gb)
            x, nfev, status = rk45_device(be, T0, eps, t_eval=t_eval)
            if status < 0 and t_eval is not None:
                raise RuntimeError("global-batch RK45 failed (step size below the spacing of t) with t_eval set: the "
                                   "t_eval outputs collected before the failure need the host controller")
        else:
            be = DeviceRk45(self.heads, pobj, x0.to(self.device), K)
            if want_process or self.ode_host_control or self.ode_trace is not None:
                # every solve_ivp output is kept: host-side controller, one error norm read per attempt
                _, nfev, status = rk45_drive(be, T0, eps, t_eval=t_eval, keep_all=want_process,
                                             trace=self.ode_trace)
            else:
                # default: the step controller runs on the device (no host round trip per attempt)
                x, nfev, status = rk45_device(be, T0, eps, t_eval=t_eval)
            if status < 0 and t_eval is not None and not want_process:
                # failed solve (step below spacing): solve_ivp returns the t_eval points collected so far and
                # cond_ode_sampler continues from res.y[:, -1]; only the host restatement keeps them all
                be = DeviceRk45(self.heads, pobj, x0.to(self.device), K)
                _, nfev, status = rk45_drive(be, T0, eps, t_eval=t_eval, keep_all=True)
                want_process = False
            if (want_process or self.ode_host_control or self.ode_trace is not None
                    or (status < 0 and t_eval is not None)):
                ys = be.outputs()                  # (n_t or 1, R*9) fp64
                if ys.shape[0] == 0:               # res.y[:, -1] of an empty solve_ivp result
                    raise IndexError("RK45 failed before collecting any t_eval point (res.y is empty)")
                x = ys[-1]
        self.last_nfev = nfev
        # denoise with the PC predictor step (samplers.py:240-249), GS, + pts_center, quaternion; its scalars depend
        # on eps and the step count only (formed once: the torch CPU ops sat between the solve and the denoise)
        key = (eps, steps)
        sc = self._denoise_scalars.get(key)
        if sc is None:
            t32, sig, _ = time_scalars(eps)
            vec_eps = torch.full((1,), eps, dtype=torch.float32)
            g2 = float(sde.diffusion(vec_eps).to(torch.float32) ** 2)
            step = float(np.float32((1 - eps) / (1000 if steps is None else steps)))
            sc = self._denoise_scalars[key] = (t32, sig, g2, step)
        t32, sig, g2, step = sc
        pose, q = self.heads.ode_denoise(pobj, t32, sig, g2, step, x, K, center, be.ws)
        in_process = None
        if want_process:
            n_t = ys.shape[0]
            xs = ys.reshape(n_t * R, -1).clone()
            xs, _ = dev.pose_epilogue_f64(xs, K, center.repeat(n_t, 1))  # row r -> object (r % R) // K
            in_process = xs.view(n_t, R, -1).permute(1, 0, 2).reshape(bs, K, n_t, -1)
        return pose.view(bs, K, -1), q.view(bs, K, -1), in_process

    # ------------------------------------------------------------------ get_energy
    @torch.no_grad()
    def get_energy(self, data, pose_samples, T=None, mode="test", extract_feature=True):
        """posenet_agent.py:608-705 (mode='test')."""
        if mode == "train":
            raise NotImplementedError("training is out of scope for the MI355X inference path")
        if mode != "test":
            raise NotImplementedError
        if self.cfg.agent_type != "energy":
            raise NotImplementedError("get_energy needs agent_type='energy'")
        self.is_testing = True
        bs, K = pose_samples.shape[0], pose_samples.shape[1]
        R = bs * K
        feat = self._encode(data) if extract_feature else dev.require_device_tensor(data["pts_feat"], "pts_feat")
        self.pts_feature = True
        pre = data.get("_energy_pobj") if not extract_feature else None
        pobj = pre[1] if pre is not None and pre[0] is feat else self.heads.object_proj(feat)
        pose = pose_samples.to(self.device).reshape(R, -1).to(torch.float32).clone()
        center = dev.require_device_tensor(data["pts_center"], "pts_center")
        pose[:, -3:] -= center.unsqueeze(1).repeat(1, K, 1).view(R, -1)
        if T is not None:
            trow, sig = self._energy_time_row(float(np.float32(T)))
            energy = self.heads.energy(pobj, trow, sig, pose, K)
        else:
            # per-object t = randint(1, 10) / 1e5 drawn from torch's default CPU generator with the
            # reference's call shape (posenet_agent.py:677-687), so torch.manual_seed reproduces its t's;
            # one time row and one energy launch per distinct t (at most 9), not per object
            ts = self.per_object_energy_t(bs)
            energy = torch.empty((R, 2), dtype=torch.float32, device=self.device)
            kk = torch.arange(K, device=self.device)
            for tv in torch.unique(ts).tolist():
                objs = torch.nonzero(ts == tv).view(-1).to(self.device)
                rows = (objs.view(-1, 1) * K + kk).view(-1)
                trow, sig = self._energy_time_row(tv)
                energy[rows] = self.heads.energy(pobj[objs].contiguous(), trow, sig, pose[rows].contiguous(), K)
        self._calls += 1
        return energy.view(bs, K, -1)

    # ------------------------------------------------------------------ pred_scale_func
    @torch.no_grad()
    def pred_scale_func(self, data):
        """posenet_agent.py:586-606 -> (axes, length (B,3))."""
        if self.cfg.agent_type != "scale":
            raise NotImplementedError("pred_scale_func needs agent_type='scale'")
        self.is_testing = True
        length = self.scale.forward(data["axes"], data["pts_feat"])
        return data["axes"], length
