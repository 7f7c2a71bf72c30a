"""Golden fixtures of the --dino pointwise image branch, made by running the REFERENCE's own code here:
``ImgEncoder`` (networks/img_encoder/img_encoder.py:6-100), the patch -> point gather of
``GFObjectPose.extract_pts_feature`` (networks/posenet.py:136-192), and a whole ``PoseNet.pred_func``
(posenet_agent.py:490-584) of the pointwise model.

The DINOv3 backbone (posenet.py:56-62, torch.hub from a local checkout with downloaded weights) is not
in this container. For the end-to-end case ``torch.hub.load`` is replaced by a stand-in whose
``get_intermediate_layers`` returns fixed synthetic layers (``dino_layers`` below): the backbone's
OUTPUT is the input of everything recorded, as for any golden vector. Everything after it -- the
ImgEncoder, the gather, Pointnet2ClsMSGFus, the score heads and the PC sampler -- is the reference's code
with the seeded synthetic weights of ``genpose2_amd.weights`` (``score_pointwise``).

Inputs are regenerated from committed seeds (``dino_layers``, ``roi_pixels`` here; points from
``genpose2_amd.synthetic``); only outputs are written.

Usage:  python tests/golden/make_golden_img.py        (golden_img.npz)
        python tests/golden/make_golden_img.py b16    (golden_img_b16.npz: B=16, K=50, T=20, per-level outputs)
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
sys.dont_write_bytecode = True

# case -> (objects, feature scale, seed): "hard" = LayerNorm-scale features (the geometric attention's
# softmax is near one-hot with the default N(0,1) position embedding), "soft" = features x 0.05 (a
# spread softmax that exercises every term)
CASES = {"hard": (2, 1.0, 8100), "soft": (2, 0.05, 8200)}
E2E = dict(cid=81, B=2, N=1024, K=10, T=20, scale=0.3, seed=8300)
# the larger end-to-end case (golden_img_b16.npz): 16 objects, K=50, and the fused encoder's per-level
# outputs of objects LEVEL_OBJS
E2E16 = dict(cid=82, B=16, N=1024, K=50, T=20, scale=0.3, seed=8400)
LEVEL_OBJS = (0, 15)


def dino_layers(b: int, scale: float, seed: int):
    """Three (b, 256, 384) float32 intermediate layers (DINOv3 get_intermediate_layers(n=[2, 6, 11],
    norm=True) output shape), from one PCG64 stream."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return [(rng.standard_normal((b, 256, 384), dtype=np.float32) * np.float32(scale)) for _ in range(3)]


def roi_pixels(b: int, n: int, seed: int):
    """(b, n) int64 roi_xs / roi_ys in [-30, 250): the 224-px roi grid plus out-of-range values, which the
    reference clamps to patch 0 / 255 (posenet.py:175-186)."""
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    return rng.integers(-30, 250, size=(b, n)), rng.integers(-30, 250, size=(b, n))


def reference_gather(feat, xs, ys):
    """posenet.py:146-192 as the reference executes it (the debugging prints dropped)."""
    import torch
    pos = (xs // 14) * 16 + ys // 14
    pos = torch.unsqueeze(pos, -1).expand(-1, -1, feat.shape[-1])
    if pos.max().item() >= feat.size(1):
        pos = pos.clamp(0, feat.size(1) - 1)
    if pos.min().item() < 0:
        pos = pos.clamp(0, feat.size(1) - 1)
    return torch.gather(feat, 1, pos.type(torch.int64))


class _Backbone:
    """Stand-in for the DINOv3 module torch.hub would load: returns fixed intermediate layers."""

    def __init__(self, layers):
        import torch
        self.layers = [torch.from_numpy(v) for v in layers]

    def requires_grad_(self, *a):
        return self

    def to(self, *a, **k):
        return self

    def get_intermediate_layers(self, x, n, reshape, norm, return_class_token):
        assert list(n) == [2, 6, 11] and not reshape and norm and not return_class_token
        return tuple(v[: x.shape[0]] for v in self.layers)


def main():
    import torch
    import make_golden as mg
    from genpose2_amd import synthetic, weights

    get_config, PoseNet = mg.import_reference("pc", E2E["T"])
    from networks.img_encoder.img_encoder import ImgEncoder

    sd = weights.synthetic_state_dict("score_pointwise", seed=0)
    enc = ImgEncoder(384, 256, 16)
    enc.load_state_dict({k[len("img_encoder."):]: torch.from_numpy(v) for k, v in sd.items()
                         if k.startswith("img_encoder.")}, strict=True)
    enc.eval()
    out = {}
    rec = {}
    enc.layer_attn.register_forward_hook(lambda m, i, o: rec.__setitem__("attn", o))
    enc.edge_guide.register_forward_hook(lambda m, i, o: rec.__setitem__("edge", o))
    for tag, (B, scale, seed) in CASES.items():
        layers = dino_layers(B, scale, seed)
        with torch.no_grad():
            final = enc([torch.from_numpy(v) for v in layers])
        xs, ys = roi_pixels(B, 1024, seed)
        g = reference_gather(final, torch.from_numpy(xs), torch.from_numpy(ys))
        out[f"{tag}_final0"] = final[0].numpy()                      # (256, 384), object 0
        out[f"{tag}_edge"] = rec["edge"].reshape(B, -1).numpy()       # (B, 96): ReLU + mean of the 3x3 conv
        out[f"{tag}_layer_w"] = torch.softmax(rec["attn"].transpose(1, 2), dim=1)[..., 0].numpy()   # (B, 3, 256)
        out[f"{tag}_gather0"] = g[0, :64].numpy()                    # (64, 384): the first 64 points of object 0
        out[f"{tag}_final_sum"] = final.double().sum(dim=(1, 2)).numpy()
    out.update(end_to_end(get_config, PoseNet, sd, E2E))
    np.savez_compressed(os.path.join(HERE, "golden_img.npz"), **out)
    print("img done", {k: v.shape for k, v in out.items()})


def end_to_end(get_config, PoseNet, sd, case, levels=()):
    """PoseNet(dino='pointwise').pred_func with the backbone stand-in; `levels`: objects whose fused-encoder
    per-level outputs (SA output, transformer output, fused input of levels 1-4; (C, M) each) are recorded."""
    import torch
    import make_golden as mg
    from genpose2_amd import synthetic
    layers = dino_layers(case["B"], case["scale"], case["seed"])
    torch.hub.load = lambda *a, **k: _Backbone(layers)
    cfg = get_config()
    cfg.dino = "pointwise"
    cfg.agent_type = "score"
    cfg.sampler_mode = ["pc"]
    cfg.sampling_steps = case["T"]
    agent = PoseNet(cfg)
    agent.net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    agent.eval()
    rec = {}
    if levels:
        enc = agent.net.pts_encoder

        def hook(name):
            def f(mod, inp, o):
                rec.setdefault(name, o)   # the first call: the encoder pass of pred_func
            return f
        for i, m in enumerate(enc.SA_modules):
            m.register_forward_hook(hook(f"sa{i}"))
        for i, m in enumerate(enc.transformer_blocks):
            m.register_forward_hook(hook(f"tf{i}"))
        for i, m in enumerate(enc.feature_fusions):
            m.register_forward_hook(hook(f"fu{i + 1}"))
    B, N, K, T = case["B"], case["N"], case["K"], case["T"]
    pts, _ = synthetic.make_batch(case["cid"], B, N)
    xs, ys = roi_pixels(B, N, case["seed"])
    d = {"pts": torch.from_numpy(pts), "pts_center": torch.from_numpy(pts).mean(dim=1),
         "roi_rgb": torch.zeros(B, 3, 4, 4), "roi_xs": torch.from_numpy(xs), "roi_ys": torch.from_numpy(ys)}
    rng = np.random.Generator(np.random.PCG64(case["seed"] + 2))
    prior = rng.standard_normal((B * K, 9)).astype(np.float32)
    zs = rng.standard_normal((2 * T, B * K, 9)).astype(np.float32)
    with mg.NoiseFeed(prior, zs) as nf:
        pose, q = agent.pred_func(d, repeat_num=K)
        assert nf.i == 2 * T
    out = dict(e2e_pts_feat=d["pts_feat"].numpy(), e2e_pred_pose=pose.numpy(), e2e_pred_q=q.numpy(),
               e2e_pts_center=d["pts_center"].numpy())
    if B * K * T <= 10 * 20 * 2:   # the small case keeps its draws; larger ones regenerate them (e2e_noise)
        out.update(e2e_prior=prior, e2e_z1=zs[0::2], e2e_z2=zs[1::2])
    objs = np.asarray(levels, np.int64)
    for i in range(5 if levels else 0):
        _, f_sa, _ = rec[f"sa{i}"]
        out[f"l{i}_sa"] = f_sa[objs].numpy()
        out[f"l{i}_tf"] = rec[f"tf{i}"][objs].numpy()
        if i > 0:
            out[f"l{i}_fused"] = rec[f"fu{i}"][objs].numpy()
    if levels:
        out["level_objs"] = objs
    return out


def e2e_noise(case):
    """The prior (B*K, 9) and the draws z1, z2 (T, B*K, 9) of an end-to-end case, regenerated from its seed."""
    B, K, T = case["B"], case["K"], case["T"]
    rng = np.random.Generator(np.random.PCG64(case["seed"] + 2))
    prior = rng.standard_normal((B * K, 9)).astype(np.float32)
    zs = rng.standard_normal((2 * T, B * K, 9)).astype(np.float32)
    return prior, zs[0::2], zs[1::2]


def main_b16():
    import make_golden as mg
    from genpose2_amd import weights
    get_config, PoseNet = mg.import_reference("pc", E2E16["T"])
    sd = weights.synthetic_state_dict("score_pointwise", seed=0)
    out = end_to_end(get_config, PoseNet, sd, E2E16, LEVEL_OBJS)
    np.savez_compressed(os.path.join(HERE, "golden_img_b16.npz"), **out)
    print("img b16 done", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    if sys.argv[1:] == ["b16"]:
        main_b16()
    else:
        main()
