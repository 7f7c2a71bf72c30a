"""Encoder arithmetic against a float64 restatement (the round-4 review's item 4 bar: per-level error vs
float64 no larger than exact fp32's). The device runs the encoder twice -- split-f16 levels 1-3 (default)
and every GEMM in exact fp32 MFMA (GENPOSE2_ENC_ARITH=f32) -- and each arithmetic's own chain of level
outputs is compared with a float64 chain over the same geometry (FPS and ball-query indices are integer
outputs, bit-identical in both arithmetics and pinned to the reference by test_encoder_levels_vs_golden).
The reference's own fp32 output (golden_encoder, object 0) is measured against the same float64 chain."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _conv_bn_relu64(h, sd, prefix):
    """Conv2d 1x1 -> BatchNorm2d(eval) -> ReLU (pytorch_utils.py:58-106) in float64 over the last axis."""
    from genpose2_amd import arch
    g = lambda k: np.asarray(sd[f"{prefix}.{k}"], np.float64)  # noqa: E731
    w = g("conv.weight")[:, :, 0, 0]
    y = h @ w.T
    y = (y - g("bn.bn.running_mean")) / np.sqrt(g("bn.bn.running_var") + arch.BN_EPS) * g("bn.bn.weight") + g("bn.bn.bias")
    return np.maximum(y, 0.0)


def _encoder64(sd, pts, levels):
    """pointnet2.py:244-252 in float64 with the device's geometry. Returns per-level point-major features
    (B, M, C) for levels 0-3 and the (B, 1024) output."""
    from genpose2_amd import arch
    xyz = pts.astype(np.float64)
    feats, out = None, []
    B = pts.shape[0]
    bi = np.arange(B)[:, None, None]
    for lv, branches in enumerate(arch.sa_branches()):
        hs = []
        if lv < 4:
            new_xyz = levels[lv]["new_xyz"].cpu().numpy().astype(np.float64)
            for br in branches:
                idx = levels[lv]["ball_idx"][br.branch].cpu().numpy().astype(np.int64)
                h = xyz[bi, idx] - new_xyz[:, :, None, :]                   # (B, M, ns, 3)
                if feats is not None:
                    h = np.concatenate([h, feats[bi, idx]], axis=-1)
                for i in range(len(br.widths) - 1):
                    h = _conv_bn_relu64(h, sd, f"pts_encoder.SA_modules.{lv}.mlps.{br.branch}.layer{i}")
                hs.append(h.max(axis=2))
            feats, xyz = np.concatenate(hs, axis=-1), new_xyz
            out.append(feats)
        else:   # GroupAll: raw xyz + features over all points
            for br in branches:
                h = np.concatenate([xyz, feats], axis=-1)
                for i in range(len(br.widths) - 1):
                    h = _conv_bn_relu64(h, sd, f"pts_encoder.SA_modules.{lv}.mlps.{br.branch}.layer{i}")
                hs.append(h.max(axis=1))
            out.append(np.concatenate(hs, axis=-1))
    return out


def _err(a, ref):
    """max and p99.9 of |a - ref| / max|ref| (the golden tests' relative measure)."""
    d = np.abs(a.astype(np.float64) - ref) / np.abs(ref).max()
    return float(d.max()), float(np.quantile(d, 0.999))


@pytest.mark.parametrize("tag", ["n1024", "n2048", "syn16"])
def test_encoder_arith_vs_float64(tag, score_sd):
    """n1024 / n2048: golden_encoder's points (B=3); syn16: 16 seeded synthetic objects of the bench's shape
    (N=1024, as config 4/5 objects)."""
    from genpose2_amd import device as gdev, synthetic
    g = golden("encoder")
    pts = g[f"{tag}_pts"] if tag != "syn16" else synthetic.make_batch(5, 16, 1024)[0]
    B, N = pts.shape[:2]
    enc = gdev.EncoderModel(score_sd, torch.device(DEV))
    res = {}
    for arith in ("split_f16", "f32"):
        enc.set_arith(arith)
        feat, ws = enc.forward(torch.from_numpy(pts).to(DEV), return_workspace=True)
        torch.cuda.synchronize()
        lv = enc.levels(B, N, ws)
        res[arith] = ([lv[k]["features"].cpu().numpy() for k in range(4)] + [feat.cpu().numpy()],
                      [{k: (v.clone() if torch.is_tensor(v) else [t.clone() for t in v]) for k, v in d.items()
                        if k != "features"} for d in lv[:4]])
    enc.set_arith("split_f16")
    # the geometry is the same in both arithmetics (integer outputs)
    for k in range(4):
        assert torch.equal(res["split_f16"][1][k]["fps_idx"], res["f32"][1][k]["fps_idx"])
        for b in range(2):
            assert torch.equal(res["split_f16"][1][k]["ball_idx"][b], res["f32"][1][k]["ball_idx"][b])
    ref64 = _encoder64(score_sd, pts, res["f32"][1])
    report = {}
    for k in range(5):
        es = _err(res["split_f16"][0][k], ref64[k])
        ef = _err(res["f32"][0][k], ref64[k])
        report[k] = (es, ef)
        print(f"{tag} level {k}: split_f16 max {es[0]:.2e} p99.9 {es[1]:.2e} | exact fp32 max {ef[0]:.2e} p99.9 {ef[1]:.2e}")
    # the reference's own fp32 run (object 0, levels 0-3 and the output) against the same float64 chain
    for k in range(4 if tag != "syn16" else 0):
        r = _err(g[f"{tag}_l{k}_feat0"].T, ref64[k][0])
        print(f"{tag} level {k}: reference fp32 (object 0) max {r[0]:.2e} p99.9 {r[1]:.2e}")
    if tag != "syn16":
        r = _err(g[f"{tag}_feat"], ref64[4])
        print(f"{tag} output: reference fp32 max {r[0]:.2e} p99.9 {r[1]:.2e}")
    # split-f16 is held to exact fp32 MFMA's own distance from float64: p99.9 within 1.25x at every level,
    # the single worst element within 2x (round 5: p99.9 ratios 0.89-1.01, max ratios 0.76-1.52)
    for k, (es, ef) in report.items():
        assert ef[0] < 1e-5 and es[0] < 1e-5, (k, es, ef)
        assert es[1] <= 1.25 * ef[1] and es[0] <= 2.0 * ef[0], (k, es, ef)
