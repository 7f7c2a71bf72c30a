"""DINO-pointwise fused encoder (Pointnet2ClsMSGFus) on a real MI355X, through the C ABI.

Each block is held to a CPU fp32 statement of the same op (torch CPU / the oracle), and the whole encoder
to the reference's own per-level outputs (golden_fus.npz, tests/golden/make_golden_fus.py). Tolerances:
FPS indices bit-exact; fp32 block outputs within 1e-5 of max|ref| (attention and LayerNorm chains
2e-5); the full encoder within 1e-5 of max|ref| per level.
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as tf

from conftest import golden

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def rel(a, b):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
    b = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else b
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def _vp(t):
    return ctypes.c_void_p(None if t is None else t.data_ptr())


def _s():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


@pytest.fixture(scope="module")
def lib():
    from genpose2_amd import _lib
    return _lib.load()


@pytest.fixture(scope="module")
def fus_sd():
    from genpose2_amd import weights
    return weights.synthetic_state_dict("score_pointwise", seed=0)


@pytest.fixture(scope="module")
def fus_model(fus_sd):
    from genpose2_amd.fus_encoder import FusEncoderModel
    return FusEncoderModel(fus_sd, torch.device(DEV))


# ---------------------------------------------------------------- blocks
@pytest.mark.parametrize("m,k,n,act,pad", [(100, 96, 288, 0, 0), (4096, 256, 1024, 1, 0), (37, 384, 96, 2, 0),
                                           (513, 1024, 192, 1, 32), (64, 2048, 1024, 0, 16), (1, 1024, 3072, 0, 0),
                                           (1500, 96, 288, 1, 0), (2000, 384, 96, 2, 16), (1031, 4096, 1024, 0, 0),
                                           (4096, 1024, 4096, 1, 0)])
def test_linear_vs_torch(lib, m, k, n, act, pad):
    from genpose2_amd._lib import check
    g = torch.Generator().manual_seed(m + k + n)
    x = torch.randn(m, k + pad, generator=g)
    w = torch.randn(n, k, generator=g) / k ** 0.5
    b = torch.randn(n, generator=g)
    ref = tf.linear(x[:, :k].double(), w.double(), b.double())
    ref = [ref, torch.relu(ref), torch.sigmoid(ref)][act].float()
    y = torch.zeros(m, n + pad, device=DEV)
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    check(lib.gp_linear(_vp(xd), k + pad, m, k, _vp(wd), _vp(bd), n, act, _vp(y), n + pad, _s()), "linear")
    torch.cuda.synchronize()
    assert rel(y[:, :n], ref) < 1e-5
    if pad:
        assert torch.all(y[:, n:] == 0)          # ldy: nothing written past n


@pytest.mark.parametrize("m,k,n,act,pad", [(100, 96, 288, 0, 0), (4096, 256, 1024, 1, 0), (37, 384, 96, 2, 0),
                                           (513, 1024, 192, 1, 32), (1500, 96, 288, 1, 0), (2000, 384, 96, 2, 16),
                                           (1031, 4096, 1024, 0, 0), (4096, 1024, 4096, 1, 0), (3000, 192, 48, 0, 0),
                                           (2500, 192, 96, 3, 0), (1100, 2048, 1024, 3, 16)])
def test_linear_split_vs_torch(lib, m, k, n, act, pad):
    """gp_linear_split (split-f16 MFMA) against the fp64 linear: the split arithmetic's bound (about 3
    fp32 roundings per product) stays well inside the fused encoder's 1e-5 budget. Rows of very different
    magnitudes (per-row scaling) and an all-zero row are included."""
    from genpose2_amd._lib import check
    from genpose2_amd.fus_encoder import pack_split_linear
    g = torch.Generator().manual_seed(m + k + n + 1)
    x = torch.randn(m, k + pad, generator=g) * torch.exp(torch.randn(m, 1, generator=g) * 3)
    x[m // 2] = 0.0
    w = torch.randn(n, k, generator=g) / k ** 0.5
    b = torch.randn(n, generator=g)
    ref = tf.linear(x[:, :k].double(), w.double(), b.double())
    if act == 3:   # the gate with GatedAttentionFusion's mix, x = [cur | att]
        gte = torch.sigmoid(ref)
        ref = gte * x[:, :n].double() + (1 - gte) * x[:, n:2 * n].double()
    else:
        ref = [ref, torch.relu(ref), torch.sigmoid(ref)][act]
    wpk = pack_split_linear(w.numpy())
    assert wpk.size == lib.gp_linear_split_words(n, k)
    y = torch.zeros(m, n + pad, device=DEV)
    xd, wd, bd = x.to(DEV), torch.from_numpy(wpk).to(DEV), b.to(DEV)
    rmax = torch.empty(m, device=DEV)
    ymax = torch.full((m,), -1.0, device=DEV) if act else None
    check(lib.gp_linear_split(_vp(xd), k + pad, m, k, _vp(wd), _vp(bd), n, act, _vp(y), n + pad, _vp(rmax), 0,
                              _vp(ymax), _s()), "linear_split")
    torch.cuda.synchronize()
    if act:   # the epilogue's row maxima of y
        assert torch.equal(ymax, y[:, :n].abs().max(1).values)
        y2 = torch.zeros_like(y)   # the same call with the row maxima handed over
        check(lib.gp_linear_split(_vp(xd), k + pad, m, k, _vp(wd), _vp(bd), n, act, _vp(y2), n + pad, _vp(rmax), 1,
                                  None, _s()), "linear_split (rmax given)")
        torch.cuda.synchronize()
        assert torch.equal(y, y2)
    # per-row bound: |err| <= 4 * 2^-22 * sum_k |x||w| (+ the bias rounding; the mix: times max(|cur|, |att|))
    bound = tf.linear(x[:, :k].double().abs(), w.double().abs()) * 4 * 2.0 ** -22 + 1e-7 * (1 + ref.abs())
    if act == 3:
        bound = bound * torch.maximum(x[:, :n].double().abs(), x[:, n:2 * n].double().abs()) + \
            4e-7 * (x[:, :n].double().abs() + x[:, n:2 * n].double().abs())
    err = (y[:, :n].cpu().double() - ref).abs()
    assert torch.all(err <= bound), float((err / bound).max())
    assert torch.equal(rmax.cpu(), x[:, :k].abs().max(1).values)   # row maxima over the k columns read
    if pad:
        assert torch.all(y[:, n:] == 0)


def test_add_layernorm_vs_torch(lib):
    from genpose2_amd._lib import check
    for m, d in ((777, 96), (300, 1024), (5, 512), (64, 256)):
        g = torch.Generator().manual_seed(d)
        x, r = torch.randn(m, d, generator=g) * 3, torch.randn(m, d, generator=g)
        gam, bet = torch.rand(d, generator=g) + 0.5, torch.randn(d, generator=g) * 0.1
        ref = tf.layer_norm(x + r, (d,), gam, bet, 1e-5)
        y = torch.empty(m, d, device=DEV)
        ymax = torch.empty(m, device=DEV)
        xd, rd, gd, bd = (t.to(DEV) for t in (x, r, gam, bet))    # held: the call only enqueues
        check(lib.gp_add_layernorm(_vp(xd), _vp(rd), m, d, _vp(gd), _vp(bd), ctypes.c_float(1e-5), _vp(y),
                                   _vp(ymax), _s()), "add_layernorm")
        torch.cuda.synchronize()
        assert rel(y, ref) < 2e-6, (m, d)
        assert torch.equal(ymax, y.abs().max(1).values)


@pytest.mark.parametrize("n", [64, 100, 512])
def test_relpe_bias_vs_oracle(lib, fus_sd, n):
    from genpose2_amd._lib import check
    from genpose2_amd.fus_encoder import pack_relpe
    from oracle import oracle
    rng = np.random.default_rng(n)
    xyz = rng.uniform(-0.1, 0.1, size=(2, n, 3)).astype(np.float32)
    xyz[1, 5] = xyz[1, 3]                          # a duplicate point: zero distance off the diagonal
    p = "pts_encoder.relative_pos_encoders.1"
    ref = oracle.relative_bias(fus_sd, p, xyz)
    out = torch.empty(2, 8, n, n, device=DEV)
    pe = torch.from_numpy(pack_relpe(fus_sd, p)).to(DEV)
    xyz_d = torch.from_numpy(xyz).to(DEV)
    check(lib.gp_relpe_bias(_vp(pe), _vp(xyz_d), 2, n, _vp(out), _s()), "relpe_bias")
    torch.cuda.synchronize()
    assert rel(out, ref) < 1e-5


@pytest.mark.parametrize("n,d,with_bias", [(512, 96, True), (256, 256, True), (128, 512, True), (64, 1024, True),
                                           (1, 1024, False), (77, 256, True)])
def test_mha_attention_vs_torch(lib, n, d, with_bias):
    from genpose2_amd._lib import check
    B, H = 2, 8
    hd = d // H
    g = torch.Generator().manual_seed(n + d)
    qkv = torch.randn(B, n, 3 * d, generator=g)
    bias = torch.randn(B, H, n, n, generator=g) * 0.5 if with_bias else None
    q, k, v = (qkv[..., i * d:(i + 1) * d].reshape(B, n, H, hd).transpose(1, 2).double() for i in range(3))
    s = torch.matmul(q, k.transpose(-2, -1)) / np.sqrt(hd)
    if bias is not None:
        s = s + bias.double()
    ref = torch.matmul(torch.softmax(s, -1), v).transpose(1, 2).reshape(B, n, d).float()
    out = torch.empty(B, n, d, device=DEV)
    ymax = torch.full((B * n,), -1.0, device=DEV)
    qkv_d, bias_d = qkv.to(DEV), (None if bias is None else bias.to(DEV))
    check(lib.gp_mha_attention(_vp(qkv_d), _vp(bias_d), B, n, d, _vp(out), _vp(ymax), _s()), "mha_attention")
    torch.cuda.synchronize()
    assert rel(out, ref) < 2e-5
    assert torch.equal(ymax, out.reshape(B * n, d).abs().max(1).values)


@pytest.mark.parametrize("n,d", [(512, 96), (256, 256), (77, 96), (130, 256), (1, 96)])
def test_mha_relpe_attention_matches_two_kernel_path(lib, fus_sd, n, d):
    """gp_mha_relpe_attention (bias in registers) against gp_relpe_bias + gp_mha_attention on the same
    inputs: the same bias bits, so only the softmax blocking differs (2e-6), and the row maxima."""
    from genpose2_amd._lib import check
    from genpose2_amd.fus_encoder import pack_relpe
    B = 3
    g = torch.Generator().manual_seed(n * 7 + d)
    qkv = torch.randn(B, n, 3 * d, generator=g).to(DEV)
    xyz = (torch.rand(B, n, 3, generator=g) * 0.2 - 0.1).to(DEV)
    if n > 5:
        xyz[1, 5] = xyz[1, 3]                          # a duplicate point
    pe = torch.from_numpy(pack_relpe(fus_sd, "pts_encoder.relative_pos_encoders.0")).to(DEV)
    bias = torch.empty(B, 8, n, n, device=DEV)
    ref = torch.empty(B, n, d, device=DEV)
    out = torch.empty(B, n, d, device=DEV)
    ymax = torch.full((B * n,), -1.0, device=DEV)
    check(lib.gp_relpe_bias(_vp(pe), _vp(xyz), B, n, _vp(bias), _s()), "relpe_bias")
    check(lib.gp_mha_attention(_vp(qkv), _vp(bias), B, n, d, _vp(ref), None, _s()), "mha_attention")
    check(lib.gp_mha_relpe_attention(_vp(qkv), _vp(xyz), _vp(pe), B, n, d, _vp(out), _vp(ymax), _s()),
          "mha_relpe_attention")
    torch.cuda.synchronize()
    assert rel(out, ref) < 2e-6
    assert torch.equal(ymax, out.reshape(B * n, d).abs().max(1).values)


@pytest.mark.parametrize("n_in,n_out,c", [(1024, 512, 384), (512, 256, 384), (300, 77, 40), (64, 64, 8)])
def test_interp_points_vs_torch(lib, n_in, n_out, c):
    from genpose2_amd._lib import check
    x = torch.randn(2, n_in, c, generator=torch.Generator().manual_seed(n_in))
    ref = tf.interpolate(x.transpose(1, 2), size=n_out, mode="linear", align_corners=False).transpose(1, 2)
    y = torch.empty(2, n_out, c, device=DEV)
    ymax = torch.empty(2 * n_out, device=DEV)
    xd = x.to(DEV)
    check(lib.gp_interp_points(_vp(xd), 2, n_in, c, n_out, _vp(y), _vp(ymax), _s()), "interp_points")
    torch.cuda.synchronize()
    assert rel(y, ref) < 1e-6
    assert torch.equal(ymax, y.reshape(2 * n_out, c).abs().max(1).values)


@pytest.mark.parametrize("k", [1, 2, 3, 4])
def test_gated_fusion_vs_oracle(fus_model, fus_sd, k):
    """GatedAttentionFusion of level k (C = level k-1's channels) vs the oracle restatement."""
    from genpose2_amd import arch
    from oracle import oracle
    c = arch.level_out_channels(k - 1)
    n = arch.NPOINTS[k - 1]
    rng = np.random.default_rng(k)
    cur = np.maximum(rng.normal(size=(2, n, c)), 0).astype(np.float32)
    orig = rng.normal(size=(2, n, 384)).astype(np.float32)
    got = fus_model.fusion(k, torch.from_numpy(cur).to(DEV), torch.from_numpy(orig).to(DEV))
    ref = oracle.gated_fusion(fus_sd, f"pts_encoder.feature_fusions.{k - 1}", cur.transpose(0, 2, 1),
                              orig.transpose(0, 2, 1)).transpose(0, 2, 1)
    torch.cuda.synchronize()
    assert rel(got, ref) < 1e-5


# ---------------------------------------------------------------- SA levels by the level API
def test_sa_level_api_equals_encoder_forward():
    """gp_encoder_fps + gp_sa_level, level by level, reproduces gp_encoder_forward bit for bit (Light encoder)."""
    from genpose2_amd import _lib, arch, synthetic, weights
    from genpose2_amd.device import EncoderModel
    enc = EncoderModel(weights.synthetic_state_dict("score"), torch.device(DEV))
    pts_np, _ = synthetic.make_batch(81, 5, 1024)
    pts = torch.from_numpy(pts_np).to(DEV)
    ref, ws_ref = enc.forward(pts, return_workspace=True)
    ref_levels = [{k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in d.items()}
                  for d in enc.levels(5, 1024, ws_ref)]
    ref = ref.clone()
    lib = _lib.load()
    ws = torch.empty(int(lib.gp_encoder_workspace_size(5, 1024)), dtype=torch.uint8, device=DEV)
    _lib.check(lib.gp_encoder_fps(_vp(pts), 5, 1024, _vp(ws), ws.numel(), _s()))
    feat = None
    for lv in range(5):
        m = arch.NPOINTS[lv] if lv < 4 else 1
        out = torch.empty(5, m, arch.level_out_channels(lv), device=DEV)
        _lib.check(lib.gp_sa_level(_vp(enc.wbuf), enc.offsets.ctypes.data_as(_lib.c_int64_p), lv,
                                   0 if feat is None else feat.shape[2], _vp(pts), 5, 1024, _vp(feat), _vp(ws),
                                   ws.numel(), _vp(out), _s()), f"sa_level {lv}")
        if lv < 4:
            assert torch.equal(out, ref_levels[lv]["features"]), lv
        feat = out
    torch.cuda.synchronize()
    assert torch.equal(feat.reshape(5, -1), ref)


def test_fus_encoder_shared_geometry_bit_exact(fus_sd):
    """Two fused encoders (different weights) of the same points over ONE geometry pass -- the first model's
    geometry() (gp_encoder_geometry), both through gp_sa_level_geom, the second on another stream -- equal each
    model's self-contained forward (gp_encoder_fps + gp_sa_level, its own ball queries) bit for bit, every level;
    geometry of other points or of a model that encoded again is refused."""
    from genpose2_amd import synthetic, weights
    from genpose2_amd.fus_encoder import FusEncoderModel
    a = FusEncoderModel(fus_sd, torch.device(DEV))
    b = FusEncoderModel(weights.synthetic_state_dict("energy_pointwise", seed=1), torch.device(DEV))
    pts_np, _ = synthetic.make_batch(82, 6, 1024, n_unique_every=3)
    p = torch.from_numpy(pts_np).to(DEV)
    rgb = torch.randn(6, 1024, 384, device=DEV, generator=torch.Generator(device=DEV).manual_seed(3))
    ref = {}
    for name, m in (("a", a), ("b", b)):
        out, lv = m.forward(p, rgb, return_levels=True)
        ref[name] = (out.clone(), [{k: v.clone() for k, v in d.items()} for d in lv])
    side = torch.cuda.Stream(device=DEV)
    for _ in range(2):
        g = a.geometry(p)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            got_b = b.forward(p, rgb, return_levels=True, geometry=g)
        got_a = a.forward(p, rgb, return_levels=True, geometry=g)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        for name, got in (("a", got_a), ("b", got_b)):
            assert torch.equal(got[0], ref[name][0]), name
            for lv, (d0, d1) in enumerate(zip(ref[name][1], got[1])):
                for k in d0:
                    assert torch.equal(d0[k], d1[k]), (name, lv, k)
    with pytest.raises(ValueError):
        b.forward(p.clone(), rgb, geometry=g)   # other points
    a.forward(p, rgb)                           # the producer encodes again: its geometry is rewritten
    with pytest.raises(ValueError, match="stale"):
        b.forward(p, rgb, geometry=g)


def test_pointwise_agents_geometry_on_side_stream_bit_exact():
    """PoseNet.encode_geometry with the DINO-pointwise encoders runs the geometry on a side stream (the image
    branches start beside it): the ScoreNet and EnergyNet agents' encode_func over that geometry -- the EnergyNet
    one on a third stream, twice in a row with no synchronisation between the steps -- equal each agent's
    self-contained encode_func bit for bit."""
    import numpy as np
    from genpose2_amd import synthetic
    from genpose2_amd.agent import PoseNet
    from genpose2_amd.config import GenPoseConfig
    B, N = 4, 1024
    cfg = GenPoseConfig(device=DEV, dino="pointwise")
    score, energy = PoseNet(cfg).eval(), PoseNet(cfg.copy(agent_type="energy")).eval()
    pts, center = synthetic.make_batch(83, B, N)
    rng = np.random.Generator(np.random.PCG64(5))
    d0 = {"pts": torch.from_numpy(pts).to(DEV), "pts_center": torch.from_numpy(center).to(DEV),
          "dino_layers": [torch.from_numpy(rng.standard_normal((B, 256, 384), dtype=np.float32)).to(DEV)
                          for _ in range(3)],
          "roi_xs": torch.from_numpy(rng.integers(0, 224, size=(B, N)).astype(np.int32)).to(DEV),
          "roi_ys": torch.from_numpy(rng.integers(0, 224, size=(B, N)).astype(np.int32)).to(DEV)}
    ref = {}
    for name, agent in (("score", score), ("energy", energy)):
        d = dict(d0)
        agent.encode_func(d)
        ref[name] = d["pts_feat"].clone()
    side = torch.cuda.Stream(device=DEV)
    main = torch.cuda.current_stream()
    got = []
    for _ in range(2):
        data, edata = dict(d0), dict(d0)
        score.encode_geometry(data)
        assert score._geom_stream is not None and data["enc_geometry"].event is not None
        edata["enc_geometry"] = data["enc_geometry"]
        side.wait_stream(main)
        with torch.cuda.stream(side):
            energy.encode_func(edata)
        score.encode_func(data)
        main.wait_stream(side)
        got.append((data["pts_feat"], edata["pts_feat"]))
    torch.cuda.synchronize()
    for fs, fe in got:
        assert torch.equal(fs, ref["score"]) and torch.equal(fe, ref["energy"])


# ---------------------------------------------------------------- whole encoder vs the reference
def test_fus_encoder_vs_reference_golden(fus_model):
    import make_golden_fus as mf
    from genpose2_amd import synthetic
    g = golden("fus")
    pts, _ = synthetic.make_batch(mf.CID, mf.B, mf.N)
    feat = mf.rgb_features(mf.B, mf.N)
    out, levels = fus_model.forward(torch.from_numpy(pts).to(DEV), torch.from_numpy(feat).to(DEV),
                                    return_levels=True)
    torch.cuda.synchronize()
    errs = {}
    for lv in range(5):
        for k in ("sa", "tf", "fused"):
            if f"l{lv}_{k}" in g:
                errs[(lv, k)] = rel(levels[lv][k][0].cpu().numpy().T, g[f"l{lv}_{k}"])
    print("fused encoder per-level rel errors", errs, "final", rel(out, g["feat"]))
    assert max(errs.values()) < 1e-5, errs
    assert rel(out, g["feat"]) < 1e-5


def test_pointwise_agent_pred_func():
    """PoseNet(dino='pointwise'): pred_func encodes with the fused encoder from data['point_rgb_feat'], sets
    data['pts_feat'] / data['rgb_feat'] = None like the reference, and samples with the pointwise heads; the
    features equal the fused encoder's, the poses equal the PC oracle on those features (injected noise)."""
    import make_golden_fus as mf
    from genpose2_amd import synthetic, weights
    from genpose2_amd.agent import NoiseFeed, PoseNet
    from genpose2_amd.config import GenPoseConfig
    from oracle import oracle
    B, K, T = 2, 4, 20
    pts, center = synthetic.make_batch(mf.CID, B, 1024)
    rgb = mf.rgb_features(B, 1024)
    agent = PoseNet(GenPoseConfig(device=DEV, sampling_steps=T, dino="pointwise")).eval()
    rng = np.random.default_rng(3)
    prior = rng.standard_normal((B * K, 9)).astype(np.float32)
    z1 = rng.standard_normal((T, B * K, 9)).astype(np.float32)
    z2 = rng.standard_normal((T, B * K, 9)).astype(np.float32)
    agent.noise_feed = NoiseFeed(torch.from_numpy(prior), torch.from_numpy(z1), torch.from_numpy(z2))
    data = {"pts": torch.from_numpy(pts).to(DEV), "pts_center": torch.from_numpy(center).to(DEV),
            "point_rgb_feat": torch.from_numpy(rgb).to(DEV)}
    pose, _ = agent.pred_func(data, repeat_num=K)
    torch.cuda.synchronize()
    assert data["rgb_feat"] is None
    sd = weights.synthetic_state_dict("score_pointwise")
    ofeat = oracle.fus_encoder_forward(sd, pts, rgb)
    assert rel(data["pts_feat"], ofeat) < 1e-5
    fr, cr = np.repeat(ofeat, K, 0), np.repeat(center, K, 0)
    sig = np.float32(0.01 * 5000.0)
    _, res = oracle.pc_sample(lambda x, t: oracle.score_forward(sd, fr, x, t), (prior * sig).astype(np.float32), cr,
                              T, z1, z2)
    got = pose.cpu().numpy().reshape(B * K, 9)
    assert np.abs(got[:, :6] - res[:, :6]).max() < 1e-4
    assert rel(got[:, 6:], res[:, 6:]) < 1e-5
    with pytest.raises(KeyError):
        agent.pred_func({"pts": data["pts"], "pts_center": data["pts_center"]}, repeat_num=K)


# ---------------------------------------------------------------- ImgEncoder + patch gather
@pytest.mark.parametrize("arith", ["split_f16", "f32"])
@pytest.mark.parametrize("tag", ["hard", "soft"])
def test_img_encoder_vs_reference_golden(tag, arith):
    """gp_img_encoder against the reference's own ImgEncoder (golden_img.npz, make_golden_img.py): the final
    (B, 256, 384) features, the layer-attention weights and the edge weights within 1e-5 of max|ref|; the
    patch -> point gather (roi pixels out of range included) bit-exact against the gathered golden rows
    and against numpy's take_along_axis of our own features."""
    import make_golden_img as mi
    from genpose2_amd import weights
    from genpose2_amd.img_encoder import ImgEncoderModel
    g = golden("img")
    B, scale, seed = mi.CASES[tag]
    model = ImgEncoderModel(weights.synthetic_state_dict("score_pointwise", seed=0), torch.device(DEV))
    model.set_arith(arith)   # the layer-attention Linear and the edge conv: split-f16 (default) or exact fp32
    layers = [torch.from_numpy(v).to(DEV) for v in mi.dino_layers(B, scale, seed)]
    final, parts = model.forward(layers, return_parts=True)
    f = final.cpu().numpy()
    errs = {"final0": rel(f[0], g[f"{tag}_final0"]), "edge": rel(parts["edge"].cpu().numpy(), g[f"{tag}_edge"]),
            "layer_w": rel(parts["layer_w"].cpu().numpy().transpose(0, 2, 1), g[f"{tag}_layer_w"]),
            "sum": float(np.abs(f.astype(np.float64).sum(axis=(1, 2)) - g[f"{tag}_final_sum"]).max()
                         / np.abs(g[f"{tag}_final_sum"]).max())}
    print(tag, arith, errs)
    assert max(errs.values()) < 1e-5, errs
    xs, ys = mi.roi_pixels(B, 1024, seed)
    got = model.gather(final, torch.from_numpy(xs), torch.from_numpy(ys)).cpu().numpy()
    pos = np.clip((xs // 14) * 16 + ys // 14, 0, 255)
    np.testing.assert_array_equal(got, np.take_along_axis(f, pos[..., None], 1))
    assert rel(got[0, :64], g[f"{tag}_gather0"]) < 1e-5


@pytest.mark.parametrize("B", [3, 40])
def test_img_encoder_implicit_im2col_vs_column_buffer(B):
    """gp_img_encoder3 (the edge conv's split GEMM gathering its im2col rows from the feature map, position-major
    planes) against gp_img_encoder2 (the formed column buffer, channel-major planes): the same products, the same
    per-row scaling (the row maxima are exact), summed in another order -- within 2e-6 of max|out| on the final
    features and the edge weights; with NULL planes (exact fp32) both run the same kernels: bit-identical."""
    import ctypes
    import make_golden_img as mi
    from genpose2_amd import _lib, weights
    from genpose2_amd.img_encoder import ImgEncoderModel
    lib = _lib.load()
    model = ImgEncoderModel(weights.synthetic_state_dict("score_pointwise", seed=0), torch.device(DEV))
    layers = [torch.from_numpy(v).to(DEV) for v in mi.dino_layers(B, 1.0, 77)]
    n, d = layers[0].shape[1], layers[0].shape[2]
    b2, gg, eg = (float(v) for v in model.scalars)
    t = model.t
    vp = lambda x: ctypes.c_void_p(None if x is None else x.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run(fn, conv_planes, split_la):
        need = max(int(lib.gp_img_encoder_workspace_size(B, n, d)), int(lib.gp_img_encoder3_workspace_size(B, n, d, 1)))
        ws = torch.empty(need, dtype=torch.uint8, device=DEV)
        out = torch.empty((B, n, d), device=DEV)
        edge = torch.empty((B, d // 4), device=DEV)
        _lib.check(fn(vp(layers[0]), vp(layers[1]), vp(layers[2]), B, n, d, vp(t["la_w1"]), vp(t["la_b1"]),
                      vp(t["la_w2"]), b2, vp(t["geo_table"]), vp(t["conv_w"]), vp(t["conv_b"]), gg, eg,
                      vp(t["la_w1_h"] if split_la else None), vp(conv_planes), vp(out), None, vp(edge), vp(ws),
                      ws.numel(), st), "img_encoder")
        return out.cpu().numpy(), edge.cpu().numpy()
    o2, e2 = run(lib.gp_img_encoder2, t["conv_w_h"], True)
    o3, e3 = run(lib.gp_img_encoder3, t["conv_w_hp"], True)
    assert rel(o3, o2) < 2e-6 and rel(e3, e2) < 2e-6, (rel(o3, o2), rel(e3, e2))
    assert not np.array_equal(e3, e2) or B < 4   # the implicit path ran (its K order rounds differently)
    f2, g2 = run(lib.gp_img_encoder2, None, False)
    f3, g3 = run(lib.gp_img_encoder3, None, False)
    np.testing.assert_array_equal(f3, f2)
    np.testing.assert_array_equal(g3, g2)


class _Backbone:
    def __init__(self, layers):
        self.layers = layers
        self.calls = 0

    def get_intermediate_layers(self, x, n, reshape, norm, return_class_token):
        assert list(n) == [2, 6, 11] and not reshape and norm and not return_class_token
        self.calls += 1
        return tuple(v[: x.shape[0]] for v in self.layers)


def test_pointwise_pred_func_end_to_end_vs_reference():
    """PoseNet(dino='pointwise').pred_func with the reference's keys (pts, pts_center, roi_xs, roi_ys, and the
    DINOv3 backbone's layers) against the reference's own pred_func run end to end (golden_img.npz e2e_*:
    ImgEncoder -> gather -> Pointnet2ClsMSGFus -> heads -> PC sampler, injected noise; the backbone replaced
    by fixed layers on both sides): pts_feat within 1e-5, rotation 1e-4, translation 1e-5 relative. The
    same call through a backbone object set on PoseNet.dino with roi_rgb gives the identical result."""
    import make_golden_img as mi
    from genpose2_amd import synthetic
    from genpose2_amd.agent import NoiseFeed, PoseNet
    from genpose2_amd.config import GenPoseConfig
    g = golden("img")
    e = mi.E2E
    B, N, K, T = e["B"], e["N"], e["K"], e["T"]
    pts, _ = synthetic.make_batch(e["cid"], B, N)
    xs, ys = mi.roi_pixels(B, N, e["seed"])
    layers = [torch.from_numpy(v).to(DEV) for v in mi.dino_layers(B, e["scale"], e["seed"])]
    agent = PoseNet(GenPoseConfig(device=DEV, sampling_steps=T, dino="pointwise")).eval()
    base = {"pts": torch.from_numpy(pts).to(DEV), "pts_center": torch.from_numpy(g["e2e_pts_center"]).to(DEV),
            "roi_xs": torch.from_numpy(xs), "roi_ys": torch.from_numpy(ys)}
    outs = []
    for how in ("layers", "backbone"):
        agent.noise_feed = NoiseFeed(*(torch.from_numpy(g[k]) for k in ("e2e_prior", "e2e_z1", "e2e_z2")))
        data = dict(base)
        if how == "layers":
            data["dino_layers"] = layers
        else:
            agent.dino = _Backbone(layers)
            data["roi_rgb"] = torch.zeros(B, 3, 224, 224, device=DEV)
        pose, q = agent.pred_func(data, repeat_num=K)
        outs.append((data["pts_feat"].clone(), pose.clone()))
        assert data["rgb_feat"] is None
    assert agent.dino.calls == 1
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    feat, pose = outs[0][0].cpu().numpy(), outs[0][1].cpu().numpy()
    ref = g["e2e_pred_pose"]
    print("e2e: pts_feat", rel(feat, g["e2e_pts_feat"]), "rotation", np.abs(pose[..., :6] - ref[..., :6]).max())
    assert rel(feat, g["e2e_pts_feat"]) < 1e-5
    assert np.abs(pose[..., :6] - ref[..., :6]).max() < 1e-4
    assert rel(pose[..., 6:], ref[..., 6:]) < 1e-5
    agent.dino = None
    with pytest.raises(KeyError):
        agent.pred_func(dict(base), repeat_num=K)


def _pointwise_case(case):
    import make_golden_img as mi
    from genpose2_amd import synthetic
    B, N = case["B"], case["N"]
    pts, _ = synthetic.make_batch(case["cid"], B, N)
    xs, ys = mi.roi_pixels(B, N, case["seed"])
    layers = [torch.from_numpy(v).to(DEV) for v in mi.dino_layers(B, case["scale"], case["seed"])]
    return pts, xs, ys, layers


def test_pointwise_b16_end_to_end_and_levels_vs_reference():
    """The larger pointwise case (golden_img_b16.npz: B=16, N=1024, K=50, T=20, R=800 rows; make_golden_img.py
    b16): the reference's pred_func end to end against PoseNet(dino='pointwise'), injected noise -- pts_feat
    within 1e-5 of max|ref| per object, rotation 1e-4, translation 1e-5 relative -- and the fused encoder's
    per-level outputs (SA output, transformer output, fused input of levels 1-4) of two objects at 1e-5."""
    import make_golden_img as mi
    from genpose2_amd.agent import NoiseFeed, PoseNet
    from genpose2_amd.config import GenPoseConfig
    g = golden("img_b16")
    e = mi.E2E16
    B, N, K, T = e["B"], e["N"], e["K"], e["T"]
    pts, xs, ys, layers = _pointwise_case(e)
    agent = PoseNet(GenPoseConfig(device=DEV, sampling_steps=T, dino="pointwise")).eval()
    prior, z1, z2 = mi.e2e_noise(e)
    agent.noise_feed = NoiseFeed(torch.from_numpy(prior), torch.from_numpy(z1), torch.from_numpy(z2))
    data = {"pts": torch.from_numpy(pts).to(DEV), "pts_center": torch.from_numpy(g["e2e_pts_center"]).to(DEV),
            "roi_xs": torch.from_numpy(xs), "roi_ys": torch.from_numpy(ys), "dino_layers": layers}
    pose, q = agent.pred_func(data, repeat_num=K)
    feat, p = data["pts_feat"].cpu().numpy(), pose.cpu().numpy()
    ref = g["e2e_pred_pose"]
    fe = np.abs(feat - g["e2e_pts_feat"]).max(1) / np.abs(g["e2e_pts_feat"]).max(1)
    rot = np.abs(p[..., :6] - ref[..., :6]).max()
    print(f"b16 e2e: pts_feat per-object max rel {fe.max():.2e}, rotation {rot:.2e}, translation rel "
          f"{rel(p[..., 6:], ref[..., 6:]):.2e}")
    assert fe.max() < 1e-5 and rot < 1e-4 and rel(p[..., 6:], ref[..., 6:]) < 1e-5
    # per-level outputs of the recorded objects, from the same per-point image features
    feat_img = agent.img_encoder.forward(layers)
    rgb = agent.img_encoder.gather(feat_img, torch.from_numpy(xs), torch.from_numpy(ys))
    out, levels = agent.encoder.forward(data["pts"], rgb, return_levels=True)
    torch.cuda.synchronize()
    assert torch.equal(out, data["pts_feat"])
    errs = {}
    for i, b in enumerate(g["level_objs"]):
        for lv in range(5):
            for k in ("sa", "tf", "fused"):
                if f"l{lv}_{k}" in g:
                    errs[(int(b), lv, k)] = rel(levels[lv][k][int(b)].cpu().numpy().T, g[f"l{lv}_{k}"][i])
    print("b16 per-level max rel", max(errs.values()))
    assert max(errs.values()) < 1e-5, {k: v for k, v in errs.items() if v >= 1e-5}


def test_pointwise_b256_batch_independence_and_properties():
    """The pointwise pipeline at the bench's full shape (B=256, N=1024, K=50; T=20 to keep the test short):
    the first 16 objects of the B=256 batch are the golden_img_b16 case itself, and their features equal the
    B=16 run's bit for bit (objects are independent; no kernel's per-object arithmetic depends on the batch),
    so the B=16 reference pin carries to the full batch; poses finite, rotations orthonormal, deterministic."""
    import make_golden_img as mi
    from genpose2_amd import synthetic
    from genpose2_amd.agent import PoseNet
    from genpose2_amd.config import GenPoseConfig
    e = mi.E2E16
    B, N, K, T = 256, e["N"], 50, 20
    pts16, xs16, ys16, layers16 = _pointwise_case(e)
    # objects 16..255: other clouds, pixels and layers
    pts_r, _ = synthetic.make_batch(e["cid"] + 1000, B - 16, N)
    rng = np.random.Generator(np.random.PCG64(e["seed"] + 77))
    xs = np.concatenate([xs16, rng.integers(-30, 250, size=(B - 16, N))])
    ys = np.concatenate([ys16, rng.integers(-30, 250, size=(B - 16, N))])
    layers = [torch.cat([l16, torch.from_numpy(rng.standard_normal((B - 16, 256, 384), dtype=np.float32) * 0.3).to(DEV)])
              for l16 in layers16]
    pts = np.concatenate([pts16, pts_r])
    agent = PoseNet(GenPoseConfig(device=DEV, sampling_steps=T, dino="pointwise", noise_seed=5)).eval()

    def run(sl, npts, nx, ny, lay):
        d = {"pts": torch.from_numpy(npts[sl]).to(DEV), "pts_center": torch.from_numpy(npts[sl].mean(1)).to(DEV),
             "roi_xs": torch.from_numpy(nx[sl]), "roi_ys": torch.from_numpy(ny[sl]), "dino_layers": [v[sl] for v in lay]}
        pose, q = agent.pred_func(d, repeat_num=K)
        return d["pts_feat"], pose, q
    f_all, p_all, q_all = run(slice(0, B), pts, xs, ys, layers)
    f16, _, _ = run(slice(0, 16), pts, xs, ys, layers)
    assert torch.equal(f_all[:16], f16)
    assert torch.isfinite(p_all).all() and torch.isfinite(q_all).all()
    r = p_all.reshape(-1, 9).double()
    assert (r[:, :3].norm(dim=1) - 1).abs().max() < 1e-5 and (r[:, 3:6].norm(dim=1) - 1).abs().max() < 1e-5
    assert (r[:, :3] * r[:, 3:6]).sum(1).abs().max() < 1e-5
    f_again, _, _ = run(slice(0, B), pts, xs, ys, layers)
    assert torch.equal(f_again, f_all)
