"""The C ABI driven the way a non-Python host would (cgo / JNI / C++), on a real MI355X: weights packed and
uploaded by gp_weights_pack from plain state-dict arrays, then the encoder, head projections and the PC
sampler called through the handle's structs. The packed bytes equal pack.py's (tests/test_cpu_host.py), so
results must equal PoseNet's bit for bit."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _vp(t):
    return ctypes.c_void_p(None if t is None else t.data_ptr())


def _pack(kind_id, sd):
    from genpose2_amd import _lib
    lib = _lib.load()
    keys = [k for k, v in sd.items() if v.dtype == np.float32]
    arrs = [np.ascontiguousarray(sd[k], np.float32) for k in keys]
    names = (ctypes.c_char_p * len(keys))(*[k.encode() for k in keys])
    data = (ctypes.c_void_p * len(keys))(*[a.ctypes.data for a in arrs])
    numel = np.array([a.size for a in arrs], np.int64)
    h = ctypes.c_void_p()
    _lib.check(lib.gp_weights_pack(kind_id, len(keys), ctypes.cast(names, ctypes.c_void_p),
                                   ctypes.cast(data, ctypes.c_void_p), numel.ctypes.data, ctypes.byref(h)),
               "weights_pack")
    return lib, h


def test_weights_pack_handle_drives_pc_pred_func():
    from genpose2_amd import _lib, arch, sde, synthetic, weights
    from genpose2_amd.agent import NoiseFeed, PoseNet
    from genpose2_amd.config import GenPoseConfig
    B, K, T = 3, 6, 20
    sd = weights.synthetic_state_dict("score")
    lib, h = _pack(0, sd)
    try:
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        pts_np, center_np = synthetic.make_batch(17, B, 1024)
        pts, center = torch.from_numpy(pts_np).to(DEV), torch.from_numpy(center_np).to(DEV)
        # encoder through the handle
        tab = _lib.c_int64_p()
        wbuf = lib.gp_weights_encoder(h, ctypes.byref(tab))
        assert wbuf
        ws = torch.empty(int(lib.gp_encoder_workspace_size(B, 1024)), dtype=torch.uint8, device=DEV)
        feat = torch.empty(B, 1024, device=DEV)
        _lib.check(lib.gp_encoder_forward(ctypes.c_void_p(wbuf), tab, _vp(pts), B, 1024, _vp(ws), ws.numel(),
                                          _vp(feat), s), "encoder_forward")
        # heads + PC sampler through the handle's gp_head_weights
        hw = lib.gp_weights_heads(h)
        pobj = torch.empty(B, 768, device=DEV)
        _lib.check(lib.gp_head_object_proj(hw, _vp(feat), B, _vp(pobj), s))
        tab_np = sde.pc_step_table(T)
        tvals = torch.from_numpy(np.ascontiguousarray(tab_np[:, 0])).to(DEV)
        tproj = torch.empty(T, 768, device=DEV)
        _lib.check(lib.gp_head_time_proj(hw, _vp(tvals), T, _vp(tproj), s))
        rng = np.random.default_rng(9)
        prior = rng.standard_normal((B * K, 9)).astype(np.float32)
        z1 = torch.from_numpy(rng.standard_normal((T, B * K, 9)).astype(np.float32)).to(DEV)
        z2 = torch.from_numpy(rng.standard_normal((T, B * K, 9)).astype(np.float32)).to(DEV)
        x = (torch.from_numpy(prior).to(DEV) * sde.prior_sigma(arch.SDE_T)).contiguous()   # as PoseNet.pred_func
        R = B * K
        res, q = torch.empty(R, 9, device=DEV), torch.empty(R, 7, device=DEV)
        pws = torch.empty(int(lib.gp_pc_workspace_size(R)), dtype=torch.uint8, device=DEV)
        stab = np.ascontiguousarray(tab_np, np.float32)
        _lib.check(lib.gp_pc_sample(hw, _vp(pobj), _vp(tproj), stab.ctypes.data_as(ctypes.c_void_p), T, _vp(x), R, K,
                                    _vp(center), _vp(z1), _vp(z2), ctypes.c_uint64(0), ctypes.c_float(arch.SNR),
                                    _vp(res), _vp(q), None, _vp(pws), pws.numel(), s), "pc_sample")
        torch.cuda.synchronize()
        # the same call through PoseNet (pack.py buffers)
        agent = PoseNet(GenPoseConfig(device=DEV, sampling_steps=T)).eval()
        agent.noise_feed = NoiseFeed(torch.from_numpy(prior), z1.cpu(), z2.cpu())
        data = {"pts": pts, "pts_center": center}
        pose, pq = agent.pred_func(data, repeat_num=K)
        torch.cuda.synchronize()
        assert torch.equal(feat, data["pts_feat"])
        assert torch.equal(res.view(B, K, 9), pose)
        assert torch.equal(q.view(B, K, 7), pq)
    finally:
        lib.gp_weights_free(h)


def test_weights_pack_scale_handle():
    from genpose2_amd import _lib, weights
    from genpose2_amd.device import ScaleModel
    sd = weights.synthetic_state_dict("scale")
    lib, h = _pack(2, sd)
    try:
        assert not lib.gp_weights_heads(h) and not lib.gp_weights_encoder(h, None)
        rng = np.random.default_rng(2)
        axes = torch.from_numpy(rng.normal(size=(4, 3, 3)).astype(np.float32)).to(DEV)
        feat = torch.from_numpy(rng.normal(size=(4, 1024)).astype(np.float32)).to(DEV)
        out = torch.empty(4, 3, device=DEV)
        _lib.check(lib.gp_scale_forward(lib.gp_weights_scale(h), _vp(axes), _vp(feat), 4, _vp(out),
                                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
        ref = ScaleModel(sd, torch.device(DEV)).forward(axes, feat)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
    finally:
        lib.gp_weights_free(h)
