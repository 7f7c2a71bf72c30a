"""Encoder on a 56-CU masked stream beside the sampler on the other 200 CUs (tuning probe).

Measured on MI355X (round 1): the sampler on a 200-CU masked stream takes 18.8 ms per 500 steps
against 10.6 ms unmasked (20.0 ms with one workgroup per CU forced), the encoder on 56 CUs 18.1 ms
against 2.8 ms: hipExtStreamCreateWithCUMask does not make batch pipelining pay on this part.
CU mask bit i maps to XCD i % 8 (then shader engine (i / 8) % 4)."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import sde, synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402


def masked_stream(first, count):
    hip = ctypes.CDLL("libamdhip64.so")
    mask = (ctypes.c_uint32 * 8)()
    for b in range(first, first + count):
        mask[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), 8, mask) == 0
    return torch.cuda.ExternalStream(s.value)


def ms(fn, stream, reps=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    agent = PoseNet(GenPoseConfig(device="cuda:0", sampling_steps=500)).eval()
    enc2 = PoseNet(GenPoseConfig(device="cuda:0", sampling_steps=500)).eval()
    pts, center = synthetic.make_batch(2, 64, 1024)
    p = torch.from_numpy(pts).to(dev)
    c = torch.from_numpy(center).to(dev)
    main_s, side_s = masked_stream(0, 200), masked_stream(200, 56)
    out = {}
    with torch.cuda.stream(side_s):
        out["enc_56cu_ms"] = ms(lambda: enc2.encoder.forward(p), side_s)
    with torch.cuda.stream(main_s):
        out["enc_200cu_ms"] = ms(lambda: agent.encoder.forward(p), main_s)
    out["enc_full_ms"] = ms(lambda: agent.encoder.forward(p), torch.cuda.current_stream())
    tab, tproj = agent._pc_table(500)
    feat = agent.encoder.forward(p)
    pobj = agent.heads.object_proj(feat)
    x0 = torch.randn(3200, 9, device=dev) * 50

    def samp():
        agent.heads.pc_sample(pobj, tproj, tab, x0.clone(), 50, c, seed=1)
    with torch.cuda.stream(main_s):
        out["sampler_200cu_ms"] = ms(samp, main_s)
    out["sampler_full_ms"] = ms(samp, torch.cuda.current_stream())
    # both at once
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(main_s):
        e0.record(main_s)
        samp()
        e1.record(main_s)
    with torch.cuda.stream(side_s):
        e2.record(side_s)
        enc2.encoder.forward(p)
        e3.record(side_s)
    torch.cuda.synchronize()
    out["concurrent_sampler_ms"] = e0.elapsed_time(e1)
    out["concurrent_encoder_ms"] = e2.elapsed_time(e3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
