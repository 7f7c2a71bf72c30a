"""Encoder on a 56-CU masked stream beside the sampler on the other 200 CUs (tuning probe).

Usage: mask_probe.py [B] (default 256, config 4). Measured on MI355X (round 1, B=64): the sampler on a 200-CU masked stream takes 18.8 ms per 500 steps
against 10.6 ms unmasked (20.0 ms with one workgroup per CU forced), the encoder on 56 CUs 18.1 ms
against 2.8 ms: hipExtStreamCreateWithCUMask does not make batch pipelining pay on this part.
CU mask bit i maps to XCD i % 8 (then shader engine (i / 8) % 4).
Round 2, config 4 (B=256, 200 one-per-CU sampler workgroups): sampler 22.3 ms on 200 masked CUs against
11.8 ms unmasked with either mask layout ("linear" bits 0-199, "xcd" 25 bits per XCD); EnergyNet encoder
on the 56 others 25.5 ms (linear) / 13.0 ms (xcd) against 3.8 ms on all CUs (profiles/r2/mask_probe.json).
The masked sampler doubles, so the energy encoder stays beside the score encoder."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import sde, synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402


def masked_stream(first, count, layout="linear"):
    """CUs [first, first + count) of a 256-bit mask; layout "xcd": the same count per XCD taken as bits
    32x + j for j in [first/8, (first + count)/8) (an XCD-major reading of the mask)."""
    hip = ctypes.CDLL("libamdhip64.so")
    mask = (ctypes.c_uint32 * 8)()
    if layout == "linear":
        bits = range(first, first + count)
    else:
        bits = [32 * x + j for x in range(8) for j in range(first // 8, (first + count) // 8)]
    for b in bits:
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    pts, center = synthetic.make_batch(4, B, 1024)
    p = torch.from_numpy(pts).to(dev)
    c = torch.from_numpy(center).to(dev)
    layout = sys.argv[2] if len(sys.argv) > 2 else "linear"
    main_s, side_s = masked_stream(0, 200, layout), masked_stream(200, 56, layout)
    energy = PoseNet(GenPoseConfig(device="cuda:0", agent_type="energy")).eval()
    out = {}
    with torch.cuda.stream(side_s):
        out["enc_56cu_ms"] = ms(lambda: enc2.encoder.forward(p), side_s)
    with torch.cuda.stream(main_s):
        out["enc_200cu_ms"] = ms(lambda: agent.encoder.forward(p), main_s)
    out["enc_full_ms"] = ms(lambda: agent.encoder.forward(p), torch.cuda.current_stream())
    tab, tproj = agent._pc_table(500)
    feat = agent.encoder.forward(p)
    pobj = agent.heads.object_proj(feat)
    x0 = torch.randn(B * 50, 9, device=dev) * 50

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
        energy.encoder.forward(p)
        e3.record(side_s)
    torch.cuda.synchronize()
    out["concurrent_sampler_ms"] = e0.elapsed_time(e1)
    out["concurrent_encoder_ms"] = e2.elapsed_time(e3)
    out["layout"] = layout
    print(json.dumps(out))


if __name__ == "__main__":
    main()
