"""Sampler (R=3200, T=500) and a concurrent encoder on a side stream (tuning probe, not a test).

Measured on MI355X (round 1): sampler alone 10.10 ms, encoder alone 2.52 ms; concurrently the
sampler takes 12.25 ms and the encoder 3.43 ms (wall 12.3 ms). With pc_step's LDS padded to 158 KB
per workgroup (no other workgroup fits beside it) the sampler still takes 12.4 ms: the encoder's
short-lived workgroups take the CUs at every sampler launch boundary, so the two serialise.
Batch pipelining (next batch's encoder beside this batch's sampler) therefore does not pay."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    agent = PoseNet(GenPoseConfig(device="cuda:0", sampling_steps=500)).eval()
    pts, center = synthetic.make_batch(2, 64, 1024)
    p = torch.from_numpy(pts).to(dev)
    c = torch.from_numpy(center).to(dev)
    tab, tproj = agent._pc_table(500)
    feat = agent.encoder.forward(p)
    pobj = agent.heads.object_proj(feat)
    x0 = torch.randn(3200, 9, device=dev) * 50
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream(device=dev)
    enc2 = PoseNet(GenPoseConfig(device="cuda:0")).eval()

    def samp():
        agent.heads.pc_sample(pobj, tproj, tab, x0.clone(), 50, c, seed=1)

    def timed(fn, stream, reps=3):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps
    out = {"sampler_ms": timed(samp, main_s)}
    with torch.cuda.stream(side):
        out["encoder_ms"] = timed(lambda: enc2.encoder.forward(p), side)
    res = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0, e1, e2, e3 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
        e0.record(main_s)
        samp()
        e1.record(main_s)
        side.wait_event(e0)
        with torch.cuda.stream(side):
            e2.record(side)
            enc2.encoder.forward(p)
            e3.record(side)
        torch.cuda.synchronize()
        res.append((e0.elapsed_time(e1), e2.elapsed_time(e3), (time.perf_counter() - t0) * 1e3))
    out["concurrent"] = [{"sampler_ms": a, "encoder_ms": b, "wall_ms": w} for a, b, w in res]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
