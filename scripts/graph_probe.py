"""PC sampler launched eagerly vs replayed from a captured HIP graph (tuning aid, not a test).

    python scripts/graph_probe.py [B] [K] [T]

The per-launch time (HIP events over the whole sampler / (T + 1)) of both, and whether the replayed graph reproduces
the eager run bit for bit (same seed, same inputs). With the trace build (GENPOSE_HIP_LIB=variants/trace/...) it also
prints the kernel-boundary gap of the last two launches from the in-kernel 100 MHz stamps.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import _lib, sde  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402


def boundary_ns(lib, T):
    if not hasattr(lib, "gp_debug_pc_trace"):
        return None
    fn = lib.gp_debug_pc_trace
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p]
    buf = np.zeros(3 * 256 * 8 * 20, np.uint64)
    assert fn(buf.ctypes.data) == 0
    tr = buf.reshape(3, 256, 8, 20).astype(np.int64)
    last, prev = tr[(T - 1) & 1], tr[(T - 2) & 1]
    valid = last[:, 0, 16] > 0
    return float(10 * (last[valid, :, 16].min() - prev[valid, :, 17].max()))


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 500
    dev = torch.device("cuda:0")
    lib = _lib.load()
    agent = PoseNet(GenPoseConfig(device="cuda:0", sampling_steps=T)).eval()
    h = agent.heads
    tab = sde.pc_step_table(T)
    tproj = h.time_proj(torch.from_numpy(tab[:, 0]).to(dev))
    pobj = h.object_proj(torch.rand(B, 1024, device=dev))
    center = torch.zeros(B, 3, device=dev)
    x0 = torch.randn(B * K, 9, device=dev) * 50
    x = x0.clone()
    out = {}

    def run():
        x.copy_(x0)
        return h.pc_sample(pobj, tproj, tab, x, K, center, seed=7)

    def timed(fn, reps=10):
        s = torch.cuda.current_stream()
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn()
            e1.record(s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts)) * 1e3 / (T + 1)

    res_e, q_e, _ = run()
    res_e, q_e = res_e.clone(), q_e.clone()
    out["eager_us_per_launch"] = timed(run)
    out["eager_boundary_ns"] = boundary_ns(lib, T)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run()   # warm: workspace allocated outside the capture
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            res_g, q_g, _ = run()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    out["graph_bit_identical"] = bool(torch.equal(res_g, res_e) and torch.equal(q_g, q_e))
    out["graph_us_per_launch"] = timed(g.replay)
    out["graph_boundary_ns"] = boundary_ns(lib, T)
    out["eager_us_per_launch_again"] = timed(run)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
