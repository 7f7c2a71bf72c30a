"""Encoder-only timing at the north-star batch: the Light encoder (gp_encoder_forward) and the DINO-pointwise
fused encoder (FusEncoderModel), B objects x N points, inputs resident in HBM. Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import synthetic, weights  # noqa: E402
from genpose2_amd.device import EncoderModel  # noqa: E402
from genpose2_amd.fus_encoder import FusEncoderModel  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda:0")
    pts_np, _ = synthetic.make_batch(4, B, 1024)
    pts = torch.from_numpy(pts_np).to(dev)
    rgb = torch.from_numpy(np.random.Generator(np.random.PCG64(1)).standard_normal((B, 1024, 384), dtype=np.float32)).to(dev)
    which = sys.argv[3] if len(sys.argv) > 3 else "both"
    out = {"B": B}
    if which in ("both", "light"):
        light = EncoderModel(weights.synthetic_state_dict("score"), dev)
        out["light_ms"] = timed(lambda: light.forward(pts), reps)
    if which in ("both", "fus"):
        fus = FusEncoderModel(weights.synthetic_state_dict("score_pointwise"), dev)
        out["fus_ms"] = timed(lambda: fus.forward(pts, rgb), reps)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
