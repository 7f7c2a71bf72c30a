"""One-off check (not a test): the DINO-pointwise fused encoder (FusEncoderModel) on seeded points and per-point
features at B objects -- an output digest and the time per pass, for comparing library builds
(GENPOSE_HIP_LIB=... python scripts/fus_digest.py [B]). Prints one JSON line."""
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import synthetic, weights  # noqa: E402
from genpose2_amd.fus_encoder import FusEncoderModel  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dev = torch.device("cuda:0")
    pts_np, _ = synthetic.make_batch(4, B, 1024)
    pts = torch.from_numpy(pts_np).to(dev)
    rgb = torch.from_numpy(np.random.Generator(np.random.PCG64(1)).standard_normal((B, 1024, 384), dtype=np.float32)).to(dev)
    fus = FusEncoderModel(weights.synthetic_state_dict("score_pointwise"), dev)
    out = fus.forward(pts, rgb)
    torch.cuda.synchronize()
    digest = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    t0 = time.perf_counter()
    for _ in range(5):
        fus.forward(pts, rgb)
    torch.cuda.synchronize()
    print(json.dumps({"lib": os.environ.get("GENPOSE_HIP_LIB", "default"), "B": B, "digest": digest,
                      "ms_per_pass": (time.perf_counter() - t0) / 5 * 1e3}))


if __name__ == "__main__":
    main()
