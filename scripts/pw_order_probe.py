"""When do the two DINO-pointwise encoders of one step start on the GPU? (tuning aid, not a test)
The bench step's order: shared geometry on the launch stream, the EnergyNet encoder on a side stream after it,
the ScoreNet encoder on the launch stream. Prints host enqueue times and GPU event times (ms from the step's first
event) for 3 steps; run under rocprofv3 --kernel-trace to see which stream's kernels run when."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from genpose2_amd import synthetic  # noqa: E402
from genpose2_amd.agent import PoseNet  # noqa: E402
from genpose2_amd.config import GenPoseConfig  # noqa: E402


def main():
    B, N = 256, 1024
    dev = torch.device("cuda:0")
    cfg = GenPoseConfig(device="cuda:0", sampling_steps=500, dino="pointwise")
    score = PoseNet(cfg).eval()
    energy = PoseNet(cfg.copy(agent_type="energy")).eval()
    pts, center = synthetic.make_batch(4, B, N)
    rng = np.random.Generator(np.random.PCG64(4242))
    d0 = {"pts": torch.from_numpy(pts).to(dev), "pts_center": torch.from_numpy(center).to(dev),
          "dino_layers": [torch.from_numpy(rng.standard_normal((B, 256, 384), dtype=np.float32)).to(dev)
                          for _ in range(3)],
          "roi_xs": torch.from_numpy(rng.integers(0, 224, size=(B, N)).astype(np.int32)).to(dev),
          "roi_ys": torch.from_numpy(rng.integers(0, 224, size=(B, N)).astype(np.int32)).to(dev)}
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev)
    mode = sys.argv[1] if len(sys.argv) > 1 else "geometry"
    for it in range(4):
        torch.cuda.synchronize()
        ev = {k: torch.cuda.Event(enable_timing=True) for k in ("start", "geo", "energy_end", "score_pre", "score_end")}
        data, edata = dict(d0), dict(d0)
        h = {}
        t0 = time.perf_counter()
        ev["start"].record(main_s)
        if mode == "geometry":
            score.encode_geometry(data)
            edata["enc_geometry"] = data["enc_geometry"]
        ev["geo"].record(main_s)
        h["geo"] = time.perf_counter() - t0
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            energy.encode_func(edata)
            ev["energy_end"].record(side)
        h["energy_enqueued"] = time.perf_counter() - t0
        ev["score_pre"].record(main_s)
        score.encode_func(data)
        ev["score_end"].record(main_s)
        h["score_enqueued"] = time.perf_counter() - t0
        main_s.wait_stream(side)
        torch.cuda.synchronize()
        out = {k: round(ev["start"].elapsed_time(v), 3) for k, v in ev.items() if k != "start"}
        out.update({f"host_{k}": round(v * 1e3, 3) for k, v in h.items()})
        print(json.dumps({"step": it, "mode": mode, **out}))


if __name__ == "__main__":
    main()
