"""Golden fixtures of the DINO-pointwise fused encoder (Pointnet2ClsMSGFus), made by
running the REFERENCE's own module in this container.

The reference is imported exactly as tests/golden/make_golden.py does (off-path stubs, the four
PointNet++ CUDA ops replaced by the oracle's CPU restatement). ``Pointnet2ClsMSGFus(384)``
(networks/pts_encoder/pointnet2.py:255-388, attention.py) is built by the reference, loaded with the
seeded synthetic weights of ``genpose2_amd.weights.fus_encoder_manifest`` and run in eval mode on

* points: ``genpose2_amd.synthetic.make_batch(CID, B, 1024)``;
* per-point image features (the output of posenet.py:136-197's DINOv3 -> ImgEncoder -> gather,
  which needs weights absent here): ``rgb_features(B, N)``, a committed-seed PCG64 stream, so
  only the outputs are committed and the inputs are regenerated wherever the test runs.

Recorded: per level the SA output (before the transformer), the transformer output, the fused input
of levels 1..4, object 0 only; the level-3 relative-PE bias of object 0; the final (B, 1024); and the
state-dict layout (key -> shape) of the reference module.

Usage:  python tests/golden/make_golden_fus.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
sys.dont_write_bytecode = True

CID, B, N, FEAT_SEED = 71, 2, 1024, 7100


def rgb_features(b: int, n: int, seed: int = FEAT_SEED) -> np.ndarray:
    """(b, n, 384) float32: LayerNorm'ed-scale per-point features (DINO get_intermediate_layers(norm=True)
    -> ImgEncoder outputs are O(1)), from one PCG64 stream."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.standard_normal((b, n, 384), dtype=np.float32)


def main():
    import torch
    import make_golden as mg
    from genpose2_amd import synthetic, weights

    mg.import_reference("pc", 20)
    from networks.pts_encoder.pointnet2 import Pointnet2ClsMSGFus

    torch.manual_seed(0)
    enc = Pointnet2ClsMSGFus(384)
    sd = {k[len("pts_encoder."):]: v for k, v in weights.synthetic_state_dict("score_pointwise", seed=0).items()
          if k.startswith("pts_encoder.")}
    layout = {k: list(v.shape) for k, v in enc.state_dict().items()}
    enc.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    enc.eval()

    pts, _ = synthetic.make_batch(CID, B, N)
    feat = rgb_features(B, N)
    pc = torch.from_numpy(np.concatenate([pts, feat], axis=-1))

    rec = {}

    def hook(name):
        def f(mod, inp, out):
            rec[name] = out
        return f
    for i, m in enumerate(enc.SA_modules):
        m.register_forward_hook(hook(f"sa{i}"))
    for i, m in enumerate(enc.transformer_blocks):
        m.register_forward_hook(hook(f"tf{i}"))
    for i, m in enumerate(enc.feature_fusions):
        m.register_forward_hook(hook(f"fu{i + 1}"))
    enc.relative_pos_encoders[3].register_forward_hook(hook("bias3"))
    with torch.no_grad():
        out = enc(pc)
    res = {"feat": out.numpy()}
    for i in range(5):
        xyz, f_sa, idx = rec[f"sa{i}"]
        res[f"l{i}_sa"] = f_sa[0].numpy()            # (C, M) object 0
        res[f"l{i}_tf"] = rec[f"tf{i}"][0].numpy()   # (C, M)
        if i > 0:
            res[f"l{i}_fused"] = rec[f"fu{i}"][0].numpy()
        if idx is not None:
            res[f"l{i}_fps"] = idx.numpy()
    res["l3_bias"] = rec["bias3"][0].numpy()         # (8, 64, 64)
    np.savez_compressed(os.path.join(HERE, "golden_fus.npz"), **res)
    with open(os.path.join(HERE, "golden_fus_layout.json"), "w") as f:
        json.dump(layout, f, indent=0, sort_keys=True)
    print("fus done", out.shape, float(out.abs().max()))


if __name__ == "__main__":
    main()
