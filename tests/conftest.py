import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)
if GOLDEN not in sys.path:     # large_noise: inputs of the large-row fixtures, regenerated from seeds
    sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


# Arithmetic of the GPU kernels a parity test runs: "fast" = the defaults (head GEMMs in f16x3: three f16
# planes and six MFMA products, fp32-faithful; encoder SA levels 1-3 / token GEMMs in split-f16), "f32" = exact
# fp32 MFMA everywhere, "heads" = the f16x3 head GEMMs over the exact-fp32 encoder (isolates the head kernels'
# arithmetic against "f32").
ARITHS = ("fast", "f32")
ARITHS3 = ("fast", "heads", "f32")


def set_arith(agent, arith, encoder=None):
    """Sets `agent`'s head arithmetic and its encoder's (or `encoder`: "fast" | "f32", default the same)."""
    enc = ("f32" if arith == "heads" else arith) if encoder is None else encoder
    agent.heads.set_arith("f32" if arith == "f32" else "f16x3")
    if hasattr(agent.encoder, "set_arith"):
        agent.encoder.set_arith("split_f16" if enc == "fast" else "f32")
    if getattr(agent, "img_encoder", None) is not None:
        agent.img_encoder.set_arith("split_f16" if enc == "fast" else "f32")


def golden(name):
    return np.load(os.path.join(GOLDEN, f"golden_{name}.npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def score_sd():
    from genpose2_amd import weights
    return weights.synthetic_state_dict("score", seed=0)


@pytest.fixture(scope="session")
def energy_sd():
    from genpose2_amd import weights
    return weights.synthetic_state_dict("energy", seed=0)


@pytest.fixture(scope="session")
def scale_sd():
    from genpose2_amd import weights
    return weights.synthetic_state_dict("scale", seed=0)


def write_reference_checkpoint(path, kind, seed=0, prefix=""):
    """A checkpoint in the file format of the reference's PoseNet.save_ckpt (posenet_agent.py:141-169,
    pinned by golden_ckpt_layout.json): {clock, model_state_dict, optimizer_state_dict (Adam),
    scheduler_state_dict (ExponentialLR)}, holding the seeded synthetic weights of `kind`.
    prefix="module." mimics a DataParallel-wrapped net."""
    import torch
    from genpose2_amd import weights
    sd = {prefix + k: torch.from_numpy(v) for k, v in weights.synthetic_state_dict(kind, seed=seed).items()}
    params = [torch.nn.Parameter(torch.zeros(2))]
    opt = torch.optim.Adam(params, betas=(0.9, 0.999), eps=1e-8, lr=1e-3)
    sched = torch.optim.lr_scheduler.ExponentialLR(opt, 0.998)
    torch.save({"clock": {"epoch": 1, "minibatch": 0, "step": 0}, "model_state_dict": sd,
                "optimizer_state_dict": opt.state_dict(), "scheduler_state_dict": sched.state_dict()}, path)
    return path
