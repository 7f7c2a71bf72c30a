"""Phase breakdown of pc_step_kernel from in-kernel s_memtime marks (tuning aid, not a test).

Needs the trace build of the library (built here, travels with the snapshot):
    make -C genpose2_amd/csrc OUT=../../variants/trace/libgenpose_hip.so BUILD=../../variants/trace/build EXTRA=-DPC_TRACE
    GENPOSE_HIP_LIB=variants/trace/libgenpose_hip.so python scripts/pc_trace.py [B] [K]
Marks (per wave): 0 start, 1 after the PC update + barrier, 2 after pose_encoder.0 + barrier, 3 after the
pose_encoder.2 stream, 4 after its epilogue + barrier, 5 after the head-layer-1 stream, 6 after the layer-2
partials + barrier, 7 after the head output, 8 end. Slots 16 / 17 hold the constant 100 MHz clock at marks 0 / 8
(one time base for the whole chip: the per-workgroup start / end histogram and the shader clock each workgroup
ran at), 18 the HW_ID register and the XCC id.
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


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 500
    warm_s = float(sys.argv[4]) if len(sys.argv) > 4 else 2.0   # back-to-back calls first: the clock settles under load
    dev = torch.device("cuda:0")
    lib = _lib.load()
    fn = lib.gp_debug_pc_trace
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p]
    agent = PoseNet(GenPoseConfig(device="cuda:0", sampling_steps=T)).eval()
    tab = sde.pc_step_table(T)
    tproj = agent.heads.time_proj(torch.from_numpy(tab[:, 0]).to(dev))
    pobj = agent.heads.object_proj(torch.rand(B, 1024, device=dev))
    center = torch.zeros(B, 3, device=dev)
    x0 = torch.randn(B * K, 9, device=dev) * 50
    import time
    t_end = time.time() + warm_s
    n = 0
    while n < 3 or time.time() < t_end:
        agent.heads.pc_sample(pobj, tproj, tab, x0.clone(), K, center, seed=1)
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    S = 20
    buf = np.zeros(3 * 256 * 8 * S, np.uint64)
    assert fn(buf.ctypes.data) == 0
    tile = int(lib.gp_pc_tile_rows(B * K, int(agent.heads.arith == "f16x3")))
    nwg = min((B * K + tile - 1) // tile, 256)
    tr = buf.reshape(3, 256, 8, S)[(T - 1) & 1, :nwg, :, :9].astype(np.int64)
    t0 = tr[:, :, 0].min()
    d = np.diff(tr, axis=-1)                       # (wg, wave, 8)
    names = ["update", "pe0", "pe2_stream", "pe2_epi+bar", "h1_stream", "l2+bar", "f", "s+norm"]
    out = {"B": B, "K": K, "T": T, "calls": n, "nwg": int(nwg),
           "phase_cycles_mean": {n: float(d[..., j].mean()) for j, n in enumerate(names)},
           "phase_cycles_max": {n: float(d[..., j].max()) for j, n in enumerate(names)},
           "wg_start_spread_cycles": float(tr[:, :, 0].min(1).max() - t0),
           "wg_end_max_cycles": float(tr[:, :, 8].max() - t0),
           "wg_lifetime_mean_cycles": float((tr[:, :, 8].max(1) - tr[:, :, 0].min(1)).mean())}
    # workgroup critical path: the last wave past each barrier
    st = tr[:, :, 0].min(1)
    crit = {"update+bar1": tr[:, :, 1].max(1) - st,
            "pe0+bar2": tr[:, :, 2].max(1) - tr[:, :, 1].max(1),
            "pe2+epi+bar4": tr[:, :, 4].max(1) - tr[:, :, 2].max(1),
            "h1 (last wave)": tr[:, :, 5].max(1) - tr[:, :, 4].max(1),
            "tail (l2, bar, s)": tr[:, :, 8].max(1) - tr[:, :, 5].max(1)}
    out["critical_path_mean"] = {k: float(v.mean()) for k, v in crit.items()}
    w0 = buf.reshape(3, 256, 8, S)[(T - 1) & 1, :nwg, 0, :].astype(np.int64)
    seq = [0, 9, 10, 11, 12, 1]
    out["wave0_update_cycles_mean"] = {f"{a}->{b}": float((w0[:, b] - w0[:, a]).mean()) for a, b in zip(seq, seq[1:])}
    # launch-to-launch: launch T-2's last wave end -> launch T-1's first wave start (same clock domain
    # only if s_memtime agrees across XCDs; reported per XCD = blockIdx % 8 as well)
    prev = buf.reshape(3, 256, 8, S)[(T - 2) & 1, :nwg, :, :9].astype(np.int64)
    out["gap_prev_end_to_start_cycles"] = float(tr[:, :, 0].min() - prev[:, :, 8].max())
    out["gap_per_xcd"] = [float(tr[x::8, :, 0].min() - prev[x::8, :, 8].max()) for x in range(8)]
    out["launch_span_cycles"] = float(tr[:, :, 8].max() - tr[:, :, 0].min())
    full = buf.reshape(3, 256, 8, S)[(T - 1) & 1, :nwg, :, :].astype(np.int64)
    # head layer 1 head by head (marks 4 -> 13 -> 14 -> 5): per wave index (mean over workgroups) and the
    # spread between a workgroup's fastest and slowest wave
    for nm, (a, b) in {"head0": (4, 13), "head1": (13, 14), "head2": (14, 5)}.items():
        if full[..., b].any():
            dd = full[..., b] - full[..., a]                  # (wg, wave)
            out.setdefault("h1_heads_per_wave_mean", {})[nm] = [round(float(v)) for v in dd.mean(0)]
            out.setdefault("h1_heads_spread_mean", {})[nm] = float((dd.max(1) - dd.min(1)).mean())
    h1 = full[..., 5] - full[..., 4]
    out["h1_per_wave_mean"] = [round(float(v)) for v in h1.mean(0)]
    out["h1_end_spread_mean"] = float((full[..., 5].max(1) - full[..., 5].min(1)).mean())
    out["h1_start_spread_mean"] = float((full[..., 4].max(1) - full[..., 4].min(1)).mean())
    # ---- one chip-wide time base (s_memrealtime, 100 MHz): workgroup start / end histogram, kernel boundary
    for nm, slot in (("last", (T - 1) & 1), ("prev", (T - 2) & 1)):
        rt = buf.reshape(3, 256, 8, S)[slot, :nwg, :, :].astype(np.int64)
        out.setdefault("realtime", {})[nm] = _realtime(rt, nwg)
    last = buf.reshape(3, 256, 8, S)[(T - 1) & 1, :nwg, :, :].astype(np.int64)
    prev = buf.reshape(3, 256, 8, S)[(T - 2) & 1, :nwg, :, :].astype(np.int64)
    out["realtime"]["boundary_prev_last_end_to_first_start_ns"] = float(10 * (last[:, :, 16].min() - prev[:, :, 17].max()))
    print(json.dumps(out, indent=1))


def _realtime(rt, nwg):
    """Per-workgroup start / end on the 100 MHz clock (ns from the launch's first start), the shader clock each
    workgroup ran at (its s_memtime span over its s_memrealtime span) and the XCC / CU it ran on."""
    st = rt[:, :, 16].min(1)
    en = rt[:, :, 17].max(1)
    t0 = st.min()
    cyc = rt[:, :, 8].max(1) - rt[:, :, 0].min(1)
    ghz = cyc / np.maximum(en - st, 1) / 10.0          # cycles per 10 ns tick / 10 = GHz
    xcc = (rt[:, 0, 18] >> 32) & 0xF
    hw = rt[:, 0, 18] & 0xFFFFFFFF
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    start_ns, end_ns = 10 * (st - t0), 10 * (en - t0)
    pct = lambda v: {p: float(np.percentile(v, p)) for p in (0, 10, 50, 90, 100)}
    return {
        "span_ns": float(end_ns.max()),
        "start_ns_pct": pct(start_ns), "end_ns_pct": pct(end_ns), "lifetime_ns_pct": pct(end_ns - start_ns),
        "shader_ghz_pct": pct(ghz),
        "start_hist_ns": np.histogram(start_ns, bins=8)[0].tolist(), "start_hist_edges": np.histogram(start_ns, bins=8)[1].round().tolist(),
        "end_hist_ns": np.histogram(end_ns, bins=8)[0].tolist(), "end_hist_edges": np.histogram(end_ns, bins=8)[1].round().tolist(),
        "per_xcc": {int(x): {"wgs": int((xcc == x).sum()), "start_ns_max": float(start_ns[xcc == x].max()),
                             "end_ns_min": float(end_ns[xcc == x].min()), "end_ns_max": float(end_ns[xcc == x].max()),
                             "ghz_mean": float(ghz[xcc == x].mean())} for x in sorted(set(xcc.tolist()))},
        "distinct_cu": int(len(set(zip(xcc.tolist(), se.tolist(), cu.tolist(), ((hw >> 12) & 1).tolist())))),
        "latest_start_wgs": np.argsort(-start_ns)[:8].tolist(), "latest_end_wgs": np.argsort(-end_ns)[:8].tolist(),
        "wg_start_end_ns": [[int(a), int(b)] for a, b in zip(start_ns, end_ns)],
    }


if __name__ == "__main__":
    main()
