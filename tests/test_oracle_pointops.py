"""Known-answer tests pinning the oracle's point ops to the reference CUDA text.

The reference's CUDA ops cannot be run here (no nvcc/GPU), so each case is
computed by hand from sampling_gpu.cu:86-209 / ball_query_gpu.cu:9-45.
"""
import numpy as np
import pytest

from oracle import oracle


def test_fps_block_size_matches_opt_n_threads():
    lib = oracle._lib()
    # cuda_utils.h:9-13: min(2^floor(log2 n), 1024)
    for n, bs in [(1, 1), (3, 2), (4, 4), (6, 4), (512, 512), (1000, 512), (1024, 1024), (2048, 1024)]:
        assert lib.oracle_fps_block_size(n) == bs


def test_fps_tie_goes_to_lower_reduction_slot_not_lowest_index():
    # bs=4, one point per thread. After idx0=0: d = [0, 1, 1, .25]. Tree: slot0=(t0,t2)->i2,
    # slot1=(t1,t3)->i1, then slot0 vs slot1 tie keeps slot0 -> 2 (not 1).
    xyz = np.array([[[0, 0, 0], [1, 0, 0], [-1, 0, 0], [0, .5, 0]]], np.float32)
    assert oracle.furthest_point_sample(xyz, 3).tolist() == [[0, 2, 1]]


def test_fps_strict_greater_within_thread():
    # n=6 -> bs=4; thread 0 scans k=0,4, thread 1 scans k=1,5. All k>=1 tie at distance 1.
    # t0 best k4, t1 keeps k1 (strict >), t2 k2, t3 k3; tree -> k4.
    xyz = np.array([[[0, 0, 0], [1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1]]], np.float32)
    assert oracle.furthest_point_sample(xyz, 2).tolist() == [[0, 4]]


def _fps_by_key(xyz, m):
    """Layout-free statement of the same rule: max distance, ties -> min key where
    key = (bitrev_log2(bs)(k % bs), k // bs). This is what the HIP kernel implements."""
    n = xyz.shape[0]
    bs = oracle._lib().oracle_fps_block_size(n)
    nb = bs.bit_length() - 1

    def bitrev(v):
        return int(format(v, f"0{nb}b")[::-1], 2) if nb else 0

    keys = np.array([bitrev(k % bs) * (n // bs + 1) + k // bs for k in range(n)])
    temp = np.full(n, 1e10, np.float32)
    out, old = [0], 0
    for _ in range(1, m):
        d = xyz - xyz[old]
        d2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
        temp = np.minimum(temp, d2.astype(np.float32))
        best = temp.max()
        cand = np.nonzero(temp == best)[0]
        old = int(cand[np.argmin(keys[cand])])
        out.append(old)
    return out


@pytest.mark.parametrize("n", [6, 37, 64, 300, 1024, 1500])
def test_fps_key_rule_equals_serialised_cuda(n):
    rng = np.random.default_rng(n)
    xyz = rng.integers(0, 4, size=(n, 3)).astype(np.float32)  # integer grid: many exact ties
    m = min(n, 40)
    assert oracle.furthest_point_sample(xyz[None], m)[0].tolist() == _fps_by_key(xyz, m)


def test_ball_query_strict_radius_pad_with_first_and_zero_when_empty():
    xyz = np.array([[[5, 5, 5], [0.5, 0, 0], [9, 9, 9], [0.1, 0, 0], [0, 0.2, 0], [3, 3, 3],
                     [0, 0, 0.3], [0, 0, 0.4]]], np.float32)
    new_xyz = np.array([[[0, 0, 0], [100, 100, 100]]], np.float32)
    idx = oracle.ball_query(0.5, 4, xyz, new_xyz)
    # k=1 at exactly r (0.25 == r^2, not <) is excluded; hits 3,4,6,7 in order
    assert idx[0, 0].tolist() == [3, 4, 6, 7]
    assert idx[0, 1].tolist() == [0, 0, 0, 0]          # no hit: zero init kept
    idx = oracle.ball_query(0.25, 5, xyz, new_xyz)       # hits 3, 4 -> pad with first hit
    assert idx[0, 0].tolist() == [3, 4, 3, 3, 3]
    idx = oracle.ball_query(0.5, 2, xyz, new_xyz)        # break at nsample
    assert idx[0, 0].tolist() == [3, 4]


def test_group_and_gather_layouts():
    f = np.arange(2 * 3 * 5, dtype=np.float32).reshape(2, 3, 5)
    idx = np.array([[[4, 0], [1, 1]], [[2, 3], [0, 4]]], np.int32)
    g = oracle.grouping_operation(f, idx)
    assert g.shape == (2, 3, 2, 2)
    assert g[1, 2, 0, 1] == f[1, 2, 3]
    gi = oracle.gather_operation(f, np.array([[4, 1], [0, 2]], np.int32))
    assert gi[0, 1].tolist() == [f[0, 1, 4], f[0, 1, 1]]


def test_philox_known_answer_vectors():
    """Random123 kat_vectors for philox4x32 (10 rounds)."""
    from oracle import oracle
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in kat:
        got = oracle.philox4x32_10(np.array(ctr, np.uint64), np.array(key, np.uint64))
        assert [int(v) for v in got] == list(want)


def test_randn_restatement_statistics():
    from oracle import oracle
    z = oracle.randn(1234, 3, 20000, 9)
    assert abs(z.mean()) < 0.02 and abs(z.std() - 1) < 0.02
