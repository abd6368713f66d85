"""The multi-device context's sharding and weighting (jt_create_multi, csrc/jt_trace.hip
multi_trace_range / multi_reduce), restated on the CPU oracle: every batch [s0, s1) of the
reference's batch loop (src/jtrace.jl:83-106) is split into contiguous per-device shares; device
d appends its share to its own running mean with weight 1/(n_d + k + 1) (the kernel's
1/(s - first + 1) with first = a - n_d), and reading the image combines sum_d mean_d * n_d / N.
This must equal the single-device running mean up to fp32 rounding, hits exactly."""
import numpy as np
import pytest

from conftest import make_params


def shares(s0, s1, D):
    L = s1 - s0
    return [(s0 + L * d // D, s0 + L * (d + 1) // D) for d in range(D)]


@pytest.mark.parametrize("D,batch", [(2, 1), (3, 2), (4, 3), (8, 5)])
def test_sharded_running_means_combine_to_the_single_device_image(abi, oracle, cornell_abi, D, batch):
    S, W, H = 12, 24, 24
    p = make_params(abi, resolution=W, samples=S)
    bvh, lights = oracle.build_bvh(cornell_abi), oracle.make_lights(cornell_abi)
    single = oracle.trace(cornell_abi, bvh, lights, p, W, H, 0, S, nthreads=4)
    states = [(np.zeros((H, W, 4), np.float32), np.zeros((H, W, 3), np.float32), np.zeros((H, W, 3), np.float32),
               np.zeros((H, W), np.int64)) for _ in range(D)]
    n = [0] * D
    for s0 in range(0, S, batch):
        s1 = min(s0 + batch, S)
        for d, (a, b) in enumerate(shares(s0, s1, D)):
            if a < b:
                oracle.trace(cornell_abi, bvh, lights, p, W, H, a, b, first=a - n[d], nthreads=4, state=states[d])
                n[d] += b - a
    assert sum(n) == S
    N = float(sum(n))
    w = [np.float32(k / N) for k in n]
    img = sum(st[0].astype(np.float64) * wk for st, wk in zip(states, w))
    alb = sum(st[1].astype(np.float64) * wk for st, wk in zip(states, w))
    hits = sum(st[3] for st in states)
    np.testing.assert_allclose(img, single[0], rtol=2e-5, atol=2e-6)
    np.testing.assert_allclose(alb, single[1], rtol=2e-5, atol=2e-6)
    assert np.array_equal(hits, single[3])


def test_shares_cover_every_batch_in_order():
    for D in (1, 2, 3, 8):
        for s0, s1 in ((0, 1), (5, 12), (0, 256)):
            sh = shares(s0, s1, D)
            assert sh[0][0] == s0 and sh[-1][1] == s1
            assert all(sh[k][1] == sh[k + 1][0] for k in range(D - 1))
