"""The multi-device context's sharding and weighting (jt_create_multi, csrc/jt_trace.hip
multi_trace_range / multi_reduce), restated on the CPU oracle: every batch [s0, s1) of the
reference's batch loop (src/jtrace.jl:83-106) is split into contiguous per-device shares; device
d appends its share to its own running mean with weight 1/(n_d + k + 1) (the kernel's
1/(s - first + 1) with first = a - n_d), and reading the image combines sum_d mean_d * n_d / N.
This must equal the single-device running mean up to fp32 rounding, hits exactly.

When a batch has fewer samples than devices (the reference's default --batch 1), a sample split
would leave all but one device idle, so the context splits by pixels instead: 8x8 tile t goes to
device t mod D, which traces every sample of every batch on its tiles with the single-device
weights; the devices' pixels are disjoint (zero elsewhere) and the reduce is a plain sum.
`split_mode` / `tile_owner` restate jt_create_multi / the kernel's tile striding
(DParams tile_stride, tile_offset)."""
import numpy as np
import pytest

from conftest import make_params


def split_mode(batch, D):
    """jt_create_multi: tiles when params.batch < D."""
    return "tiles" if batch < D else "samples"


def tile_owner(W, H, D):
    """Device of every pixel under the tile split: 8x8 tile t = ty * tiles_x + tx on t mod D."""
    tiles_x = (W + 7) // 8
    j, i = np.mgrid[0:H, 0:W]
    return ((j // 8) * tiles_x + i // 8) % D


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


@pytest.mark.parametrize("D", [2, 3, 4, 5, 6, 7, 8])
def test_tile_split_at_batch_one_keeps_every_device_busy(abi, oracle, cornell_abi, D):
    """--batch 1 over D devices: every device traces every batch (on its tiles), and the sum of
    the devices' buffers is the single-device image exactly (disjoint pixels)."""
    S, W, H, batch = 3, 72, 40, 1
    assert split_mode(batch, D) == "tiles"
    p = make_params(abi, resolution=W, samples=S, width=W, height=H)
    bvh, lights = oracle.build_bvh(cornell_abi), oracle.make_lights(cornell_abi)
    single = oracle.trace(cornell_abi, bvh, lights, p, W, H, 0, S, nthreads=4)
    owner = tile_owner(W, H, D)
    work = np.zeros(D, np.int64)
    img = np.zeros((H, W, 4), np.float32)
    hits = np.zeros((H, W), np.int64)
    for d in range(D):
        st = (np.zeros((H, W, 4), np.float32), np.zeros((H, W, 3), np.float32), np.zeros((H, W, 3), np.float32),
              np.zeros((H, W), np.int64))
        for s0 in range(0, S, batch):  # every batch, all of its samples, first = 0
            oracle.trace(cornell_abi, bvh, lights, p, W, H, s0, s0 + batch, first=0, nthreads=4, state=st)
        mine = owner == d
        work[d] = int(mine.sum()) * S
        img += np.where(mine[..., None], st[0], 0)  # the device writes only its tiles
        hits += np.where(mine, st[3], 0)
    assert np.all(work > 0), work
    assert work.sum() == W * H * S
    assert np.array_equal(img, single[0])
    assert np.array_equal(hits, single[3])


def test_split_mode_follows_the_batch_size():
    assert split_mode(1, 8) == "tiles" and split_mode(7, 8) == "tiles"
    assert split_mode(8, 8) == "samples" and split_mode(256, 8) == "samples"
    # every device owns tiles of a 1280x720 frame, and the shares differ by at most one tile
    for D in range(2, 9):
        counts = np.bincount(tile_owner(1280, 720, D)[::8, ::8].ravel(), minlength=D)
        assert counts.min() > 0 and counts.max() - counts.min() <= 1
