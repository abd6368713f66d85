"""The multi-device context (jt_create_multi: batches sharded over the listed GPUs, running
means reduced onto device 0 with one RCCL premultiplied-sum reduce inside jt_get_image).
On a one-GPU box the context runs over device 0 only, through the same launch / RCCL reduce
path: the weight is exactly 1, so everything must equal the single-device context bit for bit.
With two or more GPUs the combined image must equal the single-device one to fp32 rounding
(the weighting itself is restated on the oracle in tests/test_multi_weighting.py)."""
import ctypes as C

import numpy as np
import pytest

from conftest import make_params

pytestmark = pytest.mark.gpu


def _render(abi, lib, sa, p, nbatches, devices=None):
    from jtrace import trace
    st = trace.make_trace_state(sa, trace.make_scene_bvh(sa, False, lib), trace.make_trace_lights(sa, lib), p, lib,
                                devices=devices)
    st.set_counters(1)
    for _ in range(nbatches):
        st.trace_samples()
    out = (st.get_image(), st.get_aovs(), st.counters(), st.samples, st.describe())
    st.close()
    return out


@pytest.mark.parametrize("sampler", [1, 2])
def test_multi_context_on_one_device_equals_single(gpu, abi, lib, cornell_abi, sampler):
    p = make_params(abi, resolution=64, samples=6, batch=2, sampler=sampler)
    one = _render(abi, lib, cornell_abi, p, 3)
    multi = _render(abi, lib, cornell_abi, p, 3, devices=[0])
    assert "devices=1" in multi[4]
    assert one[3] == multi[3] == 6
    assert np.array_equal(one[0], multi[0])
    for a, b in zip(one[1], multi[1]):
        assert np.array_equal(a, b)
    for k in ("paths", "rays", "light_queries", "nodes", "instances", "prims", "shades"):
        assert one[2][k] == multi[2][k], k


def test_multi_context_over_all_devices(gpu, abi, lib, cornell_abi):
    if gpu < 2:
        pytest.skip(f"{gpu} GPU visible: the sharded path needs two (covered at N=1 and by the oracle restatement)")
    p = make_params(abi, resolution=64, samples=8, batch=3)
    one = _render(abi, lib, cornell_abi, p, 3)
    multi = _render(abi, lib, cornell_abi, p, 3, devices=list(range(min(gpu, 8))))
    np.testing.assert_allclose(multi[0], one[0], rtol=2e-5, atol=2e-6)
    assert np.array_equal(multi[1][2], one[1][2])
    for k in ("paths", "rays", "light_queries"):
        assert one[2][k] == multi[2][k], k


def test_multi_context_rejects_bad_device_lists(gpu, abi, lib, cornell_abi):
    from jtrace import trace
    p = make_params(abi, resolution=16, samples=1)
    sa = cornell_abi
    bvh, lights = trace.make_scene_bvh(sa, False, lib), trace.make_trace_lights(sa, lib)
    h = C.c_void_p()
    for devs in ([gpu], [0, 0] if gpu >= 2 else [0, 1], [-1]):
        arr = (C.c_int32 * len(devs))(*devs)
        st = lib.jt_create_multi(sa.ref, bvh.ref, lights.ref, C.byref(p), arr, len(devs), C.byref(h))
        assert st == -1, (devs, st, lib.jt_last_error())


@pytest.mark.parametrize("D", [2, 3, 8])
def test_tile_split_shares_sum_to_the_single_device_image(gpu, abi, lib, cornell_abi, D, options):
    """The tile split of jt_create_multi at batch < devices, reproduced on one GPU: contexts
    tracing every D-th 8x8 tile from offset d (option tile_share, the per-device launch parameters the
    multi-device context sets) at the reference's default --batch 1 each cover disjoint pixels,
    every one of them traces work, and their plain sum is the single-device image bit for bit."""
    p = make_params(abi, resolution=72, samples=3, batch=1)
    one = _render(abi, lib, cornell_abi, p, 3)
    img = np.zeros_like(one[0])
    alb = np.zeros_like(one[1][0])
    hits = np.zeros_like(one[1][2])
    paths = 0
    for d in range(D):
        options("tile_share", f"{D},{d}")
        part = _render(abi, lib, cornell_abi, p, 3)
        assert part[2]["paths"] > 0, d  # every device gets work at batch 1
        paths += part[2]["paths"]
        covered = np.any(part[0] != 0, axis=-1) | (part[1][2] != 0)
        assert not np.any(covered & np.any(img != 0, axis=-1)), d  # disjoint pixels
        img += part[0]
        alb += part[1][0]
        hits += part[1][2]
    assert paths == one[2]["paths"]
    assert np.array_equal(img, one[0])
    assert np.array_equal(alb, one[1][0])
    assert np.array_equal(hits, one[1][2])
