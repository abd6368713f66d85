"""Edge cases of the HIP path against the oracle on the same seeded inputs (round 6).

- Ragged and tiny framings (`--width/--height` not multiples of the 8x8 tiles, down to one
  pixel), at one sample stream (the reference's `--batch 1`) and at k > 1 streams: the partial
  edge tiles, the stream-slot arithmetic and the persistent grid with fewer units than waves.
- A random instanced scene no shipped scene resembles: rotated and scaled instance frames (the
  instance-space ray transform of `intersect_instance_bvh`, src/bvh.jl:493-520), quads, degenerate
  triangles, glossy and matte materials and emissive instances as lights, in both scene modes (LDS
  and HBM) and every traversal order, both samplers.

The bar is §8(c)'s (tests/test_gpu_parity.py): >= 99.9 % of pixels bit-identical and within 1e-3,
image mean within 1e-4, hits equal, traversal counters within 0.1 %.
"""
import numpy as np
import pytest

from conftest import compare_images, make_params
from jtrace.scene import CameraData, InstanceData, MaterialData, SceneData, ShapeData

pytestmark = pytest.mark.gpu

ORDERS = {"reference": 0, "near": 1, "wide": 2}


def _both(abi, lib, oracle, sa, params, s0, s1, options=None, lds=None):
    from jtrace import trace
    if options is not None and lds is not None:
        options("lds_scene", lds)
    bvh = trace.make_scene_bvh(sa, False, lib)
    lights = trace.make_trace_lights(sa, lib)
    st = trace.make_trace_state(sa, bvh, lights, params, lib)
    st.trace_range(s0, s1)
    g = (st.get_image(), *st.get_aovs(), st.counters())
    k, desc = st.streams, st.describe()
    st.close()
    o = oracle.trace(sa, oracle.build_bvh(sa), oracle.make_lights(sa), params, g[0].shape[1], g[0].shape[0],
                     s0, s1, streams=k)
    return g, o, k, desc


def _check(g, o, label):
    stats = compare_images(g[0], o[0])
    print(label, stats, "gpu", g[4], "oracle", o[4])
    assert stats["frac_pix_rel_le_1e-3"] >= 0.999, (label, stats)
    assert stats["bitwise_frac"] >= 0.999, (label, stats)
    assert stats["image_mean_rel"] <= 1e-4, (label, stats)
    assert np.array_equal(g[3], o[3]), label  # hit counts
    for key in ("rays", "light_queries", "nodes", "instances", "prims", "shades"):
        assert abs(g[4][key] - o[4][key]) <= 1e-3 * o[4][key] + 8, (label, key, g[4][key], o[4][key])
    for a, b in ((g[1], o[1]), (g[2], o[2])):
        assert compare_images(a, b)["frac_pix_rel_le_1e-3"] >= 0.999, label


@pytest.mark.parametrize("batch", [1, 7])
@pytest.mark.parametrize("w,h", [(1, 1), (1, 13), (13, 1), (9, 7), (17, 33), (65, 3)])
def test_ragged_framings_match_the_oracle(gpu, abi, lib, oracle, cornell_abi, w, h, batch):
    """Framings smaller than a tile or one pixel past a tile boundary: every pixel is traced once
    (paths = W*H*spp), edge tiles skip their outside pixels, and the bits equal the oracle's."""
    params = make_params(abi, width=w, height=h, samples=7, batch=batch)
    g, o, k, desc = _both(abi, lib, oracle, cornell_abi, params, 0, 7)
    assert g[0].shape[:2] == (h, w), g[0].shape
    assert k == (1 if batch == 1 else 4), desc  # k <= the batch (stream_log2)
    assert g[4]["paths"] == o[4]["paths"] == w * h * 7
    _check(g, o, f"{w}x{h}/batch{batch}/k{k}")
    # the bits do not depend on how the range is split into calls
    from jtrace import trace
    st = trace.make_trace_state(cornell_abi, trace.make_scene_bvh(cornell_abi, False, lib),
                                trace.make_trace_lights(cornell_abi, lib), params, lib)
    for a, b in ((0, 2), (2, 3), (3, 7)):
        st.trace_range(a, b)
    assert np.array_equal(st.get_image(), g[0])
    st.close()


def _rotation(rng):
    q, r = np.linalg.qr(rng.normal(size=(3, 3)))
    return q * np.sign(np.diag(r))


def random_instanced_scene(seed=7):
    """Random geometry in front of the camera: three shapes (triangles, quads with degenerate
    ones, a sliver-heavy triangle soup), six instances with rotated and non-uniformly scaled
    frames, two of them emissive (the lights), matte and glossy materials."""
    rng = np.random.default_rng(seed)
    sc = SceneData()
    cam = np.array([1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 12], np.float32)
    sc.cameras.append(CameraData(frame=cam, aspect=np.float32(1.0)))
    sc.materials += [
        MaterialData(color=np.array([0.7, 0.6, 0.5], np.float32)),
        MaterialData(type="glossy", color=np.array([0.4, 0.5, 0.8], np.float32), roughness=np.float32(0.3)),
        MaterialData(emission=np.array([6, 5, 4], np.float32), color=np.zeros(3, np.float32)),
    ]
    # shape 0: a triangle soup around the origin. The scene is small enough for the LDS blob
    # (jt_create takes LDS mode only if it keeps 4 workgroups per CU: about 6 KiB of scene here)
    n = 10
    c = rng.normal(size=(n, 1, 3)) * 1.5
    pos = (c + rng.normal(size=(n, 3, 3)) * 0.4).reshape(-1, 3).astype(np.float32)
    sc.shapes.append(ShapeData(positions=pos, triangles=np.arange(3 * n, dtype=np.int32).reshape(n, 3)))
    # shape 1: quads, every third a triangle stored as a degenerate quad (p3 == p4)
    n = 5
    c = rng.normal(size=(n, 1, 3))
    pos = (c + rng.normal(size=(n, 4, 3)) * 0.5).reshape(-1, 3).astype(np.float32)
    idx = np.arange(4 * n, dtype=np.int32).reshape(n, 4)
    idx[::3, 3] = idx[::3, 2]
    sc.shapes.append(ShapeData(positions=pos, quads=idx))
    # shape 2: a small two-triangle emitter (one BVH leaf: light chains inline)
    pos = np.array([[-0.5, -0.5, 0], [0.5, -0.5, 0], [0.5, 0.5, 0], [-0.5, 0.5, 0]], np.float32)
    sc.shapes.append(ShapeData(positions=pos, triangles=np.array([[0, 1, 2], [0, 2, 3]], np.int32)))
    for i in range(6):
        shape = 2 if i in (2, 5) else i % 2
        m = _rotation(rng) * rng.uniform(1.0, 3.0, size=3)  # rotated, non-uniformly scaled axes
        o = rng.uniform(-4, 4, size=3)
        o[2] = rng.uniform(-6, 2)
        frame = np.concatenate([m.reshape(-1), o]).astype(np.float32)
        sc.instances.append(InstanceData(frame=frame, shape=shape, material=2 if shape == 2 else i % 2))
    return sc


@pytest.fixture(scope="module")
def random_abi(abi):
    return abi.SceneABI(random_instanced_scene())


@pytest.mark.parametrize("sampler", [1, 2])
@pytest.mark.parametrize("order", ["near", "wide", "reference"])
@pytest.mark.parametrize("mode", ["lds", "hbm"])
def test_random_instanced_scene_matches_the_oracle(gpu, abi, lib, oracle, options, random_abi, mode, order, sampler):
    params = make_params(abi, resolution=80, samples=6, batch=6, sampler=sampler, traversal=order)
    g, o, k, desc = _both(abi, lib, oracle, random_abi, params, 0, 6, options=options,
                          lds="0" if mode == "hbm" else None)
    assert (f"mode={mode}" in desc) and (f"traversal={order}" in desc), desc
    assert g[3].sum() > 0 and g[0][..., :3].mean() > 0, "the scene must be hit and lit"
    _check(g, o, f"random/{mode}/{order}/{sampler}/k{k}")
