"""HIP path vs the oracle on the reference's feature scenes, and the statistical pin of the HIP
path against the reference's own renders of them (images/<scene>_<sampler>.png, block means
committed in tests/golden/scene_pins.npz by tests/golden/scripts/make_scene_pins.py).

Scene coverage of SURVEY.md §8(a):
  features1  glossy/refractive/reflective, normal map (A22), HDR env light (A9/A10/A23), quads
  features2  config 3 (hairball/displacedsubdiv missing in the reference checkout: dropped)
  materials1 glossy + rough/delta reflective (A26/A27)
  materials2 refractive + transparent (A28/A29)
  materials4 volumetric + refractive with a volume stack (A11/A30)
  shapes1    quads of several BLAS shapes, textured matte/glossy
  bathroom1  config 4 (855 instances, 572 K triangles; 3 textures missing in the checkout:
             invalid_id, i.e. constant (1,1,1,1))
  ecosys     config 5 (12.7 K instances of 139 shapes; shape002/003 missing: dropped)
  coffee     complete scene: glossy, refractive glass, reflective metal (235 K triangles)
  staircase2 complete scene: glossy/reflective/refractive, textured (31 K triangles)
Tolerance as tests/test_gpu_parity.py (>= 99.9 % of pixels within 1e-3 relative; image mean
within 1e-4 relative).
"""
from pathlib import Path

import numpy as np
import pytest

from conftest import CORNELL, ROOT, compare_images, make_params

pytestmark = pytest.mark.gpu

SCENES = ("features1", "features2", "materials1", "materials2", "materials4", "shapes1", "bathroom1", "ecosys",
          "coffee", "staircase2")
# The reference renders of these scenes hold data the checkout lacks, so the pin is loose:
# (channel-mean rtol, block-median bound). features2: two dropped shapes; bathroom1: three
# missing textures rendered as constant (1,1,1,1) (the renders are ~6 % brighter); ecosys:
# two dropped shapes (the sky shows through where they stood: +20 % channel means, yet half of
# all blocks still match to 1 %).
INCOMPLETE = {"features2": (0.05, 0.02), "bathroom1": (0.08, 0.07), "ecosys": (0.25, 0.02)}
_cache = {}


def scene_abi(name):
    if name not in _cache:
        import warnings
        from jtrace import abi, sceneio
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            sc = sceneio.load_scene(str(ROOT / "assets" / "scenes" / name / f"{name}.json"), missing="drop")
        _cache[name] = abi.SceneABI(sc)
    return _cache[name]


def render_gpu(lib, sa, params, s0, s1, high_quality=False):
    from jtrace import trace
    bvh = trace.make_scene_bvh(sa, high_quality, lib)
    lights = trace.make_trace_lights(sa, lib)
    st = trace.make_trace_state(sa, bvh, lights, params, lib)
    st.trace_range(s0, s1)
    out = (st.get_image(), *st.get_aovs(), st.counters())
    st.close()
    return out


def render_oracle(oracle, sa, params, W, H, s0, s1, high_quality=False):
    ob = oracle.build_bvh(sa, high_quality)
    ol = oracle.make_lights(sa)
    return oracle.trace(sa, ob, ol, params, W, H, s0, s1)


def oracle_with(oracle, sa, params, W, H, s0, s1, **kw):
    """The oracle with a restated library option (e.g. env_alias=True)."""
    ob = oracle.build_bvh(sa)
    ol = oracle.make_lights(sa)
    return oracle.trace(sa, ob, ol, params, W, H, s0, s1, **kw)


def check_parity(g, o, label):
    stats = compare_images(g[0], o[0])
    print(label, stats, "gpu rays", g[4]["rays"], "oracle rays", o[4]["rays"])
    assert stats["frac_pix_rel_le_1e-3"] >= 0.999, (label, stats)
    assert stats["bitwise_frac"] >= 0.999, (label, stats)  # a silent 1-ulp regression shows here
    assert stats["image_mean_rel"] <= 1e-4, (label, stats)
    assert np.array_equal(g[3], o[3]), label  # hit counts
    for k in ("rays", "light_queries", "nodes", "instances", "prims", "shades"):
        assert abs(g[4][k] - o[4][k]) <= 1e-3 * o[4][k] + 8, (label, k, g[4][k], o[4][k])
    for a, b in ((g[1], o[1]), (g[2], o[2])):
        s = compare_images(a, b)
        assert s["frac_pix_rel_le_1e-3"] >= 0.999, (label, s)


@pytest.mark.parametrize("sampler", [1, 2])
@pytest.mark.parametrize("name", SCENES)
def test_scene_parity(gpu, abi, lib, oracle, name, sampler):
    sa = scene_abi(name)
    p = make_params(abi, resolution=120, samples=6, sampler=sampler)
    g = render_gpu(lib, sa, p, 0, 6)
    o = render_oracle(oracle, sa, p, g[0].shape[1], g[0].shape[0], 0, 6)
    check_parity(g, o, f"{name}/{sampler}")


@pytest.mark.parametrize("flags", [
    dict(tentfilter=True), dict(nocaustics=True), dict(envhidden=True), dict(clamp=2),
    dict(bounces=2), dict(bounces=16, sampler=2)])
def test_param_variants_parity(gpu, abi, lib, oracle, flags):
    name = "materials2" if "nocaustics" in flags else "features1"
    sa = scene_abi(name)
    p = make_params(abi, resolution=96, samples=4, **flags)
    g = render_gpu(lib, sa, p, 0, 4)
    o = render_oracle(oracle, sa, p, g[0].shape[1], g[0].shape[0], 0, 4)
    check_parity(g, o, f"{name}/{flags}")


def test_high_quality_bvh_parity(gpu, abi, lib, oracle):
    """--highqualitybvh (SAH build, src/bvh.jl:223-304): same host build on both sides."""
    sa = scene_abi("shapes1")
    p = make_params(abi, resolution=96, samples=4)
    g = render_gpu(lib, sa, p, 0, 4, high_quality=True)
    o = render_oracle(oracle, sa, p, g[0].shape[1], g[0].shape[0], 0, 4, high_quality=True)
    check_parity(g, o, "shapes1/sah")


@pytest.mark.parametrize("sampler", [1, 2])
@pytest.mark.parametrize("name", SCENES)
def test_statistical_pin_reference_render(gpu, abi, lib, name, sampler):
    """HIP render at the reference's size, 128 spp (naive: 1024), through the sRGB + 8-bit
    pipeline, vs the reference's own PNG on 41x40 / 40x40-pixel block means (this also pins the
    HDR decode, sceneio.HDR_MODE). The reference renders of INCOMPLETE scenes hold shapes or
    textures the checkout lacks: looser channel-mean and median bounds, no p95 bound."""
    from jtrace import sceneio
    pins = np.load(Path(__file__).parent / "golden" / "scene_pins.npz")
    key = f"{name}_{'path' if sampler == 1 else 'naive'}"
    w, h = (int(v) for v in pins[key + "_size"])
    bh, bw = (int(v) for v in pins[key + "_block"])
    sa = scene_abi(name)
    spp = 128 if sampler == 1 else 1024  # the naive sampler is far noisier; the 8-bit sRGB
    p = make_params(abi, resolution=1280, samples=spp, sampler=sampler, batch=spp)  # mean is
    img = render_gpu(lib, sa, p, 0, spp)[0]  # biased low by noise (concave encode)
    assert img.shape[:2] == (h, w)
    lin = sceneio.decode_srgb8(sceneio.to_srgb8(img, w, h))[..., :3]
    bm = lin.reshape(h // bh, bh, w // bw, bw, 3).mean(axis=(1, 3))
    ref = pins[key + "_mean"]
    cm = lin.reshape(-1, 3).mean(axis=0)
    rel = np.abs(bm - ref) / np.maximum(ref, 0.02)
    print(key, "channel mean", cm, "reference", pins[key + "_channel_mean"],
          "block rel median", np.median(rel), "p95", np.percentile(rel, 95))
    rtol, med = INCOMPLETE.get(name, (0.01, 0.01))
    np.testing.assert_allclose(cm, pins[key + "_channel_mean"], rtol=rtol)
    assert np.median(rel) < med
    if name not in INCOMPLETE:
        assert np.percentile(rel, 95) < 0.04


@pytest.mark.parametrize("name,ring", [("cornellbox", 1), ("shapes1", 2), ("bathroom1", 4)])
def test_stack_overflow_to_hbm_is_exact(gpu, abi, lib, options, name, ring):
    """The LDS stack ring spills its oldest entries to HBM and reloads them when popped: with a
    deliberately tiny ring (option test_lds_ring, test-only) every deep traversal overflows, and the
    image, AOVs and traversal counters must not change at all."""
    from jtrace import sceneio, trace
    sa = abi.SceneABI(sceneio.load_scene(CORNELL)) if name == "cornellbox" else scene_abi(name)
    p = make_params(abi, resolution=96, samples=3)
    bvh = trace.make_scene_bvh(sa, False, lib)
    lights = trace.make_trace_lights(sa, lib)
    outs = []
    for env in (None, str(ring)):
        if env is None:
            options("test_lds_ring", None)
        else:
            options("test_lds_ring", env)
        st = trace.make_trace_state(sa, bvh, lights, p, lib)
        st.trace_range(0, 3)
        outs.append((st.get_image(), st.get_aovs(), st.counters(), st.describe()))
        st.close()
    assert "hbm_overflow=1" in outs[1][3], outs[1][3]
    assert np.array_equal(outs[0][0], outs[1][0])
    for a, b in zip(outs[0][1], outs[1][1]):
        assert np.array_equal(a, b)
    for k in ("rays", "light_queries", "nodes", "instances", "prims", "shades"):
        assert outs[0][2][k] == outs[1][2][k], k


@pytest.mark.parametrize("name,mask", [("bathroom1", ",8363,"), ("ecosys", ",16571,"), ("features2", ",8383,")])
def test_mesh_specialisations_bitwise_equal(gpu, abi, lib, options, name, mask):
    """Configs 3-5 run the large-scene specialisations (FT_MESH, FT_MESH_ENV, FT_MESH_ENV_QUAD,
    HBM mode with the child pre-test; features2 with light-hit steps that defer environment pdf
    terms to the shading phase): the general FT_ALL kernel
    (option features=all) must give the same image, AOVs and traversal counters, bit for bit."""
    from jtrace import trace
    sa = scene_abi(name)
    p = make_params(abi, resolution=96, samples=2)
    bvh = trace.make_scene_bvh(sa, False, lib)
    lights = trace.make_trace_lights(sa, lib)
    outs = []
    for feat in ("auto", "all"):
        options("features", feat)
        st = trace.make_trace_state(sa, bvh, lights, p, lib)
        st.set_counters(1)
        st.trace_range(0, 2)
        outs.append((st.get_image(), st.get_aovs(), st.counters(), st.describe()))
        st.close()
    assert mask in outs[0][3] and ",255," in outs[1][3], (outs[0][3], outs[1][3])
    assert np.array_equal(outs[0][0], outs[1][0])
    for a, b in zip(outs[0][1], outs[1][1]):
        assert np.array_equal(a, b)
    for k in ("paths", "rays", "light_queries", "nodes", "instances", "prims", "shades"):
        assert outs[0][2][k] == outs[1][2][k], k


@pytest.mark.parametrize("name,lds", [("cornellbox", "65536"), ("cornellbox", "0"), ("bathroom1", None),
                                      ("features2", None), ("materials1", None)])
def test_inline_light_chains_bitwise_equal(gpu, abi, lib, options, name, lds):
    """Scenes whose instance lights are one-leaf shape BVHs run sample_lights_pdf's light chain
    inline in the shading phase (DScene::light_inline) instead of through the traversal loop and
    its light-hit steps. The same node/primitive steps in the same per-lane order: images, AOVs
    and every counter must be bit-identical to the traversal path (option light_inline=0), in the
    LDS-mode FT_NONE kernel (cornellbox), its HBM mode, and the mesh kernels."""
    from jtrace import sceneio, trace
    sa = abi.SceneABI(sceneio.load_scene(CORNELL)) if name == "cornellbox" else scene_abi(name)
    if lds is not None:
        options("lds_scene", lds)
    p = make_params(abi, resolution=96, samples=3)
    bvh = trace.make_scene_bvh(sa, False, lib)
    lights = trace.make_trace_lights(sa, lib)
    outs = []
    for inl in ("1", "0"):
        options("light_inline", inl)
        st = trace.make_trace_state(sa, bvh, lights, p, lib)
        st.set_counters(1)
        st.trace_range(0, 3)
        outs.append((st.get_image(), st.get_aovs(), st.counters(), st.describe()))
        st.close()
    assert "light_inline=1" in outs[0][3] and "light_inline=0" in outs[1][3], (outs[0][3], outs[1][3])
    assert outs[0][2]["light_queries"] > 0
    assert np.array_equal(outs[0][0], outs[1][0])
    for a, b in zip(outs[0][1], outs[1][1]):
        assert np.array_equal(a, b)
    for k in ("paths", "rays", "light_queries", "nodes", "instances", "prims", "shades"):
        assert outs[0][2][k] == outs[1][2][k], k


@pytest.mark.parametrize("name,order", [("bathroom1", "wide"), ("ecosys", "wide"), ("features2", "near")])
def test_hbm_scene_streams_match_the_oracle(gpu, abi, lib, oracle, options, name, order):
    """The HBM-mode specialisations in their auto traversal and 32 sample streams (the automatic
    count for features2/bathroom1 at their spp), in two calls whose second continues every
    stream's running mean from HBM, against the oracle's restatement of the same traversal,
    streams and combination: at the parity bar, hits and paths exact."""
    from jtrace import trace
    sa = scene_abi(name)
    options("streams", "32")
    w, h, s = 120, 68, 40
    p = make_params(abi, width=w, height=h, samples=s, batch=s, traversal=order)
    bvh = trace.make_scene_bvh(sa, False, lib)
    lights = trace.make_trace_lights(sa, lib)
    st = trace.make_trace_state(sa, bvh, lights, p, lib)
    assert st.streams == 32 and "mode=hbm" in st.describe() and f"traversal={order}" in st.describe(), st.describe()
    st.trace_range(0, 24)
    st.trace_range(24, s)
    g = (st.get_image(), *st.get_aovs(), st.counters())
    st.close()
    ob, ol = oracle.build_bvh(sa), oracle.make_lights(sa)
    parts = {}
    oracle.trace(sa, ob, ol, p, w, h, 0, 24, streams=32, parts=parts, nthreads=8)
    o = oracle.trace(sa, ob, ol, p, w, h, 24, s, streams=32, parts=parts, nthreads=8,
                     state=tuple(np.zeros(x.shape, x.dtype) for x in (g[0], g[1], g[2], g[3])))
    stats = compare_images(g[0], o[0])
    print(name, order, "32 streams", stats, "gpu", g[4], "oracle", o[4])
    assert stats["frac_pix_rel_le_1e-3"] >= 0.999 and stats["image_mean_rel"] <= 1e-4, stats
    assert stats["bitwise_frac"] >= 0.999, stats  # a silent 1-ulp regression shows here
    assert np.array_equal(g[3], o[3])
    for a, b in zip(g[1:3], o[1:3]):
        assert compare_images(a, b)["frac_pix_rel_le_1e-3"] >= 0.999
    assert g[4]["paths"] == w * h * s and o[4]["paths"] == w * h * (s - 24)  # the oracle counts its second call
