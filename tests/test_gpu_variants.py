"""HIP path vs the oracle on synthetic variants of cornellbox that reach branches no shipped
config scene takes (VERDICT r01 "What's missing" 4):
  - thin lens, aperture > 0: eval_camera's lens sample through sample_disk
    (src/scene.jl:372-411, src/sampling.jl:12-16) instead of the pinhole sign shortcut;
  - the orthographic camera branch of eval_camera;
  - vertex colours: eval_color's barycentric interpolation (src/scene.jl:690-720), multiplying
    the material colour, and its alpha entering the opacity (src/scene.jl:649) — with alphas
    below 1 the opacity draw and the opacity retry (src/trace.jl:336-345) run too.
Same bar as tests/test_gpu_parity.py.
"""
import copy

import numpy as np
import pytest

from conftest import compare_images, make_params

pytestmark = pytest.mark.gpu


def _parity(abi, lib, oracle, scene, label, sampler=1, spp=6, res=96, traversal="near"):
    from jtrace import trace
    sa = abi.SceneABI(scene)
    p = make_params(abi, resolution=res, samples=spp, sampler=sampler, traversal=traversal)
    bvh = trace.make_scene_bvh(sa, False, lib)
    lights = trace.make_trace_lights(sa, lib)
    st = trace.make_trace_state(sa, bvh, lights, p, lib)
    st.set_counters(1)
    st.trace_range(0, spp)
    g = (st.get_image(), *st.get_aovs(), st.counters(), st.describe())
    st.close()
    o = oracle.trace(sa, oracle.build_bvh(sa), oracle.make_lights(sa), p, g[0].shape[1], g[0].shape[0], 0, spp)
    stats = compare_images(g[0], o[0])
    print(label, g[5], stats, "gpu", g[4], "oracle", o[4])
    assert stats["frac_pix_rel_le_1e-3"] >= 0.999, (label, stats)
    assert stats["bitwise_frac"] >= 0.999, (label, stats)  # a silent 1-ulp regression shows here
    assert stats["image_mean_rel"] <= 1e-4, (label, stats)
    assert np.array_equal(g[3], o[3]), label
    for k in ("rays", "light_queries", "nodes", "instances", "prims", "shades"):
        assert abs(g[4][k] - o[4][k]) <= 1e-3 * o[4][k] + 8, (label, k, g[4][k], o[4][k])
    for a, b in ((g[1], o[1]), (g[2], o[2])):
        assert compare_images(a, b)["frac_pix_rel_le_1e-3"] >= 0.999, label
    return g, o


@pytest.mark.parametrize("sampler", [1, 2])
def test_thin_lens_camera_parity(gpu, abi, lib, oracle, cornell, sampler):
    sc = copy.deepcopy(cornell)
    sc.cameras[0].aperture = np.float32(0.25)  # strong defocus: focus 3.9 on the back wall
    g, o = _parity(abi, lib, oracle, sc, f"aperture/{sampler}", sampler=sampler)
    # the lens really is sampled: the defocused render differs from the pinhole one
    p0 = copy.deepcopy(cornell)
    from jtrace import trace
    sa = abi.SceneABI(p0)
    p = make_params(abi, resolution=96, samples=6, sampler=sampler)
    st = trace.make_trace_state(sa, trace.make_scene_bvh(sa, False, lib), trace.make_trace_lights(sa, lib), p, lib)
    st.trace_range(0, 6)
    assert not np.array_equal(st.get_image(), g[0])
    st.close()


@pytest.mark.parametrize("sampler", [1, 2])
def test_orthographic_camera_parity(gpu, abi, lib, oracle, cornell, sampler):
    sc = copy.deepcopy(cornell)
    sc.cameras[0].orthographic = True
    sc.cameras[0].lens = np.float32(0.02)  # film/lens scale: a ~1.2-unit wide view of the box
    g, o = _parity(abi, lib, oracle, sc, f"ortho/{sampler}", sampler=sampler)
    assert g[3].sum() > 0  # it sees the scene


@pytest.mark.parametrize("sampler", [1, 2])
def test_vertex_colors_parity(gpu, abi, lib, oracle, cornell, sampler):
    sc = copy.deepcopy(cornell)
    rng = np.random.default_rng(7)
    for k, s in enumerate(sc.shapes):
        n = len(s.positions)
        col = rng.uniform(0.2, 1.0, size=(n, 4)).astype(np.float32)
        col[:, 3] = 1.0 if k % 2 else rng.uniform(0.6, 1.0, size=n).astype(np.float32)
        s.colors = col
    g, o = _parity(abi, lib, oracle, sc, f"vcolor/{sampler}", sampler=sampler)
    assert ",255," in g[5]  # FT_ATTR | FT_OPAC: the general kernel


@pytest.mark.parametrize("order", ["near", "wide", "reference"])
def test_environment_only_scene(gpu, abi, lib, oracle, order):
    """A scene without instances (features2's environment and camera only): make_bvh of no
    boxes is one leaf without primitives (src/bvh.jl:138-183), every query misses, every path
    sees the environment. Every traversal, the wide one included (an empty tree is one record
    without children), against the oracle."""
    import warnings
    from conftest import ROOT
    from jtrace import sceneio
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        sc = sceneio.load_scene(str(ROOT / "assets" / "scenes" / "features2" / "features2.json"), missing="drop")
    sc.instances = []
    g, o = _parity(abi, lib, oracle, sc, f"env-only/{order}", traversal=order)
    assert f"traversal={order}" in g[5]
    assert g[4]["rays"] > 0 and g[4]["shades"] == 0
    assert float(g[0][..., 3].min()) == 1.0  # the environment is visible everywhere


@pytest.mark.parametrize("order", ["near", "wide", "reference"])
@pytest.mark.parametrize("sampler", [1, 2])
def test_coplanar_ties_with_opacity(gpu, abi, lib, oracle, cornell, order, sampler):
    """Exact-t ties combined with opacity < 1: every cornellbox instance gets a
    coplanar twin (the same shape and frame) with a differently coloured material of opacity 0.6,
    and every shape repeats its own triangles, so almost every hit is a tie — between two
    instances (TLAS leaves) and between two triangles of one BLAS leaf — whose winner the
    reference's child order decides (src/bvh.jl:331-341, src/geometry.jl:226), and the opacity
    draw of the winner's material (src/trace.jl:336-345) then lets the path skip through and
    continue from a moved origin. Every traversal order against the oracle's restatement of it
    (the near-first orders re-run a tied query in the reference's order)."""
    from jtrace.scene import InstanceData, MaterialData
    sc = copy.deepcopy(cornell)
    rng = np.random.default_rng(11)
    for s in sc.shapes:
        s.triangles = np.concatenate([s.triangles, s.triangles[::-1]]).astype(np.int32)
    base_m = len(sc.materials)
    for m in list(sc.materials):
        sc.materials.append(MaterialData(type=m.type, emission=m.emission.copy(),
                                         color=rng.uniform(0.1, 0.9, 3).astype(np.float32), opacity=np.float32(0.6)))
    twins = [InstanceData(frame=i.frame.copy(), shape=i.shape, material=base_m + i.material, name=i.name + "_twin")
             for i in sc.instances]
    sc.instances = [x for pair in zip(sc.instances, twins) for x in pair]
    g, o = _parity(abi, lib, oracle, sc, f"ties+opacity/{order}/{sampler}", sampler=sampler, traversal=order)
    assert f"traversal={order}" in g[5] and ",255," in g[5]  # FT_OPAC: the general kernel
    assert g[3].sum() > 0 and g[4]["light_queries"] > 0 if sampler == 1 else g[3].sum() > 0
