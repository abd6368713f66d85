"""The Julia drop-in (julia-raytracer_amd/julia/JtraceHip.jl) cannot run here — there is no
Julia on either machine — so its id packing is restated in Python and driven through the same
C-ABI, on data in the reference's own convention: 1-based ids with invalid_id = -1 for "none"
(src/scene.jl:45, :95-96, :125, :241-245; TraceLight instance/environment, src/trace.jl:131,168).

A round-1 bug mapped every id with `x - 1`, turning invalid_id into -2, which jt_create rejects
(every shipped scene has a material without a texture): these tests pin the fix.
"""
import copy
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

from conftest import ROOT, make_params

SHIM = ROOT / "julia-raytracer_amd" / "julia" / "JtraceHip.jl"
TEX_FIELDS = ("emission_tex", "color_tex", "roughness_tex", "scattering_tex", "normal_tex")
FEATURES1 = str(ROOT / "assets" / "scenes" / "features1" / "features1.json")


def id0(x):
    """JtraceHip.jl `id0`: invalid_id stays -1, a 1-based id becomes 0-based."""
    return -1 if x == -1 else x - 1


def buggy_id0(x):
    """The round-1 mapping (`x - 1` for every id)."""
    return x - 1


def to_reference_convention(scene):
    """The host scene (0-based, -1 = none) as the reference's SceneData holds it: 1-based ids,
    invalid_id (-1) for none."""
    ref = copy.deepcopy(scene)
    for m in ref.materials:
        for f in TEX_FIELDS:
            v = getattr(m, f)
            setattr(m, f, -1 if v < 0 else v + 1)
    for e in ref.environments:
        e.emission_tex = -1 if e.emission_tex < 0 else e.emission_tex + 1
    return ref


def shim_pack(ref_scene, mapping):
    """pack_scene's optional-id handling (JtraceHip.jl pack_scene) applied to a reference-
    convention scene; shape/material/vertex ids go through the host loader's 0-based path."""
    out = copy.deepcopy(ref_scene)
    for m in out.materials:
        for f in TEX_FIELDS:
            setattr(m, f, mapping(getattr(m, f)))
    for e in out.environments:
        e.emission_tex = mapping(e.emission_tex)
    return out


def shim_lights(abi, lights, mapping):
    """pack_lights: TraceLight instance/environment (1-based or invalid_id) -> jt_light."""
    n = lights.struct.nlights
    arr = (abi.jt_light * max(1, n))()
    for k in range(n):
        l = lights.struct.lights[k]
        inst_ref = -1 if l.instance < 0 else l.instance + 1  # reference convention
        env_ref = -1 if l.environment < 0 else l.environment + 1
        arr[k].instance, arr[k].environment = mapping(inst_ref), mapping(env_ref)
        arr[k].ncdf, arr[k].cdf = l.ncdf, l.cdf
    return abi.jt_lights(n, arr), arr


def _create_status(abi, lib, scene, mapping, **kw):
    from jtrace import trace
    sa = abi.SceneABI(shim_pack(to_reference_convention(scene), mapping))
    bvh = trace.make_scene_bvh(sa, False, lib)
    lights = trace.make_trace_lights(sa, lib)
    jl, keep = shim_lights(abi, lights, mapping)
    p = make_params(abi, **kw)
    h = C.c_void_p()
    st = lib.jt_create(sa.ref, bvh.ref, C.byref(jl), C.byref(p), C.byref(h))
    msg = lib.jt_last_error().decode()
    if st == 0:
        lib.jt_destroy(h)
    del keep
    return st, msg


def test_shim_source_maps_optional_ids_with_id0():
    """Static check of the shim (it cannot be executed here): no optional id is shifted with a
    bare `- 1`, and every one goes through id0."""
    text = SHIM.read_text()
    assert re.search(r"id0\(x\)\s*=\s*x\s*==\s*-1\s*\?\s*Int32\(-1\)\s*:\s*Int32\(x\s*-\s*1\)", text)
    for f in TEX_FIELDS:
        assert not re.search(rf"\.{f}\s*-\s*1", text), f
        assert f"id0(m.{f})" in text or f == "emission_tex", f
    assert "id0(e.emission_tex)" in text and "id0(m.emission_tex)" in text
    assert "id0(l.instance)" in text and "id0(l.environment)" in text


@pytest.mark.parametrize("scene_path", ["cornell", FEATURES1])
def test_shim_packing_passes_jt_create_validation(abi, lib, cornell, scene_path):
    """Reference-convention data packed the shim's way passes every jt_create check (on a CPU
    container jt_create then stops at hipSetDevice with JT_ERR_DEVICE; on a GPU it succeeds);
    the round-1 packing is rejected as JT_ERR_INVALID."""
    from jtrace import sceneio
    scene = cornell if scene_path == "cornell" else sceneio.load_scene(scene_path)
    st, msg = _create_status(abi, lib, scene, id0, resolution=32, samples=1)
    assert st in (0, -3), (st, msg)
    st_bad, msg_bad = _create_status(abi, lib, scene, buggy_id0, resolution=32, samples=1)
    assert st_bad == -1 and "texture id" in msg_bad, (st_bad, msg_bad)


@pytest.mark.gpu
def test_shim_packing_renders_like_the_host_loader(gpu, abi, lib, cornell):
    """Through the restated shim packing, cornellbox renders bit for bit as through the host
    loader's own 0-based packing."""
    from jtrace import trace
    p = make_params(abi, resolution=48, samples=2)
    sa = abi.SceneABI(shim_pack(to_reference_convention(cornell), id0))
    bvh = trace.make_scene_bvh(sa, False, lib)
    lights = trace.make_trace_lights(sa, lib)
    jl, keep = shim_lights(abi, lights, id0)
    h = C.c_void_p()
    abi.check(lib, lib.jt_create(sa.ref, bvh.ref, C.byref(jl), C.byref(p), C.byref(h)))
    abi.check(lib, lib.jt_trace_range(h, 0, 2))
    a = np.empty((48, 48, 4), np.float32)
    abi.check(lib, lib.jt_get_image(h, a.ctypes.data_as(abi.f32p)))
    lib.jt_destroy(h)
    del keep
    ca = abi.SceneABI(cornell)
    st = trace.make_trace_state(ca, trace.make_scene_bvh(ca, False, lib), trace.make_trace_lights(ca, lib), p, lib)
    st.trace_range(0, 2)
    assert np.array_equal(a, st.get_image())
    st.close()
