"""The WF body (trace_body_wf: queries decoupled from path slots, any lane runs any slot's query,
any wave shades any slot) against the per-lane megakernel body (trace_body): the same float
operations in the same per-path order, so images, AOVs and every traversal counter must be
bit-identical — in LDS and HBM scene modes, the FT_NONE and FT_ALL kernels, both samplers, and
with work units of a single sample (the chunk ordering of a tile's running means)."""
import numpy as np
import pytest

from conftest import make_params

pytestmark = pytest.mark.gpu


def _run(abi, lib, sa, p, spp, env, monkeypatch):
    from jtrace import trace
    for k in ("JT_WF", "JT_LDS_SCENE", "JT_FEATURES", "JT_CHUNK", "JT_WF_GROUPS", "JT_WAIT_LANES"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    st = trace.make_trace_state(sa, trace.make_scene_bvh(sa, False, lib), trace.make_trace_lights(sa, lib), p, lib)
    st.set_counters(1)
    st.trace_range(0, spp)
    out = (st.get_image(), st.get_aovs(), st.counters(), st.describe())
    st.close()
    return out


def _same(a, b):
    assert np.array_equal(a[0], b[0]), (a[3], b[3])
    for x, y in zip(a[1], b[1]):
        assert np.array_equal(x, y)
    for k in ("paths", "rays", "light_queries", "nodes", "instances", "prims", "shades"):
        assert a[2][k] == b[2][k], (k, a[2][k], b[2][k])


@pytest.mark.parametrize("sampler", [1, 2])
@pytest.mark.parametrize("mode", [{}, {"JT_LDS_SCENE": "0"}, {"JT_FEATURES": "all"}, {"JT_CHUNK": "1"},
                                  {"JT_WF_GROUPS": "1", "JT_WAIT_LANES": "7"}])
def test_wf_body_bitwise_equals_megakernel(gpu, abi, lib, cornell_abi, sampler, mode, monkeypatch):
    p = make_params(abi, resolution=72, samples=5, sampler=sampler)
    ref = _run(abi, lib, cornell_abi, p, 5, {k: v for k, v in mode.items() if not k.startswith("JT_WF") and k != "JT_WAIT_LANES"}, monkeypatch)
    wf = _run(abi, lib, cornell_abi, p, 5, {"JT_WF": "1", **mode}, monkeypatch)
    assert "trace_kernel_wf" in wf[3] and "trace_kernel_wf" not in ref[3], (wf[3], ref[3])
    _same(ref, wf)


@pytest.mark.parametrize("name", ["features1", "materials1", "materials4"])
def test_wf_body_bitwise_on_feature_scenes(gpu, abi, lib, name, monkeypatch):
    from test_gpu_scenes import scene_abi
    sa = scene_abi(name)
    p = make_params(abi, resolution=64, samples=3)
    ref = _run(abi, lib, sa, p, 3, {}, monkeypatch)
    wf = _run(abi, lib, sa, p, 3, {"JT_WF": "1"}, monkeypatch)
    if "trace_kernel_wf" not in wf[3]:
        pytest.skip(f"{name}: stack bound above the WF body's 16 entries ({wf[3]})")
    _same(ref, wf)
