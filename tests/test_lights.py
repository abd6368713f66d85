"""make_trace_lights (src/trace.jl:117-187): product host helper vs oracle, bit for bit."""
import numpy as np

from jtrace.scene import EnvironmentData, TextureData, identity_frame
from test_bvh import random_scene


def cdfs(lights):
    return [(l.instance, l.environment, np.ctypeslib.as_array(l.cdf, shape=(l.ncdf,)).copy())
            for l in (lights.lights[k] for k in range(lights.nlights))]


def check(abi, lib, oracle, scene):
    from jtrace import trace
    sa = abi.SceneABI(scene)
    pl, ol = trace.make_trace_lights(sa, lib), oracle.make_lights(sa)
    a, b = cdfs(pl.struct), cdfs(ol.struct)
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert x[0] == y[0] and x[1] == y[1]
        assert x[2].tobytes() == y[2].tobytes()
    return a


def test_cornellbox_light(abi, lib, oracle, cornell):
    (inst, env, cdf), = check(abi, lib, oracle, cornell)
    assert inst == 4 and env == -1
    np.testing.assert_array_equal(cdf, np.array([0.125, 0.25], np.float32))  # object-space areas


def test_quads_and_environment(abi, lib, oracle):
    rng = np.random.default_rng(3)
    sc = random_scene(rng, quads=True)
    sc.materials[0].emission = np.array([1, 2, 3], np.float32)
    w, h = 64, 32
    px = rng.random((h, w, 4)).astype(np.float32)
    sc.textures.append(TextureData(width=w, height=h, linear=True, pixelsf=px))
    b8 = (rng.random((h, w, 4)) * 255).astype(np.uint8)
    sc.textures.append(TextureData(width=w, height=h, linear=False, pixelsb=b8))
    sc.environments.append(EnvironmentData(frame=identity_frame(), emission=np.ones(3, np.float32), emission_tex=0))
    sc.environments.append(EnvironmentData(frame=identity_frame(), emission=np.ones(3, np.float32), emission_tex=1))
    out = check(abi, lib, oracle, sc)
    assert sum(1 for o in out if o[1] >= 0) == 2
    assert len(out[-1][2]) == w * h
