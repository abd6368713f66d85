"""The oracle's --width/--height framing (aspect := W/H, the build's extension used by the
1280x720 headline config; src/scene.jl:377-378 sizes the film from camera.aspect).

Pinned without a GPU by two properties of eval_camera (src/scene.jl:372-411):
  - W x H equal to the camera's own aspect gives exactly the default render;
  - a 16:9 frame of the 1:1 cornellbox camera sees the central rows of the square frame: the
    bounce-0 albedo of a pixel, a function of the surface it sees, matches the square render's
    pixel 1:1 away from silhouette edges (where the jitter changes the surface hit).
"""
import numpy as np

from conftest import make_params


def _render(abi, oracle, scene_abi, bvh, lights, W, H, spp=1, **kw):
    p = make_params(abi, samples=spp, sampler=2, **kw)
    return oracle.trace(scene_abi, bvh, lights, p, W, H, 0, spp)


def test_explicit_size_with_camera_aspect_is_the_default_render(abi, oracle, cornell_abi):
    bvh, lights = oracle.build_bvh(cornell_abi), oracle.make_lights(cornell_abi)
    a = _render(abi, oracle, cornell_abi, bvh, lights, 64, 64, resolution=64)
    b = _render(abi, oracle, cornell_abi, bvh, lights, 64, 64, width=64, height=64)
    assert np.array_equal(a[0], b[0]) and a[4] == b[4]


def test_wide_frame_fits_the_film_to_w_over_h(abi, oracle, cornell_abi):
    bvh, lights = oracle.build_bvh(cornell_abi), oracle.make_lights(cornell_abi)
    W, H = 256, 144
    sq = _render(abi, oracle, cornell_abi, bvh, lights, W, W, resolution=W)
    wide = _render(abi, oracle, cornell_abi, bvh, lights, W, H, width=W, height=H)
    off = (W - H) // 2
    crop = sq[1][off:off + H]  # albedo of the square frame's central rows
    same = np.all(np.abs(crop - wide[1]) <= 1e-6, axis=-1).mean()
    # without the override the 16:9 frame would stretch the square film: rows 0..H-1 would
    # span the whole square field of view and only the centre line would agree
    stretched = sq[1][np.round(np.linspace(0, W - 1, H)).astype(int)]
    same_stretched = np.all(np.abs(stretched - wide[1]) <= 1e-6, axis=-1).mean()
    print("matching albedo: fitted", same, "stretched", same_stretched)
    assert same >= 0.99
    assert same_stretched < 0.95
