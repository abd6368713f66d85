"""HIP path vs the CPU oracle on identical seeded inputs (the parity gate).

Tolerance (float path tracer, stated per BASELINE.json north_star "within a stated per-channel
float tolerance (seeded RNG)"): both sides evaluate the same float program (no FMA contraction,
Julia min/max, double-evaluated transcendentals) on the same PCG32 streams, so almost every
pixel is bit-identical; a libm 1-ulp disagreement can flip a discrete decision (Russian
roulette, a triangle edge) and change one path. Bar, per image:
  - >= 99.9 % of pixels within 1e-3 relative on every channel,
  - per-channel image mean within 1e-4 relative,
  - the running-mean alpha / hit counts identical.
"""
import numpy as np
import pytest

from conftest import compare_images, make_params

pytestmark = pytest.mark.gpu


def _render_both(abi, lib, oracle, scene_abi, params, s0, s1, batch_calls=False):
    from jtrace import trace
    bvh = trace.make_scene_bvh(scene_abi, False, lib)
    lights = trace.make_trace_lights(scene_abi, lib)
    st = trace.make_trace_state(scene_abi, bvh, lights, params, lib)
    if batch_calls:
        for _ in range(s0, s1, params.batch):
            st.trace_samples()
    else:
        st.trace_range(s0, s1)
    gimg = st.get_image()
    galb, gnrm, ghits = st.get_aovs()
    gcnt = st.counters()
    k = st.streams
    st.close()
    ob = oracle.build_bvh(scene_abi)
    ol = oracle.make_lights(scene_abi)
    oimg, oalb, onrm, ohits, ocnt = oracle.trace(scene_abi, ob, ol, params, gimg.shape[1], gimg.shape[0], s0, s1,
                                                 streams=k)
    return (gimg, galb, gnrm, ghits, gcnt), (oimg, oalb, onrm, ohits, ocnt)


@pytest.mark.parametrize("sampler", [1, 2])
def test_cornellbox_parity(gpu, abi, lib, oracle, cornell_abi, sampler):
    params = make_params(abi, resolution=96, samples=8, sampler=sampler)
    g, o = _render_both(abi, lib, oracle, cornell_abi, params, 0, 8)
    stats = compare_images(g[0], o[0])
    print("sampler", sampler, stats, "gpu counters", g[4], "oracle counters", o[4])
    assert stats["frac_pix_rel_le_1e-3"] >= 0.999, stats
    assert stats["bitwise_frac"] >= 0.999, stats  # a silent 1-ulp regression shows here
    assert stats["image_mean_rel"] <= 1e-4, stats
    assert np.array_equal(g[3], o[3])  # hits
    assert g[4]["paths"] == o[4]["paths"] == 96 * 96 * 8
    # traversal work is deterministic given seed + BVH; allow the rare flipped path
    for k in ("rays", "light_queries", "nodes", "instances", "prims", "shades"):
        assert abs(g[4][k] - o[4][k]) <= 1e-3 * o[4][k] + 8, (k, g[4][k], o[4][k])
    astats = compare_images(g[1], o[1])
    assert astats["frac_pix_rel_le_1e-3"] >= 0.999, astats


def test_batching_is_bitwise_invariant(gpu, abi, lib, cornell_abi):
    """A render split into calls gives the bits of one call over the whole range, at one sample
    stream (trace_samples with the reference's --batch 1, 6 calls: deferred and merged into one
    chunk; the same 6 calls each flushed by jt_synchronize: one launch per sample) and at k streams
    (any split of the range: every stream sees its samples in order, the image is their combination)."""
    from jtrace import trace
    bvh = trace.make_scene_bvh(cornell_abi, False, lib)
    lights = trace.make_trace_lights(cornell_abi, lib)
    p1 = make_params(abi, resolution=64, samples=6, batch=1)
    a = trace.make_trace_state(cornell_abi, bvh, lights, p1, lib)
    assert a.streams == 1
    for _ in range(6):
        a.trace_samples()
    assert a.samples == 6
    one = trace.make_trace_state(cornell_abi, bvh, lights, p1, lib)
    one.trace_range(0, 6)
    assert np.array_equal(a.get_image(), one.get_image())
    per = trace.make_trace_state(cornell_abi, bvh, lights, p1, lib)
    for _ in range(6):
        per.trace_samples()
        per.synchronize()
    assert per.counters()["launches"] == 6 and a.counters()["launches"] == 1
    assert np.array_equal(per.get_image(), one.get_image())
    for x, y in zip(per.get_aovs(), one.get_aovs()):
        assert np.array_equal(x, y)
    a.trace_samples()  # state.samples >= params.samples: no-op, as the reference
    assert a.samples == 6
    p2 = make_params(abi, resolution=64, samples=11, batch=11)
    full = trace.make_trace_state(cornell_abi, bvh, lights, p2, lib)
    assert full.streams == 8, full.describe()
    full.trace_range(0, 11)
    ref = (full.get_image(), full.get_aovs())
    for cuts in ((0, 1, 11), (0, 3, 4, 10, 11), (0, 8, 11)):
        b = trace.make_trace_state(cornell_abi, bvh, lights, p2, lib)
        for s0, s1 in zip(cuts[:-1], cuts[1:]):
            b.trace_range(s0, s1)
        assert np.array_equal(b.get_image(), ref[0]), cuts
        for x, y in zip(b.get_aovs(), ref[1]):
            assert np.array_equal(x, y), cuts
        b.close()
    # one stream vs eight: the same samples, combined in another order (last bits only)
    stats = compare_images(full.get_image(), trace_one(cornell_abi, bvh, lights, make_params(abi, resolution=64, samples=11, batch=1), lib))
    assert stats["frac_pix_rel_le_1e-3"] >= 0.999 and stats["image_mean_rel"] <= 1e-5, stats


@pytest.mark.parametrize("scene,sampler", [("cornellbox", 1), ("cornellbox", 2), ("features1", 1), ("bathroom1", 1)])
def test_one_stream_chunks_match_per_sample_launches(gpu, abi, lib, cornell_abi, scene, sampler):
    """The reference's --batch 1 (one stream, src/jtrace.jl:83): 70 trace_samples calls are
    deferred and traced as chunks of one-sample streams folded in sample order by chain_kernel (64,
    then 6 with the first 64 as the running mean's start); the bits must be those of one launch
    per sample (each call flushed by jt_synchronize), images, AOVs, hits and counters, in LDS mode
    and in the HBM mesh kernels."""
    from jtrace import trace
    from test_gpu_scenes import scene_abi
    sa = cornell_abi if scene == "cornellbox" else scene_abi(scene)
    bvh = trace.make_scene_bvh(sa, False, lib)
    lights = trace.make_trace_lights(sa, lib)
    n = 70
    p = make_params(abi, resolution=48, samples=n, batch=1, sampler=sampler)
    outs = []
    for mode in ("per-sample", "deferred", "one call"):
        st = trace.make_trace_state(sa, bvh, lights, p, lib)
        assert st.streams == 1
        if mode == "one call":
            st.trace_range(0, n)
        else:
            for _ in range(n):
                st.trace_samples()
                if mode == "per-sample":
                    st.synchronize()
        assert st.samples == n
        outs.append((st.get_image(), st.get_aovs(), st.counters()))
        st.close()
    assert outs[0][2]["launches"] == n and outs[1][2]["launches"] == 2 and outs[2][2]["launches"] == 2, \
        [o[2]["launches"] for o in outs]
    for o in outs[1:]:
        assert np.array_equal(outs[0][0], o[0])
        for a, b in zip(outs[0][1], o[1]):
            assert np.array_equal(a, b)
        for k in ("paths", "rays", "light_queries"):
            assert outs[0][2][k] == o[2][k], k


def trace_one(sa, bvh, lights, p, lib):
    from jtrace import trace
    st = trace.make_trace_state(sa, bvh, lights, p, lib)
    st.trace_range(0, p.samples)
    img = st.get_image()
    st.close()
    return img


def test_shard_combination_matches_single(gpu, abi, lib, cornell_abi):
    """Two contexts over [0,4) and [4,8) combined by sample-weighted sum == one context [0,8)."""
    from jtrace import trace
    bvh = trace.make_scene_bvh(cornell_abi, False, lib)
    lights = trace.make_trace_lights(cornell_abi, lib)
    p = make_params(abi, resolution=64, samples=8)
    full = trace.make_trace_state(cornell_abi, bvh, lights, p, lib)
    full.trace_range(0, 8)
    s1 = trace.make_trace_state(cornell_abi, bvh, lights, p, lib)
    s1.trace_range(0, 4)
    s2 = trace.make_trace_state(cornell_abi, bvh, lights, p, lib)
    s2.trace_range(4, 8)
    comb = (s1.get_image().astype(np.float64) * 4 + s2.get_image().astype(np.float64) * 4) / 8
    np.testing.assert_allclose(comb, full.get_image(), rtol=2e-5, atol=2e-6)


def test_out_of_order_range_rejected(gpu, abi, lib, cornell_abi):
    from jtrace import trace
    bvh = trace.make_scene_bvh(cornell_abi, False, lib)
    lights = trace.make_trace_lights(cornell_abi, lib)
    st = trace.make_trace_state(cornell_abi, bvh, lights, make_params(abi, resolution=32), lib)
    st.trace_range(0, 2)
    with pytest.raises(abi.JTError) as e:
        st.trace_range(5, 6)
    assert e.value.status == -6


def cornell_with_emission(scale):
    """The cornellbox scene with every emission scaled (the pin tests' negative controls)."""
    from conftest import CORNELL
    from jtrace import abi, sceneio
    sc = sceneio.load_scene(CORNELL)
    for m in sc.materials:
        m.emission = (np.asarray(m.emission, np.float32) * np.float32(scale)).astype(np.float32)
    return abi.SceneABI(sc)


# The headline scene's pin against the reference's own render, about 3x the error measured at
# 64 spp (round 5: channel means 0.03 %, block median 0.45 %, block p95 2.1 %)
PIN_CHANNEL_RTOL, PIN_BLOCK_MEDIAN, PIN_BLOCK_P95 = 0.003, 0.015, 0.06


def cornell_pin(img):
    """(ok, stats): a 1280x1280 render through the reference's sRGB + 8-bit pipeline vs
    images/cornellbox_path.png on 40x40-pixel block means (tests/golden/cornellbox_path_blocks.npz)."""
    from pathlib import Path
    from jtrace import sceneio
    pin = np.load(Path(__file__).parent / "golden" / "cornellbox_path_blocks.npz")
    lin = sceneio.decode_srgb8(sceneio.to_srgb8(img, 1280, 1280))[..., :3]
    bm = lin.reshape(32, 40, 32, 40, 3).mean(axis=(1, 3))
    cm = lin.reshape(-1, 3).mean(axis=0)
    cm_rel = np.abs(cm / pin["channel_mean"] - 1)
    rel = np.abs(bm - pin["mean"]) / np.maximum(pin["mean"], 0.02)
    st = {"channel_mean": cm.tolist(), "reference": pin["channel_mean"].tolist(), "channel_rel": cm_rel.tolist(),
          "block_median": float(np.median(rel)), "block_p95": float(np.percentile(rel, 95))}
    ok = bool(np.all(cm_rel <= PIN_CHANNEL_RTOL) and st["block_median"] < PIN_BLOCK_MEDIAN
              and st["block_p95"] < PIN_BLOCK_P95)
    return ok, st


def test_statistical_pin_full_resolution(gpu, abi, lib, cornell_abi):
    """HIP render at the reference's own size (1280x1280, 64 spp) vs images/cornellbox_path.png
    (src/trace.jl:625-648 through save_image), at about 3x the measured error; and two negative
    controls, the same render with every emission scaled by 1.02 and by 0.98, which must fail it (a
    2 % clamp, MIS-weight or light-area bias would not pass)."""
    from jtrace import trace
    outs = {}
    for scale in (1.0, 1.02, 0.98):
        sa = cornell_abi if scale == 1.0 else cornell_with_emission(scale)
        bvh = trace.make_scene_bvh(sa, False, lib)
        lights = trace.make_trace_lights(sa, lib)
        st = trace.make_trace_state(sa, bvh, lights, make_params(abi, resolution=1280, samples=64, batch=64), lib)
        st.trace_range(0, 64)
        outs[scale] = cornell_pin(st.get_image())
        st.close()
        print("emission x", scale, outs[scale])
    assert outs[1.0][0], outs[1.0][1]
    assert not outs[1.02][0] and not outs[0.98][0], (outs[1.02][1], outs[0.98][1])


@pytest.mark.parametrize("sampler,spp", [(1, 4), (2, 4), (1, 64), (2, 96)])
def test_lds_and_hbm_scene_modes_bitwise_equal(gpu, abi, lib, cornell_abi, sampler, spp, options):
    """The small-scene LDS mode and the HBM mode run the same program on the same data, with the
    same sample streams (one batch of 4, 64 or 96 samples: 4, 64 and 64 streams in both modes)."""
    from jtrace import trace
    bvh = trace.make_scene_bvh(cornell_abi, False, lib)
    lights = trace.make_trace_lights(cornell_abi, lib)
    p = make_params(abi, resolution=80, samples=spp, sampler=sampler, batch=spp)
    imgs = []
    for mode in ("0", "65536"):
        options("lds_scene", mode)
        st = trace.make_trace_state(cornell_abi, bvh, lights, p, lib)
        assert ("mode=lds" in st.describe()) == (mode != "0"), st.describe()
        assert st.streams == min(spp, 64), st.describe()
        st.trace_range(0, spp)
        imgs.append((st.get_image(), st.get_aovs(), st.counters()))
        st.close()
    assert np.array_equal(imgs[0][0], imgs[1][0])
    for a, b in zip(imgs[0][1], imgs[1][1]):
        assert np.array_equal(a, b)
    for k in ("rays", "light_queries", "nodes", "instances", "prims", "shades"):
        assert imgs[0][2][k] == imgs[1][2][k], k


@pytest.mark.parametrize("sampler", [1, 2])
@pytest.mark.parametrize("lds", ["65536", "0"])
def test_feature_specialisation_bitwise_equal(gpu, abi, lib, cornell_abi, sampler, lds, options):
    """Cornellbox has no scene feature bit, so it runs the FT_NONE kernel; the general FT_ALL
    kernel (option features=all) must give the same bits, counters included."""
    from jtrace import trace
    bvh = trace.make_scene_bvh(cornell_abi, False, lib)
    lights = trace.make_trace_lights(cornell_abi, lib)
    p = make_params(abi, resolution=80, samples=4, sampler=sampler)
    options("lds_scene", lds)
    outs = []
    for feat in ("auto", "all"):
        options("features", feat)
        st = trace.make_trace_state(cornell_abi, bvh, lights, p, lib)
        st.set_counters(1)
        st.trace_range(0, 4)
        outs.append((st.get_image(), st.get_aovs(), st.counters(), st.describe()))
        st.close()
    assert ",8192," in outs[0][3] and ",255," in outs[1][3], (outs[0][3], outs[1][3])  # FT_NONE | FT_LINL
    assert np.array_equal(outs[0][0], outs[1][0])
    for a, b in zip(outs[0][1], outs[1][1]):
        assert np.array_equal(a, b)
    for k in ("paths", "rays", "light_queries", "nodes", "instances", "prims", "shades"):
        assert outs[0][2][k] == outs[1][2][k], k


def test_light_hit_steps_are_bitwise_invariant(gpu, abi, lib, cornell_abi, options):
    """Light-hit steps inside the traversal phase (FT_NONE kernel, path sampler) only change
    when a lane runs light_hit, not what it computes: every threshold gives the same bits."""
    from jtrace import trace
    bvh = trace.make_scene_bvh(cornell_abi, False, lib)
    lights = trace.make_trace_lights(cornell_abi, lib)
    p = make_params(abi, resolution=72, samples=5, sampler=1)
    outs = []
    options("light_inline", "0")  # cornellbox's light chains otherwise never leave the shading phase
    for ll in ("1", "7", "65"):
        options("light_lanes", ll)
        st = trace.make_trace_state(cornell_abi, bvh, lights, p, lib)
        st.set_counters(1)
        st.trace_range(0, 5)
        outs.append((st.get_image(), st.get_aovs(), st.counters()))
        st.close()
    for o in outs[1:]:
        assert np.array_equal(outs[0][0], o[0])
        for a, b in zip(outs[0][1], o[1]):
            assert np.array_equal(a, b)
        for k in ("paths", "rays", "light_queries", "nodes", "instances", "prims", "shades"):
            assert outs[0][2][k] == o[2][k], k


@pytest.mark.parametrize("sampler", [1, 2])
@pytest.mark.parametrize("k", ["2", "8", "64"])
def test_sample_streams_match_the_oracle(gpu, abi, lib, oracle, cornell_abi, sampler, k, options):
    """k sample streams per pixel (include/jtrace.h jt_trace_range), in two calls whose second
    continues every stream's running mean from HBM, against the oracle's restatement of the same
    streams and combination: at the parity bar, hits and paths exact."""
    from jtrace import trace
    options("streams", k)
    bvh = trace.make_scene_bvh(cornell_abi, False, lib)
    lights = trace.make_trace_lights(cornell_abi, lib)
    p = make_params(abi, resolution=72, samples=9, sampler=sampler)
    st = trace.make_trace_state(cornell_abi, bvh, lights, p, lib)
    assert st.streams == int(k) and f"streams={k}" in st.describe()
    st.trace_range(0, 5)
    st.trace_range(5, 9)
    g = (st.get_image(), *st.get_aovs(), st.counters())
    st.close()
    ob, ol = oracle.build_bvh(cornell_abi), oracle.make_lights(cornell_abi)
    parts = {}
    oracle.trace(cornell_abi, ob, ol, p, 72, 72, 0, 5, streams=int(k), parts=parts)
    o = oracle.trace(cornell_abi, ob, ol, p, 72, 72, 5, 9, streams=int(k), parts=parts,
                     state=tuple(np.zeros(x.shape, x.dtype) for x in (g[0], g[1], g[2], g[3])))
    stats = compare_images(g[0], o[0])
    print("streams", k, "sampler", sampler, stats)
    assert stats["frac_pix_rel_le_1e-3"] >= 0.999 and stats["image_mean_rel"] <= 1e-4, stats
    assert stats["bitwise_frac"] >= 0.999, stats  # a silent 1-ulp regression shows here
    assert np.array_equal(g[3], o[3])
    for a, b in zip(g[1:3], o[1:3]):
        assert compare_images(a, b)["frac_pix_rel_le_1e-3"] >= 0.999
    assert g[4]["paths"] == 72 * 72 * 9


def test_stream_count_rule(gpu, abi, lib, cornell_abi, options):
    """jt_get_streams: 1 at --batch 1, else the smallest power of two >= 16 (>= 32 from a batch
    of 64) with (pixels traced) x k >= 2^22, capped at min(batch, 64) and (pixels) x k <= 2^27
    (include/jtrace.h); a tile share counts its own pixels; the scene's memory mode never enters
    (cornellbox runs in LDS mode, the `lds_scene=0` option puts it in HBM mode: same k)."""
    from jtrace import trace
    bvh = trace.make_scene_bvh(cornell_abi, False, lib)
    lights = trace.make_trace_lights(cornell_abi, lib)

    def rule(px, batch):
        if batch <= 1:
            return 1
        want = 32 if batch >= 64 else 16
        while px * want < 1 << 22:
            want *= 2
        k = 1
        while 2 * k <= min(want, batch, 64) and px * 2 * k <= 1 << 27:
            k *= 2
        return k

    # (width, height, batch, tile share, HBM mode): streams
    expect = {(1280, 720, 256, 1, 0): 32, (1280, 720, 256, 1, 1): 32, (1280, 720, 32, 1, 1): 16,
              (1280, 720, 1, 1, 0): 1, (256, 256, 16, 1, 0): 16, (1920, 1080, 1024, 1, 1): 32,
              (1920, 1080, 1024, 1, 0): 32, (3840, 2160, 4096, 1, 1): 16, (1280, 720, 256, 8, 0): 64,
              (1280, 720, 256, 8, 1): 64, (64, 64, 5, 1, 0): 4, (7680, 4320, 64, 1, 1): 4}
    for (w, h, batch, share, hbm), k in expect.items():
        options("tile_share", f"{share},0" if share > 1 else None)
        options("lds_scene", "0" if hbm else None)
        st = trace.make_trace_state(cornell_abi, bvh, lights, make_params(abi, width=w, height=h, samples=batch,
                                                                          batch=batch), lib)
        assert ("mode=hbm" in st.describe()) == bool(hbm), st.describe()
        tiles = ((w + 7) // 8) * ((h + 7) // 8)
        px = w * h if share == 1 else -(-w * h // share)
        assert st.streams == rule(px, batch) == k, (w, h, batch, share, hbm, st.streams, tiles)
        st.close()


@pytest.mark.parametrize("w,h,batch,share", [(13, 7, 4, 1), (203, 77, 8, 1), (40, 330, 4, 1), (200, 72, 4, 5),
                                               (200, 72, 4, 3)])
def test_band_strip_order_covers_every_pixel_once(gpu, abi, lib, oracle, cornell_abi, w, h, batch, share, options):
    """The work-unit order (XCD bands of whole tile rows walked in 16-row strips, column by
    column; a tile share whose stride divides the tile columns walks its own grid the same way,
    others the plain split) hands out every (pixel, stream) item exactly once: odd sizes with
    partial edge tiles, fewer tile rows than bands, and tile shares on and off the strip path,
    against the oracle (the share's pixels against the oracle's full image; paths exact)."""
    options("tile_share", f"{share},1" if share > 1 else None)
    params = make_params(abi, width=w, height=h, samples=batch, batch=batch)
    g, o = _render_both(abi, lib, oracle, cornell_abi, params, 0, batch)
    tiles_x = (w + 7) // 8
    if share > 1:  # the share's pixels: tiles 1, 1 + share, ...; the oracle traced every pixel
        ty, tx = np.divmod(np.arange(tiles_x * ((h + 7) // 8)), tiles_x)
        mine = (ty * tiles_x + tx) % share == 1
        mask = np.zeros((h, w), bool)
        for t in np.nonzero(mine)[0]:
            mask[ty[t] * 8:ty[t] * 8 + 8, tx[t] * 8:tx[t] * 8 + 8] = True
        assert np.all(g[0][~mask] == 0), "a pixel outside the share was traced"
        assert g[4]["paths"] == int(mask.sum()) * batch
    else:
        mask = np.ones((h, w), bool)
        assert g[4]["paths"] == o[4]["paths"] == w * h * batch
    same = np.all(g[0][mask] == o[0][mask], axis=-1)
    print(w, h, batch, share, "pixels", int(mask.sum()), "bit-equal", float(same.mean()))
    assert same.mean() >= 0.999  # the §8(c) bar; in practice every pixel
    assert np.array_equal(g[3][mask], o[3][mask])


def test_device_buffer_view_is_the_running_mean(gpu, abi, lib, cornell_abi):
    """bench.py's multi-GPU reduce reads the library's running-mean image in place through
    __cuda_array_interface__ (jt_get_device_buffers): that view must be exactly jt_get_image, and
    the sample-weighted reduce of jtrace.parallel over a world of one rank must give it back."""
    torch = pytest.importorskip("torch")
    from jtrace import trace
    from jtrace.parallel import reduce_running_means
    bvh = trace.make_scene_bvh(cornell_abi, False, lib)
    lights = trace.make_trace_lights(cornell_abi, lib)
    st = trace.make_trace_state(cornell_abi, bvh, lights, make_params(abi, resolution=48, samples=3), lib)
    st.trace_range(0, 3)
    buf = st.device_buffers()
    H, W = st.height, st.width

    class _CAI:
        __cuda_array_interface__ = {"shape": (H * W * 4,), "typestr": "<f4", "data": (buf.image, False), "version": 3}

    dev = torch.as_tensor(_CAI(), device="cuda:0")
    torch.cuda.synchronize()
    host = st.get_image().reshape(-1)
    np.testing.assert_array_equal(dev.cpu().numpy(), host)

    class _OneRank:  # torch.distributed stand-in for a world of one rank: reduce is the identity
        class ReduceOp:
            SUM = None

        @staticmethod
        def reduce(t, dst, op):
            return None

        @staticmethod
        def get_rank():
            return 0

    out = reduce_running_means(dev, 3, 3, _OneRank, dst=0)
    np.testing.assert_allclose(out.cpu().numpy(), host, rtol=1e-6, atol=0)

    # k > 1 streams combine the AOVs only when read: through the device pointers they are
    # current after jt_synchronize, and equal jt_get_aovs (here after a second call that appends
    # to the streams' means, so a stale combine would show)
    def view(ptr, n, typestr):
        class _V:
            __cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 3}
        return torch.as_tensor(_V(), device="cuda:0")

    sk = trace.make_trace_state(cornell_abi, bvh, lights, make_params(abi, resolution=48, samples=3, batch=3), lib)
    assert sk.streams > 1, sk.describe()
    bk = sk.device_buffers()
    sk.trace_range(0, 2)
    sk.trace_range(2, 3)
    img_k = view(bk.image, H * W * 4, "<f4")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(img_k.cpu().numpy(), sk.get_image().reshape(-1))  # current at return
    sk.synchronize()
    torch.cuda.synchronize()
    alb = view(bk.albedo, H * W * 4, "<f4").cpu().numpy().reshape(-1, 4)[:, :3]
    nrm = view(bk.normal, H * W * 4, "<f4").cpu().numpy().reshape(-1, 4)[:, :3]
    hit = view(bk.hits, H * W, "<i8").cpu().numpy()
    a, n, h = sk.get_aovs()
    np.testing.assert_array_equal(alb, a.reshape(-1, 3))
    np.testing.assert_array_equal(nrm, n.reshape(-1, 3))
    np.testing.assert_array_equal(hit, h.reshape(-1))
    assert hit.sum() > 0
    sk.close()
    # a reset zeroes the running means at once once their device pointers were handed out
    st.reset()
    torch.cuda.synchronize()
    assert not dev.cpu().numpy().any()
    st.close()


def _full_parity(abi, lib, oracle, scene_abi, params, spp, label):
    g, o = _render_both(abi, lib, oracle, scene_abi, params, 0, spp)
    stats = compare_images(g[0], o[0])
    print(label, g[0].shape, stats, "gpu", g[4], "oracle", o[4])
    assert stats["frac_pix_rel_le_1e-3"] >= 0.999, stats
    assert stats["bitwise_frac"] >= 0.999, stats  # a silent 1-ulp regression shows here
    assert stats["image_mean_rel"] <= 1e-4, stats
    assert np.array_equal(g[3], o[3])
    H, W = g[0].shape[:2]
    assert g[4]["paths"] == o[4]["paths"] == W * H * spp
    for k in ("rays", "light_queries", "nodes", "instances", "prims", "shades"):
        assert abs(g[4][k] - o[4][k]) <= 1e-3 * o[4][k] + 8, (k, g[4][k], o[4][k])
    for a, b in zip(g[1:3], o[1:3]):
        assert compare_images(a, b)["frac_pix_rel_le_1e-3"] >= 0.999


# "near" is the binary near-first order (DEFAULT_TRAVERSAL), "wide" its 4-wide quantised-record
# form (JT_TRAVERSAL_WIDE), "reference" the reference's own far-first order (src/bvh.jl:331-341).
# All three are restated by the oracle.
ORDERS = ["near", "wide", "reference"]


@pytest.mark.parametrize("order", ORDERS)
def test_headline_frame_parity(gpu, abi, lib, oracle, cornell_abi, order):
    """The bench's exact framing — cornellbox path at 1280x720 through --width/--height, whose
    film is fitted to W/H (the oracle restates that override) — against the oracle, full frame,
    8 spp (the headline workload's first 8 samples of every pixel), in the benched near-first
    order and in the reference's order."""
    params = make_params(abi, width=1280, height=720, samples=8, sampler=1, traversal=order)
    _full_parity(abi, lib, oracle, cornell_abi, params, 8, f"cornellbox path 1280x720x8 traversal={order}")


@pytest.mark.parametrize("order", ORDERS)
def test_config1_full_size_parity(gpu, abi, lib, oracle, cornell_abi, order):
    """BASELINE config 1 at its own size: cornellbox naive 256x256 x 16 spp (1,048,576 paths)."""
    params = make_params(abi, resolution=256, samples=16, sampler=2, traversal=order)
    _full_parity(abi, lib, oracle, cornell_abi, params, 16, f"config1 cornellbox naive 256x256x16 traversal={order}")
