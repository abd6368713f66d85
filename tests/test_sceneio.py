"""Host scene pipeline: PLY (src/shape.jl), HDR/PNG textures (src/scene.jl:164-189), JSON
constructors and lookat (src/scene.jl:58-143), save_image (src/sceneio.jl:97-123), CLI (src/cli.jl)."""
import json
import struct

import numpy as np
import pytest

from jtrace import cli, sceneio
from jtrace.scene import find_camera, lookat_frame


def write_ply_binary(path, verts, faces, extra=()):
    names = ["x", "y", "z"] + [e[0] for e in extra]
    hdr = ["ply", "format binary_little_endian 1.0", f"element vertex {len(verts)}"]
    hdr += [f"property float {n}" for n in names]
    hdr += [f"element face {len(faces)}", "property list uchar int vertex_indices", "end_header"]
    body = b""
    for k, v in enumerate(verts):
        vals = list(v) + [e[1][k] for e in extra]
        body += struct.pack("<" + "f" * len(vals), *vals)
    for f in faces:
        body += struct.pack("<B", len(f)) + struct.pack("<" + "i" * len(f), *f)
    path.write_bytes(("\n".join(hdr) + "\n").encode() + body)


def test_cornellbox_loads(cornell):
    assert len(cornell.shapes) == 8 and len(cornell.instances) == 8 and len(cornell.materials) == 8
    assert sum(len(s.triangles) for s in cornell.shapes) == 36
    light = cornell.materials[4]
    assert list(light.emission) == [17, 12, 4] and list(light.color) == [0, 0, 0]  # color defaults to 0
    assert cornell.cameras[0].aspect == np.float32(1.0) and cornell.cameras[0].focus == np.float32(3.9)


def test_ply_faces_quads_fan_and_texcoord_flip(tmp_path):
    v = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0.5, 2, 0)]
    p = tmp_path / "a.ply"
    write_ply_binary(p, v, [[0, 1, 2, 3], [1, 2, 4]], extra=[("u", [0.1] * 5), ("v", [0.25] * 5)])
    s = sceneio.load_shape(str(p))
    # any 4-gon -> quads; the triangle becomes (a, b, c, c) (src/shape.jl:323-369)
    assert s.quads.tolist() == [[0, 1, 2, 3], [1, 2, 4, 4]] and len(s.triangles) == 0
    np.testing.assert_array_equal(s.texcoords[:, 1], np.float32(1) - np.float32(0.25))
    p2 = tmp_path / "b.ply"
    write_ply_binary(p2, v, [[0, 1, 2, 3, 4], [0, 1, 2]])  # pentagon fans into 3 triangles
    s2 = sceneio.load_shape(str(p2))
    assert s2.triangles.tolist() == [[0, 1, 2], [0, 2, 3], [0, 3, 4], [0, 1, 2]]


def test_hdr_rle_roundtrip_and_clamp(tmp_path):
    w, h = 16, 3
    rng = np.random.default_rng(0)
    rgbe = rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8)
    rgbe[..., 3] = rng.integers(120, 140, size=(h, w))
    data = b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n" + f"-Y {h} +X {w}\n".encode()
    for y in range(h):  # new-style RLE scanlines, all runs literal
        data += bytes([2, 2, w >> 8, w & 255])
        for ch in range(4):
            data += bytes([w]) + rgbe[y, :, ch].tobytes()
    f = tmp_path / "t.hdr"
    f.write_bytes(data)
    got = sceneio._read_hdr(str(f))
    ref = rgbe[..., :3].astype(np.float64) * np.ldexp(1.0, rgbe[..., 3].astype(np.int32) - 136)[..., None]
    np.testing.assert_allclose(got, ref.astype(np.float32))
    t = sceneio.load_texture(str(f))
    assert t.linear and t.pixelsf.max() <= 1.0 and np.all(t.pixelsf[..., 3] == 1)
    # default decode: clamp, sRGB-encode, 16-bit quantise (sceneio.HDR_MODE)
    c = np.clip(ref, 0, 1)
    enc = np.where(c <= 0.0031308, 12.92 * c, 1.055 * c ** (1 / 2.4) - 0.055)
    np.testing.assert_allclose(t.pixelsf[..., :3], np.round(enc * 65535) / 65535, atol=1e-7)
    np.testing.assert_array_equal(sceneio.load_texture(str(f), "clamp").pixelsf[..., :3], c.astype(np.float32))


def test_png_rgb_alpha_is_one_byte(tmp_path):
    from PIL import Image
    a = np.zeros((2, 3, 3), np.uint8)
    Image.fromarray(a, "RGB").save(tmp_path / "x.png")
    t = sceneio.load_texture(str(tmp_path / "x.png"))
    assert np.all(t.pixelsb[..., 3] == 1)  # Vec4b(::RGB) alpha = 1 (src/math.jl:39-44)


def test_save_image_pipeline(tmp_path):
    px = np.array([[[0.0, 0.002, 0.5, 1.0], [2.0, np.nan, 1.0, 0.5]]], np.float32)
    out = sceneio.to_srgb8(px, 2, 1)
    assert out[0, 0].tolist() == [0, round(12.92 * 0.002 * 255), round((1.055 * 0.5 ** (1 / 2.4) - 0.055) * 255), 255]
    assert out[0, 1].tolist() == [255, 0, 255, 128]  # clamp01nan: NaN -> 0, >1 -> 1
    sceneio.save_image(str(tmp_path / "o.png"), px, 2, 1)
    with pytest.raises(ValueError):
        sceneio.save_image(str(tmp_path / "o.jpg"), px, 2, 1)


def test_lookat_camera_and_instance(tmp_path):
    js = {"cameras": [{"name": "cam", "lookat": [0, 1, 5, 0, 1, 0, 0, 1, 0], "aspect": 2.0}],
          "materials": [{"type": "volume"}, {"type": "unknown"}], "shapes": [], "instances": []}
    f = tmp_path / "s.json"
    f.write_text(json.dumps(js))
    sc = sceneio.load_scene(str(f))
    cam = sc.cameras[0]
    assert cam.focus == np.float32(5)  # math_length(eye - center)
    np.testing.assert_allclose(cam.frame, lookat_frame(np.float32([0, 1, 5]), np.float32([0, 1, 0]),
                                                      np.float32([0, 1, 0])))
    np.testing.assert_allclose(cam.frame[6:9], [0, 0, 1])  # w = normalize(eye - center)
    assert [m.type for m in sc.materials] == ["volumetric", "matte"]
    assert find_camera(sc, "nope") == 0 and find_camera(sc, "cam") == 0


def test_missing_assets(tmp_path):
    js = {"cameras": [{}], "shapes": [{"uri": "shapes/missing.ply"}], "textures": [{"uri": "t.png"}],
          "materials": [{"color_tex": 0}], "instances": [{"shape": 0, "material": 0}]}
    f = tmp_path / "s.json"
    f.write_text(json.dumps(js))
    with pytest.raises(Exception):
        sceneio.load_scene(str(f))  # the reference throws on a missing file
    with pytest.warns(UserWarning):
        sc = sceneio.load_scene(str(f), missing="drop")
    assert len(sc.instances) == 0 and sc.materials[0].color_tex == -1


def test_cli_defaults_and_sampler_mapping():
    p = cli.parse_cli_args(["--scene", "x.json"])
    assert (p.resolution, p.samples, p.bounces, p.sampler, p.clamp, p.batch, p.bvhstacksize) == \
        (1280, 512, 8, 1, 10, 1, 128)  # src/cli.jl:14-85
    assert p.output == "tests/test_scene.png" and not p.envhidden
    assert cli.parse_cli_args(["--scene", "x", "--sampler", "naive"]).sampler == 2
    assert cli.parse_cli_args(["--scene", "x", "--sampler", "bogus"]).sampler == 1  # unknown -> path
    with pytest.raises(ValueError):
        cli.parse_cli_args(["--scene", "x", "--clamp", "2.5"])  # Params.clamp::Int -> InexactError
    assert cli.parse_cli_args(["--scene", "x", "--envhidden", "true"]).envhidden is True
