"""Host scene model — mirror of the reference's Scene module (src/scene.jl:48-370).

Field names, JSON keys, defaults and the lookat handling follow the reference constructors;
ids are stored 0-based (the reference adds 1 to the JSON ids; invalid_id = -1 either way).
All float fields are float32, as in the reference structs.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

f32 = np.float32
INVALID_ID = -1  # src/scene.jl:45

# MaterialTypes (src/scene.jl:201-211): JSON name -> enum name
MATERIAL_TYPES = {
    "matte": "matte", "glossy": "glossy", "reflective": "reflective",
    "transparent": "transparent", "refractive": "refractive", "subsurface": "subsurface",
    "volume": "volumetric", "volumetric": "volumetric", "gltfpbr": "gltfpbr",
}


def _v3(x) -> np.ndarray:
    return np.asarray(x, dtype=np.float32).reshape(3)


def _dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def _normalize(a):
    ln = np.sqrt(_dot(a, a))
    return a / ln if ln != 0 else a


def _cross(a, b):
    return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2],
                     a[0] * b[1] - a[1] * b[0]], dtype=np.float32)


def identity_frame() -> np.ndarray:
    return np.array([1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0], dtype=np.float32)


def frame_from_json(arr) -> np.ndarray:
    """Frame3f(array) (src/math.jl:47-60): identity unless exactly 12 values."""
    a = np.asarray(arr if arr is not None else [], dtype=np.float32).reshape(-1)
    return a.copy() if a.size == 12 else identity_frame()


def lookat_frame(eye, center, up, inv_xz: bool = False) -> np.ndarray:
    """lookat_frame (src/math.jl:146-155), float32 arithmetic in source order."""
    w = _normalize(eye - center)
    u = _normalize(_cross(up, w))
    v = _normalize(_cross(w, u))
    if inv_xz:
        w, u = -w, -u
    return np.concatenate([u, v, w, eye]).astype(np.float32)


def _lookat(json, frame, inv_xz):
    la = np.asarray(json["lookat"], dtype=np.float32).reshape(-1)
    eye, center, up = la[0:3], la[3:6], la[6:9]
    return lookat_frame(eye, center, up, inv_xz), eye, center


@dataclass
class CameraData:  # src/scene.jl:48-86
    frame: np.ndarray
    orthographic: bool = False
    lens: float = f32(0.050)
    film: float = f32(0.036)
    aspect: float = f32(1.5)
    focus: float = f32(10000)
    aperture: float = f32(0)
    name: str = ""

    @classmethod
    def from_json(cls, j) -> "CameraData":
        frame = frame_from_json(j.get("frame"))
        focus = f32(j.get("focus", 10000))
        if "lookat" in j:
            frame, eye, center = _lookat(j, frame, False)
            d = eye - center
            focus = f32(np.sqrt(_dot(d, d)))
        return cls(frame=frame, orthographic=bool(j.get("orthographic", False)),
                   lens=f32(j.get("lens", 0.050)), film=f32(j.get("film", 0.036)),
                   aspect=f32(j.get("aspect", 1.5)), focus=focus,
                   aperture=f32(j.get("aperture", 0)), name=j.get("name", ""))


@dataclass
class InstanceData:  # src/scene.jl:88-115
    frame: np.ndarray
    shape: int = INVALID_ID
    material: int = INVALID_ID
    name: str = ""

    @classmethod
    def from_json(cls, j) -> "InstanceData":
        frame = frame_from_json(j.get("frame"))
        if "lookat" in j:
            frame, _, _ = _lookat(j, frame, True)
        return cls(frame=frame, shape=int(j.get("shape", INVALID_ID)),
                   material=int(j.get("material", INVALID_ID)), name=j.get("name", ""))


@dataclass
class EnvironmentData:  # src/scene.jl:117-144
    frame: np.ndarray
    emission: np.ndarray
    emission_tex: int = INVALID_ID
    name: str = ""

    @classmethod
    def from_json(cls, j) -> "EnvironmentData":
        frame = frame_from_json(j.get("frame"))
        if "lookat" in j:
            frame, _, _ = _lookat(j, frame, True)
        return cls(frame=frame, emission=_v3(j.get("emission", [0, 0, 0])),
                   emission_tex=int(j.get("emission_tex", INVALID_ID)), name=j.get("name", ""))


@dataclass
class MaterialData:  # src/scene.jl:213-264
    type: str = "matte"
    emission: np.ndarray = field(default_factory=lambda: np.zeros(3, np.float32))
    color: np.ndarray = field(default_factory=lambda: np.zeros(3, np.float32))
    roughness: float = f32(0)
    metallic: float = f32(0)
    ior: float = f32(1.5)
    scattering: np.ndarray = field(default_factory=lambda: np.zeros(3, np.float32))
    scanisotropy: float = f32(0)
    trdepth: float = f32(0.01)
    opacity: float = f32(1)
    emission_tex: int = INVALID_ID
    color_tex: int = INVALID_ID
    roughness_tex: int = INVALID_ID
    scattering_tex: int = INVALID_ID
    normal_tex: int = INVALID_ID
    name: str = ""

    @classmethod
    def from_json(cls, j) -> "MaterialData":
        return cls(type=MATERIAL_TYPES.get(j.get("type", "matte"), "matte"),
                   emission=_v3(j.get("emission", [0, 0, 0])), color=_v3(j.get("color", [0, 0, 0])),
                   roughness=f32(j.get("roughness", 0)), metallic=f32(j.get("metallic", 0)),
                   ior=f32(j.get("ior", 1.5)), scattering=_v3(j.get("scattering", [0, 0, 0])),
                   scanisotropy=f32(j.get("scanisotropy", 0)), trdepth=f32(j.get("trdepth", 0.01)),
                   opacity=f32(j.get("opacity", 1)),
                   emission_tex=int(j.get("emission_tex", INVALID_ID)),
                   color_tex=int(j.get("color_tex", INVALID_ID)),
                   roughness_tex=int(j.get("roughness_tex", INVALID_ID)),
                   scattering_tex=int(j.get("scattering_tex", INVALID_ID)),
                   normal_tex=int(j.get("normal_tex", INVALID_ID)), name=j.get("name", ""))


@dataclass
class TextureData:  # src/scene.jl:146-162 — row-major RGBA, top row first
    width: int = 0
    height: int = 0
    linear: bool = False
    pixelsf: np.ndarray | None = None  # (H, W, 4) float32
    pixelsb: np.ndarray | None = None  # (H, W, 4) uint8


def _empty(shape, dtype):
    return np.zeros(shape, dtype=dtype)


@dataclass
class ShapeData:  # src/shape.jl:13-48 — indices 0-based
    points: np.ndarray = field(default_factory=lambda: _empty((0,), np.int32))
    lines: np.ndarray = field(default_factory=lambda: _empty((0, 2), np.int32))
    triangles: np.ndarray = field(default_factory=lambda: _empty((0, 3), np.int32))
    quads: np.ndarray = field(default_factory=lambda: _empty((0, 4), np.int32))
    positions: np.ndarray = field(default_factory=lambda: _empty((0, 3), np.float32))
    normals: np.ndarray = field(default_factory=lambda: _empty((0, 3), np.float32))
    texcoords: np.ndarray = field(default_factory=lambda: _empty((0, 2), np.float32))
    colors: np.ndarray = field(default_factory=lambda: _empty((0, 4), np.float32))
    radius: np.ndarray = field(default_factory=lambda: _empty((0,), np.float32))


@dataclass
class SceneData:  # src/scene.jl:337-356
    cameras: list = field(default_factory=list)
    instances: list = field(default_factory=list)
    environments: list = field(default_factory=list)
    shapes: list = field(default_factory=list)
    textures: list = field(default_factory=list)
    materials: list = field(default_factory=list)
    notes: list = field(default_factory=list)  # substitutions made for missing assets


def find_camera(scene: SceneData, name: str) -> int:
    """find_camera (src/scene.jl:358-370), 0-based (-1 when the scene has no camera)."""
    if len(scene.cameras) == 0:
        return INVALID_ID
    for n in [name, "default", "camera", "camera0", "camera1"]:
        for i, c in enumerate(scene.cameras):
            if c.name == n:
                return i
    return 0
