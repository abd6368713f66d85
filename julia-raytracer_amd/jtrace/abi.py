"""ctypes mirror of include/jtrace.h — the C-ABI drop-in boundary.

This is the Python counterpart of the Julia `ccall` shim (julia-raytracer_amd/julia/
JtraceHip.jl): it packs the host scene (scene.jl's SceneData, bvh.jl's SceneBvh,
trace.jl's TraceLights) into the flat, 0-based structs the HIP library consumes.

The product library is libjtrace_hip.so (HIP kernels + C-ABI, built for gfx950). It is loaded
by `load_library()`; there is no CPU fallback: a missing library raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_ROOT = Path(__file__).resolve().parent.parent  # julia-raytracer_amd/
LIB_PATH = PKG_ROOT / "build" / "libjtrace_hip.so"

JT_OK = 0
STATUS_NAMES = {
    0: "JT_OK",
    -1: "JT_ERR_INVALID",
    -2: "JT_ERR_UNSUPPORTED",
    -3: "JT_ERR_DEVICE",
    -4: "JT_ERR_NOMEM",
    -5: "JT_ERR_STACK",
    -6: "JT_ERR_STATE",
}

# MaterialType order of src/scene.jl:191-200
MATERIAL_TYPES = ["matte", "glossy", "reflective", "transparent", "refractive", "subsurface",
                  "volumetric", "gltfpbr"]
# jt_traversal: BVH child visit order (include/jtrace.h)
TRAVERSAL_ORDERS = ["reference", "near", "wide", "auto"]

f32p = C.POINTER(C.c_float)
i32p = C.POINTER(C.c_int32)
u8p = C.POINTER(C.c_uint8)


class jt_camera(C.Structure):
    _fields_ = [("frame", C.c_float * 12), ("orthographic", C.c_int32), ("lens", C.c_float),
                ("film", C.c_float), ("aspect", C.c_float), ("focus", C.c_float),
                ("aperture", C.c_float)]


class jt_instance(C.Structure):
    _fields_ = [("frame", C.c_float * 12), ("shape", C.c_int32), ("material", C.c_int32)]


class jt_environment(C.Structure):
    _fields_ = [("frame", C.c_float * 12), ("emission", C.c_float * 3), ("emission_tex", C.c_int32)]


class jt_material(C.Structure):
    _fields_ = [("type", C.c_int32), ("emission", C.c_float * 3), ("color", C.c_float * 3),
                ("roughness", C.c_float), ("metallic", C.c_float), ("ior", C.c_float),
                ("scattering", C.c_float * 3), ("scanisotropy", C.c_float), ("trdepth", C.c_float),
                ("opacity", C.c_float), ("emission_tex", C.c_int32), ("color_tex", C.c_int32),
                ("roughness_tex", C.c_int32), ("scattering_tex", C.c_int32), ("normal_tex", C.c_int32)]


class jt_texture(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("linear", C.c_int32),
                ("pixelsf", f32p), ("pixelsb", u8p)]


class jt_shape(C.Structure):
    _fields_ = [("npoints", C.c_int32), ("nlines", C.c_int32), ("ntriangles", C.c_int32),
                ("nquads", C.c_int32), ("points", i32p), ("lines", i32p), ("triangles", i32p),
                ("quads", i32p), ("npositions", C.c_int32), ("positions", f32p),
                ("nnormals", C.c_int32), ("normals", f32p), ("ntexcoords", C.c_int32),
                ("texcoords", f32p), ("ncolors", C.c_int32), ("colors", f32p),
                ("nradius", C.c_int32), ("radius", f32p)]


class jt_scene(C.Structure):
    _fields_ = [("ncameras", C.c_int32), ("cameras", C.POINTER(jt_camera)),
                ("ninstances", C.c_int32), ("instances", C.POINTER(jt_instance)),
                ("nenvironments", C.c_int32), ("environments", C.POINTER(jt_environment)),
                ("nshapes", C.c_int32), ("shapes", C.POINTER(jt_shape)),
                ("ntextures", C.c_int32), ("textures", C.POINTER(jt_texture)),
                ("nmaterials", C.c_int32), ("materials", C.POINTER(jt_material))]


class jt_bvh_node(C.Structure):
    _fields_ = [("bmin", C.c_float * 3), ("bmax", C.c_float * 3), ("start", C.c_int32),
                ("num", C.c_int16), ("axis", C.c_int8), ("internal", C.c_int8)]


class jt_bvh_tree(C.Structure):
    _fields_ = [("nnodes", C.c_int32), ("nodes", C.POINTER(jt_bvh_node)),
                ("nprimitives", C.c_int32), ("primitives", i32p)]


class jt_scene_bvh(C.Structure):
    _fields_ = [("tlas", jt_bvh_tree), ("nshapes", C.c_int32), ("blas", C.POINTER(jt_bvh_tree))]


class jt_light(C.Structure):
    _fields_ = [("instance", C.c_int32), ("environment", C.c_int32), ("ncdf", C.c_int32),
                ("cdf", f32p)]


class jt_lights(C.Structure):
    _fields_ = [("nlights", C.c_int32), ("lights", C.POINTER(jt_light))]


class jt_params(C.Structure):
    _fields_ = [("camera", C.c_int32), ("resolution", C.c_int32), ("width", C.c_int32),
                ("height", C.c_int32), ("samples", C.c_int32), ("bounces", C.c_int32),
                ("sampler", C.c_int32), ("clamp", C.c_int32), ("envhidden", C.c_int32),
                ("tentfilter", C.c_int32), ("nocaustics", C.c_int32), ("batch", C.c_int32),
                ("bvhstacksize", C.c_int32), ("device", C.c_int32), ("seed", C.c_uint64),
                ("traversal", C.c_int32)]


class jt_counters(C.Structure):
    _fields_ = [("paths", C.c_uint64), ("rays", C.c_uint64), ("light_queries", C.c_uint64),
                ("nodes", C.c_uint64), ("instances", C.c_uint64), ("prims", C.c_uint64),
                ("shades", C.c_uint64), ("launches", C.c_uint64), ("kernel_ms", C.c_double)]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class jt_device_buffers(C.Structure):
    _fields_ = [("image", C.c_void_p), ("albedo", C.c_void_p), ("normal", C.c_void_p),
                ("hits", C.c_void_p), ("width", C.c_int32), ("height", C.c_int32),
                ("stream", C.c_void_p)]


assert C.sizeof(jt_bvh_node) == 32


def _ptr(arr: np.ndarray | None, ctype):
    if arr is None or arr.size == 0:
        return C.cast(None, C.POINTER(ctype))
    assert arr.flags["C_CONTIGUOUS"]
    return arr.ctypes.data_as(C.POINTER(ctype))


class SceneABI:
    """Packs a host SceneData (jtrace.scene) into a jt_scene; keeps every buffer alive
    for as long as this object lives (the ccall equivalent of GC.@preserve)."""

    def __init__(self, scene):
        keep = []
        self._keep = keep
        cams = (jt_camera * max(1, len(scene.cameras)))()
        for k, c in enumerate(scene.cameras):
            cams[k].frame[:] = list(map(float, c.frame))
            cams[k].orthographic = int(c.orthographic)
            cams[k].lens, cams[k].film, cams[k].aspect = c.lens, c.film, c.aspect
            cams[k].focus, cams[k].aperture = c.focus, c.aperture
        insts = (jt_instance * max(1, len(scene.instances)))()
        for k, inst in enumerate(scene.instances):
            insts[k].frame[:] = list(map(float, inst.frame))
            insts[k].shape, insts[k].material = inst.shape, inst.material
        envs = (jt_environment * max(1, len(scene.environments)))()
        for k, e in enumerate(scene.environments):
            envs[k].frame[:] = list(map(float, e.frame))
            envs[k].emission[:] = list(map(float, e.emission))
            envs[k].emission_tex = e.emission_tex
        mats = (jt_material * max(1, len(scene.materials)))()
        for k, m in enumerate(scene.materials):
            mm = mats[k]
            mm.type = MATERIAL_TYPES.index(m.type)
            mm.emission[:] = list(map(float, m.emission))
            mm.color[:] = list(map(float, m.color))
            mm.roughness, mm.metallic, mm.ior = m.roughness, m.metallic, m.ior
            mm.scattering[:] = list(map(float, m.scattering))
            mm.scanisotropy, mm.trdepth, mm.opacity = m.scanisotropy, m.trdepth, m.opacity
            mm.emission_tex, mm.color_tex = m.emission_tex, m.color_tex
            mm.roughness_tex, mm.scattering_tex = m.roughness_tex, m.scattering_tex
            mm.normal_tex = m.normal_tex
        texs = (jt_texture * max(1, len(scene.textures)))()
        for k, t in enumerate(scene.textures):
            texs[k].width, texs[k].height, texs[k].linear = t.width, t.height, int(t.linear)
            if t.pixelsf is not None and t.pixelsf.size:
                a = np.ascontiguousarray(t.pixelsf, dtype=np.float32)
                keep.append(a)
                texs[k].pixelsf = _ptr(a, C.c_float)
            else:
                a = np.ascontiguousarray(t.pixelsb, dtype=np.uint8)
                keep.append(a)
                texs[k].pixelsb = _ptr(a, C.c_uint8)
        shps = (jt_shape * max(1, len(scene.shapes)))()
        for k, s in enumerate(scene.shapes):
            sh = shps[k]
            arrs = {}
            for name, dt in (("points", np.int32), ("lines", np.int32), ("triangles", np.int32),
                             ("quads", np.int32), ("positions", np.float32), ("normals", np.float32),
                             ("texcoords", np.float32), ("colors", np.float32), ("radius", np.float32)):
                a = getattr(s, name)
                a = np.ascontiguousarray(a if a is not None else np.zeros((0,), dt), dtype=dt)
                keep.append(a)
                arrs[name] = a
            sh.npoints, sh.nlines = len(arrs["points"]), len(arrs["lines"])
            sh.ntriangles, sh.nquads = len(arrs["triangles"]), len(arrs["quads"])
            sh.points, sh.lines = _ptr(arrs["points"], C.c_int32), _ptr(arrs["lines"], C.c_int32)
            sh.triangles, sh.quads = _ptr(arrs["triangles"], C.c_int32), _ptr(arrs["quads"], C.c_int32)
            sh.npositions, sh.positions = len(arrs["positions"]), _ptr(arrs["positions"], C.c_float)
            sh.nnormals, sh.normals = len(arrs["normals"]), _ptr(arrs["normals"], C.c_float)
            sh.ntexcoords, sh.texcoords = len(arrs["texcoords"]), _ptr(arrs["texcoords"], C.c_float)
            sh.ncolors, sh.colors = len(arrs["colors"]), _ptr(arrs["colors"], C.c_float)
            sh.nradius, sh.radius = len(arrs["radius"]), _ptr(arrs["radius"], C.c_float)
        keep.extend([cams, insts, envs, mats, texs, shps])
        self.struct = jt_scene(len(scene.cameras), cams, len(scene.instances), insts,
                               len(scene.environments), envs, len(scene.shapes), shps,
                               len(scene.textures), texs, len(scene.materials), mats)

    @property
    def ref(self):
        return C.byref(self.struct)


def make_params(params, camera: int = 0) -> jt_params:
    """Params (src/cli.jl:90-138) -> jt_params."""
    p = jt_params()
    p.camera = camera
    p.resolution = int(params.resolution)
    p.width = int(getattr(params, "width", 0) or 0)
    p.height = int(getattr(params, "height", 0) or 0)
    p.samples = int(params.samples)
    p.bounces = int(params.bounces)
    p.sampler = int(params.sampler)
    p.clamp = int(params.clamp)
    p.envhidden = int(params.envhidden)
    p.tentfilter = int(params.tentfilter)
    p.nocaustics = int(params.nocaustics)
    p.batch = int(params.batch)
    p.bvhstacksize = int(params.bvhstacksize)
    p.device = int(getattr(params, "device", 0) or 0)
    p.seed = int(getattr(params, "seed", 0x5EED))
    from .cli import DEFAULT_TRAVERSAL
    p.traversal = TRAVERSAL_ORDERS.index(getattr(params, "traversal", DEFAULT_TRAVERSAL))
    return p


class JTError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")
        self.status = status


_LIB = None


def _declare(lib):
    lib.jt_version.restype = C.c_char_p
    lib.jt_abi_version.restype = C.c_int
    lib.jt_last_error.restype = C.c_char_p
    lib.jt_device_count.argtypes = [i32p]
    lib.jt_set_option.argtypes = [C.c_char_p, C.c_char_p]
    lib.jt_build_scene_bvh.argtypes = [C.POINTER(jt_scene), C.c_int32, C.POINTER(jt_scene_bvh)]
    lib.jt_free_scene_bvh.argtypes = [C.POINTER(jt_scene_bvh)]
    lib.jt_free_scene_bvh.restype = None
    lib.jt_make_lights.argtypes = [C.POINTER(jt_scene), C.POINTER(jt_lights)]
    lib.jt_free_lights.argtypes = [C.POINTER(jt_lights)]
    lib.jt_free_lights.restype = None
    lib.jt_image_size.argtypes = [C.POINTER(jt_scene), C.POINTER(jt_params), i32p, i32p]
    lib.jt_create.argtypes = [C.POINTER(jt_scene), C.POINTER(jt_scene_bvh), C.POINTER(jt_lights),
                              C.POINTER(jt_params), C.POINTER(C.c_void_p)]
    lib.jt_create_multi.argtypes = [C.POINTER(jt_scene), C.POINTER(jt_scene_bvh), C.POINTER(jt_lights),
                                    C.POINTER(jt_params), i32p, C.c_int32, C.POINTER(C.c_void_p)]
    lib.jt_trace_samples.argtypes = [C.c_void_p]
    lib.jt_trace_range.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
    lib.jt_get_samples.argtypes = [C.c_void_p, i32p]
    lib.jt_get_streams.argtypes = [C.c_void_p, i32p]
    lib.jt_get_size.argtypes = [C.c_void_p, i32p, i32p]
    lib.jt_get_image.argtypes = [C.c_void_p, f32p]
    lib.jt_get_aovs.argtypes = [C.c_void_p, f32p, f32p, C.POINTER(C.c_int64)]
    lib.jt_get_counters.argtypes = [C.c_void_p, C.POINTER(jt_counters)]
    lib.jt_reset.argtypes = [C.c_void_p]
    lib.jt_get_device_buffers.argtypes = [C.c_void_p, C.POINTER(jt_device_buffers)]
    lib.jt_set_counters.argtypes = [C.c_void_p, C.c_int32]
    lib.jt_synchronize.argtypes = [C.c_void_p]
    lib.jt_describe.argtypes = [C.c_void_p, C.c_char_p, C.c_int32]
    lib.jt_destroy.argtypes = [C.c_void_p]
    lib.jt_destroy.restype = None
    return lib


# every symbol include/jtrace.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = [
    "jt_version", "jt_abi_version", "jt_last_error", "jt_device_count", "jt_set_option", "jt_build_scene_bvh",
    "jt_free_scene_bvh", "jt_make_lights", "jt_free_lights", "jt_image_size", "jt_create", "jt_create_multi",
    "jt_trace_samples", "jt_trace_range", "jt_get_streams", "jt_get_samples", "jt_get_size", "jt_get_image",
    "jt_get_aovs", "jt_get_counters", "jt_reset", "jt_get_device_buffers", "jt_set_counters", "jt_describe", "jt_synchronize",
    "jt_destroy",
]


def load_library(path: str | os.PathLike | None = None):
    """Load the HIP product library. Raises if it has not been built — there is no fallback."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = Path(path) if path else Path(os.environ.get("JTRACE_LIB", LIB_PATH))
    if not p.exists():
        raise RuntimeError(f"jtrace HIP library not found at {p}; run `make -C julia-raytracer_amd` "
                           "(or __graft_entry__.build()) — the product path has no CPU fallback")
    lib = _declare(C.CDLL(str(p), mode=C.RTLD_GLOBAL))
    if path is None:
        _LIB = lib
    return lib


def set_option(lib, name: str | None, value=None):
    """jt_set_option (include/jtrace.h): a process-wide run-time option for the contexts created
    afterwards; value None removes it, name None removes every option."""
    check(lib, lib.jt_set_option(None if name is None else name.encode(),
                                 None if value is None else str(value).encode()))


def check(lib, status: int):
    if status != JT_OK:
        msg = lib.jt_last_error()
        raise JTError(status, msg.decode() if msg else "")
    return status
