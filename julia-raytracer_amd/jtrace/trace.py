"""Trace module host mirror — src/trace.jl's public surface over the HIP C-ABI.

    make_trace_lights(scene)        src/trace.jl:117   -> jt_make_lights
    make_scene_bvh(scene, hq)       src/bvh.jl:66      -> jt_build_scene_bvh
    TraceState / make_trace_state   src/trace.jl:87,189 -> jt_create (device context)
    trace_samples(state)            src/trace.jl:215   -> jt_trace_samples (one batch)
    get_image(state)                src/trace.jl:676   -> jt_get_image

There is no CPU fallback anywhere in this module: every call goes through libjtrace_hip.so.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


class SceneBvh:
    """Owns a jt_scene_bvh built by the library (make_scene_bvh, src/bvh.jl:66-88)."""

    def __init__(self, scene_abi: abi.SceneABI, high_quality: bool = False, lib=None):
        self.lib = lib or abi.load_library()
        self.struct = abi.jt_scene_bvh()
        abi.check(self.lib, self.lib.jt_build_scene_bvh(scene_abi.ref, int(high_quality), C.byref(self.struct)))

    @property
    def ref(self):
        return C.byref(self.struct)

    def tree(self, which: int = -1):
        """(nodes structured array, primitives) of the TLAS (which=-1) or BLAS `which`."""
        t = self.struct.tlas if which < 0 else self.struct.blas[which]
        nodes = np.ctypeslib.as_array(C.cast(t.nodes, C.POINTER(C.c_uint8)), shape=(t.nnodes * 32,))
        dt = np.dtype([("bmin", "<f4", 3), ("bmax", "<f4", 3), ("start", "<i4"), ("num", "<i2"),
                       ("axis", "i1"), ("internal", "i1")])
        prims = np.ctypeslib.as_array(t.primitives, shape=(t.nprimitives,)) if t.nprimitives else np.zeros(0, np.int32)
        return nodes.view(dt).copy(), prims.copy()

    def __del__(self):
        if getattr(self, "lib", None) is not None and getattr(self, "struct", None) is not None:
            self.lib.jt_free_scene_bvh(C.byref(self.struct))


class TraceLights:
    """Owns a jt_lights built by the library (make_trace_lights, src/trace.jl:117-187)."""

    def __init__(self, scene_abi: abi.SceneABI, lib=None):
        self.lib = lib or abi.load_library()
        self.struct = abi.jt_lights()
        abi.check(self.lib, self.lib.jt_make_lights(scene_abi.ref, C.byref(self.struct)))

    @property
    def ref(self):
        return C.byref(self.struct)

    def cdfs(self):
        out = []
        for k in range(self.struct.nlights):
            light = self.struct.lights[k]
            out.append((light.instance, light.environment,
                        np.ctypeslib.as_array(light.cdf, shape=(light.ncdf,)).copy()))
        return out

    def __del__(self):
        if getattr(self, "lib", None) is not None and getattr(self, "struct", None) is not None:
            self.lib.jt_free_lights(C.byref(self.struct))


def make_scene_bvh(scene_abi, high_quality=False, lib=None) -> SceneBvh:
    return SceneBvh(scene_abi, high_quality, lib)


def make_trace_lights(scene_abi, lib=None) -> TraceLights:
    return TraceLights(scene_abi, lib)


def image_size(scene_abi, params: abi.jt_params, lib=None):
    lib = lib or abi.load_library()
    w, h = C.c_int32(), C.c_int32()
    abi.check(lib, lib.jt_image_size(scene_abi.ref, C.byref(params), C.byref(w), C.byref(h)))
    return w.value, h.value


class TraceState:
    """Device-resident TraceState (src/trace.jl:87-100): running-mean image/albedo/normal/hits."""

    def __init__(self, scene_abi, bvh: SceneBvh, lights: TraceLights, params: abi.jt_params, lib=None,
                 devices=None):
        """devices: None for one context on params.device (jt_create), or a list of HIP
        ordinals for one context over those GPUs (jt_create_multi: every batch sharded across
        them, the running means reduced with RCCL when read)."""
        self.lib = lib or abi.load_library()
        self._keep = (scene_abi, bvh, lights)
        self.params = params
        h = C.c_void_p()
        if devices is None:
            abi.check(self.lib, self.lib.jt_create(scene_abi.ref, bvh.ref, lights.ref, C.byref(params), C.byref(h)))
        else:
            devs = (C.c_int32 * len(devices))(*devices)
            abi.check(self.lib, self.lib.jt_create_multi(scene_abi.ref, bvh.ref, lights.ref, C.byref(params), devs,
                                                         len(devices), C.byref(h)))
        self.devices = devices
        self.handle = h
        w, hh = C.c_int32(), C.c_int32()
        abi.check(self.lib, self.lib.jt_get_size(self.handle, C.byref(w), C.byref(hh)))
        self.width, self.height = w.value, hh.value

    # --- trace.jl surface
    def trace_samples(self):
        abi.check(self.lib, self.lib.jt_trace_samples(self.handle))

    def trace_range(self, s0: int, s1: int):
        abi.check(self.lib, self.lib.jt_trace_range(self.handle, int(s0), int(s1)))

    @property
    def samples(self) -> int:
        n = C.c_int32()
        abi.check(self.lib, self.lib.jt_get_samples(self.handle, C.byref(n)))
        return n.value

    @property
    def streams(self) -> int:
        """Sample streams per pixel k (jt_get_streams): local sample t goes to stream t mod k, and
        the image is the streams' running means combined in stream order (include/jtrace.h)."""
        n = C.c_int32()
        abi.check(self.lib, self.lib.jt_get_streams(self.handle, C.byref(n)))
        return n.value

    def get_image(self) -> np.ndarray:
        out = np.empty((self.height, self.width, 4), np.float32)
        abi.check(self.lib, self.lib.jt_get_image(self.handle, out.ctypes.data_as(abi.f32p)))
        return out

    def get_aovs(self):
        n = self.width * self.height
        alb = np.empty((self.height, self.width, 3), np.float32)
        nrm = np.empty((self.height, self.width, 3), np.float32)
        hits = np.empty((self.height, self.width), np.int64)
        abi.check(self.lib, self.lib.jt_get_aovs(self.handle, alb.ctypes.data_as(abi.f32p),
                                                 nrm.ctypes.data_as(abi.f32p),
                                                 hits.ctypes.data_as(C.POINTER(C.c_int64))))
        del n
        return alb, nrm, hits

    def counters(self) -> dict:
        c = abi.jt_counters()
        abi.check(self.lib, self.lib.jt_get_counters(self.handle, C.byref(c)))
        return c.as_dict()

    def device_buffers(self) -> abi.jt_device_buffers:
        b = abi.jt_device_buffers()
        abi.check(self.lib, self.lib.jt_get_device_buffers(self.handle, C.byref(b)))
        return b

    def set_counters(self, level: int):
        abi.check(self.lib, self.lib.jt_set_counters(self.handle, int(level)))

    def describe(self) -> str:
        """Launch configuration of the next trace_range (kernel instance, scene mode, grid)."""
        buf = C.create_string_buffer(1024)
        abi.check(self.lib, self.lib.jt_describe(self.handle, buf, 1024))
        return buf.value.decode()

    @property
    def traversal(self) -> str:
        """The BVH traversal this context runs ("reference", "near" or "wide"): jt_params.traversal,
        with "auto" resolved by the library (wide for a scene in HBM mode with a stack bound above 32, near otherwise)."""
        for tok in self.describe().split():
            if tok.startswith("traversal="):
                return tok.split("=", 1)[1]
        raise RuntimeError("jt_describe reports no traversal")

    def reset(self):
        abi.check(self.lib, self.lib.jt_reset(self.handle))

    def synchronize(self):
        abi.check(self.lib, self.lib.jt_synchronize(self.handle))

    def close(self):
        if getattr(self, "handle", None):
            self.lib.jt_destroy(self.handle)
            self.handle = None

    def __del__(self):
        self.close()


def make_trace_state(scene_abi, bvh, lights, params, lib=None, devices=None) -> TraceState:
    return TraceState(scene_abi, bvh, lights, params, lib, devices)


def trace_samples(state: TraceState):
    state.trace_samples()


def get_image(state: TraceState) -> np.ndarray:
    return state.get_image()
