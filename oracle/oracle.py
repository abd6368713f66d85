"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (oracle/jt_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / the timed CPU baseline — never on the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "libjt_oracle.so"


def build():
    subprocess.run(["make", "-C", str(HERE)], check=True, capture_output=True)


def _load(abi):
    if not LIB.exists():
        build()
    lib = C.CDLL(str(LIB))
    lib.or_build_scene_bvh.argtypes = [C.POINTER(abi.jt_scene), C.c_int32, C.POINTER(abi.jt_scene_bvh)]
    lib.or_free_scene_bvh.argtypes = [C.POINTER(abi.jt_scene_bvh)]
    lib.or_free_scene_bvh.restype = None
    lib.or_make_lights.argtypes = [C.POINTER(abi.jt_scene), C.POINTER(abi.jt_lights)]
    lib.or_free_lights.argtypes = [C.POINTER(abi.jt_lights)]
    lib.or_free_lights.restype = None
    f32p, i64p = C.POINTER(C.c_float), C.POINTER(C.c_int64)
    lib.or_trace_rows.argtypes = [C.POINTER(abi.jt_scene), C.POINTER(abi.jt_scene_bvh), C.POINTER(abi.jt_lights),
                                  C.POINTER(abi.jt_params), C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                  C.c_int32, C.c_int32, C.c_int32, f32p, f32p, f32p, i64p, C.c_int32,
                                  f32p, f32p, f32p, i64p, C.c_int32, C.POINTER(Counters)]
    lib.or_order_diff.argtypes = [C.POINTER(abi.jt_scene), C.POINTER(abi.jt_scene_bvh), C.POINTER(abi.jt_lights),
                                  C.POINTER(abi.jt_params), C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                  C.c_int32, C.POINTER(C.c_uint64)]
    lib.or_intersect_triangle.argtypes = [f32p, f32p, C.c_float, C.c_float, f32p, f32p, f32p, f32p]
    lib.or_intersect_bbox.argtypes = [f32p, f32p, C.c_float, C.c_float, f32p, f32p]
    lib.or_fresnel_dielectric.argtypes = [C.c_float, f32p, f32p]
    lib.or_fresnel_dielectric.restype = C.c_float
    lib.or_rng_first.argtypes = [C.c_uint64, C.c_int32, C.c_int32, C.c_int32, f32p]
    lib.or_rng_first.restype = None
    lib.or_inverse_frame.argtypes = [f32p, C.c_int32, f32p]
    lib.or_inverse_frame.restype = None
    lib.or_srgb_to_rgb.argtypes = [C.POINTER(C.c_uint8), C.c_int32, f32p]
    lib.or_srgb_to_rgb.restype = None
    lib.or_set_env_alias.argtypes = [C.c_int32]
    lib.or_set_env_alias.restype = None
    lib.or_alias_table.argtypes = [f32p, C.c_int32, f32p, C.POINTER(C.c_int32)]
    lib.or_wide_check.argtypes = [C.POINTER(abi.jt_bvh_tree), C.POINTER(abi.jt_bvh_tree), C.c_int32,
                                  C.POINTER(C.c_int64)]
    return lib


class Counters(C.Structure):
    _fields_ = [("paths", C.c_uint64), ("rays", C.c_uint64), ("light_queries", C.c_uint64),
                ("nodes", C.c_uint64), ("instances", C.c_uint64), ("prims", C.c_uint64),
                ("shades", C.c_uint64)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class Oracle:
    def __init__(self, abi):
        self.abi = abi
        self.lib = _load(abi)

    def build_bvh(self, scene_abi, high_quality=False):
        out = self.abi.jt_scene_bvh()
        st = self.lib.or_build_scene_bvh(scene_abi.ref, int(high_quality), C.byref(out))
        if st != 0:
            raise RuntimeError(f"oracle bvh build failed: {st}")
        return _Owned(out, self.lib.or_free_scene_bvh)

    def make_lights(self, scene_abi):
        out = self.abi.jt_lights()
        st = self.lib.or_make_lights(scene_abi.ref, C.byref(out))
        if st != 0:
            raise RuntimeError(f"oracle lights failed: {st}")
        return _Owned(out, self.lib.or_free_lights)

    def alias_table(self, cdf):
        """The env_alias option's Vose table of one light CDF: (keep (n,) float32, other (n,) int32)."""
        cdf = np.ascontiguousarray(cdf, np.float32)
        keep = np.empty(len(cdf), np.float32)
        other = np.empty(len(cdf), np.int32)
        st = self.lib.or_alias_table(cdf.ctypes.data_as(C.POINTER(C.c_float)), len(cdf),
                                     keep.ctypes.data_as(C.POINTER(C.c_float)), other.ctypes.data_as(C.POINTER(C.c_int32)))
        if st != 0:
            raise RuntimeError(f"oracle alias table failed: {st}")
        return keep, other

    def wide_check(self, bvh):
        """The wide records of every tree of `bvh` (JT_TRAVERSAL_WIDE): dict of records,
        non-conservative children (must be 0), leaves, mean dequantised/exact box volume ratio."""
        out = (C.c_int64 * 4)()
        b = bvh.struct
        st = self.lib.or_wide_check(C.byref(b.tlas), b.blas, b.nshapes, out)
        if st != 0:
            raise RuntimeError(f"oracle wide check failed: {st}")
        return {"records": out[0], "violations": out[1], "leaves": out[2], "volume_ratio": out[3] / 1000.0}

    def trace(self, scene_abi, bvh, lights, params, width, height, s0, s1, first=0, rows=None,
              nthreads=None, state=None, streams=1, parts=None, env_alias=False):
        """Returns (image (H,W,4), albedo (H,W,3), normal (H,W,3), hits (H,W), counters).

        streams: the sample streams per pixel k (a power of two, the library's jt_get_streams;
        include/jtrace.h jt_trace_range states the contract). For k > 1 the streams' running
        means are kept in `parts` (a dict of arrays, created when None and filled in place), which
        a caller passes again to continue the same render with a later range.

        env_alias: restate the library's env_alias option (environment texels drawn through
        alias tables, oracle/jt_oracle.c) for this call."""
        if params.traversal not in (0, 1, 2):
            raise ValueError(f"the oracle restates an explicit BVH order (0 reference, 1 near, 2 wide), got "
                             f"{params.traversal}: resolve auto (3) to the order the library ran first")
        k = int(streams)
        if k < 1 or k > 64 or k & (k - 1):
            raise ValueError(f"streams must be a power of two in [1, 64], got {streams}")
        lk = k.bit_length() - 1
        if nthreads is None:
            nthreads = min(16, os.cpu_count() or 1)
        if state is None:
            image = np.zeros((height, width, 4), np.float32)
            albedo = np.zeros((height, width, 3), np.float32)
            normal = np.zeros((height, width, 3), np.float32)
            hits = np.zeros((height, width), np.int64)
        else:
            image, albedo, normal, hits = state
        f32p = C.POINTER(C.c_float)
        i64p = C.POINTER(C.c_int64)
        if lk > 0:
            if parts is None:
                parts = {}
            if not parts:
                parts.update(img=np.zeros((k, height, width, 4), np.float32),
                             alb=np.zeros((k, height, width, 3), np.float32),
                             nrm=np.zeros((k, height, width, 3), np.float32),
                             hits=np.zeros((k, height, width), np.int64))
            pp = (parts["img"].ctypes.data_as(f32p), parts["alb"].ctypes.data_as(f32p),
                  parts["nrm"].ctypes.data_as(f32p), parts["hits"].ctypes.data_as(i64p))
        else:
            pp = (None, None, None, None)
        r0, r1 = rows if rows is not None else (0, height)
        cnt = Counters()
        self.lib.or_set_env_alias(int(bool(env_alias)))
        try:
            st = self._trace_rows(scene_abi, bvh, lights, params, width, height, r0, r1, first, s0, s1, image, albedo,
                                  normal, hits, lk, pp, nthreads, cnt)
        finally:
            self.lib.or_set_env_alias(0)
        if st != 0:
            raise RuntimeError(f"oracle trace failed: {st}")
        return image, albedo, normal, hits, cnt.as_dict()

    def _trace_rows(self, scene_abi, bvh, lights, params, width, height, r0, r1, first, s0, s1, image, albedo,
                    normal, hits, lk, pp, nthreads, cnt):
        f32p = C.POINTER(C.c_float)
        i64p = C.POINTER(C.c_int64)
        return self.lib.or_trace_rows(scene_abi.ref, C.byref(bvh.struct), C.byref(lights.struct), C.byref(params),
                                    width, height, r0, r1, first, s0, s1, image.ctypes.data_as(f32p),
                                    albedo.ctypes.data_as(f32p), normal.ctypes.data_as(f32p),
                                    hits.ctypes.data_as(i64p), lk, *pp, nthreads, C.byref(cnt))


    def order_diff(self, scene_abi, bvh, lights, params, alt_traversal, width, height, s0, s1, nthreads=None):
        """Diagnostic: trace [s0, s1) in params.traversal and compare every closest-hit scene query
        with the same query in alt_traversal (oracle/jt_oracle.c or_order_diff)."""
        if nthreads is None:
            nthreads = min(16, os.cpu_count() or 1)
        d = (C.c_uint64 * 10)()
        st = self.lib.or_order_diff(scene_abi.ref, C.byref(bvh.struct), C.byref(lights.struct), C.byref(params),
                                    alt_traversal, width, height, s0, s1, nthreads, d)
        if st != 0:
            raise RuntimeError(f"oracle order_diff failed: {st}")
        keys = ("queries", "same", "tie", "alt_only_hit", "ref_only_hit", "alt_closer", "alt_farther", "paths_differing")
        return {k: int(d[i]) for i, k in enumerate(keys)}


class _Owned:
    def __init__(self, struct, free):
        self.struct = struct
        self._free = free

    @property
    def ref(self):
        return C.byref(self.struct)

    def __del__(self):
        try:
            self._free(C.byref(self.struct))
        except Exception:
            pass
