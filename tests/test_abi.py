"""The C-ABI library loads on the CPU and exports exactly what include/jtrace.h declares;
struct layouts agree between the header and the ctypes mirror; input validation errors are
reported (not thrown) before any device work."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import ROOT, make_params

HEADER = ROOT / "include" / "jtrace.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(jt_[a-z_]+)\s*\(", text)))


def test_header_and_mirror_agree(abi):
    assert declared_functions() == sorted(abi.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", str(Path(lib._name))], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\b[TW] (jt_[a-z_]+)\b", out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing


def test_version(lib):
    assert lib.jt_abi_version() == 5  # 2: jt_params.traversal, 3: jt_set_option, 4: sample streams, 5: deferred ranges
    assert b"gfx950" in lib.jt_version()


def _check_build_matches_source(lib):
    import sys
    sys.path.insert(0, str(ROOT / "scripts"))
    from roofline import source_hash
    m = re.search(r"source ([0-9a-f]{16}|unknown)\)", lib.jt_version().decode())
    assert m, lib.jt_version()
    assert m.group(1) == source_hash(), (f"the loaded library was built from other sources ({m.group(1)}) than "
                                         f"this tree ({source_hash()}): rebuild with make -C julia-raytracer_amd")


def test_library_built_from_this_source(lib):
    """jt_version() carries the source hash the Makefile embedded (every csrc/ file, the Makefile,
    the ABI header, the hipcc version): the loaded binary was built from these sources."""
    _check_build_matches_source(lib)


@pytest.mark.gpu
def test_gpu_box_library_built_from_this_source(gpu, lib):
    """The same check where the GPU tests run: the prebuilt library that travelled to the box
    was built from the committed sources, not from an older tree."""
    _check_build_matches_source(lib)


def test_run_time_options_are_explicit(abi, lib):
    """Run-time options come only from jt_set_option: unknown names are rejected, known ones set
    and clear, and the library never reads the environment (no getenv in the sources)."""
    assert lib.jt_set_option(b"no_such_option", b"1") == -1
    assert b"unknown option" in lib.jt_last_error()
    for name in ("env_alias", "features", "lds_scene", "lds_stack", "light_inline", "streams",
                 "wait_lanes", "light_lanes", "multi_split", "tile_share", "test_lds_ring"):
        assert lib.jt_set_option(name.encode(), b"1") == 0
        assert lib.jt_set_option(name.encode(), None) == 0
    assert lib.jt_set_option(None, b"1") == -1
    assert lib.jt_set_option(None, None) == 0
    for src in (ROOT / "julia-raytracer_amd" / "csrc").glob("*"):
        assert "getenv" not in src.read_text(), src


STRUCTS = ["jt_camera", "jt_instance", "jt_environment", "jt_material", "jt_texture", "jt_shape", "jt_scene",
           "jt_bvh_node", "jt_bvh_tree", "jt_scene_bvh", "jt_light", "jt_lights", "jt_params", "jt_counters",
           "jt_device_buffers"]


def test_struct_layouts_match_header(abi, tmp_path):
    src = tmp_path / "sz.c"
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for s in STRUCTS:
        lines.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for f, _ in getattr(abi, s)._fields_:
            lines.append(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));')
    lines.append("return 0;}")
    src.write_text("\n".join(lines))
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n") if l)
    for s in STRUCTS:
        cls = getattr(abi, s)
        assert int(got[s]) == C.sizeof(cls), s
        for f, _ in cls._fields_:
            assert int(got[f"{s}.{f}"]) == getattr(cls, f).offset, (s, f)


def _create(abi, lib, scene_abi, **kw):
    from jtrace import trace
    bvh = trace.make_scene_bvh(scene_abi, False, lib)
    lights = trace.make_trace_lights(scene_abi, lib)
    p = make_params(abi, **kw)
    h = C.c_void_p()
    st = lib.jt_create(scene_abi.ref, bvh.ref, lights.ref, C.byref(p), C.byref(h))
    if st == 0:
        lib.jt_destroy(h)
    return st, lib.jt_last_error().decode()


def test_create_rejects_what_the_reference_cannot_shade(abi, lib, cornell):
    import copy
    sc = copy.deepcopy(cornell)
    sc.materials[0].type = "gltfpbr"  # src/shading.jl:254-321 calls undefined functions
    st, msg = _create(abi, lib, abi.SceneABI(sc))
    assert st == -2 and "gltfpbr" in msg


def test_create_rejects_bad_params(abi, lib, cornell_abi):
    st, msg = _create(abi, lib, cornell_abi, sampler=3)
    assert st == -1 and "sampler" in msg
    st, msg = _create(abi, lib, cornell_abi, camera=5)
    assert st == -1 and "camera" in msg
    st, msg = _create(abi, lib, cornell_abi, bvhstacksize=2)
    assert st == -5  # the reference throws BoundsError


def test_untextured_environment_light_is_rejected(abi, lib, cornell):
    import copy
    from jtrace.scene import EnvironmentData, identity_frame
    sc = copy.deepcopy(cornell)
    sc.environments.append(EnvironmentData(frame=identity_frame(), emission=np.ones(3, np.float32)))
    lights = abi.jt_lights()
    st = lib.jt_make_lights(abi.SceneABI(sc).ref, C.byref(lights))
    assert st == -2 and "l_elements_cdf" in lib.jt_last_error().decode()


def test_image_size_follows_make_trace_state(abi, lib, cornell, cornell_abi):
    from jtrace import trace
    assert trace.image_size(cornell_abi, make_params(abi, resolution=1280), lib) == (1280, 1280)
    assert trace.image_size(cornell_abi, make_params(abi, width=1280, height=720), lib) == (1280, 720)
    import copy
    sc = copy.deepcopy(cornell)
    sc.cameras[0].aspect = np.float32(2.4)  # features2: 1920 x round(1920/2.4) = 800
    assert trace.image_size(abi.SceneABI(sc), make_params(abi, resolution=1920), lib) == (1920, 800)
    sc.cameras[0].aspect = np.float32(0.5)
    assert trace.image_size(abi.SceneABI(sc), make_params(abi, resolution=100), lib) == (50, 100)
