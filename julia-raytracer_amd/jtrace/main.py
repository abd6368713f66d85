"""Jtrace.main mirror (src/jtrace.jl:31-118): same stage banners, timers and progress lines.

    python -m jtrace --scene assets/scenes/cornellbox/cornellbox.json --samples 256 --output out.png

Scene load, BVH build, lights and PNG write are host work (as in the reference); the
per-sample loop is the HIP library behind jt_trace_samples.
"""
from __future__ import annotations

import math
import sys
import time

from . import abi
from .cli import Params, parse_cli_args
from .scene import find_camera
from .sceneio import load_scene, save_image
from .trace import make_scene_bvh, make_trace_lights, make_trace_state


def format_seconds(seconds: float) -> str:
    """format_seconds (src/utils.jl:10-32)."""
    hours = math.floor(seconds / 3600)
    minutes = math.floor((seconds - hours * 3600) / 60)
    seconds = seconds - hours * 3600 - minutes * 60
    i_seconds = math.floor(seconds)
    ms = round((seconds - i_seconds) * 1000)
    if hours == 0:
        if minutes == 0:
            return f"{i_seconds:02d}.{ms:03d}"
        return f"{minutes:02d}:{i_seconds:02d}.{ms:03d}"
    return f"{hours:02d}:{minutes:02d}:{i_seconds:02d}.{ms:03d}"


def run(params: Params, out=print) -> dict:
    if params.addsky:
        out("addsky is not yet supported")
        params.addsky = False
    if params.envname != "":
        out("envname is not yet supported")
        params.envname = ""
    if params.denoise:
        out("denoise is not yet supported")
        params.denoise = False
    render_start = time.perf_counter()
    out(f"loading scene {params.scene}...")
    t0 = time.perf_counter()
    scene = load_scene(params.scene, params.noparallel, missing=params.missing)
    out(f"loaded scene in {format_seconds(time.perf_counter() - t0)}")
    out("finding camera...")
    camera = find_camera(scene, params.camera if isinstance(params.camera, str) else "")
    lib = abi.load_library()
    scene_abi = abi.SceneABI(scene)
    out("building bvh...")
    t0 = time.perf_counter()
    bvh = make_scene_bvh(scene_abi, params.highqualitybvh, lib)
    out(f"built bvh in {format_seconds(time.perf_counter() - t0)}")
    out("making lights...")
    lights = make_trace_lights(scene_abi, lib)
    out("making state...")
    jp = abi.make_params(params, camera)
    devices = int(getattr(params, "devices", 1) or 1)
    state = make_trace_state(scene_abi, bvh, lights, jp, lib, devices=list(range(devices)) if devices > 1 else None)
    out("tracing samples...")
    sampling_start = time.perf_counter()
    for _ in range(0, params.samples, params.batch):
        batch_start = time.perf_counter()
        state.trace_samples()
        now = time.perf_counter()
        done = state.samples
        etc = (now - sampling_start) / max(done, 1) * (params.samples - done)
        out(f"sample {done:3d}/{params.samples:3d} in {format_seconds(now - batch_start)} "
            f"ETC: {format_seconds(etc)}")
    render_s = time.perf_counter() - sampling_start
    out(f"rendered in {format_seconds(render_s)} ({render_s:.3f}s)")
    out("saving image...")
    image = state.get_image()
    save_image(params.output, image, state.width, state.height)
    out(f"saved image to {params.output}")
    out(f"total time: {format_seconds(time.perf_counter() - render_start)}")
    counters = state.counters()
    state.close()
    return {"render_s": render_s, "width": state.width, "height": state.height, "counters": counters}


def main(args=None):
    """Jtrace.main(args::String) (src/jtrace.jl:116)."""
    if args is None:
        args = sys.argv[1:]
    elif isinstance(args, str):
        args = args.split()
    return run(parse_cli_args(args))


if __name__ == "__main__":
    main()
