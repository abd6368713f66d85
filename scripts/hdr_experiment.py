"""Which HDR decode matches the reference's own renders? Renders scenes with an HDR env at the
reference's size with many spp per candidate decode and compares against scene_pins.npz."""
import sys
import warnings
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "julia-raytracer_amd"))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import make_params  # noqa: E402
from jtrace import abi, sceneio, trace  # noqa: E402

warnings.simplefilter("ignore")
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 256
lib = abi.load_library()
pins = np.load(ROOT / "tests" / "golden" / "scene_pins.npz")
bh, bw = (int(v) for v in pins["block"])
for name in ("materials1", "shapes1", "features2", "materials2"):
    for mode in ("clamp", "srgb8", "srgb16", "raw"):
        sc = sceneio.load_scene(str(ROOT / "assets" / "scenes" / name / f"{name}.json"), missing="drop", hdr_mode=mode)
        sa = abi.SceneABI(sc)
        bvh = trace.make_scene_bvh(sa, False, lib)
        lights = trace.make_trace_lights(sa, lib)
        for sampler in (1, 2):
            key = f"{name}_{'path' if sampler == 1 else 'naive'}"
            p = make_params(abi, resolution=1280, samples=spp, sampler=sampler, batch=spp)
            st = trace.make_trace_state(sa, bvh, lights, p, lib)
            st.trace_range(0, spp)
            img = st.get_image()
            st.close()
            h, w = img.shape[:2]
            lin = sceneio.decode_srgb8(sceneio.to_srgb8(img, w, h))[..., :3]
            bm = lin.reshape(h // bh, bh, w // bw, bw, 3).mean(axis=(1, 3))
            ref = pins[key + "_mean"]
            rel = np.abs(bm - ref) / np.maximum(ref, 0.02)
            cm = lin.reshape(-1, 3).mean(axis=0)
            print(f"{key:18s} {mode:7s} cm {np.round(cm, 4)} ref {np.round(pins[key + '_channel_mean'], 4)} "
                  f"blk med {np.median(rel):.4f} p95 {np.percentile(rel, 95):.4f}", flush=True)
