"""Run-to-run determinism of the HIP path: renders a workload twice in one process (with a reset
between) and compares with an image saved by an earlier process (gpurun_out/<dir>/det_*.npy).
usage: python scripts/determinism.py <out_dir> [--width W --height H --spp S --tile-share k,o]"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "julia-raytracer_amd"))
from jtrace import abi, sceneio, trace  # noqa: E402
from jtrace.cli import Params  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--scene", default=str(ROOT / "assets/scenes/cornellbox/cornellbox.json"))
ap.add_argument("--width", type=int, default=1280)
ap.add_argument("--height", type=int, default=720)
ap.add_argument("--spp", type=int, default=32)
ap.add_argument("--tile-share", default=None)
a = ap.parse_args()
lib = abi.load_library()
sa = abi.SceneABI(sceneio.load_scene(a.scene, missing="drop"))
p = abi.make_params(Params(scene=a.scene, samples=a.spp, width=a.width, height=a.height, batch=a.spp), 0)
bvh = trace.make_scene_bvh(sa, False, lib)
lights = trace.make_trace_lights(sa, lib)
if a.tile_share:
    abi.set_option(lib, "tile_share", a.tile_share)
st = trace.make_trace_state(sa, bvh, lights, p, lib)
imgs = []
for _ in range(3):
    st.reset()
    st.trace_range(0, a.spp)
    imgs.append(st.get_image())
st.set_counters(1)  # the COUNT=1 kernel (parity tests' counters) against the production COUNT=0 one
st.reset()
st.trace_range(0, a.spp)
c1 = st.get_image()
st.set_counters(0)
d = c1 != imgs[0]
print("COUNT=1 vs COUNT=0 kernel: differing values", int(d.sum()), "pixels", int(np.any(d, axis=-1).sum()),
      "max rel", float(np.max(np.abs(c1 - imgs[0]) / np.maximum(np.abs(imgs[0]), 1e-6))))
out = Path(a.out)
out.mkdir(parents=True, exist_ok=True)
tag = f"{Path(a.scene).stem}_{a.width}x{a.height}x{a.spp}_{a.tile_share or 'all'}".replace(",", "-")
prev = sorted(out.glob(f"det_{tag}_*.npy"))
for i in range(1, 3):
    d = imgs[i] != imgs[0]
    print(tag, f"run {i} vs 0 in-process: differing values {int(d.sum())}, pixels {int(np.any(d, axis=-1).sum())}")
for f in prev:
    o = np.load(f)
    d = imgs[0] != o
    print(tag, f"vs {f.name}: differing values {int(d.sum())}, pixels {int(np.any(d, axis=-1).sum())}, "
          f"max rel {float(np.max(np.abs(imgs[0] - o) / np.maximum(np.abs(o), 1e-6))):.3g}")
np.save(out / f"det_{tag}_{len(prev)}.npy", imgs[0])
st.close()
