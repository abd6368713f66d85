"""Diagnostic: run the bench workload on the JT_STAMPS build and print the traversal/shading
split of wave time and step-lane utilisation (never used for timed numbers)."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["JTRACE_LIB"] = str(ROOT / "julia-raytracer_amd" / "build" / "libjtrace_hip_stamps.so")
sys.path.insert(0, str(ROOT / "julia-raytracer_amd"))
from jtrace import abi, sceneio, trace  # noqa: E402
from jtrace.cli import Params  # noqa: E402

import argparse  # noqa: E402
ap = argparse.ArgumentParser()
ap.add_argument("spp", nargs="?", type=int, default=64)
ap.add_argument("sampler", nargs="?", default="path")
ap.add_argument("--scene", default=str(ROOT / "assets/scenes/cornellbox/cornellbox.json"))
ap.add_argument("--width", type=int, default=1280)
ap.add_argument("--height", type=int, default=720)
a = ap.parse_args()
spp = a.spp
lib = abi.load_library()
lib.jt_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
import warnings  # noqa: E402
with warnings.catch_warnings():
    warnings.simplefilter("ignore")
    scene = sceneio.load_scene(a.scene, missing="drop")
sa = abi.SceneABI(scene)
sampler = 2 if a.sampler == "naive" else 1
jp = abi.make_params(Params(scene="", samples=spp, width=a.width, height=a.height, batch=spp, sampler=sampler,
                            traversal="near"), 0)
st = trace.make_trace_state(sa, trace.make_scene_bvh(sa, False, lib), trace.make_trace_lights(sa, lib), jp, lib)
st.set_counters(0)
st.trace_range(0, spp)
v = (C.c_ulonglong * 19)()
abi.check(lib, lib.jt_debug_stamps(st.handle, v))
(t_trav, t_shade, n_trav, n_shade, lanes_p, lanes_n, steps_p, steps_n, t_lhit, t_phit, t_fin, t_qb, n_lhit, n_phit, n_fin,
 dead, n_mph, n_mty, n_mid) = list(v)
tot = t_trav + t_shade
print(f"{Path(a.scene).stem} {a.width}x{a.height} {spp} spp {a.sampler}: wait_lanes={os.environ.get('JT_WAIT_LANES', 'default')} "
      f"kernel_ms={st.counters()['kernel_ms']:.1f}  {st.describe().split()[0]}")
print(f"traversal phase {t_trav / tot:.1%}  shading phase {t_shade / tot:.1%}")
print(f"trav iterations/wave-shade-phase {n_trav / max(1, n_shade):.2f}; cycles per trav iter {t_trav / max(1, n_trav):.0f}; "
      f"cycles per shading phase {t_shade / max(1, n_shade):.0f}")
print(f"prim steps {steps_p} (avg lanes {lanes_p / max(1, steps_p):.1f}), node steps {steps_n} "
      f"(avg lanes {lanes_n / max(1, steps_n):.1f})")
print(f"shading split: light_hit {t_lhit / t_shade:.1%} ({t_lhit / max(1, n_lhit):.0f} cyc x {n_lhit}), "
      f"path_hit {t_phit / t_shade:.1%} ({t_phit / max(1, n_phit):.0f} cyc x {n_phit}), "
      f"finish+restart {t_fin / t_shade:.1%} (phases with a finished sample {n_fin}), query_begin {t_qb / t_shade:.1%}")
print(f"lanes already done with their work unit, per traversal iteration: {dead / max(1, n_trav):.1f} of 64")
print(f"shading phases with surface hits {n_mph}: distinct material types per phase {n_mty / max(1, n_mph):.2f}, "
      f"distinct materials per phase {n_mid / max(1, n_mph):.2f}")
