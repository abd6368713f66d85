"""Diagnostic: run a bench workload on the JT_STAMPS build (make -C julia-raytracer_amd stamps) and
print the wave-time split between the item hand-out, the traversal phase and the shading phase,
the lanes per step kind, and the shading phases' material coherence (never used for timed
numbers). Takes bench.py's workload arguments (scripts/gpu.sh stamps:<w>)."""
import argparse
import ctypes as C
import os
import sys
import warnings
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["JTRACE_LIB"] = str(ROOT / "julia-raytracer_amd" / "build" / "libjtrace_hip_stamps.so")
sys.path.insert(0, str(ROOT / "julia-raytracer_amd"))
from jtrace import abi, sceneio, trace  # noqa: E402
from jtrace.cli import DEFAULT_TRAVERSAL, Params  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=256)
ap.add_argument("--sampler", default="path")
ap.add_argument("--scene", default=str(ROOT / "assets/scenes/cornellbox/cornellbox.json"))
ap.add_argument("--width", type=int, default=1280)
ap.add_argument("--height", type=int, default=720)
ap.add_argument("--traversal", default=DEFAULT_TRAVERSAL)
a, _ = ap.parse_known_args()
lib = abi.load_library()
lib.jt_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
with warnings.catch_warnings():
    warnings.simplefilter("ignore")
    scene = sceneio.load_scene(a.scene, missing="drop")
sa = abi.SceneABI(scene)
jp = abi.make_params(Params(scene="", samples=a.spp, width=a.width, height=a.height, batch=a.spp,
                            sampler=2 if a.sampler == "naive" else 1, traversal=a.traversal), 0)
st = trace.make_trace_state(sa, trace.make_scene_bvh(sa, False, lib), trace.make_trace_lights(sa, lib), jp, lib)
st.set_counters(0)
st.trace_range(0, a.spp)
v = (C.c_ulonglong * 24)()
abi.check(lib, lib.jt_debug_stamps(st.handle, v))
(t_trav, t_shade, n_trav, n_shade, lanes_p, lanes_n, steps_p, steps_n, _, t_hit, t_fin, t_qb, _, n_phit, n_fin,
 idle, n_mph, n_mty, n_mid, lanes_sh, lanes_hit, t_start, n_start, lanes_start) = list(v)
tot = t_trav + t_shade + t_start
cnt = st.counters()
print(f"{Path(a.scene).stem} {a.width}x{a.height} {a.spp} spp {a.sampler}: kernel_ms={cnt['kernel_ms']:.1f}  "
      f"{st.describe().split()[0]} traversal={st.traversal} streams={st.streams}")
print(f"wave time: item hand-out + sample starts {t_start / tot:.1%}, traversal phase {t_trav / tot:.1%}, "
      f"shading phase {t_shade / tot:.1%}")
print(f"loop iterations {n_start}: lanes starting a sample per iteration {lanes_start / max(1, n_start):.1f}")
print(f"traversal iterations per shading phase {n_trav / max(1, n_shade):.2f}; cycles per traversal iteration "
      f"{t_trav / max(1, n_trav):.0f}; cycles per shading phase {t_shade / max(1, n_shade):.0f}")
print(f"prim steps {steps_p} (avg lanes {lanes_p / max(1, steps_p):.1f}), node steps {steps_n} "
      f"(avg lanes {lanes_n / max(1, steps_n):.1f}); lanes without an item per traversal iteration "
      f"{idle / max(1, n_trav):.1f} of 64")
print(f"shading phases {n_shade}: lanes shading per phase {lanes_sh / max(1, n_shade):.1f}; split: hit + light chain "
      f"{t_hit / max(1, t_shade):.1%}, sample epilogue {t_fin / max(1, t_shade):.1%} (phases finishing a sample {n_fin}), "
      f"next query {t_qb / max(1, t_shade):.1%}")
print(f"shading phases with surface hits {n_mph} (lanes {lanes_hit / max(1, n_mph):.1f}): distinct material types "
      f"per phase {n_mty / max(1, n_mph):.2f}, distinct materials per phase {n_mid / max(1, n_mph):.2f}")
print(f"rays {cnt['rays']} light queries {cnt['light_queries']}")
