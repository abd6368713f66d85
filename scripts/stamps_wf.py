"""Diagnostic: the WF body's job mix on the headline workload, from the JT_STAMPS build
(never used for timed numbers).  usage: JT_WF=1 python scripts/stamps_wf.py [spp]"""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["JTRACE_LIB"] = str(ROOT / "julia-raytracer_amd" / "build" / "libjtrace_hip_stamps.so")
sys.path.insert(0, str(ROOT / "julia-raytracer_amd"))
from jtrace import abi, sceneio, trace  # noqa: E402
from jtrace.cli import Params  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 32
lib = abi.load_library()
lib.jt_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
sa = abi.SceneABI(sceneio.load_scene(str(ROOT / "assets/scenes/cornellbox/cornellbox.json")))
jp = abi.make_params(Params(scene="", samples=spp, width=1280, height=720, batch=spp), 0)
st = trace.make_trace_state(sa, trace.make_scene_bvh(sa, False, lib), trace.make_trace_lights(sa, lib), jp, lib)
st.set_counters(0)
st.trace_range(0, spp)
v = list((C.c_ulonglong * 16)())
buf = (C.c_ulonglong * 16)()
abi.check(lib, lib.jt_debug_stamps(st.handle, buf))
v = list(buf)
names = ["traverse", "shade", "start", "idle", "", "", "", "", "", "", "", "", "", "", "select"]
tot = sum(v[k] for k in (0, 1, 2, 3, 14))
print(st.describe())
print(f"spp={spp} kernel_ms={st.counters()['kernel_ms']:.1f}")
print("wave time: " + ", ".join(f"{names[k]} {v[k] / tot:.1%}" for k in (0, 1, 2, 3, 14)))
print(f"jobs {v[13]}; traversal iterations {v[4]} (per job {v[4] / max(1, v[13]):.2f}); "
      f"stepping lanes {v[5] / max(1, v[4]):.1f}, busy lanes {v[6] / max(1, v[4]):.1f}; cycles/iter {v[0] / max(1, v[4]):.0f}")
print(f"shade jobs {v[7]} (light {v[11]}), batch {v[8] / max(1, v[7]):.1f}; cycles/shade job {v[1] / max(1, v[7]):.0f}")
print(f"refills {v[9]} taking {v[10] / max(1, v[9]):.1f}; traversal ring at job entry {v[12] / max(1, v[4]):.1f}")
