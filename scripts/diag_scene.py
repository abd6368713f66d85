"""Localise a GPU-vs-oracle divergence on a scene by switching features off one at a time.
usage: python scripts/diag_scene.py features1"""
import copy
import sys
import warnings
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "julia-raytracer_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import compare_images, make_params  # noqa: E402
from jtrace import abi, sceneio, trace  # noqa: E402
from oracle import Oracle  # noqa: E402

warnings.simplefilter("ignore")
name = sys.argv[1] if len(sys.argv) > 1 else "features1"
lib = abi.load_library()
orc = Oracle(abi)
base = sceneio.load_scene(str(ROOT / "assets" / "scenes" / name / f"{name}.json"), missing="drop")


def variant(fn):
    sc = copy.deepcopy(base)
    fn(sc)
    return sc


def no_normal_tex(sc):
    for m in sc.materials:
        m.normal_tex = -1


def no_scattering(sc):
    for m in sc.materials:
        m.scattering = np.zeros(3, np.float32)


def all_matte(sc):
    for m in sc.materials:
        m.type = "matte"


def no_textures(sc):
    for m in sc.materials:
        m.color_tex = m.roughness_tex = m.emission_tex = m.scattering_tex = m.normal_tex = -1


def keep_instances(idx):
    def f(sc):
        sc.instances = [sc.instances[i] for i in idx]
    return f


def no_env(sc):
    sc.environments = []


variants = {"base": lambda sc: None, "no_normal_tex": no_normal_tex, "no_scattering": no_scattering,
            "all_matte": all_matte, "no_textures": no_textures, "no_env": no_env}
for k in range(len(base.instances)):
    variants[f"only_inst{k}+lights"] = keep_instances(sorted({0, 1, k}))
for vname, fn in variants.items():
    sc = variant(fn)
    sa = abi.SceneABI(sc)
    for sampler in (1, 2):
        for bounces in (1, 8):
            p = make_params(abi, resolution=96, samples=2, sampler=sampler, bounces=bounces)
            try:
                bvh = trace.make_scene_bvh(sa, False, lib)
                lights = trace.make_trace_lights(sa, lib)
                st = trace.make_trace_state(sa, bvh, lights, p, lib)
                st.trace_range(0, 2)
                g = (st.get_image(), *st.get_aovs(), st.counters())
                st.close()
            except Exception as e:  # noqa: BLE001
                print(vname, sampler, bounces, "ERR", e, flush=True)
                continue
            ob = orc.build_bvh(sa)
            ol = orc.make_lights(sa)
            o = orc.trace(sa, ob, ol, p, g[0].shape[1], g[0].shape[0], 0, 2)
            s = compare_images(g[0], o[0])
            sn = compare_images(g[2], o[2])
            sa_ = compare_images(g[1], o[1])
            print(f"{vname:22s} s{sampler} b{bounces} img {s['frac_pix_rel_le_1e-3']:.4f} "
                  f"normal {sn['frac_pix_rel_le_1e-3']:.4f} albedo {sa_['frac_pix_rel_le_1e-3']:.4f} "
                  f"hits_eq {np.array_equal(g[3], o[3])} rays {g[4]['rays']} {o[4]['rays']} "
                  f"lq {g[4]['light_queries']} {o[4]['light_queries']}", flush=True)
            if vname == "base" and sampler == 1 and bounces == 1:
                bad = np.argwhere(np.abs(g[0] - o[0]).max(axis=2) > 1e-3)
                for y, x in bad[:5]:
                    print("   pixel", (x, y), "gpu", g[0][y, x], "oracle", o[0][y, x],
                          "n", g[2][y, x], o[2][y, x], "alb", g[1][y, x], o[1][y, x])
