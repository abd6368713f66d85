"""The Julia drop-in (julia-raytracer_amd/julia/JtraceHip.jl) cannot run here — there is no
Julia on either machine. Two kinds of checks stand in for running it:

1. Static: the shim against the reference's module / type table (tests/golden/
   reference_modules.json, generated from /root/reference/src by tests/golden/scripts/
   make_reference_modules.py). Every name it imports must be bound by the module it imports it
   from, every field it reads must be declared on the reference type it reads it from, every
   type it names must be imported or its own, its Jt* structs must mirror include/jtrace.h field
   for field, every ccall must name a declared function with its parameter count, and
   INTEGRATION.md must include it after the files defining what it imports. Round 2's shim
   failed two of these (imports from `..Jtrace`, which binds none of those types; a Dict lookup
   of the Int `Params.sampler`): `test_checker_rejects_the_round2_shim` keeps them caught.
2. Restated packing: its id packing is restated in Python and driven through the same C-ABI, on
   data in the reference's own convention: 1-based ids with invalid_id = -1 for "none"
   (src/scene.jl:45, :95-96, :125, :241-245; TraceLight instance/environment, src/trace.jl:131,168).
   A round-1 bug mapped every id with `x - 1`, turning invalid_id into -2, which jt_create
   rejects (every shipped scene has a material without a texture): these tests pin the fix.
"""
import copy
import ctypes as C
import json
import re

import numpy as np
import pytest

from conftest import ROOT, make_params

SHIM = ROOT / "julia-raytracer_amd" / "julia" / "JtraceHip.jl"
HEADER = ROOT / "include" / "jtrace.h"
MODULES = ROOT / "tests" / "golden" / "reference_modules.json"
INTEGRATION = ROOT / "INTEGRATION.md"

# Julia / C interop names a shim may use without importing them
JULIA_BUILTIN = {"Int", "Int8", "Int16", "Int32", "Int64", "UInt8", "UInt16", "UInt32", "UInt64", "Float32",
                 "Float64", "Bool", "Any", "Nothing", "String", "Ptr", "Ref", "NTuple", "Tuple", "Vector",
                 "Array", "Cint", "Cvoid", "Cstring", "Csize_t", "Clong", "WeakKeyDict", "Dict", "IdDict"}


def reference_table():
    return json.loads(MODULES.read_text())["modules"]


def bound_names(mods, mod):
    """Names module `mod` binds: its own definitions plus what its `using` lines import."""
    info = mods[mod]
    names = set(info["structs"]) | set(info["enums"]) | set(info["consts"]) | set(info["functions"])
    for vals in info["enums"].values():
        names |= set(vals)
    for u in info["using"]:
        names |= set(u["names"])
    return names


def shim_imports(text):
    """[(module path, [names])] of the shim's `using ..X: a, b` lines; `import ..X` -> names []."""
    out = []
    for m in re.finditer(r"^(using|import)\s+(\.+)(\w+)\s*(?::\s*(.*))?$", text, re.M):
        names = [n.strip() for n in (m.group(4) or "").split(",") if n.strip()]
        out.append((m.group(2), m.group(3), names))
    return out


def struct_index(mods):
    """struct name -> (module, {field: declared type})"""
    idx = {}
    for mod, info in mods.items():
        for name, s in info["structs"].items():
            idx[name] = (mod, {f: t for f, t in s["fields"]})
    return idx


def element_type(t):
    m = re.fullmatch(r"Vector\{(\w+)\}", t)
    return m.group(1) if m else None


def functions(text):
    """(name, signature, body) of every top-level `function` / one-line `f(...) = ...` method."""
    out = []
    for m in re.finditer(r"^function\s+(\w+)\((.*?)\)\s*\n(.*?)^end", text, re.M | re.S):
        out.append((m.group(1), m.group(2), m.group(3)))
    for m in re.finditer(r"^(\w+)\(([^\n]*?)\)\s*=\s*\n?(.*?)(?=^\S)", text, re.M | re.S):
        out.append((m.group(1), m.group(2), m.group(3)))
    return out


def check_field_accesses(text, structs):
    """Every `var.field[.field...]` read on a variable whose reference type is known (a signature
    annotation, or a `for x in y.f` binding over a Vector{T} field) must name declared fields."""
    errors = []
    for fname, sig, body in functions(text):
        types = {}
        for m in re.finditer(r"(\w+)\s*::\s*(\w+)", sig):
            if m.group(2) in structs:
                types[m.group(1)] = m.group(2)
        # loop / comprehension bindings, repeated until no new binding resolves
        for _ in range(3):
            for m in re.finditer(r"for\s+(\w+)\s+in\s+(\w+)\.(\w+)", body):
                var, src, field = m.groups()
                if src in types:
                    decl = structs[types[src]][1].get(field)
                    et = element_type(decl) if decl else None
                    if et in structs:
                        types[var] = et
        for m in re.finditer(r"(?<![\w.])(\w+)((?:\.\w+)+)", body):
            var, chain = m.group(1), m.group(2).split(".")[1:]
            if var not in types:
                continue
            t = types[var]
            for f in chain:
                if t not in structs:
                    break
                fields = structs[t][1]
                if f not in fields:
                    errors.append(f"{fname}: {var}::{t} has no field {f!r} (reference fields: {sorted(fields)})")
                    break
                t = fields[f].strip()
    return errors


def c_structs(header):
    """jt_* struct name -> [field names] from include/jtrace.h."""
    out = {}
    for m in re.finditer(r"typedef struct (jt_\w+) \{(.*?)\} \1;", header, re.S):
        body = re.sub(r"/\*.*?\*/", "", m.group(2), flags=re.S)
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            decl = re.sub(r"^(const\s+)?[\w]+\s*\**", "", decl)  # drop the type
            for name in decl.split(","):
                name = re.sub(r"\[.*?\]", "", name).strip().lstrip("*").strip()
                if name:
                    fields.append(name)
        out[m.group(1)] = fields
    return out


def c_prototypes(header):
    """jt_* function -> number of parameters."""
    out = {}
    for m in re.finditer(r"^\s*(?:const\s+)?[\w]+\**\s+\**(jt_\w+)\(([^)]*)\);", header, re.M | re.S):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else len(params.split(","))
    return out


def julia_structs(text):
    """Jt* struct name -> [field names] (the shim's C mirrors)."""
    out = {}
    for m in re.finditer(r"^struct (Jt\w+)\s*(?:#[^\n]*)?\n(.*?)^end", text, re.M | re.S):
        fields = []
        for line in m.group(2).split("\n"):
            for part in line.split(";"):
                f = re.match(r"\s*(\w+)::", part)
                if f:
                    fields.append(f.group(1))
        out[m.group(1)] = fields
    return out


def strip_comments(text):
    """The code of a Julia source: docstrings and `#` comments removed."""
    text = re.sub(r'"""(.*?)"""', "", text, flags=re.S)
    return re.sub(r"#[^\n]*", "", text)


def shim_problems(text, mods, integration=None):
    """All static defects of a shim source; [] when it would load and call correctly."""
    text = strip_comments(text)
    problems = []
    structs = struct_index(mods)
    includes = mods["Jtrace"]["includes"]
    mod_file = {m: info["file"] for m, info in mods.items()}
    imported = set()
    for dots, mod, names in shim_imports(text):
        if dots != "..":
            problems.append(f"`{dots}{mod}`: the shim is a submodule of Jtrace; its siblings are `..X`")
            continue
        if mod not in mods:
            problems.append(f"`..{mod}` is not a module of the reference")
            continue
        if mod != "Jtrace" and mod_file[mod] not in includes:
            problems.append(f"`..{mod}` is not included by Jtrace")
        have = bound_names(mods, mod)
        for n in names:
            if n not in have:
                problems.append(f"`using ..{mod}: {n}`: {mod} does not bind {n}")
            imported.add(n)
    defined = set(julia_structs(text)) | {"HipState"}
    for m in re.finditer(r"::\s*([\w{}, ]+)", text):
        for t in re.findall(r"[A-Z]\w*", m.group(1)):
            if t not in JULIA_BUILTIN and t not in imported and t not in defined:
                problems.append(f"type {t} is used but neither imported nor defined")
    problems += check_field_accesses(text, structs)
    # Params.sampler is already the 1-based SAMPLER_TYPES index (src/cli.jl:104,110-116)
    ptype = structs["Params"][1]["sampler"]
    if ptype != "Int":
        problems.append(f"reference Params.sampler is {ptype}")
    if re.search(r"\w+\[\s*p\.sampler\s*\]", text) or "Int32(p.sampler)" not in text:
        problems.append("Params.sampler must be passed as Int32(p.sampler) (it is an Int index, not a name)")
    # C mirrors: field order of every Jt* struct equals include/jtrace.h's jt_* struct
    header = HEADER.read_text()
    cs = c_structs(header)
    for jname, jfields in julia_structs(text).items():
        cname = "jt_" + re.sub(r"(?<!^)(?=[A-Z])", "_", jname[2:]).lower()
        if cname not in cs:
            problems.append(f"{jname}: no {cname} in include/jtrace.h")
        elif [f.lower() for f in jfields] != [f.lower() for f in cs[cname]]:
            problems.append(f"{jname} fields {jfields} != {cname} {cs[cname]}")
    protos = c_prototypes(header)
    for m in re.finditer(r"ccall\(\(:(\w+),\s*LIB\),\s*\w+,\s*\(([^()]*?(?:\{[^}]*\}[^()]*?)*)\)", text):
        name, argt = m.group(1), m.group(2).strip()
        if name not in protos:
            problems.append(f"ccall of {name}: not declared in include/jtrace.h")
            continue
        nargs = 0 if argt == "" else len([a for a in re.sub(r"\{[^}]*\}", "", argt).split(",") if a.strip()])
        if nargs != protos[name]:
            problems.append(f"ccall of {name}: {nargs} argument types, the C prototype has {protos[name]}")
    if integration is not None:
        m = re.search(r'include\("[^"]*JtraceHip\.jl"\)\s*#\s*after include\("(\w+\.jl)"\)', integration)
        if not m:
            problems.append("INTEGRATION.md does not say after which include() the shim goes")
        else:
            after = includes.index(m.group(1)) if m.group(1) in includes else -1
            for dots, mod, _ in shim_imports(text):
                if mod in mod_file and mod != "Jtrace" and mod_file[mod] in includes and \
                        includes.index(mod_file[mod]) > after:
                    problems.append(f"the shim is included before {mod_file[mod]}, which defines {mod}")
    return problems


TEX_FIELDS = ("emission_tex", "color_tex", "roughness_tex", "scattering_tex", "normal_tex")
FEATURES1 = str(ROOT / "assets" / "scenes" / "features1" / "features1.json")


def id0(x):
    """JtraceHip.jl `id0`: invalid_id stays -1, a 1-based id becomes 0-based."""
    return -1 if x == -1 else x - 1


def buggy_id0(x):
    """The round-1 mapping (`x - 1` for every id)."""
    return x - 1


def to_reference_convention(scene):
    """The host scene (0-based, -1 = none) as the reference's SceneData holds it: 1-based ids,
    invalid_id (-1) for none."""
    ref = copy.deepcopy(scene)
    for m in ref.materials:
        for f in TEX_FIELDS:
            v = getattr(m, f)
            setattr(m, f, -1 if v < 0 else v + 1)
    for e in ref.environments:
        e.emission_tex = -1 if e.emission_tex < 0 else e.emission_tex + 1
    return ref


def shim_pack(ref_scene, mapping):
    """pack_scene's optional-id handling (JtraceHip.jl pack_scene) applied to a reference-
    convention scene; shape/material/vertex ids go through the host loader's 0-based path."""
    out = copy.deepcopy(ref_scene)
    for m in out.materials:
        for f in TEX_FIELDS:
            setattr(m, f, mapping(getattr(m, f)))
    for e in out.environments:
        e.emission_tex = mapping(e.emission_tex)
    return out


def shim_lights(abi, lights, mapping):
    """pack_lights: TraceLight instance/environment (1-based or invalid_id) -> jt_light."""
    n = lights.struct.nlights
    arr = (abi.jt_light * max(1, n))()
    for k in range(n):
        l = lights.struct.lights[k]
        inst_ref = -1 if l.instance < 0 else l.instance + 1  # reference convention
        env_ref = -1 if l.environment < 0 else l.environment + 1
        arr[k].instance, arr[k].environment = mapping(inst_ref), mapping(env_ref)
        arr[k].ncdf, arr[k].cdf = l.ncdf, l.cdf
    return abi.jt_lights(n, arr), arr


def _create_status(abi, lib, scene, mapping, **kw):
    from jtrace import trace
    sa = abi.SceneABI(shim_pack(to_reference_convention(scene), mapping))
    bvh = trace.make_scene_bvh(sa, False, lib)
    lights = trace.make_trace_lights(sa, lib)
    jl, keep = shim_lights(abi, lights, mapping)
    p = make_params(abi, **kw)
    h = C.c_void_p()
    st = lib.jt_create(sa.ref, bvh.ref, C.byref(jl), C.byref(p), C.byref(h))
    msg = lib.jt_last_error().decode()
    if st == 0:
        lib.jt_destroy(h)
    del keep
    return st, msg


def test_reference_table_fixture_is_consistent():
    """The committed table holds the modules, types and include order the shim relies on."""
    mods = reference_table()
    assert mods["Jtrace"]["includes"][-1] == "trace.jl"
    assert [f for f, _ in mods["Scene"]["structs"]["SceneData"]["fields"]][:6] == \
        ["cameras", "instances", "environments", "shapes", "textures", "materials"]
    assert mods["Cli"]["structs"]["Params"]["fields"][13] == ["sampler", "Int"]
    assert "TraceState" in mods["Trace"]["structs"] and "SceneBvh" in mods["Bvh"]["structs"]
    # what round 2 assumed: Jtrace itself binds neither SceneData nor the BVH / trace types
    assert not {"SceneData", "SceneBvh", "BvhTree", "TraceState", "TraceLights"} & bound_names(mods, "Jtrace")


def test_shim_static_checks():
    """The shim as shipped: every import, type, field, C mirror, ccall and include position
    checks out against the reference's table and include/jtrace.h."""
    problems = shim_problems(SHIM.read_text(), reference_table(), INTEGRATION.read_text())
    assert problems == [], "\n".join(problems)


def test_checker_rejects_the_round2_shim():
    """The round-2 defects, put back into the current shim, are each caught."""
    text = SHIM.read_text()
    mods = reference_table()
    bad_imports = re.sub(r"^using \.\.(Scene|Bvh|Trace|Cli):.*\n", "", text, flags=re.M)
    bad_imports = bad_imports.replace(
        "import ..Trace\n",
        "import ..Trace\nusing ..Jtrace: SceneData, SceneBvh, TraceLights, TraceState, Params, BvhTree, MaterialType\n")
    p = shim_problems(bad_imports, mods)
    assert any("Jtrace does not bind SceneData" in x for x in p), p
    assert any("Jtrace does not bind BvhTree" in x for x in p), p
    bad_sampler = text.replace("Int32(p.sampler)", "SAMPLER_IDS[p.sampler]")
    assert any("Params.sampler" in x for x in shim_problems(bad_sampler, mods))
    bad_field = text.replace("s.bvh, keep)", "s.tree, keep)")
    assert any("has no field 'tree'" in x for x in shim_problems(bad_field, mods))
    bad_mirror = text.replace("nocaustics::Int32; batch::Int32", "batch::Int32; nocaustics::Int32")
    assert any("JtParams fields" in x for x in shim_problems(bad_mirror, mods))
    bad_ccall = text.replace("(:jt_trace_samples, LIB), Cint, (Ptr{Cvoid},)",
                             "(:jt_trace_samples, LIB), Cint, (Ptr{Cvoid}, Int32)")
    assert any("jt_trace_samples: 2 argument types" in x for x in shim_problems(bad_ccall, mods))
    bad_order = INTEGRATION.read_text().replace('# after include("trace.jl")', '# after include("scene.jl")')
    assert any("included before" in x for x in shim_problems(text, mods, bad_order))


def test_shim_source_maps_optional_ids_with_id0():
    """Static check of the shim (it cannot be executed here): no optional id is shifted with a
    bare `- 1`, and every one goes through id0."""
    text = SHIM.read_text()
    assert re.search(r"id0\(x\)\s*=\s*x\s*==\s*-1\s*\?\s*Int32\(-1\)\s*:\s*Int32\(x\s*-\s*1\)", text)
    for f in TEX_FIELDS:
        assert not re.search(rf"\.{f}\s*-\s*1", text), f
        assert f"id0(m.{f})" in text or f == "emission_tex", f
    assert "id0(e.emission_tex)" in text and "id0(m.emission_tex)" in text
    assert "id0(l.instance)" in text and "id0(l.environment)" in text


@pytest.mark.parametrize("scene_path", ["cornell", FEATURES1])
def test_shim_packing_passes_jt_create_validation(abi, lib, cornell, scene_path):
    """Reference-convention data packed the shim's way passes every jt_create check (on a CPU
    container jt_create then stops at hipSetDevice with JT_ERR_DEVICE; on a GPU it succeeds);
    the round-1 packing is rejected as JT_ERR_INVALID."""
    from jtrace import sceneio
    scene = cornell if scene_path == "cornell" else sceneio.load_scene(scene_path)
    st, msg = _create_status(abi, lib, scene, id0, resolution=32, samples=1)
    assert st in (0, -3), (st, msg)
    st_bad, msg_bad = _create_status(abi, lib, scene, buggy_id0, resolution=32, samples=1)
    assert st_bad == -1 and "texture id" in msg_bad, (st_bad, msg_bad)


@pytest.mark.gpu
def test_shim_packing_renders_like_the_host_loader(gpu, abi, lib, cornell):
    """Through the restated shim packing, cornellbox renders bit for bit as through the host
    loader's own 0-based packing."""
    from jtrace import trace
    p = make_params(abi, resolution=48, samples=2)
    sa = abi.SceneABI(shim_pack(to_reference_convention(cornell), id0))
    bvh = trace.make_scene_bvh(sa, False, lib)
    lights = trace.make_trace_lights(sa, lib)
    jl, keep = shim_lights(abi, lights, id0)
    h = C.c_void_p()
    abi.check(lib, lib.jt_create(sa.ref, bvh.ref, C.byref(jl), C.byref(p), C.byref(h)))
    abi.check(lib, lib.jt_trace_range(h, 0, 2))
    a = np.empty((48, 48, 4), np.float32)
    abi.check(lib, lib.jt_get_image(h, a.ctypes.data_as(abi.f32p)))
    lib.jt_destroy(h)
    del keep
    ca = abi.SceneABI(cornell)
    st = trace.make_trace_state(ca, trace.make_scene_bvh(ca, False, lib), trace.make_trace_lights(ca, lib), p, lib)
    st.trace_range(0, 2)
    assert np.array_equal(a, st.get_image())
    st.close()
