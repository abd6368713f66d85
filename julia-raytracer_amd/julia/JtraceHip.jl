"""
    JtraceHip

Julia `ccall` shim over `libjtrace_hip.so` (include/jtrace.h): replaces the reference's
`trace_samples(state, scene, bvh, lights, params, bvh_stacks, bvh_sub_stacks, volume_stacks)`
(src/trace.jl:215-274) with the MI355X HIP path. No AMDGPU.jl, no CUDA: only `ccall`.

Where it goes: a submodule of `Jtrace`, included after `trace.jl` (it imports the reference's
types from the submodules that define them: `Scene` src/scene.jl:337, `Bvh` src/bvh.jl:46,59,
`Trace` src/trace.jl:87,111, `Cli` src/cli.jl:90). Then one changed import line in
src/jtrace.jl makes `Jtrace.main` trace on the GPU (INTEGRATION.md):

    include("../julia-raytracer_amd/julia/JtraceHip.jl")      # after include("trace.jl")
    using .Trace: make_trace_lights, make_trace_state          # trace_samples, get_image: from
    using .JtraceHip: trace_samples, get_image                 # the shim, same signatures

UNTESTED HERE: the build container and the GPU box have no Julia. The C side of every call is
exercised through the identical Python ctypes binding (julia-raytracer_amd/jtrace/abi.py) by
tests/; tests/test_julia_shim.py checks this file statically against the reference's module /
type table (tests/golden/reference_modules.json) and restates its packing.

Layout rules (include/jtrace.h "Conventions"): 0-based Int32 ids, Frame3f as 12 Float32
(x, y, z, o), host arrays owned by the caller and deep-copied by `jt_create`, so the packed
arrays only need to outlive that call (`GC.@preserve`).
"""
module JtraceHip

using ..Scene: SceneData, MaterialPoint
using ..Bvh: SceneBvh, BvhTree
using ..Trace: TraceState, TraceLights
using ..Cli: Params
import ..Trace

const LIB = get(ENV, "JTRACE_LIB", joinpath(@__DIR__, "..", "build", "libjtrace_hip.so"))

# ---- C structs (field order and padding exactly as include/jtrace.h) ----------------------
struct JtCamera
    frame::NTuple{12,Float32}
    orthographic::Int32
    lens::Float32; film::Float32; aspect::Float32; focus::Float32; aperture::Float32
end
struct JtInstance
    frame::NTuple{12,Float32}
    shape::Int32; material::Int32
end
struct JtEnvironment
    frame::NTuple{12,Float32}
    emission::NTuple{3,Float32}
    emission_tex::Int32
end
struct JtMaterial
    type::Int32
    emission::NTuple{3,Float32}; color::NTuple{3,Float32}
    roughness::Float32; metallic::Float32; ior::Float32
    scattering::NTuple{3,Float32}
    scanisotropy::Float32; trdepth::Float32; opacity::Float32
    emission_tex::Int32; color_tex::Int32; roughness_tex::Int32; scattering_tex::Int32; normal_tex::Int32
end
struct JtTexture
    width::Int32; height::Int32; linear::Int32
    pixelsf::Ptr{Float32}; pixelsb::Ptr{UInt8}
end
struct JtShape
    npoints::Int32; nlines::Int32; ntriangles::Int32; nquads::Int32
    points::Ptr{Int32}; lines::Ptr{Int32}; triangles::Ptr{Int32}; quads::Ptr{Int32}
    npositions::Int32; positions::Ptr{Float32}
    nnormals::Int32; normals::Ptr{Float32}
    ntexcoords::Int32; texcoords::Ptr{Float32}
    ncolors::Int32; colors::Ptr{Float32}
    nradius::Int32; radius::Ptr{Float32}
end
struct JtScene
    ncameras::Int32; cameras::Ptr{JtCamera}
    ninstances::Int32; instances::Ptr{JtInstance}
    nenvironments::Int32; environments::Ptr{JtEnvironment}
    nshapes::Int32; shapes::Ptr{JtShape}
    ntextures::Int32; textures::Ptr{JtTexture}
    nmaterials::Int32; materials::Ptr{JtMaterial}
end
struct JtBvhNode  # 32 B, BvhNode (src/bvh.jl:34-44) 0-based
    bmin::NTuple{3,Float32}; bmax::NTuple{3,Float32}
    start::Int32; num::Int16; axis::Int8; internal::Int8
end
struct JtBvhTree
    nnodes::Int32; nodes::Ptr{JtBvhNode}
    nprimitives::Int32; primitives::Ptr{Int32}
end
struct JtSceneBvh
    tlas::JtBvhTree
    nshapes::Int32; blas::Ptr{JtBvhTree}
end
struct JtLight
    instance::Int32; environment::Int32; ncdf::Int32; cdf::Ptr{Float32}
end
struct JtLights
    nlights::Int32; lights::Ptr{JtLight}
end
struct JtParams
    camera::Int32; resolution::Int32; width::Int32; height::Int32; samples::Int32
    bounces::Int32; sampler::Int32; clamp::Int32; envhidden::Int32; tentfilter::Int32
    nocaustics::Int32; batch::Int32; bvhstacksize::Int32; device::Int32; seed::UInt64
    traversal::Int32  # jt_traversal: 0 = the reference's BVH child order
end

check(st) = st == 0 ? nothing :
    error("jtrace: ", unsafe_string(ccall((:jt_last_error, LIB), Cstring, ())), " (status $st)")

# Frame3f = SVector{4,Vec3f} (src/math.jl:46): columns x, y, z, o -> 12 floats
frame12(f) = ntuple(k -> Float32(f[(k - 1) ÷ 3 + 1][(k - 1) % 3 + 1]), 12)
f3(v) = (Float32(v[1]), Float32(v[2]), Float32(v[3]))
ids0(v, n) = Int32[Int32(x[k] - 1) for x in v for k in 1:n]          # 1-based Int -> 0-based Int32
# an optional id (texture, light instance/environment): 1-based, or invalid_id (-1, src/scene.jl:45)
# for none; the C side's "none" is -1 too, so only real ids shift
id0(x) = x == -1 ? Int32(-1) : Int32(x - 1)
flat(v) = isempty(v) ? Float32[] : collect(reinterpret(Float32, v))
ptr(a) = isempty(a) ? C_NULL : pointer(a)

# ---- packing: Julia SceneData/SceneBvh/TraceLights -> C views (arrays kept in `keep`) -----
function pack_scene(scene::SceneData, keep::Vector{Any})
    # CameraData src/scene.jl:48, InstanceData :88, EnvironmentData :117, MaterialData :213
    cams = [JtCamera(frame12(c.frame), Int32(c.orthographic), c.lens, c.film, c.aspect, c.focus, c.aperture)
            for c in scene.cameras]
    insts = [JtInstance(frame12(i.frame), Int32(i.shape - 1), Int32(i.material - 1)) for i in scene.instances]
    envs = [JtEnvironment(frame12(e.frame), f3(e.emission), id0(e.emission_tex)) for e in scene.environments]
    mats = [JtMaterial(Int32(Int(m.type)), f3(m.emission), f3(m.color), m.roughness, m.metallic, m.ior,
                       f3(m.scattering), m.scanisotropy, m.trdepth, m.opacity, id0(m.emission_tex),
                       id0(m.color_tex), id0(m.roughness_tex), id0(m.scattering_tex), id0(m.normal_tex))
            for m in scene.materials]
    texs = JtTexture[]
    for t in scene.textures  # TextureData src/scene.jl:146
        pf = flat(t.pixelsf)
        pb = isempty(t.pixelsb) ? UInt8[] : collect(reinterpret(UInt8, t.pixelsb))
        push!(keep, pf, pb)
        push!(texs, JtTexture(Int32(t.width), Int32(t.height), Int32(t.linear), ptr(pf), ptr(pb)))
    end
    shapes = JtShape[]
    for s in scene.shapes  # ShapeData src/shape.jl:13
        pts = Int32[p - 1 for p in s.points]; lns = ids0(s.lines, 2)
        tris = ids0(s.triangles, 3); qds = ids0(s.quads, 4)
        pos = flat(s.positions); nrm = flat(s.normals); tc = flat(s.texcoords)
        col = flat(s.colors); rad = collect(Float32, s.radius)
        push!(keep, pts, lns, tris, qds, pos, nrm, tc, col, rad)
        push!(shapes, JtShape(length(s.points), length(s.lines), length(s.triangles), length(s.quads),
                              ptr(pts), ptr(lns), ptr(tris), ptr(qds), length(s.positions), ptr(pos),
                              length(s.normals), ptr(nrm), length(s.texcoords), ptr(tc),
                              length(s.colors), ptr(col), length(s.radius), ptr(rad)))
    end
    push!(keep, cams, insts, envs, mats, texs, shapes)
    JtScene(length(cams), ptr(cams), length(insts), ptr(insts), length(envs), ptr(envs),
            length(shapes), ptr(shapes), length(texs), ptr(texs), length(mats), ptr(mats))
end

function pack_tree(t::BvhTree, keep::Vector{Any})
    # BvhNode src/bvh.jl:34 (bbox::Bbox3f src/geometry.jl:22, 1-based start and axis)
    nodes = [JtBvhNode(f3(n.bbox.min), f3(n.bbox.max), Int32(n.start - 1), n.num, Int8(n.axis - 1),
                       Int8(n.internal)) for n in t.nodes]
    prims = Int32[p - 1 for p in t.primitives]
    push!(keep, nodes, prims)
    JtBvhTree(length(nodes), ptr(nodes), length(prims), ptr(prims))
end

function pack_bvh(bvh::SceneBvh, keep::Vector{Any})
    # SceneBvh src/bvh.jl:59: the instance TLAS `bvh` and one ShapeBvh (`bvh` field) per shape
    blas = [pack_tree(s.bvh, keep) for s in bvh.shapes]
    push!(keep, blas)
    JtSceneBvh(pack_tree(bvh.bvh, keep), length(blas), ptr(blas))
end

function pack_lights(lights::TraceLights, keep::Vector{Any})
    ls = JtLight[]
    for l in lights.lights  # TraceLight src/trace.jl:102
        cdf = collect(Float32, l.elements_cdf)
        push!(keep, cdf)
        push!(ls, JtLight(id0(l.instance), id0(l.environment), length(cdf), ptr(cdf)))
    end
    push!(keep, ls)
    JtLights(length(ls), ptr(ls))
end

# Params src/cli.jl:90-138: camera is find_camera's 1-based index (src/jtrace.jl:61), sampler is
# already the 1-based index into SAMPLER_TYPES = ["path", "naive"] (src/cli.jl:88,111-116) —
# the C side's jt_sampler uses the same numbering — and clamp is an Int (src/cli.jl:105)
# traversal (jt_traversal): 3 = auto, the product default (the 4-wide quantised records for a deep
# scene that runs from HBM, the binary tree near child first otherwise), 1 = near, 2 = wide, 0 = the
# reference's far-first order (src/bvh.jl:331-341); they differ only where two hits tie at exactly
# equal t or a box is culled by the slab test's rounding (a few pixels per million per sample;
# the share grows with spp: bench.py's reference-order line reports it at the configs' own spp).
# JTRACE_TRAVERSAL=0 makes the drop-in trace_samples run the reference's exact order.
pack_params(p::Params; device = 0, seed = 0x5EED, traversal = 3) =
    JtParams(Int32(p.camera - 1), Int32(p.resolution), Int32(0), Int32(0), Int32(p.samples), Int32(p.bounces),
             Int32(p.sampler), Int32(p.clamp), Int32(p.envhidden), Int32(p.tentfilter), Int32(p.nocaustics),
             Int32(p.batch), Int32(p.bvhstacksize), Int32(device), UInt64(seed), Int32(traversal))

# ---- device context ----------------------------------------------------------------------
mutable struct HipState
    ctx::Ptr{Cvoid}
    width::Int
    height::Int
end

"""make_hip_state(scene, bvh, lights, params; device = 0, devices = 1) — jt_create: uploads
everything, zeroed accumulators (make_trace_state, src/trace.jl:189-213). devices > 1:
jt_create_multi over GPUs 0 .. devices-1 — every trace_samples batch is sharded across them (by
samples, or by pixel tiles when a batch has fewer samples than devices) and get_image! returns
their RCCL-reduced running mean."""
function make_hip_state(scene::SceneData, bvh::SceneBvh, lights::TraceLights, params::Params; device = 0,
                        devices = 1, traversal = 3)
    keep = Any[]
    cs = Ref(pack_scene(scene, keep)); cb = Ref(pack_bvh(bvh, keep)); cl = Ref(pack_lights(lights, keep))
    cp = Ref(pack_params(params; device = device, traversal = traversal))
    ctx = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve keep cs cb cl cp begin
        if devices > 1
            check(ccall((:jt_create_multi, LIB), Cint, (Ref{JtScene}, Ref{JtSceneBvh}, Ref{JtLights}, Ref{JtParams},
                                                        Ptr{Int32}, Int32, Ref{Ptr{Cvoid}}),
                        cs, cb, cl, cp, C_NULL, Int32(devices), ctx))
        else
            check(ccall((:jt_create, LIB), Cint, (Ref{JtScene}, Ref{JtSceneBvh}, Ref{JtLights}, Ref{JtParams},
                                                  Ref{Ptr{Cvoid}}), cs, cb, cl, cp, ctx))
        end
    end
    w = Ref{Int32}(0); h = Ref{Int32}(0)
    check(ccall((:jt_get_size, LIB), Cint, (Ptr{Cvoid}, Ref{Int32}, Ref{Int32}), ctx[], w, h))
    st = HipState(ctx[], w[], h[])
    finalizer(s -> s.ctx == C_NULL || ccall((:jt_destroy, LIB), Cvoid, (Ptr{Cvoid},), s.ctx), st)
    st
end

"""trace_samples(hip, state) — one batch (src/trace.jl:215-274) on the GPU; advances
state.samples as the reference does (the running means stay on the device until get_image!)."""
function trace_samples(hip::HipState, state::TraceState)
    check(ccall((:jt_trace_samples, LIB), Cint, (Ptr{Cvoid},), hip.ctx))
    n = Ref{Int32}(0)
    check(ccall((:jt_get_samples, LIB), Cint, (Ptr{Cvoid}, Ref{Int32}), hip.ctx, n))
    state.samples = n[]
    nothing
end

"""get_image!(hip, state) — copies the device running means into state.image (Vector{Vec4f}),
state.albedo / state.normal (Vector{Vec3f}) and state.hits (Vector{Int}) (src/trace.jl:87-100)."""
function get_image!(hip::HipState, state::TraceState)
    GC.@preserve state begin
        check(ccall((:jt_get_image, LIB), Cint, (Ptr{Cvoid}, Ptr{Float32}), hip.ctx,
                    Ptr{Float32}(pointer(state.image))))
        check(ccall((:jt_get_aovs, LIB), Cint, (Ptr{Cvoid}, Ptr{Float32}, Ptr{Float32}, Ptr{Int64}), hip.ctx,
                    Ptr{Float32}(pointer(state.albedo)), Ptr{Float32}(pointer(state.normal)),
                    Ptr{Int64}(pointer(state.hits))))
    end
    state
end

# ---- the reference's own signatures (drop-in for Jtrace.main, src/jtrace.jl:83-110) ----------
# One device context per TraceState, created by its first trace_samples call. JTRACE_DEVICES
# (default 1) GPUs of the node; the caller's scratch stacks are not needed (the traversal stack
# lives in LDS, the volume stack in registers).
const CONTEXTS = WeakKeyDict{TraceState,HipState}()

"""trace_samples(state, scene, bvh, lights, params, bvh_stacks, bvh_sub_stacks, volume_stacks) —
the reference's signature and semantics (src/trace.jl:215-274): one batch
[state.samples, min(state.samples + params.batch, params.samples)), state.samples advanced."""
function trace_samples(state::TraceState, scene::SceneData, bvh::SceneBvh, lights::TraceLights, params::Params,
                       bvh_stacks::Vector{Vector{Int32}}, bvh_sub_stacks::Vector{Vector{Int32}},
                       volume_stacks::Vector{Vector{MaterialPoint}})
    if state.samples >= params.samples
        return
    end
    hip = get!(CONTEXTS, state) do
        make_hip_state(scene, bvh, lights, params; devices = parse(Int, get(ENV, "JTRACE_DEVICES", "1")),
                       traversal = parse(Int, get(ENV, "JTRACE_TRAVERSAL", "3")))
    end
    trace_samples(hip, state)
end

"""get_image(state) — the reference's get_image (src/trace.jl:676-680) after the device running
means of `state` (if it was traced on the GPU) have been copied into it."""
function get_image(state::TraceState)
    hip = get(CONTEXTS, state, nothing)
    hip === nothing || get_image!(hip, state)
    Trace.get_image(state)
end

end # module
