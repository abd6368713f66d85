"""
    JtraceHip

Julia `ccall` shim over `libjtrace_hip.so` (include/jtrace.h): replaces the reference's
`trace_samples(state, scene, bvh, lights, params, bvh_stacks, bvh_sub_stacks, volume_stacks)`
(src/trace.jl:215-274) with the MI355X HIP path. No AMDGPU.jl, no CUDA: only `ccall`.

UNTESTED HERE: the build container and the GPU box have no Julia. The C side of every call is
exercised through the identical Python ctypes binding (julia-raytracer_amd/jtrace/abi.py) by
tests/. Integration into src/jtrace.jl is described in INTEGRATION.md.

Layout rules (include/jtrace.h "Conventions"): 0-based Int32 ids, Frame3f as 12 Float32
(x, y, z, o), host arrays owned by the caller and deep-copied by `jt_create`, so the packed
arrays only need to outlive that call (`GC.@preserve`).
"""
module JtraceHip

using ..Jtrace: SceneData, SceneBvh, TraceLights, TraceState, Params, BvhTree, MaterialType

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
end

const SAMPLER_IDS = Dict("path" => Int32(1), "naive" => Int32(2))  # src/cli.jl:88

check(st) = st == 0 ? nothing :
    error("jtrace: ", unsafe_string(ccall((:jt_last_error, LIB), Cstring, ())), " (status $st)")

frame12(f) = ntuple(k -> Float32(reinterpret(Float32, [f])[k]), 12)  # Frame3f = 4 x Vec3f
f3(v) = (Float32(v[1]), Float32(v[2]), Float32(v[3]))
ids0(v, n) = Int32[Int32(x[k] - 1) for x in v for k in 1:n]          # 1-based Int -> 0-based Int32
# an optional id (texture, light instance/environment): 1-based, or invalid_id (-1, src/scene.jl:45)
# for none; the C side's "none" is -1 too, so only real ids shift
id0(x) = x == -1 ? Int32(-1) : Int32(x - 1)
flat(v) = isempty(v) ? Float32[] : collect(reinterpret(Float32, v))

# ---- packing: Julia SceneData/SceneBvh/TraceLights -> C views (arrays kept in `keep`) -----
function pack_scene(scene::SceneData, keep::Vector{Any})
    cams = [JtCamera(frame12(c.frame), c.orthographic, c.lens, c.film, c.aspect, c.focus, c.aperture)
            for c in scene.cameras]
    insts = [JtInstance(frame12(i.frame), i.shape - 1, i.material - 1) for i in scene.instances]
    envs = [JtEnvironment(frame12(e.frame), f3(e.emission), id0(e.emission_tex)) for e in scene.environments]
    mats = [JtMaterial(Int32(Int(m.type)), f3(m.emission), f3(m.color), m.roughness, m.metallic, m.ior,
                       f3(m.scattering), m.scanisotropy, m.trdepth, m.opacity, id0(m.emission_tex),
                       id0(m.color_tex), id0(m.roughness_tex), id0(m.scattering_tex), id0(m.normal_tex))
            for m in scene.materials]
    texs = JtTexture[]
    for t in scene.textures
        pf = isempty(t.pixelsf) ? Float32[] : flat(t.pixelsf)
        pb = isempty(t.pixelsb) ? UInt8[] : collect(reinterpret(UInt8, t.pixelsb))
        push!(keep, pf, pb)
        push!(texs, JtTexture(t.width, t.height, t.linear, isempty(pf) ? C_NULL : pointer(pf),
                              isempty(pb) ? C_NULL : pointer(pb)))
    end
    shapes = JtShape[]
    for s in scene.shapes
        pts = Int32[p - 1 for p in s.points]; lns = ids0(s.lines, 2)
        tris = ids0(s.triangles, 3); qds = ids0(s.quads, 4)
        pos = flat(s.positions); nrm = flat(s.normals); tc = flat(s.texcoords)
        col = flat(s.colors); rad = collect(Float32, s.radius)
        push!(keep, pts, lns, tris, qds, pos, nrm, tc, col, rad)
        p(a) = isempty(a) ? C_NULL : pointer(a)
        push!(shapes, JtShape(length(s.points), length(s.lines), length(s.triangles), length(s.quads),
                              p(pts), p(lns), p(tris), p(qds), length(s.positions), p(pos),
                              length(s.normals), p(nrm), length(s.texcoords), p(tc),
                              length(s.colors), p(col), length(s.radius), p(rad)))
    end
    push!(keep, cams, insts, envs, mats, texs, shapes)
    JtScene(length(cams), pointer(cams), length(insts), pointer(insts), length(envs), pointer(envs),
            length(shapes), pointer(shapes), length(texs), pointer(texs), length(mats), pointer(mats))
end

function pack_tree(t::BvhTree, keep)
    nodes = [JtBvhNode(f3(n.bbox.min), f3(n.bbox.max), Int32(n.start - 1), n.num, Int8(n.axis - 1),
                       Int8(n.internal)) for n in t.nodes]
    prims = Int32[p - 1 for p in t.primitives]
    push!(keep, nodes, prims)
    JtBvhTree(length(nodes), pointer(nodes), length(prims), pointer(prims))
end

function pack_bvh(bvh::SceneBvh, keep)
    blas = [pack_tree(s.bvh, keep) for s in bvh.shapes]
    push!(keep, blas)
    JtSceneBvh(pack_tree(bvh.bvh, keep), length(blas), pointer(blas))
end

function pack_lights(lights::TraceLights, keep)
    ls = JtLight[]
    for l in lights.lights
        cdf = collect(Float32, l.elements_cdf)
        push!(keep, cdf)
        push!(ls, JtLight(id0(l.instance), id0(l.environment), length(cdf), pointer(cdf)))
    end
    push!(keep, ls)
    JtLights(length(ls), pointer(ls))
end

pack_params(p::Params; device = 0, seed = 0x5EED) =
    JtParams(p.camera - 1, p.resolution, 0, 0, p.samples, p.bounces, SAMPLER_IDS[p.sampler], p.clamp,
             p.envhidden, p.tentfilter, p.nocaustics, p.batch, p.bvhstacksize, device, seed)

# ---- device context ----------------------------------------------------------------------
mutable struct HipState
    ctx::Ptr{Cvoid}
    width::Int
    height::Int
end

"""make_hip_state(scene, bvh, lights, params; device = 0, devices = 1) — jt_create: uploads
everything, zeroed accumulators (make_trace_state, src/trace.jl:189-213). devices > 1:
jt_create_multi over GPUs 0 .. devices-1 — every trace_samples batch is sharded across them and
get_image! returns their RCCL-reduced, sample-weighted running mean."""
function make_hip_state(scene::SceneData, bvh::SceneBvh, lights::TraceLights, params::Params; device = 0,
                        devices = 1)
    keep = Any[]
    cs = Ref(pack_scene(scene, keep)); cb = Ref(pack_bvh(bvh, keep)); cl = Ref(pack_lights(lights, keep))
    cp = Ref(pack_params(params; device = device))
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

"""trace_samples(hip, state) — one batch (src/trace.jl:215-274) on the GPU; mirrors the
running-mean image and state.samples back into the reference's TraceState."""
function trace_samples(hip::HipState, state::TraceState)
    check(ccall((:jt_trace_samples, LIB), Cint, (Ptr{Cvoid},), hip.ctx))
    n = Ref{Int32}(0)
    check(ccall((:jt_get_samples, LIB), Cint, (Ptr{Cvoid}, Ref{Int32}), hip.ctx, n))
    state.samples = n[]
    nothing
end

"""get_image!(hip, state) — copies the device running mean into state.image (Vector{Vec4f})."""
function get_image!(hip::HipState, state::TraceState)
    GC.@preserve state begin
        check(ccall((:jt_get_image, LIB), Cint, (Ptr{Cvoid}, Ptr{Float32}), hip.ctx,
                    Ptr{Float32}(pointer(state.image))))
    end
    state
end

end # module
