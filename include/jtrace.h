/*
 * jtrace.h — C-ABI drop-in boundary for the MI355X path-tracing hot path.
 *
 * The reference (Princic-1837592/julia-raytracer, pure Julia 1.8.3) has no FFI.
 * Its natural seam is the per-batch call made by Jtrace.main:
 *
 *     trace_samples(state, scene, bvh, lights, params,
 *                   bvh_stacks, bvh_sub_stacks, volume_stacks)   src/trace.jl:215-274
 *
 * This header exports exactly what a Julia `ccall` shim (julia-raytracer_amd/julia/
 * JtraceHip.jl) or the Python `ctypes` harness binds to replace that call:
 *
 *   jt_create          ~ make_trace_state (src/trace.jl:189) + device upload of SceneData,
 *                        SceneBvh and TraceLights (src/scene.jl:337, src/bvh.jl:59, src/trace.jl:111)
 *   jt_trace_samples   == trace_samples for one batch (src/trace.jl:215)
 *   jt_trace_range     == trace_samples over an explicit global sample range (multi-GPU shards)
 *   jt_get_image       == get_image (src/trace.jl:676) — the running-mean RGBA buffer
 *   jt_get_aovs        == TraceState.albedo / normal / hits (src/trace.jl:87-100)
 *   jt_destroy / jt_last_error — lifetime and error reporting (the reference throws Julia exceptions)
 *
 * Host helpers (run on the CPU, no device needed) that restate the reference's host code
 * for callers without their own:
 *   jt_build_scene_bvh ~ make_scene_bvh (src/bvh.jl:66), split_middle / split_sah exact
 *   jt_make_lights     ~ make_trace_lights (src/trace.jl:117)
 *
 * Conventions
 *   - every function returns JT_OK (0) or a negative jt_status; nothing throws across the ABI;
 *     jt_last_error() returns a thread-local message for the last failure on this thread.
 *   - all indices are 0-based int32 (the reference uses 1-based Int64; the shim subtracts 1).
 *     "none" ids (Julia invalid_id = -1, src/scene.jl:45) are -1 here too.
 *   - frames are 12 floats, column-major x, y, z, o (Frame3f, src/math.jl:46-60).
 *   - the caller owns every host array; jt_create deep-copies to the device, so host
 *     arrays may be released after it returns (Julia: GC.@preserve around the ccall).
 *   - a context is used by one host thread at a time; every call is synchronous.
 */
#ifndef JTRACE_H
#define JTRACE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JT_ABI_VERSION 5  /* 2: jt_params.traversal; 3: jt_set_option; 4: sample streams, jt_get_streams;
                            5: deferred jt_trace_range (same signatures) */

typedef enum jt_status {
    JT_OK = 0,
    JT_ERR_INVALID = -1,      /* malformed input (bad id, size, NULL pointer) */
    JT_ERR_UNSUPPORTED = -2,  /* input the reference cannot render either (see jt_create) */
    JT_ERR_DEVICE = -3,       /* HIP runtime failure / no device */
    JT_ERR_NOMEM = -4,        /* host or device allocation failed */
    JT_ERR_STACK = -5,        /* BVH deeper than params.bvhstacksize (reference: BoundsError) */
    JT_ERR_STATE = -6         /* call out of order (e.g. range outside [0, samples)) */
} jt_status;

/* MaterialType, in the order of the reference enum (src/scene.jl:191-200). */
typedef enum jt_material_type {
    JT_MATTE = 0,
    JT_GLOSSY = 1,
    JT_REFLECTIVE = 2,
    JT_TRANSPARENT = 3,
    JT_REFRACTIVE = 4,
    JT_SUBSURFACE = 5,
    JT_VOLUMETRIC = 6,
    JT_GLTFPBR = 7
} jt_material_type;

/* Samplers, index into SAMPLER_TYPES = ["path", "naive"] (src/cli.jl:88). */
typedef enum jt_sampler { JT_SAMPLER_PATH = 1, JT_SAMPLER_NAIVE = 2 } jt_sampler;

/* BVH child visit order (extension, jt_params.traversal).
 * JT_TRAVERSAL_REFERENCE: the reference's (src/bvh.jl:331-341, 396-407): for d[axis] >= 0 push
 *   start then start+1, so the upper child (start+1, higher split-axis coordinates: split_middle /
 *   split_sah partition lower centers to `start`, src/bvh.jl:171-176, 281-304) is visited first —
 *   the far child for a closest-hit query.
 * JT_TRAVERSAL_NEAR: the opposite push order, the near child by the split axis first. Fewer nodes
 *   are visited (tmax shrinks sooner). Among hits at exactly equal t the reference's later-tested
 *   one wins (src/geometry.jl:226, t > tmax rejects), which depends on the order: a near-first
 *   query that accepts a hit at exactly its current tmax is run again in the reference's child
 *   order and reports that hit (an intersect_instance_bvh of a one-leaf shape BVH has no child
 *   order and is never re-run). The closest hit then differs from the reference's only where the
 *   slab test's rounding lets one order find a hit the other culls (measured: 2e-6 of bathroom1's
 *   paths, none on cornellbox, features2, ecosys).
 * JT_TRAVERSAL_WIDE: the reference's binary tree collapsed to 4-wide records (each internal node
 *   holds its grandchildren: same leaves, same primitive order) with conservative 8-bit quantised
 *   child boxes, visited near child first in the binary DFS order (a tie's re-run: far child
 *   first, the reference's leaf sequence). A box can only pass where the exact one would, or more
 *   often, so again only boxes the exact slab test culls by rounding can resolve differently; one
 *   64-B record replaces about three 32-B node visits. */
typedef enum jt_traversal {
    JT_TRAVERSAL_REFERENCE = 0,
    JT_TRAVERSAL_NEAR = 1,
    JT_TRAVERSAL_WIDE = 2,
    JT_TRAVERSAL_AUTO = 3  /* wide for a scene that runs from HBM with a deep BVH (stack bound
                              above 32), near otherwise (LDS-mode and shallow scenes); jt_describe
                              reports the order taken ("traversal=near|wide") */
} jt_traversal;

/* CameraData (src/scene.jl:48-86), after the lookat conversion done by the loader. */
typedef struct jt_camera {
    float frame[12];
    int32_t orthographic;
    float lens, film, aspect, focus, aperture;
} jt_camera;

/* InstanceData (src/scene.jl:88-115). */
typedef struct jt_instance {
    float frame[12];
    int32_t shape;     /* 0-based shape id */
    int32_t material;  /* 0-based material id */
} jt_instance;

/* EnvironmentData (src/scene.jl:117-144). */
typedef struct jt_environment {
    float frame[12];
    float emission[3];
    int32_t emission_tex; /* -1 = none */
} jt_environment;

/* MaterialData (src/scene.jl:213-264). Texture ids are 0-based, -1 = none. */
typedef struct jt_material {
    int32_t type; /* jt_material_type */
    float emission[3];
    float color[3];
    float roughness, metallic, ior;
    float scattering[3];
    float scanisotropy, trdepth, opacity;
    int32_t emission_tex, color_tex, roughness_tex, scattering_tex, normal_tex;
} jt_material;

/* TextureData (src/scene.jl:146-162): RGBA, row-major, top row first.
 * Exactly one of pixelsf (linear float, HDR) / pixelsb (8-bit) is non-NULL. */
typedef struct jt_texture {
    int32_t width, height;
    int32_t linear;
    const float* pixelsf;   /* width*height*4 floats or NULL */
    const uint8_t* pixelsb; /* width*height*4 bytes or NULL */
} jt_texture;

/* ShapeData (src/shape.jl:13-48). Element arrays hold 0-based vertex ids.
 * Per-vertex arrays may be NULL with count 0 (the reference's empty vectors). */
typedef struct jt_shape {
    int32_t npoints, nlines, ntriangles, nquads;
    const int32_t* points;    /* npoints */
    const int32_t* lines;     /* nlines*2 */
    const int32_t* triangles; /* ntriangles*3 */
    const int32_t* quads;     /* nquads*4 */
    int32_t npositions;
    const float* positions;   /* npositions*3 */
    int32_t nnormals;
    const float* normals;     /* nnormals*3 */
    int32_t ntexcoords;
    const float* texcoords;   /* ntexcoords*2 (v already flipped by the loader, src/shape.jl:88) */
    int32_t ncolors;
    const float* colors;      /* ncolors*4 */
    int32_t nradius;
    const float* radius;      /* nradius */
} jt_shape;

/* SceneData (src/scene.jl:337-356). */
typedef struct jt_scene {
    int32_t ncameras;
    const jt_camera* cameras;
    int32_t ninstances;
    const jt_instance* instances;
    int32_t nenvironments;
    const jt_environment* environments;
    int32_t nshapes;
    const jt_shape* shapes;
    int32_t ntextures;
    const jt_texture* textures;
    int32_t nmaterials;
    const jt_material* materials;
} jt_scene;

/* BvhNode (src/bvh.jl:34-44), 0-based: `start` is the first child node (internal) or the
 * first slot of `primitives` (leaf); axis is 0..2. 32 bytes, C-compatible. */
typedef struct jt_bvh_node {
    float bmin[3];
    float bmax[3];
    int32_t start;
    int16_t num;
    int8_t axis;
    int8_t internal;
} jt_bvh_node;

/* BvhTree (src/bvh.jl:46-51). primitives[] are 0-based element (BLAS) or instance (TLAS) ids. */
typedef struct jt_bvh_tree {
    int32_t nnodes;
    jt_bvh_node* nodes;
    int32_t nprimitives;
    int32_t* primitives;
} jt_bvh_tree;

/* SceneBvh (src/bvh.jl:59-64): the instance TLAS plus one BLAS per shape. */
typedef struct jt_scene_bvh {
    jt_bvh_tree tlas;
    int32_t nshapes;
    jt_bvh_tree* blas;
} jt_scene_bvh;

/* TraceLight (src/trace.jl:102-109): exactly one of instance / environment is >= 0. */
typedef struct jt_light {
    int32_t instance;
    int32_t environment;
    int32_t ncdf;
    float* cdf;
} jt_light;

/* TraceLights (src/trace.jl:111-115). */
typedef struct jt_lights {
    int32_t nlights;
    jt_light* lights;
} jt_lights;

/* Params (src/cli.jl:90-138) restricted to the fields the hot path reads, plus the
 * build's extensions (seed, width/height override, device). */
typedef struct jt_params {
    int32_t camera;      /* 0-based camera id (find_camera result - 1) */
    int32_t resolution;  /* --resolution; W,H derived from camera aspect as make_trace_state */
    int32_t width;       /* extension: > 0 overrides W (with height) — aspect := W/H */
    int32_t height;
    int32_t samples;     /* --samples */
    int32_t bounces;     /* --bounces */
    int32_t sampler;     /* jt_sampler */
    int32_t clamp;       /* --clamp, stored as Int by the reference (src/cli.jl:105) */
    int32_t envhidden;
    int32_t tentfilter;
    int32_t nocaustics;
    int32_t batch;       /* --batch */
    int32_t bvhstacksize;
    int32_t device;      /* HIP device ordinal for this context */
    uint64_t seed;       /* extension: RNG seed; stream keyed by (seed, pixel, global sample) */
    int32_t traversal;   /* extension: jt_traversal (0 = the reference's child order) */
} jt_params;

/* Device counters accumulated over every launch of a context (diagnostic, exact). */
typedef struct jt_counters {
    uint64_t paths;          /* (pixel, sample) pairs traced */
    uint64_t rays;           /* intersect_scene_bvh calls (closest-hit scene queries) */
    uint64_t light_queries;  /* intersect_instance_bvh calls from sample_lights_pdf */
    uint64_t nodes;          /* BVH node pops (TLAS + BLAS, both query kinds) */
    uint64_t instances;      /* instance visits (TLAS leaf entries + light queries) */
    uint64_t prims;          /* triangle / quad tests */
    uint64_t shades;         /* surface hits shaded */
    uint64_t launches;       /* kernel launches */
    double kernel_ms;        /* summed device time of the trace launches (HIP events) */
} jt_counters;

/* Device pointers of a context's accumulators (for an in-place RCCL reduce). */
typedef struct jt_device_buffers {
    void* image;   /* float4[W*H]  running mean RGBA */
    void* albedo;  /* float4[W*H]  running mean albedo (w unused) */
    void* normal;  /* float4[W*H]  running mean normal (w unused) */
    void* hits;    /* int64[W*H] */
    int32_t width, height;
    void* stream;  /* hipStream_t the context launches on */
} jt_device_buffers;

typedef struct jt_ctx jt_ctx;

/* ---- library ---------------------------------------------------------------------- */
const char* jt_version(void);
int jt_abi_version(void);
const char* jt_last_error(void);
int jt_device_count(int32_t* out);

/* ---- run-time options ---------------------------------------------------------------- */
/* Process-wide switches, read by jt_create / jt_create_multi for the contexts they create
 * afterwards (a context keeps the values it was created with). The library never reads the
 * environment. name, value: NUL-terminated; value NULL removes one option, name NULL (with
 * value NULL) removes all. An unknown name fails with JT_ERR_INVALID. Unless stated, every
 * option leaves images, AOVs and counters bit-identical to the default:
 *   "env_alias" "1"          environment lights sample texels through alias tables (O(1)) instead
 *                            of upper_bound: the same distribution, so results equal the default
 *                            statistically, NOT bitwise (a variant, off by default)
 *   "features" "all"         run the general kernel instead of the scene's specialisation
 *   "lds_scene" "<bytes>"    budget of the small-scene LDS blob (0: scene arrays stay in HBM;
 *                            the stream count, hence the bits, never depend on the mode)
 *   "lds_stack" "32"         a 32-entry LDS stack ring instead of 16
 *   "light_inline" "0"       sample_lights_pdf's light queries through the traversal loop
 *   "wait_lanes", "light_lanes"  the shading gate; the light-hit step gate
 *   "multi_split" "tiles"|"samples"  jt_create_multi's split mode
 * Options that change WHAT a context traces (jt_describe reports them when set):
 *   "streams" "<k>"          sample streams per pixel (a power of two <= 64) instead of the
 *                            automatic count (jt_get_streams): the running means combine in a
 *                            different order, so images differ in the last bits
 *   "tile_share" "k,o"       trace only the 8x8 tiles o, o + k, o + 2k, ...: this process's share
 *                            of a k-way tile split when one process per GPU shards a render by
 *                            tiles (bench.py); jt_create_multi sets its own split instead
 *   "test_lds_ring" "1|2|4|8|16"  (tests only) use that many LDS ring entries, the rest overflow to
 *                            HBM: the overflow path on small scenes */
int jt_set_option(const char* name, const char* value);

/* ---- host helpers (CPU only) ------------------------------------------------------- */
/* make_scene_bvh (src/bvh.jl:66-88): one BLAS per shape (make_shape_bvh :90) and the
 * instance TLAS over transformed root boxes; split_middle (:185) or split_sah (:218). */
int jt_build_scene_bvh(const jt_scene* scene, int32_t high_quality, jt_scene_bvh* out);
void jt_free_scene_bvh(jt_scene_bvh* bvh);
/* make_trace_lights (src/trace.jl:117-187). */
int jt_make_lights(const jt_scene* scene, jt_lights* out);
void jt_free_lights(jt_lights* lights);
/* W,H as make_trace_state (src/trace.jl:189-197) or the width/height extension. */
int jt_image_size(const jt_scene* scene, const jt_params* params, int32_t* width, int32_t* height);

/* ---- device context ---------------------------------------------------------------- */
/* Uploads scene, BVH and lights; allocates zeroed accumulators (make_trace_state).
 * Rejects with JT_ERR_UNSUPPORTED what the reference cannot shade either: shapes with
 * points (src/scene.jl:429), lines without normals (src/scene.jl:605), gltfpbr materials
 * on instances (src/shading.jl:254-321 call undefined functions), and untextured
 * environment lights (src/trace.jl:1003). */
int jt_create(const jt_scene* scene, const jt_scene_bvh* bvh, const jt_lights* lights,
              const jt_params* params, jt_ctx** out);
/* jt_create over several GPUs of one node (SURVEY §8(b) "jt_create(..., num_devices, ...)"; the
 * reference's caller is Jtrace.main's batch loop, src/jtrace.jl:83-106). devices: ndevices
 * distinct HIP ordinals, or NULL for 0 .. ndevices-1 (params->device is ignored). Every other
 * function takes the returned context. Every batch is split across the devices in one of two
 * modes, fixed at creation:
 *   - sample split (params->batch >= ndevices): contiguous per-device shares of the batch's
 *     samples, traced concurrently, each device keeping its own running mean over its samples;
 *     jt_get_image / jt_get_aovs reduce them onto device 0 with one RCCL reduce whose op is a
 *     premultiplied sum (mean_d * n_d / N; hits summed), so the image equals the single-device
 *     one up to fp32 summation order;
 *   - tile split (params->batch < ndevices, e.g. the reference's default --batch 1): device d
 *     traces every sample of the batch on the interleaved 8x8 pixel tiles t with t mod ndevices
 *     == d; the reduce is a plain sum of the disjoint tiles, bit-identical to one device.
 * The option "multi_split" (jt_set_option: "tiles" | "samples") overrides the rule.
 * jt_get_counters sums the devices (kernel_ms: per launch the slowest device);
 * jt_get_device_buffers returns device 0's share. */
int jt_create_multi(const jt_scene* scene, const jt_scene_bvh* bvh, const jt_lights* lights,
                    const jt_params* params, const int32_t* devices, int32_t ndevices, jt_ctx** out);
/* trace_samples (src/trace.jl:215-274): samples [n, min(n+batch, samples)), n += batch
 * (jt_trace_range of that range: it may return before the samples are traced). */
int jt_trace_samples(jt_ctx* ctx);
/* Accumulate global samples [sample_begin, sample_end) into the running mean, in order.
 * Deferred: the range is queued behind the ranges queued before it and all are traced together
 * (one launch per 64 samples or so) once 64 samples are queued, the context's params.samples are
 * reached, or the context is read: jt_get_image / jt_get_aovs / jt_get_counters /
 * jt_get_device_buffers / jt_synchronize trace the queued samples first and report their errors
 * (a failed launch then marks the context failed, as an immediate one would). A context whose
 * device buffers were handed out (jt_get_device_buffers) traces every range at once. Merging
 * changes only the launch count (jt_counters.launches), never the bits (below). jt_get_samples
 * counts queued samples; jt_reset drops them.
 * Sample streams (fixed per context, jt_get_streams: k, a power of two): local sample
 * t = s - first_sample (first_sample: the first sample this context ever traced, 0 for a single
 * device) belongs to stream j = t mod k and is the c-th sample of that stream, c = t div k; every
 * stream keeps its own running mean (src/trace.jl:631-648, weight 1/(c + 1)), and after every
 * call the image / AOVs are the streams' means combined in stream order,
 *     image = sum_{j < min(k, n)} mean_j * w_j,  w_j = (float)((double)n_j / n),
 * n the local samples so far and n_j those of stream j (float multiply-adds without FMA,
 * starting from mean_0 * w_0); hits = sum_j hits_j. k = 1 is the reference's single running mean.
 * The result does not depend on how a render is split into calls. */
int jt_trace_range(jt_ctx* ctx, int32_t sample_begin, int32_t sample_end);
/* The context's sample streams per pixel k (jt_trace_range). Chosen by jt_create from the
 * pixels it traces and the batch only (never the scene or its LDS/HBM mode): 1 when
 * params->batch is 1 (the reference's default); otherwise the smallest power of two k >= 16
 * (>= 32 for a batch of at least 64) with (pixels the context traces) * k >= 2^22, reduced to
 * at most 64, the batch, and (pixels) * k <= 2^27 (at least 1) — halved further while the
 * stream means (48 B per pixel and stream) cannot be allocated; or the "streams" option.
 * k = 1 contexts trace a range of m > 1 samples as chunks of one-sample streams folded into the
 * single running mean in sample order: the bits of one launch per sample. */
int jt_get_streams(const jt_ctx* ctx, int32_t* streams);
int jt_get_samples(const jt_ctx* ctx, int32_t* samples);
int jt_get_size(const jt_ctx* ctx, int32_t* width, int32_t* height);
int jt_get_image(jt_ctx* ctx, float* rgba);                          /* W*H*4 */
int jt_get_aovs(jt_ctx* ctx, float* albedo, float* normal, int64_t* hits); /* W*H*3, W*H*3, W*H */
int jt_get_counters(jt_ctx* ctx, jt_counters* out);
/* zero accumulators (at once if their device pointers were handed out, else before they are
 * next read or overwritten), samples = 0, queued samples dropped */
int jt_reset(jt_ctx* ctx);
/* the accumulators' device pointers, current: queued samples are traced first, and from now on
 * every jt_trace_range traces at once and jt_reset zeroes at once. The image is current when
 * jt_trace_range returns; with k > 1 streams albedo, normal and hits are combined from the
 * streams' means only when read, so through these pointers they are current after
 * jt_synchronize (or jt_get_aovs) */
int jt_get_device_buffers(jt_ctx* ctx, jt_device_buffers* out);
/* Counter level of subsequent launches: 1 (default) counts every jt_counters field; 0 counts
 * paths, rays and light_queries only (the timed production kernel; the other fields are
 * deterministic given seed + BVH and are taken from a level-1 launch of the same range). */
int jt_set_counters(jt_ctx* ctx, int32_t level);
/* NUL-terminated one-line description of the launch configuration the next jt_trace_range
 * uses (kernel instance, LDS/HBM scene mode, stack depth, grid): names the kernel in
 * rocprofv3 traces. Truncated to n bytes. */
int jt_describe(const jt_ctx* ctx, char* buf, int32_t n);
int jt_synchronize(jt_ctx* ctx);
void jt_destroy(jt_ctx* ctx);

#ifdef __cplusplus
}
#endif

#endif /* JTRACE_H */
