/*
 * pupil_pt.h — C ABI of the MI355X wavefront path tracer (libpupil_pt.so).
 *
 * This is the drop-in boundary for the reference's OptiX path-tracing pass
 * (example/path_tracer).  Every entry point below replaces one piece of the
 * reference's launch surface:
 *
 *   pupil_pt_create          — optix::Pass::InitPipeline + PTPass::SetScene + World::GetIASHandle
 *                              (example/path_tracer/pt_pass.cpp:29-37,107-209;
 *                               framework/world/gas_manager.cpp:61-185, ias_manager.cpp:29-114)
 *   pupil_pt_set_camera      — CameraHelper::GetCudaMemory upload (framework/world/camera.cpp:72-91)
 *   pupil_pt_update_instance — IASManager::UpdateInstance + IAS::Update
 *                              (framework/world/ias_manager.cpp:116-151,187-211); the engine
 *                              refits its BVH over the moved primitives (topology kept, like
 *                              IAS::Update; PUPIL_FLAT_UPDATE / PUPIL_TL_UPDATE=rebuild rebuild it)
 *   pupil_pt_update_emitters — EmitterHelper reset on RenderInstanceUpdate (world/world.cpp:45-54)
 *   pupil_pt_render          — PTPass::OnRun: optixLaunch(w,h,1) + sync, repeated spp times
 *                              with random_seed++ / sample_cnt += accumulate
 *                              (example/path_tracer/pt_pass.cpp:39-57, main.cu:36-194)
 *   pupil_pt_stats           — no reference equivalent (ray / traversal counters)
 *   pupil_pt_destroy         — pass + world GPU resource teardown
 *
 * The scene crosses the boundary as plain arrays (pupil_scene_desc).  The C++
 * host layer (Pupil::world::World, Pupil::resource::Scene, see
 * pupiloptixlab_amd/csrc/host) produces it from mitsuba-style XML exactly as
 * the reference's World::LoadScene does (framework/world/world.cpp:101-139).
 *
 * Error convention (the reference logs then asserts, framework/cuda/util.h:15-26):
 * every function returns PUPIL_OK (0) or a negative PUPIL_ERR_* code; no C++
 * exception crosses this boundary; pupil_last_error() returns the message of
 * the last failure on the calling thread.
 *
 * Threading: an engine may be driven from any thread (the device is set on
 * every call); calls on one engine must not overlap (the reference serialises
 * SetScene and OnRun under System::m_render_system_mutex, system.cpp:93-173).
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PUPIL_OK 0
#define PUPIL_ERR_INVALID -1
#define PUPIL_ERR_HIP -2
#define PUPIL_ERR_OOM -3
#define PUPIL_ERR_IO -4
#define PUPIL_ERR_UNSUPPORTED -5

/* util::ETextureType (framework/util/texture.h:22-26) */
#define PUPIL_TEX_RGB 0u
#define PUPIL_TEX_BITMAP 1u
#define PUPIL_TEX_CHECKERBOARD 2u

/* EMatType order = framework/decl/material_decl.inl:3-11 (Unknown = 0) */
#define PUPIL_MAT_UNKNOWN 0u
#define PUPIL_MAT_DIFFUSE 1u
#define PUPIL_MAT_DIELECTRIC 2u
#define PUPIL_MAT_ROUGH_DIELECTRIC 3u
#define PUPIL_MAT_CONDUCTOR 4u
#define PUPIL_MAT_ROUGH_CONDUCTOR 5u
#define PUPIL_MAT_PLASTIC 6u
#define PUPIL_MAT_ROUGH_PLASTIC 7u
#define PUPIL_MAT_COUNT 8u

/* optix::EEmitterType (framework/render/emitter/types.h:7-14) */
#define PUPIL_EMITTER_NONE 0u
#define PUPIL_EMITTER_TRI_AREA 1u
#define PUPIL_EMITTER_SPHERE 2u
#define PUPIL_EMITTER_CONST_ENV 3u
#define PUPIL_EMITTER_ENV_MAP 4u

#define PUPIL_SHAPE_MESH 0u
#define PUPIL_SHAPE_SPHERE 1u

/* cuda::Texture (framework/cuda/texture.h:10-57): rgb colour, checkerboard
 * patches, or an RGBA float bitmap; `transform` is the row-major 4x4 to_uv
 * matrix whose rows 0 and 1 map (u, v, 0, 1). */
typedef struct pupil_texture {
    uint32_t type;
    float c0[3];          /* RGB colour, or checkerboard patch1 */
    float c1[3];          /* checkerboard patch2 */
    float transform[16];  /* row-major */
    uint32_t width, height;
    uint32_t filter;      /* BITMAP: 0 point, 1 bilinear (util::ETextureFilterMode) */
    uint32_t pad;
    const float *rgba;    /* host pointer, width*height*4 floats (BITMAP only) */
} pupil_texture;

/* resource::Material (framework/resource/material.h:60-77) flattened.
 * Texture slot meaning per type (same order as the reference's loaders,
 * framework/resource/material.cpp:26-147):
 *   diffuse:          tex[0]=reflectance
 *   dielectric:       tex[0]=specular_reflectance tex[1]=specular_transmittance
 *   rough_dielectric: tex[0]=alpha tex[1]=specular_reflectance tex[2]=specular_transmittance
 *   conductor:        tex[0]=eta tex[1]=k tex[2]=specular_reflectance
 *   rough_conductor:  tex[0]=alpha tex[1]=eta tex[2]=k tex[3]=specular_reflectance
 *   plastic:          tex[0]=diffuse_reflectance tex[1]=specular_reflectance
 *   rough_plastic:    tex[0]=alpha tex[1]=diffuse_reflectance tex[2]=specular_reflectance */
typedef struct pupil_material {
    uint32_t type;
    uint32_t twosided;
    float int_ior, ext_ior;
    uint32_t nonlinear;
    pupil_texture tex[4];
} pupil_material;

/* resource::Shape (framework/resource/shape.h:34-60): object-space mesh or the
 * unit sphere (centre 0, radius 1; radius/centre live in the instance transform,
 * shape.cpp:106-125,196-197). */
typedef struct pupil_shape {
    uint32_t kind;
    uint32_t num_vertices, num_faces;
    const float *positions;  /* 3 * num_vertices */
    const float *normals;    /* 3 * num_vertices or NULL */
    const float *texcoords;  /* 2 * num_vertices or NULL */
    const uint32_t *indices; /* 3 * num_faces */
} pupil_shape;

/* world::RenderObject + pt::HitGroupData (render_object.cpp:10-38, type.h:35-39).
 * to_world/to_object are the row-major 3x4 instance matrix and its inverse
 * (OptixInstance::transform = Transform.matrix.e[0..11], ias_manager.cpp:171). */
typedef struct pupil_instance {
    uint32_t shape;
    uint32_t material;
    float to_world[12];
    float to_object[12];
    uint32_t flip_normals;
    uint32_t flip_tex_coords;
    int32_t emitter_offset; /* first area-emitter index of this instance, -1 if not emissive */
    uint32_t pad;
} pupil_instance;

/* optix::Emitter (framework/render/emitter.h:13-24 + emitter/{area,sphere,env}.h) */
typedef struct pupil_emitter {
    uint32_t type;
    float weight;
    float select_probability;
    float area;
    pupil_texture radiance;
    float pos[3][3];   /* TriArea: world-space vertices */
    float nrm[3][3];   /* TriArea: world-space vertex normals */
    float tex[3][2];   /* TriArea: vertex texcoords */
    float center[3];   /* Sphere centre / env centre */
    float radius;      /* Sphere radius */
    float color[3];    /* ConstEnv colour */
    /* EnvMap: radiance.type == BITMAP; the CDF tables are built by the engine */
    float to_world[9]; /* EnvMap: rows of the 3x3 rotation */
    float to_local[9];
    float scale;
} pupil_emitter;

typedef struct pupil_scene_desc {
    uint32_t width, height;    /* film (scene.cpp:86-95) */
    uint32_t max_depth;        /* integrator (scene.cpp:79-82) */
    uint32_t pad0;
    float sample_to_camera[16]; /* optix::Camera (render/camera.h:7-10), row-major */
    float camera_to_world[16];
    uint32_t num_shapes;
    uint32_t num_materials;
    uint32_t num_instances;
    uint32_t num_area_emitters;
    const pupil_shape *shapes;
    const pupil_material *materials;
    const pupil_instance *instances;
    const pupil_emitter *area_emitters; /* EmitterGroup::areas, select_probability filled */
    const pupil_emitter *env;           /* EmitterGroup::env or NULL */
} pupil_scene_desc;

/* Output views: caller-owned device buffers (BufferManager in the reference,
 * framework/system/buffer.h:44-63).  Any pointer except accum may be NULL.
 * If `compact` is non-zero, buffers are indexed by the rank-local pixel index
 * (see pupil_pt_launch.tile_*), otherwise by y*width+x. */
typedef struct pupil_pt_frame {
    void *accum;  /* float4 "pt accum buffer" */
    void *frame;  /* float4 "final result" */
    void *albedo; /* float3 "albedo" */
    void *normal; /* float3 "normal" */
    void *test;   /* float  "test" */
    uint32_t compact;
    uint32_t pad;
} pupil_pt_frame;

/* One call renders `spp` consecutive frames exactly as spp calls of
 * PTPass::OnRun would (pt_pass.cpp:51-56): frame i uses
 * random_seed = random_seed + i and sample_cnt = sample_cnt + i*accumulate.
 * Tile sharding: the image is cut into tile_size x tile_size tiles numbered
 * row-major; this call renders the tiles t with t % tile_world == tile_rank.
 * tile_world = 1 renders the whole image. */
typedef struct pupil_pt_launch {
    uint32_t random_seed;
    uint32_t sample_cnt;
    uint32_t spp;
    uint32_t max_depth; /* 0 = scene value */
    uint32_t accumulate;
    uint32_t tile_size;
    uint32_t tile_rank;
    uint32_t tile_world;
    /* bit 0 (PUPIL_STATS_COUNTERS): count node visits / primitive tests and the
     * reference's shadow-ray count (slower kernels); bit 1 (PUPIL_STATS_TIMING): HIP
     * events around every stage launch for pupil_pt_stats' per-stage times (each
     * event costs ~6 us of stream gap, so production frames leave it off) */
    /* bit 2 (PUPIL_STATS_TRACE_TIMING): events around the traversal launches only (two
     * per launch); their times are summed over every render since pupil_pt_stats last
     * read them, so a timed sequence of renders reports its own traversal time */
    uint32_t collect_stats;
    /* bit 0 (PUPIL_HINT_CONTINUE): the next renders continue this one (random_seed +
     * spp each, same camera, scene, tiling, spp and max_depth), as consecutive
     * PTPass::OnRun calls do (pt_pass.cpp:55-56).  The engine then pipelines frames:
     * this render's launches also start the frames of the renders after it (camera
     * rays and first bounces, up to max_depth frames in flight), so a continued
     * sequence costs one traversal launch per render.  The render's own frame is
     * complete when its work has run, as without the hint; single-spp renders
     * pipeline without it.  Output is bit-identical either way; a render that does not
     * continue drops the frames ahead and renders its own.  (Was a padding word.) */
    uint32_t hints;
} pupil_pt_launch;

#define PUPIL_STATS_COUNTERS 1u
#define PUPIL_STATS_TIMING 2u
#define PUPIL_STATS_TRACE_TIMING 4u
#define PUPIL_HINT_CONTINUE 1u

typedef struct pupil_pt_counters {
    uint64_t primary_rays;
    uint64_t extension_rays;
    uint64_t shadow_rays;
    uint64_t path_samples;
    uint64_t node_visits;    /* only when collect_stats */
    uint64_t prim_tests;     /* only when collect_stats */
    uint64_t bvh_nodes;
    uint64_t bvh_prims;
    double build_ms;
    double last_render_ms;   /* device time of the last pupil_pt_render (events), recorded only for
                              * renders that set collect_stats or request stage times; 0 otherwise */
    double trace_ms;         /* device time of the traversal kernels in the last render (collect_stats
                              * bit 1), or in every PUPIL_STATS_TRACE_TIMING render since the last read */
    double trace_bytes;      /* algorithmic bytes of the traversal kernels (collect_stats) */
    uint64_t trace_launches;
    /* the dominant kernel (closest-hit extend) on its own: device time, launches,
     * and with collect_stats its node visits / primitive tests / algorithmic bytes */
    double extend_ms;
    uint64_t extend_launches;
    uint64_t extend_node_visits;
    uint64_t extend_prim_tests;
    double extend_bytes;
    double shade_ms;         /* device time of the shade stages (all materials) */
    uint64_t two_level;      /* 1: TLAS over instances + per-shape BLAS; 0: one flattened BVH */
    /* collect_stats: loop iterations that reached the shadow test (main.cu:113-123),
     * i.e. the shadow rays the reference traces unconditionally.  shadow_rays counts
     * only the traced ones: the engine (and the oracle) test occlusion only when
     * f * pdf_L != 0 and NoL > 0, which cannot change the radiance because
     * Eval draws no random numbers (optix_material.h:57-62). */
    uint64_t shadow_rays_reference;
    /* BVH4 levels of the acceleration structure (two-level: TLAS + deepest BLAS); at
     * create, trees needing more than the traversal stacks hold are rebuilt with the
     * Karras LBVH or rejected with PUPIL_ERR_UNSUPPORTED */
    uint64_t bvh_depth;
    /* collect_stats: node fetches counted once per distinct node per wave step (the
     * lanes of a wave on the same node share one fetch) -- the gather rate the memory
     * system serves, comparable with independent random gathers */
    uint64_t unique_node_fetches;
    /* ABI 3.  Rays (camera + extension + shadow) traced since the engine was created, by
     * every render: the exact work of a timed sequence of pipelined renders, whose
     * launches also trace rays of the frames ahead of them */
    uint64_t rays_traced_total;
    /* frames started ahead of the next render (pipelined frames) and the ring size */
    uint64_t frames_in_flight;
    uint64_t pipeline_slots;
    /* two-level structure: TLAS nodes placed by an SAH at the last TLAS build -- every node
     * of a GPU-built TLAS (world mode above 64 entries: PLOC + SAH-optimal collapse), or the
     * host builder's binned-SAH splits (entry ranges above 1024, accel_two_level.hip) */
    uint64_t tlas_sah_splits;
    /* collect_stats, persistent traversal kernels: list items the dequeue heads handed
     * out, lanes activated with them, lanes retired, and the launches' list lengths --
     * all four equal when no ray is lost or traced twice */
    uint64_t queue_handed;
    uint64_t queue_activated;
    uint64_t queue_retired;
    uint64_t queue_listed;
    /* ABI 4.  HBM held by the pipelined-frame ring (path state, queues, AOV scratch) and
     * the budget it may grow to (PUPIL_PIPE_GB, default a quarter of the device memory
     * free at pupil_pt_create) */
    uint64_t ring_bytes;
    uint64_t ring_budget_bytes;
    /* acceleration structure refits / rebuilds done for instance updates since creation:
     * one per pupil_pt_update_instances call, however many instances it moves */
    uint64_t accel_refits;
    /* DeviceScene::node_bound, the per-axis max of |o| + 512 s over the live BVH4 nodes
     * (the slab test's rounding bound is taken per ray from it) */
    float node_bound[3];
    uint32_t pad_counters;
    /* ABI 5.  collect_stats, persistent traversal kernels: SIMD efficiency -- node-loop wave
     * iterations and the lanes active in them, leaf-loop wave iterations and their active
     * lanes, refills and the lanes they activated (active lanes / (64 x iterations) = the
     * fraction of a wave's lanes doing useful work in that loop) */
    uint64_t node_loop_iters;
    uint64_t node_loop_lanes;
    uint64_t leaf_loop_iters;
    uint64_t leaf_loop_lanes;
    uint64_t refills;
    uint64_t refill_lanes;
    /* renders run as one persistent launch per frame (renders that start no frame ahead and
     * have at most PUPIL_FRAME_PATHS paths: the moving-camera OnRun, one rank's tiles) */
    uint64_t frame_launches;
    /* ABI 6.  Device time of those one-launch frames (collect_stats bit 1 / 2): the frame kernel
     * traces and shades, so it is kept out of trace_ms; PUPIL_COOP builds (collect_stats bit 0):
     * the cooperative node fetch's LDS-DMA wave-instructions and node slots */
    double frame_ms;
    uint64_t coop_dma;
    uint64_t coop_slots;
} pupil_pt_counters;

typedef struct pupil_pt pupil_pt;

const char *pupil_last_error(void);
int pupil_abi_version(void);

int pupil_pt_create(const pupil_scene_desc *scene, int device, pupil_pt **out);
int pupil_pt_set_camera(pupil_pt *pt, const float sample_to_camera[16], const float camera_to_world[16]);
/* instance = index into pupil_scene_desc.instances; to_world / to_object row-major 3x4.
 * Must not overlap a render in flight (the reference serialises both under its render mutex). */
int pupil_pt_update_instance(pupil_pt *pt, uint32_t instance, const float to_world[12], const float to_object[12]);
/* n instances at once: ids[k] gets to_world[12k..12k+11] / to_object[12k..]; ONE refit of
 * the acceleration structure covers them all (the reference refits its IAS once per OnRun,
 * however many RenderInstanceUpdate events marked it dirty: pt_pass.cpp:46,216-218).
 * Ordered after every render enqueued so far (stream events, no device-wide sync); returns
 * when the structure is updated.  pupil_pt_update_instance = n = 1. */
int pupil_pt_update_instances(pupil_pt *pt, uint32_t n, const uint32_t *ids, const float *to_world,
                              const float *to_object);
/* replaces the area-emitter table, selection CDF and env emitter (after an emissive instance moved);
 * rewritten in place on the engine's stream when their shapes are unchanged */
int pupil_pt_update_emitters(pupil_pt *pt, const pupil_scene_desc *scene);
/* Asynchronous on hip_stream (a hipStream_t; NULL = the default null stream): the
 * output buffers are complete once work later enqueued on that stream runs.  Exception:
 * with max_depth > 64 the call synchronises hip_stream every 16 bounces to read the list
 * lengths back and stops once no path is left. */
int pupil_pt_render(pupil_pt *pt, const pupil_pt_frame *out, const pupil_pt_launch *launch, void *hip_stream);
int pupil_pt_stats(pupil_pt *pt, pupil_pt_counters *out);
int pupil_pt_local_pixels(uint32_t width, uint32_t height, uint32_t tile_size, uint32_t tile_rank,
                          uint32_t tile_world, uint32_t *out_pixels, uint32_t *inout_count);
void pupil_pt_destroy(pupil_pt *pt);

/* ---- verification entry points (used by the parity tests) ----
 * closest (any_hit = 0) or any hit (any_hit = 1) for n host rays packed as
 * (ox, oy, oz, dx, dy, dz, tmin, tmax); out (host) = (t, b1, b2, prim id bits)
 * per ray, prim id = 0xFFFFFFFF and t = -1 on a miss (any hit: t = 1 if occluded). */
int pupil_pt_trace_rays(pupil_pt *pt, uint32_t n, const float *rays, float *out, int any_hit);
/* copies the flattened BVH4 the traversal kernels read (64-B quantized nodes, 12-float
 * world-space primitive records, root link) to host memory, for the CPU baseline that
 * traverses the same arrays.  Records are the device's record slots (leaf
 * links name slots; every leaf starts on an even slot), 12 floats each; a hole slot between
 * leaves has all bits of its first record's w set.  Call with nodes = records = NULL for the
 * counts.  PUPIL_ERR_UNSUPPORTED for the two-level structure. */
int pupil_pt_export_bvh4(pupil_pt *pt, uint32_t *num_nodes, void *nodes, uint32_t *num_records, float *records,
                         int32_t *root_link);
/* evaluates the device's sin, cos, acos, atan2(x, y2), sqrt, 1/x on n inputs:
 * out[6*i + k] for k in that order (bit-exactness probe for the CPU oracle) */
int pupil_debug_math(int device, uint32_t n, const float *x, const float *y2, float *out);
/* the device's emitter pick (EmitterGroup::SelectOneEmiiter, render/emitter.h:110-135)
 * for n random numbers p: out[i] = area emitter index, -1 = env, -2 = none */
int pupil_debug_select_emitter(pupil_pt *pt, uint32_t n, const float *p, int32_t *out);
/* two-level structure: fills the never-written TLAS reserve [tlas_nodes, tlas_cap) of the
 * node array with nodes whose every float is `value`, then recomputes node_bound (test of
 * the bound's live-node ranges); PUPIL_ERR_UNSUPPORTED for the flattened BVH */
int pupil_debug_fill_tlas_reserve(pupil_pt *pt, float value);

/* ---- image output (util::BitmapTexture::Save, framework/util/texture.cpp:12-85,152-160) ----
 * rgba: width*height float4, row 0 = image bottom (the "final result" order).
 * EXR: uncompressed FLOAT B,G,R, top row first; HDR: Radiance RGBE, top row first;
 * PFM: float RGB, bottom row first.  format PUPIL_IMAGE_AUTO picks by extension. */
enum { PUPIL_IMAGE_AUTO = 0, PUPIL_IMAGE_EXR = 1, PUPIL_IMAGE_HDR = 2, PUPIL_IMAGE_PFM = 3 };
int pupil_image_save(const char *path, uint32_t width, uint32_t height, const float *rgba, uint32_t format);

/* ---- image input (util::BitmapTexture::Load, framework/util/texture.cpp:87-174) ----
 * Decodes an EXR (by the exact extension ".exr": tinyexr LoadEXR semantics), a
 * Radiance HDR (by signature), a PNG or baseline JPEG (stbi_load semantics with the
 * reference's pow(v / 255, 2.2) mapping) or a PFM file into float RGBA, row 0 = image
 * top (the texture order).  Call with rgba = NULL to get the size, then with a
 * buffer of width*height*4 floats.  PUPIL_ERR_IO with pupil_last_error() when the
 * file is unreadable or its format is not supported. */
int pupil_image_load(const char *path, uint32_t *width, uint32_t *height, float *rgba);

/* ---- denoiser (substitute for optix::Denoiser, framework/optix/denoiser.h:7-66) ----
 * The OptiX AI denoiser has no ROCm equivalent; this is an edge-avoiding
 * a-trous wavelet filter (Dammertz et al. 2010): five passes of a 5x5 B3-spline
 * kernel at strides 1, 2, 4, 8, 16, each tap weighted by colour, normal and
 * albedo similarity.  Mode bits and Execute's data follow the reference:
 * UseAlbedo / UseNormal select the guides, UseTemporal blends with prev_output
 * (no motion vectors: static camera), Tiled is accepted (the whole frame is
 * filtered at once), ApplyToAOV and UseUpscale2X return PUPIL_ERR_UNSUPPORTED.
 * Buffers are device pointers: input/output/prev_output float4 per pixel,
 * albedo/normal float3 per pixel (the "albedo"/"normal" AOVs). */
enum {
    PUPIL_DENOISE_USE_ALBEDO = 1,
    PUPIL_DENOISE_USE_NORMAL = 1 << 1,
    PUPIL_DENOISE_APPLY_TO_AOV = 1 << 2,
    PUPIL_DENOISE_USE_TEMPORAL = 1 << 3,
    PUPIL_DENOISE_USE_UPSCALE_2X = 1 << 4,
    PUPIL_DENOISE_TILED = 1 << 5
};
typedef struct pupil_denoise_data {
    const void *input;        /* float4 */
    void *output;             /* float4 (may equal input) */
    const void *prev_output;  /* float4, UseTemporal only (NULL: first frame) */
    const void *albedo;       /* float3, UseAlbedo */
    const void *normal;       /* float3, UseNormal */
    const void *motion_vector; /* unused (must be NULL) */
} pupil_denoise_data;
typedef struct pupil_denoiser pupil_denoiser;
/* Denoiser(mode, stream) (denoiser.h:20-21) */
int pupil_denoiser_create(int device, uint32_t mode, pupil_denoiser **out);
/* SetMode / Setup(w, h) (denoiser.h:24-25); sigma_color scales the colour edge-stopping term (0 = 1.0) */
int pupil_denoiser_setup(pupil_denoiser *d, uint32_t mode, uint32_t width, uint32_t height, float sigma_color);
/* Execute(ExecutionData) (denoiser.h:31-40); asynchronous on hip_stream */
int pupil_denoiser_execute(pupil_denoiser *d, const pupil_denoise_data *data, void *hip_stream);
void pupil_denoiser_destroy(pupil_denoiser *d);

/* ---- host world (the reference's resource::Scene + world::World, C++ inside) ---- */
typedef struct pupil_world pupil_world;

int pupil_world_create(pupil_world **out);
/* mitsuba-3 XML subset, resource/scene.cpp:27-227 semantics */
int pupil_world_load_xml(pupil_world *w, const char *path);
/* programmatic scene building (procedural benchmark scenes) */
int pupil_world_set_film(pupil_world *w, uint32_t width, uint32_t height, uint32_t max_depth);
/* sensor: fov in degrees along fov_axis ('x' or 'y'), to_world row-major 4x4 in mitsuba convention */
int pupil_world_set_sensor(pupil_world *w, float fov, char fov_axis, float near_clip, float far_clip,
                           const float to_world[16]);
int pupil_world_add_mesh(pupil_world *w, uint32_t num_vertices, uint32_t num_faces, const float *positions,
                         const float *normals, const float *texcoords, const uint32_t *indices, uint32_t *out_shape);
int pupil_world_add_builtin_shape(pupil_world *w, const char *name /* rectangle|cube|sphere */, uint32_t *out_shape);
int pupil_world_add_material(pupil_world *w, const pupil_material *m, uint32_t *out_material);
/* is_emitter: area emitter with the given radiance texture */
int pupil_world_add_instance(pupil_world *w, uint32_t shape, uint32_t material, const float to_world[16],
                             uint32_t flip_normals, uint32_t flip_tex_coords, uint32_t is_emitter,
                             const pupil_texture *radiance, uint32_t *out_instance);
int pupil_world_add_const_env(pupil_world *w, const float radiance[3]);
/* RenderInstanceUpdate on the host side: new to_world (row-major 4x4) of instance `instance`
 * (index into pupil_scene_desc.instances); the next pupil_world_get_desc has the new
 * instance matrices and area emitters (world/world.cpp:45-54) */
int pupil_world_set_instance_transform(pupil_world *w, uint32_t instance, const float to_world[16]);
/* resolves emitters (EmitterHelper), camera matrices (CameraHelper) and fills desc;
 * pointers stay valid until the world is modified or destroyed */
int pupil_world_get_desc(pupil_world *w, pupil_scene_desc *desc);
void pupil_world_destroy(pupil_world *w);

#ifdef __cplusplus
}
#endif
