/*
 * rtg.h — C ABI of the MI355X-native render loop for the CENG795 XML ray tracer
 * (badiba/raytracer-795).  Plain C, plain pointers and sizes, no C++/torch types.
 *
 * Drop-in seam:
 *   reference  void Scene::renderScene(void)                       src/Scene.h:89, src/Scene.cpp:294-363
 *   reference  ReturnVal BVHMethods::FindIntersection(ray,objs,inst) src/Helper.h:25, src/Helper.cpp:18-80
 *
 *   rtg_scene_create()  replaces the precompute half of renderScene()
 *                        (Perlin table, ComputeObjectTransformations, smooth normals,
 *                        per-object BVH construction: src/Scene.cpp:296-323)
 *   rtg_render()        replaces the per-camera pixel loop of renderScene()
 *                        (8 std::threads of ThreadedRendering -> Single/MultiSample ->
 *                        Shading: src/Scene.cpp:329-362, 269-292, 365-411) and writes
 *                        the float RGB framebuffer the reference keeps in Image::_data
 *                        (src/Image.cpp:16-24) — [y][x][c], 0..255 scale, unclamped.
 *   rtg_trace_closest() replaces BVHMethods::FindIntersection for a batch of rays
 *                        (closest-hit with the reference's object/instance rules).
 *
 * The scene descriptor is exactly what the reference Parser leaves in the global
 * Scene after `new Scene(xml)` (src/Scene.cpp:455-504, src/Parser.h): raw vertices,
 * texture coordinates, objects with their transformation-reference lists, instances,
 * materials, textures (decoded texels), lights in the reference's light order, scalars.
 * All indices keep the reference's conventions: vertex / material / texture indices
 * are 1-based positions (materials[matIndex-1], src/Scene.cpp:375; vertices[idx-1],
 * src/Shape.cpp:300-302), transformation ids are 1-based positions into the per-kind lists
 * (src/Helper.cpp:158).
 *
 * Every function returns RTG_OK (0) or a negative rtg_status; rtg_last_error() returns
 * a thread-local message.  Nothing throws or aborts.  The library copies all inputs to
 * device memory at create time and keeps no pointer into caller memory after return.
 */
#ifndef RTG_H_
#define RTG_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTG_ABI_VERSION 9

typedef enum rtg_status {
    RTG_OK = 0,
    RTG_ERR_INVALID = -1,   /* malformed descriptor / argument */
    RTG_ERR_NO_DEVICE = -2, /* no usable gfx950 device */
    RTG_ERR_OOM = -3,       /* device or host allocation failed */
    RTG_ERR_HIP = -4,       /* HIP runtime error (message in rtg_last_error) */
    RTG_ERR_UNSUPPORTED = -5
} rtg_status;

/* ---- enums mirror src/defs.h:8-11, src/Material.h:7-8, src/Light.h:12, src/Transformation.h:7 ---- */
typedef enum rtg_object_type { RTG_OBJ_SPHERE = 0, RTG_OBJ_TRIANGLE = 1, RTG_OBJ_MESH = 2 } rtg_object_type;
typedef enum rtg_xform_type {
    RTG_XF_TRANSLATION = 1, RTG_XF_SCALING = 2, RTG_XF_ROTATION = 3, RTG_XF_COMPOSITE = 4
} rtg_xform_type;
typedef enum rtg_material_type {
    RTG_MAT_NORMAL = 0, RTG_MAT_MIRROR = 1, RTG_MAT_CONDUCTOR = 2, RTG_MAT_DIELECTRIC = 3
} rtg_material_type;
/* BRDFType order of src/Material.h:8 */
typedef enum rtg_brdf_type {
    RTG_BRDF_NONE = 0, RTG_BRDF_OBP = 1, RTG_BRDF_MBP = 2, RTG_BRDF_MBPN = 3, RTG_BRDF_OP = 4,
    RTG_BRDF_MP = 5, RTG_BRDF_MPN = 6, RTG_BRDF_TS = 7, RTG_BRDF_TSF = 8
} rtg_brdf_type;
/* DecalMode order of src/defs.h:8 */
typedef enum rtg_decal_mode {
    RTG_DECAL_REPLACE_KD = 0, RTG_DECAL_BLEND_KD = 1, RTG_DECAL_BUMP_NORMAL = 2,
    RTG_DECAL_REPLACE_NORMAL = 3, RTG_DECAL_REPLACE_ALL = 4, RTG_DECAL_REPLACE_BACKGROUND = 5,
    RTG_DECAL_NONE = 6
} rtg_decal_mode;
typedef enum rtg_interp { RTG_INTERP_NN = 0, RTG_INTERP_BILINEAR = 1 } rtg_interp;
typedef enum rtg_texture_kind { RTG_TEX_IMAGE = 0, RTG_TEX_PERLIN = 1 } rtg_texture_kind;
typedef enum rtg_noise_conv { RTG_NC_ABSVAL = 0, RTG_NC_LINEAR = 1, RTG_NC_NONE = 2 } rtg_noise_conv;
/* lights are given in the order the reference pushes them (src/Parser.h:1223-1314):
   all Point, then Directional, Spot, Area, SphericalDirectional (environment). */
typedef enum rtg_light_type {
    RTG_LIGHT_POINT = 0, RTG_LIGHT_AREA = 1, RTG_LIGHT_DIRECTIONAL = 2, RTG_LIGHT_SPOT = 3,
    RTG_LIGHT_ENVIRONMENT = 4
} rtg_light_type;

/* One entry of an object's <Transformations> list, e.g. "t1 s2 r1" (src/Parser.h:769-796).
   index is the 1-based position in the list of that kind. */
typedef struct rtg_xform_ref { int32_t type; int32_t index; } rtg_xform_ref;

typedef struct rtg_object_desc {
    int32_t type;            /* rtg_object_type */
    int32_t id;              /* XML id (MeshInstance baseMeshId lookup, src/Parser.h:1181-1186) */
    int32_t material;        /* 1-based material position */
    int32_t num_textures;    /* 0..2 (src/Parser.h:830-853) */
    int32_t textures[2];     /* 1-based texture positions */
    int32_t texture_offset;  /* Mesh: xml textureOffset - vertexOffset (src/Parser.h:1147); others 0 */
    int32_t smooth;          /* Mesh shadingMode="smooth" (src/Parser.h:958-974); ignored otherwise */
    int32_t xform_first;     /* range in rtg_scene_desc.xform_refs */
    int32_t xform_count;
    float blur[3];           /* MotionBlur translation (src/Parser.h:856-861), 0 if absent */
    /* sphere */
    int32_t center;          /* 1-based vertex index */
    float radius;
    /* triangle */
    int32_t v[3];            /* 1-based vertex indices */
    /* mesh */
    int32_t face_first;      /* range in rtg_scene_desc.faces (triples of 1-based vertex indices,
                                vertexOffset already added: src/Parser.h:1109-1149) */
    int32_t face_count;
    /* object light (hw7 <LightSphere> / <LightMesh>, pages/Page7.md:7-13; no reference code):
       is_light = 1 makes the object an emitter of `radiance` from both sides.  Only the path
       tracer (rtg_camera_desc.integrator) treats it as a light; the reference integrator
       shades it like any other object. */
    int32_t is_light;
    float radiance[3];
} rtg_object_desc;

typedef struct rtg_instance_desc {
    int32_t base_object;     /* 0-based index into objects (a Mesh) */
    int32_t id;
    int32_t material;        /* 1-based; overrides the base mesh material (src/Helper.cpp:68) */
    int32_t reset_transform; /* src/Helper.cpp:216-218 */
    int32_t xform_first;
    int32_t xform_count;
    float blur[3];
} rtg_instance_desc;

typedef struct rtg_material_desc {   /* src/Material.h:10-33, src/Parser.h:304-474 */
    int32_t type;            /* rtg_material_type */
    int32_t brdf;            /* rtg_brdf_type */
    int32_t phong_exp;
    int32_t is_rough;
    float roughness;
    float ambient[3];
    float diffuse[3];
    float specular[3];
    float mirror[3];
    float refraction_index;
    float absorption_index;
    float absorption_coeff[3];
} rtg_material_desc;

typedef struct rtg_texture_desc {    /* src/Texture.h:13-51 */
    int32_t kind;            /* rtg_texture_kind */
    int32_t decal;           /* rtg_decal_mode */
    int32_t interp;          /* rtg_interp */
    int32_t noise_conv;      /* rtg_noise_conv (Perlin) */
    int32_t normalizer;
    float noise_scale;
    float bump_factor;
    int32_t width;           /* image textures: texels is width*height*3 floats, */
    int32_t height;          /* row j=0 first, [j][i][c] — the values GetColorAtPixel returns */
    const float* texels;     /* (raw 0..255 for PNG/JPG, linear floats for EXR). */
} rtg_texture_desc;

typedef struct rtg_light_desc {      /* src/Light.h:35-139 */
    int32_t type;            /* rtg_light_type */
    float position[3];       /* point/spot/area */
    float direction[3];      /* directional/spot direction; area normal (normalized by the library) */
    float intensity[3];      /* point/spot intensity; directional/area radiance */
    float coverage_deg;      /* spot CoverageAngle */
    float falloff_deg;       /* spot FalloffAngle */
    float size;              /* area Size */
    int32_t texture;         /* environment: 0-based index into rtg_scene_desc.textures
                                (a bilinear, normalizer-1 image texture) */
} rtg_light_desc;

typedef struct rtg_scene_desc {
    int32_t abi_version;     /* RTG_ABI_VERSION */
    int32_t max_recursion_depth;   /* src/Parser.h:23 default 1 */
    float shadow_ray_eps;          /* default 0.002 */
    float intersection_test_eps;   /* default 0.001 */
    float background[3];
    float ambient_light[3];
    int32_t background_texture;    /* 0-based texture index with decal replace_background, -1 none
                                      (last such texture, src/Scene.cpp:494-500) */
    int32_t environment_light;     /* 0-based light index, -1 none (src/Parser.h:1302-1313) */

    const float* vertices;   int32_t num_vertices;    /* xyz triples */
    const float* texcoords;  int32_t num_texcoords;   /* uv pairs */
    const int32_t* faces;    int32_t num_faces;       /* mesh face triples (1-based vertex idx) */
    const float* translations; int32_t num_translations;  /* xyz */
    const float* scalings;   int32_t num_scalings;        /* xyz */
    const float* rotations;  int32_t num_rotations;       /* angle_deg, x, y, z */
    const float* composites; int32_t num_composites;      /* 16 floats, glm column-major m[col][row] */
    const rtg_xform_ref* xform_refs; int32_t num_xform_refs;
    const rtg_object_desc* objects;  int32_t num_objects;  /* order: spheres, triangles, meshes */
    const rtg_instance_desc* instances; int32_t num_instances;
    const rtg_material_desc* materials; int32_t num_materials;
    const rtg_texture_desc* textures;   int32_t num_textures;
    const rtg_light_desc* lights;       int32_t num_lights;
} rtg_scene_desc;

typedef struct rtg_camera_desc {     /* src/Camera.h:19-67; FovY/GazePoint already resolved */
    float position[3];
    float gaze[3];
    float up[3];
    float left, right, bottom, top;  /* near plane */
    float near_distance;
    int32_t nx, ny;
    int32_t num_samples;
    int32_t is_dof;                  /* FocusDistance present */
    float focus_distance;
    float aperture_size;
    int32_t left_handed;
    /* hw7 <Renderer> / <RendererParams> (pages/Page7.md:15-33, 41-45; no reference code) */
    int32_t integrator;              /* rtg_integrator */
    int32_t pt_flags;                /* rtg_pt_flags (path tracing only) */
} rtg_camera_desc;

typedef enum rtg_integrator {
    RTG_INTEGRATOR_REFERENCE = 0,    /* Scene::RecursiveShading (Whitted / distribution ray tracing) */
    RTG_INTEGRATOR_PATH = 1          /* hw7 path tracer */
} rtg_integrator;
typedef enum rtg_pt_flags {
    RTG_PT_IMPORTANCE = 1,           /* cosine-weighted hemisphere sampling (else uniform) */
    RTG_PT_NEE = 2,                  /* next event estimation towards object lights */
    RTG_PT_RUSSIAN_ROULETTE = 4      /* cosine-based termination, no MaxRecursionDepth cap */
} rtg_pt_flags;
#define RTG_PT_MAX_BOUNCES 32        /* hard cap on path length with Russian roulette */

typedef struct rtg_render_opts {
    uint64_t seed;           /* Philox key for all stochastic draws (reference: random_device) */
    int32_t row_offset;      /* render only rows y with (y / row_block) % row_stride == row_offset; */
    int32_t row_stride;      /* other rows are written as 0 (multi-GPU pixel sharding). 0/1 = all */
    int32_t traversal;       /* 0 = ordered + pruned (default), 1 = exhaustive (literal line test) */
    int32_t max_batch_rays;  /* 0 = auto */
    int32_t collect_stats;   /* 1 = count BVH node visits / triangle tests (slower) */
    int32_t collect_timing;  /* 1 = HIP-event time every closest-hit / shadow launch */
    int32_t streams;         /* passes in flight on separate HIP streams (0 = library default, 8) */
    int32_t row_block;       /* rows per shard interleave block (0/1 = single rows; the pass's pixel
                                tiles become (64/b) x b for b = 1, 2, 4, so they stay image-contiguous) */
    int32_t compact_rows;    /* 1: the output holds only the owned rows, in image order
                                (rows_owned*nx*3 floats; rows_owned = rtg_shard_rows()), for a
                                gather of the shards instead of a full-frame reduce */
    /* In-process multi-GPU fan-out (rtg_render / rtg_render_device; SURVEY.md §8(b) Threading,
       the GPU counterpart of the 8 std::threads of renderScene, src/Scene.cpp:294-363).  0/1: the
       scene's device only.  N > 1: the frame is cut into N shards of row blocks (row_block, 0 = 4;
       shard r owns the rows with (y / row_block) % N == r), one host thread per device renders
       one shard on a replica of the scene (device-to-device copies of the scene's buffers), and
       the shards' rows are gathered onto the scene's device with RCCL point-to-point transfers
       (ncclCommInitAll over the devices; librccl.so.1 is loaded on first use).  row_offset /
       row_stride / compact_rows must be 0. */
    int32_t num_devices;
    const int32_t* devices;  /* NULL: the scene's device followed by the next num_devices-1 device
                                indices (mod rtg_device_count()); else num_devices indices, devices[0]
                                = the scene's device.  A device listed twice takes no RCCL
                                communicator: its shard is copied with hipMemcpyPeer (rehearsal of
                                the N-shard path on fewer GPUs; results are identical). */
    /* ABI 7: ray scheduling.  RTG_SCHEDULE_AUTO: the stream schedule where built (the path
       tracer), else passes.  RTG_SCHEDULE_PASSES: every level of every pass is one launch.
       RTG_SCHEDULE_STREAM: steps that carry the survivors of any level together with new camera
       samples (DESIGN.md §4 "Schedules"); max_batch_rays then caps the rays of one step.  Results
       are bit-identical either way. */
    int32_t schedule;
    /* ABI 8 (these replace the environment knobs of earlier builds; 0 = the library default) */
    int32_t tile_band;       /* pixel order: bands this many 64-pixel tiles high, walked in columns of
                                tiles (0 = 64 owned rows: 8 tiles of 8 rows, 16 of a row shard's 4;
                                DESIGN.md §5).  Results do not depend on it. */
    int32_t segment_pixels;  /* stream schedule, path tracer: pixels whose samples' radiance is buffered
                                per segment (0 = as many as an eighth of the device memory holds) */
    int32_t segment_nodes;   /* stream schedule, reference integrator: a segment takes no new samples
                                once its node records exceed this many (0 = a quarter of the device
                                memory's worth).  Results do not depend on either. */
    int32_t pad_abi8;
} rtg_render_opts;
#define RTG_SCHEDULE_AUTO 0
#define RTG_SCHEDULE_PASSES 1
#define RTG_SCHEDULE_STREAM 2

/* Automatic pass size (rays per pass) of a render: at most 24M rays, lowered so that the level
   buffers of `lanes` passes in flight fit half of `device_bytes` (0 = no memory limit), at 2 x
   (228 + 68 x max(num_lights - 1, 0)) bytes per ray [+ 96 for the path tracer]; at least 64K. */
int64_t rtg_pass_rays(int32_t num_lights, int32_t path_tracer, int32_t lanes, uint64_t device_bytes);

/* Number of image rows y < ny with (y / row_block) % row_stride == row_offset. */
int32_t rtg_shard_rows(int32_t ny, int32_t row_offset, int32_t row_stride, int32_t row_block);

typedef struct rtg_render_stats {
    uint64_t primary_rays;
    uint64_t secondary_rays;
    uint64_t shadow_rays;
    uint64_t total_rays;
    double render_ms;        /* device time of the last rtg_render* call */
    int32_t passes;
    int32_t max_level;
    uint64_t node_visits;    /* collect_stats: 32-byte BVH child records read by closest-hit rays */
    uint64_t tri_tests;      /* collect_stats: triangle tests by closest-hit (primary+secondary) rays */
    uint64_t shadow_node_visits;   /* same for shadow queries */
    uint64_t shadow_tri_tests;
    double trace_ms;         /* collect_timing: summed device time of closest-hit launches */
    double shadow_ms;        /* collect_timing: summed device time of shadow launches */
    int32_t trace_launches;
    int32_t shadow_launches;
    uint64_t trace_steps;          /* collect_stats: BVH node steps (loop iterations) of closest-hit rays */
    uint64_t shadow_steps;
    uint64_t trace_lane_slots;     /* collect_stats: sum over waves of 64 x the wave's longest walk */
    uint64_t shadow_lane_slots;    /*   (SIMD efficiency = trace_steps / trace_lane_slots) */
    double shade_ms;         /* collect_timing: summed device time of the shading launches */
    int32_t shade_launches;
    int32_t devices;         /* devices that rendered the frame (num_devices fan-out or ranks: 1 here) */
    double gather_ms;        /* multi-GPU: host wall time from the last shard's end to the gathered frame */
    uint64_t shadow_blocked;       /* collect_stats: shadow queries found blocked ... */
    uint64_t shadow_blocked_steps; /*   ... their node steps and triangle tests (the remainder of */
    uint64_t shadow_blocked_tris;  /*   shadow_steps / shadow_tri_tests belongs to unblocked queries) */
    double resolve_ms;       /* collect_timing: summed device time of the bottom-up resolve launches */
    double accumulate_ms;    /* collect_timing: summed device time of the sample accumulation launches */
    int32_t resolve_launches;
    int32_t accumulate_launches;
    /* ABI 7, collect_stats: top-level entries (objects / instances) visited by the lanes -- the
       entry-start work of BVHMethods::FindIntersection's object loop (src/Helper.cpp:33-73): ray
       transform, root test, flat meshes' triangles -- and 64 x the entries each wave's loop went
       through.  (steps + entry_visits) / (lane_slots + entry_slots) is the SIMD efficiency with the
       object loop included. */
    uint64_t trace_entry_visits;
    uint64_t trace_entry_slots;
    uint64_t shadow_entry_visits;
    uint64_t shadow_entry_slots;
    /* ABI 7, collect_stats: blocked shadow queries (Light::IsShadow needs the nearest blocker,
       src/Light.cpp:188-204): histograms of the node steps taken before the eventual blocker was
       accepted (finding it) and after (proving it nearest), bins 0, 1, 2, 3-4, 5-8, 9-16, 17-32,
       > 32; and the steps before, summed */
    uint64_t shadow_hist_before[8];
    uint64_t shadow_hist_after[8];
    uint64_t shadow_blocked_steps_before;
    /* ... and the same sum with each blocked query's steps before replaced by the fewest any blocked
       query of its wave took (what sharing the first blocker found in a wave could save at most) */
    uint64_t shadow_blocked_steps_before_wavemin;
    /* ABI 8, collect_stats: wave cycles (shader clock, s_memtime, summed over waves) spent in each
       top-level entry of the linear object loop (entry-box test, ray transform, walk), closest-hit
       and shadow kernels; entries >= 15 share the last slot.  Where the traversal time goes per entry. */
    uint64_t trace_entry_cycles[16];
    uint64_t shadow_entry_cycles[16];
    /* ABI 8, collect_stats: path-tracer shading (k_pt_shade) wave cycles by phase -- hit set-up
       (ray, hit record), next-event estimation (light samples + BRDF), continuation sampling,
       compaction + record stores */
    uint64_t pt_shade_cycles[4];
    /* ABI 9, collect_stats: the flat group (untransformed small meshes tested together):
       the (lane, triangle) tests its lanes ran -- every member triangle's fast rejection, then each lane's
       own candidates' exact tests -- and 64 x the tests each wave ran (the most any of its lanes needed).
       (steps + entry_visits + group_work) / (lane_slots + entry_slots + group_slots) is the SIMD
       efficiency with the group's per-lane work counted.  group_cycles: the group's wave cycles split
       into set-up (ray transform, reciprocals, window) and tests (slot 15 of entry_cycles holds both). */
    uint64_t trace_group_work;
    uint64_t trace_group_slots;
    uint64_t shadow_group_work;
    uint64_t shadow_group_slots;
    uint64_t trace_group_cycles[2];
    uint64_t shadow_group_cycles[2];
} rtg_render_stats;

typedef struct rtg_ray {             /* src/Ray.h:10-12 */
    float origin[3];
    float direction[3];
    float time;
} rtg_ray;

typedef struct rtg_hit {             /* what FindIntersection leaves in ReturnVal for a hit */
    int32_t full;            /* 1 = hit */
    int32_t object;          /* top-level index: [0,num_objects) objects, then instances */
    int32_t prim;            /* primitive index in the object's original (parse) order */
    int32_t material;        /* 1-based material (instance override applied) */
    float t;                 /* gett() distance along the world ray (src/Helper.cpp:41) */
    float point[3];          /* world hit point = ray.getPoint(t) */
    float normal[3];         /* world normal after TransformNormal (src/Helper.cpp:75-77) */
} rtg_hit;

typedef struct rtg_scene rtg_scene;

int32_t rtg_abi_version(void);
const char* rtg_last_error(void);
int32_t rtg_device_count(void);

#define RTG_DEVICE_HOST_ONLY (-1)
/* Build device-resident scene on HIP device `device`.  RTG_DEVICE_HOST_ONLY builds only
   the host-side structures (matrices, normals, BVH) for introspection; such a scene
   cannot render or trace (RTG_ERR_NO_DEVICE). */
int32_t rtg_scene_create(const rtg_scene_desc* desc, int32_t device, rtg_scene** out);

/* BVH builder selection for rtg_scene_create_ex.  All builders produce the reference's tree
   (src/BVH.cpp:64-135) bit for bit; they differ only in where the work runs. */
typedef enum rtg_bvh_builder {
    RTG_BVH_AUTO = 0,   /* GPU for meshes of >= 4096 finite triangles on a device scene, else host
                           (the SAH traversal tree: GPU from 65536 triangles) */
    RTG_BVH_HOST = 1,   /* recursive host build */
    RTG_BVH_GPU = 2     /* level-synchronous GPU build (falls back to host for non-finite input) */
} rtg_bvh_builder;
typedef struct rtg_build_opts {
    int32_t bvh_builder;     /* rtg_bvh_builder */
    int32_t tlas;            /* top-level BVH over objects and instances, replacing the reference's
                                linear object loop (src/Helper.cpp:32-73) with the same result (ties
                                to the first entry): 0 = auto (>= 16 entries), 1 = off, 2 = on
                                (>= 2 entries) */
    int32_t traversal_tree;  /* 0 = fast rays walk an SAH 4-wide tree per mesh (candidates checked for
                                reachability in the reference tree, ties in its order: same results);
                                1 = the reference tree only */
    /* ABI 8: 0 = waves of camera samples and of their shadow queries walk the traversal tree
       together (wave-uniform node loads); 1 = every lane walks alone.  Same results. */
    int32_t uniform_walk;
} rtg_build_opts;
/* rtg_scene_create with build options (NULL = defaults). */
int32_t rtg_scene_create_ex(const rtg_scene_desc* desc, int32_t device, const rtg_build_opts* opts,
                            rtg_scene** out);
typedef struct rtg_build_stats {
    double bvh_build_ms;     /* wall time of all per-object BVH constructions */
    int32_t bvh_gpu_objects; /* objects whose BVH was built on the GPU */
    int32_t num_objects;
    int32_t tlas_nodes;      /* nodes of the top-level BVH (0: linear object loop) */
    int32_t flat_group_entries;  /* ABI 8: entries in the flat group (closest_hit) */
    /* ABI 7: wall-time split of rtg_scene_create (ms), in build order.  Together they cover the
       whole call (total_ms); the reference does this work at the start of renderScene
       (src/Scene.cpp:296-323, BVH.cpp:53-62). */
    double validate_ms;      /* descriptor checks (every face index) */
    double prep_ms;          /* vertices, per-object primitive lists, matrices, smooth normals */
    double median_tree_ms;   /* the reference's median-split trees (= bvh_build_ms) */
    double records_ms;       /* triangle records, reference-node flattening, reachability gates */
    double traversal_tree_ms;/* the SAH 4-wide traversal trees (build + collapse) */
    double top_level_ms;     /* entries, world boxes, top-level BVH, materials, textures, lights */
    double upload_ms;        /* host -> device copies of every scene buffer */
    double total_ms;         /* the whole rtg_scene_create call */
    uint64_t upload_bytes;   /* bytes copied to the device */
    /* ABI 8: traversal trees (SAH) built on the GPU (rtg_bvh_builder applies to both trees), their
       binary nodes before the 4-wide collapse, and an order-independent hash of those nodes (box and
       triangle count of every node): the host and GPU builds of a mesh give the same hash unless a
       range with all centroids equal was halved by count */
    int32_t sah_gpu_objects;
    int32_t pad_abi8;
    uint64_t traversal_nodes;
    uint64_t traversal_hash;
} rtg_build_stats;
int32_t rtg_scene_build_stats(const rtg_scene* scene, rtg_build_stats* out);
int32_t rtg_scene_destroy(rtg_scene* scene);

/* Render one camera; rgb_out is caller-owned host memory of ny*nx*3 floats ([y][x][c])
   (rows_owned*nx*3 with opts->compact_rows). */
int32_t rtg_render(rtg_scene* scene, const rtg_camera_desc* cam, const rtg_render_opts* opts,
                   float* rgb_out);
/* Same, output left in device memory (caller-owned, ny*nx*3 floats on the scene's device),
   enqueued on `stream` (hipStream_t, NULL = default stream). Synchronous on return. */
int32_t rtg_render_device(rtg_scene* scene, const rtg_camera_desc* cam,
                          const rtg_render_opts* opts, float* rgb_out_device, void* stream);
int32_t rtg_last_render_stats(const rtg_scene* scene, rtg_render_stats* out);

/* ---- multi-process multi-GPU (one process per GPU) ------------------------
   The same shard + RCCL gather as rtg_render_opts.num_devices, for callers that run one process
   (rank) per GPU, e.g. under torch.distributed.run: rank 0 makes an id with rtg_comm_unique_id,
   hands the RTG_COMM_ID_BYTES bytes to every rank (any side channel), and each rank calls
   rtg_comm_init_rank (ncclCommInitRank).  rtg_render_ranked renders this rank's row-block shard
   (row_offset = rank, row_stride = nranks, row_block = opts->row_block or 4) and gathers the
   shards' rows into `frame_device` (ny*nx*3 floats on rank 0's device; may be NULL on other
   ranks).  Every rank must call it for the same camera.  Synchronous on return. */
#define RTG_COMM_ID_BYTES 128
typedef struct rtg_comm rtg_comm;
int32_t rtg_comm_unique_id(uint8_t id[RTG_COMM_ID_BYTES]);
int32_t rtg_comm_init_rank(const uint8_t id[RTG_COMM_ID_BYTES], int32_t nranks, int32_t rank, int32_t device,
                           rtg_comm** out);
/* ABI 8: the same with a bound on every wait of the rank (communicator set-up, the failure agreement
   and the gather of rtg_render_ranked): a rank whose peers do not join within timeout_ms aborts the
   communicator (ncclCommAbort) and returns RTG_ERR_HIP instead of blocking; the communicator is then
   unusable (destroy it).  The agreement / gather deadline counts from this rank's own shard end, so it
   must also cover the peers' remaining render time (shard skew).  timeout_ms <= 0: no deadline, which is
   what rtg_comm_init_rank does (round 6, ADVICE r5: a long, imbalanced render must not abort a healthy
   rank). */
int32_t rtg_comm_init_rank_timeout(const uint8_t id[RTG_COMM_ID_BYTES], int32_t nranks, int32_t rank, int32_t device,
                                   int32_t timeout_ms, rtg_comm** out);
int32_t rtg_comm_destroy(rtg_comm* comm);
int32_t rtg_render_ranked(rtg_scene* scene, const rtg_camera_desc* cam, const rtg_render_opts* opts, rtg_comm* comm,
                          float* frame_device, void* stream);

/* hw5 tone mapping (pages/Page5.md:47-53 describes a global operator; src/ has none): the
   Photographic TMO of DESIGN.md §11, from a camera's <Tonemap> (<TMO>Photographic</TMO>
   <TMOOptions>key burn%</TMOOptions> <Saturation> <Gamma>).  Output: 0..255 floats, [y][x][c]. */
typedef enum rtg_tmo { RTG_TMO_PHOTOGRAPHIC = 0 } rtg_tmo;
typedef struct rtg_tonemap_desc {
    int32_t tmo;             /* rtg_tmo */
    float key;               /* TMOOptions[0], e.g. 0.18 */
    float burn_percent;      /* TMOOptions[1]: percentage of the brightest pixels that saturate */
    float saturation;
    float gamma;
} rtg_tonemap_desc;
/* hdr_rgb / ldr_rgb: host arrays of ny*nx*3 floats; the work runs on HIP device `device`. */
int32_t rtg_tonemap(int32_t device, const float* hdr_rgb, int32_t nx, int32_t ny, const rtg_tonemap_desc* tm,
                    float* ldr_rgb);
/* Same on device arrays, enqueued on `stream` (hipStream_t); synchronous on return. */
int32_t rtg_tonemap_device(int32_t device, const float* hdr_rgb_device, int32_t nx, int32_t ny,
                           const rtg_tonemap_desc* tm, float* ldr_rgb_device, void* stream);

/* Batch closest-hit query (BVHMethods::FindIntersection) over host arrays. */
int32_t rtg_trace_closest(rtg_scene* scene, const rtg_ray* rays, int32_t n, rtg_hit* hits,
                          int32_t traversal);

/* Introspection for BVH parity tests: per object (0-based, objects only).
   perm[k] = original primitive index at BVH position k (length num_prims).
   nodes: num_nodes * 4 int32 {left, right, start, end} in the reference's pre-order
   (node, left subtree, right subtree); left/right are node numbers or -1 (null),
   start/end is the primitive range the node covers; leaves have left=right=-1.
   boxes: num_nodes * 6 floats (min xyz, max xyz; leaves hold the leaf's own range box,
   which the reference never tests).  Pass NULL buffers to query the sizes. */
int32_t rtg_scene_object_bvh(const rtg_scene* scene, int32_t object, int32_t* num_prims,
                             int32_t* num_nodes, int32_t* perm, int32_t* nodes, float* boxes);
/* Composed matrices per top-level object (objects then instances): inverse and
   inverse-transpose, glm column-major, 16 floats each. */
int32_t rtg_scene_object_matrices(const rtg_scene* scene, int32_t top_object, float* inverse16,
                                  float* inverse_transpose16);
/* Smooth vertex normals after the precompute of renderScene (src/Scene.cpp:294-318): 3*num_vertices. */
int32_t rtg_scene_vertex_normals(const rtg_scene* scene, float* normals);

#ifdef __cplusplus
}
#endif
#endif /* RTG_H_ */
