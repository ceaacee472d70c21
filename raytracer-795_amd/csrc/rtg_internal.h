// rtg_internal.h — layouts shared by the host scene builder (rtg_host.cpp) and the
// HIP kernels (rtg_device.hip).  Everything here is device-resident, read-only data
// laid out for gfx950 gathers, plus the per-level wavefront queue records.
#pragma once
#include <climits>
#include <stdint.h>

#include <functional>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/rtg.h"

namespace rtg {

constexpr int kMaxLights = 64;      // per-node shadow slots are statically strided
constexpr int kStackDepth = 32;     // reference BVH depth cap 30 (src/BVH.cpp:55,67) + root
// The first 16 traversal-stack entries of a lane live in LDS (4 KB per 64-lane block), deeper ones
// (up to kStackDepth: the reference-tree fallback can need 31) in the lane's scratch: with the
// traversal kernels at 6 waves per SIMD, dragon 33.0 -> 31.6 ms, cornell_pt 392.8 -> 364.3 ms per
// frame (round 3, profiles/history/r3_ab_ldsstack.jsonl; 32 entries in LDS held them at 5 waves).
constexpr int kLdsStack = 16;       // traversal-stack entries per lane in LDS; deeper ones in scratch
constexpr int kTraceBlock = 64;     // threads per traversal block (LDS stack: 128 B per lane)
constexpr int kShadeBlock = 512;    // k_shade (simple variants): one queue atomic per block
constexpr int kTlasMinEntries = 16; // top-level BVH over objects / instances from this many entries on
constexpr int kTlasMaxDepth = 14;   // TLAS leaves at this depth take every remaining entry ...
constexpr int kTlasStack = 16;      // ... so a near-first walk never pushes more than this
constexpr int kTlasNoPrune = 0x40000000;   // TLAS child ref flag: no distance / behind-origin pruning

// One top-level entry of BVHMethods::FindIntersection's loop (src/Helper.cpp:32-73):
// objects first, then instances.  Read with scalar loads (wave-uniform loop).
struct TopObject {
    float inv[16];          // glm::inverse(model), column-major
    float invT[16];         // glm::inverseTranspose(model)
    float blur[3];
    int kind;               // 0 = sphere, 1 = triangle BVH (Triangle or Mesh)
    int material;           // 1-based (instance override applied)
    int geom;               // index of the geometry (base mesh for instances)
    int is_instance;
    int ident;              // 1: inv is exactly the identity (+0 off-diagonal) and blur is +0; 2: a sphere's
                            // inv is the identity up to zero signs and its blur zero (rtg_host.cpp;
                            // traversal only, transform_ray's strict)
    int wbox;               // wlo / whi valid: a transformed entry's world box (root box + eps overhang
    float wlo[3], whi[3];   // through the model matrix, blur sweep for times in [0, 1], margins)
    int grouped;            // a member of the flat group (SceneView::gents): fast rays test it there
    // round 6: a transformed mesh entry (wbox) whose world-space bounding sphere is much tighter than its
    // world box: centre + squared radius (vertices through the model matrix, blur sweep, the eps
    // overhang and margins); the object loop skips the entry for a lane whose ray line misses it
    int bsph;
    float bs[4];
};
// A sphere entry's test data (SceneView::tsph, one per entry, round 6): the object loop tests a sphere
// from this 32-byte record, whose address depends only on the entry index -- not on a dependent load
// of its Geometry record through TopObject::geom.  c = centre, radius; prim = its primitive, -1 none.
struct SphereEnt {
    float4 c;
    int prim, pad_[3];
};

// The flat group (round 5, closest_hit): the identity-transform entries whose mesh is tested without a
// node -- a root leaf, a reference root over two leaves, or a one-node traversal tree (<= kFlatMaxPrims
// triangles each) -- with their triangles in one array in the traversal-record format (p2.y reference
// position, p2.z first position of its reference leaf, p2.w gate flag).  Fast rays filter all of them
// at once and run the exact test on their own candidates only.
constexpr int kGroupMaxTris = 32;   // candidate bits of a lane
constexpr int kGroupMaxEnts = 16;
struct GroupEnt {
    int entry;              // top-level index
    int first, count;       // range in SceneView::gtris (= bits of the candidate mask)
    int root_box;           // 1: the reference root is interior (its box decides reachability)
    float root_min[3], root_max[3];
    int win;                // win_min / win_max valid (Geometry::win): a lane whose parameter window misses
    float win_min[3], win_max[3];   // this box has no candidate here, and a wave with no such lane skips the entry
};

// Per geometry (one per object; instances share their base mesh's geometry).
struct Geometry {
    int type;               // rtg_object_type
    int node_base;          // absolute index of the BVH root in the node array (-1 if root is a leaf)
    int sah_base;           // root of the traversal tree (SceneView::snodes), -1: reference-tree walk
    int root_leaf_start;    // absolute prim range when the root is a leaf (no box test)
    int root_leaf_count;    // -1: no primitives at all
    float root_min[3];      // root box (tested only when the root is interior)
    float root_max[3];
    int prim_base;          // absolute index of BVH position 0
    int nprims;
    float prune_pad;        // max distance a hit point can lie outside its primitive's box
    float win_min[3];       // root box widened by prune_pad, rounded outwards: every candidate
    float win_max[3];       // lies inside (window pruning of the whole object, visit_object)
    int num_textures;
    int textures[2];        // 1-based
    int texture_offset;
    int smooth;
    // sphere
    float center[3];
    float radius;
    int center_index;       // 1-based vertex index
    int win;                // window-test the root box before the walk (meshes of >= RTG_WIN_MIN_PRIMS)
    int flat_first;         // flat_count > 0: test the mesh's <= kFlatMaxPrims triangles without a node
    int flat_count;         // (visit_object): flat_split < 0 -- a one-node traversal tree, stris[flat_first ..];
    int flat_split;         // >= 0 -- a reference root over two leaves, tris[flat_first .. flat_split) and
                            // [flat_split .. flat_first + flat_count) (absolute positions)
};

// 64-byte BVH2 node holding both children's boxes (the reference tests a node's own box
// when it is visited; testing the child's box from its parent is the same predicate).
// a = {Lmin.xyz, Lmax.x}, b = {Lmax.yz, Rmin.xy}, c = {Rmin.z, Rmax.xyz},
// d = {lref, rref, lcount, rcount}: count 0 -> interior child (ref = absolute node index),
// count > 0 -> leaf child with prims [ref, ref+count) (absolute), count < 0 -> null child.
// A leaf child's box is the range box of its primitives, used only for pruning.
struct Node {
    float4 a, b, c;
    int4 d;
};

// 128-byte 4-wide node of a traversal tree (SAH over the triangle boxes, rtg_host.cpp
// sah_collapse).  Per-slot boxes in SoA form.  info: < 0 empty; 0 interior (ref = absolute Node4
// index); > 0 leaf of `info` triangles starting at ref (absolute index into SceneView::stris).
struct Node4 {
    float4 lox, loy, loz, hix, hiy, hiz;
    int4 ref;
    int4 info;
};

// Triangle in BVH order: the Cramer-rule operands of Triangle::bvhIntersect
// (src/Shape.cpp:299-316): a, a-b, a-c.  w lanes: x = original face index.
struct TriGeom {
    float4 p0;  // a.xyz, (a-b).x
    float4 p1;  // (a-b).yz, (a-c).xy
    float4 p2;  // (a-c).z, then (c-b).xyz in the reference-order copy (flat shading normal,
                // hit_record); the traversal copy (stris) holds the reference position, the first
                // position of its reference leaf and the gate flag (int bits) there
};

// Internal light types of hw7 object lights (appended after the scene's lights; only the
// path tracer's NEE loop reaches them).  inten = radiance; mesh: coverage = total world area,
// tri_first/tri_count = range in SceneView::emit_tris / emit_cdf; sphere: pos = world centre,
// size = world radius.
constexpr int kLightEmitMesh = 16;
constexpr int kLightEmitSphere = 17;
struct LightDev {
    int type;
    float pos[3], dir[3], inten[3];
    float coverage, fall, size;
    float normal[3], u[3], v[3];
    int tex;
    float cos_fall, cos_cov;   // host-computed cos() of fall/coverage (same convention)
    int tri_first, tri_count;  // mesh emitters
};

struct TextureDev {
    int kind, decal, interp, nc, normalizer;
    float noise_scale, bump;
    int w, h;
    long long texel_offset;    // into the texel pool (floats)
};

struct MaterialDev {
    int type, brdf, phong_exp, is_rough;
    float roughness;
    float ambient[3], diffuse[3], specular[3], mirror[3];
    float refraction_index, absorption_index;
    float absorption[3];
};

// Everything a kernel needs, passed by value.
struct SceneView {
    const TopObject* tops; int num_tops; int num_objects;
    const Geometry* geoms;
    const Node* nodes;
    const Node4* snodes;           // traversal trees (SAH, 4-wide)
    const TriGeom* stris;          // their triangles in leaf order; p2.y = reference position (int bits),
                                   // p2.z = first position of its reference leaf, p2.w = 1 if gated
    const float* gates;            // per reference position: min xyz, max xyz of its leaf's parent box
    const TriGeom* tris;
    const int4* prim_idx;          // BVH order: {v1,v2,v3 (1-based), smooth}; spheres {c,0,0,0}
    const float* vertices;         // xyz
    const float* vnormals;         // xyz
    const float* texcoords;        // uv
    int num_texcoords;
    const MaterialDev* materials; int num_materials;
    const TextureDev* textures; int num_textures;
    const float* texels;
    const LightDev* lights; int num_lights;
    int max_depth;
    float shadow_eps, int_eps;
    float background[3], ambient[3];
    int bg_texture, env_light;
    int full;                      // 0: no textures / BRDFs / area or environment lights
    int spot;                      // any spot light (its double-precision cone math is compiled in)
    int heavy;                     // a spot or environment light: the full shading variants compile in
                                   // their double-precision libm code only then (light_sample)
    int brdf_only;                 // full only because of BRDFs (no textures / area / environment)
    int brdf_ts;                   // a Torrance-Sparrow (TS / TSF) material: the path tracer's BRDF variants
                                   // compile those models in only then
    int tex;                       // any textured object or BRDF material (k_shade's TEX variant)
    int meta_free;                 // Whitted: no RNG below level 0 (no textures / area / environment
                                   // lights / rough materials): child rays need no RayMeta (their
                                   // depth is max_depth - level, slot and path are unused)
    int lean_shadow;               // one point / spot / directional light: a Whitted shadow query
                                   // stores only origin + contribution (k_shadow rebuilds d, tmax, L)
    int lit_nodes;                 // one light, < kNodeMatMax materials: Whitted nodes store their lit
                                   // colour and k_shadow restores the ambient term if blocked
    int pnt_all;                   // k_shade stores every hit point: a dielectric material absorbs
                                   // (Beer's law reads refracted children's points) or eps >= 1e17
    int has_blur;                  // some object / instance has a nonzero motion-blur vector: the
                                   // ray queues carry times (RayQ::t)
    int bary;                      // some triangle is smooth-shaded or textured: the render path's
                                   // hit records carry the winner's barycentrics (HitPlanes::bg)
    int uni_walk;                  // camera-sample waves may walk the traversal tree wave-uniformly
                                   // (rtg_build_opts.uniform_walk; off: per-lane walks, for the parity
                                   // test that the two agree)
    // hw7 path tracer (per render: the host sets pt_flags and, with NEE, counts the object
    // lights into num_lights)
    const int* top_emit;           // per top-level entry: emitter light index, -1 if not a light
    const float* emit_tris;        // 9 floats per world-space emitter triangle (parse order)
    const float* emit_cdf;         // running float sum of the triangle areas per emitter
    int num_emit;
    int pt_flags;
    // top-level BVH over the entries (Node layout: count 0 = interior child, > 0 = leaf holding
    // entries tlas_idx[ref .. ref+count)); tlas_root -1: the reference's linear loop
    const Node* tlas;
    const int* tlas_idx;
    int tlas_root;
    float tlas_k[3];               // gett() error scale of the axis-aligned entries (closest_hit)
    // the flat group (GroupEnt); num_gents 0: none (top-level BVH scenes never group)
    const TriGeom* gtris;
    const GroupEnt* gents;
    const SphereEnt* tsph;         // per top-level entry: sphere test data (SphereEnt)
    const TopObject* gtop;         // a copy of the first member's entry: the members' common transform, one
                                   // load away (not gents[0].entry -> tops[], round 6)
    int num_gtris, num_gents;
};

// Path state of one path-tracing ray (per level, next to the RayQ planes / RayMeta).
struct PathRec {       // 16 B
    float tr, tg, tb;  // throughput (after the Beer attenuation of the segment, once shaded)
    int flags;         // bit 0: previous bounce specular; bits 8..: medium material (1-based, 0 none)
};

// One batch ("pass") of the frame: pixels [p0, p0 + npass) of the tiled pixel order (8x8, or 16x4 / 32x2 / 64x1 for row-block shards;
// blocks over the rank's owned rows) x samples [s0, s0 + ns).  Ray slot = (t - p0) * ns + (s - s0):
// all samples of a pixel are adjacent, so a wavefront traces near-identical rays.
struct PassDev {
    int s0, ns, p0, npass;
    int row_offset, row_stride, rows_owned, row_block;
    int tile_h;        // pixel tile height: 8, or the shard's row block when that is smaller
    int tile_s;        // tiles per column of a band (the band is tile_s * tile_h rows high)
};

// n / d for n >= 0, d > 0: a shift when d is a power of two (round 6: the pixel order's and the shards'
// divisors -- tile widths, 64-pixel tiles, full-band columns, samples per pixel, row blocks of 1 or 4,
// one shard -- are powers of two except at the image's last band / column; a 32-bit division is ~30
// VALU instructions, and the slot -> pixel map runs for every ray of every shading kernel)
__host__ __device__ inline int idiv(int n, int d) {
    return (d & (d - 1)) == 0 ? (n >> __builtin_ctz((unsigned)d)) : n / d;
}
// Shard row ownership (rtg_render_opts.row_block): owned row k <-> image row y.
__host__ __device__ inline int shard_row(int k, int off, int stride, int block) {
    const int b = idiv(k, block);
    return (b * stride + off) * block + (k - b * block);
}
// owned index of image row y, or -1 when another shard owns it
__host__ __device__ inline int shard_owned_index(int y, int off, int stride, int block) {
    const int b = idiv(y, block);
    const int q = idiv(b, stride);
    if (b - q * stride != off) return -1;
    return q * block + (y - b * block);
}

struct CameraDev {
    float pos[3], gaze[3], up[3], right[3];
    float l, r, b, t, dist;
    int nx, ny;
    float nxDA, nyDA, pw, ph, sw, sh;
    int sample_count, total;
    int dof;
    float focus, aperture;
};

// Wavefront queue records -------------------------------------------------------
// Queued rays (the Ray of src/Ray.h) as planes: a = (o.xyz, d.x), b = (d.y, d.z), t = time.  24 B
// per ray, 28 with times: the time plane is left out (t = nullptr, every time reads 0) when no
// object or instance has a motion-blur vector -- then the time cannot change any result, since
// transform_ray multiplies it by a zero blur and render-path times are finite.  Every queued ray
// is a closest-hit query without a distance bound (tmax = FLT_MAX).
struct RayQ {
    float4* a;
    float2* b;
    float* t;
};
constexpr size_t kRayBytes = 28;    // allocation per queued ray (the three planes)
inline RayQ ray_planes(void* base, long long cap, bool times) {
    char* p = static_cast<char*>(base);
    return RayQ{reinterpret_cast<float4*>(p), reinterpret_cast<float2*>(p + 16 * cap),
                times ? reinterpret_cast<float*>(p + 24 * cap) : nullptr};
}
struct RayMeta {        // 16 B
    int slot;           // sample slot in the batch
    unsigned path_lo, path_hi;
    int depth;          // remaining recursion depth (RecursiveShading's `depth`)
};
struct HitRec {         // 16 B
    int obj;            // top-level index, -1 miss
    int prim;           // BVH-order absolute prim index
    float t;            // gett distance
    int pad;
};
// The render path's hit records (k_trace -> k_shade / k_pt_shade): (object, primitive) per ray, 8 bytes.
// k_shade re-runs the winning test (hit_record); storing the test's ray parameter and barycentrics
// instead was measured slower (round 3, DESIGN.md §4 "hit records").
struct HitPlanes {
    int2* id;       // obj, prim
};
constexpr size_t kHitBytes = 8;
__host__ __device__ inline HitPlanes hit_planes(void* base, long long) {
    return HitPlanes{reinterpret_cast<int2*>(base)};
}

enum NodeKind : int {
    NK_FINAL = 0,       // color final (basic-only leaf, background, replace_all, miss)
    NK_MIRROR = 1,
    NK_DIEL_ENTER = 2,
    NK_DIEL_TIR = 3,
    NK_DIEL_EXIT = 4,
    NK_CONDUCTOR = 5
};

struct NodeRec {        // 48 B, one per traced ray
    float px, py, pz;   // world hit point ((0,0,0) on a miss, src/Helper.cpp:21)
    float cr, cg, cb;   // basic shading, then the resolved color
    int kind;
    float F;            // dielectric Fresnel / conductor Fresnel
    int child0, child1; // refracted / reflected child index in the next level (-1 none)
    int material;
    int slot;
};

// Whitted path: a level's n node records as three planes in the same 48 n bytes (structure of
// arrays), so the kernels that only need a node's colour (accumulate, light sums, final nodes in
// resolve) read 16 B of it, and k_shade stores the point only for hits and the links only for
// non-final nodes.  The path tracer uses the same planes for nodes with traced shadow queries only:
// colour + kind, point + index of the last traced light, throughput + radiance target (PtRad).
struct NodePlanes {
    float4* col;    // cr, cg, cb, kind (int bits; kNodeHit set for hits)
    float4* pnt;    // px, py, pz, F               (hit nodes only)
    int4* link;     // child0, child1, material, -  (kind != NK_FINAL only)
};
constexpr int kNodeHit = 0x400;
constexpr int kNodeFar = 0x800;    // hit point with a coordinate >= 1e18 or not finite (k_resolve)
// Single-light Whitted path (round 5, SceneView::lit_nodes): a node whose shadow query is traced
// stores its lit colour (ambient + the light's term) and its material index in the kind word's bits
// 12..30; k_shadow rewrites the colour to the ambient term only for a blocked query.  Scenes with more
// materials keep the contribution plane (lit_nodes = lean_shadow = 0).
constexpr int kNodeMatShift = 12;
constexpr int kNodeMatMax = 1 << 19;
inline NodePlanes node_planes(NodeRec* base, long long n) {
    float4* b = reinterpret_cast<float4*>(base);
    return NodePlanes{b, b + n, reinterpret_cast<int4*>(b + 2 * n)};
}

struct ShadowRec {      // 48 B per query (the allocation unit of a level's shadow planes)
    float4 o;           // origin.xyz, time
    float4 d;           // direction.xyz, dl = |p - light point| (modes 1 / 3; k_shadow rebuilds the t bound)
    float4 c;           // contribution rgb, mode (0 none, 1 distance test, 2 any hit, 3 object light)
};

// A level's shadow records as planes (round 6): the origin per shading node (o[i]; the lean
// single-light path stores it as 12-byte records), direction + light distance and contribution per
// query, LIGHT-MAJOR: query (node i, light li) at li * nn + i, so the queries of one light that a
// wave traces (the list is light-major within a wave) read consecutive records -- node-major
// (i * nLights + li) left every 128-byte line of d / c half used by a wave (C5: 142 B per query).
// No light-point plane: k_shadow's blocking tests need only dl, and the query's mode follows from
// the light's type (shadow_mode).
struct ShadowPlanes {
    float4* o;      // origin.xyz, time                      (per node)
    float4* d;      // direction.xyz, dl                     (per query)
    float4* c;      // contribution rgb, mode                (per query; several lights: k_shadow zeroes the
                    // mode of a blocked query)
    int nn;         // nodes of the level: the light stride of d / c
};
inline ShadowPlanes shadow_planes(ShadowRec* base, int nodes, int lights) {
    float4* b = reinterpret_cast<float4*>(base);
    const long long cap = (long long)nodes * (lights > 1 ? lights : 1);
    return ShadowPlanes{b, b + nodes, b + nodes + cap, nodes};
}

struct Counters {
    unsigned long long node_visits, tri_tests;           // closest-hit kernel
    unsigned long long shadow_node_visits, shadow_tri_tests;
    unsigned long long trace_lane_slots, shadow_lane_slots, trace_steps, shadow_steps;
    // shadow queries found blocked, and the node steps / triangle tests they took (the rest of
    // shadow_steps / shadow_tri_tests went to unblocked queries)
    unsigned long long shadow_blocked, shadow_blocked_steps, shadow_blocked_tris;
    // top-level entries visited by the lanes, and 64 x the entries each wave's loop went through
    unsigned long long trace_entry_visits, trace_entry_slots, shadow_entry_visits, shadow_entry_slots;
    // blocked shadow queries: histograms (bins 0, 1, 2, 3-4, 5-8, 9-16, 17-32, >32) of the node steps
    // taken before the blocker was accepted and after it, and the summed steps before
    unsigned long long shadow_hist_before[8], shadow_hist_after[8], shadow_blocked_steps_before;
    unsigned long long shadow_blocked_steps_before_wavemin;
    // wave cycles (s_memtime) spent per top-level entry of the linear object loop (entries >= 15 pooled
    // in the last slot), closest-hit and shadow kernels: where the traversal's time goes
    unsigned long long trace_entry_cycles[16], shadow_entry_cycles[16];
    // k_pt_shade wave cycles by phase: hit set-up, next-event estimation, continuation, compaction + stores
    unsigned long long pt_shade_cycles[4];
    // the flat group (round 6): lane work (triangle tests the lanes ran) and slots (64 x the tests their
    // waves ran), and its wave cycles split into set-up and tests
    unsigned long long trace_group_work, trace_group_slots, shadow_group_work, shadow_group_slots;
    unsigned long long trace_group_cycles[2], shadow_group_cycles[2];
};

// The path tracer's radiance (round 6): the running sum L of a sample travels with its
// path.  k_pt_shade reads it from the ray's queue slot (carry_in[i]; a new sample starts from (0,0,0)).
// A vertex whose contribution is final there (no traced shadow query) adds T (x) v itself and hands L
// to its continuation (carry_out at the child's queue index) or, the path's last vertex, writes
// rad[slot]; a vertex with traced queries leaves L in its own queue slot (carry_in[i], read by then)
// and its last light's query in k_shadow (per-light launches, in light order) writes L + T (x) v to the
// target -- node-indexed, so k_shadow loads it with the node's other records in one round, and the
// last light's launch (every query in it is its node's last) loads all of them unconditionally.  No
// per-level gather kernel.  lcnt: the level's per-light shadow-list counts (light li's list at
// slist + li * n).
struct PtRad {
    float4* carry_in;
    float4* carry_out;
    float4* rad;
    unsigned* lcnt;
    int light;          // k_shadow: the light of this launch's list (its entries are light * n + node)
};
constexpr size_t kCarryBytes = 16;    // float4 per queued ray

// Host-side launchers (rtg_device.hip) ------------------------------------------------
struct LevelBuffers;
// gen_cam / gen_ps non-null: level 0 (either integrator), rays are generated in the kernel
// nq / gbase (with gen_cam): rays [0, nq) are queued, ray i >= nq is the primary ray of slot gbase + i - nq
void launch_trace(const SceneView& sv, const RayQ rays, HitRec* hits, int n, int exhaustive,
                  Counters* ctr, hipStream_t st, const CameraDev* gen_cam = nullptr, const PassDev* gen_ps = nullptr,
                  uint64_t seed = 0, bool compact = false, int nq = 0, int gbase = 0);
// gen: 1 = rays i >= nq are primary rays of slots gbase + i - nq, 0 = queued only, -1 = a pass's level
// (primaries iff rays.a is null); lv_in / lv_out: per-ray levels of a stream step (or null)
void launch_shade(const SceneView& sv, const CameraDev& cam, int level, const PassDev& ps, uint64_t seed, const RayQ rays, const RayMeta* meta, const HitRec* hits, NodeRec* nodes,
                  ShadowRec* shadows, int* slist, const RayQ next_rays, RayMeta* next_meta,
                  unsigned long long* qcount, int n, hipStream_t st,
                  int gen = -1, int nq = 0, int gbase = 0, const unsigned char* lv_in = nullptr,
                  unsigned char* lv_out = nullptr);
// the bottom-up step and the accumulation on explicit node planes (stream schedule: a step's nodes
// [0, count) against the next step's; the primaries of a pixel range at an offset of a step's planes)
void launch_resolve_planes(const SceneView& sv, const NodePlanes& self, const NodePlanes& child, int count,
                           hipStream_t st);
void launch_accumulate_planes(const SceneView& sv, const NodePlanes& level0, const NodePlanes& level1, bool resolve,
                              float* acc, const PassDev& ps, int nx, int mode, hipStream_t st);
void launch_shadow(const SceneView& sv, ShadowRec* shadows, const int* slist, const unsigned* scount, NodeRec* nodes,
                   int n, int exhaustive, Counters* ctr, unsigned* nan_queries, hipStream_t st, bool whitted = true, int uni_from = INT_MAX);  // uni_from: first camera-sample node (wave-uniform walk)
// the path tracer's queries: one launch per light, in light order (PtRad)
void launch_pt_shadow(const SceneView& sv, ShadowRec* shadows, const int* slist, NodeRec* nodes, int n, int exhaustive,
                      Counters* ctr, unsigned* nan_queries, hipStream_t st, int uni_from, const PtRad& pr);
void launch_pt_shade(const SceneView& sv, const CameraDev& cam, int level, const PassDev& ps, uint64_t seed,
                     const RayQ rays, const RayMeta* meta, const HitRec* hits, PathRec* paths, NodeRec* nodes,
                     ShadowRec* shadows, int* slist, const RayQ next_rays, RayMeta* next_meta, PathRec* next_paths,
                     unsigned long long* qcount, int n, hipStream_t st, bool gen, int nq, int gbase,
                     const unsigned char* lv_in, unsigned char* lv_out, const PtRad& pr, Counters* ctr = nullptr);
void launch_resolve(const SceneView& sv, NodeRec* nodes, const NodeRec* child_nodes, int n, int n_child,
                    hipStream_t st);
// levels p (nodes) and p + 1 (child_nodes, resolved inline, not stored) against the resolved level p + 2
void launch_resolve2(const SceneView& sv, NodeRec* nodes, const NodeRec* child_nodes, const NodeRec* grand_nodes, int n,
                     int n_child, int n_grand, hipStream_t st);
// mode: 0 = continue the running sum, 1 = start from (0,0,0), 2 = assign (single-sample camera)
// level0 / level1 hold NodePlanes over n0 / n1 nodes; whitted: resolve level 0 against level 1
// level2 (optional): level 1 is resolved inline against it (the bottom-up pass left level 1 unresolved)
void launch_accumulate(const SceneView& sv, const NodeRec* level0, const NodeRec* level1, bool resolve, float* acc,
                       const PassDev& ps, int nx, int mode, hipStream_t st, bool whitted, int n0, int n1,
                       const NodeRec* level2 = nullptr, int n2 = 0);
void launch_finalize(const float* acc, float* out, int nx, int ny, int row_offset, int row_stride, int row_block, int total,
                     hipStream_t st);
void launch_hit_details(const SceneView& sv, const RayQ rays, const HitRec* hits, struct ::rtg_hit* out,
                        const int* orig_prim, int n, hipStream_t st);

// Traversal-tree build records (rtg_host.cpp sah_split, rtg_sah_gpu.hip): one triangle's box and face
// index (32 B; the centroid is the box centre), and the binned-SAH BVH2 node over a range of them.
constexpr int kSahBins = 16;
constexpr int kSahMaxLeaf = 4;
struct SahRec {
    float lo[3], hi[3];
    int idx, pad_;
};
struct SahNode2 {
    float lo[3], hi[3];
    int left, right;          // children (-1 for a leaf)
    int start, count;         // range in the SAH primitive order (interior nodes too)
};

// Multi-GPU rows gather: shard r's compact rows start at row prefix[r] of `recv`; every frame
// row y is copied from its owning shard ((y / block) % nranks).  nranks <= kMaxRanks.
constexpr int kMaxRanks = 64;
struct ShardPrefix { int rows[kMaxRanks + 1]; };
void launch_place_rows(const float* recv, float* frame, int nx, int ny, int nranks, int block, const ShardPrefix& pre,
                       hipStream_t st);

// Hooks between the C ABI's single-device driver (rtg_host.cpp) and the multi-GPU fan-out
// (rtg_multi.cpp).  rtg_scene is the opaque ABI handle (defined in rtg_host.cpp).
struct MultiState;
void multi_free(MultiState* m);
int set_error(int code, const std::string& msg);           // sets rtg_last_error() of this thread
int scene_device(const rtg_scene* s);
int scene_render(rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_opts* o, float* out_dev, hipStream_t st);
rtg_render_stats scene_stats(const rtg_scene* s);
void scene_set_stats(rtg_scene* s, const rtg_render_stats& st);
MultiState*& scene_multi(rtg_scene* s);
int scene_replicate(rtg_scene* src, int device, rtg_scene** out);
int render_multi(rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_opts* o, float* out_dev, hipStream_t st);

// Photographic tone mapping (rtg_tonemap.hip); hdr / out are device arrays.
int tonemap_white_index(int n, float burn_percent);
int tonemap_device(const float* hdr, int nx, int ny, const rtg_tonemap_desc& tm, float* out, hipStream_t st,
                   std::string& err);

// GPU BVH construction (rtg_bvh_gpu.hip): the reference median-split tree of one object.
// nodes: breadth-first {left, right, start, end} (children -1: none); box: 6 floats per node
// (min xyz, max xyz); perm: BVH position -> original primitive.  Inputs must be finite.
// Page-locked host array (hipHostMalloc): device-to-host copies into it run at DMA speed (the
// GPU build's 84 MB result for 1 M triangles: 16 ms into pageable vectors).
template <class T>
struct PinnedBuf {
    T* p = nullptr;
    size_t n = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    PinnedBuf(PinnedBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    PinnedBuf& operator=(PinnedBuf&& o) noexcept {
        if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
        return *this;
    }
    ~PinnedBuf() { release(); }
    hipError_t alloc(size_t count) {
        release();
        if (count == 0) return hipSuccess;
        const hipError_t e = hipHostMalloc((void**)&p, sizeof(T) * count, hipHostMallocDefault);
        if (e == hipSuccess) n = count; else p = nullptr;
        return e;
    }
    void release() { if (p) (void)hipHostFree(p); p = nullptr; n = 0; }
    size_t size() const { return n; }
    T& operator[](size_t i) { return p[i]; }
    const T& operator[](size_t i) const { return p[i]; }
};

// Page-locked staging from a process-wide pool: hipHostMalloc of the ~80 MB a 1 M-triangle build
// returns costs milliseconds per scene creation, so the buffers are kept and reused.
// get returns a buffer of at least `bytes` and its real capacity in *cap; put takes the capacity back.
void* pinned_pool_get(size_t bytes, size_t* cap);
void pinned_pool_put(void* p, size_t cap);
struct PooledPinned {
    void* p = nullptr;
    size_t cap = 0;           // the buffer's real capacity (>= the bytes last asked for)
    PooledPinned() = default;
    PooledPinned(const PooledPinned&) = delete;
    PooledPinned& operator=(const PooledPinned&) = delete;
    ~PooledPinned() { if (p) pinned_pool_put(p, cap); }
    bool get(size_t b) {
        if (p && cap >= b) return true;
        if (p) pinned_pool_put(p, cap);
        cap = 0;
        p = pinned_pool_get(b, &cap);
        return p != nullptr;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};
// The GPU median-split build's result: nodes in breadth-first order (children after their parent) as
// 40-byte records {left, right, start, end, min xyz, max xyz} (the host's HNode layout), and the
// primitive permutation.
struct GpuBvh {
    PooledPinned perm;       // int[n]
    PooledPinned nodes;      // 40 B per node
    int num_nodes = 0;
    int root = -1;
};
int gpu_build_bvh(const float* centers, const float* bmin, const float* bmax, int n, GpuBvh& out, std::string& err,
                  hipStream_t st);
// GPU binned-SAH build of one mesh's traversal tree (rtg_sah_gpu.hip), collapsed to 4-wide nodes on the
// device as rtg_host.cpp collapse_node does (slot boxes widened by `pad`, leaf refs from tri_base, interior
// refs 0-based within the mesh, breadth-first): alloc4(count) returns host memory for the Node4 records
// (count 0: the root is a leaf); the face index of every SAH position into order_host[n]; the binary
// tree's node count and order-independent hash (sah_tree_stats).  Runs on its own non-blocking stream of
// the calling thread's current device.
int gpu_build_sah(const SahRec* recs_host, int n, int tri_base, float pad, const std::function<Node4*(size_t)>& alloc4,
                  int* order_host, uint64_t& bvh2_nodes, uint64_t& hash, std::string& err);
// Empty launches that load the GPU build's / the render kernels' code objects (scene-create warm-up).
void gpu_bvh_warm(hipStream_t st);
void device_warm(hipStream_t st);

}  // namespace rtg
