/*
 * rtg_oracle.h — CPU restatement of the badiba/raytracer-795 render loop.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline.
 * The product (librtg.so) never links or calls it.
 *
 * PARITY UNPINNED: the reference ships no tests, fixtures or golden vectors
 *  and cannot be compiled here (Eigen/glm are absent and the
 * task forbids stand-in headers), so this restatement is pinned only by the
 * reference's source text (file:line cited per function in rtg_oracle.c) and by
 * analytic known-answer tests in tests/.
 */
#ifndef RTG_ORACLE_H_
#define RTG_ORACLE_H_
#include "../include/rtg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

int orc_scene_create(const rtg_scene_desc* desc, orc_scene** out);
void orc_scene_destroy(orc_scene* s);

/* Render rows [row_begin,row_end) that satisfy (y / row_block) % row_stride == row_offset
   (row_block <= 1: single-row interleave; the multi-GPU shard of rtg_render_opts).
   rgb: ny*nx*3 floats (rows not rendered are left untouched).
   prim_obj/prim_prim/prim_t (optional, ny*nx each): the closest hit of the primary ray
   of sample 0 (obj -1 on miss), prim in original primitive order.
   nthreads <= 0: OpenMP default. */
int orc_render(orc_scene* s, const rtg_camera_desc* cam, uint64_t seed, int nthreads,
               int row_offset, int row_stride, int row_block, int row_begin, int row_end, float* rgb,
               int32_t* prim_obj, int32_t* prim_prim, float* prim_t);
/* rays traced by the last orc_render: [0]=primary [1]=secondary [2]=shadow */
void orc_last_ray_counts(const orc_scene* s, uint64_t counts[3]);

/* SURVEY §8(d) yardstick (not the reference's algorithm): with enable = 1, later orc_render calls
   also run the canonical ordered early-exit traversal on every ray they trace and count its work.
   out (the last render's totals, may be NULL): [0] closest-hit rays, [1] 32-byte child records,
   [2] triangle tests, [3] sphere tests, [4..7] the same for shadow rays (any hit up to the light). */
void orc_canonical_counts(orc_scene* s, int enable, uint64_t out[8]);

int orc_trace(orc_scene* s, const rtg_ray* rays, int n, rtg_hit* hits);
int orc_object_bvh(const orc_scene* s, int object, int32_t* num_prims, int32_t* num_nodes,
                   int32_t* perm, int32_t* nodes, float* boxes);
int orc_object_matrices(const orc_scene* s, int top_object, float* inv16, float* invT16);
int orc_vertex_normals(const orc_scene* s, float* normals);

/* hw5 Photographic tone mapping: hdr/out ny*nx*3 floats, out 0..255. */
int orc_tonemap(const float* hdr, int nx, int ny, const rtg_tonemap_desc* tm, float* out);

/* Raw Philox4x32-10 block (checked against the Random123 known-answer vectors). */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* Philox4x32-10 uniform draw shared bit-for-bit with the device code (for tests). */
float orc_rng_uniform(uint64_t seed, uint32_t pixel, uint32_t sample, uint64_t path,
                      uint32_t purpose, uint32_t light, uint32_t iter, int lane);

#ifdef __cplusplus
}
#endif
#endif
