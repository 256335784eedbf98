/*
 * rtw_oracle.h -- CPU oracle for the render hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / the timed CPU baseline.  The product (librtw.so) never links or
 * calls it.
 *
 * Parity status: the reference (Rust) cannot be compiled here (no cargo/rustc, crates not
 * vendored) and ships no golden vectors, so this restatement is "parity unpinned" against the
 * Rust binary; it is pinned only by the published rand_xoshiro vector and by the
 * hand-derived known-answer tests in tests/.
 */
#ifndef RTW_ORACLE_H
#define RTW_ORACLE_H

#include "../include/rtw.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RTW_ORACLE_RNG_CTR 0 /* per-(pixel, sample) streams: the device kernel's semantics */
#define RTW_ORACLE_RNG_REF 1 /* per-thread streams + sample split + merge_planes (rendering.rs) */
/* OR-ed into rng_mode: also apply the product's proximity cull (rtw_cull.h) after hit_cond.
 * Not the reference's traversal: used to check that the cull changes no result and to count
 * the culled traversal's work (the device kernel's statistics). */
#define RTW_ORACLE_CULL 0x100

/* rendering::render restated.  ctr mode: `threads` only parallelises over rows (result is
 * independent of it); honours the tile partition in params (owned tiles only, image layout).
 * ref mode: `threads` is the reference's thread_count (split_work_tasks); full image. */
RTW_API int rtw_oracle_render(const rtw_world* w, const rtw_render_params* p, int rng_mode,
                              int threads, float* out_rgb, rtw_render_stats* stats);

typedef struct rtw_oracle_hit {
    int32_t hit;
    float t;
    float position[3];
    float normal[3];
    float uv[2];
    int32_t front_face;
    int32_t material;
} rtw_oracle_hit;

/* Scene::hit (hittable.rs:130-137) for one ray; rng = xoroshiro state (in/out, volumes). */
RTW_API int rtw_oracle_scene_hit(const rtw_world* w, const float origin[3], const float dir[3],
                                 float time, float t_start, float t_end, uint64_t rng[2],
                                 rtw_oracle_hit* out);

/* Camera::ray (camera.rs:175-200) for one jittered point. */
RTW_API int rtw_oracle_camera_ray(const rtw_camera* c, float px, float py, uint64_t rng[2],
                                  float origin[3], float dir[3], float* time);

/* ray_color (rendering.rs:19-71) for one ray. */
RTW_API int rtw_oracle_ray_color(const rtw_world* w, const float origin[3], const float dir[3],
                                 float time, int32_t max_depth, int32_t mode, uint64_t rng[2],
                                 float color[3]);

/* One ctr-mode camera sample's radiance: pixel (x, y), global sample index s. */
RTW_API int rtw_oracle_sample_color(const rtw_world* w, const rtw_render_params* p, int32_t x, int32_t y,
                                    uint32_t s, float color[3]);

/* Scalar spec evaluation on the host (for the device self-test comparison). */
RTW_API int rtw_oracle_eval_scalar(int fn, const float* a, const float* b, int64_t n, float* out);

/* The reference's Aabb::hit_cond AND the product's proximity cull (same layout as
 * rtw_device_eval_node_pass; the checker for the device's node step). */
RTW_API int rtw_oracle_node_pass(const float* box, const float* ray, const float* range, const float* km, int64_t n,
                                 int32_t* out);

#ifdef __cplusplus
}
#endif

#endif
