/*
 * rtw.h -- C ABI of the MI355X path tracer (librtw.so).
 *
 * Drop-in boundary: the reference's hot path is the Rust library function
 *
 *     pub fn render(image_size: Size2i, thread_count: usize, samples_per_pixel: usize,
 *                   max_depth: i32, world: &World, render_mode: RenderMode) -> Vec<Color>
 *                                                              (src/lib/rendering.rs:121-128)
 *
 * `rtw_render` replaces it.  `World` (rendering.rs:12-17) crosses the boundary as the flat,
 * pointer-and-count struct `rtw_world` below: the camera (camera.rs:154-164), the one top-level
 * BVH the builder produces (world_builder.rs:282 -> hittable.rs:352-357) over its flattened leaf
 * list (world_builder.rs:291-328), the primitive / material / texture tables, the background
 * (background_color.rs:3-6) and the optional light-sampling rect
 * (world_scattering_distribution.rs:4-9).  A Rust caller serialises its World into this struct
 * inside the lib crate (several fields are private there); INTEGRATION.md shows that shim.
 *
 * Everything is plain C: pointers, sizes, int status codes.  No torch types.  All entry points
 * return RTW_OK (0) or an RTW_ERR_* code; `rtw_last_error()` returns a thread-local message.
 * The reference panics instead of returning errors; the Rust shim maps non-zero to panic!.
 *
 * Host-side scene construction (WorldBuilder / Camera builder / OBJ loader / demo worlds:
 * src/app/worlds/world_builder.rs, demo_worlds.rs, src/app/obj_loader.rs, camera.rs:11-152) is
 * exported too, so C++ and Python hosts can build the same worlds the Rust app builds; see the
 * second half of the file.
 */
#ifndef RTW_H
#define RTW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTW_API __attribute__((visibility("default")))
#define RTW_ABI_VERSION 2

/* ---- status codes ------------------------------------------------------------------------ */
#define RTW_OK 0
#define RTW_ERR_INVALID_ARGUMENT 1
#define RTW_ERR_NO_DEVICE 2
#define RTW_ERR_HIP 3
#define RTW_ERR_OUT_OF_MEMORY 4
#define RTW_ERR_UNSUPPORTED 5
#define RTW_ERR_IO 6
#define RTW_ERR_PARSE 7

/* ---- enums (values are ABI) ------------------------------------------------------------- */
/* Geometry (hittable.rs:104-110) */
#define RTW_GEOM_SPHERE 0
#define RTW_GEOM_RECT 1
#define RTW_GEOM_BOX 2
#define RTW_GEOM_TRIANGLE 3
/* RectPlane (rect_geometry.rs:8-21): (p0, p1, n) axes = Xy (0,1,2), Xz (0,2,1), Yz (1,2,0) */
#define RTW_PLANE_XY 0
#define RTW_PLANE_XZ 1
#define RTW_PLANE_YZ 2
/* Material (material.rs:42-49) */
#define RTW_MAT_LAMBERT 0
#define RTW_MAT_METAL 1
#define RTW_MAT_DIELECTRIC 2
#define RTW_MAT_DIFFUSE_LIGHT 3
#define RTW_MAT_ISOTROPIC 4
/* Texture (texture.rs:3-20) */
#define RTW_TEX_SOLID 0
#define RTW_TEX_CHECKER 1
#define RTW_TEX_MARBLE 2
#define RTW_TEX_IMAGE 3
/* BackgroundColor (background_color.rs:3-6) */
#define RTW_BG_SKY 0
#define RTW_BG_SOLID 1
/* RenderMode (rendering.rs:94-98) */
#define RTW_MODE_DEFAULT 0
#define RTW_MODE_NORMALS 1
/* Leaf wrappers produced by finish_internal (world_builder.rs:305-316) */
#define RTW_LEAF_VOLUME 1u    /* SceneElement::VolumeGeometry (density < 1) */
#define RTW_LEAF_TRANSFORM 2u /* wrapped in SceneElement::Transformation */
#define RTW_LEAF_ANIMATION 4u /* wrapped (outermost) in SceneElement::Animation */
/* Output layouts of rtw_render_device */
#define RTW_LAYOUT_IMAGE 0 /* W*H*3 f32, row-major from the top-left pixel */
#define RTW_LAYOUT_TILES 1 /* this partition's tiles only, tile-major, tile_w*tile_h*3 f32 each */

/* ---- flat World ------------------------------------------------------------------------- */
/* BVH node (hittable.rs:345-351).  Children: >= 0 node index, < 0 leaf ~index (= -1 - leaf). */
typedef struct rtw_bvh_node {
    float min[3];
    float max[3];
    int32_t axis;
    int32_t left;
    int32_t right;
} rtw_bvh_node;

/* One flattened scene leaf (world_builder.rs:305-316):
 *   Animation(velocity)? ( Transformation(offset, y_sin, y_cos)? ( Volume | Surface ) ) */
typedef struct rtw_leaf {
    int32_t geom_kind;  /* RTW_GEOM_* */
    int32_t geom_index; /* index into the per-kind table */
    int32_t material;   /* material index (phase function for volumes) */
    uint32_t flags;     /* RTW_LEAF_* */
    float neg_inv_density; /* VolumeGeometry::neg_inv_density = -1/density (hittable.rs:305) */
    float offset[3];       /* Transformation (transformations.rs:4-8) */
    float y_sin;
    float y_cos;
    float velocity[3]; /* Animation (hittable.rs:117) */
} rtw_leaf;

typedef struct rtw_sphere { /* sphere_geometry.rs:6-9 */
    float center[3];
    float radius;
} rtw_sphere;
typedef struct rtw_rect { /* rect_geometry.rs:25-30 */
    int32_t plane;
    float dist;
    float r0[2];
    float r1[2];
} rtw_rect;
typedef struct rtw_box { /* aabb.rs:10-13 used as a primitive */
    float min[3];
    float max[3];
} rtw_box;
typedef struct rtw_triangle { /* triangle_geometry.rs:6-10 */
    float positions[3][3];
    float normals[3][3];
    float uvs[3][2];
} rtw_triangle;

typedef struct rtw_material {
    int32_t kind;    /* RTW_MAT_* */
    int32_t texture; /* albedo / emit texture, -1 for dielectric */
    float fuzz;      /* metal */
    float index_of_refraction; /* dielectric */
} rtw_material;

typedef struct rtw_texture {
    int32_t kind; /* RTW_TEX_* */
    float color[3];      /* solid */
    float inv_frequency; /* checker */
    int32_t even, odd;   /* checker: texture indices */
    float scale;         /* marble */
    int32_t perlin;      /* marble: perlin index */
    int32_t image;       /* image: image index */
} rtw_texture;

typedef struct rtw_image { /* image::RgbImage, row 0 = top */
    int32_t width, height;
    const uint8_t* rgb; /* width*height*3 */
} rtw_image;

#define RTW_PERLIN_MAX_POINTS 256
typedef struct rtw_perlin { /* perlin.rs:10-16, bits <= 8 */
    int32_t bits;
    float ranvec[RTW_PERLIN_MAX_POINTS][3];
    uint32_t perm_x[RTW_PERLIN_MAX_POINTS];
    uint32_t perm_y[RTW_PERLIN_MAX_POINTS];
    uint32_t perm_z[RTW_PERLIN_MAX_POINTS];
} rtw_perlin;

typedef struct rtw_camera { /* camera.rs:154-164 (all fields, private ones included) */
    float position[3];
    float upper_left_corner[3];
    float unit_right[3];
    float unit_up[3];
    float scaled_right[3];
    float scaled_up[3];
    float lens_radius;
    float time0, time1;
    float shutter_pace[2];
} rtw_camera;

typedef struct rtw_background {
    int32_t kind; /* RTW_BG_* */
    float color[3];
} rtw_background;

typedef struct rtw_world {
    rtw_camera camera;
    rtw_background background;
    int32_t has_light; /* scattering_distribution_provider.is_some() */
    rtw_rect light;    /* WorldScatteringDistributionProvider::Rect */
    int32_t root;      /* BVH initial_index: node index, or ~leaf for a one-leaf scene */
    int32_t node_count;
    const rtw_bvh_node* nodes;
    int32_t leaf_count;
    const rtw_leaf* leaves;
    int32_t sphere_count;
    const rtw_sphere* spheres;
    int32_t rect_count;
    const rtw_rect* rects;
    int32_t box_count;
    const rtw_box* boxes;
    int32_t triangle_count;
    const rtw_triangle* triangles;
    int32_t material_count;
    const rtw_material* materials;
    int32_t texture_count;
    const rtw_texture* textures;
    int32_t image_count;
    const rtw_image* images;
    int32_t perlin_count;
    const rtw_perlin* perlins;
} rtw_world;

/* ---- render parameters ------------------------------------------------------------------- */
typedef struct rtw_render_params {
    int32_t width, height;      /* image_size: Size2i (width, height >= 2) */
    uint32_t samples_per_pixel; /* >= 1 */
    int32_t max_depth;          /* ray_color depth budget (rendering.rs:19-20) */
    int32_t render_mode;        /* RTW_MODE_* */
    int32_t layout;             /* RTW_LAYOUT_* (rtw_render_device only) */
    uint64_t seed;              /* replaces StdRng::from_entropy (rendering.rs:160) */
    int32_t tile_width;         /* 0 -> 8 */
    int32_t tile_height;        /* 0 -> 8 */
    int32_t part_index;         /* this caller renders tiles t with t % part_count == part_index */
    int32_t part_count;         /* 0 -> 1 */
    /* thread_count of rendering::render (rendering.rs:121-128): the reference splits the samples
     * into thread_count planes (split_work_tasks, rendering.rs:222-237: the first spp % T planes
     * take one sample more, planes of 0 samples are dropped), averages each plane over its own
     * sample count and merges them last-plane-first (merge_planes, rendering.rs:239-252).  The
     * device reproduces that arithmetic exactly (plane t sums samples start_t.. in order).
     * 0 -> 1 (one plane: sum / spp). */
    int32_t thread_count;
    int32_t reserved0; /* must be 0 */
} rtw_render_params;

/* Traversal statistics of one render (for the algorithmic-bytes model). */
typedef struct rtw_render_stats {
    uint64_t samples;
    uint64_t rays;
    uint64_t node_visits;
    uint64_t sphere_tests, rect_tests, box_tests, triangle_tests;
    uint64_t sphere_hits, rect_hits, box_hits, triangle_hits; /* closest hits */
    uint64_t material_reads;
    uint64_t texel_reads;
} rtw_render_stats;

typedef struct rtw_gpu_world rtw_gpu_world; /* a World resident in one device's HBM */

/* ---- render API (librtw.so) -------------------------------------------------------------- */
RTW_API int rtw_version(void);
RTW_API const char* rtw_last_error(void);
RTW_API int rtw_device_count(int* count);

/* Drop-in for rendering::render: uploads `world` to `device`, renders every pixel, copies the
 * linear radiance (W*H*3 f32, row-major from the top-left pixel) into host `out_rgb`. */
RTW_API int rtw_render(const rtw_world* world, const rtw_render_params* params, int device,
                       float* out_rgb);

/* rtw_render with progress reports, the analogue of the reference's progress thread
 * (rendering.rs:140-157): cb(done_samples, total_samples, user) is called from the calling
 * thread about every 50 ms while the frame renders (done_samples counts finished work items of
 * RTW_CHUNK samples), and once more with done == total before returning.  cb == NULL behaves
 * like rtw_render. */
typedef void (*rtw_progress_fn)(uint64_t done_samples, uint64_t total_samples, void* user);
RTW_API int rtw_render_progress(const rtw_world* world, const rtw_render_params* params, int device,
                                float* out_rgb, rtw_progress_fn cb, void* user);

/* rtw_render on several GPUs of one node (one call may use several devices).  The
 * frame's interleaved tile_width x tile_height tiles (params->tile_*, default 8x8) are split over the
 * list: entry i renders the tiles t with t % n_devices == i on devices[i], on its own host thread; the
 * tile buffers reach devices[0] by peer copy over xGMI and are placed there (rtw_untile_device); the
 * image is copied into host `out_rgb` as rtw_render does.  A device may repeat (several partitions on
 * one GPU).  Bit-identical to rtw_render for every list (per-(pixel, sample) RNG streams).
 * params->part_index / part_count must be 0 / 0 or 1: the call partitions the frame itself. */
RTW_API int rtw_render_devices(const rtw_world* world, const rtw_render_params* params, const int* devices,
                               int n_devices, float* out_rgb);
/* The same, resident: rtw_multi_create uploads the world to every listed device once;
 * rtw_multi_render renders one frame and leaves the W*H*3 f32 image in d_image on devices[0]
 * (synchronous: it returns when the image is complete). */
typedef struct rtw_multi rtw_multi;
RTW_API int rtw_multi_create(const rtw_world* world, const int* devices, int n_devices, rtw_multi** out);
RTW_API int rtw_multi_render(rtw_multi* m, const rtw_render_params* params, float* d_image);
RTW_API int rtw_multi_release(rtw_multi* m);
/* Tile-buffer copies this rtw_multi made with hipMemcpyPeerAsync (partitions on a device other than
 * devices[0]; with RTW_MULTI_FORCE_PEER=1 in the environment at rtw_multi_create, every partition's:
 * a same-device peer copy, so one GPU runs the path distinct devices take).  Diagnostics only. */
RTW_API int rtw_multi_peer_copies(const rtw_multi* m, uint64_t* copies);

/* Resident path: upload once, render many times into device memory. */
RTW_API int rtw_world_upload(const rtw_world* world, int device, rtw_gpu_world** out);
RTW_API int rtw_world_release(rtw_gpu_world* gw);
/* The dynamic ray-fetch threshold this world's renders settled on (tuned on the device during
 * the first long render; 0 while still exploring).  Synchronous; performance only -- images do
 * not depend on it. */
RTW_API int rtw_world_tuning(rtw_gpu_world* gw, int* trace_min);
/* The render-kernel variant this world's last render launched: LDS mode (0 scene in HBM, 1 tree +
 * leaf records in LDS, 2 + triangle records), leaf kinds (0 plain spheres .. 4 any), texture
 * kinds (0 solid only, 1 any) and search tree (0 the reference BVH, 1 the kernel's SAH tree with
 * the reference-order proof and fallback); -1 each before the first render.
 * Diagnostics only. */
RTW_API int rtw_world_kernel(rtw_gpu_world* gw, int* lds_mode, int* leaf_kinds, int* tex_kinds, int* tree);
/* The exact template name of that kernel, as profilers print it inside the demangled symbol
 * ("render_kernel<false, 1, 0, 0, false, false>": counting variant, LDS mode, leaf kinds, texture kinds,
 * generic leaf tables in LDS, whole-pixel work items), NUL-terminated into buf[0..cap); "" before the
 * first render.
 * RTW_ERR_INVALID_ARGUMENT if cap is too small.  Diagnostics only (bench.py matches PMC rows by it). */
RTW_API int rtw_world_kernel_name(rtw_gpu_world* gw, char* buf, int cap);
/* The shape of this world's last frame (rtw_render_device / rtw_render on it): render-kernel launches,
 * whether the work items were whole pixels (1: samples summed in registers, no colour buffer, DESIGN.md
 * 5.5b; 0: single samples through the colour buffer), and the dynamic-fetch threshold it ran with (the
 * world's tuned one once chosen, else the default: 32, 16 for whole-pixel frames, or RTW_TRACE_MIN);
 * -1 each before the first frame.  Synchronous; diagnostics only. */
RTW_API int rtw_world_last_frame(rtw_gpu_world* gw, int* launches, int* whole_pixel, int* trace_min);
/* Renders this partition's tiles into device buffer `d_out` (layout per params->layout) on
 * `stream` (a hipStream_t, NULL = default stream).  Asynchronous: returns after the launch. */
RTW_API int rtw_render_device(rtw_gpu_world* gw, const rtw_render_params* params, float* d_out,
                              void* stream);
/* Floats needed by one partition's RTW_LAYOUT_TILES buffer (tiles * tile_w * tile_h * 3). */
RTW_API int rtw_partition_floats(const rtw_render_params* params, int64_t* floats);
/* Scatters part_count gathered tile buffers (each padded to `stride_floats`) into a W*H*3
 * image on the device (rank 0 after the RCCL gather). */
RTW_API int rtw_untile_device(const rtw_render_params* params, const float* d_tiles,
                              int64_t stride_floats, float* d_image, void* stream);
/* Synchronous statistics render (counting variant of the kernel): the reference's traversal
 * (hittable.rs:429-473 DFS over the reference BVH, with the proximity cull). */
RTW_API int rtw_render_collect_stats(rtw_gpu_world* gw, const rtw_render_params* params,
                                     rtw_render_stats* stats);
/* The same counts for the traversal the product kernel runs (tree 1): on worlds that take the SAH
 * walk, its node and leaf visits plus the leaf-box proof and the re-traced rays; elsewhere as
 * tree 0 (= rtw_render_collect_stats).  Approximate where the product kernel uses its wave-
 * cooperative trace: the counting variant re-traces tied rays on the reference tree and
 * walks the drain's last rays instead.  No reference counterpart: feeds the measured record bytes. */
RTW_API int rtw_render_collect_stats_tree(rtw_gpu_world* gw, const rtw_render_params* params, int tree,
                                          rtw_render_stats* stats);
/* Profiling aid (no reference counterpart): the statistics render plus up to n wave-level
 * execution counters of the kernel, in this order: traversal calls, traversal loop iterations,
 * iterations that ran the node step, iterations that ran the leaf step, lane node steps, lane
 * leaf steps, live lanes and lanes waiting for shading (summed over iterations), lanes whose
 * node passed, iterations / lanes testing an inline near sphere child, the same for the far
 * child, shade calls, lanes shaded, wave cycles in traversal, wave cycles elsewhere (refill,
 * ray setup, shading). */
#define RTW_DEBUG_COUNTERS 17
RTW_API int rtw_render_debug_counters(rtw_gpu_world* gw, const rtw_render_params* params,
                                      rtw_render_stats* stats, uint64_t* counters, int n);
/* Output encoder (color.rs:43-48 to_rgb8_gamma2), on the device: d_rgb8 gets W*H*3 bytes. */
RTW_API int rtw_encode_rgb8_device(const float* d_image, int64_t pixels, uint8_t* d_rgb8,
                                   void* stream);

/* Device self-test of the shared scalar spec (rtw_scalar.h): evaluates function `fn` on n
 * inputs on the device; 0 acos, 1 atan2, 2 ln, 3 sin, 4 div, 5 sqrt, 6 rcp-refined div. */
RTW_API int rtw_device_eval_scalar(int device, int fn, const float* a, const float* b, int64_t n,
                                   float* out);

/* Device self-test of the traversal's node step (Aabb::hit_cond, aabb.rs:65-78, AND the proximity
 * cull): for each i, box[6i..] = min xyz, max xyz; ray[6i..] = origin xyz, direction xyz;
 * range[2i..] = t_start, t_end; km[2i..] = the node's cull constants; mk_world as computed at upload
 * (1: node coordinates admit the per-ray exact-division guard).  out[i] = 1 if the node passes.
 * mk_world = 2 evaluates the SAH walk's node test instead (one-multiply quotients,
 * constants widened x17/16 as uploaded) beside the cull alone with exact quotients: out[i] bit 0 =
 * SAH test passes, bit 1 = exact cull passes, bit 2 = the ray admits the exact division.
 * mk_world = 3: the same with the D^2 k term the render kernel uses (2: round 2's Dq form). */
RTW_API int rtw_device_eval_node_pass(int device, const float* box, const float* ray, const float* range,
                                      const float* km, int32_t mk_world, int64_t n, int32_t* out);

/* Device self-test of CheckerTexture's sign test (texture.rs:33-40) as the render kernel evaluates
 * it: out[i] = 1 if RN(RN(sinf(x) sinf(y)) sinf(z)) < 0 for (x, y, z) = xyz[3i..3i+2], else 0. */
RTW_API int rtw_device_eval_checker(int device, const float* xyz, int64_t n, int32_t* out);

/* Device self-check of the exact fast divisions of the render kernel, counted on
 * the device over n cases: test 0 the refined hardware reciprocal against 1/b for b = bits(base + i);
 * test 1 division by pi and tau for a = bits(base + i); test 2 Markstein's correction on random
 * pairs inside its guards; test 3 the guarded division helpers on random pairs of any kind (zeros,
 * subnormals, extremes, infinities, NaN).  *mismatches = cases whose bits differ from IEEE division
 * (NaN = NaN), *first = the first such i (~0 if none). */
RTW_API int rtw_device_check_division(int device, int test, uint64_t base, uint64_t n, uint64_t seed,
                                      uint64_t* mismatches, uint64_t* first);

/* ---- host scene construction ------------------------------------------------------------- */
typedef struct rtw_builder rtw_builder;         /* WorldBuilder + arena (world_builder.rs:7-14) */
typedef struct rtw_world_handle rtw_world_handle; /* owns a finished flat World */
typedef struct rtw_rng rtw_rng;                 /* TRng = Xoroshiro128PlusPlus (common.rs:1) */

RTW_API rtw_rng* rtw_rng_from_seed(const uint8_t seed[16]);
RTW_API void rtw_rng_free(rtw_rng* rng);
RTW_API float rtw_rng_gen_f32(rtw_rng* rng);
RTW_API uint64_t rtw_rng_next_u64(rtw_rng* rng);

RTW_API rtw_builder* rtw_builder_new(void);
RTW_API void rtw_builder_free(rtw_builder* b);
/* Textures / materials return an id >= 0, or -1 on error (see rtw_last_error). */
RTW_API int32_t rtw_texture_solid(rtw_builder* b, float r, float g, float bl);
RTW_API int32_t rtw_texture_checker(rtw_builder* b, float inv_frequency, int32_t even,
                                    int32_t odd);
RTW_API int32_t rtw_texture_marble(rtw_builder* b, float scale, rtw_rng* rng);
RTW_API int32_t rtw_texture_image_rgb8(rtw_builder* b, const uint8_t* rgb, int32_t width,
                                       int32_t height);
RTW_API int32_t rtw_material_lambert(rtw_builder* b, int32_t albedo);
RTW_API int32_t rtw_material_metal(rtw_builder* b, int32_t albedo, float fuzz);
RTW_API int32_t rtw_material_dielectric(rtw_builder* b, float index_of_refraction);
RTW_API int32_t rtw_material_diffuse_light(rtw_builder* b, int32_t emit);
RTW_API int32_t rtw_material_isotropic(rtw_builder* b, int32_t albedo);
/* Nodes (world_builder.rs:104-270). */
RTW_API int32_t rtw_node_group(rtw_builder* b);
RTW_API int32_t rtw_node_sphere(rtw_builder* b, float radius, int32_t material);
RTW_API int32_t rtw_node_rect(rtw_builder* b, int32_t plane, const float center[3], float size0,
                              float size1, int32_t material);
RTW_API int32_t rtw_node_box(rtw_builder* b, float width, float height, float depth,
                             int32_t material);
/* triangles: n records of 24 floats (positions[3][3], normals[3][3], uvs[3][2]) */
RTW_API int32_t rtw_node_mesh(rtw_builder* b, const float* triangles, int32_t n,
                              int32_t material);
RTW_API int rtw_node_add(rtw_builder* b, int32_t parent, int32_t child);
RTW_API int rtw_node_translate(rtw_builder* b, int32_t node, float x, float y, float z);
RTW_API int rtw_node_rotate_around_up(rtw_builder* b, int32_t node, float degrees);
RTW_API int rtw_node_animate_moving(rtw_builder* b, int32_t node, float x, float y, float z);
RTW_API int rtw_node_set_all_geo_as_poi(rtw_builder* b, int32_t node);
RTW_API int rtw_node_set_all_geo_density(rtw_builder* b, int32_t node, float density);

/* Camera builder (camera.rs:11-152).  fov_mode 1: vertical_fov(a, b); 0: viewport(a, b).
 * look_mode 0: orientation(up, target=forward); 1: look_at(up, target); 2: look_at_focus. */
typedef struct rtw_camera_spec {
    int32_t fov_mode;
    float fov_a, fov_b;
    float position[3];
    int32_t look_mode;
    float up[3];
    float target[3];
    int32_t has_focus_distance;
    float focus_distance;
    int32_t has_focus_point;
    float focus_point[3];
    float aperture;
    float time0, time1;
} rtw_camera_spec;
RTW_API int rtw_camera_build(const rtw_camera_spec* spec, rtw_camera* out);
RTW_API float rtw_camera_aspect_ratio(const rtw_camera* cam); /* camera.rs:171-173 */

/* NodeRef::finish (world_builder.rs:273-290): flatten + one BVH over camera.time_interval. */
RTW_API int rtw_builder_finish(rtw_builder* b, int32_t root, const rtw_background* background,
                               const rtw_camera* camera, rtw_world_handle** out);
RTW_API const rtw_world* rtw_world_get(const rtw_world_handle* h);
RTW_API void rtw_world_free(rtw_world_handle* h);

/* obj_loader.rs:7-22 load_obj_mesh, fan-triangulation quirk included.  Returns n triangles as
 * n*24 floats in *out (free with rtw_free). */
RTW_API int rtw_obj_parse(const char* text, size_t len, float** out, int32_t* n);
RTW_API void rtw_free(void* p);

/* Demo worlds (demo_worlds.rs) seeded like main.rs:24.  `name` is "final_scene1",
 * "final_scene2", "cornell_box", "cornell_box_smoke", "cornell_cube", "suzanne",
 * "earth_mapped", "earth_motion", "moving_spheres", "perlin_spheres", "simple_plane",
 * "defocus_blur".  Meshes / images the world needs come in `assets`. */
typedef struct rtw_assets {
    const float* suzanne_tris; /* n*24 floats, from rtw_obj_parse */
    int32_t suzanne_count;
    const float* cube_tris;
    int32_t cube_count;
    const uint8_t* earth_rgb; /* RGB8, row 0 = top */
    int32_t earth_width, earth_height;
} rtw_assets;
RTW_API int rtw_demo_world(const char* name, const rtw_assets* assets, rtw_world_handle** out);

#ifdef __cplusplus
}
#endif

#endif /* RTW_H */
