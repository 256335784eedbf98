// rtw_device.hip -- the MI355X (gfx950) path-tracing megakernel and its C ABI.
//
// Hot path restated for the device (reference: src/lib/rendering.rs:19-220):
//   a persistent kernel, one 1024-thread block per CU with the scene (nodes, leaf records, cull
//   constants, shading tables) staged in LDS.  Each lane runs a state machine PIXEL -> TRACE ->
//   SHADE over work items taken from 16 queues in per-wave batches: an item is one (pixel, sample)
//   -- or, with whole-pixel items, all of a pixel's samples -- and its colour goes to a per-sample
//   buffer that accumulate_kernel sums per pixel in sample order (the reference's sequential
//   `.sum::<Color>()`, rendering.rs:172-179), so the image does not depend on which lane, wave or
//   GPU rendered a sample (one RNG stream per (pixel, sample)).
//   Closest hits are found on the kernel's own SAH tree (2- or 4-wide) with the proximity cull
//   alone, then proven to be the reference DFS's answer (hittable.rs:429-473) with one slab test on
//   the leaf's parent box in the reference tree; rays the proof does not cover are re-traced on the
//   reference tree in the reference's order (near child first by ray.direction[axis] > 0, both
//   children, te shrinking).  Ties are resolved by the leaves' reference DFS keys (coop_solve).
//   Candidate tests compute only `t`; the hit record is rebuilt once for the closest leaf -- a pure
//   function of (leaf, ray, t).  Volumes draw their RNG during traversal in the reference's order
//   (their worlds keep the reference tree).
//
// Scene data lives in one HBM arena as SoA float4 streams (see DESIGN.md "Data layout").
// Numerics: -ffp-contract=off, no fast-math; shared scalar spec in include/rtw_scalar.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/rtw_scalar.h"
#include "../../include/rtw_cull.h"
#include "rtw_common.h"

#ifndef RTW_BLOCK
#define RTW_BLOCK 1024  // 16 waves: one block per CU at <= 128 VGPRs -> 4 waves per SIMD, one LDS scene copy per CU
#endif
#ifndef RTW_MIN_WAVES_PER_SIMD
#define RTW_MIN_WAVES_PER_SIMD 4
#endif
#ifndef RTW_WAVE_BATCH
#define RTW_WAVE_BATCH 128  // work items a wave reserves per global atomic (upper bound; 64: final_scene1
                            // -0.9 %, earth_motion -0.9 %, profiles/r03/v12_queue_batch_ab.txt)
#endif
#ifndef RTW_WAVE_BATCH_BIG
#define RTW_WAVE_BATCH_BIG 1024  // the same past the first items of a launch (the costly tiles in cost order)
#endif
#ifndef RTW_BIG_BATCH_FROM
#define RTW_BIG_BATCH_FROM 100  // that prefix, per mille of the launch's items (env overrides)
#endif
// The launch's work items are spread over RTW_QUEUES counters 256 B apart: queue q owns the
// granules of RTW_QGRAN consecutive items whose index is q mod RTW_QUEUES, and a wave draws from
// its own queue, moving on to the next one when that is empty.  Every queue walks the launch's
// order (chunk-major or cost order) at the same pace.  One counter served every wave's refill
// batch: a device-scope atomic on one address was the frame's limiter at 64-item batches (final_scene1
// +10 % with 1024-item batches, which in turn let costly tiles pile up in one wave's reserve).
#ifndef RTW_QUEUES
#define RTW_QUEUES 16
#endif
// (Fetching a wave's next batch one refill ahead was slower -- final_scene1 -3 %, suzanne -9 %,
// profiles/r03/v1_queue_ab.txt: the pending atomic holds back the wave's next vector-memory waits and a
// wave holds two batches -- so the batch is fetched when the reserve runs out.)
#define RTW_QGRAN 64
#define RTW_QSTRIDE 32  // u64 counters per queue slot (256 B)
// a frame's launch l takes its items from queue block min(l, RTW_QUEUE_SLOTS - 1) of the world's
// counters, so a progress poller can read how many items each launch has handed out
#define RTW_QUEUE_SLOTS 32
#define RTW_QUEUE_BLOCK (RTW_QUEUES * RTW_QSTRIDE)  // u64 per launch slot
#define RTW_QUEUE_BYTES ((size_t)RTW_QUEUE_SLOTS * RTW_QUEUE_BLOCK * sizeof(unsigned long long))
#ifndef RTW_BATCH_SPREAD
#define RTW_BATCH_SPREAD 8  // a batch is at most 1/(SPREAD x waves) of the launch's remaining items
#endif
#define RTW_STACK 32    // per-lane traversal stack (LDS), >= the BVH depth (checked at upload)
#ifndef RTW_SAH_SPLIT_BUDGET
#define RTW_SAH_SPLIT_BUDGET 1.0  // spatial splits in the SAH tree of triangle worlds: extra references per leaf
#endif
#ifndef RTW_LDS_SCENE_MAX
#define RTW_COOP_MAX 32      // drain: live lanes at most for the wave-cooperative trace (RTW_COOP_MAX=0: off); 4: suzanne -1.1 %, its 8-way shares up to 64.5 ms against 59.4 (profiles/r04/v3_experiments_ab.txt, v4_...)
#define RTW_COOP_LEAVES 4096 // ... in worlds of at most this many leaves
#define RTW_MB_POLLS (1u << 22)  // a finished wave's polls for the block's posted drain rays, at most (mb_slot)
#define RTW_LDS_SCENE_MAX (160 * 1024)  // LDS bytes per block the scene (+ stack) may take
#endif

namespace {

// ---------------------------------------------------------------------------------------------
// device data
// ---------------------------------------------------------------------------------------------
struct DWorld {
    const float4* node_a;  // {min.x, min.y, min.z, max.x}
    const float4* node_b;  // {max.y, max.z, bits(left << 2 | axis), bits(right)}
    const float2* node_km; // proximity-cull constants {k, m} (rtw_cull.h)
    const int4* leaf_info; // {geom_kind, geom_index, material, flags}
    const float4* leaf_fast; // plain sphere: {center.xyz, radius}; else w = NaN, x = a tag (1 plain triangle, 2 plain
                             // rect, 3 animated plain sphere, 0 other) and y = the primitive's index
    const float4* leaf_xf; // 3 per leaf: {neg_inv_density, off.xyz}, {ys, yc, vel.x, vel.y}, {vel.z,0,0,0}
    const float4* spheres; // {center.xyz, radius}
    const float4* rects;   // 2 per rect: {dist, r0.0, r0.1, r1.0}, {r1.1, bits(plane), 0, 0}
    const float4* boxes;   // 2 per box: {min.xyz, max.x}, {max.y, max.z, 0, 0}
    const float4* tri_fast; // 4 per tri: ray-independent part of the test (TriFast)
    const float4* tri_attr; // 4 per tri: normals and uvs packed
    const int4* materials; // {kind, texture, bits(fuzz), bits(ior)}
    const int4* textures;  // 3 per texture
    const int4* images;    // {texel offset, width, height, 0}
    const uint32_t* texels; // RGBA8, row 0 = top
    const float* perlin_ranvec; // 768 floats per perlin
    const uint32_t* perlin_perm; // 768 per perlin (x, y, z)
    const int* perlin_bits;
    const struct WorldConst* wc; // camera / light / background, read from memory when used
    // the kernel's own search tree (rtw_sah.cpp; node format of node_a / node_b) and each leaf's
    // proof box, its parent node's box in the reference tree (2 per leaf: {min.xyz, max.x},
    // {max.y, max.z, 0, 0}), for the verification (§5.5)
    // the SAH tree: node_b as the reference tree's, cull constants in sah_km -- except in plain-sphere
    // worlds (the two-children walk), whose node_b is {max.y, max.z, bits(children), m} (sah_left /
    // sah_right) with the cull constants {sah_k, m}: the world's k, the node's m, and no sah_km
    const float4* sah_a;
    const float4* sah_b;
    const float2* sah_km;
    const float4* leaf_box;
    // each leaf's place in the reference tree's DFS (coop_solve's tie resolution): {side bits, and
    // per axis the bits of the ancestors splitting on it}, bit 31 - k for the ancestor at depth k;
    // null when the reference tree is deeper than 32
    const uint4* leaf_key;
    int32_t sah_root;
    int32_t sah_root_c2;  // the SAH root's packed children word (the two-children walk's lane state)
    int32_t root;
    int32_t has_light;
    float sah_k;  // plain-sphere worlds' SAH tree: the largest finite node k (nodes of infinite k carry m = inf)
};

// Rarely-read scalars live in HBM (scalar-cache loads at their use sites) instead of kernel
// arguments, so they do not pin SGPRs across the bounce loop.
struct WorldConst {
    rtw_camera cam;
    rtw_rect light;
    rtw_background bg;
};

// On-device tuning of the dynamic-fetch threshold, kept per world.  A launch that finds chosen == 0
// and has room for it explores candidates over epochs of `tune_items` work items -- whole passes
// over the launch's pixel slots, so every epoch renders the same pixels (other samples) and epoch
// times compare like for like.  Epoch 0 warms up; epoch e = 1..EPOCHS runs candidate
// cand[e-1] (mirrored, a..h h..a).  Only the second half of an epoch is timed: a switch of
// threshold shifts how many lanes sit finished-but-unshaded, and that transient would bias the
// first half (against low thresholds after high ones).  The wave whose refill hands out the first
// item of a half-epoch records the 100 MHz clock.  Once the last epoch has ended every wave derives
// the same winner (least timed half-epoch time over its two epochs) and publishes it for the
// world's later launches.
#define RTW_TUNE_NCAND 8
#define RTW_TUNE_EPOCHS (2 * RTW_TUNE_NCAND)
#define RTW_TUNE_STAMPS (2 * RTW_TUNE_EPOCHS + 2)
struct TuneState {
    unsigned long long tb[RTW_TUNE_STAMPS];  // clock when item (k + 1) * tune_items / 2 was handed out
    int chosen;                              // the world's threshold once decided (0: not yet)
};
__constant__ const int kTuneCand[RTW_TUNE_NCAND] = {6, 8, 12, 16, 24, 32, 40, 48};

// Division by a launch-invariant u32 (Granlund & Montgomery 1994, Thm 4.2, N = 32): with
// s = ceil(log2 d) and m = floor(2^32 (2^s - d) / d) + 1, q = (mulhi(n, m) + n) >> s for every
// n < 2^32 (the sum taken in 64 bits).  Replaces the work-item decode's integer divisions.
struct FastDiv {
    uint32_t d, m, s;
};
inline FastDiv fastdiv_make(uint32_t d) {
    uint32_t s = 0;
    while (s < 32 && (1ull << s) < d) ++s;
    const uint64_t m = (((1ull << s) - d) << 32) / d + 1;
    return FastDiv{d, (uint32_t)m, s};
}
__host__ __device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
#ifdef __HIP_DEVICE_COMPILE__
    const uint32_t t = __umulhi(n, f.m);
#else
    const uint32_t t = (uint32_t)(((uint64_t)n * f.m) >> 32);
#endif
    return (uint32_t)(((uint64_t)t + n) >> f.s);
}

struct KArgs {
    DWorld w;
    int32_t width, height;
    uint32_t spp;
    int32_t max_depth;
    int32_t mode;
    int32_t layout;
    int32_t tile_w, tile_h, tiles_x, n_tiles;
    int32_t part_index, part_count;
    int32_t thread_count;    // the reference's sample-split planes (accumulation only)
    uint32_t total;          // pixel slots in this partition (owned tiles * tile_w * tile_h)
    int32_t node_count, leaf_count, rect_count, tri_count;
    unsigned long long* queue; // work-item counter (zeroed before each launch)
    // one launch renders samples [s_begin, s_end) of every slot as work items of `chunk`
    // consecutive samples (item = chunk index * total + slot); each finished sample's colour goes
    // to colors[(sample - s_begin) * total + slot] and accumulate_kernel sums them in order
    uint32_t s_begin, s_end, chunk;
    // samples [s_split, s_end) are handed out one per item (after the chunked ones): a launch then
    // drains on single samples, not on whole chunks of the rare very long paths (paths trapped
    // inside a mesh take ~100x the mean)
    uint32_t s_split;
    uint64_t items_big;  // items of the chunked range
    uint64_t items;
    uint64_t q_cap;      // local items per queue: ceil(granules / RTW_QUEUES) * RTW_QGRAN
    float* colors;
    int32_t trace_min;       // dynamic ray fetch threshold (lanes still tracing), exit mode 0
    const DWorld* wdev;      // a copy of `w` in device memory (for the out-of-line shader)
    uint64_t seed_key;
    float sx, sy;            // 1/(W-1), 1/(H-1)
    rtw_uniform ux, uy;      // pixel jitter distributions
    float* out;
    unsigned long long* stats; // 13 counters (stats variant only)
    TuneState* tune;          // in-frame threshold tuning, or null
    int32_t mk_world;         // node coordinates admit the per-ray exact-division guard (ray_pre)
    int32_t stats_tree;       // counting variant: 0 the reference tree, 1 the tree the product kernel walks
    // shading tables in LDS (float4 offsets, -1: read from HBM / L2): leaf records, materials and, in
    // solid-texture worlds, each texture's first record; the stack follows them (stack_off)
    int32_t sh_li, sh_mat, sh_tex0, stack_off;
    int32_t sh_box;  // the leaves' proof boxes (2 float4 each) in LDS after the shading tables, -1: HBM / L2
    int32_t material_count, texture_count;
    int32_t fast_off;         // LDS float4 offset of leaf 0's record (leaf_fast; held from leaf tri_prefix on)
    int32_t sah;              // 1: hits are found on the SAH tree (node_count = its nodes), verified, and
                              // re-traced on the reference tree where the proof does not hold (§5.6)
    int32_t coop_max;         // drain: a wave with at most this many live lanes traces each ray with all
                              // 64 lanes over every leaf (coop_solve); 0: never
    int32_t coop_ties;        // 1: the walk's tied rays are resolved by coop_solve (else re-traced); 2: audit
    uint64_t tune_items;      // items per tuning epoch (0: this launch does not explore)
    // 1: a work item is a whole pixel (all spp samples of a slot, one lane, in sample order): the lane
    // sums the colours in registers -- the reference's sequential .sum(), rendering.rs:172-179 -- and
    // writes sum / spp to `out` itself; no colour buffer, no accumulation kernel (thread_count 1)
    int32_t whole_pixel;
    // work order by measured cost (render_frame): costlier tiles first, all their samples together
    const uint32_t* tile_perm;  // tile rank -> local tile, null: chunk-major order
    uint32_t* slot_cost;        // per slot: bounces of the deep (> 3 bounce) paths rendered there
    uint32_t chunks;            // chunks per slot in this launch (tile_perm order)
    uint64_t big_from;          // items from here on are reserved RTW_WAVE_BATCH_BIG at a time
    // work-item decode (items < 2^32 per launch, render_frame): divisors as FastDiv
    FastDiv fd_total, fd_rank, fd_tile, fd_tiles_x, fd_tile_w;
    // the refill's batch divisor (RTW_BATCH_SPREAD x waves) and the tuner's epoch / half-epoch:
    // 64-bit divisions there expanded to ~140 instructions each
    FastDiv fd_spread, fd_epoch, fd_half;
    // (last: fields read only by some kernel variants; ahead of the others they shifted the argument
    // layout into more SGPR spills)
    // the generic leaf path's tables in LDS (float4 offsets, -1: HBM / L2; render_kernel's GEN): leaf_xf
    // (3 per leaf), spheres, boxes (2 per box); and the rects of the LDS scene
    int32_t sh_xf, sh_sph, sh_bx, sh_rect;
    int32_t sphere_count, box_count;
    // the drain's shared cooperative trace (mb_slot): the block's mailbox words in LDS (float4 offset,
    // -1: each wave traces its own drained rays), and the rays one wave's stack columns hold
    int32_t mb_off, mb_cap;
    // leaves [0, tri_prefix) are plain triangles with triangle index = leaf index (walk_leaf_record; 0: none), and
    // the LDS triangle records' component stride (LDS mode 2: the triangle count)
    int32_t tri_prefix, tri_stride;
    int32_t tri_prefix_mat, tri_prefix_w;  // the prefix leaves' material and leaf_info.w (ShadeTabsT PRE)
};

// ---------------------------------------------------------------------------------------------
// f32 vector algebra (vec3.rs), evaluated exactly as written in the reference
// ---------------------------------------------------------------------------------------------
struct V3 {
    float x, y, z;
};
__host__ __device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__host__ __device__ __forceinline__ V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__host__ __device__ __forceinline__ V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
__host__ __device__ __forceinline__ V3 mul(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 divs(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ V3 conv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__host__ __device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__host__ __device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__host__ __device__ __forceinline__ float len(V3 a) { return __builtin_sqrtf(dot(a, a)); }
__host__ __device__ __forceinline__ V3 unit(V3 a) { return mul(a, 1.0f / len(a)); }  // vec3.rs:205-210
// ---------------------------------------------------------------------------------------------
// Exact divisions without the IEEE division sequence.  The compiler's correctly
// rounded a / b is 11 VALU instructions (v_div_scale x2, v_rcp, 5 fma, v_div_fmas, v_div_fixup);
// these give the same bits in 3 or 4 where a correctly rounded reciprocal is at hand.
// rcp_nr(b): the hardware reciprocal (within 1 ulp) and one fma Newton step.  It equals IEEE 1 / b
// for every f32 with 2^-100 <= |b| <= 2^100 (exhaustive on the device, rtw_device_check_division
// test 0, tests/test_gpu_division.py); callers guard that range.
#define RTW_RCP_LO 0x1p-100f
#define RTW_RCP_HI 0x1p100f
__device__ __forceinline__ float rcp_nr(float b) {
    const float y = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, y, 1.0f), y, y);
}
// RN(1 / b) for any b: the IEEE division outside rcp_nr's range (a rare, divergent branch)
__device__ __forceinline__ float rcp_x(float b) {
    float y = rcp_nr(b);
    const float ab = __builtin_fabsf(b);
    if (__builtin_expect(!(ab >= RTW_RCP_LO && ab <= RTW_RCP_HI), 0)) y = 1.0f / b;
    return y;
}
// Markstein's correction (Markstein 1990): with y = RN(1/b), q = RN(a y), r = fma(-b, q, a) is exact
// and RN(q + r y) = RN(a / b), provided 2^-22 <= |b| <= 2^22 and 2^-80 <= |a| <= 2^80 (no
// intermediate underflows; tests/native/markstein_check.c range 2).  A zero a gives q = RN(a y) =
// a / b exactly (the correction step could flip the sign of that zero, so it is not taken).
#define RTW_MKA_LO 0x1p-80f
#define RTW_MKA_HI 0x1p80f
#define RTW_MKB_LO 0x1p-22f
#define RTW_MKB_HI 0x1p22f
__device__ __forceinline__ float mk_corr(float a, float b, float y) {
    const float q = a * y;
    return __builtin_fmaf(__builtin_fmaf(-b, q, a), y, q);
}
__device__ __forceinline__ bool mk_a_ok(float a) {
    const float x = __builtin_fabsf(a);
    return x >= RTW_MKA_LO && x <= RTW_MKA_HI;
}
// RN(a / b) given y = RN(1 / b) with 2^-22 <= |b| <= 2^22 (the caller's guarantee)
__device__ __forceinline__ float div_y(float a, float b, float y) {
    float q = mk_corr(a, b, y);
    if (__builtin_expect(!mk_a_ok(a), 0)) q = a / b;
    return q;
}
// RN(a / b) for any a, b (IEEE where the guards fail)
__device__ __forceinline__ float div_x(float a, float b) {
    const float y = rcp_nr(b);
    float q = mk_corr(a, b, y);
    const float ab = __builtin_fabsf(b);
    if (__builtin_expect(!(mk_a_ok(a) && ab >= RTW_MKB_LO && ab <= RTW_MKB_HI), 0)) q = a / b;
    return q;
}
// a / s per component, y = RN(1 / s), 2^-22 <= |s| <= 2^22; one guard for the three dividends
__device__ __forceinline__ V3 divs_y(V3 a, float s, float y) {
    V3 q = v3(mk_corr(a.x, s, y), mk_corr(a.y, s, y), mk_corr(a.z, s, y));
    const float lo = __builtin_fminf(__builtin_fminf(__builtin_fabsf(a.x), __builtin_fabsf(a.y)), __builtin_fabsf(a.z));
    const float hi = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(a.x), __builtin_fabsf(a.y)), __builtin_fabsf(a.z));
    if (__builtin_expect(!(lo >= RTW_MKA_LO && hi <= RTW_MKA_HI), 0)) q = divs(a, s);
    return q;
}
__device__ __forceinline__ V3 divs_x(V3 a, float s) {
    const float as = __builtin_fabsf(s);
    if (__builtin_expect(!(as >= RTW_MKB_LO && as <= RTW_MKB_HI), 0)) return divs(a, s);
    return divs_y(a, s, rcp_nr(s));
}
// Correctly rounded sqrt without the compiler's range handling: v_sqrt_f32 and the +-1 ulp
// correction by two fma residuals, the compiler's own sequence minus the scaling of inputs below
// 2^-96 and the zero / inf select.  Equal to sqrtf on every f32 in [2^-96, FLT_MAX] (exhaustive on
// the device, rtw_device_check_division test 4).  sqrt_nr: the caller knows the range; sqrt_x: any x.
#define RTW_SQRT_LO 0x1p-96f
__device__ __forceinline__ float sqrt_nr(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __int_as_float(__float_as_int(s) - 1), sp = __int_as_float(__float_as_int(s) + 1);
    const float rm = __builtin_fmaf(-sm, s, x), rp = __builtin_fmaf(-sp, s, x);
    float r = rm <= 0.0f ? sm : s;
    r = rp > 0.0f ? sp : r;
    return r;
}
__device__ __forceinline__ float sqrt_x(float x) {
    float r = sqrt_nr(x);
    if (__builtin_expect(!(x >= RTW_SQRT_LO && x <= 0x1.fffffep127f), 0)) r = __builtin_sqrtf(x);
    return r;
}
// Vec3::unit (vec3.rs:205-210): v * (1 / len)
__device__ __forceinline__ V3 unit_x(V3 a) { return mul(a, rcp_x(sqrt_x(dot(a, a)))); }
// a / c for a positive constant c with yc = RN(1 / c) (constant-folded), 2^-22 <= c <= 2^22: a zero
// a keeps its sign through q = a yc
__device__ __forceinline__ float div_c(float a, float c, float yc) {
    const float q = a * yc;
    float r = __builtin_fmaf(__builtin_fmaf(-c, q, a), yc, q);
    r = a == 0.0f ? q : r;
    if (__builtin_expect(!(a == 0.0f || mk_a_ok(a)), 0)) r = a / c;
    return r;
}
// An image texel's channel, byte / 255.0 (texture.rs:30-31, `rgb8 as f32 / 255.0`): Markstein's
// correction with RN(1/255) is exact for every dividend 1..255 (inside the guards), and 0 gives q = 0
// exactly with r = 0: no guard and no branch (rtw_device_check_division test 6: all 256 bytes).
// Three operations instead of the IEEE division's eleven, three times per texel.
__device__ __forceinline__ float tex255(uint32_t byte) {
    const float a = (float)byte, y = 1.0f / 255.0f;
    const float q = a * y;
    return __builtin_fmaf(__builtin_fmaf(-255.0f, q, a), y, q);
}
__device__ __forceinline__ float comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
__device__ __forceinline__ void setc(V3& a, int i, float v) {
    if (i == 0) a.x = v;
    else if (i == 1) a.y = v;
    else a.z = v;
}
__device__ __forceinline__ V3 ld3(const float* p) { return v3(p[0], p[1], p[2]); }
__device__ __forceinline__ V3 reflect(V3 d, V3 n) { return sub(d, mul(n, 2.0f * dot(d, n))); }  // vec3.rs:232
__device__ __forceinline__ V3 refract(V3 d, V3 n, float eta) {  // vec3.rs:235-240
    const float cos_theta = rtw_minr(dot(neg(d), n), 1.0f);
    const V3 perp = mul(add(d, mul(n, cos_theta)), eta);
    const float k = -sqrt_x(__builtin_fabsf(1.0f - dot(perp, perp)));
    return add(perp, mul(n, k));
}

#define F32_PI 3.14159274101257324219f
#define F32_TAU 6.28318548202514648438f
#define F32_INF (__builtin_inff())

// The RNG draws of the path (rtw_scalar.h: rand_xoshiro 0.6's Xoroshiro128PlusPlus, rand 0.8.5's
// UniformFloat, rand_distr 0.4.3's UnitDisc / UnitSphere / UnitBall), written for gfx950: the same
// values with fewer instructions.  A wave runs a rejection loop as many rounds as its unluckiest lane
// needs, so each draw's cost is paid several times over.
// * a 64-bit rotation by a constant is two v_alignbit_b32 (the compiler's 64-bit shifts and an or: 3);
// * rand's [0, 1) float (u >> 9 | bits(1.0f)) - 1 takes its or from the alignbit's high word:
//   alignbit(0x7F, u, 9) = u >> 9 | 0x7F << 23; and UnitDisc / UnitSphere / UnitBall's
//   Uniform(-1, 1) sample v * 2 + (-1) is bits(u >> 9 | 0x40000000) - 3 = 2 (1 + m) - 3, one
//   subtraction: both are 2 m - 1 exactly (m = (u >> 9) 2^-23; 2 m - 1 is a multiple of 2^-23 in
//   [-1, 1), so neither form rounds);
// * UnitSphere's sqrt(1 - sum) is sqrt_nr: 2^-24 <= 1 - sum <= 1 (sum is a float below 1).
// Every image test draws through these (parity suite: all samplers, all worlds).
__device__ __forceinline__ uint64_t d_rotl64(uint64_t x, int k) {  // k: a constant in 1..63, not 32
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    uint32_t nlo, nhi;
    if (k < 32) {
        nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - k);
        nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - k);
    } else {
        nhi = __builtin_amdgcn_alignbit(lo, hi, 64 - k);
        nlo = __builtin_amdgcn_alignbit(hi, lo, 64 - k);
    }
    return ((uint64_t)nhi << 32) | nlo;
}
// (Against drawing through rtw_scalar.h's functions: final_scene1 +2.8 %, profiles/r04/v8_device_rng_ab.txt.)
__device__ __forceinline__ uint64_t d_next_u64(rtw_xoro* r) {  // rtw_xoro_next_u64
    const uint64_t s0 = r->s0;
    uint64_t s1 = r->s1;
    const uint64_t result = d_rotl64(s0 + s1, 17) + s0;
    s1 ^= s0;
    r->s0 = d_rotl64(s0, 49) ^ s1 ^ (s1 << 21);
    r->s1 = d_rotl64(s1, 28);
    return result;
}
__device__ __forceinline__ uint32_t d_next_u32(rtw_xoro* r) { return (uint32_t)d_next_u64(r); }
__device__ __forceinline__ float d_value0_1(uint32_t u) {
    return __uint_as_float(__builtin_amdgcn_alignbit(0x7Fu, u, 9)) - 1.0f;
}
__device__ __forceinline__ float d_m1_1(rtw_xoro* r) {  // rtw_uniform_m1_1
    return __uint_as_float(__builtin_amdgcn_alignbit(0x80u, d_next_u32(r), 9)) - 3.0f;
}
__device__ __forceinline__ float d_gen_f32(rtw_xoro* r) {  // rtw_gen_f32
    return (1.0f / 16777216.0f) * (float)(d_next_u32(r) >> 8);
}
__device__ __forceinline__ bool d_gen_bool_half(rtw_xoro* r) { return d_next_u64(r) < 0x8000000000000000ull; }
__device__ __forceinline__ float d_uniform_sample(const rtw_uniform& u, rtw_xoro* r) {  // rtw_uniform_sample
    return d_value0_1(d_next_u32(r)) * u.scale + u.low;
}
__device__ __forceinline__ float d_gen_range_f32(float low, float high, rtw_xoro* r) {  // rtw_gen_range_f32
    const float scale = high - low;
    for (;;) {
        const float res = d_value0_1(d_next_u32(r)) * scale + low;
        if (res < high) return res;
    }
}
__device__ __forceinline__ void d_unit_disc(rtw_xoro* r, float& x1, float& x2) {  // rtw_unit_disc
    for (;;) {
        x1 = d_m1_1(r);
        x2 = d_m1_1(r);
        if (x1 * x1 + x2 * x2 <= 1.0f) break;
    }
}
__device__ __forceinline__ V3 d_unit_sphere(rtw_xoro* r) {  // rtw_unit_sphere
    float x1, x2, sum;
    for (;;) {
        x1 = d_m1_1(r);
        x2 = d_m1_1(r);
        sum = x1 * x1 + x2 * x2;
        if (sum < 1.0f) break;
    }
    const float factor = 2.0f * sqrt_nr(1.0f - sum);
    return v3(x1 * factor, x2 * factor, 1.0f - 2.0f * sum);
}
__device__ __forceinline__ V3 d_unit_ball(rtw_xoro* r) {  // rtw_unit_ball
    float x1, x2, x3;
    for (;;) {
        x1 = d_m1_1(r);
        x2 = d_m1_1(r);
        x3 = d_m1_1(r);
        if (x1 * x1 + x2 * x2 + x3 * x3 <= 1.0f) break;
    }
    return v3(x1, x2, x3);
}

// Out-of-line wrappers: the f64 polynomial constants need SGPR pairs (no VOP3 literals on
// gfx9); inlined into the bounce loop they get hoisted and pin ~100 SGPRs.
// The sphere uv's acosf / atan2f (vec3.rs:242-243; rtw_scalar.h's restatements of glibc's fdlibm code,
// the specification) with each IEEE division and square root replaced by div_x / sqrt_x: the same bits
// (both exact, with the IEEE operation where their guards fail), the compiler's 11-instruction division
// sequence and range-checked sqrt gone from every sphere-uv hit (earth_motion's shading).  Checked
// against the host restatements by eval_scalar_kernel (tests/test_gpu_scalar.py).
__device__ __forceinline__ float d_atanf_x(float x) {
    const float atanhi[4] = {__uint_as_float(0x3eed6338u), __uint_as_float(0x3f490fdau), __uint_as_float(0x3f7b985eu),
                             __uint_as_float(0x3fc90fdau)};
    const float atanlo[4] = {__uint_as_float(0x31ac3769u), __uint_as_float(0x33222168u), __uint_as_float(0x33140fb4u),
                             __uint_as_float(0x33a22168u)};
    const float aT0 = __uint_as_float(0x3eaaaaabu), aT1 = __uint_as_float(0xbe4ccccdu), aT2 = __uint_as_float(0x3e124925u),
                aT3 = __uint_as_float(0xbde38e38u), aT4 = __uint_as_float(0x3dba2e6eu), aT5 = __uint_as_float(0xbd9d8795u),
                aT6 = __uint_as_float(0x3d886b35u), aT7 = __uint_as_float(0xbd6ef16bu), aT8 = __uint_as_float(0x3d4bda59u),
                aT9 = __uint_as_float(0xbd15a221u), aT10 = __uint_as_float(0x3c8569d7u);
    const int32_t hx = __float_as_int(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {
        if (ix < 0x31000000) return x;
        id = -1;
    } else {
        x = __builtin_fabsf(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) {
                id = 0;
                x = div_x(2.0f * x - 1.0f, 2.0f + x);
            } else {
                id = 1;
                x = div_x(x - 1.0f, x + 1.0f);
            }
        } else if (ix < 0x401c0000) {
            id = 2;
            x = div_x(x - 1.5f, 1.0f + 1.5f * x);
        } else {
            id = 3;
            x = div_x(-1.0f, x);
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}
// The sphere uv functions (fdlibm restatements with the exact fast division): inlined into the GEN kernels (the
// image texture and moving spheres of C5: with calls their texture loop spilled VGPRs to scratch; inlined,
// earth_motion +1.9 %, 0 scratch, profiles/r06/ab_c5_spills.txt), called out of line elsewhere (inlined into
// the non-GEN textured kernels: perlin_spheres -3.6 %)
__device__ __forceinline__ float d_acosf_inl(float x) {
    const float pi = __uint_as_float(0x40490fdau), pio2_hi = __uint_as_float(0x3fc90fdau), pio2_lo = __uint_as_float(0x33a22168u);
    const float pS0 = __uint_as_float(0x3e2aaaabu), pS1 = __uint_as_float(0xbea6b090u), pS2 = __uint_as_float(0x3e4e0aa8u),
                pS3 = __uint_as_float(0xbd241146u), pS4 = __uint_as_float(0x3a4f7f04u), pS5 = __uint_as_float(0x3811ef08u);
    const float qS1 = __uint_as_float(0xc019d139u), qS2 = __uint_as_float(0x4001572du), qS3 = __uint_as_float(0xbf303361u),
                qS4 = __uint_as_float(0x3d9dc62eu);
    const int32_t hx = __float_as_int(x);
    const int32_t ix = hx & 0x7fffffff;
    if (ix == 0x3f800000) return hx > 0 ? 0.0f : pi + __uint_as_float(0x34222168u);
    if (ix > 0x3f800000) return (x - x) / (x - x);
    if (ix < 0x3f000000) {
        if (ix <= 0x32800000) return pio2_hi + pio2_lo;
        const float z = x * x;
        const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        return pio2_hi - (x - (pio2_lo - x * div_x(p, q)));
    }
    const float z = (hx < 0 ? 1.0f + x : 1.0f - x) * 0.5f;
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float s = sqrt_x(z);
    const float r = div_x(p, q);
    if (hx < 0) return pi - 2.0f * (s + (r * s - pio2_lo));
    const float df = __uint_as_float(__float_as_uint(s) & 0xfffff000u);
    const float c = div_x(z - df * df, s + df);
    return 2.0f * (df + (r * s + c));
}
__device__ __forceinline__ float d_atan2f_inl(float y, float x) {
    const float tiny = __uint_as_float(0x0da24260u);
    const float pi_o_4 = __uint_as_float(0x3f490fdbu), pi_o_2 = __uint_as_float(0x3fc90fdbu), pi = __uint_as_float(0x40490fdbu),
                pi_lo = __uint_as_float(0xb3bbbd2eu);
    const int32_t hx = __float_as_int(x), hy = __float_as_int(y);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return d_atanf_x(y);
    const int m = (int)(((uint32_t)hy >> 31) & 1u) | (int)(((uint32_t)hx >> 30) & 2u);
    if (iy == 0) return m <= 1 ? y : m == 2 ? pi + tiny : -pi - tiny;
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000)
            return m == 0 ? pi_o_4 + tiny : m == 1 ? -pi_o_4 - tiny : m == 2 ? 3.0f * pi_o_4 + tiny : -3.0f * pi_o_4 - tiny;
        return m == 0 ? 0.0f : m == 1 ? -0.0f : m == 2 ? pi + tiny : -pi - tiny;
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else z = d_atanf_x(__builtin_fabsf(div_x(y, x)));
    switch (m) {
        case 0: return z;
        case 1: return __uint_as_float(__float_as_uint(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}
__device__ __noinline__ float d_acosf(float x) { return d_acosf_inl(x); }
__device__ __noinline__ float d_atan2f(float y, float x) { return d_atan2f_inl(y, x); }
__device__ __noinline__ float d_logf(float x) { return rtw_logf(x); }
__device__ __noinline__ float d_sinf(float x) { return rtw_sinf(x); }

// CheckerTexture's test (texture.rs:33-40): is RN(RN(sinf(x) * sinf(y)) * sinf(z)) < 0?  Only the
// sign of the product is read: when rtw_sin_sign_fast decides all three sines' signs (rtw_scalar.h,
// pinned against glibc's sinf for every f32), the product is negative iff an odd number of them
// are.  Other arguments (0, huge, NaN, near a multiple of pi/2) evaluate the sines.
// the slow path: the three sines inlined in one leaf call (three calls to d_sinf from here kept x, y, z
// and the product live across calls: 16 B of scratch per lane in every texture variant)
__device__ __noinline__ bool d_sin3_negative(float x, float y, float z) {
    return rtw_sinf(x) * rtw_sinf(y) * rtw_sinf(z) < 0.0f;
}
__device__ __forceinline__ bool d_checker_odd(float x, float y, float z) {
    int nx = 0, ny = 0, nz = 0;
    const bool fast = rtw_sin_sign_fast(x, &nx) & rtw_sin_sign_fast(y, &ny) & rtw_sin_sign_fast(z, &nz);
    if (__builtin_expect(fast, 1)) return ((nx != 0) ^ (ny != 0) ^ (nz != 0)) != 0;
    return d_sin3_negative(x, y, z);
}

struct Ray {
    V3 o, d;
    float time;
};
__device__ __forceinline__ V3 at(const Ray& r, float t) { return add(r.o, mul(r.d, t)); }
__device__ __forceinline__ bool contains(float s, float e, float t) { return s <= t && t < e; }

// ---------------------------------------------------------------------------------------------
// statistics (stats variant only)
// ---------------------------------------------------------------------------------------------
enum {
    ST_SAMPLES, ST_RAYS, ST_NODES, ST_T_SPHERE, ST_T_RECT, ST_T_BOX, ST_T_TRI,
    ST_H_SPHERE, ST_H_RECT, ST_H_BOX, ST_H_TRI, ST_MAT, ST_TEXEL, ST_COUNT
};
// wave-level execution counters of the counting variant (rtw_render_debug_counters), stored
// after the ST_COUNT statistics: traversal calls / loop iterations / iterations that ran the node
// resp. leaf path / lanes stepping a node resp. a leaf / shade calls / lanes shading
enum { DB_TRAV_CALLS, DB_ITERS, DB_NODE_ITERS, DB_LEAF_ITERS, DB_NODE_LANES, DB_LEAF_LANES, DB_ALIVE_LANES,
       DB_WAIT_LANES, DB_PASS_LANES, DB_SN_ITERS, DB_SN_LANES, DB_SF_ITERS, DB_SF_LANES, DB_SHADE_CALLS,
       DB_SHADE_LANES, DB_TRAV_CYCLES, DB_REST_CYCLES, DB_COUNT };
struct Stats {
    uint32_t c[ST_COUNT];
};

// Where shading and the generic leaf path read their records: LDS float4 offsets (-1: HBM / L2).
// The chain leaf record -> material -> texture is a run of dependent loads per shaded ray, so the
// tables sit in LDS whenever they fit (launch_render), and a plain sphere's geometry comes from
// its leaf_fast copy (`fast`, also in LDS).  The generic leaf path (Transformation / Animation /
// volume leaves, boxes) reads the leaf record, its transform or velocity and then the primitive: a
// chain of three dependent loads per leaf test, from LDS too when they fit (round 5: earth_motion's
// two moving spheres, C5, waited on those global loads).
// Whether the generic tables (xf, sph, bx) and the rects are in LDS is a compile-time property of the
// kernel variant (GEN: render_kernel's template parameter, RECT: the LDS scene of a world with rect
// leaves): as runtime choices their loads became pointer selects and flat loads, and their offsets
// occupied SGPRs across the bounce loop (suzanne -3 % from the spills).
extern __shared__ __attribute__((aligned(16))) float4 smem[];
// PRE (the LK_TRIS kernels): leaves [0, pre) are the triangle prefix (walk_leaf_record), whose leaf_info
// is made up from the prefix's one material and flags word -- the LDS table holds the other leaves only
template <bool GEN, bool RECT, bool PRE = false>
struct ShadeTabsT {
    int32_t li, mat, tex0, fast;
    int32_t xf, sph, bx, rect;  // leaf_xf, spheres, boxes (GEN), rects (RECT)
    int32_t pre, pre_mat, pre_w;  // PRE: the prefix's length, material and leaf_info.w
    static constexpr bool gen = GEN, rect_lds = RECT, prefix = PRE;
};
using ShadeTabs = ShadeTabsT<false, false>;  // the tables of the device self-test kernels
__device__ __forceinline__ int4 lds_i4(int32_t i) { return reinterpret_cast<const int4*>(smem)[i]; }
template <class TB>
__device__ __forceinline__ float4 tab_gen(const TB& S, int32_t off, const float4* __restrict__ g, int i) {
    (void)S;
    if constexpr (TB::gen) return smem[off + i];
    else return g[i];
}
template <class TB>
__device__ __forceinline__ int4 leaf_info_of(const DWorld& w, const TB& S, int leaf) {
    if constexpr (TB::prefix)
        if (leaf < S.pre) return make_int4(RTW_GEOM_TRIANGLE, leaf, S.pre_mat, S.pre_w);
    int4 v;
    if (S.li >= 0) v = lds_i4(S.li + leaf);
    else v = w.leaf_info[leaf];
    return v;
}

// ---------------------------------------------------------------------------------------------
// primitives: candidate tests return t only
// ---------------------------------------------------------------------------------------------
// sphere_geometry.rs:21-41
__device__ __forceinline__ bool sphere_t(float4 s, const Ray& r, float ts, float te, float& t) {
    const V3 oc = sub(r.o, v3(s.x, s.y, s.z));
    const float half_b = dot(oc, r.d);
    const float c = dot(oc, oc) - s.w * s.w;
    const float disc = half_b * half_b - c;
    if (disc < 0.0f) return false;
    const float sq = sqrt_x(disc);
    const float small = -half_b - sq;
    if (contains(ts, te, small)) {
        t = small;
        return true;
    }
    const float large = -half_b + sq;
    if (contains(ts, te, large)) {
        t = large;
        return true;
    }
    return false;
}

__device__ __forceinline__ void rect_axes(int plane, int& p0, int& p1, int& n) {
    p0 = (plane == RTW_PLANE_YZ) ? 1 : 0;
    p1 = (plane == RTW_PLANE_XY) ? 1 : 2;
    n = (plane == RTW_PLANE_XY) ? 2 : ((plane == RTW_PLANE_XZ) ? 1 : 0);
}
struct RectG {
    int plane;
    float dist, r00, r01, r10, r11;
};
template <class TB>
__device__ __forceinline__ RectG load_rect(const DWorld& w, const TB& S, int i) {
    float4 a, b;
    if constexpr (TB::rect_lds) {
        a = smem[S.rect + 2 * i];
        b = smem[S.rect + 2 * i + 1];
    } else {
        a = w.rects[2 * i];
        b = w.rects[2 * i + 1];
    }
    return RectG{__float_as_int(b.y), a.x, a.y, a.z, a.w, b.x};
}
// rect_geometry.rs:33-46 (hit test part)
__device__ __forceinline__ bool rect_t(const RectG& g, const Ray& r, float ts, float te, float& t, V3& pos) {
    int p0, p1, n;
    rect_axes(g.plane, p0, p1, n);
    t = (g.dist - comp(r.o, n)) / comp(r.d, n);
    if (!contains(ts, te, t)) return false;
    pos = add(r.o, mul(r.d, t));
    const float a = comp(pos, p0), b = comp(pos, p1);
    return a >= g.r00 && a <= g.r01 && b >= g.r10 && b <= g.r11;
}

// the same for a Markstein-exact ray (RayPre::fast, §5.1) with y = RN(1 / d): every rect's dist
// admits the guard like a node coordinate (mk_world), so t = RN((dist - o_n) / d_n) exactly; a zero
// quotient may carry the other sign, and t = +-0 < ts = 0.001 is rejected either way
__device__ __forceinline__ bool rect_t_mk(const RectG& g, const Ray& r, V3 inv, float ts, float te, float& t) {
    int p0, p1, n;
    rect_axes(g.plane, p0, p1, n);
    t = mk_corr(g.dist - comp(r.o, n), comp(r.d, n), comp(inv, n));
    if (!contains(ts, te, t)) return false;
    const V3 pos = add(r.o, mul(r.d, t));
    const float a = comp(pos, p0), b = comp(pos, p1);
    return a >= g.r00 && a <= g.r01 && b >= g.r10 && b <= g.r11;
}

// aabb.rs:103-167
__device__ __forceinline__ bool box_line(float4 ba, float4 bb, const Ray& r, float& nt, int& np, float& ft, int& fp) {
    const V3 mn = sub(v3(ba.x, ba.y, ba.z), r.o);
    const V3 mx = sub(v3(ba.w, bb.x, bb.y), r.o);
    float near = -F32_INF, far = F32_INF;
    np = 0;
    fp = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float t1 = comp(mn, a) / comp(r.d, a);
        const float t2 = comp(mx, a) / comp(r.d, a);
        const float tmin = rtw_minr(t1, t2);
        const float tmax = rtw_maxr(t1, t2);
        if (tmin > near) {
            near = tmin;
            np = a;
        }
        if (tmax < far) {
            far = tmax;
            fp = a;
        }
        if (near > far || far < 0.0f) return false;
    }
    nt = near;
    ft = far;
    return true;
}
template <class TB>
__device__ __forceinline__ bool box_t(const DWorld& w, const TB& S, int i, const Ray& r, float ts, float te,
                                      float& t) {
    float nt, ft;
    int np, fp;
    if (!box_line(tab_gen(S, S.bx, w.boxes, 2 * i), tab_gen(S, S.bx, w.boxes, 2 * i + 1), r, nt, np, ft, fp)) return false;
    if (contains(ts, te, nt)) {
        t = nt;
        return true;
    }
    if (contains(ts, te, ft)) {
        t = ft;
        return true;
    }
    return false;
}

// triangle_geometry.rs:13-45.  Everything that does not depend on the ray -- the edges, the
// unit normal, the two barycentric axes and their denominators -- is computed once at upload with
// the same f32 operations in the same order (host and device share these helpers; both are
// IEEE f32 without contraction), so the values are bit-identical to the reference's per-test ones.
struct TriFast {
    V3 p0, n, vt1, vt2;
    float den1, den2;
    float y1, y2;  // RN(1 / den) when 2^-22 <= |den| <= 2^22, else 0 (div_tri then divides)
};
__host__ __device__ __forceinline__ TriFast tri_prepare(V3 p0, V3 p1, V3 p2) {
    TriFast f;
    const V3 dir1 = sub(p1, p0);
    const V3 dir2 = sub(p2, p0);
    f.p0 = p0;
    f.n = unit(cross(dir1, dir2));
    f.vt1 = cross(f.n, dir2);
    f.den1 = dot(dir1, f.vt1);
    f.vt2 = cross(f.n, dir1);
    f.den2 = dot(dir2, f.vt2);
    auto recip = [](float d) {
        const float a = d < 0.0f ? -d : d;
        return (a >= 0x1p-22f && a <= 0x1p22f) ? 1.0f / d : 0.0f;
    };
    f.y1 = recip(f.den1);
    f.y2 = recip(f.den2);
    return f;
}
// 4 float4 per triangle: {p0.xyz, n.x} {n.yz, vt1.xy} {vt1.z, den1, vt2.xy} {vt2.z, den2, y1, y2}
__device__ __forceinline__ TriFast load_tri(const float4* __restrict__ tf, int i) {
    const float4 a = tf[4 * i], b = tf[4 * i + 1], c = tf[4 * i + 2], d = tf[4 * i + 3];
    TriFast f;
    f.p0 = v3(a.x, a.y, a.z);
    f.n = v3(a.w, b.x, b.y);
    f.vt1 = v3(b.z, b.w, c.x);
    f.den1 = c.y;
    f.vt2 = v3(c.z, c.w, d.x);
    f.den2 = d.y;
    f.y1 = d.z;
    f.y2 = d.w;
    return f;
}
// LDS mode 2 keeps the records component-major: component k of triangle i at tf[k * stride + i]: a
// 16-lane group's reads of one component spread over all 16 slots of the 256-B bank row instead of the 4
// that 64-B records start on (4-way conflicts: suzanne's 2.8 conflict cycles per LDS instruction in round
// 2).  The stride: RTW_TRI_SOA records, a compile-time constant whose four reads share one address register
// (offsets 0, 16, 32, 48 KB in the ds_read_b128 immediate) -- except in the triangle-and-sphere kernels
// (LK_TRIS), whose stride is the world's triangle count (KArgs::tri_stride): three adds per test, and the
// 3.5 KB that let suzanne's split tree take mode 2.  (The runtime stride in every kernel cost
// cornell_cube 2 %, profiles/r06/ab_mode2_suzanne.txt.)
#ifndef RTW_TRI_SOA
#define RTW_TRI_SOA 1024
#endif
// (Indexing them by leaf instead, and loading a leaf's record with its leaf record before knowing it is a
// triangle -- one dependent LDS read less per triangle test -- lost 1.8 % on suzanne: the early record's
// 16 VGPRs; profiles/r04/v5_experiments_ab.txt.)
__device__ __forceinline__ TriFast load_tri_soa(const float4* __restrict__ tf, int i, int32_t stride) {
    const float4 a = tf[i], b = tf[stride + i], c = tf[2 * stride + i], d = tf[3 * stride + i];
    TriFast f;
    f.p0 = v3(a.x, a.y, a.z);
    f.n = v3(a.w, b.x, b.y);
    f.vt1 = v3(b.z, b.w, c.x);
    f.den1 = c.y;
    f.vt2 = v3(c.z, c.w, d.x);
    f.den2 = d.y;
    f.y1 = d.z;
    f.y2 = d.w;
    return f;
}
// a barycentric quotient a / den with the record's y = RN(1 / den) (0: den out of range)
__device__ __forceinline__ float div_tri(float a, float den, float y) {
    float q = mk_corr(a, den, y);
    if (__builtin_expect(!(mk_a_ok(a) && y != 0.0f), 0)) q = a / den;
    return q;
}
// a wave-uniform pointer in scalar registers
template <class T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return (T*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}
// the per-ray part; barycentrics are recomputed from (ray, t) by leaf_record
// t = num / denom without the division sequence: with 1e-4 < |denom| <= |d||n| ~ 1 the
// divisor is inside Markstein's guard; a dividend outside its guard is 0 or below 2^-80
// (then both quotients lie below ts = 0.001: the test fails either way) -- the upper bound holds as
// coordinates are below 2^30.  So the quotient decides contains(ts, te, t) as RN(num / denom) does and
// equals it whenever that passes: no guard, no branch (rtw_device_check_division test 5).  Against the
// IEEE division: suzanne +1.4 %, cornell_cube +1.7 % (profiles/r04/v2_experiments_ab.txt).
__device__ __forceinline__ float tri_t_mk(float num, float denom) { return mk_corr(num, denom, rcp_nr(denom)); }
__device__ __forceinline__ bool tri_test(const TriFast& T, const Ray& r, float ts, float te, float& t) {
    const float denom = dot(r.d, T.n);
    if (!(__builtin_fabsf(denom) > 0.0001f)) return false;
    t = tri_t_mk(dot(sub(T.p0, r.o), T.n), denom);
    if (!contains(ts, te, t)) return false;
    const V3 q = sub(at(r, t), T.p0);
    const float w1 = div_tri(dot(q, T.vt1), T.den1, T.y1);
    if (!(w1 > 0.0f && w1 < 1.0f)) return false;
    const float w2 = div_tri(dot(q, T.vt2), T.den2, T.y2);
    const float w0 = 1.0f - w1 - w2;
    return w2 > 0.0f && w0 > 0.0f;
}

template <bool STATS, class TB>
__device__ __forceinline__ bool geom_t(const DWorld& w, const TB& S, int kind, int idx, const Ray& r, float ts,
                                       float te, float& t, Stats& st) {
    if (STATS) st.c[ST_T_SPHERE + kind]++;
    if (kind == RTW_GEOM_SPHERE) return sphere_t(tab_gen(S, S.sph, w.spheres, idx), r, ts, te, t);
    if (kind == RTW_GEOM_RECT) {
        V3 pos;
        return rect_t(load_rect(w, S, idx), r, ts, te, t, pos);
    }
    if (kind == RTW_GEOM_BOX) return box_t(w, S, idx, r, ts, te, t);
    return tri_test(load_tri(w.tri_fast, idx), r, ts, te, t);
}

// device-only leaf_info.w bit (above the RTW_LEAF_* flags): the leaf's material samples an image
// texture somewhere in its texture tree, so its hit record needs uv
#define RTW_DLEAF_UV (1u << 16)

// ---------------------------------------------------------------------------------------------
// leaf wrappers (hittable.rs:234-244, 271-292; transformations.rs:37-111)
// ---------------------------------------------------------------------------------------------
struct Xf {
    V3 off;
    float ys, yc;
};
__device__ __forceinline__ V3 rot_up(float c, float s, V3 v) {
    return v3(c * v.x + s * v.z, v.y, -s * v.x + c * v.z);
}
__device__ __forceinline__ Ray xf_reverse(const Xf& x, const Ray& r) {
    Ray o;
    o.o = rot_up(x.yc, -x.ys, sub(r.o, x.off));
    o.d = rot_up(x.yc, -x.ys, r.d);
    o.time = r.time;
    return o;
}
template <class TB>
__device__ __forceinline__ Xf anim_xf(const DWorld& w, const TB& S, int leaf, float time) {
    const float4 b = tab_gen(S, S.xf, w.leaf_xf, 3 * leaf + 1), c = tab_gen(S, S.xf, w.leaf_xf, 3 * leaf + 2);
    const V3 vt = mul(v3(b.z, b.w, c.x), time);
    return Xf{v3(0.0f + vt.x, 0.0f + vt.y, 0.0f + vt.z), 0.0f, 1.0f};
}
template <class TB>
__device__ __forceinline__ Xf leaf_xform(const DWorld& w, const TB& S, int leaf) {
    const float4 a = tab_gen(S, S.xf, w.leaf_xf, 3 * leaf), b = tab_gen(S, S.xf, w.leaf_xf, 3 * leaf + 1);
    return Xf{v3(a.y, a.z, a.w), b.x, b.y};
}
// the ray as seen by the leaf's primitive
template <class TB>
__device__ __forceinline__ Ray leaf_local_ray(const DWorld& w, const TB& S, int leaf, uint32_t flags,
                                              const Ray& r) {
    Ray rr = r;
    if (flags & RTW_LEAF_ANIMATION) rr = xf_reverse(anim_xf(w, S, leaf, r.time), rr);
    if (flags & RTW_LEAF_TRANSFORM) rr = xf_reverse(leaf_xform(w, S, leaf), rr);
    return rr;
}

// SceneElement::hit for one leaf (candidate test: t only).  Volumes draw one f32 here.
// VOL: the world may hold volume leaves (the only leaves that draw from the path's RNG during the
// traversal); without them the RNG state never changes inside the loop
template <bool STATS, bool VOL, class TB>
__device__ __forceinline__ bool leaf_t(const DWorld& w, const TB& S, int leaf, const Ray& r, float ts, float te,
                                       rtw_xoro& rng, float& t, Stats& st) {
    const int4 info = leaf_info_of(w, S, leaf);
    const uint32_t flags = (uint32_t)info.w;
    const Ray rr = (flags & (RTW_LEAF_ANIMATION | RTW_LEAF_TRANSFORM)) ? leaf_local_ray(w, S, leaf, flags, r) : r;
    const bool volume = VOL && (flags & RTW_LEAF_VOLUME) != 0;
    // VolumeGeometry::hit (hittable.rs:309-331): boundary hit over (-inf, inf), then from t0+0.001
    float lo = volume ? -F32_INF : ts, hi = volume ? F32_INF : te;
    float t0 = 0.0f;
    for (int pass = 0;; ++pass) {
        float tt;
        if (!geom_t<STATS>(w, S, info.x, info.y, rr, lo, hi, tt, st)) return false;
        if (!volume) {
            t = tt;
            return true;
        }
        if (pass == 0) {
            t0 = tt;
            lo = t0 + 0.001f;
            continue;
        }
        const float sm = rtw_maxr(t0, ts);
        const float em = rtw_minr(tt, te);
        if (sm >= em) return false;
        const float nid = tab_gen(S, S.xf, w.leaf_xf, 3 * leaf).x;
        const float tv = rtw_maxr(sm, 0.0f) + nid * d_logf(d_gen_f32(&rng));
        if (tv > em) return false;
        t = tv;
        return true;
    }
}

// ---------------------------------------------------------------------------------------------
// hit record of the closest leaf (hittable.rs:24-102 + the primitives' record parts)
// ---------------------------------------------------------------------------------------------
struct Hit {
    V3 pos, n;
    float u, v;
    bool front;
    int material;
};
__device__ __forceinline__ void from_ray(Hit& h, const Ray& r, V3 pos, V3 sn, float u, float v) {
    h.front = dot(sn, r.d) < 0.0f;  // hittable.rs:41-46
    h.n = h.front ? sn : neg(sn);
    h.pos = pos;
    h.u = u;
    h.v = v;
}
template <class TB>
__device__ __forceinline__ void leaf_record(const DWorld& w, int leaf, const Ray& r, float t, Hit& h,
                                            const TB& S) {
    const int4 info = leaf_info_of(w, S, leaf);
    const uint32_t flags = (uint32_t)info.w;
    const Ray rr = leaf_local_ray(w, S, leaf, flags, r);
    const int kind = info.x, idx = info.y;
    if (flags & RTW_LEAF_VOLUME) {  // hittable.rs:333-340
        h.pos = at(rr, t);
        h.n = v3(0.0f, 1.0f, 0.0f);
        h.u = 0.0f;
        h.v = 0.0f;
        h.front = false;
    } else if (kind == RTW_GEOM_SPHERE) {  // sphere_geometry.rs:42-52
        // a plain sphere's leaf_fast record is {centre, radius} (the same floats as spheres[idx])
        const float4 s = (S.fast >= 0 && (flags & (RTW_LEAF_TRANSFORM | RTW_LEAF_ANIMATION)) == 0)
                             ? smem[S.fast + leaf] : tab_gen(S, S.sph, w.spheres, idx);
        const V3 pos = at(rr, t);
        const V3 sn = divs_x(sub(pos, v3(s.x, s.y, s.z)), s.w);
        // uv (vec3.rs:241-249) only reaches the image through an image texture; a pure function
        // of the normal, so skipping it where no image texture can read it changes nothing
        float u = 0.0f, v = 0.0f;
        if (flags & RTW_DLEAF_UV) {
            const float theta = TB::gen ? d_acosf_inl(sn.y) : d_acosf(sn.y);
            const float phi = (TB::gen ? d_atan2f_inl(-sn.z, sn.x) : d_atan2f(-sn.z, sn.x)) + F32_PI;
            u = div_c(phi, F32_TAU, 1.0f / F32_TAU);
            v = div_c(theta, F32_PI, 1.0f / F32_PI);
        }
        from_ray(h, rr, pos, sn, u, v);
    } else if (kind == RTW_GEOM_RECT) {  // rect_geometry.rs:37-55
        const RectG g = load_rect(w, S, idx);
        int p0, p1, n;
        rect_axes(g.plane, p0, p1, n);
        const V3 pos = add(rr.o, mul(rr.d, t));
        const float u = div_x(comp(pos, p0) - g.r00, g.r01 - g.r00);
        const float v = div_x(comp(pos, p1) - g.r10, g.r01 - g.r10);  // the :45 typo
        V3 sn = v3(0.0f, 0.0f, 0.0f);
        setc(sn, n, -1.0f);
        from_ray(h, rr, pos, sn, u, v);
    } else if (kind == RTW_GEOM_BOX) {  // aabb.rs:80-101
        const float4 ba = tab_gen(S, S.bx, w.boxes, 2 * idx), bb = tab_gen(S, S.bx, w.boxes, 2 * idx + 1);
        float nt, ft;
        int np, fp;
        box_line(ba, bb, rr, nt, np, ft, fp);
        const int plane = (t == nt) ? np : fp;
        const V3 pos = add(rr.o, mul(rr.d, t));
        const V3 bmin = v3(ba.x, ba.y, ba.z), bmax = v3(ba.w, bb.x, bb.y);
        const float center = (comp(bmax, plane) + comp(bmin, plane)) * 0.5f;
        V3 sn = v3(0.0f, 0.0f, 0.0f);
        setc(sn, plane, rtw_signum(comp(pos, plane) - center));
        from_ray(h, rr, pos, sn, 0.0f, 0.0f);
    } else {  // triangle_geometry.rs:22-39
        const TriFast T = load_tri(w.tri_fast, idx);
        const V3 pos = at(rr, t);
        const V3 q = sub(pos, T.p0);
        const float w1 = div_tri(dot(q, T.vt1), T.den1, T.y1);
        const float w2 = div_tri(dot(q, T.vt2), T.den2, T.y2);
        const float w0 = 1.0f - w1 - w2;
        const float4 a0 = w.tri_attr[4 * idx], a1 = w.tri_attr[4 * idx + 1], a2 = w.tri_attr[4 * idx + 2],
                     a3 = w.tri_attr[4 * idx + 3];
        const V3 n0 = v3(a0.x, a0.y, a0.z), n1 = v3(a0.w, a1.x, a1.y), n2 = v3(a1.z, a1.w, a2.x);
        const float u0 = a2.y, v0 = a2.z, u1 = a2.w, v1 = a3.x, u2 = a3.y, v2 = a3.z;
        const float u = u0 * w0 + u1 * w1 + u2 * w2;  // math.rs:9-16
        const float v = v0 * w0 + v1 * w1 + v2 * w2;
        const V3 sn = add(add(mul(n0, w0), mul(n1, w1)), mul(n2, w2));
        from_ray(h, rr, pos, sn, u, v);
    }
    // apply_hit_interaction, innermost wrapper first (hittable.rs:279-283)
    if (flags & RTW_LEAF_TRANSFORM) {
        const Xf x = leaf_xform(w, S, leaf);
        h.pos = add(rot_up(x.yc, x.ys, h.pos), x.off);
        h.n = rot_up(x.yc, x.ys, h.n);
    }
    if (flags & RTW_LEAF_ANIMATION) {
        const Xf x = anim_xf(w, S, leaf, r.time);
        h.pos = add(rot_up(x.yc, x.ys, h.pos), x.off);
        h.n = rot_up(x.yc, x.ys, h.n);
    }
    h.material = info.z;
}

// ---------------------------------------------------------------------------------------------
// BVH traversal (hittable.rs:429-473; aabb.rs:65-78)
// ---------------------------------------------------------------------------------------------
// Exact f32 division by a ray-direction component d with y = RN(1/d) precomputed per ray
// (Markstein): q = RN(a*y); r = fma(-d, q, a) (exact); q' = RN(q + r*y) == RN(a/d), provided
// 2^-60 <= |d| <= 2 and 2^-84 <= |a| <= 2^40, or a = 0 (then q' is a zero whose sign may differ
// from a/d's; the slab test only compares quotients, so no decision sees it).
// (tests/native/markstein_check.c checks every divisor significand under these guards.)
// The guards hold per ray, not per node: a = RN(c - o) for a node coordinate c and an origin
// component o.  If o = 0, a = c.  If |o| >= 2^-60 and c != o, |c - o| >= 2^-84 (the difference of
// two distinct floats is at least the finer one's ulp, or at least |o|/2).  So when every node
// coordinate is 0 or at least 2^-60 in magnitude (checked at upload: `mk_world`) and so is every
// origin component, each |a| is 0 or >= 2^-84; |a| <= 2^31 since coordinates are bounded by 2^30
// at upload.
#define RTW_MK_DMIN 0x1p-60f
#define RTW_MK_CMIN 0x1p-60f
__device__ __forceinline__ float mk_div(float a, float d, float y) {
    const float q = a * y;
    return __builtin_fmaf(__builtin_fmaf(-d, q, a), y, q);
}
__device__ __forceinline__ bool mk_coord_ok(float c) { return c == 0.0f || __builtin_fabsf(c) >= RTW_MK_CMIN; }

// One axis of Aabb::hit_cond (aabb.rs:65-78): (t0, t1) = minmax(qa, qb) (math.rs:35-41: `a < b`
// else swapped, so a NaN lands in t1 position of qa), tmin = max(t0, ts), tmax = min(t1, te) with
// Rust's NaN-dropping min/max, pass = !(tmax <= tmin).  te and ts are never NaN, so
//   pass <=> te > ts  &&  !(t1 <= ts)  &&  !(te <= t0)  &&  !(t1 <= t0)
// and !(t1 <= t0) <=> qa != qb (unordered-true).  The te > ts term is per node (node_pass).
__device__ __forceinline__ bool axis_pass(float qa, float qb, float ts, float te) {
    const bool lt = qa < qb;
    const float t0 = lt ? qa : qb;
    const float t1 = lt ? qb : qa;
    return (int)!(t1 <= ts) & (int)!(te <= t0) & (int)(qa != qb);  // non-short-circuit
}

struct RayPre {  // per-ray constants of the slab test
    V3 inv;
    bool fast;
};
// mk_world: every node coordinate is 0 or >= 2^-60 in magnitude (rtw_world_upload)
__device__ __forceinline__ RayPre ray_pre(const Ray& r, bool mk_world) {
    RayPre p;
    const float m = __builtin_fminf(__builtin_fminf(__builtin_fabsf(r.d.x), __builtin_fabsf(r.d.y)),
                                    __builtin_fabsf(r.d.z));
    const float M = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(r.d.x), __builtin_fabsf(r.d.y)),
                                    __builtin_fabsf(r.d.z));
    // RN(1 / d) by rcp_nr inside its range (§5.8); zero or extreme components divide
    p.inv = v3(rcp_nr(r.d.x), rcp_nr(r.d.y), rcp_nr(r.d.z));
    if (__builtin_expect(!(m >= RTW_RCP_LO && M <= RTW_RCP_HI), 0)) p.inv = v3(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
    p.fast = mk_world && (m >= RTW_MK_DMIN) && (M <= 2.0f) && mk_coord_ok(r.o.x) && mk_coord_ok(r.o.y) &&
             mk_coord_ok(r.o.z);
    return p;
}

// Aabb::hit_cond (exact quotients) AND the proximity cull (rtw_scalar.h rtw_cull_*), which
// reuses the same quotients: pass iff the segment [ts, te] meets the box grown by delta.
// FAST_ONLY: every ray of the call is Markstein-exact (render_body picks the loop per traversal
// call), so the true-division path and its per-lane branch are compiled out of the loop
template <bool FAST_ONLY = false>
__device__ __forceinline__ bool node_pass(float4 na, float4 nb, float2 km, const Ray& r, const RayPre& rp, float ts,
                                          float te) {
    const float a0 = na.x - r.o.x, b0 = na.w - r.o.x;
    const float a1 = na.y - r.o.y, b1 = nb.x - r.o.y;
    const float a2 = na.z - r.o.z, b2 = nb.y - r.o.z;
    const float delta = rtw_cull_delta(km.x, km.y, a0, b0, a1, b1, a2, b2);
    if (FAST_ONLY || __builtin_expect(rp.fast, 1)) {
        const float qa0 = mk_div(a0, r.d.x, rp.inv.x), qb0 = mk_div(b0, r.d.x, rp.inv.x);
        const float qa1 = mk_div(a1, r.d.y, rp.inv.y), qb1 = mk_div(b1, r.d.y, rp.inv.y);
        const float qa2 = mk_div(a2, r.d.z, rp.inv.z), qb2 = mk_div(b2, r.d.z, rp.inv.z);
        // Finite quotients (|a| <= 2^31, |d| >= 2^-60): no NaN, so Rust's minmax is min / max
        // (equal operands, +-0 included, only meet comparisons).
        const float t00 = __builtin_fminf(qa0, qb0), t10 = __builtin_fmaxf(qa0, qb0);
        const float t01 = __builtin_fminf(qa1, qb1), t11 = __builtin_fmaxf(qa1, qb1);
        const float t02 = __builtin_fminf(qa2, qb2), t12 = __builtin_fmaxf(qa2, qb2);
        const float t1min = __builtin_fminf(__builtin_fminf(t10, t11), t12);
        const float t0max = __builtin_fmaxf(__builtin_fmaxf(t00, t01), t02);
        // hit_cond = te > ts && t1min > ts && t0max < te && qa_i != qb_i (i.e. t1_i > t0_i) for
        // every axis.  All six are strict orderings x > y of non-NaN values (te may be +inf): the
        // quotients are finite, since upload bounds every node coordinate, leaf offset and the
        // camera by 2^30 (rtw_world_upload: "node bounds beyond 2^30"), so |a_i| <= 2^31 and
        // |q| <= 2^91 on this path's |d| >= 2^-60; no inf - inf arises.  And
        // for those x > y <=> RN(x - y) > 0 (no difference of distinct floats rounds to zero;
        // inf - finite = inf): one min over the six differences and one compare, instead of six
        // compares whose masks the scalar unit would AND together.
        const float dmin = __builtin_fminf(
            __builtin_fminf(__builtin_fminf(te - ts, t1min - ts), te - t0max),
            __builtin_fminf(__builtin_fminf(t10 - t00, t11 - t01), t12 - t02));
        // Given hit_cond, the cull's [max(ts, t0_i - w_i), min(te, t1_j + w_j)] is non-empty iff
        // max_i (t0_i - w_i) <= min_j (t1_j + w_j): ts <= te, ts < t1_j <= t1_j + w_j and
        // t0_i - w_i <= t0_i < te hold already (w_i >= 0).  A NaN delta (k = inf, D = 0, so every
        // a_i = b_i = 0 and hit_cond fails) passes, as rtw_cull_axis's NaN-dropping bounds do.
        const float w0 = delta * __builtin_fabsf(rp.inv.x), w1 = delta * __builtin_fabsf(rp.inv.y),
                    w2 = delta * __builtin_fabsf(rp.inv.z);
        const float lo = __builtin_fmaxf(__builtin_fmaxf(t00 - w0, t01 - w1), t02 - w2);
        const float hi = __builtin_fminf(__builtin_fminf(t10 + w0, t11 + w1), t12 + w2);
        return (int)(dmin > 0.0f) & (int)!(lo > hi);
    }
    const float qa0 = a0 / r.d.x, qb0 = b0 / r.d.x;
    const float qa1 = a1 / r.d.y, qb1 = b1 / r.d.y;
    const float qa2 = a2 / r.d.z, qb2 = b2 / r.d.z;
    // minmax per axis (math.rs:35-41: `a < b` else swapped)
    const bool l0 = qa0 < qb0, l1 = qa1 < qb1, l2 = qa2 < qb2;
    const float t00 = l0 ? qa0 : qb0, t10 = l0 ? qb0 : qa0;
    const float t01 = l1 ? qa1 : qb1, t11 = l1 ? qb1 : qa1;
    const float t02 = l2 ? qa2 : qb2, t12 = l2 ? qb2 : qa2;
    // hit_cond over the three axes at once: AND_i axis_pass(...) ==
    //   te > ts && !(min_i t1_i <= ts) && !(te <= max_i t0_i) && AND_i qa_i != qb_i
    // (min/max drop NaN operands, exactly the axes whose comparison is vacuously true)
    const float t1min = __builtin_fminf(__builtin_fminf(t10, t11), t12);
    const float t0max = __builtin_fmaxf(__builtin_fmaxf(t00, t01), t02);
    const int hit_cond = (int)(te > ts) & (int)!(t1min <= ts) & (int)!(te <= t0max) & (int)(qa0 != qb0) &
                         (int)(qa1 != qb1) & (int)(qa2 != qb2);
    float clo = ts, chi = te;
    rtw_cull_axis(t00, t10, delta * __builtin_fabsf(rp.inv.x), &clo, &chi);
    rtw_cull_axis(t01, t11, delta * __builtin_fabsf(rp.inv.y), &clo, &chi);
    rtw_cull_axis(t02, t12, delta * __builtin_fabsf(rp.inv.z), &clo, &chi);
    return hit_cond & (int)(clo <= chi);
}

// The SAH tree's node test: the proximity cull alone (fast rays only), i.e. the segment [ts, te]
// meets the box grown by delta.  Conservative: never rejects a node below which a leaf's test
// would accept a root in [ts, te) (§5.2), whatever the tree.  A NaN delta (k = inf, D = 0) drops
// out of the bounds, as in rtw_cull_axis.
// Cheap quotients: q = RN(a * RN(1/d)) is within 2.0001u |a/d| of a/d, where the exact-quotient
// test (the reference tree's node_pass) uses RN(a/d), within u |a/d|.  Since delta >= 64u D and
// D >= |a_i|, that error is <= w_i / 32 (w_i = delta / |d_i|), the two quotient roundings together
// <= 3 w_i / 64.  The SAH tree's k and m are uploaded x17/16 rounded up and the D term is 68u
// (sah_delta), so w_i here >= (17/16)(1 - 4u) w_i of the exact test: each bound of this interval
// lies outside the exact test's bound (RN is monotone), and this test passes every node that
// test passes.  One multiply per quotient instead of three operations.
// (Growing the box in space instead -- a_i - delta, b_i + delta, then the quotients: three operations less
// per box, the constants widened by 9/8 for the subtraction's rounding -- passed the containment and
// parity suites and was not faster: suzanne -0.5 %, profiles/r04/v7_space_margin_ab.txt.)
#define RTW_SAH_WIDEN (17.0f / 16.0f)
// DQ = false (the product): the k term takes D^2 >= Dq, so delta = fma(D, fma(k, D, 68u), m): two
// operations for five, and a delta at least as large up to two roundings (the containment argument's
// margin is 17/16 against 1 + 3/64; tests/test_gpu_node_pass.py checks both forms)
template <bool DQ = true>
__device__ __forceinline__ float sah_delta(float k, float m, float a0, float b0, float a1, float b1, float a2, float b2) {
    const float m0 = __builtin_fmaxf(__builtin_fabsf(a0), __builtin_fabsf(b0));
    const float m1 = __builtin_fmaxf(__builtin_fabsf(a1), __builtin_fabsf(b1));
    const float m2 = __builtin_fmaxf(__builtin_fabsf(a2), __builtin_fabsf(b2));
    const float d = (m0 + m1) + m2;
    if (!DQ) return __builtin_fmaf(d, __builtin_fmaf(k, d, 64.0f * RTW_SAH_WIDEN * RTW_CULL_U), m);
    const float dq = __builtin_fmaf(m2, m2, __builtin_fmaf(m1, m1, m0 * m0));
    return __builtin_fmaf(k, dq, __builtin_fmaf(64.0f * RTW_SAH_WIDEN * RTW_CULL_U, d, m));
}
template <bool DQ = true>
__device__ __forceinline__ bool node_pass_cons(float4 na, float4 nb, float2 km, const Ray& r, const RayPre& rp, float ts,
                                               float te, float& entry) {
    const float a0 = na.x - r.o.x, b0 = na.w - r.o.x;
    const float a1 = na.y - r.o.y, b1 = nb.x - r.o.y;
    const float a2 = na.z - r.o.z, b2 = nb.y - r.o.z;
    const float delta = sah_delta<DQ>(km.x, km.y, a0, b0, a1, b1, a2, b2);
    // the grown interval's ends per axis, one FMA each: (qa - delta inv, qb + delta inv) is (lo, hi) for inv > 0
    // and (hi, lo) for inv < 0 (a <= b; fast rays have finite non-zero inv), taken apart by one min and one max.
    // RN(q -+ delta |inv|) with the product exact differs from RN(q -+ RN(delta |inv|)) only by that
    // product's rounding, <= u w, far inside the w / 64 the widened constants leave (the containment
    // argument's real-valued bound holds with the exact product, and RN is monotone)
    const float qa0 = a0 * rp.inv.x, qb0 = b0 * rp.inv.x;
    const float qa1 = a1 * rp.inv.y, qb1 = b1 * rp.inv.y;
    const float qa2 = a2 * rp.inv.z, qb2 = b2 * rp.inv.z;
    const float e00 = __builtin_fmaf(delta, -rp.inv.x, qa0), e10 = __builtin_fmaf(delta, rp.inv.x, qb0);
    const float e01 = __builtin_fmaf(delta, -rp.inv.y, qa1), e11 = __builtin_fmaf(delta, rp.inv.y, qb1);
    const float e02 = __builtin_fmaf(delta, -rp.inv.z, qa2), e12 = __builtin_fmaf(delta, rp.inv.z, qb2);
    const float lo = __builtin_fmaxf(
        __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(e00, e10), __builtin_fminf(e01, e11)), __builtin_fminf(e02, e12)),
        ts);
    const float hi = __builtin_fminf(
        __builtin_fminf(__builtin_fminf(__builtin_fmaxf(e00, e10), __builtin_fmaxf(e01, e11)), __builtin_fmaxf(e02, e12)),
        te);
    entry = lo;  // where the segment enters the grown box: the near-first order of the SAH walk
    return !(lo > hi);
}

// The cull alone with exact quotients and the plain constants (the SAH node test before the cheap
// quotients; fast rays only): the reference the widened test must contain (eval_node_pass_kernel)
__device__ __forceinline__ bool node_pass_cull_exact(float4 na, float4 nb, float2 km, const Ray& r, const RayPre& rp,
                                                     float ts, float te) {
    const float a0 = na.x - r.o.x, b0 = na.w - r.o.x;
    const float a1 = na.y - r.o.y, b1 = nb.x - r.o.y;
    const float a2 = na.z - r.o.z, b2 = nb.y - r.o.z;
    const float delta = rtw_cull_delta(km.x, km.y, a0, b0, a1, b1, a2, b2);
    const float qa0 = mk_div(a0, r.d.x, rp.inv.x), qb0 = mk_div(b0, r.d.x, rp.inv.x);
    const float qa1 = mk_div(a1, r.d.y, rp.inv.y), qb1 = mk_div(b1, r.d.y, rp.inv.y);
    const float qa2 = mk_div(a2, r.d.z, rp.inv.z), qb2 = mk_div(b2, r.d.z, rp.inv.z);
    const float w0 = delta * __builtin_fabsf(rp.inv.x), w1 = delta * __builtin_fabsf(rp.inv.y),
                w2 = delta * __builtin_fabsf(rp.inv.z);
    const float lo = __builtin_fmaxf(
        __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(qa0, qb0) - w0, __builtin_fminf(qa1, qb1) - w1),
                        __builtin_fminf(qa2, qb2) - w2),
        ts);
    const float hi = __builtin_fminf(
        __builtin_fminf(__builtin_fminf(__builtin_fmaxf(qa0, qb0) + w0, __builtin_fmaxf(qa1, qb1) + w1),
                        __builtin_fmaxf(qa2, qb2) + w2),
        te);
    return !(lo > hi);
}

// Aabb::hit_cond (aabb.rs:65-78) alone, exact quotients (fast rays only): node_pass's first half
__device__ __forceinline__ bool box_hit_cond_fast(float4 na, float4 nb, const Ray& r, const RayPre& rp, float ts,
                                                  float te) {
    const float qa0 = mk_div(na.x - r.o.x, r.d.x, rp.inv.x), qb0 = mk_div(na.w - r.o.x, r.d.x, rp.inv.x);
    const float qa1 = mk_div(na.y - r.o.y, r.d.y, rp.inv.y), qb1 = mk_div(nb.x - r.o.y, r.d.y, rp.inv.y);
    const float qa2 = mk_div(na.z - r.o.z, r.d.z, rp.inv.z), qb2 = mk_div(nb.y - r.o.z, r.d.z, rp.inv.z);
    const float t00 = __builtin_fminf(qa0, qb0), t10 = __builtin_fmaxf(qa0, qb0);
    const float t01 = __builtin_fminf(qa1, qb1), t11 = __builtin_fmaxf(qa1, qb1);
    const float t02 = __builtin_fminf(qa2, qb2), t12 = __builtin_fmaxf(qa2, qb2);
    const float t1min = __builtin_fminf(__builtin_fminf(t10, t11), t12);
    const float t0max = __builtin_fmaxf(__builtin_fmaxf(t00, t01), t02);
    const float dmin = __builtin_fminf(__builtin_fminf(__builtin_fminf(te - ts, t1min - ts), te - t0max),
                                       __builtin_fminf(__builtin_fminf(t10 - t00, t11 - t01), t12 - t02));
    return dmin > 0.0f;
}

// The two-children walk's node record (build_sah_tables, plain-sphere worlds): node_b.z = axis |
// (left & 0x7FFF) << 2 | right << 17, children as in rtw_bvh_node (>= 0 node, < 0 leaf -1 - index; 15-bit
// signed: worlds of < 2^14 nodes and leaves); node_b.w = the node's cull constant m.  Its k is the world's
// (DWorld::sah_k, the largest finite node k: a larger k only grows delta, so the test stays conservative,
// DESIGN 5.2); a node whose k is infinite (no cull below it) carries m = +inf instead, which passes it as
// k = inf did.  The lane carries node_b.z itself as its packed children.  (The one-child walk of other
// worlds keeps {left << 2 | axis, right} and a cull-constant array: the folded record ran suzanne 2.7 %
// and cornell_cube 3 % slower, profiles/r05/ab_km.txt.)
__device__ __forceinline__ int32_t sah_left(int32_t bits) { return __builtin_amdgcn_sbfe(bits, 2u, 15u); }
__device__ __forceinline__ int32_t sah_right(int32_t bits) { return bits >> 17; }

// ---------------------------------------------------------------------------------------------
// textures / materials / light / background
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float perlin_noise(const float* ranvec, const uint32_t* px, int bits, V3 p) {  // perlin.rs:48-91
    const uint32_t mask = (1u << bits) - 1u;
    const uint32_t* py = px + 256;
    const uint32_t* pz = px + 512;
    const float fx = __builtin_floorf(p.x), fy = __builtin_floorf(p.y), fz = __builtin_floorf(p.z);
    const float u = p.x - fx, v = p.y - fy, ww = p.z - fz;
    const uint32_t i = (uint32_t)rtw_f2i32_sat(fx), j = (uint32_t)rtw_f2i32_sat(fy), k = (uint32_t)rtw_f2i32_sat(fz);
    const float uu = u * u * (3.0f - 2.0f * u);
    const float vv = v * v * (3.0f - 2.0f * v);
    const float wwx = ww * ww * (3.0f - 2.0f * ww);
    float accum = 0.0f;
    for (int q = 0; q < 8; ++q) {
        const int a = q >> 2, b = (q >> 1) & 1, c = q & 1;
        const uint32_t idx = px[(i + (uint32_t)a) & mask] ^ py[(j + (uint32_t)b) & mask] ^ pz[(k + (uint32_t)c) & mask];
        const V3 cv = ld3(ranvec + 3 * idx);
        const float fa = (float)a, fb = (float)b, fc = (float)c;
        const V3 weight = v3(u - fa, v - fb, ww - fc);
        accum += (fa * uu + (1.0f - fa) * (1.0f - uu)) * (fb * vv + (1.0f - fb) * (1.0f - vv)) *
                 (fc * wwx + (1.0f - fc) * (1.0f - wwx)) * dot(cv, weight);
    }
    return accum;
}

// Marble (texture.rs:44-51) with turbulence(p, 7, 0.5) (perlin.rs:37-47); rare, kept out of line
__device__ __forceinline__ float marble_k(const float* ranvec, const uint32_t* perm, int bits, float px, float py, float pz,
                                       float scale) {
    float acc = 0.0f, weight = 1.0f;
    V3 p = v3(px, py, pz);
    for (int i = 0; i < 7; ++i) {
        acc += weight * perlin_noise(ranvec, perm, bits, p);
        weight *= 0.5f;
        p = mul(p, 2.0f);
    }
    const float turb = __builtin_fabsf(acc);
    return 1.0f + d_sinf(pz * scale + 10.0f * turb);
}

// TX: the world's textures are all SolidColor (TX_SOLID) or not (TX_ANY: checker, marble, image)
enum { TX_SOLID = 0, TX_ANY = 1 };
// ImageTexture::value (texture.rs:40-53): the texel at (u, v) of the image whose texels start at `off`
template <bool STATS>
__device__ __forceinline__ V3 image_texel(const DWorld& w, int32_t off, int32_t width, int32_t height, const Hit& h,
                                          Stats& st) {
    uint32_t pu = rtw_f2u32_sat(h.u * (float)width);
    uint32_t pv = rtw_f2u32_sat(h.v * (float)height);
    pu = min(pu, (uint32_t)(width - 1));
    pv = min(pv, (uint32_t)(height - 1));
    if (STATS) st.c[ST_TEXEL]++;
    const uint32_t px = w.texels[(size_t)off + (size_t)pv * (size_t)width + pu];
    return v3(tex255(px & 255u), tex255((px >> 8) & 255u), tex255((px >> 16) & 255u));
}
// device-only material-record bit (above the RTW_MAT_* kinds): the material's texture is an image, whose
// {texel offset, width << 16 | height} the record carries in z, w (rtw_world_upload; Lambertian, Isotropic
// and DiffuseLight, which have no fuzz or index of refraction there) -- shading then reads the texel
// straight after the material record
#define RTW_DMAT_IMAGE (1 << 8)
template <bool STATS, int TX, class TB>
__device__ __forceinline__ V3 texture_sample(const DWorld& w, int tex, const Hit& h, Stats& st,
                                             const TB& S) {  // texture.rs:23-53
    for (int guard = 0; guard < 64; ++guard) {
        // the LDS table (launch_render, when it fits): solid-texture kernels each texture's first record,
        // the other non-GEN kernels all three records (earth_mapped +3 %, perlin_spheres +5 %); the GEN
        // kernels read HBM / L2 (as an LDS table
        // it cost C5 1.3 % in spills, profiles/r05/ab_tex_lds.txt)
        constexpr bool FULL = TX != TX_SOLID && !TB::gen;
        // GEN kernels with any texture kind get no table from launch_render: no LDS path compiled (with the
        // inlined uv functions above, earth_motion +1.9 %; alone -2.2 %, profiles/r06/ab_c5_spills.txt)
        constexpr bool NOTAB = TB::gen && TX != TX_SOLID;
        const int4 t0 = !NOTAB && S.tex0 >= 0 ? lds_i4(S.tex0 + (FULL ? 3 * tex : tex)) : w.textures[3 * tex];
        const int kind = t0.x;
        if (TX == TX_SOLID || kind == RTW_TEX_SOLID)
            return v3(__int_as_float(t0.y), __int_as_float(t0.z), __int_as_float(t0.w));
        // an image texture's first record is {kind, texel offset, width, height} (rtw_world_upload): the
        // texel is the second load of the chain, not the fourth (record, third record, image record, texel)
        if (kind == RTW_TEX_IMAGE) return image_texel<STATS>(w, t0.y, t0.z, t0.w, h, st);
        const int4 t1 = FULL && S.tex0 >= 0 ? lds_i4(S.tex0 + 3 * tex + 1) : w.textures[3 * tex + 1];
        if (kind == RTW_TEX_CHECKER) {
            const float f = __int_as_float(t1.x);
            const V3 s = mul(h.pos, f);
            tex = d_checker_odd(s.x, s.y, s.z) ? t1.y : t1.z;  // sines < 0
            continue;
        }
        const int4 t2 = FULL && S.tex0 >= 0 ? lds_i4(S.tex0 + 3 * tex + 2) : w.textures[3 * tex + 2];
        const int pi = t2.x;
        const float k = marble_k(w.perlin_ranvec + 768 * pi, w.perlin_perm + 768 * pi, w.perlin_bits[pi], h.pos.x,
                                 h.pos.y, h.pos.z, __int_as_float(t1.w));
        return mul(mul(v3(1.0f, 1.0f, 1.0f), 0.5f), k);
    }
    return v3(0.0f, 0.0f, 0.0f);
}

// rect_geometry.rs:60-85 (the light sampler)
__device__ __forceinline__ V3 light_generate(const rtw_rect& g, V3 origin, rtw_xoro& rng) {
    int p0, p1, n;
    rect_axes(g.plane, p0, p1, n);
    V3 e = v3(0.0f, 0.0f, 0.0f);
    setc(e, p0, d_gen_range_f32(g.r0[0], g.r0[1], &rng));
    setc(e, p1, d_gen_range_f32(g.r1[0], g.r1[1], &rng));
    setc(e, n, g.dist);
    return unit_x(sub(e, origin));
}
__device__ __forceinline__ float light_value(const rtw_rect& lg, V3 origin, V3 dir) {
    Ray r;
    r.o = origin;
    r.d = dir;
    r.time = 0.0f;
    const RectG g{lg.plane, lg.dist, lg.r0[0], lg.r0[1], lg.r1[0], lg.r1[1]};
    float t;
    V3 pos;
    if (!rect_t(g, r, 0.001f, F32_INF, t, pos)) return 0.0f;
    int p0, p1, n;
    rect_axes(g.plane, p0, p1, n);
    V3 sn = v3(0.0f, 0.0f, 0.0f);
    setc(sn, n, -1.0f);
    const V3 hn = (dot(sn, dir) < 0.0f) ? sn : neg(sn);
    const float area = (g.r01 - g.r00) * (g.r11 - g.r10);
    const float dsq = t * t;
    const float cosine = __builtin_fabsf(dot(hn, dir));
    return div_x(dsq, cosine * area);
}

// background_color.rs:9-19; `pdot` = dot((0, 1, 0), d) of the primary ray, computed once per sample
// (start_sample), so that a path carries one float instead of the direction
__device__ __forceinline__ V3 background(const rtw_background& bg, float pdot) {
    if (bg.kind == RTW_BG_SKY) {
        const float t = 0.5f * (pdot + 1.0f);
        return add(mul(v3(1.0f, 1.0f, 1.0f), 1.0f - t), mul(v3(0.5f, 0.7f, 1.0f), t));
    }
    return v3(bg.color[0], bg.color[1], bg.color[2]);
}

// Camera::ray (camera.rs:175-200)
__device__ __forceinline__ Ray camera_ray(const rtw_camera& c, rtw_xoro& rng, float px, float py) {
    V3 off = v3(0.0f, 0.0f, 0.0f);
    if (c.lens_radius > 0.0f) {
        float d0, d1;
        d_unit_disc(&rng, d0, d1);
        off = mul(add(mul(ld3(c.unit_right), d0), mul(ld3(c.unit_up), d1)), c.lens_radius);
    }
    float start;
    if (c.time0 == c.time1) start = c.time0;
    else start = d_gen_range_f32(c.time0, c.time1, &rng);
    Ray r;
    r.time = start + (c.shutter_pace[0] * px + c.shutter_pace[1] * py);
    r.o = add(ld3(c.position), off);
    r.d = unit_x(sub(sub(add(ld3(c.upper_left_corner), mul(ld3(c.scaled_right), px)), mul(ld3(c.scaled_up), py)), off));
    return r;
}

// ---------------------------------------------------------------------------------------------
// the megakernel
// ---------------------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------------------
// shading: one bounce of ray_color (rendering.rs:19-71), out of line so that its temporaries
// and hoisted invariants never pressure the traversal loop's registers
// ---------------------------------------------------------------------------------------------
// Experiment builds only (make variant DEFS=-DRTW_PHASE_TIMING): per-wave wall cycles of the main
// loop's phases, summed over waves into rtw_phase_cycles (read by rtw_debug_phase_cycles).
// The phase is a property of the wave: it lives in LDS (per wave: 8 sums, the last stamp, the current
// phase), and the first active lane switches it, so that a switch inside divergent code (the shading
// lanes' samplers) charges the wave's cycles to the right phase.  Phases: 1 refill (work items),
// 2 traversal setup, 3 traversal (walk, drain, proof, re-trace), 4 shading, 5 sample start (stream
// setup, jitter, camera ray with its UnitDisc), 6 shading's samplers (UnitSphere / UnitBall /
// gen_bool / light direction), 7 colour store and cost bookkeeping.
#ifdef RTW_PHASE_TIMING
__device__ unsigned long long rtw_phase_cycles[8];
__device__ __forceinline__ unsigned long long* pt_slot() {
    __shared__ unsigned long long s[(RTW_BLOCK / 64) * 10];
    return s + (threadIdx.x >> 6) * 10;
}
#define RTW_PT_DECL do { unsigned long long* s_ = pt_slot(); if ((threadIdx.x & 63) == 0) { for (int k_ = 0; k_ < 8; ++k_) s_[k_] = 0; s_[8] = clock64(); s_[9] = 0; } } while (0);
#define RTW_PT(k) do { if ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1) { unsigned long long* s_ = pt_slot(); const unsigned long long now_ = clock64(); s_[s_[9]] += now_ - s_[8]; s_[8] = now_; s_[9] = (k); } } while (0)
#define RTW_PT_FLUSH do { RTW_PT(0); if ((threadIdx.x & 63) == 0) for (int k_ = 0; k_ < 8; ++k_) atomicAdd(&rtw_phase_cycles[k_], pt_slot()[k_]); } while (0)
#else
#define RTW_PT_DECL
#define RTW_PT(k) do { } while (0)
#define RTW_PT_FLUSH do { } while (0)
#endif

struct Path {  // per-path state crossing the call by value (registers)
    Ray ray;
    V3 att, acc;
    int32_t depth;
    rtw_xoro rng;
};
struct ShadeOut {
    Path p;
    V3 color;
    int32_t done;   // 1: the sample is finished, `color` is its radiance
    uint32_t texels;
};

template <bool STATS, int TX, class TB>
__device__ __forceinline__ ShadeOut shade(const DWorld* __restrict__ wp, int32_t mode, Path P, int32_t found, float te,
                                       float pdot, const TB& S) {
    const DWorld& w = *wp;
    Stats st;
    st.c[ST_TEXEL] = 0;
    Ray& ray = P.ray;
    V3& att = P.att;
    V3& acc = P.acc;
    int32_t& depth = P.depth;
    rtw_xoro& rng = P.rng;
    V3 color = v3(0.0f, 0.0f, 0.0f);
    bool done = false;
    if (found >= 0) {
        Hit h;
        leaf_record(w, found, ray, te, h, S);
        if (mode == RTW_MODE_NORMALS) {  // rendering.rs:110-113
            color = mul(add(h.n, v3(1.0f, 1.0f, 1.0f)), 0.5f);
            done = true;
        } else if (depth <= 1) {  // rendering.rs:26-27
            color = v3(0.0f, 0.0f, 0.0f);
            done = true;
        } else {
                const int4 M = S.mat >= 0 ? lds_i4(S.mat + h.material) : w.materials[h.material];
                const int mkind = M.x & (RTW_DMAT_IMAGE - 1);
                const bool direct_image = TX != TX_SOLID && (M.x & RTW_DMAT_IMAGE) != 0;
                // Material::scatter (material.rs:52-114).  At most one texture lookup per bounce:
                // the albedo of a scattering material or the emission of a DiffuseLight.
                bool scatters = true;
                bool cosine = false;      // MaterialScatteringDistribution::Cosine
                bool need_sphere = false; // one UnitSphere draw site (Cosine / Isotropic)
                int tex = -1;
                V3 sdir = v3(0.0f, 0.0f, 0.0f);
                if (mkind == RTW_MAT_LAMBERT) {
                    tex = M.y;
                    cosine = true;
                } else if (mkind == RTW_MAT_METAL) {
                    const float fuzz = __int_as_float(M.z);
                    V3 fz = v3(0.0f, 0.0f, 0.0f);
                    if (fuzz > 0.0f) {
                        RTW_PT(6);
                        const V3 b = d_unit_ball(&rng);
                        RTW_PT(4);
                        fz = mul(b, fuzz);
                    }
                    const V3 dir = add(reflect(ray.d, h.n), fz);
                    if (dot(dir, h.n) > 0.0f) {
                        sdir = unit_x(dir);
                        tex = M.y;
                    } else {
                        scatters = false;
                    }
                } else if (mkind == RTW_MAT_DIELECTRIC) {
                    const float ior = __int_as_float(M.w);
                    const float ratio = h.front ? rcp_x(ior) : ior;
                    const float cos_t = rtw_minr(dot(neg(ray.d), h.n), 1.0f);
                    const float sin_t = sqrt_x(1.0f - cos_t * cos_t);
                    bool refl = ratio * sin_t > 1.0f;
                    if (!refl) {
                        const float r0 = div_x(1.0f - ratio, 1.0f + ratio);
                        const float rs = r0 * r0;
                        const float x = 1.0f - cos_t;
                        const float x2 = x * x;
                        const float p5 = x * (x2 * x2);  // powi(5)
                        refl = (rs + (1.0f - rs) * p5) > d_gen_f32(&rng);
                    }
                    sdir = unit_x(refl ? reflect(ray.d, h.n) : refract(ray.d, h.n, ratio));
                } else if (mkind == RTW_MAT_ISOTROPIC) {
                    need_sphere = true;
                    tex = M.y;
                } else {
                    scatters = false;  // DiffuseLight: emit
                    tex = M.y;
                }
                // sample_final_scattering_distribution (rendering.rs:73-92): the mixture draws its
                // bool before either generator.
                bool light_dir = false;
                RTW_PT(6);
                if (cosine) {
                    if (w.has_light) light_dir = d_gen_bool_half(&rng);
                    need_sphere = !light_dir;
                }
                if (light_dir) sdir = light_generate(w.wc->light, h.pos, rng);
                if (need_sphere) {
                    const V3 sv = d_unit_sphere(&rng);
                    if (cosine) {  // (n + UnitSphere).unit_or_else(n) (material.rs:20-22)
                        const V3 v = add(h.n, sv);
                        const float lsq = dot(v, v);
                        if (lsq > 1e-8f) {  // 1e-4 < s <= 2: inside div_y's divisor range
                            const float s = sqrt_nr(lsq);  // 1e-8 < lsq <= 4
                            sdir = divs_y(v, s, rcp_nr(s));
                        } else {
                            sdir = h.n;
                        }
                    } else {
                        sdir = sv;
                    }
                }
                RTW_PT(4);
                const V3 tc = tex < 0         ? v3(0.0f, 0.0f, 0.0f)
                              : direct_image ? image_texel<STATS>(w, M.z, (int32_t)((uint32_t)M.w >> 16), M.w & 0xFFFF, h, st)
                                             : texture_sample<STATS, TX>(w, tex, h, st, S);
                const V3 emitted = (mkind == RTW_MAT_DIFFUSE_LIGHT) ? tc : v3(0.0f, 0.0f, 0.0f);
                const V3 albedo = (mkind == RTW_MAT_DIELECTRIC) ? v3(1.0f, 1.0f, 1.0f) : tc;
                if (scatters) {
                    float prob = 1.0f;
                    if (cosine) {
                        const float mv = div_c(rtw_maxr(dot(h.n, sdir), 0.0f), F32_PI, 1.0f / F32_PI);  // Cosine::value
                        // material.rs:123-127: the same expression as mv, so without a light p = spdf
                        // and spdf / p is 1 (finite non-zero spdf) or 0 / 0
                        const float spdf = mv;
                        if (w.has_light) {
                            const float p = 0.5f * light_value(w.wc->light, h.pos, sdir) + (1.0f - 0.5f) * mv;
                            prob = div_x(spdf, p);
                        } else {
                            prob = spdf != 0.0f ? 1.0f : __builtin_nanf("");
                        }
                    }
                    acc = add(acc, conv(att, emitted));
                    att = mul(conv(att, albedo), prob);
                    ray.o = h.pos;
                    ray.d = sdir;
                    depth -= 1;
                } else {
                    color = add(acc, conv(att, emitted));
                    done = true;
                }
        }
    } else {
        // rendering.rs:67 (background of the PRIMARY ray) / :114
        color = add(acc, conv(att, background(w.wc->bg, pdot)));
        done = true;
    }
    ShadeOut o;
    o.p = P;
    o.color = color;
    o.done = done ? 1 : 0;
    o.texels = STATS ? st.c[ST_TEXEL] : 0u;
    return o;
}

// the block-shared drain's traffic (rtw_debug_drain_counts; tests): rays posted to a mailbox, posts traced
// by another wave of the block, posts traced by their owner -- counted in the block's mailbox words 33-35 (LDS
// atomics) and added here once per block at its end (as one global atomic per post, the counters cost
// suzanne's 8-way shares 13 %: every block's drain contended on three addresses)
__device__ unsigned long long rtw_drain_counts[3];

#ifdef RTW_WAVE_TIMING  // experiment builds: per-wave start / end / queue-empty wall clocks of the last launch
__device__ unsigned long long rtw_wave_times[3 * 8192];
__device__ unsigned long long rtw_wave_dry[8192];  // first time a lane of the wave found the queue empty
// per wave after the queue ran dry: busy lanes then, samples finished, their bounces (sum, max),
// cooperative rays, reference-tree re-traces, wall ticks in the re-traces and in the SAH walk + coop
__device__ unsigned long long rtw_wave_extra[8 * 8192];
#endif

// PH_REF: the ray is traced on the reference tree (the SAH path's fallback, §5.6)
// PH_DONE: the queues are empty and the lane's last path is finished (it stays in the loop, masked
// by its phase, so that the wave's remaining rays can be traced with all 64 lanes: coop_solve)
enum { PH_PIXEL = 0, PH_TRACE = 1, PH_SHADE = 2, PH_REF = 3, PH_DONE = 4 };
// traversal modes: the reference tree (DFS of hittable.rs:429-473 with hit_cond AND the cull), the
// SAH tree (cull only, closest hit with ties flagged), the reference tree for PH_REF lanes with
// the scene in HBM (the LDS holds the SAH tree)
enum { TM_REF = 0, TM_SAH = 1, TM_FALLBACK = 2 };
// Trav.fast bits above the direction signs (0-2) and the Markstein flag (3)
#define RTW_TF_SAH 16  // the ray is traced on the SAH tree; te = the closest t's successor
#define RTW_TF_TIE 32  // another leaf reported exactly the closest t


// Traversal state of one lane (by value, in registers, across the out-of-line call).
struct Trav {
    Ray ray;
    V3 inv;         // RN(1 / ray.d)
    int32_t fast;   // bits 0-2: ray.d[i] > 0 (the near child's side per axis); bit 3: Markstein division
                    // usable; RTW_TF_SAH, RTW_TF_TIE
    int32_t node;   // current node (>= 0) or ~leaf
    int32_t sp;
    float te;       // t_range.end, shrunk by every hit (hittable.rs:457)
    int32_t found;  // closest leaf so far, -1 if none
    rtw_xoro rng;   // volumes draw from the path's stream during traversal
    int32_t phase;
    // statistics of one call (counting variant); tests packed 16 bits per kind (a lane traces at
    // most one ray's remainder per call: far below 2^16 tests of one kind)
    uint32_t n_nodes, n_sph_rect, n_box_tri;
};

// The hot loop: every lane in PH_TRACE advances one node or leaf per iteration until fewer than
// `trace_min` lanes are still tracing while some lane waits for shading (dynamic ray fetch).
// Out of line so that it gets a register allocation of its own.

// LDS modes of the render kernel: 0 scene in HBM, 1 nodes + leaf records + cull constants + rect
// records in LDS, 2 also the plain-triangle records (tri_fast).  LDS layout: [node_a n][node_b n]
// [leaf_fast L][km ceil(n/2)][rects 2R][tri_fast 4T (mode 2)][stack depth x BLOCK]
// Leaf kinds of the world (LK): 0 plain spheres only, 1 plain spheres and triangles, 2 plain
// spheres / rects / triangles, 3 wrapped leaves and boxes too (the generic leaf path without
// volumes), 4 any (volumes: the generic path draws from the RNG).  A world without generic leaves
// gets a loop without that path, and one without volumes a generic path that leaves the RNG alone:
// the RNG update alone made the compiler copy the lane's traversal registers at the leaf merge on
// every leaf step.
enum { LK_SPHERES = 0, LK_TRIS = 1, LK_PLAIN = 2, LK_WRAPPED = 3, LK_ANY = 4 };
// Bytes per traversal-stack entry of render_kernel<.., LDS, LK, ..> -- the one predicate traverse's
// StackEntry, the shared drain's mailbox slots (mb_slot) and launch_render's LDS sizing all use: 16-bit
// node / leaf indices in LDS modes 1 and 2 (worlds below 2^15 nodes and leaves, checked at launch), 32-bit
// where the scene is in HBM and in the plain-sphere worlds' mode 1, whose two-children walk pushes packed
// children words (sah_left / sah_right).
__host__ __device__ constexpr int stack_entry_bytes(int lds, int lk) {
    return (lds == 2 || (lds == 1 && lk != LK_SPHERES)) ? 2 : 4;
}
// Leaves [0, tri_prefix) of a triangle-and-sphere world (LK_TRIS) are plain triangles with triangle
// index = leaf index (a mesh's leaves in order: suzanne's 968 of 969, rtw_world_upload): their leaf
// records are not read -- no dependent LDS read between the walk and the triangle record -- and not held
// in LDS, whose leaf-record section starts at leaf tri_prefix.  The record such a leaf would have
// (tag 1, its index in y, w = NaN) is made up instead.  tri_prefix = 0 in other worlds and kernels
// (rect worlds, LK_PLAIN, take every record: the test cost cornell_cube's leaf-heavy walk 2 %).
template <int LK>
__device__ __forceinline__ float4 walk_leaf_record(const float4* __restrict__ fast, int32_t leaf, int32_t tri_prefix) {
    // (the record read always and the made-up one selected: suzanne -0.4 %, profiles/r06/ab_mode2_suzanne.txt)
    if (LK == LK_TRIS && leaf < tri_prefix)
        return make_float4(__int_as_float(1), __int_as_float(leaf), 0.0f, __int_as_float(0x7FC00000));
    return fast[leaf];
}
// the LDS triangle records' stride in kernels of leaf kinds LK (see load_tri_soa)
template <int LK>
__device__ __forceinline__ int32_t tri_soa_stride(int32_t tri_stride) {
    return LK == LK_TRIS ? tri_stride : RTW_TRI_SOA;
}
template <bool STATS, int LDS, int LK, bool FAST_ONLY, int TM, class TB>
__device__ __forceinline__ Trav traverse(const DWorld* __restrict__ wp, const TB& S, Trav T, int32_t trace_min,
                                      int32_t n_nodes, int32_t n_leaves, int32_t n_rects, int32_t tri_prefix,
                                      int32_t tri_stride, int32_t stack_off, unsigned long long* dbg,
                                      int32_t coop_exit = -1) {
    // the LDS holds the tree this mode walks (the SAH tree in SAH mode); the fallback reads HBM
    constexpr bool LDS_SCENE = LDS >= 1 && TM != TM_FALLBACK;
    constexpr int ACT = TM == TM_FALLBACK ? PH_REF : PH_TRACE;  // the lanes this loop advances
    const DWorld& w = *wp;
    // the plain-triangle records' base, loaded once per call into scalar registers (the world
    // struct is read through a pointer; left in the loop it becomes a dependent global load)
    // LDS: the SAH tree has no cull-constant section (they are in node_b.w)
    constexpr bool C2 = TM == TM_SAH && LK == LK_SPHERES;  // the two-children walk (below)
    // (the LDS leaf records start at leaf tri_prefix, walk_leaf_record)
    const int32_t rect_off = 2 * n_nodes + n_leaves - tri_prefix + (C2 ? 0 : (n_nodes + 1) / 2);
    const int32_t tri_off = rect_off + 2 * n_rects;
    const float4* rects = LDS_SCENE ? smem + rect_off : uniform_ptr(w.rects);
    const float4* tri_fast = LDS == 2 && LDS_SCENE ? smem + tri_off : uniform_ptr(w.tri_fast);
    // nodes as two SoA halves (bank-conflict spread of ds_read_b128), then the leaf records
    // The LDS section offsets are held in VGPRs (opaque copies): as SGPRs they compete with the
    // loop's exec masks and get spilled to VGPR lanes, costing a v_readlane per node step.
    int32_t off_b = n_nodes, off_f = 2 * n_nodes - tri_prefix, off_k = 2 * (2 * n_nodes + n_leaves - tri_prefix);
    if (LDS_SCENE) asm volatile("" : "+v"(off_b), "+v"(off_f), "+v"(off_k));
    if (LDS == 2 && LDS_SCENE && LK == LK_TRIS) asm volatile("" : "+v"(tri_stride));
    // the two-children walk's k, also in a VGPR (a scalar would join the spilled SGPRs)
    float sah_k = C2 ? w.sah_k : 0.0f;
    if (C2) asm volatile("" : "+v"(sah_k));
    const float4* nodes_a = LDS_SCENE ? smem : TM == TM_SAH ? w.sah_a : w.node_a;
    const float4* nodes_b = LDS_SCENE ? smem + off_b : TM == TM_SAH ? w.sah_b : w.node_b;
    const float4* fast = LDS_SCENE ? smem + off_f : w.leaf_fast;
    const float2* nkm = LDS_SCENE ? reinterpret_cast<const float2*>(smem) + off_k : TM == TM_SAH ? w.sah_km : w.node_km;
    // 16-bit entries in the LDS modes (launch_render takes them only for worlds of < 2^15 nodes and
    // leaves): half the stack bytes, room for a deeper SAH tree or the triangle records -- except in
    // plain-sphere worlds, whose two-children walk pushes packed children words
    using StackEntry = std::conditional_t<stack_entry_bytes(LDS, LK) == 2, int16_t, int32_t>;
    StackEntry* stack = reinterpret_cast<StackEntry*>(smem + stack_off) + threadIdx.x;
    // a leaf's root t: the reference narrows te to it; the SAH walk keeps te = succ(closest t) so
    // that a leaf reporting exactly the closest t again (a tie, whose winner is the reference's
    // DFS order) is seen and flagged
    auto take = [&](float t, int leaf) {
        if (TM == TM_SAH) {
            // selects, not branches (+1.6 % on final_scene1: the branchy form cost exec-mask work).
            // t < te = succ(closest), so t is either the closest t again (`same`) or strictly closer.
            // Strictly closer: a new closest leaf, any earlier tie is void.  The same t from another
            // leaf: a tie.  The same t from the kept leaf itself (a leaf referenced twice -- a spatial
            // split of the SAH tree, rtw_sah.cpp): nothing changes, and a tie flagged by a third leaf
            // in between must stay (clearing it there let the proof pass without a re-trace)
            const bool same = T.found >= 0 && t == __int_as_float(__float_as_int(T.te) - 1);
            const bool tie = same && T.found != leaf;
            T.fast = same ? (tie ? (T.fast | RTW_TF_TIE) : T.fast) : (T.fast & ~RTW_TF_TIE);
            T.te = same ? T.te : __int_as_float(__float_as_int(t) + 1);  // t >= 0.001: the next float up
            T.found = same ? T.found : leaf;
        } else {
            T.te = t;
            T.found = leaf;
        }
    };
    // (take() under the hit predicate as selects, with no branch around it in the two-children step:
    // -0.8 %, profiles/r04/v19_take_sel_ab.txt)
    // SAH walk of plain-sphere worlds: two children per node step (below).  (Stack entries packing
    // the pushed child's entry t, so that a pop skips children starting beyond te, lost 5 %: the
    // skip loop's divergence costs more than the node steps it saves, profiles/r02/v9_two_child_ab.txt.)
    // The two-children step tests a leaf child's sphere at once: leaves are never pushed or stood on, so
    // the loop has no leaf steps (final_scene1 +3.0 % over round 2's leaf-then-node step,
    // profiles/r03/v9_inline_leaf_ab.txt).  The lane carries, instead of the node it stands on, that
    // node's two children packed in 16 bits each: they came with the node's box record in its parent's
    // step (nodes_b.zw), and a pushed node is pushed as its children -- one dependent LDS read less per
    // step (+0.9 %, profiles/r04/v4_experiments_ab.txt; worlds of < 2^15 nodes and leaves, checked at
    // upload).
    // the SAH node test's k term: D^2 (two operations; every world gained 0.5 % over round 2's Dq form,
    // profiles/r03/v6_delta_d2_ab.txt)
    constexpr bool SAH_DQ = false;
    // (reading the stack's top as each step starts, so that a pop finds it arrived, lost 0.4-2.3 %:
    // profiles/r04/v6_spec_pop_ab.txt)
    auto pop = [&]() {
        if (T.sp == 0) T.phase = PH_SHADE;
        else T.node = stack[(--T.sp) * RTW_BLOCK];
    };
    Stats st;
    if (STATS)
        for (int i = 0; i < ST_COUNT; ++i) st.c[i] = 0;
    const RayPre rp{T.inv, (T.fast & 8) != 0};
    // one leaf's test at the current t range (hittable.rs:436-437: a leaf is never box-tested)
    auto test_leaf = [&](int leaf) {
        const float4 sph = walk_leaf_record<LK>(fast, leaf, tri_prefix);
        if (LK == LK_SPHERES || sph.w == sph.w) {  // a plain sphere
            if (STATS) st.c[ST_T_SPHERE]++;
            float t;
            if (sphere_t(sph, T.ray, 0.001f, T.te, t)) take(t, leaf);
        } else if (LK >= LK_PLAIN && __float_as_int(sph.x) == 2) {  // a plain rect
            if (STATS) st.c[ST_T_RECT]++;
            const int ri = __float_as_int(sph.y);
            const float4 ra = rects[2 * ri], rb = rects[2 * ri + 1];
            const RectG g{__float_as_int(rb.y), ra.x, ra.y, ra.z, ra.w, rb.x};
            float t;
            V3 pos;
            if (FAST_ONLY ? rect_t_mk(g, T.ray, rp.inv, 0.001f, T.te, t) : rect_t(g, T.ray, 0.001f, T.te, t, pos))
                take(t, leaf);
        } else if (LK == LK_TRIS || LK == LK_PLAIN || __float_as_int(sph.x) == 1) {  // a plain triangle
            if (STATS) st.c[ST_T_TRI]++;
            float t;
            const int ti = __float_as_int(sph.y);
            if (tri_test(LDS == 2 && LDS_SCENE ? load_tri_soa(tri_fast, ti, tri_soa_stride<LK>(tri_stride)) : load_tri(tri_fast, ti), T.ray, 0.001f,
                         T.te, t))
                take(t, leaf);
        } else if (LK >= LK_WRAPPED && __float_as_int(sph.x) == 3) {
            // a sphere under an Animation wrapper only (C5's moving spheres): the generic path's
            // arithmetic (leaf_t: the ray moved by -velocity x time, hittable.rs:239-244, then the sphere
            // test) without its leaf-record read and kind dispatch
            if (STATS) st.c[ST_T_SPHERE]++;
            const Ray rr = xf_reverse(anim_xf(w, S, leaf, T.ray.time), T.ray);
            float t;
            if (sphere_t(tab_gen(S, S.sph, w.spheres, __float_as_int(sph.y)), rr, 0.001f, T.te, t)) take(t, leaf);
        } else if (LK >= LK_WRAPPED) {
            float t;
            if (leaf_t<STATS, LK == LK_ANY>(w, S, leaf, T.ray, 0.001f, T.te, T.rng, t, st)) take(t, leaf);
        }
    };

    // execution counters, summed over lanes at the end: wave-level events are counted by the
    // first active lane of the wave (or of the branch) only
    uint32_t db[DB_SHADE_CALLS] = {};
    const bool lead0 = (int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1;
    if (STATS && lead0) db[DB_TRAV_CALLS] = 1;
    // Each iteration a lane first tests the leaf it stands on, if any (popping the next item),
    // then tests the node it stands on, if any (pushing the far child, moving to the near one):
    // one leaf body and one node body per iteration, both in the reference's DFS order with the
    // current t_range.  A lane reaching a leaf child tests it at the start of the next iteration.
    for (;;) {
        const unsigned long long tr = __ballot(T.phase == ACT);
        if (tr == 0) break;
        // dynamic ray fetch: leave for shading when fewer than trace_min lanes still trace and some
        // lane waits (the threshold is tuned per world on the device, see TuneState); the fallback
        // (rare lanes) runs to the end
        if (TM != TM_FALLBACK && (uint32_t)__popcll(tr) < (uint32_t)trace_min && __ballot(T.phase == PH_SHADE) != 0)
            break;
        // the drain: the last few tracing lanes (the long walks) go to coop_solve
        if (TM == TM_SAH && (int32_t)__popcll(tr) <= coop_exit) break;
        if (STATS) {
            const unsigned long long lm = __ballot(T.phase == ACT && T.node < 0);
            const uint32_t alive = (uint32_t)__popcll(__ballot(T.phase != PH_DONE));
            const uint32_t waiting = (uint32_t)__popcll(__ballot(T.phase == PH_SHADE));
            if ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1) {
                db[DB_ITERS]++;
                db[DB_LEAF_ITERS] += lm != 0;
                db[DB_LEAF_LANES] += (uint32_t)__popcll(lm);
                db[DB_ALIVE_LANES] += alive;
                db[DB_WAIT_LANES] += waiting;
            }
        }
        // RTW_TRAV_UNROLL leaf + node steps per exit check: the check's ballots, popcount and
        // branches cost about as much as a node step's scalar work.  A lane that finishes inside the
        // group waits for the group's end (same-call A/B of 1/2/3/4/6/8/12: 6 is fastest,
        // final_scene1 +6 %, suzanne +4 %, cornell_cube +6 % over 1)
#ifndef RTW_TRAV_UNROLL
#define RTW_TRAV_UNROLL 6
#endif
#pragma unroll
// the two-children walk has the costlier step: 3 steps per check there (+1.0 % over 6 on
// final_scene1, 4: +0.5 %, profiles/r02/v9_take_unroll_ab.txt)
#ifndef RTW_C2_UNROLL
#define RTW_C2_UNROLL 3
#endif
#ifndef RTW_FB_UNROLL
#define RTW_FB_UNROLL 1  // the re-trace loop (rare rays): no unrolling, a smaller kernel (suzanne +0.8 %, profiles/r03/v7_code_size_ab.txt)
#endif
        for (int u = 0; u < (STATS ? 1 : C2 ? RTW_C2_UNROLL : TM == TM_FALLBACK ? RTW_FB_UNROLL : RTW_TRAV_UNROLL); ++u) {
        // leaf bodies on every step, or (LK_SPHERES, LK_TRIS) on even steps only: a lane reaching a
        // leaf then waits up to one step, and the wave runs a leaf body for twice the lanes half as
        // often.  That pays where leaf steps are a small share (final_scene1 ~0.1 leaf per node
        // step, suzanne ~0.4: +3 %, +5 %) and costs where leaves come at every turn (cornell_cube's
        // wall rects, ~0.8: -8 %), hence only for worlds without rect, box or wrapped leaves.
        // The two-children step of plain-sphere SAH walks (C2) halves the node steps between leaves:
        // there a leaf body on every step is 3 % faster (profiles/r02/v9_leaf_cadence_ab.txt).
        // (every third step instead: suzanne -8.6 %, profiles/r04/v16_leaf_cadence_ab.txt)
        if (!C2 && (STATS || u % 2 == 0 || LK >= LK_PLAIN) && T.phase == ACT && T.node < 0) {
            test_leaf(-1 - T.node);
            pop();
        }
        if (STATS) {
            const unsigned long long nm = __ballot(T.phase == ACT && T.node >= 0);
            if ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1) {
                db[DB_NODE_ITERS] += nm != 0;
                db[DB_NODE_LANES] += (uint32_t)__popcll(nm);
            }
        }
        if (C2 && T.phase == ACT) {
            // SAH walk, two children per step: the lane stands on a node already accepted (the root,
            // or a child accepted by its parent's step) and tests both children's grown boxes at once
            // (leaf children need no box: their own test follows); accepted children are visited
            // near first (a leaf first), the other one pushed.  Any visit order finds the same
            // closest root (§5.5 step 1), so only the work changes.
            const int32_t left = sah_left(T.node);
            const int32_t right = sah_right(T.node);
            float el = F32_INF, er = F32_INF;
            bool pl = false, pr = false;
            int32_t lc = left, rc = right;  // what stands for an accepted child: its packed children
            // leaf children: their sphere now (never pushed or visited); internal ones: the box
            if (left < 0) {
                if (STATS) st.c[ST_T_SPHERE]++;
                float t;
                if (sphere_t(fast[-1 - left], T.ray, 0.001f, T.te, t)) take(t, -1 - left);
            } else {
                if (STATS) st.c[ST_NODES]++;
                const float4 nb = nodes_b[left];
                pl = node_pass_cons<SAH_DQ>(nodes_a[left], nb, make_float2(sah_k, nb.w), T.ray, rp, 0.001f, T.te, el);
                lc = __float_as_int(nb.z);
            }
            if (right < 0) {
                if (STATS) st.c[ST_T_SPHERE]++;
                float t;
                if (sphere_t(fast[-1 - right], T.ray, 0.001f, T.te, t)) take(t, -1 - right);
            } else {
                if (STATS) st.c[ST_NODES]++;
                const float4 nb = nodes_b[right];
                pr = node_pass_cons<SAH_DQ>(nodes_a[right], nb, make_float2(sah_k, nb.w), T.ray, rp, 0.001f, T.te, er);
                rc = __float_as_int(nb.z);
            }
            if (pl && pr) {
                const bool lf = el <= er;
                stack[(T.sp++) * RTW_BLOCK] = (StackEntry)(lf ? rc : lc);
                T.node = lf ? lc : rc;
            } else if (pl || pr) {
                T.node = pl ? lc : rc;
            } else {
                pop();
            }
        } else if (T.phase == ACT && T.node >= 0) {
            if (STATS) st.c[ST_NODES]++;
            const float4 na = nodes_a[T.node];
            const float4 nb = nodes_b[T.node];
            const float2 km = nkm[T.node];
            float entry;
            if (TM == TM_SAH ? node_pass_cons<SAH_DQ>(na, nb, km, T.ray, rp, 0.001f, T.te, entry)
                             : node_pass<FAST_ONLY>(na, nb, km, T.ray, rp, 0.001f, T.te)) {
                if (STATS) db[DB_PASS_LANES]++;
                const int32_t lbits = __float_as_int(nb.z);
                const int32_t left = lbits >> 2;
                const int axis = lbits & 3;
                const int32_t right = __float_as_int(nb.w);
                bool fwd = __builtin_amdgcn_ubfe((uint32_t)T.fast, (uint32_t)axis, 1u) != 0u;  // ray.d[axis] > 0
                // SAH walk: a leaf child first (its hit shrinks te before the sibling subtree; suzanne
                // +2.2 %, profiles/r02/v9_two_child_ab.txt)
                if (TM == TM_SAH && (left < 0) != (right < 0)) fwd = left < 0;
                // hit_index_list order: near subtree, then far (triangle / rect worlds keep leaf steps:
                // testing leaf children inside this step cost suzanne 17 %, profiles/r03/v10_unroll_c1_ab.txt)
                // (a node whose children are both leaves standing on the pair, one leaf step testing both:
                // suzanne -5.8 %, cornell_cube -11.6 %, profiles/r04/v17_leaf_pairs_ab.txt)
                stack[(T.sp++) * RTW_BLOCK] = (StackEntry)(fwd ? right : left);
                T.node = fwd ? left : right;
            } else if (T.sp == 0) {
                T.phase = PH_SHADE;
            } else {
                pop();
            }
        }
        }
    }
    if (STATS) {
        for (int i = 0; i < DB_SHADE_CALLS; ++i)
            if (db[i]) atomicAdd(&dbg[i], (unsigned long long)db[i]);
        T.n_nodes = st.c[ST_NODES];
        T.n_sph_rect = st.c[ST_T_SPHERE] | (st.c[ST_T_RECT] << 16);
        T.n_box_tri = st.c[ST_T_BOX] | (st.c[ST_T_TRI] << 16);
    }
    return T;
}

// The frame's drain (§5.7): once the queues are empty a wave's last paths run alone, and a path
// trapped inside suzanne's mesh walks nearly every node and triangle on each of its ~50 bounces
// (~15 ms on one lane, the 8-GPU shares' tail).  When at most coop_max lanes are still live, each
// SAH ray of the wave is traced by all 64 lanes instead: lane i tests leaves i, i+64, ... with the
// walk's own leaf tests at te = inf, and a wave reduction takes the smallest root.  That is the
// walk's answer (§5.5 step 1: the walk keeps the smallest root over all leaves, and a leaf's first
// root in [ts, te) is its first root in [ts, inf) whenever that lies below te), and a second leaf
// with exactly that root makes a tie.  Plain spheres, rects and triangles only (LK <= LK_PLAIN).
// The lane's ray leaves in PH_SHADE with te = succ(t), ready for the proof step that follows the walk.
// Ties are resolved here: the reference takes the tied leaf its DFS visits first (hittable.rs:453-460:
// te narrows to t, and an equal root is not inside the narrowed range), and it does visit that leaf
// when the leaf's proof box passes at succ(t) -- before it, te > t as no smaller root exists.  So the
// tied leaf first in DFS order (leaf_key) is returned without the tie flag, and the proof step
// decides as for any hit; a lane holding two tied leaves keeps the flag (re-traced on the reference
// tree).  Rays of `todo` only (SAH rays: RTW_TF_SAH).  `audit` (tests only, RTW_COOP_AUDIT=1) takes
// the DFS-last tied leaf instead: wrong images, which shows that the resolution decides them.
// one ray of the cooperative trace, the same in every lane
struct CRay {
    Ray r;
    V3 inv;
    int32_t sgn;  // Trav.fast: bits 0-2 ray.d[axis] > 0
};
// the wave's answer for it (wave-uniform): the closest leaf (-1: none), te = succ(its t) as take()
// leaves it, and whether the tie flag stays
struct CHit {
    int32_t found;
    float te;
    bool tie;
};
template <int LDS, int LK>
__device__ __forceinline__ CHit coop_solve(const DWorld& w, const CRay& a, int32_t n_nodes, int32_t n_leaves,
                                           int32_t n_rects, int32_t fast_off, int32_t tri_prefix, int32_t tri_stride,
                                           bool audit) {
    constexpr bool LDS_SCENE = LDS >= 1;
    // the SAH tree's LDS scene: plain-sphere worlds have no cull-constant section; the leaf records start
    // at leaf tri_prefix (fast_off is leaf 0's would-be offset, walk_leaf_record)
    const int32_t rect_off = 2 * n_nodes + n_leaves - tri_prefix + (LK == LK_SPHERES ? 0 : (n_nodes + 1) / 2);
    const int32_t tri_off = rect_off + 2 * n_rects;
    const float4* rects = LDS_SCENE ? smem + rect_off : uniform_ptr(w.rects);
    const float4* tri_fast = LDS == 2 && LDS_SCENE ? smem + tri_off : uniform_ptr(w.tri_fast);
    const float4* fast = LDS_SCENE ? smem + fast_off : uniform_ptr(w.leaf_fast);
    const int lane = threadIdx.x & 63;
    const uint4* keys = uniform_ptr(w.leaf_key);
    // each lane's best leaf so far, and how many of its leaves reported exactly that t
    float best = F32_INF;
    int32_t bl = -1;
    uint32_t cnt = 0;
    auto keep = [&](bool hit, float t, int32_t leaf) {
        if (hit) {
            cnt = t == best ? cnt + 1 : t < best ? 1u : cnt;
            bl = t < best ? leaf : bl;
            best = t < best ? t : best;
        }
    };
    // a leaf's first root in [ts, te) with te = succ(the lane's best so far): a root beyond the lane's best
    // cannot change the lane's answer, and one equal to it still counts (ties); the triangle test then
    // stops at t for most leaves and reads its record's second half only for closer ones
    // (two rays per pass over the leaves, sharing the record reads, lost 2.4 % on suzanne and 3.7 % on
    // cornell_cube to spills: profiles/r04/v10_coop_ab.txt)
    // software-pipelined: the next leaf record is read before this leaf's test, so that its LDS
    // latency overlaps the triangle / rect record read that depends on this one (one round trip per
    // leaf instead of two; the drain's rays are latency-bound)
    float4 sph_n = lane < n_leaves ? walk_leaf_record<LK>(fast, lane, tri_prefix) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int32_t leaf = lane; leaf < n_leaves; leaf += 64) {
        const float4 sph = sph_n;
        if (leaf + 64 < n_leaves) sph_n = walk_leaf_record<LK>(fast, leaf + 64, tri_prefix);
        float t;
        const float te = best < F32_INF ? __int_as_float(__float_as_int(best) + 1) : F32_INF;
        if (LK == LK_SPHERES || sph.w == sph.w) {
            keep(sphere_t(sph, a.r, 0.001f, te, t), t, leaf);
        } else if (LK >= LK_PLAIN && __float_as_int(sph.x) == 2) {
            const int ri = __float_as_int(sph.y);
            const float4 ra = rects[2 * ri], rb = rects[2 * ri + 1];
            const RectG g{__float_as_int(rb.y), ra.x, ra.y, ra.z, ra.w, rb.x};
            keep(rect_t_mk(g, a.r, a.inv, 0.001f, te, t), t, leaf);  // SAH rays are Markstein-exact
        } else {
            const int ti = __float_as_int(sph.y);
            keep(tri_test(LDS == 2 ? load_tri_soa(tri_fast, ti, tri_soa_stride<LK>(tri_stride)) : load_tri(tri_fast, ti), a.r,
                          0.001f, te, t),
                 t,
                 leaf);
        }
    }
    // the wave's answer: the smallest root, its leaf, the tie resolution
    float m = best;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) m = rtw_minr(m, __shfl_xor(m, k));
    const unsigned long long at = __ballot(bl >= 0 && best == m);
    bool tie = __ballot(bl >= 0 && best == m && cnt >= 2) != 0;
    int win = at ? __ffsll((long long)at) - 1 : 0;
    if (__popcll(at) >= 2) {  // one tied leaf per lane: the first in the reference's DFS order
        if (keys) {
            uint32_t k = 0xFFFFFFFFu;
            if ((at >> lane) & 1) {
                const uint4 q = keys[bl];
                // bit = side XOR (the right child is visited first: ray.d[axis] <= 0)
                k = q.x ^ ((a.sgn & 1) ? 0u : q.y) ^ ((a.sgn & 2) ? 0u : q.z) ^ ((a.sgn & 4) ? 0u : q.w);
                if (audit) k = ~k;
            }
            uint32_t km = k;
#pragma unroll
            for (int j = 1; j < 64; j <<= 1) km = min(km, (uint32_t)__shfl_xor((int)km, j));
            win = __ffsll((long long)__ballot(((at >> lane) & 1) && k == km)) - 1;
        } else {
            tie = true;
        }
    }
    CHit h;
    h.found = at ? __shfl(bl, win) : -1;
    h.te = h.found >= 0 ? __int_as_float(__float_as_int(m) + 1) : F32_INF;
    h.tie = tie;
    return h;
}
// a lane's traversal state after coop_solve answered its ray
__device__ __forceinline__ void coop_apply(Trav& T, int32_t found, float te, bool tie) {
    T.found = found;
    T.te = te;
    T.fast = tie ? (T.fast | RTW_TF_TIE) : (T.fast & ~RTW_TF_TIE);
    T.sp = 0;
    T.phase = PH_SHADE;
}
// The drain shared by the block's waves (§5.7).  coop_solve alone leaves each wave with its own
// drained rays: one wave of a block may still trace hundreds of them (suzanne's 8-GPU shares: up to
// 6.7 ms after the queues ran dry) while its 15 neighbours have finished.  Instead, a wave whose lanes
// all trace in the drain posts its rays to a mailbox in LDS; the owner traces the posts nobody has taken
// yet (from its own lanes), and every wave of the block with no live lane left (a helper, after the
// main loop) takes posted rays and traces them (from the posts) -- both with coop_solve, one answer each.
// Mailbox of wave v: state[v] = gen << 16 | total << 8 | next (rays [next, total) not yet taken; a
// take is a CAS next -> next + 1), done[v] counts the answered rays, and `live` the block's waves that
// still have a live lane.  The rays themselves sit in the owner's traversal-stack columns (free then:
// no lane of the wave is inside a walk), 64 B each: {o, time} {d, fast bits} {inv, -} {answer}.
// Progress: a helper never waits while holding a taken ray, the owner waits only for rays taken by
// others, and a helper leaves once `live` is 0 (each wave decrements it once, on its way to helping).
#define RTW_MB_WORDS 36  // state[16], done[16], live, the drain counters (rtw_drain_counts) [3] (9 float4)
template <int LDS, int LK>
__device__ __forceinline__ float4* mb_slot(int32_t stack_off, int v, int j) {
    // the stack's entry size (traverse's StackEntry): a wave's 64 entries of one level hold ES rays
    constexpr int ES = stack_entry_bytes(LDS, LK);
    return smem + stack_off + (j / ES) * (RTW_BLOCK * ES / 16) + v * (64 * ES / 16) + (j % ES) * 4;
}
// the owner's take of its own next post (wave-uniform); false: all taken
__device__ __forceinline__ bool mb_take_own(uint32_t* mb, int v, int& j) {
    const int lane = threadIdx.x & 63;
    for (;;) {
        const uint32_t s = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)__hip_atomic_load(&mb[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if ((s & 0xFFu) >= ((s >> 8) & 0xFFu)) return false;
        uint32_t expect = s;
        bool ok = false;
        if (lane == 0)
            ok = __hip_atomic_compare_exchange_strong(&mb[v], &expect, s + 1, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__builtin_amdgcn_readfirstlane((int)ok)) {
            j = (int)(s & 0xFFu);
            return true;
        }
    }
}
// a post's answer (one lane): into its slot, then counted (release)
__device__ __forceinline__ void mb_answer(uint32_t* mb, float4* q, int u, const CHit& h) {
    q[3] = make_float4(__int_as_float(h.found), h.te, h.tie ? 1.0f : 0.0f, 0.0f);
    __hip_atomic_fetch_add(&mb[16 + u], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// one wave-uniform take: the first mailbox from wave v0 on with a ray not yet taken; -1: none
__device__ __forceinline__ int mb_take(uint32_t* mb, int v0, int& j) {
    const int lane = threadIdx.x & 63;
    constexpr int NW = RTW_BLOCK / 64;
    for (;;) {
        const int u = (v0 + lane) % NW;
        const uint32_t s = lane < NW ? __hip_atomic_load(&mb[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0u;
        const unsigned long long open = __ballot(lane < NW && (s & 0xFFu) < ((s >> 8) & 0xFFu));
        if (open == 0) return -1;
        const int i = __ffsll((long long)open) - 1;
        const int uu = (v0 + i) % NW;
        const uint32_t si = (uint32_t)__builtin_amdgcn_readlane((int)s, i);
        uint32_t expect = si;
        bool ok = false;
        if (lane == 0)
            ok = __hip_atomic_compare_exchange_strong(&mb[uu], &expect, si + 1, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__builtin_amdgcn_readfirstlane((int)ok)) {
            j = (int)(si & 0xFFu);
            return uu;
        }
    }
}

template <bool STATS, int LDS, int LK, int TX, bool GEN, bool WP>
__device__ __forceinline__ void render_body(const KArgs& A) {
    constexpr bool LDS_SCENE = LDS >= 1;
    // LDS: [scene: nodes (2 float4 each), leaf records (1 float4 each), cull constants (1 float2
    // per node)] [stack: depth x BLOCK]
    const DWorld& w = A.w;
    // SAH path (§5.6): worlds of plain spheres / triangles only; in the counting variant only when
    // asked for the product kernel's own traversal (stats_tree 1; else the reference's statistics)
    constexpr bool SAHK = LK <= LK_WRAPPED;
    const bool sah = SAHK && A.sah != 0;
    if (LDS_SCENE) {
        const float4* ga = sah ? w.sah_a : w.node_a;
        const float4* gb = sah ? w.sah_b : w.node_b;
        for (int i = threadIdx.x; i < A.node_count; i += RTW_BLOCK) {
            smem[i] = ga[i];
            smem[A.node_count + i] = gb[i];
        }
        // the leaf records from leaf tri_prefix on (walk_leaf_record)
        const int32_t n_rec = A.leaf_count - A.tri_prefix;
        for (int i = threadIdx.x; i < n_rec; i += RTW_BLOCK) smem[2 * A.node_count + i] = w.leaf_fast[A.tri_prefix + i];
        // the cull constants (the plain-sphere worlds' SAH tree keeps them in its node records)
        const bool km_rec = sah && LK == LK_SPHERES;
        const int32_t km_f4 = km_rec ? 0 : (A.node_count + 1) / 2;
        float2* km = reinterpret_cast<float2*>(smem + 2 * A.node_count + n_rec);
        const float2* gk = sah ? w.sah_km : w.node_km;
        if (!km_rec)
            for (int i = threadIdx.x; i < A.node_count; i += RTW_BLOCK) km[i] = gk[i];
        float4* rects = smem + 2 * A.node_count + n_rec + km_f4;
        for (int i = threadIdx.x; i < 2 * A.rect_count; i += RTW_BLOCK) rects[i] = w.rects[i];
        if (LDS == 2) {
            float4* tris = rects + 2 * A.rect_count;
            for (int i = threadIdx.x; i < 4 * A.tri_count; i += RTW_BLOCK) tris[(i & 3) * A.tri_stride + (i >> 2)] = w.tri_fast[i];
        }
        if (A.sh_li >= 0) {  // shading tables (launch_render decides whether they fit)
            int4* li = reinterpret_cast<int4*>(smem + A.sh_li);  // from leaf tri_prefix on (leaf_info_of)
            for (int i = A.tri_prefix + threadIdx.x; i < A.leaf_count; i += RTW_BLOCK) li[i] = w.leaf_info[i];
            int4* mt = reinterpret_cast<int4*>(smem + A.sh_mat);
            for (int i = threadIdx.x; i < A.material_count; i += RTW_BLOCK) mt[i] = w.materials[i];
            if (A.sh_box >= 0)
                for (int i = threadIdx.x; i < 2 * A.leaf_count; i += RTW_BLOCK) smem[A.sh_box + i] = w.leaf_box[i];
            if (A.sh_xf >= 0) {
                for (int i = threadIdx.x; i < 3 * A.leaf_count; i += RTW_BLOCK) smem[A.sh_xf + i] = w.leaf_xf[i];
                for (int i = threadIdx.x; i < A.sphere_count; i += RTW_BLOCK) smem[A.sh_sph + i] = w.spheres[i];
                for (int i = threadIdx.x; i < 2 * A.box_count; i += RTW_BLOCK) smem[A.sh_bx + i] = w.boxes[i];
            }
            if (A.sh_tex0 >= 0) {
                int4* tx = reinterpret_cast<int4*>(smem + A.sh_tex0);
                if constexpr (TX == TX_SOLID || GEN) {  // (the GEN kernels: -1, no table)
                    for (int i = threadIdx.x; i < A.texture_count; i += RTW_BLOCK) tx[i] = w.textures[3 * i];
                } else {  // all three records
                    for (int i = threadIdx.x; i < 3 * A.texture_count; i += RTW_BLOCK) tx[i] = w.textures[i];
                }
            }
        }
        if (A.mb_off >= 0 && threadIdx.x < RTW_MB_WORDS)  // the shared drain's mailbox (mb_slot): live = all waves
            reinterpret_cast<uint32_t*>(smem + A.mb_off)[threadIdx.x] = threadIdx.x == 32 ? RTW_BLOCK / 64 : 0u;
        __syncthreads();
    }
    // the traversal stacks follow the LDS scene and the shading tables
    const int32_t stack_off = LDS_SCENE ? A.stack_off : 0;
    // the generic tables only where the world's leaf kinds can read them (compile-time -1 elsewhere: their
    // offsets would otherwise occupy SGPRs across the bounce loop, which spills -- suzanne -3 %)
    ShadeTabsT<GEN, LDS_SCENE && LK >= LK_PLAIN, LK == LK_TRIS> stabs{
        A.sh_li, A.sh_mat, A.sh_tex0, A.sh_li >= 0 ? A.fast_off : -1,
        GEN ? A.sh_xf : -1, GEN ? A.sh_sph : -1, GEN ? A.sh_bx : -1,
        LDS_SCENE && LK >= LK_PLAIN ? A.sh_rect : -1,
        LK == LK_TRIS ? A.tri_prefix : 0, A.tri_prefix_mat, A.tri_prefix_w};
    // the shading tables' offsets in VGPRs: as SGPRs they are live across the bounce loop and spill
    asm volatile("" : "+v"(stabs.li), "+v"(stabs.mat), "+v"(stabs.tex0), "+v"(stabs.fast));
    if (LK == LK_TRIS) asm volatile("" : "+v"(stabs.pre), "+v"(stabs.pre_mat), "+v"(stabs.pre_w));
    Stats st;
    if (STATS)
        for (int i = 0; i < ST_COUNT; ++i) st.c[i] = 0;
    const int lane = threadIdx.x & 63;

    // Per-lane state machine.  Work items (a slot and a run of `chunk` consecutive samples) come
    // from a queue (wave-aggregated atomics), chunk-major so that a wave's lanes share a tile;
    // each finished sample's colour is stored and accumulate_kernel adds them per pixel in
    // sample order (the reference's sequential .sum(), rendering.rs:172-179).
    uint32_t pix = 0, slot = 0;
    float fx = 0.0f, fy = 0.0f;
    uint32_t sample = 0, sample_end = 0;
    float pdot = 0.0f;  // dot((0,1,0), primary ray direction): the background's argument
    V3 att = v3(1.0f, 1.0f, 1.0f), acc = v3(0.0f, 0.0f, 0.0f);
    V3 psum = v3(0.0f, 0.0f, 0.0f);  // whole-pixel items: the pixel's running sum
    uint32_t pcost = 0;               // ... and its deep paths' bounces (one atomic per pixel, not per path)
    int32_t depth = 0;
    Trav T;
    T.phase = PH_PIXEL;
    T.n_nodes = 0;
    T.n_sph_rect = 0;
    T.n_box_tri = 0;
    T.node = 0;
    T.sp = 0;
    T.te = F32_INF;
    T.found = -1;
    bool fresh = false;  // T.ray is new: the traversal state must be initialised
    uint64_t c_mark = STATS ? clock64() : 0;  // execution-time split (counting variant only)

    // rendering.rs:174-176: jitter (x then y), then Camera::ray
    auto start_sample = [&](int back) {
        (void)back;
        RTW_PT(5);
        T.rng = rtw_sample_stream(A.seed_key, pix, sample);
        const float jx = d_uniform_sample(A.ux, &T.rng);
        const float jy = d_uniform_sample(A.uy, &T.rng);
        T.ray = camera_ray(w.wc->cam, T.rng, fx + jx, fy + jy);
        pdot = dot(v3(0.0f, 1.0f, 0.0f), T.ray.d);  // background_color.rs:13 on the primary ray
        att = v3(1.0f, 1.0f, 1.0f);
        acc = v3(0.0f, 0.0f, 0.0f);
        depth = A.max_depth;
        fresh = true;
        RTW_PT(back);
    };

    int32_t trace_min = A.trace_min;  // this wave's dynamic-fetch threshold (tuned below)
    bool tuned = true;
    if (A.tune) {
        const int ch = __hip_atomic_load(&A.tune->chosen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ch > 0) trace_min = ch;
        else tuned = A.tune_items == 0;
    }
    // This wave's reserve of work items [w_next, w_end), in the local index space of its queue wq,
    // taken from the queue's counter in batches (one global atomic per batch, not per refill round);
    // batches shrink toward the end of the launch so that the last items still spread over all
    // waves.
    uint64_t w_next = 0, w_end = 0;
    uint32_t wq = (blockIdx.x * (RTW_BLOCK / 64) + (threadIdx.x >> 6)) % RTW_QUEUES;
    uint32_t qfail = 0;           // consecutive queues found empty: RTW_QUEUES of them end the launch
    unsigned long long pf_b = 0;  // the prefetched batch's base, in lane pf_lane (its atomic's result)
    uint64_t pf_size = 0;         // its size; 0: none in flight
    int pf_lane = 0;
    auto prefetch = [&](int leader) {  // wave-uniform
        const uint64_t rest = A.q_cap > w_end ? A.q_cap - w_end : 0;
        // small batches while the costly tiles are handed out: a wave slowed by long paths must not
        // sit on a large reserve of them (an 8-GPU suzanne rank: 2.4x at 256)
        const uint64_t cap = w_end * RTW_QUEUES >= A.big_from ? RTW_WAVE_BATCH_BIG : RTW_WAVE_BATCH;
        pf_size = max((uint64_t)1, min(cap, (uint64_t)fdiv((uint32_t)rest, A.fd_spread)));
        if (lane == leader) pf_b = atomicAdd(A.queue + wq * RTW_QSTRIDE, (unsigned long long)pf_size);
        pf_lane = leader;
    };
    RTW_PT_DECL
#ifdef RTW_WAVE_TIMING
    uint32_t wx_busy = 0, wx_n = 0, wx_sum = 0, wx_max = 0, wx_coop = 0, wx_ref = 0;
    uint64_t wx_tref = 0, wx_tsah = 0, wx_tcoop = 0;
    bool wx_dry = false;
#endif
    // the shared drain (mb_slot): worlds whose drained rays coop_solve traces, LDS modes 1 and 2
    // (its mailbox offset in a VGPR, read per use: a value live across the walk in an SGPR spills)
    // Worlds of plain spheres and triangles only (leaf kinds 1: meshes that trap paths); elsewhere the
    // code cost more than the drain gained (final_scene1 -0.8 %, cornell_cube -0.6 % with the same 8-way
    // shares: profiles/r05/ab_shared_drain.txt, r5q_part8_coop.txt)
    // whole-pixel work items (KArgs::whole_pixel) as a compile-time property of the variant: a kernel for
    // single-sample items carries no whole-pixel code (its SGPR spills 65 -> 56 on final_scene1: +0.4-0.8 %,
    // suzanne +0.4 %, cornell_cube +0.9 %, profiles/r06/ab_whole_pixel.txt).  The GEN kernels keep the run-time
    // choice (their WP = false variant serves both): as a template argument their spill layout cost C5 the
    // 1.2-1.9 % its texture change had gained (ab_whole_pixel.txt, r6e)
    static_assert(!(GEN && WP), "GEN kernels take whole-pixel items at run time");
    const bool WPX = GEN ? A.whole_pixel != 0 : WP;
    constexpr bool SHARE_K = !STATS && LDS_SCENE && LK == LK_TRIS;
    int32_t mb_v = SHARE_K ? A.mb_off : -1;
    asm volatile("" : "+v"(mb_v));
    auto share_on = [&]() { return SHARE_K && __builtin_amdgcn_readfirstlane(mb_v) >= 0; };
    auto mailbox = [&]() { return reinterpret_cast<uint32_t*>(smem + __builtin_amdgcn_readfirstlane(mb_v)); };
    for (;;) {
        if (__ballot(T.phase != PH_DONE) == 0) break;  // wave-uniform: every lane is done
        // 1. lanes without a pixel take the next items of the wave's reserve
        RTW_PT(1);
        for (;;) {
            const unsigned long long m = __ballot(T.phase == PH_PIXEL);
            if (m == 0) break;
            if (qfail >= RTW_QUEUES) {  // wave-uniform: every queue is empty
#ifdef RTW_WAVE_TIMING
                {
                    const uint32_t wv_ = (blockIdx.x * RTW_BLOCK + threadIdx.x) / 64;
                    if (wv_ < 8192) atomicMin(&rtw_wave_dry[wv_], (unsigned long long)wall_clock64());
                }
#endif
#ifdef RTW_WAVE_TIMING
                if (!wx_dry) wx_busy = (uint32_t)__popcll(__ballot(T.phase != PH_PIXEL));
                wx_dry = true;
#endif
                if (T.phase == PH_PIXEL) T.phase = PH_DONE;
                continue;
            }
            const int leader = __ffsll((long long)m) - 1;
            const uint64_t need = (uint64_t)__popcll(m);
            bool empty = false, took = false;
            if (w_next == w_end) {  // reserve used up: take the prefetched batch (fetch one if none)
                if (pf_size == 0) prefetch(leader);
                const uint64_t base =
                    ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pf_b >> 32), pf_lane) << 32) |
                    (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pf_b, pf_lane);
                const uint64_t size = pf_size;
                pf_size = 0;
                took = true;
                empty = base >= A.q_cap;
                w_next = empty ? A.q_cap : base;
                w_end = empty ? A.q_cap : min(base + size, A.q_cap);
                if (!tuned && wq == 0 && !empty) {  // wave-uniform; queue 0's batch holding a half-epoch's
                    // first item (global position ~ local x RTW_QUEUES) stamps its start
                    const uint64_t H = A.fd_half.d;
                    const uint64_t g0 = base * RTW_QUEUES, g1 = (base + size) * RTW_QUEUES;
                    const uint64_t j = fdiv((uint32_t)min(g0 + H - 1, (uint64_t)0xFFFFFFFFu), A.fd_half);
                    if (lane == leader && j >= 1 && j <= RTW_TUNE_STAMPS && j * H < g1)
                        __hip_atomic_store(&A.tune->tb[j - 1], wall_clock64(), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            const uint64_t left = min(need, w_end - w_next);  // the first `left` lanes get an item
            const uint64_t first = w_next;
            w_next += left;
            if (!tuned) {  // wave-uniform: the epoch of the items being handed out
                const uint64_t e = fdiv((uint32_t)min(w_next * RTW_QUEUES, (uint64_t)0xFFFFFFFFu), A.fd_epoch);
                if (e == 0) {
                    trace_min = A.trace_min;
                } else if (e <= RTW_TUNE_EPOCHS) {
                    const int i = (int)e - 1;
                    trace_min = kTuneCand[i < RTW_TUNE_NCAND ? i : RTW_TUNE_EPOCHS - 1 - i];
                } else {
                    // epoch e's timed second half: items [(2e+1)H, (2e+2)H) = tb[2e+1] - tb[2e].  Four
                    // stamps at a time (an array of all 34 stamps was the kernel's register peak)
                    const unsigned long long* tbp = A.tune->tb;
                    auto stamp = [&](int k) {
                        return __hip_atomic_load(&tbp[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    };
                    bool ok = stamp(0) != ~0ull && stamp(1) != ~0ull;
                    unsigned long long best_t = 0;
                    int best = A.trace_min;
#pragma nounroll
                    for (int c = 0; c < RTW_TUNE_NCAND; ++c) {
                        const int e1 = c + 1, e2 = RTW_TUNE_EPOCHS - c;
                        const unsigned long long a0 = stamp(2 * e1), a1 = stamp(2 * e1 + 1), b0 = stamp(2 * e2),
                                                 b1 = stamp(2 * e2 + 1);
                        ok = ok && a0 != ~0ull && a1 != ~0ull && b0 != ~0ull && b1 != ~0ull;
                        const unsigned long long t = (a1 - a0) + (b1 - b0);
                        if (c == 0 || t < best_t) {
                            best_t = t;
                            best = kTuneCand[c];
                        }
                    }
                    trace_min = A.trace_min;
                    if (ok) {
                        trace_min = best;
                        if (lane == leader) atomicCAS(&A.tune->chosen, 0, trace_min);
                        tuned = true;
                    }
                }
            }
            if (T.phase == PH_PIXEL) {
                const unsigned long long below = (lane == 0) ? 0ull : (m & (~0ull >> (64 - lane)));
                const uint64_t r = (uint64_t)__popcll(below);
                const uint64_t loc = first + r;
                // queue wq's local item -> the launch's item (granule loc / QGRAN of queue wq)
                const uint64_t item = ((loc / RTW_QGRAN) * RTW_QUEUES + wq) * RTW_QGRAN + loc % RTW_QGRAN;
                if (r >= left || item >= A.items) {
                    // nothing for this lane in this round: the reserve is used up (the next round takes
                    // the next batch) or a padding index of the last granule row
                } else {
                    const bool big = item < A.items_big;
                    const uint32_t rel = (uint32_t)(big ? item : item - A.items_big);  // < 2^32
                    uint32_t ck, c, lt, it;
                    if (A.tile_perm) {  // tile-major in cost order: tile rank, chunk, pixel of the tile
                        const uint32_t g = fdiv(rel, A.fd_rank);
                        const uint32_t wi = rel - g * A.fd_rank.d;
                        ck = fdiv(wi, A.fd_tile);
                        it = wi - ck * A.fd_tile.d;
                        // (a per-lane cache of it: -0.3 %, profiles/r04/v9_proof_lds_ab.txt; the reserve's tiles
                        // read at batch fetch, a wave-uniform cache: within noise, profiles/r05/ab_r5i.txt)
                        lt = A.tile_perm[g];
                        c = lt * A.fd_tile.d + it;
                    } else {  // chunk-major: pass after pass over the slots
                        ck = fdiv(rel, A.fd_total);
                        c = rel - ck * A.total;
                        lt = fdiv(c, A.fd_tile);
                        it = c - lt * A.fd_tile.d;
                    }
                    const uint32_t tile = (uint32_t)A.part_index + lt * (uint32_t)A.part_count;
                    const uint32_t ty = fdiv(tile, A.fd_tiles_x), iy = fdiv(it, A.fd_tile_w);
                    const int32_t px = (int32_t)((tile - ty * (uint32_t)A.tiles_x) * (uint32_t)A.tile_w + (it - iy * (uint32_t)A.tile_w));
                    const int32_t py = (int32_t)(ty * (uint32_t)A.tile_h + iy);
                    if (px < A.width && py < A.height) {  // else: padding slot of an edge tile
                        slot = c;
                        pix = (uint32_t)(py * A.width + px);
                        fx = (float)px * A.sx;  // size2i.rs:52-55
                        fy = (float)py * A.sy;
                        sample = big ? A.s_begin + ck * A.chunk : A.s_split + ck;
                        sample_end = big ? min(sample + A.chunk, A.s_split) : sample + 1;
                        psum = v3(0.0f, 0.0f, 0.0f);
                        pcost = 0;
                        start_sample(1);
                        T.phase = PH_TRACE;
                    }
                }
            }
            if (empty) {  // wave-uniform: queue wq is used up (no batch in flight); try the next one
                wq = (wq + 1) % RTW_QUEUES;
                ++qfail;
                w_next = w_end = 0;
            } else if (took) {
                qfail = 0;
            }
        }

        // 2. a new ray starts at the root (Scene::hit with t_range 0.001..inf, rendering.rs:25)
        RTW_PT(2);
        uint64_t c_trav = 0;
        if (STATS) {
            c_trav = clock64();
            if (lane == __ffsll((long long)__ballot(1)) - 1)
                atomicAdd(&A.stats[ST_COUNT + DB_REST_CYCLES], (unsigned long long)(c_trav - c_mark));
        }
        if (fresh) {
            fresh = false;
            const RayPre rp = ray_pre(T.ray, A.mk_world != 0);
            T.inv = rp.inv;
            T.fast = (rp.fast ? 8 : 0) | (T.ray.d.x > 0.0f ? 1 : 0) | (T.ray.d.y > 0.0f ? 2 : 0) | (T.ray.d.z > 0.0f ? 4 : 0);
            T.node = w.root;
            if (sah) {  // the SAH walk needs the exact fast division; other rays take the reference tree
                if (rp.fast) {
                    T.node = LK == LK_SPHERES ? w.sah_root_c2 : w.sah_root;
                    T.fast |= RTW_TF_SAH;
                } else {
                    T.phase = PH_REF;
                }
            }
            T.sp = 0;
            T.te = F32_INF;
            T.found = -1;
            if (STATS) st.c[ST_RAYS]++;
        }

        // 3. traversal (hittable.rs:429-473)
        RTW_PT(3);
        // (almost) every ray is Markstein-exact: such calls run a loop without the true-division
        // path (wave-uniform choice per call)
        if (sah) {
            // the drain: the walk stops when at most coop_max lanes still trace, and those rays (the
            // long walks) are traced by the whole wave (coop_solve); wave-uniform condition
            const bool dry_coop = !STATS && LK <= LK_PLAIN && qfail >= RTW_QUEUES && A.coop_max > 0;
#ifdef RTW_WAVE_TIMING
            uint64_t wx_t0 = wall_clock64();
#endif
            T = traverse<STATS, LDS, LK, true, TM_SAH>(A.wdev, stabs, T, __builtin_amdgcn_readfirstlane(trace_min), A.node_count,
                                                       A.leaf_count, A.rect_count, A.tri_prefix, A.tri_stride, stack_off,
                                                       STATS ? A.stats + ST_COUNT : nullptr, dry_coop ? A.coop_max : -1);
            // the rays coop_solve takes (one call site, inlined: as an out-of-line call taking and
            // returning Trav by value it cost 304 B of scratch per lane, saved and restored around
            // every call -- suzanne's and cornell_cube's extra write traffic): the drain's last rays
            unsigned long long coop = 0;
            if (dry_coop) {
                const unsigned long long tm = __ballot(T.phase == PH_TRACE);
#ifdef RTW_WAVE_TIMING
                if (tm != 0 && (uint32_t)__popcll(tm) <= (uint32_t)A.coop_max) wx_coop += (uint32_t)__popcll(tm);
                const uint64_t wx_tc = wall_clock64();
                wx_tsah += wx_tc - wx_t0;  // the walk part
                wx_t0 = wx_tc;
#endif
                if (tm != 0 && (uint32_t)__popcll(tm) <= (uint32_t)A.coop_max) coop = tm;
            }
            // ... and the walk's tied rays: coop_solve finds every tied leaf and keeps the reference's
            // (its DFS-first); a drained ray is traced once and leaves with its own ties resolved
            if (!STATS && LK <= LK_PLAIN && A.coop_ties)
                coop |= __ballot(T.phase == PH_SHADE && (T.fast & (RTW_TF_SAH | RTW_TF_TIE)) == (RTW_TF_SAH | RTW_TF_TIE));
            // ... shared with the block's finished waves when no lane of this wave is inside a walk (the rays
            // go to the stack columns): the mailbox, mb_slot
            const bool own = share_on() && dry_coop && coop != 0 && (__ballot(T.phase == PH_TRACE) & ~coop) == 0;
            const bool in = (coop >> lane) & 1;
            const uint32_t post_j = (uint32_t)__popcll(coop & ((1ull << lane) - 1));  // the lane's ray, in order
            const uint32_t post_k = own ? min((uint32_t)__popcll(coop), (uint32_t)A.mb_cap) : 0u;
            if (own) {
                uint32_t* mb = mailbox();
                const int v = threadIdx.x >> 6;
                if (in && post_j < post_k) {
                    float4* q = mb_slot<LDS, LK>(stack_off, v, (int)post_j);
                    q[0] = make_float4(T.ray.o.x, T.ray.o.y, T.ray.o.z, T.ray.time);
                    q[1] = make_float4(T.ray.d.x, T.ray.d.y, T.ray.d.z, __int_as_float(T.fast));
                    q[2] = make_float4(T.inv.x, T.inv.y, T.inv.z, 0.0f);
                } else if (in && T.phase == PH_TRACE) {  // beyond the mailbox: the walk starts over (its stack is gone)
                    T.node = LK == LK_SPHERES ? w.sah_root_c2 : w.sah_root;
                    T.sp = 0;
                    T.te = F32_INF;
                    T.found = -1;
                    T.fast &= ~RTW_TF_TIE;
                }
                if (lane == 0) {  // the batch's rays are written (release): open it
                    __hip_atomic_fetch_add(&mb[33], post_k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    const uint32_t s = __hip_atomic_load(&mb[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_store(&mb[16 + v], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_store(&mb[v], ((((s >> 16) + 1) & 0xFFFFu) << 16) | (post_k << 8), __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                coop = 0;
            }
            // the wave's own rays, one at a time (read from their lanes): `coop`, or this wave's posts that
            // no helper has taken yet (a take as the helpers'); every answer of a post goes to its slot
            if (!STATS && LK <= LK_PLAIN && (coop || own)) {
                uint32_t* mb = mailbox();
                const int v = threadIdx.x >> 6;
                for (;;) {  // wave-uniform
                    int src, j = 0;
                    if (own) {
                        if (!mb_take_own(mb, v, j)) break;
                        src = __ffsll((long long)__ballot(in && post_j == (uint32_t)j)) - 1;
                    } else {
                        if (!coop) break;
                        src = __ffsll((long long)coop) - 1;
                        coop &= coop - 1;
                    }
                    CRay a;
                    a.r.o = v3(__shfl(T.ray.o.x, src), __shfl(T.ray.o.y, src), __shfl(T.ray.o.z, src));
                    a.r.d = v3(__shfl(T.ray.d.x, src), __shfl(T.ray.d.y, src), __shfl(T.ray.d.z, src));
                    a.r.time = __shfl(T.ray.time, src);
                    a.inv = v3(__shfl(T.inv.x, src), __shfl(T.inv.y, src), __shfl(T.inv.z, src));
                    a.sgn = __shfl(T.fast, src);
                    const CHit h = coop_solve<LDS, LK>(w, a, A.node_count, A.leaf_count, A.rect_count, A.fast_off,
                                                       A.tri_prefix, A.tri_stride, A.coop_ties == 2);
                    if (!own) {
                        if (lane == src) coop_apply(T, h.found, h.te, h.tie);
                    } else if (lane == 0) {
                        mb_answer(mb, mb_slot<LDS, LK>(stack_off, v, j), v, h);
                        __hip_atomic_fetch_add(&mb[35], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                if (own) {  // the posts others took: wait for their answers, then every posted lane takes its own
                    while ((uint32_t)__builtin_amdgcn_readfirstlane((int)__hip_atomic_load(
                               &mb[16 + v], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) < post_k)
                        __builtin_amdgcn_s_sleep(1);
                    if (in && post_j < post_k) {
                        const float4 r = mb_slot<LDS, LK>(stack_off, v, (int)post_j)[3];
                        coop_apply(T, __float_as_int(r.x), r.y, r.z != 0.0f);
                    }
                }
            }
#ifdef RTW_WAVE_TIMING
            const uint64_t wx_t1 = wall_clock64();
            if (qfail >= RTW_QUEUES) wx_tcoop += wx_t1 - wx_t0;
#endif
            if (STATS) {
                st.c[ST_NODES] += T.n_nodes;
                st.c[ST_T_SPHERE] += T.n_sph_rect & 0xFFFFu;
                st.c[ST_T_RECT] += T.n_sph_rect >> 16;
                st.c[ST_T_BOX] += T.n_box_tri & 0xFFFFu;
                st.c[ST_T_TRI] += T.n_box_tri >> 16;
                T.n_nodes = T.n_sph_rect = T.n_box_tri = 0;
            }
            // §5.5: the SAH walk's closest leaf L (no tie) is the reference's answer when the
            // reference DFS reaches L: the reference's internal boxes are nested (checked at upload)
            // and hit_cond is monotone under box inclusion and in te, so L's parent box passing
            // hit_cond with te = succ(t) proves it.  A miss is a miss for the reference too.
            // Otherwise the ray is traced again on the reference tree.
            if (T.phase == PH_SHADE && (T.fast & RTW_TF_SAH)) {
                bool ok = (T.fast & RTW_TF_TIE) == 0;
#ifdef RTW_SAH_AUDIT_NO_TIE  // audit builds only: shows that the tie test decides images
                ok = true;
#endif
                if (T.found >= 0) {
                    if (STATS) st.c[ST_NODES]++;  // the leaf-box proof reads one 32-B box record
                    const float4 ba = A.sh_box >= 0 ? smem[A.sh_box + 2 * T.found] : w.leaf_box[2 * T.found];
                    const float4 bb = A.sh_box >= 0 ? smem[A.sh_box + 2 * T.found + 1] : w.leaf_box[2 * T.found + 1];
#ifndef RTW_SAH_AUDIT_NO_BOX  // audit builds only: shows that the leaf-box proof decides images
                    ok = ok && box_hit_cond_fast(ba, bb, T.ray, RayPre{T.inv, true}, 0.001f, T.te);
#else
                    (void)ba, (void)bb;
#endif
                    T.te = __int_as_float(__float_as_int(T.te) - 1);  // the closest t
                }
                T.fast &= ~(RTW_TF_SAH | RTW_TF_TIE);
                if (!ok) {
                    T.phase = PH_REF;
                    T.node = w.root;
                    T.sp = 0;
                    T.te = F32_INF;
                    T.found = -1;
                }
            }
#ifdef RTW_WAVE_TIMING
            if (qfail >= RTW_QUEUES) wx_ref += (uint32_t)__popcll(__ballot(T.phase == PH_REF));
            const uint64_t wx_t2 = wall_clock64();
#endif
            if (__ballot(T.phase == PH_REF) != 0)
                T = traverse<STATS, LDS, LK, false, TM_FALLBACK>(A.wdev, stabs, T, 0, A.node_count, A.leaf_count, A.rect_count,
                                                                 A.tri_prefix, A.tri_stride, stack_off,
                                                                 STATS ? A.stats + ST_COUNT : nullptr);
#ifdef RTW_WAVE_TIMING
            if (qfail >= RTW_QUEUES) wx_tref += wall_clock64() - wx_t2;
#endif
        } else if (__ballot(T.phase == PH_TRACE && (T.fast & 8) == 0) == 0) {
            T = traverse<STATS, LDS, LK, true, TM_REF>(A.wdev, stabs, T, __builtin_amdgcn_readfirstlane(trace_min), A.node_count,
                                               A.leaf_count, A.rect_count, A.tri_prefix, A.tri_stride, stack_off,
                                               STATS ? A.stats + ST_COUNT : nullptr);
        } else {
            T = traverse<STATS, LDS, LK, false, TM_REF>(A.wdev, stabs, T, __builtin_amdgcn_readfirstlane(trace_min), A.node_count,
                                                A.leaf_count, A.rect_count, A.tri_prefix, A.tri_stride, stack_off,
                                                STATS ? A.stats + ST_COUNT : nullptr);
        }
        if (STATS) {
            c_mark = clock64();
            if (lane == __ffsll((long long)__ballot(1)) - 1)
                atomicAdd(&A.stats[ST_COUNT + DB_TRAV_CYCLES], (unsigned long long)(c_mark - c_trav));
        }
        if (STATS) {
            st.c[ST_NODES] += T.n_nodes;
            st.c[ST_T_SPHERE] += T.n_sph_rect & 0xFFFFu;
            st.c[ST_T_RECT] += T.n_sph_rect >> 16;
            st.c[ST_T_BOX] += T.n_box_tri & 0xFFFFu;
            st.c[ST_T_TRI] += T.n_box_tri >> 16;
        }

        // 4. shade the lanes whose traversal finished (rendering.rs:19-71)
        RTW_PT(4);
        if (STATS) {
            const unsigned long long sm = __ballot(T.phase == PH_SHADE);
            if (sm && lane == __ffsll((long long)__ballot(1)) - 1) {
                atomicAdd(&A.stats[ST_COUNT + DB_SHADE_CALLS], 1ull);
                atomicAdd(&A.stats[ST_COUNT + DB_SHADE_LANES], (unsigned long long)__popcll(sm));
            }
        }
        if (T.phase == PH_SHADE) {
            if (STATS && T.found >= 0) {
                st.c[ST_H_SPHERE + w.leaf_info[T.found].x]++;
                st.c[ST_MAT]++;
            }
            Path P;
            P.ray = T.ray;
            P.att = att;
            P.acc = acc;
            P.depth = depth;
            P.rng = T.rng;
            const ShadeOut so = shade<STATS, TX>(A.wdev, A.mode, P, T.found, T.te, pdot, stabs);
            T.ray = so.p.ray;
            att = so.p.att;
            acc = so.p.acc;
            depth = so.p.depth;
            T.rng = so.p.rng;
            if (STATS) st.c[ST_TEXEL] += so.texels;
            T.phase = PH_TRACE;
            if (so.done) {
                RTW_PT(7);
                if (WPX) {
                    psum = add(psum, so.color);  // in sample order: this lane renders the pixel's samples in turn
                } else {
                    float* o = A.colors + ((uint64_t)(sample - A.s_begin) * A.total + slot) * 3;
                    o[0] = so.color.x;
                    o[1] = so.color.y;
                    o[2] = so.color.z;
                }
                if (STATS) st.c[ST_SAMPLES]++;
                // deep paths (rare: trapped inside meshes, up to ~100x the mean cost) mark their
                // slot for the next frame's work order
                const int32_t bounces = A.max_depth - depth;
                if (!STATS && A.slot_cost && bounces > 3) {
                    if (WPX) pcost += (uint32_t)bounces;
                    else atomicAdd(&A.slot_cost[slot], (uint32_t)bounces);
                }
#ifdef RTW_WAVE_TIMING
                if (qfail >= RTW_QUEUES) {
                    ++wx_n;
                    wx_sum += (uint32_t)bounces;
                    wx_max = max(wx_max, (uint32_t)bounces);
                }
#endif
                ++sample;
                if (sample >= sample_end) {
                    T.phase = PH_PIXEL;
                    if (WPX) {  // accumulate_kernel's last step, for this pixel
                        if (!STATS && A.slot_cost && pcost) atomicAdd(&A.slot_cost[slot], pcost);
                        const V3 px = divs(psum, (float)A.spp);
                        float* o = A.layout == RTW_LAYOUT_TILES ? A.out + 3 * (size_t)slot : A.out + 3 * (size_t)pix;
                        o[0] = px.x;
                        o[1] = px.y;
                        o[2] = px.z;
                    }
                } else {
                    start_sample(7);
                }
            } else {
                fresh = true;  // the scattered ray continues the path
            }
        }
    }
    // every lane is done: the wave traces the block's posted rays until no wave of the block is live (the
    // poll bound only ends a helper early, never a ray: owners trace their own posts too)
    if (share_on()) {
        uint32_t* mb = mailbox();
        if (lane == 0) __hip_atomic_fetch_add(&mb[32], ~0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        for (uint32_t polls = 0; polls < RTW_MB_POLLS; ++polls) {
            int j = 0;
            const int u = mb_take(mb, threadIdx.x >> 6, j);
            if (u < 0) {
                if (__builtin_amdgcn_readfirstlane(
                        (int)__hip_atomic_load(&mb[32], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) == 0)
                    break;
                __builtin_amdgcn_s_sleep(2);
                continue;
            }
            float4* q = mb_slot<LDS, LK>(stack_off, u, j);
            const float4 q0 = q[0], q1 = q[1], q2 = q[2];
            CRay a;
            a.r.o = v3(q0.x, q0.y, q0.z);
            a.r.time = q0.w;
            a.r.d = v3(q1.x, q1.y, q1.z);
            a.sgn = __float_as_int(q1.w);
            a.inv = v3(q2.x, q2.y, q2.z);
            const CHit h = coop_solve<LDS, LK>(w, a, A.node_count, A.leaf_count, A.rect_count, A.fast_off, A.tri_prefix,
                                               A.tri_stride, A.coop_ties == 2);
            if (lane == 0) {
                mb_answer(mb, q, u, h);
                __hip_atomic_fetch_add(&mb[34], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __syncthreads();  // (block-uniform branch) every wave's counts are in
        if (threadIdx.x < 3) {
            const uint32_t c = __hip_atomic_load(&mb[33 + threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (c) atomicAdd(&rtw_drain_counts[threadIdx.x], (unsigned long long)c);
        }
    }
    RTW_PT_FLUSH;
#ifdef RTW_WAVE_TIMING
    {
        const uint32_t wv_ = (blockIdx.x * RTW_BLOCK + threadIdx.x) / 64;
        if (wv_ < 8192) {
            unsigned long long* x = rtw_wave_extra + 8 * wv_;
            if (wx_busy) atomicMax(&x[0], (unsigned long long)wx_busy);
            atomicAdd(&x[1], (unsigned long long)wx_n);
            atomicAdd(&x[2], (unsigned long long)wx_sum);
            (void)wx_max;
            if (lane == 0) {  // wave-level sums (identical in every lane)
                x[4] = wx_coop;
                x[5] = wx_ref;
                x[6] = wx_tref;
                x[7] = wx_tsah;
                x[3] = wx_tcoop;  // (replaces max bounces)
            }
        }
    }
#endif
    if (STATS) {
        for (int i = 0; i < ST_COUNT; ++i)
            if (st.c[i]) atomicAdd(&A.stats[i], (unsigned long long)st.c[i]);
    }
}

template <bool STATS, int LDS, int LK, int TX, bool GEN = false, bool WP = false>
__global__ __launch_bounds__(RTW_BLOCK, RTW_MIN_WAVES_PER_SIMD) void render_kernel(KArgs A) {
#ifdef RTW_WAVE_TIMING
    const uint64_t t_start = wall_clock64();
#endif
    render_body<STATS, LDS, LK, TX, GEN, WP>(A);
#ifdef RTW_WAVE_TIMING
    const uint32_t wv = (blockIdx.x * RTW_BLOCK + threadIdx.x) / 64;
    if ((threadIdx.x & 63) == 0 && wv < 8192) {
        rtw_wave_times[3 * wv] = t_start;
        rtw_wave_times[3 * wv + 1] = wall_clock64();
        rtw_wave_times[3 * wv + 2] = rtw_wave_dry[wv];
        rtw_wave_dry[wv] = ~0ull;
    }
#endif
}
// Per slot: sum += colour of each sample of this launch, in sample order (the running sum of
// earlier launches is carried in `running`); the last launch writes sum / spp (rendering.rs:179;
// merge_planes with one plane multiplies by 1.0).
__global__ void accumulate_kernel(const float* __restrict__ colors, uint32_t n_samples, uint32_t total,
                                  float* __restrict__ running, int first, int last, uint32_t spp, float* out,
                                  int layout, int32_t width, int32_t height, int32_t tile_w, int32_t tile_h,
                                  int32_t tiles_x, int32_t part_index, int32_t part_count) {
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= total) return;
    const int32_t per_tile = tile_w * tile_h;
    const int32_t tile = part_index + (int32_t)(slot / (uint32_t)per_tile) * part_count;
    const int32_t it = (int32_t)(slot % (uint32_t)per_tile);
    const int32_t px = (tile % tiles_x) * tile_w + it % tile_w;
    const int32_t py = (tile / tiles_x) * tile_h + it / tile_w;
    if (px >= width || py >= height) return;  // padding slot of an edge tile
    V3 sum = first ? v3(0.0f, 0.0f, 0.0f) : v3(running[3 * (size_t)slot], running[3 * (size_t)slot + 1],
                                                running[3 * (size_t)slot + 2]);
    const float* c = colors + 3 * (size_t)slot;
    for (uint32_t s = 0; s < n_samples; ++s, c += 3 * (size_t)total) sum = add(sum, v3(c[0], c[1], c[2]));
    if (last) {
        const V3 pixel = divs(sum, (float)spp);
        float* o = (layout == RTW_LAYOUT_TILES) ? out + 3 * (size_t)slot : out + 3 * ((size_t)py * width + px);
        o[0] = pixel.x;
        o[1] = pixel.y;
        o[2] = pixel.z;
    } else {
        running[3 * (size_t)slot] = sum.x;
        running[3 * (size_t)slot + 1] = sum.y;
        running[3 * (size_t)slot + 2] = sum.z;
    }
}

// The reference's thread_count > 1 (rendering.rs:161-219): split_work_tasks gives plane t the
// samples [start_t, start_t + n_t) with n_t = whole + (t < rem) (planes of 0 samples dropped), each
// plane is its samples' in-order sum / n_t (rendering.rs:172-179), and merge_planes adds the last
// plane first, then planes 0..n-2 in order, then multiplies by 1/n (rendering.rs:239-252).  Per slot:
// `planes` holds the n plane partials / values between launches (plane-major, 3 floats per slot);
// this launch's samples [s0, s1) are added to the planes they belong to, a plane that ends here is
// divided by its count, and the frame's last launch merges.
__global__ void accumulate_planes_kernel(const float* __restrict__ colors, uint32_t s0, uint32_t s1, uint32_t total,
                                         float* __restrict__ planes, uint32_t n_planes, uint32_t whole, uint32_t rem,
                                         int last, float* out, int layout, int32_t width, int32_t height,
                                         int32_t tile_w, int32_t tile_h, int32_t tiles_x, int32_t part_index,
                                         int32_t part_count) {
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= total) return;
    const int32_t per_tile = tile_w * tile_h;
    const int32_t tile = part_index + (int32_t)(slot / (uint32_t)per_tile) * part_count;
    const int32_t it = (int32_t)(slot % (uint32_t)per_tile);
    const int32_t px = (tile % tiles_x) * tile_w + it % tile_w;
    const int32_t py = (tile / tiles_x) * tile_h + it / tile_w;
    if (px >= width || py >= height) return;  // padding slot of an edge tile
    const size_t pstride = 3 * (size_t)total;
    for (uint32_t t = 0; t < n_planes; ++t) {
        const uint32_t n_t = whole + (t < rem ? 1u : 0u);
        const uint32_t a = t * whole + min(t, rem), b = a + n_t;
        if (b <= s0 || a >= s1) continue;
        float* P = planes + t * pstride + 3 * (size_t)slot;
        V3 sum = a < s0 ? v3(P[0], P[1], P[2]) : v3(0.0f, 0.0f, 0.0f);
        const uint32_t lo = max(a, s0), hi = min(b, s1);
        const float* c = colors + ((size_t)(lo - s0) * total + slot) * 3;
        for (uint32_t s = lo; s < hi; ++s, c += pstride) sum = add(sum, v3(c[0], c[1], c[2]));
        if (b <= s1) sum = divs(sum, (float)n_t);  // .sum::<Color>() / real_samples_per_pixel as f32
        P[0] = sum.x;
        P[1] = sum.y;
        P[2] = sum.z;
    }
    if (!last) return;
    const float* L = planes + (n_planes - 1) * pstride + 3 * (size_t)slot;
    V3 r = v3(L[0], L[1], L[2]);  // planes.pop()
    for (uint32_t t = 0; t + 1 < n_planes; ++t) {
        const float* P = planes + t * pstride + 3 * (size_t)slot;
        r = add(r, v3(P[0], P[1], P[2]));
    }
    r = mul(r, 1.0f / (float)n_planes);  // multiplier = 1.0 / planes.len() as f32
    float* o = (layout == RTW_LAYOUT_TILES) ? out + 3 * (size_t)slot : out + 3 * ((size_t)py * width + px);
    o[0] = r.x;
    o[1] = r.y;
    o[2] = r.z;
}

// The same merge when the whole frame's samples are in one launch: each plane is summed and divided
// straight from the colour buffer, the last plane first (planes.pop()), then planes 0..n-2 are added
// in order, so no plane buffer is needed (thread_count up to spp costs no memory beyond the colours).
// Bit-identical to accumulate_planes_kernel: the same sums, divisions and merge order.
__global__ void merge_planes_direct_kernel(const float* __restrict__ colors, uint32_t total, uint32_t n_planes,
                                           uint32_t whole, uint32_t rem, float* out, int layout, int32_t width,
                                           int32_t height, int32_t tile_w, int32_t tile_h, int32_t tiles_x,
                                           int32_t part_index, int32_t part_count) {
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= total) return;
    const int32_t per_tile = tile_w * tile_h;
    const int32_t tile = part_index + (int32_t)(slot / (uint32_t)per_tile) * part_count;
    const int32_t it = (int32_t)(slot % (uint32_t)per_tile);
    const int32_t px = (tile % tiles_x) * tile_w + it % tile_w;
    const int32_t py = (tile / tiles_x) * tile_h + it / tile_w;
    if (px >= width || py >= height) return;  // padding slot of an edge tile
    const size_t pstride = 3 * (size_t)total;
    auto plane = [&](uint32_t t) {
        const uint32_t n_t = whole + (t < rem ? 1u : 0u);
        const uint32_t a = t * whole + min(t, rem);
        V3 sum = v3(0.0f, 0.0f, 0.0f);
        const float* c = colors + (size_t)a * pstride + 3 * (size_t)slot;
        for (uint32_t s = 0; s < n_t; ++s, c += pstride) sum = add(sum, v3(c[0], c[1], c[2]));
        return divs(sum, (float)n_t);
    };
    V3 r = plane(n_planes - 1);  // planes.pop()
    for (uint32_t t = 0; t + 1 < n_planes; ++t) r = add(r, plane(t));
    r = mul(r, 1.0f / (float)n_planes);
    float* o = (layout == RTW_LAYOUT_TILES) ? out + 3 * (size_t)slot : out + 3 * ((size_t)py * width + px);
    o[0] = r.x;
    o[1] = r.y;
    o[2] = r.z;
}

// per local tile: the summed slot costs (keys of the next frame's work order, saturated to 32 bits)
// and its index; the slot costs then decay by half, so the order follows the recent frames (a
// changed seed or camera re-weights within a few frames) and the per-slot counters stay bounded
// (<= 2x one frame's deep bounces: 50 x 2048 spp x 2 < 2^18 per slot)
__global__ void tile_cost_kernel(uint32_t* slot_cost, uint32_t n_tiles, uint32_t per_tile, uint32_t* tile_cost,
                                 uint32_t* tile_index) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tiles) return;
    uint64_t sum = 0;
    for (uint32_t i = 0; i < per_tile; ++i) {
        const uint32_t c = slot_cost[(size_t)t * per_tile + i];
        sum += c;
        slot_cost[(size_t)t * per_tile + i] = c >> 1;
    }
    tile_cost[t] = (uint32_t)min<uint64_t>(sum, 0xFFFFFFFFull);
    tile_index[t] = t;
}

// scatter gathered tile buffers back into the image
__global__ void untile_kernel(const float* tiles, int64_t stride, float* image, int32_t width, int32_t height,
                              int32_t tile_w, int32_t tile_h, int32_t tiles_x, int32_t n_tiles, int32_t part_count) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_tile = (int64_t)tile_w * tile_h;
    if (i >= (int64_t)n_tiles * per_tile) return;
    const int32_t tile = (int32_t)(i / per_tile);
    const int32_t in_tile = (int32_t)(i % per_tile);
    const int32_t px = (tile % tiles_x) * tile_w + in_tile % tile_w;
    const int32_t py = (tile / tiles_x) * tile_h + in_tile / tile_w;
    if (px >= width || py >= height) return;
    const int32_t part = tile % part_count, local = tile / part_count;
    const float* src = tiles + (int64_t)part * stride + ((int64_t)local * per_tile + in_tile) * 3;
    float* dst = image + ((int64_t)py * width + px) * 3;
    dst[0] = src[0];
    dst[1] = src[1];
    dst[2] = src[2];
}

// color.rs:43-48 to_rgb8_gamma2
__global__ void encode_kernel(const float* img, int64_t n, uint8_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * 3) return;
    const float v = rtw_clampr(0.0f, 255.0f, __builtin_sqrtf(img[i]) * 256.0f);
    out[i] = rtw_f2u8_sat(v);
}

__global__ void eval_scalar_kernel(int fn, const float* a, const float* b, int64_t n, float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float r;
    switch (fn) {
        case 0: r = d_acosf(a[i]); break;  // the render kernel's versions (div_x / sqrt_x inside)
        case 1: r = d_atan2f(a[i], b[i]); break;
        case 2: r = rtw_logf(a[i]); break;
        case 3: r = rtw_sinf(a[i]); break;
        case 4: r = a[i] / b[i]; break;
        case 5: r = __builtin_sqrtf(a[i]); break;
        default: r = a[i] / b[i]; break;
    }
    out[i] = r;
}

__global__ void eval_checker_kernel(const float* xyz, int64_t n, int32_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = d_checker_odd(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]) ? 1 : 0;
}

__global__ void eval_node_pass_kernel(const float* box, const float* ray, const float* range, const float* km,
                                      int32_t mk_world, int64_t n, int32_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* b = box + 6 * i;
    const float* r = ray + 6 * i;
    Ray R;
    R.o = v3(r[0], r[1], r[2]);
    R.d = v3(r[3], r[4], r[5]);
    R.time = 0.0f;
    const RayPre rp = ray_pre(R, mk_world != 0);  // modes 2 and 3: the SAH tests (mk world)
    const float4 na = make_float4(b[0], b[1], b[2], b[3]), nb = make_float4(b[4], b[5], 0.0f, 0.0f);
    if (mk_world == 2 || mk_world == 3) {
        // the SAH walk's node test (cheap quotients, constants widened as build_sah_tables uploads
        // them) beside the cull alone with exact quotients and the plain constants: bit 0 = SAH test
        // passes, bit 1 = exact cull passes, bit 2 = the ray is Markstein-exact (the SAH walk's rays)
        float k = km[2 * i], m = km[2 * i + 1];
        if (k > 0.0f) k = nextafterf(k * RTW_SAH_WIDEN, F32_INF);
        if (m > 0.0f) m = nextafterf(m * RTW_SAH_WIDEN, F32_INF);
        float e;
        const bool sah = mk_world == 2 ? node_pass_cons<true>(na, nb, make_float2(k, m), R, rp, range[2 * i], range[2 * i + 1], e)
                                       : node_pass_cons<false>(na, nb, make_float2(k, m), R, rp, range[2 * i], range[2 * i + 1], e);
        const bool exact = node_pass_cull_exact(na, nb, make_float2(km[2 * i], km[2 * i + 1]), R, rp, range[2 * i],
                                                range[2 * i + 1]);
        out[i] = (sah ? 1 : 0) | (exact ? 2 : 0) | (rp.fast ? 4 : 0);
        return;
    }
    out[i] = node_pass(na, nb, make_float2(km[2 * i], km[2 * i + 1]), R, rp, range[2 * i], range[2 * i + 1]) ? 1 : 0;
}

// Self-check of the exact fast divisions (§5.8) on the device, counted there.  Case i of [0, n):
//   test 0: b = bits(base + i): rcp_nr(b) against 1 / b (the caller picks the exponent range)
//   test 1: a = bits(base + i): div_c(a, pi), div_c(a, tau) against a / pi, a / tau (any a)
//   test 2: a random pair inside Markstein's guards: mk_corr(a, b, rcp_nr(b)) against a / b
//   test 4: a = bits(base + i): sqrt_x (and sqrt_nr inside its range) against sqrtf
//   test 3: a random pair of any kind (zeros, subnormals, extremes, inf, NaN): div_x, div_tri (y as
//           tri_prepare sets it), rcp_x and divs_x's components against IEEE division
//   test 5: tri_t_mk (the triangle's t without a guard) decides contains(0.001, .., t) as a / b does
// out[0] += mismatches, out[1] = min over mismatching i (the first one, ~0 if none)
__device__ __forceinline__ uint64_t chk_mix(uint64_t x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull; return x ^ (x >> 31);
}
__device__ __forceinline__ bool chk_same(float x, float y) { return __float_as_uint(x) == __float_as_uint(y) || (x != x && y != y); }
__device__ __forceinline__ float chk_float(uint64_t r, int e_lo, int e_hi) {  // random sign / mantissa, exponent in [e_lo, e_hi]
    const int e = e_lo + (int)((r >> 32) % (uint64_t)(e_hi - e_lo + 1));
    return __uint_as_float((uint32_t)(r & 0x807FFFFFu) | ((uint32_t)(e + 127) << 23));
}
__device__ __forceinline__ float chk_any(uint64_t r) {  // special values, extremes and plain floats
    switch ((r >> 56) & 15) {
        case 0: return (r & 1) ? -0.0f : 0.0f;
        case 1: return __uint_as_float((uint32_t)r & 0x807FFFFFu);  // subnormal
        case 2: return chk_float(r, -126, -90);
        case 3: return chk_float(r, 90, 127);
        case 4: return (r & 1) ? -F32_INF : F32_INF;
        case 5: return __uint_as_float(0x7FC00000u | ((uint32_t)r & 0x803FFFFFu));
        case 6: return chk_float(r, -104, -76);  // the guards' edges
        case 7: return chk_float(r, 76, 104);
        case 8: return chk_float(r, -24, -20);
        case 9: return chk_float(r, 20, 24);
        default: return chk_float(r, -30, 30);
    }
}
__global__ void check_division_kernel(int test, uint64_t base, uint64_t n, uint64_t seed, unsigned long long* out) {
    uint64_t bad = 0, first = ~0ull;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        bool ok = true;
        if (test == 0) {
            const float b = __uint_as_float((uint32_t)(base + i));
            ok = chk_same(rcp_nr(b), 1.0f / b);
        } else if (test == 1) {
            const float a = __uint_as_float((uint32_t)(base + i));
            ok = chk_same(div_c(a, F32_PI, 1.0f / F32_PI), a / F32_PI) && chk_same(div_c(a, F32_TAU, 1.0f / F32_TAU), a / F32_TAU);
        } else if (test == 4) {
            const float a = __uint_as_float((uint32_t)(base + i));
            ok = chk_same(sqrt_x(a), __builtin_sqrtf(a));
            if (a >= RTW_SQRT_LO && a <= 0x1.fffffep127f) ok = ok && chk_same(sqrt_nr(a), __builtin_sqrtf(a));
        } else if (test == 2) {
            const uint64_t r1 = chk_mix(seed ^ (2 * i)), r2 = chk_mix(seed ^ (2 * i + 1));
            const float a = chk_float(r1, -80, 80), b = chk_float(r2, -22, 22);
            ok = chk_same(mk_corr(a, b, rcp_nr(b)), a / b);
        } else if (test == 6) {
            // tex255 (an image texel's channel) against byte / 255.0f: bytes base + i, i < 256
            const uint32_t b = (uint32_t)(base + i) & 255u;
            ok = chk_same(tex255(b), (float)b / 255.0f);
        } else if (test == 5) {
            // tri_t_mk: a dividend of any kind (zeros, subnormals, NaN, up to 2^40 in magnitude: num is a
            // dot product of coordinates below 2^30 with a unit normal), a divisor
            // with 1e-4 < |b| <= 1.01 (tri_test's range): equal to a / b whenever that is >= 0.001, and
            // below 0.001 (or NaN alike) whenever a / b is
            const uint64_t r1 = chk_mix(seed ^ (2 * i)), r2 = chk_mix(seed ^ (2 * i + 1));
            float a = chk_any(r1);
            if (((r1 >> 60) & 3) == 0) a = chk_float(r1, -150 + 23, -60);  // tiny dividends
            if (__builtin_fabsf(a) > 0x1p40f) a = __builtin_copysignf(0x1p40f, a);
            float b = chk_float(r2, -14, 0);
            if (__builtin_fabsf(b) <= 1e-4f) b = __builtin_copysignf(1.5e-4f, b);
            const float q = tri_t_mk(a, b), e = a / b;
            ok = e >= 0.001f ? chk_same(q, e) : !(q >= 0.001f);
        } else {
            const uint64_t r1 = chk_mix(seed ^ (2 * i)), r2 = chk_mix(seed ^ (2 * i + 1));
            const float a = chk_any(r1), b = chk_any(r2);
            const float ab = __builtin_fabsf(b);
            const float y = (ab >= 0x1p-22f && ab <= 0x1p22f) ? 1.0f / b : 0.0f;  // tri_prepare's rule
            const V3 q = divs_x(v3(a, b, a * 0.5f), b), e = divs(v3(a, b, a * 0.5f), b);
            ok = chk_same(div_x(a, b), a / b) && chk_same(div_tri(a, b, y), a / b) && chk_same(rcp_x(b), 1.0f / b) &&
                 chk_same(q.x, e.x) && chk_same(q.y, e.y) && chk_same(q.z, e.z);
        }
        if (!ok) {
            ++bad;
            first = min(first, (unsigned long long)i);
        }
    }
    if (bad) {
        atomicAdd(&out[0], (unsigned long long)bad);
        atomicMin(&out[1], (unsigned long long)first);
    }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
#define HIP_TRY(expr)                                                                             \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess)                                                                     \
            return rtw::fail(RTW_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));    \
    } while (0)

inline uint32_t fbits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}
inline float ibits(int32_t i) {
    float f;
    std::memcpy(&f, &i, 4);
    return f;
}

struct Layout {
    std::vector<uint8_t> blob;
    size_t push(const void* p, size_t bytes) {
        size_t off = (blob.size() + 255) & ~(size_t)255;
        blob.resize(off + bytes);
        if (bytes) std::memcpy(blob.data() + off, p, bytes);
        return off;
    }
};

// does material m's texture tree (checker children followed, as texture_sample does) hold an
// image texture?  Conservative on cycles / deep chains (the device gives up after 64 steps).
bool material_reads_uv(const rtw_world* w, int m) {
    const rtw_material& M = w->materials[m];
    if (M.kind == RTW_MAT_DIELECTRIC) return false;
    std::vector<int> todo{M.texture};
    for (int steps = 0; !todo.empty(); ++steps) {
        if (steps > 4096) return true;
        const int t = todo.back();
        todo.pop_back();
        const rtw_texture& T = w->textures[t];
        if (T.kind == RTW_TEX_IMAGE) return true;
        if (T.kind == RTW_TEX_CHECKER) {
            todo.push_back(T.even);
            todo.push_back(T.odd);
        }
    }
    return false;
}

int check_world(const rtw_world* w, int* depth_out) {
    if (!w) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null world");
    if (w->leaf_count < 1) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "world has no leaves");
    auto bad = [&](const char* m) { return rtw::fail(RTW_ERR_INVALID_ARGUMENT, std::string("invalid world: ") + m); };
    if (w->root >= 0 ? w->root >= w->node_count : (-1 - w->root) >= w->leaf_count) return bad("root out of range");
    for (int i = 0; i < w->leaf_count; ++i) {
        const rtw_leaf& L = w->leaves[i];
        const int counts[4] = {w->sphere_count, w->rect_count, w->box_count, w->triangle_count};
        if (L.geom_kind < 0 || L.geom_kind > 3) return bad("leaf geometry kind");
        if (L.geom_index < 0 || L.geom_index >= counts[L.geom_kind]) return bad("leaf geometry index");
        if (L.material < 0 || L.material >= w->material_count) return bad("leaf material index");
    }
    for (int i = 0; i < w->material_count; ++i) {
        const rtw_material& m = w->materials[i];
        if (m.kind < 0 || m.kind > 4) return bad("material kind");
        if (m.kind != RTW_MAT_DIELECTRIC && (m.texture < 0 || m.texture >= w->texture_count)) return bad("material texture");
    }
    for (int i = 0; i < w->texture_count; ++i) {
        const rtw_texture& t = w->textures[i];
        if (t.kind == RTW_TEX_CHECKER && (t.even < 0 || t.even >= w->texture_count || t.odd < 0 || t.odd >= w->texture_count))
            return bad("checker texture ids");
        if (t.kind == RTW_TEX_IMAGE && (t.image < 0 || t.image >= w->image_count)) return bad("image id");
        if (t.kind == RTW_TEX_MARBLE && (t.perlin < 0 || t.perlin >= w->perlin_count)) return bad("perlin id");
    }
    for (int i = 0; i < w->perlin_count; ++i)
        if (w->perlins[i].bits < 1 || w->perlins[i].bits > 8) return bad("perlin bits");
    for (int i = 0; i < w->image_count; ++i)
        if (w->images[i].width < 1 || w->images[i].height < 1 || !w->images[i].rgb) return bad("image");
    // coordinate bound behind the exact fast division of the slab test (|a| <= 2^40 there):
    // every coordinate the device sees stays below 2^30 in magnitude
    const float LIM = 1073741824.0f;
    auto big = [&](const float* v, int n) {
        for (int k = 0; k < n; ++k)
            if (!(v[k] >= -LIM && v[k] <= LIM)) return true;
        return false;
    };
    for (int i = 0; i < w->node_count; ++i)
        if (big(w->nodes[i].min, 3) || big(w->nodes[i].max, 3)) return bad("node bounds beyond 2^30");
    for (int i = 0; i < w->sphere_count; ++i)
        if (big(w->spheres[i].center, 4)) return bad("sphere beyond 2^30");
    for (int i = 0; i < w->rect_count; ++i)
        if (big(&w->rects[i].dist, 1)) return bad("rect beyond 2^30");
    // an Animation offset is velocity x ray time, the rolling shutter's pace included (rtw_ray_time_range)
    float rt0 = 0.0f, rt1 = 0.0f;
    const float tmax = rtw_ray_time_range(&w->camera, &rt0, &rt1) ? std::max(std::fabs(rt0), std::fabs(rt1))
                                                                   : std::numeric_limits<float>::infinity();
    for (int i = 0; i < w->leaf_count; ++i) {
        const rtw_leaf& L = w->leaves[i];
        float vt[3];
        for (int k = 0; k < 3; ++k)
            vt[k] = (L.flags & RTW_LEAF_ANIMATION) && L.velocity[k] != 0.0f ? L.velocity[k] * tmax : 0.0f;
        if (big(L.offset, 3) || big(vt, 3)) return bad("leaf transform beyond 2^30");
    }
    if (big(w->camera.position, 3)) return bad("camera beyond 2^30");
    // node references + depth (the per-lane stack holds one entry per level)
    std::vector<std::pair<int32_t, int>> todo;
    int maxd = 0;
    std::vector<uint8_t> seen((size_t)std::max(1, w->node_count), 0);
    if (w->root >= 0) todo.emplace_back(w->root, 0);
    while (!todo.empty()) {
        auto [n, d] = todo.back();
        todo.pop_back();
        if (n < 0) {
            if (-1 - n >= w->leaf_count) return bad("leaf reference");
            continue;
        }
        if (n >= w->node_count || seen[(size_t)n]) return bad("node reference");
        seen[(size_t)n] = 1;
        const rtw_bvh_node& nd = w->nodes[n];
        if (nd.axis < 0 || nd.axis > 2) return bad("node axis");
        maxd = std::max(maxd, d + 1);
        todo.emplace_back(nd.left, d + 1);
        todo.emplace_back(nd.right, d + 1);
    }
    if (maxd > RTW_STACK) return rtw::fail(RTW_ERR_UNSUPPORTED, "BVH deeper than the device stack");
    *depth_out = maxd;
    return RTW_OK;
}

// The SAH path's tables (§5.5), or empty when the world does not qualify: no volume leaves (their
// RNG draws depend on the visit order), every leaf cullable with its true world box (rtw_cull_leaf,
// wrapped = 1: plain or Transformation / Animation spheres, triangles, rects and boxes), every box
// coordinate admitting the fast division (0 or 2^-60 .. 2^30 in magnitude), the reference tree's
// internal boxes nested (each child node's box inside its parent's), and RTW_NO_SAH unset.
// The proof box of a leaf (box_hit_cond_fast after the walk) is its parent node's box in the
// reference tree: when it passes hit_cond at te = succ(t), so do all ancestors (nested, monotone),
// and the reference DFS reaches the leaf -- whose own Aabb, for a wrapped leaf the apply_aabb
// quirk's untransformed box, need not hold the hit at all.
// the length of the world's leading run of plain triangle leaves whose triangle index is their leaf index
// (walk_leaf_record; a mesh added first, as in suzanne, or a triangle soup) ...
// and whose material is leaf 0's (leaf_info_of makes their leaf_info up)
int32_t tri_prefix_of(const rtw_world* w) {
    int32_t p = 0;
    while (p < w->leaf_count && w->leaves[p].geom_kind == RTW_GEOM_TRIANGLE && w->leaves[p].flags == 0 &&
           w->leaves[p].geom_index == p && w->leaves[p].material == w->leaves[0].material)
        ++p;
    return p;
}
// LDS bytes of mode 2 for the one-child walk's tables (launch_render's sizing: nodes, the leaf records from
// the triangle prefix on, cull constants, rect records, triangle records at the exact stride, 16-bit stack
// of `depth` entries, the drain's mailbox) -- the depth cap of the split tree (build_sah_tables) aims at it
size_t lds_mode2_bytes(size_t nodes, size_t leaf_records, size_t rects, size_t tris, int depth) {
    return (2 * nodes + leaf_records + (nodes + 1) / 2 + 2 * rects + 4 * tris) * sizeof(float4) +
           (size_t)depth * RTW_BLOCK * sizeof(int16_t) + RTW_MB_WORDS * sizeof(uint32_t);
}
struct SahTables {
    std::vector<float4> a, b;     // nodes, as node_a / node_b
    std::vector<float> km;        // cull constants, 2 per node
    std::vector<float4> box;      // 2 per leaf: the proof box (the leaf's parent box in the reference tree)
    std::vector<uint4> key;       // per leaf: its DFS key material (DWorld::leaf_key), empty if too deep
    int32_t root_c2 = 0;  // the root's children word (the two-children walk, plain-sphere worlds)
    float k = 0.0f;       // the largest finite node k (DWorld::sah_k)
    bool folded = false;  // plain-sphere world: node records carry children word + m (sah_left / sah_right)
    int32_t root = 0, depth = 0;
    bool ok = false;
};
SahTables build_sah_tables(const rtw_world* w) {
    SahTables S;
    if (const char* e = std::getenv("RTW_NO_SAH"))
        if (e[0] && e[0] != '0') return S;
    const int32_t L = w->leaf_count;
    if (L < 2 || w->root < 0 || w->node_count < 1) return S;
    auto coord_ok = [](float c) { return c == 0.0f || (std::fabs(c) >= 0x1p-60f && std::fabs(c) <= 1073741824.0f); };
    std::vector<float> lo((size_t)L * 3), hi((size_t)L * 3), lkm((size_t)L * 2);
    std::vector<uint8_t> never((size_t)L, 0);
    for (int32_t i = 0; i < L; ++i) {
        float k, m;
        int nv = 0;
        float* mn = &lo[3 * (size_t)i];
        float* mx = &hi[3 * (size_t)i];
        if (!rtw_cull_leaf(w, &w->leaves[i], 1, &k, &m, mn, mx, &nv)) return S;
        never[(size_t)i] = (uint8_t)nv;
        lkm[2 * (size_t)i] = nv ? -1.0f : k;
        lkm[2 * (size_t)i + 1] = nv ? 0.0f : m;
        if (nv) {  // a leaf that never reports a hit: any box (it only has to sit somewhere in the tree)
            const rtw_triangle& t = w->triangles[w->leaves[i].geom_index];
            for (int k2 = 0; k2 < 3; ++k2) {
                mn[k2] = rtw_minr(rtw_minr(t.positions[0][k2], t.positions[1][k2]), t.positions[2][k2]);
                mx[k2] = rtw_maxr(rtw_maxr(t.positions[0][k2], t.positions[1][k2]), t.positions[2][k2]);
            }
        }
        for (int k2 = 0; k2 < 3; ++k2)
            if (!coord_ok(mn[k2]) || !coord_ok(mx[k2])) return S;
    }
    // nested reference boxes (internal children inside their parents) and each leaf's parent
    std::vector<int32_t> parent((size_t)L, -1);
    for (int32_t n = 0; n < w->node_count; ++n) {
        const rtw_bvh_node& nd = w->nodes[n];
        for (int k2 = 0; k2 < 3; ++k2)
            if (!coord_ok(nd.min[k2]) || !coord_ok(nd.max[k2])) return S;
        for (int32_t c : {nd.left, nd.right}) {
            if (c < 0) {
                parent[(size_t)(-1 - c)] = n;
                continue;
            }
            for (int k2 = 0; k2 < 3; ++k2)
                if (!(nd.min[k2] <= w->nodes[c].min[k2] && w->nodes[c].max[k2] <= nd.max[k2])) return S;
        }
    }
    for (int32_t i = 0; i < L; ++i)
        if (parent[(size_t)i] < 0) return S;  // a leaf outside the reference tree
    std::vector<rtw_bvh_node> nodes;
    // spatial splits (rtw::sah_build_split) in worlds with plain triangles, RTW_SAH_SPLIT_BUDGET extra
    // references per leaf at most (0: the object-split tree)
    // (default 1.0: suzanne +21 % over round 4's 0.2, now that a 16-bit stack keeps the larger tree in LDS
    // mode 1, profiles/r05/split_stats.txt; round 4 measured 0.2 at +1.1 % over none)
    double budget = RTW_SAH_SPLIT_BUDGET;
    if (const char* e = std::getenv("RTW_SAH_SPLIT_BUDGET")) budget = std::max(0.0, std::atof(e));
    std::vector<float> tri;
    if (budget > 0.0) {
        tri.assign((size_t)L * 9, std::numeric_limits<float>::quiet_NaN());
        bool any = false;
        for (int32_t i = 0; i < L; ++i) {
            const rtw_leaf& l = w->leaves[i];
            if (l.geom_kind != RTW_GEOM_TRIANGLE || l.flags != 0 || never[(size_t)i]) continue;
            const rtw_triangle& t = w->triangles[l.geom_index];
            for (int v = 0; v < 3; ++v)
                for (int k2 = 0; k2 < 3; ++k2) tri[9 * (size_t)i + 3 * v + k2] = t.positions[v][k2];
            any = true;
        }
        if (!any) budget = 0.0;
    }
    if (budget > 0.0) {
        // node boxes and cull constants come from the builder: a node's box is the union of its
        // references' clipped boxes, k and m the maxima of the leaves' constants below
        std::vector<rtw_bvh_node> split;
        std::vector<float> skm;
        int32_t sroot = 0;
        int sdepth = 0;
        const char* cap_env = std::getenv("RTW_SAH_DEPTH_CAP");  // tests / audits: this cap (0: none)
        bool ok = rtw::sah_build_split(lo.data(), hi.data(), tri.data(), lkm.data(), L, budget, split, skm, &sroot, &sdepth,
                                       cap_env ? std::atoi(cap_env) : 0) == 0 &&
                  sdepth <= RTW_STACK;
        for (const rtw_bvh_node& nd : split)
            for (int k2 = 0; k2 < 3; ++k2)
                if (!coord_ok(nd.min[k2]) || !coord_ok(nd.max[k2])) ok = false;
        // The depth cap: a split tree whose 16-bit stack keeps it out of LDS mode 2 (the triangle records in
        // LDS) is rebuilt with the largest depth cap that lets it in, down to ceil(log2 L) + 5 levels (worlds
        // of plain triangles and spheres: the LK_TRIS kernels' layout, lds_mode2_bytes).
        // suzanne: depth 21 -> 16, 1770 -> 1719 nodes, node tests per ray +0.5 %, leaf tests +1.7 %
        // (tools/sah_cost.py), and the triangle records in LDS: DESIGN 4.
        bool tris_spheres = true;  // the kernels with the exact triangle stride and the prefix (LK_TRIS)
        for (int32_t i = 0; i < L; ++i)
            if ((w->leaves[i].geom_kind != RTW_GEOM_TRIANGLE && w->leaves[i].geom_kind != RTW_GEOM_SPHERE) ||
                w->leaves[i].flags != 0)
                tris_spheres = false;
        if (ok && !cap_env && tris_spheres && L < 32768) {
            int rdepth = 0;
            check_world(w, &rdepth);
            const size_t P = (size_t)tri_prefix_of(w);
            auto fits2 = [&](size_t n, int d) {
                return n < 32768 && lds_mode2_bytes(n, (size_t)L - P, (size_t)w->rect_count, (size_t)w->triangle_count,
                                                    std::max(d, rdepth)) <= RTW_LDS_SCENE_MAX;
            };
            int lb = 5;
            while ((1 << (lb - 5)) < L) ++lb;
            // the first cap tried: two levels above the deepest stack that fits with the uncapped tree's node
            // count (a capped tree has a few nodes fewer: suzanne 17, then 16 -- two builds of ~0.3 s, not five)
            int first = sdepth - 1;
            for (int d = lb; d < sdepth; ++d)
                if (fits2(split.size(), d)) first = std::min(sdepth - 1, d + 2);
            if (!fits2(split.size(), sdepth) && fits2((size_t)L - 1, lb))
                for (int c = first; c >= lb; --c) {
                    std::vector<rtw_bvh_node> s2;
                    std::vector<float> k2v;
                    int32_t r2 = 0;
                    int d2 = 0;
                    if (rtw::sah_build_split(lo.data(), hi.data(), tri.data(), lkm.data(), L, budget, s2, k2v, &r2, &d2, c) != 0)
                        break;
                    bool ok2 = d2 <= c;
                    for (const rtw_bvh_node& nd : s2)
                        for (int k3 = 0; k3 < 3; ++k3)
                            if (!coord_ok(nd.min[k3]) || !coord_ok(nd.max[k3])) ok2 = false;
                    if (ok2 && fits2(s2.size(), d2)) {
                        split.swap(s2);
                        skm.swap(k2v);
                        sroot = r2;
                        sdepth = d2;
                        break;
                    }
                }
        }
        // The extra nodes must not push the world out of the LDS modes (launch_render: mode 1 holds
        // nodes, leaf records, cull constants, rects and the 16-bit stack, mode 2 the triangle records
        // too): a split tree that fits mode 1 only beats the object-split tree in mode 2 (suzanne at
        // budget 1, 1809 nodes, depth 20: 22.9 node visits and 10.3 triangle tests per ray against 30.8
        // and 16.2 at budget 0.2, 1080p x 128 in 101.7 ms against 123.5, profiles/r05/split_stats.txt),
        // but one that leaves the LDS entirely does not (else the plain tree).  RTW_SAH_IGNORE_LDS=1
        // (tests and audits) keeps the split tree whatever the LDS mode.
        if (ok) {
            int32_t proot = 0;
            int pdepth = 0;
            std::vector<rtw_bvh_node> plain;
            if (rtw::sah_build(lo.data(), hi.data(), L, plain, &proot, &pdepth) == 0) {
                int rdepth = 0;  // the reference tree's depth: the stack serves both walks
                check_world(w, &rdepth);
                auto mode1 = [&](size_t n, int depth) {
                    return (2 * n + (size_t)L + (n + 1) / 2 + 2 * (size_t)w->rect_count) * 16 +
                           (size_t)std::max(depth, rdepth) * RTW_BLOCK * 2;
                };
                const size_t cap = RTW_LDS_SCENE_MAX;
                if (mode1(plain.size(), pdepth) <= cap && mode1(split.size(), sdepth) > cap && !std::getenv("RTW_SAH_IGNORE_LDS"))
                    ok = false;
            }
        }
        if (ok) {
            nodes.swap(split);
            S.km.swap(skm);
            S.root = sroot;
            S.depth = sdepth;
        } else {
            budget = 0.0;
        }
    }
    if (budget <= 0.0) {
        if (rtw::sah_build(lo.data(), hi.data(), L, nodes, &S.root, &S.depth) != 0 || S.depth > RTW_STACK) return S;
        // cull constants of the SAH tree over the leaves' true world boxes (wrapped leaves included)
        rtw_world tw = *w;
        tw.nodes = nodes.data();
        tw.node_count = (int32_t)nodes.size();
        tw.root = S.root;
        S.km.assign(nodes.size() * 2, 0.0f);
        rtw_cull_prepare_ex(&tw, S.km.data(), 0, 1);
    }
    for (float& c : S.km)  // x17/16 rounded up (inf stays inf): the cheap quotients' slack, node_pass_cons
        if (c > 0.0f) c = std::nextafter(c * RTW_SAH_WIDEN, std::numeric_limits<float>::infinity());
    // A node with one leaf child holds it on the left, so that a wave's two-children steps diverge less
    // between the sphere and the box test per slot (final_scene1 +0.3 %, within noise; the others
    // unchanged: profiles/r04/v15_leaf_left_ab.txt; RTW_SAH_LEAF_LEFT=0 keeps the builder's order).  The
    // walks' visit order does not depend on the slots (entry t in the two-children walk, leaf first in
    // the other), so neither do their results.
    if (const char* ll = std::getenv("RTW_SAH_LEAF_LEFT"); !(ll && ll[0] == '0'))
        for (rtw_bvh_node& n : nodes)
            if (n.left >= 0 && n.right < 0) std::swap(n.left, n.right);
    // plain-sphere worlds (the two-children walk): node records sah_left / sah_right with m, children
    // 15-bit signed (at most 2^14 - 1 nodes and 2^14 leaves), k per world (DWorld::sah_k), the root's
    // children word as the walk's first lane state; other worlds -- and plain-sphere worlds above those
    // limits, which then take the one-child walk of the triangle loop (rtw_world_upload) rather than
    // losing the SAH tree -- node_b as the reference tree's and the cull constants in sah_km
    bool plain_spheres = true;
    for (int32_t i = 0; i < L; ++i)
        if (w->leaves[i].geom_kind != RTW_GEOM_SPHERE || w->leaves[i].flags != 0) plain_spheres = false;
    if (plain_spheres && (nodes.size() >= 16384 || L > 16384)) plain_spheres = false;
    S.folded = plain_spheres;
    auto kids = [](const rtw_bvh_node& n) {
        return (int32_t)((uint32_t)n.axis | (((uint32_t)n.left & 0x7FFFu) << 2) | ((uint32_t)n.right << 17));
    };
    S.k = 0.0f;
    for (size_t i = 0; i < nodes.size(); ++i)
        if (std::isfinite(S.km[2 * i])) S.k = std::max(S.k, S.km[2 * i]);
    S.a.resize(nodes.size());
    S.b.resize(nodes.size());
    for (size_t i = 0; i < nodes.size(); ++i) {
        const rtw_bvh_node& n = nodes[i];
        const float m = std::isfinite(S.km[2 * i]) ? S.km[2 * i + 1] : std::numeric_limits<float>::infinity();
        S.a[i] = make_float4(n.min[0], n.min[1], n.min[2], n.max[0]);
        S.b[i] = plain_spheres ? make_float4(n.max[1], n.max[2], ibits(kids(n)), m)
                               : make_float4(n.max[1], n.max[2], ibits((int32_t)((uint32_t)n.left << 2) | n.axis),
                                             ibits(n.right));
    }
    S.root_c2 = kids(nodes[(size_t)S.root]);
    S.box.resize((size_t)L * 2);
    for (int32_t i = 0; i < L; ++i) {
        const rtw_bvh_node& p = w->nodes[parent[(size_t)i]];
        S.box[2 * (size_t)i] = make_float4(p.min[0], p.min[1], p.min[2], p.max[0]);
        S.box[2 * (size_t)i + 1] = make_float4(p.max[1], p.max[2], 0.0f, 0.0f);
    }
    // DFS keys: hittable.rs:441-445 visits the left child first when ray.d[axis] > 0, else the right
    // one; a leaf's place in that order is the string of its ancestors' decisions (root first)
    {
        S.key.assign((size_t)L, make_uint4(0, 0, 0, 0));
        bool ok = true;
        struct Item { int32_t node; int depth; uint32_t side, a0, a1, a2; };
        std::vector<Item> st{{w->root, 0, 0, 0, 0, 0}};
        while (!st.empty() && ok) {
            const Item it = st.back();
            st.pop_back();
            if (it.node < 0) {
                S.key[(size_t)(-1 - it.node)] = make_uint4(it.side, it.a0, it.a1, it.a2);
                continue;
            }
            if (it.depth >= 32) {
                ok = false;
                break;
            }
            const rtw_bvh_node& nd = w->nodes[it.node];
            const uint32_t bit = 1u << (31 - it.depth);
            Item c = it;
            c.depth = it.depth + 1;
            if (nd.axis == 0) c.a0 |= bit;
            else if (nd.axis == 1) c.a1 |= bit;
            else c.a2 |= bit;
            c.node = nd.left;
            st.push_back(c);
            c.node = nd.right;
            c.side |= bit;
            st.push_back(c);
        }
        if (!ok) S.key.clear();
    }
    S.ok = true;
    return S;
}

}  // namespace

struct rtw_gpu_world {
    int device = 0;
    void* arena = nullptr;
    unsigned long long* queue = nullptr;  // work-item counter (one render at a time per world)
    float* colors = nullptr;   // per-sample colours of one launch (grown on demand)
    size_t colors_bytes = 0;
    float* running = nullptr;  // per-slot running sums between launches of one frame
    size_t running_bytes = 0;
    DWorld w{};
    const DWorld* wdev = nullptr;
    int32_t node_count = 0, leaf_count = 0, depth = 1;
    int32_t tri_count = 0, rect_count = 0, material_count = 0, texture_count = 0, sphere_count = 0, box_count = 0;
    int32_t mk_world = 0;  // every node coordinate is 0 or >= 2^-60 in magnitude (ray_pre)
    int32_t tri_prefix = 0;  // leaves [0, tri_prefix): plain triangles, triangle index = leaf index (walk_leaf_record)
    int32_t tri_prefix_mat = 0, tri_prefix_w = 0;  // their material and leaf_info.w (leaf_info_of)
    int32_t sah_nodes = 0;  // nodes of the SAH tree, 0: the world takes the reference tree only (§5.6)
    bool sah_folded = false;  // its node records are the two-children walk's (plain-sphere worlds)
    int32_t leaf_kinds = LK_ANY;  // LK_*: the traversal loop the world's leaves need
    int32_t tex_kinds = TX_ANY;   // TX_*: the texture code the world's textures need
    int cus = 0;
    int lds_max = 64 * 1024;  // hipDeviceAttributeMaxSharedMemoryPerBlock
    int lds_cu = 160 * 1024;  // hipDeviceAttributeMaxSharedMemoryPerMultiprocessor
    TuneState* tune = nullptr;  // in-frame threshold tuning state
    // work order (render_frame): per-slot costs accumulated over frames of one partition shape,
    // and the tile order derived from them after each frame
    uint32_t* slot_cost = nullptr;
    uint32_t* tile_buf = nullptr;  // 4 x n_tiles: cost, index, sorted cost, permutation
    void* sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    uint64_t order_key[10] = {};   // partition shape + workload (seed, spp, max_depth, mode) of the costs
    hipEvent_t done = nullptr;     // end of the last frame rendered with this world's buffers
    bool done_recorded = false;
    uint32_t order_tiles = 0;
    bool order_valid = false;      // tile permutation computed for order_key
    // LDS mode, leaf kinds, texture kinds, tree, GEN (generic leaf tables in LDS), WP (whole-pixel items) of
    // the last render
    int32_t last_kernel[6] = {-1, -1, -1, -1, -1, -1};
    // the last frame: render launches, whole-pixel items, the default threshold, in-frame tuning on
    int32_t last_frame[4] = {-1, -1, -1, 0};
};

// experiment builds (-DRTW_WAVE_TIMING): per-wave start / end / queue-empty wall clocks (100 MHz) of
// the last launch (tools/wave_timing.py; the first launch's queue-empty stamps are not valid)
extern "C" RTW_API int rtw_debug_wave_times(unsigned long long* out24576) {
#ifdef RTW_WAVE_TIMING
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out24576, HIP_SYMBOL(rtw_wave_times), 3 * 8192 * sizeof(unsigned long long)));
    return RTW_OK;
#else
    (void)out24576;
    return rtw::fail(RTW_ERR_UNSUPPORTED, "built without RTW_WAVE_TIMING");
#endif
}
// experiment builds: per-wave drain counters of the launches since the last call (busy lanes when
// the queue ran dry: max; samples finished after it, their bounces: sums; max bounces), then reset
extern "C" RTW_API int rtw_debug_wave_extra(unsigned long long* out65536) {
#ifdef RTW_WAVE_TIMING
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out65536, HIP_SYMBOL(rtw_wave_extra), 8 * 8192 * sizeof(unsigned long long)));
    std::vector<unsigned long long> z(8 * 8192, 0);
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(rtw_wave_extra), z.data(), z.size() * sizeof(unsigned long long)));
    return RTW_OK;
#else
    (void)out65536;
    return rtw::fail(RTW_ERR_UNSUPPORTED, "built without RTW_WAVE_TIMING");
#endif
}

// tests: the block-shared drain's counters (rtw_drain_counts: rays posted, traced by helper waves, traced by
// their owners) summed over the device's launches since the last reset; reset != 0 zeroes them after reading
extern "C" RTW_API int rtw_debug_drain_counts(int device, unsigned long long* out3, int reset) {
    if (!out3) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out3, HIP_SYMBOL(rtw_drain_counts), 3 * sizeof(unsigned long long)));
    if (reset) {
        unsigned long long z[3] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(rtw_drain_counts), z, sizeof(z)));
    }
    return RTW_OK;
}

// experiment builds (-DRTW_PHASE_TIMING): read and reset the phase cycle sums
extern "C" RTW_API int rtw_debug_phase_cycles(unsigned long long* out8) {
#ifdef RTW_PHASE_TIMING
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out8, HIP_SYMBOL(rtw_phase_cycles), 8 * sizeof(unsigned long long)));
    unsigned long long z[8] = {};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(rtw_phase_cycles), z, sizeof(z)));
    return RTW_OK;
#else
    (void)out8;
    return rtw::fail(RTW_ERR_UNSUPPORTED, "built without RTW_PHASE_TIMING");
#endif
}

extern "C" RTW_API int rtw_device_count(int* count) {
    if (!count) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return RTW_OK;
}

extern "C" RTW_API int rtw_world_upload(const rtw_world* w, int device, rtw_gpu_world** out) {
    if (!out) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null out");
    int depth = 0;
    const int v = check_world(w, &depth);
    if (v != RTW_OK) return v;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return rtw::fail(RTW_ERR_NO_DEVICE, "no HIP device: the MI355X path requires a GPU (there is no CPU fallback)");
    if (device < 0 || device >= ndev) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "device index out of range");
    HIP_TRY(hipSetDevice(device));

    Layout L;
    // nodes
    // nodes: two SoA float4 halves {min.xyz, max.x}, {max.y, max.z, left<<2|axis, right}
    std::vector<float4> na((size_t)std::max(1, w->node_count)), nb((size_t)std::max(1, w->node_count));
    for (int i = 0; i < w->node_count; ++i) {
        const rtw_bvh_node& n = w->nodes[i];
        na[(size_t)i] = make_float4(n.min[0], n.min[1], n.min[2], n.max[0]);
        nb[(size_t)i] = make_float4(n.max[1], n.max[2], ibits((int32_t)((uint32_t)n.left << 2) | n.axis), ibits(n.right));
    }
    const size_t o_na = L.push(na.data(), na.size() * sizeof(float4));
    const size_t o_nb = L.push(nb.data(), nb.size() * sizeof(float4));
    // proximity-cull constants (rtw_cull.h); RTW_NO_CULL=1 in the environment disables the cull
    // (every node k = +inf: the reference traversal alone), for audits
    std::vector<float> km((size_t)std::max(1, w->node_count) * 2, 0.0f);
    {
        const char* nc = std::getenv("RTW_NO_CULL");
        rtw_cull_prepare(w, km.data(), nc && nc[0] && nc[0] != '0');
    }
    const size_t o_km = L.push(km.data(), km.size() * sizeof(float));
    // leaf records for the traversal: plain spheres inline, everything else tagged NaN
    std::vector<float4> lf((size_t)w->leaf_count);
    for (int i = 0; i < w->leaf_count; ++i) {
        const rtw_leaf& l = w->leaves[i];
        if (l.geom_kind == RTW_GEOM_SPHERE && l.flags == 0) {
            const rtw_sphere& sp = w->spheres[l.geom_index];
            lf[(size_t)i] = make_float4(sp.center[0], sp.center[1], sp.center[2], sp.radius);
        } else {
            // w = NaN: not a plain sphere; x = 1 tags a plain triangle, 2 a plain rect (index in y)
            // (3: a sphere under an Animation wrapper only, the traversal's fast path for it)
            const int tag = l.flags == RTW_LEAF_ANIMATION && l.geom_kind == RTW_GEOM_SPHERE ? 3
                            : l.flags != 0                     ? 0
                            : l.geom_kind == RTW_GEOM_TRIANGLE ? 1
                            : l.geom_kind == RTW_GEOM_RECT     ? 2
                                                               : 0;
            lf[(size_t)i] = make_float4(ibits(tag), ibits(l.geom_index), 0.0f, ibits(0x7FC00000));
        }
    }
    const size_t o_lf = L.push(lf.data(), lf.size() * sizeof(float4));
    // leaves
    std::vector<int4> li((size_t)w->leaf_count);
    std::vector<float4> lx((size_t)w->leaf_count * 3);
    for (int i = 0; i < w->leaf_count; ++i) {
        const rtw_leaf& l = w->leaves[i];
        li[(size_t)i] = make_int4(l.geom_kind, l.geom_index, l.material,
                                  (int)(l.flags | (material_reads_uv(w, l.material) ? RTW_DLEAF_UV : 0u)));
        lx[3 * (size_t)i] = make_float4(l.neg_inv_density, l.offset[0], l.offset[1], l.offset[2]);
        lx[3 * (size_t)i + 1] = make_float4(l.y_sin, l.y_cos, l.velocity[0], l.velocity[1]);
        lx[3 * (size_t)i + 2] = make_float4(l.velocity[2], 0.0f, 0.0f, 0.0f);
    }
    const size_t o_li = L.push(li.data(), li.size() * sizeof(int4));
    const size_t o_lx = L.push(lx.data(), lx.size() * sizeof(float4));
    // primitives
    std::vector<float4> sp((size_t)w->sphere_count);
    for (int i = 0; i < w->sphere_count; ++i) {
        const rtw_sphere& s = w->spheres[i];
        sp[(size_t)i] = make_float4(s.center[0], s.center[1], s.center[2], s.radius);
    }
    std::vector<float4> rc((size_t)w->rect_count * 2);
    for (int i = 0; i < w->rect_count; ++i) {
        const rtw_rect& r = w->rects[i];
        rc[2 * (size_t)i] = make_float4(r.dist, r.r0[0], r.r0[1], r.r1[0]);
        rc[2 * (size_t)i + 1] = make_float4(r.r1[1], ibits(r.plane), 0.0f, 0.0f);
    }
    std::vector<float4> bx((size_t)w->box_count * 2);
    for (int i = 0; i < w->box_count; ++i) {
        const rtw_box& b = w->boxes[i];
        bx[2 * (size_t)i] = make_float4(b.min[0], b.min[1], b.min[2], b.max[0]);
        bx[2 * (size_t)i + 1] = make_float4(b.max[1], b.max[2], 0.0f, 0.0f);
    }
    std::vector<float4> tp((size_t)w->triangle_count * 4), ta((size_t)w->triangle_count * 4);
    for (int i = 0; i < w->triangle_count; ++i) {
        const rtw_triangle& t = w->triangles[i];
        const float (*p)[3] = t.positions;
        const TriFast f = tri_prepare(v3(p[0][0], p[0][1], p[0][2]), v3(p[1][0], p[1][1], p[1][2]),
                                      v3(p[2][0], p[2][1], p[2][2]));
        tp[4 * (size_t)i] = make_float4(f.p0.x, f.p0.y, f.p0.z, f.n.x);
        tp[4 * (size_t)i + 1] = make_float4(f.n.y, f.n.z, f.vt1.x, f.vt1.y);
        tp[4 * (size_t)i + 2] = make_float4(f.vt1.z, f.den1, f.vt2.x, f.vt2.y);
        tp[4 * (size_t)i + 3] = make_float4(f.vt2.z, f.den2, f.y1, f.y2);
        const float (*n)[3] = t.normals;
        const float (*u)[2] = t.uvs;
        ta[4 * (size_t)i] = make_float4(n[0][0], n[0][1], n[0][2], n[1][0]);
        ta[4 * (size_t)i + 1] = make_float4(n[1][1], n[1][2], n[2][0], n[2][1]);
        ta[4 * (size_t)i + 2] = make_float4(n[2][2], u[0][0], u[0][1], u[1][0]);
        ta[4 * (size_t)i + 3] = make_float4(u[1][1], u[2][0], u[2][1], 0.0f);
    }
    const size_t o_sp = L.push(sp.data(), sp.size() * sizeof(float4));
    const size_t o_rc = L.push(rc.data(), rc.size() * sizeof(float4));
    const size_t o_bx = L.push(bx.data(), bx.size() * sizeof(float4));
    const size_t o_tp = L.push(tp.data(), tp.size() * sizeof(float4));
    const size_t o_ta = L.push(ta.data(), ta.size() * sizeof(float4));
    // materials / textures / images / perlin
    // each image's first texel (the texel array below holds the images in order)
    std::vector<size_t> texel_off((size_t)std::max(1, w->image_count), 0);
    for (int i = 1; i < w->image_count; ++i)
        texel_off[(size_t)i] = texel_off[(size_t)i - 1] + (size_t)w->images[i - 1].width * (size_t)w->images[i - 1].height;
    std::vector<int4> mt((size_t)w->material_count);
    for (int i = 0; i < w->material_count; ++i) {
        const rtw_material& m = w->materials[i];
        mt[(size_t)i] = make_int4(m.kind, m.texture, (int)fbits(m.fuzz), (int)fbits(m.index_of_refraction));
        // a Lambertian, Isotropic or DiffuseLight over an image texture carries the image (RTW_DMAT_IMAGE)
        if ((m.kind == RTW_MAT_LAMBERT || m.kind == RTW_MAT_ISOTROPIC || m.kind == RTW_MAT_DIFFUSE_LIGHT) &&
            w->textures[m.texture].kind == RTW_TEX_IMAGE) {
            const rtw_image& I = w->images[w->textures[m.texture].image];
            if (I.width < 65536 && I.height < 65536)
                mt[(size_t)i] = make_int4(m.kind | RTW_DMAT_IMAGE, m.texture, (int)texel_off[(size_t)w->textures[m.texture].image],
                                          (int)(((uint32_t)I.width << 16) | (uint32_t)I.height));
        }
    }
    std::vector<int4> tx((size_t)w->texture_count * 3);
    for (int i = 0; i < w->texture_count; ++i) {
        const rtw_texture& t = w->textures[i];
        // an image texture's first record: {kind, texel offset, width, height} (texture_sample reads no other)
        tx[3 * (size_t)i] = t.kind == RTW_TEX_IMAGE
                                ? make_int4(t.kind, (int)texel_off[(size_t)t.image], w->images[t.image].width,
                                            w->images[t.image].height)
                                : make_int4(t.kind, (int)fbits(t.color[0]), (int)fbits(t.color[1]), (int)fbits(t.color[2]));
        tx[3 * (size_t)i + 1] = make_int4((int)fbits(t.inv_frequency), t.even, t.odd, (int)fbits(t.scale));
        tx[3 * (size_t)i + 2] = make_int4(t.perlin, t.image, 0, 0);
    }
    std::vector<int4> im((size_t)std::max(1, w->image_count));
    std::vector<uint32_t> texels;
    for (int i = 0; i < w->image_count; ++i) {
        const rtw_image& I = w->images[i];
        im[(size_t)i] = make_int4((int)texels.size(), I.width, I.height, 0);
        const size_t n = (size_t)I.width * (size_t)I.height;
        for (size_t k = 0; k < n; ++k)
            texels.push_back((uint32_t)I.rgb[3 * k] | ((uint32_t)I.rgb[3 * k + 1] << 8) | ((uint32_t)I.rgb[3 * k + 2] << 16));
    }
    if (texels.empty()) texels.push_back(0);
    std::vector<float> pr((size_t)std::max(1, w->perlin_count) * 768);
    std::vector<uint32_t> pp((size_t)std::max(1, w->perlin_count) * 768);
    std::vector<int> pb((size_t)std::max(1, w->perlin_count));
    for (int i = 0; i < w->perlin_count; ++i) {
        const rtw_perlin& P = w->perlins[i];
        std::memcpy(&pr[(size_t)i * 768], P.ranvec, sizeof(P.ranvec));
        std::memcpy(&pp[(size_t)i * 768], P.perm_x, sizeof(P.perm_x));
        std::memcpy(&pp[(size_t)i * 768 + 256], P.perm_y, sizeof(P.perm_y));
        std::memcpy(&pp[(size_t)i * 768 + 512], P.perm_z, sizeof(P.perm_z));
        pb[(size_t)i] = P.bits;
    }
    const size_t o_mt = L.push(mt.data(), mt.size() * sizeof(int4));
    const size_t o_tx = L.push(tx.data(), tx.size() * sizeof(int4));
    const size_t o_im = L.push(im.data(), im.size() * sizeof(int4));
    const size_t o_te = L.push(texels.data(), texels.size() * sizeof(uint32_t));
    const size_t o_pr = L.push(pr.data(), pr.size() * sizeof(float));
    const size_t o_pp = L.push(pp.data(), pp.size() * sizeof(uint32_t));
    const size_t o_pb = L.push(pb.data(), pb.size() * sizeof(int));
    const SahTables sah = build_sah_tables(w);
    const size_t o_sa = sah.ok ? L.push(sah.a.data(), sah.a.size() * sizeof(float4)) : 0;
    const size_t o_sb = sah.ok ? L.push(sah.b.data(), sah.b.size() * sizeof(float4)) : 0;
    const size_t o_sk = sah.ok && !sah.folded ? L.push(sah.km.data(), sah.km.size() * sizeof(float)) : 0;
    const size_t o_lb = sah.ok ? L.push(sah.box.data(), sah.box.size() * sizeof(float4)) : 0;
    const size_t o_lk = sah.ok && !sah.key.empty() ? L.push(sah.key.data(), sah.key.size() * sizeof(uint4)) : 0;

    WorldConst wcst;
    std::memset(&wcst, 0, sizeof(wcst));
    wcst.cam = w->camera;
    wcst.light = w->light;
    wcst.bg = w->background;
    const size_t o_wc = L.push(&wcst, sizeof(wcst));
    DWorld dw_zero;
    std::memset(&dw_zero, 0, sizeof(dw_zero));
    const size_t o_dw = L.push(&dw_zero, sizeof(DWorld));  // filled once the pointers are known

    auto* g = new rtw_gpu_world;
    g->device = device;
    hipError_t e = hipMalloc(&g->arena, L.blob.size());
    if (e != hipSuccess) {
        delete g;
        return rtw::fail(RTW_ERR_OUT_OF_MEMORY, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    e = hipMemcpy(g->arena, L.blob.data(), L.blob.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(g->arena);
        delete g;
        return rtw::fail(RTW_ERR_HIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
    }
    uint8_t* base = (uint8_t*)g->arena;
    DWorld& d = g->w;
    d.node_a = (const float4*)(base + o_na);
    d.node_b = (const float4*)(base + o_nb);
    d.node_km = (const float2*)(base + o_km);
    d.leaf_fast = (const float4*)(base + o_lf);
    d.leaf_info = (const int4*)(base + o_li);
    d.leaf_xf = (const float4*)(base + o_lx);
    d.spheres = (const float4*)(base + o_sp);
    d.rects = (const float4*)(base + o_rc);
    d.boxes = (const float4*)(base + o_bx);
    d.tri_fast = (const float4*)(base + o_tp);
    d.tri_attr = (const float4*)(base + o_ta);
    d.materials = (const int4*)(base + o_mt);
    d.textures = (const int4*)(base + o_tx);
    d.images = (const int4*)(base + o_im);
    d.texels = (const uint32_t*)(base + o_te);
    d.perlin_ranvec = (const float*)(base + o_pr);
    d.perlin_perm = (const uint32_t*)(base + o_pp);
    d.perlin_bits = (const int*)(base + o_pb);
    d.root = w->root;
    if (sah.ok) {
        d.sah_a = (const float4*)(base + o_sa);
        d.sah_b = (const float4*)(base + o_sb);
        d.leaf_box = (const float4*)(base + o_lb);
        d.leaf_key = o_lk ? (const uint4*)(base + o_lk) : nullptr;
        d.sah_root = sah.root;
        d.sah_root_c2 = sah.root_c2;
        d.sah_k = sah.k;
        d.sah_km = sah.folded ? nullptr : (const float2*)(base + o_sk);
    }
    d.has_light = w->has_light;
    d.wc = (const WorldConst*)(base + o_wc);
    e = hipMemcpy(base + o_dw, &g->w, sizeof(DWorld), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(g->arena);
        delete g;
        return rtw::fail(RTW_ERR_HIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
    }
    g->wdev = (const DWorld*)(base + o_dw);
    g->node_count = w->node_count;
    g->leaf_count = w->leaf_count;
    g->depth = std::max(1, depth);
    if (sah.ok) {
        g->sah_nodes = (int32_t)sah.a.size();
        g->sah_folded = sah.folded;
        g->depth = std::max(g->depth, sah.depth);
    }
    g->tri_count = w->triangle_count;
    g->tri_prefix = tri_prefix_of(w);
    if (g->tri_prefix > 0) {
        g->tri_prefix_mat = li[0].z;
        g->tri_prefix_w = li[0].w;
    }
    g->rect_count = w->rect_count;
    g->sphere_count = w->sphere_count;
    g->box_count = w->box_count;
    g->material_count = w->material_count;
    g->texture_count = w->texture_count;
    g->mk_world = 1;
    g->leaf_kinds = LK_SPHERES;
    g->tex_kinds = TX_SOLID;
    for (int i = 0; i < w->texture_count; ++i)
        if (w->textures[i].kind != RTW_TEX_SOLID) g->tex_kinds = TX_ANY;
    for (int i = 0; i < w->leaf_count; ++i) {
        const rtw_leaf& l = w->leaves[i];
        const int need = (l.flags & RTW_LEAF_VOLUME)                   ? LK_ANY
                         : (l.flags != 0 || l.geom_kind == RTW_GEOM_BOX) ? LK_WRAPPED
                         : l.geom_kind == RTW_GEOM_RECT                 ? LK_PLAIN
                         : l.geom_kind == RTW_GEOM_TRIANGLE             ? LK_TRIS
                                                                        : LK_SPHERES;
        g->leaf_kinds = std::max(g->leaf_kinds, (int32_t)need);
    }
    // a plain-sphere world beyond the folded records' 2^14 nodes / leaves keeps an unfolded SAH tree: the
    // triangle loop (which tests plain spheres too) walks it with the one-child walk
    if (g->leaf_kinds == LK_SPHERES && g->sah_nodes > 0 && !g->sah_folded) g->leaf_kinds = LK_TRIS;
    for (int i = 0; i < w->node_count; ++i)
        for (int k = 0; k < 3; ++k)
            for (float c : {w->nodes[i].min[k], w->nodes[i].max[k]})
                if (!(c == 0.0f || std::fabs(c) >= 0x1p-60f)) g->mk_world = 0;
    // rect planes: the Markstein rect test (rect_t_mk) divides dist - o_n like a node coordinate
    for (int i = 0; i < w->rect_count; ++i)
        if (!(w->rects[i].dist == 0.0f || std::fabs(w->rects[i].dist) >= 0x1p-60f)) g->mk_world = 0;
    // audits: RTW_NO_MARKSTEIN=1 makes every ray take the true-division slab test (and the traversal
    // loop that carries it)
    if (const char* e = std::getenv("RTW_NO_MARKSTEIN"))
        if (e[0] && e[0] != '0') g->mk_world = 0;
    (void)hipDeviceGetAttribute(&g->cus, hipDeviceAttributeMultiprocessorCount, device);
    if (g->cus <= 0) g->cus = 256;
    {
        int lm = 0;
        if (hipDeviceGetAttribute(&lm, hipDeviceAttributeMaxSharedMemoryPerBlock, device) == hipSuccess && lm > 0)
            g->lds_max = lm;
        if (hipDeviceGetAttribute(&lm, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device) == hipSuccess && lm > 0)
            g->lds_cu = lm;
    }
    e = hipMalloc(&g->tune, sizeof(TuneState));
    if (e == hipSuccess) e = hipMemset(g->tune, 0, sizeof(TuneState));
    if (e == hipSuccess) e = hipMalloc(&g->queue, RTW_QUEUE_BYTES);
    if (e != hipSuccess) {
        (void)hipFree(g->arena);
        delete g;
        return rtw::fail(RTW_ERR_OUT_OF_MEMORY, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    *out = g;
    return RTW_OK;
}

// Debug (tools/ only, not part of include/rtw.h): the SAH tree build_sah_tables makes for a world --
// out[0] nodes, out[1] depth, out[2] expected node tests and out[3] expected leaf tests per ray by the
// surface-area measure (each node's and leaf reference's box area over the root's), out[4] 1 if the
// world qualifies for the SAH path.  No GPU needed.
extern "C" RTW_API int rtw_debug_sah_tree(const rtw_world* w, double* out) {
    if (!w || !out) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    const SahTables S = build_sah_tables(w);
    for (int i = 0; i < 10; ++i) out[i] = 0.0;
    out[4] = S.ok ? 1.0 : 0.0;
    if (!S.ok) return RTW_OK;
    auto area = [](float4 a, float4 b) {
        const double dx = (double)a.w - a.x, dy = (double)b.x - a.y, dz = (double)b.y - a.z;
        return dx * dy + dy * dz + dz * dx;
    };
    // measured over the subtree of the root's internal child when the other child is a leaf (suzanne's
    // ground sphere would otherwise make every mesh node's area vanish against the root's)
    // a node's children in either record format (build_sah_tables)
    auto kids = [&](int32_t i, int c) {
        const int32_t kb = (int32_t)fbits(S.b[(size_t)i].z);
        if (!S.folded) return c ? (int32_t)fbits(S.b[(size_t)i].w) : kb >> 2;
        return c ? kb >> 17 : (int32_t)((uint32_t)kb << 15) >> 17;
    };
    int32_t root = S.root;
    if (root >= 0) {
        const int32_t l = kids(root, 0), r = kids(root, 1);
        if ((l < 0) != (r < 0)) root = l >= 0 ? l : r;
    }
    double nodes = 1.0, leaves = 0.0;  // the top node's test; a child is tested when its parent passes
    if (root >= 0) {
        const double ar = area(S.a[(size_t)root], S.b[(size_t)root]);
        std::vector<int32_t> todo{root};
        while (!todo.empty()) {
            const int32_t i = todo.back();
            todo.pop_back();
            const double an = area(S.a[(size_t)i], S.b[(size_t)i]) / ar;
            for (int c = 0; c < 2; ++c) {
                const int32_t ch = kids(i, c);
                (ch < 0 ? leaves : nodes) += an;
                if (ch >= 0) todo.push_back(ch);
            }
        }
    }
    out[0] = (double)S.a.size();
    out[1] = (double)S.depth;
    out[2] = nodes;
    out[3] = leaves;
    // experiment estimates (out[5..9]): the two-children walk's steps and box tests, and those of the
    // same tree collapsed to 4 children per node (each child replaced by its children, largest box
    // first, until 4): steps, box tests, leaf tests, all per ray by the area measure
    if (root >= 0) {
        const double ar = area(S.a[(size_t)root], S.b[(size_t)root]);
        double st2 = 0.0, bx2 = 0.0, st4 = 0.0, bx4 = 0.0, lf4 = 0.0;
        std::vector<int32_t> todo{root};
        while (!todo.empty()) {
            const int32_t i = todo.back();
            todo.pop_back();
            const double an = area(S.a[(size_t)i], S.b[(size_t)i]) / ar;
            st2 += an;
            for (int c = 0; c < 2; ++c) {
                const int32_t ch = kids(i, c);
                if (ch >= 0) {
                    bx2 += an;
                    todo.push_back(ch);
                }
            }
        }
        std::vector<int32_t> todo4{root};
        while (!todo4.empty()) {
            const int32_t i = todo4.back();
            todo4.pop_back();
            const double an = area(S.a[(size_t)i], S.b[(size_t)i]) / ar;
            std::vector<int32_t> ch{kids(i, 0), kids(i, 1)};
            while (ch.size() < 4) {
                int best = -1;
                double ba = -1.0;
                for (size_t c = 0; c < ch.size(); ++c)
                    if (ch[c] >= 0 && area(S.a[(size_t)ch[c]], S.b[(size_t)ch[c]]) > ba)
                        ba = area(S.a[(size_t)ch[c]], S.b[(size_t)ch[c]]), best = (int)c;
                if (best < 0) break;
                const int32_t x = ch[(size_t)best];
                ch.erase(ch.begin() + best);
                ch.push_back(kids(x, 0));
                ch.push_back(kids(x, 1));
            }
            st4 += an;
            for (int32_t c : ch) {
                if (c >= 0) {
                    bx4 += an;
                    todo4.push_back(c);
                } else {
                    lf4 += an;
                }
            }
        }
        out[5] = st2;
        out[6] = bx2;
        out[7] = st4;
        out[8] = bx4;
        out[9] = lf4;
    }
    return RTW_OK;
}

extern "C" RTW_API int rtw_world_tuning(rtw_gpu_world* g, int* trace_min) {
    if (!g || !trace_min) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    HIP_TRY(hipSetDevice(g->device));
    int v = 0;
    HIP_TRY(hipMemcpy(&v, &g->tune->chosen, sizeof(int), hipMemcpyDeviceToHost));
    *trace_min = v;
    return RTW_OK;
}

extern "C" RTW_API int rtw_world_kernel(rtw_gpu_world* g, int* lds_mode, int* leaf_kinds, int* tex_kinds, int* tree) {
    if (!g || !lds_mode || !leaf_kinds || !tex_kinds || !tree) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    *lds_mode = g->last_kernel[0];
    *leaf_kinds = g->last_kernel[1];
    *tex_kinds = g->last_kernel[2];
    *tree = g->last_kernel[3];
    return RTW_OK;
}

extern "C" RTW_API int rtw_world_kernel_name(rtw_gpu_world* g, char* buf, int cap) {
    if (!g || !buf || cap < 1) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    char s[64] = "";
    if (g->last_kernel[0] >= 0)  // the product kernel: render_kernel<STATS = false, LDS, LK, TX, GEN, WP>
        std::snprintf(s, sizeof(s), "render_kernel<false, %d, %d, %d, %s, %s>", g->last_kernel[0], g->last_kernel[1],
                      g->last_kernel[2], g->last_kernel[4] ? "true" : "false", g->last_kernel[5] ? "true" : "false");
    if ((int)std::strlen(s) >= cap) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "buffer too small");
    std::memcpy(buf, s, std::strlen(s) + 1);
    return RTW_OK;
}

extern "C" RTW_API int rtw_world_last_frame(rtw_gpu_world* g, int* launches, int* whole_pixel, int* trace_min) {
    if (!g || !launches || !whole_pixel || !trace_min) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    *launches = g->last_frame[0];
    *whole_pixel = g->last_frame[1];
    *trace_min = g->last_frame[2];
    if (g->last_frame[3]) {  // the kernel takes the world's tuned threshold once there is one
        HIP_TRY(hipSetDevice(g->device));
        int v = 0;
        HIP_TRY(hipMemcpy(&v, &g->tune->chosen, sizeof(int), hipMemcpyDeviceToHost));
        if (v > 0) *trace_min = v;
    }
    return RTW_OK;
}

extern "C" RTW_API int rtw_world_release(rtw_gpu_world* g) {
    if (!g) return RTW_OK;
    (void)hipSetDevice(g->device);
    if (g->arena) (void)hipFree(g->arena);
    if (g->queue) (void)hipFree(g->queue);
    if (g->colors) (void)hipFree(g->colors);
    if (g->tune) (void)hipFree(g->tune);
    if (g->slot_cost) (void)hipFree(g->slot_cost);
    if (g->tile_buf) (void)hipFree(g->tile_buf);
    if (g->sort_tmp) (void)hipFree(g->sort_tmp);
    if (g->running) (void)hipFree(g->running);
    if (g->done) (void)hipEventDestroy(g->done);
    delete g;
    return RTW_OK;
}

namespace {

int make_args(const rtw_gpu_world* g, const rtw_render_params* p, KArgs& A) {
    if (!g || !p) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    if (p->width < 2 || p->height < 2)  // rendering.rs:132-138 divides by (W-1), (H-1)
        return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "image width and height must be >= 2");
    if (p->samples_per_pixel < 1) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "samples_per_pixel must be >= 1");
    if (p->render_mode != RTW_MODE_DEFAULT && p->render_mode != RTW_MODE_NORMALS)
        return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "unknown render mode");
    const int tw = p->tile_width > 0 ? p->tile_width : 8;
    const int th = p->tile_height > 0 ? p->tile_height : 8;
    const int pc = p->part_count > 0 ? p->part_count : 1;
    if (p->part_index < 0 || p->part_index >= pc) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "part_index out of range");
    if (p->thread_count < 0) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "thread_count must be >= 0");
    if (p->reserved0 != 0) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "reserved0 must be 0");
    std::memset(&A, 0, sizeof(A));
    A.thread_count = std::max(1, p->thread_count);
    A.w = g->w;
    A.width = p->width;
    A.height = p->height;
    A.spp = p->samples_per_pixel;
    A.max_depth = p->max_depth;
    A.mode = p->render_mode;
    A.layout = p->layout;
    A.tile_w = tw;
    A.tile_h = th;
    A.tiles_x = (p->width + tw - 1) / tw;
    const int tiles_y = (p->height + th - 1) / th;
    A.n_tiles = A.tiles_x * tiles_y;
    A.part_index = p->part_index;
    A.part_count = pc;
    const int64_t owned = A.n_tiles > p->part_index ? (A.n_tiles - p->part_index + pc - 1) / pc : 0;
    if (owned * tw * th >= (int64_t)0xFFFFFFFF) return rtw::fail(RTW_ERR_UNSUPPORTED, "partition too large");
    A.total = (uint32_t)(owned * tw * th);
    A.node_count = g->node_count;
    A.leaf_count = g->leaf_count;
    A.mk_world = g->mk_world;
    A.tri_count = g->tri_count;
    A.rect_count = g->rect_count;
    A.material_count = g->material_count;
    A.sphere_count = g->sphere_count;
    A.box_count = g->box_count;
    A.texture_count = g->texture_count;
    A.sh_li = A.sh_mat = A.sh_tex0 = A.sh_box = -1;
    A.sh_xf = A.sh_sph = A.sh_bx = A.sh_rect = -1;
    A.queue = g->queue;
    A.wdev = g->wdev;
    A.trace_min = 32;
    A.stats_tree = 0;
    if (const char* e = getenv("RTW_TRACE_MIN")) A.trace_min = atoi(e);
    A.seed_key = rtw_seed_key(p->seed);
    A.sx = 1.0f / (float)(p->width - 1);
    A.sy = 1.0f / (float)(p->height - 1);
    A.ux = rtw_uniform_new(0.0f, 1.0f / (float)(p->width - 1));
    A.uy = rtw_uniform_new(0.0f, 1.0f / (float)(p->height - 1));
    return RTW_OK;
}

// Launch the persistent render kernel: zero the pixel queue, stage the scene in LDS when it
// fits, size the grid to the resident block count.
enum LaunchKind { LK_RENDER, LK_STATS };
size_t env_size(const char* name, size_t dflt);
int launch_render(rtw_gpu_world* g, KArgs& A, int kind, hipStream_t stream) {
    const bool stats = kind == LK_STATS;
    const bool ktree = stats && A.stats_tree == 1;  // count the product kernel's own traversal
    // the leaf and texture kinds the world needs; RTW_LEAF_KINDS=4 / RTW_TEX_KINDS=1 force the
    // generic code (audits)
    int lk = g->leaf_kinds, tx = g->tex_kinds;
    if (const char* e = std::getenv("RTW_LEAF_KINDS")) lk = std::max(lk, std::min(4, std::atoi(e)));
    if (const char* e = std::getenv("RTW_TEX_KINDS")) tx = std::max(tx, std::min(1, std::atoi(e)));
    // the SAH tree (§5.6) replaces the reference tree in LDS; the counting variant keeps the latter
    // (a plain-sphere world's SAH records are the two-children walk's: another leaf-kind loop, forced by
    // RTW_LEAF_KINDS, takes the reference tree)
    const bool sah = (!stats || ktree) && g->sah_nodes > 0 && g->mk_world && lk <= LK_WRAPPED &&
                     g->sah_folded == (lk == LK_SPHERES);
    A.sah = sah ? 1 : 0;
    // the drain's cooperative trace (coop_solve): worlds small enough to test every leaf per ray
    A.coop_max = g->leaf_count <= RTW_COOP_LEAVES ? (int32_t)env_size("RTW_COOP_MAX", RTW_COOP_MAX) : 0;
    if (const char* e = std::getenv("RTW_COOP_MAX"))
        if (e[0] == '0') A.coop_max = 0;
    A.coop_ties = g->leaf_count <= RTW_COOP_LEAVES && g->w.leaf_key != nullptr ? 1 : 0;
    if (const char* e = std::getenv("RTW_COOP_TIES"))
        if (e[0] == '0') A.coop_ties = 0;
    if (const char* e = std::getenv("RTW_COOP_AUDIT"))  // tests only: the DFS-last tied leaf
        if (e[0] == '1' && A.coop_ties) A.coop_ties = 2;
    // a block may take its share of the CU's LDS at the kernel's target occupancy
    // (RTW_MIN_WAVES_PER_SIMD waves on each of 4 SIMDs)
    const int blocks_per_cu = std::max(1, (4 * RTW_MIN_WAVES_PER_SIMD * 64) / RTW_BLOCK);
    size_t cap = std::min({(size_t)RTW_LDS_SCENE_MAX, (size_t)g->lds_max, (size_t)g->lds_cu / blocks_per_cu});
#ifdef RTW_PHASE_TIMING
    cap -= (RTW_BLOCK / 64) * 10 * sizeof(unsigned long long);  // the per-wave phase sums (pt_slot)
#endif
    const size_t stack_bytes = (size_t)g->depth * RTW_BLOCK * sizeof(int32_t);
    const size_t stack16_bytes = stack_bytes / 2;  // 16-bit entries
    const char* lds_mode_env = std::getenv("RTW_LDS_MODE");  // audits: cap the mode
    A.node_count = sah ? g->sah_nodes : g->node_count;
    // the LK template argument of the kernel launch_render picks below (the counting variant of a world
    // without the SAH walk runs the LK_ANY loop): its stack entries are the ones the LDS must hold, and
    // only its triangle loops skip the triangle prefix's leaf records (walk_leaf_record)
    const int kernel_lk = stats && !sah ? (int)LK_ANY : lk;
    A.tri_prefix = kernel_lk == LK_TRIS ? g->tri_prefix : 0;
    A.tri_stride = kernel_lk == LK_TRIS ? std::max(1, g->tri_count) : RTW_TRI_SOA;  // tri_soa_stride
    const size_t tri_bytes = (size_t)4 * A.tri_stride * sizeof(float4);  // mode 2: component-major (load_tri_soa)
    // LDS scene: [node_a n][node_b n][leaf records L - tri_prefix][cull constants (n + 1) / 2, not in the
    // plain-sphere SAH tree][rects 2R] (+ the triangle records in mode 2)
    const size_t scene_bytes =
        (size_t)(2 * A.node_count + g->leaf_count - A.tri_prefix + (sah && lk == LK_SPHERES ? 0 : (A.node_count + 1) / 2) +
                 2 * g->rect_count) * sizeof(float4);
    A.fast_off = 2 * A.node_count - A.tri_prefix;  // where leaf 0's record would be
    if (A.fast_off < 0) return rtw::fail(RTW_ERR_UNSUPPORTED, "triangle prefix longer than the node records");
    int mode = 0;
    // 16-bit stack entries (traverse's StackEntry): worlds of < 2^15 nodes (both trees) and leaves
    const bool small = g->leaf_count < 32768 && A.node_count < 32768 && g->node_count < 32768;
    const size_t stack1_bytes = (size_t)stack_entry_bytes(1, kernel_lk) * g->depth * RTW_BLOCK;  // mode 1
    if (g->tri_count > 0 && g->tri_count <= A.tri_stride && small &&
        scene_bytes + tri_bytes + stack16_bytes + RTW_MB_WORDS * sizeof(uint32_t) <= cap)
        mode = 2;
    else if (scene_bytes + stack1_bytes <= cap && (small || stack_entry_bytes(1, kernel_lk) == 4)) mode = 1;
    if (lds_mode_env) mode = std::min(mode, std::atoi(lds_mode_env));
    size_t lds = (mode >= 1 ? scene_bytes : 0) + (mode == 2 ? tri_bytes + stack16_bytes : mode == 1 ? stack1_bytes : stack_bytes);
    // shading tables after the scene when they fit too (RTW_NO_SHADE_LDS=1: keep them in HBM / L2)
    const int32_t scene_f4 = (int32_t)((scene_bytes + (mode == 2 ? tri_bytes : 0)) / sizeof(float4));
    // the texture table (texture_sample): first records for solid-texture kernels, all three records for
    // the other non-GEN kernels (the counting variants are TX_ANY, non-GEN), none for the GEN kernels
    const char* ngl = std::getenv("RTW_NO_GEN_LDS");
    const bool gen_wanted = !stats && lk >= LK_WRAPPED && !(ngl && ngl[0] && ngl[0] != '0');
    const int tex_recs = (stats || tx != TX_SOLID) ? (gen_wanted ? 0 : 3) : 1;
    // (the leaf_info table from leaf tri_prefix on: the prefix's is made up, leaf_info_of)
    const int32_t n_li = g->leaf_count - A.tri_prefix;
    const size_t sh_bytes = (size_t)(n_li + A.material_count + tex_recs * A.texture_count) * sizeof(int4);
    const char* nsl = std::getenv("RTW_NO_SHADE_LDS");
    const char* ncs = std::getenv("RTW_NO_COOP_SHARE");
    // the shared drain's mailbox (below) keeps its 144 B ahead of the tables
    const bool mb_want = !stats && mode >= 1 && sah && lk == LK_TRIS && A.coop_max > 0 && g->depth >= 1 &&
                         !(ncs && ncs[0] && ncs[0] != '0');
    const size_t mb_bytes = mb_want ? RTW_MB_WORDS * sizeof(uint32_t) : 0;
    const bool sh = mode >= 1 && lds + sh_bytes + mb_bytes <= cap && !(nsl && nsl[0] && nsl[0] != '0');
    A.sh_li = sh ? scene_f4 - A.tri_prefix : -1;
    if (sh && A.sh_li < 0) return rtw::fail(RTW_ERR_UNSUPPORTED, "triangle prefix longer than the LDS scene");
    A.sh_mat = sh ? scene_f4 + n_li : -1;
    A.sh_tex0 = sh && tex_recs > 0 && A.texture_count > 0 ? scene_f4 + n_li + A.material_count : -1;
    A.tri_prefix_mat = A.tri_prefix > 0 ? g->tri_prefix_mat : 0;
    A.tri_prefix_w = A.tri_prefix > 0 ? g->tri_prefix_w : 0;
    A.stack_off = scene_f4 + (sh ? (int32_t)(sh_bytes / sizeof(int4)) : 0);
    if (sh) lds += sh_bytes;
    // ... and the SAH walk's proof boxes (one read per traced ray, else a dependent L2 read between the
    // walk and shading; RTW_NO_PROOF_LDS=1 keeps them in HBM / L2)
    const size_t box_bytes = (size_t)g->leaf_count * 2 * sizeof(float4);
    const char* npl = std::getenv("RTW_NO_PROOF_LDS");
    A.sh_box = -1;
    if (sh && sah && g->w.leaf_box && lds + box_bytes + mb_bytes <= cap && !(npl && npl[0] && npl[0] != '0')) {
        A.sh_box = A.stack_off;
        A.stack_off += (int32_t)(box_bytes / sizeof(float4));
        lds += box_bytes;
    }
    // ... and the generic leaf path's transforms, spheres and boxes (worlds with wrapped or box leaves, or
    // volumes; RTW_NO_GEN_LDS=1 keeps them in HBM / L2)
    A.sh_xf = A.sh_sph = A.sh_bx = -1;
    A.sh_rect = mode >= 1 ? 2 * A.node_count + g->leaf_count - A.tri_prefix + (sah && lk == LK_SPHERES ? 0 : (A.node_count + 1) / 2)
                          : -1;
    const size_t gen_bytes = (size_t)(3 * g->leaf_count + g->sphere_count + 2 * g->box_count) * sizeof(float4);
    if (sh && lk >= LK_WRAPPED && lds + gen_bytes + mb_bytes <= cap && !(ngl && ngl[0] && ngl[0] != '0')) {
        A.sh_xf = A.stack_off;
        A.sh_sph = A.sh_xf + 3 * g->leaf_count;
        A.sh_bx = A.sh_sph + g->sphere_count;
        A.stack_off += (int32_t)(gen_bytes / sizeof(float4));
        lds += gen_bytes;
    }
    // ... and the shared drain's mailbox after the stack (mb_slot; RTW_NO_COOP_SHARE=1: each wave drains
    // alone).  A wave's stack columns hold depth x (entry bytes) rays of 64 B.
    A.mb_off = -1;
    A.mb_cap = 0;
    const size_t stk_bytes = mode == 2 ? stack16_bytes : mode == 1 ? stack1_bytes : stack_bytes;
    const int stk_entry = stack_entry_bytes(mode, kernel_lk);
    // the allocation holds the kernel's entries, and 16-bit entries hold every node and leaf index
    if ((size_t)stk_entry * g->depth * RTW_BLOCK != stk_bytes || (stk_entry == 2 && !small))
        return rtw::fail(RTW_ERR_UNSUPPORTED, "traversal stack entry width does not match the LDS allocation");
    if (mb_want && lds + RTW_MB_WORDS * sizeof(uint32_t) <= cap) {
        A.mb_off = A.stack_off + (int32_t)(stk_bytes / sizeof(float4));
        A.mb_cap = std::min(64, g->depth * stk_entry);
        if (const char* e = std::getenv("RTW_MB_CAP"))  // tests: fewer posts per batch (the rest walk again)
            A.mb_cap = std::max(1, std::min(A.mb_cap, std::atoi(e)));
        lds += RTW_MB_WORDS * sizeof(uint32_t);
    }
    using KFn = void (*)(KArgs);
    // [whole-pixel items][texture kinds][leaf kinds][LDS mode]
#define RTW_KSET(LK, TX, WP) \
    {render_kernel<false, 0, LK, TX, false, WP>, render_kernel<false, 1, LK, TX, false, WP>, render_kernel<false, 2, LK, TX, false, WP>}
#define RTW_KSET_TX(TX, WP)                                                                                     \
    {RTW_KSET(LK_SPHERES, TX, WP), RTW_KSET(LK_TRIS, TX, WP), RTW_KSET(LK_PLAIN, TX, WP), RTW_KSET(LK_WRAPPED, TX, WP), \
     RTW_KSET(LK_ANY, TX, WP)}
    static const KFn fns[2][2][5][3] = {{RTW_KSET_TX(TX_SOLID, false), RTW_KSET_TX(TX_ANY, false)},
                                        {RTW_KSET_TX(TX_SOLID, true), RTW_KSET_TX(TX_ANY, true)}};
#undef RTW_KSET_TX
#undef RTW_KSET
    static const KFn fns_stats[3] = {render_kernel<true, 0, LK_ANY, TX_ANY>, render_kernel<true, 1, LK_ANY, TX_ANY>,
                                     render_kernel<true, 2, LK_ANY, TX_ANY>};
#define RTW_SSET(LK) {render_kernel<true, 0, LK, TX_ANY>, render_kernel<true, 1, LK, TX_ANY>, render_kernel<true, 2, LK, TX_ANY>}
    static const KFn fns_stats_sah[4][3] = {RTW_SSET(LK_SPHERES), RTW_SSET(LK_TRIS), RTW_SSET(LK_PLAIN),
                                            RTW_SSET(LK_WRAPPED)};
#undef RTW_SSET
    // worlds whose generic leaf tables are in LDS: the GEN variants (leaf kinds 3 and 4, LDS modes 1 and 2)
    // (whole-pixel items at run time: render_body's WPX)
#define RTW_GSET(TX)                                                                                     \
    {{render_kernel<false, 1, LK_WRAPPED, TX, true>, render_kernel<false, 2, LK_WRAPPED, TX, true>}, \
     {render_kernel<false, 1, LK_ANY, TX, true>, render_kernel<false, 2, LK_ANY, TX, true>}}
    static const KFn fns_gen[2][2][2] = {RTW_GSET(TX_SOLID), RTW_GSET(TX_ANY)};
#undef RTW_GSET
    const bool gen = !stats && A.sh_xf >= 0;  // (the counting variant reads the HBM copies)
    if (gen && tx != TX_SOLID && A.sh_tex0 >= 0)  // those kernels compile no LDS texture path (texture_sample)
        return rtw::fail(RTW_ERR_UNSUPPORTED, "GEN kernel with a texture table in LDS");
    const int wp = A.whole_pixel ? 1 : 0;  // (never in the counting variant, render_frame_body)
    const KFn kf = stats ? (sah ? fns_stats_sah[lk][mode] : fns_stats[mode])
                 : gen   ? fns_gen[tx][lk - LK_WRAPPED][mode - 1]
                         : fns[wp][tx][lk][mode];
    if (!stats) {
        g->last_kernel[0] = mode;
        g->last_kernel[1] = lk;
        g->last_kernel[2] = tx;
        g->last_kernel[3] = sah ? 1 : 0;
        g->last_kernel[4] = gen ? 1 : 0;
        g->last_kernel[5] = gen ? 0 : wp;  // (the template argument: GEN kernels take either kind of item)
    }
    const void* fn = (const void*)kf;
    HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int per_cu = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, RTW_BLOCK, lds));
    if (per_cu < 1) return rtw::fail(RTW_ERR_UNSUPPORTED, "render kernel does not fit on a CU");
    const int64_t want = (int64_t)((A.items + RTW_BLOCK - 1) / RTW_BLOCK);
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)per_cu * g->cus));
    HIP_TRY(hipMemsetAsync(A.queue, 0, RTW_QUEUE_BLOCK * sizeof(unsigned long long), stream));
    // tuning epochs: whole passes over the slots, at least 2x the resident lanes in items (the
    // items in flight blur epoch boundaries; mirrored candidates cancel the blur's bias); explore
    // only if warm-up + all epochs + one more fit (a 1080p x 512 spp frame split over 8 GPUs does)
    A.tune_items = 0;
    if (A.tune && A.total > 0 && !A.tile_perm) {  // epochs are whole passes: chunk-major order only
        const uint64_t lanes = (uint64_t)blocks * RTW_BLOCK;
        const uint64_t E = (uint64_t)A.total * ((2 * lanes + A.total - 1) / A.total);  // >= 2x the resident lanes
        if (A.items_big >= (uint64_t)(RTW_TUNE_EPOCHS + 2) * E) {
            A.tune_items = E;
            HIP_TRY(hipMemsetAsync(A.tune->tb, 0xFF, sizeof(A.tune->tb), stream));
        }
    }
    // a queue's remaining items are shared by the waves drawing from it (1 / RTW_QUEUES of them)
    A.fd_spread = fastdiv_make((uint32_t)std::max<int64_t>(1, RTW_BATCH_SPREAD * blocks * (RTW_BLOCK / 64) / RTW_QUEUES));
    A.fd_epoch = fastdiv_make((uint32_t)std::max<uint64_t>(1, A.tune_items));
    A.fd_half = fastdiv_make((uint32_t)std::max<uint64_t>(1, A.tune_items / 2));
    hipLaunchKernelGGL(kf, dim3((unsigned)blocks), dim3(RTW_BLOCK), lds, stream, A);
    HIP_TRY(hipGetLastError());
    return RTW_OK;
}

// work items of one launch: chunks of `chunk` samples, then the last RTW_TAIL_SAMPLES (default 8)
// samples of the launch's range one at a time
void set_items(KArgs& A, uint32_t chunk);

size_t env_size(const char* name, size_t dflt) {
    const char* e = std::getenv(name);
    if (!e || !e[0]) return dflt;
    const long long v = std::atoll(e);
    return v > 0 ? (size_t)v : dflt;
}

// local items per queue for a launch of `items` items (RTW_QUEUES, RTW_QGRAN)
uint64_t queue_cap(uint64_t items) {
    const uint64_t gran = (items + RTW_QGRAN - 1) / RTW_QGRAN;
    return (gran + RTW_QUEUES - 1) / RTW_QUEUES * RTW_QGRAN;
}

void set_items(KArgs& A, uint32_t chunk) {
    const uint32_t n = A.s_end - A.s_begin;
    // chunk-major order drains on single-sample items; in cost order the cheapest tiles come last
    const uint32_t tail = A.tile_perm || A.whole_pixel ? 0u : std::min<uint32_t>(n, (uint32_t)env_size("RTW_TAIL_SAMPLES", 8));
    A.chunk = chunk;
    A.s_split = A.s_end - tail;
    A.items_big = (uint64_t)A.total * ((A.s_split - A.s_begin + chunk - 1) / chunk);
    A.items = A.items_big + (uint64_t)A.total * tail;
    A.q_cap = queue_cap(A.items);
    A.chunks = (A.s_split - A.s_begin + chunk - 1) / chunk;
    // big batches after the first 10 % of the items: in cost order the costly tiles come first and a
    // wave slowed by long paths must not sit on a big reserve of them (suzanne's 8-GPU shares: 74 ms
    // at a 10 % prefix, 93-103 ms without one); each batch is a device-scope atomic whose round trip
    // stalls the wave (final_scene1 +5.6 % with 1024 over 256, profiles/r03/v2_batch_sweep.txt)
    A.big_from = A.items / 1000 * std::min<size_t>(1000, env_size("RTW_BIG_BATCH_FROM", RTW_BIG_BATCH_FROM));
    const uint32_t per_tile = (uint32_t)(A.tile_w * A.tile_h);
    A.fd_total = fastdiv_make(A.total);
    A.fd_tile = fastdiv_make(per_tile);
    A.fd_rank = fastdiv_make(per_tile * std::max<uint32_t>(1, A.chunks));
    A.fd_tiles_x = fastdiv_make((uint32_t)A.tiles_x);
    A.fd_tile_w = fastdiv_make((uint32_t)A.tile_w);
}

int grow(void** buf, size_t* have, size_t need) {
    if (*have >= need) return RTW_OK;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *have = 0;
    const hipError_t e = hipMalloc(buf, need);
    if (e != hipSuccess) return rtw::fail(RTW_ERR_OUT_OF_MEMORY, std::string("hipMalloc: ") + hipGetErrorString(e));
    *have = need;
    return RTW_OK;
}

// One frame: launches of at most RTW_SAMPLE_BUFFER_BYTES (default: half of the HBM this world could
// use, at most 64 GiB) of per-sample colours,
// each followed by the in-order accumulation; work items of RTW_CHUNK (default 1) samples.
// Launch l of a frame takes its work items from queue block min(l, RTW_QUEUE_SLOTS - 1) of the
// world's counters, so a progress poller can read how many items each launch has handed out.
int render_frame_body(rtw_gpu_world* g, KArgs& A, bool stats, float* out, hipStream_t stream,
                      std::vector<uint64_t>* launch_items);

// One render at a time per world: a frame reuses the world's queue, colour, running-sum and
// cost buffers, so a frame issued on another stream first waits for the previous frame's end.
int render_frame(rtw_gpu_world* g, KArgs& A, bool stats, float* out, hipStream_t stream,
                 std::vector<uint64_t>* launch_items = nullptr) {
    if (!g->done) HIP_TRY(hipEventCreateWithFlags(&g->done, hipEventDisableTiming));
    if (g->done_recorded) HIP_TRY(hipStreamWaitEvent(stream, g->done, 0));
    const int rc = render_frame_body(g, A, stats, out, stream, launch_items);
    HIP_TRY(hipEventRecord(g->done, stream));
    g->done_recorded = true;
    return rc;
}

int render_frame_body(rtw_gpu_world* g, KArgs& A, bool stats, float* out, hipStream_t stream,
                      std::vector<uint64_t>* launch_items) {
    if (A.total == 0) return RTW_OK;
    // Whole-pixel items (KArgs::whole_pixel): thread_count 1 only (the planes' merge needs every
    // plane's value), never in the counting variant; RTW_WHOLE_PIXEL=1 selects them (A/B runs)
    // Whole-pixel items when the frame has many pixels per resident lane (>= RTW_WHOLE_PIXEL_MIN, default
    // 16): the frame's tail (each lane's last pixel) is then short against the frame, and the colour
    // buffer's writes and the accumulation pass go away (C5 on one GPU, 32 pixels per lane: +3.6 %,
    // profiles/r04/v2_experiments_ab.txt).  With few pixels per lane (an 8-GPU share of C5: 4) single-
    // sample items balance the lanes.  RTW_WHOLE_PIXEL=1 / 0 forces them on / off.
    A.whole_pixel = 0;
    if (!stats && A.thread_count <= 1) {
        const uint64_t lanes = (uint64_t)std::max(1, g->cus) * RTW_BLOCK;
        const char* wp = std::getenv("RTW_WHOLE_PIXEL");
        if (wp && wp[0] == '1') A.whole_pixel = 1;
        else if (!(wp && wp[0] == '0') && (uint64_t)A.total >= env_size("RTW_WHOLE_PIXEL_MIN", 16) * lanes) A.whole_pixel = 1;
        // its one launch hosts no threshold tuning (the epochs are passes over the slots): a fixed
        // threshold of 16 (C5: 8 or 16 +0.7 % over 32 and 48, profiles/r04/v9_proof_lds_ab.txt)
        if (A.whole_pixel && !std::getenv("RTW_TRACE_MIN")) A.trace_min = 16;
    }
    const uint32_t chunk = A.whole_pixel ? A.spp : (uint32_t)std::max<size_t>(1, env_size("RTW_CHUNK", 1));
    // The colour buffer sets the launches per frame (C5, 4K x 2048 spp = 204 GB of colours: 13
    // launches at a fixed 16 GiB, 4 at 64 GiB, one per rank of an 8-GPU split).  Default: half of
    // the HBM this world could use (free memory plus the buffer it already holds), at most 64 GiB.
    size_t budget = env_size("RTW_SAMPLE_BUFFER_BYTES", 0);
    if (budget == 0) {
        size_t free_b = 0, total_b = 0;
        budget = (size_t)16 << 30;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
            budget = std::min<size_t>((size_t)64 << 30, std::max<size_t>((size_t)1 << 30, (free_b + g->colors_bytes) / 2));
    }
    const size_t per_sample = (size_t)A.total * 3 * sizeof(float);
    // split_work_tasks (rendering.rs:222-237): planes of spp / T samples, the first spp % T one more
    const uint32_t T = (uint32_t)std::max(1, A.thread_count);
    const uint32_t whole = A.spp / T, rem = A.spp % T;
    const uint32_t n_planes = whole > 0 ? T : rem;
    // the kernel decodes work items in 32 bits: keep a launch's items (plus a wave's overrun of
    // the queue) below 2^32
    const uint64_t item_cap = std::max<uint64_t>(chunk, ((0xFFFFFFFFull >> 1) / A.total) / chunk * chunk);
    auto launch_samples = [&](size_t bytes) {
        uint64_t n = std::max<uint64_t>(chunk, (bytes / per_sample) / chunk * chunk);
        return std::min<uint64_t>(std::min<uint64_t>(n, A.spp), item_cap);
    };
    uint64_t per_launch = launch_samples(budget);
    // More than one launch with planes: the plane partials live between launches, so their bytes
    // come out of the budget first.  One launch merges straight from the colours (no plane buffer).
    const bool plane_buffer = n_planes > 1 && per_launch < A.spp;
    if (plane_buffer) per_launch = launch_samples(budget > per_sample * n_planes ? budget - per_sample * n_planes : 0);
    if (A.whole_pixel) per_launch = A.spp;  // one launch, no colour buffer
    int rc = A.whole_pixel ? RTW_OK : grow((void**)&g->colors, &g->colors_bytes, per_sample * per_launch);
    if (rc != RTW_OK) return rc;
    if (plane_buffer) {
        rc = grow((void**)&g->running, &g->running_bytes, per_sample * n_planes);
        if (rc != RTW_OK) return rc;
    } else if (n_planes <= 1 && per_launch < A.spp) {
        rc = grow((void**)&g->running, &g->running_bytes, per_sample);
        if (rc != RTW_OK) return rc;
    }
    A.colors = g->colors;
    A.chunk = chunk;
    // In-frame tuning of the dynamic-fetch threshold (TuneState): until a world has chosen one,
    // each render launch with room for it explores candidates over pass-aligned epochs.  RTW_TRACE_MIN
    // fixes the threshold instead.
    // A whole-pixel frame keeps its fixed threshold even once an earlier per-sample frame of the world
    // has chosen one: its lanes run whole pixels, not the tuned epochs' single samples.
    A.tune = nullptr;
    // Plain-sphere worlds (the two-children walk) take a fixed threshold of 8 instead of tuning it (round 6):
    // the tuner chose 6-8 on whole final_scene1 frames but 8-24 on its 8-way shares, whose short epochs picked
    // 24 on some ranks (that share +3 %); fixed 8 runs within the noise of the best on both
    // (profiles/r06/ab_trace_min_spheres.txt).  RTW_TUNE_SPHERES=1 keeps the tuner for them.
    const bool sph_fixed = !stats && !A.whole_pixel && g->leaf_kinds == LK_SPHERES && !std::getenv("RTW_TRACE_MIN") &&
                           !std::getenv("RTW_TUNE_SPHERES");
    if (sph_fixed) A.trace_min = 8;
    if (!stats && !A.whole_pixel && !sph_fixed && !std::getenv("RTW_TRACE_MIN")) A.tune = g->tune;
    // Work order.  A frame renders tiles in the order of the deep-path cost its slots showed in
    // earlier frames of the same partition shape, costliest first, each tile's samples together:
    // the frame then ends on cheap tiles instead of waiting for paths trapped inside a mesh that
    // started late (about 100 ms per frame on suzanne).  The image does not depend on the order
    // (a sample's RNG stream is keyed by pixel and sample; accumulation is in sample order).
    // The first frame of a shape runs chunk-major (and hosts the threshold tuning).
    // RTW_NO_REORDER=1 keeps chunk-major order.
    A.slot_cost = nullptr;
    A.tile_perm = nullptr;
    const uint32_t per_tile = (uint32_t)(A.tile_w * A.tile_h);
    const uint32_t n_tiles_local = A.total / per_tile;
    const char* nr = std::getenv("RTW_NO_REORDER");
    if (!stats && !(nr && nr[0] && nr[0] != '0')) {
        const uint64_t key[10] = {A.total, (uint64_t)A.part_index, (uint64_t)A.part_count, (uint64_t)A.tiles_x,
                                  (uint64_t)A.tile_w, (uint64_t)A.tile_h, A.seed_key, A.spp, (uint64_t)(uint32_t)A.max_depth,
                                  (uint64_t)(uint32_t)A.mode};
        if (std::memcmp(key, g->order_key, sizeof(key)) != 0 || !g->slot_cost) {
            if (g->slot_cost) (void)hipFree(g->slot_cost);
            if (g->tile_buf) (void)hipFree(g->tile_buf);
            if (g->sort_tmp) (void)hipFree(g->sort_tmp);
            g->slot_cost = nullptr;
            g->tile_buf = nullptr;
            g->sort_tmp = nullptr;
            g->order_valid = false;
            HIP_TRY(hipMalloc(&g->slot_cost, (size_t)A.total * sizeof(uint32_t)));
            HIP_TRY(hipMalloc(&g->tile_buf, (size_t)n_tiles_local * 4 * sizeof(uint32_t)));
            g->sort_tmp_bytes = 0;
            HIP_TRY(rtw::sort_pairs_desc(nullptr, nullptr, nullptr, nullptr, (int)n_tiles_local, nullptr,
                                         &g->sort_tmp_bytes, stream));
            HIP_TRY(hipMalloc(&g->sort_tmp, std::max<size_t>(g->sort_tmp_bytes, 16)));
            HIP_TRY(hipMemsetAsync(g->slot_cost, 0, (size_t)A.total * sizeof(uint32_t), stream));
            std::memcpy(g->order_key, key, sizeof(key));
            g->order_tiles = n_tiles_local;
        }
        A.slot_cost = g->slot_cost;
        if (g->order_valid) A.tile_perm = g->tile_buf + 3 * (size_t)n_tiles_local;
    }
    HIP_TRY(hipMemsetAsync(g->queue, 0, RTW_QUEUE_BYTES, stream));
    int launch = 0;
    for (uint32_t s0 = 0; s0 < A.spp; s0 += (uint32_t)per_launch, ++launch) {
        const uint32_t s1 = (uint32_t)std::min<uint64_t>(A.spp, s0 + per_launch);
        A.s_begin = s0;
        A.s_end = s1;
        set_items(A, chunk);
        A.queue = g->queue + (size_t)std::min(launch, RTW_QUEUE_SLOTS - 1) * RTW_QUEUE_BLOCK;
        if (launch_items) launch_items->push_back(A.items);
        rc = launch_render(g, A, stats ? LK_STATS : LK_RENDER, stream);
        if (rc != RTW_OK) return rc;
        const unsigned blocks = (A.total + 255) / 256;
        if (A.whole_pixel) {
            // the render kernel wrote the pixels
        } else if (n_planes > 1 && !plane_buffer)
            hipLaunchKernelGGL(merge_planes_direct_kernel, dim3(blocks), dim3(256), 0, stream, (const float*)g->colors,
                               A.total, n_planes, whole, rem, out, A.layout, A.width, A.height, A.tile_w, A.tile_h,
                               A.tiles_x, A.part_index, A.part_count);
        else if (n_planes > 1)
            hipLaunchKernelGGL(accumulate_planes_kernel, dim3(blocks), dim3(256), 0, stream, (const float*)g->colors, s0,
                               s1, A.total, g->running, n_planes, whole, rem, s1 == A.spp ? 1 : 0, out, A.layout,
                               A.width, A.height, A.tile_w, A.tile_h, A.tiles_x, A.part_index, A.part_count);
        else
            hipLaunchKernelGGL(accumulate_kernel, dim3(blocks), dim3(256), 0, stream, (const float*)g->colors, s1 - s0,
                               A.total, g->running, s0 == 0 ? 1 : 0, s1 == A.spp ? 1 : 0, A.spp, out, A.layout,
                               A.width, A.height, A.tile_w, A.tile_h, A.tiles_x, A.part_index, A.part_count);
        HIP_TRY(hipGetLastError());
    }
    if (!stats) {
        g->last_frame[0] = launch;
        g->last_frame[1] = A.whole_pixel ? 1 : 0;
        g->last_frame[2] = A.trace_min;
        g->last_frame[3] = A.tune ? 1 : 0;
    }
    if (A.slot_cost && n_tiles_local > 0) {  // the next frame's tile order
        uint32_t* tb = g->tile_buf;
        const size_t n = n_tiles_local;
        hipLaunchKernelGGL(tile_cost_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, g->slot_cost,
                           (uint32_t)n, per_tile, tb, tb + n);
        HIP_TRY(hipGetLastError());
        size_t bytes = g->sort_tmp_bytes;
        HIP_TRY(rtw::sort_pairs_desc(tb, tb + 2 * n, tb + n, tb + 3 * n, (int)n, g->sort_tmp, &bytes, stream));
        g->order_valid = true;
    }
    return RTW_OK;
}

}  // namespace

extern "C" RTW_API int rtw_partition_floats(const rtw_render_params* p, int64_t* floats) {
    if (!p || !floats) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    const int tw = p->tile_width > 0 ? p->tile_width : 8;
    const int th = p->tile_height > 0 ? p->tile_height : 8;
    const int pc = p->part_count > 0 ? p->part_count : 1;
    if (p->width < 1 || p->height < 1 || p->part_index < 0 || p->part_index >= pc)
        return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "bad params");
    const int64_t n_tiles = (int64_t)((p->width + tw - 1) / tw) * ((p->height + th - 1) / th);
    const int64_t owned = n_tiles > p->part_index ? (n_tiles - p->part_index + pc - 1) / pc : 0;
    *floats = owned * tw * th * 3;
    return RTW_OK;
}

extern "C" RTW_API int rtw_render_device(rtw_gpu_world* g, const rtw_render_params* p, float* d_out, void* stream) {
    KArgs A;
    const int v = make_args(g, p, A);
    if (v != RTW_OK) return v;
    if (!d_out) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null output");
    A.out = d_out;
    HIP_TRY(hipSetDevice(g->device));
    return render_frame(g, A, false, d_out, (hipStream_t)stream);
}

namespace {
int collect_stats(rtw_gpu_world* g, const rtw_render_params* p, rtw_render_stats* s, uint64_t* dbg, int dbg_n,
                  int tree = 0) {
    KArgs A;
    const int v = make_args(g, p, A);
    if (v != RTW_OK) return v;
    A.stats_tree = tree;
    if (!s) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null stats");
    HIP_TRY(hipSetDevice(g->device));
    float* out = nullptr;
    unsigned long long* st = nullptr;
    HIP_TRY(hipMalloc(&out, (size_t)p->width * p->height * 3 * sizeof(float)));
    HIP_TRY(hipMalloc(&st, (ST_COUNT + DB_COUNT) * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(st, 0, (ST_COUNT + DB_COUNT) * sizeof(unsigned long long)));
    A.out = out;
    A.layout = RTW_LAYOUT_IMAGE;
    A.stats = st;
    {
        const int rc = render_frame(g, A, true, out, 0);
        if (rc != RTW_OK) return rc;
    }
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long h[ST_COUNT + DB_COUNT];
    HIP_TRY(hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost));
    (void)hipFree(out);
    (void)hipFree(st);
    if (dbg)
        for (int i = 0; i < dbg_n && i < DB_COUNT; ++i) dbg[i] = h[ST_COUNT + i];
    s->samples = h[ST_SAMPLES];
    s->rays = h[ST_RAYS];
    s->node_visits = h[ST_NODES];
    s->sphere_tests = h[ST_T_SPHERE];
    s->rect_tests = h[ST_T_RECT];
    s->box_tests = h[ST_T_BOX];
    s->triangle_tests = h[ST_T_TRI];
    s->sphere_hits = h[ST_H_SPHERE];
    s->rect_hits = h[ST_H_RECT];
    s->box_hits = h[ST_H_BOX];
    s->triangle_hits = h[ST_H_TRI];
    s->material_reads = h[ST_MAT];
    s->texel_reads = h[ST_TEXEL];
    return RTW_OK;
}
}  // namespace

extern "C" RTW_API int rtw_render_collect_stats(rtw_gpu_world* g, const rtw_render_params* p, rtw_render_stats* s) {
    return collect_stats(g, p, s, nullptr, 0);
}

extern "C" RTW_API int rtw_render_collect_stats_tree(rtw_gpu_world* g, const rtw_render_params* p, int tree,
                                                     rtw_render_stats* s) {
    if (tree != 0 && tree != 1) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "tree must be 0 or 1");
    return collect_stats(g, p, s, nullptr, 0, tree);
}

extern "C" RTW_API int rtw_render_debug_counters(rtw_gpu_world* g, const rtw_render_params* p, rtw_render_stats* s,
                                                 uint64_t* counters, int n) {
    if (!counters || n < 0) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null counters");
    return collect_stats(g, p, s, counters, n);
}

extern "C" RTW_API int rtw_render(const rtw_world* w, const rtw_render_params* p, int device, float* out_rgb) {
    if (!p || !out_rgb) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    rtw_gpu_world* g = nullptr;
    int rc = rtw_world_upload(w, device, &g);
    if (rc != RTW_OK) return rc;
    rtw_render_params q = *p;
    q.layout = RTW_LAYOUT_IMAGE;
    const size_t bytes = (size_t)q.width * (size_t)q.height * 3 * sizeof(float);
    float* d = nullptr;
    hipError_t e = hipMalloc(&d, bytes);
    if (e != hipSuccess) {
        rtw_world_release(g);
        return rtw::fail(RTW_ERR_OUT_OF_MEMORY, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    // pixels outside the owned partition keep the caller's values
    e = hipMemcpy(d, out_rgb, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        rc = rtw_render_device(g, &q, d, nullptr);
        if (rc == RTW_OK) {
            e = hipDeviceSynchronize();
            if (e == hipSuccess) e = hipMemcpy(out_rgb, d, bytes, hipMemcpyDeviceToHost);
        }
    }
    (void)hipFree(d);
    rtw_world_release(g);
    if (rc != RTW_OK) return rc;
    if (e != hipSuccess) return rtw::fail(RTW_ERR_HIP, std::string("render: ") + hipGetErrorString(e));
    return RTW_OK;
}

// rtw_render with progress reports (the reference's progress thread, rendering.rs:140-157): the
// frame runs on its own stream while this thread polls the launches' work-item counters (a copy
// on a second stream) every ~50 ms and calls cb(done_samples, total_samples, user), done being
// the share of work items handed out; the last call reports done == total.
extern "C" RTW_API int rtw_render_progress(const rtw_world* w, const rtw_render_params* p, int device,
                                           float* out_rgb, rtw_progress_fn cb, void* user) {
    if (!p || !out_rgb) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    if (!cb) return rtw_render(w, p, device, out_rgb);
    rtw_gpu_world* g = nullptr;
    int rc = rtw_world_upload(w, device, &g);
    if (rc != RTW_OK) return rc;
    rtw_render_params q = *p;
    q.layout = RTW_LAYOUT_IMAGE;
    const size_t bytes = (size_t)q.width * (size_t)q.height * 3 * sizeof(float);
    float* d = nullptr;
    unsigned long long* h = nullptr;
    hipStream_t rs = nullptr, ps = nullptr;
    hipEvent_t fin = nullptr;
    hipError_t e = hipMalloc(&d, bytes);
    if (e == hipSuccess) e = hipHostMalloc((void**)&h, RTW_QUEUE_BYTES);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&rs, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ps, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&fin, hipEventDisableTiming);
    if (e == hipSuccess) e = hipMemcpy(d, out_rgb, bytes, hipMemcpyHostToDevice);
    const uint64_t total = (uint64_t)q.width * (uint64_t)q.height * q.samples_per_pixel;
    if (e == hipSuccess) {
        KArgs A;
        rc = make_args(g, &q, A);
        if (rc == RTW_OK) {
            A.out = d;
            std::vector<uint64_t> items;
            rc = render_frame(g, A, false, d, rs, &items);
            uint64_t all = 0;
            for (uint64_t n : items) all += n;
            if (rc == RTW_OK) e = hipEventRecord(fin, rs);
            uint64_t last = ~0ull;
            while (rc == RTW_OK && e == hipSuccess) {
                const hipError_t qe = hipEventQuery(fin);
                if (qe == hipSuccess) break;
                if (qe != hipErrorNotReady) {
                    e = qe;
                    break;
                }
                e = hipMemcpyAsync(h, g->queue, RTW_QUEUE_BYTES, hipMemcpyDeviceToHost, ps);
                if (e == hipSuccess) e = hipStreamSynchronize(ps);
                uint64_t taken = 0;  // local items handed out, over the launch's queues (padding included)
                for (size_t l = 0; l < items.size() && l < RTW_QUEUE_SLOTS; ++l) {
                    const uint64_t cap = queue_cap(items[l]);
                    uint64_t t = 0;
                    for (int q = 0; q < RTW_QUEUES; ++q)
                        t += std::min<uint64_t>(h[l * RTW_QUEUE_BLOCK + q * RTW_QSTRIDE], cap);
                    taken += std::min<uint64_t>(t, items[l]);
                }
                const uint64_t done = all ? (uint64_t)((double)total * (double)taken / (double)all) : 0;
                if (e == hipSuccess && done != last && done < total) {
                    cb(done, total, user);
                    last = done;
                }
                struct timespec ts = {0, 50 * 1000 * 1000};
                nanosleep(&ts, nullptr);
            }
            if (rc == RTW_OK && e == hipSuccess) e = hipStreamSynchronize(rs);
            if (rc == RTW_OK && e == hipSuccess) {
                cb(total, total, user);
                e = hipMemcpy(out_rgb, d, bytes, hipMemcpyDeviceToHost);
            }
        }
    }
    if (fin) (void)hipEventDestroy(fin);
    if (ps) (void)hipStreamDestroy(ps);
    if (rs) (void)hipStreamDestroy(rs);
    if (h) (void)hipHostFree(h);
    if (d) (void)hipFree(d);
    rtw_world_release(g);
    if (rc != RTW_OK) return rc;
    if (e != hipSuccess) return rtw::fail(RTW_ERR_HIP, std::string("render: ") + hipGetErrorString(e));
    return RTW_OK;
}

extern "C" RTW_API int rtw_untile_device(const rtw_render_params* p, const float* d_tiles, int64_t stride,
                                         float* d_image, void* stream) {
    if (!p || !d_tiles || !d_image) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "null argument");
    const int tw = p->tile_width > 0 ? p->tile_width : 8;
    const int th = p->tile_height > 0 ? p->tile_height : 8;
    const int pc = p->part_count > 0 ? p->part_count : 1;
    const int tiles_x = (p->width + tw - 1) / tw;
    const int n_tiles = tiles_x * ((p->height + th - 1) / th);
    const int64_t total = (int64_t)n_tiles * tw * th;
    if (total == 0) return RTW_OK;
    hipLaunchKernelGGL(untile_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_tiles,
                       stride, d_image, p->width, p->height, tw, th, tiles_x, n_tiles, pc);
    HIP_TRY(hipGetLastError());
    return RTW_OK;
}

extern "C" RTW_API int rtw_encode_rgb8_device(const float* d_image, int64_t pixels, uint8_t* d_rgb8, void* stream) {
    if (!d_image || !d_rgb8 || pixels < 0) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "bad argument");
    if (pixels == 0) return RTW_OK;
    const int64_t n = pixels * 3;
    hipLaunchKernelGGL(encode_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_image,
                       pixels, d_rgb8);
    HIP_TRY(hipGetLastError());
    return RTW_OK;
}

namespace {
// device buffers of the self-check entry points below, freed on every return path
struct DevBufs {
    std::vector<void*> p;
    ~DevBufs() {
        for (void* q : p) (void)hipFree(q);
    }
    template <class T>
    hipError_t alloc(T** x, size_t bytes) {
        const hipError_t e = hipMalloc((void**)x, bytes);
        if (e == hipSuccess) p.push_back((void*)*x);
        return e;
    }
};
}  // namespace

extern "C" RTW_API int rtw_device_eval_node_pass(int device, const float* box, const float* ray, const float* range,
                                                 const float* km, int32_t mk_world, int64_t n, int32_t* out) {
    if (!box || !ray || !range || !km || !out || n < 0) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "bad argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return rtw::fail(RTW_ERR_NO_DEVICE, "no HIP device");
    HIP_TRY(hipSetDevice(device));
    if (n == 0) return RTW_OK;
    float *db = nullptr, *dr = nullptr, *dg = nullptr, *dk = nullptr;
    int32_t* dout = nullptr;
    DevBufs bufs;
    HIP_TRY(bufs.alloc(&db, (size_t)n * 6 * sizeof(float)));
    HIP_TRY(bufs.alloc(&dr, (size_t)n * 6 * sizeof(float)));
    HIP_TRY(bufs.alloc(&dg, (size_t)n * 2 * sizeof(float)));
    HIP_TRY(bufs.alloc(&dk, (size_t)n * 2 * sizeof(float)));
    HIP_TRY(bufs.alloc(&dout, (size_t)n * sizeof(int32_t)));
    HIP_TRY(hipMemcpy(db, box, (size_t)n * 6 * sizeof(float), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dr, ray, (size_t)n * 6 * sizeof(float), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dg, range, (size_t)n * 2 * sizeof(float), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dk, km, (size_t)n * 2 * sizeof(float), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(eval_node_pass_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, db, dr, dg, dk, mk_world,
                       n, dout);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(out, dout, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost));
    return RTW_OK;
}

extern "C" RTW_API int rtw_device_check_division(int device, int test, uint64_t base, uint64_t n, uint64_t seed,
                                                 uint64_t* mismatches, uint64_t* first) {
    if (!mismatches || !first || test < 0 || test > 6) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "bad argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return rtw::fail(RTW_ERR_NO_DEVICE, "no HIP device");
    HIP_TRY(hipSetDevice(device));
    unsigned long long* d = nullptr;
    DevBufs bufs;
    HIP_TRY(bufs.alloc(&d, 2 * sizeof(unsigned long long)));
    const unsigned long long init[2] = {0ull, ~0ull};
    HIP_TRY(hipMemcpy(d, init, sizeof(init), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(check_division_kernel, dim3(8192), dim3(256), 0, 0, test, base, n, seed, d);
    HIP_TRY(hipGetLastError());
    unsigned long long res[2];
    HIP_TRY(hipMemcpy(res, d, sizeof(res), hipMemcpyDeviceToHost));
    *mismatches = res[0];
    *first = res[1];
    return RTW_OK;
}

extern "C" RTW_API int rtw_device_eval_checker(int device, const float* xyz, int64_t n, int32_t* out) {
    if (!xyz || !out || n < 0) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "bad argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return rtw::fail(RTW_ERR_NO_DEVICE, "no HIP device");
    HIP_TRY(hipSetDevice(device));
    if (n == 0) return RTW_OK;
    float* dx = nullptr;
    int32_t* dout = nullptr;
    DevBufs bufs;
    HIP_TRY(bufs.alloc(&dx, (size_t)n * 3 * sizeof(float)));
    HIP_TRY(bufs.alloc(&dout, (size_t)n * sizeof(int32_t)));
    HIP_TRY(hipMemcpy(dx, xyz, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(eval_checker_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dx, n, dout);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(out, dout, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost));
    return RTW_OK;
}

extern "C" RTW_API int rtw_device_eval_scalar(int device, int fn, const float* a, const float* b, int64_t n, float* out) {
    if (!a || !out || n < 0 || fn < 0 || fn > 6) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "bad argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return rtw::fail(RTW_ERR_NO_DEVICE, "no HIP device");
    HIP_TRY(hipSetDevice(device));
    if (n == 0) return RTW_OK;
    float *da = nullptr, *db = nullptr, *dout = nullptr;
    const size_t bytes = (size_t)n * sizeof(float);
    DevBufs bufs;
    HIP_TRY(bufs.alloc(&da, bytes));
    HIP_TRY(bufs.alloc(&db, bytes));
    HIP_TRY(bufs.alloc(&dout, bytes));
    HIP_TRY(hipMemcpy(da, a, bytes, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(db, b ? b : a, bytes, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(eval_scalar_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, fn, da, db, n, dout);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost));
    return RTW_OK;
}
