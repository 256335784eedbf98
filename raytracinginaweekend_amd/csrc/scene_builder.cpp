// scene_builder.cpp -- host-side World construction, restating the reference's host layer:
//   camera builder            src/lib/camera.rs:11-173
//   Transformation            src/lib/transformations.rs
//   WorldBuilder / NodeBuilder / NodeRef::finish   src/app/worlds/world_builder.rs
//   Geometry::partial_apply_transformation / bounding boxes   src/lib/hittable.rs:150-292
//   BoundingVolumeHierarchy::new/_new   src/lib/hittable.rs:360-427
//   Perlin::new               src/lib/perlin.rs:19-36, 93-97
//   OBJ loader                src/app/obj_loader.rs (fan-triangulation quirk kept)
//   demo worlds               src/app/worlds/demo_worlds.rs (seeded as main.rs:24)
// The output is the flat rtw_world the device kernel consumes (include/rtw.h).  Host f32
// arithmetic follows the reference expression by expression (built with -ffp-contract=off);
// sin/cos/tan come from the platform libm like Rust's f32 methods on Linux.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rtw_scalar.h"
#include "rtw_common.h"

namespace {

// ---------------------------------------------------------------------------------------------
// f32 vector algebra (vec3.rs)
// ---------------------------------------------------------------------------------------------
struct V3 {
    float e[3];
};
inline V3 v3(float x, float y, float z) { return V3{{x, y, z}}; }
inline V3 operator+(V3 a, V3 b) { return v3(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }
inline V3 operator-(V3 a, V3 b) { return v3(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }
inline V3 operator*(V3 a, float s) { return v3(a.e[0] * s, a.e[1] * s, a.e[2] * s); }
inline V3 operator/(V3 a, float s) { return v3(a.e[0] / s, a.e[1] / s, a.e[2] / s); }
inline float dot(V3 a, V3 b) { return a.e[0] * b.e[0] + a.e[1] * b.e[1] + a.e[2] * b.e[2]; }
inline V3 cross(V3 a, V3 b) {
    return v3(a.e[1] * b.e[2] - a.e[2] * b.e[1], a.e[2] * b.e[0] - a.e[0] * b.e[2],
              a.e[0] * b.e[1] - a.e[1] * b.e[0]);
}
inline float length(V3 a) { return std::sqrt(dot(a, a)); }
inline V3 with_length(V3 a, float l) { return a * (l / length(a)); }
inline V3 unit(V3 a) { return with_length(a, 1.0f); }
inline bool eq(V3 a, V3 b) { return a.e[0] == b.e[0] && a.e[1] == b.e[1] && a.e[2] == b.e[2]; }
inline V3 load3(const float* p) { return v3(p[0], p[1], p[2]); }
inline void store3(float* p, V3 v) { p[0] = v.e[0]; p[1] = v.e[1]; p[2] = v.e[2]; }

const V3 ZERO = v3(0.0f, 0.0f, 0.0f);
const V3 UP = v3(0.0f, 1.0f, 0.0f);
const V3 DOWN = v3(0.0f, -1.0f, 0.0f);
const V3 RIGHT = v3(1.0f, 0.0f, 0.0f);
const V3 LEFT = v3(-1.0f, 0.0f, 0.0f);
const V3 FORWARD = v3(0.0f, 0.0f, -1.0f);
const V3 BACKWARD = v3(0.0f, 0.0f, 1.0f);

// f32::to_radians: self * (PI / 180.0f32)
inline float to_radians(float deg) {
    const float pi = 3.14159274101257324219f;
    const float k = pi / 180.0f;
    return deg * k;
}

// ---------------------------------------------------------------------------------------------
// Aabb helpers (aabb.rs:15-63, 169-192)
// ---------------------------------------------------------------------------------------------
struct Aabb {
    V3 min, max;
};
inline V3 min_array(V3 a, V3 b) {
    return v3(rtw_minr(a.e[0], b.e[0]), rtw_minr(a.e[1], b.e[1]), rtw_minr(a.e[2], b.e[2]));
}
inline V3 max_array(V3 a, V3 b) {
    return v3(rtw_maxr(a.e[0], b.e[0]), rtw_maxr(a.e[1], b.e[1]), rtw_maxr(a.e[2], b.e[2]));
}
Aabb surrounding_points(const V3* pts, int n) {
    V3 mn = pts[0], mx = pts[0];
    for (int i = 1; i < n; ++i) {
        mn = min_array(mn, pts[i]);
        mx = max_array(mx, pts[i]);
    }
    return Aabb{mn, mx};
}
Aabb surrounding_boxes(Aabb a, Aabb b) { return Aabb{min_array(a.min, b.min), max_array(a.max, b.max)}; }

// ---------------------------------------------------------------------------------------------
// Transformation (transformations.rs)
// ---------------------------------------------------------------------------------------------
struct Xf {
    V3 offset = ZERO;
    float ys = 0.0f;
    float yc = 1.0f;
};
inline V3 rotate_around_up(float c, float s, V3 v) {  // :107-111
    const float x = v.e[0], y = v.e[2];
    V3 r = v;
    r.e[0] = c * x + s * y;
    r.e[2] = -s * x + c * y;
    return r;
}
inline bool xf_is_zero(const Xf& x) { return eq(x.offset, ZERO) && x.ys == 0.0f && x.yc == 1.0f; }
inline Xf xf_translate(Xf x, V3 off) {  // :19-23
    x.offset = x.offset + off;
    return x;
}
inline Xf xf_rotate_around_up(const Xf& self, float angle) {  // :27-36
    Xf result = self;
    const float rad = to_radians(angle);
    const float s = std::sin(rad), c = std::cos(rad);
    result.offset = rotate_around_up(c, s, result.offset);
    V3 r = v3(self.ys, 0.0f, self.yc);
    r = rotate_around_up(c, s, r);
    result.ys = r.e[0];
    result.yc = r.e[2];
    return result;
}
inline V3 xf_apply_point(const Xf& x, V3 p) { return rotate_around_up(x.yc, x.ys, p) + x.offset; }
inline V3 xf_apply_normal(const Xf& x, V3 d) { return rotate_around_up(x.yc, x.ys, d); }
inline V3 xf_apply_direction(const Xf& x, V3 d) { return rotate_around_up(x.yc, x.ys, d); }
inline Xf xf_then(const Xf& self, const Xf& next) {  // :89-98
    Xf r;
    r.offset = xf_apply_direction(next, self.offset) + next.offset;
    r.ys = self.ys * next.yc + self.yc * next.ys;
    r.yc = self.yc * next.yc - self.ys * next.ys;
    return r;
}
// hittable.rs:285-291 apply_aabb -- the corner loop mutates copies, so only the corner
// recomputation (min + (max - min) may round) survives.
Aabb xf_apply_aabb(const Xf&, Aabb b) {
    const V3 right = v3(b.max.e[0] - b.min.e[0], 0.0f, 0.0f);
    const V3 up = v3(0.0f, b.max.e[1] - b.min.e[1], 0.0f);
    const V3 fwd = v3(0.0f, 0.0f, b.max.e[2] - b.min.e[2]);
    const V3 corners[8] = {b.min, b.min + right, b.min + up, b.min + fwd,
                           b.max, b.max - right, b.max - up, b.max - fwd};
    return surrounding_points(corners, 8);
}

// ---------------------------------------------------------------------------------------------
// Geometry (hittable.rs:104-209)
// ---------------------------------------------------------------------------------------------
struct Geom {
    int kind = RTW_GEOM_SPHERE;
    rtw_sphere sphere{};
    rtw_rect rect{};
    rtw_box box{};
    rtw_triangle tri{};
};

void rect_axes(int plane, int* p0, int* p1, int* n) {
    if (plane == RTW_PLANE_XY) { *p0 = 0; *p1 = 1; *n = 2; }
    else if (plane == RTW_PLANE_XZ) { *p0 = 0; *p1 = 2; *n = 1; }
    else { *p0 = 1; *p1 = 2; *n = 0; }
}

Aabb geom_bounding_box(const Geom& g) {
    switch (g.kind) {
        case RTW_GEOM_SPHERE: {  // aabb.rs:19-24 new_radius
            const V3 c = load3(g.sphere.center);
            const float r = g.sphere.radius;
            return Aabb{c - v3(r, r, r), c + v3(r, r, r)};
        }
        case RTW_GEOM_RECT: {  // rect_geometry.rs:87-98 with thickness 0.01
            int p0, p1, n;
            rect_axes(g.rect.plane, &p0, &p1, &n);
            V3 mn = ZERO, mx = ZERO;
            mn.e[p0] = g.rect.r0[0];
            mn.e[p1] = g.rect.r1[0];
            mn.e[n] = g.rect.dist - 0.01f;
            mx.e[p0] = g.rect.r0[1];
            mx.e[p1] = g.rect.r1[1];
            mx.e[n] = g.rect.dist + 0.01f;
            return Aabb{mn, mx};
        }
        case RTW_GEOM_BOX: return Aabb{load3(g.box.min), load3(g.box.max)};
        default: {  // triangle_geometry.rs:47-49
            const V3 p[3] = {load3(g.tri.positions[0]), load3(g.tri.positions[1]), load3(g.tri.positions[2])};
            return surrounding_points(p, 3);
        }
    }
}

// hittable.rs:165-208; returns true if a residual transformation remains.
bool partial_apply_transformation(const Geom& g, const Xf& t, Geom* out, Xf* rem) {
    *out = g;
    switch (g.kind) {
        case RTW_GEOM_SPHERE:
            store3(out->sphere.center, xf_apply_point(t, load3(g.sphere.center)));
            out->sphere.radius = g.sphere.radius;  // apply_distance is the identity
            return false;
        case RTW_GEOM_TRIANGLE:
            for (int i = 0; i < 3; ++i) {
                store3(out->tri.positions[i], xf_apply_point(t, load3(g.tri.positions[i])));
                store3(out->tri.normals[i], xf_apply_normal(t, load3(g.tri.normals[i])));
            }
            return false;
        case RTW_GEOM_BOX: {
            const V3 translation = t.offset;  // split_translation_remainder (transformations.rs:66-70)
            Xf remainder = t;
            remainder.offset = ZERO;
            store3(out->box.min, load3(g.box.min) + translation);
            store3(out->box.max, load3(g.box.max) + translation);
            if (xf_is_zero(remainder)) return false;
            *rem = remainder;
            return true;
        }
        default:  // Rect keeps the whole transformation
            if (xf_is_zero(t)) return false;
            *rem = t;
            return true;
    }
}

// ---------------------------------------------------------------------------------------------
// Scene graph (world_builder.rs:228-328)
// ---------------------------------------------------------------------------------------------
struct GeoEntry {
    Geom geo;
    int32_t material;
    bool is_poi;
    float density;
};
struct Node {
    std::vector<GeoEntry> geo;
    Xf transformation;
    V3 moving_animation = ZERO;
    std::vector<int32_t> children;
};

struct Element {  // one flattened leaf (a chain of SceneElements)
    Geom geo;
    int32_t material;
    bool volume;
    float neg_inv_density;
    bool has_xf;
    Xf xf;
    bool animated;
    V3 velocity;
};

}  // namespace

// ---------------------------------------------------------------------------------------------
// opaque handles
// ---------------------------------------------------------------------------------------------
struct rtw_builder {
    std::vector<rtw_texture> textures;
    std::vector<rtw_material> materials;
    std::vector<std::vector<uint8_t>> images;
    std::vector<std::pair<int32_t, int32_t>> image_dims;
    std::vector<rtw_perlin> perlins;
    std::vector<Node> nodes;
};

struct rtw_world_handle {
    rtw_world w{};
    std::vector<rtw_bvh_node> nodes;
    std::vector<rtw_leaf> leaves;
    std::vector<rtw_sphere> spheres;
    std::vector<rtw_rect> rects;
    std::vector<rtw_box> boxes;
    std::vector<rtw_triangle> triangles;
    std::vector<rtw_material> materials;
    std::vector<rtw_texture> textures;
    std::vector<std::vector<uint8_t>> image_data;
    std::vector<rtw_image> images;
    std::vector<rtw_perlin> perlins;
};

namespace {

bool valid_node(const rtw_builder* b, int32_t n) { return b && n >= 0 && n < (int32_t)b->nodes.size(); }
bool valid_tex(const rtw_builder* b, int32_t t) { return b && t >= 0 && t < (int32_t)b->textures.size(); }
bool valid_mat(const rtw_builder* b, int32_t m) { return b && m >= 0 && m < (int32_t)b->materials.size(); }

int32_t add_node(rtw_builder* b, Node n) {
    b->nodes.push_back(std::move(n));
    return (int32_t)b->nodes.size() - 1;
}

int32_t node_with_geo(rtw_builder* b, const Geom& g, int32_t material) {
    Node n;
    n.geo.push_back(GeoEntry{g, material, false, 1.0f});
    return add_node(b, std::move(n));
}

// finish_internal (world_builder.rs:291-328).  Reports the first POI rect (light sampler).
bool finish_internal(const rtw_builder* b, int32_t node, const Xf& parent, std::vector<Element>& out,
                     bool* have_wsd, rtw_rect* wsd, int depth) {
    if (depth > 4096) return false;  // a cycle in the node graph
    const Node& nd = b->nodes[node];
    const Xf full = xf_then(parent, nd.transformation);
    bool found = false;
    rtw_rect found_rect{};
    for (const GeoEntry& ge : nd.geo) {
        Element e{};
        Xf rem;
        e.has_xf = partial_apply_transformation(ge.geo, full, &e.geo, &rem);
        if (e.has_xf) e.xf = rem;
        e.material = ge.material;
        e.volume = ge.density < 1.0f;
        e.neg_inv_density = e.volume ? (-1.0f / ge.density) : 0.0f;  // hittable.rs:305
        e.animated = !eq(nd.moving_animation, ZERO);
        e.velocity = nd.moving_animation;
        out.push_back(e);
        if (ge.is_poi && !e.has_xf && !found && e.geo.kind == RTW_GEOM_RECT) {
            found = true;
            found_rect = e.geo.rect;
        }
    }
    for (int32_t child : nd.children) {
        bool cf = false;
        rtw_rect cr{};
        if (!finish_internal(b, child, full, out, &cf, &cr, depth + 1)) return false;
        if (!found && cf) {
            found = true;
            found_rect = cr;
        }
    }
    *have_wsd = found;
    *wsd = found_rect;
    return true;
}

// SceneElement::bounding_box (hittable.rs:249-267) for one flattened leaf
Aabb element_bounding_box(const Element& e, float t0, float t1) {
    Aabb bb = geom_bounding_box(e.geo);  // Surface / Volume (boundary)
    if (e.has_xf) bb = xf_apply_aabb(e.xf, bb);
    if (e.animated) {
        const Xf start = xf_translate(Xf{}, e.velocity * t0);
        const Xf end = xf_translate(Xf{}, e.velocity * t1);
        const Aabb sb = xf_apply_aabb(start, bb);
        const Aabb eb = xf_apply_aabb(end, bb);
        bb = surrounding_boxes(sb, eb);
    }
    return bb;
}

struct BvhItem {
    int32_t id;  // leaf encoded as -1 - index
    Aabb aabb;
};

// BoundingVolumeHierarchy::_new (hittable.rs:382-427)
int32_t bvh_new(BvhItem* items, size_t n, std::vector<rtw_bvh_node>& nodes, int axis, Aabb* out_box,
                int depth, int* max_depth) {
    if (depth > *max_depth) *max_depth = depth;
    if (n == 1) {
        *out_box = items[0].aabb;
        return items[0].id;
    }
    std::stable_sort(items, items + n, [axis](const BvhItem& a, const BvhItem& b) {
        return a.aabb.min.e[axis] < b.aabb.min.e[axis];
    });
    if (n == 2) {
        const int32_t id = (int32_t)nodes.size();
        const Aabb bb = surrounding_boxes(items[0].aabb, items[1].aabb);
        rtw_bvh_node nd{};
        store3(nd.min, bb.min);
        store3(nd.max, bb.max);
        nd.axis = axis;
        nd.left = items[0].id;
        nd.right = items[1].id;
        nodes.push_back(nd);
        *out_box = bb;
        return id;
    }
    const size_t mid = n / 2;
    const int32_t id = (int32_t)nodes.size();
    nodes.push_back(rtw_bvh_node{});
    Aabb lb, rb;
    const int32_t l = bvh_new(items, mid, nodes, (int)((axis + mid) % 3), &lb, depth + 1, max_depth);
    const int32_t r = bvh_new(items + mid, n - mid, nodes, (int)((axis + (n - mid)) % 3), &rb, depth + 1, max_depth);
    const Aabb bb = surrounding_boxes(lb, rb);
    rtw_bvh_node& nd = nodes[(size_t)id];
    store3(nd.min, bb.min);
    store3(nd.max, bb.max);
    nd.axis = axis;
    nd.left = l;
    nd.right = r;
    *out_box = bb;
    return id;
}

}  // namespace

// =============================================================================================
// C ABI: rng
// =============================================================================================
extern "C" RTW_API rtw_rng* rtw_rng_from_seed(const uint8_t seed[16]) {
    if (!seed) {
        rtw::set_error("rtw_rng_from_seed: null seed");
        return nullptr;
    }
    auto* r = new rtw_rng;
    r->s = rtw_xoro_from_seed_bytes(seed);
    return r;
}
extern "C" RTW_API void rtw_rng_free(rtw_rng* rng) { delete rng; }
extern "C" RTW_API float rtw_rng_gen_f32(rtw_rng* rng) { return rng ? rtw_gen_f32(&rng->s) : 0.0f; }
extern "C" RTW_API uint64_t rtw_rng_next_u64(rtw_rng* rng) { return rng ? rtw_xoro_next_u64(&rng->s) : 0; }

// =============================================================================================
// C ABI: builder
// =============================================================================================
extern "C" RTW_API rtw_builder* rtw_builder_new(void) { return new rtw_builder; }
extern "C" RTW_API void rtw_builder_free(rtw_builder* b) { delete b; }

extern "C" RTW_API int32_t rtw_texture_solid(rtw_builder* b, float r, float g, float bl) {
    if (!b) return rtw::fail(-1, "rtw_texture_solid: null builder"), -1;
    rtw_texture t{};
    t.kind = RTW_TEX_SOLID;
    t.color[0] = r;
    t.color[1] = g;
    t.color[2] = bl;
    t.even = t.odd = t.perlin = t.image = -1;
    b->textures.push_back(t);
    return (int32_t)b->textures.size() - 1;
}
extern "C" RTW_API int32_t rtw_texture_checker(rtw_builder* b, float inv_frequency, int32_t even, int32_t odd) {
    if (!valid_tex(b, even) || !valid_tex(b, odd)) return rtw::fail(-1, "rtw_texture_checker: bad texture id"), -1;
    rtw_texture t{};
    t.kind = RTW_TEX_CHECKER;
    t.inv_frequency = inv_frequency;
    t.even = even;
    t.odd = odd;
    t.perlin = t.image = -1;
    b->textures.push_back(t);
    return (int32_t)b->textures.size() - 1;
}
// world_builder.rs:35-40 texture_marble -> Perlin::new(8, rng) (perlin.rs:19-36)
extern "C" RTW_API int32_t rtw_texture_marble(rtw_builder* b, float scale, rtw_rng* rng) {
    if (!b || !rng) return rtw::fail(-1, "rtw_texture_marble: null argument"), -1;
    rtw_perlin p{};
    p.bits = 8;
    const uint32_t n = 1u << p.bits;
    for (uint32_t i = 0; i < n; ++i) rtw_unit_sphere(&rng->s, p.ranvec[i]);
    uint32_t* perms[3] = {p.perm_x, p.perm_y, p.perm_z};
    for (int k = 0; k < 3; ++k) {  // generate_per: identity then SliceRandom::shuffle
        uint32_t* a = perms[k];
        for (uint32_t i = 0; i < n; ++i) a[i] = i;
        for (uint32_t i = n - 1; i >= 1; --i) {
            const uint32_t j = rtw_gen_range_u32(i + 1, &rng->s);
            std::swap(a[i], a[j]);
        }
    }
    b->perlins.push_back(p);
    rtw_texture t{};
    t.kind = RTW_TEX_MARBLE;
    t.scale = scale;
    t.perlin = (int32_t)b->perlins.size() - 1;
    t.even = t.odd = t.image = -1;
    b->textures.push_back(t);
    return (int32_t)b->textures.size() - 1;
}
extern "C" RTW_API int32_t rtw_texture_image_rgb8(rtw_builder* b, const uint8_t* rgb, int32_t width, int32_t height) {
    if (!b || !rgb || width < 1 || height < 1) return rtw::fail(-1, "rtw_texture_image_rgb8: bad image"), -1;
    b->images.emplace_back(rgb, rgb + (size_t)width * (size_t)height * 3u);
    b->image_dims.emplace_back(width, height);
    rtw_texture t{};
    t.kind = RTW_TEX_IMAGE;
    t.image = (int32_t)b->images.size() - 1;
    t.even = t.odd = t.perlin = -1;
    b->textures.push_back(t);
    return (int32_t)b->textures.size() - 1;
}

static int32_t add_material(rtw_builder* b, int kind, int32_t tex, float fuzz, float ior) {
    rtw_material m{};
    m.kind = kind;
    m.texture = tex;
    m.fuzz = fuzz;
    m.index_of_refraction = ior;
    b->materials.push_back(m);
    return (int32_t)b->materials.size() - 1;
}
extern "C" RTW_API int32_t rtw_material_lambert(rtw_builder* b, int32_t albedo) {
    if (!valid_tex(b, albedo)) return rtw::fail(-1, "rtw_material_lambert: bad texture id"), -1;
    return add_material(b, RTW_MAT_LAMBERT, albedo, 0.0f, 0.0f);
}
extern "C" RTW_API int32_t rtw_material_metal(rtw_builder* b, int32_t albedo, float fuzz) {
    if (!valid_tex(b, albedo)) return rtw::fail(-1, "rtw_material_metal: bad texture id"), -1;
    return add_material(b, RTW_MAT_METAL, albedo, fuzz, 0.0f);
}
extern "C" RTW_API int32_t rtw_material_dielectric(rtw_builder* b, float ior) {
    if (!b) return rtw::fail(-1, "rtw_material_dielectric: null builder"), -1;
    return add_material(b, RTW_MAT_DIELECTRIC, -1, 0.0f, ior);
}
extern "C" RTW_API int32_t rtw_material_diffuse_light(rtw_builder* b, int32_t emit) {
    if (!valid_tex(b, emit)) return rtw::fail(-1, "rtw_material_diffuse_light: bad texture id"), -1;
    return add_material(b, RTW_MAT_DIFFUSE_LIGHT, emit, 0.0f, 0.0f);
}
extern "C" RTW_API int32_t rtw_material_isotropic(rtw_builder* b, int32_t albedo) {
    if (!valid_tex(b, albedo)) return rtw::fail(-1, "rtw_material_isotropic: bad texture id"), -1;
    return add_material(b, RTW_MAT_ISOTROPIC, albedo, 0.0f, 0.0f);
}

extern "C" RTW_API int32_t rtw_node_group(rtw_builder* b) {
    if (!b) return rtw::fail(-1, "rtw_node_group: null builder"), -1;
    return add_node(b, Node{});
}
// world_builder.rs:97-103 geo_sphere (center ORIGIN)
extern "C" RTW_API int32_t rtw_node_sphere(rtw_builder* b, float radius, int32_t material) {
    if (!valid_mat(b, material)) return rtw::fail(-1, "rtw_node_sphere: bad material id"), -1;
    if (!(radius >= 0.0f)) return rtw::fail(-1, "rtw_node_sphere: radius must be >= 0 (sphere_geometry.rs:13)"), -1;
    Geom g;
    g.kind = RTW_GEOM_SPHERE;
    g.sphere.center[0] = g.sphere.center[1] = g.sphere.center[2] = 0.0f;
    g.sphere.radius = radius;
    return node_with_geo(b, g, material);
}
// world_builder.rs:76-90 geo_rect
extern "C" RTW_API int32_t rtw_node_rect(rtw_builder* b, int32_t plane, const float center[3], float s0, float s1,
                                         int32_t material) {
    if (!valid_mat(b, material) || !center || plane < 0 || plane > 2)
        return rtw::fail(-1, "rtw_node_rect: bad argument"), -1;
    int a0, a1, n;
    rect_axes(plane, &a0, &a1, &n);
    Geom g;
    g.kind = RTW_GEOM_RECT;
    g.rect.plane = plane;
    g.rect.dist = center[n];
    g.rect.r0[0] = center[a0] - s0 * 0.5f;
    g.rect.r0[1] = center[a0] + s0 * 0.5f;
    g.rect.r1[0] = center[a1] - s1 * 0.5f;
    g.rect.r1[1] = center[a1] + s1 * 0.5f;
    return node_with_geo(b, g, material);
}
// world_builder.rs:92-97 geo_box: Aabb(ORIGIN, (w, h, d))
extern "C" RTW_API int32_t rtw_node_box(rtw_builder* b, float w, float h, float d, int32_t material) {
    if (!valid_mat(b, material)) return rtw::fail(-1, "rtw_node_box: bad material id"), -1;
    Geom g;
    g.kind = RTW_GEOM_BOX;
    g.box.min[0] = g.box.min[1] = g.box.min[2] = 0.0f;
    g.box.max[0] = w;
    g.box.max[1] = h;
    g.box.max[2] = d;
    return node_with_geo(b, g, material);
}
// world_builder.rs:177-191 new_mesh_from_file_obj_uniform_material (triangles already parsed)
extern "C" RTW_API int32_t rtw_node_mesh(rtw_builder* b, const float* tris, int32_t n, int32_t material) {
    if (!valid_mat(b, material) || (n > 0 && !tris) || n < 0) return rtw::fail(-1, "rtw_node_mesh: bad argument"), -1;
    Node nd;
    for (int32_t i = 0; i < n; ++i) {
        Geom g;
        g.kind = RTW_GEOM_TRIANGLE;
        std::memcpy(&g.tri, tris + (size_t)i * 24u, sizeof(rtw_triangle));
        nd.geo.push_back(GeoEntry{g, material, false, 1.0f});
    }
    return add_node(b, std::move(nd));
}
extern "C" RTW_API int rtw_node_add(rtw_builder* b, int32_t parent, int32_t child) {
    if (!valid_node(b, parent) || !valid_node(b, child)) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_node_add: bad node id");
    b->nodes[(size_t)parent].children.push_back(child);
    return RTW_OK;
}
extern "C" RTW_API int rtw_node_translate(rtw_builder* b, int32_t node, float x, float y, float z) {
    if (!valid_node(b, node)) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_node_translate: bad node id");
    Node& n = b->nodes[(size_t)node];
    n.transformation = xf_translate(n.transformation, v3(x, y, z));
    return RTW_OK;
}
extern "C" RTW_API int rtw_node_rotate_around_up(rtw_builder* b, int32_t node, float degrees) {
    if (!valid_node(b, node)) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_node_rotate_around_up: bad node id");
    Node& n = b->nodes[(size_t)node];
    n.transformation = xf_rotate_around_up(n.transformation, degrees);
    return RTW_OK;
}
extern "C" RTW_API int rtw_node_animate_moving(rtw_builder* b, int32_t node, float x, float y, float z) {
    if (!valid_node(b, node)) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_node_animate_moving: bad node id");
    Node& n = b->nodes[(size_t)node];
    n.moving_animation = n.moving_animation + v3(x, y, z);
    return RTW_OK;
}
extern "C" RTW_API int rtw_node_set_all_geo_as_poi(rtw_builder* b, int32_t node) {
    if (!valid_node(b, node)) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_node_set_all_geo_as_poi: bad node id");
    for (GeoEntry& g : b->nodes[(size_t)node].geo) g.is_poi = true;
    return RTW_OK;
}
extern "C" RTW_API int rtw_node_set_all_geo_density(rtw_builder* b, int32_t node, float density) {
    if (!valid_node(b, node)) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_node_set_all_geo_density: bad node id");
    if (!(density >= 0.0f && density < 1.0f))  // world_builder.rs:261-270 panics otherwise
        return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "Invalid densitity " + std::to_string(density));
    for (GeoEntry& g : b->nodes[(size_t)node].geo) g.density = density;
    return RTW_OK;
}

// =============================================================================================
// C ABI: camera (camera.rs:11-173)
// =============================================================================================
extern "C" RTW_API int rtw_camera_build(const rtw_camera_spec* s, rtw_camera* out) {
    if (!s || !out) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_camera_build: null argument");
    float vw, vh;
    if (s->fov_mode == 1) {  // vertical_fov (camera.rs:72-79)
        const float h = std::tan(to_radians(s->fov_a) * 0.5f);
        vw = 2.0f * h;
        vh = 2.0f * h * s->fov_b;
    } else {
        vw = s->fov_a;
        vh = s->fov_b;
    }
    const V3 position = load3(s->position);
    const V3 up = load3(s->up);
    V3 forward;
    float focus_distance = 1.0f;  // camera.rs:46
    if (s->look_mode == 0) {
        forward = load3(s->target);  // orientation(up, forward)
    } else {
        forward = load3(s->target) - position;  // look_at / look_at_focus
        if (s->look_mode == 2) focus_distance = length(forward);
    }
    if (s->has_focus_point) focus_distance = length(position - load3(s->focus_point));  // :109-112
    if (s->has_focus_distance) focus_distance = s->focus_distance;                       // :117-120
    // ActualCameraBuilder::build (camera.rs:132-151)
    const V3 unit_right = unit(cross(forward, up));
    const V3 unit_up = unit(cross(unit_right, forward));
    const V3 sforward = with_length(forward, focus_distance);
    const V3 ulc = (unit_right * (vw * -0.5f) + unit_up * (vh * 0.5f)) * focus_distance + sforward;
    std::memset(out, 0, sizeof(*out));
    store3(out->position, position);
    store3(out->upper_left_corner, ulc);
    store3(out->unit_right, unit_right);
    store3(out->unit_up, unit_up);
    store3(out->scaled_right, unit_right * (focus_distance * vw));
    store3(out->scaled_up, unit_up * (focus_distance * vh));
    out->lens_radius = s->aperture / 2.0f;
    out->time0 = s->time0;
    out->time1 = s->time1;
    out->shutter_pace[0] = 0.0f;  // camera.rs:50, no setter
    out->shutter_pace[1] = 0.0f;
    return RTW_OK;
}
extern "C" RTW_API float rtw_camera_aspect_ratio(const rtw_camera* c) {
    if (!c) return 0.0f;
    return length(load3(c->scaled_up)) / length(load3(c->scaled_right));
}

// =============================================================================================
// C ABI: finish (world_builder.rs:273-290)
// =============================================================================================
extern "C" RTW_API int rtw_builder_finish(rtw_builder* b, int32_t root, const rtw_background* bg,
                                          const rtw_camera* cam, rtw_world_handle** out) {
    if (!valid_node(b, root) || !bg || !cam || !out)
        return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_builder_finish: bad argument");
    std::vector<Element> elems;
    bool have_wsd = false;
    rtw_rect wsd{};
    if (!finish_internal(b, root, Xf{}, elems, &have_wsd, &wsd, 0))
        return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_builder_finish: node graph has a cycle");
    if (elems.empty())  // the reference recurses forever on an empty BVH (hittable.rs:388-426)
        return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_builder_finish: the scene has no geometry");
    auto h = std::make_unique<rtw_world_handle>();
    // leaves + primitive tables (leaf i <-> element i)
    std::vector<BvhItem> items(elems.size());
    for (size_t i = 0; i < elems.size(); ++i) {
        const Element& e = elems[i];
        rtw_leaf L{};
        L.geom_kind = e.geo.kind;
        switch (e.geo.kind) {
            case RTW_GEOM_SPHERE: L.geom_index = (int32_t)h->spheres.size(); h->spheres.push_back(e.geo.sphere); break;
            case RTW_GEOM_RECT: L.geom_index = (int32_t)h->rects.size(); h->rects.push_back(e.geo.rect); break;
            case RTW_GEOM_BOX: L.geom_index = (int32_t)h->boxes.size(); h->boxes.push_back(e.geo.box); break;
            default: L.geom_index = (int32_t)h->triangles.size(); h->triangles.push_back(e.geo.tri); break;
        }
        L.material = e.material;
        L.flags = (e.volume ? RTW_LEAF_VOLUME : 0u) | (e.has_xf ? RTW_LEAF_TRANSFORM : 0u) |
                  (e.animated ? RTW_LEAF_ANIMATION : 0u);
        L.neg_inv_density = e.neg_inv_density;
        if (e.has_xf) {
            store3(L.offset, e.xf.offset);
            L.y_sin = e.xf.ys;
            L.y_cos = e.xf.yc;
        } else {
            L.y_sin = 0.0f;
            L.y_cos = 1.0f;
        }
        store3(L.velocity, e.velocity);
        h->leaves.push_back(L);
        items[i].id = -1 - (int32_t)i;
        items[i].aabb = element_bounding_box(e, cam->time0, cam->time1);
        for (int k = 0; k < 3; ++k)
            if (items[i].aabb.min.e[k] != items[i].aabb.min.e[k])  // partial_cmp().unwrap() panics
                return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_builder_finish: NaN bounding box");
    }
    Aabb root_box;
    int max_depth = 0;
    h->w.root = bvh_new(items.data(), items.size(), h->nodes, 0, &root_box, 0, &max_depth);
    if (max_depth > 60) return rtw::fail(RTW_ERR_UNSUPPORTED, "rtw_builder_finish: BVH deeper than 60 levels");
    h->materials = b->materials;
    h->textures = b->textures;
    h->image_data = b->images;
    for (size_t i = 0; i < h->image_data.size(); ++i) {
        rtw_image im{};
        im.width = b->image_dims[i].first;
        im.height = b->image_dims[i].second;
        im.rgb = h->image_data[i].data();
        h->images.push_back(im);
    }
    h->perlins = b->perlins;
    h->w.camera = *cam;
    h->w.background = *bg;
    h->w.has_light = have_wsd ? 1 : 0;
    h->w.light = wsd;
    rtw_world& w = h->w;
    w.node_count = (int32_t)h->nodes.size();
    w.nodes = h->nodes.data();
    w.leaf_count = (int32_t)h->leaves.size();
    w.leaves = h->leaves.data();
    w.sphere_count = (int32_t)h->spheres.size();
    w.spheres = h->spheres.data();
    w.rect_count = (int32_t)h->rects.size();
    w.rects = h->rects.data();
    w.box_count = (int32_t)h->boxes.size();
    w.boxes = h->boxes.data();
    w.triangle_count = (int32_t)h->triangles.size();
    w.triangles = h->triangles.data();
    w.material_count = (int32_t)h->materials.size();
    w.materials = h->materials.data();
    w.texture_count = (int32_t)h->textures.size();
    w.textures = h->textures.data();
    w.image_count = (int32_t)h->images.size();
    w.images = h->images.data();
    w.perlin_count = (int32_t)h->perlins.size();
    w.perlins = h->perlins.data();
    *out = h.release();
    return RTW_OK;
}
extern "C" RTW_API const rtw_world* rtw_world_get(const rtw_world_handle* h) { return h ? &h->w : nullptr; }
extern "C" RTW_API void rtw_world_free(rtw_world_handle* h) { delete h; }
extern "C" RTW_API void rtw_free(void* p) { std::free(p); }

// =============================================================================================
// OBJ loader (obj_loader.rs)
// =============================================================================================
namespace {

struct Scanner {  // obj_loader.rs:31-212 (ASCII subset of char::is_numeric)
    const char* p;
    const char* end;
    bool peek_is(char c) const { return p < end && *p == c; }
    bool at_end() const { return p >= end; }
    bool take_char(char c) {
        if (peek_is(c)) { ++p; return true; }
        return false;
    }
    bool take_at_least_one_ws() {
        if (!take_char(' ')) return false;
        while (take_char(' ')) {}
        return true;
    }
    void take_any_ws() { while (take_char(' ')) {} }
    bool take_digits(std::string* s) {
        if (!(p < end && *p >= '0' && *p <= '9')) return false;
        while (p < end && *p >= '0' && *p <= '9') s->push_back(*p++);
        return true;
    }
    bool take_usize(size_t* v) {
        std::string s;
        if (!take_digits(&s)) return false;
        *v = (size_t)std::strtoull(s.c_str(), nullptr, 10);
        return true;
    }
    bool take_f32(float* v) {  // take_float_digits: -? digits (. digits)?
        std::string s;
        if (take_char('-')) s.push_back('-');
        if (!take_digits(&s)) return false;
        if (take_char('.')) {
            s.push_back('.');
            if (!take_digits(&s)) return false;
        }
        *v = std::strtof(s.c_str(), nullptr);  // correctly rounded, as str::parse::<f32>
        return true;
    }
    bool take_vec(float* v, int n) {
        for (int i = 0; i < n; ++i) {
            if (!take_at_least_one_ws()) return false;
            if (!take_f32(&v[i])) return false;
        }
        return true;
    }
    // (pos, uv?, normal?) with 1-based ids converted to 0-based
    bool take_vertex(size_t* pos, long* uv, long* nor) {
        size_t a;
        if (!take_usize(&a)) return false;
        *pos = a - 1;
        *uv = -1;
        *nor = -1;
        take_any_ws();
        if (take_char('/')) {
            take_any_ws();
            if (take_char('/')) {
                take_any_ws();
                size_t n;
                if (!take_usize(&n)) return false;
                *nor = (long)(n - 1);
            } else {
                size_t t;
                if (!take_usize(&t)) return false;
                *uv = (long)(t - 1);
                take_any_ws();
                if (take_char('/')) {
                    take_any_ws();
                    size_t n;
                    if (!take_usize(&n)) return false;
                    *nor = (long)(n - 1);
                }
            }
        }
        return true;
    }
};

}  // namespace

extern "C" RTW_API int rtw_obj_parse(const char* text, size_t len, float** out, int32_t* n_out) {
    if (!text || !out || !n_out) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_obj_parse: null argument");
    std::vector<V3> positions, normals;
    std::vector<std::pair<float, float>> uvs;
    std::vector<rtw_triangle> tris;
    size_t line_no = 0;
    const char* cur = text;
    const char* end = text + len;
    while (cur < end) {
        const char* nl = (const char*)std::memchr(cur, '\n', (size_t)(end - cur));
        const char* le = nl ? nl : end;
        const char* next = nl ? nl + 1 : end;
        if (le > cur && le[-1] == '\r') --le;  // BufRead::lines strips "\r\n"
        ++line_no;
        Scanner sc{cur, le};
        auto err = [&](const char* what) {
            return rtw::fail(RTW_ERR_PARSE, std::string("rtw_obj_parse: line ") + std::to_string(line_no) + ": " + what);
        };
        if (sc.take_char('v')) {
            float v[3];
            if (sc.take_char('n')) {
                if (!sc.take_vec(v, 3)) return err("bad vn");
                normals.push_back(v3(v[0], v[1], v[2]));
            } else if (sc.take_char('t')) {
                if (!sc.take_vec(v, 2)) return err("bad vt");
                uvs.emplace_back(v[0], v[1]);
            } else {
                if (!sc.take_vec(v, 3)) return err("bad v");
                positions.push_back(v3(v[0], v[1], v[2]));
            }
        } else if (sc.take_char('f')) {
            if (!sc.take_at_least_one_ws()) return err("expected whitespace after f");
            rtw_triangle tri{};  // all ORIGIN / ZERO (obj_loader.rs:227-231)
            int i = 0;
            while (!sc.at_end()) {
                size_t pid;
                long uid, nid;
                if (!sc.take_vertex(&pid, &uid, &nid)) return err("bad face vertex");
                sc.take_any_ws();
                if (pid >= positions.size()) return err("PosIdOutOfRange");
                const V3 position = positions[pid];
                float uv[2] = {0.0f, 0.0f};
                if (uid >= 0) {
                    if ((size_t)uid >= uvs.size()) return err("TexIdOutOfRange");
                    uv[0] = uvs[(size_t)uid].first;
                    uv[1] = uvs[(size_t)uid].second;
                }
                if (nid < 0) return rtw::fail(RTW_ERR_UNSUPPORTED, "rtw_obj_parse: faces without normals are todo!() in the reference (obj_loader.rs:249)");
                if ((size_t)nid >= normals.size()) return err("NorIdOutOfRange");
                const V3 normal = normals[(size_t)nid];
                if (i < 2) {
                    store3(tri.positions[i], position);
                    store3(tri.normals[i], normal);
                    tri.uvs[i][0] = uv[0];
                    tri.uvs[i][1] = uv[1];
                } else {  // the fan quirk: slot 1 takes slot 2's OLD value (ORIGIN for i == 2)
                    std::memcpy(tri.positions[1], tri.positions[2], sizeof(tri.positions[1]));
                    std::memcpy(tri.normals[1], tri.normals[2], sizeof(tri.normals[1]));
                    std::memcpy(tri.uvs[1], tri.uvs[2], sizeof(tri.uvs[1]));
                    store3(tri.positions[2], position);
                    store3(tri.normals[2], normal);
                    tri.uvs[2][0] = uv[0];
                    tri.uvs[2][1] = uv[1];
                    tris.push_back(tri);
                }
                ++i;
            }
        }
        // '#', 'o' and anything else: ignored
        cur = next;
    }
    float* buf = (float*)std::malloc(std::max<size_t>(1, tris.size()) * sizeof(rtw_triangle));
    if (!buf) return rtw::fail(RTW_ERR_OUT_OF_MEMORY, "rtw_obj_parse: out of memory");
    if (!tris.empty()) std::memcpy(buf, tris.data(), tris.size() * sizeof(rtw_triangle));
    *out = buf;
    *n_out = (int32_t)tris.size();
    return RTW_OK;
}
