// demo_worlds.cpp -- the reference's demo scenes (src/app/worlds/demo_worlds.rs), built through
// the WorldBuilder C ABI (scene_builder.cpp) with the scene RNG seeded as main.rs:24.
// Two composed worlds cover BASELINE configs the reference has no single scene for:
//   "cornell_cube"  C3: create_cornell_box_node(130) + cube.obj (white Lambert, vertices x82.5
//                   at load since Transformation has no scale, translated to (278, 82.5, 200))
//   "earth_motion"  C5: moving_spheres content (checker ground, two animated spheres,
//                   motion_blur(0, 0.5)) + the earth-textured sphere, camera aspect 9/16.
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rtw_scalar.h"
#include "rtw_common.h"

namespace {

struct B {  // a thin fluent wrapper over the builder C ABI
    rtw_builder* b;
    rtw_rng* rng;
    bool ok = true;
    int32_t chk(int32_t id) {
        if (id < 0) ok = false;
        return id;
    }
    int32_t tex_solid(float r, float g, float bl) { return chk(rtw_texture_solid(b, r, g, bl)); }
    int32_t lambert_solid(float r, float g, float bl) { return chk(rtw_material_lambert(b, tex_solid(r, g, bl))); }
    int32_t lambert(int32_t t) { return chk(rtw_material_lambert(b, t)); }
    int32_t metal_solid(float r, float g, float bl, float fuzz) { return chk(rtw_material_metal(b, tex_solid(r, g, bl), fuzz)); }
    int32_t dielectric(float ior) { return chk(rtw_material_dielectric(b, ior)); }
    int32_t light_solid(float r, float g, float bl) { return chk(rtw_material_diffuse_light(b, tex_solid(r, g, bl))); }
    int32_t isotropic_solid(float r, float g, float bl) { return chk(rtw_material_isotropic(b, tex_solid(r, g, bl))); }
    int32_t group() { return chk(rtw_node_group(b)); }
    int32_t sphere(float r, int32_t m) { return chk(rtw_node_sphere(b, r, m)); }
    int32_t box(float w, float h, float d, int32_t m) { return chk(rtw_node_box(b, w, h, d, m)); }
    int32_t rect(int plane, float cx, float cy, float cz, float s0, float s1, int32_t m) {
        const float c[3] = {cx, cy, cz};
        return chk(rtw_node_rect(b, plane, c, s0, s1, m));
    }
    int32_t translate(int32_t n, float x, float y, float z) {
        if (rtw_node_translate(b, n, x, y, z) != RTW_OK) ok = false;
        return n;
    }
    int32_t rotate(int32_t n, float deg) {
        if (rtw_node_rotate_around_up(b, n, deg) != RTW_OK) ok = false;
        return n;
    }
    int32_t animate(int32_t n, float x, float y, float z) {
        if (rtw_node_animate_moving(b, n, x, y, z) != RTW_OK) ok = false;
        return n;
    }
    int32_t poi(int32_t n) {
        if (rtw_node_set_all_geo_as_poi(b, n) != RTW_OK) ok = false;
        return n;
    }
    int32_t density(int32_t n, float d) {
        if (rtw_node_set_all_geo_density(b, n, d) != RTW_OK) ok = false;
        return n;
    }
    int32_t add(int32_t parent, int32_t child) {
        if (rtw_node_add(b, parent, child) != RTW_OK) ok = false;
        return parent;
    }
};

}  // namespace

namespace {

rtw_camera_spec cam_vfov(float vfov, float aspect, float px, float py, float pz, float tx, float ty, float tz) {
    rtw_camera_spec s;
    std::memset(&s, 0, sizeof(s));
    s.fov_mode = 1;
    s.fov_a = vfov;
    s.fov_b = aspect;
    s.position[0] = px;
    s.position[1] = py;
    s.position[2] = pz;
    s.look_mode = 1;  // look_at
    s.up[0] = 0.0f;
    s.up[1] = 1.0f;
    s.up[2] = 0.0f;
    s.target[0] = tx;
    s.target[1] = ty;
    s.target[2] = tz;
    return s;
}

rtw_background sky() {
    rtw_background bg;
    std::memset(&bg, 0, sizeof(bg));
    bg.kind = RTW_BG_SKY;
    return bg;
}
rtw_background solid(float r, float g, float b) {
    rtw_background bg;
    bg.kind = RTW_BG_SOLID;
    bg.color[0] = r;
    bg.color[1] = g;
    bg.color[2] = b;
    return bg;
}

// demo_worlds.rs:216-264
int32_t cornell_box_node(B& w, float light_size) {
    const int32_t red = w.lambert_solid(0.65f, 0.05f, 0.05f);
    const int32_t white = w.lambert_solid(0.73f, 0.73f, 0.73f);
    const int32_t green = w.lambert_solid(0.12f, 0.45f, 0.15f);
    const int32_t light = w.light_solid(15.0f, 15.0f, 15.0f);
    const float h = 278.0f;
    const int32_t g = w.group();
    w.add(g, w.rect(RTW_PLANE_YZ, 0.0f, h, h, 2.0f * h, 2.0f * h, red));
    w.add(g, w.rect(RTW_PLANE_YZ, 2.0f * h, h, h, 2.0f * h, 2.0f * h, green));
    w.add(g, w.rect(RTW_PLANE_XZ, h, 0.0f, h, 2.0f * h, 2.0f * h, white));
    w.add(g, w.rect(RTW_PLANE_XZ, h, 2.0f * h, h, 2.0f * h, 2.0f * h, white));
    w.add(g, w.rect(RTW_PLANE_XY, h, h, 2.0f * h, 2.0f * h, 2.0f * h, white));
    w.add(g, w.poi(w.rect(RTW_PLANE_XZ, h, 2.0f * h - 1.0f, h, light_size, light_size, light)));
    return g;
}

int32_t mesh(B& w, const float* tris, int32_t n, float scale, int32_t material) {
    std::vector<float> t(tris, tris + (size_t)n * 24u);
    if (scale != 1.0f)
        for (int32_t i = 0; i < n; ++i)
            for (int k = 0; k < 9; ++k) t[(size_t)i * 24u + (size_t)k] *= scale;  // positions only
    return w.chk(rtw_node_mesh(w.b, t.data(), n, material));
}

int finish(B& w, int32_t root, const rtw_background& bg, const rtw_camera_spec& cs, rtw_world_handle** out) {
    if (!w.ok) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_demo_world: builder call failed");
    rtw_camera cam;
    const int rc = rtw_camera_build(&cs, &cam);
    if (rc != RTW_OK) return rc;
    return rtw_builder_finish(w.b, root, &bg, &cam, out);
}

// demo_worlds.rs:395-463
int final_scene1(B& w, rtw_world_handle** out) {
    rtw_camera_spec cs = cam_vfov(60.0f, 9.0f / 16.0f, 13.0f, 2.0f, 3.0f, 0.0f, 0.0f, 0.0f);
    cs.has_focus_distance = 1;
    cs.focus_distance = 10.0f;
    cs.aperture = 0.1f;
    const int32_t mat_ground = w.lambert_solid(0.5f, 0.5f, 0.5f);
    const int32_t scene = w.group();
    const float ground_radius = 1000.0f;
    const float gcx = 0.0f, gcy = -ground_radius, gcz = 0.0f;
    w.add(scene, w.translate(w.sphere(ground_radius, mat_ground), 0.0f, 0.0f - ground_radius, 0.0f));
    const int32_t glass = w.dielectric(1.5f);
    rtw_xoro& rng = w.rng->s;
    auto gen_color = [&](float c[3]) {
        c[0] = rtw_gen_f32(&rng);
        c[1] = rtw_gen_f32(&rng);
        c[2] = rtw_gen_f32(&rng);
    };
    for (int a = -11; a <= 11; ++a) {
        for (int b = -11; b <= 11; ++b) {
            const float ox = rtw_gen_f32(&rng) * 0.9f;
            const float oz = rtw_gen_f32(&rng) * 0.9f;
            const float cx = (float)a + ox, cy = 0.2f + 0.0f, cz = (float)b + oz;
            const float dx = cx - 4.0f, dy = cy - 0.2f, dz = cz - 0.0f;
            if (std::sqrt(dx * dx + dy * dy + dz * dz) > 0.9f) {
                int32_t material;
                const float sample = rtw_gen_f32(&rng);
                if (sample < 0.8f) {
                    float c1[3], c2[3];
                    gen_color(c1);
                    gen_color(c2);
                    material = w.lambert_solid(c1[0] * c2[0], c1[1] * c2[1], c1[2] * c2[2]);
                } else if (sample < 0.95f) {
                    float c[3];
                    gen_color(c);
                    const float fuzz = rtw_gen_range_f32(0.0f, 0.5f, &rng);
                    material = w.metal_solid(c[0], c[1], c[2], fuzz);
                } else {
                    material = glass;
                }
                const float small_radius = 0.2f;
                // ground_center + (center - ground_center).with_length(R + r)
                const float vx = cx - gcx, vy = cy - gcy, vz = cz - gcz;
                const float len = std::sqrt(vx * vx + vy * vy + vz * vz);
                const float k = (ground_radius + small_radius) / len;
                const float rx = gcx + vx * k, ry = gcy + vy * k, rz = gcz + vz * k;
                w.add(scene, w.translate(w.sphere(small_radius, material), rx, ry, rz));
            }
        }
    }
    w.add(scene, w.translate(w.sphere(1.0f, glass), 0.0f, 1.0f, 0.0f));
    const int32_t big_solid = w.lambert_solid(0.4f, 0.2f, 0.1f);
    w.add(scene, w.translate(w.sphere(1.0f, big_solid), -4.0f, 1.0f, 0.0f));
    const int32_t big_metal = w.metal_solid(0.7f, 0.6f, 0.5f, 0.0f);
    w.add(scene, w.translate(w.sphere(1.0f, big_metal), 4.0f, 1.0f, 0.0f));
    return finish(w, scene, sky(), cs, out);
}

// demo_worlds.rs:30-152
int final_scene2(B& w, const rtw_assets* assets, rtw_world_handle** out) {
    rtw_camera_spec cs = cam_vfov(40.0f, 1.0f, 478.0f, 278.0f, -600.0f, 278.0f, 278.0f, 0.0f);
    cs.time0 = 0.0f;
    cs.time1 = 1.0f;
    rtw_xoro& rng = w.rng->s;
    const int32_t mat_ground = w.lambert_solid(0.48f, 0.83f, 0.53f);
    const int32_t ground = w.group();
    {
        const int n = 20;
        const float minx = -1000.0f, miny = 0.0f, minz = -1000.0f;
        const float maxx = 1000.0f, maxy = 101.0f, maxz = 1000.0f;
        const float width = (maxx - minx) / (float)n;
        const float height = maxy - miny;
        const float depth = (maxz - minz) / (float)n;
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                // range.min + Dir3(i*width, 0, j*depth) - ORIGIN
                const float mx = (minx + (float)i * width) - 0.0f;
                const float my = (miny + 0.0f) - 0.0f;
                const float mz = (minz + (float)j * depth) - 0.0f;
                const float hh = height * rtw_gen_f32(&rng);
                w.add(ground, w.translate(w.box(width, hh, depth, mat_ground), mx, my, mz));
            }
    }
    const int32_t mat_light = w.light_solid(7.0f, 7.0f, 7.0f);
    const int32_t light = w.rect(RTW_PLANE_XZ, 273.0f, 554.0f, 279.0f, 300.0f, 300.0f, mat_light);
    const int32_t mat_glass = w.dielectric(1.5f);
    const int32_t mat_metal = w.metal_solid(0.8f, 0.8f, 0.9f, 1.0f);
    const int32_t tex_marble = w.chk(rtw_texture_marble(w.b, 0.1f, w.rng));
    const int32_t mat_marble = w.lambert(tex_marble);
    if (!assets || !assets->earth_rgb) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "final_scene2 needs the earth texture");
    const int32_t tex_earth = w.chk(rtw_texture_image_rgb8(w.b, assets->earth_rgb, assets->earth_width, assets->earth_height));
    const int32_t mat_earth = w.lambert(tex_earth);
    const int32_t mat_fog = w.isotropic_solid(0.2f, 0.4f, 0.9f);
    const int32_t mat_moving = w.lambert_solid(0.7f, 0.3f, 0.1f);
    const int32_t floating = w.group();
    w.add(floating, w.translate(w.sphere(70.0f, mat_glass), 360.0f, 150.0f, 145.0f));
    w.add(floating, w.density(w.translate(w.sphere(70.0f, mat_fog), 360.0f, 150.0f, 145.0f), 0.2f));
    w.add(floating, w.translate(w.sphere(50.0f, mat_glass), 260.0f, 150.0f, 45.0f));
    w.add(floating, w.translate(w.sphere(50.0f, mat_metal), 0.0f, 150.0f, 145.0f));
    w.add(floating, w.translate(w.sphere(80.0f, mat_marble), 220.0f, 280.0f, 300.0f));
    w.add(floating, w.translate(w.sphere(100.0f, mat_earth), 400.0f, 200.0f, 400.0f));
    w.add(floating, w.animate(w.translate(w.sphere(50.0f, mat_moving), 400.0f, 400.0f, 200.0f), 30.0f, 0.0f, 0.0f));
    int32_t cube;
    {
        const int32_t material = w.lambert_solid(0.75f, 0.75f, 0.75f);
        cube = w.group();
        // rot = ZERO.rotate_around_up(15); dir_k = rot.apply_direction(RIGHT / UP / FORWARD)
        const float rad = 15.0f * (3.14159274101257324219f / 180.0f);
        const float s = std::sin(rad), c = std::cos(rad);
        // ZERO.rotate_around_up: ys' = c*0 + s*1, yc' = -s*0 + c*1
        const float ys = c * 0.0f + s * 1.0f, yc = -s * 0.0f + c * 1.0f;
        auto rot = [&](float x, float y, float z, float o[3]) {
            o[0] = yc * x + ys * z;
            o[1] = y;
            o[2] = -ys * x + yc * z;
        };
        float d1[3], d2[3], d3[3];
        rot(1.0f, 0.0f, 0.0f, d1);
        rot(0.0f, 1.0f, 0.0f, d2);
        rot(0.0f, 0.0f, -1.0f, d3);
        for (int i = 0; i < 1000; ++i) {
            const float r0 = rtw_gen_f32(&rng), r1 = rtw_gen_f32(&rng), r2 = rtw_gen_f32(&rng);
            float p[3];
            const float o[3] = {-100.0f, 270.0f, 395.0f};
            for (int k = 0; k < 3; ++k) p[k] = o[k] + ((d1[k] * r0 + d2[k] * r1) + d3[k] * r2) * 165.0f;
            w.add(cube, w.translate(w.sphere(10.0f, material), p[0], p[1], p[2]));
        }
    }
    const int32_t fog = w.density(w.sphere(5000.0f, w.isotropic_solid(1.0f, 1.0f, 1.0f)), 0.0001f);
    const int32_t scene = w.group();
    w.add(scene, fog);
    w.add(scene, ground);
    w.add(scene, cube);
    w.add(scene, floating);
    w.add(scene, light);
    return finish(w, scene, solid(0.0f, 0.0f, 0.0f), cs, out);
}

}  // namespace

extern "C" RTW_API int rtw_demo_world(const char* name, const rtw_assets* assets, rtw_world_handle** out) {
    if (!name || !out) return rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_demo_world: null argument");
    const uint8_t seed[16] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};  // main.rs:24
    rtw_builder* bld = rtw_builder_new();
    rtw_rng* rng = rtw_rng_from_seed(seed);
    B w{bld, rng};
    const std::string n(name);
    int rc;
    if (n == "final_scene1") {
        rc = final_scene1(w, out);
    } else if (n == "final_scene2") {
        rc = final_scene2(w, assets, out);
    } else if (n == "suzanne") {  // demo_worlds.rs:6-28
        if (!assets || !assets->suzanne_tris) {
            rc = rtw::fail(RTW_ERR_INVALID_ARGUMENT, "suzanne needs the suzanne mesh");
        } else {
            const rtw_camera_spec cs = cam_vfov(40.0f, 3.0f / 4.0f, 0.0f, 2.0f, 10.0f, 0.0f, 0.0f, 0.0f);
            const int32_t mat_ground = w.lambert_solid(0.4f, 0.4f, 0.4f);
            const int32_t mat_monkey = w.lambert_solid(1.0f, 0.2f, 0.2f);
            const int32_t scene = w.group();
            w.add(scene, mesh(w, assets->suzanne_tris, assets->suzanne_count, 1.0f, mat_monkey));
            w.add(scene, w.translate(w.sphere(1000.1f, mat_ground), 0.0f, -1000.0f, 0.0f));
            rc = finish(w, scene, sky(), cs, out);
        }
    } else if (n == "perlin_spheres") {  // demo_worlds.rs:154-177
        const rtw_camera_spec cs = cam_vfov(40.0f, 3.0f / 4.0f, 13.0f, 2.0f, 3.0f, 0.0f, 0.0f, 0.0f);
        const int32_t tex = w.chk(rtw_texture_marble(bld, 4.0f, rng));
        const int32_t mat = w.lambert(tex);
        const int32_t scene = w.group();
        w.add(scene, w.translate(w.sphere(1000.0f, mat), 0.0f, 0.0f - 1000.0f, 0.0f));
        w.add(scene, w.translate(w.sphere(2.0f, mat), 0.0f, 2.0f, 0.0f));
        rc = finish(w, scene, sky(), cs, out);
    } else if (n == "cornell_box" || n == "cornell_box_smoke" || n == "cornell_cube") {
        const float h = 278.0f;
        const rtw_camera_spec cs = cam_vfov(40.0f, 1.0f, h, h, -800.0f, h, h, 0.0f);
        int32_t white_or_smoke_w, black_or_white;
        if (n == "cornell_box_smoke") {  // demo_worlds.rs:179-214
            black_or_white = w.isotropic_solid(0.0f, 0.0f, 0.0f);
            white_or_smoke_w = w.isotropic_solid(1.0f, 1.0f, 1.0f);
        } else {  // demo_worlds.rs:266-296
            white_or_smoke_w = w.lambert_solid(0.73f, 0.73f, 0.73f);
            black_or_white = white_or_smoke_w;
        }
        const int32_t cbox = cornell_box_node(w, 130.0f);
        const int32_t scene = w.group();
        w.add(scene, cbox);
        if (n == "cornell_cube") {
            if (!assets || !assets->cube_tris) {
                rc = rtw::fail(RTW_ERR_INVALID_ARGUMENT, "cornell_cube needs the cube mesh");
                rtw_rng_free(rng);
                rtw_builder_free(bld);
                return rc;
            }
            w.add(scene, w.translate(mesh(w, assets->cube_tris, assets->cube_count, 82.5f, white_or_smoke_w),
                                     278.0f, 82.5f, 200.0f));
        } else {
            int32_t b1 = w.translate(w.rotate(w.box(165.0f, 330.0f, 165.0f, white_or_smoke_w), 15.0f), 265.0f, 0.0f, 295.0f);
            int32_t b2 = w.translate(w.rotate(w.box(165.0f, 165.0f, 165.0f, black_or_white), -18.0f), 130.0f, 0.0f, 65.0f);
            if (n == "cornell_box_smoke") {
                w.density(b1, 0.01f);
                w.density(b2, 0.01f);
            }
            w.add(scene, b1);
            w.add(scene, b2);
        }
        rc = finish(w, scene, solid(0.0f, 0.0f, 0.0f), cs, out);
    } else if (n == "simple_plane") {  // demo_worlds.rs:298-324
        const rtw_camera_spec cs = cam_vfov(60.0f, 9.0f / 16.0f, 0.0f, 6.0f, 10.0f, 0.0f, 0.0f, 0.0f);
        const int32_t emit = w.light_solid(1.0f * 100.0f, 1.0f * 100.0f, 1.0f * 100.0f);
        const int32_t floor = w.lambert_solid(0.0f, 0.0f, 0.4f);
        const int32_t scene = w.group();
        w.add(scene, w.poi(w.rect(RTW_PLANE_XY, 0.0f, 2.0f, 0.0f, 1.0f, 1.0f, emit)));
        w.add(scene, w.rect(RTW_PLANE_XZ, 0.0f, 0.0f, 0.0f, 10.0f, 10.0f, floor));
        rc = finish(w, scene, solid(0.1f, 0.1f, 0.1f), cs, out);
    } else if (n == "earth_mapped") {  // demo_worlds.rs:326-349
        if (!assets || !assets->earth_rgb) {
            rc = rtw::fail(RTW_ERR_INVALID_ARGUMENT, "earth_mapped needs the earth texture");
        } else {
            const rtw_camera_spec cs = cam_vfov(60.0f, 16.0f / 19.0f, 0.0f, 2.0f, 10.0f, 0.0f, 0.0f, 0.0f);
            const int32_t tex = w.chk(rtw_texture_image_rgb8(bld, assets->earth_rgb, assets->earth_width, assets->earth_height));
            const int32_t mat = w.lambert(tex);
            const int32_t scene = w.group();
            w.add(scene, w.sphere(2.0f, mat));
            rc = finish(w, scene, sky(), cs, out);
        }
    } else if (n == "moving_spheres" || n == "earth_motion") {  // demo_worlds.rs:351-393
        const bool earth = n == "earth_motion";
        if (earth && (!assets || !assets->earth_rgb)) {
            rc = rtw::fail(RTW_ERR_INVALID_ARGUMENT, "earth_motion needs the earth texture");
        } else {
            rtw_camera_spec cs = cam_vfov(60.0f, earth ? 9.0f / 16.0f : 16.0f / 19.0f, 0.0f, 2.0f, 10.0f, 0.0f, 2.0f, 0.0f);
            cs.time0 = 0.0f;
            cs.time1 = 0.5f;
            const int32_t black = w.tex_solid(0.0f, 0.0f, 0.0f);
            const int32_t whitet = w.tex_solid(1.0f, 1.0f, 1.0f);
            const int32_t checker = w.chk(rtw_texture_checker(bld, 10.0f, black, whitet));
            const int32_t mat_ground = w.lambert(checker);
            const int32_t red = w.lambert_solid(0.6f, 0.2f, 0.2f);
            const int32_t blue = w.lambert_solid(0.2f, 0.2f, 0.6f);
            const int32_t scene = w.group();
            w.add(scene, w.translate(w.sphere(100.0f, mat_ground), 0.0f, -100.0f, 0.0f));
            w.add(scene, w.animate(w.translate(w.sphere(0.5f, red), -2.0f, 1.5f, 0.0f), 2.0f, 0.0f, 0.0f));
            w.add(scene, w.animate(w.translate(w.sphere(0.5f, blue), 0.0f, 0.5f, 0.0f), 0.0f, 1.0f, 0.0f));
            if (earth) {
                const int32_t tex = w.chk(rtw_texture_image_rgb8(bld, assets->earth_rgb, assets->earth_width, assets->earth_height));
                w.add(scene, w.translate(w.sphere(2.0f, w.lambert(tex)), 2.5f, 2.0f, -3.0f));
            }
            rc = finish(w, scene, sky(), cs, out);
        }
    } else if (n == "defocus_blur") {  // demo_worlds.rs:465-508
        rtw_camera_spec cs;
        std::memset(&cs, 0, sizeof(cs));
        cs.fov_mode = 1;
        cs.fov_a = 60.0f;
        cs.fov_b = 9.0f / 16.0f;
        // ORIGIN + BACKWARD*3 + UP*3 + 3*RIGHT
        cs.position[0] = ((0.0f + 0.0f * 3.0f) + 0.0f * 3.0f) + 1.0f * 3.0f;
        cs.position[1] = ((0.0f + 0.0f * 3.0f) + 1.0f * 3.0f) + 0.0f * 3.0f;
        cs.position[2] = ((0.0f + 1.0f * 3.0f) + 0.0f * 3.0f) + 0.0f * 3.0f;
        cs.look_mode = 2;  // look_at_focus(UP, ORIGIN + FORWARD)
        cs.up[1] = 1.0f;
        cs.target[0] = 0.0f + 0.0f;
        cs.target[1] = 0.0f + 0.0f;
        cs.target[2] = 0.0f + -1.0f;
        cs.aperture = 0.1f;
        const int32_t ground = w.lambert_solid(0.8f, 0.8f, 0.0f);
        const int32_t center = w.lambert_solid(0.7f, 0.3f, 0.3f);
        const int32_t left = w.metal_solid(0.6f, 0.6f, 0.8f, 0.05f);
        const int32_t right = w.metal_solid(0.8f, 0.6f, 0.2f, 0.5f);
        const int32_t front = w.dielectric(1.5f);
        const int32_t scene = w.group();
        w.add(scene, w.translate(w.sphere(100.0f, ground), 0.0f * 100.5f, -1.0f * 100.5f, 0.0f * 100.5f));
        w.add(scene, w.translate(w.sphere(0.5f, center), 0.0f, 0.0f, -1.0f));
        w.add(scene, w.translate(w.sphere(0.5f, left), -1.0f + 0.0f, 0.0f + 0.0f, 0.0f + -1.0f));
        w.add(scene, w.translate(w.sphere(0.5f, right), 1.0f + 0.0f, 0.0f + 0.0f, 0.0f + -1.0f));
        w.add(scene, w.translate(w.sphere(0.3f, front), -1.0f * 0.5f + 0.0f * 0.3f, 0.0f * 0.5f + 1.0f * 0.3f,
                                 0.0f * 0.5f + 0.0f * 0.3f));
        rc = finish(w, scene, sky(), cs, out);
    } else {
        rc = rtw::fail(RTW_ERR_INVALID_ARGUMENT, "rtw_demo_world: unknown world '" + n + "'");
    }
    rtw_rng_free(rng);
    rtw_builder_free(bld);
    return rc;
}
