//! src/lib/gpu.rs -- the reference crate's binding to librtw.so (include/rtw.h, ABI version 2).
//!
//! `render_gpu` has exactly the signature of `rendering::render` (src/lib/rendering.rs:121-128)
//! and returns the same `Vec<Color>` (W*H linear radiance, row-major from the top-left pixel):
//! `main.rs:43-50` can call it in place of `render` and keep `to_rgb8_gamma2` + `save_buffer`
//! (main.rs:53-63).  It serialises the `World` the app's WorldBuilder produced
//! (world_builder.rs:273-328: one top-level BVH over flattened leaves) into the flat `rtw_world`
//! and calls `rtw_render_progress`, whose callback prints the reference's "\r{done} %" line.
//!
//! Install: copy this file to src/lib/gpu.rs, add `pub mod gpu;` to src/lib/lib.rs, copy
//! integration/rust/build.rs next to Cargo.toml, and widen these private fields to `pub(crate)`
//! (the serialiser reads them; nothing else changes):
//!   camera.rs:156-160          Camera::{upper_left_corner, scaled_right, scaled_up}
//!   hittable.rs:122            Scene::root
//!   hittable.rs:294-298        VolumeGeometry::{boundary, phase_function, neg_inv_density}
//!   hittable.rs:345-357        BoundingVolumeNode::{aabb, axis_id, left, right} (and the struct),
//!                              BoundingVolumeHierarchy::{items, unbounded_items, nodes, initial_index}
//!   transformations.rs:4-8     Transformation::{offset, y_sine, y_cosine}
//!   perlin.rs:10-16            Perlin::{ranvec, perm_x, perm_y, perm_z, bits}
//!
//! The `#[repr(C)]` structs below mirror include/rtw.h field for field;
//! tests/test_rust_shim.py checks their names, types, offsets and sizes against the header with
//! the C compiler (this image has no rustc), plus the constants and the extern signatures.
//!
//! Errors: librtw returns status codes; like every other failure in the reference
//! (`unwrap`, `panic!`), a non-zero code panics here, with rtw_last_error()'s message.

use crate::hittable::rect_geometry::{RectGeometry, RectPlane};
use crate::*;
use std::collections::HashMap;
use std::ffi::CStr;
use std::os::raw::{c_char, c_int, c_void};

// ---- constants (include/rtw.h) ---------------------------------------------------------------
pub const RTW_ABI_VERSION: c_int = 2;
pub const RTW_OK: c_int = 0;
pub const RTW_GEOM_SPHERE: i32 = 0;
pub const RTW_GEOM_RECT: i32 = 1;
pub const RTW_GEOM_BOX: i32 = 2;
pub const RTW_GEOM_TRIANGLE: i32 = 3;
pub const RTW_PLANE_XY: i32 = 0;
pub const RTW_PLANE_XZ: i32 = 1;
pub const RTW_PLANE_YZ: i32 = 2;
pub const RTW_MAT_LAMBERT: i32 = 0;
pub const RTW_MAT_METAL: i32 = 1;
pub const RTW_MAT_DIELECTRIC: i32 = 2;
pub const RTW_MAT_DIFFUSE_LIGHT: i32 = 3;
pub const RTW_MAT_ISOTROPIC: i32 = 4;
pub const RTW_TEX_SOLID: i32 = 0;
pub const RTW_TEX_CHECKER: i32 = 1;
pub const RTW_TEX_MARBLE: i32 = 2;
pub const RTW_TEX_IMAGE: i32 = 3;
pub const RTW_BG_SKY: i32 = 0;
pub const RTW_BG_SOLID: i32 = 1;
pub const RTW_MODE_DEFAULT: i32 = 0;
pub const RTW_MODE_NORMALS: i32 = 1;
pub const RTW_LEAF_VOLUME: u32 = 1;
pub const RTW_LEAF_TRANSFORM: u32 = 2;
pub const RTW_LEAF_ANIMATION: u32 = 4;
pub const RTW_LAYOUT_IMAGE: i32 = 0;
pub const RTW_PERLIN_MAX_POINTS: usize = 256;

// ---- flat World (include/rtw.h) --------------------------------------------------------------
#[repr(C)]
#[derive(Default, Clone, Copy)]
pub struct RtwBvhNode {
    pub min: [f32; 3],
    pub max: [f32; 3],
    pub axis: i32,
    pub left: i32,
    pub right: i32,
}

#[repr(C)]
#[derive(Default, Clone, Copy)]
pub struct RtwLeaf {
    pub geom_kind: i32,
    pub geom_index: i32,
    pub material: i32,
    pub flags: u32,
    pub neg_inv_density: f32,
    pub offset: [f32; 3],
    pub y_sin: f32,
    pub y_cos: f32,
    pub velocity: [f32; 3],
}

#[repr(C)]
#[derive(Default, Clone, Copy)]
pub struct RtwSphere {
    pub center: [f32; 3],
    pub radius: f32,
}

#[repr(C)]
#[derive(Default, Clone, Copy)]
pub struct RtwRect {
    pub plane: i32,
    pub dist: f32,
    pub r0: [f32; 2],
    pub r1: [f32; 2],
}

#[repr(C)]
#[derive(Default, Clone, Copy)]
pub struct RtwBox {
    pub min: [f32; 3],
    pub max: [f32; 3],
}

#[repr(C)]
#[derive(Default, Clone, Copy)]
pub struct RtwTriangle {
    pub positions: [[f32; 3]; 3],
    pub normals: [[f32; 3]; 3],
    pub uvs: [[f32; 2]; 3],
}

#[repr(C)]
#[derive(Default, Clone, Copy)]
pub struct RtwMaterial {
    pub kind: i32,
    pub texture: i32,
    pub fuzz: f32,
    pub index_of_refraction: f32,
}

#[repr(C)]
#[derive(Default, Clone, Copy)]
pub struct RtwTexture {
    pub kind: i32,
    pub color: [f32; 3],
    pub inv_frequency: f32,
    pub even: i32,
    pub odd: i32,
    pub scale: f32,
    pub perlin: i32,
    pub image: i32,
}

#[repr(C)]
#[derive(Clone, Copy)]
pub struct RtwImage {
    pub width: i32,
    pub height: i32,
    pub rgb: *const u8,
}

#[repr(C)]
#[derive(Clone, Copy)]
pub struct RtwPerlin {
    pub bits: i32,
    pub ranvec: [[f32; 3]; 256],
    pub perm_x: [u32; 256],
    pub perm_y: [u32; 256],
    pub perm_z: [u32; 256],
}

#[repr(C)]
#[derive(Default, Clone, Copy)]
pub struct RtwCamera {
    pub position: [f32; 3],
    pub upper_left_corner: [f32; 3],
    pub unit_right: [f32; 3],
    pub unit_up: [f32; 3],
    pub scaled_right: [f32; 3],
    pub scaled_up: [f32; 3],
    pub lens_radius: f32,
    pub time0: f32,
    pub time1: f32,
    pub shutter_pace: [f32; 2],
}

#[repr(C)]
#[derive(Default, Clone, Copy)]
pub struct RtwBackground {
    pub kind: i32,
    pub color: [f32; 3],
}

#[repr(C)]
pub struct RtwWorld {
    pub camera: RtwCamera,
    pub background: RtwBackground,
    pub has_light: i32,
    pub light: RtwRect,
    pub root: i32,
    pub node_count: i32,
    pub nodes: *const RtwBvhNode,
    pub leaf_count: i32,
    pub leaves: *const RtwLeaf,
    pub sphere_count: i32,
    pub spheres: *const RtwSphere,
    pub rect_count: i32,
    pub rects: *const RtwRect,
    pub box_count: i32,
    pub boxes: *const RtwBox,
    pub triangle_count: i32,
    pub triangles: *const RtwTriangle,
    pub material_count: i32,
    pub materials: *const RtwMaterial,
    pub texture_count: i32,
    pub textures: *const RtwTexture,
    pub image_count: i32,
    pub images: *const RtwImage,
    pub perlin_count: i32,
    pub perlins: *const RtwPerlin,
}

#[repr(C)]
#[derive(Default, Clone, Copy)]
pub struct RtwRenderParams {
    pub width: i32,
    pub height: i32,
    pub samples_per_pixel: u32,
    pub max_depth: i32,
    pub render_mode: i32,
    pub layout: i32,
    pub seed: u64,
    pub tile_width: i32,
    pub tile_height: i32,
    pub part_index: i32,
    pub part_count: i32,
    pub thread_count: i32,
    pub reserved0: i32,
}

pub type RtwProgressFn = extern "C" fn(done_samples: u64, total_samples: u64, user: *mut c_void);

#[link(name = "rtw")]
extern "C" {
    pub fn rtw_version() -> c_int;
    pub fn rtw_last_error() -> *const c_char;
    pub fn rtw_render(world: *const RtwWorld, params: *const RtwRenderParams, device: c_int, out_rgb: *mut f32) -> c_int;
    pub fn rtw_render_progress(world: *const RtwWorld, params: *const RtwRenderParams, device: c_int, out_rgb: *mut f32,
                               cb: Option<RtwProgressFn>, user: *mut c_void) -> c_int;
    pub fn rtw_render_devices(world: *const RtwWorld, params: *const RtwRenderParams, devices: *const c_int,
                              n_devices: c_int, out_rgb: *mut f32) -> c_int;
    pub fn rtw_device_count(count: *mut c_int) -> c_int;
}

fn check(rc: c_int, what: &str) {
    if rc != RTW_OK {
        let msg = unsafe { CStr::from_ptr(rtw_last_error()) }.to_string_lossy().into_owned();
        panic!("{what} failed ({rc}): {msg}");
    }
}

fn xyz(v: Vec3<f32>) -> [f32; 3] {
    v.e
}

// ---- serialiser ------------------------------------------------------------------------------
/// The flat tables of one World.  Materials, textures, images and Perlin tables are shared by
/// reference in the reference's arena; they are deduplicated by address, so each becomes one
/// table entry however many leaves use it (the device indexes them).
#[derive(Default)]
struct Flat {
    nodes: Vec<RtwBvhNode>,
    leaves: Vec<RtwLeaf>,
    spheres: Vec<RtwSphere>,
    rects: Vec<RtwRect>,
    boxes: Vec<RtwBox>,
    triangles: Vec<RtwTriangle>,
    materials: Vec<RtwMaterial>,
    textures: Vec<RtwTexture>,
    images: Vec<RtwImage>,
    perlins: Vec<RtwPerlin>,
    mat_ids: HashMap<usize, i32>,
    tex_ids: HashMap<usize, i32>,
    img_ids: HashMap<usize, i32>,
    perlin_ids: HashMap<usize, i32>,
}

fn rect(r: &RectGeometry) -> RtwRect {
    // rect_geometry.rs:8-30: (p0, p1, n) axes Xy (0,1,2), Xz (0,2,1), Yz (1,2,0)
    let plane = match r.rect_plane {
        RectPlane::Xy => RTW_PLANE_XY,
        RectPlane::Xz => RTW_PLANE_XZ,
        RectPlane::Yz => RTW_PLANE_YZ,
    };
    RtwRect { plane, dist: r.dist, r0: [r.r0.0, r.r0.1], r1: [r.r1.0, r.r1.1] }
}

impl Flat {
    /// image::RgbImage (world_builder.rs:19-31): 8-bit RGB, row 0 = top; the pixels stay in the
    /// caller's image (`rgb` borrows them for the duration of the render call).
    fn image(&mut self, img: &image::RgbImage) -> i32 {
        let key = img as *const _ as usize;
        if let Some(&id) = self.img_ids.get(&key) {
            return id;
        }
        let id = self.images.len() as i32;
        self.images.push(RtwImage { width: img.width() as i32, height: img.height() as i32, rgb: img.as_raw().as_ptr() });
        self.img_ids.insert(key, id);
        id
    }

    /// Perlin (perlin.rs:10-16): 2^bits random unit vectors and three permutations.
    fn perlin(&mut self, p: &Perlin) -> i32 {
        let key = p as *const _ as usize;
        if let Some(&id) = self.perlin_ids.get(&key) {
            return id;
        }
        let n = 1usize << p.bits;
        assert!(p.bits >= 1 && n <= RTW_PERLIN_MAX_POINTS, "render_gpu: Perlin bits must be 1..=8");
        let mut t = RtwPerlin {
            bits: p.bits as i32,
            ranvec: [[0.0; 3]; 256],
            perm_x: [0; 256],
            perm_y: [0; 256],
            perm_z: [0; 256],
        };
        for i in 0..n {
            t.ranvec[i] = xyz(p.ranvec[i].0);
            t.perm_x[i] = p.perm_x[i];
            t.perm_y[i] = p.perm_y[i];
            t.perm_z[i] = p.perm_z[i];
        }
        let id = self.perlins.len() as i32;
        self.perlins.push(t);
        self.perlin_ids.insert(key, id);
        id
    }

    /// Texture (texture.rs:3-20).  A Checker's even / odd children are serialised first (the
    /// reference graph is built bottom-up in the arena, so it has no cycles).
    fn texture(&mut self, t: &Texture) -> i32 {
        let key = t as *const _ as usize;
        if let Some(&id) = self.tex_ids.get(&key) {
            return id;
        }
        let mut r = RtwTexture { even: -1, odd: -1, perlin: -1, image: -1, ..Default::default() };
        match t {
            Texture::Solid { color } => {
                r.kind = RTW_TEX_SOLID;
                r.color = xyz(color.0);
            }
            Texture::Checker { inv_frequency, even, odd } => {
                r.kind = RTW_TEX_CHECKER;
                r.inv_frequency = *inv_frequency;
                r.even = self.texture(even);
                r.odd = self.texture(odd);
            }
            Texture::Marble { scale, noise } => {
                r.kind = RTW_TEX_MARBLE;
                r.scale = *scale;
                r.perlin = self.perlin(noise);
            }
            Texture::Image { image } => {
                r.kind = RTW_TEX_IMAGE;
                r.image = self.image(image);
            }
        }
        let id = self.textures.len() as i32;
        self.textures.push(r);
        self.tex_ids.insert(key, id);
        id
    }

    /// Material (material.rs:43-49).
    fn material(&mut self, m: &Material) -> i32 {
        let key = m as *const _ as usize;
        if let Some(&id) = self.mat_ids.get(&key) {
            return id;
        }
        let r = match *m {
            Material::Lambert { albedo } => {
                RtwMaterial { kind: RTW_MAT_LAMBERT, texture: self.texture(albedo), ..Default::default() }
            }
            Material::Metal { albedo, fuzz } => {
                RtwMaterial { kind: RTW_MAT_METAL, texture: self.texture(albedo), fuzz, ..Default::default() }
            }
            Material::Dielectric { index_of_refraction } => {
                RtwMaterial { kind: RTW_MAT_DIELECTRIC, texture: -1, fuzz: 0.0, index_of_refraction }
            }
            Material::DiffuseLight { emit } => {
                RtwMaterial { kind: RTW_MAT_DIFFUSE_LIGHT, texture: self.texture(emit), ..Default::default() }
            }
            Material::Isotropic { albedo } => {
                RtwMaterial { kind: RTW_MAT_ISOTROPIC, texture: self.texture(albedo), ..Default::default() }
            }
        };
        let id = self.materials.len() as i32;
        self.materials.push(r);
        self.mat_ids.insert(key, id);
        id
    }

    /// Geometry (hittable.rs:104-110) -> (RTW_GEOM_*, index into that kind's table).
    fn geometry(&mut self, g: &Geometry) -> (i32, i32) {
        match g {
            Geometry::Sphere(s) => {
                self.spheres.push(RtwSphere { center: xyz(s.center.0), radius: s.radius });
                (RTW_GEOM_SPHERE, self.spheres.len() as i32 - 1)
            }
            Geometry::Rect(r) => {
                self.rects.push(rect(r));
                (RTW_GEOM_RECT, self.rects.len() as i32 - 1)
            }
            Geometry::AxisAlignedBox(b) => {
                self.boxes.push(RtwBox { min: xyz(b.min.0), max: xyz(b.max.0) });
                (RTW_GEOM_BOX, self.boxes.len() as i32 - 1)
            }
            Geometry::Triangle(t) => {
                let mut r = RtwTriangle::default();
                for k in 0..3 {
                    r.positions[k] = xyz(t.positions[k].0);
                    r.normals[k] = xyz(t.normals[k].0);
                    r.uvs[k] = [t.texture_coords[k].x, t.texture_coords[k].y];
                }
                self.triangles.push(r);
                (RTW_GEOM_TRIANGLE, self.triangles.len() as i32 - 1)
            }
        }
    }

    /// One BVH item as finish_internal builds it (world_builder.rs:305-316):
    ///   [Animation(velocity)] ( [Transformation] ( SurfaceGeometry | VolumeGeometry ) )
    fn leaf(&mut self, e: &SceneElement) -> i32 {
        let mut l = RtwLeaf { y_cos: 1.0, ..Default::default() };
        let mut e = e;
        if let SceneElement::Animation(inner, velocity) = e {
            l.flags |= RTW_LEAF_ANIMATION;
            l.velocity = xyz(velocity.0);
            e = *inner;
        }
        if let SceneElement::Transformation(inner, t) = e {
            l.flags |= RTW_LEAF_TRANSFORM;
            l.offset = xyz(t.offset.0);
            l.y_sin = t.y_sine;
            l.y_cos = t.y_cosine;
            e = *inner;
        }
        match e {
            SceneElement::SurfaceGeometry(g, m) => {
                let (kind, index) = self.geometry(g);
                l.geom_kind = kind;
                l.geom_index = index;
                l.material = self.material(m);
            }
            SceneElement::VolumeGeometry(v) => {
                let (kind, index) = self.geometry(&v.boundary);
                l.flags |= RTW_LEAF_VOLUME;
                l.geom_kind = kind;
                l.geom_index = index;
                l.material = self.material(v.phase_function);
                l.neg_inv_density = v.neg_inv_density;
            }
            _ => panic!("render_gpu: a BVH item is not a leaf as WorldBuilder::finish builds it (world_builder.rs:305-316)"),
        }
        self.leaves.push(l);
        self.leaves.len() as i32 - 1
    }

    /// BoundingVolumeHierarchy (hittable.rs:352-357): nodes keep their indices; a child id
    /// `usize::MAX - i` (hittable.rs:363-366, :438) is leaf i, encoded -1 - i.
    fn bvh(&mut self, b: &BoundingVolumeHierarchy) -> i32 {
        assert!(b.unbounded_items.is_empty(), "render_gpu: unbounded BVH items are not supported");
        for it in &b.items {
            self.leaf(it);
        }
        let n_items = b.items.len();
        let enc = |id: usize| -> i32 {
            if id > n_items {
                -1 - (usize::MAX - id) as i32
            } else {
                id as i32
            }
        };
        for n in &b.nodes {
            self.nodes.push(RtwBvhNode {
                min: xyz(n.aabb.min.0),
                max: xyz(n.aabb.max.0),
                axis: n.axis_id as i32,
                left: enc(n.left),
                right: enc(n.right),
            });
        }
        enc(b.initial_index)
    }
}

/// rendering::World -> rtw_world.  The returned tables own (or borrow from `world`) every array
/// the pointers in `RtwWorld` point to; keep them alive across the call.
fn serialise(world: &World) -> (Flat, RtwWorld) {
    let mut f = Flat::default();
    let root = match world.hittable.root {
        SceneElement::BoundingVolumeHierarchy(b) => f.bvh(b),
        e => -1 - f.leaf(e), // a one-leaf scene
    };
    let c = &world.camera;
    let camera = RtwCamera {
        position: xyz(c.position.0),
        upper_left_corner: xyz(c.upper_left_corner.0),
        unit_right: xyz(c.unit_right.0),
        unit_up: xyz(c.unit_up.0),
        scaled_right: xyz(c.scaled_right.0),
        scaled_up: xyz(c.scaled_up.0),
        lens_radius: c.lens_radius,
        time0: c.time_interval.start,
        time1: c.time_interval.end,
        shutter_pace: [c.shutter_pace.x, c.shutter_pace.y],
    };
    // world_scattering_distribution.rs:4-9: the POI rect finish_internal picked (world_builder.rs:317-319)
    let (has_light, light) = match &world.scattering_distribution_provider {
        Some(WorldScatteringDistributionProvider::Rect(r)) => (1, rect(r)),
        None => (0, RtwRect::default()),
    };
    let background = match world.background {
        BackgroundColor::Sky => RtwBackground { kind: RTW_BG_SKY, color: [0.0; 3] },
        BackgroundColor::Solid { color } => RtwBackground { kind: RTW_BG_SOLID, color: xyz(color.0) },
    };
    let w = RtwWorld {
        camera,
        background,
        has_light,
        light,
        root,
        node_count: f.nodes.len() as i32,
        nodes: f.nodes.as_ptr(),
        leaf_count: f.leaves.len() as i32,
        leaves: f.leaves.as_ptr(),
        sphere_count: f.spheres.len() as i32,
        spheres: f.spheres.as_ptr(),
        rect_count: f.rects.len() as i32,
        rects: f.rects.as_ptr(),
        box_count: f.boxes.len() as i32,
        boxes: f.boxes.as_ptr(),
        triangle_count: f.triangles.len() as i32,
        triangles: f.triangles.as_ptr(),
        material_count: f.materials.len() as i32,
        materials: f.materials.as_ptr(),
        texture_count: f.textures.len() as i32,
        textures: f.textures.as_ptr(),
        image_count: f.images.len() as i32,
        images: f.images.as_ptr(),
        perlin_count: f.perlins.len() as i32,
        perlins: f.perlins.as_ptr(),
    };
    (f, w)
}

extern "C" fn print_percent(done: u64, total: u64, _user: *mut c_void) {
    // rendering.rs:149-153: "\r{done_percent} %"
    eprint!("\r{} %", 100 * done / total.max(1));
}

/// rendering::render on the MI355X, argument for argument (rendering.rs:121-128).  The samples
/// of each pixel are split into `thread_count` planes and merged exactly as split_work_tasks /
/// merge_planes do (rendering.rs:222-252); the reference seeds from entropy
/// (rendering.rs:160), and so does this (`render_gpu_seeded` takes an explicit seed and device).
pub fn render_gpu(image_size: Size2i, thread_count: usize, samples_per_pixel: usize, max_depth: i32, world: &World,
                  render_mode: RenderMode) -> Vec<Color> {
    let seed: u64 = rand::random();
    render_gpu_seeded(image_size, thread_count, samples_per_pixel, max_depth, world, render_mode, seed, 0)
}

fn params(image_size: Size2i, thread_count: usize, samples_per_pixel: usize, max_depth: i32, render_mode: RenderMode,
          seed: u64) -> RtwRenderParams {
    assert_eq!(unsafe { rtw_version() }, RTW_ABI_VERSION, "librtw.so ABI version mismatch");
    assert!(thread_count >= 1, "attempt to divide by zero"); // split_work_tasks (rendering.rs:223)
    RtwRenderParams {
        width: image_size.width,
        height: image_size.height,
        samples_per_pixel: u32::try_from(samples_per_pixel).expect("samples_per_pixel exceeds u32::MAX"),
        max_depth,
        render_mode: match render_mode {
            RenderMode::Default => RTW_MODE_DEFAULT,
            RenderMode::Normals => RTW_MODE_NORMALS,
        },
        layout: RTW_LAYOUT_IMAGE,
        seed,
        tile_width: 0,
        tile_height: 0,
        part_index: 0,
        part_count: 1,
        thread_count: thread_count.min(i32::MAX as usize) as i32,
        reserved0: 0,
    }
}

fn colors(out: Vec<f32>) -> Vec<Color> {
    out.chunks_exact(3).map(|c| Color::new_rgb(c[0], c[1], c[2])).collect()
}

pub fn render_gpu_seeded(image_size: Size2i, thread_count: usize, samples_per_pixel: usize, max_depth: i32,
                         world: &World, render_mode: RenderMode, seed: u64, device: i32) -> Vec<Color> {
    let p = params(image_size, thread_count, samples_per_pixel, max_depth, render_mode, seed);
    let (f, w) = serialise(world);
    let n = (image_size.width as usize) * (image_size.height as usize);
    let mut out = vec![0f32; n * 3];
    eprintln!("Start rendering...");
    let start = std::time::Instant::now();
    let rc = unsafe { rtw_render_progress(&w, &p, device, out.as_mut_ptr(), Some(print_percent), std::ptr::null_mut()) };
    check(rc, "rtw_render_progress");
    eprintln!("\rRendering done in {} seconds", start.elapsed().as_secs_f64());
    drop(f);
    colors(out)
}

/// rendering::render on every GPU of the node (the reference's `render` uses every core,
/// main.rs:19): the interleaved tiles are split over `devices`, rendered in parallel, gathered on
/// devices[0] over xGMI (rtw_render_devices).  Bit-identical to `render_gpu_seeded` with the same
/// seed for every device list.  An empty list means all devices.
pub fn render_gpu_devices(image_size: Size2i, thread_count: usize, samples_per_pixel: usize, max_depth: i32,
                          world: &World, render_mode: RenderMode, seed: u64, devices: &[i32]) -> Vec<Color> {
    let p = params(image_size, thread_count, samples_per_pixel, max_depth, render_mode, seed);
    let all: Vec<c_int> = if devices.is_empty() {
        let mut n: c_int = 0;
        check(unsafe { rtw_device_count(&mut n) }, "rtw_device_count");
        (0..n.max(1)).collect()
    } else {
        devices.iter().map(|&d| d as c_int).collect()
    };
    let (f, w) = serialise(world);
    let n = (image_size.width as usize) * (image_size.height as usize);
    let mut out = vec![0f32; n * 3];
    eprintln!("Start rendering on {} GPU(s)...", all.len());
    let start = std::time::Instant::now();
    let rc = unsafe { rtw_render_devices(&w, &p, all.as_ptr(), all.len() as c_int, out.as_mut_ptr()) };
    check(rc, "rtw_render_devices");
    eprintln!("Rendering done in {} seconds", start.elapsed().as_secs_f64());
    drop(f);
    colors(out)
}
