"""The reference-side Rust binding (integration/rust/gpu.rs) against the C ABI (include/rtw.h).

rustc is not in this image, so the shim cannot be compiled here; what can be enforced is that its
`#[repr(C)]` structs are the header's structs: the same fields in the same order with the same
types, and -- through the C compiler -- the same offsets and sizes (repr(C) follows the C layout
rules, computed here for the Rust declarations).  Also the shared constants and the extern
function names / parameter counts."""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rtw.h")
SHIM = os.path.join(ROOT, "integration", "rust", "gpu.rs")

C_SCALARS = {"int32_t": "i32", "uint32_t": "u32", "float": "f32", "uint64_t": "u64", "uint8_t": "u8", "int": "c_int"}
SIZES = {"i32": 4, "u32": 4, "f32": 4, "u64": 8, "u8": 1, "c_int": 4}


def rust_structs(text: str) -> dict:
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*(?:#\[derive\([^)]*\)\]\s*)?pub struct (\w+) \{(.*?)\n\}", text, re.S):
        fields = re.findall(r"pub (\w+): ([^,]+),", m.group(2))
        out[m.group(1)] = [(n, t.strip()) for n, t in fields]
    return out


def c_structs(text: str) -> dict:
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for m in re.finditer(r"typedef struct (\w+) \{(.*?)\} (\w+);", text, re.S):
        fields = []
        for decl in m.group(2).split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            dm = re.match(r"((?:const )?\w+\s*\*?)\s*(.*)", decl)
            base = dm.group(1).replace(" ", "")
            for name in dm.group(2).split(","):
                name = name.strip()
                star = name.startswith("*")
                nm = re.match(r"\*?(\w+)((?:\[\w+\])*)", name)
                dims = re.findall(r"\[(\w+)\]", nm.group(2))
                fields.append((nm.group(1), base + ("*" if star else ""), dims))
        out[m.group(3)] = fields
    return out


def snake(name: str) -> str:
    return re.sub(r"(?<!^)(?=[A-Z])", "_", name).lower()


def c_to_rust_type(base: str, dims: list, c_defs: dict) -> str:
    const = base.startswith("const")
    ptr = base.endswith("*")
    core = base.replace("const", "").rstrip("*")
    if core in C_SCALARS:
        t = C_SCALARS[core]
    else:  # a struct typedef: rtw_bvh_node -> RtwBvhNode
        t = "".join(p.capitalize() for p in core.split("_"))
    if ptr:
        t = ("*const " if const else "*mut ") + t
    for d in reversed(dims):
        t = f"[{t}; {c_defs.get(d, d)}]"
    return t


def rust_layout(structs: dict, name: str) -> tuple[int, int, list]:
    """(size, align, [(field, offset)]) of a repr(C) Rust struct."""

    def size_align(t: str):
        t = t.strip()
        if t.startswith("*"):
            return 8, 8
        m = re.match(r"\[(.*); (\w+)\]$", t)
        if m:
            s, a = size_align(m.group(1))
            return s * int(m.group(2)), a
        if t in SIZES:
            return SIZES[t], SIZES[t]
        s, a, _ = rust_layout(structs, t)
        return s, a

    off, align, offs = 0, 1, []
    for f, t in structs[name]:
        s, a = size_align(t)
        off = (off + a - 1) // a * a
        offs.append((f, off))
        off += s
        align = max(align, a)
    return (off + align - 1) // align * align, align, offs


@pytest.fixture(scope="module")
def parsed():
    return rust_structs(open(SHIM).read()), c_structs(open(HEADER).read()), open(HEADER).read(), open(SHIM).read()


def c_defines(header: str) -> dict:
    return {k: v.rstrip("u") for k, v in re.findall(r"#define (RTW_\w+) (\d+u?)\b", header)}


def test_every_header_struct_has_a_rust_mirror(parsed):
    rs, cs, header, _ = parsed
    flat = ["rtw_bvh_node", "rtw_leaf", "rtw_sphere", "rtw_rect", "rtw_box", "rtw_triangle", "rtw_material", "rtw_texture",
            "rtw_image", "rtw_perlin", "rtw_camera", "rtw_background", "rtw_world", "rtw_render_params"]
    for c in flat:
        assert c in cs, c
        assert "".join(p.capitalize() for p in c.split("_")) in rs, c


def test_fields_and_types_match_header(parsed):
    rs, cs, header, _ = parsed
    defs = c_defines(header)
    for rname, rfields in rs.items():
        cname = snake(rname)
        assert cname in cs, cname
        cf = cs[cname]
        assert [f for f, _ in rfields] == [f for f, _, _ in cf], f"{rname}: field order"
        for (f, rt), (_, base, dims) in zip(rfields, cf):
            assert rt == c_to_rust_type(base, dims, defs), f"{rname}.{f}: {rt} vs {base}{dims}"


def test_offsets_and_sizes_match_the_c_compiler(parsed):
    rs, _, _, _ = parsed
    lines = []
    for rname, fields in rs.items():
        c = snake(rname)
        lines.append(f'printf("{rname} size %zu align %zu\\n", sizeof({c}), _Alignof({c}));')
        for f, _ in fields:
            lines.append(f'printf("{rname}.{f} %zu\\n", offsetof({c}, {f}));')
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"rtw.h\"\nint main(void){\n" + "\n".join(lines) + "\nreturn 0;}\n"
    with tempfile.TemporaryDirectory() as d:
        cpath, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(cpath, "w").write(src)
        subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), cpath, "-o", exe], check=True)
        got = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.splitlines()
    c_layout = {}
    for line in got:
        parts = line.split()
        if parts[1] == "size":
            c_layout[parts[0]] = (int(parts[2]), int(parts[4]))
        else:
            c_layout[parts[0]] = int(parts[1])
    for rname in rs:
        size, align, offs = rust_layout(rs, rname)
        assert (size, align) == c_layout[rname], f"{rname}: rust {size}/{align} vs C {c_layout[rname]}"
        for f, o in offs:
            assert o == c_layout[f"{rname}.{f}"], f"{rname}.{f}: rust offset {o} vs C {c_layout[f'{rname}.{f}']}"


def test_constants_match_header(parsed):
    _, _, header, shim = parsed
    defs = c_defines(header)
    consts = re.findall(r"pub const (RTW_\w+): \w+ = (\d+);", shim)
    assert len(consts) >= 25
    for name, val in consts:
        assert name in defs, name
        assert defs[name] == val, f"{name}: {val} vs {defs[name]}"


def test_extern_functions_exist_with_parameter_counts(parsed):
    _, _, header, shim = parsed
    block = re.search(r'extern "C" \{(.*?)\n\}', shim, re.S).group(1)
    fns = re.findall(r"pub fn (rtw_\w+)\((.*?)\)", block, re.S)
    assert {f for f, _ in fns} >= {"rtw_render", "rtw_render_progress", "rtw_last_error", "rtw_version"}
    for name, params in fns:
        m = re.search(r"RTW_API [^;(]*\b" + name + r"\((.*?)\);", header, re.S)
        assert m, name
        c_params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        r_params = [p for p in params.split(",") if p.strip()]
        assert len(c_params) == len(r_params), name


def test_shim_is_complete(parsed):
    """No unimplemented!() / todo!() left: every Texture, Material, Geometry and SceneElement leaf
    form the world builder produces is serialised (texture.rs:3-20, material.rs:43-49,
    hittable.rs:104-119, world_builder.rs:305-316) and the POI light rect too."""
    _, _, _, shim = parsed
    code = re.sub(r"//.*", "", shim)
    assert "unimplemented!" not in code and "todo!" not in code
    for variant in ["Texture::Solid", "Texture::Checker", "Texture::Marble", "Texture::Image", "Material::Lambert",
                    "Material::Metal", "Material::Dielectric", "Material::DiffuseLight", "Material::Isotropic",
                    "Geometry::Sphere", "Geometry::Rect", "Geometry::AxisAlignedBox", "Geometry::Triangle",
                    "SceneElement::Animation", "SceneElement::Transformation", "SceneElement::SurfaceGeometry",
                    "SceneElement::VolumeGeometry", "SceneElement::BoundingVolumeHierarchy",
                    "WorldScatteringDistributionProvider::Rect", "BackgroundColor::Sky", "BackgroundColor::Solid"]:
        assert variant in code, variant
    assert "pub fn render_gpu(image_size: Size2i, thread_count: usize, samples_per_pixel: usize, max_depth: i32, world: &World," in code
