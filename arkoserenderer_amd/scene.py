"""Scene inputs for the DDGI path: the RT-scene data contract of GpuScene
(RT mesh table, u32 index pool, vec3 position pool, RTVertex pool, materials,
TLAS instances, lights, environment) as numpy arrays, plus loaders:

* ``load_gltf`` — glTF 2.0 (+ .bin, images) reader following the reference's
  import rules (arkcore/asset/import/GltfLoader.cpp:372-543 geometry,
  :817-1035 samplers and materials, GpuScene.cpp:1452-1580 texture formats) for
  the in-tree sample models (Cornell box, DamagedHelmet); ``merge_scenes`` puts
  several into one scene (level objects, arkoserenderer_amd/level.py).
* ``cornell_box`` — BASELINE config C2 (CornellBox.arklvl: +90 deg about X,
  camera f/11 1/125 s ISO 400, no lights, environment = white x brightness).
* ``soup`` — BASELINE config C4 synthetic triangle-strip soup (C generator in
  libark_ddgi, include/ark_scene.h).
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os
from dataclasses import dataclass, field

import numpy as np

from . import abi


def shader_material_dtype():
    return np.dtype([
        ("base_color", "<i4"), ("normal_map", "<i4"), ("metallic_roughness", "<i4"), ("emissive", "<i4"),
        ("occlusion", "<i4"), ("bent_normal_map", "<i4"), ("clearcoat", "<f4"), ("clearcoat_roughness", "<f4"),
        ("blend_mode", "<i4"), ("mask_cutoff", "<f4"), ("metallic_factor", "<f4"), ("roughness_factor", "<f4"),
        ("emissive_factor", "<f4", 3), ("brdf", "<i4"), ("dielectric_reflectance", "<f4"), ("_unused", "<f4", 3),
        ("color_tint", "<f4", 4),
    ])


MATERIAL_DTYPE = shader_material_dtype()
MESH_DTYPE = np.dtype([("first_vertex", "<i4"), ("first_index", "<i4"), ("material_index", "<i4")])
INSTANCE_DTYPE = np.dtype([("object_to_world", "<f4", 12), ("rt_mesh_index", "<u4"), ("triangle_count", "<u4"),
                           ("hit_mask", "<u4"), ("_pad", "<u4")])
VERTEX_DTYPE = np.dtype([("tex_coord", "<f4", 2), ("normal", "<f4", 3), ("tangent", "<f4", 4)])


def default_material() -> np.ndarray:
    m = np.zeros((), dtype=MATERIAL_DTYPE)
    for k in ("base_color", "normal_map", "metallic_roughness", "emissive", "occlusion", "bent_normal_map"):
        m[k] = -1  # -> default textures (white; GpuScene.cpp:1459-1464)
    m["blend_mode"] = abi.ARK_BLEND_MODE_OPAQUE
    m["mask_cutoff"] = 1.0
    m["metallic_factor"] = 1.0
    m["roughness_factor"] = 1.0
    # MaterialAsset::calculateDielectricReflectance at the default IOR 1.5 (the shaders
    # use the DIELECTRIC_REFLECTANCE constant instead, brdf.glsl:6)
    q = (np.float32(1.5) - np.float32(1.0)) / (np.float32(1.5) + np.float32(1.0))
    m["dielectric_reflectance"] = q * q
    m["color_tint"] = (1.0, 1.0, 1.0, 1.0)
    return m


@dataclass
class Texture:
    width: int
    height: int
    format: int
    data: np.ndarray
    wrap: int = abi.ARK_WRAP_REPEAT


@dataclass
class SpotLight:
    color: tuple
    direction: tuple
    right: tuple
    up: tuple
    position: tuple
    outer_cone_half_angle: float
    ies_profile_index: int = -1


def spot_array(spots) -> C.Array:
    """ArkSpotLight[] of SpotLights (SpotLightData, GpuScene.cpp:844-858)."""
    arr = (abi.ArkSpotLight * max(1, len(spots)))()
    for i, sl in enumerate(spots):
        for k in range(3):
            arr[i].color[k] = sl.color[k]
            arr[i].world_space_direction[k] = sl.direction[k]
            arr[i].world_space_right[k] = sl.right[k]
            arr[i].world_space_up[k] = sl.up[k]
            arr[i].world_space_position[k] = sl.position[k]
        arr[i].outer_cone_half_angle = sl.outer_cone_half_angle
        arr[i].ies_profile_index = sl.ies_profile_index
    return arr


def lights_abi(sun, spots) -> tuple:
    """ArkDdgiLights for ark_ddgi_set_lights: sun = (colour, direction) pre-exposed or
    None, spots = SpotLights. Returns (struct, keep-alive array)."""
    L = abi.ArkDdgiLights()
    L.struct_size = C.sizeof(abi.ArkDdgiLights)
    if sun is not None:
        L.has_directional_light = 1
        for k in range(3):
            L.directional_light.color[k] = sun[0][k]
            L.directional_light.world_space_direction[k] = sun[1][k]
    arr = spot_array(list(spots))
    L.spot_lights = C.addressof(arr)
    L.spot_light_count = len(spots)
    return L, arr


@dataclass
class SceneData:
    positions: np.ndarray            # (V, 3) float32
    vertices: np.ndarray             # (V,) VERTEX_DTYPE
    indices: np.ndarray              # (I,) uint32, local to mesh first_vertex
    meshes: np.ndarray               # (M,) MESH_DTYPE
    materials: np.ndarray            # (Mat,) MATERIAL_DTYPE
    instances: np.ndarray            # (Inst,) INSTANCE_DTYPE
    textures: list = field(default_factory=list)
    sun: tuple | None = None         # (color(3), direction(3)), color pre-exposed
    spots: list = field(default_factory=list)
    environment_texture: int = -1
    _keepalive: list = field(default_factory=list, repr=False)
    _native: object = field(default=None, repr=False)  # owning ArkSoupScene handle

    @property
    def triangle_count(self) -> int:
        return int(self.instances["triangle_count"].sum())

    def to_abi(self) -> abi.ArkDdgiScene:
        """Builds the ArkDdgiScene view. The returned struct references this
        object's arrays; keep the SceneData alive while it is used."""
        s = abi.ArkDdgiScene()
        s.struct_size = C.sizeof(abi.ArkDdgiScene)
        keep = []

        def ptr(a):
            a = np.ascontiguousarray(a)
            keep.append(a)
            return a.ctypes.data

        s.indices = ptr(self.indices.astype(np.uint32, copy=False))
        s.index_count = int(self.indices.size)
        s.positions = ptr(self.positions.astype(np.float32, copy=False))
        s.vertex_count = int(self.positions.shape[0])
        s.vertices = ptr(self.vertices)
        s.meshes = ptr(self.meshes)
        s.mesh_count = int(self.meshes.size)
        s.materials = ptr(self.materials)
        s.material_count = int(self.materials.size)
        tex = (abi.ArkTexture * max(1, len(self.textures)))()
        for i, t in enumerate(self.textures):
            tex[i].width, tex[i].height, tex[i].format, tex[i].wrap = t.width, t.height, t.format, t.wrap
            tex[i].data = ptr(t.data)
        keep.append(tex)
        s.textures = C.addressof(tex)
        s.texture_count = len(self.textures)
        s.instances = ptr(self.instances)
        s.instance_count = int(self.instances.size)
        if self.sun is not None:
            s.has_directional_light = 1
            for k in range(3):
                s.directional_light.color[k] = self.sun[0][k]
                s.directional_light.world_space_direction[k] = self.sun[1][k]
        spots = spot_array(self.spots)
        keep.append(spots)
        s.spot_lights = C.addressof(spots)
        s.spot_light_count = len(self.spots)
        s.environment_texture = self.environment_texture
        self._keepalive = keep
        return s

    def save_binary(self, path: str):
        """Writes the ARKSCN1 container read by the C++ headless driver
        (arkoserenderer_amd/host/apps/ddgi_headless.cpp)."""
        import struct

        with open(path, "wb") as fh:
            fh.write(b"ARKSCN1\0")
            fh.write(struct.pack("<7Q", self.indices.size, self.positions.shape[0], self.meshes.size, self.materials.size,
                                 self.instances.size, len(self.textures), len(self.spots)))
            sun = self.sun if self.sun is not None else ((0, 0, 0), (0, 0, 0))
            fh.write(struct.pack("<i6fi", 1 if self.sun is not None else 0, *sun[0], *sun[1], self.environment_texture))
            fh.write(np.ascontiguousarray(self.indices, np.uint32).tobytes())
            fh.write(np.ascontiguousarray(self.positions, np.float32).tobytes())
            for a in (self.vertices, self.meshes, self.materials, self.instances):
                fh.write(np.ascontiguousarray(a).tobytes())
            for sl in self.spots:
                sp = abi.ArkSpotLight()
                for k in range(3):
                    sp.color[k], sp.world_space_direction[k] = sl.color[k], sl.direction[k]
                    sp.world_space_right[k], sp.world_space_up[k], sp.world_space_position[k] = sl.right[k], sl.up[k], sl.position[k]
                sp.outer_cone_half_angle, sp.ies_profile_index = sl.outer_cone_half_angle, sl.ies_profile_index
                fh.write(bytes(sp))
            for t in self.textures:
                fh.write(struct.pack("<4i", t.width, t.height, t.format, t.wrap))
                fh.write(np.ascontiguousarray(t.data).tobytes())

    def bounds(self):
        lo = np.full(3, np.inf, np.float32)
        hi = np.full(3, -np.inf, np.float32)
        for inst in self.instances:
            mesh = self.meshes[inst["rt_mesh_index"]]
            idx = self.indices[mesh["first_index"]: mesh["first_index"] + 3 * inst["triangle_count"]]
            p = self.positions[mesh["first_vertex"] + idx.astype(np.int64)]
            M = inst["object_to_world"].reshape(3, 4)
            w = p @ M[:, :3].T + M[:, 3]
            lo = np.minimum(lo, w.min(0))
            hi = np.maximum(hi, w.max(0))
        return lo, hi


def quat_to_matrix(x, y, z, w) -> np.ndarray:
    """Rotation matrix (3x3, float32) of a unit quaternion (x, y, z, w)."""
    m = np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ], dtype=np.float64)
    return m.astype(np.float32)


_COMPONENT = {5120: np.int8, 5121: np.uint8, 5122: np.int16, 5123: np.uint16, 5125: np.uint32, 5126: np.float32}
_NCOMP = {"SCALAR": 1, "VEC2": 2, "VEC3": 3, "VEC4": 4, "MAT4": 16}


def _accessor(g, buffers, idx):
    acc = g["accessors"][idx]
    view = g["bufferViews"][acc["bufferView"]]
    dt = np.dtype(_COMPONENT[acc["componentType"]])
    n = _NCOMP[acc["type"]]
    offset = view.get("byteOffset", 0) + acc.get("byteOffset", 0)
    stride = view.get("byteStride", 0) or dt.itemsize * n
    buf = buffers[view["buffer"]]
    count = acc["count"]
    if stride == dt.itemsize * n:
        arr = np.frombuffer(buf, dtype=dt, count=count * n, offset=offset).reshape(count, n)
    else:
        arr = np.stack([np.frombuffer(buf, dtype=dt, count=n, offset=offset + i * stride) for i in range(count)])
    return arr


# glTF sampler wrap -> ImageWrapMode (GltfLoader.cpp:836-849)
_GLTF_WRAP = {10497: abi.ARK_WRAP_REPEAT, 33071: abi.ARK_WRAP_CLAMP_TO_EDGE, 33648: abi.ARK_WRAP_MIRRORED_REPEAT}


def _texture_wrap(g, tex_index: int) -> int:
    """Wrap of glTF texture `tex_index`: its sampler's wrapS / wrapT; no sampler means
    repeat in both directions (GltfLoader.cpp:826-832, glTF 2.0 defaults)."""
    t = g["textures"][tex_index]
    smp = g["samplers"][t["sampler"]] if t.get("sampler", -1) >= 0 else {}
    ws = _GLTF_WRAP[smp.get("wrapS", 10497)]
    wt = _GLTF_WRAP[smp.get("wrapT", 10497)]
    return ws if ws == wt else abi.ark_wrap_axes(ws, wt)


def _decode_image(g, base: str, buffers, image_index: int) -> np.ndarray:
    """RGBA8 pixels (H, W, 4) of glTF image `image_index`, from its uri or buffer view.
    PIL decodes (the reference's ImageAsset uses its own decoder: the texel values of
    lossy JPEGs are therefore not pinned to the reference, only the loading rules are)."""
    import io

    from PIL import Image

    img = g["images"][image_index]
    if "uri" in img:
        src = os.path.join(base, img["uri"])
    else:
        view = g["bufferViews"][img["bufferView"]]
        off = view.get("byteOffset", 0)
        src = io.BytesIO(buffers[view["buffer"]][off: off + view["byteLength"]])
    with Image.open(src) as im:
        return np.ascontiguousarray(np.asarray(im.convert("RGBA"), dtype=np.uint8))


def _gltf_material(gm: dict, texture_slot) -> np.ndarray:
    """GltfLoader::createMaterial (GltfLoader.cpp:915-1035) + GpuScene::registerMaterial
    (GpuScene.cpp:1452-1517): blend mode from alphaMode (MASK keeps alphaCutoff), the
    factors, the texture slots (sRGB: base colour, emissive; data: metallic-roughness,
    normal, occlusion; a missing slot keeps the default texture), the
    KHR_materials_pbrSpecularGlossiness / _transmission / _ior / _clearcoat extensions
    and the Arkose BRDF extra. `texture_slot(gltf_texture_index, format)` returns
    the scene texture index."""
    m = default_material()
    mode = gm.get("alphaMode", "OPAQUE")
    if mode == "BLEND":
        m["blend_mode"] = abi.ARK_BLEND_MODE_TRANSLUCENT
    elif mode == "MASK":
        m["blend_mode"] = abi.ARK_BLEND_MODE_MASKED
        m["mask_cutoff"] = float(gm.get("alphaCutoff", 0.5))
    elif mode != "OPAQUE":
        raise ValueError(f"glTF material alphaMode {mode!r}")  # ASSERT_NOT_REACHED (:925)
    m["emissive_factor"] = gm.get("emissiveFactor", [0.0, 0.0, 0.0])
    ext = gm.get("extensions", {})

    def slot(name, info, fmt):
        if info is not None and info.get("index", -1) >= 0:
            m[name] = texture_slot(int(info["index"]), fmt)

    slot("emissive", gm.get("emissiveTexture"), abi.ARK_TEX_RGBA8_SRGB)
    slot("normal_map", gm.get("normalTexture"), abi.ARK_TEX_RGBA8_UNORM)
    slot("occlusion", gm.get("occlusionTexture"), abi.ARK_TEX_RGBA8_UNORM)
    sg = ext.get("KHR_materials_pbrSpecularGlossiness")
    if sg is not None:
        # unsupported model, approximated as the reference does (:944-961)
        m["metallic_factor"] = 0.0
        m["roughness_factor"] = 0.0
        m["color_tint"] = sg.get("diffuseFactor", [1.0, 1.0, 1.0, 1.0])
        slot("base_color", sg.get("diffuseTexture"), abi.ARK_TEX_RGBA8_SRGB)
        slot("metallic_roughness", sg.get("specularGlossinessTexture"), abi.ARK_TEX_RGBA8_UNORM)
    else:
        pbr = gm.get("pbrMetallicRoughness", {})
        m["metallic_factor"] = float(pbr.get("metallicFactor", 1.0))
        m["roughness_factor"] = float(pbr.get("roughnessFactor", 1.0))
        m["color_tint"] = pbr.get("baseColorFactor", [1.0, 1.0, 1.0, 1.0])
        slot("base_color", pbr.get("baseColorTexture"), abi.ARK_TEX_RGBA8_SRGB)
        slot("metallic_roughness", pbr.get("metallicRoughnessTexture"), abi.ARK_TEX_RGBA8_UNORM)
    if "KHR_materials_transmission" in ext:
        m["blend_mode"] = abi.ARK_BLEND_MODE_TRANSLUCENT  # (:976-992)
    ior = np.float32(ext.get("KHR_materials_ior", {}).get("ior", 1.5))
    # MaterialAsset::calculateDielectricReflectance (MaterialAsset.cpp:115-121), interface IOR 1
    q = (ior - np.float32(1.0)) / (ior + np.float32(1.0))
    m["dielectric_reflectance"] = q * q
    cc = ext.get("KHR_materials_clearcoat", {})
    m["clearcoat"] = float(cc.get("clearcoatFactor", 0.0))
    m["clearcoat_roughness"] = float(cc.get("clearcoatRoughnessFactor", 0.0))
    brdf = gm.get("extras", {}).get("arkose", {}).get("brdf")
    if brdf is not None:
        m["brdf"] = {"Default": abi.ARK_BRDF_DEFAULT, "Skin": abi.ARK_BRDF_SKIN}.get(brdf, abi.ARK_BRDF_DEFAULT)
    return m


def load_gltf(path: str, transform: np.ndarray | None = None, textures: bool = True, mesh_name: str | None = None) -> SceneData:
    """Loads a .gltf + .bin as the reference imports it (GltfLoader.cpp:372-543
    geometry, :915-1035 materials, :817-913 samplers; GpuScene::registerMaterial for
    the texture formats): one RT mesh + instance per primitive (mesh segment), CCW
    winding as stored, node transforms not applied (a MeshAsset holds the raw mesh;
    the level object's transform places it). `mesh_name` keeps only that glTF mesh
    (one .arkmsh per glTF mesh). Each (glTF texture, format) pair becomes one scene
    texture, decoded to RGBA8; `textures=False` keeps the factors only."""
    with open(path) as fh:
        g = json.load(fh)
    base = os.path.dirname(path)
    buffers = [open(os.path.join(base, b["uri"]), "rb").read() for b in g["buffers"]]
    tex_list: list = []
    tex_cache: dict = {}
    decoded: dict = {}

    def texture_slot(ti: int, fmt: int) -> int:
        if not textures:
            return -1
        key = (ti, fmt)
        if key not in tex_cache:
            src = g["textures"][ti]["source"]
            if src not in decoded:
                decoded[src] = _decode_image(g, base, buffers, src)
            px = decoded[src]
            tex_cache[key] = len(tex_list)
            tex_list.append(Texture(px.shape[1], px.shape[0], fmt, px, _texture_wrap(g, ti)))
        return tex_cache[key]

    materials = [_gltf_material(gm, texture_slot) for gm in g.get("materials", [])]
    default_index = len(materials)
    materials.append(default_material())  # primitives without a material (GpuScene's default material)
    M = np.eye(3, 4, dtype=np.float32) if transform is None else np.asarray(transform, np.float32).reshape(3, 4)
    pos_l, vtx_l, idx_l, meshes, instances = [], [], [], [], []
    nv = ni = 0
    found = False
    for mesh in g["meshes"]:
        if mesh_name is not None and mesh.get("name") != mesh_name:
            continue
        found = True
        for prim in mesh["primitives"]:
            attrs = prim["attributes"]
            P = _accessor(g, buffers, attrs["POSITION"]).astype(np.float32)
            n = P.shape[0]
            vx = np.zeros(n, dtype=VERTEX_DTYPE)
            if "NORMAL" in attrs:
                vx["normal"] = _accessor(g, buffers, attrs["NORMAL"])
            if "TEXCOORD_0" in attrs:
                vx["tex_coord"] = _accessor(g, buffers, attrs["TEXCOORD_0"])
            if "TANGENT" in attrs:
                vx["tangent"] = _accessor(g, buffers, attrs["TANGENT"])
            idx = _accessor(g, buffers, prim["indices"]).reshape(-1).astype(np.uint32)
            pos_l.append(P)
            vtx_l.append(vx)
            idx_l.append(idx)
            mat = prim.get("material", -1)
            mat = default_index if mat < 0 else mat
            meshes.append((nv, ni, mat))
            inst = np.zeros((), dtype=INSTANCE_DTYPE)
            inst["object_to_world"] = M.reshape(-1)
            inst["rt_mesh_index"] = len(meshes) - 1
            inst["triangle_count"] = idx.size // 3
            bm = int(materials[mat]["blend_mode"])
            inst["hit_mask"] = {abi.ARK_BLEND_MODE_OPAQUE: abi.ARK_RT_HIT_MASK_OPAQUE,
                                abi.ARK_BLEND_MODE_MASKED: abi.ARK_RT_HIT_MASK_MASKED}.get(bm, abi.ARK_RT_HIT_MASK_BLEND)
            instances.append(inst)
            nv += n
            ni += idx.size
    if mesh_name is not None and not found:
        raise KeyError(f"{path}: no glTF mesh named {mesh_name!r}")
    return SceneData(
        positions=np.concatenate(pos_l),
        vertices=np.concatenate(vtx_l),
        indices=np.concatenate(idx_l),
        meshes=np.array(meshes, dtype=MESH_DTYPE),
        materials=np.array(materials, dtype=MATERIAL_DTYPE),
        instances=np.array(instances, dtype=INSTANCE_DTYPE),
        textures=tex_list,
    )


def merge_scenes(parts: list) -> SceneData:
    """One scene of several (GpuScene holds every registered mesh in one set of
    pools): vertex/index pools concatenated, RT meshes, materials, textures,
    instances and spot lights re-indexed. Sun and environment come from the first
    part that has one."""
    pos, vtx, idx, meshes, mats, insts, tex, spots = [], [], [], [], [], [], [], []
    sun, env = None, -1
    nv = ni = nm = nmat = 0
    for p in parts:
        nt = len(tex)
        pos.append(p.positions)
        vtx.append(p.vertices)
        idx.append(p.indices)
        m = p.meshes.copy()
        m["first_vertex"] += nv
        m["first_index"] += ni
        m["material_index"] += nmat
        meshes.append(m)
        mt = p.materials.copy()
        for k in ("base_color", "normal_map", "metallic_roughness", "emissive", "occlusion", "bent_normal_map"):
            mt[k] = np.where(mt[k] >= 0, mt[k] + nt, mt[k])
        mats.append(mt)
        it = p.instances.copy()
        it["rt_mesh_index"] += nm
        insts.append(it)
        tex.extend(p.textures)
        for sl in p.spots:
            spots.append(SpotLight(sl.color, sl.direction, sl.right, sl.up, sl.position, sl.outer_cone_half_angle,
                                   sl.ies_profile_index + nt if sl.ies_profile_index >= 0 else -1))
        if sun is None:
            sun = p.sun
        if env < 0 and p.environment_texture >= 0:
            env = p.environment_texture + nt
        nv += p.positions.shape[0]
        ni += p.indices.size
        nm += p.meshes.size
        nmat += p.materials.size
    return SceneData(positions=np.concatenate(pos), vertices=np.concatenate(vtx), indices=np.concatenate(idx),
                     meshes=np.concatenate(meshes), materials=np.concatenate(mats), instances=np.concatenate(insts),
                     textures=tex, sun=sun, spots=spots, environment_texture=env)


def manual_exposure(f_number: float, shutter: float, iso: float) -> float:
    """Camera::calculateManualExposure (arkose/scene/camera/Camera.cpp:203-214)."""
    ev100 = math.log2((f_number * f_number) / shutter * 100.0 / iso)
    return 1.0 / (1.2 * 2.0 ** ev100)


ASSET_DIRS = [
    os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "assets"),
]


def find_asset(*parts) -> str | None:
    for d in ASSET_DIRS:
        p = os.path.join(d, *parts)
        if os.path.exists(p):
            return p
    return None


def cornell_box() -> tuple[SceneData, dict]:
    """BASELINE config C2 scene: CornellBox.gltf under the CornellBox.arklvl
    transform (+90 deg about X). Returns (scene, exposure info)."""
    path = find_asset("CornellBox", "CornellBox.gltf")
    if path is None:
        raise FileNotFoundError("tests/assets/CornellBox/CornellBox.gltf missing")
    R = quat_to_matrix(0.7071068286895752, 0.0, 0.0, 0.7071067094802856)
    T = np.zeros((3, 4), np.float32)
    T[:, :3] = R
    scene = load_gltf(path, T)
    pre = manual_exposure(11.0, 0.008, 400.0)
    return scene, {"light_pre_exposure": pre, "environment_brightness": 3000.0, "z_far": 10000.0}


def damaged_helmet(textures: bool = False) -> SceneData:
    """BASELINE config C1 input: DamagedHelmet.gltf (15,452 triangles), baked in
    object space at an identity instance transform, as MeshViewerApp.cpp:845-880 sets
    up its bake scene (bakeScene->addMesh). The bake reads no texture; `textures`
    decodes the model's five 2048^2 JPEGs for DDGI shading."""
    path = find_asset("DamagedHelmet", "DamagedHelmet.gltf")
    if path is None:
        raise FileNotFoundError("tests/assets/DamagedHelmet/DamagedHelmet.gltf missing")
    return load_gltf(path, textures=textures)


def soup(triangle_count: int = 10_000_000, **overrides) -> SceneData:
    """BASELINE config C4 synthetic triangle-strip soup (PCG32 seed 0xA2C05E00)."""
    lib = abi.load_library()
    p = abi.ArkSoupParams()
    lib.ark_soup_default_params(C.byref(p))
    p.triangle_count = int(triangle_count)
    for k, v in overrides.items():
        setattr(p, k, v)
    h = C.c_void_p()
    rc = lib.ark_soup_generate(C.byref(p), C.byref(h))
    if rc != 0:
        raise abi.ArkDdgiError(rc, "ark_soup_generate failed")
    v = lib.ark_soup_scene_view(h).contents
    V = int(v.vertex_count)

    def arr(addr, dtype, count):
        buf = (C.c_char * (count * np.dtype(dtype).itemsize)).from_address(addr)
        return np.frombuffer(buf, dtype=dtype, count=count)

    scene = SceneData(
        positions=arr(v.positions, np.float32, V * 3).reshape(V, 3),
        vertices=arr(v.vertices, VERTEX_DTYPE, V),
        indices=arr(v.indices, np.uint32, int(v.index_count)),
        meshes=arr(v.meshes, MESH_DTYPE, int(v.mesh_count)),
        materials=arr(v.materials, MATERIAL_DTYPE, int(v.material_count)),
        instances=arr(v.instances, INSTANCE_DTYPE, int(v.instance_count)),
        sun=(tuple(v.directional_light.color), tuple(v.directional_light.world_space_direction)) if v.has_directional_light else None,
    )
    scene._native = _SoupHandle(lib, h)
    return scene


class _SoupHandle:
    def __init__(self, lib, h):
        self.lib, self.h = lib, h

    def __del__(self):
        try:
            self.lib.ark_soup_free(self.h)
        except Exception:
            pass


def ies_lut(source, size: int = abi.ARK_IES_LUT_SIZE):
    """IES profile -> (size x size float32 LUT, ArkIesInfo) through ark_ies_lut_*
    (IESProfile.cpp + GpuScene.cpp:1101-1124). `source` is a path or the file's text.
    Raises ValueError with the parser's reason where the reference logs Fatal."""
    import ctypes as C
    import os

    import numpy as np

    lib = abi.load_library()
    out = np.empty((size, size), np.float32)
    info = abi.ArkIesInfo()
    if isinstance(source, (str, os.PathLike)) and os.path.exists(source):
        rc = lib.ark_ies_lut_from_file(os.fsencode(source), size, out.ctypes.data, C.byref(info))
    else:
        data = source.encode() if isinstance(source, str) else bytes(source)
        rc = lib.ark_ies_lut_from_memory(data, len(data), size, out.ctypes.data, C.byref(info))
    if rc != abi.ARK_IES_OK:
        raise ValueError(f"IES profile: {lib.ark_ies_last_error().decode()} (status {rc})")
    return out, info


def ies_texture(source, size: int = abi.ARK_IES_LUT_SIZE) -> Texture:
    """The spot light's LUT texture (R32F, clamp to edge, GpuScene.cpp:1108-1115)."""
    lut, _ = ies_lut(source, size)
    return Texture(size, size, abi.ARK_TEX_R32F, lut, abi.ARK_WRAP_CLAMP_TO_EDGE)


def sponza_substitute(ies_dir: str | None = None) -> SceneData:
    """BASELINE config C3 substitute (Sponza.bin is not in the reference's
    assets, .MISSING_LARGE_BLOBS): a 262,272-triangle strip soup over [0, 31] m (the
    C4 generator at Sponza's triangle count) with the C4 sun and three spot lights
    from 20 m, pointing down, lit by the reference's multi-lobe.ies profile (LUT
    normalised by its peak candela), for the 24x12x24-probe grid of
    sponza_substitute_grid()."""
    import os

    sc = soup(262_272, extent=31.0)
    here = ies_dir or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "ies")
    lut, info = ies_lut(os.path.join(here, "multi-lobe.ies"))
    sc.textures.append(Texture(256, 256, abi.ARK_TEX_R32F, lut / np.float32(info.max_candela), abi.ARK_WRAP_CLAMP_TO_EDGE))
    t = len(sc.textures) - 1
    sc.spots = [SpotLight((200.0, 190.0, 170.0), (0.0, -1.0, 0.0), (1.0, 0.0, 0.0), (0.0, 0.0, 1.0), (x, 20.0, z), 1.0, t)
                for x, z in ((8.0, 8.0), (16.0, 24.0), (24.0, 12.0))]
    return sc


def sponza_substitute_grid():
    """(grid dims, spacing, origin) of config C3: 24x12x24 probes over the [0.5, 31.5] m box."""
    return (24, 12, 24), (31.0 / 24, 31.0 / 12, 31.0 / 24), (0.5, 0.5, 0.5)


def _box_mesh():
    """Unit cube [0,1]^3, 24 vertices (flat normals), 12 CCW triangles facing out."""
    faces = [((0, 0, 1), [(0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)]), ((0, 0, -1), [(1, 0, 0), (0, 0, 0), (0, 1, 0), (1, 1, 0)]),
             ((1, 0, 0), [(1, 0, 1), (1, 0, 0), (1, 1, 0), (1, 1, 1)]), ((-1, 0, 0), [(0, 0, 0), (0, 0, 1), (0, 1, 1), (0, 1, 0)]),
             ((0, 1, 0), [(0, 1, 1), (1, 1, 1), (1, 1, 0), (0, 1, 0)]), ((0, -1, 0), [(0, 0, 0), (1, 0, 0), (1, 0, 1), (0, 0, 1)])]
    pos, nrm, uv, idx = [], [], [], []
    for n, quad in faces:
        b = len(pos)
        pos += quad
        nrm += [n] * 4
        uv += [(0, 0), (1, 0), (1, 1), (0, 1)]
        idx += [b, b + 1, b + 2, b, b + 2, b + 3]
    return np.array(pos, np.float32), np.array(nrm, np.float32), np.array(uv, np.float32), np.array(idx, np.uint32)


def city_block(box_count: int = 250_000, extent: float = 240.0, seed: int = 0xB15780, ies_sources=None) -> SceneData:
    """BASELINE config C5 substitute (Bistro is not in the reference's
    assets): a synthetic city block of instanced boxes on a ground plane, ~12
    triangles per box (250,000 boxes ~ 3 M triangles), 8 box meshes x 8 materials,
    a sun and 4 IES spot lights at street level using the reference's sample
    profiles (assets/sample/ies: multi-lobe.ies, simple.ies; LUTs via ark_ies).
    Buildings (2 % of the boxes) stand on a street grid; the rest are props of
    0.1-1.5 m scattered over streets and building fronts up to 30 m."""
    rng = np.random.default_rng(seed)
    bp, bn, buv, bi = _box_mesh()
    n_mesh = 8
    V = len(bp)
    positions = [np.tile(bp, (n_mesh, 1)), np.array([[0, 0, 0], [extent, 0, 0], [extent, 0, extent], [0, 0, extent]], np.float32)]
    verts = np.zeros(n_mesh * V + 4, dtype=VERTEX_DTYPE)
    verts["normal"][: n_mesh * V] = np.tile(bn, (n_mesh, 1))
    verts["tex_coord"][: n_mesh * V] = np.tile(buv, (n_mesh, 1))
    verts["normal"][n_mesh * V:] = (0, 1, 0)
    verts["tex_coord"][n_mesh * V:] = [(0, 0), (8, 0), (8, 8), (0, 8)]
    indices = np.concatenate([np.tile(bi, n_mesh), np.array([0, 2, 1, 0, 3, 2], np.uint32)])
    meshes = np.zeros(n_mesh + 1, dtype=MESH_DTYPE)
    meshes["first_vertex"] = [m * V for m in range(n_mesh)] + [n_mesh * V]
    meshes["first_index"] = [m * 36 for m in range(n_mesh)] + [n_mesh * 36]
    meshes["material_index"] = list(range(n_mesh)) + [n_mesh]
    mats = np.array([default_material() for _ in range(n_mesh + 1)], dtype=MATERIAL_DTYPE)
    mats["color_tint"][:, :3] = rng.uniform(0.1, 0.9, (n_mesh + 1, 3))
    mats["metallic_factor"] = rng.uniform(0.0, 0.3, n_mesh + 1)
    mats["roughness_factor"] = rng.uniform(0.3, 1.0, n_mesh + 1)

    n_build = max(1, box_count // 50)
    n_prop = box_count - n_build
    cell = extent / math.ceil(math.sqrt(n_build))
    gx = rng.integers(0, int(extent // cell), n_build)
    gz = rng.integers(0, int(extent // cell), n_build)
    bsize = np.stack([rng.uniform(0.3, 0.75, n_build) * cell, rng.uniform(5, 35, n_build), rng.uniform(0.3, 0.75, n_build) * cell], -1)
    borig = np.stack([gx * cell + rng.uniform(0.05, 0.2, n_build) * cell, np.zeros(n_build), gz * cell + rng.uniform(0.05, 0.2, n_build) * cell], -1)
    psize = rng.uniform(0.1, 1.5, (n_prop, 3))
    porig = np.stack([rng.uniform(0, extent, n_prop), np.minimum(rng.exponential(4.0, n_prop), 30.0), rng.uniform(0, extent, n_prop)], -1)
    size = np.concatenate([bsize, psize]).astype(np.float32)
    orig = np.concatenate([borig, porig]).astype(np.float32)
    inst = np.zeros(box_count + 1, dtype=INSTANCE_DTYPE)
    m = np.zeros((box_count, 3, 4), np.float32)
    m[:, 0, 0], m[:, 1, 1], m[:, 2, 2] = size[:, 0], size[:, 1], size[:, 2]
    m[:, :, 3] = orig
    inst["object_to_world"][:box_count] = m.reshape(box_count, 12)
    inst["rt_mesh_index"][:box_count] = rng.integers(0, n_mesh, box_count)
    inst["triangle_count"][:box_count] = 12
    inst["object_to_world"][box_count] = np.eye(3, 4, dtype=np.float32).reshape(12)
    inst["rt_mesh_index"][box_count] = n_mesh
    inst["triangle_count"][box_count] = 2
    inst["hit_mask"] = abi.ARK_RT_HIT_MASK_OPAQUE

    textures = []
    if ies_sources is None:
        here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "ies")
        ies_sources = [os.path.join(here, "multi-lobe.ies"), os.path.join(here, "simple.ies")]
    for src in ies_sources:
        lut, info = ies_lut(src)
        textures.append(Texture(lut.shape[1], lut.shape[0], abi.ARK_TEX_R32F, lut / np.float32(info.max_candela), abi.ARK_WRAP_CLAMP_TO_EDGE))
    env = np.ones((4, 8, 4), np.float32)
    env[..., :3] = np.linspace(0.3, 1.2, 4)[:, None, None] * np.array([0.6, 0.75, 1.0], np.float32)
    textures.append(Texture(8, 4, abi.ARK_TEX_RGBA32F, env))
    spots = []
    for k in range(4):
        px, pz = rng.uniform(0.2, 0.8, 2) * extent
        spots.append(SpotLight((400.0, 380.0, 300.0), (0.0, -1.0, 0.0), (1.0, 0.0, 0.0), (0.0, 0.0, 1.0),
                               (float(px), 6.0, float(pz)), 1.2, k % 2))
    sun_dir = np.array([0.4, -1.0, 0.3]) / np.linalg.norm([0.4, -1.0, 0.3])
    return SceneData(positions=np.concatenate(positions), vertices=verts, indices=indices, meshes=meshes, materials=mats,
                     instances=inst, textures=textures, sun=((3.0, 2.9, 2.7), tuple(sun_dir)), spots=spots,
                     environment_texture=len(ies_sources))
