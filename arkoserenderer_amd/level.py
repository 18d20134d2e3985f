"""Level loading (.arklvl) for the DDGI path: Scene::setupFromLevel
(arkose/scene/Scene.cpp:240-292) restated for the parts the probe update reads.

* objects -> static mesh instances at the object's transform (Transform.h:160-166:
  translate * rotate * scale); a ``.arkmsh`` is resolved to the glTF mesh it was
  imported from (ArkAssetBakeTool: one MeshAsset per glTF mesh, same name);
* lights -> the light buffers GpuScene::update uploads (GpuScene.cpp:790-858):
  colour = Color::fromNonLinearSRGB(asset colour) * intensity * lightPreExposure,
  directions = the transform's forward / right / up (Transform.h:54-56), spot
  position = translation, outer cone half angle = outerConeAngle / 2, spot IES
  profile -> LUT texture (GpuScene.cpp:1101-1124, ies_profile.cpp);
* cameras -> zFar and the manual exposure (Camera.cpp:203-214) = lightPreExposure;
* environmentMap -> brightness factor (the HDRI itself is not in the tree: the
  1x1 white default, GpuScene.cpp:1041-1048);
* probeGrid -> the level's grid, else ``ProbeGrid.from_bounding_box`` as the
  apps do for levels without one (ShowcaseApp.cpp:133-134, Scene.cpp:534-583).

The float32 conversions follow the reference's header-only math library
(deps/arklib: quaternion.h rotateVector, transform.h, color.h gammaDecode) in the
same operation order; tests/test_level.py pins them bit for bit against
oracle/level_kat.cpp built on that library (tests/golden/level_kat.json).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

import numpy as np

from . import abi
from . import scene as S

F = np.float32


def _v3(d: dict) -> np.ndarray:
    return np.array([d["x"], d["y"], d["z"]], dtype=F)


def _quat(d: dict) -> np.ndarray:
    return np.array([d["x"], d["y"], d["z"], d["w"]], dtype=F)


def _cross(a, b):
    return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]], dtype=F)


def rotate_vector(q: np.ndarray, v) -> np.ndarray:
    """ark::rotateVector = quat * vec3 (arklib quaternion.h:68-77, ryg's method):
    t = 2 cross(q.xyz, v); v + q.w t + cross(q.xyz, t), in float32."""
    q = np.asarray(q, F)
    v = np.asarray(v, F)
    t = F(2.0) * _cross(q[:3], v)
    return (v + q[3] * t) + _cross(q[:3], t)


GLOBAL_RIGHT = np.array([1.0, 0.0, 0.0], F)    # arklib vector.h:865-867
GLOBAL_UP = np.array([0.0, 1.0, 0.0], F)
GLOBAL_FORWARD = np.array([0.0, 0.0, -1.0], F)


def local_matrix(t, q, s) -> np.ndarray:
    """Transform::calculateLocalMatrix (Transform.h:160-166): translate(t) *
    rotate(q) * scale(s), rotate's columns = rotateVector(q, x/y/z) (quaternion.h:260-268).
    Returns the 4x4 matrix in row-major numpy order (m[row, col])."""
    R = np.stack([rotate_vector(q, e) for e in np.eye(3, dtype=F)], axis=1)  # columns
    T4 = np.eye(4, dtype=F)
    T4[:3, 3] = t
    R4 = np.eye(4, dtype=F)
    R4[:3, :3] = R
    S4 = np.diag(np.array([s[0], s[1], s[2], 1.0], F))
    return _mat4_mul(_mat4_mul(T4, R4), S4)


def _mat4_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """arklib mat4 * mat4: column c = a.x * b[c].x + a.y * b[c].y + a.z * b[c].z + a.w * b[c].w,
    summed left to right in float32."""
    out = np.zeros((4, 4), F)
    for c in range(4):
        acc = a[:, 0] * b[0, c]
        for k in range(1, 4):
            acc = acc + a[:, k] * b[k, c]
        out[:, c] = acc
    return out


_libm = None


def _powf(x, y) -> np.float32:
    """C powf (std::pow(float, float)); numpy's float32 power rounds differently."""
    global _libm
    if _libm is None:
        import ctypes
        import ctypes.util

        _libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
        _libm.powf.restype = ctypes.c_float
        _libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]
    return F(_libm.powf(float(x), float(y)))


def gamma_decode(c) -> np.ndarray:
    """colorspace::sRGB::gammaDecode (arklib color.h:188-194), per component in float32."""
    out = []
    for x in np.asarray(c, F):
        out.append(x / F(12.92) if x < F(0.04045) else _powf((x + F(0.055)) / F(1.055), F(2.4)))
    return np.array(out, F)


@dataclass
class LevelData:
    """What a loaded level gives the DDGI node."""
    scene: S.SceneData
    probe_grid: object                 # ddgi.ProbeGrid
    probe_grid_from_level: bool
    z_far: float
    light_pre_exposure: float
    environment_brightness: float
    ambient_illuminance: float = 0.0   # Scene.h:163 (levels carry none)
    missing_meshes: list = field(default_factory=list)
    name: str = ""

    def exposure(self) -> dict:
        """Keyword arguments of ddgi.frame_params / DDGINode.construct."""
        return dict(light_pre_exposure=self.light_pre_exposure, environment_brightness=self.environment_brightness,
                    ambient_illuminance=self.ambient_illuminance)


def _asset_dirs():
    return S.ASSET_DIRS


def resolve_mesh(arkmsh_path: str) -> tuple[str, str] | None:
    """``assets/sample/models/<Model>/<mesh>.arkmsh`` -> (glTF path, glTF mesh name):
    the in-tree glTF of that model and its mesh named <mesh> (or the model's only
    mesh). None when the model is not in the tree."""
    parts = arkmsh_path.replace("\\", "/").split("/")
    if len(parts) < 2:
        return None
    model, stem = parts[-2], os.path.splitext(parts[-1])[0]
    for d in _asset_dirs():
        folder = os.path.join(d, model)
        if not os.path.isdir(folder):
            continue
        for fn in sorted(os.listdir(folder)):
            if not fn.endswith(".gltf"):
                continue
            path = os.path.join(folder, fn)
            with open(path) as fh:
                names = [m.get("name", "") for m in json.load(fh).get("meshes", [])]
            if stem in names:
                return path, stem
            if len(names) == 1:
                return path, names[0]
    return None


def resolve_ies(ies_path: str) -> str | None:
    """``assets/sample/ies/<name>.ies`` -> the in-tree copy of that profile."""
    name = os.path.basename(ies_path.replace("\\", "/"))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for d in (os.path.join(root, "tests", "golden", "ies"),):
        p = os.path.join(d, name)
        if os.path.exists(p):
            return p
    return None


def mesh_aabb(gltf_path: str, mesh_name: str) -> tuple[np.ndarray, np.ndarray]:
    """MeshAsset::boundingBox: the union of its segments' POSITION accessor min / max
    (GltfLoader.cpp:355-356), in float32."""
    with open(gltf_path) as fh:
        g = json.load(fh)
    lo = np.full(3, np.inf, F)
    hi = np.full(3, -np.inf, F)
    for m in g["meshes"]:
        if m.get("name") != mesh_name:
            continue
        for prim in m["primitives"]:
            acc = g["accessors"][prim["attributes"]["POSITION"]]
            lo = np.minimum(lo, np.array(acc["min"], F))
            hi = np.maximum(hi, np.array(acc["max"], F))
    return lo, hi


def transformed_aabb(lo, hi, M: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """ark::aabb3::transformed (arklib aabb.h:57-76): the 8 corners through mat4 * vec3
    (dotVec4WithVec3ImplicitW1, matrix.h:265-272), then their min / max."""
    rlo = np.full(3, np.inf, F)
    rhi = np.full(3, -np.inf, F)
    for cx in (lo[0], hi[0]):
        for cy in (lo[1], hi[1]):
            for cz in (lo[2], hi[2]):
                p = np.array([M[r, 0] * cx + M[r, 1] * cy + M[r, 2] * cz + M[r, 3] * F(1.0) for r in range(3)], F)
                rlo = np.minimum(rlo, p)
                rhi = np.maximum(rhi, p)
    return rlo, rhi


def load_level(path: str, allow_missing_meshes: bool = False, textures: bool = True) -> LevelData:
    """Loads an .arklvl (JSON, LevelAsset.h:143-260 via cereal) as Scene::setupFromLevel
    does for the DDGI path. A mesh whose model is not in the tree raises, unless
    `allow_missing_meshes` (then it is listed in `missing_meshes`). An unknown light
    type is ignored with an error, as Scene.cpp:270-276 logs and skips it."""
    from . import ddgi as D

    with open(path) as fh:
        L = json.load(fh)["level"]
    parts, missing = [], []
    box_lo = box_hi = None  # scene AABB of Scene::generateProbeGridFromBoundingBox (Scene.cpp:538-546)
    for obj in L.get("objects", []):
        mesh = obj.get("mesh", {})
        data = mesh.get("data") if isinstance(mesh, dict) else None
        if not isinstance(data, str) or not data:
            continue  # hasPathToMesh() false (Scene.cpp:250)
        res = resolve_mesh(data)
        if res is None:
            if not allow_missing_meshes:
                raise FileNotFoundError(f"{path}: mesh {data!r} is not in the tree")
            missing.append(data)
            continue
        tr = obj["transform"]
        M = local_matrix(_v3(tr["translation"]), _quat(tr["orientation"]), _v3(tr["scale"]))
        parts.append(S.load_gltf(res[0], M[:3, :4], textures=textures, mesh_name=res[1]))
        blo, bhi = transformed_aabb(*mesh_aabb(res[0], res[1]), M)
        box_lo = blo if box_lo is None else np.minimum(box_lo, blo)
        box_hi = bhi if box_hi is None else np.maximum(box_hi, bhi)
    # camera: the last one added is the scene's (Scene::addCamera); manual exposure only
    z_far, exposure = 10000.0, 1.0
    for cam in L.get("cameras", []):
        z_far = float(cam.get("farClipPlane", 10000.0))
        if cam.get("exposureMode", "Manual") != "Manual":
            raise ValueError(f"{path}: camera exposure mode {cam.get('exposureMode')!r} (automatic exposure needs the rendered frame)")
        exposure = S.manual_exposure(float(cam["fNumber"]), float(cam["shutterSpeed"]), float(cam["iso"]))
    pre = F(exposure)
    sun, spots, ies_textures = None, [], []
    for la in L.get("lights", []):
        kind = la.get("type")
        tr = la["transform"]
        q = _quat(tr["orientation"])
        color = gamma_decode(_v3(la["color"]))  # Light(Type, LightAsset) (Light.cpp:15-18)
        d = la["data"]["data"]
        if kind == "DirectionalLight":
            if sun is not None:
                raise ValueError(f"{path}: more than one directional light (GpuScene.cpp:803)")
            c = (color * F(d["illuminance"])) * pre
            sun = (tuple(float(x) for x in c), tuple(float(x) for x in rotate_vector(q, GLOBAL_FORWARD)))
        elif kind == "SpotLight":
            c = (color * F(d["luminousIntensity"])) * pre
            ies = -1
            src = resolve_ies(d.get("iesProfilePath", ""))
            if src is None:
                raise FileNotFoundError(f"{path}: IES profile {d.get('iesProfilePath')!r} is not in the tree")
            ies = len(ies_textures)
            ies_textures.append(S.ies_texture(src))
            spots.append(S.SpotLight(tuple(float(x) for x in c), tuple(float(x) for x in rotate_vector(q, GLOBAL_FORWARD)),
                                     tuple(float(x) for x in rotate_vector(q, GLOBAL_RIGHT)),
                                     tuple(float(x) for x in rotate_vector(q, GLOBAL_UP)),
                                     tuple(float(x) for x in _v3(tr["translation"])),
                                     float(F(d["outerConeAngle"]) / F(2.0)), ies))
        # other light types: logged and ignored by the reference (Scene.cpp:275)
    lights = S.SceneData(positions=np.zeros((0, 3), F), vertices=np.zeros(0, S.VERTEX_DTYPE), indices=np.zeros(0, np.uint32),
                         meshes=np.zeros(0, S.MESH_DTYPE), materials=np.zeros(0, S.MATERIAL_DTYPE),
                         instances=np.zeros(0, S.INSTANCE_DTYPE), textures=ies_textures, sun=sun, spots=spots)
    if not parts:
        raise ValueError(f"{path}: no mesh of the level is in the tree")
    sc = S.merge_scenes(parts + [lights])
    env = L.get("environmentMap", {})
    brightness = float(env["data"]["brightnessFactor"]) if not env.get("nullopt", True) else 1.0
    pg = L.get("probeGrid", {})
    if not pg.get("nullopt", True):
        g = pg["data"]
        grid = D.ProbeGrid(tuple(int(g["gridDimensions"][k]) for k in "xyz"),
                           tuple(float(g["probeSpacing"][k]) for k in "xyz"),
                           tuple(float(g["offsetToFirst"][k]) for k in "xyz"))
        from_level = True
    else:
        grid = D.ProbeGrid.from_bounding_box(box_lo, box_hi)
        from_level = False
    return LevelData(scene=sc, probe_grid=grid, probe_grid_from_level=from_level, z_far=z_far,
                     light_pre_exposure=float(pre), environment_brightness=brightness, missing_meshes=missing,
                     name=L.get("name", ""))
