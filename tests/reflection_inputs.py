"""Synthetic G-buffer + camera for the RT reflections raygen tests (no rasteriser:
random depth/normal/material planes in the formats GpuScene.cpp:326-360 creates)."""
import numpy as np


def camera(width, height, eye=(0.0, 1.2, 3.0), target=(0.0, 0.6, 0.0), fov_y=1.0, near=0.1, far=100.0):
    """CameraState.worldFromView / viewFromProjection (column-major float32[16]) of a
    right-handed look-at camera with a Vulkan [0, 1]-depth perspective projection."""
    eye, target = np.asarray(eye, np.float64), np.asarray(target, np.float64)
    f = target - eye
    f /= np.linalg.norm(f)
    s = np.cross(f, (0.0, 1.0, 0.0))
    s /= np.linalg.norm(s)
    u = np.cross(s, f)
    view = np.eye(4)
    view[0, :3], view[1, :3], view[2, :3] = s, u, -f
    view[:3, 3] = -view[:3, :3] @ eye
    t = 1.0 / np.tan(fov_y / 2)
    proj = np.zeros((4, 4))
    proj[0, 0], proj[1, 1] = t / (width / height), t
    proj[2, 2], proj[2, 3] = far / (near - far), far * near / (near - far)
    proj[3, 2] = -1.0
    col = lambda m: np.asarray(m, np.float32).T.reshape(16)  # noqa: E731  (column-major)
    return {"world_from_view": col(np.linalg.inv(view)), "view_from_projection": col(np.linalg.inv(proj))}


def oct_encode(n):
    n = n / np.abs(n).sum(axis=-1, keepdims=True)
    x, y, z = n[..., 0], n[..., 1], n[..., 2]
    sx, sy = np.where(x >= 0, 1.0, -1.0), np.where(y >= 0, 1.0, -1.0)
    ex = np.where(z >= 0, x, (1 - np.abs(y)) * sx)
    ey = np.where(z >= 0, y, (1 - np.abs(x)) * sy)
    return ex, ey


def gbuffer(width, height, cam, seed=5, sky_frac=0.1, rough_frac=0.2, roughness=None):
    """Normals face the viewer (dot(N, -viewRay) > 0.2): a backfacing view vector
    makes the raygen's GGX sample normalize(0) at roughness 0, undefined in GLSL."""
    rng = np.random.default_rng(seed)
    depth = rng.uniform(0.95, 0.9995, (height, width)).astype(np.float32)
    depth[rng.random((height, width)) < sky_frac] = 1.0
    ys, xs = np.mgrid[0:height, 0:width]
    ndc = np.stack([(xs + 0.5) / width * 2 - 1, (ys + 0.5) / height * 2 - 1, depth, np.ones_like(depth)], -1).astype(np.float64)
    pv = ndc @ cam["view_from_projection"].reshape(4, 4).astype(np.float64)  # column-major: rows of M^T
    v = pv[..., :3] / pv[..., 3:]
    v /= np.linalg.norm(v, axis=-1, keepdims=True)
    n = -v + 0.7 * rng.normal(size=(height, width, 3))
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    bad = np.sum(n * -v, axis=-1) < 0.2
    n[bad] = -v[bad]
    ex, ey = oct_encode(n)
    nv = np.zeros((height, width, 4), np.float16)
    nv[..., 0], nv[..., 1] = ex, ey
    mat = rng.integers(0, 256, (height, width, 4)).astype(np.uint8)
    mat[..., 0] = rng.integers(0, 150, (height, width)) if roughness is None else roughness
    mat[rng.random((height, width)) < rough_frac, 0] = 230  # >= 0.6: not traced
    mat[rng.random((height, width)) < rough_frac / 2, 0] = 160  # 0.627, in [0.6, 0.7): not traced at the node's 0.6 (RTReflectionsNode.h:20)
    noise = rng.random((64, 64, 2)).astype(np.float32)
    return {"depth": depth, "material": mat, "normal_velocity": nv.view(np.uint16), "blue_noise": noise}, n.astype(np.float32)
