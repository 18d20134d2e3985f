"""Seeded G-buffer planes and a camera for the lighting-compose parity tests
(test infrastructure)."""
from __future__ import annotations

import numpy as np


def camera(width: int, height: int, eye=(0.0, 1.0, 2.5), target=(0.0, 0.8, 0.0), fov_y=1.0, near=0.1, far=100.0):
    """CameraState matrices (shared/CameraState.h) as column-major float32[16]:
    view_from_pixel = inverse(pixelFromView), view_from_world, world_from_view."""
    eye, target = np.asarray(eye, np.float64), np.asarray(target, np.float64)
    f = target - eye
    f /= np.linalg.norm(f)
    r = np.cross(f, [0.0, 1.0, 0.0])
    r /= np.linalg.norm(r)
    u = np.cross(r, f)
    view = np.eye(4)
    view[0, :3], view[1, :3], view[2, :3] = r, u, -f
    view[:3, 3] = -view[:3, :3] @ eye
    t = 1.0 / np.tan(fov_y / 2)
    a = width / height
    proj = np.zeros((4, 4))  # Vulkan clip space, depth [0, 1]
    proj[0, 0], proj[1, 1] = t / a, -t
    proj[2, 2], proj[2, 3] = far / (near - far), near * far / (near - far)
    proj[3, 2] = -1.0
    viewport = np.array([[width / 2, 0, 0, width / 2], [0, height / 2, 0, height / 2], [0, 0, 1, 0], [0, 0, 0, 1]], np.float64)
    pixel_from_view = viewport @ proj
    col = lambda m: np.asarray(m, np.float32).T.reshape(16).copy()  # noqa: E731  (column-major)
    return {"view_from_pixel": col(np.linalg.inv(pixel_from_view)), "view_from_world": col(view),
            "world_from_view": col(np.linalg.inv(view))}


def f16(a):
    return np.asarray(a, np.float32).astype(np.float16).view(np.uint16)


def oct_encode(n):
    n = n / np.abs(n).sum(-1, keepdims=True)
    x, y, z = n[..., 0], n[..., 1], n[..., 2]
    sx, sy = np.where(x >= 0, 1.0, -1.0), np.where(y >= 0, 1.0, -1.0)
    ox = np.where(z < 0, (1 - np.abs(y)) * sx, x)
    oy = np.where(z < 0, (1 - np.abs(x)) * sy, y)
    return ox, oy


def gbuffer(width: int, height: int, seed: int = 7, sky_frac: float = 0.1, reflect_frac: float = 0.5, bent_neg_frac: float = 0.2):
    """Random but plausible planes: depth in (0.9, 1) with a sky fraction at 1.0,
    unit octahedral normals, positive radiance, bent normals of length <= 1 (some with
    a negative cone), half the pixels with a reflection direction."""
    rng = np.random.default_rng(seed)
    H, W = height, width
    depth = rng.uniform(0.90, 0.9995, (H, W)).astype(np.float32)
    depth[rng.random((H, W)) < sky_frac] = 1.0
    n = rng.normal(size=(H, W, 3))
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    ox, oy = oct_encode(n)
    nv = np.stack([ox, oy, rng.normal(0, 0.01, (H, W)), rng.normal(0, 0.01, (H, W))], -1)
    bn = rng.normal(size=(H, W, 3))
    bn /= np.linalg.norm(bn, axis=-1, keepdims=True)
    bn *= rng.uniform(0.2, 1.0, (H, W, 1))
    cone = rng.uniform(0.0, 1.0, (H, W, 1))
    cone[rng.random((H, W)) < bent_neg_frac] = -1.0
    rdir = rng.normal(size=(H, W, 3))
    rdir /= np.linalg.norm(rdir, axis=-1, keepdims=True)
    rdir[rng.random((H, W)) >= reflect_frac] = 0.0
    return {
        "depth": depth,
        "base_color": rng.integers(0, 256, (H, W, 4), dtype=np.uint8),
        "material": rng.integers(0, 256, (H, W, 4), dtype=np.uint8),
        "normal_velocity": f16(nv),
        "bent_normal": f16(np.concatenate([bn, cone], -1)),
        "direct_light": f16(rng.uniform(0, 4, (H, W, 4))),
        "diffuse_irradiance": f16(rng.uniform(0, 2, (H, W, 4))),
        "reflections": f16(rng.uniform(0, 3, (H, W, 4))),
        "reflection_direction": f16(np.concatenate([rdir, np.zeros((H, W, 1))], -1)),
        "screen_space_occlusion": rng.uniform(0, 1, (H, W)).astype(np.float32),
    }
