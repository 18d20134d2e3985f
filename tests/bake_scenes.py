"""Small closed-form scenes for the AO / bent-normal bake (test infrastructure)."""
from __future__ import annotations

import numpy as np

from arkoserenderer_amd import abi
from arkoserenderer_amd import scene as S


def _mesh(positions, normals, uvs, indices):
    n = len(positions)
    vx = np.zeros(n, dtype=S.VERTEX_DTYPE)
    vx["normal"] = normals
    vx["tex_coord"] = uvs
    return np.asarray(positions, np.float32), vx, np.asarray(indices, np.uint32)


def quad_scene(with_box: bool = False, lid: bool = False) -> S.SceneData:
    """Instance 0: the unit quad z = 0, (x, y) = (u, v), normal +z, two CCW
    triangles covering the whole UV square. with_box: a closed inward-facing cube
    [-10, 10]^3 around it (every AO ray hits). lid: a 3x3 m quad at z = 0.25 facing
    down (partial occlusion)."""
    meshes, pos, vtx, idx = [], [], [], []
    nv = ni = 0

    def add(p, n, uv, ind):
        nonlocal nv, ni
        P, V, I = _mesh(p, n, uv, ind)
        meshes.append((nv, ni, 0))
        pos.append(P)
        vtx.append(V)
        idx.append(I)
        nv += len(P)
        ni += len(I)
        return len(I) // 3

    # UV 1.0 would wrap to 0 under the vertex shader's fract() (bakeParameterization.vert:10),
    # so the quad's far edge sits at 1 - 2^-20 (it still snaps to the texture edge)
    e = np.float32(1.0 - 2.0 ** -20)
    tri_counts = [add([(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0)], [(0, 0, 1)] * 4, [(0, 0), (e, 0), (e, e), (0, e)], [0, 1, 2, 0, 2, 3])]
    if with_box:
        c = np.array([[x, y, z] for z in (-10, 10) for y in (-10, 10) for x in (-10, 10)], np.float32)
        # faces wound so that the inside is the front side (normals point inwards)
        faces = [(0, 2, 3, 1), (4, 5, 7, 6), (0, 1, 5, 4), (2, 6, 7, 3), (0, 4, 6, 2), (1, 3, 7, 5)]
        ind = []
        for a, b, cc, d in faces:
            ind += [a, cc, b, a, d, cc]
        tri_counts.append(add(c, np.zeros((8, 3), np.float32), np.zeros((8, 2), np.float32), ind))
    if lid:
        tri_counts.append(add([(-1, -1, 0.25), (2, -1, 0.25), (2, 2, 0.25), (-1, 2, 0.25)], [(0, 0, -1)] * 4,
                              [(0, 0)] * 4, [0, 2, 1, 0, 3, 2]))
    instances = []
    for m, tc in enumerate(tri_counts):
        inst = np.zeros((), dtype=S.INSTANCE_DTYPE)
        inst["object_to_world"] = np.eye(3, 4, dtype=np.float32).reshape(-1)
        inst["rt_mesh_index"] = m
        inst["triangle_count"] = tc
        inst["hit_mask"] = abi.ARK_RT_HIT_MASK_OPAQUE
        instances.append(inst)
    return S.SceneData(positions=np.concatenate(pos), vertices=np.concatenate(vtx), indices=np.concatenate(idx),
                       meshes=np.array(meshes, dtype=S.MESH_DTYPE), materials=np.array([S.default_material()], dtype=S.MATERIAL_DTYPE),
                       instances=np.array(instances, dtype=S.INSTANCE_DTYPE))
