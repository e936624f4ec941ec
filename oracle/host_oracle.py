"""TEST INFRASTRUCTURE ONLY — numpy restatements of the reference's host-side builders.

Independent of the product's C++ (hello-raytracing_amd/csrc/host/), used by tests/test_host.py to check it
byte for byte:
  camera_new     src/scene/camera.rs:15-28 with glam 0.24's scalar Vec3 (dot = x*x' + y*y' + z*z',
                 cross, normalize = v * (1/|v|)), all f32, no contraction (Rust never fuses).
  parse_obj      the parts of tobj 4.0.3 (default LoadOptions) that src/geometry/mesh.rs:11-62 consumes:
                 `v` positions and face corners in file order, models split at `o`/`g`.
  tree_build     src/scene/bvh/tree.rs:36-90 (add_mesh + build): BFS stable sort by centroid axis,
                 implicit-heap AABB unions, unit normals.
"""
from __future__ import annotations

from collections import deque

import numpy as np

f32 = np.float32
FMAX = np.finfo(np.float32).max


def _dot(a, b):
    return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def _cross(a, b):
    return np.array([f32(a[1] * b[2]) - f32(b[1] * a[2]), f32(a[2] * b[0]) - f32(b[2] * a[0]),
                     f32(a[0] * b[1]) - f32(b[0] * a[1])], dtype=np.float32)


def _normalize(v):
    rec = f32(f32(1.0) / f32(np.sqrt(_dot(v, v))))
    return (v * rec).astype(np.float32)


def camera_new(frm, to, focal, blur, fov) -> np.ndarray:
    """Camera::new -> 20 f32 (eye, direction, up, right with w = 1; focal, blur, fov, 0)."""
    frm = np.asarray(frm, dtype=np.float32)
    to = np.asarray(to, dtype=np.float32)
    direction = _normalize((to - frm).astype(np.float32))
    right = _normalize(_cross(direction, np.array([0, 1, 0], dtype=np.float32)))
    up = _normalize(_cross(right, direction))
    out = np.zeros(20, dtype=np.float32)
    for k, v in enumerate((frm, direction, up, right)):
        out[4 * k:4 * k + 3] = v
        out[4 * k + 3] = 1.0
    out[16:19] = [focal, blur, fov]
    return out


def parse_obj(text: str):
    """-> list of models, each a list of face-corner positions [(x, y, z) f32 ...] in file order,
    plus per-model unique-position counts (tobj's per-model vertex de-duplication)."""
    pos = []
    models, cur = [], []

    def flush():
        if cur:
            models.append(list(cur))
            cur.clear()

    for line in text.split("\n"):
        w = line.split()
        if not w:
            continue
        if w[0] == "v":
            pos.append(np.array([np.float32(t) for t in w[1:4]], dtype=np.float32))
        elif w[0] == "f":
            face = []
            for t in w[1:]:
                i = int(t.split("/")[0])
                face.append(len(pos) + i if i < 0 else i - 1)
            cur.append(face)
        elif w[0] in ("o", "g"):
            flush()
    flush()
    corners = [[pos[i] for f in m for i in f] for m in models]
    uniq = [len({i for f in m for i in f}) for m in models]
    return corners, uniq


def tree_build(meshes):
    """meshes: list of (corner_positions list, material_index). Returns (sizes, nodes[n,2,4], tris[m] as
    (a, b, c, custom, material))."""
    tris = []
    for corners, mat in meshes:
        for k in range(0, len(corners) - len(corners) % 3, 3):
            a, b, c = (np.append(corners[k + j], f32(1.0)).astype(np.float32) for j in range(3))
            custom = ((a + b) + c)[:3].astype(np.float32)
            tris.append([a, b, c, custom, mat])
    m = len(tris)
    n = 1
    while n < m:
        n *= 2
    q = deque([(0, n, 0)])
    while q:
        i, j, depth = q.popleft()
        lo, hi = i, min(j, m)
        if lo + 1 >= hi:
            continue
        axis = depth % 3
        keys = np.array([t[3][axis] for t in tris[lo:hi]], dtype=np.float32)
        order = np.argsort(keys, kind="stable")
        tris[lo:hi] = [tris[lo + k] for k in order]
        mid = (i + j) // 2
        q.append((i, mid, depth + 1))
        q.append((mid, j, depth + 1))
    nodes = np.empty((n, 2, 4), dtype=np.float32)
    nodes[:, 0, :] = FMAX
    nodes[:, 1, :] = -FMAX
    for i, t in enumerate(tris):
        j = (i + n) // 2
        while j > 0:
            for v in t[:3]:
                nodes[j, 0] = np.where(nodes[j, 0] < v, nodes[j, 0], v)
                nodes[j, 1] = np.where(nodes[j, 1] > v, nodes[j, 1], v)
            j //= 2
    for t in tris:
        t[3] = _normalize(_cross((t[1] - t[0])[:3], (t[2] - t[0])[:3]))
    return [n, m], nodes, tris
