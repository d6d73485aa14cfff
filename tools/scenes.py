"""Deterministic scene generators.

* ``write_avenger_proxy`` -- the reference renders ``data/6887_allied_avenger.obj``
  (pg1_embree.cpp:14), which is NOT in the reference repository (only its ``.mtl`` and
  textures are).  This writes an *avenger-proxy*: a LEGO-style spaceship OBJ with the real
  ``.mtl`` (5 materials), 94 groups (``Surfaces = 94`` in data/raytraced_avenger.png), the two
  decal textures, a closed faceted glass canopy (the only ``shader 4`` material) and studded
  wings, sized for the reference camera (tutorials.cpp:186-191).  Faces mix triangles and
  quads so the loader's quad split (objloader.cpp:455-471) is exercised.
* ``write_geosphere`` -- icosphere with ``data/sphere/geosphere.mtl`` (glass), the
  reference's second scene (pg1_embree.cpp:15, tutorials.cpp:194 camera).
* ``random_triangles`` -- BASELINE config C5: 10^6 triangles, vertices U(-100,100)^3
  (seed 42), edge length <= 2, 80 % Phong / 20 % dielectric.
"""
from __future__ import annotations

import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
AVENGER_DIR = os.path.join(ROOT, "assets", "avenger")
AVENGER_OBJ = os.path.join(AVENGER_DIR, "6887_allied_avenger_proxy.obj")
SPHERE_DIR = os.path.join(ROOT, "assets", "sphere")
SPHERE_OBJ = os.path.join(SPHERE_DIR, "geosphere_proxy.obj")

BLACK, GREEN, WHITE, ARROW, PANEL = (
    "black_plastic",
    "green_plastic_transparent",
    "white_plastic",
    "white_plastic_4150p04",
    "white_plastic_3069bp13",
)

STUD = 20.0  # LDraw units per stud pitch
PLATE = 8.0
BRICK = 24.0


class Mesh:
    """Indexed mesh grouped like a 3ds Max OBJ export: one ``g`` + ``usemtl`` per part."""

    def __init__(self):
        self.v: list = []
        self.vn: list = []
        self.vt: list = []
        self.groups: list = []  # (name, material, faces[list of list of (vi, ti, ni)])
        self.cur = None
        self.R = np.eye(3)
        self.T = np.zeros(3)
        self.scale = 1.0

    def group(self, name, material):
        self.cur = (name, material, [])
        self.groups.append(self.cur)

    def set_xform(self, R, T):
        self.R = np.asarray(R, dtype=np.float64)
        self.T = np.asarray(T, dtype=np.float64)

    def _vert(self, p, n, t=(0.0, 0.0)):
        p = self.scale * (self.R @ np.asarray(p, dtype=np.float64)) + self.T
        n = self.R @ np.asarray(n, dtype=np.float64)
        self.v.append(p)
        self.vn.append(n)
        self.vt.append(t)
        i = len(self.v)
        return (i, i, i)

    def face(self, verts):
        self.cur[2].append(verts)

    # --- primitives (local coordinates, then the current transform) ---
    def box(self, lo, hi):
        lo = np.asarray(lo, float)
        hi = np.asarray(hi, float)
        x0, y0, z0 = lo
        x1, y1, z1 = hi
        quads = [
            ([(x0, y0, z0), (x0, y1, z0), (x1, y1, z0), (x1, y0, z0)], (0, 0, -1)),
            ([(x0, y0, z1), (x1, y0, z1), (x1, y1, z1), (x0, y1, z1)], (0, 0, 1)),
            ([(x0, y0, z0), (x1, y0, z0), (x1, y0, z1), (x0, y0, z1)], (0, -1, 0)),
            ([(x0, y1, z0), (x0, y1, z1), (x1, y1, z1), (x1, y1, z0)], (0, 1, 0)),
            ([(x0, y0, z0), (x0, y0, z1), (x0, y1, z1), (x0, y1, z0)], (-1, 0, 0)),
            ([(x1, y0, z0), (x1, y1, z0), (x1, y1, z1), (x1, y0, z1)], (1, 0, 0)),
        ]
        for k, (pts, n) in enumerate(quads):
            vs = [self._vert(p, n) for p in pts]
            if k % 2 == 0:
                self.face(vs)  # quad: split by the loader into (0,1,2)+(0,2,3)
            else:
                self.face([vs[0], vs[1], vs[2]])
                self.face([vs[0], vs[2], vs[3]])

    def cylinder(self, c, r, h, seg, top=True, bottom=False, uv_disc=False, smooth=True):
        """Axis +Z from base centre c."""
        cx, cy, cz = c
        ang = [2 * math.pi * i / seg for i in range(seg)]
        ring0 = [(cx + r * math.cos(a), cy + r * math.sin(a), cz) for a in ang]
        ring1 = [(cx + r * math.cos(a), cy + r * math.sin(a), cz + h) for a in ang]
        for i in range(seg):
            j = (i + 1) % seg
            if smooth:
                ni = (math.cos(ang[i]), math.sin(ang[i]), 0.0)
                nj = (math.cos(ang[j]), math.sin(ang[j]), 0.0)
            else:
                am = 0.5 * (ang[i] + ang[i] + 2 * math.pi / seg)
                ni = nj = (math.cos(am), math.sin(am), 0.0)
            a = self._vert(ring0[i], ni)
            b = self._vert(ring0[j], nj)
            cc = self._vert(ring1[j], nj)
            d = self._vert(ring1[i], ni)
            self.face([a, b, cc])
            self.face([a, cc, d])
        if top:
            ctr_t = (0.5, 0.5)
            ctr = self._vert((cx, cy, cz + h), (0, 0, 1), ctr_t)
            for i in range(seg):
                j = (i + 1) % seg
                ti = (0.5 + 0.5 * math.cos(ang[i]), 0.5 + 0.5 * math.sin(ang[i])) if uv_disc else (0, 0)
                tj = (0.5 + 0.5 * math.cos(ang[j]), 0.5 + 0.5 * math.sin(ang[j])) if uv_disc else (0, 0)
                a = self._vert(ring1[i], (0, 0, 1), ti)
                b = self._vert(ring1[j], (0, 0, 1), tj)
                self.face([ctr, a, b])
        if bottom:
            ctr = self._vert((cx, cy, cz), (0, 0, -1))
            for i in range(seg):
                j = (i + 1) % seg
                a = self._vert(ring0[i], (0, 0, -1))
                b = self._vert(ring0[j], (0, 0, -1))
                self.face([ctr, b, a])

    def tube(self, c, r_out, r_in, h, seg):
        """Hollow anti-stud tube under a plate (open ends)."""
        self.cylinder(c, r_out, h, seg, top=False)
        cx, cy, cz = c
        ang = [2 * math.pi * i / seg for i in range(seg)]
        for i in range(seg):
            j = (i + 1) % seg
            ni = (-math.cos(ang[i]), -math.sin(ang[i]), 0.0)
            nj = (-math.cos(ang[j]), -math.sin(ang[j]), 0.0)
            p = lambda a, z: (cx + r_in * math.cos(a), cy + r_in * math.sin(a), z)
            a = self._vert(p(ang[i], cz), ni)
            b = self._vert(p(ang[j], cz), nj)
            cc = self._vert(p(ang[j], cz + h), nj)
            d = self._vert(p(ang[i], cz + h), ni)
            self.face([a, d, cc])
            self.face([a, cc, b])

    def lathe_x(self, xs, rs, seg):
        """Closed faceted solid of revolution about +X (flat facet normals)."""
        rings = []
        for x, r in zip(xs, rs):
            rings.append([(x, r * math.cos(2 * math.pi * i / seg + math.pi / seg),
                           r * math.sin(2 * math.pi * i / seg + math.pi / seg)) for i in range(seg)])
        def fn(a, b, c):
            a, b, c = map(np.asarray, (a, b, c))
            n = np.cross(b - a, c - a)
            ln = np.linalg.norm(n)
            return tuple(n / ln) if ln > 0 else (1.0, 0.0, 0.0)
        for k in range(len(rings) - 1):
            r0, r1 = rings[k], rings[k + 1]
            for i in range(seg):
                j = (i + 1) % seg
                n = fn(r0[i], r0[j], r1[j])
                vs = [self._vert(r0[i], n), self._vert(r0[j], n), self._vert(r1[j], n), self._vert(r1[i], n)]
                self.face([vs[0], vs[1], vs[2]])
                self.face([vs[0], vs[2], vs[3]])
        # caps
        for ring, sgn in ((rings[0], -1.0), (rings[-1], 1.0)):
            cx = ring[0][0]
            n = (sgn, 0.0, 0.0)
            ctr = self._vert((cx, 0.0, 0.0), n)
            for i in range(seg):
                j = (i + 1) % seg
                a = self._vert(ring[i], n)
                b = self._vert(ring[j], n)
                self.face([ctr, a, b] if sgn > 0 else [ctr, b, a])

    def sphere(self, c, r, seg=8, rings=6):
        cx, cy, cz = c
        for k in range(rings):
            t0 = math.pi * k / rings
            t1 = math.pi * (k + 1) / rings
            for i in range(seg):
                p0 = 2 * math.pi * i / seg
                p1 = 2 * math.pi * (i + 1) / seg
                def pt(t, p):
                    n = (math.sin(t) * math.cos(p), math.sin(t) * math.sin(p), math.cos(t))
                    return (cx + r * n[0], cy + r * n[1], cz + r * n[2]), n
                (a, na), (b, nb), (cc, nc), (d, nd) = pt(t0, p0), pt(t1, p0), pt(t1, p1), pt(t0, p1)
                va, vb, vc, vd = self._vert(a, na), self._vert(b, nb), self._vert(cc, nc), self._vert(d, nd)
                if k > 0:
                    self.face([va, vb, vc])
                if k < rings - 1:
                    self.face([va, vc, vd])

    def plate(self, nx, ny, x0, y0, z0, height=PLATE, studs=True, tubes=True, stud_seg=32):
        """LEGO plate/brick nx x ny studs with its lower-left corner at (x0, y0, z0)."""
        self.box((x0, y0, z0), (x0 + nx * STUD, y0 + ny * STUD, z0 + height))
        if studs:
            for i in range(nx):
                for j in range(ny):
                    self.cylinder((x0 + (i + 0.5) * STUD, y0 + (j + 0.5) * STUD, z0 + height), 6.0, 4.0,
                                  stud_seg, top=True)
        if tubes and nx > 1 and ny > 1:
            for i in range(nx - 1):
                for j in range(ny - 1):
                    self.tube((x0 + (i + 1) * STUD, y0 + (j + 1) * STUD, z0 - 0.0), 8.0, 6.0,
                              height - 1.0, stud_seg)

    def write(self, path, mtllib):
        with open(path, "w") as f:
            f.write("# avenger-proxy generated by tools/scenes.py (deterministic)\n")
            f.write(f"mtllib {mtllib}\n")
            for p in self.v:
                f.write(f"v {p[0]:.6f} {p[1]:.6f} {p[2]:.6f}\n")
            f.write(f"# {len(self.v)} vertices\n\n")
            for n in self.vn:
                f.write(f"vn {n[0]:.6f} {n[1]:.6f} {n[2]:.6f}\n")
            f.write(f"# {len(self.vn)} vertex normals\n\n")
            for t in self.vt:
                f.write(f"vt {t[0]:.6f} {t[1]:.6f} 0.000000\n")
            f.write(f"# {len(self.vt)} texture coords\n\n")
            for name, mat, faces in self.groups:
                f.write(f"g {name}\nusemtl {mat}\ns 1\n")
                for fc in faces:
                    f.write("f " + " ".join(f"{a}/{b}/{c}" for a, b, c in fc) + "\n")
                f.write(f"# {len(faces)} faces\n\n")


def _rot_z(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]])


def _rot_x(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[1.0, 0, 0], [0, c, -s], [0, s, c]])


def build_avenger_proxy(stud_seg: int = 32) -> Mesh:
    m = Mesh()
    # model built in LDraw units (stud pitch 20), exported at 0.4 -> millimetres (stud pitch 8,
    # the metric 3ds Max export the reference's objloader.h note asks for)
    m.scale = 0.62
    # ship frame: nose along +X_local; yaw so the nose points toward screen-right of the
    # reference camera (x_c = (0.78, -0.62, 0)), centred near the look-at point (0, 0, 40).
    yaw = math.atan2(-0.6247, 0.7809)
    base_R = _rot_z(yaw)
    base_T = np.array([0.0, 0.0, 40.0])

    def xf(R_local=np.eye(3), T_local=(0, 0, 0)):
        m.set_xform(base_R @ R_local, m.scale * (base_R @ np.asarray(T_local, float)) + base_T)

    n = 0

    def g(mat):
        nonlocal n
        n += 1
        m.group(f"part{n:03d}", mat)

    xf()
    # fuselage: stacked bricks and plates (black / white)
    g(BLACK); m.plate(8, 2, -100, -20, 0, height=BRICK, stud_seg=stud_seg)
    g(WHITE); m.plate(6, 2, -80, -20, BRICK, height=PLATE, stud_seg=stud_seg)
    g(BLACK); m.plate(4, 4, -60, -40, -PLATE, height=PLATE, stud_seg=stud_seg, studs=False)
    g(WHITE); m.plate(2, 2, 20, -20, BRICK, height=BRICK, stud_seg=stud_seg)
    g(BLACK); m.plate(2, 4, -120, -40, 0, height=BRICK, stud_seg=stud_seg)
    g(WHITE); m.plate(1, 2, -120, -20, BRICK, height=PLATE, stud_seg=stud_seg)
    g(BLACK); m.plate(2, 2, 40, -20, 0, height=BRICK, stud_seg=stud_seg)
    # decal panel tile on the fuselage top (3069bp13 is a 1x2 tile print)
    g(PANEL)
    m.box((-40, -10, BRICK + PLATE), (0, 10, BRICK + PLATE + 3.0))
    m.set_xform(base_R, m.scale * (base_R @ np.array([-20.0, 0.0, BRICK + PLATE + 3.0])) + base_T)
    vs = [m._vert((-20, -10, 0.05), (0, 0, 1), (0, 0)), m._vert((20, -10, 0.05), (0, 0, 1), (1, 0)),
          m._vert((20, 10, 0.05), (0, 0, 1), (1, 1)), m._vert((-20, 10, 0.05), (0, 0, 1), (0, 1))]
    m.face(vs)
    xf()
    # engines at the back (white cylinders along -X) with black nozzles
    for side in (-1, 1):
        R = np.array([[0, 0, -1.0], [0, 1, 0], [1, 0, 0]])  # +Z -> -X
        xf(R, (-120, side * 22, 14))
        g(WHITE); m.cylinder((0, 0, 0), 9.0, 30.0, stud_seg, top=True, bottom=True)
        xf(R, (-150, side * 22, 14))
        g(BLACK); m.cylinder((0, 0, 0), 6.0, 8.0, stud_seg, top=True, bottom=False)
    xf()
    # wings: studded plate rows, dihedral up on +Y, down on -Y (X-wing like silhouette)
    for side, dihedral in ((1, 0.95), (-1, -0.75)):
        for j in range(7):
            length = 9 - j
            R = _rot_x(dihedral if side > 0 else math.pi + dihedral)
            xf(R, (-110 - j * 10.0, 20.0 * side, 6.0))
            g(BLACK)
            m.plate(length, 1, 0, 20 + j * STUD - 20, 0, height=PLATE, stud_seg=stud_seg, tubes=False)
        # round decal tile (4150p04 arrow) near the wing tip
        xf(R, (-110 - 5 * 10.0, 20.0 * side, 6.0))
        g(ARROW)
        m.cylinder((40, 20 + 4 * STUD + 10, PLATE), 18.0, 3.2, 48, top=True, uv_disc=True)
    xf()
    # glass canopy: closed faceted solid at the nose, split into 4 groups
    xs = [55.0, 70.0, 95.0, 120.0, 140.0, 152.0]
    rs = [22.0, 40.0, 46.0, 44.0, 32.0, 12.0]
    xf(np.eye(3), (0, 0, 20))
    for _ in range(4):
        g(GREEN)
    # build the canopy once, then distribute its faces over the 4 groups
    start_group = len(m.groups) - 4
    keep = m.cur
    m.cur = ("tmp", GREEN, [])
    m.lathe_x(xs, rs, 8)
    for k, fc in enumerate(m.cur[2]):
        m.groups[start_group + (k % 4)][2].append(fc)
    m.cur = keep
    # cockpit interior (seen through the glass)
    xf()
    g(BLACK); m.plate(2, 2, 70, -20, 0, height=BRICK, stud_seg=stud_seg)
    g(WHITE); m.plate(1, 2, 90, -20, BRICK, height=BRICK, stud_seg=stud_seg)
    # antennas: transparent green rods with spherical tips
    for side in (-1, 1):
        xf(np.eye(3), (-30 - 25 * (side > 0), side * 12, BRICK + PLATE))
        g(GREEN); m.cylinder((0, 0, 0), 1.6, 95.0, 12, top=True, bottom=True)
        g(GREEN); m.sphere((0, 0, 97.0), 3.0, 10, 6)
    # greebles until 94 groups: small bricks/plates on the fuselage and wing roots
    rng = np.random.default_rng(6887)
    mats = [BLACK, WHITE, BLACK, WHITE, BLACK]
    while n < 94:
        xf()
        nx_, ny_ = int(rng.integers(1, 3)), int(rng.integers(1, 3))
        x0 = float(rng.integers(-7, 2)) * STUD
        y0 = float(rng.integers(-2, 1)) * STUD
        z0 = float(rng.choice([-PLATE * 2, -PLATE * 3, BRICK + 2 * PLATE]))
        h = float(rng.choice([PLATE, BRICK]))
        g(mats[n % 5])
        m.plate(nx_, ny_, x0, y0, z0, height=h, stud_seg=stud_seg)
    return m


def write_avenger_proxy(path: str = AVENGER_OBJ, stud_seg: int = 32) -> str:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    m = build_avenger_proxy(stud_seg)
    assert len(m.groups) == 94, len(m.groups)
    m.write(path, "6887_allied_avenger.mtl")
    return path


def write_geosphere(path: str = SPHERE_OBJ, subdiv: int = 3, radius: float = 1.0) -> str:
    """Icosphere with per-vertex smooth normals, one group, material wire_214229166."""
    t = (1.0 + 5 ** 0.5) / 2.0
    verts = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
             (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    verts = [np.array(v, float) / np.linalg.norm(v) for v in verts]
    faces = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2),
             (10, 7, 6), (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5),
             (2, 4, 11), (6, 2, 10), (8, 6, 7), (9, 8, 1)]
    for _ in range(subdiv):
        cache = {}
        nf = []

        def mid(a, b):
            key = (min(a, b), max(a, b))
            if key not in cache:
                p = verts[a] + verts[b]
                verts.append(p / np.linalg.norm(p))
                cache[key] = len(verts) - 1
            return cache[key]

        for a, b, c in faces:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        faces = nf
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write("# geosphere-proxy generated by tools/scenes.py\nmtllib geosphere.mtl\n")
        for v in verts:
            p = v * radius
            f.write(f"v {p[0]:.6f} {p[1]:.6f} {p[2]:.6f}\n")
        for v in verts:
            f.write(f"vn {v[0]:.6f} {v[1]:.6f} {v[2]:.6f}\n")
        for v in verts:
            f.write(f"vt {0.5 + 0.5 * v[0]:.6f} {0.5 + 0.5 * v[1]:.6f} 0.0\n")
        f.write("g GeoSphere001\nusemtl wire_214229166\n")
        for a, b, c in faces:
            f.write(f"f {a+1}/{a+1}/{a+1} {b+1}/{b+1}/{b+1} {c+1}/{c+1}/{c+1}\n")
    return path


def random_triangles(n: int = 1_000_000, seed: int = 42, n_materials: int = 100):
    """C5 synthetic soup: returns (positions 9N, normals 9N, uvs 6N, material_ids N, materials)."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(-100.0, 100.0, size=(n, 1, 3))
    d = rng.normal(size=(n, 3, 3))
    d /= np.linalg.norm(d, axis=2, keepdims=True)
    d *= rng.uniform(0.3, 1.0, size=(n, 3, 1))  # |offset| <= 1 -> edges <= 2
    p = (c + d).astype(np.float32)
    e1 = p[:, 1] - p[:, 0]
    e2 = p[:, 2] - p[:, 0]
    ng = np.cross(e1, e2)
    ng /= np.maximum(np.linalg.norm(ng, axis=1, keepdims=True), 1e-30)
    nrm = np.repeat(ng[:, None, :], 3, axis=1).astype(np.float32)
    uv = np.zeros((n, 3, 2), np.float32)
    n_dielectric = n_materials // 5
    mats = []
    for i in range(n_materials):
        if i < n_materials - n_dielectric:
            kd = rng.uniform(0.0, 1.0, size=3)
            mats.append(dict(diffuse=kd, specular=(0.8, 0.8, 0.8), shininess=32.0, ior=1.5, type=3, tex=-1))
        else:
            mats.append(dict(diffuse=(0.85, 1.0, 0.6), specular=(0.8, 0.8, 0.8), shininess=32.0, ior=1.5,
                             type=4, tex=-1))
    mat_ids = rng.integers(0, n_materials, size=n).astype(np.int32)
    return (np.ascontiguousarray(p.reshape(-1)), np.ascontiguousarray(nrm.reshape(-1)),
            np.ascontiguousarray(uv.reshape(-1)), mat_ids, mats)


def random_scene(n: int = 1_000_000, seed: int = 42, env_map: str | None = None):
    """C5 as a pgi_raytracing_amd Scene: the soup above, the reference light, optional env map."""
    from pgi_raytracing_amd.scene import LightData, MaterialData, Scene

    pos, nrm, uv, mids, mats = random_triangles(n, seed)
    md = [MaterialData(name=f"m{i}", diffuse=tuple(float(x) for x in m["diffuse"]),
                       specular=tuple(float(x) for x in m["specular"]), shininess=m["shininess"], ior=m["ior"],
                       type=m["type"]) for i, m in enumerate(mats)]
    sc = Scene(pos, nrm, uv, mids, md, [], -1, [LightData()])
    if env_map:
        sc.set_environment(env_map)
    return sc


if __name__ == "__main__":
    print(write_avenger_proxy())
    print(write_geosphere())
