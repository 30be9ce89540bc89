"""Benchmark / parity scenes (BASELINE.json configs).

* ``cornell_xml``       config 1: the reference's Cornell box (data/static/
  cornellbox.xml geometry: 6 rectangles + 2 cubes, light radiance (17,12,4)),
  written as mitsuba XML so the C++ XML loader is exercised.
* ``cornell_materials`` config 2: the Cornell box with ShortBox / TallBox and
  added spheres carrying the seven reference BSDF types (parameters of
  data/static/material_test.xml).
* ``sphere_field``      configs 3/4: procedural field of tessellated spheres
  (2,000 triangles each) over a floor, one rectangle area light.
* ``instanced_field``   config 5 geometry (instances of one sphere-field BLAS).

Geometry is generated with numpy's PCG64 from a fixed seed, so every rank of
a multi-GPU run builds the identical scene.
"""
from __future__ import annotations

import os

import numpy as np

from . import abi
from . import world as W

# data/static/cornellbox.xml transforms (row-major to_world of each shape)
CORNELL_SHAPES = [
    ("rectangle", "Floor", "0.725, 0.71, 0.68",
     "-4.37114e-008 1 4.37114e-008 0 0 -8.74228e-008 2 0 1 4.37114e-008 1.91069e-015 0 0 0 0 1"),
    ("rectangle", "Ceiling", "0.725, 0.71, 0.68",
     "-1 7.64274e-015 -1.74846e-007 0 8.74228e-008 8.74228e-008 -2 2 0 -1 -4.37114e-008 0 0 0 0 1"),
    ("rectangle", "BackWall", "0.725, 0.71, 0.68",
     "1.91069e-015 1 1.31134e-007 0 1 3.82137e-015 -8.74228e-008 1 -4.37114e-008 1.31134e-007 -2 -1 0 0 0 1"),
    ("rectangle", "RightWall", "0.14, 0.45, 0.091",
     "4.37114e-008 -1.74846e-007 2 1 1 3.82137e-015 -8.74228e-008 1 3.82137e-015 1 2.18557e-007 0 0 0 0 1"),
    ("rectangle", "LeftWall", "0.63, 0.065, 0.05",
     "-4.37114e-008 8.74228e-008 -2 -1 1 3.82137e-015 -8.74228e-008 1 0 -1 -4.37114e-008 0 0 0 0 1"),
    ("cube", "ShortBox", "0.725, 0.71, 0.68",
     "0.0851643 0.289542 1.31134e-008 0.328631 3.72265e-009 1.26563e-008 -0.3 0.3 -0.284951 0.0865363 "
     "5.73206e-016 0.374592 0 0 0 1"),
    ("cube", "TallBox", "0.725, 0.71, 0.68",
     "0.286776 0.098229 -2.29282e-015 -0.335439 -4.36233e-009 1.23382e-008 -0.6 0.6 -0.0997984 0.282266 "
     "2.62268e-008 -0.291415 0 0 0 1"),
]
CORNELL_LIGHT = ("0.235 -1.66103e-008 -7.80685e-009 -0.005 -2.05444e-008 3.90343e-009 -0.0893 1.98 "
                 "2.05444e-008 0.19 8.30516e-009 -0.03 0 0 0 1")
CORNELL_SENSOR = "-1 0 0 0 0 1 0 1 0 0 -1 6.8 0 0 0 1"


def cornell_xml(path: str, width=256, height=256, max_depth=4, bsdf_overrides=None, extra_shapes="") -> str:
    """Write the Cornell box scene (config 1) as mitsuba-3 XML and return its path.

    ``bsdf_overrides`` maps a shape id to an XML <bsdf> snippet (config 2)."""
    bsdf_overrides = bsdf_overrides or {}
    lines = [
        '<scene version="3.0.0">',
        f'  <default name="resx" value="{width}"/>',
        f'  <default name="resy" value="{height}"/>',
        f'  <default name="max_depth" value="{max_depth}"/>',
        '  <integrator type="path"><integer name="max_depth" value="$max_depth"/></integrator>',
        '  <sensor type="perspective">',
        '    <float name="fov" value="19.5"/>',
        f'    <transform name="to_world"><matrix value="{CORNELL_SENSOR}"/></transform>',
        '    <sampler type="independent"><integer name="sample_count" value="64"/></sampler>',
        '    <film type="hdrfilm"><integer name="width" value="$resx"/>'
        '<integer name="height" value="$resy"/><rfilter type="tent"/></film>',
        '  </sensor>',
    ]
    for kind, sid, refl, mat in CORNELL_SHAPES:
        bsdf = bsdf_overrides.get(sid) or (
            f'<bsdf type="twosided" id="{sid}BSDF"><bsdf type="diffuse">'
            f'<rgb name="reflectance" value="{refl}"/></bsdf></bsdf>')
        lines += [f'  <shape type="{kind}" id="{sid}">',
                  f'    <transform name="to_world"><matrix value="{mat}"/></transform>',
                  f'    {bsdf}', '  </shape>']
    lines += ['  <bsdf type="twosided" id="LightBSDF"><bsdf type="diffuse">'
              '<rgb name="reflectance" value="0, 0, 0"/></bsdf></bsdf>',
              '  <shape type="rectangle" id="Light">',
              f'    <transform name="to_world"><matrix value="{CORNELL_LIGHT}"/></transform>',
              '    <ref id="LightBSDF"/>',
              '    <emitter type="area"><rgb name="radiance" value="17, 12, 4"/></emitter>',
              '  </shape>', extra_shapes, '</scene>']
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        f.write("\n".join(lines))
    return path


# material_test.xml parameters (data/static/material_test.xml:30-114)
MATERIAL_BSDFS = {
    "dielectric": '<bsdf type="dielectric"><float name="int_ior" value="1.5"/>'
                  '<float name="ext_ior" value="1"/></bsdf>',
    "roughdielectric": '<bsdf type="roughdielectric"><float name="alpha" value="0.35"/>'
                       '<float name="int_ior" value="1.5"/><float name="ext_ior" value="1"/></bsdf>',
    "conductor": '<bsdf type="conductor"><rgb name="specular_reflectance" value="0.3, 0.3, 0.3"/>'
                 '<rgb name="eta" value="0.200438, 0.924033, 1.10221"/>'
                 '<rgb name="k" value="3.91295, 2.45285, 2.14219"/></bsdf>',
    "roughconductor": '<bsdf type="roughconductor"><float name="alpha" value="0.35"/>'
                      '<rgb name="specular_reflectance" value="0.3, 0.3, 0.3"/>'
                      '<rgb name="eta" value="0.200438, 0.924033, 1.10221"/>'
                      '<rgb name="k" value="3.91295, 2.45285, 2.14219"/></bsdf>',
    "plastic": '<bsdf type="plastic"><float name="int_ior" value="1.5"/><float name="ext_ior" value="1"/>'
               '<boolean name="nonlinear" value="false"/>'
               '<rgb name="diffuse_reflectance" value="0.647814, 0.647814, 0.647814"/></bsdf>',
    "roughplastic": '<bsdf type="roughplastic"><float name="alpha" value="0.35"/>'
                    '<float name="int_ior" value="1.5"/><float name="ext_ior" value="1"/>'
                    '<boolean name="nonlinear" value="false"/>'
                    '<rgb name="diffuse_reflectance" value="0.647814, 0.647814, 0.647814"/></bsdf>',
}


def cornell_materials_xml(path: str, width=1024, height=1024, max_depth=6) -> str:
    """Config 2: Cornell box whose boxes and five added spheres carry all seven BSDFs."""
    overrides = {"ShortBox": MATERIAL_BSDFS["roughconductor"], "TallBox": MATERIAL_BSDFS["plastic"]}
    spheres = []
    placements = [("dielectric", (-0.55, 0.25, 0.45), 0.22), ("roughdielectric", (0.0, 0.18, 0.62), 0.17),
                  ("conductor", (0.55, 0.78, 0.2), 0.17), ("roughplastic", (-0.3, 1.45, -0.4), 0.2),
                  ("roughconductor", (0.45, 1.55, -0.5), 0.15)]
    for i, (name, c, r) in enumerate(placements):
        spheres.append(f'  <shape type="sphere" id="sphere{i}"><point name="center" value="{c[0]}, {c[1]}, {c[2]}"/>'
                       f'<float name="radius" value="{r}"/>{MATERIAL_BSDFS[name]}</shape>')
    return cornell_xml(path, width, height, max_depth, overrides, "\n".join(spheres))


def uv_sphere(slices=40, stacks=26):
    """Tessellated unit sphere with 2*slices*(stacks-1) triangles (2,000 by default)."""
    verts, norms, uvs = [], [], []
    for i in range(stacks + 1):
        th = np.pi * i / stacks
        for j in range(slices + 1):
            ph = 2 * np.pi * j / slices
            p = (np.sin(th) * np.cos(ph), np.cos(th), np.sin(th) * np.sin(ph))
            verts.append(p)
            norms.append(p)
            uvs.append((j / slices, i / stacks))
    idx = []
    row = slices + 1
    for i in range(stacks):
        for j in range(slices):
            a, b = i * row + j, i * row + j + 1
            c, d = (i + 1) * row + j, (i + 1) * row + j + 1
            if i != 0:
                idx.append((a, c, b))
            if i != stacks - 1:
                idx.append((b, c, d))
    return (np.asarray(verts, np.float32), np.asarray(norms, np.float32), np.asarray(uvs, np.float32),
            np.asarray(idx, np.uint32))


def _field_geometry(num_spheres: int, seed: int, box=10.0):
    rng = np.random.Generator(np.random.PCG64(seed))
    # jittered grid keeps spheres non-overlapping at any count
    n = int(np.ceil(num_spheres ** (1.0 / 3.0)))
    cell = box / n
    cells = rng.permutation(n ** 3)[:num_spheres]
    centers, radii, albedo = [], [], []
    for c in cells:
        ix, iy, iz = c % n, (c // n) % n, c // (n * n)
        r = cell * rng.uniform(0.2, 0.4)
        jitter = (cell / 2 - r) * rng.uniform(-1, 1, 3)
        centers.append((np.array([ix, iy, iz]) + 0.5) * cell - box / 2 + jitter + np.array([0, box / 2, 0]))
        radii.append(r)
        albedo.append(rng.uniform(0.3, 0.8, 3))
    return np.asarray(centers), np.asarray(radii), np.asarray(albedo)


def sphere_field(num_spheres=500, width=1920, height=1080, max_depth=4, seed=1, slices=40, stacks=26,
                 merge=True, world=None, emissive_groups=0) -> W.World:
    """Configs 3/4: ``num_spheres`` x 2,000-triangle spheres (+2 floor, +2 light triangles).

    With ``merge`` the spheres are baked into one world-space mesh (one
    instance, like a single OBJ); otherwise one instance per sphere.  ``world``
    (e.g. an XmlWorld) receives the builder calls instead of a new World.
    ``emissive_groups`` (merged mode): that many of the 8 sphere groups become area
    emitters, one emitter per triangle (world/emitter.cpp:169-222), i.e. an
    emissive-mesh workload for NEE emitter selection."""
    wd = W.World() if world is None else world
    wd.set_film(width, height, max_depth)
    box = 10.0
    centers, radii, albedo = _field_geometry(num_spheres, seed, box)
    v, nrm, uv, idx = uv_sphere(slices, stacks)
    if merge:
        P, N, T, I = [], [], [], []
        base = 0
        mats = []
        for c, r in zip(centers, radii):
            P.append(v * r + c)
            N.append(nrm)
            T.append(uv)
            I.append(idx + base)
            base += len(v)
        # one material per sphere needs one instance per sphere; the merged
        # variant groups spheres into 8 albedo classes, one mesh each
        groups = np.arange(num_spheres) % 8
        for g in range(8):
            sel = np.nonzero(groups == g)[0]
            if sel.size == 0:
                continue
            pos = np.concatenate([P[k] for k in sel])
            nn = np.concatenate([N[k] for k in sel])
            tt = np.concatenate([T[k] for k in sel])
            off = np.cumsum([0] + [len(P[k]) for k in sel[:-1]])
            ii = np.concatenate([idx + o for o in off])
            s = wd.add_mesh(pos, ii, nn, tt)
            m = wd.add_material(W.diffuse(tuple(albedo[sel[0]])))
            if g < emissive_groups:
                wd.add_instance(s, m, emitter_radiance=(1.5 + 0.2 * g, 1.2, 0.9))
            else:
                wd.add_instance(s, m)
            mats.append(m)
    else:
        s = wd.add_mesh(v, idx, nrm, uv)
        for c, r, a in zip(centers, radii, albedo):
            m = wd.add_material(W.diffuse(tuple(a)))
            wd.add_instance(s, m, W.transform(scale=(r, r, r), translate=tuple(c)))
    _room_and_light(wd)
    return wd


def _room_and_light(wd: W.World):
    """Closed room (floor, ceiling, four walls: 12 triangles) so every camera and
    bounce ray hits geometry, a 3x3 area light under the ceiling, the camera."""
    rect = wd.add_builtin("rectangle")
    wall_m = wd.add_material(W.twosided(W.diffuse((0.6, 0.6, 0.6))))
    room = [((8, 12, 1), ((1, 0, 0), -90), (0, 0, 2)),     # floor      y = 0
            ((8, 12, 1), ((1, 0, 0), 90), (0, 14, 2)),     # ceiling    y = 14
            ((8, 7, 1), None, (0, 7, -10)),                # back wall  z = -10
            ((8, 7, 1), ((0, 1, 0), 180), (0, 7, 14)),     # front wall z = 14
            ((12, 7, 1), ((0, 1, 0), 90), (-8, 7, 2)),     # left wall  x = -8
            ((12, 7, 1), ((0, 1, 0), -90), (8, 7, 2))]     # right wall x = 8
    for sc, rot, tr in room:
        wd.add_instance(rect, wall_m, W.transform(scale=sc, rotate=rot, translate=tr))
    light_m = wd.add_material(W.twosided(W.diffuse((0.0, 0.0, 0.0))))
    wd.add_instance(rect, light_m, W.transform(scale=(3, 3, 1), rotate=((1, 0, 0), 90), translate=(0, 13.9, 0)),
                    emitter_radiance=(40.0, 38.0, 34.0))
    cam = W.look_at_mitsuba((0.0, 6.0, 13.0), (0.0, 4.6, 0.0), (0, 1, 0))
    wd.set_sensor(50.0, cam, fov_axis="y")


class XmlWorld:
    """Records the World-builder calls of a procedural scene and writes it as a
    mitsuba-style XML file plus one OBJ per mesh, the input format of the
    reference's example/path_tracer (System::SetScene(path)).  Matrices are
    written as exact float32 <matrix> values, so loading the XML gives the same
    scene description bit for bit.  Supports what the generators here use:
    meshes, the rectangle builtin, diffuse (+twosided) materials, area emitters
    and the perspective sensor."""

    RECT = -1

    def __init__(self):
        self.film = (256, 256, 4)
        self.sensor = None
        self.meshes, self.materials, self.instances = [], [], []

    def set_film(self, width, height, max_depth):
        self.film = (int(width), int(height), int(max_depth))

    def set_sensor(self, fov, to_world, fov_axis="x", near_clip=0.01, far_clip=10000.0):
        self.sensor = (float(fov), np.asarray(to_world, np.float32).reshape(16), fov_axis, near_clip, far_clip)

    def add_mesh(self, positions, indices, normals=None, texcoords=None):
        self.meshes.append((np.asarray(positions, np.float32).reshape(-1, 3),
                            np.asarray(indices, np.uint32).reshape(-1, 3),
                            None if normals is None else np.asarray(normals, np.float32).reshape(-1, 3),
                            None if texcoords is None else np.asarray(texcoords, np.float32).reshape(-1, 2)))
        return len(self.meshes) - 1

    def add_builtin(self, name):
        if name != "rectangle":
            raise ValueError("XmlWorld writes the rectangle builtin only")
        return self.RECT

    def add_material(self, m):
        if m.type != abi.MAT_DIFFUSE or m.tex[0].type != abi.TEX_RGB:
            raise ValueError("XmlWorld writes RGB diffuse materials only")
        self.materials.append((tuple(m.tex[0].c0), bool(m.twosided)))
        return len(self.materials) - 1

    def add_instance(self, shape, material, to_world=None, flip_normals=False, flip_tex_coords=False,
                     emitter_radiance=None):
        if flip_normals:
            raise ValueError("XmlWorld does not write flip_normals")
        m = np.eye(4, dtype=np.float32) if to_world is None else np.asarray(to_world, np.float32).reshape(4, 4)
        rad = None if emitter_radiance is None else tuple(float(x) for x in np.broadcast_to(emitter_radiance, 3))
        self.instances.append((shape, material, m, bool(flip_tex_coords), rad))
        return len(self.instances) - 1

    @staticmethod
    def _f(x):
        return "%.9g" % float(x)

    def save(self, path: str) -> str:
        import os

        root = os.path.dirname(os.path.abspath(path))
        os.makedirs(root, exist_ok=True)
        stem = os.path.splitext(os.path.basename(path))[0]
        f = self._f
        for k, (P, I, N, T) in enumerate(self.meshes):
            with open(os.path.join(root, f"{stem}_mesh{k}.obj"), "w") as fh:
                fh.write("".join(f"v {f(a)} {f(b)} {f(c)}\n" for a, b, c in P))
                if T is not None:
                    fh.write("".join(f"vt {f(a)} {f(b)}\n" for a, b in T))
                if N is not None:
                    fh.write("".join(f"vn {f(a)} {f(b)} {f(c)}\n" for a, b, c in N))
                J = I + 1
                if T is not None and N is not None:
                    fh.write("".join(f"f {a}/{a}/{a} {b}/{b}/{b} {c}/{c}/{c}\n" for a, b, c in J))
                elif N is not None:
                    fh.write("".join(f"f {a}//{a} {b}//{b} {c}//{c}\n" for a, b, c in J))
                else:
                    fh.write("".join(f"f {a} {b} {c}\n" for a, b, c in J))
        w, h, depth = self.film
        out = ['<scene version="3.0.0">', f'  <integrator type="path"><integer name="max_depth" value="{depth}"/></integrator>']
        if self.sensor is not None:
            fov, m, axis, nc, fc = self.sensor
            out += [f'  <sensor type="perspective"><float name="fov" value="{f(fov)}"/>'
                    f'<string name="fov_axis" value="{axis}"/><float name="near_clip" value="{f(nc)}"/>'
                    f'<float name="far_clip" value="{f(fc)}"/>',
                    '    <transform name="to_world"><matrix value="' + " ".join(f(x) for x in m) + '"/></transform>',
                    f'    <film type="hdrfilm"><integer name="width" value="{w}"/><integer name="height" value="{h}"/></film>',
                    '  </sensor>']
        for shape, mat, m, flip_tc, rad in self.instances:
            if shape == self.RECT:
                out.append('  <shape type="rectangle">')
            else:
                out.append(f'  <shape type="obj"><string name="filename" value="{stem}_mesh{shape}.obj"/>'
                           f'<boolean name="flip_tex_coords" value="{"true" if flip_tc else "false"}"/>')
            c, two = self.materials[mat]
            bsdf = f'<bsdf type="diffuse"><rgb name="reflectance" value="{f(c[0])}, {f(c[1])}, {f(c[2])}"/></bsdf>'
            out.append("    " + (f'<bsdf type="twosided">{bsdf}</bsdf>' if two else bsdf))
            out.append('    <transform name="to_world"><matrix value="' + " ".join(f(x) for x in m.reshape(-1)) +
                       '"/></transform>')
            if rad is not None:
                out.append(f'    <emitter type="area"><rgb name="radiance" value="{f(rad[0])}, {f(rad[1])}, '
                           f'{f(rad[2])}"/></emitter>')
            out.append("  </shape>")
        out.append("</scene>")
        with open(path, "w") as fh:
            fh.write("\n".join(out) + "\n")
        return path


def blas_mesh(num_spheres=125, seed=2, box=4.0, slices=40, stacks=26):
    """One object-space mesh of ``num_spheres`` 2,000-triangle spheres (config 3
    generator, centred at the origin): the 250k-triangle BLAS of config 5."""
    centers, radii, _ = _field_geometry(num_spheres, seed, box)
    centers = centers - np.array([0.0, box / 2, 0.0])
    v, nrm, uv, idx = uv_sphere(slices, stacks)
    P = np.concatenate([v * r + c for c, r in zip(centers, radii)])
    N = np.concatenate([nrm for _ in radii])
    T = np.concatenate([uv for _ in radii])
    I = np.concatenate([idx + k * len(v) for k in range(len(radii))])
    return P.astype(np.float32), I.astype(np.uint32), N.astype(np.float32), T.astype(np.float32)


def instanced_field(num_instances=40, width=3840, height=2160, max_depth=6, seed=2, spheres_per_blas=125,
                    slices=40, stacks=26, scale_range=None) -> W.World:
    """Config 5: ``num_instances`` instances of one 250k-triangle BLAS under random
    rigid transforms (seed 2), alternating rough dielectric (alpha 0.35) and rough
    plastic (alpha 0.35), material_test.xml parameters, inside the config-4 room.
    scale_range=(lo, hi) adds a random non-uniform scale per instance (tests)."""
    wd = W.World()
    wd.set_film(width, height, max_depth)
    pos, idx, nrm, uv = blas_mesh(spheres_per_blas, seed, 4.0, slices, stacks)
    blas = wd.add_mesh(pos, idx, nrm, uv)
    m_diel = wd.add_material(W.rough_dielectric(alpha=0.35, int_ior=1.5, ext_ior=1.0))
    m_plas = wd.add_material(W.rough_plastic(alpha=0.35, diffuse_reflectance=(0.647814, 0.647814, 0.647814),
                                             int_ior=1.5, ext_ior=1.0))
    rng = np.random.Generator(np.random.PCG64(seed))
    for k in range(num_instances):
        axis = rng.normal(size=3)
        axis /= np.linalg.norm(axis)
        angle = float(rng.uniform(0.0, 360.0))
        t = (float(rng.uniform(-5.0, 5.0)), float(rng.uniform(2.5, 11.5)), float(rng.uniform(-7.0, 8.0)))
        scale = (1.0, 1.0, 1.0)
        if scale_range is not None:
            scale = tuple(float(x) for x in rng.uniform(scale_range[0], scale_range[1], 3))
        wd.add_instance(blas, m_diel if k % 2 == 0 else m_plas,
                        W.transform(scale=scale, rotate=(tuple(axis), angle), translate=t))
    _room_and_light(wd)
    return wd


def triangle_count(num_spheres, slices=40, stacks=26):
    return num_spheres * 2 * slices * (stacks - 1) + 14


def _write_pfm(path: str, rgb: np.ndarray):
    """rgb: (h, w, 3) float32, row 0 = top (written bottom-up as PFM requires)."""
    h, w, _ = rgb.shape
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode())
        f.write(np.ascontiguousarray(rgb[::-1], dtype="<f4").tobytes())


def textured_env_xml(path: str, width=320, height=240, max_depth=5, seed=4, env_format="pfm",
                     tex_format="pfm") -> str:
    """Scene-input fidelity scene: an env-map emitter
    (rotated, scaled; world/emitter.cpp:107-149 CDF), bitmap textures with
    point and bilinear filtering and a to_uv scale (cuda/texture.cpp:60-102),
    a checkerboard, a small area light, open sky so the env map is seen and
    sampled.  The image files are written next to the XML: the env map as
    env_format ("pfm", "exr" or "hdr", the latter two by pupil_image_save), the
    bitmap as tex_format ("pfm", or "png" / "jpg" 8-bit through PIL)."""
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    rng = np.random.Generator(np.random.PCG64(seed))
    eh, ew = 32, 64
    yy, xx = np.mgrid[0:eh, 0:ew].astype(np.float32)
    env = np.stack([0.3 + 0.7 * (1 - yy / eh), 0.4 + 0.3 * np.sin(xx / ew * 6.283), 0.5 + 0.5 * yy / eh], -1)
    env[4:7, 40:44] = (30.0, 25.0, 18.0)  # a sun
    tex = rng.uniform(0.1, 0.9, (16, 16, 3)).astype(np.float32)
    env_file, tex_file = f"env.{env_format}", f"tex.{tex_format}"
    if env_format == "pfm":
        _write_pfm(os.path.join(d, env_file), env.astype(np.float32))
    else:
        import ctypes as C

        rgba = np.concatenate([env, np.ones((eh, ew, 1), np.float32)], -1).astype(np.float32)
        fmt = {"exr": 1, "hdr": 2}[env_format]
        abi.check(abi.load_library().pupil_image_save(os.path.join(d, env_file).encode(), ew, eh,
                                                      rgba.ctypes.data_as(abi.f32p), fmt))
    if tex_format == "pfm":
        _write_pfm(os.path.join(d, tex_file), tex)
    else:
        from PIL import Image

        Image.fromarray((tex * 255).astype(np.uint8), "RGB").save(os.path.join(d, tex_file), quality=90)
    lines = [
        '<scene version="3.0.0">',
        f'  <integrator type="path"><integer name="max_depth" value="{max_depth}"/></integrator>',
        '  <sensor type="perspective"><float name="fov" value="45"/><string name="fov_axis" value="y"/>',
        '    <transform name="to_world"><lookat origin="0, 2.2, 6" target="0, 0.8, 0" up="0, 1, 0"/></transform>',
        f'    <film type="hdrfilm"><integer name="width" value="{width}"/><integer name="height" value="{height}"/>'
        '</film>',
        '  </sensor>',
        f'  <emitter type="envmap"><string name="filename" value="{env_file}"/><float name="scale" value="1.5"/>',
        '    <transform name="to_world"><rotate y="1" angle="30"/></transform></emitter>',
        '  <shape type="rectangle"><transform name="to_world"><scale x="6" y="6" z="1"/>'
        '<rotate x="1" angle="-90"/></transform>',
        f'    <bsdf type="diffuse"><texture type="bitmap" name="reflectance"><string name="filename" value="{tex_file}"/>'
        '<string name="filter_type" value="nearest"/><transform name="to_uv"><scale x="3" y="3"/></transform>'
        '</texture></bsdf></shape>',
        '  <shape type="sphere"><point name="center" x="-1.2" y="1" z="0"/><float name="radius" value="1"/>',
        f'    <bsdf type="diffuse"><texture type="bitmap" name="reflectance"><string name="filename" value="{tex_file}"/>'
        '<string name="filter_type" value="bilinear"/></texture></bsdf></shape>',
        '  <shape type="sphere"><point name="center" x="1.2" y="0.8" z="0.3"/><float name="radius" value="0.8"/>',
        '    <bsdf type="roughplastic"><float name="alpha" value="0.2"/><float name="int_ior" value="1.5"/>'
        '<float name="ext_ior" value="1"/><texture type="checkerboard" name="diffuse_reflectance">'
        '<rgb name="color0" value="0.8, 0.2, 0.1"/><rgb name="color1" value="0.1, 0.2, 0.7"/>'
        '<transform name="to_uv"><scale x="4" y="4"/></transform></texture></bsdf></shape>',
        '  <shape type="rectangle"><transform name="to_world"><scale x="0.4" y="0.4" z="1"/>'
        '<rotate x="1" angle="90"/><translate x="0" y="3.5" z="1"/></transform>',
        '    <bsdf type="diffuse"><rgb name="reflectance" value="0, 0, 0"/></bsdf>',
        '    <emitter type="area"><rgb name="radiance" value="12, 11, 9"/></emitter></shape>',
        '</scene>',
    ]
    with open(path, "w") as f:
        f.write("\n".join(lines))
    return path
