"""Host scene layer: mitsuba XML subset, world flattening, emitters, camera
(resource/scene.cpp, resource/xml/*, world/emitter.cpp, util/camera.cpp)."""
import os

import numpy as np
import pytest

from pupiloptixlab_amd import World, abi, scenes
from pupiloptixlab_amd import world as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TMP = os.path.join(ROOT, "gpurun_out", "test_scene")


def write(name, text):
    os.makedirs(TMP, exist_ok=True)
    p = os.path.join(TMP, name)
    with open(p, "w") as f:
        f.write(text)
    return p


def inst_matrix(d, i):
    m = np.eye(4, dtype=np.float32)
    m[:3] = np.array(d.instances[i].to_world, np.float32).reshape(3, 4)
    return m


def test_cornell_world_flattening():
    d = World().load_scene(scenes.cornell_xml(os.path.join(TMP, "cb.xml"), 256, 256, 4)).desc()
    assert (d.width, d.height, d.max_depth) == (256, 256, 4)
    assert d.num_instances == 8
    faces = sum(d.shapes[d.instances[i].shape].num_faces for i in range(8))
    assert faces == 36  # 6 rectangles x 2 + 2 cubes x 12
    assert d.num_area_emitters == 2
    e0, e1 = d.area_emitters[0], d.area_emitters[1]
    assert e0.type == abi.EMITTER_TRI_AREA
    # light: 0.235 x 0.19 scale of the [-1,1]^2 rectangle -> area 4*0.235*0.19, split in two triangles
    assert np.isclose(e0.area + e1.area, 4 * 0.235 * 0.19, rtol=1e-5)
    assert np.isclose(e0.select_probability + e1.select_probability, 1.0, rtol=1e-6)
    assert np.allclose(e0.nrm[0][:], [0, -1, 0], atol=1e-6)  # faces down
    assert d.instances[7].emitter_offset == 0 and d.instances[0].emitter_offset == -1
    # every Cornell bsdf is twosided diffuse
    for i in range(8):
        m = d.materials[d.instances[i].material]
        assert m.type == abi.MAT_DIFFUSE and m.twosided == 1


def test_defaults_refs_and_sensor_flip():
    p = write("s1.xml", """<scene version="3.0.0">
      <default name="w" value="40"/><default name="depth" value="7"/>
      <integrator type="path"><integer name="max_depth" value="$depth"/></integrator>
      <sensor type="perspective"><float name="fov" value="60"/><string name="fov_axis" value="y"/>
        <transform name="to_world"><matrix value="1 0 0 1  0 1 0 2  0 0 1 3  0 0 0 1"/></transform>
        <film type="hdrfilm"><integer name="width" value="$w"/><integer name="height" value="20"/></film>
      </sensor>
      <bsdf type="plastic" id="P"><float name="int_ior" value="bk7"/><boolean name="nonlinear" value="true"/></bsdf>
      <shape type="cube"><ref id="P"/></shape>
    </scene>""")
    d = World().load_scene(p).desc()
    assert (d.width, d.height, d.max_depth) == (40, 20, 7)
    c2w = np.array(d.camera_to_world).reshape(4, 4)
    # mitsuba +X left / +Z view -> Pupil convention: columns 0 and 2 negated (scene.cpp:132-139)
    assert np.allclose(c2w[:3, :3], np.diag([-1, 1, -1]))
    assert np.allclose(c2w[:3, 3], [1, 2, 3])
    m = d.materials[d.instances[0].material]
    assert m.type == abi.MAT_PLASTIC and m.nonlinear == 1
    assert np.isclose(m.int_ior, 1.5046) and np.isclose(m.ext_ior, 1.000277)  # named IOR + default
    assert np.allclose(list(m.tex[0].c0), 0.5) and np.allclose(list(m.tex[1].c0), 1.0)


def test_fov_axis_x_conversion():
    """scene.cpp:122-127: fov along x is converted to the vertical fov."""
    p = write("s2.xml", """<scene><sensor type="perspective"><float name="fov" value="90"/>
        <film type="hdrfilm"><integer name="width" value="200"/><integer name="height" value="100"/></film>
      </sensor><shape type="rectangle"><bsdf type="diffuse"/></shape></scene>""")
    d = World().load_scene(p).desc()
    s2c = np.array(d.sample_to_camera, np.float64).reshape(4, 4)
    fovy = 2 * np.degrees(np.arctan(np.tan(np.radians(45)) * 0.5))
    # sample (1, 0.5) -> camera direction with x/z = tan(fov_x / 2) * ..., check vertical extent
    top = s2c @ np.array([0.5, 1.0, 0, 1])
    top /= top[3]
    assert np.isclose(abs(top[1] / top[2]), np.tan(np.radians(fovy / 2)), rtol=1e-5)
    right = s2c @ np.array([1.0, 0.5, 0, 1])
    right /= right[3]
    assert np.isclose(abs(right[0] / right[2]), 1.0, rtol=1e-5)  # 90 deg horizontal


def test_transform_order_scale_rotate_translate():
    """util_loader.cpp:182-198: scale, then rotate, then translate, whatever the XML order."""
    p = write("s3.xml", """<scene><shape type="rectangle"><bsdf type="diffuse"/>
        <transform name="to_world"><translate value="0, 10, 0"/><rotate x="1" angle="90"/>
          <scale x="5" y="5"/></transform></shape></scene>""")
    d = World().load_scene(p).desc()
    ref = W.transform(scale=(5, 5, 1), rotate=((1, 0, 0), 90), translate=(0, 10, 0))
    assert np.allclose(inst_matrix(d, 0), ref, atol=1e-5)


def test_sphere_center_radius_and_emitter():
    p = write("s4.xml", """<scene><shape type="sphere"><point name="center" x="1" y="2" z="3"/>
        <float name="radius" value="0.5"/><bsdf type="diffuse"/>
        <emitter type="area"><rgb name="radiance" value="1, 2, 3"/></emitter></shape>
        <emitter type="constant"><rgb name="radiance" value="0.1"/></emitter></scene>""")
    d = World().load_scene(p).desc()
    assert d.shapes[d.instances[0].shape].kind == abi.SHAPE_SPHERE
    assert np.allclose(inst_matrix(d, 0), [[0.5, 0, 0, 1], [0, 0.5, 0, 2], [0, 0, 0.5, 3], [0, 0, 0, 1]])
    e = d.area_emitters[0]
    assert e.type == abi.EMITTER_SPHERE and np.isclose(e.radius, 0.5) and np.allclose(list(e.center), [1, 2, 3])
    assert np.isclose(e.area, 4 * np.pi * 0.25, rtol=1e-6)
    # one area + one env: each gets 1/2 (emitter.cpp:321-337)
    assert np.isclose(e.select_probability, 0.5) and np.isclose(d.env.contents.select_probability, 0.5)
    assert d.env.contents.type == abi.EMITTER_CONST_ENV and np.allclose(list(d.env.contents.color), 0.1)


def test_emitter_probability_proportional_to_power():
    """Weights = max(rgb) * area (emitter.cpp:73-101,169-222)."""
    wd = World()
    wd.set_film(8, 8, 2)
    rect = wd.add_builtin("rectangle")
    m = wd.add_material(W.diffuse(0.5))
    wd.add_instance(rect, m, W.transform(scale=(1, 1, 1)), emitter_radiance=(1.0, 3.0, 2.0))
    wd.add_instance(rect, m, W.transform(scale=(2, 2, 1), translate=(5, 0, 0)), emitter_radiance=(1.0, 1.0, 1.0))
    wd.set_sensor(45, np.eye(4))
    d = wd.desc()
    p = [d.area_emitters[i].select_probability for i in range(4)]
    # areas 2 and 8 per triangle, weights 3*2 and 1*8
    assert np.allclose(p, np.array([6, 6, 8, 8]) / 28, rtol=1e-6)
    assert d.instances[0].emitter_offset == 0 and d.instances[1].emitter_offset == 2


def test_obj_loader(tmp_path):
    obj = tmp_path / "quad.obj"
    obj.write_text("v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvt 0 0\nvt 1 0\nvt 1 1\nvt 0 1\nvn 0 0 1\n"
                   "f 1/1/1 2/2/1 3/3/1 4/4/1\n")
    p = tmp_path / "s.xml"
    p.write_text(f'<scene><shape type="obj"><string name="filename" value="{obj.name}"/>'
                 '<bsdf type="diffuse"/></shape></scene>')
    d = World().load_scene(str(p)).desc()
    s = d.shapes[d.instances[0].shape]
    assert s.num_faces == 2 and s.num_vertices == 6  # quad fan-triangulated, one vertex per corner
    assert bool(s.normals) and bool(s.texcoords)
    assert d.instances[0].flip_tex_coords == 1  # OBJ default (shape.cpp:138)


def test_obj_with_several_meshes_is_skipped(tmp_path):
    """assimp splits an OBJ into one mesh per object / material; the reference loads
    only single-mesh files (resource/shape.cpp:230-233) and skips the shape otherwise."""
    quad = "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\n"
    cases = {"two_objects": quad + "o a\nf 1 2 3\no b\nf 1 3 4\n",
             "two_materials": quad + "usemtl red\nf 1 2 3\nusemtl blue\nf 1 3 4\n",
             "one_object_one_material": quad + "o a\nusemtl red\nf 1 2 3\nf 1 3 4\n",
             "same_material_twice": quad + "usemtl red\nf 1 2 3\nusemtl red\nf 1 3 4\n"}
    faces = {}
    for name, text in cases.items():
        (tmp_path / f"{name}.obj").write_text(text)
        p = tmp_path / f"{name}.xml"
        p.write_text(f'<scene><shape type="obj"><string name="filename" value="{name}.obj"/>'
                     '<bsdf type="diffuse"/></shape><shape type="rectangle"><bsdf type="diffuse"/></shape></scene>')
        d = World().load_scene(str(p)).desc()
        faces[name] = [d.shapes[d.instances[i].shape].num_faces for i in range(d.num_instances)]
    assert faces["two_objects"] == [2] and faces["two_materials"] == [2]  # only the rectangle is left
    assert faces["one_object_one_material"] == [2, 2] and faces["same_material_twice"] == [2, 2]


def test_missing_file_is_io_error():
    with pytest.raises(abi.PupilError) as e:
        World().load_scene("/nonexistent/scene.xml")
    assert e.value.code == -4


def test_malformed_xml_is_reported():
    p = write("bad.xml", "<scene><shape type='cube'></scene>")
    with pytest.raises(abi.PupilError):
        World().load_scene(p)


def test_sphere_field_generator_counts():
    for n in (1, 27, 125):
        d = scenes.sphere_field(n, 32, 18, 4).desc()
        faces = sum(d.shapes[d.instances[i].shape].num_faces if d.shapes[d.instances[i].shape].kind == 0 else 1
                    for i in range(d.num_instances))
        assert faces == scenes.triangle_count(n)


def test_env_map_and_bitmap_textures_load(tmp_path):
    from pupiloptixlab_amd import abi, scenes

    p = scenes.textured_env_xml(str(tmp_path / "texenv.xml"), 64, 48, 5)
    d = World().load_scene(p).desc()
    assert d.env and d.env.contents.type == abi.EMITTER_ENV_MAP
    assert d.env.contents.radiance.width == 64 and d.env.contents.radiance.height == 32
    assert abs(d.env.contents.scale - 1.5) < 1e-7
    kinds = [(d.materials[i].tex[0].type, d.materials[i].tex[0].filter) for i in range(d.num_materials)]
    assert (abi.TEX_BITMAP, 0) in kinds and (abi.TEX_BITMAP, 1) in kinds
    assert any(d.materials[i].tex[1].type == abi.TEX_CHECKERBOARD for i in range(d.num_materials))


def test_xml_export_of_procedural_field_loads_identically(tmp_path):
    """scenes.XmlWorld writes a generator's scene as XML + OBJ (the example's input
    format); loading it renders bit-identically to the programmatic scene."""
    import oracle
    from pupiloptixlab_amd import scenes

    xw = scenes.XmlWorld()
    scenes.sphere_field(12, 48, 32, 4, seed=3, world=xw)
    path = xw.save(str(tmp_path / "field.xml"))
    a = scenes.sphere_field(12, 48, 32, 4, seed=3).desc()
    b = World().load_scene(path).desc()
    assert (a.num_instances, a.num_area_emitters) == (b.num_instances, b.num_area_emitters)
    ra = oracle.OracleScene(a).render(spp=2)["accum"]
    rb = oracle.OracleScene(b).render(spp=2)["accum"]
    assert np.array_equal(ra.view(np.uint32), rb.view(np.uint32))
