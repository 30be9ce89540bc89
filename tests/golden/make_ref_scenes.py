"""Fixtures of the reference's own scene files (data/static/*.xml of vymv/PupilOptixLab).

Each XML is loaded by this repo's XML loader (pupiloptixlab_amd.World: the
mitsuba subset of resource/scene.cpp:27-227, shapes of resource/shape.cpp,
emitter tables of world/emitter.cpp:77-337) and the flattened scene is stored
as numbers (pupiloptixlab_amd.scene_io): meshes, material and instance records,
emitter tables, camera matrices.  The XML text itself is not kept.  The GPU
tests render these scenes without the reference tree.

usage (in a container with the reference mounted):
    python tests/golden/make_ref_scenes.py /root/reference/data/static
"""
import glob
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from pupiloptixlab_amd import World, scene_io  # noqa: E402


def main(src):
    out_dir = os.path.join(HERE, "ref_scenes")
    os.makedirs(out_dir, exist_ok=True)
    for path in sorted(glob.glob(os.path.join(src, "*.xml"))):
        name = os.path.splitext(os.path.basename(path))[0]
        desc = World().load_scene(path).desc()
        scene_io.save_desc(desc, os.path.join(out_dir, name + ".npz"))
        print(name, desc.width, desc.height, desc.max_depth, desc.num_instances, desc.num_area_emitters)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data/static")
