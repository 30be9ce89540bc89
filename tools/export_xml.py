"""Write a bench configuration's procedural scene as XML + OBJ (scenes.XmlWorld),
the input of examples/path_tracer.  usage: python tools/export_xml.py OUT.xml [config=4]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pupiloptixlab_amd import scenes  # noqa: E402

out = sys.argv[1]
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 4
xw = scenes.XmlWorld()
scenes.sphere_field({3: 125, 4: 500}[cfg], 1920, 1080, 4, seed=1, world=xw)
print(xw.save(out))
