"""pupiloptixlab_amd — MI355X-native wavefront path tracer with the
PupilOptixLab path-tracer pass API (example/path_tracer).

Native code: ``lib/libpupil_pt.so`` (HIP kernels for gfx950 + the C++ scene
layer), driven through the C ABI in ``include/pupil_pt.h``.
"""
from .abi import PupilError, load_library  # noqa: F401
from .world import World  # noqa: F401

__all__ = ["World", "PupilError", "load_library"]
