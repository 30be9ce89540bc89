"""Host-side checks of the BVH4 leaf-link limits (csrc/accel_limits.h): the
two-level build must refuse or fall back before a 28-bit record slot wraps into the sign
bit of a leaf link.  Compiled with g++ (no GPU)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "pupiloptixlab_amd", "csrc")

PROG = r"""
#include <cstdio>
#include "accel_limits.h"
#include <initializer_list>
using namespace pupil;
int main() {
    const uint64_t L = kMaxLeafFirst;
    int bad = 0;
    auto expect = [&](bool c, const char *what) { if (!c) { std::printf("FAIL %s\n", what); bad++; } };
    expect(two_level_fit(L - 1, L - 1, 0, 1, true) == TwoLevelFit::World, "world at the last slot");
    expect(two_level_fit(L - 1, L, 0, 1, true) == TwoLevelFit::Object, "world slots past the limit");
    // world mode: the meshes' world slots, then one 2-slot leaf per sphere, all below the limit
    expect(two_level_fit(10, L - 3, 1, 2, true) == TwoLevelFit::World, "one sphere leaf below the limit");
    expect(two_level_fit(10, L - 2, 1, 2, true) == TwoLevelFit::Object, "one sphere leaf reaching the limit");
    expect(two_level_fit(10, L - 4, 2, 2, true) == TwoLevelFit::Object, "two sphere leaves reaching the limit");
    expect(two_level_fit(10, L - 5, 2, 2, true) == TwoLevelFit::World, "two sphere leaves below the limit");
    expect(two_level_fit(10, L - 3, 1, 2, false) == TwoLevelFit::Object, "object mode requested");
    expect(two_level_fit(L, 0, 0, 1, true) == TwoLevelFit::None, "object slots past the limit");
    expect(two_level_fit(1, 1, 0, L, true) == TwoLevelFit::None, "instances past the limit");
    // the encoding itself: every first below the limit gives a negative link that decodes back
    for (uint64_t f : {(uint64_t)0, (uint64_t)1, L / 2, L - 1})
        for (uint32_t c = 1; c <= 8; c++) {
            const int link = make_leaf((uint32_t)f, c);
            expect(link < 0 && leaf_first(link) == f && leaf_count(link) == c, "round trip");
        }
    // ... and the first slot past it would not (the wrap the limit prevents)
    expect(make_leaf((uint32_t)L, 1) >= 0, "wrap past the limit");
    return bad;
}
"""


def test_two_level_leaf_link_limits(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(PROG)
    exe = tmp_path / "t"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-I", CSRC, str(src), "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
