"""The C++ host layer (pupiloptixlab_amd/framework: System / Pass / BufferManager /
PTPass over the C ABI) and the headless example/path_tracer equivalent."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "pupil_path_tracer")
FW = os.path.join(ROOT, "pupiloptixlab_amd", "lib", "libpupil_framework.so")
TMP = os.path.join(ROOT, "gpurun_out", "test_scenes")


def _built():
    if not (os.path.exists(EXE) and os.path.exists(FW)):
        pytest.skip("C++ host layer not built (run __graft_entry__.build())")


def test_framework_exports_reference_names():
    _built()
    out = subprocess.run(["nm", "-DC", FW], capture_output=True, text=True, check=True).stdout
    for sym in ("Pupil::pt::PTPass::OnRun()", "Pupil::pt::PTPass::SetScene(Pupil::world::World*)",
                "Pupil::pt::PTPass::Inspector()", "Pupil::System::AddPass(Pupil::Pass*)",
                "Pupil::BufferManager::AllocBuffer(Pupil::BufferDesc const&)", "Pupil::Pass::Run()"):
        assert sym in out, sym


def test_example_usage_and_missing_scene():
    _built()
    r = subprocess.run([EXE], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr
    r = subprocess.run([EXE, os.path.join(TMP, "does_not_exist.xml"), "1"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 1  # logged, no exception, no crash


def _read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), dtype="<f4" if scale < 0 else ">f4")
    return data.reshape(h, w, 3)


@pytest.mark.gpu
def test_example_matches_python_pass_and_oracle():
    """4 frames of System::Run with PTPass == 4 OnRun calls of the Python pass == oracle, bit for bit."""
    _built()
    import oracle
    from pupiloptixlab_amd import World, scenes
    from pupiloptixlab_amd.pt_pass import PTPass

    os.makedirs(TMP, exist_ok=True)
    xml = scenes.cornell_xml(os.path.join(TMP, "cb_cpp.xml"), 64, 48, 4)
    out = os.path.join(TMP, "cb_cpp.pfm")
    r = subprocess.run([EXE, xml, "4", out], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    img = _read_pfm(out).reshape(-1, 3)

    desc = World().load_scene(xml).desc()
    pt = PTPass(device=0)
    pt.set_scene(desc)
    for _ in range(4):
        pt.on_run()
    py = pt.buffers.get("final result").cpu().numpy()[:, :3]
    pt.close_engine()
    assert np.array_equal(img, py)
    ref = oracle.OracleScene(desc).render(spp=4)["accum"][:, :3]
    assert np.array_equal(img, ref)


@pytest.mark.gpu
def test_example_denoised_output_matches_python_denoiser():
    """PUPIL_DENOISE=1: the example runs Pupil::optix::Denoiser (albedo + normal guides) on
    "final result" before saving; the image equals the Python Denoiser on the same frame."""
    _built()
    import torch
    from pupiloptixlab_amd import World, scenes
    from pupiloptixlab_amd.denoiser import Denoiser
    from pupiloptixlab_amd.pt_pass import PTPass

    os.makedirs(TMP, exist_ok=True)
    xml = scenes.cornell_xml(os.path.join(TMP, "cb_cpp_dn.xml"), 64, 48, 4)
    out = os.path.join(TMP, "cb_cpp_dn.pfm")
    r = subprocess.run([EXE, xml, "4", out], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PUPIL_DENOISE="1"))
    assert r.returncode == 0, r.stderr
    img = _read_pfm(out).reshape(-1, 3)

    desc = World().load_scene(xml).desc()
    pt = PTPass(device=0)
    pt.set_scene(desc)
    for _ in range(4):
        pt.on_run()
    final = pt.buffers.get("final result")
    dn = Denoiser(Denoiser.USE_ALBEDO | Denoiser.USE_NORMAL)
    dn.setup(64, 48, 0.5)
    res = torch.empty_like(final)
    dn.execute(final, res, albedo=pt.buffers.get("albedo"), normal=pt.buffers.get("normal"))
    torch.cuda.synchronize()
    py = res.cpu().numpy()[:, :3]
    noisy = final.cpu().numpy()[:, :3]
    pt.close_engine()
    dn.close()
    assert np.array_equal(img, py)
    assert not np.array_equal(img, noisy)


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_example_rccl_tile_gather_single_rank_matches():
    """The C++ drop-in's multi-GPU path (pupil/dist.h: tile-sharded render + RCCL
    send/recv gather + scatter into rank 0's "final result"), forced on one rank with
    PUPIL_DIST=1: the saved image equals the plain single-GPU run bit for bit, and the
    C++ framework really joined an RCCL communicator (librccl is loaded)."""
    _built()
    from pupiloptixlab_amd import scenes

    os.makedirs(TMP, exist_ok=True)
    xml = scenes.cornell_xml(os.path.join(TMP, "cb_dist.xml"), 80, 56, 4)  # ragged 32-px tiles
    plain, dist = os.path.join(TMP, "cb_plain.pfm"), os.path.join(TMP, "cb_dist.pfm")
    r = subprocess.run([EXE, xml, "3", plain], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, PUPIL_DIST="1", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_PORT=str(_free_port()))
    r = subprocess.run([EXE, xml, "3", dist], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(_read_pfm(plain), _read_pfm(dist))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_example_ranks_on_one_gpu_match_one_rank(world):
    """The C++ drop-in's rank != 0 code (PTPass::SetScene's compact tile buffers,
    FrameGather's send side) with `world` rank processes sharing this box's one GPU over the
    host-staged test transport (PUPIL_GATHER_TRANSPORT=host; RCCL refuses two ranks on one
    device): every rank renders its tiles of every OnRun, rank 0 gathers and scatters them, and
    its saved image equals the single-rank run bit for bit."""
    _built()
    from pupiloptixlab_amd import scenes

    os.makedirs(TMP, exist_ok=True)
    xml = scenes.cornell_xml(os.path.join(TMP, "cb_ranks.xml"), 80, 56, 4)  # ragged 32-px tiles
    plain, multi = os.path.join(TMP, "cb_ranks_1.pfm"), os.path.join(TMP, f"cb_ranks_{world}.pfm")
    r = subprocess.run([EXE, xml, "5", plain], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    port = str(_free_port())
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, PUPIL_GATHER_TRANSPORT="host", PUPIL_RCCL_NONCE=f"ranks-test-{port}")
        procs.append(subprocess.Popen([EXE, xml, "5", multi], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True, env=env))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e
    assert all("host-staged tile gather" in e for _, e in outs)
    assert np.array_equal(_read_pfm(plain).view(np.uint32), _read_pfm(multi).view(np.uint32))


def test_framework_links_rccl():
    _built()
    out = subprocess.run(["ldd", FW], capture_output=True, text=True, check=True).stdout
    assert "librccl" in out
    syms = subprocess.run(["nm", "-DC", FW], capture_output=True, text=True, check=True).stdout
    assert "Pupil::FrameGather::Gather(void const*, void*, ihipStream_t*)" in syms


def test_rccl_id_file_rejects_a_stale_launch(tmp_path, monkeypatch):
    """The C++ drop-in's RCCL id hand-over (framework/src/dist.cpp): a file left by another
    launch (a crashed run, another job on the same MASTER_PORT) carries another launch
    nonce and is never read as this launch's id; rank 0's write replaces it atomically;
    an incomplete file reads as absent; the default path is per launch."""
    _built()
    import ctypes as C

    lib = C.CDLL(FW)
    lib.pupil_dist_write_id_file.argtypes = [C.c_char_p, C.c_char_p, C.c_void_p]
    lib.pupil_dist_read_id_file.argtypes = [C.c_char_p, C.c_char_p, C.c_void_p]
    lib.pupil_dist_id_path.argtypes = [C.c_char_p, C.c_size_t]
    path = str(tmp_path / "pupil_rccl.id").encode()
    old, new = bytes(range(128)), bytes(reversed(range(128)))
    buf = C.create_string_buffer(128)
    assert lib.pupil_dist_read_id_file(path, b"launch-2", buf) == 0  # absent
    assert lib.pupil_dist_write_id_file(path, b"launch-1", old) == 0  # a crashed earlier launch
    assert lib.pupil_dist_read_id_file(path, b"launch-2", buf) == -1  # stale: rejected
    assert lib.pupil_dist_read_id_file(path, b"launch-1", buf) == 1 and buf.raw == old
    assert lib.pupil_dist_write_id_file(path, b"launch-2", new) == 0  # rank 0 of the new launch
    assert lib.pupil_dist_read_id_file(path, b"launch-2", buf) == 1 and buf.raw == new
    with open(path, "rb") as f:
        whole = f.read()
    with open(path, "wb") as f:  # torn file: nonce present, id cut short
        f.write(whole[:-10])
    assert lib.pupil_dist_read_id_file(path, b"launch-2", buf) == 0
    out = C.create_string_buffer(512)
    monkeypatch.delenv("PUPIL_RCCL_ID_FILE", raising=False)
    monkeypatch.setenv("MASTER_PORT", "29511")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "a")
    assert lib.pupil_dist_id_path(out, 512) == 0
    pa = out.value
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "b")
    assert lib.pupil_dist_id_path(out, 512) == 0
    assert pa.startswith(b"/tmp/pupil_rccl_29511_") and out.value != pa


def test_rccl_id_file_of_a_finished_writer_is_stale(tmp_path):
    """A file with this launch's nonce whose writer (on this host) no longer runs -- a crashed
    or finished earlier launch with the same launch environment -- is never used, however
    recently it was written; the live writer's file is accepted however long ago it was
    written (no wall clocks compared: ranks may start any time apart)."""
    _built()
    import ctypes as C
    import sys

    path = str(tmp_path / "pupil_rccl.id")
    code = ("import ctypes as C; lib = C.CDLL(%r); lib.pupil_dist_write_id_file.argtypes = [C.c_char_p, C.c_char_p, "
            "C.c_void_p]; assert lib.pupil_dist_write_id_file(%r, b'launch-x', bytes(128)) == 0" % (FW, path.encode()))
    subprocess.run([sys.executable, "-c", code], check=True)  # the writer exits
    lib = C.CDLL(FW)
    lib.pupil_dist_write_id_file.argtypes = [C.c_char_p, C.c_char_p, C.c_void_p]
    lib.pupil_dist_read_id_file.argtypes = [C.c_char_p, C.c_char_p, C.c_void_p]
    buf = C.create_string_buffer(128)
    assert lib.pupil_dist_read_id_file(path.encode(), b"launch-x", buf) == -1
    assert lib.pupil_dist_write_id_file(path.encode(), b"launch-x", bytes(range(128))) == 0  # this process: alive
    os.utime(path, (1, 1))  # an mtime decades old changes nothing
    assert lib.pupil_dist_read_id_file(path.encode(), b"launch-x", buf) == 1 and buf.raw == bytes(range(128))


def test_rccl_id_file_from_another_host_is_taken_only_when_recent(tmp_path):
    """On a shared filesystem (PUPIL_RCCL_ID_FILE) a writer on another host cannot be checked
    for liveness: its file is used only if written no earlier than 60 s before the reader
    started, so a file a crashed launch left long ago is not read."""
    _built()
    import ctypes as C
    import struct

    lib = C.CDLL(FW)
    lib.pupil_dist_read_id_file.argtypes = [C.c_char_p, C.c_char_p, C.c_void_p]
    path = tmp_path / "pupil_rccl.id"
    nonce, host, ident = b"launch-r", b"another-host.invalid", bytes(range(128))
    path.write_bytes(b"PUPILID2" + struct.pack("<I", len(nonce)) + nonce + struct.pack("<I", len(host)) + host +
                     struct.pack("<qQ", 12345, 678) + ident)
    buf = C.create_string_buffer(128)
    assert lib.pupil_dist_read_id_file(str(path).encode(), nonce, buf) == 1 and buf.raw == ident
    os.utime(path, (1, 1))  # written decades before this reader started: a stale launch's file
    assert lib.pupil_dist_read_id_file(str(path).encode(), nonce, buf) == -1


def test_rccl_id_path_agrees_across_differently_started_ranks():
    """Ranks of one launch compute the same id file whatever process started them: here one
    directly and one under a `timeout` wrapper (another parent process), as
    tools/gpu_cpp_ranks.sh starts them; another run id gives another file."""
    _built()
    import shutil
    import sys

    code = ("import ctypes as C; lib = C.CDLL(%r); out = C.create_string_buffer(512); "
            "lib.pupil_dist_id_path(out, 512); print(out.value.decode())" % FW)
    env = {k: v for k, v in os.environ.items() if k != "PUPIL_RCCL_ID_FILE" and k != "PUPIL_RCCL_NONCE"}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", WORLD_SIZE="2", TORCHELASTIC_RUN_ID="r1")
    direct = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    wrapped = subprocess.run([shutil.which("timeout"), "60", sys.executable, "-c", code], env=env,
                             capture_output=True, text=True, check=True)
    assert direct.stdout.strip() == wrapped.stdout.strip() != ""
    env["TORCHELASTIC_RUN_ID"] = "r2"
    other = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    assert other.stdout.strip() != direct.stdout.strip()


@pytest.mark.gpu
@pytest.mark.parametrize("instance", [5, 7])
def test_example_render_thread_updates_match_oracle(instance, tmp_path):
    """The reference's threading contract (system.cpp:93-106, pt_pass.cpp:39-57,216-218):
    System::RunAsync renders on its own thread while the main thread, three times, takes
    the render lock, moves one instance 4 times (RenderInstanceUpdate events) and the
    camera (CameraChange).  PTPass only records the moves and refits once at the top of its
    next OnRun: 12 updates cost 3 refits.  The frames accumulated since the last change
    equal the oracle's render of the final state bit for bit.  Instance 7 is the Cornell
    box's area light (its emitter table is rewritten in place as well)."""
    _built()
    import json

    import oracle
    from pupiloptixlab_amd import World, scenes

    os.makedirs(TMP, exist_ok=True)
    xml = scenes.cornell_xml(os.path.join(TMP, "cb_thread.xml"), 64, 48, 4)
    accum = str(tmp_path / "accum.f32")
    env = dict(os.environ, PUPIL_THREAD_TEST=f"4,3,{instance}", PUPIL_BENCH_ACCUM=accum)
    r = subprocess.run([EXE, xml], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["updates"] == 12 and rec["accel_refits"] == 3, rec
    n = rec["frames_accumulated"]
    assert n >= 2 and rec["frames_rendered"] > n
    w = World().load_scene(xml)
    w.set_instance_transform(instance, np.array(rec["to_world"], np.float32).reshape(4, 4))
    desc = w.desc()
    desc.camera_to_world[:] = [float(x) for x in rec["camera_to_world"]]
    ref = oracle.OracleScene(desc).render(spp=n)["accum"]
    got = np.fromfile(accum, np.float32).reshape(-1, 4)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), \
        f"{(got.view(np.uint32) != ref.view(np.uint32)).any(axis=1).sum()} pixels differ"
