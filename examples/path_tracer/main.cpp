// examples/path_tracer/main.cpp — headless counterpart of the reference's
// example/path_tracer/main.cpp: System + PTPass + an XML scene, rendered for
// a fixed number of frames (the reference loops until the window closes),
// then "final result" is written with pupil_image_save (.exr / .hdr like
// util::BitmapTexture::Save, or .pfm).
//
// usage: pupil_path_tracer <scene.xml> [frames=16] [out.exr|.hdr|.pfm] [device=0]
//        PUPIL_BENCH=warmup,frames,spp pupil_path_tracer <scene.xml>   (drop-in cadence benchmark)
#include <algorithm>
#include <chrono>
#include <string>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include "pupil/denoiser.h"
#include "pupil/framework.h"
#include "pupil/pt_pass.h"

// PUPIL_BENCH="warmup,frames,spp": the drop-in cadence of the reference
// (pt_pass.cpp:39-57): a frame is `spp` x System::Run(1), i.e. spp x PTPass::OnRun
// of 1 spp each with its stream synchronisation, and the frames continue one
// progressive render (accumulation restarts once, through a CameraChange event, as
// when the user stops moving the camera).  `warmup` untimed and `frames` timed frames
// (steady_clock around the loop); the rays are the engine's exact running total over
// the timed OnRuns.  Every timed OnRun is also timed on its own (steady_clock around
// System::Run(1), whose OnRun ends in a stream synchronisation): the line reports the
// p50 / p99 / max OnRun time -- with frame groups one OnRun in G carries the traversal of G
// frames and the others only accumulate (System::Run -> FrameFinished shows each one,
// system.cpp:95-101).  PUPIL_BENCH_ACCUM=<file>: the final "pt accum buffer" (rank 0,
// raw float32 RGBA) for a bit-exact comparison with a batched render of the same
// seeds.  PUPIL_BENCH_MOVING=1: the interactive cadence instead -- the camera moves
// (CameraHelper::SetCameraToWorld, a CameraChange) before every OnRun, so every frame
// restarts accumulation and no render continues the previous one.  Prints one JSON line.
static double pct(std::vector<double> v, double q) {
    if (v.empty()) return 0.0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(q * (double)v.size()))];
}

static int Bench(Pupil::System &system, Pupil::pt::PTPass &pass, const char *spec) {
    int warmup = 1, frames = 5, spp = 8;
    if (std::sscanf(spec, "%d,%d,%d", &warmup, &frames, &spp) != 3 || frames < 1 || spp < 1 || warmup < 0) {
        std::fprintf(stderr, "PUPIL_BENCH must be warmup,frames,spp\n");
        return 2;
    }
    Pupil::EventDispatcher<Pupil::EWorldEvent::CameraChange>();
    const char *mv = std::getenv("PUPIL_BENCH_MOVING");
    const bool moving = mv && std::atoi(mv);
    Pupil::world::World *w = system.GetWorld();
    float s2c[16], c2w[16];
    w->camera->Snapshot(s2c, c2w);
    uint32_t step = 0;
    std::vector<double> onrun_ms;
    bool timed = false;
    auto frame = [&]() {
        for (int j = 0; j < spp; j++) {
            if (moving) {  // a camera move before every OnRun
                float c[16];
                std::memcpy(c, c2w, sizeof(c));
                c[3] += 1e-4f * (float)(++step);
                w->camera->SetCameraToWorld(c);
            }
            const auto a = std::chrono::steady_clock::now();
            system.Run(1);
            if (timed) onrun_ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count());
        }
    };
    for (int k = 0; k < warmup; k++) frame();
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    pupil_pt_counters c0{}, c1{};
    if (!pass.Stats(c0)) return 1;
    timed = true;
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < frames; k++) frame();
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!pass.Stats(c1)) return 1;
    const double rays = (double)(c1.rays_traced_total - c0.rays_traced_total);
    Pupil::FrameGather *g = system.Gather();
    if (g && g->Info().rank != 0) return 0;
    if (const char *path = std::getenv("PUPIL_BENCH_ACCUM")) {
        auto *buf = Pupil::BufferManager::instance()->GetBuffer("pt accum buffer");
        const size_t n = buf ? (size_t)buf->desc.width * buf->desc.height * 4 : 0;
        std::vector<float> host(n);
        if (!buf || hipMemcpy(host.data(), buf->cuda_ptr, n * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
            return 1;
        FILE *f = std::fopen(path, "wb");
        if (!f || std::fwrite(host.data(), sizeof(float), n, f) != n) {
            if (f) std::fclose(f);
            return 1;
        }
        std::fclose(f);
    }
    std::printf("{\"ms_per_frame\": %.4f, \"onrun_ms\": %.4f, \"onrun_ms_p50\": %.4f, \"onrun_ms_p99\": %.4f, "
                "\"onrun_ms_max\": %.4f, \"mrays_per_s_rank0\": %.2f, \"rays_per_frame_rank0\": %.0f, "
                "\"frames\": %d, \"warmup\": %d, \"spp\": %d, \"ranks\": %d, \"frames_in_flight\": %llu, "
                "\"moving_camera\": %s, \"ring_bytes\": %llu}\n",
                1e3 * s / frames, 1e3 * s / (frames * spp), pct(onrun_ms, 0.5), pct(onrun_ms, 0.99), pct(onrun_ms, 1.0),
                rays / s / 1e6, rays / frames, frames, warmup, spp, g ? g->Info().world : 1,
                (unsigned long long)c1.frames_in_flight, moving ? "true" : "false", (unsigned long long)c1.ring_bytes);
    return 0;
}

// PUPIL_BENCH_WASTE="k1,k2,...": what speculation costs when the camera moves.  For each k: a
// camera change, k static OnRuns (the engine pipelines frames ahead once the OnRuns continue
// each other), then another camera change, which drops the frames in flight.  Prints the rays
// traced over each static stretch (engine running totals) and the frames in flight that the
// move dropped; the same run with PUPIL_AHEAD=0 traces exactly the displayed frames' rays, so
// the difference of the two is the speculation the move discarded.
static int BenchWaste(Pupil::System &system, Pupil::pt::PTPass &pass, const char *spec) {
    std::vector<int> ks;
    for (const char *p = spec; *p;) {
        ks.push_back(std::atoi(p));
        while (*p && *p != ',') p++;
        if (*p == ',') p++;
    }
    Pupil::world::World *w = system.GetWorld();
    float s2c[16], c2w[16];
    w->camera->Snapshot(s2c, c2w);
    uint32_t step = 0;
    auto move = [&]() {
        float c[16];
        std::memcpy(c, c2w, sizeof(c));
        c[3] += 1e-4f * (float)(++step);
        w->camera->SetCameraToWorld(c);
    };
    std::string out = "{\"waste\": [";
    for (size_t i = 0; i < ks.size(); i++) {
        move();
        pupil_pt_counters a{}, b{};
        if (!pass.Stats(a)) return 1;
        std::vector<double> ms;
        for (int j = 0; j < ks[i]; j++) {
            const auto t0 = std::chrono::steady_clock::now();
            system.Run(1);
            ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        }
        if (hipDeviceSynchronize() != hipSuccess || !pass.Stats(b)) return 1;
        char rec[256];
        std::snprintf(rec, sizeof(rec), "%s{\"k\": %d, \"rays\": %llu, \"frames_dropped_by_move\": %llu, \"onrun_ms_max\": %.3f",
                      i ? ", " : "", ks[i], (unsigned long long)(b.rays_traced_total - a.rays_traced_total),
                      (unsigned long long)b.frames_in_flight, pct(ms, 1.0));
        out += rec;
        // the first OnRuns after the move, one by one (where the pipeline refills)
        out += ", \"onrun_ms_first\": [";
        for (size_t j = 0; j < ms.size() && j < 12; j++) {
            std::snprintf(rec, sizeof(rec), "%s%.3f", j ? ", " : "", ms[j]);
            out += rec;
        }
        out += "]}";
    }
    move();
    system.Run(1);  // the last stretch's frames in flight are dropped here
    std::printf("%s]}\n", out.c_str());
    return 0;
}

// PUPIL_THREAD_TEST="k,rounds[,instance]": the reference's threading (system.cpp:93-106):
// System::RunAsync renders on its own thread while this thread, `rounds` times, takes the
// render lock, moves `instance` k times (each a RenderInstanceUpdate) and moves the camera
// (a CameraChange), then lets a few frames render.  Afterwards the render thread is
// stopped and one JSON line reports the final instance / camera matrices, the frames
// accumulated since the last change, the acceleration refits (one per round expected:
// PTPass refits once per OnRun however many updates it was sent) and the final
// "pt accum buffer" (PUPIL_BENCH_ACCUM file) for a comparison with the oracle.
static int ThreadTest(Pupil::System &system, Pupil::pt::PTPass &pass, const char *spec) {
    int k = 4, rounds = 3, inst = 0;
    if (std::sscanf(spec, "%d,%d,%d", &k, &rounds, &inst) < 2 || k < 1 || rounds < 1) return 2;
    Pupil::world::World *w = system.GetWorld();
    if (inst < 0 || (uint32_t)inst >= w->Desc().num_instances) return 2;
    float base[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1};
    std::memcpy(base, w->Desc().instances[inst].to_world, 12 * sizeof(float));
    float s2c[16], cam[16];
    w->camera->Snapshot(s2c, cam);
    int updates = 0;
    float m[16], c[16];
    system.RunAsync();
    auto wait_frames = [&](uint64_t n) {
        const uint64_t f0 = system.FramesRendered();
        while (system.FramesRendered() < f0 + n) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    };
    wait_frames(3);
    for (int r = 1; r <= rounds; r++) {
        {
            auto lock = system.RenderLock();
            for (int j = 1; j <= k; j++) {  // absolute moves: the last one of the round stays
                std::memcpy(m, base, sizeof(m));
                m[3] += 0.01f * (float)((r - 1) * k + j);
                m[7] += 0.005f * (float)j;
                w->SetInstanceTransform((uint32_t)inst, m);
                updates++;
            }
            std::memcpy(c, cam, sizeof(c));
            c[3] += 0.002f * (float)r;  // camera position x
            w->camera->SetCameraToWorld(c);
        }
        wait_frames(2 + (uint64_t)r);
    }
    system.Stop();
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    pupil_pt_counters cnt{};
    if (!pass.Stats(cnt)) return 1;
    if (const char *path = std::getenv("PUPIL_BENCH_ACCUM")) {
        auto *buf = Pupil::BufferManager::instance()->GetBuffer("pt accum buffer");
        const size_t n = buf ? (size_t)buf->desc.width * buf->desc.height * 4 : 0;
        std::vector<float> host(n);
        FILE *f = nullptr;
        if (!buf || hipMemcpy(host.data(), buf->cuda_ptr, n * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess ||
            !(f = std::fopen(path, "wb")) || std::fwrite(host.data(), sizeof(float), n, f) != n) {
            if (f) std::fclose(f);
            return 1;
        }
        std::fclose(f);
    }
    std::printf("{\"updates\": %d, \"rounds\": %d, \"accel_refits\": %llu, \"frames_rendered\": %llu, "
                "\"frames_accumulated\": %u, \"instance\": %d, \"to_world\": [",
                updates, rounds, (unsigned long long)cnt.accel_refits, (unsigned long long)system.FramesRendered(),
                pass.SampleCount(), inst);
    for (int i = 0; i < 16; i++) std::printf("%s%.9g", i ? ", " : "", m[i]);
    std::printf("], \"camera_to_world\": [");
    for (int i = 0; i < 16; i++) std::printf("%s%.9g", i ? ", " : "", c[i]);
    std::printf("]}\n");
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <scene.xml> [frames=16] [out.exr|.hdr|.pfm] [device=0]\n", argv[0]);
        return 2;
    }
    const int frames = argc > 2 ? std::atoi(argv[2]) : 16;
    const char *out = argc > 3 ? argv[3] : "";
    auto system = Pupil::util::Singleton<Pupil::System>::instance();
    system->device = argc > 4 ? std::atoi(argv[4]) : 0;
    // multi-GPU (pupil/dist.h): one process per GPU with torchrun's RANK / WORLD_SIZE /
    // LOCAL_RANK; PUPIL_DIST=1 forces the RCCL path for a single rank
    const Pupil::DistInfo dist = Pupil::DistFromEnv();
    const char *force = std::getenv("PUPIL_DIST");
    if ((dist.world > 1 || (force && std::atoi(force))) && !system->InitDistributed(dist)) {
        std::fprintf(stderr, "rank %d: RCCL initialisation failed\n", dist.rank);
        return 1;
    }
    system->Init(false);
    int rc = 0;
    {
        auto pt_pass = std::make_unique<Pupil::pt::PTPass>("Path Tracing");
        system->AddPass(pt_pass.get());
        if (!system->SetScene(argv[1])) {
            rc = 1;
        } else if (const char *bench = std::getenv("PUPIL_BENCH")) {
            rc = Bench(*system, *pt_pass, bench);
        } else if (const char *waste = std::getenv("PUPIL_BENCH_WASTE")) {
            rc = BenchWaste(*system, *pt_pass, waste);
        } else if (const char *tt = std::getenv("PUPIL_THREAD_TEST")) {
            rc = ThreadTest(*system, *pt_pass, tt);
        } else {
            system->Run((uint32_t)frames);
            pt_pass->Inspector();
            auto *bm = Pupil::BufferManager::instance();
            auto *buf = bm->GetBuffer(Pupil::BufferManager::DEFAULT_FINAL_RESULT_BUFFER_NAME);
            const int w = system->GetWorld()->scene->sensor.film.w, h = system->GetWorld()->scene->sensor.film.h;
            const char *dn = std::getenv("PUPIL_DENOISE");  // optix::Denoiser substitute on the final result
            if (dist.rank != 0) {  // the gathered frame lives on rank 0
                system->Destroy();
                return 0;
            }
            if (buf && dn && std::atoi(dn) && !system->Gather()) {
                Pupil::optix::Denoiser denoiser(Pupil::optix::Denoiser::UseAlbedo | Pupil::optix::Denoiser::UseNormal);
                denoiser.Setup((unsigned)w, (unsigned)h);
                Pupil::optix::Denoiser::ExecutionData data;
                data.input = buf->cuda_ptr;
                data.output = buf->cuda_ptr;
                data.albedo = bm->GetBuffer("albedo")->cuda_ptr;
                data.normal = bm->GetBuffer("normal")->cuda_ptr;
                if (!denoiser.Execute(data) || hipDeviceSynchronize() != hipSuccess) rc = 1;
            }
            std::vector<float> host(4 * (size_t)w * h);
            if (!buf || hipMemcpy(host.data(), buf->cuda_ptr, host.size() * sizeof(float), hipMemcpyDeviceToHost) !=
                            hipSuccess) {
                rc = 1;
            } else if (out[0] && pupil_image_save(out, (uint32_t)w, (uint32_t)h, host.data(), PUPIL_IMAGE_AUTO) != PUPIL_OK) {
                Pupil::Log("%s", pupil_last_error());
                rc = 1;
            }
            if (rc == 0) {
                double mean = 0.0;
                for (size_t i = 0; i < host.size(); i += 4) mean += host[i] + host[i + 1] + host[i + 2];
                std::printf("frames %d, %dx%d, mean radiance %.6f, last frame %.3f ms\n", frames, w, h,
                            mean / (3.0 * w * h), pt_pass->LastExecTimeMs());
            }
        }
        system->Destroy();
    }
    return rc;
}
