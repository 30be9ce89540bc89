// examples/path_tracer/main.cpp — headless counterpart of the reference's
// example/path_tracer/main.cpp: System + PTPass + an XML scene, rendered for
// a fixed number of frames (the reference loops until the window closes),
// then "final result" is written as a PFM (rows bottom-up, which is the
// reference's pixel order: row 0 is the image bottom).
//
// usage: pupil_path_tracer <scene.xml> [frames=16] [out.pfm] [device=0]
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <vector>

#include "pupil/framework.h"
#include "pupil/pt_pass.h"

static bool write_pfm(const char *path, const float *rgba, int w, int h) {
    FILE *f = std::fopen(path, "wb");
    if (!f) return false;
    std::fprintf(f, "PF\n%d %d\n-1.0\n", w, h);
    std::vector<float> row(3 * (size_t)w);
    for (int y = 0; y < h; y++) {
        for (int x = 0; x < w; x++)
            for (int c = 0; c < 3; c++) row[3 * x + c] = rgba[4 * ((size_t)y * w + x) + c];
        std::fwrite(row.data(), sizeof(float), row.size(), f);
    }
    return std::fclose(f) == 0;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <scene.xml> [frames=16] [out.pfm] [device=0]\n", argv[0]);
        return 2;
    }
    const int frames = argc > 2 ? std::atoi(argv[2]) : 16;
    const char *out = argc > 3 ? argv[3] : "";
    auto system = Pupil::util::Singleton<Pupil::System>::instance();
    system->device = argc > 4 ? std::atoi(argv[4]) : 0;
    system->Init(false);
    int rc = 0;
    {
        auto pt_pass = std::make_unique<Pupil::pt::PTPass>("Path Tracing");
        system->AddPass(pt_pass.get());
        if (!system->SetScene(argv[1])) {
            rc = 1;
        } else {
            system->Run((uint32_t)frames);
            pt_pass->Inspector();
            auto *buf = Pupil::BufferManager::instance()->GetBuffer(Pupil::BufferManager::DEFAULT_FINAL_RESULT_BUFFER_NAME);
            const int w = system->GetWorld()->scene->sensor.film.w, h = system->GetWorld()->scene->sensor.film.h;
            std::vector<float> host(4 * (size_t)w * h);
            if (!buf || hipMemcpy(host.data(), buf->cuda_ptr, host.size() * sizeof(float), hipMemcpyDeviceToHost) !=
                            hipSuccess) {
                rc = 1;
            } else if (out[0] && !write_pfm(out, host.data(), w, h)) {
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
