// denoiser.h — C++ mirror of the reference's Pupil::optix::Denoiser
// (framework/optix/denoiser.h:7-66) over the engine's C ABI (pupil_denoiser_*):
// the same EMode bits, Setup / SetMode / Execute(ExecutionData) and tile
// settings, backed by the HIP a-trous filter (csrc/denoise.hip) because the
// OptiX AI denoiser has no ROCm counterpart.  UseUpscale2X and ApplyToAOV are
// reported as unsupported; tiles are accepted and ignored (the whole frame is
// filtered in one pass over HBM).
#pragma once

#include <hip/hip_runtime.h>

#include "../../../../include/pupil_pt.h"

namespace Pupil::optix {

class Denoiser {
public:
    enum EMode : unsigned int {
        None = 0,
        UseAlbedo = PUPIL_DENOISE_USE_ALBEDO,
        UseNormal = PUPIL_DENOISE_USE_NORMAL,
        ApplyToAOV = PUPIL_DENOISE_APPLY_TO_AOV,
        UseTemporal = PUPIL_DENOISE_USE_TEMPORAL,
        UseUpscale2X = PUPIL_DENOISE_USE_UPSCALE_2X,
        Tiled = PUPIL_DENOISE_TILED
    };

    explicit Denoiser(unsigned int mode = EMode::UseAlbedo | EMode::UseNormal, hipStream_t stream = nullptr,
                      int device = 0) noexcept
        : mode(mode), m_stream(stream) {
        if (pupil_denoiser_create(device, mode, &m_denoiser) != PUPIL_OK) m_denoiser = nullptr;
    }
    ~Denoiser() noexcept { Destroy(); }
    Denoiser(const Denoiser &) = delete;
    Denoiser &operator=(const Denoiser &) = delete;

    void SetMode(unsigned int m) noexcept {
        mode = m;
        if (input_w && input_h) Setup(input_w, input_h);
    }
    void Setup(unsigned int w, unsigned int h) noexcept {
        input_w = w;
        input_h = h;
        if (m_denoiser) m_ok = pupil_denoiser_setup(m_denoiser, mode, w, h, sigma_color) == PUPIL_OK;
    }
    void Destroy() noexcept {
        if (m_denoiser) pupil_denoiser_destroy(m_denoiser);
        m_denoiser = nullptr;
    }
    void SetTile(unsigned int w, unsigned int h) noexcept {
        tile_w = w;
        tile_h = h;
    }

    struct ExecutionData {  // device pointers (CUdeviceptr in the reference)
        const void *input = nullptr;
        void *output = nullptr;
        const void *prev_output = nullptr;
        const void *albedo = nullptr;
        const void *normal = nullptr;
        const void *motion_vector = nullptr;
    };
    bool Execute(const ExecutionData &d) noexcept {
        if (!m_denoiser || !m_ok) return false;
        const pupil_denoise_data data{d.input, d.output, d.prev_output, d.albedo, d.normal, d.motion_vector};
        return pupil_denoiser_execute(m_denoiser, &data, m_stream) == PUPIL_OK;
    }

    unsigned int mode = EMode::UseAlbedo | EMode::UseNormal;
    unsigned int input_w = 0;
    unsigned int input_h = 0;
    unsigned int tile_w = 100;
    unsigned int tile_h = 100;
    float sigma_color = 0.5f;  // colour edge-stopping scale on log radiance (no counterpart in OptiX)

private:
    pupil_denoiser *m_denoiser = nullptr;
    hipStream_t m_stream = nullptr;
    bool m_ok = false;
};

}  // namespace Pupil::optix
