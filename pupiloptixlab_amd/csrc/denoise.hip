// denoise.hip — substitute for the reference's OptiX AI denoiser
// (framework/optix/denoiser.{h,cpp}: Denoiser(mode), Setup(w, h), Execute(data)).
//
// There is no ROCm counterpart of the OptiX denoiser network, so this is an
// edge-avoiding a-trous wavelet filter (Dammertz, Sewtz, Hanika, Lensch 2010):
// five passes of the 5x5 B3-spline kernel h = (1, 4, 6, 4, 1) / 16 at strides
// 1, 2, 4, 8, 16.  Tap q of pixel p is weighted by
//     h(dx) h(dy) exp(-(|t_p - t_q|^2 / s_c^2 + |n_p - n_q|^2 / s_n^2 + |a_p - a_q|^2 / s_a^2))
// where t = log(1 + max(c, 0)) per channel (the colour edge-stopping term on
// log radiance, so HDR edges such as emitters stay sharp while the noise of
// dim regions is averaged), with the colour
// sigma halved every pass (s_c = sigma_color * 2^-pass), the
// normal / albedo terms only when the mode asks for those guides
// (OptixDenoiserOptions::guideAlbedo / guideNormal, denoiser.cpp:46-60).
// Taps outside the image are skipped.  UseTemporal blends the filtered frame
// with prev_output (out = prev + 0.2 (filtered - prev)).
//
// Layout: the guides are repacked once per call into float4 images (one 16-B
// load per tap), colour ping-pongs between two float4 images; each pass is one
// pixel per lane, 25 taps served by L1/L2 (a 1080p pass moves ~2.5 GB through
// the caches, ~0.1 ms).  The filter is pinned by a float64 numpy restatement in
// tests/test_denoise.py.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>

#include "../../include/pupil_pt.h"

namespace Pupil {
void set_last_error(const std::string &m);
}

struct pupil_denoiser {
    int device = 0;
    uint32_t mode = PUPIL_DENOISE_USE_ALBEDO | PUPIL_DENOISE_USE_NORMAL;
    uint32_t width = 0, height = 0;
    float sigma_color = 1.f;
    float4 *ping = nullptr, *pong = nullptr, *gn = nullptr, *ga = nullptr;
    void release() {
        float4 *b[] = {ping, pong, gn, ga};
        for (float4 *p : b)
            if (p) (void)hipFree(p);
        ping = pong = gn = ga = nullptr;
    }
};

namespace {

constexpr float kSigmaNormal = 0.35f;
constexpr float kSigmaAlbedo = 0.1f;
constexpr float kTemporalAlpha = 0.2f;
constexpr int kBlockX = 16, kBlockY = 16;

int fail(int code, const char *msg) {
    Pupil::set_last_error(msg);
    return code;
}

__device__ __forceinline__ float b3(int k) {  // (1, 4, 6, 4, 1) / 16
    return k == 0 ? 0.375f : ((k == 1 || k == -1) ? 0.25f : 0.0625f);
}

__global__ void k_pack_guides(const float *normal, const float *albedo, uint32_t n, float4 *gn, float4 *ga) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (gn) gn[i] = make_float4(normal[3 * i], normal[3 * i + 1], normal[3 * i + 2], 0.f);
    if (ga) ga[i] = make_float4(albedo[3 * i], albedo[3 * i + 1], albedo[3 * i + 2], 0.f);
}

template <bool N, bool A>
__global__ __launch_bounds__(kBlockX *kBlockY) void k_atrous(const float4 *cin, float4 *cout, const float4 *gn,
                                                             const float4 *ga, uint32_t w, uint32_t h, int step,
                                                             float inv_sc2) {
    const int x = blockIdx.x * kBlockX + threadIdx.x;
    const int y = blockIdx.y * kBlockY + threadIdx.y;
    if (x >= (int)w || y >= (int)h) return;
    const size_t i = (size_t)y * w + x;
    const float4 cp = cin[i];
    const float tpx = log1pf(fmaxf(cp.x, 0.f)), tpy = log1pf(fmaxf(cp.y, 0.f)), tpz = log1pf(fmaxf(cp.z, 0.f));
    float4 np = make_float4(0.f, 0.f, 0.f, 0.f), ap = np;
    if (N) np = gn[i];
    if (A) ap = ga[i];
    const float inv_sn2 = 1.f / (kSigmaNormal * kSigmaNormal);
    const float inv_sa2 = 1.f / (kSigmaAlbedo * kSigmaAlbedo);
    float sr = 0.f, sg = 0.f, sb = 0.f, ws = 0.f;
    for (int dy = -2; dy <= 2; dy++) {
        const int yy = y + dy * step;
        if (yy < 0 || yy >= (int)h) continue;
        for (int dx = -2; dx <= 2; dx++) {
            const int xx = x + dx * step;
            if (xx < 0 || xx >= (int)w) continue;
            const size_t j = (size_t)yy * w + xx;
            const float4 cq = cin[j];
            const float dr = tpx - log1pf(fmaxf(cq.x, 0.f)), dg = tpy - log1pf(fmaxf(cq.y, 0.f)),
                        db = tpz - log1pf(fmaxf(cq.z, 0.f));
            float e = (dr * dr + dg * dg + db * db) * inv_sc2;
            if (N) {
                const float4 nq = gn[j];
                const float ux = np.x - nq.x, uy = np.y - nq.y, uz = np.z - nq.z;
                e += (ux * ux + uy * uy + uz * uz) * inv_sn2;
            }
            if (A) {
                const float4 aq = ga[j];
                const float ux = ap.x - aq.x, uy = ap.y - aq.y, uz = ap.z - aq.z;
                e += (ux * ux + uy * uy + uz * uz) * inv_sa2;
            }
            const float wgt = b3(dx) * b3(dy) * expf(-e);
            sr += wgt * cq.x;
            sg += wgt * cq.y;
            sb += wgt * cq.z;
            ws += wgt;
        }
    }
    cout[i] = make_float4(sr / ws, sg / ws, sb / ws, cp.w);  // ws >= h(0)^2 > 0 (the centre tap)
}

__global__ void k_temporal(const float4 *filtered, const float4 *prev, float4 *out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 f = filtered[i], p = prev[i];
    out[i] = make_float4(p.x + kTemporalAlpha * (f.x - p.x), p.y + kTemporalAlpha * (f.y - p.y),
                         p.z + kTemporalAlpha * (f.z - p.z), f.w);
}

}  // namespace

extern "C" {

int pupil_denoiser_create(int device, uint32_t mode, pupil_denoiser **out) {
    if (!out) return fail(PUPIL_ERR_INVALID, "null argument");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(PUPIL_ERR_HIP, "no HIP device");
    if (device < 0 || device >= ndev) return fail(PUPIL_ERR_INVALID, "bad device index");
    if (mode & (PUPIL_DENOISE_APPLY_TO_AOV | PUPIL_DENOISE_USE_UPSCALE_2X))
        return fail(PUPIL_ERR_UNSUPPORTED, "ApplyToAOV / UseUpscale2X are not supported by the a-trous denoiser");
    auto d = new pupil_denoiser();
    d->device = device;
    d->mode = mode;
    *out = d;
    return PUPIL_OK;
}

int pupil_denoiser_setup(pupil_denoiser *d, uint32_t mode, uint32_t width, uint32_t height, float sigma_color) {
    if (!d || width == 0 || height == 0) return fail(PUPIL_ERR_INVALID, "bad arguments");
    if (mode & (PUPIL_DENOISE_APPLY_TO_AOV | PUPIL_DENOISE_USE_UPSCALE_2X))
        return fail(PUPIL_ERR_UNSUPPORTED, "ApplyToAOV / UseUpscale2X are not supported by the a-trous denoiser");
    if (hipSetDevice(d->device) != hipSuccess) return fail(PUPIL_ERR_HIP, "hipSetDevice failed");
    d->mode = mode;
    d->sigma_color = sigma_color > 0.f ? sigma_color : 1.f;
    if (width != d->width || height != d->height) {
        d->release();
        const size_t n = (size_t)width * height;
        if (hipMalloc((void **)&d->ping, sizeof(float4) * n) != hipSuccess ||
            hipMalloc((void **)&d->pong, sizeof(float4) * n) != hipSuccess ||
            hipMalloc((void **)&d->gn, sizeof(float4) * n) != hipSuccess ||
            hipMalloc((void **)&d->ga, sizeof(float4) * n) != hipSuccess) {
            d->release();
            d->width = d->height = 0;
            return fail(PUPIL_ERR_OOM, "denoiser workspace allocation failed");
        }
        d->width = width;
        d->height = height;
    }
    return PUPIL_OK;
}

int pupil_denoiser_execute(pupil_denoiser *d, const pupil_denoise_data *data, void *hip_stream) {
    if (!d || !data || !data->input || !data->output) return fail(PUPIL_ERR_INVALID, "null argument");
    if (!d->ping) return fail(PUPIL_ERR_INVALID, "denoiser not set up");
    if (data->motion_vector) return fail(PUPIL_ERR_UNSUPPORTED, "motion vectors are not supported");
    const bool use_n = (d->mode & PUPIL_DENOISE_USE_NORMAL) != 0;
    const bool use_a = (d->mode & PUPIL_DENOISE_USE_ALBEDO) != 0;
    if ((use_n && !data->normal) || (use_a && !data->albedo)) return fail(PUPIL_ERR_INVALID, "missing guide buffer");
    if (hipSetDevice(d->device) != hipSuccess) return fail(PUPIL_ERR_HIP, "hipSetDevice failed");
    hipStream_t s = (hipStream_t)hip_stream;
    const uint32_t w = d->width, h = d->height;
    const uint32_t n = w * h;
    if (use_n || use_a)
        hipLaunchKernelGGL(k_pack_guides, dim3((n + 255) / 256), dim3(256), 0, s, (const float *)data->normal,
                           (const float *)data->albedo, n, use_n ? d->gn : nullptr, use_a ? d->ga : nullptr);
    const dim3 grid((w + kBlockX - 1) / kBlockX, (h + kBlockY - 1) / kBlockY), block(kBlockX, kBlockY);
    const float4 *src = (const float4 *)data->input;
    float4 *bufs[2] = {d->ping, d->pong};
    for (int pass = 0; pass < 5; pass++) {
        float4 *dst = bufs[pass & 1];
        const float sc = d->sigma_color * std::ldexp(1.f, -pass);
        const float inv_sc2 = 1.f / (sc * sc);
#define ATROUS(N, A) \
    hipLaunchKernelGGL((k_atrous<N, A>), grid, block, 0, s, src, dst, d->gn, d->ga, w, h, 1 << pass, inv_sc2)
        if (use_n && use_a) ATROUS(true, true);
        else if (use_n) ATROUS(true, false);
        else if (use_a) ATROUS(false, true);
        else ATROUS(false, false);
#undef ATROUS
        src = dst;
    }
    if ((d->mode & PUPIL_DENOISE_USE_TEMPORAL) && data->prev_output) {
        hipLaunchKernelGGL(k_temporal, dim3((n + 255) / 256), dim3(256), 0, s, src, (const float4 *)data->prev_output,
                           (float4 *)data->output, n);
    } else if (hipMemcpyAsync(data->output, src, sizeof(float4) * n, hipMemcpyDeviceToDevice, s) != hipSuccess) {
        return fail(PUPIL_ERR_HIP, "output copy failed");
    }
    if (hipGetLastError() != hipSuccess) return fail(PUPIL_ERR_HIP, "denoiser launch failed");
    return PUPIL_OK;
}

void pupil_denoiser_destroy(pupil_denoiser *d) {
    if (!d) return;
    (void)hipSetDevice(d->device);
    d->release();
    delete d;
}

}  // extern "C"
