// pt_frame.hip — one persistent launch per frame for small frames (r05): the whole path loop of
// example/path_tracer/main.cu:36-193 -- camera ray, closest hit, shade, shadow ray, next
// bounce -- for every path of a frame that the stage pipeline would run as D traversal
// launches, D shade launches and D - 1 flags partitions.
//
// Why: a frame that is never continued (the camera moves before every OnRun, world.cpp:15-43,
// pt_pass.cpp:40-49) cannot be pipelined, and a small one (one rank's tile share at N = 8:
// 260 k paths at 1080p) pays a launch, a persistent-kernel drain and a partition per bounce
// for very little work each (r05 shard probe, moving camera: 2.66x at N = 8).  Here every
// wave owns the paths it starts until they end: a wave-local trace queue and shade queue in
// LDS hand each path from its traversal to its shade and back, with no global queue, no
// partition and no grid-wide step between bounces.
//
// Per path the operations and their order are the stage pipeline's (the same device
// functions, pt_shade.h / pt_traverse.h).  A wave works in rounds: it traces every queued
// ray (a bounce's shadow and extension rays concurrently, each path's shadow contribution added
// at its retire), and only once none is left does it shade the paths whose extension rays hit --
// so a shadow contribution is always added before the next bounce's shade adds to the radiance
// (main.cu:119-140 before :165-185), the sums keep the reference's order and every pixel is
// bit-identical to the oracle.
#include "pt_kernels.h"
#include "pt_shade.h"
#include "pt_shading.h"
#include "pt_trace.h"
#include "pt_traverse.h"

#include <algorithm>
#include <cstdlib>

namespace pupil {

namespace {

using namespace tr;

// queue entries: path id | kind
constexpr uint32_t kQKindShadow = 0x80000000u;  // shadow ray of the path's current bounce
constexpr uint32_t kQPath = 0x7FFFFFFFu;
constexpr uint32_t kFrameQ = 128;  // entries per wave and queue (a wave owns at most 64 paths, 2 rays each)
constexpr uint32_t kFrameWaves = kTraceBlock / 64;
// waves per SIMD of the one-launch frame kernel (its registers: trace + shade state); A/B builds
#ifndef PUPIL_FRAME_WAVES
#define PUPIL_FRAME_WAVES 4
#endif
constexpr uint32_t kFrameWavesPerSimd = PUPIL_FRAME_WAVES;

struct FrameJob {
    uint32_t *work;      // kWorkKind counters (XCD-sharded dequeue heads + exit counters), zero at launch
    uint32_t n_paths;    // paths of the frame (spp x local pixels), ids [0, n_paths)
    uint32_t refill;     // refill a wave's idle lanes once this many are idle
    uint32_t node_min;
    uint32_t spp;        // dequeue the spp samples of a pixel on consecutive lanes (0: path order)
    uint32_t num_local;
    unsigned long long *ray_cum;  // running totals: [0] extension rays (bounce >= 1), [1] shadow rays
};

// material bin of a hit record slot (flat / world-mode records: trace4_body's retire)
__device__ __forceinline__ uint32_t record_bin(const DeviceScene &sc, uint32_t best_idx) {
    const uint32_t mt = __float_as_uint(sc.prims[kRecF4 * best_idx + 2].w);
    return (mt >= 1u && mt <= 7u) ? mt : 8u;
}

template <uint32_t MAT>
__device__ __forceinline__ uint32_t shade_path(const DeviceScene &sc, const FrameParams &fp, const PathState &ps,
                                               uint32_t p, uint32_t bin) {
    if (bin == 0u) {
        shade_miss(sc, fp, ps, p, false, 0u, 0u);
        return 0u;
    }
    if (MAT != 0xFFu) return shade_hit<MAT>(sc, fp, ps, p, false, 0u, 0u);
    switch (bin) {
    case PUPIL_MAT_DIFFUSE: return shade_hit<PUPIL_MAT_DIFFUSE>(sc, fp, ps, p, false, 0u, 0u);
    case PUPIL_MAT_DIELECTRIC: return shade_hit<PUPIL_MAT_DIELECTRIC>(sc, fp, ps, p, false, 0u, 0u);
    case PUPIL_MAT_ROUGH_DIELECTRIC: return shade_hit<PUPIL_MAT_ROUGH_DIELECTRIC>(sc, fp, ps, p, false, 0u, 0u);
    case PUPIL_MAT_CONDUCTOR: return shade_hit<PUPIL_MAT_CONDUCTOR>(sc, fp, ps, p, false, 0u, 0u);
    case PUPIL_MAT_ROUGH_CONDUCTOR: return shade_hit<PUPIL_MAT_ROUGH_CONDUCTOR>(sc, fp, ps, p, false, 0u, 0u);
    case PUPIL_MAT_PLASTIC: return shade_hit<PUPIL_MAT_PLASTIC>(sc, fp, ps, p, false, 0u, 0u);
    case PUPIL_MAT_ROUGH_PLASTIC: return shade_hit<PUPIL_MAT_ROUGH_PLASTIC>(sc, fp, ps, p, false, 0u, 0u);
    default: return shade_hit<0u>(sc, fp, ps, p, false, 0u, 0u);
    }
}

// Wave-uniform ring of kFrameQ path entries in LDS (one per wave and queue).
struct WaveQueue {
    uint32_t *e;
    uint32_t head, tail;  // wave-uniform
    __device__ __forceinline__ uint32_t size() const { return tail - head; }
    // every lane with `has` appends `v`, in lane order
    __device__ __forceinline__ void push(bool has, uint32_t v) {
        const unsigned long long m = __ballot(has);
        if (has) e[(tail + (uint32_t)__popcll(m & lanemask_lt())) % kFrameQ] = v;
        tail += (uint32_t)__popcll(m);
    }
    // the lanes with `want` take the next entries, in lane order, while there are any
    __device__ __forceinline__ bool pop(bool want, uint32_t &v) {
        const unsigned long long m = __ballot(want);
        const uint32_t k = (uint32_t)__popcll(m & lanemask_lt());
        const uint32_t n = min((uint32_t)__popcll(m), size());
        const bool got = want && k < n;
        if (got) v = e[(head + k) % kFrameQ];
        head += n;
        return got;
    }
};

template <uint32_t MAT>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(kFrameWavesPerSimd))) void k_frame(
    DeviceScene sc, FrameParams fp, PathState ps, FrameJob job, int *ovf, uint32_t ovf_threads) {
    constexpr float kInf = __builtin_huge_valf();
    __shared__ int s_ring[kRing * kTraceBlock];
    __shared__ float s_aux[4 * kTraceBlock];
    __shared__ uint32_t s_q[kFrameWaves][2][kFrameQ];
    const uint32_t wv = threadIdx.x / 64u;
    WaveQueue tq{s_q[wv][0], 0u, 0u};  // rays to trace
    WaveQueue sq{s_q[wv][1], 0u, 0u};  // paths whose extension ray has its hit: to shade

    LinStack st;
    st.lds = s_ring + threadIdx.x;
    st.ovf_blk = ovf + blockIdx.x * blockDim.x;
    st.lds0 = s_ring;
    st.ovf_stride = ovf_threads;
    st.reset();
    float &b1 = s_aux[threadIdx.x];
    float &b2 = s_aux[kTraceBlock + threadIdx.x];
    uint32_t &p = reinterpret_cast<uint32_t *>(s_aux)[2 * kTraceBlock + threadIdx.x];
    uint32_t &best_idx = reinterpret_cast<uint32_t *>(s_aux)[3 * kTraceBlock + threadIdx.x];
    b1 = b2 = 0.f;
    p = 0;
    best_idx = kMissIndex;

    uint32_t n_ext = 0, n_shadow = 0;  // rays traced by this lane (extension rays of bounces >= 1, shadow rays)
    uint32_t shard = blockIdx.x % kWorkShards, tried = 0;
    bool drained = false;  // the frame's paths are all handed out
    bool active = false, any = false, found = false;
    uint32_t best_key = 0;
    RayPre r{};
    vec3 be = v3(0.f);
    float tmax = 0.f;
    constexpr float tmin = 0.001f;
    int node = kSentinel, leaf = 0;
    auto ray_dir = [&]() -> vec3 { return f3(any ? ld_ps(ps.sh_d + p) : ld_ps(ps.ray_d + p)); };
    // a lane starts tracing: the path's shadow ray (any hit) or its extension / camera ray
    auto start = [&](float4 o, float4 d, bool shadow) {
        any = shadow;
        tmax = shadow ? o.w : kMaxDistance;
        r = ray_pre(f3(o), f3(d));
        best_key = 0xFFFFFFFFu;
        best_idx = kMissIndex;
        b1 = b2 = 0.f;
        found = false;
        st.reset();
        node = (int)sc.root_link4;
        leaf = 0;
        be = slab_errors(r.o, r.idir, sc.node_bound);
        if (node < 0) {
            leaf = node;
            node = kSentinel;
        }
        active = true;
    };

    for (;;) {
        // ---- shade, between rounds: once no lane of the wave traces, every path whose extension
        // ray has its hit is shaded (64 per pass).  The traversal state is reset first, so it is
        // dead here and the shade runs in registers of its own.
        if (!__any(active) && tq.size() == 0) {
            node = kSentinel;
            leaf = 0;
            r = RayPre{};
            be = v3(0.f);
            tmax = 0.f;
            best_key = 0;
            any = found = false;
            st.reset();
            while (sq.size() > 0) {
                uint32_t q = 0;
                const bool mine = sq.pop(true, q);
                uint32_t flags = 0;
                if (mine) {
                    const bool miss = __float_as_uint(ld_ps(ps.hit + q).w) == kMissIndex;
                    flags = shade_path<MAT>(sc, fp, ps, q, miss ? 0u : (sc.single_bin ? sc.single_bin : ps.mbin[q]));
                    if (!sc.single_bin) ps.mbin[q] = 0xFFu;  // the bins-mode invariant: untraced paths read 0xFF
                }
                // both rays of the bounce are traced in the next round, concurrently; the round ends
                // before any path is shaded again, so a shadow contribution is always added before
                // the next bounce's shade adds to the radiance (main.cu:119-140 before :165-185)
                tq.push((flags & 2u) != 0u, q | kQKindShadow);
                tq.push((flags & 1u) != 0u, q);
            }
            if (drained && tq.size() == 0) break;  // every path of the frame has ended
        }
        // ---- refill idle lanes: queued rays first; new paths of the frame when a round starts
        // (nothing queued), so a wave owns at most 64 paths at a time
        const unsigned long long idle = __ballot(!active);
        const uint32_t n_idle = (uint32_t)__popcll(idle);
        if (n_idle >= job.refill || n_idle == 64u) {
            uint32_t e = 0;
            const bool queued = tq.size() > 0;
            if (tq.pop(!active, e)) {
                p = e & kQPath;
                const bool shadow = (e & kQKindShadow) != 0u;
                if (shadow) n_shadow++;
                else n_ext++;
                start(ld_ps(ps.ray_o + p), shadow ? ld_ps(ps.sh_d + p) : ld_ps(ps.ray_d + p), shadow);
            }
            const unsigned long long still = __ballot(!active);
            const uint32_t n_still = (uint32_t)__popcll(still);
            if (!drained && !queued && n_still == 64u) {
                // XCD-sharded dequeue of new paths (trace4_body's protocol): chunk `shard` of the path range
                const uint32_t lo = (uint32_t)((uint64_t)job.n_paths * shard / kWorkShards);
                const uint32_t len = (uint32_t)((uint64_t)job.n_paths * (shard + 1) / kWorkShards) - lo;
                uint32_t base = 0;
                if (lane_id() == 0) base = atomicAdd(job.work + shard * kWorkStride, n_still);
                base = __shfl(base, 0);
                if (base + n_still >= len) {
                    shard = shard + 1 == kWorkShards ? 0u : shard + 1;
                    if (++tried == kWorkShards) drained = true;
                }
                const uint32_t k = base + (uint32_t)__popcll(still & lanemask_lt());
                if (!active && k < len) {
                    // a camera ray (main.cu:53-75), generated here; its path state stored whole (k_generate
                    // with full = 1: throughput 1, radiance 0, the RNG after the two film draws)
                    const uint32_t i = lo + k;
                    p = job.spp ? (i % job.spp) * job.num_local + i / job.spp : i;
                    vec3 dir;
                    const uint32_t rng = fresh_path(sc, fp, p, fp.seed0, dir);
                    const float4 o = f4(camera_origin(sc.camera), 0.f), d = make_float4(dir.x, dir.y, dir.z, 0.f);
                    st_ps(ps.ray_o + p, o);
                    st_ps(ps.ray_d + p, d);
                    st_ps(ps.thr + p, make_float4(1.f, 1.f, 1.f, 0.f));
                    st_ps(ps.rad + p, make_float4(0.f, 0.f, 0.f, 0.f));
                    st_ps(ps.misc + p, make_uint4(rng, 0u, 0u, 0u));
                    start(o, d, false);
                }
            }
        }
        if (!__any(active)) continue;  // the shade above, or another dequeue
        // ---- traverse (trace4_body's while-while loops, flat BVH4)
        if (active) {
            while ((uint32_t)node < (uint32_t)kSentinel) {
                const Bvh4Node n = load_node4(sc, node);
                float t[4];
                int l[4];
                visit4(n, r.o, r.idir, be, tmin, tmax, t, l);
                if (t[0] == kInf) {
                    node = st.pop();
                } else {
                    node = l[0];
                    st.reserve3();
                    st.push3(l[1], l[2], l[3], t[1] != kInf, t[2] != kInf, t[3] != kInf);
                    if (node == kEmptyLink) node = st.pop();
                }
                if (node < 0 && leaf >= 0) {
                    leaf = node;
                    node = st.pop();
                }
                if ((uint32_t)__popcll(__ballot(leaf >= 0)) < job.node_min) break;
            }
            while (leaf < 0) {
                uint32_t np_cnt = 0;
                if (intersect_leaf_dyn<false>(sc, r, leaf, tmin, tmax, best_key, best_idx, b1, b2, np_cnt, found, any,
                                              ray_dir))
                    break;
                leaf = node;
                if (node < 0) node = st.pop();
            }
        }
        const bool done = active && ((node == kSentinel && leaf >= 0) || (any && found));
        // ---- retire
        if (done && !any) {  // extension / camera ray: the hit record, then the path waits for its shade
            const uint32_t hidx = sc.two_level ? best_key : best_idx;
            st_ps(ps.hit + p, make_float4(found ? tmax : -1.f, b1, b2, __uint_as_float(found ? hidx : kMissIndex)));
            if (!sc.single_bin) ps.mbin[p] = (uint8_t)(found ? record_bin(sc, best_idx) : 0u);
        }
        if (done && any && !found) {  // main.cu:124-139
            const float4 c = ld_ps(ps.sh_c + p);
            float4 L = ld_ps(ps.rad + p);
            L.x = L.x + c.x;
            L.y = L.y + c.y;
            L.z = L.z + c.z;
            st_ps(ps.rad + p, L);
        }
        sq.push(done && !any, p);
        if (done) active = false;
    }
    // ray counts into the running totals (one atomic per wave and kind)
    unsigned long long a = n_ext, b = n_shadow;
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o);
        b += __shfl_xor(b, o);
    }
    if (lane_id() == 0) {
        if (a) atomicAdd(job.ray_cum + 0, a);
        if (b) atomicAdd(job.ray_cum + 1, b);
        // the last wave out resets the dequeue heads (trace4_body's exit counting)
        const uint32_t sub = blockIdx.x % kWorkShards;
        const uint32_t groups = min(gridDim.x, kWorkShards);
        const uint32_t sub_waves = (gridDim.x - sub + kWorkShards - 1u) / kWorkShards * (blockDim.x / 64u);
        if (atomicAdd(job.work + (kWorkShards + 1u + sub) * kWorkStride, 1u) == sub_waves - 1u &&
            atomicAdd(job.work + kWorkShards * kWorkStride, 1u) == groups - 1u) {
            for (uint32_t k = 0; k < 2u * kWorkShards + 1u; k++) atomicExch(job.work + k * kWorkStride, 0u);
        }
    }
}

}  // namespace

bool frame_kernel_supported(const DeviceScene &sc) { return !(sc.two_level && !sc.tl_world); }

// One persistent launch over every path of a frame (pt_frame.hip header).  Grid: the resident
// capacity at 4 waves per SIMD, capped at one wave per 64 paths.
void launch_frame(const DeviceScene &sc, const FrameParams &fp, const PathState &ps, uint32_t *work,
                  unsigned long long *ray_cum, int *ovf, uint32_t ovf_threads, uint32_t interleave_spp, hipStream_t s) {
    FrameJob job{work, fp.num_paths, sc.trace_refill, sc.trace_node_min, interleave_spp, fp.num_local, ray_cum};
    const uint32_t resident = sc.num_cus * 4u * kFrameWavesPerSimd / kFrameWaves;
    const uint32_t by_paths = (fp.num_paths + kTraceBlock - 1) / kTraceBlock;
    const uint32_t blocks = std::min(ovf_threads / kTraceBlock, std::max(1u, std::min(resident, by_paths)));
    switch (sc.single_bin) {
    case PUPIL_MAT_DIFFUSE:
        hipLaunchKernelGGL(k_frame<PUPIL_MAT_DIFFUSE>, dim3(blocks), dim3(kTraceBlock), 0, s, sc, fp, ps, job, ovf,
                           ovf_threads);
        break;
    default:
        hipLaunchKernelGGL(k_frame<0xFFu>, dim3(blocks), dim3(kTraceBlock), 0, s, sc, fp, ps, job, ovf, ovf_threads);
        break;
    }
}

}  // namespace pupil
