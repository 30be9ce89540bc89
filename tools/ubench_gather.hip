// Micro-benchmark: dependent random 64-B node gathers, the memory pattern of
// incoherent BVH traversal.  Each lane follows its own chain of `steps`
// random nodes in a table of `nodes` x 64 B (next index read from the node).
//   A: every lane loads its own node with 4 x global_load_dwordx4
//   B: 4 lanes cooperate per node (lane i loads quarter i&3 of the node of lane
//      16*j + i/4 in instruction j), then the quarters are transposed through LDS
//   C: every lane loads 16 B of its own node (1 x dwordx4): per-line cost floor
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_gather.hip -o build/ubench_gather
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(x)                                                               \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

constexpr int kBlock = 128;

__global__ __launch_bounds__(kBlock) void kA(const uint4 *tab, uint32_t mask, int steps, uint32_t *out) {
    uint32_t idx = (blockIdx.x * kBlock + threadIdx.x) * 2654435761u & mask;
    uint32_t acc = 0;
    for (int s = 0; s < steps; s++) {
        const uint4 *n = tab + 4 * (size_t)idx;
        const uint4 a = n[0], b = n[1], c = n[2], d = n[3];
        acc += a.y + b.x + c.z + d.w;
        idx = (a.x ^ d.y) & mask;
    }
    out[blockIdx.x * kBlock + threadIdx.x] = acc;
}

__global__ __launch_bounds__(kBlock) void kB(const uint4 *tab, uint32_t mask, int steps, uint32_t *out) {
    __shared__ uint4 xch[kBlock * 4];
    const int lane = threadIdx.x & 63;
    uint4 *w = xch + (threadIdx.x & ~63) * 4;  // this wave's 64 nodes x 4 quarters
    uint32_t idx = (blockIdx.x * kBlock + threadIdx.x) * 2654435761u & mask;
    uint32_t acc = 0;
    for (int s = 0; s < steps; s++) {
        uint4 q[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int owner = 16 * j + (lane >> 2);
            const uint32_t oi = __shfl(idx, owner);
            q[j] = tab[4 * (size_t)oi + (lane & 3)];
        }
#pragma unroll
        for (int j = 0; j < 4; j++) w[(16 * j + (lane >> 2)) * 4 + (lane & 3)] = q[j];
        __builtin_amdgcn_wave_barrier();
        const uint4 a = w[lane * 4 + 0], b = w[lane * 4 + 1], c = w[lane * 4 + 2], d = w[lane * 4 + 3];
        __builtin_amdgcn_wave_barrier();
        acc += a.y + b.x + c.z + d.w;
        idx = (a.x ^ d.y) & mask;
    }
    out[blockIdx.x * kBlock + threadIdx.x] = acc;
}

__global__ __launch_bounds__(kBlock) void kC(const uint4 *tab, uint32_t mask, int steps, uint32_t *out) {
    uint32_t idx = (blockIdx.x * kBlock + threadIdx.x) * 2654435761u & mask;
    uint32_t acc = 0;
    for (int s = 0; s < steps; s++) {
        const uint4 a = tab[4 * (size_t)idx];
        acc += a.y;
        idx = (a.x ^ a.w) & mask;
    }
    out[blockIdx.x * kBlock + threadIdx.x] = acc;
}

int main(int argc, char **argv) {
    // usage: ubench_gather [log2_nodes=18] [--json]
    //   --json: one line {"table_mb", "ceiling_gnodes_per_s", "per_waves_per_simd": {...}} with the best
    //   variant-A rate (each lane fetches its own 64-B node, the traversal's access shape)
    const uint32_t log_nodes = argc > 1 ? atoi(argv[1]) : 18;  // 2^18 x 64 B = 16 MB
    const bool json = argc > 2 && std::string(argv[2]) == "--json";
    const int steps = 64;
    const uint32_t nodes = 1u << log_nodes, mask = nodes - 1;
    std::vector<uint4> h(4 * (size_t)nodes);
    uint64_t x = 88172645463325252ull;
    for (auto &v : h) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        v = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)(x * 3), (uint32_t)(x >> 17));
    }
    uint4 *d;
    uint32_t *out;
    CHECK(hipMalloc(&d, h.size() * sizeof(uint4)));
    CHECK(hipMemcpy(d, h.data(), h.size() * sizeof(uint4), hipMemcpyHostToDevice));
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    double best_a = 0.0;
    std::string per;
    for (int wpe : {2, 4, 6, 7, 8}) {
        const int blocks = cus * 4 * wpe / 2;
        CHECK(hipMalloc(&out, sizeof(uint32_t) * blocks * kBlock));
        for (int k = 0; k < (json ? 1 : 3); k++) {
            hipEvent_t e0, e1;
            CHECK(hipEventCreate(&e0));
            CHECK(hipEventCreate(&e1));
            float best = 1e30f;
            for (int rep = 0; rep < 4; rep++) {
                CHECK(hipEventRecord(e0));
                if (k == 0) hipLaunchKernelGGL(kA, dim3(blocks), dim3(kBlock), 0, 0, d, mask, steps, out);
                if (k == 1) hipLaunchKernelGGL(kB, dim3(blocks), dim3(kBlock), 0, 0, d, mask, steps, out);
                if (k == 2) hipLaunchKernelGGL(kC, dim3(blocks), dim3(kBlock), 0, 0, d, mask, steps, out);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                if (rep) best = ms < best ? ms : best;
            }
            CHECK(hipEventDestroy(e0));
            CHECK(hipEventDestroy(e1));
            const double fetches = (double)blocks * kBlock * steps;
            const double rate = fetches / best / 1e6;  // G fetches/s
            if (k == 0) {
                best_a = rate > best_a ? rate : best_a;
                char buf[64];
                std::snprintf(buf, sizeof(buf), "%s\"%d\": %.2f", per.empty() ? "" : ", ", wpe, rate);
                per += buf;
            }
            if (!json)
                std::printf("table %6.1f MB waves/SIMD %d variant %c: %.3f ms, %.2f G node-fetches/s, %.0f GB/s (64 B each)\n",
                            nodes * 64.0 / 1e6, wpe, "ABC"[k], best, rate, rate * 64);
        }
        CHECK(hipFree(out));
    }
    CHECK(hipFree(d));
    if (json)
        std::printf("{\"table_mb\": %.2f, \"ceiling_gnodes_per_s\": %.2f, \"per_waves_per_simd\": {%s}}\n",
                    nodes * 64.0 / 1e6, best_a, per.c_str());
    return 0;
}
