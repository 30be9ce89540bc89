// Micro-benchmark: what one vector-memory load instruction costs the CU's data-return path
// (TA / TD) as a function of its width and its active lanes, with the data resident in the
// L1 (a 16-KiB table per workgroup's working set), so the loads never wait on a miss.
// The traversal (k_trace4) is bound by the TD; this decides whether
// a narrower load (dwordx3 for a 36-B triangle, dwordx2 for packed fields) is cheaper than
// a dwordx4 or costs the same per instruction.
//   W  = dwords per lane (1, 2, 3, 4)
//   L  = active lanes per wave (64 or 1)
//   P  = address pattern: 0 scattered lines (each lane its own pseudo-random slot),
//        1 one slot for the whole wave (broadcast), 2 lane-contiguous slots (coalesced: a
//        wave touches 64 x W dwords in order)
// Every wave issues `iters` x 8 independent loads; reported: ns per wave-instruction per CU
// and cycles at the clock given on the command line.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_td.hip -o build/ubench_td
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

constexpr int kBlock = 256;
constexpr uint32_t kTabDwords = 4096;  // 16 KiB: L1-resident

template <int W>
struct Vec;
template <>
struct Vec<1> {
    typedef unsigned T;
    __device__ static unsigned fold(T v) { return v; }
};
template <>
struct Vec<2> {
    typedef unsigned T __attribute__((ext_vector_type(2)));
    __device__ static unsigned fold(T v) { return v.x ^ v.y; }
};
template <>
struct Vec<3> {
    typedef unsigned T __attribute__((ext_vector_type(3)));
    __device__ static unsigned fold(T v) { return v.x ^ v.y ^ v.z; }
};
template <>
struct Vec<4> {
    typedef unsigned T __attribute__((ext_vector_type(4)));
    __device__ static unsigned fold(T v) { return v.x ^ v.y ^ v.z ^ v.w; }
};

template <int W, int L, int P>
__global__ __launch_bounds__(kBlock) void k_loads(const unsigned *tab, int iters, unsigned *out) {
    typedef typename Vec<W>::T T;
    const uint32_t lane = __lane_id();
    uint32_t h = (blockIdx.x * kBlock + threadIdx.x) * 2654435761u;
    unsigned acc = 0;
    if (L == 64 || lane == 0) {
        for (int it = 0; it < iters; it++) {
            T v[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                h = h * 1664525u + 1013904223u;
                // dword offset: a 16-B aligned slot per lane (P 0), per wave (P 1), or lane-contiguous
                // W-dword elements from a wave-uniform 1-KiB block (P 2)
                uint32_t off;
                if (P == 0) {
                    off = 4u * ((h >> 20) & (kTabDwords / 4 - 1));
                } else {
                    const uint32_t u = __builtin_amdgcn_readfirstlane(h >> 20);
                    off = P == 1 ? 4u * (u & (kTabDwords / 4 - 1)) : (u & 15u) * 256u + lane * W;
                    asm volatile("v_mov_b32 %0, %1" : "=v"(off) : "v"(off));  // keep it a vector load
                }
                v[j] = *reinterpret_cast<const T *>(tab + off);
            }
#pragma unroll
            for (int j = 0; j < 8; j++) acc ^= Vec<W>::fold(v[j]);
        }
    }
    out[blockIdx.x * kBlock + threadIdx.x] = acc;
}

template <int W, int L, int P>
static void run(const unsigned *tab, unsigned *out, int blocks, int iters, double ghz, int cus) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_loads<W, L, P>), dim3(blocks), dim3(kBlock), 0, 0, tab, iters, out);  // warm
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL((k_loads<W, L, P>), dim3(blocks), dim3(kBlock), 0, 0, tab, iters, out);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    const double insts = (double)blocks * (kBlock / 64) * iters * 8.0;  // wave-instructions
    const double per_cu = insts / cus;
    const double ns = best * 1e6 / per_cu;
    std::printf("W=%d lanes=%2d pattern=%s  %.3f ms  %.3f ns/inst/CU  %.2f cycles/inst/CU at %.2f GHz\n", W, L,
                P == 2 ? "coalesced" : (P ? "broadcast" : "scattered"), best, ns, ns * ghz, ghz);
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
}

int main(int argc, char **argv) {
    const double ghz = argc > 1 ? std::atof(argv[1]) : 2.4;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 256;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = cus * 8;  // 8 x 4 waves per CU: 8 waves per SIMD
    unsigned *tab, *out;
    CHECK(hipMalloc(&tab, kTabDwords * 4));
    CHECK(hipMalloc(&out, (size_t)blocks * kBlock * 4));
    CHECK(hipMemset(tab, 0x5a, kTabDwords * 4));
    std::printf("# %d CUs, %d blocks x %d threads, %d x 8 loads per lane\n", cus, blocks, kBlock, iters);
    run<1, 64, 0>(tab, out, blocks, iters, ghz, cus);
    run<2, 64, 0>(tab, out, blocks, iters, ghz, cus);
    run<3, 64, 0>(tab, out, blocks, iters, ghz, cus);
    run<4, 64, 0>(tab, out, blocks, iters, ghz, cus);
    run<1, 1, 0>(tab, out, blocks, iters, ghz, cus);
    run<4, 1, 0>(tab, out, blocks, iters, ghz, cus);
    run<1, 64, 1>(tab, out, blocks, iters, ghz, cus);
    run<4, 64, 1>(tab, out, blocks, iters, ghz, cus);
    run<1, 64, 2>(tab, out, blocks, iters, ghz, cus);
    run<2, 64, 2>(tab, out, blocks, iters, ghz, cus);
    run<4, 64, 2>(tab, out, blocks, iters, ghz, cus);
    CHECK(hipFree(tab));
    CHECK(hipFree(out));
    return 0;
}
