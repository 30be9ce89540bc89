// queue_partition.hip — stable partition of path ids by a per-path key byte.
//
// The wavefront stages no longer append path ids to queues with atomics (which
// leaves every queue in completion order, so the next stage gathers its 16-B
// path-state records from random addresses).  Instead each stage writes one
// key byte per path (extend: material bin; shade: next/shadow flags) and this
// partition lists the ids of every bin in increasing path order, so the next
// stage reads and writes path state in runs of consecutive records.
//
//   k_part_count    per block tile of 4 waves x rounds x 64 paths: count of each
//                   bin (wave ballots); rounds is sized so that a launch has
//                   about kPartTargetBlocks blocks (a 2M-path shard of an 8-GPU
//                   frame fills the chip as well as a 16M-path 1-GPU frame)
//   k_part_scan     one block: exclusive scan of the bin-major histogram,
//                   per-bin start and count
//   k_part_scatter  per tile: recount per wave, then rank with ballots and write
//
// Modes (PartMode, pt_kernels.h): exclusive (bin = key >> shift, 0xFF none),
// flags (bit b puts the path in bin b when the key's bounce tag, bits 2..7,
// equals `shift`; a path can be in several bins).
#include <algorithm>
#include <cstdlib>

#include "pt_kernels.h"

namespace pupil {

namespace {

constexpr int kPartBlock = 256;               // 4 waves
constexpr uint32_t kPartMaxRounds = 64;       // rounds of 64 paths per wave
constexpr uint32_t kPartTargetBlocks = 2048;

// launch-size target, <= kPartTargetBlocks (PUPIL_PART_BLOCKS, A/B: fewer blocks shorten the scan)
uint32_t part_target() {
    static const uint32_t t = [] {
        const char *e = std::getenv("PUPIL_PART_BLOCKS");
        const int v = e ? std::atoi(e) : (int)kPartTargetBlocks;
        return (uint32_t)std::min((int)kPartTargetBlocks, std::max(64, v));
    }();
    return t;
}
uint32_t part_rounds(uint32_t n) {
    const uint32_t tb = part_target();
    const uint32_t r = (uint32_t)(((uint64_t)n + 256ull * tb - 1) / (256ull * tb));
    return std::max(1u, std::min(kPartMaxRounds, r));
}
uint32_t part_blocks(uint32_t n) {
    const uint32_t tile = 256u * part_rounds(n);
    return (uint32_t)(((uint64_t)n + tile - 1) / tile);
}

// key value that is in no bin
template <int MODE>
__device__ __forceinline__ uint32_t no_key() {
    return MODE == kPartExclusive ? 0xFFu : 0u;
}

template <int MODE>
__device__ __forceinline__ bool in_bin(uint32_t k, uint32_t b, uint32_t shift) {
    if (MODE == kPartExclusive) return (k >> shift) == b && k != 0xFFu;
    return ((k >> b) & 1u) != 0u && (k >> 2) == shift;  // kPartFlags: shift carries the bounce tag
}

__device__ __forceinline__ unsigned long long lanes_below() { return (1ull << __lane_id()) - 1ull; }

// A wave's key bytes, kPartBatch rounds at a time: the loads of a batch are issued together, so
// a wave pays one memory latency per batch instead of one per round (r06: the rounds were a
// chain of dependent byte loads, 84 + 150 us of count + scatter per config-4 step)
constexpr uint32_t kPartBatch = 8;
template <int MODE>
__device__ __forceinline__ void load_keys(const uint8_t *keys, uint32_t n, uint32_t base, uint32_t r0,
                                          uint32_t rounds, uint32_t k[kPartBatch]) {
#pragma unroll
    for (uint32_t j = 0; j < kPartBatch; j++) {
        const uint32_t i = base + (r0 + j) * 64u + __lane_id();
        k[j] = r0 + j < rounds && i < n ? keys[i] : no_key<MODE>();
    }
}

template <int MODE>
__device__ __forceinline__ void count_wave(const uint8_t *keys, uint32_t n, uint32_t bin_mask, uint32_t shift,
                                           uint32_t base, uint32_t rounds, uint32_t cnt[kPartMaxBins]) {
#pragma unroll
    for (int b = 0; b < kPartMaxBins; b++) cnt[b] = 0;
    for (uint32_t r0 = 0; r0 < rounds; r0 += kPartBatch) {
        uint32_t k[kPartBatch];
        load_keys<MODE>(keys, n, base, r0, rounds, k);
#pragma unroll
        for (uint32_t j = 0; j < kPartBatch; j++)
#pragma unroll
            for (int b = 0; b < kPartMaxBins; b++)
                if ((bin_mask >> b) & 1u)
                    cnt[b] += (uint32_t)__popcll(__ballot(in_bin<MODE>(k[j], (uint32_t)b, shift)));
    }
}

template <int MODE>
__global__ __launch_bounds__(kPartBlock) void k_part_count(const uint8_t *keys, uint32_t n, uint32_t nbins,
                                                           uint32_t bin_mask, uint32_t shift, uint32_t *hist,
                                                           uint32_t nblk, uint32_t rounds) {
    __shared__ uint32_t s[4][kPartMaxBins];
    const uint32_t wave = threadIdx.x >> 6;
    uint32_t cnt[kPartMaxBins];
    count_wave<MODE>(keys, n, bin_mask, shift, (blockIdx.x * 4u + wave) * 64u * rounds, rounds, cnt);
    if (__lane_id() == 0)
        for (int b = 0; b < kPartMaxBins; b++) s[wave][b] = cnt[b];
    __syncthreads();
    const uint32_t t = threadIdx.x;
    if (t < nbins) hist[t * nblk + blockIdx.x] = s[0][t] + s[1][t] + s[2][t] + s[3][t];
}

// Exclusive scan of m = nbins * nblk entries in one block of 1024 threads.
// The histogram streams through LDS in chunks of kScanChunk entries: coalesced
// loads, a serial scan of 16 consecutive entries per thread in LDS, a block
// scan of the per-thread sums, coalesced stores (the scan sits between two
// full-chip kernels, so its latency is on the frame's critical path).
constexpr uint32_t kScanPer = 16;
constexpr uint32_t kScanChunk = 1024u * kScanPer;

__global__ __launch_bounds__(1024) void k_part_scan(uint32_t *hist, uint32_t nblk, uint32_t nbins,
                                                    uint32_t *counts_out, uint32_t *starts_out,
                                                    uint32_t *total_out, uint32_t *log_out,
                                                    unsigned long long *cum_out, unsigned long long *snap_out) {
    __shared__ uint32_t sh[kScanChunk];
    __shared__ uint32_t wave_sum[16];
    __shared__ uint32_t carry_s;
    const uint32_t m = nbins * nblk;
    const uint32_t t = threadIdx.x;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < m; c0 += kScanChunk) {
        const uint32_t len = min(kScanChunk, m - c0);
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; k++) {
            const uint32_t i = k * 1024u + t;
            sh[i] = i < len ? hist[c0 + i] : 0u;
        }
        __syncthreads();
        uint32_t sum = 0;
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; k++) sum += sh[t * kScanPer + k];
        uint32_t inc = sum;  // inclusive wave scan of the per-thread sums
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(inc, o);
            if ((int)__lane_id() >= o) inc += v;
        }
        if (__lane_id() == 63) wave_sum[t >> 6] = inc;
        __syncthreads();
        if (t < 64) {
            const uint32_t w = t < 16 ? wave_sum[t] : 0u;
            uint32_t winc = w;
            for (int o = 1; o < 16; o <<= 1) {
                const uint32_t v = __shfl_up(winc, o);
                if ((int)t >= o) winc += v;
            }
            if (t < 16) wave_sum[t] = winc - w;  // exclusive wave offsets
            if (t == 15) carry_s = winc;         // chunk total
        }
        __syncthreads();
        uint32_t run = carry + wave_sum[t >> 6] + inc - sum;
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; k++) {
            const uint32_t v = sh[t * kScanPer + k];
            sh[t * kScanPer + k] = run;
            run += v;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; k++) {
            const uint32_t i = k * 1024u + t;
            if (i < len) hist[c0 + i] = sh[i];
        }
        carry += carry_s;
        __syncthreads();
    }
    __threadfence_block();
    __syncthreads();
    if (t < nbins) {
        const uint32_t start = hist[t * nblk];
        const uint32_t next = t + 1 < nbins ? hist[(t + 1) * nblk] : carry;
        starts_out[t] = start;
        counts_out[t] = next - start;
        if (log_out) log_out[t] = next - start;
        if (snap_out) snap_out[t] = cum_out[t];  // the totals before this partition
        if (cum_out) cum_out[t] += next - start;  // one block, stream-ordered: no atomics needed
    }
    if (t == 0 && total_out) *total_out = carry;
}

template <int MODE>
__global__ __launch_bounds__(kPartBlock) void k_part_scatter(const uint8_t *keys, uint32_t n, uint32_t bin_mask,
                                                             uint32_t shift, const uint32_t *hist, uint32_t nblk,
                                                             uint32_t *out, uint32_t rounds) {
    __shared__ uint32_t s[4][kPartMaxBins];
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t base = (blockIdx.x * 4u + wave) * 64u * rounds;
    uint32_t off[kPartMaxBins];
    count_wave<MODE>(keys, n, bin_mask, shift, base, rounds, off);
    if (__lane_id() == 0)
        for (int b = 0; b < kPartMaxBins; b++) s[wave][b] = off[b];
    __syncthreads();
#pragma unroll
    for (int b = 0; b < kPartMaxBins; b++) {
        if (!((bin_mask >> b) & 1u)) continue;
        uint32_t o = hist[b * nblk + blockIdx.x];
        for (uint32_t w = 0; w < wave; w++) o += s[w][b];
        off[b] = o;
    }
    for (uint32_t r0 = 0; r0 < rounds; r0 += kPartBatch) {
        uint32_t k[kPartBatch];
        load_keys<MODE>(keys, n, base, r0, rounds, k);
#pragma unroll
        for (uint32_t j = 0; j < kPartBatch; j++) {
            const uint32_t i = base + (r0 + j) * 64u + __lane_id();
#pragma unroll
            for (int b = 0; b < kPartMaxBins; b++) {
                if (!((bin_mask >> b) & 1u)) continue;
                const bool mine = in_bin<MODE>(k[j], (uint32_t)b, shift);  // no_key past n / rounds: in no bin
                const unsigned long long m = __ballot(mine);
                if (mine) out[off[b] + (uint32_t)__popcll(m & lanes_below())] = i;
                off[b] += (uint32_t)__popcll(m);
            }
        }
    }
}

}  // namespace

// part_blocks(m) <= max(kPartTargetBlocks, ceil(m / (256 * kPartMaxRounds))) for every m, a bound
// that grows with n: the scratch sized for the capacity serves every smaller batch
uint32_t partition_hist_entries(uint32_t n) {
    return kPartMaxBins * std::max(kPartTargetBlocks, (n + 256u * kPartMaxRounds - 1) / (256u * kPartMaxRounds));
}

void launch_partition(const uint8_t *keys, uint32_t n, uint32_t nbins, PartMode mode, uint32_t shift, uint32_t *out,
                      uint32_t *hist, uint32_t *counts_out, uint32_t *starts_out, uint32_t *total_out, uint32_t *log_out,
                      hipStream_t s, unsigned long long *cum_out, unsigned long long *snap_out, uint32_t bin_mask) {
    // the bins a key can name (the others are counted as empty without a ballot each)
    const uint32_t all = (1u << nbins) - 1u;
    bin_mask = bin_mask ? (bin_mask & all) : all;
    const uint32_t nblk = part_blocks(n);
    const uint32_t rounds = part_rounds(n);
    if (nblk == 0) {
        (void)hipMemsetAsync(counts_out, 0, sizeof(uint32_t) * nbins, s);
        (void)hipMemsetAsync(starts_out, 0, sizeof(uint32_t) * nbins, s);
        if (total_out) (void)hipMemsetAsync(total_out, 0, sizeof(uint32_t), s);
        if (log_out) (void)hipMemsetAsync(log_out, 0, sizeof(uint32_t) * nbins, s);
        if (snap_out && cum_out)
            (void)hipMemcpyAsync(snap_out, cum_out, sizeof(unsigned long long) * nbins, hipMemcpyDeviceToDevice, s);
        return;
    }
#define PART_RUN(M)                                                                                                \
    hipLaunchKernelGGL(k_part_count<M>, dim3(nblk), dim3(kPartBlock), 0, s, keys, n, nbins, bin_mask, shift, hist, \
                       nblk, rounds);                                                                                    \
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(1024), 0, s, hist, nblk, nbins, counts_out, starts_out,          \
                       total_out, log_out, cum_out, snap_out);                                                                      \
    hipLaunchKernelGGL(k_part_scatter<M>, dim3(nblk), dim3(kPartBlock), 0, s, keys, n, bin_mask, shift, hist, nblk, \
                       out, rounds)
    switch (mode) {
    case kPartExclusive: PART_RUN(kPartExclusive); break;
    case kPartFlags: PART_RUN(kPartFlags); break;
    }
#undef PART_RUN
}

}  // namespace pupil
