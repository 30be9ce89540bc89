// dist.h — multi-GPU sharding of the drop-in (BASELINE.json north_star: image-space
// tiles across the GPUs of one node, scene replicated in HBM, per-tile radiance
// gathered over RCCL).  The reference is single-GPU; each pixel's path depends only
// on (pixel_index, random_seed) and the read-only scene (example/path_tracer/
// main.cu:40,53), so ranks render disjoint tile sets of the same frame and the
// result is bit-identical to one GPU.
//
// One process per GPU, launched like torchrun does (RANK, WORLD_SIZE, LOCAL_RANK,
// MASTER_PORT in the environment).  Tile t (32 x 32, row-major) belongs to rank
// t % world (pupil_pt_local_pixels).  Once per OnRun every rank sends its compact
// "final result" tiles to rank 0 (ncclSend / ncclRecv in one group: one message
// per rank, ~4 MB at 1080p and 8 GPUs, over xGMI), and rank 0 scatters them into
// its full-frame "final result" with one kernel.  No collective sits inside the
// render; the gather is the only exchange.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <string>
#include <vector>

namespace Pupil {

struct DistInfo {
    int rank = 0;
    int world = 1;
    int local_rank = 0;
    uint32_t tile = 32;
};

// RANK / WORLD_SIZE / LOCAL_RANK (torchrun's variables); world = 1 without them.
DistInfo DistFromEnv() noexcept;

// Identity of this launch, the same on every rank of it however each rank was started:
// launch-wide environment only (MASTER_ADDR / MASTER_PORT, WORLD_SIZE,
// TORCHELASTIC_RUN_ID / _RESTART_COUNT, SLURM_JOB_ID / _STEP_ID); PUPIL_RCCL_NONCE
// overrides it.
std::string DistLaunchNonce() noexcept;
// Node-local file through which rank 0 hands its ncclUniqueId to the other ranks:
// PUPIL_RCCL_ID_FILE, else /tmp/pupil_rccl_<MASTER_PORT>_<hash of the nonce>.id.
std::string DistIdPath() noexcept;
// The id file: magic, the launch nonce, the writer (host name, pid and the process start
// time in clock ticks since boot, /proc/<pid>/stat field 22), the id.  Write removes any
// previous file first and renames a complete temporary into place.  Read returns 1 (id of
// this launch), 0 (absent or incomplete) or -1 (never used: another launch's nonce, or a
// writer on this host that is no longer running -- a crashed or finished earlier launch
// with the same environment).  No wall clock is compared, so ranks may start any time apart.
bool WriteIdFile(const std::string &path, const std::string &nonce, const void *id, size_t size) noexcept;
int ReadIdFile(const std::string &path, const std::string &nonce, void *id, size_t size) noexcept;

class FrameGather {
public:
    FrameGather() noexcept = default;
    ~FrameGather() noexcept;
    FrameGather(const FrameGather &) = delete;
    FrameGather &operator=(const FrameGather &) = delete;

    // Collective over all ranks: rank 0 creates the RCCL unique id and hands it to
    // the others through `id_path` (a file on the node's local filesystem, written
    // atomically); every rank then joins the communicator on `device`.
    bool Init(const DistInfo &d, int device, const std::string &id_path) noexcept;
    // PUPIL_GATHER_TRANSPORT=host (tests only, never the default): no RCCL communicator;
    // every rank stages its compact tiles through pinned host memory and a file in a
    // per-launch directory (DistIdPath() + ".d"), which rank 0 reads back.  It lets N rank
    // processes share ONE GPU (RCCL refuses two ranks on one device), so the rank != 0 paths
    // of Gather and PTPass::SetScene run on a single-GPU box; the frames are bit-identical
    // to the RCCL transport's (the same bytes move).
    // Per frame size: the tile maps of every rank (rank 0 keeps them on the device).
    bool Setup(uint32_t width, uint32_t height) noexcept;
    // Gathers every rank's compact float4 buffer (this rank's `LocalPixels()` pixels,
    // in map order) into rank 0's full float4 image on `stream`; asynchronous.
    bool Gather(const void *local, void *full, hipStream_t stream) noexcept;

    uint32_t LocalPixels() const noexcept { return m_counts.empty() ? 0u : m_counts[(size_t)m_info.rank]; }
    const DistInfo &Info() const noexcept { return m_info; }

private:
    DistInfo m_info{};
    ncclComm_t m_comm = nullptr;
    uint32_t m_w = 0, m_h = 0;
    std::vector<uint32_t> m_counts;   // pixels per rank
    std::vector<uint32_t *> m_maps;   // rank 0: device pixel map per rank
    std::vector<float *> m_staging;   // rank 0: received compact buffers per rank
    // host transport (tests): exchange directory, frames gathered so far, pinned staging
    bool m_host = false;
    std::string m_dir;
    uint64_t m_frame = 0;
    std::vector<float *> m_pinned;    // rank 0: one per rank; others: their own tiles
    bool GatherHost(const void *local, hipStream_t stream) noexcept;
    bool Scatter(const void *local, void *full, hipStream_t stream) noexcept;
    void Release() noexcept;
};

}  // namespace Pupil
