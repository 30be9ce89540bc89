// dist.cpp — RCCL tile gather of the C++ drop-in (see pupil/dist.h).
#include "pupil/dist.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "../../../include/pupil_pt.h"
#include "pupil/framework.h"

namespace Pupil {

namespace {

int env_int(const char *name, int def) {
    const char *v = std::getenv(name);
    return v && *v ? std::atoi(v) : def;
}

// rank 0 -> the others: the 128-byte ncclUniqueId through a file, renamed into place
bool exchange_id(const DistInfo &d, const std::string &path, ncclUniqueId &id) {
    if (d.rank == 0) {
        if (ncclGetUniqueId(&id) != ncclSuccess) return false;
        const std::string tmp = path + ".tmp";
        FILE *f = std::fopen(tmp.c_str(), "wb");
        if (!f) return false;
        const bool ok = std::fwrite(&id, sizeof(id), 1, f) == 1;
        if (std::fclose(f) != 0 || !ok) return false;
        return std::rename(tmp.c_str(), path.c_str()) == 0;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        if (FILE *f = std::fopen(path.c_str(), "rb")) {
            const bool ok = std::fread(&id, sizeof(id), 1, f) == 1;
            std::fclose(f);
            if (ok) return true;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) return false;
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
}

__global__ void k_scatter_tiles(const float4 *src, const uint32_t *map, uint32_t n, float4 *full) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) full[map[i]] = src[i];
}

}  // namespace

DistInfo DistFromEnv() noexcept {
    DistInfo d;
    d.world = std::max(1, env_int("WORLD_SIZE", 1));
    d.rank = env_int("RANK", 0);
    d.local_rank = env_int("LOCAL_RANK", d.rank);
    if (d.rank < 0 || d.rank >= d.world) d = DistInfo{};
    return d;
}

FrameGather::~FrameGather() noexcept {
    Release();
    if (m_comm) (void)ncclCommDestroy(m_comm);
}

void FrameGather::Release() noexcept {
    for (auto *p : m_maps)
        if (p) (void)hipFree(p);
    for (auto *p : m_staging)
        if (p) (void)hipFree(p);
    m_maps.clear();
    m_staging.clear();
}

bool FrameGather::Init(const DistInfo &d, int device, const std::string &id_path) noexcept {
    m_info = d;
    if (hipSetDevice(device) != hipSuccess) return false;
    ncclUniqueId id;
    if (!exchange_id(d, id_path, id)) {
        Log("rank %d: RCCL unique id exchange through %s failed", d.rank, id_path.c_str());
        return false;
    }
    const ncclResult_t r = ncclCommInitRank(&m_comm, d.world, id, d.rank);
    if (r != ncclSuccess) {
        Log("rank %d: ncclCommInitRank failed: %s", d.rank, ncclGetErrorString(r));
        m_comm = nullptr;
        return false;
    }
    if (d.rank == 0) std::remove(id_path.c_str());  // every rank has joined
    return true;
}

bool FrameGather::Setup(uint32_t width, uint32_t height) noexcept {
    Release();
    m_w = width;
    m_h = height;
    const uint32_t world = (uint32_t)m_info.world;
    m_counts.assign(world, 0);
    for (uint32_t r = 0; r < world; r++) {
        uint32_t n = 0;
        if (pupil_pt_local_pixels(width, height, m_info.tile, r, world, nullptr, &n) != PUPIL_OK) return false;
        m_counts[r] = n;
    }
    if (m_info.rank != 0) return true;
    m_maps.assign(world, nullptr);
    m_staging.assign(world, nullptr);
    for (uint32_t r = 0; r < world; r++) {
        std::vector<uint32_t> map(std::max(1u, m_counts[r]));
        uint32_t n = m_counts[r];
        if (pupil_pt_local_pixels(width, height, m_info.tile, r, world, map.data(), &n) != PUPIL_OK) return false;
        if (hipMalloc((void **)&m_maps[r], sizeof(uint32_t) * map.size()) != hipSuccess ||
            hipMemcpy(m_maps[r], map.data(), sizeof(uint32_t) * map.size(), hipMemcpyHostToDevice) != hipSuccess ||
            hipMalloc((void **)&m_staging[r], sizeof(float4) * map.size()) != hipSuccess)
            return false;
    }
    return true;
}

bool FrameGather::Gather(const void *local, void *full, hipStream_t stream) noexcept {
    if (!m_comm) return false;
    const int world = m_info.world;
    if (ncclGroupStart() != ncclSuccess) return false;
    if (m_info.rank == 0) {
        for (int r = 1; r < world; r++)
            if (ncclRecv(m_staging[(size_t)r], 4 * (size_t)m_counts[(size_t)r], ncclFloat32, r, m_comm, stream) !=
                ncclSuccess)
                return false;
    } else if (ncclSend(local, 4 * (size_t)m_counts[(size_t)m_info.rank], ncclFloat32, 0, m_comm, stream) !=
               ncclSuccess) {
        return false;
    }
    if (ncclGroupEnd() != ncclSuccess) return false;
    if (m_info.rank != 0) return true;
    for (int r = 0; r < world; r++) {
        const uint32_t n = m_counts[(size_t)r];
        if (!n) continue;
        const float4 *src = r == 0 ? static_cast<const float4 *>(local) : reinterpret_cast<const float4 *>(m_staging[(size_t)r]);
        hipLaunchKernelGGL(k_scatter_tiles, dim3((n + 255) / 256), dim3(256), 0, stream, src, m_maps[(size_t)r], n,
                           static_cast<float4 *>(full));
    }
    return hipGetLastError() == hipSuccess;
}

}  // namespace Pupil
