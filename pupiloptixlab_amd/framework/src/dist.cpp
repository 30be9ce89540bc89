// dist.cpp — RCCL tile gather of the C++ drop-in (see pupil/dist.h).
#include "pupil/dist.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include <cerrno>

#include <dirent.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../../include/pupil_pt.h"
#include "pupil/framework.h"

namespace Pupil {

namespace {

int env_int(const char *name, int def) {
    const char *v = std::getenv(name);
    return v && *v ? std::atoi(v) : def;
}

constexpr char kIdMagic[8] = {'P', 'U', 'P', 'I', 'L', 'I', 'D', '2'};

// start time of process `pid` in clock ticks since boot (/proc/<pid>/stat field 22), 0 when
// it does not exist: (pid, start time) names one process for the lifetime of the host
uint64_t proc_start_ticks(long pid) {
    char path[64];
    std::snprintf(path, sizeof(path), "/proc/%ld/stat", pid);
    FILE *f = std::fopen(path, "r");
    if (!f) return 0;
    char buf[1024];
    const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
    std::fclose(f);
    buf[n] = '\0';
    const char *p = std::strrchr(buf, ')');  // the command name may hold spaces and parentheses
    if (!p) return 0;
    unsigned long long v = 0;
    // fields 3..21 after the name, then 22 = starttime
    if (std::sscanf(p + 2, "%*c %*d %*d %*d %*d %*d %*u %*u %*u %*u %*u %*u %*u %*d %*d %*d %*d %*d %*d %llu", &v) != 1)
        return 0;
    return v;
}

// wall-clock start of this process (boot time + its start ticks), 0 when unknown
int64_t self_start_wall() {
    FILE *f = std::fopen("/proc/stat", "r");
    if (!f) return 0;
    char line[256];
    long long btime = 0;
    while (std::fgets(line, sizeof(line), f))
        if (std::sscanf(line, "btime %lld", &btime) == 1) break;
    std::fclose(f);
    const long hz = sysconf(_SC_CLK_TCK);
    const uint64_t ticks = proc_start_ticks((long)getpid());
    return btime > 0 && hz > 0 && ticks ? (int64_t)btime + (int64_t)(ticks / (uint64_t)hz) : 0;
}

// an id file whose writer ran on another host (shared filesystem) cannot be checked for
// liveness: it is taken only if written no earlier than kRemoteIdSlack seconds before this
// reader started, so a file a crashed launch left long ago is never read
constexpr int64_t kRemoteIdSlack = 60;

std::string host_name() {
    char h[256] = {0};
    if (gethostname(h, sizeof(h) - 1) != 0) return "?";
    return h;
}

bool write_str(FILE *f, const std::string &s) {
    const uint32_t n = (uint32_t)s.size();
    return std::fwrite(&n, sizeof(n), 1, f) == 1 && (n == 0 || std::fwrite(s.data(), n, 1, f) == 1);
}
bool read_str(FILE *f, std::string &s, uint32_t max) {
    uint32_t n = 0;
    if (std::fread(&n, sizeof(n), 1, f) != 1 || n > max) return false;
    s.assign(n, '\0');
    return n == 0 || std::fread(s.data(), n, 1, f) == 1;
}

// rank 0 -> the others: the 128-byte ncclUniqueId through a file, renamed into place.
// The file carries the launch nonce (DistLaunchNonce): a file left by an earlier or
// another launch -- a crashed run, another job on the same MASTER_PORT -- has another
// nonce and is never used; the other ranks keep waiting for rank 0 to replace it.
bool exchange_id(const DistInfo &d, const std::string &path, ncclUniqueId &id) {
    const std::string nonce = DistLaunchNonce();
    if (d.rank == 0) {
        if (ncclGetUniqueId(&id) != ncclSuccess) return false;
        return WriteIdFile(path, nonce, &id, sizeof(id));
    }
    const auto t0 = std::chrono::steady_clock::now();
    bool warned = false;
    for (;;) {
        const int r = ReadIdFile(path, nonce, &id, sizeof(id));
        if (r > 0) return true;
        if (r < 0 && !warned) {
            Log("rank %d: ignoring %s, left by another launch (waiting for rank 0)", d.rank, path.c_str());
            warned = true;
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

std::string DistLaunchNonce() noexcept {
    if (const char *n = std::getenv("PUPIL_RCCL_NONCE"); n && *n) return n;
    // launch-wide environment only: the ranks of one launch agree on it however each rank
    // was started (torchrun, mpirun, a slurm step, or a `timeout` wrapper per rank, whose
    // parent processes differ), and another launch differs in its run id / restart count /
    // job step / port.  A stale file of an earlier launch with the same environment is
    // rejected by its writer's liveness on the same host, and by its age against this
    // process's start for a writer on another host (ReadIdFile).
    auto env = [](const char *k) {
        const char *v = std::getenv(k);
        return std::string(v && *v ? v : "-");
    };
    std::string n;
    for (const char *k : {"MASTER_ADDR", "MASTER_PORT", "WORLD_SIZE", "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT",
                          "SLURM_JOB_ID", "SLURM_STEP_ID"})
        n += env(k) + ".";
    return n;
}

std::string DistIdPath() noexcept {
    if (const char *p = std::getenv("PUPIL_RCCL_ID_FILE"); p && *p) return p;
    const char *port = std::getenv("MASTER_PORT");
    const std::string nonce = DistLaunchNonce();
    uint64_t h = 1469598103934665603ull;  // FNV-1a of the nonce: one file per launch
    for (unsigned char c : nonce) h = (h ^ c) * 1099511628211ull;
    char hex[17];
    std::snprintf(hex, sizeof(hex), "%016llx", (unsigned long long)h);
    return "/tmp/pupil_rccl_" + std::string(port && *port ? port : "0") + "_" + hex + ".id";
}

bool WriteIdFile(const std::string &path, const std::string &nonce, const void *id, size_t size) noexcept {
    (void)std::remove(path.c_str());  // no reader may see a previous launch's id while this one is written
    const std::string tmp = path + ".tmp" + std::to_string((long long)getpid());
    FILE *f = std::fopen(tmp.c_str(), "wb");
    if (!f) return false;
    const int64_t pid = (int64_t)getpid();
    const uint64_t start = proc_start_ticks((long)pid);
    bool ok = std::fwrite(kIdMagic, sizeof(kIdMagic), 1, f) == 1 && write_str(f, nonce) && write_str(f, host_name()) &&
              std::fwrite(&pid, sizeof(pid), 1, f) == 1 && std::fwrite(&start, sizeof(start), 1, f) == 1 &&
              std::fwrite(id, size, 1, f) == 1;
    ok = std::fclose(f) == 0 && ok;
    if (!ok) {
        (void)std::remove(tmp.c_str());
        return false;
    }
    return std::rename(tmp.c_str(), path.c_str()) == 0;
}

int ReadIdFile(const std::string &path, const std::string &nonce, void *id, size_t size) noexcept {
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) return 0;
    char magic[8];
    std::string got, host;
    int64_t pid = 0;
    uint64_t start = 0;
    int r = -1;
    if (std::fread(magic, sizeof(magic), 1, f) == 1 && std::memcmp(magic, kIdMagic, sizeof(magic)) == 0 &&
        read_str(f, got, 4096) && got == nonce) {
        // the rest may still be missing (a torn file reads as absent, the reader waits)
        if (read_str(f, host, 255) && std::fread(&pid, sizeof(pid), 1, f) == 1 &&
            std::fread(&start, sizeof(start), 1, f) == 1 && std::fread(id, size, 1, f) == 1) {
            // a writer on this host must still run (rank 0 waits in ncclCommInitRank until every
            // rank has joined); on a shared filesystem another host's file must be no older than
            // this reader's start less kRemoteIdSlack (a relaunch within that window on another
            // host with the same environment can still meet the earlier launch's file)
            if (host == host_name()) {
                r = start != 0 && proc_start_ticks((long)pid) == start ? 1 : -1;
            } else {
                struct stat st;
                const int64_t t0 = self_start_wall();
                r = fstat(fileno(f), &st) == 0 && (t0 == 0 || (int64_t)st.st_mtime >= t0 - kRemoteIdSlack) ? 1 : -1;
            }
        } else {
            r = 0;
        }
    }
    std::fclose(f);
    return r;
}

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
    if (m_host && m_info.rank == 0) {  // empty once every frame was consumed
        (void)std::remove((m_dir + "/ready").c_str());
        (void)rmdir(m_dir.c_str());
    }
    if (m_comm) (void)ncclCommDestroy(m_comm);
}

void FrameGather::Release() noexcept {
    for (auto *p : m_maps)
        if (p) (void)hipFree(p);
    for (auto *p : m_staging)
        if (p) (void)hipFree(p);
    for (auto *p : m_pinned)
        if (p) (void)hipHostFree(p);
    m_maps.clear();
    m_staging.clear();
    m_pinned.clear();
}

bool FrameGather::Init(const DistInfo &d, int device, const std::string &id_path) noexcept {
    m_info = d;
    if (hipSetDevice(device) != hipSuccess) return false;
    if (const char *tr = std::getenv("PUPIL_GATHER_TRANSPORT"); tr && std::strcmp(tr, "host") == 0) {
        // test transport (dist.h): a per-launch directory instead of a communicator
        m_host = true;
        m_dir = id_path + ".d";
        if (mkdir(m_dir.c_str(), 0700) != 0 && errno != EEXIST) {
            Log("rank %d: cannot create %s", d.rank, m_dir.c_str());
            return false;
        }
        // rank 0 empties the directory (tile files a crashed earlier run left) and then
        // publishes a `ready` marker naming itself; the other ranks write no tiles before that
        // marker exists with a live writer, so no stale f<r>_<frame> is ever read
        const std::string ready = m_dir + "/ready";
        if (d.rank == 0) {
            if (DIR *dir = opendir(m_dir.c_str())) {
                while (dirent *e = readdir(dir))
                    if (std::strcmp(e->d_name, ".") != 0 && std::strcmp(e->d_name, "..") != 0)
                        (void)std::remove((m_dir + "/" + e->d_name).c_str());
                closedir(dir);
            }
            if (!WriteIdFile(ready, DistLaunchNonce(), &d.world, sizeof(d.world))) return false;
        } else {
            int world = 0;
            const auto t0 = std::chrono::steady_clock::now();
            while (ReadIdFile(ready, DistLaunchNonce(), &world, sizeof(world)) <= 0) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) {
                    Log("rank %d: no live rank 0 behind %s", d.rank, ready.c_str());
                    return false;
                }
                std::this_thread::sleep_for(std::chrono::milliseconds(2));
            }
        }
        Log("rank %d of %d: host-staged tile gather through %s (test transport)", d.rank, d.world, m_dir.c_str());
        return true;
    }
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
    if (m_info.rank != 0) {
        if (!m_host) return true;
        m_pinned.assign(1, nullptr);  // this rank's tiles on their way to the exchange file
        return hipHostMalloc((void **)&m_pinned[0], sizeof(float4) * std::max(1u, m_counts[(size_t)m_info.rank])) ==
               hipSuccess;
    }
    m_maps.assign(world, nullptr);
    m_staging.assign(world, nullptr);
    if (m_host) m_pinned.assign(world, nullptr);
    for (uint32_t r = 0; r < world; r++) {
        std::vector<uint32_t> map(std::max(1u, m_counts[r]));
        uint32_t n = m_counts[r];
        if (pupil_pt_local_pixels(width, height, m_info.tile, r, world, map.data(), &n) != PUPIL_OK) return false;
        if (hipMalloc((void **)&m_maps[r], sizeof(uint32_t) * map.size()) != hipSuccess ||
            hipMemcpy(m_maps[r], map.data(), sizeof(uint32_t) * map.size(), hipMemcpyHostToDevice) != hipSuccess ||
            hipMalloc((void **)&m_staging[r], sizeof(float4) * map.size()) != hipSuccess ||
            (m_host && r > 0 && hipHostMalloc((void **)&m_pinned[r], sizeof(float4) * map.size()) != hipSuccess))
            return false;
    }
    return true;
}

// Test transport: rank r != 0 copies its tiles to pinned memory and publishes them as
// <dir>/f<r>_<frame> (complete temporary renamed into place), after rank 0 consumed its
// previous frame; rank 0 waits for every rank's file of this frame, uploads it into the
// staging buffer and removes it.  Every wait is bounded (120 s).
bool FrameGather::GatherHost(const void *local, hipStream_t stream) noexcept {
    const int world = m_info.world;
    auto name = [&](int r, uint64_t f) { return m_dir + "/f" + std::to_string(r) + "_" + std::to_string(f); };
    auto wait_for = [&](const std::string &path, bool present) {
        const auto t0 = std::chrono::steady_clock::now();
        struct stat st;
        while ((stat(path.c_str(), &st) == 0) != present) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) return false;
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
        return true;
    };
    const uint64_t frame = m_frame++;
    if (m_info.rank != 0) {
        const size_t bytes = sizeof(float4) * m_counts[(size_t)m_info.rank];
        if (frame > 0 && !wait_for(name(m_info.rank, frame - 1), false)) return false;
        if (hipMemcpyAsync(m_pinned[0], local, bytes, hipMemcpyDeviceToHost, stream) != hipSuccess ||
            hipStreamSynchronize(stream) != hipSuccess)
            return false;
        const std::string tmp = name(m_info.rank, frame) + ".tmp";
        FILE *f = std::fopen(tmp.c_str(), "wb");
        if (!f) return false;
        const bool written = bytes == 0 || std::fwrite(m_pinned[0], bytes, 1, f) == 1;
        const bool closed = std::fclose(f) == 0;
        return written && closed && std::rename(tmp.c_str(), name(m_info.rank, frame).c_str()) == 0;
    }
    for (int r = 1; r < world; r++) {
        const size_t bytes = sizeof(float4) * m_counts[(size_t)r];
        const std::string path = name(r, frame);
        if (!wait_for(path, true)) {
            Log("rank 0: no tiles from rank %d for frame %llu", r, (unsigned long long)frame);
            return false;
        }
        FILE *f = std::fopen(path.c_str(), "rb");
        const bool ok = f && (bytes == 0 || std::fread(m_pinned[(size_t)r], bytes, 1, f) == 1);
        if (f) std::fclose(f);
        (void)std::remove(path.c_str());
        if (!ok || hipMemcpyAsync(m_staging[(size_t)r], m_pinned[(size_t)r], bytes, hipMemcpyHostToDevice, stream) !=
                       hipSuccess)
            return false;
    }
    // the pinned buffers are rewritten by the next frame's reads: the uploads must have run
    return hipStreamSynchronize(stream) == hipSuccess;
}

bool FrameGather::Gather(const void *local, void *full, hipStream_t stream) noexcept {
    const int world = m_info.world;
    if (m_host) {
        if (!GatherHost(local, stream)) return false;
        return m_info.rank != 0 || Scatter(local, full, stream);
    }
    if (!m_comm) return false;
    if (ncclGroupStart() != ncclSuccess) return false;
    bool posted = true;
    if (m_info.rank == 0) {
        for (int r = 1; r < world && posted; r++)
            posted = ncclRecv(m_staging[(size_t)r], 4 * (size_t)m_counts[(size_t)r], ncclFloat32, r, m_comm, stream) ==
                     ncclSuccess;
    } else {
        posted = ncclSend(local, 4 * (size_t)m_counts[(size_t)m_info.rank], ncclFloat32, 0, m_comm, stream) ==
                 ncclSuccess;
    }
    // the group is closed on every path (an open group would swallow the next RCCL calls)
    if (ncclGroupEnd() != ncclSuccess || !posted) return false;
    return m_info.rank != 0 || Scatter(local, full, stream);
}

// rank 0: every rank's compact tiles (its own from `local`, the others' received into the
// staging buffers) into the full frame, one kernel per rank
bool FrameGather::Scatter(const void *local, void *full, hipStream_t stream) noexcept {
    for (int r = 0; r < m_info.world; r++) {
        const uint32_t n = m_counts[(size_t)r];
        if (!n) continue;
        const float4 *src = r == 0 ? static_cast<const float4 *>(local) : reinterpret_cast<const float4 *>(m_staging[(size_t)r]);
        hipLaunchKernelGGL(k_scatter_tiles, dim3((n + 255) / 256), dim3(256), 0, stream, src, m_maps[(size_t)r], n,
                           static_cast<float4 *>(full));
    }
    return hipGetLastError() == hipSuccess;
}

}  // namespace Pupil

// C hooks for the CPU tests of the id-file protocol (tests/test_cpp_host.py)
extern "C" int pupil_dist_write_id_file(const char *path, const char *nonce, const void *id128) {
    return Pupil::WriteIdFile(path, nonce, id128, 128) ? 0 : -1;
}
extern "C" int pupil_dist_read_id_file(const char *path, const char *nonce, void *id128) {
    return Pupil::ReadIdFile(path, nonce, id128, 128);
}
extern "C" int pupil_dist_id_path(char *out, size_t size) {
    const std::string p = Pupil::DistIdPath();
    if (!out || size <= p.size()) return -1;
    std::memcpy(out, p.c_str(), p.size() + 1);
    return 0;
}
