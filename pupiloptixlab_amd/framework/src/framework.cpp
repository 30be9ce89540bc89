// framework.cpp — Pass timing, BufferManager, event table, headless System.
#include "pupil/framework.h"

#include <chrono>
#include <cstdarg>
#include <cstdio>

#include "pupil/world.h"

namespace Pupil {

void Log(const char *fmt, ...) noexcept {
    std::va_list ap;
    va_start(ap, fmt);
    std::fputs("[pupil] ", stderr);
    std::vfprintf(stderr, fmt, ap);
    std::fputc('\n', stderr);
    va_end(ap);
}

// ---------------------------------------------------------------- Pass
void Pass::Run() noexcept {
    if (!m_enable) return;
    const auto t0 = std::chrono::steady_clock::now();
    OnRun();
    m_last_exec_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void Pass::Inspector() noexcept { Log("%s: %.3f ms", name.c_str(), m_last_exec_ms); }

// ---------------------------------------------------------------- buffers
Buffer::~Buffer() noexcept {
    if (cuda_ptr) (void)hipFree(cuda_ptr);
}

Buffer *BufferManager::AllocBuffer(const BufferDesc &desc) noexcept {
    const size_t bytes = (size_t)desc.width * desc.height * desc.stride_in_byte;
    auto it = m_buffers.find(desc.name);
    if (it != m_buffers.end() && it->second->bytes == bytes) {
        it->second->desc = desc;
        (void)hipMemset(it->second->cuda_ptr, 0, bytes);
        return it->second.get();
    }
    auto buf = std::make_unique<Buffer>();
    buf->desc = desc;
    buf->bytes = bytes;
    if (bytes && (hipMalloc(&buf->cuda_ptr, bytes) != hipSuccess || hipMemset(buf->cuda_ptr, 0, bytes) != hipSuccess)) {
        Log("buffer '%s': device allocation of %zu bytes failed", desc.name.c_str(), bytes);
        buf->cuda_ptr = nullptr;
        return nullptr;
    }
    Buffer *raw = buf.get();
    if (it == m_buffers.end()) m_names.push_back(desc.name);
    m_buffers[desc.name] = std::move(buf);
    return raw;
}

Buffer *BufferManager::GetBuffer(std::string_view name) noexcept {
    auto it = m_buffers.find(name);
    return it == m_buffers.end() ? nullptr : it->second.get();
}

void BufferManager::Destroy() noexcept {
    m_buffers.clear();
    m_names.clear();
}

// ---------------------------------------------------------------- events
namespace detail {
void EventTable::Bind(uint64_t key, std::function<void(void *)> fn) noexcept {
    std::scoped_lock lock(m_mutex);
    m_handlers[key].push_back(std::move(fn));
}

void EventTable::Fire(uint64_t key, void *arg) noexcept {
    std::vector<std::function<void(void *)>> handlers;
    {
        std::scoped_lock lock(m_mutex);
        auto it = m_handlers.find(key);
        if (it == m_handlers.end()) return;
        handlers = it->second;
    }
    for (auto &h : handlers) h(arg);
}
}  // namespace detail

// ---------------------------------------------------------------- System
void System::Init(bool has_window) noexcept {
    (void)has_window;
    if (hipSetDevice(device) != hipSuccess) Log("hipSetDevice(%d) failed", device);
}

void System::AddPass(Pass *pass) noexcept {
    if (pass) m_passes.push_back(pass);
}

bool System::SetScene(const std::filesystem::path &xml) noexcept {
    auto w = std::make_unique<world::World>();
    if (!w->LoadScene(xml)) return false;
    return SetScene(std::move(w));
}

bool System::InitDistributed(const DistInfo &d) noexcept {
    device = d.local_rank;
    auto g = std::make_unique<FrameGather>();
    if (!g->Init(d, device, DistIdPath())) return false;
    m_gather = std::move(g);
    return true;
}

bool System::SetScene(std::unique_ptr<world::World> w) noexcept {
    if (!w) return false;
    std::scoped_lock render_lock(m_render_system_mutex);  // system.cpp:145
    (void)hipSetDevice(device);
    if (m_gather && !m_gather->Setup((uint32_t)w->scene->sensor.film.w, (uint32_t)w->scene->sensor.film.h)) {
        Log("tile maps for the multi-GPU gather could not be set up");
        return false;
    }
    BufferDesc desc;
    desc.name = std::string(BufferManager::DEFAULT_FINAL_RESULT_BUFFER_NAME);
    desc.flag = EBufferFlag::AllowDisplay;
    desc.width = (uint32_t)w->scene->sensor.film.w;
    desc.height = (uint32_t)w->scene->sensor.film.h;
    desc.stride_in_byte = sizeof(float) * 4;
    if (!BufferManager::instance()->AllocBuffer(desc)) return false;
    m_world = std::move(w);
    EventDispatcher<ESystemEvent::SceneLoad>(m_world.get());
    return true;
}

void System::RenderFrame() noexcept {
    for (Pass *p : m_passes) p->Run();
    m_frames++;
}

void System::Run(uint32_t frames) noexcept {
    (void)hipSetDevice(device);
    for (uint32_t f = 0; f < frames; f++) {
        {
            std::scoped_lock render_lock(m_render_system_mutex);
            RenderFrame();
        }
        EventDispatcher<ESystemEvent::FrameFinished>();
    }
}

void System::RunAsync() noexcept {
    if (m_render_thread.joinable()) return;
    m_quit = false;
    m_render_thread = std::thread([this] {
        (void)hipSetDevice(device);  // HIP's current device is per thread
        while (!m_quit) {
            while (m_lock_waiters.load() > 0 && !m_quit) std::this_thread::yield();  // no starvation
            {
                std::scoped_lock render_lock(m_render_system_mutex);
                if (m_quit) break;
                RenderFrame();
            }
            EventDispatcher<ESystemEvent::FrameFinished>();
        }
    });
}

std::unique_lock<std::mutex> System::RenderLock() noexcept {
    m_lock_waiters++;
    std::unique_lock<std::mutex> lock(m_render_system_mutex);
    m_lock_waiters--;
    return lock;
}

void System::Stop() noexcept {
    m_quit = true;
    if (m_render_thread.joinable()) m_render_thread.join();
}

void System::Destroy() noexcept {
    Stop();
    EventDispatcher<ESystemEvent::Quit>();
    m_passes.clear();
    m_world.reset();
    m_gather.reset();
    BufferManager::instance()->Destroy();
}

}  // namespace Pupil
