// framework.h — headless C++ host layer of the MI355X path tracer, above the
// C ABI of include/pupil_pt.h.  It keeps the reference's host-side names and
// call pattern so example/path_tracer code drops in:
//   Pass / EPassTag          framework/system/pass.h:6-39   (Run() times OnRun(), pass.cpp:6-11)
//   BufferDesc / Buffer /    framework/system/buffer.h:21-63 (named device buffers; "final result"
//   BufferManager                                            allocated by System::SetScene, system.cpp:151-161)
//   EventBinder /            framework/util/event.h         (ESystemEvent::SceneLoad, EWorldEvent::*)
//   EventDispatcher
//   System                   framework/system/system.h:22-41 (Init / AddPass / SetScene / Run / Destroy)
// The GUI, DX12 interop and the window loop are out of scope:
// System::Run renders a fixed number of frames.  Like the reference, nothing
// here throws; failures are logged to stderr and reported by return values.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <filesystem>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <vector>
#include <atomic>

#include "../../../../include/pupil_pt.h"
#include "dist.h"

namespace Pupil {

namespace util {
// Process-wide instance, created on first use.
template <class T>
class Singleton {
public:
    static T *instance() noexcept {
        static T obj;
        return &obj;
    }
};
}  // namespace util

void Log(const char *fmt, ...) noexcept;  // "[pupil] ..." on stderr

// ---------------------------------------------------------------- passes
enum class EPassTag : uint32_t { None = 0, Pre = 1u << 0, Post = 1u << 1, Asyn = 1u << 2 };

class Pass {
public:
    const std::string name;
    const EPassTag tag;

    explicit Pass(std::string_view pass_name, EPassTag pass_tag = EPassTag::None) noexcept
        : name(pass_name), tag(pass_tag) {}
    virtual ~Pass() noexcept = default;

    virtual void Run() noexcept;        // OnRun() when enabled, wall time recorded
    virtual void Inspector() noexcept;  // headless: one status line
    virtual void OnRun() noexcept = 0;

    void Toggle() noexcept { m_enable = !m_enable; }
    void SetEnablility(bool enable) noexcept { m_enable = enable; }
    bool IsEnabled() const noexcept { return m_enable; }
    double LastExecTimeMs() const noexcept { return m_last_exec_ms; }

protected:
    double m_last_exec_ms = 0.0;
    bool m_enable = true;
};

// ---------------------------------------------------------------- buffers
enum class EBufferFlag : uint32_t { None = 0, AllowDisplay = 1u << 0 };

struct BufferDesc {
    std::string name;
    EBufferFlag flag = EBufferFlag::None;
    uint32_t width = 1;
    uint32_t height = 1;
    uint32_t stride_in_byte = 1;
};

// `cuda_ptr` keeps the reference's field name; it is a HIP device pointer in HBM.
struct Buffer {
    BufferDesc desc;
    void *cuda_ptr = nullptr;
    size_t bytes = 0;
    ~Buffer() noexcept;
};

class BufferManager : public util::Singleton<BufferManager> {
public:
    static constexpr std::string_view DEFAULT_FINAL_RESULT_BUFFER_NAME = "final result";

    // (Re)allocates `desc.name`, zero-filled; returns nullptr on failure.
    Buffer *AllocBuffer(const BufferDesc &desc) noexcept;
    Buffer *GetBuffer(std::string_view name) noexcept;
    const std::vector<std::string> &GetBufferNameList() const noexcept { return m_names; }
    void Destroy() noexcept;

private:
    std::map<std::string, std::unique_ptr<Buffer>, std::less<>> m_buffers;
    std::vector<std::string> m_names;
};

// ---------------------------------------------------------------- events
enum class ESystemEvent : uint32_t { SceneLoad, FrameFinished, Quit };
enum class EWorldEvent : uint32_t { CameraChange, RenderInstanceUpdate };

namespace detail {
class EventTable : public util::Singleton<EventTable> {
public:
    void Bind(uint64_t key, std::function<void(void *)> fn) noexcept;
    void Fire(uint64_t key, void *arg) noexcept;

private:
    std::mutex m_mutex;
    std::map<uint64_t, std::vector<std::function<void(void *)>>> m_handlers;
};
template <class E>
constexpr uint64_t event_family() noexcept {
    return std::is_same_v<E, ESystemEvent> ? 1ull : 2ull;
}
}  // namespace detail

template <auto kEvent, class Fn>
void EventBinder(Fn &&fn) noexcept {
    detail::EventTable::instance()->Bind((detail::event_family<decltype(kEvent)>() << 32) | (uint64_t)kEvent,
                                         std::function<void(void *)>(std::forward<Fn>(fn)));
}

template <auto kEvent>
void EventDispatcher(void *arg = nullptr) noexcept {
    detail::EventTable::instance()->Fire((detail::event_family<decltype(kEvent)>() << 32) | (uint64_t)kEvent, arg);
}

namespace world {
class World;
}

// ---------------------------------------------------------------- system
class System : public util::Singleton<System> {
public:
    int device = 0;  // HIP device the passes render on

    void Init(bool has_window = false) noexcept;  // headless; has_window is accepted and ignored
    void AddPass(Pass *pass) noexcept;
    // Loads a mitsuba XML scene (resource/scene.cpp subset), allocates the
    // "final result" buffer and fires ESystemEvent::SceneLoad with the World --
    // under the render mutex, as system.cpp:142-165 does, so no frame is in flight.
    bool SetScene(const std::filesystem::path &xml) noexcept;
    bool SetScene(std::unique_ptr<world::World> world) noexcept;  // programmatic scenes
    // `frames` frames on the caller's thread, each under the render mutex
    void Run(uint32_t frames) noexcept;
    // The reference's render thread (system.cpp:93-106): a thread that renders frames
    // (every enabled pass, then ESystemEvent::FrameFinished) under the render mutex
    // until Stop() or Destroy().  Other threads meanwhile fire events (a camera move,
    // RenderInstanceUpdate), which the passes pick up at the top of their next OnRun.
    void RunAsync() noexcept;
    void Stop() noexcept;
    uint64_t FramesRendered() const noexcept { return m_frames.load(); }
    // Holds off the render thread (e.g. to apply several scene edits as one change).
    std::unique_lock<std::mutex> RenderLock() noexcept;
    void Destroy() noexcept;
    world::World *GetWorld() noexcept { return m_world.get(); }

    // Multi-GPU (dist.h): call before SetScene in every rank's process; selects
    // device = local_rank and joins the RCCL communicator (also for world = 1, which
    // then gathers to itself).  Passes render this rank's tiles and PTPass gathers
    // the frame into rank 0's "final result".
    bool InitDistributed(const DistInfo &d) noexcept;
    FrameGather *Gather() noexcept { return m_gather.get(); }

private:
    void RenderFrame() noexcept;  // caller holds m_render_system_mutex

    std::vector<Pass *> m_passes;
    std::unique_ptr<world::World> m_world;
    std::unique_ptr<FrameGather> m_gather;
    std::mutex m_render_system_mutex;
    std::thread m_render_thread;
    std::atomic_bool m_quit{false};
    std::atomic<uint64_t> m_frames{0};
    std::atomic<int> m_lock_waiters{0};  // RenderLock callers: the render thread lets them in first
};

}  // namespace Pupil
