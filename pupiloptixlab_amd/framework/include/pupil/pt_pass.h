// pt_pass.h — the path-tracing pass (example/path_tracer/pt_pass.h:20-43),
// rendering with the HIP wavefront engine through the C ABI instead of an
// OptiX pipeline + SBT.  Same constructor, OnRun, Inspector, SetScene and
// event bindings; same buffers ("pt accum buffer", "albedo", "normal",
// "test", writing "final result").
#pragma once

#include <atomic>
#include <mutex>
#include <string_view>
#include <vector>

#include "framework.h"
#include "world.h"

namespace Pupil::pt {

class PTPass : public Pass {
public:
    PTPass(std::string_view name = "Path Tracing") noexcept;
    ~PTPass() noexcept override;

    void OnRun() noexcept override;
    void Inspector() noexcept override;
    void SetScene(world::World *world) noexcept;

    // headless accessors (the reference shows these in its ImGui inspector)
    uint32_t SampleCount() const noexcept { return m_sample_cnt; }
    int MaxDepth() const noexcept { return m_max_depth; }
    void SetMaxDepth(int depth) noexcept;
    void SetAccumulate(bool on) noexcept;
    bool Stats(pupil_pt_counters &out) noexcept;

private:
    void BindingEventCallback() noexcept;

    pupil_pt *m_engine = nullptr;
    hipStream_t m_stream = nullptr;
    world::World *m_world = nullptr;
    pupil_pt_frame m_frame{};
    void *m_full_result = nullptr;  // System's full-frame "final result" (the gather target)
    uint32_t m_random_seed = 0;
    uint32_t m_sample_cnt = 0;
    uint32_t m_frame_max_depth = 1;  // value in effect for the running accumulation
    int m_max_depth = 1;
    bool m_accumulated_flag = true;
    std::atomic_bool m_dirty = true;
    // instances moved since the last OnRun (RenderInstanceUpdate only records them, as the
    // reference's handler only sets m_dirty, pt_pass.cpp:216-218; OnRun refits once)
    std::mutex m_pending_mutex;
    std::vector<uint32_t> m_pending;
};

}  // namespace Pupil::pt
