// pt_pass.cpp — PTPass over the HIP engine (example/path_tracer/pt_pass.cpp).
#include "pupil/pt_pass.h"

#include <algorithm>
#include <cstring>

namespace Pupil::pt {

PTPass::PTPass(std::string_view name) noexcept : Pass(name) {
    if (hipStreamCreateWithFlags(&m_stream, hipStreamNonBlocking) != hipSuccess) {
        Log("%s: stream creation failed", this->name.c_str());
        m_stream = nullptr;
    }
    BindingEventCallback();
}

PTPass::~PTPass() noexcept {
    if (m_engine) pupil_pt_destroy(m_engine);
    if (m_stream) (void)hipStreamDestroy(m_stream);
}

// pt_pass.cpp:39-57: refresh on dirty (camera, instances moved since the last frame,
// depth, accumulation reset), one 1-spp frame, synchronise, advance seed and sample
// count.  Runs on the render thread; events may arrive from any other thread.
void PTPass::OnRun() noexcept {
    if (!m_engine) return;
    if (m_dirty) {
        m_dirty = false;  // an event after this point marks the next frame dirty again
        std::vector<uint32_t> moved;
        {
            std::scoped_lock lock(m_pending_mutex);
            moved.swap(m_pending);
        }
        float s2c[16], c2w[16];
        m_world->camera->Snapshot(s2c, c2w);
        pupil_pt_set_camera(m_engine, s2c, c2w);
        if (!moved.empty()) {  // m_world->GetIASHandle(2, true) + the emitter group (pt_pass.cpp:46-47)
            std::scoped_lock lock(m_world->Mutex());
            const pupil_scene_desc &d = m_world->Desc();
            std::vector<float> tw(12 * moved.size()), to(12 * moved.size());
            bool emissive = false;
            for (size_t k = 0; k < moved.size(); k++) {
                const pupil_instance &ins = d.instances[moved[k]];
                std::memcpy(&tw[12 * k], ins.to_world, sizeof(ins.to_world));
                std::memcpy(&to[12 * k], ins.to_object, sizeof(ins.to_object));
                emissive = emissive || ins.emitter_offset >= 0;
            }
            if (pupil_pt_update_instances(m_engine, (uint32_t)moved.size(), moved.data(), tw.data(), to.data()) !=
                PUPIL_OK)
                Log("%s: instance update failed: %s", name.c_str(), pupil_last_error());
            else if (emissive && pupil_pt_update_emitters(m_engine, &d) != PUPIL_OK)
                Log("%s: emitter update failed: %s", name.c_str(), pupil_last_error());
        }
        m_frame_max_depth = (uint32_t)m_max_depth;
        m_sample_cnt = 0;
        m_random_seed = 0;
    }
    pupil_pt_launch launch{};
    launch.random_seed = m_random_seed;
    launch.sample_cnt = m_sample_cnt;
    launch.spp = 1;
    launch.max_depth = m_frame_max_depth;
    launch.accumulate = m_accumulated_flag ? 1u : 0u;
    FrameGather *gather = util::Singleton<System>::instance()->Gather();
    if (gather) {  // this rank's tiles only (dist.h)
        launch.tile_size = gather->Info().tile;
        launch.tile_rank = (uint32_t)gather->Info().rank;
        launch.tile_world = (uint32_t)gather->Info().world;
    }
    if (pupil_pt_render(m_engine, &m_frame, &launch, m_stream) != PUPIL_OK) {
        Log("%s: render failed: %s", name.c_str(), pupil_last_error());
        return;
    }
    if (gather && !gather->Gather(m_frame.frame, m_full_result, m_stream)) {
        Log("%s: tile gather failed", name.c_str());
        return;
    }
    (void)hipStreamSynchronize(m_stream);
    m_sample_cnt += m_accumulated_flag ? 1u : 0u;
    ++m_random_seed;
}

void PTPass::SetScene(world::World *world) noexcept {
    if (!world) return;
    m_world = world;
    {
        std::scoped_lock lock(m_pending_mutex);  // moves of the previous world
        m_pending.clear();
    }
    if (m_engine) {
        pupil_pt_destroy(m_engine);
        m_engine = nullptr;
    }
    int w = world->scene->sensor.film.w, h = world->scene->sensor.film.h;
    m_max_depth = world->scene->integrator.max_depth;
    m_accumulated_flag = true;
    auto *bm = BufferManager::instance();
    Buffer *final_result = bm->GetBuffer(BufferManager::DEFAULT_FINAL_RESULT_BUFFER_NAME);
    m_full_result = final_result ? final_result->cuda_ptr : nullptr;
    FrameGather *gather = util::Singleton<System>::instance()->Gather();
    if (gather) {  // multi-GPU: the pass's buffers hold this rank's tiles, compact (dist.h)
        w = (int)std::max(1u, gather->LocalPixels());
        h = 1;
        BufferDesc tiles;
        tiles.name = "final result (local tiles)";
        tiles.width = (uint32_t)w;
        tiles.height = 1;
        tiles.stride_in_byte = sizeof(float) * 4;
        final_result = bm->AllocBuffer(tiles);
    }
    BufferDesc desc;
    desc.width = (uint32_t)w;
    desc.height = (uint32_t)h;
    desc.name = "pt accum buffer";
    desc.stride_in_byte = sizeof(float) * 4;
    Buffer *accum = bm->AllocBuffer(desc);
    desc.name = "albedo";
    desc.flag = EBufferFlag::AllowDisplay;
    desc.stride_in_byte = sizeof(float) * 3;
    Buffer *albedo = bm->AllocBuffer(desc);
    desc.name = "normal";
    Buffer *normal = bm->AllocBuffer(desc);
    desc.name = "test";
    desc.stride_in_byte = sizeof(float);
    Buffer *test = bm->AllocBuffer(desc);
    if (!final_result || !accum || !albedo || !normal || !test) {
        Log("%s: output buffers unavailable", name.c_str());
        return;
    }
    m_frame = pupil_pt_frame{accum->cuda_ptr, final_result->cuda_ptr, albedo->cuda_ptr, normal->cuda_ptr,
                             test->cuda_ptr, gather ? 1u : 0u, 0u};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (pupil_pt_create(&world->Desc(), dev, &m_engine) != PUPIL_OK) {
        Log("%s: engine creation failed: %s", name.c_str(), pupil_last_error());
        m_engine = nullptr;
        return;
    }
    m_dirty = true;
}

void PTPass::SetMaxDepth(int depth) noexcept {
    depth = std::clamp(depth, 1, 128);  // Inspector clamp, pt_pass.cpp:229
    if (depth != m_max_depth) {
        m_max_depth = depth;
        m_dirty = true;
    }
}

void PTPass::SetAccumulate(bool on) noexcept {
    if (on != m_accumulated_flag) {
        m_accumulated_flag = on;
        m_dirty = true;
    }
}

bool PTPass::Stats(pupil_pt_counters &out) noexcept { return m_engine && pupil_pt_stats(m_engine, &out) == PUPIL_OK; }

void PTPass::BindingEventCallback() noexcept {
    EventBinder<EWorldEvent::CameraChange>([this](void *) { m_dirty = true; });
    EventBinder<EWorldEvent::RenderInstanceUpdate>([this](void *p) {
        // only recorded: the next OnRun refits once for every instance moved since the last
        // (ias_manager.cpp:116-151, world.cpp:45-54) and restarts accumulation
        const auto *u = static_cast<const world::InstanceUpdate *>(p);
        if (u && u->world == m_world) {
            std::scoped_lock lock(m_pending_mutex);
            if (std::find(m_pending.begin(), m_pending.end(), u->instance) == m_pending.end())
                m_pending.push_back(u->instance);
        }
        m_dirty = true;
    });
    EventBinder<ESystemEvent::SceneLoad>([this](void *p) { SetScene(static_cast<world::World *>(p)); });
}

void PTPass::Inspector() noexcept {
    Pass::Inspector();
    Log("  sample count: %u, max trace depth: %d, accumulate radiance: %s", m_sample_cnt + 1, m_max_depth,
        m_accumulated_flag ? "on" : "off");
}

}  // namespace Pupil::pt
