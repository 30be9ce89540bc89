// world.cpp — World / CameraHelper over the engine's pupil_world.
#include "pupil/world.h"

#include <cstring>

namespace Pupil::world {

void CameraHelper::Load(const pupil_scene_desc &d) noexcept {
    std::memcpy(m_s2c, d.sample_to_camera, sizeof(m_s2c));
    std::memcpy(m_c2w, d.camera_to_world, sizeof(m_c2w));
}

void CameraHelper::SetCameraToWorld(const float c2w[16]) noexcept {
    {
        std::unique_lock<std::mutex> lock;
        if (m_lock) lock = std::unique_lock<std::mutex>(*m_lock);
        std::memcpy(m_c2w, c2w, sizeof(m_c2w));
    }
    EventDispatcher<EWorldEvent::CameraChange>(this);
}

void CameraHelper::Snapshot(float s2c[16], float c2w[16]) const noexcept {
    std::unique_lock<std::mutex> lock;
    if (m_lock) lock = std::unique_lock<std::mutex>(*m_lock);
    std::memcpy(s2c, m_s2c, sizeof(m_s2c));
    std::memcpy(c2w, m_c2w, sizeof(m_c2w));
}

World::World() noexcept {
    if (pupil_world_create(&m_world) != PUPIL_OK) {
        Log("world creation failed: %s", pupil_last_error());
        m_world = nullptr;
    }
    scene = std::make_unique<SceneInfo>();
    camera = std::make_unique<CameraHelper>();
    camera->m_lock = &m_mutex;
}

World::~World() noexcept {
    if (m_world) pupil_world_destroy(m_world);
}

bool World::LoadScene(const std::filesystem::path &xml) noexcept {
    if (!m_world) return false;
    if (pupil_world_load_xml(m_world, xml.string().c_str()) != PUPIL_OK) {
        Log("scene '%s': %s", xml.string().c_str(), pupil_last_error());
        return false;
    }
    return Finalize();
}

bool World::Finalize() noexcept {
    if (!m_world || pupil_world_get_desc(m_world, &m_desc) != PUPIL_OK) {
        Log("scene description failed: %s", pupil_last_error());
        return false;
    }
    scene->sensor.film.w = (int)m_desc.width;
    scene->sensor.film.h = (int)m_desc.height;
    scene->integrator.max_depth = (int)m_desc.max_depth;
    camera->Load(m_desc);
    return true;
}

bool World::SetInstanceTransform(uint32_t instance, const float to_world[16]) noexcept {
    {
        std::scoped_lock lock(m_mutex);
        if (!m_world || pupil_world_set_instance_transform(m_world, instance, to_world) != PUPIL_OK) {
            Log("instance update failed: %s", pupil_last_error());
            return false;
        }
        // the desc only: the camera keeps any SetCameraToWorld made since the load
        if (pupil_world_get_desc(m_world, &m_desc) != PUPIL_OK) {
            Log("scene description failed: %s", pupil_last_error());
            return false;
        }
    }
    InstanceUpdate u{this, instance};
    EventDispatcher<EWorldEvent::RenderInstanceUpdate>(&u);
    return true;
}

}  // namespace Pupil::world
