// world.h — host scene of the C++ layer (framework/world/world.h:25-70 names).
// Wraps the engine's pupil_world (XML loader, programmatic builder, emitter
// table, camera matrices) and exposes the fields PTPass reads in the
// reference: world->scene->sensor.film.{w,h}, world->scene->integrator.max_depth,
// world->camera (CameraHelper, world/camera.h).
#pragma once

#include <filesystem>
#include <memory>

#include "framework.h"

namespace Pupil::world {

struct SceneInfo {
    struct {
        struct {
            int w = 0, h = 0;
        } film;
    } sensor;
    struct {
        int max_depth = 1;
    } integrator;
};

class CameraHelper {
public:
    // Unsynchronised views (single-threaded use); a render thread takes Snapshot().
    const float *SampleToCamera() const noexcept { return m_s2c; }
    const float *CameraToWorld() const noexcept { return m_c2w; }
    // Replace the camera-to-world matrix (row-major 4x4) and fire
    // EWorldEvent::CameraChange, like CameraHelper's setters (world/camera.cpp).
    // Safe from any thread (the World's mutex guards the matrices).
    void SetCameraToWorld(const float c2w[16]) noexcept;
    void Snapshot(float s2c[16], float c2w[16]) const noexcept;
    void Load(const pupil_scene_desc &d) noexcept;

private:
    friend class World;
    std::mutex *m_lock = nullptr;  // the owning World's mutex
    float m_s2c[16] = {};
    float m_c2w[16] = {};
};

class World;
// payload of EWorldEvent::RenderInstanceUpdate
struct InstanceUpdate {
    World *world;
    uint32_t instance;  // index into Desc().instances
};

class World {
public:
    std::unique_ptr<SceneInfo> scene;
    std::unique_ptr<CameraHelper> camera;

    World() noexcept;
    ~World() noexcept;
    World(const World &) = delete;
    World &operator=(const World &) = delete;

    bool LoadScene(const std::filesystem::path &xml) noexcept;
    // Programmatic scenes: the caller filled `handle()` through pupil_world_*.
    bool Finalize() noexcept;
    // Moves instance `instance` (row-major 4x4), refreshes Desc() (instance
    // matrices, area emitters) and fires EWorldEvent::RenderInstanceUpdate.  Safe from
    // any thread: the edit happens under Mutex(), the event is fired after it.
    bool SetInstanceTransform(uint32_t instance, const float to_world[16]) noexcept;

    pupil_world *handle() noexcept { return m_world; }
    // Flattened scene for pupil_pt_create (valid until the world changes); a thread
    // reading it while another may edit the world holds Mutex().
    const pupil_scene_desc &Desc() const noexcept { return m_desc; }
    std::mutex &Mutex() noexcept { return m_mutex; }

private:
    pupil_world *m_world = nullptr;
    pupil_scene_desc m_desc{};
    std::mutex m_mutex;
};

}  // namespace Pupil::world
