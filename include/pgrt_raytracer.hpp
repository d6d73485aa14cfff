// pgrt_raytracer.hpp -- C++ host facade over the C ABI, shaped like the reference renderer.
//
// The reference's compute classes (src/pg/pg1_embree: Raytracer raytracer.h:15-52,
// PinHoleCamera PinHoleCamera.h:14-41, LightSource LightSource.h, Material material.h:34-125,
// Texture texture.h:14-33, SphericalMap SphericalMap.h) keep their names and argument meaning;
// what changes is that a frame is rendered on the GPU in one call (Render) and get_pixel reads
// it.  Header-only; link with -lpgrt -lpgrt_image.  Errors throw pgrt::Exception (this header is the C++
// side: exceptions never cross the C ABI itself).
#pragma once

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "pgrt.h"
#include "pgrt_image.h"

namespace pgrt {

struct Exception : std::runtime_error {
    int code;
    Exception(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline void check(pgrt_ctx* ctx, int rc, const char* what) {
    if (rc != PGRT_OK)
        throw Exception(rc, std::string(what) + ": " + (ctx ? pgrt_last_error(ctx) : "") + " (code " +
                                std::to_string(rc) + ")");
}

struct Vector3 {  // vector3.h (only what the host side needs)
    float x = 0, y = 0, z = 0;
    Vector3() = default;
    Vector3(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
};

struct Color4f {  // structs.h:11-14
    float r, g, b, a;
};

constexpr int kHwQueues = 16;  // GPU_MAX_HW_QUEUES the library is benched with (prefer_hw_queues)

inline float deg2rad(const float x) { return x * float(3.14159265358979323846) / 180.0f; }  // mymath.h:27-30

// Texture(file_name) (texture.h:14-33, texture.cpp:5-54): the file decoded into FreeImage's raw
// layout (texture.cpp:43-47) -- BGR(A), top-down, 4-byte aligned pitch -- by libpgrt_image
// (pgrt_image.h): the format from the file signature, JPEG with FreeImage's JPEG_DEFAULT
// settings (IJG libjpeg, IFAST IDCT, no fancy upsampling), PNG through libpng.  Link with
// -lpgrt_image.
class Texture {
public:
    Texture() = default;
    explicit Texture(const char* file_name) { load(file_name); }
    int width() const { return width_; }
    int height() const { return height_; }
    pgrt_texture desc() const { return pgrt_texture{width_, height_, pitch_, bpp_, data_.data()}; }
    bool ok() const { return !data_.empty(); }

private:
    void load(const char* file_name) {
        int w = 0, h = 0, bpp = 0, pitch = 0;
        if (pgrt_image_decode(file_name, &w, &h, &bpp, &pitch, nullptr, 0) != 0)
            throw Exception(PGRT_ERR_IO, std::string("Texture: ") + pgrt_image_error());
        data_.assign((size_t)pitch * h, 0);
        if (pgrt_image_decode(file_name, &w, &h, &bpp, &pitch, data_.data(), data_.size()) != 0) {
            data_.clear();
            throw Exception(PGRT_ERR_IO, std::string("Texture: ") + pgrt_image_error());
        }
        width_ = w;
        height_ = h;
        pitch_ = pitch;
        bpp_ = bpp;
    }
    int width_ = 0, height_ = 0, pitch_ = 0, bpp_ = 0;
    std::vector<unsigned char> data_;
};

class LightSource {  // LightSource.h; GenerateRay's quirk lives in the device shadow stage
public:
    LightSource(Vector3 position, Vector3 ambient, Vector3 diffuse, Vector3 spectular)
        : position_(position), ambient_(ambient), diffuse_(diffuse), spectular_(spectular) {}
    Vector3 position_, ambient_, diffuse_, spectular_;
};

class PinHoleCamera {  // PinHoleCamera(width, height, fov_y, view_from, view_at)
public:
    PinHoleCamera() = default;
    PinHoleCamera(int width, int height, float fov_y, Vector3 view_from, Vector3 view_at)
        : width_(width), height_(height), fov_y_(fov_y), view_from_(view_from), view_at_(view_at) {}
    pgrt_camera desc() const {
        return pgrt_camera{width_, height_, fov_y_, {view_from_.x, view_from_.y, view_from_.z},
                           {view_at_.x, view_at_.y, view_at_.z}, {up_.x, up_.y, up_.z}};
    }
    int width_ = 640, height_ = 480;
    float fov_y_ = 0.785f;
    Vector3 view_from_, view_at_, up_{0.0f, 0.0f, 1.0f};  // PinHoleCamera.h:36
};

// Hardware queues for libpgrt's streams.  HIP reads GPU_MAX_HW_QUEUES once, when its runtime
// initialises (the first HIP call of the process), and defaults to 4 (the MI355X boxes this was
// measured on export GPU_MAX_HW_QUEUES=4).  libpgrt keeps every call in flight and both pipeline
// slots of a synchronous frame on streams of their own, so with 4 queues they share hardware
// queues: measured (profiles/r6/r6b_hw_queues.txt) the throughput line is the same but one
// synchronous C2 frame takes 0.66-0.70 ms instead of 0.54.  bench.py and the drop-in run with 16:
// prefer_hw_queues raises an unset or smaller value to n (a larger one is kept, <= 32) in the
// process environment -- in-process, never a re-exec -- and only takes effect if no HIP call ran
// in this process before.
inline void prefer_hw_queues(int n = kHwQueues) {
    const char* v = std::getenv("GPU_MAX_HW_QUEUES");
    if (!v || std::atoi(v) < n) setenv("GPU_MAX_HW_QUEUES", std::to_string(n).c_str(), 1);
}

// Raytracer(width, height, fov_y, view_from, view_at) (raytracer.h:18-20)
class Raytracer {
public:
    Raytracer(const int width, const int height, const float fov_y, const Vector3 view_from,
              const Vector3 view_at, const int hip_device = 0)
        : camera_(width, height, fov_y, view_from, view_at) {
        prefer_hw_queues();  // before pgrt_create: the process's first HIP call
        check(nullptr, pgrt_create(hip_device, &ctx_), "pgrt_create");
        init();
    }
    // one process, several GPUs (pgrt_create_devices): every frame is rendered tile-wise on all of
    // hip_devices and gathered on hip_devices[0]; the rest of the class is unchanged
    Raytracer(const int width, const int height, const float fov_y, const Vector3 view_from,
              const Vector3 view_at, const std::vector<int>& hip_devices)
        : camera_(width, height, fov_y, view_from, view_at) {
        prefer_hw_queues();
        check(nullptr, pgrt_create_devices(hip_devices.data(), (int)hip_devices.size(), &ctx_),
              "pgrt_create_devices");
        init();
    }
    ~Raytracer() { pgrt_destroy(ctx_); }
    Raytracer(const Raytracer&) = delete;
    Raytracer& operator=(const Raytracer&) = delete;

private:
    void init() {
        pgrt_camera c = camera_.desc();
        check(ctx_, pgrt_set_camera(ctx_, &c), "pgrt_set_camera");
        params_.spp_side = 3;          // raytracer.cpp:398
        params_.max_level = 7;         // raytracer.cpp:282
        params_.dof = 1;               // get_pixel always uses the thin-lens ray (:415)
        params_.focal_distance = 200;  // :399
        params_.aperture = 5;          // :400
        params_.gamma_level = gamma_level;
        params_.jitter = PGRT_JITTER_HASH;
        params_.seed = 1234;
    }

public:
    float gamma_level = 0.5f;  // UI slider default (raytracer.cpp:450,464-465)

    // LoadScene (raytracer.cpp:48-128): LoadOBJ + SphericalMap + one white light, then the
    // device copy and LBVH build replace the Embree geometry upload.
    void LoadScene(const std::string object_file_name, const std::string background_file_name) {
        pgrt_obj* obj = nullptr;
        int rc = pgrt_obj_load(object_file_name.c_str(), 0, &obj);
        if (rc != PGRT_OK) throw Exception(rc, std::string("LoadOBJ: ") + pgrt_obj_error());
        std::unique_ptr<pgrt_obj, void (*)(pgrt_obj*)> guard(obj, pgrt_obj_free);
        int ns = 0, nm = 0, nt = 0;
        pgrt_obj_counts(obj, &ns, &nm, &nt);
        surfaces_ = ns;
        materials_ = nm - 1;  // minus the trailing default Material()
        textures_.clear();
        for (int i = 0; i < nt; ++i) textures_.emplace_back(new Texture(pgrt_obj_texture_path(obj, i)));
        if (!background_file_name.empty()) textures_.emplace_back(new Texture(background_file_name.c_str()));
        lights_.clear();
        lights_.emplace_back(Vector3(-500, -100, 500), Vector3(1, 1, 1), Vector3(1, 1, 1), Vector3(1, 1, 1));
        std::vector<pgrt_texture> tex;
        for (auto& t : textures_) tex.push_back(t->desc());
        std::vector<pgrt_light> lights;
        for (auto& l : lights_)
            lights.push_back(pgrt_light{{l.position_.x, l.position_.y, l.position_.z},
                                        {l.diffuse_.x, l.diffuse_.y, l.diffuse_.z},
                                        {l.spectular_.x, l.spectular_.y, l.spectular_.z}});
        pgrt_scene_desc d;
        pgrt_obj_scene(obj, &d);
        d.num_textures = (int)tex.size();
        d.textures = tex.data();
        d.env_texture = background_file_name.empty() ? -1 : (int)tex.size() - 1;
        d.num_lights = (int)lights.size();
        d.lights = lights.data();
        check(ctx_, pgrt_set_scene(ctx_, &d), "pgrt_set_scene");
        frame_.clear();
    }

    // One frame of the Producer loop (simpleguidx11.cpp:105-118) on the GPU.
    pgrt_stats Render() {
        params_.gamma_level = gamma_level;
        frame_.resize((size_t)camera_.width_ * camera_.height_ * 4);
        pgrt_stats st{};
        check(ctx_, pgrt_render(ctx_, &params_, frame_.data(), &st), "pgrt_render");
        ++params_.frame;
        return st;
    }

    // The Producer loop as a frame sink: one more frame (next jitter / lens sample set) into
    // the device-side progressive mean, which becomes the frame get_pixel reads.
    int RenderProgressive(bool restart = false) {
        if (restart) check(ctx_, pgrt_accumulate_reset(ctx_), "pgrt_accumulate_reset");
        params_.gamma_level = gamma_level;
        frame_.resize((size_t)camera_.width_ * camera_.height_ * 4);
        int frames = 0;
        check(ctx_, pgrt_render_accumulate(ctx_, &params_, frame_.data(), &frames, nullptr),
              "pgrt_render_accumulate");
        ++params_.frame;
        return frames;
    }

    // Frames in flight (pgrt_render_device_async): the Producer loop without a host round trip
    // per frame.  Submit enqueues the next frame into a device framebuffer (pgrt_device_alloc,
    // W*H*4 floats) and returns at once; Wait completes every frame up to the ticket.
    void SetFramesInFlight(int n) { check(ctx_, pgrt_set_frames_in_flight(ctx_, n), "pgrt_set_frames_in_flight"); }
    unsigned long long Submit(void* rgba_device) {
        params_.gamma_level = gamma_level;
        unsigned long long t = 0;
        check(ctx_, pgrt_render_device_async(ctx_, &params_, rgba_device, &t), "pgrt_render_device_async");
        ++params_.frame;
        return t;
    }
    // Batched frames (pgrt_render_frames_device_async): nframes consecutive frames (frame indices
    // params.frame .. + nframes - 1) in one launch sequence, frame f at rgba_device + f*W*H*4.
    unsigned long long SubmitFrames(int nframes, void* rgba_device) {
        params_.gamma_level = gamma_level;
        unsigned long long t = 0;
        check(ctx_, pgrt_render_frames_device_async(ctx_, &params_, nframes, rgba_device, &t),
              "pgrt_render_frames_device_async");
        params_.frame += (unsigned)nframes;
        return t;
    }
    pgrt_stats Wait(unsigned long long ticket) {
        pgrt_stats st{};
        check(ctx_, pgrt_render_wait(ctx_, ticket, &st), "pgrt_render_wait");
        return st;
    }

    // get_pixel(x, y, t) (raytracer.cpp:396-437): reads the last rendered frame.
    Color4f get_pixel(const int x, const int y, const float /*t*/ = 0.0f) {
        if (frame_.empty()) Render();
        const float* p = &frame_[((size_t)y * camera_.width_ + x) * 4];
        return Color4f{p[0], p[1], p[2], p[3]};
    }

    const std::vector<float>& frame() const { return frame_; }
    pgrt_render_params& params() { return params_; }
    pgrt_ctx* context() { return ctx_; }
    int surfaces() const { return surfaces_; }
    int materials() const { return materials_; }

    // rtcIntersect1 for a batch (raytracer.cpp:130-148)
    std::vector<float> Intersect(const std::vector<float>& rays) {
        std::vector<float> hits(rays.size() / 8 * 4);
        check(ctx_, pgrt_intersect_closest(ctx_, rays.data(), (int)(rays.size() / 8), hits.data()),
              "pgrt_intersect_closest");
        return hits;
    }

    // rtcOccluded1 for a batch (any hit in (tnear, tfar])
    std::vector<int> Occluded(const std::vector<float>& rays) {
        std::vector<int> occ(rays.size() / 8);
        check(ctx_, pgrt_occluded(ctx_, rays.data(), (int)(rays.size() / 8), occ.data()), "pgrt_occluded");
        return occ;
    }

private:
    pgrt_ctx* ctx_ = nullptr;
    PinHoleCamera camera_;
    pgrt_render_params params_{};
    std::vector<std::unique_ptr<Texture>> textures_;
    std::vector<LightSource> lights_;
    std::vector<float> frame_;
    int surfaces_ = 0, materials_ = 0;
};

// Write an RGBA float frame as a PFM (RGB, bottom-up as the format requires).
inline bool write_pfm(const char* path, const float* rgba, int w, int h) {
    FILE* f = std::fopen(path, "wb");
    if (!f) return false;
    std::fprintf(f, "PF\n%d %d\n-1.0\n", w, h);
    std::vector<float> row((size_t)w * 3);
    for (int y = h - 1; y >= 0; --y) {
        for (int x = 0; x < w; ++x)
            for (int c = 0; c < 3; ++c) row[(size_t)x * 3 + c] = rgba[((size_t)y * w + x) * 4 + c];
        std::fwrite(row.data(), sizeof(float), row.size(), f);
    }
    std::fclose(f);
    return true;
}

}  // namespace pgrt
