// camera_hip.h -- HIPImpl::Camera, the MI355X sibling of the reference's CPUImpl::Camera
// (src/camera_cpu.h:3-30).  Link with librt_hip.so.
//
//   render(world)            -> flatten the scene, rt_upload_scene_ex, rt_render_frame on
//                               device `device` (fp32 by default, RT_PREC_F64 for the
//                               reference-exact arithmetic), PPM P3 on stdout.
//                               With `devices` set ({0,1,...,7}) the frame is split over
//                               those GPUs in one process (rt_render_frame_multi: one
//                               context per GPU, shards gathered to devices[0] over xGMI).
//                               The environment sets it for an unchanged main.cpp:
//                               RT_DEVICES=all or RT_DEVICES=0,1,2,3.
//   ray_color(r, depth, world)-> one ray on the device in fp64, consuming the host's
//                               reference stream exactly as camera_cpu.h:8-26 would
//                               (a tape of uniforms cut from a copy of the stream; the
//                               stream then advances by the number used).
// Render sampling: each (pixel, sample) path draws from its own counter stream keyed by
// `seed` (rt_hip.h), which is what makes the frame parallel; the reference's single
// sequential stream cannot be split across GPU lanes.
#pragma once
#include <cstdlib>
#include <string>
#include <vector>

#include "camera.h"

namespace HIPImpl {

class Camera : public camera {
  public:
    int device = 0;
    uint64_t seed = 0x5EED;
    int precision = RT_PREC_F32;
    bool binary_ppm = false;   // false: P3 text as the reference prints; true: P6 (same 8-bit values)
    std::vector<int> devices;  // empty: `device` only; else one context per listed GPU

    Camera() { devices = devices_from_env(); }
    Camera(const Camera&) = delete;
    Camera& operator=(const Camera&) = delete;
    ~Camera() override {
        rt_destroy(ctx_);
        rt_destroy(tape_ctx_);
        for (rt_ctx* c : multi_) rt_destroy(c);
    }

    color ray_color(const ray& r, int depth, const hittable& world) const override {
        if (!tape_ctx_) {
            tape_ctx_ = rt_create(device, seed, RT_PREC_F64);
            if (!tape_ctx_) throw std::runtime_error("rt_create failed (no HIP device?)");
        }
        if (tape_world_ != &world) {
            upload(tape_ctx_, world);
            tape_world_ = &world;
        }
        const double r7[7] = {r.origin()[0], r.origin()[1], r.origin()[2], r.direction()[0],
                              r.direction()[1], r.direction()[2], r.time()};
        std::vector<double> tape(256);
        double out[3];
        int used = 0;
        for (;;) {
            std::mt19937 probe = rt_host::generator();        // copy: do not advance yet
            std::uniform_real_distribution<double> unit(0.0, 1.0);
            for (auto& u : tape) u = unit(probe);
            check(tape_ctx_, rt_trace_tape(tape_ctx_, r7, depth, tape.data(), (int)tape.size(), out, &used));
            if (used <= (int)tape.size()) break;
            tape.resize((size_t)used * 2);
        }
        for (int k = 0; k < used; ++k) random_double();       // the stream the reference would leave
        return color(out[0], out[1], out[2]);
    }

  protected:
    void render_pixels(const hittable& world, std::vector<int32_t>& rgb) override {
        rgb.resize((size_t)native_.image_width * native_.image_height * 3);
        if (devices.size() > 1) {
            if (multi_.empty())
                for (int d : devices) {
                    rt_ctx* c = rt_create(d, seed, precision);
                    if (!c) throw std::runtime_error("rt_create failed on device " + std::to_string(d));
                    multi_.push_back(c);
                }
            for (rt_ctx* c : multi_) upload(c, world);
            check(multi_[0], rt_render_frame_multi(multi_.data(), (int)multi_.size(), &native_, samples_per_pixel,
                                                   max_depth, nullptr, rgb.data()));
            return;
        }
        if (!ctx_) {
            ctx_ = rt_create(device, seed, precision);
            if (!ctx_) throw std::runtime_error("rt_create failed (no HIP device?)");
        }
        upload(ctx_, world);
        check(ctx_, rt_render_frame(ctx_, &native_, samples_per_pixel, max_depth, nullptr, rgb.data(), nullptr));
    }

    void write_image(std::ostream& os, const std::vector<int32_t>& rgb) const override {
        if (!binary_ppm) return camera::write_image(os, rgb);
        std::string out = "P6\n" + std::to_string(image_width) + ' ' + std::to_string(image_height) + "\n255\n";
        const size_t head = out.size();
        out.resize(head + rgb.size());
        for (size_t k = 0; k < rgb.size(); ++k) {
            if (rgb[k] < 0 || rgb[k] > 255) throw std::runtime_error("P6: pixel value outside 0..255 (NaN sum)");
            out[head + k] = (char)(unsigned char)rgb[k];
        }
        os << out;
    }

  private:
    static std::vector<int> devices_from_env() {
        std::vector<int> d;
        const char* e = std::getenv("RT_DEVICES");
        if (!e || !*e) return d;
        if (std::string(e) == "all") {
            for (int k = 0, n = rt_device_count(); k < n; ++k) d.push_back(k);
            return d;
        }
        for (const char* p = e; *p;) {
            char* end = nullptr;
            const long v = std::strtol(p, &end, 10);
            if (end == p) throw std::runtime_error(std::string("RT_DEVICES: cannot parse '") + e + "'");
            d.push_back((int)v);
            p = *end == ',' ? end + 1 : end;
        }
        return d;
    }
    static void check(rt_ctx* c, int rc) {
        if (rc != RT_OK) throw std::runtime_error(std::string(rt_error_string(rc)) + ": " + rt_last_error(c));
    }
    static void upload(rt_ctx* c, const hittable& world) {
        scene_builder sb;
        world.flatten(sb);
        check(c, rt_upload_scene_ex(c, sb.spheres.data(), (int)sb.spheres.size(), sb.materials.data(),
                                    (int)sb.materials.size(), sb.triangles.data(), (int)sb.triangles.size()));
    }

    rt_ctx* ctx_ = nullptr;
    std::vector<rt_ctx*> multi_;
    mutable rt_ctx* tape_ctx_ = nullptr;
    mutable const hittable* tape_world_ = nullptr;
};

}  // namespace HIPImpl
