// camera.h -- drop-in for src/camera.h.
//
// Same public fields and defaults (camera.h:15-26), same initialize() arithmetic (done by
// rt_camera_initialize in the library), same host get_ray() on the reference's random
// stream, same PPM P3 output of render().  What changes is where the pixel x sample loop
// and the ray_color recursion run: render() hands the whole frame to the device through
// the virtual render_pixels() (HIPImpl::Camera in camera_hip.h).
#pragma once
#include <cstdio>
#include <iostream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "color.h"
#include "hittable.h"
#include "material.h"
#include "rtweekend.h"

class camera {
  protected:
    virtual ~camera() = default;

  public:
    double aspect_ratio = 1.0;
    int image_width = 100;
    int samples_per_pixel = 10;
    int max_depth = 10;

    double vfov = 90;
    point3 lookfrom = point3(0, 0, -1);
    point3 lookat = point3(0, 0, 0);
    vec3 vup = vec3(0, 1, 0);

    double defocus_angle = 0;
    double focus_dist = 10;

    auto image_size() const { return std::make_pair(image_width, image_height); }

    // camera.h:32-50: P3 header, one "r g b" line per pixel (write_color), progress on clog.
    void render(const hittable& world) {
        initialize();
        std::vector<int32_t> rgb;
        std::clog << "\rRendering " << image_width << 'x' << image_height << " @ " << samples_per_pixel
                  << " spp on the GPU " << std::flush;
        render_pixels(world, rgb);
        write_image(std::cout, rgb);
        std::clog << "\rDone.                 \n";
    }

    // camera.h:52-85
    void initialize() {
        rt_camera_desc d{};
        d.aspect_ratio = aspect_ratio;
        d.image_width = image_width;
        d.samples_per_pixel = samples_per_pixel;
        d.max_depth = max_depth;
        d.vfov = vfov;
        for (int k = 0; k < 3; ++k) {
            d.lookfrom[k] = lookfrom[k];
            d.lookat[k] = lookat[k];
            d.vup[k] = vup[k];
        }
        d.defocus_angle = defocus_angle;
        d.focus_dist = focus_dist;
        if (rt_camera_initialize(&d, &native_) != RT_OK) throw std::invalid_argument("camera: bad image size/aspect");
        image_height = native_.image_height;
        auto v = [](const double* p) { return vec3(p[0], p[1], p[2]); };
        center = v(native_.center);
        pixel00_loc = v(native_.pixel00_loc);
        pixel_delta_u = v(native_.pixel_delta_u);
        pixel_delta_v = v(native_.pixel_delta_v);
        defocus_disk_u = v(native_.defocus_disk_u);
        defocus_disk_v = v(native_.defocus_disk_v);
    }

    // camera.h:87-113, on the host's reference stream (rtweekend.h random_double).
    ray get_ray(int i, int j) const {
        const point3 pixel_center = pixel00_loc + (i * pixel_delta_u) + (j * pixel_delta_v);
        const point3 pixel_sample = pixel_center + pixel_sample_square();
        const point3 origin = (defocus_angle <= 0) ? center : defocus_disk_sample();
        const double time = random_double();
        return ray(origin, pixel_sample - origin, time);
    }

    virtual color ray_color(const ray& r, int depth, const hittable& world) const = 0;

  protected:
    // The device render of the whole frame: W*H*3 ints as write_color prints them.
    virtual void render_pixels(const hittable& world, std::vector<int32_t>& rgb) = 0;

    // camera.h:35 + color.h:32-34: P3 text, one "r g b" line per pixel.
    virtual void write_image(std::ostream& os, const std::vector<int32_t>& rgb) const {
        std::string text = "P3\n" + std::to_string(image_width) + ' ' + std::to_string(image_height) + "\n255\n";
        text.reserve(text.size() + rgb.size() * 4 + 16);
        char buf[48];
        for (size_t p = 0; p + 2 < rgb.size(); p += 3) {
            int n = std::snprintf(buf, sizeof buf, "%d %d %d\n", rgb[p], rgb[p + 1], rgb[p + 2]);
            text.append(buf, (size_t)n);
        }
        os << text;
    }

    vec3 pixel_sample_square() const {
        const double px = -0.5 + random_double();
        const double py = -0.5 + random_double();
        return (px * pixel_delta_u) + (py * pixel_delta_v);
    }
    point3 defocus_disk_sample() const {
        const vec3 p = random_in_unit_disk();
        return center + (p[0] * defocus_disk_u) + (p[1] * defocus_disk_v);
    }

    rt_camera native_{};
    int image_height = 0;
    point3 center, pixel00_loc;
    vec3 pixel_delta_u, pixel_delta_v, defocus_disk_u, defocus_disk_v;
};
