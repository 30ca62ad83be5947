// mesh_scene.cpp -- BASELINE.json config 4 through the C++ drop-in: the ground sphere of
// main.cpp:14-15 plus an OBJ mesh (lambertian, main.cpp's material2), main.cpp's camera,
// rendered on the GPU; PPM on stdout.
//   mesh_scene MODEL.obj [width=400] [spp=10] [p3|p6] [f32|f64]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>

#include "camera_hip.h"
#include "hittable_list.h"
#include "material.h"
#include "sphere.h"
#include "triangle_mesh.h"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s MODEL.obj [width] [spp] [p3|p6] [f32|f64]\n", argv[0]);
        return 2;
    }
    HIPImpl::Camera cam;
    cam.aspect_ratio = 16.0 / 9.0;
    cam.image_width = argc > 2 ? std::atoi(argv[2]) : 400;
    cam.samples_per_pixel = argc > 3 ? std::atoi(argv[3]) : 10;
    cam.max_depth = 50;
    cam.vfov = 20;
    cam.lookfrom = point3(13, 2, 3);
    cam.lookat = point3(0, 0, 0);
    cam.vup = vec3(0, 1, 0);
    cam.defocus_angle = 0.6;
    cam.focus_dist = 10.0;
    cam.binary_ppm = argc > 4 && std::strcmp(argv[4], "p6") == 0;
    cam.precision = argc > 5 && std::strcmp(argv[5], "f64") == 0 ? RT_PREC_F64 : RT_PREC_F32;

    hittable_list world;
    world.add(make_shared<sphere>(point3(0, -1000, 0), 1000, make_shared<lambertian>(color(0.5, 0.5, 0.5))));
    try {
        auto mesh = triangle_mesh::load_obj(argv[1], make_shared<lambertian>(color(0.4, 0.2, 0.1)));
        std::fprintf(stderr, "%zu triangles\n", mesh->num_triangles());
        world.add(mesh);
        cam.render(world);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
