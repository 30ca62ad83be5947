// obj_dump.cpp -- TEST INFRASTRUCTURE.  Loads an OBJ with the reference's vendored
// tinyobjloader (dependencies/tinyobjloader, LoadObj at tiny_obj_loader.h:605, compiled
// from its own tiny_obj_loader.cc by oracle/Makefile) and prints what it parsed, so
// tests/test_mesh.py can cross-check rt_obj_load:
//   V <num_vertices>  then one "x y z" per vertex (%.9g of tinyobj's float real_t)
//   T <num_triangles> then one "a b c" per triangle (0-based vertex indices)
#include <cstdio>
#include <string>
#include <vector>

#include "tiny_obj_loader.h"

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    tinyobj::attrib_t attrib;
    std::vector<tinyobj::shape_t> shapes;
    std::vector<tinyobj::material_t> materials;
    std::string warn, err;
    if (!tinyobj::LoadObj(&attrib, &shapes, &materials, &warn, &err, argv[1], nullptr, true)) {
        std::fprintf(stderr, "LoadObj failed: %s\n", err.c_str());
        return 1;
    }
    std::printf("V %zu\n", attrib.vertices.size() / 3);
    for (size_t k = 0; k < attrib.vertices.size(); k += 3)
        std::printf("%.9g %.9g %.9g\n", attrib.vertices[k], attrib.vertices[k + 1], attrib.vertices[k + 2]);
    size_t nt = 0;
    for (auto& s : shapes) nt += s.mesh.indices.size() / 3;
    std::printf("T %zu\n", nt);
    for (auto& s : shapes)
        for (size_t k = 0; k + 2 < s.mesh.indices.size(); k += 3)
            std::printf("%d %d %d\n", s.mesh.indices[k].vertex_index, s.mesh.indices[k + 1].vertex_index,
                        s.mesh.indices[k + 2].vertex_index);
    return 0;
}
