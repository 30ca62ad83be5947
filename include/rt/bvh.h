// bvh.h -- drop-in for src/bvh.h.  The reference's bvh_node has an empty constructor
// (bvh.h:12-14); here it records the object range and the device library builds the
// actual tree (SAH, rt_bvh.cpp) when the scene is uploaded, so wrapping a list in a
// bvh_node never changes a pixel.
#pragma once
#include <vector>

#include "hittable_list.h"

class bvh_node : public hittable {
  public:
    bvh_node(const hittable_list& list) : bvh_node(list.objects, 0, list.objects.size()) {}
    bvh_node(const std::vector<shared_ptr<hittable>>& src, size_t start, size_t end)
        : objects(src.begin() + start, src.begin() + end) {
        for (const auto& o : objects) bbox = aabb(bbox, o->bounding_box());
    }

    aabb bounding_box() const override { return bbox; }
    void flatten(scene_builder& out) const override {
        for (const auto& o : objects) o->flatten(out);
    }

  private:
    std::vector<shared_ptr<hittable>> objects;
    aabb bbox;
};
