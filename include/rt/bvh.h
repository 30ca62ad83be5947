// bvh.h -- drop-in for src/bvh.h.  The reference's bvh_node has an empty constructor
// (bvh.h:12-14); here it records the object range and the device library builds the
// actual tree (SAH, rt_bvh.cpp) when the scene is uploaded, so wrapping a list in a
// bvh_node never changes a pixel.
#pragma once
#include <utility>
#include <vector>

#include "hittable_list.h"

class bvh_node : public hittable {
  public:
    bvh_node(const hittable_list& list) : bvh_node(list.objects, 0, list.objects.size()) {}
    bvh_node(const std::vector<shared_ptr<hittable>>& src, size_t start, size_t end)
        : objects(src.begin() + start, src.begin() + end) {
        for (const auto& o : objects) bbox = aabb(bbox, o->bounding_box());
    }

    // bvh.h:16-24 (box test, then the children with a shrinking bound): the node's box,
    // then its objects in order -- the same closest hit as the list it was built from
    bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
        if (!box_hit(r, ray_t)) return false;
        bool any = false;
        hit_record h;
        for (const auto& o : objects)
            if (o->hit(r, interval(ray_t.min, any ? rec.t : ray_t.max), h)) {
                any = true;
                rec = h;
            }
        return any;
    }
    aabb bounding_box() const override { return bbox; }
    void flatten(scene_builder& out) const override {
        for (const auto& o : objects) o->flatten(out);
    }

  private:
    // aabb.h:35-53: slab test per axis with 1/d, the interval narrowing as it goes
    bool box_hit(const ray& r, interval t) const {
        for (int a = 0; a < 3; ++a) {
            const double inv = 1 / r.direction()[a];
            double t0 = (bbox.axis(a).min - r.origin()[a]) * inv;
            double t1 = (bbox.axis(a).max - r.origin()[a]) * inv;
            if (inv < 0) std::swap(t0, t1);
            if (t0 > t.min) t.min = t0;
            if (t1 < t.max) t.max = t1;
            if (t.max <= t.min) return false;
        }
        return true;
    }

    std::vector<shared_ptr<hittable>> objects;
    aabb bbox;
};
