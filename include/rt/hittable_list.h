// hittable_list.h -- drop-in for src/hittable_list.h: an ordered list of hittables whose
// box grows as objects are added.  The closest-hit loop over it (hittable_list.h:25-39)
// is replaced on the device by BVH traversal with the same result.
#pragma once
#include <vector>

#include "hittable.h"

class hittable_list : public hittable {
  public:
    std::vector<shared_ptr<hittable>> objects;

    hittable_list() {}
    hittable_list(shared_ptr<hittable> object) { add(object); }

    void clear() { objects.clear(); }
    void add(shared_ptr<hittable> object) {
        objects.push_back(object);
        bbox = aabb(bbox, object->bounding_box());
    }

    // hittable_list.h:25-39: every object against a shrinking upper bound; the last
    // (closest) hit's record wins
    bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
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
    aabb bbox;
};
