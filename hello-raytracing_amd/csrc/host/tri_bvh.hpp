// tri_bvh.hpp — opt-in binned-SAH BVH2 over the triangle program's triangles (rt_params.tri_bvh = 1).
//
// The reference walks its own median-split implicit heap (tree.rs:36-72, shader_tris.wgsl:268-301),
// ~50 node tests per ray on Suzanne. SURVEY §8(f) 2 allows a SAH tree only as an opt-in, non-parity mode:
// the closest hit is the same (t, triangle index) lexicographic minimum the reference's ordered walk
// keeps, but the reference's 600-step cap and its unpadded float slab tests can drop a triangle the SAH
// walk finds (grazing rays), so results may differ in rare pixels. Boxes are built over the triangle as
// Moller-Trumbore sees it (a, a + e1, a + e2 from the device's f32 a, e1, e2, summed in double) and
// rounded outward; the kernel pads them further per query.
#pragma once

#include <cstdint>
#include <vector>

#include "sphere_bvh.hpp"  // SphereBvhNode: the 64-byte two-child node layout, BVH_LEAF_BIT

namespace hrt {

struct TriBvh {
    std::vector<SphereBvhNode> nodes;  // nodes[0] = root when the root is internal
    std::vector<uint32_t> order;       // triangle indices in leaf order
    uint32_t root_word = 0x80000000u;  // child word of the root (empty leaf until built)
    float root_center[3] = {0, 0, 0};
    float root_radius = 0;             // >= half-diagonal of the root box
    uint32_t depth = 0;
};

// aee: 9 floats per triangle (a.xyz, e1.xyz, e2.xyz) exactly as uploaded to the device.
TriBvh build_tri_bvh(const std::vector<float>& aee);

}  // namespace hrt
