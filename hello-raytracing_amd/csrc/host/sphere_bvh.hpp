// sphere_bvh.hpp — host builder of the culling BVH over sphere slots (build-side of SCAN_BVH).
//
// The reference scans every sphere slot for every ray (shader_sphere.wgsl:218-229). The MI355X path
// keeps that result bit for bit but visits only spheres the ray can reach: a binned-SAH BVH2 over the
// "small" spheres, plus a short always-scanned list of "large" ones (ground planes made of r = 1000
// spheres would make every box huge). Boxes are rounded outward so they contain each sphere exactly;
// the kernel pads them further per query (DESIGN.md §Sphere BVH exactness).
#pragma once

#include <cstdint>
#include <vector>

namespace hrt {

struct SphereBvhNode {     // 64 B, both children's boxes stored in the parent
    float lmin[3];
    uint32_t left;         // child word: internal node index, or LEAF_BIT | first << 4 | count
    float lmax[3];
    uint32_t pad0;
    float rmin[3];
    uint32_t right;
    float rmax[3];
    uint32_t pad1;
};
static_assert(sizeof(SphereBvhNode) == 64, "SphereBvhNode");

constexpr uint32_t BVH_LEAF_BIT = 0x80000000u;
constexpr uint32_t BVH_MAX_LEAF = 4;
constexpr uint32_t BVH_MAX_DEPTH = 30;  // informational; the kernel falls back to the exact scan on stack overflow

struct SphereBvh {
    std::vector<SphereBvhNode> nodes;  // nodes[0] = root (empty when the tree holds < 2 spheres)
    std::vector<float> sph;            // 4 floats per leaf sphere, BVH order: cx, cy, cz, r*r
    std::vector<int32_t> slot;         // original slot of each leaf sphere
    std::vector<int32_t> large;        // slots scanned linearly for every ray (ascending)
    uint32_t root_word = 0x80000000u;  // child word of the root (an empty leaf until built)
    float root_center[3] = {0, 0, 0};  // centre of the root box
    float root_radius = 0;             // >= half-diagonal of the root box (rounded up)
    float r_min = 0, r_max = 0;        // radius range of the BVH spheres
    uint32_t depth = 0;
};

// centers_radii: 4 floats per slot (cx, cy, cz, radius). Slots with non-finite data go to `large`.
SphereBvh build_sphere_bvh(const std::vector<float>& centers_radii);

}  // namespace hrt
