// sphere_bvh.cpp — binned-SAH BVH2 over sphere slots, with outward-rounded boxes.
#include "sphere_bvh.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <limits>

namespace hrt {
namespace {

struct Box {
    float lo[3] = {INFINITY, INFINITY, INFINITY};
    float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const Box& b) {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    double area() const {
        double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
        if (!(dx >= 0 && dy >= 0 && dz >= 0)) return 0.0;
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

// c - r rounded toward -inf and c + r toward +inf, with one extra ulp of slack each way.
float down(double v) {
    float f = (float)v;
    if ((double)f > v) f = std::nextafter(f, -INFINITY);
    return std::nextafter(f, -INFINITY);
}
float up(double v) {
    float f = (float)v;
    if ((double)f < v) f = std::nextafter(f, INFINITY);
    return std::nextafter(f, INFINITY);
}

struct Prim {
    Box box;
    float cen[3];
    int32_t slot;
};

struct Builder {
    std::vector<Prim> prims;
    SphereBvh* out;
    uint32_t max_depth = 0;
    // leaf policy (fixed: the library reads no environment variable; tuned values below)
#ifndef HRT_BVH_MAX_LEAF
#define HRT_BVH_MAX_LEAF BVH_MAX_LEAF
#endif
#ifndef HRT_BVH_TCOST
#define HRT_BVH_TCOST 0.5
#endif
    uint32_t max_leaf = HRT_BVH_MAX_LEAF;
#ifndef HRT_BVH_LEAF_DEPTH
#define HRT_BVH_LEAF_DEPTH 0
#endif
    uint32_t leaf_depth = HRT_BVH_LEAF_DEPTH;  // any subtree of <= max_leaf spheres becomes a leaf (measured best on C3)
    double traversal_cost = HRT_BVH_TCOST;
    // binned SAH over all three axes (all_axes false: the widest axis, 16 bins, as first built). C3,
    // Grays/s by bin count: 8 25.9, 16 26.8, 24 26.9, 32 27.7, 48 26.8, 64 28.0 (box / sphere tests per ray
    // 16.0 / 4.5 at 64, 16.8 / 5.4 first); an exact sweep SAH gave 26.9: tree shape matters more than
    // SAH accuracy here, and 64 bins measured best
    bool all_axes = true;
    int bins = 64;  // 2..64 with all_axes

    uint32_t leaf_word(size_t first, size_t count) {
        uint32_t f = (uint32_t)out->slot.size();
        for (size_t i = first; i < first + count; i++) {
            const Prim& p = prims[i];
            out->slot.push_back(p.slot);
            (void)p;
        }
        return BVH_LEAF_BIT | (f << 4) | (uint32_t)count;
    }

    // Returns the child word of the subtree over prims[first, first+count).
    uint32_t build(size_t first, size_t count, uint32_t depth, Box* bounds) {
        Box b;
        for (size_t i = first; i < first + count; i++) b.grow(prims[i].box);
        *bounds = b;
        max_depth = std::max(max_depth, depth);
        if (count <= 1 || (count <= max_leaf && depth >= leaf_depth)) return leaf_word(first, count);

        // centroid bounds
        float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t i = first; i < first + count; i++)
            for (int k = 0; k < 3; k++) {
                clo[k] = std::min(clo[k], prims[i].cen[k]);
                chi[k] = std::max(chi[k], prims[i].cen[k]);
            }
        int axis = 0;
        for (int k = 1; k < 3; k++)
            if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;

        size_t mid = first + count / 2;
        bool use_median = depth >= 20 || !(chi[axis] - clo[axis] > 0.0f);
        if (!use_median) {
            const int NB = bins;
            double best = std::numeric_limits<double>::infinity();
            int best_k = -1, best_axis = axis;
            // binned SAH over every axis with extent (all_axes) or the widest one
            for (int ax = 0; ax < 3; ax++) {
                if (!all_axes && ax != axis) continue;
                const float ext = chi[ax] - clo[ax];
                if (!(ext > 0.0f)) continue;
                Box bb[64];
                size_t bc[64] = {0};
                for (size_t i = first; i < first + count; i++) {
                    int k = (int)((prims[i].cen[ax] - clo[ax]) / ext * (all_axes ? NB : 16));
                    k = std::min((all_axes ? NB : 16) - 1, std::max(0, k));
                    bb[k].grow(prims[i].box);
                    bc[k]++;
                }
                const int nb = all_axes ? NB : 16;
                for (int k = 1; k < nb; k++) {
                    Box L, R;
                    size_t nl = 0, nr = 0;
                    for (int j = 0; j < k; j++) { if (bc[j]) { L.grow(bb[j]); nl += bc[j]; } }
                    for (int j = k; j < nb; j++) { if (bc[j]) { R.grow(bb[j]); nr += bc[j]; } }
                    if (!nl || !nr) continue;
                    double cost = L.area() * (double)nl + R.area() * (double)nr;
                    if (cost < best) { best = cost; best_k = k; best_axis = ax; }
                }
            }
            const double leaf_cost = b.area() * (double)count;
            if (count <= max_leaf && !(best + traversal_cost * b.area() < leaf_cost)) return leaf_word(first, count);
            if (best_k < 0) {
                use_median = true;
            } else {
                const int ax = best_axis, nb = all_axes ? NB : 16;
                const float ext = chi[ax] - clo[ax];
                auto bin_of = [&](const Prim& p) {
                    int i = (int)((p.cen[ax] - clo[ax]) / ext * nb);
                    return std::min(nb - 1, std::max(0, i));
                };
                auto it = std::stable_partition(prims.begin() + (long)first, prims.begin() + (long)(first + count),
                                                [&](const Prim& p) { return bin_of(p) < best_k; });
                mid = (size_t)(it - prims.begin());
                if (mid == first || mid == first + count) use_median = true;
            }
        }
        if (use_median) {
            std::stable_sort(prims.begin() + (long)first, prims.begin() + (long)(first + count),
                             [&](const Prim& a, const Prim& c) { return a.cen[axis] < c.cen[axis]; });
            mid = first + count / 2;
        }
        const uint32_t idx = (uint32_t)out->nodes.size();
        out->nodes.push_back(SphereBvhNode{});
        Box lb, rb;
        const uint32_t lw = build(first, mid - first, depth + 1, &lb);
        const uint32_t rw = build(mid, first + count - mid, depth + 1, &rb);
        SphereBvhNode& n = out->nodes[idx];
        for (int k = 0; k < 3; k++) {
            n.lmin[k] = lb.lo[k]; n.lmax[k] = lb.hi[k];
            n.rmin[k] = rb.lo[k]; n.rmax[k] = rb.hi[k];
        }
        n.left = lw;
        n.right = rw;
        return idx;
    }
};

}  // namespace

SphereBvh build_sphere_bvh(const std::vector<float>& cr) {
    SphereBvh out;
    const size_t n = cr.size() / 4;
    std::vector<float> radii;
    for (size_t i = 0; i < n; i++) {
        const float* s = &cr[4 * i];
        if (std::isfinite(s[0]) && std::isfinite(s[1]) && std::isfinite(s[2]) && std::isfinite(s[3]))
            radii.push_back(std::fabs(s[3]));
    }
    float median = 0.0f;
    if (!radii.empty()) {
        std::nth_element(radii.begin(), radii.begin() + (long)(radii.size() / 2), radii.end());
        median = radii[radii.size() / 2];
    }
    Builder b;
    b.out = &out;
    // (the tree-shape parameters are fixed: Builder's defaults, chosen by the round-2 sweeps in DESIGN.md §4)
    bool any = false;
    for (size_t i = 0; i < n; i++) {
        const float* s = &cr[4 * i];
        const bool finite = std::isfinite(s[0]) && std::isfinite(s[1]) && std::isfinite(s[2]) && std::isfinite(s[3]);
        const float r = std::fabs(s[3]);
        if (!finite || r > 32.0f * median + 1e-30f) {
            out.large.push_back((int32_t)i);
            continue;
        }
        Prim p;
        for (int k = 0; k < 3; k++) {
            p.box.lo[k] = down((double)s[k] - (double)r);
            p.box.hi[k] = up((double)s[k] + (double)r);
            p.cen[k] = s[k];
        }
        p.slot = (int32_t)i;
        b.prims.push_back(p);
        if (!any) { out.r_min = out.r_max = r; any = true; }
        out.r_min = std::min(out.r_min, r);
        out.r_max = std::max(out.r_max, r);
    }
    Box root;
    out.root_word = b.build(0, b.prims.size(), 0, &root);
    out.depth = b.max_depth;
    // leaf sphere data in BVH order
    out.sph.resize(out.slot.size() * 4);
    for (size_t k = 0; k < out.slot.size(); k++) {
        const float* s = &cr[4 * (size_t)out.slot[k]];
        out.sph[4 * k + 0] = s[0];
        out.sph[4 * k + 1] = s[1];
        out.sph[4 * k + 2] = s[2];
        out.sph[4 * k + 3] = s[3] * s[3];  // radius*radius, the same f32 product as the reference
    }
    if (!b.prims.empty()) {
        double diag2 = 0.0;
        for (int k = 0; k < 3; k++) {
            const double c = 0.5 * ((double)root.lo[k] + (double)root.hi[k]);
            out.root_center[k] = (float)c;
            const double h = std::max((double)root.hi[k] - (double)out.root_center[k],
                                      (double)out.root_center[k] - (double)root.lo[k]);
            diag2 += h * h;
        }
        out.root_radius = up(std::sqrt(diag2) * (1.0 + 1e-6));
    }
    return out;
}

}  // namespace hrt
