// scene.hpp — host-side scene description of the MI355X path tracer.
//
// Mirrors the reference's Rust host layer (hucancode/hello-raytracing, src/scene/*, src/geometry/*):
// the same #[repr(C)] POD layouts (so the bytes handed to the renderer are the reference's bytes) and
// the same f32 arithmetic as glam 0.24 (scalar Vec3, no contraction) for the few host computations
// that feed the hot path: Camera::new, Tree::add_mesh/build, Mesh::load_obj.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace hrt {

struct Vec3 {
    float x, y, z;
};
struct Vec4 {
    float x, y, z, w;
};

// glam 0.24 Vec3 (scalar implementation): dot = (x*x') + (y*y') + (z*z'); normalize = v * (1 / |v|).
inline Vec3 operator+(Vec3 a, Vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline Vec3 operator-(Vec3 a, Vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline Vec3 operator*(Vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
float glam_dot(Vec3 a, Vec3 b);
Vec3 glam_cross(Vec3 a, Vec3 b);
Vec3 glam_normalize(Vec3 v);

// src/scene/camera.rs:6-12 — 80 bytes.
struct Camera {
    Vec4 eye, direction, up, right, params;
    // Camera::new, camera.rs:15-28.
    static Camera make(Vec3 from, Vec3 to, float focal_length, float focal_blur_amount, float fov);
};
static_assert(sizeof(Camera) == 80, "Camera layout");

constexpr uint32_t LAMBERTIAN = 1, METAL = 2, DIELECTRIC = 3;  // material.rs:4-6

// src/scene/material.rs:9-13 — 32 bytes.
struct Material {
    Vec4 albedo;
    Vec3 params;
    uint32_t kind;
    static Material lambertian(Vec3 albedo);            // material.rs:17-23
    static Material metal(Vec3 albedo, float fuzzy);    // material.rs:24-30
    static Material dielectric(float ir);               // material.rs:31-37
};
static_assert(sizeof(Material) == 32, "Material layout");

// src/scene/sphere.rs:6-10 — 48 bytes.
struct Sphere {
    Vec3 center;
    float radius;
    Material material;
};
static_assert(sizeof(Sphere) == 48, "Sphere layout");

// src/scene/bvh/node.rs:6-9 — 32 bytes; Default = (+MAX, -MAX) (node.rs:20-27).
struct Node {
    Vec4 bound_min, bound_max;
    static Node empty();
    void unite(Vec4 v);  // Node::union, node.rs:40-43 (glam Vec4 min/max = SSE minps/maxps)
};
static_assert(sizeof(Node) == 32, "Node layout");

// src/scene/bvh/triangle.rs:7-13 — 64 bytes. `custom` = 3 x centroid before build, unit normal after.
struct Triangle {
    Vec4 a, b, c;
    Vec3 custom;
    uint32_t material;
};
static_assert(sizeof(Triangle) == 64, "Triangle layout");

// src/geometry/vertex.rs:5-9.
struct Vertex {
    float position[4], normal[4], color[4];
};

// src/geometry/mesh.rs:4-8.
struct Mesh {
    std::vector<Vertex> vertices;
    std::vector<uint32_t> indices;
    Material material;
    // Mesh::load_obj, mesh.rs:11-62 (tobj 4.0.3, default LoadOptions). Parse failure -> empty mesh.
    static Mesh load_obj(const char* data, size_t len, const Material& material);
};

// src/scene/bvh/tree.rs:8-14.
struct Tree {
    uint32_t sizes[2] = {0, 0};
    std::vector<Node> nodes;
    std::vector<Triangle> triangles;
    std::vector<Material> materials;
    void add_mesh(const Mesh& mesh);  // tree.rs:74-90
    void build(unsigned threads = 0);  // tree.rs:36-72; threads 0 = min(16, cores)
};

// render_ppm.rs:38-57 (pixel formatting part).
std::string render_ppm(const float* rgb, uint32_t width, uint32_t height);
// rendering_tests.rs:84-131. Returns 0 ok, 1 DifferentDimensions, 2 PixelCountMismatch, 3 ExcessiveDifference.
int compare_ppm_images(const std::string& a, const std::string& b, float tolerance_percent, float* avg_diff_percent);

}  // namespace hrt
