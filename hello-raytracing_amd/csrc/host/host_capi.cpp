// host_capi.cpp — rt_host_* C-ABI over the host scene builders (scene.hpp). Pure CPU.
#include <cstring>
#include <new>
#include <string>

#include "../../../include/hrt.h"
#include "scene.hpp"

struct rt_mesh {
    hrt::Mesh mesh;
};
struct rt_tree {
    hrt::Tree tree;
};

extern "C" {

int rt_host_camera_new(const float from[3], const float to[3], float focal_length, float focal_blur_amount,
                       float fov, void* camera80_out) {
    if (!from || !to || !camera80_out) return RT_ERR_ARG;
    hrt::Camera c = hrt::Camera::make({from[0], from[1], from[2]}, {to[0], to[1], to[2]}, focal_length,
                                      focal_blur_amount, fov);
    std::memcpy(camera80_out, &c, sizeof c);
    return RT_OK;
}

int rt_host_mesh_load_obj(const char* data, size_t len, const void* material32, rt_mesh** out) {
    if (!out || !material32 || (len && !data)) return RT_ERR_ARG;
    hrt::Material mat;
    std::memcpy(&mat, material32, sizeof mat);
    rt_mesh* m = new (std::nothrow) rt_mesh();
    if (!m) return RT_ERR_ALLOC;
    m->mesh = hrt::Mesh::load_obj(data, len, mat);
    *out = m;
    return RT_OK;
}

int rt_host_mesh_counts(const rt_mesh* m, uint32_t* nv, uint32_t* ni) {
    if (!m) return RT_ERR_ARG;
    if (nv) *nv = (uint32_t)m->mesh.vertices.size();
    if (ni) *ni = (uint32_t)m->mesh.indices.size();
    return RT_OK;
}

int rt_host_mesh_destroy(rt_mesh* m) {
    delete m;
    return RT_OK;
}

int rt_host_tree_new(rt_tree** out) {
    if (!out) return RT_ERR_ARG;
    *out = new (std::nothrow) rt_tree();
    return *out ? RT_OK : RT_ERR_ALLOC;
}

int rt_host_tree_add_mesh(rt_tree* t, const rt_mesh* m) {
    if (!t || !m) return RT_ERR_ARG;
    t->tree.add_mesh(m->mesh);
    return RT_OK;
}

int rt_host_tree_build(rt_tree* t) {
    if (!t) return RT_ERR_ARG;
    t->tree.build();
    return RT_OK;
}

int rt_host_tree_build_threads(rt_tree* t, int threads) {
    if (!t || threads < 0) return RT_ERR_ARG;
    t->tree.build((unsigned)threads);
    return RT_OK;
}

int rt_host_tree_view(const rt_tree* t, uint32_t sizes[2], const void** nodes32, uint32_t* n_nodes,
                      const void** tris64, uint32_t* n_tris, const void** mats32, uint32_t* n_mats) {
    if (!t) return RT_ERR_ARG;
    const hrt::Tree& tr = t->tree;
    if (sizes) { sizes[0] = tr.sizes[0]; sizes[1] = tr.sizes[1]; }
    if (nodes32) *nodes32 = tr.nodes.data();
    if (n_nodes) *n_nodes = (uint32_t)tr.nodes.size();
    if (tris64) *tris64 = tr.triangles.data();
    if (n_tris) *n_tris = (uint32_t)tr.triangles.size();
    if (mats32) *mats32 = tr.materials.data();
    if (n_mats) *n_mats = (uint32_t)tr.materials.size();
    return RT_OK;
}

int rt_host_tree_destroy(rt_tree* t) {
    delete t;
    return RT_OK;
}

int rt_host_render_ppm(const float* rgb, uint32_t width, uint32_t height, char* out, size_t cap, size_t* len) {
    if (!rgb || !len) return RT_ERR_ARG;
    std::string s = hrt::render_ppm(rgb, width, height);
    *len = s.size();
    if (out && cap) std::memcpy(out, s.data(), s.size() < cap ? s.size() : cap);
    return RT_OK;
}

int rt_host_compare_ppm(const char* img1, size_t len1, const char* img2, size_t len2, float tolerance_percent,
                        int* code, float* avg_diff_percent) {
    if ((len1 && !img1) || (len2 && !img2)) return RT_ERR_ARG;
    int c = hrt::compare_ppm_images(std::string(img1 ? img1 : "", len1), std::string(img2 ? img2 : "", len2),
                                    tolerance_percent, avg_diff_percent);
    if (code) *code = c;
    return c == 0 ? RT_OK : RT_ERR_COMPARE;
}

}  // extern "C"
