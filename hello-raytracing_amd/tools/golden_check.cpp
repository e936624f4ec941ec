// golden_check.cpp — native restatement of the reference's golden-image harness
// (hucancode/hello-raytracing tests/rendering_tests.rs), driving the MI355X renderer through the C-ABI
// only, the way a Rust caller would: #[repr(C)] PODs built on the host, Scene::init (set_camera +
// write_scene_data), TEST_FRAMES x {set_time(1000 + i*10); draw()}, render_ppm, compare_ppm_images.
//
// usage: golden_check <golden_dir> <output_dir> [frames=100] [tolerance_percent=2.0]
// golden_dir holds <name>.ppm (ASCII P3, the reference's files). Exit status 0 iff every scene passes.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/hrt.h"

namespace {

// src/scene/material.rs:9-13, sphere.rs:6-10 (as the Rust side lays them out)
struct Material {
    float albedo[4];
    float params[3];
    uint32_t kind;
};
struct Sphere {
    float center[3];
    float radius;
    Material material;
};
static_assert(sizeof(Sphere) == 48, "Sphere POD");

Sphere lambertian(float x, float y, float z, float r, float cr, float cg, float cb) {
    return Sphere{{x, y, z}, r, Material{{cr, cg, cb, 1.0f}, {0, 0, 0}, RT_LAMBERTIAN}};
}
Sphere metal(float x, float y, float z, float r, float cr, float cg, float cb, float fuzz) {
    return Sphere{{x, y, z}, r, Material{{cr, cg, cb, 1.0f}, {fuzz, fuzz, fuzz}, RT_METAL}};
}
Sphere dielectric(float x, float y, float z, float r, float ir) {
    return Sphere{{x, y, z}, r, Material{{1, 1, 1, 1}, {ir, ir, ir}, RT_DIELECTRIC}};
}

struct Scene {
    std::string name;
    unsigned char camera[80];
    std::vector<Sphere> objects;
};

void camera(unsigned char* out, float fx, float fy, float fz, float tx, float ty, float tz, float focal, float blur,
            float fov) {
    const float from[3] = {fx, fy, fz}, to[3] = {tx, ty, tz};
    if (rt_host_camera_new(from, to, focal, blur, fov, out) != RT_OK) std::abort();
}

// rendering_tests.rs:134-509; the default camera is SceneSphere::new's (scene_sphere.rs:38-39)
std::vector<Scene> golden_scenes() {
    const float PI = 3.14159265358979323846f;
    std::vector<Scene> s(7);
    for (auto& sc : s) camera(sc.camera, 0, 0, 3.5f, 0, 0, 0, 3.5f, 0.04f, PI * 0.2f);
    s[0].name = "lambertian_materials";
    s[0].objects = {lambertian(-2, 0, -5, 1, 0.8f, 0.2f, 0.2f), lambertian(0, 0, -5, 1, 0.2f, 0.8f, 0.2f),
                    lambertian(2, 0, -5, 1, 0.2f, 0.2f, 0.8f), lambertian(0, -101, -5, 100, 0.5f, 0.5f, 0.5f)};
    s[1].name = "metal_materials";
    s[1].objects = {metal(-2, 0, -5, 1, 0.8f, 0.8f, 0.8f, 0.0f), metal(0, 0, -5, 1, 0.8f, 0.6f, 0.2f, 0.2f),
                    metal(2, 0, -5, 1, 0.6f, 0.2f, 0.8f, 0.5f), lambertian(0, -101, -5, 100, 0.5f, 0.5f, 0.5f)};
    s[2].name = "dielectric_materials";
    s[2].objects = {dielectric(0, 0, -5, 1.5f, 1.5f), dielectric(-2, 0, -4, 0.5f, 1.33f),
                    dielectric(2, 0, -4, 0.5f, 2.4f), lambertian(0, 0, -8, 1, 1, 0, 0),
                    lambertian(0, -101.5f, -5, 100, 0.5f, 0.5f, 0.5f)};
    s[3].name = "camera_position";
    for (int i = -2; i <= 2; i++)
        s[3].objects.push_back(lambertian((float)i * 1.5f, 0, -5.0f - (float)std::abs(i), 0.5f, 0.5f + (float)i * 0.1f,
                                          0.5f, 0.5f - (float)i * 0.1f));
    s[3].objects.push_back(lambertian(0, -100.5f, -5, 100, 0.5f, 0.5f, 0.5f));
    camera(s[3].camera, 3.0f, 1.5f, -2.0f, 0, 0, -5, 5.0f, 0.1f, 0.8f);
    s[4].name = "depth_of_field";
    for (int i = -3; i <= 3; i++)
        s[4].objects.push_back(lambertian((float)i, 0, -3.0f - (float)std::abs(i) * 2.0f, 0.4f,
                                          1.0f - (float)(i + 3) / 6.0f, 0.5f, (float)(i + 3) / 6.0f));
    s[4].objects.push_back(lambertian(0, -100.4f, -5, 100, 0.5f, 0.5f, 0.5f));
    camera(s[4].camera, 0, 1, 0, 0, 0, -5, 5.0f, 0.3f, 0.8f);
    s[5].name = "complex_scene";
    for (int i = -2; i <= 2; i++)
        for (int j = -2; j <= 2; j++) {
            if (i == 0 && j == 0) {
                s[5].objects.push_back(dielectric(0, 0, -5, 0.8f, 1.5f));
                continue;
            }
            const float x = (float)i * 1.2f, z = -5.0f + (float)j * 1.2f;
            switch (std::abs(i + j) % 3) {
            case 0: s[5].objects.push_back(lambertian(x, 0, z, 0.3f, 0.7f, 0.3f, 0.3f)); break;
            case 1: s[5].objects.push_back(metal(x, 0, z, 0.3f, 0.7f, 0.7f, 0.7f, 0.1f)); break;
            default: s[5].objects.push_back(dielectric(x, 0, z, 0.3f, 1.33f)); break;
            }
        }
    s[5].objects.push_back(lambertian(0, -100.3f, -5, 100, 0.5f, 0.5f, 0.5f));
    s[6].name = "shadow_rendering";
    s[6].objects = {lambertian(0, 2, -5, 2, 0.7f, 0.3f, 0.3f), lambertian(0, -0.5f, -5, 0.5f, 0.3f, 0.7f, 0.3f),
                    lambertian(0, -101, -5, 100, 0.8f, 0.8f, 0.8f)};
    return s;
}

bool read_file(const std::string& path, std::string* out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    *out = ss.str();
    return true;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <golden_dir> <output_dir> [frames=100] [tolerance=2.0]\n", argv[0]);
        return 2;
    }
    const std::string gdir = argv[1], odir = argv[2];
    const uint32_t frames = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 100u;
    const float tol = argc > 4 ? (float)std::atof(argv[4]) : 2.0f;
    const uint32_t W = 512, H = 512;
    int failures = 0;
    for (const Scene& sc : golden_scenes()) {
        rt_renderer* r = nullptr;
        if (rt_create(W, H, RT_MODE_SPHERE, &r) != RT_OK) {
            std::fprintf(stderr, "rt_create: %s\n", rt_last_error());
            return 3;
        }
        // Scene::init (mod.rs:69-72): set_camera + write_scene_data (scene_sphere.rs:24-31) (truncated to MAX_OBJECT_IN_SCENE)
        const uint32_t n = (uint32_t)std::min<size_t>(sc.objects.size(), RT_MAX_OBJECT_IN_SCENE);
        if (rt_set_camera(r, sc.camera) || rt_set_spheres(r, sc.objects.data(), n)) return 3;
        for (uint32_t i = 0; i < frames; i++) {  // rendering_tests.rs:22-25
            if (rt_set_time(r, 1000 + i * 10) || rt_draw(r)) {
                std::fprintf(stderr, "draw: %s\n", rt_last_error());
                return 3;
            }
        }
        std::vector<float> img((size_t)W * H * 3);
        if (rt_read_image(r, img.data(), img.size())) return 3;
        rt_destroy(r);
        size_t len = 0;
        rt_host_render_ppm(img.data(), W, H, nullptr, 0, &len);
        std::string ppm(len, '\0');
        rt_host_render_ppm(img.data(), W, H, &ppm[0], len, &len);
        std::ofstream(odir + "/" + sc.name + ".ppm", std::ios::binary) << ppm;
        std::string golden;
        if (!read_file(gdir + "/" + sc.name + ".ppm", &golden)) {
            std::printf("%-22s MISSING golden\n", sc.name.c_str());
            failures++;
            continue;
        }
        int code = 0;
        float pct = NAN;
        const int rc = rt_host_compare_ppm(ppm.data(), ppm.size(), golden.data(), golden.size(), tol, &code, &pct);
        std::printf("%-22s %s avg_diff=%.4f%% (tolerance %.2f%%)\n", sc.name.c_str(), rc == RT_OK ? "PASS" : "FAIL", pct,
                    tol);
        if (rc != RT_OK) failures++;
    }
    return failures ? 1 : 0;
}
