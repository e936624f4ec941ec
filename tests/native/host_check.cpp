// host_check.cpp — TEST INFRASTRUCTURE: the host-side code (OBJ ingest, Tree::build, the sphere and triangle
// BVH builders, render_ppm / compare_ppm_images) and the CPU oracle, built with -fsanitize=address,undefined
// (tests/native/Makefile, SAN=1) and driven over the shipped assets, a corpus of malformed OBJ inputs and
// seeded random mutations of them (sanitizers on the CPU restatement and the host builders;
// VERDICT r2 item 7). Run by tests/test_sanitizers.py; any ASan/UBSan report aborts with a non-zero status.
//
// usage: host_check <dir with decompressed *.obj assets> [mutations]
#include <dirent.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../hello-raytracing_amd/csrc/host/scene.hpp"
#include "../../hello-raytracing_amd/csrc/host/sphere_bvh.hpp"
#include "../../hello-raytracing_amd/csrc/host/tri_bvh.hpp"
#include "../../include/hrt.h"

extern "C" {
// oracle/rt_oracle.c (its o_params layout: 16 u32)
struct o_params {
    uint32_t width, height, mode, bounces, ema_cap, frame0, time0, dtime, frames, x0, nx, row0, row_step, nrows,
        row_block, step_cap;
};
uint64_t oracle_render(const o_params* p, const void* camera80, const void* spheres48, uint32_t nslots,
                       const uint32_t* sizes, const void* nodes32, const void* tris64, const void* mats32,
                       float* image, int threads, uint64_t* counts);
uint32_t oracle_sizeof(int which);
}

namespace {

int g_fail = 0;
#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                             \
        }                                                                         \
    } while (0)

uint64_t g_rng = 0x9E3779B97F4A7C15ull;
uint64_t rnd() {  // xorshift64*
    g_rng ^= g_rng >> 12;
    g_rng ^= g_rng << 25;
    g_rng ^= g_rng >> 27;
    return g_rng * 2685821657736338717ull;
}

const hrt::Material kMat = hrt::Material::lambertian({0.5f, 0.5f, 0.5f});

struct Loaded {
    uint32_t nv = 0, ni = 0;
    rt_mesh* m = nullptr;
};

Loaded load(const std::string& text) {
    Loaded L;
    CHECK(rt_host_mesh_load_obj(text.data(), text.size(), &kMat, &L.m) == RT_OK);
    CHECK(rt_host_mesh_counts(L.m, &L.nv, &L.ni) == RT_OK);
    return L;
}

// Tree::add_mesh + Tree::build (sequential and threaded: byte-identical), and the SAH triangle tree over it.
void build_trees(const rt_mesh* m, bool sah) {
    rt_tree* t1 = nullptr;
    rt_tree* t4 = nullptr;
    CHECK(rt_host_tree_new(&t1) == RT_OK && rt_host_tree_new(&t4) == RT_OK);
    CHECK(rt_host_tree_add_mesh(t1, m) == RT_OK && rt_host_tree_add_mesh(t4, m) == RT_OK);
    CHECK(rt_host_tree_build_threads(t1, 1) == RT_OK && rt_host_tree_build_threads(t4, 4) == RT_OK);
    uint32_t s1[2], s4[2], nn1, nt1, nm1, nn4, nt4, nm4;
    const void *n1, *tr1, *m1, *n4, *tr4, *m4;
    CHECK(rt_host_tree_view(t1, s1, &n1, &nn1, &tr1, &nt1, &m1, &nm1) == RT_OK);
    CHECK(rt_host_tree_view(t4, s4, &n4, &nn4, &tr4, &nt4, &m4, &nm4) == RT_OK);
    CHECK(s1[0] == s4[0] && s1[1] == s4[1] && nn1 == nn4 && nt1 == nt4);
    CHECK(nn1 == 0 || std::memcmp(n1, n4, (size_t)nn1 * 32) == 0);
    CHECK(nt1 == 0 || std::memcmp(tr1, tr4, (size_t)nt1 * 64) == 0);
    if (sah && nt1) {
        const hrt::Triangle* T = (const hrt::Triangle*)tr1;
        std::vector<float> aee;
        for (uint32_t j = 0; j < nt1; j++) {
            const float v[9] = {T[j].a.x, T[j].a.y, T[j].a.z, T[j].b.x - T[j].a.x, T[j].b.y - T[j].a.y,
                                T[j].b.z - T[j].a.z, T[j].c.x - T[j].a.x, T[j].c.y - T[j].a.y, T[j].c.z - T[j].a.z};
            aee.insert(aee.end(), v, v + 9);
        }
        const hrt::TriBvh b = hrt::build_tri_bvh(aee);
        CHECK(b.order.size() <= nt1);  // triangles with non-finite vertices are left out (tri_bvh.cpp)
    }
    rt_host_tree_destroy(t1);
    rt_host_tree_destroy(t4);
}

std::string read_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

void check_assets(const std::string& dir, std::vector<std::string>& texts) {
    DIR* d = opendir(dir.c_str());
    CHECK(d != nullptr);
    if (!d) return;
    int n = 0;
    while (dirent* e = readdir(d)) {
        const std::string name = e->d_name;
        if (name.size() < 5 || name.substr(name.size() - 4) != ".obj") continue;
        const std::string text = read_file(dir + "/" + name);
        Loaded L = load(text);
        CHECK(L.ni > 0 && L.ni % 3 == 0);  // every shipped OBJ loads, all faces triangles
        build_trees(L.m, L.ni <= 3 * 60000);
        rt_host_mesh_destroy(L.m);
        std::printf("asset %s: %u vertices, %u indices\n", name.c_str(), L.nv, L.ni);
        if (text.size() < 300000) texts.push_back(text);
        n++;
    }
    closedir(d);
    CHECK(n > 0);
}

// Malformed inputs (tobj LoadError -> an empty mesh, mesh.rs:53-59) and a few well-formed edge cases.
void check_malformed() {
    const std::string tri = "v 0 0 0\nv 1 0 0\nv 0 1 0\n";
    struct Case {
        std::string text;
        int expect_indices;  // -1: any
    };
    const std::vector<Case> cases = {
        {"", 0},
        {"# only a comment\n", 0},
        {tri + "f 1 2 3\n", 3},
        {tri + "f 1 2 3", 3},                       // no final newline
        {tri + "f 1 2 3\r\n", 3},                   // CRLF
        {tri + "f -3 -2 -1\n", 3},                  // relative indices
        {tri + "f 1/1/1 2/2/2 3/3/3\n", 3},         // position/texture/normal triples
        {tri + "f 0 1 2\n", 0},                     // index 0 (1-based format)
        {tri + "f 1 2 4\n", 0},                     // one past the end
        {tri + "f 1 2 -4\n", 0},                    // relative before the first vertex
        {tri + "f 1 2 99999999999999999999\n", 0},  // overflows i64
        {tri + "f 1 2 6148914691236517206\n", 0},   // (v - 1) * 3 wraps size_t
        {tri + "f 1 2 9223372036854775807\n", 0},
        {tri + "f 1 2 -9223372036854775808\n", 0},
        {tri + "f 1 2 3x\n", 0},                    // trailing garbage
        {tri + "f 1 2 /3\n", 0},                    // empty position index
        {tri + "f 1 2 3/\n", 3},
        {tri + "f\n", 0},                           // face without corners
        {tri + "f 1 2\n", 2},                       // two corners: indices, no triangle
        {"v 0 0\n", 0},                             // truncated position
        {"v 0 0 nan(1)\n", 0},
        {"v 0x1p3 0 0\n", 0},                       // hex float (Rust rejects)
        {"v inf -inf NaN\nv 1 0 0\nv 0 1 0\nf 1 2 3\n", 3},
        {"v 1e39 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n", 3},  // overflows f32: inf
        {tri + "f 1 2 3\n\xff\n", 0},               // invalid UTF-8 line: ReadError
        {tri + "f 1 2 3\n# caf\xc3\xa9\n", 3},      // valid UTF-8 in a comment
        {tri + "f 1 2 \xc3\n", 0},                  // truncated UTF-8 sequence
        {tri + "f 1 2 \xed\xa0\x80\n", 0},          // surrogate
        {tri + "f 1\xc2\xa0" "2 3\n", 3},           // U+00A0 splits words (char::is_whitespace)
        {tri + "o a\nf 1 2 3\no b\nf 3 2 1\n", 6},  // two models
        {tri + "g\ng\nf 1 2 3\n", 3},
        {std::string("v 0 0 0\0v 1 0 0\n", 16), 0},  // NUL inside a word
    };
    for (size_t k = 0; k < cases.size(); k++) {
        Loaded L = load(cases[k].text);
        if (cases[k].expect_indices >= 0 && (int)L.ni != cases[k].expect_indices) {
            std::fprintf(stderr, "malformed case %zu: %u indices, expected %d\n", k, L.ni, cases[k].expect_indices);
            g_fail++;
        }
        build_trees(L.m, true);
        rt_host_mesh_destroy(L.m);
    }
    std::printf("malformed corpus: %zu cases\n", cases.size());
}

// Seeded mutations of real OBJ text: byte flips, random bytes, truncation, line duplication / deletion.
void check_mutations(const std::vector<std::string>& texts, int count) {
    if (texts.empty()) return;
    const char alphabet[] = "vf/-+.0123456789 \n\teEnaix\xff\xc3\x80og#";
    int nonempty = 0;
    for (int k = 0; k < count; k++) {
        std::string t = texts[rnd() % texts.size()];
        const int edits = 1 + (int)(rnd() % 8);
        for (int e = 0; e < edits && !t.empty(); e++) {
            const size_t at = rnd() % t.size();
            switch (rnd() % 6) {
            case 0: t[at] = (char)(rnd() & 0xFF); break;
            case 1: t[at] = alphabet[rnd() % (sizeof alphabet - 1)]; break;
            case 2: t.resize(at); break;
            case 3: t.insert(at, 1, alphabet[rnd() % (sizeof alphabet - 1)]); break;
            case 4: {
                const size_t nl = t.find('\n', at);
                if (nl != std::string::npos) t.insert(at, t.substr(at, nl - at + 1));
                break;
            }
            default: {
                const size_t nl = t.find('\n', at);
                t.erase(at, nl == std::string::npos ? std::string::npos : nl - at);
                break;
            }
            }
        }
        Loaded L = load(t);
        nonempty += L.ni > 0;
        build_trees(L.m, (k % 16) == 0);
        rt_host_mesh_destroy(L.m);
    }
    std::printf("mutations: %d (%d loaded non-empty)\n", count, nonempty);
}

void check_ppm() {
    const uint32_t W = 7, H = 5;
    std::vector<float> img(W * H * 3);
    for (size_t i = 0; i < img.size(); i++) {
        const uint64_t r = rnd();
        const float special[] = {NAN, INFINITY, -INFINITY, -0.0f, 1e30f, -1e30f, 0.999999f, 1.0f};
        img[i] = (r & 7) == 0 ? special[(r >> 3) & 7] : (float)((double)(r >> 11) / 9007199254740992.0 * 1.5);
    }
    size_t len = 0;
    CHECK(rt_host_render_ppm(img.data(), W, H, nullptr, 0, &len) == RT_OK && len > 0);
    std::string a(len, '\0');
    CHECK(rt_host_render_ppm(img.data(), W, H, &a[0], len, &len) == RT_OK);
    std::string small(8, '\0');
    size_t len2 = 0;
    CHECK(rt_host_render_ppm(img.data(), W, H, &small[0], small.size(), &len2) == RT_OK && len2 == len);
    int code = 0;
    float pct = -1.0f;
    CHECK(rt_host_compare_ppm(a.data(), a.size(), a.data(), a.size(), 2.0f, &code, &pct) == RT_OK && pct == 0.0f);
    const std::vector<std::string> bad = {"", "P3\n", "P3\n7 5 255\n", "P3\n7 5 255\n1 2", "P6\n7 5 255\n",
                                          "P3\n-1 5 255\n", "P3\n99999999999 5 255\n", "P3\n7 5 255\n300 -4 x ",
                                          std::string("P3\n7 5 255\n\0\0", 13), a.substr(0, a.size() / 2)};
    for (const std::string& b : bad) {
        code = 0;
        (void)rt_host_compare_ppm(a.data(), a.size(), b.data(), b.size(), 2.0f, &code, &pct);
        (void)rt_host_compare_ppm(b.data(), b.size(), a.data(), a.size(), 2.0f, &code, &pct);
    }
    for (int k = 0; k < 200; k++) {  // random bytes as both images
        std::string r1(rnd() % 64, '\0'), r2 = a;
        for (char& c : r1) c = (char)(rnd() & 0xFF);
        r2[rnd() % r2.size()] = (char)(rnd() & 0xFF);
        (void)rt_host_compare_ppm(r1.data(), r1.size(), r2.data(), r2.size(), 2.0f, &code, &pct);
        (void)rt_host_compare_ppm(r2.data(), r2.size(), a.data(), a.size(), 2.0f, &code, &pct);
    }
    std::printf("ppm: ok\n");
}

// The culling BVH builder over random and degenerate sphere sets (zero, NaN, infinite and huge radii).
void check_sphere_bvh() {
    for (int k = 0; k < 60; k++) {
        const size_t n = rnd() % 600;
        std::vector<float> cr(4 * n);
        for (size_t i = 0; i < n; i++) {
            for (int c = 0; c < 3; c++) cr[4 * i + c] = (float)((int64_t)(rnd() % 2001) - 1000) * 0.01f;
            cr[4 * i + 3] = 0.01f + (float)(rnd() % 100) * 0.01f;
            switch (rnd() % 40) {
            case 0: cr[4 * i + 3] = 0.0f; break;
            case 1: cr[4 * i + 3] = NAN; break;
            case 2: cr[4 * i] = INFINITY; break;
            case 3: cr[4 * i + 3] = 1000.0f; break;
            case 4: cr[4 * i + 3] = -0.5f; break;
            case 5: cr[4 * i + 1] = 1e30f; break;
            default: break;
            }
        }
        const hrt::SphereBvh b = hrt::build_sphere_bvh(cr);
        CHECK(b.slot.size() + b.large.size() <= n);
        for (int32_t s : b.slot) CHECK(s >= 0 && (size_t)s < n);
    }
    std::printf("sphere bvh: ok\n");
}

// The oracle (sphere, triangle and mixed programs) on a few small scenes.
void check_oracle(const std::string& suzanne) {
    CHECK(oracle_sizeof(5) == sizeof(o_params));
    const hrt::Camera cam = hrt::Camera::make({0.0f, 1.0f, 4.0f}, {0.0f, 0.0f, 0.0f}, 4.0f, 0.05f, 0.9f);
    std::vector<hrt::Sphere> sph;
    for (int i = 0; i < 40; i++) {
        hrt::Sphere s{};
        s.center = {(float)(i % 7) - 3.0f, 0.0f, (float)(i / 7) - 3.0f};
        s.radius = 0.3f;
        s.material = i % 3 == 0 ? hrt::Material::dielectric(1.5f)
                                : i % 3 == 1 ? hrt::Material::metal({0.8f, 0.8f, 0.8f}, 0.2f) : kMat;
        sph.push_back(s);
    }
    o_params p{};
    p.width = 24;
    p.height = 16;
    p.bounces = 8;
    p.ema_cap = 1000;
    p.time0 = 1000;
    p.dtime = 10;
    p.frames = 3;
    p.nx = p.width;
    p.row0 = 1;
    p.row_step = 2;
    p.row_block = 3;
    p.nrows = 8;
    p.step_cap = 600;
    std::vector<float> img((size_t)p.nrows * p.nx * 3);
    uint64_t counts[4];
    p.mode = 0;
    CHECK(oracle_render(&p, &cam, sph.data(), (uint32_t)sph.size(), nullptr, nullptr, nullptr, nullptr, img.data(), 2,
                        counts) > 0);
    Loaded L = load(suzanne);
    rt_tree* t = nullptr;
    CHECK(rt_host_tree_new(&t) == RT_OK && rt_host_tree_add_mesh(t, L.m) == RT_OK && rt_host_tree_build(t) == RT_OK);
    uint32_t sizes[2], nn, nt, nm;
    const void *nodes, *tris, *mats;
    CHECK(rt_host_tree_view(t, sizes, &nodes, &nn, &tris, &nt, &mats, &nm) == RT_OK);
    for (uint32_t mode = 1; mode <= 2; mode++) {
        p.mode = mode;
        p.bounces = 5;
        std::fill(img.begin(), img.end(), 0.0f);
        CHECK(oracle_render(&p, &cam, mode == 2 ? sph.data() : nullptr, mode == 2 ? 4u : 0u, sizes, nodes, tris, mats,
                            img.data(), 2, counts) > 0);
    }
    rt_host_tree_destroy(t);
    rt_host_mesh_destroy(L.m);
    std::printf("oracle: ok\n");
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <asset dir> [mutations]\n", argv[0]);
        return 2;
    }
    const int mutations = argc > 2 ? std::atoi(argv[2]) : 3000;
    std::vector<std::string> texts;
    check_assets(argv[1], texts);
    check_malformed();
    check_mutations(texts, mutations);
    check_ppm();
    check_sphere_bvh();
    std::string suzanne;
    for (const std::string& t : texts)
        if (t.find("o Suzanne") != std::string::npos) suzanne = t;
    if (suzanne.empty() && !texts.empty()) suzanne = texts[0];
    check_oracle(suzanne);
    std::printf("host_check: %d failures\n", g_fail);
    return g_fail ? 1 : 0;
}
