// scene.cpp — Camera::new, Material/Node helpers, Tree::add_mesh/build, render_ppm, compare_ppm_images.
// Compiled with -ffp-contract=off: Rust never contracts a*b+c, so neither do we.
#include "scene.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <thread>
#include <cstdlib>
#include <iterator>
#include <sstream>
#include <tuple>

namespace hrt {

float glam_dot(Vec3 a, Vec3 b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); }

Vec3 glam_cross(Vec3 a, Vec3 b) {
    return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}

Vec3 glam_normalize(Vec3 v) {
    float recip = 1.0f / std::sqrt(glam_dot(v, v));  // length_recip()
    return v * recip;
}

static Vec4 extend(Vec3 v, float w) { return {v.x, v.y, v.z, w}; }

Camera Camera::make(Vec3 from, Vec3 to, float focal_length, float focal_blur_amount, float fov) {
    // camera.rs:16-19
    Vec3 eye = from;
    Vec3 direction = glam_normalize(to - from);
    Vec3 right = glam_normalize(glam_cross(direction, Vec3{0.0f, 1.0f, 0.0f}));
    Vec3 up = glam_normalize(glam_cross(right, direction));
    Camera c;
    c.eye = extend(eye, 1.0f);
    c.direction = extend(direction, 1.0f);
    c.up = extend(up, 1.0f);
    c.right = extend(right, 1.0f);
    c.params = {focal_length, focal_blur_amount, fov, 0.0f};
    return c;
}

Material Material::lambertian(Vec3 albedo) { return {extend(albedo, 1.0f), {0.0f, 0.0f, 0.0f}, LAMBERTIAN}; }
Material Material::metal(Vec3 albedo, float fuzzy) { return {extend(albedo, 1.0f), {fuzzy, fuzzy, fuzzy}, METAL}; }
Material Material::dielectric(float ir) { return {{1.0f, 1.0f, 1.0f, 1.0f}, {ir, ir, ir}, DIELECTRIC}; }

Node Node::empty() { return {{FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX}, {-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX}}; }

// _mm_min_ps(a, b) = a < b ? a : b ; _mm_max_ps(a, b) = a > b ? a : b (second operand on NaN).
static inline float sse_min(float a, float b) { return a < b ? a : b; }
static inline float sse_max(float a, float b) { return a > b ? a : b; }

void Node::unite(Vec4 v) {
    bound_min = {sse_min(bound_min.x, v.x), sse_min(bound_min.y, v.y), sse_min(bound_min.z, v.z),
                 sse_min(bound_min.w, v.w)};
    bound_max = {sse_max(bound_max.x, v.x), sse_max(bound_max.y, v.y), sse_max(bound_max.z, v.z),
                 sse_max(bound_max.w, v.w)};
}

void Tree::add_mesh(const Mesh& mesh) {
    // tree.rs:74-90: one material per mesh; triangles in index order; custom = (a + b + c).xyz().
    uint32_t material = (uint32_t)materials.size();
    materials.push_back(mesh.material);
    for (size_t k = 0; k + 3 <= mesh.indices.size(); k += 3) {
        const float* pa = mesh.vertices[mesh.indices[k]].position;
        const float* pb = mesh.vertices[mesh.indices[k + 1]].position;
        const float* pc = mesh.vertices[mesh.indices[k + 2]].position;
        Triangle t;
        t.a = {pa[0], pa[1], pa[2], pa[3]};
        t.b = {pb[0], pb[1], pb[2], pb[3]};
        t.c = {pc[0], pc[1], pc[2], pc[3]};
        t.custom = {(pa[0] + pb[0]) + pc[0], (pa[1] + pb[1]) + pc[1], (pa[2] + pb[2]) + pc[2]};
        t.material = material;
        triangles.push_back(t);
    }
}

static size_t next_power_of_two(size_t v) {
    size_t n = 1;
    while (n < v) n <<= 1;
    return n;
}

namespace {

// Stable sort of (key, index) pairs by key, `a.first < b.first` (NaN never less: partial_cmp Equal).
// Without NaN keys it is an LSD radix sort on an order-preserving u32 image of the key (+0 and -0 mapped
// together, as `<` treats them as equal), which equals std::stable_sort element for element; any NaN key
// falls back to std::stable_sort itself.
void stable_sort_pairs(std::vector<std::pair<float, uint32_t>>& v, std::vector<std::pair<uint32_t, uint32_t>>& a,
                       std::vector<std::pair<uint32_t, uint32_t>>& b) {
    const size_t len = v.size();
    bool nan = false;
    for (const auto& p : v) nan |= std::isnan(p.first);
    if (len < 512 || nan) {
        std::stable_sort(v.begin(), v.end(), [](const std::pair<float, uint32_t>& x, const std::pair<float, uint32_t>& y) {
            return x.first < y.first;
        });
        return;
    }
    a.resize(len);
    b.resize(len);
    for (size_t k = 0; k < len; k++) {
        const float f = v[k].first == 0.0f ? 0.0f : v[k].first;
        uint32_t u;
        std::memcpy(&u, &f, 4);
        a[k] = {(u & 0x80000000u) ? ~u : (u | 0x80000000u), v[k].second};
    }
    for (int shift = 0; shift < 32; shift += 8) {
        size_t count[257] = {0};
        for (size_t k = 0; k < len; k++) count[((a[k].first >> shift) & 255u) + 1]++;
        if (count[((a[0].first >> shift) & 255u) + 1] == len) continue;  // one bucket: pass is a no-op
        for (int d = 0; d < 256; d++) count[d + 1] += count[d];
        for (size_t k = 0; k < len; k++) b[count[(a[k].first >> shift) & 255u]++] = a[k];
        a.swap(b);
    }
    for (size_t k = 0; k < len; k++) v[k].second = a[k].second;  // keys are not needed after the sort
}

// (the library reads no environment variables: a caller that wants another count passes it to
// rt_host_tree_build_threads)
unsigned default_threads() { return std::max(1u, std::min(16u, std::thread::hardware_concurrency())); }

}  // namespace

void Tree::build(unsigned threads) {
    // tree.rs:36-56: BFS over the padded power-of-two index space; stable sort of each range by the
    // centroid coordinate of axis depth % 3 (partial_cmp, NaN = Equal), split at the index midpoint.
    // Here the sorts permute a u32 index array (the 64-byte triangles move once, at the end), and a range
    // only needs its parent's sort to have happened first, so once the top levels have produced one range
    // per thread, each thread finishes whole subtrees on its own. A stable sort's output is unique for
    // the comparator, so the tree is byte-identical to the sequential BFS for any thread count.
    if (threads == 0) threads = default_threads();
    const size_t m = triangles.size();
    const size_t n = next_power_of_two(m);
    std::vector<uint32_t> perm(m);
    for (size_t k = 0; k < m; k++) perm[k] = (uint32_t)k;
    const float* key = m ? &triangles[0].custom.x : nullptr;  // custom of triangle k at key[k * 16 + axis]
    static_assert(sizeof(Triangle) == 64, "Triangle stride");
    // sort (key, index) pairs in a per-thread buffer: contiguous keys instead of one gather per compare
    using Pairs = std::vector<std::pair<float, uint32_t>>;
    using Keys = std::vector<std::pair<uint32_t, uint32_t>>;
    auto sort_range = [&](size_t i, size_t j, size_t depth, Pairs& tmp, Keys& ra, Keys& rb) -> bool {
        const size_t l = i, r = std::min(j, m);  // false: the range is not split further
        if (l + 1 >= r) return false;
        const size_t axis = depth % 3;
        tmp.resize(r - l);
        for (size_t k = l; k < r; k++) tmp[k - l] = {key[(size_t)perm[k] * 16u + axis], perm[k]};
        stable_sort_pairs(tmp, ra, rb);
        for (size_t k = l; k < r; k++) perm[k] = tmp[k - l].second;
        return true;
    };
    struct Range {
        size_t i, j, depth;
    };
    std::vector<Range> level{{0, n, 0}};
    Pairs tmp0;
    Keys ra0, rb0;
    while (!level.empty() && level.size() < threads) {  // top levels, sequentially
        std::vector<Range> next;
        for (const Range& g : level)
            if (sort_range(g.i, g.j, g.depth, tmp0, ra0, rb0)) {
                const size_t mid = (g.i + g.j) / 2;
                next.push_back({g.i, mid, g.depth + 1});
                next.push_back({mid, g.j, g.depth + 1});
            }
        level.swap(next);
    }
    auto subtrees = [&](size_t first, size_t step) {  // whole subtrees, depth first
        std::vector<Range> stack;
        Pairs tmp;
        Keys ra, rb;
        for (size_t k = first; k < level.size(); k += step) {
            stack.push_back(level[k]);
            while (!stack.empty()) {
                const Range g = stack.back();
                stack.pop_back();
                if (!sort_range(g.i, g.j, g.depth, tmp, ra, rb)) continue;
                const size_t mid = (g.i + g.j) / 2;
                stack.push_back({mid, g.j, g.depth + 1});
                stack.push_back({g.i, mid, g.depth + 1});
            }
        }
    };
    if (threads > 1 && level.size() > 1) {
        std::vector<std::thread> pool;
        for (unsigned t = 0; t < threads; t++) pool.emplace_back(subtrees, (size_t)t, (size_t)threads);
        for (auto& t : pool) t.join();
    } else {
        subtrees(0, 1);
    }
    std::vector<Triangle> sorted(m);
    for (size_t k = 0; k < m; k++) sorted[k] = triangles[perm[k]];
    triangles.swap(sorted);
    // tree.rs:57-65: leaf i is heap node i + n; every ancestor's box is the union of its vertices, united
    // triangle by triangle in index order. Without NaN coordinates that fold equals a bottom-up merge:
    // SSE min/max keep the LAST element equal to the extremum, and min(fold(L), fold(R)) picks exactly
    // that element of L ++ R (also for +-0). NaN makes the fold order-dependent: then the literal loop.
    nodes.assign(n, Node::empty());
    bool has_nan = false;
    for (const Triangle& t : triangles)
        for (const Vec4* v : {&t.a, &t.b, &t.c})
            has_nan |= std::isnan(v->x) || std::isnan(v->y) || std::isnan(v->z) || std::isnan(v->w);
    if (!has_nan) {
        for (size_t j = n / 2; j < n; j++)  // parents of leaves 2j, 2j + 1
            for (size_t c = 2 * j; c <= 2 * j + 1; c++)
                if (c - n < m) {
                    const Triangle& t = triangles[c - n];
                    nodes[j].unite(t.a);
                    nodes[j].unite(t.b);
                    nodes[j].unite(t.c);
                }
        for (size_t j = n / 2; j-- > 1;) {
            const Node& l = nodes[2 * j];
            const Node& r = nodes[2 * j + 1];
            nodes[j].bound_min = {sse_min(l.bound_min.x, r.bound_min.x), sse_min(l.bound_min.y, r.bound_min.y),
                                  sse_min(l.bound_min.z, r.bound_min.z), sse_min(l.bound_min.w, r.bound_min.w)};
            nodes[j].bound_max = {sse_max(l.bound_max.x, r.bound_max.x), sse_max(l.bound_max.y, r.bound_max.y),
                                  sse_max(l.bound_max.z, r.bound_max.z), sse_max(l.bound_max.w, r.bound_max.w)};
        }
    } else {
        for (size_t i = 0; i < m; i++) {
            const Triangle& t = triangles[i];
            size_t j = (i + n) / 2;
            while (j > 0) {
                nodes[j].unite(t.a);
                nodes[j].unite(t.b);
                nodes[j].unite(t.c);
                j /= 2;
            }
        }
    }
    // tree.rs:66-70: custom := unit geometric normal.
    for (Triangle& t : triangles) {
        Vec3 e1{t.b.x - t.a.x, t.b.y - t.a.y, t.b.z - t.a.z};
        Vec3 e2{t.c.x - t.a.x, t.c.y - t.a.y, t.c.z - t.a.z};
        t.custom = glam_normalize(glam_cross(e1, e2));
    }
    sizes[0] = (uint32_t)n;
    sizes[1] = (uint32_t)m;
}

// Rust `f as u8`: saturating, truncating toward zero, NaN -> 0.
static inline unsigned to_u8(float v) {
    if (!(v > 0.0f)) return 0;  // NaN, negatives, zero
    if (v >= 255.0f) return 255;
    return (unsigned)v;
}

std::string render_ppm(const float* rgb, uint32_t width, uint32_t height) {
    std::string out;
    out.reserve((size_t)width * height * 12 + 32);
    out += "P3\n";
    out += std::to_string(width) + " " + std::to_string(height) + " 255\n";
    char buf[32];
    const size_t npx = (size_t)width * height;
    for (size_t i = 0; i < npx; i++) {
        int len = std::snprintf(buf, sizeof buf, "%u %u %u ", to_u8(rgb[3 * i] * 255.0f),
                                to_u8(rgb[3 * i + 1] * 255.0f), to_u8(rgb[3 * i + 2] * 255.0f));
        out.append(buf, (size_t)len);
    }
    return out;
}

// str::lines(): split on '\n', strip one trailing '\r', no final empty line.
static std::vector<std::string> rust_lines(const std::string& s) {
    std::vector<std::string> out;
    size_t start = 0;
    while (start < s.size()) {
        size_t e = s.find('\n', start);
        size_t end = e == std::string::npos ? s.size() : e;
        std::string line = s.substr(start, end - start);
        if (!line.empty() && line.back() == '\r') line.pop_back();
        out.push_back(line);
        if (e == std::string::npos) break;
        start = e + 1;
    }
    return out;
}

// lines[2..].join(" ").split_whitespace().filter_map(|s| s.parse::<u8>().ok())
static std::vector<uint8_t> parse_pixels(const std::vector<std::string>& lines) {
    std::vector<uint8_t> px;
    for (size_t li = 2; li < lines.size(); li++) {
        std::istringstream ss(lines[li]);
        std::string tok;
        while (ss >> tok) {
            const char* p = tok.c_str();
            if (*p == '+') p++;  // u8::from_str accepts one leading '+'
            if (!*p) continue;
            unsigned v = 0;
            bool ok = true;
            for (; *p; p++) {
                if (*p < '0' || *p > '9') { ok = false; break; }
                v = v * 10 + (unsigned)(*p - '0');
                if (v > 255) { ok = false; break; }
            }
            if (ok) px.push_back((uint8_t)v);
        }
    }
    return px;
}

int compare_ppm_images(const std::string& a, const std::string& b, float tolerance_percent, float* avg_diff_percent) {
    auto l1 = rust_lines(a), l2 = rust_lines(b);
    if (l1.size() < 2 || l2.size() < 2 || l1[1] != l2[1]) return 1;
    auto p1 = parse_pixels(l1), p2 = parse_pixels(l2);
    if (p1.size() != p2.size()) return 2;
    float total = 0.0f;  // Iterator<f32>::sum: sequential f32 accumulation
    for (size_t i = 0; i < p1.size(); i++) total += std::fabs((float)p1[i] - (float)p2[i]);
    float avg = total / (float)p1.size();
    float pct = (avg / 255.0f) * 100.0f;
    if (avg_diff_percent) *avg_diff_percent = pct;
    return pct > tolerance_percent ? 3 : 0;
}

}  // namespace hrt
