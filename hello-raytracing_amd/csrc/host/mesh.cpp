// mesh.cpp — Mesh::load_obj (src/geometry/mesh.rs:11-62) over a minimal tobj-4.0.3-compatible parser.
//
// What the hot path depends on is only the triangle list that Tree::add_mesh derives from it: face
// corners in file order, models concatenated in file order, positions parsed as correctly rounded f32.
// The parser also reproduces tobj's per-model vertex numbering (default LoadOptions: single_index =
// false, triangulate = false -> positions are de-duplicated per model by position index, in order of
// first reference), so Mesh::vertices.len() matches the reference's unit tests (mesh.rs:64-89).
// Like the reference, any tobj LoadError (bad float, out-of-bounds face index, a line that is not UTF-8:
// BufRead::lines() -> ReadError) yields an EMPTY mesh. Words are split as Rust's str::split_whitespace does
// (Unicode White_Space, not only ASCII).
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "scene.hpp"

namespace hrt {
namespace {

struct ObjModel {
    std::vector<float> positions;  // de-duplicated per model
    std::vector<uint32_t> indices;
};

struct Parser {
    std::vector<float> pos;  // all `v` positions of the file (x, y, z)
    std::vector<std::vector<long>> faces;  // position index per corner, resolved to 0-based
    std::vector<ObjModel> models;
    bool failed = false;

    static bool parse_f32(const std::string& w, float* out) {
        if (w.empty()) return false;
        const char* s = w.c_str();
        char* end = nullptr;
        errno = 0;
        float v = std::strtof(s, &end);
        if (end != s + w.size()) return false;
        // Rust's f32::from_str rejects hex floats and "nan(...)"; strtof accepts them.
        if (w.find_first_of("xX(") != std::string::npos) return false;
        *out = v;
        return true;
    }

    // tobj parse_index: 1-based, negative = relative to the current count; empty = missing.
    static bool parse_index(const std::string& s, size_t count, long* out) {
        if (s.empty()) { *out = -1; return true; }
        char* end = nullptr;
        long i = std::strtol(s.c_str(), &end, 10);
        if (end != s.c_str() + s.size()) return false;
        *out = i < 0 ? (long)count + i : i - 1;
        return true;
    }

    void flush_model() {
        if (faces.empty()) return;
        ObjModel m;
        std::unordered_map<long, uint32_t> index_map;  // export_faces_multi_index / add_vertex_multi_index
        for (const auto& f : faces) {
            for (long v : f) {
                auto it = index_map.find(v);
                if (it != index_map.end()) {
                    m.indices.push_back(it->second);
                    continue;
                }
                if (v < 0 || (size_t)v >= pos.size() / 3) { failed = true; return; }  // FaceVertexOutOfBounds
                uint32_t next = (uint32_t)index_map.size();
                m.positions.push_back(pos[(size_t)v * 3]);
                m.positions.push_back(pos[(size_t)v * 3 + 1]);
                m.positions.push_back(pos[(size_t)v * 3 + 2]);
                m.indices.push_back(next);
                index_map.emplace(v, next);
            }
        }
        models.push_back(std::move(m));
        faces.clear();
    }

    // One UTF-8 scalar value at ln[i]: its length in bytes (0 = invalid: overlong, surrogate, > U+10FFFF,
    // truncated) and the code point.
    static size_t utf8_at(const std::string& ln, size_t i, uint32_t* cp) {
        const unsigned char c = (unsigned char)ln[i];
        if (c < 0x80) { *cp = c; return 1; }
        size_t n = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC2 ? 2 : 0;
        if (n == 0 || c > 0xF4 || i + n > ln.size()) return 0;
        uint32_t v = c & (0x7Fu >> n);
        for (size_t k = 1; k < n; k++) {
            const unsigned char d = (unsigned char)ln[i + k];
            if ((d & 0xC0) != 0x80) return 0;
            v = (v << 6) | (d & 0x3Fu);
        }
        if ((n == 3 && v < 0x800) || (n == 4 && (v < 0x10000 || v > 0x10FFFF)) || (v >= 0xD800 && v <= 0xDFFF)) return 0;
        *cp = v;
        return n;
    }
    // char::is_whitespace (Unicode White_Space)
    static bool is_ws(uint32_t c) {
        return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
               (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
    }

    void line(const std::string& ln) {
        std::vector<std::string> w;
        size_t i = 0, s = 0;
        bool in_word = false;
        while (i < ln.size()) {
            uint32_t cp = 0;
            const size_t n = utf8_at(ln, i, &cp);
            if (n == 0) { failed = true; return; }  // not UTF-8: tobj's lines() fails with ReadError
            if (is_ws(cp)) {
                if (in_word) w.push_back(ln.substr(s, i - s));
                in_word = false;
            } else if (!in_word) {
                in_word = true;
                s = i;
            }
            i += n;
        }
        if (in_word) w.push_back(ln.substr(s));
        if (w.empty()) return;
        const std::string& key = w[0];
        if (key == "v") {
            if (w.size() < 4) { failed = true; return; }  // PositionParseError
            float xyz[3];
            for (int k = 0; k < 3; k++)
                if (!parse_f32(w[1 + k], &xyz[k])) { failed = true; return; }
            pos.insert(pos.end(), xyz, xyz + 3);
        } else if (key == "f" || key == "l" || key == "p") {
            std::vector<long> corners;
            for (size_t k = 1; k < w.size(); k++) {
                std::string vtx = w[k];
                size_t slash = vtx.find('/');
                std::string vs = slash == std::string::npos ? vtx : vtx.substr(0, slash);
                long idx;
                if (!parse_index(vs, pos.size() / 3, &idx) || idx < 0) { failed = true; return; }  // FaceParseError
                corners.push_back(idx);
            }
            if (corners.empty()) { failed = true; return; }
            faces.push_back(std::move(corners));
        } else if (key == "o" || key == "g") {
            flush_model();
        }
        // vt, vn, s, usemtl, mtllib, comments: no effect on positions / face corners.
    }
};

}  // namespace

Mesh Mesh::load_obj(const char* data, size_t len, const Material& material) {
    Mesh mesh;
    mesh.material = material;
    Parser p;
    size_t start = 0;
    while (start < len && !p.failed) {
        const char* nl = (const char*)std::memchr(data + start, '\n', len - start);
        size_t end = nl ? (size_t)(nl - data) : len;
        p.line(std::string(data + start, end - start));
        start = end + 1;
    }
    if (!p.failed) p.flush_model();
    if (p.failed) return mesh;  // mesh.rs:53-59: Err -> empty mesh
    // mesh.rs:23-47: concatenate models with an index offset; vertex = [x, y, z, 1].
    for (const ObjModel& m : p.models) {
        uint32_t offset = (uint32_t)mesh.vertices.size();
        size_t nv = m.positions.size() / 3;
        for (size_t i = 0; i < nv; i++) {
            Vertex v{};
            v.position[0] = m.positions[3 * i];
            v.position[1] = m.positions[3 * i + 1];
            v.position[2] = m.positions[3 * i + 2];
            v.position[3] = 1.0f;
            v.normal[0] = 0.0f; v.normal[1] = 0.0f; v.normal[2] = 1.0f; v.normal[3] = 1.0f;
            // color 0xffff00ff (mesh.rs:43, vertex.rs:20-31)
            v.color[0] = 1.0f; v.color[1] = 1.0f; v.color[2] = 0.0f; v.color[3] = 1.0f;
            mesh.vertices.push_back(v);
        }
        for (uint32_t i : m.indices) mesh.indices.push_back(offset + i);
    }
    return mesh;
}

}  // namespace hrt
