// renderer.cpp — the rt_* C-ABI: device buffers, frame protocol and kernel launches on one HIP stream.
//
// Replaces the reference's wgpu Renderer (hucancode/hello-raytracing src/renderer.rs): the group0/group1
// bind-group buffers become device allocations owned by the handle, queue.write_buffer becomes a
// copy + layout conversion (AoS reference PODs -> the kernel's layout), and draw() becomes a kernel
// launch. There is no CPU fallback: without a gfx950 device every call that needs one returns
// RT_ERR_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hrt.h"
#include "../../include/hrt_testing.h"
#include "host/scene.hpp"
#include "host/sphere_bvh.hpp"
#include "host/tri_bvh.hpp"
#include "rt_device.hpp"

hipError_t hrt_launch_render(int mode, int variant, const hrt_dev::KParams& P, hipStream_t stream);
hipError_t hrt_launch_accumulate(const hrt_dev::KParams& P, hipStream_t stream);
hipError_t hrt_launch_trace(int mode, int variant, const hrt_dev::KParams& P, hipStream_t stream);
hipError_t hrt_launch_order(uint32_t* pixel_cost, uint32_t ntiles, uint32_t* tile_sum, uint32_t* order, uint32_t* scratch,
                            hipStream_t stream);
uint32_t hrt_order_scratch_words(uint32_t ntiles);
const char* hrt_last_kernel();
void hrt_reset_last_kernel();
hipError_t hrt_check_exact_math(unsigned long long n, uint32_t seed, unsigned long long* out_dev, hipStream_t st);

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(RT_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));    \
    } while (0)

template <typename T>
struct DevBuf {
    T* ptr = nullptr;
    size_t cap = 0;  // elements
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    uint64_t bytes() const { return ptr ? (uint64_t)cap * sizeof(T) : 0u; }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
    }
};

// fail_above: fault injection for tests (rt_testing_set_faults), an allocation above that many bytes
// fails as a refused hipMalloc would (0 = off)
template <typename T>
int ensure(DevBuf<T>& b, size_t n, size_t fail_above = 0) {
    if (n <= b.cap && b.ptr) return RT_OK;
    b.release();
    size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    if (fail_above && bytes > fail_above)
        return fail(RT_ERR_ALLOC, "hipMalloc: injected failure (rt_testing_set_faults)");
    hipError_t e = hipMalloc((void**)&b.ptr, bytes);
    if (e != hipSuccess) {
        b.ptr = nullptr;
        return fail(RT_ERR_ALLOC, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    b.cap = std::max<size_t>(n, 1);
    return RT_OK;
}

// ensure() for the sample queue's colour-fold memory, which must stay within rt_params.queue_budget_mb: a buffer
// left larger by an earlier draw is given back when it exceeds `budget` bytes or twice what this draw needs.
template <typename T>
int ensure_within(DevBuf<T>& b, size_t n, size_t budget, size_t fail_above) {
    if (b.ptr && (b.cap * sizeof(T) > budget || b.cap > 2 * std::max<size_t>(n, 1))) b.release();
    return ensure(b, n, fail_above);
}

// Makes `device` current for one rt_* call and restores the caller's device after it: a renderer's memory, stream
// and launches stay on the GPU it was created on whatever device the calling thread has current (one process
// driving several GPUs, or a caller that switches devices between calls).
struct DeviceScope {
    int prev = -1, rc = RT_OK;
    explicit DeviceScope(int device) {
        int cur = -1;
        if (hipGetDevice(&cur) != hipSuccess) {
            rc = fail(RT_ERR_DEVICE, "hipGetDevice failed");
            return;
        }
        if (cur == device) return;
        if (hipSetDevice(device) != hipSuccess) {
            rc = fail(RT_ERR_DEVICE, "hipSetDevice to the renderer's device failed");
            return;
        }
        prev = cur;
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};

int check_device(int* dev_out) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(RT_ERR_DEVICE, "no HIP device visible (the renderer has no CPU fallback)");
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, dev));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(RT_ERR_DEVICE, std::string("device is ") + prop.gcnArchName + ", this build targets gfx950 only");
    *dev_out = dev;
    return RT_OK;
}

// Rows owned by a renderer: blocks of `block` rows starting at row0, row0 + step*block, ... (block 1: the
// interleaved rows row0, row0 + step, ...); the last block may be cut by the image bottom.
uint32_t local_rows_of(uint32_t H, uint32_t row0, uint32_t step, uint32_t block) {
    if (row0 >= H || step == 0) return 0;
    block = std::max(block, 1u);
    const uint64_t stride = (uint64_t)step * block;
    const uint64_t nblocks = ((uint64_t)H - row0 + stride - 1) / stride;
    const uint64_t last0 = row0 + (nblocks - 1) * stride;  // first row of the last block
    return (uint32_t)((nblocks - 1) * block + std::min<uint64_t>(block, H - last0));
}

}  // namespace

struct rt_renderer {
    int device = 0;
    int mode = RT_MODE_SPHERE;
    uint32_t width = 0, height = 0;
    rt_params params{};
    hrt::Camera camera{};
    bool has_camera = false;
    uint32_t time = 0, frame_count = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;

    DevBuf<float> image;
    DevBuf<float4> sph_geo;
    DevBuf<hrt_dev::SphereAux> sph_aux;
    DevBuf<hrt_dev::SpherePair> sph_pairs;
    uint32_t n_spheres = 0;
    // culling BVH over the sphere slots (SCAN_BVH)
    DevBuf<float4> bvh_nodes, bvh_sph;
    DevBuf<uint4> bvh_hnodes;
    DevBuf<int> bvh_slot, bvh_large;
    hrt::SphereBvh bvh_host;
    DevBuf<float4> nodes;
    DevBuf<float> nodes_so;  // the same nodes as (lo, hi, lo) per axis (pack_nodes_so)
    bool so_ok = false;
    DevBuf<hrt_dev::TriDev> tris;
    DevBuf<float> tri_geo;  // a | e1 | e2 per triangle, 9 floats (the deferred tests' operands; KParams::tri_geo)
    DevBuf<hrt_dev::MatDev> mats;
    uint32_t bvh_n = 0, bvh_m = 0;
    // opt-in SAH triangle tree, built on first use after rt_set_bvh
    std::vector<float> tri_aee;  // a, e1, e2 of every triangle as uploaded
    bool tri_tree_dirty = true;
    hrt::TriBvh tri_tree;
    DevBuf<uint4> tb_hnodes;
    DevBuf<uint32_t> tb_order;
    DevBuf<unsigned long long> counter;
    DevBuf<unsigned long long> count_spread;  // the work counters' CSPREAD copies (rt_kernels.hip flush_counts)
    DevBuf<unsigned long long> steal_slots;  // sample queue: one word per resident wave (frame-block work stealing)
    DevBuf<unsigned long long> queues;       // sample buffer: the per-XCD job counters (rt_kernels.hip queue_take_lane0)
    uint32_t cus = 0;                        // compute units of the renderer's device
    DevBuf<float> samples;      // sample-queue colour buffer (frames x tiles x 64 px x 3), tile-major (ring_mode 0)
    DevBuf<float> samples2;     // the odd launches' buffer when each launch folds the one before (rt_params.fold 3)
    bool last_fold_next = false;
    DevBuf<float4> ring;        // sample-queue fold ring: job slots x job_frames x 64 px (rgb, unused) (ring_mode 1)
    DevBuf<uint32_t> ring_ctl;  // zeroed per launch: tile fold words (2 words per tile), the free queue (4 per
                                // slot) and its tail (4); then the job -> slot map
    // cost-ordered dealing (rt_params.cost_order): per-pixel query counts of a learning launch (zeroed again by the
    // sort), per-tile sums, the tile order built from them, the counting sort's histogram / cursors; cost_tiles: the
    // tile count they were set up for, order_tiles: the tile count tile_order holds a permutation of (0: none yet);
    // cost_learn: the next sample-buffer launch learns (set by every scene, camera, size or parameter change)
    DevBuf<uint32_t> tile_cost, tile_sum, tile_order, order_scratch;
    uint32_t cost_tiles = 0, order_tiles = 0;
    bool cost_learn = true;
    uint32_t last_ordered = 0;  // trace launches of the last sample-queue draw that dealt in cost order
    DevBuf<unsigned long long> wave_trace;  // diagnostic build only
    size_t wave_trace_words = 0;

    // host copy of the spheres (slot arrays are rebuilt when min_sphere_slots changes)
    std::vector<hrt::Sphere> spheres;

    rt_stats stats{};
    bool timing_pending = false;
    int last_variant = 0;
    std::vector<hipEvent_t> ev_trace;  // start/stop pairs around each k_trace launch of the last draw
    uint32_t trace_pairs = 0, trace_pairs_pending = 0;
    uint32_t last_schedule = 0;
    uint32_t last_suspend = 0;
    uint32_t test_ring_slots_max = 0, test_fail_alloc_above_mb = 0;  // hrt_testing.h fault injection
    uint32_t ring_slots = 0;  // fold-ring slots of the last sample-queue draw
    uint32_t ring_tiles = 0, ring_nchunks = 0;  // (diagnostics: HRT_RING_DUMP)
    size_t ring_ctl_words = 0;
    uint64_t fold_bytes = 0;  // device memory of the last sample-queue draw's colour fold (rt_stats.fold_bytes)
    uint32_t last_launch_frames = 0;  // frames per trace launch of the last sample-queue draw (rt_stats.launch_frames)
    unsigned long long raw_counters[RT_RAW_COUNTERS] = {};

    uint32_t row_block() const { return std::max(params.row_block, 1u); }
    uint64_t device_bytes() const {
        return image.bytes() + sph_geo.bytes() + sph_aux.bytes() + sph_pairs.bytes() + bvh_nodes.bytes() + bvh_sph.bytes() +
               bvh_hnodes.bytes() + bvh_slot.bytes() + bvh_large.bytes() + nodes.bytes() + nodes_so.bytes() + tris.bytes() +
               tri_geo.bytes() + mats.bytes() +
               tb_hnodes.bytes() + tb_order.bytes() + counter.bytes() + count_spread.bytes() + samples.bytes() + samples2.bytes() + ring.bytes() + ring_ctl.bytes() +
               wave_trace.bytes() + steal_slots.bytes() + queues.bytes() + tile_cost.bytes() + tile_sum.bytes() + tile_order.bytes() +
               order_scratch.bytes();
    }
    uint32_t local_rows() const { return local_rows_of(height, params.row0, params.row_step, row_block()); }
    size_t image_floats() const { return (size_t)local_rows() * width * 3u; }
};

#ifndef HRT_LNODES
#define HRT_LNODES 1
#endif
// heap-top configuration of k_trace_split_tris when rt_params.heap_lds = 0 (rt_kernels.hip heap_top_n)
#ifndef HRT_HEAP_AUTO
#define HRT_HEAP_AUTO 3u
#endif

namespace {

// The dielectric scatter arm's per-hit divisions, done once per material with the kernels' f32 operations
// (shader_sphere.wgsl:185-199: ir = 1 / params.x on a front face; reflectance's r0 = (1 - ir) / (1 + ir)).
hrt_dev::DielConsts dielectric_consts(float param) {
    auto r0sq = [](float ir) {
        const float r0 = (1.0f - ir) / (1.0f + ir);
        return r0 * r0;
    };
    const float inv = 1.0f / param;
    return hrt_dev::DielConsts{inv, r0sq(inv), r0sq(param)};
}

int zero_image(rt_renderer* r) {
    int rc = ensure(r->image, r->image_floats());
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(r->image.ptr, 0, std::max<size_t>(r->image_floats(), 1) * sizeof(float), r->stream));
    return RT_OK;
}

// Nodes of a two-child BVH as the kernels read them: 4 float4 per node, boxes relative to `center`,
// rounded outward again after the shift.
std::vector<float4> pack_bvh_nodes(const std::vector<hrt::SphereBvhNode>& nodes, const float center[3]) {
    std::vector<float4> out(4 * std::max<size_t>(nodes.size(), 1));
    auto rel_lo = [&](float v, int k) { return std::nextafter((float)((double)v - (double)center[k]), -INFINITY); };
    auto rel_hi = [&](float v, int k) { return std::nextafter((float)((double)v - (double)center[k]), INFINITY); };
    for (size_t j = 0; j < nodes.size(); j++) {
        const hrt::SphereBvhNode& n = nodes[j];
        float4* o = &out[4 * j];
        o[0] = float4{rel_lo(n.lmin[0], 0), rel_lo(n.lmin[1], 1), rel_lo(n.lmin[2], 2), __builtin_bit_cast(float, n.left)};
        o[1] = float4{rel_hi(n.lmax[0], 0), rel_hi(n.lmax[1], 1), rel_hi(n.lmax[2], 2), 0.0f};
        o[2] = float4{rel_lo(n.rmin[0], 0), rel_lo(n.rmin[1], 1), rel_lo(n.rmin[2], 2), __builtin_bit_cast(float, n.right)};
        o[3] = float4{rel_hi(n.rmax[0], 0), rel_hi(n.rmax[1], 1), rel_hi(n.rmax[2], 2), 0.0f};
    }
    return out;
}

// The heap's nodes for the sign-ordered node test (rt_kernels.hip node_hit_so; tests/test_sign_ordered_slab.py):
// (lo, hi, lo) per axis, 9 floats per node, with lo <= hi — an axis with min > max (padding nodes: +MAX / -MAX) is
// swapped, which changes nothing in intersect_node (shader_tris.wgsl:150-159: min / max take the pair in either order).
// A NaN bound leaves its axis as given and clears so_ok (the kernels then use the reference form on this layout).
std::vector<float> pack_nodes_so(const float* nodes, uint32_t n, bool& so_ok) {
    std::vector<float> out(9 * (size_t)std::max<uint32_t>(n, 1), 0.0f);
    so_ok = true;
    for (uint32_t i = 0; i < n; i++) {
        for (int k = 0; k < 3; k++) {
            float lo = nodes[8 * (size_t)i + k], hi = nodes[8 * (size_t)i + 4 + k];
            if (std::isnan(lo) || std::isnan(hi)) so_ok = false;
            else if (lo > hi) std::swap(lo, hi);
            out[9 * (size_t)i + 3 * k] = lo;
            out[9 * (size_t)i + 3 * k + 1] = hi;
            out[9 * (size_t)i + 3 * k + 2] = lo;
        }
    }
    return out;
}

// The culling BVH's nodes with fp16 boxes (k_trace_split): 32 B per node instead of 64 — per child the
// box relative to `center` as six halves rounded outward (min down, max up: containment holds, so the walk
// stays exact; the boxes only grow by at most one half ulp), then the child word:
//   (min.x | min.y << 16, min.z | max.x << 16, max.y | max.z << 16, left word), the same for the right.
uint16_t f16_bits(_Float16 h) { return __builtin_bit_cast(uint16_t, h); }
_Float16 f16_from_bits(uint16_t b) { return __builtin_bit_cast(_Float16, b); }
_Float16 f16_step(_Float16 h, bool up) {
    uint16_t b = f16_bits(h);
    if ((b & 0x7FFFu) == 0u) return f16_from_bits(up ? 0x0001u : 0x8001u);  // +-0 -> smallest subnormal
    const bool neg = (b & 0x8000u) != 0u;
    b = (uint16_t)((up != neg) ? b + 1u : b - 1u);
    return f16_from_bits(b);
}
uint32_t f16_dir(float x, bool up) {
    _Float16 h = (_Float16)x;
    if (up ? (float)h < x : (float)h > x) h = f16_step(h, up);
    return f16_bits(h);
}
std::vector<uint4> pack_bvh_hnodes(const std::vector<hrt::SphereBvhNode>& nodes, const float center[3]) {
    std::vector<uint4> out(2 * std::max<size_t>(nodes.size(), 1), uint4{0u, 0u, 0u, 0u});
    auto rel = [&](float v, int k, bool up) {
        const float f = std::nextafter((float)((double)v - (double)center[k]), up ? INFINITY : -INFINITY);
        return f16_dir(f, up);
    };
    for (size_t j = 0; j < nodes.size(); j++) {
        const hrt::SphereBvhNode& n = nodes[j];
        const float* mn[2] = {n.lmin, n.rmin};
        const float* mx[2] = {n.lmax, n.rmax};
        const uint32_t w[2] = {n.left, n.right};
        for (int c = 0; c < 2; c++) {
            // per axis one [min | max] pair of halves (k_trace_split rotates a pair to [near | far]: box_hit_so)
            out[2 * j + c] = uint4{rel(mn[c][0], 0, false) | rel(mx[c][0], 0, true) << 16,
                                   rel(mn[c][1], 1, false) | rel(mx[c][1], 1, true) << 16,
                                   rel(mn[c][2], 2, false) | rel(mx[c][2], 2, true) << 16, w[c]};
        }
    }
    return out;
}

int upload_tri_tree(rt_renderer* r) {
    if (!r->tri_tree_dirty) return RT_OK;
    r->tri_tree = hrt::build_tri_bvh(r->tri_aee);
    const std::vector<uint4> hpacked = pack_bvh_hnodes(r->tri_tree.nodes, r->tri_tree.root_center);
    int rc = ensure(r->tb_hnodes, hpacked.size());
    if (!rc) rc = ensure(r->tb_order, std::max<size_t>(r->tri_tree.order.size(), 1));
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(r->tb_hnodes.ptr, hpacked.data(), hpacked.size() * sizeof(uint4), hipMemcpyHostToDevice,
                           r->stream));
    if (!r->tri_tree.order.empty())
        HIP_TRY(hipMemcpyAsync(r->tb_order.ptr, r->tri_tree.order.data(), r->tri_tree.order.size() * sizeof(uint32_t),
                               hipMemcpyHostToDevice, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    r->tri_tree_dirty = false;
    return RT_OK;
}

int upload_spheres(rt_renderer* r) {
    const uint32_t nslots = std::max<uint32_t>((uint32_t)r->spheres.size(), r->params.min_sphere_slots);
    std::vector<float4> geo(nslots, float4{0.0f, 0.0f, 0.0f, 0.0f});
    std::vector<hrt_dev::SphereAux> aux(nslots);
    std::memset(aux.data(), 0, aux.size() * sizeof(aux[0]));
    for (uint32_t i = (uint32_t)r->spheres.size(); i < nslots; i++) {  // zero slots: params 0, id 0 (default arm)
        const hrt_dev::DielConsts dc = dielectric_consts(0.0f);
        aux[i].inv_param = dc.inv_param;
        aux[i].r0sq_front = dc.r0sq_front;
        aux[i].r0sq_back = dc.r0sq_back;
    }
    for (size_t i = 0; i < r->spheres.size(); i++) {
        const hrt::Sphere& s = r->spheres[i];
        const float rr = s.radius * s.radius;  // radius*radius, shader_sphere.wgsl:142
        geo[i] = float4{s.center.x, s.center.y, s.center.z, rr};
        const hrt_dev::DielConsts dc = dielectric_consts(s.material.params.x);
        const bool rad_ok = std::fabs(s.radius) >= 0x1p-60f && std::fabs(s.radius) <= 0x1p60f;
        aux[i] = hrt_dev::SphereAux{s.center.x, s.center.y, s.center.z, s.radius,
                                    s.material.albedo.x, s.material.albedo.y, s.material.albedo.z,
                                    s.material.params.x, s.material.kind, dc.inv_param, dc.r0sq_front, dc.r0sq_back,
                                    rad_ok ? 1.0f / s.radius : 0.0f, 0.0f, 0.0f, 0.0f};
    }
    // slot pairs for the packed scan; an odd tail slot is paired with a NaN-centre slot (never accepted)
    const uint32_t npairs = (nslots + 1) / 2;
    const float qnan = std::nanf("");
    std::vector<hrt_dev::SpherePair> pairs(npairs);
    for (uint32_t p = 0; p < npairs; p++) {
        for (int k = 0; k < 2; k++) {
            const uint32_t i = 2 * p + (uint32_t)k;
            const float4 g = i < nslots ? geo[i] : float4{qnan, qnan, qnan, 0.0f};
            pairs[p].cx[k] = g.x;
            pairs[p].cy[k] = g.y;
            pairs[p].cz[k] = g.z;
            pairs[p].rr[k] = g.w;
        }
    }
    // culling BVH: boxes stored relative to the root centre (rounded outward again after the shift)
    std::vector<float> cr(4 * (size_t)nslots);
    for (uint32_t i = 0; i < nslots; i++) {
        const bool real = i < r->spheres.size();
        cr[4 * i + 0] = geo[i].x;
        cr[4 * i + 1] = geo[i].y;
        cr[4 * i + 2] = geo[i].z;
        cr[4 * i + 3] = real ? r->spheres[i].radius : 0.0f;
    }
    r->bvh_host = hrt::build_sphere_bvh(cr);
    const hrt::SphereBvh& B = r->bvh_host;
    const std::vector<float4> bnodes = pack_bvh_nodes(B.nodes, B.root_center);
    const std::vector<uint4> hnodes = pack_bvh_hnodes(B.nodes, B.root_center);
    const size_t nleaf = B.slot.size();
    int rc = ensure(r->sph_geo, nslots);
    if (!rc) rc = ensure(r->sph_aux, nslots);
    if (!rc) rc = ensure(r->sph_pairs, npairs);
    if (!rc) rc = ensure(r->bvh_nodes, bnodes.size());
    if (!rc) rc = ensure(r->bvh_hnodes, hnodes.size());
    if (!rc) rc = ensure(r->bvh_sph, std::max<size_t>(nleaf, 1));
    if (!rc) rc = ensure(r->bvh_slot, std::max<size_t>(nleaf, 1));
    if (!rc) rc = ensure(r->bvh_large, std::max<size_t>(B.large.size(), 1));
    if (rc) return rc;
    if (nslots) {
        HIP_TRY(hipMemcpyAsync(r->sph_geo.ptr, geo.data(), nslots * sizeof(float4), hipMemcpyHostToDevice, r->stream));
        HIP_TRY(hipMemcpyAsync(r->sph_aux.ptr, aux.data(), nslots * sizeof(aux[0]), hipMemcpyHostToDevice, r->stream));
        HIP_TRY(hipMemcpyAsync(r->sph_pairs.ptr, pairs.data(), npairs * sizeof(pairs[0]), hipMemcpyHostToDevice,
                               r->stream));
        HIP_TRY(hipMemcpyAsync(r->bvh_nodes.ptr, bnodes.data(), bnodes.size() * sizeof(float4),
                               hipMemcpyHostToDevice, r->stream));
        HIP_TRY(hipMemcpyAsync(r->bvh_hnodes.ptr, hnodes.data(), hnodes.size() * sizeof(uint4),
                               hipMemcpyHostToDevice, r->stream));
        if (nleaf) {
            HIP_TRY(hipMemcpyAsync(r->bvh_sph.ptr, B.sph.data(), nleaf * sizeof(float4), hipMemcpyHostToDevice,
                                   r->stream));
            HIP_TRY(hipMemcpyAsync(r->bvh_slot.ptr, B.slot.data(), nleaf * sizeof(int), hipMemcpyHostToDevice,
                                   r->stream));
        }
        if (!B.large.empty())
            HIP_TRY(hipMemcpyAsync(r->bvh_large.ptr, B.large.data(), B.large.size() * sizeof(int),
                                   hipMemcpyHostToDevice, r->stream));
        HIP_TRY(hipStreamSynchronize(r->stream));  // host staging vectors die here
    }
    r->n_spheres = nslots;
    return RT_OK;
}

// Event pairs for `pairs + 1` k_trace launches (created on demand, kept for the renderer's life).
int trace_events(rt_renderer* r, uint32_t pair) {
    while (r->ev_trace.size() < 2u * (pair + 1u)) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        r->ev_trace.push_back(e);
    }
    return RT_OK;
}

// schedule 0 = the sample queue (load-balanced at sample granularity), except for
// draws too small to fill the persistent grid for long (< 1.5 Mi samples: e.g. a 512x512 interactive
// frame, C1), where the tiles kernel's single launch has less fixed cost. Measured per step (ms, tiles vs
// queue): C1 0.13 vs 0.16; 512x512 x1 0.22 vs 0.29; C2 x2 frames (1.8 M) 0.54 vs 0.50; one 1080p frame
// of C3 (2.1 M) 1.55 vs 1.33.
uint32_t resolve_schedule(const rt_renderer* r, uint32_t count) {
    if (r->params.schedule) return r->params.schedule;
    const uint64_t samples = (uint64_t)count * r->local_rows() * r->width;
    return samples < (3ull << 19) ? RT_SCHEDULE_TILES : RT_SCHEDULE_QUEUE;
}

// variant 0 = the fastest exact scan measured for the slot count: the culling BVH from 32 slots up, the
// deferred packed scan from 9, the simple scan below (C2, 4 slots: 50.8 vs 48.0 Grays/s deferred).
int resolve_variant(const rt_renderer* r) {
    if (r->params.variant) return (int)r->params.variant;
    if (r->n_spheres >= 32) return hrt_dev::SCAN_BVH;
    return r->n_spheres > 8 ? hrt_dev::SCAN_DEFER : hrt_dev::SCAN_SIMPLE;
}

int launch_frames(rt_renderer* r, uint32_t count, uint32_t time0, uint32_t dtime) {
    if (!r->has_camera) return fail(RT_ERR_STATE, "rt_set_camera must be called before drawing");
    if (r->mode == RT_MODE_SPHERE && r->sph_geo.ptr == nullptr) {
        int rc = upload_spheres(r);  // empty scene: min_sphere_slots zero slots, like an unwritten buffer
        if (rc) return rc;
    }
    // RT_RAW_COUNTERS exported words, then the sample queue's fold-ring watchdog (rt_kernels.hip idle_spin)
    int rc = ensure(r->counter, hrt_dev::COUNTER_WORDS);
    if (!rc) rc = ensure(r->count_spread, (size_t)hrt_dev::CSPREAD * hrt_dev::CSTRIDE);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(r->counter.ptr, 0, hrt_dev::COUNTER_WORDS * sizeof(unsigned long long), r->stream));
    HIP_TRY(hipMemsetAsync(r->count_spread.ptr, 0, (size_t)hrt_dev::CSPREAD * hrt_dev::CSTRIDE * sizeof(unsigned long long),
                           r->stream));

    hrt_dev::KParams P{};
    {
        hrt_dev::CamDev& cd = P.cam;
        const hrt::Camera& c = r->camera;
        const float* cam = &c.eye.x;
        for (int i = 0; i < 4; i++) {
            cd.eye[i] = cam[i];
            cd.dir[i] = cam[4 + i];
            cd.up[i] = cam[8 + i];
            cd.right[i] = cam[12 + i];
        }
        cd.focal = c.params.x;
        cd.blur = c.params.y;
        cd.k = std::tan(c.params.z * 0.5f);  // tan(camera.fov*0.5), make_ray :124 (libm tanf, as the oracle)
        cd.aspect = (float)r->width / (float)r->height;
        cd.wm1 = (float)r->width - 1.0f;
        cd.hm1 = (float)r->height - 1.0f;
        // for the fast exact divisions of make_ray's px / wm1, py / hm1 (div_rn_mid's operand range)
        const auto inv_in_range = [](float l) { return l >= 0x1p-60f && l <= 0x1p60f ? 1.0f / l : 0.0f; };
        cd.inv_wm1 = inv_in_range(cd.wm1);
        cd.inv_hm1 = inv_in_range(cd.hm1);
        cd.H = r->height;
    }
    P.W = r->width;
    P.H = r->height;
    P.dtime = dtime;
    P.bounces = r->params.bounces;
    P.ema_cap = (float)r->params.ema_cap;
    P.nslots = r->mode == RT_MODE_TRIS ? 0u : r->n_spheres;
    P.npairs = (P.nslots + 1) / 2;
    P.sph_pairs = r->sph_pairs.ptr;
    P.n = r->mode == RT_MODE_SPHERE ? 0u : r->bvh_n;
    P.m = r->mode == RT_MODE_SPHERE ? 0u : r->bvh_m;
    P.row0 = r->params.row0;
    P.row_step = r->params.row_step;
    P.row_block = r->row_block();
    P.row_stride = r->params.row_step * P.row_block;
    P.nrows = r->local_rows();
    P.image = r->image.ptr;
    P.sph_geo = r->sph_geo.ptr;
    P.sph_aux = r->sph_aux.ptr;
    P.nodes = r->nodes.ptr;
    P.nodes_so = r->nodes_so.ptr;
    P.so_ok = r->so_ok ? 1u : 0u;
    P.count_tests = r->params.count_tests;
    P.tris = r->tris.ptr;
    P.tri_geo = r->tri_geo.ptr;
    P.tri_bvh = (r->mode != RT_MODE_SPHERE && r->params.tri_bvh) ? 1u : 0u;
    if (P.tri_bvh) {
        rc = upload_tri_tree(r);
        if (rc) return rc;
        P.tb_hnodes = r->tb_hnodes.ptr;
        P.tb_rr_h = std::nextafter(r->tri_tree.root_radius * (1.0f + 0x1p-9f), INFINITY);
        P.tb_order = r->tb_order.ptr;
        P.tb_root = r->tri_tree.root_word;
        for (int k = 0; k < 3; k++) P.tb_rc[k] = r->tri_tree.root_center[k];
        P.tb_rr = r->tri_tree.root_radius;
    }
    P.mats = r->mats.ptr;
    P.counter = r->counter.ptr;
    P.count_spread = r->count_spread.ptr;
#ifdef HRT_STAMPS
    {
        // k_render's waves, or the persistent kernels' (at most steal_cap = 32 per CU)
        const size_t wave_words = 8ull * std::max<size_t>((size_t)((r->width + 15u) / 16u) * ((P.nrows + 15u) / 16u) * 4u,
                                                          32ull * std::max(r->cus, 1u));
        const size_t words = wave_words + (1ull << 21);  // + one word per job (k_trace's job_trace)
        int rc2 = ensure(r->wave_trace, words);
        if (rc2) return rc2;
        HIP_TRY(hipMemsetAsync(r->wave_trace.ptr, 0, words * sizeof(unsigned long long), r->stream));
        r->wave_trace_words = words;
        P.wave_trace = r->wave_trace.ptr;
        P.job_trace = r->wave_trace.ptr + wave_words;
    }
#endif
    const hrt::SphereBvh& B = r->bvh_host;
    P.bvh_nodes = r->bvh_nodes.ptr;
    P.bvh_sph = r->bvh_sph.ptr;
    P.bvh_slot = r->bvh_slot.ptr;
    P.large_slots = r->bvh_large.ptr;
    P.nlarge = (uint32_t)B.large.size();
    P.bvh_nleaf = (uint32_t)B.slot.size();
    P.bvh_root = B.root_word;
    for (int k = 0; k < 3; k++) P.bvh_rc[k] = B.root_center[k];
    P.bvh_rr = B.root_radius;
    P.bvh_hnodes = r->bvh_hnodes.ptr;
    // fp16 boxes reach up to one half ulp (2^-11 relative) past the f32 root box
    P.bvh_rr_h = std::nextafter(B.root_radius * (1.0f + 0x1p-9f), INFINITY);
    P.bvh_nnodes = (uint32_t)B.nodes.size();
    P.bvh_lnodes = (HRT_LNODES && B.nodes.size() <= hrt_dev::LNODE_CAP && B.depth <= hrt_dev::LNODE_DEPTH) ? 1u : 0u;
    // (0 auto = off: the packet walk measured -8 % on C3)
    P.packet = (P.bvh_lnodes && r->params.packet == 2u) ? 1u : 0u;
    // delta = 8u r_max + min(16u D^2 / r_min, 2e-3 D) + 4u D + 4e-23/|d|  (u = 2^-24)
    const float u = 0x1p-24f;
    P.pad_k1 = 8.0f * u * B.r_max;
    P.pad_k2 = B.r_min > 0.0f ? 16.0f * u / B.r_min : INFINITY;
    P.pad_k3 = 2e-3f;
    P.pad_k4 = 4.0f * u;
    const int variant = r->mode == RT_MODE_TRIS ? hrt_dev::SCAN_SIMPLE : resolve_variant(r);
    const uint32_t schedule = resolve_schedule(r, count);
    r->last_variant = variant;
    r->last_schedule = schedule;
    r->last_suspend = 0;

    uint32_t launches = 0, ordered = 0;
    hrt_reset_last_kernel();  // (a draw that launches nothing reports no kernel)
    if (P.nrows == 0u) {  // a renderer that owns no rows (row0 at or below the last row): nothing to trace
        r->trace_pairs = 0;
        HIP_TRY(hipEventRecord(r->ev_start, r->stream));
    } else if (schedule == RT_SCHEDULE_QUEUE) {
        r->trace_pairs_pending = 0;
        P.tiles_w = (r->width + 7u) / 8u;
        P.tiles_h = (P.nrows + 7u) / 8u;
        const uint32_t ntiles = P.tiles_w * P.tiles_h;
        // suspendable walks (k_trace_split / k_trace_split_tris): the sphere program's culling BVH, the heap walk
        // of the triangle / mixed programs; not the opt-in SAH walk
        const bool split = !P.tri_bvh && (r->mode != RT_MODE_SPHERE || variant == hrt_dev::SCAN_BVH);
        // k_trace_split_tris<.., HL > 0> (heap top in LDS, 8 leaf-pair list words per lane): the mixed program's
        // sphere walk (culling BVH, begin phase) fits an 8-entry stack (a path holds at most depth pending siblings;
        // deeper trees would only fall back to the exact full scan, but keep the 16-entry kernel for them)
        // (and heaps of at most 2^24 nodes: node_hit_so addresses node i with a 24-bit multiply-add)
        P.tri_small = 0u;
        if (r->mode != RT_MODE_SPHERE &&
            (r->mode == RT_MODE_TRIS || variant != hrt_dev::SCAN_BVH || r->bvh_host.depth <= 8u) && r->params.heap_lds != 1u &&
            r->bvh_n <= (1u << 24))
            P.tri_small = HRT_HEAP_AUTO;
        if (variant == hrt_dev::SCAN_DEFER && r->mode == RT_MODE_MIXED && P.tri_small > 1u) P.tri_small = 1u;
        // job_frames 0 = per kernel: 32 for the suspendable walks (C3 +0.7 %, C4 +1.5 % over 16), 16 for k_trace's
        // cheap sphere scans (C2: 32 costs 3 %); a power of two (the ring's slot layout)
        uint32_t jf = r->params.job_frames ? r->params.job_frames : (split ? 32u : 16u);
        P.jf_log2 = 0;
        while ((2u << P.jf_log2) <= std::min(jf, 1024u)) P.jf_log2++;
        jf = 1u << P.jf_log2;
        // How the colours are folded (rt_params.queue_budget_mb, fold): the sample buffer (every colour
        // of a launch, then k_accumulate) in launches of equal frame counts, or the bounded-memory fold ring.
        //   queue_budget_mb 0 (auto, the default): floor(count / 320) launches (at least one) of whole jobs. A launch of
        //     320+ frames loses ~2 % to one launch of every frame (C3 3 x 342 frames: 33.8 vs 34.5 Grays/s), shorter ones
        //     lose more (fewer jobs per tile spread the waves over more of the image; C3 at 82 / 164 frames 29.3 / 31.5,
        //     C4 in launches of 345 + 167 frames -13 %), so the buffer holds at most ~640 frames (C3: 8.8 GB, not 25.5),
        //     or every frame that fits AUTO_FIT if that is more, and at most AUTO_BUDGET;
        //   queue_budget_mb > 0: a cap in MiB, launches of as many frames as it holds, balanced;
        //   the fold ring (fold 0) when a launch would get fewer than min(count, 320) frames.
        // (Pipelined launches of tile-row bands x every frame, which keep every frame of a tile in one launch within a
        // bounded buffer, measured bit-identical but slower than these launches at the same budget: C3 tie, C4 -13 %,
        // C5 -19 %; profiles/r04/band/.)
        constexpr size_t AUTO_BUDGET = 32768ull << 20, AUTO_FIT = 8192ull << 20;
        const size_t frame_floats = (size_t)ntiles * 64u * 3u;  // tile-padded
        const size_t frame_bytes = frame_floats * 4u;
        const uint32_t nframes_all = std::max(count, 1u);
        size_t budget = (size_t)r->params.queue_budget_mb << 20;
        // equal launches of at most `fit` frames, rounded up to whole jobs where that still fits: every launch but the
        // last then holds whole jobs, so the tail split applies (C3: 352 + 352 + 320 frames, not 3 x 342)
        auto balanced = [&](size_t fit) {
            fit = std::max<size_t>(1, std::min<size_t>(fit, nframes_all));
            const size_t n = (nframes_all + fit - 1u) / fit;
            const size_t c = (nframes_all + n - 1u) / n, cj = (c + jf - 1u) / jf * jf;
            return (uint32_t)(cj <= fit ? cj : c);
        };
        if (r->params.queue_budget_mb == 0u) {
            // the 320-frame rule, or as many frames as AUTO_FIT holds when that is more (a renderer with few rows —
            // a rank of a multi-GPU render, C3 / 8 = 3.2 GB — draws in one launch, without the extra drains)
            const uint32_t n = std::max(1u, nframes_all / 320u);
            const size_t c = (nframes_all + n - 1u) / n, cj = (c + jf - 1u) / jf * jf;
            const size_t frames =
                std::max(std::min<size_t>(cj, nframes_all), std::min<size_t>(AUTO_FIT / frame_bytes, nframes_all));
            budget = std::min(AUTO_BUDGET, frames * frame_bytes);
        }
        uint32_t chunk = balanced(budget / frame_bytes), log2s = 0;
        P.ring_mode = chunk < std::min(nframes_all, 320u) ? 1u : 0u;
        if (r->params.fold == RT_FOLD_BUFFER || r->params.fold == RT_FOLD_NEXT) P.ring_mode = 0u;  // forced (measurements, tests)
        if (r->params.fold == RT_FOLD_RING) P.ring_mode = 1u;
        const size_t fail_above = (size_t)r->test_fail_alloc_above_mb << 20;
        size_t zero_words = 0;
        if (!P.ring_mode) {
            r->ring.release();  // the other fold's memory: the draw's colour memory stays within the budget
            r->ring_ctl.release();
            // a device short of memory gets smaller launches, down to one frame, instead of a failed draw
            const size_t buf_budget = std::max(budget, frame_bytes);
            while ((rc = ensure_within(r->samples, (size_t)chunk * frame_floats, buf_budget, fail_above)) == RT_ERR_ALLOC &&
                   chunk > 1u) {
                (void)hipGetLastError();  // clear the failed hipMalloc's sticky status
                chunk = (chunk + 1u) / 2u;
            }
            if (rc) return rc;
            P.samples = r->samples.ptr;
            r->ring_slots = 0;
            r->fold_bytes = (uint64_t)chunk * frame_bytes;
        } else {
            r->samples.release();
            // frames per launch: at most FOLD_MAX_JOBS jobs per tile (the done bits of the tile's fold word)
            chunk = std::max(1u, std::min(count, hrt_dev::FOLD_MAX_JOBS * jf));
            const uint32_t nchunks_max = (chunk + jf - 1u) / jf;
            // a power-of-two number of job slots (jf x 64 px x 16 B each) in the budget, at most one per job of a
            // launch; a device short of memory gets a halved budget instead of a failed draw
            budget = std::min<size_t>(budget, 2047ull << 20);
            const uint64_t jobs = (uint64_t)ntiles * nchunks_max;
            for (;;) {
                const size_t fit = std::max<size_t>(1, budget / ((size_t)jf << 10));
                log2s = 0;
                while ((2ull << log2s) <= fit && (1ull << log2s) < jobs && log2s < 20u) log2s++;
                // rt_testing_set_faults caps the slots (tests: jobs then wait in the free queue for a slot)
                while (r->test_ring_slots_max && log2s > 0 && (1ull << log2s) > r->test_ring_slots_max) log2s--;
                zero_words = 2ull * ntiles + (4ull << log2s) + 4u;
                const size_t ring_floats4 = ((size_t)jf << log2s) * 64u;
                rc = ensure_within(r->ring, ring_floats4, std::max(budget, ring_floats4 * 16u), fail_above);
                const size_t ctl_words = zero_words + (size_t)ntiles * nchunks_max;
                if (!rc) rc = ensure_within(r->ring_ctl, ctl_words, ctl_words * 4u, fail_above);
                if (rc != RT_ERR_ALLOC || budget <= ((size_t)jf << 10)) break;
                (void)hipGetLastError();
                r->ring.release();  // retry both with half the budget
                r->ring_ctl.release();
                budget /= 2u;
            }
            if (rc) return rc;
            P.ring = r->ring.ptr;
            P.ring_log2 = log2s;
            P.ring_bytes = (uint32_t)(((size_t)jf << log2s) * 1024u);
            P.tile_fold = (unsigned long long*)r->ring_ctl.ptr;
            P.ring_q = r->ring_ctl.ptr + 2ull * ntiles;
            P.ring_tail = P.ring_q + (4u << log2s);
            P.job_slot = r->ring_ctl.ptr + zero_words;
            r->ring_slots = 1u << log2s;
            r->ring_tiles = ntiles;
            r->ring_ctl_words = zero_words + (size_t)ntiles * nchunks_max;
            r->fold_bytes = (uint64_t)P.ring_bytes + 4ull * (4u * r->ring_slots + 4u) + 4ull * r->ring_ctl_words -
                            4ull * zero_words + 8ull * ntiles;
        }
        // frame-block work stealing (rt_kernels.hip steal_block): the suspendable-walk kernels with the sample
        // buffer; one slot per resident wave, at most 32 waves per CU
        P.steal_cap = 32u * std::max(r->cus, 1u);
        rc = ensure(r->steal_slots, P.steal_cap);
        if (rc) return rc;
        P.steal_slots = r->steal_slots.ptr;
        // Cost-ordered dealing (rt_params.cost_order; rt_kernels.hip k_order_*): a learning launch counts its samples'
        // queries per pixel and the tiles are split into the most expensive half, sorted by cost, and the rest in
        // raster order; the following launches (of this draw and the next ones) deal that head first, so the jobs that
        // take longest start early instead of trailing the launch. The renderer learns in its first ordered launch after
        // any scene, camera, size, row, bounce-cap, slot or triangle-walk change (cost_order 3: in every launch).
        // Auto: a rank's share of a row partition (row_step > 1), which then does not steal, and the suspendable-walk
        // kernels' full images — measured (profiles/r05/t/, u/, y/): 8-way splits C3 0.940 -> 0.96, C5 0.974 -> 0.987,
        // C2 0.52 -> 0.66 and C4 0.755 -> 0.84 with the short-launch job size below; full images C3 +0.6 %, C5 +0.3 %,
        // C4 flat, C2 (k_trace, not ordered) -1.5 %. Bit-identical in any order.
        const bool order_any = !P.ring_mode && r->params.cost_order != 1u;
        // (full images too for the suspendable-walk kernels: C3 38.29 -> 38.53 Grays/s, C5 +0.3 %, C4 flat; not for
        // k_trace's full images: C2 -1.5 %; profiles/r05/y/)
        const bool want_order = order_any && (r->params.cost_order >= 2u || r->params.row_step > 1u || split);
        // Short launches (a rank's share of a row partition, small images): fewer than 32 jobs per resident wave at the
        // kernel's job size. Their jobs are halved (job_frames 0 only), so a job on a costly tile no longer outlasts the
        // launch: C4's 8-way shares in cost order 0.43 with 32-frame jobs, 0.82 with 16; C2's shares 1.00 ms with 8-frame
        // jobs against 1.16 with 16, C3's flat (profiles/r05/r/, t/). Long launches keep the larger jobs (C2 full image
        // -2.6 % with 8, C4 -1.2 % with 16).
        if (!P.ring_mode && r->params.job_frames == 0u && jf > 1u &&
            (uint64_t)ntiles * ((chunk + jf - 1u) / jf) < 32ull * 24u * std::max(r->cus, 1u)) {
            jf >>= 1;
            P.jf_log2--;
        }
        P.queue = r->counter.ptr + 15u;
        // the sample buffer's jobs from one counter per XCD (HRT_NQ 0: the single counter)
#ifndef HRT_NQ
#define HRT_NQ 1
#endif
        constexpr size_t QWORDS = (size_t)hrt_dev::NQ * hrt_dev::QSTRIDE;
        P.queues = nullptr;
        if (!P.ring_mode) {  // (+ the fold counter, below)
            rc = ensure(r->queues, QWORDS + hrt_dev::QSTRIDE);
            if (rc) return rc;
        }
        // Each launch folds the one before (rt_params.fold 3; rt_kernels.hip fold_prev_tiles): two sample buffers, launch
        // k writes buffer k % 2 while every FOLD_WAVE_MOD-th wave first folds buffer (k - 1) % 2 into the image;
        // k_accumulate folds the last launch only. The suspendable-walk kernels, draws of two or more launches; auto with
        // the automatic colour budget (it doubles the colour memory: C3 17.5 GB). C3 38.38 -> 38.76-38.83 Grays/s with 1 in
        // 32 / 64 / 128 waves folding, 38.62-38.65 with 1 in 16, 38.30-38.44 with 1 in 1 or 4; C5 +0.2 %
        // (profiles/r06/fold_next/).
#ifndef HRT_FOLD_WAVE_MOD
#define HRT_FOLD_WAVE_MOD 64
#endif
        constexpr uint32_t FOLD_WAVE_MOD = HRT_FOLD_WAVE_MOD;
        bool fold_next = !P.ring_mode && split && count > chunk &&
                         (r->params.fold == RT_FOLD_NEXT || (r->params.fold == RT_FOLD_AUTO && r->params.queue_budget_mb == 0u));
        if (fold_next) {
            rc = ensure_within(r->samples2, (size_t)chunk * frame_floats, std::max(budget, frame_bytes), fail_above);
            if (rc == RT_ERR_ALLOC) {
                (void)hipGetLastError();
                fold_next = false;
            } else if (rc) {
                return rc;
            }
        }
        if (!fold_next) r->samples2.release();
        else r->fold_bytes *= 2u;
        r->last_fold_next = fold_next;
        // (suspend_below 0: the same kernels with a threshold no wave reaches, 1 walking lane: no suspension)
        P.suspend_below = split ? std::max(r->params.suspend_below, 1u) : 0u;
        r->last_suspend = split ? r->params.suspend_below : 0u;
        P.job_frames = jf;
        HIP_TRY(hipEventRecord(r->ev_start, r->stream));
        P.fold_prev = nullptr;
        for (uint32_t done = 0, k = 0; done < count; done += chunk, k++) {
            if (fold_next) {
                P.samples = (k & 1u) ? r->samples2.ptr : r->samples.ptr;
                if (k > 0u) {  // the launch before: its buffer, frames and first frame
                    P.fold_prev = (k & 1u) ? r->samples.ptr : r->samples2.ptr;
                    P.fold_nframes = P.nframes;
                    P.fold_frame0 = P.frame0;
                    P.fold_next = (uint32_t*)(r->queues.ptr + QWORDS);
                    P.fold_mod = FOLD_WAVE_MOD;
                    HIP_TRY(hipMemsetAsync(P.fold_next, 0, sizeof(uint32_t), r->stream));
                }
            }
            P.nframes = std::min(chunk, count - done);
            P.time0 = time0 + done * dtime;
            P.frame0 = r->frame_count + done;
            P.nchunks = (P.nframes + P.job_frames - 1u) / P.job_frames;
            P.njobs = (unsigned long long)ntiles * P.nchunks;
            // Auto stealing: on for launches with fewer than 16 jobs per resident wave (about 24 per CU), where a job
            // dealt late can outlast the launch (C4's 8-way split: 0.47 -> 0.71 of the full image's rate); off for
            // long launches, where the claims cost 2-4 % and there is no tail to win back (C3: 8-way split 0.90 ->
            // 0.88)
            {
                const bool fits = ntiles < (1u << 25) - 1u && P.nchunks < 2048u;  // the slot's tile and chunk fields
                // (not once the launch can deal in cost order: C4's 8-way shares 0.755 with stealing, 0.82 in order)
                const bool want = r->params.steal == 2u ||
                                  (r->params.steal == 0u && P.njobs < 16ull * 24u * std::max(r->cus, 1u) &&
                                   !(want_order && r->order_tiles == ntiles));
                // (k_trace's frame-block refill for the linear sphere scan with the same stealing ran 3x slower, C2 80 ->
                // 26 Grays/s: a claim per 64 cheap samples stalls the wave; profiles/r05/o/)
                P.steal = (split && !P.ring_mode && fits && want) ? 1u : 0u;
            }
            // Tail split (the suspendable-walk kernels with the sample buffer, no stealing): the last ~2 jobs per
            // resident wave are dealt in parts (rt_params.tail_split: 2 quarters, 3 eighths; 0 auto = quarters),
            // so the launch's drain waits for a part, not a whole job (job_frames a multiple of the part count and
            // whole chunks only; tail_split 1 turns it off)
            P.tail_from = 0xFFFFFFFFu;
            P.tail_shift = r->params.tail_split == 3u ? 3u : 2u;
            // (k_trace's frame-block refill could decode them too, without spills: C2's full image ran 9 % slower with the
            // parts, 74.1 vs 81.3 Grays/s, for its 8-way split 0.51 -> 0.55; round 5, profiles/r05/f/)
            if (split && P.suspend_below > 0u && !P.ring_mode && !P.steal && P.job_frames % (1u << P.tail_shift) == 0u &&
                P.nframes % P.job_frames == 0u && r->params.tail_split != 1u && P.njobs < (1ull << 29)) {
                const unsigned long long q = std::min<unsigned long long>(P.njobs, 64ull * std::max(r->cus, 1u));
                P.tail_from = (uint32_t)(P.njobs - q);
                P.njobs += ((1ull << P.tail_shift) - 1u) * q;
            }
            r->ring_nchunks = P.nchunks;
            HIP_TRY(hipMemsetAsync(P.queue, 0, sizeof(unsigned long long), r->stream));
            // (not with stealing: its launches are short, and the per-XCD fetch spilled SGPRs in the stealing kernels)
            P.queues = HRT_NQ && !P.ring_mode && !P.steal ? r->queues.ptr : nullptr;
            if (P.queues) HIP_TRY(hipMemsetAsync(P.queues, 0, QWORDS * sizeof(unsigned long long), r->stream));
            if (P.steal) HIP_TRY(hipMemsetAsync(P.steal_slots, 0, P.steal_cap * sizeof(unsigned long long), r->stream));
            if (P.ring_mode) HIP_TRY(hipMemsetAsync(r->ring_ctl.ptr, 0, zero_words * sizeof(uint32_t), r->stream));
            rc = trace_events(r, r->trace_pairs_pending);
            if (rc) return rc;
            HIP_TRY(hipEventRecord(r->ev_trace[2 * r->trace_pairs_pending], r->stream));
            const bool order_on = want_order && (r->params.cost_order >= 2u || !P.steal);
            if (want_order && r->cost_tiles != ntiles) {
                const size_t SCRATCH = hrt_order_scratch_words(ntiles);
                rc = ensure(r->tile_cost, (size_t)ntiles * 64u);
                if (!rc) rc = ensure(r->tile_sum, ntiles);
                if (!rc) rc = ensure(r->tile_order, ntiles);
                if (!rc) rc = ensure(r->order_scratch, SCRATCH);
                if (rc) return rc;
                HIP_TRY(hipMemsetAsync(r->tile_cost.ptr, 0, (size_t)ntiles * 64u * sizeof(uint32_t), r->stream));
                HIP_TRY(hipMemsetAsync(r->order_scratch.ptr, 0, SCRATCH * sizeof(uint32_t), r->stream));
                r->cost_tiles = ntiles;
                r->order_tiles = 0;
                r->cost_learn = true;
            }
            P.tile_order = order_on && r->order_tiles == ntiles ? r->tile_order.ptr : nullptr;
            ordered += P.tile_order ? 1u : 0u;
            // (a launch that steals still learns, so the next one can deal in cost order instead)
            const bool learn = want_order && (r->cost_learn || r->params.cost_order == 3u);
            P.tile_cost = learn ? r->tile_cost.ptr : nullptr;
            HIP_TRY(hrt_launch_trace(r->mode, variant, P, r->stream));
            HIP_TRY(hipEventRecord(r->ev_trace[2 * r->trace_pairs_pending + 1], r->stream));
            r->trace_pairs_pending++;
            launches++;
            if (learn) {  // (three small kernels, not counted in rt_stats.launches)
                HIP_TRY(hrt_launch_order(r->tile_cost.ptr, ntiles, r->tile_sum.ptr, r->tile_order.ptr, r->order_scratch.ptr,
                                         r->stream));
                r->order_tiles = ntiles;
                r->cost_learn = false;
            }
            if (!P.ring_mode && (!fold_next || done + chunk >= count)) {
                HIP_TRY(hrt_launch_accumulate(P, r->stream));
                launches++;
            }
        }
        r->last_launch_frames = chunk;
        r->last_ordered = ordered;
        r->trace_pairs = r->trace_pairs_pending;
        r->trace_pairs_pending = 0;
    } else {
        const uint32_t fpl = std::max<uint32_t>(1u, r->params.frames_per_launch);
        HIP_TRY(hipEventRecord(r->ev_start, r->stream));
        for (uint32_t done = 0; done < count; done += fpl) {
            P.nframes = std::min(fpl, count - done);
            P.time0 = time0 + done * dtime;
            P.frame0 = r->frame_count + done;
            HIP_TRY(hrt_launch_render(r->mode, variant, P, r->stream));
            launches++;
        }
        r->trace_pairs = 0;  // k_render is the whole draw: trace time = kernel time
    }
    HIP_TRY(hipEventRecord(r->ev_stop, r->stream));
    r->frame_count += count;  // end_frame, renderer.rs:409
    r->stats = rt_stats{};
    r->stats.samples = (uint64_t)count * P.nrows * r->width;
    r->stats.launches = launches;
    r->stats.local_rows = P.nrows;
    std::snprintf(r->stats.kernel, sizeof r->stats.kernel, "%s", hrt_last_kernel());
    if (schedule == RT_SCHEDULE_QUEUE && count && P.nrows) {
        r->stats.fold_ring = P.ring_mode ? 1u : r->last_fold_next ? 2u : 0u;
        r->stats.fold_bytes = r->fold_bytes;
        r->stats.launch_frames = std::min(count, r->last_launch_frames);
        r->stats.ordered_launches = r->last_ordered;
    }
    r->stats.device_bytes = r->device_bytes();
    r->timing_pending = true;
    return RT_OK;
}

int finish_stats(rt_renderer* r) {
    if (!r->timing_pending) return RT_OK;
    HIP_TRY(hipEventSynchronize(r->ev_stop));
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, r->ev_start, r->ev_stop));
    unsigned long long* q = r->raw_counters;
    unsigned long long wd[4] = {};
    HIP_TRY(hipMemcpy(q, r->counter.ptr, RT_RAW_COUNTERS * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    {  // the work counters' copies (rt_kernels.hip flush_counts) into words 0-4
        std::vector<unsigned long long> sp((size_t)hrt_dev::CSPREAD * hrt_dev::CSTRIDE);
        HIP_TRY(hipMemcpy(sp.data(), r->count_spread.ptr, sp.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        for (uint32_t k = 0; k < hrt_dev::CSPREAD; k++)
            for (uint32_t c = 0; c < 5u; c++) q[c] += sp[(size_t)k * hrt_dev::CSTRIDE + c];
    }
    HIP_TRY(hipMemcpy(wd, r->counter.ptr + hrt_dev::WATCHDOG, sizeof wd, hipMemcpyDeviceToHost));
    if (wd[0] || wd[3]) {  // waves gave up waiting for a fold-ring slot: the image is incomplete; report, do not hang
        // diagnostic build: HRT_RING_DUMP=path writes the fold-ring control words (tile done masks, tile locks and
        // cursors, free queue, tail) and the counters as raw little-endian words
#ifdef HRT_STAMPS
        if (const char* path = std::getenv("HRT_RING_DUMP")) {
            std::vector<uint32_t> ctl(r->ring_ctl_words);
            if (!ctl.empty())
                HIP_TRY(hipMemcpy(ctl.data(), r->ring_ctl.ptr, ctl.size() * 4u, hipMemcpyDeviceToHost));
            unsigned long long cnt[hrt_dev::COUNTER_WORDS];
            HIP_TRY(hipMemcpy(cnt, r->counter.ptr, sizeof cnt, hipMemcpyDeviceToHost));
            if (FILE* f = std::fopen(path, "wb")) {
                const uint32_t hdr[4] = {r->ring_tiles, r->ring_slots, r->ring_nchunks, (uint32_t)ctl.size()};
                std::fwrite(hdr, 4, 4, f);
                std::fwrite(cnt, 8, hrt_dev::COUNTER_WORDS, f);
                std::fwrite(ctl.data(), 4, ctl.size(), f);
                std::fclose(f);
            }
        }
#endif
        char msg[200];
        std::snprintf(msg, sizeof msg, "sample queue: %llu waves waited > 2^24 idle rounds for a fold-ring slot "
                      "(last: job %llu, entry flags %llx); %llu free-queue overruns", wd[0], wd[1], wd[2], wd[3]);
        r->timing_pending = false;
        return fail(RT_ERR_DEVICE, msg);
    }
    r->stats.kernel_ms = ms;
    r->stats.trace_ms = ms;
    r->stats.trace_launches = r->stats.launches;
    if (r->trace_pairs) {
        double tms = 0.0;
        for (uint32_t k = 0; k < r->trace_pairs; k++) {
            float e = 0.0f;
            HIP_TRY(hipEventElapsedTime(&e, r->ev_trace[2 * k], r->ev_trace[2 * k + 1]));
            tms += e;
        }
        r->stats.trace_ms = tms;
        r->stats.trace_launches = r->trace_pairs;
    }
    r->stats.queries = q[0];
    r->stats.box_tests = q[1];
    r->stats.sphere_tests = q[2];
    r->stats.node_tests = q[3];
    r->stats.tri_tests = q[4];
    r->stats.variant = (uint32_t)r->last_variant;
    r->stats.schedule = r->last_schedule;
    r->stats.suspend_below = r->last_suspend;
    r->timing_pending = false;
    return RT_OK;
}

void delete_buffers(rt_renderer* r) {
    r->image.release();
    r->sph_geo.release();
    r->sph_aux.release();
    r->sph_pairs.release();
    r->bvh_nodes.release();
    r->bvh_sph.release();
    r->bvh_hnodes.release();
    r->bvh_slot.release();
    r->bvh_large.release();
    r->nodes.release();
    r->nodes_so.release();
    r->tris.release();
    r->tri_geo.release();
    r->mats.release();
    r->tb_hnodes.release();
    r->tb_order.release();
    r->counter.release();
    r->count_spread.release();
    r->steal_slots.release();
    r->queues.release();
    r->samples.release();
    r->samples2.release();
    r->ring.release();
    r->ring_ctl.release();
    r->wave_trace.release();
    r->tile_cost.release();
    r->tile_sum.release();
    r->tile_order.release();
    r->order_scratch.release();
    r->cost_tiles = r->order_tiles = 0;
}

}  // namespace

extern "C" {

const char* rt_last_error(void) { return g_last_error.c_str(); }

int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* rt_build_info(void) {
    return "hrt gfx950 (HIP " HIP_VERSION_BUILD_NAME ") k_trace_split, k_trace_split_tris, k_trace, k_accumulate, "
           "k_render";
}

int rt_create(uint32_t width, uint32_t height, int mode, rt_renderer** out) {
    if (!out || width == 0 || height == 0) return fail(RT_ERR_ARG, "rt_create: null out or zero size");
    if (mode < RT_MODE_SPHERE || mode > RT_MODE_MIXED) return fail(RT_ERR_ARG, "rt_create: bad mode");
    *out = nullptr;
    int dev = 0;
    int rc = check_device(&dev);
    if (rc) return rc;
    rt_renderer* r = new rt_renderer();
    r->device = dev;
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
            delete r;
            return fail(RT_ERR_DEVICE, "rt_create: hipDeviceGetAttribute(multiprocessor count) failed");
        }
        r->cus = (uint32_t)cus;
    }
    r->mode = mode;
    r->width = width;
    r->height = height;
    r->params.bounces = mode == RT_MODE_SPHERE ? 10u : 5u;  // BOUNCE_MAX
    r->params.ema_cap = RT_SAMPLE_FRAME;
    // arrayLength(&scene) = the 100-slot buffer in the sphere program; no such floor in the others.
    r->params.min_sphere_slots = mode == RT_MODE_SPHERE ? RT_MAX_OBJECT_IN_SCENE : 0u;
    r->params.row0 = 0;
    r->params.row_step = 1;
    r->params.row_block = 1;
    r->params.frames_per_launch = 32;
    r->params.schedule = RT_SCHEDULE_AUTO;
    // auto: balanced launches of 320-639 frames of whole jobs (C3: 352 + 352 + 320 frames, 8.8 GB of colours; launch_frames)
    r->params.queue_budget_mb = 0;
    // frames per 8x8-tile job; measured with the frame-block refill: C2 59.5 (8) -> 69.1 (16) -> 68.2 (32),
    // C3 +1 % at 16, C4 equal at 8/16 and -13 % at 32, C5 +0.7 % at 16
    r->params.job_frames = 0;  // per kernel (rt_draw_frames)
    // measured: C3 (sphere) 0 -> 21.2, 8 -> 23.4, 16 -> 23.8, 24 -> 23.7, 32 -> 22.7 Grays/s (first split
    //           kernel); with the frame-block refill and 16-frame jobs 16 -> 25.2, 24 -> 25.9, 32 -> 25.2;
    //           C4 (mixed) 0 -> 7.02, 8 -> 7.74, 16 -> 8.00, 24 -> 8.15, 32 -> 8.22, 48 -> 7.92; round 4 (final
    //           kernels, profiles/r04/so/sweep_sb_mixed.txt): C4 24 = 32 (13.22), C5 16/20/24/28/32 -> 10.26/10.27/
    //           10.30/10.28/10.24: the mixed program takes 24 too, the triangle program keeps 32
    r->params.suspend_below = mode == RT_MODE_TRIS ? 32u : 24u;
    bool ok = hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreate(&r->ev_start) == hipSuccess && hipEventCreate(&r->ev_stop) == hipSuccess;
    if (!ok) {
        rt_destroy(r);
        return fail(RT_ERR_DEVICE, "rt_create: stream/event creation failed");
    }
    rc = zero_image(r);
    if (rc) {
        rt_destroy(r);
        return rc;
    }
    *out = r;
    return RT_OK;
}

int rt_destroy(rt_renderer* r) {
    if (!r) return RT_OK;
    DeviceScope ds(r->device);  // (frees on the renderer's device even if switching failed)
    if (r->stream) (void)hipStreamSynchronize(r->stream);
    delete_buffers(r);
    for (hipEvent_t e : r->ev_trace) (void)hipEventDestroy(e);
    if (r->ev_start) (void)hipEventDestroy(r->ev_start);
    if (r->ev_stop) (void)hipEventDestroy(r->ev_stop);
    if (r->stream) (void)hipStreamDestroy(r->stream);
    delete r;
    return RT_OK;
}

int rt_abi_version(uint32_t* version, uint32_t* params_bytes, uint32_t* stats_bytes) {
    if (version) *version = RT_ABI_VERSION;
    if (params_bytes) *params_bytes = (uint32_t)sizeof(rt_params);
    if (stats_bytes) *stats_bytes = (uint32_t)sizeof(rt_stats);
    return RT_OK;
}

int rt_get_params(const rt_renderer* r, rt_params* out) {
    if (!r || !out) return fail(RT_ERR_ARG, "rt_get_params: null");
    *out = r->params;
    return RT_OK;
}

int rt_set_params(rt_renderer* r, const rt_params* p) {
    if (!r || !p) return fail(RT_ERR_ARG, "rt_set_params: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    // (row0 >= height: the renderer owns no rows, e.g. a rank beyond the image's last row block; its draws
    // render nothing and its image is empty)
    if (p->row_step == 0) return fail(RT_ERR_ARG, "rt_set_params: bad row partition (row_step 0)");
    if ((uint64_t)p->row_step * std::max(p->row_block, 1u) > (1ull << 30))
        return fail(RT_ERR_ARG, "rt_set_params: row_step x row_block too large");
    if (p->variant != 0 && p->variant != 1 && p->variant != 3 && p->variant != 4)
        return fail(RT_ERR_ARG, "rt_set_params: unknown variant (0 auto, 1 simple, 3 deferred, 4 culling BVH)");
    if (p->schedule > RT_SCHEDULE_QUEUE) return fail(RT_ERR_ARG, "rt_set_params: unknown schedule");
    if (p->tri_bvh > 1) return fail(RT_ERR_ARG, "rt_set_params: tri_bvh must be 0 or 1");
    if (p->suspend_below > 64) return fail(RT_ERR_ARG, "rt_set_params: suspend_below must be 0..64");
    if (p->fold > RT_FOLD_NEXT)
        return fail(RT_ERR_ARG, "rt_set_params: fold must be 0 auto, 1 buffer, 2 ring or 3 buffers folded by the next launch");
    if (p->heap_lds > 2) return fail(RT_ERR_ARG, "rt_set_params: heap_lds must be 0 auto, 1 off or 2 on");
    if (p->steal > 2) return fail(RT_ERR_ARG, "rt_set_params: steal must be 0 auto, 1 off or 2 on");
    if (p->tail_split > 3) return fail(RT_ERR_ARG, "rt_set_params: tail_split must be 0 auto, 1 off, 2 quarters or 3 eighths");
    if (p->count_tests > 1) return fail(RT_ERR_ARG, "rt_set_params: count_tests must be 0 or 1");
    if (p->packet > 2) return fail(RT_ERR_ARG, "rt_set_params: packet must be 0 auto, 1 off or 2 on");
    if (p->cost_order > 3)
        return fail(RT_ERR_ARG, "rt_set_params: cost_order must be 0 auto, 1 off, 2 on or 3 on, learning in every launch");
    const bool rows_changed = p->row0 != r->params.row0 || p->row_step != r->params.row_step ||
                              std::max(p->row_block, 1u) != r->row_block();
    const bool slots_changed = p->min_sphere_slots != r->params.min_sphere_slots;
    // the tiles' costs (queries per sample) change with the rows, the bounce cap and the scene's slots or triangle walk,
    // not with the kernels' knobs (count_tests, job size, ...: bench.py toggles count_tests around every warmup step)
    if (rows_changed || slots_changed || p->bounces != r->params.bounces || p->tri_bvh != r->params.tri_bvh)
        r->cost_learn = true;
    r->params = *p;
    if (rows_changed) {
        r->frame_count = 0;
        int rc = zero_image(r);
        if (rc) return rc;
    }
    if (slots_changed && r->sph_geo.ptr) return upload_spheres(r);
    return RT_OK;
}

int rt_set_camera(rt_renderer* r, const void* camera80) {
    if (!r || !camera80) return fail(RT_ERR_ARG, "rt_set_camera: null");
    std::memcpy(&r->camera, camera80, sizeof(hrt::Camera));
    r->has_camera = true;
    r->cost_learn = true;
    return RT_OK;
}

int rt_set_spheres(rt_renderer* r, const void* spheres48, uint32_t n) {
    if (!r || (n && !spheres48)) return fail(RT_ERR_ARG, "rt_set_spheres: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    // a hit carries its slot in 29 bits (rt_kernels.hip Hit::id)
    if (n >= (1u << 28)) return fail(RT_ERR_ARG, "rt_set_spheres: more than 2^28 spheres");
    r->spheres.resize(n);
    if (n) std::memcpy(r->spheres.data(), spheres48, (size_t)n * sizeof(hrt::Sphere));
    r->cost_learn = true;
    return upload_spheres(r);
}

int rt_set_bvh(rt_renderer* r, const uint32_t sizes[2], const void* nodes32, uint32_t n_nodes, const void* tris64,
               uint32_t n_tris, const void* mats32, uint32_t n_mats) {
    if (!r || !sizes) return fail(RT_ERR_ARG, "rt_set_bvh: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    const uint32_t n = sizes[0], m = sizes[1];
    if (int rc = rt_host_check_bvh_sizes(sizes, n_nodes, n_tris, n_mats)) return rc;
    if ((n && !nodes32) || (m && !tris64) || (n_mats && !mats32)) return fail(RT_ERR_ARG, "rt_set_bvh: null buffer");
    r->cost_learn = true;
    const hrt::Triangle* T = (const hrt::Triangle*)tris64;
    std::vector<hrt_dev::TriDev> td(m);
    for (uint32_t j = 0; j < m; j++) {
        const hrt::Triangle& t = T[j];
        if (t.material >= n_mats) return fail(RT_ERR_ARG, "rt_set_bvh: triangle material index out of range");
        hrt_dev::TriDev d;
        d.a = float4{t.a.x, t.a.y, t.a.z, 0.0f};
        d.e1 = float4{t.b.x - t.a.x, t.b.y - t.a.y, t.b.z - t.a.z, 0.0f};  // edge1 = b - a
        d.e2 = float4{t.c.x - t.a.x, t.c.y - t.a.y, t.c.z - t.a.z, 0.0f};  // edge2 = c - a
        d.nx = t.custom.x;
        d.ny = t.custom.y;
        d.nz = t.custom.z;
        d.material = t.material;
        td[j] = d;
    }
    r->tri_aee.resize(9 * (size_t)m);
    for (uint32_t j = 0; j < m; j++) {
        const float v[9] = {td[j].a.x, td[j].a.y, td[j].a.z, td[j].e1.x, td[j].e1.y, td[j].e1.z,
                            td[j].e2.x, td[j].e2.y, td[j].e2.z};
        std::copy(v, v + 9, &r->tri_aee[9 * (size_t)j]);
    }
    r->tri_tree_dirty = true;
    const hrt::Material* M = (const hrt::Material*)mats32;
    std::vector<hrt_dev::MatDev> md(n_mats);
    for (uint32_t k = 0; k < n_mats; k++)
    {
        const hrt_dev::DielConsts dc = dielectric_consts(M[k].params.x);
        md[k] = hrt_dev::MatDev{M[k].albedo.x, M[k].albedo.y, M[k].albedo.z, M[k].params.x, M[k].kind,
                                dc.inv_param, dc.r0sq_front, dc.r0sq_back};
    }
    // The sign-ordered copy (36 B per node) only where a kernel reads it: the heap-top kernels run for heaps of at
    // most 2^24 nodes (launch_frames, tri_small); a larger tree would pay up to ~2.4 GB of host and device memory
    // for nothing
    const bool want_so = n <= (1u << 24);
    bool so_ok = false;
    std::vector<float> so;
    if (want_so) so = pack_nodes_so((const float*)nodes32, n, so_ok);
    else r->nodes_so.release();
    int rc = ensure(r->nodes, 2 * (size_t)std::max<uint32_t>(n, 1));
    if (!rc && want_so) rc = ensure(r->nodes_so, so.size());
    if (!rc) rc = ensure(r->tris, std::max<uint32_t>(m, 1));
    if (!rc) rc = ensure(r->tri_geo, 9 * (size_t)std::max<uint32_t>(m, 1));
    if (!rc) rc = ensure(r->mats, std::max<uint32_t>(n_mats, 1));
    if (rc) return rc;
    if (n) HIP_TRY(hipMemcpyAsync(r->nodes.ptr, nodes32, (size_t)n * 32u, hipMemcpyHostToDevice, r->stream));
    if (want_so)
        HIP_TRY(hipMemcpyAsync(r->nodes_so.ptr, so.data(), so.size() * sizeof(float), hipMemcpyHostToDevice, r->stream));
    if (m) HIP_TRY(hipMemcpyAsync(r->tris.ptr, td.data(), (size_t)m * sizeof(td[0]), hipMemcpyHostToDevice, r->stream));
    if (m)  // (tri_aee: the same a, e1, e2 floats, 9 per triangle)
        HIP_TRY(hipMemcpyAsync(r->tri_geo.ptr, r->tri_aee.data(), r->tri_aee.size() * sizeof(float), hipMemcpyHostToDevice,
                               r->stream));
    if (n_mats)
        HIP_TRY(hipMemcpyAsync(r->mats.ptr, md.data(), (size_t)n_mats * sizeof(md[0]), hipMemcpyHostToDevice, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    r->bvh_n = n;
    r->bvh_m = m;
    r->so_ok = so_ok;
    return RT_OK;
}

int rt_host_check_bvh_sizes(const uint32_t sizes[2], uint32_t n_nodes, uint32_t n_tris, uint32_t n_mats) {
    if (!sizes) return fail(RT_ERR_ARG, "rt_set_bvh: null sizes");
    const uint32_t n = sizes[0], m = sizes[1];
    // The kernel reads nodes[i] for i < n and triangles[j] for j < m only; validate so it cannot fault.
    if (n_nodes < n || n_tris < m) return fail(RT_ERR_ARG, "rt_set_bvh: sizes exceed the buffers given");
    // Tree::build (tree.rs:38) makes n = m.next_power_of_two() (>= 1); the walks rely on it (leaf pairs: the
    // children of nodes n/2 .. n-1 are leaves)
    if (n == 0 || (n & (n - 1u)) != 0) return fail(RT_ERR_ARG, "rt_set_bvh: sizes[0] must be a power of two");
    // The walks load nodes (32 B) and triangles (64 B) through buffer descriptors with 32-bit byte sizes and
    // offsets (rt_kernels.hip node_hit_top, tri_test<TBUF>): n x 32 and m x 64 must stay below 2^32.
    if (n > RT_MAX_TREE_NODES) return fail(RT_ERR_ARG, "rt_set_bvh: more than RT_MAX_TREE_NODES (2^26) nodes");
    if (m >= (1u << 26)) return fail(RT_ERR_ARG, "rt_set_bvh: 2^26 or more triangles");
    if (n_mats >= (1u << 28)) return fail(RT_ERR_ARG, "rt_set_bvh: more than 2^28 materials");
    return RT_OK;
}

int rt_testing_set_faults(rt_renderer* r, uint32_t ring_slots_max, uint32_t fail_alloc_above_mb) {
    if (!r) return fail(RT_ERR_ARG, "rt_testing_set_faults: null");
    r->test_ring_slots_max = ring_slots_max;
    r->test_fail_alloc_above_mb = fail_alloc_above_mb;
    return RT_OK;
}

int rt_set_time(rt_renderer* r, uint32_t time) {
    if (!r) return fail(RT_ERR_ARG, "rt_set_time: null");
    r->time = time;
    return RT_OK;
}

int rt_set_frame_count(rt_renderer* r, uint32_t fc) {
    if (!r) return fail(RT_ERR_ARG, "rt_set_frame_count: null");
    r->frame_count = fc;
    return RT_OK;
}

int rt_get_frame_count(const rt_renderer* r, uint32_t* out) {
    if (!r || !out) return fail(RT_ERR_ARG, "rt_get_frame_count: null");
    *out = r->frame_count;
    return RT_OK;
}

int rt_draw(rt_renderer* r) {
    if (!r) return fail(RT_ERR_ARG, "rt_draw: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    return launch_frames(r, 1, r->time, 0);
}

int rt_draw_frames(rt_renderer* r, uint32_t count, uint32_t time0, uint32_t dtime) {
    if (!r) return fail(RT_ERR_ARG, "rt_draw_frames: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    if (count == 0) return RT_OK;
    int rc = launch_frames(r, count, time0, dtime);
    if (!rc) r->time = time0 + (count - 1) * dtime;
    return rc;
}

int rt_read_image(rt_renderer* r, float* out, size_t n_floats) {
    if (!r || !out) return fail(RT_ERR_ARG, "rt_read_image: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    if (n_floats != r->image_floats()) return fail(RT_ERR_ARG, "rt_read_image: size mismatch");
    HIP_TRY(hipMemcpyAsync(out, r->image.ptr, n_floats * sizeof(float), hipMemcpyDeviceToHost, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    return finish_stats(r);
}

int rt_write_image(rt_renderer* r, const float* in, size_t n_floats) {
    if (!r || !in) return fail(RT_ERR_ARG, "rt_write_image: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    if (n_floats != r->image_floats()) return fail(RT_ERR_ARG, "rt_write_image: size mismatch");
    HIP_TRY(hipMemcpyAsync(r->image.ptr, in, n_floats * sizeof(float), hipMemcpyHostToDevice, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    return RT_OK;
}

int rt_copy_image_to_device(rt_renderer* r, void* dst, size_t n_floats) {
    if (!r || !dst) return fail(RT_ERR_ARG, "rt_copy_image_to_device: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    if (n_floats != r->image_floats()) return fail(RT_ERR_ARG, "rt_copy_image_to_device: size mismatch");
    HIP_TRY(hipMemcpyAsync(dst, r->image.ptr, n_floats * sizeof(float), hipMemcpyDeviceToDevice, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    return finish_stats(r);
}

int rt_reset_frame_count(rt_renderer* r) {
    if (!r) return fail(RT_ERR_ARG, "rt_reset_frame_count: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    r->frame_count = 0;
    return zero_image(r);
}

int rt_resize(rt_renderer* r, uint32_t width, uint32_t height) {
    if (!r) return fail(RT_ERR_ARG, "rt_resize: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    r->width = std::max<uint32_t>(1, width);  // renderer.rs:274-275
    r->height = std::max<uint32_t>(1, height);
    r->cost_learn = true;
    r->frame_count = 0;
    return zero_image(r);
}

int rt_synchronize(rt_renderer* r) {
    if (!r) return fail(RT_ERR_ARG, "rt_synchronize: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    HIP_TRY(hipStreamSynchronize(r->stream));
    return finish_stats(r);
}

int rt_release_scratch(rt_renderer* r) {
    if (!r) return fail(RT_ERR_ARG, "rt_release_scratch: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    if (r->timing_pending) {
        const int rc = finish_stats(r);  // the pending draws' counters, and their kernels done
        if (rc) return rc;
    }
    HIP_TRY(hipStreamSynchronize(r->stream));
    r->samples.release();
    r->samples2.release();
    r->ring.release();
    r->ring_ctl.release();
    return RT_OK;
}

int rt_get_stats(const rt_renderer* r, rt_stats* out) {
    if (!r || !out) return fail(RT_ERR_ARG, "rt_get_stats: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    int rc = finish_stats(const_cast<rt_renderer*>(r));
    if (rc) return rc;
    *out = r->stats;
    return RT_OK;
}

int rt_get_raw_counters(const rt_renderer* r, uint64_t* out, int n) {
    if (!r || !out || n < 0) return fail(RT_ERR_ARG, "rt_get_raw_counters: bad argument");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    int rc = finish_stats(const_cast<rt_renderer*>(r));
    if (rc) return rc;
    for (int i = 0; i < n; i++) out[i] = i < RT_RAW_COUNTERS ? r->raw_counters[i] : 0;
    return RT_OK;
}

int rt_get_wave_trace(rt_renderer* r, uint64_t* out, size_t n_words) {
    if (!r || !out) return fail(RT_ERR_ARG, "rt_get_wave_trace: null");
    DeviceScope ds(r->device);
    if (ds.rc) return ds.rc;
    if (n_words > r->wave_trace_words) return fail(RT_ERR_ARG, "rt_get_wave_trace: more words than recorded");
    if (n_words) HIP_TRY(hipMemcpy(out, r->wave_trace.ptr, n_words * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_get_device(const rt_renderer* r, int32_t* ordinal, int32_t pci[3]) {
    if (!r || !ordinal || !pci) return fail(RT_ERR_ARG, "rt_get_device: null");
    int v[3] = {0, 0, 0};
    HIP_TRY(hipDeviceGetAttribute(&v[0], hipDeviceAttributePciDomainId, r->device));
    HIP_TRY(hipDeviceGetAttribute(&v[1], hipDeviceAttributePciBusId, r->device));
    HIP_TRY(hipDeviceGetAttribute(&v[2], hipDeviceAttributePciDeviceId, r->device));
    *ordinal = r->device;
    for (int k = 0; k < 3; k++) pci[k] = v[k];
    return RT_OK;
}

int rt_check_exact_math(uint64_t n, uint32_t seed, uint64_t mismatches[3]) {
    if (!mismatches) return fail(RT_ERR_ARG, "rt_check_exact_math: null");
    int dev = 0;
    int rc = check_device(&dev);
    if (rc) return rc;
    unsigned long long* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, 3 * sizeof(unsigned long long)));
    hipError_t e = hipMemset(d, 0, 3 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hrt_check_exact_math(n, seed, d, nullptr);
    if (e == hipSuccess) e = hipMemcpy(mismatches, d, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(RT_ERR_DEVICE, std::string("rt_check_exact_math: ") + hipGetErrorString(e));
    return RT_OK;
}

int rt_diagnostic_build(void) {
#ifdef HRT_STAMPS
    return 1;
#else
    return 0;
#endif
}

}  // extern "C"
