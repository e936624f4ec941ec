// rt_device.hpp — device-side data layout and math of the MI355X path tracer (gfx950).
//
// Every formula restates the reference WGSL (hucancode/hello-raytracing src/shaders/shader_sphere.wgsl,
// shader_tris.wgsl) under the build's float contract, which the CPU oracle
// follows independently:
//   * IEEE f32, no contraction (compiled with -ffp-contract=off), denormals kept, correctly rounded
//     division and sqrt (HIP default -fhip-fp32-correctly-rounded-divide-sqrt);
//   * fused multiply-add ONLY in dot products (x*x', fma y, fma z [, fma w]), in the sphere
//     discriminant fma(b, b, -(4a*c)) and in point_on_ray fma(t, d, o);
//   * normalize(v) = v / sqrt(dot(v, v)); pow(x, 5) = ((x*x)*(x*x))*x; min/max = IEEE minNum/maxNum.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hrt_dev {

constexpr float FLT_MAX_REF = 3.40282e+38f;  // shader_*.wgsl:4
constexpr int MODE_SPHERE = 0, MODE_TRIS = 1, MODE_MIXED = 2;

// Dielectric constants the scatter arm would otherwise derive per hit with two IEEE divisions, computed on
// the host with the same f32 operations (renderer.cpp dielectric_consts): 1 / param (the ratio of a
// front-face hit) and reflectance's r0 * r0 for ir = 1 / param (front) and ir = param (back).
struct DielConsts {
    float inv_param, r0sq_front, r0sq_back;
};

// Winner-only sphere data (loaded once per query, for the closest sphere). inv_radius = RN(1 / radius) when
// radius lies in [2^-60, 2^60] (else 0: the hit normal divides exactly by radius the slow way).
struct SphereAux {
    float cx, cy, cz, radius;
    float ar, ag, ab, param;  // albedo.rgb, params.x
    uint32_t id;
    float inv_param, r0sq_front, r0sq_back;  // DielConsts
    float inv_radius, pad0, pad1, pad2;
};
static_assert(sizeof(SphereAux) == 64, "SphereAux");

// Triangle as the kernel reads it: a, e1 = b - a, e2 = c - a (host-precomputed with the same f32
// subtraction Moller-Trumbore performs, shader_tris.wgsl:168-169), stored normal + material index.
struct TriDev {
    float4 a;   // a.xyz, unused
    float4 e1;  // (b - a).xyz, unused
    float4 e2;  // (c - a).xyz, unused
    float nx, ny, nz;
    uint32_t material;
};
static_assert(sizeof(TriDev) == 64, "TriDev");

struct MatDev {
    float ar, ag, ab, param;
    uint32_t id;
    float inv_param, r0sq_front, r0sq_back;  // DielConsts
};
static_assert(sizeof(MatDev) == 32, "MatDev");

// Two sphere slots side by side for the packed-FP32 scan (v_pk_{add,mul,fma}_f32 work on lanes .x/.y):
// slot 2p in .x, slot 2p+1 in .y. An odd slot count is padded with a NaN-centre slot, which no test
// can accept (every comparison on NaN is false), so it never changes a result.
typedef float v2f __attribute__((ext_vector_type(2)));
struct SpherePair {
    v2f cx, cy, cz, rr;  // centre and radius*radius
};
static_assert(sizeof(SpherePair) == 32, "SpherePair");

// Closest-sphere scan implementations (rt_params.variant). Variants 2 and 5-10 of earlier builds (packed
// interval scan, while-while, lane state machine, LDS nodes, pop re-culling, 4-wide tree) were measured
// slower than 4 and removed (history).
constexpr int SCAN_SIMPLE = 1;  // one slot per iteration, exact sqrt/div whenever disc >= 0 && b < 0
constexpr int SCAN_DEFER = 3;   // slot pairs, packed math, candidate list in LDS, exact resolution after
constexpr int SCAN_BVH = 4;     // conservative BVH culling + exact tests, (t, slot) lexicographic min
constexpr uint32_t BVH_LEAF_BIT = 0x80000000u;
#ifndef HRT_BVH_STACK
#define HRT_BVH_STACK 24
#endif
constexpr int BVH_STACK = HRT_BVH_STACK;  // traversal stack entries per lane (LDS); overflow -> exact full scan

// Small culling BVHs (<= LNODE_CAP nodes, depth <= LNODE_DEPTH) are read from LDS by k_trace_split<true>
// (renderer.cpp decides, the kernel bounds its copy by the same constant).
// device counter words: [0, 16) exported (include/hrt.h RT_RAW_COUNTERS; [15] = the job queue), then the
// fold-ring watchdog: fires, the last firing wave's waiting job and its entry flags, free-queue overruns
constexpr uint32_t WATCHDOG = 16, COUNTER_WORDS = 20;
// the five work counters (queries, box / sphere tests, node / triangle tests) as CSPREAD copies, CSTRIDE words apart:
// a wave adds its sums to one copy (rt_kernels.hip flush_counts; CSPREAD a power of two), the host adds the copies
#ifndef HRT_CSPREAD
#define HRT_CSPREAD 64
#endif
constexpr uint32_t CSPREAD = HRT_CSPREAD, CSTRIDE = 16;
// the sample buffer's job queue: NQ counters (one per XCD of MI355X's 8), QSTRIDE words apart (rt_kernels.hip queue_take;
// renderer.cpp allocates and zeroes NQ x QSTRIDE words)
constexpr uint32_t NQ = 8, QSTRIDE = 16;

// fold ring: jobs per tile and launch (the done bits of a tile's fold word, rt_kernels.hip)
constexpr uint32_t FOLD_MAX_JOBS = 48;

constexpr uint32_t LNODE_CAP = 192;
constexpr uint32_t LNODE_DEPTH = 8;

// Camera-derived constants of make_ray / fs_main, read only when primary rays are generated (once per frame
// block in the sample queue). The kernels read them through kargs() (below), a pointer to the kernarg segment
// the compiler cannot see through, so the loads stay where they are used instead of being hoisted to the
// kernel entry and kept in SGPRs across the persistent loops (round-1 code objects kept these 28 values
// resident and spilled 51-54 SGPRs to VGPR lanes in k_trace_split).
struct CamDev {
    float eye[4], dir[4], up[4], right[4];
    float focal, blur, k;         // k = tan(fov / 2), host libm tanf
    float aspect, wm1, hm1;       // f32(W)/f32(H), f32(W) - 1, f32(H) - 1 (host, same IEEE ops)
    float inv_wm1, inv_hm1;       // 1 / wm1, 1 / hm1 correctly rounded (host), 0 outside [2^-60, 2^60]
    uint32_t H, pad;
};

// Kernel arguments (passed by value in the kernarg segment).
struct KParams {
    CamDev cam;                   // make_ray constants (read through kargs())
    uint32_t W, H;
    uint32_t time0, dtime, frame0, nframes;
    uint32_t bounces;
    float ema_cap;                // f32(SAMPLE_FRAME)
    uint32_t nslots;              // sphere slots scanned (arrayLength semantics)
    uint32_t npairs;              // ceil(nslots / 2) entries of sph_pairs
    uint32_t n, m;                // bvh_tree_size
    // local row kr is global row row0 + (kr / row_block) * row_stride + kr % row_block (row_stride =
    // row_step * row_block): blocks of row_block rows dealt round-robin (multi-GPU split; rt_params)
    uint32_t row0, row_step, nrows, row_block, row_stride;
    float* image;                 // nrows x W x 3
    const float4* sph_geo;        // (cx, cy, cz, r*r) per slot
    const SphereAux* sph_aux;     // per slot
    const SpherePair* sph_pairs;  // per slot pair
    // SCAN_BVH culling structure (host/sphere_bvh.hpp); boxes are relative to bvh_rc
    const float4* bvh_nodes;      // 4 float4 per node: lmin|left, lmax, rmin|right, rmax
    const float4* bvh_sph;        // leaf spheres in BVH order: cx, cy, cz, r*r
    const int* bvh_slot;          // original slot of each leaf sphere
    const int* large_slots;       // slots scanned linearly for every ray
    uint32_t nlarge, bvh_root;    // large-list length, root child word
    uint32_t bvh_nleaf, pad_l;    // spheres in the BVH (bvh_sph / bvh_slot entries)
    float bvh_rc[3], bvh_rr;      // root box centre and radius bound
    const uint4* bvh_hnodes;      // the nodes with fp16 boxes, 2 uint4 per node (every sphere-BVH walk;
                                  // renderer.cpp pack_bvh_hnodes); bvh_nodes is the f32 form (bvh_run<.., false>)
    float bvh_rr_h;               // radius bound of the fp16 boxes (>= their half-diagonal)
    uint32_t bvh_nnodes;          // nodes in bvh_hnodes
    uint32_t bvh_lnodes;          // 1: k_trace_split keeps the nodes in LDS (<= LNODE_CAP nodes, depth <= 8)
    uint32_t packet;              // 1 (with bvh_lnodes): k_trace_split<.., PACKET> walks primary rays as packets
    float pad_k1, pad_k2, pad_k3, pad_k4;  // per-query padding constants (DESIGN.md §Sphere BVH)
    // opt-in SAH triangle tree (rt_params.tri_bvh; host/tri_bvh.hpp), nodes with fp16 boxes like bvh_hnodes
    const uint32_t* tb_order;     // triangle index of each leaf entry
    uint32_t tb_root, tri_bvh;    // root child word; 1 = walk the SAH tree instead of the reference heap
    float tb_rc[3], tb_rr;        // root box centre (nodes are relative to it) and radius bound
    const uint4* tb_hnodes;       // 2 uint4 per node (renderer.cpp pack_bvh_hnodes)
    float tb_rr_h, tb_pad16;      // radius bound of the fp16 boxes; padding
    const float4* nodes;          // 2 float4 per node: min, max
    const TriDev* tris;
    const MatDev* mats;
    unsigned long long* counter;  // [0] closest-hit queries, [1] box tests, [2] exact sphere tests
    unsigned long long* wave_trace;  // diagnostic build: 8 words per wave (rt_kernels.hip WaveRecord)
    // diagnostic build: per job (tile * nchunks + chunk, < 2^21), k_trace: the ticks from its take to the wave's next take
    // (or drain) | the take's s_memrealtime low 32 bits << 32
    unsigned long long* job_trace;
    // sample-queue schedule (k_trace, k_trace_split, k_trace_split_tris). Two ways to fold the sample colours
    // into the image in frame order: the sample buffer (ring_mode 0: every colour of the launch, folded by
    // k_accumulate after it; fastest, memory O(frames x pixels)) or the fold ring (ring_mode 1: a job's samples go
    // to a ring slot taken from a free queue when the job is dealt; each tile's jobs are folded in order inside
    // the launch as they complete and their slots return to the queue; memory O(jobs in flight)).
    float* samples;               // mode 0: nframes x (tiles_w * tiles_h) x 64 px x 3 colours, frame- then tile-major
    uint32_t ring_mode, pad_m;
    float4* ring;                 // ring_jobs x job_frames x 64 px colour (r, g, b, unused)
    uint32_t* ring_q;             // [4 ring_jobs]: free queue: slot | (lap & 0x7FF) << 20 | valid << 31
    uint32_t* ring_tail;          // free-queue tickets issued (slots returned)
    uint32_t* job_slot;           // [tile * nchunks + chunk]: the job's slot (for its folder)
    unsigned long long* tile_fold;  // [tile]: bit c = job c stored (c < 48), bits 48-54 jobs folded, bit 63 lock
    uint32_t ring_log2;           // ring_jobs = 1 << ring_log2 (<= 2^20)
    uint32_t ring_bytes;          // size of `ring` (buffer-descriptor range)
    uint32_t jf_log2, pad_r;      // job_frames = 1 << jf_log2
    unsigned long long* queue;    // next job index (zeroed before each k_trace launch)
    // sample buffer: NQ job counters, one per XCD, QSTRIDE words apart (rt_kernels.hip queue_take; null: `queue` alone)
    unsigned long long* queues;
    unsigned long long njobs;     // tiles_w * tiles_h * ceil(nframes / job_frames), + 3 per job split in quarters
    uint32_t tail_from;           // sample buffer: jobs from this index on are parts of jobs (2^tail_shift per job)
    uint32_t tail_shift;
    uint32_t tiles_w, tiles_h;    // 8x8 tiles over W x nrows
    uint32_t job_frames, nchunks; // frames per job (a job = one tile x job_frames frames), chunks per tile
    uint32_t suspend_below;       // k_trace_split: suspend the walks once fewer lanes than this still walk
    uint32_t tri_small;           // k_trace_split_tris<.., SMALL>: 16-bit triangle lists + the heap top in LDS
    // frame-block work stealing (k_trace_split / k_trace_split_tris with the sample buffer; rt_kernels.hip steal_block)
    unsigned long long* steal_slots;  // one per wave: (job + 1) << 32 | frames claimed; zeroed per launch
    uint32_t steal, nwaves;       // on; waves of the launch (launch_persistent)
    uint32_t steal_cap, pad_s;    // slots allocated (bounds the grid)
    // the heap's nodes as (lo, hi, lo) per axis, 9 floats per node (renderer.cpp pack_nodes_so; the heap-top kernels'
    // sign-ordered node test, rt_kernels.hip node_hit_so); so_ok 0: a NaN bound, the reference form only
    const float* nodes_so;
    uint32_t so_ok;
    uint32_t count_tests;         // k_trace_split<.., COUNT>: box / sphere test counts (rt_params.count_tests)
    // the triangles' test operands alone, a | e1 | e2 as 9 floats (36 B) per triangle (the deferred tests of the
    // split kernels, tri_test<TBUF>): 35 KB for Suzanne instead of the 64-B records' 63 KB in the CU's 32-KB L1
    const float* tri_geo;
    // cost-ordered dealing (sample buffer; rt_params.cost_order): in a learning launch every finished sample adds its
    // query count to its pixel's counter (tile_cost[pix], null = not learning); tile_order (null = raster order): the
    // tiles in descending order of their last learnt cost (rt_kernels.hip k_order_*)
    uint32_t* tile_cost;
    const uint32_t* tile_order;
    unsigned long long* count_spread;  // CSPREAD x CSTRIDE words: the work counters' copies
    // fold of the previous launch's sample buffer inside this launch (rt_kernels.hip fold_prev_tiles; null: none):
    // every fold_mod-th wave folds tiles taken from *fold_next before it traces
    const float* fold_prev;
    uint32_t* fold_next;
    uint32_t fold_nframes, fold_frame0, fold_mod, pad_f;
};

// KParams in the kernarg segment (constant address space: scalar loads), as a pointer the compiler cannot
// trace back to the kernel's entry, so every use is a fresh s_load (K$) instead of a live SGPR.
typedef const __attribute__((address_space(4))) KParams* KPtr;

// Global image row of this renderer's local row kr (seed and camera ray use global coordinates).
__device__ __forceinline__ uint32_t global_row(uint32_t row0, uint32_t row_block, uint32_t row_stride, uint32_t kr) {
    const uint32_t b = kr / row_block;
    return row0 + b * row_stride + (kr - b * row_block);
}
typedef const __attribute__((address_space(4))) CamDev* CamPtr;
__device__ __forceinline__ KPtr kargs() {
    const unsigned long long v = (unsigned long long)__builtin_amdgcn_kernarg_segment_ptr();
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    asm volatile("" : "+s"(lo), "+s"(hi));
    return (KPtr)(((unsigned long long)hi << 32) | lo);
}

struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 operator*(float s, f3 a) { return mk(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x)); }
__device__ __forceinline__ float length(f3 a) { return __builtin_sqrtf(dot(a, a)); }
__device__ __forceinline__ f3 normalize(f3 a) {
    float l = length(a);
    return mk(a.x / l, a.y / l, a.z / l);
}
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ f3 point_on_ray(f3 o, f3 d, float t) {
    return mk(__builtin_fmaf(t, d.x, o.x), __builtin_fmaf(t, d.y, o.y), __builtin_fmaf(t, d.z, o.z));
}
__device__ __forceinline__ float fmin_ieee(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ float fmax_ieee(float a, float b) { return __builtin_fmaxf(a, b); }

// Correctly rounded sqrt for x in [2^-100, 2^100] or x == 0: v_sqrt_f32 (<= 1 ulp) then the Tuckerman
// rounding test that the HIP library sequence applies (one ulp down / up, chosen by the sign of the exact FMA
// residual), without that sequence's denormal scaling and special-class fix-up, which such x never need.
__device__ __forceinline__ float sqrt_rn_mid(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    const float rd = __builtin_fmaf(-sd, s, x), ru = __builtin_fmaf(-su, s, x);
    const float t = rd <= 0.0f ? sd : s;
    return ru > 0.0f ? su : t;
}

// Correctly rounded x / l for several x sharing one divisor: v_rcp_f32 refined by one Newton step, then
// q = x r and two exact-residual corrections (the FMA steps of the HIP division sequence, whose
// v_div_scale / v_div_fmas / v_div_fixup only handle operands near the ends of the range). Valid when l
// and every nonzero |x| lie in [2^-60, 2^60] (all intermediates normal, residuals exact); x = +0 gives +0.
struct RcpRN {
    float l, r;
};
// The refined reciprocal: v_rcp_f32 (<= 1 ulp) and one Newton step whose residual 1 - l r0 is exact. It is
// itself RN(1 / l) for |l| in [2^-60, 2^60]: for every significand and every r0 within 1 ulp of 1 / l the step
// lands on the correctly rounded value except r0 = 2^k under an all-ones significand, where r0 + r0 (1 - l r0)
// is a tie that rounds back to r0 (tests/test_rcp_exact.py enumerates both); the GPU self-check
// (k_check_exact_math) runs every significand through v_rcp_f32 itself.
__device__ __forceinline__ float rcp_rn_mid(float l) {
    const float r0 = __builtin_amdgcn_rcpf(l);
    return __builtin_fmaf(__builtin_fmaf(-l, r0, 1.0f), r0, r0);
}
__device__ __forceinline__ RcpRN rcp_rn_setup(float l) { return RcpRN{l, rcp_rn_mid(l)}; }
// 1 / l, bit-identical to the IEEE division: the refined reciprocal where |l| lies in [2^-60, 2^60], else `/`.
__device__ __forceinline__ float rcp_exact(float l) {
    const float al = __builtin_fabsf(l);
    if (al >= 0x1p-60f && al <= 0x1p60f) return rcp_rn_mid(l);
    return 1.0f / l;
}
__device__ __forceinline__ float div_rn_mid(float x, const RcpRN& d) {
    float q = x * d.r;
    q = __builtin_fmaf(__builtin_fmaf(-d.l, q, x), d.r, q);
    return __builtin_fmaf(__builtin_fmaf(-d.l, q, x), d.r, q);
}

// normalize() of a vector of rng floats (each 0 or in [2^-32, 1], not all 0): dot in [2^-64, 3], so the
// length and the three quotients stay inside the ranges above; bit-identical to normalize().
__device__ __forceinline__ f3 normalize_rng(f3 a) {
    const RcpRN d = rcp_rn_setup(sqrt_rn_mid(dot(a, a)));
    return mk(div_rn_mid(a.x, d), div_rn_mid(a.y, d), div_rn_mid(a.z, d));
}

// sqrt / division with the sequences above where their ranges hold, else the IEEE operation; bit-identical.
__device__ __forceinline__ float sqrt_exact(float x) {
    return (x >= 0x1p-100f && x <= 0x1p100f) ? sqrt_rn_mid(x) : __builtin_sqrtf(x);
}
__device__ __forceinline__ float div_exact(float x, float l) {
    const float ax = __builtin_fabsf(x), al = __builtin_fabsf(l);
    if (ax >= 0x1p-60f && ax <= 0x1p60f && al >= 0x1p-60f && al <= 0x1p60f) return div_rn_mid(x, rcp_rn_setup(l));
    return x / l;
}

// normalize() of any vector: the sequences above when every component's magnitude lies in [2^-40, 2^40] (then
// dot is in [2^-80, 3 x 2^80] and the length and quotients inside their ranges), else the IEEE operations;
// bit-identical to normalize() either way (GPU self-check: rt_check_exact_math).
__device__ __forceinline__ f3 normalize_exact(f3 a) {
    const float lo = fmin_ieee(fmin_ieee(__builtin_fabsf(a.x), __builtin_fabsf(a.y)), __builtin_fabsf(a.z));
    const float hi = fmax_ieee(fmax_ieee(__builtin_fabsf(a.x), __builtin_fabsf(a.y)), __builtin_fabsf(a.z));
    if (lo >= 0x1p-40f && hi <= 0x1p40f) {
        const RcpRN d = rcp_rn_setup(sqrt_rn_mid(dot(a, a)));
        return mk(div_rn_mid(a.x, d), div_rn_mid(a.y, d), div_rn_mid(a.z, d));
    }
    return normalize(a);
}

// The guarded sequences above with their range guard as ONE wave-uniform branch (k_trace_split's shading): the fast
// sequence runs for every lane, and only a wave with a lane outside its range recomputes that lane with the guarded
// function itself. The same bits; in the common case a compare and a scalar branch instead of an exec-mask save, a
// branch and a restore around each arm.
__device__ __forceinline__ float sqrt_exact_u(float x) {
    float s = sqrt_rn_mid(x);
    const bool slow = !(x >= 0x1p-100f && x <= 0x1p100f);
    if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
        if (slow) s = __builtin_sqrtf(x);
    }
    return s;
}
__device__ __forceinline__ f3 normalize_exact_u(f3 a) {
    const float lo = fmin_ieee(fmin_ieee(__builtin_fabsf(a.x), __builtin_fabsf(a.y)), __builtin_fabsf(a.z));
    const float hi = fmax_ieee(fmax_ieee(__builtin_fabsf(a.x), __builtin_fabsf(a.y)), __builtin_fabsf(a.z));
    const RcpRN d = rcp_rn_setup(sqrt_rn_mid(dot(a, a)));
    f3 q = mk(div_rn_mid(a.x, d), div_rn_mid(a.y, d), div_rn_mid(a.z, d));
    const bool slow = !(lo >= 0x1p-40f && hi <= 0x1p40f);
    if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
        if (slow) q = normalize(a);
    }
    return q;
}

// PCG hash step — shader_sphere.wgsl:87-93.
__device__ __forceinline__ uint32_t pcg_next(uint32_t s) {
    uint32_t old = s + 747796405u + 2891336453u;
    uint32_t word = ((old >> ((old >> 28u) + 4u)) ^ old) * 277803737u;
    return (word >> 22u) ^ word;
}
// rng_float — :94-97: f32(state) / f32(0xffffffff) = round(state) * 2^-32.
__device__ __forceinline__ float rng_float(uint32_t& s) {
    s = pcg_next(s);
    return (float)s * 2.3283064365386963e-10f;
}

// reflect / refract / reflectance — shader_sphere.wgsl:156-171.
__device__ __forceinline__ f3 reflect(f3 v, f3 n) { return v - (2.0f * dot(v, n)) * n; }
// FAST: the range-guarded exact square roots (sphere program); else the IEEE ones (the same bits). U: their guards as
// wave-uniform branches (sqrt_exact_u).
template <bool FAST = true, bool U = false>
__device__ __forceinline__ f3 refract(f3 uv, f3 n, float e) {
    float cos_t = fmin_ieee(dot(-uv, n), 1.0f);
    f3 perp = e * (uv + cos_t * n);
    float len = FAST ? (U ? sqrt_exact_u(dot(perp, perp)) : sqrt_exact(dot(perp, perp))) : length(perp);
    const float q = __builtin_fabsf(1.0f - len * len);
    f3 par = (-(FAST ? (U ? sqrt_exact_u(q) : sqrt_exact(q)) : __builtin_sqrtf(q))) * n;
    return perp + par;
}
__device__ __forceinline__ float reflectance(float cosine, float ref_idx) {
    float r0 = (1.0f - ref_idx) / (1.0f + ref_idx);
    r0 = r0 * r0;
    float x = 1.0f - cosine;
    float x2 = x * x;
    return r0 + (1.0f - r0) * ((x2 * x2) * x);
}
// reflectance() with r0 * r0 precomputed (the same f32 operations, on the host).
__device__ __forceinline__ float reflectance_r0sq(float cosine, float r0) {
    float x = 1.0f - cosine;
    float x2 = x * x;
    return r0 + (1.0f - r0) * ((x2 * x2) * x);
}

}  // namespace hrt_dev
