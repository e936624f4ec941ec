// rt_kernels.hip — the per-pixel path-tracing loop for MI355X (gfx950), hand-written HIP.
//
// Replaces the reference's WGSL fragment program fs_main (hucancode/hello-raytracing
// src/shaders/shader_sphere.wgsl:251-273, shader_tris.wgsl:325-347) run once per pixel per frame by
// a full-screen draw (src/renderer.rs:382-399). Design:
//   * one thread per pixel; a wave64 covers an 8x8 pixel tile (ray coherence for the wave-uniform
//     sphere scan), a 256-thread workgroup a 16x16 tile;
//   * F frames (samples) per launch, looped IN the kernel: the accumulation (WGSL mix, :264-271) runs
//     in registers and the framebuffer is read once and written once per launch;
//   * the bounce loop is flattened into a per-lane query loop: each iteration is ONE closest-hit query
//     for every live lane; a lane whose path ends (miss or bounce cap) accumulates and immediately
//     starts its next frame's primary ray, so lanes never idle waiting for the wave's longest path
//     (lane-level refill instead of wave-level compaction);
//   * the sphere list is scanned in slot order with a wave-uniform index, so the per-sphere data are
//     scalar (SGPR) loads shared by the 64 lanes; only the winning sphere's record is gathered;
//   * the implicit-heap BVH walk (shader_tris.wgsl:268-301) is per lane, with the reference's
//     traversal order and 600-step cap.
#include "rt_device.hpp"

#include <algorithm>
#include <type_traits>

using namespace hrt_dev;

namespace {

struct Ray {
    f3 o, d;
};

#ifdef HRT_STAMPS
// In-kernel stamp (diagnostic build): one s_memtime with its wait inside the statement, fenced from
// scheduling (cdna_hip_programming.md §7, In-kernel stamps).
__device__ __forceinline__ unsigned long long hrt_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
// Constant 100 MHz clock (s_memrealtime), to calibrate s_memtime and measure wave residency.
__device__ __forceinline__ unsigned long long hrt_realtime() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#endif

struct Hit {
    f3 p, n;
    float t;
    float ar, ag, ab, param;
    // material arm in bits 0-1 (1 lambertian, 2 metal, 0 dielectric / default), bit 2 set for a sphere hit,
    // and above them the sphere slot (sph_aux) or material index (mats) the dielectric constants are read from
    uint32_t id;
    bool front;
};

// intersect_all_sphere + intersect_sphere (shader_sphere.wgsl:218-229, :136-155). Returns the slot of
// the closest root with t > 0 && t < best (first slot wins ties), or -1. Skipping b >= 0 is exact:
// then -b - sqrt(disc) <= 0, so t <= 0 (or NaN) and the reference rejects it too.
// (PP: a KParams pointer, generic or the kernarg segment's constant one: kargs())
template <typename PP>
__device__ __forceinline__ int scan_spheres_p(PP P, const Ray& r, float& best) {
    const float a = dot(r.d, r.d);
    const float a4 = 4.0f * a;
    const float a2 = 2.0f * a;
    int bi = -1;
    const float4* __restrict__ geo = P->sph_geo;
    const uint32_t ns = P->nslots;
    for (uint32_t i = 0; i < ns; i++) {
        const float4 g = geo[i];  // wave-uniform: scalar load
        const float ocx = r.o.x - g.x, ocy = r.o.y - g.y, ocz = r.o.z - g.z;
        const float b = 2.0f * __builtin_fmaf(ocz, r.d.z, __builtin_fmaf(ocy, r.d.y, ocx * r.d.x));
        const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - g.w;
        const float disc = __builtin_fmaf(b, b, -(a4 * c));
        if (disc >= 0.0f && b < 0.0f) {
            const float t = (-b - __builtin_sqrtf(disc)) / a2;
            if (t > 0.0f && t < best) {
                best = t;
                bi = (int)i;
            }
        }
    }
    return bi;
}
__device__ __forceinline__ int scan_spheres(const KParams& P, const Ray& r, float& best) {
    return scan_spheres_p(&P, r, best);
}


// The reference's t for slot i, recomputed exactly as the scan computes it (scalar IEEE ops give the
// same bits as the packed lanes). Returns -1 when the reference would give t = -1 (disc < 0).
__device__ __forceinline__ float exact_sphere_t(const KParams& P, const Ray& r, int i, float a4, float a2) {
    const float4 g = P.sph_geo[i];
    const float ocx = r.o.x - g.x, ocy = r.o.y - g.y, ocz = r.o.z - g.z;
    const float bd = __builtin_fmaf(ocz, r.d.z, __builtin_fmaf(ocy, r.d.y, ocx * r.d.x));
    const float b = bd + bd;
    const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - g.w;
    const float disc = __builtin_fmaf(b, b, (-a4) * c);
    if (disc < 0.0f) return -1.0f;
    return (-b - __builtin_sqrtf(disc)) / a2;
}

// Deferred scan, bit-identical to scan_spheres. Pass 1 (uniform over all slot pairs, packed math)
// only decides which pairs hold a candidate (disc >= 0 && b <= 0, or NaN: conservative) and appends
// the pair index to this lane's list in LDS (ascending). Pass 2 resolves the few candidates with the
// reference's exact arithmetic in slot order, so `t > 0 && t < best` and first-slot-wins ties are
// reproduced literally. A lane whose list overflows falls back to the full exact scan.
// list entries per lane; slot CAND_CAP is a write sink past overflow (14, not 15: the wave job words then fit
// beside the mixed deferred-scan kernels' 32 KB of LDS at 5 workgroups per CU)
constexpr int CAND_CAP = 14;

__device__ __forceinline__ int scan_spheres_deferred(const KParams& P, const Ray& r, float& best,
                                                     uint16_t* __restrict__ lds_list) {
    const float a = dot(r.d, r.d);
    const float a4 = 4.0f * a;
    const float a2 = 2.0f * a;
    const v2f ox = {r.o.x, r.o.x}, oy = {r.o.y, r.o.y}, oz = {r.o.z, r.o.z};
    const v2f dx = {r.d.x, r.d.x}, dy = {r.d.y, r.d.y}, dz = {r.d.z, r.d.z};
    const v2f na4 = {-a4, -a4};
    uint32_t cnt = 0;

    const SpherePair* __restrict__ pairs = P.sph_pairs;
    const uint32_t np = P.npairs;
#pragma unroll 2
    for (uint32_t p = 0; p < np; p++) {
        const SpherePair q = pairs[p];  // wave-uniform: scalar loads
        const v2f ocx = ox - q.cx, ocy = oy - q.cy, ocz = oz - q.cz;
        v2f bd = ocx * dx;
        bd = __builtin_elementwise_fma(ocy, dy, bd);
        bd = __builtin_elementwise_fma(ocz, dz, bd);
        const v2f b = bd + bd;
        v2f cd = ocx * ocx;
        cd = __builtin_elementwise_fma(ocy, ocy, cd);
        cd = __builtin_elementwise_fma(ocz, ocz, cd);
        const v2f c = cd - q.rr;
        const v2f disc = __builtin_elementwise_fma(b, b, na4 * c);
        const float x0 = __builtin_fminf(disc.x, -b.x);
        const float x1 = __builtin_fminf(disc.y, -b.y);
        if (__builtin_fmaxf(x0, x1) >= 0.0f) {
            lds_list[(cnt < (uint32_t)CAND_CAP ? cnt : (uint32_t)CAND_CAP) * 256u] = (uint16_t)p;
            cnt++;
        }
    }
    if (cnt > (uint32_t)CAND_CAP) return scan_spheres(P, r, best);  // overflow: exact full scan

    int bi = -1;
    float bt = best;
    for (uint32_t k = 0; k < cnt; k++) {
        const uint32_t p = lds_list[k * 256u];
#pragma unroll
        for (uint32_t s = 0; s < 2; s++) {
            const uint32_t i = 2 * p + s;
            if (i >= P.nslots) break;
            const float t = exact_sphere_t(P, r, (int)i, a4, a2);
            if (t > 0.0f && t < bt) {
                bt = t;
                bi = (int)i;
            }
        }
    }
    best = bt;
    return bi;
}

// Lane 0 of a wave, at its end: its work counts (queries, box / sphere tests, node / triangle tests) added to its copy of
// the counters (wave id % CSPREAD). One set of counters for every wave made the launch's last ~1 ms a queue of
// same-address atomics (C2: 6144 waves x 5).
__device__ __forceinline__ void flush_counts(const unsigned long long (&sums)[5]) {
#if defined(HRT_STAMPS) && defined(HRT_DIAG_NOFLUSH)  // (timing-only diagnostic build: no work counters)
    if (sums[0] != ~0ull) return;
#endif
    // (any spread of the waves over the copies will do: the wave's hardware slot — wave, SIMD, CU, shader engine in
    // HW_ID, a scalar read here — and its workgroup; threadIdx-based indices kept a VGPR alive across the kernel)
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const uint32_t idx = (hw ^ (hw >> 8) ^ (hw >> 13) ^ blockIdx.x) & (CSPREAD - 1u);
    unsigned long long* const c = kargs()->count_spread + idx * CSTRIDE;
#pragma unroll
    for (int k = 0; k < 5; k++) atomicAdd(c + k, sums[k]);
}

struct Tally {
    uint32_t boxes = 0, spheres = 0;  // sphere culling BVH box tests, ray-sphere tests
    uint32_t nodes = 0, tris = 0;     // triangle program: implicit-heap node tests, triangle tests
#ifdef HRT_STAMPS
    // diagnostic build, k_trace_split: lane and wave counts of walk steps (internal node / leaf), rounds,
    // lanes shading per round, rounds with a shading lane
    uint32_t lbox = 0, wbox = 0, lleaf = 0, wleaf = 0, rounds = 0, lshade = 0, wshade = 0;
    // lanes / waves per outer walk iteration (descent + leaf + pop) and lanes walking when the walk is entered
    uint32_t lwalk = 0, wwalk = 0, lentry = 0;
    // the mixed kernel's run-to-completion sphere walk (k_trace_split_tris, begin phase): walks entered (waves), and the
    // box / leaf steps run with fewer than DIAG_LOW lanes (waves, lanes)
    uint32_t wentry = 0, wbox_low = 0, lbox_low = 0, wleaf_low = 0, lleaf_low = 0;
#endif
};

#ifdef HRT_STAMPS
__device__ __forceinline__ bool first_active_lane() {
    return __lane_id() == (unsigned)(__ffsll((unsigned long long)__ballot(1)) - 1);
}
#endif

// (t, slot) lexicographic minimum = the reference's linear scan: strict `t < best` keeps the first slot
// among equal t, so a later-visited lower slot with the same t must win.
__device__ __forceinline__ bool beats(float t, int i, float bt, int bi) {
    return t > 0.0f && (t < bt || (t == bt && bi >= 0 && i < bi));
}

// The reference's t for a sphere given its (cx, cy, cz, r*r) — same ops as exact_sphere_t.
// FAST: the range-guarded exact sqrt / division (the sphere program's split kernel); else IEEE (same bits).
template <bool FAST = false>
__device__ __forceinline__ float exact_t_geo(const float4 g, const Ray& r, float a4, float a2) {
    const float ocx = r.o.x - g.x, ocy = r.o.y - g.y, ocz = r.o.z - g.z;
    const float bd = __builtin_fmaf(ocz, r.d.z, __builtin_fmaf(ocy, r.d.y, ocx * r.d.x));
    const float b = bd + bd;
    const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - g.w;
    const float disc = __builtin_fmaf(b, b, (-a4) * c);
    if (!(disc >= 0.0f && b <= 0.0f)) return -1.0f;  // t would be <= 0, NaN or -1: never accepted
    if (FAST) return div_exact(-b - sqrt_exact(disc), a2);
    return (-b - __builtin_sqrtf(disc)) / a2;
}

// exact_t_geo's own test, alone: true when exact_t_geo goes on to the root (the same operations, so the same verdict)
__device__ __forceinline__ bool sphere_candidate(const float4 g, const Ray& r, float a4) {
    const float ocx = r.o.x - g.x, ocy = r.o.y - g.y, ocz = r.o.z - g.z;
    const float bd = __builtin_fmaf(ocz, r.d.z, __builtin_fmaf(ocy, r.d.y, ocx * r.d.x));
    const float b = bd + bd;
    const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - g.w;
    const float disc = __builtin_fmaf(b, b, (-a4) * c);
    return disc >= 0.0f && b <= 0.0f;
}

// exact_t_geo<true> of a sphere sphere_candidate accepted (disc >= 0, b <= 0: its test is not repeated), with the
// range guards of sqrt_exact / div_exact as one wave-uniform branch: the fast sequences run for every lane, and only a
// wave with a lane outside their ranges (disc outside [2^-100, 2^100], a numerator or 2a outside [2^-60, 2^60], a zero
// numerator) recomputes those lanes with exact_t_geo's own operations. The same bits as exact_t_geo<true>.
// (need false: the lane's result is discarded — it takes no fallback)
__device__ __forceinline__ float candidate_t(const float4 g, const Ray& r, float a4, float a2, bool need = true) {
    const float ocx = r.o.x - g.x, ocy = r.o.y - g.y, ocz = r.o.z - g.z;
    const float bd = __builtin_fmaf(ocz, r.d.z, __builtin_fmaf(ocy, r.d.y, ocx * r.d.x));
    const float b = bd + bd;
    const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - g.w;
    const float disc = __builtin_fmaf(b, b, (-a4) * c);
    const float num = -b - sqrt_rn_mid(disc);
    float t = div_rn_mid(num, rcp_rn_setup(a2));
    const float an = __builtin_fabsf(num);
    const bool slow = need && !(disc >= 0x1p-100f && disc <= 0x1p100f && an >= 0x1p-60f && an <= 0x1p60f &&
                                a2 >= 0x1p-60f && a2 <= 0x1p60f);
    if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
        if (slow) t = div_exact(-b - sqrt_exact(disc), a2);
    }
    return t;
}

// 1/d for the slab tests, |d| >= 1e-30 (else +-1e30). v_rcp_f32 (1 ulp) by default: the padding budget
// covers it (DESIGN.md §Sphere BVH exactness, slab arithmetic).
__device__ __forceinline__ float robust_inv(float d) {
    return __builtin_fabsf(d) >= 1e-30f ? __builtin_amdgcn_rcpf(d) : __builtin_copysignf(1e30f, d);
}

// Per-query slab constants: the box bound b (relative to bvh_rc) enters as t = (b - o' -/+ pad) / d.
struct Slab {
    f3 inv;     // robust 1/d
    f3 lo, hi;  // (-o' - pad) * inv and (-o' + pad) * inv
};

// Slab test of the ray against a box padded by `pad` on every side. Visits when the padded box is entered
// before it is left, not behind the origin, and not beyond the current best t (equality visits: ties must
// be seen). One fma per plane, t = fma(b, inv, (-o' -/+ pad) * inv); its rounding error in
// distance units is <= 3.02 u D (+1 u with v_rcp), inside the 1.02 delta >= 4.08 u D margin the padding leaves.
__device__ __forceinline__ bool padded_box_hit(const float4 mn, const float4 mx, const Slab& S, float bt,
                                               float& tenter) {
    const float t0x = __builtin_fmaf(mn.x, S.inv.x, S.lo.x), t1x = __builtin_fmaf(mx.x, S.inv.x, S.hi.x);
    const float t0y = __builtin_fmaf(mn.y, S.inv.y, S.lo.y), t1y = __builtin_fmaf(mx.y, S.inv.y, S.hi.y);
    const float t0z = __builtin_fmaf(mn.z, S.inv.z, S.lo.z), t1z = __builtin_fmaf(mx.z, S.inv.z, S.hi.z);
    const float tmin = fmax_ieee(fmax_ieee(fmin_ieee(t0x, t1x), fmin_ieee(t0y, t1y)), fmax_ieee(fmin_ieee(t0z, t1z), 0.0f));
    const float tmax = fmin_ieee(fmin_ieee(fmax_ieee(t0x, t1x), fmax_ieee(t0y, t1y)), fmin_ieee(fmax_ieee(t0z, t1z), bt));
    tenter = tmin;
    return tmin <= tmax;
}

// padded_box_hit with the best-t bound as a separate compare: tmin <= min(tmax, bt) <=> tmin <= tmax &&
// tmin <= bt (no NaN here: finite slabs, bt finite), without the per-iteration canonicalize of bt.
__device__ __forceinline__ bool padded_box_hit_nb(const float4 mn, const float4 mx, const Slab& S, float bt,
                                                  float& tenter) {
    const float t0x = __builtin_fmaf(mn.x, S.inv.x, S.lo.x), t1x = __builtin_fmaf(mx.x, S.inv.x, S.hi.x);
    const float t0y = __builtin_fmaf(mn.y, S.inv.y, S.lo.y), t1y = __builtin_fmaf(mx.y, S.inv.y, S.hi.y);
    const float t0z = __builtin_fmaf(mn.z, S.inv.z, S.lo.z), t1z = __builtin_fmaf(mx.z, S.inv.z, S.hi.z);
    const float tmin = fmax_ieee(fmax_ieee(fmin_ieee(t0x, t1x), fmin_ieee(t0y, t1y)), fmax_ieee(fmin_ieee(t0z, t1z), 0.0f));
    const float tmax = fmin_ieee(fmin_ieee(fmax_ieee(t0x, t1x), fmax_ieee(t0y, t1y)), fmax_ieee(t0z, t1z));
    tenter = tmin;
    return tmin <= tmax && tmin <= bt;
}

// BVH scan, bit-identical to scan_spheres: every sphere the reference could accept lies in a box the
// padded slab test visits (float-error bound on the discriminant, DESIGN.md §Sphere BVH exactness), every
// visited sphere is tested with the reference arithmetic, and the winner is the (t, slot) minimum.
// Rays the bound does not cover (non-finite origin, 2a outside [2^-100, 2^100]) or a stack overflow fall
// back to the full exact scan. `stack` is this lane's slot of the workgroup's LDS stack (stride 256).
//
// The query is split in three so a traversal can be suspended and resumed (k_trace_split): bvh_begin
// (large list, slab constants), bvh_run (the walk; with SUSPEND it returns early once fewer than
// `below` lanes of the wave are still walking, leaving the state in BvhQuery and the LDS stack) and
// bvh_end (winner slot, or the exact full scan for the fallback cases).
struct BvhQuery {
    Slab S;
    float bt;
    int bc;          // running winner as a code: BVH-order position (< nleaf) or nleaf + large-list index
    uint32_t node;   // next child word to visit
    int sp;
    uint32_t full_scan;  // uncovered ray or stack overflow: bvh_end runs the exact full scan
};

__device__ __forceinline__ int bvh_slot_of(const KParams& P, int code) {
    return (uint32_t)code < P.bvh_nleaf ? P.bvh_slot[code] : P.large_slots[code - (int)P.bvh_nleaf];
}

template <bool H16, bool SO>
__device__ __forceinline__ void bvh_slab(const KParams& P, const Ray& r, BvhQuery& Q);

// Returns true when the walk has to run (false: bvh_end does the full scan).
// SO (k_trace_split's sign-ordered box test, box_hit_so): Q.S.lo / hi hold the near / far plane constants instead of
// the min / max ones (swapped per axis where 1/d < 0).
// COUNT false (k_trace_split without rt_params.count_tests): no box / sphere test counts (1.3 % of C3's kernel time).
template <bool H16 = false, bool FAST = false, bool KA = false, bool SO = false, bool COUNT = true>
__device__ __forceinline__ bool bvh_begin(const KParams& P, const Ray& r, float best, BvhQuery& Q, Tally& tally) {
    const float a = dot(r.d, r.d);
    const float a4 = 4.0f * a, a2 = 2.0f * a;  // recomputed by bvh_run: fewer registers live across rounds
    Q.sp = 0;
    const bool finite_o = __builtin_isfinite(r.o.x) && __builtin_isfinite(r.o.y) && __builtin_isfinite(r.o.z);
    if (!(a2 > 0x1p-100f && a2 < 0x1p100f) || !finite_o) {
        Q.full_scan = 1u;
        return false;
    }
    Q.full_scan = 0u;
    // The running winner is kept as a code, so a leaf test needs no slot load; slots are fetched only
    // to break an exact t tie and at the end.
    const uint32_t nleaf = P.bvh_nleaf;
    float bt = best;
    int bc = -1;
    const uint32_t nlarge = KA ? kargs()->nlarge : P.nlarge;  // (KA: loaded per query, not held in SGPRs)
#ifndef HRT_CAND_T
#define HRT_CAND_T 2
#endif
    for (uint32_t k = 0; k < nlarge; k++) {  // ascending slots: a later equal t never wins here
        const int i = P.large_slots[k];
        float t;
        if constexpr (FAST && HRT_CAND_T >= 2) {  // (the root for every lane, selected by the test: no branch around it)
            const float4 g = P.sph_geo[i];
            const bool cand = sphere_candidate(g, r, a4);
            t = candidate_t(g, r, a4, a2, cand);
            t = cand ? t : -1.0f;
        } else {
            t = exact_t_geo<FAST>(P.sph_geo[i], r, a4, a2);
        }
        if (beats(t, i, bt, bc >= 0 ? bvh_slot_of(P, bc) : -1)) { bt = t; bc = (int)(nleaf + k); }
    }
    if constexpr (COUNT) tally.spheres += nlarge;
    Q.bt = bt;
    Q.bc = bc;
    bvh_slab<H16, SO>(P, r, Q);
    Q.node = P.bvh_root;
    return true;
}

// The walk's slab constants (bvh_begin)
template <bool H16, bool SO>
__device__ __forceinline__ void bvh_slab(const KParams& P, const Ray& r, BvhQuery& Q) {
    const float a = dot(r.d, r.d);
    // per-query padding: delta >= the distance by which a float-accepted sphere can miss geometrically
    const f3 op = mk(r.o.x - P.bvh_rc[0], r.o.y - P.bvh_rc[1], r.o.z - P.bvh_rc[2]);
    const float dl = __builtin_amdgcn_sqrtf(dot(op, op));
    const float D = dl * 1.001f + (H16 ? P.bvh_rr_h : P.bvh_rr);
    // the last term bounds 4e-23 / |d| from above: v_rsq_f32 (1 ulp) times 1 + 2.5e-5 (no IEEE division per query)
    const float delta = P.pad_k1 + fmin_ieee(P.pad_k2 * (D * D), P.pad_k3 * D) + P.pad_k4 * D +
                        4.0001e-23f * __builtin_amdgcn_rsqf(a);
    const float pad = 2.02f * delta;
    Q.S.inv = mk(robust_inv(r.d.x), robust_inv(r.d.y), robust_inv(r.d.z));
    if constexpr (SO) {
        // near / far: the pad signed like 1/d (x - (-p) = x + p exactly: the same two constants, swapped where 1/d < 0)
        const f3 ps = mk(__builtin_copysignf(pad, Q.S.inv.x), __builtin_copysignf(pad, Q.S.inv.y),
                         __builtin_copysignf(pad, Q.S.inv.z));
        Q.S.lo = mk(-op.x - ps.x, -op.y - ps.y, -op.z - ps.z);
        Q.S.hi = mk(-op.x + ps.x, -op.y + ps.y, -op.z + ps.z);
    } else {
        Q.S.lo = mk(-op.x - pad, -op.y - pad, -op.z - pad);
        Q.S.hi = mk(-op.x + pad, -op.y + pad, -op.z + pad);
    }
    Q.S.lo = Q.S.lo * Q.S.inv;
    Q.S.hi = Q.S.hi * Q.S.inv;
}

// The walk. Returns true when it has finished; with SUSPEND it may return false after a pop, once fewer
// than `below` lanes of the wave are still walking (every call makes progress: the check follows a pop).
typedef _Float16 hrt_h2 __attribute__((ext_vector_type(2)));
// fp16 box decode for the k_trace_split walk (P.bvh_hnodes): the slab FMAs take the halves directly
// (v_fma_mix_f32: the f16 operand is widened exactly inside the f32 FMA, no conversions).
__device__ __forceinline__ float h16_lo(uint32_t u) { return (float)__builtin_bit_cast(hrt_h2, u).x; }
__device__ __forceinline__ float h16_hi(uint32_t u) { return (float)__builtin_bit_cast(hrt_h2, u).y; }
// a node with fp16 boxes (2 uint4: per child [min|max] halves of x, y, z and the child word; renderer.cpp
// pack_bvh_hnodes) as the 4 float4 of the f32 layout: lmin|left, lmax, rmin|right, rmax
__device__ __forceinline__ void load_hnode(const uint4* __restrict__ hn, uint32_t node, float4& n0, float4& n1,
                                           float4& n2, float4& n3) {
    const uint4 c0 = hn[2 * node], c1 = hn[2 * node + 1];
    n0 = float4{h16_lo(c0.x), h16_lo(c0.y), h16_lo(c0.z), __uint_as_float(c0.w)};
    n1 = float4{h16_hi(c0.x), h16_hi(c0.y), h16_hi(c0.z), 0.0f};
    n2 = float4{h16_lo(c1.x), h16_lo(c1.y), h16_lo(c1.z), __uint_as_float(c1.w)};
    n3 = float4{h16_hi(c1.x), h16_hi(c1.y), h16_hi(c1.z), 0.0f};
}

// Sign-ordered padded box test (k_trace_split; the nodes' [min|max] fp16 pairs): each pair rotated by 16 bits where
// 1/d < 0 (sh = 16) puts the near plane in the low half, so with the near / far constants of bvh_begin<.., SO> the
// planes' t values are those of padded_box_hit_nb — one FMA per plane, the same roundings — and near <= far without a
// min / max per axis (min <= max, a bound and its constant order the same way, FMA rounding is monotone; 1/d is never
// 0 or NaN: robust_inv). One rotate per axis replaces a min and a max: the same visits, bit for bit.
__device__ __forceinline__ bool box_hit_so(uint32_t px, uint32_t py, uint32_t pz, uint32_t shx, uint32_t shy, uint32_t shz,
                                           const Slab& S, float bt, float& tenter) {
    const uint32_t x = __builtin_amdgcn_alignbit(px, px, shx), y = __builtin_amdgcn_alignbit(py, py, shy),
                   z = __builtin_amdgcn_alignbit(pz, pz, shz);
    const float tnx = __builtin_fmaf(h16_lo(x), S.inv.x, S.lo.x), tfx = __builtin_fmaf(h16_hi(x), S.inv.x, S.hi.x);
    const float tny = __builtin_fmaf(h16_lo(y), S.inv.y, S.lo.y), tfy = __builtin_fmaf(h16_hi(y), S.inv.y, S.hi.y);
    const float tnz = __builtin_fmaf(h16_lo(z), S.inv.z, S.lo.z), tfz = __builtin_fmaf(h16_hi(z), S.inv.z, S.hi.z);
    const float tmin = fmax_ieee(fmax_ieee(tnx, tny), fmax_ieee(tnz, 0.0f));
    const float tmax = fmin_ieee(fmin_ieee(tfx, tfy), tfz);
    tenter = tmin;
    return tmin <= tmax && tmin <= bt;
}

// NOOVF: the stack cannot overflow — a tree of depth <= STACK (renderer.cpp gates k_trace_split<LNODES> and the
// mixed kernels' 8-entry stack on depth <= 8): visiting a node of depth d the stack holds at most d entries (one
// pending sibling per level above it), so a push at an internal node (d <= depth - 1) leaves at most depth. The
// push then needs no bound check and the walk no overflow flag (5 VALU of a ~50-VALU box step).
// SO (with H16; Q from bvh_begin<.., SO>): box_hit_so.
template <bool SUSPEND, int STACK = BVH_STACK, bool SELECT = false, bool H16 = false, uint32_t LS = 256,
          bool NOOVF = false, bool SO = false, bool COUNT = true>
__device__ __forceinline__ bool bvh_run(const KParams& P, const Ray& r, BvhQuery& Q, uint32_t* stack,
                                        Tally& tally, uint32_t below, const uint4* __restrict__ hn = nullptr) {
    static_assert(!SO || H16, "the sign-ordered box test reads fp16 pairs");
    const float4* __restrict__ nodes = P.bvh_nodes;
    const Slab S = Q.S;
    // SO: the rotation of each axis pair, 16 where 1/d < 0 (recomputed per call: not kept across rounds)
    const uint32_t shx = SO ? (__float_as_uint(S.inv.x) >> 27) & 16u : 0u, shy = SO ? (__float_as_uint(S.inv.y) >> 27) & 16u : 0u,
                   shz = SO ? (__float_as_uint(S.inv.z) >> 27) & 16u : 0u;
    const float a = dot(r.d, r.d);  // the same value bvh_begin computed
    const float a4 = 4.0f * a, a2 = 2.0f * a;
    uint32_t node = Q.node;
    int sp = Q.sp;
    float bt = Q.bt;
    int bc = Q.bc;
    // overflow and finished are kept as integers (VGPRs): an i1 lane mask carried through the nested
    // divergent loops of k_trace_split was observed to keep stale overflow bits (sticky full scans)
    uint32_t overflow = 0u, finished = 0u;
#ifndef HRT_BTEST
#define HRT_BTEST 1
#endif
#ifndef HRT_LEAFIV
#define HRT_LEAFIV 1
#endif
#ifndef HRT_LEAF_DEFER
#define HRT_LEAF_DEFER 1
#endif
    if constexpr (NOOVF && SO && HRT_BTEST) {
        // The sign-ordered walks without overflow (k_trace_split with LDS nodes, the HL3 mixed kernels) with the
        // descent as a bottom-tested loop: one exit (a miss, or a leaf reached) and the node / stack depth updated
        // in place, where the top-tested form below kept two loop-header copies and more exec-mask bookkeeping
        // per box step (C3 +3.2 %). Same visits in the same order (the child order is the three-way form's).
#ifdef HRT_STAMPS
        tally.lentry++;
        if (first_active_lane()) tally.wentry++;
#endif
        while (true) {
#ifdef HRT_STAMPS
            tally.lwalk++;
            if (first_active_lane()) tally.wwalk++;
#endif
            if (!(node & BVH_LEAF_BIT)) {
                bool any;
                do {
#ifdef HRT_STAMPS
                    {
                        constexpr uint32_t DIAG_LOW = 24u;
                        const bool low = (uint32_t)__popcll(__ballot(1)) < DIAG_LOW;
                        tally.lbox++;
                        tally.lbox_low += low ? 1u : 0u;
                        if (first_active_lane()) {
                            tally.wbox++;
                            tally.wbox_low += low ? 1u : 0u;
                        }
                    }
#endif
                    float tl, tr;
                    const uint4 c0 = hn[2 * node], c1 = hn[2 * node + 1];
                    const bool hl = box_hit_so(c0.x, c0.y, c0.z, shx, shy, shz, S, bt, tl);
                    const bool hr = box_hit_so(c1.x, c1.y, c1.z, shx, shy, shz, S, bt, tr);
                    if constexpr (COUNT) tally.boxes += 2;
                    const bool lfirst = hl && (!hr || tl <= tr);
                    const uint32_t near = lfirst ? c0.w : c1.w, far = lfirst ? c1.w : c0.w;
                    const bool both = hl && hr;
                    any = hl || hr;
#ifndef HRT_PUSH_ALWAYS
#define HRT_PUSH_ALWAYS 1
#endif
                    // (HRT_PUSH_ALWAYS: the far child is written whether or not it is pushed — one slot past the top
                    // when it is not, never read since sp does not advance, and inside the stack: a box step runs at a
                    // node of depth d <= depth - 1 with sp <= d — so the store needs no branch and exec-mask save)
                    if (HRT_PUSH_ALWAYS || both) stack[sp * LS] = far;
                    sp += both ? 1 : 0;
                    node = any ? near : node;
                } while (any && !(node & BVH_LEAF_BIT));
            }
            if (node & BVH_LEAF_BIT) {
#ifdef HRT_STAMPS
                {
                    constexpr uint32_t DIAG_LOW = 24u;
                    const bool low = (uint32_t)__popcll(__ballot(1)) < DIAG_LOW;
                    tally.lleaf++;
                    tally.lleaf_low += low ? 1u : 0u;
                    if (first_active_lane()) {
                        tally.wleaf++;
                        tally.wleaf_low += low ? 1u : 0u;
                    }
                }
#endif
                const uint32_t first = (node >> 4) & 0x07FFFFFFu, cnt = node & 15u;
#if HRT_LEAF_DEFER
                if constexpr (SELECT) {
                    // Two passes over the leaf (k_trace_split): the cheap discriminant test of every sphere first, the
                    // lane's candidates (disc >= 0 && b <= 0: 13 % of C3's leaf tests) kept as a bit mask; then the exact
                    // roots of the candidates only. In one pass the root sequence (sqrt, division, the tie check: ~45
                    // instructions) ran for every sphere of the leaf in which ANY walking lane had a candidate — nearly
                    // every one, at a few lanes each; now it runs once per candidate of the lane with the most (mostly
                    // once per leaf). C3 +1.0 % (profiles/r06/leaf_defer/); the mixed kernels' sphere walk (C5, inside
                    // the begin phase) keeps one pass: two passes measured -0.2 % with its IEEE roots, -0.25 % with
                    // these. Exact: the same spheres are tested with the same arithmetic, the (t, slot) minimum does not
                    // depend on the order, and bt (the boxes' bound) is final before the next box step either way.
                    typedef float f4v __attribute__((ext_vector_type(4)));
                    const __amdgpu_buffer_rsrc_t rs =
                        __builtin_amdgcn_make_buffer_rsrc((void*)P.bvh_sph, (short)0, (int)(P.bvh_nleaf * 16u), 0x00020000);
                    auto leaf_geo = [&](uint32_t o) -> float4 {
                        const f4v v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o, 0, 0);
                        return float4{v.x, v.y, v.z, v.w};
                    };
                    uint32_t cand = 0u;
                    for (uint32_t o = first * 16u, oe = (first + cnt) * 16u, bit = 1u; o != oe; o += 16u, bit <<= 1) {
                        if (sphere_candidate(leaf_geo(o), r, a4)) cand |= bit;
                    }
                    while (cand != 0u) {
                        const uint32_t o = (first + (uint32_t)__builtin_ctz(cand)) * 16u;
                        cand &= cand - 1u;
                        const float t = HRT_CAND_T ? candidate_t(leaf_geo(o), r, a4, a2) : exact_t_geo<true>(leaf_geo(o), r, a4, a2);
                        if (t > 0.0f && t <= bt) {  // beats(): a tie needs both slots (rare)
                            const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(
                                (void*)P.bvh_slot, (short)0, (int)(P.bvh_nleaf * 4u), 0x00020000);
                            const int slot = (int)__builtin_amdgcn_raw_buffer_load_b32(rsl, (int)(o >> 2), 0, 0);
                            if (t < bt || (bc >= 0 && slot < bvh_slot_of(P, bc))) { bt = t; bc = (int)(o >> 4); }
                        }
                    }
                } else
#endif
#if HRT_LEAFIV
                // one induction variable: the sphere's byte offset (slot word at o / 4, BVH position o / 16)
                for (uint32_t o = first * 16u, oe = (first + cnt) * 16u; o != oe; o += 16u) {
                    float4 g;
                    if constexpr (SELECT) {  // (as below: buffer loads and the fast exact division in k_trace_split)
                        typedef float f4v __attribute__((ext_vector_type(4)));
                        const __amdgpu_buffer_rsrc_t rs =
                            __builtin_amdgcn_make_buffer_rsrc((void*)P.bvh_sph, (short)0, (int)(P.bvh_nleaf * 16u), 0x00020000);
                        const f4v v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o, 0, 0);
                        g = float4{v.x, v.y, v.z, v.w};
                    } else {
                        g = P.bvh_sph[o >> 4];
                    }
                    const float t = exact_t_geo<SELECT>(g, r, a4, a2);
                    if (t > 0.0f && t <= bt) {  // beats(): a tie needs both slots (rare)
                        int slot;
                        if constexpr (SELECT) {
                            const __amdgpu_buffer_rsrc_t rsl =
                                __builtin_amdgcn_make_buffer_rsrc((void*)P.bvh_slot, (short)0, (int)(P.bvh_nleaf * 4u), 0x00020000);
                            slot = (int)__builtin_amdgcn_raw_buffer_load_b32(rsl, (int)(o >> 2), 0, 0);
                        } else {
                            slot = P.bvh_slot[o >> 4];
                        }
                        if (t < bt || (bc >= 0 && slot < bvh_slot_of(P, bc))) { bt = t; bc = (int)(o >> 4); }
                    }
                }
#else
                for (uint32_t j = 0; j < cnt; j++) {
                    float4 g;
                    if constexpr (SELECT) {  // (as below: buffer loads and the fast exact division in k_trace_split)
                        typedef float f4v __attribute__((ext_vector_type(4)));
                        const __amdgpu_buffer_rsrc_t rs =
                            __builtin_amdgcn_make_buffer_rsrc((void*)P.bvh_sph, (short)0, (int)(P.bvh_nleaf * 16u), 0x00020000);
                        const f4v v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((first + j) * 16u), 0, 0);
                        g = float4{v.x, v.y, v.z, v.w};
                    } else {
                        g = P.bvh_sph[first + j];
                    }
                    const float t = exact_t_geo<SELECT>(g, r, a4, a2);
                    if (t > 0.0f && t <= bt) {  // beats(): a tie needs both slots (rare)
                        int slot;
                        if constexpr (SELECT) {
                            const __amdgpu_buffer_rsrc_t rsl =
                                __builtin_amdgcn_make_buffer_rsrc((void*)P.bvh_slot, (short)0, (int)(P.bvh_nleaf * 4u), 0x00020000);
                            slot = (int)__builtin_amdgcn_raw_buffer_load_b32(rsl, (int)((first + j) * 4u), 0, 0);
                        } else {
                            slot = P.bvh_slot[first + j];
                        }
                        if (t < bt || (bc >= 0 && slot < bvh_slot_of(P, bc))) { bt = t; bc = (int)(first + j); }
                    }
                }
#endif
                if constexpr (COUNT) tally.spheres += cnt;
            }
            if (sp == 0) {
                finished = 1u;
                break;
            }
            node = stack[(--sp) * LS];
            if constexpr (SUSPEND) {
                if ((uint32_t)__popcll(__ballot(1)) < below) break;
            }
        }
    } else
    while (true) {
        if (!(node & BVH_LEAF_BIT)) {
#ifdef HRT_STAMPS
            if constexpr (SUSPEND) {
                tally.lbox++;
                if (first_active_lane()) tally.wbox++;
            }
#endif
            float tl, tr;
            bool hl, hr;
            uint32_t left, right;
            if constexpr (SO) {
                const uint4 c0 = hn[2 * node], c1 = hn[2 * node + 1];
                hl = box_hit_so(c0.x, c0.y, c0.z, shx, shy, shz, S, bt, tl);
                hr = box_hit_so(c1.x, c1.y, c1.z, shx, shy, shz, S, bt, tr);
                left = c0.w;
                right = c1.w;
            } else {
                float4 n0, n1, n2, n3;
                if constexpr (H16) {
                    load_hnode(hn, node, n0, n1, n2, n3);
                } else {
                    n0 = nodes[4 * node + 0];
                    n1 = nodes[4 * node + 1];
                    n2 = nodes[4 * node + 2];
                    n3 = nodes[4 * node + 3];
                }
                // SELECT (k_trace_split): best-t bound as a separate compare (no per-step canonicalize of bt)
                // and select-form child order, +1 % on C3; the three-way branch below keeps k_trace's mixed
                // program (C5) free of spills (the select form spilled 12 VGPRs there, -1.5 %).
                hl = SELECT ? padded_box_hit_nb(n0, n1, S, bt, tl) : padded_box_hit(n0, n1, S, bt, tl);
                hr = SELECT ? padded_box_hit_nb(n2, n3, S, bt, tr) : padded_box_hit(n2, n3, S, bt, tr);
                left = __float_as_uint(n0.w);
                right = __float_as_uint(n2.w);
            }
            if constexpr (COUNT) tally.boxes += 2;
            if constexpr (SELECT && NOOVF) {
                // (updates written unconditionally: the node and stack depth stay in one register each across the
                // descent loop instead of being copied at its head)
                const bool lfirst = hl && (!hr || tl <= tr);
                const uint32_t near = lfirst ? left : right, far = lfirst ? right : left;
                const bool both = hl && hr, any = hl || hr;
                if (both) stack[sp * LS] = far;
                sp += both ? 1 : 0;
                node = any ? near : node;
                if (any) continue;
            } else if constexpr (SELECT) {
                const bool lfirst = hl && (!hr || tl <= tr);
                const uint32_t near = lfirst ? left : right, far = lfirst ? right : left;
                if (hl && hr) {
                    if (NOOVF || sp < STACK) {
                        stack[sp * LS] = far;
                        sp++;
                    } else {
                        overflow = 1u;
                    }
                }
                if (hl || hr) { node = near; continue; }
            } else {
                if (hl && hr) {
                    const bool lfirst = tl <= tr;
                    if (NOOVF || sp < STACK) {
                        stack[sp * LS] = lfirst ? right : left;
                        sp++;
                    } else {
                        overflow = 1u;
                    }
                    node = lfirst ? left : right;
                    continue;
                }
                if (hl) { node = left; continue; }
                if (hr) { node = right; continue; }
            }
        } else {
#ifdef HRT_STAMPS
            if constexpr (SUSPEND) {
                tally.lleaf++;
                if (first_active_lane()) tally.wleaf++;
            }
#endif
            const uint32_t first = (node >> 4) & 0x07FFFFFFu, cnt = node & 15u;
            for (uint32_t j = 0; j < cnt; j++) {
                float4 g;
                if constexpr (SELECT) {  // (k_trace_split) buffer loads at 32-bit offsets: no 64-bit address kept and
                                         // stepped per sphere (C3 +0.5 %; the mixed kernels have no SGPRs for the
                                         // descriptors)
                    typedef float f4v __attribute__((ext_vector_type(4)));
                    const __amdgpu_buffer_rsrc_t rs =
                        __builtin_amdgcn_make_buffer_rsrc((void*)P.bvh_sph, (short)0, (int)(P.bvh_nleaf * 16u), 0x00020000);
                    const f4v v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((first + j) * 16u), 0, 0);
                    g = float4{v.x, v.y, v.z, v.w};
                } else {
                    g = P.bvh_sph[first + j];
                }
                const float t = exact_t_geo<SELECT>(g, r, a4, a2);
                if (t > 0.0f && t <= bt) {  // beats(): a tie needs both slots (rare)
                    int slot;
                    if constexpr (SELECT) {
                        const __amdgpu_buffer_rsrc_t rsl =
                            __builtin_amdgcn_make_buffer_rsrc((void*)P.bvh_slot, (short)0, (int)(P.bvh_nleaf * 4u), 0x00020000);
                        slot = (int)__builtin_amdgcn_raw_buffer_load_b32(rsl, (int)((first + j) * 4u), 0, 0);
                    } else {
                        slot = P.bvh_slot[first + j];
                    }
                    if (t < bt || (bc >= 0 && slot < bvh_slot_of(P, bc))) { bt = t; bc = (int)(first + j); }
                }
            }
            if constexpr (COUNT) tally.spheres += cnt;
        }
        if (sp == 0) {
            finished = 1u;
            break;
        }
        node = stack[(--sp) * LS];
        if constexpr (SUSPEND) {
            if ((uint32_t)__popcll(__ballot(1)) < below) break;
        }
    }
    Q.node = node;
    Q.sp = sp;
    Q.bt = bt;
    Q.bc = bc;
    Q.full_scan |= overflow;
    return finished != 0u;
}

// KA: the fallback scan reads its constants through kargs() (k_trace_split: no SGPRs held for the rare path)
template <bool KA = false>
__device__ __forceinline__ int bvh_end(const KParams& P, const Ray& r, const BvhQuery& Q, float& best,
                                       Tally& tally) {
    if (Q.full_scan != 0u) {
        if constexpr (KA) {
            const KPtr K = kargs();
            tally.spheres += K->nslots;
            return scan_spheres_p(K, r, best);
        }
        tally.spheres += P.nslots;
        return scan_spheres(P, r, best);
    }
    best = Q.bt;
    return Q.bc >= 0 ? bvh_slot_of(P, Q.bc) : -1;
}

template <int STACK = BVH_STACK, bool H16 = true, uint32_t LS = 256, bool KA = false, bool NOOVF = false, bool SO = false>
__device__ __forceinline__ int scan_spheres_bvh(const KParams& P, const Ray& r, float& best, uint32_t* stack,
                                                Tally& tally) {
    BvhQuery Q;
    if (bvh_begin<H16, false, KA, SO>(P, r, best, Q, tally))
        bvh_run<false, STACK, false, H16, LS, NOOVF, SO>(P, r, Q, stack, tally, 0u, P.bvh_hnodes);
    return bvh_end<KA>(P, r, Q, best, tally);
}

// (p - c) / radius, exact: the host's correctly rounded 1 / radius and two residual corrections
// (div_rn_mid) where both operands lie in its proven range [2^-60, 2^60], the IEEE division elsewhere (zero,
// tiny or huge components, radius outside [2^-60, 2^60]: inv_radius = 0).
__device__ __forceinline__ float div_by_radius(float x, float radius, float inv_radius) {
    const float ax = __builtin_fabsf(x);
    if (inv_radius != 0.0f && ax >= 0x1p-60f && ax <= 0x1p60f) return div_rn_mid(x, RcpRN{radius, inv_radius});
    return x / radius;
}

// div_by_radius of the three components with the guards as one wave-uniform branch (as sqrt_exact_u): the same bits
__device__ __forceinline__ f3 div_by_radius3_u(f3 n, float radius, float inv_radius) {
    const RcpRN d{radius, inv_radius};
    f3 q = mk(div_rn_mid(n.x, d), div_rn_mid(n.y, d), div_rn_mid(n.z, d));
    const float lo = fmin_ieee(fmin_ieee(__builtin_fabsf(n.x), __builtin_fabsf(n.y)), __builtin_fabsf(n.z));
    const float hi = fmax_ieee(fmax_ieee(__builtin_fabsf(n.x), __builtin_fabsf(n.y)), __builtin_fabsf(n.z));
    const bool slow = !(inv_radius != 0.0f && lo >= 0x1p-60f && hi <= 0x1p60f);
    if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
        if (slow) q = mk(div_by_radius(n.x, radius, inv_radius), div_by_radius(n.y, radius, inv_radius),
                         div_by_radius(n.z, radius, inv_radius));
    }
    return q;
}

// The hit record from the hit point p = point_on_ray(o, d, t) (k_trace_split's packet-resolved primary rays carry p
// instead of the origin; h.t is not read after the record is made). U: the guards as wave-uniform branches.
template <bool U = false>
__device__ __forceinline__ void sphere_record_p(const KParams& P, const f3 p, const f3 d, int bi, float t, Hit& h) {
    const SphereAux s = P.sph_aux[bi];
    f3 n = p - mk(s.cx, s.cy, s.cz);
    if constexpr (U) {
        n = div_by_radius3_u(n, s.radius, s.inv_radius);
    } else {
        n = mk(div_by_radius(n.x, s.radius, s.inv_radius), div_by_radius(n.y, s.radius, s.inv_radius),
               div_by_radius(n.z, s.radius, s.inv_radius));
    }
    const bool front = dot(d, n) < 0.0f;
    if (!front) n = -n;
    h.p = p;
    h.n = n;
    h.t = t;
    h.ar = s.ar; h.ag = s.ag; h.ab = s.ab; h.param = s.param;
    h.id = ((uint32_t)bi << 3) | 4u | (s.id == 1u || s.id == 2u ? s.id : 0u);
    h.front = front;
}
template <bool U = false>
__device__ __forceinline__ void sphere_record(const KParams& P, const Ray& r, int bi, float t, Hit& h) {
    sphere_record_p<U>(P, point_on_ray(r.o, r.d, t), r.d, bi, t, h);
}

// Coherent primary rays walked as one packet (k_trace_split<.., PACKET>). The 64 primary rays of
// a frame block (one frame of one 8x8 tile) are nearly parallel: the union of the nodes their own walks visit is
// barely larger than one walk (C3 model, scripts/studies/packet_sim.cpp: 7.7 node steps per block for 7.4 per ray).
// The calling lanes (those whose query needs the walk, bvh_begin true) walk that union together: every decision is
// wave-uniform — a child is visited when any lane's padded box test passes, the near child first by the lanes' vote —
// so each step runs with every lane, the node words come from LDS at one address, and the stack is one VGPR (lane k
// holds the k-th pending node; depth <= LNODE_DEPTH). Every lane tests every sphere of a visited leaf with the
// reference arithmetic and keeps the (t, slot) lexicographic minimum, which does not depend on the visiting order.
// Exact for the same reason bvh_run is: a lane's best t never drops below its winner's t, so the lane's own padded
// test passes every box on the path to its winner's leaf, the packet visits that leaf, and the lane tests the winner;
// the spheres the packet adds are real candidates and cannot displace it. Same bits and query count as bvh_run.
template <bool COUNT>
__device__ __forceinline__ bool packet_walk(const KParams& P, const float4* __restrict__ e, BvhQuery& Q,
                                            const uint4* __restrict__ hn, Tally& tally, bool part) {
    // Called by all 64 lanes (the wave-uniform stack lives in one VGPR whose lane k every lane must be able to write);
    // `part`: the lane's ray takes part — a lane outside the image or with an uncovered ray enters with best t = -1,
    // so no box or sphere test of it passes and it never votes. The participants' direction signs must agree (C3:
    // all but the tiles a coordinate plane of the direction crosses): the sign-ordered test's pair rotations are then
    // wave-uniform (SGPRs). Else the rays stay unresolved and walk on their own (qs 0).
    const Slab S = Q.S;
    const uint32_t nx = __float_as_uint(S.inv.x) >> 31, ny = __float_as_uint(S.inv.y) >> 31,
                   nz = __float_as_uint(S.inv.z) >> 31;
    if (__ballot(1) != ~0ull) return false;  // (every lane must be active: see above)
    const unsigned long long act = __ballot(part);
    const unsigned long long bx = __ballot(part && nx != 0u), by = __ballot(part && ny != 0u), bz = __ballot(part && nz != 0u);
    if (act == 0ull || (bx != 0ull && bx != act) || (by != 0ull && by != act) || (bz != 0ull && bz != act)) return false;
    const uint32_t shx = bx ? 16u : 0u, shy = by ? 16u : 0u, shz = bz ? 16u : 0u;
    float bt = Q.bt;
    int bc = Q.bc;
    uint32_t node = P.bvh_root;  // wave-uniform (SGPRs): the walk's node, stack depth and child words
    uint32_t stk = 0u, sp = 0u;  // the stack: lane k holds the k-th pending node
    typedef float f4v __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)P.bvh_sph, (short)0, (int)(P.bvh_nleaf * 16u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc((void*)P.bvh_slot, (short)0, (int)(P.bvh_nleaf * 4u), 0x00020000);
    while (true) {
        if (!(node & BVH_LEAF_BIT)) {
            float tl, tr;
            const uint4 c0 = hn[2 * node], c1 = hn[2 * node + 1];
            const bool hl = box_hit_so(c0.x, c0.y, c0.z, shx, shy, shz, S, bt, tl);
            const bool hr = box_hit_so(c1.x, c1.y, c1.z, shx, shy, shz, S, bt, tr);
            const uint32_t left = __builtin_amdgcn_readfirstlane(c0.w), right = __builtin_amdgcn_readfirstlane(c1.w);
            if constexpr (COUNT) tally.boxes += part ? 2u : 0u;
            const unsigned long long ml = __ballot(hl), mr = __ballot(hr);
            if ((ml | mr) != 0ull) {
                if (ml != 0ull && mr != 0ull) {
                    // the near child of most lanes first (lanes that enter one child only vote for it)
                    const unsigned long long vl = __ballot(hl && (!hr || tl <= tr));
                    const bool lf = 2u * (uint32_t)__popcll(vl) >= (uint32_t)__popcll(ml | mr);
                    stk = __lane_id() == sp ? (lf ? right : left) : stk;  // (no v_writelane builtin here)
                    sp++;
                    node = lf ? left : right;
                } else {
                    node = ml != 0ull ? left : right;
                }
                continue;
            }
        } else {
            // the ray from the lane's block entry (not held in registers through the walk)
            const float4 e0 = e[0], e1 = e[1];
            const Ray r = {mk(e0.x, e0.y, e0.z), mk(e0.w, e1.x, e1.y)};
            const float a = dot(r.d, r.d);
            const float a4 = 4.0f * a, a2 = 2.0f * a;
            const uint32_t first = (node >> 4) & 0x07FFFFFFu, cnt = node & 15u;
            for (uint32_t o = first * 16u, oe = (first + cnt) * 16u; o != oe; o += 16u) {
                const f4v v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o, 0, 0);
                const float t = exact_t_geo<true>(float4{v.x, v.y, v.z, v.w}, r, a4, a2);
                if (t > 0.0f && t <= bt) {  // beats(): a tie needs both slots (rare)
                    const int slot = (int)__builtin_amdgcn_raw_buffer_load_b32(rsl, (int)(o >> 2), 0, 0);
                    if (t < bt || (bc >= 0 && slot < bvh_slot_of(P, bc))) { bt = t; bc = (int)(o >> 4); }
                }
            }
            if constexpr (COUNT) tally.spheres += part ? cnt : 0u;
        }
        if (sp == 0u) break;
        sp--;
        node = __builtin_amdgcn_readlane(stk, sp);
    }
    Q.bt = bt;
    Q.bc = bc;
    return true;
}

// intersect_node (shader_tris.wgsl:150-159); inv = 1/d is the same value for every node of a query.
__device__ __forceinline__ bool node_slab(const float4 mn, const float4 mx, const f3& o, const f3& inv) {
    const float t0x = (mn.x - o.x) * inv.x, t0y = (mn.y - o.y) * inv.y, t0z = (mn.z - o.z) * inv.z;
    const float t1x = (mx.x - o.x) * inv.x, t1y = (mx.y - o.y) * inv.y, t1z = (mx.z - o.z) * inv.z;
    const float tmin = fmax_ieee(fmax_ieee(fmin_ieee(t0x, t1x), fmin_ieee(t0y, t1y)), fmin_ieee(t0z, t1z));
    const float tmax = fmin_ieee(fmin_ieee(fmax_ieee(t0x, t1x), fmax_ieee(t0y, t1y)), fmax_ieee(t0z, t1z));
    return tmin <= tmax && tmax >= 0.0f;
}
__device__ __forceinline__ bool node_hit(const KParams& P, uint32_t i, const f3& o, const f3& inv) {
    return node_slab(P.nodes[2 * i], P.nodes[2 * i + 1], o, inv);
}

// The top of the implicit heap in LDS (k_trace_split_tris<.., HL > 0>): nodes 1 .. HT - 1, copied once per
// workgroup. On Suzanne (C4, C5) the first eight levels take 72 % of the walk's node tests (the oracle's walk, by
// depth: 2 / 3 / 6 / 7 / 12 / 13 / 13 / 14 % for depths 0-7, 15 / 15 % for 8-9), and every ray starts at the root.
// Same node bytes, same test.

// Wave-uniform: a step reads LDS when every walking lane of the wave is inside the top, else every lane reads
// L1/L2 (C4 +5.6 %, C5 +4.3 % over no LDS top). Measured and not kept: lanes inside the top from LDS and the others
// from L1/L2 in the same step, merged by selects (C4 -4.6 %, C5 -2 %): the extra selects, and the wave still waits
// for the slowest load of the step. The nodes below the top are read through a buffer descriptor: plain global
// loads in the other arm get merged with the LDS loads into flat loads of a selected pointer.

// Sign-ordered node test (the heap-top kernels, HT > 0; tests/test_sign_ordered_slab.py). The nodes are laid out as
// (lo, hi, lo) per axis, 36 B per node, lo <= hi (renderer.cpp pack_nodes_so swaps padding / inverted axes: the
// reference's min / max take the pair in either order). Reading two floats at axis * 12 + 4 * (1/d < 0) gives the
// near plane, then the far one, so each axis needs no min / max:
//   max3(tnear) <= min3(tfar) && min3(tfar) >= 0  ==  intersect_node (shader_tris.wgsl:150-159)
// whenever 1/d and the origin are finite and no bound is NaN (with lo <= hi and a finite nonzero 1/d, RN keeps
// (lo - o) / d and (hi - o) / d in the order of the sign of 1/d, so min / max would pick exactly those two; zeros of
// either sign only reach comparisons). A wave with any non-finite 1/d or origin (a direction component of +-0 or
// below 2^-126: 0 x inf), or a tree with a NaN bound (KParams so_ok 0), uses the reference form on the same layout
// (lo, hi at axis * 12). 6 VALU fewer per node test for 3 address multiply-adds (the per-lane offsets ox, oy, oz).
constexpr uint32_t SO_NODE_BYTES = 36;
typedef __attribute__((address_space(3))) float lds_f32;
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ bool node_slab_so(const f2v x, const f2v y, const f2v z, const f3& o, const f3& inv) {
    const float tnx = (x.x - o.x) * inv.x, tny = (y.x - o.y) * inv.y, tnz = (z.x - o.z) * inv.z;
    const float tfx = (x.y - o.x) * inv.x, tfy = (y.y - o.y) * inv.y, tfz = (z.y - o.z) * inv.z;
    const float tmin = fmax_ieee(fmax_ieee(tnx, tny), tnz);
    const float tmax = fmin_ieee(fmin_ieee(tfx, tfy), tfz);
    return tmin <= tmax && tmax >= 0.0f;
}
__device__ __forceinline__ bool node_slab_lohi(const f2v x, const f2v y, const f2v z, const f3& o, const f3& inv) {
    return node_slab(float4{x.x, y.x, z.x, 0.0f}, float4{x.y, y.y, z.y, 0.0f}, o, inv);
}
__device__ __forceinline__ f2v lds_pair(uint32_t a) {
    return f2v{*(const lds_f32*)(uintptr_t)a, *(const lds_f32*)(uintptr_t)(a + 4u)};
}
__device__ __forceinline__ f2v buf_pair(__amdgpu_buffer_rsrc_t rs, uint32_t a) {
    typedef uint32_t u2v __attribute__((ext_vector_type(2)));
    const u2v v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)a, 0, 0);
    return f2v{__uint_as_float(v.x), __uint_as_float(v.y)};
}

// nodes_so based at -tb (the LDS top's byte addresses reach the same node), from fresh scalar loads (four SGPRs held
// across the walk spilled in the C5 kernel)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t so_rsrc(uint32_t tb) {
    const KPtr K = kargs();
    return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)K->nodes_so - tb), (short)0,
                                             (int)(K->n * SO_NODE_BYTES + tb), 0x00020000);
}

// Node i through the sign-ordered layout: from the LDS top (nodes 0 .. HT - 1, byte address tb + i * 36) when every
// walking lane of the wave is inside it, else through nodes_so (so_rsrc: the same byte addresses). The pairs at
// ox / oy / oz (+ i * 36): SO, tb + axis * 12 + 4 * (1/d < 0), near then far; else tb + axis * 12, lo then hi, tested
// with the reference's min / max. (One loop with a wave-uniform branch between the two tests, instead of two
// instantiations of the walk, measured C4 -1.5 %, C5 -1.2 %.)
template <uint32_t HT, bool SO, bool FULL = false>
__device__ __forceinline__ bool node_hit_so(uint32_t i, const f3& o, const f3& inv, uint32_t tb, uint32_t ox, uint32_t oy,
                                            uint32_t oz) {
    const bool lds = FULL || __ballot(i >= HT) == 0ull;  // FULL: every internal node is in the top (n <= HT)
    const uint32_t ax = __umul24(i, SO_NODE_BYTES) + ox, ay = __umul24(i, SO_NODE_BYTES) + oy,
                   az = __umul24(i, SO_NODE_BYTES) + oz;
    if constexpr (SO) {
        if (lds) return node_slab_so(lds_pair(ax), lds_pair(ay), lds_pair(az), o, inv);
        const __amdgpu_buffer_rsrc_t rs = so_rsrc(tb);
        return node_slab_so(buf_pair(rs, ax), buf_pair(rs, ay), buf_pair(rs, az), o, inv);
    } else {
        if (lds) return node_slab_lohi(lds_pair(ax), lds_pair(ay), lds_pair(az), o, inv);
        const __amdgpu_buffer_rsrc_t rs = so_rsrc(tb);
        return node_slab_lohi(buf_pair(rs, ax), buf_pair(rs, ay), buf_pair(rs, az), o, inv);
    }
}

// intersect_triangle, Moller-Trumbore (shader_tris.wgsl:161-202): the candidate t, or -1 when the
// determinant, u or v test rejects (the t >= 1e-4 and t < best tests are the caller's).
__device__ __forceinline__ float tri_t(const Ray& r, const TriDev& tr) {
    const f3 e1 = mk(tr.e1.x, tr.e1.y, tr.e1.z);
    const f3 e2 = mk(tr.e2.x, tr.e2.y, tr.e2.z);
    const f3 hh = cross(r.d, e2);
    const float det = dot(e1, hh);
    if (__builtin_fabsf(det) < 1e-4f) return -1.0f;
    // = 1.0f / det (rcp_rn_mid: |det| >= 1e-4 here unless NaN, which takes the division)
    float inv_det = rcp_rn_mid(det);
    if (__builtin_expect(!(__builtin_fabsf(det) <= 0x1p60f), 0)) inv_det = 1.0f / det;
    const f3 s = r.o - mk(tr.a.x, tr.a.y, tr.a.z);
    const float u = inv_det * dot(s, hh);
    if (u < 0.0f || u > 1.0f) return -1.0f;
    const f3 q = cross(s, e1);
    const float v = inv_det * dot(r.d, q);
    if (v < 0.0f || u + v > 1.0f) return -1.0f;
    return inv_det * dot(e2, q);
}

__device__ __forceinline__ void tri_record(const KParams& P, const Ray& r, const TriDev& tr, float t, Hit& h) {
    const MatDev m = P.mats[tr.material];
    h.p = point_on_ray(r.o, r.d, t);
    h.n = mk(tr.nx, tr.ny, tr.nz);
    h.t = t;
    h.ar = m.ar; h.ag = m.ag; h.ab = m.ab; h.param = m.param;
    h.id = (tr.material << 3) | (m.id == 1u || m.id == 2u ? m.id : 0u);
    h.front = dot(h.n, r.d) > 0.0f;
}

#ifndef HRT_TRI_NESTED
#define HRT_TRI_NESTED 1
#endif
// The reference's per-leaf update: accept t in [1e-4, best). The walks only track (best, bj); the hit
// record is built once for the winner (closest_hit), which keeps fewer registers live during the walk.
template <bool TBUF = false>
__device__ __forceinline__ void tri_test(const KParams& P, const Ray& r, uint32_t j, float& best, int& bj) {
    TriDev tr;
    if constexpr (TBUF) {
#ifndef HRT_TRI_GEO
#define HRT_TRI_GEO 1
#endif
#if HRT_TRI_GEO
        // a, e1, e2 from the compact 36-B operand array (tri_geo) through buffer loads at 32-bit offsets
        typedef uint32_t u3v __attribute__((ext_vector_type(3)));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)P.tri_geo, (short)0, (int)(P.m * 36u), 0x00020000);
        const u3v a = __builtin_amdgcn_raw_buffer_load_b96(rs, (int)(j * 36u), 0, 0);
        const u3v e1 = __builtin_amdgcn_raw_buffer_load_b96(rs, (int)(j * 36u + 12u), 0, 0);
        const u3v e2 = __builtin_amdgcn_raw_buffer_load_b96(rs, (int)(j * 36u + 24u), 0, 0);
        tr.a = float4{__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z), 0.0f};
        tr.e1 = float4{__uint_as_float(e1.x), __uint_as_float(e1.y), __uint_as_float(e1.z), 0.0f};
        tr.e2 = float4{__uint_as_float(e2.x), __uint_as_float(e2.y), __uint_as_float(e2.z), 0.0f};
#else
        // a, e1, e2 through buffer loads at 32-bit offsets (no 64-bit address per triangle)
        typedef float f4v __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)P.tris, (short)0, (int)(P.m * 64u), 0x00020000);
        const f4v a = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(j * 64u), 0, 0);
        const f4v e1 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(j * 64u + 16u), 0, 0);
        const f4v e2 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(j * 64u + 32u), 0, 0);
        tr.a = float4{a.x, a.y, a.z, a.w};
        tr.e1 = float4{e1.x, e1.y, e1.z, e1.w};
        tr.e2 = float4{e2.x, e2.y, e2.z, e2.w};
#endif
    } else {
        tr = P.tris[j];
    }
#if HRT_TRI_NESTED
    // tri_t's tests as nested branches (no -1 sentinel carried to a merge: its moves and select per triangle)
    const f3 e1 = mk(tr.e1.x, tr.e1.y, tr.e1.z);
    const f3 e2 = mk(tr.e2.x, tr.e2.y, tr.e2.z);
    const f3 hh = cross(r.d, e2);
    const float det = dot(e1, hh);
    if (__builtin_fabsf(det) < 1e-4f) return;
    float inv_det = rcp_rn_mid(det);
    if (__builtin_expect(!(__builtin_fabsf(det) <= 0x1p60f), 0)) inv_det = 1.0f / det;
    const f3 s = r.o - mk(tr.a.x, tr.a.y, tr.a.z);
    const float u = inv_det * dot(s, hh);
    if (u < 0.0f || u > 1.0f) return;
    const f3 q = cross(s, e1);
    const float v = inv_det * dot(r.d, q);
    if (v < 0.0f || u + v > 1.0f) return;
    const float t = inv_det * dot(e2, q);
#else
    const float t = tri_t(r, tr);
#endif
    if (t >= 1e-4f && t < best) {
        best = t;
        bj = (int)j;
    }
}

// intersect_all_node (shader_tris.wgsl:268-301): stackless DFS over the implicit heap, 600-step cap.
// The walk's path never depends on hits (intersect_node has no best-t test), so the triangle tests of
// the leaves it reaches are deferred into a per-lane list (`cand`, LDS, stride 256) and run in batches:
// whenever some lane's list is full, every active lane tests its pending triangles, in the order reached
// (= the reference's sequential `t >= best` rule, so the same winner). The walk loop then carries only
// node tests, and triangle tests run with most lanes active instead of one divergent branch per step.
constexpr uint32_t TRI_BATCH = 16;  // measured on C4: 4 -> 5.89, 8 -> 6.28, 16 -> 6.38 Grays/s

// The walk is split for k_trace_split_tris: heap_begin / heap_run (suspendable: returns false once fewer than
// `below` lanes of the wave are still walking, after a flush, so no deferred triangle is pending) with the walk
// state in HeapWalk; walk_bvh runs it to completion (k_trace, k_render).
struct HeapWalk {
    f3 inv;           // 1 / d, the value intersect_node recomputes per node
    uint32_t i, step;
    float best;       // starts at the sphere winner's t (triangles must beat it: `t >= best` rejects)
    int bj;           // winning triangle (-1: none)
};

// FAST: 1 / d per component by the refined reciprocals when every |d| lies in [2^-60, 2^60] (rcp_exact), else the
// IEEE divisions; the same bits. (Measured: C4 +0.2 % on top of the refined 1/det; C5 -0.4 %, so its kernel keeps
// the divisions.)
template <bool FAST = true>
__device__ __forceinline__ void heap_begin(const Ray& r, float best, HeapWalk& W) {
    if constexpr (FAST) {
        const float lo = fmin_ieee(fmin_ieee(__builtin_fabsf(r.d.x), __builtin_fabsf(r.d.y)), __builtin_fabsf(r.d.z));
        const float hi = fmax_ieee(fmax_ieee(__builtin_fabsf(r.d.x), __builtin_fabsf(r.d.y)), __builtin_fabsf(r.d.z));
        W.inv = mk(rcp_rn_mid(r.d.x), rcp_rn_mid(r.d.y), rcp_rn_mid(r.d.z));
        const bool slow = !(lo >= 0x1p-60f && hi <= 0x1p60f);
        if (__builtin_expect(__ballot(slow) != 0ull, 0)) {  // (a wave-uniform branch, as sqrt_exact_u)
            if (slow) W.inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
        }
    } else {
        W.inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
    }
    W.i = 1u;
    W.step = 0u;
    W.best = best;
    W.bj = -1;
}

// Leaf pairs. A bottom node i (n/2 <= i < n) has the leaves 2i and 2i + 1 as children, and when the reference's
// walk hits it, its next two loop bodies are exactly those leaves (2i is even, so the walk steps to 2i + 1), after
// which it climbs from 2i + 1, i.e. from i: (2i + 1) >> ctz(~(2i + 1)) = i >> ctz(~i). So one loop iteration here
// is one node test, and a hit bottom node appends both its leaves to the deferred list as one entry (j0 = 2i - n,
// PAIR_BIT when j0 + 1 is a triangle too) and advances the step count by the two leaf bodies. Every iteration runs
// the same node test: no lane sits out a leaf body while the others test nodes (the per-step leaf branch was
// 17 % of C4's walk steps). Visits, the order of the triangle tests, the 600-step cap (a leaf body the cap cuts
// off is not run) and the walk's end at the first leaf j >= m are the reference's; so are the node and triangle
// counts.
constexpr uint32_t PAIR_BIT = 0x80000000u;

// HT: nodes 1 .. HT - 1 of the heap are in LDS (`top`; 0 = none); LS: lanes per workgroup, the stride of the
// lane's list words (`cand` = this lane's first word; entry k at cand[k * LS]); CAP: list entries per lane.
// (The node count is not kept per iteration: every iteration adds one node test and one step, a pair two steps and
// two triangles, and an append that ends the walk one of each, so the run's node tests are its steps less its
// triangles.)
typedef __attribute__((address_space(3))) uint32_t lds_u32;  // 32-bit LDS addressing for the list

template <bool SUSPEND, uint32_t HT = 0, uint32_t LS = 256, uint32_t CAP = TRI_BATCH, bool TBUF = false, bool SO = false,
          bool FULL = false>
__device__ __forceinline__ bool heap_run(const KParams& P, const Ray& r, HeapWalk& W, Tally& tally, uint32_t* cand_g,
                                         uint32_t below, const float* __restrict__ top = nullptr) {
    // the list's LDS byte address (32-bit arithmetic): entry k at c0 + k * 4 LS
    const uint32_t c0 = (uint32_t)(uintptr_t)(lds_u32*)cand_g;
    const f3 inv = W.inv;
    // HT > 0: the sign-ordered layout (node_hit_so), LDS top at byte address tb
    uint32_t tb = 0u, ox = 0u, oy = 0u, oz = 0u;
    if constexpr (HT > 0) {
        tb = (uint32_t)(uintptr_t)(const lds_f32*)top;
        const uint32_t sm = SO ? 4u : 0u;  // (the sign offsets only with the sign-ordered test)
        ox = tb + ((__float_as_uint(inv.x) >> 29) & sm);
        oy = tb + 12u + ((__float_as_uint(inv.y) >> 29) & sm);
        oz = tb + 24u + ((__float_as_uint(inv.z) >> 29) & sm);
    }
    const uint32_t n = P.n, m = P.m;
    uint32_t i = W.i, step = W.step, nc = 0u;
    const uint32_t step0 = step, tris0 = tally.tris;
    uint32_t walking = 1u;  // an integer, not an i1 lane mask (see bvh_run)
    float best = W.best;
    int bj = W.bj;
    if (i >= n) {  // n == 1: the root is leaf 0, the walk's only body (heap_begin starts every walk at i = 1)
        if (m != 0u) {
            tally.tris++;
            step++;
            *(lds_u32*)(uintptr_t)c0 = 0u;
            nc = 1u;
        }
        walking = 0u;
    }
    while (true) {
        while (walking != 0u && __ballot(nc == CAP) == 0ull) {
            step++;
            asm volatile("" : "+v"(step));  // the branches below add to this value, not to the last trip's
            bool hit;
            if constexpr (HT > 0) hit = node_hit_so<HT, SO, FULL>(i, r.o, inv, tb, ox, oy, oz);
            else hit = node_hit(P, i, r.o, inv);
            const bool down = hit && 2u * i < n;
            if (hit && !down) {  // bottom node: the leaf bodies 2i, 2i + 1
                const uint32_t j0 = 2u * i - n;
                if (j0 + 2u <= m && step <= 598u) {
                    tally.tris += 2u;
                    *(lds_u32*)(uintptr_t)(c0 + __umul24(nc, 4u * LS)) = j0 | PAIR_BIT;
                    nc++;
                    step += 2u;
                } else {  // the cap or the end of the triangles cuts the pair (once per walk at most)
                    walking = 0u;  // this walk ends within the two leaf bodies (the cap, or j >= m: break)
                    if (step < 600u && j0 < m) {
                        tally.tris++;
                        step++;
                        *(lds_u32*)(uintptr_t)(c0 + __umul24(nc, 4u * LS)) = j0;
                        nc++;
                    }
                }
            }
            const uint32_t ip1 = i + 1u;
            const uint32_t up = ip1 >> __builtin_ctz(ip1);  // while (i & 1) i /= 2; i++ (1: i was 2^k - 1, the end)
            if (!down && up == 1u) walking = 0u;
            i = down ? 2u * i : up;
            if (step >= 600u) walking = 0u;  // the reference's step cap
        }
        for (uint32_t k = 0; k < nc; k++) {  // in the order reached
            const uint32_t e = *(const lds_u32*)(uintptr_t)(c0 + __umul24(k, 4u * LS));
            const uint32_t j = e & ~PAIR_BIT;
            tri_test<TBUF>(P, r, j, best, bj);
            if (e & PAIR_BIT) tri_test<TBUF>(P, r, j + 1u, best, bj);
        }
        nc = 0u;
        if (walking == 0u) break;
        if constexpr (SUSPEND) {
            if ((uint32_t)__popcll(__ballot(1)) < below) break;
        }
    }
    tally.nodes += (step - step0) - (tally.tris - tris0);
    W.i = i;
    W.step = step;
    W.best = best;
    W.bj = bj;
    return walking == 0u;
}

__device__ __forceinline__ void walk_bvh(const KParams& P, const Ray& r, float& best, int& bj, Tally& tally,
                                         uint32_t* cand) {
    HeapWalk W;
    heap_begin(r, best, W);
    heap_run<false>(P, r, W, tally, cand, 0u);
    best = W.best;
    bj = W.bj;
}

// Opt-in triangle walk (rt_params.tri_bvh = 1; host/tri_bvh.hpp): an ordered, culling stack walk of a
// binned-SAH BVH2 with the same Moller-Trumbore arithmetic, keeping the (t, triangle index)
// lexicographic minimum — the winner of the reference's ordered walk, which reaches leaves in increasing
// index and keeps the first of equal t (a sphere hit of the mixed program keeps ties, as there). Boxes
// are padded by 2^-12 of the distance scale of the query. Not parity-exact by contract:
// the reference's 600-step cap and unpadded slab tests can drop a triangle this walk finds. A stack
// overflow falls back to the reference walk.
constexpr int TRI_STACK = 24;

// (the SAH tree's constants are read through kargs() where they are used, not held in SGPRs across the persistent
// loop: the mixed kernels with this walk spilled 2-10 SGPRs otherwise)
__device__ __forceinline__ void walk_sah(const KParams& /*P*/, const Ray& r, float& best, int& bj, Tally& tally,
                                         uint32_t* stack) {
    const KPtr P = kargs();
    const f3 op = mk(r.o.x - P->tb_rc[0], r.o.y - P->tb_rc[1], r.o.z - P->tb_rc[2]);
    const float D = __builtin_amdgcn_sqrtf(dot(op, op)) * 1.001f + P->tb_rr_h;
    const float pad = D * 0x1p-12f;
    Slab S;
    S.inv = mk(robust_inv(r.d.x), robust_inv(r.d.y), robust_inv(r.d.z));
    S.lo = mk(-op.x - pad, -op.y - pad, -op.z - pad);
    S.hi = mk(-op.x + pad, -op.y + pad, -op.z + pad);
    S.lo = S.lo * S.inv;
    S.hi = S.hi * S.inv;
    uint32_t node = P->tb_root;  // bj: index of the best triangle (-1: none, or the best is a sphere)
    int sp = 0;
    uint32_t overflow = 0u;  // an integer, not an i1 lane mask (see bvh_run)
    while (true) {
        if (!(node & BVH_LEAF_BIT)) {
            float4 n0, n1, n2, n3;
            load_hnode(P->tb_hnodes, node, n0, n1, n2, n3);
            float tl, tr;
            const bool hl = padded_box_hit(n0, n1, S, best, tl);
            const bool hr = padded_box_hit(n2, n3, S, best, tr);
            tally.nodes += 2;
            const uint32_t left = __float_as_uint(n0.w), right = __float_as_uint(n2.w);
            if (hl && hr) {
                const bool lfirst = tl <= tr;
                if (sp < TRI_STACK) {
                    stack[sp * 256] = lfirst ? right : left;
                    sp++;
                } else {
                    overflow = 1u;
                }
                node = lfirst ? left : right;
                continue;
            }
            if (hl) { node = left; continue; }
            if (hr) { node = right; continue; }
        } else {
            const uint32_t first = (node >> 4) & 0x07FFFFFFu, cnt = node & 15u;
            for (uint32_t k = 0; k < cnt; k++) {
                const uint32_t j = P->tb_order[first + k];
                const float t = tri_t(r, P->tris[j]);
                tally.tris++;
                if (t >= 1e-4f && (t < best || (t == best && bj >= 0 && (int)j < bj))) {
                    best = t;
                    bj = (int)j;
                }
            }
        }
        if (sp == 0) break;
        node = stack[(--sp) * 256];
    }
    if (overflow != 0u) {  // a dropped subtree: finish with the lexicographic minimum over every triangle
        for (uint32_t j = 0; j < P->m; j++) {
            const float t = tri_t(r, P->tris[j]);
            if (t >= 1e-4f && (t < best || (t == best && bj >= 0 && (int)j < bj))) {
                best = t;
                bj = (int)j;
            }
        }
        tally.tris += P->m;
    }
}

template <int MODE, int SCAN, bool TSAH = false, bool U = false>  // U: sphere_record_p<U>
__device__ __forceinline__ bool closest_hit(const KParams& P, const Ray& r, Hit& h, void* lds, Tally& tally,
                                            uint32_t* tri_cand, uint32_t* tri_stack) {
    float best = FLT_MAX_REF;
    int bi = -1, bj = -1;  // winning sphere slot / triangle index
    if (MODE != MODE_TRIS) {
        if constexpr (SCAN == SCAN_BVH) {
            // (with the SAH triangle walk the sphere walk's rare-path constants are read through kargs(): 0 SGPR spills)
            bi = scan_spheres_bvh<BVH_STACK, true, 256, TSAH>(P, r, best, (uint32_t*)lds, tally);
        } else if constexpr (SCAN == SCAN_DEFER) {
            bi = scan_spheres_deferred(P, r, best, (uint16_t*)lds);
            tally.spheres += P.nslots;
        } else {
            bi = scan_spheres(P, r, best);
            tally.spheres += P.nslots;
        }
    }
    if (MODE != MODE_SPHERE) {  // triangles after spheres, `t >= best` rejected: ties keep the sphere
        if constexpr (TSAH) walk_sah(P, r, best, bj, tally, tri_stack);
        else walk_bvh(P, r, best, bj, tally, tri_cand);
    }
    // every accepted t is < FLT_MAX_REF, so `abs(hit.t - FLT_MAX) < EPSILON` (shader_sphere.wgsl:235) is
    // "nothing accepted"
    if (bj >= 0) {
        tri_record(P, r, P.tris[bj], best, h);
        return true;
    }
    if (bi >= 0) {
        sphere_record<U>(P, r, bi, best, h);
        return true;
    }
    h.t = FLT_MAX_REF;
    return false;
}

// random_on_hemisphere (shader_sphere.wgsl:107-117): normalised vector in the +++ octant, flipped to n's side.
template <int MODE>
__device__ __forceinline__ f3 random_on_hemisphere(uint32_t& s, const f3& n) {
    constexpr float EPS = MODE == MODE_SPHERE ? 1e-6f : 1e-4f;
    const float x = rng_float(s);
    const float y = rng_float(s);
    const float z = rng_float(s);
    // normalize() with the range-restricted exact sequences (rt_device.hpp normalize_rng): 30 instead of 52 VALU
    const f3 v = normalize_rng(mk(x, y, z));
    // `length(v) < EPSILON` (:110) never holds here, so it is not evaluated: x, y, z are rng floats in
    // [0, 1]; either all are 0 (v = NaN, and NaN < EPS is false) or the largest is >= 2^-32, dot(v, v) is a
    // normal float and the normalised v has length >= 0.577. The oracle keeps the test; parity compares.
    (void)EPS;
    if (dot(v, n) > 0.0f) return v;
    return -v;
}

// scatter (shader_sphere.wgsl:172-217; shader_tris.wgsl:222-267 reflects the raw direction for metal).
// The three material arms share code so a wave holding several materials runs one hemisphere sample and
// one final normalize instead of one per arm; every lane still performs exactly its own arm's operations
// (and RNG draws) in the reference's order, so results are unchanged.
template <int MODE, bool U = false>  // U (sphere program): the exact sequences' guards as wave-uniform branches
__device__ __forceinline__ void scatter(const KParams& P, uint32_t& s, Ray& r, const Hit& h) {
    const bool lambert = (h.id & 3u) == 1u, metal = (h.id & 3u) == 2u;
    f3 hemi = mk(0.0f, 0.0f, 0.0f);
    if (lambert || metal) hemi = random_on_hemisphere<MODE>(s, h.n);  // 3 draws, both arms
    f3 u = hemi;
    if (metal) {
        const f3 in = MODE == MODE_SPHERE ? (U ? normalize_exact_u(r.d) : normalize_exact(r.d)) : r.d;
        u = reflect(in, h.n) + h.param * hemi;
    } else if (!lambert) {  // MAT_DIELECTRIC and the default arm
        // ir = front ? 1 / param : param, and reflectance's r0 * r0 for that ir, from the host (DielConsts)
        const float* dc = (MODE == MODE_SPHERE || (MODE != MODE_TRIS && (h.id & 4u))) ? &P.sph_aux[h.id >> 3].inv_param
                                                                                     : &P.mats[h.id >> 3].inv_param;
        const float ir = h.front ? dc[0] : h.param;
        const float cos_t = fmin_ieee(dot(-r.d, h.n), 1.0f);
        const float sin_t = MODE == MODE_SPHERE ? (U ? sqrt_exact_u(1.0f - cos_t * cos_t) : sqrt_exact(1.0f - cos_t * cos_t))
                                                : __builtin_sqrtf(1.0f - cos_t * cos_t);
        bool refl = ir * sin_t > 1.0f;  // cannot_refract; WGSL || short-circuits the RNG draw
        if (!refl) {
            const float f = rng_float(s);
            refl = reflectance_r0sq(cos_t, h.front ? dc[1] : dc[2]) > (f - __builtin_floorf(f));
        }
        u = refl ? reflect(r.d, h.n) : refract<MODE == MODE_SPHERE, U>(r.d, h.n, ir);
    }
    r.o = h.p;
    // (the triangle / mixed kernels keep the IEEE form: the fast one costs them spills)
    r.d = lambert ? hemi : (MODE == MODE_SPHERE ? (U ? normalize_exact_u(u) : normalize_exact(u)) : normalize(u));
}

// (a, b) / sqrt(fma(b, b, a * a)) for two rng floats (each 0 or in [2^-32, 1]; the AA jitter and the disk direction
// of make_ray): the fast correctly rounded sqrt / division sequences (rt_device.hpp, ranges as normalize_rng) unless
// both are 0 (0 / 0: the IEEE operations give the reference's NaN); bit-identical either way. FAST false: IEEE.
template <bool FAST>
__device__ __forceinline__ void div_by_len_rng(float a, float b, float& qa, float& qb) {
    const float d = __builtin_fmaf(b, b, a * a);
    if (FAST && d >= 0x1p-100f) {  // not both 0: d in [2^-64, 2], the length in [2^-32, 1.5]
        const RcpRN r = rcp_rn_setup(sqrt_rn_mid(d));
        qa = div_rn_mid(a, r);
        qb = div_rn_mid(b, r);
    } else {
        const float l = __builtin_sqrtf(d);
        qa = a / l;
        qb = b / l;
    }
}

// x / l for make_ray's px / wm1 and py / hm1: FAST (sphere program), div_rn_mid with the host's correctly rounded
// 1 / l where l (inv != 0) and x lie in its range [2^-60, 2^60] (x = pixel + 0.5 + jitter >= 0.5; a NaN jitter takes
// the division); else the IEEE division. Bit-identical either way.
template <bool FAST>
__device__ __forceinline__ float div_cam(float x, float l, float inv) {
    if (FAST && inv != 0.0f && x >= 0x1p-60f && x <= 0x1p60f) return div_rn_mid(x, RcpRN{l, inv});
    return x / l;
}

// fs_main prologue + make_ray (shader_sphere.wgsl:253-258, :123-135; shader_tris.wgsl:136-148).
// FASTRNG: the jitter / disk / px, py divisions by the fast exact sequences (the sphere program everywhere; the other
// programs' split kernels, whose frame-block refill has the registers for them — k_render<2, 4, false> spilled)
// div_by_len_rng<true> / div_cam<true> with their guards as one wave-uniform branch (as sqrt_exact_u): the same bits
__device__ __forceinline__ void div_by_len_rng_u(float a, float b, float& qa, float& qb) {
    const float d = __builtin_fmaf(b, b, a * a);
    const RcpRN r = rcp_rn_setup(sqrt_rn_mid(d));
    qa = div_rn_mid(a, r);
    qb = div_rn_mid(b, r);
    const bool slow = !(d >= 0x1p-100f);
    if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
        if (slow) div_by_len_rng<false>(a, b, qa, qb);
    }
}
__device__ __forceinline__ float div_cam_u(float x, float l, float inv) {
    float q = div_rn_mid(x, RcpRN{l, inv});
    const bool slow = !(inv != 0.0f && x >= 0x1p-60f && x <= 0x1p60f);
    if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
        if (slow) q = x / l;
    }
    return q;
}

// U (sphere program, FASTRNG): the guards of the fast sequences as wave-uniform branches (k_trace's frame block, C2:
// +0.9 %, profiles/r06/leaf_defer/ab_c2_uniform_guards_primary.txt; k_trace_split's measured -0.45 %,
// ab_c3_uniform_guards_primary.txt)
template <int MODE, bool FASTRNG = (MODE == MODE_SPHERE), bool U = false>
__device__ __forceinline__ Ray primary_ray(CamPtr C, uint32_t x, uint32_t y, uint32_t time, uint32_t& s) {
    static_assert(!U || (FASTRNG && MODE == MODE_SPHERE), "uniform guards: the sphere program's fast sequences");
    s = (x * C->H + y) * time;
    const float r1 = rng_float(s);
    const float r2 = rng_float(s);
    float j1, j2;
    if constexpr (U) div_by_len_rng_u(r1, r2, j1, j2);
    else div_by_len_rng<FASTRNG>(r1, r2, j1, j2);
    const float px = ((float)x + 0.5f) + j1;
    const float py = ((float)y + 0.5f) + j2;
    const float ux = (2.0f * (U ? div_cam_u(px, C->wm1, C->inv_wm1) : div_cam<FASTRNG>(px, C->wm1, C->inv_wm1)) - 1.0f) * C->aspect;
    const float uy = (2.0f * (U ? div_cam_u(py, C->hm1, C->inv_hm1) : div_cam<FASTRNG>(py, C->hm1, C->inv_hm1)) - 1.0f) * -1.0f;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = ((C->right[i] * ux) * C->k + (C->up[i] * uy) * C->k) + C->dir[i];
    const float dv = __builtin_fmaf(v[3], v[3], __builtin_fmaf(v[2], v[2], __builtin_fmaf(v[1], v[1], v[0] * v[0])));
    float vn[4];
    // sphere program: v / |v| by the fast sequences where |v0..2| lie in [2^-40, 2^40] and |v3| <= 2^40 (dv, the
    // length and the quotients inside their ranges, as normalize_exact); v[3] / |v| is unused there (f4[3])
    const float vlo = fmin_ieee(fmin_ieee(__builtin_fabsf(v[0]), __builtin_fabsf(v[1])), __builtin_fabsf(v[2]));
    const float vhi = fmax_ieee(fmax_ieee(__builtin_fabsf(v[0]), __builtin_fabsf(v[1])),
                                fmax_ieee(__builtin_fabsf(v[2]), __builtin_fabsf(v[3])));
    if constexpr (U) {
        const float lv = sqrt_rn_mid(dv);
        const RcpRN rl = rcp_rn_setup(lv);
#pragma unroll
        for (int i = 0; i < 3; i++) vn[i] = div_rn_mid(v[i], rl);
        vn[3] = 0.0f;  // (unused by the sphere program: f4[3] is not read)
        const bool slow = !(vlo >= 0x1p-40f && vhi <= 0x1p40f);
        if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
            if (slow) {
                const float l = __builtin_sqrtf(dv);
#pragma unroll
                for (int i = 0; i < 3; i++) vn[i] = v[i] / l;
            }
        }
    } else if (MODE == MODE_SPHERE && vlo >= 0x1p-40f && vhi <= 0x1p40f) {
        const float lv = sqrt_rn_mid(dv);
        const RcpRN rl = rcp_rn_setup(lv);
#pragma unroll
        for (int i = 0; i < 3; i++) vn[i] = div_rn_mid(v[i], rl);
        vn[3] = v[3] / lv;
    } else {
        const float lv = __builtin_sqrtf(dv);
#pragma unroll
        for (int i = 0; i < 4; i++) vn[i] = v[i] / lv;
    }
    float f4[4];
#pragma unroll
    for (int i = 0; i < 4; i++) f4[i] = C->eye[i] + vn[i] * C->focal;
    // random_on_disk (:118-122): +x,+y quadrant unit vector times rng*radius, in world xy.
    const float q1 = rng_float(s);
    const float q2 = rng_float(s);
    float e1, e2;
    if constexpr (U) div_by_len_rng_u(q1, q2, e1, e2);
    else div_by_len_rng<FASTRNG>(q1, q2, e1, e2);
    const float rr = rng_float(s) * C->blur;
    float o4[4];
    o4[0] = C->eye[0] + e1 * rr;
    o4[1] = C->eye[1] + e2 * rr;
    o4[2] = C->eye[2] + 0.0f * rr;
    o4[3] = C->eye[3] + 1.0f;
    Ray r;
    r.o = mk(o4[0], o4[1], o4[2]);
    if (MODE == MODE_SPHERE) {
        r.d = mk(f4[0] - o4[0], f4[1] - o4[1], f4[2] - o4[2]);
    } else {
        float g[4];
#pragma unroll
        for (int i = 0; i < 4; i++) g[i] = f4[i] - o4[i];
        const float lg = __builtin_sqrtf(__builtin_fmaf(g[3], g[3], __builtin_fmaf(g[2], g[2], __builtin_fmaf(g[1], g[1], g[0] * g[0]))));
        r.d = mk(g[0] / lg, g[1] / lg, g[2] / lg);
    }
    return r;
}

// Per-lane LDS lists of a 256-lane workgroup (lane stride 256): the sphere scan's candidate list or
// stack, and the triangle program's deferred-triangle list, which is also the opt-in SAH walk's stack
// (never live together). The triangle list aliases the sphere BVH stack, free again once the sphere scan
// has returned; the u16 candidate list of the deferred scan cannot be aliased (its lane stride differs,
// so one wave's entries would overlap another wave's).
struct LaneLists {
    void* sphere;
    uint32_t* tri;
};

template <int MODE, int SCAN>
__device__ __forceinline__ LaneLists lane_lists() {
    LaneLists L{nullptr, nullptr};
    constexpr int TRI_WORDS = (int)TRI_BATCH > TRI_STACK ? (int)TRI_BATCH : TRI_STACK;
    if constexpr (SCAN == SCAN_DEFER) {
        __shared__ uint16_t cand[(CAND_CAP + 1) * 256];
        L.sphere = cand + threadIdx.x;
        if constexpr (MODE != MODE_SPHERE) {
            __shared__ uint32_t tri_list_d[TRI_WORDS * 256];
            L.tri = tri_list_d + threadIdx.x;
        }
    } else if constexpr (SCAN == SCAN_BVH) {
        constexpr int WORDS = MODE == MODE_SPHERE || BVH_STACK >= TRI_WORDS ? BVH_STACK : TRI_WORDS;
        __shared__ uint32_t bvh_stack[WORDS * 256];
        L.sphere = bvh_stack + threadIdx.x;
        L.tri = bvh_stack + threadIdx.x;
    } else if constexpr (MODE != MODE_SPHERE) {
        __shared__ uint32_t tri_list[TRI_WORDS * 256];
        L.tri = tri_list + threadIdx.x;
    }
    return L;
}

// ---- The fold ring (sample queue) ----
// A job is one 8x8 tile x job_frames frames, taken by ONE wave from the queue; a tile's jobs are dealt one
// after another (tile-major), so they run at once on neighbouring waves. A job takes a ring slot from a free
// queue when it is dealt (job j takes the (j - ring_jobs)-th returned slot, so slots go out in job order and a
// job never waits on a later one), and each sample's colour goes to its job's slot (frame-major, 16 B per
// pixel) as a write-through (sc1) store. A wave tracks
// its jobs (WaveJobs); when every sample of one has been stored it drains its stores (s_waitcnt vmcnt(0)), sets
// the job's bit in the tile's done mask and tries the tile's fold lock. The lock holder folds the tile's jobs
// in order, as far as they are done, into the image (the expression of k_render, frame by frame; sc1 loads and
// stores), returns their slots, releases the lock and re-checks the mask (a job that completed meanwhile found
// the lock taken and left its fold to the holder). So folding trails each tile's slowest job by one job's fold,
// memory is O(jobs in flight) instead of O(frames x pixels), and there is no separate fold pass.
// Hand-off form: MI355X_MICROARCH.md § visibility, row 1 of the sc1 table (the storing unit is the wave, which
// drains before its atomic; the consumer learns by the value an atomic returned; every load of handed-off
// bytes, slot or image, is an sc1 load).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ring_rsrc() {
    const KPtr K = kargs();
    return __builtin_amdgcn_make_buffer_rsrc((void*)K->ring, (short)0, (int)K->ring_bytes, 0x00020000);
}

// Free-queue entry of return m (m-th slot returned; taken by job ticket m + ring_jobs): the slot, the lap of the
// queue (4 x ring_jobs entries) it was written in, valid bit. A waiting job polls its entry every round, so the
// entry is taken long before return m + 4 ring_jobs overwrites it (an overwrite is detected, never misread).
__device__ __forceinline__ uint32_t ring_q_entry(uint32_t slot, uint32_t m, uint32_t ring_log2) {
    return slot | ((((m >> (ring_log2 + 2u)) + 1u) & 0x7FFu) << 20) | 0x80000000u;
}

// Byte offset of (slot, frame within the job, pixel) in the ring.
__device__ __forceinline__ uint32_t ring_off(uint32_t slot, uint32_t fj, uint32_t px, uint32_t jf_log2) {
    return (((slot << jf_log2) + fj) << 10) | (px << 4);
}

// Per-tile fold word (64 bits): bit c = job c has all its samples stored (c < 48), bits 48-54 = jobs folded
// (the cursor), bit 63 = fold lock.
constexpr unsigned long long TF_LOCK = 1ull << 63;
constexpr uint32_t TF_CURSOR_SHIFT = 48;  // (jobs per tile and launch <= FOLD_MAX_JOBS, rt_device.hpp)
static_assert(FOLD_MAX_JOBS <= TF_CURSOR_SHIFT, "done bits below the cursor");

__device__ __forceinline__ unsigned long long bcast64(unsigned long long v) {
    return ((unsigned long long)uniform(__shfl((uint32_t)(v >> 32), 0)) << 32) | uniform(__shfl((uint32_t)v, 0));
}

// The lock holder's fold session for `tile`, `v` the fold word it holds (locked, with its own job's bit): folds
// the done jobs from the cursor on, in order, into the image (lane = pixel; the pixel's running value stays in
// registers across the session's jobs), returns their slots to the free queue, then releases the lock with a
// compare-and-swap that fails, and so folds on, if another job's bit arrived meanwhile.
// U: frames loaded per round trip (registers: k_trace_split, at its 72-VGPR budget, folds with 1)
template <uint32_t U>
__device__ __forceinline__ void fold_session(uint32_t tile, unsigned long long v, uint32_t lane) {
    const KPtr K = kargs();
    const uint32_t nc = K->nchunks;
    const uint32_t x = (tile % K->tiles_w) * 8u + (lane & 7u);
    const uint32_t kr = (tile / K->tiles_w) * 8u + (lane >> 3);
    const bool ok = x < K->W && kr < K->nrows;
    float* px = K->image + ((size_t)(ok ? kr : 0u) * K->W + (ok ? x : 0u)) * 3u;
    unsigned long long* word = K->tile_fold + tile;
    // the tile's job -> slot map, lane i holding job i's (written before each job's bit was set)
    uint32_t slots = 0;
    if (lane < nc) slots = __hip_atomic_load(K->job_slot + tile * nc + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
    bool loaded = false;
    const __amdgpu_buffer_rsrc_t rs = ring_rsrc();
    const float cap = K->ema_cap;
    // v: the word as last seen in memory (locked by us; its cursor changes only when we release); p: jobs folded
    uint32_t p = (uint32_t)(v >> TF_CURSOR_SHIFT) & 0x7Fu;
#pragma nounroll
    while (true) {
        const uint32_t p0 = p;
#pragma nounroll
        while (p < nc && ((v >> p) & 1ull)) {
            if (!loaded) {  // the pixel's value before this session (an earlier session or launch stored it)
                if (ok) {
                    a0 = __hip_atomic_load(px + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    a1 = __hip_atomic_load(px + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    a2 = __hip_atomic_load(px + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                loaded = true;
            }
            if (p >= 64u) break;  // (nc <= TF_MAX_JOBS: never)
            const uint32_t slot = uniform(__shfl(slots, (int)p));
            const uint32_t f0 = p << K->jf_log2, nf = min(1u << K->jf_log2, K->nframes - f0);
            const uint32_t frame0 = K->frame0 + f0;
            uint32_t off = ring_off(slot, 0u, lane, K->jf_log2);
            uint32_t f = 0;
            for (; f + U <= nf; f += U) {
                u32x4 c[U];
#pragma unroll
                for (uint32_t u = 0; u < U; u++) c[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off + (u << 10)), 0, 16);
#pragma unroll
                for (uint32_t u = 0; u < U; u++) {
                    const float w = 1.0f / (fmin_ieee((float)(frame0 + f + u), cap) + 1.0f);
                    const float omw = 1.0f - w;
                    a0 = a0 * omw + (0.0f + __uint_as_float(c[u].x)) * w;
                    a1 = a1 * omw + (0.0f + __uint_as_float(c[u].y)) * w;
                    a2 = a2 * omw + (0.0f + __uint_as_float(c[u].z)) * w;
                }
                off += U << 10;
            }
            for (; f < nf; f++, off += 1u << 10) {
                const u32x4 c = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 16);
                const float w = 1.0f / (fmin_ieee((float)(frame0 + f), cap) + 1.0f);
                const float omw = 1.0f - w;
                a0 = a0 * omw + (0.0f + __uint_as_float(c.x)) * w;
                a1 = a1 * omw + (0.0f + __uint_as_float(c.y)) * w;
                a2 = a2 * omw + (0.0f + __uint_as_float(c.z)) * w;
            }
            p++;
        }
        if (p > p0) {
            if (ok) {
                __hip_atomic_store(px + 0, a0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(px + 1, a1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(px + 2, a2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // the folded jobs' slots (their loads have returned: the values are in the sums) go back to the free
            // queue, for the jobs whose tickets are these returns' + ring_jobs
            uint32_t m = 0;
            if (lane == 0) m = __hip_atomic_fetch_add(K->ring_tail, p - p0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            m = uniform(__shfl(m, 0));
            const uint32_t k = lane;
            const uint32_t slot = __shfl(slots, (int)((p0 + k) & 63u));  // (all lanes: the sources must be active)
            if (k < p - p0)
                __hip_atomic_store(K->ring_q + ((m + k) & ((4u << K->ring_log2) - 1u)),
                                   ring_q_entry(slot, m + k, K->ring_log2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // image stores before the release
        }
        const unsigned long long nv = (v & ~(TF_LOCK | (0x7Full << TF_CURSOR_SHIFT))) |
                                      ((unsigned long long)p << TF_CURSOR_SHIFT);
        unsigned long long r = v;
        if (lane == 0) {
            unsigned long long expect = v;
            __hip_atomic_compare_exchange_strong(word, &expect, nv, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            r = expect;  // the word's value before the exchange (== v on success)
        }
        r = bcast64(r);
        if (r == v) return;
        v = r;  // new bits arrived: fold on from p, with the slots of the jobs that just completed
        if (lane < nc) slots = __hip_atomic_load(K->job_slot + tile * nc + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The wave's jobs whose samples are not all stored yet: the current one (being dealt, or waiting for its ring
// slot) and up to WJ_NE - 1 older ones with samples still in flight (a 50-bounce path can outlive several
// jobs of its wave). Kept in LDS, one block of words per wave (every lane reads and writes the same values),
// not in registers: the walk kernels have no SGPRs to spare.
constexpr uint32_t WJ_NE = 4;
// per entry: tile, first frame, samples in flight, ring slot (the job id while waiting for one)
enum : uint32_t { WJ_TILE = 0, WJ_F0 = WJ_NE, WJ_LIVE = 2 * WJ_NE, WJ_SLOT = 3 * WJ_NE, WJ_FLAGS = 4 * WJ_NE,
                  WJ_IDLE = 4 * WJ_NE + 1, WJ_STAT = 4 * WJ_NE + 2 };
// flags: busy bit per entry (bits 0..WJ_NE-1), the current entry (bits 8-9), dealing, waiting
// (slotted: the waiting current job has its slot)
enum : uint32_t { WJ_BUSY = (1u << WJ_NE) - 1u, WJ_CUR_SHIFT = 8, WJ_DEALING = 1u << 12, WJ_WAITING = 1u << 13,
                  WJ_SLOTTED = 1u << 14, WJ_TAILPH = 1u << 15 /* the wave has dealt a tail part (TAIL): CLAIM_FREE */ };
struct WaveJobs {
    uint32_t* w;  // this wave's words
    __device__ uint32_t get(uint32_t i) const { return uniform(w[i]); }
    __device__ void set(uint32_t i, uint32_t v) const { w[i] = v; }
    __device__ bool dealing() const { return (get(WJ_FLAGS) & WJ_DEALING) != 0u; }
    __device__ bool idle() const { return (get(WJ_FLAGS) & WJ_BUSY) == 0u; }
    __device__ uint32_t cur() const { return (get(WJ_FLAGS) >> WJ_CUR_SHIFT) & 3u; }
};

// A dealt sample's job reference (`fl` in the kernels): with the fold ring its wave's entry and its frame within
// the job; with the sample buffer its frame of the launch.
__device__ __forceinline__ uint32_t sample_ref(const WaveJobs& J, uint32_t f0, uint32_t fj) {
    return kargs()->ring_mode ? (J.cur() << 16) | fj : f0 + fj;
}

// cost: the sample's queries (its tile's cost for the next launch's deal order, cost-ordered dealing)
__device__ __forceinline__ void ring_store(const WaveJobs& J, uint32_t pix, uint32_t ref, const f3 c, uint32_t cost) {
    const KPtr K = kargs();
    if (!K->ring_mode) {  // sample buffer: the colour at its frame of the launch, folded by k_accumulate
        const uint32_t npix = K->tiles_w * K->tiles_h * 64u;  // tile-padded pixels of a frame (< 2^32)
        float* o = K->samples + ((unsigned long long)ref * npix + pix) * 3u;  // one 32 x 32 + 64 multiply-add
#if defined(HRT_STAMPS) && defined(HRT_DIAG_NOSTORE)  // (timing-only diagnostic build: wrong images)
        if (c.x != -12345.0f) return;
#endif
        o[0] = c.x;
        o[1] = c.y;
        o[2] = c.z;
        // (one counter per pixel: a wave's stores of one tile-frame add to 64 different words; one word per tile
        // serialised the 64 atomics and cost C3 4x in the launches that counted)
        if (uint32_t* const tc = K->tile_cost) __hip_atomic_fetch_add(tc + pix, cost, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const uint32_t slot = J.w[WJ_SLOT + (ref >> 16)];  // per-lane entry: an LDS read, not a uniform value
    const uint32_t off = ring_off(slot, ref & 0xFFFFu, pix & 63u, K->jf_log2);
    const u32x4 v = {__float_as_uint(c.x), __float_as_uint(c.y), __float_as_uint(c.z), 0u};
    __builtin_amdgcn_raw_buffer_store_b128(v, ring_rsrc(), (int)off, 0, 16 /* sc1: write-through */);
}

// Folds the sample buffer's colours of one tile's pixels into the image in frame order with the mix k_render uses
// (WGSL mix, shader_sphere.wgsl:264-271) for k_accumulate. `tile` (wave-uniform) points at the
// tile's frame 0, frame f at tile + f * fstride; the lane's pixel is 3 floats at lane3. U frames' loads are issued
// before their mixes (a wave's frame is 768 B: one load in flight per wave left k_accumulate latency-bound); the
// uniform frame address + a 32-bit lane offset keeps each load to one VGPR of address (global_load saddr).
template <int U>
__device__ __forceinline__ void fold_pixel(float* px, const float* tile, uint32_t lane3, size_t fstride, uint32_t nframes,
                                           uint32_t frame0, float ema_cap) {
    float acc0 = px[0], acc1 = px[1], acc2 = px[2];
    uint32_t f = 0;
    for (; f + (uint32_t)U <= nframes; f += (uint32_t)U, tile += (size_t)U * fstride) {
        float v[U][3];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const float* fr = tile + (size_t)j * fstride;
            v[j][0] = fr[lane3];
            v[j][1] = fr[lane3 + 1u];
            v[j][2] = fr[lane3 + 2u];
        }
#pragma unroll
        for (int j = 0; j < U; j++) {
            const float w = 1.0f / (fmin_ieee((float)(frame0 + f + (uint32_t)j), ema_cap) + 1.0f);
            const float omw = 1.0f - w;
            acc0 = acc0 * omw + (0.0f + v[j][0]) * w;
            acc1 = acc1 * omw + (0.0f + v[j][1]) * w;
            acc2 = acc2 * omw + (0.0f + v[j][2]) * w;
        }
    }
    for (; f < nframes; f++, tile += fstride) {
        const float w = 1.0f / (fmin_ieee((float)(frame0 + f), ema_cap) + 1.0f);
        const float omw = 1.0f - w;
        acc0 = acc0 * omw + (0.0f + tile[lane3]) * w;
        acc1 = acc1 * omw + (0.0f + tile[lane3 + 1u]) * w;
        acc2 = acc2 * omw + (0.0f + tile[lane3 + 2u]) * w;
    }
    px[0] = acc0;
    px[1] = acc1;
    px[2] = acc2;
}

// The previous launch's sample buffer folded inside this launch (rt_params.fold 3, RT_FOLD_NEXT; renderer.cpp: two
// sample buffers): every fold_mod-th wave takes tiles from a counter and folds each like k_accumulate before it starts
// tracing, so the fold's HBM reads run beside the other waves' tracing instead of in a launch of their own between two
// trace launches (the persistent grid holds every wave slot: a k_accumulate on a second stream only trickles in; DESIGN.md
// §6 Round 6). The folds stay in frame order: launch k's buffer is folded inside launch k + 1, before launch k + 1's own
// buffer is folded. The suspendable-walk kernels only (k_trace_split, k_trace_split_tris: their register allocation is
// unchanged by it; k_trace's loses a wave).
__device__ __forceinline__ void fold_prev_tiles(const KParams& P, uint32_t lane) {
    // Wave 0 of every m-th group of 8 consecutive workgroups (m = fold_mod / waves per workgroup): blocks are dealt to
    // the 8 XCDs round-robin, so the folders sit on all eight. (Every fold_mod-th wave of the grid would, with 4-wave
    // workgroups, be wave 0 of every 16th block — all on one XCD: C3 -0.3 %.)
    const uint32_t m = max(P.fold_mod / (blockDim.x >> 6), 1u);
    if ((threadIdx.x >> 6) != 0u || (blockIdx.x >> 3) % m != 0u) return;
    const uint32_t ntiles = P.tiles_w * P.tiles_h;
    const size_t npad3 = (size_t)ntiles * 192u;
    for (;;) {
        uint32_t t = 0;
        if (lane == 0u) t = __hip_atomic_fetch_add(P.fold_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = __builtin_amdgcn_readfirstlane(t);
        if (t >= ntiles) break;
        const uint32_t x = (t % P.tiles_w) * 8u + (lane & 7u);
        const uint32_t kr = (t / P.tiles_w) * 8u + (lane >> 3);
        if (x < P.W && kr < P.nrows)
            fold_pixel<8>(P.image + ((size_t)kr * P.W + x) * 3u, P.fold_prev + (size_t)t * 192u, lane * 3u, npad3,
                          P.fold_nframes, P.fold_frame0, P.ema_cap);
    }
}

#ifdef HRT_RINGSTAT
// diagnostic build: per-wave ring statistics (stall rounds: every entry busy; slot-wait rounds; folds; fold
// cycles / 16), summed into counter[5..8] at wave exit
#define WJ_WORDS (WJ_STAT + 4u)
#define RINGSTAT_ADD(J, i, v) (J).set(WJ_STAT + (i), (J).get(WJ_STAT + (i)) + (uint32_t)(v))
#else
#define WJ_WORDS (WJ_STAT)
#define RINGSTAT_ADD(J, i, v) ((void)0)
#endif

__device__ __forceinline__ WaveJobs wave_jobs(uint32_t* lds) {
    WaveJobs J{lds + (threadIdx.x >> 6) * WJ_WORDS};
    if ((threadIdx.x & 63u) < WJ_WORDS) J.w[threadIdx.x & 63u] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return J;
}

// A round with nothing in flight (the current job waits for a ring slot): sleep. A wave idle for 2^24 rounds in
// a row (seconds) would mean a broken protocol: it records itself in the watchdog words and leaves (true), so
// the launch ends and the draw reports an error instead of hanging the device. Any round with work resets it.
__device__ __forceinline__ bool idle_spin(const WaveJobs& J, uint32_t lane) {
    __builtin_amdgcn_s_sleep(2);
    const uint32_t n = J.get(WJ_IDLE) + 1u;
    J.set(WJ_IDLE, n);
    if (n < (1u << 24)) return false;
    if (lane == 0) {
        const KPtr K = kargs();
        atomicAdd(K->counter + WATCHDOG, 1ull);
        atomicExch(K->counter + WATCHDOG + 1, (unsigned long long)J.get(WJ_SLOT + J.cur()));
        atomicExch(K->counter + WATCHDOG + 2, (unsigned long long)J.get(WJ_FLAGS));
    }
    return true;
}

// One job of the wave is complete (every sample stored): set its bit in the tile's fold word and, in the same
// atomic, try the fold lock; the wave that gets it folds (fold_session), else the holder folds this job too.
template <uint32_t U>
__device__ __forceinline__ void job_complete(uint32_t tile, uint32_t c, uint32_t slot, uint32_t lane) {
    const KPtr K = kargs();
    if (!K->ring_mode) return;  // sample buffer: k_accumulate folds after the launch
    if (lane == 0) __hip_atomic_store(K->job_slot + tile * K->nchunks + c, slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sample stores (and the slot) have reached memory
    unsigned long long old = 0;
    if (lane == 0)
        old = __hip_atomic_fetch_or(K->tile_fold + tile, (1ull << c) | TF_LOCK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = bcast64(old);
    if (old & TF_LOCK) return;
    fold_session<U>(tile, old | (1ull << c) | TF_LOCK, lane);
}

// The current job is dealt out (it completes in job_account once nothing of it is in flight).
__device__ __forceinline__ void job_close(const WaveJobs& J, uint32_t /*lane*/) {
    J.set(WJ_FLAGS, J.get(WJ_FLAGS) & ~WJ_DEALING);
}

// The waiting current job polls the free queue for its slot (job j >= ring_jobs takes return j - ring_jobs).
__device__ __forceinline__ bool slot_poll(const WaveJobs& J, uint32_t flags, uint32_t lane) {
    if (flags & WJ_SLOTTED) return true;
    const KPtr K = kargs();
    if (!K->ring_mode) {  // sample buffer: no slot to wait for
        J.set(WJ_FLAGS, flags | WJ_SLOTTED);
        return true;
    }
    const uint32_t cur = (flags >> WJ_CUR_SHIFT) & 3u;
    const uint32_t job = J.get(WJ_SLOT + cur);  // waiting: the job id is its free-queue ticket
    uint32_t slot = job;                        // the first ring_jobs jobs take the slots in order
    if (job >> K->ring_log2) {
        const uint32_t m = job - (1u << K->ring_log2);
        uint32_t v = 0;
        if (lane == 0) v = __hip_atomic_load(K->ring_q + (m & ((4u << K->ring_log2) - 1u)), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        v = uniform(__shfl(v, 0));
        const uint32_t want = ring_q_entry(0u, m, K->ring_log2);
        if ((v & 0xFFF00000u) != want) {  // not returned yet (or, never expected, already overwritten)
            if ((v & 0x80000000u) && (((v >> 20) - (want >> 20)) & 0x7FFu) < 0x400u && lane == 0)
                atomicAdd(K->counter + WATCHDOG + 3, 1ull);
            RINGSTAT_ADD(J, 1, 1);
            return false;
        }
        slot = v & 0xFFFFFu;
    }
    J.set(WJ_SLOT + cur, slot);
    J.set(WJ_FLAGS, flags | WJ_SLOTTED);
    return true;
}

// The sample buffer's job queue: NQ counters (renderer.cpp), queue q handing out the jobs k * NQ + q; a wave takes from
// its XCD's queue first, then from the others in turn (the queues it found exhausted kept in its WJ_QDEAD word: the
// ring's slot words, unused with the sample buffer). With one counter for the whole GPU every job fetch is an atomic
// on one address from every XCD. Lane 0; returns >= njobs when every queue is exhausted.
constexpr uint32_t WJ_QDEAD = WJ_SLOT;  // (NQ, QSTRIDE: rt_device.hpp)
__device__ __forceinline__ uint32_t queue_take_lane0(const WaveJobs& J, const KPtr K) {
    unsigned long long* const qs = K->queues;
    if (qs == nullptr) return (uint32_t)min(atomicAdd(K->queue, 1ull), 0xFFFFFFFFull);
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    uint32_t dead = J.w[WJ_QDEAD], j = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < NQ; i++) {
        const uint32_t q = (x + i) & (NQ - 1u);
        if ((dead >> q) & 1u) continue;
        const unsigned long long jj = atomicAdd(qs + q * QSTRIDE, 1ull) * NQ + q;
        if (jj < K->njobs) {
            j = (uint32_t)jj;
            break;
        }
        dead |= 1u << q;
    }
    J.w[WJ_QDEAD] = dead;
    return j;
}

// Makes a job current and dealable: fetch one into a free entry and wait for its slot.
// false: nothing to deal now (queue drained -> `drained`; every entry still in flight; slot still folding).
// TAIL: the sample buffer's quarter jobs at the end of the launch (renderer.cpp tail_from; k_trace_split only:
// the decode cost the walk kernels of the other programs 2-6 spilled VGPRs).
template <bool TAIL = false>
__device__ __forceinline__ bool job_acquire(const WaveJobs& J, uint32_t lane, bool& drained, uint32_t& job_tile,
                                            uint32_t& job_f0, uint32_t& job_nf) {
    const KPtr K = kargs();
    uint32_t flags = J.get(WJ_FLAGS);
    if (!K->ring_mode) {  // sample buffer: no entries, no slots
        uint32_t j = 0;
        if (lane == 0) j = queue_take_lane0(J, K);
        j = uniform(__shfl(j, 0));
        if (j >= K->njobs) {
            drained = true;
            return false;
        }
        J.set(WJ_FLAGS, flags | WJ_DEALING);
        if constexpr (TAIL) {
            // The launch's last jobs are dealt in parts (2^tail_shift per job): a job dealt late then ends soon after
            // the queue drains instead of holding the launch for a whole job (whole chunks of a job_frames multiple of
            // the part count)
            const uint32_t tail = K->tail_from, ts = K->tail_shift;
            const bool part = j >= tail;
            const uint32_t q = j - tail;
            const uint32_t jj = part ? tail + (q >> ts) : j;
            job_tile = jj / K->nchunks;
            job_f0 = (jj - job_tile * K->nchunks) * K->job_frames;
            if (const uint32_t* const ord = K->tile_order) job_tile = ord[job_tile];
            job_nf = min(K->job_frames, K->nframes - job_f0);
            if (part) {
                job_nf >>= ts;
                job_f0 += (q & ((1u << ts) - 1u)) * job_nf;
                J.set(WJ_FLAGS, flags | WJ_DEALING | WJ_TAILPH);
            }
        } else {
            job_tile = j / K->nchunks;
            job_f0 = (j % K->nchunks) * K->job_frames;
            if (const uint32_t* const ord = K->tile_order) job_tile = ord[job_tile];
            job_nf = min(K->job_frames, K->nframes - job_f0);
        }
        return true;
    }
    if (!(flags & WJ_WAITING)) {
        if ((flags & WJ_BUSY) == WJ_BUSY) {  // every entry still has samples in flight
            RINGSTAT_ADD(J, 0, 1);
            return false;
        }
        const uint32_t e = (uint32_t)__builtin_ctz(~flags & WJ_BUSY);
        uint32_t j = 0;
        if (lane == 0) j = (uint32_t)atomicAdd(K->queue, 1ull);
        j = uniform(__shfl(j, 0));
        if (j >= K->njobs) {
            drained = true;
            return false;
        }
        J.set(WJ_TILE + e, j / K->nchunks);
        J.set(WJ_F0 + e, (j % K->nchunks) * K->job_frames);
        J.set(WJ_LIVE + e, 0u);
        J.set(WJ_SLOT + e, j);
        flags = (flags & ~((3u << WJ_CUR_SHIFT) | WJ_SLOTTED)) | (1u << e) | (e << WJ_CUR_SHIFT) | WJ_WAITING;
        J.set(WJ_FLAGS, flags);
    }
    if (!slot_poll(J, flags, lane)) return false;
    const uint32_t cur = (flags >> WJ_CUR_SHIFT) & 3u;
    J.set(WJ_FLAGS, (flags & ~(WJ_WAITING | WJ_SLOTTED)) | WJ_DEALING);
    job_tile = J.get(WJ_TILE + cur);
    job_f0 = J.get(WJ_F0 + cur);
    job_nf = min(K->job_frames, K->nframes - job_f0);
    return true;
}

// Samples just dealt from the current job (lanes that took one).
__device__ __forceinline__ void job_dealt(const WaveJobs& J, uint32_t n) {
    if (n == 0u || !kargs()->ring_mode) return;
    J.set(WJ_IDLE, 0u);
    const uint32_t i = WJ_LIVE + ((J.get(WJ_FLAGS) >> WJ_CUR_SHIFT) & 3u);
    J.set(i, J.get(i) + n);
}

// End of a round: lanes whose sample finished (`fin`, colour stored) are counted off their jobs (the busy entry
// whose tile and frames hold the sample); jobs neither current nor with anything in flight complete, and a job
// that completes its tile folds it.
template <uint32_t U = 2>
__device__ __forceinline__ void job_account(const WaveJobs& J, bool fin, uint32_t ref, uint32_t lane) {
    if (!kargs()->ring_mode) return;  // sample buffer: nothing to track
    const unsigned long long any = __ballot(fin);
    if (any != 0ull) {
        const uint32_t idx = ref >> 16;
#pragma unroll
        for (uint32_t e = 0; e < WJ_NE; e++) {
            const uint32_t n = (uint32_t)__popcll(__ballot(fin && idx == e));
            if (n) J.set(WJ_LIVE + e, J.get(WJ_LIVE + e) - n);
        }
    }
    {
        const uint32_t flags = J.get(WJ_FLAGS);
        if (flags & WJ_WAITING) (void)slot_poll(J, flags, lane);  // every round, not only when lanes are free
    }
#pragma nounroll
    for (uint32_t e = 0; e < WJ_NE; e++) {
        const uint32_t flags = J.get(WJ_FLAGS);
        const bool current = ((flags >> WJ_CUR_SHIFT) & 3u) == e && (flags & (WJ_DEALING | WJ_WAITING));
        if (((flags >> e) & 1u) && J.get(WJ_LIVE + e) == 0u && !current) {
            J.set(WJ_FLAGS, flags & ~(1u << e));
#ifdef HRT_RINGSTAT
            const unsigned long long t0 = __builtin_readcyclecounter();
#endif
            job_complete<U>(J.get(WJ_TILE + e), J.get(WJ_F0 + e) >> kargs()->jf_log2, J.get(WJ_SLOT + e), lane);
#ifdef HRT_RINGSTAT
            RINGSTAT_ADD(J, 2, 1);
            RINGSTAT_ADD(J, 3, (__builtin_readcyclecounter() - t0) >> 4);
#endif
        }
    }
}

// ---- Frame-block work stealing (sample buffer; the suspendable-walk kernels; rt_params.steal) ----
// A job is one 8x8 tile x job_frames frames, and a wave deals its frames one frame block (the tile's 64 pixels in
// one frame) at a time. A job's cost varies by orders of magnitude across the image (sky: one query per sample;
// glass and crevices: up to the bounce cap), so once the job queue is drained the launch used to wait for the
// slowest job dealt last (C4's 8-way split: shares of 24 ms ideal took 33-55 ms). Here each wave publishes its
// current job in a 64-bit slot and claims its frames with atomicAdd, STEAL_OWN frames at a time (one atomic per
// frame block cost C3 2 %); a wave that finds the queue drained claims single frames of other waves' jobs the
// same way. The atomic decides every frame exactly once; a sample's colour goes to its (frame, pixel) place of the
// sample buffer whichever wave traced it, so the image bits do not change. Slot: (tile + 1) << 39 | chunk << 28 |
// frames of the job << 16 | frames claimed — everything a thief needs, without a division (renderer.cpp enables
// stealing for < 2^25 - 1 tiles and < 2^11 chunks; claims stop once a slot reads exhausted, so the 16-bit count
// stays far below its field's end). Wave state in the WaveJobs words the sample buffer leaves unused: flags (own
// job, queue drained, lost race), the last victim, and the claimed frames not dealt yet.
#ifndef HRT_STEAL_OWN
#define HRT_STEAL_OWN 1  // (4 before round 5: the owner's claims of 4 frames held them from idle thieves in the tail;
                         // 4 only for jobs dealt early, while the queue holds > 2 jobs per wave: C4 8-way 0.756 -> 0.70,
                         // the early jobs still running at the drain are the long ones, profiles/r05/p/)
#endif
#ifndef HRT_CLAIM_FREE
#define HRT_CLAIM_FREE 32
#endif
constexpr uint32_t STEAL_OWN = HRT_STEAL_OWN;
constexpr uint32_t ST_OWN = 1u, ST_QEMPTY = 2u, ST_RETRY = 4u;
// The tail (round 5): once the job queue is drained, a wave whose lanes are not all free claims another frame block only
// when at least CLAIM_FREE of them are. A block claimed for a few free lanes waits for this wave's busy ones (paths of
// up to 50 bounces) while other waves have run dry and exited: C4's 1/8 share drained its queue at 18.1 ms and ran to
// 23.5 ms (`scripts/wave_tail.py`, profiles/r05/). A wave with every lane free always claims, so the launch drains.
constexpr uint32_t CLAIM_FREE = HRT_CLAIM_FREE;
// The same rule for a wave that has dealt a tail part (job_acquire<TAIL>, no stealing): its next part waits for
// CLAIM_FREE free lanes (HRT_TAIL_CLAIM 0 = round 4: a part for any free lane).
#ifndef HRT_TAIL_CLAIM
#define HRT_TAIL_CLAIM 1
#endif
constexpr bool TAIL_CLAIM = HRT_TAIL_CLAIM != 0;


enum : uint32_t { WJ_ST = WJ_TILE, WJ_VICTIM = WJ_TILE + 1, WJ_PRIV_F = WJ_TILE + 2, WJ_PRIV_N = WJ_TILE + 3,
                  WJ_CLAIM_F = WJ_F0, WJ_CLAIM_T = WJ_LIVE };

// true when the job queue is drained (known to this wave, or read from the queue counter: one load per call)
__device__ __forceinline__ bool queue_drained(const WaveJobs& J, uint32_t lane) {
    if (J.get(WJ_ST) & ST_QEMPTY) return true;
    const KPtr K = kargs();
    // (stealing launches run on the single counter: renderer.cpp gives them no per-XCD queues)
    uint32_t d = 0;
    if (lane == 0) d = __hip_atomic_load(K->queue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= K->njobs ? 1u : 0u;
    return uniform(__shfl(d, 0)) != 0u;
}

__device__ __forceinline__ bool slot_open(unsigned long long w) {
    return (w >> 39) != 0ull && (uint32_t)(w & 0xFFFFu) < (uint32_t)((w >> 16) & 0xFFFu);
}

// Lane 0, after its claim of up to `want` frames returned the slot's old value v: the claimed frames go to the
// wave's words (first frame and tile, then the rest as private frames); every lane reads them with claim_read.
// (Through LDS, not a cross-lane register broadcast: the walk kernels spilled with the latter.)
__device__ __forceinline__ void claim_publish(const WaveJobs& J, const KPtr K, unsigned long long v, uint32_t want) {
    if (slot_open(v)) {
        const uint32_t got = (uint32_t)(v & 0xFFFFu), nf = (uint32_t)((v >> 16) & 0xFFFu);
        const uint32_t f = ((uint32_t)(v >> 28) & 0x7FFu) * K->job_frames + got;
        J.w[WJ_CLAIM_F] = f;
        J.w[WJ_CLAIM_T] = (uint32_t)(v >> 39) - 1u;
        J.w[WJ_PRIV_F] = f + 1u;
        J.w[WJ_PRIV_N] = min(want, nf - got) - 1u;
    } else {
        J.w[WJ_CLAIM_F] = ~0u;
    }
}
__device__ __forceinline__ bool claim_read(const WaveJobs& J, uint32_t& tile, uint32_t& frame) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    frame = J.get(WJ_CLAIM_F);
    tile = J.get(WJ_CLAIM_T);
    return frame != ~0u;
}

// The cold part (only once the job queue is drained): every wave's slot, 64 at a time, from the last victim on; one
// claim attempt per 64 slots (a lost race moves on; the next call comes back).
__device__ __forceinline__ bool steal_scan(const WaveJobs& J, uint32_t lane, uint32_t& tile, uint32_t& frame) {
    const KPtr K = kargs();
    unsigned long long* const slots = K->steal_slots;
    const uint32_t nw = K->nwaves, start = J.get(WJ_VICTIM);
    for (uint32_t k = 0; k < nw; k += 64u) {
        uint32_t idx = start + k + lane;
        idx = idx >= nw ? idx - nw : idx;
        const unsigned long long m =
            __ballot(k + lane < nw && slot_open(__hip_atomic_load(slots + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
        if (m != 0ull) {
            const uint32_t vi = uniform(__shfl(idx, __ffsll((long long)m) - 1));
            if (lane == 0) claim_publish(J, K, atomicAdd(slots + vi, 1ull), 1u);
            if (claim_read(J, tile, frame)) {
                J.set(WJ_VICTIM, vi);
                return true;
            }
            J.set(WJ_ST, J.get(WJ_ST) | ST_RETRY);
        }
    }
    return false;
}

// The wave's next frame block (tile, frame of the launch): a claimed frame not dealt yet, new frames of its own
// job, the first frames of a new job, or once the queue is drained a frame claimed from another wave's job. false:
// nothing claimed; then steal_drained() tells whether no frame is left unclaimed anywhere — none can appear (jobs
// come only from the drained queue), so the caller stops asking — or an open slot was seen whose claim lost a
// race (ask again later).
__device__ __forceinline__ bool steal_block_claim(const WaveJobs& J, uint32_t lane, uint32_t& tile, uint32_t& frame) {
    const uint32_t priv = J.get(WJ_PRIV_N);
    if (priv != 0u) {
        frame = J.get(WJ_PRIV_F);
        tile = J.get(WJ_CLAIM_T);
        J.set(WJ_PRIV_F, frame + 1u);
        J.set(WJ_PRIV_N, priv - 1u);
        return true;
    }
    const KPtr K = kargs();
    unsigned long long* const slots = K->steal_slots;
    const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t st = J.get(WJ_ST);
    if (st & ST_OWN) {
        if (lane == 0) claim_publish(J, K, atomicAdd(slots + wid, (unsigned long long)STEAL_OWN), STEAL_OWN);
        if (claim_read(J, tile, frame)) return true;
        J.set(WJ_ST, st & ~ST_OWN);
    }
    if (!(st & ST_QEMPTY)) {
        if (lane == 0) {
            // (stealing launches fetch from the single counter: renderer.cpp passes no per-XCD queues with steal)
            const uint32_t j = (uint32_t)min(atomicAdd(K->queue, 1ull), 0xFFFFFFFFull);
            unsigned long long v = 0;
            if (j < K->njobs) {  // the new job's first STEAL_OWN frames are ours with the exchange
                const uint32_t tj = j / K->nchunks, c = j - tj * K->nchunks;
                const uint32_t t = K->tile_order ? K->tile_order[tj] : tj;
                const uint32_t nf = min(K->job_frames, K->nframes - c * K->job_frames);
                v = ((unsigned long long)(t + 1u) << 39) | ((unsigned long long)c << 28) | ((unsigned long long)nf << 16);
                (void)atomicExch(slots + wid, v + STEAL_OWN);
            }
            claim_publish(J, K, v, STEAL_OWN);
        }
        if (claim_read(J, tile, frame)) {
            J.set(WJ_ST, ST_OWN);
            return true;
        }
    }
    J.set(WJ_ST, ST_QEMPTY);  // (clears ST_RETRY)
    return steal_scan(J, lane, tile, frame);
}
__device__ __forceinline__ bool steal_block(const WaveJobs& J, uint32_t lane, uint32_t& tile, uint32_t& frame) {
    const bool got = steal_block_claim(J, lane, tile, frame);
    if (got) J.set(WJ_IDLE, 0u);  // idle_spin's watchdog counts CONSECUTIVE rounds without work (lost races)
    return got;
}
__device__ __forceinline__ bool steal_drained(const WaveJobs& J) { return (J.get(WJ_ST) & ST_RETRY) == 0u; }

// Refill with primary rays by frame block (k_trace with the simple sphere scan): when the wave's block
// (one frame of its job's 8x8 tile) is used up, every lane computes the primary ray of its own pixel for
// the next frame at once (all lanes busy), and lanes that need a sample fetch one from the block's owner
// lane with cross-lane reads, instead of each freed lane computing its own with a few lanes active
// (k_trace_split does the same inline).
#ifdef HRT_STAMPS
constexpr uint32_t JOB_TRACE_CAP = 1u << 21;
// the job's duration (take to the next take or the drain, 100 MHz ticks) | its take time's low 32 bits << 32
__device__ __forceinline__ void job_trace_put(const KParams& P, uint32_t id, unsigned long long t0, unsigned long long t1) {
    if (P.job_trace == nullptr || id >= JOB_TRACE_CAP || (threadIdx.x & 63u) != 0u) return;
    P.job_trace[id] = min(t1 - t0, 0xFFFFFFFFull) | (t0 << 32);
}
#endif
struct BlockQueue {
    uint32_t job_tile = 0, job_f0 = 0, job_nf = 0, blk_f = 0, blk_next = 64;  // wave-uniform
    f3 pr_o = {0.0f, 0.0f, 0.0f}, pr_d = {0.0f, 0.0f, 0.0f};
    uint32_t pr_s = 0, pr_ok = 0;  // this lane's pixel's primary ray for the block, and whether it exists
#ifdef HRT_STAMPS
    uint32_t njobs = 0;                // (diagnostic build: jobs this wave took, when it took its last one, and
    unsigned long long last_job = 0;   // the longest time between two of its job fetches)
    unsigned long long max_job = 0;
    uint32_t took_job = 0;             // (a job was taken this round)
    uint32_t job_id = 0xFFFFFFFFu;     // (the current job's index, for P.job_trace)
#endif
};

// Free lanes (!have) take the next samples; sets drained once the job queue is empty.
template <int MODE>
__device__ __forceinline__ void refill_block(const KParams& P, BlockQueue& B, const WaveJobs& J, bool& drained, uint32_t lane,
                                             unsigned long long below, bool& have, Ray& ray, f3& att,
                                             float& sky_t, uint32_t& s, uint32_t& bounce, uint32_t& pix,
                                             uint32_t& fl) {
    bool need = !have && !drained;
    unsigned long long m = __ballot(need);
    while (m != 0ull) {
        if (B.blk_next == 64u) {
            if (J.dealing()) {
                B.blk_f++;
            } else {
                if (!job_acquire(J, lane, drained, B.job_tile, B.job_f0, B.job_nf)) break;
                B.blk_f = 0;
#ifdef HRT_STAMPS
                {
                    const unsigned long long now = hrt_realtime();
                    if (B.njobs) B.max_job = max(B.max_job, now - B.last_job);
                    job_trace_put(P, B.job_id, B.last_job, now);
                    B.njobs++;
                    B.last_job = now;
                    B.took_job = 1u;
                    B.job_id = B.job_tile * P.nchunks + B.job_f0 / max(P.job_frames, 1u);
                }
#endif
            }
            B.blk_next = 0;
            const uint32_t x = (B.job_tile % P.tiles_w) * 8u + (lane & 7u);
            const uint32_t kr = (B.job_tile / P.tiles_w) * 8u + (lane >> 3);
            B.pr_ok = (x < P.W && kr < P.nrows) ? 1u : 0u;  // ragged edge tiles: no sample
            if (B.pr_ok) {
                const uint32_t y = global_row(P.row0, P.row_block, P.row_stride, kr);
#ifndef HRT_UGUARD_KTRACE_PRIMARY
#define HRT_UGUARD_KTRACE_PRIMARY 1
#endif
                const Ray pr = primary_ray<MODE, MODE == MODE_SPHERE, MODE == MODE_SPHERE && HRT_UGUARD_KTRACE_PRIMARY != 0>(
                    &kargs()->cam, x, y, P.time0 + (B.job_f0 + B.blk_f) * P.dtime, B.pr_s);
                B.pr_o = pr.o;
                B.pr_d = pr.d;
            }
        }
        const uint32_t avail = 64u - B.blk_next;
        const uint32_t rank = (uint32_t)__popcll(m & below);
        const int src = (int)((B.blk_next + rank) & 63u);
        const float ox = __shfl(B.pr_o.x, src), oy = __shfl(B.pr_o.y, src), oz = __shfl(B.pr_o.z, src);
        const float dx = __shfl(B.pr_d.x, src), dy = __shfl(B.pr_d.y, src), dz = __shfl(B.pr_d.z, src);
        const uint32_t ss = __shfl(B.pr_s, src), ok = __shfl(B.pr_ok, src);
        bool took = false;
        if (need && rank < avail) {
            need = false;
            if (ok) {
                ray.o = mk(ox, oy, oz);
                ray.d = mk(dx, dy, dz);
                s = ss;
                fl = sample_ref(J, B.job_f0, B.blk_f);
                pix = B.job_tile * 64u + (uint32_t)src;
                sky_t = ray.d.y * 0.5f + 0.5f;
                att = mk(1.0f, 1.0f, 1.0f);
                bounce = 0;
                have = true;
                took = true;
            }
        }
        job_dealt(J, (uint32_t)__popcll(__ballot(took)));
        B.blk_next += min((uint32_t)__popcll(m), avail);
        if (B.blk_next == 64u && B.blk_f + 1u >= B.job_nf) job_close(J, lane);
        m = __ballot(need);
    }
}

}  // namespace

// Tiles schedule (rt_params.schedule = RT_SCHEDULE_TILES): one launch = P.nframes frames over this
// renderer's rows; a lane owns one pixel for all of them and accumulates in registers.
// Grid: (ceil(W/16), ceil(nrows/16)).
template <int MODE, int SCAN, bool TSAH = false>
__global__ __launch_bounds__(256) void k_render(const KParams P) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const LaneLists lists = lane_lists<MODE, SCAN>();
    void* const lds_list = lists.sphere;
    uint32_t* const tri_cand = lists.tri;
    uint32_t* const tri_stack = lists.tri;
    Tally tally;
    const uint32_t x = blockIdx.x * 16u + (wave & 1u) * 8u + (lane & 7u);
    const uint32_t kr = blockIdx.y * 16u + (wave >> 1) * 8u + (lane >> 3);
    const bool valid = x < P.W && kr < P.nrows;
    const uint32_t y = global_row(P.row0, P.row_block, P.row_stride, kr);
    float* px = P.image + ((size_t)kr * P.W + x) * 3u;

    float acc0 = 0.0f, acc1 = 0.0f, acc2 = 0.0f;
    if (valid) {
        acc0 = px[0];
        acc1 = px[1];
        acc2 = px[2];
    }
    uint32_t f = valid ? 0u : P.nframes;
    uint32_t queries = 0;

    // Path state of the lane's current sample.
    Ray ray;
    f3 att = mk(1.0f, 1.0f, 1.0f);
    float sky_t = 0.0f;
    uint32_t s = 0, bounce = 0;
    if (f < P.nframes) {
        ray = primary_ray<MODE>(&kargs()->cam, x, y, P.time0, s);
        sky_t = ray.d.y * 0.5f + 0.5f;
    }

#ifdef HRT_STAMPS  // diagnostic build only (lib/libhrt_diag.so): wave cycles per region
    unsigned long long st_trav = 0, st_shade = 0, st_gen = 0, st_ta, st_tb = 0, st_tc;
    const unsigned long long st_start = hrt_stamp();
    const unsigned long long rt_start = hrt_realtime();
#endif
    while (f < P.nframes) {
        bool done = true;
#ifdef HRT_STAMPS
        st_ta = hrt_stamp();
#endif
        if (bounce < P.bounces) {
            Hit h;
            const bool hit = closest_hit<MODE, SCAN, TSAH>(P, ray, h, lds_list, tally, tri_cand, tri_stack);
            queries++;
#ifdef HRT_STAMPS
            st_tb = hrt_stamp();
            st_trav += st_tb - st_ta;
#endif
            if (hit) {
                scatter<MODE>(P, s, ray, h);
                att = att * mk(h.ar * 0.7f, h.ag * 0.7f, h.ab * 0.7f);
                bounce++;
                done = bounce >= P.bounces;
            }
        }
#ifdef HRT_STAMPS
        st_tc = hrt_stamp();
        st_shade += st_tc - st_tb;
#endif
        if (done) {
            // trace() epilogue (:241-242) + accumulation (:264-271).
            const float u = 1.0f - sky_t;
            const f3 sky = mk(0.54f * u + 0.54f * sky_t, 0.86f * u + 0.7f * sky_t, 0.92f * u + 0.98f * sky_t);
            const f3 c = att * sky;
            const float fc = (float)(P.frame0 + f);
            const float w = 1.0f / (fmin_ieee(fc, P.ema_cap) + 1.0f);
            const float omw = 1.0f - w;
            acc0 = acc0 * omw + (0.0f + c.x) * w;
            acc1 = acc1 * omw + (0.0f + c.y) * w;
            acc2 = acc2 * omw + (0.0f + c.z) * w;
            f++;
            if (f < P.nframes) {
                ray = primary_ray<MODE>(&kargs()->cam, x, y, P.time0 + f * P.dtime, s);
                sky_t = ray.d.y * 0.5f + 0.5f;
                att = mk(1.0f, 1.0f, 1.0f);
                bounce = 0;
            }
        }
#ifdef HRT_STAMPS
        st_gen += hrt_stamp() - st_tc;
#endif
    }

    if (valid) {
        px[0] = acc0;
        px[1] = acc1;
        px[2] = acc2;
    }
#ifdef HRT_STAMPS
    // Loop-carried sums are per lane (a lane stops adding once its frames are done), so summed over the
    // lanes they give lane-cycles per region; the lifetime is counted per lane too (x64), and the
    // remainder is lane-cycles spent idle behind the wave's slowest lane.
    {
        unsigned long long life = valid ? hrt_stamp() - st_start : 0ull;
        unsigned long long v[5] = {st_trav, st_shade, st_gen, life, queries};
        if (!valid) v[0] = v[1] = v[2] = 0ull;
#pragma unroll
        for (int c = 0; c < 5; c++) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v[c] += __shfl_xor(v[c], off);
        }
        if (lane == 0) {
            for (int c = 0; c < 4; c++) atomicAdd(P.counter + 8 + c, v[c]);
            // wave residency in 100 MHz ticks, wave count, and the memtime ticks of the same interval
            const unsigned long long t1 = hrt_stamp(), r1 = hrt_realtime();
            atomicAdd(P.counter + 12, r1 - rt_start);
            atomicAdd(P.counter + 13, 1ull);
            atomicAdd(P.counter + 14, t1 - st_start);
            if (P.wave_trace) {
                // one record per wave of the FIRST launch of the draw (frame0 == trace frame): start/end in
                // 100 MHz ticks, HW_ID | XCC_ID << 32, queries of lane 0's pixel
                unsigned hw, xcc;
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
                const size_t wid = ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 4u + wave;
                unsigned long long* rec = P.wave_trace + 8u * wid;  // (8-word records, WaveRecord; words 4-7 unused here)
                rec[0] = rt_start;
                rec[1] = r1;
                rec[2] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
                rec[3] = v[4];
            }
        }
    }
#endif
    // One atomic per wave and counter: rays, box tests, sphere tests, tri-program node and triangle tests.
    unsigned long long sums[5] = {queries, tally.boxes, tally.spheres, tally.nodes, tally.tris};
#pragma unroll
    for (int c = 0; c < 5; c++) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sums[c] += __shfl_xor(sums[c], off);
    }
    if (lane == 0) flush_counts(sums);
}

// ---------------------------------------------------------------------------------------------------
// Sample-queue schedule (rt_params.schedule = RT_SCHEDULE_QUEUE). The tiles schedule (k_render) gives
// every lane one pixel for all frames of a launch, so a pixel whose paths are long (glass, crevices:
// 20+ queries per sample) serialises its whole frame chunk on one lane and the launch waits for it
// (wave records: one C4 wave ran 128 ms of a 129 ms launch while the GPU averaged < 1 resident wave
// per SIMD), and a workgroup's slots stay taken until its slowest wave ends.
// Here a persistent grid (resident capacity) pulls JOBS from a global counter: a job is one 8x8 tile
// and `job_frames` frames, i.e. 64 x job_frames samples. A wave hands the samples of its current job
// to its lanes as they become free (wave-uniform bookkeeping, no per-sample atomics), and takes the
// next job as soon as the current one has no samples left, while older samples are still in flight.
// Lanes therefore never idle until the queue is empty, a wave's lanes stay inside one tile (ray
// coherence: an incoherent sample queue measured 2.65x slower on C3), and one tile's frames are
// spread over many waves. Each sample's colour goes to its tile's slot of the fold ring, and the wave that
// completes a tile's last job folds the slot into the image in frame order per pixel with the reference's
// mix (shader_sphere.wgsl:264-271; fold_session), so the image is bit-identical to k_render's and to
// count x rt_draw.
#ifdef HRT_STAMPS
// Diagnostic build: the persistent kernels' per-wave record (rt_get_wave_trace; scripts/wave_tail.py), 8 words per wave
// at wave id blockIdx.x * waves per workgroup + wave: start and end (100 MHz ticks, s_memrealtime), HW_ID | XCC_ID << 32,
// and (ticks from start until the wave first found no frame block left to take) | frame blocks it generated << 32.
struct WaveRecord {
    // 8 words per wave (rt_get_wave_trace): [0] start, [1] end (s_memrealtime, 100 MHz); [2] HW_ID (k_trace: the longest
    // job in bits 0-23) | XCC_ID << 32 | k_trace: the last job's take << 40; [3] ticks until the wave first found no work |
    // frame blocks generated << 32 (k_trace: jobs taken); [4] / [5] s_memtime (shader clock) at start / end; [6] shader
    // clock ticks from start to the drain (0: never drained) | k_trace: to its last job take << 32; [7] k_trace: lanes
    // holding a sample at the drain | samples finished after the last job take << 8 | rounds after the drain << 24 |
    // rounds from the last job take to the drain << 36 | all rounds << 48 (the C2 launch-end tail)
    unsigned long long start = 0, drained = 0, start_clk = 0, drained_clk = 0, job_clk = 0;
    uint32_t inflight = 0, fin_after_job = 0, rounds_after_drain = 0, rounds_job = 0, rounds = 0;
    __device__ void begin() {
        start = hrt_realtime();
        start_clk = hrt_stamp();
    }
    __device__ void drain(bool d, uint32_t in_flight = 0) {
        if (d && drained == 0ull) {
            drained = hrt_realtime() - start;
            drained_clk = hrt_stamp();
            inflight = in_flight;
        }
    }
    __device__ void round(uint32_t finished, bool took_job) {  // (k_trace: once per round, wave-uniform)
        rounds++;
        if (took_job) {
            fin_after_job = 0;
            rounds_job = 0;
            job_clk = hrt_stamp();
        }
        fin_after_job += finished;
        if (drained) rounds_after_drain++;
        else rounds_job++;
    }
    // last_job (k_trace): when the wave took its last job (s_memrealtime; 0: not recorded), as ticks from its start in
    // bits 40-63 of word 2
    // max_job (k_trace): the longest time between two job fetches, in bits 0-23 of word 2 (the HW_ID then dropped)
    __device__ void finish(const KParams& P, uint32_t lane, uint32_t nblocks, unsigned long long last_job = 0,
                           unsigned long long max_job = 0) {
        if (lane != 0u || P.wave_trace == nullptr) return;
        const unsigned long long end = hrt_realtime(), end_clk = hrt_stamp();
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const size_t wid = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        unsigned long long* rec = P.wave_trace + 8u * wid;
        rec[0] = start;
        rec[1] = end;
        const unsigned long long lj = last_job ? min(last_job - start, 0xFFFFFFull) : 0ull;
        const unsigned long long w0 = last_job ? min(max_job, 0xFFFFFFull) : (unsigned long long)hw;
        rec[2] = w0 | ((unsigned long long)(xcc & 0xFFu) << 32) | (lj << 40);
        rec[3] = (drained ? drained : end - start) | ((unsigned long long)nblocks << 32);
        rec[4] = start_clk;
        rec[5] = end_clk;
        rec[6] = (drained_clk ? min(drained_clk - start_clk, 0xFFFFFFFFull) : 0ull) |
                 ((job_clk ? min(job_clk - start_clk, 0xFFFFFFFFull) : 0ull) << 32);
        rec[7] = (unsigned long long)min(inflight, 0xFFu) | ((unsigned long long)min(fin_after_job, 0xFFFFu) << 8) |
                 ((unsigned long long)min(rounds_after_drain, 0xFFFu) << 24) | ((unsigned long long)min(rounds_job, 0xFFFu) << 36) |
                 ((unsigned long long)min(rounds, 0xFFFFu) << 48);
    }
};
#endif

struct BlockState {
    uint32_t job_tile = 0, job_f0 = 0, job_nf = 0, blk_f = 0, blk_next = 64;  // wave-uniform
#ifdef HRT_STAMPS
    uint32_t nblocks = 0;  // (diagnostic build: frame blocks this wave generated, for its wave record)
#endif
};
#ifndef HRT_UGUARD_KTRACE
#define HRT_UGUARD_KTRACE 1  // (k_trace's sphere program: the exact sequences' guards as wave-uniform branches)
#endif
template <int MODE, int SCAN, bool TSAH = false>
// 6 waves per SIMD: the register budget is 80 VGPRs (84 unconstrained = 5 waves; measured +8% on C3)
// (the mixed program's deferred scan holds 32 KB of LDS per workgroup: 5 waves/SIMD whatever the VGPRs)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(
    TSAH || (MODE == MODE_MIXED && SCAN == SCAN_DEFER) ? 5 : 6))) void k_trace(const KParams P) {
    const uint32_t lane = threadIdx.x & 63u;
    const LaneLists lists = lane_lists<MODE, SCAN>();
    void* const lds_list = lists.sphere;
    uint32_t* const tri_cand = lists.tri;
    uint32_t* const tri_stack = lists.tri;
    Tally tally;
    uint32_t queries = 0;
    const unsigned long long below = (1ull << lane) - 1ull;

    // wave-uniform job state
    uint32_t job_tile = 0, job_f0 = 0, job_nf = 0, job_next = 0, job_total = 0;
    BlockQueue BQ;  // frame-block refill (simple sphere scan only)
    __shared__ uint32_t wjobs[4 * WJ_WORDS];
    const WaveJobs J = wave_jobs(wjobs);
    bool drained = false;
    // lane state
    Ray ray;
    f3 att = mk(1.0f, 1.0f, 1.0f);
    float sky_t = 0.0f;
    uint32_t s = 0, bounce = 0, pix = 0, fl = 0;  // pix = tile * 64 + pixel-in-tile
    bool have = false;
#ifdef HRT_STAMPS
    unsigned long long st_trav = 0, st_shade = 0, st_gen = 0, st_ta, st_tb;
    unsigned long long st_pq = 0, st_pbox = 0, st_ptrav = 0;
    const unsigned long long st_start = hrt_stamp();
    const unsigned long long rt_start = hrt_realtime();
    WaveRecord wrec;
    wrec.begin();
#endif
    while (true) {
#ifdef HRT_STAMPS
        st_ta = hrt_stamp();
#endif
        // refill: free lanes take the next samples of the wave's job, fetching jobs as they run out
        // frame-block primary rays for the simple sphere scan (C2: 51.8 -> 59.5 Grays/s); the other
        // instantiations have no registers to spare for the block's 7 values
        constexpr bool BLOCK_REFILL = MODE == MODE_SPHERE && SCAN == SCAN_SIMPLE;
        bool need = !have && !drained;
        if constexpr (BLOCK_REFILL) {
            refill_block<MODE>(P, BQ, J, drained, lane, below, have, ray, att, sky_t, s, bounce, pix, fl);
            need = false;
        }
        unsigned long long m = __ballot(need);
        while (m != 0ull) {
            if (!J.dealing()) {
                // tile-major job order: one tile's frame chunks are handed out together and run on
                // neighbouring waves at once, so an expensive tile finishes early instead of trailing
                if (!job_acquire(J, lane, drained, job_tile, job_f0, job_nf)) break;
                job_total = 64u * job_nf;
                job_next = 0;
            }
            const uint32_t avail = job_total - job_next;
            const uint32_t rank = (uint32_t)__popcll(m & below);
            bool took_ok = false;
            if (need && rank < avail) {
                const uint32_t sid = job_next + rank;
                const uint32_t l = sid & 63u;
                fl = sample_ref(J, job_f0, sid >> 6);
                pix = job_tile * 64u + l;
                // (the SAH-walk kernels read the tile map, row map and time through kargs() here: SGPRs)
#define HRT_KF(f) (TSAH ? kargs()->f : P.f)
                const uint32_t x = (job_tile % HRT_KF(tiles_w)) * 8u + (l & 7u);
                const uint32_t kr = (job_tile / HRT_KF(tiles_w)) * 8u + (l >> 3);
                need = false;
                if (x < HRT_KF(W) && kr < HRT_KF(nrows)) {  // ragged edge tiles: samples outside the image are skipped
                    const uint32_t y = global_row(HRT_KF(row0), HRT_KF(row_block), HRT_KF(row_stride), kr);
                    ray = primary_ray<MODE>(&kargs()->cam, x, y, HRT_KF(time0) + (job_f0 + (sid >> 6)) * HRT_KF(dtime), s);
#undef HRT_KF
                    sky_t = ray.d.y * 0.5f + 0.5f;
                    att = mk(1.0f, 1.0f, 1.0f);
                    bounce = 0;
                    have = true;
                    took_ok = true;
                }
            }
            job_dealt(J, (uint32_t)__popcll(__ballot(took_ok)));
            const uint32_t took = min((uint32_t)__popcll(m), avail);
            job_next += took;
            if (job_next == job_total) job_close(J, lane);
            m = __ballot(need);
        }
#ifdef HRT_STAMPS
        st_tb = hrt_stamp();
        if (have) st_gen += st_tb - st_ta;
        if (drained && wrec.drained == 0ull && BQ.job_id != 0xFFFFFFFFu) job_trace_put(P, BQ.job_id, BQ.last_job, hrt_realtime());
        wrec.drain(drained, (uint32_t)__popcll(__ballot(have)));
#endif
        if (__ballot(have) == 0ull) {
            if (drained && J.idle()) break;
            if (!drained && idle_spin(J, lane)) break;  // nothing in flight: the next job waits for its ring slot
        }
        bool fin = false;
        bool done = have;
        if (have && bounce < P.bounces) {
            Hit h;
#ifdef HRT_STAMPS
            const uint32_t boxes0 = tally.boxes;
#endif
            constexpr bool UG = MODE == MODE_SPHERE && HRT_UGUARD_KTRACE != 0;
            const bool hit = closest_hit<MODE, SCAN, TSAH, UG>(P, ray, h, lds_list, tally, tri_cand, tri_stack);
            queries++;
#ifdef HRT_STAMPS
            st_ta = hrt_stamp();
            st_trav += st_ta - st_tb;
            if (bounce == 0) {  // primary queries: count, box tests, lane-cycles
                st_pq++;
                st_pbox += tally.boxes - boxes0;
                st_ptrav += st_ta - st_tb;
            }
            st_tb = st_ta;
#endif
            if (hit) {
                scatter<MODE, UG>(P, s, ray, h);
                att = att * mk(h.ar * 0.7f, h.ag * 0.7f, h.ab * 0.7f);
                bounce++;
                done = bounce >= P.bounces;
            }
        }
        if (done) {
            // trace() epilogue (:241-242): the sample colour, to the fold ring
            const float u = 1.0f - sky_t;
            const f3 sky = mk(0.54f * u + 0.54f * sky_t, 0.86f * u + 0.7f * sky_t, 0.92f * u + 0.98f * sky_t);
            const f3 c = att * sky;
            ring_store(J, pix, fl, c, bounce + 1u);
            have = false;
            fin = true;
        }
#ifdef HRT_STAMPS
        st_shade += hrt_stamp() - st_tb;
        wrec.round((uint32_t)__popcll(__ballot(fin)), BQ.took_job != 0u);
        BQ.took_job = 0u;
#endif
        job_account(J, fin, fl, lane);
    }
#ifdef HRT_STAMPS
    wrec.finish(P, lane, BQ.njobs, BQ.last_job, BQ.max_job);
    {
        // per-lane sums (a lane accrues a region only while it holds a sample): lane-cycles per region;
        // the remainder of the lifetime x 64 is lane-cycles without a sample (refill waits, drain tail)
        unsigned long long v[8] = {st_trav, st_shade, st_gen, hrt_stamp() - st_start, queries,
                                   st_pq, st_pbox, st_ptrav};
#pragma unroll
        for (int c = 0; c < 8; c++) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v[c] += __shfl_xor(v[c], off);
        }
        if (lane == 0) {
            for (int c = 0; c < 4; c++) atomicAdd(P.counter + 8 + c, v[c]);
            const unsigned long long t1 = hrt_stamp(), r1 = hrt_realtime();
            atomicAdd(P.counter + 12, r1 - rt_start);
            atomicAdd(P.counter + 13, 1ull);
            atomicAdd(P.counter + 14, t1 - st_start);
            atomicAdd(P.counter + 5, v[5]);  // primary queries, their box tests and lane-cycles
            atomicAdd(P.counter + 6, v[6]);
            atomicAdd(P.counter + 7, v[7]);
        }
    }
#endif
#ifdef HRT_RINGSTAT
    if (lane == 0)
        for (uint32_t c = 0; c < 4u; c++) atomicAdd(P.counter + 5 + c, (unsigned long long)J.get(WJ_STAT + c));
#endif
    unsigned long long sums[5] = {queries, tally.boxes, tally.spheres, tally.nodes, tally.tris};
#pragma unroll
    for (int c = 0; c < 5; c++) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sums[c] += __shfl_xor(sums[c], off);
    }
    if (lane == 0) flush_counts(sums);
}


// Frame-block refill with the block in LDS (k_trace_split_tris; k_trace_split has the same code inline, which
// compiles spill-free there): when the wave's block (one frame
// of its job's 8x8 tile) is used up, every lane computes its own pixel's primary ray for the next frame at
// once into the wave's slice of `blk` (o, d and, SEED, the RNG state after the primary ray: 7 floats per lane; the
// block's in-image pixels as a 64-bit mask in the wave's two `okw` words — a ragged edge tile's missing pixels take no
// sample; d = 0 is no marker: with focal_length 0 and blur 0 every primary ray of the triangle / mixed programs has
// d = (g / |g|).xyz = 0, and the reference traces it), and lanes that need a sample read theirs. Without
// SEED (6 floats per lane) a taken sample's RNG state is recomputed from its pixel: it starts at (x * H + y) * time
// (primary_ray) = the row's (x0 * H + y) * time + (x - x0) * H * time, per-row words in `rows` (9 per wave), then
// five PCG steps. (Two float4 per lane before round 4: the bytes saved hold the whole heap top.)


template <int MODE, bool STEAL, bool SEED>
__device__ __forceinline__ void refill_block_lds(const KParams& P, BlockState& B, const WaveJobs& J, float* blk,
                                                 uint32_t* rows, uint32_t* okw, bool& drained,
                                                 uint32_t lane, unsigned long long below, bool& have,
                                                 uint32_t& qs, Ray& ray, f3& att, float& sky_t, uint32_t& s,
                                                 uint32_t& bounce, uint32_t& pix, uint32_t& fl) {
    constexpr uint32_t BW = SEED ? 7u : 6u;  // floats per frame-block entry
    bool need = !have && !drained;
    unsigned long long m = __ballot(need);
    while (m != 0ull) {
        if (B.blk_next == 64u) {
            const KPtr K = kargs();  // queue and camera constants: loaded here, not held in SGPRs
            if constexpr (STEAL) {  // one frame block at a time, stolen once the queue is drained (steal_block)
                if ((uint32_t)__popcll(m) < CLAIM_FREE && J.get(WJ_PRIV_N) == 0u && __ballot(have) != 0ull &&
                    queue_drained(J, lane))
                    break;  // (the tail: leave the block to a wave with more free lanes, CLAIM_FREE)
                if (!steal_block(J, lane, B.job_tile, B.job_f0)) {
                    drained = steal_drained(J);
                    break;
                }
                B.blk_f = 0;
                B.job_nf = 1;
            } else {
                if (J.dealing()) {
                    B.blk_f++;
                } else {
                    // (the tail: once this wave dealt a tail part, a new one only for CLAIM_FREE free lanes, as stealing)
                    if (TAIL_CLAIM && (J.get(WJ_FLAGS) & WJ_TAILPH) && (uint32_t)__popcll(m) < CLAIM_FREE && __ballot(have) != 0ull) break;
                    if (!job_acquire<true>(J, lane, drained, B.job_tile, B.job_f0, B.job_nf)) break;
                    B.blk_f = 0;
                }
            }
            B.blk_next = 0;
#ifdef HRT_STAMPS
            B.nblocks++;
#endif
            const uint32_t x = (B.job_tile % K->tiles_w) * 8u + (lane & 7u);
            const uint32_t kr = (B.job_tile / K->tiles_w) * 8u + (lane >> 3);
            const uint32_t pok = (x < K->W && kr < K->nrows) ? 1u : 0u;  // ragged edge tiles: no sample
            Ray pr = {mk(0.0f, 0.0f, 0.0f), mk(0.0f, 0.0f, 0.0f)};
            uint32_t ps = 0;
            const uint32_t y = global_row(K->row0, K->row_block, K->row_stride, kr);
            const uint32_t time = K->time0 + (B.job_f0 + B.blk_f) * K->dtime;
            if (pok) pr = primary_ray<MODE, true>(&kargs()->cam, x, y, time, ps);
            {
                const unsigned long long okm = __ballot(pok != 0u);
                uint32_t* const ow = okw + 2u * (threadIdx.x >> 6);
                if (lane == 0u) {
                    ow[0] = (uint32_t)okm;
                    ow[1] = (uint32_t)(okm >> 32);
                }
            }
            float* const e = blk + BW * threadIdx.x;
            e[0] = pr.o.x;
            e[1] = pr.o.y;
            e[2] = pr.o.z;
            e[3] = pr.d.x;
            e[4] = pr.d.y;
            e[5] = pr.d.z;
            if constexpr (SEED) {
                e[6] = __uint_as_float(ps);
            } else {
                uint32_t* const rw = rows + 9u * (threadIdx.x >> 6);
                if ((lane & 7u) == 0u) rw[lane >> 3] = (x * K->cam.H + y) * time;  // the row's state seed at x0
                if (lane == 0u) rw[8] = K->cam.H * time;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        const uint32_t avail = 64u - B.blk_next;
        const uint32_t rank = (uint32_t)__popcll(m & below);
        const uint32_t src = (B.blk_next + rank) & 63u;
        const float* const e = blk + BW * ((threadIdx.x & ~63u) + src);
        const float ox = e[0], oy = e[1], oz = e[2], dx = e[3], dy = e[4], dz = e[5];
        bool took = false;
        const uint32_t okb = (okw[2u * (threadIdx.x >> 6) + (src >> 5)] >> (src & 31u)) & 1u;
        if (need && rank < avail) {
            need = false;
            if (okb) {  // (a pixel outside the image: no sample)
                ray.o = mk(ox, oy, oz);
                ray.d = mk(dx, dy, dz);
                if constexpr (SEED) {
                    s = __float_as_uint(e[6]);
                } else {
                    const uint32_t* const rw = rows + 9u * (threadIdx.x >> 6);
                    uint32_t st = rw[src >> 3] + (src & 7u) * rw[8];
#pragma unroll
                    for (int k = 0; k < 5; k++) st = pcg_next(st);  // primary_ray's five draws (r1, r2, q1, q2, rr)
                    s = st;
                }
                fl = sample_ref(J, B.job_f0, B.blk_f);
                pix = B.job_tile * 64u + src;
                sky_t = ray.d.y * 0.5f + 0.5f;
                att = mk(1.0f, 1.0f, 1.0f);
                bounce = 0;
                have = true;
                qs = 0;
                took = true;
            }
        }
        job_dealt(J, (uint32_t)__popcll(__ballot(took)));
        B.blk_next += min((uint32_t)__popcll(m), avail);
        if (B.blk_next == 64u && B.blk_f + 1u >= B.job_nf) job_close(J, lane);
        m = __ballot(need);
    }
}

#ifdef HRT_PHASES  // diagnostic build (-DHRT_STAMPS -DHRT_PHASES): wave cycles per phase of a round, phase lanes
#define HRT_PHASE_DECL                                                                       \
    unsigned long long ph[5] = {0, 0, 0, 0, 0}, pl[4] = {0, 0, 0, 0}, pr[4] = {0, 0, 0, 0}; \
    const unsigned long long ph_start = hrt_stamp();                                         \
    unsigned long long ph_t = ph_start
#define HRT_PHASE(k)                                                                         \
    do {                                                                                     \
        const unsigned long long t_ = hrt_stamp();                                          \
        ph[k] += t_ - ph_t;                                                                  \
        ph_t = t_;                                                                           \
    } while (0)
#define HRT_LANES(k, pred)                                                                   \
    do {                                                                                     \
        const uint32_t c_ = (uint32_t)__popcll(__ballot(pred));                              \
        if (c_) { pl[k] += c_; pr[k]++; }                                                    \
    } while (0)
// counter[8..11] wave cycles in refill, begin, walk, shade (+ job accounting); [12] wave lifetime cycles;
// [5] / [6] / [7] lanes summed over the rounds that ran begin / walk / shade, [13] / [14] the rounds that ran
// begin / shade (phase utilisation = lanes / rounds)
#define HRT_PHASE_FLUSH                                                                      \
    if (lane == 0) {                                                                         \
        for (int k = 0; k < 4; k++) atomicAdd(P.counter + 8 + k, ph[k]);                     \
        atomicAdd(P.counter + 12, hrt_stamp() - ph_start);                                   \
        for (int k = 0; k < 3; k++) atomicAdd(P.counter + 5 + k, pl[k]);                     \
        atomicAdd(P.counter + 13, pr[0]);                                                    \
        atomicAdd(P.counter + 14, pr[2]);                                                    \
    }
#else
#define HRT_PHASE_DECL do { } while (0)
#define HRT_PHASE(k) do { } while (0)
#define HRT_LANES(k, pred) do { } while (0)
#define HRT_PHASE_FLUSH
#endif

// Sample queue with suspendable walks (sphere program, culling BVH; rt_params.suspend_below > 0).
// In k_trace a wave's query step lasts as long as its slowest lane's walk: secondary rays of one wave
// take very different paths through the tree, so most lanes idle at the end of every step (PMC of
// k_trace on C3: 26 of 64 lanes active per VALU instruction). Here the walk is suspended, state kept
// (BvhQuery in registers, stack in LDS), as soon as fewer than `suspend_below` lanes of the wave are still
// walking; the finished lanes shade, start their next query (or sample) and all lanes walk on together.
// Every lane computes exactly the same query as k_trace, so the sample colours are bit-identical.
// 7 waves per SIMD (72-VGPR budget, no spills since bvh_run recomputes a = d.d instead of carrying it): the
// frame block lives in LDS (8 KB per workgroup)
// next to a 14-entry stack (14 KB), 22 KB x 7 workgroups fitting the CU's 160 KB. Measured on C3: block in
// VGPRs at 6 waves (20-entry stack) 26.1 Grays/s, block in LDS at 7 waves 26.5; per-lane primary rays were
// 24.5. A stack overflow (BVH deeper than 14 along a path) falls back to the exact full scan.
// LNODES (small trees: <= LNODE_CAP nodes, depth <= 8): the fp16 nodes are copied into LDS once per
// workgroup and the stack shrinks to 8 entries (a path holds at most depth pending siblings), 22 KB in all.
// STEAL: frame-block work stealing (sample buffer; renderer.cpp turns it on for launches with few jobs per wave).
// A separate instantiation: the runtime-switched form cost C3 3 % with stealing off (register allocation).
// PACKET (with LNODES; rt_params.packet): each frame block's primary rays are walked as one packet when the block is
// made (packet_walk: all 64 lanes, wave-uniform traversal), and the block entry carries the resolved first hit — the
// hit point in place of the origin and the winner's slot — so a lane that takes the sample shades it at once (qs 4)
// instead of walking its primary ray beside the wave's incoherent secondary walks. Same bits and query counts.
template <bool LNODES, bool STEAL, bool COUNT, bool PACKET>
#ifndef HRT_PACKET_WAVES
#define HRT_PACKET_WAVES 7
#endif
#ifndef HRT_PACKET_STEAL_WAVES
#define HRT_PACKET_STEAL_WAVES 6  // (the stealing packet kernel spills 6 VGPRs at 7 waves)
#endif
#ifndef HRT_SPLIT_WAVES
#define HRT_SPLIT_WAVES 7
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PACKET ? (STEAL ? HRT_PACKET_STEAL_WAVES : HRT_PACKET_WAVES) : HRT_SPLIT_WAVES))) void k_trace_split(const KParams P) {
    static_assert(!PACKET || LNODES, "the packet walk reads the LDS nodes and keeps its stack in one VGPR (depth <= 8)");
    constexpr int MODE = MODE_SPHERE;
    constexpr int SPLIT_STACK = LNODES ? (int)LNODE_DEPTH : 14;
    const uint32_t lane = threadIdx.x & 63u;
    __shared__ uint32_t bvh_stack[SPLIT_STACK * 256];
    __shared__ uint4 lnodes[LNODES ? 2 * LNODE_CAP : 1];
    if constexpr (LNODES) {
        const uint32_t nn = 2u * min(P.bvh_nnodes, LNODE_CAP);  // renderer.cpp gates LNODES on the same cap
        for (uint32_t i = threadIdx.x; i < nn; i += 256u) lnodes[i] = P.bvh_hnodes[i];
        __syncthreads();
    }
    __shared__ float4 blk[2 * 256];  // the wave's frame block: (o.xyz, d.x), (d.yz, state bits, ok) per lane
    uint32_t* const stack = bvh_stack + threadIdx.x;
    Tally tally;
    uint32_t queries = 0;
    const unsigned long long below = (1ull << lane) - 1ull;
    const uint32_t suspend_below = P.suspend_below;

    bool drained = false;
    Ray ray;
    f3 att = mk(1.0f, 1.0f, 1.0f);
    float sky_t = 0.0f;
    uint32_t s = 0, bounce = 0, pix = 0, fl = 0;
    bool have = false;
    uint32_t qs = 0;  // query state of the lane's sample: 0 start a query, 1 walking, 2 walk finished
    BvhQuery Q;
    // Primary rays are generated a frame-block at a time: when the wave's block (one frame of its job's
    // 8x8 tile) is used up, every lane computes the primary ray of its own pixel for the next frame at
    // once (all lanes busy) into the wave's slice of `blk`, and lanes that need a sample read theirs from
    // it, instead of each freed lane computing its own with a few lanes active.
    uint32_t job_tile = 0, job_f0 = 0, job_nf = 0, blk_f = 0, blk_next = 64;  // wave-uniform
    __shared__ uint32_t wjobs[4 * WJ_WORDS];
    const WaveJobs J = wave_jobs(wjobs);
    if (P.fold_prev != nullptr) fold_prev_tiles(P, lane);
    HRT_PHASE_DECL;
#ifdef HRT_STAMPS
    WaveRecord wrec;
    wrec.begin();
    uint32_t nblocks = 0;
#endif
    while (true) {
        bool need = !have && !drained;
        unsigned long long m = __ballot(need);
        while (m != 0ull) {
            if (blk_next == 64u) {
                if constexpr (STEAL) {  // one frame block at a time, stolen once the queue is drained (steal_block)
                    if ((uint32_t)__popcll(m) < CLAIM_FREE && J.get(WJ_PRIV_N) == 0u && __ballot(have) != 0ull &&
                        queue_drained(J, lane))
                        break;  // (the tail: leave the block to a wave with more free lanes, CLAIM_FREE)
                    if (!steal_block(J, lane, job_tile, job_f0)) {
                        drained = steal_drained(J);
                        break;
                    }
                    blk_f = 0;
                    job_nf = 1;
                } else {
                    if (J.dealing()) {
                        blk_f++;
                    } else {
                        // (the tail: once this wave dealt a tail part, a new one only for CLAIM_FREE free lanes, as stealing)
                        if (TAIL_CLAIM && (J.get(WJ_FLAGS) & WJ_TAILPH) && (uint32_t)__popcll(m) < CLAIM_FREE && __ballot(have) != 0ull)
                            break;
                        if (!job_acquire<true>(J, lane, drained, job_tile, job_f0, job_nf)) break;
                        blk_f = 0;
                    }
                }
                blk_next = 0;
#ifdef HRT_STAMPS
                nblocks++;
#endif
                const uint32_t x = (job_tile % P.tiles_w) * 8u + (lane & 7u);
                const uint32_t kr = (job_tile / P.tiles_w) * 8u + (lane >> 3);
                const uint32_t pok = (x < P.W && kr < P.nrows) ? 1u : 0u;  // ragged edge tiles: no sample
                Ray pr = {mk(0.0f, 0.0f, 0.0f), mk(0.0f, 0.0f, 0.0f)};
                uint32_t ps = 0;
                uint32_t ew = pok;  // entry word: bit 0 in the image, PACKET: bit 1 resolved, bit 2 hit, slot << 3
                if (pok) {
                    const KPtr K = kargs();  // row map and time: loaded here, not held in SGPRs
                    const uint32_t y = global_row(K->row0, K->row_block, K->row_stride, kr);
                    pr = primary_ray<MODE>(&K->cam, x, y, K->time0 + (job_f0 + blk_f) * K->dtime, ps);
                }
                blk[2 * threadIdx.x] = float4{pr.o.x, pr.o.y, pr.o.z, pr.d.x};
                blk[2 * threadIdx.x + 1] = float4{pr.d.y, pr.d.z, __uint_as_float(ps), __uint_as_float(ew)};
                if constexpr (PACKET) {
                    // (bounce cap 0: no query; rays bvh_begin leaves to the full scan: resolved later, qs 0)
#ifndef HRT_PACKET_DRY
#define HRT_PACKET_DRY 0  // (A/B builds only: 1 = the packet kernel without its walk, every primary ray unresolved)
#endif
                    if (P.bounces > 0u && !HRT_PACKET_DRY) {  // (wave-uniform: every lane enters the packet walk)
                        BvhQuery Qp;
                        // slab constants only (bvh_begin's uncovered-ray rule); the large list after the walk: the
                        // (t, slot) minimum does not depend on the order, and the walk then holds fewer registers
                        const float a2 = 2.0f * dot(pr.d, pr.d);
                        const bool cov = pok && (a2 > 0x1p-100f && a2 < 0x1p100f) && __builtin_isfinite(pr.o.x) &&
                                         __builtin_isfinite(pr.o.y) && __builtin_isfinite(pr.o.z);
                        Qp.bt = cov ? FLT_MAX_REF : -1.0f;  // (-1: no test passes)
                        Qp.bc = -1;
                        bvh_slab<true, true>(P, pr, Qp);
                        if (packet_walk<COUNT>(P, blk + 2 * threadIdx.x, Qp, lnodes, tally, cov) && cov) {
                            // the entry: the hit point in place of the origin and the winner's slot, or a resolved miss
                            // (everything re-read from the entry: nothing of the block kept in registers through the walk)
                            uint32_t rw = 3u;
                            const float4 e0 = blk[2 * threadIdx.x], e1 = blk[2 * threadIdx.x + 1];
                            const Ray re = {mk(e0.x, e0.y, e0.z), mk(e0.w, e1.x, e1.y)};
                            {
                                const float a = dot(re.d, re.d);
                                const uint32_t nlarge = kargs()->nlarge;
                                for (uint32_t k = 0; k < nlarge; k++) {
                                    const int i = P.large_slots[k];
                                    const float t = exact_t_geo<true>(P.sph_geo[i], re, 4.0f * a, 2.0f * a);
                                    if (beats(t, i, Qp.bt, Qp.bc >= 0 ? bvh_slot_of(P, Qp.bc) : -1)) {
                                        Qp.bt = t;
                                        Qp.bc = (int)(P.bvh_nleaf + k);
                                    }
                                }
                                if constexpr (COUNT) tally.spheres += nlarge;
                            }
                            if (Qp.bc >= 0) {
                                const f3 ph = point_on_ray(re.o, re.d, Qp.bt);
                                blk[2 * threadIdx.x].x = ph.x;
                                blk[2 * threadIdx.x].y = ph.y;
                                blk[2 * threadIdx.x].z = ph.z;
                                rw = 7u | ((uint32_t)bvh_slot_of(P, Qp.bc) << 3);
                            }
                            blk[2 * threadIdx.x + 1].w = __uint_as_float(rw);
                        }
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            const uint32_t avail = 64u - blk_next;
            // (PACKET: the rank by mbcnt, no 64-bit lane mask held in VGPRs — the packet kernel's register budget; the
            // other instantiations keep the mask: same-box A/B, the mbcnt form cost C3 0.3 %)
            const uint32_t rank = PACKET ? __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))
                                         : (uint32_t)__popcll(m & below);
            const int src = (int)((blk_next + rank) & 63u);
            const float4 b0 = blk[2 * ((threadIdx.x & ~63u) + (uint32_t)src)];
            const float4 b1 = blk[2 * ((threadIdx.x & ~63u) + (uint32_t)src) + 1];
            const float ox = b0.x, oy = b0.y, oz = b0.z, dx = b0.w, dy = b1.x, dz = b1.y;
            const uint32_t ss = __float_as_uint(b1.z), ok = __float_as_uint(b1.w);
            bool took = false;
            if (need && rank < avail) {
                need = false;
                if (ok & 1u) {
                    ray.o = mk(ox, oy, oz);  // (PACKET, resolved hit: the hit point)
                    ray.d = mk(dx, dy, dz);
                    s = ss;
                    fl = sample_ref(J, job_f0, blk_f);
                    pix = job_tile * 64u + (uint32_t)src;
                    sky_t = ray.d.y * 0.5f + 0.5f;
                    att = mk(1.0f, 1.0f, 1.0f);
                    bounce = 0;
                    have = true;
                    qs = 0;
                    if constexpr (PACKET) {
                        if (ok & 2u) {  // resolved by the packet: shade at once, the winner's slot (or -1) in Q.bc
                            qs = 4u;
                            Q.bc = (ok & 4u) ? (int)(ok >> 3) : -1;
                        }
                    }
                    took = true;
                }
            }
            job_dealt(J, (uint32_t)__popcll(__ballot(took)));
            blk_next += min((uint32_t)__popcll(m), avail);
            if (blk_next == 64u && blk_f + 1u >= job_nf) job_close(J, lane);
            m = __ballot(need);
        }
#ifdef HRT_STAMPS
        wrec.drain(drained);
#endif
        if (__ballot(have) == 0ull) {
            if (drained && J.idle()) break;
            if (!drained && idle_spin(J, lane)) break;  // nothing in flight: the next job waits for its ring slot
        }
        bool fin = false;
#ifdef HRT_STAMPS
        if (lane == 0) tally.rounds++;
#endif
        HRT_PHASE(0);
        HRT_LANES(0, have && qs == 0u);
        if (have && qs == 0u) {
            if (bounce < P.bounces) {
                qs = bvh_begin<true, true, true, true, COUNT>(P, ray, FLT_MAX_REF, Q, tally) ? 1u : 2u;
            } else {  // bounce cap 0: the sample is the sky colour
                qs = 3u;
            }
        }
        HRT_PHASE(1);
        HRT_LANES(1, have && qs == 1u);
        if (have && qs == 1u) {
            if constexpr (LNODES) {  // (depth <= LNODE_DEPTH = SPLIT_STACK: no overflow)
                if (bvh_run<true, SPLIT_STACK, true, true, 256, true, true, COUNT>(P, ray, Q, stack, tally, suspend_below, lnodes))
                    qs = 2u;
            } else {
                if (bvh_run<true, SPLIT_STACK, true, true, 256, false, true, COUNT>(P, ray, Q, stack, tally, suspend_below, P.bvh_hnodes))
                    qs = 2u;
            }
        }
        HRT_PHASE(2);
        HRT_LANES(2, have && qs >= 2u);
        // (PACKET: the queries shaded this round counted per wave — a wave-uniform count needs no VGPR; the others count
        // per lane, as before)
        if constexpr (PACKET) queries += (uint32_t)__popcll(__ballot(have && (qs == 2u || qs == 4u)));
        if (have && qs >= 2u) {
#ifdef HRT_STAMPS
            tally.lshade++;
            if (first_active_lane()) tally.wshade++;
#endif
            bool done = true;
            if (qs == 2u || (PACKET && qs == 4u)) {
                float best = FLT_MAX_REF;
                int bi;
                f3 p;
                if (PACKET && qs == 4u) {  // a primary ray the packet resolved: ray.o is its hit point
                    bi = Q.bc;
                    p = ray.o;
                } else {
                    bi = bvh_end<true>(P, ray, Q, best, tally);
                    p = point_on_ray(ray.o, ray.d, best);
                }
                if constexpr (!PACKET) queries++;
                if (bi >= 0) {
                    Hit h;
#ifndef HRT_UGUARD
#define HRT_UGUARD 1
#endif
                    sphere_record_p<HRT_UGUARD != 0>(P, p, ray.d, bi, best, h);
                    scatter<MODE, HRT_UGUARD != 0>(P, s, ray, h);
                    att = att * mk(h.ar * 0.7f, h.ag * 0.7f, h.ab * 0.7f);
                    bounce++;
                    done = bounce >= P.bounces;
                }
            }
            if (done) {
                const float u = 1.0f - sky_t;
                const f3 sky = mk(0.54f * u + 0.54f * sky_t, 0.86f * u + 0.7f * sky_t, 0.92f * u + 0.98f * sky_t);
                const f3 c = att * sky;
                ring_store(J, pix, fl, c, bounce + 1u);
                have = false;
                fin = true;
            }
            qs = 0u;
        }
        job_account<1>(J, fin, fl, lane);
        HRT_PHASE(3);
    }
#ifdef HRT_STAMPS
    wrec.finish(P, lane, nblocks);
#endif
    HRT_PHASE_FLUSH
#if defined(HRT_STAMPS) && !defined(HRT_PHASES)
    {
        unsigned long long v[10] = {tally.lbox, tally.wbox, tally.lleaf, tally.wleaf, tally.rounds, tally.lshade,
                                    tally.wshade, tally.lwalk, tally.wwalk, tally.lentry};
#pragma unroll
        for (int c = 0; c < 10; c++) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v[c] += __shfl_xor(v[c], off);
        }
        if (lane == 0)
            for (int c = 0; c < 10; c++) atomicAdd(P.counter + 5 + c, v[c]);  // counters 5-14 ([15] is the job queue)
    }
#endif
#ifdef HRT_RINGSTAT
    if (lane == 0)
        for (uint32_t c = 0; c < 4u; c++) atomicAdd(P.counter + 5 + c, (unsigned long long)J.get(WJ_STAT + c));
#endif
    unsigned long long sums[5] = {(!PACKET || lane == 0u) ? queries : 0u, tally.boxes, tally.spheres, tally.nodes, tally.tris};
#pragma unroll
    for (int c = 0; c < 5; c++) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sums[c] += __shfl_xor(sums[c], off);
    }
    if (lane == 0) flush_counts(sums);
}

// Sample queue with suspendable walks for the triangle and mixed programs (reference heap walk; the
// sphere part of the mixed program is `SCAN`: the linear scan, simple or deferred, or the culling BVH
// walked to completion). A lane's query goes begin (sphere scan) -> heap walk -> shade; the wave
// suspends the heap walk once fewer than `suspend_below` lanes are still walking, so lanes whose rays
// miss the mesh (one node test) do not idle behind the wave's longest walk (C4: 7.0 -> 8.2 Grays/s;
// C5: 6.25 -> 6.55). Bit-identical to k_trace, with the same node/triangle counts.
// HL: the heap's top in LDS (renderer.cpp decides: rt_params.heap_lds not 1 (off), and with the culling BVH a
// sphere tree of depth <= 8, whose walk fits the 8-entry stack). 0: none, 256-lane workgroups, a 16-entry leaf-pair
// list per lane; 1, 3: an 8-entry leaf-pair list (32-bit entries: j0 | PAIR_BIT) that shares its words with the
// 8-entry sphere-walk stack, which makes room for the heap's top at 6 waves per SIMD: 3 = nodes 1..1023 of sign-ordered
// 36-B nodes, the whole heap of a tree of up to 1024 nodes (Suzanne), with 768-lane workgroups (two per CU: 80 KB
// each), the default (1..991 in the 32-B layout before; 881 / 971 / 1023 nodes: C4 11.77 / 12.09 / 12.74 Grays/s); 1 = nodes 1..255 (9 KB) with 256-lane workgroups, only for the mixed program's
// deferred sphere scan (its candidate lists assume 256 lanes). (Nodes 1..511 with 512-lane workgroups, measured
// between the two in round 3, was retired.)
constexpr uint32_t heap_wg(int hl) { return hl == 3 ? 768u : 256u; }
// Every HL3 kernel holds the whole heap of a tree of up to 1024 nodes (Suzanne: nodes 1..1023) in LDS, so the walk
// reads nothing but LDS (FULL): the linear sphere scans (no sphere-walk stack in the list words) with a 7-entry list,
// the culling-BVH sphere walk (8-entry stack) with 24-B frame-block entries (refill_block_lds)
constexpr uint32_t heap_list_words(int hl, int scan) { return hl == 0 ? TRI_BATCH : (hl == 3 && scan != SCAN_BVH) ? 7u : 8u; }
constexpr uint32_t heap_top_n(int hl, int scan) { return hl == 0 ? 0u : hl == 1 ? 256u : 1024u; }

#ifndef HRT_HEAP_FAST_BVH
#define HRT_HEAP_FAST_BVH 0  // (1: the culling-BVH mixed kernel (C5) takes heap_begin's refined reciprocals too: -0.2 %)
#endif
#ifndef HRT_UGUARD_TRIS
#define HRT_UGUARD_TRIS 1  // (the mixed kernels' sphere hit record with the linear scan (C4): its normal division's guard as
#endif                     //  a wave-uniform branch, +0.3 %; with the culling BVH (C5) -0.1 %, so not there)
template <int MODE, int SCAN, int HL, bool STEAL>
__global__ __launch_bounds__(heap_wg(HL)) __attribute__((amdgpu_waves_per_eu(SCAN == SCAN_DEFER ? 5 : 6))) void
k_trace_split_tris(const KParams P) {
    static_assert(MODE != MODE_SPHERE, "k_trace_split covers the sphere program");
    constexpr uint32_t WGT = heap_wg(HL), HT = heap_top_n(HL, SCAN);
    const uint32_t lane = threadIdx.x & 63u;
    // per-lane deferred-triangle list (leaf-pair entries); with the culling BVH also the sphere walk's stack (never
    // live together: the sphere scan finishes in the begin phase)
    constexpr uint32_t LIST_WORDS = heap_list_words(HL, SCAN);
    constexpr int SPHERE_STACK = (int)LIST_WORDS;
    static_assert(SCAN != SCAN_BVH || HL == 0 || LIST_WORDS == 8, "the culling walk's stack needs 8 entries");
    __shared__ uint32_t lane_words[LIST_WORDS * WGT];
    uint32_t* const cand = lane_words + threadIdx.x;  // entry k at cand[k * WGT]: a lane's entries stay in its own words
    uint32_t* const sstack = lane_words + threadIdx.x;
    __shared__ float heap_top[HL > 0 ? 9 * HT : 1];  // sign-ordered nodes 0 .. HT - 1 (node_hit_so)
    if constexpr (HL > 0) {
        const uint32_t nf = 9u * min(P.n, HT);
        for (uint32_t t = threadIdx.x; t < nf; t += WGT) heap_top[t] = P.nodes_so[t];
        __syncthreads();
    }
    uint16_t* defer_list = nullptr;
    if constexpr (SCAN == SCAN_DEFER) {
        static_assert(HL <= 1, "the deferred scan's lists assume 256-lane workgroups");
        __shared__ uint16_t defer_cand[(CAND_CAP + 1) * 256];
        defer_list = defer_cand + threadIdx.x;
    }
    Tally tally;
    uint32_t queries = 0;
    const unsigned long long below = (1ull << lane) - 1ull;
    const uint32_t suspend_below = P.suspend_below;

    // the wave's frame block (refill_block_lds): the seed stored (7 floats per lane) unless the culling-BVH sphere walk's
    // 8-entry stack needs the list words (6 floats per lane, the seed recomputed: C5 +4.6 %, C4 -1.4 %)
    constexpr bool SEED = !(HL == 3 && SCAN == SCAN_BVH);
    __shared__ float blk[(SEED ? 7 : 6) * WGT];
    __shared__ uint32_t blk_rows[SEED ? 1 : 9 * (WGT / 64u)];
    __shared__ uint32_t blk_ok[2 * (WGT / 64u)];  // per wave: the block's in-image pixels (64-bit mask)
    BlockState B;
    __shared__ uint32_t wjobs[(WGT / 64u) * WJ_WORDS];
    const WaveJobs J = wave_jobs(wjobs);
    if (P.fold_prev != nullptr) fold_prev_tiles(P, lane);
    bool drained = false;
    Ray ray;
    f3 att = mk(1.0f, 1.0f, 1.0f);
    float sky_t = 0.0f;
    uint32_t s = 0, bounce = 0, pix = 0, fl = 0;
    bool have = false;
    // query state: 0 start, 3 heap walk, 4 shade, 5 sky only
    uint32_t qs = 0;
    // the sphere winner rides in the heap walk's winner code: W.bj = -2 - slot until a triangle beats it (-1: no hit)
    HeapWalk W;
    HRT_PHASE_DECL;
#ifdef HRT_STAMPS
    WaveRecord wrec;
    wrec.begin();
#endif
    while (true) {
        refill_block_lds<MODE, STEAL, SEED>(P, B, J, blk, blk_rows, blk_ok, drained, lane, below, have, qs, ray, att, sky_t, s,
                                            bounce, pix, fl);
#ifdef HRT_STAMPS
        wrec.drain(drained);
#endif
        if (__ballot(have) == 0ull) {
            if (drained && J.idle()) break;
            if (!drained && idle_spin(J, lane)) break;  // nothing in flight: the next job waits for its ring slot
        }
        HRT_PHASE(0);
        HRT_LANES(0, have && qs == 0u);
        bool fin = false;
        if (have && qs == 0u) {
            if (bounce >= P.bounces) {
                qs = 5u;  // bounce cap 0: the sample is the sky colour
            } else if constexpr (MODE == MODE_TRIS) {
                heap_begin(ray, FLT_MAX_REF, W);
                qs = 3u;
            } else {
                float sb = FLT_MAX_REF;
                int bi;
                // (HL > 0: renderer.cpp runs these only for sphere trees of depth <= 8 = SPHERE_STACK: no overflow)
                if constexpr (SCAN == SCAN_BVH) bi = scan_spheres_bvh<SPHERE_STACK, true, WGT, true, (HL > 0), true>(P, ray, sb, sstack, tally);
                else if constexpr (SCAN == SCAN_DEFER) bi = scan_spheres_deferred(P, ray, sb, defer_list);
                else bi = scan_spheres(P, ray, sb);
                if constexpr (SCAN != SCAN_BVH) tally.spheres += P.nslots;  // the BVH scan counts its own
                heap_begin<SCAN != SCAN_BVH || HRT_HEAP_FAST_BVH != 0>(ray, sb, W);
                W.bj = -2 - bi;
                qs = 3u;
            }
        }
        HRT_PHASE(1);
        HRT_LANES(1, have && qs == 3u);
        if (have && qs == 3u) {
            // (triangles through a buffer descriptor: C4 +0.7 %; the culling-BVH mixed kernel makes room for it by reading
            // its sphere walk's rare-path constants through kargs(): C5 +1.2 %)
            bool walked;
            if constexpr (HL > 0) {
                // the sign-ordered node test unless a walking lane has a non-finite 1/d or origin (node_hit_so)
                const bool fin3 = __builtin_isfinite(W.inv.x) && __builtin_isfinite(W.inv.y) && __builtin_isfinite(W.inv.z) &&
                                  __builtin_isfinite(ray.o.x) && __builtin_isfinite(ray.o.y) && __builtin_isfinite(ray.o.z);
                constexpr bool CAN_FULL = HT >= 1024u;
                if (P.so_ok && __ballot(!fin3) == 0ull) {
                    if (CAN_FULL && kargs()->n <= HT)  // (a fresh scalar load: the flag held in SGPRs spilled)
                        walked = heap_run<true, HT, WGT, LIST_WORDS, true, true, CAN_FULL>(P, ray, W, tally, cand, suspend_below, heap_top);
                    else
                        walked = heap_run<true, HT, WGT, LIST_WORDS, true, true>(P, ray, W, tally, cand, suspend_below, heap_top);
                } else
                    walked = heap_run<true, HT, WGT, LIST_WORDS, true, false>(P, ray, W, tally, cand, suspend_below, heap_top);
            } else {
                walked = heap_run<true, HT, WGT, LIST_WORDS, true>(P, ray, W, tally, cand, suspend_below);
            }
            if (walked) qs = 4u;
        }
        HRT_PHASE(2);
        HRT_LANES(2, have && qs >= 4u);
        if (have && qs >= 4u) {
            bool done = true;
            if (qs == 4u) {
                queries++;
                Hit h;
                bool hit = true;
                if (W.bj >= 0) tri_record(P, ray, P.tris[W.bj], W.best, h);
                else if (W.bj <= -2) sphere_record<HRT_UGUARD_TRIS != 0 && SCAN != SCAN_BVH>(P, ray, -2 - W.bj, W.best, h);
                else hit = false;
                if (hit) {
                    scatter<MODE>(P, s, ray, h);
                    att = att * mk(h.ar * 0.7f, h.ag * 0.7f, h.ab * 0.7f);
                    bounce++;
                    done = bounce >= P.bounces;
                }
            }
            if (done) {
                const float u = 1.0f - sky_t;
                const f3 sky = mk(0.54f * u + 0.54f * sky_t, 0.86f * u + 0.7f * sky_t, 0.92f * u + 0.98f * sky_t);
                const f3 c = att * sky;
                ring_store(J, pix, fl, c, bounce + 1u);
                have = false;
                fin = true;
            }
            qs = 0u;
        }
        job_account<SCAN == SCAN_BVH ? 1 : 2>(J, fin, fl, lane);
        HRT_PHASE(3);
    }
#ifdef HRT_STAMPS
    wrec.finish(P, lane, B.nblocks);
#ifndef HRT_PHASES
    {
        // the begin phase's sphere walk (scripts/diag_tris.py): counter[5..14]
        unsigned long long v[10] = {tally.lbox, tally.wbox, tally.lleaf, tally.wleaf, tally.lbox_low, tally.wbox_low,
                                    tally.lleaf_low, tally.wleaf_low, tally.lentry, tally.wentry};
#pragma unroll
        for (int c = 0; c < 10; c++) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v[c] += __shfl_xor(v[c], off);
        }
        if (lane == 0)
            for (int c = 0; c < 10; c++) atomicAdd(P.counter + 5 + c, v[c]);
    }
#endif
#endif
    HRT_PHASE_FLUSH
#ifdef HRT_RINGSTAT
    if (lane == 0)
        for (uint32_t c = 0; c < 4u; c++) atomicAdd(P.counter + 5 + c, (unsigned long long)J.get(WJ_STAT + c));
#endif
    unsigned long long sums[5] = {queries, tally.boxes, tally.spheres, tally.nodes, tally.tris};
#pragma unroll
    for (int c = 0; c < 5; c++) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sums[c] += __shfl_xor(sums[c], off);
    }
    if (lane == 0) flush_counts(sums);
}

// Sample buffer (ring_mode 0): folds P.nframes sample colours per pixel into the image, in frame order, with the
// expression k_render uses (WGSL mix, shader_sphere.wgsl:264-271). One thread per tile-padded pixel, in the
// buffer's tile-major order, so the frame-major colour reads are contiguous across the wave.
__global__ __launch_bounds__(256) void k_accumulate(const KParams P) {
    const size_t npad = (size_t)P.tiles_w * P.tiles_h * 64u;
    const size_t q = (size_t)blockIdx.x * 256u + threadIdx.x;
    if (q >= npad) return;
    const uint32_t tile = (uint32_t)(q >> 6), l = (uint32_t)(q & 63u);
    const uint32_t x = (tile % P.tiles_w) * 8u + (l & 7u);
    const uint32_t kr = (tile / P.tiles_w) * 8u + (l >> 3);
    if (x >= P.W || kr >= P.nrows) return;
    const uint32_t wtile = __builtin_amdgcn_readfirstlane(tile);  // (a wave is one tile)
    fold_pixel<8>(P.image + ((size_t)kr * P.W + x) * 3u, P.samples + (size_t)wtile * 192u, l * 3u, npad * 3u, P.nframes,
                  P.frame0, P.ema_cap);
}

hipError_t hrt_launch_accumulate(const KParams& P, hipStream_t stream) {
    const size_t npad = (size_t)P.tiles_w * P.tiles_h * 64u;
    if (npad == 0 || P.nframes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_accumulate, dim3((unsigned)((npad + 255u) / 256u)), dim3(256), 0, stream, P);
    return hipGetLastError();
}

// Cost-ordered dealing (rt_params.cost_order; renderer.cpp): a learning launch sums its samples' queries per pixel
// (pixel_cost, ring_store); the tiles are then split into a head — the most expensive ones, at most ORDER_HEAD_PCT (50) % of
// them, by log-scale cost classes — sorted by class, most expensive first (raster order within a class at the grain of
// ORDER_BLOCK tiles), and the rest in raster order; later launches deal the head first (job_acquire, steal_block_claim:
// tile_order[job / nchunks]). A tile whose paths bounce up to the cap costs many times a sky tile; dealt late, its jobs
// outlast the launch. A full sort by cost measured slower: the GPU then works on tiles from all over the image at once
// (C4 -2.3 %, C2 -5 %, C3 -0.8 % on full images: the rays of a band of adjacent tiles share their scene data in the
// caches); the head's expensive tiles cluster on the same objects. Which wave traces a sample never changes its colour
// or its place in the sample buffer, so the image is bit-identical in any order.
#ifndef HRT_ORDER_HEAD_PCT
#define HRT_ORDER_HEAD_PCT 50  // (12 / 25 / 50 / 100: C4 8-way 0.82 / 0.82 / 0.84 / 0.83, C2 0.66 / 0.65 / 0.66 / 0.65; profiles/r05/v/)
#endif
constexpr uint32_t ORDER_BUCKETS = 128, ORDER_HEAD_PCT = HRT_ORDER_HEAD_PCT, ORDER_BLOCK = 1024;
__device__ __forceinline__ uint32_t order_bucket(uint32_t cost) {
    // floor(4 * log2(cost + 1)) from the float's exponent and top two significand bits (cost + 1 >= 1, <= 2^32: the
    // class of 2^32 is clamped), most expensive first
    const uint32_t k = (__float_as_uint((float)cost + 1.0f) >> 21) - (127u << 2);
    return (ORDER_BUCKETS - 1u) - min(k, ORDER_BUCKETS - 1u);
}
// scratch words: [0, 128) class histogram (zero between sorts), [128] the head's classes (class < cut), [129] head
// size, [256, 384) the head classes' first positions, [384, 384 + blocks) head tiles per ORDER_BLOCK tiles, then their
// exclusive prefix sums, then blocks x 128 head tiles per block and class, then the positions where they go
constexpr uint32_t OS_HIST = 0, OS_CUT = ORDER_BUCKETS, OS_NHEAD = ORDER_BUCKETS + 1, OS_CBASE = 2 * ORDER_BUCKETS,
                   OS_BLK = 3 * ORDER_BUCKETS;
__device__ __forceinline__ uint32_t os_cls(uint32_t nblocks, uint32_t blk, uint32_t c) {
    return OS_BLK + nblocks + blk * ORDER_BUCKETS + c;
}
// one wave per tile: the tile's 64 pixel counters summed (saturating) into tile_sum and zeroed for the next learning
// launch, the tile's class counted
__global__ __launch_bounds__(256) void k_order_hist(uint32_t* __restrict__ pixel_cost, uint32_t ntiles,
                                                    uint32_t* __restrict__ tile_sum, uint32_t* scratch) {
    __shared__ uint32_t h[ORDER_BUCKETS];
    for (uint32_t b = threadIdx.x; b < ORDER_BUCKETS; b += 256u) h[b] = 0u;
    __syncthreads();
    const uint32_t t = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (t < ntiles) {  // (wave-uniform)
        unsigned long long v = pixel_cost[(size_t)t * 64u + lane];
        pixel_cost[(size_t)t * 64u + lane] = 0u;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0u) {
            const uint32_t c = (uint32_t)min(v, 0xFFFFFFFFull);
            tile_sum[t] = c;
            atomicAdd(&h[order_bucket(c)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < ORDER_BUCKETS; b += 256u)
        if (h[b]) atomicAdd(scratch + OS_HIST + b, h[b]);
}
// one thread: the head = the most expensive classes holding at most ORDER_HEAD_PCT % of the tiles (the histogram
// zeroed for the next sort)
__global__ void k_order_cut(uint32_t* scratch, uint32_t ntiles) {
    if (threadIdx.x != 0u) return;
    const uint32_t cap = (uint32_t)((unsigned long long)ntiles * ORDER_HEAD_PCT / 100u);
    uint32_t n = 0, cut = 0;
    bool open = true;
    for (uint32_t b = 0; b < ORDER_BUCKETS; b++) {
        const uint32_t c = scratch[OS_HIST + b];
        scratch[OS_HIST + b] = 0u;
        if (open && n + c <= cap) {
            scratch[OS_CBASE + b] = n;
            n += c;
            cut = b + 1u;
        } else {
            open = false;
        }
    }
    scratch[OS_CUT] = cut;
    scratch[OS_NHEAD] = n;
}
// head tiles per block of ORDER_BLOCK tiles (256 threads x 4 tiles), in all and per class
__global__ __launch_bounds__(256) void k_order_count(const uint32_t* __restrict__ tile_sum, uint32_t ntiles, uint32_t* scratch,
                                                     uint32_t nblocks) {
    __shared__ uint32_t h[ORDER_BUCKETS];
    __shared__ uint32_t w[4];
    for (uint32_t b = threadIdx.x; b < ORDER_BUCKETS; b += 256u) h[b] = 0u;
    __syncthreads();
    const uint32_t cut = scratch[OS_CUT];
    uint32_t c = 0;
    for (uint32_t k = 0; k < 4u; k++) {
        const uint32_t t = blockIdx.x * ORDER_BLOCK + k * 256u + threadIdx.x;
        if (t < ntiles) {
            const uint32_t cls = order_bucket(tile_sum[t]);
            if (cls < cut) {
                c++;
                atomicAdd(&h[cls], 1u);
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63u) == 0u) w[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) scratch[OS_BLK + blockIdx.x] = w[0] + w[1] + w[2] + w[3];
    for (uint32_t b = threadIdx.x; b < ORDER_BUCKETS; b += 256u) scratch[os_cls(nblocks, blockIdx.x, b)] = h[b];
}
// one workgroup: exclusive prefix sums of the blocks' head counts, in place (nblocks <= 2^15)
__global__ __launch_bounds__(1024) void k_order_blockscan(uint32_t* scratch, uint32_t nblocks) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (nblocks + 1023u) / 1024u, b0 = threadIdx.x * per;
    uint32_t s = 0;
    for (uint32_t k = 0; k < per && b0 + k < nblocks; k++) s += scratch[OS_BLK + b0 + k];
    part[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t o = 1; o < 1024u; o <<= 1) {
        const uint32_t add = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
        __syncthreads();
        part[threadIdx.x] += add;
        __syncthreads();
    }
    uint32_t run = threadIdx.x ? part[threadIdx.x - 1u] : 0u;
    for (uint32_t k = 0; k < per && b0 + k < nblocks; k++) {
        const uint32_t c = scratch[OS_BLK + b0 + k];
        scratch[OS_BLK + b0 + k] = run;
        run += c;
    }
    // the head classes: a class's tiles go to its first position onwards, block by block
    const uint32_t cls = threadIdx.x;
    if (cls < scratch[OS_CUT]) {
        uint32_t pos = scratch[OS_CBASE + cls];
        for (uint32_t b = 0; b < nblocks; b++) {
            const uint32_t i = os_cls(nblocks, b, cls), n = scratch[i];
            scratch[i] = pos;
            pos += n;
        }
    }
}
// head tiles to [0, nhead) by class (most expensive first; within a class block by block), the others to
// [nhead, ntiles) in tile order
__global__ __launch_bounds__(256) void k_order_scatter(const uint32_t* __restrict__ tile_sum, uint32_t ntiles,
                                                       const uint32_t* scratch, uint32_t* __restrict__ order, uint32_t nblocks) {
    __shared__ uint32_t w[4];
    __shared__ uint32_t next[ORDER_BUCKETS];
    for (uint32_t b = threadIdx.x; b < ORDER_BUCKETS; b += 256u) next[b] = scratch[os_cls(nblocks, blockIdx.x, b)];
    __syncthreads();
    const uint32_t nhead = scratch[OS_NHEAD], cut = scratch[OS_CUT];
    uint32_t before = scratch[OS_BLK + blockIdx.x];  // head tiles before this block's current group of 256
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    for (uint32_t k = 0; k < 4u; k++) {
        const uint32_t t = blockIdx.x * ORDER_BLOCK + k * 256u + threadIdx.x;
        const uint32_t cls = t < ntiles ? order_bucket(tile_sum[t]) : ORDER_BUCKETS;
        const bool h = cls < cut;
        const unsigned long long m = __ballot(h);
        if (lane == 0u) w[wv] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t r = before + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        for (uint32_t q = 0; q < wv; q++) r += w[q];
        if (h) order[atomicAdd(&next[cls], 1u)] = t;
        else if (t < ntiles) order[nhead + (t - r)] = t;
        before += w[0] + w[1] + w[2] + w[3];
        __syncthreads();
    }
}
// scratch: hrt_order_scratch_words(ntiles) words, the histogram zero on the first call
hipError_t hrt_launch_order(uint32_t* pixel_cost, uint32_t ntiles, uint32_t* tile_sum, uint32_t* order, uint32_t* scratch,
                            hipStream_t stream) {
    if (ntiles == 0) return hipSuccess;
    const uint32_t nblocks = (ntiles + ORDER_BLOCK - 1u) / ORDER_BLOCK;
    if (nblocks > 32768u) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_order_hist, dim3((ntiles + 3u) / 4u), dim3(256), 0, stream, pixel_cost, ntiles, tile_sum, scratch);
    hipLaunchKernelGGL(k_order_cut, dim3(1), dim3(64), 0, stream, scratch, ntiles);
    hipLaunchKernelGGL(k_order_count, dim3(nblocks), dim3(256), 0, stream, tile_sum, ntiles, scratch, nblocks);
    hipLaunchKernelGGL(k_order_blockscan, dim3(1), dim3(1024), 0, stream, scratch, nblocks);
    hipLaunchKernelGGL(k_order_scatter, dim3(nblocks), dim3(256), 0, stream, tile_sum, ntiles, scratch, order, nblocks);
    return hipGetLastError();
}
uint32_t hrt_order_scratch_words(uint32_t ntiles) {
    const uint32_t nblocks = (ntiles + ORDER_BLOCK - 1u) / ORDER_BLOCK;
    return OS_BLK + nblocks + nblocks * ORDER_BUCKETS;
}

// Exactness check of the range-restricted sqrt / division sequences (rt_device.hpp) against the IEEE
// operations (correctly rounded in this build): n random cases per test, counted mismatches in out[0..2]:
// [0] normalize_rng vs normalize on vectors of rng floats (the hemisphere sample) and normalize_exact vs
// normalize on signed vectors (magnitudes 2^-48 .. 2^48), [1] div_rn_mid vs `/` on
// log-uniform operands in [2^-60, 2^60] (random signs, and x = 0) and rcp_rn_mid vs 1 / l over every significand
// (n >= 2^23; case i's operand is fixed by i), [2] sqrt_rn_mid vs sqrtf on [2^-100, 2^100].
__global__ __launch_bounds__(256) void k_check_exact_math(unsigned long long n, uint32_t seed,
                                                          unsigned long long* out) {
    unsigned long long bad[3] = {0, 0, 0};
    const unsigned long long stride = (unsigned long long)gridDim.x * 256u;
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256u + threadIdx.x; i < n; i += stride) {
        uint32_t s = (uint32_t)i * 2654435761u ^ seed ^ (uint32_t)(i >> 32) * 40503u;
        const f3 v = mk(rng_float(s), rng_float(s), rng_float(s));
        const f3 a = normalize(v), b = normalize_rng(v);
        if (__float_as_uint(a.x) != __float_as_uint(b.x) || __float_as_uint(a.y) != __float_as_uint(b.y) ||
            __float_as_uint(a.z) != __float_as_uint(b.z))
            bad[0]++;
        // normalize_exact on signed vectors with component magnitudes 2^-48 .. 2^48 (some outside its fast range)
        {
            uint32_t t = pcg_next(s ^ 0x9E3779B9u);
            float w[3];
            for (int k = 0; k < 3; k++) {
                t = pcg_next(t);
                const uint32_t e = 127u - 48u + (t % 97u);
                w[k] = __uint_as_float((e << 23) | (pcg_next(t) & 0x7FFFFFu) | (t & 0x80000000u));
            }
            const f3 g = mk(w[0], w[1], w[2]);
            const f3 ga = normalize(g), gb = normalize_exact(g);
            if (__float_as_uint(ga.x) != __float_as_uint(gb.x) || __float_as_uint(ga.y) != __float_as_uint(gb.y) ||
                __float_as_uint(ga.z) != __float_as_uint(gb.z))
                bad[0]++;
        }
        // log-uniform magnitudes: exponent in [-60, 60), random mantissa and sign
        s = pcg_next(s);
        const uint32_t ex = 67u + (s % 120u), ey = 67u + ((s >> 8) % 120u);
        const uint32_t mx = pcg_next(s), my = pcg_next(mx);
        float x = __uint_as_float((ex << 23) | (mx & 0x7FFFFFu) | (mx & 0x80000000u));
        const float l = __uint_as_float((ey << 23) | (my & 0x7FFFFFu) | (my & 0x80000000u));
        if ((mx & 0xFFu) == 0u) x = 0.0f;
        if (__float_as_uint(x / l) != __float_as_uint(div_rn_mid(x, rcp_rn_setup(l)))) bad[1]++;
        // rcp_rn_mid vs 1 / l by enumeration: case i takes significand i mod 2^23 under sign / exponent pair
        // (i >> 23) mod 242 — both signs of every binade 2^-60 .. 2^60 (biased exponents 67 .. 187) — so n = 242 x 2^23
        // runs every significand of the range the kernels use it on (no scaling assumption left)
        {
            const uint32_t se = (uint32_t)((i >> 23) % 242u);
            const uint32_t e = 67u + (se >> 1);
            const float r = __uint_as_float(((se & 1u) << 31) | (e << 23) | ((uint32_t)i & 0x7FFFFFu));
            if (__float_as_uint(1.0f / r) != __float_as_uint(rcp_rn_mid(r))) bad[1]++;
        }
        const uint32_t es = 27u + (my % 200u);
        const float q = __uint_as_float((es << 23) | (pcg_next(my) & 0x7FFFFFu));
        if (__float_as_uint(__builtin_sqrtf(q)) != __float_as_uint(sqrt_rn_mid(q))) bad[2]++;
    }
#pragma unroll
    for (int c = 0; c < 3; c++) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) bad[c] += __shfl_xor(bad[c], off);
        if ((threadIdx.x & 63u) == 0 && bad[c]) atomicAdd(out + c, bad[c]);
    }
}

hipError_t hrt_check_exact_math(unsigned long long n, uint32_t seed, unsigned long long* out_dev, hipStream_t st) {
    hipLaunchKernelGGL(k_check_exact_math, dim3(4096), dim3(256), 0, st, n, seed, out_dev);
    return hipGetLastError();
}

// Demangled-symbol form of the kernel a draw ran ("k_trace_split<true>"): rt_stats.kernel, and the key
// bench.py matches against rocprofv3 summaries.
// Per host thread (renderers driven from several threads each see their own launch); renderer.cpp copies it
// into the renderer's stats right after its launches and clears it before them.
static thread_local char g_kernel_name[64] = "";
const char* hrt_last_kernel() { return g_kernel_name; }
void hrt_reset_last_kernel() { g_kernel_name[0] = '\0'; }
static const char* kname_bbbb(const char* base, int a, int b, int c, int d) {  // <bool, bool, bool, bool>
    snprintf(g_kernel_name, sizeof g_kernel_name, "%s<%s, %s, %s, %s>", base, a ? "true" : "false", b ? "true" : "false",
             c ? "true" : "false", d ? "true" : "false");
    return g_kernel_name;
}
static const char* kname_iiib(const char* base, int a, int b, int c, int d) {  // <int, int, int, bool>
    snprintf(g_kernel_name, sizeof g_kernel_name, "%s<%d, %d, %d, %s>", base, a, b, c, d ? "true" : "false");
    return g_kernel_name;
}
static const char* kname(const char* base, int a, int b = -1, int c = -1) {
    if (b < 0) snprintf(g_kernel_name, sizeof g_kernel_name, "%s<%s>", base, a ? "true" : "false");
    else if (c < 0) snprintf(g_kernel_name, sizeof g_kernel_name, "%s<%d, %d>", base, a, b);
    else snprintf(g_kernel_name, sizeof g_kernel_name, "%s<%d, %d, %s>", base, a, b, c ? "true" : "false");
    return g_kernel_name;
}

template <typename K>
static hipError_t launch_persistent(K kernel, const KParams& P, hipStream_t stream, const char* /*name*/,
                                    uint32_t wgt = 256) {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
    }
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, (int)wgt, 0);
    if (e != hipSuccess) return e;
    const unsigned long long wpb = wgt / 64u;
    const unsigned long long want = (P.njobs + wpb - 1ull) / wpb;  // no more waves than jobs
    const unsigned long long cap = (unsigned long long)std::max(1, per_cu) * (unsigned long long)cus;
    const dim3 grid((unsigned)std::min(want, std::min(cap, (unsigned long long)P.steal_cap / wpb)));
    KParams Q = P;
    Q.nwaves = (uint32_t)(grid.x * wpb);  // work stealing: one slot per wave (renderer.cpp zeroes steal_cap of them)
    hipLaunchKernelGGL(kernel, grid, dim3((unsigned)wgt), 0, stream, Q);
    return hipGetLastError();
}

// k_trace_split_tris<MODE, SCAN, HL, STEAL> by P.tri_small (the heap-top configuration) / P.steal
template <int MODE, int SCAN, int HL>
static hipError_t launch_split_tris_hl(const KParams& P, hipStream_t stream) {
    const char* base = "k_trace_split_tris";
    return P.steal ? launch_persistent(k_trace_split_tris<MODE, SCAN, HL, true>, P, stream, kname_iiib(base, MODE, SCAN, HL, 1), heap_wg(HL))
                   : launch_persistent(k_trace_split_tris<MODE, SCAN, HL, false>, P, stream, kname_iiib(base, MODE, SCAN, HL, 0), heap_wg(HL));
}
template <int MODE, int SCAN>
static hipError_t launch_split_tris(const KParams& P, hipStream_t stream) {
    if constexpr (SCAN == SCAN_DEFER) {  // (its deferred-scan lists assume 256-lane workgroups)
        if (P.tri_small > 1u) return hipErrorInvalidValue;
        return P.tri_small ? launch_split_tris_hl<MODE, SCAN, 1>(P, stream) : launch_split_tris_hl<MODE, SCAN, 0>(P, stream);
    } else {
        if (P.tri_small != 0u && P.tri_small != 3u) return hipErrorInvalidValue;
        return P.tri_small ? launch_split_tris_hl<MODE, SCAN, 3>(P, stream) : launch_split_tris_hl<MODE, SCAN, 0>(P, stream);
    }
}

// Sample queue, part 1: trace every sample of the chunk into P.samples.
// variant: SCAN_SIMPLE, SCAN_DEFER or SCAN_BVH (resolved by the host); P.tri_bvh picks the triangle walk.
// The reference heap walk (triangle / mixed programs) and the sphere program's culling BVH always run in the
// suspendable-walk kernels (renderer.cpp sets suspend_below >= 1 for them; 1 = a wave never leaves a walk early);
// k_trace is instantiated only for what has no split kernel: the sphere program's linear scans and the opt-in SAH
// triangle walk (tri_bvh = 1).
template <int MODE, bool TSAH>
static hipError_t launch_trace_mode(int variant, const KParams& P, hipStream_t stream) {
    if constexpr (MODE != MODE_SPHERE && !TSAH) {
        if (P.suspend_below == 0u) return hipErrorInvalidValue;
        // The mixed program with the culling BVH runs its sphere walk to completion in the begin phase
        // (stack in the triangle-batch LDS) and suspends only the heap walk: C5 at 256 spp 6.25 -> 6.55
        // Grays/s. (Splitting both walks measured 5.93; an earlier heap-only form with the stack in
        // the LDS block region, 6.05.)
        if constexpr (MODE == MODE_TRIS) {
            return launch_split_tris<MODE, SCAN_SIMPLE>(P, stream);
        } else {
            if (variant == SCAN_SIMPLE) return launch_split_tris<MODE, SCAN_SIMPLE>(P, stream);
            if (variant == SCAN_DEFER) return launch_split_tris<MODE, SCAN_DEFER>(P, stream);
            return launch_split_tris<MODE, SCAN_BVH>(P, stream);
        }
    } else if constexpr (MODE == MODE_TRIS) {
        return launch_persistent(k_trace<MODE, SCAN_SIMPLE, TSAH>, P, stream, kname("k_trace", MODE, SCAN_SIMPLE, (int)TSAH));
    } else {
        if (variant == SCAN_SIMPLE) return launch_persistent(k_trace<MODE, SCAN_SIMPLE, TSAH>, P, stream, kname("k_trace", MODE, SCAN_SIMPLE, (int)TSAH));
        if (variant == SCAN_DEFER) return launch_persistent(k_trace<MODE, SCAN_DEFER, TSAH>, P, stream, kname("k_trace", MODE, SCAN_DEFER, (int)TSAH));
        if constexpr (MODE == MODE_SPHERE) {
            return hipErrorInvalidValue;  // the culling BVH runs in k_trace_split
        } else {
            return launch_persistent(k_trace<MODE, SCAN_BVH, TSAH>, P, stream, kname("k_trace", MODE, SCAN_BVH, (int)TSAH));
        }
    }
}

// k_trace_split<LNODES, STEAL, COUNT, PACKET> by P.bvh_lnodes / P.steal / P.packet (PACKET only with LNODES)
template <bool COUNT>
static hipError_t launch_trace_split(const KParams& P, hipStream_t stream) {
    const char* base = "k_trace_split";
    if (P.bvh_lnodes && P.packet) {
        return P.steal ? launch_persistent(k_trace_split<true, true, COUNT, true>, P, stream, kname_bbbb(base, 1, 1, COUNT, 1))
                       : launch_persistent(k_trace_split<true, false, COUNT, true>, P, stream, kname_bbbb(base, 1, 0, COUNT, 1));
    }
    if (P.steal)
        return P.bvh_lnodes ? launch_persistent(k_trace_split<true, true, COUNT, false>, P, stream, kname_bbbb(base, 1, 1, COUNT, 0))
                            : launch_persistent(k_trace_split<false, true, COUNT, false>, P, stream, kname_bbbb(base, 0, 1, COUNT, 0));
    return P.bvh_lnodes ? launch_persistent(k_trace_split<true, false, COUNT, false>, P, stream, kname_bbbb(base, 1, 0, COUNT, 0))
                        : launch_persistent(k_trace_split<false, false, COUNT, false>, P, stream, kname_bbbb(base, 0, 0, COUNT, 0));
}

hipError_t hrt_launch_trace(int mode, int variant, const KParams& P, hipStream_t stream) {
    if (P.njobs == 0) return hipSuccess;
    // parts of jobs (tail_from) are decoded by the suspendable-walk kernels with the sample buffer and no stealing only
    // (job_acquire<TAIL>): k_trace_split and k_trace_split_tris (not the opt-in SAH walk's k_trace)
    const bool split_kernel = mode == MODE_SPHERE ? (variant == SCAN_BVH && P.suspend_below > 0u) : !P.tri_bvh;
    if (P.tail_from != 0xFFFFFFFFu && !(split_kernel && !P.steal && !P.ring_mode)) return hipErrorInvalidValue;
    switch (mode) {
    case MODE_SPHERE:
        if (variant == SCAN_BVH && P.suspend_below > 0u)
        {
            return P.count_tests ? launch_trace_split<true>(P, stream) : launch_trace_split<false>(P, stream);
        }
        return launch_trace_mode<MODE_SPHERE, false>(variant, P, stream);
    case MODE_TRIS:
        return P.tri_bvh ? launch_trace_mode<MODE_TRIS, true>(variant, P, stream)
                         : launch_trace_mode<MODE_TRIS, false>(variant, P, stream);
    default:
        return P.tri_bvh ? launch_trace_mode<MODE_MIXED, true>(variant, P, stream)
                         : launch_trace_mode<MODE_MIXED, false>(variant, P, stream);
    }
}

// Host-side launcher of the tiles schedule (called from renderer.cpp; no HIP types in the C-ABI).
// variant: SCAN_SIMPLE, SCAN_DEFER or SCAN_BVH (resolved by the host).
template <int MODE, bool TSAH>
static void launch_render_mode(int variant, const KParams& P, dim3 grid, dim3 block, hipStream_t stream) {
    (void)kname("k_render", MODE, MODE == MODE_TRIS ? SCAN_SIMPLE : variant, (int)TSAH);
    if constexpr (MODE == MODE_TRIS) {
        hipLaunchKernelGGL((k_render<MODE, SCAN_SIMPLE, TSAH>), grid, block, 0, stream, P);
    } else {
        if (variant == SCAN_SIMPLE) hipLaunchKernelGGL((k_render<MODE, SCAN_SIMPLE, TSAH>), grid, block, 0, stream, P);
        else if (variant == SCAN_DEFER) hipLaunchKernelGGL((k_render<MODE, SCAN_DEFER, TSAH>), grid, block, 0, stream, P);
        else hipLaunchKernelGGL((k_render<MODE, SCAN_BVH, TSAH>), grid, block, 0, stream, P);
    }
}

hipError_t hrt_launch_render(int mode, int variant, const KParams& P, hipStream_t stream) {
    dim3 block(256);
    dim3 grid((P.W + 15u) / 16u, (P.nrows + 15u) / 16u);
    if (grid.x == 0 || grid.y == 0) return hipSuccess;
    switch (mode) {
    case MODE_SPHERE: launch_render_mode<MODE_SPHERE, false>(variant, P, grid, block, stream); break;
    case MODE_TRIS:
        if (P.tri_bvh) launch_render_mode<MODE_TRIS, true>(variant, P, grid, block, stream);
        else launch_render_mode<MODE_TRIS, false>(variant, P, grid, block, stream);
        break;
    default:
        if (P.tri_bvh) launch_render_mode<MODE_MIXED, true>(variant, P, grid, block, stream);
        else launch_render_mode<MODE_MIXED, false>(variant, P, grid, block, stream);
        break;
    }
    return hipGetLastError();
}
