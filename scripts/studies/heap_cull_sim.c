/* heap_cull_sim.c — STUDY (round 5), not product code: the oracle (oracle/rt_oracle.c) with its heap walk run twice per
 * query — the reference's intersect_all_node, and a walk that skips hit subtrees whose entry t exceeds the current best
 * (the sphere winner, then the triangle winner at each flush of a deferred list) with the reference's 600-step cap tracked
 * through an upper bound of the reference's step count (a test at a possibly capped position counts as a fallback to
 * the full walk). It measures how much of the reference walk culling could save before any kernel is written.
 * Build: gcc -O2 -fopenmp -fPIC -shared -ffp-contract=off -o /tmp/liboracle_cull.so heap_cull_sim.c -lm
 * Run:   python scripts/studies/heap_cull_run.py c4 8 0.0009765625 1e-3 600   (DESIGN.md §4 Round 5 has the results)
 */
/*
 * rt_oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference's per-pixel ray loop.
 *
 * This file is the parity oracle (and the timed "port" CPU baseline) for the MI355X path tracer in
 * hello-raytracing_amd/. It restates, statement by statement, the two WGSL fragment shaders of
 * hucancode/hello-raytracing:
 *     src/shaders/shader_sphere.wgsl   (sphere list, BOUNCE_MAX = 10, EPSILON = 1e-6)
 *     src/shaders/shader_tris.wgsl     (implicit-heap BVH + triangles, BOUNCE_MAX = 5, EPSILON = 1e-4)
 * plus the frame protocol of src/renderer.rs (frame_count / time uniforms, :315-323, :355-410).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code, and only as
 * the checker. The product (hello-raytracing_amd/) never includes, links or calls it.
 *
 * Pinning: the reference is Rust + WGSL run through wgpu; there is no Rust toolchain, no wgpu and no
 * GPU here, so it cannot be built. This restatement is pinned by the reference's
 * own golden images (tests/rendering_tests.rs:134-509, tests/golden/NAME.ppm): >= 99.9 % of u8 channels
 * bit-exact on the five non-glass scenes, harness metric (mean |du8| <= 2 % of 255) on all seven.
 * The triangle/BVH path has no image golden in the reference: it is pinned structurally only
 * (bvh/tree.rs:93-126) — "parity unpinned" at image level for tris mode.
 *
 * Float semantics (build-defined, documented in DESIGN.md §Numerics; the HIP kernels follow the same
 * rules, written independently):
 *   - IEEE f32, round-to-nearest, no contraction (compile with -ffp-contract=off), denormals kept;
 *   - fused multiply-add in exactly three places: dot products (x*x' then fma(y), fma(z)[, fma(w)]),
 *     the sphere discriminant fma(b, b, -(4a*c)), and point_on_ray fma(t, d, o);
 *   - normalize(v) = v / sqrt(dot(v, v)) component-wise; division and sqrt correctly rounded;
 *   - pow(x, 5.0) = ((x*x)*(x*x))*x;  min/max = fminf/fmaxf (IEEE minNum/maxNum);
 *   - tan(fov/2) by libm tanf (the device path receives the same host-computed value).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define FLT_MAX_REF 3.40282e+38f /* shader_*.wgsl:4 */

/*
 * Float-contract study (tests/golden/contract_study.py): the reference GPU's compiler may fuse
 * or reassociate differently. ORACLE_CONTRACT selects a variant at build time; 0 (the default, and the only
 * one the kernels implement) is the contract above.
 *   1: no fused multiply-add anywhere (dot products, discriminant, point_on_ray unfused);
 *   2: contract 0 plus every a*b+c of the shaders fused (make_ray, mix, reflect, refract, reflectance, sky, c);
 *   3: contract 0 with normalize(v) = v * (1 / sqrt(dot(v, v)));
 *   4: contracts 2 and 3 together;
 *   5: every division by a computed value as a * (1 / b) (the reciprocal-based division GPU compilers emit
 *      for WGSL's 2.5-ulp `/`), normalize included.
 * Hardware-approximate forms a WGSL compiler may emit, alone (6-8) and together (9):
 *   6: pow(x, 5) of reflectance (shader_sphere.wgsl:166-171) as exp2(5 * log2(x)) (libm exp2f / log2f);
 *   7: normalize(v) (every site: make_ray's 4-D normalise, the AA and disk vectors, hemisphere, scatter) as
 *      v * rsq(dot(v, v)) with a 1-ulp rsq: the correctly rounded 1/sqrt moved by -1, 0 or +1 ulp, chosen by a
 *      hash of the operand's bits (a deterministic stand-in for an unknown hardware rsq);
 *   8: tan(fov / 2) of make_ray (:124) as sin * (1 / cos) in f32 (not correctly rounded);
 *   9: 6 + 7 + 8.
 */
#ifndef ORACLE_CONTRACT
#define ORACLE_CONTRACT 0
#endif
#define OC_NOFMA (ORACLE_CONTRACT == 1)
#define OC_FUSE (ORACLE_CONTRACT == 2 || ORACLE_CONTRACT == 4)
#define OC_RCPNORM (ORACLE_CONTRACT == 3 || ORACLE_CONTRACT == 4 || ORACLE_CONTRACT == 5)
#define OC_RCPDIV (ORACLE_CONTRACT == 5)
#define OC_POWEXP (ORACLE_CONTRACT == 6 || ORACLE_CONTRACT == 9)
#define OC_RSQNORM (ORACLE_CONTRACT == 7 || ORACLE_CONTRACT == 9)
#define OC_TANSC (ORACLE_CONTRACT == 8 || ORACLE_CONTRACT == 9)
static inline float fmaf_c(float a, float b, float c) { return OC_NOFMA ? a * b + c : fmaf(a, b, c); }
/* a*b + c at the sites a compiler may fuse */
static inline float madd(float a, float b, float c) { return OC_FUSE ? fmaf(a, b, c) : a * b + c; }
/* a / b at the sites whose divisor is computed */
static inline float divf(float a, float b) { return OC_RCPDIV ? a * (1.0f / b) : a / b; }
/* contract 7: a 1-ulp reciprocal square root (correctly rounded 1/sqrt(a), moved by -1 / 0 / +1 ulp by a hash of
 * a's bits), the scale normalize multiplies by */
static inline float rsq_1ulp(float a) {
    float r = (float)(1.0 / sqrt((double)a));
    uint32_t u;
    memcpy(&u, &a, 4);
    u = (u ^ (u >> 16)) * 0x45d9f3bu;
    u ^= u >> 16;
    const int k = (int)(u % 3u) - 1;
    if (k > 0) r = nextafterf(r, INFINITY);
    if (k < 0) r = nextafterf(r, 0.0f);
    return r;
}
/* v_i / |v| at a normalize site, |v|^2 = ss (contract 7: v_i * rsq(ss)) */
static inline float nrm_div(float vi, float ss, float len) { return OC_RSQNORM ? vi * rsq_1ulp(ss) : vi / len; }

enum { MODE_SPHERE = 0, MODE_TRIS = 1, MODE_MIXED = 2 };

/* ---- reference POD layouts (bytemuck #[repr(C)]), src/scene/{camera,material,sphere}.rs, bvh/ ---- */
typedef struct { float eye[4], dir[4], up[4], right[4], params[4]; } o_camera;          /* 80 B */
typedef struct { float albedo[4]; float params[3]; uint32_t id; } o_material;              /* 32 B */
typedef struct { float center[3]; float radius; o_material mat; } o_sphere;                /* 48 B */
typedef struct { float bmin[4]; float bmax[4]; } o_node;                                   /* 32 B */
typedef struct { float a[4], b[4], c[4]; float normal[3]; uint32_t material; } o_triangle; /* 64 B */

typedef struct {
    uint32_t width, height;   /* resolution uniform (renderer.rs:242-247)                       */
    uint32_t mode;            /* MODE_*                                                          */
    uint32_t bounces;         /* BOUNCE_MAX (10 sphere / 5 tris in the reference)                */
    uint32_t ema_cap;         /* SAMPLE_FRAME (1000)                                             */
    uint32_t frame0;          /* frame_count of the first frame drawn                            */
    uint32_t time0, dtime;    /* time of frame f = time0 + f*dtime (tests: 1000 + 10 i)          */
    uint32_t frames;          /* frames drawn by this call                                       */
    uint32_t x0, nx;          /* column window                                                   */
    uint32_t row0, row_step, nrows; /* rows row0 + k*row_step, k < nrows                         */
    uint32_t row_block;       /* 0/1: rows as above; b > 1: local row k is row0 + (k/b)*row_step*b + k%b
                                 (the renderer's blocked row partition, rt_params.row_block)          */
    uint32_t step_cap;        /* intersect_all_node step cap: 600 in the reference (shader_tris.wgsl:274);
                                 0 = uncapped, only to check the opt-in SAH walk (non-parity mode)   */
} o_params;

typedef struct { float x, y, z; } v3;
static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 smul(float s, v3 a) { return V(s * a.x, s * a.y, s * a.z); }
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
static inline float dot3(v3 a, v3 b) { return fmaf_c(a.z, b.z, fmaf_c(a.y, b.y, a.x * b.x)); }
static inline float len3(v3 a) { return sqrtf(dot3(a, a)); }
static inline v3 norm3(v3 a) {
    if (OC_RSQNORM) { float q = rsq_1ulp(dot3(a, a)); return V(a.x * q, a.y * q, a.z * q); }
    float l = len3(a);
    if (OC_RCPNORM) { float r = 1.0f / l; return V(a.x * r, a.y * r, a.z * r); }
    return V(a.x / l, a.y / l, a.z / l);
}
static inline v3 cross3(v3 a, v3 b) {
    return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline v3 ld3(const float *p) { return V(p[0], p[1], p[2]); }

/* rng_int / rng_float / rng_vec2 / rng_vec3: shader_sphere.wgsl:87-103 (= shader_tris.wgsl:99-115) */
static inline void rng_int(uint32_t *s) {
    uint32_t old = *s + 747796405u + 2891336453u;
    uint32_t word = ((old >> ((old >> 28u) + 4u)) ^ old) * 277803737u;
    *s = (word >> 22u) ^ word;
}
static inline float rng_float(uint32_t *s) { rng_int(s); return (float)(*s) / 4294967296.0f; }
static inline v3 rng_vec3(uint32_t *s) {
    float x = rng_float(s); float y = rng_float(s); float z = rng_float(s);
    return V(x, y, z);
}

typedef struct { v3 o, d; } ray_t;
typedef struct { v3 p, n; float t; const o_material *mat; int front; } hit_t;

typedef struct {
    const o_camera *cam; float k;            /* k = tan(fov*0.5) */
    const o_sphere *spheres; uint32_t nslots;
    const o_node *nodes; const o_triangle *tris; const o_material *mats; uint32_t n, m;
    uint32_t mode, bounces; float eps;
    uint32_t step_cap;
} o_scene;

/* random_on_hemisphere: shader_sphere.wgsl:107-117 / shader_tris.wgsl:119-128 */
static inline v3 random_on_hemisphere(uint32_t *s, v3 n, float eps) {
    v3 v = norm3(rng_vec3(s));
    if (len3(v) < eps) return n;
    if (dot3(v, n) > 0.0f) return v;
    return vneg(v);
}

/* make_ray: shader_sphere.wgsl:123-135 (direction not normalised) / shader_tris.wgsl:136-148 */
static ray_t make_ray(const o_scene *sc, float ux, float uy, uint32_t *s) {
    const o_camera *c = sc->cam;
    float v[4], d4[4], f4[4], o4[4];
    for (int i = 0; i < 4; i++) {
        float xx = (c->right[i] * ux) * sc->k;
        v[i] = madd(c->up[i] * uy, sc->k, xx) + c->dir[i];
    }
    float ss = fmaf_c(v[3], v[3], fmaf_c(v[2], v[2], fmaf_c(v[1], v[1], v[0] * v[0])));
    float l = sqrtf(ss);
    for (int i = 0; i < 4; i++) d4[i] = OC_RCPNORM ? v[i] * (1.0f / l) : nrm_div(v[i], ss, l);
    for (int i = 0; i < 4; i++) f4[i] = madd(d4[i], c->params[0], c->eye[i]);
    /* random_on_disk: shader_sphere.wgsl:118-122 */
    float r1 = rng_float(s), r2 = rng_float(s);
    float ss2 = fmaf_c(r2, r2, r1 * r1);
    float l2 = sqrtf(ss2);
    float vx = OC_RCPNORM ? r1 * (1.0f / l2) : nrm_div(r1, ss2, l2);
    float vy = OC_RCPNORM ? r2 * (1.0f / l2) : nrm_div(r2, ss2, l2);
    float rr = rng_float(s) * c->params[1];
    o4[0] = madd(vx, rr, c->eye[0]);
    o4[1] = madd(vy, rr, c->eye[1]);
    o4[2] = c->eye[2] + 0.0f * rr;
    o4[3] = c->eye[3] + 1.0f;
    ray_t r;
    r.o = V(o4[0], o4[1], o4[2]);
    if (sc->mode == MODE_SPHERE) {
        r.d = V(f4[0] - o4[0], f4[1] - o4[1], f4[2] - o4[2]);
    } else {
        float g[4];
        for (int i = 0; i < 4; i++) g[i] = f4[i] - o4[i];
        float sg = fmaf_c(g[3], g[3], fmaf_c(g[2], g[2], fmaf_c(g[1], g[1], g[0] * g[0])));
        float lg = sqrtf(sg);
        r.d = OC_RCPNORM ? V(g[0] * (1.0f / lg), g[1] * (1.0f / lg), g[2] * (1.0f / lg))
                         : V(nrm_div(g[0], sg, lg), nrm_div(g[1], sg, lg), nrm_div(g[2], sg, lg));
    }
    return r;
}

/* intersect_all_sphere + intersect_sphere: shader_sphere.wgsl:218-229, :136-155.
 * Closest accepted root over ALL slots (arrayLength = buffer capacity, zero-filled past N). */
static void closest_sphere(const o_scene *sc, ray_t r, hit_t *h) {
    float a = dot3(r.d, r.d);
    float best = h->t;
    int idx = -1;
    for (uint32_t i = 0; i < sc->nslots; i++) {
        const o_sphere *sp = &sc->spheres[i];
        v3 oc = vsub(r.o, ld3(sp->center));
        float b = 2.0f * dot3(oc, r.d);
        float c = OC_FUSE ? fmaf(-sp->radius, sp->radius, dot3(oc, oc)) : dot3(oc, oc) - sp->radius * sp->radius;
        float disc = fmaf_c(b, b, -((4.0f * a) * c));
        if (disc < 0.0f) continue; /* t = -1 */
        float t = divf(-b - sqrtf(disc), 2.0f * a);
        if (t > 0.0f && t < best) { best = t; idx = (int)i; }
    }
    if (idx < 0) return;
    const o_sphere *sp = &sc->spheres[idx];
    v3 p = V(fmaf_c(best, r.d.x, r.o.x), fmaf_c(best, r.d.y, r.o.y), fmaf_c(best, r.d.z, r.o.z));
    v3 n = vsub(p, ld3(sp->center));
    n = V(divf(n.x, sp->radius), divf(n.y, sp->radius), divf(n.z, sp->radius));
    int front = dot3(r.d, n) < 0.0f;
    if (!front) n = vneg(n);
    h->p = p; h->n = n; h->t = best; h->mat = &sp->mat; h->front = front;
}

/* intersect_node: shader_tris.wgsl:150-159 (inv_d hoisted: identical value for every node) */
static inline int node_hit(v3 o, v3 inv, const o_node *nd) {
    float t0x = (nd->bmin[0] - o.x) * inv.x, t0y = (nd->bmin[1] - o.y) * inv.y, t0z = (nd->bmin[2] - o.z) * inv.z;
    float t1x = (nd->bmax[0] - o.x) * inv.x, t1y = (nd->bmax[1] - o.y) * inv.y, t1z = (nd->bmax[2] - o.z) * inv.z;
    float tmin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    float tmax = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    return tmin <= tmax && tmax >= 0.0f;
}

/* intersect_triangle (Moller-Trumbore): shader_tris.wgsl:161-202 */
static inline void tri_test(const o_scene *sc, ray_t r, uint32_t j, hit_t *h) {
    const o_triangle *tr = &sc->tris[j];
    v3 a = ld3(tr->a), b = ld3(tr->b), c = ld3(tr->c);
    v3 e1 = vsub(b, a), e2 = vsub(c, a);
    v3 hh = cross3(r.d, e2);
    float det = dot3(e1, hh);
    if (fabsf(det) < 1e-4f) return;
    float inv_det = 1.0f / det;
    v3 s = vsub(r.o, a);
    float u = inv_det * dot3(s, hh);
    if (u < 0.0f || u > 1.0f) return;
    v3 q = cross3(s, e1);
    float v = inv_det * dot3(r.d, q);
    if (v < 0.0f || u + v > 1.0f) return;
    float t = inv_det * dot3(e2, q);
    if (t < 1e-4f || t >= h->t) return;
    h->p = V(fmaf_c(t, r.d.x, r.o.x), fmaf_c(t, r.d.y, r.o.y), fmaf_c(t, r.d.z, r.o.z));
    h->n = ld3(tr->normal);
    h->t = t;
    h->mat = &sc->mats[tr->material];
    h->front = dot3(h->n, r.d) > 0.0f;
}

/* ---- culling simulation (round 5 study): the reference walk vs a walk that skips hit subtrees whose entry t exceeds
   the current best (+ margin), with the 600-step cap tracked through an upper bound of the reference's step count ---- */
#include <stdatomic.h>
static _Atomic uint64_t g_stat[12];
uint64_t cull_stat(int i) { return g_stat[i]; }
static int g_batch = 8;      /* deferred leaf entries before a flush (best updated at flush) */
static float g_margin_rel = 1.0f / 1024.0f, g_margin_abs = 1e-3f;
static int g_cull_limit = 600;
void cull_config(int batch, float mrel, float mabs, int limit) { g_batch = batch; g_margin_rel = mrel; g_margin_abs = mabs; g_cull_limit = limit; }
static inline int node_hit_t(v3 o, v3 inv, const o_node *nd, float *tmin_out) {
    float t0x = (nd->bmin[0] - o.x) * inv.x, t0y = (nd->bmin[1] - o.y) * inv.y, t0z = (nd->bmin[2] - o.z) * inv.z;
    float t1x = (nd->bmax[0] - o.x) * inv.x, t1y = (nd->bmax[1] - o.y) * inv.y, t1z = (nd->bmax[2] - o.z) * inv.z;
    float tmin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    float tmax = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    *tmin_out = tmin;
    return tmin <= tmax && tmax >= 0.0f;
}
static void tri_test(const o_scene *sc, ray_t r, uint32_t j, hit_t *h);
/* returns steps taken; result in *hh; *fallback set when a test happened at a possibly capped reference position */
static uint32_t culled_walk(const o_scene *sc, ray_t r, hit_t *hh, int *fallback, uint32_t *tris_out) {
    v3 inv = V(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
    uint32_t i = 1, n = sc->n, m = sc->m, step = 0, slack = 0, tris = 0;
    int L = 0; while ((1u << L) < n) L++;
    uint32_t pend[64]; int np = 0;
    float cullb = hh->t;  /* best as known to the walk (updated at flushes) */
    *fallback = 0;
    while (step < 600) {
        step++;
        if (i < n) {
            float tmin;
            int hit = node_hit_t(r.o, inv, &sc->nodes[i], &tmin);
            if (hit) {
                int d = 31 - __builtin_clz(i);
                uint32_t maxsub = (2u << (L - d)) - 2u;
                if (tmin > cullb + cullb * g_margin_rel + g_margin_abs && step + slack + maxsub < (uint32_t)g_cull_limit) {
                    slack += maxsub;  /* skip: climb as after a miss */
                } else { i *= 2u; continue; }
            }
        }
        if (i >= n) {
            uint32_t j = i - n;
            if (j >= m) break;
            if (step + slack >= 600) { *fallback = 1; return step; }
            pend[np++] = j; tris++;
            if (np == g_batch) { for (int k = 0; k < np; k++) tri_test(sc, r, pend[k], hh); np = 0; cullb = hh->t; }
        }
        while ((i & 1u) == 1u) i /= 2u;
        if (i == 0u) break;
        i++;
    }
    for (int k = 0; k < np; k++) tri_test(sc, r, pend[k], hh);
    *tris_out = tris;
    return step;
}

/* intersect_all_node: shader_tris.wgsl:268-301 — stackless walk of the implicit heap, 600-step cap */
static void closest_bvh_ref(const o_scene *sc, ray_t r, hit_t *h, uint64_t *cnt);
static void closest_bvh(const o_scene *sc, ray_t r, hit_t *h, uint64_t *cnt) {
    hit_t h2 = *h;
    uint64_t c2[4] = {0, 0, 0, 0};
    closest_bvh_ref(sc, r, h, c2);
    cnt[1] += c2[1]; cnt[2] += c2[2]; cnt[3] += c2[3];
    int fb = 0; uint32_t tr = 0;
    uint32_t st = culled_walk(sc, r, &h2, &fb, &tr);
    g_stat[0] += c2[1] + c2[2];          /* reference steps */
    g_stat[1] += c2[1];                  /* reference node tests */
    g_stat[2] += c2[2];                  /* reference tri tests */
    g_stat[9] += 1;                      /* walks */
    if (fb) { g_stat[3] += 1; g_stat[4] += st + c2[1] + c2[2]; g_stat[5] += tr + c2[2]; }
    else {
        g_stat[4] += st; g_stat[5] += tr;
        if (h2.t != h->t || (h2.t < 3e38f && h2.mat != h->mat) || memcmp(&h2.n, &h->n, sizeof(v3)) != 0) g_stat[6] += 1;
    }
}
static void closest_bvh_ref(const o_scene *sc, ray_t r, hit_t *h, uint64_t *cnt) {
    v3 inv = V(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
    uint32_t i = 1, n = sc->n, m = sc->m;
    const uint32_t cap = sc->step_cap ? sc->step_cap : 0xFFFFFFFFu;
    uint32_t step = 0;
    while (step < cap) {
        step++;
        if (i < n) {
            cnt[1]++; /* node (slab) tests */
            if (node_hit(r.o, inv, &sc->nodes[i])) { i *= 2u; continue; }
        }
        if (i >= n) {
            uint32_t j = i - n;
            if (j >= m) break;
            cnt[2]++; /* triangle tests */
            tri_test(sc, r, j, h);
        }
        while ((i & 1u) == 1u) i /= 2u;
        if (i == 0u) break;
        i++;
    }
    if (step == cap && i != 0u) cnt[3]++; /* walks the step cap cut short (bookkeeping, not semantics) */
}

static inline v3 reflect3(v3 v, v3 n) {
    float k = 2.0f * dot3(v, n);
    if (OC_FUSE) return V(fmaf(-k, n.x, v.x), fmaf(-k, n.y, v.y), fmaf(-k, n.z, v.z));
    return vsub(v, smul(k, n));
}
static inline v3 refract3(v3 uv, v3 n, float e) { /* shader_sphere.wgsl:159-165 */
    float cos_t = fminf(dot3(vneg(uv), n), 1.0f);
    v3 perp = smul(e, V(madd(cos_t, n.x, uv.x), madd(cos_t, n.y, uv.y), madd(cos_t, n.z, uv.z)));
    float len = len3(perp);
    v3 par = smul(-sqrtf(fabsf(1.0f - len * len)), n);
    return vadd(perp, par);
}
static inline float reflectance(float cosine, float ref_idx) { /* :166-171, pow(x,5) = x^4*x */
    float r0 = divf(1.0f - ref_idx, 1.0f + ref_idx);
    r0 = r0 * r0;
    float x = 1.0f - cosine;
    float x2 = x * x;
    float p5 = OC_POWEXP ? exp2f(5.0f * log2f(x)) : (x2 * x2) * x; /* contract 6: pow as exp2(5 log2 x) */
    return madd(1.0f - r0, p5, r0);
}

/* scatter: shader_sphere.wgsl:172-217 / shader_tris.wgsl:222-267 (metal: tris reflects the raw d) */
static ray_t scatter(const o_scene *sc, uint32_t *s, ray_t r, const hit_t *h) {
    ray_t out; out.o = h->p;
    uint32_t id = h->mat->id;
    if (id == 1u) {
        out.d = random_on_hemisphere(s, h->n, sc->eps);
    } else if (id == 2u) {
        float fuzz = h->mat->params[0];
        v3 in = sc->mode == MODE_SPHERE ? norm3(r.d) : r.d;
        v3 refl = reflect3(in, h->n);
        v3 hemi = random_on_hemisphere(s, h->n, sc->eps);
        out.d = norm3(V(madd(fuzz, hemi.x, refl.x), madd(fuzz, hemi.y, refl.y), madd(fuzz, hemi.z, refl.z)));
    } else { /* MAT_DIELECTRIC and default */
        float ir = h->mat->params[0];
        if (h->front) ir = 1.0f / ir;
        float cos_t = fminf(dot3(vneg(r.d), h->n), 1.0f);
        float sin_t = sqrtf(1.0f - cos_t * cos_t);
        int cannot = ir * sin_t > 1.0f;
        int refl = cannot;
        if (!refl) { /* WGSL || short-circuits: no RNG draw when cannot_refract */
            float f = rng_float(s);
            refl = reflectance(cos_t, ir) > (f - floorf(f));
        }
        out.d = refl ? norm3(reflect3(r.d, h->n)) : norm3(refract3(r.d, h->n, ir));
    }
    return out;
}

/* trace: shader_sphere.wgsl:230-243 / shader_tris.wgsl:303-316 */
static v3 trace(const o_scene *sc, ray_t primary, uint32_t *s, uint64_t *cnt) {
    v3 att = V(1.0f, 1.0f, 1.0f);
    ray_t cur = primary;
    for (uint32_t b = 0; b < sc->bounces; b++) {
        hit_t h = {{0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}, FLT_MAX_REF, 0, 0};
        if (sc->mode != MODE_TRIS) closest_sphere(sc, cur, &h);
        if (sc->mode != MODE_SPHERE) closest_bvh(sc, cur, &h, cnt);
        cnt[0]++; /* closest-hit queries (rays) */
        if (fabsf(h.t - FLT_MAX_REF) < sc->eps) break;
        cur = scatter(sc, s, cur, &h);
        const float *al = h.mat->albedo;
        att = vmul(att, V(al[0] * 0.7f, al[1] * 0.7f, al[2] * 0.7f));
    }
    float tt = primary.d.y * 0.5f + 0.5f;
    v3 sky = V(madd(0.54f, tt, 0.54f * (1.0f - tt)), madd(0.7f, tt, 0.86f * (1.0f - tt)),
               madd(0.98f, tt, 0.92f * (1.0f - tt)));
    return vmul(att, sky);
}

/* fs_main: shader_sphere.wgsl:251-273 — one pixel, one frame */
static v3 sample_pixel(const o_scene *sc, uint32_t W, uint32_t H, uint32_t x, uint32_t y, uint32_t time,
                       uint64_t *cnt) {
    uint32_t s = (x * H + y) * time;
    float aspect = divf((float)W, (float)H);
    float r1 = rng_float(&s), r2 = rng_float(&s);
    float ssa = fmaf_c(r2, r2, r1 * r1);
    float l = sqrtf(ssa);
    float px = ((float)x + 0.5f) + (OC_RCPNORM ? r1 * (1.0f / l) : nrm_div(r1, ssa, l));
    float py = ((float)y + 0.5f) + (OC_RCPNORM ? r2 * (1.0f / l) : nrm_div(r2, ssa, l));
    float ux = divf(px, (float)W - 1.0f), uy = divf(py, (float)H - 1.0f);
    ux = madd(2.0f, ux, -1.0f) * aspect;
    uy = madd(2.0f, uy, -1.0f) * -1.0f;
    ray_t r = make_ray(sc, ux, uy, &s);
    v3 c = trace(sc, r, &s, cnt);
    return V(0.0f + c.x, 0.0f + c.y, 0.0f + c.z);
}

/*
 * oracle_render: draw p->frames frames into `image` (rows k < nrows, columns x0..x0+nx, RGB f32,
 * layout ((k*nx) + (x-x0))*3), continuing the accumulation already in `image` exactly as
 * repeated Renderer::draw() calls do (renderer.rs:355-410, accumulation at shader_sphere.wgsl:264-271).
 * Returns the number of closest-hit queries (rays) traced; if `counts` is given it receives
 * {rays, triangle-program node tests, triangle tests, walks cut short by the 600-step cap}.
 */
uint64_t oracle_render(const o_params *p, const void *camera80, const void *spheres48, uint32_t nslots,
                       const uint32_t *sizes, const void *nodes32, const void *tris64, const void *mats32,
                       float *image, int threads, uint64_t *counts) {
    o_scene sc;
    sc.cam = (const o_camera *)camera80;
    sc.k = OC_TANSC ? sinf(sc.cam->params[2] * 0.5f) * (1.0f / cosf(sc.cam->params[2] * 0.5f)) /* contract 8 */
                    : tanf(sc.cam->params[2] * 0.5f);
    sc.spheres = (const o_sphere *)spheres48; sc.nslots = spheres48 ? nslots : 0;
    sc.nodes = (const o_node *)nodes32; sc.tris = (const o_triangle *)tris64; sc.mats = (const o_material *)mats32;
    sc.n = sizes ? sizes[0] : 0; sc.m = sizes ? sizes[1] : 0;
    sc.mode = p->mode; sc.bounces = p->bounces; sc.step_cap = p->step_cap;
    sc.eps = p->mode == MODE_SPHERE ? 1e-6f : 1e-4f;
    uint64_t total = 0, tnodes = 0, ttris = 0, tcapped = 0;
    /* work items: (row, 64-column chunk) pairs, so a render of a few long rows (the full-frame-count checks of the
       timed configurations: 1-3 rows x 1024-4096 frames) still spreads over every thread; pixels are independent */
    const uint32_t XC = 64u, nxc = (p->nx + XC - 1u) / XC;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total, tnodes, ttris, tcapped)
#endif
    for (int64_t item = 0; item < (int64_t)p->nrows * nxc; item++) {
        const int64_t k = item / nxc;
        const uint32_t xa = p->x0 + (uint32_t)(item % nxc) * XC, xb = xa + XC < p->x0 + p->nx ? xa + XC : p->x0 + p->nx;
        const uint32_t rb = p->row_block > 1 ? p->row_block : 1;
        uint32_t y = p->row0 + ((uint32_t)k / rb) * p->row_step * rb + (uint32_t)k % rb;
        uint64_t q[4] = {0, 0, 0, 0};
        for (uint32_t x = xa; x < xb; x++) {
            float *px = image + ((size_t)k * p->nx + (x - p->x0)) * 3;
            float r = px[0], g = px[1], b = px[2];
            for (uint32_t f = 0; f < p->frames; f++) {
                uint32_t fc = p->frame0 + f;
                uint32_t time = p->time0 + f * p->dtime;
                v3 c = sample_pixel(&sc, p->width, p->height, x, y, time, q);
                float w = 1.0f / (fminf((float)fc, (float)p->ema_cap) + 1.0f);
                r = madd(c.x, w, r * (1.0f - w));
                g = madd(c.y, w, g * (1.0f - w));
                b = madd(c.z, w, b * (1.0f - w));
            }
            px[0] = r; px[1] = g; px[2] = b;
        }
        total += q[0];
        tnodes += q[1];
        ttris += q[2];
        tcapped += q[3];
    }
    if (counts) {
        counts[0] = total;
        counts[1] = tnodes;
        counts[2] = ttris;
        counts[3] = tcapped;
    }
    return total;
}

/* Size checks so the ctypes wrapper can verify it agrees on the POD layouts. */
uint32_t oracle_sizeof(int which) {
    switch (which) {
    case 0: return sizeof(o_camera);
    case 1: return sizeof(o_material);
    case 2: return sizeof(o_sphere);
    case 3: return sizeof(o_node);
    case 4: return sizeof(o_triangle);
    case 5: return sizeof(o_params);
    default: return 0;
    }
}
