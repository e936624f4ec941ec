// packet_sim.cpp — STUDY (round 6), not product code. Cost model of walking a frame block's 64 primary rays as one
// coherent packet through the culling BVH, before any kernel is written.
//
// For sampled 8x8 tiles x frames of a sphere scene it generates the reference's primary rays (the oracle's make_ray,
// oracle/rt_oracle.c) and traces every sample's whole path with the oracle's closest hit. For every query it counts
// what today's per-lane walk does (k_trace_split's bvh_run: near child first, a child visited when its box is entered
// no later than the lane's best t; the large list scanned first), and for the primary rays of a block what a
// wave-uniform walk of the union of the 64 lanes' nodes does (a child visited when any lane enters it; every lane
// tests every sphere of a visited leaf). Boxes are the builder's f32 boxes unpadded — a model, not the kernel's
// exact padded fp16 test.
//
// Build: g++ -O2 -fopenmp -ffp-contract=off -I hello-raytracing_amd/csrc -o /tmp/packet_sim scripts/studies/packet_sim.cpp \
//        hello-raytracing_amd/csrc/host/sphere_bvh.cpp
// Run:   python scripts/studies/packet_run.py c3        (DESIGN.md §4 Round 6 has the results)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "host/sphere_bvh.hpp"

extern "C" {
#include "../../oracle/rt_oracle.c"
}

struct Stats {
    double q = 0, box = 0, leaf = 0, sph = 0;  // per-lane walk: queries, node visits (2 box tests each), leaves, spheres
};

static const hrt::SphereBvh* G;
static const float* GS;  // sph: cx cy cz r2 per leaf sphere

static inline bool box_hit(const float* mn, const float* mx, v3 o, v3 inv, float bt, float& te) {
    float t0x = (mn[0] - o.x) * inv.x, t1x = (mx[0] - o.x) * inv.x;
    float t0y = (mn[1] - o.y) * inv.y, t1y = (mx[1] - o.y) * inv.y;
    float t0z = (mn[2] - o.z) * inv.z, t1z = (mx[2] - o.z) * inv.z;
    float tmin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), 0.0f));
    float tmax = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    te = tmin;
    return tmin <= tmax && tmin <= bt;
}

static inline float sph_t(int k, v3 o, v3 d, float a) {
    const float* g = GS + 4 * k;
    v3 oc = V(o.x - g[0], o.y - g[1], o.z - g[2]);
    float b = 2.0f * dot3(oc, d), c = dot3(oc, oc) - g[3];
    float disc = fmaf(b, b, -((4.0f * a) * c));
    if (disc < 0.0f) return -1.0f;
    return (-b - sqrtf(disc)) / (2.0f * a);
}

static float large_best(const o_scene* sc, v3 o, v3 d) {
    float a = dot3(d, d), bt = FLT_MAX_REF;
    for (int s : G->large) {
        const o_sphere* sp = &sc->spheres[s];
        v3 oc = vsub(o, ld3(sp->center));
        float b = 2.0f * dot3(oc, d), c = dot3(oc, oc) - sp->radius * sp->radius;
        float disc = fmaf(b, b, -((4.0f * a) * c));
        if (disc < 0.0f) continue;
        float t = (-b - sqrtf(disc)) / (2.0f * a);
        if (t > 0.0f && t < bt) bt = t;
    }
    return bt;
}

// today's walk for one ray (bvh_run: near child first, far pushed)
static void lane_walk(const o_scene* sc, v3 o, v3 d, Stats& S) {
    float a = dot3(d, d), bt = large_best(sc, o, d);
    v3 inv = V(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    uint32_t stack[64];
    int sp = 0;
    uint32_t node = G->root_word;
    S.q++;
    while (true) {
        if (!(node & hrt::BVH_LEAF_BIT)) {
            const hrt::SphereBvhNode& n = G->nodes[node];
            float tl, tr;
            bool hl = box_hit(n.lmin, n.lmax, o, inv, bt, tl), hr = box_hit(n.rmin, n.rmax, o, inv, bt, tr);
            S.box++;
            bool lf = hl && (!hr || tl <= tr);
            if (hl && hr) stack[sp++] = lf ? n.right : n.left;
            if (hl || hr) { node = lf ? n.left : n.right; continue; }
        } else {
            uint32_t first = (node >> 4) & 0x07FFFFFFu, cnt = node & 15u;
            S.leaf++;
            S.sph += cnt;
            for (uint32_t j = 0; j < cnt; j++) {
                float t = sph_t(first + j, o, d, a);
                if (t > 0.0f && t < bt) bt = t;
            }
        }
        if (sp == 0) break;
        node = stack[--sp];
    }
}

struct Packet {
    double steps = 0, box = 0, leaf = 0, sph = 0, lanes_box = 0, lanes_leaf = 0;
};

// wave-uniform walk of the union: one step per visited node for all lanes; order by majority vote
static void packet_walk(const o_scene* sc, const v3* o, const v3* d, int n, Packet& P, int order, bool late = false) {
    float bt[64], a[64];
    v3 inv[64];
    for (int l = 0; l < n; l++) {
        a[l] = dot3(d[l], d[l]);
        bt[l] = late ? FLT_MAX_REF : large_best(sc, o[l], d[l]);  // late: the large list after the walk
        inv[l] = V(1.0f / d[l].x, 1.0f / d[l].y, 1.0f / d[l].z);
    }
    uint32_t stack[64];
    int sp = 0;
    uint32_t node = G->root_word;
    while (true) {
        if (!(node & hrt::BVH_LEAF_BIT)) {
            const hrt::SphereBvhNode& nd = G->nodes[node];
            int cl = 0, cr = 0, vote = 0;
            for (int l = 0; l < n; l++) {
                float tl, tr;
                bool hl = box_hit(nd.lmin, nd.lmax, o[l], inv[l], bt[l], tl), hr = box_hit(nd.rmin, nd.rmax, o[l], inv[l], bt[l], tr);
                cl += hl;
                cr += hr;
                if (hl && (!hr || tl <= tr)) vote++;
                else if (hr) vote--;
            }
            P.box++;
            P.lanes_box += (cl > cr ? cl : cr);
            bool lf = order == 0 ? vote >= 0 : (cl >= cr);
            bool hl = cl > 0, hr = cr > 0;
            if (hl && hr) stack[sp++] = lf ? nd.right : nd.left;
            if (hl || hr) { node = (hl && hr) ? (lf ? nd.left : nd.right) : (hl ? nd.left : nd.right); continue; }
        } else {
            uint32_t first = (node >> 4) & 0x07FFFFFFu, cnt = node & 15u;
            P.leaf++;
            P.sph += cnt;
            for (int l = 0; l < n; l++)
                for (uint32_t j = 0; j < cnt; j++) {
                    float t = sph_t(first + j, o[l], d[l], a[l]);
                    if (t > 0.0f && t < bt[l]) bt[l] = t;
                }
        }
        if (sp == 0) break;
        node = stack[--sp];
    }
}

// the reference heap walk (intersect_all_node, shader_tris.wgsl:268-301) for one ray: steps (visited indices)
static double heap_lane(const o_scene* sc, v3 o, v3 d) {
    v3 inv = V(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    uint32_t i = 1, n = sc->n, m = sc->m, step = 0;
    while (step < 600u) {
        step++;
        if (i < n && node_hit(o, inv, &sc->nodes[i])) { i *= 2u; continue; }
        if (i >= n && i - n >= m) break;
        while ((i & 1u) == 1u) i /= 2u;
        if (i == 0u) break;
        i++;
    }
    return step;
}

// the union of a packet's heap walks, each lane counting its own visits: the wave visits index i
// when some lane is inside i's subtree (every ancestor hit for it, not stopped); a lane stops at its first empty leaf or
// its 600th step. Returns the union's steps; *lanes += participating lanes summed over the steps.
static double heap_union(const o_scene* sc, const v3* o, const v3* d, int nl, double* lanes) {
    v3 inv[64];
    uint32_t hd[64], st[64];
    bool term[64];
    for (int l = 0; l < nl; l++) {
        inv[l] = V(1.0f / d[l].x, 1.0f / d[l].y, 1.0f / d[l].z);
        hd[l] = 0, st[l] = 0, term[l] = false;
    }
    uint32_t i = 1, depth = 0, n = sc->n, m = sc->m;
    double steps = 0;
    while (true) {
        bool any_hit = false, any = false;
        for (int l = 0; l < nl; l++) {
            if (term[l] || hd[l] < depth) continue;
            any = true;
            st[l]++;
            if (i < n) {
                bool h = node_hit(o[l], inv[l], &sc->nodes[i]);
                hd[l] = h ? depth + 1 : depth;
                any_hit |= h;
            } else if (i - n >= m) {
                term[l] = true;
            }
            if (st[l] >= 600u) term[l] = true;
        }
        if (any) {
            steps++;
            for (int l = 0; l < nl; l++) *lanes += (!term[l] || st[l] >= 600u) && hd[l] >= depth ? 1 : 0;
        }
        if (i < n && any_hit) { i *= 2u; depth++; continue; }
        while ((i & 1u) == 1u) { i /= 2u; depth--; }
        if (i == 0u) break;
        i++;
        bool live = false;
        for (int l = 0; l < nl; l++) live |= !term[l];
        if (!live) break;
    }
    return steps;
}

int main(int argc, char** argv) {
    if (argc < 7) {
        fprintf(stderr, "usage: packet_sim scene.bin W H bounces ntiles frames\n");
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    uint32_t nsl;
    float cam[20];
    if (fread(cam, 4, 20, f) != 20 || fread(&nsl, 4, 1, f) != 1) return 3;
    std::vector<o_sphere> sph(nsl);
    if (fread(sph.data(), sizeof(o_sphere), nsl, f) != nsl) return 3;
    uint32_t tm[4] = {0, 0, 0, 0};  // mode, n, m, k
    std::vector<o_node> nodes;
    std::vector<o_triangle> tris;
    std::vector<o_material> mats;
    if (fread(tm, 4, 4, f) == 4 && tm[0] != MODE_SPHERE) {
        nodes.resize(tm[1]);
        tris.resize(tm[2]);
        mats.resize(tm[3]);
        if (fread(nodes.data(), 32, tm[1], f) != tm[1] || fread(tris.data(), 64, tm[2], f) != tm[2] ||
            fread(mats.data(), 32, tm[3], f) != tm[3])
            return 3;
    }
    fclose(f);
    const uint32_t W = atoi(argv[2]), H = atoi(argv[3]), B = atoi(argv[4]), NT = atoi(argv[5]), NF = atoi(argv[6]);
    std::vector<float> cr(4 * nsl);
    for (uint32_t i = 0; i < nsl; i++) {
        cr[4 * i] = sph[i].center[0], cr[4 * i + 1] = sph[i].center[1], cr[4 * i + 2] = sph[i].center[2];
        cr[4 * i + 3] = sph[i].radius;
    }
    hrt::SphereBvh bvh = hrt::build_sphere_bvh(cr);
    G = &bvh;
    GS = bvh.sph.data();
    o_scene sc;
    memset(&sc, 0, sizeof sc);
    sc.cam = (const o_camera*)cam;
    sc.k = tanf(sc.cam->params[2] * 0.5f);
    sc.spheres = sph.data();
    sc.nslots = nsl;
    sc.mode = tm[0];
    sc.bounces = B;
    sc.eps = tm[0] == MODE_SPHERE ? 1e-6f : 1e-4f;
    sc.step_cap = 600;
    if (tm[0] != MODE_SPHERE) {
        sc.nodes = nodes.data(), sc.tris = tris.data(), sc.mats = mats.data(), sc.n = tm[1], sc.m = tm[2];
        if (tm[0] == MODE_TRIS) sc.nslots = 0;
    }
    const bool heap = tm[0] != MODE_SPHERE;
    double hp = 0, hs = 0, nhp = 0, nhs = 0, hu = 0, hul = 0, rc_hit = 0, rc_cull = 0, rc_steps = 0;
    const uint32_t tw = (W + 7) / 8, th = (H + 7) / 8;
    Stats prim, sec;
    Packet pk[3];
    double npk = 0, nrays_pk = 0;
    uint32_t seed = 12345u;
    for (uint32_t it = 0; it < NT; it++) {
        rng_int(&seed);
        const uint32_t tile = seed % (tw * th);
        for (uint32_t fr = 0; fr < NF; fr++) {
            const uint32_t time = 1000u + 10u * (fr * 97u + it);
            v3 po[64], pd[64];
            int n = 0;
            for (int l = 0; l < 64; l++) {
                uint32_t x = (tile % tw) * 8 + (l & 7), y = (tile / tw) * 8 + (l >> 3);
                if (x >= W || y >= H) continue;
                // fs_main prologue (oracle sample_pixel)
                uint32_t s = (x * H + y) * time;
                float aspect = (float)W / (float)H;
                float r1 = rng_float(&s), r2 = rng_float(&s);
                float ssa = fmaf(r2, r2, r1 * r1), len = sqrtf(ssa);
                float px = ((float)x + 0.5f) + r1 / len, py = ((float)y + 0.5f) + r2 / len;
                float ux = (2.0f * (px / ((float)W - 1.0f)) - 1.0f) * aspect, uy = (2.0f * (py / ((float)H - 1.0f)) - 1.0f) * -1.0f;
                ray_t r = make_ray(&sc, ux, uy, &s);
                po[n] = r.o;
                pd[n] = r.d;
                n++;
                // the sample's path: primary walk counted apart from the secondary ones
                ray_t cur = r;
                for (uint32_t b = 0; b < B; b++) {
                    if (sc.nslots) lane_walk(&sc, cur.o, cur.d, b == 0 ? prim : sec);
                    if (heap) {
                        const double st = heap_lane(&sc, cur.o, cur.d);
                        (b == 0 ? hp : hs) += st, (b == 0 ? nhp : nhs) += 1;
                        // root cull (mixed program): the mesh's root box entered beyond the sphere winner's t
                        if (sc.nslots) {
                            hit_t hs0 = {{0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}, FLT_MAX_REF, 0, 0};
                            closest_sphere(&sc, cur, &hs0);
                            v3 inv = V(1.0f / cur.d.x, 1.0f / cur.d.y, 1.0f / cur.d.z);
                            const o_node* nd = &sc.nodes[1];
                            float t0x = (nd->bmin[0] - cur.o.x) * inv.x, t1x = (nd->bmax[0] - cur.o.x) * inv.x;
                            float t0y = (nd->bmin[1] - cur.o.y) * inv.y, t1y = (nd->bmax[1] - cur.o.y) * inv.y;
                            float t0z = (nd->bmin[2] - cur.o.z) * inv.z, t1z = (nd->bmax[2] - cur.o.z) * inv.z;
                            float tmin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
                            float tmax = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
                            const bool root_hit = tmin <= tmax && tmax >= 0.0f;
                            if (root_hit) rc_hit++;
                            if (root_hit && tmin > hs0.t * 1.001f) rc_cull++, rc_steps += st;
                        }
                    }
                    hit_t h = {{0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}, FLT_MAX_REF, 0, 0};
                    if (sc.mode != MODE_TRIS) closest_sphere(&sc, cur, &h);
                    if (heap) {
                        uint64_t cnt[4] = {0, 0, 0, 0};
                        closest_bvh(&sc, cur, &h, cnt);
                    }
                    if (fabsf(h.t - FLT_MAX_REF) < sc.eps) break;
                    cur = scatter(&sc, &s, cur, &h);
                }
            }
            if (n == 0) continue;
            if (heap) hu += heap_union(&sc, po, pd, n, &hul);
            if (!sc.nslots) { npk++; nrays_pk += n; continue; }
            packet_walk(&sc, po, pd, n, pk[0], 0);
            packet_walk(&sc, po, pd, n, pk[1], 1);
            packet_walk(&sc, po, pd, n, pk[2], 0, true);
            npk++;
            nrays_pk += n;
        }
    }
    if (heap)
        printf("heap walk: per-lane steps per query: primary %.2f secondary %.2f (primary share of queries %.3f); union steps "
               "per packet of %.1f rays %.2f (participating lanes per step %.1f)\nHJSON {\"hp\": %.4f, \"hs\": %.4f, \"fp\": %.4f, "
               "\"rpp\": %.3f, \"hu\": %.4f, \"hul\": %.3f}\n",
               hp / nhp, hs / nhs, nhp / (nhp + nhs), nrays_pk / npk, hu / npk, hul / hu, hp / nhp, hs / nhs, nhp / (nhp + nhs),
               nrays_pk / npk, hu / npk, hul / hu);
    if (heap && sc.nslots)
        printf("root cull: queries %.0f, root box hit %.0f (%.3f), culled (entry > sphere t x 1.001) %.0f (%.3f of queries); "
               "heap steps they take %.0f = %.3f of all heap steps\n",
               nhp + nhs, rc_hit, rc_hit / (nhp + nhs), rc_cull, rc_cull / (nhp + nhs), rc_steps, rc_steps / (hp + hs));
    if (!sc.nslots) return 0;
    const double qall = prim.q + sec.q;
    printf("queries %.0f (primary %.0f = %.3f)\n", qall, prim.q, prim.q / qall);
    printf("per-lane walk, primary:   box %.2f leaf %.2f spheres %.2f per query\n", prim.box / prim.q, prim.leaf / prim.q, prim.sph / prim.q);
    printf("per-lane walk, secondary: box %.2f leaf %.2f spheres %.2f per query\n", sec.box / sec.q, sec.leaf / sec.q, sec.sph / sec.q);
    for (int k = 0; k < 3; k++)
        printf("packet walk (order %s): per packet of %.1f rays: box %.2f leaf %.2f spheres %.2f; lanes hitting per box step %.1f\n",
               k == 0 ? "vote" : k == 1 ? "count" : "vote, large list after the walk", nrays_pk / npk, pk[k].box / npk, pk[k].leaf / npk, pk[k].sph / npk, pk[k].lanes_box / pk[k].box);
    printf("JSON {\"q\": %.0f, \"qp\": %.0f, \"pbox\": %.4f, \"pleaf\": %.4f, \"psph\": %.4f, \"sbox\": %.4f, \"sleaf\": %.4f, \"ssph\": %.4f, "
           "\"rays_per_packet\": %.3f, \"ubox\": %.4f, \"uleaf\": %.4f, \"usph\": %.4f}\n",
           qall, prim.q, prim.box / prim.q, prim.leaf / prim.q, prim.sph / prim.q, sec.box / sec.q, sec.leaf / sec.q,
           sec.sph / sec.q, nrays_pk / npk, pk[0].box / npk, pk[0].leaf / npk, pk[0].sph / npk);
    return 0;
}
