/*
 * hrt.h — C-ABI of the MI355X-native path tracer (drop-in for hucancode/hello-raytracing's per-pixel ray
 * loop). Plain pointers, sizes and int status codes; no C++ or torch types cross this boundary.
 *
 * Two groups of entry points:
 *   rt_*  (renderer)  replace the wgpu Renderer + bind-group ABI + WGSL fs_main of the reference
 *                     (src/renderer.rs, src/shaders/shader_{sphere,tris}.wgsl). Backed by HIP kernels
 *                     for gfx950; they fail with RT_ERR_DEVICE when no MI355X is present — there is
 *                     no CPU fallback.
 *   rt_host_* (scene) host-side builders whose output bytes feed the renderer: Camera::new, Mesh::load_obj,
 *                     Tree::add_mesh/build, render_ppm, compare_ppm_images. Pure CPU.
 *
 * Every input buffer uses the reference's #[repr(C)] bytemuck POD layout byte for byte:
 *   Camera   80 B  {eye, direction, up, right: vec4<f32>; params: (focal, blur, fov, 0)} src/scene/camera.rs:6-12
 *   Material 32 B  {albedo: vec4<f32>; params: vec3<f32>; kind: u32}                      src/scene/material.rs:9-13
 *   Sphere   48 B  {center: vec3<f32>; radius: f32; material: Material}                   src/scene/sphere.rs:6-10
 *   Node     32 B  {bound_min: vec4<f32>; bound_max: vec4<f32>}                          src/scene/bvh/node.rs:6-9
 *   Triangle 64 B  {a, b, c: vec4<f32>; custom(normal): vec3<f32>; material: u32}       src/scene/bvh/triangle.rs:7-13
 * The callee copies every input (caller keeps ownership), as wgpu's queue.write_buffer does
 * (renderer.rs:350-353). One handle must not be used from two threads at once. A renderer stays on the
 * GPU that was current when it was created: every call that touches the device makes that GPU current for
 * its duration and restores the caller's current device before returning.
 */
#ifndef HRT_H
#define HRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (the reference panics via unwrap/expect instead, e.g. renderer.rs:64,83,117) ---- */
#define RT_OK 0
#define RT_ERR_ARG (-1)      /* null pointer, zero size, bad mode, size mismatch                   */
#define RT_ERR_DEVICE (-2)   /* no gfx950 device / HIP runtime error                               */
#define RT_ERR_ALLOC (-3)    /* device or host allocation failed                                   */
#define RT_ERR_STATE (-4)    /* call out of protocol order (e.g. draw before camera)               */
#define RT_ERR_PARSE (-5)    /* OBJ parse error (tobj LoadError)                                   */
#define RT_ERR_COMPARE (-6)  /* compare_ppm_images failed (see rt_host_compare_ppm)                */

/* ---- scene modes: which WGSL program the renderer runs ---- */
#define RT_MODE_SPHERE 0 /* shader_sphere.wgsl: sphere list, BOUNCE_MAX 10, EPSILON 1e-6             */
#define RT_MODE_TRIS 1   /* shader_tris.wgsl: implicit-heap BVH of triangles, BOUNCE_MAX 5, EPS 1e-4 */
#define RT_MODE_MIXED 2  /* build-defined union (tris constants + sphere list), DESIGN.md §Mixed     */

/* Material kinds, src/scene/material.rs:4-6 */
#define RT_LAMBERTIAN 1u
#define RT_METAL 2u
#define RT_DIELECTRIC 3u

#define RT_MAX_OBJECT_IN_SCENE 100u /* scene_sphere.rs:15 — sphere buffer capacity = arrayLength */
#define RT_SAMPLE_FRAME 1000u        /* shader_*.wgsl SAMPLE_FRAME: EMA cap of the accumulation     */

typedef struct rt_renderer rt_renderer;

/* Runtime knobs that are compile-time constants in the WGSL (shader_sphere.wgsl:3-12). */
typedef struct rt_params {
    uint32_t bounces;          /* BOUNCE_MAX; default 10 (sphere) / 5 (tris, mixed)                     */
    uint32_t ema_cap;          /* SAMPLE_FRAME; default 1000                                          */
    uint32_t min_sphere_slots; /* arrayLength(&scene) floor; default 100 (zero-filled slots traced)    */
    uint32_t row0, row_step;   /* this renderer owns rows row0, row0+row_step, ... (multi-GPU tiles); with
                                  row_block > 1 the blocks of row_block rows starting there (below)    */
    uint32_t frames_per_launch;/* frames fused into one kernel launch by rt_draw_frames (default 32)   */
    uint32_t variant;          /* sphere-scan kernel: 0 auto (4 from 32 slots, 3 from 9, else 1), 1 simple,
                                  3 packed + deferred exact candidates, 4 conservative culling BVH;
                                  all bit-identical. 2 and 5-10 were removed.    */
    uint32_t schedule;         /* work schedule of rt_draw / rt_draw_frames: 0 auto (queue from 1.5M
                                  samples per draw, else tiles), 1 tiles (one lane per pixel for a
                                  launch's frames, in-register accumulation), 2 sample queue (persistent
                                  grid pulling 8x8-tile x job_frames jobs, colours folded in frame
                                  order); bit-identical                       */
    uint32_t queue_budget_mb;  /* sample-queue colour memory: 0 (default) auto = the sample buffer in
                                  floor(frames / 320) balanced launches of whole jobs (at least one), or as
                                  many frames per launch as 8 GiB holds if that is more, at most 32 GiB
                                  (C3: 352 + 352 + 320 frames, 8.8 GB; a rank of an 8-way C3: one launch);
                                  else a cap in MiB: balanced launches of as many frames as it holds. The
                                  fold ring (bounded memory, slower) when a launch would get fewer than
                                  min(frames, 320) frames                                 */
    uint32_t job_frames;       /* sample queue: frames per job (a job = one 8x8 tile), rounded down to a
                                  power of two (at most 1024); default 0 = per kernel: 32 with the
                                  suspendable walks, 16 for the linear sphere scans                      */
    uint32_t tri_bvh;          /* triangle program: 0 the reference's implicit-heap walk (default,
                                  parity), 1 opt-in binned-SAH tree with an ordered culling walk — the
                                  same closest hit except where the reference's 600-step cap or
                                  unpadded slab tests drop a triangle (non-parity)  */
    uint32_t suspend_below;    /* sample queue: a wave suspends its walks (sphere culling BVH of the sphere
                                  program; reference heap walk of the triangle / mixed programs) once
                                  fewer than this many of its 64 lanes are still walking, so finished
                                  lanes shade and start their next query instead of idling (0 = no wave
                                  leaves a walk before all of its lanes finish); default 24 (sphere and
                                  mixed) / 32 (triangle); not used by tri_bvh = 1 or the linear sphere scans.
                                  Bit-identical either way                      */
    uint32_t row_block;        /* rows per block of the row partition (default 1; 0 reads as 1): the renderer
                                  owns rows row0 + k*row_step*row_block + j, j < row_block, in that order.
                                  Rank r of N with row_block 8 and row0 = 8r, row_step = N owns whole
                                  8-row tile rows dealt round-robin (bench.py)            */
    uint32_t fold;             /* sample queue colour fold: 0 auto (by queue_budget_mb, above; with the automatic
                                  budget, draws of two or more launches of the suspendable-walk kernels fold as 3),
                                  1 the sample buffer + k_accumulate after every launch, 2 the fold ring (bounded
                                  memory), 3 two sample buffers: each launch's waves fold the launch before it (1 in
                                  64 waves first folds tiles, then traces), k_accumulate the last launch only —
                                  twice the colour memory of 1 (C3 17.5 GB), C3 +1 %;
                                  k_trace's draws fold as 1; bit-identical                               */
    uint32_t heap_lds;         /* triangle / mixed programs: the top of the implicit heap in LDS, 0 auto = on,
                                  1 off (every node from L1/L2), 2 on: nodes 1..1023 as sign-ordered nodes
                                  (768-lane workgroups; nodes 1..255 with the deferred sphere scan; heaps of
                                  at most 2^24 nodes); bit-identical always                               */
    uint32_t steal;            /* sample queue with the sample buffer, suspendable-walk kernels: frame-block work
                                  stealing (a wave whose job queue is drained claims single frames of other
                                  waves' jobs, so no long job trails the launch): 0 auto = on for launches of
                                  fewer than 16 jobs per resident wave, 1 off, 2 on; bit-identical always  */
    uint32_t tail_split;       /* suspendable-walk kernels (k_trace_split, k_trace_split_tris) with the sample
                                  buffer and no stealing: the launch's last ~2 jobs per resident wave are dealt
                                  in parts, so the drain waits for a part of a job: 0 auto (quarters), 1 off,
                                  2 quarters, 3 eighths (job_frames a multiple of the part count);
                                  bit-identical                                                          */
    uint32_t count_tests;      /* 1: count the sphere program's culling-walk box and sphere tests
                                  (rt_stats.box_tests / sphere_tests); 0 (default): the sphere program's
                                  k_trace_split does not count them (reported 0; 1.3 % of C3's kernel
                                  time); the other kernels always count                                  */
    uint32_t cost_order;       /* sample queue with the sample buffer: deal a launch's most expensive tiles first
                                  (half of them, sorted by the queries their samples took in a learning launch;
                                  then the rest in raster order), so the slowest jobs do not trail
                                  the launch. The first launch after a change of scene, camera, size, rows,
                                  bounce cap, sphere slots or triangle walk learns (and deals in the last order
                                  learnt, or raster order).
                                  0 auto = on for a rank's share of a row partition (row_step > 1), which then
                                  does not steal once it has learnt, and for the suspendable-walk kernels (not
                                  the linear scans' full images), 1 off, 2 on, 3 on with every launch learning;
                                  bit-identical always                           */
    uint32_t packet;           /* sphere program, culling BVH with its nodes in LDS (k_trace_split): walk each frame
                                  block's 64 primary rays as one coherent packet when the block is made (one
                                  wave-uniform traversal of the union of their nodes) and hand the samples out with
                                  their first hit resolved: 0 auto = off, 1 off, 2 on; bit-identical images and
                                  query counts (box / sphere test counts then count the packet's tests). Off by
                                  default: C3 35.2 vs 38.3 Grays/s                 */
} rt_params;

#define RT_FOLD_AUTO 0u
#define RT_FOLD_BUFFER 1u
#define RT_FOLD_RING 2u
#define RT_FOLD_NEXT 3u

#define RT_SCHEDULE_AUTO 0u
#define RT_SCHEDULE_TILES 1u
#define RT_SCHEDULE_QUEUE 2u

typedef struct rt_stats {
    uint64_t queries;      /* closest-hit queries (rays) traced by the last draw call                  */
    uint64_t samples;      /* pixel-samples (pixels x frames) of the last draw call                    */
    double kernel_ms;      /* HIP-event time of the last draw call's kernels, on the renderer stream   */
    uint32_t launches;     /* kernel launches of the last draw call                                    */
    uint32_t local_rows;   /* rows owned by this renderer                                              */
    uint64_t box_tests;    /* padded-box tests of the sphere culling BVH (variant 4), last draw call    */
    uint64_t sphere_tests; /* ray-sphere tests (slots scanned, or BVH leaf + large-list tests)          */
    uint32_t variant;      /* sphere-scan variant the last draw call ran (1, 3, 4)                       */
    uint32_t schedule;     /* schedule the last draw call ran (RT_SCHEDULE_TILES / _QUEUE)             */
    uint64_t node_tests;   /* triangle program: implicit-heap node (slab) tests                         */
    uint64_t tri_tests;    /* triangle program: Moller-Trumbore tests                                   */
    double trace_ms;       /* HIP-event time of the ray-tracing kernels alone (k_render / k_trace)      */
    uint32_t trace_launches; /* launches of those kernels (the dominant kernel's launch count)          */
    uint32_t suspend_below; /* walks suspended below this many walking lanes in the last draw (k_trace_split*);
                              0 = every query ran to completion (k_trace, k_render)                    */
    char kernel[64];       /* the ray-tracing kernel the last draw ran, as rocprofv3 names it without
                              "void " and the argument list, e.g. "k_trace_split<true>"                 */
    uint64_t fold_bytes;   /* device memory the sample queue's colour fold used in the last draw: the sample
                              buffer (frames per launch x pixels x 12 B) or the fold ring (job slots x
                              job_frames x 64 px x 16 B plus control words); 0 for the tiles schedule    */
    uint32_t fold_ring;    /* 1: the last draw folded through the fold ring (bounded memory), 0: through the
                              sample buffer and k_accumulate, 2: through two sample buffers, each launch folded
                              inside the next (rt_params.fold 3; rt_params.queue_budget_mb decides)        */
    uint32_t launch_frames; /* sample queue: frames per trace launch of the last draw (the last launch may
                              have fewer; rt_params.queue_budget_mb)                                   */
    uint64_t device_bytes; /* device memory the renderer holds after the last draw call (image, scene,
                              colour fold, counters): the fold's share stays within queue_budget_mb      */
    uint32_t ordered_launches; /* trace launches of the last draw that dealt their tiles in cost order
                              (rt_params.cost_order)                                                    */
    uint32_t reserved;
} rt_stats;

/* Renderer::new(RenderOutput::Headless(w, h), ..) — renderer.rs:46-269. Zeroes the image (:249-257),
 * frame_count = 0. Selects the program (mode) like include_str!(shader) does (scene_sphere.rs:186). */
int rt_create(uint32_t width, uint32_t height, int mode, rt_renderer **out);
int rt_destroy(rt_renderer *r);
int rt_get_params(const rt_renderer *r, rt_params *out);
/* Changing row0/row_step re-allocates and zeroes the image (like resize). */
int rt_set_params(rt_renderer *r, const rt_params *p);

/* Renderer::set_camera — renderer.rs:324-328 (group0 binding 4, 80 B). */
int rt_set_camera(rt_renderer *r, const void *camera80);
/* SceneSphere::write_scene_data -> Renderer::write_buffer(data, 0) — scene_sphere.rs:24-31,
 * renderer.rs:350-353 (group1 binding 0). n spheres of 48 B; slots past n are zero, like the wgpu buffer. */
int rt_set_spheres(rt_renderer *r, const void *spheres48, uint32_t n);
/* SceneTris::write_tree_data — scene_tris.rs:21-44 (group1 bindings 0..3): sizes = [n, m] (bvh_tree_size),
 * n Node (index 0 unused), m Triangle, k Material. n must be a power of two, as Tree::build makes it
 * (tree.rs:38, m.next_power_of_two()), and at most RT_MAX_TREE_NODES (the kernels read nodes and triangles
 * through buffer descriptors with 32-bit byte offsets: n x 32 B and m x 64 B stay below 4 GiB); RT_ERR_ARG
 * otherwise (rt_host_check_bvh_sizes applies the same rules without a device). */
int rt_set_bvh(rt_renderer *r, const uint32_t sizes[2], const void *nodes32, uint32_t n_nodes,
               const void *tris64, uint32_t n_tris, const void *mats32, uint32_t n_mats);
#define RT_MAX_TREE_NODES (1u << 26) /* 2^26 nodes (2 GiB), up to 2^26 - 1 triangles (4 GiB)            */

/* Renderer::set_time / set_frame_count — renderer.rs:315-323. */
int rt_set_time(rt_renderer *r, uint32_t time);
int rt_set_frame_count(rt_renderer *r, uint32_t frame_count);
int rt_get_frame_count(const rt_renderer *r, uint32_t *out);

/* Renderer::draw — renderer.rs:355-410: one frame (one sample per pixel) at the current time,
 * frame_count += 1. Asynchronous on the renderer's HIP stream. */
int rt_draw(rt_renderer *r);
/* `count` frames with time_f = time0 + f*dtime, frame_count advancing by one per frame: bit-identical
 * to count x {rt_set_time(time_f); rt_draw()}. The tiles schedule accumulates in registers in-kernel; the
 * sample queue stores each sample's colour (sample buffer or fold ring) and folds them in frame order with
 * the same expression (k_accumulate after the launch, or inside it), see rt_params.fold. */
int rt_draw_frames(rt_renderer *r, uint32_t count, uint32_t time0, uint32_t dtime);

/* render_ppm's copy_image_buffer — render_ppm.rs:7-36: blocking readback of the f32 RGB image,
 * row-major, (local_rows x width x 3) floats. */
int rt_read_image(rt_renderer *r, float *out, size_t n_floats);
/* Restore an accumulation state (checkpoint/resume: image + rt_set_frame_count). */
int rt_write_image(rt_renderer *r, const float *in, size_t n_floats);
/* Device-to-device copy of the image into caller memory on the caller's device (multi-GPU gather). */
int rt_copy_image_to_device(rt_renderer *r, void *dst_device, size_t n_floats);
/* Renderer::reset_frame_count / resize — renderer.rs:336-348, :271-313 (both zero the image). */
int rt_reset_frame_count(rt_renderer *r);
int rt_resize(rt_renderer *r, uint32_t width, uint32_t height);
int rt_synchronize(rt_renderer *r);
int rt_get_stats(const rt_renderer *r, rt_stats *out);
/* Frees the sample queue's colour-fold memory (the sample buffer or the fold ring, rt_stats.fold_bytes)
 * after the pending draws; the next queue draw allocates it again. For a renderer kept alive between
 * renders beside other work: one C3 render holds 8.8 GB under the default budget (352 frames x 24.9 MB;
 * rt_stats.fold_bytes has the figure of the last draw) (no reference counterpart: wgpu frees nothing
 * either, but the reference has no per-sample buffer). */
int rt_release_scratch(rt_renderer *r);

/* Test-only entry points (fault injection) are declared in hrt_testing.h, not here: they are not part of
 * the drop-in surface. */

/* Raw per-draw device counters (no reference counterpart; diagnostics). Slots 0-4 are the rt_stats
 * work counters; in the diagnostic build (rt_diagnostic_build() == 1, lib/libhrt_diag.so) slots 8-11
 * hold summed wave clock cycles spent in closest-hit queries, shading, sample generation/accumulation
 * and whole wave lifetimes. Writes min(n, RT_RAW_COUNTERS) values, zero beyond. */
#define RT_RAW_COUNTERS 16
int rt_get_raw_counters(const rt_renderer *r, uint64_t *out, int n);
int rt_diagnostic_build(void);
/* Diagnostic build: per-wave records of the last launch of the last draw, 8 words per wave (waves in blockIdx.x *
 * waves per workgroup + wave order): start and end (s_memrealtime, 100 MHz ticks); HW_ID | XCC_ID << 32 (k_trace: the
 * longest time between two job takes in bits 0-23, its last job take << 40); the ticks until the wave first found no
 * work left | the frame blocks it generated << 32 (k_trace: the JOBS it took); the shader clock (s_memtime) at start,
 * end and that first drain; k_trace: lanes holding a sample at the drain | samples finished after the last job take
 * << 16 | rounds after the drain << 40 (scripts/wave_tail.py). Zero words in the product build. */
int rt_get_wave_trace(rt_renderer *r, uint64_t *out, size_t n_words);

/* Self-check of the kernels' range-restricted correctly rounded sqrt / division sequences against the IEEE
 * operations on n random cases each (diagnostics): mismatches[0] normalize of rng
 * vectors and normalize_exact of signed vectors, [1] division on [2^-60, 2^60] and the reciprocal of every
 * significand (case i's operand is fixed by i: n = 242 x 2^23 covers each under both signs of every binade
 * 2^-60 .. 2^60), [2] sqrt on [2^-100, 2^100].
 * All three must be 0. */
int rt_check_exact_math(uint64_t n, uint32_t seed, uint64_t mismatches[3]);

/* The GPU a renderer draws on (no reference counterpart; the multi-GPU bench checks every rank's renderer against
 * its torch device): the HIP device ordinal that was current at rt_create, and that device's PCI location
 * {domain, bus, device}. A process must load ONE HIP runtime for the ordinal to mean what the caller's runtime
 * means (hrt/_lib.py loads the one torch uses). */
int rt_get_device(const rt_renderer *r, int32_t *ordinal, int32_t pci[3]);

/* ABI guard (no reference counterpart): rt_params and rt_stats grow at their ends between versions, and rt_set_params
 * / rt_get_stats copy this header's sizes. A caller built against another header checks *version == RT_ABI_VERSION (or
 * the two sizes against its own sizeof) before the first rt_set_params / rt_get_stats. Any pointer may be NULL. */
#define RT_ABI_VERSION 6u /* 6: rt_params.packet (round 6); 5: rt_params.cost_order, rt_stats.ordered_launches */
int rt_abi_version(uint32_t *version, uint32_t *params_bytes, uint32_t *stats_bytes);

/* Thread-local message for the last failing call. */
const char *rt_last_error(void);
/* Number of visible gfx950 devices (0 on a CPU-only host; never an error). */
int rt_device_count(void);
/* Build string of the device code object ("gfx950 ..."), for the load check. */
const char *rt_build_info(void);

/* ================================ host-side scene builders ================================ */

/* Camera::new(from, to, focal_length, focal_blur_amount, fov) — src/scene/camera.rs:15-28 (glam 0.24 f32). */
int rt_host_camera_new(const float from[3], const float to[3], float focal_length, float focal_blur_amount,
                       float fov, void *camera80_out);

typedef struct rt_mesh rt_mesh;
typedef struct rt_tree rt_tree;

/* Mesh::load_obj(source, material) — src/geometry/mesh.rs:11-62 (tobj 4.0.3 default LoadOptions).
 * Like the reference, a parse failure yields an EMPTY mesh (status RT_OK) — see rt_host_mesh_counts. */
int rt_host_mesh_load_obj(const char *data, size_t len, const void *material32, rt_mesh **out);
int rt_host_mesh_counts(const rt_mesh *m, uint32_t *n_vertices, uint32_t *n_indices);
int rt_host_mesh_destroy(rt_mesh *m);

/* The size rules rt_set_bvh applies (sizes [n, m], buffer lengths, materials), without a device: RT_OK or
 * RT_ERR_ARG with rt_last_error() naming the rule. */
int rt_host_check_bvh_sizes(const uint32_t sizes[2], uint32_t n_nodes, uint32_t n_tris, uint32_t n_mats);

/* Tree::new / Tree::add_mesh / Tree::build — src/scene/bvh/tree.rs:20-90. */
int rt_host_tree_new(rt_tree **out);
int rt_host_tree_add_mesh(rt_tree *t, const rt_mesh *m);
int rt_host_tree_build(rt_tree *t);
/* Tree::build on `threads` host threads (0 = min(16, cores); rt_host_tree_build uses 0).
 * Level-synchronous BFS with concurrent stable sorts: byte-identical to the sequential build. */
int rt_host_tree_build_threads(rt_tree *t, int threads);
/* Views into the tree (valid until the next mutation): sizes [n, m], n nodes, m triangles, k materials. */
int rt_host_tree_view(const rt_tree *t, uint32_t sizes[2], const void **nodes32, uint32_t *n_nodes,
                      const void **tris64, uint32_t *n_tris, const void **mats32, uint32_t *n_mats);
int rt_host_tree_destroy(rt_tree *t);

/* render_ppm — src/scene/render_ppm.rs:38-57: ASCII P3, `(v*255) as u8` (saturating, truncating,
 * NaN -> 0). Writes at most cap bytes to out (may be NULL to query); *len = full length. */
int rt_host_render_ppm(const float *rgb, uint32_t width, uint32_t height, char *out, size_t cap, size_t *len);
/* compare_ppm_images — tests/rendering_tests.rs:84-131. Returns RT_OK if mean |du8| <= tolerance % of 255;
 * otherwise RT_ERR_COMPARE with *code = 1 DifferentDimensions, 2 PixelCountMismatch,
 * 3 ExcessiveDifference. *avg_diff_percent is filled whenever the pixel lists were compared. */
int rt_host_compare_ppm(const char *img1, size_t len1, const char *img2, size_t len2, float tolerance_percent,
                        int *code, float *avg_diff_percent);

#ifdef __cplusplus
}
#endif
#endif /* HRT_H */
