/*
 * mafrix_rt.h — C ABI of the MI355X (gfx950) path-tracing hot path.
 *
 * This is the drop-in boundary for NAIVEddd/MafrixRaytracing's F# EngineCore hot path:
 * the F# `Scene` constructor and `Scene.Render` (EngineCore/Scene/Scene.fs:298-333) bind these
 * entry points through P/Invoke instead of running `PixelIntegrator`
 * (EngineCore/Core/Integrator/Integrators.fs:143-172) on the .NET thread pool.
 *
 * Conventions
 *  - extern "C", cdecl, plain pointers and sizes, no C++ or torch types.
 *  - Every struct is blittable (sequential layout, natural alignment) so .NET can pin it.
 *  - Return value: 0 on success, a negative MFX_E_* code on failure; mfx_last_error()
 *    gives a thread-local message. Nothing ever falls back to a CPU path.
 *  - One mfx_ctx is driven by one host thread at a time (the reference calls Sample from its
 *    single render thread, Film.fs:32, and fans out internally, Integrators.fs:164).
 *  - All calls are synchronous: when a call returns, its output buffer is complete.
 *
 * Numerics contract: every decision the reference makes in FP64
 * (camera ray, AABB slab test, Möller–Trumbore, sphere roots, rejection-sampled hemisphere,
 * light sample point, shadow distance) is made in FP64 with the reference's operation order
 * and no FMA contraction, so GPU paths follow the CPU oracle's paths bit for bit; the
 * BVH traversal that *finds* candidate leaves runs in FP32 with conservatively widened boxes.
 */
#ifndef MAFRIX_RT_H
#define MAFRIX_RT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MFX_ABI_VERSION 6  /* 6: device lists partition the film by tile rows; MFX_F_ROW_PARTITION */
#define MFX_MAX_DEVICES 64
#define MFX_MAX_RENDER_AHEAD 1024

/* error codes */
#define MFX_OK 0
#define MFX_E_INVALID (-1)   /* bad argument / malformed scene */
#define MFX_E_DEVICE (-2)    /* HIP runtime error, no device, kernel fault */
#define MFX_E_NOMEM (-3)     /* host or device allocation failed */
#define MFX_E_STATE (-4)     /* call out of order (e.g. render before create) */

/* Primitive kinds: the three IHitable structs the reference's Bvh holds (BvhNode.fs:24). */
#define MFX_PRIM_TRIANGLE 0  /* Triangle(v0,v1,v2,mat)        Core/Shape/Trangle.fs:107-119 */
#define MFX_PRIM_RECT 1      /* Rect(v0,v1,v2,v3,mat) = two triangles (v0,v1,v2),(v0,v2,v3)  Rect.fs:11-20 */
#define MFX_PRIM_SPHERE 2    /* Sphere(center,radius,mat)     Core/Shape/Sphere.fs:9-16 */

/* One primitive of the scene, in the order of Scene state.shapes (Scene.fs:168-177, 301).
 * The order matters: it is the index space Bvh.Build sorts (BvhNode.fs:25).
 *  TRIANGLE: p[0..2] = v0,v1,v2
 *  RECT:     p[0..3] = v0,v1,v2,v3 (the four OBJ face vertices, ObjModelLoader.fs:84-89)
 *  SPHERE:   p[0] = center, p[1][0] = radius                                              */
typedef struct mfx_prim {
    int32_t kind;
    int32_t material; /* index into mfx_scene_desc.albedo (MaterialManager order, IMaterial.fs:20-35) */
    double p[4][3];
} mfx_prim; /* 104 bytes */

/* NewAreaLight(p0,p1,p2,p3,normal,intensity) (Core/Lights/Light.fs:31-40), as built by
 * Scene.fs:193 from a Rect: (trig1.v0, trig1.v1, trig1.v2, trig2.v2, trig1.normal, I). */
typedef struct mfx_quad_light {
    double p[4][3];
    double normal[3];
    double intensity[3];
} mfx_quad_light;

/* PinholeCamera(pos, dir, fov, aspectRatio) (Core/Camera.fs:122-133). With derived == 0 the
 * library runs the constructor (CameraCoordinate + tan); with derived != 0 it takes an existing
 * camera's fields as they are — PinholeCamera.position, .topleft, .coord.right, .coord.down —
 * which is what the F# shim passes, so GetRay (Camera.fs:134-139) starts from identical bits. */
typedef struct mfx_pinhole {
    double position[3];
    double direction[3];
    double fov;    /* degrees, as in Scene.xml; effective horizontal FOV is fov/2 (Camera.fs:125) */
    double aspect; /* aspectratio attribute; NOT derived from the film size (Scene.fs:61-72) */
    double topleft[3], right[3], down[3];
    int32_t derived;
    int32_t reserved;
} mfx_pinhole;

/* The scene a `Scene` is constructed from (Scene.fs:298-313). Deep-copied by mfx_create. */
typedef struct mfx_scene_desc {
    const mfx_prim* prims;
    int64_t nprims;
    const double* albedo; /* [nmat][3] Lambert albedo per MaterialManager slot (Material.fs:29-37);
                             Metal -> its albedo (Material.fs:68), SpecularTransmission -> 0 (:121) */
    int32_t nmat;      /* at most 65,536 (the path pool keeps a vertex's material in 16 bits) */
    int32_t width;     /* Film width  (Scene.fs:201-211) */
    int32_t height;    /* Film height */
    int32_t max_depth; /* PathIntegrator maxDepth; the reference hard-codes 3 (Scene.fs:304) */
    mfx_quad_light light;
    mfx_pinhole camera;
} mfx_scene_desc;

/* Context options.
 * Devices: with ndevices == 0 the context runs on `device`. With ndevices > 0 it drives
 * devices[0..ndevices) from this one process (the reference's in-process fan-out,
 * Integrators.fs:164, across GPUs) by an image partition: device g of G traces the film's
 * 8-pixel tile rows of band g of G — one of each G consecutive tile rows, at offset g in even groups
 * and G - 1 - g in odd ones (serpentine) — every sample of the context's sample partition, on its own
 * stream. Every per-pixel operation (the sample-order sum, Film.AddSample, the post) therefore runs
 * on one device in the one-device order, and every output is bit-identical to a one-device
 * context's. mfx_render_rgba8 (render-ahead included) copies each device's rows of the RGBA8
 * frame straight into the caller's buffer; mfx_sample and mfx_film_mean merge the devices' FP64
 * buffers on devices[0] (one RCCL reduce over a communicator the library owns, ncclCommInitAll over
 * the list; a pixel is +0.0 on every device but its own, so the sum is an exact merge). A list that
 * repeats a device (e.g. {0,0}) merges by device-ordered adds instead (RCCL needs distinct devices). */
typedef struct mfx_options {  /* ABI 4: the former `reserved` field is render_ahead (0 = off); layout unchanged since */
    uint64_t seed;      /* counter-RNG seed; the reference uses unseeded System.Random */
    int32_t device;     /* HIP device ordinal when ndevices == 0 */
    int32_t flags;      /* MFX_F_* */
    int32_t part_index; /* this context renders sample partition part_index of part_count */
    int32_t part_count; /* (multi-process: one context per rank; partitions are disjoint sample sets;
                           with MFX_F_ROW_PARTITION disjoint sets of tile rows: band part_index of part_count) */
    int32_t ndevices;   /* 0: one device (`device`); 1..MFX_MAX_DEVICES: the device list below */
    int32_t render_ahead; /* 0 or 1: off. K in 2..MFX_MAX_RENDER_AHEAD: one-sample mfx_render_rgba8
                             calls (Scene.Render) take their sample from a batch of the next K
                             samples traced at once, on every device of a list (mfx_render_rgba8)  */
    const int32_t* devices; /* [ndevices] HIP device ordinals; devices[0] is the primary */
} mfx_options; /* 40 bytes */

#define MFX_F_NONE 0
#define MFX_F_COUNT_STATS 1 /* count traversal node/leaf/prim visits (slower; for the roofline model) */
#define MFX_F_MEGAKERNEL 2  /* one persistent megakernel instead of the wavefront pipeline */
#define MFX_F_HOST_BVH 4    /* build the traversal BVH on the host CPU (default: on the GPU; the same tree) */
#define MFX_F_WAVEFRONT 8   /* always the wavefront pipeline. Default: a call in which a device renders one
                               sample per pixel (Scene.Render) runs the megakernel, which is faster there
                               and gives the same bits (one path per pixel: no summation order) */
#define MFX_F_FLATTEN 16    /* mfx_create_instanced: flatten every instance into one BVH (no two-level
                               traversal); the same world scene, hits and images */
#define MFX_F_TWO_LEVEL 32  /* mfx_create_instanced: keep the two-level traversal. Default (neither flag):
                               flattened when the flat image fits MFX_FLATTEN_MAX_BYTES (env; default
                               2 GiB at 512 B per traversal slot of the expansion) and a sixteenth of
                               the device's free memory, two-level otherwise. Both flags: MFX_E_INVALID */
#define MFX_F_ROW_PARTITION 64 /* part_index / part_count partition the film's 8-pixel tile rows (serpentine
                               band part_index of part_count, as a device list's devices) instead of the
                               samples: a rank traces every sample of its rows,
                               its accumulator is +0.0 elsewhere, and a sum-reduce over the ranks is an exact
                               merge (the multi-process image partition; mfx_trace_accumulate)       */
#define MFX_F_IN_FLIGHT 128 /* the caller keeps frames in flight on several contexts of this device (each its
                               own pool and stream, frames alternating): the wavefront launches fetch larger
                               chunks of paths, since another frame's launches fill each launch's tail.
                               Scheduling only: the same images and ray counts (ABI 6, additive)     */

/* One entry of an instanced scene (mfx_create_instanced; an extension: the reference has no
 * instancing, its scenes are flat lists). The world primitive list — the index space Bvh.Build
 * sorts (BvhNode.fs:25) and every result refers to — is the concatenation, in entry order, of
 * each entry's copy of template primitives prims[first .. first + count): translated by `offset`
 * (every vertex, or a sphere's centre, + offset: one FP64 rounding per coordinate), or copied as
 * they are with MFX_INSTANCE_VERBATIM. Translated entries that share one template range are traced
 * through one template BVH (two-level traversal); everything else is flattened into the top level.
 * Results equal those of mfx_create on the expanded list (mfx_expand_instances), bit for bit.   */
typedef struct mfx_instance {
    int64_t first;
    int64_t count;
    double offset[3];
    int32_t flags;    /* MFX_INSTANCE_* */
    int32_t reserved;
} mfx_instance; /* 48 bytes */

#define MFX_INSTANCE_VERBATIM 1

typedef struct mfx_ctx mfx_ctx;

/* ---- lifetime ------------------------------------------------------------------------- */

/* Replaces `new Scene(state)` (Scene.fs:298-313): builds the reference's heap BVH leaf grouping
 * (BvhNode.fs:24-61), the GPU traversal BVH over it, uploads everything to HBM.            */
int mfx_create(const mfx_scene_desc* scene, const mfx_options* opt, mfx_ctx** out);
void mfx_destroy(mfx_ctx* ctx);
/* mfx_create for an instanced scene: scene->prims are the template primitives, `instances`
 * lists the entries whose expansion is the world scene (see mfx_instance).                    */
int mfx_create_instanced(const mfx_scene_desc* scene, const mfx_instance* instances, int32_t ninstances,
                         const mfx_options* opt, mfx_ctx** out);
/* Host-only: the world primitive list an instanced scene stands for (the library's own
 * expansion). out may be NULL to query the count; *nout = world primitives.                  */
int mfx_expand_instances(const mfx_prim* prims, int64_t nprims, const mfx_instance* instances,
                         int32_t ninstances, mfx_prim* out, int64_t cap, int64_t* nout);
/* How a context traces instances: out[0] = instances traced two-level, out[1] = template BVHs,
 * out[2] = top-level BVH4 nodes, out[3] = template BVH4 nodes, out[4] = slots per run of the
 * templates (each traced instance has its own run of world slots), out[5] = top-level slots,
 * out[6] = world slots, out[7] = bytes of the traversal images (nodes, slots, instance table).
 * All 0 but [5..7] for a flat context.                                                         */
int mfx_instancing_info(mfx_ctx* ctx, double out[8]);
/* Host-only (no device needed): the same figures for a scene built on the host from an instanced
 * description (MFX_F_FLATTEN honoured), plus the traversal stack bound. Without a device it
 * applies MFX_FLATTEN_MAX_BYTES alone: mfx_create_instanced also caps the flat image at a
 * sixteenth of the device's free memory, so on a nearly full device a context may trace two-level
 * where this reports flat (mfx_instancing_info out[0] > 0 tells a context's actual choice; the
 * images are the same either way).                                                              */
int mfx_build_instanced_info(const mfx_scene_desc* scene, const mfx_instance* instances, int32_t ninstances,
                             int32_t flags, double out[8], int32_t* stack_entries);

/* ---- the reference's render API --------------------------------------------------------- */

/* == IPixelIntegrator.Sample(spp) (IIntegrator.fs:35-40, Integrators.fs:161-172):
 * renders spp fresh samples per pixel and writes their mean as Color[w,h], x-major:
 * frame[(i*h + j)*4 + {0,1,2,3}] = r,g,b,1.0 for column i, row j (row 0 = top).
 * Successive calls draw successive global sample indices (the reference's RNG keeps
 * running between calls).                                                                  */
int mfx_sample(mfx_ctx* ctx, int32_t spp, double* frame_xmajor_rgba);

/* == Film.GetFrame(integrator, spp) + Scene.PostProcessAndToScreenBuffer
 * (Film.fs:18-34, Scene.fs:315-333): adds spp samples per pixel to the film, then writes the
 * progressive mean through ACES -> sqrt -> int(255.99 c) as RGBA8, y-major:
 * rgba[(y*w + x)*4 + {0,1,2,3}]. `Scene.Render(delta, buffer)` is this call with spp = 1.
 * rgba may be NULL (accumulate only).
 * Render-ahead (mfx_options.render_ahead = K > 1, part_count 1): one-sample calls are
 * served from batches of K samples. A call whose global sample is not held traces the next K
 * samples in one batched pass that runs the film add and post of all K calls ahead, in call
 * order; each call of the batch then only copies its RGBA8 frame, and while a batch is served the
 * next one is traced in the background (two buffers of K x 4 B + 48 B per pixel). Every frame's
 * bytes and the film equal the one-sample path's (a sample's image depends only on the seed and
 * its global index); after mfx_reset, an spp != 1 call or mfx_sample the next one-sample call
 * traces a batch again from the film as it then is. mfx_stats: the first call
 * served from a batch reports the K samples' rays and device time, the others 0 rays in 0 s. The
 * two buffers take at most MFX_RENDER_AHEAD_MAX_BYTES (environment; default 2 GiB) and a quarter of
 * the free HBM: K is cut to fit two buffers while at least 8 samples fit in each (1080p: 2 x 64 in 1.26 GB),
 * else one buffer of as many samples as fit (no background batch); when not even two samples fit,
 * the context frees the buffers and renders one sample per call from then on. A background batch
 * is traced once a batch starts being served, so an application that stops early has traced at
 * most one batch ahead. The accumulator (mfx_accum_read_mean) does not hold the samples of calls
 * served from batches. On a device list every device serves its tile rows from its own batches
 * (the same K on each: the tightest device's budget, shared by a list's contexts on one GPU).
 * mfx_film_mean after calls served mid-batch traces each served sample again once, film only.   */
int mfx_render_rgba8(mfx_ctx* ctx, int32_t spp, uint8_t* rgba_ymajor);

/* The same call under SURVEY.md §8(b)'s name for it (Film.GetFrame + PostProcess). */
int mfx_accumulate_render_rgba8(mfx_ctx* ctx, int32_t spp, uint8_t* rgba_ymajor);

/* == Film.Reset (Film.fs:26-30): zero the film accumulator and its frame count. */
int mfx_reset(mfx_ctx* ctx);

/* Film mean (target texture, Film.fs:23) as x-major RGBA doubles. */
int mfx_film_mean(mfx_ctx* ctx, double* frame_xmajor_rgba);

/* ---- lower-level entry points (multi-GPU composition, benchmarking) -------------------- */

/* Adds, for global samples [sample_base, sample_base + spp) of this context's partition,
 * the per-pixel radiance sums into the context's device accumulator (FP64, 3 planes of w*h,
 * plane-major, x-major pixels); on a multi-device context each device into its own.
 * Does not synchronise; mfx_sync() does.                                                     */
int mfx_trace_accumulate(mfx_ctx* ctx, int32_t spp, int64_t sample_base);
/* Multi-device context: sum every device's accumulator into the primary's (RCCL reduce, root
 * devices[0]), ordered after each device's trace: after a clear and a trace, an exact merge of
 * the devices' tile rows. No-op on a single-device context, and on an accumulator already merged
 * since the last trace, clear or attach. mfx_sample calls it itself.                             */
int mfx_accum_reduce(mfx_ctx* ctx);
int mfx_accum_clear(mfx_ctx* ctx);
/* Device pointer + byte size of the (primary device's) FP64 accumulator (for an RCCL reduce
 * across ranks).                                                                             */
int mfx_accum_device_ptr(mfx_ctx* ctx, void** dptr, int64_t* nbytes);
/* Use caller-owned device memory (>= the size above, on this context's device) as the
 * accumulator — e.g. a buffer an RCCL reduce then works on in place; NULL restores the
 * context's own buffer. The caller keeps it alive until detached or mfx_destroy.            */
int mfx_accum_attach(mfx_ctx* ctx, void* dptr, int64_t nbytes);
/* Copy accumulator / count to host as x-major RGBA doubles (alpha = 1): the division by the
 * sample count itself, as `color / float n` (Integrators.fs:171). count must be > 0. On a device
 * list it reads the merged accumulator: a trace not merged since (mfx_trace_accumulate, or the
 * trace of an mfx_render_rgba8 call without render-ahead) is merged first (mfx_accum_reduce).   */
int mfx_accum_read_mean(mfx_ctx* ctx, double count, double* frame_xmajor_rgba);
int mfx_sync(mfx_ctx* ctx);
/* The HIP stream (hipStream_t) the context launches on, for event timing by the caller.   */
int mfx_stream(mfx_ctx* ctx, void** stream);

/* Device time (ms) of the last mfx_trace_accumulate, from HIP events recorded on the
 * context's stream around its kernels (waits for them to finish).                           */
int mfx_last_trace_ms(mfx_ctx* ctx, double* ms);

/* Per-stage device time of the last mfx_trace_accumulate (wavefront pipeline), summed over its
 * iterations from HIP events around each kernel: out[0] = whole call, out[2] = the closest-hit
 * kernels (path start + closest hit: k_camera and k_extend), out[4] = k_shadow (shading + shadow
 * ray + path finish); out[1] = the part of out[2] spent in k_camera (each generation's camera
 * rays traced as packets, flat scenes) and out[3] = its launches (0 when k_extend traced them);
 * the per-generation k_resolve launches make up the rest of out[0]; out[5] = iterations
 * (max_depth + 1 per generation), out[6] = launches of each stage (= out[5]), out[7] =
 * generations. Megakernel: out[0] = out[2] = its single launch.                               */
int mfx_trace_timing(mfx_ctx* ctx, double out[8]);

/* Ray counters of the last mfx_trace_accumulate / mfx_sample call:
 * out[0] = primary, out[1] = extension (closest-hit queries actually traced, excluding the
 * reference's discarded depth -1 query), out[2] = shadow, out[3] = paths; with
 * MFX_F_COUNT_STATS: out[4..6] = internal-node visits, cluster (reference leaf) visits and
 * primitive tests of the closest-hit queries, out[7..9] the same for the shadow queries, and
 * out[10] / out[11] = the camera-ray packets' own fetches (k_camera: wave-uniform 128-B node
 * steps and leaf slots, once per wave; the per-ray visits of packet lanes are in out[4..6]).    */
int mfx_ray_counts(mfx_ctx* ctx, double out[16]);

/* The same counters summed over every mfx_trace_accumulate (and mfx_sample / mfx_render_rgba8
 * without render-ahead) since the context was created or last reset: each trace adds its counters
 * to device-side totals in stream order, so back-to-back traces need no host read in between (the
 * benchmark's timed steps). Waits for the context's work; reset != 0 zeroes the totals after the read. */
int mfx_ray_counts_total(mfx_ctx* ctx, double out[16], int32_t reset);

/* SURVEY.md §8(b)'s stats call, for the Mrays/s metric (§8(d)): rays = primary + extension +
 * shadow rays traced by the last mfx_sample / mfx_render_rgba8 / mfx_trace_accumulate call (the
 * sum of mfx_ray_counts out[0..2]), seconds = its device time (mfx_last_trace_ms / 1000; waits
 * for the call's kernels). Either pointer may be NULL.                                        */
int mfx_stats(mfx_ctx* ctx, double* rays, double* seconds);

/* ---- query entry points (parity tests of the BVH/intersection layer) ----------------- */

/* Closest hit, == Bvh.Hit(ray, tmin, tmax) (BvhNode.fs:62-83) for n rays given as
 * rays[k*6 + 0..2] = origin, [3..5] = unit direction. Outputs t (0 when no hit), prim index
 * (-1 when no hit; index into the mfx_prim array), and the hit normal.                      */
int mfx_closest_hit(mfx_ctx* ctx, int64_t n, const double* rays, double tmin, double tmax,
                    double* t_out, int32_t* prim_out, double* normal_out);
/* Shadow query, == Bvh.Hit(...).hit with per-ray tmax: occluded[k] = 1/0.                  */
int mfx_any_hit(mfx_ctx* ctx, int64_t n, const double* rays, double tmin, const double* tmax,
                int32_t* occluded_out);

/* Reference heap-BVH leaf grouping used for the exact leaf semantics (BvhNode.fs:24-61):
 * indices[nprims] after Subdivide; leaf_first/leaf_count per reference leaf in heap order.  */
int mfx_ref_leaves(mfx_ctx* ctx, int32_t* indices_out, int32_t* leaf_first_out,
                   int32_t* leaf_count_out, int32_t* nleaves_out);

/* Host-only (no device needed): the same leaf grouping computed straight from a scene
 * description, plus the traversal BVH's shape: info[0] = clusters, info[1] = internal BVH4
 * nodes, info[2] = LDS stack entries per lane, info[3] = traversal slots. Any output pointer
 * may be NULL.                                                                                */
int mfx_build_leaves(const mfx_scene_desc* scene, int32_t* indices_out, int32_t* leaf_first_out,
                     int32_t* leaf_count_out, int32_t* nleaves_out, int32_t info_out[4]);

/* How mfx_create built the scene (Scene ctor, Scene.fs:298-313; Bvh.Build, BvhNode.fs:24-61):
 * out[0] = ms for the reference leaf grouping (host), out[1] = ms for the traversal BVH2
 * (GPU incl. transfers, or host; with the GPU image layout: the whole traversal image), out[2] = ms
 * for the whole scene preparation, out[3] = 1 if the BVH2 was built on the GPU, 2 if its BVH4
 * collapse and image layout ran there too (flat scenes), out[4] = BVH4 nodes, out[5] = traversal slots, out[6] = BVH2
 * internal nodes, out[7] = BVH2 build levels. digest (may be NULL) = FNV-1a of the device
 * images (nodes, slots, slot_ref, ref_blob, shade): equal digests mean identical traversal.    */
int mfx_build_info(mfx_ctx* ctx, double out[8], uint64_t* digest);

/* Device FP64 self-test: computes a/b, sqrt(a) on the GPU for n pairs (bit-exactness check
 * of the device math the numerics contract relies on).                                      */
int mfx_fp64_selftest(int32_t device, int64_t n, const double* a, const double* b,
                      double* div_out, double* sqrt_out);

/* Device self-test of the exact shortcuts the traversal puts in front of AABB.hit
 * (IHitable.fs:18-54): rec = n records of 24 doubles (lo[3], hi[3], origin[3], direction[3],
 * tMin, tMax, a triangle's v0[3], e1[3], e2[3] whose vertex box lies inside [lo, hi], one pad);
 * out = 3 int32 per record: the FP64 test's answer (0/1), the FP32 screen's (1 hit, 0 miss, -1
 * left to the FP64 test) and the vertex-box proof's (1 proved to pass, 0 not proved). Wherever a
 * shortcut decides it must agree with the FP64 answer.                                         */
int mfx_aabb_selftest(int32_t device, int64_t n, const double* rec, int32_t* out);

/* How a context's work is laid over devices (ABI 6, additive): out[0] = devices G, out[1] = RCCL
 * communicators the context created (G for a list of distinct devices, else 0), out[2] = how
 * mfx_accum_reduce merges (0 one device, 1 RCCL reduce, 2 device-ordered adds: a repeated device),
 * out[3] / out[4] = the primary's tile-row band (band_index, band_count: the serpentine band
 * band_index), out[5 + g] = device g's HIP ordinal. cap = entries of out (>= 5 + G).          */
int mfx_device_info(mfx_ctx* ctx, int32_t* out, int32_t cap);

/* ---- misc -------------------------------------------------------------------------------- */
const char* mfx_last_error(void);
int mfx_abi_version(void);
int mfx_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* MAFRIX_RT_H */
