// mfx_wavefront.h — path-slot pool (SoA in HBM) of the wavefront pipeline.
//
// A frame's paths run in generations of at most `pool` paths: slot j of a generation holds path
// path_base + j for the generation's whole life, so no slot is recycled and nothing needs a path
// counter. A generation is max_depth + 1 iterations of (k_extend, k_shadow) — one bounce of every
// live path per iteration — and then k_resolve, which adds each pixel's finished paths into the
// accumulator in sample order (no FP64 atomics; the image is run-to-run deterministic).
//
// Each slot carries its path through a state machine; each kernel scans the pool for the slots
// in its state, so no ray queue (and no hot queue-tail atomic) exists:
//   FREE (iteration 1) | NEED_EXT -(k_extend: camera or extension ray, closest hit)-> HIT | MISS
//   HIT -(k_shadow: shade + shadow ray)-> NEED_EXT, DONE (a lit vertex recorded) or FREE (none)
//   MISS stays: a finished path (its state word holds the lit vertices; k_resolve folds it), black
//   for a camera ray's MISS | FRESH
// A path's radiance is not summed forward. Each vertex v records the operands of its BRDF factor
// c_v = col (the cosine ei and the material) and, when its shadow ray reaches the light, those of
// its direct term a_v = l / pdf_li (the cosine cs and the solid-angle factor), and k_resolve
// rebuilds c_v and a_v with the same FP64 expressions and folds them from the deepest lit vertex
// back to the camera, acc = (a_v + acc) * c_v: the reference's recursion (l / pdf_li +
// TraceRay(next)) * col / pdf (Integrators.fs:135-136, pdf = 1) in its own operation order, so the
// image is the oracle's bit for bit.
// A HIT state word also carries the hit's shade[] index, so the shading needs no extra lookup.
// The only atomics are per-wave chunk fetches, spread over WF_SHARDS counters (a returning
// atomic on one word saturates near 88 per microsecond).
#ifndef MFX_WAVEFRONT_H
#define MFX_WAVEFRONT_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mfx_layout.h"

#define WF_FREE 0
#define WF_NEED_EXT 1
#define WF_HIT 2    // k_extend found a hit: hit point in ox..oz, shade index in the state word
#define WF_MISS 3   // k_extend found no hit
#define WF_FRESH 4  // flag on WF_HIT / WF_MISS: the path's camera ray. Its throughput (1), radiance
                    // (0), draw count (2) and depth (max_depth) are implicit: never stored
#define WF_DONE 8   // finished with a lit vertex: k_resolve folds its vertices and adds them to its pixel
// A finished path's state word (WF_DONE, or WF_MISS left by k_extend) carries its lit-vertex mask
// << WF_SHADE_SHIFT, so k_resolve reads no depth word
#define WF_STATE_MASK 15
// A NEED_EXT state word written in place carries the path's lit mask << WF_SHADE_SHIFT too; k_extend's
// pending entries hold a slot index in 28 bits (pools of at most 2^28 slots), the mask above it
#define WF_ENTRY_SLOT 0x0fffffff
// scene kinds of the trace kernels' instances (k_extend / k_shadow SK)
#define WF_SK_FLAT 0
#define WF_SK_INST 1  // two-level (instanced) scene
#define WF_SK_SLDS 2  // small flat scene: every slot's test prefix in the kernel's LDS
#define WF_SHADE_SHIFT 4  // WF_HIT state word: shade[] index << WF_SHADE_SHIFT | flags
// depth word of a slot: remaining depth (low 8 bits) | lit-vertex mask << 8 (bit v: vertex v's
// shadow ray reached the light); so at most WF_MAX_VERTS vertices (max_depth < WF_MAX_VERTS)
#define WF_MAX_VERTS 16
#define WF_LIT_SHIFT 8

#ifndef WF_SHARDS
#define WF_SHARDS 64  // returning atomics on one word serialize (~88 per us): 8 shards -> 64 is +13 % on C2
#endif
#define WF_CHUNK_MAX 4096  // slots per chunk fetch, at most
#ifndef WF_LOOKAHEAD
#define WF_LOOKAHEAD 4  // windows whose state words a scan loads in one round
#endif
#define WF_NCTR 24  // counters per shard: [0..2] rays, [3] unused, [4..9] traversal statistics, [10..17] diagnostics,
                    // [WF_CTR_ITER + d] extension rays of iteration d (1 <= d < WF_ITER_CTRS; [1]
                    // holds the others, and the host's sums add these into it)
#define WF_CTR_ITER 18
#define WF_ITER_CTRS 6
// control words (unsigned long long) in WfParams.ctl. Shard g's counter of each array sits at
// [g * WF_HS]: device-scope atomics execute at the memory side one at a time per line, so each
// shard's counter has lines of its own (adjacent counters shared 4 lines between 64 shards, and the
// wave convoys at the end of every launch serialized on them)
#ifndef WF_HS
#define WF_HS 32  // unsigned long longs from one shard's counter to the next (256 B)
#endif
#define WF_CTL_EXT 0                       // [WF_SHARDS * WF_HS] k_extend slot-chunk heads
#define WF_CTL_SHD (WF_SHARDS * WF_HS)     // [WF_SHARDS * WF_HS] k_shadow slot-chunk heads
#define WF_CTL_CLOSED_EXT (2 * WF_SHARDS * WF_HS)       // k_extend's closed-shard mask (a line of its own)
#define WF_CTL_CLOSED_SHD (2 * WF_SHARDS * WF_HS + 16)  // k_shadow's
#define WF_NCTL (2 * WF_SHARDS * WF_HS + 32)
// the ray queues' shard counts sit on either side of the heads, so one memset per iteration clears
// the heads and the next queue's counts: [WF_CTL_Q0 | heads | WF_CTL_Q1], P.ctl = the heads
#define WF_CTL_Q0 (-WF_SHARDS * WF_HS)
#define WF_CTL_Q1 (WF_NCTL)
#define WF_CTL_ALLOC (WF_NCTL + 2 * WF_SHARDS * WF_HS)

// A vertex record's material: 16 bits (k_resolve reads every vertex level's array nearly whole, so
// its bytes are the kernel's cost); scenes are limited to 65,536 materials (mfx_create checks).
typedef uint16_t WfMat;
#define WF_MAT_MAX 65536

struct WfParams {
    // scene
    const MfxNode* nodes;
    const MfxSlot* slots;
    const int32_t* slot_ref;
    const uint8_t* ref_blob;
    const MfxShade* shade;
    const MfxInstance* inst;  // two-level scenes: instances (null for a flat scene)
    MfxLight light;  // by value: kernel arguments are scalar-loaded, never per-lane gathers (k_resolve)
    const MfxCamera* cam_dev;   // the camera in device memory: k_camera copies it into LDS
#if MFX_NODE_F16
    const MfxNodeH* nodes_h;    // MFX_NODE_F16 builds: the per-lane kernels' FP16 nodes (else null)
#endif
    const MfxLight* light_dev;
    const void* const* refs_dev;  // {slot_ref, ref_blob} in device memory (k_shadow copies them into LDS)  // the same in device memory: k_shadow copies it into LDS, so its 52
                                // dwords are not held in scalar registers through the kernel's loops
    MfxCamera cam;
    double* accum;  // [3][w*h]
    // render-ahead (k_resolve's frames mode): film != null makes the call's samples one-sample render
    // calls, added in order to the film state film[3][w*h] instead of accum, frames != null also gets
    // each call's RGBA8 frame (y-major, w*h*4 per sample index of the call), frameCount = count0 +
    // the sample's index + 1
    double* film;
    uint8_t* frames;
    double count0;
    // path slots (SoA)
    double *ox, *oy, *oz;  // ray origin; k_extend overwrites it with the hit point
    double *dx, *dy, *dz;  // ray direction
    double* vei;           // [vertex][stride] the vertex's cosine ei = n . wi (Material.fs:35)
    WfMat* vmat;           // [vertex][stride] its material (MaterialManager slot)
    double* vls;           // [vertex][2][stride] a lit vertex's cs = unit . n and solid = |cos_o| A / dist^2;
                           // gray_light: [vertex][0][stride] its direct term a_v itself
    int32_t gray_light;    // 1: the light's three intensities are bitwise equal, so a_v = (cs * (solid * I)) /
                           // pdf_li is one value for every channel: k_shadow records it (one double, one
                           // store) and k_resolve reads it instead of cs and solid (the same expression)
    int32_t lit_in_hit;    // 1 (max_depth <= 3, shade indices < 2^25): in place, a HIT state word carries the
                           // path's lit mask in bits 29..31 and k_shadow takes the remaining depth from the
                           // iteration, so no depth word is written or read in place
    int64_t vstride;       // slots per vertex-record row (the allocated pool)
    const double* albedo;  // [nmat][3] Lambert albedo per material (Material.fs:29-37)
    int32_t nmat;
    uint32_t* rn;          // RNG draws used so far
    int32_t* depth;        // remaining depth (PathIntegrator's d)
    int32_t* state;
    // Ray queues (MFX_RAY_QUEUE; null: every iteration works on the slot pool in place). From the
    // second iteration on, the arrays above are a queue's: entry i holds a continuing path's ray,
    // draw count, depth word and state, and qslot[i] names its slot, which keeps the path's
    // vertex records (vei, vmat, vls) and its final state word (fstate, with the lit mask: what
    // k_resolve reads). k_shadow appends the paths that continue to the next queue (n*), so the
    // sparse later bounces read and write dense memory instead of scattered slots.
    const int32_t* qslot;             // entry -> slot (null: entry = slot, the pool itself)
    const unsigned long long* qcount; // [WF_SHARDS * WF_HS] entries of each shard range of this iteration's queue (null: the pool)
    int32_t* fstate;                  // the slot pool's state words (== state in place)
    double *nox, *noy, *noz, *ndx, *ndy, *ndz;  // the next queue (null: continue in place)
    uint32_t* nrn;
    int32_t *ndepth, *nstate, *nslot;
    unsigned long long* ncount;       // [WF_SHARDS * WF_HS] its counts (beside ctl; zeroed with the heads)
    // control
    unsigned long long* ctl;              // [WF_NCTL]
    unsigned long long* counters;         // [WF_SHARDS][WF_NCTR] ray / traversal counters
    int64_t total;                        // paths of this generation (edge-tile padding included)
    int64_t path_base;                    // first path index of this generation
    uint64_t seed;
    int64_t sample_base;
    int32_t part_index, part_count;
    // image partition (a device list's devices, MFX_F_ROW_PARTITION ranks): this trace covers the
    // 8-pixel tile rows band_tile_row(band_index, band_count, k) (mfx_device.h: serpentine), band_rows
    // of them (1 / 0 / all: the whole film)
    int32_t band_index, band_count, band_rows;
    int32_t pool;                         // slots scanned (>= total, a multiple of 64)
    int32_t width, height, max_depth;
    int32_t stack_size;                   // traversal stack bound (entries per lane)
    int32_t stack_lds_ext, stack_lds_shd; // of which in LDS, per kernel; the rest in `spill`
    int32_t* spill;                       // [stack_size - stack_lds][grid * 256] deep stack entries
    int32_t chunk;                        // slots per chunk fetch of the kernels
    int32_t chunk_shd;                    // k_shadow's (half of chunk in place on a frame of at most 2^25 paths)
    int32_t start;                        // 1 in a generation's first iteration: FREE slots start paths
    int32_t tile_padding;                 // 1 if 8 does not divide the film: some path indices are padding
    int64_t base_smp, base_q;             // path_base = base_smp * per_sample + base_q
    int32_t ntop_ext, ntop_shd;           // top BVH nodes each trace kernel keeps in LDS (<= nodes)
    int32_t nslot_ext, nslot_shd;         // slots each trace kernel keeps in LDS (all of a small scene's, or 0)
    int32_t shadow_waves;                 // k_shadow instance: 3 or 4 waves per SIMD (register budget)
    int32_t ninst_lds;                    // two-level scenes: instances each trace kernel keeps in LDS
    int32_t cam_grid;                     // > 0: a generation's camera rays run k_camera (packets) on this grid
    int32_t iter;                         // the iteration (0 = camera rays); k_extend counts its rays per iteration
    int32_t res_tx0, res_ntx;             // k_resolve: only tile columns [res_tx0, res_tx0 + res_ntx) (0: every column)
};

#ifndef MFX_RAY_QUEUE
#define MFX_RAY_QUEUE 1  // continuing paths move to dense ray queues after the first vertex (MFX_RAY_QUEUE=0 at run time: in place)
#endif
// 8-byte and 4-byte words per slot in the SoA pool: o, d, and per vertex ei, cs, solid (8 B) and
// the material (4 B); with ray queues, two queues of o, d (8 B) and rn, depth, state, slot (4 B)
// per slot (queue 0 its own o, d, rn, depth, state, slot; queue 1 reuses the pool's o, d and rn,
// dead after the pool's last iteration, plus its own depth, state and slot). No RNG key is
// stored: k_shadow derives it from the path's slot at every vertex.
#define WF_DOUBLES_PER_SLOT(nvert) (6 + 3 * (nvert) + (MFX_RAY_QUEUE ? 6 : 0))
#define WF_WORDS_PER_SLOT(nvert) (3 + (nvert) + (MFX_RAY_QUEUE ? 7 : 0))  // rn, depth, state + the vertices' materials
// the two ray queues' share of that (queue 0's ray and draw count; both queues' depth, state and slot)
#define WF_QUEUE_BYTES_PER_SLOT (MFX_RAY_QUEUE ? 6 * 8 + 7 * 4 : 0)

#ifndef WF_STACK_LDS
#define WF_STACK_LDS 16  // traversal stack entries per lane kept in LDS (deeper ones spill to HBM/L2)
#endif
#ifndef WF_INST_LDS
#define WF_INST_LDS 64  // instance records (48 B) a trace kernel keeps in LDS, at most; more stay in global memory
#endif
#ifndef WF_SLOT_LDS_MAX
#define WF_SLOT_LDS_MAX 256  // slots a trace kernel may keep in LDS (80 B each; the whole array or none)
#endif
#ifndef WF_NTOP_MAX
#define WF_NTOP_MAX MFX_TOP_NODES  // top BVH nodes a trace kernel may keep in LDS (mfx_scene.cpp numbers them first)
#endif
// resident blocks per CU of k_extend / k_shadow with `stack_lds` stack entries per lane (spill: the
// SpillStack instance), ntop top BVH nodes and min(ninst, WF_INST_LDS) instance records in LDS
// (and nslot slots' test prefixes)
hipError_t mfx_wf_kernel_occupancy(bool shadow, int stack_lds, bool spill, int ntop, int ninst, int* blocks_per_cu,
                                   int nslot = 0);
// resident blocks per CU of k_camera (camera-ray packets)
hipError_t mfx_cam_occupancy(int stack_size, int* blocks_per_cu);
// a ray queue's arrays (MFX_RAY_QUEUE): entries in the pool's shard ranges, counts per shard
struct WfQueue {
    double *ox, *oy, *oz, *dx, *dy, *dz;
    uint32_t* rn;
    int32_t *depth, *state, *slot;
    unsigned long long* count;  // [WF_SHARDS * WF_HS]
};
// one iteration (extend, shadow); ev[0] is recorded between the two kernels (ev may be null)
hipError_t mfx_wf_iteration(const WfParams& P, int ext_grid, int shd_grid, bool stats, hipStream_t st,
                            hipEvent_t* ev);
// after a generation's last iteration: add its finished paths' radiance to their pixels
hipError_t mfx_wf_resolve(const WfParams& P, hipStream_t st);


#endif
