// mfx_wavefront.h — path-slot pool (SoA in HBM) of the wavefront pipeline.
//
// Each slot carries one path through a small state machine; every stage scans the pool and
// handles the slots in its state, so no ray queue (and no hot queue-tail atomic) exists:
//   FREE -> (logic) NEED_EXT -> (extend) EXT_DONE -> (shade) SHADOW_CONT | SHADOW_END | DONE
//   SHADOW_CONT -> (shadow) NEED_EXT,  SHADOW_END -> (shadow) DONE,  DONE -> (logic) FREE
// The only atomics are per-wave chunk fetches and per-block path allocations, spread over
// WF_SHARDS counters (a returning atomic on one word saturates near 88 per microsecond).
#ifndef MFX_WAVEFRONT_H
#define MFX_WAVEFRONT_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mfx_layout.h"

#define WF_FREE 0
#define WF_NEED_EXT 1
#define WF_EXT_DONE 2
#define WF_SHADOW_CONT 3
#define WF_SHADOW_END 4
#define WF_DONE 5

#define WF_SHARDS 8
// control words (unsigned long long) in WfParams.ctl
#define WF_CTL_PATH 0                 // [WF_SHARDS] path counters, shard g owns [g*T/8, (g+1)*T/8)
#define WF_CTL_EXT (WF_SHARDS)        // [WF_SHARDS] extend-kernel slot-chunk heads
#define WF_CTL_SHD (2 * WF_SHARDS)    // [WF_SHARDS] shadow-kernel slot-chunk heads
#define WF_NCTL (3 * WF_SHARDS)

struct WfParams {
    // scene
    const MfxNode* nodes;
    const uint8_t* blob;
    const MfxShade* shade;
    const double* albedo;
    const MfxLight* light;
    const MfxCamera* cam;
    double* accum;  // [3][w*h]
    // path slots (SoA)
    double *ox, *oy, *oz, *dx, *dy, *dz;  // current ray; origin = last hit point after shading
    double *tx, *ty, *tz;                 // throughput
    double *lx, *ly, *lz;                 // radiance
    double *sdx, *sdy, *sdz, *stmax;      // shadow ray direction, tmax = dist - 1e-6
    double *scx, *scy, *scz;              // this vertex's direct term if unoccluded
    double* hit_t;                        // closest hit t, -1 = miss
    int32_t* hit_slot;
    uint64_t* key;
    uint32_t* rn;
    int32_t* depth;
    int32_t* pixel;
    int32_t* state;
    // control
    unsigned long long* ctl;              // [WF_NCTL]
    unsigned long long* counters;         // [16] ray / traversal counters
    int64_t total;                        // path indices this call (incl. padding of edge tiles)
    uint64_t seed;
    int64_t sample_base;
    int32_t part_index, part_count;
    int32_t pool;
    int32_t width, height, max_depth;
    int32_t root_is_leaf;
    int32_t stack_size;
    int32_t chunk;                        // slots per chunk fetch of the traversal kernels
};

// doubles and 4-byte words per slot in the SoA pool
#define WF_DOUBLES_PER_SLOT 21
#define WF_WORDS_PER_SLOT 7  // key (2), rn, depth, pixel, state, hit_slot

hipError_t mfx_wf_occupancy(int stack_size, int* ext_blocks_per_cu, int* shd_blocks_per_cu);
// one iteration (logic, extend, shade, shadow); ev[0..2] are recorded after logic, extend, shade
hipError_t mfx_wf_iteration(const WfParams& P, int ext_grid, int shd_grid, bool stats, hipStream_t st,
                            hipEvent_t* ev);
hipError_t mfx_wf_finish(const WfParams& P, hipStream_t st);

#endif
