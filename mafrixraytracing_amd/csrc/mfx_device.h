// mfx_device.h — kernel parameter blocks and host-side launcher declarations.
#ifndef MFX_DEVICE_H
#define MFX_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mfx_layout.h"

// Image partition (device lists, MFX_F_ROW_PARTITION ranks): band bi of bc owns one 8-pixel tile row
// of each group of bc consecutive tile rows, at offset bi in even groups and bc - 1 - bi in odd ones
// (serpentine), so a band's rows sit at every offset within the groups alike and a gradient of work
// down a group (C2: +4.5 % rays from its top tile row to its bottom one, r06b rank_rays_rel) does
// not load one band more than another. Its k-th tile row, and how many of the film's tr it owns:
__host__ __device__ inline int band_tile_row(int bi, int bc, int k) { return k * bc + ((k & 1) ? bc - 1 - bi : bi); }
__host__ __device__ inline int band_row_count(int bi, int bc, int tr) {
    const int g = tr / bc, off = (g & 1) ? bc - 1 - bi : bi;
    return g + (off < tr - g * bc ? 1 : 0);
}

struct TraceParams {
    const MfxNode* nodes;
    const MfxSlot* slots;
    const int32_t* slot_ref;
    const uint8_t* ref_blob;
    const MfxShade* shade;
    const MfxInstance* inst;         // two-level scenes (null for a flat scene)
    double* accum;                   // [3][w*h] FP64 radiance sums, x-major pixels
    unsigned long long* work_counter;
    unsigned long long* counters;    // [8] ray / traversal counters
    MfxLight light;                  // by value: kernel arguments are scalar-loaded, never per-lane gathers
    MfxCamera cam;
    uint64_t seed;
    int64_t sample_base;             // first global sample index of this call
    int64_t nsamples;                // samples this context renders per pixel in this call
    int32_t part_index, part_count;  // global sample = sample_base + part_index + s * part_count
    int32_t band_index, band_count, band_rows;  // image partition: tile rows band_tile_row(band_index, band_count, k)
    int32_t width, height, max_depth;
    int32_t stack_size;              // LDS traversal stack entries per lane
    int32_t chunk;                   // path indices a wave takes per atomic
    double* vscratch;                // [max_depth + 1][6][grid * 256] per-lane vertex records (a_v, c_v)
    int32_t waves;                   // the kernel instance: 4 (128-VGPR budget) or 1 (unbounded)
};

struct QueryParams {
    const MfxNode* nodes;
    const MfxSlot* slots;
    const int32_t* slot_ref;
    const uint8_t* ref_blob;
    const MfxShade* shade;
    const MfxInstance* inst;
    const double* rays;
    const double* tmax_per_ray;
    double* t_out;
    int32_t* prim_out;
    double* normal_out;
    int32_t* occ_out;
    int64_t n;
    double tmin, tmax;
    int32_t stack_size;
};

hipError_t mfx_launch_trace(const TraceParams& P, bool stats, int grid, hipStream_t st);
hipError_t mfx_trace_occupancy(int stack_size, int* blocks_per_cu, bool inst = false, int waves = 1);
hipError_t mfx_launch_query(const QueryParams& Q, bool shadow, hipStream_t st);
hipError_t mfx_launch_mean(const double* accum, int64_t npix, double n, double* out, hipStream_t st, int64_t p0 = 0,
                           int64_t p1 = -1);
// pixels [p0, p1) of the mean as interleaved RGB (3 doubles a pixel): mfx_sample's staged readback
hipError_t mfx_launch_mean_rgb(const double* accum, int64_t npix, double n, double* out, hipStream_t st, int64_t p0,
                               int64_t p1);
hipError_t mfx_launch_film_post(const double* accum, double* film, int w, int h, double spp, double frame_count,
                                int add, uint8_t* rgba, hipStream_t st);
hipError_t mfx_launch_film_mean(const double* film, int64_t npix, double frame_count, double* out, hipStream_t st);
hipError_t mfx_launch_accum_add(double* dst, const double* src, int64_t n, hipStream_t st);
hipError_t mfx_launch_counters_add(unsigned long long* total, const unsigned long long* c, int n, hipStream_t st);
hipError_t mfx_launch_fp64_selftest(const double* a, const double* b, int64_t n, double* dvo, double* sqo,
                                    hipStream_t st);
hipError_t mfx_launch_aabb_selftest(const double* rec, int64_t n, int32_t* out, hipStream_t st);

#endif
