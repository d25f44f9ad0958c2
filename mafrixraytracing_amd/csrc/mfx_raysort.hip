// mfx_raysort.hip — optional global reordering of the extension rays before a bounce's k_extend
// (MFX_RAY_SORT; an experiment, off by default: DESIGN.md §9 has the A/B).
//
// Bounce rays of a diffuse surface leave in all directions, so a wave of 64 neighbouring pixels'
// rays (the slot order of the pool) walks 64 unrelated BVH paths. Before k_extend of an iteration
// d >= 1, every NEED_EXT slot gets a 16-bit key — its origin's Morton cell (`obits` bits per axis,
// over the scene's bounds) above its direction bin (the octant, or one of 64 octahedral bins) —
// and the (key, slot) pairs of the whole pool are radix-sorted (stable: equal keys keep slot
// order); k_extend then takes its rays from the sorted slot list instead of scanning state words.
// Results do not depend on the order (each ray's closest hit is its own; k_resolve sums in sample
// order), so images stay bit-exact.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "mfx_wavefront.h"

__device__ __forceinline__ uint32_t spread3(uint32_t x) {  // bits of x at every third position
    x &= 0x3ffu;
    x = (x | (x << 16)) & 0x030000ffu;
    x = (x | (x << 8)) & 0x0300f00fu;
    x = (x | (x << 4)) & 0x030c30c3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}

// keys[j] = cell << dbits | direction bin for a NEED_EXT slot, 0xffff otherwise; vals[j] = j or -1
__global__ void __launch_bounds__(256) k_ray_keys(WfParams P, uint16_t* __restrict__ keys, int32_t* __restrict__ vals,
                                                  float3 lo, float3 scale, int obits, int dbits) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= P.pool) return;
    const int st = P.state[j];
    if ((st & WF_STATE_MASK) != WF_NEED_EXT) {
        keys[j] = 0xffff;
        vals[j] = -1;
        return;
    }
    uint32_t cell = 0;
    if (obits > 0) {
        const float m = (float)((1 << obits) - 1);
        const float fx = fminf(fmaxf(((float)P.ox[j] - lo.x) * scale.x, 0.f), m);
        const float fy = fminf(fmaxf(((float)P.oy[j] - lo.y) * scale.y, 0.f), m);
        const float fz = fminf(fmaxf(((float)P.oz[j] - lo.z) * scale.z, 0.f), m);
        cell = spread3((uint32_t)fx) | (spread3((uint32_t)fy) << 1) | (spread3((uint32_t)fz) << 2);
    }
    uint32_t dir;
    if (dbits == 3) {
        dir = (st >> WF_OCT_SHIFT) & 7;  // k_shadow's octant of the new direction
    } else {  // 64 octahedral bins
        const float dx = (float)P.dx[j], dy = (float)P.dy[j], dz = (float)P.dz[j];
        const float n = fabsf(dx) + fabsf(dy) + fabsf(dz);
        float u = dx / n, v = dy / n;
        if (dz < 0.f) {
            const float uu = (1.f - fabsf(v)) * (u < 0.f ? -1.f : 1.f);
            v = (1.f - fabsf(u)) * (v < 0.f ? -1.f : 1.f);
            u = uu;
        }
        const int bu = min(7, (int)((u + 1.f) * 4.f)), bv = min(7, (int)((v + 1.f) * 4.f));
        dir = (uint32_t)(bu * 8 + bv);
    }
    keys[j] = (uint16_t)((cell << dbits) | dir);
    vals[j] = (int32_t)j;
}

hipError_t mfx_raysort(const WfParams& P, const float lo[3], const float hi[3], int obits, int dbits, uint16_t* keys_in,
                       uint16_t* keys_out, int32_t* vals_in, int32_t* vals_out, void* tmp, size_t tmp_bytes,
                       hipStream_t st) {
    float3 l = make_float3(lo[0], lo[1], lo[2]), sc;
    const float cells = (float)(1 << obits);
    sc.x = cells / fmaxf(hi[0] - lo[0], 1e-20f);
    sc.y = cells / fmaxf(hi[1] - lo[1], 1e-20f);
    sc.z = cells / fmaxf(hi[2] - lo[2], 1e-20f);
    hipLaunchKernelGGL(k_ray_keys, dim3((unsigned)((P.pool + 255) / 256)), dim3(256), 0, st, P, keys_in, vals_in, l, sc,
                       obits, dbits);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int end_bit = 3 * obits + dbits + 1;  // + 1: the invalid key 0xffff sorts after every valid one
    return hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, (int)P.pool, 0,
                                              end_bit > 16 ? 16 : end_bit, st);
}

size_t mfx_raysort_tmp_bytes(int64_t n) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (uint16_t*)nullptr, (uint16_t*)nullptr,
                                             (int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, 16, (hipStream_t)0);
    return bytes;
}
