// Micro-benchmark: throughput of scattered per-lane gathers on gfx950 (how the vector memory
// path prices divergent, uncoalesced loads such as BVH node fetches). Each lane performs ITERS
// rounds of ILP independent loads of W bytes at hashed addresses in a table of TB bytes; only
// the first ACT lanes of each wave are active; GROUP consecutive lanes share one 64-B line.
// Prints wave-instructions and lane-accesses per CU-cycle.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

template <int W>
struct Vec;
template <> struct Vec<4> { using T = uint32_t; };
template <> struct Vec<8> { using T = uint2; };
template <> struct Vec<16> { using T = uint4; };
__device__ __forceinline__ uint32_t fold(uint32_t v) { return v; }
__device__ __forceinline__ uint32_t fold(uint2 v) { return v.x ^ v.y; }
__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

template <int W, int ILP>
__global__ void __launch_bounds__(256) gather(const uint8_t* __restrict__ tab, uint32_t lines_mask, int iters,
                                              int act, int group, uint32_t* out, uint32_t far_mask,
                                              uint32_t far_thresh) {
    using T = typename Vec<W>::T;
    const int lane = threadIdx.x & 63;
    if (lane >= act) return;
    uint32_t h = (blockIdx.x * 256 + threadIdx.x / group) * 0x9e3779b1u + 12345u;
    uint32_t acc = 0;
    const int sub = (lane % group) * W;  // position inside the shared 64-B line
    for (int it = 0; it < iters; ++it) {
        T v[ILP];
#pragma unroll
        for (int k = 0; k < ILP; ++k) {
            h = h * 1664525u + 1013904223u + acc;  // depends on acc: rounds are serial, loads in a round are not
            // a fraction far_thresh / 2^16 of the accesses go to a large table (L1 misses)
            const uint32_t line = ((h >> 16) & 0xffffu) < far_thresh ? (((h >> 3) & far_mask) + (1u << 16)) : ((h >> 7) & lines_mask);
            v[k] = *(const T*)(tab + (size_t)line * 64 + (sub & 63));
        }
#pragma unroll
        for (int k = 0; k < ILP; ++k) acc += fold(v[k]);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int clk_khz = 0;
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    const size_t maxtab = 64u << 20;
    uint8_t* tab;
    uint32_t* out;
    hipMalloc(&tab, maxtab);
    hipMalloc(&out, 64);
    hipMemset(tab, 1, maxtab);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = cus * 8;  // 8 blocks of 4 waves per CU = 8 waves / SIMD
    const int iters = 256;
    printf("cus %d clock %.0f MHz\n", cus, clk_khz / 1e3);
    // `td_gather peak`: only the TD roof case — every lane of every wave a distinct 64-B line of an
    // L1-resident 16 KB table, 16-B loads, 4 independent loads per round — for a PMC pass whose
    // TCP_TOTAL_ACCESSES / GRBM_GUI_ACTIVE per dispatch is the peak the trace kernels are held to
    // (scripts/pmc_td_roof.sh)
    const bool peak_only = argc > 1 && std::string(argv[1]) == "peak";
    printf("%8s %5s %3s %3s %5s %3s %12s %14s %14s\n", "table", "far%", "W", "act", "group", "ilp", "ms", "winst/CUclk", "lanes/CUclk");
    const size_t tb = 16 << 10;
    for (double farp : {0.0, 0.01, 0.02, 0.05, 0.1, 0.2, 1.0})
        for (int w : {16})
            for (int act : {64, 22})
                if (!peak_only || (farp == 0.0 && act == 64))
                for (int group : {1}) {
                    const uint32_t far_mask = (1u << 14) - 1;  // 1 MB far table (L2-resident)
                    const uint32_t far_thresh = (uint32_t)(farp * 65536.0);
                    if ((size_t)((1u << 16) + far_mask + 1) * 64 > maxtab || tb > maxtab) { printf("bounds\n"); return 1; }
                    if (group * w > 64) continue;
                    const uint32_t mask = (uint32_t)(tb / 64 - 1);
                    auto run = [&]() {
                        if (w == 4) hipLaunchKernelGGL((gather<4, 4>), dim3(blocks), dim3(256), 0, 0, tab, mask, iters, act, group, out, far_mask, far_thresh);
                        if (w == 8) hipLaunchKernelGGL((gather<8, 4>), dim3(blocks), dim3(256), 0, 0, tab, mask, iters, act, group, out, far_mask, far_thresh);
                        if (w == 16) hipLaunchKernelGGL((gather<16, 4>), dim3(blocks), dim3(256), 0, 0, tab, mask, iters, act, group, out, far_mask, far_thresh);
                    };
                    run();
                    hipEventRecord(e0);
                    for (int r = 0; r < 5; ++r) run();
                    hipEventRecord(e1);
                    if (hipEventSynchronize(e1) != hipSuccess) { printf("error\n"); return 1; }
                    float ms = 0;
                    hipEventElapsedTime(&ms, e0, e1);
                    ms /= 5;
                    const double winst = (double)blocks * 4 * iters * 4;  // waves * iters * ILP
                    const double cuclk = ms * 1e-3 * clk_khz * 1e3 * cus;
                    printf("%8zu %5.1f %3d %3d %5d %3d %12.3f %14.4f %14.3f\n", tb, farp * 100, w, act, group, 4, ms, winst / cuclk, winst * act / cuclk);
                }
    return 0;
}
