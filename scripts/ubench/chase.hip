// Micro-benchmark: dependent pointer chase through a table of 128-B nodes, NL 16-B loads per
// step (all from the same node), like one BVH node step; reports cycles per step per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int NL>
__global__ void __launch_bounds__(256) chase(const uint4* __restrict__ tab, uint32_t mask, int steps, uint32_t* out,
                                             unsigned long long* cyc) {
    uint32_t node = (blockIdx.x * 256 + threadIdx.x) * 2654435761u & mask;
    uint32_t acc = 0;
    const unsigned long long t0 = clock64();
    for (int s = 0; s < steps; ++s) {
        const uint4* q = tab + (size_t)node * 8;
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            const uint4 v = q[k];
            x += v.x ^ v.y ^ v.z ^ v.w;
        }
        node = (node * 1664525u + 1013904223u + x) & mask;  // next node depends on this node's data
        acc += x;
    }
    const unsigned long long t1 = clock64();
    if (acc == 0x12345678u) out[0] = acc;
    if ((threadIdx.x & 63) == 0) atomicAdd(cyc, t1 - t0);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t maxnodes = 1 << 20;  // 128 MB of nodes
    uint4* tab;
    uint32_t* out;
    unsigned long long* cyc;
    hipMalloc(&tab, maxnodes * 128);
    hipMalloc(&out, 64);
    hipMalloc(&cyc, 8);
    hipMemset(tab, 0, maxnodes * 128);
    const int steps = 2000;
    printf("%10s %4s %8s %14s\n", "table_KB", "NL", "waves/CU", "cycles/step");
    for (size_t nodes : {(size_t)256, (size_t)1 << 11, (size_t)1 << 14, (size_t)1 << 20})
        for (int bpc : {1, 3})
            for (int nl : {1, 4, 7}) {
                const uint32_t mask = (uint32_t)(nodes - 1);
                const int blocks = cus * bpc;
                hipMemset(cyc, 0, 8);
                if (nl == 1) hipLaunchKernelGGL((chase<1>), dim3(blocks), dim3(256), 0, 0, tab, mask, steps, out, cyc);
                else if (nl == 4) hipLaunchKernelGGL((chase<4>), dim3(blocks), dim3(256), 0, 0, tab, mask, steps, out, cyc);
                else hipLaunchKernelGGL((chase<7>), dim3(blocks), dim3(256), 0, 0, tab, mask, steps, out, cyc);
                if (hipDeviceSynchronize() != hipSuccess) { printf("error\n"); return 1; }
                unsigned long long c = 0;
                hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
                printf("%10zu %4d %8d %14.1f\n", nodes * 128 / 1024, nl, bpc * 4, (double)c / (blocks * 4) / steps);
            }
    return 0;
}
