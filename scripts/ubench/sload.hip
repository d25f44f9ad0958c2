// Micro-benchmark: throughput of wave-uniform (scalar-cache) loads on gfx950 — how k_camera's packet
// traversal reads its nodes and slots (mfx_trace_common.h: packet_node_step, load_slot_u). Each wave
// runs ITERS rounds; a round reads ILP 128-B "nodes" (two 64-B scalar loads each) at wave-uniform
// hashed indices of a table of TB bytes, the next round's indices depending on the data. Prints
// scalar load instructions and bytes per CU-cycle; `peak` runs the case scripts/pmc_td_roof.sh
// profiles (SQ_INSTS_SMEM over GPU clocks) as the roof of k_camera.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

typedef int i16v __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(4))) const i16v cst16;

template <int ILP>
__global__ void __launch_bounds__(256) sgather(const int* __restrict__ tab, uint32_t nodes_mask, int iters, int* out) {
    uint32_t h = __builtin_amdgcn_readfirstlane((blockIdx.x * 4 + (threadIdx.x >> 6)) * 0x9e3779b1u + 777u);
    int acc = 0;
    for (int it = 0; it < iters; ++it) {
        i16v a[ILP], b[ILP];
#pragma unroll
        for (int k = 0; k < ILP; ++k) {
            h = h * 1664525u + 1013904223u + (uint32_t)acc;
            const uint32_t node = __builtin_amdgcn_readfirstlane((h >> 8) & nodes_mask);
            cst16* p = (cst16*)(tab + (size_t)node * 32);
            a[k] = p[0];
            b[k] = p[1];
        }
#pragma unroll
        for (int k = 0; k < ILP; ++k) {  // every dword used, as a node step uses its whole line
            const i16v x = a[k] ^ b[k];
            acc += x.s0 ^ x.s1 ^ x.s2 ^ x.s3 ^ x.s4 ^ x.s5 ^ x.s6 ^ x.s7 ^ x.s8 ^ x.s9 ^ x.sa ^ x.sb ^ x.sc ^ x.sd ^
                   x.se ^ x.sf;
        }
        acc = __builtin_amdgcn_readfirstlane(acc);
    }
    if (acc == 0x12345678 && threadIdx.x == 0) out[0] = acc;
}

template <int ILP>
static float run(const int* tab, uint32_t nodes, int blocks, int iters, int* out) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(sgather<ILP>, dim3(blocks), dim3(256), 0, 0, tab, nodes - 1, 2, out);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(sgather<ILP>, dim3(blocks), dim3(256), 0, 0, tab, nodes - 1, iters, out);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ms;
}

int main(int argc, char** argv) {
    const bool peak = argc > 1 && !strcmp(argv[1], "peak");
    int cus = 0, clk_khz = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    int *tab, *out;
    const size_t maxtab = 16u << 20;
    hipMalloc(&tab, maxtab);
    hipMalloc(&out, 64);
    hipMemset(tab, 1, maxtab);
    const int iters = 2000;
    // table sizes: 16 KB (scalar-cache resident), 256 KB (C2's BVH4 nodes), 4 MB (an XCD's L2)
    const uint32_t sizes[] = {16u << 10, 256u << 10, 4u << 20};
    for (uint32_t tb : sizes) {
        if (peak && tb != (256u << 10)) continue;
        const uint32_t nodes = tb / 128;
        for (int wpc : {16}) {  // waves per CU: 4 per SIMD, k_camera's occupancy
            const int blocks = cus * wpc / 4;
            const float ms = run<4>(tab, nodes, blocks, iters, out);
            const double insts = (double)blocks * 4 * iters * 4 * 2;  // waves x rounds x ILP x 2 loads
            const double cyc = ms * 1e-3 * clk_khz * 1e3;
            printf("table %7u B waves/CU %2d: %.3f ms, %.3f scalar loads per CU-cycle (%.1f B/CU-cycle) at the "
                   "nominal %d MHz\n", tb, wpc, ms, insts / cus / cyc, insts * 64 / cus / cyc, clk_khz / 1000);
        }
    }
    hipFree(tab);
    hipFree(out);
    return 0;
}
