// mfx_build.h — the traversal BVH built on the GPU (mfx_build.hip).
#ifndef MFX_BUILD_H
#define MFX_BUILD_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

// A binned-SAH BVH2 over primitives, as mfx_scene.cpp's host SahBuilder produces it: internal
// node i has two children (>= 0 internal node, < 0 ~leaf) and their FP32 boxes; leaf l is the
// range [leaf_b[l], leaf_e[l]) of the primitive permutation `ids`. Node and leaf numbering is the
// build's own; everything downstream follows child references only.
struct MfxBvh2 {
    std::vector<float> box;       // [nodes][2][6]: child box lo xyz, hi xyz
    std::vector<int32_t> child;   // [nodes][2]
    std::vector<int32_t> leaf_b, leaf_e;
    std::vector<int32_t> ids;     // primitive permutation
    int32_t root = 0;             // 0 (internal) or ~0 (the whole scene is one leaf)
    float root_box[6] = {0, 0, 0, 0, 0, 0};
    int32_t levels = 0;           // breadth-first levels (kernel launches)
};

// Build on the current HIP device. prim_box: [n][6] conservative FP32 boxes (lo xyz, hi xyz);
// cent: [n][3] centroids; weight: [n] slots per primitive (the intersection cost weight).
// Same parameters as SahBuilder: leaves of at most max_leaf primitives, intersection cost c_isect.
hipError_t mfx_gpu_sah_build(const float* prim_box, const float* cent, const int32_t* weight, int n, int max_leaf,
                             float c_isect, MfxBvh2& out);

#endif
