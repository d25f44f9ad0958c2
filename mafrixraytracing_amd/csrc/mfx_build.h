// mfx_build.h — the traversal BVH built on the GPU (mfx_build.hip).
#ifndef MFX_BUILD_H
#define MFX_BUILD_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "mfx_layout.h"

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

// The whole traversal image of a flat scene on the GPU: the BVH2 above, its BVH4 collapse and the
// layout (nodes renumbered, traversal leaves' slots in depth-first order) — the bytes the host
// path (mfx_scene.cpp: Collapse4 + layout) produces. Per primitive p the caller gives its slots
// pslots[slot_of[p] .. slot_of[p + 1]) with the reference-leaf box, `first` and the info bits
// other than the shade index already set, their shade records and the reference leaf's ref_blob
// offset.
struct MfxGpuLayoutIn {
    const MfxSlot* pslots;
    const MfxShade* pshade;
    const int32_t* slot_of;   // [n + 1]
    const int32_t* ref16_of;  // [n]
    int32_t nslots;
    int32_t top_nodes;        // nodes numbered breadth-first first (MFX_TOP_NODES), the rest in preorder
};
struct MfxGpuImages {
    std::vector<MfxNode> nodes;
    std::vector<MfxSlot> slots;       // + MFX_LEAF_SLOTS_MAX zero records
    std::vector<int32_t> slot_ref;
    std::vector<MfxShade> shade;
    std::vector<int32_t> shade_of;    // [n] shade index (= slot) of each primitive's first slot
    int32_t max_depth = 0, max_stack = 0, nodes2 = 0, nleaves = 0, levels = 0;
};
hipError_t mfx_gpu_build_images(const float* prim_box, const float* cent, const int32_t* weight, int n, int max_leaf,
                                float c_isect, const MfxGpuLayoutIn& in, MfxGpuImages& out);

#endif
