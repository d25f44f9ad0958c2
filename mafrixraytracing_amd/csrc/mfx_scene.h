// mfx_scene.h — host-side scene preparation (runs once per `Scene`, Scene.fs:298-313).
#ifndef MFX_SCENE_H
#define MFX_SCENE_H

#include <string>
#include <vector>

#include "../../include/mafrix_rt.h"
#include "mfx_layout.h"

struct MfxHostScene {
    // reference heap-BVH leaf grouping (BvhNode.fs:24-61)
    std::vector<int32_t> ref_indices;                  // `indices` after Subdivide
    std::vector<int32_t> leaf_first, leaf_count;       // leaves in heap (DFS) order
    // device images
    std::vector<MfxNode> nodes;     // BVH4 over primitives (preorder)
    std::vector<MfxSlot> slots;     // traversal leaves: runs of MfxSlot records, DFS order
    std::vector<int32_t> slot_ref;  // per slot: 16-byte offset of its reference leaf in ref_blob
    std::vector<uint8_t> ref_blob;  // reference leaves: MfxLeaf headers + slot copies, heap order
    std::vector<MfxShade> shade;    // per traversal slot, in slots[] order
    std::vector<MfxInstance> inst;  // two-level scenes: instances traced through a template BVH
    int32_t nclusters = 0;          // reference leaves
    int32_t ntleaves = 0;           // traversal leaves
    int32_t world_slots = 0;        // slots of the world primitives (what a flat image holds)
    int32_t tlas_nodes = 0, blas_nodes = 0, blas_slots = 0, ntemplates = 0, top_slots = 0;  // two-level shape (blas_slots: one run per template)
    std::vector<double> albedo;  // [nmat][3]
    MfxLight light;
    MfxCamera camera;
    int32_t width = 0, height = 0, max_depth = 3;
    int32_t bvh_depth = 0;     // longest root-to-leaf path in nodes[]
    int32_t stack_entries = 1; // traversal stack bound: pushes along any root-to-node path
    float eps = 0.f;           // conservative box widening
    // build record (mfx_build_info)
    bool bvh_gpu = false;      // traversal BVH2 built on the GPU (mfx_build.hip)
    bool images_gpu = false;   // and its BVH4 collapse and image layout too (flat scenes)
    int32_t bvh_levels = 0;    // its breadth-first levels (GPU) / depth + 1 (host)
    int32_t nodes2 = 0;        // its internal nodes
    double ms_ref_bvh = 0, ms_bvh = 0, ms_total = 0;
};

// Builds everything from the C-ABI scene description; returns false with `err` set on bad input.
// gpu_bvh: build the traversal BVH2 on the current HIP device (the same tree as the host build).
// instances (mfx_create_instanced): d->prims are templates, the world scene is their expansion;
// flatten: trace it through one flat BVH instead of two levels.
bool mfx_build_scene(const mfx_scene_desc* d, MfxHostScene& s, std::string& err, bool gpu_bvh = false,
                     const mfx_instance* instances = nullptr, int ninstances = 0, bool flatten = false);
// The world primitive list of an instanced scene (mfx_instance: template + offset, FP64).
bool mfx_expand(const mfx_prim* prims, int64_t nprims, const mfx_instance* inst, int ninst,
                std::vector<mfx_prim>& world, std::string& err);

#endif
