// mfx_wide.h — the per-lane traversal's BVH8 image (MfxNode8H, mfx_layout.h), derived on the host
// from a flat scene's BVH4 image when a context is created.
#ifndef MFX_WIDE_H
#define MFX_WIDE_H

#include <string>
#include <vector>

#include "mfx_layout.h"

struct MfxWideImage {
    std::vector<MfxNode8H> nodes;  // [0] is the root; the first MFX_TOP_NODES breadth-first, the rest in preorder
    int32_t stack_entries = 1;     // traversal stack bound of node_step over this image
    MfxWideXf xf{0, 0, 0, 1};      // the frame the planes are stored in
    int32_t depth = 0;             // longest root-to-leaf path in wide nodes
};

// BVH4 (root 0, flat scene: no instance codes) -> BVH8. False with `err` set on a malformed image.
bool mfx_build_wide(const std::vector<MfxNode>& n4, MfxWideImage& out, std::string& err);

// The image's invariants against the BVH4 it came from (every leaf once; boxes contain their
// subtrees); false with `err` set otherwise.
bool mfx_check_wide(const std::vector<MfxNode>& n4, const MfxWideImage& w, std::string& err, double* mean_entries,
                    int64_t* nleaves);

// FP16 bits of the largest half <= v (up = false) or the smallest half >= v (up = true); +-inf
// outside the finite range.
uint16_t mfx_half_round(double v, bool up);
double mfx_half_value(uint16_t h);

#endif
