// mfx_layout.h — HBM data layout shared by the host builder (mfx_scene.cpp) and the gfx950
// kernels. See DESIGN.md §2 for the layout rationale.
//
//   nodes[]     BVH2 over the individual primitives (binned SAH, leaves of <= 4 primitives),
//               64 B per internal node with both child boxes stored in the parent (one node
//               fetch = two FP32 slab tests). child >= 0 is an internal node index; child < 0 is
//               ~(16-byte offset of a leaf record in blob[]). Boxes are the primitives' FP64
//               boxes widened by eps and rounded outward (conservative: every primitive whose
//               reference leaf the F#'s FP64 slab test accepts is reached).
//   blob[]      traversal leaves in DFS order: a 16-B MfxTLeaf header, then the leaf's primitives'
//               FP64 MfxSlot records (Triangle 1 slot, Rect 2, Sphere 1). Every slot names its
//               reference leaf (`ref16`) and its position in it (`info`), which is all the exact
//               semantics need (mfx_trace_common.h: leaf_hit).
//   ref_blob[]  one record per leaf of the reference's heap BVH (BvhNode.fs:36-39, count <= 3): a
//               64-B MfxLeaf header (its exact FP64 box, InitNode BvhNode.fs:32-37; its position in
//               `indices`) followed by copies of its primitives' slots. Read for the FP64 leaf-box
//               test of a winning candidate and, rarely, to evaluate a whole reference leaf.
//   shade[]     per traversal slot: face normal (FP64, Trangle.fs:108-113) — a sphere's centre —,
//               material index, original primitive index and kind.
#ifndef MFX_LAYOUT_H
#define MFX_LAYOUT_H

#include <stdint.h>

#define MFX_KIND_TRI 0
#define MFX_KIND_RECT 1
#define MFX_KIND_SPHERE 2

struct alignas(16) MfxNode {
    float c0lox, c0hix, c0loy, c0hiy;  // child 0 box x,y
    float c1lox, c1hix, c1loy, c1hiy;  // child 1 box x,y
    float c0loz, c0hiz, c1loz, c1hiz;  // both z
    int32_t child0, child1, pad0, pad1;
};

// reference leaf header (ref_blob[]); copies of its primitives' slots follow
struct alignas(16) MfxLeaf {
    double lo[3];
    double hi[3];
    int32_t count;  // primitives in this reference leaf, 1..3
    int32_t kinds;  // 2 bits per primitive, in the reference's `indices` order
    int32_t first;  // position of the leaf in `indices` (heap order of leaves = ascending first)
    int32_t pad;
};

#define MFX_INFO_SHADE_MASK 0x0fffffff  // MfxSlot.info: shade[] index | position in its reference leaf << 28
#define MFX_INFO_POS_SHIFT 28

struct alignas(16) MfxSlot {
    double a[3];   // tri: v0      sphere: center
    double b[3];   // tri: e1      sphere: {radius, 0, 0}
    double c[3];   // tri: e2
    int32_t ref16;  // 16-byte offset of the primitive's reference leaf in ref_blob[]
    int32_t info;   // shade[] index of this slot | (position of the primitive in its reference leaf) << 28
};

// traversal leaf header (blob[]); the slots follow
struct alignas(16) MfxTLeaf {
    int32_t count;  // primitives, 1..4
    int32_t kinds;  // 2 bits per primitive
    int32_t pad0, pad1;
};

struct alignas(16) MfxShade {
    double n[3];        // face normal of this triangle slot; a sphere's centre
    int32_t material;   // MaterialManager slot
    int32_t prim_kind;  // original primitive index (mfx_prim order) << 2 | MFX_KIND_*
};

// Quad light = NewAreaLight (Light.fs:31-64): two sample triangles (v0, e1, e2), normal, color.
struct MfxLight {
    double v0[2][3], e1[2][3], e2[2][3];
    double normal[3];
    double color[3];
    double area;    // rect.Area() = trig1.area + trig2.area (Rect.fs:19)
    double pdf;     // 1. / rect.area (Light.fs:57-59)
};

// PinholeCamera after its constructor (Camera.fs:122-133), FP64.
struct MfxCamera {
    double position[3], topleft[3], right[3], down[3];
};

#endif
