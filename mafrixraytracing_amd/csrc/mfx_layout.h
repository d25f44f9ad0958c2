// mfx_layout.h — HBM data layout shared by the host builder (mfx_scene.cpp) and the gfx950
// kernels. See DESIGN.md §2 for the layout rationale.
//
//   nodes[]  BVH2 over the reference's leaves ("clusters"), 64 B per internal node, both child
//            boxes stored in the parent (one node fetch = two FP32 slab tests). child >= 0 is an
//            internal node index; child < 0 is ~(16-byte offset of a leaf record in blob[]).
//            Boxes are the clusters' FP64 boxes rounded outward and widened by eps (conservative:
//            every cluster the reference's FP64 slab test accepts is reached).
//   blob[]   one record per leaf of the reference's heap BVH (BvhNode.fs:36-39, count <= 3), laid
//            out in the traversal BVH's depth-first leaf order: a 64-B MfxLeaf header (its exact
//            FP64 box, InitNode BvhNode.fs:32-37) followed by its primitives' FP64 MfxSlot records
//            (a Triangle takes 1 slot, a Rect 2, a Sphere 1). A leaf is fetched in one round trip.
//   shade[]  per slot: face normal (FP64, Trangle.fs:108-113) — the centre for a sphere —,
//            material index, original primitive index and kind.
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

struct alignas(16) MfxLeaf {
    double lo[3];
    double hi[3];
    int32_t count;       // primitives in this reference leaf, 1..3
    int32_t kinds;       // 2 bits per primitive, in the reference's `indices` order
    int32_t first;       // position of the leaf in `indices` (heap order of leaves = ascending first)
    int32_t shade_base;  // shade[] index of the leaf's first slot
};

struct alignas(16) MfxSlot {
    double a[3];  // tri: v0      sphere: center
    double b[3];  // tri: e1      sphere: {radius, 0, 0}
    double c[3];  // tri: e2
    double pad;
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
