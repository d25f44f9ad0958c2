// mfx_layout.h — HBM data layout shared by the host builder (mfx_scene.cpp) and the gfx950
// kernels. See DESIGN.md §2 for the layout rationale.
//
//   nodes[]     BVH4 over the individual primitives (binned-SAH BVH2, leaves of <= 4 primitives,
//               collapsed to 4-wide), 128 B per internal node with all child boxes stored in the
//               parent (one node fetch = four FP32 slab tests). child >= 0 is an internal node
//               index; child < 0 is ~(16-byte offset of a leaf record in blob[]). Boxes are the primitives' FP64
//               boxes widened by eps and rounded outward (conservative: every primitive whose
//               reference leaf the F#'s FP64 slab test accepts is reached).
//   slots[]     traversal leaves in DFS order, each a run of 128-B FP64 MfxSlot records (Triangle 1
//               slot, Rect 2, Sphere 1). Every slot carries its reference leaf's FP64 box, `first`
//               and its position in it, which is all the exact semantics need
//               (mfx_trace_common.h: leaf_hit); slot_ref[] names the reference leaf record for
//               the rare whole-leaf evaluation.
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

// Diagnostic-only kernel options (timing stamps, occlusion statistics, the stage-removal timing
// builds of scripts/diag_variant.py) exist only in a build with -DMFX_DIAG; the shipped library
// has none of them.
#if !defined(MFX_DIAG) && (defined(MFX_DIAG_STAMPS) || defined(MFX_DIAG_OCCLUSION) || \
                           defined(MFX_DIAG_SKIP_SHADOW_TRAV) || defined(MFX_DIAG_ONE_TRIAL))
#error "MFX_DIAG_* options need a -DMFX_DIAG build"
#endif

struct alignas(16) MfxNode {  // BVH4 node: four child boxes, 128 B (one cache line)
    float lox[4], hix[4], loy[4], hiy[4], loz[4], hiz[4];
    int32_t child[4];  // >= 0 node index, < 0 ~(leaf code), MFX_CHILD_EMPTY (box lo = hi = FLT_MAX: never hit)
    int32_t pad[4];
};
#define MFX_CHILD_EMPTY (-0x7fffffff - 1)

// The per-lane kernels' (k_extend, k_shadow) BVH4 nodes with the FP32 planes rounded outward to FP16
// (IEEE binary16 bits), 64 B a node: four 16-B loads instead of seven, two nodes a cache line; an
// empty child's planes are all +inf. k_camera's packets and the megakernel keep the FP32 nodes.
// Round 6 A/B (profiles/r06/r06v_ab_fp16_nodes.txt): C2 +1.4 %, Renault +2.6 %; -DMFX_NODE_F16=0 builds
// the FP32-only library.
#ifndef MFX_NODE_F16
#define MFX_NODE_F16 1
#endif
struct alignas(16) MfxNodeH {
    uint16_t lox[4], hix[4], loy[4], hiy[4], loz[4], hiz[4];
    int32_t child[4];
};

// nodes[0 .. MFX_TOP_NODES) are the BVH's top levels in breadth-first order (the trace kernels
// keep a prefix of them in LDS); the rest follow in preorder
#ifndef MFX_TOP_NODES
#define MFX_TOP_NODES 128
#endif

// reference leaf header (ref_blob[]); copies of its primitives' slots follow
struct alignas(16) MfxLeaf {
    double lo[3];
    double hi[3];
    int32_t count;  // primitives in this reference leaf, 1..3
    int32_t kinds;  // 2 bits per primitive, in the reference's `indices` order
    int32_t first;  // position of the leaf in `indices` (heap order of leaves = ascending first)
    int32_t pad;
};

// MfxSlot.info: shade[] index | position in its reference leaf | kind | second triangle of a rect
#define MFX_INFO_SHADE_MASK 0x03ffffff
#define MFX_INFO_POS_SHIFT 26
#define MFX_INFO_KIND_SHIFT 28
#define MFX_INFO_RECT2 (1 << 30)

// One traversal slot, 128 B (one cache line): the geometry the exact FP64 test reads, then what a
// winning candidate needs — its reference leaf's FP64 box and `first` — so a leaf visit is one
// round of independent loads. A leaf is a run of consecutive slots; the node's child code says
// where it starts and how many slots it has.
struct alignas(16) MfxSlot {
    double a[3];    // tri: v0      sphere: center
    double b[3];    // tri: e1      sphere: {radius, 0, 0}
    double c[3];    // tri: e2
    int32_t first;  // MfxLeaf.first of the primitive's reference leaf
    int32_t info;   // MFX_INFO_* fields        (bytes 0..79: five 16-B loads per test)
    double lo[3];   // FP64 box of that reference leaf (InitNode, BvhNode.fs:32-37)
    double hi[3];
};

// leaf child code: ~((first slot << 3) | (slots - 1)), at most 8 slots (4 primitives, rects take 2)
#define MFX_LEAF_SLOTS_MAX 8
#define MFX_SLOTS_MAX (1 << 27)  // leaf codes stay below MFX_INST_FLAG

struct alignas(16) MfxShade {
    double n[3];        // face normal of this triangle slot; a sphere's centre
    double albedo[3];   // MaterialManager[material] flattened to its Lambert albedo (Material.fs:52-68)
    int32_t material;   // MaterialManager slot
    int32_t prim_kind;  // original primitive index (mfx_prim order) << 2 | MFX_KIND_*
};

// ---- two-level scenes (mfx_create_instanced) ----------------------------------------------------
// The top-level BVH (nodes[0..)) holds the loose primitives' leaves and, as leaf children, the
// instances: child = ~(MFX_INST_FLAG | instance). Entering one records the traversal stack depth,
// moves the ray's FP32 origin into the template's frame (o - off) and continues at the template
// BVH's root, whose boxes are the template primitives' (local coordinates); a pop below the
// recorded depth returns to the world frame. The template BVH is shared; its leaf codes count slots
// from the instance's own run of world slots (slot_base), which hold the world primitives exactly
// as a flat image does (FP64 geometry of the expansion, reference-leaf box, `first`, info), so a
// template leaf is tested by the same exact leaf test at a per-instance slot base.
#define MFX_INST_FLAG (1 << 30)                 // leaf codes stay below it (first slot < 2^27)
#define MFX_INST_MAX 0x3ffffffe

struct alignas(16) MfxInstance {
    double off[3];      // world = template + off, one FP64 rounding per coordinate
    int32_t root;       // its template BVH's root node
    int32_t slot_base;  // slots[] index of the instance's run of world slots
    int32_t pad[2];
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
