// mfx_trace_common.h — device code shared by the megakernel (mfx_kernels.hip) and the wavefront
// pipeline (mfx_wavefront.hip): FP64 vector helpers, the counter RNG, the exact FP64 leaf-level
// tests and the FP32 cluster-BVH traversal.
//
// Compiled with -ffp-contract=off: every FP64 expression follows the reference F#'s operation
// order (cited per function) with one rounding per operation, so the device makes the same
// discrete decisions (hit / miss / which primitive / rejection accept) as the CPU oracle.
// FP32 work (the BVH2 slab tests that only *find* candidate clusters) uses explicit fmaf.
#ifndef MFX_TRACE_COMMON_H
#define MFX_TRACE_COMMON_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mfx_layout.h"

// ----------------------------------------------------------------------------------------------
// FP64 value helpers — Point.fs:35-68 (same order as the host code and the oracle)
// ----------------------------------------------------------------------------------------------
struct DV {
    double x, y, z;
};
__device__ __forceinline__ DV dv(double x, double y, double z) { return DV{x, y, z}; }
__device__ __forceinline__ DV ld3(const double* p) { return DV{p[0], p[1], p[2]}; }
__device__ __forceinline__ DV vsub(DV a, DV b) { return dv(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ DV vadd(DV a, DV b) { return dv(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ DV vmul(DV v, double a) { return dv(v.x * a, v.y * a, v.z * a); }
__device__ __forceinline__ DV vdiv(DV v, double a) { return dv(v.x / a, v.y / a, v.z / a); }
__device__ __forceinline__ double vdot(DV a, DV b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ DV vcross(DV a, DV v) {
    return dv(a.y * v.z - a.z * v.y, a.z * v.x - a.x * v.z, a.x * v.y - a.y * v.x);
}
__device__ __forceinline__ double vlen(DV v) { return sqrt(v.x * v.x + v.y * v.y + v.z * v.z); }
__device__ __forceinline__ DV vnormalize(DV v) {
    double l = vlen(v);
    if (l == 0.0) return dv(0, 0, 0);
    return dv(v.x / l, v.y / l, v.z / l);
}

// ----------------------------------------------------------------------------------------------
// Counter-based RNG — identical to oracle/mfx_oracle.c rng_*
// ----------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z ^= z >> 30;
    z *= 0xbf58476d1ce4e5b9ULL;
    z ^= z >> 27;
    z *= 0x94d049bb133111ebULL;
    z ^= z >> 31;
    return z;
}
__device__ __forceinline__ uint64_t path_key(uint64_t seed, uint64_t pixel, uint64_t sample) {
    return mix64(seed ^ mix64((pixel << 32) | (sample & 0xffffffffULL)));
}
__device__ __forceinline__ double rng_next(uint64_t key, uint32_t& n) {
    n += 1;
    uint64_t z = mix64(key + (uint64_t)n * 0x9e3779b97f4a7c15ULL);
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

// ----------------------------------------------------------------------------------------------
// Exact FP64 leaf-level tests
// ----------------------------------------------------------------------------------------------
// AABB.hit — IHitable.fs:18-54
__device__ __forceinline__ bool aabb_hit64(const double* lo, const double* hi, DV o, DV d, double tMin, double tMax) {
    double tmin, tmax, tymin, tymax, tzmin, tzmax;
    if (d.x >= 0.) { tmin = (lo[0] - o.x) / d.x; tmax = (hi[0] - o.x) / d.x; }
    else { tmin = (hi[0] - o.x) / d.x; tmax = (lo[0] - o.x) / d.x; }
    if (d.y >= 0.) { tymin = (lo[1] - o.y) / d.y; tymax = (hi[1] - o.y) / d.y; }
    else { tymin = (hi[1] - o.y) / d.y; tymax = (lo[1] - o.y) / d.y; }
    if (tmin > tymax || tymin > tmax) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    if (d.z >= 0.) { tzmin = (lo[2] - o.z) / d.z; tzmax = (hi[2] - o.z) / d.z; }
    else { tzmin = (hi[2] - o.z) / d.z; tzmax = (lo[2] - o.z) / d.z; }
    if (tmin > tzmax || tzmin > tmax) return false;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    return tmin < tMax && tmax > tMin;
}

// Triangle.PreCalcu + Hit — Trangle.fs:120-155 (tMax deliberately not checked, :148)
__device__ __forceinline__ bool tri_hit64(const MfxSlot& s, DV o, DV d, double tMin, double& t) {
    DV e1 = ld3(s.b), e2 = ld3(s.c);
    DV s1 = vcross(d, e2);
    double divisor = vdot(s1, e1);
    if (fabs(divisor) < 1e-6) return false;
    double inv = 1. / divisor;
    DV dd = vsub(o, ld3(s.a));
    double b1 = vdot(dd, s1) * inv;
    if (b1 < 0. || b1 > 1.) return false;
    DV s2 = vcross(dd, e1);
    double b2 = vdot(d, s2) * inv;
    if (b2 < 0. || (b1 + b2) >= 1.) return false;
    t = vdot(e2, s2) * inv;
    return t > tMin;
}

// Sphere.Hit — Sphere.fs:21-43
__device__ __forceinline__ bool sphere_hit64(const MfxSlot& s, DV o, DV d, double tMin, double tMax, double& t) {
    DV oc = vsub(o, ld3(s.a));
    double a = 1.;
    double b = 2.0 * vdot(oc, d);
    double c = vdot(oc, oc) - s.b[0] * s.b[0];
    double disc = b * b - 4.0 * a * c;
    if (disc > 0) {
        double rd = sqrt(disc);
        double q = (b < 0.) ? -0.5 * (b - rd) : -0.5 * (b + rd);
        double t0 = q, t1 = c / q;
        double tmn = t0 < t1 ? t0 : t1, tmx = t0 > t1 ? t0 : t1;
        if (tmn >= tMin && tmn < tMax) { t = tmn; return true; }
        if (tmx > tMin && tmx < tMax) { t = tmx; return true; }
    }
    return false;
}

struct SceneView {
    const MfxNode* __restrict__ nodes;
    const uint8_t* __restrict__ blob;  // MfxLeaf + inline MfxSlot records
    int32_t root_is_leaf;
};

struct Stats {
    uint32_t nodes, clusters, prims;
};

// One reference leaf: exact FP64 box test, then Array.minBy over its primitives with key
// (hit ? t : tMax), first minimum wins (BvhNode.fs:76-80). Returns whether the leaf's result is
// a hit; t and the shade[] index of the hit slot. The header and the slots are contiguous.
//
// The leaf's result is (box hit) && (minBy result is a hit); neither test has side effects, so
// the primitives run first and the FP64 box test (six divisions) only when it can still change
// the answer: the minBy result is a hit and, for closest queries, its t does not exceed the best
// hit so far (`reject_above`; a larger t can never be accepted by the caller's tie rule). SHADOW
// queries stop at the first primitive hit with t < tMax: its key is below every miss's key
// (tMax), so the minBy result is a hit whatever follows. A hit beyond tMax (Triangle.Hit ignores
// tMax, Trangle.fs:148) does not stop the scan — a later miss can still win the minBy.
template <bool SHADOW, bool STATS>
__device__ __forceinline__ bool cluster_hit(const SceneView& S, int off16, DV o, DV d, double tMin, double tMax,
                                            double reject_above, double& t_out, int& slot_out, int& first_out,
                                            Stats& st) {
    const MfxLeaf* __restrict__ lf = (const MfxLeaf*)(S.blob + (size_t)off16 * 16);
    const MfxSlot* __restrict__ sl = (const MfxSlot*)(lf + 1);
    // only the 16-B tail (count, kinds, first, shade_base) now; the box is read (L1/L2 hit)
    // after the primitives, when needed — keeping six doubles live costs occupancy
    struct Meta {
        int32_t count, kinds, first, shade_base;
    };
    const Meta c = *(const Meta*)((const uint8_t*)lf + offsetof(MfxLeaf, count));
    if (STATS) st.clusters++;
    bool best_hit = false;
    double best_key = 0.0, best_t = 0.0;
    int best_slot = -1;
    int cur = 0;
    for (int k = 0; k < c.count; ++k) {
        const int kind = (c.kinds >> (2 * k)) & 3;
        if (STATS) st.prims++;
        double t = 0.0;
        int hs = cur;
        bool h;
        if (kind == MFX_KIND_SPHERE) {
            h = sphere_hit64(sl[cur], o, d, tMin, tMax, t);
            cur += 1;
        } else {
            h = tri_hit64(sl[cur], o, d, tMin, t);
            if (kind == MFX_KIND_RECT) {
                if (!h) {  // Rect.Hit: trig1, else trig2 (Rect.fs:26-31)
                    hs = cur + 1;
                    h = tri_hit64(sl[cur + 1], o, d, tMin, t);
                }
                cur += 2;
            } else {
                cur += 1;
            }
        }
        const double key = h ? t : tMax;
        if (k == 0 || key < best_key) {
            best_key = key;
            best_hit = h;
            best_t = t;
            best_slot = hs;
        }
        if (SHADOW && h && t < tMax) break;
    }
    if (!best_hit || best_t > reject_above) return false;
    if (!aabb_hit64(lf->lo, lf->hi, o, d, tMin, tMax)) return false;
    t_out = best_t;
    slot_out = c.shade_base + best_slot;
    first_out = c.first;
    return true;
}

__device__ __forceinline__ float f_round_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = nextafterf(f, __builtin_inff());
    return f;
}

// FP32 ray for the cluster-BVH slab tests
struct RayF {
    float ix, iy, iz, oix, oiy, oiz;
};
__device__ __forceinline__ RayF make_rayf(DV o, DV d) {
    // tiny direction components clamped so 1/d stays finite (no 0*inf NaNs)
    float dx = (float)d.x, dy = (float)d.y, dz = (float)d.z;
    const float tiny = 1e-20f;
    if (fabsf(dx) < tiny) dx = copysignf(tiny, dx);
    if (fabsf(dy) < tiny) dy = copysignf(tiny, dy);
    if (fabsf(dz) < tiny) dz = copysignf(tiny, dz);
    RayF r;
    r.ix = 1.0f / dx; r.iy = 1.0f / dy; r.iz = 1.0f / dz;
    r.oix = (float)o.x * r.ix; r.oiy = (float)o.y * r.iy; r.oiz = (float)o.z * r.iz;
    return r;
}

#define MFX_TRAV_EXIT (-0x7fffffff - 1)  // node value: traversal finished (stack empty, no hit child)

// One internal-node step of the cluster BVH2, branch-free: both child slab tests, then
// near-first descent / push of the far child / pop, chosen with selects. The far child is
// written to the stack slot unconditionally and sp only advances when both children are hit;
// the pop candidate (top of stack) is read before the node's boxes arrive, so the LDS read
// overlaps the HBM/L2 load. Returns the next node: >= 0 internal, < 0 a leaf (~offset), or
// MFX_TRAV_EXIT when nothing is left.
__device__ __forceinline__ int node_step(const MfxNode* __restrict__ nodes, int node, const RayF& r, float tlim,
                                         int* __restrict__ stack, int& sp) {
    const int top = stack[(sp > 0 ? sp - 1 : 0) * 64];
    const MfxNode nd = nodes[node];
    float a0 = fmaf(nd.c0lox, r.ix, -r.oix), a1 = fmaf(nd.c0hix, r.ix, -r.oix);
    float b0 = fmaf(nd.c0loy, r.iy, -r.oiy), b1 = fmaf(nd.c0hiy, r.iy, -r.oiy);
    float c0 = fmaf(nd.c0loz, r.iz, -r.oiz), c1 = fmaf(nd.c0hiz, r.iz, -r.oiz);
    const float n0 = fmaxf(fmaxf(fminf(a0, a1), fminf(b0, b1)), fmaxf(fminf(c0, c1), 0.0f));
    const float f0 = fminf(fminf(fmaxf(a0, a1), fmaxf(b0, b1)), fminf(fmaxf(c0, c1), tlim));
    a0 = fmaf(nd.c1lox, r.ix, -r.oix); a1 = fmaf(nd.c1hix, r.ix, -r.oix);
    b0 = fmaf(nd.c1loy, r.iy, -r.oiy); b1 = fmaf(nd.c1hiy, r.iy, -r.oiy);
    c0 = fmaf(nd.c1loz, r.iz, -r.oiz); c1 = fmaf(nd.c1hiz, r.iz, -r.oiz);
    const float n1 = fmaxf(fmaxf(fminf(a0, a1), fminf(b0, b1)), fmaxf(fminf(c0, c1), 0.0f));
    const float f1 = fminf(fminf(fmaxf(a0, a1), fmaxf(b0, b1)), fminf(fmaxf(c0, c1), tlim));
    const bool h0 = n0 <= f0, h1 = n1 <= f1;
    const bool both = h0 && h1;
    const bool take1 = h1 && (!h0 || n1 < n0);  // child 1 is the one to descend into
    const int near = take1 ? nd.child1 : nd.child0;
    const int far = take1 ? nd.child0 : nd.child1;
    stack[sp * 64] = far;  // kept only if sp advances
    const bool any = h0 || h1;
    const bool pop = !any && sp > 0;
    sp += (both ? 1 : 0) - (pop ? 1 : 0);
    return any ? near : (pop ? top : MFX_TRAV_EXIT);
}

// Bvh.Hit over the cluster BVH2. SHADOW: returns occluded (any leaf reporting a hit; the
// reference's combine returns a hit iff some visited leaf does). Otherwise: closest leaf hit,
// ties going to the later leaf (the reference's `if l.t < r.t then l else r`, BvhNode.fs:70).
// The stack lives in LDS, one column per lane (stride 64 dwords: conflict-free).
template <bool SHADOW, bool STATS>
__device__ bool traverse(const SceneView& S, DV o, DV d, double tMin, double tMax, int* __restrict__ stack,
                         double& t_best, int& slot_best, Stats& st) {
    t_best = tMax;
    slot_best = -1;
    int first_best = -1;
    bool found = false;
    if (S.root_is_leaf) {
        double t;
        int s, f;
        if (cluster_hit<SHADOW, STATS>(S, 0, o, d, tMin, tMax, __builtin_inf(), t, s, f, st)) {
            t_best = t;
            slot_best = s;
            return true;
        }
        return false;
    }
    const RayF rf = make_rayf(o, d);
    float tlim = f_round_up(tMax);
    int sp = 0;
    int node = 0;
    while (true) {
        // ---- internal nodes ----
        while (node >= 0) {
            if (STATS) st.nodes++;
            node = node_step(S.nodes, node, rf, tlim, stack, sp);
        }
        if (node == MFX_TRAV_EXIT) return found;
        // ---- leaf: one reference leaf (cluster) ----
        {
            double t;
            int s, f;
            if (cluster_hit<SHADOW, STATS>(S, ~node, o, d, tMin, tMax, found ? t_best : __builtin_inf(), t, s, f,
                                           st)) {
                if (SHADOW) {
                    t_best = t;
                    slot_best = s;
                    return true;
                }
                if (!found || t < t_best || (t == t_best && f > first_best)) {
                    found = true;
                    t_best = t;
                    slot_best = s;
                    first_best = f;
                    tlim = f_round_up(t);
                }
            }
        }
        if (sp == 0) return found;
        node = stack[(--sp) * 64];
    }
}

static constexpr double INVPI = 1. / 3.141592653589793;  // Material.fs:26
static constexpr double TWOPI = 2. * 3.141592653589793;  // Material.fs:27

#endif
