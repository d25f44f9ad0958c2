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
// draw n's 64 raw bits (rng_next = rng_unit(rng_bits))
__device__ __forceinline__ uint64_t rng_bits(uint64_t key, uint32_t& n) {
    n += 1;
    return mix64(key + (uint64_t)n * 0x9e3779b97f4a7c15ULL);
}
__device__ __forceinline__ double rng_unit(uint64_t z) { return (double)(z >> 11) * (1.0 / 9007199254740992.0); }
// the same draw truncated to 24 bits, as an FP32 value (|rng_unit(z) - rng_unit24(z)| < 2^-24)
__device__ __forceinline__ float rng_unit24(uint64_t z) { return (float)(uint32_t)(z >> 40) * 0x1p-24f; }

// GetRandomInUnitSphere(nm) (Material.fs:9-14): rejection from the unit ball until n.p > 0, with
// the reference's draw order (x, y, z per trial). Each trial is decided in FP32 when the FP32
// value lies at least 1e-5 from the decision boundary (|p.p - 1| and |n.p|: their FP32 error is
// below 1.3e-6 for |n| = 1 and draws truncated to 24 bits), otherwise in FP64 exactly as the
// oracle; the accepted point is formed in FP64 from the same draws. So the accepted trial, p and
// the draw count are exactly the FP64 loop's, at about 60 % of its cost per trial.
#ifndef MFX_HEMI_TRIALS
#define MFX_HEMI_TRIALS 2  // rejection trials per round (measured: 2 +0.3 to +1 %, 3 and 4 no better)
#endif
__device__ __forceinline__ bool hemi_trial(DV nm, float nx, float ny, float nz, uint64_t zx, uint64_t zy, uint64_t zz,
                                           DV& p) {
    const float fx = 2.f * rng_unit24(zx) - 1.f, fy = 2.f * rng_unit24(zy) - 1.f, fz = 2.f * rng_unit24(zz) - 1.f;
    const float pp = fx * fx + fy * fy + fz * fz;
    const float np = nx * fx + ny * fy + nz * fz;
    if (pp > 1.f + 1e-5f || np < -1e-5f) return false;  // rejected in FP64 too
    p = dv(rng_unit(zx) * 2.0 - 1.0, rng_unit(zy) * 2.0 - 1.0, rng_unit(zz) * 2.0 - 1.0);
    return (pp < 1.f - 1e-5f && np > 1e-5f) || !(vdot(p, p) >= 1.0 || vdot(nm, p) <= 0.);
}
__device__ __forceinline__ DV hemisphere_ball(DV nm, uint64_t key, uint32_t& rn) {
    const float nx = (float)nm.x, ny = (float)nm.y, nz = (float)nm.z;
#if MFX_HEMI_TRIALS > 1
    // MFX_HEMI_TRIALS trials per round (their draws independent): a wave loops until its slowest
    // lane accepts, and the draws' multiply chains are latency-bound, so extra trials per round
    // are nearly free. The first accepted trial wins and only its draws and earlier ones count.
    while (true) {
        const uint32_t r0 = rn;
        uint64_t z[3 * MFX_HEMI_TRIALS];
#pragma unroll
        for (int i = 0; i < 3 * MFX_HEMI_TRIALS; ++i) z[i] = rng_bits(key, rn);
        DV p;
        for (int i = 0; i < MFX_HEMI_TRIALS; ++i)  // left rolled: the early return keeps it from unrolling
            if (hemi_trial(nm, nx, ny, nz, z[3 * i], z[3 * i + 1], z[3 * i + 2], p)) {
                rn = r0 + 3 * (i + 1);
                return p;
            }
    }
#endif
    while (true) {
        const uint64_t zx = rng_bits(key, rn), zy = rng_bits(key, rn), zz = rng_bits(key, rn);
        const float fx = 2.f * rng_unit24(zx) - 1.f, fy = 2.f * rng_unit24(zy) - 1.f, fz = 2.f * rng_unit24(zz) - 1.f;
        const float pp = fx * fx + fy * fy + fz * fz;
        const float np = nx * fx + ny * fy + nz * fz;
        if (pp > 1.f + 1e-5f || np < -1e-5f) continue;  // rejected in FP64 too
        const DV p = dv(rng_unit(zx) * 2.0 - 1.0, rng_unit(zy) * 2.0 - 1.0, rng_unit(zz) * 2.0 - 1.0);
        if ((pp < 1.f - 1e-5f && np > 1e-5f) || !(vdot(p, p) >= 1.0 || vdot(nm, p) <= 0.)) return p;
    }
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

// AABB.hit decided in FP32 where that is provably the FP64 answer (1 hit, 0 miss; -1: undecided,
// take aabb_hit64). For non-NaN slab values the reference's test (early-outs included) is the
// conjunction of: every axis's entry value <= every other axis's exit value, every entry < tMax,
// every exit > tMin (an axis's own entry <= exit holds for lo <= hi). Each slab value is the
// reference's FP64 difference b - o, rounded to FP32 and multiplied by rcp_f32(d): relative error
// < 2^-21 against the FP64 quotient (three roundings of 2^-24 and v_rcp_f32's 1 ulp). A condition
// counts as decided when its two sides are apart by more than 2^-18 of the larger magnitude taking
// part (S, or |tMax|, |tMin|) — more than twice their combined error — so only grazing rays,
// out-of-range values and zero direction components fall back to the divisions.
__device__ __forceinline__ int aabb_screen32(const double* lo, const double* hi, DV o, DV d, double tMin, double tMax) {
    const double dd[3] = {d.x, d.y, d.z}, oo[3] = {o.x, o.y, o.z};
    float mn[3], mx[3];
    bool ok = true;
    float S = 0.f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float df = (float)dd[a];
        const float al = (float)(lo[a] - oo[a]), ah = (float)(hi[a] - oo[a]);  // the reference's FP64 differences
        const float adf = fabsf(df), aal = fabsf(al), aah = fabsf(ah);
        ok = ok && adf >= 0x1p-60f && adf <= 0x1p60f && aal <= 0x1p60f && aah <= 0x1p60f &&
             (aal >= 0x1p-60f || al == 0.f) && (aah >= 0x1p-60f || ah == 0.f);
        const float r = __builtin_amdgcn_rcpf(df);
        const float ql = al * r, qh = ah * r;
        mn[a] = dd[a] >= 0. ? ql : qh;  // the reference's branch on d >= 0 (-0.0 counts as >= 0)
        mx[a] = dd[a] >= 0. ? qh : ql;
        S = fmaxf(S, fmaxf(fabsf(ql), fabsf(qh)));
    }
    if (!ok) return -1;
    const float m = S * 0x1p-18f;
    int res = 1;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            if (i == j) continue;
            if (mn[i] - mx[j] > m) return 0;   // an entry past another axis's exit: certainly a miss
            if (!(mx[j] - mn[i] > m)) res = -1;
        }
    const float tx = (float)tMax, tn = (float)tMin;
    const float mX = fmaxf(S, fabsf(tx)) * 0x1p-18f, mN = fmaxf(S, fabsf(tn)) * 0x1p-18f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (mn[i] - tx > mX) return 0;  // an entry at or beyond tMax
        if (!(tx - mn[i] > mX)) res = -1;
        if (tn - mx[i] > mN) return 0;  // an exit at or before tMin
        if (!(mx[i] - tn > mN)) res = -1;
    }
    return res;
}
__device__ __forceinline__ bool aabb_hit(const double* lo, const double* hi, DV o, DV d, double tMin, double tMax) {
#if MFX_AABB_SCREEN
    const int r = aabb_screen32(lo, hi, o, d, tMin, tMax);
    if (r >= 0) return r == 1;
#endif
    return aabb_hit64(lo, hi, o, d, tMin, tMax);
}

// Triangle.PreCalcu + Hit — Trangle.fs:120-155 (tMax deliberately not checked, :148); fields
// loaded where used (the rare whole-reference-leaf evaluation)
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

// a reference leaf's arrays, read where a candidate needs its whole reference leaf (rare: a hit at
// t >= tMax); k_shadow keeps them in LDS instead of in scalar registers (SceneView::refs)
struct SceneRefs {
    const int32_t* slot_ref;
    const uint8_t* ref_blob;
};
struct SceneView {
    const MfxNode* __restrict__ nodes;
    const MfxSlot* __restrict__ slots;     // traversal leaves: runs of MfxSlot records
    const int32_t* __restrict__ slot_ref;  // per slot: 16-byte offset of its reference leaf in ref_blob
    const uint8_t* __restrict__ ref_blob;  // reference leaves: MfxLeaf + slot copies
    const MfxInstance* __restrict__ inst;  // two-level scenes: the instances (else null)
    const MfxInstance* inst_lds;           // LDS copy of instances [0, ninst_lds) (wavefront kernels)
    int ninst_lds;
    // LDS copy of every slot's 80-B test prefix (a small scene's whole slot array, five 16-B columns
    // per slot; wavefront kernels), or none: nslot_lds is the slot count or 0
    const int4* slots_lds;
    int nslot_lds;
    const SceneRefs* refs = nullptr;  // non-null: slot_ref / ref_blob are read from here (LDS)
};

// An instance's record: from the kernel's LDS copy when it holds it, else from global memory
struct InstR {
    DV off;
    int root, slot_base;
};
__device__ __forceinline__ InstR load_inst(const SceneView& S, int k) {
    InstR r;
    if (k < S.ninst_lds) {
        const MfxInstance& I = S.inst_lds[k];
        r = InstR{ld3(I.off), I.root, I.slot_base};
    } else {
        const MfxInstance& I = S.inst[k];
        r = InstR{ld3(I.off), I.root, I.slot_base};
    }
    return r;
}
// block-wide copy of the first n instances into LDS at kernel start (ends with a barrier)
__device__ __forceinline__ void load_inst_lds(MfxInstance* lds, const MfxInstance* __restrict__ g, int n) {
    const int4* __restrict__ src = (const int4*)g;
    int4* dst = (int4*)lds;
    for (int i = threadIdx.x; i < n * (int)(sizeof(MfxInstance) / 16); i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

struct Stats {
    uint32_t nodes, clusters, prims;  // internal-node visits, leaf visits, primitive tests
#ifdef MFX_DIAG_OCCLUSION
    uint32_t after_nodes, after_leaves;  // closest-hit visits made after the ray's first hit
#endif
};

// The best hit so far under the reference's order: smallest t; equal t -> the later reference
// leaf (larger `first`: `if l.t < r.t then l else r`, BvhNode.fs:70, ties go right); equal t in
// one leaf -> the earlier primitive (Array.minBy keeps the first minimum, BvhNode.fs:80).
struct Best {
    double t;
    int info;   // MfxSlot.info of the hit slot: shade[] index | position in its reference leaf
    int first;  // MfxLeaf.first of its reference leaf
    bool found;
};
__device__ __forceinline__ bool beats(const Best& B, double t, int first, int info) {
    if (!B.found || t < B.t) return true;
    if (t > B.t) return false;
    const unsigned pos = ((unsigned)info >> MFX_INFO_POS_SHIFT) & 3u, bpos = ((unsigned)B.info >> MFX_INFO_POS_SHIFT) & 3u;
    return first > B.first || (first == B.first && pos < bpos);
}

// One whole reference leaf, exactly as CheckHit evaluates it (BvhNode.fs:64-80): its FP64 box
// test, then Array.minBy over its primitives with key (hit ? t : tMax), first minimum wins.
// Returns whether the leaf's result is a hit, with its t, the hit slot's info and the leaf's
// `first`. The two tests have no side effects, so the primitives run first and the box (six
// FP64 divisions) only when the answer still depends on it.
// shadow: an any-hit query (the first hit below tMax decides the leaf)
__device__ bool ref_leaf_hit(const uint8_t* __restrict__ ref_blob, int off16, DV o, DV d, double tMin, double tMax,
                             double& t_out, int& info_out, int& first_out, bool shadow) {
    const MfxLeaf* __restrict__ lf = (const MfxLeaf*)(ref_blob + (size_t)off16 * 16);
    const MfxSlot* __restrict__ sl = (const MfxSlot*)(lf + 1);
    const int count = lf->count, kinds = lf->kinds;
    bool best_hit = false;
    double best_key = 0.0, best_t = 0.0;
    int best_slot = 0;
    int cur = 0;
    for (int k = 0; k < count; ++k) {
        const int kind = (kinds >> (2 * k)) & 3;
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
        // a hit below tMax has a key below every miss's: the minBy result is a hit
        if (shadow && h && t < tMax) break;
    }
    if (!best_hit) return false;
    if (!aabb_hit64(lf->lo, lf->hi, o, d, tMin, tMax)) return false;
    t_out = best_t;
    info_out = sl[best_slot].info;
    first_out = lf->first;
    return true;
}

#ifndef MFX_AABB_SCREEN
#define MFX_AABB_SCREEN 1  // the winning candidate's reference-leaf box test screened in FP32 (exact)
#endif

#ifndef MFX_TRI_BOX_PROOF
#define MFX_TRI_BOX_PROOF 1  // a triangle winner's leaf-box test proved from its own vertices (tri_box_pass)
#endif
#ifndef MFX_LEAF_PRELOAD
// 0: fields loaded where used; 1: a slot's 80-B test prefix in one round; 2: + its box (+5 % on C2
// when every winner read it; with MFX_TRI_BOX_PROOF few do)
#define MFX_LEAF_PRELOAD (MFX_TRI_BOX_PROOF ? 1 : 2)
#endif
#ifndef MFX_SHADOW_PRELOAD
#define MFX_SHADOW_PRELOAD MFX_LEAF_PRELOAD  // the same for shadow queries (a hit ends them: the box is rarely needed)
#endif

// A traversal slot's test prefix (bytes 0..79: geometry, `first`, `info`) in registers, loaded
// as five independent 16-B loads in one round before any test arithmetic. Loading fields where
// they are used puts two dependent memory round trips into every triangle test (e1/e2 first, v0
// only after the divisor cull), which the compiler may not hoist above the branch.
struct SlotR {
    DV a, b, c;
    int first, info;
};
__device__ __forceinline__ double i2d(int lo, int hi) { return __hiloint2double(hi, lo); }
__device__ __forceinline__ SlotR load_slot(const MfxSlot* __restrict__ p) {
    const int4* __restrict__ q = (const int4*)p;
    const int4 r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4];
    SlotR s;
    s.a = dv(i2d(r0.x, r0.y), i2d(r0.z, r0.w), i2d(r1.x, r1.y));
    s.b = dv(i2d(r1.z, r1.w), i2d(r2.x, r2.y), i2d(r2.z, r2.w));
    s.c = dv(i2d(r3.x, r3.y), i2d(r3.z, r3.w), i2d(r4.x, r4.y));
    s.first = r4.z;
    s.info = r4.w;
    return s;
}
// The same prefix from a wave-uniform slot address through scalar loads (packet traversal: every
// lane tests the same slot, so the data comes from the scalar cache, not per lane)
typedef int mfx_i4 __attribute__((ext_vector_type(4)));
typedef float mfx_f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const mfx_i4 mfx_ci4;
typedef __attribute__((address_space(4))) const mfx_f4 mfx_cf4;
__device__ __forceinline__ SlotR load_slot_u(const MfxSlot* __restrict__ p) {
    mfx_ci4* q = (mfx_ci4*)p;
    const mfx_i4 r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4];
    SlotR s;
    s.a = dv(i2d(r0.x, r0.y), i2d(r0.z, r0.w), i2d(r1.x, r1.y));
    s.b = dv(i2d(r1.z, r1.w), i2d(r2.x, r2.y), i2d(r2.z, r2.w));
    s.c = dv(i2d(r3.x, r3.y), i2d(r3.z, r3.w), i2d(r4.x, r4.y));
    s.first = r4.z;
    s.info = r4.w;
    return s;
}
// a slot's reference-leaf box (bytes 80..127) through scalar loads
__device__ __forceinline__ void load_box_u(const MfxSlot* __restrict__ p, double lo[3], double hi[3]) {
    mfx_ci4* q = (mfx_ci4*)p;
    const mfx_i4 r5 = q[5], r6 = q[6], r7 = q[7];
    lo[0] = i2d(r5.x, r5.y); lo[1] = i2d(r5.z, r5.w); lo[2] = i2d(r6.x, r6.y);
    hi[0] = i2d(r6.z, r6.w); hi[1] = i2d(r7.x, r7.y); hi[2] = i2d(r7.z, r7.w);
}

// The same prefix from the kernel's LDS copy of the slots (SceneView::slots_lds)
__device__ __forceinline__ SlotR load_slot_lds(const int4* t, int slot) {
    const int4* q = t + 5 * slot;
    const int4 r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4];
    SlotR s;
    s.a = dv(i2d(r0.x, r0.y), i2d(r0.z, r0.w), i2d(r1.x, r1.y));
    s.b = dv(i2d(r1.z, r1.w), i2d(r2.x, r2.y), i2d(r2.z, r2.w));
    s.c = dv(i2d(r3.x, r3.y), i2d(r3.z, r3.w), i2d(r4.x, r4.y));
    s.first = r4.z;
    s.info = r4.w;
    return s;
}
// block-wide copy of n slots' test prefixes into LDS at kernel start (ends with a barrier)
__device__ __forceinline__ void load_slots_lds(int4* lds, const MfxSlot* __restrict__ g, int n) {
    for (int i = threadIdx.x; i < 5 * n; i += blockDim.x) lds[i] = ((const int4*)(g + i / 5))[i % 5];
    __syncthreads();
}

// Triangle.PreCalcu + Hit — Trangle.fs:120-155 (tMax deliberately not checked, :148)
__device__ __forceinline__ bool tri_hit64(const SlotR& s, DV o, DV d, double tMin, double& t) {
    DV s1 = vcross(d, s.c);
    double divisor = vdot(s1, s.b);
    if (fabs(divisor) < 1e-6) return false;
    double inv = 1. / divisor;
    DV dd = vsub(o, s.a);
    double b1 = vdot(dd, s1) * inv;
    if (b1 < 0. || b1 > 1.) return false;
    DV s2 = vcross(dd, s.b);
    double b2 = vdot(d, s2) * inv;
    if (b2 < 0. || (b1 + b2) >= 1.) return false;
    t = vdot(s.c, s2) * inv;
    return t > tMin;
}
// Sphere.Hit — Sphere.fs:21-43
__device__ __forceinline__ bool sphere_hit64(const SlotR& s, DV o, DV d, double tMin, double tMax, double& t) {
    DV oc = vsub(o, s.a);
    double a = 1.;
    double b = 2.0 * vdot(oc, d);
    double c = vdot(oc, oc) - s.b.x * s.b.x;
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

// The reference leaf's box test (AABB.hit, IHitable.fs:18-54) for a triangle candidate, proved to
// pass without reading the box: the leaf box contains the triangle's vertex box (InitNode unions
// the primitives' bounds, BvhNode.fs:32-37; Triangle's bound is its vertices', Trangle.fs:113) and
// the rounded slab test is monotone in the bounds, so an upper bound on every axis's entry value
// and a lower bound on every exit value that satisfy aabb_screen32's conjunction (entries <= other
// axes' exits, entries < tMax, exits > tMin) prove the FP64 test passes. The bounds are the vertex
// box's slab values in FP32 — vertices relative to the origin from the FP64 difference v0 - o and
// the stored edges — whose error against the FP64 values is below 2^-21 (R / |d| + |q|), R =
// |v0 - o| + |e1| + |e2| per axis; each comparison needs a gap of 2^-18 of that on both sides.
// false: not proved (grazing rays, hits within ~1e-5 of the vertex box's faces, zero or tiny
// direction components, t next to tMin/tMax): the caller runs the FP64 test on the loaded box.
__device__ __forceinline__ bool tri_box_pass(DV a, DV e1, DV e2, DV o, DV d, double tMin, double tMax) {
    const double aa[3] = {a.x, a.y, a.z}, b1[3] = {e1.x, e1.y, e1.z}, b2[3] = {e2.x, e2.y, e2.z};
    const double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    float U[3], L[3], E[3];
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float A = (float)(aa[k] - oo[k]), p = (float)b1[k], q = (float)b2[k];
        const float x1 = A + p, x2 = A + q;
        const float mn = fminf(A, fminf(x1, x2)), mx = fmaxf(A, fmaxf(x1, x2));
        const float R = fabsf(A) + fabsf(p) + fabsf(q);
        const float df = (float)dd[k], adf = fabsf(df);
        ok = ok && adf >= 0x1p-60f && adf <= 0x1p60f && R >= 0x1p-60f && R <= 0x1p60f;
        const float rc = __builtin_amdgcn_rcpf(df);
        const float qm = mn * rc, qM = mx * rc;
        U[k] = dd[k] >= 0. ? qm : qM;  // entry <= the vertex box's entry value
        L[k] = dd[k] >= 0. ? qM : qm;  // exit >= the vertex box's exit value
        E[k] = (R * fabsf(rc) + fmaxf(fabsf(qm), fabsf(qM))) * 0x1p-18f;
    }
    if (!ok) return false;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if (i != j) ok = ok && L[j] - U[i] > E[i] + E[j];
    const float tx = (float)tMax, tn = (float)tMin;
    const float ex = fabsf(tx) * 0x1p-22f, en = fabsf(tn) * 0x1p-22f;
#pragma unroll
    for (int i = 0; i < 3; ++i) ok = ok && tx - U[i] > E[i] + ex && L[i] - tn > E[i] + en;
    return ok;
}

// One traversal leaf (1..4 primitives of possibly different reference leaves; child code = first
// slot << 3 | slots - 1). Each primitive hit is a candidate for its reference leaf's result: with
// t < tMax the reference leaf's minBy result is a hit of t no larger (the leaf's other primitives
// are tested in their own traversal leaves), so the candidate counts iff it beats the best hit
// under the reference's order and its reference leaf passes the exact FP64 box test (ancestor
// boxes contain it, and the rounded slab test is monotone in the bounds, so they pass too). Both
// the box and `first` sit in the slot's own cache line. A hit at t >= tMax (Triangle.Hit ignores
// tMax, Trangle.fs:148) is where the leaf's minBy can prefer a miss: that reference leaf is then
// evaluated whole. SHADOW: returns true at the first occluding candidate. Closest: returns true
// when B improved.
// base: the slot index the code counts from (an instance's run of world slots; 0 otherwise).
// UNI: the leaf is wave-uniform (packet traversal): its slots are read through scalar loads.
// SLDS: the slots are read from the kernel's LDS copy (S.slots_lds holds every slot of a small scene).
template <bool SHADOW, bool STATS, bool UNI = false, bool SLDS = false>
__device__ __forceinline__ bool leaf_hit(const SceneView& S, int code, DV o, DV d, double tMin, double tMax,
                                         Best& B, Stats& st, int base = 0) {
    constexpr bool shd = SHADOW;
    const int s0 = base + (code >> 3), n = (code & 7) + 1;
    const MfxSlot* __restrict__ sl = S.slots + s0;
    if (STATS) st.clusters++;
    bool improved = false;
    constexpr int PRE = SHADOW ? MFX_SHADOW_PRELOAD : MFX_LEAF_PRELOAD;
    constexpr bool in_lds = SLDS && !UNI;
    for (int k = 0; k < n; ++k) {
#if MFX_LEAF_PRELOAD
        SlotR r = UNI ? load_slot_u(sl + k) : (in_lds ? load_slot_lds(S.slots_lds, s0 + k) : load_slot(sl + k));
        // the reference leaf's box (bytes 80..127; both slots of a rect carry the same one)
        double2 bx0 = make_double2(0, 0), bx1 = bx0, bx2 = bx0;
        if (PRE == 2) {
            bx0 = *(const double2*)sl[k].lo;
            bx1 = *(const double2*)(sl[k].lo + 2);
            bx2 = *(const double2*)(sl[k].hi + 1);
        }
        int info = r.info;
        const int kind = (info >> MFX_INFO_KIND_SHIFT) & 3;
        if (STATS) st.prims++;
        double t = 0.0;
        int hs = k;
        int first = r.first;
        bool hit;
        if (kind == MFX_KIND_SPHERE) {
            hit = sphere_hit64(r, o, d, tMin, tMax, t);
        } else {
            hit = tri_hit64(r, o, d, tMin, t);
            if (kind == MFX_KIND_RECT) {
                ++k;  // Rect.Hit: trig1, else trig2 (Rect.fs:26-31); the second slot follows
                if (!hit) {
                    hs = k;
                    r = UNI ? load_slot_u(sl + k) : (in_lds ? load_slot_lds(S.slots_lds, s0 + k) : load_slot(sl + k));
                    hit = tri_hit64(r, o, d, tMin, t);
                    info = r.info;
                    first = r.first;
                }
            }
        }
#else
        int info = sl[k].info;
        const int kind = (info >> MFX_INFO_KIND_SHIFT) & 3;
        if (STATS) st.prims++;
        double t = 0.0;
        int hs = k;
        bool hit;
        if (kind == MFX_KIND_SPHERE) {
            hit = sphere_hit64(load_slot(sl + k), o, d, tMin, tMax, t);
        } else {
            hit = tri_hit64(load_slot(sl + k), o, d, tMin, t);
            if (kind == MFX_KIND_RECT) {
                ++k;
                if (!hit) {
                    hs = k;
                    hit = tri_hit64(load_slot(sl + k), o, d, tMin, t);
                    info = sl[k].info;
                }
            }
        }
        const int first = sl[hs].first;
#endif
        if (!hit) continue;
        if (t >= tMax) {
            double t2;
            int info2, first2;
            const int32_t* sref = S.refs ? S.refs->slot_ref : S.slot_ref;
            const uint8_t* rblob = S.refs ? S.refs->ref_blob : S.ref_blob;
            if (ref_leaf_hit(rblob, sref[s0 + hs], o, d, tMin, tMax, t2, info2, first2, shd)) {
                if (shd) return true;
                if (beats(B, t2, first2, info2)) {
                    B = Best{t2, info2, first2, true};
                    improved = true;
                }
            }
            continue;
        }
        if (!shd && B.found && t > B.t) continue;  // cannot win: skip the box test
        if (!shd && !beats(B, t, first, info)) continue;
#if MFX_TRI_BOX_PROOF && MFX_LEAF_PRELOAD
        if (kind != MFX_KIND_SPHERE && tri_box_pass(r.a, r.b, r.c, o, d, tMin, tMax)) {
            // the reference leaf's box test passes (proved; its box is not read)
        } else
#endif
        if (PRE == 2) {
            const double blo[3] = {bx0.x, bx0.y, bx1.x}, bhi[3] = {bx1.y, bx2.x, bx2.y};
            if (!aabb_hit(blo, bhi, o, d, tMin, tMax)) continue;
        } else if (UNI) {
            double blo[3], bhi[3];
            load_box_u(sl + hs, blo, bhi);
            if (!aabb_hit(blo, bhi, o, d, tMin, tMax)) continue;
        } else {
            if (!aabb_hit(sl[hs].lo, sl[hs].hi, o, d, tMin, tMax)) continue;
        }
        if (shd) return true;
        B = Best{t, info, first, true};
        improved = true;
    }
    return improved;
}

__device__ __forceinline__ float f_round_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = nextafterf(f, __builtin_inff());
    return f;
}
// a node step's distance limit: x rounded up, at most FLT_MAX, so a box whose entry distance
// overflows to +inf (an empty child's +inf planes, mfx_api.cpp node_to_half) is never entered
__device__ __forceinline__ float f_tlim(double x) { return fminf(f_round_up(x), 3.402823466e38f); }

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
// the same ray from another origin (an instance frame's o - off, or back to the world's o): the
// direction terms are the ray's own, so only the origin products are recomputed, with make_rayf's
// expressions (the result is make_rayf(o, d) bit for bit)
__device__ __forceinline__ void rayf_origin(RayF& r, DV o) {
    r.oix = (float)o.x * r.ix; r.oiy = (float)o.y * r.iy; r.oiz = (float)o.z * r.iz;
}

// PostProcessAndToScreenBuffer's per-channel byte (Scene.fs:280-289, 315-330): ACES tone curve,
// clamp, sqrt (gamma 2), 255.99 scale, truncated
__device__ __forceinline__ double clamp01(double x) { return x < 0. ? 0. : (x > 1. ? 1. : x); }
__device__ __forceinline__ double aces1(double x) {
    const double a = 2.51, b = 0.03, c = 2.43, d = 0.59, e = 0.14;
    return clamp01((x * (a * x + b)) / (x * (c * x + d) + e));
}
__device__ __forceinline__ uint8_t post_byte(double t) { return (uint8_t)(int)(255.99 * sqrt(aces1(t))); }

#define MFX_TRAV_EXIT (-0x7fffffff - 1)  // node value: traversal finished (stack empty, no hit child)

// two-level scenes: a node value that enters an instance (~(MFX_INST_FLAG | instance)); leaf codes
// stay below MFX_INST_FLAG
__device__ __forceinline__ bool is_inst_code(int node) { return node > MFX_TRAV_EXIT && node <= ~MFX_INST_FLAG; }
// the FP32 search ray in the frame of instance `inst` (-1: the world): origin o - off
__device__ __forceinline__ RayF frame_ray(const SceneView& S, int inst, DV o, DV d) {
    if (inst >= 0) o = vsub(o, load_inst(S, inst).off);
    return make_rayf(o, d);
}

// A lane's traversal stack. LdsStack: the whole bound in an LDS column (stride 64 dwords:
// conflict-free). SpillStack: the first `nlds` entries in LDS and deeper ones in a global column
// (stride `gstride`), so the LDS a wave needs — which caps the resident waves — no longer grows
// with the BVH's depth; pushes that deep are rare.
// `deep` is wave-uniform: false when no lane of the wave touches an entry past nlds, so the common
// case runs plain LDS accesses behind one scalar branch.
struct LdsStack {
    int* lds;
    __device__ __forceinline__ bool deep(int) const { return false; }
    __device__ __forceinline__ int get(int i, bool) const { return lds[i * 64]; }
    __device__ __forceinline__ void put(int i, int v, bool) const { lds[i * 64] = v; }
};
struct SpillStack {
    int* lds;
    int* spill;
    int nlds, gstride;
    __device__ __forceinline__ bool deep(int top) const { return __ballot(top > nlds) != 0; }  // top: highest index + 1
    __device__ __forceinline__ int get(int i, bool dp) const {
        if (!dp) return lds[i * 64];
        return i < nlds ? lds[i * 64] : spill[(i - nlds) * gstride];
    }
    __device__ __forceinline__ void put(int i, int v, bool dp) const {
        if (!dp || i < nlds) lds[i * 64] = v;
        else spill[(i - nlds) * gstride] = v;
    }
};

// One internal-node step of the BVH4, branch-free: four child slab tests, the hit children sorted
// near to far (5-comparator network over (entry distance, child), misses sorted last at +inf),
// then descend into the nearest, push the others far-first, or pop. The pop candidate (top of
// stack) is read before the node's boxes arrive, so the LDS read overlaps the L2 load. Returns the
// next node: >= 0 internal, < 0 a leaf (~offset), or MFX_TRAV_EXIT when nothing is left. An empty
// child (box at FLT_MAX) never hits.
// FAR (shadow rays): the children are visited far to near by exit distance. Whether a shadow ray
// is occluded does not depend on the order (the any-hit test keeps tMax fixed, and a leaf that
// reports a hit under a shrunken tMax also does under the original one), and the occluder of a
// ray leaving a surface is seldom near its origin. Near-first walked every node around the origin
// first: C2 shadow rays 7.26 -> 5.58 node and 2.32 -> 1.57 leaf visits, +12 % on the frame.
__device__ __forceinline__ void cswap(float& da, int& ca, float& db, int& cb) {
    const bool s = db < da;
    const float t = da;
    const int u = ca;
    da = s ? db : da;
    ca = s ? cb : ca;
    db = s ? t : db;
    cb = s ? u : cb;
}
// LDS copy of the first `ntop` nodes (the BVH's top levels: mfx_scene.cpp numbers them first, in
// breadth-first order). Node n's 16-B column c sits at float4 n * 8 + (c ^ ((n >> 1) & 7)), so
// lanes reading the same column of different nodes spread over the LDS banks.
struct TopNodes {
    const float4* lds;
    int ntop;
#if MFX_NODE_F16
    const MfxNodeH* nodes_h = nullptr;  // the per-lane kernels' FP16 nodes (the LDS copy alike)
#endif
};
__device__ __forceinline__ int top_col(int n, int c) { return n * 8 + (c ^ ((n >> 1) & 7)); }
// block-wide copy at kernel start (all threads; ends with a barrier); a node is eight 16-B columns
static_assert(sizeof(MfxNode) == 128, "top nodes are 8 columns");
__device__ __forceinline__ void load_top_nodes(float4* lds, const void* __restrict__ nodes, int ntop) {
    const float4* __restrict__ g = (const float4*)nodes;
    for (int i = threadIdx.x; i < ntop * 8; i += blockDim.x) lds[top_col(i >> 3, i & 7)] = g[i];
    __syncthreads();
}
#if MFX_NODE_F16
// an FP16 node's four 16-B columns at float4 n * 8 + (c ^ ((n >> 1) & 3))
__device__ __forceinline__ void load_top_nodes_h(float4* lds, const MfxNodeH* __restrict__ nodes, int ntop) {
    const float4* __restrict__ g = (const float4*)nodes;
    for (int i = threadIdx.x; i < ntop * 4; i += blockDim.x) lds[(i >> 2) * 8 + ((i & 3) ^ ((i >> 3) & 3))] = g[i];
    __syncthreads();
}
typedef _Float16 mfx_h2 __attribute__((ext_vector_type(2)));
// four FP16 planes (two dwords) as floats
__device__ __forceinline__ float4 h4f(uint32_t a, uint32_t b) {
    const mfx_h2 x = __builtin_bit_cast(mfx_h2, a), y = __builtin_bit_cast(mfx_h2, b);
    return make_float4((float)x.x, (float)x.y, (float)y.x, (float)y.y);
}
#endif

// Two-level frame bookkeeping after a step or a pop. A lane in an instance remembers the stack
// depth at which it entered (inst_sp): entries below it belong to the world frame, so a pop below
// it leaves the instance (world FP32 ray). An instance code is entered: its template's root, the
// ray moved into its frame (origin o - off), from one read of its record.
__device__ __forceinline__ int inst_frame(const SceneView& S, int node, int& inst, int& inst_sp, int sp, DV o, DV d,
                                          RayF& rf) {
    if (inst >= 0 && sp < inst_sp) {
        inst = -1;
        rayf_origin(rf, o);
    }
    if (is_inst_code(node)) {
        inst = ~node & ~MFX_INST_FLAG;
        inst_sp = sp;
        const InstR r = load_inst(S, inst);
        rayf_origin(rf, vsub(o, r.off));
        node = r.root;
    }
    return node;
}

// The slab distances of a BVH4 node's four children for one FP32 ray: plane * (1/d) - o * (1/d),
// one rounding each (fmaf). (Two children per v_pk_fma_f32, gfx950's packed FP32 FMA — the same
// fused operation, the same bits — measured: k_camera unchanged, the per-lane kernels' extra
// register pairs C2 -2.6 %, C4 -2.2 %; r05f_ab_pk_slab.txt. Not kept.)
struct Slab4 {
    float a0[4], a1[4], b0[4], b1[4], c0[4], c1[4];
};
__device__ __forceinline__ void slab4(const float4& lx, const float4& hx, const float4& ly, const float4& hy,
                                      const float4& lz, const float4& hz, const RayF& r, Slab4& S) {
    const float LX[4] = {lx.x, lx.y, lx.z, lx.w}, HX[4] = {hx.x, hx.y, hx.z, hx.w};
    const float LY[4] = {ly.x, ly.y, ly.z, ly.w}, HY[4] = {hy.x, hy.y, hy.z, hy.w};
    const float LZ[4] = {lz.x, lz.y, lz.z, lz.w}, HZ[4] = {hz.x, hz.y, hz.z, hz.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        S.a0[k] = fmaf(LX[k], r.ix, -r.oix); S.a1[k] = fmaf(HX[k], r.ix, -r.oix);
        S.b0[k] = fmaf(LY[k], r.iy, -r.oiy); S.b1[k] = fmaf(HY[k], r.iy, -r.oiy);
        S.c0[k] = fmaf(LZ[k], r.iz, -r.oiz); S.c1[k] = fmaf(HZ[k], r.iz, -r.oiz);
    }
}

// Diagnostic builds (-DMFX_DIAG_STAMPS, scripts/latency_roof.py): `lat` != null accumulates the wave's
// cycles from the node loads' issue to their first use (the slab tests), the step's round trip.
__device__ __forceinline__ uint64_t diag_clock() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#if MFX_NODE_F16
// node_step on the FP16 node (VERDICT r05 Next #4b): four 16-B loads instead of seven, the planes
// widened exactly (v_cvt_f32_f16), then the same FP32 slab test, order and pushes. The boxes are the
// FP32 ones rounded outward, so a lane visits a superset of its FP32 walk's nodes; the leaf tests
// decide the hits (§3), and the images are the same bits
template <bool TOP, bool FAR, typename ST>
__device__ __forceinline__ int node_step_h(int node, const RayF& r, float tlim, const ST& stack, int& sp, TopNodes tn,
                                           uint64_t* lat) {
    const bool dp = stack.deep(sp + 3);
    const int top = stack.get(sp > 0 ? sp - 1 : 0, dp);
    const uint64_t t_issue = lat ? diag_clock() : 0;
    uint4 A, B, C;
    int4 ch;
    if (TOP && node < tn.ntop) {
        const int sw = (node >> 1) & 3;
        const uint4* t = (const uint4*)tn.lds + node * 8;
        A = t[0 ^ sw]; B = t[1 ^ sw]; C = t[2 ^ sw];
        const uint4 c4 = t[3 ^ sw];
        ch = make_int4((int)c4.x, (int)c4.y, (int)c4.z, (int)c4.w);
    } else {
        const uint4* __restrict__ q = (const uint4*)(tn.nodes_h + node);
        A = q[0]; B = q[1]; C = q[2];
        ch = *(const int4*)(q + 3);
    }
    Slab4 SL;
    slab4(h4f(A.x, A.y), h4f(A.z, A.w), h4f(B.x, B.y), h4f(B.z, B.w), h4f(C.x, C.y), h4f(C.z, C.w), r, SL);
    if (lat) *lat += diag_clock() - t_issue;
    float d[4];
    int c[4] = {ch.x, ch.y, ch.z, ch.w};
    int nh = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float a0 = SL.a0[k], a1 = SL.a1[k], b0 = SL.b0[k], b1 = SL.b1[k], c0 = SL.c0[k], c1 = SL.c1[k];
        const float n = fmaxf(fmaxf(fminf(a0, a1), fminf(b0, b1)), fmaxf(fminf(c0, c1), 0.0f));
        const float f = fminf(fminf(fmaxf(a0, a1), fmaxf(b0, b1)), fminf(fmaxf(c0, c1), tlim));
        const bool h = n <= f;
        d[k] = h ? (FAR ? -f : n) : __builtin_inff();
        nh += h ? 1 : 0;
    }
    cswap(d[0], c[0], d[1], c[1]);
    cswap(d[2], c[2], d[3], c[3]);
    cswap(d[0], c[0], d[2], c[2]);
    cswap(d[1], c[1], d[3], c[3]);
    cswap(d[1], c[1], d[2], c[2]);
    if (nh >= 2) stack.put(sp, nh == 4 ? c[3] : (nh == 3 ? c[2] : c[1]), dp);
    if (nh >= 3) stack.put(sp + 1, nh == 4 ? c[2] : c[1], dp);
    if (nh >= 4) stack.put(sp + 2, c[1], dp);
    const bool pop = nh == 0 && sp > 0;
    const int next = nh > 0 ? c[0] : (pop ? top : MFX_TRAV_EXIT);
    sp += nh > 0 ? nh - 1 : (pop ? -1 : 0);
    return next;
}
#endif
template <bool TOP = false, bool FAR = false, typename ST>
__device__ __forceinline__ int node_step(const MfxNode* __restrict__ nodes, int node, const RayF& r, float tlim,
                                         const ST& stack, int& sp, TopNodes tn = TopNodes{nullptr, 0},
                                         uint64_t* lat = nullptr) {
#if MFX_NODE_F16
    if (tn.nodes_h) return node_step_h<TOP, FAR>(node, r, tlim, stack, sp, tn, lat);
#endif
    const bool dp = stack.deep(sp + 3);  // this step reads sp - 1 and may write sp .. sp + 2
    const int top = stack.get(sp > 0 ? sp - 1 : 0, dp);
    const uint64_t t_issue = lat ? diag_clock() : 0;
    // Lanes at a top-level node read LDS, the others global memory. In a wave with both, the two
    // reads land in the same registers, so the LDS reads wait for the global loads (measured
    // alternatives: LDS only when the whole wave is at top nodes, -0.5 to -2 %; both reads by every
    // lane into separate registers, global ones through out-of-range buffer offsets, -1.5 to -9 %).
    float4 lx, hx, ly, hy, lz, hz;
    int4 ch;
    if (TOP && node < tn.ntop) {
        const int sw = (node >> 1) & 7;
        const float4* t = tn.lds + node * 8;
        lx = t[0 ^ sw]; hx = t[1 ^ sw]; ly = t[2 ^ sw]; hy = t[3 ^ sw]; lz = t[4 ^ sw]; hz = t[5 ^ sw];
        const float4 c4 = t[6 ^ sw];
        ch = make_int4(__float_as_int(c4.x), __float_as_int(c4.y), __float_as_int(c4.z), __float_as_int(c4.w));
    } else {
        const float4* __restrict__ q = (const float4*)(nodes + node);
        lx = q[0]; hx = q[1]; ly = q[2]; hy = q[3]; lz = q[4]; hz = q[5];
        ch = *(const int4*)(q + 6);
    }
    float d[4];
    int c[4] = {ch.x, ch.y, ch.z, ch.w};
    int nh = 0;
    Slab4 SL;
    slab4(lx, hx, ly, hy, lz, hz, r, SL);
    if (lat) *lat += diag_clock() - t_issue;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float a0 = SL.a0[k], a1 = SL.a1[k], b0 = SL.b0[k], b1 = SL.b1[k], c0 = SL.c0[k], c1 = SL.c1[k];
        const float n = fmaxf(fmaxf(fminf(a0, a1), fminf(b0, b1)), fmaxf(fminf(c0, c1), 0.0f));
        const float f = fminf(fminf(fmaxf(a0, a1), fmaxf(b0, b1)), fminf(fmaxf(c0, c1), tlim));
        const bool h = n <= f;
        d[k] = h ? (FAR ? -f : n) : __builtin_inff();
        nh += h ? 1 : 0;
    }
    cswap(d[0], c[0], d[1], c[1]);
    cswap(d[2], c[2], d[3], c[3]);
    cswap(d[0], c[0], d[2], c[2]);
    cswap(d[1], c[1], d[3], c[3]);
    cswap(d[1], c[1], d[2], c[2]);
    // far-first pushes: stack[sp + j] = c[nh - 1 - j] for j < nh - 1 (exec-masked stores, so the
    // stack never holds more than the pushes themselves: mfx_scene.cpp's Collapse4 bound)
    if (nh >= 2) stack.put(sp, nh == 4 ? c[3] : (nh == 3 ? c[2] : c[1]), dp);
    if (nh >= 3) stack.put(sp + 1, nh == 4 ? c[2] : c[1], dp);
    if (nh >= 4) stack.put(sp + 2, c[1], dp);
    const bool pop = nh == 0 && sp > 0;
    const int next = nh > 0 ? c[0] : (pop ? top : MFX_TRAV_EXIT);
    sp += nh > 0 ? nh - 1 : (pop ? -1 : 0);
    return next;
}

// ---- Packet traversal for coherent rays (the camera rays of one 8x8 tile: k_camera) ----------------
// The wave walks the BVH4 together: the node is wave-uniform and read through scalar loads, each
// lane tests the four children with its own FP32 ray and limit, and a child is visited when any
// lane's test hits it. Each lane therefore visits a superset of the nodes its own traversal would
// (a lane's limit only falls, so a child all lanes miss holds no candidate better than any lane's
// final hit), and tests every leaf the wave visits; the per-candidate leaf semantics (leaf_hit)
// make extra candidates harmless, so every lane's closest hit is the single-ray traversal's. Visit
// order: near to far by the entry distances of the first active lane (children it misses last).
// The stack is wave-uniform, in LDS.
// the node-step sort network over (distance, child, lane mask) triples
__device__ __forceinline__ void cswap3(float& da, int& ca, uint64_t& ma, float& db, int& cb, uint64_t& mb) {
    const bool s = db < da;
    const float t = da;
    const int u = ca;
    const uint64_t w = ma;
    da = s ? db : da;
    ca = s ? cb : ca;
    ma = s ? mb : ma;
    db = s ? t : db;
    cb = s ? u : cb;
    mb = s ? w : mb;
}
// The node columns (MfxNode: lo x, hi x, lo y, hi y, lo z, hi z as float4 over the four children)
// of the near and far planes per axis, for a packet whose active lanes' directions share their signs
// on every axis (the camera rays of almost every tile): a child's near plane on an axis is its lo
// plane where the direction is positive and its hi plane where it is negative. Because fmaf rounds
// monotonically and a child's lo <= hi (outward-rounded boxes; an empty child is lo = hi = FLT_MAX),
// fmaf(near, 1/d, -o/d) is exactly min(fmaf(lo, ...), fmaf(hi, ...)): the slab test keeps its
// bits without the per-axis min / max pairs (VALU issue is the packet step's bound).
struct PacketPlanes {
    int nx, fx, ny, fy, nz, fz;
};

// One node of the packet walk. `mask`, kept beside every stack entry, names the lanes whose own
// test hit the node: only they test its children, so a leaf is tested by the lanes whose ray hits
// its box (child boxes lie inside their parent's, so a lane that missed a node misses its subtree).
// The stack is wave-uniform: stk[] nodes and stm[] masks in LDS.
// (The sort on the scalar unit instead — integer keys, the ballots and'ed with the node's mask —
// halves the step's vector instructions but doubles its scalar ones, and the scalar unit issues
// for one SIMD per cycle, as the vector unit: k_camera 4.40 -> 4.61 ms, r06o. The step balances
// the two as it is: ~90 vector, ~80 scalar instructions.)
template <bool UNI>
__device__ __forceinline__ int packet_node_step(const MfxNode* __restrict__ nodes, int node, uint64_t& mask,
                                                const RayF& r, float tlim, int* stk, uint64_t* stm, int& sp, int rep,
                                                const PacketPlanes& pp) {
    mfx_cf4* q = (mfx_cf4*)(nodes + node);
    float n[4], f[4];
    const mfx_i4 ch = ((mfx_ci4*)q)[6];
    if (UNI) {
        const mfx_f4 NX = q[pp.nx], FX = q[pp.fx], NY = q[pp.ny], FY = q[pp.fy], NZ = q[pp.nz], FZ = q[pp.fz];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float ax = fmaf(NX[k], r.ix, -r.oix), bx = fmaf(FX[k], r.ix, -r.oix);
            const float ay = fmaf(NY[k], r.iy, -r.oiy), by = fmaf(FY[k], r.iy, -r.oiy);
            const float az = fmaf(NZ[k], r.iz, -r.oiz), bz = fmaf(FZ[k], r.iz, -r.oiz);
            n[k] = fmaxf(fmaxf(ax, ay), fmaxf(az, 0.0f));
            f[k] = fminf(fminf(bx, by), fminf(bz, tlim));
        }
    } else {
        const mfx_f4 lx = q[0], hx = q[1], ly = q[2], hy = q[3], lz = q[4], hz = q[5];
        Slab4 SL;
        slab4(float4{lx.x, lx.y, lx.z, lx.w}, float4{hx.x, hx.y, hx.z, hx.w}, float4{ly.x, ly.y, ly.z, ly.w},
              float4{hy.x, hy.y, hy.z, hy.w}, float4{lz.x, lz.y, lz.z, lz.w}, float4{hz.x, hz.y, hz.z, hz.w}, r, SL);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float a0 = SL.a0[k], a1 = SL.a1[k], b0 = SL.b0[k], b1 = SL.b1[k], c0 = SL.c0[k], c1 = SL.c1[k];
            n[k] = fmaxf(fmaxf(fminf(a0, a1), fminf(b0, b1)), fmaxf(fminf(c0, c1), 0.0f));
            f[k] = fminf(fminf(fmaxf(a0, a1), fmaxf(b0, b1)), fminf(fmaxf(c0, c1), tlim));
        }
    }
    int c[4] = {ch.x, ch.y, ch.z, ch.w};
    uint64_t m[4];
    int nh = 0;
    float d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        // the lanes of the node's mask whose test hits: the compare's lane mask and'ed with it (no
        // per-lane copy of the node's mask), back to a lane predicate for the select below
        m[k] = __builtin_amdgcn_ballot_w64(n[k] <= f[k]) & mask;
        const bool h = __builtin_amdgcn_inverse_ballot_w64(m[k]);
        // the representative lane's entry distance, read across lanes into a scalar register
        // (v_readlane: rep is wave-uniform; a __shfl is an LDS permute on the step's chain)
        const float kd = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(h ? n[k] : 3.0e38f), rep));
        d[k] = m[k] ? kd : __builtin_inff();
        nh += m[k] ? 1 : 0;
    }
    cswap3(d[0], c[0], m[0], d[1], c[1], m[1]);
    cswap3(d[2], c[2], m[2], d[3], c[3], m[3]);
    cswap3(d[0], c[0], m[0], d[2], c[2], m[2]);
    cswap3(d[1], c[1], m[1], d[3], c[3], m[3]);
    cswap3(d[1], c[1], m[1], d[2], c[2], m[2]);
    nh = __builtin_amdgcn_readfirstlane(nh);
    if (__lane_id() == 0) {  // the pushes are wave-uniform: one lane writes them
        if (nh >= 2) {
            stk[sp] = nh == 4 ? c[3] : (nh == 3 ? c[2] : c[1]);
            stm[sp] = nh == 4 ? m[3] : (nh == 3 ? m[2] : m[1]);
        }
        if (nh >= 3) {
            stk[sp + 1] = nh == 4 ? c[2] : c[1];
            stm[sp + 1] = nh == 4 ? m[2] : m[1];
        }
        if (nh >= 4) {
            stk[sp + 2] = c[1];
            stm[sp + 2] = m[1];
        }
    }
    int next;
    if (nh > 0) {
        next = c[0];
        mask = m[0];
        sp += nh - 1;
    } else if (sp > 0) {
        --sp;
        next = stk[sp];
        mask = stm[sp];
    } else {
        next = MFX_TRAV_EXIT;
    }
    mask = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(mask >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)mask);
    return __builtin_amdgcn_readfirstlane(next);
}

// Closest hits of the wave's active lanes (act) by packet traversal; B per lane as traverse() gives.
// STATS: besides the per-lane visits (st), the wave's own fetches: wave-uniform node steps (one
// 128-B node each) and leaf slots (an 80-B test prefix each), counted on every lane alike.
// PH (diagnostic builds, -DMFX_DIAG_STAMPS=3): ph[0] += the wave's cycles in node steps, ph[1] += in
// leaf tests, ph[2] += node steps, ph[3] += leaf visits
template <bool STATS, bool PH, bool UNI>
__device__ __forceinline__ void packet_walk(const SceneView& S, DV o, DV d, const RayF& rf, uint64_t mask, Best& B,
                                            int* stk, uint64_t* stm, Stats& st, uint32_t& pk_nodes,
                                            uint32_t& pk_slots, uint64_t* ph, const PacketPlanes& pp) {
    const double tMax = B.t;
    float tlim = f_tlim(tMax);
    const int rep = __builtin_ctzll(mask);
    int sp = 0, node = 0;
    uint64_t t0 = 0;
    while (true) {
        if (PH) t0 = diag_clock();
        while (node >= 0) {
            if (STATS && ((mask >> __lane_id()) & 1)) st.nodes++;
            if (STATS) pk_nodes++;
            if (PH) ph[2]++;
            node = packet_node_step<UNI>(S.nodes, node, mask, rf, tlim, stk, stm, sp, rep, pp);
        }
        if (PH) {
            const uint64_t t1 = diag_clock();
            ph[0] += t1 - t0;
            t0 = t1;
        }
        if (node == MFX_TRAV_EXIT) return;
        if (STATS) pk_slots += (~node & 7) + 1;
        if ((mask >> __lane_id()) & 1) {  // the lanes whose ray hits the leaf's box
            leaf_hit<false, STATS, true>(S, ~node, o, d, 1e-6, tMax, B, st);
            tlim = f_tlim(B.t);
        }
        if (PH) {
            ph[1] += diag_clock() - t0;
            ph[3]++;
        }
        if (sp > 0) {
            --sp;
            node = __builtin_amdgcn_readfirstlane(stk[sp]);
            const uint64_t mm = stm[sp];
            mask = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(mm >> 32)) << 32) |
                   (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)mm);
        } else {
            return;
        }
    }
}
// the walk specialised on the packet's direction signs: one walk with the near / far columns of the
// tile's octant when its active lanes agree on every axis, the general slab test otherwise
template <bool STATS, bool PH = false>
__device__ __forceinline__ void packet_closest(const SceneView& S, bool act, DV o, DV d, double tMax, Best& B,
                                               int* stk, uint64_t* stm, Stats& st, uint32_t& pk_nodes,
                                               uint32_t& pk_slots, uint64_t* ph = nullptr) {
    B = Best{tMax, -1, -1, false};
    const RayF rf = make_rayf(o, d);
    const uint64_t mask = __ballot(act);
    if (mask == 0) return;
    const uint64_t nx = __ballot(act && rf.ix < 0.0f), ny = __ballot(act && rf.iy < 0.0f),
                   nz = __ballot(act && rf.iz < 0.0f);
    const bool uni = (nx == 0 || nx == mask) && (ny == 0 || ny == mask) && (nz == 0 || nz == mask);
    if (uni) {
        const int sx = nx ? 1 : 0, sy = ny ? 1 : 0, sz = nz ? 1 : 0;
        const PacketPlanes pp{sx, 1 - sx, 2 + sy, 3 - sy, 4 + sz, 5 - sz};
        packet_walk<STATS, PH, true>(S, o, d, rf, mask, B, stk, stm, st, pk_nodes, pk_slots, ph, pp);
    } else {
        const PacketPlanes pp{0, 1, 2, 3, 4, 5};
        packet_walk<STATS, PH, false>(S, o, d, rf, mask, B, stk, stm, st, pk_nodes, pk_slots, ph, pp);
    }
}

// Bvh.Hit over the primitive BVH4 (megakernel and query kernels). SHADOW: returns occluded
// (the reference's combine returns a hit iff some visited leaf does). Otherwise: the closest hit
// under the reference's order (Best). The stack lives in LDS, one column per lane (stride 64
// dwords: conflict-free).
// INST: a two-level scene (instances entered and left through inst_frame).
template <bool SHADOW, bool STATS, bool INST = false>
__device__ bool traverse(const SceneView& S, DV o, DV d, double tMin, double tMax, int* __restrict__ stack,
                         Best& B, Stats& st) {
    B = Best{tMax, -1, -1, false};
    RayF rf = make_rayf(o, d);
    float tlim = f_tlim(tMax);
    int sp = 0;
    int node = 0;
    int inst = -1, inst_sp = 0;
    const LdsStack stk{stack};
    while (true) {
        // ---- internal nodes ----
        while (node >= 0) {
            if (STATS) st.nodes++;
            node = node_step<false, SHADOW>(S.nodes, node, rf, tlim, stk, sp);
            if (INST) node = inst_frame(S, node, inst, inst_sp, sp, o, d, rf);
        }
        if (node == MFX_TRAV_EXIT) return B.found;
        // ---- leaf ----
        const int base = (INST && inst >= 0) ? load_inst(S, inst).slot_base : 0;
        const bool better = leaf_hit<SHADOW, STATS>(S, ~node, o, d, tMin, tMax, B, st, base);
        if (better) {
            if (SHADOW) {
                B.found = true;
                return true;
            }
            tlim = f_tlim(B.t);
        }
        if (sp == 0) return B.found;
        node = stack[(--sp) * 64];
        if (INST) node = inst_frame(S, node, inst, inst_sp, sp, o, d, rf);
    }
}

static constexpr double INVPI = 1. / 3.141592653589793;  // Material.fs:26
static constexpr double TWOPI = 2. * 3.141592653589793;  // Material.fs:27

#endif
