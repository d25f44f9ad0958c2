/*
 * mfx_oracle.c — CPU ORACLE (test infrastructure, NOT the product).
 *
 * A plain-C, FP64 restatement of NAIVEddd/MafrixRaytracing's path-tracing hot path, written to
 * follow the reference F# line by line (file:line cited on every function). It is the checker
 * for the HIP path in mafrixraytracing_amd/ and the CPU baseline timed by bench.py
 * (cpu_baseline.kind = "port"). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it; the product never links or calls it.
 *
 * PARITY STATUS: the reference cannot run here (no .NET toolchain; it has no tests, golden
 * images or fixtures — SURVEY.md §4, §8c). This oracle is pinned by hand-derived known-answer
 * tests (tests/golden/kat_*.json, tests/test_oracle_kat.py) for every function on the path; the
 * end-to-end image is otherwise "parity unpinned" against the F# binary itself.
 *
 * Deliberate, documented differences from the F# (DESIGN.md §4):
 *  - RNG: the reference draws from unseeded, racily shared System.Random instances
 *    (Integrators.fs:162, Material.fs:11, Trangle.fs:160-161, Rect.fs:34). Here every draw is a
 *    counter-based SplitMix64 value keyed by (seed, pixel, global sample, draw index) — the same
 *    stream the GPU consumes — so oracle and GPU agree path by path. Each draw is consumed in
 *    the reference's evaluation order.
 *  - The depth -1 closest-hit query whose result the reference discards (Integrators.fs:108-109
 *    with depth = -1) is skipped; it cannot change the output.
 * Everything else — FP64 arithmetic in the reference's operation order, the median-split heap BVH
 * built with .NET 6's introsort tie order, the recursive both-children traversal without tMax
 * pruning, Triangle.Hit ignoring tMax, the leaf minBy, the half-triangle light sampling, the
 * unclamped cosine, the A/dist^2 light term divided by pdf = 1/A — is reproduced as is.
 *
 * Build: oracle/Makefile (gcc -O2 -fno-fast-math -ffp-contract=off -fopenmp).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/mafrix_rt.h"

/* ------------------------------------------------------------------------------------------ */
/* Math value types — Core/Point.fs:35-68, Core/Color.fs:4-20, Core/Ray.fs:5-9                  */
/* ------------------------------------------------------------------------------------------ */
typedef struct { double x, y, z; } V3;
typedef struct { double r, g, b; } C3; /* Color; alpha is irrelevant to the RGB output */

static inline V3 v3(double x, double y, double z) { V3 v = {x, y, z}; return v; }
static inline V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }      /* Point.fs:31-32,63 */
static inline V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }      /* Point.fs:59-60 */
static inline V3 vmul(V3 v, double a) { return v3(v.x * a, v.y * a, v.z * a); }       /* Point.fs:65-66 */
static inline V3 vdiv(V3 v, double a) { return v3(v.x / a, v.y / a, v.z / a); }       /* Point.fs:67 */
static inline V3 vneg(V3 v) { return v3(-v.x, -v.y, -v.z); }                          /* Point.fs:64 */
static inline double vdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }   /* Point.fs:58 */
static inline V3 vcross(V3 a, V3 v) {                                                  /* Point.fs:57 */
    return v3(a.y * v.z - a.z * v.y, a.z * v.x - a.x * v.z, a.x * v.y - a.y * v.x);
}
static inline double vlen(V3 v) { return sqrt(v.x * v.x + v.y * v.y + v.z * v.z); }  /* Point.fs:50-51 */
static inline V3 vnormalize(V3 v) {                                                    /* Point.fs:52-56 */
    double l = vlen(v);
    if (l == 0.0) return v3(0, 0, 0);
    return v3(v.x / l, v.y / l, v.z / l);
}
static inline double vget(V3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); } /* Point.fs:43-49 */
static inline double fmin_(double x, double y) { return x < y ? x : y; }
static inline double fmax_(double x, double y) { return x > y ? x : y; }

static inline C3 c3(double r, double g, double b) { C3 c = {r, g, b}; return c; }
static inline C3 cadd(C3 l, C3 r) { return c3(l.r + r.r, l.g + r.g, l.b + r.b); }     /* Color.fs:16 */
static inline C3 cmul(C3 l, C3 r) { return c3(l.r * r.r, l.g * r.g, l.b * r.b); }     /* Color.fs:12 */
static inline C3 cscale(double l, C3 r) { return c3(l * r.r, l * r.g, l * r.b); }    /* Color.fs:13-14 */
static inline C3 cdivf(C3 l, double r) { return c3(l.r / r, l.g / r, l.b / r); }      /* Color.fs:18 */

/* ------------------------------------------------------------------------------------------ */
/* Bound — Core/Aggregate.fs:5-87                                                              */
/* ------------------------------------------------------------------------------------------ */
typedef struct { V3 pmin, pmax; } Bound;

static Bound bound2(V3 p1, V3 p2) { /* Aggregate.fs:9-11 */
    Bound b;
    b.pmin = v3(fmin_(p1.x, p2.x), fmin_(p1.y, p2.y), fmin_(p1.z, p2.z));
    b.pmax = v3(fmax_(p1.x, p2.x), fmax_(p1.y, p2.y), fmax_(p1.z, p2.z));
    return b;
}
static Bound bound_union_p(Bound b1, V3 p) { /* Aggregate.fs:54-57 */
    return bound2(v3(fmin_(b1.pmin.x, p.x), fmin_(b1.pmin.y, p.y), fmin_(b1.pmin.z, p.z)),
                  v3(fmax_(b1.pmax.x, p.x), fmax_(b1.pmax.y, p.y), fmax_(b1.pmax.z, p.z)));
}
static Bound bound_union(Bound b1, Bound b2) { /* Aggregate.fs:58-61 */
    return bound2(v3(fmin_(b1.pmin.x, b2.pmin.x), fmin_(b1.pmin.y, b2.pmin.y), fmin_(b1.pmin.z, b2.pmin.z)),
                  v3(fmax_(b1.pmax.x, b2.pmax.x), fmax_(b1.pmax.y, b2.pmax.y), fmax_(b1.pmax.z, b2.pmax.z)));
}
static int bound_max_extent(Bound b) { /* Aggregate.fs:29-36 */
    V3 d = vsub(b.pmax, b.pmin);
    if (d.x > d.y && d.x > d.z) return 0;
    else if (d.y > d.z) return 1;
    return 2;
}

/* AABB.hit — Core/Interfaces/IHitable.fs:18-54 (Williams et al. slab test) */
static int aabb_hit(V3 pmin, V3 pmax, V3 o, V3 d, double tMin, double tMax) {
    double tmin, tmax, tymin, tymax, tzmin, tzmax;
    if (d.x >= 0.) { tmin = (pmin.x - o.x) / d.x; tmax = (pmax.x - o.x) / d.x; }
    else { tmin = (pmax.x - o.x) / d.x; tmax = (pmin.x - o.x) / d.x; }
    if (d.y >= 0.) { tymin = (pmin.y - o.y) / d.y; tymax = (pmax.y - o.y) / d.y; }
    else { tymin = (pmax.y - o.y) / d.y; tymax = (pmin.y - o.y) / d.y; }
    if (tmin > tymax || tymin > tmax) return 0;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    if (d.z >= 0.) { tzmin = (pmin.z - o.z) / d.z; tzmax = (pmax.z - o.z) / d.z; }
    else { tzmin = (pmax.z - o.z) / d.z; tzmax = (pmin.z - o.z) / d.z; }
    if (tmin > tzmax || tzmin > tmax) return 0;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    return tmin < tMax && tmax > tMin;
}

/* ------------------------------------------------------------------------------------------ */
/* Shapes — Trangle.fs:98-169, Rect.fs:11-38, Sphere.fs:9-44, HitRecord.fs:5-15                */
/* ------------------------------------------------------------------------------------------ */
typedef struct { int hit; double t; V3 point; V3 normal; int material; int prim; } HitRecord;
static const HitRecord HIT_EMPTY = {0, 0.0, {0, 0, 0}, {0, 0, 0}, 0, -1};

typedef struct { V3 v0, v1, v2; double area; V3 normal; int material; Bound bound; } Triangle;

static Triangle tri_make(V3 v0, V3 v1, V3 v2, int mat) { /* Trangle.fs:107-119 */
    Triangle t;
    V3 e1 = vsub(v1, v0), e2 = vsub(v2, v0);
    V3 a = vcross(e1, e2);
    double al = vlen(a);
    t.v0 = v0; t.v1 = v1; t.v2 = v2;
    t.normal = vdiv(a, al);
    t.area = al * 0.5;
    t.material = mat;
    t.bound = bound_union_p(bound2(v0, v1), v2);
    return t;
}

/* Triangle.PreCalcu + Triangle.Hit — Trangle.fs:120-155. Note: tMax is NOT checked (:148). */
static HitRecord tri_hit(const Triangle* tr, V3 o, V3 d, double tMin, double tMax) {
    (void)tMax;
    V3 e1 = vsub(tr->v1, tr->v0), e2 = vsub(tr->v2, tr->v0);
    V3 s1 = vcross(d, e2);
    double divisor = vdot(s1, e1);
    if (fabs(divisor) < 1e-6) return HIT_EMPTY;
    double inv = 1. / divisor;
    V3 dd = vsub(o, tr->v0);
    double b1 = vdot(dd, s1) * inv;
    if (b1 < 0. || b1 > 1.) return HIT_EMPTY;
    V3 s2 = vcross(dd, e1);
    double b2 = vdot(d, s2) * inv;
    if (b2 < 0. || (b1 + b2) >= 1.) return HIT_EMPTY;
    double t = vdot(e2, s2) * inv;
    if (!(t > tMin)) return HIT_EMPTY;
    HitRecord h;
    h.hit = 1; h.t = t;
    h.point = vadd(o, vmul(d, t)); /* Ray.PointAtParameter, Ray.fs:8-9 */
    h.normal = tr->normal;
    h.material = tr->material;
    h.prim = -1;
    return h;
}

/* Triangle.SamplePoint — Trangle.fs:157-169 (reaches only half of the triangle; reproduced) */
static V3 tri_sample_point(const Triangle* tr, double tu, double tv) {
    double u = tu, v = tv;
    if (tu + tv > 1.) { u = 1. - tu; v = 1. - tv; }
    V3 e1 = vsub(tr->v1, tr->v0), e2 = vsub(tr->v2, tr->v0);
    double sq = sqrt(1. - u);
    double s1 = 1. - sq;
    double s2 = v * sq;
    return vadd(vadd(tr->v0, vmul(e1, s1)), vmul(e2, s2));
}

typedef struct { Triangle t1, t2; Bound bound; double area; } Rect;
static Rect rect_make(V3 v0, V3 v1, V3 v2, V3 v3_, int mat) { /* Rect.fs:11-20 */
    Rect r;
    r.t1 = tri_make(v0, v1, v2, mat);
    r.t2 = tri_make(v0, v2, v3_, mat);
    r.bound = bound_union(r.t1.bound, r.t2.bound);
    r.area = r.t1.area + r.t2.area;
    return r;
}
static HitRecord rect_hit(const Rect* r, V3 o, V3 d, double tMin, double tMax) { /* Rect.fs:26-31 */
    HitRecord h1 = tri_hit(&r->t1, o, d, tMin, tMax);
    if (h1.hit) return h1;
    return tri_hit(&r->t2, o, d, tMin, tMax);
}

typedef struct { V3 center; double radius; Bound bound; int material; } Sphere;
static Sphere sphere_make(V3 c, double r, int mat) { /* Sphere.fs:9-16 */
    Sphere s;
    V3 v = v3(r, r, r);
    s.center = c; s.radius = r; s.material = mat;
    s.bound = bound2(vsub(c, v), vadd(c, v));
    return s;
}
static HitRecord sphere_hit(const Sphere* s, V3 o, V3 d, double tMin, double tMax) { /* Sphere.fs:21-43 */
    V3 oc = vsub(o, s->center);
    double a = 1.;
    double b = 2.0 * vdot(oc, d);
    double c = vdot(oc, oc) - s->radius * s->radius;
    double disc = b * b - 4.0 * a * c;
    if (disc > 0) {
        double rd = sqrt(disc);
        double q = (b < 0.) ? -0.5 * (b - rd) : -0.5 * (b + rd);
        double t0 = q, t1 = c / q;
        double tmin = fmin_(t0, t1), tmax = fmax_(t0, t1);
        HitRecord h;
        if (tmin >= tMin && tmin < tMax) {
            h.hit = 1; h.t = tmin; h.point = vadd(o, vmul(d, tmin));
        } else if (tmax > tMin && tmax < tMax) {
            h.hit = 1; h.t = tmax; h.point = vadd(o, vmul(d, tmax));
        } else {
            return HIT_EMPTY;
        }
        h.normal = vnormalize(vsub(h.point, s->center));
        h.material = s->material;
        h.prim = -1;
        return h;
    }
    return HIT_EMPTY;
}

typedef struct { int kind; Triangle tri; Rect rect; Sphere sph; } Prim;

static Bound prim_bound(const Prim* p) {
    if (p->kind == MFX_PRIM_TRIANGLE) return p->tri.bound;
    if (p->kind == MFX_PRIM_RECT) return p->rect.bound;
    return p->sph.bound;
}
static HitRecord prim_hit(const Prim* p, V3 o, V3 d, double tMin, double tMax) {
    if (p->kind == MFX_PRIM_TRIANGLE) return tri_hit(&p->tri, o, d, tMin, tMax);
    if (p->kind == MFX_PRIM_RECT) return rect_hit(&p->rect, o, d, tMin, tMax);
    return sphere_hit(&p->sph, o, d, tMin, tMax);
}

/* ------------------------------------------------------------------------------------------ */
/* .NET 6 GenericArraySortHelper<double,int> introsort (System.Private.CoreLib,                 */
/* ArraySortHelper.cs) — the sort F#'s Array.sortInPlaceBy reaches with a null comparer.        */
/* Third-party algorithm not in /root/reference; restated so the median split's tie order, and  */
/* with it the leaf grouping (which the shadow-ray leaf quirk depends on), matches.             */
/* ------------------------------------------------------------------------------------------ */
static void ns_swap(double* k, int* v, int i, int j) {
    double tk = k[i]; k[i] = k[j]; k[j] = tk;
    int tv = v[i]; v[i] = v[j]; v[j] = tv;
}
static void ns_swap_if_greater(double* k, int* v, int i, int j) {
    if (k[i] > k[j]) ns_swap(k, v, i, j);
}
static void ns_insertion_sort(double* k, int* v, int n) {
    for (int i = 0; i < n - 1; i++) {
        double t = k[i + 1];
        int tv = v[i + 1];
        int j = i;
        while (j >= 0 && t < k[j]) {
            k[j + 1] = k[j];
            v[j + 1] = v[j];
            j--;
        }
        k[j + 1] = t;
        v[j + 1] = tv;
    }
}
static void ns_down_heap(double* k, int* v, int i, int n) {
    double d = k[i - 1];
    int dv = v[i - 1];
    while (i <= n >> 1) {
        int child = 2 * i;
        if (child < n && k[child - 1] < k[child]) child++;
        if (!(d < k[child - 1])) break;
        k[i - 1] = k[child - 1];
        v[i - 1] = v[child - 1];
        i = child;
    }
    k[i - 1] = d;
    v[i - 1] = dv;
}
static void ns_heap_sort(double* k, int* v, int n) {
    for (int i = n >> 1; i >= 1; i--) ns_down_heap(k, v, i, n);
    for (int i = n; i > 1; i--) {
        ns_swap(k, v, 0, i - 1);
        ns_down_heap(k, v, 1, i - 1);
    }
}
static int ns_pick_pivot_and_partition(double* k, int* v, int n) {
    int hi = n - 1;
    int middle = hi >> 1;
    ns_swap_if_greater(k, v, 0, middle);
    ns_swap_if_greater(k, v, 0, hi);
    ns_swap_if_greater(k, v, middle, hi);
    double pivot = k[middle];
    ns_swap(k, v, middle, hi - 1);
    int left = 0, right = hi - 1;
    while (left < right) {
        while (pivot > k[++left]) {}
        while (pivot < k[--right]) {}
        if (left >= right) break;
        ns_swap(k, v, left, right);
    }
    if (left != hi - 1) ns_swap(k, v, left, hi - 1);
    return left;
}
static void ns_intro_sort(double* k, int* v, int n, int depth_limit) {
    int size = n;
    while (size > 1) {
        if (size <= 16) {
            if (size == 2) { ns_swap_if_greater(k, v, 0, 1); return; }
            if (size == 3) {
                ns_swap_if_greater(k, v, 0, 1);
                ns_swap_if_greater(k, v, 0, 2);
                ns_swap_if_greater(k, v, 1, 2);
                return;
            }
            ns_insertion_sort(k, v, size);
            return;
        }
        if (depth_limit == 0) { ns_heap_sort(k, v, size); return; }
        depth_limit--;
        int p = ns_pick_pivot_and_partition(k, v, size);
        ns_intro_sort(k + p + 1, v + p + 1, size - (p + 1), depth_limit);
        size = p;
    }
}
static int ns_log2(unsigned x) { int r = 0; while (x >>= 1) r++; return r; }
/* Array.Sort<double,int>(keys, items, null) — the NaN pre-pass is a no-op for finite keys */
static void dotnet_sort(double* keys, int* items, int n) {
    if (n < 2) return;
    ns_intro_sort(keys, items, n, 2 * (ns_log2((unsigned)n) + 1));
}

/* ------------------------------------------------------------------------------------------ */
/* Bvh — Core/Accelerate/BvhNode.fs:18-83                                                      */
/* ------------------------------------------------------------------------------------------ */
typedef struct { Bound bound; int first, count; } BvhNode;
typedef struct { int n; int* indices; BvhNode* nodes; int nnodes; const Prim* prims; } Bvh;

static BvhNode bvh_init_node(const Prim* prims, const int* indices, int start, int count) { /* :32-37 */
    BvhNode nd;
    nd.bound = prim_bound(&prims[indices[start]]);
    for (int k = 1; k < count; k++) nd.bound = bound_union(nd.bound, prim_bound(&prims[indices[start + k]]));
    nd.first = start;
    nd.count = count;
    return nd;
}
static void bvh_subdivide(Bvh* b, int i, double* keybuf, int* idxbuf) { /* :42-61 */
    BvhNode node = b->nodes[i];
    if (node.count > 3) {
        int axis = bound_max_extent(node.bound);
        for (int k = 0; k < node.count; k++) {
            int pi = b->indices[node.first + k];
            Bound pb = prim_bound(&b->prims[pi]);
            V3 dig = vmul(vsub(pb.pmax, pb.pmin), 0.5);
            V3 c = vadd(pb.pmin, dig);
            keybuf[k] = vget(c, axis);
            idxbuf[k] = pi;
        }
        dotnet_sort(keybuf, idxbuf, node.count);
        memcpy(b->indices + node.first, idxbuf, sizeof(int) * node.count);
        int leftcount = node.count / 2;
        int l = 2 * i + 1, r = 2 * i + 2;
        b->nodes[l] = bvh_init_node(b->prims, b->indices, node.first, leftcount);
        b->nodes[r] = bvh_init_node(b->prims, b->indices, node.first + leftcount, node.count - leftcount);
        bvh_subdivide(b, l, keybuf, idxbuf);
        bvh_subdivide(b, r, keybuf, idxbuf);
    }
}
static int bvh_build(Bvh* b, const Prim* prims, int n) { /* :24-30 */
    if (n < 1) return -1; /* Array.zeroCreate (2N-1) with N = 0 throws in the reference */
    b->n = n;
    b->prims = prims;
    b->indices = (int*)malloc(sizeof(int) * n);
    b->nnodes = 2 * n - 1;
    b->nodes = (BvhNode*)calloc((size_t)b->nnodes, sizeof(BvhNode));
    double* keybuf = (double*)malloc(sizeof(double) * n);
    int* idxbuf = (int*)malloc(sizeof(int) * n);
    if (!b->indices || !b->nodes || !keybuf || !idxbuf) return -1;
    for (int k = 0; k < n; k++) b->indices[k] = k;
    b->nodes[0] = bvh_init_node(prims, b->indices, 0, n);
    bvh_subdivide(b, 0, keybuf, idxbuf);
    free(keybuf);
    free(idxbuf);
    return 0;
}

/* per-thread traversal counters (for the strict-mode statistics) */
typedef struct { int64_t nodes, leaves, prims; } TravStats;

/* Bvh.CheckHit — BvhNode.fs:62-82 (both children, same tMax, ties go right; leaf minBy) */
static HitRecord bvh_check_hit(const Bvh* b, V3 o, V3 d, double tMin, double tMax, int idx, TravStats* st) {
    const BvhNode* node = &b->nodes[idx];
    if (st) st->nodes++;
    if (aabb_hit(node->bound.pmin, node->bound.pmax, o, d, tMin, tMax)) {
        if (node->count > 3) {
            HitRecord l = bvh_check_hit(b, o, d, tMin, tMax, 2 * idx + 1, st);
            HitRecord r = bvh_check_hit(b, o, d, tMin, tMax, 2 * idx + 2, st);
            if (l.hit && r.hit) return (l.t < r.t) ? l : r;
            else if (l.hit) return l;
            return r;
        } else {
            /* Array.map Hit |> Array.minBy (fun h -> if h.hit then h.t else tMax): first minimum */
            HitRecord best = HIT_EMPTY;
            double bestkey = 0.0;
            if (st) { st->leaves++; st->prims += node->count; }
            for (int k = 0; k < node->count; k++) {
                int pi = b->indices[node->first + k];
                HitRecord h = prim_hit(&b->prims[pi], o, d, tMin, tMax);
                h.prim = pi;
                double key = h.hit ? h.t : tMax;
                if (k == 0 || key < bestkey) { best = h; bestkey = key; }
            }
            if (!best.hit) { best = HIT_EMPTY; }
            return best;
        }
    }
    return HIT_EMPTY;
}
static HitRecord bvh_hit(const Bvh* b, V3 o, V3 d, double tMin, double tMax, TravStats* st) { /* :83 */
    return bvh_check_hit(b, o, d, tMin, tMax, 0, st);
}

/* ------------------------------------------------------------------------------------------ */
/* "fast" mode — the CPU baseline's second figure, NOT the reference          */
/* algorithm: a 16-bin SAH BVH2 (leaves <= 4 primitives), closest hit front to back with tMax   */
/* culling and hits beyond the current best rejected, and any-hit shadow rays that stop at the  */
/* first occluder in (tMin, tMax). It shows what a conventional CPU tracer of the same         */
/* integrator does; its results can differ from "strict" where the reference's missing tMax     */
/* check in Triangle.Hit decides (the leaf quirk).                                */
/* ------------------------------------------------------------------------------------------ */
typedef struct { double lo[3], hi[3]; int first, count; } FNode; /* count > 0: leaf; else first = left child */
typedef struct { FNode* nodes; int* idx; int nnodes; } FastBvh;

static void fb_box(const Prim* prims, const int* idx, int n, double lo[3], double hi[3], int centroid) {
    for (int a = 0; a < 3; a++) { lo[a] = INFINITY; hi[a] = -INFINITY; }
    for (int k = 0; k < n; k++) {
        Bound b = prim_bound(&prims[idx[k]]);
        for (int a = 0; a < 3; a++) {
            double l = vget(b.pmin, a), h = vget(b.pmax, a);
            if (centroid) l = h = 0.5 * (l + h);
            if (l < lo[a]) lo[a] = l;
            if (h > hi[a]) hi[a] = h;
        }
    }
}
static double fb_area(const double lo[3], const double hi[3]) {
    double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return (dx < 0 || dy < 0 || dz < 0) ? 0.0 : 2.0 * (dx * dy + dy * dz + dz * dx);
}
/* A split level adds at most one stack entry in fast_hit (two pushes, one pop), so capping the
 * depth at FB_MAX_DEPTH bounds its fixed stack: a deeper range becomes one (long) leaf.        */
enum { FB_MAX_DEPTH = 100, FB_STACK = FB_MAX_DEPTH + 4 };
static int fb_build(FastBvh* f, const Prim* prims, int* idx, int first, int n, int depth) {
    const int me = f->nnodes++;
    FNode* nd = &f->nodes[me];
    fb_box(prims, idx + first, n, nd->lo, nd->hi, 0);
    double clo[3], chi[3];
    fb_box(prims, idx + first, n, clo, chi, 1);
    int axis = 0;
    for (int a = 1; a < 3; a++) if (chi[a] - clo[a] > chi[axis] - clo[axis]) axis = a;
    const double ext = chi[axis] - clo[axis];
    int best_split = -1;
    double best_cost = (double)n;
    enum { NB = 16 };
    if (n > 4 && ext > 0) {
        int cnt[NB] = {0};
        double blo[NB][3], bhi[NB][3];
        for (int b = 0; b < NB; b++) for (int a = 0; a < 3; a++) { blo[b][a] = INFINITY; bhi[b][a] = -INFINITY; }
        for (int k = 0; k < n; k++) {
            Bound bb = prim_bound(&prims[idx[first + k]]);
            double c = 0.5 * (vget(bb.pmin, axis) + vget(bb.pmax, axis));
            int b = (int)((c - clo[axis]) / ext * NB);
            if (b >= NB) b = NB - 1;
            if (b < 0) b = 0;
            cnt[b]++;
            for (int a = 0; a < 3; a++) {
                if (vget(bb.pmin, a) < blo[b][a]) blo[b][a] = vget(bb.pmin, a);
                if (vget(bb.pmax, a) > bhi[b][a]) bhi[b][a] = vget(bb.pmax, a);
            }
        }
        const double inv = 1.0 / fb_area(nd->lo, nd->hi);
        for (int sp = 1; sp < NB; sp++) {
            double llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            double rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            int nl = 0, nr = 0;
            for (int b = 0; b < NB; b++) {
                double* lo = b < sp ? llo : rlo;
                double* hi = b < sp ? lhi : rhi;
                if (b < sp) nl += cnt[b]; else nr += cnt[b];
                for (int a = 0; a < 3; a++) {
                    if (blo[b][a] < lo[a]) lo[a] = blo[b][a];
                    if (bhi[b][a] > hi[a]) hi[a] = bhi[b][a];
                }
            }
            if (!nl || !nr) continue;
            const double cost = 0.125 + (nl * fb_area(llo, lhi) + nr * fb_area(rlo, rhi)) * inv;
            if (cost < best_cost) { best_cost = cost; best_split = sp; }
        }
    }
    if (best_split < 0 && n > 8) best_split = NB / 2; /* no SAH win but too many to test: median-ish */
    if (depth >= FB_MAX_DEPTH) best_split = -1;
    if (best_split < 0) {
        nd->first = first;
        nd->count = n;
        return me;
    }
    /* partition by bin (stable enough for a baseline); fall back to halves if a side is empty */
    int mid = first;
    for (int k = first; k < first + n; k++) {
        Bound bb = prim_bound(&prims[idx[k]]);
        double c = 0.5 * (vget(bb.pmin, axis) + vget(bb.pmax, axis));
        int b = ext > 0 ? (int)((c - clo[axis]) / ext * NB) : 0;
        if (b >= NB) b = NB - 1;
        if (b < best_split) { int t = idx[k]; idx[k] = idx[mid]; idx[mid] = t; mid++; }
    }
    if (mid == first || mid == first + n) mid = first + n / 2;
    nd->count = 0;
    fb_build(f, prims, idx, first, mid - first, depth + 1);
    f->nodes[me].first = fb_build(f, prims, idx, mid, first + n - mid, depth + 1);
    return me;
}
static void fast_bvh_build(FastBvh* f, const Prim* prims, int n) {
    f->idx = (int*)malloc(sizeof(int) * (size_t)n);
    for (int k = 0; k < n; k++) f->idx[k] = k;
    f->nodes = (FNode*)calloc((size_t)(2 * n), sizeof(FNode));
    f->nnodes = 0;
    fb_build(f, prims, f->idx, 0, n, 0);
}
/* slab test with precomputed reciprocals; returns the entry distance or INFINITY */
static double fb_slab(const FNode* nd, const double o[3], const double inv[3], double tMin, double tMax) {
    double t0 = tMin, t1 = tMax;
    for (int a = 0; a < 3; a++) {
        double ta = (nd->lo[a] - o[a]) * inv[a], tb = (nd->hi[a] - o[a]) * inv[a];
        if (ta > tb) { double t = ta; ta = tb; tb = t; }
        if (ta > t0) t0 = ta;
        if (tb < t1) t1 = tb;
        if (t0 > t1) return INFINITY;
    }
    return t0;
}
static HitRecord fast_hit(const FastBvh* f, const Prim* prims, V3 o, V3 d, double tMin, double tMax, int any,
                          TravStats* st) {
    const double oo[3] = {o.x, o.y, o.z};
    const double inv[3] = {1.0 / d.x, 1.0 / d.y, 1.0 / d.z};
    HitRecord best = HIT_EMPTY;
    double tbest = tMax;
    int stack[FB_STACK], sp = 0; /* depth <= FB_MAX_DEPTH: at most depth + 2 entries */
    stack[sp++] = 0;
    while (sp) {
        const FNode* nd = &f->nodes[stack[--sp]];
        if (st) st->nodes++;
        if (fb_slab(nd, oo, inv, tMin, tbest) == INFINITY) continue;
        if (nd->count > 0) {
            if (st) { st->leaves++; st->prims += nd->count; }
            for (int k = 0; k < nd->count; k++) {
                const int pi = f->idx[nd->first + k];
                HitRecord h = prim_hit(&prims[pi], o, d, tMin, tbest);
                if (h.hit && h.t < tbest) {
                    h.prim = pi;
                    best = h;
                    tbest = h.t;
                    if (any) return best;
                }
            }
            continue;
        }
        const int l = (int)(nd - f->nodes) + 1, r = nd->first;
        const double tl = fb_slab(&f->nodes[l], oo, inv, tMin, tbest), tr = fb_slab(&f->nodes[r], oo, inv, tMin, tbest);
        if (tl <= tr) { if (tr != INFINITY) stack[sp++] = r; if (tl != INFINITY) stack[sp++] = l; }
        else { if (tl != INFINITY) stack[sp++] = l; if (tr != INFINITY) stack[sp++] = r; }
    }
    return best;
}

/* ------------------------------------------------------------------------------------------ */
/* Counter-based RNG shared with the GPU                                         */
/* ------------------------------------------------------------------------------------------ */
static inline uint64_t mix64(uint64_t z) {
    z ^= z >> 30; z *= 0xbf58476d1ce4e5b9ULL;
    z ^= z >> 27; z *= 0x94d049bb133111ebULL;
    z ^= z >> 31;
    return z;
}
typedef struct { uint64_t key; uint64_t n; } Rng;
static inline Rng rng_path(uint64_t seed, uint64_t pixel, uint64_t sample) {
    Rng r;
    r.key = mix64(seed ^ mix64((pixel << 32) | (sample & 0xffffffffULL)));
    r.n = 0;
    return r;
}
static inline double rng_next(Rng* r) { /* System.Random.NextDouble: [0,1) */
    r->n += 1;
    uint64_t z = mix64(r->key + r->n * 0x9e3779b97f4a7c15ULL);
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

/* ------------------------------------------------------------------------------------------ */
/* Camera — Core/Camera.fs:88-142                                                              */
/* ------------------------------------------------------------------------------------------ */
typedef struct { V3 position, topleft, right, down; } Pinhole;

static Pinhole pinhole_make(V3 pos, V3 dir, double fov, double aspect) {
    /* CameraCoordinate(dir) :96-104 */
    V3 fwd = vnormalize(dir);
    V3 up0 = vnormalize(v3(0, 1, 0));
    V3 hori0 = vcross(fwd, vnormalize(up0));
    V3 vert0 = vcross(hori0, fwd);
    /* PinholeCamera ctor :122-133 */
    double hori = tan(0.5 * fov * 3.141592653589793 / 360.);
    double vert = hori / aspect;
    V3 up = vmul(vert0, vert);
    V3 right = vmul(hori0, hori);
    Pinhole c;
    c.position = pos;
    c.right = right;
    c.down = vneg(up);
    /* CameraCoordinate.TopLeft(pos, 0.5) :110-111 */
    c.topleft = vadd(vsub(vadd(pos, vmul(fwd, 0.5)), vmul(right, 0.5)), vmul(up, 0.5));
    return c;
}
static void pinhole_get_ray(const Pinhole* c, double u, double v, V3* o, V3* d) { /* :134-139 */
    V3 target = vadd(vadd(c->topleft, vmul(c->right, u)), vmul(c->down, v));
    *o = c->position;
    *d = vnormalize(vsub(target, c->position));
}

/* ------------------------------------------------------------------------------------------ */
/* Scene state                                                                                 */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    int nprims;
    Prim* prims;
    Bvh bvh;
    int nmat;
    C3* albedo;
    Rect light_rect;    /* NewAreaLight.rect  Light.fs:37 */
    V3 light_normal;    /* NewAreaLight.normal */
    C3 light_color;     /* NewAreaLight.color */
    Pinhole cam;
    int width, height, max_depth;
    FastBvh fast; /* built on first use of the "fast" mode */
} OScene;

static V3 arr3(const double* p) { return v3(p[0], p[1], p[2]); }

OScene* oracle_create(const mfx_scene_desc* d) {
    if (!d || d->nprims < 1 || d->width < 1 || d->height < 1 || d->nmat < 1) return NULL;
    OScene* s = (OScene*)calloc(1, sizeof(OScene));
    s->nprims = (int)d->nprims;
    s->prims = (Prim*)calloc((size_t)s->nprims, sizeof(Prim));
    for (int i = 0; i < s->nprims; i++) {
        const mfx_prim* p = &d->prims[i];
        Prim* q = &s->prims[i];
        q->kind = p->kind;
        if (p->kind == MFX_PRIM_TRIANGLE)
            q->tri = tri_make(arr3(p->p[0]), arr3(p->p[1]), arr3(p->p[2]), p->material);
        else if (p->kind == MFX_PRIM_RECT)
            q->rect = rect_make(arr3(p->p[0]), arr3(p->p[1]), arr3(p->p[2]), arr3(p->p[3]), p->material);
        else
            q->sph = sphere_make(arr3(p->p[0]), p->p[1][0], p->material);
    }
    if (bvh_build(&s->bvh, s->prims, s->nprims) != 0) return NULL;
    s->nmat = d->nmat;
    s->albedo = (C3*)calloc((size_t)d->nmat, sizeof(C3));
    for (int m = 0; m < d->nmat; m++) s->albedo[m] = c3(d->albedo[3 * m], d->albedo[3 * m + 1], d->albedo[3 * m + 2]);
    /* NewAreaLight(p0,p1,p2,p3,nm,c): rect = Rect(p0,p1,p2,p3,0)   Light.fs:31-40 */
    s->light_rect = rect_make(arr3(d->light.p[0]), arr3(d->light.p[1]), arr3(d->light.p[2]), arr3(d->light.p[3]), 0);
    s->light_normal = arr3(d->light.normal);
    s->light_color = c3(d->light.intensity[0], d->light.intensity[1], d->light.intensity[2]);
    s->cam = pinhole_make(arr3(d->camera.position), arr3(d->camera.direction), d->camera.fov, d->camera.aspect);
    if (d->camera.derived) { /* an existing PinholeCamera's fields (Camera.fs:113-119) */
        s->cam.topleft = arr3(d->camera.topleft);
        s->cam.right = arr3(d->camera.right);
        s->cam.down = arr3(d->camera.down);
    }
    s->width = d->width;
    s->height = d->height;
    s->max_depth = d->max_depth;
    return s;
}

void oracle_destroy(OScene* s) {
    if (!s) return;
    free(s->bvh.indices);
    free(s->bvh.nodes);
    free(s->fast.nodes);
    free(s->fast.idx);
    free(s->prims);
    free(s->albedo);
    free(s);
}

/* ------------------------------------------------------------------------------------------ */
/* Integrator — Integrators.fs:19-54 (direct), 96-141 (path), 143-172 (pixel)                  */
/* ------------------------------------------------------------------------------------------ */
typedef struct { int64_t primary, extension, shadow, paths; TravStats trav; } RayCounts;

static const double INVPI = 1. / 3.141592653589793;  /* Material.fs:26 */
static const double TWOPI = 2. * 3.141592653589793;  /* Material.fs:27 */

/* GetRandomInUnitSphere(nm) — Material.fs:9-14: rejection from the unit ball, n.p > 0 */
static V3 random_in_hemisphere_ball(V3 nm, Rng* rng) {
    V3 p = v3(20, 20, 20);
    while (vdot(p, p) >= 1.0 || vdot(nm, p) <= 0.) {
        double x = rng_next(rng), y = rng_next(rng), z = rng_next(rng);
        p = vsub(vmul(v3(x, y, z), 2.0), v3(1, 1, 1));
    }
    return p;
}

/* The same distribution drawn directly (statistical check only): the rejection
 * sampler above keeps a point uniform in the unit ball with n.p > 0, whose direction is uniform on
 * the hemisphere around n; so is (cos t = u1, phi = 2 pi u2) around an orthonormal frame of n. Two
 * draws instead of ~11.5; a different sample sequence with the same expectation. */
static V3 direct_hemisphere_dir(V3 nm, Rng* rng) {
    const double z = rng_next(rng), phi = TWOPI * rng_next(rng);
    const double r = sqrt(fmax(0.0, 1.0 - z * z));
    const V3 a = fabs(nm.x) > 0.9 ? v3(0, 1, 0) : v3(1, 0, 0);
    const V3 t = vnormalize(vcross(a, nm)), b = vcross(nm, t);
    return vadd(vadd(vmul(t, r * cos(phi)), vmul(b, r * sin(phi))), vmul(nm, z));
}

/* NewAreaLight.Sample_Li / GetDirection / L — Light.fs:42-59; Rect.SamplePoint Rect.fs:33-38 */
static V3 light_sample_point(const OScene* s, Rng* rng) {
    double sel = rng_next(rng);
    const Triangle* tr = (sel < 0.5) ? &s->light_rect.t1 : &s->light_rect.t2;
    double tu = rng_next(rng);
    double tv = rng_next(rng);
    return tri_sample_point(tr, tu, tv);
}
static C3 light_L(const OScene* s, V3 toLight) {
    double cos_o = vdot(toLight, s->light_normal);
    if (cos_o < 0.) {
        double dist2 = toLight.x * toLight.x + toLight.y * toLight.y + toLight.z * toLight.z;
        double solid = fabs(cos_o) * s->light_rect.area / dist2;
        return cscale(solid, s->light_color);
    }
    return c3(0, 0, 0);
}

/* PathIntegrator.TraceRay — Integrators.fs:107-137 (recursive, as the reference) */
/* the closest-hit / shadow query of the selected mode: strict = the reference's Bvh.Hit */
static HitRecord scene_hit(const OScene* s, int fast, int shadow, V3 o, V3 d, double tMin, double tMax, TravStats* st) {
    if (fast) return fast_hit(&s->fast, s->prims, o, d, tMin, tMax, shadow, st);
    return bvh_hit(&s->bvh, o, d, tMin, tMax, st);
}

/* mode bit 0: fast traversal; bit 1: the direct hemisphere sampler (statistical check only) */
static C3 trace_ray(const OScene* s, V3 o, V3 d, int depth, Rng* rng, RayCounts* rc, int mode) {
    const int fast = mode & 1;
    if (depth < 0) return c3(0, 0, 0); /* the discarded depth -1 query (:108-109) is skipped */
    HitRecord hit = scene_hit(s, fast, 0, o, d, 1e-6, 99999999., rc ? &rc->trav : NULL);
    if (hit.hit && depth >= 0) {
        /* bxdf.SampleF — Material.fs:33-36 */
        C3 a = s->albedo[hit.material];
        V3 wi = (mode & 2) ? direct_hemisphere_dir(vnormalize(hit.normal), rng)
                           : vnormalize(random_in_hemisphere_ball(hit.normal, rng));
        double ei = vdot(hit.normal, wi);
        C3 col = cscale(TWOPI, cscale(ei, cscale(INVPI, a)));
        double pdf = 1.;
        /* SingleDirectLightIntegrator.Eval — Integrators.fs:41-52 */
        V3 lp = light_sample_point(s, rng);
        V3 toLight = vsub(lp, hit.point);
        double dist = vlen(toLight);
        double pdf_li = 1. / s->light_rect.area;
        V3 unitToLight = vdiv(toLight, dist);
        if (rc) rc->shadow++;
        HitRecord sh = scene_hit(s, fast, 1, hit.point, unitToLight, 1e-6, dist - 1e-6, rc ? &rc->trav : NULL);
        C3 l;
        if (sh.hit) l = c3(0, 0, 0);
        else l = cscale(vdot(unitToLight, hit.normal), light_L(s, toLight));
        /* (l / pdf_li + TraceRay(Ray(hit.point, wi), depth - 1)) * col / pdf   (:135-136) */
        if (rc && depth - 1 >= 0) rc->extension++;
        C3 ind = trace_ray(s, hit.point, wi, depth - 1, rng, rc, mode);
        return cdivf(cmul(cadd(cdivf(l, pdf_li), ind), col), pdf);
    }
    return c3(0, 0, 0);
}

/* One path's radiance for (pixel column i, row j, global sample) — Integrators.fs:166-170 */
static C3 render_path(const OScene* s, uint64_t seed, int i, int j, int64_t sample, RayCounts* rc, int mode) {
    Rng rng = rng_path(seed, (uint64_t)i * (uint64_t)s->height + (uint64_t)j, (uint64_t)sample);
    double u = ((double)i + rng_next(&rng)) / (double)s->width;
    double v = ((double)j + rng_next(&rng)) / (double)s->height;
    V3 o, d;
    pinhole_get_ray(&s->cam, u, v, &o, &d);
    if (rc) { rc->primary++; rc->paths++; }
    return trace_ray(s, o, d, s->max_depth, &rng, rc, mode);
}

/* PixelIntegrator.Sample(n) — Integrators.fs:161-172. frame is Color[w,h] x-major RGBA.
 * stats (optional, 8 doubles): primary, extension, shadow, paths, nodes, leaves, prims, seconds */
int oracle_sample(const OScene* s, uint64_t seed, int32_t spp, int64_t sample_base, int32_t nthreads,
                  double* frame, double* stats) {
    if (!s || spp < 1 || !frame) return -1;
    const int w = s->width, h = s->height;
    const int64_t npix = (int64_t)w * h;
    int64_t tp = 0, te = 0, ts = 0, tpaths = 0, tn = 0, tl = 0, tpr = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
    double t0 = omp_get_wtime();
#endif
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : tp, te, ts, tpaths, tn, tl, tpr)
    for (int64_t q = 0; q < npix; q++) {
        int i = (int)(q / h), j = (int)(q % h); /* Array.allPairs [0..w-1] [0..h-1] order (:156) */
        C3 color = c3(0, 0, 0);
        RayCounts rc;
        memset(&rc, 0, sizeof(rc));
        for (int sidx = 0; sidx < spp; sidx++)
            color = cadd(color, render_path(s, seed, i, j, sample_base + sidx, stats ? &rc : NULL, 0));
        C3 m = cdivf(color, (double)spp);
        frame[q * 4 + 0] = m.r;
        frame[q * 4 + 1] = m.g;
        frame[q * 4 + 2] = m.b;
        frame[q * 4 + 3] = 1.0;
        tp += rc.primary; te += rc.extension; ts += rc.shadow; tpaths += rc.paths;
        tn += rc.trav.nodes; tl += rc.trav.leaves; tpr += rc.trav.prims;
    }
    if (stats) {
        stats[0] = (double)tp; stats[1] = (double)te; stats[2] = (double)ts; stats[3] = (double)tpaths;
        stats[4] = (double)tn; stats[5] = (double)tl; stats[6] = (double)tpr;
#ifdef _OPENMP
        stats[7] = omp_get_wtime() - t0;
#else
        stats[7] = 0.0;
#endif
    }
    return 0;
}

/* Radiance of an explicit list of (pixel, sample) paths — for timing a bounded sample of a
 * workload (bench.py cpu_baseline) and for per-path parity tests. out[k*3+c].
 * mode 0 = strict (the reference algorithm), 1 = fast (SAH BVH2, tMax culling, any-hit shadows),
 * 2 = strict with the direct hemisphere sampler (the statistical check of SURVEY.md §8(c)). */
int oracle_paths_mode(OScene* s, uint64_t seed, int64_t n, const int32_t* px, const int32_t* py,
                      const int64_t* sample, int32_t nthreads, int32_t mode, double* out, double* stats) {
    if (mode == 1 && !s->fast.nodes) fast_bvh_build(&s->fast, s->prims, s->nprims);
    int64_t tp = 0, te = 0, ts = 0, tpaths = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
    double t0 = omp_get_wtime();
#endif
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : tp, te, ts, tpaths)
    for (int64_t k = 0; k < n; k++) {
        RayCounts rc;
        memset(&rc, 0, sizeof(rc));
        C3 c = render_path(s, seed, px[k], py[k], sample[k], &rc, mode);
        out[k * 3 + 0] = c.r; out[k * 3 + 1] = c.g; out[k * 3 + 2] = c.b;
        tp += rc.primary; te += rc.extension; ts += rc.shadow; tpaths += rc.paths;
    }
    if (stats) {
        stats[0] = (double)tp; stats[1] = (double)te; stats[2] = (double)ts; stats[3] = (double)tpaths;
#ifdef _OPENMP
        stats[7] = omp_get_wtime() - t0;
#endif
    }
    return 0;
}

int oracle_paths(OScene* s, uint64_t seed, int64_t n, const int32_t* px, const int32_t* py,
                 const int64_t* sample, int32_t nthreads, double* out, double* stats) {
    return oracle_paths_mode(s, seed, n, px, py, sample, nthreads, 0, out, stats);
}

/* Bvh.Hit for a batch of rays (closest hit). rays[k*6..]: origin, direction. */
int oracle_closest_hit(const OScene* s, int64_t n, const double* rays, double tmin, double tmax,
                       double* t_out, int32_t* prim_out, double* normal_out) {
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t k = 0; k < n; k++) {
        V3 o = arr3(rays + 6 * k), d = arr3(rays + 6 * k + 3);
        HitRecord h = bvh_hit(&s->bvh, o, d, tmin, tmax, NULL);
        t_out[k] = h.hit ? h.t : 0.0;
        prim_out[k] = h.hit ? h.prim : -1;
        if (normal_out) {
            normal_out[3 * k] = h.normal.x; normal_out[3 * k + 1] = h.normal.y; normal_out[3 * k + 2] = h.normal.z;
        }
    }
    return 0;
}
int oracle_any_hit(const OScene* s, int64_t n, const double* rays, double tmin, const double* tmax,
                   int32_t* occ_out) {
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t k = 0; k < n; k++) {
        V3 o = arr3(rays + 6 * k), d = arr3(rays + 6 * k + 3);
        occ_out[k] = bvh_hit(&s->bvh, o, d, tmin, tmax[k], NULL).hit ? 1 : 0;
    }
    return 0;
}

/* Heap BVH inspection: indices after Subdivide and (first,count) of every leaf in heap order */
int oracle_bvh_leaves(const OScene* s, int32_t* indices, int32_t* leaf_first, int32_t* leaf_count, int32_t* nleaves) {
    for (int k = 0; k < s->bvh.n; k++) indices[k] = s->bvh.indices[k];
    /* walk the heap: a node is used if it is the root or its parent is an internal node */
    int nl = 0;
    int* stack = (int*)malloc(sizeof(int) * 128);
    int sp = 0;
    stack[sp++] = 0;
    while (sp) {
        int i = stack[--sp];
        const BvhNode* nd = &s->bvh.nodes[i];
        if (nd->count > 3) { stack[sp++] = 2 * i + 2; stack[sp++] = 2 * i + 1; }
        else { leaf_first[nl] = nd->first; leaf_count[nl] = nd->count; nl++; }
    }
    free(stack);
    *nleaves = nl;
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Known-answer entry points (one reference function each)                                    */
/* ------------------------------------------------------------------------------------------ */
int oracle_kat_aabb(const double* pmin, const double* pmax, const double* o, const double* d, double tmin, double tmax) {
    return aabb_hit(arr3(pmin), arr3(pmax), arr3(o), arr3(d), tmin, tmax);
}
/* prim: one mfx_prim; out: t, point[3], normal[3]; returns hit flag */
int oracle_kat_prim_hit(const mfx_prim* p, const double* o, const double* d, double tmin, double tmax, double* out) {
    Prim q;
    memset(&q, 0, sizeof(q));
    q.kind = p->kind;
    if (p->kind == MFX_PRIM_TRIANGLE) q.tri = tri_make(arr3(p->p[0]), arr3(p->p[1]), arr3(p->p[2]), p->material);
    else if (p->kind == MFX_PRIM_RECT) q.rect = rect_make(arr3(p->p[0]), arr3(p->p[1]), arr3(p->p[2]), arr3(p->p[3]), p->material);
    else q.sph = sphere_make(arr3(p->p[0]), p->p[1][0], p->material);
    HitRecord h = prim_hit(&q, arr3(o), arr3(d), tmin, tmax);
    out[0] = h.t;
    out[1] = h.point.x; out[2] = h.point.y; out[3] = h.point.z;
    out[4] = h.normal.x; out[5] = h.normal.y; out[6] = h.normal.z;
    return h.hit;
}
int oracle_kat_camera_ray(const mfx_pinhole* cam, double u, double v, double* out6) {
    Pinhole c = pinhole_make(arr3(cam->position), arr3(cam->direction), cam->fov, cam->aspect);
    V3 o, d;
    pinhole_get_ray(&c, u, v, &o, &d);
    out6[0] = o.x; out6[1] = o.y; out6[2] = o.z; out6[3] = d.x; out6[4] = d.y; out6[5] = d.z;
    return 0;
}
int oracle_kat_tri_sample(const double* v0, const double* v1, const double* v2, double tu, double tv, double* out3) {
    Triangle t = tri_make(arr3(v0), arr3(v1), arr3(v2), 0);
    V3 p = tri_sample_point(&t, tu, tv);
    out3[0] = p.x; out3[1] = p.y; out3[2] = p.z;
    return 0;
}
/* light: NewAreaLight.L(hit, toLight) */
int oracle_kat_light_L(const mfx_quad_light* L, const double* toLight, double* out3) {
    OScene s;
    memset(&s, 0, sizeof(s));
    s.light_rect = rect_make(arr3(L->p[0]), arr3(L->p[1]), arr3(L->p[2]), arr3(L->p[3]), 0);
    s.light_normal = arr3(L->normal);
    s.light_color = c3(L->intensity[0], L->intensity[1], L->intensity[2]);
    C3 c = light_L(&s, arr3(toLight));
    out3[0] = c.r; out3[1] = c.g; out3[2] = c.b;
    return 0;
}
/* hemisphere sample with the shared RNG — returns the number of draws consumed */
int oracle_kat_hemisphere(const double* nm, uint64_t seed, uint64_t pixel, uint64_t sample, int32_t skip, double* out3) {
    Rng r = rng_path(seed, pixel, sample);
    for (int k = 0; k < skip; k++) rng_next(&r);
    V3 p = vnormalize(random_in_hemisphere_ball(arr3(nm), &r));
    out3[0] = p.x; out3[1] = p.y; out3[2] = p.z;
    return (int)r.n;
}
int oracle_rng_draws(uint64_t seed, uint64_t pixel, uint64_t sample, int32_t n, double* out) {
    Rng r = rng_path(seed, pixel, sample);
    for (int k = 0; k < n; k++) out[k] = rng_next(&r);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Film + post — Film.fs:13-34, Scene.fs:273-330                                               */
/* ------------------------------------------------------------------------------------------ */
static double clamp01(double x) { return x < 0. ? 0. : (x > 1. ? 1. : x); } /* Scene.fs:273 */
static C3 aces(C3 x) { /* Scene.fs:280-289: (x*(a*x+b))/(x*(c*x+d)+e), then saturate */
    const double a = 2.51, b = 0.03, c = 2.43, d = 0.59, e = 0.14;
    C3 num = cmul(x, c3(a * x.r + b, a * x.g + b, a * x.b + b));
    C3 den = c3(x.r * (c * x.r + d) + e, x.g * (c * x.g + d) + e, x.b * (c * x.b + d) + e);
    C3 col = c3(num.r / den.r, num.g / den.g, num.b / den.b);
    return c3(clamp01(col.r), clamp01(col.g), clamp01(col.b));
}
int oracle_kat_aces(const double* in3, double* out3) {
    C3 c = aces(c3(in3[0], in3[1], in3[2]));
    out3[0] = c.r; out3[1] = c.g; out3[2] = c.b;
    return 0;
}
/* Scene.PostProcessAndToScreenBuffer — Scene.fs:315-330: x-major Color[w,h] -> RGBA8 y-major */
int oracle_post_rgba8(const double* frame, int32_t w, int32_t h, uint8_t* rgba) {
    for (int x = 0; x < w; x++)
        for (int y = 0; y < h; y++) {
            const double* c = frame + ((int64_t)x * h + y) * 4;
            C3 col = aces(c3(c[0], c[1], c[2]));
            col = c3(sqrt(col.r), sqrt(col.g), sqrt(col.b));
            int ir = (int)(255.99 * col.r), ig = (int)(255.99 * col.g), ib = (int)(255.99 * col.b);
            uint8_t* o = rgba + ((int64_t)y * w + x) * 4;
            o[0] = (uint8_t)ir; o[1] = (uint8_t)ig; o[2] = (uint8_t)ib; o[3] = 255;
        }
    return 0;
}
/* Film.AddSample (Film.fs:18-23): accum += frame; frameCount += 1; target = accum / frameCount */
int oracle_film_add(double* accum, double* target, double* frame_count, const double* frame, int64_t npix) {
    *frame_count += 1.;
    for (int64_t q = 0; q < npix; q++)
        for (int c = 0; c < 3; c++) {
            double v = accum[q * 4 + c] + frame[q * 4 + c];
            accum[q * 4 + c] = v;
            target[q * 4 + c] = v / *frame_count;
        }
    for (int64_t q = 0; q < npix; q++) { accum[q * 4 + 3] = 1.0; target[q * 4 + 3] = 1.0; }
    return 0;
}

int oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
