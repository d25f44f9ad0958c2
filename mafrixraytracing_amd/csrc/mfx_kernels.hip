// mfx_kernels.hip — gfx950 (MI355X, CDNA4) kernels of the path-tracing hot path.
//
// Compiled with -ffp-contract=off: every FP64 expression below follows the reference F#'s
// operation order (cited per function) with one rounding per operation, so the device makes the
// same discrete decisions (hit / miss / which primitive / rejection accept) as the CPU oracle.
// FP32 work (the BVH2 slab tests that only *find* candidate clusters) uses explicit fmaf.
//
// Kernels
//   trace_kernel      persistent megakernel: one lane = one path; lanes whose path ends refill
//                     from a per-wave chunk of path indices (ballot + popcount compaction), so a
//                     wave stays full across bounces; chunks come from one global atomic.
//   query kernels     Bvh.Hit closest / shadow for explicit ray lists (parity tests).
//   film/post         accumulate -> mean -> ACES -> sqrt -> RGBA8 (Scene.fs:273-330, Film.fs:18-23).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mfx_layout.h"
#include "mfx_device.h"

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
    const MfxCluster* __restrict__ clusters;
    const int32_t* __restrict__ pinfo;
    const MfxSlot* __restrict__ slots;
    const MfxShade* __restrict__ shade;
    int32_t root_is_leaf;
};

struct Stats {
    uint32_t nodes, clusters, prims;
};

// One reference leaf: exact FP64 box test, then Array.minBy over its primitives with key
// (hit ? t : tMax), first minimum wins (BvhNode.fs:76-80). Returns whether the leaf's result is
// a hit; (t, slot) of that result.
template <bool STATS>
__device__ __forceinline__ bool cluster_hit(const SceneView& S, int ci, DV o, DV d, double tMin, double tMax,
                                            double& t_out, int& slot_out, int& first_out, Stats& st) {
    const MfxCluster& c = S.clusters[ci];
    if (STATS) st.clusters++;
    if (!aabb_hit64(c.lo, c.hi, o, d, tMin, tMax)) return false;
    bool best_hit = false;
    double best_key = 0.0, best_t = 0.0;
    int best_slot = -1;
    for (int k = 0; k < c.count; ++k) {
        const int info = S.pinfo[c.first + k];
        const int kind = info & 3, slot = info >> 2;
        if (STATS) st.prims++;
        double t = 0.0;
        int hs = slot;
        bool h;
        if (kind == MFX_KIND_SPHERE) {
            h = sphere_hit64(S.slots[slot], o, d, tMin, tMax, t);
        } else {
            h = tri_hit64(S.slots[slot], o, d, tMin, t);
            if (!h && kind == MFX_KIND_RECT) {  // Rect.Hit: trig1, else trig2 (Rect.fs:26-31)
                hs = slot + 1;
                h = tri_hit64(S.slots[slot + 1], o, d, tMin, t);
            }
        }
        const double key = h ? t : tMax;
        if (k == 0 || key < best_key) {
            best_key = key;
            best_hit = h;
            best_t = t;
            best_slot = hs;
        }
    }
    if (best_hit) {
        t_out = best_t;
        slot_out = best_slot;
        first_out = c.first;
    }
    return best_hit;
}

__device__ __forceinline__ float f_round_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = nextafterf(f, __builtin_inff());
    return f;
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
        if (cluster_hit<STATS>(S, 0, o, d, tMin, tMax, t, s, f, st)) {
            t_best = t;
            slot_best = s;
            return true;
        }
        return false;
    }
    // FP32 ray; tiny direction components clamped so 1/d stays finite (no 0*inf NaNs)
    float dx = (float)d.x, dy = (float)d.y, dz = (float)d.z;
    const float tiny = 1e-20f;
    if (fabsf(dx) < tiny) dx = copysignf(tiny, dx);
    if (fabsf(dy) < tiny) dy = copysignf(tiny, dy);
    if (fabsf(dz) < tiny) dz = copysignf(tiny, dz);
    const float ix = 1.0f / dx, iy = 1.0f / dy, iz = 1.0f / dz;
    const float oix = (float)o.x * ix, oiy = (float)o.y * iy, oiz = (float)o.z * iz;
    float tlim = f_round_up(tMax);
    int sp = 0;
    int node = 0;
    while (true) {
        // ---- internal nodes ----
        while (node >= 0) {
            const MfxNode nd = S.nodes[node];
            if (STATS) st.nodes++;
            float a0 = fmaf(nd.c0lox, ix, -oix), a1 = fmaf(nd.c0hix, ix, -oix);
            float b0 = fmaf(nd.c0loy, iy, -oiy), b1 = fmaf(nd.c0hiy, iy, -oiy);
            float c0 = fmaf(nd.c0loz, iz, -oiz), c1 = fmaf(nd.c0hiz, iz, -oiz);
            float n0 = fmaxf(fmaxf(fminf(a0, a1), fminf(b0, b1)), fmaxf(fminf(c0, c1), 0.0f));
            float f0 = fminf(fminf(fmaxf(a0, a1), fmaxf(b0, b1)), fminf(fmaxf(c0, c1), tlim));
            a0 = fmaf(nd.c1lox, ix, -oix); a1 = fmaf(nd.c1hix, ix, -oix);
            b0 = fmaf(nd.c1loy, iy, -oiy); b1 = fmaf(nd.c1hiy, iy, -oiy);
            c0 = fmaf(nd.c1loz, iz, -oiz); c1 = fmaf(nd.c1hiz, iz, -oiz);
            float n1 = fmaxf(fmaxf(fminf(a0, a1), fminf(b0, b1)), fmaxf(fminf(c0, c1), 0.0f));
            float f1 = fminf(fminf(fmaxf(a0, a1), fmaxf(b0, b1)), fminf(fmaxf(c0, c1), tlim));
            const bool h0 = n0 <= f0, h1 = n1 <= f1;
            if (h0 && h1) {
                int near = nd.child0, far = nd.child1;
                if (n1 < n0) { near = nd.child1; far = nd.child0; }
                stack[(sp++) * 64] = far;
                node = near;
            } else if (h0) {
                node = nd.child0;
            } else if (h1) {
                node = nd.child1;
            } else {
                if (sp == 0) return found;
                node = stack[(--sp) * 64];
            }
        }
        // ---- leaf: one reference leaf (cluster) ----
        {
            double t;
            int s, f;
            if (cluster_hit<STATS>(S, ~node, o, d, tMin, tMax, t, s, f, st)) {
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

// ----------------------------------------------------------------------------------------------
// The integrator megakernel
// ----------------------------------------------------------------------------------------------
static constexpr double INVPI = 1. / 3.141592653589793;  // Material.fs:26
static constexpr double TWOPI = 2. * 3.141592653589793;  // Material.fs:27

template <bool STATS>
__global__ void __launch_bounds__(256) trace_kernel(TraceParams P) {
    extern __shared__ int lds[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    int* stack = lds + wave * P.stack_size * 64 + lane;
    const SceneView S{P.nodes, P.clusters, P.pinfo, P.slots, P.shade, P.root_is_leaf};
    const int W = P.width, H = P.height;
    const int64_t npix = (int64_t)W * H;
    const int tiles_x = (W + 7) >> 3;
    const int64_t per_sample = (int64_t)tiles_x * ((H + 7) >> 3) * 64;
    const int64_t total = per_sample * P.nsamples;

    // path state
    bool alive = false;
    int depth = 0;
    int64_t pixel = 0;
    uint64_t key = 0;
    uint32_t rn = 0;
    DV o = dv(0, 0, 0), d = dv(0, 0, 0), T = dv(0, 0, 0), L = dv(0, 0, 0);
    uint32_t c_primary = 0, c_ext = 0, c_shadow = 0;
    Stats st{0, 0, 0};

    // per-wave work chunk (wave-uniform)
    int64_t chunk_next = 0, chunk_end = 0;
    bool exhausted = false;

    while (true) {
        // ---- refill finished lanes: ballot the lanes that need a path, hand out consecutive
        //      indices by rank (popcount of lower lanes) ----
        bool need = !alive;
        uint64_t m = __ballot(need);
        while (m != 0 && !exhausted) {
            if (chunk_next >= chunk_end) {
                int64_t base = 0;
                if (lane == 0) base = (int64_t)atomicAdd(P.work_counter, (unsigned long long)P.chunk);
                base = __shfl(base, 0);
                if (base >= total) {
                    exhausted = true;
                    break;
                }
                chunk_next = base;
                chunk_end = base + P.chunk < total ? base + P.chunk : total;
            }
            const int avail = (int)(chunk_end - chunk_next);
            const int rank = __popcll(m & ((1ULL << lane) - 1ULL));
            if (need && rank < avail) {
                const int64_t p = chunk_next + rank;
                need = false;
                // path index -> (sample, 8x8 tile, pixel); sample-major for coherent waves
                const int64_t s = p / per_sample;
                const int64_t q = p - s * per_sample;
                const int64_t tile = q >> 6;
                const int within = (int)(q & 63);
                const int x = (int)(tile % tiles_x) * 8 + (within & 7);
                const int y = (int)(tile / tiles_x) * 8 + (within >> 3);
                if (x < W && y < H) {
                    // PixelIntegrator.Sample (Integrators.fs:166-169) + PinholeCamera.GetRay (Camera.fs:134-139)
                    pixel = (int64_t)x * H + y;  // Color[w,h] x-major
                    const int64_t gsample = P.sample_base + P.part_index + s * P.part_count;
                    key = path_key(P.seed, (uint64_t)pixel, (uint64_t)gsample);
                    rn = 0;
                    const double u = ((double)x + rng_next(key, rn)) / (double)W;
                    const double v = ((double)y + rng_next(key, rn)) / (double)H;
                    const DV target = vadd(vadd(ld3(P.cam.topleft), vmul(ld3(P.cam.right), u)), vmul(ld3(P.cam.down), v));
                    o = ld3(P.cam.position);
                    d = vnormalize(vsub(target, o));
                    T = dv(1, 1, 1);
                    L = dv(0, 0, 0);
                    depth = P.max_depth;
                    alive = true;
                    c_primary++;
                }
            }
            const int took = __popcll(m) < avail ? __popcll(m) : avail;
            chunk_next += took;
            m = __ballot(need);
        }
        if (!__any(alive)) {
            if (exhausted || chunk_next >= chunk_end) {
                if (exhausted) break;
            }
            continue;
        }
        if (!alive) continue;

        // ---- closest hit: bvh.Hit(ray, 1e-6, 99999999.)  (Integrators.fs:108) ----
        double th;
        int slot;
        const bool hit = traverse<false, STATS>(S, o, d, 1e-6, 99999999., stack, th, slot, st);
        if (depth != P.max_depth) c_ext++;
        bool finish = !hit;
        if (hit) {
            const MfxShade sh = S.shade[slot];
            const DV hp = vadd(o, vmul(d, th));  // Ray.PointAtParameter (Ray.fs:8-9)
            DV nm;
            if ((sh.prim_kind & 3) == MFX_KIND_SPHERE) {
                nm = vnormalize(vsub(hp, ld3(S.slots[slot].a)));  // Sphere.fs:39-43
            } else {
                nm = ld3(sh.n);
            }
            // LambertianBrdf.SampleF — Material.fs:33-36; GetRandomInUnitSphere :9-14
            DV p = dv(20, 20, 20);
            while (vdot(p, p) >= 1.0 || vdot(nm, p) <= 0.) {
                const double rx = rng_next(key, rn);
                const double ry = rng_next(key, rn);
                const double rz = rng_next(key, rn);
                p = vsub(vmul(dv(rx, ry, rz), 2.0), dv(1, 1, 1));
            }
            const DV wi = vnormalize(p);
            const double ei = vdot(nm, wi);
            const double* a = P.albedo + 3 * sh.material;
            const DV col = dv(TWOPI * (ei * (INVPI * a[0])), TWOPI * (ei * (INVPI * a[1])), TWOPI * (ei * (INVPI * a[2])));
            // NewAreaLight.Sample_Li — Light.fs:42-47,57-59; Rect/Triangle.SamplePoint
            const double sel = rng_next(key, rn);
            const int lt = sel < 0.5 ? 0 : 1;
            const double tu = rng_next(key, rn);
            const double tv = rng_next(key, rn);
            double uu = tu, vv = tv;
            if (tu + tv > 1.) { uu = 1. - tu; vv = 1. - tv; }
            const double sq = sqrt(1. - uu);
            const double s1 = 1. - sq, s2 = vv * sq;
            const DV lp = vadd(vadd(ld3(P.light.v0[lt]), vmul(ld3(P.light.e1[lt]), s1)), vmul(ld3(P.light.e2[lt]), s2));
            const DV toLight = vsub(lp, hp);
            const double dist = vlen(toLight);
            const DV unit = vdiv(toLight, dist);
            // SingleDirectLightIntegrator.Eval — Integrators.fs:41-52
            double tsh;
            int ssh;
            const bool occluded = traverse<true, STATS>(S, hp, unit, 1e-6, dist - 1e-6, stack, tsh, ssh, st);
            c_shadow++;
            DV ld = dv(0, 0, 0);
            if (!occluded) {
                const double cos_o = vdot(toLight, ld3(P.light.normal));  // NewAreaLight.L, Light.fs:48-56
                if (cos_o < 0.) {
                    const double dist2 = toLight.x * toLight.x + toLight.y * toLight.y + toLight.z * toLight.z;
                    const double solid = fabs(cos_o) * P.light.area / dist2;
                    const double cs = vdot(unit, nm);
                    ld = dv(cs * (solid * P.light.color[0]), cs * (solid * P.light.color[1]), cs * (solid * P.light.color[2]));
                }
            }
            // (l / pdf_li + TraceRay(next)) * col / pdf, unrolled forward (Integrators.fs:135-136)
            L.x += T.x * ((ld.x / P.light.pdf) * col.x);
            L.y += T.y * ((ld.y / P.light.pdf) * col.y);
            L.z += T.z * ((ld.z / P.light.pdf) * col.z);
            T = dv(T.x * col.x, T.y * col.y, T.z * col.z);
            depth -= 1;
            if (depth < 0) {
                finish = true;  // the depth -1 query's result is discarded by the reference
            } else {
                o = hp;
                d = wi;
            }
        }
        if (finish) {
            if (L.x != 0.0) unsafeAtomicAdd(P.accum + pixel, L.x);
            if (L.y != 0.0) unsafeAtomicAdd(P.accum + npix + pixel, L.y);
            if (L.z != 0.0) unsafeAtomicAdd(P.accum + 2 * npix + pixel, L.z);
            alive = false;
        }
    }
    // ---- counters: one atomic per wave ----
    for (int off = 32; off > 0; off >>= 1) {
        c_primary += __shfl_xor(c_primary, off);
        c_ext += __shfl_xor(c_ext, off);
        c_shadow += __shfl_xor(c_shadow, off);
        if (STATS) {
            st.nodes += __shfl_xor(st.nodes, off);
            st.clusters += __shfl_xor(st.clusters, off);
            st.prims += __shfl_xor(st.prims, off);
        }
    }
    if (lane == 0) {
        atomicAdd(P.counters + 0, (unsigned long long)c_primary);
        atomicAdd(P.counters + 1, (unsigned long long)c_ext);
        atomicAdd(P.counters + 2, (unsigned long long)c_shadow);
        if (STATS) {
            atomicAdd(P.counters + 4, (unsigned long long)st.nodes);
            atomicAdd(P.counters + 5, (unsigned long long)st.clusters);
            atomicAdd(P.counters + 6, (unsigned long long)st.prims);
        }
    }
}

// ----------------------------------------------------------------------------------------------
// Query kernels (Bvh.Hit on explicit rays)
// ----------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) closest_kernel(QueryParams Q) {
    extern __shared__ int lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int* stack = lds + wave * Q.stack_size * 64 + lane;
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= Q.n) return;
    const SceneView S{Q.nodes, Q.clusters, Q.pinfo, Q.slots, Q.shade, Q.root_is_leaf};
    const DV o = ld3(Q.rays + 6 * k), d = ld3(Q.rays + 6 * k + 3);
    double t;
    int slot;
    Stats st{0, 0, 0};
    const bool h = traverse<false, false>(S, o, d, Q.tmin, Q.tmax, stack, t, slot, st);
    if (h) {
        const MfxShade sh = S.shade[slot];
        Q.t_out[k] = t;
        Q.prim_out[k] = sh.prim_kind >> 2;
        DV nm;
        if ((sh.prim_kind & 3) == MFX_KIND_SPHERE)
            nm = vnormalize(vsub(vadd(o, vmul(d, t)), ld3(S.slots[slot].a)));
        else
            nm = ld3(sh.n);
        Q.normal_out[3 * k] = nm.x;
        Q.normal_out[3 * k + 1] = nm.y;
        Q.normal_out[3 * k + 2] = nm.z;
    } else {
        Q.t_out[k] = 0.0;
        Q.prim_out[k] = -1;
        Q.normal_out[3 * k] = Q.normal_out[3 * k + 1] = Q.normal_out[3 * k + 2] = 0.0;
    }
}

__global__ void __launch_bounds__(256) anyhit_kernel(QueryParams Q) {
    extern __shared__ int lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int* stack = lds + wave * Q.stack_size * 64 + lane;
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= Q.n) return;
    const SceneView S{Q.nodes, Q.clusters, Q.pinfo, Q.slots, Q.shade, Q.root_is_leaf};
    const DV o = ld3(Q.rays + 6 * k), d = ld3(Q.rays + 6 * k + 3);
    double t;
    int slot;
    Stats st{0, 0, 0};
    Q.occ_out[k] = traverse<true, false>(S, o, d, Q.tmin, Q.tmax_per_ray[k], stack, t, slot, st) ? 1 : 0;
}

// ----------------------------------------------------------------------------------------------
// Film + post (FP64, reference order)
// ----------------------------------------------------------------------------------------------
// mean of this call's samples -> x-major RGBA doubles (texture[i,j] <- color / float n)
__global__ void mean_kernel(const double* __restrict__ accum, int64_t npix, double n, double* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= npix) return;
    out[4 * q + 0] = accum[q] / n;
    out[4 * q + 1] = accum[npix + q] / n;
    out[4 * q + 2] = accum[2 * npix + q] / n;
    out[4 * q + 3] = 1.0;
}

__device__ __forceinline__ double clamp01(double x) { return x < 0. ? 0. : (x > 1. ? 1. : x); }
__device__ __forceinline__ double aces1(double x) {  // Scene.fs:280-289
    const double a = 2.51, b = 0.03, c = 2.43, d = 0.59, e = 0.14;
    return clamp01((x * (a * x + b)) / (x * (c * x + d) + e));
}

// Film.AddSample (Film.fs:18-23) with frame = accum / spp, then PostProcessAndToScreenBuffer
// (Scene.fs:315-330) on target = film / frameCount.
__global__ void film_post_kernel(const double* __restrict__ accum, double* __restrict__ film, int w, int h,
                                 double spp, double frame_count, int add, uint8_t* __restrict__ rgba) {
    const int64_t npix = (int64_t)w * h;
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= npix) return;
    double tgt[3];
    for (int c = 0; c < 3; ++c) {
        double v = film[c * npix + q];
        if (add) {
            v = v + accum[c * npix + q] / spp;
            film[c * npix + q] = v;
        }
        tgt[c] = v / frame_count;
    }
    if (rgba) {
        const int x = (int)(q / h), y = (int)(q % h);
        uint8_t* o = rgba + ((int64_t)y * w + x) * 4;
        for (int c = 0; c < 3; ++c) o[c] = (uint8_t)(int)(255.99 * sqrt(aces1(tgt[c])));
        o[3] = 255;
    }
}

__global__ void film_mean_kernel(const double* __restrict__ film, int64_t npix, double frame_count, double* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= npix) return;
    for (int c = 0; c < 3; ++c) out[4 * q + c] = frame_count > 0 ? film[c * npix + q] / frame_count : 0.0;
    out[4 * q + 3] = 1.0;
}

__global__ void fp64_selftest_kernel(const double* a, const double* b, int64_t n, double* dv_out, double* sq_out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    dv_out[k] = a[k] / b[k];
    sq_out[k] = sqrt(a[k]);
}

// ----------------------------------------------------------------------------------------------
// Host-side launchers (called from mfx_api.cpp)
// ----------------------------------------------------------------------------------------------
static inline unsigned grid_for(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

hipError_t mfx_launch_trace(const TraceParams& P, bool stats, int grid, hipStream_t st) {
    const size_t lds = (size_t)4 * P.stack_size * 64 * sizeof(int);
    if (stats)
        hipLaunchKernelGGL(trace_kernel<true>, dim3(grid), dim3(256), lds, st, P);
    else
        hipLaunchKernelGGL(trace_kernel<false>, dim3(grid), dim3(256), lds, st, P);
    return hipGetLastError();
}

hipError_t mfx_trace_occupancy(int stack_size, int* blocks_per_cu) {
    const size_t lds = (size_t)4 * stack_size * 64 * sizeof(int);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, trace_kernel<false>, 256, lds);
}

hipError_t mfx_launch_query(const QueryParams& Q, bool shadow, hipStream_t st) {
    const size_t lds = (size_t)4 * Q.stack_size * 64 * sizeof(int);
    if (shadow)
        hipLaunchKernelGGL(anyhit_kernel, dim3(grid_for(Q.n, 256)), dim3(256), lds, st, Q);
    else
        hipLaunchKernelGGL(closest_kernel, dim3(grid_for(Q.n, 256)), dim3(256), lds, st, Q);
    return hipGetLastError();
}

hipError_t mfx_launch_mean(const double* accum, int64_t npix, double n, double* out, hipStream_t st) {
    hipLaunchKernelGGL(mean_kernel, dim3(grid_for(npix, 256)), dim3(256), 0, st, accum, npix, n, out);
    return hipGetLastError();
}

hipError_t mfx_launch_film_post(const double* accum, double* film, int w, int h, double spp, double frame_count,
                                int add, uint8_t* rgba, hipStream_t st) {
    const int64_t npix = (int64_t)w * h;
    hipLaunchKernelGGL(film_post_kernel, dim3(grid_for(npix, 256)), dim3(256), 0, st, accum, film, w, h, spp,
                       frame_count, add, rgba);
    return hipGetLastError();
}

hipError_t mfx_launch_film_mean(const double* film, int64_t npix, double frame_count, double* out, hipStream_t st) {
    hipLaunchKernelGGL(film_mean_kernel, dim3(grid_for(npix, 256)), dim3(256), 0, st, film, npix, frame_count, out);
    return hipGetLastError();
}

hipError_t mfx_launch_fp64_selftest(const double* a, const double* b, int64_t n, double* dvo, double* sqo, hipStream_t st) {
    hipLaunchKernelGGL(fp64_selftest_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, a, b, n, dvo, sqo);
    return hipGetLastError();
}
