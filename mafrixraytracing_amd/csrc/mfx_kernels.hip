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

#include <algorithm>
#include <cstdlib>
#include <stdint.h>

#include "mfx_layout.h"
#include "mfx_device.h"
#include "mfx_trace_common.h"


// ----------------------------------------------------------------------------------------------
// The integrator megakernel
// ----------------------------------------------------------------------------------------------
// WAVES: the register budget, as minimum waves per SIMD: 1 (no limit: ~152 VGPRs, 3 waves) or 4
// (128 VGPRs, ~90 B of spills per lane). Measured at one sample per pixel (r02as): 4 waves C2
// +2.4 %, C5 +9.8 %, C4 -3.4 % (the deep stack: bound 44); mfx_api picks 4 for bounds <= 36.
template <bool STATS, bool INST, int WAVES>
__global__ void __launch_bounds__(256, WAVES) trace_kernel(TraceParams P) {
    // one traversal-stack column per lane in LDS. (The top BVH levels in LDS, as the wavefront
    // kernels keep them, measured -21 % here at 1 spp, r02i: the per-node LDS/global branch.)
    extern __shared__ int lds[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    int* stack = lds + wave * P.stack_size * 64 + lane;
    const SceneView S{P.nodes, P.slots, P.slot_ref, P.ref_blob, P.inst, nullptr, 0};
    const MfxLight& LT = P.light;
    const MfxCamera& CAM = P.cam;
    const int W = P.width, H = P.height;
    const int64_t npix = (int64_t)W * H;
    const int tiles_x = (W + 7) >> 3;
    const int64_t per_sample = (int64_t)tiles_x * P.band_rows * 64;  // the band's tile rows (image partition)
    const int64_t total = per_sample * P.nsamples;

    // path state. A vertex's direct term a_v and col c_v go to this lane's scratch column and are
    // folded back to the camera when the path ends, in the reference's recursion order (see k_resolve)
    bool alive = false;
    int depth = 0;
    int lit = 0;  // bit v: vertex v's a_v is recorded
    int64_t pixel = 0;
    uint64_t key = 0;
    uint32_t rn = 0;
    DV o = dv(0, 0, 0), d = dv(0, 0, 0);
    const int64_t vstride = (int64_t)gridDim.x * blockDim.x;
    double* const vs = P.vscratch + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // [v][a/c][rgb][vstride]
    uint32_t c_primary = 0, c_ext = 0, c_shadow = 0;
    Stats st{0, 0, 0}, st2{0, 0, 0};

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
                const int y = band_tile_row(P.band_index, P.band_count, (int)(tile / tiles_x)) * 8 + (within >> 3);
                if (x < W && y < H) {
                    // PixelIntegrator.Sample (Integrators.fs:166-169) + PinholeCamera.GetRay (Camera.fs:134-139)
                    pixel = (int64_t)x * H + y;  // Color[w,h] x-major
                    const int64_t gsample = P.sample_base + P.part_index + s * P.part_count;
                    key = path_key(P.seed, (uint64_t)pixel, (uint64_t)gsample);
                    rn = 0;
                    const double u = ((double)x + rng_next(key, rn)) / (double)W;
                    const double v = ((double)y + rng_next(key, rn)) / (double)H;
                    const DV target = vadd(vadd(ld3(CAM.topleft), vmul(ld3(CAM.right), u)), vmul(ld3(CAM.down), v));
                    o = ld3(CAM.position);
                    d = vnormalize(vsub(target, o));
                    lit = 0;
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
        Best hb;
        const bool hit = traverse<false, STATS, INST>(S, o, d, 1e-6, 99999999., stack, hb, st);
        const double th = hb.t;
        const int slot = hb.info & MFX_INFO_SHADE_MASK;
        if (depth != P.max_depth) c_ext++;
        bool finish = !hit;
        if (hit) {
            const MfxShade sh = P.shade[slot];
            const DV hp = vadd(o, vmul(d, th));  // Ray.PointAtParameter (Ray.fs:8-9)
            DV nm;
            if ((sh.prim_kind & 3) == MFX_KIND_SPHERE) {
                nm = vnormalize(vsub(hp, ld3(sh.n)));  // Sphere.fs:39-43
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
            const double* a = sh.albedo;
            const int v = P.max_depth - depth;  // this vertex's index
            double* vrec = vs + (int64_t)(6 * v) * vstride;
            vrec[3 * vstride] = TWOPI * (ei * (INVPI * a[0]));  // c_v = col (Material.fs:36)
            vrec[4 * vstride] = TWOPI * (ei * (INVPI * a[1]));
            vrec[5 * vstride] = TWOPI * (ei * (INVPI * a[2]));
            // NewAreaLight.Sample_Li — Light.fs:42-47,57-59; Rect/Triangle.SamplePoint
            const double sel = rng_next(key, rn);
            const int lt = sel < 0.5 ? 0 : 1;
            const double tu = rng_next(key, rn);
            const double tv = rng_next(key, rn);
            double uu = tu, vv = tv;
            if (tu + tv > 1.) { uu = 1. - tu; vv = 1. - tv; }
            const double sq = sqrt(1. - uu);
            const double s1 = 1. - sq, s2 = vv * sq;
            const DV lv0 = lt ? ld3(LT.v0[1]) : ld3(LT.v0[0]);
            const DV le1 = lt ? ld3(LT.e1[1]) : ld3(LT.e1[0]);
            const DV le2 = lt ? ld3(LT.e2[1]) : ld3(LT.e2[0]);
            const DV lp = vadd(vadd(lv0, vmul(le1, s1)), vmul(le2, s2));
            const DV toLight = vsub(lp, hp);
            const double dist = vlen(toLight);
            const DV unit = vdiv(toLight, dist);
            // NewAreaLight.L (Light.fs:48-56) and the cosine (Integrators.fs:52) depend only on the
            // sample, so they are formed before the shadow query: less state lives across it.
            const double cos_o = vdot(toLight, ld3(LT.normal));
            const double dist2 = toLight.x * toLight.x + toLight.y * toLight.y + toLight.z * toLight.z;
            const double solid = fabs(cos_o) * LT.area / dist2;
            const double cs = vdot(unit, nm);
            const bool lightable = cos_o < 0.;
            // SingleDirectLightIntegrator.Eval — Integrators.fs:41-52
            Best sb;
            const bool occluded = traverse<true, STATS, INST>(S, hp, unit, 1e-6, dist - 1e-6, stack, sb, st2);
            c_shadow++;
            if (!occluded && lightable) {  // a_v = l / pdf_li
                vrec[0] = (cs * (solid * LT.color[0])) / LT.pdf;
                vrec[vstride] = (cs * (solid * LT.color[1])) / LT.pdf;
                vrec[2 * vstride] = (cs * (solid * LT.color[2])) / LT.pdf;
                lit |= 1 << v;
            }
            depth -= 1;
            if (depth < 0) {
                finish = true;  // the depth -1 query's result is discarded by the reference
            } else {
                o = hp;
                d = wi;
            }
        }
        if (finish) {
            if (lit) {  // (l / pdf_li + TraceRay(next)) * col / pdf, deepest lit vertex first (Integrators.fs:136)
                double fx = 0.0, fy = 0.0, fz = 0.0;
                for (int v = 31 - __builtin_clz(lit); v >= 0; --v) {
                    const double* vv = vs + (int64_t)(6 * v) * vstride;
                    const bool l = (lit >> v) & 1;
                    fx = ((l ? vv[0] : 0.0) + fx) * vv[3 * vstride];
                    fy = ((l ? vv[vstride] : 0.0) + fy) * vv[4 * vstride];
                    fz = ((l ? vv[2 * vstride] : 0.0) + fz) * vv[5 * vstride];
                }
                // one path per pixel and call (Scene.Render): the add onto the zeroed accumulator is exact
                if (fx != 0.0) unsafeAtomicAdd(P.accum + pixel, fx);
                if (fy != 0.0) unsafeAtomicAdd(P.accum + npix + pixel, fy);
                if (fz != 0.0) unsafeAtomicAdd(P.accum + 2 * npix + pixel, fz);
            }
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
            st2.nodes += __shfl_xor(st2.nodes, off);
            st2.clusters += __shfl_xor(st2.clusters, off);
            st2.prims += __shfl_xor(st2.prims, off);
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
            atomicAdd(P.counters + 7, (unsigned long long)st2.nodes);
            atomicAdd(P.counters + 8, (unsigned long long)st2.clusters);
            atomicAdd(P.counters + 9, (unsigned long long)st2.prims);
        }
    }
}

// ----------------------------------------------------------------------------------------------
// Query kernels (Bvh.Hit on explicit rays)
// ----------------------------------------------------------------------------------------------
template <bool INST>
__global__ void __launch_bounds__(256) closest_kernel(QueryParams Q) {
    extern __shared__ int lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int* stack = lds + wave * Q.stack_size * 64 + lane;
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= Q.n) return;
    const SceneView S{Q.nodes, Q.slots, Q.slot_ref, Q.ref_blob, Q.inst, nullptr, 0};
    const DV o = ld3(Q.rays + 6 * k), d = ld3(Q.rays + 6 * k + 3);
    Best B;
    Stats st{0, 0, 0};
    const bool h = traverse<false, false, INST>(S, o, d, Q.tmin, Q.tmax, stack, B, st);
    const double t = B.t;
    const int slot = B.info & MFX_INFO_SHADE_MASK;
    if (h) {
        const MfxShade sh = Q.shade[slot];
        Q.t_out[k] = t;
        Q.prim_out[k] = sh.prim_kind >> 2;
        DV nm;
        if ((sh.prim_kind & 3) == MFX_KIND_SPHERE)
            nm = vnormalize(vsub(vadd(o, vmul(d, t)), ld3(sh.n)));
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

template <bool INST>
__global__ void __launch_bounds__(256) anyhit_kernel(QueryParams Q) {
    extern __shared__ int lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int* stack = lds + wave * Q.stack_size * 64 + lane;
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= Q.n) return;
    const SceneView S{Q.nodes, Q.slots, Q.slot_ref, Q.ref_blob, Q.inst, nullptr, 0};
    const DV o = ld3(Q.rays + 6 * k), d = ld3(Q.rays + 6 * k + 3);
    Best B;
    Stats st{0, 0, 0};
    Q.occ_out[k] = traverse<true, false, INST>(S, o, d, Q.tmin, Q.tmax_per_ray[k], stack, B, st) ? 1 : 0;
}

#ifndef MFX_EXPERIMENT_PACKET16
#define MFX_EXPERIMENT_PACKET16 0  // the variant build only (Makefile `experiments`: build_variants/pk16.so)
#endif
#if MFX_EXPERIMENT_PACKET16
// Measured and lost (2.9x slower than one ray per lane), so not in the shipped library:
// Experiment (VERDICT r04 Next #4a; MFX_ANYHIT_PACKET=16 switches mfx_any_hit to it): the any-hit
// query traced as four 16-lane sub-packets per wave. A sub-packet walks the BVH4 together: its
// lanes load the same node (per-lane loads of one address), each tests the four children with its
// own FP32 ray and limit, a child is visited when some live lane of the sub-packet hits it, far to
// near by the exit distances of the sub-packet's first live lane, and the stack (node + the 64-bit
// mask of the lanes whose own test hit it, only this sub-packet's 16 bits set) is the sub-packet's,
// in LDS. A lane tests exactly the leaves its own ray's box tests reach, as its single-ray walk
// would (child boxes lie inside their parents'), and leaves its sub-packet once occluded; whether a
// ray is occluded does not depend on the visit order (node_step's FAR note), so every answer is the
// single-ray kernel's (tests/test_gpu_edge_parity.py). STATS: wave node steps and leaf rounds in
// steps[0], steps[1] (one count per wave iteration), per-lane visits in steps[2], steps[3].
template <bool STATS>
__global__ void __launch_bounds__(256) anyhit_packet16_kernel(QueryParams Q, unsigned long long* steps) {
    extern __shared__ int lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
    const uint64_t gbits = 0xffffULL << (16 * g);
    int* stk = lds + (wave * 4 + g) * Q.stack_size * 3;  // per entry: node, mask low, mask high
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = k < Q.n;
    const SceneView S{Q.nodes, Q.slots, Q.slot_ref, Q.ref_blob, Q.inst, nullptr, 0};
    DV o = dv(0, 0, 0), d = dv(0, 0, 1);
    double tmax = 0.0;
    if (act) {
        o = ld3(Q.rays + 6 * k);
        d = ld3(Q.rays + 6 * k + 3);
        tmax = Q.tmax_per_ray[k];
    }
    const RayF rf = make_rayf(o, d);
    const float tlim = f_tlim(tmax);
    bool alive = act;  // not (yet) found occluded
    bool occ = false;
    uint64_t mask = __ballot(alive) & gbits;  // sub-packet-uniform: its lanes whose test hit `node`
    int node = mask ? 0 : MFX_TRAV_EXIT, sp = 0;
    Best B;
    Stats st{0, 0, 0};
    uint32_t w_nodes = 0, w_leaves = 0;
    while (__any(node != MFX_TRAV_EXIT)) {
        const bool mine = ((mask >> lane) & 1) && alive;
        bool pop = false;
        if (node >= 0) {  // the sub-packet's node step
            if (STATS) w_nodes += lane == 0 ? 1 : 0;
            if (STATS && mine) st.nodes++;
            const float4* __restrict__ q = (const float4*)(Q.nodes + node);
            const float4 lx = q[0], hx = q[1], ly = q[2], hy = q[3], lz = q[4], hz = q[5];
            const int4 ch = *(const int4*)(q + 6);
            Slab4 SL;
            slab4(lx, hx, ly, hy, lz, hz, rf, SL);
            const uint64_t live = __ballot(alive) & gbits;
            const int rep = __builtin_ctzll((mask & live) | (1ULL << (16 * g)));  // the sub-packet's first live lane
            float dk[4];
            int c[4] = {ch.x, ch.y, ch.z, ch.w};
            uint64_t m[4];
            int nh = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float n = fmaxf(fmaxf(fminf(SL.a0[j], SL.a1[j]), fminf(SL.b0[j], SL.b1[j])), fmaxf(fminf(SL.c0[j], SL.c1[j]), 0.0f));
                const float f = fminf(fminf(fmaxf(SL.a0[j], SL.a1[j]), fmaxf(SL.b0[j], SL.b1[j])), fminf(fmaxf(SL.c0[j], SL.c1[j]), tlim));
                const bool h = mine && n <= f;
                m[j] = __ballot(h) & gbits;
                const float kd = __shfl(h ? -f : 3.0e38f, rep);  // far first: the representative's exit
                dk[j] = m[j] ? kd : __builtin_inff();
                nh += m[j] ? 1 : 0;
            }
            cswap3(dk[0], c[0], m[0], dk[1], c[1], m[1]);
            cswap3(dk[2], c[2], m[2], dk[3], c[3], m[3]);
            cswap3(dk[0], c[0], m[0], dk[2], c[2], m[2]);
            cswap3(dk[1], c[1], m[1], dk[3], c[3], m[3]);
            cswap3(dk[1], c[1], m[1], dk[2], c[2], m[2]);
            if (lane == 16 * g) {  // far-first pushes, one lane per sub-packet
                for (int j = nh - 1; j >= 1; --j) {
                    int* e = stk + 3 * (sp + nh - 1 - j);
                    e[0] = c[j];
                    e[1] = (int)(uint32_t)m[j];
                    e[2] = (int)(uint32_t)(m[j] >> 32);
                }
            }
            if (nh > 0) {
                sp += nh - 1;
                node = c[0];
                mask = m[0];
            } else {
                pop = true;
            }
        } else if (node != MFX_TRAV_EXIT) {  // a leaf: its live lanes test it (any hit)
            if (STATS) w_leaves += lane == 0 ? 1 : 0;
            if (mine && leaf_hit<true, STATS>(S, ~node, o, d, Q.tmin, tmax, B, st)) {
                occ = true;
                alive = false;
            }
            pop = true;
        }
        if (pop) {  // the next entry with a live lane, or the end of the sub-packet's walk
            const uint64_t live = __ballot(alive) & gbits;
            node = MFX_TRAV_EXIT;
            while (sp > 0) {
                --sp;
                const int* e = stk + 3 * sp;
                const uint64_t mm = ((uint64_t)(uint32_t)e[2] << 32) | (uint32_t)e[1];
                if (mm & live) {
                    node = e[0];
                    mask = mm & live;
                    break;
                }
            }
        }
    }
    if (act) Q.occ_out[k] = occ ? 1 : 0;
    if (STATS && steps) {
        if (lane == 0) {
            atomicAdd(steps + 0, (unsigned long long)w_nodes);
            atomicAdd(steps + 1, (unsigned long long)w_leaves);
        }
        atomicAdd(steps + 2, (unsigned long long)st.nodes);
        atomicAdd(steps + 3, (unsigned long long)st.clusters);
    }
}
#endif  // MFX_EXPERIMENT_PACKET16

// ----------------------------------------------------------------------------------------------
// Film + post (FP64, reference order)
// ----------------------------------------------------------------------------------------------
// mean of this call's samples -> x-major RGBA doubles (texture[i,j] <- color / float n)
// (pixels [p0, p1) only: mfx_sample's banded readback)
__global__ void mean_kernel(const double* __restrict__ accum, int64_t npix, double n, double* __restrict__ out,
                            int64_t p0, int64_t p1) {
    const int64_t q = p0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= p1) return;
    // two 16-B stores per pixel (a wave writes 2 KB in order: whole lines, also when `out` is
    // page-locked host memory written across the fabric, mfx_sample's zero-copy readback)
    double2* o = (double2*)out + 2 * q;
    o[0] = make_double2(accum[q] / n, accum[npix + q] / n);
    o[1] = make_double2(accum[2 * npix + q] / n, 1.0);
}

// the same means as interleaved RGB: the alpha channel (1.0) is the host's to write, so the readback
// carries three quarters of the bytes
__global__ void mean_rgb_kernel(const double* __restrict__ accum, int64_t npix, double n, double* __restrict__ out,
                                int64_t p0, int64_t p1) {
    const int64_t q = p0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= p1) return;
    double* o = out + 3 * q;
    o[0] = accum[q] / n;
    o[1] = accum[npix + q] / n;
    o[2] = accum[2 * npix + q] / n;
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
        for (int c = 0; c < 3; ++c) o[c] = post_byte(tgt[c]);
        o[3] = 255;
    }
}

__global__ void film_mean_kernel(const double* __restrict__ film, int64_t npix, double frame_count, double* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= npix) return;
    for (int c = 0; c < 3; ++c) out[4 * q + c] = frame_count > 0 ? film[c * npix + q] / frame_count : 0.0;
    out[4 * q + 3] = 1.0;
}

// dst += src, element-wise: one device's accumulator added into another's (the in-order device
// reduce of a context whose device list repeats a device, where RCCL cannot form a communicator)
__global__ void accum_add_kernel(double* __restrict__ dst, const double* __restrict__ src, int64_t n) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) dst[k] = dst[k] + src[k];
}

// a trace's ray / traversal counters added to the context's running totals (mfx_ray_counts_total):
// stream-ordered, so back-to-back traces need no host read in between
__global__ void counters_add_kernel(unsigned long long* __restrict__ total, const unsigned long long* __restrict__ c, int n) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) total[k] += c[k];
}

__global__ void fp64_selftest_kernel(const double* a, const double* b, int64_t n, double* dv_out, double* sq_out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    dv_out[k] = a[k] / b[k];
    sq_out[k] = sqrt(a[k]);
}

// The exact shortcuts in front of the reference-leaf box test against aabb_hit64 (AABB.hit,
// IHitable.fs:18-54): rec = 24 doubles per case (lo, hi, o, d, tMin, tMax, then a triangle v0, e1,
// e2 whose vertex box lies in [lo, hi], one pad); out = 3 per case: the FP64 test's answer (0/1),
// aabb_screen32's (1, 0 or -1 when it leaves the case to the FP64 test) and tri_box_pass's (1
// proved to pass, 0 not proved)
__global__ void aabb_selftest_kernel(const double* rec, int64_t n, int32_t* out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double* r = rec + 24 * k;
    const DV o = ld3(r + 6), d = ld3(r + 9);
    out[3 * k] = aabb_hit64(r, r + 3, o, d, r[12], r[13]) ? 1 : 0;
    out[3 * k + 1] = aabb_screen32(r, r + 3, o, d, r[12], r[13]);
    out[3 * k + 2] = tri_box_pass(ld3(r + 14), ld3(r + 17), ld3(r + 20), o, d, r[12], r[13]) ? 1 : 0;
}

// ----------------------------------------------------------------------------------------------
// Host-side launchers (called from mfx_api.cpp)
// ----------------------------------------------------------------------------------------------
static inline unsigned grid_for(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

static size_t trace_lds_bytes(int stack_size) { return (size_t)4 * stack_size * 64 * sizeof(int); }

hipError_t mfx_launch_trace(const TraceParams& P, bool stats, int grid, hipStream_t st) {
    const size_t lds = trace_lds_bytes(P.stack_size);
    if (P.waves == 4) {
        if (P.inst) {
            if (stats) hipLaunchKernelGGL((trace_kernel<true, true, 4>), dim3(grid), dim3(256), lds, st, P);
            else hipLaunchKernelGGL((trace_kernel<false, true, 4>), dim3(grid), dim3(256), lds, st, P);
        } else {
            if (stats) hipLaunchKernelGGL((trace_kernel<true, false, 4>), dim3(grid), dim3(256), lds, st, P);
            else hipLaunchKernelGGL((trace_kernel<false, false, 4>), dim3(grid), dim3(256), lds, st, P);
        }
    } else {
        if (P.inst) {
            if (stats) hipLaunchKernelGGL((trace_kernel<true, true, 1>), dim3(grid), dim3(256), lds, st, P);
            else hipLaunchKernelGGL((trace_kernel<false, true, 1>), dim3(grid), dim3(256), lds, st, P);
        } else {
            if (stats) hipLaunchKernelGGL((trace_kernel<true, false, 1>), dim3(grid), dim3(256), lds, st, P);
            else hipLaunchKernelGGL((trace_kernel<false, false, 1>), dim3(grid), dim3(256), lds, st, P);
        }
    }
    return hipGetLastError();
}

hipError_t mfx_trace_occupancy(int stack_size, int* blocks_per_cu, bool inst, int waves) {
    const size_t lds = trace_lds_bytes(stack_size);
    const void* k = waves == 4 ? (inst ? (const void*)trace_kernel<false, true, 4> : (const void*)trace_kernel<false, false, 4>)
                               : (inst ? (const void*)trace_kernel<false, true, 1> : (const void*)trace_kernel<false, false, 1>);
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k, 256, lds);
    // gfx950 allocates LDS in 1,280-byte granules of its 160 KB (the API counts finer ones)
    const size_t g = 1280;
    *blocks_per_cu = std::min(*blocks_per_cu, (int)(160 * 1024 / ((lds + g - 1) / g * g)));
    return e;
}

hipError_t mfx_launch_query(const QueryParams& Q, bool shadow, hipStream_t st) {
    const size_t lds = (size_t)4 * Q.stack_size * 64 * sizeof(int);
    const dim3 g(grid_for(Q.n, 256));
    if (shadow) {
#if MFX_EXPERIMENT_PACKET16
        const char* pk = getenv("MFX_ANYHIT_PACKET");  // the sub-packet experiment (flat scenes)
        if (pk && atoi(pk) == 16 && !Q.inst)
            hipLaunchKernelGGL(anyhit_packet16_kernel<false>, g, dim3(256), (size_t)16 * Q.stack_size * 3 * sizeof(int),
                               st, Q, nullptr);
        else
#endif
        if (Q.inst) hipLaunchKernelGGL(anyhit_kernel<true>, g, dim3(256), lds, st, Q);
        else hipLaunchKernelGGL(anyhit_kernel<false>, g, dim3(256), lds, st, Q);
    } else {
        if (Q.inst) hipLaunchKernelGGL(closest_kernel<true>, g, dim3(256), lds, st, Q);
        else hipLaunchKernelGGL(closest_kernel<false>, g, dim3(256), lds, st, Q);
    }
    return hipGetLastError();
}

hipError_t mfx_launch_mean(const double* accum, int64_t npix, double n, double* out, hipStream_t st, int64_t p0,
                           int64_t p1) {
    if (p1 < 0) p1 = npix;
    if (p1 <= p0) return hipSuccess;
    hipLaunchKernelGGL(mean_kernel, dim3(grid_for(p1 - p0, 256)), dim3(256), 0, st, accum, npix, n, out, p0, p1);
    return hipGetLastError();
}

hipError_t mfx_launch_mean_rgb(const double* accum, int64_t npix, double n, double* out, hipStream_t st, int64_t p0,
                               int64_t p1) {
    if (p1 <= p0) return hipSuccess;
    hipLaunchKernelGGL(mean_rgb_kernel, dim3(grid_for(p1 - p0, 256)), dim3(256), 0, st, accum, npix, n, out, p0, p1);
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

hipError_t mfx_launch_aabb_selftest(const double* rec, int64_t n, int32_t* out, hipStream_t st) {
    hipLaunchKernelGGL(aabb_selftest_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, rec, n, out);
    return hipGetLastError();
}

hipError_t mfx_launch_counters_add(unsigned long long* total, const unsigned long long* c, int n, hipStream_t st) {
    hipLaunchKernelGGL(counters_add_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, total, c, n);
    return hipGetLastError();
}

hipError_t mfx_launch_accum_add(double* dst, const double* src, int64_t n, hipStream_t st) {
    hipLaunchKernelGGL(accum_add_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, dst, src, n);
    return hipGetLastError();
}
