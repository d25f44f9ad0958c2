// mfx_wavefront.hip — wavefront path tracing on gfx950: the integrator loop
// (Integrators.fs:107-137, 161-172) split into four kernels over a pool of path slots:
//
//   k_logic    DONE slots -> FP64 atomic add of L into the pixel sums; FREE slots take new path
//              indices (block-aggregated allocation from 8 sharded counters) and generate camera
//              rays (PixelIntegrator.Sample + PinholeCamera.GetRay)
//   k_traverse<closest>  persistent bvh.Hit(ray, 1e-6, 1e8) over NEED_EXT slots
//   k_shade    LambertianBrdf.SampleF (rejection hemisphere), NewAreaLight.Sample_Li, throughput,
//              the shadow ray of the vertex and the continuing ray
//   k_traverse<shadow>   persistent any-hit over SHADOW_* slots; unoccluded -> L += direct term
//
// The traversal kernels keep lanes busy: a lane that finishes its ray takes the next pending
// slot at the next step (persistent while-while with dynamic fetch, Aila & Laine 2009). Pending
// slots are found by scanning 64-slot windows: wave ballot of the state test + popcount ranks
// (the active-ray compaction), parked in a 64-entry LDS list per wave. Path state lives in HBM
// as SoA FP64; every arithmetic step is the same FP64 expression as the megakernel / oracle.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mfx_device.h"
#include "mfx_trace_common.h"
#include "mfx_wavefront.h"

#ifndef MFX_TRAV_WAVES
#define MFX_TRAV_WAVES 1  // min waves per SIMD requested from the register allocator
#endif

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ uint64_t lanes_below() { return (1ULL << lane_id()) - 1ULL; }

// per-block reduction of a per-lane counter, one atomic per block (the counters are sharded too)
template <int NW>
__device__ __forceinline__ void block_add(unsigned long long* dst, uint32_t v, uint32_t* red) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    __syncthreads();
    if (lane_id() == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (int w = 0; w < NW; ++w) s += red[w];
        if (s) atomicAdd(dst, s);
    }
}

// ------------------------------------------------------------------------------------------------
// k_logic: retire finished paths, start new ones (1024 threads per block)
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_logic(WfParams P) {
    __shared__ uint32_t wcnt[16];
    __shared__ unsigned long long blk_base;
    __shared__ uint32_t blk_got;
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    const int wave = threadIdx.x >> 6;
    const bool in = s < P.pool;
    int st = in ? P.state[s] : WF_NEED_EXT;
    if (st == WF_DONE) {
        const int64_t pix = P.pixel[s];
        const int64_t npix = (int64_t)P.width * P.height;
        const double lx = P.lx[s], ly = P.ly[s], lz = P.lz[s];
        if (lx != 0.0) unsafeAtomicAdd(P.accum + pix, lx);
        if (ly != 0.0) unsafeAtomicAdd(P.accum + npix + pix, ly);
        if (lz != 0.0) unsafeAtomicAdd(P.accum + 2 * npix + pix, lz);
        st = WF_FREE;
    }
    const bool need = in && st == WF_FREE;
    const uint64_t m = __ballot(need);
    if (lane_id() == 0) wcnt[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t want = 0;
        for (int w = 0; w < 16; ++w) want += wcnt[w];
        unsigned long long base = 0;
        uint32_t got = 0;
        if (want) {
            // block-aggregated allocation from the path-index shards (shard g owns [g*T/8, (g+1)*T/8))
            for (int k = 0; k < WF_SHARDS && got == 0; ++k) {
                const int g = (blockIdx.x + k) & (WF_SHARDS - 1);
                const int64_t lo = P.total * g / WF_SHARDS, hi = P.total * (g + 1) / WF_SHARDS;
                const unsigned long long c = atomicAdd(P.ctl + WF_CTL_PATH + g, (unsigned long long)want);
                if ((int64_t)c < hi - lo) {
                    base = (unsigned long long)lo + c;
                    got = (uint32_t)min((int64_t)want, hi - lo - (int64_t)c);
                }
            }
        }
        blk_base = base;
        blk_got = got;
    }
    __syncthreads();
    uint32_t off = 0;
    for (int w = 0; w < wave; ++w) off += wcnt[w];
    const uint32_t idx = off + (uint32_t)__popcll(m & lanes_below());
    bool started = false;
    if (need && idx < blk_got) {
        const int64_t p = (int64_t)blk_base + idx;
        // path index -> (sample, 8x8 tile, pixel): sample-major, tile-coherent
        const int W = P.width, H = P.height;
        const int tiles_x = (W + 7) >> 3;
        const int64_t per_sample = (int64_t)tiles_x * ((H + 7) >> 3) * 64;
        const int64_t smp = p / per_sample;
        const int64_t q = p - smp * per_sample;
        const int64_t tile = q >> 6;
        const int within = (int)(q & 63);
        const int x = (int)(tile % tiles_x) * 8 + (within & 7);
        const int y = (int)(tile / tiles_x) * 8 + (within >> 3);
        if (x < W && y < H) {
            const MfxCamera& CAM = *P.cam;
            const int64_t pixel = (int64_t)x * H + y;  // Color[w,h] x-major
            const int64_t gsample = P.sample_base + P.part_index + smp * P.part_count;
            const uint64_t key = path_key(P.seed, (uint64_t)pixel, (uint64_t)gsample);
            uint32_t rn = 0;
            // PixelIntegrator.Sample (Integrators.fs:167-169) + GetRay (Camera.fs:134-139)
            const double u = ((double)x + rng_next(key, rn)) / (double)W;
            const double v = ((double)y + rng_next(key, rn)) / (double)H;
            const DV target = vadd(vadd(ld3(CAM.topleft), vmul(ld3(CAM.right), u)), vmul(ld3(CAM.down), v));
            const DV o = ld3(CAM.position);
            const DV d = vnormalize(vsub(target, o));
            P.ox[s] = o.x; P.oy[s] = o.y; P.oz[s] = o.z;
            P.dx[s] = d.x; P.dy[s] = d.y; P.dz[s] = d.z;
            P.tx[s] = 1.0; P.ty[s] = 1.0; P.tz[s] = 1.0;
            P.lx[s] = 0.0; P.ly[s] = 0.0; P.lz[s] = 0.0;
            P.key[s] = key;
            P.rn[s] = rn;
            P.depth[s] = P.max_depth;
            P.pixel[s] = (int32_t)pixel;
            st = WF_NEED_EXT;
            started = true;
        }
    }
    if (in) P.state[s] = st;
    block_add<16>(P.counters + 16 * (blockIdx.x & (WF_SHARDS - 1)) + 0, started ? 1u : 0u, wcnt);
}

// ------------------------------------------------------------------------------------------------
// Persistent traversal (closest hit or shadow) with per-lane dynamic fetch
// ------------------------------------------------------------------------------------------------
template <bool SHADOW, bool STATS>
__global__ void __launch_bounds__(256, MFX_TRAV_WAVES) k_traverse(WfParams P) {
    extern __shared__ int lds[];
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    int* stack = lds + wave * P.stack_size * 64 + lane;
    int* pend = lds + 4 * P.stack_size * 64 + wave * 64;  // this wave's list of pending slots
    uint32_t* red = (uint32_t*)(lds + 4 * P.stack_size * 64 + 4 * 64);
    const SceneView S{P.nodes, P.blob, P.root_is_leaf};
    const int shard_size = P.pool / WF_SHARDS;
    unsigned long long* heads = P.ctl + (SHADOW ? WF_CTL_SHD : WF_CTL_EXT);

    bool active = false;
    int s = 0;
    DV o = dv(0, 0, 0), d = dv(0, 0, 0);
    double tmax64 = 0.0, best_t = 0.0;
    RayF rf{0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float tlim = 0.f;
    int node = 0, sp = 0, best_slot = -1, best_first = -1;
    bool found = false;
    int win_next = 0, win_end = 0;   // slot window being scanned (wave-uniform)
    int pend_lo = 0, pend_hi = 0;    // pending list [pend_lo, pend_hi) in LDS (wave-uniform)
    int shard_try = 0;
    bool exhausted = false;
    uint32_t c_rays = 0, c_ext = 0;
    Stats st{0, 0, 0};

    while (true) {
        // ---- dynamic fetch: idle lanes take pending slots by rank ----
        bool idle = !active;
        uint64_t m = __ballot(idle);
        while (m != 0 && !exhausted) {
            if (pend_lo == pend_hi) {
                if (win_next >= win_end) {
                    // next chunk of slots from this block's shard, then the others
                    int base = -1, g = 0;
                    while (shard_try < WF_SHARDS) {
                        g = (blockIdx.x + shard_try) & (WF_SHARDS - 1);
                        unsigned long long c = 0;
                        if (lane == 0) c = atomicAdd(heads + g, (unsigned long long)P.chunk);
                        c = __shfl(c, 0);
                        if ((int64_t)c < shard_size) {
                            base = (int)c;
                            break;
                        }
                        ++shard_try;
                    }
                    if (base < 0) {
                        exhausted = true;
                        break;
                    }
                    win_next = g * shard_size + base;
                    win_end = g * shard_size + min(base + P.chunk, shard_size);
                }
                // scan a 64-slot window: ballot + rank = compacted pending list
                const int j = win_next + lane;
                const int sj = j < win_end ? P.state[j] : WF_FREE;
                const bool cand = SHADOW ? (sj == WF_SHADOW_CONT || sj == WF_SHADOW_END) : (sj == WF_NEED_EXT);
                const uint64_t cm = __ballot(cand);
                if (cand) pend[__popcll(cm & lanes_below())] = j;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                pend_lo = 0;
                pend_hi = __popcll(cm);
                win_next += 64;
                continue;
            }
            const int avail = pend_hi - pend_lo;
            const int rank = __popcll(m & lanes_below());
            if (idle && rank < avail) {
                s = pend[pend_lo + rank];
                idle = false;
                active = true;
                o = dv(P.ox[s], P.oy[s], P.oz[s]);
                if (SHADOW) {
                    d = dv(P.sdx[s], P.sdy[s], P.sdz[s]);
                    tmax64 = P.stmax[s];  // dist - 1e-6 (Integrators.fs:44)
                } else {
                    d = dv(P.dx[s], P.dy[s], P.dz[s]);
                    tmax64 = 99999999.;   // Integrators.fs:108
                    if (P.depth[s] != P.max_depth) c_ext++;
                }
                c_rays++;
                rf = make_rayf(o, d);
                tlim = f_round_up(tmax64);
                best_t = tmax64;
                best_slot = -1;
                best_first = -1;
                found = false;
                sp = 0;
                node = S.root_is_leaf ? ~0 : 0;
            }
            const int pm = __popcll(m);
            pend_lo += pm < avail ? pm : avail;
            m = __ballot(idle);
        }
        if (!__any(active)) break;  // every chunk taken and every pending slot traced
        if (active) {
            // ---- internal nodes until this lane reaches a leaf (while-while) ----
            while (node >= 0) {
                if (STATS) st.nodes++;
                node = node_step(S.nodes, node, rf, tlim, stack, sp);
            }
            bool done = node == MFX_TRAV_EXIT;
            // ---- one reference leaf (exact FP64) ----
            if (!done) {
                double t;
                int sl, f;
                if (cluster_hit<SHADOW, STATS>(S, ~node, o, d, 1e-6, tmax64, found ? best_t : __builtin_inf(), t, sl,
                                               f, st)) {
                    if (SHADOW) {
                        found = true;
                        done = true;
                    } else if (!found || t < best_t || (t == best_t && f > best_first)) {
                        found = true;
                        best_t = t;
                        best_slot = sl;
                        best_first = f;
                        tlim = f_round_up(t);
                    }
                }
                if (!done) {
                    if (sp == 0) done = true;
                    else node = stack[(--sp) * 64];
                }
            }
            if (done) {
                if (SHADOW) {
                    if (!found) {  // unoccluded: add this vertex's direct-light term
                        P.lx[s] += P.scx[s];
                        P.ly[s] += P.scy[s];
                        P.lz[s] += P.scz[s];
                    }
                    P.state[s] = P.state[s] == WF_SHADOW_CONT ? WF_NEED_EXT : WF_DONE;
                } else {
                    P.hit_t[s] = found ? best_t : -1.0;
                    P.hit_slot[s] = best_slot;
                    P.state[s] = WF_EXT_DONE;
                }
                active = false;
            }
        }
    }
    unsigned long long* cnt = P.counters + 16 * (blockIdx.x & (WF_SHARDS - 1));
    block_add<4>(cnt + (SHADOW ? 2 : 1), SHADOW ? c_rays : c_ext, red);
    if (STATS) {
        const int b = SHADOW ? 7 : 4;
        block_add<4>(cnt + b, st.nodes, red);
        block_add<4>(cnt + b + 1, st.clusters, red);
        block_add<4>(cnt + b + 2, st.prims, red);
    }
}

// ------------------------------------------------------------------------------------------------
// k_shade: one vertex of PathIntegrator.TraceRay (Integrators.fs:109-136) per EXT_DONE slot
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_shade(WfParams P) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.pool || P.state[s] != WF_EXT_DONE) return;
    const double th = P.hit_t[s];
    if (th < 0.0) {
        P.state[s] = WF_DONE;  // miss: TraceRay returns black (Integrators.fs:137)
        return;
    }
    const int slot = P.hit_slot[s];
    const DV o = dv(P.ox[s], P.oy[s], P.oz[s]), d = dv(P.dx[s], P.dy[s], P.dz[s]);
    const MfxShade sh = P.shade[slot];
    const DV hp = vadd(o, vmul(d, th));  // Ray.PointAtParameter (Ray.fs:8-9)
    DV nm;
    if ((sh.prim_kind & 3) == MFX_KIND_SPHERE) nm = vnormalize(vsub(hp, ld3(sh.n)));  // Sphere.fs:39-43
    else nm = ld3(sh.n);
    const uint64_t key = P.key[s];
    uint32_t rn = P.rn[s];
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
    // NewAreaLight.Sample_Li — Light.fs:42-47,57-59; Rect/Triangle.SamplePoint
    const MfxLight& LT = *P.light;
    const double sel = rng_next(key, rn);
    const int lt = sel < 0.5 ? 0 : 1;
    const double tu = rng_next(key, rn);
    const double tv = rng_next(key, rn);
    double uu = tu, vv = tv;
    if (tu + tv > 1.) { uu = 1. - tu; vv = 1. - tv; }
    const double sq = sqrt(1. - uu);
    const double s1 = 1. - sq, s2 = vv * sq;
    const DV lp = vadd(vadd(ld3(LT.v0[lt]), vmul(ld3(LT.e1[lt]), s1)), vmul(ld3(LT.e2[lt]), s2));
    const DV toLight = vsub(lp, hp);
    const double dist = vlen(toLight);
    const DV unit = vdiv(toLight, dist);
    // NewAreaLight.L (Light.fs:48-56) and the unclamped cosine (Integrators.fs:52)
    const double cos_o = vdot(toLight, ld3(LT.normal));
    const double dist2 = toLight.x * toLight.x + toLight.y * toLight.y + toLight.z * toLight.z;
    const double solid = fabs(cos_o) * LT.area / dist2;
    const double cs = vdot(unit, nm);
    const double Tx = P.tx[s] * (TWOPI * (ei * (INVPI * a[0])));
    const double Ty = P.ty[s] * (TWOPI * (ei * (INVPI * a[1])));
    const double Tz = P.tz[s] * (TWOPI * (ei * (INVPI * a[2])));
    // (l / pdf_li + TraceRay(next)) * col / pdf, unrolled forward (Integrators.fs:135-136)
    if (cos_o < 0.) {
        P.scx[s] = Tx * ((cs * (solid * LT.color[0])) / LT.pdf);
        P.scy[s] = Ty * ((cs * (solid * LT.color[1])) / LT.pdf);
        P.scz[s] = Tz * ((cs * (solid * LT.color[2])) / LT.pdf);
    } else {
        P.scx[s] = 0.0; P.scy[s] = 0.0; P.scz[s] = 0.0;
    }
    P.tx[s] = Tx; P.ty[s] = Ty; P.tz[s] = Tz;
    P.ox[s] = hp.x; P.oy[s] = hp.y; P.oz[s] = hp.z;
    P.sdx[s] = unit.x; P.sdy[s] = unit.y; P.sdz[s] = unit.z;
    P.stmax[s] = dist - 1e-6;
    P.rn[s] = rn;
    const int depth = P.depth[s] - 1;
    P.depth[s] = depth;
    if (depth < 0) {
        P.state[s] = WF_SHADOW_END;  // the depth -1 query's result is discarded (Integrators.fs:109)
    } else {
        P.dx[s] = wi.x; P.dy[s] = wi.y; P.dz[s] = wi.z;
        P.state[s] = WF_SHADOW_CONT;
    }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
static size_t wf_lds_bytes(int stack_size) { return (size_t)4 * (stack_size * 64 + 64) * sizeof(int) + 64; }

hipError_t mfx_wf_occupancy(int stack_size, int* ext_blocks_per_cu, int* shd_blocks_per_cu) {
    const size_t lds = wf_lds_bytes(stack_size);
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(ext_blocks_per_cu, k_traverse<false, false>, 256, lds);
    if (e != hipSuccess) return e;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(shd_blocks_per_cu, k_traverse<true, false>, 256, lds);
}

hipError_t mfx_wf_iteration(const WfParams& P, int ext_grid, int shd_grid, bool stats, hipStream_t st,
                            hipEvent_t* ev) {
    const unsigned logic_blocks = (unsigned)((P.pool + 1023) / 1024);
    const unsigned pool_blocks = (unsigned)((P.pool + 255) / 256);
    const size_t lds = wf_lds_bytes(P.stack_size);
    hipError_t e = hipMemsetAsync(P.ctl + WF_CTL_EXT, 0, 2 * WF_SHARDS * sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_logic, dim3(logic_blocks), dim3(1024), 0, st, P);
    if ((e = hipEventRecord(ev[0], st)) != hipSuccess) return e;
    if (stats)
        hipLaunchKernelGGL((k_traverse<false, true>), dim3(ext_grid), dim3(256), lds, st, P);
    else
        hipLaunchKernelGGL((k_traverse<false, false>), dim3(ext_grid), dim3(256), lds, st, P);
    if ((e = hipEventRecord(ev[1], st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_shade, dim3(pool_blocks), dim3(256), 0, st, P);
    if ((e = hipEventRecord(ev[2], st)) != hipSuccess) return e;
    if (stats)
        hipLaunchKernelGGL((k_traverse<true, true>), dim3(shd_grid), dim3(256), lds, st, P);
    else
        hipLaunchKernelGGL((k_traverse<true, false>), dim3(shd_grid), dim3(256), lds, st, P);
    return hipGetLastError();
}

hipError_t mfx_wf_finish(const WfParams& P, hipStream_t st) {
    const unsigned logic_blocks = (unsigned)((P.pool + 1023) / 1024);
    hipLaunchKernelGGL(k_logic, dim3(logic_blocks), dim3(1024), 0, st, P);
    return hipGetLastError();
}
