// mfx_wavefront.hip — wavefront path tracing on gfx950: the integrator loop
// (Integrators.fs:107-137, 161-172) as two persistent kernels per iteration over a pool of
// path slots, one bounce of every live path per iteration (mfx_wavefront.h):
//
//   k_extend   bvh.Hit(ray, 1e-6, 99999999.) (Integrators.fs:108) for NEED_EXT slots; in a
//              generation's first iteration every FREE slot j starts path path_base + j
//              (PixelIntegrator.Sample + PinholeCamera.GetRay, Integrators.fs:161-169,
//              Camera.fs:134-139). Writes the hit point and the hit's shade index.
//   k_shadow   one vertex of PathIntegrator.TraceRay for HIT slots: LambertianBrdf.SampleF and
//              NewAreaLight.Sample_Li (Integrators.fs:110-134), recording the vertex's col, then
//              its shadow ray (Integrators.fs:44) traced by a lane of the same wave; unoccluded ->
//              the vertex's direct term l / pdf_li is recorded too (mfx_wavefront.h).
//   k_resolve  after a generation: each finished path's vertices folded back to the camera in the
//              reference's recursion order, (l / pdf_li + TraceRay(next)) * col (Integrators.fs:136),
//              and added to its pixel in sample order (`color <- color + ...`, Integrators.fs:169).
//
// Both trace kernels keep lanes busy: a lane that finishes its ray takes the next pending ray at
// the next step (persistent while-while with dynamic fetch, Aila & Laine 2009). Pending rays come
// from scanning 64-slot windows with the whole wave: only the state words are read (several
// windows per memory round trip, WF_LOOKAHEAD), the slots to work on are compacted (ballot +
// popcount ranks) into a per-wave LDS list, and the per-slot data is loaded by the lane that takes
// the entry. k_shadow shades 64 listed hits at a time with all lanes and hands the shadow rays to
// the traversal in LDS, so a shadow ray never round-trips through HBM. Path state lives in HBM as
// SoA FP64; every arithmetic step is the same FP64 expression as the oracle, in the same order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "mfx_device.h"
#include "mfx_trace_common.h"
#include "mfx_wavefront.h"

#ifndef MFX_TRAV_WAVES
#define MFX_TRAV_WAVES 4  // min waves per SIMD requested from the register allocator (128 VGPRs; a few spills)
#endif

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }


#ifndef MFX_SHADOW_ORDER
#define MFX_SHADOW_ORDER 1  // shadow rays' child order: 0 near-first, 1 far-first (by exit distance)
#endif

#ifndef MFX_NODE_LANES_MIN
#define MFX_NODE_LANES_MIN 16  // node-loop early exit: fewer lanes than this still stepping
#endif
#ifndef MFX_NODE_LANES_MIN_SHD
#define MFX_NODE_LANES_MIN_SHD 12  // the same for shadow rays
#endif

#ifndef MFX_DIAG_STAMPS
#define MFX_DIAG_STAMPS 0  // diagnostic build only: 1 = k_extend phase stamps, 2 = k_shadow, 3 = k_camera
#endif
struct DiagAcc {
    uint64_t fetch, node, leaf, fin, last, scan, shade, lat;  // lat: node loads' issue-to-use cycles (node_step)
    uint32_t outer, node_iters, windows;
};
__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define DIAG_MARK(acc, field, on)              \
    do {                                       \
        if (on) {                              \
            const uint64_t _t = stamp();       \
            (acc).field += _t - (acc).last;    \
            (acc).last = _t;                   \
        }                                      \
    } while (0)
__device__ __forceinline__ uint64_t lanes_below() { return (1ULL << lane_id()) - 1ULL; }

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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
// Slot windows: a wave takes chunks of P.chunk slots (its block's shard first, then the others)
// and scans them 64 at a time.
// ------------------------------------------------------------------------------------------------
static_assert(WF_SHARDS == 64, "shard masks are one bit per lane of a wave");

// Shards of a sharded counter set that are still open (counter below its capacity), one bit per
// shard, from one vector load of all 64 counters (lane g reads shard g). Counters only grow, so a
// stale value can only report a closed shard as open: the caller's atomic then fails and it asks
// again. This replaces walking the shards with one returning atomic each, which cost every wave
// up to 64 serialized round trips at the end of each kernel.
__device__ __forceinline__ uint64_t open_shards(const unsigned long long* ctr, int cap) {
    const unsigned long long v = __hip_atomic_load(ctr + lane_id() * WF_HS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __ballot((int64_t)v < (int64_t)cap);
}

// the first open shard at or after `home` (cyclically); `open` must be non-zero
__device__ __forceinline__ int next_open(uint64_t open, int home) {
    const uint64_t r = home ? ((open >> home) | (open << (64 - home))) : open;
    return (home + __builtin_ctzll(r)) & (WF_SHARDS - 1);
}

#ifndef WF_CLOSED_MASK
#define WF_CLOSED_MASK 1  // closed shards are found from one mask word, not from a load of all 64 heads
#endif
struct Scanner {
    int win_next, win_end, shard;
    bool exhausted;
    uint64_t closed_seen;  // WF_CLOSED_MASK: shards this wave found closed itself
    // state words of the next WF_LOOKAHEAD windows of the chunk, loaded in one round of
    // independent loads (b[0] = the current window; -1 past the chunk's end): windows without
    // work are skipped with no further memory round trip. Slots of a taken chunk change only
    // through this wave, so the words stay current.
    int b[WF_LOOKAHEAD];
    int nbuf;
    // Make [win_next, win_end) non-empty; false once every chunk has been taken. A wave takes
    // chunks from its block's home shard while it lasts, then from the next open shard.
    // qcount: a ray queue's per-shard entry counts (MFX_RAY_QUEUE: a queue fills shard g's range from
    // its start); null: whole shards
    // closed: the launch's closed-shard mask (WF_CLOSED_MASK): bit g set by the one fetch that
    // crosses shard g's end (the fetch whose start lands in [cap, cap + chunk)); a wave also skips the
    // shards its own fetches found closed, so an unset bit never makes it retry one
    // LOAD = false (k_camera: every slot of a generation's first iteration is FREE): no state words
    template <bool LOAD = true>
    __device__ __forceinline__ bool window(unsigned long long* heads, int chunk, int shard_size,
                                           const int32_t* __restrict__ state, const unsigned long long* qcount,
                                           unsigned long long* closed) {
        if (win_next < win_end) return true;
        if (exhausted) return false;
        while (true) {
            unsigned long long c = 0;
            if (lane_id() == 0) c = atomicAdd(heads + shard * WF_HS, (unsigned long long)chunk);
            c = __shfl(c, 0);
            const int cap = qcount ? (int)qcount[shard * WF_HS] : shard_size;
            if ((int64_t)c < cap) {
                win_next = shard * shard_size + (int)c;
                win_end = shard * shard_size + min((int)c + chunk, cap);
                if (LOAD) fill(state);
                return true;
            }
#if WF_CLOSED_MASK
            if (lane_id() == 0 && (int64_t)c < (int64_t)cap + chunk) atomicOr(closed, 1ull << shard);
            closed_seen |= 1ull << shard;
            unsigned long long cm = 0;
            if (lane_id() == 0) cm = __hip_atomic_load(closed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            cm = __shfl(cm, 0);
            const uint64_t open = ~(cm | closed_seen);
#else
            const uint64_t open = open_shards(heads, qcount ? (int)qcount[lane_id() * WF_HS] : shard_size);
#endif
            if (open == 0) {
                exhausted = true;
                return false;
            }
            // the next open shard after this one (a per-wave pseudo-random start instead, WF_SPREAD,
            // measured C2 -0.4 %, C4 -1.9 %, r04c)
            shard = next_open(open, shard);
        }
    }
    __device__ __forceinline__ void fill(const int32_t* __restrict__ state) {
#pragma unroll
        for (int k = 0; k < WF_LOOKAHEAD; ++k) {
            const int j = win_next + 64 * k + lane_id();
            b[k] = j < win_end ? state[j] : -1;
        }
        nbuf = WF_LOOKAHEAD;
    }
    // this lane's state word in the current window
    __device__ __forceinline__ int word() const { return b[0]; }
    __device__ __forceinline__ void advance(const int32_t* __restrict__ state) {
        win_next += 64;
#pragma unroll
        for (int k = 0; k + 1 < WF_LOOKAHEAD; ++k) b[k] = b[k + 1];
        b[WF_LOOKAHEAD - 1] = -1;
        if (--nbuf == 0 && win_next < win_end) fill(state);
    }
};

// the lane's stack: all of it in LDS, or the first P.stack_lds entries (the rest in P.spill)
template <bool SPILL>
__device__ __forceinline__ typename std::conditional<SPILL, SpillStack, LdsStack>::type make_stack(int* lds,
                                                                                                  const WfParams& P,
                                                                                                  int nlds) {
    if constexpr (SPILL)
        return SpillStack{lds, P.spill + blockIdx.x * 256 + threadIdx.x, nlds, (int)gridDim.x * 256};
    else
        return LdsStack{lds};
}

// Traversal state of one lane (one ray) across outer-loop iterations
struct Trav {
#ifdef MFX_DIAG_OCCLUSION
    uint32_t n0, l0;  // the lane's node / cluster counts when this ray started
#endif
    DV o, d;
    double tmax64;
    Best B;
    int node, sp;
    int inst;   // two-level scenes: the instance whose template the lane is in (-1: the world)
    int inst_sp;  // and the stack depth at which it entered (entries below belong to the world)
};

__device__ __forceinline__ void trav_begin(Trav& T, const SceneView& S, DV o, DV d, double tmax) {
    T.o = o;
    T.d = d;
    T.tmax64 = tmax;
    T.B = Best{tmax, -1, -1, false};
    T.sp = 0;
    T.node = 0;
    T.inst = -1;
    T.inst_sp = 0;
}

// one node step of the per-lane traversal (BVH4; shadow rays far-first)
template <bool SHADOW, typename ST>
__device__ __forceinline__ int trav_node_step(const SceneView& S, int node, const RayF& rf, float tlim, const ST& stack,
                                              int& sp, TopNodes tn, uint64_t* lat) {
    return node_step<true, SHADOW && MFX_SHADOW_ORDER == 1>(S.nodes, node, rf, tlim, stack, sp, tn, lat);
}

// Internal nodes until this lane reaches a leaf (while-while), then that one reference leaf in
// exact FP64. Returns true when the ray is finished (closest: stack empty; shadow: occluded or
// stack empty).
// INST: a two-level scene; a lane enters and leaves instances inside the node loop (inst_frame).
// SLDS: the scene's slots are read from the kernel's LDS copy (a small flat scene, SceneView::slots_lds).
template <bool SHADOW, bool STATS, bool INST, bool SLDS, typename ST>
__device__ __forceinline__ bool trav_step(Trav& T, const SceneView& S, const ST& stack, TopNodes tn, Stats& st,
                                          DiagAcc& dg, bool diag) {
    // the frame of the entry popped at the end of the last round (an instance left or entered)
    RayF rf{};  // (the frame switch's own ray update is superseded below)
    if (INST) T.node = inst_frame(S, T.node, T.inst, T.inst_sp, T.sp, T.o, T.d, rf);
    // the FP32 ray and the node-test limit are recomputed each round (the same values) rather than
    // held through the leaf tests: fewer live registers, fewer spills (+1 to +5 %)
    rf = INST ? frame_ray(S, T.inst, T.o, T.d) : make_rayf(T.o, T.d);
    const float tlim = f_tlim(T.B.t);  // the query's tMax until the first hit, then the best t
    while (T.node >= 0) {
        if (STATS) st.nodes++;
#ifdef MFX_DIAG_OCCLUSION
        if (STATS && !SHADOW && T.B.found) st.after_nodes++;
#endif
        if (diag && lane_id() == __builtin_amdgcn_readfirstlane(lane_id())) dg.node_iters++;  // once per wave iteration
        T.node = trav_node_step<SHADOW>(S, T.node, rf, tlim, stack, T.sp, tn, diag ? &dg.lat : nullptr);
        if (INST) T.node = inst_frame(S, T.node, T.inst, T.inst_sp, T.sp, T.o, T.d, rf);
        // leave the node loop once few lanes still step: the rest resume next round, after the
        // leaf tests and a refill of the idle lanes
        if (__popcll(__ballot(T.node >= 0)) < (SHADOW ? MFX_NODE_LANES_MIN_SHD : MFX_NODE_LANES_MIN)) break;
    }
    DIAG_MARK(dg, node, diag);
    if (T.node >= 0) return false;
    if (T.node == MFX_TRAV_EXIT) return true;
#ifdef MFX_DIAG_OCCLUSION
    if (STATS && !SHADOW && T.B.found) st.after_leaves++;
#endif
    const int base = (INST && T.inst >= 0) ? load_inst(S, T.inst).slot_base : 0;
    const bool better = leaf_hit<SHADOW, STATS, false, SLDS>(S, ~T.node, T.o, T.d, 1e-6, T.tmax64, T.B, st, base);
    if (better) {
        if (SHADOW) {
            T.B.found = true;
            return true;
        }
    }
    if (T.sp == 0) return true;
    T.node = stack.get(T.sp - 1, stack.deep(T.sp));
    --T.sp;
    return false;
}

// Path index of this generation -> (sample, 8x8 pixel tile, pixel), sample-major and
// tile-coherent. False for the padding indices of edge tiles (no path). A banded
// trace (image partition) numbers only its own tile rows: its k-th tile row is film tile row
// band_index + k * band_count, so pixels, keys and samples are the whole-film trace's.
// PP: WfParams, or k_shadow's LDS copy of the fields it needs (PixParams)
template <typename PP>
__device__ __forceinline__ bool path_pixel(const PP& P, int64_t p, int& x, int& y, int64_t& smp) {
    // p = path_base + s: the 64-bit split of path_base is done once per generation on the host
    // (base_smp, base_q), so only 32-bit divisions remain here (base_q + s < 2^32)
    const unsigned tiles_x = (unsigned)(P.width + 7) >> 3;
    const unsigned per_sample = tiles_x * (unsigned)P.band_rows * 64;  // < 2^31 (film limit)
    const unsigned qs = (unsigned)P.base_q + (unsigned)(p - P.path_base);
    const unsigned ds = qs / per_sample;
    smp = P.base_smp + ds;
    const unsigned q = qs - ds * per_sample;
    const unsigned tile = q >> 6, within = q & 63;
    const unsigned tyl = tile / tiles_x;
    const unsigned ty = (unsigned)band_tile_row(P.band_index, P.band_count, (int)tyl);
    x = (int)((tile - tyl * tiles_x) * 8 + (within & 7));
    y = (int)(ty * 8 + (within >> 3));
    return x < P.width && y < P.height;
}

#define WF_EXT_PEND 128  // k_extend per-wave pending list: slot indices (sign bit: camera ray)
#define WF_SHD_LIST 128  // k_shadow per-wave shade list entries

__device__ __forceinline__ bool cont0(int vflag) { return (vflag & 1) != 0; }  // k_shadow: the path continues

// Per-wave LDS list of k_shadow's pending shadow rays: ray index, a flag word, the path's slot and
// its next-queue entry (MFX_RAY_QUEUE) and 6 doubles (direction, tmax, the direct term's operands
// cs and solid), each field a 64-entry column (conflict-free).
struct PendShd {
    static constexpr int BYTES = 64 * (4 + 4 + 8 * 6);
    int* slot;  // the shadow ray's origin, the hit point: its index in the ray arrays, or (a path
                // that continues into the next queue, MFX_RAY_QUEUE) its entry there
    int* flag;
    double* v;  // v[f * 64 + entry]
    __device__ __forceinline__ PendShd(uint8_t* base) {
        slot = (int*)base;
        flag = slot + 64;
        v = (double*)(base + 512);
    }
};

// k_shadow derives a path's key from its slot (as k_extend did for the camera ray) at every vertex:
// no key is stored (r02bs: derived at the first vertex, C2 +0.9 to +2.5 %; at every vertex, r03av:
// -0.3 to -1.2 % then, r05m: C2 +0.5 %, Renault +0.7 % once the depth word was gone too)
#ifndef MFX_HEMI_WAVE_FIRST
#define MFX_HEMI_WAVE_FIRST 1  // trials each owner makes alone before the wave shares them (r02bi: 1 vs 2, C3 +0.8 %, C4 +0.6 %, C2 -0.5 %)
#endif

// GetRandomInUnitSphere(nm) (Material.fs:9-14) for the wave's shading lanes (`own`), the same
// accepted trial, point and draw count as hemisphere_ball. A lane's loop runs until its first
// accepted trial (3.8 trials on average), but the wave runs until its slowest lane's (about 16):
// after a first round in which every owner tries its own first MFX_HEMI_WAVE_FIRST trials, the owners
// still rejecting share the wave's 64 lanes, m = 2^k consecutive trials each (np * m <= 64), and
// each owner takes the lowest accepted trial of its round (all lower ones were rejected before).
// A worker lane draws from the owner's key and draw count (the trial's three draws at their
// counter positions) and decides with hemi_trial, so p is the owner's own computation's bits.
// scratch: 64 ints of the wave's LDS (owner lane ids in rank order).
__device__ __forceinline__ DV hemisphere_ball_wave(bool own, DV nm, uint64_t key, uint32_t& rn, int* scratch) {
    const int lane = lane_id();
    DV p = dv(0, 0, 0);
    bool done = !own;
    const uint32_t base = rn;  // draws used before trial 0
    if (own) {  // round 0: the owner's own first MFX_HEMI_WAVE_FIRST trials
        const float nx = (float)nm.x, ny = (float)nm.y, nz = (float)nm.z;
        uint32_t r = base;
        uint64_t z[3 * MFX_HEMI_WAVE_FIRST];
#pragma unroll
        for (int i = 0; i < 3 * MFX_HEMI_WAVE_FIRST; ++i) z[i] = rng_bits(key, r);
        for (int i = 0; i < MFX_HEMI_WAVE_FIRST; ++i)
            if (hemi_trial(nm, nx, ny, nz, z[3 * i], z[3 * i + 1], z[3 * i + 2], p)) {
                rn = base + 3 * (i + 1);
                done = true;
                break;
            }
    }
    uint32_t next = MFX_HEMI_WAVE_FIRST;  // the owner's next trial index
    while (true) {
        const uint64_t pend = __ballot(!done);
        if (pend == 0) break;
        const int np = __popcll(pend);
        int sh = 0;  // trials per pending owner: m = 2^sh, np * m <= 64
        while ((np << (sh + 1)) <= 64) ++sh;
        const int rank = __popcll(pend & lanes_below());
        if (!done) scratch[rank] = lane;
        wave_lds_sync();
        const int slot = lane >> sh, t = lane & ((1 << sh) - 1);
        const bool work = slot < np;
        const int owner = work ? scratch[slot] : lane;
        wave_lds_sync();
        const uint64_t k = __shfl(key, owner);
        const uint32_t b = (uint32_t)__shfl((int)base, owner);
        const uint32_t nt = (uint32_t)__shfl((int)next, owner);
        const DV q = dv(__shfl(nm.x, owner), __shfl(nm.y, owner), __shfl(nm.z, owner));
        bool acc = false;
        DV pt = dv(0, 0, 0);
        if (work) {
            uint32_t r = b + 3 * (nt + (uint32_t)t);
            const uint64_t zx = rng_bits(k, r);
            const uint64_t zy = rng_bits(k, r);
            const uint64_t zz = rng_bits(k, r);
            acc = hemi_trial(q, (float)q.x, (float)q.y, (float)q.z, zx, zy, zz, pt);
        }
        const uint64_t A = __ballot(acc);
        const int first_lane = done ? lane : (rank << sh);
        const uint64_t seg = done ? 0 : (A >> first_lane) & (sh == 6 ? ~0ULL : ((1ULL << (1 << sh)) - 1));
        const int src = done ? lane : first_lane + (seg ? __builtin_ctzll(seg) : 0);
        const DV ps = dv(__shfl(pt.x, src), __shfl(pt.y, src), __shfl(pt.z, src));
        if (!done) {
            if (seg) {
                p = ps;
                rn = base + 3 * (next + (uint32_t)__builtin_ctzll(seg) + 1);
                done = true;
            } else {
                next += 1u << sh;
            }
        }
    }
    return p;
}

// One vertex of PathIntegrator.TraceRay (Integrators.fs:109-134) for the wave's `own` lanes, at the
// hit point hp with normal nm: LambertianBrdf.SampleF (Material.fs:33-36; the rejection sampler
// spread over the wave, hemisphere_ball_wave) gives the next direction wi and its cosine ei;
// NewAreaLight.Sample_Li (Light.fs:42-47,57-59; Rect/Triangle.SamplePoint) the shadow ray's unit
// direction and length, and the operands of the direct term l / pdf_li, l = (unit . n) *
// L(hit, toLight) (Integrators.fs:52, Light.fs:48-56): cs = unit . n and solid = |cos_o| A / dist^2,
// L black unless cos_o < 0 (lightable). Called by the whole wave; scratch: 64 ints of its LDS.
struct VertexSample {
    DV wi, unit;
    double ei, dist, cs, solid;
    bool lightable;
};
// LT: the light (k_shadow's LDS copy).
__device__ __forceinline__ VertexSample sample_vertex(const MfxLight& LT, bool own, DV hp, DV nm, uint64_t key,
                                                      uint32_t& rn, int* scratch) {
    VertexSample V{};
#if defined(MFX_DIAG_ONE_TRIAL)  // timing experiment only: the first trial, mirrored into the hemisphere
    DV p = dv(rng_next(key, rn) * 2.0 - 1.0, rng_next(key, rn) * 2.0 - 1.0, rng_next(key, rn) * 2.0 - 1.0);
    if (vdot(nm, p) <= 0.) p = vmul(p, -1.0);
#else
    const DV p = hemisphere_ball_wave(own, nm, key, rn, scratch);
#endif
    if (!own) return V;
    V.wi = vnormalize(p);
    V.ei = vdot(nm, V.wi);
    const double sel = rng_next(key, rn);
    const int lt = sel < 0.5 ? 0 : 1;
    const double tu = rng_next(key, rn);
    const double tv = rng_next(key, rn);
    double uu = tu, vv = tv;
    if (tu + tv > 1.) { uu = 1. - tu; vv = 1. - tv; }
    const double sq = sqrt(1. - uu);
    const double s1 = 1. - sq, s2 = vv * sq;
    // both halves from scalar registers, selected per lane
    const DV lv0 = lt ? ld3(LT.v0[1]) : ld3(LT.v0[0]);
    const DV le1 = lt ? ld3(LT.e1[1]) : ld3(LT.e1[0]);
    const DV le2 = lt ? ld3(LT.e2[1]) : ld3(LT.e2[0]);
    const DV lp = vadd(vadd(lv0, vmul(le1, s1)), vmul(le2, s2));
    const DV toLight = vsub(lp, hp);
    V.dist = vlen(toLight);
    V.unit = vdiv(toLight, V.dist);
    // NewAreaLight.L (Light.fs:48-56) and the unclamped cosine (Integrators.fs:52)
    const double cos_o = vdot(toLight, ld3(LT.normal));
    const double dist2 = toLight.x * toLight.x + toLight.y * toLight.y + toLight.z * toLight.z;
    V.solid = fabs(cos_o) * LT.area / dist2;
    V.cs = vdot(V.unit, nm);
    V.lightable = cos_o < 0.;
    return V;
}

// ------------------------------------------------------------------------------------------------
// k_extend: closest hit for NEED_EXT slots; in a generation's first iteration FREE slots start paths
// ------------------------------------------------------------------------------------------------
// Q: the instance for the iterations on ray queues (MFX_RAY_QUEUE; P.qcount); the in-place one
// has none of their code
// SK: the scene kind (WF_SK_FLAT, WF_SK_INST: two-level, WF_SK_SLDS: a small flat scene whose whole
// slot array sits in LDS); only a small scene's instances carry the LDS slot reads (r04c: the runtime
// branch in every leaf test cost C2 1.8 % and C4 4 %)
// START: the instance for a generation's first iteration when k_camera does not take its camera
// rays (two-level scenes, MFX_CAMERA_PACKETS=0); only it carries the camera-ray code (GetRay, the
// path key, the camera's fields), so the bounce instances hold fewer live scalar registers
template <bool STATS, bool SPILL, int SK, bool Q, bool START = false>
__global__ void __launch_bounds__(256, MFX_TRAV_WAVES) k_extend(WfParams P) {
    constexpr bool INST = SK == WF_SK_INST, SLDS = SK == WF_SK_SLDS;
    extern __shared__ int lds_all[];
#if MFX_NODE_F16
    const TopNodes tn{(const float4*)lds_all, P.ntop_ext, P.nodes_h};
#else
    const TopNodes tn{(const float4*)lds_all, P.ntop_ext};
#endif
#if MFX_NODE_F16
    if (P.nodes_h) load_top_nodes_h((float4*)lds_all, P.nodes_h, P.ntop_ext);
    else
#endif
        load_top_nodes((float4*)lds_all, P.nodes, P.ntop_ext);
    MfxInstance* inst_lds = (MfxInstance*)(lds_all + P.ntop_ext * 32);
    if (INST) load_inst_lds(inst_lds, P.inst, P.ninst_lds);
    int4* slot_lds = (int4*)(inst_lds + (INST ? P.ninst_lds : 0));
    const int nslot = SLDS ? P.nslot_ext : 0;
    if (SLDS) load_slots_lds(slot_lds, P.slots, nslot);
    int* lds = (int*)(slot_lds + 5 * nslot);
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    using Stack = typename std::conditional<SPILL, SpillStack, LdsStack>::type;
    const Stack stack = make_stack<SPILL>(lds + wave * P.stack_lds_ext * 64 + lane, P, P.stack_lds_ext);
    int* pend = lds + 4 * P.stack_lds_ext * 64 + wave * WF_EXT_PEND;
    uint32_t* red = (uint32_t*)(lds + 4 * P.stack_lds_ext * 64 + 4 * WF_EXT_PEND);
    const SceneView S{P.nodes, P.slots, P.slot_ref, P.ref_blob, P.inst, inst_lds, INST ? P.ninst_lds : 0, slot_lds, nslot};
    const int shard_size = P.pool / WF_SHARDS;

    Scanner sc{};
    sc.shard = blockIdx.x & (WF_SHARDS - 1);
    int pend_lo = 0, pend_hi = 0;
    bool active = false;
    int se = 0;  // the lane's listed entry: slot (WF_ENTRY_SLOT), lit mask << 28, camera-ray flag (sign)
    Trav T{};
    // rays started by this wave: every listed entry is started, so the wave counts its lists (a
    // wave-uniform sum) instead of each lane its rays (a per-lane counter spilled to scratch, whose
    // increment put a scratch round trip into every refill)
    uint32_t c_listed = 0;
    Stats st{0, 0, 0};
    constexpr bool DG = MFX_DIAG_STAMPS == 1;
    DiagAcc dg{};
    if (DG) dg.last = stamp();
    // An in-place extension ray's entry carries the path's lit-vertex mask (k_shadow wrote it into
    // the NEED_EXT state word) in bits 28..30 when it fits (iterations 1..3: vertices 0..2), so a
    // miss writes its finished state word, mask included, without loading the depth word (r04b:
    // +0.5 % over that load; k_resolve reading the depth words of misses instead, r04g: -0.3 %).
    // The lane keeps the entry itself: no register for the mask or the camera-ray flag.
    const bool lit_in_entry = !Q && P.iter <= 3;
    // the lane takes listed entry e: its camera ray (FREE slot) or the slot's extension ray
    auto start_ray = [&](int e) {
        se = e;
        const int s = e & WF_ENTRY_SLOT;
        const bool fresh = START && e < 0;
        DV o, d;
        if (fresh) {
            // PixelIntegrator.Sample (Integrators.fs:167-169) + GetRay (Camera.fs:134-139)
            int x, y;
            int64_t smp;
            path_pixel(P, P.path_base + s, x, y, smp);
            const int64_t pixel = (int64_t)x * P.height + y;  // Color[w,h] x-major
            const int64_t gsample = P.sample_base + P.part_index + smp * P.part_count;
            const uint64_t key = path_key(P.seed, (uint64_t)pixel, (uint64_t)gsample);
            uint32_t rn = 0;
            const double u = ((double)x + rng_next(key, rn)) / (double)P.width;
            const double v = ((double)y + rng_next(key, rn)) / (double)P.height;
            const MfxCamera& CAM = P.cam;
            const DV target = vadd(vadd(ld3(CAM.topleft), vmul(ld3(CAM.right), u)), vmul(ld3(CAM.down), v));
            o = ld3(CAM.position);
            d = vnormalize(vsub(target, o));
            // throughput 1, radiance 0, rn 2 and depth max_depth stay implicit (WF_FRESH); the
            // key is derived again by k_shadow
        } else {
            o = dv(P.ox[s], P.oy[s], P.oz[s]);
            d = dv(P.dx[s], P.dy[s], P.dz[s]);
        }
        trav_begin(T, S, o, d, 99999999.);  // Integrators.fs:108
        active = true;
    };
    // the lane's ray is finished: its closest hit (hit point, shade index) or its miss
    auto finish_ray = [&]() {
        const int s = se & WF_ENTRY_SLOT;
        const bool fresh = START && se < 0;
        const int fl = fresh ? WF_FRESH : 0;
        if (T.B.found) {
            const DV hp = vadd(T.o, vmul(T.d, T.B.t));  // Ray.PointAtParameter (Ray.fs:8-9)
            P.ox[s] = hp.x; P.oy[s] = hp.y; P.oz[s] = hp.z;
            // in place (lit_in_hit): the path's lit mask rides in bits 29..31 for k_shadow
            const int lm = (P.lit_in_hit && lit_in_entry && !fresh) ? ((se >> 28) & 7) << 29 : 0;
            P.state[s] = ((T.B.info & MFX_INFO_SHADE_MASK) << WF_SHADE_SHIFT) | WF_HIT | fl | lm;
        } else {  // a later miss finishes the path: its lit mask goes into the state word
            const int lm = fresh || Q ? 0 : (lit_in_entry ? (se >> 28) & 7 : (P.depth[s] >> WF_LIT_SHIFT) & 0xffff);
            P.state[s] = WF_MISS | (lm << WF_SHADE_SHIFT) | fl;
        }
        active = false;
    };

    while (true) {
        // ---- dynamic fetch: idle lanes take pending rays by rank ----
        bool idle = !active;
        uint64_t m = __ballot(idle);
        while (m != 0) {
            if (pend_lo == pend_hi) {
                // list at least 64 slots to trace (or all that are left) from as many windows as it
                // takes; only state words are read here, WF_LOOKAHEAD windows per round trip
                int n = 0;
                while (n < 64 && sc.window(P.ctl + WF_CTL_EXT, P.chunk, shard_size, P.state, Q ? P.qcount : nullptr, P.ctl + WF_CTL_CLOSED_EXT)) {
                    if (DG) dg.windows++;
                    const int j = sc.win_next + lane;
                    const int sj = sc.word();
                    bool take = (sj & WF_STATE_MASK) == WF_NEED_EXT;
                    if (START && sj == WF_FREE && j < P.total) {
                        int x, y;
                        int64_t smp;
                        // edge-tile padding starts no path (none when 8 divides the film size)
                        take = !P.tile_padding || path_pixel(P, P.path_base + j, x, y, smp);
                    }
                    const uint64_t tm = __ballot(take);
                    // entry: slot | camera-ray flag << 31, or slot | lit mask << 28 (lit_in_entry)
                    if (take)
                        pend[n + __popcll(tm & lanes_below())] =
                            (START && sj == WF_FREE) ? (j | (int)0x80000000)
                                          : (lit_in_entry ? j | (((unsigned)sj >> WF_SHADE_SHIFT) & 7) << 28 : j);
                    n += __popcll(tm);
                    sc.advance(P.state);
                }
                wave_lds_sync();
                pend_lo = 0;
                pend_hi = n;
                c_listed += (uint32_t)n;
                if (n == 0) break;  // every chunk scanned
            }
            const int avail = pend_hi - pend_lo;
            const int rank = __popcll(m & lanes_below());
            if (idle && rank < avail) {
                start_ray(pend[pend_lo + rank]);
                idle = false;
            }
            const int pm = __popcll(m);
            pend_lo += pm < avail ? pm : avail;
            m = __ballot(idle);
        }
        if (!__any(active)) break;  // every chunk taken and every pending ray traced
        DIAG_MARK(dg, fetch, DG);
        if (DG) dg.outer++;
        bool fin = false;
        if (active) fin = trav_step<false, STATS, INST, SLDS>(T, S, stack, tn, st, dg, DG);
        DIAG_MARK(dg, leaf, DG);
        if (fin) finish_ray();
        DIAG_MARK(dg, fin, DG);
    }
    unsigned long long* cnt = P.counters + WF_NCTR * (blockIdx.x & (WF_SHARDS - 1));
    // a generation's first iteration lists camera rays only (every slot FREE), the others extension
    // rays only; lane 0 carries the wave's count
    const uint32_t c_wave = lane == 0 ? c_listed : 0u;
    block_add<4>(cnt + 0, P.start ? c_wave : 0u, red);
    // extension rays: per iteration where it has a counter (the paths that went on; the host adds
    // them into counter 1)
    block_add<4>(cnt + (P.iter > 0 && P.iter < WF_ITER_CTRS ? WF_CTR_ITER + P.iter : 1), P.start ? 0u : c_wave, red);
    if (DG) block_add<4>(cnt + 15, dg.node_iters, red);
    if (DG && lane == 0) {
        atomicAdd(cnt + 10, (unsigned long long)dg.fetch);
        atomicAdd(cnt + 11, (unsigned long long)dg.node);
        atomicAdd(cnt + 12, (unsigned long long)dg.leaf);
        atomicAdd(cnt + 13, (unsigned long long)dg.fin);
        atomicAdd(cnt + 14, (unsigned long long)dg.outer);
        atomicAdd(cnt + 3, (unsigned long long)dg.lat);  // (counter 3: unused by the shipped kernels)
    }
    if (STATS) {
        block_add<4>(cnt + 4, st.nodes, red);
        block_add<4>(cnt + 5, st.clusters, red);
        block_add<4>(cnt + 6, st.prims, red);
#ifdef MFX_DIAG_OCCLUSION
        block_add<4>(cnt + 13, st.after_nodes, red);
        block_add<4>(cnt + 14, st.after_leaves, red);
#endif
    }
}

// ------------------------------------------------------------------------------------------------
// k_camera: a generation's first iteration, camera rays traced as packets (MFX_CAMERA_PACKETS). A
// 64-slot window is one 8x8 tile of one sample: its 64 camera rays are coherent, so
// the wave traces them together (packet_closest: uniform nodes through scalar loads, one lane per
// ray). Writes what k_extend writes for a camera ray: the hit point and HIT | FRESH | shade index,
// or MISS | FRESH. Flat scenes only (two-level scenes take k_extend).
// ------------------------------------------------------------------------------------------------
#ifndef MFX_CAM_WAVES
// k_camera's register budget: waves per SIMD (a packet walk is one chain of scalar loads per wave).
// Five (96 VGPRs, 56 B of spill) beat four (112 VGPRs, none): 4.30 -> 4.12 ms per C2 launch, Renault
// 6.46 -> 6.19 (interleaved A/B, profiles/r06/r06r_ab_camera_five_waves.txt): the walk waits on its
// loads more than it issues, and the fifth wave fills those waits
#define MFX_CAM_WAVES 5
#endif
template <bool STATS>
__global__ void __launch_bounds__(256, MFX_CAM_WAVES) k_camera(WfParams P) {
    extern __shared__ int lds_all[];
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    uint64_t* stm = (uint64_t*)lds_all + wave * P.stack_size;  // per wave: stack masks, then nodes
    int* stk = (int*)((uint64_t*)lds_all + 4 * P.stack_size) + wave * P.stack_size;
    uint32_t* red = (uint32_t*)((int*)((uint64_t*)lds_all + 4 * P.stack_size) + 4 * P.stack_size);
    // the camera in LDS (read per window), not held in scalar registers through the packet walk
    MfxCamera* cam_lds = (MfxCamera*)(red + 16);
    if (threadIdx.x < sizeof(MfxCamera) / 8) ((double*)cam_lds)[threadIdx.x] = ((const double*)P.cam_dev)[threadIdx.x];
    // the reference-leaf arrays too (as k_shadow): `nodes` and `slots` alone stay in scalar registers
    SceneRefs* refs_lds = (SceneRefs*)(cam_lds + 1);
    if (threadIdx.x == 64) *refs_lds = SceneRefs{(const int32_t*)P.refs_dev[0], (const uint8_t*)P.refs_dev[1]};
    __syncthreads();
    const SceneView S{P.nodes, P.slots, nullptr, nullptr, P.inst, nullptr, 0, nullptr, 0, refs_lds};
    const int shard_size = P.pool / WF_SHARDS;
    Scanner sc{};
    sc.shard = blockIdx.x & (WF_SHARDS - 1);
    uint32_t c_primary = 0;
    Stats st{0, 0, 0};
    uint32_t pk_nodes = 0, pk_slots = 0;  // STATS: the wave's own node and slot fetches (every lane counts them)
#if MFX_DIAG_STAMPS == 3
    // the wave's cycles per phase (window scan, camera ray, node steps, leaf tests, result writes) and
    // its node steps and leaf visits (scripts/camera_phases.py); the shipped build has none of it
    uint64_t ph[4] = {0, 0, 0, 0}, t_scan = 0, t_gen = 0, t_out = 0, t_last = stamp();
#define CAM_MARK(acc)                  \
    do {                               \
        const uint64_t _t = stamp();   \
        (acc) += _t - t_last;          \
        t_last = _t;                   \
    } while (0)
#else
#define CAM_MARK(acc) \
    do {              \
    } while (0)
#endif
    // Every slot is FREE in a generation's first iteration (wf_trace zeroes the state words), so the
    // windows are taken without reading them, and a window is one 8x8 tile of one sample: its
    // (sample, tile) come from one wave-uniform path_pixel (scalar arithmetic), the lanes' pixels by
    // offset (the same x, y, sample path_pixel gives each slot; r06: the per-lane 32-bit divisions and
    // state loads were the window scan's 12 % of k_camera's wave time, scripts/latency_roof.py)
    while (sc.window<false>(P.ctl + WF_CTL_EXT, P.chunk, shard_size, P.state, nullptr, P.ctl + WF_CTL_CLOSED_EXT)) {
        const int jw = __builtin_amdgcn_readfirstlane(sc.win_next);
        sc.win_next += 64;
        const int j = jw + lane;
        int x = 0, y = 0;
        int64_t smp = 0;
        path_pixel(P, P.path_base + jw, x, y, smp);  // the window's first slot: its tile's corner
        x += lane & 7;
        y += lane >> 3;
        // edge-tile padding starts no path
        const bool act = j < P.total && x < P.width && y < P.height;
        if (!__any(act)) continue;
        CAM_MARK(t_scan);
        DV o = dv(0, 0, 0), d = dv(0, 0, 1);
        if (act) {  // PixelIntegrator.Sample (Integrators.fs:167-169) + GetRay (Camera.fs:134-139)
            const int64_t pixel = (int64_t)x * P.height + y;  // Color[w,h] x-major
            const int64_t gsample = P.sample_base + P.part_index + smp * P.part_count;
            const uint64_t key = path_key(P.seed, (uint64_t)pixel, (uint64_t)gsample);
            uint32_t rn = 0;
            const double u = ((double)x + rng_next(key, rn)) / (double)P.width;
            const double v = ((double)y + rng_next(key, rn)) / (double)P.height;
            const MfxCamera& CAM = *cam_lds;
            const DV target = vadd(vadd(ld3(CAM.topleft), vmul(ld3(CAM.right), u)), vmul(ld3(CAM.down), v));
            o = ld3(CAM.position);
            d = vnormalize(vsub(target, o));
            c_primary++;
        }
        Best B;
#if MFX_DIAG_STAMPS == 3
        CAM_MARK(t_gen);
        packet_closest<STATS, true>(S, act, o, d, 99999999., B, stk, stm, st, pk_nodes, pk_slots, ph);
        t_last = stamp();
#else
        packet_closest<STATS>(S, act, o, d, 99999999., B, stk, stm, st, pk_nodes, pk_slots);  // Integrators.fs:108
#endif
        if (act) {
            if (B.found) {
                const DV hp = vadd(o, vmul(d, B.t));  // Ray.PointAtParameter (Ray.fs:8-9)
                P.ox[j] = hp.x; P.oy[j] = hp.y; P.oz[j] = hp.z;
                P.state[j] = ((B.info & MFX_INFO_SHADE_MASK) << WF_SHADE_SHIFT) | WF_HIT | WF_FRESH;
            } else {
                P.state[j] = WF_MISS | WF_FRESH;
            }
        }
        CAM_MARK(t_out);
    }
#undef CAM_MARK
    unsigned long long* cnt = P.counters + WF_NCTR * (blockIdx.x & (WF_SHARDS - 1));
    block_add<4>(cnt + 0, c_primary, red);
#if MFX_DIAG_STAMPS == 3
    if (lane == 0) {  // (MFX_DIAG_ITER prints counters 10..17 as "stamps ... outer ... node ... scan shade")
        atomicAdd(cnt + 10, (unsigned long long)t_scan);
        atomicAdd(cnt + 11, (unsigned long long)t_gen);
        atomicAdd(cnt + 12, (unsigned long long)ph[0]);
        atomicAdd(cnt + 13, (unsigned long long)ph[1]);
        atomicAdd(cnt + 14, (unsigned long long)t_out);
        atomicAdd(cnt + 15, (unsigned long long)ph[2]);
        atomicAdd(cnt + 16, (unsigned long long)ph[3]);
    }
#endif
    if (STATS) {
        block_add<4>(cnt + 4, st.nodes, red);
        block_add<4>(cnt + 5, st.clusters, red);
        block_add<4>(cnt + 6, st.prims, red);
        // packet fetches, once per wave (lane 0's count): mfx_ray_counts out[10], out[11]
        block_add<4>(cnt + 10, lane == 0 ? pk_nodes : 0u, red);
        block_add<4>(cnt + 11, lane == 0 ? pk_slots : 0u, red);
    }
}

// the fields path_pixel and path_key read, in k_shadow's LDS (after its array pointers): a shading
// vertex derives its path's key from the slot, and these are not held in scalar registers through
// the traversal loop
struct PixParams {
    int64_t path_base, base_q, base_smp, sample_base;
    uint64_t seed;
    int32_t width, height, band_index, band_count, band_rows, part_index, part_count, pad;
};
// k_shadow's array pointers in its LDS (after the light)
struct ShdPtrs {
    double *ox, *oy, *oz, *dx, *dy, *dz, *vei, *vls;
    WfMat* vmat;
    uint32_t* rn;
    int32_t* depth;
    const MfxShade* shade;
    int32_t* fstate;
    const int32_t* qslot;
    double *nox, *noy, *noz, *ndx, *ndy, *ndz;
    uint32_t* nrn;
    int32_t *ndepth, *nstate, *nslot;
    unsigned long long* ncount;
    unsigned long long *ctl, *counters;
    int32_t* state;
    const unsigned long long* qcount;
};

// ------------------------------------------------------------------------------------------------
// k_shadow: shade HIT slots (listed at scan time), trace the vertex's shadow ray, continue or finish
// ------------------------------------------------------------------------------------------------
// Q: the instance that reads a ray queue (P.qslot) or writes the next one (P.ncount), MFX_RAY_QUEUE
template <bool STATS, bool SPILL, int WAVES, int SK, bool Q>
__global__ void __launch_bounds__(256, WAVES) k_shadow(WfParams P) {
    constexpr bool INST = SK == WF_SK_INST, SLDS = SK == WF_SK_SLDS;
    extern __shared__ int lds_all[];
#if MFX_NODE_F16
    const TopNodes tn{(const float4*)lds_all, P.ntop_shd, P.nodes_h};
#else
    const TopNodes tn{(const float4*)lds_all, P.ntop_shd};
#endif
    MfxInstance* inst_lds = (MfxInstance*)(lds_all + P.ntop_shd * 32);
    int4* slot_lds = (int4*)(inst_lds + (INST ? P.ninst_lds : 0));
    const int nslot = SLDS ? P.nslot_shd : 0;
    int* lds = (int*)(slot_lds + 5 * nslot);
    uint8_t* pend_base = (uint8_t*)(lds + 4 * P.stack_lds_shd * 64);
    uint32_t* red = (uint32_t*)(pend_base + 4 * PendShd::BYTES);
    // the light, after the four waves' shade lists (8-B aligned): copied before load_top_nodes' barrier
    MfxLight* light_lds = (MfxLight*)((int*)(red + 16) + 4 * 2 * WF_SHD_LIST);
    if (threadIdx.x < sizeof(MfxLight) / 8)
        ((double*)light_lds)[threadIdx.x] = ((const double*)P.light_dev)[threadIdx.x];
    if (threadIdx.x == 0)
        *(ShdPtrs*)(light_lds + 1) = ShdPtrs{P.ox, P.oy, P.oz, P.dx, P.dy, P.dz, P.vei, P.vls, P.vmat, P.rn, P.depth,
                                            P.shade, P.fstate, P.qslot, P.nox, P.noy, P.noz, P.ndx, P.ndy, P.ndz,
                                            P.nrn, P.ndepth, P.nstate, P.nslot, P.ncount, P.ctl, P.counters, P.state,
                                            P.qcount};
    SceneRefs* refs_lds = (SceneRefs*)((PixParams*)((ShdPtrs*)(light_lds + 1) + 1) + 1);
    if (threadIdx.x == 2)  // (from device memory: kernel arguments beside `nodes` would be loaded with it)
        *refs_lds = SceneRefs{(const int32_t*)P.refs_dev[0], (const uint8_t*)P.refs_dev[1]};
    if (threadIdx.x == 1)
        *(PixParams*)((ShdPtrs*)(light_lds + 1) + 1) =
            PixParams{P.path_base, P.base_q, P.base_smp, P.sample_base, P.seed, P.width, P.height, P.band_index,
                      P.band_count, P.band_rows, P.part_index, P.part_count, 0};
#if MFX_NODE_F16
    if (P.nodes_h) load_top_nodes_h((float4*)lds_all, P.nodes_h, P.ntop_shd);
    else
#endif
        load_top_nodes((float4*)lds_all, P.nodes, P.ntop_shd);
    if (INST) load_inst_lds(inst_lds, P.inst, P.ninst_lds);
    if (SLDS) load_slots_lds(slot_lds, P.slots, nslot);
    const MfxLight& LT = *light_lds;
    // the pool's and the queues' array pointers, read from LDS where they are used (the shading batch,
    // the records) instead of held in scalar registers through the traversal loop
    const ShdPtrs& C = *(const ShdPtrs*)(light_lds + 1);
    const PixParams& PX = *(const PixParams*)((const ShdPtrs*)(light_lds + 1) + 1);
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    using Stack = typename std::conditional<SPILL, SpillStack, LdsStack>::type;
    const Stack stack = make_stack<SPILL>(lds + wave * P.stack_lds_shd * 64 + lane, P, P.stack_lds_shd);
    const PendShd pd(pend_base + wave * PendShd::BYTES);
    const SceneView S{P.nodes, P.slots, nullptr, nullptr, P.inst, inst_lds, INST ? P.ninst_lds : 0, slot_lds, nslot, refs_lds};
    const int shard_size = P.pool / WF_SHARDS;

    int* shl = (int*)(red + 16) + wave * 2 * WF_SHD_LIST;  // shade list: [0,128) path slots, [128,256) shade indices
    Scanner sc{};
    sc.shard = blockIdx.x & (WF_SHARDS - 1);
    int nshade = 0;      // wave-uniform: hits listed for shading
    int pend_lo = 0, pend_hi = 0;
    bool active = false;
    int s = 0;
    Trav T{};
    double scs = 0.0, ssolid = 0.0;  // the operands of this vertex's direct term a_v (cs, solid; gray light: a_v, -)
    int vflag = 0;  // the lane's vertex: bit 0 the path continues, bit 1 lightable (cos_o < 0),
                    // bits 2..5 its index v, bits 8.. the path's lit mask so far (PD_* below)
    uint32_t c_shadow = 0;
    Stats st{0, 0, 0};
#ifdef MFX_DIAG_OCCLUSION
    uint32_t dg_occ = 0, dg_occ_nodes = 0, dg_occ_leaves = 0;
#endif
    constexpr bool DG = MFX_DIAG_STAMPS == 2;
    DiagAcc dg{};
    if (DG) dg.last = stamp();

    while (true) {
        bool idle = !active;
        uint64_t m = __ballot(idle);
        while (m != 0) {
            if (pend_lo == pend_hi) {
                // list hits from as many windows as it takes (state words only): a camera ray's miss
                // frees its slot (TraceRay returns black, Integrators.fs:137), a later miss finishes
                // its path with the radiance already in the slot
                while (nshade < 64 && sc.window(C.ctl + WF_CTL_SHD, P.chunk_shd, shard_size, C.state, Q ? C.qcount : nullptr, C.ctl + WF_CTL_CLOSED_SHD)) {
                    if (DG) dg.windows++;
                    const int j = sc.win_next + lane;
                    const int sj = sc.word();
                    const int sv = sj & WF_STATE_MASK;
                    const bool hit = (sv & ~WF_FRESH) == WF_HIT;
                    // a pool slot's miss stays as k_extend wrote it: k_resolve takes MISS as finished
                    // (its state word holds the lit vertices) and a camera ray's MISS | FRESH as black
                    if (Q && C.qslot && sv == WF_MISS) {  // a queue entry: its slot finishes (no lit vertex: stays unfinished)
                        const int dw = C.depth[j];
                        if (dw >> WF_LIT_SHIFT) C.fstate[C.qslot[j]] = WF_DONE | ((dw >> WF_LIT_SHIFT) << WF_SHADE_SHIFT);
                    }
                    const uint64_t hm = __ballot(hit);
                    if (hit) {
                        const int r = nshade + __popcll(hm & lanes_below());
                        // sign bit: first vertex; lit_in_hit: the lit mask in bits 28..30 (slots < 2^28)
                        const bool lh = P.lit_in_hit && !(Q && C.qslot);
                        shl[r] = (sv & WF_FRESH) ? (j | (int)0x80000000) : (lh ? j | (int)(((unsigned)sj >> 29) << 28) : j);
                        shl[WF_SHD_LIST + r] = (int)(((unsigned)sj >> WF_SHADE_SHIFT) & (lh ? 0x1ffffffu : 0x0fffffffu));
                    }
                    nshade += __popcll(hm);
                    sc.advance(C.state);
                }
                wave_lds_sync();
                DIAG_MARK(dg, scan, DG);
                if (nshade == 0) break;  // every chunk scanned, every hit shaded, every ray handed out
                // ---- shade up to 64 listed hits with all lanes: one vertex of PathIntegrator.TraceRay
                //      (Integrators.fs:109-136) each; every one yields a shadow ray ----
                const int cnt = nshade < 64 ? nshade : 64;
                const bool own = lane < cnt;
                int j = 0, mat = 0, jr = 0, dw = 0;
                bool first = false;
                DV hp = dv(0, 0, 0), nm = dv(0, 0, 0);
                uint64_t key = 0;
                uint32_t rn = 0;
                if (own) {
                    j = shl[lane] & WF_ENTRY_SLOT;
                    first = shl[lane] < 0;  // draws 2, depth max_depth, no lit vertex: implicit
                    const int slot = shl[WF_SHD_LIST + lane];
                    jr = (Q && C.qslot) ? C.qslot[j] : j;
                    // remaining depth | lit mask << 8: in place with lit_in_hit, the iteration's and
                    // the mask the state word carried; otherwise the depth word
                    dw = first ? P.max_depth
                               : ((P.lit_in_hit && !(Q && C.qslot))
                                      ? (P.max_depth - P.iter) | ((((unsigned)shl[lane] >> 28) & 7) << WF_LIT_SHIFT)
                                      : C.depth[j]);
                    hp = dv(C.ox[j], C.oy[j], C.oz[j]);
                    const MfxShade sh = C.shade[slot];
                    if ((sh.prim_kind & 3) == MFX_KIND_SPHERE) nm = vnormalize(vsub(hp, ld3(sh.n)));  // Sphere.fs:39-43
                    else nm = ld3(sh.n);
                    mat = sh.material;
                    // the key k_extend derived for the path's camera ray (same expressions), derived
                    // again at every vertex from the path's slot instead of stored (8 B written at the
                    // first vertex and read at every later one: C2 +0.5 %, r05m)
                    {
                        int x, y;
                        int64_t smp;
                        path_pixel(PX, PX.path_base + jr, x, y, smp);
                        const int64_t pixel = (int64_t)x * PX.height + y;
                        key = path_key(PX.seed, (uint64_t)pixel, (uint64_t)(PX.sample_base + PX.part_index + smp * PX.part_count));
                    }
                    rn = first ? 2u : C.rn[j];  // the camera ray drew u, v
                }
                // the depth -1 query's result is discarded (Integrators.fs:109): never traced
                const bool cn = own && (dw & 0xff) - 1 >= 0;
                // MFX_RAY_QUEUE: a continuing path's entry in the next queue, in the range of its
                // source shard (capacity: that shard's size), one atomic per shard in the batch
                int qi = 0;
                if (Q && C.ncount) {
                    const int g = cn ? j / shard_size : 0;
                    uint64_t rem = __ballot(cn);
                    while (rem) {
                        const int gl = __shfl(g, __builtin_ctzll(rem));
                        const uint64_t gm = __ballot(cn && g == gl);
                        unsigned long long base = 0;
                        if (lane == __builtin_ctzll(gm)) base = atomicAdd(C.ncount + gl * WF_HS, (unsigned long long)__popcll(gm));
                        base = __shfl(base, __builtin_ctzll(gm));
                        if (cn && g == gl) qi = gl * shard_size + (int)base + __popcll(gm & lanes_below());
                        rem &= ~gm;
                    }
                }
                wave_lds_sync();  // every owner has read its shl entries: shl[0, 64) is the sampler's scratch
                const VertexSample V = sample_vertex(LT, own, hp, nm, key, rn, shl);
                if (own) {
                    const DV wi = V.wi, unit = V.unit;
                    const double dist = V.dist, cs = V.cs, solid = V.solid;
                    const bool lightable = V.lightable;
                    const int v = P.max_depth - (dw & 0xff);          // this vertex's index
                    // the operands of col = INVPI * a * ei * TwoPi (Material.fs:36), c_v (k_resolve)
                    C.vei[v * P.vstride + jr] = V.ei;
                    C.vmat[v * P.vstride + jr] = (WfMat)mat;
                    if (Q && cn && C.ncount) {  // the next vertex's ray in the next queue (its depth word and
                                           // state are written after the shadow ray)
                        C.nox[qi] = hp.x; C.noy[qi] = hp.y; C.noz[qi] = hp.z;
                        C.ndx[qi] = wi.x; C.ndy[qi] = wi.y; C.ndz[qi] = wi.z;
                        C.nrn[qi] = rn;
                        C.nslot[qi] = jr;
                    } else if (cn) {  // what the next vertex reads, in place
                        C.rn[j] = rn;
                        C.dx[j] = wi.x; C.dy[j] = wi.y; C.dz[j] = wi.z;
                    }
                    // shadow bvh.Hit(Ray(hit.point, unit), 1e-6, dist - 1e-6) (Integrators.fs:44)
                    pd.slot[lane] = (Q && cn && C.ncount) ? qi : j;
                    pd.flag[lane] = (cn ? 1 : 0) | (lightable ? 2 : 0) | (v << 2) | (dw & ~0xff);
                    pd.v[0 * 64 + lane] = unit.x; pd.v[1 * 64 + lane] = unit.y; pd.v[2 * 64 + lane] = unit.z;
                    pd.v[3 * 64 + lane] = dist - 1e-6;
                    // a gray light: the direct term itself, (cs * (solid * I)) / pdf_li (Integrators.fs:52,
                    // Light.fs:52-53), the expression k_resolve evaluates per channel otherwise
                    pd.v[4 * 64 + lane] = P.gray_light ? (cs * (solid * LT.color[0])) / LT.pdf : cs;
                    pd.v[5 * 64 + lane] = solid;
                    c_shadow++;
                }
                // the unshaded rest of the list moves to its front
                const int rest = nshade - cnt;
                int mv_j = 0, mv_s = 0;
                if (lane < rest) { mv_j = shl[cnt + lane]; mv_s = shl[WF_SHD_LIST + cnt + lane]; }
                wave_lds_sync();
                if (lane < rest) { shl[lane] = mv_j; shl[WF_SHD_LIST + lane] = mv_s; }
                wave_lds_sync();
                nshade = rest;
                pend_lo = 0;
                pend_hi = cnt;
                DIAG_MARK(dg, shade, DG);
                continue;
            }
            const int avail = pend_hi - pend_lo;
            const int rank = __popcll(m & lanes_below());
            if (idle && rank < avail) {
                const int e = pend_lo + rank;
                s = pd.slot[e];
                vflag = pd.flag[e];
                scs = pd.v[4 * 64 + e];
                ssolid = P.gray_light ? 0.0 : pd.v[5 * 64 + e];
                // origin = the hit point k_extend stored (a cache hit: the shading just read it), or
                // its copy in the next queue. That copy (nox..noz, and nslot below) was stored in this
                // kernel by the lane that shaded the hit, which may be another lane of this wave: the
                // read is ordered after that store by the wave_lds_sync() calls that end the shading
                // batch (release / acquire fences at wavefront scope cover global memory as well as
                // LDS), and one wave's vector memory operations reach its L1 in order.
                const bool nq = Q && (vflag & 1) && C.ncount;
                const double* hx = nq ? C.nox : C.ox;
                const double* hy = nq ? C.noy : C.oy;
                const double* hz = nq ? C.noz : C.oz;
                trav_begin(T, S, dv(hx[s], hy[s], hz[s]), dv(pd.v[0 * 64 + e], pd.v[1 * 64 + e], pd.v[2 * 64 + e]),
                           pd.v[3 * 64 + e]);

#ifdef MFX_DIAG_OCCLUSION
                T.n0 = st.nodes;
                T.l0 = st.clusters;
#endif
                idle = false;
                active = true;
            }
            const int pm = __popcll(m);
            pend_lo += pm < avail ? pm : avail;
            m = __ballot(idle);
        }
        if (!__any(active)) break;
        DIAG_MARK(dg, fetch, DG);
        if (DG) dg.outer++;
        bool fin = false;
#ifdef MFX_DIAG_SKIP_SHADOW_TRAV
        if (active) {
            T.B.found = false;
            fin = true;
        }
#else
        if (active) fin = trav_step<true, STATS, INST, SLDS>(T, S, stack, tn, st, dg, DG);
#endif
        DIAG_MARK(dg, leaf, DG);
        if (fin) {
#ifdef MFX_DIAG_OCCLUSION  // STATS build: occluded shadow rays and their node / cluster visits
            if (STATS && T.B.found) {
                dg_occ++;
                dg_occ_nodes += st.nodes - T.n0;
                dg_occ_leaves += st.clusters - T.l0;
            }
#endif
            const int v = (vflag >> 2) & 15;
            int mask = (vflag >> WF_LIT_SHIFT) & 0xffff;
            // MFX_RAY_QUEUE: s is the path's next-queue entry (it continues) or its entry in this
            // iteration's queue; its slot is read back where the slot's records are written
            const bool nq = Q && cont0(vflag) && C.ncount;
            if (!T.B.found && (vflag & 2)) {  // unoccluded: record the operands of its direct term a_v
                const int jr = nq ? C.nslot[s] : ((Q && C.qslot) ? C.qslot[s] : s);
                double* vl = C.vls + (int64_t)(2 * v) * P.vstride + jr;
                vl[0] = scs;
                if (!P.gray_light) vl[P.vstride] = ssolid;
                mask |= 1 << v;
            }
            const bool cont = (vflag & 1) != 0;
            // continue with the next vertex's remaining depth; or finished: k_resolve folds the
            // recorded vertices (none lit: nothing to add, FREE)
            const int dwn = ((P.max_depth - v - 1) & 0xff) | (mask << WF_LIT_SHIFT);
            // in place, NEED_EXT carries the lit mask for k_extend's pending entries (lit_in_entry)
            const int need = WF_NEED_EXT | (nq ? 0 : mask << WF_SHADE_SHIFT);
            if (nq) {
                C.ndepth[s] = dwn;
                C.nstate[s] = need;
            } else if (Q && (C.ncount || C.qslot)) {  // finished; the pool's slot keeps its final words
                if (mask) C.fstate[C.qslot ? C.qslot[s] : s] = WF_DONE | (mask << WF_SHADE_SHIFT);
            } else {
                if (cont && !P.lit_in_hit) C.depth[s] = dwn;
                C.state[s] = cont ? need : (mask ? WF_DONE | (mask << WF_SHADE_SHIFT) : WF_FREE);
            }
            active = false;
        }
        DIAG_MARK(dg, fin, DG);
    }
    unsigned long long* cnt = C.counters + WF_NCTR * (blockIdx.x & (WF_SHARDS - 1));
    block_add<4>(cnt + 2, c_shadow, red);
    if (DG) block_add<4>(cnt + 15, dg.node_iters, red);
    if (DG && lane == 0) {
        atomicAdd(cnt + 10, (unsigned long long)dg.fetch);
        atomicAdd(cnt + 11, (unsigned long long)dg.node);
        atomicAdd(cnt + 12, (unsigned long long)dg.leaf);
        atomicAdd(cnt + 13, (unsigned long long)dg.fin);
        atomicAdd(cnt + 14, (unsigned long long)dg.outer);
        atomicAdd(cnt + 16, (unsigned long long)dg.scan);
        atomicAdd(cnt + 17, (unsigned long long)dg.shade);
        atomicAdd(cnt + 3, (unsigned long long)dg.lat);
    }
    if (STATS) {
        block_add<4>(cnt + 7, st.nodes, red);
#ifdef MFX_DIAG_OCCLUSION
        block_add<4>(cnt + 10, dg_occ, red);
        block_add<4>(cnt + 11, dg_occ_nodes, red);
        block_add<4>(cnt + 12, dg_occ_leaves, red);
#endif
        block_add<4>(cnt + 8, st.clusters, red);
        block_add<4>(cnt + 9, st.prims, red);
    }
}

#ifndef WF_RES_VERTS
#define WF_RES_VERTS 4  // vertices k_resolve loads in one round (max_depth 3 paths); deeper ones in a loop
#endif
#ifndef WF_RES_MAT_LDS
#define WF_RES_MAT_LDS 256  // materials whose albedo k_resolve keeps in LDS (more: read from global memory)
#endif
#ifndef WF_RES_SAMPLES
#define WF_RES_SAMPLES 1  // samples of a pixel whose path records k_resolve loads together
#endif

// One path's vertex records as loaded by k_resolve: for the first WF_RES_VERTS vertices up to its
// deepest lit one, ei and the material; cs and solid for the lit ones. Loaded in one round of
// independent loads (the state word came in the round before), so a path costs two
// dependent memory round trips instead of one per vertex and field.
struct PathRec {
    int mask;  // lit-vertex mask (0: black path, or not a finished path of this generation)
    double ei[WF_RES_VERTS], cs[WF_RES_VERTS], so[WF_RES_VERTS];
    int mat[WF_RES_VERTS];
};
__device__ __forceinline__ void load_path(const WfParams& P, int64_t j, int mask, PathRec& R) {
    R.mask = mask;
    if (mask == 0) return;
    const int top = 31 - __builtin_clz(mask);
#pragma unroll
    for (int v = 0; v < WF_RES_VERTS; ++v) {
        R.ei[v] = 0.0; R.cs[v] = 0.0; R.so[v] = 0.0; R.mat[v] = 0;
        if (v <= top) {
            R.ei[v] = P.vei[v * P.vstride + j];
            R.mat[v] = P.vmat[v * P.vstride + j];
            if ((mask >> v) & 1) {
                const double* vl = P.vls + (int64_t)(2 * v) * P.vstride + j;
                R.cs[v] = vl[0];  // (a gray light: a_v itself)
                if (!P.gray_light) R.so[v] = vl[P.vstride];
            }
        }
    }
}
// The path's radiance: its vertices folded from the deepest lit one back to the camera, f starting
// as TraceRay below the deepest lit vertex (Color(), black):
//   c_v = col = TwoPi * (ei * (INVPI * a))            (Material.fs:36, the expression k_shadow had)
//   a_v = (cs * (solid * I)) / pdf_li, 0 if unlit     (Integrators.fs:52, Light.fs:52-53)
//   f  <- (a_v + f) * c_v                             (Integrators.fs:135-136, pdf = 1)
__device__ __forceinline__ void fold_vertex(const WfParams& P, bool lit, double ei, int mat, double cs, double so,
                                            const double* alb_lds, double& fx, double& fy, double& fz) {
    const MfxLight& LT = P.light;
    const double* al = mat < WF_RES_MAT_LDS ? alb_lds + 3 * mat : P.albedo + 3 * mat;
    const double cx = TWOPI * (ei * (INVPI * al[0]));
    const double cy = TWOPI * (ei * (INVPI * al[1]));
    const double cz = TWOPI * (ei * (INVPI * al[2]));
    double ax = 0.0, ay = 0.0, az = 0.0;
    if (lit && P.gray_light) {  // cs holds a_v, recorded by k_shadow with the same expression
        ax = ay = az = cs;
    } else if (lit) {
        ax = (cs * (so * LT.color[0])) / LT.pdf;
        ay = (cs * (so * LT.color[1])) / LT.pdf;
        az = (cs * (so * LT.color[2])) / LT.pdf;
    }
    fx = (ax + fx) * cx;
    fy = (ay + fy) * cy;
    fz = (az + fz) * cz;
}
__device__ __forceinline__ void fold_path(const WfParams& P, int64_t j, const PathRec& R, const double* alb_lds,
                                          double& fx, double& fy, double& fz) {
    const int top = 31 - __builtin_clz(R.mask);
    // vertices deeper than the batched records (max_depth >= WF_RES_VERTS), read here
    for (int v = top; v >= WF_RES_VERTS; --v) {
        const bool lit = (R.mask >> v) & 1;
        const double* vl = P.vls + (int64_t)(2 * v) * P.vstride + j;
        fold_vertex(P, lit, P.vei[v * P.vstride + j], P.vmat[v * P.vstride + j], lit ? vl[0] : 0.0,
                    lit ? vl[P.vstride] : 0.0, alb_lds, fx, fy, fz);
    }
    // the batched ones, indices known at compile time (the records stay in registers)
#pragma unroll
    for (int v = WF_RES_VERTS - 1; v >= 0; --v)
        if (v <= top) fold_vertex(P, (R.mask >> v) & 1, R.ei[v], R.mat[v], R.cs[v], R.so[v], alb_lds, fx, fy, fz);
}

// ------------------------------------------------------------------------------------------------
// k_resolve: after a generation, every pixel adds its finished paths' radiance in sample order
// (PixelIntegrator.Sample: color <- color + TraceRay(...), Integrators.fs:169). A path's radiance
// is its recorded vertices folded from the deepest lit one back to the camera: TraceRay returns
// (l / pdf_li + TraceRay(next)) * col / pdf (Integrators.fs:135-136; pdf = 1, so the division is
// exact), black below the last lit vertex, and l = 0 at an occluded or unlit one. One thread per
// tile-ordered pixel position q; for a fixed sample, consecutive q are consecutive slots, so the
// loads are coalesced. No atomics: one thread owns each pixel, generations are stream-ordered.
// The records of WF_RES_SAMPLES samples are loaded together (state words, which carry a finished
// path's lit mask, then vertex records: two rounds of independent loads), then folded and added in
// sample order.
// Render-ahead (P.film, the frames mode): the samples are one-sample render calls. Each adds its
// 1-spp image — 0.0 + its path, what a one-sample call's zeroed accumulator holds, 0.0 for a black
// one — to the film state in sample order (Film.AddSample, Film.fs:18-23: film + frame / 1.0),
// and with P.frames writes that call's RGBA8 frame (PostProcessAndToScreenBuffer of film /
// frameCount, Scene.fs:315-330; frameCount = count0 + the sample's index + 1): the FP64 operations
// film_post_kernel runs per call, in the same order, so every frame is that call's bytes. The film
// state (P.film) carries across a call's generations.
// ------------------------------------------------------------------------------------------------
// FRAMES: the render-ahead instance (P.film); the accumulator instance carries none of its code
// (with it, k_resolve took 99 VGPRs instead of 88, 4 waves per SIMD instead of 5, and twice the time)
template <bool FRAMES>
__global__ void __launch_bounds__(256) k_resolve(WfParams P) {
    __shared__ double alb[3 * WF_RES_MAT_LDS];
    const int nm = P.nmat < WF_RES_MAT_LDS ? P.nmat : WF_RES_MAT_LDS;
    for (int i = threadIdx.x; i < 3 * nm; i += blockDim.x) alb[i] = P.albedo[i];
    __syncthreads();
    const int tiles_x = (P.width + 7) >> 3;
    const int64_t per_sample = (int64_t)tiles_x * P.band_rows * 64;
    int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (P.res_ntx > 0) {  // a band of tile columns (mfx_sample's banded resolve): thread -> its tile's q
        const int64_t tl = q >> 6;
        if (tl >= (int64_t)P.res_ntx * P.band_rows) return;
        q = ((tl / P.res_ntx) * tiles_x + P.res_tx0 + tl % P.res_ntx) * 64 + (q & 63);
    }
    if (q >= per_sample) return;
    const int64_t tile = q >> 6;
    const int within = (int)(q & 63);
    const int x = (int)(tile % tiles_x) * 8 + (within & 7);
    const int y = band_tile_row(P.band_index, P.band_count, (int)(tile / tiles_x)) * 8 + (within >> 3);  // the band's film row
    if (x >= P.width || y >= P.height) return;
    const int64_t npix = (int64_t)P.width * P.height;
    const int64_t pixel = (int64_t)x * P.height + y;
    const int64_t end = P.path_base + P.total;
    double* acc = FRAMES ? P.film : P.accum;
    double ax = acc[pixel], ay = acc[npix + pixel], az = acc[2 * npix + pixel];
    constexpr int U = WF_RES_SAMPLES;
    for (int64_t smp0 = P.path_base / per_sample; smp0 * per_sample < end; smp0 += U) {
        int64_t jv[U];
        bool in[U];
        int sw[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t p = (smp0 + u) * per_sample + q;
            in[u] = p >= P.path_base && p < end;
            jv[u] = in[u] ? p - P.path_base : 0;
            sw[u] = in[u] ? P.state[jv[u]] : 0;
        }
        int mask[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            mask[u] = ((sw[u] & WF_STATE_MASK) == WF_DONE || (sw[u] & WF_STATE_MASK) == WF_MISS)
                          ? ((unsigned)sw[u] >> WF_SHADE_SHIFT) & 0xffff : 0;
        }
        PathRec R[U];
#pragma unroll
        for (int u = 0; u < U; ++u) load_path(P, jv[u], mask[u], R[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!in[u]) continue;
            double fx = 0.0, fy = 0.0, fz = 0.0;
            if (R[u].mask) fold_path(P, jv[u], R[u], alb, fx, fy, fz);
            if (FRAMES) {
                ax = ax + (0.0 + fx) / 1.0;
                ay = ay + (0.0 + fy) / 1.0;
                az = az + (0.0 + fz) / 1.0;
                if (P.frames) {
                    const double cnt = P.count0 + (double)(smp0 + u + 1);
                    uint8_t* o = P.frames + (smp0 + u) * npix * 4 + ((int64_t)y * P.width + x) * 4;
                    o[0] = post_byte(ax / cnt);
                    o[1] = post_byte(ay / cnt);
                    o[2] = post_byte(az / cnt);
                    o[3] = 255;
                }
            } else if (R[u].mask) {  // a path with no lit vertex adds nothing
                ax += fx;
                ay += fy;
                az += fz;
            }
        }
    }
    acc[pixel] = ax;
    acc[npix + pixel] = ay;
    acc[2 * npix + pixel] = az;
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
// top nodes, instances, slots, stacks, pending-ray lists, block reduction scratch (64 B) and, for
// k_shadow, the shade lists
static size_t wf_lds_bytes(int stack_size, bool shadow, int ntop, int ninst, int nslot = 0) {
    const size_t stacks = (size_t)ntop * sizeof(MfxNode) + (size_t)ninst * sizeof(MfxInstance) + (size_t)nslot * 80 +
                          (size_t)4 * stack_size * 64 * sizeof(int);
    return shadow ? stacks + 4 * PendShd::BYTES + 64 + 4 * 2 * WF_SHD_LIST * sizeof(int) + sizeof(MfxLight) + sizeof(ShdPtrs) +
                        sizeof(PixParams) + sizeof(SceneRefs)
                  : stacks + 4 * WF_EXT_PEND * sizeof(int) + 64;
}

// Blocks per CU the LDS allows. gfx950 allocates LDS in 1,280-byte granules out of 160 KB per CU;
// hipOccupancyMaxActiveBlocksPerMultiprocessor counts finer granules, so near a boundary it
// reports one block more than fits (measured: k_shadow at 53,952 B per block runs 2 blocks per CU
// where the API says 3, a 10 % loss).
static int wf_lds_blocks(size_t bytes) {
    const size_t g = 1280, per_cu = 160 * 1024;
    return (int)(per_cu / ((bytes + g - 1) / g * g));
}

// the scene kind a kernel instance is built for (k_extend / k_shadow SK)
static int scene_kind(bool inst, int nslot) { return inst ? WF_SK_INST : (nslot > 0 ? WF_SK_SLDS : WF_SK_FLAT); }

template <int SK>
static const void* occ_kernel(bool shadow, bool spill) {
    if (shadow)
        return spill ? (const void*)k_shadow<false, true, 4, SK, false> : (const void*)k_shadow<false, false, 4, SK, false>;
    // (the START instance: a superset of the bounce instance's code)
    return spill ? (const void*)k_extend<false, true, SK, false, true> : (const void*)k_extend<false, false, SK, false, true>;
}

hipError_t mfx_wf_kernel_occupancy(bool shadow, int stack_lds, bool spill, int ntop, int ninst, int* blocks_per_cu,
                                   int nslot) {
    const size_t lds = wf_lds_bytes(stack_lds, shadow, ntop, std::min(ninst, WF_INST_LDS), nslot);
    const int sk = scene_kind(ninst > 0, nslot);
    const void* k = sk == WF_SK_INST ? occ_kernel<WF_SK_INST>(shadow, spill)
                                     : (sk == WF_SK_SLDS ? occ_kernel<WF_SK_SLDS>(shadow, spill) : occ_kernel<WF_SK_FLAT>(shadow, spill));
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k, 256, lds);
    *blocks_per_cu = std::min(*blocks_per_cu, wf_lds_blocks(lds));
    return e;
}

template <bool SPILL, int SK, bool Q, bool START = false>
static void launch_extend_q(const WfParams& P, int grid, bool stats, hipStream_t st, size_t lds) {
    if (stats)
        hipLaunchKernelGGL((k_extend<true, SPILL, SK, Q, START>), dim3(grid), dim3(256), lds, st, P);
    else
        hipLaunchKernelGGL((k_extend<false, SPILL, SK, Q, START>), dim3(grid), dim3(256), lds, st, P);
}
template <bool SPILL, int SK>
static void launch_extend(const WfParams& P, int grid, bool stats, hipStream_t st, size_t lds) {
    if (P.qcount) launch_extend_q<SPILL, SK, true>(P, grid, stats, st, lds);
    else if (P.start) launch_extend_q<SPILL, SK, false, true>(P, grid, stats, st, lds);
    else launch_extend_q<SPILL, SK, false>(P, grid, stats, st, lds);
}
template <bool SPILL, int WAVES, int SK, bool Q>
static void launch_shadow_q(const WfParams& P, int grid, bool stats, hipStream_t st, size_t lds) {
    if (stats)
        hipLaunchKernelGGL((k_shadow<true, SPILL, WAVES, SK, Q>), dim3(grid), dim3(256), lds, st, P);
    else
        hipLaunchKernelGGL((k_shadow<false, SPILL, WAVES, SK, Q>), dim3(grid), dim3(256), lds, st, P);
}
// MFX_SHADOW_Q_WAVES=3 (an A/B knob, VERDICT r05 Next #7): the queue instances of a 4-wave k_shadow
// run the 3-wave build instead (no scratch spill; 3 of the grid's 4 blocks per CU)
static int shadow_q_waves() {
    static const int w = getenv("MFX_SHADOW_Q_WAVES") ? atoi(getenv("MFX_SHADOW_Q_WAVES")) : 0;
    return w;
}
template <bool SPILL, int WAVES, int SK>
static void launch_shadow(const WfParams& P, int grid, bool stats, hipStream_t st, size_t lds) {
    if (P.qslot || P.ncount) {
        if (WAVES == 4 && shadow_q_waves() == 3) launch_shadow_q<SPILL, 3, SK, true>(P, grid / 4 * 3, stats, st, lds);
        else launch_shadow_q<SPILL, WAVES, SK, true>(P, grid, stats, st, lds);
    } else {
        launch_shadow_q<SPILL, WAVES, SK, false>(P, grid, stats, st, lds);
    }
}
template <int SK>
static void launch_shadow_sk(const WfParams& P, int grid, bool stats, hipStream_t st, size_t lds) {
    // k_shadow is compiled for 3 waves per SIMD (up to 168 VGPRs) when its LDS allows no more blocks anyway
    const bool spill = P.stack_lds_shd < P.stack_size, w3 = P.shadow_waves == 3;
    if (spill && w3) launch_shadow<true, 3, SK>(P, grid, stats, st, lds);
    else if (spill) launch_shadow<true, 4, SK>(P, grid, stats, st, lds);
    else if (w3) launch_shadow<false, 3, SK>(P, grid, stats, st, lds);
    else launch_shadow<false, 4, SK>(P, grid, stats, st, lds);
}
template <int SK>
static void launch_extend_sk(const WfParams& P, int grid, bool stats, hipStream_t st, size_t lds) {
    // each kernel keeps its own share of the traversal stack in LDS (the rest spills)
    if (P.stack_lds_ext < P.stack_size) launch_extend<true, SK>(P, grid, stats, st, lds);
    else launch_extend<false, SK>(P, grid, stats, st, lds);
}

static size_t cam_lds_bytes(int stack_size) {
    return (size_t)4 * stack_size * (sizeof(int) + sizeof(uint64_t)) + 64 + sizeof(MfxCamera) + sizeof(SceneRefs);
}

hipError_t mfx_cam_occupancy(int stack_size, int* blocks_per_cu) {
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, (const void*)k_camera<false>, 256,
                                                                      cam_lds_bytes(stack_size));
    return e;
}

static hipError_t launch_iteration(const WfParams& P, int ext_grid, int shd_grid, bool stats, hipStream_t st,
                                   hipEvent_t* ev, size_t lds_e, size_t lds_s) {
    const bool inst = P.inst != nullptr;
    if (!inst && P.start && P.cam_grid > 0) {  // camera rays as packets
        if (stats) hipLaunchKernelGGL(k_camera<true>, dim3(P.cam_grid), dim3(256), cam_lds_bytes(P.stack_size), st, P);
        else hipLaunchKernelGGL(k_camera<false>, dim3(P.cam_grid), dim3(256), cam_lds_bytes(P.stack_size), st, P);
    } else {
        switch (scene_kind(inst, P.nslot_ext)) {
            case WF_SK_INST: launch_extend_sk<WF_SK_INST>(P, ext_grid, stats, st, lds_e); break;
            case WF_SK_SLDS: launch_extend_sk<WF_SK_SLDS>(P, ext_grid, stats, st, lds_e); break;
            default: launch_extend_sk<WF_SK_FLAT>(P, ext_grid, stats, st, lds_e);
        }
    }
    if (ev) {  // between the two kernels (per-stage timing); null: not recorded
        const hipError_t e = hipEventRecord(ev[0], st);
        if (e != hipSuccess) return e;
    }
    switch (scene_kind(inst, P.nslot_shd)) {
        case WF_SK_INST: launch_shadow_sk<WF_SK_INST>(P, shd_grid, stats, st, lds_s); break;
        case WF_SK_SLDS: launch_shadow_sk<WF_SK_SLDS>(P, shd_grid, stats, st, lds_s); break;
        default: launch_shadow_sk<WF_SK_FLAT>(P, shd_grid, stats, st, lds_s);
    }
    return hipSuccess;
}

hipError_t mfx_wf_iteration(const WfParams& P, int ext_grid, int shd_grid, bool stats, hipStream_t st,
                            hipEvent_t* ev) {
    const int ni = P.inst ? P.ninst_lds : 0;
    const size_t lds_e = wf_lds_bytes(P.stack_lds_ext, false, P.ntop_ext, ni, P.nslot_ext);
    const size_t lds_s = wf_lds_bytes(P.stack_lds_shd, true, P.ntop_shd, ni, P.nslot_shd);
    // the chunk heads and, beside them (WF_CTL_Q0 / WF_CTL_Q1), the next queue's shard counts
    unsigned long long* z = P.ctl;
    size_t nz = WF_NCTL;
    if (P.ncount) {
        nz += WF_SHARDS * WF_HS;
        if (P.ncount < P.ctl) z = P.ncount;
    }
    hipError_t e = hipMemsetAsync(z, 0, nz * sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    e = launch_iteration(P, ext_grid, shd_grid, stats, st, ev, lds_e, lds_s);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t mfx_wf_resolve(const WfParams& P, hipStream_t st) {
    const int64_t per_sample = (int64_t)(P.res_ntx > 0 ? P.res_ntx : (P.width + 7) >> 3) * P.band_rows * 64;
    if (P.film) hipLaunchKernelGGL(k_resolve<true>, dim3((unsigned)((per_sample + 255) / 256)), dim3(256), 0, st, P);
    else hipLaunchKernelGGL(k_resolve<false>, dim3((unsigned)((per_sample + 255) / 256)), dim3(256), 0, st, P);
    return hipGetLastError();
}
