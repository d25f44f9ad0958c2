// mfx_build.hip — the traversal BVH built on the GPU (the reference builds its
// BVH on the host, Bvh.Build / Subdivide, BvhNode.fs:24-61, O(N log^2 N) with array copies).
//
// What is built here is exactly the tree of mfx_scene.cpp's host SahBuilder: a binned-SAH BVH2
// over the individual primitives with the same 32 bins per axis in the same FP32 arithmetic
// (-ffp-contract=off on both sides), the same first-minimum rule over (axis, bin), the same leaf
// rule and the same stable partition. The host collapse (BVH4) and image assembly that follow
// therefore produce byte-identical device images from either build (tests/test_gpu_build.py
// compares digests). The reference's own leaf grouping (median split with .NET introsort ties,
// BvhNode.fs:42-61) stays on the host: it decides results through its tie order, not speed.
//
// Breadth-first: one launch per tree level, one wave per node of the level.
//   pass 1  the node's primitive box, centroid box and slot weight (wave min / max / sum)
//   pass 2  3 axes x 32 bins (count, weight, box) with LDS atomics (box bounds as
//           order-preserving ints; counts and weights are integers, so every sum is exact)
//   SAH     lane k holds bin k; prefix and suffix scans by shuffles give every split's cost; the
//           wave argmin keeps the host's tie order (strict <, axes 0..2, bins ascending)
//   pass 3  a leaf, or a stable partition (ballot ranks) through a scratch array and two child
//           tasks for the next level
// Node and leaf indices come from atomic counters, so their numbering differs from the host's
// preorder; nothing downstream depends on it (the collapse follows child references).
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <numeric>

#include "mfx_build.h"

namespace {

constexpr int NB = 32;  // SahBuilder::NB

struct BTask {
    int b, e, parent, side;  // primitive range [b, e) of ids; parent node (-1: root) and child side
};

struct BArgs {
    const float* __restrict__ box;     // [n][6]
    const float* __restrict__ cent;    // [n][3]
    const int* __restrict__ weight;    // [n]
    int* ids;                          // [n] permutation, partitioned in place
    int* tmp;                          // [n] partition scratch
    float* node_box;                   // [n][2][6]
    int* node_child;                   // [n][2]
    int2* leaves;                      // [n]
    int* counters;                     // [0] nodes, [1] leaves, [2] next level's tasks
    float* root_box;                   // [6]
    int* root_ref;
    int max_leaf;
    float c_isect;
};

__device__ __forceinline__ int ford(float f) {  // order-preserving float -> int (no NaNs here)
    const int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float fback(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

__device__ __forceinline__ float wave_min(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_sum(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// FBox::area (mfx_scene.cpp), the same operations
__device__ __forceinline__ float box_area(float lx, float ly, float lz, float hx, float hy, float hz) {
    const float dx = hx - lx, dy = hy - ly, dz = hz - lz;
    if (dx < 0 || dy < 0 || dz < 0) return 0.f;
    return 2.f * (dx * dy + dx * dz + dy * dz);
}

// bin of a centroid coordinate: SahBuilder::build's (int)((c - lo) / ext * NB), clamped
__device__ __forceinline__ int bin_of(float c, float lo, float ext) {
    int k = (int)((c - lo) / ext * NB);
    return min(NB - 1, max(0, k));
}

__global__ void __launch_bounds__(256) k_sah_level(BArgs A, const BTask* __restrict__ tin, int ntin,
                                                   BTask* __restrict__ tout) {
    __shared__ int bins[4][3][NB][8];  // per wave: count, weight, lo xyz, hi xyz (ordered ints)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + wave;
    if (t >= ntin) return;  // the whole wave leaves; no block-wide barrier follows
    const BTask T = tin[t];
    const int b = T.b, e = T.e, n = e - b;
    const uint64_t below = (1ull << lane) - 1ull;

    // ---- pass 1: primitive box, centroid box, weight ----
    float cl[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, ch[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    float bl[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, bh[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    int ws = 0;
    for (int i = b + lane; i < e; i += 64) {
        const int id = A.ids[i];
        for (int a = 0; a < 3; ++a) {
            const float c = A.cent[3 * id + a];
            cl[a] = fminf(cl[a], c);
            ch[a] = fmaxf(ch[a], c);
            bl[a] = fminf(bl[a], A.box[6 * id + a]);
            bh[a] = fmaxf(bh[a], A.box[6 * id + 3 + a]);
        }
        ws += A.weight[id];
    }
    for (int a = 0; a < 3; ++a) {
        cl[a] = wave_min(cl[a]);
        ch[a] = wave_max(ch[a]);
        bl[a] = wave_min(bl[a]);
        bh[a] = wave_max(bh[a]);
    }
    ws = wave_sum(ws);

    bool leaf = n == 1;
    int best_axis = -1, best_split = 0, best_nl = 0;
    float best_cost = FLT_MAX;
    float ext[3];
    for (int a = 0; a < 3; ++a) ext[a] = ch[a] - cl[a];
    if (!leaf) {
        // ---- pass 2: bins ----
        int* bw = &bins[wave][0][0][0];
        for (int q = lane; q < 3 * NB * 8; q += 64) {
            const int f = q & 7;
            bw[q] = f < 2 ? 0 : (f < 5 ? ford(FLT_MAX) : ford(-FLT_MAX));
        }
        wave_sync();
        for (int i = b + lane; i < e; i += 64) {
            const int id = A.ids[i];
            const int w = A.weight[id];
            for (int a = 0; a < 3; ++a) {
                if (!(ext[a] > 0.f)) continue;
                int* s = bw + (a * NB + bin_of(A.cent[3 * id + a], cl[a], ext[a])) * 8;
                atomicAdd(s + 0, 1);
                atomicAdd(s + 1, w);
                for (int c = 0; c < 3; ++c) {
                    atomicMin(s + 2 + c, ford(A.box[6 * id + c]));
                    atomicMax(s + 5 + c, ford(A.box[6 * id + 3 + c]));
                }
            }
        }
        wave_sync();
        // ---- SAH over the 31 split planes of each axis (SahBuilder::build's sweeps) ----
        for (int a = 0; a < 3; ++a) {
            if (!(ext[a] > 0.f)) continue;
            int c = 0, w = 0;
            float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
            if (lane < NB) {
                const int* s = bw + (a * NB + lane) * 8;
                c = s[0];
                w = s[1];
                for (int k = 0; k < 3; ++k) {
                    lo[k] = fback(s[2 + k]);
                    hi[k] = fback(s[5 + k]);
                }
            }
            // suffix over bins lane..NB-1 (right side) and prefix over 0..lane (left side)
            int rc = c, rw = w, lc = c, lw = w;
            float rlo[3], rhi[3], llo[3], lhi[3];
            for (int k = 0; k < 3; ++k) {
                rlo[k] = llo[k] = lo[k];
                rhi[k] = lhi[k] = hi[k];
            }
            for (int o = 1; o < 64; o <<= 1) {
                const int rc2 = __shfl_down(rc, o), rw2 = __shfl_down(rw, o);
                const int lc2 = __shfl_up(lc, o), lw2 = __shfl_up(lw, o);
                float r2lo[3], r2hi[3], l2lo[3], l2hi[3];
                for (int k = 0; k < 3; ++k) {
                    r2lo[k] = __shfl_down(rlo[k], o);
                    r2hi[k] = __shfl_down(rhi[k], o);
                    l2lo[k] = __shfl_up(llo[k], o);
                    l2hi[k] = __shfl_up(lhi[k], o);
                }
                if (lane + o < 64) {
                    rc += rc2;
                    rw += rw2;
                    for (int k = 0; k < 3; ++k) {
                        rlo[k] = fminf(rlo[k], r2lo[k]);
                        rhi[k] = fmaxf(rhi[k], r2hi[k]);
                    }
                }
                if (lane >= o) {
                    lc += lc2;
                    lw += lw2;
                    for (int k = 0; k < 3; ++k) {
                        llo[k] = fminf(llo[k], l2lo[k]);
                        lhi[k] = fmaxf(lhi[k], l2hi[k]);
                    }
                }
            }
            const float ra = box_area(rlo[0], rlo[1], rlo[2], rhi[0], rhi[1], rhi[2]);
            const float la = box_area(llo[0], llo[1], llo[2], lhi[0], lhi[1], lhi[2]);
            const int rc1 = __shfl_down(rc, 1), rw1 = __shfl_down(rw, 1);
            const float ra1 = __shfl_down(ra, 1);
            // split after bin `lane`: left = bins 0..lane, right = lane+1..NB-1
            const bool valid = lane < NB - 1 && lc != 0 && rc1 != 0;
            float cost = valid ? la * (float)lw + ra1 * (float)rw1 : FLT_MAX;
            int idx = lane;
            for (int o = 32; o > 0; o >>= 1) {  // argmin, ties to the lower bin (first minimum)
                const float c2 = __shfl_xor(cost, o);
                const int i2 = __shfl_xor(idx, o);
                if (c2 < cost || (c2 == cost && i2 < idx)) {
                    cost = c2;
                    idx = i2;
                }
            }
            const bool any_valid = __ballot(valid) != 0;
            if (any_valid && cost < best_cost) {  // strict: an earlier axis keeps a tie
                best_cost = cost;
                best_axis = a;
                best_split = idx;
                best_nl = __shfl(lc, idx);
            }
        }
        // SAH: leaf if testing everything here is no dearer than one more node step plus the split
        const float area = box_area(bl[0], bl[1], bl[2], bh[0], bh[1], bh[2]);
        const float wsum = (float)ws;
        if (n <= A.max_leaf && (best_axis < 0 || A.c_isect * wsum * area <= area + A.c_isect * best_cost))
            leaf = true;
    }

    int ref = 0, mid = 0;
    if (leaf) {
        int l = 0;
        if (lane == 0) l = atomicAdd(A.counters + 1, 1);
        l = __shfl(l, 0);
        if (lane == 0) A.leaves[l] = make_int2(b, e);
        ref = ~l;
    } else {
        int self = 0;
        if (lane == 0) self = atomicAdd(A.counters + 0, 1);
        self = __shfl(self, 0);
        ref = self;
        if (best_axis < 0) {
            mid = (b + e) / 2;  // all centroids coincide: split by position
        } else {
            // ---- pass 3: stable partition by bin <= best_split ----
            const float lo = cl[best_axis], ex = ext[best_axis];
            int nl = 0, nr = 0;
            for (int i0 = b; i0 < e; i0 += 64) {
                const int i = i0 + lane;
                const bool v = i < e;
                const int id = v ? A.ids[i] : 0;
                const bool left = v && bin_of(A.cent[3 * id + best_axis], lo, ex) <= best_split;
                const uint64_t lm = __ballot(left), rm = __ballot(v && !left);
                if (left) A.tmp[b + nl + __popcll(lm & below)] = id;
                if (v && !left) A.tmp[b + best_nl + nr + __popcll(rm & below)] = id;
                nl += __popcll(lm);
                nr += __popcll(rm);
            }
            __threadfence();  // the copy below reads other lanes' stores
            for (int i = b + lane; i < e; i += 64) A.ids[i] = A.tmp[i];
            mid = b + best_nl;
            if (mid == b || mid == e) mid = (b + e) / 2;
        }
        int pos = 0;
        if (lane == 0) pos = atomicAdd(A.counters + 2, 2);
        pos = __shfl(pos, 0);
        if (lane == 0) {
            tout[pos] = BTask{b, mid, self, 0};
            tout[pos + 1] = BTask{mid, e, self, 1};
        }
    }
    // link into the parent: child reference and the subtree box (primitive box union)
    if (lane == 0) {
        float* bx;
        if (T.parent < 0) {
            *A.root_ref = ref;
            bx = A.root_box;
        } else {
            A.node_child[2 * T.parent + T.side] = ref;
            bx = A.node_box + (2 * T.parent + T.side) * 6;
        }
        for (int k = 0; k < 3; ++k) {
            bx[k] = bl[k];
            bx[3 + k] = bh[k];
        }
    }
}

template <typename T>
hipError_t dalloc(T** p, size_t n) {
    return hipMalloc((void**)p, std::max<size_t>(1, n) * sizeof(T));
}

}  // namespace

hipError_t mfx_gpu_sah_build(const float* prim_box, const float* cent, const int32_t* weight, int n, int max_leaf,
                             float c_isect, MfxBvh2& out) {
    BArgs A{};
    float *d_box = nullptr, *d_cent = nullptr;
    int* d_weight = nullptr;
    BTask *t0 = nullptr, *t1 = nullptr;
    hipError_t e = hipSuccess;
    auto ok = [&](hipError_t r) {
        if (e == hipSuccess) e = r;
        return e == hipSuccess;
    };
    std::vector<int32_t> iota(n);
    std::iota(iota.begin(), iota.end(), 0);
    ok(dalloc(&d_box, 6 * (size_t)n));
    ok(dalloc(&d_cent, 3 * (size_t)n));
    ok(dalloc(&d_weight, (size_t)n));
    ok(dalloc(&A.ids, (size_t)n));
    ok(dalloc(&A.tmp, (size_t)n));
    ok(dalloc(&A.node_box, 12 * (size_t)n));
    ok(dalloc(&A.node_child, 2 * (size_t)n));
    ok(dalloc(&A.leaves, (size_t)n));
    ok(dalloc(&A.counters, 4));
    ok(dalloc(&A.root_box, 6));
    ok(dalloc(&A.root_ref, 1));
    ok(dalloc(&t0, (size_t)n));
    ok(dalloc(&t1, (size_t)n));
    if (e == hipSuccess) {
        ok(hipMemcpy(d_box, prim_box, sizeof(float) * 6 * (size_t)n, hipMemcpyHostToDevice));
        ok(hipMemcpy(d_cent, cent, sizeof(float) * 3 * (size_t)n, hipMemcpyHostToDevice));
        ok(hipMemcpy(d_weight, weight, sizeof(int) * (size_t)n, hipMemcpyHostToDevice));
        ok(hipMemcpy(A.ids, iota.data(), sizeof(int) * (size_t)n, hipMemcpyHostToDevice));
        ok(hipMemset(A.counters, 0, 4 * sizeof(int)));
        const BTask root{0, n, -1, 0};
        ok(hipMemcpy(t0, &root, sizeof(BTask), hipMemcpyHostToDevice));
    }
    A.box = d_box;
    A.cent = d_cent;
    A.weight = d_weight;
    A.max_leaf = max_leaf;
    A.c_isect = c_isect;
    int ntasks = 1, levels = 0;
    while (e == hipSuccess && ntasks > 0) {
        ok(hipMemset(A.counters + 2, 0, sizeof(int)));
        hipLaunchKernelGGL(k_sah_level, dim3((ntasks + 3) / 4), dim3(256), 0, 0, A, t0, ntasks, t1);
        ok(hipGetLastError());
        ok(hipMemcpy(&ntasks, A.counters + 2, sizeof(int), hipMemcpyDeviceToHost));
        std::swap(t0, t1);
        ++levels;
        if (levels > 4 * 64 + n) ok(hipErrorUnknown);  // cannot happen: every level splits ranges
    }
    int cnt[2] = {0, 0};
    if (e == hipSuccess) {
        ok(hipMemcpy(cnt, A.counters, 2 * sizeof(int), hipMemcpyDeviceToHost));
        out.box.resize(12 * (size_t)cnt[0]);
        out.child.resize(2 * (size_t)cnt[0]);
        std::vector<int2> lv(cnt[1]);
        out.ids.resize(n);
        ok(hipMemcpy(out.box.data(), A.node_box, sizeof(float) * out.box.size(), hipMemcpyDeviceToHost));
        ok(hipMemcpy(out.child.data(), A.node_child, sizeof(int) * out.child.size(), hipMemcpyDeviceToHost));
        ok(hipMemcpy(lv.data(), A.leaves, sizeof(int2) * lv.size(), hipMemcpyDeviceToHost));
        ok(hipMemcpy(out.ids.data(), A.ids, sizeof(int) * (size_t)n, hipMemcpyDeviceToHost));
        ok(hipMemcpy(&out.root, A.root_ref, sizeof(int), hipMemcpyDeviceToHost));
        ok(hipMemcpy(out.root_box, A.root_box, sizeof(float) * 6, hipMemcpyDeviceToHost));
        out.leaf_b.resize(lv.size());
        out.leaf_e.resize(lv.size());
        for (size_t l = 0; l < lv.size(); ++l) {
            out.leaf_b[l] = lv[l].x;
            out.leaf_e[l] = lv[l].y;
        }
        out.levels = levels;
    }
    void* bufs[] = {d_box, d_cent, d_weight, A.ids, A.tmp, A.node_box, A.node_child, A.leaves, A.counters,
                    A.root_box, A.root_ref, t0, t1};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    return e;
}
