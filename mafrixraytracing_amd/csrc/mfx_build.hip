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

// ------------------------------------------------------------------------------------------------
// BVH4 collapse and image layout on the device (the host's Collapse4 + mfx_build_scene layout, the
// same bytes). Level by level from the root: a BVH4 node is a BVH2 node that adopts the children of
// its largest-area internal child until it has four (first maximum, children replaced in place);
// its internal children, in order, form the next level, so the levels' concatenation is the
// breadth-first order. Subtree node and slot counts go bottom-up, preorder indices, slot offsets
// and stack depths top-down; then nodes are renumbered (the first MFX_TOP_NODES breadth-first,
// the rest in preorder) and the traversal leaves' slots scattered in depth-first order.
// ------------------------------------------------------------------------------------------------
struct W4 {
    float box[4][6];
    int ch[4];  // BVH2 refs: >= 0 internal, < 0 ~leaf
    int cv[4];  // breadth-first index of an internal child (else -1)
    int nc;
};

__device__ __forceinline__ float fbox_area(const float* b) { return box_area(b[0], b[1], b[2], b[3], b[4], b[5]); }

// one BVH4 node per frontier entry (a BVH2 node, or ~leaf for a tree that is one leaf)
__global__ void k_collapse(const int* __restrict__ F, int nF, const float* __restrict__ node_box,
                           const int* __restrict__ node_child, const float* __restrict__ root_box, W4* __restrict__ W,
                           int* __restrict__ cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nF) return;
    const int r = F[i];
    W4 w;
    int nc = 2;
    if (r < 0) {  // the whole scene is one leaf: a root node with one child
        nc = 1;
        w.ch[0] = r;
        for (int a = 0; a < 6; ++a) w.box[0][a] = root_box[a];
    } else {
        for (int k = 0; k < 2; ++k) {
            w.ch[k] = node_child[2 * r + k];
            for (int a = 0; a < 6; ++a) w.box[k][a] = node_box[(2 * r + k) * 6 + a];
        }
    }
    while (nc > 1 && nc < 4) {
        int best = -1;
        float ba = -1.f;
        for (int k = 0; k < nc; ++k)
            if (w.ch[k] >= 0 && fbox_area(w.box[k]) > ba) {
                ba = fbox_area(w.box[k]);
                best = k;
            }
        if (best < 0) break;
        const int m = w.ch[best];
        for (int k = nc; k > best + 1; --k) {  // the children of `best` replace it in place
            w.ch[k] = w.ch[k - 1];
            for (int a = 0; a < 6; ++a) w.box[k][a] = w.box[k - 1][a];
        }
        for (int q = 0; q < 2; ++q) {
            w.ch[best + q] = node_child[2 * m + q];
            for (int a = 0; a < 6; ++a) w.box[best + q][a] = node_box[(2 * m + q) * 6 + a];
        }
        ++nc;
    }
    w.nc = nc;
    int c = 0;
    for (int k = 0; k < 4; ++k) {
        w.cv[k] = -1;
        if (k < nc && w.ch[k] >= 0) ++c;
    }
    W[i] = w;
    cnt[i] = c;
}

// exclusive scan of cnt[0..n) in place (one block), the total in *total
__global__ void __launch_bounds__(1024) k_scan(int* cnt, int n, int* total) {
    __shared__ int part[1024];
    int carry = 0;
    for (int base = 0; base < n; base += 1024) {
        const int i = base + threadIdx.x;
        const int v = i < n ? cnt[i] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const int t = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
            __syncthreads();
            part[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < n) cnt[i] = carry + part[threadIdx.x] - v;
        carry += part[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

// the next level: internal children in order; their breadth-first indices into the parents
__global__ void k_frontier(W4* __restrict__ W, int nF, const int* __restrict__ pos, int next_base, int* __restrict__ F2) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nF) return;
    int p = pos[i];
    for (int k = 0; k < W[i].nc; ++k)
        if (W[i].ch[k] >= 0) {
            F2[p] = W[i].ch[k];
            W[i].cv[k] = next_base + p;
            ++p;
        }
}

struct LArgs {
    const W4* W;             // [n4] breadth-first
    const int2* leaves;      // [nleaves] ranges of ids
    const int* ids;
    const int* slot_of;      // [n + 1] first slot of each primitive in the per-primitive slot array
    int* size;               // [n4] BVH4 nodes in the subtree
    int* nslots;             // [n4] slots in the subtree
    int* pre;                // [n4] preorder index
    int* sstart;             // [n4] first slot of the subtree (depth-first leaf order)
    int* pushed;             // [n4] stack entries when the node is reached
    int* leaf_start;         // [nleaves] first slot of the traversal leaf
    int* idx;                // [n4] final node index
    int* max_stack;
};

__device__ __forceinline__ int leaf_slots(const LArgs& A, int l) {
    const int2 r = A.leaves[l];
    int s = 0;
    for (int k = r.x; k < r.y; ++k) s += A.slot_of[A.ids[k] + 1] - A.slot_of[A.ids[k]];
    return s;
}

__global__ void k_sizes(LArgs A, int lo, int hi) {  // bottom-up, one level [lo, hi)
    const int v = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= hi) return;
    const W4& w = A.W[v];
    int n = 1, s = 0;
    for (int k = 0; k < w.nc; ++k) {
        if (w.ch[k] >= 0) {
            n += A.size[w.cv[k]];
            s += A.nslots[w.cv[k]];
        } else {
            s += leaf_slots(A, ~w.ch[k]);
        }
    }
    A.size[v] = n;
    A.nslots[v] = s;
}

__global__ void k_preorder(LArgs A, int lo, int hi) {  // top-down, one level [lo, hi)
    const int v = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= hi) return;
    const W4& w = A.W[v];
    int next = A.pre[v] + 1, slot = A.sstart[v];
    const int push = A.pushed[v] + w.nc - 1;  // node_step writes stack[pushed .. pushed + nc - 2]
    atomicMax(A.max_stack, push);
    for (int k = 0; k < w.nc; ++k) {
        if (w.ch[k] >= 0) {
            const int c = w.cv[k];
            A.pre[c] = next;
            A.sstart[c] = slot;
            A.pushed[c] = push;
            next += A.size[c];
            slot += A.nslots[c];
        } else {
            A.leaf_start[~w.ch[k]] = slot;
            slot += leaf_slots(A, ~w.ch[k]);
        }
    }
}

// final index: the first MFX_TOP_NODES breadth-first, the rest by preorder rank among the others
__global__ void k_index(LArgs A, int n4, int top_nodes) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n4) return;
    const int ntop = min(n4, top_nodes);
    if (v < ntop) {
        A.idx[v] = v;
        return;
    }
    const int p = A.pre[v];
    int below = 0;
    for (int u = 0; u < ntop; ++u) below += A.pre[u] < p ? 1 : 0;
    A.idx[v] = ntop + p - below;
}

__global__ void k_nodes(LArgs A, int n4, MfxNode* __restrict__ out) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n4) return;
    const W4& w = A.W[v];
    MfxNode nd;
    for (int k = 0; k < 4; ++k) {
        const bool e = k < w.nc;
        nd.lox[k] = e ? w.box[k][0] : FLT_MAX;
        nd.loy[k] = e ? w.box[k][1] : FLT_MAX;
        nd.loz[k] = e ? w.box[k][2] : FLT_MAX;
        nd.hix[k] = e ? w.box[k][3] : FLT_MAX;
        nd.hiy[k] = e ? w.box[k][4] : FLT_MAX;
        nd.hiz[k] = e ? w.box[k][5] : FLT_MAX;
        int c = MFX_CHILD_EMPTY;
        if (e && w.ch[k] >= 0) c = A.idx[w.cv[k]];
        else if (e) c = ~((A.leaf_start[~w.ch[k]] << 3) | (leaf_slots(A, ~w.ch[k]) - 1));
        nd.child[k] = c;
        nd.pad[k] = 0;
    }
    out[A.idx[v]] = nd;
}

// one traversal leaf: its primitives' slots at its offset, in its order; a slot's shade[] index
// is its own index (the info field's low bits)
__global__ void k_slots(LArgs A, int nleaves, const MfxSlot* __restrict__ pslots, const MfxShade* __restrict__ pshade,
                        const int32_t* __restrict__ ref16_of, MfxSlot* __restrict__ slots, int32_t* __restrict__ slot_ref,
                        MfxShade* __restrict__ shade, int32_t* __restrict__ shade_of) {
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= nleaves) return;
    const int2 r = A.leaves[l];
    int at = A.leaf_start[l];
    for (int k = r.x; k < r.y; ++k) {
        const int p = A.ids[k];
        shade_of[p] = at;
        for (int q = A.slot_of[p]; q < A.slot_of[p + 1]; ++q, ++at) {
            MfxSlot sl = pslots[q];
            sl.info |= at;
            slots[at] = sl;
            slot_ref[at] = ref16_of[p];
            shade[at] = pshade[q];
        }
    }
}

}  // namespace

// The BVH2 build on the device; its arrays stay there for the collapse and layout
struct DevBvh2 {
    BArgs A{};
    float* d_box = nullptr;
    float* d_cent = nullptr;
    int* d_weight = nullptr;
    BTask* t0 = nullptr;
    BTask* t1 = nullptr;
    int nodes = 0, nleaves = 0, levels = 0, root = 0;
};

static void bvh2_free(DevBvh2& D) {
    void* bufs[] = {D.d_box, D.d_cent, D.d_weight, D.A.ids, D.A.tmp, D.A.node_box, D.A.node_child, D.A.leaves,
                    D.A.counters, D.A.root_box, D.A.root_ref, D.t0, D.t1};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    D = DevBvh2{};
}

static hipError_t bvh2_build(const float* prim_box, const float* cent, const int32_t* weight, int n, int max_leaf,
                             float c_isect, DevBvh2& D) {
    BArgs& A = D.A;
    hipError_t e = hipSuccess;
    auto ok = [&](hipError_t r) {
        if (e == hipSuccess) e = r;
        return e == hipSuccess;
    };
    std::vector<int32_t> iota(n);
    std::iota(iota.begin(), iota.end(), 0);
    ok(dalloc(&D.d_box, 6 * (size_t)n));
    ok(dalloc(&D.d_cent, 3 * (size_t)n));
    ok(dalloc(&D.d_weight, (size_t)n));
    ok(dalloc(&A.ids, (size_t)n));
    ok(dalloc(&A.tmp, (size_t)n));
    ok(dalloc(&A.node_box, 12 * (size_t)n));
    ok(dalloc(&A.node_child, 2 * (size_t)n));
    ok(dalloc(&A.leaves, (size_t)n));
    ok(dalloc(&A.counters, 4));
    ok(dalloc(&A.root_box, 6));
    ok(dalloc(&A.root_ref, 1));
    ok(dalloc(&D.t0, (size_t)n));
    ok(dalloc(&D.t1, (size_t)n));
    if (e == hipSuccess) {
        ok(hipMemcpy(D.d_box, prim_box, sizeof(float) * 6 * (size_t)n, hipMemcpyHostToDevice));
        ok(hipMemcpy(D.d_cent, cent, sizeof(float) * 3 * (size_t)n, hipMemcpyHostToDevice));
        ok(hipMemcpy(D.d_weight, weight, sizeof(int) * (size_t)n, hipMemcpyHostToDevice));
        ok(hipMemcpy(A.ids, iota.data(), sizeof(int) * (size_t)n, hipMemcpyHostToDevice));
        ok(hipMemset(A.counters, 0, 4 * sizeof(int)));
        const BTask root{0, n, -1, 0};
        ok(hipMemcpy(D.t0, &root, sizeof(BTask), hipMemcpyHostToDevice));
    }
    A.box = D.d_box;
    A.cent = D.d_cent;
    A.weight = D.d_weight;
    A.max_leaf = max_leaf;
    A.c_isect = c_isect;
    int ntasks = 1;
    while (e == hipSuccess && ntasks > 0) {
        ok(hipMemset(A.counters + 2, 0, sizeof(int)));
        hipLaunchKernelGGL(k_sah_level, dim3((ntasks + 3) / 4), dim3(256), 0, 0, A, D.t0, ntasks, D.t1);
        ok(hipGetLastError());
        ok(hipMemcpy(&ntasks, A.counters + 2, sizeof(int), hipMemcpyDeviceToHost));
        std::swap(D.t0, D.t1);
        ++D.levels;
        if (D.levels > 4 * 64 + n) ok(hipErrorUnknown);  // cannot happen: every level splits ranges
    }
    int cnt[2] = {0, 0};
    ok(hipMemcpy(cnt, A.counters, 2 * sizeof(int), hipMemcpyDeviceToHost));
    ok(hipMemcpy(&D.root, A.root_ref, sizeof(int), hipMemcpyDeviceToHost));
    D.nodes = cnt[0];
    D.nleaves = cnt[1];
    return e;
}

hipError_t mfx_gpu_sah_build(const float* prim_box, const float* cent, const int32_t* weight, int n, int max_leaf,
                             float c_isect, MfxBvh2& out) {
    DevBvh2 D;
    hipError_t e = bvh2_build(prim_box, cent, weight, n, max_leaf, c_isect, D);
    auto ok = [&](hipError_t r) {
        if (e == hipSuccess) e = r;
        return e == hipSuccess;
    };
    if (e == hipSuccess) {
        const BArgs& A = D.A;
        out.box.resize(12 * (size_t)D.nodes);
        out.child.resize(2 * (size_t)D.nodes);
        std::vector<int2> lv(D.nleaves);
        out.ids.resize(n);
        ok(hipMemcpy(out.box.data(), A.node_box, sizeof(float) * out.box.size(), hipMemcpyDeviceToHost));
        ok(hipMemcpy(out.child.data(), A.node_child, sizeof(int) * out.child.size(), hipMemcpyDeviceToHost));
        ok(hipMemcpy(lv.data(), A.leaves, sizeof(int2) * lv.size(), hipMemcpyDeviceToHost));
        ok(hipMemcpy(out.ids.data(), A.ids, sizeof(int) * (size_t)n, hipMemcpyDeviceToHost));
        ok(hipMemcpy(out.root_box, A.root_box, sizeof(float) * 6, hipMemcpyDeviceToHost));
        out.root = D.root;
        out.leaf_b.resize(lv.size());
        out.leaf_e.resize(lv.size());
        for (size_t l = 0; l < lv.size(); ++l) {
            out.leaf_b[l] = lv[l].x;
            out.leaf_e[l] = lv[l].y;
        }
        out.levels = D.levels;
    }
    bvh2_free(D);
    return e;
}

hipError_t mfx_gpu_build_images(const float* prim_box, const float* cent, const int32_t* weight, int n, int max_leaf,
                                float c_isect, const MfxGpuLayoutIn& in, MfxGpuImages& out) {
    DevBvh2 D;
    hipError_t e = bvh2_build(prim_box, cent, weight, n, max_leaf, c_isect, D);
    auto ok = [&](hipError_t r) {
        if (e == hipSuccess) e = r;
        return e == hipSuccess;
    };
    const int n4max = D.nodes + 1;
    W4* W = nullptr;
    int *F = nullptr, *cnt = nullptr, *total = nullptr, *slot_of = nullptr, *ref16 = nullptr, *shade_of = nullptr;
    int *size = nullptr, *nsl = nullptr, *pre = nullptr, *sstart = nullptr, *pushed = nullptr, *lstart = nullptr,
        *idx = nullptr, *mstack = nullptr;
    MfxSlot *pslots = nullptr, *slots = nullptr;
    MfxShade *pshade = nullptr, *shade = nullptr;
    MfxNode* nodes = nullptr;
    int32_t* slot_ref = nullptr;
    const size_t ns = (size_t)in.nslots;
    ok(dalloc(&W, n4max));
    ok(dalloc(&F, n4max));
    ok(dalloc(&cnt, n4max));
    ok(dalloc(&total, 1));
    ok(dalloc(&size, n4max));
    ok(dalloc(&nsl, n4max));
    ok(dalloc(&pre, n4max));
    ok(dalloc(&sstart, n4max));
    ok(dalloc(&pushed, n4max));
    ok(dalloc(&idx, n4max));
    ok(dalloc(&mstack, 1));
    ok(dalloc(&lstart, (size_t)std::max(1, D.nleaves)));
    ok(dalloc(&slot_of, (size_t)n + 1));
    ok(dalloc(&ref16, (size_t)n));
    ok(dalloc(&shade_of, (size_t)n));
    ok(dalloc(&pslots, ns));
    ok(dalloc(&pshade, ns));
    ok(dalloc(&slots, ns + MFX_LEAF_SLOTS_MAX));
    ok(dalloc(&slot_ref, ns));
    ok(dalloc(&shade, ns));
    ok(dalloc(&nodes, n4max));
    if (e == hipSuccess) {
        ok(hipMemcpy(slot_of, in.slot_of, sizeof(int) * ((size_t)n + 1), hipMemcpyHostToDevice));
        ok(hipMemcpy(ref16, in.ref16_of, sizeof(int) * (size_t)n, hipMemcpyHostToDevice));
        ok(hipMemcpy(pslots, in.pslots, sizeof(MfxSlot) * ns, hipMemcpyHostToDevice));
        ok(hipMemcpy(pshade, in.pshade, sizeof(MfxShade) * ns, hipMemcpyHostToDevice));
        ok(hipMemset(slots + ns, 0, sizeof(MfxSlot) * MFX_LEAF_SLOTS_MAX));  // speculative loads stay in bounds
        ok(hipMemcpy(F, &D.root, sizeof(int), hipMemcpyHostToDevice));
        ok(hipMemset(pre, 0, sizeof(int)));
        ok(hipMemset(sstart, 0, sizeof(int)));
        ok(hipMemset(pushed, 0, sizeof(int)));
        ok(hipMemset(mstack, 0, sizeof(int)));
    }
    // collapse, level by level: frontier [base, base + nF) of F is a level in breadth-first order
    std::vector<int> lo;
    int base = 0, nF = 1;
    while (e == hipSuccess && nF > 0) {
        if (base + nF > n4max) {
            ok(hipErrorUnknown);
            break;
        }
        lo.push_back(base);
        const dim3 g((nF + 255) / 256);
        hipLaunchKernelGGL(k_collapse, g, dim3(256), 0, 0, F + base, nF, D.A.node_box, D.A.node_child, D.A.root_box,
                           W + base, cnt + base);
        hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, 0, cnt + base, nF, total);
        hipLaunchKernelGGL(k_frontier, g, dim3(256), 0, 0, W + base, nF, cnt + base, base + nF, F + base + nF);
        ok(hipGetLastError());
        int t = 0;
        ok(hipMemcpy(&t, total, sizeof(int), hipMemcpyDeviceToHost));
        base += nF;
        nF = t;
    }
    const int n4 = base;
    lo.push_back(n4);
    const int nlev = (int)lo.size() - 1;
    LArgs A{W, D.A.leaves, D.A.ids, slot_of, size, nsl, pre, sstart, pushed, lstart, idx, mstack};
    for (int L = nlev - 1; L >= 0 && e == hipSuccess; --L)
        hipLaunchKernelGGL(k_sizes, dim3((lo[L + 1] - lo[L] + 255) / 256), dim3(256), 0, 0, A, lo[L], lo[L + 1]);
    for (int L = 0; L < nlev && e == hipSuccess; ++L)
        hipLaunchKernelGGL(k_preorder, dim3((lo[L + 1] - lo[L] + 255) / 256), dim3(256), 0, 0, A, lo[L], lo[L + 1]);
    if (e == hipSuccess && n4 > 0) {
        hipLaunchKernelGGL(k_index, dim3((n4 + 255) / 256), dim3(256), 0, 0, A, n4, in.top_nodes);
        hipLaunchKernelGGL(k_nodes, dim3((n4 + 255) / 256), dim3(256), 0, 0, A, n4, nodes);
        hipLaunchKernelGGL(k_slots, dim3((D.nleaves + 255) / 256), dim3(256), 0, 0, A, D.nleaves, pslots, pshade, ref16,
                           slots, slot_ref, shade, shade_of);
        ok(hipGetLastError());
    }
    if (e == hipSuccess) {
        out.nodes.resize(n4);
        out.slots.resize(ns + MFX_LEAF_SLOTS_MAX);
        out.slot_ref.resize(ns);
        out.shade.resize(ns);
        out.shade_of.resize(n);
        ok(hipMemcpy(out.nodes.data(), nodes, sizeof(MfxNode) * n4, hipMemcpyDeviceToHost));
        ok(hipMemcpy(out.slots.data(), slots, sizeof(MfxSlot) * out.slots.size(), hipMemcpyDeviceToHost));
        ok(hipMemcpy(out.slot_ref.data(), slot_ref, sizeof(int32_t) * ns, hipMemcpyDeviceToHost));
        ok(hipMemcpy(out.shade.data(), shade, sizeof(MfxShade) * ns, hipMemcpyDeviceToHost));
        ok(hipMemcpy(out.shade_of.data(), shade_of, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost));
        ok(hipMemcpy(&out.max_stack, mstack, sizeof(int), hipMemcpyDeviceToHost));
        out.max_depth = nlev - 1;
        out.nodes2 = D.nodes;
        out.nleaves = D.nleaves;
        out.levels = D.levels;
    }
    void* bufs[] = {W, F, cnt, total, size, nsl, pre, sstart, pushed, idx, mstack, lstart, slot_of, ref16, shade_of,
                    pslots, pshade, slots, slot_ref, shade, nodes};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    bvh2_free(D);
    return e;
}
