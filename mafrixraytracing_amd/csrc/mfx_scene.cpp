// mfx_scene.cpp — host-side preparation of a scene for the gfx950 kernels.
//
// 1. Primitive records in FP64, with exactly the reference constructors' arithmetic
//    (Triangle: Trangle.fs:107-119, Rect: Rect.fs:11-20, Sphere: Sphere.fs:9-16).
// 2. The reference's heap BVH (BvhNode.fs:24-61) is built only for its LEAF GROUPING: which
//    2-3 primitives share a leaf decides the shadow-ray result when every primitive of a leaf
//    is hit beyond tMax (Triangle.Hit ignores tMax, Trangle.fs:148; the leaf minBy, :76-80).
//    Its median split sorts with F#'s Array.sortInPlaceBy = .NET 6 introsort, restated here so
//    ties fall the same way.
// 3. A binned-SAH BVH2 over the individual primitives, collapsed to a BVH4, is what the GPU
//    traverses, in FP32 with conservatively widened boxes. Every primitive slot carries its reference leaf and position,
//    so the reference's leaf semantics are applied exactly per candidate hit.
#include "mfx_scene.h"

#include <chrono>

#include "mfx_build.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace {

struct D3 {
    double x, y, z;
};
inline D3 d3(const double* p) { return {p[0], p[1], p[2]}; }
inline D3 sub(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline D3 add(D3 a, D3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline D3 scale(D3 v, double a) { return {v.x * a, v.y * a, v.z * a}; }
inline D3 cross(D3 a, D3 v) { return {a.y * v.z - a.z * v.y, a.z * v.x - a.x * v.z, a.x * v.y - a.y * v.x}; }
inline double len(D3 v) { return std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z); }
inline D3 normalize(D3 v) {
    double l = len(v);
    if (l == 0.0) return {0, 0, 0};
    return {v.x / l, v.y / l, v.z / l};
}
inline double comp(D3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
inline double mn(double a, double b) { return a < b ? a : b; }
inline double mx(double a, double b) { return a > b ? a : b; }
inline void put(double* dst, D3 v) { dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; }

struct Box {
    D3 lo, hi;
};
inline Box box2(D3 p, D3 q) {  // Bound(p1, p2), Aggregate.fs:9-11
    return {{mn(p.x, q.x), mn(p.y, q.y), mn(p.z, q.z)}, {mx(p.x, q.x), mx(p.y, q.y), mx(p.z, q.z)}};
}
inline Box join(Box a, Box b) {  // Bound.Union, Aggregate.fs:58-61
    return box2({mn(a.lo.x, b.lo.x), mn(a.lo.y, b.lo.y), mn(a.lo.z, b.lo.z)},
                {mx(a.hi.x, b.hi.x), mx(a.hi.y, b.hi.y), mx(a.hi.z, b.hi.z)});
}
inline Box join_pt(Box a, D3 p) {
    return box2({mn(a.lo.x, p.x), mn(a.lo.y, p.y), mn(a.lo.z, p.z)}, {mx(a.hi.x, p.x), mx(a.hi.y, p.y), mx(a.hi.z, p.z)});
}
inline Box tri_box(D3 a, D3 b, D3 c) { return join_pt(box2(a, b), c); }  // Trangle.fs:113

// ---- .NET 6 GenericArraySortHelper<double,int>.IntroSort (tie behaviour of Array.Sort) ------
struct NetSort {
    double* k;
    int32_t* v;
    void swap(int i, int j) {
        std::swap(k[i], k[j]);
        std::swap(v[i], v[j]);
    }
    void swap_if_greater(int i, int j) {
        if (k[i] > k[j]) swap(i, j);
    }
    void insertion(int n) {
        for (int i = 0; i < n - 1; ++i) {
            double t = k[i + 1];
            int32_t tv = v[i + 1];
            int j = i;
            for (; j >= 0 && t < k[j]; --j) {
                k[j + 1] = k[j];
                v[j + 1] = v[j];
            }
            k[j + 1] = t;
            v[j + 1] = tv;
        }
    }
    void down_heap(int i, int n) {
        double d = k[i - 1];
        int32_t dv = v[i - 1];
        while (i <= n >> 1) {
            int c = 2 * i;
            if (c < n && k[c - 1] < k[c]) ++c;
            if (!(d < k[c - 1])) break;
            k[i - 1] = k[c - 1];
            v[i - 1] = v[c - 1];
            i = c;
        }
        k[i - 1] = d;
        v[i - 1] = dv;
    }
    void heap(int n) {
        for (int i = n >> 1; i >= 1; --i) down_heap(i, n);
        for (int i = n; i > 1; --i) {
            swap(0, i - 1);
            down_heap(1, i - 1);
        }
    }
    int partition(int n) {
        const int hi = n - 1, mid = hi >> 1;
        swap_if_greater(0, mid);
        swap_if_greater(0, hi);
        swap_if_greater(mid, hi);
        const double pivot = k[mid];
        swap(mid, hi - 1);
        int l = 0, r = hi - 1;
        while (l < r) {
            while (pivot > k[++l]) {
            }
            while (pivot < k[--r]) {
            }
            if (l >= r) break;
            swap(l, r);
        }
        if (l != hi - 1) swap(l, hi - 1);
        return l;
    }
    static void intro(double* kk, int32_t* vv, int n, int depth) {
        while (n > 1) {
            NetSort s{kk, vv};
            if (n <= 16) {
                if (n == 2) {
                    s.swap_if_greater(0, 1);
                } else if (n == 3) {
                    s.swap_if_greater(0, 1);
                    s.swap_if_greater(0, 2);
                    s.swap_if_greater(1, 2);
                } else {
                    s.insertion(n);
                }
                return;
            }
            if (depth == 0) {
                s.heap(n);
                return;
            }
            --depth;
            int p = s.partition(n);
            intro(kk + p + 1, vv + p + 1, n - p - 1, depth);
            n = p;
        }
    }
    static void sort(double* kk, int32_t* vv, int n) {
        if (n < 2) return;
        int lg = 0;
        for (unsigned x = (unsigned)n; x >>= 1;) ++lg;
        intro(kk, vv, n, 2 * (lg + 1));
    }
};

// ---- reference heap BVH: leaf grouping only ------------------------------------------------
// Subtrees are independent: each sorts only its own index range (keys / tmp are indexed by the
// range, not from 0), so the two halves of the top splits run on their own host threads and their
// leaves are concatenated left to right — the same leaves, in the same order, as the sequential
// recursion (the introsort of every range is unchanged).
struct RefBvh {
    const std::vector<Box>& pb;
    std::vector<int32_t>& idx;
    std::vector<double> keys;
    std::vector<int32_t> tmp;

    Box bound(int first, int count) const {  // InitNode, BvhNode.fs:32-37
        Box b = pb[idx[first]];
        for (int k = 1; k < count; ++k) b = join(b, pb[idx[first + k]]);
        return b;
    }
    // Subdivide (BvhNode.fs:42-61), visiting leaves left to right; `par` more levels split onto
    // a second thread (ranges of at least 8,192 primitives)
    void subdivide(int first, int count, Box b, std::vector<int32_t>& lf, std::vector<int32_t>& lc, int par) {
        if (count <= 3) {
            lf.push_back(first);
            lc.push_back(count);
            return;
        }
        D3 d = sub(b.hi, b.lo);  // MaximumExtent, Aggregate.fs:29-36
        int axis = (d.x > d.y && d.x > d.z) ? 0 : (d.y > d.z ? 1 : 2);
        double* kk = keys.data() + first;
        int32_t* tt = tmp.data() + first;
        for (int k = 0; k < count; ++k) {
            int p = idx[first + k];
            const Box& q = pb[p];
            D3 c = add(q.lo, scale(sub(q.hi, q.lo), 0.5));
            kk[k] = comp(c, axis);
            tt[k] = p;
        }
        NetSort::sort(kk, tt, count);
        std::memcpy(&idx[first], tt, sizeof(int32_t) * count);
        int left = count / 2;
        Box bl = bound(first, left), br = bound(first + left, count - left);
        if (par > 0 && count >= 8192) {
            std::vector<int32_t> lf2, lc2;
            std::thread t([&] { subdivide(first + left, count - left, br, lf2, lc2, par - 1); });
            subdivide(first, left, bl, lf, lc, par - 1);
            t.join();
            lf.insert(lf.end(), lf2.begin(), lf2.end());
            lc.insert(lc.end(), lc2.begin(), lc2.end());
        } else {
            subdivide(first, left, bl, lf, lc, 0);
            subdivide(first + left, count - left, br, lf, lc, 0);
        }
    }
};

// ---- binned SAH BVH2 over clusters ---------------------------------------------------------
struct FBox {
    float lo[3], hi[3];
    void grow(const FBox& b) {
        for (int i = 0; i < 3; ++i) {
            lo[i] = std::min(lo[i], b.lo[i]);
            hi[i] = std::max(hi[i], b.hi[i]);
        }
    }
    float area() const {
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (dx < 0 || dy < 0 || dz < 0) return 0.f;
        return 2.f * (dx * dy + dx * dz + dy * dz);
    }
    static FBox empty() {
        FBox b;
        for (int i = 0; i < 3; ++i) {
            b.lo[i] = FLT_MAX;
            b.hi[i] = -FLT_MAX;
        }
        return b;
    }
};

struct Node2 {  // binned-SAH BVH2 node (host only; collapsed to MfxNode BVH4 for the device)
    FBox box[2];
    int32_t child[2];
};

struct SahBuilder {
    std::vector<FBox> cb;       // item boxes (conservative FP32)
    std::vector<float> cent;    // centroids [3*n]
    std::vector<float> weight;  // intersection cost of an item (slots it tests)
    std::vector<int32_t> ids;   // permutation being partitioned
    std::vector<char> solo;     // optional: items that must sit alone in a leaf (instances)
    std::vector<std::pair<int, int>> leaves;  // [b, e) ranges of ids, in creation order
    std::vector<Node2>& nodes;
    int max_depth = 0;
    int max_leaf = 4;
    float c_isect = 1.5f;  // cost of one primitive slot test relative to one node step
    static constexpr int NB = 32;

    explicit SahBuilder(std::vector<Node2>& n) : nodes(n) {}

    int make_leaf(int b, int e, FBox& out) {
        out = FBox::empty();
        for (int i = b; i < e; ++i) out.grow(cb[ids[i]]);
        leaves.emplace_back(b, e);
        return ~(int)(leaves.size() - 1);
    }

    // returns child reference (>= 0 node, < 0 ~leaf); fills `out` with the subtree box
    int build(int b, int e, int depth, FBox& out) {
        max_depth = std::max(max_depth, depth);
        const int n = e - b;
        if (n == 1) return make_leaf(b, e, out);
        FBox cbox = FBox::empty(), box = FBox::empty();
        float wsum = 0.f;
        bool any_solo = false;
        for (int i = b; i < e; ++i) {
            if (!solo.empty() && solo[ids[i]]) any_solo = true;
            FBox p;
            for (int a = 0; a < 3; ++a) p.lo[a] = p.hi[a] = cent[3 * ids[i] + a];
            cbox.grow(p);
            box.grow(cb[ids[i]]);
            wsum += weight[ids[i]];
        }
        int best_axis = -1, best_split = 0;
        float best_cost = FLT_MAX;
        for (int a = 0; a < 3; ++a) {
            float ext = cbox.hi[a] - cbox.lo[a];
            if (!(ext > 0.f)) continue;
            FBox bb[NB];
            float wb[NB] = {0};
            int cnt[NB] = {0};
            for (int k = 0; k < NB; ++k) bb[k] = FBox::empty();
            for (int i = b; i < e; ++i) {
                int k = (int)((cent[3 * ids[i] + a] - cbox.lo[a]) / ext * NB);
                k = std::min(NB - 1, std::max(0, k));
                cnt[k]++;
                wb[k] += weight[ids[i]];
                bb[k].grow(cb[ids[i]]);
            }
            float ra[NB], rw[NB];
            int rc[NB];
            FBox acc = FBox::empty();
            int c = 0;
            float w = 0.f;
            for (int k = NB - 1; k > 0; --k) {
                acc.grow(bb[k]);
                c += cnt[k];
                w += wb[k];
                ra[k] = acc.area();
                rc[k] = c;
                rw[k] = w;
            }
            acc = FBox::empty();
            c = 0;
            w = 0.f;
            for (int k = 0; k < NB - 1; ++k) {
                acc.grow(bb[k]);
                c += cnt[k];
                w += wb[k];
                if (c == 0 || rc[k + 1] == 0) continue;
                float cost = acc.area() * w + ra[k + 1] * rw[k + 1];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = a;
                    best_split = k;
                }
            }
        }
        // SAH: leaf if testing everything here is no dearer than one more node step plus the split
        const float area = box.area();
        if (n <= max_leaf && !any_solo && (best_axis < 0 || c_isect * wsum * area <= area + c_isect * best_cost))
            return make_leaf(b, e, out);
        int mid;
        if (best_axis < 0) {
            mid = (b + e) / 2;  // all centroids coincide: split by position
        } else {
            const float lo = cbox.lo[best_axis], ext = cbox.hi[best_axis] - cbox.lo[best_axis];
            // stable: the GPU build (mfx_build.hip) partitions the same way, so both builds agree
            auto it = std::stable_partition(ids.begin() + b, ids.begin() + e, [&](int id) {
                int k = (int)((cent[3 * id + best_axis] - lo) / ext * NB);
                k = std::min(NB - 1, std::max(0, k));
                return k <= best_split;
            });
            mid = (int)(it - ids.begin());
            if (mid == b || mid == e) mid = (b + e) / 2;
        }
        int self = (int)nodes.size();
        nodes.push_back(Node2{});
        FBox lb, rb;
        int l = build(b, mid, depth + 1, lb);
        int r = build(mid, e, depth + 1, rb);
        Node2& nd = nodes[self];
        nd.box[0] = lb;
        nd.box[1] = rb;
        nd.child[0] = l;
        nd.child[1] = r;
        out = lb;
        out.grow(rb);
        return self;
    }
};

// BVH2 -> BVH4: a node adopts the children of its largest-area internal child until it has four
// (Wald et al. 2008 style collapse). Preorder output; records the depth and the stack bound
// (max over nodes of the pushes its ancestors can leave on the stack plus its own).
struct Collapse4 {
    const std::vector<Node2>& n2;
    std::vector<MfxNode>& out;
    int max_depth = 0, max_stack = 0;
    std::vector<int>* leaf_stack = nullptr;  // optional: per leaf, the stack entries when it is reached

    int run(int ref, int depth, int pushed, const FBox* leaf_box = nullptr) {
        if (ref < 0 && depth > 0) {
            if (leaf_stack) (*leaf_stack)[~ref] = pushed;
            return ref;
        }
        max_depth = std::max(max_depth, depth);
        int ch[4];
        FBox bx[4];
        int nc = 2;
        if (ref < 0) {  // the whole scene is one leaf: a root node with one child
            nc = 1;
            ch[0] = ref;
            bx[0] = *leaf_box;
        } else {
            for (int k = 0; k < 2; ++k) {
                ch[k] = n2[ref].child[k];
                bx[k] = n2[ref].box[k];
            }
        }
        while (nc > 1 && nc < 4) {
            int best = -1;
            float ba = -1.f;
            for (int k = 0; k < nc; ++k)
                if (ch[k] >= 0 && bx[k].area() > ba) {
                    ba = bx[k].area();
                    best = k;
                }
            if (best < 0) break;
            const Node2& m = n2[ch[best]];
            for (int k = nc; k > best + 1; --k) {  // children of `best` replace it in place
                ch[k] = ch[k - 1];
                bx[k] = bx[k - 1];
            }
            ch[best] = m.child[0];
            bx[best] = m.box[0];
            ch[best + 1] = m.child[1];
            bx[best + 1] = m.box[1];
            ++nc;
        }
        max_stack = std::max(max_stack, pushed + nc - 1);  // node_step writes stack[pushed .. pushed + nc - 2]
        const int self = (int)out.size();
        out.push_back(MfxNode{});
        int ref4[4];
        for (int k = 0; k < nc; ++k) ref4[k] = run(ch[k], depth + 1, pushed + nc - 1);
        MfxNode& nd = out[self];
        for (int k = 0; k < 4; ++k) {
            const bool v = k < nc;
            nd.lox[k] = v ? bx[k].lo[0] : FLT_MAX;
            nd.hix[k] = v ? bx[k].hi[0] : FLT_MAX;
            nd.loy[k] = v ? bx[k].lo[1] : FLT_MAX;
            nd.hiy[k] = v ? bx[k].hi[1] : FLT_MAX;
            nd.loz[k] = v ? bx[k].lo[2] : FLT_MAX;
            nd.hiz[k] = v ? bx[k].hi[2] : FLT_MAX;
            nd.child[k] = v ? ref4[k] : MFX_CHILD_EMPTY;
            nd.pad[k] = 0;
        }
        return self;
    }
};

inline float round_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -FLT_MAX);
    return f;
}
inline float round_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, FLT_MAX);
    return f;
}

// FP64 box of a primitive in its own coordinates (Trangle.fs:113, Rect.fs:18, Sphere.fs:14-15)
Box prim_box(const mfx_prim& p) {
    if (p.kind == MFX_PRIM_SPHERE) {
        const double r = p.p[1][0];
        const D3 c = d3(p.p[0]), v{r, r, r};
        return box2(sub(c, v), add(c, v));
    }
    const Box b = tri_box(d3(p.p[0]), d3(p.p[1]), d3(p.p[2]));
    return p.kind == MFX_PRIM_RECT ? join(b, tri_box(d3(p.p[0]), d3(p.p[2]), d3(p.p[3]))) : b;
}

// A binned-SAH BVH2 over items (their conservative FP32 boxes, centroids and slot weights), built
// on the current HIP device (mfx_build.hip: the host builder's tree exactly) or on the host.
struct Tree {
    std::vector<Node2> nodes2;
    std::vector<std::pair<int, int>> leaves;  // [b, e) ranges of ids
    std::vector<int32_t> ids;
    int root2 = 0;
    FBox rootbox;
    int levels = 0;
};
bool build_tree(const std::vector<FBox>& cb, const std::vector<float>& cent, const std::vector<int32_t>& weight,
                const std::vector<char>* solo, bool gpu, int max_leaf, float c_isect, Tree& t, std::string& err) {
    const int n = (int)cb.size();
    t.nodes2.clear();
    if (gpu && !solo) {
        std::vector<float> pbox(6 * (size_t)n);
        for (int i = 0; i < n; ++i)
            for (int a = 0; a < 3; ++a) {
                pbox[6 * (size_t)i + a] = cb[i].lo[a];
                pbox[6 * (size_t)i + 3 + a] = cb[i].hi[a];
            }
        MfxBvh2 g;
        const hipError_t he = mfx_gpu_sah_build(pbox.data(), cent.data(), weight.data(), n, max_leaf, c_isect, g);
        if (he != hipSuccess) {
            err = std::string("GPU BVH build: ") + hipGetErrorString(he);
            return false;
        }
        t.nodes2.resize(g.child.size() / 2);
        for (size_t i = 0; i < t.nodes2.size(); ++i)
            for (int k = 0; k < 2; ++k) {
                t.nodes2[i].child[k] = g.child[2 * i + k];
                for (int a = 0; a < 3; ++a) {
                    t.nodes2[i].box[k].lo[a] = g.box[(2 * i + k) * 6 + a];
                    t.nodes2[i].box[k].hi[a] = g.box[(2 * i + k) * 6 + 3 + a];
                }
            }
        t.leaves.clear();
        for (size_t l = 0; l < g.leaf_b.size(); ++l) t.leaves.emplace_back(g.leaf_b[l], g.leaf_e[l]);
        t.ids = g.ids;
        t.root2 = g.root;
        for (int a = 0; a < 3; ++a) {
            t.rootbox.lo[a] = g.root_box[a];
            t.rootbox.hi[a] = g.root_box[3 + a];
        }
        t.levels = g.levels;
        return true;
    }
    SahBuilder sb(t.nodes2);
    sb.max_leaf = max_leaf;
    sb.c_isect = c_isect;
    sb.cb = cb;
    sb.cent = cent;
    sb.weight.resize(n);
    sb.ids.resize(n);
    for (int i = 0; i < n; ++i) {
        sb.weight[i] = (float)weight[i];
        sb.ids[i] = i;
    }
    if (solo) sb.solo = *solo;
    t.root2 = sb.build(0, n, 0, t.rootbox);
    t.levels = sb.max_depth + 1;
    t.leaves = sb.leaves;
    t.ids = sb.ids;
    return true;
}

// leaves (~child refs) of a BVH4 in depth-first order, children in order
std::vector<int> dfs_leaves(const std::vector<MfxNode>& nodes, int root) {
    std::vector<int> order, st{root};
    while (!st.empty()) {
        const int ref = st.back();
        st.pop_back();
        if (ref < 0) {
            order.push_back(~ref);
        } else {
            for (int k = 3; k >= 0; --k)
                if (nodes[ref].child[k] != MFX_CHILD_EMPTY) st.push_back(nodes[ref].child[k]);
        }
    }
    return order;
}

}  // namespace

bool mfx_expand(const mfx_prim* prims, int64_t nprims, const mfx_instance* inst, int ninst,
                std::vector<mfx_prim>& world, std::string& err) {
    world.clear();
    if (!prims || nprims < 1 || !inst || ninst < 1) {
        err = "an instanced scene needs template primitives and at least one instance";
        return false;
    }
    int64_t total = 0;
    for (int k = 0; k < ninst; ++k) {
        const mfx_instance& e = inst[k];
        if (e.first < 0 || e.count < 0 || e.first > nprims || e.count > nprims - e.first) {
            err = "instance " + std::to_string(k) + " names primitives outside the template array";
            return false;
        }
        if (e.flags & ~MFX_INSTANCE_VERBATIM) {
            err = "instance " + std::to_string(k) + " has unknown flags";
            return false;
        }
        total += e.count;
    }
    if (total < 1 || total > (1 << 28)) {
        err = total < 1 ? "the instances expand to no primitive" : "too many primitives";
        return false;
    }
    world.reserve((size_t)total);
    for (int k = 0; k < ninst; ++k) {
        const mfx_instance& e = inst[k];
        for (int64_t i = 0; i < e.count; ++i) {
            mfx_prim p = prims[e.first + i];
            if (!(e.flags & MFX_INSTANCE_VERBATIM)) {
                const int nv = p.kind == MFX_PRIM_SPHERE ? 1 : (p.kind == MFX_PRIM_RECT ? 4 : 3);
                for (int v = 0; v < nv; ++v)
                    for (int a = 0; a < 3; ++a) p.p[v][a] = p.p[v][a] + e.offset[a];
            }
            world.push_back(p);
        }
    }
    return true;
}

bool mfx_build_scene(const mfx_scene_desc* d0, MfxHostScene& s, std::string& err, bool gpu_bvh,
                     const mfx_instance* instances, int ninstances, bool flatten) {
    using clock = std::chrono::steady_clock;
    const auto t_start = clock::now();
    auto ms_since = [](clock::time_point t0) {
        return std::chrono::duration<double, std::milli>(clock::now() - t0).count();
    };
    // ---- an instanced scene stands for its expansion (mfx_instance); translated entries that
    //      share a template range are traced two-level through one template BVH ----------------
    const mfx_scene_desc* d = d0;
    mfx_scene_desc dw;
    std::vector<mfx_prim> world;
    struct Use {
        int64_t wbase, count;  // its world primitives
        double off[3];
        int tmpl;
    };
    std::vector<Use> uses;
    std::vector<std::pair<int64_t, int64_t>> templates;  // (first, count) in the template array
    if (instances) {
        if (!d0) {
            err = "null scene";
            return false;
        }
        if (!mfx_expand(d0->prims, d0->nprims, instances, ninstances, world, err)) return false;
        dw = *d0;
        dw.prims = world.data();
        dw.nprims = (int64_t)world.size();
        d = &dw;
        std::vector<int> uses_of_range(ninstances, 0);
        for (int k = 0; k < ninstances; ++k)
            for (int q = 0; q < ninstances; ++q)
                if (!(instances[q].flags & MFX_INSTANCE_VERBATIM) && instances[q].first == instances[k].first &&
                    instances[q].count == instances[k].count)
                    ++uses_of_range[k];
        int64_t wb = 0;
        for (int k = 0; k < ninstances; ++k) {
            const mfx_instance& e = instances[k];
            if (!flatten && !(e.flags & MFX_INSTANCE_VERBATIM) && e.count > 0 && uses_of_range[k] >= 2) {
                int tm = 0;
                while (tm < (int)templates.size() && templates[tm] != std::make_pair(e.first, e.count)) ++tm;
                if (tm == (int)templates.size()) templates.emplace_back(e.first, e.count);
                uses.push_back(Use{wb, e.count, {e.offset[0], e.offset[1], e.offset[2]}, tm});
            }
            wb += e.count;
        }
        if ((int)uses.size() > MFX_INST_MAX) {
            err = "too many instances";
            return false;
        }
    }
    if (!d || !d->prims || d->nprims < 1) {
        err = "scene has no primitives (Bvh.Build on an empty array throws, BvhNode.fs:26)";
        return false;
    }
    if (d->nprims > (1 << 28)) {
        err = "too many primitives";
        return false;
    }
    if (d->width < 1 || d->height < 1 || d->nmat < 1 || !d->albedo) {
        err = "invalid film size or empty material table";
        return false;
    }
    // one sample of the film is ceil(w/8) * ceil(h/8) 8x8 tiles of path slots, indexed in 32-bit
    // arithmetic by the kernels (path_pixel, k_resolve): reject films whose count reaches 2^31
    if ((int64_t)((d->width + 7) / 8) * ((d->height + 7) / 8) * 64 >= ((int64_t)1 << 31)) {
        err = "film too large: padded paths per sample must stay below 2^31";
        return false;
    }
    // PathIntegrator(bvh, maxDepth, light) with maxDepth < 0 still traces the camera ray and
    // returns black (Integrators.fs:108-109); the reference only ever passes 3 (Scene.fs:304)
    if (d->max_depth < 0) {
        err = "max_depth must be >= 0";
        return false;
    }
    // a path's vertices are recorded for the exact fold (mfx_wavefront.h): at most 16 of them
    if (d->max_depth >= 16) {
        err = "max_depth must be <= 15 (the reference uses 3, Scene.fs:304)";
        return false;
    }
    const int n = (int)d->nprims;
    s.width = d->width;
    s.height = d->height;
    s.max_depth = d->max_depth;
    s.albedo.assign(d->albedo, d->albedo + 3 * (size_t)d->nmat);

    // ---- primitives: FP64 bounds + slot records (in primitive order for now) ---------------
    std::vector<Box> pb(n);
    std::vector<int32_t> slot_of(n), nslot_of(n);
    std::vector<MfxSlot> pslots;
    std::vector<MfxShade> pshade;
    auto add_tri = [&](D3 v0, D3 v1, D3 v2, int mat, int prim, int kind) {
        MfxSlot t{};
        D3 e1 = sub(v1, v0), e2 = sub(v2, v0);
        put(t.a, v0);
        put(t.b, e1);
        put(t.c, e2);
        pslots.push_back(t);
        MfxShade sh{};
        D3 a = cross(e1, e2);
        double al = len(a);
        put(sh.n, D3{a.x / al, a.y / al, a.z / al});  // Trangle.fs:110-111
        sh.material = mat;
        std::memcpy(sh.albedo, d->albedo + 3 * (size_t)mat, sizeof(sh.albedo));
        sh.prim_kind = (prim << 2) | kind;
        pshade.push_back(sh);
    };
    for (int i = 0; i < n; ++i) {
        const mfx_prim& p = d->prims[i];
        if (p.material < 0 || p.material >= d->nmat) {
            err = "primitive " + std::to_string(i) + " has material index out of range";
            return false;
        }
        slot_of[i] = (int)pslots.size();
        if (p.kind == MFX_PRIM_TRIANGLE) {
            D3 v0 = d3(p.p[0]), v1 = d3(p.p[1]), v2 = d3(p.p[2]);
            pb[i] = tri_box(v0, v1, v2);
            add_tri(v0, v1, v2, p.material, i, MFX_KIND_TRI);
        } else if (p.kind == MFX_PRIM_RECT) {
            D3 v0 = d3(p.p[0]), v1 = d3(p.p[1]), v2 = d3(p.p[2]), v3 = d3(p.p[3]);
            pb[i] = join(tri_box(v0, v1, v2), tri_box(v0, v2, v3));  // Rect.fs:18
            add_tri(v0, v1, v2, p.material, i, MFX_KIND_RECT);
            add_tri(v0, v2, v3, p.material, i, MFX_KIND_RECT);
        } else if (p.kind == MFX_PRIM_SPHERE) {
            D3 c = d3(p.p[0]);
            double r = p.p[1][0];
            D3 v{r, r, r};
            pb[i] = box2(sub(c, v), add(c, v));  // Sphere.fs:14-15
            MfxSlot t{};
            put(t.a, c);
            t.b[0] = r;
            pslots.push_back(t);
            MfxShade sh{};
            put(sh.n, c);  // the shade record of a sphere carries its centre
            sh.material = p.material;
            std::memcpy(sh.albedo, d->albedo + 3 * (size_t)p.material, sizeof(sh.albedo));
            sh.prim_kind = (i << 2) | MFX_KIND_SPHERE;
            pshade.push_back(sh);
        } else {
            err = "primitive " + std::to_string(i) + " has an unknown kind";
            return false;
        }
        nslot_of[i] = (int)pslots.size() - slot_of[i];
    }

    // ---- reference leaf grouping -----------------------------------------------------------
    s.ref_indices.resize(n);
    for (int i = 0; i < n; ++i) s.ref_indices[i] = i;
    s.leaf_first.clear();
    s.leaf_count.clear();
    {
        const auto t0 = clock::now();
        RefBvh rb{pb, s.ref_indices, std::vector<double>(n), std::vector<int32_t>(n)};
        Box root = rb.bound(0, n);
        rb.subdivide(0, n, root, s.leaf_first, s.leaf_count, 3);  // up to 8 host threads
        s.ms_ref_bvh = ms_since(t0);
    }
    const int nc = (int)s.leaf_first.size();
    std::vector<MfxLeaf> leaves(nc);
    for (int c = 0; c < nc; ++c) {
        MfxLeaf& lf = leaves[c];
        Box b = pb[s.ref_indices[s.leaf_first[c]]];
        for (int k = 1; k < s.leaf_count[c]; ++k) b = join(b, pb[s.ref_indices[s.leaf_first[c] + k]]);
        put(lf.lo, b.lo);
        put(lf.hi, b.hi);
        lf.first = s.leaf_first[c];
        lf.count = s.leaf_count[c];
        lf.pad = 0;
        lf.kinds = 0;
        for (int k = 0; k < lf.count; ++k) lf.kinds |= d->prims[s.ref_indices[lf.first + k]].kind << (2 * k);
    }

    // ---- camera (Camera.fs:96-133) and light (Light.fs:31-40) -------------------------------
    {
        const mfx_pinhole& c = d->camera;
        D3 fwd = normalize(d3(c.direction));
        D3 up0 = normalize(D3{0, 1, 0});
        D3 hori0 = cross(fwd, normalize(up0));
        D3 vert0 = cross(hori0, fwd);
        double hori = std::tan(0.5 * c.fov * 3.141592653589793 / 360.);
        double vert = hori / c.aspect;
        D3 up = scale(vert0, vert), right = scale(hori0, hori);
        D3 pos = d3(c.position);
        D3 tl = add(sub(add(pos, scale(fwd, 0.5)), scale(right, 0.5)), scale(up, 0.5));
        put(s.camera.position, pos);
        put(s.camera.topleft, tl);
        put(s.camera.right, right);
        put(s.camera.down, D3{-up.x, -up.y, -up.z});
        if (c.derived) {  // an existing PinholeCamera's fields, taken as they are
            put(s.camera.topleft, d3(c.topleft));
            put(s.camera.right, d3(c.right));
            put(s.camera.down, d3(c.down));
        }
    }
    {
        const mfx_quad_light& L = d->light;
        D3 q[4] = {d3(L.p[0]), d3(L.p[1]), d3(L.p[2]), d3(L.p[3])};
        D3 tv[2][3] = {{q[0], q[1], q[2]}, {q[0], q[2], q[3]}};
        double area = 0;
        for (int t = 0; t < 2; ++t) {
            D3 e1 = sub(tv[t][1], tv[t][0]), e2 = sub(tv[t][2], tv[t][0]);
            put(s.light.v0[t], tv[t][0]);
            put(s.light.e1[t], e1);
            put(s.light.e2[t], e2);
            double al = len(cross(e1, e2));
            double ta = al * 0.5;  // Trangle.fs:114
            area = (t == 0) ? ta : area + ta;
        }
        s.light.area = area;
        s.light.pdf = 1. / area;
        put(s.light.normal, d3(L.normal));
        put(s.light.color, d3(L.intensity));
    }

    // ---- conservative FP32 primitive boxes --------------------------------------------------
    double R = 0, T = 0;
    {
        Box all = pb[0];
        for (int i = 1; i < n; ++i) all = join(all, pb[i]);
        for (double v : {all.lo.x, all.lo.y, all.lo.z, all.hi.x, all.hi.y, all.hi.z}) R = std::max(R, std::fabs(v));
        for (int a = 0; a < 3; ++a) R = std::max(R, std::fabs(d->camera.position[a]));
        T = len(sub(all.hi, all.lo)) + len(sub(d3(d->camera.position), scale(add(all.lo, all.hi), 0.5)));
        for (int k = 0; k < 4; ++k)
            for (int a = 0; a < 3; ++a) R = std::max(R, std::fabs(d->light.p[k][a]));
    }
    s.eps = (float)std::ldexp(R + T, -19);
    int max_leaf = 4;
    float c_isect = 1.5f;
    if (const char* e = getenv("MFX_LEAF_MAX")) max_leaf = std::max(1, std::min(4, atoi(e)));
    if (const char* e = getenv("MFX_SAH_CI")) c_isect = (float)atof(e);
    auto fbox_of = [&](const Box& b, float eps) {
        FBox f;
        for (int a = 0; a < 3; ++a) {
            f.lo[a] = round_down(comp(b.lo, a) - (double)eps);
            f.hi[a] = round_up(comp(b.hi, a) + (double)eps);
        }
        return f;
    };
    const auto t_bvh = clock::now();
    s.bvh_gpu = gpu_bvh;
    s.bvh_levels = 0;
    s.nodes2 = 0;

    // ---- where each primitive sits in the reference grouping --------------------------------
    std::vector<int32_t> ref_leaf_of(n), pos_of(n);
    for (int c = 0; c < nc; ++c)
        for (int k = 0; k < leaves[c].count; ++k) {
            ref_leaf_of[s.ref_indices[leaves[c].first + k]] = c;
            pos_of[s.ref_indices[leaves[c].first + k]] = k;
        }
    std::vector<int32_t> ref16(nc);
    {
        size_t off = 0;
        for (int c = 0; c < nc; ++c) {
            ref16[c] = (int32_t)(off / 16);
            off += sizeof(MfxLeaf);
            for (int k = 0; k < leaves[c].count; ++k) off += sizeof(MfxSlot) * nslot_of[s.ref_indices[leaves[c].first + k]];
        }
        if (off / 16 >= (size_t)0x7fffffff) {
            err = "reference-leaf image too large";
            return false;
        }
    }
    auto slot_info = [&](int p, int j, int32_t shade) {
        return shade | (pos_of[p] << MFX_INFO_POS_SHIFT) | (d->prims[p].kind << MFX_INFO_KIND_SHIFT) |
               (j == 1 ? MFX_INFO_RECT2 : 0);
    };

    // ---- traversal images --------------------------------------------------------------------
    std::vector<int32_t> shade_of(n, -1);  // shade[] index of each world primitive's first slot
    s.slots.clear();
    s.slot_ref.clear();
    s.shade.clear();
    s.inst.clear();
    s.tlas_nodes = s.blas_nodes = s.blas_slots = s.ntemplates = 0;
    s.top_slots = 0;
    s.images_gpu = false;
    // a world primitive's slots at the end of slots[] (the top level / the flat BVH), shade[] in step
    auto emit_world_prim = [&](int p) {
        const MfxLeaf& rl = leaves[ref_leaf_of[p]];
        shade_of[p] = (int32_t)s.shade.size();
        for (int j = 0; j < nslot_of[p]; ++j) {
            MfxSlot sl = pslots[slot_of[p] + j];
            std::memcpy(sl.lo, rl.lo, sizeof(sl.lo));
            std::memcpy(sl.hi, rl.hi, sizeof(sl.hi));
            sl.first = rl.first;
            sl.info = slot_info(p, j, (int32_t)s.shade.size());
            s.slots.push_back(sl);
            s.slot_ref.push_back(ref16[ref_leaf_of[p]]);
            s.shade.push_back(pshade[slot_of[p] + j]);
        }
    };
    // a traversal leaf's child code once its slots [s0, slots.size()) are emitted
    auto leaf_code = [&](int s0, int32_t& code) {
        const int ns = (int)s.slots.size() - s0;
        if (ns > MFX_LEAF_SLOTS_MAX || s0 >= MFX_SLOTS_MAX) {
            err = "scene too large for the traversal image";
            return false;
        }
        code = (s0 << 3) | (ns - 1);
        return true;
    };
    std::vector<int> roots;  // tree roots in nodes[] before renumbering: the top level first
    if (uses.empty()) {
        // ---- flat: one SAH BVH2 over the primitives, collapsed to a BVH4 ---------------------
        std::vector<FBox> cb(n);
        std::vector<float> cent(3 * (size_t)n);
        std::vector<int32_t> w(n);
        for (int i = 0; i < n; ++i) {
            cb[i] = fbox_of(pb[i], s.eps);
            for (int a = 0; a < 3; ++a) cent[3 * i + a] = 0.5f * (cb[i].lo[a] + cb[i].hi[a]);
            w[i] = nslot_of[i];
        }
        if (gpu_bvh) {
            // the whole image on the GPU: BVH2, BVH4 collapse, renumbering, slots in depth-first
            // order (mfx_build.hip; the host path's bytes)
            std::vector<MfxSlot> ps(pslots.size());
            std::vector<int32_t> so(n + 1), r16(n);
            for (int p = 0; p < n; ++p) {
                so[p] = slot_of[p];
                r16[p] = ref16[ref_leaf_of[p]];
                const MfxLeaf& rl = leaves[ref_leaf_of[p]];
                for (int j = 0; j < nslot_of[p]; ++j) {
                    MfxSlot sl = pslots[slot_of[p] + j];
                    std::memcpy(sl.lo, rl.lo, sizeof(sl.lo));
                    std::memcpy(sl.hi, rl.hi, sizeof(sl.hi));
                    sl.first = rl.first;
                    sl.info = slot_info(p, j, 0);
                    ps[slot_of[p] + j] = sl;
                }
            }
            so[n] = (int32_t)pslots.size();
            if (pslots.size() >= (size_t)MFX_SLOTS_MAX) {
                err = "scene too large for the traversal image";
                return false;
            }
            std::vector<float> pbox(6 * (size_t)n);
            for (int i = 0; i < n; ++i)
                for (int a = 0; a < 3; ++a) {
                    pbox[6 * (size_t)i + a] = cb[i].lo[a];
                    pbox[6 * (size_t)i + 3 + a] = cb[i].hi[a];
                }
            MfxGpuImages g;
            const hipError_t he = mfx_gpu_build_images(
                pbox.data(), cent.data(), w.data(), n, max_leaf, c_isect,
                MfxGpuLayoutIn{ps.data(), pshade.data(), so.data(), r16.data(), (int32_t)pslots.size(), MFX_TOP_NODES},
                g);
            if (he != hipSuccess) {
                err = std::string("GPU BVH build: ") + hipGetErrorString(he);
                return false;
            }
            s.nodes.swap(g.nodes);
            s.slots.swap(g.slots);
            s.slots.resize(pslots.size());
            s.slot_ref.swap(g.slot_ref);
            s.shade.swap(g.shade);
            shade_of.swap(g.shade_of);
            s.bvh_levels = g.levels;
            s.nodes2 = g.nodes2;
            s.bvh_depth = g.max_depth;
            s.stack_entries = std::max(1, g.max_stack);
            s.ntleaves = g.nleaves;
            s.top_slots = (int32_t)s.slots.size();
            s.images_gpu = true;
            roots.push_back(0);  // already numbered: the renumbering below is the identity
        } else {
        Tree t;
        if (!build_tree(cb, cent, w, nullptr, false, max_leaf, c_isect, t, err)) return false;
        s.bvh_levels = t.levels;
        s.nodes2 = (int32_t)t.nodes2.size();
        s.nodes.clear();
        Collapse4 c4{t.nodes2, s.nodes};
        const int root = c4.run(t.root2, 0, 0, &t.rootbox);  // always an internal node (a lone leaf gets a parent)
        s.bvh_depth = c4.max_depth;
        s.stack_entries = std::max(1, c4.max_stack);
        std::vector<int32_t> code_of(t.leaves.size());
        for (int l : dfs_leaves(s.nodes, root)) {
            const int s0 = (int)s.slots.size();
            for (int k = t.leaves[l].first; k < t.leaves[l].second; ++k) emit_world_prim(t.ids[k]);
            if (!leaf_code(s0, code_of[l])) return false;
        }
        for (MfxNode& nd : s.nodes)
            for (int k = 0; k < 4; ++k)
                if (nd.child[k] != MFX_CHILD_EMPTY && nd.child[k] < 0) nd.child[k] = ~code_of[~nd.child[k]];
        s.ntleaves = (int32_t)t.leaves.size();
        s.top_slots = (int32_t)s.slots.size();
        roots.push_back(root);
        }
    } else {
        // ---- two levels: a top-level BVH over the loose primitives and the instances, one
        //      template BVH per distinct template range (local coordinates) ---------------------
        const int K = (int)uses.size();
        std::vector<int> use_of(n, -1);
        for (int k = 0; k < K; ++k)
            for (int64_t i = 0; i < uses[k].count; ++i) use_of[uses[k].wbase + i] = k;
        double offmax = 0;
        for (const Use& u : uses)
            for (int a = 0; a < 3; ++a) offmax = std::max(offmax, std::fabs(u.off[a]));
        // template frame: coordinates and ray origins up to R + |off| in magnitude
        const float eps_t = (float)std::ldexp(R + offmax + T, -19);
        // top level: loose primitives (items 0 .. nl-1), then the instances (solo leaves)
        std::vector<int> loose;
        for (int i = 0; i < n; ++i)
            if (use_of[i] < 0) loose.push_back(i);
        const int nl = (int)loose.size(), ni = nl + K;
        std::vector<FBox> cb(ni);
        std::vector<float> cent(3 * (size_t)ni);
        std::vector<int32_t> w(ni);
        std::vector<char> solo(ni, 0);
        for (int i = 0; i < nl; ++i) {
            cb[i] = fbox_of(pb[loose[i]], s.eps);
            w[i] = nslot_of[loose[i]];
        }
        for (int k = 0; k < K; ++k) {
            FBox f = FBox::empty();
            for (int64_t i = 0; i < uses[k].count; ++i) f.grow(fbox_of(pb[uses[k].wbase + i], s.eps));
            cb[nl + k] = f;
            w[nl + k] = 8;  // ~ a few node steps and leaves: only steers the top-level SAH
            solo[nl + k] = 1;
        }
        for (int i = 0; i < ni; ++i)
            for (int a = 0; a < 3; ++a) cent[3 * i + a] = 0.5f * (cb[i].lo[a] + cb[i].hi[a]);
        Tree tt;
        if (!build_tree(cb, cent, w, &solo, false, max_leaf, c_isect, tt, err)) return false;
        std::vector<MfxNode> top;
        std::vector<int> at_leaf(tt.leaves.size(), 0);
        Collapse4 ct{tt.nodes2, top};
        ct.leaf_stack = &at_leaf;
        const int troot = ct.run(tt.root2, 0, 0, &tt.rootbox);
        if (tt.root2 < 0) at_leaf[~tt.root2] = 0;  // a lone leaf under the root: nothing pushed
        std::vector<int32_t> tcode(tt.leaves.size());
        for (int l : dfs_leaves(top, troot)) {
            const int b = tt.leaves[l].first, e = tt.leaves[l].second;
            if (e - b == 1 && tt.ids[b] >= nl) {  // an instance: entered, not tested
                tcode[l] = MFX_INST_FLAG | (tt.ids[b] - nl);
                continue;
            }
            const int s0 = (int)s.slots.size();
            for (int k = b; k < e; ++k) emit_world_prim(loose[tt.ids[k]]);
            if (!leaf_code(s0, tcode[l])) return false;
        }
        s.nodes = top;
        for (MfxNode& nd : s.nodes)
            for (int k = 0; k < 4; ++k)
                if (nd.child[k] != MFX_CHILD_EMPTY && nd.child[k] < 0) nd.child[k] = ~tcode[~nd.child[k]];
        s.tlas_nodes = (int32_t)top.size();
        s.top_slots = (int32_t)s.slots.size();
        s.ntleaves = (int32_t)tt.leaves.size();
        roots.push_back(troot);
        s.bvh_depth = ct.max_depth;
        std::vector<int> blas_stack;
        int blas_depth = 0;
        s.blas_slots = 0;
        // template BVHs over the template primitives (local coordinates); their leaf codes count
        // slots from the instance's own run of world slots: tslot[t][i] = template primitive i's
        // first slot in such a run (the template's depth-first leaf order)
        std::vector<int> tmpl_root, tmpl_nslots;
        std::vector<std::vector<int32_t>> tslot;
        for (int tm = 0; tm < (int)templates.size(); ++tm) {
            const int64_t tf = templates[tm].first;
            const int tn = (int)templates[tm].second;
            std::vector<FBox> tb(tn);
            std::vector<float> tc(3 * (size_t)tn);
            std::vector<int32_t> tw(tn);
            for (int i = 0; i < tn; ++i) {
                const mfx_prim& p = d0->prims[tf + i];
                tb[i] = fbox_of(prim_box(p), eps_t);
                for (int a = 0; a < 3; ++a) tc[3 * i + a] = 0.5f * (tb[i].lo[a] + tb[i].hi[a]);
                tw[i] = p.kind == MFX_PRIM_RECT ? 2 : 1;
            }
            const int base = (int)s.nodes.size();
            std::vector<int32_t> ts(tn);
            std::vector<MfxNode> bn;
            int broot = 0, local = 0, nleaves = 0;
            if (gpu_bvh) {  // BVH2, collapse and layout on the GPU, nodes in preorder (as Collapse4 emits them)
                std::vector<int32_t> so(tn + 1), r16(tn, 0);
                for (int i = 0; i <= tn; ++i) so[i] = i == 0 ? 0 : so[i - 1] + tw[i - 1];
                std::vector<MfxSlot> ps(so[tn]);
                std::vector<MfxShade> psh(so[tn]);
                std::vector<float> pbox(6 * (size_t)tn);
                for (int i = 0; i < tn; ++i)
                    for (int a = 0; a < 3; ++a) {
                        pbox[6 * (size_t)i + a] = tb[i].lo[a];
                        pbox[6 * (size_t)i + 3 + a] = tb[i].hi[a];
                    }
                MfxGpuImages g;
                const hipError_t he = mfx_gpu_build_images(pbox.data(), tc.data(), tw.data(), tn, max_leaf, c_isect,
                                                           MfxGpuLayoutIn{ps.data(), psh.data(), so.data(), r16.data(),
                                                                          so[tn], 0},
                                                           g);
                if (he != hipSuccess) {
                    err = std::string("GPU BVH build: ") + hipGetErrorString(he);
                    return false;
                }
                bn.swap(g.nodes);
                ts.swap(g.shade_of);  // a template primitive's first slot in the run
                local = so[tn];
                nleaves = g.nleaves;
                blas_stack.push_back(g.max_stack);
                blas_depth = std::max(blas_depth, g.max_depth);
                s.bvh_levels = std::max(s.bvh_levels, g.levels);
                s.nodes2 += g.nodes2;
                for (MfxNode& nd : bn)
                    for (int k = 0; k < 4; ++k)
                        if (nd.child[k] >= 0) nd.child[k] += base;
            } else {
                Tree bt;
                if (!build_tree(tb, tc, tw, nullptr, false, max_leaf, c_isect, bt, err)) return false;
                s.bvh_levels = std::max(s.bvh_levels, bt.levels);
                s.nodes2 += (int32_t)bt.nodes2.size();
                Collapse4 cbv{bt.nodes2, bn};
                broot = cbv.run(bt.root2, 0, 0, &bt.rootbox);
                blas_stack.push_back(cbv.max_stack);
                blas_depth = std::max(blas_depth, cbv.max_depth);
                std::vector<int32_t> bcode(bt.leaves.size());
                for (int l : dfs_leaves(bn, broot)) {
                    const int s0 = local;
                    for (int k = bt.leaves[l].first; k < bt.leaves[l].second; ++k) {
                        const int i = bt.ids[k];
                        ts[i] = local;
                        local += tw[i];
                    }
                    if (local - s0 > MFX_LEAF_SLOTS_MAX || s0 >= MFX_SLOTS_MAX) {
                        err = "scene too large for the traversal image";
                        return false;
                    }
                    bcode[l] = (s0 << 3) | (local - s0 - 1);
                }
                for (MfxNode& nd : bn)
                    for (int k = 0; k < 4; ++k) {
                        if (nd.child[k] == MFX_CHILD_EMPTY) continue;
                        nd.child[k] = nd.child[k] >= 0 ? nd.child[k] + base : ~bcode[~nd.child[k]];
                    }
                nleaves = (int)bt.leaves.size();
            }
            s.nodes.insert(s.nodes.end(), bn.begin(), bn.end());
            tmpl_root.push_back(base + broot);
            tmpl_nslots.push_back(local);
            roots.push_back(base + broot);
            tslot.push_back(std::move(ts));
            s.ntleaves += nleaves;
            s.blas_nodes += (int32_t)bn.size();
            s.blas_slots += local;
        }
        s.ntemplates = (int32_t)templates.size();
        // per instance: its own run of world slots (exact world geometry and reference-leaf data, as
        // a flat image holds them) in its template's slot order; shade[] stays in slots[] order
        for (int k = 0; k < K; ++k) {
            const Use& u = uses[k];
            const int tm = u.tmpl, nts = tmpl_nslots[tm];
            MfxInstance I{};
            std::memcpy(I.off, u.off, sizeof(I.off));
            I.root = tmpl_root[tm];
            I.slot_base = (int32_t)s.slots.size();
            if ((int64_t)I.slot_base + nts >= MFX_SLOTS_MAX) {
                err = "scene too large for the traversal image";
                return false;
            }
            s.slots.resize(s.slots.size() + nts);
            s.slot_ref.resize(s.slot_ref.size() + nts);
            s.shade.resize(s.shade.size() + nts);
            for (int64_t i = 0; i < u.count; ++i) {
                const int p = (int)(u.wbase + i);
                const int at = I.slot_base + tslot[tm][i];
                shade_of[p] = at;
                const MfxLeaf& rl = leaves[ref_leaf_of[p]];
                for (int j = 0; j < nslot_of[p]; ++j) {
                    MfxSlot sl = pslots[slot_of[p] + j];
                    std::memcpy(sl.lo, rl.lo, sizeof(sl.lo));
                    std::memcpy(sl.hi, rl.hi, sizeof(sl.hi));
                    sl.first = rl.first;
                    sl.info = slot_info(p, j, at + j);
                    s.slots[at + j] = sl;
                    s.slot_ref[at + j] = ref16[ref_leaf_of[p]];
                    s.shade[at + j] = pshade[slot_of[p] + j];
                }
            }
            s.inst.push_back(I);
        }
        // the top level's entries when an instance is reached, then the template's own
        int bound = ct.max_stack;
        for (size_t l = 0; l < tt.leaves.size(); ++l) {
            const int b = tt.leaves[l].first;
            if (tt.leaves[l].second - b == 1 && tt.ids[b] >= nl)
                bound = std::max(bound, at_leaf[l] + blas_stack[uses[tt.ids[b] - nl].tmpl]);
        }
        s.stack_entries = std::max(1, bound);
        s.bvh_depth += blas_depth;
    }
    s.ms_bvh = ms_since(t_bvh);
    if (s.shade.size() > MFX_INFO_SHADE_MASK) {
        err = "scene too large for the traversal image";
        return false;
    }
    s.slots.resize(s.slots.size() + MFX_LEAF_SLOTS_MAX, MfxSlot{});  // speculative slot loads stay in bounds

    // ---- renumber: the first MFX_TOP_NODES nodes breadth-first from the root(s) — the top level,
    //      then the template BVHs' top levels —, then the rest in their order (mfx_layout.h) ------
    {
        const int nn = (int)s.nodes.size();
        std::vector<int> bfs{roots[0]};
        size_t h = 0, next_root = 1;
        while ((int)bfs.size() < MFX_TOP_NODES) {
            if (h == bfs.size()) {
                if (next_root == roots.size()) break;
                bfs.push_back(roots[next_root++]);
                continue;
            }
            for (int k = 0; k < 4 && (int)bfs.size() < MFX_TOP_NODES; ++k)
                if (s.nodes[bfs[h]].child[k] >= 0) bfs.push_back(s.nodes[bfs[h]].child[k]);
            ++h;
        }
        std::vector<int> idx(nn, -1);
        int next = 0;
        for (int v : bfs) idx[v] = next++;
        for (int v = 0; v < nn; ++v)
            if (idx[v] < 0) idx[v] = next++;
        std::vector<MfxNode> renum(nn);
        for (int v = 0; v < nn; ++v) {
            MfxNode nd = s.nodes[v];
            for (int k = 0; k < 4; ++k)
                if (nd.child[k] >= 0) nd.child[k] = idx[nd.child[k]];
            renum[idx[v]] = nd;
        }
        s.nodes.swap(renum);
        for (MfxInstance& I : s.inst) I.root = idx[I.root];
    }

    // ---- reference leaves (heap order): FP64 box header + slot copies ----------------------
    s.ref_blob.clear();
    for (int c = 0; c < nc; ++c) {
        const uint8_t* hp = (const uint8_t*)&leaves[c];
        s.ref_blob.insert(s.ref_blob.end(), hp, hp + sizeof(MfxLeaf));
        for (int k = 0; k < leaves[c].count; ++k) {
            const int p = s.ref_indices[leaves[c].first + k];
            for (int j = 0; j < nslot_of[p]; ++j) {
                MfxSlot sl = pslots[slot_of[p] + j];
                std::memcpy(sl.lo, leaves[c].lo, sizeof(sl.lo));
                std::memcpy(sl.hi, leaves[c].hi, sizeof(sl.hi));
                sl.first = leaves[c].first;
                sl.info = (shade_of[p] + j) | (k << MFX_INFO_POS_SHIFT);
                const uint8_t* sp = (const uint8_t*)&sl;
                s.ref_blob.insert(s.ref_blob.end(), sp, sp + sizeof(MfxSlot));
            }
        }
    }
    s.ref_blob.resize(s.ref_blob.size() + 3 * sizeof(MfxSlot), 0);
    s.nclusters = nc;
    s.world_slots = (int32_t)pslots.size();
    s.ms_total = ms_since(t_start);
    return true;
}
