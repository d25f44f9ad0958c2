// mfx_wide.cpp — BVH4 -> BVH8 for the per-lane traversal (MfxNode8H, mfx_layout.h).
//
// The per-lane kernels (k_extend, k_shadow, the megakernel, the query kernels) pay a wave-wide
// round of the node loop per node step, and a wave's node loop runs until its slowest lane is
// done. A wider node needs fewer rounds for the same line per lane per round, as
// long as the node stays one 128-B line: 8 child boxes in FP16 (outward-rounded, so they contain
// the FP32 boxes the search is conservative over) and 8 child codes. The camera packets (k_camera)
// keep the BVH4: their node loads are scalar, and a packet tests every child anyway.
//
// Collapse (the usual greedy one): a wide node starts as a BVH4 node's children and repeatedly
// replaces the internal child of largest surface area by that child's children while the entries
// stay at most 8. Leaves keep their BVH4 leaf codes, so leaf_hit, the slots and every result are
// unchanged: the leaf semantics are per candidate and independent of the visiting order
// (mfx_trace_common.h, leaf_hit).
#include "mfx_wide.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <functional>

static uint16_t half_bits_at(int k) {  // the non-NaN FP16 values in ascending order: 0 is -inf
    return k <= 0x7C00 ? (uint16_t)(0x8000 | (0x7C00 - k)) : (uint16_t)(k - 0x7C01);
}
static int half_index(uint16_t h) { return (h & 0x8000) ? 0x7C00 - (h & 0x7FFF) : h + 0x7C01; }
static const int kHalfMax = 2 * 0x7C00 + 1;  // index of +inf

double mfx_half_value(uint16_t h) {
    const int e = (h >> 10) & 31, m = h & 1023;
    const double v = e == 31 ? INFINITY : (e == 0 ? std::ldexp((double)m, -24) : std::ldexp((double)(1024 + m), e - 25));
    return (h & 0x8000) ? -v : v;
}

uint16_t mfx_half_round(double v, bool up) {
    _Float16 f = (_Float16)v;  // nearest (or within one step of it): then walk to the directed one
    uint16_t h;
    std::memcpy(&h, &f, 2);
    if ((h & 0x7C00) == 0x7C00 && (h & 0x3FF)) h = 0x7C00;  // NaN in: treated as +inf
    int k = half_index(h);
    if (up) {
        while (k < kHalfMax && mfx_half_value(half_bits_at(k)) < v) ++k;
        while (k > 0 && mfx_half_value(half_bits_at(k - 1)) >= v) --k;
    } else {
        while (k > 0 && mfx_half_value(half_bits_at(k)) > v) --k;
        while (k < kHalfMax && mfx_half_value(half_bits_at(k + 1)) <= v) ++k;
    }
    return half_bits_at(k);
}

namespace {
struct Ent {
    float lo[3], hi[3];
    int32_t code;  // >= 0: BVH4 node; < 0: leaf code
};
double area(const Ent& e) {
    const double x = std::max(0.0, (double)e.hi[0] - e.lo[0]), y = std::max(0.0, (double)e.hi[1] - e.lo[1]),
                 z = std::max(0.0, (double)e.hi[2] - e.lo[2]);
    return x * y + y * z + z * x;
}
void kids(const MfxNode& n, std::vector<Ent>& out) {
    for (int k = 0; k < 4; ++k) {
        if (n.child[k] == MFX_CHILD_EMPTY) continue;
        out.push_back(Ent{{n.lox[k], n.loy[k], n.loz[k]}, {n.hix[k], n.hiy[k], n.hiz[k]}, n.child[k]});
    }
}
int nkids(const MfxNode& n) {
    int c = 0;
    for (int k = 0; k < 4; ++k) c += n.child[k] != MFX_CHILD_EMPTY;
    return c;
}
// (v - c) * s rounded outward to FP16; the double difference of two floats is exact unless their
// exponents are far apart, and then one more step outward keeps the bound
uint16_t plane(float v, double c, double s, bool up) {
    const double d = (double)v - c;
    uint16_t h = mfx_half_round(d * s, up);
    if (d + c != (double)v || (double)v - d != c) {
        int k = half_index(h);
        k = up ? std::min(kHalfMax, k + 1) : std::max(0, k - 1);
        h = half_bits_at(k);
    }
    return h;
}
}  // namespace

bool mfx_build_wide(const std::vector<MfxNode>& n4, MfxWideImage& out, std::string& err) {
    out = MfxWideImage{};
    const int N4 = (int)n4.size();
    if (N4 == 0) {
        err = "empty BVH4 image";
        return false;
    }
    // ---- collapse, wide nodes in breadth-first order ----
    std::vector<int> root4{0};                 // the BVH4 node each wide node starts from
    std::vector<std::vector<Ent>> ents;
    std::vector<int> wid_of(N4, -1);
    wid_of[0] = 0;
    for (size_t h = 0; h < root4.size(); ++h) {
        std::vector<Ent> e;
        kids(n4[root4[h]], e);
        while (true) {
            int best = -1;
            double ba = -1.0;
            for (int i = 0; i < (int)e.size(); ++i) {
                if (e[i].code < 0) continue;
                if (e[i].code >= N4) {
                    err = "BVH4 child index out of range";
                    return false;
                }
                if ((int)e.size() - 1 + nkids(n4[e[i].code]) > 8) continue;
                const double a = area(e[i]);
                if (a > ba) {
                    ba = a;
                    best = i;
                }
            }
            if (best < 0) break;
            const int x = e[best].code;
            e.erase(e.begin() + best);
            kids(n4[x], e);
        }
        for (const Ent& x : e) {
            if (x.code < 0) continue;
            if (wid_of[x.code] >= 0) {
                err = "BVH4 image is not a tree";
                return false;
            }
            wid_of[x.code] = (int)root4.size();
            root4.push_back(x.code);
        }
        ents.push_back(std::move(e));
    }
    const int W = (int)root4.size();
    // ---- numbering: the first MFX_TOP_NODES breadth-first (the LDS prefix), the rest in preorder ----
    std::vector<int> nid(W, -1);
    const int T = std::min(W, MFX_TOP_NODES);
    for (int w = 0; w < T; ++w) nid[w] = w;
    int next = T;
    std::vector<int> st{0};
    while (!st.empty()) {
        const int w = st.back();
        st.pop_back();
        if (nid[w] < 0) nid[w] = next++;
        for (int i = (int)ents[w].size() - 1; i >= 0; --i)
            if (ents[w][i].code >= 0) st.push_back(wid_of[ents[w][i].code]);
    }
    // ---- stack bound and depth (children follow their parent in breadth-first order) ----
    std::vector<int> bound(W, 0), depth(W, 1);
    for (int w = W - 1; w >= 0; --w) {
        int b = 0, d = 0;
        for (const Ent& x : ents[w])
            if (x.code >= 0) {
                b = std::max(b, bound[wid_of[x.code]]);
                d = std::max(d, depth[wid_of[x.code]]);
            }
        bound[w] = std::max(0, (int)ents[w].size() - 1) + b;
        depth[w] = 1 + d;
    }
    out.stack_entries = std::max(1, bound[0]);
    out.depth = depth[0];
    // ---- frame: centre of the root's box, a power-of-2 scale that puts every plane within 2^15 ----
    double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
    for (const Ent& x : ents[0])
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], (double)x.lo[a]);
            hi[a] = std::max(hi[a], (double)x.hi[a]);
        }
    double c[3] = {0, 0, 0};
    if (!ents[0].empty())
        for (int a = 0; a < 3; ++a) c[a] = (double)(float)(0.5 * lo[a] + 0.5 * hi[a]);
    double maxabs = 0.0;
    for (const auto& e : ents)
        for (const Ent& x : e)
            for (int a = 0; a < 3; ++a)
                maxabs = std::max({maxabs, std::fabs((double)x.lo[a] - c[a]), std::fabs((double)x.hi[a] - c[a])});
    double s = 1.0;
    if (maxabs > 0.0 && std::isfinite(maxabs)) {
        int ex;
        (void)std::frexp(maxabs, &ex);  // maxabs < 2^ex
        s = std::ldexp(1.0, std::max(-60, std::min(60, 15 - ex)));
    }
    out.xf = MfxWideXf{c[0], c[1], c[2], s};
    // ---- encode ----
    out.nodes.resize(W);
    for (int w = 0; w < W; ++w) {
        MfxNode8H& o = out.nodes[nid[w]];
        for (int k = 0; k < 8; ++k) {
            if (k >= (int)ents[w].size()) {
                o.lox[k] = o.hix[k] = o.loy[k] = o.hiy[k] = o.loz[k] = o.hiz[k] = 0x7C00;  // +inf: never entered
                o.child[k] = MFX_CHILD_EMPTY;
                continue;
            }
            const Ent& x = ents[w][k];
            o.lox[k] = plane(x.lo[0], c[0], s, false);
            o.hix[k] = plane(x.hi[0], c[0], s, true);
            o.loy[k] = plane(x.lo[1], c[1], s, false);
            o.hiy[k] = plane(x.hi[1], c[1], s, true);
            o.loz[k] = plane(x.lo[2], c[2], s, false);
            o.hiz[k] = plane(x.hi[2], c[2], s, true);
            o.child[k] = x.code >= 0 ? nid[wid_of[x.code]] : x.code;
        }
    }
    return true;
}

// Every BVH4 leaf is reached exactly once, and each wide entry's box (back in the world frame)
// contains the BVH4 boxes of every leaf under it: the BVH8 search finds whatever the BVH4 search
// would (mfx_wide_info, tests/test_wide.py).
bool mfx_check_wide(const std::vector<MfxNode>& n4, const MfxWideImage& w, std::string& err, double* mean_entries,
                    int64_t* nleaves) {
    struct LB {
        float lo[3], hi[3];
        int seen;
    };
    std::vector<std::pair<int32_t, LB>> leaves;
    for (const MfxNode& n : n4)
        for (int k = 0; k < 4; ++k)
            if (n.child[k] < 0 && n.child[k] != MFX_CHILD_EMPTY)
                leaves.push_back({n.child[k], LB{{n.lox[k], n.loy[k], n.loz[k]}, {n.hix[k], n.hiy[k], n.hiz[k]}, 0}});
    std::sort(leaves.begin(), leaves.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (size_t i = 1; i < leaves.size(); ++i)
        if (leaves[i].first == leaves[i - 1].first) {
            err = "BVH4 leaf code twice";
            return false;
        }
    const int W = (int)w.nodes.size();
    const long double c[3] = {w.xf.cx, w.xf.cy, w.xf.cz};
    const long double s = w.xf.s;
    int64_t entries = 0;
    std::vector<int> state(W, 0);
    // post-order: a node's box union over its leaves
    std::function<bool(int, long double*, long double*)> visit = [&](int v, long double* lo, long double* hi) -> bool {
        if (v < 0 || v >= W || state[v]) {
            err = v < 0 || v >= W ? "wide child out of range" : "wide image is not a tree";
            return false;
        }
        state[v] = 1;
        const MfxNode8H& n = w.nodes[v];
        const uint16_t* L[3] = {n.lox, n.loy, n.loz};
        const uint16_t* H[3] = {n.hix, n.hiy, n.hiz};
        for (int a = 0; a < 3; ++a) {
            lo[a] = INFINITY;
            hi[a] = -INFINITY;
        }
        for (int k = 0; k < 8; ++k) {
            if (n.child[k] == MFX_CHILD_EMPTY) continue;
            ++entries;
            long double el[3], eh[3];
            if (n.child[k] >= 0) {
                if (!visit(n.child[k], el, eh)) return false;
            } else {
                auto it = std::lower_bound(leaves.begin(), leaves.end(), n.child[k],
                                           [](const auto& a, int32_t code) { return a.first < code; });
                if (it == leaves.end() || it->first != n.child[k] || it->second.seen) {
                    err = "wide leaf not a BVH4 leaf, or reached twice";
                    return false;
                }
                it->second.seen = 1;
                for (int a = 0; a < 3; ++a) {
                    el[a] = it->second.lo[a];
                    eh[a] = it->second.hi[a];
                }
            }
            for (int a = 0; a < 3; ++a) {
                if (!((long double)mfx_half_value(L[a][k]) <= (el[a] - c[a]) * s) ||
                    !((long double)mfx_half_value(H[a][k]) >= (eh[a] - c[a]) * s)) {
                    err = "wide box does not contain its subtree";
                    return false;
                }
                lo[a] = std::min(lo[a], el[a]);
                hi[a] = std::max(hi[a], eh[a]);
            }
        }
        return true;
    };
    long double lo[3], hi[3];
    if (!visit(0, lo, hi)) return false;
    for (const auto& l : leaves)
        if (!l.second.seen) {
            err = "BVH4 leaf not reached by the wide image";
            return false;
        }
    if (mean_entries) *mean_entries = W ? (double)entries / W : 0.0;
    if (nleaves) *nleaves = (int64_t)leaves.size();
    return true;
}
