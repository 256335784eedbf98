// rtw_sah.cpp -- the render kernel's own search tree over the world's leaves (host, upload time).
//
// The reference's BVH (hittable.rs:382-427) splits at the median of box minima on a cycling
// axis; a huge leaf (final_scene1's ground sphere) then sits in a chain of huge boxes that every
// ray enters.  The kernel answers "which leaf is closest" on a surface-area-heuristic tree built
// here, visited with the proximity cull alone (conservative: never skips a leaf whose test would
// accept a root in [ts, te)), and proves the answer is the reference's with one slab test on the
// found leaf's own box.  The tree's shape affects speed only.
#include <algorithm>
#include <cmath>
#include <vector>

#include "rtw_common.h"

namespace {

struct Item {
    float lo[3], hi[3];
    float c[3];  // box centre (split key)
    int32_t id;  // leaf, encoded -1 - index
};

#ifndef RTW_OBJ_BINS
// the object-split builder's bins: 128 against 32 gives final_scene1 16.55 node tests per random line
// instead of 16.63 and +0.7 % on its frame (profiles/r05/ab_obj_bins.txt)
#define RTW_OBJ_BINS 128
#endif
constexpr int kBins = RTW_OBJ_BINS;
#ifndef RTW_SPLIT_BINS
#define RTW_SPLIT_BINS 64
#endif
// the spatial-split builder's bins (object and spatial passes): 64 against 32 gives suzanne's budget-1
// tree 1770 nodes instead of 1809 and 71.3 / 37.4 node / leaf tests per random line instead of 72.1 /
// 37.6 (48, 80, 96, 128: between), +0.9 % on its frame (profiles/r05/ab_split_bins.txt)
constexpr int kSBins = RTW_SPLIT_BINS;
constexpr int kSahDepth = 24;  // deeper subtrees split at the median (bounded stack)

double half_area(const float lo[3], const float hi[3]) {
    const double dx = std::max(0.0, (double)hi[0] - lo[0]), dy = std::max(0.0, (double)hi[1] - lo[1]),
                 dz = std::max(0.0, (double)hi[2] - lo[2]);
    return dx * dy + dy * dz + dz * dx;
}

struct Box {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const float l[3], const float h[3]) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], l[k]);
            hi[k] = std::max(hi[k], h[k]);
        }
    }
};

int32_t build(Item* it, size_t n, std::vector<rtw_bvh_node>& nodes, int depth, int* max_depth) {
    if (depth > *max_depth) *max_depth = depth;
    if (n == 1) return it[0].id;
    Box box, cb;
    for (size_t i = 0; i < n; ++i) {
        box.grow(it[i].lo, it[i].hi);
        cb.grow(it[i].c, it[i].c);
    }
    int axis = -1;
    size_t mid = n / 2;
    if (depth < kSahDepth) {
        // binned SAH over the box centres, every axis; cost = A_l N_l + A_r N_r
        double best = INFINITY;
        int best_bin = -1;
        for (int k = 0; k < 3; ++k) {
            const double ext = (double)cb.hi[k] - cb.lo[k];
            if (!(ext > 0.0)) continue;
            Box bins[kBins];
            size_t cnt[kBins] = {};
            auto bin_of = [&](const Item& x) {
                const int b = (int)(((double)x.c[k] - cb.lo[k]) / ext * kBins);
                return std::min(kBins - 1, std::max(0, b));
            };
            for (size_t i = 0; i < n; ++i) {
                const int b = bin_of(it[i]);
                bins[b].grow(it[i].lo, it[i].hi);
                ++cnt[b];
            }
            double right_cost[kBins] = {};
            Box acc;
            size_t acc_n = 0;
            for (int b = kBins - 1; b >= 1; --b) {
                acc.grow(bins[b].lo, bins[b].hi);
                acc_n += cnt[b];
                right_cost[b] = acc_n ? half_area(acc.lo, acc.hi) * (double)acc_n : 0.0;
            }
            Box lacc;
            size_t l_n = 0;
            for (int b = 0; b < kBins - 1; ++b) {
                lacc.grow(bins[b].lo, bins[b].hi);
                l_n += cnt[b];
                if (l_n == 0 || l_n == n) continue;
                const double cost = half_area(lacc.lo, lacc.hi) * (double)l_n + right_cost[b + 1];
                if (cost < best) {
                    best = cost;
                    axis = k;
                    best_bin = b;
                }
            }
        }
        if (axis >= 0) {
            const double ext = (double)cb.hi[axis] - cb.lo[axis];
            Item* m = std::partition(it, it + n, [&](const Item& x) {
                const int b = std::min(kBins - 1, std::max(0, (int)(((double)x.c[axis] - cb.lo[axis]) / ext * kBins)));
                return b <= best_bin;
            });
            mid = (size_t)(m - it);
        }
    }
    if (axis < 0) {  // median split on the widest centre axis (coincident centres: any halves)
        axis = 0;
        for (int k = 1; k < 3; ++k)
            if ((double)cb.hi[k] - cb.lo[k] > (double)cb.hi[axis] - cb.lo[axis]) axis = k;
        mid = n / 2;
        std::nth_element(it, it + mid, it + n, [axis](const Item& a, const Item& b) { return a.c[axis] < b.c[axis]; });
    }
    const int32_t id = (int32_t)nodes.size();
    nodes.push_back(rtw_bvh_node{});
    const int32_t l = build(it, mid, nodes, depth + 1, max_depth);
    const int32_t r = build(it + mid, n - mid, nodes, depth + 1, max_depth);
    rtw_bvh_node& nd = nodes[(size_t)id];
    for (int k = 0; k < 3; ++k) {
        nd.min[k] = box.lo[k];
        nd.max[k] = box.hi[k];
    }
    nd.axis = axis;  // left = the lower centres: the near side when ray.d[axis] > 0
    nd.left = l;
    nd.right = r;
    return id;
}

// ---------------------------------------------------------------------------------------------
// Spatial splits (Stich, Friedrich & Dietrich 2009, "Spatial splits in bounding volume
// hierarchies"): a node may split space at a plane instead of splitting its references by centre; a
// triangle straddling the plane is then referenced on both sides, each reference with the box of its
// part (the triangle clipped to the side, exactly, in double, rounded outward to f32).  The union of
// a leaf's reference boxes covers the leaf, so a walk with the proximity cull still tests, somewhere,
// every leaf whose test would accept a root; a leaf met twice reports the same t.
// Non-triangle references straddling a plane are clipped as boxes (their box cut by the plane).
// ---------------------------------------------------------------------------------------------
// f32 box outward from a double box: below 2^-60 in magnitude a bound snaps outward to 0 or +-2^-60
// (every SAH box coordinate stays 0 or >= 2^-60, as the upload checks)
void round_out(const double lo[3], const double hi[3], float flo[3], float fhi[3]) {
    const double tiny = 0x1p-60;
    for (int k = 0; k < 3; ++k) {
        double l = lo[k] - std::fabs(lo[k]) * 0x1p-45, h = hi[k] + std::fabs(hi[k]) * 0x1p-45;
        if (std::fabs(l) < tiny) l = l < 0.0 ? -tiny : 0.0;
        if (std::fabs(h) < tiny) h = h > 0.0 ? tiny : 0.0;
        float a = (float)l, b = (float)h;
        if ((double)a > l) a = std::nextafter(a, -INFINITY);
        if ((double)b < h) b = std::nextafter(b, INFINITY);
        flo[k] = a;
        fhi[k] = b;
    }
}

struct Ref {
    double lo[3], hi[3];  // the reference's box (exact clip results; rounded outward at the end)
    int32_t leaf;         // leaf index
};

struct SplitBuilder {
    const float* tri;  // 9 floats per leaf (the triangle's vertices), x = NaN: not a clippable triangle
    const float* lkm;  // per leaf {k, m} proximity-cull constants; k < 0: a leaf that never reports a hit
    int64_t extra;     // references still allowed beyond one per leaf
    std::vector<rtw_bvh_node>* nodes;
    std::vector<float>* km;  // 2 per node: the maxima over the leaves below
    int max_depth = 0;
    int depth_cap = 0;  // > 0: no leaf deeper (children of a node at depth d hold <= 2^(cap - d - 1) references)
    bool bad = false;  // a reference box came out empty or not finite: the caller takes the object-split tree
    struct Out {
        int32_t id;
        float lo[3], hi[3];
        float k, m;
    };

    static double area(const double lo[3], const double hi[3]) {
        const double dx = std::max(0.0, hi[0] - lo[0]), dy = std::max(0.0, hi[1] - lo[1]), dz = std::max(0.0, hi[2] - lo[2]);
        return dx * dy + dy * dz + dz * dx;
    }
    // the box of (the reference's leaf) within [lo, hi] (a sub-box of the reference's box)
    void clip(const Ref& r, const double lo[3], const double hi[3], double olo[3], double ohi[3]) const {
        const float* t = tri ? tri + 9 * (size_t)r.leaf : nullptr;
        if (!t || t[0] != t[0]) {  // a box: cut it
            for (int k = 0; k < 3; ++k) {
                olo[k] = std::max(r.lo[k], lo[k]);
                ohi[k] = std::min(r.hi[k], hi[k]);
            }
            return;
        }
        // Sutherland-Hodgman against the six planes of [lo, hi]
        double poly[2][16][3];
        int n = 3, cur = 0;
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 3; ++k) poly[0][v][k] = t[3 * v + k];
        for (int k = 0; k < 3 && n > 0; ++k)
            for (int side = 0; side < 2 && n > 0; ++side) {
                const double c = side ? hi[k] : lo[k];
                auto inside = [&](const double* p) { return side ? p[k] <= c : p[k] >= c; };
                int m = 0;
                for (int v = 0; v < n; ++v) {
                    const double* p = poly[cur][v];
                    const double* q = poly[cur][(v + 1) % n];
                    const bool pi = inside(p), qi = inside(q);
                    if (pi) {
                        for (int j = 0; j < 3; ++j) poly[cur ^ 1][m][j] = p[j];
                        ++m;
                    }
                    if (pi != qi) {
                        const double f = (c - p[k]) / (q[k] - p[k]);
                        for (int j = 0; j < 3; ++j) poly[cur ^ 1][m][j] = p[j] + f * (q[j] - p[j]);
                        poly[cur ^ 1][m][k] = c;
                        ++m;
                    }
                }
                n = m;
                cur ^= 1;
            }
        for (int k = 0; k < 3; ++k) {
            olo[k] = INFINITY;
            ohi[k] = -INFINITY;
        }
        for (int v = 0; v < n; ++v)
            for (int k = 0; k < 3; ++k) {
                olo[k] = std::min(olo[k], poly[cur][v][k]);
                ohi[k] = std::max(ohi[k], poly[cur][v][k]);
            }
        for (int k = 0; k < 3; ++k) {  // inside the clip box and the reference's box (rounding in the clip)
            olo[k] = std::max(olo[k], std::max(lo[k], r.lo[k]));
            ohi[k] = std::min(ohi[k], std::min(hi[k], r.hi[k]));
        }
        // the clip can lose the whole polygon to rounding (a triangle grazing the cut): an empty box
        // would round out to NaN (INF - INF) and vanish from a node union.  Keep the reference's box
        // cut by [lo, hi] instead (it holds the part of the triangle inside, whatever the rounding)
        bool empty = false;
        for (int k = 0; k < 3; ++k) empty = empty || !(olo[k] <= ohi[k]);
        if (empty)
            for (int k = 0; k < 3; ++k) {
                olo[k] = std::max(r.lo[k], lo[k]);
                ohi[k] = std::min(r.hi[k], hi[k]);
            }
    }

    Out build(std::vector<Ref>& refs, int depth) {
        max_depth = std::max(max_depth, depth);
        const size_t n = refs.size();
        if (n == 1) {
            Out o;
            o.id = -1 - refs[0].leaf;
            round_out(refs[0].lo, refs[0].hi, o.lo, o.hi);
            for (int k = 0; k < 3; ++k)  // every reference box finite and non-empty, or no split tree
                if (!(std::isfinite(o.lo[k]) && std::isfinite(o.hi[k]) && o.lo[k] <= o.hi[k])) bad = true;
            const float k = lkm[2 * (size_t)refs[0].leaf], m = lkm[2 * (size_t)refs[0].leaf + 1];
            o.k = k < 0.0f ? 0.0f : k;  // a leaf that never reports a hit constrains nothing
            o.m = k < 0.0f ? 0.0f : m;
            return o;
        }
        double blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (const Ref& r : refs)
            for (int k = 0; k < 3; ++k) {
                blo[k] = std::min(blo[k], r.lo[k]);
                bhi[k] = std::max(bhi[k], r.hi[k]);
                const double c = 0.5 * (r.lo[k] + r.hi[k]);
                clo[k] = std::min(clo[k], c);
                chi[k] = std::max(chi[k], c);
            }
        // the depth cap: each child of this node holds at most lim references (a median split always
        // does, by induction from the root's n <= 2^cap)
        const size_t lim = depth_cap > 0 && depth_cap - depth - 1 < 62 ? (size_t)1 << std::max(0, depth_cap - depth - 1)
                                                                      : SIZE_MAX;
        // object split: binned SAH over the centres
        double best = INFINITY;
        int axis = -1, best_bin = -1;
        if (depth < kSahDepth)
            for (int k = 0; k < 3; ++k) {
                const double ext = chi[k] - clo[k];
                if (!(ext > 0.0)) continue;
                double bl[kSBins][3], bh[kSBins][3];
                size_t cnt[kSBins] = {};
                for (int b = 0; b < kSBins; ++b)
                    for (int j = 0; j < 3; ++j) bl[b][j] = INFINITY, bh[b][j] = -INFINITY;
                for (const Ref& r : refs) {
                    const int b = std::min(kSBins - 1, std::max(0, (int)((0.5 * (r.lo[k] + r.hi[k]) - clo[k]) / ext * kSBins)));
                    ++cnt[b];
                    for (int j = 0; j < 3; ++j) bl[b][j] = std::min(bl[b][j], r.lo[j]), bh[b][j] = std::max(bh[b][j], r.hi[j]);
                }
                double rc[kSBins] = {}, al[3] = {INFINITY, INFINITY, INFINITY}, ah[3] = {-INFINITY, -INFINITY, -INFINITY};
                size_t rn = 0;
                for (int b = kSBins - 1; b >= 1; --b) {
                    for (int j = 0; j < 3; ++j) al[j] = std::min(al[j], bl[b][j]), ah[j] = std::max(ah[j], bh[b][j]);
                    rn += cnt[b];
                    rc[b] = rn ? area(al, ah) * (double)rn : 0.0;
                }
                double ll[3] = {INFINITY, INFINITY, INFINITY}, lh[3] = {-INFINITY, -INFINITY, -INFINITY};
                size_t ln = 0;
                for (int b = 0; b < kSBins - 1; ++b) {
                    for (int j = 0; j < 3; ++j) ll[j] = std::min(ll[j], bl[b][j]), lh[j] = std::max(lh[j], bh[b][j]);
                    ln += cnt[b];
                    if (ln == 0 || ln == n || ln > lim || n - ln > lim) continue;
                    const double c = area(ll, lh) * (double)ln + rc[b + 1];
                    if (c < best) best = c, axis = k, best_bin = b;
                }
            }
        // spatial split: bins over the node box; a reference counts on every side it reaches
        double sbest = INFINITY, splane = 0.0;
        int saxis = -1;
        if (depth < kSahDepth && extra > 0)
            for (int k = 0; k < 3; ++k) {
                const double ext = bhi[k] - blo[k];
                if (!(ext > 0.0)) continue;
                double bl[kSBins][3], bh[kSBins][3];
                size_t enter[kSBins] = {}, leave[kSBins] = {};
                for (int b = 0; b < kSBins; ++b)
                    for (int j = 0; j < 3; ++j) bl[b][j] = INFINITY, bh[b][j] = -INFINITY;
                auto pos = [&](int b) { return b == kSBins ? bhi[k] : blo[k] + ext * b / kSBins; };
                for (const Ref& r : refs) {
                    const int b0 = std::min(kSBins - 1, std::max(0, (int)((r.lo[k] - blo[k]) / ext * kSBins)));
                    const int b1 = std::min(kSBins - 1, std::max(b0, (int)((r.hi[k] - blo[k]) / ext * kSBins)));
                    ++enter[b0];
                    ++leave[b1];
                    for (int b = b0; b <= b1; ++b) {
                        double lo[3] = {blo[0], blo[1], blo[2]}, hi[3] = {bhi[0], bhi[1], bhi[2]}, ol[3], oh[3];
                        lo[k] = pos(b);
                        hi[k] = pos(b + 1);
                        if (b0 == b1) {
                            for (int j = 0; j < 3; ++j) ol[j] = r.lo[j], oh[j] = r.hi[j];
                        } else {
                            clip(r, lo, hi, ol, oh);
                        }
                        for (int j = 0; j < 3; ++j) bl[b][j] = std::min(bl[b][j], ol[j]), bh[b][j] = std::max(bh[b][j], oh[j]);
                    }
                }
                double rc[kSBins] = {}, al[3] = {INFINITY, INFINITY, INFINITY}, ah[3] = {-INFINITY, -INFINITY, -INFINITY};
                size_t rn = 0;
                for (int b = kSBins - 1; b >= 1; --b) {
                    for (int j = 0; j < 3; ++j) al[j] = std::min(al[j], bl[b][j]), ah[j] = std::max(ah[j], bh[b][j]);
                    rn += leave[b];
                    rc[b] = rn ? area(al, ah) * (double)rn : 0.0;
                }
                double ll[3] = {INFINITY, INFINITY, INFINITY}, lh[3] = {-INFINITY, -INFINITY, -INFINITY};
                size_t ln = 0, rn2 = n;
                for (int b = 0; b < kSBins - 1; ++b) {
                    for (int j = 0; j < 3; ++j) ll[j] = std::min(ll[j], bl[b][j]), lh[j] = std::max(lh[j], bh[b][j]);
                    ln += enter[b];
                    rn2 -= leave[b];
                    if (ln == 0 || rn2 == 0 || ln == n || rn2 == n || (int64_t)(ln + rn2 - n) > extra || ln > lim || rn2 > lim)
                        continue;
                    const double c = area(ll, lh) * (double)ln + rc[b + 1];
                    if (c < sbest) sbest = c, saxis = k, splane = pos(b + 1);
                }
            }
        std::vector<Ref> left, right;
        if (saxis >= 0 && sbest < best) {
            for (const Ref& r : refs) {
                if (r.hi[saxis] <= splane) {
                    left.push_back(r);
                } else if (r.lo[saxis] >= splane) {
                    right.push_back(r);
                } else {
                    Ref a = r, b = r;
                    double lo[3] = {r.lo[0], r.lo[1], r.lo[2]}, hi[3] = {r.hi[0], r.hi[1], r.hi[2]};
                    hi[saxis] = splane;
                    clip(r, lo, hi, a.lo, a.hi);
                    lo[saxis] = splane;
                    hi[saxis] = r.hi[saxis];
                    clip(r, lo, hi, b.lo, b.hi);
                    left.push_back(a);
                    right.push_back(b);
                }
            }
            if (left.empty() || right.empty() || left.size() == n || right.size() == n ||
                (int64_t)(left.size() + right.size() - n) > extra || left.size() > lim || right.size() > lim) {
                left.clear();
                right.clear();
            } else {
                extra -= (int64_t)(left.size() + right.size() - n);
                axis = saxis;
            }
        }
        if (left.empty()) {
            if (axis >= 0 && best_bin >= 0) {
                const double ext = chi[axis] - clo[axis];
                for (const Ref& r : refs) {
                    const int b = std::min(kSBins - 1, std::max(0, (int)((0.5 * (r.lo[axis] + r.hi[axis]) - clo[axis]) / ext * kSBins)));
                    (b <= best_bin ? left : right).push_back(r);
                }
            }
            if (left.empty() || right.empty() || left.size() > lim || right.size() > lim) {  // median split on the widest centre axis
                left.clear();
                right.clear();
                axis = 0;
                for (int k = 1; k < 3; ++k)
                    if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
                std::vector<Ref> v = refs;
                const size_t mid = n / 2;
                std::nth_element(v.begin(), v.begin() + (long)mid, v.end(), [axis](const Ref& a, const Ref& b) {
                    return a.lo[axis] + a.hi[axis] < b.lo[axis] + b.hi[axis];
                });
                left.assign(v.begin(), v.begin() + (long)mid);
                right.assign(v.begin() + (long)mid, v.end());
            }
        }
        refs.clear();
        refs.shrink_to_fit();
        const int32_t id = (int32_t)nodes->size();
        nodes->push_back(rtw_bvh_node{});
        km->push_back(0.0f);
        km->push_back(0.0f);
        const Out l = build(left, depth + 1);
        const Out r = build(right, depth + 1);
        Out o;
        o.id = id;
        rtw_bvh_node& nd = (*nodes)[(size_t)id];
        for (int k = 0; k < 3; ++k) {
            o.lo[k] = nd.min[k] = std::min(l.lo[k], r.lo[k]);
            o.hi[k] = nd.max[k] = std::max(l.hi[k], r.hi[k]);
        }
        o.k = std::max(l.k, r.k);
        o.m = std::max(l.m, r.m);
        (*km)[2 * (size_t)id] = o.k;
        (*km)[2 * (size_t)id + 1] = o.m;
        nd.axis = axis;  // left = the lower side: the near side when ray.d[axis] > 0
        nd.left = l.id;
        nd.right = r.id;
        return o;
    }
};

}  // namespace

namespace rtw {

int sah_build_split(const float* lo, const float* hi, const float* tri, const float* leaf_km, int32_t n, double budget,
                    std::vector<rtw_bvh_node>& nodes, std::vector<float>& km, int32_t* root, int* depth, int depth_cap) {
    nodes.clear();
    km.clear();
    if (n <= 1) return -1;
    std::vector<Ref> refs((size_t)n);
    for (int32_t i = 0; i < n; ++i) {
        for (int k = 0; k < 3; ++k) {
            refs[(size_t)i].lo[k] = lo[3 * (size_t)i + k];
            refs[(size_t)i].hi[k] = hi[3 * (size_t)i + k];
        }
        refs[(size_t)i].leaf = i;
    }
    SplitBuilder B;
    B.tri = tri;
    B.lkm = leaf_km;
    B.extra = (int64_t)(budget * n);
    // a cap the root's references cannot meet is no cap (median splits need n <= 2^cap)
    B.depth_cap = depth_cap > 0 && depth_cap < 62 && (int64_t)n <= ((int64_t)1 << depth_cap) ? depth_cap : 0;
    B.nodes = &nodes;
    B.km = &km;
    nodes.reserve((size_t)n + (size_t)B.extra);
    *root = B.build(refs, 0).id;
    *depth = B.max_depth;
    return B.bad ? -1 : 0;
}

int sah_build(const float* lo, const float* hi, int32_t n, std::vector<rtw_bvh_node>& nodes, int32_t* root,
              int* depth) {
    nodes.clear();
    if (n <= 0) return -1;
    std::vector<Item> items((size_t)n);
    for (int32_t i = 0; i < n; ++i) {
        Item& x = items[(size_t)i];
        for (int k = 0; k < 3; ++k) {
            x.lo[k] = lo[3 * (size_t)i + k];
            x.hi[k] = hi[3 * (size_t)i + k];
            x.c[k] = (float)(0.5 * ((double)x.lo[k] + (double)x.hi[k]));
        }
        x.id = -1 - i;
    }
    nodes.reserve((size_t)n);
    int d = 0;
    *root = build(items.data(), items.size(), nodes, 0, &d);
    *depth = d;  // nodes on the longest root-to-leaf path
    return 0;
}

}  // namespace rtw
