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

constexpr int kBins = 32;
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

}  // namespace

namespace rtw {

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
