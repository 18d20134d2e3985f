// bvh_builder.cpp — binned SAH BVH2 over world-space triangles (host, C++ threads).
#include "bvh_builder.h"

#include "../../include/ark_ddgi_debug.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <thread>

namespace ark {
namespace {

struct Aabb {
    float lo[3] = { INFINITY, INFINITY, INFINITY };
    float hi[3] = { -INFINITY, -INFINITY, -INFINITY };
    void grow(const float p[3])
    {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], p[a]);
            hi[a] = std::max(hi[a], p[a]);
        }
    }
    void grow(const Aabb& b)
    {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], b.lo[a]);
            hi[a] = std::max(hi[a], b.hi[a]);
        }
    }
    float area() const
    {
        float d0 = hi[0] - lo[0], d1 = hi[1] - lo[1], d2 = hi[2] - lo[2];
        if (!(d0 >= 0.0f)) return 0.0f;
        return 2.0f * (d0 * d1 + d1 * d2 + d2 * d0);
    }
    // SAH surface with per-face weights w = {xy, yz, zx} (BvhBuildOptions::area_w):
    // {1, 1, 1} is the surface area; rays parallel to z (the light-space BVH of the
    // sun's shadow rays) cross a box with a probability proportional to its xy face
    float area(const float* w) const
    {
        float d0 = hi[0] - lo[0], d1 = hi[1] - lo[1], d2 = hi[2] - lo[2];
        if (!(d0 >= 0.0f)) return 0.0f;
        return 2.0f * (w[0] * d0 * d1 + w[1] * d1 * d2 + w[2] * d2 * d0);
    }
};

struct Ref {
    Aabb box;
    float c[3];
    uint32_t tri; // the BuildTriangle this reference stands for
};

// --- early split clipping (BvhBuildOptions::presplit_levels) -----------------------
struct Poly {
    double p[9][3]; // a triangle clipped by up to 6 planes has at most 9 vertices
    int n = 0;
};

// The part of `in` on one side of the plane x[axis] = at (keepLow: <=), exactly in
// double but for the interpolated crossing points.
Poly clipPoly(const Poly& in, int axis, double at, bool keepLow)
{
    Poly out;
    for (int i = 0; i < in.n; ++i) {
        const double* a = in.p[i];
        const double* b = in.p[(i + 1) % in.n];
        const double da = keepLow ? at - a[axis] : a[axis] - at, db = keepLow ? at - b[axis] : b[axis] - at;
        if (da >= 0.0 && out.n < 9) std::memcpy(out.p[out.n++], a, sizeof(double) * 3);
        if ((da >= 0.0) != (db >= 0.0) && out.n < 9) {
            const double t = da / (da - db);
            for (int k = 0; k < 3; ++k) out.p[out.n][k] = a[k] + (b[k] - a[k]) * t;
            out.p[out.n][axis] = at; // on the plane
            out.n++;
        }
    }
    return out;
}

// float bounds of a double polygon, rounded outward (plus a relative hair for the
// crossing points' interpolation error), so the box contains the exact piece
Aabb polyBox(const Poly& P)
{
    Aabb b;
    for (int i = 0; i < P.n; ++i)
        for (int a = 0; a < 3; ++a) {
            const double v = P.p[i][a], e = std::fabs(v) * 1e-12 + 1e-30;
            b.lo[a] = std::min(b.lo[a], std::nextafter(static_cast<float>(v - e), -INFINITY));
            b.hi[a] = std::max(b.hi[a], std::nextafter(static_cast<float>(v + e), INFINITY));
        }
    return b;
}

void splitRefs(const Poly& P, const Aabb& box, uint32_t tri, int level, double stopArea, std::vector<Ref>& out)
{
    const float e0 = box.hi[0] - box.lo[0], e1 = box.hi[1] - box.lo[1], e2 = box.hi[2] - box.lo[2];
    if (level == 0 || box.area() <= stopArea) {
        Ref r;
        r.box = box;
        for (int a = 0; a < 3; ++a) r.c[a] = 0.5f * (box.lo[a] + box.hi[a]);
        r.tri = tri;
        out.push_back(r);
        return;
    }
    const int axis = (e0 >= e1 && e0 >= e2) ? 0 : (e1 >= e2 ? 1 : 2);
    const double at = 0.5 * (static_cast<double>(box.lo[axis]) + static_cast<double>(box.hi[axis]));
    for (int side = 0; side < 2; ++side) {
        const Poly Q = clipPoly(P, axis, at, side == 0);
        if (Q.n < 3) continue;
        Aabb qb = polyBox(Q);
        for (int a = 0; a < 3; ++a) { // never outside the parent's (already conservative) box
            qb.lo[a] = std::max(qb.lo[a], box.lo[a]);
            qb.hi[a] = std::min(qb.hi[a], box.hi[a]);
        }
        splitRefs(Q, qb, tri, level - 1, stopArea, out);
    }
}

struct Range {
    int32_t code; // >= 0 node index, < 0 leaf code
    Aabb box;
};

// f(begin, end) over [0, n) in `threads` contiguous chunks (one when n is small)
template<class F>
void parallelFor(size_t n, int threads, F f)
{
    const int T = std::max(1, std::min<int>(threads, static_cast<int>(n >> 16) + 1));
    std::vector<std::thread> pool;
    for (int t = 1; t < T; ++t) pool.emplace_back([&, t] { f(n * t / T, n * (t + 1) / T); });
    f(0, n / T);
    for (std::thread& th : pool) th.join();
}

class Builder {
public:
    Builder(const std::vector<BuildTriangle>& tris, const BvhBuildOptions& opt, uint32_t nodeBase, uint32_t triBase)
        : m_opt(opt), m_nodeBase(nodeBase), m_triBase(triBase)
    {
        const size_t nt = tris.size();
        const int hw = opt.threads > 0 ? opt.threads : static_cast<int>(std::thread::hardware_concurrency());
        m_refs.resize(nt);
        parallelFor(nt, hw, [&](size_t b, size_t e) {
            for (size_t i = b; i < e; ++i) {
                Ref& r = m_refs[i];
                r.box.grow(tris[i].v0);
                r.box.grow(tris[i].v1);
                r.box.grow(tris[i].v2);
                for (int a = 0; a < 3; ++a) r.c[a] = 0.5f * (r.box.lo[a] + r.box.hi[a]);
                r.tri = static_cast<uint32_t>(i);
            }
        });
        if (opt.presplit_levels > 0) {
            std::vector<Ref> refs;
            refs.reserve(nt + nt / 2);
            for (size_t i = 0; i < nt; ++i) {
                const BuildTriangle& t = tris[i];
                double e1[3], e2[3];
                for (int a = 0; a < 3; ++a) {
                    e1[a] = static_cast<double>(t.v1[a]) - t.v0[a];
                    e2[a] = static_cast<double>(t.v2[a]) - t.v0[a];
                }
                const double cx = e1[1] * e2[2] - e1[2] * e2[1], cy = e1[2] * e2[0] - e1[0] * e2[2], cz = e1[0] * e2[1] - e1[1] * e2[0];
                const double area2 = std::sqrt(cx * cx + cy * cy + cz * cz); // twice the area
                const double stop = opt.presplit_ratio * area2;
                if (!(m_refs[i].box.area() > stop)) {
                    refs.push_back(m_refs[i]);
                    continue;
                }
                Poly P;
                P.n = 3;
                for (int a = 0; a < 3; ++a) {
                    P.p[0][a] = t.v0[a];
                    P.p[1][a] = t.v1[a];
                    P.p[2][a] = t.v2[a];
                }
                const size_t before = refs.size();
                splitRefs(P, m_refs[i].box, static_cast<uint32_t>(i), opt.presplit_levels, stop, refs);
                if (refs.size() == before) refs.push_back(m_refs[i]); // degenerate clip: keep the whole
            }
            m_refs.swap(refs);
        }
        const size_t n = m_refs.size();
        // a binary tree over n leaves has at most n - 1 internal nodes (+ node 0's slot);
        // written before read, so not zero-filled (1.3 GB at C4)
        m_nodes.reset(new GpuBvhNode[n + 1]);
        m_threads = std::max(1, hw);
        m_threadsAvail = std::max(0, hw - 1);
    }

    BvhBuildResult run(const std::vector<BuildTriangle>& tris)
    {
        BvhBuildResult res;
        const uint32_t n = static_cast<uint32_t>(m_refs.size());
        m_nodeCount = 1; // node 0 = root
        Bin all = binRange(0, n, nullptr, nullptr);
        Range root = buildRange(0, n, 1, all.b, all.c, 0);
        if (root.code < 0) {
            // whole set fits one leaf: root with the leaf + an unreachable far child
            Aabb far;
            const float p[3] = { 1e30f, 1e30f, 1e30f };
            far.grow(p);
            writeNode(0, root.box, root.code, far, ~0);
        }
        res.nodes.assign(m_nodes.get(), m_nodes.get() + m_nodeCount.load());
        m_nodes.reset();
        res.tris.resize(n);
        parallelFor(n, m_threads, [&](size_t b, size_t e) {
            for (size_t i = b; i < e; ++i) res.tris[i] = make_gpu_triangle(tris[m_refs[i].tri]);
        });
        res.max_depth = m_maxDepth.load();
        res.max_leaf = m_maxLeaf.load();
        res.sah_cost = sahCost(res.nodes, root.box);
        return res;
    }

private:
    float sahCost(const std::vector<GpuBvhNode>& nodes, const Aabb& rootBox) const
    {
        const float ra = rootBox.area();
        if (!(ra > 0.0f)) return 0.0f;
        double cost = 0.0;
        for (const GpuBvhNode& nd : nodes) {
            Aabb b[2];
            b[0].lo[0] = nd.n0[0]; b[0].hi[0] = nd.n0[1]; b[0].lo[1] = nd.n0[2]; b[0].hi[1] = nd.n0[3];
            b[1].lo[0] = nd.n1[0]; b[1].hi[0] = nd.n1[1]; b[1].lo[1] = nd.n1[2]; b[1].hi[1] = nd.n1[3];
            b[0].lo[2] = nd.n2[0]; b[0].hi[2] = nd.n2[1]; b[1].lo[2] = nd.n2[2]; b[1].hi[2] = nd.n2[3];
            for (int c = 0; c < 2; ++c) {
                if (b[c].lo[0] > 1e29f) continue;
                double a = b[c].area() / ra;
                if (nd.child[c] >= 0) cost += m_opt.traversal_cost * a;
                else cost += m_opt.intersection_cost * a * ((static_cast<uint32_t>(~nd.child[c]) & (kMaxLeafSize - 1)) + 1);
            }
        }
        return static_cast<float>(cost + m_opt.traversal_cost);
    }

    void writeNode(uint32_t local, const Aabb& b0, int32_t c0, const Aabb& b1, int32_t c1)
    {
        GpuBvhNode& nd = m_nodes[local];
        Aabb bb[2] = { b0, b1 };
        for (int c = 0; c < 2; ++c) {
            Aabb& b = bb[c];
            if (b.lo[0] > 1e29f) continue; // far sentinel stays exact
            float m = 0.0f, e = 0.0f;
            for (int a = 0; a < 3; ++a) {
                m = std::max(m, std::max(std::fabs(b.lo[a]), std::fabs(b.hi[a])));
                e = std::max(e, b.hi[a] - b.lo[a]);
            }
            const float eps = m * 2e-6f + e * 1e-5f + 1e-7f + m_opt.inflate_abs;
            for (int a = 0; a < 3; ++a) {
                b.lo[a] -= eps;
                b.hi[a] += eps;
            }
        }
        nd.n0[0] = bb[0].lo[0]; nd.n0[1] = bb[0].hi[0]; nd.n0[2] = bb[0].lo[1]; nd.n0[3] = bb[0].hi[1];
        nd.n1[0] = bb[1].lo[0]; nd.n1[1] = bb[1].hi[0]; nd.n1[2] = bb[1].lo[1]; nd.n1[3] = bb[1].hi[1];
        nd.n2[0] = bb[0].lo[2]; nd.n2[1] = bb[0].hi[2]; nd.n2[2] = bb[1].lo[2]; nd.n2[3] = bb[1].hi[2];
        nd.child[0] = c0;
        nd.child[1] = c1;
        nd.child[2] = 0;
        nd.child[3] = 0;
    }

    int32_t leafCode(uint32_t first, uint32_t count) const
    {
        uint32_t v = ((m_triBase + first) << kLeafCountBits) | (count - 1u);
        return ~static_cast<int32_t>(v);
    }

    // Bounds of a run of references (box of their boxes, box of their centroids) and
    // their count; with scale != null also their binning along all three axes at once
    // (bins[a][k]: the references whose centroid falls in bin k of axis a of `cbox`).
    // The references are the builder's own array, partitioned in place level by level,
    // so every pass reads them sequentially.
    struct Bin {
        Aabb b, c;
        uint32_t n = 0;
        void add(const Ref& r)
        {
            b.grow(r.box);
            c.grow(r.c);
            ++n;
        }
        void add(const Bin& o)
        {
            b.grow(o.b);
            c.grow(o.c);
            n += o.n;
        }
    };
    static constexpr int kMaxBins = 64;
    struct Bins {
        Bin k[3][kMaxBins];
    };

    Bin binRange(uint32_t first, uint32_t count, const Aabb* cbox, Bins* bins) const
    {
        const int B = std::max(4, std::min(m_opt.bins, kMaxBins));
        float lo[3] = { 0, 0, 0 }, scale[3] = { 0, 0, 0 };
        bool axis[3] = { false, false, false };
        if (bins)
            for (int a = 0; a < 3; ++a) {
                const float ext = cbox->hi[a] - cbox->lo[a];
                axis[a] = ext > 0.0f;
                lo[a] = cbox->lo[a];
                scale[a] = axis[a] ? static_cast<float>(B) / ext : 0.0f;
            }
        auto work = [&](uint32_t b, uint32_t e, Bin& all, Bins* out) {
            for (uint32_t i = b; i < e; ++i) {
                const Ref& r = m_refs[i];
                all.add(r);
                if (out)
                    for (int a = 0; a < 3; ++a)
                        if (axis[a]) out->k[a][std::min(B - 1, std::max(0, static_cast<int>((r.c[a] - lo[a]) * scale[a])))].add(r);
            }
        };
        Bin all;
        // the top levels in parallel: per-thread partial bins, merged (unions and counts
        // do not depend on the order)
        const int T = count >= (1u << 20) ? std::min(m_threads, static_cast<int>(count >> 18)) : 1;
        if (T <= 1) {
            work(first, first + count, all, bins);
            return all;
        }
        std::vector<Bin> part(T);
        std::vector<Bins> partBins(bins ? T : 0);
        std::vector<std::thread> pool;
        for (int t = 0; t < T; ++t) {
            const uint32_t b = first + static_cast<uint32_t>(static_cast<uint64_t>(count) * t / T);
            const uint32_t e = first + static_cast<uint32_t>(static_cast<uint64_t>(count) * (t + 1) / T);
            pool.emplace_back([&, t, b, e] { work(b, e, part[t], bins ? &partBins[t] : nullptr); });
        }
        for (std::thread& th : pool) th.join();
        for (int t = 0; t < T; ++t) {
            all.add(part[t]);
            if (bins)
                for (int a = 0; a < 3; ++a)
                    for (int k = 0; k < B; ++k) bins->k[a][k].add(partBins[t].k[a][k]);
        }
        return all;
    }

    // box / cbox: the bounds of the range (from the parent's bins)
    Range buildRange(uint32_t first, uint32_t count, int depth, const Aabb& box, const Aabb& cbox, int forcedLocal = -1)
    {
        {
            int md = m_maxDepth.load();
            while (depth > md && !m_maxDepth.compare_exchange_weak(md, depth)) {}
        }
        const int maxLeaf = std::min(m_opt.max_leaf_size, kMaxLeafSize);
        if (count == 1 || (count <= 2 && maxLeaf >= 2)) return makeLeaf(first, count, box);

        // split: binned SAH over 3 axes, object-median fallback near the depth cap
        const int log2n = static_cast<int>(std::ceil(std::log2(std::max(1.0, static_cast<double>(count) / maxLeaf))));
        const bool forceMedian = depth + log2n + 2 >= m_opt.max_depth;
        uint32_t mid = first + count / 2;
        bool split = true, childBounds = false;
        Bin left, right;
        if (!forceMedian) {
            const int B = std::max(4, std::min(m_opt.bins, kMaxBins));
            float bestCost = INFINITY;
            int bestAxis = -1, bestBin = -1;
            if (count <= kSmallCount) {
                // few references: the same SAH sweep over the bins they occupy only (a
                // split between two occupied bins equals the one at the upper bin, which
                // the full sweep - descending, strict < - would keep), without
                // initialising 3 x B bins per node
                bestSmallSplit(first, count, cbox, B, bestCost, bestAxis, bestBin);
            }
            Bins bins;
            if (count > kSmallCount) binRange(first, count, &cbox, &bins);
            for (int a = 0; a < 3 && count > kSmallCount; ++a) {
                const float ext = cbox.hi[a] - cbox.lo[a];
                if (!(ext > 0.0f)) continue;
                const Bin* bb = bins.k[a];
                float leftArea[kMaxBins];
                uint32_t leftCount[kMaxBins];
                Aabb acc;
                uint32_t n = 0;
                for (int k = 0; k < B - 1; ++k) {
                    acc.grow(bb[k].b);
                    n += bb[k].n;
                    leftArea[k] = acc.area(m_opt.area_w);
                    leftCount[k] = n;
                }
                Aabb accR;
                uint32_t nr = 0;
                for (int k = B - 1; k > 0; --k) {
                    accR.grow(bb[k].b);
                    nr += bb[k].n;
                    const uint32_t nl = leftCount[k - 1];
                    if (nl == 0 || nr == 0) continue;
                    const float cost = leftArea[k - 1] * nl + accR.area(m_opt.area_w) * nr;
                    if (cost < bestCost) {
                        bestCost = cost;
                        bestAxis = a;
                        bestBin = k;
                    }
                }
            }
            const float area = box.area(m_opt.area_w);
            const float splitCost = m_opt.traversal_cost + (area > 0.0f ? bestCost / area : 0.0f) * m_opt.intersection_cost;
            const float leafCost = m_opt.intersection_cost * count;
            if (static_cast<int>(count) <= maxLeaf && (bestAxis < 0 || leafCost <= splitCost)) split = false;
            if (split && bestAxis >= 0) {
                const int a = bestAxis;
                const float ext = cbox.hi[a] - cbox.lo[a];
                const float scale = static_cast<float>(B) / ext;
                const float lo = cbox.lo[a];
                auto it = std::partition(m_refs.begin() + first, m_refs.begin() + first + count, [&](const Ref& r) {
                    int k = std::min(B - 1, std::max(0, static_cast<int>((r.c[a] - lo) * scale)));
                    return k < bestBin;
                });
                mid = static_cast<uint32_t>(it - m_refs.begin());
                // the children's bounds are their bins' unions
                if (count > kSmallCount) {
                    for (int k = 0; k < B; ++k) (k < bestBin ? left : right).add(bins.k[a][k]);
                    childBounds = true;
                }
            }
            if (split && (bestAxis < 0 || mid == first || mid == first + count)) {
                medianSplit(first, count, cbox);
                mid = first + count / 2;
                childBounds = false;
            }
        } else {
            if (static_cast<int>(count) <= maxLeaf) split = false;
            else medianSplit(first, count, cbox);
        }
        if (!split) return makeLeaf(first, count, box);

        const uint32_t local = forcedLocal >= 0 ? static_cast<uint32_t>(forcedLocal) : m_nodeCount.fetch_add(1);
        Range l, r;
        const uint32_t nl = mid - first, nr = first + count - mid;
        if (!childBounds) {
            left = binRange(first, nl, nullptr, nullptr);
            right = binRange(mid, nr, nullptr, nullptr);
        }
        bool spawned = false;
        if (count > 65536) {
            int avail = m_threadsAvail.fetch_sub(1);
            if (avail > 0) {
                spawned = true;
                std::thread t([&] { l = buildRange(first, nl, depth + 1, left.b, left.c); });
                r = buildRange(mid, nr, depth + 1, right.b, right.c);
                t.join();
            }
            m_threadsAvail.fetch_add(1);
        }
        if (!spawned) {
            l = buildRange(first, nl, depth + 1, left.b, left.c);
            r = buildRange(mid, nr, depth + 1, right.b, right.c);
        }
        writeNode(local, l.box, l.code, r.box, r.code);
        return Range { static_cast<int32_t>(m_nodeBase + local), box };
    }

    static constexpr uint32_t kSmallCount = 48;
    void bestSmallSplit(uint32_t first, uint32_t count, const Aabb& cbox, int B, float& bestCost, int& bestAxis, int& bestBin) const
    {
        for (int a = 0; a < 3; ++a) {
            const float ext = cbox.hi[a] - cbox.lo[a];
            if (!(ext > 0.0f)) continue;
            const float scale = static_cast<float>(B) / ext;
            int key[kSmallCount];
            uint32_t ord[kSmallCount];
            for (uint32_t i = 0; i < count; ++i) {
                key[i] = std::min(B - 1, std::max(0, static_cast<int>((m_refs[first + i].c[a] - cbox.lo[a]) * scale)));
                ord[i] = i;
            }
            std::sort(ord, ord + count, [&](uint32_t x, uint32_t y) { return key[x] < key[y]; });
            // prefix boxes over the occupied bins in ascending order
            Aabb pre[kSmallCount];
            Aabb acc;
            for (uint32_t j = 0; j < count; ++j) {
                acc.grow(m_refs[first + ord[j]].box);
                pre[j] = acc;
            }
            Aabb accR;
            for (uint32_t j = count; j-- > 0;) {
                accR.grow(m_refs[first + ord[j]].box);
                // a candidate split at k = key of the first reference of a bin run
                if (j == 0 || key[ord[j - 1]] == key[ord[j]]) continue;
                const uint32_t nl = j, nr = count - j;
                const float cost = pre[j - 1].area(m_opt.area_w) * nl + accR.area(m_opt.area_w) * nr;
                if (cost < bestCost) {
                    bestCost = cost;
                    bestAxis = a;
                    bestBin = key[ord[j]];
                }
            }
        }
    }

    void medianSplit(uint32_t first, uint32_t count, const Aabb& cbox)
    {
        int a = 0;
        float e0 = cbox.hi[0] - cbox.lo[0], e1 = cbox.hi[1] - cbox.lo[1], e2 = cbox.hi[2] - cbox.lo[2];
        if (e1 > e0 && e1 >= e2) a = 1;
        else if (e2 > e0 && e2 > e1) a = 2;
        std::nth_element(m_refs.begin() + first, m_refs.begin() + first + count / 2, m_refs.begin() + first + count,
                         [&](const Ref& x, const Ref& y) { return x.c[a] < y.c[a]; });
    }

    Range makeLeaf(uint32_t first, uint32_t count, const Aabb& box)
    {
        // (two split references of one triangle in one leaf stay two records: the
        // collapse merges leaves as contiguous ranges of the leaf order, so a leaf
        // range must not leave a gap)
        uint32_t ml = m_maxLeaf.load();
        while (count > ml && !m_maxLeaf.compare_exchange_weak(ml, count)) {}
        return Range { leafCode(first, count), box };
    }

    const BvhBuildOptions m_opt;
    const uint32_t m_nodeBase, m_triBase;
    std::vector<Ref> m_refs; // partitioned in place: leaf order at the end
    std::unique_ptr<GpuBvhNode[]> m_nodes;
    int m_threads = 1;
    std::atomic<uint32_t> m_nodeCount { 0 };
    std::atomic<int> m_maxDepth { 0 };
    std::atomic<uint32_t> m_maxLeaf { 0 };
    std::atomic<int> m_threadsAvail { 0 };
};

// --- 8-wide collapse -------------------------------------------------------------

struct Child8 {
    int32_t code; // BVH2 child code: >= 0 internal node, < 0 leaf
    Aabb box;
};

void childrenOf(const GpuBvhNode& nd, Child8 out[2], int& n)
{
    n = 0;
    const float lo[2][3] = { { nd.n0[0], nd.n0[2], nd.n2[0] }, { nd.n1[0], nd.n1[2], nd.n2[2] } };
    const float hi[2][3] = { { nd.n0[1], nd.n0[3], nd.n2[1] }, { nd.n1[1], nd.n1[3], nd.n2[3] } };
    for (int c = 0; c < 2; ++c) {
        if (lo[c][0] > 1e29f) continue; // far sentinel of a single-leaf root
        Child8& ch = out[n++];
        ch.code = nd.child[c];
        for (int a = 0; a < 3; ++a) {
            ch.box.lo[a] = lo[c][a];
            ch.box.hi[a] = hi[c][a];
        }
    }
}

// Grid for one axis of a node box [L, H]: step 2^e, anchor p = k * 2^e <= L with
// p + 255 * 2^e >= H and |k| + 256 < 2^24 (every plane p + q * 2^e exact in fp32).
void quantGrid(float L, float H, int& e, double& p)
{
    const double ext = static_cast<double>(H) - static_cast<double>(L);
    e = ext > 0.0 ? static_cast<int>(std::ceil(std::log2(ext / 255.0))) : -100;
    e = std::max(-100, e);
    for (;; ++e) {
        const double step = std::ldexp(1.0, e);
        const double k = std::floor(static_cast<double>(L) / step);
        if (std::fabs(k) + 256.0 >= 16777216.0) continue;
        p = k * step;
        if (p + 255.0 * step < static_cast<double>(H)) continue;
        return;
    }
}

// First-fit placement of a node's leaf-triangle rows (a 24-bit pattern over
// positions base + 0..23) into the triangle array: the lowest base, at most
// kRowWindow below the end of the array, whose positions are all free. The search
// is bounded, so the collapse stays linear; rows of neighbouring nodes interleave.
class RowPlacer {
public:
    uint32_t place(uint32_t pattern)
    {
        constexpr uint32_t back = kRowWindow;
        uint32_t lo = m_end > back ? m_end - back : 0u;
        // every position below m_firstFree is taken, so no base whose lowest pattern
        // position falls below it fits: the same first fit, without re-testing the
        // filled front of the window for every node (C4 collapse 6.5 -> s)
        const uint32_t low = static_cast<uint32_t>(__builtin_ctz(pattern));
        if (m_firstFree > low) lo = std::max(lo, m_firstFree - low);
        for (uint32_t b = lo;; ++b)
            if ((window(b) & pattern) == 0) {
                mark(b, pattern);
                while (taken(m_firstFree)) ++m_firstFree;
                return b;
            }
    }

private:
    static constexpr uint32_t kRowWindow = 512;
    uint64_t window(uint32_t b) const // occupancy of positions b .. b + 23
    {
        const size_t i = b >> 6;
        const uint32_t sh = b & 63u;
        uint64_t w = i < m_bits.size() ? m_bits[i] >> sh : 0u;
        if (sh && i + 1 < m_bits.size()) w |= m_bits[i + 1] << (64u - sh);
        return w & 0xffffffu;
    }
    void mark(uint32_t b, uint32_t pattern)
    {
        const size_t i = b >> 6;
        const uint32_t sh = b & 63u;
        if (m_bits.size() < i + 2) m_bits.resize(i + 2, 0u);
        m_bits[i] |= static_cast<uint64_t>(pattern) << sh;
        if (sh > 40u) m_bits[i + 1] |= static_cast<uint64_t>(pattern) >> (64u - sh);
        m_end = std::max(m_end, b + 32u - static_cast<uint32_t>(__builtin_clz(pattern)));
    }
    bool taken(uint32_t p) const { return (p >> 6) < m_bits.size() && ((m_bits[p >> 6] >> (p & 63u)) & 1u); }
    std::vector<uint64_t> m_bits;
    uint32_t m_end = 0;
    uint32_t m_firstFree = 0; // lowest position not taken
};

// The smallest row stride (GpuBvh8Node) under which every position s + stride * i
// (i < 3) of a leaf slot s is free or s's own triangle i, so a hit leaf slot's
// spread never reaches another slot's triangle, and the rows fit in 24 positions.
uint32_t leafRowStride(const uint32_t cnt[8])
{
    for (uint32_t st = 1u; st < 8; ++st) {
        int owner[24];
        for (int& o : owner) o = -1;
        bool ok = true;
        for (uint32_t s = 0; s < 8 && ok; ++s)
            for (uint32_t i = 0; i < cnt[s] && ok; ++i) {
                const uint32_t p = s + st * i;
                ok = p < 24u && owner[p] < 0;
                if (ok) owner[p] = static_cast<int>(s);
            }
        for (uint32_t s = 0; s < 8 && ok; ++s)
            if (cnt[s])
                for (uint32_t i = 0; i < 3u && ok; ++i) {
                    const uint32_t p = s + st * i;
                    ok = p >= 24u || owner[p] < 0 || owner[p] == static_cast<int>(s);
                }
        if (ok) return st;
    }
    return 8u;
}

} // namespace

GpuTriangle make_gpu_triangle(const BuildTriangle& t)
{
    GpuTriangle g;
    float e1[3], e2[3];
    for (int a = 0; a < 3; ++a) {
        e1[a] = t.v1[a] - t.v0[a];
        e2[a] = t.v2[a] - t.v0[a];
    }
    g.t0[0] = t.v0[0]; g.t0[1] = t.v0[1]; g.t0[2] = t.v0[2]; g.t0[3] = e1[0];
    g.t1[0] = e1[1]; g.t1[1] = e1[2]; g.t1[2] = e2[0]; g.t1[3] = e2[1];
    g.t2[0] = e2[2];
    std::memcpy(&g.t2[1], &t.instance, 4);
    std::memcpy(&g.t2[2], &t.primitive, 4);
    std::memcpy(&g.t2[3], &t.flip_facing, 4);
    return g;
}

GpuTriangle holeTriangle()
{
    GpuTriangle t;
    std::memset(&t, 0, sizeof(t));
    std::memcpy(&t.t2[1], &kHoleInstance, 4);
    return t;
}

bool isHoleTriangle(const GpuTriangle& t)
{
    uint32_t inst;
    std::memcpy(&inst, &t.t2[1], 4);
    return inst == kHoleInstance;
}

int bvh8SlotTriangles(const GpuBvh8Node& nd, int s, uint32_t out[kBvh8MaxLeafSize])
{
    const bool leaf = (nd.leaf_mask >> s) & 1u;
    if (!leaf) return 0;
    if (((nd.imask >> s) & 1u) || nd.tri_stride < 1u || nd.tri_stride > 8u) return -1;
    int n = 0;
    bool ended = false;
    for (uint32_t i = 0; i < static_cast<uint32_t>(kBvh8MaxLeafSize); ++i) {
        const uint32_t pos = static_cast<uint32_t>(s) + nd.tri_stride * i;
        const bool set = pos < 24u && ((nd.leaf_tris >> pos) & 1u);
        if (set && ended) return -1; // the slot's spread reaches another slot's triangle
        if (!set) ended = true;
        else out[n++] = nd.tri_base + pos;
    }
    return n > 0 ? n : -1;
}

float bvh8_inflation(const float* xyz, uint64_t nTriangles)
{
    float lo[3] = { INFINITY, INFINITY, INFINITY }, hi[3] = { -INFINITY, -INFINITY, -INFINITY };
    for (uint64_t i = 0; i < nTriangles * 3; ++i)
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], xyz[3 * i + a]);
            hi[a] = std::max(hi[a], xyz[3 * i + a]);
        }
    return bvh8_inflation_box(lo, hi);
}

float bvh8_inflation_box(const float lo[3], const float hi[3])
{
    double d2 = 0.0;
    for (int a = 0; a < 3; ++a)
        if (hi[a] >= lo[a]) d2 += (static_cast<double>(hi[a]) - lo[a]) * (static_cast<double>(hi[a]) - lo[a]);
    return static_cast<float>(1e-6 * std::sqrt(d2));
}

// SAH-optimal collapse plan (Ylitie, Karras, Laine 2017, "Efficient incoherent ray
// traversal on GPUs through compressed wide BVHs", §3.1). For every BVH2 internal
// node n and i = 1..8: cost[n][i] = the least SAH cost of the subtree below n when it
// is represented by at most i children of a BVH8 node - n itself as one BVH8 node
// (A(n) Cnode + its best 8-way distribution) or one leaf slot (A(n) Ctri T(n), when its
// T(n) <= kBvh8MaxLeafSize triangles, contiguous in leaf order), or its two subtrees
// sharing the i slots. Leaf children of the BVH2 stay leaves (A Ctri count).
struct CollapsePlan {
    std::vector<float> cost;    // [node][8]
    std::vector<uint8_t> pick;  // [node][8]: i = 1: 0 node, 1 leaf; i >= 2: 0 = as i - 1, else k slots to the left child
    std::vector<uint32_t> first, count; // triangle range of the subtree (leaf order)
    float cNode = 1.0f, cTri = 1.0f;
    float areaW[3] = { 1.0f, 1.0f, 1.0f };
};

float childCost(const CollapsePlan& P, const Child8& c, int i)
{
    if (c.code >= 0) return P.cost[8u * static_cast<uint32_t>(c.code) + (i - 1)];
    return P.cTri * c.box.area(P.areaW) * static_cast<float>((static_cast<uint32_t>(~c.code) & (kMaxLeafSize - 1)) + 1);
}

// The plan of BVH2 node k from its children's (planCollapse).
void planNode(const BvhBuildResult& bvh2, CollapsePlan& P, size_t k)
{
    const float cNode = P.cNode, cTri = P.cTri;
    {
        Child8 ch[2];
        int m = 0;
        childrenOf(bvh2.nodes[k], ch, m);
        uint32_t lo = UINT32_MAX, tot = 0;
        for (int c = 0; c < m; ++c) {
            if (ch[c].code >= 0) {
                lo = std::min(lo, P.first[ch[c].code]);
                tot += P.count[ch[c].code];
            } else {
                const uint32_t code = static_cast<uint32_t>(~ch[c].code);
                lo = std::min(lo, code >> kLeafCountBits);
                tot += (code & (kMaxLeafSize - 1)) + 1u;
            }
        }
        P.first[k] = lo;
        P.count[k] = tot;
        Aabb box;
        for (int c = 0; c < m; ++c) box.grow(ch[c].box);
        const float area = box.area(P.areaW);
        float* C = &P.cost[8 * k];
        uint8_t* pk = &P.pick[8 * k];
        // distributions of j slots over the two subtrees
        auto dist = [&](int j, int& bestK) {
            float best = INFINITY;
            bestK = 0;
            if (m == 1) {
                bestK = j;
                return childCost(P, ch[0], j);
            }
            for (int kk = 1; kk < j; ++kk) {
                const float v = childCost(P, ch[0], kk) + childCost(P, ch[1], j - kk);
                if (v < best) {
                    best = v;
                    bestK = kk;
                }
            }
            return best;
        };
        int k8;
        const float asNode = cNode * area + dist(8, k8);
        const float asLeaf = tot <= static_cast<uint32_t>(kBvh8MaxLeafSize) ? cTri * area * static_cast<float>(tot) : INFINITY;
        C[0] = std::min(asNode, asLeaf);
        pk[0] = asLeaf < asNode ? 1 : 0;
        for (int i = 2; i <= 8; ++i) {
            int kk;
            const float d = dist(i, kk);
            if (d < C[i - 2]) {
                C[i - 1] = d;
                pk[i - 1] = static_cast<uint8_t>(kk);
            } else {
                C[i - 1] = C[i - 2];
                pk[i - 1] = 0;
            }
        }
    }
}

// Children before parents: the subtrees of the top levels on their own threads (each
// node's plan reads only its children's), identical to a sweep in decreasing index.
void planSubtree(const BvhBuildResult& bvh2, CollapsePlan& P, size_t k, int spawnLevels)
{
    Child8 ch[2];
    int m = 0;
    childrenOf(bvh2.nodes[k], ch, m);
    int32_t inner[2];
    int ni = 0;
    for (int c = 0; c < m; ++c)
        if (ch[c].code >= 0) inner[ni++] = ch[c].code;
    if (ni == 2 && spawnLevels > 0) {
        std::thread t([&] { planSubtree(bvh2, P, static_cast<size_t>(inner[0]), spawnLevels - 1); });
        planSubtree(bvh2, P, static_cast<size_t>(inner[1]), spawnLevels - 1);
        t.join();
    } else {
        for (int c = 0; c < ni; ++c) planSubtree(bvh2, P, static_cast<size_t>(inner[c]), spawnLevels - 1);
    }
    planNode(bvh2, P, k);
}

CollapsePlan planCollapse(const BvhBuildResult& bvh2, float cNode, float cTri, const float* areaW, int threads)
{
    CollapsePlan P;
    P.cNode = cNode;
    P.cTri = cTri;
    for (int k = 0; k < 3; ++k) P.areaW[k] = areaW[k];
    const size_t N = bvh2.nodes.size();
    P.cost.assign(8 * N, 0.0f);
    P.pick.assign(8 * N, 0);
    P.first.assign(N, 0);
    P.count.assign(N, 0);
    int levels = 0;
    for (int t = threads > 0 ? threads : static_cast<int>(std::thread::hardware_concurrency()); (1 << levels) < 2 * t && levels < 8; ++levels) {}
    if (N > (1u << 16)) planSubtree(bvh2, P, 0, levels);
    else
        for (size_t k = N; k-- > 0;) planNode(bvh2, P, k); // children have larger indices
    return P;
}

// The children the plan gives a subtree (BVH2 item `c`) when it gets `i` slots.
void emitChildren(const BvhBuildResult& bvh2, const CollapsePlan& P, const Child8& c, int i, Child8* out, int& n)
{
    if (c.code < 0) {
        out[n++] = c;
        return;
    }
    const uint32_t k = static_cast<uint32_t>(c.code);
    while (i > 1 && P.pick[8 * k + (i - 1)] == 0) --i;
    if (i == 1) {
        Child8 x = c;
        if (P.pick[8 * k] == 1) // the whole subtree as one leaf slot
            x.code = ~static_cast<int32_t>((P.first[k] << kLeafCountBits) | (P.count[k] - 1u));
        out[n++] = x;
        return;
    }
    Child8 two[2];
    int m = 0;
    childrenOf(bvh2.nodes[k], two, m);
    const int kk = P.pick[8 * k + (i - 1)];
    if (m == 1) {
        emitChildren(bvh2, P, two[0], i, out, n);
        return;
    }
    emitChildren(bvh2, P, two[0], kk, out, n);
    emitChildren(bvh2, P, two[1], i - kk, out, n);
}

namespace {
struct CollapseItem {
    uint32_t src;   // BVH2 node
    uint32_t dst;   // BVH8 node (index in its part)
    uint32_t depth;
};

// One part of a collapse: the BVH8 nodes of a subtree (or of the top levels) in BFS
// order with part-local child and triangle indices, its triangle rows.
struct CollapsePart {
    std::vector<GpuBvh8Node> nodes;
    std::vector<GpuTriangle> tris;
    RowPlacer rows;
    uint32_t max_depth = 0;
    uint32_t leaf_children = 0;
    uint64_t triangles = 0;
    double sah = 0.0;
};

// Collapses the queue's items breadth first into `out`; items deeper than stopDepth go
// to `frontier` unprocessed (their node slots are allocated).
void collapseQueue(const BvhBuildResult& bvh2, const CollapsePlan& plan, const Bvh8CollapseOptions& copt, double& rootArea, CollapsePart& out,
                   std::vector<CollapseItem> queue, uint32_t stopDepth, std::vector<CollapseItem>* frontier)
{
    for (size_t qi = 0; qi < queue.size(); ++qi) {
        const CollapseItem it = queue[qi];
        if (it.depth > stopDepth) {
            frontier->push_back(it);
            continue;
        }
        const bool isRoot = frontier && qi == 0; // the top part's first item is the BVH's root
        out.max_depth = std::max(out.max_depth, it.depth);
        Child8 ch[8];
        int n = 0;
        if (copt.sah_optimal) {
            // the plan's best 8-way distribution below this node
            Child8 two[2];
            int m = 0;
            childrenOf(bvh2.nodes[it.src], two, m);
            if (m == 1) {
                emitChildren(bvh2, plan, two[0], 8, ch, n);
            } else {
                const uint32_t src = it.src;
                int kk = 1;
                float best = INFINITY;
                for (int k = 1; k < 8; ++k) {
                    const float v = childCost(plan, two[0], k) + childCost(plan, two[1], 8 - k);
                    if (v < best) {
                        best = v;
                        kk = k;
                    }
                }
                (void)src;
                emitChildren(bvh2, plan, two[0], kk, ch, n);
                emitChildren(bvh2, plan, two[1], 8 - kk, ch, n);
            }
        } else {
            // gather up to 8 children: open the largest-area internal child first
            {
                Child8 two[2];
                int m = 0;
                childrenOf(bvh2.nodes[it.src], two, m);
                for (int c = 0; c < m; ++c) ch[n++] = two[c];
            }
            for (;;) {
                int best = -1;
                float bestArea = -1.0f;
                for (int c = 0; c < n; ++c)
                    if (ch[c].code >= 0 && ch[c].box.area() > bestArea) {
                        bestArea = ch[c].box.area();
                        best = c;
                    }
                if (best < 0) break;
                Child8 two[2];
                int m = 0;
                childrenOf(bvh2.nodes[ch[best].code], two, m);
                if (n - 1 + m > 8) break;
                ch[best] = two[0];
                for (int c = 1; c < m; ++c) ch[n++] = two[c];
                if (m == 0) ch[best] = ch[--n];
            }
        }
        // octant slots: greedy on the alignment of child centre offsets with slot signs
        Aabb box;
        for (int c = 0; c < n; ++c) box.grow(ch[c].box);
        // SAH cost of the result (node cost 1, the plan's triangle cost), for reports
        if (isRoot) {
            rootArea = std::max(1e-30, static_cast<double>(box.area()));
            out.sah += 1.0;
        }
        for (int c = 0; c < n; ++c) {
            const double a = ch[c].box.area() / rootArea;
            out.sah += ch[c].code >= 0 ? a : a * copt.tri_cost * static_cast<double>((static_cast<uint32_t>(~ch[c].code) & (kMaxLeafSize - 1)) + 1);
        }
        float pc[3];
        for (int a = 0; a < 3; ++a) pc[a] = 0.5f * (box.lo[a] + box.hi[a]);
        struct Cand {
            float score;
            int c, s;
        };
        // Internal children take their octant slots first; leaf children only decide
        // which triangles a hit slot adds (their order does not matter), so they fill
        // the remaining slots in ascending order, most triangles first, which keeps a
        // node's triangle rows compact (leafRowStride; leaves competing for octant slots
        // like internal children measured no better, round 3).
        constexpr bool leafOctant = false;
        Cand cand[64];
        int nc = 0;
        int slotOf[8], childIn[8];
        for (int k = 0; k < 8; ++k) slotOf[k] = childIn[k] = -1;
        if (copt.slot_sort_axis >= 0 && copt.slot_sort_axis < 3) {
            // one ray direction (+axis): internal children in slots 0, 1, ... by the
            // lower bound of their box along it, the order a ray from below meets them
            const int ax = copt.slot_sort_axis;
            int internal[8], ni = 0;
            for (int c = 0; c < n; ++c)
                if (ch[c].code >= 0 || leafOctant) internal[ni++] = c;
            std::stable_sort(internal, internal + ni, [&](int a, int b) { return ch[a].box.lo[ax] < ch[b].box.lo[ax]; });
            for (int k = 0; k < ni; ++k) {
                slotOf[internal[k]] = k;
                childIn[k] = internal[k];
            }
        } else {
            for (int c = 0; c < n; ++c)
                for (int s = 0; s < 8; ++s) {
                    if (!leafOctant && ch[c].code < 0) break;
                    float sc = 0.0f;
                    for (int a = 0; a < 3; ++a) {
                        const float off = 0.5f * (ch[c].box.lo[a] + ch[c].box.hi[a]) - pc[a];
                        sc += ((s >> a) & 1) ? off : -off;
                    }
                    cand[nc++] = { sc, c, s };
                }
            std::stable_sort(cand, cand + nc, [](const Cand& x, const Cand& y) { return x.score > y.score; });
            for (int k = 0; k < nc; ++k)
                if (slotOf[cand[k].c] < 0 && childIn[cand[k].s] < 0) {
                    slotOf[cand[k].c] = cand[k].s;
                    childIn[cand[k].s] = cand[k].c;
                }
        }
        if (!leafOctant) {
            int leaves[8], nl = 0;
            for (int c = 0; c < n; ++c)
                if (ch[c].code < 0) leaves[nl++] = c;
            auto cnt = [&](int c) { return (static_cast<uint32_t>(~ch[c].code) & (kMaxLeafSize - 1)) + 1u; };
            std::stable_sort(leaves, leaves + nl, [&](int a, int b) { return cnt(a) > cnt(b); });
            int sl = 0;
            for (int i = 0; i < nl; ++i) {
                while (childIn[sl] >= 0) ++sl;
                slotOf[leaves[i]] = sl;
                childIn[sl] = leaves[i];
            }
        }
        // quantization grid of this node
        GpuBvh8Node nd;
        std::memset(&nd, 0, sizeof(nd));
        double step[3], p[3];
        for (int a = 0; a < 3; ++a) {
            int e;
            quantGrid(box.lo[a], box.hi[a], e, p[a]);
            step[a] = std::ldexp(1.0, e);
            nd.p[a] = static_cast<float>(p[a]);
            nd.e[a] = static_cast<uint8_t>(e + 127);
        }
        // children in slot order: internal ones get consecutive node indices; leaf
        // triangle i of slot s goes to position s + stride * i (GpuBvh8Node), the
        // rows placed at the first base in the tail of the array where all of their
        // positions are free
        const uint32_t childBase = static_cast<uint32_t>(out.nodes.size());
        uint32_t leafCnt[8] = {}, leafMask = 0;
        for (int s = 0; s < 8; ++s) {
            const int c = childIn[s];
            if (c < 0 || ch[c].code >= 0) continue;
            leafCnt[s] = (static_cast<uint32_t>(~ch[c].code) & (kMaxLeafSize - 1)) + 1u;
            leafMask |= 1u << s;
        }
        const uint32_t stride = leafRowStride(leafCnt);
        uint32_t rows = 0;
        for (uint32_t s = 0; s < 8; ++s)
            for (uint32_t i = 0; i < leafCnt[s]; ++i) rows |= 1u << (s + stride * i);
        const uint32_t triStart = rows ? out.rows.place(rows) : 0u;
        if (rows && out.tris.size() < triStart + 24u) out.tris.resize(triStart + 24u, holeTriangle());
        nd.child_base = childBase; // local: offset when the parts are joined
        nd.tri_base = triStart;
        nd.leaf_tris = rows;
        nd.tri_stride = static_cast<uint8_t>(stride);
        nd.leaf_mask = static_cast<uint8_t>(leafMask);
        uint32_t nInternal = 0;
        for (int s = 0; s < 8; ++s) {
            const int c = childIn[s];
            if (c < 0) continue;
            const Child8& k = ch[c];
            for (int a = 0; a < 3; ++a) {
                double ql = std::floor((static_cast<double>(k.box.lo[a]) - p[a]) / step[a]);
                double qh = std::ceil((static_cast<double>(k.box.hi[a]) - p[a]) / step[a]);
                ql = std::min(255.0, std::max(0.0, ql));
                qh = std::min(255.0, std::max(0.0, qh));
                // outward rounding, checked on the exact fp32 decode
                while (ql > 0.0 && static_cast<double>(static_cast<float>(p[a] + ql * step[a])) > k.box.lo[a]) ql -= 1.0;
                while (qh < 255.0 && static_cast<double>(static_cast<float>(p[a] + qh * step[a])) < k.box.hi[a]) qh += 1.0;
                nd.qlo[a][s] = static_cast<uint8_t>(ql);
                nd.qhi[a][s] = static_cast<uint8_t>(qh);
            }
            if (k.code >= 0) {
                nd.imask |= static_cast<uint8_t>(1u << s);
                queue.push_back({ static_cast<uint32_t>(k.code), childBase + nInternal, it.depth + 1 });
                nInternal++;
            } else {
                const uint32_t code = static_cast<uint32_t>(~k.code);
                const uint32_t first = code >> kLeafCountBits, cnt = (code & (kMaxLeafSize - 1)) + 1u;
                for (uint32_t i = 0; i < cnt; ++i) out.tris[triStart + static_cast<uint32_t>(s) + stride * i] = bvh2.tris[first + i];
                out.leaf_children++;
                out.triangles += cnt;
            }
        }
        out.nodes.resize(out.nodes.size() + nInternal);
        out.nodes[it.dst] = nd;
    }
}
} // namespace

// The top levels (BVH8 depth <= kTopDepth) are collapsed first, then the subtrees below
// them in parallel, each a part with its own node and triangle-row arrays, joined in
// order: the top levels stay breadth first at the front (k_trace_shadow caches the
// first nodes in LDS), every subtree is breadth first in its block. (One sequential
// breadth-first pass took 6.2 s of a C4 build; the plan's DP is shared.)
Bvh8BuildResult collapse_bvh8(const BvhBuildResult& bvh2, uint32_t node_base, uint32_t tri_base, const Bvh8CollapseOptions& copt)
{
    Bvh8BuildResult res;
    if (bvh2.nodes.empty()) return res;
    CollapsePlan plan;
    if (copt.sah_optimal) plan = planCollapse(bvh2, copt.node_cost, copt.tri_cost, copt.area_w, copt.threads);
    constexpr uint32_t kTopDepth = 3;
    double rootArea = 0.0;
    CollapsePart top;
    top.nodes.resize(1);
    std::vector<CollapseItem> frontier;
    collapseQueue(bvh2, plan, copt, rootArea, top, { { 0u, 0u, 1u } }, kTopDepth, &frontier);
    std::vector<CollapsePart> parts(frontier.size());
    {
        const int hw = copt.threads > 0 ? copt.threads : static_cast<int>(std::thread::hardware_concurrency());
        const int T = std::max(1, std::min<int>(hw, static_cast<int>(frontier.size())));
        std::atomic<size_t> next { 0 };
        auto worker = [&] {
            for (size_t f; (f = next.fetch_add(1)) < frontier.size();) {
                parts[f].nodes.resize(1);
                double ra = rootArea;
                collapseQueue(bvh2, plan, copt, ra, parts[f], { { frontier[f].src, 0u, frontier[f].depth } }, UINT32_MAX, nullptr);
            }
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < T; ++t) pool.emplace_back(worker);
        worker();
        for (std::thread& th : pool) th.join();
    }
    // join: subtree f's root fills its frontier slot of the top part, its other nodes
    // follow the top part's nodes; its rows follow the top part's rows
    auto trimHoles = [](std::vector<GpuTriangle>& t) {
        while (!t.empty() && isHoleTriangle(t.back())) t.pop_back();
    };
    trimHoles(top.tris);
    size_t nodeCount = top.nodes.size(), triCount = top.tris.size();
    std::vector<size_t> nodeOff(parts.size()), triOff(parts.size());
    for (size_t f = 0; f < parts.size(); ++f) {
        trimHoles(parts[f].tris);
        nodeOff[f] = nodeCount;
        triOff[f] = triCount;
        nodeCount += parts[f].nodes.size() - 1;
        triCount += parts[f].tris.size();
    }
    res.nodes.resize(nodeCount);
    res.tris.reserve(triCount);
    auto place = [&](GpuBvh8Node nd, size_t nodeShift, size_t triShift) {
        nd.child_base = node_base + static_cast<uint32_t>(nd.child_base + nodeShift);
        nd.tri_base = tri_base + static_cast<uint32_t>(nd.leaf_tris ? nd.tri_base + triShift : 0u);
        return nd;
    };
    for (size_t k = 0; k < top.nodes.size(); ++k) res.nodes[k] = place(top.nodes[k], 0, 0);
    res.tris.insert(res.tris.end(), top.tris.begin(), top.tris.end());
    res.max_depth = top.max_depth;
    res.leaf_children = top.leaf_children;
    res.triangles = top.triangles;
    double sah = top.sah;
    for (size_t f = 0; f < parts.size(); ++f) {
        const CollapsePart& P = parts[f];
        // part-local node k >= 1 -> nodeOff + k - 1 (its children are all >= 1)
        const size_t shift = nodeOff[f] - 1;
        res.nodes[frontier[f].dst] = place(P.nodes[0], shift, triOff[f]);
        for (size_t k = 1; k < P.nodes.size(); ++k) res.nodes[shift + k] = place(P.nodes[k], shift, triOff[f]);
        res.tris.insert(res.tris.end(), P.tris.begin(), P.tris.end());
        res.max_depth = std::max(res.max_depth, P.max_depth);
        res.leaf_children += P.leaf_children;
        res.triangles += P.triangles;
        sah += P.sah;
    }
    res.sah_cost = static_cast<float>(sah);
    return res;
}

BvhBuildResult build_bvh(const std::vector<BuildTriangle>& tris, const BvhBuildOptions& opt, uint32_t node_base, uint32_t tri_base)
{
    if (tris.empty()) return {};
    Builder b(tris, opt, node_base, tri_base);
    return b.run(tris);
}

} // namespace ark

// ark_ddgi_debug.h: host-side structural check of the BVH8 (see the header).
extern "C" int ark_ddgi_debug_bvh8_check(const float* triangles, uint64_t n, uint64_t* out)
{
    return ark_ddgi_debug_bvh8_check_opts(triangles, n, 1, 0.0f, out);
}

extern "C" int ark_ddgi_debug_bvh8_check_opts(const float* triangles, uint64_t n, int sah_optimal, float tri_cost, uint64_t* out)
{
    using namespace ark;
    std::vector<BuildTriangle> tris(n);
    for (uint64_t i = 0; i < n; ++i) {
        for (int a = 0; a < 3; ++a) {
            tris[i].v0[a] = triangles[9 * i + a];
            tris[i].v1[a] = triangles[9 * i + 3 + a];
            tris[i].v2[a] = triangles[9 * i + 6 + a];
        }
        tris[i].instance = 0;
        tris[i].primitive = static_cast<uint32_t>(i);
        tris[i].flip_facing = 0;
    }
    BvhBuildOptions opt;
    opt.max_leaf_size = kBvh8MaxLeafSize;
    opt.inflate_abs = bvh8_inflation(triangles, n);
    const BvhBuildResult r2 = build_bvh(tris, opt, 0u, 0u);
    Bvh8CollapseOptions copt;
    copt.sah_optimal = sah_optimal != 0;
    if (tri_cost > 0.0f) copt.tri_cost = std::max(0.01f, tri_cost);
    const Bvh8BuildResult r8 = collapse_bvh8(r2, 0u, 0u, copt);
    uint64_t violations = 0, internalChildren = 0;
    std::vector<uint32_t> seen(n, 0);
    struct Box {
        float lo[3], hi[3];
    };
    struct Item {
        uint32_t node;
        std::vector<Box> anc;
    };
    std::vector<Item> work;
    if (!r8.nodes.empty()) work.push_back({ 0u, {} });
    while (!work.empty()) {
        Item it = std::move(work.back());
        work.pop_back();
        if (it.node >= r8.nodes.size()) {
            violations++;
            continue;
        }
        const GpuBvh8Node& nd = r8.nodes[it.node];
        uint32_t internal = 0;
        for (int s = 0; s < 8; ++s) {
            const bool in = (nd.imask >> s) & 1u;
            uint32_t slotTris[kBvh8MaxLeafSize];
            const int cnt = bvh8SlotTriangles(nd, s, slotTris);
            if (cnt < 0) {
                violations++;
                continue;
            }
            if (!in && cnt == 0) continue;
            Box b;
            for (int a = 0; a < 3; ++a) {
                const float step = std::ldexp(1.0f, static_cast<int>(nd.e[a]) - 127);
                b.lo[a] = std::fma(static_cast<float>(nd.qlo[a][s]), step, nd.p[a]);
                b.hi[a] = std::fma(static_cast<float>(nd.qhi[a][s]), step, nd.p[a]);
                if (static_cast<double>(b.lo[a]) != static_cast<double>(nd.p[a]) + nd.qlo[a][s] * static_cast<double>(step)) violations++;
                if (static_cast<double>(b.hi[a]) != static_cast<double>(nd.p[a]) + nd.qhi[a][s] * static_cast<double>(step)) violations++;
            }
            std::vector<Box> anc = it.anc;
            anc.push_back(b);
            if (in) {
                internalChildren++;
                work.push_back({ nd.child_base + internal++, std::move(anc) });
                continue;
            }
            for (int ti = 0; ti < cnt; ++ti) {
                const uint32_t t = slotTris[ti];
                if (t >= r8.tris.size() || isHoleTriangle(r8.tris[t])) {
                    violations++;
                    continue;
                }
                const GpuTriangle& g = r8.tris[t];
                uint32_t prim;
                std::memcpy(&prim, &g.t2[2], 4);
                if (prim < n) seen[prim]++;
                if (prim >= n) continue;
                const float* verts[3] = { tris[prim].v0, tris[prim].v1, tris[prim].v2 };
                for (int k = 0; k < 3; ++k)
                    for (int a = 0; a < 3; ++a)
                        for (const Box& bx : anc)
                            if (verts[k][a] < bx.lo[a] || verts[k][a] > bx.hi[a]) violations++;
            }
        }
    }
    for (uint64_t i = 0; i < n; ++i)
        if (seen[i] != 1) violations++;
    if (out) {
        out[0] = r8.nodes.size();
        out[1] = r8.leaf_children;
        out[2] = r8.max_depth;
        out[3] = violations;
        out[4] = r8.triangles;
        out[5] = r2.nodes.size();
        out[6] = internalChildren;
        out[7] = static_cast<uint64_t>(static_cast<double>(r8.sah_cost) * 1e6); // BVH8 SAH cost x 1e6
    }
    return violations == 0 ? 0 : 1;
}

namespace ark {

// The sun's shadow rays (opaque.rchit:35-54, the sun branch :56-73) all travel along
// L = -normalize(sun direction) - the fp32 value k_shadow_gen gives them. In the
// orthonormal frame (u, v, w = L / |L|) they are rays along +w: a child box is crossed
// iff the ray's (u, v) lies in the box's u-v rectangle and the box reaches above its
// origin, a containment test in the node's quantized grid with no division and no
// per-child multiply (k_trace_shadow<SUN>, visitNodeSun). The light-space BVH holds
// every triangle of every hit-mask class (shadow rays test all three with the Opaque
// flag, no alpha test) with the world-space triangle records, so the any-hit tests and
// their results are those of the world BVHs.
void sun_frame(const float sunDir[3], double frame[3][3])
{
    // L = -normalize(dir) in fp32, the operation order of normalize() in the kernels
    // (v * (1 / sqrt(dot(v, v))), dot left to right)
    const float dd = sunDir[0] * sunDir[0] + sunDir[1] * sunDir[1] + sunDir[2] * sunDir[2];
    const float sc = 1.0f / std::sqrt(dd);
    const float L[3] = { -(sunDir[0] * sc), -(sunDir[1] * sc), -(sunDir[2] * sc) };
    double w[3] = { L[0], L[1], L[2] };
    const double wl = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    for (double& x : w) x /= wl;
    const double h[3] = { std::fabs(w[0]) < 0.9 ? 1.0 : 0.0, std::fabs(w[0]) < 0.9 ? 0.0 : 1.0, 0.0 };
    double u[3] = { h[1] * w[2] - h[2] * w[1], h[2] * w[0] - h[0] * w[2], h[0] * w[1] - h[1] * w[0] };
    const double ul = std::sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    for (double& x : u) x /= ul;
    const double v[3] = { w[1] * u[2] - w[2] * u[1], w[2] * u[0] - w[0] * u[2], w[0] * u[1] - w[1] * u[0] };
    for (int k = 0; k < 3; ++k) {
        frame[0][k] = u[k];
        frame[1][k] = v[k];
        frame[2][k] = w[k];
    }
}

// Light-space build triangles of world-space records: rec(i) gives triangle i's record.
template<class RecordOf>
static void sunAddRecords(SunBvhInput& in, size_t n, RecordOf rec, int threads)
{
    const size_t base = in.world.size();
    in.tris.resize(base + n);
    in.world.resize(base + n);
    // independent per triangle: in chunks on `threads` threads, the largest |coordinate|
    // reduced at the end (a max does not depend on the order)
    const int T = std::max(1, std::min<int>(threads > 0 ? threads : static_cast<int>(std::thread::hardware_concurrency()), static_cast<int>(n >> 16) + 1));
    std::vector<float> maxAbs(T, 0.0f);
    auto work = [&](int t) {
        const size_t b = n * t / T, e = n * (t + 1) / T;
        for (size_t i = b; i < e; ++i) {
            const GpuTriangle rc = rec(i);
            // the triangle Möller–Trumbore tests: v0, v0 + e1, v0 + e2 (exact, from the record)
            double V[3][3];
            for (int a = 0; a < 3; ++a) V[0][a] = rc.t0[a];
            const double e1[3] = { rc.t0[3], rc.t1[0], rc.t1[1] }, e2[3] = { rc.t1[2], rc.t1[3], rc.t2[0] };
            for (int a = 0; a < 3; ++a) {
                V[1][a] = V[0][a] + e1[a];
                V[2][a] = V[0][a] + e2[a];
                maxAbs[t] = std::max(maxAbs[t], static_cast<float>(std::max({ std::fabs(V[0][a]), std::fabs(V[1][a]), std::fabs(V[2][a]) })));
            }
            BuildTriangle& l = in.tris[base + i];
            float* dst[3] = { l.v0, l.v1, l.v2 };
            for (int k = 0; k < 3; ++k)
                for (int r = 0; r < 3; ++r)
                    dst[k][r] = static_cast<float>(in.frame[r][0] * V[k][0] + in.frame[r][1] * V[k][1] + in.frame[r][2] * V[k][2]);
            l.instance = 0;
            l.primitive = static_cast<uint32_t>(base + i);
            l.flip_facing = 0;
            in.world[base + i] = rc;
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < T; ++t) pool.emplace_back(work, t);
    work(0);
    for (std::thread& th : pool) th.join();
    for (float m : maxAbs) in.maxAbs = std::max(in.maxAbs, m);
}

void sun_add_triangles(SunBvhInput& in, const std::vector<BuildTriangle>& tris, int threads)
{
    sunAddRecords(in, tris.size(), [&](size_t i) { return make_gpu_triangle(tris[i]); }, threads);
}

void sun_add_records(SunBvhInput& in, const std::vector<GpuTriangle>& records, int threads)
{
    std::vector<uint32_t> live;
    live.reserve(records.size());
    for (size_t i = 0; i < records.size(); ++i)
        if (!isHoleTriangle(records[i])) live.push_back(static_cast<uint32_t>(i));
    sunAddRecords(in, live.size(), [&](size_t i) { return records[live[i]]; }, threads);
}

bool build_sun_bvh(SunBvhInput& in, const BvhBuildOptions& opt, const Bvh8CollapseOptions& copt, Bvh8BuildResult& out)
{
    // light-space box inflation: the rounding of the light coordinates to fp32 here and
    // of the origin's (u, v, w) in the kernel (a 3-term fp32 dot product, about 3 ulp of
    // |P|), Möller–Trumbore's acceptance margin (as the world BVHs: bvh8_inflation_box,
    // 1e-6 of the diagonal) - each covered twice over
    float lo[3] = { INFINITY, INFINITY, INFINITY }, hi[3] = { -INFINITY, -INFINITY, -INFINITY };
    for (const BuildTriangle& t : in.tris)
        for (const float* v : { t.v0, t.v1, t.v2 })
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], v[a]);
                hi[a] = std::max(hi[a], v[a]);
            }
    BvhBuildOptions lopt = opt;
    lopt.max_leaf_size = kBvh8MaxLeafSize;
    lopt.inflate_abs = 2.0f * bvh8_inflation_box(lo, hi) + 2e-6f * in.maxAbs;
    in.inflateAbs = lopt.inflate_abs;
    BvhBuildResult r2 = build_bvh(in.tris, lopt, 0u, 0u);
    std::vector<BuildTriangle>().swap(in.tris);
    if (r2.max_leaf > static_cast<uint32_t>(kBvh8MaxLeafSize)) return false;
    Bvh8CollapseOptions lc = copt;
    lc.slot_sort_axis = 2; // every ray goes along +w
    out = collapse_bvh8(r2, 0u, 0u, lc);
    // the leaves' records become the world-space ones (primitive = world index)
    for (GpuTriangle& g : out.tris) {
        if (isHoleTriangle(g)) continue;
        uint32_t idx;
        std::memcpy(&idx, &g.t2[2], 4);
        g = in.world[idx];
    }
    std::vector<GpuTriangle>().swap(in.world);
    return true;
}

void sun_sample_origins(const std::vector<GpuTriangle>& tris, const float L[3], uint32_t n, std::vector<float>& out)
{
    out.clear();
    if (tris.empty() || n == 0) return;
    uint64_t x = 0x9E3779B97F4A7C15ull; // xorshift64: the same samples every build
    auto next = [&]() {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        return x;
    };
    for (uint64_t tries = 0; out.size() < 3ull * n && tries < 32ull * n; ++tries) {
        const GpuTriangle& g = tris[next() % tris.size()];
        if (isHoleTriangle(g)) continue;
        const double e1[3] = { g.t0[3], g.t1[0], g.t1[1] }, e2[3] = { g.t1[2], g.t1[3], g.t2[0] };
        const double nrm[3] = { e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0] };
        uint32_t flip;
        std::memcpy(&flip, &g.t2[3], 4);
        const double dn = (nrm[0] * L[0] + nrm[1] * L[1] + nrm[2] * L[2]) * (flip ? -1.0 : 1.0);
        if (!(dn > 0.0)) continue; // the front face (CCW, mirrored instances flipped) must face the sun
        const double r1 = static_cast<double>(next() >> 11) * 0x1p-53, r2 = static_cast<double>(next() >> 11) * 0x1p-53;
        const double sq = std::sqrt(r1), b1 = sq * (1.0 - r2), b2 = sq * r2;
        for (int a = 0; a < 3; ++a) out.push_back(static_cast<float>(g.t0[a] + b1 * e1[a] + b2 * e2[a]));
    }
}

double sun_shadow_cost(const std::vector<GpuBvh8Node>& nodes, const std::vector<GpuTriangle>& tris, const int32_t* roots, int nRoots,
                       const double (*frame)[3], const float L[3], const std::vector<float>& origins)
{
    const size_t n = origins.size() / 3;
    if (n == 0) return 0.0;
    const float tmin = 0.025f, tmax = 1e30f;
    uint64_t steps = 0;
    std::vector<uint32_t> stack;
    for (size_t r = 0; r < n; ++r) {
        const float* P = &origins[3 * r];
        float ob[3], db[3];
        for (int a = 0; a < 3; ++a) {
            ob[a] = frame ? static_cast<float>(frame[a][0] * P[0] + frame[a][1] * P[1] + frame[a][2] * P[2]) : P[a];
            db[a] = frame ? (a == 2 ? 1.0f : 0.0f) : L[a];
        }
        float idir[3];
        for (int a = 0; a < 3; ++a) idir[a] = 1.0f / (std::fabs(db[a]) < 1e-20f ? std::copysign(1e-20f, db[a]) : db[a]);
        bool hit = false;
        for (int k = 0; k < nRoots && !hit; ++k) {
            if (roots[k] < 0) continue;
            stack.assign(1, static_cast<uint32_t>(roots[k]));
            while (!stack.empty() && !hit) {
                const GpuBvh8Node& nd = nodes[stack.back()];
                stack.pop_back();
                steps++;
                struct Cand { float tn; int s; } hc[8];
                int nh = 0;
                uint32_t before[8], cnt = 0;
                for (int s = 0; s < 8; ++s) {
                    before[s] = cnt;
                    if ((nd.imask >> s) & 1u) cnt++;
                    if (!((nd.imask >> s) & 1u) && !((nd.leaf_mask >> s) & 1u)) continue;
                    float tn = tmin, tf = tmax;
                    for (int a = 0; a < 3; ++a) {
                        const float step = std::ldexp(1.0f, static_cast<int>(nd.e[a]) - 127);
                        float t0 = (std::fma(static_cast<float>(nd.qlo[a][s]), step, nd.p[a]) - ob[a]) * idir[a];
                        float t1 = (std::fma(static_cast<float>(nd.qhi[a][s]), step, nd.p[a]) - ob[a]) * idir[a];
                        if (t0 > t1) std::swap(t0, t1);
                        tn = std::max(tn, t0);
                        tf = std::min(tf, t1);
                    }
                    if (tn <= tf * 1.00001f + 1e-7f) hc[nh++] = { tn, s };
                }
                std::sort(hc, hc + nh, [](const Cand& p, const Cand& q) { return p.tn < q.tn; });
                // the node's leaf triangles first (the dual step), nearest leaf first
                for (int i = 0; i < nh && !hit; ++i) {
                    if ((nd.imask >> hc[i].s) & 1u) continue;
                    uint32_t t[kBvh8MaxLeafSize];
                    const int c = bvh8SlotTriangles(nd, hc[i].s, t);
                    for (int j = 0; j < c && !hit; ++j) {
                        steps++;
                        const GpuTriangle& g = tris[t[j]];
                        const float v0[3] = { g.t0[0], g.t0[1], g.t0[2] }, e1[3] = { g.t0[3], g.t1[0], g.t1[1] }, e2[3] = { g.t1[2], g.t1[3], g.t2[0] };
                        const float pv[3] = { L[1] * e2[2] - L[2] * e2[1], L[2] * e2[0] - L[0] * e2[2], L[0] * e2[1] - L[1] * e2[0] };
                        const float det = e1[0] * pv[0] + e1[1] * pv[1] + e1[2] * pv[2];
                        if (det == 0.0f) continue;
                        const float inv = 1.0f / det;
                        const float sv[3] = { P[0] - v0[0], P[1] - v0[1], P[2] - v0[2] };
                        const float u = (sv[0] * pv[0] + sv[1] * pv[1] + sv[2] * pv[2]) * inv;
                        if (!(u >= 0.0f && u <= 1.0f)) continue;
                        const float q[3] = { sv[1] * e1[2] - sv[2] * e1[1], sv[2] * e1[0] - sv[0] * e1[2], sv[0] * e1[1] - sv[1] * e1[0] };
                        const float v = (L[0] * q[0] + L[1] * q[1] + L[2] * q[2]) * inv;
                        if (!(v >= 0.0f && u + v <= 1.0f)) continue;
                        const float tt = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * inv;
                        hit = tt >= tmin && tt <= tmax;
                    }
                }
                for (int i = nh - 1; i >= 0 && !hit; --i)
                    if ((nd.imask >> hc[i].s) & 1u) stack.push_back(nd.child_base + before[hc[i].s]);
            }
        }
    }
    return static_cast<double>(steps) / static_cast<double>(n);
}

} // namespace ark


// ark_ddgi_debug.h: the sun's light-space BVH on the host (no GPU), checked against
// brute force. Builds it as set_scene does (sun_frame, sun_add_triangles,
// build_sun_bvh), then for every origin traces a sun shadow ray (L = -normalize(sun
// dir) in fp32, [0.025, tmax]) twice: through the BVH with a host restatement of
// k_trace_shadow<SUN>'s node test (visitNodeSun: the same fp32 quantized coordinate,
// floor / ceil, integer plane compares) and against every triangle; both use the same
// Möller–Trumbore (the kernels' operation order). out[8] = {rays, occluded (brute
// force), occluded (BVH), mismatches, node visits, triangle tests, BVH8 nodes, max
// stack depth}. A mismatch would be a culled occluder: the node test must be
// conservative.
extern "C" int ark_ddgi_debug_sun_bvh_check(const float* triangles, uint64_t n, const float* sun_dir, const float* origins, uint64_t n_rays, float tmax,
                                             uint64_t* out)
{
    using namespace ark;
    std::vector<BuildTriangle> tris(n);
    for (uint64_t i = 0; i < n; ++i) {
        for (int a = 0; a < 3; ++a) {
            tris[i].v0[a] = triangles[9 * i + a];
            tris[i].v1[a] = triangles[9 * i + 3 + a];
            tris[i].v2[a] = triangles[9 * i + 6 + a];
        }
        tris[i].instance = 0;
        tris[i].primitive = static_cast<uint32_t>(i);
        tris[i].flip_facing = 0;
    }
    SunBvhInput in;
    sun_frame(sun_dir, in.frame);
    sun_add_triangles(in, tris);
    std::vector<GpuTriangle> world = in.world;
    BvhBuildOptions opt;
    opt.threads = 8;
    Bvh8CollapseOptions copt;
    Bvh8BuildResult r;
    if (n == 0 || !build_sun_bvh(in, opt, copt, r)) return 1;
    float F[9];
    for (int a = 0; a < 3; ++a)
        for (int k = 0; k < 3; ++k) F[a * 3 + k] = static_cast<float>(in.frame[a][k]);
    const float dd = sun_dir[0] * sun_dir[0] + sun_dir[1] * sun_dir[1] + sun_dir[2] * sun_dir[2];
    const float sc = 1.0f / std::sqrt(dd);
    const float L[3] = { -(sun_dir[0] * sc), -(sun_dir[1] * sc), -(sun_dir[2] * sc) };
    const float tmin = 0.025f;
    // the kernels' Möller–Trumbore (intersectTri: crossFma / dotFma3, 1 / det)
    auto mt = [&](const float o[3], const GpuTriangle& g) {
        const float v0[3] = { g.t0[0], g.t0[1], g.t0[2] }, e1[3] = { g.t0[3], g.t1[0], g.t1[1] }, e2[3] = { g.t1[2], g.t1[3], g.t2[0] };
        auto cr = [](const float* a, const float* b, float* c) {
            c[0] = std::fma(a[1], b[2], -(a[2] * b[1]));
            c[1] = std::fma(a[2], b[0], -(a[0] * b[2]));
            c[2] = std::fma(a[0], b[1], -(a[1] * b[0]));
        };
        auto dt = [](const float* a, const float* b) { return std::fma(a[0], b[0], std::fma(a[1], b[1], a[2] * b[2])); };
        float p[3], q[3];
        cr(L, e2, p);
        const float det = dt(e1, p);
        const float inv = 1.0f / det;
        const float s[3] = { o[0] - v0[0], o[1] - v0[1], o[2] - v0[2] };
        const float u = dt(s, p) * inv;
        cr(s, e1, q);
        const float v = dt(L, q) * inv;
        const float t = dt(e2, q) * inv;
        return (u >= 0.0f) & (v >= 0.0f) & (u + v <= 1.0f) & (t >= tmin) & (t <= tmax);
    };
    std::atomic<uint64_t> occB { 0 }, occV { 0 }, mism { 0 }, visits { 0 }, tests { 0 }, maxDepth { 0 };
    auto worker = [&](uint64_t r0, uint64_t r1) {
        for (uint64_t ri = r0; ri < r1; ++ri) {
            const float* o = origins + 3 * ri;
            bool brute = false;
            for (const GpuTriangle& g : world)
                if (mt(o, g)) {
                    brute = true;
                    break;
                }
            // light-space traversal (visitNodeSun)
            const float pl[3] = { std::fma(o[0], F[0], std::fma(o[1], F[1], o[2] * F[2])), std::fma(o[0], F[3], std::fma(o[1], F[4], o[2] * F[5])),
                                  std::fma(o[0], F[6], std::fma(o[1], F[7], o[2] * F[8])) };
            std::vector<uint32_t> stack { 0u };
            bool bvh = false;
            uint64_t nv = 0, nt = 0, md = 0;
            while (!stack.empty() && !bvh) {
                const GpuBvh8Node& nd = r.nodes[stack.back()];
                stack.pop_back();
                nv++;
                int F_[2], C_[3];
                float Q[3];
                for (int a = 0; a < 3; ++a) {
                    const float q = std::ldexp(pl[a] - nd.p[a], 127 - static_cast<int>(nd.e[a]));
                    Q[a] = std::min(258.0f, std::max(-2.0f, q));
                }
                F_[0] = static_cast<int>(std::floor(Q[0]));
                F_[1] = static_cast<int>(std::floor(Q[1]));
                for (int a = 0; a < 3; ++a) C_[a] = static_cast<int>(std::ceil(Q[a]));
                uint32_t internalBefore = 0;
                std::vector<uint32_t> push;
                for (int sl = 0; sl < 8; ++sl) {
                    const bool internal = (nd.imask >> sl) & 1u;
                    const bool hitc = nd.qlo[0][sl] <= F_[0] && nd.qhi[0][sl] >= C_[0] && nd.qlo[1][sl] <= F_[1] && nd.qhi[1][sl] >= C_[1] &&
                                      nd.qhi[2][sl] >= C_[2];
                    if (internal) {
                        if (hitc) push.push_back(nd.child_base + internalBefore);
                        internalBefore++;
                        continue;
                    }
                    if (!hitc || !((nd.leaf_mask >> sl) & 1u)) continue;
                    uint32_t st[kBvh8MaxLeafSize];
                    const int cnt = bvh8SlotTriangles(nd, sl, st);
                    for (int i = 0; i < cnt && !bvh; ++i) {
                        nt++;
                        bvh = mt(o, r.tris[st[i]]);
                    }
                }
                for (size_t i = push.size(); i-- > 0;) stack.push_back(push[i]);
                md = std::max<uint64_t>(md, stack.size());
            }
            occB += brute ? 1 : 0;
            occV += bvh ? 1 : 0;
            mism += brute != bvh ? 1 : 0;
            visits += nv;
            tests += nt;
            uint64_t m = maxDepth.load();
            while (md > m && !maxDepth.compare_exchange_weak(m, md)) {}
        }
    };
    const int T = 8;
    std::vector<std::thread> pool;
    for (int t = 0; t < T; ++t) pool.emplace_back(worker, n_rays * t / T, n_rays * (t + 1) / T);
    for (auto& th : pool) th.join();
    if (out) {
        out[0] = n_rays;
        out[1] = occB.load();
        out[2] = occV.load();
        out[3] = mism.load();
        out[4] = visits.load();
        out[5] = tests.load();
        out[6] = r.nodes.size();
        out[7] = maxDepth.load();
    }
    return mism.load() == 0 ? 0 : 2;
}


// ark_ddgi_debug.h: set_scene's choice between the light-space BVH and the world BVH
// for the sun's shadow rays, on a triangle soup (one hit-mask class).
extern "C" int ark_ddgi_debug_sun_choice(const float* triangles, uint64_t n, const float* sun_dir, uint32_t n_samples, double* out)
{
    using namespace ark;
    if (n == 0 || !out) return 1;
    std::vector<BuildTriangle> tris(n);
    for (uint64_t i = 0; i < n; ++i) {
        for (int a = 0; a < 3; ++a) {
            tris[i].v0[a] = triangles[9 * i + a];
            tris[i].v1[a] = triangles[9 * i + 3 + a];
            tris[i].v2[a] = triangles[9 * i + 6 + a];
        }
        tris[i].instance = 0;
        tris[i].primitive = static_cast<uint32_t>(i);
        tris[i].flip_facing = 0;
    }
    SunBvhInput in;
    sun_frame(sun_dir, in.frame);
    sun_add_triangles(in, tris);
    double frame[3][3];
    std::memcpy(frame, in.frame, sizeof(frame));
    BvhBuildOptions opt;
    opt.max_leaf_size = kBvh8MaxLeafSize;
    opt.inflate_abs = bvh8_inflation(triangles, n);
    opt.threads = 8;
    Bvh8CollapseOptions copt;
    const BvhBuildResult r2 = build_bvh(tris, opt, 0u, 0u);
    if (r2.max_leaf > static_cast<uint32_t>(kBvh8MaxLeafSize)) return 1;
    const Bvh8BuildResult w8 = collapse_bvh8(r2, 0u, 0u, copt);
    Bvh8BuildResult s8;
    if (!build_sun_bvh(in, opt, copt, s8)) return 1;
    const float dd = sun_dir[0] * sun_dir[0] + sun_dir[1] * sun_dir[1] + sun_dir[2] * sun_dir[2];
    const float sc = 1.0f / std::sqrt(dd);
    const float L[3] = { -(sun_dir[0] * sc), -(sun_dir[1] * sc), -(sun_dir[2] * sc) };
    std::vector<float> origins;
    sun_sample_origins(w8.tris, L, n_samples, origins);
    const int32_t root = 0;
    out[0] = sun_shadow_cost(w8.nodes, w8.tris, &root, 1, nullptr, L, origins);
    out[1] = sun_shadow_cost(s8.nodes, s8.tris, &root, 1, frame, L, origins);
    out[2] = sun_bvh_pays(out[0], out[1]) ? 1.0 : 0.0;
    out[3] = static_cast<double>(origins.size() / 3);
    return 0;
}
