// rt_layout.hpp — host side of rt_context_set_scene: the device layouts of the scene (grouped
// sphere records, filter streams, the k-d sweep layout with its box levels, group-local frames and
// the mega walk's tier table).  Host code only; included by rt_kernel.hip.
#pragma once
#include "rt_common.hpp"

using namespace rt;

// Grouped, padded sphere records (layout at SphGroup) + AoS centre table, in precision T.
template <typename T>
static void pack_scene(const rt_scene* s, std::vector<T>& grp, std::vector<T>& cen, std::vector<MatT<T>>& mats,
                       uint32_t& n_groups) {
    const uint32_t G = kGroup<T>;
    const uint32_t n = s->n_spheres;
    n_groups = (n + G - 1) / G;
    const uint32_t npad = n_groups * G;
    cen.assign((size_t)4 * (n ? n : 1), T(0));
    for (uint32_t i = 0; i < n; ++i) {
        const T r = (T)s->radius[i];
        cen[4 * i + 0] = (T)s->center[3 * i + 0];
        cen[4 * i + 1] = (T)s->center[3 * i + 1];
        cen[4 * i + 2] = (T)s->center[3 * i + 2];
        cen[4 * i + 3] = r;       // signed radius (scalar-mode normal, objects.rs:242)
    }
    auto field = [&](uint32_t i, int f) -> T {   // dummies: centre 0, r^2 = -inf (never hit)
        if (i >= n) return f == 3 ? -std::numeric_limits<T>::infinity() : T(0);
        return f == 3 ? cen[4 * i + 3] * cen[4 * i + 3] : cen[4 * i + f];   // r.powi(2) in T (objects.rs:256)
    };
    grp.assign((size_t)64 / sizeof(T) * (n_groups + 1), T(0));   // + 1 dummy group: prefetch target
    for (uint32_t i = 0; i < npad + G; ++i) {
        const uint32_t g = i / G, j = i % G;
        T* out = &grp[(size_t)g * (64 / sizeof(T))];
        for (int f = 0; f < 4; ++f) {
            if (sizeof(T) == 4) out[8 * (j / 2) + 2 * f + (j % 2)] = field(i, f);   // pair-interleaved
            else out[4 * j + f] = field(i, f);                                     // AoS
        }
    }
    mats.resize(s->n_materials ? s->n_materials : 1);
    for (uint32_t i = 0; i < s->n_materials; ++i) {
        const rt_material& m = s->materials[i];
        const T ior = (T)m.ior, one = T(1.0);
        const T inv = one / ior;
        const T qf = (one - inv) / (one + inv), qb = (one - ior) / (one + ior);
        if (m.kind == RT_DIELECTRIC) mats[i] = MatT<T>{m.kind, m.hollow, {ior, inv, qf * qf, qb * qb}};
        else mats[i] = MatT<T>{m.kind, m.hollow, {(T)m.albedo[0], (T)m.albedo[1], (T)m.albedo[2], (T)m.fuzz}};
    }
}

// Filter stream for rays in precision T (layout at SphGroup, fp32, 4 spheres per group): centres
// as the T kernel sees them, converted to fp32; r2f = the kernel's r^2 (r.powi(2) in T) rounded up
// to fp32; +inf for "always exact" spheres; -inf for dummies.  Returns the margin bounds over the
// other spheres: max |c|_1 (rounded up) and max r2f.
template <typename T>
static void pack_filter(const std::vector<T>& cen, uint32_t n, std::vector<float>& grp, uint32_t& n_fgroups,
                        float& cmax, float& r2max, float& r2min, std::vector<float>& frec) {
    n_fgroups = (n + 3) / 4;
    std::vector<double> key(n);
    for (uint32_t i = 0; i < n; ++i)
        key[i] = std::fabs((double)cen[4 * i]) + std::fabs((double)cen[4 * i + 1]) + std::fabs((double)cen[4 * i + 2]) +
                 std::fabs((double)cen[4 * i + 3]);
    double median = 0.0;
    if (n) {
        std::vector<double> k2 = key;
        std::nth_element(k2.begin(), k2.begin() + n / 2, k2.end());
        median = k2[n / 2];
    }
    auto up32 = [](double v) -> float {   // fp32 >= v
        float f = (float)v;
        if ((double)f < v) f = std::nextafter(f, std::numeric_limits<float>::infinity());
        return f;
    };
    // The kernel scales each lane's filter basis by 1/sqrt(1 + m/r2min), which inflates every r2f
    // by the factor (1 + m/r2min) >= 1 + m/r2f.  A floor on r2f (tiny spheres filtered as if of the
    // floor radius, conservative) keeps one tiny sphere from inflating all the others.
    double cm = 0.0, rm = 0.0;
    for (uint32_t i = 0; i < n; ++i) {
        const double c1 = std::fabs((double)(float)cen[4 * i]) + std::fabs((double)(float)cen[4 * i + 1]) +
                          std::fabs((double)(float)cen[4 * i + 2]);
        const double r2 = (double)(cen[4 * i + 3] * cen[4 * i + 3]);
        if (std::isfinite(key[i]) && std::isfinite(r2) && std::isfinite(c1) && !(key[i] > kExactRatio * median)) {
            cm = std::max(cm, c1);
            rm = std::max(rm, r2);
        }
    }
    const double floor2 = std::max(rm * 0x1.0p-10, cm * cm * 0x1.0p-16);
    double rmin = std::numeric_limits<double>::infinity();
    cm = 0.0; rm = 0.0;
    grp.assign((size_t)16 * (n_fgroups + 1), 0.0f);
    frec.assign((size_t)4 * n, 0.0f);
    for (uint32_t i = 0; i < 4 * (n_fgroups + 1); ++i) {
        float f[4] = {0.0f, 0.0f, 0.0f, -std::numeric_limits<float>::infinity()};
        if (i < n) {
            const T r2 = cen[4 * i + 3] * cen[4 * i + 3];   // as pack_scene: r.powi(2) in T
            f[0] = (float)cen[4 * i]; f[1] = (float)cen[4 * i + 1]; f[2] = (float)cen[4 * i + 2];
            const double c1 = std::fabs((double)f[0]) + std::fabs((double)f[1]) + std::fabs((double)f[2]);
            const bool finite = std::isfinite(key[i]) && std::isfinite((double)r2) && std::isfinite(c1);
            if (!finite || key[i] > kExactRatio * median) {
                f[3] = std::numeric_limits<float>::infinity();
            } else {
                f[3] = up32(std::max((double)r2, floor2));
                cm = std::max(cm, c1);
                rm = std::max(rm, (double)f[3]);
                rmin = std::min(rmin, (double)f[3]);
            }
        }
        const uint32_t g = i / 4, j = i % 4;
        for (int q = 0; q < 4; ++q) grp[(size_t)16 * g + 8 * (j / 2) + 2 * q + (j % 2)] = f[q];   // pair-interleaved
        if (i < n) for (int q = 0; q < 4; ++q) frec[(size_t)4 * i + q] = f[q];
    }
    cmax = up32(cm);
    r2max = up32(rm);
    r2min = std::isfinite(rmin) ? (float)rmin : 0.0f;   // exact: rmin is an fp32 value
}

// Spatial clusters for the general sweep's two-level filter (nearest_hit).  Slot order: first the
// "always exact" spheres (pack_filter's rule: non-finite, or |c|_1 + r above 8x the median, e.g. a
// ground sphere; and up to kBigExact spheres of more than kBigRatio x the median radius) in scene
// order, padded to whole groups -- every ray tests them exactly; then the
// filterable spheres, split k-d style (median along the longest extent of the centres) into
// clusters of at most kClusterMax = 16 spheres, each cluster in 4 whole groups (dummy-padded).  The
// cluster count is padded to whole top groups of 4 with empty clusters (never taken).  The sweep
// visits spheres in slot order, not scene order: hit_update's tie rule (equal t -> the later scene
// index wins; scalar mode: the earlier) makes the nearest hit independent of the visiting order.
constexpr uint32_t kClusterMax = 16;
constexpr double kBigRatio = 3.0;   // "big": radius above 3x the median radius of the filtered spheres
constexpr size_t kBigExact = 8;     // at most this many big spheres join the always-exact ones
struct SweepLayout {
    std::vector<int32_t> slot;                   // slot -> scene index, -1 = dummy (4 slots per group)
    std::vector<std::vector<uint32_t>> members;  // per cluster (count padded to a multiple of 4)
    uint32_t n_xg = 0;                           // leading groups of always-exact spheres
    uint32_t n_xs = 0;                           // always-exact spheres (slots 0 .. n_xs-1)
    bool giga = false;                           // splits aligned to gigas (1024 spheres) as well
};
static SweepLayout build_layout(const rt_scene* s) {
    const uint32_t n = s->n_spheres;
    std::vector<double> key(n);
    for (uint32_t i = 0; i < n; ++i)
        key[i] = std::fabs(s->center[3 * i]) + std::fabs(s->center[3 * i + 1]) + std::fabs(s->center[3 * i + 2]) +
                 std::fabs(s->radius[i]);
    double median = 0.0;
    if (n) {
        std::vector<double> k2 = key;
        std::nth_element(k2.begin(), k2.begin() + n / 2, k2.end());
        median = k2[n / 2];
    }
    std::vector<uint32_t> filt, exact;
    for (uint32_t i = 0; i < n; ++i) {
        const bool fin = std::isfinite(key[i]) && std::isfinite(s->radius[i] * s->radius[i]);
        (fin && !(key[i] > kExactRatio * median) ? filt : exact).push_back(i);
    }
    // A few spheres far larger than the typical one (RTIOW's three radius-1 spheres among radius-0.2
    // ones) are tested exactly by every ray too: in a cluster, one of them made its box 5x taller, and
    // every ray passing over the small spheres near it walked the cluster.  At most kBigExact of them
    // (more stay in clusters: exact tests for every ray would cost more).  Same-box C fp32 +5.1 %,
    // fp64 +5.4 %, B +4.1 %, E +3.1 % (profiles/r03/experiments/big_exact.txt).
    {
        std::vector<double> rr;
        for (uint32_t i : filt) rr.push_back(std::fabs(s->radius[i]));
        if (!rr.empty()) {
            std::nth_element(rr.begin(), rr.begin() + rr.size() / 2, rr.end());
            const double mr = rr[rr.size() / 2];
            std::vector<uint32_t> keep, big;
            for (uint32_t i : filt) (std::fabs(s->radius[i]) > kBigRatio * mr ? big : keep).push_back(i);
            if (!big.empty() && big.size() <= kBigExact) {
                filt.swap(keep);
                exact.insert(exact.end(), big.begin(), big.end());
                std::sort(exact.begin(), exact.end());
            }
        }
    }
    SweepLayout L;
    for (uint32_t i : exact) L.slot.push_back((int32_t)i);
    L.n_xs = (uint32_t)exact.size();
    while (L.slot.size() % 4) L.slot.push_back(-1);
    L.n_xg = (uint32_t)(L.slot.size() / 4);
    // k-d split (median along the longest extent of the centres), aligned to the box hierarchy above
    // the clusters: a node of more than 256 spheres (4 supers = one mega) gives its left part a
    // multiple of 256, a node of 65..256 a multiple of 64 (one super), smaller nodes a multiple of 16,
    // and each child's clusters are padded with empty ones to a whole number of its parent's unit
    // (the next sibling then starts on a super / mega boundary).  So every super box and mega box
    // bounds one k-d subtree.  Round 2 split at multiples of 16 only:
    // at config E (10 000 spheres, a 313-cluster left half) every super and mega on the right of a
    // split took clusters of two subtrees, and their boxes spanned both.
    auto build = [&](auto&& self, size_t b, size_t e, size_t pad) -> void {   // pad: clusters per block
        const size_t N = e - b, c0 = L.members.size();
        if (N <= kClusterMax) {
            if (e > b) L.members.emplace_back(filt.begin() + b, filt.begin() + e);
            while ((L.members.size() - c0) % pad) L.members.emplace_back();
            return;
        }
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t k = b; k < e; ++k)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], s->center[3 * filt[k] + a]);
                hi[a] = std::max(hi[a], s->center[3 * filt[k] + a]);
            }
        int ax = 0;
        for (int a = 1; a < 3; ++a) if (hi[a] - lo[a] > hi[ax] - lo[ax]) ax = a;
        const size_t unit = L.giga && N > 64 * kClusterMax ? 64 * kClusterMax : N > 16 * kClusterMax ? 16 * kClusterMax
                          : N > 4 * kClusterMax ? 4 * kClusterMax : kClusterMax;
        const size_t m = b + std::min(N - 1, (N + 2 * unit - 1) / (2 * unit) * unit);
        std::nth_element(filt.begin() + b, filt.begin() + m, filt.begin() + e, [&](uint32_t x, uint32_t y) {
            const double cx = s->center[3 * x + ax], cy = s->center[3 * y + ax];
            return cx < cy || (cx == cy && x < y);
        });
        self(self, b, m, unit / kClusterMax);
        self(self, m, e, unit / kClusterMax);
        while ((L.members.size() - c0) % pad) L.members.emplace_back();
    };
    L.giga = filt.size() > 128 * kClusterMax;   // the mega kernels' scenes (more than 8 super groups)
    build(build, 0, filt.size(), 1);
    while (L.members.size() % 4) L.members.emplace_back();
    // Members ordered by k-d halving (16 -> 8|8 -> 4|4 -> 2|2), so each filter group and each exact pair
    // holds neighbours: a lane's passes concentrate in fewer groups and pairs.  Scene-index order (round
    // 2) grouped spheres along the generator's loop.  Same-box C fp32 +0.5 %, fp64 +0.7 %, E +0.4 %.
    auto kd_order = [&](auto&& self, std::vector<uint32_t>& v, size_t b, size_t e) -> void {
        if (e - b <= 2) return;
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t k = b; k < e; ++k)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], s->center[3 * v[k] + a]);
                hi[a] = std::max(hi[a], s->center[3 * v[k] + a]);
            }
        int ax = 0;
        for (int a = 1; a < 3; ++a) if (hi[a] - lo[a] > hi[ax] - lo[ax]) ax = a;
        size_t half = 1;
        while (2 * half < e - b) half *= 2;   // power-of-two left part: groups of 4 stay whole
        const size_t m = b + half;
        std::nth_element(v.begin() + b, v.begin() + m, v.begin() + e, [&](uint32_t x, uint32_t y) {
            const double cx = s->center[3 * x + ax], cy = s->center[3 * y + ax];
            return cx < cy || (cx == cy && x < y);
        });
        self(self, v, b, m);
        self(self, v, m, e);
    };
    for (auto& c : L.members) {
        std::sort(c.begin(), c.end());
        kd_order(kd_order, c, 0, c.size());
        for (uint32_t k = 0; k < kClusterMax; ++k) L.slot.push_back(k < c.size() ? (int32_t)c[k] : -1);
    }
    return L;
}

// Slot-order streams for rays in precision T: the exact groups (SphGroup layout of pack_scene),
// the fp32 filter groups (pack_filter's records) and the top stream of cluster bounds: axis-aligned
// boxes {centre C, half-extent h} in fp32, 4 per 96-byte group (BoxGroup), enclosing every member
// with its filter radius sqrt(r2f) (so the floor applies: h >= sqrt(r2min) on every axis), h rounded
// up and widened by 2^-20 relative and 4 u |C| for the fp32 rounding of C; h = +inf if a member is
// always exact in T, -inf for an empty cluster.  |C|_1 + |h|_1 enters the margin bound cmax.
template <typename T>
static void pack_sweep(const std::vector<T>& cen, const std::vector<float>& frec, const SweepLayout& L,
                       std::vector<T>& rgrp, std::vector<float>& rfgrp, std::vector<float>& top, float& cmax,
                       float& r2max, std::vector<float>& sup, std::vector<float>& meg) {
    auto up32 = [](double v) -> float {
        float f = (float)v;
        if ((double)f < v) f = std::nextafter(f, std::numeric_limits<float>::infinity());
        return f;
    };
    const size_t ns = L.slot.size(), nfg = ns / 4;
    constexpr uint32_t G = kGroup<T>, NE = 64 / sizeof(T);
    rgrp.assign((size_t)NE * (ns / G + 1), T(0));
    rfgrp.assign((size_t)16 * (nfg + 1), 0.0f);
    for (size_t i = 0; i < ns + G; ++i) {   // exact groups, + one dummy group
        const int32_t sc = i < ns ? L.slot[i] : -1;
        const size_t g = i / G, j = i % G;
        for (int f = 0; f < 4; ++f) {
            T v = f == 3 ? -std::numeric_limits<T>::infinity() : T(0);
            if (sc >= 0) v = f == 3 ? cen[4 * sc + 3] * cen[4 * sc + 3] : cen[4 * sc + f];   // r.powi(2) in T
            if (sizeof(T) == 4) rgrp[g * NE + 8 * (j / 2) + 2 * f + (j % 2)] = v;
            else rgrp[g * NE + 4 * j + f] = v;
        }
    }
    for (size_t i = 0; i < ns + 4; ++i) {   // filter groups, + one dummy group (prefetch target)
        const int32_t sc = i < ns ? L.slot[i] : -1;
        for (int f = 0; f < 4; ++f) {
            const float fv = sc >= 0 ? frec[(size_t)4 * sc + f] : (f == 3 ? -INFINITY : 0.0f);
            rfgrp[(size_t)16 * (i / 4) + 8 * ((i % 4) / 2) + 2 * f + (i % 2)] = fv;
        }
    }
    const size_t nc = L.members.size();
    top.assign((size_t)kBoxFloats / 4 * (nc + 4), 0.0f);   // + one empty top group (prefetch target)
    double cm = cmax;
    for (size_t k = 0; k < nc + 4; ++k) {
        float b[6] = {0.0f, 0.0f, 0.0f, -INFINITY, -INFINITY, -INFINITY};   // empty: never passes
        if (k < nc && !L.members[k].empty()) {
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            bool inf = false;
            for (uint32_t i : L.members[k]) {
                const double r = std::sqrt((double)frec[4 * i + 3]);   // the filter's (floored) radius
                if (!(frec[4 * i + 3] < INFINITY)) inf = true;
                for (int a = 0; a < 3; ++a) {
                    lo[a] = std::min(lo[a], (double)frec[4 * i + a] - r);
                    hi[a] = std::max(hi[a], (double)frec[4 * i + a] + r);
                }
            }
            double c1 = 0.0;
            for (int a = 0; a < 3; ++a) {
                b[a] = (float)(0.5 * (lo[a] + hi[a]));
                const double h = std::max(hi[a] - (double)b[a], (double)b[a] - lo[a]);
                b[3 + a] = inf ? INFINITY : up32(h * (1.0 + 0x1.0p-20) + 0x1.0p-22 * std::fabs((double)b[a]));
                c1 += std::fabs((double)b[a]) + (double)b[3 + a];
            }
            if (!inf) cm = std::max(cm, c1);
        }
        // pair-interleaved: pair q of a group at 12 q, {cx0,cx1, cy0,cy1, cz0,cz1, hx0,hx1, hy0,hy1, hz0,hz1}
        const size_t tg = k / 4, j = k % 4;
        for (int f = 0; f < 6; ++f) top[kBoxFloats * tg + 12 * (j / 2) + 2 * f + (j % 2)] = b[f];
    }
    // Super boxes: the union of the 4 cluster boxes of each top group, same rounding; 4 per group,
    // padded with empty boxes plus one empty group (prefetch target).  Mega boxes likewise over the
    // 4 supers of each super group, when there are more than 8 super groups (one sweep chunk).
    auto unite = [&](const std::vector<float>& lower, size_t nup, std::vector<float>& upper) {
        const size_t ng = (nup + 3) / 4;
        upper.assign((size_t)kBoxFloats * (ng + 1), 0.0f);
        for (size_t k = 0; k < 4 * (ng + 1); ++k) {
            float b[6] = {0.0f, 0.0f, 0.0f, -INFINITY, -INFINITY, -INFINITY};
            if (k < nup) {
                double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
                bool inf = false, any = false;
                for (size_t j = 0; j < 4; ++j) {
                    const float* t = &lower[kBoxFloats * k + 12 * (j / 2) + (j % 2)];
                    if (!(t[6] > -INFINITY)) continue;   // empty box
                    any = true;
                    for (int a = 0; a < 3; ++a) {
                        if (!(t[6 + 2 * a] < INFINITY)) inf = true;
                        lo[a] = std::min(lo[a], (double)t[2 * a] - (double)t[6 + 2 * a]);
                        hi[a] = std::max(hi[a], (double)t[2 * a] + (double)t[6 + 2 * a]);
                    }
                }
                if (any) {
                    double c1 = 0.0;
                    for (int a = 0; a < 3; ++a) {
                        b[a] = inf ? 0.0f : (float)(0.5 * (lo[a] + hi[a]));
                        const double h = std::max(hi[a] - (double)b[a], (double)b[a] - lo[a]);
                        b[3 + a] = inf ? INFINITY : up32(h * (1.0 + 0x1.0p-20) + 0x1.0p-22 * std::fabs((double)b[a]));
                        c1 += std::fabs((double)b[a]) + (double)b[3 + a];
                    }
                    if (!inf) cm = std::max(cm, c1);
                }
            }
            const size_t tg = k / 4, j = k % 4;
            for (int f = 0; f < 6; ++f) upper[kBoxFloats * tg + 12 * (j / 2) + 2 * f + (j % 2)] = b[f];
        }
    };
    const size_t nsup = nc / 4, nsg = (nsup + 3) / 4;
    unite(top, nsup, sup);
    if (nsg > 8) unite(sup, nsg, meg);
    else meg.clear();
    cmax = up32(cm);
    (void)r2max;
}

// Cluster-local filter records for the MEGA kernels (nearest_hit).  Far from the origin the scene-wide
// margin of the sphere filter, 48 u ((max|c|_1 + |o|_1)^2 + max r2f), grows with the coordinates'
// magnitudes (config E: ~0.06 against r^2 = 0.04), though the rounding it covers grows with the
// distances involved.  In a frame centred on the cluster (C_k: its box centre, an fp32 value) the
// filter sees c' = RN_f(c - C_k) and o' = o - C_k, and the same margin formula with |c'|_1 <= Rc_k and
// |o'|_1 in place of the scene-wide magnitudes bounds the same errors (tests/filter_margin_fuzz.c,
// local mode).  r2f is floored per cluster at 2^-10 of its largest (a tiny sphere cannot inflate the
// others by more than that ratio).  Slot order and group layout as the scene-wide filter stream;
// always-exact slots get dummies (they are never filtered).
template <typename T>
static void pack_local(const std::vector<T>& cen, const SweepLayout& L, const std::vector<float>& top,
                       std::vector<float>& lfgrp, std::vector<float>& lrec, std::vector<float>& r2l) {
    auto up32 = [](double v) -> float {
        float f = (float)v;
        if ((double)f < v) f = std::nextafter(f, std::numeric_limits<float>::infinity());
        return f;
    };
    const size_t ns = L.slot.size(), nc = L.members.size();
    lfgrp.assign((size_t)16 * (ns / 4 + 1), 0.0f);
    for (size_t i = 0; i < ns + 4; ++i) lfgrp[(size_t)16 * (i / 4) + 8 * ((i % 4) / 2) + 6 + (i % 2)] = -INFINITY;
    lrec.assign((size_t)8 * (nc ? nc : 1), 0.0f);
    for (size_t k = 0; k < nc; ++k) {
        const auto& m = L.members[k];
        if (m.empty()) continue;
        float Ck[3];
        for (int f = 0; f < 3; ++f) Ck[f] = top[kBoxFloats * (k / 4) + 12 * ((k % 4) / 2) + 2 * f + (k % 2)];
        double r2max = 0.0, rc = 0.0;
        for (uint32_t i : m) r2max = std::max(r2max, (double)(cen[4 * i + 3] * cen[4 * i + 3]));   // r.powi(2) in T
        const double floor2 = r2max * 0x1.0p-10;
        double r2min = INFINITY, r2fmax = 0.0;
        for (uint32_t j = 0; j < m.size(); ++j) {
            const uint32_t i = m[j];
            const size_t slot = (size_t)4 * L.n_xg + kClusterMax * k + j;   // members in cluster-slot order
            float f[4];
            for (int a = 0; a < 3; ++a) f[a] = (float)((double)cen[4 * i + a] - (double)Ck[a]);   // RN_f(c - C_k)
            const T r2 = cen[4 * i + 3] * cen[4 * i + 3];
            f[3] = up32(std::max((double)r2, floor2));
            if (r2l.size() <= i) r2l.resize((size_t)i + 1, -INFINITY);
            r2l[i] = f[3];
            rc = std::max(rc, std::fabs((double)f[0]) + std::fabs((double)f[1]) + std::fabs((double)f[2]));
            r2min = std::min(r2min, (double)f[3]);
            r2fmax = std::max(r2fmax, (double)f[3]);
            for (int q = 0; q < 4; ++q) lfgrp[(size_t)16 * (slot / 4) + 8 * ((slot % 4) / 2) + 2 * q + (slot % 2)] = f[q];
        }
        float* r = &lrec[8 * k];
        r[0] = Ck[0]; r[1] = Ck[1]; r[2] = Ck[2];
        r[3] = up32(rc);
        r[4] = up32(r2fmax);
        r[5] = up32(1.0 / r2min);
    }
}

// The MEGA kernels' box levels in group-local frames.  World boxes as pack_sweep builds them, but
// around the spheres' locally floored radii (pack_local's r2f), so a far-from-origin scene keeps its
// boxes tight: clusters, their union per super, the supers' union per mega.  Every box group is then
// stored around its own frame S (the fp32 centre of its boxes' union): 24 floats of boxes with
// C' = RN_f(C - S) and H widened by 2^-22 |C'|, then {S, Rg = max |C'|_1 + |H'|_1} (LBoxGroup); the
// lane tests it with o' = o - S and the margin from |o'|_1 + Rg (nearest_hit; tests/box_cull_fuzz.c,
// local mode).  One empty group past the end of each level (prefetch target).
constexpr uint32_t kLBoxFloats = 32;
template <typename T>
static void pack_local_boxes(const std::vector<T>& cen, const SweepLayout& L, const std::vector<float>& r2l,
                             std::vector<float>& lclb, std::vector<float>& lsup, std::vector<float>& lmeg,
                             std::vector<float>& lgig, float& r2max, float& r2min, std::vector<float>* wmeg = nullptr) {
    auto up32 = [](double v) -> float {
        float f = (float)v;
        if ((double)f < v) f = std::nextafter(f, std::numeric_limits<float>::infinity());
        return f;
    };
    const size_t nc = L.members.size();
    // world boxes, BoxGroup layout (4 per 24 floats), like pack_sweep's, around sqrt(local r2f)
    auto put = [](std::vector<float>& v, size_t k, const float b[6]) {
        const size_t tg = k / 4, j = k % 4;
        for (int f = 0; f < 6; ++f) v[kBoxFloats * tg + 12 * (j / 2) + 2 * f + (j % 2)] = b[f];
    };
    auto get = [](const std::vector<float>& v, size_t k, float b[6]) {
        const size_t tg = k / 4, j = k % 4;
        for (int f = 0; f < 6; ++f) b[f] = v[kBoxFloats * tg + 12 * (j / 2) + 2 * f + (j % 2)];
    };
    auto box_of = [&](double lo[3], double hi[3], bool inf, float b[6]) {
        for (int a = 0; a < 3; ++a) {
            b[a] = inf ? 0.0f : (float)(0.5 * (lo[a] + hi[a]));
            const double h = std::max(hi[a] - (double)b[a], (double)b[a] - lo[a]);
            b[3 + a] = inf ? INFINITY : up32(h * (1.0 + 0x1.0p-20) + 0x1.0p-22 * std::fabs((double)b[a]));
        }
    };
    const float kEmpty[6] = {0.0f, 0.0f, 0.0f, -INFINITY, -INFINITY, -INFINITY};
    std::vector<float> wcl((size_t)kBoxFloats * ((nc + 3) / 4 + 1));
    for (size_t k = 0; k < 4 * (wcl.size() / kBoxFloats); ++k) put(wcl, k, kEmpty);
    double rmax = 0.0, rmin = INFINITY;
    for (size_t k = 0; k < nc; ++k) {
        if (L.members[k].empty()) continue;
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        bool inf = false;
        for (uint32_t i : L.members[k]) {
            if (!(r2l[i] < INFINITY)) inf = true;
            rmax = std::max(rmax, (double)r2l[i]);
            rmin = std::min(rmin, (double)r2l[i]);
            const double r = std::sqrt((double)r2l[i]);
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], (double)(float)cen[4 * i + a] - r);
                hi[a] = std::max(hi[a], (double)(float)cen[4 * i + a] + r);
            }
        }
        float b[6];
        box_of(lo, hi, inf, b);
        put(wcl, k, b);
    }
    r2max = up32(rmax);
    r2min = std::isfinite(rmin) ? (float)rmin : 0.0f;
    auto unite = [&](const std::vector<float>& lower, size_t nup, std::vector<float>& upper) {
        upper.assign((size_t)kBoxFloats * ((nup + 3) / 4 + 1), 0.0f);
        for (size_t k = 0; k < 4 * (upper.size() / kBoxFloats); ++k) put(upper, k, kEmpty);
        for (size_t k = 0; k < nup; ++k) {
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            bool inf = false, any = false;
            for (size_t j = 0; j < 4; ++j) {
                float t[6];
                get(lower, 4 * k + j, t);
                if (!(t[3] > -INFINITY)) continue;
                any = true;
                for (int a = 0; a < 3; ++a) {
                    if (!(t[3 + a] < INFINITY)) inf = true;
                    lo[a] = std::min(lo[a], (double)t[a] - (double)t[3 + a]);
                    hi[a] = std::max(hi[a], (double)t[a] + (double)t[3 + a]);
                }
            }
            if (!any) continue;
            float b[6];
            box_of(lo, hi, inf, b);
            put(upper, k, b);
        }
    };
    const size_t nsup = nc / 4, nsg = (nsup + 3) / 4;
    std::vector<float> wsu, wme;
    unite(wcl, nsup, wsu);
    unite(wsu, nsg, wme);
    if (wmeg) *wmeg = wme;
    // group-local frames: group g of `world` (4 boxes) -> LBoxGroup g
    auto localise = [&](const std::vector<float>& world, size_t ng, std::vector<float>& out) {
        out.assign((size_t)kLBoxFloats * (ng + 1), 0.0f);
        for (size_t g = 0; g < ng + 1; ++g) {
            float* o = &out[kLBoxFloats * g];
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            bool any = false, inf = false;
            float bx[4][6];
            for (size_t j = 0; j < 4; ++j) {
                if (g < ng) get(world, 4 * g + j, bx[j]);
                else for (int f = 0; f < 6; ++f) bx[j][f] = kEmpty[f];
                if (!(bx[j][3] > -INFINITY)) continue;
                any = true;
                for (int a = 0; a < 3; ++a) {
                    if (!(bx[j][3 + a] < INFINITY)) { inf = true; continue; }
                    lo[a] = std::min(lo[a], (double)bx[j][a] - (double)bx[j][3 + a]);
                    hi[a] = std::max(hi[a], (double)bx[j][a] + (double)bx[j][3 + a]);
                }
            }
            float Sg[3] = {0.0f, 0.0f, 0.0f};
            if (any && !inf)
                for (int a = 0; a < 3; ++a) Sg[a] = (float)(0.5 * (lo[a] + hi[a]));
            double rg = 0.0;
            for (size_t j = 0; j < 4; ++j) {
                float b[6];
                for (int f = 0; f < 6; ++f) b[f] = bx[j][f];
                if (b[3] > -INFINITY) {
                    for (int a = 0; a < 3; ++a) {
                        const float cl = (float)((double)b[a] - (double)Sg[a]);   // RN_f(C - S)
                        b[3 + a] = b[3 + a] < INFINITY ? up32((double)b[3 + a] + 0x1.0p-22 * std::fabs((double)cl)) : INFINITY;
                        b[a] = b[3 + a] < INFINITY ? cl : 0.0f;
                    }
                    rg = std::max(rg, std::fabs((double)b[0]) + std::fabs((double)b[1]) + std::fabs((double)b[2]) +
                                          (double)b[3] + (double)b[4] + (double)b[5]);
                }
                for (int f = 0; f < 6; ++f) o[12 * (j / 2) + 2 * f + (j % 2)] = b[f];
            }
            o[24] = Sg[0]; o[25] = Sg[1]; o[26] = Sg[2];
            o[27] = std::isfinite(rg) ? up32(rg) : INFINITY;
        }
    };
    localise(wcl, (nc + 3) / 4, lclb);
    localise(wsu, nsg, lsup);
    localise(wme, (nsg + 3) / 4, lmeg);
    // gigas: the union of each mega group's 4 megas (build_layout aligns them to k-d subtrees in scenes
    // of more than 2048 filtered spheres)
    const size_t nmg = (nsg + 3) / 4;
    std::vector<float> wgi;
    unite(wme, nmg, wgi);
    localise(wgi, (nmg + 3) / 4, lgig);
}

// The mega walk's order table (nearest_hit, MEGA): a grid of cubic cells (<= 4096, <= 64 per axis)
// over the union of the mega boxes (world frame, BoxGroup layout); per cell four u64 masks over the
// megas (<= 64): those whose box touches the cell, those within a quarter and within a half of the
// median mega size, and 0 (nested, so the walk's tiers partition the passing megas; the kernel's
// default uses the first two).  A heuristic:
// the order changes which boxes get culled early, never the hits.
struct MegaTiers { std::vector<uint64_t> t; float lo[3] = {0, 0, 0}, inv = 0; uint32_t n[3] = {1, 1, 1}; };
static MegaTiers pack_mega_tiers(const std::vector<float>& wme, size_t nm) {
    MegaTiers M;
    M.t.assign(4, 0ull);
    if (nm == 0 || nm > 64) return M;
    std::vector<std::array<double, 6>> bx;
    std::vector<size_t> id;
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    std::vector<double> size;
    for (size_t k = 0; k < nm; ++k) {
        std::array<double, 6> b;
        for (int f = 0; f < 6; ++f) b[f] = wme[kBoxFloats * (k / 4) + 12 * ((k % 4) / 2) + 2 * f + (k % 2)];
        if (!(b[3] > -INFINITY) || !std::isfinite(b[3] + b[4] + b[5] + b[0] + b[1] + b[2])) continue;
        bx.push_back(b);
        id.push_back(k);
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], b[a] - b[3 + a]);
            hi[a] = std::max(hi[a], b[a] + b[3 + a]);
        }
        size.push_back(2.0 * std::max(b[3], std::max(b[4], b[5])));
    }
    if (bx.empty()) return M;
    std::nth_element(size.begin(), size.begin() + size.size() / 2, size.end());
    const double L = size[size.size() / 2];
    double ext = 0.0;
    for (int a = 0; a < 3; ++a) ext = std::max(ext, hi[a] - lo[a]);
    double cs = ext > 0.0 ? ext / 64.0 : 1.0;
    for (;;) {
        uint64_t prod = 1;
        for (int a = 0; a < 3; ++a) {
            M.n[a] = (uint32_t)std::min(64.0, std::max(1.0, std::ceil((hi[a] - lo[a]) / cs)));
            prod *= M.n[a];
        }
        if (prod <= 4096) break;
        cs *= 1.25;
    }
    for (int a = 0; a < 3; ++a) M.lo[a] = (float)lo[a];
    M.inv = (float)(1.0 / cs);
    M.t.assign((size_t)4 * M.n[0] * M.n[1] * M.n[2], 0ull);
    for (uint32_t z = 0; z < M.n[2]; ++z)
        for (uint32_t y = 0; y < M.n[1]; ++y)
            for (uint32_t x = 0; x < M.n[0]; ++x) {
                const double cc[3] = {lo[0] + (x + 0.5) * cs, lo[1] + (y + 0.5) * cs, lo[2] + (z + 0.5) * cs};
                uint64_t* t = &M.t[(size_t)4 * (x + M.n[0] * (y + M.n[1] * z))];
                for (size_t j = 0; j < bx.size(); ++j) {
                    double d2 = 0.0;
                    for (int a = 0; a < 3; ++a) {
                        const double g = std::max(0.0, std::fabs(cc[a] - bx[j][a]) - (0.5 * cs + bx[j][3 + a]));
                        d2 += g * g;
                    }
                    const double d = std::sqrt(d2);
                    const uint64_t bit = 1ull << id[j];
                    if (d <= 0.0) t[0] |= bit;
                    if (d <= 0.25 * L) t[1] |= bit;
                    if (d <= 0.5 * L) t[2] |= bit;
                }
            }
    return M;
}
