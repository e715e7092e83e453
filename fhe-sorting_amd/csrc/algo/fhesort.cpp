// Rank-sort comparator hot path on the MI355X engine (see fhesort.hpp).
//
// The operation sequences here are the spec that the CPU
// oracle restates; GPU results are bit-identical to it.  Reference call sites
// replaced (file:line in oksuman/FHE-Sorting):
//   src/sign.cpp:9-60 (g_3/f_3), :62-158 (g_4/f_4), :160-185 (compositeSign),
//   :635-651 (sign); src/comparison.cpp:4-40; src/rotation.h:54-233;
//   src/sort_algo.h:326-366 (vecRotsOpt), :368-506 (constructRank),
//   :561-584 (blindRotationOptN), :658-750 (rotationIndexCheckN), :752-774.
#include "fhesort.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <fstream>
#include <map>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <tuple>
#include <exception>
#include <thread>

namespace fhe {

// ===================================================== Chebyshev (PS) ======
namespace {

int ceil_log2(long x) {
    int r = 0;
    while ((1L << r) < x) ++r;
    return r;
}
void trim_zeros(std::vector<double> &a) {
    while (a.size() > 1 && a.back() == 0.0) a.pop_back();
}
// leaves per linear-sum pass: every leaf of a pass shares one read of the baby
// steps (dev::LEAF_G = 32 per leaf-sum launch; FHE_PS_CHUNK for A/B timing,
// 16 = the round-4 passes: sort 543.1 / 546.8 -> 538.2 / 537.9 ms with the window
// kernel, profiles/r5_o; with the folded kernel 536.3 -> 523.2, profiles/r5_p)
size_t ps_chunk() {
    static const size_t v = [] {
        const char *e = std::getenv("FHE_PS_CHUNK");
        const int c = e ? std::atoi(e) : 32;
        return (size_t)std::min(32, std::max(1, c));
    }();
    return v;
}

// Levels OpenFHE's EvalChebyshevSeriesPS consumes for a degree-d series: the
// reference's multDepth tables (src/sort_algo.h:87-201) budget these, and its
// tests assert the output level (tests/DirectSortTest.cpp:128).  Degrees < 5
// go through EvalChebyshevSeriesLinear (T_1..T_d, then one constant product);
// up to 2204 OpenFHE picks (k, m) from a fixed table whose depth bands are the
// published ones below; above, ComputeDegreesPS's heuristic: minimise
// k + 2m + 2^(m-1) - 4 over k*(2^m - 1) > d with floor(log2 k) within 1 of
// floor(log2 sqrt(d/2)); depth ceil(log2 k) + m.  The evaluation itself stays
// depth-optimal; a series whose optimal depth is below this one is evaluated
// to the lower output level (its leaves absorb the extra rescale).
int openfhe_ps_depth(int d) {
    if (d < 5) return ceil_log2(d) + 1;
    static const int band_top[] = {5, 13, 27, 59, 119, 247, 495, 1007, 2031, 2204};
    for (int i = 0; i < 10; ++i)
        if (d <= band_top[i]) return 3 + i;
    const double f = std::floor(std::log2(std::sqrt(d / 2.0)));
    long best = -1;
    int depth = 0;
    for (long k = 1; k <= d; ++k) {
        if (std::fabs(std::floor(std::log2((double)k)) - f) > 1) continue;
        const int mmax = (int)std::ceil(std::log2((double)d / k) + 1) + 1;
        for (int m = 1; m <= mmax; ++m)
            if ((long)d - k * ((1L << m) - 1) < 0) {
                const long mult = k + 2 * m + (1L << (m - 1)) - 4;
                if (best < 0 || mult < best) {
                    best = mult;
                    depth = ceil_log2(k) + m;
                }
            }
    }
    return depth;
}

// Leaves are sum_{i<=B} a_i T_i (depth log2(B)+1); a node p = q T_G + r with
// G a power of two; capacity at depth D is 2^D - B, so a degree-d series
// costs ceil(log2(d+1)) levels.
struct PSEval {
    Engine &cc;
    int B = 1, beta = 1, D = 1;
    std::map<int, CtPtr> T;

    PSEval(Engine &c, const Ciphertext &x, int d) : cc(c) {
        D = std::max(1, ceil_log2((long)d + 1));
        const long bmax = (1L << D) - d;
        const double lim = std::sqrt(2.0 * d);
        long b = 1;
        while (b * 2 <= bmax && (double)(b * 2) <= lim) b *= 2;
        B = (int)b;
        beta = ceil_log2(B) + 1;
        T[1] = cc.clone(x);
    }
    void build_baby() {
        for (int i = 2; i <= B; ++i) {
            const int a = 1 << (ceil_log2(i) - 1), b = i - a;
            CtPtr t = (a == b) ? cc.square(*T[a]) : cc.mul(*T[a], *T[b]);
            t = cc.add(*t, *t);
            if (a == b)
                cc.add_const_inplace(t, -1.0);
            else
                t = cc.sub(*t, *T[a - b]);
            T[i] = t;
        }
    }
    const Ciphertext &giant(int G) {
        auto it = T.find(G);
        if (it != T.end()) return *it->second;
        const Ciphertext &h = giant(G / 2);
        CtPtr t = cc.square(h);
        t = cc.add(*t, *t);
        cc.add_const_inplace(t, -1.0);
        T[G] = t;
        return *T[G];
    }
    // ---- leaves.  The recursion below consumes leaves in a fixed order; they
    // are collected first, and leaves sharing a target level are evaluated
    // up to 8 at a time by one multi-output linear sum over the baby steps
    // (each baby step is streamed once per 8 leaves).  Every leaf equals
    // linear_sum_to(its nonzero terms) + a_0, word for word.
    struct Leaf {
        std::vector<double> a;
        int target;
        bool raw;  // folded remainder: the un-rescaled sum feeds mul_add_raw
    };
    std::vector<Leaf> leaves;
    std::map<size_t, CtPtr> ready;
    size_t next_leaf = 0;

    void split(const std::vector<double> &a, int d, std::vector<double> &q, std::vector<double> &r, int &G) const {
        int Dpp = beta + 1;
        while ((1L << Dpp) - B < d) ++Dpp;
        G = 1 << (Dpp - 1);
        while (G > d) G >>= 1;
        q.assign(d - G + 1, 0.0);
        r.assign(a.begin(), a.begin() + G);
        q[0] = a[G];
        for (int j = 1; j <= d - G; ++j) {
            q[j] = 2.0 * a[G + j];
            r[G - j] -= a[G + j];
        }
    }
    void collect(std::vector<double> a, int target) {
        trim_zeros(a);
        const int d = (int)a.size() - 1;
        if (d <= B) {
            leaves.push_back({a, target, false});
            return;
        }
        std::vector<double> q, r;
        int G;
        split(a, d, q, r, G);
        collect(q, target - 1);
        trim_zeros(r);
        if (r.size() == 1 && r[0] == 0.0) return;
        if (folded(r)) {  // summed into the product before its rescale (eval)
            leaves.push_back({r, target, true});
            return;
        }
        collect(r, target);
    }
    // a remainder that is a leaf with terms is added before the product's
    // rescale (mul_add) instead of being evaluated on its own
    bool folded(const std::vector<double> &r) const {
        const int dr = (int)r.size() - 1;
        return dr >= 1 && dr <= B;
    }
    static bool has_terms(const std::vector<double> &a) {
        for (size_t i = 1; i < a.size(); ++i)
            if (a[i] != 0.0) return true;
        return false;
    }
    void evaluate_chunk(size_t first) {
        const int target = leaves[first].target;
        const bool raw = leaves[first].raw;
        // up to ps_chunk() leaves per linear-sum pass (one read of the baby steps
        // for all of them)
        const size_t max_chunk = ps_chunk();
        std::vector<size_t> chunk;
        for (size_t i = first; i < leaves.size() && chunk.size() < max_chunk; ++i)
            if (leaves[i].target == target && leaves[i].raw == raw && !ready.count(i) && has_terms(leaves[i].a))
                chunk.push_back(i);
        std::vector<int> idx;  // union of the baby steps the chunk uses
        for (size_t c : chunk)
            for (size_t i = 1; i < leaves[c].a.size(); ++i)
                if (leaves[c].a[i] != 0.0) idx.push_back((int)i);
        std::sort(idx.begin(), idx.end());
        idx.erase(std::unique(idx.begin(), idx.end()), idx.end());
        std::vector<const Ciphertext *> xs;
        for (int i : idx) xs.push_back(T.at(i).get());
        std::vector<std::vector<double>> rows;
        for (size_t c : chunk) {
            std::vector<double> row;
            for (int i : idx) row.push_back((size_t)i < leaves[c].a.size() ? leaves[c].a[i] : 0.0);
            rows.push_back(row);
        }
        auto outs = cc.linear_sums_to(xs, rows, target, !raw);
        for (size_t g = 0; g < chunk.size(); ++g) {
            CtPtr r = std::move(outs[g]);
            if (!raw && leaves[chunk[g]].a[0] != 0.0) cc.add_const_inplace(r, leaves[chunk[g]].a[0]);
            ready[chunk[g]] = r;
        }
    }
    CtPtr leaf() {
        const size_t i = next_leaf++;
        const Leaf &L = leaves.at(i);
        if (!has_terms(L.a)) {
            CtPtr r = cc.trivial_const(0.0, L.target, T[1]->slots, T[1]->batch);
            if (L.a[0] != 0.0) cc.add_const_inplace(r, L.a[0]);
            return r;
        }
        if (!ready.count(i)) evaluate_chunk(i);
        CtPtr r = ready.at(i);
        ready.erase(i);
        return r;
    }
    CtPtr eval(std::vector<double> a, int target) {
        trim_zeros(a);
        const int d = (int)a.size() - 1;
        if (d <= B) return leaf();
        std::vector<double> q, r;
        int G;
        split(a, d, q, r, G);
        CtPtr qv = eval(q, target - 1);
        trim_zeros(r);
        if (r.size() == 1 && r[0] == 0.0) return cc.mul(*qv, giant(G));
        if (folded(r)) {
            CtPtr rawsum = leaf();  // the collected raw leaf (same order as collect)
            CtPtr out = cc.mul_add_raw(*qv, giant(G), *rawsum);
            if (r[0] != 0.0) cc.add_const_inplace(out, r[0]);
            return out;
        }
        CtPtr prod = cc.mul(*qv, giant(G));
        CtPtr rv = eval(r, target);
        return cc.add(*prod, *rv);
    }
    CtPtr run(const std::vector<double> &a, int target) {
        collect(a, target);
        return eval(a, target);
    }
};

// ------------------------------------------------ OpenFHE's split (spec 1) --
// OpenFHE's EvalChebyshevSeriesPS / InnerEvalChebyshevPS (ckksrns-advancedshe.cpp)
// with ComputeDegreesPS and LongDivisionChebyshev (ckksrns-utils.cpp): baby
// steps T_1..T_k, giant steps T_{k 2^i}, the series padded to degree
// k(2^m - 1) by a monic T term that is subtracted again at the end, and at
// every node  f = (T_{k 2^(mm-1)} + c) q + s  from two long divisions.  The
// quotients stay monic (leading coefficient a power of two), so |q(x)| is
// bounded by ~2^(mm-1) at every node: fresh noise in a giant step is never
// multiplied by the tail of the series.  DESIGN.md §3 measures the effect
// (scripts/ps_noise_model.py).  oracle: oracle_algo.cpp PSOpenFHE.

// last index with a nonzero coefficient (OpenFHE Degree: exact zero test)
int degree_of(const std::vector<double> &c) {
    for (int i = (int)c.size() - 1; i >= 0; --i)
        if (c[i] != 0.0) return i;
    return 0;
}

// OpenFHE ComputeDegreesPS(n): the (k, m) minimising k + 2m + 2^(m-1) - 4 over
// k (2^m - 1) > n with |floor(log2 k) - floor(log2 sqrt(n/2))| <= 1 (integer
// n/2 and n/k as the unsigned original); ties: the first (smallest k).  Up to
// degree 2204 OpenFHE's depth is its published band (openfhe_ps_depth, the
// budget of the reference's multDepth tables); the heuristic exceeds the band by
// one level at 46 degrees (12-13, 56-59, 240-247, 992-1007, 2016-2031, none of
// them a degree the reference evaluates), so candidates deeper than the band
// are excluded there (and the window dropped if that leaves none).
void openfhe_degrees_ps(int n, int &k_out, int &m_out) {
    const double sqn2 = std::floor(std::log2(std::sqrt((double)(unsigned)(n / 2))));
    const int band = n <= 2204 ? openfhe_ps_depth(n) : 1 << 30;
    for (int window = 1; window >= 0; --window) {
        long best = -1;
        for (long k = 1; k <= n; ++k) {
            const long q = n / k;
            if (q == 0) break;
            const double mmax = std::ceil(std::log2((double)q) + 1) + 1;
            for (long m = 1; (double)m <= mmax; ++m) {
                if ((long)n - k * ((1L << m) - 1) >= 0) continue;
                if (window && std::fabs(std::floor(std::log2((double)k)) - sqn2) > 1) continue;
                if (ceil_log2(k) + m > band) continue;
                const long mult = k + 2 * m + (1L << (m - 1)) - 4;
                if (best < 0 || mult < best) {
                    best = mult;
                    k_out = (int)k;
                    m_out = (int)m;
                }
            }
        }
        if (best >= 0) return;
    }
    throw std::invalid_argument("openfhe_degrees_ps: no (k, m) for this degree");
}

// OpenFHE LongDivisionChebyshev: f = q g + r for series in the c_0/2 convention
// (q returned in the same convention).  The divisors used here are monic or
// have a power-of-two leading coefficient, so every step is exact in its
// leading term.
void long_division_chebyshev(const std::vector<double> &f, const std::vector<double> &g, std::vector<double> &q,
                             std::vector<double> &r) {
    int n = degree_of(f);
    const int k = degree_of(g);
    if (n != (int)f.size() - 1 || k != (int)g.size() - 1)
        throw std::invalid_argument("long_division_chebyshev: zero leading coefficient");
    r = f;
    if (n - k < 0) {
        q.assign(1, 0.0);
        return;
    }
    q.assign(n - k + 1, 0.0);
    const double gk = g[k];
    while (n - k > 0) {
        q[n - k] = 2 * r.back();
        if (gk != 1.0) q[n - k] /= gk;
        std::vector<double> d(n + 1, 0.0);
        if (k == n - k) {
            d[0] = 2 * g[n - k];
            for (int i = 1; i < 2 * k + 1; ++i) d[i] = g[std::abs(n - k - i)];
        } else if (k > n - k) {
            d[0] = 2 * g[n - k];
            for (int i = 1; i < k - (n - k) + 1; ++i) d[i] = g[std::abs(n - k - i)] + g[n - k + i];
            for (int i = k - (n - k) + 1; i < n + 1; ++i) d[i] = g[std::abs(i - n + k)];
        } else {
            d[n - k] = g[0];
            for (int i = n - 2 * k; i < n + 1; ++i)
                if (i != n - k) d[i] = g[std::abs(i - n + k)];
        }
        const double rn = r.back();
        if (rn != 1.0)
            for (double &v : d) v *= rn;
        if (gk != 1.0)
            for (double &v : d) v /= gk;
        for (size_t i = 0; i < r.size(); ++i) r[i] -= d[i];
        if (r.size() > 1) {
            const int n_old = n;
            n = degree_of(r);
            r.resize(n + 1);
            // a non-finite or non-cancelling leading term would loop forever
            if (n >= n_old) throw std::invalid_argument("evalChebyshevSeriesPS: long division does not converge");
        }
    }
    if (n == k) {
        q[0] = r.back();
        if (gk != 1.0) q[0] /= gk;
        std::vector<double> d(g);
        const double rn = r.back();
        if (rn != 1.0)
            for (double &v : d) v *= rn;
        if (gk != 1.0)
            for (double &v : d) v /= gk;
        for (size_t i = 0; i < r.size(); ++i) r[i] -= d[i];
        if (r.size() > 1) {
            n = degree_of(r);
            r.resize(n + 1);
        }
    }
    q[0] *= 2;
}

// The division tree of one series, computed once per coefficient table.
// Leaves are linear sums over T_1..T_k: `a` holds sum a_i T_i (a[0] the
// constant added afterwards, already halved).
struct OFNode {
    int mm = 0;
    int cu = -1;          // leaf index of c(u), or -1 (then c0 is the constant)
    double c0 = 0.0;      // c's constant when cu < 0
    int qleaf = -1, sleaf = -1;  // leaf indices, or -1 (child nodes)
    std::unique_ptr<OFNode> qn, sn;
};
struct OFLeaf {
    std::vector<double> a;  // size k+1
    int mm;                 // node depth: target level = lk + mm - 1
    bool raw;               // s-leaf: folded into the node's product before its rescale
};
struct OFPlan {
    int k = 0, m = 0;
    std::unique_ptr<OFNode> root;
    std::vector<OFLeaf> leaves;
    double cmax = 0.0;  // largest |c| quotient coefficient of the tree
};
// OpenFHE's padding keeps every quotient bounded (|c| <= 2m for the series the
// reference evaluates: sinc tables, g_4, EvalMod) only while the monic T term
// dominates the series.  A series with O(1) coefficients that do not decay
// makes the second division ill-conditioned (|c| ~ 1e7 at degree 60, 1e46 at
// 126: the evaluation then cancels to garbage), so such a series, or one whose
// division does not converge, is evaluated with the power-of-two split.
constexpr double OF_CMAX = 1024.0;

int of_leaf(OFPlan &P, const std::vector<double> &c, int upto, int mm, bool raw) {
    OFLeaf L;
    L.a.assign(P.k + 1, 0.0);
    for (int i = 1; i <= upto && i < (int)c.size(); ++i) L.a[i] = c[i];
    L.a[0] = c[0] / 2;
    L.mm = mm;
    L.raw = raw;
    P.leaves.push_back(std::move(L));
    return (int)P.leaves.size() - 1;
}

std::unique_ptr<OFNode> of_build(OFPlan &P, const std::vector<double> &f, int mm) {
    const int k = P.k;
    auto node = std::make_unique<OFNode>();
    node->mm = mm;
    const int k2m2k = k * (1 << (mm - 1)) - k;
    std::vector<double> Tkm(k2m2k + k + 1, 0.0), q, r, cq, cr;
    Tkm.back() = 1.0;
    long_division_chebyshev(f, Tkm, q, r);
    std::vector<double> r2 = r;
    if (k2m2k - degree_of(r) <= 0) {
        r2[k2m2k] -= 1;
        r2.resize(degree_of(r2) + 1);
    } else {
        r2.resize(k2m2k + 1, 0.0);
        r2.back() = -1;
    }
    long_division_chebyshev(r2, q, cq, cr);
    std::vector<double> s2 = cr;
    s2.resize(k2m2k + 1, 0.0);
    s2.back() = 1;
    const int dc = degree_of(cq);
    for (double v : cq) P.cmax = std::max(P.cmax, std::fabs(v));
    if (dc >= 1)
        node->cu = of_leaf(P, cq, dc, mm, false);
    else
        node->c0 = cq[0] / 2;
    if (degree_of(q) > k)
        node->qn = of_build(P, q, mm - 1);
    else
        node->qleaf = of_leaf(P, q, k, mm, false);  // q[k] is the power-of-two leading term
    if (degree_of(s2) > k)
        node->sn = of_build(P, s2, mm - 1);
    else
        node->sleaf = of_leaf(P, s2, k, mm, true);  // s2[k] = 1 (monic)
    return node;
}

// Division trees cached by coefficient vector: built outside the lock (the
// degree-6510 series' first build does not block other lanes' lookups), least
// recently used entries evicted beyond OF_CACHE_MAX series.
constexpr size_t OF_CACHE_MAX = 64;
std::shared_ptr<const OFPlan> of_plan_build(const std::vector<double> &c) {
    auto P = std::make_shared<OFPlan>();
    const int n = degree_of(c);
    openfhe_degrees_ps(n, P->k, P->m);
    if (P->m < 2) return nullptr;
    const int k2m2k = P->k * (1 << (P->m - 1)) - P->k;
    std::vector<double> f2(c.begin(), c.begin() + n + 1);
    f2.resize(2 * k2m2k + P->k + 1, 0.0);
    f2.back() = 1;  // + T_{k(2^m - 1)}, subtracted after the evaluation
    try {
        P->root = of_build(*P, f2, P->m);
    } catch (const std::invalid_argument &) {
        P->cmax = INFINITY;
    }
    if (!(P->cmax <= OF_CMAX)) return nullptr;  // ill-conditioned: power-of-two split
    return P;
}
std::shared_ptr<const OFPlan> of_plan(const std::vector<double> &c) {
    struct Entry {
        std::shared_ptr<const OFPlan> plan;
        uint64_t used;
    };
    static std::mutex mu;
    static std::map<std::vector<double>, Entry> cache;
    static uint64_t tick = 0;
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find(c);
        if (it != cache.end()) {
            it->second.used = ++tick;
            return it->second.plan;
        }
    }
    std::shared_ptr<const OFPlan> plan = of_plan_build(c);  // deterministic: a racing build gives the same plan
    std::lock_guard<std::mutex> g(mu);
    auto ins = cache.emplace(c, Entry{plan, ++tick});
    if (!ins.second) {
        ins.first->second.used = tick;
        return ins.first->second.plan;
    }
    while (cache.size() > OF_CACHE_MAX) {
        auto lru = cache.begin();
        for (auto it = cache.begin(); it != cache.end(); ++it)
            if (it->second.used < lru->second.used) lru = it;
        cache.erase(lru);
    }
    return plan;
}

struct PSOpenFHE {
    Engine &cc;
    std::shared_ptr<const OFPlan> P;
    int k, m, lk;
    std::vector<CtPtr> T;   // T[i] = T_i, 1 <= i <= k
    std::vector<CtPtr> T2;  // T2[j] = T_{k 2^j}
    std::map<size_t, CtPtr> ready;

    PSOpenFHE(Engine &c, const Ciphertext &x, std::shared_ptr<const OFPlan> plan)
        : cc(c), P(std::move(plan)), k(P->k), m(P->m), lk(x.level + ceil_log2(P->k)) {
        T.resize(k + 1);
        T[1] = cc.clone(x);
    }
    // 2 a b (+ c x): the doubling is applied to an operand, before the product's
    // single rescale (OpenFHE doubles before its deferred rescale as well); an
    // operand below the other's level is doubled by the level-adjusting
    // constant product itself
    CtPtr twice_prod(const Ciphertext &a, const Ciphertext &b, const Ciphertext *x, double cx) {
        const Ciphertext *lo = &a, *hi = &b;
        if (lo->level > hi->level) std::swap(lo, hi);
        CtPtr a2 = lo->level < hi->level ? cc.mul_const_to(*lo, 2.0, hi->level) : cc.add(*lo, *lo);
        if (!x) return cc.mul(*a2, *hi);
        return cc.mul_add(*a2, *hi, {x}, {cx});
    }
    // T_i: powers of two and even i by 2 T_{i/2}^2 - 1, odd i by 2 T_{i/2} T_{i/2+1} - T_1
    void build() {
        for (int i = 2; i <= k; ++i) {
            if (i % 2 == 0) {
                T[i] = twice_prod(*T[i / 2], *T[i / 2], nullptr, 0.0);
                cc.add_const_inplace(T[i], -1.0);
            } else {
                T[i] = twice_prod(*T[i / 2], *T[i / 2 + 1], T[1].get(), -1.0);
            }
        }
        T2.push_back(T[k]);
        for (int j = 1; j < m; ++j) {
            T2.push_back(twice_prod(*T2[j - 1], *T2[j - 1], nullptr, 0.0));
            cc.add_const_inplace(T2.back(), -1.0);
        }
    }
    // T_{k(2^m - 1)} = 2 T_{k(2^(j) - 1)} T_{k 2^j} - T_k, j = 1..m-1
    CtPtr t2km1() {
        CtPtr t = T2[0];
        for (int j = 1; j < m; ++j) t = twice_prod(*t, *T2[j], T2[0].get(), -1.0);
        return t;
    }
    // leaves sharing (target, raw) are evaluated up to ps_chunk() per linear-sum
    // pass (the leaf-sum kernel's outputs; any grouping gives the same words)
    void evaluate_chunk(size_t first) {
        const OFLeaf &L0 = P->leaves[first];
        std::vector<size_t> chunk;
        const size_t max_chunk = ps_chunk();
        for (size_t i = first; i < P->leaves.size() && chunk.size() < max_chunk; ++i)
            if (P->leaves[i].mm == L0.mm && P->leaves[i].raw == L0.raw && !ready.count(i)) chunk.push_back(i);
        std::vector<int> idx;
        for (size_t c : chunk)
            for (int i = 1; i <= k; ++i)
                if (P->leaves[c].a[i] != 0.0) idx.push_back(i);
        std::sort(idx.begin(), idx.end());
        idx.erase(std::unique(idx.begin(), idx.end()), idx.end());
        const int target = lk + L0.mm - 1 + (L0.raw ? 1 : 0);
        // every leaf has a T term: c(u) only exists with degree >= 1, q and s2
        // end in their (power-of-two / monic) T_k term
        if (idx.empty()) throw std::logic_error("openfhe split: leaf without T terms");
        std::vector<const Ciphertext *> xs;
        for (int i : idx) xs.push_back(T[i].get());
        std::vector<std::vector<double>> rows;
        for (size_t c : chunk) {
            std::vector<double> row;
            for (int i : idx) row.push_back(P->leaves[c].a[i]);
            rows.push_back(row);
        }
        auto outs = cc.linear_sums_to(xs, rows, target, !L0.raw);
        for (size_t g = 0; g < chunk.size(); ++g) {
            CtPtr r = std::move(outs[g]);
            if (!L0.raw && P->leaves[chunk[g]].a[0] != 0.0) cc.add_const_inplace(r, P->leaves[chunk[g]].a[0]);
            ready[chunk[g]] = r;
        }
    }
    CtPtr leaf(int i) {
        if (!ready.count(i)) evaluate_chunk(i);
        CtPtr r = ready.at(i);
        ready.erase(i);
        return r;
    }
    // node at depth mm: (T2[mm-1] + c) q + s, output level lk + mm
    CtPtr node(const OFNode &N) {
        // a = T2[mm-1] + c(u): with c(u) a leaf the sum is formed inside the
        // product's tensor pass (Engine::mul_add's a_add; same words)
        CtPtr cu = N.cu >= 0 ? leaf(N.cu) : nullptr;
        CtPtr a = cu ? T2[N.mm - 1] : (N.c0 != 0.0 ? cc.add_const(*T2[N.mm - 1], N.c0) : T2[N.mm - 1]);
        CtPtr qu = N.qn ? node(*N.qn) : leaf(N.qleaf);
        if (N.sn) {
            CtPtr su = node(*N.sn);  // level lk + mm - 1: added before the product's rescale
            return cc.mul_add(*a, *qu, {su.get()}, {1.0}, nullptr, cu.get());
        }
        const double s0 = P->leaves[N.sleaf].a[0];
        CtPtr raw = leaf(N.sleaf);
        CtPtr out = cc.mul_add_raw(*a, *qu, *raw, cu.get());
        if (s0 != 0.0) cc.add_const_inplace(out, s0);
        return out;
    }
    CtPtr run() {
        build();
        CtPtr top = node(*P->root);
        return cc.sub(*top, *t2km1());
    }
};

}  // namespace

// (the conditioning fallback never changes the depth: for every degree >= 5
// OpenFHE's ceil(log2 k) + m equals the power-of-two split's max(D, OpenFHE's
// published band), tests/test_oracle.py::test_ps_depth_tables)
int chebPSDepthSplit(int d, int split) {
    if (split == PS_SPLIT_OPENFHE && d >= 5) {
        int k = 0, m = 0;
        openfhe_degrees_ps(d, k, m);
        if (m >= 2) return ceil_log2(k) + m;
    }
    return std::max(std::max(1, ceil_log2((long)d + 1)), openfhe_ps_depth(d));
}
int chebPSDepth(int d) { return chebPSDepthSplit(d, PS_SPLIT_OPENFHE); }

bool chebPSUsesOpenFHE(const std::vector<double> &coeffs) {
    std::vector<double> c(coeffs);
    trim_zeros(c);
    return c.size() >= 6 && of_plan(c) != nullptr;
}

CtPtr evalChebyshevSeriesPS(Engine &cc, const Ciphertext &x0, const std::vector<double> &coeffs, double a,
                            double b) {
    std::vector<double> c(coeffs);
    trim_zeros(c);
    if (c.empty()) throw std::invalid_argument("evalChebyshevSeriesPS: empty coefficients");
    CtPtr x = cc.clone(x0);
    if (!(a == -1.0 && b == 1.0)) {
        x = cc.mul_const(*x, 2.0 / (b - a));
        cc.add_const_inplace(x, -(a + b) / (b - a));
    }
    const int d = (int)c.size() - 1;
    if (cc.ps_split() == PS_SPLIT_OPENFHE && d >= 5) {
        if (auto plan = of_plan(c)) {
            PSOpenFHE ev(cc, *x, plan);
            return ev.run();
        }
    }
    std::vector<double> s(c);
    s[0] = c[0] / 2.0;
    if (d == 0) return cc.add_const(*cc.trivial_const(0.0, x->level, x->slots, x->batch), s[0]);
    PSEval ev(cc, *x, d);
    ev.build_baby();
    return ev.run(s, x->level + std::max(ev.D, openfhe_ps_depth(d)));
}

// ====================================================== composite sign =====
namespace {

// c1 x + c3 x^3 + c5 x^5 + c7 x^7 in depth 3 (src/sign.cpp:15-59): the terms
// that join a product are added before its rescale (mul_add), so only c3 x
// and c7 x are rescaled on their own (oracle: oracle_algo.cpp odd7)
CtPtr odd7(Engine &cc, const Ciphertext &x, double c1, double c3, double c5, double c7) {
    CtPtr x2 = cc.square(x);
    CtPtr x4 = cc.square(*x2);
    CtPtr t3 = cc.mul(*cc.mul_const(x, c3), *x2);
    CtPtr u = cc.mul_add(*cc.mul_const(x, c7), *x2, {&x}, {c5});
    return cc.mul_add(*u, *x4, {&x, t3.get()}, {c1, 1.0});
}
// g_3 = (4589x - 16577x^3 + 25614x^5 - 12860x^7)/2^10       (src/sign.cpp:15-36)
CtPtr g3(Engine &cc, const Ciphertext &x) {
    return odd7(cc, x, 4589.0 / 1024.0, -16577.0 / 1024.0, 25614.0 / 1024.0, -12860.0 / 1024.0);
}
// f_3 = (35x - 35x^3 + 21x^5 - 5x^7)/2^4                    (src/sign.cpp:38-59)
CtPtr f3(Engine &cc, const Ciphertext &x) { return odd7(cc, x, 35.0 / 16.0, -35.0 / 16.0, 21.0 / 16.0, -5.0 / 16.0); }

// g_4: degree-27 Chebyshev series on [-1, 1]                  (src/sign.cpp:66-77)
const std::vector<double> &g4_coeffs() {
    static const std::vector<double> c = {
        0.0, 1.077117252745569,    0.0, -0.36166113998402755, 0.0, 0.2137420717859748,
        0.0, -0.15635204788780485, 0.0, 0.11749645501187332,  0.0, -0.10074154666447852,
        0.0, 0.08002086947825496,  0.0, -0.07533558758484624, 0.0, 0.059514472116534836,
        0.0, -0.06146663712787884, 0.0, 0.04570084927999001,  0.0, -0.05403683682999072,
        0.0, 0.03364293851188723,  0.0, -0.054459493266273494};
    return c;
}
CtPtr g4(Engine &cc, const Ciphertext &x) { return evalChebyshevSeriesPS(cc, x, g4_coeffs(), -1.0, 1.0); }

// f_4: odd degree-15 polynomial                               (src/sign.cpp:79-157)
CtPtr f4(Engine &cc, const Ciphertext &x) {
    const double c1 = 3.14208984375, c3 = -7.33154296875, c5 = 13.19677734375, c7 = -15.71044921875,
                 c9 = 12.21923828125, c11 = -5.99853515625, c13 = 1.69189453125, c15 = -0.20947265625;
    const int l = x.level;
    CtPtr x2 = cc.square(x);
    CtPtr x4 = cc.square(*x2);
    CtPtr x8 = cc.square(*x4);
    CtPtr c3x3 = cc.mul(*cc.mul_const(x, c3), *x2);
    CtPtr c7x3 = cc.mul(*cc.mul_const(x, c7), *x2);
    CtPtr c11x3 = cc.mul(*cc.mul_const(x, c11), *x2);
    CtPtr c15x3 = cc.mul(*cc.mul_const(x, c15), *x2);
    CtPtr v1 = cc.mul(*cc.add(*cc.mul_const_to(x, c5, l + 2), *c7x3), *x4);
    CtPtr bt = cc.add(*cc.mul_const_to(x, c9, l + 2), *c11x3);
    CtPtr w = cc.mul(*cc.add(*cc.mul_const_to(x, c13, l + 2), *c15x3), *x4);
    CtPtr tmp1 = cc.add(*cc.level_adjust(*bt, l + 3), *w);
    CtPtr z = cc.mul(*tmp1, *x8);
    CtPtr y = cc.add(*cc.mul_const_to(x, c1, l + 4), *cc.level_adjust(*c3x3, l + 4));
    y = cc.add(*y, *cc.level_adjust(*v1, l + 4));
    return cc.add(*y, *z);
}

}  // namespace

CtPtr compositeSignN(Engine &cc, const Ciphertext &x, int n, const SignConfig &cfg) {
    if (n != 3 && n != 4) throw std::invalid_argument("compositeSign: n must be 3 or 4");
    auto g = [&](const Ciphertext &v) { return n == 3 ? g3(cc, v) : g4(cc, v); };
    auto f = [&](const Ciphertext &v) { return n == 3 ? f3(cc, v) : f4(cc, v); };
    // lazyBootstrap (src/sign.cpp:164-170): g_depth = f_depth = n (3 or 4)
    const int L = cc.params().L;
    auto lazy = [&](const Ciphertext &c) -> CtPtr {
        if (!(cfg.boot && L - c.level < n + 2)) return nullptr;
        CtPtr b = cfg.boot(c);
        if (std::getenv("FHE_KWAY_TRACE")) {  // diagnostics: lazy bootstrap error
            const auto u = cc.decrypt(c), v = cc.decrypt(*b);
            double e = 0, mx = 0;
            for (size_t i = 0; i < u.size(); ++i) {
                e = std::max(e, std::fabs(u[i] - v[i]));
                mx = std::max(mx, std::fabs(u[i]));
            }
            std::fprintf(stderr, "  sign boot at level %d: max|in| %.6g, max|out - in| %.3g\n", c.level, mx, e);
        }
        return b;
    };
    CtPtr b = lazy(x);
    CtPtr y = g(b ? *b : x);  // applied once even when dg == 0 (src/sign.cpp:173)
    for (int i = 1; i < cfg.compos.dg; ++i) {
        if ((b = lazy(*y))) y = b;
        y = g(*y);
    }
    for (int i = 0; i < cfg.compos.df; ++i) {
        if ((b = lazy(*y))) y = b;
        y = f(*y);
    }
    return y;
}

CtPtr sign(const Ciphertext &x, Engine &cc, SignFunc func, const SignConfig &cfg) {
    if (func != SignFunc::CompositeSign)
        throw std::invalid_argument("sign: only SignFunc::CompositeSign is implemented on the GPU path");
    return compositeSignN(cc, x, cfg.compos.n, cfg);
}

CtPtr Comparison::compare(Engine &cc, const Ciphertext &a, const Ciphertext &b, SignFunc f, const SignConfig &cfg) {
    CtPtr diff = cc.sub(a, b);
    if (cfg.boot && std::getenv("FHE_KWAY_TRACE")) {
        double mx = 0;
        for (double v : cc.decrypt(*diff)) mx = std::max(mx, std::fabs(v));
        std::fprintf(stderr, "  compare: level %d, max|a - b| %.6g\n", diff->level, mx);
    }
    CtPtr s = sign(*diff, cc, f, cfg);
    cc.add_const_inplace(s, 1.0);
    return cc.mul_const(*s, 0.5);
}

CtPtr Comparison::indicator(Engine &cc, const Ciphertext &x, double c, SignFunc f, const SignConfig &cfg) {
    CtPtr d1 = cc.add_const(x, c);
    CtPtr d2 = cc.add_const(x, -c);
    CtPtr s1 = sign(*d1, cc, f, cfg);
    CtPtr s2 = sign(*d2, cc, f, cfg);
    cc.add_const_inplace(s1, 1.0);
    cc.add_const_inplace(s2, 1.0);
    CtPtr c1 = cc.mul_const(*s1, 0.5);
    CtPtr c2 = cc.mul_const(*s2, 0.5);
    CtPtr om = cc.add_const(*cc.negate(*c2), 1.0);
    return cc.mul(*c1, *om);
}

// ================================================ Decomposer / composer =====
DecomposerN::DecomposerN(int N_, std::vector<int> rot) : N(N_), maxDecomposed(0), rotIndices(std::move(rot)) {
    if (rotIndices.empty()) throw std::invalid_argument("Decomposer: empty rotation index set");
    std::sort(rotIndices.begin(), rotIndices.end());
    int step = 1;
    for (int idx : rotIndices) {
        if (step == idx / 2) maxDecomposed += idx;
        step = idx;
    }
}

std::vector<Step> DecomposerN::decompose(int rotation, int wrapN, DecomposeAlgo algo) const {
    std::vector<Step> steps;
    const int largest = rotIndices.back();
    while (rotation >= largest) {
        steps.push_back({1, largest});
        rotation -= largest;
    }
    if (!rotation) return steps;
    while (rotation > maxDecomposed) {
        const int legal = *(std::lower_bound(rotIndices.begin(), rotIndices.end(), rotation) - 1);
        steps.push_back({1, legal});
        rotation -= legal;
    }
    if (!rotation) return steps;
    std::vector<Step> rem;
    if (algo == DecomposeAlgo::BINARY) {
        for (int i = 30; i >= 0; --i) {
            const int s = 1 << i;
            if (s < N && (rotation & s)) rem.push_back({1, s});
        }
    } else if (algo == DecomposeAlgo::NAF) {
        int r = rotation, i = 0;
        while (r != 0) {
            if (r & 1) {
                const int z = (r & 2) ? -1 : 1;
                const int s = z * (1 << i);
                if (s == -N / 2)
                    rem.push_back({-z, -s});
                else
                    rem.push_back({z, s});
                r -= z;
            }
            r >>= 1;
            ++i;
        }
        std::reverse(rem.begin(), rem.end());
    } else {
        std::vector<int> digits;
        int Kk = rotation;
        while (Kk != 0) {
            int ki = Kk % 2;
            Kk = (Kk - ki) / 2;
            if (ki > 1 || (ki == 1 && (Kk % 2) >= 1)) {
                ki -= 2;
                Kk += 1;
            }
            digits.push_back(ki);
        }
        for (size_t i = 0; i < digits.size(); ++i)
            if (digits[i] != 0) rem.push_back({digits[i], (int)((long)digits[i] * (1L << i))});
        std::reverse(rem.begin(), rem.end());
    }
    steps.insert(steps.end(), rem.begin(), rem.end());
    steps.erase(std::remove_if(steps.begin(), steps.end(), [wrapN](const Step &s) { return s.stepSize % wrapN == 0; }),
                steps.end());
    return steps;
}

RotationComposerN::RotationComposerN(Engine &c, int N, const std::vector<int> &rotIndices, DecomposeAlgo a)
    : cc(c), dec(N, rotIndices), algo(a), avail(rotIndices.begin(), rotIndices.end()) {}

CtPtr RotationComposerN::rotate(const Ciphertext &in, int rotation) {
    if (rotation % in.slots == 0) return cc.clone(in);
    if (avail.count(rotation)) return cc.rotate(in, rotation);
    CtPtr r = cc.clone(in);
    for (const Step &s : dec.decompose(rotation, in.slots, algo)) r = cc.rotate(*r, s.stepSize);
    return r;
}

std::vector<CtPtr> RotationComposerN::rotateMany(const Ciphertext &in, const std::vector<int> &rotations) {
    std::vector<CtPtr> out(rotations.size());
    std::vector<long> keyed;
    std::vector<size_t> where;
    for (size_t i = 0; i < rotations.size(); ++i) {
        const int r = rotations[i];
        if (r % in.slots == 0)
            out[i] = cc.clone(in);
        else if (avail.count(r)) {
            keyed.push_back(r);
            where.push_back(i);
        } else
            out[i] = rotate(in, r);
    }
    if (!keyed.empty()) {
        auto h = cc.rotate_hoisted(in, keyed);  // one ModUp shared by all keyed rotations
        for (size_t i = 0; i < h.size(); ++i) out[where[i]] = h[i];
    }
    return out;
}

std::vector<CtPtr> RotationComposerN::rotateMembers(const Ciphertext &in, const std::vector<int> &rotations) {
    const int B = in.batch;
    if ((int)rotations.size() != B) throw std::invalid_argument("rotateMembers: one rotation per member");
    const long half = (long)cc.n() / 2;
    std::vector<std::vector<int>> steps(B);  // the keyed steps rotate() would apply
    size_t depth = 0;
    for (int m = 0; m < B; ++m) {
        const int r = rotations[m];
        if (r % in.slots == 0)
            ;
        else if (avail.count(r))
            steps[m].push_back(r);
        else
            for (const Step &st : dec.decompose(r, in.slots, algo))
                if (st.stepSize % half) steps[m].push_back(st.stepSize);  // (a step = 0 mod n/2 is the identity)
        depth = std::max(depth, steps[m].size());
    }
    std::vector<CtPtr> cur(B);
    for (int m = 0; m < B; ++m) cur[m] = cc.member(in, m);
    for (size_t j = 0; j < depth; ++j) {
        std::vector<int> act;
        std::vector<long> ks;
        for (int m = 0; m < B; ++m)
            if (steps[m].size() > j) {
                act.push_back(m);
                ks.push_back(steps[m][j]);
            }
        if (act.size() == 1) {
            cur[act[0]] = cc.rotate(*cur[act[0]], ks[0]);
            continue;
        }
        CtPtr r;
        if (j == 0 && (int)act.size() == B) {
            r = cc.rotate_members(in, ks);
        } else {
            std::vector<const Ciphertext *> v;
            for (int m : act) v.push_back(cur[m].get());
            r = cc.rotate_members(*cc.stack(v), ks);
        }
        for (size_t i = 0; i < act.size(); ++i) cur[act[i]] = cc.member(*r, (int)i);
    }
    for (int m = 0; m < B; ++m)
        if (steps[m].empty()) cur[m] = cc.clone(*cur[m]);  // as rotate(): a copy, not a view
    return cur;
}

// ============================================================ DirectSort ===
// ---------------------------------------------------------- RotationTree ----
RotationTreeN::RotationTreeN(Engine &c, int N, const std::vector<int> &rotIndices, DecomposeAlgo a)
    : cc(c), dec(N, rotIndices), algo(a), root(std::make_unique<Node>(0, nullptr)) {}

void RotationTreeN::buildTree(int start, int end) {  // src/rotation.h:272-279
    for (int i = start; i <= end; ++i) addToTree(root.get(), dec.decompose(i, end, algo), 0, i);
}

void RotationTreeN::addToTree(Node *node, const std::vector<Step> &steps, size_t i, int value) {  // :293-312
    for (; i < steps.size(); ++i) {
        if (steps[i].value == 0) continue;
        auto &child = node->children[steps[i].stepSize];
        if (!child) child = std::make_unique<Node>(steps[i].stepSize, node);
        node = child.get();
    }
    node->finalValues.push_back(value);
}

CtPtr RotationTreeN::treeRotate(const Ciphertext &input, int rotation) {  // :281-291
    auto steps = dec.decompose(rotation, input.slots, algo);
    return traverse(cc.clone(input), root.get(), steps, 0);
}

CtPtr RotationTreeN::traverse(const CtPtr &input, Node *node, const std::vector<Step> &steps, size_t i) {
    for (; i < steps.size() && steps[i].value == 0; ++i) {
    }
    if (i >= steps.size()) return input;
    auto it = node->children.find(steps[i].stepSize);
    if (it == node->children.end()) {  // the reference reports and returns the partial rotation (:323-327)
        std::fprintf(stderr, "Error: Child node not found for step size %d\n", steps[i].stepSize);
        return input;
    }
    Node *child = it->second.get();
    if (child->rotated) {
        ++stats.cacheHits;
    } else {
        // all not-yet-rotated children of this node share the node's ModUp
        std::vector<Node *> todo;
        std::vector<long> ks;
        for (auto &kv : node->children)
            if (!kv.second->rotated) {
                todo.push_back(kv.second.get());
                ks.push_back(kv.first);
            }
        auto outs = cc.rotate_hoisted(*input, ks);
        for (size_t j = 0; j < todo.size(); ++j) todo[j]->rotated = outs[j];
        stats.cacheMisses += 1;
        stats.fastRotationCount += todo.size();
        stats.totalRotationCount += todo.size();
    }
    return traverse(child->rotated, child, steps, i + 1);
}

void directSortSizeParameters(int N, int &multDepth, std::vector<int> &r) {
    // restated from src/sort_algo.h:87-201 (depth, rotation-key set per N)
    switch (N) {
    case 4: multDepth = 23; r = {1, 2, 4, 8, 16}; break;
    case 8: multDepth = 24; r = {1, 2, 4, 6, 8, 16, 32, 64}; break;
    case 16: multDepth = 25; r = {1, 2, 3, 4, 8, 12, 16, 32, 64, 128, 256}; break;
    case 32: multDepth = 28; r = {1, 2, 3, 4, 8, 12, 16, 20, 24, 28, 32, 64, 128, 256, 512, 1024}; break;
    case 64:
        multDepth = 29;
        r = {1, 2, 3, 4, 5, 6, 7, 8, 16, 24, 32, 40, 48, 56, 64, 128, 256, 512, 1024, 2048, 4096};
        break;
    case 128:
        multDepth = 30;
        r = {1, 2, 3, 4, 5, 6, 7, 8, 16, 24, 32, 40, 48, 56, 64, 72, 80, 88, 96, 104, 112, 120, 128, 256, 512, 1024,
             2048, 4096, 8192, 16384};
        break;
    case 256: {
        multDepth = 34;
        r.clear();
        for (int i = 1; i <= 16; ++i) r.push_back(i);
        for (int i = 24; i <= 128; i += 8) r.push_back(i);
        for (int i = 129; i <= 135; ++i) r.push_back(i);
        for (int i = 144; i <= 256; i += 16) r.push_back(i);
        for (int i = 512; i <= 32768; i *= 2) r.push_back(i);
        break;
    }
    case 512: {
        multDepth = 35;
        r.clear();
        for (int i = 1; i <= 16; ++i) r.push_back(i);
        for (int i = 24; i <= 64; i += 8) r.push_back(i);
        for (int b = 64; b <= 448; b += 64) {
            for (int i = 1; i <= 7; ++i) r.push_back(b + i);
            for (int i = b + 16; i <= b + 64; i += 16) r.push_back(i);
        }
        for (int i = 1024; i <= 32768; i *= 2) r.push_back(i);
        std::sort(r.begin(), r.end());
        r.erase(std::unique(r.begin(), r.end()), r.end());
        break;
    }
    case 1024: {
        multDepth = 39;
        r.clear();
        for (int i = 1; i <= 35; ++i) r.push_back(i);
        for (int b = 64; b <= 992; b += 32)
            for (int i = 0; i <= 3; ++i) r.push_back(b + i);
        for (int i = 1024; i <= 32768; i *= 2) r.push_back(i);
        break;
    }
    case 2048:  // DirectSortNTest's largest size (tests/DirectSortNTest.cpp:387)
        multDepth = 52;
        r = {
            1, 2, 4, 8, 16, 31, 32, 64, 115, 128, 179, 211, 227, 241, 242, 243, 256, 307, 339, 355, 369, 370,
            371, 403, 419, 433, 434, 435, 451, 465, 466, 467, 481, 482, 483, 496, 497, 498, 499, 512, 563, 595,
            611, 625, 626, 627, 659, 675, 689, 690, 691, 707, 721, 722, 723, 737, 738, 739, 752, 753, 754, 755,
            787, 803, 817, 818, 819, 835, 849, 850, 851, 865, 866, 867, 880, 881, 882, 883, 899, 913, 914, 915,
            929, 930, 931, 944, 945, 946, 947, 961, 962, 963, 976, 977, 978, 979, 992, 993, 994, 995, 1008,
            1009, 1010, 1011, 1024, 1075, 1107, 1123, 1137, 1138, 1139, 1171, 1187, 1201, 1202, 1203, 1219,
            1233, 1234, 1235, 1249, 1250, 1251, 1264, 1265, 1266, 1267, 1299, 1315, 1329, 1330, 1331, 1347,
            1361, 1362, 1363, 1377, 1378, 1379, 1392, 1393, 1394, 1395, 1411, 1425, 1426, 1427, 1441, 1442,
            1443, 1456, 1457, 1458, 1459, 1473, 1474, 1475, 1488, 1489, 1490, 1491, 1504, 1505, 1506, 1507,
            1520, 1521, 1522, 1523, 1555, 1571, 1585, 1586, 1587, 1603, 1617, 1618, 1619, 1633, 1634, 1635,
            1648, 1649, 1650, 1651, 1667, 1681, 1682, 1683, 1697, 1698, 1699, 1712, 1713, 1714, 1715, 1729,
            1730, 1731, 1744, 1745, 1746, 1747, 1760, 1761, 1762, 1763, 1776, 1777, 1778, 1779, 1795, 1809,
            1810, 1811, 1825, 1826, 1827, 1840, 1841, 1842, 1843, 1857, 1858, 1859, 1872, 1873, 1874, 1875,
            1888, 1889, 1890, 1891, 1904, 1905, 1906, 1907, 1921, 1922, 1923, 1937, 1938, 1939, 1953, 1954,
            1955, 1968, 1969, 1970, 1971, 1985, 1986, 1987, 2000, 2001, 2002, 2003, 2016, 2017, 2018, 2019,
            2032, 2033, 2034, 2035, 2048, 4096, 8192, 16384, 32768};
        break;
    default: throw std::invalid_argument("DirectSort::getSizeParameters: unsupported N");
    }
}

static int rank_np(int N, int P) {  // src/sort_algo.h:383-416
    switch (N) {
    case 4: case 8: return std::min(2, P);
    case 16: case 32: return std::min(4, P);
    case 64: case 128: return std::min(8, P);
    case 256: case 512: return std::min(16, P);
    case 1024: case 2048: return std::min(32, P);
    default: return 1;
    }
}
static int check_np(int N) {  // src/sort_algo.h:670-703
    switch (N) {
    case 4: case 8: return 2;
    case 16: case 32: return 4;
    case 64: case 128: return 8;
    case 256: return 16;
    case 512: case 1024: return 8;
    default: return 4;
    }
}
SortShape rankShape(int N, int max_batch) {
    SortShape s;
    s.N = N;
    s.num_partition = std::min(N, max_batch / N);
    if (s.num_partition < 1) throw std::invalid_argument("DirectSort: N*N exceeds ring capacity");
    s.num_batch = N / s.num_partition;
    s.num_slots = N * s.num_partition;
    s.np = rank_np(N, s.num_partition);
    return s;
}
SortShape checkShape(int N, int max_batch) {
    SortShape s = rankShape(N, max_batch);
    s.np = check_np(N);
    return s;
}

namespace {
std::vector<double> mask_vector(int num_slots, int N, int k) {  // src/sort_algo.h:206-233
    std::vector<double> v(num_slots, 0.0);
    for (int i = k * N; i < (k + 1) * N; ++i) v[i] = 1.0;
    return v;
}
std::vector<double> vector_rotate(std::vector<double> v, int r) {  // src/sort_algo.h:289-306
    const int n = (int)v.size();
    if (r > 0)
        std::rotate(v.begin(), v.begin() + r, v.end());
    else if (r < 0)
        std::rotate(v.begin(), v.begin() + (r + n), v.end());
    return v;
}
std::vector<double> checking_vector(int num_slots, int N, int k) {  // src/sort_algo.h:272-286
    std::vector<double> v(num_slots);
    int idx = 0, cur = k;
    while (idx < num_slots) {
        for (int i = 0; i < N && idx < num_slots; ++i) v[idx++] = cur;
        cur = (cur + 1) % N;
    }
    return v;
}
}  // namespace

DirectSortN::DirectSortN(Engine &c, int N_, const std::vector<int> &rotIndices)
    : cc(c), N(N_), rot(c, N_, rotIndices), max_batch((int)(c.n() / 2)), rot_indices(rotIndices) {}

DirectSortN::Lane DirectSortN::lane(int l) {
    if (l == 0) return Lane{&cc, &rot};
    while ((int)lane_eng.size() < l) {
        lane_eng.push_back(cc.fork());
        lane_rot.push_back(std::make_unique<RotationComposerN>(*lane_eng.back(), N, rot_indices));
    }
    return Lane{lane_eng[l - 1].get(), lane_rot[l - 1].get()};
}

// Split `batches` into contiguous groups, one per lane; lane 0 runs on this
// thread with the context's engine, the others on their own threads and
// forked engines.  Everything the lanes read must be complete on the main
// stream (callers sync before).  Returns each lane's partial (may be null),
// with every lane stream drained.
template <class F>
std::vector<CtPtr> DirectSortN::run_lanes(const std::vector<int> &batches, F &&work) {
    const int L = std::max(1, std::min(lanes, (int)batches.size()));
    std::vector<std::vector<int>> groups(L);
    for (size_t i = 0; i < batches.size(); ++i) groups[i * L / batches.size()].push_back(batches[i]);
    std::vector<Lane> ls;
    for (int l = 0; l < L; ++l) ls.push_back(lane(l));
    std::vector<CtPtr> parts(L);
    std::vector<std::exception_ptr> errs(L);
    std::vector<std::thread> th;
    for (int l = 1; l < L; ++l)
        th.emplace_back([&, l] {
            try {
                parts[l] = work(ls[l], groups[l]);
                ls[l].eng->sync();
            } catch (...) {
                errs[l] = std::current_exception();
            }
        });
    try {
        parts[0] = work(ls[0], groups[0]);
    } catch (...) {
        errs[0] = std::current_exception();
    }
    for (auto &t : th) t.join();
    for (int l = 1; l < L; ++l) {  // the context's counters cover every lane
        cc.ctr += ls[l].eng->ctr;
        ls[l].eng->ctr = Counters();
    }
    for (auto &e : errs)
        if (e) std::rethrow_exception(e);
    return parts;
}

// kind 0: mask_vector(k) rotated by `r` (vector_rotate); kind 1: checking vector(k)
// Encoded outside the lock, so concurrent lanes encode their masks in parallel;
// a mask two lanes race for is encoded twice (identical words) and the first
// published copy is kept.
const Plaintext &DirectSortN::mask(Engine &E, int kind, int num_slots, int k, int r, int level) {
    auto key = std::make_tuple(kind, num_slots, k, r, level);
    {
        std::lock_guard<std::mutex> lk(mask_mu);
        auto it = mask_cache.find(key);
        if (it != mask_cache.end()) return *it->second;
    }
    static const bool host_masks = [] {
        const char *e = std::getenv("FHE_HOST_MASKS");
        return e && std::atoi(e) == 1;
    }();
    PtPtr p;
    if (host_masks) {
        std::vector<double> v =
            kind == 0 ? vector_rotate(mask_vector(num_slots, N, k), r) : checking_vector(num_slots, N, k);
        p = E.encode(v, num_slots, level);
    } else {
        p = E.encode_masks({Engine::MaskSpec{kind, k, r, level}}, num_slots, N)[0];  // word-identical
    }
    E.sync();  // complete before another lane's stream reads it
    std::lock_guard<std::mutex> lk(mask_mu);
    auto ins = mask_cache.emplace(key, p);
    return *ins.first->second;
}

void checkShardWorld(const host::Params &P, int world) {
    u64 qmax = 0;
    for (size_t i = 0; i < P.nq(); ++i) qmax = std::max(qmax, P.primes[i]);
    if (world < 1 || (u64)world > ~0ULL / qmax)
        throw std::invalid_argument("sharded run: world " + std::to_string(world) +
                                    " ranks would overflow the u64 sum of residues (world * q_max >= 2^64)");
}
ShardHeader checkShardHeader(const u64 h[4]) {
    const u64 present = h[0], s1 = h[1], s2 = h[2], limbs = h[3];
    if (present == 0) throw std::runtime_error("sharded run: no shard produced a partial");
    // all present partials share one level iff sum(l)^2 == present * sum(l^2)
    if ((unsigned __int128)s1 * s1 != (unsigned __int128)present * s2 || s1 % present || limbs % present)
        throw std::runtime_error("sharded run: ranks' partials differ in level or limb count");
    return ShardHeader{(int)(s1 / present) - 1, (size_t)(limbs / present)};
}

// algorithm phase of the clocked kernels (bench.py roofline.phases; DirectSort:
// rank_baby / rank_batches / rank_fold / index_batches / index_fold, MEHP24:
// its sortFG phases).  Thread-local, so set again inside each lane's work.
struct AlgoPhase {
    const char *prev;
    explicit AlgoPhase(const char *p) : prev(Engine::set_algo_phase(p)) {}
    ~AlgoPhase() { Engine::set_algo_phase(prev); }
};

void reducePartial(Engine &cc, const Shard &sh, CtPtr &acc, int slots) {
    // a single rank reduces only when the caller gave it a collective (an
    // RCCL communicator of world 1 still runs the all-reduce)
    if (!sh.allreduce) {
        if (sh.world > 1) throw std::runtime_error("sharded run without an allreduce hook");
        return;
    }
    checkShardWorld(cc.params(), sh.world);
    if (acc && acc->batch != 1) throw std::invalid_argument("sharded run: a partial must be a single ciphertext");
    // header: presence, level + 1, (level + 1)^2, limbs -- summed over ranks.
    // Every rank sees the same sums, so every rank takes the same branch below.
    // The exchange's time (bench.py: allreduce_ms beside rank_compute_ms) runs
    // from a drained stream -- this rank's compute is done -- to the reduced
    // data; the two drains that bracket it are taken only when the time is
    // wanted (FHE_TIME_COLLECTIVES=1, set by bench.py; advisor r4)
    static const bool timed = [] {
        const char *e = std::getenv("FHE_TIME_COLLECTIVES");
        return e && std::atoi(e) != 0;
    }();
    if (timed) cc.sync();
    const auto t0 = std::chrono::steady_clock::now();
    auto hdr = cc.alloc_u64(4);
    const u64 l1 = acc ? (u64)(acc->level + 1) : 0;
    u64 h[4] = {acc ? 1ULL : 0ULL, l1, l1 * l1, acc ? (u64)acc->limbs : 0};
    cc.h2d(hdr.ptr, h, 4);
    sh.allreduce(hdr.ptr, 4);
    cc.d2h(h, hdr.ptr, 4);
    const ShardHeader H = checkShardHeader(h);
    if (!acc) acc = cc.zero_like(H.level, slots);
    if (acc->limbs != H.limbs) throw std::runtime_error("sharded run: partial limb count differs from the header");
    sh.allreduce(acc->data, 2 * acc->limbs * cc.n());
    cc.reduce_after_allreduce(*acc);
    if (timed) {
        cc.sync();
        cc.ctr.allreduce_ns += (u64)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                   std::chrono::steady_clock::now() - t0).count();
    }
    cc.ctr.allreduce_calls += 1;
}
void DirectSortN::reducePartial(CtPtr &acc, int slots) {
    Shard sh;
    sh.rank = shard_rank;
    sh.world = shard_world;
    sh.allreduce = allreduce;
    fhe::reducePartial(cc, sh, acc, slots);
}

// The np baby-step rotations x, rot(x,1), ..., rot(x,np-1) of vecRotsOpt
// (src/sort_algo.h:383-416) feed every comparator batch, so every rank computes
// all of them (hoisted: one ModUp).  Sharding them (rank r computes steps
// r mod world, one all-reduce of the zero-padded stack gathers them) saved 7 ms
// of compute per rank at world 8 but moves 1.3 GB through the collective --
// about as long over xGMI -- so they stay replicated.
std::vector<CtPtr> DirectSortN::babySteps(const Ciphertext &x, int np) {
    std::vector<int> idx(np);
    for (int i = 0; i < np; ++i) idx[i] = i;
    return rot.rotateMany(x, idx);
}

CtPtr DirectSortN::vecRotsOpt(Lane L, const std::vector<CtPtr> &baby, int num_partition, int num_slots, int np,
                              int is) {
    CtPtr result;
    for (int j = 0; j < num_partition / np; ++j) {
        std::vector<const Ciphertext *> cs;
        std::vector<const Plaintext *> ps;
        for (int i = 0; i < np; ++i) {
            cs.push_back(baby[i].get());
            ps.push_back(&mask(*L.eng, 0, num_slots, np * j + i, -is * num_partition - j * np, baby[i]->level));
        }
        CtPtr Tj = L.eng->mul_plain_sum(cs, ps);  // one rescale per masked sum (src/sort_algo.h:341-346)
        CtPtr o = L.rot->rotate(*Tj, is * num_partition + j * np);
        L.eng->add_inplace(result, *o);
    }
    return result;
}

std::vector<CtPtr> DirectSortN::vecRotsOptMany(Lane L, const std::vector<CtPtr> &baby, int num_partition,
                                               int num_slots, int np, const std::vector<int> &iss) {
    if (iss.size() == 1) return {vecRotsOpt(L, baby, num_partition, num_slots, np, iss[0])};
    std::vector<CtPtr> result(iss.size());
    for (int j = 0; j < num_partition / np; ++j) {
        std::vector<CtPtr> T(iss.size());
        std::vector<const Ciphertext *> tp;
        std::vector<int> rots;
        for (size_t b = 0; b < iss.size(); ++b) {
            std::vector<const Ciphertext *> cs;
            std::vector<const Plaintext *> ps;
            for (int i = 0; i < np; ++i) {
                cs.push_back(baby[i].get());
                ps.push_back(&mask(*L.eng, 0, num_slots, np * j + i, -iss[b] * num_partition - j * np, baby[i]->level));
            }
            T[b] = L.eng->mul_plain_sum(cs, ps);
            tp.push_back(T[b].get());
            rots.push_back(iss[b] * num_partition + j * np);
        }
        auto o = L.rot->rotateMembers(*L.eng->stack(tp), rots);
        for (size_t b = 0; b < iss.size(); ++b) L.eng->add_inplace(result[b], *o[b]);
    }
    return result;
}

// The comparator batches run stacked: their inputs differ, but the sign() op
// sequence is identical, so one compare over a ciphertext batch replaces
// max_stack sequential ones, on `lanes` concurrent streams.
// compare(x, s_b) = ((sign(x - s_b) + 1) / 2); the per-batch results are summed
// exactly mod q, so the rank equals the reference's batch-by-batch
// accumulation (src/sort_algo.h:474-491) word for word.
CtPtr DirectSortN::constructRank(const Ciphertext &x, SignFunc f, const SignConfig &cfg) {
    const SortShape s = rankShape(N, max_batch);
    std::optional<AlgoPhase> ph;
    ph.emplace("rank_baby");
    std::vector<CtPtr> baby = babySteps(x, s.np);
    for (auto &b : baby) b->slots = s.num_slots;
    ph.reset();
    std::vector<int> mine;
    for (int b = 0; b < s.num_batch; ++b)
        if (b % shard_world == shard_rank) mine.push_back(b);
    CtPtr dup = cc.clone(x);
    dup->slots = s.num_slots;
    cc.sync();  // baby steps and dup are read by every lane
    const size_t chunk = (size_t)std::max(1, max_stack);
    auto parts = run_lanes(mine, [&](Lane L, const std::vector<int> &bs) -> CtPtr {
        Engine &E = *L.eng;
        AlgoPhase lane_ph("rank_batches");
        CtPtr acc;
        for (size_t c0 = 0; c0 < bs.size(); c0 += chunk) {
            std::vector<int> iss(bs.begin() + c0, bs.begin() + std::min(bs.size(), c0 + chunk));
            std::vector<CtPtr> shifted = vecRotsOptMany(L, baby, s.num_partition, s.num_slots, s.np, iss);
            std::vector<const Ciphertext *> ptrs;
            for (auto &x : shifted) ptrs.push_back(x.get());
            // x - s_b of every batch written straight into the stacked ciphertext
            CtPtr d = ptrs.size() == 1 ? E.sub(*dup, *shifted[0]) : E.sub_stacked(*dup, ptrs);
            shifted.clear();
            CtPtr sg = sign(*d, E, f, cfg);
            E.add_const_inplace(sg, 1.0);
            CtPtr c = E.mul_const(*sg, 0.5);
            E.add_inplace(acc, c->batch == 1 ? *c : *E.sum_members(*c));
        }
        return acc;
    });
    CtPtr rank;
    for (auto &p : parts)
        if (p) cc.add_inplace(rank, *p);
    cc.sync();  // lane buffers return to their pools only after the main stream read them
    parts.clear();
    reducePartial(rank, s.num_slots);
    ph.emplace("rank_fold");
    for (int i = 1; i < std::log2((double)s.num_partition) + 1; ++i)
        rank = cc.add(*rank, *rot.rotate(*rank, s.num_slots / (1 << i)));
    rank->slots = N;
    cc.add_const_inplace(rank, -0.5);
    return rank;
}

CtPtr DirectSortN::blindRotationOptN(const std::vector<CtPtr> &mi, int num_slots, int np, int ib, int num_partition) {
    return blindRotationStacked(lane(0), mi, num_slots, np, {ib}, num_partition);
}

CtPtr DirectSortN::blindRotationStacked(Lane L, const std::vector<CtPtr> &mi, int num_slots, int np,
                                        const std::vector<int> &ibs, int num_partition) {
    Engine &E = *L.eng;
    CtPtr result;
    for (int i = 0; i < (num_slots / N) / np; ++i) {
        std::vector<const Ciphertext *> cs;
        std::vector<const Plaintext *> ps;
        for (int j = 0; j < np; ++j) {
            cs.push_back(mi[j].get());
            ps.push_back(&mask(E, 0, num_slots, np * i + j, j, mi[j]->level));
        }
        CtPtr tmp = E.mul_plain_sum(cs, ps);  // src/sort_algo.h:573-577
        if (tmp->batch == 1) {
            E.add_inplace(result, *L.rot->rotate(*tmp, ibs[0] * num_partition + i * np));
            continue;
        }
        // every batch's giant-step rotation (its own amount) in shared launches;
        // the sum mod q does not depend on the order of the terms
        std::vector<int> rots;
        for (size_t m = 0; m < ibs.size(); ++m) rots.push_back(ibs[m] * num_partition + i * np);
        for (auto &o : L.rot->rotateMembers(*tmp, rots)) E.add_inplace(result, *o);
    }
    return result;
}

// Index check, stacked like constructRank: the doubled-sinc PS (the dominant
// cost, ~200 HMult per batch at N=1024) and the masking product run once over
// a batch of max_stack inputs per lane; only the per-batch giant-step
// rotations run member by member (src/sort_algo.h:713-742).
CtPtr DirectSortN::rotationIndexCheckN(const Ciphertext &rank, const Ciphertext &x) {
    const SortShape s = checkShape(N, max_batch);
    std::vector<double> idx(N);
    for (int i = 0; i < N; ++i) idx[i] = (double)i;
    PtPtr idxpt = cc.encode(idx, N, rank.level);
    CtPtr imr = cc.plain_sub(*idxpt, rank);
    imr->slots = s.num_slots;
    CtPtr xs = cc.clone(x);
    xs->slots = s.num_slots;
    const std::vector<double> &coeffs = sincCoefficients();
    std::vector<int> ridx(s.np);
    for (int i = 0; i < s.np; ++i) ridx[i] = i;
    std::vector<int> mine;
    for (int b = 0; b < s.num_batch; ++b)
        if (b % shard_world == shard_rank) mine.push_back(b);
    cc.sync();  // imr and xs are read by every lane
    const size_t chunk = (size_t)std::max(1, max_stack);
    auto parts = run_lanes(mine, [&](Lane L, const std::vector<int> &bs) -> CtPtr {
        Engine &E = *L.eng;
        AlgoPhase lane_ph("index_batches");
        CtPtr acc;
        for (size_t c0 = 0; c0 < bs.size(); c0 += chunk) {
            std::vector<const Plaintext *> chks;
            std::vector<int> ibs;
            for (size_t i = c0; i < std::min(bs.size(), c0 + chunk); ++i) {
                const int b = bs[i];
                chks.push_back(&mask(E, 1, s.num_slots, b * s.num_partition, 0, imr->level));
                ibs.push_back(b);
            }
            // (imr - checking vector_b) / 2N of every batch: the differences written
            // straight into one stacked ciphertext, one scaling for all of them
            CtPtr r = E.mul_const(*(chks.size() == 1 ? E.sub_plain(*imr, *chks[0]) : E.sub_plain_stacked(*imr, chks)),
                                  1.0 / N / 2);
            r = evalChebyshevSeriesPS(E, *r, coeffs, -1.0, 1.0);
            CtPtr masked = E.mul(*r, *xs);  // xs broadcast over the members
            r.reset();
            std::vector<CtPtr> mi = L.rot->rotateMany(*masked, ridx);
            masked.reset();
            E.add_inplace(acc, *blindRotationStacked(L, mi, s.num_slots, s.np, ibs, s.num_partition));
        }
        return acc;
    });
    CtPtr out;
    for (auto &p : parts)
        if (p) cc.add_inplace(out, *p);
    cc.sync();
    parts.clear();
    reducePartial(out, s.num_slots);
    AlgoPhase ph("index_fold");
    for (int i = 1; i < std::log2((double)s.num_partition) + 1; ++i)
        out = cc.add(*out, *rot.rotate(*out, s.num_slots / (1 << i)));
    out->slots = N;
    return out;
}

// Re-encodes every cached mask (the reference's per-use encoding,
// src/sort_algo.h:341-342, 714-716) for sort() with mask caching off.  Chunks
// of REFRESH_CHUNK masks: each chunk's new plaintexts replace (and release) old
// ones before the next chunk is encoded, so the peak is about one chunk above
// the mask set instead of twice the set (advisor r4).  The other
// fhe_direct_sort modes (rank only, index check only) keep the cached masks.
void DirectSortN::refresh_masks() {
    constexpr size_t REFRESH_CHUNK = 128;
    cc.sync();
    for (auto &e : lane_eng) e->sync();  // nothing of the last sort still reads the old masks
    std::map<int, std::vector<std::tuple<int, int, int, int, int>>> by_slots;
    {
        std::lock_guard<std::mutex> lk(mask_mu);
        for (auto &kv : mask_cache) by_slots[std::get<1>(kv.first)].push_back(kv.first);
    }
    for (auto &g : by_slots) {
        for (size_t a = 0; a < g.second.size(); a += REFRESH_CHUNK) {
            const size_t b = std::min(g.second.size(), a + REFRESH_CHUNK);
            std::vector<Engine::MaskSpec> specs;
            for (size_t i = a; i < b; ++i) {
                const auto &key = g.second[i];
                specs.push_back(Engine::MaskSpec{std::get<0>(key), std::get<2>(key), std::get<3>(key), std::get<4>(key)});
            }
            auto pts = cc.encode_masks(specs, g.first, N);  // synchronises the main stream
            std::lock_guard<std::mutex> lk(mask_mu);
            for (size_t i = a; i < b; ++i) mask_cache[g.second[i]] = pts[i - a];
        }
    }
}

CtPtr DirectSortN::sort(const Ciphertext &x, SignFunc f, const SignConfig &cfg) {
    if (!cache_masks) refresh_masks();
    CtPtr rank = constructRank(x, f, cfg);
    return rotationIndexCheckN(*rank, x);
}

// ============================================================== MEHP24 ======
// Mazzone et al. ranking / sorting (src/mehp24/mehp24_sort.cpp,
// mehp24_utils.cpp).  A vector of length m lives in an m x m slot matrix
// (slot = m * row + col).  The reference runs its independent pair compares
// and indicators on OpenMP threads; here they run stacked: one ciphertext
// batch per level group through one sign pipeline (chunks of max_stack
// members), each member bit-identical to the oracle's one-by-one evaluation.
// ------------------------------------------------------------ sort_hybrid ----
namespace {
// getBinaryPath (src/sort_algo.h:814-821): bits of `index`, most significant first
std::vector<bool> binaryPath(size_t index, size_t m) {
    const size_t lm = (size_t)ceil_log2((long)m);
    std::vector<bool> path(lm);
    for (size_t k = 0; k < lm; ++k) path[k] = (index >> (lm - 1 - k)) & 1;
    return path;
}
// sumColumnsToTarget (:824-855) / transposeColumnTarget (:857-891): a binary tree
// of rotations by +-step (the sign from the target's bits), then a 0/1 mask
CtPtr columnsToTarget(Engine &cc, RotationComposerN &rot, CtPtr c, size_t m, size_t target, bool transpose,
                      bool mask) {
    auto path = binaryPath(target, m);
    long step = transpose ? (long)(m * (m - 1) / 2) : (long)(m >> 1);
    c->slots = (int)(m * m);
    for (size_t i = 0; i < path.size(); ++i, step >>= 1) c = cc.add(*c, *rot.rotate(*c, path[i] ? -step : step));
    if (mask) {
        std::vector<double> msk(m * m, 0.0);
        for (size_t i = 0; i < m; ++i) msk[transpose ? m * target + i : m * i + target] = 1.0;
        c = cc.mul_plain(*c, *cc.encode(msk, c->slots, c->level));
    }
    return c;
}
}  // namespace

// rotationIndexCheckHybrid (:893-1047): the rank vector, reinterpreted as an
// m x m slot matrix (m = min(N, maxArraySize); N > m: num_batch = N / m blocks
// over the full slot count), is compared with the row index of each block b:
// entry (i, j) of pair (b, k) is [rank_e == b m + i] with e = j + m((i + k) mod
// num_batch) -- the scaled-sinc PS for N < 256, Comparison::indicator above --
// times the input at e; the column sums then hold the sorted values.  The
// num_batch^2 masks of this rank's blocks run as one stacked batch.
CtPtr DirectSortN::rotationIndexCheckHybrid(const Ciphertext &rank, const Ciphertext &x) {
    const size_t maxA = (size_t)hybrid_max_array;
    size_t num_slots, num_batch;
    if ((size_t)N > maxA) {
        num_slots = (size_t)max_batch;
        num_batch = (size_t)N / maxA;
    } else {
        num_slots = (size_t)N * (size_t)N;
        num_batch = 1;
    }
    const size_t A = std::min((size_t)N, maxA);
    if (A * A != num_slots) throw std::invalid_argument("sort_hybrid: maxArraySize^2 must equal the slot count");
    CtPtr rk = cc.clone(rank);
    rk->slots = (int)num_slots;
    CtPtr r = cc.mul_const(*rk, 1.0 / N);
    CtPtr in = cc.clone(x);
    in->slots = (int)num_slots;
    std::vector<CtPtr> rots_rank(num_batch), rots_in(num_batch);
    for (size_t b = 0; b < num_batch; ++b) {
        rots_rank[b] = rot.rotate(*r, (int)(b * maxA));
        rots_in[b] = rot.rotate(*in, (int)(b * maxA));
    }
    int mode = hybrid_mask;
    if (mode == 0) mode = N < 256 ? 1 : N < 512 ? 2 : 3;
    std::vector<size_t> mine;
    for (size_t b = 0; b < num_batch; ++b)
        if (shard_world <= 1 || b % (size_t)shard_world == (size_t)shard_rank) mine.push_back(b);
    // the masks (b, k) of this rank's blocks, stacked
    std::vector<CtPtr> ms, ins;
    for (size_t b : mine) {
        std::vector<double> sub(num_slots, 0.0);
        for (size_t i = 0; i < A; ++i)
            for (size_t j = 0; j < A; ++j) sub[i * A + j] = (double)(b * A + i) / (double)N;
        PtPtr subpt = cc.encode(sub, (int)num_slots, r->level);
        for (size_t k = 0; k < num_batch; ++k) {
            ms.push_back(cc.plain_sub(*subpt, *rots_rank[k]));
            ins.push_back(rots_in[k]);
        }
    }
    CtPtr result;
    const size_t chunk = (size_t)std::max(1, max_stack);
    std::vector<CtPtr> prod(ms.size());
    for (size_t c0 = 0; c0 < ms.size(); c0 += chunk) {
        const size_t c1 = std::min(ms.size(), c0 + chunk);
        std::vector<const Ciphertext *> mp, ip;
        for (size_t i = c0; i < c1; ++i) {
            mp.push_back(ms[i].get());
            ip.push_back(ins[i].get());
        }
        CtPtr m = mp.size() == 1 ? ms[c0] : cc.stack(mp);
        if (mode == 1)
            m = evalChebyshevSeriesPS(cc, *m, scaledSincCoefficients(N), -1.0, 1.0);
        else
            m = Comparison().indicator(cc, *m, 0.5 / N, SignFunc::CompositeSign,
                                       SignConfig(CompositeSignConfig(3, mode == 2 ? 4 : 5, 2)));
        CtPtr t = cc.mul(*(ip.size() == 1 ? ins[c0] : cc.stack(ip)), *m);
        for (size_t i = c0; i < c1; ++i) prod[i] = t->batch == 1 ? t : cc.member(*t, (int)(i - c0));
    }
    ms.clear();
    for (size_t q = 0; q < mine.size(); ++q) {
        const size_t b = mine[q];
        CtPtr acc;
        for (size_t k = 0; k < num_batch; ++k) cc.add_inplace(acc, *prod[q * num_batch + k]);
        acc = columnsToTarget(cc, rot, acc, (size_t)N / num_batch, b, false, true);
        acc = columnsToTarget(cc, rot, acc, (size_t)N / num_batch, b, true, true);
        cc.add_inplace(result, *acc);
    }
    prod.clear();
    reducePartial(result, (int)num_slots);
    return result;
}

CtPtr DirectSortN::sort_hybrid(const Ciphertext &x, SignFunc f, const SignConfig &cfg) {
    CtPtr rank = constructRank(x, f, cfg);
    return rotationIndexCheckHybrid(*rank, x);
}

// tests/DirectSortHTest.cpp:23-104 (ring 2^17, scale 2^40)
void hybridSortSizeParameters(int N, int &multDepth, std::vector<int> &r) {
    switch (N) {
    case 4: multDepth = 24; r = {1, 2, 3, 4, 6, 8}; break;
    case 8: multDepth = 25; r = {1, 2, 4, 6, 7, 8, 14, 16, 28, 32}; break;
    case 16: multDepth = 25; r = {1, 2, 3, 4, 8, 12, 15, 16, 30, 32, 60, 64, 120, 128}; break;
    case 32:
        multDepth = 29;
        r = {1, 2, 3, 4, 8, 12, 16, 20, 24, 28, 31, 32, 62, 64, 124, 128, 248, 256, 496, 512};
        break;
    case 64:
        multDepth = 30;
        r = {1, 2, 3, 4, 6, 7, 8, 16, 24, 32, 40, 48, 56, 63, 64, 126, 128, 252, 256, 504, 512, 1008, 1024, 2016, 2048};
        break;
    case 128:
        multDepth = 31;
        r = {1,   2,   3,   4,   5,   6,    7,    8,    16,   24,   32,   40,   48,   56,   64,  72,  80,  88,
             96,  104, 112, 120, 127, 128,  254,  256,  508,  512,  1016, 1024, 2032, 2048, 4064, 4096, 8128, 8192};
        break;
    case 256:
        multDepth = 44;
        r = {1,   2,   3,   4,   5,   6,   7,   8,   9,    10,   11,   12,   13,   14,   15,    16,
             32,  48,  64,  80,  96,  112, 128, 144, 160,  176,  192,  208,  224,  240,  255,   256,
             510, 512, 1020, 1024, 2040, 2048, 4080, 4096, 8160, 8192, 16320, 16384, 32640, 32768};
        break;
    case 512:
        multDepth = 47;
        r = {-255, -1,  1,   2,    3,    4,    5,    6,    7,    8,     9,     10,    11,    12,    13,   14,
             15,   16,  32,  48,   64,   80,   96,   112,  128,  144,   160,   176,   192,   208,   224,  240,
             255,  256, 272, 288,  304,  320,  336,  352,  368,  384,   400,   416,   432,   448,   464,  480,
             496,  510, 512, 1020, 1024, 2040, 2048, 4080, 4096, 8160,  8192,  16320, 16384, 32640, 32768};
        break;
    case 1024:
        multDepth = 50;
        r = {-510, -255, -2,  -1,  1,   2,   3,   4,   5,    6,    7,    8,    9,    10,    11,    12,
             13,   14,   15,  16,  17,  28,  18,  20,  21,   22,   23,   24,   25,   26,    27,    29,
             30,   31,   32,  64,  96,  128, 160, 192, 224,  255,  256,  288,  320,  352,   384,   416,
             448,  480,  510, 512, 544, 576, 608, 640, 672,  704,  736,  768,  800,  832,   864,   896,
             928,  960,  992, 1020, 1024, 2040, 2048, 4080, 4096, 8160, 8192, 16320, 16384, 32640, 32768};
        break;
    default: throw std::invalid_argument("sort_hybrid: N must be a power of two in [4, 1024]");
    }
}

namespace mehp24 {

namespace {
size_t lg(size_t x) { return (size_t)ceil_log2((long)x); }  // LOG2 (mehp24_utils.h:25)
}  // namespace

namespace utils {

std::vector<int> getRotationIndices(size_t m, size_t sub) {  // mehp24_utils.cpp:197-225
    size_t sz = m;
    std::vector<int> idx;
    if (m > sub) {
        for (size_t i = 0; i < m / sub; ++i) {
            idx.push_back((int)(i * sub));
            idx.push_back(-(int)(i * sub));
        }
        sz = sub;
    }
    for (size_t i = 0; i < lg(sz); ++i) {
        const int t = (int)(sz * (sz - 1) / (1u << (i + 1)));
        for (int k : {1 << i, -(1 << i), -(1 << (lg(sz) + i)), t, -t}) idx.push_back(k);
    }
    std::vector<int> out;
    for (int k : idx)
        if (k != 0 && std::find(out.begin(), out.end(), k) == out.end()) out.push_back(k);
    return out;
}

const Plaintext &Masks::get(Engine &cc, int kind, size_t m, size_t idx, int level, int slots) {
    auto key = std::make_tuple(kind, m, idx, level, slots);
    auto it = cache.find(key);
    if (it != cache.end()) return *it->second;
    std::vector<double> v(m * m, 0.0);
    for (size_t i = 0; i < m; ++i) v[kind == 0 ? m * idx + i : m * i + idx] = 1.0;  // 0: row idx, 1: column idx
    return *(cache[key] = cc.encode(v, slots, level));
}

CtPtr maskRow(Engine &cc, Masks &mk, const Ciphertext &c, size_t m, size_t row) {  // :21-30
    return cc.mul_plain(c, mk.get(cc, 0, m, row, c.level, c.slots));
}
CtPtr maskColumn(Engine &cc, Masks &mk, const Ciphertext &c, size_t m, size_t col) {  // :32-42
    return cc.mul_plain(c, mk.get(cc, 1, m, col, c.level, c.slots));
}
CtPtr replicateRow(Engine &cc, CtPtr c, size_t m) {  // :44-50
    for (size_t i = 0; i < lg(m); ++i) c = cc.add(*c, *cc.rotate(*c, -(1L << (lg(m) + i))));
    return c;
}
CtPtr replicateColumn(Engine &cc, CtPtr c, size_t m) {  // :52-58
    for (size_t i = 0; i < lg(m); ++i) c = cc.add(*c, *cc.rotate(*c, -(1L << i)));
    return c;
}
CtPtr sumRows(Engine &cc, Masks &mk, CtPtr c, size_t m, bool mask, size_t row) {  // :60-69
    c = replicateRow(cc, c, m);
    return mask ? maskRow(cc, mk, *c, m, row) : c;
}
CtPtr sumColumns(Engine &cc, Masks &mk, CtPtr c, size_t m, bool mask) {  // :71-80
    for (size_t i = 0; i < lg(m); ++i) c = cc.add(*c, *cc.rotate(*c, 1L << i));
    return mask ? maskColumn(cc, mk, *c, m, 0) : c;
}
CtPtr transposeRow(Engine &cc, Masks &mk, CtPtr c, size_t m, bool mask) {  // :82-91
    for (size_t i = 1; i <= lg(m); ++i) c = cc.add(*c, *cc.rotate(*c, -(long)(m * (m - 1) / (1u << i))));
    return mask ? maskColumn(cc, mk, *c, m, 0) : c;
}
CtPtr transposeColumn(Engine &cc, Masks &mk, CtPtr c, size_t m, bool mask) {  // :93-103
    for (size_t i = 1; i <= lg(m); ++i) c = cc.add(*c, *cc.rotate(*c, (long)(m * (m - 1) / (1u << i))));
    return mask ? maskRow(cc, mk, *c, m, 0) : c;
}

// signAdv (mehp24_utils.cpp:244-260): g3 dg times, f3 df-1 times, then the
// final 0.5 + f3/2 (output in [0, 1])
CtPtr signAdv(Engine &cc, CtPtr c, size_t dg, size_t df) {
    for (size_t d = 0; d < dg; ++d) c = g3(cc, *c);
    for (size_t d = 0; d + 1 < df; ++d) c = f3(cc, *c);
    c = odd7(cc, *c, 35.0 / 32.0, -35.0 / 32.0, 21.0 / 32.0, -5.0 / 32.0);
    cc.add_const_inplace(c, 0.5);
    return c;
}

}  // namespace utils

namespace {

// fn applied member-wise to xs: inputs grouped by level (stacking needs one
// level; the oracle evaluates each at its own level), chunks of <= max_stack
// stacked into one batch, results returned as member views in input order
template <class Fn>
std::vector<CtPtr> stacked(Engine &cc, const std::vector<CtPtr> &xs, int max_stack, Fn &&fn) {
    std::vector<CtPtr> out(xs.size());
    std::map<int, std::vector<size_t>> groups;
    for (size_t i = 0; i < xs.size(); ++i) groups[xs[i]->level].push_back(i);
    for (auto &g : groups) {
        const auto &ids = g.second;
        for (size_t b = 0; b < ids.size(); b += (size_t)max_stack) {
            const size_t e = std::min(ids.size(), b + (size_t)max_stack);
            if (e - b == 1) {
                out[ids[b]] = fn(*xs[ids[b]]);
                continue;
            }
            std::vector<const Ciphertext *> v;
            for (size_t i = b; i < e; ++i) v.push_back(xs[ids[i]].get());
            CtPtr r = fn(*cc.stack(v));
            for (size_t i = b; i < e; ++i) out[ids[i]] = cc.member(*r, (int)(i - b));
        }
    }
    return out;
}
// binary variant: pairs (xs[i], ys[i]); each side must share one level
template <class Fn>
std::vector<CtPtr> stacked2(Engine &cc, const std::vector<CtPtr> &xs, const std::vector<CtPtr> &ys, int max_stack,
                            Fn &&fn) {
    std::vector<CtPtr> out(xs.size());
    std::map<std::pair<int, int>, std::vector<size_t>> groups;
    for (size_t i = 0; i < xs.size(); ++i) groups[{xs[i]->level, ys[i]->level}].push_back(i);
    for (auto &g : groups) {
        const auto &ids = g.second;
        for (size_t b = 0; b < ids.size(); b += (size_t)max_stack) {
            const size_t e = std::min(ids.size(), b + (size_t)max_stack);
            if (e - b == 1) {
                out[ids[b]] = fn(*xs[ids[b]], *ys[ids[b]]);
                continue;
            }
            std::vector<const Ciphertext *> u, v;
            for (size_t i = b; i < e; ++i) {
                u.push_back(xs[ids[i]].get());
                v.push_back(ys[ids[i]].get());
            }
            CtPtr r = fn(*cc.stack(u), *cc.stack(v));
            for (size_t i = b; i < e; ++i) out[ids[i]] = cc.member(*r, (int)(i - b));
        }
    }
    return out;
}
// members of a stacked ciphertext
std::vector<CtPtr> members(Engine &cc, const Ciphertext &s) {
    std::vector<CtPtr> v;
    for (int m = 0; m < s.batch; ++m) v.push_back(cc.member(s, m));
    return v;
}

// indicatorAdv (mehp24_utils.cpp:166-174) of every x in xs: 1 on |x| < 1/2
// for x in [-b, b].  The 2|xs| signAdv chains run stacked.
std::vector<CtPtr> indicators(Engine &cc, const std::vector<CtPtr> &xs, double b, size_t dg, size_t df,
                              int max_stack) {
    const size_t n = xs.size();
    std::vector<CtPtr> c12(2 * n);
    auto t = stacked(cc, xs, max_stack, [&](const Ciphertext &x) { return cc.mul_const(x, 1.0 / b); });
    for (size_t i = 0; i < n; ++i) {
        c12[i] = cc.add_const(*t[i], 0.5 / b);
        c12[n + i] = cc.add_const(*t[i], -0.5 / b);
    }
    t.clear();
    auto sa = stacked(cc, c12, max_stack, [&](const Ciphertext &x) {
        return utils::signAdv(cc, cc.clone(x), dg, df);
    });
    c12.clear();
    std::vector<CtPtr> s1(sa.begin(), sa.begin() + n), s2(sa.begin() + n, sa.end());
    return stacked2(cc, s1, s2, max_stack, [&](const Ciphertext &a, const Ciphertext &c) {
        return cc.mul(a, *cc.add_const(*cc.negate(c), 1.0));
    });
}

}  // namespace

CtPtr indicatorAdv(Engine &cc, const Ciphertext &c, double b, size_t dg, size_t df) {
    return indicators(cc, {cc.clone(c)}, b, dg, df, 1)[0];
}

// sortFG, one ciphertext of m values (mehp24_sort.cpp:248-283)
CtPtr sortFG(const Ciphertext &c0, size_t m, SignFunc f, const SignConfig &cfg, uint32_t dg_i, uint32_t df_i,
             Engine &cc, int max_stack) {
    using namespace utils;
    Masks mk;
    CtPtr c = cc.clone(c0);
    CtPtr VR = replicateRow(cc, c, m);
    CtPtr VC = replicateColumn(cc, transposeRow(cc, mk, c, m, true), m);
    CtPtr C = Comparison().compare(cc, *VR, *VC, f, cfg);
    CtPtr R = sumRows(cc, mk, C, m, false, 0);
    std::vector<double> sub(m * m);
    for (size_t i = 0; i < m; ++i)
        for (size_t j = 0; j < m; ++j) sub[i * m + j] = -1.0 * (double)i - 0.5;
    CtPtr x = cc.add_plain(*R, *cc.encode(sub, R->slots, R->level));
    CtPtr M = indicators(cc, {x}, (double)m, dg_i, df_i, max_stack)[0];
    CtPtr S = sumColumns(cc, mk, cc.mul(*M, *VR), m, true);
    return transposeColumn(cc, mk, S, m, true);
}

// sortFG over parts of `sub` values (mehp24_sort.cpp:445-604): the part-wise
// rotation chains run on one stacked batch of all parts, the P(P+1)/2 pair
// compares and the P^2 indicators stacked
std::vector<CtPtr> sortFG(const std::vector<CtPtr> &c, size_t sub, SignFunc f, const SignConfig &cfg, uint32_t dg_i,
                          uint32_t df_i, Engine &cc, int max_stack, const Shard &sh) {
    using namespace utils;
    const size_t P = c.size(), m = sub * P;
    Masks mk;
    std::vector<const Ciphertext *> cv;
    for (auto &x : c) cv.push_back(x.get());
    CtPtr parts = P > 1 ? cc.stack(cv) : cc.clone(*c[0]);
    std::optional<AlgoPhase> ph;
    ph.emplace("replicate");
    auto R = members(cc, *replicateRow(cc, parts, sub));
    auto Cc = members(cc, *replicateColumn(cc, transposeRow(cc, mk, parts, sub, true), sub));
    parts.reset();

    std::vector<CtPtr> A, B;
    std::vector<std::pair<size_t, size_t>> jk;
    size_t pair = 0;  // pair index in the order of mehp24_sort.cpp:480-495 (the shard key)
    for (size_t j = 0; j < P; ++j)
        for (size_t k = j; k < P; ++k, ++pair) {
            if (!sh.mine(pair)) continue;
            jk.push_back({j, k});
            A.push_back(R[j]);
            B.push_back(Cc[k]);
        }
    ph.reset();
    ph.emplace("compare");
    auto Cjk = stacked2(cc, A, B, max_stack, [&](const Ciphertext &a, const Ciphertext &b) {
        return Comparison().compare(cc, a, b, f, cfg);
    });
    ph.reset();
    ph.emplace("rank_sums");
    A.clear();
    B.clear();
    std::vector<CtPtr> Cv(P), Ch(P);
    for (size_t i = 0; i < jk.size(); ++i) {
        const size_t j = jk[i].first, k = jk[i].second;
        cc.add_inplace(Cv[j], *Cjk[i]);
        if (j != k) cc.add_inplace(Ch[k], *cc.add_const(*cc.negate(*Cjk[i]), 1.0));
    }
    Cjk.clear();
    const int slots = R[0]->slots;
    for (size_t j = 0; j < P; ++j) reducePartial(cc, sh, Cv[j], slots);
    for (size_t k = 1; k < P; ++k) reducePartial(cc, sh, Ch[k], slots);
    std::vector<CtPtr> s(P);
    for (size_t j = 0; j < P; ++j) s[j] = sumRows(cc, mk, Cv[j], sub, false, 0);
    if (P > 1) {  // the column sums of every Ch[j], j > 0, as one batch
        std::vector<const Ciphertext *> hv;
        for (size_t j = 1; j < P; ++j) hv.push_back(Ch[j].get());
        CtPtr h = P > 2 ? cc.stack(hv) : cc.clone(*Ch[1]);
        h = replicateRow(cc, transposeColumn(cc, mk, sumColumns(cc, mk, h, sub, true), sub, true), sub);
        for (size_t j = 1; j < P; ++j) s[j] = cc.add(*s[j], *cc.member(*h, (int)j - 1));
    }
    Cv.clear();
    Ch.clear();

    ph.reset();
    ph.emplace("indicator");
    std::vector<CtPtr> X, RR;
    for (size_t j = 0; j < P; ++j) {
        std::vector<double> sm(sub * sub);
        for (size_t a = 0; a < sub; ++a)
            for (size_t b = 0; b < sub; ++b) sm[a * sub + b] = -1.0 * (double)(j * sub + a) - 0.5;
        std::map<int, PtPtr> by_level;
        for (size_t k = 0; k < P; ++k) {
            if (!sh.mine(j * P + k)) continue;
            PtPtr &pt = by_level[s[k]->level];
            if (!pt) pt = cc.encode(sm, s[k]->slots, s[k]->level);
            X.push_back(cc.add_plain(*s[k], *pt));
            RR.push_back(R[k]);
        }
    }
    auto ind = indicators(cc, X, (double)m, dg_i, df_i, max_stack);
    X.clear();
    ph.reset();
    ph.emplace("select");
    auto prod = stacked2(cc, ind, RR, max_stack, [&](const Ciphertext &a, const Ciphertext &b) { return cc.mul(a, b); });
    ind.clear();
    std::vector<CtPtr> acc(P);
    for (size_t j = 0, i = 0; j < P; ++j)
        for (size_t k = 0; k < P; ++k)
            if (sh.mine(j * P + k)) cc.add_inplace(acc[j], *prod[i++]);
    prod.clear();
    for (size_t j = 0; j < P; ++j) reducePartial(cc, sh, acc[j], slots);
    ph.reset();
    ph.emplace("recombine");
    std::vector<const Ciphertext *> av;
    for (auto &x : acc) av.push_back(x.get());
    CtPtr out = P > 1 ? cc.stack(av) : acc[0];
    out = transposeColumn(cc, mk, sumColumns(cc, mk, out, sub, true), sub, true);
    return members(cc, *out);
}

// sortLargeArrayFG (mehp24_sort.cpp:623-645, utils :265-303): split into
// parts of `sub` values, sort them as one vector, recombine
CtPtr sortLargeArrayFG(const Ciphertext &c, size_t total, size_t sub, SignFunc f, const SignConfig &cfg,
                       uint32_t dg_i, uint32_t df_i, Engine &cc, int max_stack, const Shard &sh) {
    const size_t P = total / sub;
    if (P * sub != total || P == 0) throw std::invalid_argument("sortLargeArrayFG: totalLength % subLength != 0");
    std::vector<CtPtr> parts(P);
    std::optional<AlgoPhase> ph;
    ph.emplace("split");
    for (size_t i = 0; i < P; ++i) {  // splitCiphertext
        std::vector<double> mask(total, 0.0);
        for (size_t j = 0; j < sub; ++j) mask[i * sub + j] = 1.0;
        CtPtr part = cc.mul_plain(c, *cc.encode(mask, c.slots, c.level));
        if (i > 0) part = cc.rotate(*part, (long)(i * sub));
        parts[i] = part;
    }
    ph.reset();
    auto sorted = sortFG(parts, sub, f, cfg, dg_i, df_i, cc, max_stack, sh);
    ph.emplace("recombine");
    CtPtr r = sorted[0];  // combineCiphertext
    for (size_t i = 1; i < P; ++i) r = cc.add(*r, *cc.rotate(*sorted[i], -(long)(i * sub)));
    return r;
}

// the reference test's parameters (tests/mehp24/Mehp24SortTest.cpp:26-128)
Parameters parameters(size_t N) {
    // 4096 extends the reference table (BASELINE config 5): same CompositeSign(3,5,2)
    // and dg_i = 6 as 2048, so the same depth; measured on the engine: output at
    // level 56 of 65, max error 1.2e-5
    static const std::map<size_t, int> depth = {{4, 31},    {8, 35},    {16, 35},   {32, 42},
                                                {64, 42},   {128, 46},  {256, 49},  {512, 57},
                                                {1024, 60}, {2048, 64}, {4096, 64}};
    auto it = depth.find(N);
    if (it == depth.end()) throw std::invalid_argument("mehp24: N must be a power of two in [4, 4096]");
    Parameters p;
    p.multDepth = it->second;
    p.levels = p.multDepth + 1;  // + the FLEXIBLEAUTOEXT encryption level (Engine::encrypt_ext)
    // OpenFHE's default for depth > 3 (the reference sets no digit count): 3 digits of
    // <= 22 primes, within the engine's alpha <= 24 / K <= 16 (the 4096 table: K = 16)
    p.dnum = std::max(3, (p.levels + 1 + 22) / 23);
    p.logRingDim = 17;
    p.scaleModSize = 40;
    p.cfg = SignConfig(CompositeSignConfig(3, N <= 16 ? 2 : N <= 128 ? 3 : N <= 512 ? 4 : 5, 2));
    p.dg_i = (uint32_t)((std::log2((double)N) + 1) / 2);
    p.df_i = 2;
    p.subLength = N <= 256 ? 0 : 256;
    p.rotations = utils::getRotationIndices(N);
    return p;
}

}  // namespace mehp24

// ================================================== coefficient tables =====
namespace {
std::string g_dir = "fhe-sorting_amd/data";
std::map<std::string, std::vector<double>> g_cache;
std::mutex g_mu;
}  // namespace
void setCoefficientDir(const std::string &dir) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_dir = dir;
    g_cache.clear();
}
static const std::vector<double> &coefficientTable(const std::string &kind, int N) {
    std::lock_guard<std::mutex> lk(g_mu);
    const std::string path = g_dir + "/" + kind + "_" + std::to_string(N) + ".f64";
    auto it = g_cache.find(path);
    if (it != g_cache.end()) return it->second;
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("missing coefficient file " + path);
    f.seekg(0, std::ios::end);
    const size_t bytes = (size_t)f.tellg();
    f.seekg(0);
    std::vector<double> v(bytes / 8);
    f.read(reinterpret_cast<char *>(v.data()), (std::streamsize)bytes);
    return g_cache[path] = std::move(v);
}
const std::vector<double> &doubledSincCoefficients(int N) { return coefficientTable("doubled_sinc", N); }
const std::vector<double> &scaledSincCoefficients(int N) { return coefficientTable("scaled_sinc", N); }
const std::vector<double> &evalModCoefficients(int K, int r, int degree) {
    return coefficientTable("evalmod_k" + std::to_string(K) + "r" + std::to_string(r), degree);
}
const std::vector<double> &DirectSortN::sincCoefficients() const { return doubledSincCoefficients(N); }

}  // namespace fhe
