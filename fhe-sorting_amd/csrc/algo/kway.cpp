// k-way sorting network (reference: src/k-way/*.cpp, src/kway_adapter.h);
// see kway.hpp for the map.  Every ciphertext operation runs on the GPU
// through fhe::Engine; masks are encoded at the level of the ciphertext they
// meet (FLEXIBLEAUTO re-encodes a plaintext at its operand's level).
#include "kway.hpp"

#include <chrono>
#include <exception>
#include <thread>

#include <cstdio>
#include <map>
#include <string>
#include <cstdlib>

#include <cmath>
#include <stdexcept>

namespace fhe {
namespace kwaySort {

namespace {
long ipow(long b, long e) {
    long r = 1;
    while (e-- > 0) r *= b;
    return r;
}
long nextPow2(long n) {
    long p = 1;
    while (p < n) p <<= 1;
    return p;
}
}  // namespace

// Masking.cpp:25-48: stage -> (m, logDist, slope).  Rounds r = 0, 1, ... have
// 1 + r * ceil(k/2) stages; f(r) = r + r(r-1)/2 * ceil(k/2) stages precede round r.
std::tuple<int, int, int> sortType(int k, int M, int stage) {
    (void)M;
    const int up = (k + 1) / 2;
    int r = 0;
    while (stage >= r + 1 + r * (r + 1) / 2 * up) ++r;
    const int n = stage - (r + r * (r - 1) / 2 * up);
    const int m = (n + up - 1) / up;
    const int slope = n == 0 ? 0 : (n - 1) % up + 1;
    return std::make_tuple(m, r - m, slope);
}

int stageCount(int k, int M) { return M + M * (M - 1) / 2 * ((k + 1) / 2); }

// Masking.cpp:50-146.  res[0][slot] = size of the sorting group the slot takes
// part in (0: none), res[1][slot] = its position (1-based) in that group.
std::vector<std::vector<int>> genIndices(long numSlots, long k, long M, long m, long logDist, long slope) {
    std::vector<std::vector<int>> res(2, std::vector<int>((size_t)numSlots, 0));
    const long km = ipow(k, m), dist = ipow(k, logDist), next = ipow(k, m + 1), total = ipow(k, M);
    auto put = [&](long here, int a, int b) {
        res[0][(size_t)here] = a;
        res[1][(size_t)here] = b;
    };
    // one anti-diagonal walk starting at (row, col): positions loc = 1, 2, ...;
    // when the walk ends, the whole chain is re-labelled from its far end
    auto diagonal = [&](long start, long row0, long col0) {
        long row = row0, col = col0;
        int loc = 1;
        while (row < km && col >= 0) {
            for (long d = 0; d < dist; ++d) {
                const long here = start + dist * (col + k * row) + d;
                res[0][(size_t)here] = loc;
                if (row == km - 1 || col - slope < 0) {
                    for (int i = 0; i < loc; ++i) {
                        const long h2 = start + dist * ((col + i * slope) + k * (row - i)) + d;
                        res[1][(size_t)h2] = loc - i;
                        res[0][(size_t)h2] += i;
                    }
                }
            }
            ++loc;
            ++row;
            col -= slope;
        }
    };
    for (long start = 0; start < total; start += dist * next) {
        if (slope == 0) {
            for (long s = 0; s < km; ++s)
                for (long col = 0; col < k; ++col)  // row stays s: loc = col + 1
                    for (long d = 0; d < dist; ++d) put(start + dist * (s + km * col) + d, (int)k, (int)col + 1);
        } else if (slope > k / 2) {
            for (long t = 0; t + 1 < km; ++t) {
                const long col = k - k / 2;
                for (long loc = 1; loc < k; ++loc)
                    for (long d = 0; d < dist; ++d)
                        put(start + dist * (col + k * t + loc - 1) + d, (int)(k - 1), (int)loc);
            }
        } else {
            for (long t = slope; t < k; ++t) diagonal(start, 0, t);
            for (long s = 1; s + 1 < km; ++s)
                for (long t = k - slope; t < k; ++t) diagonal(start, s, t);
        }
    }
    return res;
}

void genMask(const std::vector<std::vector<int>> &indices, long index0, long index1, std::vector<double> &mask) {
    const size_t ns = indices[0].size();
    mask.assign(ns, 0.0);
    for (size_t i = 0; i < ns; ++i)
        if (indices[0][i] == index0 && indices[1][i] == index1) mask[i] = 1.0;
}

long getRotateDistance(long k, long logDist, long slope) {  // Masking.cpp:155-165
    const long dist = ipow(k, logDist);
    return (slope == 0 || slope == k / 2 + 1) ? dist : dist * (k - slope);
}

std::vector<int> rotationIndices(int N) {  // kway_adapter.h:45-49
    std::vector<int> r;
    for (int i = 1; i < N; i *= 2) {
        r.push_back(i);
        r.push_back(-i);
    }
    return r;
}

// ------------------------------------------------------------- Sorter ----
Sorter::Sorter(Engine &cc_, long numSlots_, long k_, long M_)
    : cc(cc_), numSlots(numSlots_), k(k_), M(M_), level{0, 1, 3, 5, 6, 7} {
    if (k != 2 && k != 3 && k != 5) throw std::invalid_argument("k-way: only k = 2, 3, 5 are supported");
    if (M < 1 || ipow(k, M) != numSlots) throw std::invalid_argument("k-way: k^M must equal the input length");
}

const Plaintext &Sorter::mask(const std::vector<double> &v, const Ciphertext &like) {
    auto key = std::make_pair(v, like.level);
    auto it = masks.find(key);
    if (it != masks.end()) return *it->second;
    return *(masks[key] = cc.encode(v, like.slots, like.level));
}

// EvalUtils::checkLevelAndBoot (EvalUtils.cpp:59-86): bootstrap when fewer
// than need + 1 levels remain (cfg.boot); without a bootstrapper that is an error
CtPtr checkLevelAndBoot(Engine &cc, const CtPtr &c, int need, const SignConfig &cfg, bool *booted) {
    if (booted) *booted = false;
    if (cc.params().L - c->level >= need + 1) return c;
    if (!cfg.boot) throw std::runtime_error("k-way: no levels left (set up bootstrapping for this depth)");
    if (booted) *booted = true;
    return cfg.boot(*c);
}

void Sorter::checkLevel(CtPtr &c, int need, const SignConfig &cfg) {
    bool booted = false;
    CtPtr in = c;
    c = checkLevelAndBoot(cc, c, need, cfg, &booted);
    if (!booted) return;
    ++bootstraps;
    if (std::getenv("FHE_KWAY_TRACE")) {
        const auto a = cc.decrypt(*in), b = cc.decrypt(*c);
        double e = 0, mx = 0;
        for (size_t i = 0; i < (size_t)numSlots && i < a.size(); ++i) {
            e = std::max(e, std::fabs(a[i] - b[i]));
            mx = std::max(mx, std::fabs(a[i]));
        }
        std::fprintf(stderr, "  boot %d at level %d: max|in| %.6g, max|out - in| %.3g\n", bootstraps, in->level, mx, e);
    }
}

namespace {
// FHE_KWAY_TIMES (diagnostics): wall time per phase of sorter(), the engine
// synchronised at every phase boundary; printed to stderr after the sort
struct PhaseTimes {
    bool on = std::getenv("FHE_KWAY_TIMES") != nullptr;
    std::map<std::string, double> s;
    std::chrono::steady_clock::time_point t0;
    void start(Engine &cc) {
        if (!on) return;
        cc.sync();
        t0 = std::chrono::steady_clock::now();
    }
    void stop(Engine &cc, const char *what) {
        if (!on) return;
        cc.sync();
        s[what] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
};
// run `lane` on a second host thread while `main` runs on this one; both
// finish (and the lane's stream drains) before any exception is rethrown
template <class A, class B>
void concurrently(A &&main, B &&lane) {
    std::exception_ptr err;
    std::thread t([&] {
        try {
            lane();
        } catch (...) {
            err = std::current_exception();
        }
    });
    try {
        main();
    } catch (...) {
        t.join();
        throw;
    }
    t.join();
    if (err) std::rethrow_exception(err);
}
}  // namespace

void Sorter::checkLevel2(CtPtr &c1, CtPtr &c2, int need, const SignConfig &cfg) {
    const int L = cc.params().L;
    if (!laneEng || L - c1->level >= need + 1 || L - c2->level >= need + 1) {
        checkLevel(c1, need, cfg);  // at most one bootstrap: on this engine
        checkLevel(c2, need, cfg);
        return;
    }
    // both need a bootstrap: c2's runs on the lane (its own bootstrapper)
    if (!cfg.boot || !laneCfg.boot) throw std::runtime_error("k-way: no levels left (set up bootstrapping for this depth)");
    cc.sync();
    CtPtr b2;
    concurrently([&] { c1 = cfg.boot(*c1); },
                 [&] {
                     b2 = laneCfg.boot(*c2);
                     laneEng->sync();
                 });
    c2 = b2;
    bootstraps += 2;
    cc.ctr += laneEng->ctr;
    laneEng->ctr = Counters();
}

// EvalUtils.cpp:113-146: binary decomposition, ascending powers of two
CtPtr Sorter::leftRotate(const CtPtr &c, long r) {
    CtPtr o = c;
    for (long p = 1; r > 0; p <<= 1, r >>= 1)
        if (r & 1) o = cc.rotate(*o, p);
    return o;
}
CtPtr Sorter::rightRotate(const CtPtr &c, long r) {
    CtPtr o = c;
    for (long p = 1; r > 0; p <<= 1, r >>= 1)
        if (r & 1) o = cc.rotate(*o, -p);
    return o;
}
// Several leftRotate (amt > 0) / rightRotate (amt < 0) chains at once: the j-th
// power-of-two rotation of every chain at one level runs as one batch with a
// rotation per member (Engine::rotate_members), so a stage's 4-12 rotation
// chains cost one key-switch pipeline per step instead of one per rotation.
// Each chain applies the same rotations in the same order as above.
std::vector<CtPtr> Sorter::rotateMany(const std::vector<CtPtr> &src, const std::vector<long> &amt) {
    const size_t m = src.size();
    std::vector<CtPtr> cur = src;
    std::vector<long> rem(m), pw(m, 1);
    for (size_t i = 0; i < m; ++i) rem[i] = amt[i] < 0 ? -amt[i] : amt[i];
    for (;;) {
        std::map<int, std::vector<size_t>> at;  // level -> chains with a rotation this step
        std::vector<long> step(m, 0);
        for (size_t i = 0; i < m; ++i) {
            while (rem[i] > 0 && !(rem[i] & 1)) {
                rem[i] >>= 1;
                pw[i] <<= 1;
            }
            if (rem[i] == 0) continue;
            step[i] = amt[i] > 0 ? pw[i] : -pw[i];
            rem[i] >>= 1;
            pw[i] <<= 1;
            at[cur[i]->level].push_back(i);
        }
        if (at.empty()) break;
        for (auto &kv : at) {
            const auto &idx = kv.second;
            if (idx.size() == 1) {
                cur[idx[0]] = cc.rotate(*cur[idx[0]], step[idx[0]]);
                continue;
            }
            std::vector<const Ciphertext *> ptrs;
            std::vector<long> ks;
            for (size_t i : idx) {
                ptrs.push_back(cur[i].get());
                ks.push_back(step[i]);
            }
            const CtPtr r = cc.rotate_members(*cc.stack(ptrs), ks);
            for (size_t j = 0; j < idx.size(); ++j) cur[idx[j]] = cc.member(*r, (int)j);
        }
    }
    return cur;
}

// EvalUtils::flipCtxt(ctxt, mask) = mask - ctxt (EvalUtils.cpp:102-105)
CtPtr Sorter::flip(const CtPtr &c, const std::vector<double> &m) { return cc.plain_sub(mask(m, *c), *c); }
CtPtr Sorter::maskMul(const CtPtr &c, const std::vector<double> &m) { return cc.mul_plain(*c, mask(m, *c)); }

// SortUtils.cpp:5-16: cmp * (a - b) + b  (= max(a, b) when cmp = [a > b])
CtPtr Sorter::fcnL(const CtPtr &a, const CtPtr &b, const CtPtr &cmp) {
    return cc.add(*cc.mul(*cc.sub(*a, *b), *cmp), *b);
}
// SortUtils.cpp:32-54: out = [min, max]
void Sorter::twoSorter(const CtPtr &a, const CtPtr &b, const CtPtr &cmp, CtPtr *out) {
    out[1] = fcnL(a, b, cmp);
    out[0] = cc.sub(*cc.add(*a, *b), *out[1]);
}
// SortUtils.cpp:56-77; cmp = [a>b, a>c, b>c]
void Sorter::threeSorter(const CtPtr *x, const CtPtr *cmp, CtPtr *out) {
    CtPtr ab[2], abc[2];
    twoSorter(x[0], x[1], cmp[0], ab);
    twoSorter(cmp[1], cmp[2], cmp[0], abc);     // [min(a,b) > c, max(a,b) > c]
    out[2] = fcnL(ab[1], x[2], abc[1]);          // compareMax
    out[0] = fcnL(x[2], ab[0], abc[0]);          // compareMin
    out[1] = cc.sub(*cc.sub(*cc.add(*cc.add(*x[0], *x[1]), *x[2]), *out[0]), *out[2]);
}
// SortUtils.cpp:79-129; cmp = [a>b, a>c, a>d, b>c, b>d, c>d]
void Sorter::fourSorter(const CtPtr *x, const CtPtr *cmp, CtPtr *out) {
    CtPtr ab[2], cd[2], vsC[2], vsD[2], Mx[2], mn[2];
    twoSorter(x[0], x[1], cmp[0], ab);
    twoSorter(x[2], x[3], cmp[5], cd);
    twoSorter(cmp[1], cmp[3], cmp[0], vsC);
    twoSorter(cmp[2], cmp[4], cmp[0], vsD);
    twoSorter(vsC[1], vsD[1], cmp[5], Mx);
    twoSorter(vsC[0], vsD[0], cmp[5], mn);
    out[3] = fcnL(ab[1], cd[1], Mx[1]);
    const CtPtr left = fcnL(ab[0], cd[1], mn[1]), right = fcnL(ab[1], cd[0], Mx[0]);
    out[2] = fcnL(left, right, Mx[1]);
    out[0] = fcnL(cd[0], ab[0], mn[0]);
    CtPtr s = x[0];
    for (int i = 1; i < 4; ++i) s = cc.add(*s, *x[i]);
    for (int i : {0, 2, 3}) s = cc.sub(*s, *out[i]);
    out[1] = s;
}
// SortUtils.cpp:131-208; cmp = [a>b a>c a>d a>e b>c b>d b>e c>d c>e d>e]
void Sorter::fiveSorter(const CtPtr *x, const CtPtr *cmp, CtPtr *out) {
    const CtPtr abcIn[3] = {x[0], x[1], x[2]}, abcCmp[3] = {cmp[0], cmp[1], cmp[4]};
    CtPtr abc[3], de[2];
    threeSorter(abcIn, abcCmp, abc);
    twoSorter(x[3], x[4], cmp[9], de);
    const CtPtr vsDIn[3] = {cmp[2], cmp[5], cmp[7]}, vsEIn[3] = {cmp[3], cmp[6], cmp[8]};
    CtPtr vsD[3], vsE[3];
    threeSorter(vsDIn, abcCmp, vsD);
    threeSorter(vsEIn, abcCmp, vsE);
    CtPtr hi[2], mid[2], lo[2];
    twoSorter(vsD[2], vsE[2], cmp[9], hi);
    twoSorter(vsD[1], vsE[1], cmp[9], mid);
    twoSorter(vsD[0], vsE[0], cmp[9], lo);
    out[4] = fcnL(abc[2], de[1], hi[1]);
    out[0] = fcnL(de[0], abc[0], lo[0]);
    CtPtr left = fcnL(abc[1], de[1], mid[1]), right = fcnL(abc[2], de[0], hi[0]);
    out[3] = fcnL(left, right, hi[1]);
    left = fcnL(de[0], abc[1], mid[0]);
    right = fcnL(de[1], abc[0], lo[1]);
    out[1] = fcnL(right, left, lo[0]);
    CtPtr s = x[0];
    for (int i = 1; i < 5; ++i) s = cc.add(*s, *x[i]);
    for (int i : {0, 1, 3, 4}) s = cc.sub(*s, *out[i]);
    out[2] = s;
}
std::vector<CtPtr> Sorter::kSorter(int kk, const std::vector<CtPtr> &x, const std::vector<CtPtr> &cmp) {
    const size_t nx = kk == 1 ? 2 : (size_t)kk, nc = kk == 1 ? 1 : (size_t)(kk * (kk - 1) / 2);
    if (kk < 1 || kk > 5 || x.size() != nx || cmp.size() != nc)
        throw std::invalid_argument("kway sorter: kk in 1..5 with kk (2 for fcnL) inputs and kk(kk-1)/2 comparisons");
    std::vector<CtPtr> out(kk == 1 ? 1 : (size_t)kk);
    switch (kk) {
    case 1: out[0] = fcnL(x[0], x[1], cmp[0]); break;
    case 2: twoSorter(x[0], x[1], cmp[0], out.data()); break;
    case 3: threeSorter(x.data(), cmp.data(), out.data()); break;
    case 4: fourSorter(x.data(), cmp.data(), out.data()); break;
    default: fiveSorter(x.data(), cmp.data(), out.data()); break;
    }
    return out;
}
// SortUtils.cpp:424-433
CtPtr Sorter::slotAssemble(const CtPtr *s, long num, long shift) {
    std::vector<CtPtr> src;
    std::vector<long> amt;
    for (long i = 1; i < num; ++i) {
        src.push_back(s[i]);
        amt.push_back(-i * shift);
    }
    const auto r = rotateMany(src, amt);
    CtPtr o = s[0];
    for (auto &c : r) o = cc.add(*o, *c);
    return o;
}

namespace {
std::vector<double> groupMask(const std::vector<std::vector<int>> &ind, long size) {
    std::vector<double> m;
    genMask(ind, size, 1, m);
    return m;
}
}  // namespace

// Sorter.cpp:9-36 (+ slotMatching2, SortUtils.cpp:210-217)
CtPtr Sorter::runTwoSorter(const CtPtr &x, const std::vector<std::vector<int>> &ind, long shift, const CtPtr &c) {
    const auto m2 = groupMask(ind, 2);
    CtPtr s[2];
    twoSorter(x, leftRotate(x, shift), c, s);
    for (auto &v : s) v = maskMul(v, m2);
    return slotAssemble(s, 2, shift);
}
// Sorter.cpp:38-68 (+ slotMatching3, SortUtils.cpp:219-241)
CtPtr Sorter::runThreeSorter(const CtPtr &x, const std::vector<std::vector<int>> &ind, long shift, const CtPtr &c) {
    const auto m3 = groupMask(ind, 3);
    const auto r = rotateMany({x, x, c, c}, {shift, 2 * shift, shift, 2 * shift});
    const CtPtr xs[3] = {x, r[0], r[1]};
    const CtPtr cs[3] = {flip(r[2], m3), c, flip(r[3], m3)};
    CtPtr s[3];
    threeSorter(xs, cs, s);
    for (auto &v : s) v = maskMul(v, m3);
    return slotAssemble(s, 3, shift);
}
// Sorter.cpp:70-85 (+ slotMatching4, SortUtils.cpp:243-287; the reference's
// masked products at :262-267 are overwritten before use and are skipped)
CtPtr Sorter::runFourSorter(const CtPtr &x, const std::vector<std::vector<int>> &ind, long shift, const CtPtr &c1,
                            const CtPtr &c2) {
    std::vector<double> m41;
    genMask(ind, 4, 1, m41);
    const auto r = rotateMany({c1, c1, c1, c2, x, x, x},
                              {shift, 2 * shift, 3 * shift, shift, shift, 2 * shift, 3 * shift});
    CtPtr cs[6];
    cs[2] = c1;
    cs[0] = flip(r[0], m41);
    cs[3] = flip(r[1], m41);
    cs[5] = flip(r[2], m41);
    cs[1] = c2;
    cs[4] = r[3];
    CtPtr xs[4];
    xs[0] = maskMul(x, m41);
    for (int i = 1; i < 4; ++i) xs[i] = maskMul(r[3 + (size_t)i], m41);
    CtPtr s[4];
    fourSorter(xs, cs, s);
    return slotAssemble(s, 4, shift);
}
// Sorter.cpp:87-115 (+ slotMatching5, SortUtils.cpp:289-323)
CtPtr Sorter::runFiveSorter(const CtPtr &x, const std::vector<std::vector<int>> &ind, long shift, const CtPtr &c1,
                            const CtPtr &c2) {
    const auto m5 = groupMask(ind, 5);
    CtPtr xs[5], cs[10];
    const auto r = rotateMany({x, x, x, x, c1, c1, c1, c1, c2, c2, c2, c2},
                              {shift, 2 * shift, 3 * shift, 4 * shift, shift, 2 * shift, 3 * shift, 4 * shift,
                               shift, 2 * shift, 3 * shift, 4 * shift});
    xs[0] = x;
    for (int i = 1; i < 5; ++i) xs[i] = r[(size_t)i - 1];
    cs[3] = c1;
    cs[0] = r[4];
    cs[4] = r[5];
    cs[7] = r[6];
    cs[9] = r[7];
    cs[2] = c2;
    cs[6] = r[8];
    cs[1] = r[9];
    cs[5] = r[10];
    cs[8] = r[11];
    for (int i : {0, 1, 4, 5, 7, 8, 9}) cs[i] = flip(cs[i], m5);
    CtPtr s[5];
    fiveSorter(xs, cs, s);
    for (auto &v : s) v = maskMul(v, m5);
    return slotAssemble(s, 5, shift);
}
// Sorter.cpp:117-185 (+ slotMatching2345, SortUtils.cpp:325-422)
CtPtr Sorter::run2345Sorter(const CtPtr &x, const std::vector<std::vector<int>> &ind, long shift, const CtPtr &c1,
                            const CtPtr &c2) {
    const size_t ns = ind[0].size();
    std::vector<double> m2345(ns, 0.0), m45(ns, 0.0), m345(ns, 0.0), m3(ns, 0.0), m4(ns, 0.0), m5(ns, 0.0);
    for (size_t i = 0; i < ns; ++i) {
        if (ind[1][i] != 1) continue;
        const int g = ind[0][i];
        if (g >= 2 && g <= 5) m2345[i] = 1.0;
        if (g >= 3 && g <= 5) m345[i] = 1.0;
        if (g == 4 || g == 5) m45[i] = 1.0;
        if (g == 3) m3[i] = 1.0;
        if (g == 4) m4[i] = 1.0;
        if (g == 5) m5[i] = 1.0;
    }
    CtPtr xs[5], cs[10];
    const auto r = rotateMany({x, x, x, x, c1, c1, c1, c1, c2, c2, c2, c2},
                              {shift, 2 * shift, 3 * shift, 4 * shift, shift, 2 * shift, 3 * shift, 4 * shift,
                               shift, 2 * shift, 3 * shift, 4 * shift});
    xs[0] = x;
    for (int i = 1; i < 5; ++i) xs[i] = r[(size_t)i - 1];
    const CtPtr *c1r = &r[4] - 1, *c2r = &r[8] - 1;  // c1r[i] = leftRotate(c1, i shift), i >= 1
    cs[0] = flip(c1r[1], m2345);
    cs[1] = cc.add(*maskMul(c1, m3), *flip(maskMul(c2r[2], m45), m45));
    cs[2] = cc.add(*maskMul(c1, m4), *maskMul(c2, m5));
    cs[3] = maskMul(c1, m5);
    cs[4] = flip(maskMul(c1r[2], m345), m345);
    cs[5] = flip(maskMul(c2r[3], m45), m45);
    cs[6] = maskMul(c2r[1], m5);
    cs[7] = flip(maskMul(c1r[3], m45), m45);
    cs[8] = flip(maskMul(c2r[4], m5), m5);
    cs[9] = flip(maskMul(c1r[4], m5), m5);
    CtPtr s[5];
    fiveSorter(xs, cs, s);
    s[0] = maskMul(s[0], m2345);
    s[1] = maskMul(s[1], m2345);
    s[2] = maskMul(s[2], m345);
    s[3] = maskMul(s[3], m45);
    s[4] = maskMul(s[4], m5);
    return slotAssemble(s, 5, shift);
}

// Sorter.cpp:187-256.  rot = the input moved so that every slot meets its
// comparison partner; fix (optional) = the slots outside every group.
void Sorter::rightRotateForSort(const CtPtr &x, const std::vector<std::vector<int>> &ind, long logDist, long slope,
                                CtPtr &rot, CtPtr *fix) {
    const size_t ns = (size_t)numSlots;
    std::vector<double> left(ns, 0.0);
    std::vector<std::vector<double>> right((size_t)k, std::vector<double>(ns, 0.0));
    for (size_t i = 0; i < ns; ++i) {
        if (ind[1][i] < ind[0][i]) left[i] = 1.0;
        if (ind[0][i] > 0 && ind[0][i] == ind[1][i]) right[(size_t)ind[0][i] - 1][i] = 1.0;
    }
    const CtPtr xl = maskMul(x, left);
    const long r = getRotateDistance(k, logDist, slope);
    if (slope == 0 || slope == k / 2 + 1) {
        const long g = slope == 0 ? k - 1 : k - 2;  // the one group size present
        const CtPtr xr = maskMul(x, right[(size_t)g]);
        if (slope != 0 && fix) *fix = cc.sub(*cc.sub(*x, *xl), *xr);
        const auto rr = rotateMany({xl, xr}, {-r, g * r});
        rot = cc.add(*rr[0], *rr[1]);
        return;
    }
    std::vector<CtPtr> xr((size_t)k);
    for (long i = 0; i < k; ++i) xr[(size_t)i] = maskMul(x, right[(size_t)i]);
    if (fix) {
        CtPtr f = cc.sub(*x, *xl);
        for (long i = 0; i < k; ++i) f = cc.sub(*f, *xr[(size_t)i]);
        *fix = f;
    }
    std::vector<CtPtr> src{xl};
    std::vector<long> amt{-r};
    for (long i = 1; i < k; ++i) {
        src.push_back(xr[(size_t)i]);
        amt.push_back(i * r);
    }
    const auto rr = rotateMany(src, amt);
    rot = rr[0];
    for (size_t i = 1; i < rr.size(); ++i) rot = cc.add(*rot, *rr[i]);
}

// Sorter.cpp:258-268: comp = [x > rot(x)]
CtPtr Sorter::comparisonForSort(const CtPtr &x, const std::vector<std::vector<int>> &ind, long logDist, long slope,
                                CtPtr &fix, const SignConfig &cfg) {
    CtPtr rot;
    rightRotateForSort(x, ind, logDist, slope, rot, &fix);
    return comp.compare(cc, *x, *rot, SignFunc::CompositeSign, cfg);
}
// Sorter.cpp:270-287 (the second rotation's fix part is unused and not formed)
void Sorter::comparisonForSort2(const CtPtr &x, const std::vector<std::vector<int>> &ind, long logDist, long slope,
                                CtPtr &c1, CtPtr &c2, CtPtr &fix, const SignConfig &cfg) {
    CtPtr r1, r2;
    rightRotateForSort(x, ind, logDist, slope, r1, &fix);
    rightRotateForSort(r1, ind, logDist, slope, r2, nullptr);
    if (!laneEng) {
        c1 = comp.compare(cc, *x, *r1, SignFunc::CompositeSign, cfg);
        c2 = comp.compare(cc, *x, *r2, SignFunc::CompositeSign, cfg);
        return;
    }
    cc.sync();  // x, r2 complete before the lane's stream reads them
    CtPtr d2;
    concurrently([&] { c1 = comp.compare(cc, *x, *r1, SignFunc::CompositeSign, cfg); },
                 [&] {
                     d2 = comp.compare(*laneEng, *x, *r2, SignFunc::CompositeSign, laneCfg);
                     laneEng->sync();
                 });
    c2 = d2;
    cc.ctr += laneEng->ctr;
    laneEng->ctr = Counters();
}

// Sorter.cpp:289-404
CtPtr Sorter::sorter(const Ciphertext &input, const SignConfig &cfg) {
    CtPtr ct = cc.clone(input), fix, c1, c2;
    const int stages = stageCount((int)k, (int)M);
    stagesRun = 0;
    PhaseTimes T;
    bootstraps = 0;
    for (int stage = 0; stage < stages; ++stage) {
        int m, logDist, slope;
        std::tie(m, logDist, slope) = sortType((int)k, (int)M, stage);
        const long shift = getRotateDistance(k, logDist, slope);
        const auto ind = genIndices(numSlots, k, M, m, logDist, slope);
        if (slope == 0) {
            T.start(cc);
            checkLevel(ct, level[(size_t)k], cfg);
            T.stop(cc, "level checks / bootstraps");
            if (k == 5) {
                T.start(cc);
                comparisonForSort2(ct, ind, logDist, slope, c1, c2, fix, cfg);
                T.stop(cc, "comparisons");
                T.start(cc);
                checkLevel2(c1, c2, level[5], cfg);
                T.stop(cc, "level checks / bootstraps");
                T.start(cc);
                ct = runFiveSorter(ct, ind, shift, c1, c2);
                T.stop(cc, "sorting networks");
            } else {
                T.start(cc);
                c1 = comparisonForSort(ct, ind, logDist, slope, fix, cfg);
                T.stop(cc, "comparisons");
                T.start(cc);
                checkLevel(c1, level[(size_t)k], cfg);
                T.stop(cc, "level checks / bootstraps");
                ct = k == 2 ? runTwoSorter(ct, ind, shift, c1) : runThreeSorter(ct, ind, shift, c1);
            }
        } else if (slope == k / 2 + 1) {  // k = 3 or 5 (k = 2 has slopes 0, 1 only)
            T.start(cc);
            checkLevel(ct, level[(size_t)k - 1], cfg);
            T.stop(cc, "level checks / bootstraps");
            if (k == 3) {
                T.start(cc);
                c1 = comparisonForSort(ct, ind, logDist, slope, fix, cfg);
                T.stop(cc, "comparisons");
                T.start(cc);
                checkLevel(c1, level[2], cfg);
                T.stop(cc, "level checks / bootstraps");
                T.start(cc);
                ct = runTwoSorter(ct, ind, shift, c1);
                T.stop(cc, "sorting networks");
            } else {
                T.start(cc);
                comparisonForSort2(ct, ind, logDist, slope, c1, c2, fix, cfg);
                T.stop(cc, "comparisons");
                T.start(cc);
                checkLevel2(c1, c2, level[4], cfg);
                T.stop(cc, "level checks / bootstraps");
                T.start(cc);
                ct = runFourSorter(ct, ind, shift, c1, c2);
                T.stop(cc, "sorting networks");
            }
            ct = cc.add(*ct, *fix);
        } else if (k == 5 && slope == 1) {
            T.start(cc);
            checkLevel(ct, level[5], cfg);
            T.stop(cc, "level checks / bootstraps");
            T.start(cc);
            comparisonForSort2(ct, ind, logDist, slope, c1, c2, fix, cfg);
            T.stop(cc, "comparisons");
            T.start(cc);
            checkLevel2(c1, c2, level[5], cfg);
            T.stop(cc, "level checks / bootstraps");
            T.start(cc);
            ct = cc.add(*run2345Sorter(ct, ind, shift, c1, c2), *fix);
            T.stop(cc, "sorting networks");
        } else if ((k == 5 && slope == 2) || (k == 3 && slope == 1)) {
            T.start(cc);
            checkLevel(ct, level[3], cfg);
            T.stop(cc, "level checks / bootstraps");
            T.start(cc);
            c1 = comparisonForSort(ct, ind, logDist, slope, fix, cfg);
            T.stop(cc, "comparisons");
            T.start(cc);
            checkLevel(c1, level[2], cfg);  // Sorter.cpp:373-376: checked for 2, then for 3
            T.stop(cc, "level checks / bootstraps");
            T.start(cc);
            const CtPtr two = runTwoSorter(ct, ind, shift, c1);
            T.stop(cc, "sorting networks");
            T.start(cc);
            checkLevel(c1, level[3], cfg);
            T.stop(cc, "level checks / bootstraps");
            T.start(cc);
            const CtPtr three = runThreeSorter(ct, ind, shift, c1);
            T.stop(cc, "sorting networks");
            ct = cc.add(*cc.add(*two, *fix), *three);
        } else if (k == 2 && slope == 1) {
            T.start(cc);
            checkLevel(ct, level[2], cfg);
            T.stop(cc, "level checks / bootstraps");
            T.start(cc);
            c1 = comparisonForSort(ct, ind, logDist, slope, fix, cfg);
            T.stop(cc, "comparisons");
            T.start(cc);
            checkLevel(c1, level[2], cfg);
            T.stop(cc, "level checks / bootstraps");
            T.start(cc);
            ct = cc.add(*runTwoSorter(ct, ind, shift, c1), *fix);
            T.stop(cc, "sorting networks");
        } else {
            throw std::invalid_argument("k-way: no matching k and slope");
        }
        ++stagesRun;
        if (std::getenv("FHE_KWAY_TRACE")) {  // diagnostics: decrypted range after every stage
            const auto v = cc.decrypt(*ct);
            double lo = 1e300, hi = -1e300;
            for (size_t i = 0; i < (size_t)numSlots && i < v.size(); ++i) {
                lo = std::min(lo, v[i]);
                hi = std::max(hi, v[i]);
            }
            std::fprintf(stderr, "kway stage %d (m %d dist %d slope %d): level %d, values [%.6g, %.6g], boots %d\n",
                         stage, m, logDist, slope, ct->level, lo, hi, bootstraps);
        }
    }
    if (T.on)
        for (auto &kv : T.s) std::fprintf(stderr, "k-way %-26s %8.3f s\n", kv.first.c_str(), kv.second);
    return ct;
}

}  // namespace kwaySort
}  // namespace fhe
