// CPU ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h header).
//
// Restatement of the reference's k-way sorting network (src/k-way/*.cpp,
// src/kway_adapter.h) on the oracle's RNS-CKKS core, without bootstrapping:
// where EvalUtils::checkLevelAndBoot (src/k-way/EvalUtils.cpp:59-86) would
// bootstrap, the context must still hold the levels ("no levels left"
// otherwise).  Masks are encoded at the level of the ciphertext they meet.
#include <map>
#include <stdexcept>

#include "oracle.h"

namespace oracle {
namespace kway {

namespace {
long pw(long b, long e) {
    long r = 1;
    for (long i = 0; i < e; ++i) r *= b;
    return r;
}
}  // namespace

int stage_count(int k, int M) { return M + M * (M - 1) / 2 * ((k + 1) / 2); }

// Masking.cpp:25-48
void sort_type(int k, int stage, int &m, int &log_dist, int &slope) {
    const int up = (k + 1) / 2;
    int r = 0;
    for (;;) {  // r = the round containing `stage`; round r starts after r + r(r-1)/2 * up stages
        const int next_start = (r + 1) + (r + 1) * r / 2 * up;
        if (stage < next_start) break;
        ++r;
    }
    const int off = stage - (r + r * (r - 1) / 2 * up);
    m = (off + up - 1) / up;
    log_dist = r - m;
    slope = off == 0 ? 0 : 1 + (off - 1) % up;
}

long rotate_distance(long k, long log_dist, long slope) {  // Masking.cpp:155-165
    const long d = pw(k, log_dist);
    if (slope == 0 || slope == k / 2 + 1) return d;
    return d * (k - slope);
}

// Masking.cpp:50-146 -> (group size, position) per slot
void gen_indices(long ns, long k, long M, long m, long log_dist, long slope, std::vector<int> &grp,
                 std::vector<int> &pos) {
    grp.assign((size_t)ns, 0);
    pos.assign((size_t)ns, 0);
    const long km = pw(k, m), dist = pw(k, log_dist), block = dist * pw(k, m + 1), total = pw(k, M);
    auto slot = [&](long start, long row, long col, long d) { return (size_t)(start + dist * (col + k * row) + d); };
    auto walk = [&](long start, long row, long col) {
        for (int loc = 1; row < km && col >= 0; ++loc, ++row, col -= slope) {
            for (long d = 0; d < dist; ++d) {
                grp[slot(start, row, col, d)] = loc;
                if (row != km - 1 && col - slope >= 0) continue;
                for (int i = 0; i < loc; ++i) {  // chain complete: number it from this end
                    const size_t h = slot(start, row - i, col + i * slope, d);
                    pos[h] = loc - i;
                    grp[h] += i;
                }
            }
        }
    };
    for (long start = 0; start < total; start += block) {
        if (slope == 0) {
            for (long s = 0; s < km; ++s)
                for (long c = 0; c < k; ++c)
                    for (long d = 0; d < dist; ++d) {
                        const size_t h = (size_t)(start + dist * (s + km * c) + d);
                        grp[h] = (int)k;
                        pos[h] = (int)c + 1;
                    }
        } else if (slope > k / 2) {
            const long c0 = k - k / 2;
            for (long t = 0; t < km - 1; ++t)
                for (long loc = 1; loc < k; ++loc)
                    for (long d = 0; d < dist; ++d) {
                        const size_t h = (size_t)(start + dist * (c0 + k * t + loc - 1) + d);
                        grp[h] = (int)(k - 1);
                        pos[h] = (int)loc;
                    }
        } else {
            for (long t = slope; t < k; ++t) walk(start, 0, t);
            for (long s = 1; s < km - 1; ++s)
                for (long t = k - slope; t < k; ++t) walk(start, s, t);
        }
    }
}

std::vector<int> rotation_indices(int N) {
    std::vector<int> r;
    for (int p = 1; p < N; p <<= 1) {
        r.push_back(p);
        r.push_back(-p);
    }
    return r;
}

namespace {

using Mask = std::vector<double>;

struct Net {
    Context &cc;
    long ns, k, M;
    SignConfig cfg;
    static constexpr int lv[6] = {0, 1, 3, 5, 6, 7};  // Sorter.h:85-93
    std::map<std::pair<Mask, int>, Plaintext> cache;
    std::vector<int> grp, pos;

    const Plaintext &pt(const Mask &m, const Ciphertext &c) {
        auto key = std::make_pair(m, c.level);
        auto it = cache.find(key);
        if (it == cache.end()) it = cache.emplace(key, cc.encode(m, c.slots, c.level)).first;
        return it->second;
    }
    Mask sel(int g, int p) const {  // genMask(indices, g, p)
        Mask m((size_t)ns, 0.0);
        for (size_t i = 0; i < (size_t)ns; ++i) m[i] = (grp[i] == g && pos[i] == p) ? 1.0 : 0.0;
        return m;
    }
    // EvalUtils::checkLevelAndBoot (EvalUtils.cpp:59-86): bootstrap when fewer
    // than l + 1 levels remain (cfg.boot); without a bootstrapper that is an error
    void need(CtPtr &c, int l) const {
        if (cc.P.L - c->level >= l + 1) return;
        if (!cfg.boot) throw std::runtime_error("k-way: no levels left (set up bootstrapping for this depth)");
        c = cfg.boot(*c);
    }
    CtPtr rot(CtPtr c, long r, long sign) {  // EvalUtils::leftRotate / rightRotate
        for (long p = 1; r > 0; p *= 2, r /= 2)
            if (r % 2) c = cc.rotate(*c, sign * p);
        return c;
    }
    CtPtr L(const CtPtr &c, long r) { return rot(c, r, 1); }
    CtPtr R(const CtPtr &c, long r) { return rot(c, r, -1); }
    CtPtr mul(const CtPtr &c, const Mask &m) { return cc.mul_plain(*c, pt(m, *c)); }
    CtPtr flip(const CtPtr &c, const Mask &m) { return cc.plain_sub(pt(m, *c), *c); }
    CtPtr fcn(const CtPtr &a, const CtPtr &b, const CtPtr &s) { return cc.add(*cc.mul(*cc.sub(*a, *b), *s), *b); }
    CtPtr vmax(const CtPtr &a, const CtPtr &b, const CtPtr &s) { return fcn(a, b, s); }
    CtPtr vmin(const CtPtr &a, const CtPtr &b, const CtPtr &s) { return fcn(b, a, s); }
    void sort2(const CtPtr &a, const CtPtr &b, const CtPtr &s, CtPtr &lo, CtPtr &hi) {
        hi = fcn(a, b, s);
        lo = cc.sub(*cc.add(*a, *b), *hi);
    }
    // v = [a, b, c], s = [a>b, a>c, b>c] -> out ascending (SortUtils.cpp:56-77)
    void sort3(const CtPtr *v, const CtPtr *s, CtPtr *out) {
        CtPtr lo, hi, clo, chi;
        sort2(v[0], v[1], s[0], lo, hi);
        sort2(s[1], s[2], s[0], clo, chi);
        out[2] = vmax(hi, v[2], chi);
        out[0] = vmin(lo, v[2], clo);
        out[1] = cc.sub(*cc.sub(*cc.add(*cc.add(*v[0], *v[1]), *v[2]), *out[0]), *out[2]);
    }
    // SortUtils.cpp:79-129
    void sort4(const CtPtr *v, const CtPtr *s, CtPtr *out) {
        CtPtr l1, h1, l2, h2, cl, ch, dl, dh, Hl, Hh, ml, mh;
        sort2(v[0], v[1], s[0], l1, h1);
        sort2(v[2], v[3], s[5], l2, h2);
        sort2(s[1], s[3], s[0], cl, ch);
        sort2(s[2], s[4], s[0], dl, dh);
        sort2(ch, dh, s[5], Hl, Hh);
        sort2(cl, dl, s[5], ml, mh);
        out[3] = vmax(h1, h2, Hh);
        out[2] = vmax(vmax(l1, h2, mh), vmax(h1, l2, Hl), Hh);
        out[0] = vmin(l1, l2, ml);
        CtPtr t = cc.add(*cc.add(*cc.add(*v[0], *v[1]), *v[2]), *v[3]);
        out[1] = cc.sub(*cc.sub(*cc.sub(*t, *out[0]), *out[2]), *out[3]);
    }
    // SortUtils.cpp:131-208
    void sort5(const CtPtr *v, const CtPtr *s, CtPtr *out) {
        const CtPtr sabc[3] = {s[0], s[1], s[4]};
        CtPtr abc[3], dl, dh, vd[3], ve[3];
        sort3(v, sabc, abc);
        sort2(v[3], v[4], s[9], dl, dh);
        const CtPtr ind[3] = {s[2], s[5], s[7]}, ine[3] = {s[3], s[6], s[8]};
        sort3(ind, sabc, vd);
        sort3(ine, sabc, ve);
        CtPtr Hl, Hh, Ml, Mh, ll, lh;
        sort2(vd[2], ve[2], s[9], Hl, Hh);
        sort2(vd[1], ve[1], s[9], Ml, Mh);
        sort2(vd[0], ve[0], s[9], ll, lh);
        out[4] = vmax(abc[2], dh, Hh);
        out[0] = vmin(abc[0], dl, ll);
        const CtPtr a1 = vmax(abc[1], dh, Mh), b1 = vmax(abc[2], dl, Hl);
        out[3] = vmax(a1, b1, Hh);
        const CtPtr a2 = vmin(abc[1], dl, Ml), b2 = vmin(abc[0], dh, lh);
        out[1] = vmin(a2, b2, ll);
        CtPtr t = v[0];
        for (int i = 1; i < 5; ++i) t = cc.add(*t, *v[i]);
        for (int i = 0; i < 5; ++i)
            if (i != 2) t = cc.sub(*t, *out[i]);
        out[2] = t;
    }
    CtPtr assemble(const CtPtr *s, int num, long shift) {  // SortUtils.cpp:424-433
        CtPtr o = s[0];
        for (int i = 1; i < num; ++i) o = cc.add(*o, *R(s[i], i * shift));
        return o;
    }
    // Sorter.cpp:187-256
    CtPtr align(const CtPtr &x, long log_dist, long slope, CtPtr *fix) {
        Mask left((size_t)ns, 0.0);
        std::vector<Mask> right((size_t)k, Mask((size_t)ns, 0.0));
        for (size_t i = 0; i < (size_t)ns; ++i) {
            if (pos[i] < grp[i]) left[i] = 1.0;
            if (grp[i] > 0 && grp[i] == pos[i]) right[(size_t)grp[i] - 1][i] = 1.0;
        }
        const CtPtr xl = mul(x, left);
        const long r = rotate_distance(k, log_dist, slope);
        if (slope == 0) return cc.add(*R(xl, r), *L(mul(x, right[(size_t)k - 1]), (k - 1) * r));
        if (slope == k / 2 + 1) {
            const CtPtr xr = mul(x, right[(size_t)k - 2]);
            if (fix) *fix = cc.sub(*cc.sub(*x, *xl), *xr);
            return cc.add(*R(xl, r), *L(xr, (k - 2) * r));
        }
        std::vector<CtPtr> xr;
        for (long i = 0; i < k; ++i) xr.push_back(mul(x, right[(size_t)i]));
        if (fix) {
            *fix = cc.sub(*x, *xl);
            for (auto &t : xr) *fix = cc.sub(**fix, *t);
        }
        CtPtr o = R(xl, r);
        for (long i = 1; i < k; ++i) o = cc.add(*o, *L(xr[(size_t)i], i * r));
        return o;
    }
    CtPtr cmp(const CtPtr &a, const CtPtr &b) { return compare(cc, *a, *b, SignFunc::CompositeSign, cfg); }

    CtPtr run2(const CtPtr &x, long sh, const CtPtr &c) {  // Sorter.cpp:9-36
        const Mask m = sel(2, 1);
        CtPtr lo, hi;
        sort2(x, L(x, sh), c, lo, hi);
        lo = mul(lo, m);
        hi = mul(hi, m);
        return cc.add(*lo, *R(hi, sh));
    }
    CtPtr run3(const CtPtr &x, long sh, const CtPtr &c) {  // Sorter.cpp:38-68
        const Mask m = sel(3, 1);
        const CtPtr v[3] = {x, L(x, sh), L(x, 2 * sh)};
        const CtPtr s[3] = {flip(L(c, sh), m), c, flip(L(c, 2 * sh), m)};
        CtPtr o[3];
        sort3(v, s, o);
        for (auto &t : o) t = mul(t, m);
        return cc.add(*cc.add(*o[0], *R(o[1], sh)), *R(o[2], 2 * sh));
    }
    CtPtr run4(const CtPtr &x, long sh, const CtPtr &c1, const CtPtr &c2) {  // Sorter.cpp:70-85
        const Mask m = sel(4, 1);
        CtPtr s[6];
        s[2] = c1;
        s[0] = flip(L(c1, sh), m);
        s[3] = flip(L(c1, 2 * sh), m);
        s[5] = flip(L(c1, 3 * sh), m);
        s[1] = c2;
        s[4] = L(c2, sh);
        CtPtr v[4], o[4];
        for (int i = 0; i < 4; ++i) v[i] = mul(L(x, i * sh), m);
        sort4(v, s, o);
        return assemble(o, 4, sh);
    }
    CtPtr run5(const CtPtr &x, long sh, const CtPtr &c1, const CtPtr &c2) {  // Sorter.cpp:87-115
        const Mask m = sel(5, 1);
        CtPtr v[5], s[10], o[5];
        for (int i = 0; i < 5; ++i) v[i] = L(x, i * sh);
        const int from1[5] = {3, 0, 4, 7, 9}, from2[5] = {2, 6, 1, 5, 8};
        for (int i = 0; i < 5; ++i) {
            s[from1[i]] = L(c1, i * sh);
            s[from2[i]] = L(c2, i * sh);
        }
        for (int i : {0, 1, 4, 5, 7, 8, 9}) s[i] = flip(s[i], m);
        sort5(v, s, o);
        for (auto &t : o) t = mul(t, m);
        return assemble(o, 5, sh);
    }
    CtPtr run2345(const CtPtr &x, long sh, const CtPtr &c1, const CtPtr &c2) {  // Sorter.cpp:117-185
        Mask any((size_t)ns, 0.0), ge3 = any, ge4 = any, e3 = any, e4 = any, e5 = any;
        for (size_t i = 0; i < (size_t)ns; ++i) {
            if (pos[i] != 1 || grp[i] < 2 || grp[i] > 5) continue;
            any[i] = 1.0;
            ge3[i] = grp[i] >= 3 ? 1.0 : 0.0;
            ge4[i] = grp[i] >= 4 ? 1.0 : 0.0;
            (grp[i] == 3 ? e3 : grp[i] == 4 ? e4 : grp[i] == 5 ? e5 : any)[i] = 1.0;
        }
        CtPtr v[5], s[10], o[5];
        for (int i = 0; i < 5; ++i) v[i] = L(x, i * sh);
        s[0] = flip(L(c1, sh), any);
        s[1] = cc.add(*mul(c1, e3), *flip(mul(L(c2, 2 * sh), ge4), ge4));
        s[2] = cc.add(*mul(c1, e4), *mul(c2, e5));
        s[3] = mul(c1, e5);
        s[4] = flip(mul(L(c1, 2 * sh), ge3), ge3);
        s[5] = flip(mul(L(c2, 3 * sh), ge4), ge4);
        s[6] = mul(L(c2, sh), e5);
        s[7] = flip(mul(L(c1, 3 * sh), ge4), ge4);
        s[8] = flip(mul(L(c2, 4 * sh), e5), e5);
        s[9] = flip(mul(L(c1, 4 * sh), e5), e5);
        sort5(v, s, o);
        const Mask *post[5] = {&any, &any, &ge3, &ge4, &e5};
        for (int i = 0; i < 5; ++i) o[i] = mul(o[i], *post[i]);
        return assemble(o, 5, sh);
    }

    CtPtr run(const Ciphertext &input) {  // Sorter.cpp:289-404
        CtPtr ct = cc.clone(input);
        for (int stage = 0; stage < stage_count((int)k, (int)M); ++stage) {
            int m, ld, sl;
            sort_type((int)k, stage, m, ld, sl);
            const long sh = rotate_distance(k, ld, sl);
            gen_indices(ns, k, M, m, ld, sl, grp, pos);
            CtPtr fix, c1, c2;
            auto one = [&](int before, int after) {
                need(ct, before);
                c1 = cmp(ct, align(ct, ld, sl, &fix));
                need(c1, after);
            };
            auto two = [&](int before, int after) {
                need(ct, before);
                const CtPtr r1 = align(ct, ld, sl, &fix);
                const CtPtr r2 = align(r1, ld, sl, nullptr);
                c1 = cmp(ct, r1);
                c2 = cmp(ct, r2);
                need(ct, before);  // Sorter.cpp:351 (k = 5, middle slope): a second check of ctxt
                need(c1, after);
                need(c2, after);
            };
            if (sl == 0) {
                if (k == 5) {
                    two(lv[5], lv[5]);
                    ct = run5(ct, sh, c1, c2);
                } else {
                    one(lv[k], lv[k]);
                    ct = k == 2 ? run2(ct, sh, c1) : run3(ct, sh, c1);
                }
            } else if (sl == k / 2 + 1) {
                if (k == 3) {
                    one(lv[2], lv[2]);
                    ct = cc.add(*run2(ct, sh, c1), *fix);
                } else {
                    two(lv[4], lv[4]);
                    ct = cc.add(*run4(ct, sh, c1, c2), *fix);
                }
            } else if (k == 5 && sl == 1) {
                two(lv[5], lv[5]);
                ct = cc.add(*run2345(ct, sh, c1, c2), *fix);
            } else if ((k == 5 && sl == 2) || (k == 3 && sl == 1)) {
                one(lv[3], lv[2]);  // Sorter.cpp:370-378: c1 checked for 2, then for 3
                const CtPtr a = run2(ct, sh, c1);
                need(c1, lv[3]);
                const CtPtr b = run3(ct, sh, c1);
                ct = cc.add(*cc.add(*a, *fix), *b);
            } else if (k == 2 && sl == 1) {
                one(lv[2], lv[2]);
                ct = cc.add(*run2(ct, sh, c1), *fix);
            } else {
                throw std::invalid_argument("k-way: no matching k and slope");
            }
        }
        return ct;
    }
};

}  // namespace

// SortUtils::fcnL (kk = 1: out[0] = fcnL(x0, x1, s0)) and the 2/3/4/5-sorters
// (SortUtils.cpp:5-208) on their own, for SortUtilsTest's known answers
std::vector<CtPtr> sorter(Context &cc, int kk, const std::vector<CtPtr> &x, const std::vector<CtPtr> &s) {
    const size_t nx = kk == 1 ? 2 : (size_t)kk, ns = kk == 1 ? 1 : (size_t)(kk * (kk - 1) / 2);
    if (kk < 1 || kk > 5 || x.size() != nx || s.size() != ns) throw std::invalid_argument("k-way sorter: bad arity");
    Net net{cc, (long)x[0]->slots, 5, 2, SignConfig{}, {}, {}, {}};
    std::vector<CtPtr> out(kk == 1 ? 1 : (size_t)kk);
    if (kk == 1)
        out[0] = net.fcn(x[0], x[1], s[0]);
    else if (kk == 2)
        net.sort2(x[0], x[1], s[0], out[0], out[1]);
    else if (kk == 3)
        net.sort3(x.data(), s.data(), out.data());
    else if (kk == 4)
        net.sort4(x.data(), s.data(), out.data());
    else
        net.sort5(x.data(), s.data(), out.data());
    return out;
}

CtPtr sort(Context &cc, const Ciphertext &x, int k, int M, const SignConfig &cfg) {
    if (k != 2 && k != 3 && k != 5) throw std::invalid_argument("k-way: only k = 2, 3, 5 are supported");
    if (M < 1 || pw(k, M) > x.slots) throw std::invalid_argument("k-way: k^M exceeds the slots");
    Net net{cc, pw(k, M), k, M, cfg, {}, {}, {}};
    return net.run(x);
}

}  // namespace kway
}  // namespace oracle
