// CKKS bootstrapping on the engine (see bootstrap.hpp).  Reference call sites:
// tests/k-way/KWaySort235Test.cpp:46-48 (setup + key generation),
// src/k-way/EvalUtils.cpp:76 and src/sign.cpp:168 (EvalBootstrap).
//
// The homomorphic DFT is emb / emb^-1 of the canonical-embedding encoder
// (host::special_fft / special_ifft) without their bit reversals: CoeffsToSlots
// leaves the subring coefficients in bit-reversed order, EvalMod is slot-wise,
// and SlotsToCoeffs consumes that order.  Vectors live in the 2s-slot view of
// the sparse ciphertext (its n/2 slots are 2s-periodic), so each radix-2
// butterfly is three diagonals {0, +h, -h}; the stages of one level are
// multiplied out in fp64 (fixed order, -ffp-contract=off), and every level
// is a baby-step giant-step sum over those diagonals.
#include "bootstrap.hpp"

#include <algorithm>
#include <climits>
#include <cmath>
#include <set>
#include <stdexcept>

#include "fhesort.hpp"

namespace fhe {
namespace {

using cd = std::complex<double>;
using DiagMap = std::map<long, std::vector<cd>>;  // offset (mod m) -> m slot values

cd unit_root(uint64_t k, uint64_t M) {
    const double ang = 2.0 * M_PI * (double)k / (double)M;
    return cd(std::cos(ang), std::sin(ang));
}

// butterfly of half-size h of emb^-1 (enc = true) or emb (enc = false) on the
// 2s-slot view: three diagonals; rg[j] = 5^j mod M
DiagMap butterfly(long m, long h, uint64_t M, const std::vector<uint64_t> &rg, bool enc) {
    const uint64_t lenq = 8 * (uint64_t)h, gap = M / lenq;
    std::vector<cd> zero(m), plus(m), minus(m);
    for (long k = 0; k < m; ++k) {
        const long p = k % (2 * h);
        if (enc) {  // (u, v) -> (u + v, (u - v) xi^-1)
            if (p < h) {
                zero[k] = 1.0;
                plus[k] = 1.0;
            } else {
                const cd w = unit_root((lenq - rg[p - h] % lenq) * gap, M);
                minus[k] = w;
                zero[k] = -w;
            }
        } else {  // (u, v) -> (u + xi v, u - xi v)
            if (p < h) {
                zero[k] = 1.0;
                plus[k] = unit_root((rg[p] % lenq) * gap, M);
            } else {
                minus[k] = 1.0;
                zero[k] = -unit_root((rg[p - h] % lenq) * gap, M);
            }
        }
    }
    DiagMap D;
    D[0] = zero;
    D[h] = plus;
    D[m - h] = minus;
    return D;
}

// SlotsToCoeffs entry: lo + i hi into both halves of the 2s-slot view
DiagMap join_halves(long m) {
    const long s = m / 2;
    std::vector<cd> zero(m), half(m);
    for (long k = 0; k < m; ++k) {
        zero[k] = k < s ? cd(1, 0) : cd(0, 1);
        half[k] = k < s ? cd(0, 1) : cd(1, 0);
    }
    DiagMap D;
    D[0] = zero;
    D[s] = half;
    return D;
}

// product of two diagonal-form matrices: (A B)_d = sum_{a+b=d} A_a * rot(B_b, a)
DiagMap compose(const DiagMap &A, const DiagMap &B, long m) {
    DiagMap C;
    for (const auto &a : A)
        for (const auto &b : B) {
            auto &c = C[(a.first + b.first) % m];
            if (c.empty()) c.assign(m, cd(0, 0));
            for (long k = 0; k < m; ++k) c[k] += a.second[k] * b.second[(k + a.first) % m];
        }
    for (auto it = C.begin(); it != C.end();) {
        const bool zero = std::all_of(it->second.begin(), it->second.end(), [](const cd &v) { return v == cd(0, 0); });
        it = zero ? C.erase(it) : std::next(it);
    }
    return C;
}

// Partial trace: log2(n / 2s) doubling steps x += rot(x, 2^b s), taken three at
// a time as one hoisted sum x + sum_{0 < j < 8} rot(x, j 2^b0 s) (one ModUp and
// one ModDown per chunk instead of one of each per step)
std::vector<std::vector<long>> traceChunks(size_t n, long s) {
    int t = 0;
    while (((size_t)s << (t + 1)) <= n / 2) ++t;
    std::vector<std::vector<long>> out;
    for (int b0 = 0; b0 < t; b0 += 3) {
        const int c = std::min(3, t - b0);
        std::vector<long> ks;
        for (long j = 1; j < (1L << c); ++j) ks.push_back(j * (s << b0));
        out.push_back(std::move(ks));
    }
    return out;
}

// stages per level: the first (stages mod budget) levels take one more
std::vector<int> level_sizes(int stages, int budget) {
    budget = std::max(1, std::min(budget, stages));
    std::vector<int> g((size_t)budget, stages / budget);
    for (int i = 0; i < stages % budget; ++i) ++g[(size_t)i];
    return g;
}

// baby-step giant-step schedule: diagonal x step = G + (emin + i) step with
// baby i < b (the babies centred on the diagonals, so a level that fits in one
// giant needs no giant rotation).  A baby costs one key product inside
// linear_transform_ext (it is never brought down to Q); a rotated giant a
// ModDown, a ModUp and a key switch of its own, priced at kGiantCost babies.
constexpr long kGiantCost = 8;
Bootstrapper::Level schedule(const DiagMap &D, long m) {
    long step = m;
    for (const auto &kv : D)
        while (kv.first % step) step >>= 1;
    std::vector<long> e;
    for (const auto &kv : D) e.push_back((kv.first > m / 2 ? kv.first - m : kv.first) / step);
    const long emin = *std::min_element(e.begin(), e.end());
    auto baby_rot = [&](long i) { return (((emin + i) * step) % m + m) % m; };
    long bsel = 1, best = LONG_MAX;
    for (long b = 1; b <= 64; b <<= 1) {
        std::set<long> bs, gs;
        for (long x : e) {
            const long i = (x - emin) % b;
            bs.insert(baby_rot(i));
            gs.insert((((x - emin - i) * step) % m + m) % m);
        }
        const long cost = (long)bs.size() - (long)bs.count(0) + kGiantCost * ((long)gs.size() - (long)gs.count(0));
        if (cost < best) {
            best = cost;
            bsel = b;
        }
    }
    Bootstrapper::Level lv;
    std::set<long> used;
    for (long x : e) used.insert((x - emin) % bsel);
    std::map<long, int> slot;
    for (long i : used) {
        slot[i] = (int)lv.baby.size();
        lv.baby.push_back(baby_rot(i));
    }
    std::map<long, Bootstrapper::GiantStep> giants;
    size_t j = 0;
    for (const auto &kv : D) {
        const long x = e[j++];
        const long i = (x - emin) % bsel;
        const long G = (((x - emin - i) * step) % m + m) % m;
        auto &g = giants[G];
        g.shift = G;
        g.baby.push_back(slot[i]);
        std::vector<cd> v((size_t)m);  // rot(diag, -G)
        for (long k = 0; k < m; ++k) v[(size_t)k] = kv.second[(size_t)(((k - G) % m + m) % m)];
        g.diag.push_back(std::move(v));
    }
    for (auto &kv : giants) lv.giants.push_back(std::move(kv.second));
    return lv;
}

}  // namespace

Bootstrapper::Bootstrapper(Engine &c, const BootstrapConfig &cf) : cc(c), cfg(cf) {
    const auto &P = cc.params();
    const size_t n = P.n;
    const long s = cfg.slots, m = 2 * s;
    if (s < 2 || (s & (s - 1)) || (size_t)m > n / 2)
        throw std::invalid_argument("bootstrap: slots must be a power of two in [2, n/4]");
    if (cfg.budgetEnc < 1 || cfg.budgetDec < 1 || cfg.r < 0 || cfg.K < 1 || cfg.degree < 1)
        throw std::invalid_argument("bootstrap: bad configuration");
    // the message is scaled to q0 2^-bits before ModRaise; 2^bits / (4 pi) is
    // folded into SlotsToCoeffs (decInt doubles up to it): bounded so that
    // stays finite and the integer factor fits a long
    if (cfg.correctionBits < 1 || cfg.correctionBits > 40)
        throw std::invalid_argument("bootstrap: correction bits must be in 1..40");
    int logs = 0;
    while ((1L << logs) < s) ++logs;
    const uint64_t M = 2 * (uint64_t)n;
    std::vector<uint64_t> rg((size_t)s);
    for (long j = 0, g = 1; j < s; ++j, g = (long)((uint64_t)g * 5 % M)) rg[(size_t)j] = (uint64_t)g;
    // CoeffsToSlots maps the raised slots (t at scale Delta_0, trace factor
    // n/2s, conjugate-add factor 2) to t / (K q0): c_enc = Delta_0 / (n q0 K)
    const double q0 = (double)P.primes[0];
    const double c_enc = cc.delta(0) / ((double)n * q0 * (double)cfg.K);
    // SlotsToCoeffs maps sin(2 pi t / q0) ~ 2 pi 2^-b m back to m / 2; the
    // closing x + conj(x) keeps the real part (OpenFHE bootstraps real data;
    // an imaginary residue would grow through every later sign polynomial)
    const double c_dec = std::ldexp(1.0, cfg.correctionBits) / (4.0 * M_PI);
    const auto le = level_sizes(logs, cfg.budgetEnc), ld = level_sizes(logs, cfg.budgetDec);
    int t = 0;
    for (size_t li = 0; li < le.size(); ++li) {
        DiagMap cur;
        for (int j = 0; j < le[li]; ++j, ++t) {
            DiagMap S = butterfly(m, s >> (t + 1), M, rg, true);
            cur = cur.empty() ? S : compose(S, cur, m);
        }
        const double f = std::pow(c_enc, 1.0 / (double)le.size());
        for (auto &kv : cur)
            for (long k = 0; k < m; ++k) {
                kv.second[(size_t)k] *= f;
                if (li + 1 == le.size() && k >= s) kv.second[(size_t)k] *= cd(0, -1);  // upper half: x (-i)
            }
        enc.push_back(schedule(cur, m));
    }
    // per-level factor <= 2 keeps merged diagonals below 4 (63-bit coefficients
    // at 60-bit scales); the power-of-two rest is one integer product
    while (std::pow(c_dec / (double)decInt, 1.0 / (double)ld.size()) > 2.0 && decInt < (1L << 50)) decInt *= 2;
    t = 0;
    for (size_t li = 0; li < ld.size(); ++li) {
        DiagMap cur = li == 0 ? join_halves(m) : DiagMap();
        for (int j = 0; j < ld[li]; ++j, ++t) {
            DiagMap S = butterfly(m, 1L << t, M, rg, false);
            cur = cur.empty() ? S : compose(S, cur, m);
        }
        const double f = std::pow(c_dec / (double)decInt, 1.0 / (double)ld.size());
        for (auto &kv : cur)
            for (auto &v : kv.second) v *= f;
        dec.push_back(schedule(cur, m));
    }
    cheb = evalModCoefficients(cfg.K, cfg.r, cfg.degree);
}

std::vector<int> Bootstrapper::rotationIndices() const {
    std::set<long> r;
    const long s = cfg.slots;
    for (const auto &ks : traceChunks(cc.params().n, s))
        for (long k : ks) r.insert(k);
    for (const auto *levels : {&enc, &dec})
        for (const Level &lv : *levels) {
            for (long b : lv.baby)
                if (b) r.insert(b);
            for (const GiantStep &g : lv.giants)
                if (g.shift) r.insert(g.shift);
        }
    return std::vector<int>(r.begin(), r.end());
}

void Bootstrapper::keyGen() {
    cc.gen_rotation_keys(rotationIndices());
    cc.gen_galois_keys({2 * (uint64_t)cc.params().n - 1});
}

int Bootstrapper::depth() const {
    return (int)(enc.size() + dec.size()) + chebPSDepthSplit((int)cheb.size() - 1, cc.ps_split()) + cfg.r;
}

CtPtr Bootstrapper::transform(const Ciphertext &x, const Level &lv, int tag) {
    const int m = 2 * cfg.slots;
    auto key = std::make_pair(tag, x.level);
    auto it = pts.find(key);
    if (it == pts.end()) {  // diagonals over Q_level u P, encoded once per (level, ciphertext level), kept in HBM
        std::vector<std::vector<PtPtr>> enc_pts;
        for (const GiantStep &g : lv.giants) {
            std::vector<PtPtr> row;
            for (const auto &v : g.diag) row.push_back(cc.encode_complex_ext(v, m, x.level, cc.delta(x.level)));
            enc_pts.push_back(std::move(row));
        }
        it = pts.emplace(key, std::move(enc_pts)).first;
    }
    // double hoisting: one ModUp, babies over Q u P, one ModDown per level
    std::vector<Engine::LtGiant> G(lv.giants.size());
    for (size_t gi = 0; gi < lv.giants.size(); ++gi) {
        G[gi].shift = lv.giants[gi].shift;
        G[gi].baby = lv.giants[gi].baby;
        for (const auto &p : it->second[gi]) G[gi].pts.push_back(p.get());
    }
    return cc.linear_transform_ext(x, lv.baby, G);
}

CtPtr Bootstrapper::coeffsToSlots(const Ciphertext &raised) {
    CtPtr x = cc.clone(raised);
    for (size_t i = 0; i < enc.size(); ++i) x = transform(*x, enc[i], (int)i);
    x = cc.add(*x, *cc.conjugate(*x));
    x->slots = 2 * cfg.slots;
    return x;
}

CtPtr Bootstrapper::evalMod(const Ciphertext &x) {
    CtPtr y = evalChebyshevSeriesPS(cc, x, cheb, -1.0, 1.0);
    for (int i = 0; i < cfg.r; ++i) {  // cos(2a) = 2 cos(a)^2 - 1
        y = cc.square(*y);
        y = cc.add(*y, *y);
        y = cc.add_const(*y, -1.0);
    }
    return y;
}

CtPtr Bootstrapper::slotsToCoeffs(const Ciphertext &x) {
    CtPtr y = decInt > 1 ? cc.mul_int(x, decInt) : cc.clone(x);
    for (size_t i = 0; i < dec.size(); ++i) y = transform(*y, dec[i], 100 + (int)i);
    y = cc.add(*y, *cc.conjugate(*y));
    y->slots = cfg.slots;
    return y;
}

CtPtr Bootstrapper::evalBootstrap(const Ciphertext &in) {
    const int L = cc.params().L;
    if (in.batch != 1) throw std::invalid_argument("bootstrap: one ciphertext at a time");
    if (in.slots != cfg.slots) throw std::invalid_argument("bootstrap: ciphertext slots differ from the setup's");
    if (in.level >= L)
        throw std::runtime_error("bootstrap: no level left for the scale adjustment (level " + std::to_string(in.level) +
                                 " == multDepth)");
    const double q0 = (double)cc.params().primes[0];
    CtPtr x = cc.mul_const_to(in, std::ldexp(q0, -cfg.correctionBits) / cc.delta(L), L);
    x = cc.mod_raise(*x);
    for (const auto &ks : traceChunks(cc.params().n, cfg.slots)) x = cc.rotate_sum_hoisted(*x, ks);  // partial trace
    x = coeffsToSlots(*x);
    x = evalMod(*x);
    return slotsToCoeffs(*x);
}

}  // namespace fhe
