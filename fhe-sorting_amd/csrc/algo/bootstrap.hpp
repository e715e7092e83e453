// CKKS bootstrapping on the MI355X engine: the operation the reference gets
// from OpenFHE's FHECKKSRNS (EvalBootstrapSetup / EvalBootstrapKeyGen /
// EvalBootstrap), used by the k-way network (tests/k-way/KWaySort235Test.cpp:
// 46-48, src/k-way/EvalUtils.cpp:59-86) and by compositeSign's lazy bootstrap
// (src/sign.cpp:164-170).  Sparse packing (slots s <= n/4); every step is a
// composition of engine ops that run as batched HIP kernels:
//
//   scale adjustment  mul_const_to(x, q0 2^-b / Delta_L, L)
//   ModRaise          Engine::mod_raise (inverse NTT of one limb, centred
//                     lift kernel, forward NTT of every Q limb)
//   partial trace     log2(n/2s) rotations by j s
//   CoeffsToSlots     budget_enc BSGS levels: hoisted baby rotations (one
//                     ModUp), one mul_plain_sum per giant step, giant rotation
//   real part         x + conjugate(x)
//   EvalMod           evalChebyshevSeriesPS of cos(2 pi (K u - 1/4) / 2^r),
//                     then r double angles 2 y^2 - 1
//   SlotsToCoeffs     budget_dec BSGS levels, then x + conj(x): real slots
//
// The diagonals and the schedule are the spec DESIGN.md §9d states; the CPU
// oracle (oracle/oracle_boot.cpp) restates it and the GPU output is
// word-identical to it (tests/test_gpu_bootstrap.py).
#pragma once
#include <complex>
#include <map>
#include <vector>

#include "../engine/engine.hpp"

namespace fhe {

struct BootstrapConfig {
    int slots = 0;                       // s: power of two, 2 <= s <= n/4 (EvalBootstrapSetup numSlots)
    int budgetEnc = 4, budgetDec = 4;    // levelBudget (kway_adapter.h:56-62: {4,4} / {5,5})
    int K = 512;                         // EvalMod range |t / q0| <= K (uniform ternary secret)
    int r = 6;                           // double-angle iterations
    int degree = 88;                     // Chebyshev degree of the cosine
    int correctionBits = 10;             // message scaled to q0 2^-bits before ModRaise
};

class Bootstrapper {
  public:
    Bootstrapper(Engine &cc, const BootstrapConfig &cfg);
    // rotation indices the transforms use (the conjugation key is separate)
    std::vector<int> rotationIndices() const;
    void keyGen();          // EvalBootstrapKeyGen: rotation keys + conjugation key
    int depth() const;      // output level of evalBootstrap
    // EvalBootstrap: input level <= L-1 (one level pays the scale adjustment)
    CtPtr evalBootstrap(const Ciphertext &ct);
    // the stages on their own (parity tests)
    CtPtr coeffsToSlots(const Ciphertext &raised);
    CtPtr evalMod(const Ciphertext &x);
    CtPtr slotsToCoeffs(const Ciphertext &x);

    struct GiantStep {
        long shift = 0;                                     // giant rotation (mod 2s)
        std::vector<int> baby;                              // indices into Level::baby
        std::vector<std::vector<std::complex<double>>> diag;  // pre-rotated diagonals (2s entries)
    };
    struct Level {
        std::vector<long> baby;  // baby rotations (mod 2s)
        std::vector<GiantStep> giants;
    };

    Engine &cc;
    const BootstrapConfig cfg;
    std::vector<Level> enc, dec;
    std::vector<double> cheb;
    long decInt = 1;  // power-of-two factor of the SlotsToCoeffs scale, applied as an integer product

  private:
    CtPtr transform(const Ciphertext &x, const Level &lv, int tag);
    std::map<std::pair<int, int>, std::vector<std::vector<PtPtr>>> pts;  // (tag, level) -> [giant][baby]
};

}  // namespace fhe
