// k-way sorting network over the GPU engine.
//
// Mirrors the reference's kwaySort namespace:
//   sortType / genIndices / genMask / getRotateDistance   src/k-way/Masking.cpp:25-167
//   EvalUtils::{flipCtxt, leftRotate, rightRotate,
//               checkLevelAndBoot}                         src/k-way/EvalUtils.cpp:59-146
//   SortUtils::{fcnL, compareMax/Min, two/three/four/
//               fiveSorter, slotMatching*, slotAssemble}   src/k-way/SortUtils.cpp:5-433
//   Sorter::{run*Sorter, rightRotateForSort,
//            comparisonForSort(2), sorter}                 src/k-way/Sorter.cpp:9-404
//   KWayAdapter<N>::getSizeParameters                      src/kway_adapter.h:38-62
//
// Bootstrapping: where the reference calls EvalBootstrap (checkLevelAndBoot,
// and compositeSign's lazy bootstrap inside every comparison) the sorter calls
// cfg.boot -- an fhe::Bootstrapper (bootstrap.hpp) at the C-ABI.  Without one a
// network runs only when the context depth covers all of its stages and
// otherwise fails with "no levels left" (FHE_EDEPTH).
#pragma once
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "fhesort.hpp"

namespace fhe {
namespace kwaySort {

std::tuple<int, int, int> sortType(int k, int M, int stage);  // (m, logDist, slope)
std::vector<std::vector<int>> genIndices(long numSlots, long k, long M, long m, long logDist, long slope);
void genMask(const std::vector<std::vector<int>> &indices, long index0, long index1, std::vector<double> &mask);
long getRotateDistance(long k, long logDist, long slope);
int stageCount(int k, int M);  // M + M(M-1)/2 * ceil(k/2)  (Sorter.cpp:290)

// KWayAdapter<N>::getSizeParameters: rotations +-2^i for 2^i < N
std::vector<int> rotationIndices(int N);

// EvalUtils::checkLevelAndBoot (EvalUtils.cpp:57-86): c bootstrapped (cfg.boot)
// when fewer than need + 1 levels remain, else c itself; *booted says which
CtPtr checkLevelAndBoot(Engine &cc, const CtPtr &c, int need, const SignConfig &cfg, bool *booted = nullptr);

class Sorter {
  public:
    // numSlots = k^M values; the ciphertext holds next_pow2(numSlots) slots
    Sorter(Engine &cc, long numSlots, long k, long M);
    CtPtr sorter(const Ciphertext &x, const SignConfig &cfg);
    int stagesRun = 0;   // stages completed by the last sorter() call
    int bootstraps = 0;  // checkLevelAndBoot bootstraps of the last sorter() call
    // optional second lane: a forked engine (own stream and pool, shared keys)
    // and the sign configuration to use on it (its own bootstrapper).  The two
    // comparisons of a k = 5 stage and their level checks then run on two host
    // threads at once; every operation is the same, so the words are too.
    Engine *laneEng = nullptr;
    SignConfig laneCfg;
    // SortUtils::fcnL (kk = 1: returns {fcnL(x0, x1, c0)}) or the kk-sorter,
    // kk = 2..5 (SortUtils.cpp:5-208), on their own: SortUtilsTest's cases
    std::vector<CtPtr> kSorter(int kk, const std::vector<CtPtr> &x, const std::vector<CtPtr> &cmp);

  private:
    Engine &cc;
    long numSlots, k, M;
    std::vector<int> level;  // Sorter::initLevels (Sorter.h:85-93)
    Comparison comp;
    std::map<std::pair<std::vector<double>, int>, PtPtr> masks;

    const Plaintext &mask(const std::vector<double> &v, const Ciphertext &like);
    void checkLevel(CtPtr &c, int need, const SignConfig &cfg);
    // checkLevel of c1 (this engine) and c2 (the lane, when set) at once
    void checkLevel2(CtPtr &c1, CtPtr &c2, int need, const SignConfig &cfg);
    CtPtr leftRotate(const CtPtr &c, long r);
    CtPtr rightRotate(const CtPtr &c, long r);
    std::vector<CtPtr> rotateMany(const std::vector<CtPtr> &src, const std::vector<long> &amt);
    CtPtr flip(const CtPtr &c, const std::vector<double> &m);
    CtPtr maskMul(const CtPtr &c, const std::vector<double> &m);
    CtPtr fcnL(const CtPtr &a, const CtPtr &b, const CtPtr &cmp);
    void twoSorter(const CtPtr &a, const CtPtr &b, const CtPtr &cmp, CtPtr *out);
    void threeSorter(const CtPtr *x, const CtPtr *cmp, CtPtr *out);
    void fourSorter(const CtPtr *x, const CtPtr *cmp, CtPtr *out);
    void fiveSorter(const CtPtr *x, const CtPtr *cmp, CtPtr *out);
    CtPtr slotAssemble(const CtPtr *s, long num, long shift);
    CtPtr runTwoSorter(const CtPtr &x, const std::vector<std::vector<int>> &ind, long shift, const CtPtr &c);
    CtPtr runThreeSorter(const CtPtr &x, const std::vector<std::vector<int>> &ind, long shift, const CtPtr &c);
    CtPtr runFourSorter(const CtPtr &x, const std::vector<std::vector<int>> &ind, long shift, const CtPtr &c1,
                        const CtPtr &c2);
    CtPtr runFiveSorter(const CtPtr &x, const std::vector<std::vector<int>> &ind, long shift, const CtPtr &c1,
                        const CtPtr &c2);
    CtPtr run2345Sorter(const CtPtr &x, const std::vector<std::vector<int>> &ind, long shift, const CtPtr &c1,
                        const CtPtr &c2);
    void rightRotateForSort(const CtPtr &x, const std::vector<std::vector<int>> &ind, long logDist, long slope,
                            CtPtr &rot, CtPtr *fix);
    CtPtr comparisonForSort(const CtPtr &x, const std::vector<std::vector<int>> &ind, long logDist, long slope,
                            CtPtr &fix, const SignConfig &cfg);
    void comparisonForSort2(const CtPtr &x, const std::vector<std::vector<int>> &ind, long logDist, long slope,
                            CtPtr &c1, CtPtr &c2, CtPtr &fix, const SignConfig &cfg);
};

}  // namespace kwaySort
}  // namespace fhe
