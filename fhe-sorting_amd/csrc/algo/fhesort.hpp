// C++ call surface of the rank-sort comparator hot path, MI355X edition.
//
// Mirrors the reference's interface (names, argument meaning, error
// behaviour) so a caller of oksuman/FHE-Sorting finds the same entry points:
//   enum SignFunc, CompositeSignConfig, SignConfig      src/sign.h:6-32
//   compositeSign<n>(), sign()                          src/sign.h:35-41
//   Comparison::compare / indicator                     src/comparison.h:81-101
//   DecomposeAlgo, Step, Decomposer<N>                  src/rotation.h:12-166
//   RotationComposer<N>::rotate                         src/rotation.h:193-233
//   DirectSort<N>::{getSizeParameters, constructRank,
//                   rotationIndexCheckN, sort}          src/sort_algo.h:61-774
// Every operation executes on the GPU through fhe::Engine (engine.hpp); the
// templates are thin wrappers over runtime-N implementations.
#pragma once
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <tuple>
#include <vector>

#include "../engine/engine.hpp"

namespace fhe {

enum class SignFunc { CompositeSign = 0, SignumPolycircuit = 1, Tanh = 2, NaiveDiscrete = 3 };

struct CompositeSignConfig {
    int n, dg, df;
    CompositeSignConfig(int n_, int dg_, int df_) : n(n_), dg(dg_), df(df_) {}
};
struct SignConfig {
    CompositeSignConfig compos{0, 0, 0};
    int multDepth = 100;  // src/sign.h:27-28
    // compositeSign's lazyBootstrap (src/sign.cpp:164-170): when set, g_n / f_n
    // run on a bootstrapped input whenever fewer than depth + 2 levels remain
    // (the context's depth is the reference's Cfg.multDepth)
    std::function<CtPtr(const Ciphertext &)> boot;
    SignConfig() = default;
    explicit SignConfig(CompositeSignConfig c) : compos(c) {}
    SignConfig(CompositeSignConfig c, int depth) : compos(c), multDepth(depth) {}
};

// Chebyshev series sum c_0/2 + sum_{i>=1} c_i T_i((2x-a-b)/(b-a)) by
// Paterson-Stockmeyer; replaces OpenFHE EvalChebyshevSeriesPS.  The split is
// cc.ps_split: OpenFHE's (default) or the engine's power-of-two one.
CtPtr evalChebyshevSeriesPS(Engine &cc, const Ciphertext &x, const std::vector<double> &coeffs, double a,
                            double b);
// levels evalChebyshevSeriesPS consumes for a degree-d series (OpenFHE split /
// given split)
int chebPSDepth(int degree);
// true iff evalChebyshevSeriesPS under PS_SPLIT_OPENFHE evaluates these
// coefficients with OpenFHE's division tree (false: the power-of-two fallback
// of an ill-conditioned or degree < 5 series)
bool chebPSUsesOpenFHE(const std::vector<double> &coeffs);
int chebPSDepthSplit(int degree, int split);

CtPtr compositeSignN(Engine &cc, const Ciphertext &x, int n, const SignConfig &cfg);
template <int n>
CtPtr compositeSign(const Ciphertext &x, Engine &cc, const SignConfig &cfg) {
    return compositeSignN(cc, x, n, cfg);
}
CtPtr sign(const Ciphertext &x, Engine &cc, SignFunc func, const SignConfig &cfg);

class Comparison {
  public:
    CtPtr compare(Engine &cc, const Ciphertext &a, const Ciphertext &b, SignFunc f, const SignConfig &cfg);
    CtPtr indicator(Engine &cc, const Ciphertext &x, double c, SignFunc f, const SignConfig &cfg);
};

enum class DecomposeAlgo { NAF = 0, BNAF = 1, BINARY = 2 };
struct Step {
    int value;
    int stepSize;
};

class DecomposerN {
  public:
    DecomposerN(int N, std::vector<int> rot);
    std::vector<Step> decompose(int rotation, int wrapN, DecomposeAlgo algo) const;
    const std::vector<int> &getRotIndices() const { return rotIndices; }
    int N, maxDecomposed;
    std::vector<int> rotIndices;
};
template <int SIZE>
class Decomposer : public DecomposerN {
  public:
    explicit Decomposer(std::vector<int> rot) : DecomposerN(SIZE, std::move(rot)) {}
};

class RotationComposerN {
  public:
    RotationComposerN(Engine &cc, int N, const std::vector<int> &rotIndices,
                      DecomposeAlgo algo = DecomposeAlgo::BINARY);
    CtPtr rotate(const Ciphertext &in, int rotation);
    // several rotations of one input; single keyed steps share one ModUp
    std::vector<CtPtr> rotateMany(const Ciphertext &in, const std::vector<int> &rotations);
    // member m of the batch `in` rotated by rotations[m] through the same keyed
    // steps rotate() takes; step j of every member that has one runs in one
    // multi-key launch sequence (Engine::rotate_members).  Same words as
    // rotate() member by member.
    std::vector<CtPtr> rotateMembers(const Ciphertext &in, const std::vector<int> &rotations);
    Engine &cc;
    DecomposerN dec;
    DecomposeAlgo algo;
    std::set<int> avail;
};
template <int SIZE>
class RotationComposer : public RotationComposerN {
  public:
    RotationComposer(Engine &cc, const std::vector<int> &rot, DecomposeAlgo a = DecomposeAlgo::BINARY)
        : RotationComposerN(cc, SIZE, rot, a) {}
};

// src/rotation.h:168-191
struct RotationStats {
    size_t fastRotationCount = 0, normalRotationCount = 0, totalRotationCount = 0, cacheHits = 0, cacheMisses = 0;
    void reset() { *this = RotationStats(); }
};

// RotationTree<N> (src/rotation.h:240-358): rotations by any k as paths of
// keyed steps in a prefix tree; every node's rotated ciphertext is cached, and
// the children of a node are rotations of one ciphertext, so they share one
// ModUp.  The reference computes a child on first use with
// EvalFastRotation(node precompute); here the first use of any child of a
// node computes all of that node's built children in one hoisted launch
// sequence (fhe_rotate_hoisted) -- hoisted and single rotations are
// bit-identical in this engine, so results do not depend on the order of
// requests.  As in the reference, the cache belongs to the first input
// rotated: one tree per input ciphertext.
class RotationTreeN {
  public:
    RotationTreeN(Engine &cc, int N, const std::vector<int> &rotIndices, DecomposeAlgo algo = DecomposeAlgo::NAF);
    void buildTree(int start, int end);
    CtPtr treeRotate(const Ciphertext &input, int rotation);
    const RotationStats &getStats() const { return stats; }

  private:
    struct Node {
        int stepSize;
        Node *parent;
        std::map<int, std::unique_ptr<Node>> children;
        std::vector<int> finalValues;
        CtPtr rotated;
        Node(int s, Node *p) : stepSize(s), parent(p) {}
    };
    void addToTree(Node *node, const std::vector<Step> &steps, size_t i, int value);
    CtPtr traverse(const CtPtr &input, Node *node, const std::vector<Step> &steps, size_t i);
    Engine &cc;
    DecomposerN dec;
    DecomposeAlgo algo;
    std::unique_ptr<Node> root;
    RotationStats stats;
};
template <int SIZE>
class RotationTree : public RotationTreeN {
  public:
    RotationTree(Engine &cc, const std::vector<int> &rot, DecomposeAlgo a = DecomposeAlgo::NAF)
        : RotationTreeN(cc, SIZE, rot, a) {}
};

struct SortShape {
    int N, num_partition, num_batch, num_slots, np;
};
void directSortSizeParameters(int N, int &multDepth, std::vector<int> &rotations);
// the hybrid sort test's parameters (tests/DirectSortHTest.cpp:23-104, ring 2^17)
void hybridSortSizeParameters(int N, int &multDepth, std::vector<int> &rotations);
SortShape rankShape(int N, int max_batch);
SortShape checkShape(int N, int max_batch);

// Sums a ciphertext's u64 limbs over ranks in place (device pointer, count
// u64); the engine reduces mod q afterwards.  nullptr = single rank.
using CtAllReduce = std::function<void(u64 *dev_data, size_t count)>;

// Independent work items i handled by this rank iff i % world == rank; partial
// sums combined by `allreduce`.
struct Shard {
    int rank = 0, world = 1;
    CtAllReduce allreduce;
    bool mine(size_t i) const { return world <= 1 || (int)(i % (size_t)world) == rank; }
};
// Combines per-rank partial sums of one ciphertext: a 4-word header
// (presence, level + 1, (level + 1)^2, limbs) is summed first so ranks that
// hold no partial agree on the level and contribute a zero ciphertext, and
// ranks whose partials disagree on level or limbs all fail with the same error
// instead of entering mismatched collectives; then the limbs are summed as u64
// and reduced mod q.  No-op for one rank.
void reducePartial(Engine &cc, const Shard &sh, CtPtr &acc, int slots);

// The u64 sum of `world` residues, each < q_max, must not wrap: world * q_max
// < 2^64 (world <= 16 for the 60-bit first prime).  Throws otherwise.
void checkShardWorld(const host::Params &P, int world);
struct ShardHeader {
    int level;
    size_t limbs;
};
ShardHeader checkShardHeader(const u64 h[4]);

class DirectSortN {
  public:
    DirectSortN(Engine &cc, int N, const std::vector<int> &rotIndices);
    CtPtr constructRank(const Ciphertext &x, SignFunc f, const SignConfig &cfg);
    CtPtr rotationIndexCheckN(const Ciphertext &rank, const Ciphertext &x);
    CtPtr sort(const Ciphertext &x, SignFunc f, const SignConfig &cfg);
    // sort_hybrid (src/sort_algo.h:1050-1064): constructRank, then the MEHP24-style
    // matrix index check rotationIndexCheckHybrid (:893-1047); its num_batch^2
    // masks run stacked, blocks b shard over ranks like the rank-sort batches
    CtPtr rotationIndexCheckHybrid(const Ciphertext &rank, const Ciphertext &x);
    CtPtr sort_hybrid(const Ciphertext &x, SignFunc f, const SignConfig &cfg);
    int hybrid_max_array = 256;  // maxArraySize (:899)
    int hybrid_mask = 0;         // 0: by N as the reference; 1: scaled-sinc PS; 2: indicator (3,4,2); 3: (3,5,2)
    const std::vector<double> &sincCoefficients() const;

    int shard_rank = 0, shard_world = 1;
    CtAllReduce allreduce;
    Engine &cc;
    int N;
    RotationComposerN rot;
    int max_batch;
    // how many of this rank's batches run stacked through one compare / one PS
    // (every launch then carries that many ciphertexts; memory grows with it)
    int max_stack = 32;
    // concurrent lanes: the rank's batches are split over `lanes` host threads,
    // each driving a forked engine (own HIP stream and pool, shared keys)
    int lanes = 2;
    // public masks and checking vectors: true = encoded once per context and
    // kept; false = every sort re-encodes all of them on the device before it
    // starts (the reference encodes them on every use, src/sort_algo.h:341-342,
    // 714-716); masks are encoded on the device either way (FHE_HOST_MASKS=1:
    // the host encoder, A/B)
    bool cache_masks = true;

  private:
    struct Lane {
        Engine *eng;
        RotationComposerN *rot;
    };
    Lane lane(int l);
    template <class F>
    std::vector<CtPtr> run_lanes(const std::vector<int> &batches, F &&work);
    CtPtr vecRotsOpt(Lane L, const std::vector<CtPtr> &baby, int num_partition, int num_slots, int np, int is);
    // vecRotsOpt of several batches: the giant-step rotations of all of them
    // (one amount per batch) run in shared launches (RotationComposerN::rotateMembers)
    std::vector<CtPtr> vecRotsOptMany(Lane L, const std::vector<CtPtr> &baby, int num_partition, int num_slots,
                                      int np, const std::vector<int> &iss);
    CtPtr blindRotationOptN(const std::vector<CtPtr> &masked, int num_slots, int np, int ib, int num_partition);
    // blindRotationOptN over a stacked `masked` (member m belongs to batch ibs[m]), summed over members
    CtPtr blindRotationStacked(Lane L, const std::vector<CtPtr> &masked, int num_slots, int np,
                               const std::vector<int> &ibs, int num_partition);
    void reducePartial(CtPtr &acc, int slots);
    std::vector<CtPtr> babySteps(const Ciphertext &x, int np);
    // encoded on the calling lane's engine, published once complete (thread-safe)
    const Plaintext &mask(Engine &E, int kind, int num_slots, int k, int rot, int level);
    // re-encode every cached mask in device batches on the main engine
    void refresh_masks();
    std::map<std::tuple<int, int, int, int, int>, PtPtr> mask_cache;
    std::mutex mask_mu;
    std::vector<int> rot_indices;
    std::vector<std::unique_ptr<Engine>> lane_eng;
    std::vector<std::unique_ptr<RotationComposerN>> lane_rot;
};
template <int SIZE>
class DirectSort : public DirectSortN {
  public:
    DirectSort(Engine &cc, const std::vector<int> &rot) : DirectSortN(cc, SIZE, rot) {}
    static void getSizeParameters(int &multDepth, std::vector<int> &rotations) {
        directSortSizeParameters(SIZE, multDepth, rotations);
    }
};

// MEHP24 (Mazzone et al.) ranking / sorting, src/mehp24/mehp24_sort.h and
// mehp24_utils.h.  max_stack bounds how many independent compares /
// indicators run stacked in one batch (memory grows with it).
namespace mehp24 {
namespace utils {
// `sub` = sortLargeArrayFG's part length (256 in the reference)
std::vector<int> getRotationIndices(size_t N, size_t sub = 256);
// 0/1 row / column masks, encoded once per (kind, m, index, level, slots)
struct Masks {
    const Plaintext &get(Engine &cc, int kind, size_t m, size_t idx, int level, int slots);
    std::map<std::tuple<int, size_t, size_t, int, int>, PtPtr> cache;
};
CtPtr maskRow(Engine &cc, Masks &mk, const Ciphertext &c, size_t m, size_t row);
CtPtr maskColumn(Engine &cc, Masks &mk, const Ciphertext &c, size_t m, size_t col);
CtPtr replicateRow(Engine &cc, CtPtr c, size_t m);
CtPtr replicateColumn(Engine &cc, CtPtr c, size_t m);
CtPtr sumRows(Engine &cc, Masks &mk, CtPtr c, size_t m, bool mask, size_t row);
CtPtr sumColumns(Engine &cc, Masks &mk, CtPtr c, size_t m, bool mask);
CtPtr transposeRow(Engine &cc, Masks &mk, CtPtr c, size_t m, bool mask);
CtPtr transposeColumn(Engine &cc, Masks &mk, CtPtr c, size_t m, bool mask);
CtPtr signAdv(Engine &cc, CtPtr c, size_t dg, size_t df);
}  // namespace utils
CtPtr indicatorAdv(Engine &cc, const Ciphertext &c, double b, size_t dg, size_t df);
CtPtr sortFG(const Ciphertext &c, size_t vectorLength, SignFunc f, const SignConfig &cfg, uint32_t dg_i,
             uint32_t df_i, Engine &cc, int max_stack = 32);
// Multi-ciphertext sortFG shards its P(P+1)/2 pair compares and its P^2
// indicators over `sh` (one all-reduce per partial Cv / Ch / result sum);
// everything else is replicated.  The output does not depend on the sharding.
std::vector<CtPtr> sortFG(const std::vector<CtPtr> &c, size_t subVectorLength, SignFunc f, const SignConfig &cfg,
                          uint32_t dg_i, uint32_t df_i, Engine &cc, int max_stack = 32, const Shard &sh = Shard());
CtPtr sortLargeArrayFG(const Ciphertext &c, size_t totalLength, size_t subLength, SignFunc f,
                       const SignConfig &cfg, uint32_t dg_i, uint32_t df_i, Engine &cc, int max_stack = 32,
                       const Shard &sh = Shard());
struct Parameters {
    int multDepth = 0, logRingDim = 17, scaleModSize = 40, dnum = 3;
    int levels = 0;  // context depth: multDepth + 1 (input encrypted with encrypt_ext)
    SignConfig cfg;
    uint32_t dg_i = 0, df_i = 2;
    size_t subLength = 0;  // 0: sortFG on one ciphertext, else sortLargeArrayFG
    std::vector<int> rotations;
};
Parameters parameters(size_t N);
}  // namespace mehp24

// coefficient tables (generated offline by data/gen_doubled_sinc.py)
void setCoefficientDir(const std::string &dir);
const std::vector<double> &doubledSincCoefficients(int N);
const std::vector<double> &scaledSincCoefficients(int N);  // selectCoefficients<N>()
// bootstrapping's EvalMod cosine (data/gen_evalmod.py): evalmod_k<K>r<r>_<degree>.f64
const std::vector<double> &evalModCoefficients(int K, int r, int degree);

}  // namespace fhe
