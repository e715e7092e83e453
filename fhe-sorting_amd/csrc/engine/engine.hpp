// MI355X RNS-CKKS ciphertext-op engine — host-side C++ interface.
//
// One Engine per GPU (one process per GPU).  Ciphertexts live in HBM for
// their whole life: [2][limbs][n] u64 in NTT (evaluation) form.  Every op is
// enqueued on the engine's HIP stream; nothing synchronises the host except
// downloads/decryption.  The op set and its semantics (levels, canonical
// scales, rounding of constants) are the spec of DESIGN.md §3, which the CPU
// oracle (oracle/) restates independently; results are bit-identical.
//
// The reference reaches these operations through OpenFHE's CryptoContext
// (EvalAdd/EvalSub/EvalMult/EvalSquare/EvalMultAndRelinearize/EvalRotate/
// EvalFastRotation/EvalChebyshevSeriesPS, called from src/sign.cpp,
// src/comparison.cpp, src/rotation.h and src/sort_algo.h).
#pragma once
#include <complex>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../host/hostmath.hpp"

namespace fhe {

using u64 = uint64_t;
using i64 = int64_t;

struct DevMem;  // pooled device allocation (engine.hip)

// A ciphertext batch: `batch` independent ciphertexts at one level, stored
// [batch][2][limbs][n].  Every op applies member-wise in the same launches, so
// the comparator / index-check pipelines of all rank-sort batches run as one
// (DESIGN.md §6).  batch = 1 is an ordinary ciphertext.
struct Ciphertext {
    std::shared_ptr<DevMem> mem;
    u64 *data = nullptr;  // [batch][2][limbs][n]
    int level = 0;
    int slots = 0;
    double scale = 0;
    size_t limbs = 0;
    int batch = 1;
};
using CtPtr = std::shared_ptr<Ciphertext>;

struct Plaintext {
    std::shared_ptr<DevMem> mem;
    u64 *data = nullptr;  // [limbs][n]
    int level = 0;
    int slots = 0;
    double scale = 0;
    size_t limbs = 0;
};
using PtPtr = std::shared_ptr<Plaintext>;

struct Counters {
    u64 hmult = 0, keyswitch = 0, rotations = 0, rescale = 0, ptmult = 0, constmult = 0;
    // op-level algorithmic HBM bytes (SURVEY §8(d)'s per-op formulas, each op
    // at its own level; B = 8n per limb): HMult (4l + 2 digits(l)(l+K) + 2l) B,
    // rotation (2l + 2 digits(l)(l+K) + 2l) B, ct x pt 5l B, ct x const 4l B,
    // add 6l B, linear sum of m terms (2l m + 2l) B -- per ciphertext
    u64 opbytes = 0;
    // sharded runs: host wall time inside the partial-sum exchanges (header +
    // data all-reduce, from a drained stream to the reduced data), and their count
    u64 allreduce_ns = 0, allreduce_calls = 0;
    Counters &operator+=(const Counters &o) {
        opbytes += o.opbytes;
        allreduce_ns += o.allreduce_ns;
        allreduce_calls += o.allreduce_calls;
        hmult += o.hmult;
        keyswitch += o.keyswitch;
        rotations += o.rotations;
        rescale += o.rescale;
        ptmult += o.ptmult;
        constmult += o.constmult;
        return *this;
    }
};

// Paterson-Stockmeyer split used by evalChebyshevSeriesPS (csrc/algo): OpenFHE's
// (k, m) long-division split (the default, as the reference), or the
// power-of-two split of rounds 1-2
enum : int { PS_SPLIT_ENGINE = 0, PS_SPLIT_OPENFHE = 1 };

class Engine {
  public:
    Engine(int logN, int L, int scale_bits, int first_bits, int dnum, int device, u64 seed);
    // the Paterson-Stockmeyer split, one value shared by this engine and every
    // fork of it (lane engines cached by the sorters read the current split, so
    // a change after a sort cannot leave lanes on the old one)
    int ps_split() const { return *ps_split_; }
    void set_ps_split(int split) { *ps_split_ = split; }
    ~Engine();
    // A second engine on its own HIP stream and memory pool sharing this one's
    // keys and tables: independent work issued to both (from two host threads)
    // runs concurrently on the GPU.  Keys must be complete before forking.
    std::unique_ptr<Engine> fork() const;
    // order this engine's stream after everything enqueued on `other` so far
    void wait_for(const Engine &other);
    Engine(const Engine &) = delete;
    Engine &operator=(const Engine &) = delete;

    const host::Params &params() const;
    size_t n() const;
    double delta(int level) const;

    // ------------------------------------------------------------ keys ---
    void keygen();
    void gen_rotation_keys(const std::vector<int> &rot);
    void load_secret(const u64 *s_ntt);           // [nall][n]
    void load_public(const u64 *pk);              // [2][nq][n]
    void load_relin(const u64 *key);              // [digits][2][nall][n]
    void load_rotation(long k, const u64 *key);   // [digits][2][nall][n]
    bool has_rotation_key(long k) const;
    // keys of arbitrary automorphisms X -> X^g (rotations: g = 5^k; conjugation: 2n - 1)
    void gen_galois_keys(const std::vector<u64> &gs);
    void load_galois(u64 g, const u64 *key);      // [digits][2][nall][n]
    bool has_galois_key(u64 g) const;
    size_t key_bytes() const;
    // key export (wire format, csrc/wire): same layouts as the loads above;
    // a missing key throws std::invalid_argument
    int key_digits() const;
    size_t switch_key_words() const;              // digits * 2 * nall * n
    bool has_secret() const;
    bool has_public() const;
    bool has_relin() const;
    void export_secret(u64 *out);
    void export_public(u64 *out);
    void export_relin(u64 *out);
    std::vector<u64> galois_elements() const;     // ascending
    void export_galois(u64 g, u64 *out);

    // ------------------------------------------------- encode / encrypt ---
    PtPtr encode(const std::vector<double> &v, int slots, int level);
    PtPtr encode_scaled(const std::vector<double> &v, int slots, int level, double scale);
    PtPtr encode_complex(const std::vector<std::complex<double>> &v, int slots, int level, double scale);
    // the same plaintext over Q_level u P (ell + K limbs, special primes last)
    PtPtr encode_complex_ext(const std::vector<std::complex<double>> &v, int slots, int level, double scale);
    // Device encoding (csrc/device/encode.hip), word-identical to encode():
    // the special inverse FFT, rounding, RNS split and NTT of a batch in a few
    // launches.  encode_masks generates the sort's public masks on the device
    // (kind 0: mask_vector(k) rotated by r, kind 1: checking_vector(k),
    // src/sort_algo.h:206-233, 272-286; slots num_slots, block size N);
    // encode_device takes arbitrary real slot vectors.
    struct MaskSpec {
        int kind, k, r, level;
    };
    std::vector<PtPtr> encode_masks(const std::vector<MaskSpec> &specs, int num_slots, int N);
    std::vector<PtPtr> encode_device(const std::vector<std::vector<double>> &vs, int slots, const std::vector<int> &levels);
    CtPtr encrypt(const std::vector<double> &v, int slots, int level = 0);
    CtPtr encrypt_pt(const Plaintext &pt);
    // OpenFHE FLEXIBLEAUTOEXT-style encryption: one extra level absorbs the
    // encryption noise (divided by q_L); the result sits at level 1
    CtPtr encrypt_ext(const std::vector<double> &v, int slots);
    std::vector<double> decrypt(const Ciphertext &ct);
    CtPtr upload(const u64 *host, size_t limbs, int level, int slots, double scale);
    void download(const Ciphertext &ct, u64 *host);
    PtPtr upload_pt(const u64 *host, size_t limbs, int level, int slots, double scale);

    // -------------------------------------------------------------- ops ---
    CtPtr clone(const Ciphertext &a);
    CtPtr add(const Ciphertext &a, const Ciphertext &b);
    CtPtr sub(const Ciphertext &a, const Ciphertext &b);
    void add_inplace(CtPtr &acc, const Ciphertext &b);
    CtPtr negate(const Ciphertext &a);
    CtPtr add_plain(const Ciphertext &a, const Plaintext &p);
    CtPtr sub_plain(const Ciphertext &a, const Plaintext &p);
    CtPtr plain_sub(const Plaintext &p, const Ciphertext &a);
    CtPtr add_const(const Ciphertext &a, double c);
    // a = a + c, in place on the c0 limbs when a is exclusively owned (else add_const)
    void add_const_inplace(CtPtr &a, double c);
    CtPtr mul_int(const Ciphertext &a, i64 k);
    CtPtr mul_const(const Ciphertext &a, double c);
    CtPtr mul_const_to(const Ciphertext &a, double c, int target);
    CtPtr level_adjust(const Ciphertext &a, int target);
    void match_levels(CtPtr &a, CtPtr &b);
    void count_bytes(double limb_units, int members);
    double ks_units(size_t ell) const;
    CtPtr mul_plain(const Ciphertext &a, const Plaintext &p);
    // sum_i a_i * p_i with one rescale (masked sums of src/sort_algo.h:341-346, 573-577)
    CtPtr mul_plain_sum(const std::vector<const Ciphertext *> &a, const std::vector<const Plaintext *> &p);
    CtPtr mul(const Ciphertext &a, const Ciphertext &b);
    // a*b + sum_i c_i x_i with one rescale (lazy rescaling of PS remainders)
    // a_add (optional): the left operand is a + a_add, formed inside the tensor
    // pass (same words as add(a, a_add) first)
    CtPtr mul_add(const Ciphertext &a, const Ciphertext &b, const std::vector<const Ciphertext *> &xs,
                  const std::vector<double> &cs, const Ciphertext *raw = nullptr, const Ciphertext *a_add = nullptr);
    // same with the sum already formed: raw = linear_sums_to(xs, {c}, level+1, false)[0]
    CtPtr mul_add_raw(const Ciphertext &a, const Ciphertext &b, const Ciphertext &raw, const Ciphertext *a_add = nullptr);
    CtPtr square(const Ciphertext &a);
    CtPtr rotate(const Ciphertext &a, long k);
    std::vector<CtPtr> rotate_hoisted(const Ciphertext &a, const std::vector<long> &ks);
    // member m of a batch rotated by ks[m] (all keyed): the giant steps of a
    // BSGS linear transform as one pipeline
    CtPtr rotate_members(const Ciphertext &a, const std::vector<long> &ks);
    // x + sum_k rotate(x, k) with one ModUp and one ModDown (the key products of
    // every rotation summed over Q u P, the rotated c0s added after the ModDown;
    // oracle: Context::rotate_sum_hoisted) -- the bootstrap's partial trace
    CtPtr rotate_sum_hoisted(const Ciphertext &x, const std::vector<long> &ks);
    // Double-hoisted baby-step giant-step linear transform (oracle:
    // Context::linear_transform_ext): one ModUp of x, the baby rotations kept
    // over Q u P and multiplied there by extended plaintexts (encode_complex_ext),
    // the unrotated giant as the starting accumulator, every rotated giant brought
    // down, rotated and summed over Q u P, one final ModDown, then the rescale.
    struct LtGiant {
        long shift = 0;
        std::vector<int> baby;               // indices into `baby`
        std::vector<const Plaintext *> pts;  // extended plaintexts at x's level
    };
    CtPtr linear_transform_ext(const Ciphertext &x, const std::vector<long> &baby, const std::vector<LtGiant> &giants);
    // keyed automorphisms sharing one ModUp; conjugate = g 2n - 1
    std::vector<CtPtr> apply_galois_hoisted(const Ciphertext &a, const std::vector<u64> &gs);
    CtPtr conjugate(const Ciphertext &a);
    // ModRaise (bootstrapping): last-level ciphertext (one limb) re-read over
    // every Q prime by the centred lift; level 0, scale Delta_0
    CtPtr mod_raise(const Ciphertext &a);
    CtPtr rescale(const Ciphertext &a);
    CtPtr drop_to(const Ciphertext &a, int level);
    CtPtr linear_sum_to(const std::vector<const Ciphertext *> &xs, const std::vector<double> &c, int target);
    // several linear sums of the same inputs (PS leaves): one output per row of c
    // (rescale = false: the raw sums at level target-1 and the pre-rescale scale, for mul_add_raw)
    std::vector<CtPtr> linear_sums_to(const std::vector<const Ciphertext *> &xs,
                                      const std::vector<std::vector<double>> &c, int target, bool rescale = true);
    CtPtr trivial_const(double c, int level, int slots, int batch = 1);
    CtPtr zero_like(int level, int slots, int batch = 1);
    // batches: stack (copies; equal levels), member view (no copy), member sum
    CtPtr stack(const std::vector<const Ciphertext *> &xs);
    CtPtr member(const Ciphertext &a, int m);
    // batches built in place (no stack copies): member i = a - bs[i] (a brought to
    // the bs' level once), and member i = a - ps[i]
    CtPtr sub_stacked(const Ciphertext &a, const std::vector<const Ciphertext *> &bs);
    CtPtr sub_plain_stacked(const Ciphertext &a, const std::vector<const Plaintext *> &ps);
    CtPtr sum_members(const Ciphertext &a);
    // sum over ranks already done into ct (u64 add, no reduction): reduce mod q
    void reduce_after_allreduce(Ciphertext &ct);

    // ---------------------------------------------- kernel-level access ---
    // host in/out, for parity tests
    void ntt_host(u64 *data, int prime_index, int limbs, bool inverse);
    void modup_host(const u64 *d, size_t ell, u64 *ext);          // ext [digits][ell+K][n] NTT
    void moddown_host(const u64 *in, size_t ell, u64 *out);        // in [ell+K][n] -> [ell][n]
    void automorph_host(const u64 *in, size_t limbs, u64 g, u64 *out);
    // device-resident variants: enqueued on `stream` (nullptr:
    // the engine stream), no host synchronisation.  ntt_dev transforms `limbs`
    // consecutive-prime limbs of `segments` polynomials in place (segment s at
    // data + s * seg_stride); automorph_dev writes in[...] o X -> X^g (NTT form).
    void ntt_dev(u64 *data, int prime_index, int limbs, int segments, size_t seg_stride, bool inverse, void *stream);
    void automorph_dev(const u64 *in, u64 *out, size_t limbs, u64 g, void *stream);
    // time `iters` back-to-back launches of one kernel on the engine stream
    // (HIP events), shaped like a key switch at `limbs` Q limbs; returns the
    // average ms per launch and the algorithmic HBM bytes per launch.
    void time_kernel(const std::string &name, size_t limbs, int iters, double &avg_ms, double &bytes);
    // live per-launch clock over real work: between start and stop every NTT
    // pass is bracketed by HIP events on the engine stream; stop() returns JSON
    // {"kernel": {"launches": c, "ms": total, "bytes": total_algorithmic}, ...}
    // device pool: release cached blocks; bytes live / cached / peak live
    // process-wide host costs: {encodes, encode seconds, pool-miss hipMallocs,
    // hipMalloc seconds} (the cold-sort breakdown)
    static void host_stats_get(double out[4]);
    static void host_stats_reset();
    void pool_trim();
    void pool_stats(size_t &live, size_t &cached, size_t &peak) const;
    void kernel_clock_start();
    std::string kernel_clock_stop();
    // algorithm phase the clocked kernels and op bytes are booked under
    // (nullptr = none); returns the previous one
    static const char *set_algo_phase(const char *phase);

    // small device scratch (for collectives / headers); copies are synchronous
    struct DevBuf {
        std::shared_ptr<DevMem> mem;
        u64 *ptr = nullptr;
    };
    DevBuf alloc_u64(size_t count);
    void h2d(u64 *dst, const u64 *src, size_t count);
    void d2h(u64 *dst, const u64 *src, size_t count);

    void sync();
    void *stream_handle();   // hipStream_t
    int device() const;
    Counters ctr;

    struct Impl;
    std::unique_ptr<Impl> impl;

  private:
    struct ForkTag {};
    explicit Engine(ForkTag);

  private:
    std::shared_ptr<int> ps_split_ = std::make_shared<int>(PS_SPLIT_OPENFHE);
    CtPtr new_ct(int level, int slots, double scale, size_t limbs, int batch = 1);
};

// Raised on a rotation index with no key (the reference's OpenFHE raises on
// EvalRotate with a missing key).
struct NoKeyError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

}  // namespace fhe
