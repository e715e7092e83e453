// Wire format of the engine's objects: contexts, keys and ciphertexts as files.
//
// The reference's CLI (src/sort.h:31-74, 97-102; src/main.cpp:9-44) moves the
// crypto context, the public / eval-mult / eval-automorphism keys and the input
// and output ciphertexts through OpenFHE's Serial::{Serialize,Deserialize}ToFile
// and CryptoContext::{Serialize,Deserialize}Eval{Mult,Automorphism}Key in
// SerType::BINARY.  That byte format belongs to OpenFHE's cereal archives, and
// its key material is tied to OpenFHE's own prime generation and digit split, so
// this engine reads and writes its own format instead:
//
//   header   8 x u64:  magic "FHESORTW", version | kind << 32, params_id,
//                      log_n, nq (Q primes), K (special primes), body_words, 0
//   body     body_words x u64 (layout per kind below)
//   trailer  u64 checksum (wire::checksum over header words 1..7 and the body)
//
//   kind 1 context        log_n, mult_depth, scale_bits, first_bits, dnum, 0 (the
//                         seed word: always written 0 and ignored on read, a
//                         context file never carries key-generation entropy),
//                         nall, primes[nall]
//   kind 2 public key     [2][nq][n]
//   kind 3 eval-mult key  digits, [digits][2][nall][n]
//   kind 4 automorphism   count, then count x (galois element, [digits][2][nall][n])
//   kind 5 ciphertext     level, slots, limbs, batch (1), scale (f64 bits), [2][limbs][n]
//   kind 6 secret key     [nall][n]
//
// Every polynomial is in the engine's evaluation (NTT) form, residues < q_i,
// little-endian.  params_id hashes (log_n, mult_depth, scale_bits, first_bits,
// dnum, primes): a key or ciphertext file is only accepted by a context with
// the same modulus chain.  Readers verify the checksum over the whole file
// before anything is loaded, so a truncated or corrupted file changes nothing.
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../engine/engine.hpp"

namespace fhe {
namespace wire {

enum Kind : uint32_t { Context = 1, PublicKey = 2, EvalMultKey = 3, Automorphism = 4, CiphertextK = 5, SecretKey = 6 };
constexpr uint32_t kVersion = 1;
constexpr uint64_t kMagic = 0x5754524f53454846ull;  // "FHESORTW"

// raised on file-system failures and malformed / corrupted files
struct IoError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

struct CtxParams {
    int log_n = 0, mult_depth = 0, scale_bits = 0, first_bits = 0, dnum = 0;
    uint64_t seed = 0;  // in memory only: never serialised (save_context writes 0)
};

struct Info {
    uint32_t kind = 0, version = 0;
    uint64_t params_id = 0, log_n = 0, nq = 0, K = 0, body_words = 0;
};

// 4-lane multiply-rotate word hash (streamed; order-dependent)
class Checksum {
  public:
    void update(const uint64_t *w, size_t count);
    uint64_t digest() const;

  private:
    uint64_t lane_[4] = {0x9e3779b97f4a7c15ull, 0xc2b2ae3d27d4eb4full, 0x165667b19e3779f9ull, 0x27d4eb2f165667c5ull};
    uint64_t count_ = 0;
};

uint64_t params_id(const CtxParams &p, const std::vector<uint64_t> &primes);
const char *kind_name(uint32_t kind);

// header + checksum validation of any wire file (no engine needed)
Info inspect(const std::string &path);

void save_context(const Engine &e, const CtxParams &p, const std::string &path);
// the parameters stored in a context file (the caller builds the engine from
// them, then calls check_context to compare its primes with the file's)
CtxParams read_context(const std::string &path);
void check_context(const Engine &e, const CtxParams &p, const std::string &path);

void save_public_key(Engine &e, const CtxParams &p, const std::string &path);
void load_public_key(Engine &e, const CtxParams &p, const std::string &path);
void save_secret_key(Engine &e, const CtxParams &p, const std::string &path);
void load_secret_key(Engine &e, const CtxParams &p, const std::string &path);
void save_eval_mult_key(Engine &e, const CtxParams &p, const std::string &path);
void load_eval_mult_key(Engine &e, const CtxParams &p, const std::string &path);
// every galois key the engine holds (rotations and conjugation)
void save_automorphism_keys(Engine &e, const CtxParams &p, const std::string &path);
// returns the number of keys loaded
int load_automorphism_keys(Engine &e, const CtxParams &p, const std::string &path);
void save_ciphertext(Engine &e, const CtxParams &p, const Ciphertext &ct, const std::string &path);
CtPtr load_ciphertext(Engine &e, const CtxParams &p, const std::string &path);

}  // namespace wire
}  // namespace fhe
