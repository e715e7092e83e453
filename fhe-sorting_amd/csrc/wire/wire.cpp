// Wire format reader / writer (layout: wire.hpp).  Host-only C++: objects move
// between HBM and the file through the engine's key export / load calls and
// ciphertext download / upload, one key (≤ a few hundred MB) at a time.
#include "wire.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cmath>
#include <cstring>
#include <memory>
#include <stdexcept>

namespace fhe {
namespace wire {

namespace {
constexpr size_t kHeaderWords = 8;
constexpr size_t kChunkWords = size_t(1) << 20;  // 8 MiB per read/write call

inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
constexpr uint64_t P1 = 0x9e3779b185ebca87ull, P2 = 0xc2b2ae3d27d4eb4full;

struct File {
    FILE *f = nullptr;
    std::string path;
    File() = default;
    File(const std::string &p, const char *mode) : path(p) {
        f = std::fopen(p.c_str(), mode);
        if (!f) throw IoError("cannot open " + p + (mode[0] == 'w' ? " for writing" : " for reading"));
    }
    ~File() {
        if (f) std::fclose(f);
    }
    void close() {
        if (f && std::fclose(f) != 0) {
            f = nullptr;
            throw IoError("write error on " + path);
        }
        f = nullptr;
    }
};

// the process umask without changing it (umask(2) can only be read by setting
// it, which would race with other threads creating files): /proc/self/status
mode_t current_umask() {
    if (FILE *f = std::fopen("/proc/self/status", "r")) {
        char line[256];
        unsigned m = 022;
        bool found = false;
        while (std::fgets(line, sizeof line, f))
            if (std::sscanf(line, "Umask: %o", &m) == 1) {
                found = true;
                break;
            }
        std::fclose(f);
        if (found) return (mode_t)m;
    }
    return 022;
}

// Writes go to a temporary file beside the target that replaces the target by
// rename() only once the whole object is written: a failed write never leaves
// a truncated file in place of a good one.  The temporary name has a random
// suffix and is created exclusively (mkostemp: O_CREAT | O_EXCL, never through
// an existing file or symlink, so concurrent writers of one path and other
// users of the directory cannot hand it an inode of theirs); its mode is set
// on the descriptor before any byte is written: 0600 for a secret key, 0644
// less the umask otherwise.
class Writer {
  public:
    Writer(const std::string &path, Kind kind, uint64_t pid, const host::Params &P, uint64_t body_words)
        : target_(path) {
        std::string tmpl = path + ".tmp.XXXXXX";
        const int fd = ::mkostemp(&tmpl[0], O_CLOEXEC);
        if (fd < 0) throw IoError("cannot open " + path + " for writing");
        tmp_ = tmpl;
        const mode_t mode = kind == SecretKey ? 0600 : 0644 & ~current_umask();
        if (::fchmod(fd, mode) != 0) {
            ::close(fd);
            ::unlink(tmp_.c_str());
            throw IoError("cannot set the mode of " + path);
        }
        file_.path = path;
        file_.f = ::fdopen(fd, "wb");
        if (!file_.f) {
            ::close(fd);
            ::unlink(tmp_.c_str());
            throw IoError("cannot open " + path + " for writing");
        }
        // the destructor does not run for a throwing constructor: a failed header
        // write removes the temporary file here
        try {
            const uint64_t h[kHeaderWords] = {kMagic, (uint64_t)kVersion | ((uint64_t)kind << 32), pid,
                                              (uint64_t)P.logN, P.nq(), (uint64_t)P.K, body_words, 0};
            raw(h, 1);
            put(h + 1, kHeaderWords - 1);
        } catch (...) {
            std::fclose(file_.f);
            file_.f = nullptr;
            ::unlink(tmp_.c_str());
            throw;
        }
        left_ = body_words;
    }
    ~Writer() {
        if (!done_) {
            if (file_.f) std::fclose(file_.f);
            file_.f = nullptr;
            ::unlink(tmp_.c_str());
        }
    }
    void put(const uint64_t *w, size_t count) {
        sum_.update(w, count);
        raw(w, count);
    }
    void body(const uint64_t *w, size_t count) {
        if (count > left_) throw std::logic_error("wire: body larger than declared");
        left_ -= count;
        put(w, count);
    }
    void word(uint64_t w) { body(&w, 1); }
    void finish() {
        if (left_) throw std::logic_error("wire: body shorter than declared");
        const uint64_t d = sum_.digest();
        raw(&d, 1);
        if (std::fflush(file_.f) != 0 || ::fsync(::fileno(file_.f)) != 0) throw IoError("write error on " + target_);
        file_.close();
        if (::rename(tmp_.c_str(), target_.c_str()) != 0) throw IoError("cannot replace " + target_);
        done_ = true;
    }

  private:
    void raw(const uint64_t *w, size_t count) {
        if (std::fwrite(w, 8, count, file_.f) != count) throw IoError("write error on " + file_.path);
    }
    std::string target_, tmp_;
    File file_;
    Checksum sum_;
    uint64_t left_ = 0;
    bool done_ = false;
};

// opens a file, validates header and checksum (one streaming pass), then
// serves the body from its start
class Reader {
  public:
    Reader(const std::string &path) : file_(path, "rb") {
        uint64_t h[kHeaderWords];
        if (std::fread(h, 8, kHeaderWords, file_.f) != kHeaderWords) throw IoError(path + ": not a wire file (short header)");
        if (h[0] != kMagic) throw IoError(path + ": not a wire file (bad magic)");
        info.version = (uint32_t)h[1];
        info.kind = (uint32_t)(h[1] >> 32);
        if (info.version != kVersion)
            throw IoError(path + ": wire version " + std::to_string(info.version) + " (this build reads " +
                          std::to_string(kVersion) + ")");
        info.params_id = h[2];
        info.log_n = h[3];
        info.nq = h[4];
        info.K = h[5];
        info.body_words = h[6];
        if (std::fseek(file_.f, 0, SEEK_END) != 0) throw IoError(path + ": cannot seek");
        const long long size = std::ftell(file_.f);
        if (size < 0 || (uint64_t)size != (kHeaderWords + info.body_words + 1) * 8)
            throw IoError(path + ": truncated or oversized (" + std::to_string(size) + " bytes, header declares " +
                          std::to_string((kHeaderWords + info.body_words + 1) * 8) + ")");
        Checksum sum;
        sum.update(h + 1, kHeaderWords - 1);
        seek_body();
        std::vector<uint64_t> buf(std::min<uint64_t>(kChunkWords, std::max<uint64_t>(info.body_words, 1)));
        for (uint64_t left = info.body_words; left;) {
            const size_t c = (size_t)std::min<uint64_t>(left, buf.size());
            raw(buf.data(), c);
            sum.update(buf.data(), c);
            left -= c;
        }
        uint64_t d = 0;
        raw(&d, 1);
        if (d != sum.digest()) throw IoError(path + ": checksum mismatch (corrupted file)");
        seek_body();
    }
    void expect(Kind k, uint64_t pid, const host::Params &P) {
        if (info.kind != (uint32_t)k)
            throw std::invalid_argument(file_.path + " holds a " + kind_name(info.kind) + ", not a " + kind_name(k));
        if (info.params_id != pid || info.log_n != (uint64_t)P.logN || info.nq != P.nq() || info.K != (uint64_t)P.K)
            throw std::invalid_argument(file_.path + ": " + kind_name(k) +
                                        " was written under a different crypto context (ring 2^" +
                                        std::to_string(info.log_n) + ", " + std::to_string(info.nq) +
                                        " Q primes; this context: ring 2^" + std::to_string(P.logN) + ", " +
                                        std::to_string(P.nq()) + ")");
    }
    void get(uint64_t *w, size_t count) {
        if (count > left_) throw IoError(file_.path + ": body shorter than its contents");
        left_ -= count;
        raw(w, count);
    }
    uint64_t word() {
        uint64_t w;
        get(&w, 1);
        return w;
    }
    void done() {
        if (left_) throw IoError(file_.path + ": " + std::to_string(left_) + " trailing body words");
    }
    Info info;
    const std::string &path() const { return file_.path; }
    void rewind() { seek_body(); }

  private:
    void seek_body() {
        if (std::fseek(file_.f, (long)(kHeaderWords * 8), SEEK_SET) != 0) throw IoError(file_.path + ": cannot seek");
        left_ = info.body_words;
    }
    void raw(uint64_t *w, size_t count) {
        if (std::fread(w, 8, count, file_.f) != count) throw IoError(file_.path + ": read error");
    }
    File file_;
    uint64_t left_ = 0;
};

// residues of `limbs` polynomials of n words over primes[first..first+limbs)
void check_residues(const uint64_t *w, size_t limbs, size_t n, const std::vector<uint64_t> &primes, size_t first,
                    const std::string &path) {
    for (size_t l = 0; l < limbs; ++l) {
        const uint64_t q = primes[first + l];
        const uint64_t *p = w + l * n;
        uint64_t bad = 0;
        for (size_t k = 0; k < n; ++k) bad |= (uint64_t)(p[k] >= q);
        if (bad) throw std::invalid_argument(path + ": residue out of range for prime " + std::to_string(first + l));
    }
}
// a switching key [digits][2][nall][n]
void check_switch_key(const uint64_t *w, const host::Params &P, int digits, const std::string &path) {
    for (int j = 0; j < 2 * digits; ++j) check_residues(w + (size_t)j * P.nall() * P.n, P.nall(), P.n, P.primes, 0, path);
}
uint64_t pid_of(const Engine &e, const CtxParams &p) { return params_id(p, e.params().primes); }
}  // namespace

void Checksum::update(const uint64_t *w, size_t count) {
    size_t i = 0;
    // the lane of word j is (count_ + j) & 3: keep the 4-word rhythm across calls
    while (i < count && ((count_ + i) & 3)) {
        uint64_t &l = lane_[(count_ + i) & 3];
        l = rotl(l ^ (w[i] * P1), 31) * P2;
        ++i;
    }
    uint64_t a = lane_[0], b = lane_[1], c = lane_[2], d = lane_[3];
    for (; i + 4 <= count; i += 4) {
        a = rotl(a ^ (w[i] * P1), 31) * P2;
        b = rotl(b ^ (w[i + 1] * P1), 31) * P2;
        c = rotl(c ^ (w[i + 2] * P1), 31) * P2;
        d = rotl(d ^ (w[i + 3] * P1), 31) * P2;
    }
    lane_[0] = a, lane_[1] = b, lane_[2] = c, lane_[3] = d;
    for (; i < count; ++i) {
        uint64_t &l = lane_[(count_ + i) & 3];
        l = rotl(l ^ (w[i] * P1), 31) * P2;
    }
    count_ += count;
}
uint64_t Checksum::digest() const {
    uint64_t h = rotl(lane_[0], 1) + rotl(lane_[1], 7) + rotl(lane_[2], 12) + rotl(lane_[3], 18);
    h ^= count_ * P1;
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    return h;
}

uint64_t params_id(const CtxParams &p, const std::vector<uint64_t> &primes) {
    Checksum s;
    const uint64_t w[5] = {(uint64_t)p.log_n, (uint64_t)p.mult_depth, (uint64_t)p.scale_bits, (uint64_t)p.first_bits,
                           (uint64_t)p.dnum};
    s.update(w, 5);
    s.update(primes.data(), primes.size());
    return s.digest();
}

const char *kind_name(uint32_t kind) {
    switch (kind) {
    case Context: return "crypto context";
    case PublicKey: return "public key";
    case EvalMultKey: return "eval-mult key";
    case Automorphism: return "eval-automorphism key set";
    case CiphertextK: return "ciphertext";
    case SecretKey: return "secret key";
    default: return "unknown object";
    }
}

Info inspect(const std::string &path) { return Reader(path).info; }

// ------------------------------------------------------------- context ---
void save_context(const Engine &e, const CtxParams &p, const std::string &path) {
    const auto &P = e.params();
    Writer w(path, Context, pid_of(e, p), P, 7 + P.nall());
    // the seed word stays 0: a context file goes to the untrusted evaluator, and
    // a deterministic seed would let it regenerate the secret key
    const uint64_t h[7] = {(uint64_t)p.log_n, (uint64_t)p.mult_depth, (uint64_t)p.scale_bits, (uint64_t)p.first_bits,
                           (uint64_t)p.dnum, 0, (uint64_t)P.nall()};
    w.body(h, 7);
    w.body(P.primes.data(), P.nall());
    w.finish();
}
CtxParams read_context(const std::string &path) {
    Reader r(path);
    if (r.info.kind != Context)
        throw std::invalid_argument(path + " holds a " + kind_name(r.info.kind) + ", not a crypto context");
    CtxParams p;
    p.log_n = (int)r.word();
    p.mult_depth = (int)r.word();
    p.scale_bits = (int)r.word();
    p.first_bits = (int)r.word();
    p.dnum = (int)r.word();
    (void)r.word();  // seed word: never taken from a file (a deserialised context samples from getrandom)
    p.seed = 0;
    if (p.log_n != (int)r.info.log_n || (uint64_t)p.mult_depth + 1 != r.info.nq)
        throw IoError(path + ": context header and body disagree");
    // a context file drives allocations: refuse parameters no engine build uses
    if (p.log_n < 10 || p.log_n > 17 || p.mult_depth < 1 || p.mult_depth > 200 || p.scale_bits < 20 ||
        p.scale_bits > 60 || p.first_bits < 20 || p.first_bits > 60 || p.dnum < 1 || p.dnum > 64)
        throw std::invalid_argument(path + ": context parameters out of range (ring 2^" + std::to_string(p.log_n) +
                                    ", depth " + std::to_string(p.mult_depth) + ")");
    return p;
}
void check_context(const Engine &e, const CtxParams &p, const std::string &path) {
    Reader r(path);
    const auto &P = e.params();
    r.expect(Context, pid_of(e, p), P);  // params_id covers the primes
    for (int i = 0; i < 6; ++i) r.word();
    const uint64_t nall = r.word();
    std::vector<uint64_t> primes(nall);
    r.get(primes.data(), nall);
    r.done();
    if (primes != P.primes) throw std::invalid_argument(path + ": the file's primes differ from this build's");
}

// ---------------------------------------------------------------- keys ---
void save_public_key(Engine &e, const CtxParams &p, const std::string &path) {
    const auto &P = e.params();
    std::vector<uint64_t> pk(2 * P.nq() * P.n);
    e.export_public(pk.data());
    Writer w(path, PublicKey, pid_of(e, p), P, pk.size());
    w.body(pk.data(), pk.size());
    w.finish();
}
void load_public_key(Engine &e, const CtxParams &p, const std::string &path) {
    const auto &P = e.params();
    Reader r(path);
    r.expect(PublicKey, pid_of(e, p), P);
    std::vector<uint64_t> pk(2 * P.nq() * P.n);
    r.get(pk.data(), pk.size());
    r.done();
    for (int c = 0; c < 2; ++c) check_residues(pk.data() + c * P.nq() * P.n, P.nq(), P.n, P.primes, 0, path);
    e.load_public(pk.data());
}
void save_secret_key(Engine &e, const CtxParams &p, const std::string &path) {
    const auto &P = e.params();
    std::vector<uint64_t> s(P.nall() * P.n);
    e.export_secret(s.data());
    Writer w(path, SecretKey, pid_of(e, p), P, s.size());
    w.body(s.data(), s.size());
    w.finish();
}
void load_secret_key(Engine &e, const CtxParams &p, const std::string &path) {
    const auto &P = e.params();
    Reader r(path);
    r.expect(SecretKey, pid_of(e, p), P);
    std::vector<uint64_t> s(P.nall() * P.n);
    r.get(s.data(), s.size());
    r.done();
    check_residues(s.data(), P.nall(), P.n, P.primes, 0, path);
    e.load_secret(s.data());
}
void save_eval_mult_key(Engine &e, const CtxParams &p, const std::string &path) {
    const auto &P = e.params();
    std::vector<uint64_t> k(e.switch_key_words());
    e.export_relin(k.data());
    Writer w(path, EvalMultKey, pid_of(e, p), P, 1 + k.size());
    w.word((uint64_t)e.key_digits());
    w.body(k.data(), k.size());
    w.finish();
}
void load_eval_mult_key(Engine &e, const CtxParams &p, const std::string &path) {
    const auto &P = e.params();
    Reader r(path);
    r.expect(EvalMultKey, pid_of(e, p), P);
    if (r.word() != (uint64_t)e.key_digits()) throw std::invalid_argument(path + ": key digit count differs");
    std::vector<uint64_t> k(e.switch_key_words());
    r.get(k.data(), k.size());
    r.done();
    check_switch_key(k.data(), P, e.key_digits(), path);
    e.load_relin(k.data());
}
void save_automorphism_keys(Engine &e, const CtxParams &p, const std::string &path) {
    const auto &P = e.params();
    const auto gs = e.galois_elements();
    const size_t kw = e.switch_key_words();
    Writer w(path, Automorphism, pid_of(e, p), P, 2 + gs.size() * (1 + kw));
    w.word((uint64_t)e.key_digits());
    w.word(gs.size());
    std::vector<uint64_t> k(kw);
    for (uint64_t g : gs) {
        e.export_galois(g, k.data());
        w.word(g);
        w.body(k.data(), kw);
    }
    w.finish();
}
int load_automorphism_keys(Engine &e, const CtxParams &p, const std::string &path) {
    const auto &P = e.params();
    Reader r(path);
    r.expect(Automorphism, pid_of(e, p), P);
    if (r.word() != (uint64_t)e.key_digits()) throw std::invalid_argument(path + ": key digit count differs");
    const uint64_t count = r.word();
    const size_t kw = e.switch_key_words();
    if (r.info.body_words != 2 + count * (1 + kw)) throw IoError(path + ": key count and body size disagree");
    // validate every key before installing any
    std::vector<uint64_t> k(kw);
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1) {
            r.rewind();
            r.word();
            r.word();
        }
        for (uint64_t i = 0; i < count; ++i) {
            const uint64_t g = r.word();
            if (!(g & 1) || g >= 2 * P.n) throw std::invalid_argument(path + ": bad galois element " + std::to_string(g));
            r.get(k.data(), kw);
            if (pass == 0)
                check_switch_key(k.data(), P, e.key_digits(), path);
            else
                e.load_galois(g, k.data());
        }
    }
    r.done();
    return (int)count;
}

// ---------------------------------------------------------- ciphertext ---
void save_ciphertext(Engine &e, const CtxParams &p, const Ciphertext &ct, const std::string &path) {
    if (ct.batch != 1) throw std::invalid_argument("serialize: one ciphertext at a time (member() of a batch)");
    const auto &P = e.params();
    std::vector<uint64_t> d(2 * ct.limbs * P.n);
    e.download(ct, d.data());
    Writer w(path, CiphertextK, pid_of(e, p), P, 5 + d.size());
    uint64_t sc;
    std::memcpy(&sc, &ct.scale, 8);
    const uint64_t h[5] = {(uint64_t)ct.level, (uint64_t)ct.slots, (uint64_t)ct.limbs, 1, sc};
    w.body(h, 5);
    w.body(d.data(), d.size());
    w.finish();
}
CtPtr load_ciphertext(Engine &e, const CtxParams &p, const std::string &path) {
    const auto &P = e.params();
    Reader r(path);
    r.expect(CiphertextK, pid_of(e, p), P);
    uint64_t h[5];
    r.get(h, 5);
    const int level = (int)h[0], slots = (int)h[1];
    const size_t limbs = (size_t)h[2];
    double scale;
    std::memcpy(&scale, &h[4], 8);
    if (h[0] > (uint64_t)P.L || limbs != P.limbs_at(level))
        throw std::invalid_argument(path + ": level " + std::to_string(h[0]) + " / " + std::to_string(h[2]) +
                                    " limbs do not fit this context");
    if (h[3] != 1) throw std::invalid_argument(path + ": batched ciphertext files are not supported");
    if (h[1] == 0 || h[1] > P.n / 2 || (h[1] & (h[1] - 1)))
        throw std::invalid_argument(path + ": slot count " + std::to_string(h[1]) + " is not a power of two <= n/2");
    if (!(scale > 0) || !std::isfinite(scale)) throw std::invalid_argument(path + ": bad scale");
    std::vector<uint64_t> d(2 * limbs * P.n);
    r.get(d.data(), d.size());
    r.done();
    for (int c = 0; c < 2; ++c) check_residues(d.data() + c * limbs * P.n, limbs, P.n, P.primes, 0, path);
    return e.upload(d.data(), limbs, level, slots, scale);
}

}  // namespace wire
}  // namespace fhe
