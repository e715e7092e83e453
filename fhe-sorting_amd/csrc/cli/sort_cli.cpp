// fhesort — the reference's competition CLI (src/main.cpp:9-44 + SortContext,
// src/sort.h:15-103) on the MI355X engine, written against the C-ABI only.
//
//   fhesort --cc CC --key_pub PK --key_mult MK --key_rot RK --input CT --output OUT
//
// Same flags and flow as the reference: deserialise the crypto context, public
// key, eval-mult key, eval-automorphism keys and the input ciphertext (exit 1
// with the reference's message when one fails), run DirectSort<128> with
// CompositeSign(4, 3, 3) over the rotation set of main.cpp:38-40, serialise the
// sorted ciphertext.  Files are in the engine's wire format (csrc/wire/wire.hpp),
// not OpenFHE's BINARY archives.
//
// Extensions (all optional): --n N (array size, default 128; other sizes use
// getSizeParameters' rotation set), --sign n,dg,df, --device D, --coeff-dir DIR
// (default <binary>/../data), --stack / --lanes (fhe_set_sort_stack / _lanes),
// --timing (phase times on stderr).
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/fhe_gpu.h"

namespace {

[[noreturn]] void die(const char *msg) {
    std::fprintf(stderr, "%s\n", msg);
    std::exit(1);
}
void detail() {
    const char *e = fhe_last_error();
    if (e && *e) std::fprintf(stderr, "  (%s)\n", e);
}
std::string exe_dir() {
    char buf[4096];
    const ssize_t k = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
    if (k <= 0) return ".";
    buf[k] = 0;
    std::string s(buf);
    const size_t p = s.rfind('/');
    return p == std::string::npos ? "." : s.substr(0, p);
}
double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

int main(int argc, char **argv) {
    std::string pub, mult, rot, cc, array, output, coeff_dir;
    int N = 128, sn = 4, sdg = 3, sdf = 3, device = 0, stack = 0, lanes = 0;
    bool timing = false;
    // flag / value pairs, as main.cpp:14-30 (an unpaired trailing flag is ignored)
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--timing") {
            timing = true;
            continue;
        }
        if (i + 1 >= argc) break;
        const char *v = argv[++i];
        if (a == "--key_pub") pub = v;
        else if (a == "--key_mult") mult = v;
        else if (a == "--key_rot") rot = v;
        else if (a == "--cc") cc = v;
        else if (a == "--input" || a == "--array") array = v;
        else if (a == "--output") output = v;
        else if (a == "--n") N = std::atoi(v);
        else if (a == "--sign") {
            if (std::sscanf(v, "%d,%d,%d", &sn, &sdg, &sdf) != 3) die("--sign takes n,dg,df");
        } else if (a == "--device") device = std::atoi(v);
        else if (a == "--coeff-dir") coeff_dir = v;
        else if (a == "--stack") stack = std::atoi(v);
        else if (a == "--lanes") lanes = std::atoi(v);
        else {
            std::fprintf(stderr, "unknown flag %s\n", a.c_str());
            return 2;
        }
    }
    if (coeff_dir.empty()) coeff_dir = exe_dir() + "/../data";
    if (fhe_set_coeff_dir(coeff_dir.c_str()) != FHE_OK) die("Could not set the coefficient directory");

    // rotation set: main.cpp:38-40 for the reference's N = 128, else getSizeParameters'
    std::vector<int32_t> rots;
    if (N == 128) {
        rots = {-1, -2, -4, -8, -16, -32, 1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384};
    } else {
        int depth = 0;
        rots.resize(256);
        const int nr = fhe_size_parameters(N, &depth, rots.data(), (int)rots.size());
        if (nr < 0) die("Unsupported array size");
        rots.resize(nr);
    }

    const double t0 = now();
    fhe_ctx *ctx = nullptr;
    if (fhe_deserialize_context(cc.c_str(), device, &ctx) != FHE_OK) {
        std::fprintf(stderr, "Could not deserialize cryptocontext file\n");
        detail();
        return 1;
    }
    if (fhe_deserialize_public_key(ctx, pub.c_str()) != FHE_OK) {
        std::fprintf(stderr, "Could not deserialize public key file\n");
        detail();
        return 1;
    }
    if (fhe_deserialize_eval_mult_key(ctx, mult.c_str()) != FHE_OK) {
        std::fprintf(stderr, "Could not deserialize mult key file\n");
        detail();
        return 1;
    }
    int nkeys = 0;
    if (fhe_deserialize_eval_automorphism_key(ctx, rot.c_str(), &nkeys) != FHE_OK) {
        std::fprintf(stderr, "Could not deserialize eval rot key file\n");
        detail();
        return 1;
    }
    fhe_ct *x = nullptr;
    if (fhe_deserialize_ciphertext(ctx, array.c_str(), &x) != FHE_OK) {
        std::fprintf(stderr, "Could not deserialize array cipher\n");
        detail();
        return 1;
    }
    const double t1 = now();
    if (stack > 0) fhe_set_sort_stack(ctx, stack);
    if (lanes > 0) fhe_set_sort_lanes(ctx, lanes);

    // SortContext::eval (src/sort.h:76-95): DirectSort<N>::sort, CompositeSign(4, 3, 3)
    fhe_ct *y = nullptr;
    if (fhe_direct_sort(ctx, x, nullptr, N, rots.data(), (int)rots.size(), sn, sdg, sdf, 0, 0, 1, nullptr, nullptr,
                        &y) != FHE_OK) {
        std::fprintf(stderr, "Sort failed\n");
        detail();
        return 1;
    }
    fhe_sync(ctx);
    const double t2 = now();
    // deserializeOutput (src/sort.h:97-102): the reference prints and carries on;
    // here the failure is also the exit status
    int rc = 0;
    if (fhe_serialize_ciphertext(ctx, y, output.c_str()) != FHE_OK) {
        std::fprintf(stderr, " Error writing ciphertext 1\n");
        detail();
        rc = 1;
    }
    const double t3 = now();
    if (timing) {
        int level = 0;
        fhe_ct_info(y, &level, nullptr, nullptr, nullptr);
        std::fprintf(stderr,
                     "{\"load_s\": %.3f, \"sort_s\": %.3f, \"store_s\": %.3f, \"rotation_keys\": %d, \"N\": %d, "
                     "\"output_level\": %d}\n",
                     t1 - t0, t2 - t1, t3 - t2, nkeys, N, level);
    }
    fhe_ct_free(y);
    fhe_ct_free(x);
    fhe_ctx_destroy(ctx);
    return rc;
}
