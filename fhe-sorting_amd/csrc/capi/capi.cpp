// extern "C" boundary of the MI355X engine (declarations: include/fhe_gpu.h).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <map>
#include <memory>
#include <new>
#include <string>

#include "../../../include/fhe_gpu.h"
#include "../algo/bootstrap.hpp"
#include "../algo/fhesort.hpp"
#include "../device/kernels.hpp"
#include "../algo/kway.hpp"
#include "../engine/engine.hpp"
#include "../wire/wire.hpp"

using namespace fhe;

struct fhe_ctx {
    std::unique_ptr<Engine> eng;
    wire::CtxParams params;  // what the context was built from (wire format)
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1;
    // one rank sorter per (N, rotation set): its encoded public masks persist
    // across sorts like the keys do
    std::map<std::pair<int, std::vector<int>>, std::unique_ptr<DirectSortN>> sorters;
    int sort_stack = 32;
    int sort_lanes = 2;
    bool mask_cache = true;  // fhe_set_mask_cache
    std::unique_ptr<Engine> kway_lane;  // the k-way sorter's second lane (forked on first use)
};
struct fhe_ct {
    CtPtr p;
};
struct fhe_pt {
    PtPtr p;
};
struct fhe_boot {
    std::unique_ptr<Bootstrapper> b;
    std::unique_ptr<Bootstrapper> lane_b;  // the same setup on the context's k-way lane
};
struct fhe_rot_tree {
    std::unique_ptr<RotationTreeN> t;
};

namespace {
thread_local std::string g_err;

template <class F>
int guard(F &&f) {
    try {
        f();
        return FHE_OK;
    } catch (const NoKeyError &e) {
        g_err = e.what();
        return FHE_ENOKEY;
    } catch (const wire::IoError &e) {
        g_err = e.what();
        return FHE_EIO;
    } catch (const std::invalid_argument &e) {
        g_err = e.what();
        return FHE_EINVAL;
    } catch (const std::out_of_range &e) {
        g_err = e.what();
        return FHE_EINVAL;
    } catch (const std::bad_alloc &e) {
        g_err = e.what();
        return FHE_ENOMEM;
    } catch (const std::runtime_error &e) {
        g_err = e.what();
        const std::string m = e.what();
        if (m.find("no levels left") != std::string::npos) return FHE_EDEPTH;
        if (m.find("HIP error") != std::string::npos) return FHE_EHIP;
        return FHE_EINTERNAL;
    } catch (...) {
        g_err = "unknown error";
        return FHE_EINTERNAL;
    }
}
inline fhe_ct *wrap(CtPtr p) { return new fhe_ct{std::move(p)}; }
SignConfig cfgof(int n, int dg, int df) { return SignConfig(CompositeSignConfig(n, dg, df)); }
#define NEED(x)                                                   \
    do {                                                          \
        if (!(x)) throw std::invalid_argument("null argument: " #x); \
    } while (0)
}  // namespace

extern "C" {

const char *fhe_last_error(void) { return g_err.c_str(); }

int fhe_prng_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3], uint32_t out[16]) {
    return guard([&] {
        NEED(key);
        NEED(nonce);
        NEED(out);
        host::chacha20_block(key, counter, nonce, out);
    });
}

int fhe_ctx_create(const fhe_params *p, int device, fhe_ctx **out) {
    return guard([&] {
        NEED(p);
        NEED(out);
        auto c = std::make_unique<fhe_ctx>();
        c->eng = std::make_unique<Engine>(p->log_n, p->mult_depth, p->scale_bits, p->first_bits, p->dnum, device,
                                          p->seed);
        c->params = wire::CtxParams{p->log_n, p->mult_depth, p->scale_bits, p->first_bits, p->dnum, p->seed};
        *out = c.release();
    });
}
int fhe_ctx_destroy(fhe_ctx *ctx) {
    return guard([&] {
        if (!ctx) return;
        if (ctx->comm) ncclCommDestroy(ctx->comm);
        delete ctx;
    });
}
int fhe_ctx_info(fhe_ctx *ctx, int *nq, int *K, int *alpha, uint64_t *primes, double *deltas) {
    return guard([&] {
        NEED(ctx);
        const auto &P = ctx->eng->params();
        if (nq) *nq = (int)P.nq();
        if (K) *K = P.K;
        if (alpha) *alpha = P.alpha;
        if (primes) std::memcpy(primes, P.primes.data(), P.primes.size() * 8);
        if (deltas) std::memcpy(deltas, P.delta.data(), P.delta.size() * 8);
    });
}
int fhe_set_coeff_dir(const char *dir) {
    return guard([&] {
        NEED(dir);
        setCoefficientDir(dir);
    });
}

int fhe_keygen(fhe_ctx *ctx) { return guard([&] { ctx->eng->keygen(); }); }
int fhe_gen_rotation_keys(fhe_ctx *ctx, const int32_t *idx, int n) {
    return guard([&] { ctx->eng->gen_rotation_keys(std::vector<int>(idx, idx + n)); });
}
int fhe_ctx_load_secret(fhe_ctx *ctx, const uint64_t *s) { return guard([&] { ctx->eng->load_secret(s); }); }
int fhe_ctx_load_public(fhe_ctx *ctx, const uint64_t *pk) { return guard([&] { ctx->eng->load_public(pk); }); }
int fhe_ctx_load_keys(fhe_ctx *ctx, const uint64_t *relin, const int32_t *rot_idx, const uint64_t *const *rot_keys,
                      int nrot) {
    return guard([&] {
        if (relin) ctx->eng->load_relin(relin);
        for (int i = 0; i < nrot; ++i) ctx->eng->load_rotation(rot_idx[i], rot_keys[i]);
    });
}
uint64_t fhe_key_bytes(fhe_ctx *ctx) { return ctx ? ctx->eng->key_bytes() : 0; }

int fhe_encrypt(fhe_ctx *ctx, const double *v, int len, int slots, int level, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->encrypt(std::vector<double>(v, v + len), slots, level)); });
}
int fhe_encrypt_ext(fhe_ctx *ctx, const double *v, int len, int slots, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->encrypt_ext(std::vector<double>(v, v + len), slots)); });
}
int fhe_decrypt(fhe_ctx *ctx, const fhe_ct *ct, double *out) {
    return guard([&] {
        auto v = ctx->eng->decrypt(*ct->p);
        std::memcpy(out, v.data(), v.size() * 8);
    });
}
int fhe_ct_upload(fhe_ctx *ctx, const uint64_t *h, int limbs, int level, int slots, double scale, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->upload(h, (size_t)limbs, level, slots, scale)); });
}
int fhe_ct_download(fhe_ctx *ctx, const fhe_ct *ct, uint64_t *h) {
    return guard([&] { ctx->eng->download(*ct->p, h); });
}
int fhe_ct_info(const fhe_ct *ct, int *level, int *slots, double *scale, int *limbs) {
    return guard([&] {
        NEED(ct);
        if (level) *level = ct->p->level;
        if (slots) *slots = ct->p->slots;
        if (scale) *scale = ct->p->scale;
        if (limbs) *limbs = (int)ct->p->limbs;
    });
}
int fhe_ct_set_slots(fhe_ct *ct, int slots) {
    return guard([&] {
        NEED(ct);
        ct->p->slots = slots;
    });
}
int fhe_ct_free(fhe_ct *ct) {
    delete ct;
    return FHE_OK;
}
int fhe_mul_plain_sum(fhe_ctx *ctx, const fhe_ct *const *cts, const fhe_pt *const *pts, int m, fhe_ct **out) {
    return guard([&] {
        NEED(ctx);
        std::vector<const Ciphertext *> a;
        std::vector<const Plaintext *> p;
        for (int i = 0; i < m; ++i) {
            NEED(cts[i]);
            NEED(pts[i]);
            a.push_back(cts[i]->p.get());
            p.push_back(pts[i]->p.get());
        }
        *out = wrap(ctx->eng->mul_plain_sum(a, p));
    });
}
int fhe_ct_stack(fhe_ctx *ctx, const fhe_ct *const *xs, int m, fhe_ct **out) {
    return guard([&] {
        NEED(ctx);
        std::vector<const Ciphertext *> v;
        for (int i = 0; i < m; ++i) {
            NEED(xs[i]);
            v.push_back(xs[i]->p.get());
        }
        *out = wrap(ctx->eng->stack(v));
    });
}
int fhe_ct_member(fhe_ctx *ctx, const fhe_ct *a, int m, fhe_ct **out) {
    return guard([&] {
        NEED(a);
        *out = wrap(ctx->eng->member(*a->p, m));
    });
}
int fhe_ct_sum_members(fhe_ctx *ctx, const fhe_ct *a, fhe_ct **out) {
    return guard([&] {
        NEED(a);
        *out = wrap(ctx->eng->sum_members(*a->p));
    });
}
int fhe_pt_encode(fhe_ctx *ctx, const double *v, int len, int slots, int level, fhe_pt **out) {
    return guard([&] { *out = new fhe_pt{ctx->eng->encode(std::vector<double>(v, v + len), slots, level)}; });
}
int fhe_pt_limbs(const fhe_pt *pt) { return pt && pt->p ? (int)pt->p->limbs : -FHE_EINVAL; }
int fhe_pt_download(fhe_ctx *ctx, const fhe_pt *pt, uint64_t *out) {
    return guard([&] {
        NEED(ctx);
        NEED(pt);
        NEED(pt->p);
        NEED(out);
        ctx->eng->sync();
        if (hipMemcpy(out, pt->p->data, pt->p->limbs * ctx->eng->n() * 8, hipMemcpyDeviceToHost) != hipSuccess)
            throw std::runtime_error("HIP error: plaintext download");
    });
}
int fhe_pt_encode_device(fhe_ctx *ctx, const double *v, int len, int slots, int level, fhe_pt **out) {
    return guard([&] {
        NEED(ctx);
        NEED(v);
        *out = new fhe_pt{ctx->eng->encode_device({std::vector<double>(v, v + len)}, slots, {level})[0]};
    });
}
int fhe_pt_encode_masks(fhe_ctx *ctx, const int32_t *spec, int count, int num_slots, int N, fhe_pt **out) {
    return guard([&] {
        NEED(ctx);
        NEED(spec);
        NEED(out);
        if (count < 0) throw std::invalid_argument("fhe_pt_encode_masks: negative count");
        std::vector<Engine::MaskSpec> m(count);
        for (int i = 0; i < count; ++i) {
            if (spec[4 * i] != 0 && spec[4 * i] != 1) throw std::invalid_argument("fhe_pt_encode_masks: kind must be 0 or 1");
            m[i] = Engine::MaskSpec{spec[4 * i], spec[4 * i + 1], spec[4 * i + 2], spec[4 * i + 3]};
        }
        auto pts = ctx->eng->encode_masks(m, num_slots, N);
        for (int i = 0; i < count; ++i) out[i] = new fhe_pt{pts[i]};
    });
}
int fhe_pt_upload(fhe_ctx *ctx, const uint64_t *h, int limbs, int level, int slots, double scale, fhe_pt **out) {
    return guard([&] { *out = new fhe_pt{ctx->eng->upload_pt(h, (size_t)limbs, level, slots, scale)}; });
}
int fhe_pt_free(fhe_pt *pt) {
    delete pt;
    return FHE_OK;
}

#define OP1(name, expr) \
    int name(fhe_ctx *ctx, const fhe_ct *a, fhe_ct **out) { return guard([&] { *out = wrap(expr); }); }
OP1(fhe_negate, ctx->eng->negate(*a->p))
OP1(fhe_rescale, ctx->eng->rescale(*a->p))
OP1(fhe_square_relin, ctx->eng->square(*a->p))
int fhe_add(fhe_ctx *ctx, const fhe_ct *a, const fhe_ct *b, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->add(*a->p, *b->p)); });
}
int fhe_sub(fhe_ctx *ctx, const fhe_ct *a, const fhe_ct *b, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->sub(*a->p, *b->p)); });
}
int fhe_mul_relin(fhe_ctx *ctx, const fhe_ct *a, const fhe_ct *b, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->mul(*a->p, *b->p)); });
}
int fhe_add_const(fhe_ctx *ctx, const fhe_ct *a, double c, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->add_const(*a->p, c)); });
}
int fhe_mul_const(fhe_ctx *ctx, const fhe_ct *a, double c, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->mul_const(*a->p, c)); });
}
int fhe_mul_const_to(fhe_ctx *ctx, const fhe_ct *a, double c, int t, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->mul_const_to(*a->p, c, t)); });
}
int fhe_mul_int(fhe_ctx *ctx, const fhe_ct *a, int64_t k, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->mul_int(*a->p, k)); });
}
int fhe_level_adjust(fhe_ctx *ctx, const fhe_ct *a, int t, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->level_adjust(*a->p, t)); });
}
int fhe_mul_plain(fhe_ctx *ctx, const fhe_ct *a, const fhe_pt *p, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->mul_plain(*a->p, *p->p)); });
}
int fhe_add_plain(fhe_ctx *ctx, const fhe_ct *a, const fhe_pt *p, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->add_plain(*a->p, *p->p)); });
}
int fhe_rotate(fhe_ctx *ctx, const fhe_ct *a, int k, fhe_ct **out) {
    return guard([&] { *out = wrap(ctx->eng->rotate(*a->p, k)); });
}
int fhe_rotate_hoisted(fhe_ctx *ctx, const fhe_ct *a, const int32_t *ks, int m, fhe_ct **outs) {
    return guard([&] {
        auto v = ctx->eng->rotate_hoisted(*a->p, std::vector<long>(ks, ks + m));
        for (int i = 0; i < m; ++i) outs[i] = wrap(v[i]);
    });
}
int fhe_linear_sum_to(fhe_ctx *ctx, const fhe_ct *const *xs, const double *c, int m, int t, fhe_ct **out) {
    return guard([&] {
        std::vector<const Ciphertext *> v;
        for (int i = 0; i < m; ++i) v.push_back(xs[i]->p.get());
        *out = wrap(ctx->eng->linear_sum_to(v, std::vector<double>(c, c + m), t));
    });
}
int fhe_cheb_ps(fhe_ctx *ctx, const fhe_ct *a, const double *coeffs, int nc, double lo, double hi, fhe_ct **out) {
    return guard([&] {
        *out = wrap(evalChebyshevSeriesPS(*ctx->eng, *a->p, std::vector<double>(coeffs, coeffs + nc), lo, hi));
    });
}
int fhe_sign_composite(fhe_ctx *ctx, const fhe_ct *x, int n, int dg, int df, fhe_ct **out) {
    return guard([&] { *out = wrap(sign(*x->p, *ctx->eng, SignFunc::CompositeSign, cfgof(n, dg, df))); });
}
int fhe_compare(fhe_ctx *ctx, const fhe_ct *a, const fhe_ct *b, int n, int dg, int df, fhe_ct **out) {
    return guard([&] {
        Comparison c;
        *out = wrap(c.compare(*ctx->eng, *a->p, *b->p, SignFunc::CompositeSign, cfgof(n, dg, df)));
    });
}
int fhe_indicator(fhe_ctx *ctx, const fhe_ct *x, double k, int n, int dg, int df, fhe_ct **out) {
    return guard([&] {
        Comparison c;
        *out = wrap(c.indicator(*ctx->eng, *x->p, k, SignFunc::CompositeSign, cfgof(n, dg, df)));
    });
}
int fhe_compose_rotate(fhe_ctx *ctx, const fhe_ct *a, int N, const int32_t *rots, int nrot, int algo, int rotation,
                       fhe_ct **out) {
    return guard([&] {
        RotationComposerN rc(*ctx->eng, N, std::vector<int>(rots, rots + nrot), (DecomposeAlgo)algo);
        *out = wrap(rc.rotate(*a->p, rotation));
    });
}
int fhe_compose_rotate_members(fhe_ctx *ctx, const fhe_ct *a, int N, const int32_t *rots, int nrot, int algo,
                               const int32_t *rotations, int count, fhe_ct **out) {
    return guard([&] {
        NEED(ctx);
        NEED(a);
        NEED(a->p);
        NEED(out);
        if (nrot > 0) NEED(rots);
        if (nrot < 0 || count < 0) throw std::invalid_argument("compose_rotate_members: negative count");
        if (count != a->p->batch) throw std::invalid_argument("compose_rotate_members: one rotation per member");
        if (count > 0) NEED(rotations);
        RotationComposerN rc(*ctx->eng, N, std::vector<int>(rots, rots + nrot), (DecomposeAlgo)algo);
        auto m = rc.rotateMembers(*a->p, std::vector<int>(rotations, rotations + count));
        std::vector<const Ciphertext *> v;
        for (auto &x : m) v.push_back(x.get());
        *out = wrap(v.size() == 1 ? ctx->eng->clone(*m[0]) : ctx->eng->stack(v));
    });
}
int fhe_rotation_tree_create(fhe_ctx *ctx, int N, const int32_t *rots, int nrot, int algo, fhe_rot_tree **out) {
    return guard([&] {
        NEED(ctx);
        if (algo < 0 || algo > 2) throw std::invalid_argument("rotation tree: algo must be 0 (NAF), 1 (BNAF), 2 (BINARY)");
        auto t = std::make_unique<fhe_rot_tree>();
        t->t = std::make_unique<RotationTreeN>(*ctx->eng, N, std::vector<int>(rots, rots + nrot), (DecomposeAlgo)algo);
        *out = t.release();
    });
}
int fhe_rotation_tree_build(fhe_rot_tree *t, int start, int end) {
    return guard([&] {
        NEED(t);
        t->t->buildTree(start, end);
    });
}
int fhe_rotation_tree_rotate(fhe_rot_tree *t, const fhe_ct *a, int rotation, fhe_ct **out) {
    return guard([&] {
        NEED(t);
        NEED(a);
        *out = wrap(t->t->treeRotate(*a->p, rotation));
    });
}
int fhe_rotation_tree_stats(const fhe_rot_tree *t, uint64_t stats[5]) {
    return guard([&] {
        NEED(t);
        const RotationStats &s = t->t->getStats();
        const uint64_t v[5] = {s.fastRotationCount, s.normalRotationCount, s.totalRotationCount, s.cacheHits,
                               s.cacheMisses};
        for (int i = 0; i < 5; ++i) stats[i] = v[i];
    });
}
void fhe_rotation_tree_destroy(fhe_rot_tree *t) { delete t; }
int fhe_decompose(int N, const int32_t *rots, int nrot, int rotation, int wrap_n, int algo, int32_t *values,
                  int32_t *sizes, int max_steps) {
    int count = -1;
    int rc = guard([&] {
        DecomposerN d(N, std::vector<int>(rots, rots + nrot));
        auto s = d.decompose(rotation, wrap_n, (DecomposeAlgo)algo);
        count = (int)s.size();
        for (int i = 0; i < count && i < max_steps; ++i) {
            values[i] = s[i].value;
            sizes[i] = s[i].stepSize;
        }
    });
    return rc == FHE_OK ? count : -rc;
}
int fhe_size_parameters(int N, int *depth, int32_t *rots, int max_rots) {
    int count = -1;
    int rc = guard([&] {
        std::vector<int> r;
        directSortSizeParameters(N, *depth, r);
        count = (int)r.size();
        for (int i = 0; i < count && i < max_rots; ++i) rots[i] = r[i];
    });
    return rc == FHE_OK ? count : -rc;
}

// The reduction a sharded sort uses: the caller's hook if given, else RCCL on
// the context's communicator (fhe_comm_init), on the engine stream.
// The reduction of a sharded sort (fhe_gpu.h, fhe_direct_sort):
//  * 1 <= shard_world and 0 <= shard_rank < shard_world, always;
//  * a caller hook, when given, is used (any shard world);
//  * else the RCCL communicator of fhe_comm_init is used iff shard_world equals
//    its world (then shard_rank must be this context's rank): an unsharded sort
//    (0, 1) on a context of a world-8 communicator runs locally, a world-1
//    communicator runs the reduction through RCCL;
//  * else shard_world must be 1 (local).
static CtAllReduce make_allreduce(fhe_ctx *ctx, int shard_rank, int shard_world, fhe_allreduce_fn fn, void *user) {
    if (shard_world < 1 || shard_rank < 0 || shard_rank >= shard_world)
        throw std::invalid_argument("sharded sort: need 1 <= shard_world and 0 <= shard_rank < shard_world");
    if (shard_world > 1) checkShardWorld(ctx->eng->params(), shard_world);  // before any work
    if (fn) {
        // the partial sums are produced asynchronously on the context stream:
        // drain it so the callback sees finished data (it must complete the
        // reduction before returning)
        Engine *eng = ctx->eng.get();
        return [fn, user, eng](u64 *d, size_t c) {
            eng->sync();
            const int rc = fn(d, (uint64_t)c, user);
            if (rc != 0) throw std::runtime_error("HIP error: allreduce hook returned " + std::to_string(rc));
        };
    }
    if (!ctx->comm || shard_world != ctx->world) {
        if (shard_world > 1)
            throw std::invalid_argument(ctx->comm ? "sharded sort: shard world differs from the communicator's world"
                                                  : "sharded sort needs fhe_comm_init or an allreduce hook");
        return nullptr;
    }
    if (shard_rank != ctx->rank)
        throw std::invalid_argument("sharded sort: shard_rank must equal the communicator rank of this context");
    ncclComm_t comm = ctx->comm;
    hipStream_t st = static_cast<hipStream_t>(ctx->eng->stream_handle());
    return [comm, st](u64 *d, size_t c) {
        if (ncclAllReduce(d, d, c, ncclUint64, ncclSum, comm, st) != ncclSuccess)
            throw std::runtime_error("HIP error: ncclAllReduce failed");
    };
}
int fhe_direct_sort(fhe_ctx *ctx, const fhe_ct *x, const fhe_ct *rank, int N, const int32_t *rots, int nrot, int n,
                    int dg, int df, int mode, int shard_rank, int shard_world, fhe_allreduce_fn fn, void *user,
                    fhe_ct **out) {
    return guard([&] {
        NEED(ctx);
        NEED(x);
        CtAllReduce reduce = make_allreduce(ctx, shard_rank, shard_world, fn, user);  // validates the shard first
        auto key = std::make_pair(N, std::vector<int>(rots, rots + nrot));
        auto &slot = ctx->sorters[key];
        if (!slot) slot = std::make_unique<DirectSortN>(*ctx->eng, N, key.second);
        DirectSortN &ds = *slot;
        ds.max_stack = ctx->sort_stack;
        ds.lanes = ctx->sort_lanes;
        ds.cache_masks = ctx->mask_cache;
        ds.shard_rank = shard_rank;
        ds.shard_world = shard_world;
        ds.allreduce = std::move(reduce);
        const SignConfig cfg = cfgof(n, dg, df);
        if (mode == 1)
            *out = wrap(ds.constructRank(*x->p, SignFunc::CompositeSign, cfg));
        else if (mode == 2) {
            NEED(rank);
            *out = wrap(ds.rotationIndexCheckN(*rank->p, *x->p));
        } else
            *out = wrap(ds.sort(*x->p, SignFunc::CompositeSign, cfg));
    });
}

int fhe_sort_hybrid(fhe_ctx *ctx, const fhe_ct *x, const fhe_ct *rank, int N, const int32_t *rots, int nrot, int n,
                    int dg, int df, int mode, int max_array, int mask_mode, int shard_rank, int shard_world,
                    fhe_allreduce_fn fn, void *user, fhe_ct **out) {
    return guard([&] {
        NEED(ctx);
        NEED(x);
        if (max_array < 1 || (max_array & (max_array - 1))) throw std::invalid_argument("sort_hybrid: bad max_array");
        if (mask_mode < 0 || mask_mode > 3) throw std::invalid_argument("sort_hybrid: mask_mode must be 0..3");
        if (shard_world < 1 || shard_rank < 0 || shard_rank >= shard_world)
            throw std::invalid_argument("sort_hybrid: bad shard");
        auto key = std::make_pair(N, std::vector<int>(rots, rots + nrot));
        auto &slot = ctx->sorters[key];
        if (!slot) slot = std::make_unique<DirectSortN>(*ctx->eng, N, key.second);
        DirectSortN &ds = *slot;
        ds.max_stack = ctx->sort_stack;
        ds.lanes = ctx->sort_lanes;
        ds.shard_rank = shard_rank;
        ds.shard_world = shard_world;
        ds.allreduce = make_allreduce(ctx, shard_rank, shard_world, fn, user);
        ds.hybrid_max_array = max_array;
        ds.hybrid_mask = mask_mode;
        if (mode == 1) {
            NEED(rank);
            *out = wrap(ds.rotationIndexCheckHybrid(*rank->p, *x->p));
        } else {
            *out = wrap(ds.sort_hybrid(*x->p, SignFunc::CompositeSign, cfgof(n, dg, df)));
        }
    });
}
int fhe_hybrid_parameters(int N, int *mult_depth, int32_t *rots, int max_rots) {
    int count = -1;
    int rc = guard([&] {
        std::vector<int> r;
        hybridSortSizeParameters(N, *mult_depth, r);
        count = (int)r.size();
        for (int i = 0; i < count && i < max_rots; ++i) rots[i] = r[i];
    });
    return rc == FHE_OK ? count : -rc;
}
int fhe_mehp24_parameters(int N, int *depth, int *log_ring, int *scale_bits, int *dnum, int cfg[3], int *dg_i,
                          int *df_i, int *sub_length, int32_t *rots, int max_rots) {
    int count = -1;
    int rc = guard([&] {
        auto p = mehp24::parameters((size_t)N);
        *depth = p.multDepth;
        *log_ring = p.logRingDim;
        *scale_bits = p.scaleModSize;
        *dnum = p.dnum;
        cfg[0] = p.cfg.compos.n;
        cfg[1] = p.cfg.compos.dg;
        cfg[2] = p.cfg.compos.df;
        *dg_i = (int)p.dg_i;
        *df_i = (int)p.df_i;
        *sub_length = (int)p.subLength;
        count = (int)p.rotations.size();
        for (int i = 0; i < count && i < max_rots; ++i) rots[i] = p.rotations[i];
    });
    return rc == FHE_OK ? count : -rc;
}
int fhe_mehp24_rotation_indices(int N, int sub, int32_t *rots, int max_rots) {
    int count = -1;
    int rc = guard([&] {
        if (N < 1 || sub < 1) throw std::invalid_argument("mehp24: N and sub must be positive");
        auto r = mehp24::utils::getRotationIndices((size_t)N, (size_t)sub);
        count = (int)r.size();
        for (int i = 0; i < count && i < max_rots; ++i) rots[i] = r[i];
    });
    return rc == FHE_OK ? count : -rc;
}
int fhe_mehp24_sort(fhe_ctx *ctx, const fhe_ct *x, int N, int sub, int n, int dg, int df, int dg_i, int df_i,
                    fhe_ct **out) {
    return fhe_mehp24_sort_sharded(ctx, x, N, sub, n, dg, df, dg_i, df_i, 0, 1, nullptr, nullptr, out);
}
int fhe_mehp24_sort_sharded(fhe_ctx *ctx, const fhe_ct *x, int N, int sub, int n, int dg, int df, int dg_i,
                            int df_i, int shard_rank, int shard_world, fhe_allreduce_fn fn, void *user,
                            fhe_ct **out) {
    return guard([&] {
        NEED(ctx);
        NEED(x);
        if (N < 2 || (N & (N - 1))) throw std::invalid_argument("mehp24: N must be a power of two >= 2");
        if (shard_world < 1 || shard_rank < 0 || shard_rank >= shard_world)
            throw std::invalid_argument("mehp24: bad shard");
        Shard sh;
        sh.rank = shard_rank;
        sh.world = shard_world;
        sh.allreduce = make_allreduce(ctx, shard_rank, shard_world, fn, user);
        const SignConfig cfg = cfgof(n, dg, df);
        if (sub == 0) {
            if ((long)N * N != (long)x->p->slots) throw std::invalid_argument("mehp24 sortFG: needs N*N slots");
            *out = wrap(mehp24::sortFG(*x->p, N, SignFunc::CompositeSign, cfg, dg_i, df_i, *ctx->eng,
                                       ctx->sort_stack));
        } else {
            if (sub < 2 || (sub & (sub - 1)) || N % sub) throw std::invalid_argument("mehp24: bad part length");
            if ((long)sub * sub != (long)x->p->slots) throw std::invalid_argument("mehp24: needs sub*sub slots");
            *out = wrap(mehp24::sortLargeArrayFG(*x->p, N, sub, SignFunc::CompositeSign, cfg, dg_i, df_i,
                                                 *ctx->eng, ctx->sort_stack, sh));
        }
    });
}
int fhe_mehp24_indicator(fhe_ctx *ctx, const fhe_ct *x, double b, int dg, int df, fhe_ct **out) {
    return guard([&] {
        NEED(ctx);
        NEED(x);
        *out = wrap(mehp24::indicatorAdv(*ctx->eng, *x->p, b, dg, df));
    });
}

// ------------------------------------------------------------- k-way ----
int fhe_kway_sort(fhe_ctx *ctx, const fhe_ct *x, int k, int M, int dg, int df, fhe_ct **out) {
    return guard([&] {
        NEED(ctx);
        NEED(x);
        NEED(out);
        if (k < 2 || M < 1) throw std::invalid_argument("k-way: k >= 2 and M >= 1 required");
        long N = 1;
        for (int i = 0; i < M && N <= x->p->slots; ++i) N *= k;
        if (N > x->p->slots) throw std::invalid_argument("k-way: k^M exceeds the ciphertext's slots");
        kwaySort::Sorter s(*ctx->eng, N, k, M);
        *out = wrap(s.sorter(*x->p, SignConfig(CompositeSignConfig(3, dg, df), ctx->eng->params().L)));
    });
}

int fhe_kway_sort_boot(fhe_ctx *ctx, const fhe_ct *x, int k, int M, int dg, int df, fhe_boot *boot,
                       int *bootstraps, fhe_ct **out) {
    return guard([&] {
        NEED(ctx);
        NEED(x);
        NEED(out);
        if (k < 2 || M < 1) throw std::invalid_argument("k-way: k >= 2 and M >= 1 required");
        long N = 1;
        for (int i = 0; i < M && N <= x->p->slots; ++i) N *= k;
        if (N > x->p->slots) throw std::invalid_argument("k-way: k^M exceeds the ciphertext's slots");
        if (boot && &boot->b->cc != ctx->eng.get()) throw std::invalid_argument("k-way: bootstrapper of another context");
        kwaySort::Sorter s(*ctx->eng, N, k, M);
        SignConfig cfg(CompositeSignConfig(3, dg, df), ctx->eng->params().L);
        if (boot) {
            Bootstrapper *B = boot->b.get();
            cfg.boot = [B](const Ciphertext &c) { return B->evalBootstrap(c); };
        }
        if (ctx->sort_lanes >= 2) {  // the two comparisons of a stage on two streams
            if (!ctx->kway_lane) ctx->kway_lane = ctx->eng->fork();
            s.laneEng = ctx->kway_lane.get();
            s.laneCfg = cfg;
            if (boot) {
                if (!boot->lane_b) boot->lane_b = std::make_unique<Bootstrapper>(*ctx->kway_lane, boot->b->cfg);
                Bootstrapper *LB = boot->lane_b.get();
                s.laneCfg.boot = [LB](const Ciphertext &c) { return LB->evalBootstrap(c); };
            }
        }
        *out = wrap(s.sorter(*x->p, cfg));
        if (bootstraps) *bootstraps = s.bootstraps;
    });
}

int fhe_check_level_and_boot(fhe_ctx *ctx, const fhe_ct *x, int need, fhe_boot *boot, int *booted, fhe_ct **out) {
    return guard([&] {
        NEED(ctx);
        NEED(x);
        NEED(out);
        if (boot && &boot->b->cc != ctx->eng.get()) throw std::invalid_argument("bootstrapper of another context");
        SignConfig cfg(CompositeSignConfig(3, 2, 2), ctx->eng->params().L);
        if (boot) {
            Bootstrapper *B = boot->b.get();
            cfg.boot = [B](const Ciphertext &c) { return B->evalBootstrap(c); };
        }
        bool b = false;
        *out = wrap(kwaySort::checkLevelAndBoot(*ctx->eng, x->p, need, cfg, &b));
        if (booted) *booted = b ? 1 : 0;
    });
}

int fhe_kway_sorter(fhe_ctx *ctx, int kk, const fhe_ct *const *x, int nx, const fhe_ct *const *cmp, int ncmp,
                    fhe_ct **out) {
    return guard([&] {
        NEED(ctx);
        NEED(x);
        NEED(cmp);
        NEED(out);
        std::vector<CtPtr> xv, cv;
        for (int i = 0; i < nx; ++i) {
            NEED(x[i]);
            xv.push_back(x[i]->p);
        }
        for (int i = 0; i < ncmp; ++i) {
            NEED(cmp[i]);
            cv.push_back(cmp[i]->p);
        }
        if (xv.empty()) throw std::invalid_argument("fhe_kway_sorter: no inputs");
        kwaySort::Sorter s(*ctx->eng, 25, 5, 2);  // the network shape is unused here
        auto o = s.kSorter(kk, xv, cv);
        for (size_t i = 0; i < o.size(); ++i) out[i] = wrap(o[i]);
    });
}
// ----------------------------------------------------- bootstrapping ----
int fhe_boot_create(fhe_ctx *ctx, const fhe_boot_params *p, fhe_boot **out) {
    return guard([&] {
        NEED(ctx);
        NEED(p);
        NEED(out);
        BootstrapConfig c;
        c.slots = p->slots;
        if (p->level_budget_enc) c.budgetEnc = p->level_budget_enc;
        if (p->level_budget_dec) c.budgetDec = p->level_budget_dec;
        if (p->K) c.K = p->K;
        if (p->r) c.r = p->r;
        if (p->degree) c.degree = p->degree;
        if (p->correction_bits) c.correctionBits = p->correction_bits;
        auto b = std::make_unique<fhe_boot>();
        b->b = std::make_unique<Bootstrapper>(*ctx->eng, c);
        *out = b.release();
    });
}
int fhe_boot_destroy(fhe_boot *b) {
    return guard([&] { delete b; });
}
int fhe_boot_keygen(fhe_boot *b) {
    return guard([&] {
        NEED(b);
        b->b->keyGen();
    });
}
int fhe_boot_rotation_indices(const fhe_boot *b, int32_t *rots, int max_rots) {
    int n = -1;
    const int st = guard([&] {
        NEED(b);
        auto r = b->b->rotationIndices();
        for (int i = 0; rots && i < std::min((int)r.size(), max_rots); ++i) rots[i] = r[(size_t)i];
        n = (int)r.size();
    });
    return st == FHE_OK ? n : -st;
}
int fhe_boot_depth(const fhe_boot *b) { return b ? b->b->depth() : -FHE_EINVAL; }
int fhe_bootstrap(fhe_boot *b, const fhe_ct *x, fhe_ct **out) {
    return guard([&] {
        NEED(b);
        NEED(x);
        NEED(out);
        *out = wrap(b->b->evalBootstrap(*x->p));
    });
}
int fhe_bootstrap_stage(fhe_boot *b, const fhe_ct *x, int stage, fhe_ct **out) {
    return guard([&] {
        NEED(b);
        NEED(x);
        NEED(out);
        Bootstrapper &B = *b->b;
        switch (stage) {
            case 0: *out = wrap(B.evalBootstrap(*x->p)); break;
            case 1: *out = wrap(B.coeffsToSlots(*x->p)); break;
            case 2: *out = wrap(B.evalMod(*x->p)); break;
            case 3: *out = wrap(B.slotsToCoeffs(*x->p)); break;
            case 4: *out = wrap(B.cc.mod_raise(*x->p)); break;
            default: throw std::invalid_argument("fhe_bootstrap_stage: stage 0..4");
        }
    });
}
int fhe_conjugate(fhe_ctx *ctx, const fhe_ct *a, fhe_ct **out) {
    return guard([&] {
        NEED(ctx);
        NEED(a);
        NEED(out);
        *out = wrap(ctx->eng->conjugate(*a->p));
    });
}
int fhe_gen_galois_keys(fhe_ctx *ctx, const uint64_t *g, int n) {
    return guard([&] {
        NEED(ctx);
        NEED(g);
        const uint64_t m2 = 2 * (uint64_t)ctx->eng->params().n;
        for (int i = 0; i < n; ++i)
            if (!(g[i] & 1) || g[i] >= m2) throw std::invalid_argument("galois element must be odd and < 2n");
        ctx->eng->gen_galois_keys(std::vector<uint64_t>(g, g + n));
    });
}
int fhe_ctx_load_galois_key(fhe_ctx *ctx, uint64_t g, const uint64_t *key) {
    return guard([&] {
        NEED(ctx);
        NEED(key);
        if (!(g & 1) || g >= 2 * (uint64_t)ctx->eng->params().n) throw std::invalid_argument("galois element must be odd and < 2n");
        ctx->eng->load_galois(g, key);
    });
}
int fhe_pt_encode_complex(fhe_ctx *ctx, const double *re, const double *im, int len, int slots, int level,
                          double scale, fhe_pt **out) {
    return guard([&] {
        NEED(ctx);
        NEED(re);
        NEED(im);
        NEED(out);
        if (level < 0 || level > ctx->eng->params().L) throw std::invalid_argument("level out of range");
        std::vector<std::complex<double>> v;
        for (int i = 0; i < len; ++i) v.emplace_back(re[i], im[i]);
        *out = new fhe_pt{ctx->eng->encode_complex(v, slots, level, scale)};
    });
}

int fhe_kway_sort_type(int k, int M, int stage, int *m, int *log_dist, int *slope) {
    return guard([&] {
        NEED(m);
        NEED(log_dist);
        NEED(slope);
        if (k < 2 || k > 16 || M < 1 || M > 30 || stage < 0 || stage >= kwaySort::stageCount(k, M))
            throw std::invalid_argument("k-way: stage out of range");
        std::tie(*m, *log_dist, *slope) = kwaySort::sortType(k, M, stage);
    });
}

int fhe_kway_stage_count(int k, int M) {
    return (k < 2 || k > 16 || M < 1 || M > 30) ? -FHE_EINVAL : kwaySort::stageCount(k, M);
}

int fhe_kway_rotate_distance(int k, int log_dist, int slope) {
    if (k < 2 || k > 16 || log_dist < 0 || slope < 0 || slope > k) return -FHE_EINVAL;
    long d = 1;
    for (int i = 0; i < log_dist; ++i)
        if ((d *= k) > (1L << 30)) return -FHE_EINVAL;
    return (int)kwaySort::getRotateDistance(k, log_dist, slope);
}

int fhe_kway_gen_indices(int num_slots, int k, int M, int m, int log_dist, int slope, int32_t *group,
                         int32_t *position) {
    return guard([&] {
        NEED(group);
        NEED(position);
        if (k < 2 || k > 16 || M < 1 || M > 30 || m < 0 || log_dist < 0 || m + 1 + log_dist > 30 || num_slots < 1)
            throw std::invalid_argument("k-way: bad index layout");
        long N = 1, blk = 1;
        for (int i = 0; i < M && N <= num_slots; ++i) N *= k;
        for (int i = 0; i < m + 1 + log_dist; ++i) blk *= k;  // dist * k^(m+1): one group block
        if (num_slots < (N + blk - 1) / blk * blk) throw std::invalid_argument("k-way: layout exceeds num_slots");
        auto ind = kwaySort::genIndices(num_slots, k, M, m, log_dist, slope);
        for (int i = 0; i < num_slots; ++i) {
            group[i] = ind[0][(size_t)i];
            position[i] = ind[1][(size_t)i];
        }
    });
}

int fhe_kway_rotation_indices(int N, int32_t *rots, int max_rots) {
    int count = -1;
    int rc = guard([&] {
        if (N < 1 || N > (1 << 30)) throw std::invalid_argument("k-way: N must be in 1..2^30");
        auto r = kwaySort::rotationIndices(N);
        count = (int)r.size();
        for (int i = 0; i < count && i < max_rots; ++i) rots[i] = r[(size_t)i];
    });
    return rc ? -rc : count;
}

int fhe_set_mask_cache(fhe_ctx *ctx, int cache) {
    return guard([&] {
        NEED(ctx);
        ctx->mask_cache = cache != 0;
    });
}

int fhe_set_sort_stack(fhe_ctx *ctx, int max_stack) {
    return guard([&] {
        NEED(ctx);
        if (max_stack < 1) throw std::invalid_argument("max_stack must be >= 1");
        ctx->sort_stack = max_stack;
    });
}

int fhe_set_sort_lanes(fhe_ctx *ctx, int lanes) {
    return guard([&] {
        NEED(ctx);
        if (lanes < 1 || lanes > 8) throw std::invalid_argument("lanes must be in 1..8");
        ctx->sort_lanes = lanes;
    });
}

int fhe_set_ps_split(fhe_ctx *ctx, int split) {
    return guard([&] {
        NEED(ctx);
        if (split != FHE_PS_SPLIT_ENGINE && split != FHE_PS_SPLIT_OPENFHE)
            throw std::invalid_argument("ps split must be FHE_PS_SPLIT_ENGINE or FHE_PS_SPLIT_OPENFHE");
        ctx->eng->set_ps_split(split);
    });
}

int fhe_get_ps_split(const fhe_ctx *ctx) { return ctx ? ctx->eng->ps_split() : -FHE_EINVAL; }

int fhe_cheb_ps_depth(int degree, int split) {
    int d = -1;
    const int rc = guard([&] {
        if (degree < 0 || (split != FHE_PS_SPLIT_ENGINE && split != FHE_PS_SPLIT_OPENFHE))
            throw std::invalid_argument("fhe_cheb_ps_depth: bad degree or split");
        d = chebPSDepthSplit(degree, split);
    });
    return rc ? -rc : d;
}

int fhe_cheb_ps_plan(const double *coeffs, int ncoeffs) {
    int r = -1;
    const int rc = guard([&] {
        NEED(coeffs);
        if (ncoeffs < 1) throw std::invalid_argument("fhe_cheb_ps_plan: no coefficients");
        r = chebPSUsesOpenFHE(std::vector<double>(coeffs, coeffs + ncoeffs)) ? 1 : 0;
    });
    return rc ? -rc : r;
}

int fhe_comm_get_unique_id(uint8_t id[128]) {
    return guard([&] {
        ncclUniqueId u;
        if (ncclGetUniqueId(&u) != ncclSuccess) throw std::runtime_error("HIP error: ncclGetUniqueId failed");
        static_assert(sizeof(u) == 128, "ncclUniqueId size");
        std::memcpy(id, &u, 128);
    });
}
int fhe_comm_init(fhe_ctx *ctx, const uint8_t id[128], int rank, int world) {
    return guard([&] {
        NEED(ctx);
        NEED(id);
        if (rank < 0 || rank >= world) throw std::invalid_argument("fhe_comm_init: rank outside [0, world)");
        checkShardWorld(ctx->eng->params(), world);  // before RCCL is touched
        ncclUniqueId u;
        std::memcpy(&u, id, 128);
        if (hipSetDevice(ctx->eng->device()) != hipSuccess) throw std::runtime_error("HIP error: hipSetDevice");
        if (ncclCommInitRank(&ctx->comm, world, u, rank) != ncclSuccess)
            throw std::runtime_error("HIP error: ncclCommInitRank failed");
        ctx->rank = rank;
        ctx->world = world;
    });
}
int fhe_comm_destroy(fhe_ctx *ctx) {
    return guard([&] {
        if (ctx->comm) ncclCommDestroy(ctx->comm);
        ctx->comm = nullptr;
    });
}
int fhe_ct_allreduce(fhe_ctx *ctx, fhe_ct *ct) {
    if (!ctx || !ctx->comm) {
        g_err = "fhe_ct_allreduce: no communicator";
        return FHE_ENOCOMM;
    }
    return guard([&] {
        NEED(ct);
        // the u64 sum of residues is exact only while world * q_max < 2^64
        checkShardWorld(ctx->eng->params(), ctx->world);
        hipStream_t st = static_cast<hipStream_t>(ctx->eng->stream_handle());
        const size_t cnt = 2 * (size_t)ct->p->batch * ct->p->limbs * ctx->eng->n();
        if (ncclAllReduce(ct->p->data, ct->p->data, cnt, ncclUint64, ncclSum, ctx->comm, st) != ncclSuccess)
            throw std::runtime_error("HIP error: ncclAllReduce failed");
        ctx->eng->reduce_after_allreduce(*ct->p);
    });
}

int fhe_ntt(fhe_ctx *ctx, uint64_t *h, int prime_index, int limbs, int inverse) {
    return guard([&] { ctx->eng->ntt_host(h, prime_index, limbs, inverse != 0); });
}
int fhe_ntt_dev(fhe_ctx *ctx, uint64_t *dev_limbs, int first_prime, int nlimbs, int segments, uint64_t seg_stride,
                int inverse, void *stream) {
    return guard([&] {
        NEED(ctx);
        NEED(dev_limbs);
        ctx->eng->ntt_dev(dev_limbs, first_prime, nlimbs, segments, (size_t)seg_stride, inverse != 0, stream);
    });
}
int fhe_automorph_dev(fhe_ctx *ctx, const uint64_t *dev_in, int limbs, uint64_t galois, uint64_t *dev_out,
                      void *stream) {
    return guard([&] {
        NEED(ctx);
        NEED(dev_in);
        NEED(dev_out);
        ctx->eng->automorph_dev(dev_in, dev_out, (size_t)limbs, galois, stream);
    });
}
int fhe_set_mfma_sums(int mask) { return fhe::dev::set_mfma_sums(mask); }
int fhe_modup(fhe_ctx *ctx, const uint64_t *d, int ell, uint64_t *ext) {
    return guard([&] { ctx->eng->modup_host(d, (size_t)ell, ext); });
}
int fhe_moddown(fhe_ctx *ctx, const uint64_t *in, int ell, uint64_t *out) {
    return guard([&] { ctx->eng->moddown_host(in, (size_t)ell, out); });
}
int fhe_automorph(fhe_ctx *ctx, const uint64_t *in, int limbs, uint64_t g, uint64_t *out) {
    return guard([&] { ctx->eng->automorph_host(in, (size_t)limbs, g, out); });
}
int fhe_counters(fhe_ctx *ctx, uint64_t out[7]) {
    return guard([&] {
        const auto &c = ctx->eng->ctr;
        out[0] = c.hmult;
        out[1] = c.keyswitch;
        out[2] = c.rotations;
        out[3] = c.rescale;
        out[4] = c.ptmult;
        out[5] = c.constmult;
        out[6] = c.opbytes;
    });
}
int fhe_collective_stats(fhe_ctx *ctx, uint64_t out[2]) {
    return guard([&] {
        NEED(ctx);
        out[0] = ctx->eng->ctr.allreduce_ns;
        out[1] = ctx->eng->ctr.allreduce_calls;
    });
}
int fhe_reset_counters(fhe_ctx *ctx) {
    return guard([&] { ctx->eng->ctr = Counters(); });
}
int fhe_sync(fhe_ctx *ctx) { return guard([&] { ctx->eng->sync(); }); }
int fhe_region_marker(fhe_ctx *ctx, int begin) {
    return guard([&] {
        NEED(ctx);
        fhe::dev::region_marker(begin != 0, static_cast<hipStream_t>(ctx->eng->stream_handle()));
    });
}
void *fhe_stream(fhe_ctx *ctx) { return ctx ? ctx->eng->stream_handle() : nullptr; }
int fhe_time_kernel(fhe_ctx *ctx, const char *name, int limbs, int iters, double *avg_ms, double *bytes) {
    return guard([&] {
        NEED(name);
        ctx->eng->time_kernel(name, (size_t)limbs, iters, *avg_ms, *bytes);
    });
}

int fhe_host_stats(double out[4]) {
    return guard([&] {
        NEED(out);
        Engine::host_stats_get(out);
    });
}
int fhe_host_stats_reset(void) {
    return guard([&] { Engine::host_stats_reset(); });
}
int fhe_pool_trim(fhe_ctx *ctx) {
    return guard([&] { ctx->eng->pool_trim(); });
}
int fhe_pool_stats(fhe_ctx *ctx, uint64_t *live, uint64_t *cached, uint64_t *peak) {
    return guard([&] {
        size_t l, c, p;
        ctx->eng->pool_stats(l, c, p);
        *live = l;
        *cached = c;
        *peak = p;
    });
}
int fhe_kernel_clock_start(fhe_ctx *ctx) {
    return guard([&] { ctx->eng->kernel_clock_start(); });
}
int fhe_kernel_clock_stop(fhe_ctx *ctx, char *json, size_t cap, size_t *needed) {
    return guard([&] {
        const std::string s = ctx->eng->kernel_clock_stop();
        if (needed) *needed = s.size() + 1;
        if (json && cap) {
            const size_t m = std::min(cap - 1, s.size());
            std::memcpy(json, s.data(), m);
            json[m] = 0;
        }
    });
}

/* ------------------------------------------------------------ wire format */
int fhe_wire_inspect(const char *path, fhe_wire_info *info) {
    return guard([&] {
        NEED(path);
        NEED(info);
        const auto i = wire::inspect(path);
        info->kind = i.kind;
        info->version = i.version;
        info->params_id = i.params_id;
        info->log_n = i.log_n;
        info->nq = i.nq;
        info->K = i.K;
        info->body_words = i.body_words;
    });
}
int fhe_serialize_context(fhe_ctx *ctx, const char *path) {
    return guard([&] {
        NEED(ctx);
        NEED(path);
        wire::save_context(*ctx->eng, ctx->params, path);
    });
}
int fhe_deserialize_context(const char *path, int device, fhe_ctx **out) {
    return guard([&] {
        NEED(path);
        NEED(out);
        const auto p = wire::read_context(path);
        auto c = std::make_unique<fhe_ctx>();
        c->eng = std::make_unique<Engine>(p.log_n, p.mult_depth, p.scale_bits, p.first_bits, p.dnum, device, p.seed);
        c->params = p;
        wire::check_context(*c->eng, p, path);
        *out = c.release();
    });
}
#define WIRE_KEY(name, call)                     \
    int name(fhe_ctx *ctx, const char *path) {   \
        return guard([&] {                       \
            NEED(ctx);                           \
            NEED(path);                          \
            call(*ctx->eng, ctx->params, path);  \
        });                                      \
    }
WIRE_KEY(fhe_serialize_public_key, wire::save_public_key)
WIRE_KEY(fhe_deserialize_public_key, wire::load_public_key)
WIRE_KEY(fhe_serialize_secret_key, wire::save_secret_key)
WIRE_KEY(fhe_deserialize_secret_key, wire::load_secret_key)
WIRE_KEY(fhe_serialize_eval_mult_key, wire::save_eval_mult_key)
WIRE_KEY(fhe_deserialize_eval_mult_key, wire::load_eval_mult_key)
WIRE_KEY(fhe_serialize_eval_automorphism_key, wire::save_automorphism_keys)
#undef WIRE_KEY
int fhe_deserialize_eval_automorphism_key(fhe_ctx *ctx, const char *path, int *count) {
    return guard([&] {
        NEED(ctx);
        NEED(path);
        const int c = wire::load_automorphism_keys(*ctx->eng, ctx->params, path);
        if (count) *count = c;
    });
}
int fhe_serialize_ciphertext(fhe_ctx *ctx, const fhe_ct *ct, const char *path) {
    return guard([&] {
        NEED(ctx);
        NEED(ct);
        NEED(path);
        wire::save_ciphertext(*ctx->eng, ctx->params, *ct->p, path);
    });
}
int fhe_deserialize_ciphertext(fhe_ctx *ctx, const char *path, fhe_ct **out) {
    return guard([&] {
        NEED(ctx);
        NEED(path);
        NEED(out);
        *out = wrap(wire::load_ciphertext(*ctx->eng, ctx->params, path));
    });
}

}  // extern "C"
