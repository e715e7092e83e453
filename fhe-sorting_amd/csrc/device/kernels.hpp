// Launch wrappers for the gfx950 kernels (kernels.hip).  All pointers are
// device pointers; every launch is asynchronous on `st`.
//
// Conventions:
//   * a "poly array" is [segments][limbs][n] u64, segment stride `seg`
//     elements; limb l of a Q-basis object uses prime index l.
//   * a "prime map" (pmap) gives the prime index of each limb of a batch when
//     the limbs are not Q primes 0..ell-1 (extended Q u P basis).
#pragma once
#include <string>
#include <utility>
#include <vector>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstddef>
#include <cstdint>

#include "modmath.hpp"

namespace fhe {
namespace dev {

struct NttTables {
    const ulonglong2 *fwd2;    // [nprimes][n] {psi^brev(k), Shoup companion}
    const ulonglong2 *inv2;    // [nprimes][n] {psi^-brev(k), Shoup companion}
    const u64 *ninv, *ninv_s;  // [nprimes]
    const Mod *mods;           // [nprimes]
    int logN;
    // fp64 butterflies (primes q < 2^41, ntt_fp_prime): twiddles as doubles
    // ([nprimes][n], entries of other primes unused) and {q, 1/q} per prime
    const double *fwdd = nullptr, *invd = nullptr;
    const double2 *qd = nullptr;
    const uint8_t *fp_host = nullptr;  // HOST array [nprimes]: 1 = the prime takes the FP launches
};
// q < 2^41: the NTT passes of this prime run on fp64 butterflies (ntt.hip)
bool ntt_fp_prime(u64 q);
// host copy of a device prime map (engine tables), so a launch over mapped
// limbs can be split by prime class; unknown maps launch on the integer path
void ntt_register_map(const int *dev, const int *host, size_t count);
void ntt_unregister_map(const int *dev);

// Optional per-launch clock used by the bench roofline: while one is installed,
// the NTT passes are bracketed by HIP events on the stream they launch on and
// reported with their algorithmic bytes.  Process-global; diagnostics only.
struct LaunchClock {
    virtual ~LaunchClock() = default;
    // events handed to hipExtLaunchKernelGGL (recorded at the kernel's own start /
    // end); returns the slot to book the launch under.  Thread-safe.
    virtual int events(hipEvent_t &start, hipEvent_t &stop) = 0;
    virtual void record(int slot, const char *kernel, double bytes) = 0;
};
LaunchClock *&launch_clock();
// caller tag appended to clocked NTT names ("k_ntt_fwd<8, 4, true>@modup"); per thread
const char *&launch_phase();
// algorithm phase of the calling thread ("compare", "indicator", ...; null:
// none), booked by the live clock beside each kernel (bench.py roofline.phases)
const char *&algo_phase();
// a stable, process-lifetime copy of s (thread-safe)
const char *intern_name(const std::string &s);
// "base<V0, V1, ...>", the instantiation as rocprofv3 spells it, so the clock
// books template instantiations apart (bench.py roofline.by_symbol); the plain
// base name when no clock is installed (no string work on the hot path)
template <int... V>
inline const char *inst_name(const char *base) {
    if (!launch_clock()) return base;
    std::string r(base);
    r += '<';
    const int v[] = {V...};
    for (size_t i = 0; i < sizeof...(V); ++i) r += (i ? ", " : "") + std::to_string(v[i]);
    r += '>';
    return intern_name(r);
}

// Fault diagnostics (environment FHE_FAULT_REPORT=1): every launch notes its
// kernel and grid in a process-global record, and install_fault_report() (the
// engine calls it once) adds a SIGSEGV / SIGBUS handler that prints the faulting
// PC and address, the thread, the launch count, the last launch and the
// /proc/self/maps lines holding the PC and the address, then chains to the
// previous handler (a profiler's, or the default).  Off: one predictable branch.
bool fault_report_enabled();
void note_launch_slow(const char *name, dim3 grid, dim3 block);
inline void note_launch(const char *name, dim3 grid, dim3 block) {
    if (fault_report_enabled()) note_launch_slow(name, grid, block);
}
void install_fault_report();

// Launch through hipExtLaunchKernelGGL; when a clock is installed the launch is
// timed by events recorded at the kernel's own start/end and booked under
// `name` with its algorithmic HBM bytes.
template <typename Kern, typename... Args>
inline void launch_clocked(const char *name, double bytes, Kern kernel, dim3 grid, dim3 block, hipStream_t st,
                           Args... args) {
    LaunchClock *clk = launch_clock();
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const int slot = clk ? clk->events(e0, e1) : -1;
    note_launch(name, grid, block);
    hipExtLaunchKernelGGL(kernel, grid, block, 0, st, e0, e1, 0, args...);
    if (clk) clk->record(slot, name, bytes);
}

// forward / inverse negacyclic NTT of `limbs` limbs x `segs` segments
void ntt_forward(u64 *data, int limbs, int segs, size_t seg, const int *pmap, const NttTables &T,
                 hipStream_t st);
// raw = true: the inverse omits its final n^-1 scaling and leaves values in
// [0, 2q) -- for the ModUp / ModDown conversions, whose first constant
// (q-hat^-1, P-hat^-1) carries n^-1 instead (host::LevelTables)
void ntt_inverse(u64 *data, int limbs, int segs, size_t seg, const int *pmap, const NttTables &T,
                 hipStream_t st, bool raw = false);
// Operands of the fused forward NTTs (ntt.hip): the column pass can load the
// centred lift of a coefficient-form limb; the row pass can finish a rescale
// or an HMult tail in its store instead of writing the transform back.
struct NttFuse {
    const u64 *last = nullptr;  // [segs][n] coefficient-form limb to lift (prime lastp)
    size_t seg_last = 0;
    int lastp = 0;
    u64 *out = nullptr;  // [segs][limbs][n] result
    size_t seg_out = 0;
    const u64 *x = nullptr;  // rescale: the input; HMult: the accumulators
    size_t seg_x = 0;
    const u64 *d = nullptr;  // HMult: d01
    size_t seg_d = 0;
    const u64 *c1 = nullptr, *c1s = nullptr;  // per limb: q_last^-1 (rescale) or (P q_last)^-1 (HMult)
    const u64 *c2 = nullptr, *c2s = nullptr;  // per limb: P mod q_i (HMult)
    const u64 *src = nullptr;  // inverse: out-of-place input of the first pass
    size_t seg_src = 0;
    int64_t scalar = 0;  // rescale: multiply the input by scalar * 2^scalar_sh first (0 = none)
    int scalar_sh = 0;
    bool raw = false;    // inverse: skip the n^-1 scaling of the last pass
    int lsegb = 0, segs = 0;  // shuffle row passes: log2 segments per block, segment count (set at launch)
    // limb runs of a launch split by prime class (set at launch): grid limb z is
    // limb zs0 + z for z < zn0, else zs1 + z - zn0
    int zs0 = 0, zn0 = 1 << 30, zs1 = 0;
    __host__ __device__ int limb_of(int z) const { return z < zn0 ? zs0 + z : zs1 + (z - zn0); }
};
// inverse NTT reading the input from `src` (segment z, limb l at src + z*seg_src + l*n), writing dst
void ntt_inverse_from(u64 *dst, const u64 *src, size_t seg_src, int limbs, int segs, size_t seg, const int *pmap,
                      const NttTables &T, hipStream_t st, bool raw = false);
// rescale of `segs` polys: out = (x - NTT(lift(last))) * c1 over `limbs` = ell-1 limbs (tmp: scratch)
void ntt_forward_rescale(u64 *tmp, int limbs, int segs, const NttFuse &F, const NttTables &T, hipStream_t st);
// HMult tail: out = (x + d * c2 - NTT(corr)) * c1 (corr is overwritten by the first pass only)
void ntt_forward_multail(u64 *corr, int limbs, int segs, const NttFuse &F, const NttTables &T, hipStream_t st);
// key-switch ModDown finish: out = (x - NTT(conv)) * c1 + d (d on even segments, member z / 2)
void ntt_forward_ksfinish(u64 *conv, int limbs, int segs, const NttFuse &F, const NttTables &T, hipStream_t st);
// one row pass (forward: the second pass; inverse: the first) alone, for kernel timing
void ntt_row_pass(u64 *data, int limbs, int segs, size_t seg, const int *pmap, const NttTables &T, hipStream_t st,
                  bool forward);
// forward NTT of `count` limbs scattered in each of `segs` segments: limb y
// of segment z sits at data + z * seg + smap[y] * n and belongs to prime
// pmap[y] (ModUp: every digit of every member at once)
void ntt_forward_mapped(u64 *data, int count, int segs, size_t seg, const int *smap, const int *pmap,
                        const NttTables &T, hipStream_t st);

// Segment strides (u64 units) of the output and the two inputs of an
// element-wise launch: segment z of out/a/b starts at z*o / z*a / z*b.
// A ciphertext batch of B members [B][2][limbs][n] is 2B segments of stride
// limbs*n; a plaintext operand is broadcast with stride 0.
struct Seg {
    size_t o, a, b;
};

// element-wise, Q basis (limb l <-> prime l); out may alias inputs
void ew_add(u64 *out, const u64 *a, const u64 *b, int limbs, int segs, Seg S, const Mod *mods, int logN,
            hipStream_t st);
void ew_sub(u64 *out, const u64 *a, const u64 *b, int limbs, int segs, Seg S, const Mod *mods, int logN,
            hipStream_t st);
void ew_neg(u64 *out, const u64 *a, int limbs, int segs, Seg S, const Mod *mods, int logN, hipStream_t st);
// out = a * (K 2^sh mod q_l)   (K: signed integer constant, reduced in-kernel)
void ew_mul_scalar(u64 *out, const u64 *a, int64_t K, int limbs, int segs, Seg S, const Mod *mods, int logN,
                   hipStream_t st, int sh = 0);
// out[l] += a[l] * W.w[l] for l < limbs (constants already reduced mod q_l)
constexpr int LIMB_CONSTS_MAX = 32;
struct LimbConsts {
    u64 w[LIMB_CONSTS_MAX];
};
void ew_add_scaled(u64 *out, const u64 *a, const LimbConsts &W, int limbs, Seg S, const Mod *mods, int logN,
                   hipStream_t st);
// out = a + (K 2^sh mod q_l)
void ew_add_scalar(u64 *out, const u64 *a, int64_t K, int limbs, int segs, Seg S, const Mod *mods, int logN,
                   hipStream_t st, int sh = 0);
// out[s] = a[s] * p[s]  (Barrett; S.b = 0 broadcasts one plaintext)
void ew_mul_plain(u64 *out, const u64 *a, const u64 *p, int limbs, int segs, Seg S, const Mod *mods, int logN,
                  hipStream_t st);
// per member m: d0 = a0 b0, d1 = a0 b1 + a1 b0 -> d01 [m][2][limbs][n]; d2 = a1 b1 -> d2 [m][limbs][n]
// (a member m at m * sa, b member at m * sb; sb = 0 broadcasts one ciphertext)
void ew_tensor(u64 *d01, u64 *d2, const u64 *a, const u64 *b, int limbs, int members, size_t sa, size_t sb,
               const Mod *mods, int logN, hipStream_t st, const u64 *a2 = nullptr, size_t sa2 = 0);
// ew_tensor with d_p += sum_i (K_i 2^sh_i mod q) x_i[2 member + p] (x_i segment
// stride xseg) for 1 <= m <= 4 summands; false (nothing launched) otherwise.
// Word-identical to ew_tensor then ew_linear_sum(d01, ..., accumulate).
bool ew_tensor_lin(u64 *d01, u64 *d2, const u64 *a, const u64 *b, int limbs, int members, size_t sa, size_t sb,
                   const u64 *const *xs, const int64_t *K, const uint8_t *sh, int m, size_t xseg, const Mod *mods,
                   int logN, hipStream_t st, const u64 *a2 = nullptr, size_t sa2 = 0);
// out [2][limbs][n] = sum_m in [m][2][limbs][n]
void ew_sum_members(u64 *out, const u64 *in, int members, int limbs, const Mod *mods, int logN, hipStream_t st);
// out (+)= sum_i (K_i 2^sh_i mod q_l) * x_i   (x_i: [segs][limbs][n], common segment stride; sh may be null)
void ew_linear_sum(u64 *out, const u64 *const *xs, const int64_t *K, int m, int limbs, int segs, size_t seg,
                   size_t xseg, const Mod *mods, int logN, hipStream_t st, bool accumulate = false,
                   const uint8_t *sh = nullptr);
// outs[g] = sum_i (K[g*m + i] 2^sh[g*m + i] mod q_l) * x_i for g < G <= 32 (the
// Paterson-Stockmeyer leaves of one level; x_i: [segs][limbs][n] with segment
// stride xseg[i]; outs: stride seg).  On the matrix cores (set_mfma_sums bit 1)
// one pass reads every input once for up to 32 outputs and 64 inputs; the
// constants then come from the device copies dK / dsh of K / sh ([G][m]).  The
// VALU kernel (mask bit clear, no device copies, or m > 64) takes passes of
// <= 10 outputs x 32 inputs from the host arrays.
constexpr int LEAF_G = 32, LEAF_M = 64;
void ew_linear_sum_multi(u64 *const *outs, int G, const u64 *const *xs, const size_t *xseg, const int64_t *K, int m,
                         int limbs, int segs, size_t seg, const Mod *mods, int logN, hipStream_t st,
                         const uint8_t *sh, const int64_t *dK, const uint8_t *dsh);
// true iff ew_linear_sum_multi runs on the matrix cores at this ring (it then reads dK / dsh)
bool linear_sums_on_mfma(int logN);
// out [members][2][limbs][n] = sum_i ct_i * pt_i  (ct_i member stride cmember, 0 = broadcast;
// c1 at + cpoly; pt_i [limbs][n] shared), lazy 128-bit accumulation
void ew_mul_plain_sum(u64 *out, const u64 *const *cts, const u64 *const *pts, int m, int limbs, int members,
                      size_t cmember, size_t cpoly, const Mod *mods, int logN, hipStream_t st);
// out[l][k] = in[l][perm[k]]
void ew_permute(u64 *out, const u64 *in, const uint32_t *perm, int limbs, int segs, Seg S, int logN,
                hipStream_t st);
// out[l][k] = coef[k] mod q_{pmap[l]} (signed 64-bit coefficients)
// out = a ([members][2][limbs][n]) with every member's c0 changed: mode 0 c0 + K 2^sh,
// 1 c0 + p, 2 c0 - p, 3 (p - c0, -c1); p [limbs][n] shared by the members
void ew_c0_op(u64 *out, const u64 *a, const u64 *p, int64_t K, int sh, int mode, int limbs, int members,
              const Mod *mods, int logN, hipStream_t st);
void ew_signed_to_rns(u64 *out, const int64_t *coef, int limbs, const int *pmap, const Mod *mods, int logN,
                      hipStream_t st, int members = 1, size_t out_stride = 0, size_t coef_stride = 0);

// ------------------------------------------------------------ device encode
// (encode.hip) special inverse FFT of B members of S slots in place (v [B][S]),
// then coef [B][n] = round(scale[b] * coefficients), word-identical to
// host::encode_coeffs_complex; ksi [2n + 1], rot [n / 2] are the host encoder's
// tables; *overflow |= 1 if a scaled coefficient reaches 9.2e18
void encode_ifft(double2 *v, int64_t *coef, int B, int S, int n, const double2 *ksi, const uint32_t *rot,
                 const double *scale, unsigned *overflow, hipStream_t st);
// the sort's masks as slot values: spec [B][3] = {kind, k, r}: kind 0
// mask_vector(S, N, k) rotated by r, kind 1 checking_vector(S, N, k)
void mask_slots(double2 *v, int B, int S, int N, const int *spec, hipStream_t st);

// ---------------------------------------------------------------- keyswitch
// ext[m][j][t][k] for every member m, digit j and target t not in digit j
// (coefficient in, unscaled: the q-hat^-1 constants carry n^-1; NTT NOT applied);
// coef member stride coef_stride, ext member stride ext_stride
// mask of the sums-of-products kernels that run on the i8 matrix cores (1 PS
// linear sums, 2 ModUp, 4 ModDown+rescale); mask < 0 only reads it.  Returns
// the previous mask.
int set_mfma_sums(int mask);
void modup_convert(u64 *ext, const u64 *coef, int ell, int K, int alpha, int digits, int members,
                   size_t coef_stride, size_t ext_stride, const int *pmap_ext,
                   const u64 *tabs /* packed, see engine */, const size_t *tab_off, const Mod *mods, int logN,
                   hipStream_t st,
                   // given (host::LevelTables modup_fp*, fpmid >= 0): the fp64 kernel
                   const double *fptab = nullptr, const size_t *fp_off = nullptr, int fpmid = -1);
// acc0/acc1 [W][n] per member: sum_j ext_j * key_j   (own-digit limbs read from dntt)
struct KsStrides {
    size_t acc = 0, ext = 0, d = 0;  // member strides of acc [2][W][n], ext, dntt
    // target runs (ks_inner with a target subset): grid target z is target
    // zs0 + z for z < zn0, else zs1 + z - zn0 (default: every target)
    int zs0 = 0, zn0 = 1 << 30, zs1 = 0;
    __host__ __device__ int target_of(int z) const { return z < zn0 ? zs0 + z : zs1 + (z - zn0); }
};
// optional HMult fold: limb ell-1 of the accumulators starts at w * d[k], w * d[seg + k]
struct KsFold {
    const u64 *d = nullptr;  // d0[ell-1] (NTT) of member 0; d1[ell-1] at d + seg
    size_t seg = 0, member = 0;
    u64 w = 0, ws = 0;       // P mod q_{ell-1} and its Shoup companion
};
// (tcount >= 0: only tcount targets, through str's target runs)
void ks_inner(u64 *acc, const u64 *ext, const u64 *dntt, const u64 *key, int ell, int K, int nq, int nall,
              int alpha, int digits, const uint32_t *perm, const int *pmap_ext, const Mod *mods, int logN,
              hipStream_t st, int members, KsStrides str, KsFold fold = KsFold(), int tcount = -1);
// ModUp's forward NTT split in two for the relinearisation (ntt.hip): the
// column pass alone over the mapped limbs (as ntt_forward_mapped), then
// ntt_row_ks -- the row pass of every digit's target limb fused with the
// key-switch inner product of ks_inner (no permutation): acc[m][0/1][t] =
// sum_j NTT_row(ext_j)[t] * key_j (own digit: dntt) (+ the fold on t = ell-1),
// so ext never returns to HBM in NTT form.  Same words as ntt_forward_mapped +
// ks_inner.  Members in blocks of 16 (one transform each, one row per block).
void ntt_forward_mapped_cols(u64 *data, int count, int segs, size_t seg, const int *smap, const int *pmap,
                             const NttTables &T, hipStream_t st);
// fp_only: the targets of integer-class primes are left to the caller (their
// row pass: ntt_forward_mapped_rows; their inner product: ks_inner over the
// integer runs, ntt_class_runs) -- measured faster there
void ntt_row_ks(u64 *acc, const u64 *ext, const u64 *dntt, const u64 *key, int ell, int K, int nall, int alpha,
                int digits, const int *pmap_ext, int members, KsStrides str, KsFold fold, const NttTables &T,
                hipStream_t st, bool fp_only = false);
// the row pass alone over mapped limbs (second half of ntt_forward_mapped)
void ntt_forward_mapped_rows(u64 *data, int count, int segs, size_t seg, const int *smap, const int *pmap,
                             const NttTables &T, hipStream_t st);
// the limbs z < count of a prime map (pmap, registered; null = identity) whose
// class is FP (fp = true) or integer, as runs (start, length)
std::vector<std::pair<int, int>> ntt_class_runs(const int *pmap, int count, bool fp, const NttTables &T);
// several key switches in one launch (hoisted rotations by different
// amounts, or one rotation per member of a batch): member m < count uses key
// keys[m] and reads ext through perm[m]; strides in `str` (0 = shared input)
constexpr int KS_MAXKEYS = 16;
struct KsKeys {
    const u64 *key[KS_MAXKEYS];
    const uint32_t *perm[KS_MAXKEYS];
};
// acc [2][ell+K][n] (+)= sum over the count members of their key products
// (member m: ext at m * str.ext, own digit at m * str.d, keys.key/perm[m])
void ks_inner_multikey_sum(u64 *acc, const u64 *ext, const u64 *dntt, const KsKeys &keys, int count, bool accumulate,
                           int ell, int K, int nall, int alpha, int digits, const int *pmap_ext, const Mod *mods,
                           int logN, hipStream_t st, KsStrides str);
// Baby steps of a double-hoisted linear transform (bootstrap CoeffsToSlots /
// SlotsToCoeffs): out [2][W][n] (+)= sum_b pt_b * baby_b over Q u P, where baby b
// is (P sigma_b(c0), 0) + <sigma_b(ext), key_b> (key null: (P c0, P c1)), never
// brought down to Q.  c: the ciphertext [2][ell][n]; ext its c1's ModUp.
constexpr int LT_MAXB = 16;
struct LtArgs {
    const u64 *key[LT_MAXB];
    const uint32_t *perm[LT_MAXB];
    const u64 *pt[LT_MAXB];  // extended plaintexts [W][n]
    int nb;
};
void lt_inner(u64 *out, const u64 *ext, const u64 *c, const LtArgs &A, bool accumulate, int ell, int K, int nall,
              int alpha, int digits, const int *pmap_ext, const u64 *pmodq, const u64 *pmodq_s, const Mod *mods,
              int logN, hipStream_t st);
// out [limbs][n] (+)= sum_m in_m o keys.perm[m] (member m at m * in_stride)
void ew_permute_sum(u64 *out, const u64 *in, const KsKeys &keys, int limbs, int count, bool accumulate, size_t in_stride,
                    const Mod *mods, int logN, hipStream_t st);
void ks_inner_multikey(u64 *acc, const u64 *ext, const u64 *dntt, const KsKeys &keys, int count, int ell, int K,
                       int nall, int alpha, int digits, const int *pmap_ext, const Mod *mods, int logN,
                       hipStream_t st, KsStrides str);
// out[m][l][k] = in[m][l][perms[m][k]] for m < count (in stride S.a, 0 = shared; out stride S.o)
void ew_permute_multi(u64 *out, const u64 *in, const KsKeys &keys, int limbs, int count, Seg S, int logN,
                      hipStream_t st);
// fused ModDown + rescale of an HMult (see kernels.hip): corr [segs][ell-1][n]
// from acc [segs][W][n] whose limbs ell-1 .. W-1 are in coefficient form,
// unscaled (ntt_inverse raw: n x); ninv [nall]: n^-1 mod each prime
void moddown_rescale_convert(u64 *corr, const u64 *acc, int ell, int K, int nq, size_t seg_acc, size_t seg_corr,
                             int segs, const u64 *phinv, const u64 *phinv_s, const u64 *phat, const u64 *pinv,
                             const u64 *pinv_s, const u64 *pmod, const double *pinvd, const u64 *ninv,
                             const u64 *ninv_s, const Mod *mods, int logN, hipStream_t st,
                             const u64 *pmod_s = nullptr,  // given: the MFMA kernel
                             // given (host::LevelTables mdfp_*, fpmid >= 0): the fp64 kernel
                             const double *fpc = nullptr, const double *fpq = nullptr, int fpmid = -1);
// conv[s][i][k] = (sum_k' y_k' phat[i][k'] - v P) mod q_i for i < ell, y_k' =
// pc[s][k'] * phinv_k' (pc: unscaled inverse NTT, phinv carries n^-1),
// v = round(sum_k' y_k' pinvd_k'): the centred Conv_{P->q_i}
void moddown_convert(u64 *conv, const u64 *pc, int ell, int K, int nq, size_t seg_in, size_t seg_out, int segs,
                     const u64 *phinv, const u64 *phinv_s, const u64 *phat, const u64 *pmod, const double *pinvd,
                     const Mod *mods, int logN, hipStream_t st);
// out[s][i] = (acc[s][i] - conv[s][i]) * Pinv_i (+ add[s/2][i] on even s, i.e. c0 of each member)
void moddown_finish(u64 *out, const u64 *acc, const u64 *conv, const u64 *add, int ell, int segs, size_t seg_out,
                    size_t seg_acc, size_t seg_add, const u64 *pinv, const u64 *pinv_s, const Mod *mods, int logN,
                    hipStream_t st);

// ModRaise: out[z][l][k] = centred lift of in[z][k] (a residue mod prime `src`,
// coefficient form, < 2 q_src) reduced mod q_l for l < limbs
void ew_lift_centered(u64 *out, const u64 *in, int src, int limbs, int segs, size_t seg_in, size_t seg_out,
                      const Mod *mods, int logN, hipStream_t st);
// u64 all-reduce fix-up: x mod q_l per limb
void ew_reduce(u64 *x, int limbs, int segs, size_t seg, const Mod *mods, int logN, hipStream_t st);
// k_region_begin / k_region_end on `st` (profiling region delimiters)
void region_marker(bool begin, hipStream_t st);

}  // namespace dev
}  // namespace fhe
