"""Stage-by-stage MEHP24 sortFG on the engine with plaintext expectations
(diagnostics): prints the max error of every intermediate."""
import sys
import numpy as np
sys.path.insert(0, 'fhe-sorting_amd')
import fhesort as F

N = int(sys.argv[1]); logN = int(sys.argv[2]); depth = int(sys.argv[3]); dnum = int(sys.argv[4])
cfg = (3, 2, 2) if N <= 16 else (3, 3, 2) if N <= 128 else (3, 4, 2)
dg_i = (int(np.log2(N)) + 1) // 2
rots = F.mehp24_rotation_indices(N)
ext = len(sys.argv) > 5 and sys.argv[5] == 'ext'
ctx = F.Context(logN, depth + (1 if ext else 0), 40, 60, dnum, seed=N)
ctx.gen_rotation_keys(rots)
S = N * N
x = np.random.default_rng(N).permutation(N) / N
lg = int(np.log2(N))


def chk(name, ct, want):
    got = ctx.decrypt(ct)[:S]
    w = np.zeros(S); w[:len(want)] = want
    print(f'{name:16s} level {ct.level:3d} err {np.max(np.abs(got - w)):.3g}', flush=True)


def rot(c, k): return ctx.rotate(c, k)
def prot(v, k): return np.roll(v, -k)


c = ctx.encrypt_ext(x, S) if ext else ctx.encrypt(x, S)
v = np.zeros(S); v[:N] = x
chk('input', c, v)
# replicateRow
VR, pv = c, v.copy()
for i in range(lg):
    k = -(1 << (lg + i)); VR = ctx.add(VR, rot(VR, k)); pv = pv + prot(pv, k)
chk('VR', VR, pv)
pVR = pv
# transposeRow + mask col 0
T, pt = c, v.copy()
for i in range(1, lg + 1):
    k = -(N * (N - 1) // (1 << i)); T = ctx.add(T, rot(T, k)); pt = pt + prot(pt, k)
chk('transposeRow', T, pt)
mcol = (np.arange(S) % N == 0).astype(float)
T = ctx.mul_plain(T, ctx.encode(mcol, S, T.level)); pt = pt * mcol
chk('maskCol', T, pt)
VC, pc = T, pt
for i in range(lg):
    k = -(1 << i); VC = ctx.add(VC, rot(VC, k)); pc = pc + prot(pc, k)
chk('VC', VC, pc)
C = ctx.compare(VR, VC, *cfg)
pC = (pVR > pc).astype(float) + 0.5 * (pVR == pc)
chk('compare', C, pC)
R, pr = C, pC
for i in range(lg):
    k = -(1 << (lg + i)); R = ctx.add(R, rot(R, k)); pr = pr + prot(pr, k)
chk('R', R, pr)
sub = np.array([-(i // N) - 0.5 for i in range(S)])
X = ctx.add_plain(R, ctx.encode(sub, S, R.level)); px = pr + sub
chk('R+sub', X, px)
M = ctx.mehp24_indicator(X, float(N), dg_i, 2); pm = (np.abs(px) < 0.5).astype(float)
chk('indicator', M, pm)
P = ctx.mul(M, VR); pp = pm * pVR
chk('M*VR', P, pp)
