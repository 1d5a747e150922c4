"""Bank-aware entry order of the balanced CG's virtual rows, modelled on the kernel's own dealing
(diagnostic, CPU).   python tools/bank_order_sim.py [fullysup|ns] [B]

cg_vr_kernel (solve.hip) deals virtual rows thread-major: thread t owns rows t, t+512, t+1024, its
virtual rows are numbered by an exclusive scan over the threads, and virtual row v sits in
register j = v / 512 of thread v % 512.  One gather instruction (j, k) of wave w reads entry k of
the 64 virtual rows v = j*512 + 64w + lane.  Cost per instruction (MI355X_MICROARCH.md, LDS):
ds_read_b32, two lane groups of 32, bank = (addr/4) mod 32, each extra distinct address on a bank
adds one cycle; equal addresses broadcast.  Compared: the stored order (ascending column), and the
ballot sweep vr_order_kernel runs (per slot, banks 0..31 in turn, the lowest free lane of each half
holding an entry on that bank takes it; lanes left over take their first remaining entry; padding
copies an address already read in its half).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphlearninglayer_amd.synth import CONFIGS, synth  # noqa: E402

NT, KVS = 512, 8


def urows(cfg, seed):
    c = CONFIGS[cfg]
    X, _ = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=seed)
    Xd = X.astype(np.float64)
    sq = (Xd * Xd).sum(1)
    D = sq[:, None] + sq[None, :] - 2 * Xd @ Xd.T
    np.fill_diagonal(D, -1.0)
    ind = np.argsort(D, axis=1, kind="stable")[:, : c["k"]]
    n, base = X.shape[0], c["base"]
    nb = [set() for _ in range(n)]
    for i in range(n):
        for j in ind[i, 1:]:
            nb[i].add(int(j))
            nb[int(j)].add(i)
    return [sorted(cc - base for cc in nb[base + u] if cc >= base) for u in range(c["batch"])]


def deal(rows, m):
    R = (m + NT - 1) // NT
    vr = []   # in scan order
    for t in range(NT):
        for q in range(R):
            u = t + NT * q
            if u >= m:
                continue
            L = rows[u]
            for j in range(0, len(L), KVS):
                vr.append(L[j:j + KVS])
    return vr


def cost(cols):
    t = 0
    for g0 in (0, 32):
        banks = {}
        for cc in cols[g0:g0 + 32]:
            if cc is None:
                continue
            banks.setdefault(cc % 32, set()).add(cc)
        t += max([len(s) for s in banks.values()] + [1])
    return t


def ballot_order(lanes, nslot):
    rem = [list(x) for x in lanes]
    out = [[None] * nslot for _ in lanes]
    for k in range(nslot):
        took = [False] * 64
        for b in range(32):
            for g0 in (0, 32):
                for l in range(g0, g0 + 32):
                    if took[l]:
                        continue
                    hit = [i for i, cc in enumerate(rem[l]) if cc % 32 == b]
                    if hit:
                        out[l][k] = rem[l].pop(hit[0])
                        took[l] = True
                        break
        for l in range(64):   # left over: first remaining entry
            if not took[l] and rem[l]:
                out[l][k] = rem[l].pop(0)
                took[l] = True
        # padding broadcasts an address already read in its half
        for g0 in (0, 32):
            seen = [out[l][k] for l in range(g0, g0 + 32) if out[l][k] is not None]
            for l in range(g0, g0 + 32):
                if out[l][k] is None and seen:
                    out[l][k] = seen[0]
    return out


def simulate(vr, greedy):
    V = len(vr)
    RV = (V + NT - 1) // NT
    tot = n = 0
    for j in range(RV):
        for w in range(NT // 64):
            lanes = [list(vr[v]) if v < V else [] for v in (j * NT + w * 64 + l for l in range(64))]
            vmax = max(len(x) for x in lanes)
            if vmax == 0:
                continue
            nslot = 4 if vmax <= 4 else 8
            if greedy:
                ordl = ballot_order(lanes, nslot)
            else:
                ordl = [x + [0] * (nslot - len(x)) for x in lanes]   # padding reads offset 0
            for k in range(nslot):
                tot += cost([o[k] for o in ordl])
                n += 1
    return tot, n


if __name__ == "__main__":
    cfg = sys.argv[1] if len(sys.argv) > 1 else "fullysup"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    m = CONFIGS[cfg]["batch"]
    for seed in range(B):
        vr = deal(urows(cfg, seed), m)
        for g in (False, True):
            t, n = simulate(vr, g)
            print(f"{cfg} seed {seed} V {len(vr)} {'ballot' if g else 'stored'}: "
                  f"{t} LDS cycles over {n} gather instructions, {t / n:.2f} per instruction")
