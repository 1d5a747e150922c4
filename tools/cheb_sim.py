"""Host model of the CG -> Chebyshev hybrid for the per-column solves (design aid, CPU only).

Builds Luu of the bench shapes with the oracle and counts matrix passes of
  * Jacobi PCG (Chronopoulos-Gear, what cg_ell_kernel MODE 1 runs), rtol 1e-6, and
  * k0 PCG iterations, Ritz bounds of the Lanczos matrix they define, then preconditioned
    Chebyshev for a pass count computed from those bounds, one residual check, PCG after.
    python tools/cheb_sim.py [ns|fullysup] [k0] [lo_margin] [hi_margin] [safety]
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402
from oracle import gll_oracle as O  # noqa: E402


def pcg(A, Dinv, b, rtol, maxit=1000, x=None, r=None):
    x = np.zeros_like(b) if x is None else x.copy()
    r = b.copy() if r is None else r.copy()
    bb = b @ b
    z = Dinv * r
    p = z.copy()
    rz = r @ z
    al, be = [], []
    it = 0
    passes = 0
    while r @ r > rtol * rtol * bb and it < maxit:
        s = A @ p
        passes += 1
        a = rz / (p @ s)
        x += a * p
        r -= a * s
        z = Dinv * r
        rz2 = r @ z
        b_ = rz2 / rz
        al.append(a)
        be.append(b_)
        p = z + b_ * p
        rz = rz2
        it += 1
    return x, r, it, passes, al, be


def ritz(al, be):
    k = len(al)
    T = np.zeros((k, k))
    for j in range(k):
        T[j, j] = 1 / al[j] + (be[j - 1] / al[j - 1] if j else 0)
        if j + 1 < k:
            T[j, j + 1] = T[j + 1, j] = np.sqrt(be[j]) / al[j]
    ev = np.linalg.eigvalsh(T)
    return ev[0], ev[-1]


def hybrid(A, Dinv, b, rtol, k0, lom, him, safety):
    x, r, it, passes, al, be = pcg(A, Dinv, b, rtol, maxit=k0)
    if r @ r <= rtol * rtol * (b @ b):
        return passes, 0, 0
    lmin, lmax = ritz(al, be)
    lo = lmin * lom
    # lambda_max(D^-1 A) <= 2 - lambda_min(D^-1 A): D^-1 A = I - D^-1 N with D^-1 N >= 0, whose
    # most negative eigenvalue is >= -rho(D^-1 N) = lambda_min - 1 (Perron); valid when lo is
    hi = max(2.0 - lo, lmax * him) if him > 0 else 2.0 - lo
    th, de = (hi + lo) / 2, (hi - lo) / 2
    sg = th / de
    ratio = np.sqrt((r @ r) / (rtol * rtol * (b @ b))) * safety
    N = int(np.ceil(np.arccosh(ratio) / np.arccosh(sg)))
    rho = 1 / sg
    d = Dinv * r / th
    for _ in range(N):
        w = A @ d
        passes += 1
        x += d
        r -= w
        rn = 1 / (2 * sg - rho)
        d = rn * rho * d + (2 * rn / de) * (Dinv * r)
        rho = rn
    extra = 0
    if r @ r > rtol * rtol * (b @ b):
        x, r, it2, p2, _, _ = pcg(A, Dinv, b, rtol, x=x, r=r)
        passes += p2
        extra = p2
    return passes, N, extra


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "ns"
    k0 = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    lom = float(sys.argv[3]) if len(sys.argv) > 3 else 0.9
    him = float(sys.argv[4]) if len(sys.argv) > 4 else 1.05
    safety = float(sys.argv[5]) if len(sys.argv) > 5 else 2.0
    c = CONFIGS[cfg]
    tot = [0, 0, 0]
    for seed in range(4):
        X, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=seed)
        Y = one_hot(lab[: c["base"]])
        U, st = O.forward(X, Y, 0.07, 1.0, c["k"])
        A = st.Luu.tocsr()
        Dinv = 1 / A.diagonal()
        rhs = A @ U
        g = seeded_gbar(c["batch"], 10, 1234 + seed)
        for name, B in (("fwd", rhs), ("bwd", g)):
            cg_p, hy_p, ns, ex = [], [], [], []
            for col in range(B.shape[1]):
                b = B[:, col]
                cg_p.append(pcg(A, Dinv, b, 1e-6)[3])
                p, N, e = hybrid(A, Dinv, b, 1e-6, k0, lom, him, safety)
                hy_p.append(p)
                ns.append(N)
                ex.append(e)
            tot[0] += max(cg_p)
            tot[1] += max(hy_p)
            tot[2] += max(ex) > 0
            print(f"seed {seed} {name}: CG passes max {max(cg_p)}  hybrid max {max(hy_p)} "
                  f"(cheb {min(ns)}-{max(ns)}, fallback cols {sum(e > 0 for e in ex)})")
    print(f"total CG {tot[0]}  hybrid {tot[1]}  solves with fallback {tot[2]}")


if __name__ == "__main__":
    main()
