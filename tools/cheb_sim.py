"""Host model of Chebyshev variants of the per-column solves (design aid, CPU only; round 6).

The per-column CG (cg_ell_kernel) is bound by each workgroup's iteration chain: a publish
barrier, the LDS gathers, then a fused three-value reduction and the step sizes
(profiles/r05e_trace_sell_b64.txt, B = 64 NS, iteration 3 in shader cycles: update+store ~190,
publish barrier ~160, spmv+dots ~1,800, reduce ~480, alpha/beta+p,s ~600 -> ~3,300).
Chebyshev iteration needs no reduction -- only the spectrum's bounds -- so its iteration is
priced here at ~2,050 cycles (no reduce, no step sizes) plus ~500 per residual check.  This
script counts iterations and prices three schemes against Jacobi PCG (what MODE 1 runs) on
Luu of the bench shapes (oracle graphs, 4 seeds, 10 columns, rtol 1e-6, the slowest column
of each solve):
  hybrid   k0 PCG iterations, Ritz bounds of their Lanczos matrix, then Chebyshev with a
           residual check every ck iterations (the forward: nothing is known in advance);
  adjoint  Chebyshev from x = 0 with the bounds of the FORWARD solve's Lanczos matrices
           (min / max over its columns, with margins), checks every ck iterations;
  and the same adjoint scheme under the Neumann-1 preconditioner (MODE 3, single graphs).
    python tools/cheb_sim.py [ns|fullysup]
Result (NS, round 6): hybrid 1.00-1.41x the PCG cost (never cheaper); adjoint 0.76-0.82x
with Jacobi (12-15 iterations against 11-12) but 8-9 iterations against 6-7 with Neumann-1
(no gain).  So only the batched adjoint launch could gain (~2.5 us of a 660 us B = 64 call):
not built.
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from graphlearninglayer_amd.synth import CONFIGS, one_hot, seeded_gbar, synth  # noqa: E402
from oracle import gll_oracle as O  # noqa: E402

C_CG, C_CHEB, C_CHECK, C_EIG = 3300, 2050, 500, 300   # shader cycles (see the docstring)


def pcg(A, Minv, b, rtol, maxit=1000, x=None, r=None):
    x = np.zeros_like(b) if x is None else x.copy()
    r = b.copy() if r is None else r.copy()
    bb = b @ b
    z = Minv(r)
    p = z.copy()
    rz = r @ z
    al, be = [], []
    it = 0
    while r @ r > rtol * rtol * bb and it < maxit:
        s = A @ p
        a = rz / (p @ s)
        x += a * p
        r -= a * s
        z = Minv(r)
        rz2 = r @ z
        al.append(a)
        be.append(rz2 / rz)
        p = z + (rz2 / rz) * p
        rz = rz2
        it += 1
    return x, r, it, al, be


def ritz(al, be):
    """Extreme eigenvalues of the Lanczos matrix PCG's coefficients define."""
    k = len(al)
    T = np.zeros((k, k))
    for j in range(k):
        T[j, j] = 1 / al[j] + (be[j - 1] / al[j - 1] if j else 0)
        if j + 1 < k:
            T[j, j + 1] = T[j + 1, j] = np.sqrt(be[j]) / al[j]
    ev = np.linalg.eigvalsh(T)
    return ev[0], ev[-1]


def chebyshev(A, Minv, b, rtol, lo, hi, ck, x=None, r=None, cap=300):
    """Preconditioned Chebyshev iteration on [lo, hi]; (iterations, checks) to rtol."""
    x = np.zeros_like(b) if x is None else x
    r = b.copy() if r is None else r
    tol2 = rtol * rtol * (b @ b)
    th, de = (hi + lo) / 2, (hi - lo) / 2
    sg = th / de
    rho = 1 / sg
    d = Minv(r) / th
    n = checks = 0
    while n < cap:
        w = A @ d
        n += 1
        x += d
        r -= w
        rn = 1 / (2 * sg - rho)
        d = rn * rho * d + (2 * rn / de) * Minv(r)
        rho = rn
        if n % ck == 0:
            checks += 1
            if r @ r <= tol2:
                break
    return n, checks


def graphs(cfg, seeds=4):
    c = CONFIGS[cfg]
    for seed in range(seeds):
        X, lab = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=seed)
        Y = one_hot(lab[: c["base"]])
        U, st = O.forward(X, Y, 0.07, 1.0, c["k"])
        A = st.Luu.tocsr()
        Di = 1 / A.diagonal()
        N = A.copy()
        N.setdiag(0)
        N = -N
        yield seed, A, Di, N, A @ U, seeded_gbar(c["batch"], 10, 1234 + seed)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "ns"
    print("== forward hybrid (k0 PCG, Ritz bounds, Chebyshev with checks), Jacobi")
    for k0, lom, ck, him in [(3, 0.9, 3, 1.1), (4, 0.9, 3, 1.1), (5, 0.95, 3, 1.05)]:
        tot_h = tot_cg = 0
        for seed, A, Di, N, rhs, g in graphs(cfg):
            Minv = lambda r: Di * r   # noqa: E731
            for B in (rhs, g):
                hs, cs = [], []
                for col in range(B.shape[1]):
                    b = B[:, col]
                    _, _, itc, _, _ = pcg(A, Minv, b, 1e-6)
                    cs.append(itc * C_CG)
                    x, r, it, al, be = pcg(A, Minv, b, 1e-6, maxit=k0)
                    if r @ r <= 1e-12 * (b @ b):
                        hs.append(it * C_CG)
                        continue
                    lmin, lmax = ritz(al, be)
                    n, chk = chebyshev(A, Minv, b, 1e-6, lmin * lom, lmax * him, ck, x, r)
                    hs.append(it * C_CG + C_EIG + n * C_CHEB + chk * C_CHECK)
                tot_h += max(hs)
                tot_cg += max(cs)
        print(f"  k0 {k0} lo x{lom} hi x{him} check/{ck}: cost vs PCG {tot_h / tot_cg:.3f}")
    for name in ("jacobi", "neumann-1"):
        print(f"== adjoint Chebyshev with the forward's Ritz bounds, {name}")
        for lom, him, ck in [(0.95, 1.05, 3), (0.97, 1.02, 2)]:
            its_cg, its_ch, cost_r = [], [], []
            for seed, A, Di, N, rhs, g in graphs(cfg):
                if name == "jacobi":
                    Minv = lambda r: Di * r   # noqa: E731
                else:
                    Minv = lambda r: Di * r + Di * (N @ (Di * r))   # noqa: E731
                los, his = [], []
                for col in range(rhs.shape[1]):
                    *_, al, be = pcg(A, Minv, rhs[:, col], 1e-6)
                    lmin, lmax = ritz(al, be)
                    los.append(lmin)
                    his.append(lmax)
                lo, hi = min(los) * lom, max(his) * him
                cg = max(pcg(A, Minv, g[:, col], 1e-6)[2] for col in range(g.shape[1]))
                ch = [chebyshev(A, Minv, g[:, col], 1e-6, lo, hi, ck) for col in range(g.shape[1])]
                n = max(c[0] for c in ch)
                chk = max(c[1] for c in ch)
                its_cg.append(cg)
                its_ch.append(n)
                cost_r.append((n * C_CHEB + chk * C_CHECK) / (cg * C_CG))
            print(f"  lo x{lom} hi x{him} check/{ck}: PCG iterations {its_cg}, Chebyshev "
                  f"{its_ch}, cost vs PCG {np.mean(cost_r):.3f}"
                  + ("  (Neumann iterations cost ~0.74 of a PCG one: two gathers each)"
                     if name != "jacobi" else ""))


if __name__ == "__main__":
    main()
