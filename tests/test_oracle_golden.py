"""The oracle restatements against fixtures produced by the reference GLL.py itself.

This pins the oracle before it is trusted as the checker of the HIP path (CPU only)."""
import os

import numpy as np
import pytest
import torch

from oracle import gll_oracle as O
from oracle import gll_port as PT
from tests.golden_io import Case, nan_aware, names

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CASES = names()


def test_fixtures_present():
    assert len(CASES) >= 18
    # round 6: the reference itself pins C != 10, wide k and eps = 0
    for want in ("ns_eps1p0_tau0p07_f32_C3", "ns_epsauto_tau0p0_i64_C17",
                 "ns_eps1p0_tau0p07_f32_k64", "ns_epsauto_tau0p07_f32_k100",
                 "plumbing_eps0p0_tau0p07_f32"):
        assert want in CASES


def test_eps_zero_fixture_is_the_reference_nan_gradient():
    """GLL.py:233-234 with eps = 0: W = exp(-inf) = 0 -> U = 0; V = -8 * 0 / 0 = NaN -> the
    whole feature gradient is NaN.  The fixture records exactly that."""
    c = Case("plumbing_eps0p0_tau0p07_f32")
    assert np.all(c.U == 0)
    assert np.isnan(c.z["grad"]).all()


@pytest.mark.parametrize("name", CASES)
def test_inputs_regenerate_bit_exact(name):
    assert Case(name).x_ok, "synthetic X differs from the fixture's sha256"


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name):
    c = Case(name)
    ind, _ = O.knn_exact(c.X, c.k)
    assert np.array_equal(ind, c.knn)
    with np.errstate(divide="ignore", invalid="ignore"):   # eps = 0 divides by zero
        U, st = O.forward(c.X, c.Y, c.tau, c.eps, c.k)
        grad = O.backward(st, c.gbar)
    assert nan_aware(O.rel_err)(U, c.U) < 1e-12
    # the reference casts the edge values to fp32 before G @ X (GLL.py:154): fp32 floor
    assert c.grad_error(grad, O.rel_err) < 2e-6


@pytest.mark.parametrize("name", [n for n in CASES if n.startswith(("plumbing", "ns"))])
def test_port_matches_reference(name):
    c = Case(name)
    Xt = torch.from_numpy(c.X).requires_grad_(True)
    with np.errstate(divide="ignore", invalid="ignore"):
        U, saved = PT.forward(Xt, torch.from_numpy(c.Y), c.tau, c.eps, c.k)
        g = PT.backward(saved, torch.from_numpy(c.gbar)).numpy()
    assert nan_aware(O.rel_err)(U.numpy(), c.U) < 1e-12
    assert c.grad_error(g, O.rel_err) < 2e-6


def test_oracle_with_given_knn_equals_search():
    c = Case(CASES[0])
    U1, _ = O.forward(c.X, c.Y, c.tau, c.eps, c.k)
    U2, _ = O.forward(c.X, c.Y, c.tau, c.eps, c.k, knn=(c.knn, None))
    assert O.rel_err(U2, U1) < 1e-12


def test_fd_gradient_plumbing():
    """Backward is the exact gradient of forward for a frozen graph."""
    c = Case("plumbing_epsauto_tau0p07_f32")
    X = c.X.astype(np.float64)
    U, st = O.forward(X, c.Y, c.tau, c.eps, c.k)
    g = O.backward(st, c.gbar)
    rng = np.random.default_rng(0)
    D = rng.standard_normal(X.shape)
    h = 1e-6
    Up, _ = O.forward(X + h * D, c.Y, c.tau, c.eps, c.k, knn=(c.knn, None))
    Um, _ = O.forward(X - h * D, c.Y, c.tau, c.eps, c.k, knn=(c.knn, None))
    fd = np.sum((Up - Um) * c.gbar) / (2 * h)
    an = np.sum(g * D)
    assert abs(fd - an) / abs(an) < 1e-6


@pytest.mark.parametrize("fname", ["laplace_small", "laplace_k64"])
def test_oracle_laplace_matches_reference_fixture(fname):
    """utils.laplace: the closed-form oracle vs the reference pipeline
    (reference knn_sym_dist + stable_conjgrad driven by utils.py:570-593's glue)."""
    import json
    from graphlearninglayer_amd.synth import sha256, synth
    z = np.load(os.path.join(GOLDEN, fname + ".npz"))
    p = json.loads(str(z["meta"]))
    X, labels = synth(p["labeled"], p["unlabeled"], p["d"], C=10, r=p["r"], seed=p["seed"])
    assert sha256(X) == p["x_sha256"]
    np.testing.assert_array_equal(labels, z["labels"])
    U = O.laplace(X, labels[: p["labeled"]], knn_num=p["knn_num"], epsilon=p["epsilon"],
                  tau=p["tau"])
    assert O.rel_err(U, z["U"]) <= 1e-9
