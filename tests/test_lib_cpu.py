"""CPU-side checks of the C ABI library and the host logic (no GPU calls)."""
import ctypes as ct
import os
import re

import numpy as np
import pytest
import torch

from graphlearninglayer_amd import _lib
from graphlearninglayer_amd import GLL as G
from graphlearninglayer_amd.synth import CONFIGS, one_hot, sha256, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "gll.h")).read()
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(gll_\w+)\s*\(", src, flags=re.M)))


def test_library_loads_and_exports_every_header_symbol():
    lib = _lib.lib()
    declared = header_functions()
    assert len(declared) >= 10
    assert set(declared) == set(_lib.EXPORTS)
    for name in declared:
        assert hasattr(lib, name), name


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_problem_struct_matches_header():
    src = open(os.path.join(ROOT, "include", "gll.h")).read()
    body = src[src.index("typedef struct gll_problem"):src.index("} gll_problem;")]
    fields = re.findall(r"(int32_t\*?|float)\s+(\w+);", body)
    assert [f for _, f in fields] == [f for f, _ in _lib.Problem._fields_]
    assert ct.sizeof(_lib.Problem) == 4 * (len(fields) - 1) + 8   # 10 words + one pointer


def test_view_struct_matches_header():
    src = open(os.path.join(ROOT, "include", "gll.h")).read()
    body = src[src.index("typedef struct gll_view"):src.index("} gll_view;")]
    names = re.findall(r"\*\s*(\w+);", body)
    assert names == [f for f, _ in _lib.View._fields_]


def test_workspace_bytes_and_validation():
    lib = _lib.lib()
    p = G.make_problem(1000, 512, 500, 10, 10, 0.07, 1.0)
    nb = lib.gll_workspace_bytes(ct.byref(p))
    # dominated by the n x n squared-distance planes (two at NS: the split-phase Gram) and the
    # n x d hi/lo bf16 planes of the pre-split Gram (knn.hip gram_split_kernel)
    assert 2 * 1000 * 1000 * 4 < nb < 2 * 1000 * 1000 * 4 + 1000 * 512 * 4 + 4 * 2**20
    bad = G.make_problem(1000, 512, 500, 10, 10, 0.07, 1.0)
    bad.K = 1
    assert lib.gll_workspace_bytes(ct.byref(bad)) == 0
    wide_k = G.make_problem(1000, 512, 500, 10, 100, 0.07, 1.0)
    assert lib.gll_workspace_bytes(ct.byref(wide_k)) > nb   # the wide select (K - 1 <= 128)
    huge_k = G.make_problem(1000, 512, 500, 10, 257, 0.07, 1.0)
    assert lib.gll_workspace_bytes(ct.byref(huge_k)) > 0    # K - 1 <= 256 (kMaxKm1Huge)
    big_k = G.make_problem(1000, 512, 500, 10, 258, 0.07, 1.0)
    assert lib.gll_workspace_bytes(ct.byref(big_k)) == 0   # K - 1 > 256 unsupported
    assert lib.gll_strerror(-2).decode().startswith("unsupported")


@pytest.mark.parametrize("shape", [
    # (n, d, base, C, K, cap in MB): NS, FullySup, stress, k = 129, the 60k utils.laplace graph
    (1000, 512, 500, 10, 10, 14), (1500, 128, 250, 10, 25, 22), (8192, 1024, 4096, 10, 30, 370),
    (2000, 64, 500, 10, 129, 84), (60250, 128, 250, 10, 50, 15500)])
def test_workspace_bytes_bounded_per_row(shape):
    """Advisor (round 5): the row slot width must not grow with the reverse-list capacity.  Past
    the n x n distances (and the hi/lo Gram planes) a row costs the six slot arrays (24 B a slot,
    Wcap = 5(K-1)+8 slots plus the 2(K-1) bump share), the reverse list (8 B x RCAP = 8(K-1)+8),
    the overflow triples, the kNN lists and O(C) vectors -- nothing more."""
    n, d, base, C, K, cap_mb = shape
    lib = _lib.lib()
    nb = lib.gll_workspace_bytes(ct.byref(G.make_problem(n, d, base, C, K, 0.07, 1.0)))
    assert 0 < nb <= cap_mb * 1e6
    ks = 2 if ((n + 63) // 64 <= 16 and 256 < d <= 512) else 1
    dense = ks * n * ((n + 3) & ~3) * 4 + n * ((d + 63) // 64 * 64) * 4
    km1 = K - 1
    per_row = (24 * (7 * km1 + 8) + 8 * (8 * km1 + 8) + 12 * km1 + 8 * K + 16 * 24
               + 48 * 63 + 24 * C + 64)
    assert nb - dense <= n * per_row + 64 * 1024, (nb - dense) / n


def test_every_launched_kernel_has_device_code():
    """Every kernel the host code launches (a __device_stub__ in libgll.so) has its kernel
    descriptor (<name>.kd) in the embedded gfx950 code object: a host pass and a device pass
    compiled from different versions of a source (an object rebuilt while its file changed)
    would otherwise fail only at run time ('Cannot find Symbol'), on the GPU."""
    import re
    data = open(os.path.join(ROOT, "graphlearninglayer_amd", "libgll.so"), "rb").read()
    stubs = set(re.findall(rb"_ZN3gll(\d+)__device_stub__([A-Za-z0-9_]+)", data))
    kds = set(re.findall(rb"(_ZN3gll[0-9]+[A-Za-z0-9_]+)\.kd", data))
    assert stubs and kds
    missing = []
    for ln, rest in stubs:
        name = b"_ZN3gll" + str(int(ln) - len("__device_stub__")).encode() + rest
        if name not in kds:
            missing.append(name.decode())
    assert missing == [], missing[:5]


def test_workspace_row_panels():
    """The distance buffer is n x n up to 32 GiB and a row panel past it (include/gll.h
    GLL_FLAG_KNN_PANEL; gll_internal.h panel_rows): forced panels of 1,024 rows shrink the
    workspace by the rows left out, small graphs never take panels, and at n = 100,000 (40 GB
    of n x n distances) the workspace holds an 8 GiB panel instead."""
    lib = _lib.lib()

    def nbytes(n, d, flags=0):
        return lib.gll_workspace_bytes(ct.byref(G.make_problem(n, d, 0, 1, 10, 0.0, 1.0,
                                                               flags=flags)))
    for n in (100, 1000, 1024):   # panels never shorter than the graph
        assert nbytes(n, 64, _lib.FLAG_KNN_PANEL) == nbytes(n, 64)
    whole, panel = nbytes(5000, 64), nbytes(5000, 64, _lib.FLAG_KNN_PANEL)
    assert whole - panel == (5000 - 1024) * 5000 * 4
    big = nbytes(100_000, 64)
    assert 8 * 2**30 - 100_000 * 4 * 128 <= big < 9 * 2**30


def test_entry_points_reject_bad_arguments_without_touching_the_gpu():
    lib = _lib.lib()
    p = G.make_problem(100, 16, 50, 10, 5, 0.0, 1.0)
    assert lib.gll_forward(ct.byref(p), None, None, 0, None, None, None) == -1
    assert lib.gll_backward(ct.byref(p), None, None, 0, None, None, 0, None, None) == -1
    assert lib.gll_graph(ct.byref(p), None, None, None) == -1
    assert lib.gll_cg_csr(0, 1, None, None, None, None, None, 1e-6, 10, None, None, None,
                          None) == -1
    assert lib.gll_prof_enable(99, 1) == -1


def test_kernel_names():
    names = [_lib.kernel_name(k) for k in range(_lib.K_COUNT)]
    assert names[_lib.K_GRAM] == "gram_d2_kernel"
    assert names[_lib.K_CG] == "cg_kernel"
    assert names[_lib.K_FINALIZE] == "row_build_kernel"


def test_eps_and_problem_mapping():
    assert G._eps_value("auto") == 0.0
    assert G._eps_value(1) == 1.0
    with pytest.warns(UserWarning):
        assert G._eps_value(0.0) > 0.0
    # GLL.py:233-234 use eps only as eps[rows] * eps[cols]: a negative eps is |eps| + the warning
    with pytest.warns(UserWarning):
        assert G._eps_value(-0.5) == 0.5
    with pytest.raises(ValueError):
        G._eps_value("bogus")
    p = G.make_problem(8, 4, 3, 2, k=25)
    assert p.K == 8   # k clamped to n like np.minimum(knn_ind.shape[1], k), GLL.py:187


def test_no_gpu_means_loud_failure():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    X = torch.zeros(10, 4)
    Y = torch.zeros(5, 2)
    with pytest.raises(RuntimeError, match="GPU"):
        G.LaplaceLearningSparseHard.apply(X, Y, 0.0, 1.0)


def test_synth_is_deterministic_and_unit_norm():
    c = CONFIGS["plumbing"]
    X1, l1 = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=3)
    X2, l2 = synth(c["base"], c["batch"], c["d"], r=c["r"], seed=3)
    assert sha256(X1) == sha256(X2)
    assert np.allclose(np.linalg.norm(X1, axis=1), 1.0, atol=1e-6)
    assert (l1[: 10] == np.arange(10)).all()
    Y = one_hot(l1[: c["base"]])
    assert Y.shape == (64, 10) and (Y.sum(1) == 1).all()


def test_product_package_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "graphlearninglayer_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle\b", src, flags=re.M), f
                assert "oracle." not in src, f


def test_torch_extension_module_loads():
    from graphlearninglayer_amd import GLL as GG
    ext = GG._ext()
    assert ext is not None, "_gll_torch.so missing: run __graft_entry__.build()"
    assert callable(ext.apply)
    assert GG.LaplaceLearningSparseHard.apply is ext.apply   # the native function, no wrapper


def test_k_outside_the_supported_range_raises_a_clear_error():
    """k (neighbours incl. self) must satisfy 2 <= min(k, n) <= 257 (include/gll.h): the Python
    layer says so before anything reaches the device."""
    import torch
    from graphlearninglayer_amd import GLL
    X = torch.zeros(400, 8)
    Y = torch.zeros(10, 3)
    for k in (1, 258, 300):
        with pytest.raises(ValueError, match="2 <= min"):
            GLL.LaplaceLearningSparseHard.apply(X, Y, 0.0, 1.0, k)
    with pytest.raises(ValueError, match="2 <= min"):
        GLL.device_graph(X, 260)


def test_product_library_reads_no_switch_but_debug():
    """The product libgll.so reads no environment switch that skips work or changes a path:
    the only GLL_* name in it is GLL_DEBUG (prints launch errors).  Code paths for tests are
    gll_problem.flags and gll_set_knob (include/gll.h), which tests compare against the
    default path; bench.py refuses a value when another GLL_* variable is set."""
    import subprocess
    from graphlearninglayer_amd import _lib
    out = subprocess.run(["strings", "-a", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    names = sorted(set(re.findall(r"\bGLL_[A-Z0-9_]+", out)))
    assert names == ["GLL_DEBUG"], names
