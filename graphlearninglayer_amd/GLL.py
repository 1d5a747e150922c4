"""Host-side mirror of /root/reference/GLL.py on the MI355X HIP path.

Same names, argument meaning and error behaviour as the reference module:

  LaplaceLearningSparseHard.apply(X, label_matrix, tau=0, epsilon='auto'[, k=25])
                                                           GLL.py:10-177
  knn_sym_dist(data, k=25, epsilon='auto') -> W, V, mod_V, C, knn_ind   GLL.py:180-244
  stable_conjgrad(A, b, x0=None, max_iter=1e5, tol=1e-10)              GLL.py:247-276

Every numerical step runs in libgll.so (include/gll.h): exact kNN on fp32 MFMA, CSR graph
build, Jacobi-CG solves, edge gradient and Laplacian SpMM.  PyTorch provides device memory
(the caching allocator hands out the per-call workspace), the current stream and autograd.
There is no CPU fallback: a missing library or a missing GPU raises.

Deliberate differences from the reference (all documented in DESIGN.md):
  * kNN is exact (the reference's annoy index is approximate);
  * the solves are fp32 Jacobi-CG to rtol 1e-6 instead of float64 SuperLU;
  * outputs are placed on X.device (the reference uses the *current* device, GLL.py:15-18);
  * an optional 5th positional argument `k` replaces the hard-coded k=25 (GLL.py:27);
  * X may carry a leading batch dimension (B x n x d, labels B x base x C or shared):
    B independent graphs in one launch per kernel, U is B x m x C.
"""
from __future__ import annotations

import ctypes as ct
import warnings

import numpy as np
import torch

from . import _lib

DEFAULT_K = 25          # GLL.py:27
MAX_K = 257             # include/gll.h: 2 <= K <= 257 (neighbours incl. self; kMaxKm1Huge = 256)
DEFAULT_RTOL = 1e-6     # fp32 Jacobi-CG at 1e-6 matches SuperLU to <1e-5
DEFAULT_MAX_ITER = 1000


def _check_k(k, n):
    """The kNN count the C ABI supports (include/gll.h gll_problem.K): a clear error here
    instead of the ABI's generic 'unsupported problem size'."""
    kk = min(int(k), int(n))
    if kk < 2 or kk > MAX_K:
        raise ValueError(f"k = {k} (n = {n}): the kNN count incl. self must satisfy "
                         f"2 <= min(k, n) <= {MAX_K}")


def _load_ext():
    """_gll_torch.so: LaplaceLearningSparseHard.apply in native code (csrc/torch_ext.cpp) and
    the per-device status sink.  Built in-tree with libgll.so; there is no fallback."""
    try:
        from . import _gll_torch
    except ImportError as e:
        raise ImportError("graphlearninglayer_amd: _gll_torch.so is missing or does not load "
                          "(build it: python graphlearninglayer_amd/build.py). There is no "
                          f"CPU fallback. ({e})") from e
    return _gll_torch


_ext_mod = _load_ext()


def _ext():
    return _ext_mod


# Device status -> the reference's warnings, without a host sync on the hot path: every call's
# kernels OR/max/add their status words into a sticky per-device sink (gll_problem.status_sink,
# owned by _gll_torch); every 64 calls the sink is copied to pinned memory and cleared on the
# stream, and completed copies are turned into warnings (GLL.py:240-241, 273-274) at a later
# call, or at check_status().
def check_status():
    """Flush every device's status sink now and raise the pending warnings (syncs)."""
    _ext_mod.check_status()


def _warn_from(st):
    """The warnings / error of one copy of the status words (as _gll_torch raises them), for
    callers of the C ABI that read the words themselves."""
    if st[_lib.ST_SOLVE_FAILED]:
        raise RuntimeError("GLL: the fused backward's gradient gave up waiting for the adjoint "
                           "solves; its grad_X was written as NaN")
    if st[_lib.ST_GRID_RESCUED]:
        warnings.warn(f"GLL: {st[_lib.ST_GRID_RESCUED]} whole-GPU CG solve(s) lost their grid "
                      "barrier (other kernels held the CUs) and were solved by one workgroup "
                      "instead: correct, slower", RuntimeWarning)
    if st[_lib.ST_TINY_EPS]:
        warnings.warn("Epsilon in KNN is very close to zero.", UserWarning)  # GLL.py:240-241
    if st[_lib.ST_FWD_NONCONV]:
        warnings.warn(f"GLL forward CG: {st[_lib.ST_FWD_NONCONV]} column solve(s) reached "
                      f"max_iter ({st[_lib.ST_FWD_ITERS]} iterations)", RuntimeWarning)
    if st[_lib.ST_BWD_NONCONV]:
        warnings.warn(f"GLL adjoint CG: {st[_lib.ST_BWD_NONCONV]} column solve(s) reached "
                      f"max_iter ({st[_lib.ST_BWD_ITERS]} iterations)", RuntimeWarning)


def _poll_status(dev=None):
    idx = torch.cuda.current_device() if dev is None else dev.index
    _ext_mod.poll_status(idx)


def set_grad_diagnostics(threshold=10.0):
    """Print the reference's 'possible exploding gradient' report when ||grad_X||_F exceeds
    `threshold` (the inline copy of train_and_adversarial.py:177-183 uses 10) for calls made
    from now on; None switches the check off (the default).  The check synchronises."""
    _ext_mod.set_grad_diagnostics(-1.0 if threshold is None else float(threshold))


def _device_for(X: torch.Tensor) -> torch.device:
    if X.is_cuda:
        return X.device
    if not torch.cuda.is_available():
        raise RuntimeError("graphlearninglayer_amd needs a ROCm GPU (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def _features(X: torch.Tensor, dev) -> torch.Tensor:
    X32 = X.detach().to(device=dev, dtype=torch.float32).contiguous()
    if X32.data_ptr() % 16:      # the 16-B vector path needs an aligned base
        X32 = X32.clone()
    return X32


def _typed(t: torch.Tensor, dev):
    t = t.detach().to(dev)
    if t.dtype == torch.float32:
        code = _lib.GLL_DT_F32
    elif t.dtype == torch.float64:
        code = _lib.GLL_DT_F64
    elif t.dtype == torch.int64:
        code = _lib.GLL_DT_I64
    else:
        t, code = t.float(), _lib.GLL_DT_F32
    return t.contiguous(), code


def _eps_value(epsilon) -> float:
    if isinstance(epsilon, str):
        if epsilon != "auto":
            raise ValueError(f"epsilon must be a number or 'auto', got {epsilon!r}")
        return 0.0
    e = float(epsilon)
    if not e > 0.0:
        # GLL.py:240-241 warns for any eps < 1e-10.  The reference uses eps only as the product
        # eps[rows] * eps[cols] (GLL.py:233-234), so a negative eps builds the graph of |eps|;
        # eps = 0 (or NaN) divides by zero there, here it disconnects the graph (W = 0)
        warnings.warn("Epsilon in KNN is very close to zero.", UserWarning)
        return -e if e < 0.0 else 1e-30
    return e


def make_problem(n, d, base, C, k=DEFAULT_K, tau=0.0, epsilon="auto",
                 rtol=DEFAULT_RTOL, max_iter=DEFAULT_MAX_ITER, flags=0) -> _lib.Problem:
    return _lib.Problem(n=int(n), d=int(d), base=int(base), C=int(C), K=int(min(k, n)),
                        max_iter=int(max_iter), tau=float(tau), eps=_eps_value(epsilon),
                        rtol=float(rtol), flags=int(flags))


def _stream(dev) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


class LaplaceLearningSparseHard(torch.autograd.Function):
    """Graph Laplace learning layer; labeled rows of X come first (GLL.py:11).

    `LaplaceLearningSparseHard.apply(X, label_matrix, tau=0, epsilon='auto'[, k=25])` is the
    native function of _gll_torch.so (csrc/torch_ext.cpp): argument checks, the forward
    kernels and one autograd node whose backward runs the backward kernels -- the whole host
    side of a call in C++.  `apply_python` is the same call as a Python
    torch.autograd.Function over the ctypes binding of the same C ABI (tests compare the two
    bitwise).  Both execute only the HIP kernels of libgll.so."""

    apply = staticmethod(_ext_mod.apply)

    @classmethod
    def apply_python(cls, X, label_matrix, tau=0, epsilon="auto", k=DEFAULT_K):
        """The Python torch.autograd.Function path (ctypes onto the same C ABI)."""
        _check_k(k, X.shape[-2])
        return super().apply(X, label_matrix, tau, epsilon, k)

    @staticmethod
    def forward(ctx, X, label_matrix, tau=0, epsilon="auto", k=DEFAULT_K):
        dev = _device_for(X)
        _poll_status(dev)
        if X.dim() not in (2, 3) or label_matrix.dim() not in (2, X.dim()):
            raise ValueError("X must be n x d (or B x n x d), label_matrix base x C "
                             "(or B x base x C)")
        B = X.shape[0] if X.dim() == 3 else 1
        n, d = X.shape[-2:]
        base, C = label_matrix.shape[-2:]
        with torch.cuda.device(dev):
            X32 = _features(X, dev)
            Y, ydt = _typed(label_matrix, dev)
            if X.dim() == 3 and Y.dim() == 2:
                Y = Y.unsqueeze(0).expand(B, base, C).contiguous()   # shared labels
            if X.dim() == 3 and Y.shape[0] != B:
                raise ValueError(f"label_matrix batch {Y.shape[0]} != {B}")
            prob = make_problem(n, d, base, C, k, tau, epsilon)
            prob.status_sink = _ext_mod.status_sink(dev.index)
            nbytes = _lib.lib().gll_workspace_bytes(ct.byref(prob))
            if nbytes == 0:
                raise ValueError(f"unsupported GLL problem n={n} d={d} base={base} C={C} k={k}")
            ws = torch.empty(nbytes * B, dtype=torch.uint8, device=dev)
            U = torch.empty(X.shape[:-2] + (n - base, C), dtype=torch.float64, device=dev)
            _lib.check(_lib.lib().gll_forward_batched(ct.byref(prob), B, X32.data_ptr(),
                                                      Y.data_ptr(), ydt, ws.data_ptr(),
                                                      U.data_ptr(), _stream(dev)),
                       "gll_forward")
            _ext_mod.note_call(dev.index)
        ctx.save_for_backward(X)
        ctx.prob, ctx.ws, ctx.dev, ctx.B = prob, ws, dev, B
        return U if X.is_cuda else U.cpu()

    @staticmethod
    def backward(ctx, grad_output):
        (X,) = ctx.saved_tensors
        dev, prob = ctx.dev, ctx.prob
        with torch.cuda.device(dev):
            X32 = _features(X, dev)
            g, gdt = _typed(grad_output, dev)
            if gdt == _lib.GLL_DT_I64:
                g, gdt = g.double(), _lib.GLL_DT_F64
            gradX = torch.empty(X.shape, dtype=torch.float32, device=dev)
            _lib.check(_lib.lib().gll_backward_batched(ct.byref(prob), ctx.B, X32.data_ptr(),
                                                       ctx.ws.data_ptr(), g.data_ptr(), gdt,
                                                       gradX.data_ptr(), _stream(dev)),
                       "gll_backward")
        if gradX.device != X.device or gradX.dtype != X.dtype:
            gradX = gradX.to(device=X.device, dtype=X.dtype)
        return gradX, None, None, None, None


# ----------------------------------------------------------------------------------------
# knn_sym_dist: device graph, returned as the reference's scipy objects
# ----------------------------------------------------------------------------------------
def device_graph(X: torch.Tensor, k: int = DEFAULT_K, epsilon="auto", flags: int = 0):
    """Build the symmetric kNN graph on the GPU; returns a dict of device tensors
    (knn_idx, knn_d2, eps, row_ptr, col, w, d2, deg).  `flags`: gll_problem.flags
    (e.g. _lib.FLAG_KNN_PANEL, row panels instead of the n x n distances)."""
    _check_k(k, X.shape[0])
    dev = _device_for(X)
    n, d = X.shape
    with torch.cuda.device(dev):
        X32 = _features(X, dev)
        prob = make_problem(n, d, 0, 1, k, 0.0, epsilon, flags=flags)
        nbytes = _lib.lib().gll_workspace_bytes(ct.byref(prob))
        if nbytes == 0:
            raise ValueError(f"unsupported graph problem n={n} d={d} k={k}")
        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        _lib.check(_lib.lib().gll_graph(ct.byref(prob), X32.data_ptr(), ws.data_ptr(),
                                        _stream(dev)), "gll_graph")
        view = _lib.View()
        _lib.check(_lib.lib().gll_workspace_view(ct.byref(prob), ws.data_ptr(), ct.byref(view)),
                   "gll_workspace_view")
        K = prob.K
        base_ptr = ws.data_ptr()

        def arr(ptr, count, dtype):
            off = ptr - base_ptr
            esz = torch.empty(0, dtype=dtype).element_size()
            return ws[off: off + count * esz].view(dtype)

        # padded device rows (row_start, row_len) -> compact CSR
        starts = arr(view.row_start, n, torch.int32).long()
        lens = arr(view.row_len, n, torch.int32).long()
        span = int((starts + lens).max().item())
        row_ptr = torch.zeros(n + 1, dtype=torch.long, device=dev)
        row_ptr[1:] = torch.cumsum(lens, 0)
        E = int(row_ptr[-1].item())
        rows = torch.repeat_interleave(torch.arange(n, device=dev), lens)
        src = starts[rows] + (torch.arange(E, device=dev) - row_ptr[rows])
        out = dict(
            knn_idx=arr(view.knn_idx, n * K, torch.int32).view(n, K),
            knn_d2=arr(view.knn_d2, n * K, torch.float32).view(n, K),
            eps=arr(view.eps, n, torch.float32),
            row_ptr=row_ptr.int(),
            col=arr(view.col, span, torch.int32)[src],
            w=arr(view.w, span, torch.float32)[src],
            d2=arr(view.d2, span, torch.float32)[src],
            deg=arr(view.deg, n, torch.float32),
            status=arr(view.status, _lib.ST_NWORDS, torch.int32),
            workspace=ws,
        )
    return out


def knn_sym_dist(data, k=DEFAULT_K, epsilon="auto"):
    """Mirror of GLL.py:180-244: returns (W, V, mod_V, C, knn_ind) as scipy/numpy objects.

    The graph is built on the GPU (exact kNN); only the final arrays travel to the host."""
    import scipy.sparse as sparse

    X = data if torch.is_tensor(data) else torch.from_numpy(np.ascontiguousarray(data))
    g = device_graph(X, k, epsilon)
    n = X.shape[0]
    rp = g["row_ptr"].cpu().numpy().astype(np.int64)
    col = g["col"].cpu().numpy().astype(np.int64)
    w = g["w"].cpu().numpy().astype(np.float64)
    d2 = g["d2"].cpu().numpy().astype(np.float64)
    eps = g["eps"].cpu().numpy().astype(np.float64)
    knn_ind = g["knn_idx"].cpu().numpy().astype(np.int64)
    rows = np.repeat(np.arange(n), np.diff(rp))
    W = sparse.csr_matrix((w, col, rp), shape=(n, n))
    Vv = -8.0 * w / (eps[rows] * eps[col])
    V = sparse.csr_matrix((Vv, col, rp), shape=(n, n))
    if isinstance(epsilon, str):
        mod_V = sparse.csr_matrix((d2 * Vv / eps[rows] ** 2 / 2, col, rp), shape=(n, n))
        C = sparse.csr_matrix((np.ones(n), (knn_ind[:, -1], knn_ind[:, 0])), shape=(n, n))
    else:
        mod_V, C = 0, 0
    _poll_status()
    return W, V, mod_V, C, knn_ind


# ----------------------------------------------------------------------------------------
# stable_conjgrad: device multi-RHS CG
# ----------------------------------------------------------------------------------------
def refined_solve(rp, ci, val64, B, x=None, tol=1e-10, max_iter=100000, weight=None):
    """Solve A x = B (A SPD, device CSR: int32 row_ptr / col, float64 values; B m x C float64)
    to max_c ||weight * (B - A x)_c||_2 <= tol.

    fp32 Jacobi-CG corrections (libgll gll_cg_csr: the whole-GPU CG for m > 2048) inside
    float64 iterative refinement; the float64 residual uses torch sparse on the GPU.
    Returns (x, err, CG iterations)."""
    dev = B.device
    m, C = B.shape
    val32 = val64.float().contiguous()
    with warnings.catch_warnings():   # "sparse CSR support is in beta" (torch 2.10)
        warnings.simplefilter("ignore", UserWarning)
        A64 = torch.sparse_csr_tensor(rp.long(), ci.long(), val64, size=(m, m))
    x = torch.zeros_like(B) if x is None else x
    ws = torch.empty(_lib.lib().gll_cg_csr_workspace_bytes(m, C), dtype=torch.uint8, device=dev)
    counters = torch.zeros(2, dtype=torch.int32, device=dev)
    total = 0
    max_iter = int(max_iter)

    def residual(x):
        r = B - (A64 @ x)
        rw = r if weight is None else r * weight[:, None]
        return r, torch.linalg.vector_norm(rw, dim=0).max().item()

    r, err = residual(x)
    for _ in range(32):  # refinement sweeps
        if err <= tol or total >= max_iter:
            break
        scale = max(torch.linalg.vector_norm(r, dim=0).max().item(), 1e-300)
        r32 = (r / scale).float().contiguous()
        d32 = torch.empty_like(r32)
        counters.zero_()
        _lib.check(_lib.lib().gll_cg_csr(m, C, rp.data_ptr(), ci.data_ptr(), val32.data_ptr(),
                                         r32.data_ptr(), d32.data_ptr(),
                                         ct.c_float(1e-6), max_iter - total,
                                         counters.data_ptr(), counters[1:].data_ptr(),
                                         ws.data_ptr(), _stream(dev)), "gll_cg_csr")
        total += int(counters[0].item())
        x = x + scale * d32.double()
        r, err = residual(x)
    return x, err, total


def stable_conjgrad(A, b, x0=None, max_iter=1e5, tol=1e-10):
    """Mirror of GLL.py:247-276: solve A x = b (A SPD, b n x C) to max_col ||r||_2 <= tol.

    Mixed precision on the device: fp32 Jacobi-CG (libgll gll_cg_csr) inside float64
    iterative refinement (residual r = b - A x in float64 with torch sparse on the GPU),
    so the float64 tolerance of the reference is reachable."""
    import scipy.sparse as sparse

    if not torch.cuda.is_available():
        raise RuntimeError("graphlearninglayer_amd needs a ROCm GPU (no CPU fallback)")
    dev = torch.device("cuda", torch.cuda.current_device())
    A = sparse.csr_matrix(A)
    b_np = np.asarray(b, dtype=np.float64)
    vec = b_np.ndim == 1
    B = torch.from_numpy(b_np.reshape(b_np.shape[0], -1)).to(dev)
    m, C = B.shape
    rp = torch.from_numpy(A.indptr.astype(np.int32)).to(dev)
    ci = torch.from_numpy(A.indices.astype(np.int32)).to(dev)
    val64 = torch.from_numpy(A.data.astype(np.float64)).to(dev)
    x = None if x0 is None else torch.from_numpy(
        np.asarray(x0, dtype=np.float64).reshape(m, C)).to(dev)
    x, err, total = refined_solve(rp, ci, val64, B, x, tol, max_iter)
    if err > tol:
        print("max iter reached: ", total, " iters")  # GLL.py:273-274
    out = x.cpu().numpy()
    return out.ravel() if vec else out
