"""Device mirror of the reference's large-graph Laplace learning evaluation.

  one_hot_encode(labels, n_classes='auto')                              utils.py:556-568
  laplace(X, train_labels, knn_num=50, epsilon='auto', n_classes='auto', tau=1e-8)
                                                                        utils.py:570-593
  gl_accuracy(train_data, train_label, test_data, test_label, unlabeled_data=None, ...)
                                  the numerical part of test_GL_NP,     utils.py:637-660

The reference builds the kNN graph of ~60k points (250 labeled, 50k unlabeled training and
10k test features, k = 50) with annoy on the CPU and solves the Jacobi-scaled system with
stable_conjgrad to 1e-10 every `--plot_freq_ss` epochs.  Here the graph comes from the HIP
kNN/graph kernels (exact kNN, libgll gll_graph) and the solve from the whole-GPU CG inside
float64 iterative refinement, stopped on the reference's criterion: the residual of the
SCALED system M Luu M y = M rhs (M = diag(Luu + 1e-10)^(-1/2)), i.e. max_c ||M (rhs - Luu x)||
<= tol.  The returned prediction is the reference's `M * Pred` (= x), a host float64 array.
"""
from __future__ import annotations

import numpy as np
import torch

from . import GLL


def one_hot_encode(labels, n_classes="auto"):
    """utils.py:556-568."""
    labels = np.asarray(labels)
    n_labels = len(labels)
    if n_classes == "auto":
        n_classes = len(np.unique(labels))
    one_hot = np.zeros((n_labels, int(n_classes)))
    one_hot[np.arange(n_labels), labels] = 1
    return one_hot


def laplace(X, train_labels, knn_num=50, epsilon="auto", n_classes="auto", tau=1e-8,
            tol=1e-10, max_iter=100000):
    """utils.py:570-593 on the GPU: labeled rows of X first (the reference: 'labeled indices
    are 0,1,2,...,k-1').  Returns the m x C float64 prediction of the unlabeled rows."""
    Xt = X if torch.is_tensor(X) else torch.from_numpy(np.ascontiguousarray(X))
    dev = GLL._device_for(Xt)
    Y = one_hot_encode(train_labels, n_classes)
    k = Y.shape[0]
    n = Xt.shape[0]
    m = n - k
    with torch.cuda.device(dev):
        g = GLL.device_graph(Xt, knn_num, epsilon)            # W of knn_sym_dist, utils.py:574
        rp, col = g["row_ptr"].long(), g["col"].long()
        w = g["w"].double()
        rows = torch.repeat_interleave(torch.arange(n, device=dev), rp[1:] - rp[:-1])
        deg = torch.zeros(n, dtype=torch.float64, device=dev).index_add_(0, rows, w)
        del g
        # Luu = L[k:, k:] + tau I with L = D - W (csgraph.laplacian, utils.py:575-584)
        uu = (rows >= k) & (col >= k)
        ur, uc, uw = rows[uu] - k, col[uu] - k, -w[uu]
        diag = deg[k:] + tau
        ar = torch.cat([ur, torch.arange(m, device=dev)])
        ac = torch.cat([uc, torch.arange(m, device=dev)])
        av = torch.cat([uw, diag])
        order = torch.argsort(ar * m + ac)
        ar, ac, av = ar[order], ac[order], av[order]
        arp = torch.zeros(m + 1, dtype=torch.long, device=dev)
        arp[1:] = torch.cumsum(torch.bincount(ar, minlength=m), 0)
        # rhs = -Lul Y = W_ul Y (utils.py:590)
        ul = (rows >= k) & (col < k)
        Yd = torch.from_numpy(Y).to(dev)
        rhs = torch.zeros(m, Y.shape[1], dtype=torch.float64, device=dev)
        rhs.index_add_(0, rows[ul] - k, w[ul][:, None] * Yd[col[ul]])
        # stable_conjgrad(M Luu M, M rhs) to tol on the scaled residual (utils.py:586-591)
        M = 1.0 / torch.sqrt(diag + 1e-10)
        x, err, iters = GLL.refined_solve(arp.int(), ac.int(), av, rhs, None, tol, max_iter,
                                          weight=M)
    if err > tol:
        print("max iter reached: ", iters, " iters")   # GLL.py:273-274 via stable_conjgrad
    return x.cpu().numpy()


def gl_accuracy(train_data, train_label, test_data, test_label, unlabeled_data=None,
                epsilon=1.0, tau=1e-8, knn_num=50):
    """The numerical part of test_GL_NP (utils.py:637-660) on feature arrays: Laplace learning
    on [train; unlabeled; test], accuracy (%) of argmax on the test rows."""
    parts = [train_data] + ([unlabeled_data] if unlabeled_data is not None else []) + [test_data]
    all_data = np.concatenate([np.asarray(p, dtype=np.float32) for p in parts], axis=0)
    U = laplace(all_data, np.asarray(train_label), knn_num=knn_num, epsilon=epsilon,
                n_classes="auto", tau=tau)
    pred = np.argmax(U, axis=1)
    correct = int(np.sum(pred[-len(test_data):] == np.asarray(test_label)))
    return 100.0 * correct / len(test_data)
