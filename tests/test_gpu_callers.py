"""the adversarial scripts' call pattern through the layer, on the GPU.

train_and_adversarial.py:545-552 / 711-749 and adversarial.py:529-564, 671-691 call the layer
as `lap(features, one_hot(target)[:k, :])` -- int64 labels, tau = 0, epsilon = 'auto',
k = 25 -- behind a network, take `torch.autograd.grad(custom_ce_loss(...), [data])` w.r.t. the
input images (FGSM / PGD) and edit the output in place (CW).  Checked against the float64
oracle wrapped as a CPU autograd node, chained through the same network in float64 and fed
the GPU's kNN lists (so fp32 near-ties in the search do not enter the comparison).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import gll_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-4


def custom_ce_loss(softmax_logits, targets):
    """losses.py:128-136."""
    batch_size, num_classes = softmax_logits.shape
    one_hot_targets = F.one_hot(targets, num_classes=num_classes).to(softmax_logits.dtype)
    return -torch.sum(one_hot_targets * torch.log(softmax_logits + 1e-8)) / batch_size


class OracleLayer(torch.autograd.Function):
    """The float64 closed-form oracle as an autograd node (CPU, test infrastructure)."""

    @staticmethod
    def forward(ctx, X, Y, knn_ind):
        U, st = O.forward(X.detach().numpy(), Y.numpy(), tau=0.0, epsilon="auto", K=25,
                          knn=(knn_ind, None))
        ctx.st = st
        return torch.from_numpy(U)

    @staticmethod
    def backward(ctx, g):
        return torch.from_numpy(O.backward(ctx.st, g.detach().numpy())), None, None


def _model(dtype, device):
    gen = torch.Generator().manual_seed(7)
    W1 = torch.randn(64, 96, generator=gen, dtype=torch.float64) / 8.0
    W2 = torch.randn(96, 32, generator=gen, dtype=torch.float64) / 10.0
    W1, W2 = W1.to(device, dtype), W2.to(device, dtype)
    return lambda x: torch.tanh(x @ W1) @ W2


def _batch():
    from graphlearninglayer_amd.synth import synth
    images, target = synth(100, 200, 64, C=10, r=1.5, seed=4)   # 8x8 "images", base rows first
    return images, torch.from_numpy(target)


def test_fgsm_gradient_wrt_inputs_matches_oracle():
    from graphlearninglayer_amd import GLL
    images, target = _batch()
    k = 100
    # GPU: the caller's code, verbatim in structure (train_and_adversarial.py:711-733)
    data = torch.from_numpy(images).cuda()
    data.requires_grad = True
    lap = GLL.LaplaceLearningSparseHard.apply
    label_matrix = F.one_hot(target.cuda(), num_classes=10)          # int64
    features = _model(torch.float32, "cuda")(data)
    output = lap(features, label_matrix[:k, :])
    loss = custom_ce_loss(output, target.cuda()[k:])
    grad, grad_feat = torch.autograd.grad(loss, [data, features])
    assert output.dtype == torch.float64 and grad.shape == data.shape
    # oracle: same network in float64, oracle layer, autograd on the CPU
    ind = GLL.device_graph(features.detach(), 25, "auto")["knn_idx"].cpu().numpy().astype(np.int64)
    d64 = torch.from_numpy(images.astype(np.float64)).requires_grad_(True)
    f64 = _model(torch.float64, "cpu")(d64)
    Yo = F.one_hot(target, num_classes=10)[:k, :].to(torch.float64)
    out64 = OracleLayer.apply(f64, Yo, ind)
    loss64 = custom_ce_loss(out64, target[k:])
    g64 = torch.autograd.grad(loss64, [d64])[0]
    assert O.rel_err(output.detach().cpu().numpy(), out64.detach().numpy()) <= TOL
    assert abs(loss.item() - loss64.item()) <= TOL * abs(loss64.item())
    # the layer itself at the 1e-4 bar: its gradient w.r.t. the features it was given (the
    # GPU's fp32 features, in float64, through the oracle layer and the same loss)
    fo = features.detach().cpu().double().requires_grad_(True)
    lo = custom_ce_loss(OracleLayer.apply(fo, Yo, ind), target[k:])
    go = torch.autograd.grad(lo, [fo])[0]
    assert O.rel_err(grad_feat.cpu().numpy(), go.numpy()) <= TOL
    # through the fp32 network to the input images: the network's own fp32 rounding (against
    # the float64 network of the oracle chain) adds to the layer's error here
    assert O.rel_err(grad.cpu().numpy(), g64.numpy()) <= 5 * TOL


def test_pgd_loop_and_cw_inplace_edit():
    """A 3-step PGD loop (train_and_adversarial.py:705-749) and the CW in-place edit of the
    output (adversarial.py:688-691): runs, stays finite, leaves later calls unaffected."""
    from graphlearninglayer_amd import GLL
    images, target = _batch()
    k = 100
    lap = GLL.LaplaceLearningSparseHard.apply
    model = _model(torch.float32, "cuda")
    base_data = torch.from_numpy(images[:k]).cuda()
    train_data = torch.from_numpy(images[k:]).cuda()
    tgt = target.cuda()
    label_matrix = F.one_hot(tgt, num_classes=10)
    perturbed = train_data.clone()
    alpha, eps_box = 0.01, 0.03
    for _ in range(3):
        data = torch.vstack((base_data, perturbed))
        data.requires_grad = True
        output = lap(model(data), label_matrix[:k, :])
        loss = custom_ce_loss(output, tgt[k:])
        grad = torch.autograd.grad(loss, [data])[0][k:]
        assert torch.isfinite(grad).all()
        perturbed = perturbed.detach() + alpha * torch.sign(grad.detach())
        perturbed = torch.clamp(perturbed, train_data - eps_box, train_data + eps_box)
    with torch.no_grad():
        output = lap(model(torch.vstack((base_data, perturbed))), label_matrix[:k, :])
        ref = output.clone()
        idx = torch.arange(output.shape[0], device=output.device)
        init_pred = output.max(1, keepdim=False)[1]
        output[idx, init_pred] = -1000000                          # adversarial.py:691
        again = lap(model(torch.vstack((base_data, perturbed))), label_matrix[:k, :])
    torch.testing.assert_close(again, ref, rtol=0, atol=0)


def test_exploding_gradient_diagnostic(capsys):
    """train_and_adversarial.py:177-183: with the diagnostic on, a feature gradient whose norm
    exceeds the threshold prints the reference's messages."""
    from graphlearninglayer_amd import GLL
    images, target = _batch()
    X = (torch.from_numpy(images).cuda() * 50.0).requires_grad_(True)
    Y = F.one_hot(target.cuda(), num_classes=10)[:100, :]
    GLL.set_grad_diagnostics(1e-6)
    try:
        U = GLL.LaplaceLearningSparseHard.apply(X, Y)
        (g,) = torch.autograd.grad(U.sum(), X)
    finally:
        GLL.set_grad_diagnostics(None)
    out = capsys.readouterr().out
    assert "possible exploding gradient" in out and "grad norm:" in out
    torch.cuda.synchronize()
    assert torch.isfinite(g).all()


def test_fullysup_step_with_device_base_loader():
    """§8f-4: the FullySup GL step (FullySup.py:134-157) with the base set drawn from the
    HBM-resident provider instead of `next(iter(base_loader))`: the draw is a permutation of
    the base set on the GPU, and the step's prediction and input gradient match the float64
    oracle chained through the same network."""
    from graphlearninglayer_amd import GLL
    from graphlearninglayer_amd.base_data import DeviceBaseLoader
    g = torch.Generator().manual_seed(0)
    nb, m, k = 100, 300, 25
    base_imgs = torch.rand(nb, 3, 8, 8, generator=g)
    base_lab = torch.arange(nb) % 10
    imgs = torch.rand(m, 3, 8, 8, generator=g)
    lab = torch.randint(0, 10, (m,), generator=g)
    W = torch.randn(192, 32, generator=g, dtype=torch.float64) / 8
    prov = DeviceBaseLoader(base_imgs, base_lab, device="cuda", seed=5)
    bi, bl = next(iter(prov))
    assert bi.is_cuda and sorted(bl.tolist()) == sorted(base_lab.tolist())
    x = torch.cat((bi, imgs.cuda()), 0).requires_grad_(True)          # FullySup.py:154
    feats = F.normalize(x.flatten(1).double() @ W.cuda(), dim=1).float()
    pred = GLL.LaplaceLearningSparseHard.apply(feats, prov.label_matrix(bl), 0.07, 1.0, k)
    loss = custom_ce_loss(pred, lab.cuda())
    (gx,) = torch.autograd.grad(loss, [x])
    # oracle chained through the same network in float64, on the GPU's kNN lists
    ind = GLL.device_graph(feats.detach(), k, 1.0)["knn_idx"].cpu().numpy().astype(np.int64)
    xc = x.detach().cpu().requires_grad_(True)
    fc = F.normalize(xc.flatten(1).double() @ W, dim=1).float().double()
    Uo, st = O.forward(fc.detach().numpy(), prov.label_matrix(bl).cpu().numpy(), 0.07, 1.0, k,
                       knn=(ind, None))
    assert O.rel_err(pred.detach().cpu().numpy(), Uo) < TOL
    Ut = torch.from_numpy(Uo).requires_grad_(True)
    lo = custom_ce_loss(Ut, lab)
    (gU,) = torch.autograd.grad(lo, [Ut])
    gf = torch.from_numpy(O.backward(st, gU.numpy()))
    (gxo,) = torch.autograd.grad(fc, [xc], gf)
    assert O.rel_err(gx.cpu().numpy(), gxo.numpy()) < TOL
