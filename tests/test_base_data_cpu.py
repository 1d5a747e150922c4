"""Sampling contract of the device-resident base provider, on the CPU.

The reference draws `next(iter(base_loader))` every step (FullySup.py:135) from a DataLoader
with batch_size=len(base set) and shuffle=True (FullySup.py:262-266): the whole base set, in a
fresh uniformly random order, images and labels aligned.  DeviceBaseLoader must deliver the
same contract from device memory.
"""
import numpy as np
import torch

from graphlearninglayer_amd.base_data import DeviceBaseLoader


def _base(n=250, c=10):
    labels = torch.arange(n) % c
    # each image carries its own index and label, so alignment is checkable after a shuffle
    data = torch.zeros(n, 3, 4, 4)
    data[:, 0, 0, 0] = torch.arange(n, dtype=torch.float32)
    data[:, 1, 0, 0] = labels.float()
    return data, labels


def test_draw_is_an_aligned_permutation_of_the_whole_set():
    data, labels = _base()
    p = DeviceBaseLoader(data, labels, device="cpu", seed=0)
    imgs, lab = next(iter(p))                      # the reference's call form
    assert imgs.shape == data.shape and lab.shape == labels.shape and lab.dtype == torch.int64
    idx = imgs[:, 0, 0, 0].long()
    assert sorted(idx.tolist()) == list(range(len(data)))            # every sample once
    assert torch.equal(imgs[:, 1, 0, 0].long(), lab)                 # labels follow images
    assert torch.equal(labels[idx], lab)
    assert not torch.equal(idx, torch.arange(len(data)))             # actually shuffled


def test_same_contract_as_the_reference_dataloader():
    """DataLoader(batch_size=N, shuffle=True) over the same set yields one batch holding the
    same multiset of (image, label) pairs as a provider draw."""
    from torch.utils.data import DataLoader, TensorDataset
    data, labels = _base(60)
    (dl_imgs, dl_lab), = list(DataLoader(TensorDataset(data, labels), batch_size=60, shuffle=True))
    imgs, lab = DeviceBaseLoader(data, labels, device="cpu", seed=3).sample()
    key = lambda im, lb: sorted(zip(im[:, 0, 0, 0].tolist(), lb.tolist()))
    assert key(dl_imgs, dl_lab) == key(imgs, lab)


def test_seeded_draws_reproduce_and_successive_draws_differ():
    data, labels = _base()
    a = DeviceBaseLoader(data, labels, device="cpu", seed=7)
    b = DeviceBaseLoader(data, labels, device="cpu", seed=7)
    a1, b1 = a.sample()[1], b.sample()[1]
    assert torch.equal(a1, b1)
    assert not torch.equal(a.sample()[0], a.sample()[0])


def test_positions_are_uniform():
    """Each sample lands in position 0 with probability 1/N (chi-square, 2000 draws)."""
    n, draws = 5, 2000
    p = DeviceBaseLoader(torch.arange(n).float(), torch.arange(n), device="cpu", seed=11)
    counts = np.bincount([int(p.sample()[1][0]) for _ in range(draws)], minlength=n)
    chi2 = float(((counts - draws / n) ** 2 / (draws / n)).sum())
    assert chi2 < 20.5          # 4 dof, p ~ 4e-4


def test_no_shuffle_keeps_order_and_label_matrix():
    data, labels = _base(30)
    p = DeviceBaseLoader(data, labels, device="cpu", shuffle=False)
    imgs, lab = p.sample()
    assert torch.equal(imgs, data) and torch.equal(lab, labels)
    Y = p.label_matrix(lab)
    assert Y.dtype == torch.float32 and Y.shape == (30, 10)
    assert torch.equal(Y, torch.nn.functional.one_hot(labels, 10).float())   # FullySup.py:153


def test_from_dataset_and_update():
    class CustomDataset(torch.utils.data.Dataset):   # shape of utils.py:170-187
        def __init__(self, data, labels, transform=None):
            self.data, self.labels, self.transform = data, labels, transform

        def __len__(self):
            return len(self.data)

        def __getitem__(self, i):
            return self.data[i], self.labels[i]

    data, labels = _base(40)
    p = DeviceBaseLoader.from_dataset(CustomDataset(data, labels), device="cpu", seed=1)
    assert len(p) == 40
    idx = p.sample()[0][:, 0, 0, 0].long()
    assert sorted(idx.tolist()) == list(range(40))
    d2, l2 = _base(20)
    p.update(d2, l2)                                   # re-selected base set (FullySup.py:278)
    assert len(p) == 20 and sorted(p.sample()[1].tolist()) == sorted(l2.tolist())


def test_rejects_misaligned_or_float_labels():
    import pytest
    data, labels = _base(10)
    with pytest.raises(ValueError):
        DeviceBaseLoader(data, labels[:9], device="cpu")
    with pytest.raises(TypeError):
        DeviceBaseLoader(data, labels.float(), device="cpu")


def test_label_matrix_default_follows_the_latest_draw():
    """`Y = p.label_matrix()` right after `imgs, _ = next(iter(p))` lines up with those images
    (the draw's permuted labels, not the stored order); before any draw it is an error."""
    import pytest
    data, labels = _base(50)
    p = DeviceBaseLoader(data, labels, device="cpu", seed=4)
    with pytest.raises(RuntimeError):
        p.label_matrix()
    imgs, lab = next(iter(p))
    Y = p.label_matrix()
    idx = imgs[:, 0, 0, 0].long()                      # sample i of the draw is base row idx[i]
    assert torch.equal(Y, torch.nn.functional.one_hot(labels[idx], 10).float())
    assert torch.equal(Y, p.label_matrix(lab))
