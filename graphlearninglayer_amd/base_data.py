"""Device-resident base (labeled) sample provider for the GLL training step.

The reference's training step draws its labeled base set with

    base_images, base_labels = next(iter(base_loader))          FullySup.py:135
                                                                compare_to_mlp.py:43

where `base_loader` is a DataLoader over the whole base set (`select_base_data`,
utils.py:768-808: a CustomDataset of stacked tensors, transform=None) with
batch_size=len(dataset), shuffle=True, pin_memory=True and opt.num_workers workers
(FullySup.py:262-266, rebuilt at :278-281 when the base set is re-selected).  Every step
therefore creates a fresh iterator -- worker processes, per-sample __getitem__, collation,
pinning and an H2D copy -- to deliver the same N images in a new order: the logged step time
is DT 7.66 s of BT 8.05 s (save/.../output_record_20240718-235017.txt:14).

`DeviceBaseLoader` keeps the base images and labels resident in device memory (a few MB:
250 CIFAR images are 3 MB in HBM) and serves each draw as one on-device random permutation
(`torch.randperm` with the loader's own generator, then `index_select`), which is the
distribution the DataLoader's RandomSampler produces.  It is a drop-in for the loader at the
call site: `next(iter(provider))` yields one (images, labels) batch like the DataLoader does,
and `label_matrix()` gives the one-hot float matrix FullySup.py:153 builds for
`LaplaceLearningSparseHard.apply`.  `update()` replaces the base set when the caller
re-selects it (FullySup.py:278).
"""
from __future__ import annotations

import torch


class DeviceBaseLoader:
    """Whole-base-set batches from device memory, one random permutation per draw.

    data:   N x ... tensor of base samples (any dtype; images as the loader would collate them)
    labels: N integer class labels
    device: where the set lives (default: the current CUDA device, else the CPU)
    shuffle: permute every draw (the reference loader uses shuffle=True)
    seed:   seeds the loader's own generator (None: nondeterministic, like the DataLoader)
    """

    def __init__(self, data, labels, device=None, shuffle=True, seed=None, num_classes=10):
        if device is None:
            device = (torch.device("cuda", torch.cuda.current_device())
                      if torch.cuda.is_available() else torch.device("cpu"))
        self.device = torch.device(device)
        self.shuffle = bool(shuffle)
        self.num_classes = int(num_classes)
        self._gen = torch.Generator(device=self.device)
        if seed is None:
            self._gen.seed()
        else:
            self._gen.manual_seed(int(seed))
        self.update(data, labels)

    @classmethod
    def from_dataset(cls, dataset, **kw):
        """Build from a map-style dataset of (sample, label) items -- the CustomDataset that
        select_base_data returns (utils.py:806), whose .data / .labels tensors are used as they
        are when its transform is None."""
        if getattr(dataset, "transform", None) is None and hasattr(dataset, "data") \
                and hasattr(dataset, "labels"):
            data, labels = torch.as_tensor(dataset.data), torch.as_tensor(dataset.labels)
        else:
            items = [dataset[i] for i in range(len(dataset))]
            data = torch.stack([torch.as_tensor(x) for x, _ in items])
            labels = torch.as_tensor([int(y) for _, y in items])
        return cls(data, labels, **kw)

    def update(self, data, labels) -> None:
        """Replace the base set (the reference re-selects it every gl_update_base_epochs)."""
        data = torch.as_tensor(data)
        labels = torch.as_tensor(labels)
        if data.shape[0] != labels.shape[0]:
            raise ValueError(f"{data.shape[0]} samples but {labels.shape[0]} labels")
        if labels.dtype.is_floating_point or labels.dtype == torch.bool:
            raise TypeError("labels must be integer class indices")
        self.data = data.to(self.device).contiguous()
        self.labels = labels.to(self.device, torch.int64).contiguous()
        self._last_labels = None   # labels of the latest draw, in that draw's order

    def __len__(self) -> int:
        return int(self.data.shape[0])

    def sample(self):
        """One draw: (images, labels) of the whole base set in a fresh random order."""
        if not self.shuffle:
            self._last_labels = self.labels
            return self.data, self.labels
        perm = torch.randperm(len(self), device=self.device, generator=self._gen)
        lab = self.labels.index_select(0, perm)
        self._last_labels = lab
        return self.data.index_select(0, perm), lab

    def __iter__(self):
        # one batch per iterator, as DataLoader(batch_size=len(dataset)) yields
        yield self.sample()

    def label_matrix(self, labels=None) -> torch.Tensor:
        """One-hot float32 label matrix of a draw (FullySup.py:153).  Without `labels`: the
        labels of the latest draw, in that draw's order, so the rows line up with the images
        `next(iter(provider))` returned; before any draw that is an error (the stored order
        matches no batch the caller holds)."""
        if labels is None:
            if self._last_labels is None:
                raise RuntimeError("label_matrix(): no draw yet -- pass the labels of the batch")
            labels = self._last_labels
        return torch.nn.functional.one_hot(labels, num_classes=self.num_classes).float()
