"""Models and datasets the driver needs — subset of the reference's src/modules.py.

Only the state_dict layouts matter to the aggregation path (pinned by
tests/golden/layouts.json).  Datasets: when torchvision or the CIFAR files are unavailable
(no network here or on the GPU box) a deterministic synthetic CIFAR-shaped dataset is used;
set TAL_SYNTHETIC_DATA=1 to force it.
"""
from __future__ import annotations

import os
import pathlib

import torch
from torch import nn
from torch.utils.data import Dataset

from src.types import DataChoices


class CifarModule(nn.Module):
    """CIFAR CNN (reference src/modules.py:18-54): 6 conv + 3 linear layers in `network`."""

    def __init__(self, num_classes: int):
        super().__init__()
        self.num_classes = num_classes

        def conv(cin, cout):
            return nn.Conv2d(cin, cout, kernel_size=3, stride=1, padding=1)

        self.network = nn.Sequential(
            conv(3, 32), nn.ReLU(), conv(32, 64), nn.ReLU(), nn.MaxPool2d(2, 2),
            conv(64, 128), nn.ReLU(), conv(128, 128), nn.ReLU(), nn.MaxPool2d(2, 2),
            conv(128, 256), nn.ReLU(), conv(256, 256), nn.ReLU(), nn.MaxPool2d(2, 2),
            nn.Flatten(), nn.Linear(256 * 4 * 4, 1024), nn.ReLU(), nn.Linear(1024, 512), nn.ReLU(),
            nn.Linear(512, num_classes),
        )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.network(x)


def create_model(data: DataChoices, n_layer: int = 4, max_ctx: int = 150) -> nn.Module:
    """Model for a dataset choice (reference src/modules.py:226-311; the CIFAR CNN and the
    ResNets — the BASELINE layouts — are provided)."""
    name = data.value.lower()
    if name in ("cifar10", "cifar10_augment"):
        return CifarModule(10)
    if name == "cifar100":
        return CifarModule(100)
    if name == "cifar10_restnet18":
        from src.models.resnet import ResNet18

        return ResNet18()
    if name == "cifar10_restnet50":
        from src.models.resnet import ResNet50

        return ResNet50()
    raise NotImplementedError(f"model for {data.value!r} is outside the accelerated path's layouts")


class SyntheticImages(Dataset):
    """Deterministic CIFAR-shaped data: x ~ N(0,1) [3,32,32], y in [0, num_classes)."""

    def __init__(self, n: int, num_classes: int = 10, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        self.data = torch.randn(n, 3, 32, 32, generator=g)
        self.targets = torch.randint(0, num_classes, (n,), generator=g).tolist()

    def __len__(self) -> int:
        return len(self.targets)

    def __getitem__(self, i):
        return self.data[i], self.targets[i]


def load_data(data_name: DataChoices, root: pathlib.Path, train: bool, download: bool = False, **_kw) -> Dataset:
    """Training / test set (reference src/modules.py:479-671)."""
    name = data_name.value.lower()
    ncls = 100 if "cifar100" in name else 10
    n = int(os.environ.get("TAL_SYNTHETIC_SAMPLES", "512" if train else "128"))
    if os.environ.get("TAL_SYNTHETIC_DATA", "0") != "1":
        try:
            import torchvision  # noqa: F401
            from torchvision import datasets, transforms

            tf = transforms.Compose([transforms.ToTensor(), transforms.Normalize((0.5,) * 3, (0.5,) * 3)])
            cls = datasets.CIFAR100 if ncls == 100 else datasets.CIFAR10
            return cls(root=root, train=train, transform=tf, download=False)
        except Exception:  # noqa: BLE001 - no torchvision / no files: fall back below
            pass
    return SyntheticImages(n, ncls, seed=0 if train else 1)
