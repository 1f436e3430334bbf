"""Result alias and dataset enum (reference: src/types.py:14, :18-40)."""
from __future__ import annotations

import enum
from typing import Any, Dict

Result = Dict[str, Any]
"""Result type for each FL epoch, round, and task."""


class DataChoices(enum.Enum):
    """Dataset options (values are the reference's CLI strings)."""

    CIFAR10_AUGMENT = "cifar10_augment"
    CIFAR10_AUGMENT_VGG = "cifar10_augment_vgg"
    CIFAR10_VGG = "cifar10_vgg"
    CIFAR100_VGG = "cifar100_vgg"
    CIFAR10_DROPOUT = "cifar10_dropout"
    CIFAR10_AUGMENT_DROPOUT = "cifar10_augment_dropout"
    CIFAR10_MOBILE = "cifar10_mobile"
    CIFAR10_VIT = "cifar10_vit"
    CIFAR10_RESTNET18 = "cifar10_restnet18"
    CIFAR10_RESTNET50 = "cifar10_restnet50"
    CIFAR10 = "cifar10"
    CIFAR100 = "cifar100"
    FMNIST = "fmnist"
    MNIST = "mnist"
    TINYMEM = "tiny_mem"
    TINYMEM_EVEN_INCREMENT_ONE = "tiny_mem_even_increment_one"
