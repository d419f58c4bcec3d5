"""Model zoo and the name -> model factory.

Parity: ``PyTorch-parameter-server/src/util.py:7-18`` (``build_model``).  The reference accepts
``LeNet``, ``ResNet18``, ``ResNet34`` (broken), ``ResNet50`` (ignores num_classes) and ``VGG11``
(= vgg11_bn) and silently returns ``None`` otherwise.  Here names are case-insensitive, the README
aliases (``ResNet`` -> ResNet18, ``Resnet50``) work, every model honours ``num_classes`` and an
unknown name raises.
"""
from .lenet import KerasMnistCNN, LeNet, MnistNet
from .resnet import ResNet, ResNet18, ResNet34, ResNet50, ResNet101, ResNet152
from .vgg import (VGG, vgg11, vgg11_bn, vgg13, vgg13_bn, vgg16, vgg16_bn, vgg19,
                  vgg19_bn)

# name -> (factory(num_classes, **kw), expected input shape (C, H, W))
_REGISTRY = {
    "lenet": (lambda n, **kw: LeNet(n, **kw), (1, 28, 28)),
    "mnistnet": (lambda n, **kw: MnistNet(n), (1, 28, 28)),
    "kerasmnistcnn": (lambda n, **kw: KerasMnistCNN(n), (1, 28, 28)),
    "vgg11": (lambda n, **kw: vgg11_bn(n), (3, 32, 32)),  # reference "VGG11" is the BN variant
    "vgg11_bn": (lambda n, **kw: vgg11_bn(n), (3, 32, 32)),
    "vgg11_nobn": (lambda n, **kw: vgg11(n), (3, 32, 32)),
    "vgg13": (lambda n, **kw: vgg13_bn(n), (3, 32, 32)),
    "vgg13_nobn": (lambda n, **kw: vgg13(n), (3, 32, 32)),
    "vgg16": (lambda n, **kw: vgg16_bn(n), (3, 32, 32)),
    "vgg16_nobn": (lambda n, **kw: vgg16(n), (3, 32, 32)),
    "vgg19": (lambda n, **kw: vgg19_bn(n), (3, 32, 32)),
    "vgg19_nobn": (lambda n, **kw: vgg19(n), (3, 32, 32)),
    "resnet18": (lambda n, **kw: ResNet18(n), (3, 32, 32)),
    "resnet34": (lambda n, **kw: ResNet34(n), (3, 32, 32)),
    "resnet50": (lambda n, **kw: ResNet50(n), (3, 32, 32)),
    "resnet101": (lambda n, **kw: ResNet101(n), (3, 32, 32)),
    "resnet152": (lambda n, **kw: ResNet152(n), (3, 32, 32)),
    "resnet50_imagenet": (lambda n, **kw: ResNet50(n, stem="imagenet"), (3, 224, 224)),
    "resnet18_imagenet": (lambda n, **kw: ResNet18(n, stem="imagenet"), (3, 224, 224)),
}
_ALIASES = {"resnet": "resnet18", "vgg": "vgg11"}


def canonical_name(name: str) -> str:
    key = name.strip().lower().replace("-", "_")
    key = _ALIASES.get(key, key)
    if key not in _REGISTRY:
        raise ValueError(f"unknown network {name!r}; known: {sorted(_REGISTRY)}")
    return key


def model_names():
    return sorted(_REGISTRY)


def input_shape(name: str):
    return _REGISTRY[canonical_name(name)][1]


def fused_fp32_beats_amp(name: str) -> bool:
    """Whether the named model's fused fp32 training step is faster than its bf16 autocast path
    (a class attribute, ``LeNet.fused_fp32_beats_amp``): the trainer keeps that step under
    ``--amp bf16``."""
    entry = _REGISTRY.get(canonical_name(name))
    cls = {"lenet": LeNet}.get(canonical_name(name))
    return bool(entry is not None and cls is not None and getattr(cls, "fused_fp32_beats_amp",
                                                                  False))


def build_model(name: str, num_classes: int = 10, **kw):
    return _REGISTRY[canonical_name(name)][0](num_classes, **kw)


__all__ = [
    "KerasMnistCNN", "LeNet", "MnistNet", "VGG", "ResNet", "ResNet18", "ResNet34", "ResNet50", "ResNet101",
    "ResNet152", "vgg11", "vgg11_bn", "vgg13", "vgg13_bn", "vgg16", "vgg16_bn", "vgg19",
    "vgg19_bn", "build_model", "canonical_name", "input_shape", "model_names",
]
