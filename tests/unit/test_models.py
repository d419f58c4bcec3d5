"""Model zoo: parameter counts match the reference models."""
import pytest
import torch

from ewdml.models import build_model, canonical_name, input_shape, model_names

COUNTS = {  # (name, classes) -> (params, tensors), measured by instantiating the reference models
    ("LeNet", 10): (431080, 8),
    ("VGG11", 10): (9756426, 38),
    ("ResNet18", 10): (11173962, 62),
    ("ResNet50", 10): (23520842, 161),
}


@pytest.mark.parametrize("name,classes", list(COUNTS))
def test_param_counts(name, classes):
    m = build_model(name, classes)
    params = list(m.parameters())
    assert sum(p.numel() for p in params) == COUNTS[(name, classes)][0]
    assert len(params) == COUNTS[(name, classes)][1]


def test_lenet_shapes_match_reference():
    m = build_model("LeNet")
    shapes = [tuple(p.shape) for p in m.parameters()]
    assert shapes == [(20, 1, 5, 5), (20,), (50, 20, 5, 5), (50,), (500, 800), (500,), (10, 500),
                      (10,)]


@pytest.mark.parametrize("name", ["LeNet", "mnistnet", "VGG11", "vgg13", "ResNet18", "ResNet34"])
def test_forward_shapes(name):
    m = build_model(name, 10).eval()
    x = torch.randn(2, *input_shape(name))
    assert m(x).shape == (2, 10)


def test_aliases_and_num_classes():
    assert canonical_name("ResNet") == "resnet18"
    assert canonical_name("Resnet50") == "resnet50"
    assert canonical_name("vgg11") == "vgg11"
    m = build_model("ResNet50", 100)  # the reference's ResNet50() ignores num_classes
    assert m.linear.out_features == 100
    with pytest.raises(ValueError):
        build_model("NoSuchNet")
    assert "resnet50_imagenet" in model_names()


def test_imagenet_resnet50_224():
    m = build_model("resnet50_imagenet", 1000).eval()
    with torch.no_grad():
        assert m(torch.randn(1, 3, 224, 224)).shape == (1, 1000)
