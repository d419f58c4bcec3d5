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


def test_vgg_fused_features_is_a_plain_sequential_on_cpu():
    """FusedFeatures keeps nn.Sequential's modules/state_dict keys and is exactly its forward on
    the CPU; its plan groups conv-BN-ReLU[-pool]."""
    import torch.nn as nn

    from ewdml.models.fused import FusedFeatures

    torch.manual_seed(0)
    m = build_model("VGG11", 10).train()
    assert isinstance(m.features, FusedFeatures)
    keys = list(m.state_dict())
    assert keys[:6] == ["features.0.weight", "features.0.bias", "features.1.weight",
                        "features.1.bias", "features.1.running_mean", "features.1.running_var"]
    plan = m.features._plan()
    assert [k for k, _, _ in plan] == ["cbr"] * 8
    assert [p for _, _, p in plan] == [True, True, False, True, False, True, False, True]
    x = torch.randn(4, 3, 32, 32)
    ref = nn.Sequential(*list(m.features))
    torch.testing.assert_close(m.features(x), ref(x), rtol=0, atol=0)


def test_flat_model_keeps_channels_last_param_layout():
    from ewdml.parallel.flat import FlatModel

    m = build_model("VGG11", 10).to(memory_format=torch.channels_last)
    w = m.features[4].weight
    flat = FlatModel(m, attach_grads=False)
    assert w.is_contiguous(memory_format=torch.channels_last)
    x = torch.randn(2, 3, 32, 32).contiguous(memory_format=torch.channels_last)
    flat.zero_grad()
    m(x).sum().backward()
    g_before = w.grad
    grads = [g for b in flat.buckets for g in flat.bucket_grads(b)]
    # a gradient already in the parameter's memory order is read in place (no copy)
    assert any(g.data_ptr() == g_before.data_ptr() for g in grads)
    assert w.grad.stride() == w.stride()
