"""The ResNets' parameter layout against torchvision's PUBLISHED numbers (an
independent pin for tests/golden/state_dict_keys.json, which torchvision's
absence forces us to generate from our own resnet.py).

torchvision 0.15's weight metadata (``ResNet18_Weights.IMAGENET1K_V1.meta
["num_params"]`` etc., shown in its model table) lists 11,689,512 /
25,557,032 / 60,192,808 parameters for ResNet-18/50/152 with 1000 classes;
the torchvision module structure fixes the key names (``conv1``, ``bn1``,
``layerN.M.convK`` / ``bnK`` / ``downsample.0|1``, ``fc``) and three buffers per
BatchNorm (``running_mean``, ``running_var``, ``num_batches_tracked``)."""
import re

import pytest
import torch

from distributed_training_amd.resnet import MODELS

PUBLISHED = {"resnet18": 11_689_512, "resnet50": 25_557_032, "resnet152": 60_192_808}
BLOCKS = {"resnet18": [2, 2, 2, 2], "resnet50": [3, 4, 6, 3], "resnet152": [3, 8, 36, 3]}


@pytest.mark.parametrize("name", sorted(PUBLISHED))
def test_param_count_and_keys_match_torchvision(name):
    m = MODELS[name](num_classes=1000)
    assert sum(p.numel() for p in m.parameters()) == PUBLISHED[name]
    keys = list(m.state_dict().keys())
    bottleneck = name != "resnet18"
    convs = 3 if bottleneck else 2
    want = ["conv1.weight", "bn1.weight", "bn1.bias", "bn1.running_mean", "bn1.running_var",
            "bn1.num_batches_tracked"]
    for li, nb in enumerate(BLOCKS[name], start=1):
        for b in range(nb):
            pre = f"layer{li}.{b}"
            for k in range(1, convs + 1):
                want += [f"{pre}.conv{k}.weight", f"{pre}.bn{k}.weight", f"{pre}.bn{k}.bias",
                         f"{pre}.bn{k}.running_mean", f"{pre}.bn{k}.running_var", f"{pre}.bn{k}.num_batches_tracked"]
            if b == 0 and (bottleneck or li > 1):
                want += [f"{pre}.downsample.0.weight", f"{pre}.downsample.1.weight", f"{pre}.downsample.1.bias",
                         f"{pre}.downsample.1.running_mean", f"{pre}.downsample.1.running_var",
                         f"{pre}.downsample.1.num_batches_tracked"]
    want += ["fc.weight", "fc.bias"]
    assert keys == want
    n_bn = sum(1 for k in keys if k.endswith("num_batches_tracked"))
    assert len(keys) == len(list(m.parameters())) + 3 * n_bn


def test_torchvision_init_scheme():
    """kaiming_normal_(fan_out, relu) convs, BN weight 1 / bias 0, nn.Linear's
    default fc init (torchvision ResNet.__init__)."""
    torch.manual_seed(0)
    m = MODELS["resnet50"]()
    for name, mod in m.named_modules():
        if isinstance(mod, torch.nn.Conv2d):
            fan_out = mod.out_channels * mod.kernel_size[0] * mod.kernel_size[1]
            std = (2.0 / fan_out) ** 0.5
            s = float(mod.weight.std())
            assert abs(s - std) < 0.2 * std, (name, s, std)
        elif isinstance(mod, torch.nn.BatchNorm2d):
            assert torch.equal(mod.weight, torch.ones_like(mod.weight)) and torch.equal(mod.bias, torch.zeros_like(mod.bias))
    bound = 1 / 2048 ** 0.5
    assert float(m.fc.weight.abs().max()) <= bound and re.match(r"Linear", type(m.fc).__name__)
