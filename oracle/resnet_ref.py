"""ORACLE (test infrastructure): CPU restatement of the ResNet-101 encoder.

The reference builds its encoder from ``torchvision.models.resnet101``
(models/encoder.py:9-20) and keeps ``children()[:-2]`` + AdaptiveAvgPool2d(14,14)
+ permute(0,2,3,1) (models/encoder.py:88-92,107-110). torchvision is a
third-party dependency that is not vendored in /root/reference and not
installed here; no version is pinned anywhere in the reference (SURVEY.md
§8c). This file restates torchvision's *published* ResNet-101 layout:

  conv1 7x7/2 p3 -> bn1 -> relu -> maxpool 3x3/2 p1 -> layer1..layer4
  Bottleneck (expansion 4, "v1.5": stride on the 3x3 conv):
      conv1 1x1 -> bn1 -> relu -> conv2 3x3/s p1 -> bn2 -> relu
      -> conv3 1x1 -> bn3 ; + identity (downsample = 1x1/s conv + bn) ; relu
  BatchNorm2d eps 1e-5, momentum 0.1; blocks per stage (3, 4, 23, 3).

Parity status: conv/BN arithmetic is *parity unpinned* against the reference
(no reference test or fixture covers it); it is checked against torch-CPU
F.conv2d / F.batch_norm, which is what torchvision itself calls.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1, downsample=False):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, width * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(width * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = None
        if downsample:
            self.downsample = nn.Sequential(
                nn.Conv2d(cin, width * 4, 1, stride=stride, bias=False),
                nn.BatchNorm2d(width * 4))

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return self.relu(y + idt)


class ResNet101(nn.Module):
    """children() order matches torchvision: conv1, bn1, relu, maxpool,
    layer1..4, avgpool, fc (so the reference's children()[:-2] / [:-1]
    slicing at models/encoder.py:38,90 means the same thing)."""

    def __init__(self, layers=(3, 4, 23, 3), num_classes=1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        cin = 64
        for i, (n, w, s) in enumerate(zip(layers, (64, 128, 256, 512), (1, 2, 2, 2))):
            blocks = []
            for b in range(n):
                blocks.append(Bottleneck(cin, w, s if b == 0 else 1, downsample=(b == 0)))
                cin = w * 4
            setattr(self, f"layer{i + 1}", nn.Sequential(*blocks))
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def build_resnet101(params=None, layers=(3, 4, 23, 3)):
    """ResNet-101 with the given numpy/torch state (names as tests/golden/gen.py)."""
    m = ResNet101(layers)
    if params is not None:
        sd = m.state_dict()
        for k, v in params.items():
            sd[k] = torch.as_tensor(v).clone()
        m.load_state_dict(sd)
    return m


def encoder_attention_forward(resnet, imgs, out_hw=(14, 14)):
    """models/encoder.py:97-110: resnet children()[:-2] -> AdaptiveAvgPool2d(14,14)
    -> permute(0,2,3,1). BN mode follows ``resnet.training`` (the reference
    calls encoder.train(), models/attention.py:374, so batch statistics)."""
    x = resnet.maxpool(resnet.relu(resnet.bn1(resnet.conv1(imgs))))
    x = resnet.layer4(resnet.layer3(resnet.layer2(resnet.layer1(x))))
    x = F.adaptive_avg_pool2d(x, out_hw)
    return x.permute(0, 2, 3, 1)


def conv_bn_stats_ref(y):
    """Per-channel batch mean / biased var / unbiased var of an NCHW tensor,
    as F.batch_norm(training=True) uses them (normalise with biased var,
    update running_var with the unbiased one)."""
    n = y.numel() // y.shape[1]
    mean = y.mean(dim=(0, 2, 3))
    var = y.var(dim=(0, 2, 3), unbiased=False)
    return mean, var, var * n / max(n - 1, 1)
