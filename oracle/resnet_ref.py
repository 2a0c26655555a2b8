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


def _bf16(x):
    """fp32 -> nearest bf16 (RNE) -> fp32."""
    return x.to(torch.bfloat16).to(torch.float32)


def _bn_train_fp64(y, bn):
    """Train-mode BN scale / shift from the batch statistics of the STORED values y (NCHW fp32), summed in
    fp64 and rounded as the GPU finalize rounds them (csrc/bn_final.h: var = E[y^2] - mean^2, clamped at 0)."""
    yd = y.double()
    n = yd.numel() // yd.shape[1]
    s, q = yd.sum((0, 2, 3)), (yd * yd).sum((0, 2, 3))
    mean = s / n
    var = (q / n - mean * mean).clamp_min(0)
    sc = (bn.weight.double() * (1.0 / torch.sqrt(var + bn.eps))).float()
    sh = (bn.bias.double() - mean * sc.double()).float()
    return sc.view(1, -1, 1, 1), sh.view(1, -1, 1, 1)


@torch.no_grad()
def encoder_forward_bf16_emulated(resnet, imgs):
    """CPU restatement of the GPU bf16 encoder's ARITHMETIC (BASELINE config 5; capmi.resnet._forward_bf16),
    for test infrastructure only: the layer4 map (N, 7, 7, 2048) NHWC fp32 of train-mode ResNet-101 where
    * conv1 multiplies bf16-rounded images and weights with fp32 accumulation into an fp32 output, then BN + ReLU
      + maxpool in fp32 and the result rounded to bf16 (capmi_bn_relu_maxpool, capmi_f32_to_bf16);
    * every other conv multiplies bf16 activations by bf16-rounded weights with fp32 accumulation and stores
      its output rounded to bf16 (CAPMI_GEMM_BF16_IO); BN statistics are those of the stored values;
    * a conv input is bf16(relu(y * scale + shift)) (capmi_bn_relu_bf16), a block output
      bf16(relu(y3 * s3 + b3 + res')) with res' = the bf16 block input, or yd * sd + bd for the downsample
      branch (capmi_bn_add_relu_bf16).
    The products of bf16 values are exact in fp32; only the fp32 summation order differs from the GPU's, so this
    path's error against fp64 is the error the bf16 arithmetic itself makes."""
    def conv(x, c):
        return F.conv2d(x, _bf16(c.weight.float()), stride=c.stride, padding=c.padding)
    r = resnet
    y = F.conv2d(_bf16(imgs.float()), _bf16(r.conv1.weight.float()), stride=2, padding=3)
    sc, sh = _bn_train_fp64(y, r.bn1)
    x = _bf16(F.max_pool2d(torch.relu(y * sc + sh), 3, 2, 1))
    for layer in (r.layer1, r.layer2, r.layer3, r.layer4):
        for blk in layer:
            y1 = _bf16(conv(x, blk.conv1))
            s1, b1 = _bn_train_fp64(y1, blk.bn1)
            y1 = _bf16(torch.relu(y1 * s1 + b1))
            y2 = _bf16(conv(y1, blk.conv2))
            s2, b2 = _bn_train_fp64(y2, blk.bn2)
            y2 = _bf16(torch.relu(y2 * s2 + b2))
            y3 = _bf16(conv(y2, blk.conv3))
            s3, b3 = _bn_train_fp64(y3, blk.bn3)
            if blk.downsample is not None:
                yd = _bf16(conv(x, blk.downsample[0]))
                sd, bd = _bn_train_fp64(yd, blk.downsample[1])
                res = yd * sd + bd
            else:
                res = x
            x = _bf16(torch.relu(y3 * s3 + b3 + res))
    return x.permute(0, 2, 3, 1)
