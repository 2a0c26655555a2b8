"""ResNet-101 encoders with the reference surface (models/encoder.py of
SarahAlkhateeb/Image-Captioning-with-Different-Decoders).

``EncoderAttention`` (reference :72-121) and ``Encoder`` (:22-69) keep their
constructor, ``forward`` and ``fine_tune`` signatures, the ``resnet`` /
``adaptive_pool`` / ``embed`` attributes and the state-dict keys
(``resnet.<i>...`` over torchvision's children()). On HIP tensors the conv
stack runs through libcapmi (capmi.resnet.EncoderRunner); on CPU tensors the
ordinary nn modules run, as the reference does on its CPU config.
"""
import os

import torch
from torch import nn

from capmi import kernels as K
from capmi.resnet import EncoderRunner, FineTuneRunner, resnet101, trainable_encoder_params

_LOCAL_WEIGHTS = os.path.join("models", "resnet101.pth")


def _load_resnet101_model():
    """Reference :9-20 loads torchvision weights (a local models/resnet101.pth, or a download).
    Offline, this loads $CAPMI_RESNET101_WEIGHTS or models/resnet101.pth when present
    (weights_only=True), else keeps torchvision's random init (seeded by the caller)."""
    path = os.environ.get("CAPMI_RESNET101_WEIGHTS")
    if path is None and os.path.exists(_LOCAL_WEIGHTS):
        path = _LOCAL_WEIGHTS
    return resnet101(path)


class _ResNetView:
    """Attribute view of Sequential(children()[:-2 or -1]) for the fused runner."""

    def __init__(self, seq):
        self.conv1, self.bn1 = seq[0], seq[1]
        self.layer1, self.layer2, self.layer3, self.layer4 = seq[4], seq[5], seq[6], seq[7]


def _check_frozen(module):
    if torch.is_grad_enabled() and any(p.requires_grad for p in module.parameters()):
        raise NotImplementedError(
            "capmi: a trainable Encoder (baseline model) is not on the capmi path; EncoderAttention "
            "supports fine_tune() (layer2-4)")


def _fine_tuned(seq):
    """True when any parameter of the resnet requires grad; only children()[5:] (layer2-4, what
    fine_tune() switches, models/encoder.py:112-121) may: the stem and layer1 stay frozen."""
    if not any(p.requires_grad for p in seq.parameters()):
        return False
    for i in range(5):
        if any(p.requires_grad for p in seq[i].parameters()):
            raise NotImplementedError("capmi: only layer2-4 (EncoderAttention.fine_tune) can be trained")
    return True


class EncoderFineTuneFn(torch.autograd.Function):
    """Differentiable EncoderAttention.forward for fine_tune(True): the fused forward keeps the
    trainable stages' activations, backward runs capmi's conv dgrad/wgrad + BN backward."""

    @staticmethod
    def forward(ctx, module, imgs, *params):
        ctx.module = module
        ctx.n = len(params)
        return module.ft_forward(imgs)

    @staticmethod
    def backward(ctx, dfeat):
        m = ctx.module
        plist = trainable_encoder_params(_ResNetView(m.resnet))
        grads = {id(p): torch.empty_like(p) for p in plist if p.requires_grad}
        m.ft_backward(dfeat.contiguous(), grads)
        return (None, None) + tuple(grads.get(id(p)) for p in plist)



def _runner_free_state(module):
    """Pickle state of an encoder module without its launch caches (workspaces, packed
    weights): torch.save(encoder) writes only what the reference's whole-module checkpoints
    hold (checkpoint.py:39-62); the runner is rebuilt, with its precision, on load."""
    st = module.__dict__.copy()
    runner = st.pop("_runner", None)
    st.pop("_ft_runner", None)
    st["_capmi_bf16"] = bool(runner is not None and runner.bf16)
    st["_capmi_x3"] = bool(runner is not None and getattr(runner, "x3", False))
    return st


def _runner_restore(module, st):
    bf16 = st.pop("_capmi_bf16", False)
    x3 = st.pop("_capmi_x3", False)
    nn.Module.__setstate__(module, st)
    module._runner = EncoderRunner()
    module._runner.bf16 = bf16
    module._runner.x3 = x3

class Encoder(nn.Module):
    """CNN encoder of the baseline model (reference :22-69)."""

    def __init__(self, embed_size):
        super().__init__()
        resnet = _load_resnet101_model()
        modules = list(resnet.children())[:-1]
        self.resnet = nn.Sequential(*modules)
        self.embed = nn.Linear(resnet.fc.in_features, embed_size)
        for param in self.resnet.parameters():
            param.requires_grad = False
        self._runner = EncoderRunner()

    def __getstate__(self):
        return _runner_free_state(self)

    def __setstate__(self, st):
        _runner_restore(self, st)

    def forward(self, imgs):
        if not imgs.is_cuda:
            features = self.resnet(imgs)
            return self.embed(features.view(features.size(0), -1))
        _check_frozen(self.resnet)
        feats = self._runner.forward(_ResNetView(self.resnet), imgs.contiguous(), (1, 1),
                                     train=self.training)
        N = feats.shape[0]
        out = torch.empty(N, self.embed.out_features, device=imgs.device, dtype=torch.float32)
        if torch.is_grad_enabled() and self.embed.weight.requires_grad:
            return torch.nn.functional.linear(feats.view(N, -1), self.embed.weight, self.embed.bias)
        K.gemm(K.problem(N, self.embed.out_features, 2048, feats, 2048, self.embed.weight, 2048, out,
                         self.embed.out_features, bias=self.embed.bias), 0, 0, K.TILE_64)
        return out

    def fine_tune(self, on=True):
        for conv_block in list(self.resnet.children())[5:]:
            for param in conv_block.parameters():
                param.requires_grad = on


class EncoderAttention(nn.Module):
    """CNN encoder of the attention model (reference :72-121): (B,3,H,W) -> (B,14,14,2048)."""

    def __init__(self):
        super().__init__()
        resnet = _load_resnet101_model()
        modules = list(resnet.children())[:-2]
        self.resnet = nn.Sequential(*modules)
        self.adaptive_pool = nn.AdaptiveAvgPool2d((14, 14))
        for param in self.resnet.parameters():
            param.requires_grad = False
        self._runner = EncoderRunner()

    def __getstate__(self):
        return _runner_free_state(self)

    def __setstate__(self, st):
        _runner_restore(self, st)

    def set_compute_precision(self, precision):
        """'fp32' (the reference's: v_mfma_f32_32x32x2_f32), 'fp32-x3' (fp32-accurate: the convs'
        fp32 operands split exactly into three bf16 terms whose six significant cross products are
        accumulated in fp32 on the bf16 matrix cores; fp32 activations, statistics and features) or
        'bf16': the frozen forward on bf16 NHWC activations and weights, bf16 MFMA with fp32
        accumulation and fp32 BatchNorm statistics, features returned fp32 -- the bf16 config
        (BASELINE config 5)."""
        if precision not in ("fp32", "fp32-x3", "bf16"):
            raise ValueError(precision)
        self._runner.bf16 = precision == "bf16"
        self._runner.x3 = precision == "fp32-x3"

    def _out_hw(self):
        out_hw = self.adaptive_pool.output_size
        return (out_hw, out_hw) if isinstance(out_hw, int) else tuple(out_hw)

    def forward(self, imgs):
        if not imgs.is_cuda:
            features = self.adaptive_pool(self.resnet(imgs))
            return features.permute(0, 2, 3, 1)
        if torch.is_grad_enabled() and _fine_tuned(self.resnet):
            if not self.training:
                raise NotImplementedError("capmi: fine-tuning runs BatchNorm in train mode (encoder.train())")
            plist = trainable_encoder_params(_ResNetView(self.resnet))
            return EncoderFineTuneFn.apply(self, imgs.contiguous(), *plist)
        return self._runner.forward(_ResNetView(self.resnet), imgs.contiguous(), self._out_hw(),
                                    train=self.training)

    # ---- fine-tune path (capmi's train step calls these directly) -------------------
    def _ft(self):
        ft = getattr(self, "_ft_runner", None)
        if ft is None:
            ft = FineTuneRunner(self._runner)
            self._ft_runner = ft
        return ft

    def ft_forward(self, imgs, out=None, pooled=True):
        """Train-mode forward that keeps layer2-4's activations for ft_backward (fp32). pooled=False:
        the layer4 map (see forward_into); ft_backward then takes its gradient."""
        if self._runner.bf16:
            raise NotImplementedError("capmi: the fine-tune path runs fp32 (set_compute_precision('fp32'))")
        return self._ft().forward(_ResNetView(self.resnet), imgs.contiguous(),
                                  self._out_hw() if pooled else None, out=out)

    def ft_backward(self, dfeat, grads, hook=None, on_layer=None):
        """d(loss)/d(features) (B,14,14,2048) -> parameter gradients of layer2-4 written into
        ``grads`` (dict id(param) -> tensor). ``on_layer(li)``: called as stage li's gradients
        become final (layer4, layer3, layer2; capmi.resnet.FineTuneRunner.backward)."""
        self._ft().backward(dfeat, grads, hook=hook, on_layer=on_layer)

    def forward_into(self, imgs, out, pooled=True):
        """forward() writing the (B,14,14,2048) features into a caller-owned buffer (the
        pipelined training step keeps two of them). pooled=False: the (B,7,7,2048) layer4 map
        before adaptive_pool -- the distinct rows of the pooled features when the pool only
        repeats pixels (capmi.resnet.pool_dup; the training step's decoder runs on them)."""
        _check_frozen(self.resnet)
        return self._runner.forward(_ResNetView(self.resnet), imgs.contiguous(),
                                    self._out_hw() if pooled else None, train=self.training, out=out)

    def fine_tune(self, on=True):
        for conv_block in list(self.resnet.children())[5:]:
            for param in conv_block.parameters():
                param.requires_grad = on
