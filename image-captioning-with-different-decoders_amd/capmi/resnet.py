"""ResNet-101 (torchvision layout) with a fused MI355X forward.

The module tree mirrors torchvision.models.resnet101 exactly (names, children()
order: conv1, bn1, relu, maxpool, layer1..4, avgpool, fc), so the reference's
``list(resnet.children())[:-2]`` / ``[:-1]`` slicing (models/encoder.py:38,90)
and its state-dict keys (a local ``resnet101.pth``) mean the same thing here.

On a HIP device, ``fused_forward`` runs the conv stack through libcapmi:
every Conv2d is an implicit GEMM on fp32 MFMA over NHWC activations; the
BatchNorm that follows it is split into (a) batch statistics accumulated in
the conv GEMM's epilogue, (b) a tiny finalize kernel (mean/var -> scale/shift,
running-stat update in train mode) and (c) the apply+ReLU, fused into the next
conv's A-tile load or into the bottleneck tail kernel (BN + residual + ReLU).
On CPU tensors the modules run their ordinary nn forward (config 1 plumbing).
"""
import os

import torch
import torch.nn as nn

from . import kernels as K
from ._lib import CAPMI_A_CONV_NHWC, CAPMI_A_CONV_NHWC4, CAPMI_A_KMAJOR, CAPMI_A_MMAJOR, CAPMI_B_CONV_NHWC
from ._lib import CAPMI_B_KROWS, CAPMI_B_NMAJOR_W, CAPMI_GEMM_BF16, CAPMI_GEMM_SPLIT3

AK, AMM, AC = CAPMI_A_KMAJOR, CAPMI_A_MMAJOR, CAPMI_A_CONV_NHWC
BW, BKR, BCONV = CAPMI_B_NMAJOR_W, CAPMI_B_KROWS, CAPMI_B_CONV_NHWC


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
            self.downsample = nn.Sequential(nn.Conv2d(cin, width * 4, 1, stride=stride, bias=False),
                                            nn.BatchNorm2d(width * 4))
        self.stride = stride

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        return self.relu(self.bn3(self.conv3(y)) + idt)


class ResNet101(nn.Module):
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
        self.reset_parameters()

    def reset_parameters(self):
        """torchvision's init: kaiming_normal_(fan_out, relu) convs, BN weight 1 / bias 0."""
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet101(weights_path=None):
    """Seeded-random ResNet-101 (torch RNG), or the weights of a local torchvision
    checkpoint (``weights_path``, loaded with weights_only=True). Never downloads."""
    m = ResNet101()
    if weights_path is not None:
        m.load_state_dict(torch.load(weights_path, map_location="cpu", weights_only=True))
    return m


# ======================================================================================
# fused forward
# ======================================================================================
class _Packed:
    """Conv weights in the GEMM's B layout: [Cout][KH][KW][Cin] (K-contiguous; Cin padded to 4
    for conv1)."""

    def __init__(self):
        self.cache = {}

    def get(self, conv):
        w = conv.weight
        co, ci, kh, kw = w.shape
        if kh == 1 and kw == 1:
            return w  # [Cout][Cin] already
        cp = 4 if ci <= 4 else ci  # conv1 (Cin = 3): channels zero-padded to 4 (NHWC4 input)
        key = id(conv)
        ent = self.cache.get(key)
        if ent is None or ent[0] != w._version or ent[1] != w.data_ptr():
            packed = torch.empty(co, kh, kw, cp, device=w.device, dtype=w.dtype)
            K.conv_weight_pack_pad(w.detach().contiguous(), cp, packed)
            ent = (w._version, w.data_ptr(), packed)
            self.cache[key] = ent
        return ent[2]


def feature_hw(H, W):
    """Side of ResNet-101's layer4 map for an H x W image (conv1 7x7/2, maxpool 3x3/2, three
    stride-2 stages): 224 -> 7."""
    def down(x, k, st, pad):
        return (x + 2 * pad - k) // st + 1
    h, w = down(down(H, 7, 2, 3), 3, 2, 1), down(down(W, 7, 2, 3), 3, 2, 1)
    for _ in range(3):
        h, w = down(h, 3, 2, 1), down(w, 3, 2, 1)
    return h, w


def pool_dup(H, W, out_hw):
    """d when AdaptiveAvgPool2d(out_hw) of the H x W image's layer4 map only repeats pixels
    (out side = d x map side, d integer, equal in both directions; every window holds one input
    pixel, so the pooled value IS that pixel), else 1."""
    fh, fw = feature_hw(H, W)
    oh, ow = out_hw
    if fh <= 0 or fw <= 0 or oh % fh or ow % fw or oh // fh != ow // fw:
        return 1
    return oh // fh


# x3 mode: convs with K <= this run both operands split in-kernel (CAPMI_GEMM_SPLIT3) instead of gemm_x3
_X3_SMALLK = int(os.environ.get("CAPMI_X3_SMALLK", "0"))
# x3 mode: route the shapes where it measured fastest to the x3d kernel (CAPMI_X3D=0: off, A/B)
_X3D = os.environ.get("CAPMI_X3D", "1") != "0"
# x3 mode: layer1's K = 64 1x1 convs on the short-k streaming kernel (CAPMI_X3S=0: off, A/B)
_X3S = os.environ.get("CAPMI_X3S", "1") != "0"
# x3 mode (round 4): layer1's 3x3 on the direct conv (gemm_x3c.hip: each input element split once per 32-channel
# slice instead of once per tap; CAPMI_X3C=0: gemm_x3, A/B)
_X3C = os.environ.get("CAPMI_X3C", "1") != "0"

class EncoderRunner:
    """Launch plan for the frozen ResNet-101 conv stack (children()[:-2] of torchvision's
    resnet101) on NHWC fp32 activations. Buffers are cached per input shape."""

    def __init__(self):
        self.packed = _Packed()
        self._ws = None
        self._ws_key = None
        self.conv_hook = None  # optional callable(tag, flops, launch_fn, kernel_key) (bench timing)
        # bf16 forward (the bf16 config, BASELINE config 5): bf16 NHWC activations and weights, bf16
        # MFMA with fp32 accumulation, fp32 BN statistics (_forward_bf16); fp32 is the reference's
        self.bf16 = False
        # fp32 convs as fp32-accurate three-term bf16 split GEMMs (CAPMI_GEMM_X3, gemm_x3.hip) instead
        # of v_mfma_f32_32x32x2_f32; same fp32 activations, statistics and outputs
        self.x3 = False

    def _workspace(self, N, H, W, device):
        key = (N, H, W, str(device))
        if self._ws_key != key:
            H1, W1 = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
            big = N * H1 * W1 * 64  # conv1 output; layer1 outputs are N*(H1/2)^2*256 = same
            big = max(big, N * ((H1 + 1) // 2) * ((W1 + 1) // 2) * 256)
            f = dict(device=device, dtype=torch.float32)
            ws = {n: torch.empty(big, **f) for n in ("x", "y1", "y2", "y3", "yd", "out")}
            ws["stats"] = torch.empty(2 * ((N * H1 * W1 + 63) // 64) * 256, **f)
            # zeroed once: holds the BN finalize arrival counters, re-armed by the kernel
            ws["bnwork"] = torch.zeros(K.bn_work_doubles(2048), device=device, dtype=torch.float64)
            ws["ss"] = {}
            ws["sk"] = K.gemm_workspace(device)  # stream-K partials + flags (zeroed once)
            ws["img4"] = torch.empty(N * H * W * 4, **f)  # conv1 input, NHWC padded to 4 channels
            ws["x3p"] = None
            self._ws, self._ws_key = ws, key
        return self._ws

    def _x3p_buffer(self, ws):
        if ws["x3p"] is None:  # three bf16 planes of the largest conv input (x3 path only)
            ws["x3p"] = torch.empty(3 * ws["x"].numel(), device=ws["x"].device, dtype=torch.bfloat16)
        return ws["x3p"]

    def _ss(self, ws, bn):
        ent = ws["ss"].get(id(bn))
        if ent is None:
            C = bn.num_features
            ent = torch.empty(2, C, device=bn.weight.device, dtype=torch.float32)
            ws["ss"][id(bn)] = ent
        return ent[0], ent[1]

    def _bn(self, ws, bn, rows, train):
        """BatchNorm params for the conv output just produced: batch stats (train) or running."""
        s, b = self._ss(ws, bn)
        C = bn.num_features
        if train:
            tiles = K.stat_tiles(rows)
            mom = 0.1 if bn.momentum is None else bn.momentum
            K.bn_finalize(ws["stats"], tiles, C, rows, bn.weight, bn.bias,
                          bn.running_mean if bn.track_running_stats else None,
                          bn.running_var if bn.track_running_stats else None, mom, bn.eps, s, b,
                          ws["bnwork"])
        else:
            K.bn_eval_params(bn.weight, bn.bias, bn.running_mean, bn.running_var, C, bn.eps, s, b)
        return s, b

    def _conv(self, tag, x, conv, out, N, H, W, train, in_ss=None, nchw=False):
        co, ci, kh, kw = conv.weight.shape
        st, pd = conv.stride[0], conv.padding[0]
        Ho, Wo = (H + 2 * pd - kh) // st + 1, (W + 2 * pd - kw) // st + 1
        rows = N * Ho * Wo
        Kd = ci * kh * kw
        geo = dict(N=N, H=H, W=W, Cin=ci, KH=kh, KW=kw, stride=st, pad=pd, Ho=Ho, Wo=Wo)
        stats = ws_stats = self._ws["stats"] if train else None
        kw_ = dict(stats=ws_stats)
        # conv1 stays on the fp32 MFMA kernel in the x3 mode: SPLIT3 measured 264 vs 261 us there (the
        # 7x7/2 im2col gather over the NHWC4 images bounds it, not the MFMA)
        split3 = False
        # the x3 kernels address their A operand with 32-bit buffer offsets (< 2 GiB: fp32 for x3d /
        # gemm_x3, three bf16 planes for x3p); a bigger per-GPU batch runs that conv on the fp32 MFMA
        # kernel instead of failing in the planner (CAPMI_ERANGE)
        a_elems = N * H * W * ci
        x3 = self.x3 and a_elems * 4 < (1 << 31)
        smallk = not nchw and x3 and Kd <= _X3_SMALLK
        # x3d (A fp32 split in-kernel, B planes by LDS-DMA, 256x128 tiles; tools/x3_ab.py at batch 64,
        # profiles/r02_x3_ab_x3d.md, round 4 tools/r03/conv_ab.py): the stride-2 convs, the first c1 of a
        # stage (Cin = 2 Cout), every layer4-sized grid, and the c3 of layer2/3 (round 4: with the packed
        # split, layer2 c3 and layer4's plain c1 moved here too: 6028-6044 -> 6114-6126 img/s, one box) --
        # faster per launch than gemm_x3 / the split pass + x3p there; elsewhere gemm_x3 or x3p stay ahead
        x3d = (_X3D and not nchw and not smallk and x3 and ci % 32 == 0 and Kd % 32 == 0 and (
            st == 2
            or (kh == 1 and in_ss is None and ci == 2 * co)
            or rows <= 3136
            or (kh == 1 and in_ss is not None and co == 4 * ci)))
        x3p = (not nchw and not smallk and not x3d and x3 and in_ss is not None
               and co >= 128
               and ci % 32 == 0 and Kd >= 128 and rows >= 12544 and a_elems * 6 < (1 << 31))
        # x3s (round 3): layer1's K = 64 1x1 convs (layer1.0 conv1 / downsample on the pooled stem, every
        # layer1 conv3 on relu(bn2(y2))) on the short-k streaming kernel (gemm_x3s.hip: weight in VGPRs,
        # persistent 64-row tiles, two workgroups per CU)
        x3s = (_X3S and x3 and not nchw and Kd == 64 and kh == 1 and st == 1 and pd == 0 and co in (64, 128, 256)
               and rows * co * 4 < (1 << 31))  # (its store-only epilogue addresses C with 32-bit offsets)
        if x3s:
            w3 = self._packed_x3(conv)
            if in_ss is None:
                prob, mode = K.problem(rows, co, Kd, x, ci, w3, Kd, out, co, **kw_), CAPMI_A_KMAJOR
            else:
                prob = K.problem(rows, co, Kd, x, 0, w3, Kd, out, co, conv=geo, in_scale=in_ss[0],
                                 in_shift=in_ss[1], **kw_)
                mode = CAPMI_A_CONV_NHWC
            launch = lambda: K.gemm_x3s(prob, mode)  # noqa: E731
            if self.conv_hook is not None:
                self.conv_hook(tag, 2.0 * rows * co * Kd, launch, K.gemm_x3s_kernel_name(prob, mode))
            else:
                launch()
            return Ho, Wo, rows
        x3c = (_X3C and x3 and not nchw and kh == 3 and kw == 3 and st == 1 and pd == 1 and co == 64
               and ci % 32 == 0 and W <= 64 and rows * co * 4 < (1 << 31))
        if x3c:
            w3 = self._packed_x3(conv, tap_inner=True)
            sc, sh = in_ss if in_ss is not None else (None, None)
            prob = K.problem(rows, co, Kd, x, 0, w3, Kd, out, co, conv=geo, in_scale=sc, in_shift=sh, **kw_)
            x3c = K.gemm_x3c_ok(prob)  # (the planner also bounds the staged band: many tiny images do not fit)
        if x3c:
            launch = lambda: K.gemm_x3c(prob)  # noqa: E731
            if self.conv_hook is not None:
                self.conv_hook(tag, 2.0 * rows * co * Kd, launch, K.gemm_x3c_kernel_name(prob))
            else:
                launch()
            return Ho, Wo, rows
        # the fp32 packed weight is fetched (and packed when stale) only by the routes that read it: the x3 routes
        # read their split planes, built from it only when those are rebuilt
        if nchw:
            w = self.packed.get(conv)
            # conv1: the NCHW images are re-laid out once as NHWC with 4 channels (one float4 per
            # pixel); the implicit GEMM then runs over k = (kh, kw, c4), the 4th channel zero
            img4 = self._ws["img4"]
            K.image_nhwc4(x, img4)
            K4 = kh * kw * 4
            geo["Cin"] = 4
            prob = K.problem(rows, co, K4, img4, 0, w, K4, out, co, conv=geo, **kw_)
            mode = CAPMI_A_CONV_NHWC4
        elif smallk:
            # short-k convs (layer1's K = 64): both operands split in-kernel on the 256-thread kernel
            # (CAPMI_GEMM_SPLIT3, two workgroups per CU overlap one's epilogue with the other's loads)
            sc, sh = in_ss if in_ss is not None else (None, None)
            w = self.packed.get(conv)
            if kh == 1 and st == 1 and in_ss is None:
                prob, mode = K.problem(rows, co, Kd, x, ci, w, Kd, out, co, **kw_), CAPMI_A_KMAJOR
            else:
                prob = K.problem(rows, co, Kd, x, 0, w, Kd, out, co, conv=geo, in_scale=sc, in_shift=sh, **kw_)
                mode = CAPMI_A_CONV_NHWC
            split3 = True
        elif x3d:
            w3 = self._packed_x3(conv, tap_inner=True)
            if kh == 1 and st == 1 and pd == 0:  # 1x1: dense rows, the BN prologue (if any) per k = channel
                sc, sh = in_ss if in_ss is not None else (None, None)
                prob = K.problem(rows, co, Kd, x, ci, w3, Kd, out, co, in_scale=sc, in_shift=sh, **kw_)
                mode = CAPMI_A_KMAJOR
            else:
                sc, sh = in_ss if in_ss is not None else (None, None)
                prob = K.problem(rows, co, Kd, x, 0, w3, Kd, out, co, conv=geo, in_scale=sc, in_shift=sh, **kw_)
                mode = CAPMI_A_CONV_NHWC
            launch = lambda: K.gemm_x3d(prob, mode, self._ws["sk"])  # noqa: E731
            if self.conv_hook is not None:
                self.conv_hook(tag, 2.0 * rows * co * Kd, launch, K.gemm_x3d_kernel_name(prob, mode))
            else:
                launch()
            return Ho, Wo, rows
        elif x3p:
            # x3p: the conv input relu(bn(y)) split once into three bf16 planes, then the GEMM with
            # both operands pre-split (gemm_x3p.hip). Where it pays (tools/x3_ab.py, batch 64): the
            # 3x3 convs of layer2/3 and the c3 convs of layer2/3 (their A tiles are re-staged 9x /
            # 4-8x); layer1's K = 64 c3 (no gain once the split pass is counted) and layer4's
            # 3136-row grids keep the in-kernel split (gemm_x3.hip)
            xp = self._x3p_buffer(self._ws)
            K.bn_relu_split3(x, in_ss[0], in_ss[1], N * H * W, ci, xp)
            w3 = self._packed_x3(conv, tap_inner=True)
            if kh == 1 and st == 1:
                prob, mode = K.problem(rows, co, Kd, xp, ci, w3, Kd, out, co, **kw_), CAPMI_A_KMAJOR
            else:
                prob, mode = K.problem(rows, co, Kd, xp, 0, w3, Kd, out, co, conv=geo, **kw_), CAPMI_A_CONV_NHWC
            launch = lambda: K.gemm_x3p(prob, mode, self._ws["sk"])  # noqa: E731
            if self.conv_hook is not None:
                self.conv_hook(tag, 2.0 * rows * co * Kd, launch, K.gemm_x3p_kernel_name(prob, mode))
            else:
                launch()
            return Ho, Wo, rows
        elif kh == 1 and st == 1 and in_ss is None:
            w = self._packed_x3(conv) if x3 and Kd % 32 == 0 else self.packed.get(conv)
            prob = K.problem(rows, co, Kd, x, ci, w, Kd, out, co, **kw_)
            mode = CAPMI_A_KMAJOR
        else:
            sc, sh = in_ss if in_ss is not None else (None, None)
            w = self._packed_x3(conv) if x3 and Kd % 32 == 0 and ci % 32 == 0 else self.packed.get(conv)
            prob = K.problem(rows, co, Kd, x, 0, w, Kd, out, co, conv=geo, in_scale=sc, in_shift=sh, **kw_)
            mode = CAPMI_A_CONV_NHWC
        if w.dtype == torch.bfloat16:  # the three-plane split weight: fp32-accurate x3 GEMM
            launch = lambda: K.gemm_x3(prob, mode, self._ws["sk"])  # noqa: E731
            if self.conv_hook is not None:
                self.conv_hook(tag, 2.0 * rows * co * Kd, launch, K.gemm_x3_kernel_name(prob, mode))
            else:
                launch()
            return Ho, Wo, rows
        # conv1 in the x3 mode: both operands split in-kernel (CAPMI_GEMM_SPLIT3; its K = 7*7*4 is
        # not the gemm_x3 kernel's multiple of 32)
        flags = CAPMI_GEMM_BF16 if self.bf16 else (CAPMI_GEMM_SPLIT3 if split3 else 0)
        launch = lambda: K.gemm_sk(prob, mode, self._ws["sk"], K.TILE_AUTO, flags=flags)  # noqa: E731
        if self.conv_hook is not None:
            key = K.gemm_sk_kernel_name(prob, mode, flags=flags)
            self.conv_hook(tag, 2.0 * rows * co * Kd, launch, key)
        else:
            launch()
        del stats
        return Ho, Wo, rows

    def _packed_x3(self, conv, tap_inner=False):
        """[3][Cout][K] bf16 split of the packed fp32 weight (B operand of gemm_x3; with ``tap_inner``
        in gemm_x3p's conv k order), refreshed when the weight tensor changes. The fused Adam writes the
        weights in place without bumping their version, so FineTuneRunner.forward refreshes the trainable
        convs' entries itself: the ones its batched job array covers in that launch, every other one (and
        the fp32 pack they are made from) dropped, to be rebuilt here from the current weights."""
        w = conv.weight
        key = ("x3p" if tap_inner else "x3", id(conv))
        ent = self.packed.cache.get(key)
        if ent is None or ent[0] != w._version or ent[1] != w.data_ptr():
            src = self.packed.get(conv)
            if tap_inner:
                co, ci, kh, kw = w.shape
                src = K.conv_weight_order_x3p(src, kh, kw, ci)
            src = src.contiguous()
            dst = torch.empty(3 * src.numel(), device=w.device, dtype=torch.bfloat16)
            K.split3_bf16(src, dst)
            ent = (w._version, w.data_ptr(), dst)
            self.packed.cache[key] = ent
        return ent[2]

    # ---- bf16 activations (BASELINE config 5) -------------------------------------------------
    def _packed_bf16(self, conv):
        """bf16 copy of the packed [Cout][KH][KW][Cin] weight, refreshed when the weight changes."""
        w = conv.weight
        key = ("bf16", id(conv))
        ent = self.packed.cache.get(key)
        if ent is None or ent[0] != w._version or ent[1] != w.data_ptr():
            src = self.packed.get(conv).contiguous()
            dst = torch.empty(src.shape, device=w.device, dtype=torch.bfloat16)
            K.f32_to_bf16(src, dst)
            ent = (w._version, w.data_ptr(), dst)
            self.packed.cache[key] = ent
        return ent[2]

    def _conv_bf16(self, tag, x, conv, out, N, H, W, train):
        """bf16 NHWC x -> bf16 NHWC out (CAPMI_GEMM_BF16_IO), BN statistics into ws['stats']; x is the conv
        input itself (relu(bn(y)) materialised in bf16 by capmi_bn_relu_bf16)."""
        co, ci, kh, kw = conv.weight.shape
        st, pd = conv.stride[0], conv.padding[0]
        Ho, Wo = (H + 2 * pd - kh) // st + 1, (W + 2 * pd - kw) // st + 1
        rows = N * Ho * Wo
        Kd = ci * kh * kw
        w = self._packed_bf16(conv)
        stats = self._ws["stats"] if train else None
        if kh == 1 and st == 1:
            prob, mode = K.problem_bf16(rows, co, Kd, x, ci, w, Kd, out, co, stats=stats), AK
        else:
            geo = dict(N=N, H=H, W=W, Cin=ci, KH=kh, KW=kw, stride=st, pad=pd, Ho=Ho, Wo=Wo)
            prob, mode = K.problem_bf16(rows, co, Kd, x, 0, w, Kd, out, co, stats=stats, conv=geo), AC
        launch = lambda: K.gemm_bf16(prob, mode, self._ws["sk"], K.TILE_AUTO)  # noqa: E731
        if self.conv_hook is not None:
            key = K.gemm_bf16_kernel_name(prob, mode)  # the launcher's own plan (gemm.hip bf16_io_plan)
            self.conv_hook(tag, 2.0 * rows * co * Kd, launch, key)
        else:
            launch()
        return Ho, Wo, rows

    def _bn_relu_bf16(self, ws, bn, rows, train, y):
        """relu(bn(y)) in place on a bf16 conv output (the next conv's input)."""
        s, b = self._bn(ws, bn, rows, train)
        K.bn_relu_bf16(y, s, b, rows, bn.num_features, y)

    def _forward_bf16(self, net, imgs, out_hw, train, out):
        """The conv stack on bf16 NHWC activations: every conv but conv1 on CAPMI_GEMM_BF16_IO (bf16
        operands, fp32 accumulation, bf16 output, fp32 BN statistics of the stored values), the BN
        apply + ReLU of each conv input materialised once in bf16 (capmi_bn_relu_bf16), bottleneck
        tails in bf16; conv1 (Cin = 3) reads the fp32 images with bf16 operand staging; the features
        come out fp32 (adaptive pool), as the decoder expects."""
        N, C0, H, W = imgs.shape
        ws = self._workspace(N, H, W, imgs.device)
        if "bf" not in ws:
            big = ws["x"].numel()
            ws["bf"] = {n: torch.empty(big, device=imgs.device, dtype=torch.bfloat16)
                        for n in ("x", "y1", "y2", "y3", "yd", "out")}
        bf = ws["bf"]
        H1, W1, rows = self._conv("conv1", imgs, net.conv1, ws["y1"], N, H, W, train, nchw=True)
        s, b = self._bn(ws, net.bn1, rows, train)
        Hp, Wp = (H1 + 2 - 3) // 2 + 1, (W1 + 2 - 3) // 2 + 1
        K.bn_relu_maxpool(ws["y1"], s, b, ws["x"], N, H1, W1, 64, Hp, Wp)
        K.f32_to_bf16(ws["x"][: N * Hp * Wp * 64], bf["x"])
        x, xo = bf["x"], bf["out"]
        H, W, Cx = Hp, Wp, 64
        bns = []
        for li in range(1, 5):
            for bi, blk in enumerate(getattr(net, f"layer{li}")):
                tag = f"layer{li}.{bi}"
                _, _, r1 = self._conv_bf16(tag + ".conv1", x, blk.conv1, bf["y1"], N, H, W, train)
                self._bn_relu_bf16(ws, blk.bn1, r1, train, bf["y1"])
                H2, W2, r2 = self._conv_bf16(tag + ".conv2", bf["y1"], blk.conv2, bf["y2"], N, H, W, train)
                self._bn_relu_bf16(ws, blk.bn2, r2, train, bf["y2"])
                _, _, r3 = self._conv_bf16(tag + ".conv3", bf["y2"], blk.conv3, bf["y3"], N, H2, W2, train)
                Cout = blk.conv3.out_channels
                if blk.downsample is not None:
                    s3, b3 = self._bn(ws, blk.bn3, r3, train)  # (the downsample conv reuses the stats buffer)
                    self._conv_bf16(tag + ".downsample", x, blk.downsample[0], bf["yd"], N, H, W, train)
                    sd, bd = self._bn(ws, blk.downsample[1], r3, train)
                    K.bn_add_relu_bf16(bf["y3"], s3, b3, bf["yd"], xo, r3, Cout, res_scale=sd, res_shift=bd)
                    bns.append(blk.downsample[1])
                else:
                    s3, b3 = self._bn(ws, blk.bn3, r3, train)
                    K.bn_add_relu_bf16(bf["y3"], s3, b3, x, xo, r3, Cout)
                bns += [blk.bn1, blk.bn2, blk.bn3]
                x, xo = xo, x
                H, W, Cx = H2, W2, Cout
        if train:
            bns.append(net.bn1)
            nbt = [m.num_batches_tracked for m in bns if m.num_batches_tracked is not None]
            if nbt:
                torch._foreach_add_(nbt, 1)
        # out_hw None: the layer4 map itself, converted to fp32 (an identity "pool")
        OH, OW = out_hw if out_hw is not None else (H, W)
        if out is None:
            out = torch.empty(N, OH, OW, Cx, device=imgs.device, dtype=torch.float32)
        K.adaptive_avgpool_bf16(x, N, H, W, Cx, OH, OW, out)
        return out

    @torch.no_grad()
    def forward(self, net, imgs, out_hw=(14, 14), train=True, out=None):
        """imgs (N,3,H,W) fp32 contiguous on the device -> (N, OH, OW, 2048) NHWC (= the
        reference's adaptive_pool + permute(0,2,3,1), models/encoder.py:107-110). out_hw=None:
        the layer4 map itself (N, H/32, W/32, 2048), written by the last block straight into
        ``out`` (the decoder's distinct rows when the pool only repeats pixels, feature_hw)."""
        if imgs.dtype != torch.float32 or not imgs.is_contiguous():
            raise TypeError("encoder input must be contiguous float32 (N,3,H,W)")
        N, C0, H, W = imgs.shape
        if self.bf16:
            return self._forward_bf16(net, imgs, out_hw, train, out)
        ws = self._workspace(N, H, W, imgs.device)
        # conv1 7x7/2 -> bn1 -> relu -> maxpool (children 0-3)
        H1, W1, rows = self._conv("conv1", imgs, net.conv1, ws["y1"], N, H, W, train, nchw=True)
        s, b = self._bn(ws, net.bn1, rows, train)
        Hp, Wp = (H1 + 2 - 3) // 2 + 1, (W1 + 2 - 3) // 2 + 1
        K.bn_relu_maxpool(ws["y1"], s, b, ws["x"], N, H1, W1, 64, Hp, Wp)
        x, xo = ws["x"], ws["out"]
        H, W, Cx = Hp, Wp, 64
        bns = []
        direct = out_hw is None and out is not None
        n4 = len(net.layer4)
        for li in range(1, 5):
            layer = getattr(net, f"layer{li}")
            for bi, blk in enumerate(layer):
                if direct and li == 4 and bi == n4 - 1:
                    xo = out  # the last block's output is the result
                tag = f"layer{li}.{bi}"
                _, _, r1 = self._conv(tag + ".conv1", x, blk.conv1, ws["y1"], N, H, W, train)
                ss1 = self._bn(ws, blk.bn1, r1, train)
                H2, W2, r2 = self._conv(tag + ".conv2", ws["y1"], blk.conv2, ws["y2"], N, H, W, train, in_ss=ss1)
                ss2 = self._bn(ws, blk.bn2, r2, train)
                _, _, r3 = self._conv(tag + ".conv3", ws["y2"], blk.conv3, ws["y3"], N, H2, W2, train, in_ss=ss2)
                Cout = blk.conv3.out_channels
                if blk.downsample is not None:
                    s3, b3 = self._bn(ws, blk.bn3, r3, train)  # (the downsample conv reuses the stats buffer)
                    self._conv(tag + ".downsample", x, blk.downsample[0], ws["yd"], N, H, W, train)
                    sd, bd = self._bn(ws, blk.downsample[1], r3, train)
                    K.bn_add_relu(ws["y3"], s3, b3, ws["yd"], xo, r3, Cout, res_scale=sd, res_shift=bd)
                    bns.append(blk.downsample[1])
                else:
                    s3, b3 = self._bn(ws, blk.bn3, r3, train)
                    K.bn_add_relu(ws["y3"], s3, b3, x, xo, r3, Cout)
                bns += [blk.bn1, blk.bn2, blk.bn3]
                x, xo = xo, x
                H, W, Cx = H2, W2, Cout
        if train:
            bns.append(net.bn1)
            nbt = [m.num_batches_tracked for m in bns if m.num_batches_tracked is not None]
            if nbt:
                torch._foreach_add_(nbt, 1)
        if out_hw is None:
            return x if direct else x[: N * H * W * Cx].view(N, H, W, Cx).clone()
        OH, OW = out_hw
        if out is None:
            out = torch.empty(N, OH, OW, Cx, device=imgs.device, dtype=torch.float32)
        K.adaptive_avgpool_nhwc(x, N, H, W, Cx, OH, OW, out)
        return out


def conv_flops_per_image(net, H=224, W=224):
    """Algorithmic FLOPs of the conv stack for one image (2*Ho*Wo*Cout*Cin*KH*KW summed)."""
    tot = 0
    h, w = H, W
    convs = [net.conv1]
    c = net.conv1
    h, w = (h + 6 - 7) // 2 + 1, (w + 6 - 7) // 2 + 1
    tot += 2 * h * w * c.out_channels * c.in_channels * 49
    h, w = (h + 2 - 3) // 2 + 1, (w + 2 - 3) // 2 + 1
    for li in range(1, 5):
        for blk in getattr(net, f"layer{li}"):
            tot += 2 * h * w * blk.conv1.out_channels * blk.conv1.in_channels
            s = blk.conv2.stride[0]
            h2, w2 = (h + 2 - 3) // s + 1, (w + 2 - 3) // s + 1
            tot += 2 * h2 * w2 * blk.conv2.out_channels * blk.conv2.in_channels * 9
            tot += 2 * h2 * w2 * blk.conv3.out_channels * blk.conv3.in_channels
            if blk.downsample is not None:
                d = blk.downsample[0]
                tot += 2 * h2 * w2 * d.out_channels * d.in_channels
            h, w = h2, w2
    del convs
    return tot


# ======================================================================================
# fine-tune: forward that keeps the trainable stages' activations, and their backward
# ======================================================================================
class _Pool:
    """Named device buffers, allocated once per (name, numel) and reused every step."""

    def __init__(self):
        self.bufs = {}

    def get(self, name, n, device, dtype=torch.float32):
        t = self.bufs.get(name)
        if t is None or t.numel() < n or t.device != torch.device(device) or t.dtype != dtype:
            t = torch.empty(n, device=device, dtype=dtype)
            self.bufs[name] = t
        return t[:n]


_FT_DGRAD_X3 = os.environ.get("CAPMI_FT_DGRAD_X3", "1") != "0"
_FT_WGRAD_X3 = os.environ.get("CAPMI_FT_WGRAD_X3", "1") != "0"
# x3 mode: 3x3 / sub-pixel data gradients on x3d (dY split in registers x the x3p-ordered split of
# the packed dgrad weight, re-split every step) instead of the split-staging nts form
_FT_DGRAD_X3D = os.environ.get("CAPMI_FT_DGRAD_X3D", "1") != "0"
# the 3x3 dgrad weight packed, ordered and split in one kernel (0: three passes, A/B)
_FT_PACK_X3 = os.environ.get("CAPMI_FT_PACK_X3", "1") != "0"
# 1x1 dgrads read the weight itself as k rows (CAPMI_B_KROWS) instead of a per-step transposed pack
_FT_DGRAD1_KROWS = os.environ.get("CAPMI_FT_DGRAD1_KROWS", "0") != "0"
# 1x1 dgrads on x3d: neutral in round 2 (1666 both); with the store-only / beta epilogue
# 1676-1680 -> 1711-1716 img/s (two pairs, one box): on
_FT_DGRAD1_X3D = os.environ.get("CAPMI_FT_DGRAD1_X3D", "1") != "0"
# of those, the long-k ones (K >= 4 N: conv3's) on gemm_x3 instead of x3d (CAPMI_FT_DGRAD1_X3=0: all x3d)
_FT_DGRAD1_X3 = os.environ.get("CAPMI_FT_DGRAD1_X3", "1") != "0"
# x3 mode: the weight gradients on the x3w kernel (round 4: both fp32 operands split in-kernel, transposed
# LDS reads, k-split slabs; CAPMI_FT_WGRAD_X3W=0: the split-staging nts kernel)
_FT_WGRAD_X3W = os.environ.get("CAPMI_FT_WGRAD_X3W", "1") != "0"
# round 5: every trainable conv's three-plane weights (forward B planes, data-gradient planes) refreshed by ONE
# capmi_weight_x3_batch launch per step, from the second step on (the first records what the step uses);
# CAPMI_FT_WPREP_BATCH=0: the per-conv packs and splits (A/B)
_FT_WPREP_BATCH = os.environ.get("CAPMI_FT_WPREP_BATCH", "1") != "0"
# round 6 (opt-in): the weight gradients on a second HIP stream beside the data-gradient chain (they are off its
# critical path: nothing in the chain reads them), their inputs double-buffered by block parity so the chain waits
# only for the weight gradients of two blocks back. CAPMI_FT_WGRAD_SIDE=1: the side stream at the high end of the
# priority range (the chain on the caller's stream); "lo": at the low end. Off by default: measured slower (DESIGN
# 4.23) -- the chain's stream-K data gradients hand partials between co-resident workgroups, and a weight gradient
# holding CUs beside them leaves owners spinning for producers that have no CU yet
_FT_WGRAD_SIDE = os.environ.get("CAPMI_FT_WGRAD_SIDE", "0")


class FineTuneRunner:
    """EncoderAttention.fine_tune(True) (models/encoder.py:112-121): layer2, layer3 and layer4
    (children()[5:]) are trainable, BatchNorm stays in train mode (batch statistics).

    ``forward`` runs the same fused conv stack as EncoderRunner but writes every trainable
    block's tensors (raw conv outputs y1/y2/y3/yd, block output, BN batch mean/var) into
    buffers that live until ``backward``. ``backward`` walks the trainable blocks in reverse:
    BN(train)+ReLU backward as reduce + apply kernels, conv weight gradients as
    dY^T x im2col(X) GEMMs (the conv input re-derived from the saved pre-BN output through the
    GEMM's BN-apply+ReLU prologue), data gradients as convs of dY with flipped weights
    (zero-upsampled dY for the stride-2 3x3 convs, a strided-row GEMM store for the stride-2
    downsample), residual gradients accumulated by the GEMM epilogue (beta = 1)."""

    def __init__(self, runner, first_layer=2):
        self.r = runner
        self.first = first_layer
        self.saved = _Pool()
        self.grad = _Pool()
        self.state = None
        # batched weight preparation (_FT_WPREP_BATCH): per (weight, ph, pw) the data-gradient planes, the job
        # specs recorded on the first step, their device array once built
        self._dgrad_x3 = {}
        self._wx3_specs = []
        self._wx3 = None
        self._wx3_n = 0  # jobs in the device array (fixed when it is built)
        self._wx3_fwd = {}  # cache key -> the forward planes buffer the array refreshes
        # weight gradients beside the data-gradient chain (_FT_WGRAD_SIDE); None: one stream
        self.wgrad_side = _FT_WGRAD_SIDE != "0"
        self._side = None
        self._side_ws = None

    # ------------------------------------------------------------------ forward
    def _bn_save(self, ws, bn, rows):
        s, b = self.r._ss(ws, bn)
        C = bn.num_features
        ms = self.saved.get(f"ms.{id(bn)}", 2 * C, bn.weight.device).view(2, C)
        mom = 0.1 if bn.momentum is None else bn.momentum
        K.bn_finalize(ws["stats"], K.stat_tiles(rows), C, rows, bn.weight, bn.bias,
                      bn.running_mean if bn.track_running_stats else None,
                      bn.running_var if bn.track_running_stats else None, mom, bn.eps, s, b,
                      ws["bnwork"], save_mean=ms[0], save_var=ms[1])
        return s, b, ms

    @torch.no_grad()
    def forward(self, net, imgs, out_hw=(14, 14), out=None):
        r = self.r
        if imgs.dtype != torch.float32 or not imgs.is_contiguous():
            raise TypeError("encoder input must be contiguous float32 (N,3,H,W)")
        N, _, H, W = imgs.shape
        dev = imgs.device
        ws = r._workspace(N, H, W, dev)
        # the optimizer updates trainable weights in place (same storage, same _version): refresh every
        # trainable conv's planes in one launch (the cache entries keep their buffers), or drop the packed copies
        # so this forward re-packs them
        # Entries the job array does not refresh are dropped every step, whichever route created them: the fp32
        # [Cout][KH][KW][Cin] pack of every trainable 3x3 (the source a rebuilt split is made from) and any split
        # entry created after the array was built (a batch or image size that routes a conv differently, e.g. a
        # ragged last batch, or a weight whose storage moved) -- those are rebuilt from the current weights
        # whenever a forward uses them.
        if self._wx3 is not None:
            K.weight_x3_batch(self._wx3, self._wx3_n)
        for li in range(self.first, 5):
            for blk in getattr(net, f"layer{li}"):
                r.packed.cache.pop(id(blk.conv2), None)
                convs = [blk.conv1, blk.conv2, blk.conv3] + ([blk.downsample[0]] if blk.downsample is not None else [])
                for c in convs:
                    for key in (("x3", id(c)), ("x3p", id(c))):
                        ent = r.packed.cache.get(key)
                        if ent is not None and self._wx3_fwd.get(key) is not ent[2]:
                            del r.packed.cache[key]
        H1, W1, rows = r._conv("conv1", imgs, net.conv1, ws["y1"], N, H, W, True, nchw=True)
        s, b = r._bn(ws, net.bn1, rows, True)
        Hp, Wp = (H1 + 2 - 3) // 2 + 1, (W1 + 2 - 3) // 2 + 1
        K.bn_relu_maxpool(ws["y1"], s, b, ws["x"], N, H1, W1, 64, Hp, Wp)
        x, xo = ws["x"], ws["out"]
        H, W, Cx = Hp, Wp, 64
        bns = [net.bn1]
        blocks = []
        for li in range(1, 5):
            for bi, blk in enumerate(getattr(net, f"layer{li}")):
                tag = f"layer{li}.{bi}"
                wd, Cout = blk.conv1.out_channels, blk.conv3.out_channels
                st = blk.conv2.stride[0]
                H2, W2 = (H + 2 - 3) // st + 1, (W + 2 - 3) // st + 1
                r1, r3 = N * H * W, N * H2 * W2
                if li < self.first:  # frozen stage: rotating workspace buffers
                    y1, y2, y3, yd, o = ws["y1"], ws["y2"], ws["y3"], ws["yd"], xo
                else:
                    g = self.saved.get
                    y1 = g(tag + ".y1", r1 * wd, dev)
                    y2 = g(tag + ".y2", r3 * wd, dev)
                    y3 = g(tag + ".y3", r3 * Cout, dev)
                    yd = g(tag + ".yd", r3 * Cout, dev) if blk.downsample is not None else None
                    o = g(tag + ".out", r3 * Cout, dev)
                trainable = li >= self.first
                bnf = (lambda bn, rows: self._bn_save(ws, bn, rows)) if trainable else \
                    (lambda bn, rows: r._bn(ws, bn, rows, True) + (None,))
                r._conv(tag + ".conv1", x, blk.conv1, y1, N, H, W, True)
                s1, b1, m1 = bnf(blk.bn1, r1)
                r._conv(tag + ".conv2", y1, blk.conv2, y2, N, H, W, True, in_ss=(s1, b1))
                s2, b2, m2 = bnf(blk.bn2, r3)
                r._conv(tag + ".conv3", y2, blk.conv3, y3, N, H2, W2, True, in_ss=(s2, b2))
                s3, b3, m3 = bnf(blk.bn3, r3)
                md = sd = bd = None
                if blk.downsample is not None:
                    r._conv(tag + ".downsample", x, blk.downsample[0], yd, N, H, W, True)
                    sd, bd, md = bnf(blk.downsample[1], r3)
                    K.bn_add_relu(y3, s3, b3, yd, o, r3, Cout, res_scale=sd, res_shift=bd)
                    bns.append(blk.downsample[1])
                else:
                    K.bn_add_relu(y3, s3, b3, x, o, r3, Cout)
                bns += [blk.bn1, blk.bn2, blk.bn3]
                if trainable:
                    blocks.append(dict(blk=blk, tag=tag, li=li, x=x, Cin=Cx, H=H, W=W, H2=H2, W2=W2, wd=wd, Cout=Cout,
                                       stride=st, y1=y1, y2=y2, y3=y3, yd=yd, out=o,
                                       ss=[(s1, b1, m1), (s2, b2, m2), (s3, b3, m3), (sd, bd, md)]))
                    x = o
                else:
                    x, xo = o, x
                H, W, Cx = H2, W2, Cout
        nbt = [m.num_batches_tracked for m in bns if m.num_batches_tracked is not None]
        if nbt:
            torch._foreach_add_(nbt, 1)
        # out_hw None: the layer4 map itself (identity pool: a copy; its backward a copy too)
        OH, OW = out_hw if out_hw is not None else (H, W)
        if out is None:
            out = torch.empty(N, OH, OW, Cx, device=dev, dtype=torch.float32)
        K.adaptive_avgpool_nhwc(x, N, H, W, Cx, OH, OW, out)
        self.state = dict(N=N, H=H, W=W, C=Cx, OH=OH, OW=OW, blocks=blocks, device=dev)
        return out

    # ------------------------------------------------------------------ backward
    def _flags(self, prob, amode, bmode):
        """In the x3 mode the backward GEMMs run the fp32-accurate three-term split (CAPMI_GEMM_SPLIT3):
        the data gradients (convs of dY / 1x1 GEMMs on the transposed weight) and the weight gradients
        (CAPMI_FT_WGRAD_X3=0: those fp32). CAPMI_FT_DGRAD_X3=0: all fp32."""
        if not (self.r.x3 and _FT_DGRAD_X3):
            return 0
        if bmode == CAPMI_B_NMAJOR_W and amode in (CAPMI_A_KMAJOR, CAPMI_A_CONV_NHWC) and not prob.in_scale:
            return CAPMI_GEMM_SPLIT3
        if bmode == CAPMI_B_KROWS and amode == CAPMI_A_KMAJOR:  # 1x1 dgrads on the weight itself
            return CAPMI_GEMM_SPLIT3
        if amode == CAPMI_A_MMAJOR and bmode in (CAPMI_B_KROWS, CAPMI_B_CONV_NHWC) and _FT_WGRAD_X3:
            # weight gradients dY^T X: on a materialised input (k rows) or the implicit im2col of the
            # saved pre-BN output with the BN-apply + ReLU prologue
            return CAPMI_GEMM_SPLIT3
        return 0

    def _gemm(self, prob, amode, bmode, tile=K.TILE_AUTO, ws=None):
        K.gemm_sk(prob, amode, self.r._ws["sk"] if ws is None else ws, tile, bmode,
                  flags=self._flags(prob, amode, bmode))

    @torch.no_grad()
    def backward(self, dfeat, grads, hook=None, on_layer=None):
        """dfeat: (N, OH, OW, 2048) gradient of the features. grads: dict id(param) -> tensor
        receiving d(loss)/d(param) (conv weights in nn.Conv2d layout, BN weight/bias); missing
        entries are skipped. ``hook(tag, flops, launch, key)`` optionally wraps every conv GEMM.
        ``on_layer(li)`` is called (in stream order) as soon as stage li's gradients are final --
        after its first block, before the next stage's backward is launched: layer4, layer3,
        layer2 -- so a data-parallel step can all-reduce each stage's bucket beside the rest of
        the backward (nothing launched after the call reads or writes stage li's gradients)."""
        stt = self.state
        if stt is None:
            raise RuntimeError("FineTuneRunner.backward without a saved forward")
        N, dev = stt["N"], stt["device"]
        if hook is None:
            hook = self.r.conv_hook  # bench timing of the backward GEMMs (None: plain launches)
        gp = self.grad.get
        blocks = stt["blocks"]
        big = max(b["H"] * b["W"] * max(b["Cin"], b["Cout"], b["wd"]) for b in blocks) * N
        dA = [gp("dA0", big, dev), gp("dA1", big, dev)]
        # two streams (weight gradients beside the chain) only without the timing hook: the bench's roofline pass
        # times each GEMM alone on the chip
        two = self.wgrad_side and hook is None and dev.type == "cuda"
        main = torch.cuda.current_stream(dev) if two else None
        if two and self._side is None:
            lo, hi = torch.cuda.Stream.priority_range()
            self._side = torch.cuda.Stream(device=dev, priority=lo if _FT_WGRAD_SIDE == "lo" else hi)
            self._side_ws = K.gemm_workspace(dev)
        side_done = []  # per block (in backward order): event after its weight gradients on the side stream
        joined = 0  # side_done[:joined] are behind a join of the chain (no wait needed; across graph segments none is
        # allowed: an event recorded in one capture cannot be waited on in another)
        # the chain's buffers the weight gradients read (dy3, dmid = da2, da1, dyd): one set per block parity with
        # two streams, so block j's chain only waits for the weight gradients of block j - 2
        npar = 2 if two else 1
        dmid_p = [gp(f"dmid{i}", big, dev) for i in range(npar)]
        dy3_p = [gp(f"dy3{i}", big, dev) for i in range(npar)]
        dyd_p = [gp(f"dyd{i}", big, dev) for i in range(npar)]
        da1_p = [gp(f"da1{i}", big, dev) for i in range(npar)] if two else dy3_p  # (one stream: da1 reuses dy3)
        wmax = max(b["wd"] * 9 * b["wd"] for b in blocks)
        dwp = gp("dw_packed", wmax, dev)
        wdg = gp("w_dgrad", wmax, dev)
        # 1x1 dgrads read the weight transposed (B = W^T[n][k], CAPMI_B_NMAJOR_W), packed per step
        # by conv_weight_pack_dgrad: that opens the 512-thread 128x128 form and the row-major B
        # path, 10-15 % faster per launch than the k-rows B form on every layer2-4 1x1 dgrad
        # (tools/bwd_gemm_ab.py); one buffer, reused in stream order
        w1max = max(max(b["Cout"] * b["wd"], b["wd"] * b["Cin"], b["Cout"] * b["Cin"]) for b in blocks)
        wt = gp("w1x1_t", w1max, dev)
        coef = gp("coef", 2 * 4 * 2048, dev).view(2, 4 * 2048)
        work = gp("bnwork", K.bnb_work_floats(2048), dev)

        def G(p):
            return grads.get(id(p))

        def run(tag, flops, prob, amode, bmode, tile=K.TILE_AUTO, ws=None):
            if amode == AMM and self.r.x3 and _FT_WGRAD_X3W and K.gemm_x3w_ok(prob, bmode):
                wsk = self.r._ws["sk"] if ws is None else ws
                launch = lambda: K.gemm_x3w(prob, bmode, wsk)  # noqa: E731
                if hook is None:
                    launch()
                else:
                    hook(tag, flops, launch, K.gemm_x3w_kernel_name(prob, bmode))
                return
            if hook is None:
                self._gemm(prob, amode, bmode, tile, ws)
            else:
                hook(tag, flops, lambda: self._gemm(prob, amode, bmode, tile, ws),
                     K.gemm_sk_kernel_name(prob, amode, bmode, tile=tile, flags=self._flags(prob, amode, bmode)))

        x3d = self.r.x3 and _FT_DGRAD_X3 and _FT_DGRAD_X3D
        x3d1 = self.r.x3 and _FT_DGRAD_X3 and _FT_DGRAD1_X3D
        if x3d or x3d1:
            word = gp("w_dgrad_ord", max(wmax, w1max), dev)
            w3 = gp("w_dgrad_x3", 3 * max(wmax, w1max), dev, dtype=torch.bfloat16)

        def run_dgrad(tag, flops, prob, w, kh=1, kw=1, cin=None, conv_w=None, ph=-1, pw=-1, w1=None):
            """Data gradient with B = the packed dgrad weight w ([N][K]); A = dY (3x3 / sub-pixel:
            through the implicit im2col, kh x kw taps of cin channels). x3 mode: x3d on w re-ordered
            to the x3p k order and split (CAPMI_FT_DGRAD_X3D / CAPMI_FT_DGRAD1_X3D for the 1x1s); for
            a 3x3 conv_w (the nn.Conv2d weight) is packed, ordered and split in one pass instead. w1: a 1x1
            conv's weight, packed transposed into w here. With the batched weight preparation the split planes
            of conv_w / w1 are the ones the forward's capmi_weight_x3_batch launch refreshed (the first step
            computes them per conv into their own buffer and records the job)."""
            n, kd = prob.N, prob.K
            conv = kh * kw > 1 or cin is not None
            amode = AC if conv else AK
            use = (x3d if conv else x3d1) and kd % 32 == 0 and (not conv or cin % 32 == 0)
            batch = _FT_WPREP_BATCH and use and ((conv_w is not None and _FT_PACK_X3) or w1 is not None)
            key = ((conv_w if conv_w is not None else w1).data_ptr(), ph, pw) if batch else None
            planes = self._dgrad_x3.get(key) if batch else None
            # jobs are recorded only before the array is built; a key it does not cover (a weight whose storage
            # moved) takes the per-conv path into the shared scratch planes from then on
            record = batch and self._wx3 is None
            if planes is not None and self._wx3 is not None:
                prob.B = planes.data_ptr()  # refreshed this step by the forward's batched launch
                conv_w = w1 = None
            else:
                if w1 is not None:
                    K.conv_weight_pack_dgrad(w1, w[:n * kd])
                if conv_w is not None and not (use and _FT_PACK_X3):  # the fp32 pack
                    if ph < 0:
                        K.conv_weight_pack_dgrad(conv_w, w[:n * kd])
                    else:
                        K.conv_weight_pack_dgrad_s2(conv_w, ph, pw, w[:n * kd])
                    conv_w = None
                if not use:
                    return run(tag, flops, prob, amode, BW)
                dst = w3
                if record:  # first step: this conv's own planes, recorded as a job of the batched launch
                    dst = self._dgrad_x3.get(key)
                    if dst is None:
                        dst = torch.empty(3 * n * kd, device=dev, dtype=torch.bfloat16)
                        self._dgrad_x3[key] = dst
                        src = conv_w if conv_w is not None else w1
                        self._wx3_specs.append((src, dst, K.WX3_DGRAD if conv_w is not None else K.WX3_DGRAD_T, ph, pw))
                if conv_w is not None:
                    K.conv_weight_pack_dgrad_x3(conv_w, dst[:3 * n * kd], ph, pw)
                else:
                    src = w[:n * kd].view(n, kd)
                    if kh * kw > 1:
                        word[:n * kd].view(n, kd).copy_(K.conv_weight_order_x3p(src, kh, kw, cin))
                        src = word[:n * kd]
                    K.split3_bf16(src, dst[:3 * n * kd])
                prob.B = dst.data_ptr()
            if not conv and _FT_DGRAD1_X3 and kd >= 4 * n and prob.c_r1 <= 0:
                # long-k 1x1 data gradients (conv3's: K = 4 N) on gemm_x3 (the same split planes; 1x1: plain k
                # order), as the forward's long-k plain c1 convs
                launch = lambda: K.gemm_x3(prob, amode, self.r._ws["sk"])  # noqa: E731
                name = K.gemm_x3_kernel_name(prob, amode)
            else:
                launch = lambda: K.gemm_x3d(prob, amode, self.r._ws["sk"])  # noqa: E731
                name = K.gemm_x3d_kernel_name(prob, amode)
            if hook is None:
                launch()
            else:
                hook(tag, flops, launch, name)

        def wgrad(fn):
            """A weight gradient (and what finishes it): on the side stream after everything the chain has
            launched so far (its inputs), else inline."""
            if not two:
                fn()
                return
            self._side.wait_stream(main)
            with torch.cuda.stream(self._side):
                fn()

        K.adaptive_avgpool_bwd_nhwc(dfeat.contiguous(), N, stt["H"], stt["W"], stt["C"], stt["OH"], stt["OW"],
                                    dA[0])
        cur = 0
        wsw = self._side_ws if two else None
        for bi in range(len(blocks) - 1, -1, -1):
            b = blocks[bi]
            j = len(blocks) - 1 - bi  # blocks done before this one
            par = j % npar
            if two and j >= 2 and j - 2 >= joined:  # this block's buffers were read by block j - 2's weight gradients
                main.wait_event(side_done[j - 2])
            dmid, dy3, dyd, da1buf = dmid_p[par], dy3_p[par], dyd_p[par], da1_p[par]
            blk, tag = b["blk"], b["tag"]
            H, W, H2, W2, s = b["H"], b["W"], b["H2"], b["W2"], b["stride"]
            Cin, wd, Cout = b["Cin"], b["wd"], b["Cout"]
            r1, r3 = N * H * W, N * H2 * W2
            (s1, b1, m1), (s2, b2, m2), (s3, b3, m3), (sd, bd, md) = b["ss"]
            dout = dA[cur]
            need_dx = bi > 0
            dx = dA[cur ^ 1] if need_dx else None
            ds = blk.downsample
            # ---- tail: out = relu(bn3(y3) + res)
            bn3 = blk.bn3
            K.bn_bwd_reduce(K.BNB_RELU_OUT, dout, b["y3"], b["out"], None, None, bn3.weight, m3[0], m3[1],
                            bn3.eps, r3, Cout, G(bn3.weight), G(bn3.bias), coef[0], work)
            if ds is not None:
                bnd = ds[1]
                K.bn_bwd_reduce(K.BNB_RELU_OUT, dout, b["yd"], b["out"], None, None, bnd.weight, md[0], md[1],
                                bnd.eps, r3, Cout, G(bnd.weight), G(bnd.bias), coef[1], work)
                K.bn_bwd_apply(K.BNB_RELU_OUT, dout, b["yd"], b["out"], None, None, coef[1], r3, Cout, dyd)
            K.bn_bwd_apply(K.BNB_RELU_OUT, dout, b["y3"], b["out"], None, None, coef[0], r3, Cout, dy3,
                           dz_out=dx if (need_dx and ds is None) else None)
            # ---- conv3 (1x1): input relu(bn2(y2)) through the prologue
            c3 = blk.conv3
            geo3 = dict(N=N, H=H2, W=W2, Cin=wd, KH=1, KW=1, stride=1, pad=0, Ho=H2, Wo=W2)
            if G(c3.weight) is not None:
                wgrad(lambda: run(tag + ".conv3.wgrad", 2.0 * r3 * Cout * wd,
                                  K.problem(Cout, wd, r3, dy3, Cout, b["y2"], 0, G(c3.weight), wd, conv=geo3,
                                            in_scale=s2, in_shift=b2), AMM, BCONV, ws=wsw))
            da2 = dmid[:r3 * wd]
            if _FT_DGRAD1_KROWS:
                run(tag + ".conv3.dgrad", 2.0 * r3 * Cout * wd,
                    K.problem(r3, wd, Cout, dy3, Cout, c3.weight.detach(), wd, da2, wd), AK, BKR)
            else:
                run_dgrad(tag + ".conv3.dgrad", 2.0 * r3 * Cout * wd,
                          K.problem(r3, wd, Cout, dy3, Cout, wt, Cout, da2, wd), wt, w1=c3.weight.detach())
            # ---- bn2 + relu
            bn2 = blk.bn2
            K.bn_bwd_reduce(K.BNB_RELU_Y, da2, b["y2"], None, s2, b2, bn2.weight, m2[0], m2[1], bn2.eps, r3, wd,
                            G(bn2.weight), G(bn2.bias), coef[0], work)
            K.bn_bwd_apply(K.BNB_RELU_Y, da2, b["y2"], None, s2, b2, coef[0], r3, wd, da2)
            # ---- conv2 (3x3, stride s): input relu(bn1(y1)) through the prologue
            c2 = blk.conv2
            geo2 = dict(N=N, H=H, W=W, Cin=wd, KH=3, KW=3, stride=s, pad=1, Ho=H2, Wo=W2)
            if G(c2.weight) is not None:
                def c2w():
                    run(tag + ".conv2.wgrad", 2.0 * r3 * wd * 9 * wd,
                        K.problem(wd, 9 * wd, r3, da2, wd, b["y1"], 0, dwp, 9 * wd, conv=geo2, in_scale=s1,
                                  in_shift=b1), AMM, BCONV, ws=wsw)
                    K.conv_weight_unpack(dwp, tuple(c2.weight.shape), G(c2.weight))
                wgrad(c2w)
            da1 = da1buf[:r1 * wd]  # (one stream: dy3, consumed)
            if s == 1:
                geod = dict(N=N, H=H, W=W, Cin=wd, KH=3, KW=3, stride=1, pad=1, Ho=H, Wo=W)
                run_dgrad(tag + ".conv2.dgrad", 2.0 * r3 * wd * 9 * wd,
                          K.problem(r1, wd, 9 * wd, da2, 0, wdg, 9 * wd, da1, wd, conv=geod), wdg, 3, 3, wd,
                          conv_w=c2.weight.detach().contiguous())
            else:
                # sub-pixel form: input pixel (2i+ph, 2j+pw) is a (ph+1)x(pw+1) stride-1 pad-0 conv of
                # dY (9 taps over the 4 classes, vs 36 on a zero-upsampled grid); the class's rows
                # land at stride 2 through the output remap (H = 2*H2, W = 2*W2)
                assert H == 2 * H2 and W == 2 * W2
                for ph in (0, 1):
                    for pw in (0, 1):
                        th, tw = ph + 1, pw + 1
                        kk = th * tw * wd
                        geoc = dict(N=N, H=H2, W=W2, Cin=wd, KH=th, KW=tw, stride=1, pad=0, Ho=H2, Wo=W2)
                        run_dgrad(tag + f".conv2.dgrad.p{ph}{pw}", 2.0 * r3 * wd * kk,
                                  K.problem(r3, wd, kk, da2, 0, wdg, kk, da1[(ph * W + pw) * wd:], 2 * wd,
                                            conv=geoc, c_r1=W2, c_s2=2 * W * wd), wdg, th, tw, wd,
                                  conv_w=c2.weight.detach().contiguous(), ph=ph, pw=pw)
            # ---- bn1 + relu
            bn1 = blk.bn1
            K.bn_bwd_reduce(K.BNB_RELU_Y, da1, b["y1"], None, s1, b1, bn1.weight, m1[0], m1[1], bn1.eps, r1, wd,
                            G(bn1.weight), G(bn1.bias), coef[0], work)
            K.bn_bwd_apply(K.BNB_RELU_Y, da1, b["y1"], None, s1, b1, coef[0], r1, wd, da1)
            # ---- conv1 (1x1) on the block input x
            c1 = blk.conv1
            if G(c1.weight) is not None:
                wgrad(lambda: run(tag + ".conv1.wgrad", 2.0 * r1 * wd * Cin,
                                  K.problem(wd, Cin, r1, da1, wd, b["x"], Cin, G(c1.weight), Cin), AMM, BKR, ws=wsw))
            if need_dx:
                if _FT_DGRAD1_KROWS:
                    run(tag + ".conv1.dgrad", 2.0 * r1 * wd * Cin,
                        K.problem(r1, Cin, wd, da1, wd, c1.weight.detach(), Cin, dx, Cin,
                                  beta=1.0 if ds is None else 0.0), AK, BKR)
                else:
                    run_dgrad(tag + ".conv1.dgrad", 2.0 * r1 * wd * Cin,
                              K.problem(r1, Cin, wd, da1, wd, wt, wd, dx, Cin, beta=1.0 if ds is None else 0.0), wt,
                              w1=c1.weight.detach())
            # ---- downsample (1x1, stride s) on x
            if ds is not None:
                cd = ds[0]
                geodn = dict(N=N, H=H, W=W, Cin=Cin, KH=1, KW=1, stride=s, pad=0, Ho=H2, Wo=W2)
                if G(cd.weight) is not None:
                    wgrad(lambda: run(tag + ".downsample.wgrad", 2.0 * r3 * Cout * Cin,
                                      K.problem(Cout, Cin, r3, dyd, Cout, b["x"], 0, G(cd.weight), Cin, conv=geodn),
                                      AMM, BCONV, ws=wsw))
                if need_dx:
                    # dX[n, s*i, s*j, :] += dYd[n, i, j, :] W_d  (rows (n, i, j) -> strided NHWC rows)
                    rm = dict(c_r1=W2, c_s2=s * W * Cin) if s > 1 else {}
                    if _FT_DGRAD1_KROWS:
                        run(tag + ".downsample.dgrad", 2.0 * r3 * Cout * Cin,
                            K.problem(r3, Cin, Cout, dyd, Cout, cd.weight.detach(), Cin, dx, s * Cin, beta=1.0, **rm),
                            AK, BKR)
                    else:
                        run_dgrad(tag + ".downsample.dgrad", 2.0 * r3 * Cout * Cin,
                                  K.problem(r3, Cin, Cout, dyd, Cout, wt, Cout, dx, s * Cin, beta=1.0, **rm), wt,
                                  w1=cd.weight.detach())
            cur ^= 1
            if two:
                side_done.append(torch.cuda.Event())
                side_done[-1].record(self._side)
            if on_layer is not None and (bi == 0 or blocks[bi - 1]["li"] != b["li"]):
                if two:  # the stage's weight gradients are final once the side stream's work so far is
                    main.wait_stream(self._side)
                    joined = len(side_done)
                on_layer(b["li"])
        if two:  # join: the caller's stream sees every gradient (and a graph capture ends joined)
            main.wait_stream(self._side)
        self.state = None
        if _FT_WPREP_BATCH and self._wx3 is None and self.r.x3:
            self._build_wx3(stt)

    def _build_wx3(self, stt):
        """After the first step: the batched weight preparation's job array -- the forward's three-plane
        weights of every trainable conv (the cache entries this step created, refreshed in place from now on)
        and the data-gradient planes run_dgrad recorded."""
        specs = list(self._wx3_specs)
        fwd = {}
        for b in stt["blocks"]:
            blk = b["blk"]
            convs = [blk.conv1, blk.conv2, blk.conv3] + ([blk.downsample[0]] if blk.downsample is not None else [])
            for c in convs:
                for tag, mode in (("x3", K.WX3_FWD), ("x3p", K.WX3_FWD_X3P)):
                    ent = self.r.packed.cache.get((tag, id(c)))
                    if ent is not None:
                        specs.append((c.weight.detach(), ent[2], mode, -1, -1))
                        fwd[(tag, id(c))] = ent[2]
        if specs:
            self._wx3_specs = specs
            self._wx3_fwd = fwd
            self._wx3_n = len(specs)
            self._wx3 = K.wx3_jobs(specs, stt["device"])


def trainable_encoder_params(net, first_layer=2):
    """Parameters of layer{first_layer}..layer4 (children()[5:] for first_layer = 2)."""
    ps = []
    for li in range(first_layer, 5):
        ps += list(getattr(net, f"layer{li}").parameters())
    return ps
