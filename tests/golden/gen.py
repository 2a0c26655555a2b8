"""Deterministic, version-stable generators for parity inputs and weights.

TEST INFRASTRUCTURE. Used by ``make_golden.py`` (run once, in the survey
container, against the real reference) and by the tests (here and on the GPU
box) to rebuild exactly the same inputs and weights from a seed, so the
committed fixtures only need to hold seeds, dims and outputs.

Every tensor is drawn from its own ``numpy.random.default_rng([seed, tag])``
stream (PCG64 is stable across numpy versions), so adding or resizing one
tensor never shifts another.
"""
import zlib

import numpy as np

ENCODER_DIM = 2048  # models/attention.py:88 ("Set in stone")

IMG_MEAN = np.array([0.485, 0.456, 0.406], np.float32)  # models/attention.py:300
IMG_STD = np.array([0.229, 0.224, 0.225], np.float32)   # models/attention.py:301


def _rng(seed, name):
    return np.random.default_rng([int(seed), zlib.crc32(name.encode())])


def uniform(seed, name, shape, lo, hi, dtype=np.float32):
    return _rng(seed, name).uniform(lo, hi, size=shape).astype(dtype)


def normal(seed, name, shape, std, dtype=np.float32):
    return (_rng(seed, name).standard_normal(size=shape) * std).astype(dtype)


# --------------------------------------------------------------------------
# Attention decoder (reference: models/attention.py:18-126)
# --------------------------------------------------------------------------

def decoder_param_shapes(A, D, M, V, E=ENCODER_DIM):
    """State-dict names/shapes of the reference AttentionDecoder (models/attention.py:103-117)."""
    return [
        ("attention.enc_att.weight", (A, E)), ("attention.enc_att.bias", (A,)),
        ("attention.dec_att.weight", (A, D)), ("attention.dec_att.bias", (A,)),
        ("attention.full_att.weight", (1, A)), ("attention.full_att.bias", (1,)),
        ("decode_step.weight_ih", (4 * D, M + E)), ("decode_step.weight_hh", (4 * D, D)),
        ("decode_step.bias_ih", (4 * D,)), ("decode_step.bias_hh", (4 * D,)),
        ("h_lin.weight", (D, E)), ("h_lin.bias", (D,)),
        ("c_lin.weight", (D, E)), ("c_lin.bias", (D,)),
        ("f_beta.weight", (E, D)), ("f_beta.bias", (E,)),
        ("fc.weight", (V, D)), ("fc.bias", (V,)),
        ("embedding.weight", (V, M)),
    ]


def decoder_params(seed, A, D, M, V, emb_dtype=np.float32):
    """Seeded weights with the reference init *distributions* (torch Linear / LSTMCell
    default U(+-1/sqrt(fan_in)); fc and embedding U(+-0.1), models/attention.py:120-122).
    fc.bias is drawn non-zero on purpose so bias bugs are visible."""
    out = {}
    for name, shape in decoder_param_shapes(A, D, M, V):
        if name.startswith("decode_step"):
            b = 1.0 / np.sqrt(D)
        elif name.startswith(("fc.", "embedding.")):
            b = 0.1
        else:
            fan_in = shape[1] if len(shape) == 2 else dict(decoder_param_shapes(A, D, M, V))[
                name.replace("bias", "weight")][1]
            b = 1.0 / np.sqrt(fan_in)
        dt = emb_dtype if name == "embedding.weight" else np.float32
        out[name] = uniform(seed, name, shape, -b, b, dt)
    return out


def encoder_features(seed, B, P=196, E=ENCODER_DIM, name="enc"):
    """Post-ReLU-like encoder features, U[0,1) (layout (B,14,14,E) when P=196)."""
    x = uniform(seed, name, (B, P, E), 0.0, 1.0)
    if P == 196:
        x = x.reshape(B, 14, 14, E)
    return x


def captions(seed, B, L, V, lengths=None):
    """Padded captions in the reference vocabulary layout (vocabulary.py:52-58):
    pad=0, words 1..V-4, <start>=V-3, <end>=V-2, <unk>=V-1."""
    rng = _rng(seed, "caps")
    if lengths is None:
        lengths = [L] * B
    caps = np.zeros((B, L), np.int64)
    for b, l in enumerate(lengths):
        caps[b, 0] = V - 3
        caps[b, 1:l - 1] = rng.integers(1, V - 3, size=l - 2)
        caps[b, l - 1] = V - 2
    return caps


def images(seed, B, H=224, W=224, name="img"):
    """U[0,1) pixels, then Normalize(mean, std) as models/attention.py:296-301."""
    x = uniform(seed, name, (B, 3, H, W), 0.0, 1.0)
    return ((x - IMG_MEAN[None, :, None, None]) / IMG_STD[None, :, None, None]).astype(np.float32)


# --------------------------------------------------------------------------
# ResNet-101 (torchvision layout; models/encoder.py:9-20,88-92)
# --------------------------------------------------------------------------

RESNET101_LAYERS = (3, 4, 23, 3)


def resnet101_param_shapes(layers=RESNET101_LAYERS):
    """torchvision resnet101 state-dict names/shapes (Bottleneck, expansion 4, v1.5)."""
    shapes = [("conv1.weight", (64, 3, 7, 7))]
    shapes += _bn("bn1", 64)
    cin = 64
    for li, (n, width) in enumerate(zip(layers, (64, 128, 256, 512))):
        for bi in range(n):
            p = f"layer{li + 1}.{bi}"
            shapes.append((f"{p}.conv1.weight", (width, cin, 1, 1)))
            shapes += _bn(f"{p}.bn1", width)
            shapes.append((f"{p}.conv2.weight", (width, width, 3, 3)))
            shapes += _bn(f"{p}.bn2", width)
            shapes.append((f"{p}.conv3.weight", (width * 4, width, 1, 1)))
            shapes += _bn(f"{p}.bn3", width * 4)
            if bi == 0:
                shapes.append((f"{p}.downsample.0.weight", (width * 4, cin, 1, 1)))
                shapes += _bn(f"{p}.downsample.1", width * 4)
            cin = width * 4
    return shapes


def _bn(p, c):
    return [(f"{p}.weight", (c,)), (f"{p}.bias", (c,)), (f"{p}.running_mean", (c,)),
            (f"{p}.running_var", (c,))]


def resnet101_params(seed, layers=RESNET101_LAYERS):
    """Kaiming-normal(fan_out) conv weights (torchvision init); BN affine drawn
    around (1, 0) so the affine path is exercised; running stats 0 / 1."""
    out = {}
    for name, shape in resnet101_param_shapes(layers):
        if len(shape) == 4:
            fan_out = shape[0] * shape[2] * shape[3]
            out[name] = normal(seed, name, shape, np.sqrt(2.0 / fan_out))
        elif name.endswith(".weight"):
            out[name] = uniform(seed, name, shape, 0.5, 1.5)
        elif name.endswith(".bias"):
            out[name] = uniform(seed, name, shape, -0.2, 0.2)
        elif name.endswith("running_mean"):
            out[name] = np.zeros(shape, np.float32)
        else:
            out[name] = np.ones(shape, np.float32)
    return out


def probe_indices(n, k=64, seed=7):
    """Fixed sample positions used to store strided samples of large tensors."""
    rng = np.random.default_rng([seed, n])
    return np.sort(rng.choice(n, size=min(k, n), replace=False))


def digest(x):
    """Size-independent fingerprint of a float tensor: (sum, sum|x|, <x, w>) with a
    fixed pseudo-random weight vector w, accumulated in float64."""
    x = np.asarray(x, np.float64).ravel()
    w = np.random.default_rng([11, x.size]).uniform(-1, 1, size=x.size)
    return np.array([x.sum(), np.abs(x).sum(), float(x @ w)], np.float64)
