"""CPU: the oracle restatement of the reference image transform (oracle/image_ref.py) is
bit-identical to Pillow's own Image.resize(BILINEAR) -- the arithmetic torchvision's Resize
uses on PIL images (models/attention.py:296-301) -- for reductions, enlargements, identity and
odd sizes; ToTensor + Normalize follow torchvision's fp32 ops."""
import numpy as np
import pytest
from PIL import Image

from oracle import image_ref as R


def _img(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


@pytest.mark.parametrize("h,w,oh,ow", [(37, 23, 16, 16), (48, 64, 21, 33), (20, 30, 45, 50), (16, 16, 16, 16),
                                       (9, 120, 17, 19)])
def test_resample_matches_pillow(h, w, oh, ow):
    a = _img(h, w, h * 1000 + w)
    want = np.asarray(Image.fromarray(a).resize((ow, oh), Image.BILINEAR))
    got = R.resize_bilinear(a, (oh, ow))
    assert got.shape == want.shape
    assert np.array_equal(got, want), int(np.abs(got.astype(int) - want).max())


def test_transform_is_totensor_normalize():
    a = _img(30, 40, 7)
    r = np.asarray(Image.fromarray(a).resize((20, 20), Image.BILINEAR))
    import torch
    t = torch.from_numpy(r).permute(2, 0, 1).float().div(255)           # ToTensor
    m = torch.tensor(R.MEAN).view(3, 1, 1)
    s = torch.tensor(R.STD).view(3, 1, 1)
    t = t.sub(m).div(s)                                                   # Normalize
    assert np.array_equal(R.transform(a, (20, 20)), t.numpy())
