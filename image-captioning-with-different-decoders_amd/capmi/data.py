"""Synthetic COCO-shaped training data (BASELINE.json / SURVEY.md §8d).

Images: (3,224,224) pixels U[0,1) normalised with the reference's mean/std
(models/attention.py:296-301). Captions: <start> + words U{1..V-4} + <end>,
vocabulary layout of vocabulary.py:52-58 (pad 0, words, <start>, <end>, <unk>).
The real COCO pipeline (dataset.py, nltk, JPEG decode) is SURVEY.md §8f rank 3.
"""
import os

import torch

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def synthetic_requested(args):
    return bool(getattr(args, "synthetic", False)) or os.environ.get("CAPMI_SYNTHETIC") == "1"


def normalize_(x):
    m = torch.tensor(MEAN, device=x.device, dtype=x.dtype).view(1, 3, 1, 1)
    s = torch.tensor(STD, device=x.device, dtype=x.dtype).view(1, 3, 1, 1)
    return x.sub_(m).div_(s)


def synthetic_batch(B, L=25, V=8100, device="cpu", seed=1234, H=224, W=224):
    """One batch on ``device``: (imgs (B,3,H,W) fp32, captions (B,L) int64, lengths [L]*B)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    imgs = normalize_(torch.rand(B, 3, H, W, generator=g, device=device))
    caps = torch.randint(1, V - 3, (B, L), generator=g, device=device)
    caps[:, 0] = V - 3
    caps[:, -1] = V - 2
    return imgs, caps, [L] * B


class SyntheticCOCO(torch.utils.data.Dataset):
    """Dataset with the COCODataset surface the train loop uses (``vocab``, items (img, caption))."""

    def __init__(self, n, V=8100, L=25, ragged=False, seed=1234):
        from vocabulary import synthetic_vocab
        self.vocab = synthetic_vocab(V)
        self.n, self.V, self.L, self.ragged, self.seed = n, V, L, ragged, seed

    @classmethod
    def from_args(cls, args):
        return cls(int(getattr(args, "synthetic_size", 0) or 64 * 16), V=int(getattr(args, "vocab_size", 8100)),
                   L=int(getattr(args, "synthetic_len", 25)))

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        img = normalize_(torch.rand(1, 3, 224, 224, generator=g))[0]
        L = self.L if not self.ragged else int(torch.randint(5, self.L + 1, (1,), generator=g))
        cap = torch.randint(1, self.V - 3, (L,), generator=g)
        cap[0] = self.V - 3
        cap[-1] = self.V - 2
        return img, cap


class SyntheticBertEmbedder:
    """Stand-in for the reference's BERT features (models/attention.py:166-215): bert-base-uncased
    cannot be fetched offline, so the (B, L+1, 768) word-level features are a seeded per-token
    vector plus a per-position vector, with a fixed [CLS] row prepended (:170 prepends '[CLS] ').
    Deterministic for a given caption; frozen (no gradient), as the reference's no_grad BERT."""

    def __init__(self, V, dim=768, max_len=64, seed=768, device="cpu", scale=0.5):
        g = torch.Generator().manual_seed(seed)
        self.tok = ((torch.rand(V, dim, generator=g) - 0.5) * 2 * scale).to(device)
        self.pos = ((torch.rand(max_len + 1, dim, generator=g) - 0.5) * 2 * scale * 0.2).to(device)
        self.cls = ((torch.rand(dim, generator=g) - 0.5) * 2 * scale).to(device)

    def __call__(self, encoded_captions):
        caps = encoded_captions.to(self.tok.device)
        B, L = caps.shape
        out = torch.empty(B, L + 1, self.tok.shape[1], device=self.tok.device, dtype=torch.float32)
        out[:, 0] = self.cls
        out[:, 1:] = self.tok[caps] + self.pos[1:L + 1]
        return out
