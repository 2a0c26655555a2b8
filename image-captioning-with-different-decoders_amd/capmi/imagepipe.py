"""The reference's image transform on the GPU.

Reference (models/attention.py:296-301 + dataset.py:55-59): every DataLoader worker decodes a
JPEG, applies Resize((224, 224)) -> ToTensor -> Normalize on the CPU and the collate stacks
(B, 3, 224, 224) fp32. Here the workers only decode (PIL) and the collate packs the uint8 RGB
pixels of the batch into one (pinned) buffer; on the device ``GpuImageTransform`` runs
``capmi_resize_normalize_u8`` (csrc/image.hip): the same resample, bit-identical to Pillow's,
then ToTensor + Normalize. The host keeps only the JPEG decode: resampling a 640x480 image and
normalising it costs the CPU several ms, which at ~4000 training images/s per GPU would take tens
of cores. PCIe then carries the decoded uint8 pixels (0.92 MB for 640x480, ~1.5x the 0.6 MB fp32
tensor the reference copies; 3.7 GB/s at that rate).
"""
import numpy as np
import torch

from . import kernels as K

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


class PackedImages:
    """A batch of decoded RGB images, uint8 HWC, packed back to back (the collate's output)."""

    def __init__(self, arrays, pin=True):
        sizes = [a.shape[0] * a.shape[1] * 3 for a in arrays]
        self.heights = torch.tensor([a.shape[0] for a in arrays], dtype=torch.int32)
        self.widths = torch.tensor([a.shape[1] for a in arrays], dtype=torch.int32)
        self.offsets = torch.tensor(np.concatenate([[0], np.cumsum(sizes)[:-1]]) if arrays else [],
                                    dtype=torch.int64)
        buf = torch.empty(int(sum(sizes)), dtype=torch.uint8)
        o = 0
        for a, n in zip(arrays, sizes):
            if a.ndim != 3 or a.shape[2] != 3 or a.dtype != np.uint8:
                raise ValueError("PackedImages takes (H, W, 3) uint8 arrays")
            buf[o:o + n] = torch.from_numpy(np.ascontiguousarray(a).reshape(-1))
            o += n
        self.data = buf.pin_memory() if pin and torch.cuda.is_available() else buf

    def __len__(self):
        return int(self.heights.numel())

    def pin_memory(self):  # DataLoader(pin_memory=True) calls this on custom batch types
        if not self.data.is_pinned():
            self.data = self.data.pin_memory()
        return self


class GpuImageTransform:
    """PackedImages -> (B, 3, OH, OW) fp32 on `device`: Resize (PIL bilinear, bit-exact) +
    ToTensor + Normalize(MEAN, STD). Workspaces grow to the largest batch seen and are reused."""

    def __init__(self, device, size=(224, 224), mean=MEAN, std=STD):
        self.device = torch.device(device)
        self.size = tuple(size)
        self.mean, self.std = tuple(mean), tuple(std)
        self._tmp = None

    def __call__(self, batch: PackedImages):
        dev = self.device
        B = len(batch)
        OH, OW = self.size
        out = torch.empty(B, 3, OH, OW, device=dev, dtype=torch.float32)
        if B == 0:
            return out
        max_h, max_w = int(batch.heights.max()), int(batch.widths.max())
        src = batch.data.to(dev, non_blocking=True)
        offs = batch.offsets.to(dev, non_blocking=True)
        hs = batch.heights.to(dev, non_blocking=True)
        ws = batch.widths.to(dev, non_blocking=True)
        need = B * max_h * OW * 3
        if self._tmp is None or self._tmp.numel() < need:
            self._tmp = torch.empty(need, device=dev, dtype=torch.uint8)
        K.resize_normalize_u8(src, offs, hs, ws, max_h, max_w, OH, OW, self.mean, self.std, self._tmp, out)
        return out


def decode_rgb(path):
    """JPEG (any PIL format) -> (H, W, 3) uint8, as the reference's Image.open(...).convert('RGB')
    (dataset.py:55-56)."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert('RGB'))
