"""GPU: the reference image transform on the device (capmi_resize_normalize_u8)
is bit-identical to torchvision's PIL path -- Pillow's Image.resize(BILINEAR), ToTensor, Normalize
-- restated by oracle/image_ref.py and pinned to Pillow by tests/test_image_cpu.py: one batch of
mixed sizes (COCO-like reductions, an enlargement, identity, odd shapes) must match exactly. Then
the COCO path end to end: COCODataset without a transform -> packed uint8 batches -> GPU transform
-> the attention train() step on a tiny COCO tree."""
import pickle
import types

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import image_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_resize_normalize_matches_pil():
    from capmi.imagepipe import GpuImageTransform, PackedImages
    rng = np.random.default_rng(3)
    sizes = [(480, 640), (375, 500), (224, 224), (100, 150), (333, 251), (1000, 90), (17, 300)]
    arrs = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in sizes]
    out = GpuImageTransform(DEV)(PackedImages(arrs))
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for i, a in enumerate(arrs):
        want = R.transform(a)
        assert np.array_equal(got[i], want), (sizes[i], float(np.abs(got[i] - want).max()))
        # and the uint8 resample itself is Pillow's
        pil = np.asarray(Image.fromarray(a).resize((224, 224), Image.BILINEAR)).astype(np.float32) / np.float32(255)
        m = np.array(R.MEAN, np.float32).reshape(1, 1, 3)
        s = np.array(R.STD, np.float32).reshape(1, 1, 3)
        assert np.array_equal(got[i], ((pil - m) / s).transpose(2, 0, 1))


def test_coco_train_end_to_end(tmp_path, monkeypatch):
    import checkpoint as C
    from pathconf import PathConfig
    from test_data_cpu import make_coco
    anno, img_dir, vocab = make_coco(tmp_path, n_img=4)
    vf = tmp_path / "vocab.pkl"
    with open(vf, "wb") as f:
        pickle.dump(vocab, f)
    monkeypatch.setattr(PathConfig, "train_anno_file", str(anno))
    monkeypatch.setattr(PathConfig, "train_img_dir", str(img_dir))
    monkeypatch.setattr(PathConfig, "vocab_file", str(vf))
    monkeypatch.setattr(C, "CHECKPOINTS_DIR", str(tmp_path / "ck"))
    from models.attention import train
    args = types.SimpleNamespace(
        model_name="coco_tiny", model="attention", attention_dim=64, decoder_dim=64, decoder_dropout=0.5,
        embed_size=32, epochs=1, batch_size=4, workers=0, encoder_lr=1e-4, decoder_lr=1e-4, grad_clip=5.0,
        alpha_c=1.0, fine_tune_encoder=False, fine_tune_embedding=False, checkpoint=None, print_freq=1,
        use_glove=False, max_caption_length=-1, use_bert=False, synthetic=False, synthetic_size=0,
        vocab_size=len(vocab), trusted_checkpoint=False)
    train(torch.device(DEV), args)
    ck = torch.load(tmp_path / "ck" / "coco_tiny_0.pth.tar", weights_only=True)
    losses = ck["metrics"]["epoch_losses"][0]
    assert len(losses) == 2 and all(np.isfinite(losses)), losses
