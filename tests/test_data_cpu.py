"""CPU: the COCO data path around the GPU image transform: the captions
tokenizer (nltk's Treebank rules restated; nltk is absent, so expected tokens are nltk's documented
behaviour -- parity unpinned), the COCO captions index standing in for pycocotools, COCODataset's
reference surface (dataset.py:14-75) on a tiny COCO tree written here, and the uint8 packing the
loader hands to the GPU."""
import json
import types

import numpy as np
import pytest
import torch
from PIL import Image

from capmi.text import _treebank


@pytest.mark.parametrize("text,tokens", [
    ("a man riding a wave on top of a surfboard.", "a man riding a wave on top of a surfboard ."),
    ("a dog, a cat and a bird", "a dog , a cat and a bird"),
    ("the man's hat isn't red.", "the man 's hat is n't red ."),
    ("two (2) people", "two ( 2 ) people"),
    ('a "big" dog; cannot run!', "a `` big '' dog ; can not run !"),
    ("near 1,000 fans at 3:45...", "near 1,000 fans at 3:45 ..."),
])
def test_treebank_tokenizer(text, tokens):
    assert _treebank(text) == tokens.split()


def make_coco(root, n_img=3, sizes=((480, 640), (375, 500), (224, 224))):
    """A tiny COCO captions tree: images/ + annotations JSON + a vocabulary over its words."""
    img_dir = root / "images"
    img_dir.mkdir()
    images, anns = [], []
    caps = ["a man riding a wave on top of a surfboard.", "a dog, a cat and a bird",
            "two people on a bench", "a red bus on the street.", "a plate of food"]
    rng = np.random.default_rng(0)
    k = 0
    for i in range(n_img):
        h, w = sizes[i % len(sizes)]
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(img_dir / f"{i:03d}.jpg", quality=92)
        images.append({"id": 100 + i, "file_name": f"{i:03d}.jpg", "height": h, "width": w})
        for j in range(2):
            anns.append({"id": 1000 + k, "image_id": 100 + i, "caption": caps[k % len(caps)]})
            k += 1
    anno = root / "captions.json"
    anno.write_text(json.dumps({"images": images, "annotations": anns}))
    from vocabulary import END_TOKEN, PAD_TOKEN, START_TOKEN, UNK_TOKEN, Vocabulary
    vocab = Vocabulary()
    vocab.add_word(PAD_TOKEN)
    for c in caps:
        for t in _treebank(c):
            vocab.add_word(t)
    for t in (START_TOKEN, END_TOKEN, UNK_TOKEN):
        vocab.add_word(t)
    return anno, img_dir, vocab


def test_coco_dataset_surface(tmp_path, monkeypatch):
    from pathconf import PathConfig
    anno, img_dir, vocab = make_coco(tmp_path)
    monkeypatch.setattr(PathConfig, "train_anno_file", str(anno))
    monkeypatch.setattr(PathConfig, "train_img_dir", str(img_dir))
    monkeypatch.setattr(PathConfig, "val_anno_file", str(anno))
    monkeypatch.setattr(PathConfig, "val_img_dir", str(img_dir))
    from dataset import COCODataset
    ds = COCODataset("train", caption_max_len=-1, vocab=vocab)
    assert len(ds) == 6
    img, cap = ds[0]
    assert isinstance(img, np.ndarray) and img.dtype == np.uint8 and img.shape == (480, 640, 3)
    words = "a man riding a wave on top of a surfboard .".split()
    assert cap.tolist() == [vocab("<start>")] + [vocab(w) for w in words] + [vocab("<end>")]
    # caption_max_len filters on the raw caption length (dataset.py:33-34)
    assert len(COCODataset("train", caption_max_len=25, vocab=vocab)) == 4
    # val mode: image path and every caption of the image
    v = COCODataset("val", caption_max_len=-1, vocab=vocab)
    img, cap, path, all_caps = v[1]
    assert path.endswith("000.jpg") and len(all_caps) == 2
    # with a transform the PIL image goes through it (reference behaviour)
    t = COCODataset("train", img_transform=lambda im: im.size, caption_max_len=-1, vocab=vocab)
    assert t[0][0] == (640, 480)


def test_packed_images():
    from capmi.imagepipe import PackedImages
    arrs = [np.full((h, w, 3), i, np.uint8) for i, (h, w) in enumerate([(4, 5), (2, 3), (6, 1)])]
    p = PackedImages(arrs, pin=False)
    assert len(p) == 3 and p.heights.tolist() == [4, 2, 6] and p.widths.tolist() == [5, 3, 1]
    assert p.offsets.tolist() == [0, 60, 78] and p.data.numel() == 96
    assert torch.equal(p.data[60:78], torch.full((18,), 1, dtype=torch.uint8))
