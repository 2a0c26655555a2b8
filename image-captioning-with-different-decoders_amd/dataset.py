"""COCO captions dataset with the reference surface (dataset.py:14-75).

COCODataset(mode, img_transform=None, caption_max_len=50): items are (image, caption) in 'train'
mode and (image, caption, img_path, all_captions) in 'val' mode, captions numericalized as
<start> + vocab(tokens of the lower-cased caption) + <end>. With an `img_transform` the image is
the transform of the PIL RGB image, as in the reference. Without one (the MI355X path) it is the
decoded (H, W, 3) uint8 array: the loader packs those (capmi.imagepipe.PackedImages) and the GPU
applies Resize/ToTensor/Normalize bit-identically to torchvision's PIL transform.

pycocotools and nltk are used when importable; otherwise capmi.coco.COCO (the captions JSON) and
capmi.text.word_tokenize (Treebank rules) stand in for them.
"""
import os

import torch
import torch.utils.data as data

from pathconf import PathConfig
from vocabulary import END_TOKEN, START_TOKEN, load_vocab


def _coco(anno_file):
    try:
        from pycocotools.coco import COCO
    except ImportError:
        from capmi.coco import COCO
    return COCO(anno_file)


class COCODataset(data.Dataset):
    def __init__(self, mode, img_transform=None, caption_max_len=50, vocab=None):
        assert mode in ['train', 'val']
        self.mode = mode
        self.img_transform = img_transform
        self.vocab = load_vocab() if vocab is None else vocab
        self.caption_max_len = caption_max_len if not caption_max_len == -1 else float('inf')
        self.anno_file = get_anno_file(mode)
        self.img_dir = get_img_dir(mode)
        self.coco = _coco(self.anno_file)
        self.img_ids = list(sorted(self.coco.imgs.keys()))
        self.caption_img_mappings = self._build_caption_img_mappings()

    def _build_caption_img_mappings(self):
        mappings = []
        for img_id in self.img_ids:
            for ann in self._get_annotations(img_id):
                if len(ann['caption']) <= self.caption_max_len:
                    mappings.append({'caption': ann['caption'], 'img_id': img_id})
        return mappings

    def _get_annotations(self, img_id):
        return self.coco.loadAnns(self.coco.getAnnIds(imgIds=img_id))

    def _numericalize_caption(self, caption):
        from capmi.text import word_tokenize
        tokens = word_tokenize(str(caption).lower())
        return torch.LongTensor([self.vocab(START_TOKEN)] + [self.vocab(t) for t in tokens] +
                                [self.vocab(END_TOKEN)])

    def _img_path(self, img_id):
        return os.path.join(self.img_dir, self.coco.loadImgs(img_id)[0]['file_name'])

    def _get_transformed_img(self, img_id):
        path = self._img_path(img_id)
        if self.img_transform is None:
            from capmi.imagepipe import decode_rgb
            return decode_rgb(path)
        from PIL import Image
        with Image.open(path) as im:
            return self.img_transform(im.convert('RGB'))

    def __getitem__(self, idx):
        mapping = self.caption_img_mappings[idx]
        caption, img_id = mapping['caption'], mapping['img_id']
        img = self._get_transformed_img(img_id)
        caption = self._numericalize_caption(caption)
        if self.mode == 'train':
            return img, caption
        all_captions = [self._numericalize_caption(a['caption']) for a in self._get_annotations(img_id)]
        return img, caption, self._img_path(img_id), all_captions

    def __len__(self):
        return len(self.caption_img_mappings)


def get_anno_file(mode):
    return PathConfig.train_anno_file if mode == 'train' else PathConfig.val_anno_file


def get_img_dir(mode):
    return PathConfig.train_img_dir if mode == 'train' else PathConfig.val_img_dir
