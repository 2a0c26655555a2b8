"""Minimal COCO captions index (the part of pycocotools.coco.COCO that dataset.py and
vocabulary.py use: imgs, anns, getAnnIds(imgIds=), loadAnns, loadImgs). pycocotools is absent
here (the reference vendors cp36-38 binaries of it, which are never loaded); the annotation file
is the standard captions JSON ({"images": [{id, file_name, ...}], "annotations": [{id, image_id,
caption}]})."""
import json
from collections import defaultdict


class COCO:
    def __init__(self, annotation_file):
        with open(annotation_file) as f:
            d = json.load(f)
        self.dataset = d
        self.imgs = {im['id']: im for im in d.get('images', [])}
        self.anns = {a['id']: a for a in d.get('annotations', [])}
        self.img_to_anns = defaultdict(list)
        for a in d.get('annotations', []):
            self.img_to_anns[a['image_id']].append(a['id'])

    def getAnnIds(self, imgIds=()):
        ids = imgIds if isinstance(imgIds, (list, tuple)) else [imgIds]
        return [a for i in ids for a in self.img_to_anns.get(i, [])]

    def loadAnns(self, ids):
        ids = ids if isinstance(ids, (list, tuple)) else [ids]
        return [self.anns[i] for i in ids]

    def loadImgs(self, ids):
        ids = ids if isinstance(ids, (list, tuple)) else [ids]
        return [self.imgs[i] for i in ids]
