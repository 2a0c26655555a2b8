"""Vocabulary (reference vocabulary.py:9-71): special tokens, w2i/i2w, pickle I/O.

``build_vocab`` needs the COCO captions and nltk (absent offline); it is kept
with the reference signature and raises with an explanation when they are
missing. ``synthetic_vocab`` builds a vocabulary of the reference layout
(pad=0, words, <start>, <end>, <unk>) for synthetic runs.
"""
import pickle
from collections import Counter

from pathconf import PathConfig

PAD_TOKEN = '<pad>'      # Padding
START_TOKEN = '<start>'  # Start of sentence
END_TOKEN = '<end>'      # End of sentence
UNK_TOKEN = '<unk>'      # Out of vocabulary (unknown)


class Vocabulary(object):
    """Word <-> index map; unknown words map to <unk> (reference :15-35)."""

    def __init__(self):
        self.w2i = {}
        self.i2w = {}
        self.idx = 0

    def add_word(self, word):
        if word not in self.w2i:
            self.w2i[word] = self.idx
            self.i2w[self.idx] = word
            self.idx += 1

    def __call__(self, word):
        if word not in self.w2i:
            return self.w2i[UNK_TOKEN]
        return self.w2i[word]

    def __len__(self):
        return len(self.w2i)


def build_vocab(threshold=6):
    """Reference :38-60: words with >= threshold occurrences in the COCO train captions."""
    try:
        import nltk
        from pycocotools.coco import COCO
    except ImportError as e:  # pragma: no cover - depends on optional data deps
        raise RuntimeError("build_vocab needs nltk and pycocotools with the COCO annotations") from e
    coco = COCO(PathConfig.train_anno_file)
    counter = Counter()
    for ann_id in coco.anns.keys():
        counter.update(nltk.tokenize.word_tokenize(str(coco.anns[ann_id]['caption']).lower()))
    vocab = Vocabulary()
    vocab.add_word(PAD_TOKEN)
    for word in [w for w, c in counter.items() if c >= threshold]:
        vocab.add_word(word)
    for tok in (START_TOKEN, END_TOKEN, UNK_TOKEN):
        vocab.add_word(tok)
    return vocab


def synthetic_vocab(size):
    """A vocabulary of ``size`` entries in the reference layout (pad, words, start, end, unk)."""
    vocab = Vocabulary()
    vocab.add_word(PAD_TOKEN)
    for i in range(size - 4):
        vocab.add_word(f"w{i}")
    for tok in (START_TOKEN, END_TOKEN, UNK_TOKEN):
        vocab.add_word(tok)
    return vocab


def save_vocab(vocab):
    with open(PathConfig.vocab_file, 'wb') as f:
        pickle.dump(vocab, f)


def load_vocab():
    """Loads the vocabulary pickle written by save_vocab (a file this framework wrote)."""
    with open(PathConfig.vocab_file, 'rb') as f:
        return pickle.load(f)
