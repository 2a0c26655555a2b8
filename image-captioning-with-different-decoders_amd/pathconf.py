"""Static data paths (reference pathconf.py:4-20)."""


class PathConfig:
    vocab_file = 'pkldata/vocab.pkl'
    glove_vectors = 'pkldata/glove_vectors.pkl'
    train_anno_file = 'cocoapi/annotations/captions_train2014.json'
    val_anno_file = 'cocoapi/annotations/captions_val2014.json'
    train_img_dir = 'cocoapi/images/train2014'
    val_img_dir = 'cocoapi/images/val2014'
