"""GloVe table loading (reference embed.py:64-68): a (V, 300) float64 matrix (Q7).
Building it (embed.py:12-61) needs glove.6B and bcolz (setup-time, offline-unavailable)."""
import pickle

import numpy as np
import torch

from pathconf import PathConfig


def load_glove_vectors():
    """Loads the (V,300) fp64 table. The reference pickles a numpy array; this reads that
    file with numpy only when it is a plain .npy, else with pickle (files this project wrote)."""
    print('Loading glove vectors.')
    path = PathConfig.glove_vectors
    if path.endswith('.npy'):
        return torch.tensor(np.load(path))
    with open(path, 'rb') as f:
        return torch.tensor(pickle.load(f))
