"""Caption generation with beam search (reference gen_captions.py:16-131), same function name and
signature. On a HIP device the decode runs on capmi's kernels (capmi.beam.BeamSearch); the
encoder is the capmi EncoderAttention. Image loading / plotting of the reference's CLI
(imageio, matplotlib, checkpoints of whole modules) is outside the built path."""
import torch

from capmi.beam import BeamSearch
from vocabulary import END_TOKEN, START_TOKEN


def attention_caption_image_beam_search(device, args, img, encoder, decoder, vocab):
    """Reads an image and captions it with beam search (reference :16-131).

    Returns (caption token ids, attention weights (steps+1, 14, 14) as nested lists, finished)."""
    with torch.no_grad():
        encoder_out = encoder(img)  # (1, 14, 14, 2048)
    return BeamSearch(decoder, args.beam_size).search(encoder_out, vocab(START_TOKEN), vocab(END_TOKEN))
