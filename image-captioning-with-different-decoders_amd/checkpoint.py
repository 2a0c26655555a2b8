"""Per-epoch checkpoints (reference checkpoint.py:8-62).

Two formats, one API:
  * default: the reference's dict keys holding state_dicts, so a checkpoint loads with
    torch.load(..., weights_only=True) (the reference's own files fail on torch >= 2.6, Q13);
  * ``save_checkpoint(..., whole_modules=True)``: the reference's format itself -- the encoder,
    decoder and optimizer OBJECTS pickled under their class paths (models.encoder.EncoderAttention,
    models.attention.AttentionDecoder, capmi.optim.Adam), for eval.py / gen_captions.py-style
    callers that unpack modules (eval.py:35-36). Loading those executes pickle code:
    ``load_checkpoint(..., weights_only=False)``, for files you wrote yourself only.
``unpack_checkpoint`` returns what is stored (modules or state_dicts); ``train()`` takes either.
"""
import os

import torch

CHECKPOINTS_DIR = 'checkpoints'


def save_checkpoint(args, epoch, encoder, decoder, encoder_optimizer, decoder_optimizer, metrics,
                    verbose=True, whole_modules=False):
    if whole_modules:  # the reference's checkpoint.py:51-58 layout
        state = {'epoch': epoch, 'metrics': metrics, 'encoder': encoder, 'decoder': decoder,
                 'encoder_optimizer': encoder_optimizer, 'decoder_optimizer': decoder_optimizer}
    else:
        state = {
            'epoch': epoch,
            'metrics': metrics,
            'encoder': encoder.state_dict(),
            'decoder': decoder.state_dict(),
            'encoder_optimizer': None if encoder_optimizer is None else encoder_optimizer.state_dict(),
            'decoder_optimizer': decoder_optimizer.state_dict(),
        }
    os.makedirs(CHECKPOINTS_DIR, exist_ok=True)
    path = os.path.join(CHECKPOINTS_DIR, f'{args.model_name}_{epoch}.pth.tar')
    torch.save(state, path)
    if verbose:
        print(f'Saved checkpoint to {path}')


def load_checkpoint(device, args, verbose=True, weights_only=True):
    path = os.path.join(CHECKPOINTS_DIR, f'{args.checkpoint}')
    if verbose:
        print(f'Loading checkpoint {path}')
    return torch.load(path, map_location=str(device), weights_only=weights_only)


def unpack_checkpoint(chkpt):
    return (chkpt['epoch'], chkpt['encoder'], chkpt['decoder'], chkpt['encoder_optimizer'],
            chkpt['decoder_optimizer'], chkpt['metrics'])
