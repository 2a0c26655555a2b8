"""Per-epoch checkpoints (reference checkpoint.py:8-62).

The reference pickles whole modules and optimizers. This keeps the same dict
keys but stores state_dicts, so a checkpoint loads with torch.load(...,
weights_only=True) (the reference's own files fail on torch >= 2.6, Q13).
"""
import os

import torch

CHECKPOINTS_DIR = 'checkpoints'


def save_checkpoint(args, epoch, encoder, decoder, encoder_optimizer, decoder_optimizer, metrics,
                    verbose=True):
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


def load_checkpoint(device, args, verbose=True):
    path = os.path.join(CHECKPOINTS_DIR, f'{args.checkpoint}')
    if verbose:
        print(f'Loading checkpoint {path}')
    return torch.load(path, map_location=str(device), weights_only=True)


def unpack_checkpoint(chkpt):
    return (chkpt['epoch'], chkpt['encoder'], chkpt['decoder'], chkpt['encoder_optimizer'],
            chkpt['decoder_optimizer'], chkpt['metrics'])
