"""Training entry point with the reference CLI (train.py:11-86).

    python train.py basic_att --model attention --batch_size 64 [--synthetic True]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py basic_att --model attention ...

Flags, defaults and the argparse ``type=bool`` quirk (any non-empty string is True,
Q10) are the reference's. Added: ``--synthetic`` (COCO-shaped synthetic data; the COCO
pipeline is not part of this build) and data parallelism from torchrun's env.
"""
import argparse
import os
import sys

sys.path.append('cocoapi/PythonAPI/')
import torch  # noqa: E402

from pathconf import PathConfig  # noqa: E402


def parse_args(argv=None):
    parser = argparse.ArgumentParser(description='Train')
    parser.add_argument('model_name', type=str,
                        help='unique name of model setting; saved with this name in checkpoints folder.')
    parser.add_argument('--model', type=str, choices=['baseline', 'attention'], help='Model to train')
    parser.add_argument('--attention_dim', type=int, default=512, help='attention dimension.')
    parser.add_argument('--decoder_dim', type=int, default=512, help='decoder dimension.')
    parser.add_argument('--decoder_dropout', type=float, default=0.5, help='decoder dropout probability.')
    parser.add_argument('--embed_size', type=int, default=512,
                        help='embedding dimension. If using pre-trained glove vectors, use 300.')
    parser.add_argument('--epochs', type=int, default=1, help='number of epochs to train for.')
    parser.add_argument('--batch_size', type=int, default=32, help='batch_size.')
    parser.add_argument('--workers', type=int, default=1, help='for data-loading.')
    parser.add_argument('--encoder_lr', type=float, default=1e-4, help='learning rate for encoder if fine-tuning.')
    parser.add_argument('--decoder_lr', type=float, default=1e-4, help='learning rate for decoder.')
    parser.add_argument('--grad_clip', type=float, default=5., help='clip gradients at an absolute value of.')
    parser.add_argument('--alpha_c', type=float, default=1.,
                        help='regularization parameter for doubly stochastic attention, as in the paper.')
    parser.add_argument('--fine_tune_encoder', type=bool, default=False, help='whether to fine-tune encoder or not.')
    parser.add_argument('--fine_tune_embedding', type=bool, default=False,
                        help='whether to fine-tune word embeddings or not.')
    parser.add_argument('--checkpoint', default=None, type=str,
                        help='name of checkpoint in ./checkpoints folder; None if none.')
    parser.add_argument('--print_freq', type=int, default=1, help='print training/validation stats every __ batches.')
    parser.add_argument('--use_glove', type=bool, default=False, help='whether to use pre-trained glove embeddings.')
    parser.add_argument('--max_caption_length', type=int, default=-1,
                        help='only use captions with caption length <= 50 when training.')
    parser.add_argument('--use_bert', type=bool, default=False, help='whether to use BERT embeddigns for attention model.')
    # capmi additions
    parser.add_argument('--trusted_checkpoint', type=bool, default=False,
                        help='--checkpoint is a whole-module pickle you wrote yourself (load with weights_only=False).')
    parser.add_argument('--synthetic', type=bool, default=False, help='COCO-shaped synthetic data.')
    parser.add_argument('--synthetic_size', type=int, default=0, help='samples in the synthetic dataset.')
    parser.add_argument('--vocab_size', type=int, default=8100, help='synthetic vocabulary size.')
    return parser.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    device = torch.device('cuda' if torch.cuda.is_available() else 'cpu')
    from capmi.data import synthetic_requested
    if not synthetic_requested(args) and not os.path.exists(PathConfig.vocab_file):
        raise SystemError('Must run "python init.py --vocab True" before training.')
    if args.use_glove:
        if not os.path.exists(PathConfig.glove_vectors):
            raise SystemError('Must run "python init.py --glove True" when using glove vectors.')
        assert args.embed_size == 300, 'Expected embedding size of 300 for glove vectors.'
    if args.use_bert:
        assert args.model == 'attention', 'BERT is only used for attention model.'
        assert args.embed_size == 768, 'Expected embedding size of 768 for BERT.'
    if args.model == 'baseline':
        from models.baseline import train as train_baseline_model
        print('Training baseline model...')
        train_baseline_model(device, args)
        return
    if args.model == 'attention':
        from models.attention import train as train_attention_model
        print('Training attention model...')
        train_attention_model(device, args)
        return


if __name__ == '__main__':
    main()
