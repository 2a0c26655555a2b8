"""Baseline LSTM captioner with the reference surface (models/baseline.py:19-374).

BASELINE.json config 1 ("'baseline' LSTM decoder, batch_size 4 ... on CPU;
plumbing, no GPU"): on CPU tensors the decoder is the plain nn modules (nn.LSTM /
Linear), as in the reference. On HIP tensors forward()
is capmi.baseline_fn.BaselineDecoderFn: the same parameters, hoisted input and
vocabulary GEMMs, the fused LSTM cell per step and a BPTT backward on the capmi
kernels. The ResNet-101 encoder (models.encoder.Encoder) runs the capmi kernels
when given HIP tensors.
"""
import time

import torch
import torch.nn as nn

from checkpoint import save_checkpoint
from metric import AccumulatingMetric
from models.encoder import Encoder
from train_utils import clip_gradient
from vocabulary import PAD_TOKEN


class BaselineDecoderParams:
    hidden_size = 512
    embed_size = 512  # Use 300 if glove.
    vocab_size = None  # Must override.


class BaselineDecoder(nn.Module):
    def __init__(self, params):
        super().__init__()
        assert isinstance(params, BaselineDecoderParams)
        assert params.vocab_size is not None
        self.embed_size = params.embed_size
        self.hidden_size = params.hidden_size
        self.embedding = nn.Embedding(params.vocab_size, params.embed_size)
        self.lstm = nn.LSTM(input_size=params.embed_size, hidden_size=params.hidden_size, num_layers=1,
                            bias=True, batch_first=True, dropout=0, bidirectional=False)
        self.linear = nn.Linear(params.hidden_size, params.vocab_size)

    def load_pretrained_embeddins(self, embeddings):
        self.embedding.weight = nn.Parameter(embeddings)

    def fine_tune_embeddings(self, on=True):
        for param in self.embedding.parameters():
            param.requires_grad = on

    def _capmi_ws(self, device):
        """stream-K workspace of the decoder's GEMMs (runtime state: not pickled)."""
        ws = self.__dict__.get("_capmi_sk")
        if ws is None or ws.device != torch.device(device):
            from capmi import kernels as K
            ws = K.gemm_workspace(device)
            self.__dict__["_capmi_sk"] = ws
        return ws

    def __getstate__(self):
        st = self.__dict__.copy()
        st.pop("_capmi_sk", None)
        return st

    def forward(self, img_features, captions):
        """(B,M) image features, (B,L) captions -> (B,L,V) scores: the image feature is
        step 0, the caption without <end> follows (reference :81-111)."""
        if img_features.is_cuda:
            from capmi.baseline_fn import baseline_forward
            return baseline_forward(self, img_features, captions)
        captions = captions[:, :-1]
        embeddings = self.embedding(captions)
        embeddings = torch.cat((img_features.unsqueeze(1).float(), embeddings.float()), dim=1)
        lstm_out, _ = self.lstm(embeddings)
        return self.linear(lstm_out)


def train(device, args):
    """Reference :114-264 (CE with ignore_index=PAD against the captions incl. <start>)."""
    from capmi.data import SyntheticCOCO, synthetic_requested
    from torch.nn.utils.rnn import pad_sequence
    if synthetic_requested(args):
        dataset = SyntheticCOCO.from_args(args)
    else:
        from dataset import COCODataset
        dataset = COCODataset(mode='train', caption_max_len=args.max_caption_length)
    pad_idx = dataset.vocab(PAD_TOKEN)

    def collate_fn(data):
        imgs, captions = zip(*data)
        return torch.stack(imgs, 0), pad_sequence(captions, batch_first=True, padding_value=pad_idx)

    loader = torch.utils.data.DataLoader(dataset, batch_size=args.batch_size, shuffle=True,
                                         num_workers=args.workers, collate_fn=collate_fn)
    encoder = Encoder(args.embed_size)
    # reference :279-282: only the (trainable) embed Linear, since fine_tune() is never called
    encoder_optimizer = torch.optim.Adam(params=filter(lambda p: p.requires_grad, encoder.parameters()),
                                         lr=args.encoder_lr) if args.fine_tune_encoder else None
    params = BaselineDecoderParams()
    params.embed_size, params.hidden_size, params.vocab_size = args.embed_size, args.decoder_dim, len(dataset.vocab)
    decoder = BaselineDecoder(params)
    if args.use_glove:
        from embed import load_glove_vectors
        decoder.load_pretrained_embeddins(load_glove_vectors())
    decoder.fine_tune_embeddings(on=args.fine_tune_embedding)
    decoder_optimizer = torch.optim.Adam(params=filter(lambda p: p.requires_grad, decoder.parameters()),
                                         lr=args.decoder_lr)
    encoder, decoder = encoder.to(device), decoder.to(device)
    criterion = nn.CrossEntropyLoss(ignore_index=pad_idx).to(device)
    decoder.train()
    encoder.train()
    train_start = time.time()
    num_batches = len(loader)
    epoch_losses = []
    for epoch in range(args.epochs):
        batch_losses = []
        accum_loss, accum_time = AccumulatingMetric(), AccumulatingMetric()
        start = time.time()
        for batch_idx, (imgs, captions) in enumerate(loader):
            imgs, captions = imgs.to(device), captions.to(device)
            scores = decoder(encoder(imgs), captions)
            loss = criterion(scores.reshape(-1, scores.shape[2]), captions.reshape(-1))
            decoder_optimizer.zero_grad()
            if encoder_optimizer is not None:
                encoder_optimizer.zero_grad()
            loss.backward()
            clip_gradient(decoder_optimizer, args.grad_clip)
            if encoder_optimizer is not None:
                clip_gradient(encoder_optimizer, args.grad_clip)
            decoder_optimizer.step()
            if encoder_optimizer is not None:
                encoder_optimizer.step()
            batch_losses.append(loss.item())
            accum_loss.update(loss.item())
            accum_time.update(time.time() - start)
            if batch_idx % args.print_freq == 0:
                print(f'Epoch {epoch+1}/{args.epochs}, Batch {batch_idx+1}/{num_batches}, '
                      f'Loss {accum_loss.avg():.4f}, Time: {accum_time.val:.4f}')
            start = time.time()
        epoch_losses.append(batch_losses)
        save_checkpoint(args, epoch, encoder, decoder, encoder_optimizer, decoder_optimizer,
                        {'epoch_losses': epoch_losses})
    print(f'Model {args.model_name} finished training for {args.epochs} epochs in '
          f'{time.time() - train_start:.4f} seconds.')


def evaluate(device, args, encoder, decoder):
    raise NotImplementedError("evaluation / caption scoring is not part of the training path")
