"""One 'attention' training step on the MI355X (models/attention.py:386-430).

    feats = encoder(imgs)                        fused ResNet-101, BN in train mode
    loss, grads = decoder fwd + CE + alpha-reg + BPTT   (capmi.decoder_fn, grads in place)
    grads <- all-reduce mean over ranks          (DP only; RCCL, async)
    params <- clamp(+-grad_clip) + Adam          (one kernel)

With more than one rank the all-reduce of step k is issued asynchronously and
its clamp+Adam update is applied at the start of step k+1's decoder, after
step k+1's encoder forward has been launched: the encoder does not read the
decoder's weights, so the collective overlaps the ResNet forward. ``flush()``
completes the last pending update (call it before reading weights / timing).
"""
import torch

from . import decoder_fn as DF
from . import dist as cdist
from .decoder_core import PNAMES


class AttentionTrainStep:
    def __init__(self, encoder, decoder, optimizer, ctx=None, alpha_c=1.0, overlap=True):
        self.encoder, self.decoder, self.opt = encoder, decoder, optimizer
        self.ctx = ctx or cdist.DistCtx(device=next(decoder.parameters()).device)
        self.alpha_c = alpha_c
        self.overlap = overlap and self.ctx.distributed
        self._pending = None
        named = dict(decoder.named_parameters())
        self.need = [n for n in PNAMES if named[n].requires_grad]
        self.params = named

    def _grads(self):
        return {n: self.params[n].grad for n in self.need}

    def _apply_pending(self):
        if self._pending is not None:
            for w in self._pending:
                w.wait()
            self._pending = None
            self.opt.step()

    def __call__(self, imgs, captions, caption_lengths):
        feats = self.encoder(imgs)
        self._apply_pending()
        loss, _, _ = DF.fused_loss_and_grads(self.decoder, feats, captions, caption_lengths,
                                             self.alpha_c, self._grads(), need=self.need)
        if self.ctx.distributed:
            works = cdist.allreduce_mean_(self.opt.grad_buffers(), self.ctx, async_op=self.overlap)
            if self.overlap:
                self._pending = works
                return loss
        self.opt.step()
        return loss

    def flush(self):
        self._apply_pending()
