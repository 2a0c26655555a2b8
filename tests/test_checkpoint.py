"""Checkpoint interop (reference checkpoint.py:8-62, eval.py:35-36): the default
state_dict format loads with weights_only=True; the reference's whole-module format
(save_checkpoint(..., whole_modules=True)) round-trips the encoder, decoder and optimizer OBJECTS
under their class paths -- without the encoder's launch caches -- and train() resumes from either."""
import types

import pytest
import torch

import checkpoint as C
from helpers import make_decoder


def _models():
    from capmi.optim import Adam
    from models.encoder import EncoderAttention
    torch.manual_seed(0)
    enc = EncoderAttention()
    enc.set_compute_precision("bf16")
    enc._runner.packed.cache["junk"] = (0, 0, torch.zeros(1 << 20))  # a launch cache: must not be saved
    dec, _ = make_decoder(32, 32, 16, 50, 3, "cpu")
    opt = Adam([p for p in dec.parameters() if p.requires_grad], lr=1e-4)
    for p in opt.param_groups[0]["params"]:
        p.grad.fill_(0.01) if p.grad is not None else None
    return enc, dec, opt


def test_state_dict_checkpoint_weights_only(tmp_path, monkeypatch):
    monkeypatch.setattr(C, "CHECKPOINTS_DIR", str(tmp_path))
    enc, dec, opt = _models()
    args = types.SimpleNamespace(model_name="att", checkpoint="att_3.pth.tar")
    C.save_checkpoint(args, 3, enc, dec, None, opt, {"epoch_losses": [1.0]}, verbose=False)
    ep, e, d, eo, do, m = C.unpack_checkpoint(C.load_checkpoint("cpu", args, verbose=False))
    assert ep == 3 and m == {"epoch_losses": [1.0]} and eo is None
    assert all(torch.equal(e[k], v) for k, v in enc.state_dict().items())
    assert all(torch.equal(d[k], v) for k, v in dec.state_dict().items())
    assert do is not None


def test_whole_module_checkpoint_round_trip(tmp_path, monkeypatch):
    from models.attention import AttentionDecoder
    from models.encoder import EncoderAttention
    monkeypatch.setattr(C, "CHECKPOINTS_DIR", str(tmp_path))
    enc, dec, opt = _models()
    args = types.SimpleNamespace(model_name="att", checkpoint="att_1.pth.tar")
    C.save_checkpoint(args, 1, enc, dec, None, opt, {}, verbose=False, whole_modules=True)
    size = (tmp_path / "att_1.pth.tar").stat().st_size
    n_state = sum(v.numel() * v.element_size() for v in list(enc.state_dict().values()) + list(dec.state_dict().values()))
    assert size < n_state * 1.5 + (8 << 20), (size, n_state)  # no workspaces / packed-weight caches
    ep, e, d, eo, do, _ = C.unpack_checkpoint(C.load_checkpoint("cpu", args, verbose=False, weights_only=False))
    assert isinstance(e, EncoderAttention) and isinstance(d, AttentionDecoder) and type(do) is type(opt)
    assert e._runner.bf16 and not e._runner.packed.cache  # precision kept, caches rebuilt empty
    for k, v in enc.state_dict().items():
        assert torch.equal(e.state_dict()[k], v), k
    for k, v in dec.state_dict().items():
        assert torch.equal(d.state_dict()[k], v), k
    # optimizer state survives (train() takes .state_dict() of a pickled optimizer)
    sd1, sd2 = opt.state_dict(), do.state_dict()
    assert sd1.keys() == sd2.keys()


@pytest.mark.gpu
def test_whole_module_checkpoint_gpu(tmp_path, monkeypatch):
    """After GPU forwards (launch caches populated), the pickled modules load and give bit-identical
    encoder features and decoder predictions."""
    import gen
    from helpers import t
    monkeypatch.setattr(C, "CHECKPOINTS_DIR", str(tmp_path))
    enc, dec, opt = _models()
    enc._runner.packed.cache.clear()
    enc.set_compute_precision("fp32")
    enc, dec = enc.cuda().eval(), dec.cuda().eval()
    imgs = t(gen.images(3, 2, 64, 64), "cuda")
    caps = torch.randint(1, 46, (2, 6), device="cuda")
    with torch.no_grad():
        f1 = enc(imgs)
        p1 = dec(f1, caps, [6, 6])[0]
    args = types.SimpleNamespace(model_name="att", checkpoint="att_0.pth.tar")
    C.save_checkpoint(args, 0, enc, dec, None, opt, {}, verbose=False, whole_modules=True)
    _, e, d, _, _, _ = C.unpack_checkpoint(C.load_checkpoint("cuda", args, verbose=False, weights_only=False))
    with torch.no_grad():
        f2 = e.eval()(imgs)
        p2 = d.eval()(f2, caps, [6, 6])[0]
    torch.cuda.synchronize()
    assert torch.equal(f1, f2) and torch.equal(p1, p2)


@pytest.mark.parametrize("fmt", ["state_dict", "whole_modules"])
def test_resume_keeps_use_bert(tmp_path, monkeypatch, fmt):
    """train()'s resume branch rebuilds the decoder with the run's --use_bert (the reference
    resumes the pickled module, which keeps it): a BERT checkpoint must not resume on the
    word-embedding path."""
    from models import attention as MA
    from vocabulary import synthetic_vocab
    monkeypatch.setattr(C, "CHECKPOINTS_DIR", str(tmp_path))
    vocab = synthetic_vocab(50)
    args = types.SimpleNamespace(model_name="bert_att", checkpoint=None, fine_tune_encoder=False,
                                 attention_dim=32, decoder_dim=32, embed_size=768, decoder_dropout=0.5,
                                 use_bert=True, use_glove=False, fine_tune_embedding=False)
    enc, dec, _, _, _, _ = MA._build_models(args, vocab, "cpu")
    assert dec.use_bert
    from capmi.optim import Adam
    opt = Adam([p for p in dec.parameters() if p.requires_grad], lr=1e-4)
    C.save_checkpoint(args, 2, enc, dec, None, opt, {}, verbose=False, whole_modules=(fmt == "whole_modules"))
    args.checkpoint = "bert_att_2.pth.tar"
    args.trusted_checkpoint = fmt == "whole_modules"
    enc2, dec2, ep, _, ost, _ = MA._build_models(args, vocab, "cpu")
    assert ep == 3 and dec2.use_bert and ost is not None
    for k, v in dec.state_dict().items():
        assert torch.equal(dec2.state_dict()[k], v), k
