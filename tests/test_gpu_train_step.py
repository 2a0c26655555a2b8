"""GPU: the whole training step (encoder + decoder + fused loss + clamp/Adam) through
AttentionTrainStep, eager vs HIP-graph replay, and against the oracle step."""
import copy

import numpy as np
import pytest
import torch

import gen
from helpers import assert_close, make_decoder, t

pytestmark = pytest.mark.gpu
DEV = "cuda"
NAMES = ["conv1", "bn1", "relu", "maxpool", "layer1", "layer2", "layer3", "layer4"]


def _encoder(seed):
    from models.encoder import EncoderAttention
    params = gen.resnet101_params(seed)
    enc = EncoderAttention()
    sd = enc.state_dict()
    for k, v in params.items():
        head, rest = k.split(".", 1)
        sd[f"resnet.{NAMES.index(head)}.{rest}"] = torch.from_numpy(v).clone()
    enc.load_state_dict(sd)
    return enc.to(DEV).train()


def _setup(dropout):
    from capmi.optim import Adam
    from capmi.train_step import AttentionTrainStep
    enc = _encoder(3)
    dec, _ = make_decoder(32, 32, 16, 50, 9, DEV, dropout=dropout)
    dec.fine_tune_embeddings(False)  # reference default; keeps the step free of atomics
    dec.train()
    opt = Adam([q for q in dec.parameters() if q.requires_grad], lr=1e-3)
    opt.set_clip(5.0)
    return enc, dec, opt, AttentionTrainStep


@pytest.mark.parametrize("dropout", [0.0, 0.5])
def test_graph_replay_equals_eager(dropout):
    B, L, V = 4, 7, 50
    imgs = t(gen.images(5, B, 64, 64), DEV)
    caps = t(gen.captions(5, B, L, V), DEV)
    lens = [L] * B
    res = {}
    for mode in ("eager", "graph"):
        enc, dec, opt, Step = _setup(dropout)
        step = Step(enc, dec, opt, alpha_c=1.0, graph=(mode == "graph"), seed=123)
        losses = [float(step(imgs, caps, lens)) for _ in range(3)]
        torch.cuda.synchronize()
        res[mode] = (losses, {n: q.detach().clone() for n, q in dec.named_parameters()}, opt.step_count,
                     {k: v.clone() for k, v in enc.state_dict().items() if "running" in k or "num_batches" in k})
    le, pe, se, re_ = res["eager"]
    lg, pg, sg, rg = res["graph"]
    assert se == sg == 3
    # the capture warm-ups' BN running-stat updates and dropout-seed advances are rolled back:
    # the replayed sequence is the eager one bit for bit, dropout masks and running stats included
    np.testing.assert_allclose(lg, le, rtol=0, atol=0)
    for n in pe:
        assert torch.equal(pe[n], pg[n]), n
    for k in re_:
        assert torch.equal(re_[k], rg[k]), k


def test_train_step_matches_oracle_end_to_end():
    """Encoder (train-mode BN) -> decoder -> loss -> clamp/Adam vs the oracle chain on CPU."""
    from oracle import decoder_ref as R
    from oracle.resnet_ref import build_resnet101, encoder_attention_forward
    B, L, V = 2, 6, 50
    enc, dec, opt, Step = _setup(0.0)
    p0 = {n: q.detach().cpu().clone() for n, q in dec.named_parameters()}
    imgs = gen.images(6, B, 64, 64)
    caps = gen.captions(6, B, L, V)
    step = Step(enc, dec, opt, alpha_c=1.0, graph=False, seed=1)
    loss = step(t(imgs, DEV), t(caps, DEV), [L] * B)
    torch.cuda.synchronize()
    net = build_resnet101(gen.resnet101_params(3)).train()
    with torch.no_grad():
        feats = encoder_attention_forward(net, t(imgs))
    trainable = set(n for n, q in dec.named_parameters() if q.requires_grad)
    rl, _, _, _, _, rnew, _ = R.train_step(p0, trainable, feats, t(caps), [L] * B, lr=1e-3)
    # train-mode BN at 64x64 input is ill-conditioned (layer4 has 2x2 pixels): loose loss check,
    # and the Adam step (~lr*sign(g)) is compared where the oracle moved a weight by > lr/2
    assert abs(float(loss) - float(rl)) < 1e-3 * abs(float(rl))
    named = dict(dec.named_parameters())
    for n in ("fc.weight", "decode_step.weight_hh", "attention.dec_att.weight"):
        upd = named[n].detach().cpu() - p0[n]
        rupd = rnew[n] - p0[n]
        big = rupd.abs() > 5e-4
        agree = (torch.sign(upd[big]) == torch.sign(rupd[big])).float().mean().item()
        assert agree > 0.99, (n, agree)
    _ = copy


@pytest.mark.parametrize("dropout", [0.0, 0.5])
def test_pipelined_equals_eager(dropout):
    """Two-stream pipelined step (encoder of batch k beside the decoder step of batch k-1) gives
    bit-identical losses and parameters to the sequential step on the same batch sequence."""
    B, L, V = 4, 7, 50
    batches = [(t(gen.images(20 + i, B, 64, 64), DEV), t(gen.captions(20 + i, B, L, V), DEV)) for i in range(3)]
    res = {}
    for mode in ("eager", "pipe"):
        enc, dec, opt, Step = _setup(dropout)
        step = Step(enc, dec, opt, alpha_c=1.0, graph=False, seed=9, pipeline=(mode == "pipe"))
        # eager/graph calls return the step's loss buffer (overwritten by the next call): clone
        # it; the pipelined step returns its own copy, produced on the decoder stream (read it
        # only after synchronizing)
        out = []
        for im, cp in batches:
            x = step(im, cp, [L] * B)
            out.append(x.clone() if mode == "eager" else x)
        last = step.flush()
        torch.cuda.synchronize()
        losses = [float(x) for x in out if x is not None] + ([float(last)] if last is not None else [])
        res[mode] = (losses, {n: q.detach().clone() for n, q in dec.named_parameters()},
                     {k: v.clone() for k, v in enc.state_dict().items() if "running" in k})
    le, pe, re_ = res["eager"]
    lp, pp, rp = res["pipe"]
    assert len(le) == len(lp) == 3
    np.testing.assert_array_equal(np.array(lp), np.array(le))
    for n in pe:
        assert torch.equal(pe[n], pp[n]), n
    for k in re_:
        assert torch.equal(re_[k], rp[k]), k


@pytest.mark.parametrize("dropout", [0.0, 0.5])
def test_pipelined_graphs_equal_eager(dropout):
    """Pipelined step with both streams replaying captured HIP graphs (the bench default) gives
    bit-identical losses, decoder parameters and encoder BN running statistics to the eager
    sequential step (the capture warm-ups' effects on the running statistics and the dropout
    seed counter are rolled back)."""
    B, L, V = 4, 7, 50
    batches = [(t(gen.images(40 + i, B, 64, 64), DEV), t(gen.captions(40 + i, B, L, V), DEV)) for i in range(4)]
    res = {}
    for mode in ("eager", "pipe_graph"):
        enc, dec, opt, Step = _setup(dropout)
        step = Step(enc, dec, opt, alpha_c=1.0, graph=(mode != "eager"), seed=9, pipeline=(mode != "eager"))
        out = []
        for im, cp in batches:
            x = step(im, cp, [L] * B)
            out.append(x.clone() if mode == "eager" else x)
        last = step.flush()
        torch.cuda.synchronize()
        losses = [float(x) for x in out if x is not None] + ([float(last)] if last is not None else [])
        res[mode] = (losses, {n: q.detach().clone() for n, q in dec.named_parameters()},
                     {k: v.clone() for k, v in enc.state_dict().items() if "running" in k or "num_batches" in k})
    le, pe, re_ = res["eager"]
    lp, pp, rp = res["pipe_graph"]
    assert len(le) == len(lp) == 4
    np.testing.assert_array_equal(np.array(lp), np.array(le))
    for n in pe:
        assert torch.equal(pe[n], pp[n]), n
    for k in re_:
        assert torch.equal(re_[k], rp[k]), k


def test_pipelined_inputs_freed_and_reallocated():
    """The pipelined step reads the caller's image / caption tensors on its side streams. Drop
    each batch's tensors right after the call and allocate the next batch on the caller's stream
    with no synchronisation (the allocator may hand out the same blocks): the losses and
    parameters must equal the sequential step's on the same batch contents."""
    B, L, V = 4, 7, 50
    host = [(gen.images(60 + i, B, 64, 64), gen.captions(60 + i, B, L, V)) for i in range(5)]
    res = {}
    for mode in ("eager", "pipe", "pipe_graph"):
        enc, dec, opt, Step = _setup(0.0)
        step = Step(enc, dec, opt, alpha_c=1.0, graph=(mode == "pipe_graph"), seed=9, pipeline=(mode != "eager"))
        out = []
        for im, cp in host:
            imgs = t(im, DEV)          # fresh device blocks each call, on the caller's stream
            caps = t(cp, DEV)
            x = step(imgs, caps, [L] * B)
            out.append(x.clone() if mode == "eager" else x)
            del imgs, caps            # freed while the side streams may still be reading them
            junk = torch.full((B * 3 * 64 * 64 + B * L,), 7.0, device=DEV)  # reuse the blocks at once
            del junk
        last = step.flush()
        torch.cuda.synchronize()
        losses = [float(x) for x in out if x is not None] + ([float(last)] if last is not None else [])
        res[mode] = (losses, {n: q.detach().clone() for n, q in dec.named_parameters()})
    le, pe = res["eager"]
    for mode in ("pipe", "pipe_graph"):
        lp, pp = res[mode]
        np.testing.assert_array_equal(np.array(lp), np.array(le), err_msg=mode)
        for n in pe:
            assert torch.equal(pe[n], pp[n]), (mode, n)


@pytest.mark.parametrize("pipeline", [False, True])
def test_graph_cache_over_mixed_shapes_equals_eager(pipeline):
    """Per-shape graph cache: batches of three shapes (image side 64 / 96, caption length 7 / 9) in an
    interleaved order are each captured once and replayed from then on -- every replay running on the
    workspaces its own capture pinned, although later shapes replace the workspace caches -- and a cache of
    two shapes runs the third shape eagerly. Losses, decoder parameters and BN running statistics equal the
    eager sequential step's bit for bit."""
    B, V = 4, 50
    shapes = [(64, 7), (96, 7), (64, 9), (64, 7), (96, 7), (64, 9), (96, 7), (64, 7)]
    batches = [(t(gen.images(80 + i, B, s, s), DEV), t(gen.captions(80 + i, B, L, V), DEV), L)
               for i, (s, L) in enumerate(shapes)]
    res = {}
    for mode in ("eager", "graph", "graph_cap2"):
        enc, dec, opt, Step = _setup(0.5)
        step = Step(enc, dec, opt, alpha_c=1.0, graph=(mode != "eager"), seed=9, pipeline=pipeline and mode != "eager")
        if mode == "graph_cap2":
            step.graph_cache_size = 2
        out = []
        for im, cp, L in batches:
            x = step(im, cp, [L] * B)
            out.append(x.clone() if not step.pipeline else x)
        last = step.flush()
        torch.cuda.synchronize()
        losses = [float(x) for x in out if x is not None] + ([float(last)] if last is not None else [])
        res[mode] = (losses, {n: q.detach().clone() for n, q in dec.named_parameters()},
                     {k: v.clone() for k, v in enc.state_dict().items() if "running" in k or "num_batches" in k},
                     dict(step.counts))
    le, pe, re_, _ = res["eager"]
    assert len(le) == len(batches)
    for mode, (cap, rep) in (("graph", (3, 8)), ("graph_cap2", (2, 6))):
        lg, pg, rg, cnt = res[mode]
        assert cnt["capture"] == cap and cnt["replay"] == rep, (mode, cnt)
        np.testing.assert_array_equal(np.array(lg), np.array(le), err_msg=mode)
        for n in pe:
            assert torch.equal(pe[n], pg[n]), (mode, n)
        for k in re_:
            assert torch.equal(re_[k], rg[k]), (mode, k)


def test_train_loop_replays_graphs_and_equals_eager(tmp_path, monkeypatch):
    """models.attention.train() runs the launch mode bench.py measures (pipelined HIP-graph
    replay). Over a synthetic fixed-length dataset it captures once and replays every later batch, and its
    logged losses equal those of CAPMI_TRAIN_GRAPH=0 (eager pipelined launches) bit for bit."""
    import types
    import checkpoint as C
    from models import attention as A
    monkeypatch.setattr(C, "CHECKPOINTS_DIR", str(tmp_path / "ck"))
    losses, counts = {}, {}
    for mode in ("0", "1"):
        monkeypatch.setenv("CAPMI_TRAIN_GRAPH", mode)
        torch.manual_seed(0)
        args = types.SimpleNamespace(
            model_name=f"syn{mode}", model="attention", attention_dim=32, decoder_dim=32, decoder_dropout=0.5,
            embed_size=16, epochs=1, batch_size=4, workers=0, encoder_lr=1e-4, decoder_lr=1e-4, grad_clip=5.0,
            alpha_c=1.0, fine_tune_encoder=False, fine_tune_embedding=False, checkpoint=None, print_freq=2,
            use_glove=False, max_caption_length=-1, use_bert=False, synthetic=True, synthetic_size=20,
            synthetic_len=9, vocab_size=50, trusted_checkpoint=False)
        A.train(torch.device(DEV), args)
        ck = torch.load(tmp_path / "ck" / f"syn{mode}_0.pth.tar", weights_only=True)
        losses[mode] = ck["metrics"]["epoch_losses"][0]
        step = A.train.last_step
        counts[mode] = dict(step.counts)
        assert step.pipeline and step.pipe_graph == (mode == "1")
    assert len(losses["1"]) == 5 and all(np.isfinite(losses["1"]))
    assert counts["1"]["capture"] == 1 and counts["1"]["replay"] == 5 and counts["1"]["eager"] == 0, counts
    assert counts["0"]["replay"] == 0, counts
    np.testing.assert_array_equal(np.array(losses["1"]), np.array(losses["0"]))
