"""GPU, world_size 2 on ONE device (gloo backend, two processes sharing cuda:0): the data-parallel
training steps run end to end (RCCL refuses two ranks on one GPU, and the 8-GPU node is the
driver's), i.e. capmi.train_step's DP logic with real HIP kernels:

  * frozen encoder (config 3), pipelined two-stream step, eager and on HIP graphs (the bench
    default; the all-reduce + update run after the decoder graph's replay): after the step the gradient buffer of
    every rank equals the mean of the per-shard gradients, computed in the same process by the
    non-DP fused path on each shard; parameters are identical on both ranks;
  * encoder fine-tune (config 4), eager and on HIP graph segments: the same for the decoder AND
    the encoder gradient buffers (the decoder bucket all-reduced beside the encoder backward, the
    layer4 / layer3 / layer2 buckets each as the backward leaves that stage).

Equality is to fp32 summation order (rtol 1e-6 relative to max|g|): the only difference is
(g0 + g1) / 2 vs the gloo SUM-then-scale."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _setup(fine_tune, seed=3):
    import gen
    from capmi.optim import Adam
    from helpers import make_decoder, t
    from models.encoder import EncoderAttention
    torch.manual_seed(seed)
    enc = EncoderAttention()
    sd = enc.state_dict()
    names = ["conv1", "bn1", "relu", "maxpool", "layer1", "layer2", "layer3", "layer4"]
    for k, v in gen.resnet101_params(seed).items():
        head, rest = k.split(".", 1)
        sd[f"resnet.{names.index(head)}.{rest}"] = t(v).clone()
    enc.load_state_dict(sd)
    if fine_tune:
        enc.fine_tune(True)
    enc = enc.cuda().train()
    dec, _ = make_decoder(32, 32, 16, 50, seed, "cuda")
    dec.train()
    dopt = Adam([q for q in dec.parameters() if q.requires_grad], lr=1e-4)
    eopt = Adam([q for q in enc.parameters() if q.requires_grad], lr=1e-4) if fine_tune else None
    for o in (dopt, eopt):
        if o is not None:
            o.set_clip(5.0)
    return enc, dec, dopt, eopt


class _Probe:
    """The attributes AttentionTrainStep._feat_layout reads."""

    def __init__(self, enc, fine_tune):
        self.encoder, self.dedup, self.fine_tune = enc, os.environ.get("CAPMI_ATT_DEDUP", "1") != "0", fine_tune


def _worker(rank, world, port, fine_tune, q, graph=False, backend="gloo"):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "image-captioning-with-different-decoders_amd"),
              os.path.dirname(here), os.path.join(here, "golden"), here):
        sys.path.insert(0, p)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), CAPMI_DIST_FORCE="1")
    try:
        import gen
        from capmi import decoder_fn as DF
        from capmi import dist as cdist
        from capmi.train_step import AttentionTrainStep
        from helpers import t
        ctx = cdist.init_from_env("cuda", backend=backend)
        assert ctx.distributed and ctx.backend == backend, (ctx, backend)
        B, L, V = 2, 6, 50
        imgs = t(gen.images(11, B * world, 64, 64), "cuda")
        caps = t(gen.captions(11, B * world, L, V), "cuda")
        # reference: non-DP fused gradients of each shard, on a fresh copy of the same model
        enc, dec, dopt, eopt = _setup(fine_tune)
        ref_d, ref_e = [], []
        for r in range(world):
            sl = slice(r * B, (r + 1) * B)
            g = {n: torch.zeros_like(q) for n, q in dec.named_parameters() if q.requires_grad}
            # same feature layout as the step (the distinct-row map when the pool only repeats
            # pixels), so the two differ only in the all-reduce
            shape, dup = AttentionTrainStep._feat_layout(_Probe(enc, fine_tune), imgs[sl])
            if fine_tune:
                f = enc.ft_forward(imgs[sl], pooled=dup == 1)
                denc = torch.empty_like(f)
                DF.fused_loss_and_grads(dec, f, caps[sl], [L] * B, 1.0, g, denc=denc, dup=dup)
                eg = {id(q): torch.zeros_like(q) for q in enc.parameters() if q.requires_grad}
                enc.ft_backward(denc, eg)
                ref_e.append(torch.cat([eg[id(q)].reshape(-1) for q in enc.parameters() if q.requires_grad]))
            else:
                f = torch.empty(shape, device="cuda")
                with torch.no_grad():
                    AttentionTrainStep._encode_into(_Probe(enc, fine_tune), imgs[sl], f, dup)
                DF.fused_loss_and_grads(dec, f, caps[sl], [L] * B, 1.0, g, dup=dup)
            ref_d.append(torch.cat([g[n].reshape(-1) for n, q in dec.named_parameters() if q.requires_grad]))
        torch.cuda.synchronize()
        # the DP step on this rank's shard (fresh model: BN running stats / weights as above)
        enc, dec, dopt, eopt = _setup(fine_tune)
        step = AttentionTrainStep(enc, dec, dopt, ctx, seed=9, pipeline=not fine_tune, encoder_optimizer=eopt,
                                  graph=graph)
        sl = slice(rank * B, (rank + 1) * B)
        step(imgs[sl], caps[sl], [L] * B)
        step.flush()
        torch.cuda.synchronize()
        got_d = torch.cat([q.grad.reshape(-1) for q in dec.parameters() if q.requires_grad])
        want_d = sum(ref_d) / world
        err_d = float((got_d - want_d).abs().max() / want_d.abs().max())
        err_e = 0.0
        if fine_tune:
            got_e = torch.cat([q.grad.reshape(-1) for q in enc.parameters() if q.requires_grad])
            want_e = sum(ref_e) / world
            err_e = float((got_e - want_e).abs().max() / want_e.abs().max())
        p = torch.cat([q.detach().reshape(-1) for q in dec.parameters()]).cpu()
        if fine_tune:
            p = torch.cat([p, torch.cat([q.detach().reshape(-1) for q in enc.parameters()]).cpu()])
        import hashlib
        digest = hashlib.sha256(p.numpy().tobytes()).hexdigest()  # (a 170 MB tensor does not cross the queue)
        q.put((rank, err_d, err_e, digest, list(step.schedule)))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "error", traceback.format_exc(), None, None))
        raise e
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("fine_tune,graph", [(False, False), (False, True), (True, False), (True, True)])
def test_dp_two_ranks_one_gpu(fine_tune, graph):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, fine_tune, q, graph)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r = q.get(timeout=180)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
    for r in res.values():
        assert r[1] != "error", r[2]
    for r in (0, 1):
        assert res[r][1] < 1e-6, ("decoder grads", res[r][1])
        assert res[r][2] < 1e-6, ("encoder grads", res[r][2])
    assert res[0][3] == res[1][3]  # identical parameters after the update (sha256 of every parameter)


# what a fine-tune step issues, in order: the graph segments (cut where a bucket becomes final) with each
# bucket's all-reduce issued between the segment that finalises it and the next one's replay; eager: the
# same collectives in the same order, issued from inside the backward
_FT_GRAPH_SCHEDULE = ["seg0", "ar:dec", "seg1", "ar:layer4", "seg2", "ar:layer3", "seg3", "ar:layer2", "ar:rest",
                      "update"]
_FT_EAGER_SCHEDULE = ["ar:dec", "ar:layer4", "ar:layer3", "ar:layer2", "ar:rest", "update"]


@pytest.mark.parametrize("fine_tune,graph", [(False, False), (False, True), (True, False), (True, True)])
def test_dp_rccl_one_rank(fine_tune, graph):
    """The RCCL ("nccl" backend) branch of capmi.dist -- init_process_group(device_id=...), the
    async ReduceOp.AVG all-reduce of the flat buffers (the fc bucket beside the BPTT loop, the rest
    after; in fine-tune the decoder's beside the encoder backward and the encoder's per stage) -- at
    world size 1 (CAPMI_DIST_FORCE=1; RCCL refuses two ranks on one GPU). AVG over one rank is the
    identity, so the gradient buffers must equal the non-DP ones bit for bit -- for the segmented
    fine-tune graph too, i.e. cutting the step into segments changes nothing -- and the fine-tune step
    must issue its collectives between the segments that finalise their buckets."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), fine_tune, q, graph, "nccl"))
    p.start()
    r = q.get(timeout=180)
    p.join(timeout=60)
    assert r[1] != "error", r[2]
    assert r[1] == 0.0, ("decoder grads", r[1])
    assert r[2] == 0.0, ("encoder grads", r[2])
    if fine_tune:
        assert r[4] == (_FT_GRAPH_SCHEDULE if graph else _FT_EAGER_SCHEDULE), r[4]


@pytest.mark.parametrize("captured", [False, True])
def test_fc_bucket_cut_is_race_free(captured):
    """The data-parallel step all-reduces the fc gradient bucket (fc.weight, fc.bias and their 256-B
    padding) while the backward-through-time continues (eager: on_fc_grads callback; pipelined graphs:
    AttentionTrainStep._capture_split cuts the decoder graph there). That is race-free only if nothing
    after the cut reads or writes the bucket. Proof without a second GPU: the callback overwrites the
    whole bucket with a sentinel; after the rest of the backward (eager, or the second graph's replay)
    the sentinel must be intact and every other gradient bit-identical to a run without the cut."""
    from capmi import decoder_fn as DF
    from capmi.optim import Adam
    from capmi.train_step import AttentionTrainStep
    from helpers import make_decoder, t
    import gen
    V, B, L, seed = 8100, 8, 25, 61
    dec, _ = make_decoder(512, 512, 512, V, seed, DEV)
    dec.train()
    dec.fine_tune_embeddings(False)
    opt = Adam([q for q in dec.parameters() if q.requires_grad], lr=1e-4)
    named = dict(dec.named_parameters())
    head, rest = opt.grad_buckets({named["fc.weight"], named["fc.bias"]})
    need = [n for n, q in named.items() if q.requires_grad]
    grads = {n: named[n].grad for n in need}
    enc = t(gen.encoder_features(seed, B, P=49), DEV).view(B, 7, 7, 2048)
    caps = t(gen.captions(seed, B, L, V), DEV)
    sentinel = 12345.0

    def body(cut):
        return DF.fused_loss_and_grads(dec, enc, caps, [L] * B, 1.0, grads, need=need, on_fc_grads=cut, dup=2)

    body(None)
    torch.cuda.synchronize()
    want = [r.clone() for r in rest]

    def fill():
        for h in head:
            h.fill_(sentinel)

    for g_ in opt.grad_buffers():
        g_.zero_()
    if not captured:
        body(fill)
    else:
        def cut_and_fill(cut):
            return body(cut)
        _, g1, g2 = AttentionTrainStep._capture_split(cut_and_fill)
        g1.replay()
        fill()
        g2.replay()
    torch.cuda.synchronize()
    for h in head:
        assert bool((h == sentinel).all()), "the backward after the cut touched the fc bucket"
    for r, w in zip(rest, want):
        assert torch.equal(r, w)


@pytest.mark.parametrize("captured", [False, True])
def test_encoder_stage_buckets_cut_is_race_free(captured):
    """The fine-tune step all-reduces each encoder stage's gradient bucket (layer4, then layer3, then layer2)
    while the backward of the lower stages continues (eager: FineTuneRunner.backward's on_layer callback;
    graph mode: segments cut there). Race-free only if nothing launched after a stage's callback reads or
    writes that stage's bucket. Proof on one GPU: at each callback the stage's span is first copied, then
    overwritten whole (padding included) with a sentinel. Every copy must equal the reference gradients bit
    for bit (a lower stage that read a higher stage's bucket would see the sentinel), and after the whole
    backward (eager, or the remaining segments' replays) every sentinel must be intact."""
    from capmi.train_step import AttentionTrainStep
    from helpers import t
    import gen
    enc, dec, dopt, eopt = _setup(True)
    buckets = AttentionTrainStep._stage_buckets(enc, eopt)
    assert all(buckets[f"layer{li}"] for li in (2, 3, 4))
    imgs = t(gen.images(13, 2, 64, 64), "cuda")
    feats = enc.ft_forward(imgs)
    dfeat = torch.rand(feats.shape, device="cuda", generator=torch.Generator(device="cuda").manual_seed(4)) - 0.5
    grads = {id(q): q.grad for q in enc.parameters() if q.requires_grad}
    sentinel = 4321.0
    enc.ft_backward(dfeat, grads)  # (also records the weight-prep jobs: later passes allocate nothing new)
    torch.cuda.synchronize()
    want = {li: [v.clone() for v in buckets[f"layer{li}"]] for li in (2, 3, 4)}
    snap, order = {}, []

    def hand_over(li):
        order.append(li)
        snap[li] = [v.clone() for v in buckets[f"layer{li}"]]
        for v in buckets[f"layer{li}"]:
            v.fill_(sentinel)

    for g_ in eopt.grad_buffers():
        g_.zero_()
    if not captured:
        enc.ft_forward(imgs)
        enc.ft_backward(dfeat, grads, on_layer=hand_over)
    else:
        def body(cut):
            enc.ft_forward(imgs)
            enc.ft_backward(dfeat, grads, on_layer=lambda li: cut(li) if li != 2 else None)
        _, graphs, labels = AttentionTrainStep._capture_segments(body)
        assert labels == [4, 3, None], labels
        for g_ in eopt.grad_buffers():
            g_.zero_()
        for g, lab in zip(graphs, labels):
            g.replay()
            hand_over(lab if lab is not None else 2)
    torch.cuda.synchronize()
    assert order == [4, 3, 2], order
    for li in (2, 3, 4):
        for v, c, w in zip(buckets[f"layer{li}"], snap[li], want[li]):
            assert torch.equal(c, w), f"layer{li}'s gradients differ once the higher stages' buckets are handed over"
            assert bool((v == sentinel).all()), f"the backward after layer{li}'s callback touched its bucket"
