"""Headline benchmark: 'attention' captioner training images/sec on MI355X.

python bench.py --gpus N --steps K --warmup W     (N > 1: launched by torchrun, one rank per GPU)

One step = the reference's training step (models/attention.py:386-430) on a resident
synthetic batch of 64 (image 3x224x224, 25-token caption, V = 8100) per GPU: ResNet-101
encoder forward (frozen, BatchNorm in train mode), 24-step soft-attention decoder
forward + backward, CE + doubly-stochastic loss, (DP: gradient all-reduce over RCCL),
clamp + Adam. fp32 throughout (the reference's precision). Weights: torch.manual_seed(0)
random init of the reference architecture (no checkpoints offline).

Default launch: pipelined over two HIP streams, each replaying captured HIP graphs -- call k runs the frozen encoder of batch k
beside the decoder step of batch k-1 (bit-identical to the sequential order; the K timed
calls run exactly K encoder passes and K decoder/optimizer passes: the pipeline is filled in
warm-up and drained after the clock stops). ``--sequential`` runs the whole step as one HIP
graph instead.

Rank 0 prints ONE JSON line. ``roofline`` is for the dominant kernel: the conv implicit-GEMM
instantiation with the most time per step (the conv family is 86% of the step's FLOPs; the
family aggregate is reported beside it). achieved = that kernel's algorithmic conv FLOPs /
its summed launch time, HIP events on the launch stream around every conv launch.
``cpu_baseline`` times the CPU oracle (op-for-op restatement of the reference step) on
the host cores, rank 0 at N = 1 only, on a small bounded sample.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "image-captioning-with-different-decoders_amd")
for _p in (PKG, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

FP32_MFMA_PEAK_TF = 157.3   # MI355X fp32 matrix peak (MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TF = 2500.0  # MI355X dense bf16 matrix peak (MI355X_MICROARCH.md; no sparsity)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="per-GPU batch")
    ap.add_argument("--caption-len", type=int, default=25)
    ap.add_argument("--vocab", type=int, default=8100)
    ap.add_argument("--no-roofline", action="store_true", help="skip per-conv event timing")
    ap.add_argument("--sequential", action="store_true",
                    help="no encoder/decoder pipelining: the whole step in one HIP graph (or --eager)")
    ap.add_argument("--eager", action="store_true",
                    help="with --sequential: launch every kernel from Python (no HIP graph)")
    ap.add_argument("--config", default="attention", choices=["attention", "glove_finetune", "bert_attention"],
                    help="attention = BASELINE config 2/3 (frozen encoder, the headline); glove_finetune = "
                         "config 4 (GloVe-300 fp64 embedding fine-tuned + encoder layer2-4 fine-tuned); "
                         "bert_attention = config 5 (768-d word features instead of the table, synthetic)")
    ap.add_argument("--fp32", action="store_true", help="bert_attention: keep the encoder convs fp32")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    return ap.parse_args()


class ConvTimer:
    """HIP-event bracket around every conv GEMM launch (on the launch stream), per kernel."""

    def __init__(self):
        self.events = []  # (kernel key, flops, start event, end event)
        self.enabled = False

    def __call__(self, tag, flops, launch, key):
        if not self.enabled:
            launch()
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        launch()
        e.record()
        self.events.append((key, flops, s, e))

    def result(self):
        """{kernel key: [launches, flops, ms]} and the family total."""
        per = {}
        for key, f, s, e in self.events:
            ent = per.setdefault(key, [0, 0.0, 0.0])
            ent[0] += 1
            ent[1] += f
            ent[2] += s.elapsed_time(e)
        return per


def _traffic_file(config):
    """The committed PMC summary of ``config``'s own run (a kernel name can stand for different
    shapes in different configs, so each config reads only its own passes)."""
    return "r01_pmc_traffic.json" if config == "attention" else f"r01_pmc_traffic_{config}.json"


def _traffic(kernel, config="attention"):
    """HBM bytes per launch of ``kernel`` from the committed PMC summary of this config's run
    (2*FETCH_SIZE + WRITE_SIZE, gfx950 correction; tools/pmc_traffic.py), or None."""
    path = os.path.join(REPO, "profiles", _traffic_file(config))
    try:
        with open(path) as f:
            tab = json.load(f)
    except (OSError, ValueError):
        return None
    ent = tab.get("kernels", {}).get(kernel)
    return None if ent is None else ent.get("hbm_bytes_per_launch")


def cpu_baseline(args, seconds):
    """Oracle (CPU restatement of the reference step) on a bounded sample: B=2, full
    ResNet-101 encoder forward + the unhoisted 24-step decoder fwd/bwd + clamp + Adam."""
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import gen
    from oracle import decoder_ref as R
    from oracle.resnet_ref import build_resnet101, encoder_attention_forward
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    B, L, V = 2, args.caption_len, args.vocab
    bert = args.config == "bert_attention"
    M = 768 if bert else 512
    net = build_resnet101(gen.resnet101_params(5)).train()
    p = {k: torch.from_numpy(v) for k, v in gen.decoder_params(5, 512, 512, M, V).items()}
    trainable = set(k for k in p if k != "embedding.weight")
    imgs = torch.from_numpy(gen.images(5, B))
    caps = torch.from_numpy(gen.captions(5, B, L, V))
    emb = None
    if bert:
        from capmi.data import SyntheticBertEmbedder
        emb = SyntheticBertEmbedder(V, 768)(caps)
    state, n, t0 = {}, 0, None
    while True:
        with torch.no_grad():
            feats = encoder_attention_forward(net, imgs)
        out = R.train_step(p, trainable, feats, caps, [L] * B, state=state, embeddings=emb)
        p.update(out[5])
        state = out[6]
        n += 1
        if t0 is None:          # first step is warm-up
            t0, n = time.perf_counter(), 0
        elif time.perf_counter() - t0 > seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": round(B * n / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} oracle train steps at B={B} (ResNet-101 fwd + unhoisted decoder fwd/bwd + "
                      f"clamp/Adam, L={L}, V={V}, M={M}), torch CPU fp32, {threads} threads, {dt:.1f} s"}


def cpu_baseline_finetune(args, seconds):
    """Oracle fine-tune step (oracle/finetune_ref.py: ResNet-101 fwd+bwd of layer2-4, decoder
    fwd/bwd with fp64 GloVe-300 embedding, clamp + two Adams) at B=2 on the host cores."""
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import gen
    from oracle.finetune_ref import finetune_train_step
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    B, L, V = 2, args.caption_len, args.vocab
    rp = gen.resnet101_params(5)
    p = {k: torch.from_numpy(v) for k, v in gen.decoder_params(5, 512, 512, 300, V, emb_dtype=np.float64).items()}
    imgs = torch.from_numpy(gen.images(5, B))
    caps = torch.from_numpy(gen.captions(5, B, L, V))
    n, t0 = 0, None
    while True:
        finetune_train_step(rp, p, set(p), imgs, caps, [L] * B)
        n += 1
        if t0 is None:
            t0, n = time.perf_counter(), 0
        elif time.perf_counter() - t0 > seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": round(B * n / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} oracle fine-tune train steps at B={B} (ResNet-101 fwd + layer2-4 bwd, unhoisted "
                      f"decoder fwd/bwd, fp64 GloVe-300 embedding, clamp/2x Adam, L={L}, V={V}), torch CPU fp32, "
                      f"{threads} threads, {dt:.1f} s"}


def main():
    args = parse()
    from capmi import dist as cdist
    ctx = cdist.init_from_env("cuda")
    dev = ctx.device
    from capmi.data import synthetic_batch
    from capmi.optim import Adam
    from capmi.train_step import AttentionTrainStep
    from models.attention import AttentionDecoder, AttentionDecoderParams
    from models.encoder import EncoderAttention
    from vocabulary import synthetic_vocab

    torch.manual_seed(0)
    ft = args.config == "glove_finetune"
    bert = args.config == "bert_attention"
    encoder = EncoderAttention().to(dev).train()
    prm = AttentionDecoderParams()
    prm.vocab = synthetic_vocab(args.vocab)
    prm.embed_size = 300 if ft else (768 if bert else 512)
    prm.use_bert = bert
    decoder = AttentionDecoder(dev, prm)
    if bert:
        from capmi.data import SyntheticBertEmbedder
        decoder.bert_embedder = SyntheticBertEmbedder(args.vocab, 768, device=dev)
        if not args.fp32:
            encoder.set_compute_precision("bf16")  # config 5 is the bf16 config
    if ft:
        # synthetic GloVe-300 table, fp64 like load_glove_vectors (embed.py:64-68, Q7)
        g = torch.Generator().manual_seed(300)
        decoder.load_pretrained_embeddins((torch.rand(args.vocab, 300, generator=g, dtype=torch.float64) - 0.5))
    decoder = decoder.to(dev).train()
    # glove_att: --fine_tune_embedding True (Makefile:13); bert: the table is unused; else Q8 default
    decoder.fine_tune_embeddings(ft)
    cdist.broadcast_module(decoder, ctx)
    opt = Adam(filter(lambda q: q.requires_grad, decoder.parameters()), lr=1e-4)
    opt.set_clip(5.0)
    enc_opt = None
    if ft:
        encoder.fine_tune(True)
        cdist.broadcast_module(encoder, ctx)
        enc_opt = Adam(filter(lambda q: q.requires_grad, encoder.parameters()), lr=1e-4)
        enc_opt.set_clip(5.0)
    pipe = not args.sequential and not ft
    step = AttentionTrainStep(encoder, decoder, opt, ctx, alpha_c=1.0, graph=not args.eager,
                              seed=77 + ctx.rank, pipeline=pipe, encoder_optimizer=enc_opt)
    timer = ConvTimer()
    encoder._runner.conv_hook = None if args.no_roofline else timer
    B = args.batch
    imgs, caps, lens = synthetic_batch(B, args.caption_len, args.vocab, dev, seed=1234 + ctx.rank)

    for _ in range(args.warmup):
        step(imgs, caps, lens)
    if not pipe:  # pipelined: keep one encoder pass in flight (its decoder runs in timed step 1)
        step.flush()
    torch.cuda.synchronize()
    cdist.barrier(ctx)
    torch.cuda.synchronize()
    timer.enabled = args.eager and not args.no_roofline
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step(imgs, caps, lens)
    if not pipe:
        step.flush()
    torch.cuda.synchronize()
    cdist.barrier(ctx)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    timer.enabled = False
    dt = cdist.max_over_ranks(dt, ctx)
    if pipe:  # K encoder and K decoder passes were timed; drain the in-flight encoder pass
        step.flush()
        torch.cuda.synchronize()
    loss_v = float(loss.item())
    if pipe and not args.eager and not args.no_roofline:
        # graph replays cannot bracket single kernels: time the conv launches of `steps` more
        # pipelined steps launched eagerly (the encoder sharing the GPU with the decoder as in
        # the timed region), right after it
        step2 = AttentionTrainStep(encoder, decoder, opt, ctx, alpha_c=1.0, graph=False, seed=99 + ctx.rank,
                                   pipeline=True)
        step2(imgs, caps, lens)
        torch.cuda.synchronize()
        timer.enabled = True
        for _ in range(args.steps):
            step2(imgs, caps, lens)
        torch.cuda.synchronize()
        timer.enabled = False
        step2.flush()
        torch.cuda.synchronize()
    elif not (args.eager or pipe) and not args.no_roofline:
        # graph replays cannot bracket single kernels: time the same conv launches (same shapes,
        # same inputs) in eager encoder forwards right after the timed region
        timer.enabled = True
        with torch.no_grad():
            for _ in range(args.steps):
                if ft:  # fine-tune: the forward and the layer2-4 backward GEMMs
                    f = encoder.ft_forward(imgs)
                    encoder.ft_backward(torch.ones_like(f) * 1e-4, {id(q): q.grad for q in enc_opt.param_groups[0]["params"]},
                                        hook=timer)
                else:
                    encoder(imgs)
        torch.cuda.synchronize()
        timer.enabled = False

    N = ctx.world
    value = N * B * args.steps / dt
    roof = None
    if not args.no_roofline and timer.events:
        per = timer.result()
        # the dominant kernel: the conv GEMM instantiation with the most time
        key = max(per, key=lambda k: per[k][2])
        n, flops, ms = per[key]
        ach = flops / (ms * 1e-3) / 1e12
        fam_flops = sum(v[1] for v in per.values())
        fam_ms = sum(v[2] for v in per.values())
        per_img = sum(v[1] for v in per.values()) / args.steps / B
        peak = BF16_MFMA_PEAK_TF if encoder._runner.bf16 else FP32_MFMA_PEAK_TF
        roof = {"bound": "mfma", "achieved": round(ach, 3), "peak": peak, "unit": "TFLOP/s",
                "frac": round(ach / peak, 4), "traffic": _traffic(key, args.config),
                "kernel": key,
                "launches_per_step": n // args.steps,
                "flops_per_launch": round(flops / n), "avg_launch_us": round(ms * 1e3 / n, 2),
                "traffic_unit": f"HBM bytes per launch (2*FETCH_SIZE + WRITE_SIZE, profiles/{_traffic_file(args.config)})",
                "conv_family": {"achieved_tflops": round(fam_flops / (fam_ms * 1e-3) / 1e12, 3),
                                "frac": round(fam_flops / (fam_ms * 1e-3) / 1e12 / peak, 4),
                                "conv_ms_per_step": round(fam_ms / args.steps, 3),
                                "conv_gflop_per_image": round(per_img / 1e9, 3)},
                "timing": "HIP events around each conv launch on its stream, " + (
                    "inside the timed steps (pipelined, eager: while the decoder step shares the GPU)"
                    if pipe and args.eager else
                    f"{args.steps} eagerly launched pipelined steps after the timed graph replays (the decoder "
                    "step sharing the GPU as in the timed region)" if pipe else
                    "inside the timed steps" if args.eager else
                    f"{args.steps} eager encoder forwards after the timed graph replays")}
    cpu = None
    if ctx.rank == 0 and N == 1 and not args.no_cpu_baseline:
        cpu = (cpu_baseline_finetune if ft else cpu_baseline)(args, args.cpu_seconds)
    if ctx.rank == 0:
        line = {
            "metric": "training images/sec (whole node), 'attention' decoder, at 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "images/s", "n_gpus": N, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if encoder._runner.bf16 else "fp32",
            "data": "synthetic (resident in HBM; random-init weights, torch.manual_seed(0))",
            "config": {"workload": ("'glove_att' decoder (GloVe-300 fp64 embedding, fine-tuned) + ResNet-101 "
                                    "encoder fine-tuned (layer2-4, BN train mode), one training step per batch")
                       if ft else ("'bert_attention' decoder (768-d synthetic BERT word features) + frozen "
                                   "ResNet-101 encoder (BN train mode), one training step per batch" +
                                   ("; encoder convs bf16 MFMA (fp32 accumulate), decoder fp32 (the reference "
                                    "forces fp32 at the LSTM input)" if encoder._runner.bf16 else "")) if bert else
                       ("'attention' decoder + frozen ResNet-101 encoder (BN train mode), "
                        "one training step per batch"),
                       "per_gpu_batch": B, "global_batch": B * N,
                       "caption_len": args.caption_len, "decode_steps": args.caption_len - 1,
                       "vocab": args.vocab, "attention_dim": 512, "decoder_dim": 512, "embed_size": prm.embed_size,
                       "parallelism": f"dp{N}"},
            "loss_last_step": round(loss_v, 5),
            "launch": ("pipelined_2stream_eager" if args.eager else "pipelined_2stream_hip_graphs") if pipe
            else ("eager" if args.eager else "hip_graph"),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
