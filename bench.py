"""Headline benchmark: 'attention' captioner training images/sec on MI355X.

python bench.py --gpus N --steps K --warmup W

N > 1: one rank per GPU over RCCL. Under torchrun (WORLD_SIZE set) the ranks are the launcher's;
without it, this process starts ``python -m torch.distributed.run --nproc-per-node N`` on itself
as a CHILD process before anything touches the GPU, waits for it and exits with its code (it
never exec()s). Every rank checks that the world size equals --gpus.

One step = the reference's training step (models/attention.py:386-430) on a resident
synthetic batch of 64 (image 3x224x224, 25-token caption, V = 8100) per GPU: ResNet-101
encoder forward (frozen, BatchNorm in train mode), 24-step soft-attention decoder
forward + backward, CE + doubly-stochastic loss, (DP: gradient all-reduce over RCCL),
clamp + Adam. Arithmetic (defaults --conv x3 --dec auto): fp32 activations, statistics and
optimizer state; the convs and the decoder GEMMs run "x3" -- every fp32 operand split exactly into
three bf16 terms whose six significant cross products accumulate in fp32 on the bf16 matrix cores
(error against fp64 at or below the fp32-MFMA kernel's: tests/test_gpu_x3.py, tests/test_gpu_finetune.py);
``--conv native --dec fp32`` reproduces the plain fp32 MFMA arithmetic (v_mfma_f32_32x32x2_f32). The
decoder runs on the 49 distinct rows of the 7x7 layer4 map, which AdaptiveAvgPool2d(14) only repeats
(exact; ``config.decoder_rows`` in the line). Weights: torch.manual_seed(0) random init
of the reference architecture (no checkpoints offline).

Default launch: pipelined over two HIP streams, each replaying captured HIP graphs -- call k runs the frozen encoder of batch k
beside the decoder step of batch k-1 (bit-identical to the sequential order; the K timed
calls run exactly K encoder passes and K decoder/optimizer passes: the pipeline is filled in
warm-up and drained after the clock stops). ``--sequential`` runs the whole step as one HIP
graph instead.

Rank 0 prints ONE JSON line. ``roofline`` is for the dominant kernel: the conv implicit-GEMM
instantiation with the most time per step (the conv family is 86% of the step's FLOPs; the
family aggregate is reported beside it). achieved = that kernel's algorithmic conv FLOPs /
its summed launch time. The launch times come from a timing pass right after the timed region:
--steps more eager calls of the step, every conv GEMM with a pair of HIP events that receive its
dispatch's own start / end timestamps (capmi_timing_arm -> hipExtLaunchKernel: the duration
rocprofv3 reports for that dispatch), encoder and decoder on one stream -- the condition a rocprofv3
kernel trace runs the bench in (its tracing serializes the two streams), so the committed trace
summary of the same command gives the same per-launch average. ``roofline.in_pipeline`` repeats the
pass with the timed region's two-stream pipelining: the same kernel slowed by the decoder's kernels.
``cpu_baseline`` times the CPU oracle (op-for-op restatement of the reference step) on the
host cores, rank 0 at N = 1 only: the full batch (64 images) for at least one step.

``--config baseline_cpu`` is BASELINE config 1 (the 'baseline' LSTM captioner at batch 4 on
the CPU, the reference's plumbing config): torch CPU modules, gloo for N > 1 (the CPU tests
drive the multi-rank launch through it).
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
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default 64; baseline_cpu: 4)")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--caption-len", type=int, default=25)
    ap.add_argument("--vocab", type=int, default=8100)
    ap.add_argument("--no-roofline", action="store_true", help="skip per-conv event timing")
    ap.add_argument("--sequential", action="store_true",
                    help="no encoder/decoder pipelining: the whole step in one HIP graph (or --eager)")
    ap.add_argument("--eager", action="store_true",
                    help="with --sequential: launch every kernel from Python (no HIP graph)")
    ap.add_argument("--config", default="attention",
                    choices=["attention", "glove_finetune", "bert_attention", "baseline_cpu"],
                    help="attention = BASELINE config 2/3 (frozen encoder, the headline); glove_finetune = "
                         "config 4 (GloVe-300 fp64 embedding fine-tuned + encoder layer2-4 fine-tuned); "
                         "bert_attention = config 5 (768-d word features instead of the table, synthetic); "
                         "baseline_cpu = config 1 (baseline LSTM captioner, batch 4, CPU, gloo)")
    ap.add_argument("--fp32", action="store_true", help="bert_attention: keep the encoder convs fp32")
    ap.add_argument("--conv", default="x3", choices=["x3", "native"],
                    help="fp32 configs: x3 = fp32-accurate convs on the bf16 matrix cores (operands split exactly "
                         "into three bf16 terms, six cross products accumulated in fp32; gemm_x3*.hip), native = "
                         "v_mfma_f32_32x32x2_f32")
    ap.add_argument("--dec", default="auto", choices=["auto", "x3", "fp32", "bf16"],
                    help="decoder GEMM arithmetic (AttentionDecoder.set_compute_precision): auto = bf16 for the "
                         "bf16 config, else x3 (fp32-accurate three-term split on the bf16 matrix cores: 1.80 vs "
                         "1.92 ms of decoder GEMMs per step, +0.4 %% img/s); fp32 = v_mfma_f32_32x32x2_f32")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0,
                    help="cpu_baseline: keep stepping the oracle at the full batch until this much time "
                         "has passed (at least one step)")
    ap.add_argument("--master-port", type=int, default=0, help="N > 1 self-launch: rendezvous port (0: free)")
    args = ap.parse_args()
    if args.batch is None:
        args.batch = 4 if args.config == "baseline_cpu" else 64
    return args


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """--gpus N > 1 outside torchrun: run torch.distributed.run on this script as a child process
    (nothing has touched the GPU yet in this process) and return its exit code."""
    import subprocess
    port = args.master_port or _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between processes)
    return subprocess.call(cmd, env=env)


class ConvTimer:
    """Times every conv GEMM launch of the timing pass, per kernel: each launch (eager) gets a pair of
    HIP timing events that record its dispatch's own start and end timestamps
    (capmi.kernels.timed_launch -> capmi_timing_arm -> hipExtLaunchKernel), i.e. the kernel duration
    rocprofv3 reports for that dispatch -- no event packets between kernels, so no per-measurement
    overhead. Launches under graph capture, or while disabled, run untimed."""

    def __init__(self):
        self.events = []  # (kernel key, flops, start event, end event)
        self.enabled = False
        self.checked = 0
        self.mismatch = set()  # (priced key, launched instantiation) pairs that differ

    def __call__(self, tag, flops, launch, key):
        if not self.enabled or torch.cuda.is_current_stream_capturing():
            launch()
            return
        from capmi.kernels import TimingEvent, last_launch_name, timed_launch
        s, e = TimingEvent(), TimingEvent()
        timed_launch(launch, s, e)
        # the name this launch is priced under (the planner's plan query) against the instantiation the launcher
        # actually ran (capmi_last_launch_name): roofline.kernel / traffic attribution cannot drift from the planner
        self.checked += 1
        got = last_launch_name()
        if got != key:
            self.mismatch.add((key, got))
        self.events.append((key, flops, s, e))

    def result(self):
        """{kernel key: [launches, flops, ms]} (synchronize first)."""
        per = {}
        for key, f, s, e in self.events:
            ent = per.setdefault(key, [0, 0.0, 0.0])
            ent[0] += 1
            ent[1] += f
            ent[2] += s.elapsed_ms(e)
        return per


def _traffic_file(config):
    """The committed PMC summary of ``config``'s own run (a kernel name can stand for different
    shapes in different configs, so each config reads only its own passes); the newest round's."""
    name = "pmc_traffic.json" if config == "attention" else f"pmc_traffic_{config}.json"
    rounds = sorted((f.split("_", 1)[0] for f in os.listdir(os.path.join(REPO, "profiles"))
                     if f.endswith("_" + name) and f[0] == "r" and f.split("_", 1)[0][1:].isdigit()),
                    key=lambda r: int(r[1:]), reverse=True)
    return f"{rounds[0]}_{name}" if rounds else f"r01_{name}"


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


def _cgroup_cpus():
    """CPUs this process's cgroup may use (cgroup v2 cpu.max quota / period), or None (no quota)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        return None


def _host_threads():
    """Threads for the CPU baseline: every CPU the box grants this process -- its cgroup CPU quota
    (on the GPU boxes cpu.max = 1600000 100000: 16 CPUs of the 256 the node shows, one GPU's share;
    OMP_NUM_THREADS is set to the same 16), else the CPUs in its affinity mask."""
    q = _cgroup_cpus()
    if q is not None:
        try:
            return min(q, len(os.sched_getaffinity(0)))
        except AttributeError:
            return q
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _oracle_loop(step_fn, B, seconds, desc, threads):
    """Full-batch oracle steps until ``seconds`` have passed (at least one; no warm-up step: a
    batch-64 step is seconds long, its first-call overheads are noise)."""
    n, t0 = 0, time.perf_counter()
    while True:
        step_fn()
        n += 1
        if time.perf_counter() - t0 > seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": round(B * n / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "host_cpus_visible": os.cpu_count(),
            "host_cpus_granted": _cgroup_cpus() or threads,
            "sample": f"{n} oracle train step(s) at B={B} ({desc}), torch CPU fp32, {threads} threads, {dt:.1f} s"}


def cpu_baseline(args, seconds):
    """Oracle (CPU restatement of the reference step) at the full batch: ResNet-101 encoder
    forward (train-mode BN) + the unhoisted 24-step decoder fwd/bwd + clamp + Adam."""
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import gen
    from oracle import decoder_ref as R
    from oracle.resnet_ref import build_resnet101, encoder_attention_forward
    threads = _host_threads()
    torch.set_num_threads(threads)
    B, L, V = args.batch, args.caption_len, args.vocab
    bert = args.config == "bert_attention"
    M = 768 if bert else 512
    net = build_resnet101(gen.resnet101_params(5)).train()
    p = {k: torch.from_numpy(v) for k, v in gen.decoder_params(5, 512, 512, M, V).items()}
    trainable = set(k for k in p if k != "embedding.weight")
    imgs = torch.from_numpy(gen.images(5, B, args.image_size, args.image_size))
    caps = torch.from_numpy(gen.captions(5, B, L, V))
    emb = None
    if bert:
        from capmi.data import SyntheticBertEmbedder
        emb = SyntheticBertEmbedder(V, 768)(caps)
    state = {}

    def one():
        nonlocal state
        with torch.no_grad():
            feats = encoder_attention_forward(net, imgs)
        out = R.train_step(p, trainable, feats, caps, [L] * B, state=state, embeddings=emb)
        p.update(out[5])
        state = out[6]

    return _oracle_loop(one, B, seconds, f"ResNet-101 fwd + unhoisted decoder fwd/bwd + clamp/Adam, L={L}, "
                                         f"V={V}, M={M}", threads)


def cpu_baseline_finetune(args, seconds):
    """Oracle fine-tune step (oracle/finetune_ref.py: ResNet-101 fwd+bwd of layer2-4, decoder
    fwd/bwd with fp64 GloVe-300 embedding, clamp + two Adams) at the full batch."""
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import gen
    from oracle.finetune_ref import finetune_train_step
    threads = _host_threads()
    torch.set_num_threads(threads)
    B, L, V = args.batch, args.caption_len, args.vocab
    rp = gen.resnet101_params(5)
    p = {k: torch.from_numpy(v) for k, v in gen.decoder_params(5, 512, 512, 300, V, emb_dtype=np.float64).items()}
    imgs = torch.from_numpy(gen.images(5, B, args.image_size, args.image_size))
    caps = torch.from_numpy(gen.captions(5, B, L, V))
    return _oracle_loop(lambda: finetune_train_step(rp, p, set(p), imgs, caps, [L] * B), B, seconds,
                        f"ResNet-101 fwd + layer2-4 bwd, unhoisted decoder fwd/bwd, fp64 GloVe-300 embedding, "
                        f"clamp/2x Adam, L={L}, V={V}", threads)


def run_baseline_cpu(args, ctx):
    """BASELINE config 1: the 'baseline' captioner (models/baseline.py: ResNet-101 + Linear encoder,
    nn.LSTM decoder) trained on the CPU at batch 4, as the reference's train loop does
    (models/baseline.py:114-264: CE ignore_index=PAD, backward, clamp, Adam); N > 1 ranks average
    the gradients over gloo. Returns (seconds for the timed steps, last loss)."""
    from capmi import dist as cdist
    from models.baseline import BaselineDecoder, BaselineDecoderParams
    from models.encoder import Encoder
    from train_utils import clip_gradient
    torch.set_num_threads(max(1, _host_threads() // ctx.world))
    torch.manual_seed(0)
    enc = Encoder(512).train()
    prm = BaselineDecoderParams()
    prm.vocab_size = args.vocab
    dec = BaselineDecoder(prm).train()
    dec.fine_tune_embeddings(False)  # --fine_tune_embedding default (train.py:41-42)
    cdist.broadcast_module(enc, ctx)
    cdist.broadcast_module(dec, ctx)
    params = [q for q in dec.parameters() if q.requires_grad]
    opt = torch.optim.Adam(params, lr=1e-4)
    crit = torch.nn.CrossEntropyLoss(ignore_index=0)
    from capmi.data import synthetic_batch
    imgs, caps, _ = synthetic_batch(args.batch, args.caption_len, args.vocab, "cpu", seed=1234 + ctx.rank,
                                    H=args.image_size, W=args.image_size)

    def one():
        with torch.no_grad():
            feats = enc(imgs)  # frozen ResNet (the reference's baseline trains only the decoder by default)
        scores = dec(feats, caps)
        loss = crit(scores.reshape(-1, scores.shape[2]), caps.reshape(-1))
        opt.zero_grad()
        loss.backward()
        if ctx.distributed:
            flat = torch.cat([q.grad.reshape(-1) for q in params])
            cdist.allreduce_mean_([flat], ctx)
            o = 0
            for q in params:
                q.grad.copy_(flat[o:o + q.numel()].view_as(q))
                o += q.numel()
        clip_gradient(opt, 5.0)
        opt.step()
        return loss

    for _ in range(args.warmup):
        one()
    cdist.barrier(ctx)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = one()
    cdist.barrier(ctx)
    return time.perf_counter() - t0, float(loss.detach())


def timing_pass(args, make_step, imgs, caps, lens, timer, encoder, pipeline):
    """Right after the timed region: --steps more calls of the step, launched eagerly so that every
    conv GEMM can take a pair of dispatch-timestamp events (ConvTimer). ``pipeline`` False: encoder and
    decoder on one stream, each kernel alone on the chip -- the condition a rocprofv3 kernel trace runs
    the bench in (its tracing serializes the two streams: 1.3 % of dispatches overlap in
    profiles/r03_bench_kernels.md), so these durations are the ones its summary reports. True: the timed
    region's pipelining (the previous batch's decoder beside the encoder), i.e. the durations the convs
    take inside the timed step, decoder interference included."""
    step2 = make_step(seed_off=99, graph=False, pipeline=pipeline)
    encoder._runner.conv_hook = timer
    step2(imgs, caps, lens)  # warm (pipelined: fills the pipeline with the first encoder pass), untimed
    if not pipeline:
        step2.flush()
    torch.cuda.synchronize()
    timer.enabled = True
    for _ in range(args.steps):
        step2(imgs, caps, lens)
    timer.enabled = False
    step2.flush()
    torch.cuda.synchronize()
    encoder._runner.conv_hook = None
    return (f"HIP events holding each conv GEMM dispatch's own start/end timestamps (hipExtLaunchKernel; what "
            f"rocprofv3 reports as its duration), {args.steps} eager calls of the step right after the timed region, "
            + ("pipelined as the timed region (the previous batch's decoder beside the encoder)" if pipeline else
               "encoder and decoder on one stream (each kernel alone on the chip, as under a rocprofv3 kernel trace)"))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    from capmi import dist as cdist
    cpu_cfg = args.config == "baseline_cpu"
    ctx = cdist.init_from_env("cpu" if cpu_cfg else "cuda", backend="gloo" if cpu_cfg else None)
    if ctx.world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started {ctx.world} rank(s)")
    if cpu_cfg:
        return main_baseline_cpu(args, ctx)
    if ctx.device.type != "cuda":
        raise SystemExit("bench: no HIP device (the GPU configs need an MI355X; --config baseline_cpu runs on CPU)")
    dev = ctx.device
    from capmi.data import synthetic_batch
    from capmi.optim import Adam
    from capmi.train_step import AttentionTrainStep
    from capmi import kernels as K
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
    if not encoder._runner.bf16 and args.conv == "x3":
        encoder.set_compute_precision("fp32-x3")
    dec_prec = args.dec if args.dec != "auto" else ("bf16" if encoder._runner.bf16 else "x3")
    decoder.set_compute_precision({"x3": "fp32-x3", "fp32": "fp32", "bf16": "bf16"}[dec_prec])
    if ft:
        # synthetic GloVe-300 table, fp64 like load_glove_vectors (embed.py:64-68, Q7)
        g = torch.Generator().manual_seed(300)
        decoder.load_pretrained_embeddins((torch.rand(args.vocab, 300, generator=g, dtype=torch.float64) - 0.5))
    decoder = decoder.to(dev).train()
    # glove_att: --fine_tune_embedding True (Makefile:13); bert: the table is unused; else Q8 default
    decoder.fine_tune_embeddings(ft)
    cdist.broadcast_module(encoder, ctx)
    cdist.broadcast_module(decoder, ctx)
    opt = Adam(filter(lambda q: q.requires_grad, decoder.parameters()), lr=1e-4)
    opt.set_clip(5.0)
    enc_opt = None
    if ft:
        encoder.fine_tune(True)
        enc_opt = Adam(filter(lambda q: q.requires_grad, encoder.parameters()), lr=1e-4)
        enc_opt.set_clip(5.0)
    pipe = not args.sequential and not ft

    def make_step(seed_off=0, graph=not args.eager, pipeline=pipe):
        return AttentionTrainStep(encoder, decoder, opt, ctx, alpha_c=1.0, graph=graph,
                                  seed=77 + seed_off + ctx.rank, pipeline=pipeline, encoder_optimizer=enc_opt)

    step = make_step()
    timer = ConvTimer()
    timer_pipe = None
    encoder._runner.conv_hook = None if args.no_roofline or not args.eager else timer
    B = args.batch
    imgs, caps, lens = synthetic_batch(B, args.caption_len, args.vocab, dev, seed=1234 + ctx.rank,
                                       H=args.image_size, W=args.image_size)

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
    dt_rank = time.perf_counter() - t0
    timer.enabled = False
    rank_dts = cdist.gather_floats(dt_rank, ctx)
    dt = max(rank_dts)
    if pipe:  # K encoder and K decoder passes were timed; drain the in-flight encoder pass
        step.flush()
        torch.cuda.synchronize()
    loss_v = float(loss.item())
    K.sk_check()  # stream-K hand-off invariant over the timed run (raises if a hand-off timed out)
    timing = None
    if not args.no_roofline:
        if args.eager:
            timing = ("HIP events holding each conv GEMM dispatch's own start/end timestamps (hipExtLaunchKernel), "
                      "inside the timed (eager) steps")
        else:
            timing = timing_pass(args, make_step, imgs, caps, lens, timer, encoder, pipeline=False)
            K.sk_check()
            if pipe:
                timer_pipe = ConvTimer()
                timing_pass(args, make_step, imgs, caps, lens, timer_pipe, encoder, pipeline=True)
                K.sk_check()

    N = ctx.world
    value = N * B * args.steps / dt
    roof = None
    per = timer.result() if not args.no_roofline else {}
    if per:
        # the dominant kernel: the conv GEMM instantiation with the most time
        key = max(per, key=lambda k: per[k][2])
        n, flops, ms = per[key]
        ach = flops / (ms * 1e-3) / 1e12
        fam_flops = sum(v[1] for v in per.values())
        fam_ms = sum(v[2] for v in per.values())
        per_img = sum(v[1] for v in per.values()) / args.steps / B
        peak = BF16_MFMA_PEAK_TF if encoder._runner.bf16 else FP32_MFMA_PEAK_TF
        if "x3" in key or (key.startswith("gemm_nts_kernel<") and key.split(",")[5].strip().startswith("3")):
            # the x3 kernels run six bf16 MFMAs per fp32 multiply-add: their matrix-core bound for
            # fp32 arithmetic is the dense bf16 peak / 6 (417 TF/s)
            peak = round(BF16_MFMA_PEAK_TF / 6, 1)
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
                "timing": timing,
                "kernel_names": {"launches_checked": timer.checked,
                                 "priced_vs_launched_mismatches": sorted(f"{a} != {b}" for a, b in timer.mismatch)},
                # which pass gives achieved / frac: the serialized one (encoder and decoder on one
                # stream, as the rocprofv3 kernel trace runs the bench) unless the steps themselves were eager;
                # in_pipeline below is the same kernel with the decoder stream beside it
                "frac_pass": "timed eager steps" if args.eager else "serialized timing pass (after the timed region)"}
        if timer_pipe is not None:
            pp = timer_pipe.result().get(key)
            if pp:
                # the same kernel's launches inside the pipelined step (decoder kernels sharing the CUs)
                roof["in_pipeline"] = {"pass": "pipelined timing pass (two streams, as the timed step)",
                                       "avg_launch_us": round(pp[2] * 1e3 / pp[0], 2),
                                       "achieved": round(pp[1] / (pp[2] * 1e-3) / 1e12, 3),
                                       "frac": round(pp[1] / (pp[2] * 1e-3) / 1e12 / peak, 4)}
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
            "conv_arithmetic": ("bf16 MFMA, fp32 accumulate" if encoder._runner.bf16 else
                                "fp32-accurate x3: each fp32 operand split exactly into three bf16 terms, the six cross "
                                "products above 2^-23|a||b| accumulated in fp32 on bf16 MFMA (error vs fp64 <= the "
                                "fp32-MFMA kernel's, tests/test_gpu_x3.py)" if encoder._runner.x3 else
                                "fp32 MFMA (v_mfma_f32_32x32x2_f32)"),
            "decoder_gemm_arithmetic": {"fp32-x3": "fp32-accurate x3 split (CAPMI_GEMM_SPLIT3, tests/test_gpu_split_gemm.py)",
                                        "bf16": "bf16 operands, fp32 accumulate (CAPMI_GEMM_BF16)",
                                        "fp32": "fp32 MFMA"}[decoder.compute_precision],
            "data": "synthetic (resident in HBM; random-init weights, torch.manual_seed(0))",
            "config": {"workload": ("'glove_att' decoder (GloVe-300 fp64 embedding, fine-tuned) + ResNet-101 "
                                    "encoder fine-tuned (layer2-4, BN train mode), one training step per batch")
                       if ft else ("'bert_attention' decoder (768-d synthetic BERT word features) + frozen "
                                   "ResNet-101 encoder (BN train mode), one training step per batch" +
                                   ("; encoder convs bf16 MFMA (fp32 accumulate), decoder GEMMs "
                                    f"{decoder.compute_precision} (attention / LSTM pointwise / softmax / loss fp32)"
                                    if encoder._runner.bf16 else "")) if bert else
                       ("'attention' decoder + frozen ResNet-101 encoder (BN train mode), "
                        "one training step per batch"),
                       "per_gpu_batch": B, "global_batch": B * N, "image_size": args.image_size,
                       "caption_len": args.caption_len, "decode_steps": args.caption_len - 1,
                       "vocab": args.vocab, "attention_dim": 512, "decoder_dim": 512, "embed_size": prm.embed_size,
                       "decoder_rows": ("49 distinct (AdaptiveAvgPool 7->14 replicate; exact, DESIGN.md 4.4)"
                                        if step._feat_layout(imgs)[1] > 1 else "196 pooled"),
                       "parallelism": f"dp{N}"},
            "dist": {"world_size": N, "backend": ctx.backend or "none",
                     "rank_ms_per_step": [round(x / args.steps * 1e3, 3) for x in rank_dts]},
            "loss_last_step": round(loss_v, 5),
            "launch": ("pipelined_2stream_eager" if args.eager else "pipelined_2stream_hip_graphs") if pipe
            else ("eager" if args.eager else "hip_graph"),
            # models.attention.train() builds the same step: pipelined (frozen encoder) or sequential (fine-tune),
            # replaying per-shape HIP graphs (CAPMI_TRAIN_GRAPH=0: eager)
            "launch_is_train_default": not args.eager and pipe == (not ft),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)


def main_baseline_cpu(args, ctx):
    dt_rank, loss_v = run_baseline_cpu(args, ctx)
    from capmi import dist as cdist
    rank_dts = cdist.gather_floats(dt_rank, ctx)
    dt = max(rank_dts)
    N = ctx.world
    if ctx.rank == 0:
        print(json.dumps({
            "metric": "training images/sec (whole node), 'baseline' decoder on CPU (BASELINE config 1)",
            "value": round(N * args.batch * args.steps / dt, 3), "unit": "images/s", "n_gpus": 0,
            "n_ranks": N, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32", "data": "synthetic (random-init weights, torch.manual_seed(0))",
            "config": {"workload": "'baseline' LSTM captioner (ResNet-101 + Linear encoder frozen, nn.LSTM "
                                   "decoder), CPU, one training step per batch",
                       "per_rank_batch": args.batch, "global_batch": args.batch * N, "image_size": args.image_size,
                       "caption_len": args.caption_len, "vocab": args.vocab, "parallelism": f"dp{N} (gloo, CPU)"},
            "dist": {"world_size": N, "backend": ctx.backend or "none",
                     "rank_ms_per_step": [round(x / args.steps * 1e3, 3) for x in rank_dts]},
            "loss_last_step": round(loss_v, 5), "roofline": None, "cpu_baseline": None}), flush=True)


if __name__ == "__main__":
    main()
