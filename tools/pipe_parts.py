"""Where the pipelined step's time goes: the bench's 'attention' step (pipelined HIP graphs, B = 64) timed whole,
then its encoder graph and its decoder graph (decoder step + clamp / Adam) each replayed alone on the chip.
python tools/pipe_parts.py [--steps 20] [--bert]  (--bert: config 5, bf16 encoder + 768-d synthetic word features)
The step is max(encoder, decoder) when the two streams share the chip perfectly; what it costs above that is
the interference of the decoder's kernels with the encoder's persistent grids."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-captioning-with-different-decoders_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--only", choices=["enc", "dec"], default=None,
                    help="after the warm-up, only replay that graph --steps times (a rocprofv3 trace of one part)")
    ap.add_argument("--bert", action="store_true", help="BASELINE config 5 (bench.py --config bert_attention)")
    a = ap.parse_args()
    from capmi.data import synthetic_batch
    from capmi.optim import Adam
    from capmi.train_step import AttentionTrainStep
    from models.attention import AttentionDecoder, AttentionDecoderParams
    from models.encoder import EncoderAttention
    from vocabulary import synthetic_vocab
    dev = torch.device("cuda")
    torch.manual_seed(0)
    enc = EncoderAttention().to(dev).train()
    enc.set_compute_precision("bf16" if a.bert else "fp32-x3")
    prm = AttentionDecoderParams()
    prm.vocab = synthetic_vocab(8100)
    prm.embed_size = 768 if a.bert else 512
    prm.use_bert = a.bert
    dec = AttentionDecoder(dev, prm)
    if a.bert:
        from capmi.data import SyntheticBertEmbedder
        dec.bert_embedder = SyntheticBertEmbedder(8100, 768, device=dev)
    dec.set_compute_precision("bf16" if a.bert else "fp32-x3")
    dec = dec.to(dev).train()
    dec.fine_tune_embeddings(False)
    opt = Adam(filter(lambda q: q.requires_grad, dec.parameters()), lr=1e-4)
    opt.set_clip(5.0)
    step = AttentionTrainStep(enc, dec, opt, alpha_c=1.0, graph=True, pipeline=True, seed=77)
    imgs, caps, lens = synthetic_batch(64, 25, 8100, dev, seed=1234, H=224, W=224)
    for _ in range(5):
        step(imgs, caps, lens)
    torch.cuda.synchronize()

    def clock(fn, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / n

    if a.only:
        step.flush()
        torch.cuda.synchronize()
        g = step._pg[0]["g_" + a.only]
        print(f"{a.only} graph alone {clock(g.replay, a.steps):.3f} ms")
        return
    t_step = clock(lambda: step(imgs, caps, lens), a.steps)
    step.flush()
    torch.cuda.synchronize()
    st = step._pg[0]
    t_enc = clock(st["g_enc"].replay, a.steps)
    t_dec = clock(st["g_dec"].replay, a.steps)
    t_seq = clock(lambda: (st["g_enc"].replay(), st["g_dec"].replay()), a.steps)
    print(f"pipelined step {t_step:.3f} ms | encoder graph alone {t_enc:.3f} | decoder graph alone {t_dec:.3f} | "
          f"both back to back {t_seq:.3f} | interference {t_step - max(t_enc, t_dec):.3f} ms")


if __name__ == "__main__":
    main()
