"""Generate the golden parity fixtures from the REAL reference code.

TEST INFRASTRUCTURE -- run only in the survey/build container, where
/root/reference exists:

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

What it does: imports the reference's own modules (models/attention.py,
models/baseline.py, models/encoder.py, train_utils.py, vocabulary.py) with
``sys.modules`` stubs for the packages that are absent offline and that the
hot path never uses for arithmetic (torchvision.transforms, pytorch_pretrained_bert,
bcolz, nltk, pycocotools). ``torchvision.models.resnet101`` -- the one third-party
piece that IS arithmetic -- is stubbed with oracle/resnet_ref.py (torchvision is
not installed and nothing in the reference pins its version), so the encoder
fixtures pin the reference *wrapper* semantics, not torchvision's conv arithmetic.

Weights and inputs come from tests/golden/gen.py (seeded, version-stable), so
the fixtures hold seeds, dims and outputs only. No reference source or
bytecode is written into the repo (sys.dont_write_bytecode).
"""
import json
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
import gen  # noqa: E402
from oracle.resnet_ref import build_resnet101  # noqa: E402

_RESNET_SEED = [1234]


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def _install_stubs():
    tv = _stub("torchvision")
    tv.transforms = _stub("torchvision.transforms", Compose=lambda x: x, Resize=lambda *a, **k: None,
                          ToTensor=lambda *a, **k: None, Normalize=lambda *a, **k: None)

    def resnet101(pretrained=False):
        return build_resnet101(gen.resnet101_params(_RESNET_SEED[0]))

    tv.models = _stub("torchvision.models", resnet101=resnet101)
    _stub("pytorch_pretrained_bert", BertTokenizer=None, BertModel=None)
    _stub("bcolz")
    _stub("nltk")
    _stub("pycocotools")
    _stub("pycocotools.coco", COCO=None)
    sys.path.insert(0, REF)


def _vocab(V):
    from vocabulary import Vocabulary, PAD_TOKEN, START_TOKEN, END_TOKEN, UNK_TOKEN
    v = Vocabulary()
    v.add_word(PAD_TOKEN)
    for i in range(V - 4):
        v.add_word(f"w{i}")
    for w in (START_TOKEN, END_TOKEN, UNK_TOKEN):
        v.add_word(w)
    assert len(v) == V
    return v


def _t(x):
    return torch.from_numpy(np.ascontiguousarray(x))


def _load(module, params):
    sd = module.state_dict()
    for k, v in params.items():
        sd[k] = _t(v).clone()
    module.load_state_dict(sd)


def _params(A, D, M, V, emb=None):
    import models.attention as RA
    p = RA.AttentionDecoderParams()
    p.attention_dim, p.decoder_dim, p.embed_size, p.vocab = A, D, M, _vocab(V)
    p.dropout = 0.0
    return p


def _save(name, arrays, meta):
    arrays = dict(arrays)
    arrays["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
    print("wrote", name, sum(np.asarray(a).nbytes for a in arrays.values()), "bytes raw")


def _samples(prefix, x, k=256):
    x = np.asarray(x).ravel()
    idx = gen.probe_indices(x.size, k)
    return {prefix + "__idx": idx, prefix + "__val": x[idx], prefix + "__digest": gen.digest(x)}


# ---------------------------------------------------------------------------

def soft_attention_cases():
    import models.attention as RA
    for tag, (B, P, E, D, A, seed) in {
        "prod": (2, 196, 2048, 512, 512, 21),
        "small": (3, 10, 96, 40, 24, 22),
    }.items():
        m = RA.SoftAttention(E, D, A)
        sd = {"enc_att.weight": gen.uniform(seed, "ea.w", (A, E), -E ** -.5, E ** -.5),
              "enc_att.bias": gen.uniform(seed, "ea.b", (A,), -E ** -.5, E ** -.5),
              "dec_att.weight": gen.uniform(seed, "da.w", (A, D), -D ** -.5, D ** -.5),
              "dec_att.bias": gen.uniform(seed, "da.b", (A,), -D ** -.5, D ** -.5),
              "full_att.weight": gen.uniform(seed, "fa.w", (1, A), -A ** -.5, A ** -.5),
              "full_att.bias": gen.uniform(seed, "fa.b", (1,), -A ** -.5, A ** -.5)}
        _load(m, sd)
        enc = gen.uniform(seed, "enc", (B, P, E), 0, 1)
        h = gen.uniform(seed, "h", (B, D), -1, 1)
        with torch.no_grad():
            awe, alpha = m(_t(enc), _t(h))
        _save(f"soft_attention_{tag}", {"awe": awe.numpy(), "alpha": alpha.numpy()},
              {"B": B, "P": P, "E": E, "D": D, "A": A, "seed": seed,
               "ref": "models/attention.py:43-61"})


def decoder_forward_cases():
    import models.attention as RA
    cases = {
        # tag: (A, D, M, V, B, L, lengths, seed)
        "small_ragged": (32, 32, 16, 50, 3, 7, [7, 5, 4], 31),
        "small_full": (32, 32, 16, 50, 3, 7, None, 32),
        "prod": (512, 512, 512, 8100, 2, 25, None, 33),
    }
    for tag, (A, D, M, V, B, L, lengths, seed) in cases.items():
        dec = RA.AttentionDecoder(torch.device("cpu"), _params(A, D, M, V))
        prm = gen.decoder_params(seed, A, D, M, V)
        _load(dec, prm)
        dec.eval()
        enc = gen.encoder_features(seed, B)
        caps = gen.captions(seed, B, L, V, lengths)
        lens = list(lengths) if lengths else [L] * B
        with torch.no_grad():
            h0, c0 = dec.init_hidden_state(_t(enc).view(B, -1, 2048))
            preds, _, dl, alphas = dec(_t(enc), _t(caps), lens)
        out = {"captions": caps, "h0": h0.numpy(), "c0": c0.numpy(), "alphas": alphas.numpy()}
        if tag == "prod":
            out.update(_samples("predictions", preds.numpy(), 1024))
        else:
            out["predictions"] = preds.numpy()
        _save(f"decoder_forward_{tag}", out,
              {"A": A, "D": D, "M": M, "V": V, "B": B, "L": L, "lengths": lens,
               "decode_lengths": dl, "seed": seed, "ref": "models/attention.py:151-164,218-284"})


class _FakeCOCO(torch.utils.data.Dataset):
    """Stands in for dataset.COCODataset: seeded images + variable-length captions."""

    def __init__(self, vocab, n, lengths, seed, V):
        self.vocab = vocab
        self.n = n
        self.lengths = lengths
        self.seed = seed
        self.V = V
        self.requested = []

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        self.requested.append(int(i))
        img = gen.images(self.seed, 1, name=f"img{i}")[0]
        cap = gen.captions(self.seed + 1000 + i, 1, self.lengths[i], self.V)[0]
        return _t(img), _t(cap)


def train_step_cases():
    import models.attention as RA
    import models.encoder as RE
    cases = {
        # tag: A, D, M, V, B, lengths, glove(fp64 emb + fine-tune), seed
        "small": (32, 32, 16, 50, 3, [6, 4, 5], False, 41),
        "glove_small": (32, 32, 300, 50, 3, [6, 6, 3], True, 42),
        "prod": (512, 512, 512, 8100, 2, [25, 25], False, 43),
    }
    for tag, (A, D, M, V, B, lengths, glove, seed) in cases.items():
        _RESNET_SEED[0] = 1234 + seed
        vocab = _vocab(V)
        ds = _FakeCOCO(vocab, B, lengths, seed, V)
        prm = gen.decoder_params(seed, A, D, M, V, emb_dtype=np.float64 if glove else np.float32)
        cap = {}
        orig_init = RA.AttentionDecoder.__init__
        orig_fwd = RA.AttentionDecoder.forward
        orig_enc_fwd = RE.EncoderAttention.forward
        orig_clip = RA.clip_gradient

        def init(self, device, params, _o=orig_init):
            _o(self, device, params)
            _load(self, {k: v for k, v in prm.items() if k != "embedding.weight" or not glove})

        def fwd(self, enc, caps, lens, _o=orig_fwd):
            out = _o(self, enc, caps, lens)
            cap["dec_in"] = (enc.detach().numpy().copy(), caps.numpy().copy(), list(lens))
            cap["dec_out"] = (out[0].detach().numpy().copy(), out[3].detach().numpy().copy(), out[2])
            return out

        def enc_fwd(self, imgs, _o=orig_enc_fwd):
            cap["imgs_digest"] = gen.digest(imgs.numpy())
            return _o(self, imgs)

        def clip(opt, c, _o=orig_clip):
            if "grads_raw" not in cap:
                cap["grads_raw"] = {n: p.grad.detach().numpy().copy() for n, p in cap["named"]
                                    if p.grad is not None}
            _o(opt, c)

        def save_ckpt(args, epoch, encoder, decoder, eo, do, metrics):
            cap["post"] = {k: v.detach().numpy().copy() for k, v in decoder.state_dict().items()}
            cap["loss"] = metrics["epoch_losses"][-1][-1]
            cap["enc_post"] = {k: v.detach().numpy().copy() for k, v in encoder.state_dict().items()
                               if "running" in k or "num_batches" in k}

        RA.AttentionDecoder.__init__ = init
        RA.AttentionDecoder.forward = fwd
        RE.EncoderAttention.forward = enc_fwd
        RA.clip_gradient = clip
        RA.COCODataset = lambda mode, img_transform=None, caption_max_len=50: ds
        RA.save_checkpoint = save_ckpt
        RA.load_glove_vectors = lambda: _t(prm["embedding.weight"]).clone()
        orig_adam = torch.optim.Adam

        def adam(params, lr, _o=orig_adam):
            params = list(params)
            return _o(params, lr=lr)

        RA.torch.optim.Adam = adam

        args = types.SimpleNamespace(
            attention_dim=A, decoder_dim=D, embed_size=M, decoder_dropout=0.0, epochs=1,
            batch_size=B, workers=0, encoder_lr=1e-4, decoder_lr=1e-4, grad_clip=5.0, alpha_c=1.0,
            fine_tune_encoder=False, fine_tune_embedding=glove, checkpoint=None, print_freq=1,
            use_glove=glove, max_caption_length=-1, use_bert=False, model_name=f"golden_{tag}")

        # record the decoder's named parameters once it exists (for grad capture)
        def fwd2(self, enc, caps, lens, _f=fwd):
            cap["named"] = list(self.named_parameters())
            return _f(self, enc, caps, lens)
        RA.AttentionDecoder.forward = fwd2
        torch.manual_seed(seed)
        try:
            RA.train(torch.device("cpu"), args)
        finally:
            RA.AttentionDecoder.__init__ = orig_init
            RA.AttentionDecoder.forward = orig_fwd
            RE.EncoderAttention.forward = orig_enc_fwd
            RA.clip_gradient = orig_clip
            RA.torch.optim.Adam = orig_adam
        enc, caps, lens = cap["dec_in"]
        preds, alphas, dl = cap["dec_out"]
        full = tag != "prod"
        out = {"captions": caps, "order": np.array(ds.requested), "loss": np.array(cap["loss"]),
               "alphas": alphas, "imgs_digest": cap["imgs_digest"]}
        out.update(_samples("enc", enc, 2048))
        if full:
            out["predictions"] = preds
        else:
            out.update(_samples("predictions", preds, 2048))
        for k, g in cap["grads_raw"].items():
            if full:
                out["grad." + k] = g
            else:
                out.update(_samples("grad." + k, g, 512))
        for k, v in cap["post"].items():
            if full:
                out["post." + k] = v
            else:
                out.update(_samples("post." + k, v, 512))
        for k, v in cap["enc_post"].items():
            if v.size > 1:
                out.update(_samples("enc_post." + k, v, 128))
        _save(f"train_step_{tag}", out,
              {"A": A, "D": D, "M": M, "V": V, "B": B, "lengths": lengths, "glove": glove,
               "seed": seed, "resnet_seed": 1234 + seed, "caption_lengths_seen": lens,
               "decode_lengths": dl, "trainable": sorted(cap["grads_raw"].keys()),
               "emb_dtype": str(prm["embedding.weight"].dtype),
               "ref": "models/attention.py:287-452 (one batch), train_utils.py:2-12"})


def baseline_cases():
    import models.baseline as RB
    B, L, M, H, V, seed = 4, 9, 24, 32, 40, 51
    p = RB.BaselineDecoderParams()
    p.embed_size, p.hidden_size, p.vocab_size = M, H, V
    dec = RB.BaselineDecoder(p)
    sd = {}
    for k, v in dec.state_dict().items():
        sd[k] = gen.uniform(seed, k, tuple(v.shape), -0.2, 0.2)
    _load(dec, sd)
    feats = gen.uniform(seed, "feats", (B, M), -1, 1)
    caps = gen.captions(seed, B, L, V, [9, 7, 7, 4])
    with torch.no_grad():
        scores = dec(_t(feats), _t(caps))
        loss = torch.nn.CrossEntropyLoss(ignore_index=0)(scores.reshape(-1, V), _t(caps).reshape(-1))
    _save("baseline_forward", {"captions": caps, "scores": scores.numpy(), "loss": np.array(loss.item())},
          {"B": B, "L": L, "M": M, "H": H, "V": V, "seed": seed,
           "ref": "models/baseline.py:81-111,194-195,224-225"})


def encoder_wrapper_cases():
    """EncoderAttention around the restated resnet: pins children()[:-2] +
    adaptive pool (14,14) + permute, eval and train-mode BN (models/encoder.py:72-110)."""
    import models.encoder as RE
    seed = 61
    _RESNET_SEED[0] = 61
    enc = RE.EncoderAttention()
    for mode in ("eval", "train"):
        for (B, H) in ((2, 224), (1, 160)):
            getattr(enc, mode)()
            x = gen.images(seed, B, H, H, name=f"img_{mode}_{H}")
            with torch.no_grad():
                y = enc(_t(x))
            _save(f"encoder_{mode}_{B}x{H}", _samples("features", y.numpy(), 4096) |
                  {"shape": np.array(y.shape)},
                  {"B": B, "H": H, "mode": mode, "resnet_seed": seed,
                   "ref": "models/encoder.py:72-110 around oracle/resnet_ref.py (parity unpinned for conv arithmetic)"})


def decoder_denc_cases():
    """d(loss)/d(encoder_out) through the reference decoder's own autograd (what flows into the
    encoder when it is fine-tuned): AttentionDecoder.forward (models/attention.py:218-284) in
    train mode (dropout p = 0), the loss of :401-414 (pack_padded CE + alpha regulariser)."""
    import models.attention as RA
    from torch.nn.utils.rnn import pack_padded_sequence
    cases = {
        # tag: (A, D, M, V, B, L, lengths, seed)
        "small": (32, 32, 16, 50, 3, 7, [7, 5, 4], 35),
        "prod": (512, 512, 512, 8100, 2, 25, None, 36),
    }
    for tag, (A, D, M, V, B, L, lengths, seed) in cases.items():
        dec = RA.AttentionDecoder(torch.device("cpu"), _params(A, D, M, V))
        _load(dec, gen.decoder_params(seed, A, D, M, V))
        dec.train()
        enc = _t(gen.encoder_features(seed, B)).requires_grad_()
        caps = gen.captions(seed, B, L, V, lengths)
        lens = list(lengths) if lengths else [L] * B
        scores, caps_sorted, dl, alphas = dec(enc, _t(caps), lens)
        targets = caps_sorted[:, 1:]
        scores = pack_padded_sequence(scores, dl, batch_first=True).data
        targets = pack_padded_sequence(targets, dl, batch_first=True).data
        loss = torch.nn.CrossEntropyLoss()(scores, targets)
        loss = loss + ((1.0 - alphas.sum(dim=1)) ** 2).mean()
        loss.backward()
        g = enc.grad.numpy()
        out = {"captions": caps, "loss": np.array(loss.item())}
        out.update(_samples("denc", g, 8192))
        out["denc__absmax"] = np.array(np.abs(g).max())
        _save(f"decoder_denc_{tag}", out,
              {"A": A, "D": D, "M": M, "V": V, "B": B, "L": L, "lengths": lens, "seed": seed,
               "ref": "models/attention.py:43-61,151-164,218-284 (autograd to encoder_out), :401-414"})


def finetune_train_step_cases():
    """One batch of the reference train() (models/attention.py:287-452) with
    --fine_tune_encoder. Q9: the reference builds the encoder optimizer over
    filter(requires_grad, encoder.parameters()) while every parameter is frozen and
    fine_tune() is never called (ValueError: empty parameter list); the only patch here is
    EncoderAttention.__init__ calling fine_tune(True) (models/encoder.py:112-121), i.e. what
    BASELINE config 4 means. Everything else is the reference loop: encoder.train(),
    decoder, CE + alpha reg, backward, clip_gradient on both optimizers, both Adam steps."""
    import models.attention as RA
    import models.encoder as RE
    A, D, M, V, B, lengths, seed = 32, 32, 16, 50, 2, [6, 6], 45
    _RESNET_SEED[0] = 1234 + seed
    vocab = _vocab(V)
    ds = _FakeCOCO(vocab, B, lengths, seed, V)
    prm = gen.decoder_params(seed, A, D, M, V)
    cap = {"clip": []}
    orig = dict(init=RA.AttentionDecoder.__init__, fwd=RA.AttentionDecoder.forward,
                einit=RE.EncoderAttention.__init__, efwd=RE.EncoderAttention.forward, clip=RA.clip_gradient,
                adam=torch.optim.Adam)

    def init(self, device, params, _o=orig["init"]):
        _o(self, device, params)
        _load(self, prm)
        cap["decoder"] = self

    def einit(self, _o=orig["einit"]):
        _o(self)
        self.fine_tune(True)  # Q9
        cap["encoder"] = self

    def fwd(self, enc, caps, lens, _o=orig["fwd"]):
        cap["dec_in_enc"] = enc.detach().numpy().copy()
        return _o(self, enc, caps, lens)

    def clip(opt, c, _o=orig["clip"]):
        cap["clip"].append({id(p): p.grad.detach().numpy().copy() for grp in opt.param_groups
                            for p in grp["params"] if p.grad is not None})
        _o(opt, c)

    def save_ckpt(args, epoch, encoder, decoder, eo, do, metrics):
        cap["post_enc"] = {k: v.detach().numpy().copy() for k, v in encoder.state_dict().items()}
        cap["post_dec"] = {k: v.detach().numpy().copy() for k, v in decoder.state_dict().items()}
        cap["loss"] = metrics["epoch_losses"][-1][-1]

    def adam(params, lr, _o=orig["adam"]):
        return _o(list(params), lr=lr)

    RA.AttentionDecoder.__init__ = init
    RA.AttentionDecoder.forward = fwd
    RE.EncoderAttention.__init__ = einit
    RA.EncoderAttention = RE.EncoderAttention
    RA.clip_gradient = clip
    RA.COCODataset = lambda mode, img_transform=None, caption_max_len=50: ds
    RA.save_checkpoint = save_ckpt
    RA.torch.optim.Adam = adam
    args = types.SimpleNamespace(
        attention_dim=A, decoder_dim=D, embed_size=M, decoder_dropout=0.0, epochs=1, batch_size=B, workers=0,
        encoder_lr=1e-4, decoder_lr=1e-4, grad_clip=5.0, alpha_c=1.0, fine_tune_encoder=True,
        fine_tune_embedding=False, checkpoint=None, print_freq=1, use_glove=False, max_caption_length=-1,
        use_bert=False, model_name="golden_finetune")
    torch.manual_seed(seed)
    try:
        RA.train(torch.device("cpu"), args)
    finally:
        RA.AttentionDecoder.__init__ = orig["init"]
        RA.AttentionDecoder.forward = orig["fwd"]
        RE.EncoderAttention.__init__ = orig["einit"]
        RA.clip_gradient = orig["clip"]
        RA.torch.optim.Adam = orig["adam"]
    enc_named = dict(cap["encoder"].named_parameters())
    dec_named = dict(cap["decoder"].named_parameters())
    raw = {}
    for d in cap["clip"]:
        for nm, prm_ in list(enc_named.items()) + [("dec." + k, v) for k, v in dec_named.items()]:
            if id(prm_) in d:
                raw[nm] = d[id(prm_)]
    out = {"order": np.array(ds.requested), "loss": np.array(cap["loss"])}
    out.update(_samples("enc", cap["dec_in_enc"], 2048))
    enc_grads = sorted(k for k in raw if not k.startswith("dec."))
    for k in sorted(raw):
        out.update(_samples("grad." + k, raw[k], 64))
        out["gradnorm." + k] = np.array(np.linalg.norm(raw[k].astype(np.float64)))
    for k, v in cap["post_enc"].items():
        if v.size > 1 and (k in enc_named or "running" in k):
            out.update(_samples("post_enc." + k, v, 64))
    for k, v in cap["post_dec"].items():
        out.update(_samples("post_dec." + k, v, 64))
    _save("train_step_finetune", out,
          {"A": A, "D": D, "M": M, "V": V, "B": B, "lengths": lengths, "seed": seed, "resnet_seed": 1234 + seed,
           "enc_trainable": enc_grads, "n_enc_trainable": len(enc_grads),
           "dec_trainable": sorted(k[4:] for k in raw if k.startswith("dec.")),
           "ref": "models/attention.py:287-452 with --fine_tune_encoder (+ fine_tune(True), Q9), "
                  "models/encoder.py:72-121, train_utils.py:2-12"})


def beam_search_cases():
    """The reference's own beam search (gen_captions.py:16-131) on seeded weights. fc.weight is
    scaled (fc_scale) and fc.bias of <end> raised (end_bias) so that some beams finish early and
    others run to the 50-step cap, exercising the finished-beam bookkeeping over many steps;
    'noend' never finishes (the failure return)."""
    _stub("imageio")
    import gen_captions as RG
    import models.attention as RA
    for tag, (A, D, M, V, k, fc_scale, end_bias, seed) in {
        "small": (32, 32, 16, 50, 3, 10.0, 1.0, 61),
        "k5": (64, 48, 32, 120, 5, 10.0, 3.0, 62),
        "noend": (32, 32, 16, 50, 2, 1.0, -50.0, 63),
    }.items():
        vocab = _vocab(V)
        dec = RA.AttentionDecoder(torch.device("cpu"), _params(A, D, M, V))
        prm = gen.decoder_params(seed, A, D, M, V)
        prm["fc.weight"] = prm["fc.weight"] * np.float32(fc_scale)
        prm["fc.bias"] = prm["fc.bias"].copy()
        prm["fc.bias"][vocab("<end>")] += end_bias
        _load(dec, prm)
        dec.eval()
        feats = _t(gen.encoder_features(seed, 1)).view(1, 14, 14, 2048)
        args = types.SimpleNamespace(beam_size=k)
        seq, alphas, ok = RG.attention_caption_image_beam_search(torch.device("cpu"), args, None,
                                                                lambda img: feats, dec, vocab)
        _save(f"beam_search_{tag}", {"seq": np.array(seq), "alphas": np.array(alphas, dtype=np.float32),
                                     "ok": np.array(ok), "end_bias": np.array(end_bias),
                                     "fc_scale": np.array(fc_scale)},
              {"A": A, "D": D, "M": M, "V": V, "k": k, "seed": seed, "start": vocab("<start>"),
               "end": vocab("<end>"), "ref": "gen_captions.py:16-131"})


CASES = {"soft_attention": soft_attention_cases, "decoder_forward": decoder_forward_cases,
         "baseline": baseline_cases, "train_step": train_step_cases, "encoder_wrapper": encoder_wrapper_cases,
         "decoder_denc": decoder_denc_cases, "train_step_finetune": finetune_train_step_cases,
         "beam_search": beam_search_cases}


def main():
    """python make_golden.py [case ...]   (default: every case)"""
    _install_stubs()
    cwd = os.getcwd()
    todo = sys.argv[1:] or list(CASES)
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)
        try:
            torch.set_num_threads(8)
            for c in todo:
                CASES[c]()
        finally:
            os.chdir(cwd)


if __name__ == "__main__":
    main()
