"""Per-layer accuracy trace of the fine-tune forward/backward on the shallow (1,1,2,1) stack
(tests/test_gpu_finetune.py::test_encoder_finetune_backward_shallow_tight), fp32 MFMA vs x3.

For every trainable conv it prints
  prop  : relative L2 error of the saved raw conv output vs the fp64 CPU forward (propagated);
  local : the same conv recomputed in fp64 from the GPU's OWN input (its saved predecessor and
          BN scale/shift), i.e. the error this kernel alone adds;
  stats : the saved batch mean / var vs fp64 statistics of the GPU's own output.
Then the per-tensor gradient error table of both GPU precisions against fp64 autograd, next to
the CPU fp32 path's."""
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "image-captioning-with-different-decoders_amd"), REPO,
          os.path.join(REPO, "tests", "golden"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import gen  # noqa: E402
from helpers import ft_relu_masks, mask_flips, rel_err, t  # noqa: E402
from oracle.resnet_ref import build_resnet101, encoder_attention_forward  # noqa: E402
from oracle.finetune_ref import encoder_backward_masked, trainable_names  # noqa: E402

DEV = "cuda"
LAYERS = tuple(int(v) for v in os.environ.get("TRACE_LAYERS", "1,1,2,1").split(","))
SEED = int(os.environ.get("TRACE_SEED", "83"))
B = int(os.environ.get("TRACE_B", "2"))


def _rand(shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1


def cpu_run(params, imgs, dfeat, dtype):
    net = build_resnet101(params, LAYERS).to(dtype).train()
    names = trainable_names(net)
    for n, q in net.named_parameters():
        q.requires_grad_(n in names)
    acts = {}
    for name, m in net.named_modules():
        if isinstance(m, nn.Conv2d) and name.startswith(("layer2", "layer3", "layer4")):
            m.register_forward_hook(lambda mod, i, o, name=name: acts.__setitem__(name, o.detach().clone()))
    feats = encoder_attention_forward(net, imgs.to(dtype))
    feats.backward(dfeat.to(dtype))
    named = dict(net.named_parameters())
    return acts, {n: named[n].grad.detach().clone() for n in names}, feats.detach()


def gpu_run(params, imgs, dfeat, x3):
    from capmi.resnet import EncoderRunner, FineTuneRunner, ResNet101
    net = ResNet101(LAYERS)
    sd = net.state_dict()
    for k, v in params.items():
        sd[k] = t(v).clone()
    net.load_state_dict(sd)
    net = net.to(DEV).train()
    runner = EncoderRunner()
    runner.x3 = x3
    ft = FineTuneRunner(runner)
    feats = ft.forward(net, t(imgs, DEV))
    torch.cuda.synchronize()
    masks = ft_relu_masks(ft)
    saved = []
    for b in ft.state["blocks"]:
        N, H, W, H2, W2 = B, b["H"], b["W"], b["H2"], b["W2"]

        def nchw(x, h, w, c):
            return x[: N * h * w * c].view(N, h, w, c).permute(0, 3, 1, 2).double().cpu()
        ent = dict(tag=b["tag"], blk=b["blk"], stride=b["stride"],
                   x=nchw(b["x"], H, W, b["Cin"]), y1=nchw(b["y1"], H, W, b["wd"]),
                   y2=nchw(b["y2"], H2, W2, b["wd"]), y3=nchw(b["y3"], H2, W2, b["Cout"]),
                   yd=nchw(b["yd"], H2, W2, b["Cout"]) if b["yd"] is not None else None,
                   ss=[tuple(v.detach().double().cpu().clone() if v is not None else None for v in trip)
                       for trip in b["ss"]])
        saved.append(ent)
    named = {k: q for k, q in net.named_parameters() if k.startswith(("layer2", "layer3", "layer4"))}
    grads = {id(q): torch.zeros_like(q) for q in named.values()}
    ft.backward(dfeat.float().to(DEV), grads)
    torch.cuda.synchronize()
    return saved, {k: grads[id(q)].double().cpu() for k, q in named.items()}, feats.double().cpu(), masks


def local_refs(ent, params):
    """fp64 recomputation of each conv of the block from the GPU's own saved input."""
    tag, s = ent["tag"], ent["stride"]
    w = {k: torch.as_tensor(params[f"{tag}.{k}.weight"]).double() for k in ("conv1", "conv2", "conv3")}
    (s1, b1, _), (s2, b2, _), _, _ = ent["ss"]
    a1 = torch.relu(ent["y1"] * s1.view(1, -1, 1, 1) + b1.view(1, -1, 1, 1))
    a2 = torch.relu(ent["y2"] * s2.view(1, -1, 1, 1) + b2.view(1, -1, 1, 1))
    out = {"conv1": F.conv2d(ent["x"], w["conv1"]),
           "conv2": F.conv2d(a1, w["conv2"], stride=s, padding=1),
           "conv3": F.conv2d(a2, w["conv3"])}
    ins = {"conv1": ent["x"], "conv2": a1, "conv3": a2}
    if ent["yd"] is not None:
        wd = torch.as_tensor(params[f"{tag}.downsample.0.weight"]).double()
        out["downsample.0"] = F.conv2d(ent["x"], wd, stride=s)
        ins["downsample.0"] = ent["x"]
    return out, ins


def main():
    torch.set_num_threads(16)
    params = gen.resnet101_params(SEED, LAYERS)
    imgs = gen.images(SEED, B)
    dfeat = _rand((B, 14, 14, 2048), 18)
    a64, g64, f64 = cpu_run(params, t(imgs), dfeat, torch.float64)
    a32, g32, f32 = cpu_run(params, t(imgs), dfeat.float(), torch.float32)
    runs = {"fp32": gpu_run(params, imgs, dfeat, False), "x3": gpu_run(params, imgs, dfeat, True)}
    print(f"layers {LAYERS} seed {SEED} B {B}")
    print(f"feats: cpu32 {rel_err(f32, f64):.3g} " + " ".join(f"{k} {rel_err(v[2], f64):.3g}" for k, v in runs.items()))
    key = {"conv1": "y1", "conv2": "y2", "conv3": "y3", "downsample.0": "yd"}
    bnk = {"conv1": 0, "conv2": 1, "conv3": 2, "downsample.0": 3}
    print(f"{'conv':24s} {'prop cpu32':>10s} {'prop fp32':>10s} {'prop x3':>10s} | {'loc cpu32':>10s} "
          f"{'loc fp32':>10s} {'loc x3':>10s} | {'mean fp32':>9s} {'mean x3':>9s} {'var fp32':>9s} {'var x3':>9s}")
    for i in range(len(runs["fp32"][0])):  # noqa: C901
        tag = runs["fp32"][0][i]["tag"]
        loc = {}
        for rk, (saved, _, _, _) in runs.items():
            loc[rk] = local_refs(saved[i], params)
        for cv in ("conv1", "conv2", "conv3", "downsample.0"):
            name = f"{tag}.{cv}"
            if name not in a64:
                continue
            row = [rel_err(a32[name], a64[name])]
            row += [rel_err(runs[rk][0][i][key[cv]], a64[name]) for rk in runs]
            # CPU fp32 local error: the fp32 conv of the fp32-rounded GPU input
            ref, ins = loc["fp32"]
            wname = f"{tag}.{cv}.weight"
            w32 = torch.as_tensor(params[wname]).float()
            st = runs["fp32"][0][i]["stride"] if cv in ("conv2", "downsample.0") else 1
            cpu_loc = F.conv2d(ins[cv].float(), w32, stride=st, padding=1 if cv == "conv2" else 0)
            row.append(rel_err(cpu_loc, ref[cv]))
            row += [rel_err(runs[rk][0][i][key[cv]], loc[rk][0][cv]) for rk in runs]
            st_err = []
            for rk in runs:
                y = runs[rk][0][i][key[cv]]
                m64, v64 = y.mean(dim=(0, 2, 3)), y.var(dim=(0, 2, 3), unbiased=False)
                _, _, ms = runs[rk][0][i]["ss"][bnk[cv]]
                st_err.append((rel_err(ms[0], m64), rel_err(ms[1], v64)))
            print(f"{name:24s} " + " ".join(f"{v:10.3g}" for v in row[:4]) + " | " +
                  " ".join(f"{v:10.3g}" for v in row[4:]) + " | " +
                  f"{st_err[0][0]:9.3g} {st_err[1][0]:9.3g} {st_err[0][1]:9.3g} {st_err[1][1]:9.3g}")
    print("\ngradients: rel err vs fp64 (cpu32 / gpu fp32 / gpu x3)")
    cat = lambda d: torch.cat([d[k].double().reshape(-1) for k in g64])  # noqa: E731
    print(f"{'aggregate':32s} {rel_err(cat(g32), cat(g64)):10.3g} {rel_err(cat(runs['fp32'][1]), cat(g64)):10.3g} "
          f"{rel_err(cat(runs['x3'][1]), cat(g64)):10.3g}")
    for k in g64:
        print(f"{k:32s} {rel_err(g32[k], g64[k]):10.3g} {rel_err(runs['fp32'][1][k], g64[k]):10.3g} "
              f"{rel_err(runs['x3'][1][k], g64[k]):10.3g}")

    # ---- the same comparison on each run's own ReLU branch (oracle.encoder_backward_masked)
    rec64, pre64, rec32 = {}, {}, {}
    _, h64, _ = encoder_backward_masked(params, t(imgs), dfeat, torch.float64, LAYERS, record=rec64, pre=pre64)
    print(f"\nfp64 masked forward == plain fp64 autograd: {rel_err(cat(h64), cat(g64)):.3g}")
    _, c32, _ = encoder_backward_masked(params, t(imgs), dfeat.float(), torch.float32, LAYERS, record=rec32)
    _, c64, _ = encoder_backward_masked(params, t(imgs), dfeat, torch.float64, LAYERS, masks=rec32)
    aligned = {"cpu32": (c32, c64, rec32)}
    for rk, run in runs.items():
        _, r64, _ = encoder_backward_masked(params, t(imgs), dfeat, torch.float64, LAYERS, masks=run[3])
        aligned[rk] = (run[1], r64, run[3])
    print("ReLU flips vs fp64's own branch, and |pre-activation| / rms of the flipped elements:")
    for rk, (_, _, m) in aligned.items():
        rows = []
        for k in rec64:
            bad = m[k] != rec64[k]
            if bad.any():
                z = pre64[k]
                rows.append(f"{k}: {int(bad.sum())} ({float(z[bad].abs().max() / z.pow(2).mean().sqrt()):.2g})")
        print(f"  {rk:6s} {mask_flips(m, rec64)} flips  " + "; ".join(rows))
    print("gradients on each run's own branch: rel err vs fp64 on that branch")
    print(f"{'aggregate':32s} " + " ".join(f"{rel_err(cat(g), cat(r)):10.3g}" for g, r, _ in aligned.values()))
    for k in g64:
        print(f"{k:32s} " + " ".join(f"{rel_err(g[k], r[k]):10.3g}" for g, r, _ in aligned.values()))


if __name__ == "__main__":
    main()
