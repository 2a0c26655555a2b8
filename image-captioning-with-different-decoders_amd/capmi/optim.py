"""Adam with the reference's element-wise gradient clamp fused in (one kernel per dtype).

Drop-in for ``torch.optim.Adam(params, lr=...)`` as used at models/attention.py:352-355
(defaults: betas (0.9, 0.999), eps 1e-8, no weight decay) followed by
``clip_gradient(optimizer, grad_clip)`` (train_utils.py:2-12): ``clip_gradient``
records the bound, ``step()`` clamps and updates in one pass.

Parameters (and their ``.grad``) are re-homed into one flat buffer per dtype
(fp32, plus fp64 for a GloVe table, Q7), so the data-parallel all-reduce and the
update each touch one contiguous buffer. The modules keep their Parameters
(same objects, same names/shapes); only their storage moves.
"""
import math

import torch

from . import kernels as K


class Adam:
    fused_clamp = True

    def __init__(self, params, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0):
        if weight_decay:
            raise ValueError("capmi Adam: weight decay is not used by the reference")
        params = [p for p in params]
        if not params:
            raise ValueError("optimizer got an empty parameter list")  # same as torch (Q9)
        self.param_groups = [{"params": params, "lr": lr, "betas": betas, "eps": eps,
                              "weight_decay": 0, "amsgrad": False}]
        self.clip = math.inf
        # the step count lives on the device: step() is then replayable inside a HIP graph
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=params[0].device)
        self.flats = []  # (dtype, p_flat, g_flat, m, v, [(param, offset, numel)])
        for dt in sorted({p.dtype for p in params}, key=str):
            ps = [p for p in params if p.dtype == dt]
            # every tensor starts on a 256-byte boundary (the kernels' 16-B vector loads and
            # their coalescing need aligned operands); the gaps stay zero and are never read
            al = 256 // torch.empty(0, dtype=dt).element_size()
            offs, n = [], 0
            for p in ps:
                offs.append(n)
                n += (p.numel() + al - 1) // al * al
            dev = ps[0].device
            pf = torch.zeros(n, device=dev, dtype=dt)
            gf = torch.zeros(n, device=dev, dtype=dt)
            layout = []
            for p, off in zip(ps, offs):
                k = p.numel()
                pf[off:off + k].copy_(p.detach().reshape(-1))
                p.data = pf[off:off + k].view_as(p)
                p.grad = gf[off:off + k].view_as(p)
                layout.append((p, off, k))
            self.flats.append([dt, pf, gf, torch.zeros_like(pf), torch.zeros_like(pf), layout])

    # ------------------------------------------------------------------
    def set_clip(self, c):
        self.clip = float(c)

    def grad_buffers(self):
        return [f[2] for f in self.flats]

    def grad_spans(self, groups):
        """Split the flat gradient buffers into contiguous views, one list per group of ``groups``
        (sets of Parameter objects, each group's parameters adjacent in the layout; 256-B aligned
        slots, so a span also holds its parameters' zero padding), and a last list with the rest.
        Data-parallel steps all-reduce a group's span as soon as its gradients are final (the fc
        bucket beside the decoder's BPTT; layer4 / layer3 / layer2 of a fine-tuned encoder as its
        backward leaves each stage), the rest after the backward."""
        out = [[] for _ in range(len(groups) + 1)]
        for dt, pf, gf, m, v, layout in self.flats:
            cuts = []
            for gi, grp in enumerate(groups):
                ids = {id(q) for q in grp}
                idx = [i for i, (p, off, k) in enumerate(layout) if id(p) in ids]
                if not idx:
                    continue
                if idx != list(range(idx[0], idx[-1] + 1)):
                    raise ValueError(f"grad_spans: the parameters of group {gi} are not contiguous")
                lo = layout[idx[0]][1]
                hi = layout[idx[-1] + 1][1] if idx[-1] + 1 < len(layout) else gf.numel()
                cuts.append((lo, hi, gi))
            cuts.sort()
            pos = 0
            for lo, hi, gi in cuts:
                if lo < pos:
                    raise ValueError("grad_spans: groups overlap")
                if lo > pos:
                    out[-1].append(gf[pos:lo])
                out[gi].append(gf[lo:hi])
                pos = hi
            if pos < gf.numel():
                out[-1].append(gf[pos:])
        return out

    def grad_buckets(self, first):
        """(span of the parameters in ``first``, the rest): grad_spans with one group."""
        head, rest = self.grad_spans([first])
        return head, rest

    def zero_grad(self, set_to_none=False):
        for f in self.flats:
            f[2].zero_()
            for p, off, k in f[5]:
                p.grad = f[2][off:off + k].view_as(p)

    @property
    def step_count(self):
        return int(self.step_dev.item())

    @torch.no_grad()
    def step(self, closure=None):
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        clip = self.clip if math.isfinite(self.clip) else 3.0e38
        K.counter_add(self.step_dev, 1)
        for dt, pf, gf, m, v, _ in self.flats:
            K.adam_clamp(pf, gf, m, v, g["lr"], b1, b2, g["eps"], 0.0, 0.0, clip, step_dev=self.step_dev)

    # ---- torch.optim.Adam-compatible state dict --------------------------
    def state_dict(self):
        state = {}
        i = 0
        for dt, pf, gf, m, v, layout in self.flats:
            for p, off, k in layout:
                state[i] = {"step": torch.tensor(float(self.step_count)),
                            "exp_avg": m[off:off + k].view_as(p).clone(),
                            "exp_avg_sq": v[off:off + k].view_as(p).clone()}
                i += 1
        g = dict(self.param_groups[0])
        g["params"] = list(range(i))
        return {"state": state, "param_groups": [g]}

    def load_state_dict(self, sd):
        i = 0
        for dt, pf, gf, m, v, layout in self.flats:
            for p, off, k in layout:
                st = sd["state"].get(i)
                if st is not None:
                    m[off:off + k].copy_(st["exp_avg"].reshape(-1))
                    v[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                    self.step_dev.fill_(int(float(st["step"])))
                i += 1
        pg = sd["param_groups"][0]
        for key in ("lr", "betas", "eps"):
            if key in pg:
                self.param_groups[0][key] = pg[key]
