"""One 'attention' training step on the MI355X (models/attention.py:386-430).

    feats = encoder(imgs)                        fused ResNet-101, BN in train mode
    loss, grads = decoder fwd + CE + alpha-reg + BPTT   (capmi.decoder_fn, grads in place)
    grads <- all-reduce mean over ranks          (DP only; RCCL)
    params <- clamp(+-grad_clip) + Adam          (one kernel)

Launch modes:
  * eager: every call launches the ~530 kernels of the step from Python;
  * pipelined (``pipeline=True``): call k runs the encoder of batch k on a high-priority stream
    while the decoder step of batch k-1 runs on a low-priority one (round 6; before, the other way round). The encoder is frozen and
    reads no decoder state, so the result is bit-identical to the sequential order; the
    decoder's latency-bound per-timestep kernels leave most CUs idle, which the encoder's
    GEMMs fill. Each call returns the loss of the previous batch (None on the first);
    ``flush()`` runs the last decoder step and returns its loss;
  * pipelined graphs (``pipeline=True, graph=True``): as pipelined, but each stream replays a
    captured graph (encoder forward per feature slot on the high-priority stream, decoder step +
    update per slot on the low-priority one), which removes the launch gaps of ~530 short kernels;
  * graph (``graph=True``): the step is captured once into a HIP graph (torch.cuda.CUDAGraph)
    and replayed; inputs are copied into static buffers first. Everything that changes from
    step to step lives on the device (Adam's step count, the dropout seed counter), so a
    replay is exactly an eager step. With DP the graph ends after the backward pass: the
    all-reduce and the update run eagerly after it (RCCL is not captured).

With more than one rank (eager mode) the all-reduce of step k is issued asynchronously and
its clamp+Adam update is applied at the start of step k+1's decoder, after step k+1's
encoder forward has been launched: the encoder does not read the decoder's weights, so the
collective overlaps the ResNet forward. ``flush()`` completes the last pending update.

Encoder fine-tune (config 4) with more than one rank, eager and graph alike: the decoder's
gradient bucket is all-reduced as soon as the decoder backward ends, beside the encoder
backward; the encoder's layer4, layer3 and layer2 buckets each as the backward leaves that
stage (FineTuneRunner.backward's ``on_layer``); clamp + Adam once all are in
(models/attention.py:417-430). In graph mode the step is captured as segments cut at exactly
those points and the collectives are issued between the segments' replays. ``schedule`` lists
what the last call issued, in order ("seg0", "ar:dec", "seg1", "ar:layer4", ...).
"""
import os

import torch

from . import decoder_fn as DF
from . import dist as cdist
from . import kernels as K
from .decoder_core import PNAMES
from .resnet import feature_hw, pool_dup


class AttentionTrainStep:
    def __init__(self, encoder, decoder, optimizer, ctx=None, alpha_c=1.0, overlap=True, graph=False,
                 seed=None, pipeline=False, encoder_optimizer=None):
        self.encoder, self.decoder, self.opt = encoder, decoder, optimizer
        # encoder fine-tune (config 4): the encoder's layer2-4 train with their own Adam
        # (models/attention.py:332-335,424-430); the decoder then also returns d(features)
        self.enc_opt = encoder_optimizer
        self.fine_tune = encoder_optimizer is not None
        if self.fine_tune:
            pipeline = False  # the encoder of batch k needs the update of batch k-1
            self._denc = None
            self.enc_params = [q for grp in encoder_optimizer.param_groups for q in grp["params"]]
            # per-stage gradient buckets of the encoder (contiguous spans of its flat buffer): layer4, layer3,
            # layer2 (children 7, 6, 5 of resnet, models/encoder.py:112-121), and whatever else is trainable
            self._enc_buckets = self._stage_buckets(encoder, encoder_optimizer)
        dev = next(decoder.parameters()).device
        self.ctx = ctx or cdist.DistCtx(device=dev)
        self.alpha_c = alpha_c
        # the decoder on the distinct rows of pixel-duplicated features (the 7x7 map the reference
        # pools to 14x14, DecoderCore.forward); CAPMI_ATT_DEDUP=0 decodes the pooled map (A/B)
        self.dedup = os.environ.get("CAPMI_ATT_DEDUP", "1") != "0"
        self.overlap = overlap and self.ctx.distributed and not graph
        self.graph_mode = graph
        self._pending = None
        named = dict(decoder.named_parameters())
        self.need = [n for n in PNAMES if named[n].requires_grad]
        self.params = named
        # data parallel: the fc gradients are final before the backward-through-time loop starts
        # (decoder_core.backward computes them first), so their bucket is all-reduced beside the
        # loop; the rest after it
        self._b_fc, self._b_rest = optimizer.grad_buckets({named["fc.weight"], named["fc.bias"]})
        s = int(torch.randint(0, 2 ** 62, (1,)).item()) if seed is None else int(seed)
        self.seed_dev = torch.full((1,), s, dtype=torch.int64, device=dev)
        self._graph = None
        self._static = None
        # per-shape graph cache: key (image shape, caption shape, lengths) -> captured graphs and the
        # workspaces they hold raw pointers into (pinned: the per-shape workspace caches keep only the
        # latest shape). Once CAPMI_GRAPH_CACHE keys are held, a new key runs eagerly (no eviction, so a
        # stream of one-off caption lengths cannot make every call a capture).
        self._gcache = {}
        self.graph_cache_size = int(os.environ.get("CAPMI_GRAPH_CACHE", "8"))
        self.counts = {"replay": 0, "eager": 0, "capture": 0}
        # optional callable(label) run before each graph capture (bench: graph-node timing), and
        # the labels of the graphs the last call replayed ("enc0"/"dec1"..., or "step")
        self.capture_hook = None
        self.replayed = []
        self.schedule = []  # graph segments replayed and collectives issued by the last call, in order
        self._segs = None  # data-parallel graph mode: (graphs, the bucket label ending each)
        self._capturing = False  # inside _capture (warm-ups and capture: no collectives, no update)
        # pipelined mode: the frozen encoder of batch k runs on its own stream while the decoder
        # step of batch k-1 runs (the encoder reads no decoder state); see _pipe_call
        self.pipeline = pipeline
        if pipeline:
            # pipeline + graph: each stream replays its own captured graph (per feature slot), so the
            # ~530 short kernels of a step leave no launch gaps (eager Python launches of the
            # latency-bound decoder kernels left the GPU idle ~10 % of the step)
            self.pipe_graph = graph
            self.graph_mode = False
            self._pg = None
            lo, hi = torch.cuda.Stream.priority_range()
            # encoder high / decoder low since round 6 (same box, three interleaved rounds: config 2 6300 -> 6321,
            # config 5 13137 -> 13254 img/s); CAPMI_PIPE_PRIO=dec: decoder high (the earlier default), equal: one level
            pe, pd = {"dec": (lo, hi), "equal": (lo, lo)}.get(os.environ.get("CAPMI_PIPE_PRIO", ""), (hi, lo))
            self.s_enc = torch.cuda.Stream(device=dev, priority=pe)
            self.s_dec = torch.cuda.Stream(device=dev, priority=pd)
            self._feats = [None, None]
            self._slot = 0
            self._pend = None
            self._ev_dec = None

    def _grads(self):
        return {n: self.params[n].grad for n in self.need}

    @staticmethod
    def _stage_buckets(encoder, opt):
        """{"layer4": views, "layer3": ..., "layer2": ..., "rest": ...} over the encoder optimizer's flat
        gradient buffer (Adam.grad_spans); stages with no trainable parameter map to []."""
        seq = getattr(encoder, "resnet", None)
        owned = {id(q) for grp in opt.param_groups for q in grp["params"]}
        groups, names = [], []
        if seq is not None and len(seq) >= 8:
            for li in (4, 3, 2):
                ps = [q for q in seq[li + 3].parameters() if id(q) in owned]
                if ps:
                    groups.append(set(ps))
                    names.append(f"layer{li}")
        spans = opt.grad_spans(groups)
        out = {f"layer{li}": [] for li in (2, 3, 4)}
        out.update(dict(zip(names, spans[:-1])))
        out["rest"] = spans[-1]
        return out

    def _bucket(self, label):
        if label == "dec":
            return self.opt.grad_buffers()
        if label == "fc":
            return self._b_fc
        if label == "dec_rest":
            return self._b_rest
        return self._enc_buckets[label]

    def _pins(self):
        """References to every per-shape workspace a capture's kernels address (encoder runner, fine-tune
        pools, decoder core and fused-loss buffers): held by the cache entry, so a later shape replacing
        them in those caches does not free memory a cached graph still replays into."""
        pins = [dict(DF.CORE._ws), dict(vars(DF._FS))]
        r = getattr(self.encoder, "_runner", None)
        if r is not None:
            pins.append(r._ws)
        ft = getattr(self.encoder, "_ft_runner", None)
        if ft is not None:
            pins += [dict(ft.saved.bufs), dict(ft.grad.bufs)]
        if getattr(self, "_denc", None) is not None:
            pins.append(self._denc)
        return pins

    def _cache_room(self, key):
        return key in self._gcache or len(self._gcache) < self.graph_cache_size

    def _issue(self, label, works):
        """All-reduce (mean, async) the bucket ``label`` on the collective stream, behind the work queued so far."""
        works.extend(cdist.allreduce_mean_(self._bucket(label), self.ctx, async_op=True))
        self.schedule.append(f"ar:{label}")

    def _feat_layout(self, imgs):
        """(feature buffer shape, dup) for a batch: the layer4 map when the encoder's pool only
        repeats its pixels (dup = 2 at 224x224: 7x7 -> 14x14), else the pooled map (dup = 1)."""
        N, _, H, W = imgs.shape
        enc = self.encoder
        out_hw = enc._out_hw() if hasattr(enc, "_out_hw") else (14, 14)
        d = 1
        if self.dedup and hasattr(enc, "_runner") and not (self.fine_tune and enc._runner.bf16):
            d = pool_dup(H, W, out_hw)
        if d > 1:
            fh, fw = feature_hw(H, W)
            return (N, fh, fw, 2048), d
        return (N, out_hw[0], out_hw[1], 2048), 1

    def _encode_into(self, imgs, out, dup):
        if dup > 1:
            self.encoder.forward_into(imgs, out, pooled=False)
        else:
            self.encoder.forward_into(imgs, out)

    def _snapshot(self):
        """Device state a capture warm-up must not change: the encoder's BatchNorm buffers
        (running mean/var, num_batches_tracked: train-mode forwards update them) and the dropout
        seed counter. Restored after the warm-ups, so a graph replay sequence equals the eager one."""
        return [(b, b.detach().clone()) for b in self.encoder.buffers()] + [(self.seed_dev, self.seed_dev.clone())]

    @staticmethod
    def _restore(snap):
        torch.cuda.synchronize()
        with torch.no_grad():
            for b, v in snap:
                b.copy_(v)
        torch.cuda.synchronize()

    def _grad_buffers(self):
        bufs = list(self.opt.grad_buffers())
        if self.fine_tune:
            bufs += list(self.enc_opt.grad_buffers())
        return bufs

    def _step_all(self):
        self.opt.step()
        if self.fine_tune:
            self.enc_opt.step()

    def _apply_pending(self):
        if self._pending is not None:
            for w in self._pending:
                w.wait()
            self._pending = None
            self._step_all()

    # ---------------------------------------------------------------- eager
    def _body_ft(self, imgs, captions, caption_lengths, with_update, cut=None):
        """Fine-tune step: encoder forward keeping layer2-4 activations, decoder fwd/bwd also
        producing d(features), encoder backward into the encoder optimizer's gradients.

        Data parallel: each bucket is handed over where its gradients become final -- the decoder's
        after the decoder backward (it overlaps the encoder backward), layer4 / layer3 / layer2 as
        the encoder backward leaves each stage (they overlap the lower stages' backward). Eager
        (``cut`` None): the all-reduces are issued right there and the update follows once all
        are in. Graph capture: ``cut(label)`` ends the segment being captured there; _replay
        issues the bucket's all-reduce between that segment's replay and the next one's."""
        K.counter_add(self.seed_dev, 1)
        self._apply_pending()
        _, dup = self._feat_layout(imgs)
        feats = self.encoder.ft_forward(imgs, pooled=dup == 1)
        if self._denc is None or self._denc.shape != feats.shape:
            self._denc = torch.empty_like(feats)
        loss, _, _ = DF.fused_loss_and_grads(self.decoder, feats, captions, caption_lengths,
                                             self.alpha_c, self._grads(), need=self.need,
                                             seed_dev=self.seed_dev, denc=self._denc, dup=dup)
        dp = self.ctx.distributed
        works = []
        hand = None
        if dp and cut is not None:
            # the lowest trainable stage finishes with the backward itself: its bucket is issued after the
            # last segment (a cut there would leave an empty graph)
            last = f"layer{self.encoder._ft().first}"

            def hand(label):
                if label != last:
                    cut(label)
        elif dp and not self._capturing:
            def hand(label):
                self._issue(label, works)
        if hand is not None:
            hand("dec")  # the decoder's gradients are final
        self.encoder.ft_backward(self._denc, {id(q): q.grad for q in self.enc_params},
                                 on_layer=None if hand is None else (lambda li: hand(f"layer{li}")))
        if dp and cut is None and not self._capturing:
            self._issue("rest", works)
            for w in works:
                w.wait()
            self._step_all()
            self.schedule.append("update")
        elif with_update:
            self._step_all()
        return loss

    def _body(self, imgs, captions, caption_lengths, with_update, cut=None):
        if self.fine_tune:
            return self._body_ft(imgs, captions, caption_lengths, with_update, cut=cut)
        K.counter_add(self.seed_dev, 1)
        shape, dup = self._feat_layout(imgs)
        if hasattr(self.encoder, "forward_into"):
            feats = torch.empty(shape, device=imgs.device, dtype=torch.float32)
            self._encode_into(imgs, feats, dup)
        else:
            feats, dup = self.encoder(imgs), 1
        self._apply_pending()
        loss, _, _ = DF.fused_loss_and_grads(self.decoder, feats, captions, caption_lengths,
                                             self.alpha_c, self._grads(), need=self.need,
                                             seed_dev=self.seed_dev, dup=dup,
                                             on_fc_grads=None if cut is None else (lambda: cut("fc")))
        if with_update:
            self.opt.step()
        return loss

    def _dec_body(self, feats, captions, caption_lengths, with_update, on_fc=None, dup=1):
        K.counter_add(self.seed_dev, 1)
        self._apply_pending()
        loss, _, _ = DF.fused_loss_and_grads(self.decoder, feats, captions, caption_lengths,
                                             self.alpha_c, self._grads(), need=self.need,
                                             seed_dev=self.seed_dev, on_fc_grads=on_fc, dup=dup)
        if with_update:
            self.opt.step()
        return loss

    def _pipe_call(self, imgs, captions, caption_lengths):
        """Call k: encoder(batch k) on s_enc, concurrently decoder step of batch k-1 on s_dec.
        Returns the loss of batch k-1 (None on the first call); flush() runs the last decoder.
        The returned loss lives on s_dec: synchronize before reading it."""
        cur = torch.cuda.current_stream()
        self.replayed = []
        slot = self._slot
        self._slot ^= 1
        shape, dup = self._feat_layout(imgs)
        if self._feats[slot] is None or tuple(self._feats[slot].shape) != shape:
            self._feats[slot] = torch.empty(shape, device=imgs.device, dtype=torch.float32)
        # the slot's previous reader is the decoder of call k-1
        self.s_enc.wait_stream(cur)
        if self._ev_dec is not None:
            self.s_enc.wait_event(self._ev_dec)
        with torch.cuda.stream(self.s_enc):
            self._encode_into(imgs, self._feats[slot], dup)
            ev_enc = torch.cuda.Event()
            ev_enc.record(self.s_enc)
        # the caller's tensors are read on the side streams: keep their blocks from being handed
        # to a later allocation on the caller's stream until those reads are done
        imgs.record_stream(self.s_enc)
        captions.record_stream(self.s_dec)
        loss = self._pipe_decoder()
        self._pend = ("eager", slot, captions, caption_lengths, ev_enc, dup)
        return loss

    # ------------------------------------------------------- pipelined graphs
    def _pg_capture(self, imgs, captions, caption_lengths, key, warmup=2):
        """Capture, per feature slot, the encoder forward (replayed on s_enc) and the decoder step
        with its update (replayed on s_dec). Warm-up runs on a side stream first, so every
        workspace is allocated outside the graphs' pools; each graph keeps its own pool (the two
        streams' graphs run concurrently)."""
        dev = imgs.device
        upd = not self.ctx.distributed
        snap = self._snapshot()
        shape, dup = self._feat_layout(imgs)
        feats = [torch.empty(shape, device=dev, dtype=torch.float32) for _ in range(2)]
        pg = []
        for slot in range(2):
            pg.append({"imgs": imgs.detach().clone(), "caps": captions.detach().clone(),
                       "lens": list(caption_lengths), "slot": slot})
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._encode_into(pg[0]["imgs"], feats[0], dup)
                self._dec_body(feats[0], pg[0]["caps"], pg[0]["lens"], with_update=False, dup=dup)
        torch.cuda.current_stream().wait_stream(s)
        self._restore(snap)
        for slot in range(2):
            st = pg[slot]
            g = torch.cuda.CUDAGraph()
            if self.capture_hook is not None:
                self.capture_hook(f"enc{slot}")
            with torch.cuda.graph(g):
                self._encode_into(st["imgs"], feats[slot], dup)
            st["g_enc"] = g
            st["feats"] = feats[slot]  # the graphs hold raw pointers: keep the buffer alive
            if self.capture_hook is not None:
                self.capture_hook(f"dec{slot}")
            if upd:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    st["loss"] = self._dec_body(feats[slot], st["caps"], st["lens"], with_update=True,
                                                dup=dup)
                st["g_dec"] = g
            else:
                # data parallel: two graphs cut where the fc gradients are final, so their all-reduce
                # is issued between the replays and runs beside the backward-through-time graph
                st["loss"], st["g_dec"], st["g_dec2"] = self._capture_split(
                    lambda cut: self._dec_body(feats[slot], st["caps"], st["lens"], with_update=False, on_fc=cut,
                                               dup=dup))
        torch.cuda.synchronize()
        pg[0]["pins"] = self._pins()
        self.counts["capture"] += 1
        return pg

    @staticmethod
    def _capture_segments(body):
        """Capture ``body(cut)`` into a chain of HIP graphs sharing one memory pool: every
        ``cut(label)`` ends the graph being captured and starts the next. Returns (body's result,
        [graphs], [the label of the cut that ended each graph; None for the last])."""
        graphs, labels = [torch.cuda.CUDAGraph()], []
        pool = torch.cuda.graph_pool_handle()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())

        def cut(label):
            graphs[-1].capture_end()
            labels.append(label)
            graphs.append(torch.cuda.CUDAGraph())
            graphs[-1].capture_begin(pool=pool)

        with torch.cuda.stream(cs):
            graphs[0].capture_begin(pool=pool)
            out = body(cut)
            graphs[-1].capture_end()
            labels.append(None)
        torch.cuda.current_stream().wait_stream(cs)
        return out, graphs, labels

    @staticmethod
    def _capture_split(body):
        """Capture ``body(cut)`` into two HIP graphs sharing one memory pool: the first ends where
        body calls ``cut()``. Returns (body's result, graph 1, graph 2)."""
        g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        pool = torch.cuda.graph_pool_handle()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        cut_done = []

        def cut():
            g1.capture_end()
            g2.capture_begin(pool=pool)
            cut_done.append(True)

        with torch.cuda.stream(cs):
            g1.capture_begin(pool=pool)
            out = body(cut)
            if not cut_done:  # body never cut: everything is in graph 1, graph 2 stays empty
                cut()
            g2.capture_end()
        torch.cuda.current_stream().wait_stream(cs)
        return out, g1, g2

    def _dp_update(self, fc_works):
        """All-reduce the remaining gradient bucket, wait for both (stream-level), clamp + Adam."""
        works = list(fc_works) + cdist.allreduce_mean_(self._b_rest, self.ctx, async_op=True)
        for w in works:
            w.wait()
        self.opt.step()

    def _pg_call(self, imgs, captions, caption_lengths):
        key = (tuple(imgs.shape), tuple(captions.shape), tuple(caption_lengths))
        pg = self._gcache.get(key)
        early = None
        if pg is None:
            if not self._cache_room(key):
                return self._pipe_call(imgs, captions, caption_lengths)  # cache full: this key runs eagerly
            if self._pend is not None:
                early = self.flush()  # the pending batch's loss: returned by this call, as the pipeline would
            pg = self._pg_capture(imgs, captions, caption_lengths, key)
            self._gcache[key] = pg
        self._pg = pg
        cur = torch.cuda.current_stream()
        slot = self._slot
        self._slot ^= 1
        st = pg[slot]
        # the slot's static inputs and features were last read by the decoder of the previous call
        self.s_enc.wait_stream(cur)
        if self._ev_dec is not None:
            self.s_enc.wait_event(self._ev_dec)
        with torch.cuda.stream(self.s_enc):
            if imgs.data_ptr() != st["imgs"].data_ptr():
                st["imgs"].copy_(imgs, non_blocking=True)
                imgs.record_stream(self.s_enc)  # read on s_enc: see _pipe_call
            if captions.data_ptr() != st["caps"].data_ptr():
                st["caps"].copy_(captions, non_blocking=True)
                captions.record_stream(self.s_enc)
            st["g_enc"].replay()
            ev_enc = torch.cuda.Event()
            ev_enc.record(self.s_enc)
        self.replayed = [f"enc{slot}"]
        self.counts["replay"] += 1
        loss = self._pipe_decoder()
        if early is not None:
            loss = early
        self._pend = ("graph", st, captions, caption_lengths, ev_enc, None)
        return loss

    def _pipe_decoder(self):
        if self._pend is None:
            return None
        # dispatch on how the pending batch's encoder was launched (a ragged batch runs eagerly
        # between graph-replayed ones)
        if self._pend[0] == "graph":
            _, st, _, _, ev, _ = self._pend
            self._pend = None
            self.s_dec.wait_event(ev)
            self.s_dec.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.s_dec):
                st["g_dec"].replay()
                self.replayed.append(f"dec{st['slot']}")
                if self.ctx.distributed:
                    fc_works = cdist.allreduce_mean_(self._b_fc, self.ctx, async_op=True)
                    st["g_dec2"].replay()
                    self._dp_update(fc_works)
                loss = st["loss"].detach().clone()
                self._ev_dec = torch.cuda.Event()
                self._ev_dec.record(self.s_dec)
            return loss
        _, pslot, caps, lens, ev, dup = self._pend
        self._pend = None
        self.counts["eager"] += 1
        self._feats[pslot].record_stream(self.s_dec)  # a later shape may replace the slot's buffer
        self.s_dec.wait_event(ev)
        self.s_dec.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.s_dec):
            if self.ctx.distributed:
                fc_works = []
                loss = self._dec_body(self._feats[pslot], caps, lens, with_update=False,
                                      on_fc=lambda: fc_works.extend(
                                          cdist.allreduce_mean_(self._b_fc, self.ctx, async_op=True)), dup=dup)
                self._dp_update(fc_works)
            else:
                loss = self._dec_body(self._feats[pslot], caps, lens, with_update=True, dup=dup)
            loss = loss.detach().clone()  # the loss buffer is reused by the next decoder step
            self._ev_dec = torch.cuda.Event()
            self._ev_dec.record(self.s_dec)
        return loss

    def __call__(self, imgs, captions, caption_lengths):
        self.schedule = []
        if self.pipeline:
            if self.pipe_graph and len(set(caption_lengths)) == 1:
                return self._pg_call(imgs, captions, caption_lengths)
            return self._pipe_call(imgs, captions, caption_lengths)
        if self.graph_mode:
            return self._replay(imgs, captions, caption_lengths)
        return self._eager(imgs, captions, caption_lengths)

    def _eager(self, imgs, captions, caption_lengths):
        self.counts["eager"] += 1
        if not self.ctx.distributed or self.fine_tune:  # fine-tune: DP exchange inside _body_ft
            return self._body(imgs, captions, caption_lengths, with_update=True)
        loss = self._body(imgs, captions, caption_lengths, with_update=False)
        works = cdist.allreduce_mean_(self._grad_buffers(), self.ctx, async_op=self.overlap)
        if self.overlap:
            self._pending = works
        else:
            self._step_all()
        return loss

    def flush(self):
        """Complete all outstanding work (pipelined decoder step, pending DP update) and make the
        current stream wait for it."""
        loss = None
        if self.pipeline:
            loss = self._pipe_decoder()
            torch.cuda.current_stream().wait_stream(self.s_dec)
            torch.cuda.current_stream().wait_stream(self.s_enc)
        self._apply_pending()
        return loss

    # ---------------------------------------------------------------- graph
    def _replay(self, imgs, captions, caption_lengths):
        if len(set(caption_lengths)) != 1:
            # ragged batches (never produced by the reference collate, Q1) need a host->device
            # copy of the per-step batch sizes: run them eagerly
            return self._eager(imgs, captions, caption_lengths)
        key = (tuple(imgs.shape), tuple(captions.shape), tuple(caption_lengths))
        ent = self._gcache.get(key)
        if ent is None:
            if not self._cache_room(key):
                return self._eager(imgs, captions, caption_lengths)  # cache full: this key runs eagerly
            self._capture(imgs, captions, caption_lengths, key)
            ent = self._gcache[key] = (self._graph, self._static, self._segs)
        self._graph, self._static, self._segs = ent
        self.counts["replay"] += 1
        st = self._static
        if imgs.data_ptr() != st["imgs"].data_ptr():
            st["imgs"].copy_(imgs, non_blocking=True)
        if captions.data_ptr() != st["caps"].data_ptr():
            st["caps"].copy_(captions, non_blocking=True)
        self.schedule = []
        if self._segs is None:
            self._graph.replay()
            self.replayed = ["step"]
            self.schedule.append("step")
            return st["loss"]
        # data parallel: the segments, each bucket's all-reduce issued as soon as the segment that
        # finalises it has been queued (it then runs beside the next segment's replay)
        graphs, labels = self._segs
        works = []
        self.replayed = []
        for i, (g, label) in enumerate(zip(graphs, labels)):
            g.replay()
            self.replayed.append(f"seg{i}")
            self.schedule.append(f"seg{i}")
            if label is not None:
                self._issue(label, works)
        tail = [f"layer{self.encoder._ft().first}", "rest"] if self.fine_tune else ["dec_rest"]
        for label in tail:
            self._issue(label, works)
        for w in works:
            w.wait()
        self._step_all()
        self.schedule.append("update")
        return st["loss"]

    def _capture(self, imgs, captions, caption_lengths, key, warmup=2):
        upd = not self.ctx.distributed
        st = {"key": key, "imgs": imgs.detach().clone(), "caps": captions.detach().clone(),
              "lens": list(caption_lengths)}
        # warm-up on a side stream: allocates every workspace outside the graph's pool. No
        # parameter update here (gradients are overwritten by the next step), so the first
        # call still applies exactly one update; the BN running statistics and the dropout seed
        # counter the warm-up forwards advance are restored afterwards (graph == eager).
        snap = self._snapshot()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        self._capturing = True
        try:
            with torch.cuda.stream(s):
                for _ in range(warmup):
                    self._body(st["imgs"], st["caps"], st["lens"], with_update=False)
            torch.cuda.current_stream().wait_stream(s)
            self._restore(snap)
            self._capture_graphs(st, upd)
        finally:
            self._capturing = False

    def _capture_graphs(self, st, upd):
        if self.capture_hook is not None:
            self.capture_hook("step")
        if upd:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                st["loss"] = self._body(st["imgs"], st["caps"], st["lens"], with_update=True)
            self._segs = None
        else:
            # data parallel: segments cut where buckets become final (fc / decoder, layer4, layer3, layer2)
            st["loss"], graphs, labels = self._capture_segments(
                lambda cut: self._body(st["imgs"], st["caps"], st["lens"], with_update=False, cut=cut))
            g = graphs[0]
            self._segs = (graphs, labels)
        st["pins"] = self._pins()
        self.counts["capture"] += 1
        self._graph, self._static = g, st
