"""oracle/ -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's hot path (the 'attention' training step of
SarahAlkhateeb/Image-Captioning-with-Different-Decoders), used as the parity
checker. Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import anything from here, and only as the checker
or the timed CPU baseline -- never as part of the shipped product path.

Pinning (see DESIGN.md "Oracle"):
  * decoder side (``decoder_ref``): pinned against golden vectors produced by
    the real reference code (``tests/golden/make_golden.py`` imports
    /root/reference with module stubs in the survey container);
  * encoder side (``resnet_ref``): the ResNet-101 arithmetic lives in
    torchvision, absent here and unpinned by any reference test, so the
    conv/BN arithmetic is *parity unpinned* beyond torch-CPU F.conv2d /
    F.batch_norm; the reference wrapper semantics (children()[:-2],
    AdaptiveAvgPool2d(14,14), permute, BN in train mode) are pinned by the
    train-step golden, which ran the reference's EncoderAttention around this
    restatement.
"""
