"""CPU: libcapmi.so loads, exports every symbol include/capmi.h declares, the ctypes
struct mirrors the C struct, argument validation rejects bad calls without touching a
GPU, and the reference surface (classes, attributes, state-dict keys, CLI) is intact."""
import ctypes
import os
import re

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "capmi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?(?:\w+\s+)*\w+\*?\s+\*?(capmi_\w+)\s*\(", src, flags=re.M)))


def test_exports_match_header():
    import capmi
    declared = header_functions()
    assert len(declared) >= 25
    lib = ctypes.CDLL(capmi.LIB_PATH)
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in capmi.h but not exported"
    assert sorted(capmi.EXPORTS) == declared, "ctypes signature table out of sync with capmi.h"


def test_struct_layout():
    from capmi._lib import GemmProblem
    # 4 ints, 15 pointer/longlong, 2 floats + int, 10 ints -> layout checked via offsets of anchors
    assert GemmProblem.A.offset == 16
    assert GemmProblem.in_shift.offset + 8 == ctypes.sizeof(GemmProblem)
    assert GemmProblem.in_shift.offset == GemmProblem.in_scale.offset + 8


def test_abi_and_errors():
    import capmi
    from capmi._lib import lib
    assert lib.capmi_abi_version() == capmi.ABI_VERSION
    assert b"invalid" in lib.capmi_strerror(1001)
    # validation happens before any launch: null pointers are rejected without a GPU
    assert lib.capmi_bn_add_relu(None, None, None, None, None, None, None, 4, 3, None) == 1001
    assert lib.capmi_adam_clamp(None, None, None, None, 4, 1e-4, .9, .999, 1e-8, 1.0, 1.0, 5.0, None, None) == 1001
    assert lib.capmi_counter_add(None, 1, None) == 1001


def test_gemm_rejects_bad_shapes():
    from capmi._lib import GemmProblem, lib
    p = GemmProblem()
    p.M, p.N, p.K, p.ksplit = 4, 4, 4, 0  # ksplit 0 invalid
    arr = (GemmProblem * 1)(p)
    assert lib.capmi_gemm(arr, 1, 0, 0, 0, None) == 1001
    assert lib.capmi_gemm(arr, 0, 0, 0, 0, None) == 1001
    assert lib.capmi_gemm(arr, 1, 7, 0, 0, None) == 1001


def test_gemm_sk_plan_on_host():
    """The launch plan is host logic (no GPU work): the 512-thread form for a wide conv, the
    256-thread kernel for N = 64 or with the bf16-operand flag, unknown flags rejected."""
    from capmi._lib import GemmProblem, lib
    c_int = ctypes.c_int

    def plan(N, flags=0, M=12544, Cin=256):
        p = GemmProblem()
        p.M, p.N, p.K, p.ksplit = M, N, 9 * Cin, 1
        p.A = p.B = p.C = 256  # 16-B aligned stand-ins: the plan never dereferences them
        p.ldb = 9 * Cin
        p.cN, p.cH, p.cW, p.cCin, p.cKH, p.cKW = M // 196, 14, 14, Cin, 3, 3
        p.cStride, p.cPad, p.cHo, p.cWo = 1, 1, 14, 14
        v = [c_int(0) for _ in range(5)]
        rc = lib.capmi_gemm_sk_plan(ctypes.byref(p), 2, 0, 3, flags, *[ctypes.byref(x) for x in v])
        return rc, tuple(x.value for x in v)

    rc, (bm, bn, sk, generic, nt) = plan(256)
    assert rc == 0 and (bm, bn, generic, nt) == (128, 128, 0, 512)
    assert plan(64)[1][4] == 256
    assert plan(256, flags=1)[1][4] == 256
    assert plan(256, flags=128)[0] == 1001  # unknown flag
    assert plan(256, flags=1 | 16)[0] == 1001  # flags do not combine
    # CAPMI_GEMM_SPLIT3 (16) on a conv: the 256-thread split-staged kernel, two workgroups per CU
    # for 64x64 (stream-K sized for that)
    rc, (bm, bn, sk, generic, nt) = plan(256, flags=16)
    assert rc == 0 and nt == 256 and generic == 0
    # CAPMI_GEMM_X3 (4): 128x128 tiles, 512 threads; CAPMI_GEMM_X3P (8): 256x128
    rc, (bm, bn, sk, generic, nt) = plan(256, flags=4)
    assert rc == 0 and (bm, bn, generic, nt) == (128, 128, 0, 512)
    assert plan(64, flags=4)[1][1] == 64
    # gemm_x3 runs data-parallel by default (CAPMI_SK_FAMILY_OFF bit 1): 196 tiles -> no stream-K; a grid
    # under a quarter of the CUs (three images: 10 tiles of 72 k-steps) keeps it
    assert sk == 0
    rc, (bm, bn, sk, generic, nt) = plan(256, flags=4, M=588)
    assert rc == 0 and sk == 1
    # X3P reports its k-tile depth in `generic`: 32 + stream-K for 98 tiles (< 256 CUs), 16 (two
    # workgroups per CU, data-parallel) for 1568 tiles (0.77 of 4 rounds of 512 slots)
    rc, (bm, bn, sk, generic, nt) = plan(256, flags=8)
    assert rc == 0 and (bm, bn, generic, nt) == (256, 128, 32, 512) and sk == 1
    rc, (bm, bn, sk, generic, nt) = plan(256, flags=8, M=200704)
    assert rc == 0 and (bm, bn, generic, nt) == (256, 128, 16, 512) and sk == 0
    assert plan(256, flags=8, Cin=20)[0] == 1001  # Cin % 32 != 0
    assert plan(64, flags=8)[1][1] == 128  # N = 64: the 256 x 128 tile too (the 256 x 64 form was dropped, round 4)
    # CAPMI_GEMM_X3S (64, ABI 17): K = 64 only -- the 3x3 conv above is rejected; a 1x1 layer1 conv3 with
    # the BN prologue (M = 200704, N = 256) gets 64-row tiles, 256 threads, no stream-K, the persistent
    # grid (two workgroups per CU) in `generic`
    assert plan(256, flags=64)[0] == 1001

    def x3s_plan(N, M=200704, alpha=1.0, beta=0.0):
        p = GemmProblem()
        p.M, p.N, p.K, p.ksplit = M, N, 64, 1
        p.A = p.B = p.C = p.in_scale = p.in_shift = 256
        p.ldb, p.ldc, p.alpha, p.beta = 64, N, alpha, beta
        p.cN, p.cH, p.cW, p.cCin, p.cKH, p.cKW = M // 3136, 56, 56, 64, 1, 1
        p.cStride, p.cPad, p.cHo, p.cWo = 1, 0, 56, 56
        v = [c_int(0) for _ in range(5)]
        rc = lib.capmi_gemm_sk_plan(ctypes.byref(p), 2, 0, 3, 64, *[ctypes.byref(x) for x in v])
        return rc, tuple(x.value for x in v)

    rc, (bm, bn, sk, grid, nt) = x3s_plan(256)
    assert rc == 0 and (bm, bn, sk, nt) == (64, 256, 0, 256) and grid == 512  # 256 CUs with no GPU attached
    assert x3s_plan(64)[0] == 0 and x3s_plan(64)[1][1] == 64
    assert x3s_plan(512)[0] == 1001  # N outside {64, 128, 256}
    assert x3s_plan(256, beta=1.0)[0] == 1001  # not the store-only epilogue
    assert x3s_plan(256, M=3136)[1][3] == 49  # one image: grid = tiles when fewer than two per CU

    def wgrad_plan(Cout, Cin, k):
        # dW[Cout, (kh, kw, ci)] over k = 64*14*14 output pixels (A_MMAJOR x B_CONV_NHWC)
        p = GemmProblem()
        p.M, p.N, p.K, p.ksplit = Cout, k * k * Cin, 12544, 1
        p.A = p.B = p.C = 256
        p.lda, p.ldc = Cout, k * k * Cin
        p.cN, p.cH, p.cW, p.cCin, p.cKH, p.cKW = 64, 14, 14, Cin, k, k
        p.cStride, p.cPad, p.cHo, p.cWo = 1, k // 2, 14, 14
        v = [c_int(0) for _ in range(5)]
        rc = lib.capmi_gemm_sk_plan(ctypes.byref(p), 1, 2, 3, 0, *[ctypes.byref(x) for x in v])
        assert rc == 0
        return tuple(x.value for x in v)

    assert wgrad_plan(256, 256, 3)[:2] == (128, 128)  # wide 3x3 weight gradient
    assert wgrad_plan(1024, 256, 1)[:2] == (128, 64)  # 1x1 weight gradient

    def x3c_plan(n, h, w, Cin=64):
        # CAPMI_GEMM_X3C (256): layer1's direct 3x3; the padded band of a 256-pixel tile must fit its LDS
        p = GemmProblem()
        p.M, p.N, p.K, p.ksplit = n * h * w, 64, 9 * Cin, 1
        p.A = p.B = p.C = 256
        p.ldb, p.ldc, p.alpha = 9 * Cin, 64, 1.0
        p.cN, p.cH, p.cW, p.cCin, p.cKH, p.cKW = n, h, w, Cin, 3, 3
        p.cStride, p.cPad, p.cHo, p.cWo = 1, 1, h, w
        v = [c_int(0) for _ in range(5)]
        rc = lib.capmi_gemm_sk_plan(ctypes.byref(p), 2, 0, 3, 256, *[ctypes.byref(x) for x in v])
        return rc, tuple(x.value for x in v)

    rc, (bm, bn, sk, tiles, nt) = x3c_plan(50, 56, 56)
    assert rc == 0 and (bm, bn, sk, nt) == (256, 64, 0, 512) and tiles == 50 * 3136 // 256 + 1
    assert x3c_plan(5, 7, 7)[0] == 0 and x3c_plan(1, 64, 64)[0] == 0
    assert x3c_plan(2, 66, 66)[0] == 1001  # W > 64
    assert x3c_plan(64, 1, 32)[0] == 1001  # eight 1-row images per tile: 24 padded rows x 34 > 640 positions
    assert x3c_plan(4, 56, 56, Cin=48)[0] == 1001  # Cin % 32 != 0

    def bf16_plan(M, N, K, conv=None):
        # CAPMI_GEMM_BF16_IO (2, ABI 25): the launcher's own plan (gemm.hip bf16_io_plan)
        p = GemmProblem()
        p.M, p.N, p.K, p.ksplit = M, N, K, 1
        p.A = p.B = p.C = 256
        p.lda, p.ldb, p.ldc, p.alpha = K, K, N, 1.0
        amode = 0
        if conv is not None:
            n, h, cin, k, s = conv
            p.cN, p.cH, p.cW, p.cCin, p.cKH, p.cKW = n, h, h, cin, k, k
            p.cStride, p.cPad, p.cHo, p.cWo = s, k // 2, h // s, h // s
            amode = 2
        v = [c_int(0) for _ in range(5)]
        rc = lib.capmi_gemm_sk_plan(ctypes.byref(p), amode, 0, 3, 2, *[ctypes.byref(x) for x in v])
        return rc, tuple(x.value for x in v)

    # config 5 at batch 64: the K <= 256 1x1s (layer2's c3, layer1's c1, layer3's c3) take the one-stage 128x64
    # form; layer3's 3x3 (196 tiles of
    # 128x128: one round on 256 CUs) the four-deep DMA ring on 512 threads; layer2's 3x3 (392 tiles) the two-deep
    # ring; layer4's 3x3 (100 tiles: at most half of the CUs) 128x64 tiles (200), four deep on 256 threads
    rc, (bm, bn, sk, stages, nt) = bf16_plan(50176, 512, 128)
    assert rc == 0 and (bm, bn, sk, stages, nt) == (128, 64, 0, 1, 256)
    assert bf16_plan(200704, 64, 256)[1] == (128, 64, 0, 1, 256)
    assert bf16_plan(12544, 1024, 256)[1] == (128, 64, 0, 1, 256)
    assert bf16_plan(12544, 256, 1024)[1] == (128, 128, 0, 4, 512)
    assert bf16_plan(12544, 256, 2304, conv=(64, 14, 256, 3, 1))[1] == (128, 128, 0, 4, 512)
    assert bf16_plan(50176, 128, 1152, conv=(64, 28, 128, 3, 1))[1] == (128, 128, 0, 2, 512)
    assert bf16_plan(3136, 512, 4608, conv=(64, 7, 512, 3, 1))[1] == (128, 64, 0, 4, 256)
    assert bf16_plan(200704, 64, 576, conv=(64, 56, 64, 3, 1))[1] == (128, 64, 0, 2, 256)
    assert bf16_plan(3136, 512, 100)[0] == 1001  # K % 64 != 0


def test_device_tensors_required():
    from capmi import kernels as K
    x = torch.zeros(4, 4)
    with pytest.raises(ValueError):
        K.mean_rows(x, 1, 4, 4, x)


def test_reference_surface():
    from models.attention import AttentionDecoder, AttentionDecoderParams, SoftAttention
    from vocabulary import synthetic_vocab
    p = AttentionDecoderParams()
    p.attention_dim, p.decoder_dim, p.embed_size = 32, 32, 16
    p.vocab = synthetic_vocab(50)
    d = AttentionDecoder(torch.device("cpu"), p)
    keys = set(d.state_dict().keys())
    for k in ["attention.enc_att.weight", "attention.dec_att.bias", "attention.full_att.weight",
              "decode_step.weight_ih", "decode_step.bias_hh", "h_lin.weight", "c_lin.bias",
              "f_beta.weight", "fc.weight", "embedding.weight"]:
        assert k in keys
    for attr in ("embedding", "attention", "f_beta", "sigmoid", "decode_step", "fc", "init_hidden_state",
                 "device", "dropout", "load_pretrained_embeddins", "fine_tune_embeddings"):
        assert hasattr(d, attr)
    assert isinstance(d.attention, SoftAttention)
    assert float(d.fc.bias.abs().sum()) == 0.0  # reference :120
    assert d.embedding.weight.requires_grad  # fine-tuned by default at construction (:126)
    with pytest.raises(AssertionError):
        p2 = AttentionDecoderParams()
        AttentionDecoder(torch.device("cpu"), p2)  # vocab must be a Vocabulary (:84)
    with pytest.raises(RuntimeError):
        d(torch.zeros(2, 14, 14, 2048), torch.zeros(2, 5, dtype=torch.long), [5, 5])  # HIP only


def test_train_cli_quirks():
    from train import parse_args
    a = parse_args(["x", "--model", "attention", "--fine_tune_embedding", "False"])
    assert a.fine_tune_embedding is True  # argparse type=bool quirk kept (Q10)
    assert a.batch_size == 32 and a.grad_clip == 5.0 and a.print_freq == 1 and a.alpha_c == 1.0


def test_clip_gradient_torch_optimizer():
    from train_utils import clip_gradient
    w = torch.nn.Parameter(torch.zeros(5))
    w.grad = torch.tensor([-9.0, -5.0, 0.0, 4.0, 7.5])
    opt = torch.optim.Adam([w], lr=1e-4)
    clip_gradient(opt, 5.0)
    assert w.grad.tolist() == [-5.0, -5.0, 0.0, 4.0, 5.0]


def test_vocabulary_layout():
    from vocabulary import END_TOKEN, PAD_TOKEN, START_TOKEN, UNK_TOKEN, synthetic_vocab
    v = synthetic_vocab(8100)
    assert len(v) == 8100 and v(PAD_TOKEN) == 0 and v(START_TOKEN) == 8097 and v(END_TOKEN) == 8098
    assert v(UNK_TOKEN) == 8099 and v("never-seen") == 8099


def test_struct_layout_matches_c_compiler(tmp_path):
    """Every ctypes mirror (_lib.py) has the C compiler's size and field offsets for its struct in capmi.h
    (gcc on a probe that prints offsetof of each mirrored field; a field name missing in C fails the build)."""
    import shutil
    import subprocess
    from capmi._lib import DstepEpi, DstepSeg, GemmProblem, Wx3Job
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    mirrors = [(GemmProblem, "capmi_gemm_problem"), (Wx3Job, "capmi_wx3_job"), (DstepSeg, "capmi_dstep_seg"),
               (DstepEpi, "capmi_dstep_epi")]
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "capmi.h"', "int main(void) {"]
    want = []
    for cls, cname in mirrors:
        lines.append(f'  printf("%zu\\n", sizeof({cname}));')
        want.append(ctypes.sizeof(cls))
        for f in cls._fields_:
            lines.append(f'  printf("%zu\\n", offsetof({cname}, {f[0]}));')
            want.append(getattr(cls, f[0]).offset)
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert got == want


def test_grad_spans_cover_the_flat_buffer():
    """Adam.grad_spans (the DP buckets: fc beside the BPTT loop; an encoder's layer4 / layer3 / layer2 as its
    backward leaves each stage): one contiguous view per group, each holding exactly its parameters' slots and
    padding, the groups disjoint, and the groups plus the rest tiling the flat gradient buffer in order."""
    import torch
    from capmi.optim import Adam
    from capmi.train_step import AttentionTrainStep
    torch.manual_seed(0)
    seq = torch.nn.Sequential(*[torch.nn.Linear(3 + i, 5) for i in range(8)])
    for i in range(5):
        for q in seq[i].parameters():
            q.requires_grad = False
    opt = Adam([q for q in seq.parameters() if q.requires_grad], lr=1e-3)
    gf = opt.grad_buffers()[0]
    spans = opt.grad_spans([set(seq[7].parameters()), set(seq[5].parameters())])
    assert len(spans) == 3 and all(len(s) == 1 for s in spans[:2])
    for grp, (view,) in zip((seq[7], seq[5]), spans[:2]):
        for q in grp.parameters():
            assert q.grad.data_ptr() >= view.data_ptr()
            assert q.grad.data_ptr() + q.numel() * 4 <= view.data_ptr() + view.numel() * 4
    pieces = sorted([v for s in spans for v in s], key=lambda v: v.data_ptr())
    pos = gf.data_ptr()
    for v in pieces:
        assert v.data_ptr() == pos
        pos += v.numel() * 4
    assert pos == gf.data_ptr() + gf.numel() * 4
    head, rest = opt.grad_buckets(set(seq[6].parameters()))
    assert len(head) == 1 and len(rest) == 2
    # the train step's per-stage encoder buckets: children 5, 6, 7 = layer2, layer3, layer4
    enc = type("E", (), {"resnet": seq})()
    b = AttentionTrainStep._stage_buckets(enc, opt)
    assert [v.data_ptr() for v in b["layer4"]] == [spans[0][0].data_ptr()]
    assert [v.data_ptr() for v in b["layer2"]] == [spans[1][0].data_ptr()]
    assert b["rest"] == []
    with pytest.raises(ValueError):
        opt.grad_spans([set(seq[5].parameters()) | set(seq[7].parameters())])  # not contiguous
