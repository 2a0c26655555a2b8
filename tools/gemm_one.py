"""Repeat one conv GEMM launch (for PMC / clock measurements of a single kernel).

python tools/gemm_one.py --shape l3c2 --reps 50 [--tile 3]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "image-captioning-with-different-decoders_amd"))
import torch  # noqa: E402

from capmi import kernels as K  # noqa: E402
from capmi._lib import CAPMI_A_CONV_NHWC, CAPMI_A_KMAJOR  # noqa: E402

SHAPES = {  # name: (Cin, H, W, Cout, k, prologue[, stride]) -- ResNet-101 encoder convs at 224x224
    "l3c2": (256, 14, 14, 256, 3, True), "l3c3": (256, 14, 14, 1024, 1, True),
    "l3c1": (1024, 14, 14, 256, 1, False), "l1c2": (64, 56, 56, 64, 3, True),
    "l1c3": (64, 56, 56, 256, 1, True), "l4c2": (512, 7, 7, 512, 3, True), "l2c2": (128, 28, 28, 128, 3, True),
    "l1c2s": (64, 56, 56, 64, 3, True),
    "l1c1": (256, 56, 56, 64, 1, False), "l2c1": (512, 28, 28, 128, 1, False), "l2c3": (128, 28, 28, 512, 1, True),
    "l4c1": (2048, 7, 7, 512, 1, False), "l4c3": (512, 7, 7, 2048, 1, True),
    "l2c2s": (128, 56, 56, 128, 3, True, 2), "l3c2s": (256, 28, 28, 256, 3, True, 2),
    "l4c2s": (512, 14, 14, 512, 3, True, 2), "ds1": (64, 56, 56, 256, 1, False, 1),
    "ds2": (256, 56, 56, 512, 1, False, 2), "ds3": (512, 28, 28, 1024, 1, False, 2),
    "ds4": (1024, 14, 14, 2048, 1, False, 2)}


def parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="l3c2")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--tile", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--bf16io", action="store_true", help="bf16 activations/weights/output (CAPMI_GEMM_BF16_IO)")
    ap.add_argument("--nopro", action="store_true", help="drop the BN-apply+ReLU prologue (1x1: dense A)")
    ap.add_argument("--x3", action="store_true", help="fp32-accurate three-term bf16 split GEMM (CAPMI_GEMM_X3)")
    ap.add_argument("--x3p", action="store_true", help="x3 with the A operand pre-split too (CAPMI_GEMM_X3P)")
    ap.add_argument("--x3d", action="store_true", help="x3 with the fp32 A split in-kernel, B by LDS-DMA (CAPMI_GEMM_X3D)")
    ap.add_argument("--x3s", action="store_true", help="short-k streaming x3 kernel (gemm_x3s.hip)")
    ap.add_argument("--x3c", action="store_true", help="the direct 3x3 conv (gemm_x3c.hip; N = 64, stride 1)")
    ap.add_argument("--x3w", action="store_true", help="the conv's WEIGHT gradient on gemm_x3w.hip (dW = dY^T im2col(X))")
    ap.add_argument("--dense", action="store_true",
                    help="x3d on a 1x1 / stride-1 conv as dense rows with the BN prologue per k = channel "
                         "(the bench's gemm_x3p_kernel<0, *, 32, true, true> form; default: conv mode)")
    return ap


def setup(a):
    """(run, M, N, K) of one conv GEMM launch as the options describe (tensors held by the closure)."""
    dev = "cuda"
    ci, H, W, co, k, pro, *st = SHAPES[a.shape]
    stride = st[0] if st else 1
    pro = pro and not a.nopro
    N = a.batch
    Ho, Wo = (H + 2 * (k // 2) - k) // stride + 1, (W + 2 * (k // 2) - k) // stride + 1
    M, Kd = N * Ho * Wo, ci * k * k
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(N, H, W, ci, device=dev, generator=g) - 0.5
    w = torch.rand(co, Kd, device=dev, generator=g) - 0.5
    y = torch.empty(M, co, device=dev)
    stats = torch.empty(K.stat_tiles(M, 1) * co * 2 + 64, device=dev)
    sc = torch.rand(ci, device=dev, generator=g) + 0.5
    sh = torch.rand(ci, device=dev, generator=g) - 0.5
    geo = dict(N=N, H=H, W=W, Cin=ci, KH=k, KW=k, stride=stride, pad=k // 2, Ho=Ho, Wo=Wo)
    if k == 1 and not pro and stride == 1:
        prob, mode = K.problem(M, co, Kd, x, ci, w, Kd, y, co, stats=stats), CAPMI_A_KMAJOR
    else:
        prob = K.problem(M, co, Kd, x, 0, w, Kd, y, co, conv=geo, stats=stats,
                         in_scale=sc if pro else None, in_shift=sh if pro else None)
        mode = CAPMI_A_CONV_NHWC
    ws = K.gemm_workspace(dev)
    if a.bf16io:
        xb, wb = x.to(torch.bfloat16), w.to(torch.bfloat16)
        yb = torch.empty(M, co, device=dev, dtype=torch.bfloat16)
        if k == 1 and stride == 1:
            prob, mode = K.problem_bf16(M, co, Kd, xb, ci, wb, Kd, yb, co, stats=stats), CAPMI_A_KMAJOR
        else:
            prob = K.problem_bf16(M, co, Kd, xb, 0, wb, Kd, yb, co, stats=stats, conv=geo)
            mode = CAPMI_A_CONV_NHWC
        run = lambda: K.gemm_bf16(prob, mode, ws, a.tile)  # noqa: E731
    elif a.x3p:
        w3 = torch.empty(3 * w.numel(), device=dev, dtype=torch.bfloat16)
        K.split3_bf16(K.conv_weight_order_x3p(w, k, k, ci).contiguous(), w3)
        xp = torch.empty(3 * x.numel(), device=dev, dtype=torch.bfloat16)
        K.bn_relu_split3(x, sc if pro else None, sh if pro else None, x.numel() // ci, ci, xp)
        if k == 1 and stride == 1:
            prob, mode = K.problem(M, co, Kd, xp, ci, w3, Kd, y, co, stats=stats), CAPMI_A_KMAJOR
        else:
            prob, mode = K.problem(M, co, Kd, xp, 0, w3, Kd, y, co, conv=geo, stats=stats), CAPMI_A_CONV_NHWC
        print("x3p kernel:", K.gemm_x3p_kernel_name(prob, mode))
        run = lambda: K.gemm_x3p(prob, mode, ws)  # noqa: E731
    elif a.x3d:
        w3 = torch.empty(3 * w.numel(), device=dev, dtype=torch.bfloat16)
        K.split3_bf16(K.conv_weight_order_x3p(w, k, k, ci).contiguous(), w3)
        if a.dense and k == 1 and stride == 1:  # dense rows, the prologue per k = channel (EncoderRunner's 1x1 form)
            prob, mode = K.problem(M, co, Kd, x, ci, w3, Kd, y, co, stats=stats, in_scale=sc if pro else None,
                                   in_shift=sh if pro else None), CAPMI_A_KMAJOR
        prob.B = w3.data_ptr()
        print("x3d kernel:", K.gemm_x3d_kernel_name(prob, mode))
        run = lambda: K.gemm_x3d(prob, mode, ws)  # noqa: E731
    elif a.x3s:
        w3 = torch.empty(3 * w.numel(), device=dev, dtype=torch.bfloat16)
        K.split3_bf16(w, w3)
        prob.B = w3.data_ptr()
        print("x3s kernel:", K.gemm_x3s_kernel_name(prob, mode))
        run = lambda: K.gemm_x3s(prob, mode)  # noqa: E731
    elif a.x3c:
        w3 = torch.empty(3 * w.numel(), device=dev, dtype=torch.bfloat16)
        K.split3_bf16(K.conv_weight_order_x3p(w, k, k, ci).contiguous(), w3)
        prob.B = w3.data_ptr()
        print("x3c kernel:", K.gemm_x3c_kernel_name(prob))
        run = lambda: K.gemm_x3c(prob)  # noqa: E731
    elif a.x3w:  # dW[co][k*k*ci] = sum over output pixels of dY[p][co] x im2col(relu(bn(x)))[p][n]
        from capmi._lib import CAPMI_B_CONV_NHWC, CAPMI_B_KROWS
        dy = torch.rand(M, co, device=dev, generator=g) - 0.5
        dw = torch.empty(co, Kd, device=dev)
        bmode = CAPMI_B_KROWS if (k == 1 and stride == 1 and not pro) else CAPMI_B_CONV_NHWC
        if bmode == CAPMI_B_KROWS:
            prob = K.problem(co, Kd, M, dy, co, x, ci, dw, Kd)
        else:
            prob = K.problem(co, Kd, M, dy, co, x, 0, dw, Kd, conv=geo, in_scale=sc if pro else None,
                             in_shift=sh if pro else None)
        print("x3w kernel:", K.gemm_x3w_kernel_name(prob, bmode))
        run = lambda: K.gemm_x3w(prob, bmode, ws)  # noqa: E731
    elif a.x3:
        w3 = torch.empty(3 * w.numel(), device=dev, dtype=torch.bfloat16)
        K.split3_bf16(w, w3)
        prob.B = w3.data_ptr()
        print("x3 kernel:", K.gemm_x3_kernel_name(prob, mode, a.tile))
        run = lambda: K.gemm_x3(prob, mode, ws, a.tile)  # noqa: E731
    else:
        print("plan (bm, bn, stream_k, generic, threads):", K.gemm_sk_plan(prob, mode, a.tile, bf16=a.bf16, threads=True))
        run = lambda: K.gemm_sk(prob, mode, ws, a.tile, bf16=a.bf16)  # noqa: E731
    keep = (x, w, y, stats, sc, sh, prob, ws, locals().get("w3"), locals().get("xp"), locals().get("dy"),
            locals().get("dw"), locals().get("xb"), locals().get("wb"), locals().get("yb"))
    f = lambda: (run(), keep)[0]  # noqa: E731
    f.out = locals()["dw"] if a.x3w else locals()["yb"] if a.bf16io else y  # what the launch writes (ab_inproc compares builds on it)
    return f, M, co, Kd


def main():
    a = parser().parse_args()
    run, M, co, Kd = setup(a)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    run()
    torch.cuda.synchronize()
    s.record()
    for _ in range(a.reps):
        run()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / a.reps
    print(f"{a.shape}: M={M} N={co} K={Kd}: {us:.1f} us/launch, {2.0 * M * co * Kd / us / 1e6:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
