"""x3w debug / timing: CAPMI_GEMM_X3W on dense k rows (and conv shapes) repeated, reporting zero outputs and the
partial slabs' state; then per-shape time of x3w vs the split-staging nts weight gradient."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-captioning-with-different-decoders_amd"))
import torch  # noqa: E402

from capmi import kernels as K  # noqa: E402
from capmi._lib import CAPMI_A_MMAJOR, CAPMI_B_CONV_NHWC, CAPMI_B_KROWS, CAPMI_GEMM_SPLIT3  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
for (M, N, Kp) in [(256, 1024, 12544), (2048, 512, 3136), (128, 512, 3000), (256, 1024, 12544)]:
    for rep in range(3):
        a = torch.rand(Kp, M, device=dev) * 2 - 1
        b = torch.rand(Kp, N, device=dev) * 2 - 1
        ref = (a.double().t() @ b.double())
        c = torch.full((M, N), 7.0, device=dev)
        prob = K.problem(M, N, Kp, a, M, b, N, c, N)
        ws = K.gemm_workspace(dev)
        plan = K.gemm_sk_plan(prob, CAPMI_A_MMAJOR, bmode=CAPMI_B_KROWS, flags=128)
        K.gemm_x3w(prob, CAPMI_B_KROWS, ws)
        torch.cuda.synchronize()
        err = float((c.double() - ref).norm() / ref.norm())
        part = ws[int(K.lib.capmi_gemm_workspace_flag_bytes()) // 4:].view(torch.float32)
        S = plan[3]
        ldp = -(-N // 128) * 128
        slabs = part[: S * M * ldp].view(S, M, ldp)
        nz = [float(slabs[s].abs().sum()) for s in range(S)]
        print(f"M{M} N{N} K{Kp} rep{rep} plan{plan} err {err:.3g} c.abs.max {float(c.abs().max()):.3g} "
              f"zero slabs {sum(1 for v in nz if v == 0)}/{S}", flush=True)


def t_us(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


ws = K.gemm_workspace(dev)
print("| wgrad | M | N | K | x3w us | nts us | x3w TF/s |")
for tag, (Nb, H, Cin, Cout, k, s) in {"l3c2": (64, 14, 256, 256, 3, 1), "l3c3": (64, 14, 256, 1024, 1, 1),
                                       "l3c1": (64, 14, 1024, 256, 1, 1), "l2c2": (64, 28, 128, 128, 3, 1),
                                       "l4c2": (64, 7, 512, 512, 3, 1), "l3c2s2": (64, 28, 256, 256, 3, 2),
                                       "l3ds": (64, 28, 512, 1024, 1, 2)}.items():
    pad = k // 2
    Ho = (H + 2 * pad - k) // s + 1
    y = torch.rand(Nb * H * H * Cin, device=dev)
    dy = torch.rand(Nb * Ho * Ho * Cout, device=dev) - 0.5
    sc, sh = torch.rand(Cin, device=dev) + 0.5, torch.rand(Cin, device=dev) - 0.5
    out = torch.empty(Cout * k * k * Cin, device=dev)
    geo = dict(N=Nb, H=H, W=H, Cin=Cin, KH=k, KW=k, stride=s, pad=pad, Ho=Ho, Wo=Ho)
    prob = K.problem(Cout, k * k * Cin, Nb * Ho * Ho, dy, Cout, y, 0, out, k * k * Cin, conv=geo, in_scale=sc,
                     in_shift=sh)
    tx = t_us(lambda: K.gemm_x3w(prob, CAPMI_B_CONV_NHWC, ws))
    tn = t_us(lambda: K.gemm_sk(prob, CAPMI_A_MMAJOR, ws, K.TILE_AUTO, CAPMI_B_CONV_NHWC, flags=CAPMI_GEMM_SPLIT3))
    fl = 2.0 * Cout * k * k * Cin * Nb * Ho * Ho
    print(f"| {tag} | {Cout} | {k * k * Cin} | {Nb * Ho * Ho} | {tx:.1f} | {tn:.1f} | {fl / tx / 1e6:.1f} |", flush=True)
