"""Per-shape time of the plain 1x1 c1 convs (dense rows, no prologue) on gemm_x3 (128 x 128), x3d (256 x 128)
and the wide x3d (128 x 256, CAPMI_TILE_128x256), batch 64; checks the wide result against x3d's."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "image-captioning-with-different-decoders_amd"))
import torch  # noqa: E402

from capmi import kernels as K  # noqa: E402
from capmi._lib import CAPMI_A_KMAJOR as AK, CAPMI_TILE_128x256  # noqa: E402

dev = "cuda"


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
print("| conv | M | N | K | gemm_x3 us | x3d us | x3d wide us | wide vs x3d rel |")
for tag, (M, N, Kd) in {"l3c1": (12544, 256, 1024), "l2c1": (50176, 128, 512), "l4c1": (3136, 512, 2048),
                        "l3c1-pro": (12544, 256, 1024)}.items():
    x = torch.rand(M * Kd, device=dev) - 0.3
    w = (torch.rand(N, Kd, device=dev) - 0.5) * 0.05
    w3 = torch.empty(3 * N * Kd, device=dev, dtype=torch.bfloat16)
    K.split3_bf16(w.contiguous(), w3)
    stats = torch.zeros(2 * K.stat_tiles(M) * N, device=dev)
    outs = [torch.empty(M * N, device=dev) for _ in range(3)]
    pro = tag.endswith("pro")
    sc, sh = torch.rand(Kd, device=dev) + 0.5, torch.rand(Kd, device=dev) - 0.5
    kw = dict(in_scale=sc, in_shift=sh) if pro else {}
    p0 = K.problem(M, N, Kd, x, Kd, w3, Kd, outs[0], N, stats=stats)
    p1 = K.problem(M, N, Kd, x, Kd, w3, Kd, outs[1], N, stats=stats, **kw)
    p2 = K.problem(M, N, Kd, x, Kd, w3, Kd, outs[2], N, stats=stats, **kw)
    t0 = t_us(lambda: K.gemm_x3(p0, AK, ws)) if not pro else float("nan")
    t1 = t_us(lambda: K.gemm_x3d(p1, AK, ws))
    t2 = t_us(lambda: K.gemm_x3d(p2, AK, ws, tile=CAPMI_TILE_128x256))
    torch.cuda.synchronize()
    K.sk_check([ws])
    print(f"| {tag} | {M} | {N} | {Kd} | {t0:.1f} | {t1:.1f} | {t2:.1f} | {float((outs[1]-outs[2]).norm()/outs[1].norm()):.2g} |",
          flush=True)
