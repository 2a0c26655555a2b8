"""round 5, probe 17: config 5's bf16 GEMM (gemm_bf16_kernel) -- data-parallel vs persistent grid
(CAPMI_BF16_PERSIST, read per call), outputs compared bit for bit, on the l3c3 (dense K=256) and l3c2 (3x3) shapes."""
import os
import statistics as st
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402
from gemm_one import parser, setup  # noqa: E402

for shape, extra in [("l3c3", []), ("l3c2", []), ("l2c3", []), ("l4c3", []), ("l1c3", [])]:
    g = parser().parse_args(["--shape", shape, "--bf16io"] + extra)
    run, M, N, Kd = setup(g)
    outs, times = {}, {"0": [], "1": []}
    for arm in ("0", "1"):
        os.environ["CAPMI_BF16_PERSIST"] = arm
        run.out.zero_()
        run()
        torch.cuda.synchronize()
        outs[arm] = run.out.clone()
    for _ in range(7):
        for arm in ("0", "1"):
            os.environ["CAPMI_BF16_PERSIST"] = arm
            run()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                run()
            e.record()
            torch.cuda.synchronize()
            times[arm].append(s.elapsed_time(e) * 1e3 / 20)
    print(f"{shape}: M={M} N={N} K={Kd} dp {st.median(times['0']):.2f} us, persistent {st.median(times['1']):.2f} us, "
          f"equal={torch.equal(outs['0'], outs['1'])}", flush=True)
