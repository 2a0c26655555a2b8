"""GPU: the kernel names the bench prices are the instantiations the launcher runs.

bench.py attributes conv time to a kernel key (roofline.kernel, the PMC traffic lookup) that comes from the planner's
plan query (capmi_gemm_sk_plan; for the bf16 convs since ABI 25 the launcher's own bf16_io_plan). Here every conv
GEMM of the benchmarked configs at batch 64 -- config 2 (x3 forward), config 4 (x3 fine-tune forward and layer2-4
backward: dgrad / wgrad) and config 5 (bf16 forward) -- goes through the encoder's conv hook, and the key it is
priced under must equal the demangled instantiation the launch actually ran (capmi_last_launch_name: the kernel
pointer CAPMI_KLAUNCH recorded, named by the HIP runtime)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


class _Check:
    def __init__(self):
        self.n, self.bad, self.keys = 0, [], set()

    def __call__(self, tag, flops, launch, key):
        from capmi.kernels import last_launch_name
        launch()
        got = last_launch_name()
        self.n += 1
        self.keys.add(key)
        if got != key:
            self.bad.append((tag, key, got))


@pytest.mark.parametrize("config", ["attention", "glove_finetune", "bert_attention"])
def test_priced_kernel_names_equal_launched(config):
    from models.encoder import EncoderAttention
    from capmi.data import synthetic_batch
    torch.manual_seed(0)
    enc = EncoderAttention().to(DEV).train()
    enc.set_compute_precision("bf16" if config == "bert_attention" else "fp32-x3")
    imgs, _, _ = synthetic_batch(64, 25, 8100, DEV, seed=1234)
    chk = _Check()
    enc._runner.conv_hook = chk
    with torch.no_grad():
        if config == "glove_finetune":
            enc.fine_tune(True)
            feats = enc.ft_forward(imgs)
            grads = {id(q): torch.zeros_like(q) for q in enc.parameters() if q.requires_grad}
            enc.ft_backward(torch.rand_like(feats) - 0.5, grads)
        else:
            enc.forward_into(imgs, torch.empty(64, 14, 14, 2048, device=DEV))
    torch.cuda.synchronize()
    enc._runner.conv_hook = None
    want = {"attention": 104, "bert_attention": 104}.get(config)
    assert chk.n >= (want or 104), chk.n
    assert not chk.bad, chk.bad[:10]
