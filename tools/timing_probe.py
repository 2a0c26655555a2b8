"""GPU probe: timing events as graph nodes around a captured kernel (capmi_timing_event_record)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "image-captioning-with-different-decoders_amd"))
import torch
from capmi import kernels as K
x = torch.zeros(1, dtype=torch.int64, device="cuda")
a = torch.randn(4096, 4096, device="cuda")
s0, s1 = K.TimingEvent(), K.TimingEvent()
g = torch.cuda.CUDAGraph()
st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(st):
    b = a @ a
torch.cuda.current_stream().wait_stream(st)
with torch.cuda.graph(g):
    s0.record()
    b = a @ a
    s1.record()
    K.counter_add(x, 1)
for i in range(3):
    g.replay()
    torch.cuda.synchronize()
    print("replay", i, "ms", s0.elapsed_ms(s1), "counter", int(x.item()))
