import os, sys, torch
sys.path.insert(0, "/root/repo")
from quantizers_amd import ops
from quantizers_amd.quantization import QuantizationArgs
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
R, C = 11008, 4096
copies = [(torch.randn(R, C, device=dev, generator=g) * 0.02).to(torch.bfloat16) for _ in range(12)]
a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
outs = [ops.alloc_outputs((R, C), a, None, dev) for _ in range(4)]
prep = [ops.PreparedQuantize(copies[0], a, outs[j]) for j in range(4)]
gqs = [ops.GroupedQuantize([copies[i]], a, outs=[outs[i % 4]]) for i in range(12)]
def t(fn, n=60):
    for i in range(10): fn(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n): fn(i)
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n
for r in range(5):
    a1 = t(lambda i: prep[i % 4].run(copies[i % 12]))
    a2 = t(lambda i: gqs[i % 12].run())
    print(f"round {r}: per-weight LDS-DMA {a1:.2f} us   grouped n=1 (register loads) {a2:.2f} us", flush=True)
