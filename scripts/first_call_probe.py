import time, torch
dev = torch.device("cuda:0")
t = time.time(); torch.zeros(1, device=dev); torch.cuda.synchronize(); print(f"cuda init + first kernel {time.time()-t:.3f}s")
def tm(name, fn):
    for k in range(2):
        t = time.time(); fn(); torch.cuda.synchronize(); print(f"{name} call {k}: {time.time()-t:.4f}s")
w = torch.randn(151936, 2560, device=dev).to(torch.bfloat16)
ids = torch.randint(0, 151936, (1, 2048), device=dev)
tm("embedding", lambda: torch.embedding(w, ids))
a = torch.ones(1, 64, 1, device=dev); b = torch.arange(2048, device=dev, dtype=torch.float)[None, None, :]
tm("f32 bmm [1,64,1]x[1,1,2048]", lambda: a @ b)
e = torch.randn(1, 2048, 64, device=dev)
tm("cat+cos+sin", lambda: (torch.cat((e, e), -1).cos(), torch.cat((e, e), -1).sin()))
x = torch.randn(2048, 2560, device=dev).to(torch.bfloat16); W = torch.randn(4096, 2560, device=dev).to(torch.bfloat16)
tm("bf16 linear [2048,2560]x[4096,2560]", lambda: torch.nn.functional.linear(x, W))
xb = torch.randn(32768, 2560, device=dev).to(torch.bfloat16)
tm("bf16 linear [32768,2560]x[4096,2560]", lambda: torch.nn.functional.linear(xb, W))
q = torch.randn(1, 32, 2048, 128, device=dev).to(torch.bfloat16); k = torch.randn(1, 8, 2048, 128, device=dev).to(torch.bfloat16)
tm("sdpa", lambda: torch.nn.functional.scaled_dot_product_attention(q, k.repeat_interleave(4, 1), k.repeat_interleave(4, 1), is_causal=True))
