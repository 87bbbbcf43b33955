"""Driver for PMC passes over the fused GEMM-loss prototype: MODE (env, default 7) launched 20
times on the Qwen3-30B-A3B w2 problem, plus 20 hipBLASLt mm of the same shape for comparison."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P, I64 = ctypes.c_void_p, ctypes.c_int64
lib = ctypes.CDLL(os.path.join(ROOT, "quantizers_amd/csrc/proto/libqz_proto.so"))
lib.qzp_gemm_sqerr.argtypes = [P, I64, I64, I64, I64, P, ctypes.c_int, P]
lib.qzp_gemm_sqerr_tiles.argtypes = [I64, I64]
lib.qzp_gemm_sqerr_tiles.restype = I64
dev = torch.device("cuda:0")
T, N, K = 32768, 2048, 768
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(T, K, device=dev, generator=g).to(torch.bfloat16)
w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
r = torch.nn.functional.linear(x, w)
nb = lib.qzp_gemm_sqerr_tiles(T, N)
part = torch.zeros(nb, dtype=torch.float64, device=dev)
tab = torch.tensor([[x.data_ptr(), w.data_ptr(), r.data_ptr(), part.data_ptr(), T]], dtype=torch.int64, device=dev)
c = torch.empty_like(r)
mode = int(os.environ.get("MODE", 7))
st = torch.cuda.current_stream()
for _ in range(20):
    assert lib.qzp_gemm_sqerr(P(tab.data_ptr()), 1, T, N, K, P(c.data_ptr()), mode, P(st.cuda_stream)) == 0
for _ in range(20):
    torch.mm(x, w.t(), out=c)
torch.cuda.synchronize()
print("done")
