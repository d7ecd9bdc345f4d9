"""The vendor GEMM (hipBLASLt through torch.nn.functional.linear) at the c5 and fp16-inference FC shapes,
a few launches each, for `rocprofv3 --kernel-trace --stats`: the kernel names it picks (Tensile names
encode the macro tile, MFMA shape, prefetch depths, stream-K) are what our fc_bf16_p is compared with."""
import torch

DEV = "cuda:0"
SHAPES = [(torch.bfloat16, 100_000, 2048, 2048), (torch.bfloat16, 100_000, 2048, 4096),
          (torch.float16, 100_000, 1024, 1024), (torch.float16, 100_000, 1024, 2048)]
for dt, M, N, K in SHAPES:
    A = torch.randn(M, K, device=DEV).to(dt)
    W = (torch.randn(N, K, device=DEV) * 0.03).to(dt)
    b = torch.randn(N, device=DEV).to(dt)
    for _ in range(5):
        y = torch.nn.functional.linear(A, W, b)
    torch.cuda.synchronize()
    print(dt, M, N, K, float(y[0, 0]), flush=True)
