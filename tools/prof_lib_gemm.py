"""hipBLASLt's kernels (names encode the macro tile) on the step's forward shapes, for
rocprofv3 --kernel-trace: python tools/prof_lib_gemm.py"""
import torch
import torch.nn.functional as F
torch.backends.cuda.preferred_blas_library("hipblaslt")
dev, bf = "cuda", torch.bfloat16
for M in (50432, 27580, 22852):
    for K, N in ((768, 2304), (768, 768), (3072, 768), (768, 3072)):
        x = torch.randn(M, K, device=dev).to(bf)
        w = (torch.randn(N, K, device=dev) * 0.05).to(bf)
        b = torch.randn(N, device=dev).to(bf)
        dy = torch.randn(M, N, device=dev).to(bf)
        for _ in range(3):
            F.linear(x, w, b)
            torch.matmul(dy, w)
        torch.cuda.synchronize()
