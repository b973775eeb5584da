import torch
for (M, N, K) in ((8192, 8192, 8192), (2048, 16384, 4096), (2048, 4096, 16384)):
    a = (torch.rand(M, K, device='cuda') * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device='cuda') * 2 - 1).to(torch.bfloat16)
    for _ in range(3):
        torch.matmul(a, b.t())
    torch.cuda.synchronize()
