import torch
A = torch.randn(65536, 768, device="cuda").to(torch.bfloat16)
W = torch.randn(50432, 768, device="cuda").to(torch.bfloat16)
W2 = torch.randn(3072, 768, device="cuda").to(torch.bfloat16)
for _ in range(3):
    y = A @ W.t(); z = A @ W2.t()
torch.cuda.synchronize()
