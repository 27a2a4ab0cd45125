import torch
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
for (N, K) in [(1536, 512), (512, 512), (2048, 512), (512, 2048)]:
    w = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(8192, K, device=dev, generator=g).to(torch.bfloat16)
    res = []
    for (m1, m2) in [(192, 384), (384, 768), (768, 1536), (1536, 3072), (4096, 8192)]:
        a = torch.nn.functional.linear(x[:m1], w)
        b = torch.nn.functional.linear(x[:m2], w)[:m1]
        res.append(f"{m1}/{m2}:{'eq' if torch.equal(a, b) else 'DIFF'}")
    print(N, K, " ".join(res))
