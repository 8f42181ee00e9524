import torch, time
d = torch.device("cuda")
g = torch.Generator(device=d); g.manual_seed(0)
for n in (1_080_000, 8_400_000):
    for _ in range(2):
        torch.randperm(n, generator=g, device=d) % 60000
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        p = torch.randperm(n, generator=g, device=d) % 60000
    torch.cuda.synchronize()
    print(n, (time.perf_counter() - t) / 5 * 1e3, "ms")
