import torch, time
dev = torch.device("cuda:0")
for n in (10_000_000, 15_000_000):
    for bits in (26,):
        k = torch.randint(0, 1 << bits, (n,), dtype=torch.int32, device=dev)
        for _ in range(2):
            torch.cuda.synchronize(); t0 = time.perf_counter()
            s, i = torch.sort(k, stable=True)
            torch.cuda.synchronize(); t1 = time.perf_counter()
        print(n, bits, "torch.sort stable int32", round((t1 - t0) * 1e3, 3), "ms", flush=True)
        x = torch.rand(n, 3, device=dev)
        for _ in range(2):
            torch.cuda.synchronize(); t0 = time.perf_counter()
            y = x[i]
            torch.cuda.synchronize(); t1 = time.perf_counter()
        print(n, "gather xyz by perm", round((t1 - t0) * 1e3, 3), "ms", flush=True)
