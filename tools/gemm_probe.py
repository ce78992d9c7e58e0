import torch, time
dev = torch.device("cuda", 0)
for (M, N, K) in [(96000, 2048, 512), (96000, 1536, 512), (96000, 512, 2048), (96000, 512, 512)]:
    A = torch.randn(M, K, device=dev).half()
    W = torch.randn(N, K, device=dev).half()
    for _ in range(3):
        C = A @ W.T
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        C = A @ W.T
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"torch fp16 {M}x{N}x{K}: {ms*1000:.1f} us {2*M*N*K/ms/1e9:.0f} TF/s", flush=True)
