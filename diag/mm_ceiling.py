# hipBLASLt (torch.matmul) fp16 GEMM throughput at the encoder's batched shapes: a ceiling reference only
import torch, time
torch.backends.cuda.matmul.allow_fp16_reduced_precision_reduction = False
M = 96000
for (N, K, name) in [(3840, 1280, "qkv"), (1280, 1280, "o"), (5120, 1280, "fc1"), (1280, 5120, "fc2")]:
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    w = torch.randn(N, K, device="cuda", dtype=torch.float16)
    for dt in (torch.float16, torch.bfloat16):
        aa, ww = a.to(dt), w.to(dt)
        for _ in range(3): c = aa @ ww.t()
        torch.cuda.synchronize()
        n = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n): c = aa @ ww.t()
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        print(f"{name} {dt} M={M} N={N} K={K}: {ms:.3f} ms  {2*M*N*K/ms/1e9:.1f} TF/s", flush=True)
