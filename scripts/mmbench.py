import torch, time
dev='cuda'
def bench(f, n=20):
    for _ in range(3): f()
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(n): f()
    torch.cuda.synchronize(); return (time.perf_counter()-t)/n
for (M,N,K) in [(1024,65536,256),(1024,65536,512),(1024,65536,768),(256,65536,1024),(256,65536,2048)]:
    a32=torch.randn(N,K,device=dev); w32=torch.randn(M,K,device=dev)
    a16=a32.half(); w16=w32.half()
    t32=bench(lambda: a32@w32.T)
    t16=bench(lambda: a16@w16.T)
    fl=2*M*N*K
    print(f"M={M} N={N} K={K}: fp32 {t32*1e6:.0f} us {fl/t32/1e12:.0f} TF/s | f16 {t16*1e6:.0f} us {fl/t16/1e12:.0f} TF/s")
