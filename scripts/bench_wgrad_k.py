import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dltb  # noqa
import torch, time
from dltb.utils.gemm_tuning import setup_tunableop
print(setup_tunableop("use"))
dev="cuda"; bf=torch.bfloat16; L=16
def tm(fn, it=10):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s=torch.cuda.Event(enable_timing=True); e=torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e)/it*1e3
tot={}
for name,(o,i) in {"qkv":(3072,1024),"out":(1024,1024),"fc1":(4096,1024),"fc2":(1024,4096)}.items():
    for K in (2048, 8192):
        dy=torch.randn(L,K,o,device=dev,dtype=bf); x=torch.randn(L,K,i,device=dev,dtype=bf)
        dw=torch.randn(L,o,i,device=dev,dtype=bf)
        t=tm(lambda: dw.baddbmm_(dy.transpose(1,2), x))
        fl=2*L*K*o*i
        print(f"{name} K={K}: {t:8.1f} us  {fl/t/1e6:7.1f} TF/s  per-2048-tokens {t*2048/K:7.1f} us", flush=True)
        tot[(name,K)]=t*2048/K
for K in (2048,8192):
    V=32000
    dl=torch.randn(K,V,device=dev,dtype=bf); h=torch.randn(K,1024,device=dev,dtype=bf); dw=torch.randn(V,1024,device=dev,dtype=bf)
    t=tm(lambda: dw.addmm_(dl.t(), h))
    print(f"head K={K}: {t:8.1f} us  {2*K*V*1024/t/1e6:7.1f} TF/s per-2048 {t*2048/K:7.1f}", flush=True)
    tot[("head",K)]=t*2048/K
for K in (2048,8192): print(K, sum(v for (n,k),v in tot.items() if k==K))
