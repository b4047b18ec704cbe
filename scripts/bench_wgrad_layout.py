import os, sys, torch
sys.path.insert(0, os.getcwd())
import dltb
from dltb.ops import functional as F_
from dltb.utils.gemm_tuning import setup_tunableop
print(setup_tunableop("use"))
def tm(fn, it=10):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s=torch.cuda.Event(enable_timing=True); e=torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e)/it*1e3
bf=torch.bfloat16
T=4096
for o,i in [(28672,4096),(4096,14336),(6144,4096),(4096,4096)]:
    dy=torch.randn(T,o,device="cuda",dtype=bf); x=torch.randn(T,i,device="cuda",dtype=bf)
    dw=torch.empty(o,i,device="cuda",dtype=bf)
    t_old=tm(lambda: torch.mm(dy.t(), x, out=dw))
    t_new=tm(lambda: F_.linear_wgrad(dy, x, dw, None, False))
    small = x if x.numel() <= dy.numel() else dy
    tt = torch.empty(small.shape[1], small.shape[0], device="cuda", dtype=bf)
    t_tr=tm(lambda: dltb.ops._ext.ext().transpose_into(small, tt))
    xt = torch.empty(i, T, device="cuda", dtype=bf); dyt=torch.empty(o,T,device="cuda",dtype=bf)
    t_mm_x=tm(lambda: torch.mm(dy.t(), xt.t(), out=dw))
    t_mm_dy=tm(lambda: torch.mm(dyt, x, out=dw))
    print(f"out {o} in {i}: old {t_old:.1f} us  new(linear_wgrad) {t_new:.1f}  transpose {t_tr:.1f}  mm(x^T copy) {t_mm_x:.1f}  mm(dy^T copy) {t_mm_dy:.1f}", flush=True)
print("--- breakdown (out 28672, in 4096)")
o, i = 28672, 4096
dy=torch.randn(T,o,device="cuda",dtype=bf); x=torch.randn(T,i,device="cuda",dtype=bf)
dw=torch.empty(o,i,device="cuda",dtype=bf)
a, b = F_.wgrad_operands(dy, x)
print("a", tuple(a.shape), a.stride(), "b", tuple(b.shape), b.stride())
print("mm(a,b) out=dw", tm(lambda: torch.mm(a, b, out=dw)))
print("wgrad_operands", tm(lambda: F_.wgrad_operands(dy, x)))
print("linear_wgrad", tm(lambda: F_.linear_wgrad(dy, x, dw, None, False)))
from dltb.ops import blaslt
print("blaslt enabled", blaslt.enabled(), "mm->", blaslt.mm(a, b, dw, False))
blaslt.disable()
print("linear_wgrad (table off)", tm(lambda: F_.linear_wgrad(dy, x, dw, None, False)))
