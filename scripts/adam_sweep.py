"""AdamW launch-shape sweep at GPT-2 345M size (355M elements): unroll x max blocks."""
import sys, torch, statistics
sys.path.insert(0, '/root/repo')
from mxtrain.ops import optim as O, _lib
n = 355_000_000 // 64 * 64
d='cuda'
m=torch.randn(n,device=d); a=torch.zeros(n,device=d); v=torch.zeros(n,device=d)
g=torch.randn(n,device=d,dtype=torch.bfloat16); p=torch.empty(n,device=d,dtype=torch.bfloat16)
h=torch.tensor([1e-4,0.9,0.999,1e-8,0.01,0.1,0.001,1.0,1.0],device=d)
ns=torch.ones(1,device=d)
cfg=_lib._fn("mx_adamw_config")
for u in (1,2):
    for b in (8192,16384,32768,65536,131072):
        cfg(u,b)
        ts=[]
        for it in range(12):
            s,e=torch.cuda.Event(True),torch.cuda.Event(True)
            s.record(); O.adamw_step(m,a,v,g,p,h,normsq=ns); e.record(); torch.cuda.synchronize()
            ts.append(s.elapsed_time(e)*1e3)
        print(u,b,round(statistics.median(ts[2:]),1), flush=True)
