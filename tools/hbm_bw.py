import torch
dev='cuda:0'
def t(fn, it=20):
    for _ in range(3): fn()
    s,e=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize(); return s.elapsed_time(e)/it
n=204800*256
a=torch.empty(n,device=dev); b=torch.empty(n,device=dev)
ms=t(lambda: a.fill_(1.0)); print('fill 210MB: %.1f us %.2f TB/s'%(ms*1e3, n*4/ms/1e9))
ms=t(lambda: b.copy_(a)); print('copy 210MB: %.1f us %.2f TB/s (r+w)'%(ms*1e3, 2*n*4/ms/1e9))
x=torch.empty(204800*64,device=dev)
ms=t(lambda: torch.add(a.view(204800,256)[:, :64], 0, out=x.view(204800,64)) )
