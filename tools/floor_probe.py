import torch, json
dev=torch.device('cuda:0')
res={}
for mb in (21, 26, 85, 512):
    n=mb*(1<<20)//8
    x=torch.randint(0,1<<40,(n,),dtype=torch.int64,device=dev)
    acc=torch.empty((),dtype=torch.int64,device=dev)
    y=torch.empty_like(x)
    for name,fn in (("sum",lambda: torch.sum(x,dim=0,out=acc)),("copy",lambda: y.copy_(x))):
        for _ in range(200): fn()
        torch.cuda.synchronize()
        a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(100): fn()
        b.record(); b.synchronize()
        res[f"{name}_{mb}MB_us"]=a.elapsed_time(b)/100*1000
print(json.dumps(res,indent=1))
