import torch, time, json
dev='cuda'
res={}
for (M,N,K) in [(2150400,768,256),(2150400,256,256),(2150400,80,256),(1638400,256,128),(51200,1024,256),(51200,256,1024)]:
    A=torch.randn(M,K,device=dev).to(torch.bfloat16); W=torch.randn(K,N,device=dev).to(torch.bfloat16)
    for _ in range(3): C=A@W
    torch.cuda.synchronize(); e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): C=A@W
    e1.record(); torch.cuda.synchronize(); ms=e0.elapsed_time(e1)/10
    byt=(M*K+M*N+K*N)*2
    res[f"{M}x{N}x{K}"]={"ms":round(ms,4),"TBps":round(byt/ms/1e9,2),"TF":round(2*M*N*K/ms/1e9,1)}
    # copy bandwidth reference
print(json.dumps(res))
x=torch.empty(2150400*768, dtype=torch.bfloat16, device=dev); y=torch.empty_like(x)
for _ in range(3): y.copy_(x)
torch.cuda.synchronize(); e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True); e0.record()
for _ in range(10): y.copy_(x)
e1.record(); torch.cuda.synchronize(); ms=e0.elapsed_time(e1)/10
print("copy TB/s", round(2*x.numel()*2/ms/1e9,2))
