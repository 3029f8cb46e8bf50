import sys, time, json, torch, torch.nn.functional as F
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from systemml_amd.ops import kernels as K
dev = torch.device('cuda:0')
cases = [(64, 64, 56, 56, 64, 3, 1, 1), (64, 256, 14, 14, 256, 3, 1, 1), (128, 3, 224, 224, 64, 7, 2, 3), (64, 512, 7, 7, 512, 3, 1, 1), (256, 32, 12, 12, 64, 5, 1, 2)]
for dt in (torch.bfloat16, torch.float32):
  for (N, C, H, W, Fo, k, s, p) in cases:
    X = torch.randn(N, C*H*W, device=dev, dtype=dt); Wt = torch.randn(Fo, C*k*k, device=dev, dtype=dt)
    Ho = (H+2*p-k)//s+1; Wo=(W+2*p-k)//s+1
    G = torch.randn(N, Fo*Ho*Wo, device=dev, dtype=dt)
    flops = 2.0*N*Fo*Ho*Wo*C*k*k
    res = {"N":N,"C":C,"H":H,"F":Fo,"k":k,"s":s,"dtype":str(dt)}
    for name, fn in (("fwd", lambda: K.conv2d(0, X, Wt, None, N, C, H, W, Fo, k, k, s, s, p, p)),
                     ("bwd_data", lambda: K.conv2d(1, None, Wt, G, N, C, H, W, Fo, k, k, s, s, p, p)),
                     ("bwd_filter", lambda: K.conv2d(2, X, None, G, N, C, H, W, Fo, k, k, s, s, p, p)),
                     ("miopen_fwd", lambda: F.conv2d(X.view(N,C,H,W), Wt.view(Fo,C,k,k), stride=s, padding=p)),
                     ("miopen_bwd_data", lambda: torch.nn.grad.conv2d_input((N,C,H,W), Wt.view(Fo,C,k,k), G.view(N,Fo,Ho,Wo), stride=s, padding=p)),
                     ("miopen_bwd_filter", lambda: torch.nn.grad.conv2d_weight(X.view(N,C,H,W), (Fo,C,k,k), G.view(N,Fo,Ho,Wo), stride=s, padding=p))):
        fn(); torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5): fn()
        torch.cuda.synchronize()
        ms = (time.perf_counter()-t)/5*1e3
        res[name+"_ms"] = round(ms, 3); res[name+"_TF"] = round(flops/ms/1e9, 1)
    print(json.dumps(res), flush=True)
