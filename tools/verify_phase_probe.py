import sys, os
sys.path.insert(0, "tools"); sys.path.insert(0, ".")
import torch, microbench, mydatastore_amd as mde
eng = mde.Engine(0)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
for B in (1000, 64):
    print("B", B, flush=True)
    microbench.bench_verify(eng, P=1, B=B, mode=0)
    torch.cuda.synchronize()
