"""Toolchain probe on the GPU box: load the in-tree HIP module under PyTorch's HIP runtime."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
t0 = time.time()
print("torch", torch.__version__, "hip", torch.version.hip, "cuda avail", torch.cuda.is_available(), flush=True)
from rocfm import _rocfm_hip as H
print("arch", H.arch(), flush=True)
x = torch.zeros(1024, device="cuda")
H.probe(x.data_ptr(), x.numel(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
print("probe out", x[:4].tolist(), x[60:68].tolist(), flush=True)
g = torch.cuda.CUDAGraph()
y = torch.zeros(256, device="cuda")
with torch.cuda.graph(g):
    H.probe(y.data_ptr(), y.numel(), torch.cuda.current_stream().cuda_stream)
g.replay(); torch.cuda.synchronize()
print("graph probe", y[:2].tolist(), "ok", time.time() - t0, flush=True)
