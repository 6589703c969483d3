import sys; sys.path[:0]=['.','mh-spgemm_amd','tests']
import torch, mhspgemm
from mhspgemm import synth
t = mhspgemm.Tool(0)
print("ctx ok", torch.cuda.is_available()); sys.stdout.flush()
x = torch.zeros(4, device='cuda:0'); torch.cuda.synchronize(); print("torch ok"); sys.stdout.flush()
A = synth.cage4_like(); A.H2D(0); print("h2d ok"); sys.stdout.flush()
C, tm = mhspgemm.spgemm(t, A, A); print("spgemm ok", C.nnz); sys.stdout.flush()
