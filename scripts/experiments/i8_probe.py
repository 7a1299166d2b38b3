# layout probe for the P_I8 GEMM: y[m][n] = sum_k q[m][k] w[n][k] with unit scales, structured data
import sys, os, types
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mipipe.ops.kernels import gemm_i8, EPI_STORE
M, n, k = 65, 32, 256
w = types.SimpleNamespace(n=n, k=k, n_pad=n, k_pad=k, ntiles=n // 16, nsb=k // 256)
W = torch.zeros(n, k, dtype=torch.int8)
for r in range(n):
    W[r, r] = 1; W[r, (5 * r + 3) % k] = 2
w.q = W.cuda()
v = w.q.view(w.ntiles, 16, w.nsb, 2, 2, 4, 16)
w.dev = v.permute(0, 2, 3, 4, 5, 1, 6).contiguous().view(-1)
w.ws = torch.ones(n, device="cuda")
X = torch.zeros(M, k, dtype=torch.int8)
for m in range(M):
    X[m, m % k] = 1; X[m, (7 * m + 1) % k] = 3
xs = torch.ones(M, device="cuda")
y = gemm_i8(w, xq=(X.cuda(), xs), epi=EPI_STORE).cpu()
ref = X.float() @ W.float().T
bad = (y != ref).nonzero()
print("mismatches", len(bad))
for m in range(4):
    print("row", m, "y nz", [(int(j), float(y[m, j])) for j in y[m].nonzero().flatten()][:8])
    print("row", m, "ref nz", [(int(j), float(ref[m, j])) for j in ref[m].nonzero().flatten()][:8])
