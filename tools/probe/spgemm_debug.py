"""Debug probe: SpGEMM mismatches vs a dense reference (row counts, duplicate columns)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import torch
import test_sparse_gpu as T
from systemml_amd.ops import kernels
T._need_gpu()
a = T._csr(1000, 700, 0.01, seed=1, empty_rows=125)
b = T._csr(700, 5000, 0.005, skew=True, seed=2)
A = a.to("cuda", torch.float32).to_sparse_csr()
B = b.to("cuda", torch.float32).to_sparse_csr()
ref = a @ b
for trial in range(3):
    C = kernels.spgemm(A, B)
    D = C.to_dense().double().cpu()
    bad = ((D - ref).abs() > 1e-3).nonzero()
    crow = C.crow_indices().cpu()
    refcnt = (ref != 0).sum(1)
    cnt = crow[1:] - crow[:-1]
    print("trial", trial, "bad", bad.shape[0], "rows with count mismatch", int((cnt != refcnt).sum()))
    for r, c in bad[:5].tolist():
        print("  ", r, c, float(D[r, c]), float(ref[r, c]), "cnt", int(cnt[r]), "ref", int(refcnt[r]))
print("B rows nnz max", int((b != 0).sum(1).max()), "A rows nnz max", int((a != 0).sum(1).max()))
