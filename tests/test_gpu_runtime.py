"""GPU runtime tests: buffer-pool eviction under a zero HBM budget must not change results."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_bufferpool_eviction_keeps_results(gpu_config):
    from systemml_amd.api.executor import run
    gpu_config.bufferpool_hbm_fraction = 0.0        # evict every idle variable after each block
    X = np.random.default_rng(0).standard_normal((4096, 300))
    src = '''
A = X %*% t(X[1:300,])
B = A * 2
s = 0
for (i in 1:3) {
  C = B + i
  s = s + sum(C)
}
D = t(A) %*% B
'''
    from systemml_amd.utils.stats import Statistics
    st = Statistics(enabled=True)
    r = run(src, inputs={"X": X}, outputs=["s", "D"], config=gpu_config, stats=st)
    A = X @ X[:300].T
    B = 2 * A
    ref_s = sum((B + i).sum() for i in (1, 2, 3))
    np.testing.assert_allclose(r["s"], ref_s, rtol=1e-4)
    ref_d = A.T @ B
    np.testing.assert_allclose(r["D"].cpu().double().numpy(), ref_d, rtol=1e-3, atol=1e-5 * np.abs(ref_d).max())
    assert st.counters.get("bufferpool.evict_host", 0) > 0 and st.counters.get("bufferpool.restore", 0) > 0


def test_sparse_ops_on_gpu(gpu_config):
    from systemml_amd.api.executor import run
    from systemml_amd.ops import sparse as SP
    r = run("""A = rand(rows=20000, cols=800, sparsity=0.01, seed=5)
v = rand(rows=800, cols=1, seed=6)
u = A %*% v
g = t(A) %*% u
B = t(A) %*% A
s = sum(A)
""", outputs=["A", "v", "u", "g", "B", "s"], config=gpu_config)
    A = r["A"]
    assert SP.is_sparse(A) and A.is_cuda
    Ad = A.to_dense().double().cpu().numpy()
    v = r["v"].double().cpu().numpy()
    np.testing.assert_allclose(r["u"].double().cpu().numpy(), Ad @ v, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(r["g"].double().cpu().numpy(), Ad.T @ (Ad @ v), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(r["B"].double().cpu().numpy(), Ad.T @ Ad, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(r["s"], Ad.sum(), rtol=1e-5)
