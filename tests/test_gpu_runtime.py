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
    np.testing.assert_allclose(r["D"].cpu().double().numpy(), A.T @ B, rtol=1e-3)
    assert st.counters.get("bufferpool.evict_host", 0) > 0 and st.counters.get("bufferpool.restore", 0) > 0
