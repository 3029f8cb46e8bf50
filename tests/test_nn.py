"""nn library tests: numerical gradient checks of every layer's backward pass (the
reference's scripts/nn/test/grad_check.dml strategy, driven from Python) plus the
optimizers and a small end-to-end training run."""
import numpy as np
import pytest

from systemml_amd.api.executor import run
from systemml_amd.conf import DMLConfig

CFG = DMLConfig(gpu=False)


def dml(src, inputs, outputs):
    res = run(src, inputs=inputs, outputs=outputs, config=CFG, out=lambda s: None)
    return {k: (v.numpy() if hasattr(v, "numpy") else v) for k, v in res.items()}


def gradcheck(layer, fwd_args, bwd_args, inputs, wrt, loss_w, extra_fwd_out="", h=1e-6, tol=1e-5):
    """Check d(sum(out * loss_w))/d(wrt) from <layer>::backward against finite differences."""
    src_f = f'source("nn/layers/{layer}.dml") as L\n[out{extra_fwd_out}] = L::forward({fwd_args})\nl = sum(out * LW)'
    src_b = (f'source("nn/layers/{layer}.dml") as L\n[out{extra_fwd_out}] = L::forward({fwd_args})\n'
             f'dout = LW\n{bwd_args}')
    ins = dict(inputs)
    ins["LW"] = loss_w
    grads = dml(src_b, ins, ["d" + w for w in wrt])
    rng = np.random.default_rng(0)
    for w in wrt:
        A = inputs[w]
        G = grads["d" + w]
        for _ in range(6):
            i = rng.integers(0, A.shape[0])
            j = rng.integers(0, A.shape[1])
            Ap, Am = A.copy(), A.copy()
            Ap[i, j] += h
            Am[i, j] -= h
            lp = dml(src_f, {**ins, w: Ap}, ["l"])["l"]
            lm = dml(src_f, {**ins, w: Am}, ["l"])["l"]
            num = (lp - lm) / (2 * h)
            assert abs(num - G[i, j]) <= tol * max(1.0, abs(num)), (layer, w, i, j, num, G[i, j])


rng = np.random.default_rng(42)


def R(*s):
    return rng.standard_normal(s)


def test_affine():
    gradcheck("affine", "X, W, b", "[dX, dW, db] = L::backward(dout, X, W, b)",
              {"X": R(4, 5), "W": R(5, 3), "b": R(1, 3)}, ["X", "W", "b"], R(4, 3))


@pytest.mark.parametrize("layer", ["relu", "sigmoid", "tanh"])
def test_activations(layer):
    gradcheck(layer, "X", "dX = L::backward(dout, X)", {"X": R(4, 5) + 0.01}, ["X"], R(4, 5))


def test_softmax():
    gradcheck("softmax", "X", "dX = L::backward(dout, X)", {"X": R(4, 5)}, ["X"], R(4, 5))


def test_conv2d_builtin():
    C, H, W, F, Hf = 2, 5, 5, 3, 3
    gradcheck("conv2d_builtin", f"X, W, b, {C}, {H}, {W}, {Hf}, {Hf}, 1, 1, 1, 1", ", Hout, Wout".join(["", ""])
              and f"[dX, dW, db] = L::backward(dout, Hout, Wout, X, W, b, {C}, {H}, {W}, {Hf}, {Hf}, 1, 1, 1, 1)",
              {"X": R(2, C * H * W), "W": R(F, C * Hf * Hf), "b": R(F, 1)}, ["X", "W", "b"],
              R(2, F * H * W), extra_fwd_out=", Hout, Wout")


def test_max_pool():
    C, H, W = 2, 4, 4
    X = rng.permutation(2 * C * H * W).reshape(2, C * H * W).astype(float)   # no ties
    gradcheck("max_pool2d_builtin", f"X, {C}, {H}, {W}, 2, 2, 2, 2, 0, 0",
              f"dX = L::backward(dout, Hout, Wout, X, {C}, {H}, {W}, 2, 2, 2, 2, 0, 0)",
              {"X": X}, ["X"], R(2, C * 4), extra_fwd_out=", Hout, Wout", h=1e-3)


def test_batch_norm1d():
    gradcheck("batch_norm1d", "X, g, b, 'train', em, ev, 0.9, 1e-5",
              "[dX, dg, db] = L::backward(dout, out, a, bb, cm, cv, cn, X, g, b, 'train', em, ev, 0.9, 1e-5)",
              {"X": R(6, 4), "g": R(1, 4), "b": R(1, 4), "em": np.zeros((1, 4)), "ev": np.ones((1, 4))},
              ["X", "g", "b"], R(6, 4), extra_fwd_out=", a, bb, cm, cv, cn")


def test_batch_norm2d():
    C, H, W = 2, 3, 3
    gradcheck("batch_norm2d", f"X, g, b, {C}, {H}, {W}, 'train', em, ev, 0.9, 1e-5",
              f"[dX, dg, db] = L::backward(dout, out, a, bb, cm, cv, cn, X, g, b, {C}, {H}, {W}, 'train', em, ev, 0.9, 1e-5)",
              {"X": R(4, C * H * W), "g": R(C, 1), "b": R(C, 1), "em": np.zeros((C, 1)), "ev": np.ones((C, 1))},
              ["X", "g", "b"], R(4, C * H * W), extra_fwd_out=", a, bb, cm, cv, cn")


def test_losses():
    pred = np.abs(R(5, 3)) + 0.1
    pred = pred / pred.sum(1, keepdims=True)
    y = np.eye(3)[rng.integers(0, 3, 5)]
    for layer in ("cross_entropy_loss", "l2_loss", "l1_loss"):
        r = dml(f'source("nn/layers/{layer}.dml") as L\nl = L::forward(p, y)\nd = L::backward(p, y)',
                {"p": pred, "y": y}, ["l", "d"])
        h = 1e-6
        P2 = pred.copy()
        P2[1, 2] += h
        r2 = dml(f'source("nn/layers/{layer}.dml") as L\nl = L::forward(p, y)', {"p": P2, "y": y}, ["l"])
        assert abs((r2["l"] - r["l"]) / h - r["d"][1, 2]) < 1e-4


def test_optimizers_decrease_quadratic():
    for opt, call, init in [
        ("sgd", "X = O::update(X, dX, 0.1)", ""),
        ("sgd_momentum", "[X, v] = O::update(X, dX, 0.05, 0.9, v)", "v = O::init(X)"),
        ("sgd_nesterov", "[X, v] = O::update(X, dX, 0.05, 0.9, v)", "v = O::init(X)"),
        ("adagrad", "[X, c] = O::update(X, dX, 0.5, 1e-8, c)", "c = O::init(X)"),
        ("rmsprop", "[X, c] = O::update(X, dX, 0.05, 0.9, 1e-8, c)", "c = O::init(X)"),
        ("adam", "[X, m, v] = O::update(X, dX, 0.1, 0.9, 0.999, 1e-8, i - 1, m, v)", "[m, v] = O::init(X)"),
    ]:
        r = dml(f'source("nn/optim/{opt}.dml") as O\n{init}\nfor (i in 1:100) {{ dX = 2 * X\n {call} }}\n'
                f'l = sum(X ^ 2)', {"X": np.ones((3, 2))}, ["l"])
        assert r["l"] < 6 * 0.1, (opt, r["l"])


def test_train_softmax_classifier():
    X = R(200, 4)
    y = np.eye(3)[np.argmax(X[:, :3], 1)]
    src = '''
source("nn/layers/affine.dml") as affine
source("nn/layers/softmax.dml") as softmax
source("nn/layers/cross_entropy_loss.dml") as ce
source("nn/optim/sgd.dml") as sgd
[W, b] = affine::init(4, 3)
for (e in 1:200) {
  s = affine::forward(X, W, b)
  p = softmax::forward(s)
  dp = ce::backward(p, Y)
  ds = softmax::backward(dp, s)
  [dX, dW, db] = affine::backward(ds, X, W, b)
  W = sgd::update(W, dW, 0.5)
  b = sgd::update(b, db, 0.5)
}
acc = mean(rowIndexMax(softmax::forward(affine::forward(X, W, b))) == rowIndexMax(Y))
'''
    assert dml(src, {"X": X, "Y": y}, ["acc"])["acc"] > 0.9


def test_rnn():
    N, T, D, M = 3, 4, 2, 3
    gradcheck("rnn", f"X, W, b, {T}, {D}, TRUE, h0",
              f"[dX, dW, db, dh0] = L::backward(dout, X, W, b, {T}, {D}, TRUE, h0, cache)",
              {"X": R(N, T * D), "W": R(D + M, M) * 0.5, "b": R(1, M), "h0": R(N, M)}, ["X", "W", "b", "h0"],
              R(N, T * M), extra_fwd_out=", cache")


def test_lstm():
    N, T, D, M = 2, 3, 2, 3
    gradcheck("lstm", f"X, W, b, {T}, {D}, TRUE, h0, c0",
              f"[dX, dW, db, dh0, dc0] = L::backward(dout, dc, X, W, b, {T}, {D}, TRUE, h0, c0, co, cc, cifog)",
              {"X": R(N, T * D), "W": R(D + M, 4 * M) * 0.5, "b": R(1, 4 * M), "h0": R(N, M), "c0": R(N, M),
               "dc": np.zeros((N, M))}, ["X", "W", "b", "h0", "c0"], R(N, T * M),
              extra_fwd_out=", c, co, cc, cifog")


def test_conv2d_transpose():
    C, H, W, F, Hf = 2, 3, 3, 3, 3
    Ho = 2 * (H - 1) - 2 + Hf + 1
    gradcheck("conv2d_transpose", f"X, W, b, {C}, {H}, {W}, {Hf}, {Hf}, 2, 2, 1, 1, 1, 1",
              f"[dX, dW, db] = L::backward(dout, Hout, Wout, X, W, b, {C}, {H}, {W}, {Hf}, {Hf}, 2, 2, 1, 1)",
              {"X": R(2, C * H * W), "W": R(C, F * Hf * Hf), "b": R(F, 1)}, ["X", "W", "b"],
              R(2, F * Ho * Ho), extra_fwd_out=", Hout, Wout")


def test_upsample2d_and_fm():
    gradcheck("upsample2d", "X, 2, 2, 3, 2, 2", "dX = L::backward(dout, 2, 2, 3, 2, 2)",
              {"X": R(2, 12)}, ["X"], R(2, 48))
    gradcheck("fm", "X, w0, W, V", "[dw0, dW, dV] = L::backward(dout, X, w0, W, V)",
              {"X": R(5, 4), "w0": R(1, 1), "W": R(4, 1), "V": R(4, 2)}, ["w0", "W", "V"], R(5, 1))


def test_depthwise():
    C, H, W, M, Hf = 2, 4, 4, 2, 3
    gradcheck("conv2d_depthwise", f"X, W, b, {H}, {W}, {M}, {Hf}, {Hf}, 1, 1, 1, 1",
              f"[dX, dW, db] = L::backward(dout, Hout, Wout, X, W, b, {H}, {W}, {M}, {Hf}, {Hf}, 1, 1, 1, 1)",
              {"X": R(2, C * H * W), "W": R(C, M * Hf * Hf), "b": R(C * M, 1)}, ["X", "W", "b"],
              R(2, C * M * H * W), extra_fwd_out=", Hout, Wout")
    gradcheck("conv2d_transpose_depthwise", f"X, W, b, 4, 3, 3, 2, 3, 3, 1, 1, 1, 1, 0, 0",
              f"[dX, dW, db] = L::backward(dout, Hout, Wout, X, W, b, 4, 3, 3, 2, 3, 3, 1, 1, 1, 1)",
              {"X": R(2, 4 * 9), "W": R(2, 2 * 9), "b": R(2, 1)}, ["X", "W", "b"],
              R(2, 2 * 9), extra_fwd_out=", Hout, Wout")


def test_lenet_example_trains_on_dummy_data():
    src = '''
source("nn/examples/mnist_lenet.dml") as lenet
N = 128
K = 10
X = rand(rows = N, cols = 1 * 12 * 12, pdf = "normal", seed = 1)
cls = rowIndexMax(X[, 1:K])
Y = table(seq(1, N), cls, N, K)
[W1, b1, W2, b2, W3, b3, W4, b4] = lenet::train(X, Y, X, Y, 1, 12, 12, 1)
p = lenet::predict(X, 1, 12, 12, W1, b1, W2, b2, W3, b3, W4, b4)
s = sum(p)
'''
    r = dml(src, {}, ["s"])
    assert abs(r["s"] - 128) < 1e-6


def test_dml_nn_test_suite():
    """scripts/nn/test/run_tests.dml: directional-derivative grad checks of every layer plus
    unit tests (the reference's in-DML test suite) report zero failures."""
    import os
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    path = os.path.join(SCRIPTS_DIR, "nn", "test", "run_tests.dml")
    out = []
    run(open(path).read(), config=CFG, out=out.append, filename=path)
    errors = [s for s in out if s.startswith("ERROR")]
    assert not errors, errors
    assert out[-1] == "NN TESTS FAILED: 0"


def test_nn_example_drivers(tmp_path):
    """Softmax / LeNet train + predict drivers, the data-parallel LeNet and the FM dummy-data
    drivers run end to end on small synthetic CSV data."""
    import os
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    from systemml_amd.io.readers import read_matrix
    import torch
    from systemml_amd.io.writers import write_matrix
    ex = os.path.join(SCRIPTS_DIR, "nn", "examples")
    g = np.random.default_rng(0)
    lab = g.integers(0, 10, (60, 1)).astype(float)
    data = np.hstack([lab, g.integers(0, 256, (60, 64)).astype(float)])
    write_matrix(torch.from_numpy(data), str(tmp_path / "train.csv"), "csv")

    def go(name, args):
        p = os.path.join(ex, name)
        out = []
        run(open(p).read(), args=args, config=CFG, out=out.append, filename=p)
        return out

    out = go("mnist_softmax-train.dml", dict(train=str(tmp_path / "train.csv"), test=str(tmp_path / "train.csv"),
                                             out_dir=str(tmp_path)))
    assert any(s.startswith("Test Accuracy") for s in out)
    write_matrix(torch.from_numpy(data[:, 1:]), str(tmp_path / "X.csv"), "csv")
    go("mnist_softmax-predict.dml", dict(X=str(tmp_path / "X.csv"), model_dir=str(tmp_path), out_dir=str(tmp_path)))
    P = read_matrix(str(tmp_path / "probs")).numpy()
    np.testing.assert_allclose(P.sum(axis=1), 1, atol=1e-9)
    out = go("mnist_lenet_distrib_sgd-train-dummy-data.dml", dict(N=16, Nval=8, Hin=8, Win=8, batch_size=4,
                                                                  parallel_batches=2, epochs=1))
    assert any("Dummy data validation" in s for s in out)
    out = go("fm-regression-dummy-data.dml", dict(n=50, d=3))
    assert any("Validation loss" in s for s in out)
