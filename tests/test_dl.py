"""Caffe2DML / Keras2DML (reference: src/main/python/tests/test_mllearn_*.py train the
generated nn-library networks; here on a small synthetic image task)."""
import json

import numpy as np
import pytest

from systemml_amd.models.dl import Caffe2DML, Keras2DML, parse_prototxt

NET = """
name: "tiny"
layer { name: "data" type: "Data" top: "data" top: "label" }
layer { name: "conv1" type: "Convolution" bottom: "data" top: "conv1"
        convolution_param { num_output: 4 kernel_size: 3 stride: 1 pad: 1 } }
layer { name: "relu1" type: "ReLU" bottom: "conv1" top: "conv1" }
layer { name: "pool1" type: "Pooling" bottom: "conv1" top: "pool1"
        pooling_param { pool: MAX kernel_size: 2 stride: 2 } }
layer { name: "ip1" type: "InnerProduct" bottom: "pool1" top: "ip1" inner_product_param { num_output: 16 } }
layer { name: "relu2" type: "ReLU" bottom: "ip1" top: "ip1" }
layer { name: "drop" type: "Dropout" bottom: "ip1" top: "ip1" dropout_param { dropout_ratio: 0.1 } }
layer { name: "ip2" type: "InnerProduct" bottom: "ip1" top: "ip2" inner_product_param { num_output: 3 } }
layer { name: "loss" type: "SoftmaxWithLoss" bottom: "ip2" bottom: "label" top: "loss" }
"""


def _images(n=300, seed=0):
    rng = np.random.default_rng(seed)
    y = rng.integers(0, 3, n)
    X = rng.random((n, 1, 8, 8)) * 0.2
    for k in range(3):                       # class k: bright band at rows 2k .. 2k+2
        X[y == k, 0, 2 * k:2 * k + 3, :] += 1.0
    return X.reshape(n, -1), y


def test_prototxt_parser():
    d = parse_prototxt(NET)
    assert len(d["layer"]) == 9 and d["layer"][1]["convolution_param"]["num_output"] == 4
    assert d["layer"][0]["top"] == ["data", "label"] and d["layer"][3]["pooling_param"]["pool"] == "MAX"


def test_caffe2dml_trains(tmp_path):
    X, y = _images()
    (tmp_path / "net.prototxt").write_text(NET)
    (tmp_path / "solver.prototxt").write_text(
        'net: "net.prototxt"\nbase_lr: 0.05\nmomentum: 0.9\nweight_decay: 0.0001\nlr_policy: "fixed"\n'
        'max_iter: 150\ntype: "SGD"\n')
    m = Caffe2DML(solver=str(tmp_path / "solver.prototxt"), input_shape=(1, 8, 8)).set(batch_size=32)
    assert "conv1" in m.summary()
    m.fit(X, y)
    Xt, yt = _images(seed=1)
    assert m.score(Xt, yt) > 0.9
    assert "conv2d::forward" in m.train_script_ and "optim::update" in m.train_script_


def test_keras2dml_from_json_and_weights():
    X, y = _images(seed=2)
    cfg = {"class_name": "Sequential", "config": {"layers": [
        {"class_name": "Conv2D", "config": {"name": "c1", "filters": 4, "kernel_size": [3, 3], "strides": [1, 1],
                                            "padding": "same", "activation": "relu"}},
        {"class_name": "MaxPooling2D", "config": {"name": "p1", "pool_size": [2, 2]}},
        {"class_name": "Flatten", "config": {"name": "f"}},
        {"class_name": "Dense", "config": {"name": "d1", "units": 3, "activation": "softmax"}}]}}
    m = Keras2DML(keras_model=json.dumps(cfg), input_shape=(8, 8, 1), batch_size=32, max_iter=200,
                  optimizer="adam", lr=0.01, lr_policy="fixed", weight_decay=0.0)
    m.fit(X, y)
    assert m.score(X, y) > 0.9
    assert set(m.model_) == {"W_c1", "b_c1", "W_d1", "b_d1"}


def test_caffe2dml_load_converted_caffemodel(tmp_path):
    """convert_caffemodel output (<layer>_weight/_bias.mtx) warm-starts Caffe2DML."""
    from systemml_amd.io.writers import write_matrix
    import torch
    (tmp_path / "net.prototxt").write_text(NET)
    (tmp_path / "solver.prototxt").write_text('net: "net.prototxt"\nbase_lr: 0.0\nmax_iter: 1\ntype: "SGD"\n')
    m = Caffe2DML(solver=str(tmp_path / "solver.prototxt"), input_shape=(1, 8, 8))
    rng = np.random.default_rng(3)
    w = {"conv1_weight": rng.standard_normal((4, 9)), "conv1_bias": rng.standard_normal((4, 1)),
         "ip1_weight": rng.standard_normal((64, 16)), "ip1_bias": rng.standard_normal((1, 16))}
    d = tmp_path / "weights"
    d.mkdir()
    for k, v in w.items():
        write_matrix(torch.from_numpy(v), str(d / (k + ".mtx")), "csv")
    m.load(str(d), ignore_weights=["ip1"])
    assert set(m.init_weights_) == {"W_conv1", "b_conv1"}
    np.testing.assert_allclose(m.init_weights_["W_conv1"], w["conv1_weight"])
    m.load(str(d))
    assert set(m.init_weights_) == {"W_conv1", "b_conv1", "W_ip1", "b_ip1"}


RESNET = """
name: "res"
layer { name: "data" type: "Data" top: "data" top: "label" }
layer { name: "c1" type: "Convolution" bottom: "data" top: "c1" convolution_param { num_output: 4 kernel_size: 3 pad: 1 } }
layer { name: "bn1" type: "BatchNorm" bottom: "c1" top: "c1" }
layer { name: "sc1" type: "Scale" bottom: "c1" top: "c1" }
layer { name: "r1" type: "ReLU" bottom: "c1" top: "c1" }
layer { name: "c2" type: "Convolution" bottom: "c1" top: "c2" convolution_param { num_output: 4 kernel_size: 3 pad: 1 } }
layer { name: "c3" type: "Convolution" bottom: "c1" top: "c3" convolution_param { num_output: 2 kernel_size: 1 } }
layer { name: "sum" type: "Eltwise" bottom: "c1" bottom: "c2" top: "sum" eltwise_param { operation: SUM coeff: 1 coeff: 0.5 } }
layer { name: "cat" type: "Concat" bottom: "sum" bottom: "c3" top: "cat" }
layer { name: "pool" type: "Pooling" bottom: "cat" top: "pool" pooling_param { pool: AVE kernel_size: 2 stride: 2 } }
layer { name: "ip" type: "InnerProduct" bottom: "pool" top: "ip" inner_product_param { num_output: 3 } }
layer { name: "loss" type: "SoftmaxWithLoss" bottom: "ip" bottom: "label" top: "loss" }
"""


def _grad_script(layers, input_shape):
    """Forward + loss + backward of a generated network on fixed inputs (no update)."""
    from systemml_amd.models import dl
    gen = dl._Gen(layers, input_shape)
    lines = gen.sources() + ["Xb = X", "Yb = Y"] + gen.forward(train=True) + [f"loss = {gen.loss_expr()}"] + \
        gen.backward()
    grads = {t: gen.grad_of(t) for t in dl.trainable(gen.layers)}
    return "\n".join(lines), grads, dl.state_vars(gen.layers)


def test_dag_network_gradients_match_finite_differences():
    """Residual add with coefficients, channel concat of two branches, one activation
    consumed by three layers (gradient accumulation), BatchNorm + Scale: the generated
    backward pass agrees with central differences of the generated forward pass."""
    import os
    from systemml_amd.api.executor import run
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    from systemml_amd.conf import DMLConfig
    from systemml_amd.models import dl
    layers = dl.caffe_layers(parse_prototxt(RESNET))
    src, grads, state = _grad_script(layers, (1, 4, 4))
    rng = np.random.default_rng(0)
    X = rng.standard_normal((6, 16))
    Y = np.eye(3)[rng.integers(0, 3, 6)]
    init = dl._Gen(layers, (1, 4, 4)).init()
    w = run("\n".join(dl._Gen(layers, (1, 4, 4)).sources() + init), outputs=state, config=DMLConfig(gpu=False),
            out=lambda s: None, filename=os.path.join(SCRIPTS_DIR, "g.dml"))
    w = {k: np.asarray(v.double().numpy() if hasattr(v, "numpy") else v) for k, v in w.items()}
    cfg = DMLConfig(gpu=False)

    def ev(ws, outs):
        return run(src, inputs=dict(ws, X=X, Y=Y), outputs=outs, config=cfg, out=lambda s: None,
                   filename=os.path.join(SCRIPTS_DIR, "g.dml"))
    res = ev(w, ["loss"] + list(grads.values()))
    checked = 0
    for t, g in grads.items():
        G = res[g].double().numpy().reshape(w[t].shape)
        for idx in [(0, 0), tuple(np.array(w[t].shape) - 1)]:
            wp = {k: v.copy() for k, v in w.items()}
            wm = {k: v.copy() for k, v in w.items()}
            h = 1e-5
            wp[t][idx] += h
            wm[t][idx] -= h
            num = (ev(wp, ["loss"])["loss"] - ev(wm, ["loss"])["loss"]) / (2 * h)
            assert abs(num - G[idx]) < 1e-6 + 1e-4 * abs(num), (t, idx, num, G[idx])
            checked += 1
    assert checked == 2 * len(grads) and {"g_sc1", "be_sc1", "W_c2", "W_c3", "W_ip"} <= set(grads)


def test_caffe_residual_network_trains_all_algorithms(tmp_path):
    X, y = _images(n=240, seed=4)
    (tmp_path / "net.prototxt").write_text(RESNET)
    (tmp_path / "solver.prototxt").write_text('net: "net.prototxt"\nbase_lr: 0.05\nmomentum: 0.9\nlr_policy: "fixed"\n'
                                              'max_iter: 60\ntype: "SGD"\n')
    for algo in ("minibatch", "allreduce_parallel_batches"):
        m = Caffe2DML(solver=str(tmp_path / "solver.prototxt"), input_shape=(1, 8, 8))
        m.set(batch_size=16, train_algo=algo, parallel_batches=3, test_algo="allreduce")
        m.fit(X, y)
        assert m.score(X, y) > 0.9, algo
        assert {"em_bn1", "ev_bn1", "g_sc1", "be_sc1"} <= set(m.model_)
        if algo != "minibatch":
            assert "parfor (j in 1:ntask)" in m.train_script_
        assert "parfor (i in 1:iters)" in m.predict_script_
    with pytest.raises(ValueError):
        m.set(train_algo="nonsense")


def test_keras_functional_and_lstm():
    X, y = _images(n=240, seed=5)
    cfg = {"class_name": "Model", "config": {"layers": [
        {"class_name": "InputLayer", "name": "in", "config": {"name": "in"}, "inbound_nodes": []},
        {"class_name": "Conv2D", "name": "a", "config": {"name": "a", "filters": 3, "kernel_size": [3, 3],
                                                          "padding": "same", "activation": "relu"},
         "inbound_nodes": [[["in", 0, 0, {}]]]},
        {"class_name": "Conv2D", "name": "b", "config": {"name": "b", "filters": 3, "kernel_size": [1, 1],
                                                          "activation": "linear"},
         "inbound_nodes": [[["in", 0, 0, {}]]]},
        {"class_name": "Add", "name": "add", "config": {"name": "add"}, "inbound_nodes": [[["a", 0, 0, {}], ["b", 0, 0, {}]]]},
        {"class_name": "Concatenate", "name": "cat", "config": {"name": "cat", "axis": -3},
         "inbound_nodes": [[["add", 0, 0, {}], ["a", 0, 0, {}]]]},
        {"class_name": "Flatten", "name": "f", "config": {"name": "f"}, "inbound_nodes": [[["cat", 0, 0, {}]]]},
        {"class_name": "Dense", "name": "d", "config": {"name": "d", "units": 3, "activation": "softmax"},
         "inbound_nodes": [[["f", 0, 0, {}]]]}]}}
    m = Keras2DML(keras_model=json.dumps(cfg), input_shape=(1, 8, 8), batch_size=32, max_iter=120,
                  optimizer="adam", lr=0.01, lr_policy="fixed", weight_decay=0.0)
    m.fit(X, y)
    assert m.score(X, y) > 0.9
    # sequence classification with an LSTM: the class is which third of the sequence is bright
    rng = np.random.default_rng(6)
    n, T, D = 240, 6, 3
    ys = rng.integers(0, 3, n)
    S = rng.random((n, T, D)) * 0.2
    for k in range(3):
        S[ys == k, 2 * k:2 * k + 2, :] += 1.0
    seq = {"class_name": "Sequential", "config": {"layers": [
        {"class_name": "LSTM", "config": {"name": "lstm", "units": 8, "return_sequences": False}},
        {"class_name": "Dense", "config": {"name": "out", "units": 3, "activation": "softmax"}}]}}
    m2 = Keras2DML(keras_model=json.dumps(seq), input_shape=(T, D), batch_size=24, max_iter=150,
                   optimizer="adam", lr=0.02, lr_policy="fixed", weight_decay=0.0)
    m2.fit(S.reshape(n, -1), ys)
    assert m2.score(S.reshape(n, -1), ys) > 0.9
    assert "lstm::backward" in m2.train_script_
