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
