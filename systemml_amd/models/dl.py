"""Deep-learning model import: Caffe2DML and Keras2DML (reference: scala
org/apache/sysml/api/dl/{Caffe2DML,CaffeLayer,CaffeNetwork,CaffeSolver,DMLGenerator}.scala and
src/main/python/systemml/mllearn/{estimators.py (Caffe2DML, Keras2DML), keras2caffe.py}).

The reference converts a Keras model to a Caffe network + solver, then Caffe2DML generates
a DML training / prediction script over the nn library.  Here both front ends produce the
same small layer IR, and one generator emits DML that calls scripts/nn (conv2d_builtin,
affine, max/avg pooling, relu/sigmoid/tanh, dropout, softmax + cross-entropy) with the
solver's optimizer (SGD, momentum, Nesterov, Adam, AdaGrad, RMSProp), learning-rate policy
(fixed / step / exp / inv) and L2 weight decay.  The generated script runs on the MI355X
backend like any other DML (conv / pool go to MIOpen through torch, affine to hipBLASLt).

Supported networks: sequential chains (one bottom / top per layer).
Front ends:
  * Caffe: network and solver prototxt text (a protobuf text-format parser is included).
  * Keras: a Keras model object (duck-typed: `model.layers[i].get_config()` and
    `__class__.__name__`), or its `model.to_json()` string / dict -- keras itself is not
    required.
"""
from __future__ import annotations

import json
import math
import os
import re

import numpy as np

from .mllearn import BaseSystemMLClassifier, _np, _out
from ..api.executor import run
from ..api.mlcontext import SCRIPTS_DIR


# ============================================================================
# protobuf text format (Caffe prototxt)
# ============================================================================
_TOK = re.compile(r'\s*(?:(#[^\n]*)|("(?:[^"\\]|\\.)*")|([{}:])|([^\s{}:#"]+))')


def parse_prototxt(text):
    """Protobuf text format -> nested dict; repeated fields become lists."""
    toks = []
    pos = 0
    while pos < len(text):
        m = _TOK.match(text, pos)
        if not m or m.end() == pos:
            break
        pos = m.end()
        if m.group(1):
            continue
        toks.append(m.group(2) or m.group(3) or m.group(4))
    i = 0

    def value(t):
        if t.startswith('"'):
            return bytes(t[1:-1], "utf-8").decode("unicode_escape")
        if t in ("true", "false"):
            return t == "true"
        try:
            return int(t)
        except ValueError:
            try:
                return float(t)
            except ValueError:
                return t          # enum

    def msg(end):
        nonlocal i
        out = {}
        rep = set()
        while i < len(toks) and toks[i] != end:
            key = toks[i]
            i += 1
            if toks[i] == ":":
                i += 1
            if toks[i] == "{":
                i += 1
                v = msg("}")
                i += 1
            else:
                v = value(toks[i])
                i += 1
            if key in out:
                if key not in rep:
                    out[key] = [out[key]]
                    rep.add(key)
                out[key].append(v)
            else:
                out[key] = v
        return out

    return msg(None)


def _as_list(v):
    if v is None:
        return []
    return v if isinstance(v, list) else [v]


# ============================================================================
# layer IR
# ============================================================================
class Layer:
    def __init__(self, kind, name, **p):
        self.kind = kind          # conv | dense | pool | relu | sigmoid | tanh | dropout | softmax | flatten
        self.name = re.sub(r"\W", "_", name)
        self.p = p
        self.shape_in = None
        self.shape_out = None     # (C, H, W); dense outputs (D, 1, 1)

    def __repr__(self):
        return f"{self.kind}:{self.name}{self.p}"


def caffe_layers(net):
    """Caffe NetParameter dict -> layer IR (data / accuracy layers dropped)."""
    out = []
    for L in _as_list(net.get("layer") or net.get("layers")):
        t = str(L.get("type", "")).lower()
        name = str(L.get("name", t))
        if t in ("data", "input", "memorydata", "accuracy", "silence"):
            continue
        if t == "convolution":
            cp = L.get("convolution_param", {})
            k = cp.get("kernel_size", 3)
            k = k[0] if isinstance(k, list) else k
            out.append(Layer("conv", name, F=int(cp["num_output"]), kh=int(cp.get("kernel_h", k)),
                             kw=int(cp.get("kernel_w", k)), sh=int(cp.get("stride_h", _first(cp.get("stride", 1)))),
                             sw=int(cp.get("stride_w", _first(cp.get("stride", 1)))),
                             ph=int(cp.get("pad_h", _first(cp.get("pad", 0)))),
                             pw=int(cp.get("pad_w", _first(cp.get("pad", 0))))))
        elif t == "innerproduct":
            out.append(Layer("dense", name, M=int(L.get("inner_product_param", {})["num_output"])))
        elif t == "pooling":
            pp = L.get("pooling_param", {})
            k = int(pp.get("kernel_size", 2))
            s = int(pp.get("stride", 1))
            out.append(Layer("pool", name, mode=str(pp.get("pool", "MAX")).upper(), kh=int(pp.get("kernel_h", k)),
                             kw=int(pp.get("kernel_w", k)), sh=int(pp.get("stride_h", s)), sw=int(pp.get("stride_w", s)),
                             ph=int(pp.get("pad_h", pp.get("pad", 0))), pw=int(pp.get("pad_w", pp.get("pad", 0)))))
        elif t in ("relu", "sigmoid", "tanh"):
            out.append(Layer(t, name))
        elif t == "dropout":
            out.append(Layer("dropout", name, rate=float(L.get("dropout_param", {}).get("dropout_ratio", 0.5))))
        elif t in ("softmax", "softmaxwithloss"):
            out.append(Layer("softmax", name))
        elif t == "flatten":
            out.append(Layer("flatten", name))
        else:
            raise ValueError(f"Caffe2DML: unsupported layer type {L.get('type')}")
    return out


def _first(v):
    return v[0] if isinstance(v, list) else v


def _pair(v, d):
    if v is None:
        return (d, d)
    if isinstance(v, (list, tuple)):
        return (int(v[0]), int(v[1] if len(v) > 1 else v[0]))
    return (int(v), int(v))


def keras_layers(model):
    """Keras Sequential model / JSON config -> (layer IR, keras weight arrays by layer name)."""
    weights = {}
    if isinstance(model, (str, bytes)):
        model = json.loads(model)
    if isinstance(model, dict):
        cfg = model.get("config", model)
        specs = [(l["class_name"], l.get("config", {})) for l in (cfg["layers"] if isinstance(cfg, dict) else cfg)]
    else:
        specs = []
        for l in model.layers:
            specs.append((type(l).__name__, l.get_config()))
            w = l.get_weights() if hasattr(l, "get_weights") else []
            if w:
                weights[re.sub(r"\W", "_", l.get_config().get("name", ""))] = [np.asarray(a) for a in w]
    out = []
    for cls, c in specs:
        name = c.get("name", cls.lower() + str(len(out)))
        act = c.get("activation")
        if cls in ("InputLayer",):
            continue
        if cls in ("Conv2D", "Convolution2D"):
            kh, kw = _pair(c.get("kernel_size"), 3)
            sh, sw = _pair(c.get("strides"), 1)
            same = c.get("padding", "valid") == "same"
            out.append(Layer("conv", name, F=int(c.get("filters")), kh=kh, kw=kw, sh=sh, sw=sw,
                             ph=(kh - 1) // 2 if same else 0, pw=(kw - 1) // 2 if same else 0))
        elif cls == "Dense":
            out.append(Layer("dense", name, M=int(c.get("units"))))
        elif cls in ("MaxPooling2D", "AveragePooling2D"):
            kh, kw = _pair(c.get("pool_size"), 2)
            sh, sw = _pair(c.get("strides") or (kh, kw), kh)
            out.append(Layer("pool", name, mode="MAX" if cls.startswith("Max") else "AVE", kh=kh, kw=kw, sh=sh, sw=sw,
                             ph=0, pw=0))
        elif cls == "Flatten":
            out.append(Layer("flatten", name))
        elif cls == "Dropout":
            out.append(Layer("dropout", name, rate=float(c.get("rate", 0.5))))
        elif cls == "Activation":
            act = c.get("activation")
            cls = None
        else:
            raise ValueError(f"Keras2DML: unsupported layer {cls}")
        if act and act != "linear":
            if act not in ("relu", "sigmoid", "tanh", "softmax"):
                raise ValueError(f"Keras2DML: unsupported activation {act}")
            out.append(Layer(act, f"{name}_{act}"))
    return out, weights


def infer_shapes(layers, input_shape):
    C, H, W = input_shape
    shape = (C, H, W)
    for L in layers:
        L.shape_in = shape
        c, h, w = shape
        if L.kind == "conv":
            ho = (h + 2 * L.p["ph"] - L.p["kh"]) // L.p["sh"] + 1
            wo = (w + 2 * L.p["pw"] - L.p["kw"]) // L.p["sw"] + 1
            shape = (L.p["F"], ho, wo)
        elif L.kind == "pool":
            ho = (h + 2 * L.p["ph"] - L.p["kh"]) // L.p["sh"] + 1
            wo = (w + 2 * L.p["pw"] - L.p["kw"]) // L.p["sw"] + 1
            shape = (c, ho, wo)
        elif L.kind == "dense":
            shape = (L.p["M"], 1, 1)
        L.shape_out = shape
    return shape


# ============================================================================
# DML generation
# ============================================================================
_SRC = {"conv": ("conv2d", "nn/layers/conv2d_builtin.dml"), "dense": ("affine", "nn/layers/affine.dml"),
        "relu": ("relu", "nn/layers/relu.dml"), "sigmoid": ("sigmoid", "nn/layers/sigmoid.dml"),
        "tanh": ("tanh", "nn/layers/tanh.dml"), "dropout": ("dropout", "nn/layers/dropout.dml"),
        "softmax": ("softmax", "nn/layers/softmax.dml")}
_OPT = {"sgd": "nn/optim/sgd.dml", "momentum": "nn/optim/sgd_momentum.dml", "nesterov": "nn/optim/sgd_nesterov.dml",
        "adam": "nn/optim/adam.dml", "adagrad": "nn/optim/adagrad.dml", "rmsprop": "nn/optim/rmsprop.dml"}


def _params(layers):
    return [L for L in layers if L.kind in ("conv", "dense")]


def _sources(layers, opt=None):
    kinds = {L.kind for L in layers}
    lines = []
    for k in ("conv", "dense", "relu", "sigmoid", "tanh", "dropout", "softmax"):
        if k in kinds:
            ns, path = _SRC[k]
            lines.append(f'source("{path}") as {ns}')
    if "pool" in kinds:
        modes = {L.p["mode"] for L in layers if L.kind == "pool"}
        if "MAX" in modes:
            lines.append('source("nn/layers/max_pool2d_builtin.dml") as max_pool2d')
        if modes - {"MAX"}:
            lines.append('source("nn/layers/avg_pool2d_builtin.dml") as avg_pool2d')
    lines.append('source("nn/layers/cross_entropy_loss.dml") as cross_entropy_loss')
    if opt:
        lines.append(f'source("{_OPT[opt]}") as optim')
    return "\n".join(lines)


def _forward(layers, train):
    """Forward pass over `Xb`; returns (code, name of the final output, per-layer outputs)."""
    code = []
    cur = "Xb"
    for i, L in enumerate(layers):
        o = f"out{i}"
        c, h, w = L.shape_in
        if L.kind == "conv":
            p = L.p
            code.append(f"[{o}, Ho{i}, Wo{i}] = conv2d::forward({cur}, W_{L.name}, b_{L.name}, {c}, {h}, {w}, "
                        f"{p['kh']}, {p['kw']}, {p['sh']}, {p['sw']}, {p['ph']}, {p['pw']})")
        elif L.kind == "pool":
            p = L.p
            ns = "max_pool2d" if p["mode"] == "MAX" else "avg_pool2d"
            code.append(f"[{o}, Ho{i}, Wo{i}] = {ns}::forward({cur}, {c}, {h}, {w}, {p['kh']}, {p['kw']}, "
                        f"{p['sh']}, {p['sw']}, {p['ph']}, {p['pw']})")
        elif L.kind == "dense":
            code.append(f"{o} = affine::forward({cur}, W_{L.name}, b_{L.name})")
        elif L.kind in ("relu", "sigmoid", "tanh", "softmax"):
            code.append(f"{o} = {L.kind}::forward({cur})")
        elif L.kind == "dropout":
            if train:
                code.append(f"[{o}, mask{i}] = dropout::forward({cur}, {1 - L.p['rate']}, -1)")
            else:
                code.append(f"{o} = {cur}")
        else:   # flatten: DML activations are already N x (C*H*W)
            code.append(f"{o} = {cur}")
        cur = o
    return code, cur


def _backward(layers):
    code = []
    n = len(layers)
    for i in range(n - 1, -1, -1):
        L = layers[i]
        inp = "Xb" if i == 0 else f"out{i - 1}"
        d_out, d_in = f"dout{i}", f"dout{i - 1}" if i > 0 else "dXb"
        c, h, w = L.shape_in
        if L.kind == "conv":
            p = L.p
            code.append(f"[{d_in}, dW_{L.name}, db_{L.name}] = conv2d::backward({d_out}, Ho{i}, Wo{i}, {inp}, "
                        f"W_{L.name}, b_{L.name}, {c}, {h}, {w}, {p['kh']}, {p['kw']}, {p['sh']}, {p['sw']}, "
                        f"{p['ph']}, {p['pw']})")
        elif L.kind == "pool":
            p = L.p
            ns = "max_pool2d" if p["mode"] == "MAX" else "avg_pool2d"
            code.append(f"{d_in} = {ns}::backward({d_out}, Ho{i}, Wo{i}, {inp}, {c}, {h}, {w}, {p['kh']}, "
                        f"{p['kw']}, {p['sh']}, {p['sw']}, {p['ph']}, {p['pw']})")
        elif L.kind == "dense":
            code.append(f"[{d_in}, dW_{L.name}, db_{L.name}] = affine::backward({d_out}, {inp}, W_{L.name}, b_{L.name})")
        elif L.kind in ("relu", "sigmoid", "tanh", "softmax"):
            code.append(f"{d_in} = {L.kind}::backward({d_out}, {inp})")
        elif L.kind == "dropout":
            code.append(f"{d_in} = dropout::backward({d_out}, {inp}, {1 - L.p['rate']}, mask{i})")
        else:
            code.append(f"{d_in} = {d_out}")
    return code


def _init(layers, seed):
    code = []
    for L in _params(layers):
        c, h, w = L.shape_in
        if L.kind == "conv":
            code.append(f"[W_{L.name}, b_{L.name}] = conv2d::init({L.p['F']}, {c}, {L.p['kh']}, {L.p['kw']})")
        else:
            code.append(f"[W_{L.name}, b_{L.name}] = affine::init({c * h * w}, {L.p['M']})")
    return code


def generate_train_dml(layers, input_shape, solver, epochs, batch_size, seed=-1):
    infer_shapes(layers, input_shape)
    if not layers or layers[-1].kind != "softmax":
        layers.append(Layer("softmax", "prob"))
        infer_shapes(layers, input_shape)
    opt = solver.get("type", "sgd")
    lr = float(solver.get("base_lr", 0.01))
    mom = float(solver.get("momentum", 0.9))
    wd = float(solver.get("weight_decay", 0.0))
    policy = str(solver.get("lr_policy", "fixed")).lower()
    gamma = float(solver.get("gamma", 0.95))
    step = int(solver.get("stepsize", 1000))
    power = float(solver.get("power", 1.0))
    beta2 = float(solver.get("momentum2", 0.999))
    eps = float(solver.get("delta", 1e-8))
    decay = float(solver.get("rms_decay", 0.99))
    P = _params(layers)
    fwd, prob = _forward(layers, train=True)
    bwd = _backward(layers)
    lines = [_sources(layers, opt), "", "X = read($X)", "Y = read($Y)", "N = nrow(X)",
             f"epochs = {int(epochs)}", f"bs = {int(batch_size)}", f"lr0 = {lr}", "lr = lr0"]
    lines += _init(layers, seed)
    for L in P:
        for v in ("W", "b"):
            t = f"{v}_{L.name}"
            if opt in ("momentum", "nesterov"):
                lines.append(f"v_{t} = optim::init({t})")
            elif opt == "adam":
                lines.append(f"[m_{t}, s_{t}] = optim::init({t})")
            elif opt in ("adagrad", "rmsprop"):
                lines.append(f"c_{t} = optim::init({t})")
    lines += ["iters = as.integer(ceil(N / bs))", "it = 0", "loss = 0.0", "for (e in 1:epochs) {",
              "  for (i in 1:iters) {", "    beg = (i - 1) * bs + 1", "    end = min(N, beg + bs - 1)",
              "    Xb = X[beg:end, ]", "    Yb = Y[beg:end, ]"]
    lines += ["    " + c for c in fwd]
    lines += [f"    loss = cross_entropy_loss::forward({prob}, Yb)",
              f"    dout{len(layers) - 1} = cross_entropy_loss::backward({prob}, Yb)"]
    lines += ["    " + c for c in bwd]
    for L in P:
        for v in ("W", "b"):
            t = f"{v}_{L.name}"
            g = f"d{t}"
            if wd > 0 and v == "W":
                lines.append(f"    {g} = {g} + {wd} * {t}")
            if opt == "sgd":
                lines.append(f"    {t} = optim::update({t}, {g}, lr)")
            elif opt in ("momentum", "nesterov"):
                lines.append(f"    [{t}, v_{t}] = optim::update({t}, {g}, lr, {mom}, v_{t})")
            elif opt == "adam":
                lines.append(f"    [{t}, m_{t}, s_{t}] = optim::update({t}, {g}, lr, {mom}, {beta2}, {eps}, it, "
                             f"m_{t}, s_{t})")
            elif opt == "adagrad":
                lines.append(f"    [{t}, c_{t}] = optim::update({t}, {g}, lr, {eps}, c_{t})")
            elif opt == "rmsprop":
                lines.append(f"    [{t}, c_{t}] = optim::update({t}, {g}, lr, {decay}, {eps}, c_{t})")
    lines.append("    it = it + 1")
    if policy == "step":
        lines.append(f"    lr = lr0 * {gamma} ^ floor(it / {step})")
    elif policy == "exp":
        lines.append(f"    lr = lr0 * {gamma} ^ it")
    elif policy == "inv":
        lines.append(f"    lr = lr0 * (1 + {gamma} * it) ^ (-{power})")
    lines += ["  }", '  print("Epoch " + e + ": loss " + loss)', "}"]
    return "\n".join(lines), [f"{v}_{L.name}" for L in P for v in ("W", "b")]


def generate_predict_dml(layers, input_shape, batch_size):
    infer_shapes(layers, input_shape)
    fwd, prob = _forward(layers, train=False)
    lines = [_sources(layers), "", "X = read($X)", "N = nrow(X)", f"bs = {int(batch_size)}",
             f"P = matrix(0, rows = N, cols = {layers[-1].shape_out[0]})",
             "iters = as.integer(ceil(N / bs))", "for (i in 1:iters) {", "  beg = (i - 1) * bs + 1",
             "  end = min(N, beg + bs - 1)", "  Xb = X[beg:end, ]"]
    lines += ["  " + c for c in fwd]
    lines += [f"  P[beg:end, ] = {prob}", "}"]
    return "\n".join(lines)


# ============================================================================
# estimators
# ============================================================================
class Caffe2DML(BaseSystemMLClassifier):
    """Train / score a Caffe-defined network on the DML nn library.

    solver: path of a solver prototxt (its `net:` field names the network prototxt) or a
    dict of solver fields; network: optional network prototxt path / text (overrides
    `net:`); input_shape: (C, H, W) of one example (rows of X are C*H*W, channel-major).
    """

    def __init__(self, sparkSession=None, solver=None, input_shape=None, network=None, transferUsingDF=False):
        super().__init__(sparkSession)
        self.solver = self._read_solver(solver)
        net = network if network is not None else self.solver.get("net")
        if net is None:
            raise ValueError("Caffe2DML: no network prototxt given")
        text = open(net).read() if isinstance(net, str) and os.path.exists(net) else net
        self.layers = caffe_layers(parse_prototxt(text) if isinstance(text, str) else text)
        self.input_shape = tuple(int(v) for v in input_shape)
        self.max_iter = int(self.solver.get("max_iter", 100))
        self.batch_size = 64
        self.debug = False

    @staticmethod
    def _read_solver(solver):
        if solver is None:
            return {}
        if isinstance(solver, dict):
            s = dict(solver)
        else:
            text = open(solver).read() if os.path.exists(solver) else solver
            s = parse_prototxt(text)
            net = s.get("net")
            if isinstance(net, str) and not os.path.isabs(net) and os.path.exists(str(solver)):
                cand = os.path.join(os.path.dirname(solver), net)
                if os.path.exists(cand):
                    s["net"] = cand
        typ = str(s.get("type", s.get("solver_type", "SGD"))).lower()
        s["type"] = {"sgd": "momentum" if float(s.get("momentum", 0)) > 0 else "sgd", "nesterov": "nesterov",
                     "adam": "adam", "adagrad": "adagrad", "rmsprop": "rmsprop"}.get(typ, "sgd")
        return s

    def set(self, debug=None, train_algo=None, test_algo=None, parallel_batches=None, output_activations=None,
            perform_one_hot_encoding=None, parfor_parameters=None, batch_size=None):
        if debug is not None:
            self.debug = bool(debug)
        if batch_size is not None:
            self.batch_size = int(batch_size)
        return self

    def summary(self):
        infer_shapes(self.layers, self.input_shape)
        rows = ["Layer                Type       Output shape     Params"]
        for L in self.layers:
            npar = 0
            if L.kind == "conv":
                npar = L.p["F"] * (L.shape_in[0] * L.p["kh"] * L.p["kw"] + 1)
            elif L.kind == "dense":
                npar = L.p["M"] * (int(np.prod(L.shape_in)) + 1)
            rows.append(f"{L.name:<20s} {L.kind:<10s} {str(L.shape_out):<16s} {npar}")
        s = "\n".join(rows)
        print(s)
        return s

    def fit(self, X, y, params=None):
        X = _np(X)
        Y = np.eye(len(np.unique(y)))[self.encode(y).ravel().astype(int) - 1]
        n = X.shape[0]
        epochs = max(1, math.ceil(self.max_iter * self.batch_size / n))
        src, wnames = generate_train_dml(self.layers, self.input_shape, self.solver, epochs, self.batch_size)
        self.train_script_ = src
        inputs = {"X": X, "Y": Y}
        if getattr(self, "init_weights_", None):
            # warm start: replace the init() calls by bound inputs
            src = "\n".join(l for l in src.split("\n") if not re.match(r"\[W_\w+, b_\w+\] = \w+::init", l))
            inputs.update(self.init_weights_)
        out = []
        res = run(src, args={"X": "X", "Y": "Y"}, inputs=inputs, outputs=wnames, config=self.config,
                  out=out.append, filename=os.path.join(SCRIPTS_DIR, "caffe2dml_train.dml"))
        self.log_ = out
        self.model_ = {k: _out(v) for k, v in res.items()}
        return self

    def predict_proba(self, X):
        src = generate_predict_dml(self.layers, self.input_shape, max(self.batch_size, 256))
        self.predict_script_ = src
        inputs = {"X": _np(X)}
        inputs.update(self.model_)
        res = run(src, args={"X": "X"}, inputs=inputs, outputs=["P"], config=self.config, out=lambda s: None,
                  filename=os.path.join(SCRIPTS_DIR, "caffe2dml_predict.dml"))
        return _out(res["P"])

    def load(self, weights=None, sep="/", ignore_weights=None, eager=False):
        """Warm start from a directory of <layer>_weight.mtx / <layer>_bias.mtx matrices
        (as written by converters.convert_caffemodel); layers in ignore_weights keep their
        initialisation (reference: Caffe2DML.load in the Python mllearn API)."""
        from ..io.readers import read_matrix
        ignore = set(ignore_weights or [])
        found = {}
        for L in _params(self.layers):
            if L.name in ignore:
                continue
            for part, key in (("weight", "W"), ("bias", "b")):
                path = f"{weights}{sep}{L.name}_{part}.mtx"
                if os.path.exists(path):
                    found[f"{key}_{L.name}"] = _np(read_matrix(path))
        self.init_weights_ = found or None
        return self

    @property
    def model_keys(self):
        return [f"{v}_{L.name}" for L in _params(self.layers) for v in ("W", "b")]


class Keras2DML(Caffe2DML):
    """Keras Sequential model -> DML (reference: Keras2DML via keras2caffe + Caffe2DML)."""

    def __init__(self, sparkSession=None, keras_model=None, input_shape=None, transferUsingDF=False,
                 load_keras_weights=True, weights=None, labels=None, batch_size=64, max_iter=2000, test_iter=10,
                 test_interval=500, display=100, lr_policy="step", weight_decay=5e-4, regularization_type="L2",
                 optimizer="sgd", lr=0.01, momentum=0.9):
        BaseSystemMLClassifier.__init__(self, sparkSession)
        self.layers, kw = keras_layers(keras_model)
        if input_shape is not None and len(input_shape) == 3 and input_shape[-1] in (1, 3) and input_shape[0] not in (1, 3):
            input_shape = (input_shape[2], input_shape[0], input_shape[1])     # Keras HWC -> CHW
        self.input_shape = tuple(int(v) for v in (input_shape if len(input_shape) == 3 else (input_shape[0], 1, 1)))
        opt = {"sgd": "momentum" if momentum > 0 else "sgd", "adam": "adam", "adagrad": "adagrad",
               "rmsprop": "rmsprop", "nesterov": "nesterov"}[optimizer.lower()]
        self.solver = {"type": opt, "base_lr": lr, "momentum": momentum, "lr_policy": lr_policy,
                       "weight_decay": weight_decay if regularization_type == "L2" else 0.0, "gamma": 0.95,
                       "stepsize": test_interval}
        self.max_iter = int(max_iter)
        self.batch_size = int(batch_size)
        self.debug = False
        self.init_weights_ = None
        if load_keras_weights and kw:
            self.init_weights_ = self._convert_keras_weights(kw)

    def _convert_keras_weights(self, kw):
        infer_shapes(self.layers, self.input_shape)
        out = {}
        for L in _params(self.layers):
            w = kw.get(L.name)
            if not w:
                continue
            W, b = w[0], w[1] if len(w) > 1 else np.zeros(w[0].shape[-1])
            if L.kind == "conv":       # (kh, kw, C, F) -> F x (C*kh*kw)
                W = np.transpose(W, (3, 2, 0, 1)).reshape(W.shape[3], -1)
                out[f"W_{L.name}"], out[f"b_{L.name}"] = W, b.reshape(-1, 1)
            else:                      # Dense kernel (in, out) == affine W; bias row vector
                if len(L.shape_in) == 3 and L.shape_in[1] * L.shape_in[2] > 1:
                    c, h, w_ = L.shape_in  # Keras flattens HWC, DML rows are CHW
                    W = W.reshape(h, w_, c, -1).transpose(2, 0, 1, 3).reshape(c * h * w_, -1)
                out[f"W_{L.name}"], out[f"b_{L.name}"] = W, b.reshape(1, -1)
        return out
