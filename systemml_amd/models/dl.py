"""Deep-learning model import: Caffe2DML and Keras2DML (reference: scala
org/apache/sysml/api/dl/{Caffe2DML,CaffeLayer,CaffeNetwork,CaffeSolver,DMLGenerator}.scala and
src/main/python/systemml/mllearn/{estimators.py (Caffe2DML, Keras2DML), keras2caffe.py}).

The reference converts a Keras model to a Caffe network + solver, then Caffe2DML generates
a DML training / prediction script over the nn library.  Here both front ends produce the
same layer DAG (blobs named by bottom / top; in-place layers renamed SSA-style), and one
generator emits DML over scripts/nn in topological order -- forward, then backward in
reverse order with gradient accumulation for blobs consumed by several layers -- with the
solver's optimizer (SGD, momentum, Nesterov, Adam, AdaGrad, RMSProp), learning-rate policy
(fixed / step / exp / inv) and L2 weight decay.

Layers: Convolution, Deconvolution, InnerProduct, Pooling (MAX / AVE), ReLU, Sigmoid, TanH,
ELU, Threshold, Dropout, BatchNorm, Scale, Eltwise (SUM with coefficients / PROD / MAX),
Concat (channels), LSTM, RNN, Upsample, Flatten, Softmax; losses SoftmaxWithLoss,
EuclideanLoss, SigmoidCrossEntropyLoss (reference CaffeLayer.scala).  Keras: Conv2D,
Conv2DTranspose, Dense, Max/AveragePooling2D, Flatten, Dropout, Activation,
BatchNormalization, Add / Subtract / Multiply / Maximum, Concatenate, LSTM, SimpleRNN,
UpSampling2D, ELU -- Sequential and functional models.
Training algorithms (set(train_algo=...)): minibatch, batch, allreduce and
allreduce_parallel_batches; the last two compute per-task gradients in a parfor, which
the SPMD backend runs across GPU ranks (runtime/parfor.exec_parfor_spmd).
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
# layer IR: a DAG of layers over named blobs
# ============================================================================
class Layer:
    """One network layer.  `bottoms` / `tops` name blobs (SSA: an in-place Caffe layer gets a
    fresh top name), so non-sequential nets (residual adds, concatenations, several
    consumers of one activation) are plain DAGs."""

    def __init__(self, kind, name, bottoms=None, tops=None, **p):
        self.kind = kind
        self.name = re.sub(r"\W", "_", name)
        self.bottoms = list(bottoms or [])
        self.tops = list(tops or [])
        self.p = p
        self.shape_in = None      # shape of the first bottom (C, H, W)
        self.shapes_in = []
        self.shape_out = None     # (C, H, W); dense outputs (D, 1, 1); sequences (T, D, 1)

    def __repr__(self):
        return f"{self.kind}:{self.name}{self.bottoms}->{self.tops}{self.p}"


INPUT = "data"
_LOSS = {"softmax_loss", "l2_loss", "sigmoid_loss"}
_PARAM = {"conv", "deconv", "dense", "lstm", "rnn", "scale", "batchnorm"}


def _ident(s):
    return re.sub(r"\W", "_", str(s))


def _chain(layers):
    """Wire a sequential layer list into a DAG (each layer consumes the previous top)."""
    prev = INPUT
    for i, L in enumerate(layers):
        L.bottoms = [prev]
        L.tops = [f"{L.name}_out"]
        prev = L.tops[0]
    return layers


def caffe_layers(net):
    """Caffe NetParameter dict -> layer DAG (data / accuracy layers become the input blob or
    are dropped; label blobs are implicit).  Reference: CaffeNetwork.scala / CaffeLayer.scala."""
    out = []
    cur = {}                 # caffe blob name -> current IR blob name
    labels = set()
    for nm in _as_list(net.get("input")):
        cur[nm] = INPUT
        break
    for L in _as_list(net.get("layer") or net.get("layers")):
        t = str(L.get("type", "")).lower()
        name = _ident(L.get("name", t))
        bots = [str(b) for b in _as_list(L.get("bottom"))]
        tops = [str(b) for b in _as_list(L.get("top"))]
        phase = [r.get("phase") for r in _as_list(L.get("include")) if isinstance(r, dict)]
        if "TEST" in phase:
            continue
        if t in ("data", "input", "memorydata", "imagedata", "hdf5data", "dummydata"):
            if tops:
                cur[tops[0]] = INPUT
            labels.update(tops[1:])
            continue
        if t in ("accuracy", "silence"):
            continue
        ins = [cur[b] for b in bots if b not in labels and b in cur]
        outs = []
        for tp in tops:
            nm = _ident(tp)
            if tp in cur or nm == INPUT:
                nm = f"{nm}_{name}"
            outs.append(nm)
        if t == "convolution" or t == "deconvolution":
            cp = L.get("convolution_param", {})
            k = _first(cp.get("kernel_size", 3))
            st = _first(cp.get("stride", 1))
            pd = _first(cp.get("pad", 0))
            lay = Layer("conv" if t == "convolution" else "deconv", name, ins, outs, F=int(cp["num_output"]),
                        kh=int(cp.get("kernel_h", k)), kw=int(cp.get("kernel_w", k)),
                        sh=int(cp.get("stride_h", st)), sw=int(cp.get("stride_w", st)),
                        ph=int(cp.get("pad_h", pd)), pw=int(cp.get("pad_w", pd)))
        elif t == "innerproduct":
            lay = Layer("dense", name, ins, outs, M=int(L.get("inner_product_param", {})["num_output"]))
        elif t == "pooling":
            pp = L.get("pooling_param", {})
            k = int(pp.get("kernel_size", 2))
            s = int(pp.get("stride", 1))
            lay = Layer("pool", name, ins, outs, mode=str(pp.get("pool", "MAX")).upper(), kh=int(pp.get("kernel_h", k)),
                        kw=int(pp.get("kernel_w", k)), sh=int(pp.get("stride_h", s)), sw=int(pp.get("stride_w", s)),
                        ph=int(pp.get("pad_h", pp.get("pad", 0))), pw=int(pp.get("pad_w", pp.get("pad", 0))))
        elif t in ("relu", "sigmoid", "tanh", "softmax"):
            lay = Layer(t, name, ins, outs)
        elif t == "elu":
            lay = Layer("elu", name, ins, outs, alpha=float(L.get("elu_param", {}).get("alpha", 1.0)))
        elif t == "threshold":
            lay = Layer("threshold", name, ins, outs, t=float(L.get("threshold_param", {}).get("threshold", 0.0)))
        elif t == "dropout":
            lay = Layer("dropout", name, ins, outs, rate=float(L.get("dropout_param", {}).get("dropout_ratio", 0.5)))
        elif t == "softmaxwithloss":
            lay = Layer("softmax_loss", name, ins[:1], outs)
        elif t == "euclideanloss":
            lay = Layer("l2_loss", name, ins[:1], outs)
        elif t == "sigmoidcrossentropyloss":
            lay = Layer("sigmoid_loss", name, ins[:1], outs)
        elif t == "flatten":
            lay = Layer("flatten", name, ins, outs)
        elif t == "batchnorm":
            bp = L.get("batch_norm_param", {})
            lay = Layer("batchnorm", name, ins, outs, affine=False,
                        mu=float(bp.get("moving_average_fraction", 0.999)), eps=float(bp.get("eps", 1e-5)))
        elif t == "scale":
            lay = Layer("scale", name, ins, outs)
        elif t == "eltwise":
            ep = L.get("eltwise_param", {})
            op = str(ep.get("operation", "SUM")).upper()
            coeff = [float(c) for c in _as_list(ep.get("coeff"))] or [1.0] * len(ins)
            lay = Layer("eltwise", name, ins, outs, op=op, coeff=coeff)
        elif t == "concat":
            axis = int(L.get("concat_param", {}).get("axis", 1))
            if axis != 1:
                raise ValueError("Caffe2DML: Concat is supported along the channel axis only")
            lay = Layer("concat", name, ins, outs)
        elif t in ("lstm", "rnn"):
            rp = L.get("recurrent_param", {})
            lay = Layer(t, name, ins, outs, M=int(rp["num_output"]),
                        rs=bool(rp.get("return_sequences", False)))
        elif t == "upsample":
            up = L.get("upsample_param", {})
            lay = Layer("upsample", name, ins, outs, sh=int(up.get("size_h", up.get("scale", 2))),
                        sw=int(up.get("size_w", up.get("scale", 2))))
        else:
            raise ValueError(f"Caffe2DML: unsupported layer type {L.get('type')}")
        out.append(lay)
        for tp, nm in zip(tops, outs):
            cur[tp] = nm
    return out


def _first(v):
    return v[0] if isinstance(v, list) else v


def _pair(v, d):
    if v is None:
        return (d, d)
    if isinstance(v, (list, tuple)):
        return (int(v[0]), int(v[1] if len(v) > 1 else v[0]))
    return (int(v), int(v))


_KERAS_ACT = ("relu", "sigmoid", "tanh", "softmax", "elu")


def _keras_layer(cls, c, name, ins, outs):
    """One Keras layer -> IR layer(s) (a fused activation becomes a separate layer)."""
    act = c.get("activation")
    res = []
    mid = outs[0] + "_pre" if act and act != "linear" and cls != "Activation" else outs[0]
    if cls in ("Conv2D", "Convolution2D", "Conv2DTranspose"):
        kh, kw = _pair(c.get("kernel_size"), 3)
        sh, sw = _pair(c.get("strides"), 1)
        same = c.get("padding", "valid") == "same"
        res.append(Layer("conv" if cls != "Conv2DTranspose" else "deconv", name, ins, [mid], F=int(c.get("filters")),
                         kh=kh, kw=kw, sh=sh, sw=sw, ph=(kh - 1) // 2 if same else 0, pw=(kw - 1) // 2 if same else 0))
    elif cls == "Dense":
        res.append(Layer("dense", name, ins, [mid], M=int(c.get("units"))))
    elif cls in ("MaxPooling2D", "AveragePooling2D"):
        kh, kw = _pair(c.get("pool_size"), 2)
        sh, sw = _pair(c.get("strides") or (kh, kw), kh)
        res.append(Layer("pool", name, ins, [mid], mode="MAX" if cls.startswith("Max") else "AVE", kh=kh, kw=kw,
                         sh=sh, sw=sw, ph=0, pw=0))
    elif cls in ("Flatten", "Reshape", "InputLayer"):
        res.append(Layer("flatten", name, ins, [mid]))
    elif cls == "Dropout":
        res.append(Layer("dropout", name, ins, [mid], rate=float(c.get("rate", 0.5))))
    elif cls == "Activation":
        act = c.get("activation")
        if act not in _KERAS_ACT:
            raise ValueError(f"Keras2DML: unsupported activation {act}")
        res.append(Layer(act, name, ins, outs, **({"alpha": 1.0} if act == "elu" else {})))
        return res
    elif cls == "BatchNormalization":
        res.append(Layer("batchnorm", name, ins, [mid], affine=True, mu=float(c.get("momentum", 0.99)),
                         eps=float(c.get("epsilon", 1e-3))))
    elif cls in ("Add", "Multiply", "Maximum", "Subtract"):
        op = {"Add": "SUM", "Multiply": "PROD", "Maximum": "MAX", "Subtract": "SUM"}[cls]
        coeff = [1.0, -1.0] if cls == "Subtract" else [1.0] * len(ins)
        res.append(Layer("eltwise", name, ins, [mid], op=op, coeff=coeff))
    elif cls == "Concatenate":
        if int(c.get("axis", -1)) not in (1, -3):
            raise ValueError("Keras2DML: Concatenate is supported along the channel axis only")
        res.append(Layer("concat", name, ins, [mid]))
    elif cls in ("LSTM", "SimpleRNN"):
        res.append(Layer("lstm" if cls == "LSTM" else "rnn", name, ins, [mid], M=int(c.get("units")),
                         rs=bool(c.get("return_sequences", False))))
    elif cls == "UpSampling2D":
        sh, sw = _pair(c.get("size"), 2)
        res.append(Layer("upsample", name, ins, [mid], sh=sh, sw=sw))
    elif cls == "ELU":
        res.append(Layer("elu", name, ins, [mid], alpha=float(c.get("alpha", 1.0))))
    else:
        raise ValueError(f"Keras2DML: unsupported layer {cls}")
    if mid != outs[0]:
        if act not in _KERAS_ACT:
            raise ValueError(f"Keras2DML: unsupported activation {act}")
        res.append(Layer(act, f"{name}_{act}", [mid], outs, **({"alpha": 1.0} if act == "elu" else {})))
    return res


def _inbound(nodes):
    """Source layer names of a functional-model layer's first call (Keras 2 lists
    [[name, node, tensor, kwargs], ...] or Keras 3 {"args": [keras tensors]})."""
    if not nodes:
        return []
    n0 = nodes[0]
    if isinstance(n0, list):
        return [e[0] for e in n0]
    out = []

    def walk(a):
        if isinstance(a, dict):
            h = a.get("config", {}).get("keras_history") if a.get("class_name") == "__keras_tensor__" else None
            if h:
                out.append(h[0])
            else:
                for v in a.values():
                    walk(v)
        elif isinstance(a, (list, tuple)):
            for v in a:
                walk(v)
    walk(n0.get("args", []))
    return out


def keras_layers(model):
    """Keras Sequential or functional model / JSON config -> (layer DAG, keras weights by
    layer name).  Reference: keras2caffe.py (Keras -> Caffe network) + Caffe2DML."""
    weights = {}
    if isinstance(model, (str, bytes)):
        model = json.loads(model)
    if not isinstance(model, dict):
        for l in model.layers:
            w = l.get_weights() if hasattr(l, "get_weights") else []
            if w:
                weights[_ident(l.get_config().get("name", ""))] = [np.asarray(a) for a in w]
        model = json.loads(model.to_json()) if hasattr(model, "to_json") else \
            {"class_name": "Sequential", "config": [{"class_name": type(l).__name__, "config": l.get_config()}
                                                    for l in model.layers]}
    cfg = model.get("config", model)
    specs = cfg["layers"] if isinstance(cfg, dict) else cfg
    functional = any(l.get("inbound_nodes") for l in specs)
    out = []
    if not functional:
        prev = INPUT
        for l in specs:
            cls, c = l["class_name"], l.get("config", {})
            if cls == "InputLayer":
                continue
            name = _ident(c.get("name", cls.lower() + str(len(out))))
            top = f"{name}_out"
            out += _keras_layer(cls, c, name, [prev], [top])
            prev = top
        return out, weights
    blob = {}
    for l in specs:
        cls, c = l["class_name"], l.get("config", {})
        name = _ident(l.get("name", c.get("name")))
        if cls == "InputLayer":
            blob[name] = INPUT
            continue
        ins = [blob[_ident(src)] for src in _inbound(l.get("inbound_nodes") or [])]
        top = f"{name}_out"
        out += _keras_layer(cls, c, name, ins, [top])
        blob[name] = top
    return out, weights


# ============================================================================
# shapes
# ============================================================================
def _toposort(layers):
    made = {INPUT}
    todo = list(layers)
    order = []
    while todo:
        progress = False
        for L in list(todo):
            if all(b in made for b in L.bottoms):
                order.append(L)
                made.update(L.tops)
                todo.remove(L)
                progress = True
        if not progress:
            raise ValueError(f"network has unreachable or cyclic layers: {[L.name for L in todo]}")
    return order


def infer_shapes(layers, input_shape):
    """Blob shapes (C, H, W) in topological order; returns the shape of the last layer."""
    shape = {INPUT: tuple(int(v) for v in input_shape)}
    last = shape[INPUT]
    for L in _toposort(layers):
        L.shapes_in = [shape[b] for b in L.bottoms]
        L.shape_in = L.shapes_in[0]
        c, h, w = L.shape_in
        k = L.kind
        if k in ("conv", "pool"):
            ho = (h + 2 * L.p["ph"] - L.p["kh"]) // L.p["sh"] + 1
            wo = (w + 2 * L.p["pw"] - L.p["kw"]) // L.p["sw"] + 1
            out = (L.p["F"] if k == "conv" else c, ho, wo)
        elif k == "deconv":
            out = (L.p["F"], L.p["sh"] * (h - 1) - 2 * L.p["ph"] + L.p["kh"],
                   L.p["sw"] * (w - 1) - 2 * L.p["pw"] + L.p["kw"])
        elif k == "dense":
            out = (L.p["M"], 1, 1)
        elif k == "concat":
            if any(s[1:] != L.shape_in[1:] for s in L.shapes_in):
                raise ValueError(f"{L.name}: Concat inputs differ in spatial size {L.shapes_in}")
            out = (sum(s[0] for s in L.shapes_in), h, w)
        elif k == "eltwise":
            if any(s != L.shape_in for s in L.shapes_in):
                raise ValueError(f"{L.name}: Eltwise inputs differ in shape {L.shapes_in}")
            out = L.shape_in
        elif k in ("lstm", "rnn"):
            T, D = c, h * w
            L.p["T"], L.p["D"] = T, D
            out = (T, L.p["M"], 1) if L.p["rs"] else (L.p["M"], 1, 1)
        elif k == "upsample":
            out = (c, h * L.p["sh"], w * L.p["sw"])
        else:
            out = L.shape_in
        L.shape_out = out
        for t in L.tops:
            shape[t] = out
        last = out
    return last


def _n(shape):
    return int(np.prod(shape))


# ============================================================================
# DML generation (reference: DMLGenerator.scala + CaffeLayer.scala forward/backward)
# ============================================================================
_SRC = {"conv": ("conv2d", "nn/layers/conv2d_builtin.dml"),
        "deconv": ("conv2d_transpose", "nn/layers/conv2d_transpose.dml"),
        "dense": ("affine", "nn/layers/affine.dml"), "relu": ("relu", "nn/layers/relu.dml"),
        "sigmoid": ("sigmoid", "nn/layers/sigmoid.dml"), "tanh": ("tanh", "nn/layers/tanh.dml"),
        "elu": ("elu", "nn/layers/elu.dml"), "dropout": ("dropout", "nn/layers/dropout.dml"),
        "softmax": ("softmax", "nn/layers/softmax.dml"), "softmax_loss": ("softmax", "nn/layers/softmax.dml"),
        "sigmoid_loss": ("sigmoid", "nn/layers/sigmoid.dml"),
        "batchnorm": ("bn2d", "nn/layers/batch_norm2d.dml"), "scale": ("ss2d", "nn/layers/scale_shift2d.dml"),
        "lstm": ("lstm", "nn/layers/lstm.dml"), "rnn": ("rnn", "nn/layers/rnn.dml"),
        "upsample": ("upsample2d", "nn/layers/upsample2d.dml")}
_LOSS_SRC = {"softmax_loss": ("cross_entropy_loss", "nn/layers/cross_entropy_loss.dml"),
             "l2_loss": ("l2_loss", "nn/layers/l2_loss.dml"),
             "sigmoid_loss": ("log_loss", "nn/layers/log_loss.dml")}
_OPT = {"sgd": "nn/optim/sgd.dml", "momentum": "nn/optim/sgd_momentum.dml", "nesterov": "nn/optim/sgd_nesterov.dml",
        "adam": "nn/optim/adam.dml", "adagrad": "nn/optim/adagrad.dml", "rmsprop": "nn/optim/rmsprop.dml"}


def _params(layers):
    return [L for L in layers if L.kind in _PARAM]


def trainable(layers):
    """Names of the trained parameters, in layer order."""
    out = []
    for L in layers:
        if L.kind in ("conv", "deconv", "dense", "lstm", "rnn"):
            out += [f"W_{L.name}", f"b_{L.name}"]
        elif L.kind == "scale" or (L.kind == "batchnorm" and L.p.get("affine")):
            out += [f"g_{L.name}", f"be_{L.name}"]
    return out


def state_vars(layers):
    """All model variables: trained parameters plus batch-norm running statistics (and the
    fixed gamma / beta of a Caffe BatchNorm)."""
    out = trainable(layers)
    for L in layers:
        if L.kind == "batchnorm":
            if not L.p.get("affine"):
                out += [f"g_{L.name}", f"be_{L.name}"]
            out += [f"em_{L.name}", f"ev_{L.name}"]
    return out


def _ensure_loss(layers, input_shape):
    infer_shapes(layers, input_shape)
    order = _toposort(layers)
    if any(L.kind in _LOSS for L in layers):
        return layers
    last = order[-1]
    if last.kind == "softmax":
        last.kind = "softmax_loss"
    else:
        layers.append(Layer("softmax_loss", "prob", [last.tops[0]], ["prob_out"]))
    infer_shapes(layers, input_shape)
    return layers


class _Gen:
    def __init__(self, layers, input_shape):
        self.layers = _ensure_loss(layers, input_shape)
        self.order = _toposort(self.layers)
        self.loss = next(L for L in self.order if L.kind in _LOSS)

    def var(self, blob):
        return "Xb" if blob == INPUT else f"o_{blob}"

    def sources(self, opt=None):
        seen = []
        for L in self.order:
            for tbl in (_SRC, _LOSS_SRC):
                if L.kind in tbl and tbl[L.kind] not in seen:
                    seen.append(tbl[L.kind])
            if L.kind == "pool":
                e = ("max_pool2d", "nn/layers/max_pool2d_builtin.dml") if L.p["mode"] == "MAX" else \
                    ("avg_pool2d", "nn/layers/avg_pool2d_builtin.dml")
                if e not in seen:
                    seen.append(e)
        lines = [f'source("{path}") as {ns}' for ns, path in seen]
        if opt:
            lines.append(f'source("{_OPT[opt]}") as optim')
        return lines

    def init(self):
        code = []
        for L in self.order:
            n = L.name
            c, h, w = L.shape_in
            if L.kind == "conv":
                code.append(f"[W_{n}, b_{n}] = conv2d::init({L.p['F']}, {c}, {L.p['kh']}, {L.p['kw']})")
            elif L.kind == "deconv":
                code.append(f"[W_{n}, b_{n}] = conv2d_transpose::init({L.p['F']}, {c}, {L.p['kh']}, {L.p['kw']})")
            elif L.kind == "dense":
                code.append(f"[W_{n}, b_{n}] = affine::init({c * h * w}, {L.p['M']})")
            elif L.kind == "lstm":
                code.append(f"[W_{n}, b_{n}, h0_{n}, c0_{n}] = lstm::init(1, {L.p['D']}, {L.p['M']})")
            elif L.kind == "rnn":
                code.append(f"[W_{n}, b_{n}, h0_{n}] = rnn::init(1, {L.p['D']}, {L.p['M']})")
            elif L.kind == "batchnorm":
                code.append(f"[g_{n}, be_{n}, em_{n}, ev_{n}] = bn2d::init({c})")
            elif L.kind == "scale":
                code.append(f"[g_{n}, be_{n}] = ss2d::init({c})")
        return code

    def forward(self, train):
        code = []
        for i, L in enumerate(self.order):
            n, p = L.name, L.p
            x = self.var(L.bottoms[0]) if L.bottoms else "Xb"
            o = self.var(L.tops[0])
            c, h, w = L.shape_in
            k = L.kind
            if k == "conv":
                code.append(f"[{o}, Ho_{n}, Wo_{n}] = conv2d::forward({x}, W_{n}, b_{n}, {c}, {h}, {w}, {p['kh']}, "
                            f"{p['kw']}, {p['sh']}, {p['sw']}, {p['ph']}, {p['pw']})")
            elif k == "deconv":
                code.append(f"[{o}, Ho_{n}, Wo_{n}] = conv2d_transpose::forward({x}, W_{n}, b_{n}, {c}, {h}, {w}, "
                            f"{p['kh']}, {p['kw']}, {p['sh']}, {p['sw']}, {p['ph']}, {p['pw']}, 0, 0)")
            elif k == "pool":
                ns = "max_pool2d" if p["mode"] == "MAX" else "avg_pool2d"
                code.append(f"[{o}, Ho_{n}, Wo_{n}] = {ns}::forward({x}, {c}, {h}, {w}, {p['kh']}, {p['kw']}, "
                            f"{p['sh']}, {p['sw']}, {p['ph']}, {p['pw']})")
            elif k == "dense":
                code.append(f"{o} = affine::forward({x}, W_{n}, b_{n})")
            elif k in ("relu", "sigmoid", "tanh", "softmax"):
                code.append(f"{o} = {k}::forward({x})")
            elif k == "elu":
                code.append(f"{o} = elu::forward({x}, {p['alpha']})")
            elif k == "threshold":
                code.append(f"{o} = {x} > {p['t']}")
            elif k == "dropout":
                code.append(f"[{o}, mask_{n}] = dropout::forward({x}, {1 - p['rate']}, -1)" if train else f"{o} = {x}")
            elif k == "flatten":
                code.append(f"{o} = {x}")
            elif k == "batchnorm":
                mode = '"train"' if train else '"test"'
                code.append(f"[{o}, em_upd_{n}, ev_upd_{n}, cm_{n}, cv_{n}, cn_{n}] = bn2d::forward({x}, g_{n}, be_{n}, "
                            f"{c}, {h}, {w}, {mode}, em_{n}, ev_{n}, {p['mu']}, {p['eps']})")
            elif k == "scale":
                code.append(f"{o} = ss2d::forward({x}, g_{n}, be_{n}, {c}, {h}, {w})")
            elif k == "eltwise":
                xs = [self.var(b) for b in L.bottoms]
                if p["op"] == "SUM":
                    code.append(f"{o} = " + " + ".join(f"{cf} * {v}" if cf != 1.0 else v for cf, v in zip(p["coeff"], xs)))
                elif p["op"] == "PROD":
                    code.append(f"{o} = " + " * ".join(xs))
                else:
                    e = xs[0]
                    for v in xs[1:]:
                        e = f"max({e}, {v})"
                    code.append(f"{o} = {e}")
            elif k == "concat":
                code.append(f"{o} = cbind(" + ", ".join(self.var(b) for b in L.bottoms) + ")")
            elif k == "lstm":
                rs = "TRUE" if p["rs"] else "FALSE"
                code.append(f"h0b_{n} = matrix(0, rows = nrow({x}), cols = {p['M']})")
                code.append(f"c0b_{n} = matrix(0, rows = nrow({x}), cols = {p['M']})")
                code.append(f"[{o}, cl_{n}, cout_{n}, cc_{n}, cifog_{n}] = lstm::forward({x}, W_{n}, b_{n}, {p['T']}, "
                            f"{p['D']}, {rs}, h0b_{n}, c0b_{n})")
            elif k == "rnn":
                rs = "TRUE" if p["rs"] else "FALSE"
                code.append(f"h0b_{n} = matrix(0, rows = nrow({x}), cols = {p['M']})")
                code.append(f"[{o}, cout_{n}] = rnn::forward({x}, W_{n}, b_{n}, {p['T']}, {p['D']}, {rs}, h0b_{n})")
            elif k == "upsample":
                code.append(f"{o} = upsample2d::forward({x}, {c}, {h}, {w}, {p['sh']}, {p['sw']})")
            elif k == "softmax_loss":
                code.append(f"{o} = softmax::forward({x})")
            elif k == "sigmoid_loss":
                code.append(f"{o} = sigmoid::forward({x})")
            elif k == "l2_loss":
                code.append(f"{o} = {x}")
            else:
                raise ValueError(k)
        return code

    def loss_expr(self):
        L = self.loss
        ns = _LOSS_SRC[L.kind][0]
        return f"{ns}::forward({self.var(L.tops[0])}, Yb)"

    def backward(self):
        code = []
        have = set()

        def acc(blob, expr):
            if blob == INPUT:
                code.append(f"dXb_unused = {expr}")
                return
            d = f"d_{blob}"
            if blob in have:
                code.append(f"{d} = {d} + {expr}")
            else:
                code.append(f"{d} = {expr}")
                have.add(blob)

        for L in reversed(self.order):
            n, p, k = L.name, L.p, L.kind
            x = self.var(L.bottoms[0]) if L.bottoms else "Xb"
            o = self.var(L.tops[0])
            dout = f"d_{L.tops[0]}"
            c, h, w = L.shape_in
            b0 = L.bottoms[0] if L.bottoms else INPUT
            if k in _LOSS:
                ns = _LOSS_SRC[k][0]
                if k == "softmax_loss":
                    acc(b0, f"softmax::backward({ns}::backward({o}, Yb), {x})")
                elif k == "sigmoid_loss":
                    acc(b0, f"sigmoid::backward({ns}::backward({o}, Yb), {x})")
                else:
                    acc(b0, f"{ns}::backward({o}, Yb)")
                continue
            if L.tops[0] not in have:
                continue                      # output does not reach the loss
            if k == "conv":
                code.append(f"[g_in_{n}, dW_{n}, db_{n}] = conv2d::backward({dout}, Ho_{n}, Wo_{n}, {x}, W_{n}, b_{n}, "
                            f"{c}, {h}, {w}, {p['kh']}, {p['kw']}, {p['sh']}, {p['sw']}, {p['ph']}, {p['pw']})")
                acc(b0, f"g_in_{n}")
            elif k == "deconv":
                code.append(f"[g_in_{n}, dW_{n}, db_{n}] = conv2d_transpose::backward({dout}, Ho_{n}, Wo_{n}, {x}, W_{n}, "
                            f"b_{n}, {c}, {h}, {w}, {p['kh']}, {p['kw']}, {p['sh']}, {p['sw']}, {p['ph']}, {p['pw']})")
                acc(b0, f"g_in_{n}")
            elif k == "pool":
                ns = "max_pool2d" if p["mode"] == "MAX" else "avg_pool2d"
                acc(b0, f"{ns}::backward({dout}, Ho_{n}, Wo_{n}, {x}, {c}, {h}, {w}, {p['kh']}, {p['kw']}, "
                        f"{p['sh']}, {p['sw']}, {p['ph']}, {p['pw']})")
            elif k == "dense":
                code.append(f"[g_in_{n}, dW_{n}, db_{n}] = affine::backward({dout}, {x}, W_{n}, b_{n})")
                acc(b0, f"g_in_{n}")
            elif k == "relu":       # from the output (y > 0 iff x > 0): the input need not stay live
                acc(b0, f"relu::backward({dout}, {o})")
            elif k in ("sigmoid", "tanh", "softmax"):
                acc(b0, f"{k}::backward({dout}, {x})")
            elif k == "elu":
                acc(b0, f"elu::backward({dout}, {x}, {p['alpha']})")
            elif k == "threshold":
                acc(b0, f"0 * {dout}")
            elif k == "dropout":
                acc(b0, f"dropout::backward({dout}, {x}, {1 - p['rate']}, mask_{n})")
            elif k == "flatten":
                acc(b0, dout)
            elif k == "batchnorm":
                code.append(f"[g_in_{n}, dg_{n}, dbe_{n}] = bn2d::backward({dout}, {o}, em_upd_{n}, ev_upd_{n}, cm_{n}, "
                            f"cv_{n}, cn_{n}, {x}, g_{n}, be_{n}, {c}, {h}, {w}, \"train\", em_{n}, ev_{n}, "
                            f"{p['mu']}, {p['eps']})")
                acc(b0, f"g_in_{n}")
            elif k == "scale":
                code.append(f"[g_in_{n}, dg_{n}, dbe_{n}] = ss2d::backward({dout}, {o}, {x}, g_{n}, be_{n}, {c}, {h}, {w})")
                acc(b0, f"g_in_{n}")
            elif k == "eltwise":
                xs = [self.var(b) for b in L.bottoms]
                for j, b in enumerate(L.bottoms):
                    if p["op"] == "SUM":
                        cf = p["coeff"][j]
                        acc(b, dout if cf == 1.0 else f"{cf} * {dout}")
                    elif p["op"] == "PROD":
                        others = [v for q, v in enumerate(xs) if q != j]
                        acc(b, f"{dout} * " + " * ".join(others))
                    else:
                        acc(b, f"{dout} * ({xs[j]} == {o})")
            elif k == "concat":
                a = 0
                for b, sh in zip(L.bottoms, L.shapes_in):
                    m = _n(sh)
                    acc(b, f"{dout}[, {a + 1}:{a + m}]")
                    a += m
            elif k == "lstm":
                rs = "TRUE" if p["rs"] else "FALSE"
                code.append(f"dcl_{n} = matrix(0, rows = nrow({x}), cols = {p['M']})")
                code.append(f"[g_in_{n}, dW_{n}, db_{n}, dh0_{n}, dc0_{n}] = lstm::backward({dout}, dcl_{n}, {x}, W_{n}, "
                            f"b_{n}, {p['T']}, {p['D']}, {rs}, h0b_{n}, c0b_{n}, cout_{n}, cc_{n}, cifog_{n})")
                acc(b0, f"g_in_{n}")
            elif k == "rnn":
                rs = "TRUE" if p["rs"] else "FALSE"
                code.append(f"[g_in_{n}, dW_{n}, db_{n}, dh0_{n}] = rnn::backward({dout}, {x}, W_{n}, b_{n}, {p['T']}, "
                            f"{p['D']}, {rs}, h0b_{n}, cout_{n})")
                acc(b0, f"g_in_{n}")
            elif k == "upsample":
                acc(b0, f"upsample2d::backward({dout}, {c}, {h}, {w}, {p['sh']}, {p['sw']})")
        return code

    def grad_of(self, t):
        """Gradient variable of trainable parameter t (W_x -> dW_x, g_x -> dg_x, ...)."""
        pre, _, rest = t.partition("_")
        return {"W": "dW_", "b": "db_", "g": "dg_", "be": "dbe_"}[pre] + rest

    def bn_updates(self):
        return [(f"em_{L.name}", f"em_upd_{L.name}") for L in self.order if L.kind == "batchnorm"] + \
               [(f"ev_{L.name}", f"ev_upd_{L.name}") for L in self.order if L.kind == "batchnorm"]


def _solver_consts(solver):
    return dict(opt=solver.get("type", "sgd"), lr=float(solver.get("base_lr", 0.01)),
                mom=float(solver.get("momentum", 0.9)), wd=float(solver.get("weight_decay", 0.0)),
                policy=str(solver.get("lr_policy", "fixed")).lower(), gamma=float(solver.get("gamma", 0.95)),
                step=int(solver.get("stepsize", 1000)), power=float(solver.get("power", 1.0)),
                beta2=float(solver.get("momentum2", 0.999)), eps=float(solver.get("delta", 1e-8)),
                decay=float(solver.get("rms_decay", 0.99)))


def _opt_init(opt, params):
    lines = []
    for t in params:
        if opt in ("momentum", "nesterov"):
            lines.append(f"v_{t} = optim::init({t})")
        elif opt == "adam":
            lines.append(f"[m_{t}, s_{t}] = optim::init({t})")
        elif opt in ("adagrad", "rmsprop"):
            lines.append(f"c_{t} = optim::init({t})")
    return lines


def _opt_update(sc, gen, params, ind):
    lines = []
    for t in params:
        g = gen.grad_of(t)
        if sc["wd"] > 0 and t.startswith("W_"):
            lines.append(f"{ind}{g} = {g} + {sc['wd']} * {t}")
        opt = sc["opt"]
        if opt == "sgd":
            lines.append(f"{ind}{t} = optim::update({t}, {g}, lr)")
        elif opt in ("momentum", "nesterov"):
            lines.append(f"{ind}[{t}, v_{t}] = optim::update({t}, {g}, lr, {sc['mom']}, v_{t})")
        elif opt == "adam":
            lines.append(f"{ind}[{t}, m_{t}, s_{t}] = optim::update({t}, {g}, lr, {sc['mom']}, {sc['beta2']}, "
                         f"{sc['eps']}, it, m_{t}, s_{t})")
        elif opt == "adagrad":
            lines.append(f"{ind}[{t}, c_{t}] = optim::update({t}, {g}, lr, {sc['eps']}, c_{t})")
        elif opt == "rmsprop":
            lines.append(f"{ind}[{t}, c_{t}] = optim::update({t}, {g}, lr, {sc['decay']}, {sc['eps']}, c_{t})")
    lines.append(f"{ind}it = it + 1")
    if sc["policy"] == "step":
        lines.append(f"{ind}lr = lr0 * {sc['gamma']} ^ floor(it / {sc['step']})")
    elif sc["policy"] == "exp":
        lines.append(f"{ind}lr = lr0 * {sc['gamma']} ^ it")
    elif sc["policy"] == "inv":
        lines.append(f"{ind}lr = lr0 * (1 + {sc['gamma']} * it) ^ (-{sc['power']})")
    return lines


TRAIN_ALGOS = ("minibatch", "batch", "allreduce", "allreduce_parallel_batches")
TEST_ALGOS = ("minibatch", "batch", "allreduce")


def generate_train_dml(layers, input_shape, solver, epochs, batch_size, seed=-1, train_algo="minibatch",
                       parallel_batches=2, spmd=False):
    """Training script for the network.  train_algo (reference Caffe2DML.scala):
      minibatch  -- one update per mini-batch;
      batch      -- full-batch gradient descent;
      allreduce_parallel_batches -- synchronous data parallelism: each step takes
                    `parallel_batches` mini-batches, a parfor computes their gradients
                    (one mini-batch per worker / GPU rank under the SPMD backend), the
                    gradients are averaged and one update is applied;
      allreduce  -- the same with one example per parfor task."""
    if train_algo not in TRAIN_ALGOS:
        raise ValueError(f"Caffe2DML: unsupported train_algo {train_algo} (one of {TRAIN_ALGOS})")
    gen = _Gen(layers, input_shape)
    sc = _solver_consts(solver)
    params = trainable(gen.layers)
    lines = gen.sources(sc["opt"]) + ["", "X = read($X)", "Y = read($Y)", "N = nrow(X)",
                                      f"epochs = {int(epochs)}", f"bs = {int(batch_size)}", f"lr0 = {sc['lr']}",
                                      "lr = lr0", "it = 0", "loss = 0.0"]
    lines += gen.init()
    lines += _opt_init(sc["opt"], params)
    fwd = gen.forward(train=True)
    bwd = gen.backward()
    bn = gen.bn_updates()
    if train_algo in ("minibatch", "batch"):
        if train_algo == "batch":
            lines.append("bs = N")
        lines += ["iters = as.integer(ceil(N / bs))", "for (e in 1:epochs) {", "  for (i in 1:iters) {",
                  "    beg = (i - 1) * bs + 1", "    end = min(N, beg + bs - 1)", "    Xb = X[beg:end, ]",
                  "    Yb = Y[beg:end, ]"]
        lines += ["    " + c for c in fwd]
        lines.append(f"    loss = {gen.loss_expr()}")
        lines += ["    " + c for c in bwd]
        lines += [f"    {a} = {b}" for a, b in bn]
        lines += _opt_update(sc, gen, params, "    ")
        lines += ["  }", '  print("Epoch " + e + ": loss " + loss)', "}"]
        return "\n".join(lines), state_vars(gen.layers)
    if spmd:
        # synchronous data parallelism over SPMD ranks (one per GPU), with the parfor form's
        # semantics (below): a step takes the same group of rows (bs for allreduce, P * bs for
        # allreduce_parallel_batches), split into W contiguous shares; rank r computes the
        # gradients of its share, weights them (and its loss and batch-norm statistics) by its
        # share of the group's rows, and one bucketed all-reduce (_dp_allreduce: RCCL over
        # xGMI) sums them -- every rank then applies the same update (Caffe2DML.scala:396-405
        # without the parfor's per-task gradient matrices).  A rank with an empty share of a
        # short last group still joins the collective, with weight 0.
        grads = [gen.grad_of(t) for t in params]
        P = int(parallel_batches) if train_algo == "allreduce_parallel_batches" else 1
        lines += ["W = _dp_world()", "r = _dp_rank()", f"gsz = {P} * bs", "groups = as.integer(ceil(N / gsz))",
                  "for (e in 1:epochs) {", "  for (g in 1:groups) {",
                  "    gb = ((g - 1) * gsz) %% N + 1", "    ge = min(N, gb + gsz - 1)", "    ng = ge - gb + 1",
                  "    share = as.integer(ceil(ng / W))", "    lo = gb + r * share",
                  "    hi = min(ge, lo + share - 1)", "    wt = max(0, hi - lo + 1) / ng",
                  "    lo = min(lo, ge)", "    hi = max(hi, lo)",
                  "    Xb = X[lo:hi, ]", "    Yb = Y[lo:hi, ]"]
        lines += ["    " + c for c in fwd]
        lines.append(f"    loss = {gen.loss_expr()}")
        lines += ["    " + c for c in bwd]
        red = grads + [b for _, b in bn]
        lines += [f"    {v} = wt * {v}" for v in red]
        lines.append("    Lm = matrix(wt * loss, rows = 1, cols = 1)")
        lines.append("    [" + ", ".join(red + ["Lm"]) + "] = _dp_allreduce(" + ", ".join(red + ["Lm"]) + ")")
        lines.append("    loss = as.scalar(Lm)")
        lines += [f"    {a} = {b}" for a, b in bn]
        lines += _opt_update(sc, gen, params, "    ")
        lines += ["  }", '  print("Epoch " + e + ": loss " + loss)', "}"]
        return "\n".join(lines), state_vars(gen.layers)
    # data-parallel: gradients of the parfor tasks land in rows of G_<param>, then averaged
    P = int(parallel_batches) if train_algo == "allreduce_parallel_batches" else None
    if P is not None:
        lines += [f"P = {P}", "gsz = P * bs", "groups = as.integer(ceil(N / gsz))"]
    else:
        lines += ["groups = as.integer(ceil(N / bs))"]
    lines += ["for (e in 1:epochs) {", "  for (g in 1:groups) {"]
    if P is not None:
        lines += ["    gb = ((g - 1) * gsz) %% N + 1", "    ge = min(N, gb + gsz - 1)", "    ng = ge - gb + 1",
                  "    ntask = P"]
    else:
        lines += ["    gb = (g - 1) * bs + 1", "    ge = min(N, gb + bs - 1)", "    ng = ge - gb + 1", "    ntask = ng"]
    for t in params:
        lines.append(f"    G_{t} = matrix(0, rows = ntask, cols = length({t}))")
    for a, _ in bn:
        lines.append(f"    G_{a} = matrix(0, rows = ntask, cols = length({a}))")
    lines.append("    Lg = matrix(0, rows = ntask, cols = 1)")
    lines.append("    parfor (j in 1:ntask) {")
    if P is not None:
        lines += ["      lo = gb + ((j - 1) * bs) %% ng", "      hi = min(ge, lo + bs - 1)"]
    else:
        lines += ["      lo = gb + j - 1", "      hi = lo"]
    lines += ["      Xb = X[lo:hi, ]", "      Yb = Y[lo:hi, ]", "      wt = (hi - lo + 1) / ng"]
    lines += ["      " + c for c in fwd]
    lines.append(f"      Lg[j, 1] = wt * {gen.loss_expr()}")
    lines += ["      " + c for c in bwd]
    for t in params:
        lines.append(f"      G_{t}[j, ] = wt * matrix({gen.grad_of(t)}, rows = 1, cols = length({t}))")
    for a, b in bn:
        lines.append(f"      G_{a}[j, ] = wt * matrix({b}, rows = 1, cols = length({a}))")
    lines.append("    }")
    for t in params:
        lines.append(f"    {gen.grad_of(t)} = matrix(colSums(G_{t}), rows = nrow({t}), cols = ncol({t}))")
    for a, _ in bn:
        lines.append(f"    {a} = matrix(colSums(G_{a}), rows = nrow({a}), cols = ncol({a}))")
    lines.append("    loss = sum(Lg)")
    lines += _opt_update(sc, gen, params, "    ")
    lines += ["  }", '  print("Epoch " + e + ": loss " + loss)', "}"]
    return "\n".join(lines), state_vars(gen.layers)


def generate_predict_dml(layers, input_shape, batch_size, test_algo="minibatch"):
    if test_algo not in TEST_ALGOS:
        raise ValueError(f"Caffe2DML: unsupported test_algo {test_algo} (one of {TEST_ALGOS})")
    gen = _Gen(layers, input_shape)
    fwd = gen.forward(train=False)
    prob = gen.var(gen.loss.tops[0])
    K = _n(gen.loss.shape_out)
    lines = gen.sources() + ["", "X = read($X)", "N = nrow(X)", f"bs = {int(batch_size)}"]
    if test_algo == "batch":
        lines.append("bs = N")
    lines += [f"P = matrix(0, rows = N, cols = {K})", "iters = as.integer(ceil(N / bs))"]
    loop = "parfor" if test_algo == "allreduce" else "for"
    lines += [f"{loop} (i in 1:iters) {{", "  beg = (i - 1) * bs + 1", "  end = min(N, beg + bs - 1)",
              "  Xb = X[beg:end, ]"]
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
    `net:`); input_shape: (C, H, W) of one example (rows of X are C*H*W, channel-major;
    sequence models: (T, D, 1)).
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
        self._defaults()

    def _defaults(self):
        self.batch_size = getattr(self, "batch_size", 64)
        self.debug = False
        self.train_algo = "minibatch"
        self.test_algo = "minibatch"
        self.parallel_batches = 2
        self.init_weights_ = getattr(self, "init_weights_", None)

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
        """Reference Caffe2DML.set: train_algo in minibatch | batch | allreduce |
        allreduce_parallel_batches, test_algo in minibatch | batch | allreduce."""
        if debug is not None:
            self.debug = bool(debug)
        if batch_size is not None:
            self.batch_size = int(batch_size)
        if train_algo is not None:
            if str(train_algo).lower() not in TRAIN_ALGOS:
                raise ValueError(f"unsupported train_algo {train_algo} (one of {TRAIN_ALGOS})")
            self.train_algo = str(train_algo).lower()
        if test_algo is not None:
            if str(test_algo).lower() not in TEST_ALGOS:
                raise ValueError(f"unsupported test_algo {test_algo} (one of {TEST_ALGOS})")
            self.test_algo = str(test_algo).lower()
        if parallel_batches is not None:
            self.parallel_batches = int(parallel_batches)
        if perform_one_hot_encoding is not None:
            self.one_hot = bool(perform_one_hot_encoding)
        if parfor_parameters is not None:
            self.parfor_parameters = dict(parfor_parameters)
        return self

    def summary(self):
        infer_shapes(self.layers, self.input_shape)
        rows = ["Layer                Type         Bottom(s)            Output shape     Params"]
        for L in _toposort(self.layers):
            c = L.shape_in[0]
            k = L.kind
            npar = 0
            if k in ("conv", "deconv"):
                npar = L.p["F"] * c * L.p["kh"] * L.p["kw"] + L.p["F"]
            elif k == "dense":
                npar = L.p["M"] * (_n(L.shape_in) + 1)
            elif k == "lstm":
                npar = (L.p["D"] + L.p["M"]) * 4 * L.p["M"] + 4 * L.p["M"]
            elif k == "rnn":
                npar = (L.p["D"] + L.p["M"]) * L.p["M"] + L.p["M"]
            elif k in ("scale", "batchnorm"):
                npar = 2 * c
            rows.append(f"{L.name:<20s} {k:<12s} {','.join(L.bottoms)[:20]:<20s} {str(L.shape_out):<16s} {npar}")
        s = "\n".join(rows)
        print(s)
        return s

    def fit(self, X, y, params=None):
        X = _np(X)
        gen_layers = self.layers
        regress = any(L.kind == "l2_loss" for L in gen_layers)
        if regress:
            Y = np.asarray(y, dtype=float).reshape(X.shape[0], -1)
        else:
            Y = np.eye(len(np.unique(y)))[self.encode(y).ravel().astype(int) - 1]
        n = X.shape[0]
        if self.train_algo == "batch":
            epochs = max(1, self.max_iter)
        else:
            per_step = self.batch_size * (self.parallel_batches if self.train_algo == "allreduce_parallel_batches" else 1)
            epochs = max(1, math.ceil(self.max_iter * per_step / n))
        from ..parallel import dist as D
        dctx = D.get_context()
        spmd = dctx is not None and dctx.world > 1 and self.train_algo in ("allreduce", "allreduce_parallel_batches")
        src, wnames = generate_train_dml(gen_layers, self.input_shape, self.solver, epochs, self.batch_size,
                                         train_algo=self.train_algo, parallel_batches=self.parallel_batches,
                                         spmd=spmd)
        self.train_script_ = src
        inputs = {"X": X, "Y": Y}
        if getattr(self, "init_weights_", None):
            # warm start: replace the init() calls by bound inputs
            keep = []
            for l in src.split("\n"):
                m = re.match(r"\[([\w, ]+)\] = \w+::init", l)
                if m and all(v.strip() in self.init_weights_ for v in m.group(1).split(",")
                             if not re.match(r"[hc]0_", v.strip())):
                    continue
                keep.append(l)
            src = "\n".join(keep)
            inputs.update(self.init_weights_)
        out = []
        res = run(src, args={"X": "X", "Y": "Y"}, inputs=inputs, outputs=wnames, config=self.config,
                  out=out.append, filename=os.path.join(SCRIPTS_DIR, "caffe2dml_train.dml"))
        self.log_ = out
        self.model_ = {k: _out(v) for k, v in res.items()}
        return self

    def predict_proba(self, X):
        src = generate_predict_dml(self.layers, self.input_shape, max(self.batch_size, 256), self.test_algo)
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
            keys = (("weight", "W"), ("bias", "b")) if L.kind not in ("scale", "batchnorm") else \
                (("weight", "g"), ("bias", "be"), ("mean", "em"), ("variance", "ev"))
            for part, key in keys:
                path = f"{weights}{sep}{L.name}_{part}.mtx"
                if os.path.exists(path):
                    found[f"{key}_{L.name}"] = _np(read_matrix(path))
        self.init_weights_ = found or None
        return self

    @property
    def model_keys(self):
        return state_vars(self.layers)


class Keras2DML(Caffe2DML):
    """Keras Sequential / functional model -> DML (reference: Keras2DML via keras2caffe +
    Caffe2DML)."""

    def __init__(self, sparkSession=None, keras_model=None, input_shape=None, transferUsingDF=False,
                 load_keras_weights=True, weights=None, labels=None, batch_size=64, max_iter=2000, test_iter=10,
                 test_interval=500, display=100, lr_policy="step", weight_decay=5e-4, regularization_type="L2",
                 optimizer="sgd", lr=0.01, momentum=0.9):
        BaseSystemMLClassifier.__init__(self, sparkSession)
        self.layers, kw = keras_layers(keras_model)
        if input_shape is not None and len(input_shape) == 3 and input_shape[-1] in (1, 3) and input_shape[0] not in (1, 3):
            input_shape = (input_shape[2], input_shape[0], input_shape[1])     # Keras HWC -> CHW
        if len(input_shape) == 2:                                            # (timesteps, features)
            input_shape = (input_shape[0], input_shape[1], 1)
        self.input_shape = tuple(int(v) for v in (input_shape if len(input_shape) == 3 else (input_shape[0], 1, 1)))
        opt = {"sgd": "momentum" if momentum > 0 else "sgd", "adam": "adam", "adagrad": "adagrad",
               "rmsprop": "rmsprop", "nesterov": "nesterov"}[optimizer.lower()]
        self.solver = {"type": opt, "base_lr": lr, "momentum": momentum, "lr_policy": lr_policy,
                       "weight_decay": weight_decay if regularization_type == "L2" else 0.0, "gamma": 0.95,
                       "stepsize": test_interval}
        self.max_iter = int(max_iter)
        self.batch_size = int(batch_size)
        self._defaults()
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
            n = L.name
            if L.kind == "conv":       # (kh, kw, C, F) -> F x (C*kh*kw)
                W = w[0]
                b = w[1] if len(w) > 1 else np.zeros(W.shape[-1])
                out[f"W_{n}"], out[f"b_{n}"] = np.transpose(W, (3, 2, 0, 1)).reshape(W.shape[3], -1), b.reshape(-1, 1)
            elif L.kind == "deconv":   # (kh, kw, F, C) -> C x (F*kh*kw)
                W = w[0]
                b = w[1] if len(w) > 1 else np.zeros(W.shape[2])
                out[f"W_{n}"], out[f"b_{n}"] = np.transpose(W, (3, 2, 0, 1)).reshape(W.shape[3], -1), b.reshape(-1, 1)
            elif L.kind == "dense":    # kernel (in, out) == affine W; bias row vector
                W = w[0]
                b = w[1] if len(w) > 1 else np.zeros(W.shape[-1])
                if len(L.shape_in) == 3 and L.shape_in[1] * L.shape_in[2] > 1:
                    c, h, w_ = L.shape_in  # Keras flattens HWC, DML rows are CHW
                    W = W.reshape(h, w_, c, -1).transpose(2, 0, 1, 3).reshape(c * h * w_, -1)
                out[f"W_{n}"], out[f"b_{n}"] = W, b.reshape(1, -1)
            elif L.kind == "lstm":     # kernel (D, 4M), recurrent (M, 4M), bias (4M); Keras gates i,f,c,o
                M = L.p["M"]
                Wk = np.vstack([w[0], w[1]])
                b = w[2] if len(w) > 2 else np.zeros(4 * M)
                perm = np.concatenate([np.arange(0, 2 * M), np.arange(3 * M, 4 * M), np.arange(2 * M, 3 * M)])
                out[f"W_{n}"], out[f"b_{n}"] = Wk[:, perm], b[perm].reshape(1, -1)
            elif L.kind == "rnn":
                out[f"W_{n}"] = np.vstack([w[0], w[1]])
                out[f"b_{n}"] = (w[2] if len(w) > 2 else np.zeros(L.p["M"])).reshape(1, -1)
            elif L.kind == "batchnorm":  # gamma, beta, moving_mean, moving_variance
                out[f"g_{n}"], out[f"be_{n}"] = w[0].reshape(-1, 1), w[1].reshape(-1, 1)
                out[f"em_{n}"], out[f"ev_{n}"] = w[2].reshape(-1, 1), w[3].reshape(-1, 1)
        return out
