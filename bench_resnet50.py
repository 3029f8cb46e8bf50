"""ResNet-50 training throughput through the DML nn library (BASELINE.json config 5:
"Keras2DML / scripts/nn ResNet-50 training bf16"), on synthetic data and random-init weights.

The network is built as a Caffe2DML layer DAG (models/dl.py: Convolution + BatchNorm + Scale +
ReLU bottlenecks with Eltwise residual sums, 3x3/2 max pool, 7x7 average pool, InnerProduct,
SoftmaxWithLoss), the generated forward / backward / SGD-momentum DML runs on the MI355X
backend: every conv2d / conv2d_backward_* / pooling / bias op is a hand-written kernel --
implicit-GEMM convolutions of ops/hip/dnn.hip, and for 1x1 stride-1 convolutions, small-image
im2col forward and col2im backward-data the image-blocked MFMA GEMM of ops/hip/gemm.hip
(no library GEMM kernel runs in a step: profiles/resnet50_step_kernels_b256_r5.txt);
convolutions compute on bf16 MFMA with fp32 accumulation, activations and
their gradients are stored bf16 (fp32 arithmetic in every kernel), weights, weight gradients
and the optimizer state stay fp32 (--fp32-activations: fp32 activations too).

    python bench_resnet50.py [--batch 32] [--steps 3] [--warmup 1] [--image 224]
Prints one JSON line (images/s over the timed steps).
"""
import argparse
import json
import os
import re
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402


def resnet50_layers(classes=1000, stages=(3, 4, 6, 3), image=224):
    """Layer DAG of ResNet-50 (torchvision layout: stride on the 3x3 conv of a bottleneck)."""
    from systemml_amd.models.dl import Layer, INPUT
    L = []

    def conv(name, bottom, F, k, s, p):
        L.append(Layer("conv", name, [bottom], [name], F=F, kh=k, kw=k, sh=s, sw=s, ph=p, pw=p))
        return name

    def bn_relu(name, bottom, relu=True):
        L.append(Layer("batchnorm", "bn_" + name, [bottom], ["bn_" + name], affine=False, mu=0.9, eps=1e-5))
        L.append(Layer("scale", "sc_" + name, ["bn_" + name], ["sc_" + name]))
        top = "sc_" + name
        if relu:
            L.append(Layer("relu", "relu_" + name, [top], ["relu_" + name]))
            top = "relu_" + name
        return top

    x = bn_relu("conv1", conv("conv1", INPUT, 64, 7, 2, 3))
    L.append(Layer("pool", "pool1", [x], ["pool1"], mode="MAX", kh=3, kw=3, sh=2, sw=2, ph=1, pw=1))
    x = "pool1"
    width = 64
    for si, nblk in enumerate(stages):
        for b in range(nblk):
            s = 2 if (b == 0 and si > 0) else 1
            nm = f"s{si + 1}b{b + 1}"
            y = bn_relu(nm + "a", conv(nm + "a", x, width, 1, 1, 0))
            y = bn_relu(nm + "b", conv(nm + "b", y, width, 3, s, 1))
            y = bn_relu(nm + "c", conv(nm + "c", y, width * 4, 1, 1, 0), relu=False)
            sc = x
            if b == 0:
                sc = bn_relu(nm + "p", conv(nm + "p", x, width * 4, 1, s, 0), relu=False)
            L.append(Layer("eltwise", nm + "sum", [y, sc], [nm + "sum"], op="SUM", coeff=[1.0, 1.0]))
            L.append(Layer("relu", nm + "out", [nm + "sum"], [nm + "out"]))
            x = nm + "out"
        width *= 2
    g = -(-image // 32)                       # final feature map side (7 at 224)
    L.append(Layer("pool", "gap", [x], ["gap"], mode="AVE", kh=g, kw=g, sh=1, sw=1, ph=0, pw=0))
    L.append(Layer("dense", "fc", ["gap"], ["fc"], M=classes))
    L.append(Layer("softmax_loss", "loss", ["fc"], ["prob"]))
    return L


def build_script(layers, input_shape, steps, batch, dp=False):
    from systemml_amd.models import dl
    gen = dl._Gen(layers, input_shape)
    params = dl.trainable(gen.layers)
    sc = dl._solver_consts({"type": "momentum", "base_lr": 0.01, "momentum": 0.9, "weight_decay": 1e-4})
    # benchSync (registered by main): waits for the device and returns a host clock in ns.  The
    # calls sit in their own basic blocks (inside `if`), so every operator of the step has been
    # issued before the device is synchronised: a step's time is its completed device work.
    lines = gen.sources("momentum") + [
        'benchSync = externalFunction(Matrix[Double] A) return (Double t) implemented in (classname="sysml.bench.Sync")',
        "X = read($X)", "Y = read($Y)", "N = nrow(X)", f"bs = {batch}", "lr0 = 0.01", "lr = lr0", "it = 0",
        "t0 = 0", "t1 = 0"]
    lines += gen.init()
    lines += dl._opt_init("momentum", params)
    lines += [f"for (i in 1:{steps}) {{", "  if (i > 0) {", "    t0 = benchSync(X)", "  }",
              "  beg = ((i - 1) * bs) %% N + 1",
              "  end = min(N, beg + bs - 1)", "  Xb = X[beg:end, ]", "  Yb = Y[beg:end, ]"]
    lines += ["  " + c for c in gen.forward(train=True)]
    lines.append(f"  loss = {gen.loss_expr()}")
    lines += ["  " + c for c in gen.backward()]
    if dp:
        # data parallelism over ranks (one per GPU): one bucketed RCCL all-reduce of every
        # gradient per step (Caffe2DML allreduce, models/dl.py)
        grads = [gen.grad_of(t) for t in params]
        lines.append("  [" + ", ".join(grads) + "] = _dp_allreduce(" + ", ".join(grads) + ")")
    lines += [f"  {a} = {b}" for a, b in gen.bn_updates()]
    lines += dl._opt_update(sc, gen, params, "  ")
    lines += ["  if (i > 0) {", f"    t1 = benchSync({params[-1]})", "  }",
              '  print("STEP " + i + " loss " + loss + " ns " + as.integer(t1 - t0))', "}"]
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--gpus", type=int, default=1,
                    help="run under torchrun with one rank per GPU: data parallel, --batch images per rank")
    ap.add_argument("--exact-fp32", action="store_true", help="convolutions on exact fp32 MFMA instead of bf16")
    ap.add_argument("--no-fusion", action="store_true", help="disable operator fusion (codegen templates)")
    ap.add_argument("--fp32-activations", action="store_true",
                    help="keep activations / their gradients fp32 (default: stored bf16, fp32 math)")
    a = ap.parse_args()
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    ctx = None
    if world > 1:
        from systemml_amd.parallel import dist as D
        ctx = D.init()
    rank = ctx.rank if ctx is not None else 0
    from systemml_amd.api.executor import compile_script, execute
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import kernels as K
    K.CONV_BF16_FP32 = not a.exact_fp32
    from systemml_amd.runtime.udf import register_udf

    def bench_sync(ctx, A):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        return (float(time.perf_counter_ns()),)
    register_udf("sysml.bench.Sync", bench_sync)
    layers = resnet50_layers(image=a.image)
    shape = (3, a.image, a.image)
    total = a.steps + a.warmup
    src = build_script(layers, shape, total, a.batch, dp=world > 1)
    rng = np.random.default_rng(rank)          # each rank trains on its own images
    n = a.batch * min(total, 2)
    X = rng.standard_normal((n, 3 * a.image * a.image)).astype(np.float32)
    Y = np.eye(1000, dtype=np.float32)[rng.integers(0, 1000, n)]
    # bf16 activations: fused cellwise results, conv outputs and pooling results of >= 4M cells
    # are stored bf16 (fp32 math); every weight / weight-gradient matrix of ResNet-50 is smaller
    # (largest: 512 x 4608), so parameters and the optimizer state stay fp32
    act = 0 if (a.fp32_activations or a.exact_fp32) else 1 << 22
    cfg = DMLConfig(precision="single", gpu_min_cells=0, fusion=not a.no_fusion, act_bf16_min_cells=act)
    cs = compile_script(src, {"X": "X", "Y": "Y"}, inputs={"X": X, "Y": Y}, config=cfg,
                        filename=os.path.join(SCRIPTS_DIR, "resnet50_bench.dml"))
    out = []
    # the compiled program lives for the whole run: keep it out of the cyclic collector's
    # generations so gen-2 collections during the steps stay short (as bench.py does)
    import gc
    gc.collect()
    gc.freeze()
    t = time.perf_counter()
    execute(cs, {"X": X, "Y": Y}, out=out.append)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    wall = time.perf_counter() - t
    steps = [(int(m.group(1)), float(m.group(2)), int(m.group(3))) for m in
             (re.match(r"STEP (\d+) loss (\S+) ns (\d+)", s) for s in out) if m]
    timed = [ns for i, _, ns in steps if i > a.warmup]
    ms = sum(timed) / len(timed) / 1e6 if timed else 0.0
    n_phys = 1
    if ctx is not None:
        ms = ctx.allreduce_scalar(ms, "max")          # rank 0 prints; the slowest rank sets the pace
        import torch.distributed as tdist
        devs = [None] * world
        tdist.all_gather_object(devs, (os.uname().nodename, torch.cuda.current_device() if torch.cuda.is_available() else -1))
        n_phys = len(set(devs))
    if rank != 0:
        if ctx is not None:
            from systemml_amd.parallel import dist as D
            D.shutdown()
        return
    print(json.dumps({"metric": "ResNet-50 training images/s (scripts/nn via Caffe2DML layer DAG)",
                      "value": round(world * a.batch / (ms / 1e3), 2), "unit": "images/s", "n_gpus": n_phys,
                      "scaling": "weak", "parallelism": f"dp{world}",
                      "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 2),
                      "higher_is_better": True, "dtype": "fp32-exact" if a.exact_fp32 else ("bf16 conv MFMA / fp32" if not act
                                                                       else "bf16 activations + MFMA / fp32 weights"),
                      "data": "synthetic N(0,1) images, random labels, random-init weights",
                      "losses": [round(l, 4) for _, l, _ in steps], "wall_s": round(wall, 1),
                      "step_ms": [round(ns / 1e6, 1) for _, _, ns in steps],
                      "kernel_counters": {k: v for k, v in K.counters.items() if k.startswith(("conv", "pool", "bias"))},
                      "config": {"model": "ResNet-50", "batch": a.batch, "global_batch": world * a.batch,
                                 "image": a.image, "classes": 1000}}))
    from systemml_amd.ops import cell as CE
    if CE.TRACE:
        print("cell stats", CE.stats, file=sys.stderr)
        for k, v in sorted(CE.fallbacks.items(), key=lambda kv: -kv[1])[:40]:
            print(f"  fallback x{v}: {k}", file=sys.stderr)
    if ctx is not None:
        from systemml_amd.parallel import dist as D
        D.shutdown()


if __name__ == "__main__":
    main()
