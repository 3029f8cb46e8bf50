"""Prints the fused operators (Cell / MAgg / Row programs) of the ResNet-50 training step's
main loop with their input shapes, one line each: which BN / ReLU / residual work is one
kernel and what each kernel reads and writes.  CPU only (plans at a small image size).

    python tools/probe/spoof_plan.py [--image 32] [--batch 4]
"""
import argparse
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))


def walk(blocks, out, seen):
    from systemml_amd.compiler.blocks import BasicBlock
    for b in blocks:
        if isinstance(b, BasicBlock):
            st = list(b.roots) + list(b.env_out.values())
            while st:
                h = st.pop()
                if h.id in seen:
                    continue
                seen.add(h.id)
                if h.op in ("cell", "magg", "row"):
                    out.append(h)
                st.extend(h.inputs)
            continue
        for attr in ("body", "then_blocks", "else_blocks"):
            sub = getattr(b, attr, None)
            if isinstance(sub, list):
                walk(sub, out, seen)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--image", type=int, default=32)
    ap.add_argument("--batch", type=int, default=4)
    a = ap.parse_args()
    from test_resnet_plan import _compile
    cs, _, _ = _compile(image=a.image, batch=a.batch)
    hs = []
    walk(cs.cp.blocks, hs, set())
    hs.sort(key=lambda h: h.id)
    for h in hs:
        prog = h.p.get("prog")
        d = prog.describe() if hasattr(prog, "describe") else str(prog)
        shp = " ".join(f"{i.dim1}x{i.dim2}" for i in h.inputs)
        print(f"{h.op:5s} out {h.dim1}x{h.dim2}  in [{shp}]  {d}")


if __name__ == "__main__":
    main()
