"""Per-case kernel times from a rocprofv3 kernel trace of tools/bench_conv.py: for every
conv kernel dispatch (ours: sysml_dnn::*, MIOpen / hipBLASLt otherwise) the median time, in
dispatch order.   python tools/conv_trace_summary.py TRACE.csv"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    out, last, ds = [], None, []
    for r in rows:
        n = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        if d < 2.0 or "distribution" in n or "fillBuffer" in n:
            continue
        key = n[:90]
        if key != last and ds:
            ds.sort()
            out.append((last, len(ds), ds[len(ds) // 2]))
            ds = []
        last = key
        ds.append(d)
    if ds:
        ds.sort()
        out.append((last, len(ds), ds[len(ds) // 2]))
    for n, c, med in out:
        print(f"{c:3d} x {med:9.1f} us  {n}")


if __name__ == "__main__":
    main()
